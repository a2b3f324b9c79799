# round 4: folded level-0 binning v2 (no spills, 16-bit tile keys): parity subset, then timing vs the three-pass binning + kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_large_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread -k "not from_disk and not sharded_8_ranks and not config5_sharded" > gpurun_out/r4_t_fold3.log 2>&1 || { echo "fold tests failed"; tail -30 gpurun_out/r4_t_fold2.log; exit 2; }
tail -2 gpurun_out/r4_t_fold3.log
for v in fold nofold fold; do
  if [ $v = nofold ]; then export PCC_NO_FOLD=1; else unset PCC_NO_FOLD; fi
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r4_b3_$v.json 2> gpurun_out/r4_b3_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r4_b3_$v.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4_b3_$v.json'));print('$v', round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
unset PCC_NO_FOLD
bash scripts/ktrace.sh r4_kt_fold3 > gpurun_out/r4_kt_fold3.txt; head -8 gpurun_out/r4_kt_fold3.txt
