# round 4: level-0 run-read probe; folded level-0 binning parity (small + config 4)
# and timing against the three-pass binning; extra-VALU A/B of the dense kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./scripts/run_probe > gpurun_out/r4_run_probe.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r4_run_probe.log; exit 1; }
cat gpurun_out/r4_run_probe.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_large_gpu.py -x -q --timeout 300 --timeout-method thread -k "not from_disk and not sharded" > gpurun_out/r4_t_fold.log 2>&1 || { echo "fold tests failed"; tail -30 gpurun_out/r4_t_fold.log; exit 2; }
tail -2 gpurun_out/r4_t_fold.log
for v in fold nofold fold; do
  if [ $v = nofold ]; then export PCC_NO_FOLD=1; else unset PCC_NO_FOLD; fi
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r4_b_$v.json 2> gpurun_out/r4_b_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r4_b_$v.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4_b_$v.json'));print('$v', round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
unset PCC_NO_FOLD
bash scripts/ab.sh r4xv > gpurun_out/r4xv.log 2>&1; rc=$?
tail -30 gpurun_out/r4xv.log
exit $rc
