# round 5: the modulo-4 level-0 fold (config 3): its tests, the parity subset, the config-3
# digests and the full-size sharded config 4, then config 3 with and without it (two rounds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5f}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_dist_gpu.py -m gpu -x -v -k "fold or single_level0 or level0_paths" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_fold.log 2>&1 || { echo "fold tests failed"; tail -60 gpurun_out/${TAG}_fold.log; exit 2; }
tail -1 gpurun_out/${TAG}_fold.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_nonfinite_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/${TAG}_par.log; exit 2; }
tail -1 gpurun_out/${TAG}_par.log
timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py -m gpu -x -v -k "config3_gaussian or config4_sharded" --timeout 500 --timeout-method thread > gpurun_out/${TAG}_large.log 2>&1 || { echo "large failed"; tail -40 gpurun_out/${TAG}_large.log; exit 2; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/${TAG}_large.log | tail -4
for round in 1 2; do
for v in fold4 nofold4; do
  if [ $v = nofold4 ]; then export PCC_NO_FOLD4=1; else unset PCC_NO_FOLD4; fi
  timeout -k 10 200 python bench.py --points 100000000 --kind 2 --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/$TAG/c3_$v.$round.json 2> gpurun_out/$TAG/c3_$v.$round.err || { echo "bench $v failed"; tail -3 gpurun_out/$TAG/c3_$v.$round.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/c3_$v.$round.json'));print('$v', $round, round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
done
