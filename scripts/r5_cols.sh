# round 5: keys past 2^32 on thread ranks (HIP ops); the level-0 pass-2 column unit order
# (PCC_L0_COLS) against the default on config 4, two interleaved rounds; a config-3 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5c}
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v -k "past_2p32" --timeout 250 --timeout-method thread > gpurun_out/${TAG}_2p32.log 2>&1 || { echo "2^32 tests failed"; tail -60 gpurun_out/${TAG}_2p32.log; exit 2; }
tail -1 gpurun_out/${TAG}_2p32.log
for round in 1 2; do
for v in rows cols; do
  if [ $v = cols ]; then export PCC_L0_COLS=1; else unset PCC_L0_COLS; fi
  timeout -k 10 200 python bench.py --steps 3 --warmup 2 --cpu-sample 0 > gpurun_out/$TAG/$v.$round.json 2> gpurun_out/$TAG/$v.$round.err || { echo "bench $v failed"; tail -3 gpurun_out/$TAG/$v.$round.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/$v.$round.json'));print('$v', $round, round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
done
unset PCC_L0_COLS
bash scripts/ktrace.sh $TAG/kt_c3 --points 100000000 --kind 2 || exit 2
