# merge mode with the grid seeds' slot records precomputed at adoption
# (k_seed_rec): merge parity (small, sharded, full-size config 5), then the
# config-5 bench and its kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/srec
timeout -k 10 1100 python -u -m pytest tests/test_merge_gpu.py tests/test_dist_gpu.py tests/test_large_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread -k "merge or prior or config5 or adopt" > gpurun_out/srec/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/srec/tests.log; exit 1; }
tail -2 gpurun_out/srec/tests.log
for round in 1 2; do
  timeout -k 10 400 python -u bench.py --merge-prior 1000000000 --points 100000000 --seed 5 --cpu-sample 0 > gpurun_out/srec/c5.$round.json 2> gpurun_out/srec/c5.$round.err || { echo "c5 failed"; tail -5 gpurun_out/srec/c5.$round.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/srec/c5.$round.json'));print('c5', $round, round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
bash scripts/ktrace.sh srec/kt --merge-prior 1000000000 --points 100000000 --seed 5 | grep "k_slab\|sum" || exit 3
