# k_next_emit with 16-byte row copies: parity (parity, merge, large), then
# config 4 and 5 bench lines (next_ms)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/nxt
timeout -k 10 1100 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_large_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/nxt/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/nxt/tests.log; exit 1; }
tail -1 gpurun_out/nxt/tests.log
for round in 1 2; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/nxt/c4.$round.json 2> gpurun_out/nxt/c4.$round.err || exit 2
  timeout -k 10 400 python bench.py --merge-prior 1000000000 --points 100000000 --seed 5 --cpu-sample 0 > gpurun_out/nxt/c5.$round.json 2> gpurun_out/nxt/c5.$round.err || exit 3
  for c in c4 c5; do python3 -c "import json;d=json.load(open('gpurun_out/nxt/$c.$round.json'));print('$c', $round, round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"; done
done
