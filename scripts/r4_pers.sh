# persistent dense-slab kernel (k_slab PERS) against one block per slab: parity
# (round 4: the persistent variant was reverted after this A/B)
# subset, then the 1B bench and config 3 interleaved, and a kernel trace of each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/pers
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_large_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or config4 or config3 or config5 or overflow or merge or level" > gpurun_out/pers/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pers/tests.log; exit 1; }
tail -2 gpurun_out/pers/tests.log
for round in 1 2; do
for v in 4 0; do
  PCC_PERS=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/pers/b$v.$round.json 2> gpurun_out/pers/b$v.$round.err || { echo "bench $v failed"; tail -3 gpurun_out/pers/b$v.$round.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/pers/b$v.$round.json'));print('pers=$v', $round, round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
  PCC_PERS=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --points 100000000 --kind 2 --seed 3 > gpurun_out/pers/c3_$v.$round.json 2> gpurun_out/pers/c3_$v.$round.err || { echo "bench c3 $v failed"; tail -3 gpurun_out/pers/c3_$v.$round.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/pers/c3_$v.$round.json'));print('c3 pers=$v', $round, round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
done
for v in 4 0; do
  echo "== pers=$v"; PCC_PERS=$v bash scripts/ktrace.sh pers/kt_$v | grep "k_slab\|sum" || exit 4
done
