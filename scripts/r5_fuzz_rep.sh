# round 5: the randomised sweep repeated in fresh processes (looking for the one
# intermittent kept-list mismatch seen once); REPS runs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD} && mkdir -p gpurun_out
for i in $(seq 1 ${1:-3}); do
  timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_fuzz_gpu.py > gpurun_out/rep$i.log 2>&1
  rc=$?; tail -1 gpurun_out/rep$i.log; grep -E "^E .*AssertionError" gpurun_out/rep$i.log | head -3
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
