set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD} && mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_fuzz_gpu.py -k "test_fuzz_matches_oracle or nonfinite_matches" > gpurun_out/rep$i.log 2>&1
  rc=$?; tail -2 gpurun_out/rep$i.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
