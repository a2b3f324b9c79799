set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD} && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r5_suite.log 2>&1
rc=$?; tail -4 gpurun_out/r5_suite.log; grep -E "^FAILED" gpurun_out/r5_suite.log | head; exit $rc
