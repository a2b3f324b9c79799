# round 5: the randomised GPU-vs-oracle sweep (tests/test_fuzz_gpu.py: 48 mid-size, 12 merges, 16 large)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --maxfail 5 --timeout 120 --timeout-method thread tests/test_fuzz_gpu.py > gpurun_out/r5_fuzz.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r5_fuzz.log | tail -30
exit $rc
