# round 5: the randomised GPU-vs-oracle sweep (tests/test_fuzz_gpu.py: plain, merge, large, sharded,
# sharded merge, non-finite plain / merge / sharded), plus the sharded GPU tests when DIST=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
T="tests/test_fuzz_gpu.py"
[ "${DIST:-0}" = 1 ] && T="$T tests/test_dist_gpu.py"
[ $# -gt 0 ] && T="$T $*"   # more test files as arguments
timeout -k 10 900 python -u -m pytest -v --maxfail 5 --timeout 120 --timeout-method thread $T > gpurun_out/r5_fuzz.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r5_fuzz.log | tail -30
exit $rc
