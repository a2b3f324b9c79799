# round 5: sub-grid dimensions beyond 96 (build_wide) and the sharded wide path, then the parity subset
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5w}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_dist_gpu.py -m gpu -x -v -k "wide" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_wide.log 2>&1 || { echo "wide tests failed"; tail -60 gpurun_out/${TAG}_wide.log; exit 2; }
grep -E "PASSED|FAILED" gpurun_out/${TAG}_wide.log; tail -1 gpurun_out/${TAG}_wide.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_nonfinite_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/${TAG}_par.log; exit 2; }
tail -1 gpurun_out/${TAG}_par.log
