# round 5: the non-finite merge / sharded GPU tests, the full GPU suite, then the dense A/B (scripts/ab.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5n}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_nonfinite_gpu.py tests/test_dist_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "nonfinite or infinite" > gpurun_out/${TAG}_nf.log 2>&1 || { echo "nonfinite tests failed"; tail -60 gpurun_out/${TAG}_nf.log; exit 2; }
tail -2 gpurun_out/${TAG}_nf.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/${TAG}_suite.log; exit 3; }
tail -2 gpurun_out/${TAG}_suite.log
bash scripts/ab.sh ${TAG}_ab
