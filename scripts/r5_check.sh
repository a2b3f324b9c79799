# round 5: the GPU parity suite, then an A/B of the product build against build/var_* (scripts/ab.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5c}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/${TAG}_suite.log; exit 2; }
tail -2 gpurun_out/${TAG}_suite.log
bash scripts/ab.sh ${TAG}_ab
