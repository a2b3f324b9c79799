# round 5: an engine change (prod) against the previous build (build/var_head; first use: packed pinned
# readbacks + the small-slab counts read back behind the dense launch)
# parity subset, then config 4 and config 3 A/Bs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5rb}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_nonfinite_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/${TAG}_par.log; exit 2; }
tail -1 gpurun_out/${TAG}_par.log
bash scripts/ab.sh ${TAG}_c4 || exit 3
BENCH_ARGS="--points 100000000 --kind 2 --seed 3" bash scripts/ab.sh ${TAG}_c3 || exit 4
