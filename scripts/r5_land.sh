# round 5: the landed-input (exchange overlap) GPU tests, the dense parity subset, then scripts/ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5l}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v -k "landed or exchange_rounds or sharded_threads_match or event_table" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_land.log 2>&1 || { echo "landing tests failed"; tail -60 gpurun_out/${TAG}_land.log; exit 2; }
tail -1 gpurun_out/${TAG}_land.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_nonfinite_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/${TAG}_par.log; exit 2; }
tail -1 gpurun_out/${TAG}_par.log
bash scripts/ab.sh ${TAG}_ab
