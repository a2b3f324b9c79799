set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dist.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_dist.log; exit 1; }
tail -1 gpurun_out/t_dist.log
bash scripts/r3_stages.sh || exit 3
bash scripts/r3_mode_a.sh || exit 4
