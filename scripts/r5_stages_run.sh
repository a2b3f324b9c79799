set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dist_gpu.py -m gpu > gpurun_out/r5s_tests.log 2>&1 || { tail -30 gpurun_out/r5s_tests.log; exit 3; }
tail -2 gpurun_out/r5s_tests.log
bash scripts/r5_stages.sh
