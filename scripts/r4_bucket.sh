# bucket resolution in two launches: parity (the forced two-launch test, the
# parity suite, the full-size digests), then the one-launch / split A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/bkt
timeout -k 10 1000 python -u -m pytest tests/test_parity_gpu.py tests/test_large_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bkt/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bkt/tests.log; exit 1; }
tail -2 gpurun_out/bkt/tests.log
bash scripts/r4_bucket_ab.sh || exit 2
