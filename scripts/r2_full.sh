set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 || { echo "gpu tests failed"; exit 1; }
echo tests-ok
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; exit 2; }
echo bench-ok
