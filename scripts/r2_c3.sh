set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_large_gpu.py -k "config3" > gpurun_out/c3test.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --points 100000000 --kind 2 --seed 3 --cpu-sample 0 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3kt -o kt -- python3 bench.py --points 100000000 --kind 2 --seed 3 --cpu-sample 0 --steps 2 --warmup 1 > gpurun_out/c3kt.json 2> gpurun_out/c3kt.err || exit 3
echo ok
