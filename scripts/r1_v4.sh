set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/t_v4.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_v4.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/b_v4.json 2> gpurun_out/b_v4.err || { echo "bench failed"; exit 2; }
PCC_LIB=$R/point-cloud_amd/build/stamps/libpcconv.so timeout -k 10 200 python bench.py --points 200000000 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/stamps_v4.json 2> gpurun_out/stamps_v4.err || { echo "stamps failed"; exit 3; }
echo ok
