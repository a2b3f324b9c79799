set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread -k "bucket_resolution or export_grid or split_cells or gloo" > gpurun_out/t_dist.log 2>&1 || { echo "dist tests failed"; tail -30 gpurun_out/t_dist.log; exit 1; }
tail -1 gpurun_out/t_dist.log
timeout -k 10 300 python -u -m pytest tests/test_inputs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_inputs.log 2>&1 || { echo "inputs tests failed"; tail -30 gpurun_out/t_inputs.log; exit 1; }
tail -1 gpurun_out/t_inputs.log
bash scripts/r3_rccl.sh || { echo "rccl probe failed"; exit 2; }
bash scripts/r3_stages.sh || exit 3
