set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
PCC_LIB=$R/point-cloud_amd/build/var_l0pf2/libpcconv.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread -k "not cli" > gpurun_out/t_parity_pf2.log 2>&1 || { echo "pf2 parity failed"; tail -30 gpurun_out/t_parity_pf2.log; exit 2; }
tail -1 gpurun_out/t_parity_pf2.log
PCC_LIB=$R/point-cloud_amd/build/var_l0pf2/libpcconv.so timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py -x -q --timeout 500 --timeout-method thread -k "config4_uniform_1b" > gpurun_out/t_large_pf2.log 2>&1 || { echo "pf2 large failed"; tail -30 gpurun_out/t_large_pf2.log; exit 3; }
tail -1 gpurun_out/t_large_pf2.log
timeout -k 10 300 python -u -m pytest tests/test_inputs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_inputs.log 2>&1 || { echo "inputs failed"; tail -30 gpurun_out/t_inputs.log; exit 4; }
tail -1 gpurun_out/t_inputs.log
bash scripts/ab.sh l0pf || exit 5
