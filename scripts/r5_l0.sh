# round 5: level-0 changes (pass-2 unit order by columns, the modulo-4 fold's group and unit sizes):
# level-0 tests, parity subset, config-3 digests, then bench A/Bs and a config-3 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5l0}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_dist_gpu.py -m gpu -x -v -k "fold or single_level0 or level0_paths or upload_in_pieces or landed" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_l0.log 2>&1 || { echo "level-0 tests failed"; tail -60 gpurun_out/${TAG}_l0.log; exit 2; }
tail -1 gpurun_out/${TAG}_l0.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_nonfinite_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/${TAG}_par.log; exit 2; }
tail -1 gpurun_out/${TAG}_par.log
timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py -m gpu -x -v -k "config3_gaussian or config4_uniform" --timeout 500 --timeout-method thread > gpurun_out/${TAG}_large.log 2>&1 || { echo "large failed"; tail -40 gpurun_out/${TAG}_large.log; exit 2; }
grep -E "PASSED|FAILED" gpurun_out/${TAG}_large.log | tail -4
bash scripts/r5_envab.sh ${TAG}_c4 "" cols= rows=PCC_L0_ROWS=1 || exit 2
bash scripts/r5_envab.sh ${TAG}_c3 "--points 100000000 --kind 2" g512= g2048=PCC_L0_GROUPS6=2048 g256=PCC_L0_GROUPS6=256 nofold4=PCC_NO_FOLD4=1 || exit 2
bash scripts/ktrace.sh ${TAG}/kt_c3 --points 100000000 --kind 2 | grep "k_l0\|sum" || exit 2
