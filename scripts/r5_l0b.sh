# round 5: the arena-overflow path and the sharded tests after the collective error flags,
# then config-3 bench A/Bs of the modulo-4 fold's group count and a config-3 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5l0b}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_dist_gpu.py -m gpu -x -v -k "arena or sharded_threads or landed or past_2p32" --timeout 250 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/${TAG}_t.log; exit 2; }
tail -1 gpurun_out/${TAG}_t.log
bash scripts/r5_envab.sh ${TAG}_c3 "--points 100000000 --kind 2" g512= g2048=PCC_L0_GROUPS6=2048 g256=PCC_L0_GROUPS6=256 nofold4=PCC_NO_FOLD4=1 || exit 2
bash scripts/ktrace.sh ${TAG}/kt_c3 --points 100000000 --kind 2 | grep "k_l0\|sum" || exit 2
