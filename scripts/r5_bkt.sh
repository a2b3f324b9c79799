# round 5: kept lists ordered by the LSD radix sort (prod) against the bitonic network
# (build/var_bitonic, -DPCC_BKT_RADIX=0): parity subset + large digests, then config 3 and 4 A/Bs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5bkt}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_merge_gpu.py tests/test_nonfinite_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/${TAG}_par.log; exit 2; }
tail -1 gpurun_out/${TAG}_par.log
timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py -m gpu -x -v -k "config3_gaussian or config4_uniform or config5_merge_100m_into_1b" --timeout 500 --timeout-method thread > gpurun_out/${TAG}_large.log 2>&1 || { echo "large failed"; tail -40 gpurun_out/${TAG}_large.log; exit 2; }
grep -E "PASSED|FAILED" gpurun_out/${TAG}_large.log | tail -5
BENCH_ARGS="--points 100000000 --kind 2 --seed 3" bash scripts/ab.sh ${TAG}_c3 || exit 3
bash scripts/ab.sh ${TAG}_c4 || exit 4
