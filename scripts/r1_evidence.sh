# round-1 evidence for the current kernels: parity suite, bench lines (config 4 with the CPU
# baseline, config-3 shape, config 5), kernel-trace stats, PMC traffic passes of the config-4 build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/ev_pytest.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/ev_pytest.log; exit 1; }
tail -1 gpurun_out/ev_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/ev_bench_c4.json 2> gpurun_out/ev_bench_c4.err || { echo "bench c4 failed"; exit 2; }
timeout -k 10 300 python bench.py --points 100000000 --kind 1 --seed 3 --cpu-sample 10000000 > gpurun_out/ev_bench_c3.json 2> gpurun_out/ev_bench_c3.err || { echo "bench c3 failed"; exit 3; }
timeout -k 10 600 python -u bench.py --merge-prior 1000000000 --points 100000000 --seed 5 --cpu-sample 2000000 > gpurun_out/ev_bench_c5.json 2> gpurun_out/ev_bench_c5.err || { echo "bench c5 failed"; exit 4; }
bash scripts/pmc.sh || exit 5
echo evidence-ok
