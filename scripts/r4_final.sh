# round 4: full GPU suite, smoke, the driver's bench command, kernel trace, FETCH/WRITE and SQ passes of the HEAD tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_final_suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/r4_final_suite.log; exit 2; }
tail -2 gpurun_out/r4_final_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4_final_smoke.log; exit 3; }
tail -2 gpurun_out/r4_final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err || { echo "bench failed"; tail -5 gpurun_out/r4_final_bench.err; exit 4; }
cat gpurun_out/r4_final_bench.json
bash scripts/ktrace.sh r4_final_kt > gpurun_out/r4_final_kt.txt || exit 5
tail -3 gpurun_out/r4_final_kt.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4_final_stats -o st -- python3 $R/bench.py --cpu-sample 0 > $R/gpurun_out/r4_final_stats.json 2> $R/gpurun_out/r4_final_stats.err || { echo "stats failed"; exit 6; }
cd $R
bash scripts/pmc.sh || exit 7
bash scripts/pmc_sq.sh || exit 8
echo final-ok
