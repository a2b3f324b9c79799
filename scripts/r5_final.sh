# round 5: full GPU suite, smoke, the driver's bench command (config 4), configs 3 / 5 / 2 bench
# lines, kernel trace with stats; TAG names the outputs under gpurun_out/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r5_final}
cd $R && mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/${TAG}_suite.log; exit 2; }
tail -2 gpurun_out/${TAG}_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 3; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 4; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 200 python bench.py --points 100000000 --kind 2 --seed 3 --cpu-sample 0 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo "c3 failed"; exit 5; }
timeout -k 10 300 python bench.py --merge-prior 1000000000 --points 100000000 --seed 5 --cpu-sample 0 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { echo "c5 failed"; exit 6; }
timeout -k 10 200 python bench.py --points 10000000 --seed 2 --cpu-sample 0 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || { echo "c2 failed"; exit 7; }
for c in c3 c5 c2; do python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$c.json'));print('$c', round(d['ms_per_step'],2), d['value'], d['unit'], {k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_stats -o st -- python3 $R/bench.py --cpu-sample 0 > $R/gpurun_out/${TAG}_stats.json 2> $R/gpurun_out/${TAG}_stats.err || { echo "stats failed"; exit 8; }
cd $R && python3 scripts/ktsum.py gpurun_out/${TAG}_stats/st_kernel_trace.csv
echo final-ok
