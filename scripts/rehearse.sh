# Round-end rehearsal of the driver's sequence: GPU suite, smoke, default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_final.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_final.log; exit 1; }
tail -1 gpurun_out/t_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_final.log; exit 2; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo "bench failed"; tail gpurun_out/bench_final.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_final.json'));print(round(d['ms_per_step'],2), d['value']/1e9, d['roofline']['frac'], d['cpu_baseline']['value'])"
