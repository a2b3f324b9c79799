# round 4: full GPU suite after the non-finite support, then bench + kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_suite4.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/r4_suite4.log; exit 2; }
tail -2 gpurun_out/r4_suite4.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r4_b4.json 2> gpurun_out/r4_b4.err || { echo "bench failed"; tail -3 gpurun_out/r4_b4.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r4_b4.json'));print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
bash scripts/ktrace.sh r4_kt4 > gpurun_out/r4_kt4.txt; head -12 gpurun_out/r4_kt4.txt
