# round 4: dense kernel NaN rules behind a template flag: non-finite + parity tests, bench, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_nonfinite_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_t5.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4_t5.log; exit 2; }
tail -2 gpurun_out/r4_t5.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r4_b5.json 2> gpurun_out/r4_b5.err || { echo "bench failed"; tail -3 gpurun_out/r4_b5.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r4_b5.json'));print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
bash scripts/ktrace.sh r4_kt5 > gpurun_out/r4_kt5.txt; head -14 gpurun_out/r4_kt5.txt
