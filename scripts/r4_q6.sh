# round 4: level-0 fold without the mid-level host sync (device unit plan): parity subset, bench, trace; octant probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_nonfinite_gpu.py tests/test_large_gpu.py -x -q --timeout 300 --timeout-method thread -k "not from_disk and not sharded" > gpurun_out/r4_t6.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4_t6.log; exit 2; }
tail -2 gpurun_out/r4_t6.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r4_b6.json 2> gpurun_out/r4_b6.err || { echo "bench failed"; tail -3 gpurun_out/r4_b6.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r4_b6.json'));print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
bash scripts/ktrace.sh r4_kt6 > gpurun_out/r4_kt6.txt; head -4 gpurun_out/r4_kt6.txt
timeout -k 10 400 python -u scripts/octant_probe.py > gpurun_out/octant_probe.jsonl 2> gpurun_out/octant_probe.err || { echo "octant probe failed"; tail -5 gpurun_out/octant_probe.err; exit 4; }
cat gpurun_out/octant_probe.jsonl
