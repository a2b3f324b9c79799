# merge with grid seeds written straight into the slot tables: merge parity (incl. config 5 at full size) and the config-5 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "merge or config5 or dist" > gpurun_out/t_sf.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_sf.log; exit 1; }
tail -1 gpurun_out/t_sf.log
timeout -k 10 400 python bench.py --points 100000000 --seed 5 --merge-prior 1000000000 --cpu-sample 0 > gpurun_out/c5_sf.json 2> gpurun_out/c5_sf.err || { echo "c5 failed"; tail gpurun_out/c5_sf.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/c5_sf.json'));print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)}, d['config']['arrivals_W'])"
