# round 4: bench lines of configs 2, 3 and 5 on the round's tree (config 4 is r4_final.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/cfg
timeout -k 10 300 python bench.py --points 10000000 --seed 2 --cpu-sample 2000000 > gpurun_out/cfg/c2.json 2> gpurun_out/cfg/c2.err || { echo "c2 failed"; tail -5 gpurun_out/cfg/c2.err; exit 1; }
timeout -k 10 300 python bench.py --points 100000000 --kind 2 --seed 3 --cpu-sample 2000000 > gpurun_out/cfg/c3.json 2> gpurun_out/cfg/c3.err || { echo "c3 failed"; tail -5 gpurun_out/cfg/c3.err; exit 2; }
timeout -k 10 600 python -u bench.py --merge-prior 1000000000 --points 100000000 --seed 5 --cpu-sample 2000000 > gpurun_out/cfg/c5.json 2> gpurun_out/cfg/c5.err || { echo "c5 failed"; tail -5 gpurun_out/cfg/c5.err; exit 3; }
for c in c2 c3 c5; do python3 -c "import json;d=json.load(open('gpurun_out/cfg/$c.json'));print('$c', d['config']['workload'], round(d['ms_per_step'],3), round(d['value']/1e9,3), 'G/s', {k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)}, 'cpu', round(d['cpu_baseline']['value']/1e6,3))"; done
