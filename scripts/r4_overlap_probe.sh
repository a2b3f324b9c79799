# level-0 pass 2 beside (1) or before (2) the level-0 dense launch (PCC_OVERLAP_PROBE):
# (round 4: the engine code of this probe was removed after the measurement)
# the pair's time, from the engine's events, for the 1B bench build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/ovp
for round in 1 2; do
for m in 2 1; do
  PCC_OVERLAP_PROBE=$m timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/ovp/m$m.$round.json 2> gpurun_out/ovp/m$m.$round.err || { echo "probe $m failed"; tail -5 gpurun_out/ovp/m$m.$round.err; exit 1; }
  grep "\[probe\]" gpurun_out/ovp/m$m.$round.err | tail -3
done
done
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/ovp/plain.json 2> gpurun_out/ovp/plain.err || exit 2
python3 -c "import json;d=json.load(open('gpurun_out/ovp/plain.json'));print('plain', round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
