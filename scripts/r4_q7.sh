# round 4: A/B of the device-planned level-0 pass 2 (one sync) against the host plan; octant probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
for v in dev host dev host; do
  if [ $v = host ]; then export PCC_L0_HOSTPLAN=1; else unset PCC_L0_HOSTPLAN; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/r4_b7_$v.json 2> gpurun_out/r4_b7_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r4_b7_$v.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4_b7_$v.json'));print('$v', round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
unset PCC_L0_HOSTPLAN
timeout -k 10 400 python -u scripts/octant_probe.py > gpurun_out/octant_probe.jsonl 2> gpurun_out/octant_probe.err || { echo "octant probe failed"; tail -5 gpurun_out/octant_probe.err; exit 4; }
cat gpurun_out/octant_probe.jsonl
