# round 5: per-stage timing of the sharded config-4 and config-3 steps, 8 processes on one MI355X
# (gloo, one hardware queue per process), with rank-local keys (no key rebuild) and the fused
# bbox + slab histogram; summaries of non-build work against the builds run alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
for c in ${CONFIGS:-4 3}; do
  GPU_MAX_HW_QUEUES=1 timeout -k 10 600 python -u scripts/rank_stages.py --config $c --world 8 > gpurun_out/r5_stages_c$c.json 2> gpurun_out/r5_stages_c$c.err || { echo "c$c failed"; tail -20 gpurun_out/r5_stages_c$c.err; exit 2; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/r5_stages_c$c.json').read().strip().splitlines()[-1])   # gloo may print first
for r in d['ranks']:
    print($c, r['rank'], 'build alone', round(r['build_ms_alone'],2), 'non-build', round(r['non_build_local_ms'],2), 'ratio', round(r['non_build_over_build_alone'] or 0,3), {k: round(v,2) for k,v in r['non_build_device_alone_ms'].items()})
"
done
