# round 4: per-stage timing of the sharded config-4 step (fused bbox + slab histogram), 8 processes, 1 HW queue each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=1 timeout -k 10 600 python -u scripts/rank_stages.py --config 4 --world 8 > gpurun_out/stages_c4_fused.json 2> gpurun_out/stages_c4_fused.err || { echo "c4 failed"; tail -20 gpurun_out/stages_c4_fused.err; exit 2; }
python3 -c "
import json
d=json.loads(open('gpurun_out/stages_c4_fused.json').read().strip().split('\n')[-1])
for r in d['ranks']:
    print(r['rank'], 'alone', {k: round(v,2) for k,v in r['alone'].items()})
"
