# round 4: per-stage timing of the sharded config-4 step, 8 processes on one MI355X (gloo), with the
# default 4 hardware queues per process (32 queues: the box's hardware scheduler oversubscribed)
# and with 1 queue per process (8 queues)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=1 timeout -k 10 600 python -u scripts/rank_stages.py --config 4 --world 8 > gpurun_out/stages_c4_q1.json 2> gpurun_out/stages_c4_q1.err || { echo "c4 q1 failed"; tail -20 gpurun_out/stages_c4_q1.err; exit 2; }
echo q1-ok
timeout -k 10 600 python -u scripts/rank_stages.py --config 4 --world 8 > gpurun_out/stages_c4_q4.json 2> gpurun_out/stages_c4_q4.err || { echo "c4 q4 failed"; tail -20 gpurun_out/stages_c4_q4.err; exit 3; }
echo q4-ok
for q in q1 q4; do python3 -c "
import json
d=json.load(open('gpurun_out/stages_c4_$q.json'))
print('$q', [round(r['alone']['build'],2) for r in d['ranks']], [round(r['ms']['build'],1) for r in d['ranks']])
"; done
