# bucket resolution A/B in one process per line: one launch (64 KB sort array,
# PCC_BKT_ONE=1) against the product (levels of >= 8192 buckets: a 256-thread launch
# with an 8 KB sort array, longer kept lists deferred to resident 64 KB workgroups)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/bktab
for round in 1 2; do
for m in one split; do
  env $( [ $m = one ] && echo PCC_BKT_ONE=1 ) timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/bktab/c4_$m.$round.json 2> gpurun_out/bktab/c4_$m.$round.err || { echo "bench failed"; exit 2; }
  env $( [ $m = one ] && echo PCC_BKT_ONE=1 ) timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 --points 100000000 --kind 2 --seed 3 > gpurun_out/bktab/c3_$m.$round.json 2> gpurun_out/bktab/c3_$m.$round.err || { echo "bench c3 failed"; exit 3; }
  python3 -c "import json;a=json.load(open('gpurun_out/bktab/c4_$m.$round.json'));b=json.load(open('gpurun_out/bktab/c3_$m.$round.json'));print('mode $m round $round c4', round(a['ms_per_step'],2), 'bucket', round(a['stage_ms']['bucket_ms'],3), '| c3', round(b['ms_per_step'],2), 'bucket', round(b['stage_ms']['bucket_ms'],3))"
done
done
