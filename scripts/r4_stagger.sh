# diagnostic: do the dense levels' slabs run in lockstep (all CUs in their
# (round 4: the engine code of this probe was removed after the measurement)
# end-of-slab gathers at once)?  The first 256 blocks start PCC_STAGGER us apart
# in total; the rest follow the freed CUs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out/stg
for round in 1 2; do
for v in 0 130 260; do
  env $( [ $v != 0 ] && echo PCC_STAGGER=$v ) timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/stg/s$v.$round.json 2> gpurun_out/stg/s$v.$round.err || { echo "bench $v failed"; tail -3 gpurun_out/stg/s$v.$round.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/stg/s$v.$round.json'));print('stagger $v', $round, round(d['ms_per_step'],2), round(d['stage_ms']['dense_ms'],3))"
done
done
for v in 0 260; do
  echo "== $v"; env $( [ $v != 0 ] && echo PCC_STAGGER=$v ) bash scripts/ktrace.sh stg/kt_$v | grep "k_slab<" || exit 3
done
