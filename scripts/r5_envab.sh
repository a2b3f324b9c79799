# round 5: bench A/B of environment knobs in one build.  Usage:
#   bash scripts/r5_envab.sh TAG "BENCH ARGS" name1=ENV1=v,ENV2=v name2= ...   (two interleaved rounds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=$1; ARGS=$2; shift 2
cd $R && mkdir -p gpurun_out/$TAG
for round in 1 2; do
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
    timeout -k 10 200 python bench.py --steps 3 --warmup 2 --cpu-sample 0 $ARGS > gpurun_out/$TAG/$name.$round.json 2> gpurun_out/$TAG/$name.$round.err ) || { echo "bench $name failed"; tail -3 gpurun_out/$TAG/$name.$round.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/$name.$round.json'));print('$name', $round, round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
done
