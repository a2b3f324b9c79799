# A/B timing of diagnostic builds (build/var_*/libpcconv.so) against the product build:
# two rounds of one 1B bench line each (2 warmup + 3 timed builds), variants
# interleaved, then per-launch kernel durations (rocprofv3 kernel trace) once each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-ab}
cd $R && mkdir -p gpurun_out/$TAG
VARS="prod $(ls $R/point-cloud_amd/build | grep '^var_' | sed 's/^var_//')"
lib() { if [ $1 = prod ]; then echo $R/point-cloud_amd/build/libpcconv.so; else echo $R/point-cloud_amd/build/var_$1/libpcconv.so; fi; }
for round in 1 2; do
for v in $VARS; do
  PCC_LIB=$(lib $v) timeout -k 10 200 python bench.py --steps 3 --warmup 2 --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/$TAG/$v.$round.json 2> gpurun_out/$TAG/$v.$round.err || { echo "bench $v failed"; tail -3 gpurun_out/$TAG/$v.$round.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/$v.$round.json'));print('$v', $round, round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
done
for v in $VARS; do
  echo "== $v"; PCC_LIB=$(lib $v) bash scripts/ktrace.sh $TAG/kt_$v ${BENCH_ARGS} | grep "k_slab\|k_l0\|sum" || exit 2
done
