# round 5: exchange / level-0 overlap evidence (scripts/r5_overlap.py) with the exchange in
# 4 rounds and in one, 2 thread ranks x 200M points on one GPU, kernel trace each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
for rounds in 4 0; do
  D=$R/gpurun_out/r5ovl_r$rounds
  mkdir -p $D
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o kt -- python3 $R/scripts/r5_overlap.py --rounds $rounds --stages $D/stages.json > $D/run.log 2>&1 || { echo "overlap run $rounds failed"; tail -20 $D/run.log; exit 2; }
  cd $R && python3 scripts/r5_overlap.py --trace $D/kt_kernel_trace.csv --stages $D/stages.json > $R/gpurun_out/r5ovl_r$rounds.json || exit 2
  python3 -c "import json;d=json.load(open('$R/gpurun_out/r5ovl_r$rounds.json'));print({k:v for k,v in d.items() if k!='ranks'});[print(r) for r in d['ranks']]"
done
