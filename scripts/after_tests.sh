# Does the bench run slower right after the GPU test suite?  pytest, then the bench three times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_at.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/t_at.log; exit 1; }
tail -1 gpurun_out/t_at.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bu_at$i.json 2> gpurun_out/bu_at$i.err || { echo "bench $i failed"; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/bu_at$i.json'));print($i, round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
  [ $i -eq 1 ] && sleep 30
done
df -h /tmp | tail -1
PCC_VERBOSE=1 timeout -k 10 400 python -u scripts/merge_disk_bench.py > gpurun_out/merge_disk.json 2> gpurun_out/merge_disk.err || { echo "merge disk bench failed"; tail -5 gpurun_out/merge_disk.err; exit 3; }
cat gpurun_out/merge_disk.json
