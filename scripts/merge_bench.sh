# config 5 on one GPU: merge tests, then +100M new points (seed 5) merged into the 1B config-4 cloud
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_merge_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_merge.log 2>&1 || { echo "merge tests failed"; tail -20 gpurun_out/t_merge.log; exit 1; }
tail -1 gpurun_out/t_merge.log
timeout -k 10 600 python -u bench.py --merge-prior 1000000000 --points 100000000 --seed 5 --cpu-sample 2000000 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "c5 bench failed"; tail -20 gpurun_out/bench_c5.err; exit 2; }
python3 -c "
import json; d = json.load(open('gpurun_out/bench_c5.json')); print(d['ms_per_step'], d['value'], d['stage_ms'], d['config'], d.get('cpu_baseline'))"
