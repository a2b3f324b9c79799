# quick GPU check: parity suite + uniform 1B and clustered 100M bench lines (no CPU baseline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-q}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bu_$TAG.json 2> gpurun_out/bu_$TAG.err || { echo "uniform bench failed"; tail gpurun_out/bu_$TAG.err; exit 2; }
timeout -k 10 300 python bench.py --points 100000000 --kind 1 --seed 3 --cpu-sample 0 > gpurun_out/bc_$TAG.json 2> gpurun_out/bc_$TAG.err || { echo "clustered bench failed"; tail gpurun_out/bc_$TAG.err; exit 3; }
python3 - gpurun_out/bu_$TAG.json gpurun_out/bc_$TAG.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f)); print(f, round(d["ms_per_step"], 2), {k: round(v, 2) if isinstance(v, float) else v for k, v in d["stage_ms"].items()})
PY
