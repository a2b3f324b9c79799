# round-3 GPU check: parity suite, default bench, kernel trace, stamped diagnostic build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-q3}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bu_$TAG.json 2> gpurun_out/bu_$TAG.err || { echo "bench failed"; tail gpurun_out/bu_$TAG.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/bu_$TAG.json'));print(round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)}, round(d['roofline']['frac'],3))"
bash scripts/ktrace.sh kt_$TAG | grep -v "k_bucket\|k_next" || exit 3
PCC_LIB=$R/point-cloud_amd/build/stamps/libpcconv.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/stamps_$TAG.json 2> gpurun_out/stamps_$TAG.err || { echo "stamps failed"; exit 4; }
grep stamps gpurun_out/stamps_$TAG.err
