# round-1 GPU pass: parity suite, bench (with CPU baseline), kernel-trace profile of the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-pass}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed rc=$?"; exit 2; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --cpu-sample 0 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/prof_$TAG.err || { echo "rocprof failed rc=$?"; exit 3; }
echo done
