# round-1 GPU pass: parity suite, bench (with CPU baseline), kernel-trace profile of the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/t_full.log 2>&1 || { echo "pytest failed rc=$?"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err || { echo "bench failed rc=$?"; exit 2; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o r1 -- python3 $R/bench.py --cpu-sample 0 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err || { echo "rocprof failed rc=$?"; exit 3; }
echo done
