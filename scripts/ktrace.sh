# per-launch kernel durations of one 1B build (kernel trace only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-kt}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG -o kt -- python3 $R/bench.py --steps 1 --warmup 1 --cpu-sample 0 ${@:2} > $R/gpurun_out/$TAG.json 2> $R/gpurun_out/$TAG.err || { echo "ktrace failed"; tail -5 $R/gpurun_out/$TAG.err; exit 1; }
python3 $R/scripts/ktsum.py $R/gpurun_out/$TAG/kt_kernel_trace.csv
