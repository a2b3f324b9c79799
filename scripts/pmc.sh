# HBM traffic of the 1B bench build (MI355X_MICROARCH.md "HBM [CDNA4]"): FETCH_SIZE and
# WRITE_SIZE in separate passes (TCC slots), kernel trace in the same passes; then a
# --kernel-trace --stats pass for per-kernel durations.  One build per pass (no warmup).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PCC_VERBOSE=1 timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o fetch -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/pmc_fetch.json 2> $R/gpurun_out/pmc_fetch.err || { echo "fetch pass failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o write -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/pmc_write.json 2> $R/gpurun_out/pmc_write.err || { echo "write pass failed"; exit 2; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ktrace -o kt -- python3 $R/bench.py --cpu-sample 0 > $R/gpurun_out/ktrace.json 2> $R/gpurun_out/ktrace.err || { echo "ktrace pass failed"; exit 3; }
echo pmc-ok
