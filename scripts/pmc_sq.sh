# SQ counters of the slab kernels (two passes, separate runs, no trace domains besides the kernel trace).
# Argument: points of the bench build (default: the benched 1B workload).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
PTS=${1:-1000000000}
mkdir -p $R/gpurun_out/sq
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/sq/counters.txt 2>&1 || true
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/sq/a -o a -- python3 $R/bench.py --points $PTS --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/sq/a.json 2> $R/gpurun_out/sq/a.err || { echo "pass a failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/sq/b -o b -- python3 $R/bench.py --points $PTS --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/sq/b.json 2> $R/gpurun_out/sq/b.err || { echo "pass b failed"; exit 2; }
echo sq-ok
