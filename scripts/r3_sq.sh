# SQ counters of the slab kernels at 1B (config 4, one build per pass), three passes,
# separate runs, kernel trace only besides the counters (no other trace domains).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/sq3
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/sq3/a -o a -- $B > $R/gpurun_out/sq3/a.json 2> $R/gpurun_out/sq3/a.err || { echo "pass a failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/sq3/b -o b -- $B > $R/gpurun_out/sq3/b.json 2> $R/gpurun_out/sq3/b.err || { echo "pass b failed"; exit 2; }
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/sq3/counters.txt 2>&1 || true
echo sq-ok
