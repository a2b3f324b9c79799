# SQ counters of the slab kernels (one pass, 8 SQ slots), 200M-point build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq -o sq -- python3 $R/bench.py --points 200000000 --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/pmc_sq.json 2> $R/gpurun_out/pmc_sq.err || { echo "sq pass failed"; exit 1; }
echo sq-ok
