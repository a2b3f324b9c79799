# SQ counters for the slab kernels (separate --pmc passes; no trace domains mixed in)
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/pmc1 -o run --output-format csv -- python $R/bench.py --points 200000000 --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS -d $R/gpurun_out/pmc2 -o run --output-format csv -- python $R/bench.py --points 200000000 --steps 1 --warmup 0 --cpu-sample 0 > $R/gpurun_out/pmc2.log 2>&1 || exit 1
