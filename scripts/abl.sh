# dense slab kernel ablations (diagnostic builds; timings only; later levels may fail)
R=${GRAFT_REPO_ROOT:-$PWD}
for a in ${ABL:-8 16 32 56}; do
  echo "== abl $a"
  PCC_LIB=$R/point-cloud_amd/build/abl$a/libpcconv.so bash $R/scripts/ktrace.sh abl$a > /dev/null 2>&1
  python3 $R/scripts/ktsum.py $R/gpurun_out/abl$a/kt_kernel_trace.csv | grep "k_slab(" | head -2
done
