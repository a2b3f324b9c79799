# DIAGNOSTIC: dense-slab grid extraction variants (make -C point-cloud_amd gxvar), per-level k_slab times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
for v in base 24576_8 24576_12 8192_4 0_4; do
  if [ $v = base ]; then export PCC_LIB=$R/point-cloud_amd/build/libpcconv.so; else export PCC_LIB=$R/point-cloud_amd/build/gx_$v/libpcconv.so; fi
  bash scripts/ktrace.sh gx_$v > gpurun_out/gx_$v.txt || { echo "variant $v failed"; exit 1; }
  echo "$v: $(grep -E 'k_slab<' gpurun_out/gx_$v.txt | awk '{print $1}' | tr '\n' ' ') $(tail -1 gpurun_out/gx_$v.txt)"
done
