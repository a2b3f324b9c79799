# DIAGNOSTIC: dense-slab prefetch depth 2 (product) vs 3 (make -C point-cloud_amd pf3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
PCC_LIB=$R/point-cloud_amd/build/pf3/libpcconv.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_golden.py tests/test_parity_gpu.py -k "not cli" > gpurun_out/pf3_t.log 2>&1 || { echo "pf3 parity failed"; tail -20 gpurun_out/pf3_t.log; exit 1; }
tail -1 gpurun_out/pf3_t.log
for v in base pf3 base pf3; do
  if [ $v = base ]; then export PCC_LIB=$R/point-cloud_amd/build/libpcconv.so; else export PCC_LIB=$R/point-cloud_amd/build/pf3/libpcconv.so; fi
  bash scripts/ktrace.sh pf_$v > gpurun_out/pf_$v.txt || { echo "variant $v failed"; exit 1; }
  echo "$v: $(grep -E 'k_slab<' gpurun_out/pf_$v.txt | awk '{print $1}' | tr '\n' ' ') $(tail -1 gpurun_out/pf_$v.txt)"
done
