# round 4: pending GPU checks: pre6 (upload-time pass 1) parity + PCIe A/B, the 5+6-bit level-0 binning (PCC_L0_SWAP)
# parity + A/B, device-side level start, KF dense variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
PCC_PRE6=1 timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py tests/test_nonfinite_gpu.py tests/test_merge_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_t9.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4_t9.log; exit 2; }
tail -2 gpurun_out/r4_t9.log
for v in swap base swap base; do
  if [ $v = swap ]; then export PCC_L0_SWAP=1; else unset PCC_L0_SWAP; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/r4_b9_$v.json 2> gpurun_out/r4_b9_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r4_b9_$v.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4_b9_$v.json'));print('$v', round(d['ms_per_step'],2),{k:round(v,2) for k,v in d['stage_ms'].items() if isinstance(v,float)})"
done
unset PCC_L0_SWAP
PCC_L0_SWAP=1 bash scripts/ktrace.sh r4_kt9s > gpurun_out/r4_kt9s.txt; head -5 gpurun_out/r4_kt9s.txt
for v in pre6 pre0; do
  if [ $v = pre0 ]; then unset PCC_PRE6; else export PCC_PRE6=1; fi
  timeout -k 10 300 python -u scripts/pcie_bench.py > gpurun_out/r4_pcie_$v.json 2> gpurun_out/r4_pcie_$v.err || { echo "pcie $v failed"; tail -5 gpurun_out/r4_pcie_$v.err; exit 4; }
  echo $v; cat gpurun_out/r4_pcie_$v.json
done
