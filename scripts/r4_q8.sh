# round 4: folded level-0 pass 1 behind the upload: parity (pieces), GPU suite subset, PCIe-inclusive A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
PCC_PRE6=1 timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_inputs_gpu.py tests/test_nonfinite_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_t8.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4_t8.log; exit 2; }
tail -2 gpurun_out/r4_t8.log
for v in pre6 pre0 pre6; do
  if [ $v = pre0 ]; then unset PCC_PRE6; else export PCC_PRE6=1; fi
  timeout -k 10 300 python -u scripts/pcie_bench.py > gpurun_out/r4_pcie_$v.json 2> gpurun_out/r4_pcie_$v.err || { echo "pcie $v failed"; tail -5 gpurun_out/r4_pcie_$v.err; exit 3; }
  echo $v; cat gpurun_out/r4_pcie_$v.json
done
