# round 4: upload-time pass 1 by default: upload tests, PCIe-inclusive A/B (interleaved)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "upload_in_pieces or config1 or ragged or clustered" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_t10.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4_t10.log; exit 2; }
tail -2 gpurun_out/r4_t10.log
for v in pre6 pre0; do
  if [ $v = pre0 ]; then export PCC_NO_PRE6=1; else unset PCC_NO_PRE6; fi
  timeout -k 10 300 python -u scripts/pcie_bench.py > gpurun_out/r4_pcie2_$v.json 2> gpurun_out/r4_pcie2_$v.err || { echo "pcie $v failed"; tail -5 gpurun_out/r4_pcie2_$v.err; exit 4; }
  echo $v; cat gpurun_out/r4_pcie2_$v.json
done
