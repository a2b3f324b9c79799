# round 4, first GPU call: level-0 run-read probe, then the extra-VALU A/B of the dense kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 ./scripts/run_probe > gpurun_out/r4_run_probe.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r4_run_probe.log; exit 1; }
cat gpurun_out/r4_run_probe.log
bash scripts/ab.sh r4xv > gpurun_out/r4xv.log 2>&1; rc=$?
tail -30 gpurun_out/r4xv.log
exit $rc
