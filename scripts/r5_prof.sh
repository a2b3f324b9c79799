# round 5 profiles of the benched 1B workload (config 4): kernel stats + FETCH/WRITE passes
# (scripts/pmc.sh) and the SQ passes (scripts/pmc_sq.sh), all under gpurun_out/.  Summaries
# (made where gpurun_out/ was merged back):
#   python3 scripts/pmc_summary.py gpurun_out <tag>_pmc_traffic_1b gpurun_out/pmc_fetch.json
#   python3 scripts/ktsum.py gpurun_out/ktrace/kt_kernel_trace.csv > profiles/<tag>_kernel_trace_1b.txt
#   python3 scripts/sq_summary.py gpurun_out/sq k_slab k_l0 > profiles/<tag>_pmc_sq_1b.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
bash scripts/pmc.sh || exit 2
python3 scripts/ktsum.py gpurun_out/ktrace/kt_kernel_trace.csv || exit 3
bash scripts/pmc_sq.sh 1000000000 || exit 4
