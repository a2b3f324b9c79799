# refresh round-1 evidence for the current kernels: PMC traffic passes + kernel-trace stats (1B uniform),
# then the config-3 shape (100M clustered) bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
bash $R/scripts/pmc.sh || exit 1
cd $R
timeout -k 10 300 python bench.py --points 100000000 --kind 1 --seed 3 --cpu-sample 10000000 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { echo "c3 bench failed"; exit 4; }
echo refresh-ok
