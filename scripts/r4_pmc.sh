# round 4: HBM traffic (FETCH/WRITE passes + kernel trace) and SQ counters of the benched tree (1B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
bash scripts/pmc.sh || exit 1
sed -i 's/--points 200000000 //' scripts/pmc_sq.sh
bash scripts/pmc_sq.sh || exit 2
echo r4-pmc-ok
