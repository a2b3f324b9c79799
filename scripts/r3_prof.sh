# round-3 profiles of the 1B bench build: HBM traffic (FETCH/WRITE passes), kernel stats, SQ counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
bash $R/scripts/pmc.sh || exit 1
bash $R/scripts/r3_sq.sh || exit 2
