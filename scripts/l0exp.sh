# DIAGNOSTIC: level-0 single-upsweep binning, pass-1 group count x pass-2 unit size
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
for cfg in ${L0EXP_CFGS:-"512 8192" "2048 8192" "512 2048"}; do
  set -- $cfg
  export PCC_L0_GROUPS=$1 PCC_L0_UNIT_DIV=$2
  bash scripts/ktrace.sh l0e_$1_$2 > gpurun_out/l0e_$1_$2.txt || exit 1
  echo "groups=$1 div=$2: $(grep -E 'down6g|down5g|gprefix' gpurun_out/l0e_$1_$2.txt | awk '{print $1}' | tr '\n' ' ') $(tail -1 gpurun_out/l0e_$1_$2.txt)"
done
