# per-stage timing of the sharded step, one process per rank on one MI355X (gloo)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/rank_stages.py --config 3 --world 8 > gpurun_out/stages_c3.json 2> gpurun_out/stages_c3.err || { echo "c3 failed"; tail -20 gpurun_out/stages_c3.err; exit 1; }
echo c3-ok
timeout -k 10 600 python -u scripts/rank_stages.py --config 4 --world 8 > gpurun_out/stages_c4.json 2> gpurun_out/stages_c4.err || { echo "c4 failed"; tail -20 gpurun_out/stages_c4.err; exit 2; }
echo c4-ok
