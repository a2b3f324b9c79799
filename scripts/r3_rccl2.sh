# RCCL > 2^30-byte self transfer: first bad byte vs size and element type
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
PROBE_SWEEP=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=COLL,P2P timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29621 scripts/rccl_probe.py > gpurun_out/rccl_sweep.out 2> gpurun_out/rccl_sweep.err || exit 1
grep '"sweep"' gpurun_out/rccl_sweep.out
