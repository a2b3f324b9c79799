# RCCL > 2^30-byte self transfer: default, and with RCCL's P2P channels limited
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R && mkdir -p gpurun_out
run() { timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $1 scripts/rccl_probe.py 2>>gpurun_out/rccl_probe.err | grep '"bytes"' >> gpurun_out/rccl_probe.jsonl; }
run 29611 || exit 1
NCCL_MAX_P2P_NCHANNELS=1 run 29612 || exit 2
NCCL_P2P_DISABLE=1 run 29613 || exit 3
NCCL_MIN_P2P_NCHANNELS=4 NCCL_MAX_P2P_NCHANNELS=4 run 29614 || exit 4
cat gpurun_out/rccl_probe.jsonl
