"""Diagnostic: the sharded path under torchrun + RCCL (TorchComm) against a
single-converter build of the same synthetic points (canonical compare).
Usage: torchrun --nproc-per-node W scripts/sharded_check.py N [kind]"""
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import pcconv  # noqa: E402
from pcconv.dist import HipShardOps, TorchComm, key_range, shard_build  # noqa: E402

n = int(sys.argv[1])
kind = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
local = int(os.environ.get("LOCAL_RANK", "0"))
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
out = sys.argv[3] if len(sys.argv) > 3 else "/tmp/pcc_sharded_check"
a, b = key_range(n, rank, world)
pts = torch.empty((b - a, 4), dtype=torch.int32, device=dev)
pcconv.synth_device(pts.data_ptr(), a, b - a, 7, kind, -1000.0, 2000.0, local)
torch.cuda.synchronize()
ops = HipShardOps(local, out_dir=os.path.join(out, "sharded"))
res = shard_build(TorchComm(dev), ops, pts, a, [n], write=True)
ops.close()
dist.barrier()
if rank == 0:
    ref = os.path.join(out, "single")
    c = pcconv.Converter(ref, device=local)
    c.add_synthetic(7, kind, n)
    c.finish()
    from gpu_util import compare_dirs
    d, ma, mb = compare_dirs(os.path.join(out, "sharded"), ref, fast=True)
    print("sharded-check n=%d world=%d recv=%d diff=%d meta_equal=%s" % (n, world, res.recv_points, len(d), ma == mb),
          flush=True)
    if d:
        print(d[:5])
dist.destroy_process_group()
