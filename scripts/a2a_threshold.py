"""Diagnostic (not part of the product): where does a single RCCL all_to_all_single
at world 1 start returning wrong data?  Same byte counts as int32 rows and as
uint8 elements (element-count vs byte-count overflow), around 2^30 and 2^31
bytes, plus grouped P2P send/recv to self of the same sizes.
  torchrun --nproc-per-node 1 scripts/a2a_threshold.py"""
import os
import torch
import torch.distributed as dist

dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)


def check(nbytes, dtype):
    es = torch.empty((), dtype=dtype).element_size()
    n = nbytes // es
    x = torch.arange(n, dtype=torch.int64, device=dev).to(dtype) if dtype != torch.uint8 else \
        (torch.arange(n, dtype=torch.int64, device=dev) % 251).to(torch.uint8)
    y = torch.zeros_like(x)
    dist.all_to_all_single(y, x, [n], [n])
    torch.cuda.synchronize()
    ok = bool(torch.equal(x, y))
    bad = "" if ok else " first bad element %d (byte %d)" % (int(torch.nonzero(x != y)[0].item()), int(torch.nonzero(x != y)[0].item()) * es)
    print("a2a %-12s bytes=%d (2^%.3f) elements=%d equal=%s%s" % (str(dtype), nbytes, torch.log2(torch.tensor(float(nbytes))).item(), n, ok, bad), flush=True)
    del y
    z = torch.zeros_like(x)
    ops = [dist.P2POp(dist.isend, x, 0), dist.P2POp(dist.irecv, z, 0)]
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    torch.cuda.synchronize()
    print("p2p %-12s bytes=%d equal=%s" % (str(dtype), nbytes, bool(torch.equal(x, z))), flush=True)
    del x, z
    torch.cuda.empty_cache()


for nb in [(1 << 30) - 4096, 1 << 30, (1 << 30) + 4096, 1200 << 20, 1600 << 20, (1 << 31) - 4096, (1 << 31) + 4096]:
    for dt in (torch.int32, torch.uint8):
        check(nb, dt)
dist.destroy_process_group()
