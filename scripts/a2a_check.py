"""Diagnostic: RCCL all_to_all_single round trip at world 1 for a given number of 16-B rows
(raw call, then TorchComm.alltoallv with its chunking)."""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from pcconv.dist import TorchComm  # noqa: E402

n = int(sys.argv[1])
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.arange(n * 4, dtype=torch.int32, device=dev).view(n, 4)
y = torch.empty_like(x)
dist.all_to_all_single(y, x, [n], [n])
torch.cuda.synchronize()
print("raw rows=%d equal=%s" % (n, bool(torch.equal(x, y))), flush=True)
del y
z = TorchComm(dev).alltoallv(x, [n], [n])
torch.cuda.synchronize()
print("chunked rows=%d equal=%s" % (n, bool(torch.equal(x, z))), flush=True)
dist.destroy_process_group()
