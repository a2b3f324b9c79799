"""Diagnostic (not part of the product): what the second half of a > 2^30-byte
RCCL self transfer (world 1) holds, and whether limiting RCCL's point-to-point
channels changes it.  One 1.25 GiB uint8 all_to_all_single and P2P send/recv:
the first bad byte, and whether the bad region is untouched (still the fill
value), a copy of the first half, or shifted data.
  torchrun --nproc-per-node 1 scripts/rccl_probe.py   (env: NCCL_* knobs)"""
import json
import os

import torch
import torch.distributed as dist

dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
if os.environ.get("PROBE_SWEEP"):   # first bad byte vs message size (MiB) and element type, all_to_all_single
    out = []
    for mib, dt in ((1023, torch.uint8), (1025, torch.uint8), (1280, torch.uint8), (1536, torch.uint8),
                    (2047, torch.uint8), (1280, torch.int32), (1280, torch.int64)):
        n = (mib << 20) // torch.tensor([], dtype=dt).element_size()
        x = (torch.arange(n, dtype=torch.int64, device=dev) * 7 % 251).to(dt)
        y = torch.full((n,), 255, dtype=dt, device=dev)
        dist.all_to_all_single(y, x, [n], [n])
        torch.cuda.synchronize()
        bad = torch.nonzero(x != y)
        b0 = int(bad[0].item()) * x.element_size() if bad.numel() else None
        out.append({"mib": mib, "dtype": str(dt), "elements": n, "first_bad_byte": b0,
                    "first_bad_over_bytes": None if b0 is None else b0 / (mib << 20),
                    "untouched": bool(torch.all(y[bad[0]:] == 255).item()) if bad.numel() else None})
        del x, y
        torch.cuda.empty_cache()
    print(json.dumps({"sweep": out}), flush=True)
    dist.destroy_process_group()
    raise SystemExit(0)
n = 1280 << 20
x = (torch.arange(n, dtype=torch.int64, device=dev) * 7 % 251).to(torch.uint8)
res = {"env": {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))}, "bytes": n}
for mode in ("a2a", "p2p"):
    y = torch.full((n,), 255, dtype=torch.uint8, device=dev)   # 255: never produced by x (values < 251)
    if mode == "a2a":
        dist.all_to_all_single(y, x, [n], [n])
    else:
        for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, x, 0), dist.P2POp(dist.irecv, y, 0)]):
            r.wait()
    torch.cuda.synchronize()
    bad = torch.nonzero(x != y)
    r = {"equal": bool(bad.numel() == 0)}
    if bad.numel():
        b0 = int(bad[0].item())
        tail = y[b0:]
        r["first_bad_byte"] = b0
        r["first_bad_over_bytes"] = b0 / n
        r["bad_bytes"] = int(bad.numel())
        r["bad_region_untouched"] = bool(torch.all(tail == 255).item())
        h = n - b0
        r["bad_region_equals_first_part"] = bool(torch.equal(tail, x[:h])) if h <= b0 else None
        # shifted: does y[b0:b0+4096] occur in x at another offset (mod 251 pattern: offset = shift)
        probe = y[b0:b0 + 8].tolist()
        r["probe"] = probe
    res[mode] = r
print(json.dumps(res), flush=True)
dist.destroy_process_group()
