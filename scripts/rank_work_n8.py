#!/usr/bin/env python3
"""Diagnostic: the per-rank GPU work of one config-4 step at N = 8, measured
on one GPU without the exchange: the route of a rank's 125M-point key range
(8 destinations) and the build of one octant's 125M points."""
import json, os, sys, time
import torch
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))
import pcconv  # noqa: E402
from pcconv.dist import shard_grid  # noqa: E402

torch.cuda.init()
dev = torch.device("cuda", 0)
n = 125_000_000
pts = torch.empty((n, 4), dtype=torch.int32, device=dev)
pcconv.synth_device(pts.data_ptr(), 0, n, 4, 0, -1000.0, 2000.0, 0)
torch.cuda.synchronize()
g = shard_grid([-1000.0] * 3, [999.99] * 3, 1000.0)
owner = torch.arange(g.ncells, dtype=torch.int32, device=dev) % 8
send = torch.empty_like(pts)
keys = torch.empty(n, dtype=torch.int32, device=dev)
out = {}
for name, fn in [("bbox", lambda: pcconv.shard_bbox(pts.data_ptr(), n)),
                 ("slab_hist", lambda: pcconv.shard_slab_histogram(pts.data_ptr(), n, g, 96, torch.empty(g.ncells * 256, dtype=torch.int32, device=dev).data_ptr())),
                 ("route", lambda: pcconv.shard_route(pts.data_ptr(), n, 0, g, owner.data_ptr(), 8, send.data_ptr(), keys.data_ptr()))]:
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    out[name + "_ms"] = (time.perf_counter() - t0) / 5 * 1e3
# one octant's build (125M uniform points in [0,1000)^3)
c = pcconv.Converter("/tmp/pcc_rank_n8")
c.add_synthetic(4, 0, n, 0.0, 1000.0)
c.build()
t0 = time.perf_counter()
for _ in range(5):
    st = c.build()
out["octant_build_ms"] = (time.perf_counter() - t0) / 5 * 1e3
c.close()
# the same octant handed over with keys, as a rank receives it after the exchange
oct_pts = torch.empty((n, 4), dtype=torch.int32, device=dev)
pcconv.synth_device(oct_pts.data_ptr(), 0, n, 4, 0, 0.0, 1000.0, 0)
oct_keys = torch.arange(n, dtype=torch.int32, device=dev) * 8
torch.cuda.synchronize()
c = pcconv.Converter("/tmp/pcc_rank_n8k")
c.declare_files([8 * n])
c.set_keyed_points_device(oct_pts.data_ptr(), oct_keys.data_ptr(), n)
c.build()
t0 = time.perf_counter()
for _ in range(5):
    st = c.build()
out["octant_build_keyed_ms"] = (time.perf_counter() - t0) / 5 * 1e3

c.close()
print(json.dumps(out))
