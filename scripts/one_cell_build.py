#!/usr/bin/env python3
"""Three builds of one level-0 cell of uniform points (a rank's octant of
config 4 after the sharded exchange: 125M points in [0, 1000)^3), for a kernel
trace of the per-rank build."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))
import pcconv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
c = pcconv.Converter("/tmp/pcc_onecell", batch_size=10_000)
c.add_synthetic(4, 0, n, 0.0, 1000.0)
for r in range(3):
    t0 = time.perf_counter()
    s = c.build()
    print(f"build {r}: {(time.perf_counter() - t0) * 1e3:.2f} ms levels {s['levels']} arrivals {s['arrivals']}", flush=True)
c.close()
