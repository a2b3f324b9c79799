#!/usr/bin/env python3
"""The build of one level-0 octant of config 4 (the rank's share after the
sharded exchange), per octant, in ONE process: does the octant decide the
build time (the 22 ms ranks of profiles/r3_stages_config4_8ranks_onepass.json)?
Prints one JSON line per octant with the best of 3 build times and the stage
split, then the same for the whole cloud."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))
import torch  # noqa: E402
import pcconv  # noqa: E402


def timed_build(pts, keys=None, reps=3):
    c = pcconv.Converter("/tmp/pcc_octant_probe", batch_size=10_000)
    try:
        c.set_profiling(True) if hasattr(c, "set_profiling") else None
        torch.cuda.synchronize()   # the points come from torch's stream
        c.add_points_device(pts.data_ptr(), pts.shape[0])
        best, st = None, None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s = c.build()
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) * 1e3
            if best is None or t < best:
                best, st = t, s
        return best, st
    finally:
        c.close()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    dev = torch.device("cuda", 0)
    # generated and split in chunks of 125M points (tensors below 2^31 elements:
    # boolean-mask selection over a 4e9-element tensor returned corrupt rows here)
    chunk = 125_000_000
    parts = [[] for _ in range(8)]
    for a in range(0, n, chunk):
        m = min(chunk, n - a)
        pts = torch.empty((m, 4), dtype=torch.int32, device=dev)
        pcconv.synth_device(pts.data_ptr(), a, m, 4, 0, -1000.0, 2000.0, 0)
        torch.cuda.synchronize()
        f = pts.view(torch.float32)
        code = (f[:, 0] < 0).to(torch.int32) | ((f[:, 1] < 0).to(torch.int32) << 1) | ((f[:, 2] < 0).to(torch.int32) << 2)
        for o in range(8):
            parts[o].append(pts[code == o].clone())
        del pts, f, code
    torch.cuda.synchronize()
    for o in range(8):
        sel = torch.cat(parts[o]).contiguous()
        parts[o] = None
        ms, st = timed_build(sel)
        print(json.dumps({"octant": o, "neg_xyz": [o & 1, (o >> 1) & 1, (o >> 2) & 1], "points": int(sel.shape[0]),
                          "build_ms": round(ms, 3), "levels": st.get("levels"), "cells": st.get("cells"),
                          "slabs": st.get("slabs"), "arrivals": st.get("arrivals")}), flush=True)
        del sel
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
