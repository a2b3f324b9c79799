#!/usr/bin/env python3
"""Diagnostic (not part of the product): measured work of every level-1 and
level-2 sub-tree of a synthetic configuration, next to the point counts the
sharding plan sees, for calibrating pcconv.dist.plan_split's cost model.

Builds the configuration on cuda:0, walks its cells (pcc_visit_cells) and sums
W = sum (h+1) * total over each ancestor; histograms the input per level-1/-2
cell on the device.  Writes gpurun_out/subtree_work_<seed>_<kind>_<n>.json.

  python scripts/subtree_work.py --seed 3 --kind 2 --n 100000000
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))
import pcconv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--kind", type=int, default=2)
    ap.add_argument("--n", type=int, default=100_000_000)
    a = ap.parse_args()
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    pts = torch.empty((a.n, 4), dtype=torch.int32, device=dev)
    pcconv.synth_device(pts.data_ptr(), 0, a.n, a.seed, a.kind, -1000.0, 2000.0, 0)
    torch.cuda.synchronize()
    xyz = pts[:, :3].view(torch.float32)
    hist = {}
    for lv in (1, 2, 3):
        cs = 1000.0 / (1 << lv)
        ix = torch.floor(xyz / cs).to(torch.int64)
        u, c = torch.unique(ix, dim=0, return_counts=True)
        hist[lv] = {",".join(map(str, t)): int(n) for t, n in zip(u.cpu().tolist(), c.cpu().tolist())}
    conv = pcconv.Converter("/tmp/pcc_subtree_work", batch_size=10_000, device=0)
    conv.add_points_device(pts.data_ptr(), a.n)
    st = conv.build()
    work = {1: {}, 2: {}}

    def visit(vp):
        v = pcconv.CellView.from_address(vp)
        w = (v.hierarchy + 1) * v.total_number_of_points
        for lv in (1, 2):
            if v.hierarchy >= lv:
                s = v.hierarchy - lv
                k = f"{v.x >> s},{v.y >> s},{v.z >> s}"
                work[lv][k] = work[lv].get(k, 0) + w
        return 0

    conv.visit_cells(visit)
    conv.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = os.path.join(ROOT, "gpurun_out", f"subtree_work_{a.seed}_{a.kind}_{a.n}.json")
    with open(out, "w") as f:
        json.dump({"arrivals": st["arrivals"], "hist": hist, "work": work}, f)
    print(out, st["arrivals"])


if __name__ == "__main__":
    main()
