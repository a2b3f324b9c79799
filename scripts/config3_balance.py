#!/usr/bin/env python3
"""Config-3 load balance study (CPU; verdict r1 item 6).

Streams the config-3 generator (synthetic kind 2, seed 3, 100M points in
[-1000,1000)^3; oracle/pcc_oracle.c orc_synth) in chunks, histograms it per
level-0 cell and per level-1 cell, and writes tests/golden/config3_hist.json.
Then reports, for 2/4/8 ranks, the rank loads of assign_owners (whole level-0
cells per rank): max/mean of points and of W (W per level-0 sub-tree from
tests/golden/large_digests.json).  The measured loads with heavy cells shared
slab by slab (plan_split) come from the full-size GPU run,
tests/test_large_gpu.py::test_config3_sharded_8_ranks_split_cells
(profiles/r2_config3_split_balance_8ranks.json).

  python scripts/config3_balance.py [--out profiles/r2_config3_balance.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle_ctypes import synth  # noqa: E402
from pcconv.dist import assign_owners  # noqa: E402

N, SEED, KIND, CHUNK = 100_000_000, 3, 2, 5_000_000


def cell_hist(level):
    cs = np.float32(1000.0 / (1 << level))
    counts = {}
    for a in range(0, N, CHUNK):
        p = synth(SEED, KIND, min(CHUNK, N - a), first=a)
        ix = np.stack([np.floor(p[k] / cs).astype(np.int64) for k in "xyz"], axis=1)
        u, c = np.unique(ix, axis=0, return_counts=True)
        for t, n in zip(map(tuple, u), c):
            counts[t] = counts.get(t, 0) + int(n)
    return counts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r2_config3_balance.json"))
    a = ap.parse_args()
    fix = os.path.join(ROOT, "tests", "golden", "config3_hist.json")
    if not os.path.exists(fix):
        h0, h1 = cell_hist(0), cell_hist(1)
        with open(fix, "w") as f:
            json.dump({"_generator": "scripts/config3_balance.py (orc_synth kind 2, seed 3, 100M)",
                       "level0": [[*map(int, k), int(v)] for k, v in sorted(h0.items())],
                       "level1": [[*map(int, k), int(v)] for k, v in sorted(h1.items())]}, f)
    rep = balance_report(json.load(open(fix)))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps(rep, indent=1))


def grids(fx):
    """Dense level-0 / level-1 grids over the occupied cells (ids z fastest, like
    the shard grid) with the level-0 -> children map."""
    l0 = np.array(fx["level0"], dtype=np.int64)
    l1 = np.array(fx["level1"], dtype=np.int64)
    lo0, hi0 = l0[:, :3].min(0), l0[:, :3].max(0)
    d0 = hi0 - lo0 + 1
    lo1, d1 = 2 * lo0, 2 * d0
    def lin(t, lo, d):
        q = t - lo
        return (q[:, 0] * d[1] + q[:, 1]) * d[2] + q[:, 2]
    hist0 = np.zeros(int(np.prod(d0)), dtype=np.int64)
    hist0[lin(l0[:, :3], lo0, d0)] = l0[:, 3]
    hist1 = np.zeros(int(np.prod(d1)), dtype=np.int64)
    hist1[lin(l1[:, :3], lo1, d1)] = l1[:, 3]
    ids = np.arange(len(hist0))
    t0 = np.stack([ids // (d0[1] * d0[2]) + lo0[0], (ids // d0[2]) % d0[1] + lo0[1], ids % d0[2] + lo0[2]], axis=1)
    ch = np.zeros((len(hist0), 8), dtype=np.int64)
    for o in range(8):
        ch[:, o] = lin(2 * t0 + np.array([o & 1, (o >> 1) & 1, (o >> 2) & 1]), lo1, d1)
    return hist0, hist1, ch, t0


def balance_report(fx):
    hist0, hist1, ch, t0 = grids(fx)
    with open(os.path.join(ROOT, "tests", "golden", "large_digests.json")) as f:
        subs = {tuple(s["subtree"]): s["W"] for s in json.load(f)["config3"]["subtrees"]}
    W = np.array([subs.get(tuple(t), 0) for t in t0.tolist()], dtype=np.int64)
    out = {"input": "config 3 (kind 2, seed 3, 100M)", "level0_cells": int((hist0 > 0).sum()),
           "level1_cells": int((hist1 > 0).sum()), "ranks": {}}
    for world in (2, 4, 8):
        o = assign_owners(hist0, world)
        lp = np.array([hist0[o == r].sum() for r in range(world)])
        lw = np.array([W[o == r].sum() for r in range(world)])
        out["ranks"][str(world)] = {"assign_owners_points_max_over_mean": float(lp.max() / lp.mean()),
                                    "assign_owners_W_max_over_mean": float(lw.max() / lw.mean())}
    return out


if __name__ == "__main__":
    main()
