"""CPU test double of pcconv.dist.HipShardOps — TEST INFRASTRUCTURE ONLY.

Lets the sharded orchestration (pcconv/dist.py: bbox/histogram all-reduce,
owner table, all-to-all-v routing, global metadata) run on CPU ranks (gloo or
threads).  Local histogram/route are numpy restatements of the HIP kernels in
point-cloud_amd/csrc/engine.hip (shard section); the per-shard build is the C
oracle fed batch by batch with the GLOBAL batch structure (lib.rs:31-52), which
is exactly what the keyed GPU build must reproduce.
"""
from __future__ import annotations

import json
import os
import shutil
import tempfile

import numpy as np
import torch

import pcconv
from oracle_ctypes import POINT_DTYPE, Oracle


def as_points(t: torch.Tensor) -> np.ndarray:
    return np.ascontiguousarray(t.cpu().numpy()).view(POINT_DTYPE).reshape(-1)


def as_tensor(p: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(p, dtype=POINT_DTYPE).view(np.int32).reshape(-1, 4).copy())


def cell_index(v: np.ndarray, cs: float) -> np.ndarray:
    """metadata.rs:100-102 per axis: (floor(p / cs) as f32) as i32, saturating."""
    q = np.floor(v.astype(np.float32) / np.float32(cs)).astype(np.float64)
    return np.clip(q, -2147483648.0, 2147483647.0).astype(np.int64)


class NumpyShardOps:
    def __init__(self, out_dir: str, batch_size: int = 10_000, config: dict | None = None, merge: bool = False):
        self.out_dir = out_dir
        self.batch = batch_size
        self.cfg = dict(config or {})
        self.max_cell_size = float(self.cfg.get("max_cell_size", 1000.0))
        self.oracle = None
        self.merge = merge
        self.subtree_dir = None

    def prior_meta(self):
        from pcconv.dist import read_prior_meta
        return read_prior_meta(self.out_dir)

    def set_subtrees(self, cells):
        """Merge mode: a copy of the existing cloud holding only the cells below
        these level-0 cells (what pcc_open_subtrees loads), for the oracle's loader."""
        keep = {tuple(int(v) for v in c) for c in np.asarray(cells).reshape(-1, 3)}
        if self.subtree_dir is not None:
            shutil.rmtree(self.subtree_dir, ignore_errors=True)
        d = self.subtree_dir = tempfile.mkdtemp(prefix="pcc_np_subtrees_")
        shutil.copy(os.path.join(self.out_dir, "metadata.json"), d)
        for name in os.listdir(self.out_dir):
            if not name.startswith("h_"):
                continue
            h = int(name[2:])
            os.makedirs(os.path.join(d, name), exist_ok=True)
            for fn in os.listdir(os.path.join(self.out_dir, name)):
                x, y, z = (int(v) for v in fn[2:-4].split("_"))
                if (x >> h, y >> h, z >> h) in keep:
                    shutil.copy(os.path.join(self.out_dir, name, fn), os.path.join(d, name, fn))

    def bbox(self, pts):
        p = as_points(pts)
        return ([float(p[a].min()) for a in "xyz"], [float(p[a].max()) for a in "xyz"])

    def grid(self, gmin, gmax):
        return pcconv.shard_grid_from_bbox(gmin, gmax, self.max_cell_size)   # host-only C-ABI helper

    def _cells(self, p, grid):
        ix = [cell_index(p[a], grid.cell_size) - grid.lo[i] for i, a in enumerate("xyz")]
        d = [int(v) for v in grid.dims]
        assert all(((v >= 0) & (v < d[i])).all() for i, v in enumerate(ix))
        return (ix[0] * d[1] + ix[1]) * d[2] + ix[2]

    def histogram(self, pts, grid):
        c = self._cells(as_points(pts), grid)
        return torch.from_numpy(np.bincount(c, minlength=grid.ncells).astype(np.int32))

    def route(self, pts, key0, grid, owner, world):
        p = as_points(pts)
        own = owner.cpu().numpy().astype(np.int64)[self._cells(p, grid)]
        order = np.argsort(own, kind="stable")
        counts = np.bincount(own, minlength=world)[:world]
        keys = (key0 + order).astype(np.uint32).view(np.int32)
        return as_tensor(p[order]), torch.from_numpy(keys.copy()), [int(c) for c in counts]

    def build(self, file_points, pts, keys) -> dict:
        p = as_points(pts)
        k = (np.arange(len(p), dtype=np.int64) if keys is None
             else keys.cpu().numpy().view(np.uint32).astype(np.int64))
        assert (np.diff(k) > 0).all(), "keyed input must arrive in global key order"
        if self.oracle is not None:
            self.oracle.close()
        o = self.oracle = Oracle(self.cfg)
        if self.merge:
            o.load(self.subtree_dir)
        g = 0
        for fp in file_points:
            off = 0
            while True:   # lib.rs:31-52 (do-while: an empty file is one empty batch)
                m = min(self.batch, fp - off)
                lo, hi = np.searchsorted(k, g + off), np.searchsorted(k, g + off + m)
                o.add_batch(p[lo:hi])
                off += m
                if off >= fp:
                    break
            g += fp
        assert o.error == 0
        return {"hierarchies": o.hierarchies, "arrivals": o.arrivals, "cells": o.num_cells, "levels": o.hierarchies,
                "slabs": 0}

    def write(self, summary, cells: bool, metadata: bool):
        os.makedirs(self.out_dir, exist_ok=True)
        if cells:
            tmp = tempfile.mkdtemp(prefix="pcc_np_shard_")
            try:
                self.oracle.write(tmp)
                for name in os.listdir(tmp):
                    if name.startswith("h_"):
                        os.makedirs(os.path.join(self.out_dir, name), exist_ok=True)
                        for fn in os.listdir(os.path.join(tmp, name)):
                            shutil.copy(os.path.join(tmp, name, fn), os.path.join(self.out_dir, name, fn))
            finally:
                shutil.rmtree(tmp, ignore_errors=True)
        if metadata:
            cfg = dict(dict(cell_point_overflow_limit=5000, sub_grid_dimension=96, max_cell_size=1000.0), **self.cfg)
            meta = {"version": "1.0", "name": "Unknown", "number_of_points": summary["number_of_points"],
                    "hierarchies": summary["hierarchies"],
                    "bounding_box": {"min": [float(np.float32(v)) for v in summary["bbox_min"]],
                                     "max": [float(np.float32(v)) for v in summary["bbox_max"]]},
                    "config": cfg}
            with open(os.path.join(self.out_dir, "metadata.json"), "w") as f:
                json.dump(meta, f, indent=2)

    def close(self):
        if self.oracle is not None:
            self.oracle.close()
            self.oracle = None
        if self.subtree_dir is not None:
            shutil.rmtree(self.subtree_dir, ignore_errors=True)
            self.subtree_dir = None
