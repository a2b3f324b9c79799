"""ctypes loader for the C oracle — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  Builds oracle/build/liboracle.so on demand with the committed Makefile.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("rgba", "u1", (4,))])


class OrcConfig(C.Structure):
    _fields_ = [("cell_point_overflow_limit", C.c_uint32), ("sub_grid_dimension", C.c_uint32),
                ("max_cell_size", C.c_float)]


_lib = None


def build() -> str:
    srcs = [os.path.join(HERE, f) for f in ("pcc_oracle.c", "digest.c", "digest.h")]
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", HERE, "build/liboracle.so"])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_new.restype = C.c_void_p
        L.orc_new.argtypes = [C.POINTER(OrcConfig)]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_add_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_add_file.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32]
        L.orc_write.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_write.restype = C.c_int
        L.orc_error.argtypes = [C.c_void_p]
        L.orc_error.restype = C.c_int
        L.orc_arrivals.argtypes = [C.c_void_p]
        L.orc_arrivals.restype = C.c_uint64
        L.orc_num_cells.argtypes = [C.c_void_p]
        L.orc_num_cells.restype = C.c_uint64
        L.orc_hierarchies.argtypes = [C.c_void_p]
        L.orc_hierarchies.restype = C.c_uint32
        L.orc_synth.argtypes = [C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, C.c_float, C.c_float, C.c_void_p]
        L.orc_load.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_set_lru.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32]
        L.orc_lru_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.orc_set_level_range.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_pending_count.argtypes = [C.c_void_p]
        L.orc_pending_count.restype = C.c_uint64
        L.orc_pending_get.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_add_batch_raw0.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.orc_cell_get.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_int32), C.POINTER(C.c_uint32)]
        L.orc_cell_grid.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p]
        L.orc_load.restype = C.c_int
        # canonical digests (digest.c)
        L.dg_new.restype = C.c_void_p
        L.dg_free.argtypes = [C.c_void_p]
        L.dg_add_view.argtypes = [C.c_void_p, C.c_void_p]
        L.dg_count.argtypes = [C.c_void_p]
        L.dg_count.restype = C.c_uint64
        L.dg_get.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_int64), C.POINTER(C.c_uint64)]
        L.dg_totals.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.dg_view_size.restype = C.c_uint64
        L.orc_digest.argtypes = [C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def synth(seed: int, kind: int, n: int, first: int = 0, lo: float = -1000.0, ext: float = 2000.0) -> np.ndarray:
    out = np.empty(n, dtype=POINT_DTYPE)
    lib().orc_synth(seed, kind, first, n, lo, ext, out.ctypes.data)
    return out


DEFAULT = dict(cell_point_overflow_limit=5000, sub_grid_dimension=96, max_cell_size=1000.0)


class Oracle:
    """Sequential reference restatement (pcc_oracle.c)."""

    def __init__(self, cfg: dict | None = None):
        cfg = dict(DEFAULT, **(cfg or {}))
        self.cfg = cfg
        c = OrcConfig(cfg["cell_point_overflow_limit"], cfg["sub_grid_dimension"], cfg["max_cell_size"])
        self._h = lib().orc_new(C.byref(c))

    def add_file(self, pts: np.ndarray, batch: int = 10_000):
        pts = np.ascontiguousarray(pts, dtype=POINT_DTYPE)
        lib().orc_add_file(self._h, pts.ctypes.data, len(pts), batch)

    def add_batch(self, pts: np.ndarray):
        pts = np.ascontiguousarray(pts, dtype=POINT_DTYPE)
        lib().orc_add_batch(self._h, pts.ctypes.data, len(pts))

    def set_lru(self, out_dir: str, capacity: int = 100):
        """Mode (A): at most `capacity` cells in memory
        (converter.rs:92), evicted cells written back to out_dir and read back
        when touched again (converter.rs:160-216).  write() must use out_dir."""
        lib().orc_set_lru(self._h, out_dir.encode(), capacity)

    def lru_stats(self) -> dict:
        st = (C.c_uint64 * 2)()
        lib().orc_lru_stats(self._h, st)
        return {"loads": int(st[0]), "evictions": int(st[1])}

    def set_level_range(self, root: int, max_levels: int):
        """Batches enter at level `root`; with max_levels > 0 the points forwarded
        to level root+max_levels are recorded (pending()) instead of added."""
        lib().orc_set_level_range(self._h, root, max_levels)

    def pending(self, with_keys: bool = False):
        """(points, batch number per point, level cell (n,3)[, causing keys]) in
        forwarding order (keys only from add_batch_raw0)."""
        n = lib().orc_pending_count(self._h)
        p = np.zeros(n, dtype=POINT_DTYPE)
        b = np.zeros(n, dtype=np.uint32)
        xyz = np.zeros((n, 3), dtype=np.int32)
        k = np.zeros(n, dtype=np.uint32)
        if n:
            lib().orc_pending_get(self._h, p.ctypes.data, b.ctypes.data, xyz.ctypes.data, k.ctypes.data)
        return (p, b, xyz, k) if with_keys else (p, b, xyz)

    def cells(self):
        """[(h, (x, y, z), grid points)] of every cell (grid only: for raw level-0 pieces)."""
        out = []
        hx, cnt = (C.c_int32 * 4)(), (C.c_uint32 * 3)()
        for i in range(self.num_cells):
            lib().orc_cell_get(self._h, i, hx, cnt)
            g = np.zeros(cnt[1], dtype=POINT_DTYPE)
            if cnt[1]:
                lib().orc_cell_grid(self._h, i, g.ctypes.data)
            out.append((hx[0], (hx[1], hx[2], hx[3]), g))
        return out

    def add_batch_raw0(self, pts: np.ndarray, keys: np.ndarray):
        """Level 0 only, no overflow lists: every emission becomes pending with
        the key of the arrival that caused it."""
        pts = np.ascontiguousarray(pts, dtype=POINT_DTYPE)
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        lib().orc_add_batch_raw0(self._h, pts.ctypes.data, keys.ctypes.data, len(pts))

    def load(self, out_dir: str):
        """Existing converted cloud as the starting state (lib.rs:86-101 +
        converter.rs:187-207): its metadata.json config replaces this oracle's."""
        r = lib().orc_load(self._h, out_dir.encode())
        if r:
            raise OSError(-r, "oracle load failed", out_dir)

    def write(self, out_dir: str):
        r = lib().orc_write(self._h, out_dir.encode())
        if r:
            raise OSError(-r, "oracle write failed", out_dir)

    @property
    def error(self) -> int:
        return lib().orc_error(self._h)

    @property
    def arrivals(self) -> int:
        return lib().orc_arrivals(self._h)

    @property
    def num_cells(self) -> int:
        return lib().orc_num_cells(self._h)

    @property
    def hierarchies(self) -> int:
        return lib().orc_hierarchies(self._h)

    def close(self):
        if self._h:
            lib().orc_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Digest:
    """Canonical digests per level-0 subtree (digest.c): feed cell views of
    either side (the HIP build's pcc_cell_view through pcc_visit_cells, or the
    oracle's own cells), then compare `result()`."""

    def __init__(self):
        self._h = lib().dg_new()

    def add_view(self, view_ptr: int):
        lib().dg_add_view(self._h, C.c_void_p(view_ptr))

    def add_oracle(self, o: "Oracle"):
        lib().orc_digest(o._h, self._h)

    def result(self) -> dict:
        L = lib()
        n = L.dg_count(self._h)
        subs = []
        ai, au = (C.c_int64 * 4)(), (C.c_uint64 * 4)()
        for i in range(n):
            L.dg_get(self._h, i, ai, au)
            subs.append({"subtree": [ai[0], ai[1], ai[2]], "levels": ai[3], "cells": au[0], "points": au[1],
                         "W": au[2], "digest": "%016x" % au[3]})
        t = (C.c_uint64 * 2)()
        L.dg_totals(self._h, t)
        return {"subtrees": subs, "grid_points": t[0], "kept_points": t[1]}

    def close(self):
        if self._h:
            lib().dg_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
