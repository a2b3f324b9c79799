"""Inputs with NaN and +-inf coordinates mixed into a multi-level cloud (the
reference's semantics for them: bounding-volume/src/lib.rs:23-31 f32::min/max
skip NaN; metadata.rs:100-102 and hex.rs:67-85 `as i32` saturates, NaN -> 0;
cell.rs:77-80 `new_distance < old_distance` is false for NaN).  Shared by the
oracle test (CPU) and the GPU parity test."""
import numpy as np

from oracle_ctypes import synth

NONFINITE_CFG = {"sub_grid_dimension": 8, "cell_point_overflow_limit": 40, "max_cell_size": 1000.0}


def nonfinite_files(seed: int = 7, n: int = 120_000, kinds: str = "mixed"):
    """Two files: a clustered cloud around the origin (so cells touching x = 0
    or y = 0 hold finite points in the slot (0, 0) a NaN x or y maps to), with
    ~3 % of the points given NaN / +inf / -inf coordinates in every
    combination, plus exact duplicates of some of them.  kinds="nan": NaN only."""
    rng = np.random.default_rng(seed)
    base = synth(seed, 1, n, lo=-300.0, ext=600.0)
    near = synth(seed + 1, 0, n // 10, lo=-8.0, ext=16.0)   # finite points around the origin slots
    pts = np.concatenate([base, near])
    rng.shuffle(pts)
    m = len(pts) // 30
    idx = rng.choice(len(pts), size=m, replace=False)
    specials = np.array([np.nan, np.inf, -np.inf] if kinds == "mixed" else [np.nan], dtype=np.float32)
    for j, i in enumerate(idx):
        # one or two special axes: with all three special a point has no finite
        # coordinate to separate it from its twins, and more than the overflow
        # limit of them descend without end (the reference overflows at h = 32)
        axes = rng.choice(3, size=1 + (j % 2), replace=False)
        for a in axes:
            v = specials[rng.integers(0, len(specials))] if j % 5 else np.float32(np.nan)
            pts[i][("x", "y", "z")[a]] = v
    dup = pts[idx[: m // 8]].copy()
    pts = np.concatenate([pts, dup])
    cut = len(pts) // 3
    return [pts[:cut], pts[cut:]]
