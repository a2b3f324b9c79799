"""Randomised mid-size conversion cases for the GPU-vs-oracle sweep
(tests/test_fuzz_gpu.py): every config knob of metadata.rs:67-88 drawn at random
(sub_grid_dimension 1-96, cell_point_overflow_limit 1-20 000, max_cell_size
0.125-12 345), batch sizes 1-50 000 (lib.rs:11-60 batching), level-0 grids of 1-7
cells per axis (the fold's modulo-2 / modulo-4 paths and the three-pass path),
and point sets that stress the slot replay (cell.rs:70-94): uniform, Gaussian
clusters, planes, lines, lattices (equal distances: key-order ties) and exact
duplicates, split over 1-3 files (one may be empty)."""
import numpy as np

from oracle_ctypes import POINT_DTYPE

DIMS = [1, 2, 3, 5, 8, 13, 16, 24, 32, 47, 64, 80, 95, 96]
CELL_SIZES = [0.125, 1.0, 7.5, 100.0, 1000.0, 12345.0]
KINDS = ["uniform", "gauss", "plane", "line", "lattice"]


def mid_case(seed: int, nonfinite: bool = False, far: float = 0.0):
    """(files, cfg, batch, kind) for one seed; at most ~600 000 points and about
    5 000 cells (each cell is a file the canonical compare reads).  nonfinite:
    ~0.5 % of the points get NaN / +inf / -inf in one or two coordinates
    (bounding-volume/src/lib.rs:23-31, metadata.rs:100-102, cell.rs:77-80)."""
    rng = np.random.default_rng(7919 + seed)
    cs = float(rng.choice(CELL_SIZES))
    dim = int(rng.choice(DIMS))
    limit = int(np.exp(rng.uniform(0.0, np.log(20_000))))
    batch = int(rng.choice([1, 7, 100, 1000, 10_000, 50_000, int(rng.integers(2, 30_000))]))
    n = int(np.exp(rng.uniform(np.log(20_000), np.log(600_000))))
    cap = min(dim ** 3, 20_000) + limit   # points a cell holds, roughly
    n = max(1000, min(n, 5000 * cap))
    if batch < 10:
        n = min(n, 60_000)
    kind = KINDS[seed % len(KINDS)]
    ext = cs * rng.uniform(0.3, 6.5, 3)   # 1-7 level-0 cells per axis
    off = cs * (rng.integers(-3, 4, 3) + rng.uniform(0.0, 1.0, 3))
    if far:   # the cloud moved far from the origin (far cells: f32 spacing near the sub-cell size)
        off = off + cs * far * np.sign(rng.uniform(-1.0, 1.0, 3))
    u = rng.uniform(0.0, 1.0, (n, 3))
    if kind == "gauss":
        k = int(rng.integers(1, 9))
        ctr = rng.uniform(0.0, 1.0, (k, 3))
        sig = rng.uniform(0.01, 0.2, (k, 1))
        c = rng.integers(0, k, n)
        u = np.mod(ctr[c] + rng.standard_normal((n, 3)) * sig[c], 1.0)   # (wrapped: clipping piles points up)
    elif kind == "plane":
        u[:, int(rng.integers(0, 3))] = rng.uniform(0.0, 1.0)
    elif kind == "line":
        a = int(rng.integers(0, 3))
        for b in range(3):
            if b != a:
                u[:, b] = rng.uniform(0.0, 1.0)
    elif kind == "lattice":
        q = int(np.ceil(n ** (1.0 / 3.0) * rng.uniform(1.5, 3.0)))
        u = np.floor(u * q) / q
    xyz = (off + u * ext).astype(np.float32)
    nd = int(n * rng.uniform(0.0, 0.05))   # exact duplicates of earlier points
    if nd:
        dst = rng.integers(1, n, nd)
        src = (rng.uniform(0.0, 1.0, nd) * dst).astype(np.int64)
        xyz[dst] = xyz[src]
    if nonfinite:
        m = max(1, n // 200)
        idx = rng.choice(n, size=m, replace=False)
        specials = np.array([np.nan, np.inf, -np.inf], dtype=np.float32)
        for j, i in enumerate(idx):
            # one or two special axes (all three leave nothing to tell twins
            # apart: more than the limit of them never terminate in the reference)
            for a in rng.choice(3, size=1 + (j % 2), replace=False):
                xyz[i, a] = specials[rng.integers(0, 3)]
    pts = np.zeros(n, dtype=POINT_DTYPE)
    pts["x"], pts["y"], pts["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    pts["rgba"] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    nf = int(rng.integers(1, 4))
    cuts = sorted(int(v) for v in rng.integers(0, n + 1, nf - 1))
    files = [pts[a:b] for a, b in zip([0] + cuts, cuts + [n])]
    cfg = dict(cell_point_overflow_limit=limit, sub_grid_dimension=dim, max_cell_size=cs)
    return files, cfg, batch, kind


def halves(files):
    """(first, second): the case's points cut in two, as two file lists."""
    allp = np.concatenate(files)
    h = len(allp) // 2
    return [allp[:h]], [allp[h:]]


def big_case(seed: int):
    """(files, cfg, batch, kind): 1-6 M points over 1-3 level-0 cells per axis,
    sub-grids of 16-96, so that level 0 and 1 run as dense slabs of thousands
    to hundreds of thousands of arrivals (the 1 024-thread kernel, k_slab)."""
    rng = np.random.default_rng(104729 + seed)
    cs = float(rng.choice(CELL_SIZES))
    dim = int(rng.choice([16, 24, 32, 47, 64, 80, 95, 96]))
    limit = int(np.exp(rng.uniform(np.log(100), np.log(20_000))))
    batch = int(rng.choice([1000, 7777, 10_000, 50_000]))
    n = int(rng.integers(1_000_000, 6_000_000))
    kind = KINDS[seed % len(KINDS)]
    ext = cs * rng.uniform(0.3, 2.5, 3)
    off = cs * (rng.integers(-2, 3, 3) + rng.uniform(0.0, 1.0, 3))
    u = rng.uniform(0.0, 1.0, (n, 3)).astype(np.float32)
    if kind == "gauss":
        k = int(rng.integers(1, 9))
        ctr = rng.uniform(0.0, 1.0, (k, 3))
        sig = rng.uniform(0.02, 0.2, (k, 1))
        c = rng.integers(0, k, n)
        u = np.mod(ctr[c] + rng.standard_normal((n, 3)) * sig[c], 1.0)
    elif kind == "plane":
        u[:, int(rng.integers(0, 3))] = rng.uniform(0.0, 1.0)
    elif kind == "line":   # a thin beam rather than a line: a line of 6 M points piles up
        a = int(rng.integers(0, 3))
        for b in range(3):
            if b != a:
                u[:, b] = rng.uniform(0.0, 0.9) + u[:, b] * 0.05
    elif kind == "lattice":
        q = int(np.ceil(n ** (1.0 / 3.0) * rng.uniform(1.5, 3.0)))
        u = np.floor(u * q) / q
    xyz = (off + u * ext).astype(np.float32)
    pts = np.zeros(n, dtype=POINT_DTYPE)
    pts["x"], pts["y"], pts["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    pts["rgba"] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    nf = int(rng.integers(1, 4))
    cuts = sorted(int(v) for v in rng.integers(0, n + 1, nf - 1))
    files = [pts[a:b] for a, b in zip([0] + cuts, cuts + [n])]
    cfg = dict(cell_point_overflow_limit=limit, sub_grid_dimension=dim, max_cell_size=cs)
    return files, cfg, batch, kind
