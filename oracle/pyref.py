"""pyref.py — TEST INFRASTRUCTURE ONLY.

Two independent pure-Python restatements of the reference `point-converter`
hierarchy/LOD build, used to pin the C oracle (oracle/pcc_oracle.c) and to
check the level-synchronous design the HIP build implements.  Never imported
by the product.  PARITY UNPINNED against the Rust reference itself (it cannot
be built here and ships no fixtures for this path).

* ``convert_sequential`` — batch-by-batch restatement of
  point-converter/src/converter.rs:96-139 and cell.rs:70-153 (hash maps,
  overflow buckets, recursion), with f32 arithmetic done in numpy float32.
* ``convert_keyed``      — the key-ordered, level-synchronous restatement of
  SURVEY.md Appendix C: per level, per (cell, slot) strict prefix-min records
  in key order; emissions keyed by their causing arrival; buckets spill by
  count/batch rules.  This is the algorithm point-cloud_amd/csrc implements.

Both return the canonical form used by tests (see tests/canon.py): a dict
``{(h, x, y, z): CellCanon}`` plus a metadata dict.
"""
from __future__ import annotations

import numpy as np

F = np.float32
SQRT_3 = F(1.73205080757)  # hex.rs:3


def _i32(v) -> int:
    """Rust `f32 as i32` (saturating, NaN -> 0)."""
    v = float(v)
    if v != v:
        return 0
    if v >= 2147483648.0:
        return 2147483647
    if v <= -2147483648.0:
        return -2147483648
    return int(v)  # trunc toward zero


def cell_size(cfg, h: int) -> np.float32:  # metadata.rs:91-93
    return F(cfg["max_cell_size"]) / F(2 ** h)


def sub_cell_size(cfg, cs) -> np.float32:  # metadata.rs:95-97
    return F(cs) / F(cfg["sub_grid_dimension"])


def cell_index(p, cs):  # metadata.rs:100-102
    return tuple(_i32(np.floor(F(p[a]) / F(cs))) for a in range(3))


def cell_pos(idx, cs):  # metadata.rs:104-106
    cs = F(cs)
    return tuple(F(F(idx[a]) * cs) + F(cs / F(2.0)) for a in range(3))


def hex_from_world(p, cr):  # hex.rs:67-85 then to_offset hex.rs:45-51
    cr = F(cr)
    x = F(p[0]) / F(cr * SQRT_3)
    y = F(p[1]) / F(F(-cr) * SQRT_3)
    t = F(SQRT_3 * y) + F(1.0)
    t1 = np.floor(F(t + x))
    t2 = F(t - x)
    t3 = F(F(2.0) * x) + F(1.0)
    qf = F(t1 + t3) / F(3.0)
    rf = F(t1 + t2) / F(3.0)
    q = _i32(np.floor(qf))
    r = -_i32(np.floor(rf))
    h = _i32(F(p[2]) / cr)
    return (q + (r - (r & 1)) // 2, r, h)  # (r - (r&1)) is even: // == Rust /


def hex_to_world(o, cr):  # hex.rs:18-24, 55-65
    cr = F(cr)
    yy = o[1]
    q = o[0] - (yy - (yy & 1)) // 2
    qf, rf, hf = F(q), F(yy), F(o[2])
    X = cr * F(F(SQRT_3 * qf) + F(F(SQRT_3 / F(2.0)) * rf))
    Y = F(F(cr * F(3.0)) / F(2.0)) * rf
    Z = hf * cr
    return (F(X), F(Y), F(Z))


def dist2(c, p):  # glam Vec3::distance_squared
    dx, dy, dz = F(c[0] - F(p[0])), F(c[1] - F(p[1])), F(c[2] - F(p[2]))
    return F(F(F(dx * dx) + F(dy * dy)) + F(dz * dz))


def _pt(p):
    """hashable point: (x, y, z as float32 bit patterns, rgba tuple)."""
    return (int(np.float32(p[0]).view(np.uint32)), int(np.float32(p[1]).view(np.uint32)),
            int(np.float32(p[2]).view(np.uint32)), tuple(int(c) for c in p[3]))


def _pos(pt):
    return tuple(np.uint32(pt[a]).view(np.float32) for a in range(3))


def _unpt(pt):
    """inverse of _pt: (x, y, z float32, rgba tuple)."""
    return _pos(pt) + (pt[3],)


# --------------------------------------------------------------------------- sequential
class _Cell:
    def __init__(self, h, idx, cfg):
        self.h, self.idx = h, idx
        self.size = cell_size(cfg, h)
        self.sub = sub_cell_size(cfg, self.size)
        self.pos = cell_pos(idx, self.size)
        self.total = self.number = self.overflow = 0
        self.grid = {}      # slot -> point
        self.buckets = {}   # child idx -> list | None


def convert_sequential(files, cfg, batch=10_000, prior=None):
    """files: list of point lists (each point = (x, y, z, rgba)).  lib.rs:11-60.

    prior: optional (canonical cells, canonical metadata) of an existing cloud
    (tests/canon.py form) = the state lib.rs:86-101 + converter.rs:187-207
    load from disk before the new files are added (incremental merge)."""
    cells = {}
    meta = dict(number_of_points=0, hierarchies=0, bmin=None, bmax=None)
    if prior is not None:
        pcells, pmeta = prior
        meta = dict(number_of_points=pmeta["number_of_points"], hierarchies=pmeta["hierarchies"],
                    bmin=[F(v) for v in pmeta["bmin"]], bmax=[F(v) for v in pmeta["bmax"]])
        for key, pc in pcells.items():
            c = _Cell(key[0], tuple(key[1:]), cfg)
            c.total, c.number, c.overflow = pc["header"][:3]
            c.grid = {s: _unpt(p) for s, p in pc["grid"]}
            c.buckets = {ci: (None if b is None else [_unpt(p) for p in b]) for ci, b in pc["buckets"]}
            cells[(key[0], tuple(key[1:]))] = c
    L = cfg["cell_point_overflow_limit"]

    def add_in_hierarchy(h, groups):  # converter.rs:114-139
        while True:
            if h >= 31:
                raise RuntimeError("hierarchy depth limit")
            if meta["hierarchies"] <= h:  # create_hierarchy_folder runs even for an empty batch
                meta["hierarchies"] += 1
            nxt = {}
            ccs = cell_size(cfg, h + 1)
            for idx, pts in groups.items():
                c = cells.get((h, idx))
                if c is None:
                    c = cells[(h, idx)] = _Cell(h, idx, cfg)
                over = []
                cr = F(c.sub / F(2.0))
                for p in pts:  # cell.rs:70-106
                    s = hex_from_world(p, cr)
                    if s not in c.grid:
                        c.grid[s] = p
                        c.total += 1
                        c.number += 1
                        continue
                    ctr = hex_to_world(s, F(c.sub / F(2.0)))
                    old = c.grid[s]
                    if dist2(ctr, p) < dist2(ctr, old):
                        c.grid[s] = p
                        over.append(old)
                    else:
                        over.append(p)
                og = {}
                for p in over:
                    og.setdefault(cell_index(p, ccs), []).append(p)
                for ci, lst in og.items():  # cell.rs:108-153
                    if ci not in c.buckets:
                        if len(lst) <= L:
                            c.total += len(lst)
                            c.overflow += len(lst)
                            c.buckets[ci] = list(lst)
                        else:
                            c.buckets[ci] = None
                            nxt.setdefault(ci, []).extend(lst)
                    elif c.buckets[ci] is None:
                        nxt.setdefault(ci, []).extend(lst)
                    else:
                        b = c.buckets[ci]
                        old_len = len(b)
                        b.extend(lst)
                        if len(b) < L:
                            c.total += len(lst)
                            c.overflow += len(lst)
                        else:
                            c.total -= old_len
                            c.overflow -= old_len
                            c.buckets[ci] = None
                            nxt.setdefault(ci, []).extend(b)
            groups = nxt
            if not groups:
                return
            h += 1

    def add_batch(pts):  # converter.rs:96-112
        if pts:
            mn = [F(pts[0][a]) for a in range(3)]
            mx = list(mn)
            for p in pts[1:]:
                for a in range(3):
                    mn[a] = min(mn[a], F(p[a]))
                    mx[a] = max(mx[a], F(p[a]))
            if meta["number_of_points"] == 0:
                meta["bmin"], meta["bmax"] = mn, mx
            else:
                meta["bmin"] = [min(u, v) for u, v in zip(meta["bmin"], mn)]
                meta["bmax"] = [max(u, v) for u, v in zip(meta["bmax"], mx)]
        meta["number_of_points"] += len(pts)
        groups = {}
        cs0 = cell_size(cfg, 0)
        for p in pts:
            groups.setdefault(cell_index(p, cs0), []).append(p)
        add_in_hierarchy(0, groups)

    for f in files:
        off = 0
        while True:
            add_batch(f[off:off + batch])
            off += batch
            if off >= len(f):
                break

    out = {}
    for (h, idx), c in cells.items():
        out[(h,) + idx] = dict(
            header=(c.total, c.number, c.overflow, _bits(c.size), _bits(c.sub), tuple(_bits(v) for v in c.pos)),
            grid=sorted((s, _pt(p)) for s, p in c.grid.items()),
            buckets=sorted((ci, None if b is None else [_pt(p) for p in b]) for ci, b in c.buckets.items()),
        )
    return out, _meta_canon(meta, cfg)


def _bits(v):
    return int(np.float32(v).view(np.uint32))


def _meta_canon(meta, cfg):
    # Aabb::default() is all zeros (bounding-volume/src/lib.rs:4) until a non-empty batch arrives
    return dict(number_of_points=meta["number_of_points"], hierarchies=meta["hierarchies"],
                bmin=[0.0] * 3 if meta["bmin"] is None else [float(v) for v in meta["bmin"]],
                bmax=[0.0] * 3 if meta["bmax"] is None else [float(v) for v in meta["bmax"]],
                config=dict(cfg))


# --------------------------------------------------------------------------- keyed
def convert_keyed(files, cfg, batch=10_000):
    """level-synchronous, key-ordered restatement.

    Arrival key = global input index; event batch = global get_batch counter
    (lib.rs:32 restarts alignment at every file)."""
    L = cfg["cell_point_overflow_limit"]
    arr = []  # (key, eb, point)
    key = 0
    eb = 0
    meta = dict(number_of_points=0, hierarchies=0, bmin=None, bmax=None)
    for f in files:
        off = 0
        while True:
            chunk = f[off:off + batch]
            if chunk:
                mn = [min(F(p[a]) for p in chunk) for a in range(3)]
                mx = [max(F(p[a]) for p in chunk) for a in range(3)]
                if meta["number_of_points"] == 0:
                    meta["bmin"], meta["bmax"] = mn, mx
                else:
                    meta["bmin"] = [min(u, v) for u, v in zip(meta["bmin"], mn)]
                    meta["bmax"] = [max(u, v) for u, v in zip(meta["bmax"], mx)]
            meta["number_of_points"] += len(chunk)
            meta["hierarchies"] = max(meta["hierarchies"], 1)  # empty batch still creates h_0
            for p in chunk:
                arr.append((key, eb, p))
                key += 1
            eb += 1
            off += batch
            if off >= len(f):
                break

    out = {}
    # level 0 arrivals grouped by cell
    cs = cell_size(cfg, 0)
    percell = {}
    for a in arr:
        percell.setdefault(cell_index(a[2], cs), []).append(a)
    h = 0
    while percell:
        if h >= 31:
            raise RuntimeError("hierarchy depth limit")
        meta["hierarchies"] = max(meta["hierarchies"], h + 1)
        ccs = cell_size(cfg, h + 1)
        nxt = {}
        for idx, arrivals in percell.items():
            arrivals.sort(key=lambda t: t[0])
            size = cell_size(cfg, h)
            sub = sub_cell_size(cfg, size)
            cr = F(sub / F(2.0))
            occ = {}  # slot -> (d2, point)
            emis = []  # (key, eb, point)
            for k, e, p in arrivals:
                s = hex_from_world(p, cr)
                ctr = hex_to_world(s, cr)
                d = dist2(ctr, p)
                if s not in occ:
                    occ[s] = (d, p)
                    continue
                od, op = occ[s]
                if d < od:
                    occ[s] = (d, p)
                    emis.append((k, e, op))
                else:
                    emis.append((k, e, p))
            buckets = {}
            for k, e, p in emis:  # already in key order
                buckets.setdefault(cell_index(p, ccs), []).append((k, e, p))
            total = len(occ)
            ovf = 0
            bout = []
            for ci, lst in buckets.items():
                tot = len(lst)
                spilled = tot > L or (tot == L and lst[0][1] != lst[-1][1])
                if not spilled:
                    ovf += tot
                    bout.append((ci, [_pt(p) for _, _, p in lst]))
                    continue
                bout.append((ci, None))
                e0 = lst[0][1]
                if lst[L - 1][1] != e0 or lst[L][1] == e0:
                    sb = lst[L - 1][1]
                else:
                    sb = lst[L][1]
                nxt[ci] = [(k, max(e, sb), p) for k, e, p in lst]
            out[(h,) + idx] = dict(
                header=(total + ovf, total, ovf, _bits(size), _bits(sub),
                        tuple(_bits(v) for v in cell_pos(idx, size))),
                grid=sorted((s, _pt(p)) for s, (d, p) in occ.items()),
                buckets=sorted(bout),
            )
        percell = nxt
        h += 1
    return out, _meta_canon(meta, cfg)


DEFAULT_CONFIG = dict(cell_point_overflow_limit=5000, sub_grid_dimension=96, max_cell_size=1000.0)
