"""Canonical form of a converted point cloud directory.

The reference writes grid points in FxHashMap order (cell.rs:158-160) and
overflow entries in FxHashMap order (cell.rs:164); neither is reproducible, so
parity is defined on:
  * per cell: header values (bit-exact f32), grid points keyed by their slot
    OffsetIndex (recomputed exactly like Cell::read_from, cell.rs:197-203),
  * overflow entries sorted by child index, each list in STORED order,
  * metadata.json compared as parsed values.
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np

import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
from pyref import _bits, _pt, hex_from_world  # noqa: E402

F = np.float32
PT = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("rgba", "u1", (4,))])


def read_cell(path: str, slots: bool = True) -> dict:
    with open(path, "rb") as f:
        data = f.read()
    h, x, y, z, total, number, overflow = struct.unpack_from("<IiiiIII", data, 0)
    size, sub, px, py, pz = struct.unpack_from("<5f", data, 28)
    off = 48
    grid = np.frombuffer(data, dtype=PT, count=number, offset=off)
    off += 16 * number
    nb = data[off]
    off += 1
    buckets = []
    for _ in range(nb):
        cx, cy, cz, n = struct.unpack_from("<iiiI", data, off)
        off += 16
        if n == 0:
            buckets.append(((cx, cy, cz), None))
        else:
            lst = np.frombuffer(data, dtype=PT, count=n, offset=off)
            off += 16 * n
            buckets.append(((cx, cy, cz), [_pt((p["x"], p["y"], p["z"], p["rgba"])) for p in lst]))
    assert off == len(data), f"{path}: trailing bytes"
    cr = F(F(sub) / F(2.0))
    if slots:
        g = sorted((hex_from_world((p["x"], p["y"], p["z"]), cr), _pt((p["x"], p["y"], p["z"], p["rgba"])))
                   for p in grid)
    else:
        g = sorted(_pt((p["x"], p["y"], p["z"], p["rgba"])) for p in grid)
    return dict(id=(h, x, y, z),
                header=(total, number, overflow, _bits(F(size)), _bits(F(sub)),
                        (_bits(F(px)), _bits(F(py)), _bits(F(pz)))),
                grid=g, buckets=sorted(buckets, key=lambda t: t[0]))


def read_dir(out_dir: str, slots: bool = True):
    cells = {}
    with open(os.path.join(out_dir, "metadata.json")) as f:
        meta = json.load(f)
    for name in sorted(os.listdir(out_dir)):
        if not name.startswith("h_"):
            continue
        hdir = os.path.join(out_dir, name)
        for fn in os.listdir(hdir):
            c = read_cell(os.path.join(hdir, fn), slots=slots)
            assert fn == "c_%d_%d_%d.bin" % c["id"][1:], fn
            assert name == "h_%d" % c["id"][0]
            cells[c["id"]] = dict(header=c["header"], grid=c["grid"], buckets=c["buckets"])
    return cells, _meta(meta)


def _f32_or_null(v):
    """A metadata float; serde_json writes a non-finite f32 as null."""
    return None if v is None else float(F(v))


def _meta(meta: dict) -> dict:
    return dict(number_of_points=meta["number_of_points"], hierarchies=meta["hierarchies"],
                bmin=[_f32_or_null(v) for v in meta["bounding_box"]["min"]],
                bmax=[_f32_or_null(v) for v in meta["bounding_box"]["max"]],
                config=dict(meta["config"]))


def diff(a, b, limit: int = 10) -> list[str]:
    """Human-readable differences between two canonical cell dicts."""
    out = []
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            out.append(f"cell {k} only in {'b' if k not in a else 'a'}")
        else:
            ca, cb = a[k], b[k]
            for f in ("header", "grid", "buckets"):
                if ca[f] != cb[f]:
                    if f == "grid":
                        sa, sb = set(ca[f]), set(cb[f])
                        out.append(f"cell {k} grid: {len(sa - sb)} only-a, {len(sb - sa)} only-b")
                    elif f == "buckets":
                        for (ia, la), (ib, lb) in zip(ca[f], cb[f]):
                            if ia != ib or la != lb:
                                out.append(f"cell {k} bucket {ia}/{ib}: "
                                           f"{'None' if la is None else len(la)} vs {'None' if lb is None else len(lb)}")
                        if len(ca[f]) != len(cb[f]):
                            out.append(f"cell {k} #buckets {len(ca[f])} vs {len(cb[f])}")
                    else:
                        out.append(f"cell {k} {f}: {ca[f]} vs {cb[f]}")
        if len(out) >= limit:
            break
    return out


def digest(cells) -> str:
    """Order-independent digest of canonical cells (for large-config fixtures)."""
    import hashlib
    h = hashlib.sha256()
    for k in sorted(cells):
        c = cells[k]
        h.update(repr((k, c["header"], c["grid"], c["buckets"])).encode())
    return h.hexdigest()


def read_dir_fast(out_dir: str):
    """Vectorised canonical form for large outputs: per cell the header, the
    sorted multiset of grid point records (slots are a function of the point
    and the header's sub_cell_size, so equal multisets imply equal slot maps)
    and the overflow entries (child index, None | stored-order bytes)."""
    cells = {}
    with open(os.path.join(out_dir, "metadata.json")) as f:
        meta = json.load(f)
    for name in os.listdir(out_dir):
        if not name.startswith("h_"):
            continue
        hdir = os.path.join(out_dir, name)
        for fn in os.listdir(hdir):
            with open(os.path.join(hdir, fn), "rb") as f:
                data = f.read()
            h, x, y, z, total, number, overflow = struct.unpack_from("<IiiiIII", data, 0)
            hdr = data[16:48]
            grid = np.frombuffer(data, dtype="V16", count=number, offset=48)
            off = 48 + 16 * number
            nb = data[off]
            off += 1
            buckets = []
            for _ in range(nb):
                cx, cy, cz, n = struct.unpack_from("<iiiI", data, off)
                off += 16
                buckets.append(((cx, cy, cz), None if n == 0 else data[off:off + 16 * n]))
                off += 16 * n
            assert off == len(data)
            cells[(h, x, y, z)] = (hdr, np.sort(grid).tobytes(), tuple(sorted(buckets, key=lambda t: t[0])))
    return cells, _meta(meta)


def diff_fast(a, b, limit: int = 10) -> list[str]:
    out = []
    for k in sorted(set(a) | set(b)):
        if k not in a or k not in b:
            out.append(f"cell {k} only in {'b' if k not in a else 'a'}")
        elif a[k] != b[k]:
            ha, ga, ba = a[k]
            hb, gb, bb = b[k]
            what = []
            if ha != hb:
                what.append(f"header {struct.unpack('<III5f', ha)} vs {struct.unpack('<III5f', hb)}")
            if ga != gb:
                what.append(f"grid {len(ga) // 16} vs {len(gb) // 16} pts")
            if ba != bb:
                what.append("buckets " + str([(i, None if l is None else len(l) // 16) for i, l in ba]) + " vs "
                            + str([(i, None if l is None else len(l) // 16) for i, l in bb]))
            out.append(f"cell {k}: " + "; ".join(what))
        if len(out) >= limit:
            break
    return out
