#!/usr/bin/env python3
"""Generate the golden fixtures of tests/golden/ — TEST INFRASTRUCTURE.

The reference (Rust) cannot be built here and holds no fixtures or known-answer
tests for this path, so these vectors are PARITY-UNPINNED
against the reference binary.  Each vector is accepted only when three
independent restatements agree on it bit for bit (canonical form, tests/canon.py):
  * oracle/pyref.convert_sequential  (pure Python, batch by batch, hash maps)
  * oracle/pyref.convert_keyed       (pure Python)
  * oracle/pcc_oracle.c              (C, sequential)
Large cases store only an order-independent digest.

Usage:  python tests/golden/make_golden.py        (rewrites tests/golden/*.json)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import canon  # noqa: E402
import pyref  # noqa: E402
from oracle_ctypes import POINT_DTYPE, Oracle, synth  # noqa: E402

F = np.float32


def P(x, y, z, c=(0, 0, 0, 255)):
    return (F(x), F(y), F(z), tuple(c))


def case_slot_ties():
    """One sub-grid slot, equidistant arrivals: strict '<' keeps the old point
    (cell.rs:84-90); a closer arrival replaces and emits the occupant."""
    r = 250.0   # dim 2: sub cell 500, hex radius 250; slot (0,0,0) centre at the origin region
    pts = [P(10, 10, 10, (1, 0, 0, 255)), P(-10, -10, 10, (2, 0, 0, 255)), P(10, 10, 10, (3, 0, 0, 255)),
           P(1, 1, 1, (4, 0, 0, 255)), P(-1, -1, 1, (5, 0, 0, 255)), P(1, 1, 1, (6, 0, 0, 255)),
           P(0.5, 0.5, 0.5, (7, 0, 0, 255)), P(r * 0.9, 0, 0, (8, 0, 0, 255)), P(-r * 0.9, 0, 0, (9, 0, 0, 255))]
    return [pts], dict(cell_point_overflow_limit=2, sub_grid_dimension=2, max_cell_size=1000.0), 3


def case_limit_spill():
    """Overflow buckets (cell.rs:108-153): Some(list) below/at the limit, None
    after a spill within one batch and across batches, forwards to level 1."""
    rng = np.random.default_rng(5)
    pts = [P(*(rng.uniform(0, 999, 3).astype(F)), (i % 256, 7, 7, 255)) for i in range(60)]
    pts += [P(400, 400, 400, (9, 9, 9, 9))] * 5   # duplicates
    return [pts], dict(cell_point_overflow_limit=3, sub_grid_dimension=1, max_cell_size=1000.0), 4


def case_boundaries():
    """Exact cell boundaries, signed zeros, hex z-layer truncation at +-r,
    large and tiny magnitudes."""
    vals = [0.0, -0.0, 1000.0, -1000.0, 999.99994, -1e-7, 1e-7, 1e6, -1e6, 500.0, -500.0, 2.6041667, -2.6041667]
    pts = []
    k = 0
    for a in vals:
        for b in vals[::3]:
            for c in vals[::4]:
                pts.append(P(a, b, c, (k % 256, k // 256, 0, 255)))
                k += 1
    return [pts], dict(cell_point_overflow_limit=2, sub_grid_dimension=3, max_cell_size=1000.0), 7


def case_ragged_files():
    """Several input files incl. an empty one: a file end is a batch boundary (lib.rs:31-52)."""
    a = synth(41, 0, 7)
    c = synth(42, 1, 13, lo=-50.0, ext=100.0)
    f = lambda arr: [P(p["x"], p["y"], p["z"], tuple(p["rgba"])) for p in arr]  # noqa: E731
    return [f(a), [], f(c)], dict(cell_point_overflow_limit=2, sub_grid_dimension=2, max_cell_size=1000.0), 5


def case_synthetic_deep():
    """Clustered points, tiny sub-grid and limit: deep hierarchy."""
    a = synth(43, 1, 2500)
    pts = [P(p["x"], p["y"], p["z"], tuple(p["rgba"])) for p in a]
    return [pts], dict(cell_point_overflow_limit=8, sub_grid_dimension=2, max_cell_size=1000.0), 500


CASES = {
    "slot_ties": case_slot_ties,
    "limit_spill": case_limit_spill,
    "boundaries": case_boundaries,
    "ragged_files": case_ragged_files,
    "synthetic_deep": case_synthetic_deep,
}

# larger: digest only (SURVEY §8d config 1 = 100 000 uniform points, seed 1, default config)
DIGEST_CASES = {
    "config1_uniform_100k": (1, 0, 100_000, None, 10_000),
    "clustered_50k_small_grid": (3, 1, 50_000, dict(cell_point_overflow_limit=100, sub_grid_dimension=8,
                                                     max_cell_size=1000.0), 2_000),
}


def to_np(pts):
    a = np.zeros(len(pts), dtype=POINT_DTYPE)
    for i, p in enumerate(pts):
        a[i] = (p[0], p[1], p[2], p[3])
    return a


def oracle_canon(files_np, cfg, batch):
    o = Oracle(cfg)
    for f in files_np:
        o.add_file(f, batch)
    assert o.error == 0
    with tempfile.TemporaryDirectory() as d:
        o.write(d)
        o.close()
        return canon.read_dir(d)


def jsonable(x):
    if isinstance(x, (tuple, list)):
        return [jsonable(v) for v in x]
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    return x


def canon_json(cells, meta):
    return {"cells": [{"id": list(k), "header": jsonable(c["header"]), "grid": jsonable(c["grid"]),
                       "buckets": jsonable(c["buckets"])} for k, c in sorted(cells.items())],
            "metadata": jsonable(meta)}


def records_hex(files_np):
    return [f.tobytes().hex() for f in files_np]


def main():
    for name, fn in CASES.items():
        files, cfg, batch = fn()
        seq, mseq = pyref.convert_sequential(files, cfg, batch)
        key, mkey = pyref.convert_keyed(files, cfg, batch)
        files_np = [to_np(f) for f in files]
        orc, morc = oracle_canon(files_np, cfg, batch)
        assert seq == key == orc, (name, canon.diff(seq, orc)[:3], canon.diff(seq, key)[:3])
        assert mseq == mkey, name
        assert {k: v for k, v in morc.items() if k != "config"} == {k: v for k, v in mseq.items() if k != "config"}
        out = {"case": name, "doc": fn.__doc__.strip(), "config": cfg, "batch": batch,
               "files_hex": records_hex(files_np), "expected": canon_json(orc, morc),
               "agreement": "pyref.convert_sequential == pyref.convert_keyed == pcc_oracle.c"}
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(out, f, indent=1)
        print(name, len(orc), "cells")
    for name, (seed, kind, n, cfg, batch) in DIGEST_CASES.items():
        cfgd = dict(dict(cell_point_overflow_limit=5000, sub_grid_dimension=96, max_cell_size=1000.0), **(cfg or {}))
        arr = synth(seed, kind, n)
        files = [[P(p["x"], p["y"], p["z"], tuple(p["rgba"])) for p in arr]]
        seq, mseq = pyref.convert_sequential(files, cfgd, batch)
        orc, morc = oracle_canon([arr], cfgd, batch)
        assert seq == orc, (name, canon.diff(seq, orc)[:3])
        out = {"case": name, "synth": {"seed": seed, "kind": kind, "n": n, "lo": -1000.0, "extent": 2000.0},
               "config": cfgd, "batch": batch, "cells": len(orc), "digest": canon.digest(orc),
               "metadata": jsonable(morc),
               "input_sha256": hashlib.sha256(arr.tobytes()).hexdigest(),
               "agreement": "pyref.convert_sequential == pcc_oracle.c"}
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(out, f, indent=1)
        print(name, len(orc), "cells (digest)")


if __name__ == "__main__":
    main()
