"""Pin the C oracle against two independent Python restatements (CPU only).

The reference has no executable form or fixtures here (parity unpinned,
SURVEY.md §8c), so the oracle is pinned by agreement of three restatements:
  * oracle/pcc_oracle.c            — sequential, hash maps (the checker)
  * oracle/pyref.convert_sequential — sequential, written independently
  * oracle/pyref.convert_keyed      — SURVEY Appendix C level-synchronous form
on adversarial small cases: tiny sub-grids, tiny overflow limits, tiny
batches, half-step quantised coordinates and exact duplicates (ties).
"""
import os
import random
import sys
import tempfile

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, HERE)

import canon  # noqa: E402
import pyref  # noqa: E402
from oracle_ctypes import POINT_DTYPE, Oracle  # noqa: E402


def _case(seed):
    rng = random.Random(seed)
    n = rng.randint(40, 500)
    dim = rng.randint(1, 3)
    L = rng.randint(1, 7)
    batch = rng.randint(1, 40)
    step = rng.choice([125.0, 250.0, 62.5, 0.0])
    pts = []
    for _ in range(n):
        if pts and rng.random() < 0.1:
            pts.append(pts[rng.randrange(len(pts))])  # exact duplicate
            continue
        p = []
        for _ in range(3):
            v = rng.uniform(-2000, 2000)
            if step:
                v = round(v / step) * step
            p.append(np.float32(v))
        pts.append((p[0], p[1], p[2], (rng.randrange(256), rng.randrange(256), rng.randrange(256), 255)))
    nfiles = rng.randint(1, 3)
    cuts = sorted(rng.randint(0, n) for _ in range(nfiles - 1))
    files, prev = [], 0
    for c in cuts + [n]:
        files.append(pts[prev:c])
        prev = c
    cfg = dict(cell_point_overflow_limit=L, sub_grid_dimension=dim, max_cell_size=1000.0)
    return files, cfg, batch


def _to_np(pts):
    a = np.zeros(len(pts), dtype=POINT_DTYPE)
    for i, p in enumerate(pts):
        a[i] = (p[0], p[1], p[2], p[3])
    return a


def _oracle(files, cfg, batch, tmp):
    o = Oracle(cfg)
    for f in files:
        o.add_file(_to_np(f), batch)
    assert o.error == 0
    o.write(tmp)
    return canon.read_dir(tmp)


@pytest.mark.parametrize("seed", range(60))
def test_three_restatements_agree(seed):
    files, cfg, batch = _case(seed)
    seq, mseq = pyref.convert_sequential(files, cfg, batch)
    key, mkey = pyref.convert_keyed(files, cfg, batch)
    assert canon.diff(seq, key) == []
    assert seq == key
    assert mseq == mkey
    with tempfile.TemporaryDirectory() as tmp:
        cells, meta = _oracle(files, cfg, batch, tmp)
    assert canon.diff(seq, cells) == []
    assert cells == seq
    assert meta == mseq


def test_default_config_uniform_small():
    """Default config (L=5000, dim 96), 30k uniform points over 3 files."""
    from oracle_ctypes import synth
    pts = synth(7, 0, 30_000)
    py = [(p["x"], p["y"], p["z"], tuple(p["rgba"])) for p in pts]
    files = [py[:12_345], py[12_345:12_345], py[12_345:]]
    cfg = dict(pyref.DEFAULT_CONFIG)
    key, mkey = pyref.convert_keyed(files, cfg)
    with tempfile.TemporaryDirectory() as tmp:
        o = Oracle(cfg)
        for f in (pts[:12_345], pts[12_345:12_345], pts[12_345:]):
            o.add_file(f)
        o.write(tmp)
        cells, meta = canon.read_dir(tmp)
    assert canon.diff(key, cells) == []
    assert meta == mkey


def test_empty_input_file():
    """An empty file still runs one empty batch: h_0 exists, hierarchies == 1 (converter.rs:141-158)."""
    cfg = dict(pyref.DEFAULT_CONFIG)
    seq, mseq = pyref.convert_sequential([[]], cfg)
    key, mkey = pyref.convert_keyed([[]], cfg)
    assert seq == key == {}
    assert mseq == mkey and mseq["hierarchies"] == 1 and mseq["number_of_points"] == 0
    with tempfile.TemporaryDirectory() as tmp:
        o = Oracle(cfg)
        o.add_file(np.zeros(0, dtype=POINT_DTYPE))
        o.write(tmp)
        cells, meta = canon.read_dir(tmp)
        assert os.path.isdir(os.path.join(tmp, "h_0"))
    assert cells == {} and meta == mseq
