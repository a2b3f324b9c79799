"""Mode (A) of the CPU baseline: the oracle with the reference's
LRU cell cache (converter.rs:92 capacity, converter.rs:160-216 write-back and
reload) must write the same cloud as the in-memory mode (B): the cache changes
I/O, not results.  Small capacities force evictions and reloads of cells with
grid points, Some lists and None buckets."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import canon  # noqa: E402
from oracle_ctypes import Oracle, synth  # noqa: E402


def _convert(out, files, cfg, lru=None, batch=10_000):
    o = Oracle(cfg)
    if lru is not None:
        o.set_lru(out, lru)
    for f in files:
        o.add_file(f, batch)
    st = o.lru_stats()
    assert o.error == 0
    o.write(out)
    o.close()
    return st


@pytest.mark.parametrize("cap", [1, 3, 100])
def test_lru_mode_a_equals_in_memory(tmp_path, cap):
    cfg = dict(cell_point_overflow_limit=40, sub_grid_dimension=6, max_cell_size=100.0)
    files = [synth(31, 1, 30_000, lo=-300.0, ext=600.0), synth(32, 0, 7_000, lo=-300.0, ext=600.0)]
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    st = _convert(a, files, cfg, lru=cap, batch=2_000)
    _convert(b, files, cfg)
    if cap < 100:
        assert st["evictions"] > 0 and st["loads"] > 0
    ca, ma = canon.read_dir(a)
    cb, mb = canon.read_dir(b)
    assert canon.diff(ca, cb) == []
    assert ma == mb


def test_lru_mode_a_merge_equals_in_memory(tmp_path):
    """Config-5 shape in mode (A): the existing cloud's cells are read lazily from
    the output directory (converter.rs:187-207) while new points merge in."""
    cfg = dict(cell_point_overflow_limit=40, sub_grid_dimension=6, max_cell_size=100.0)
    first = [synth(33, 0, 20_000, lo=-300.0, ext=600.0)]
    second = [synth(34, 1, 9_000, lo=-300.0, ext=600.0)]
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    _convert(a, first, cfg)
    o = Oracle(cfg)
    o.set_lru(a, 2)
    for f in second:
        o.add_file(f, 3_000)
    assert o.error == 0 and o.lru_stats()["loads"] > 0
    o.write(a)
    o.close()
    _convert(b, first + second, cfg)
    ca, ma = canon.read_dir(a)
    cb, mb = canon.read_dir(b)
    assert canon.diff(ca, cb) == []
    assert ma == mb
