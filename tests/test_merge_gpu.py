"""GPU parity of the incremental merge (config 5 shape; lib.rs:86-101 +
converter.rs:187-207): the HIP build opened on a
directory that already holds a converted cloud, fed new files, must write
exactly the cloud the sequential oracle produces when it converts the old and
the new files in one run (the equivalence tests/test_merge_oracle.py pins on
the CPU).  The existing cloud is written by the oracle, or by the HIP build
itself, so both writers' files are read back."""
import os
import shutil
import tempfile

import pytest

from gpu_util import compare_dirs, run_gpu, run_oracle  # noqa: E402
from oracle_ctypes import synth  # noqa: E402
from test_merge_oracle import _split  # noqa: E402
from test_oracle_xcheck import _case, _to_np  # noqa: E402

pytestmark = pytest.mark.gpu


def _merge_check(first, second, cfg=None, batch=10_000, prior_by="oracle", fast=False):
    with tempfile.TemporaryDirectory() as tg, tempfile.TemporaryDirectory() as to:
        if prior_by == "oracle":
            err, _ = run_oracle(tg, first, cfg=cfg, batch=batch)
            assert err == 0
        else:
            run_gpu(tg, first, cfg=cfg, batch=batch)
        st = run_gpu(tg, second, cfg=None, batch=batch)   # config comes from the existing metadata.json
        err, _ = run_oracle(to, first + second, cfg=cfg, batch=batch)
        assert err == 0
        d, mg, mo = compare_dirs(tg, to, fast=fast)
        assert d == [], d
        assert mg == mo
        assert st["grid_points"] + st["kept_points"] == st["number_of_points"]
        return st


@pytest.mark.parametrize("seed", range(40))
def test_merge_adversarial_small(seed):
    files, cfg, batch = _case(seed)
    first, second = _split(files, seed)
    _merge_check([_to_np(f) for f in first], [_to_np(f) for f in second], cfg=cfg, batch=batch)


def test_merge_uniform_prior_from_gpu():
    pts = synth(21, 0, 400_000)
    _merge_check([pts[:300_000]], [pts[300_000:]], prior_by="gpu", fast=True)


def test_merge_clustered_deep():
    a = synth(22, 1, 600_000)
    b = synth(23, 1, 250_000)
    st = _merge_check([a], [b[:100_000], b[100_000:]], fast=True)
    assert st["levels"] >= 3


@pytest.mark.parametrize("seed", [3, 11, 29])
def test_merge_with_every_seed_record_flagged(seed, monkeypatch):
    """The grid seeds' slot-table records made at adoption (k_seed_rec) all
    flagged (PCC_NO_SEED_REC): every seed goes through the kernels' own slot and
    route arithmetic instead, with the same result (cell.rs:183-229)."""
    monkeypatch.setenv("PCC_NO_SEED_REC", "1")
    files, cfg, batch = _case(seed)
    first, second = _split(files, seed)
    _merge_check([_to_np(f) for f in first], [_to_np(f) for f in second], cfg=cfg, batch=batch)
    a = synth(22, 1, 600_000)
    b = synth(23, 1, 250_000)
    _merge_check([a], [b], fast=True)


@pytest.mark.parametrize("seed", [5, 17])
def test_merge_with_bucket_resolution_in_two_launches(seed, monkeypatch):
    """A merge (existing Some / None buckets, cell.rs:108-153) through the
    two-launch bucket resolution, forced at every level (PCC_BKT_SPLIT_MIN=1)."""
    monkeypatch.setenv("PCC_BKT_SPLIT_MIN", "1")
    files, cfg, batch = _case(seed)
    first, second = _split(files, seed)
    _merge_check([_to_np(f) for f in first], [_to_np(f) for f in second], cfg=cfg, batch=batch)
    pts = synth(24, 0, 60_000, lo=-40.0, ext=80.0)
    cfg = dict(cell_point_overflow_limit=1500, sub_grid_dimension=6, max_cell_size=64.0)
    _merge_check([pts[:20_000], pts[20_000:30_000]], [pts[30_000:]], cfg=cfg, batch=777)


def test_merge_small_limit_spills_kept_lists():
    """Tiny limit: existing Some lists spill in the merge, existing None buckets forward."""
    pts = synth(24, 0, 60_000, lo=-40.0, ext=80.0)
    cfg = dict(cell_point_overflow_limit=4, sub_grid_dimension=6, max_cell_size=64.0)
    _merge_check([pts[:20_000], pts[20_000:30_000]], [pts[30_000:]], cfg=cfg, batch=777)


def test_merge_no_new_points_keeps_cloud():
    pts = synth(25, 0, 50_000)
    with tempfile.TemporaryDirectory() as tg, tempfile.TemporaryDirectory() as to:
        run_oracle(to, [pts])
        shutil.rmtree(tg)
        shutil.copytree(to, tg)
        run_gpu(tg, [pts[:0]])
        d, mg, mo = compare_dirs(tg, to, fast=False)
        assert d == [] and mg == mo


def test_adopt_prior_equals_directory_merge():
    """pcc_adopt_prior (bench.py config 5, no files) == opening the directory."""
    import pcconv
    a = synth(26, 0, 200_000)
    b = synth(27, 0, 80_000)
    with tempfile.TemporaryDirectory() as t0, tempfile.TemporaryDirectory() as t1, \
            tempfile.TemporaryDirectory() as to:
        src = pcconv.Converter(t0)
        src.add_points(a)
        src.build()
        dst = pcconv.Converter(t1)
        dst.adopt_prior(src)
        src.close()
        dst.add_points(b)
        st = dst.build()
        dst.write()
        dst.close()
        run_oracle(to, [a, b])
        d, mg, mo = compare_dirs(t1, to, fast=True)
        assert d == [] and mg == mo
        assert st["number_of_points"] == 280_000


@pytest.mark.parametrize("meta", ["removed", "zero_points"])
def test_stale_cells_merge_like_the_reference(meta):
    """Cell files without a valid cloud behind them (metadata.json missing, or a
    metadata.json that counts no points: a run that never reached Drop,
    converter.rs:241-246).  The reference opens every touched cell's existing
    file (converter.rs:187-207) whatever lib.rs:86-101 found, so the stale cells
    are merged while the counters start again from metadata.json or zero.  The
    HIP build must write what the oracle (orc_load: metadata optional, every cell
    file) writes for the same directory."""
    import json
    from gpu_util import Oracle
    cfg = dict(sub_grid_dimension=16, cell_point_overflow_limit=100)
    old, new = [synth(71, 1, 200_000)], [synth(72, 1, 80_000)]
    with tempfile.TemporaryDirectory() as tg, tempfile.TemporaryDirectory() as to:
        run_gpu(tg, old, cfg=cfg)
        mp = os.path.join(tg, "metadata.json")
        if meta == "removed":
            os.remove(mp)
        else:
            m = json.load(open(mp))
            m["number_of_points"], m["hierarchies"] = 0, 0
            m["bounding_box"] = {"min": [0.0, 0.0, 0.0], "max": [0.0, 0.0, 0.0]}
            json.dump(m, open(mp, "w"), indent=2)
        shutil.rmtree(to)
        shutil.copytree(tg, to)
        o = Oracle(cfg)
        o.load(to)
        for f in new:
            o.add_file(f, 10_000)
        assert o.error == 0
        o.write(to)
        o.close()
        run_gpu(tg, new, cfg=cfg)
        d, mg, mo = compare_dirs(tg, to)
        assert d == [], d
        assert mg == mo
        assert mg["number_of_points"] == len(new[0])


def test_poisoned_device_cache_parity_and_merge():
    """PCC_POISON_CACHE=1 fills every block the device cache hands out again with
    0xFF: a read of memory the build never wrote then changes cell contents.  Two
    rounds of a plain build and a merge (the second round runs on recycled blocks)
    against the oracle's digests."""
    import pcconv
    pcconv.release_device_cache()
    old = os.environ.get("PCC_POISON_CACHE")
    os.environ["PCC_POISON_CACHE"] = "1"
    try:
        a = synth(25, 1, 300_000)
        b = synth(26, 0, 200_000)
        for _ in range(2):
            _merge_check([a], [b[:120_000], b[120_000:]], prior_by="gpu", fast=True)
            files, cfg, batch = _case(7)
            first, second = _split(files, 7)
            _merge_check([_to_np(f) for f in first], [_to_np(f) for f in second], cfg=cfg, batch=batch)
    finally:
        if old is None:
            os.environ.pop("PCC_POISON_CACHE", None)
        else:
            os.environ["PCC_POISON_CACHE"] = old
        pcconv.release_device_cache()


def test_merge_small_slab_with_large_child_rooms():
    """A merge whose level-0 slabs are small (a dim-8 layer holds <= 196 grid
    seeds, plus a few new points: the one-wave kernel) while their 24 child
    slabs hold ~36 000 seeds each (level-1 cells that kept lists of ~94 000
    points under a limit of 200 000): the slab's destination span is far above
    2^16, so a displaced seed's position must not pass through a 16-bit field.
    The new points sit exactly at the slot centres of 400 existing points, so
    each displaces its slot's grid seed (d^2 = 0, cell.rs:77-80)."""
    import numpy as np
    import pyref
    cfg = dict(sub_grid_dimension=8, cell_point_overflow_limit=200_000, max_cell_size=1000.0)
    old = synth(71, 0, 6_000_000, lo=0.0, ext=999.0)
    cr = pyref.sub_cell_size(cfg, pyref.cell_size(cfg, 0)) / np.float32(2.0)
    pick = old[np.random.default_rng(5).choice(len(old), 400, replace=False)]
    new = pick.copy()
    for i, p in enumerate(pick):
        c = pyref.hex_to_world(pyref.hex_from_world((p["x"], p["y"], p["z"]), cr), cr)
        new[i]["x"], new[i]["y"], new[i]["z"] = c
    _merge_check([old], [new], cfg=cfg, fast=True)
