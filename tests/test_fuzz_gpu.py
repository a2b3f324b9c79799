"""Randomised GPU-vs-oracle sweep (tests/fuzz_cases.py): 48 mid-size cases with
every config knob, batch size, level-0 grid shape and point pattern drawn at
random, converted by the HIP build through the C ABI and by the C oracle, and
compared on the canonical form (per cell: header bytes, the grid multiset, the
overflow lists in stored order; metadata values).  Every fourth case is also run
as a merge: the first half written by the oracle, the second half merged into it
by the HIP build (lib.rs:86-101), against the oracle's one-run conversion.  16
larger cases (1-6 M points in 1-3 level-0 cells per axis) run the dense slab
kernel on slabs of thousands to hundreds of thousands of arrivals."""
import os
import tempfile

import pytest

from fuzz_cases import big_case, halves, mid_case
from gpu_util import compare_dirs, run_gpu, run_oracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _shm():
    return "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None


def _explain(files, ga, gb):
    """For the first cell whose canonical forms differ: its first differing
    overflow list (or grid) on both sides as input indices (a plain build's keys)."""
    import numpy as np
    import canon
    ca, cb = canon.read_dir_fast(ga)[0], canon.read_dir_fast(gb)[0]
    allp = np.concatenate(files)
    index = {}
    for i in range(len(allp)):
        index.setdefault(bytes(allp[i].tobytes()), i)
    ids = lambda blob: [index.get(bytes(blob[j:j + 16]), -1) for j in range(0, len(blob or b""), 16)]
    for k in sorted(set(ca) & set(cb)):
        if ca[k] == cb[k]:
            continue
        if ca[k][1] != cb[k][1]:
            return f"cell {k} grid: {sorted(ids(ca[k][1]))[:32]} vs {sorted(ids(cb[k][1]))[:32]}"
        for (ia, la), (ib, lb) in zip(ca[k][2], cb[k][2]):
            if la != lb:
                return f"cell {k} child {ia}: {ids(la)[:64]} vs {ids(lb)[:64]}"
    return "?"


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_matches_oracle(seed):
    import pcconv
    files, cfg, batch, kind = mid_case(seed)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        err, arrivals = run_oracle(to, files, cfg=cfg, batch=batch)
        if err:   # (a case the reference cannot convert: the GPU build must refuse it too)
            with pytest.raises(pcconv.PccError):
                run_gpu(tg, files, cfg=cfg, batch=batch)
            return
        st = run_gpu(tg, files, cfg=cfg, batch=batch)
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d, _explain(files, to, tg))
        assert mg == mo
        assert st["arrivals"] == arrivals
        assert st["grid_points"] + st["kept_points"] == st["number_of_points"]
        assert st["sequential_replay"] == 0   # (the parallel levels, not the fallback)


@pytest.mark.parametrize("seed", range(0, 48, 4))
def test_fuzz_merge_matches_oracle(seed):
    files, cfg, batch, kind = mid_case(seed)
    pts = [f for f in files if len(f)]
    allp = pts[0] if len(pts) == 1 else __import__("numpy").concatenate(pts)
    h = len(allp) // 2
    first, second = [allp[:h]], [allp[h:]]
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        err, _ = run_oracle(tg, first, cfg=cfg, batch=batch)
        assert err == 0
        st = run_gpu(tg, second, cfg=None, batch=batch)   # the config comes from the existing metadata.json
        err, _ = run_oracle(to, first + second, cfg=cfg, batch=batch)
        assert err == 0
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d)
        assert mg == mo
        assert st["grid_points"] + st["kept_points"] == st["number_of_points"]


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_big_matches_oracle(seed):
    import pcconv
    files, cfg, batch, kind = big_case(seed)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        conv = pcconv.Converter(tg, batch_size=batch, config=cfg)
        try:
            for f in files:
                conv.add_points(f)
            conv.set_profiling(True)
            st = conv.build()
            kt = conv.kernel_times()
            conv.write()
        finally:
            conv.close()
        err, arrivals = run_oracle(to, files, cfg=cfg, batch=batch)
        assert err == 0
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d)
        assert mg == mo
        assert st["arrivals"] == arrivals
        assert kt["dense_launches"] > 0 and kt["dense_arrivals"] > 0


def _sharded(tmp_path, files, cfg, batch, world, rounds, merge=False, prior=None):
    """files over `world` thread ranks on cuda:0 (pcconv.dist), written to out;
    with merge the existing cloud `prior` (file list) is written first by the oracle."""
    import threading
    import numpy as np
    import torch
    from pcconv.dist import HipShardOps, ThreadComm, ThreadGroup, key_range, shard_build
    from shard_np import as_tensor
    fp = [len(f) for f in files]
    allp = np.concatenate(files)
    out = str(tmp_path / "out")
    if merge:
        assert run_oracle(out, prior, cfg=cfg, batch=batch)[0] == 0
    dev = torch.device("cuda", 0)
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            torch.cuda.set_device(dev)
            a, b = key_range(len(allp), r, world)
            ops = HipShardOps(0, out_dir=out, batch_size=batch, config=None if merge else cfg, merge=merge)
            ops.landing_rounds = rounds
            t = as_tensor(allp[a:b]).to(dev)
            res[r] = shard_build(ThreadComm(grp, r, dev), ops, t, a, fp, write=True, merge=merge)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, (cfg, batch, world, errs)
    assert sum(r.recv_points for r in res) == len(allp)
    return out, res


@pytest.mark.parametrize("seed", range(1, 48, 3))
def test_fuzz_sharded_threads_match_oracle(seed, tmp_path):
    """The sweep's cases sharded over 2-8 thread ranks on cuda:0 (pcconv.dist:
    level-0 cells or slabs owned per rank, the exchange in 0 or 2-5 rounds with
    level-0 pass 1 behind it), merged output against the oracle's one-process run."""
    from test_dist_cpu import check_against_oracle
    files, cfg, batch, kind = mid_case(seed)
    out, res = _sharded(tmp_path, files, cfg, batch, [2, 3, 4, 5, 8][seed % 5], [0, 2, 3, 5][seed % 4])
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg, batch=batch)


@pytest.mark.parametrize("seed", range(2, 48, 4))
def test_fuzz_sharded_merge_matches_oracle(seed, tmp_path):
    """Sharded merge (config 5's shape): the first half written by the oracle,
    the second half merged by 2-5 thread ranks (pcc_open_subtrees per rank)."""
    from test_dist_cpu import check_against_oracle
    files, cfg, batch, kind = mid_case(seed)
    first, second = halves(files)
    out, res = _sharded(tmp_path, second, cfg, batch, [2, 3, 4, 5][seed % 4], 0, merge=True, prior=first)
    check_against_oracle(tmp_path, first + second, out, res[0].summary, cfg=cfg, batch=batch)


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_nonfinite_matches_oracle(seed):
    """The sweep's cases with ~0.5 % of the points given NaN / +-inf coordinates."""
    import pcconv
    files, cfg, batch, kind = mid_case(seed, nonfinite=True)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        err, arrivals = run_oracle(to, files, cfg=cfg, batch=batch)
        assert err == 0
        st = run_gpu(tg, files, cfg=cfg, batch=batch)
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d)
        assert mg == mo
        assert st["grid_points"] + st["kept_points"] == st["number_of_points"]


@pytest.mark.parametrize("seed", range(0, 24, 3))
def test_fuzz_nonfinite_merge_matches_oracle(seed):
    """NaN in the existing cloud (its box stays finite: NaN is skipped) and NaN /
    +-inf in the merged points.  An infinite coordinate in the existing cloud
    would make its metadata.json box null, which neither the reference's
    serde_json nor this loader reads back (test_parity_gpu.py)."""
    import numpy as np
    files, cfg, batch, kind = mid_case(seed, nonfinite=True)
    first, second = halves(files)
    f = first[0]
    first = [f[~(np.isinf(f["x"]) | np.isinf(f["y"]) | np.isinf(f["z"]))]]   # (the existing cloud: NaN only)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        assert run_oracle(tg, first, cfg=cfg, batch=batch)[0] == 0
        st = run_gpu(tg, second, cfg=None, batch=batch)
        assert run_oracle(to, first + second, cfg=cfg, batch=batch)[0] == 0
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d)
        assert mg == mo


@pytest.mark.parametrize("seed", range(1, 24, 3))
def test_fuzz_nonfinite_sharded_matches_oracle(seed, tmp_path):
    from test_dist_cpu import check_against_oracle
    files, cfg, batch, kind = mid_case(seed, nonfinite=True)
    out, res = _sharded(tmp_path, files, cfg, batch, [2, 3, 4][seed % 3], [0, 3][seed % 2])
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg, batch=batch)


def test_saturated_hexagon_indices_replayed_sequentially():
    """NaN-collapsed points on a line far from the origin (the sweep's case 8 with
    non-finite coordinates) recurse to level 24, where x / hex radius no longer
    fits an i32: the reference saturates (hex.rs:67-85), the parallel slot
    geometry cannot, so the build is replayed sequentially on the GPU (stats
    sequential_replay) == the oracle; with the replay disabled it is an error."""
    import pcconv
    files, cfg, batch, kind = mid_case(8, nonfinite=True)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        assert run_oracle(to, files, cfg=cfg, batch=batch)[0] == 0
        st = run_gpu(tg, files, cfg=cfg, batch=batch)
        assert st["sequential_replay"] == 1
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], d
        assert mg == mo
        assert mg["hierarchies"] >= 20


def test_saturated_hexagon_indices_error_without_replay(monkeypatch):
    import pcconv
    monkeypatch.setenv("PCC_NO_REPLAY", "1")
    files, cfg, batch, kind = mid_case(8, nonfinite=True)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg:
        with pytest.raises(pcconv.PccError) as ei:
            run_gpu(tg, files, cfg=cfg, batch=batch)
        assert "device error flags" in str(ei.value)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_big_sharded_matches_oracle(seed, tmp_path):
    """1-6 M points over 3-8 thread ranks: dense slabs on every rank, heavy cells
    shared when the clouds are clustered."""
    from test_dist_cpu import check_against_oracle
    files, cfg, batch, kind = big_case(seed)
    out, res = _sharded(tmp_path, files, cfg, batch, [3, 4, 8][seed % 3], [0, 4][seed % 2])
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg, batch=batch)


@pytest.mark.parametrize("seed", range(6, 10))
def test_fuzz_big_merge_matches_oracle(seed):
    files, cfg, batch, kind = big_case(seed)
    first, second = halves(files)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        assert run_oracle(tg, first, cfg=cfg, batch=batch)[0] == 0
        st = run_gpu(tg, second, cfg=None, batch=batch)
        assert run_oracle(to, first + second, cfg=cfg, batch=batch)[0] == 0
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d, _explain(first + second, to, tg))
        assert mg == mo


@pytest.mark.parametrize("seed", range(8))
def test_fuzz_wide_subgrid_matches_oracle(seed):
    """Sub-grids of 97-200 (metadata.rs:67-78 reads any u32): the sequential
    replay on the GPU, on the sweep's cases cut to 40 000 points."""
    import numpy as np
    files, cfg, batch, kind = mid_case(seed)
    cfg = dict(cfg, sub_grid_dimension=int(np.random.default_rng(seed).integers(97, 201)))
    left, cut = 40_000, []
    for f in files:
        cut.append(f[:max(0, min(len(f), left))])
        left -= len(cut[-1])
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        assert run_oracle(to, cut, cfg=cfg, batch=batch)[0] == 0
        st = run_gpu(tg, cut, cfg=cfg, batch=batch)
        assert st["sequential_replay"] == 1
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d, _explain(cut, to, tg))
        assert mg == mo


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_far_from_origin_matches_oracle(seed):
    """The sweep's cases moved 10^3-10^7 cells from the origin, where the f32
    spacing of the coordinates reaches the sub-cell size: points collapse onto
    few slots and recurse deep (metadata.rs:100-102, hex.rs:67-85).  Where the
    oracle converts, the GPU build equals it; where the reference cannot (the
    depth limit, metadata.rs:92), the GPU build refuses too."""
    import pcconv
    far = [1e3, 1e4, 1e5, 3e5, 1e6, 1e7][seed % 6]
    files, cfg, batch, kind = mid_case(seed, far=far)
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        err, arrivals = run_oracle(to, files, cfg=cfg, batch=batch)
        if err:
            with pytest.raises(pcconv.PccError):
                run_gpu(tg, files, cfg=cfg, batch=batch)
            return
        st = run_gpu(tg, files, cfg=cfg, batch=batch)
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, far, d, _explain(files, to, tg))
        assert mg == mo
        if far <= 1e4:
            assert st["sequential_replay"] == 0


@pytest.mark.parametrize("seed", range(1, 48, 4))
def test_fuzz_merge_displacing_seeds(seed):
    """Merges whose new points sit exactly at the level-0 slot centres of
    existing points (d^2 = 0: each displaces its slot's grid seed, cell.rs:77-80)
    plus 2 % random ones, over the sweep's configs."""
    import numpy as np
    import pyref
    files, cfg, batch, kind = mid_case(seed)
    first, _ = halves(files)
    old = first[0]
    rng = np.random.default_rng(seed)
    cr = pyref.sub_cell_size(cfg, pyref.cell_size(cfg, 0)) / np.float32(2.0)
    pick = old[rng.choice(len(old), min(len(old), 500), replace=False)]
    new = pick.copy()
    for i, p in enumerate(pick):
        c = pyref.hex_to_world(pyref.hex_from_world((p["x"], p["y"], p["z"]), cr), cr)
        new[i]["x"], new[i]["y"], new[i]["z"] = c
    extra = old[rng.choice(len(old), max(1, len(old) // 50), replace=False)].copy()
    extra["x"] += np.float32(cfg["max_cell_size"] / 1000.0)
    second = [np.concatenate([new, extra])]
    with tempfile.TemporaryDirectory(dir=_shm()) as tg, tempfile.TemporaryDirectory(dir=_shm()) as to:
        assert run_oracle(tg, first, cfg=cfg, batch=batch)[0] == 0
        st = run_gpu(tg, second, cfg=None, batch=batch)
        assert run_oracle(to, first + second, cfg=cfg, batch=batch)[0] == 0
        d, mg, mo = compare_dirs(tg, to, fast=True)
        assert d == [], (kind, cfg, batch, d, _explain(first + second, to, tg))
        assert mg == mo
