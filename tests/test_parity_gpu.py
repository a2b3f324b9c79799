"""GPU parity: the HIP build (through the C ABI, libpcconv.so) against the C
oracle on identical inputs, compared on the canonical form of the output
directory (tests/canon.py: headers bit-exact, grid membership, overflow lists
in stored order, metadata values).  Oracle parity is unpinned against the Rust
reference itself; see tests/test_oracle_xcheck.py."""
import os
import tempfile

import numpy as np
import pytest

from gpu_util import compare_dirs, run_gpu, run_oracle  # noqa: E402
from oracle_ctypes import POINT_DTYPE, synth  # noqa: E402
from test_oracle_xcheck import _case, _to_np  # noqa: E402

pytestmark = pytest.mark.gpu


def _shm():
    """tmpfs for outputs of hundreds of thousands of cell files (creating and
    deleting them on the box's overlay file system can take minutes)."""
    return "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None


def _check(files, cfg=None, batch=10_000, fast=False, synth_files=None, base=None):
    with tempfile.TemporaryDirectory(dir=base) as tg, tempfile.TemporaryDirectory(dir=base) as to:
        st = run_gpu(tg, files if not synth_files else [], cfg=cfg, batch=batch, synth=synth_files)
        err, arrivals = run_oracle(to, files, cfg=cfg, batch=batch)
        assert err == 0
        d, mg, mo = compare_dirs(tg, to, fast=fast)
        assert d == [], d
        assert mg == mo
        assert st["arrivals"] == arrivals
        assert st["grid_points"] + st["kept_points"] == st["number_of_points"]
        # the parallel levels ran, not the sequential replay (which sub-grids
        # beyond the dense slot table take, from 97 or a little above)
        if os.environ.get("PCC_TEST_WIDE"):
            assert st["sequential_replay"] == 1
        elif (cfg or {}).get("sub_grid_dimension", 96) <= 96:
            assert st["sequential_replay"] == 0
        return st


@pytest.mark.parametrize("seed", range(60))
def test_adversarial_small(seed):
    """Tiny sub-grids, limits 1-7, batches 1-40, ties and duplicates, 1-3 files."""
    files, cfg, batch = _case(seed)
    _check([_to_np(f) for f in files], cfg=cfg, batch=batch)


@pytest.mark.parametrize("env", [{}, {"PCC_NO_FOLD": "1"}], ids=["fold", "threepass"])
def test_single_level0_cell(env, monkeypatch):
    """Every point in one level-0 cell (a rank's octant after the sharded
    exchange): a 1 x 1 x 1 level-0 grid through both level-0 binnings."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pts = synth(41, 0, 2_000_000, lo=0.0, ext=1000.0)
    st = _check([pts], fast=True)
    assert st["levels"] >= 2


@pytest.mark.parametrize("env", [{"PCC_PRE_PIECE": "40000"}, {"PCC_PRE_PIECE": "40000", "PCC_NO_PRE6": "1"},
                                 {"PCC_PRE_PIECE": "3072"}], ids=["pass1", "pass0", "tile_pieces"])
def test_upload_in_pieces_with_level0_pass_behind(env, monkeypatch):
    """Host input copied in pieces with level-0 work behind each copy
    (Engine::pre0_count): the folded pass 1 over the groups each piece completes
    (pre6_run; the build finishes the rest), or pass 0 (PCC_NO_PRE6); two files,
    pieces that end mid-tile and mid-group."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pts = synth(43, 0, 330_001)
    _check([pts[:200_003], pts[200_003:]], fast=True)


def test_config1_uniform_100k():
    pts = synth(1, 0, 100_000)
    st = _check([pts])
    assert st["hierarchies"] == 1 and st["cells"] == 8


def test_ragged_files_and_empty_file():
    pts = synth(11, 0, 123_457)
    files = [pts[:1], pts[1:1], pts[1:50_001], pts[50_001:]]
    _check(files)


def test_batch_size_one_and_tiny_limit():
    pts = synth(12, 0, 3000, lo=-10.0, ext=20.0)
    _check([pts], cfg=dict(cell_point_overflow_limit=3, sub_grid_dimension=4, max_cell_size=8.0), batch=1)


@pytest.mark.parametrize("n", [66_000, 140_000])
def test_max_overflow_limit_kept_lists(n):
    """Kept lists at the GPU's LDS sort capacity: cell_point_overflow_limit = 8192 (the
    largest the GPU build accepts) with a 4-slot-wide sub-grid, so most points
    overflow and buckets of up to 8192 points are kept and sorted by key in k_bucket
    (cell.rs:108-153), or spilled around the threshold, over several files.  At 66 000
    points the oracle keeps lists of up to 8 178 points (three above 4 096) and spills
    five; at 140 000 every level-0 bucket spills."""
    pts = synth(21, 0, n, lo=0.0, ext=7.999)
    k = n // 3
    _check([pts[:k], pts[k:2 * k], pts[2 * k:]],
           cfg=dict(cell_point_overflow_limit=8192, sub_grid_dimension=4, max_cell_size=8.0))


@pytest.mark.parametrize("limit,n", [(20_000, 150_000), (12_000, 95_000)])
def test_overflow_limit_above_lds_sort(limit, n):
    """cell_point_overflow_limit above the k_bucket LDS sort capacity (8 192):
    kept lists of 8 192 < n <= limit points are sorted by key in a global-memory
    scratch (cell.rs:108-153), the others in LDS; some buckets spill around the
    threshold."""
    pts = synth(22, 0, n, lo=0.0, ext=7.999)
    k = n // 2
    st = _check([pts[:k], pts[k:]], cfg=dict(cell_point_overflow_limit=limit, sub_grid_dimension=4, max_cell_size=8.0))
    assert st["kept_points"] > 8192


@pytest.mark.parametrize("limit,n", [(8192, 66_000), (20_000, 150_000), (3000, 40_000)])
def test_bucket_resolution_in_two_launches(limit, n, monkeypatch):
    """The two-launch bucket resolution that levels of >= 8 192 buckets take
    (k_bucket: kept lists of <= 1 024 points sorted in an 8 KB LDS array, longer
    ones deferred to resident 64 KB workgroups, above 8 192 through the global
    scratch), forced at every level here (PCC_BKT_SPLIT_MIN=1) on inputs whose
    kept lists span all three sizes; cell.rs:108-153."""
    monkeypatch.setenv("PCC_BKT_SPLIT_MIN", "1")
    pts = synth(23, 0, n, lo=0.0, ext=7.999)
    k = n // 2
    st = _check([pts[:k], pts[k:]], cfg=dict(cell_point_overflow_limit=limit, sub_grid_dimension=4, max_cell_size=8.0))
    assert st["kept_points"] > 1024


def test_gui_batch_size_50k():
    """The GUI path's default batch size (src/plugins/converter.rs:198-201,604: 50 000 per
    batch) over ragged files: batch boundaries move the event batches."""
    pts = synth(14, 1, 1_300_000)
    files = [pts[:420_001], pts[420_001:420_001], pts[420_001:]]
    _check(files, batch=50_000, fast=True)


def test_clustered_1m():
    pts = synth(3, 1, 1_000_000)
    st = _check([pts], fast=True)
    assert st["levels"] >= 3


def _thin_layer_points(n, seed):
    """x, y uniform over a 2 x 2 cell footprint, z inside one level-0 hex layer
    (trunc(z / r0) constant, r0 = 1000/96/2): every point has the same low 6
    layer bits, so one pass-1 bucket holds the whole input."""
    p = synth(seed, 0, n, lo=-1000.0, ext=2000.0)
    p["z"] = (np.float32(100.5) + (p["z"] - np.float32(-1000.0)) * np.float32(3.0 / 2000.0)).astype(np.float32)
    return p


@pytest.mark.parametrize("env", [{}, {"PCC_L0_GROUPS": "1"}, {"PCC_L0_TWO_UPSWEEPS": "1"}],
                         ids=["units", "one-group", "two-upsweeps"])
def test_level0_paths_thin_layer(env):
    """Level-0 binning paths on input whose points all share one low-6-bit layer
    digit: the one-upsweep path (pass-2 units cut from one bucket); one tile group
    (one segment holds the whole input: a single pass-2 unit); and the upsweep
    passes forced (PCC_L0_TWO_UPSWEEPS)."""
    pts = _thin_layer_points(1_000_003, 41)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        _check([pts[:400_000], pts[400_000:]], fast=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_skewed_level_largest_first_order():
    """A level whose dense slabs are skewed: 2M uniform points (≈ 1 300 arrivals in
    each of the ≈ 1 536 level-0 slabs) and 1M points in one hex layer over four
    cells (four slabs of ≈ 250 000).  max_slab x dense slabs ≈ 3.8e8 > 1.5 x 3e6
    arrivals, so the level's dense slabs are launched largest first (k_lpt_order);
    the launch order must not change any cell."""
    uni = synth(43, 0, 2_000_000, lo=-1000.0, ext=2000.0)
    thin = _thin_layer_points(1_000_000, 44)
    _check([uni[:1_000_000], thin, uni[1_000_000:]], fast=True)


def test_config2_uniform_10m_synthetic_on_device():
    """Config 2: 10M uniform points generated in HBM; the oracle generates the same
    points on the host with its own copy of the generator."""
    n = 10_000_000
    pts = synth(2, 0, n)
    st = _check([pts], fast=True, synth_files=[(2, 0, n)])
    assert st["levels"] == 2 and st["cells"] == 72


def test_device_cache_reuse_and_release():
    """A closed converter's large buffers are reused by the next one (same stats),
    and pcc_release_device_cache frees them (a second call finds nothing)."""
    import pcconv
    stats = []
    with tempfile.TemporaryDirectory() as d:
        for _ in range(2):
            c = pcconv.Converter(d, batch_size=10_000)
            c.add_synthetic(7, 0, 5_000_000)
            stats.append(c.build())
            c.close()
    for s in stats:
        s.pop("build_ms", None)
    assert stats[0] == stats[1]
    assert pcconv.release_device_cache() >= 64 << 20   # at least the 80 MB input
    assert pcconv.release_device_cache() == 0


def test_duplicates_exact_limit_chains():
    """Thousands of exact duplicates (ties everywhere, multi-level spill chains)."""
    base = synth(13, 0, 20_000)
    dup = np.repeat(base[:3], 3000)
    files = [np.concatenate([base, dup]), np.repeat(base[:1], 1000)]
    _check(files, batch=10_000, fast=True)


def _outliers(n, lo, hi, seed):
    rng = np.random.default_rng(seed)
    o = np.zeros(n, dtype=POINT_DTYPE)
    for a in "xyz":
        o[a] = rng.uniform(lo, hi, n).astype(np.float32)
    o["rgba"] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    return o


def test_sparse_bbox_far_outliers():
    """Bounding box spanning > 2^20 level-0 cells (far outliers): the GPU build
    switches to the hashed level-0 cell set (sparse mode)."""
    pts = synth(51, 1, 300_000)
    out = _outliers(64, -4.0e7, 4.0e7, 51)
    allp = np.concatenate([pts[:150_000], out, pts[150_000:]])
    _check([allp], fast=True)


def test_sparse_bbox_small_cells_many_occupied():
    """Tiny max_cell_size: ~4 * 10^5 occupied level-0 cells over a 2^30-cell box."""
    pts = synth(52, 0, 400_000, lo=-500.0, ext=1000.0)
    _check([pts], cfg=dict(cell_point_overflow_limit=4, sub_grid_dimension=2, max_cell_size=1.0), fast=True,
           base=_shm())


def test_bbox_beyond_hashed_range_is_an_error():
    """More than 2^21 level-0 cells along an axis: explicit error, no wrong output."""
    import pcconv
    p = _outliers(1000, -5.0e9, 5.0e9, 53)
    with tempfile.TemporaryDirectory() as tg:
        c = pcconv.Converter(tg)
        c.add_points(p)
        with pytest.raises(pcconv.PccError) as ei:
            c.build()
        assert ei.value.code == -27
        c.close()


def test_depth_limit_is_an_error():
    """More than L identical points never terminate in the reference (metadata.rs:92
    overflows 2u32.pow(h) at h = 32); the GPU build reports it instead of hanging."""
    import pcconv
    p = np.zeros(6000, dtype=POINT_DTYPE)
    p["x"], p["y"], p["z"] = 1.0, 2.0, 3.0
    with tempfile.TemporaryDirectory() as tg:
        c = pcconv.Converter(tg)
        c.add_points(p)
        with pytest.raises(pcconv.PccError) as ei:
            c.build()
        assert "depth" in str(ei.value)
        c.close()


def test_merge_into_cloud_with_infinite_bbox_is_an_error():
    """A cloud with infinite coordinates writes its bounding box as null
    (serde_json), which the reference cannot read back (lib.rs:86-101 unwraps
    serde_json's error); a merge into it fails with an explicit error.  NaN and
    +-inf points merge into a finite cloud: tests/test_nonfinite_gpu.py."""
    import pcconv
    with tempfile.TemporaryDirectory() as tg:
        c = pcconv.Converter(tg)
        p = synth(1, 0, 1000)
        p["x"][5] = np.inf
        c.add_points(p)
        c.build()
        c.write()
        c.close()
        with pytest.raises(pcconv.PccError) as ei:
            c = pcconv.Converter(tg)
        assert "not finite" in str(ei.value)


def test_ply_cli_roundtrip():
    """Config 1 through the CLI binary with a binary-LE PLY, plus an ASCII PLY whose
    points the reference drops (ply.rs:43-51) but whose batches still count."""
    import subprocess
    import pcconv
    pts = synth(1, 0, 100_000)
    with tempfile.TemporaryDirectory() as td:
        a = os.path.join(td, "a.ply")
        b = os.path.join(td, "b.ply")
        pcconv.write_ply(a, pts[:60_000])
        pcconv.write_ply(b, pts[:25_000], ascii=True)
        c = os.path.join(td, "c.ply")
        pcconv.write_ply(c, pts[60_000:])
        out = os.path.join(td, "out")
        exe = os.path.join(os.path.dirname(pcconv.LIB_PATH), "point_converter")
        r = subprocess.run([exe, "-o", out, "-f", a, "-f", b, "-f", c], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert "Finished converting after" in r.stderr
        ref = os.path.join(td, "ref")
        from oracle_ctypes import Oracle
        o = Oracle()
        o.add_file(pts[:60_000])
        for _ in range(3):   # 25 000 ASCII points -> 3 empty batches
            o.add_batch(pts[:0])
        o.add_file(pts[60_000:])
        o.write(ref)
        o.close()
        d, mg, mo = compare_dirs(out, ref)
        assert d == [] and mg == mo


def test_wide_slab_over_2_23_arrivals():
    """One level-0 slab of 9M arrivals (> 2^23): the wide slot-table entry layout
    (28-bit arrival index, displaced occupants routed from their payload)."""
    rng = np.random.default_rng(31)
    n = 9_000_000
    pts = np.zeros(n, dtype=POINT_DTYPE)
    pts["x"] = rng.uniform(0.0, 1000.0, n).astype(np.float32)
    pts["y"] = rng.uniform(0.0, 1000.0, n).astype(np.float32)
    pts["z"] = rng.uniform(0.0, 5.0, n).astype(np.float32)   # hex layer 0 of level 0 (r = 5.2083)
    pts["rgba"] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    st = _check([pts], fast=True)
    assert st["levels"] >= 2


def _fold_kind(files, cs=1000.0):
    """The level-0 binning a cloud takes: 3 (at most two level-0 cells per axis),
    6 (at most four), 0 (more: the three/four-pass path)."""
    allp = np.concatenate(files)
    ext = 0
    for a in "xyz":
        v = allp[a].astype(np.float32)
        ext = max(ext, int(np.floor(v.max() / np.float32(cs))) - int(np.floor(v.min() / np.float32(cs))))
    return 3 if ext < 2 else 6 if ext < 4 else 0


def _reshape(p, sx, ox, sy, oy, sz, oz):
    q = p.copy()
    for a, s, o in (("x", sx, ox), ("y", sy, oy), ("z", sz, oz)):
        q[a] = (q[a] * np.float32(s) + np.float32(o)).astype(np.float32)
    return q


@pytest.mark.parametrize("case,env", [("4x4x4", {}), ("4x4x4", {"PCC_NO_FOLD4": "1"}), ("3x4x2", {}), ("2x3x1", {}),
                                      ("gauss", {}), ("5x4x4", {})])
def test_level0_fold_modulo4(case, env, monkeypatch):
    """The two-pass level-0 fold over grids of up to four cells per axis (cells
    named by their absolute indices modulo 4, config 3's 64 cells), against the
    oracle; PCC_NO_FOLD4 and a grid of five cells take the four-pass path."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if case == "gauss":   # the config-3 generator (Gaussian mixture)
        files = [synth(91, 2, 900_000), synth(92, 2, 300_001)]
    else:
        p = synth(93, 0, 1_200_000, lo=-2000.0, ext=4000.0)   # cells -2 .. 1 on every axis
        p = {"4x4x4": p, "3x4x2": _reshape(p, 0.75, 500.0, 1.0, 0.0, 0.5, 0.0),
             "2x3x1": _reshape(p, 0.5, 0.0, 0.75, 500.0, 0.25, 500.0),
             "5x4x4": _reshape(p, 1.25, 0.0, 1.0, 0.0, 1.0, 0.0)}[case]
        files = [p[:500_000], p[500_000:]]
    want = _fold_kind(files)
    if case.startswith("4") or case.startswith("3"):
        assert want == 6
    st = _check(files, cfg=dict(sub_grid_dimension=64, cell_point_overflow_limit=1000), fast=True)
    assert st["level0_fold"] == (0 if env else want), st


def test_arena_overflow_is_reported(monkeypatch, tmp_path):
    """Child-slab capacities beyond the next level's arena (forced with a test
    cap): the clamped kernels run, and the build fails with the arena message."""
    import pcconv
    monkeypatch.setenv("PCC_TEST_ARENA_CAP", "1000")
    c = pcconv.Converter(str(tmp_path / "g"), config=dict(sub_grid_dimension=16, cell_point_overflow_limit=50))
    try:
        c.add_points(synth(95, 0, 200_000))
        with pytest.raises(pcconv.PccError, match="exceed the next level's arena"):
            c.build()
    finally:
        c.close()


@pytest.mark.parametrize("dim,n,limit", [(97, 80_000, 200), (128, 120_000, 500), (200, 60_000, 50), (128, 30_001, 1)])
def test_wide_subgrid_matches_oracle(dim, n, limit):
    """sub_grid_dimension beyond the dense slot table (> 96, which the
    reference allows: metadata.rs:17-18) through the sequential replay
    (build_wide), against the oracle; several files and a ragged batch."""
    p = synth(96 + dim, 1, n)
    st = _check([p[: n // 3], p[n // 3:]], cfg=dict(sub_grid_dimension=dim, cell_point_overflow_limit=limit), batch=7_777)
    assert st["levels"] >= 1


def test_wide_path_forced_equals_slab_path(monkeypatch):
    """The sequential replay forced at a dimension the slab kernels handle
    (PCC_TEST_WIDE) writes the same cloud as the oracle, NaN and infinite
    coordinates included."""
    from nonfinite_input import nonfinite_files
    monkeypatch.setenv("PCC_TEST_WIDE", "1")
    _check(nonfinite_files(seed=13, n=20_000, kinds="mixed"), cfg=dict(sub_grid_dimension=16, cell_point_overflow_limit=40))
    _check([synth(97, 0, 150_000)], cfg=dict(sub_grid_dimension=32, cell_point_overflow_limit=300))


@pytest.mark.parametrize("limit", [1024, 1500, 4000, 8192])
def test_long_kept_lists_radix_sorted(limit):
    """Kept overflow lists of a thousand points and more (the bucket kernel's
    radix sort, from kBktRadixMin = 1024 up to the 8 192-word LDS capacity),
    against the oracle: a small sub-grid sends most points to the overflow,
    several files and ragged batches interleave their keys."""
    p = synth(98, 1, 400_000)
    _check([p[:150_000], p[150_000:151_111], p[151_111:]], cfg=dict(sub_grid_dimension=8, cell_point_overflow_limit=limit),
           batch=6_000, fast=True)


def test_upload_growing_past_the_first_reservation():
    """Files added one by one, each growing the reserved input: level-0 pass 1
    behind the upload was decided on the first file's reservation, and the
    second file's tiles reached past the arenas sized for it (found by the
    bulk sweep, seed 1658: a line of points whose key order the stray stores
    permuted).  Pass 1 now stops behind the upload when the input outgrows the
    arenas; == the oracle, and == the build with that pass disabled."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fuzz_cases import mid_case
    files, cfg, batch, _ = mid_case(1658)
    assert [len(f) for f in files] == [4084, 4030, 14950]
    _check(files, cfg=cfg, batch=batch, fast=True)
    p = synth(77, 0, 50_000)
    _check([p[:5000], p[5000:11000], p[11000:]], fast=True)
