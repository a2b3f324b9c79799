"""Sharded build on the GPU through the C-ABI.

One MI355X per test box, so ranks are threads of one process sharing cuda:0
(pcconv.dist.ThreadComm): the exchange moves real device tensors and every
rank runs the product path (HipShardOps -> libpcconv.so).  The merged output
must equal the single-process sequential oracle.
"""
import os
import sys
import threading

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))

import pcconv  # noqa: E402
from pcconv.dist import HipShardOps, ThreadComm, ThreadGroup, key_range, shard_build  # noqa: E402
from shard_np import NumpyShardOps, as_points, as_tensor  # noqa: E402
from test_dist_cpu import check_against_oracle, make_input, make_merge_input, rank_slice  # noqa: E402
from gpu_util import run_oracle  # noqa: E402
from oracle_ctypes import synth  # noqa: E402
from gpu_util import compare_dirs, run_gpu  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_keyed_input_equals_plain_input(tmp_path):
    """All points keyed 0..N-1 with the declared file structure == pcc_add_points."""
    files = [synth(21, 0, 150_000), synth(22, 1, 61_234)]
    allp = np.concatenate(files)
    plain = str(tmp_path / "plain")
    run_gpu(plain, files)
    keyed = str(tmp_path / "keyed")
    c = pcconv.Converter(keyed)
    c.declare_files([len(f) for f in files])
    pts = as_tensor(allp).to(DEV)
    keys = torch.arange(len(allp), dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    c.add_keyed_points_device(pts.data_ptr(), keys.data_ptr(), len(allp))
    c.finish()
    d, ma, mb = compare_dirs(plain, keyed)
    assert not d, d
    assert ma == mb


@pytest.mark.parametrize("lo,ext,fold", [(-1000.0, 2000.0, 3), (-2000.0, 4000.0, 6)])
def test_keyed_input_level0_folds(tmp_path, lo, ext, fold):
    """Keyed device input (pass 1 stages the keys beside the points) through both
    level-0 folds: 2 and 4 cells per axis, against the plain input's output."""
    files = [synth(27, 0, 400_000, lo=lo, ext=ext), synth(28, 0, 333_333, lo=lo, ext=ext)]
    allp = np.concatenate(files)
    cfg = dict(sub_grid_dimension=48)
    plain = str(tmp_path / "plain")
    run_gpu(plain, files, cfg=cfg)
    keyed = str(tmp_path / "keyed")
    c = pcconv.Converter(keyed, config=cfg)
    c.declare_files([len(f) for f in files])
    pts = as_tensor(allp).to(DEV)
    keys = torch.arange(len(allp), dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    c.add_keyed_points_device(pts.data_ptr(), keys.data_ptr(), len(allp))
    st = c.build()
    c.write()
    c.close()
    assert st["level0_fold"] == fold
    d, ma, mb = compare_dirs(plain, keyed)
    assert not d, d
    assert ma == mb


def test_shard_histogram_and_route_match_numpy():
    pts_np = synth(23, 1, 200_001, lo=-2500.0, ext=5000.0)
    pts = as_tensor(pts_np).to(DEV)
    ref = NumpyShardOps("/nonexistent")
    gmin, gmax = ref.bbox(as_tensor(pts_np))
    assert pcconv.shard_bbox(pts.data_ptr(), len(pts_np)) == (gmin, gmax)
    g = pcconv.shard_grid_from_bbox(gmin, gmax)
    h = torch.empty(g.ncells, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    pcconv.shard_histogram(pts.data_ptr(), len(pts_np), g, h.data_ptr())
    href = ref.histogram(as_tensor(pts_np), g)
    assert torch.equal(h.cpu(), href)
    for world in (2, 3, 5):
        owner = torch.from_numpy((np.arange(g.ncells) * 7 % world).astype(np.int32))
        send = torch.empty_like(pts)
        keys = torch.empty(len(pts_np), dtype=torch.int32, device=DEV)
        od = owner.to(DEV)
        torch.cuda.synchronize()
        counts = pcconv.shard_route(pts.data_ptr(), len(pts_np), 1000, g, od.data_ptr(), world, send.data_ptr(),
                                    keys.data_ptr())
        s2, k2, c2 = ref.route(as_tensor(pts_np), 1000, g, owner, world)
        assert counts == c2
        assert torch.equal(send.cpu(), s2)
        assert torch.equal(keys.cpu(), k2)
    # a destination past nranks is an error, not a silent drop
    bad = torch.full((g.ncells,), 3, dtype=torch.int32, device=DEV)
    with pytest.raises(Exception):
        pcconv.shard_route(pts.data_ptr(), len(pts_np), 0, g, bad.data_ptr(), 3, send.data_ptr(), keys.data_ptr())


def test_shard_slab_histogram_and_route_match_numpy():
    """Slab mode (cell, hex z-layer) units: histogram and the stable partition
    (tile count -> scan -> scatter) against numpy, up to 64 destinations."""
    pts_np = synth(29, 2, 300_007, lo=-2500.0, ext=5000.0)
    pts = as_tensor(pts_np).to(DEV)
    ref = NumpyShardOps("/nonexistent")
    gmin, gmax = ref.bbox(as_tensor(pts_np))
    g = pcconv.shard_grid_from_bbox(gmin, gmax)
    dim = int(ref.cfg_full()["sub_grid_dimension"])
    nu = g.ncells * pcconv.SHARD_LAYERS
    h = torch.empty(nu, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    pcconv.shard_slab_histogram(pts.data_ptr(), len(pts_np), g, dim, h.data_ptr())
    assert torch.equal(h.cpu(), ref.slab_histogram(as_tensor(pts_np), g))
    for world in (4, 64):
        table = torch.from_numpy((np.arange(nu) * 11 % world).astype(np.int32))
        send = torch.empty_like(pts)
        keys = torch.empty(len(pts_np), dtype=torch.int32, device=DEV)
        td = table.to(DEV)
        torch.cuda.synchronize()
        counts = pcconv.shard_route_slabs(pts.data_ptr(), len(pts_np), 77, g, dim, td.data_ptr(), world,
                                          send.data_ptr(), keys.data_ptr())
        s2, k2, c2 = ref.route_slabs(as_tensor(pts_np), 77, g, table, world)
        assert counts == c2
        assert torch.equal(send.cpu(), s2)
        assert torch.equal(keys.cpu(), k2)


@pytest.mark.parametrize("slabs,world", [(False, 3), (False, 8), (True, 16), (True, 64)])
def test_route_bitmaps_and_key_rebuild_match_numpy(slabs, world):
    """pcc_shard_route_bitmaps == the numpy restatement (points, counts, every
    bitmap word), and pcc_shard_keys_from_bitmaps rebuilds each receiver's keys
    from the senders' rows (three senders of different sizes and key offsets)."""
    ref = NumpyShardOps("/nonexistent")
    senders = [synth(31 + q, 1 + (q % 2), m, lo=-2500.0, ext=5000.0) for q, m in enumerate((100_003, 64, 77_777))]
    allp = np.concatenate(senders)
    gmin, gmax = ref.bbox(as_tensor(allp))
    g = pcconv.shard_grid_from_bbox(gmin, gmax)
    nu = g.ncells * (pcconv.SHARD_LAYERS if slabs else 1)
    table = torch.from_numpy((np.arange(nu) * 13 % world).astype(np.int32))
    td = table.to(DEV)
    rows, key0, k = [], [], 0
    for sp in senders:
        pts = as_tensor(sp).to(DEV)
        ops = HipShardOps.__new__(HipShardOps)
        ops.dev, ops.cfg = 0, {}
        send, bm, counts = ops.route_bitmaps(pts, g, td, world, slabs)
        s2, b2, c2 = ref.route_bitmaps(as_tensor(sp), g, table, world, slabs)
        assert counts == c2
        assert torch.equal(send.cpu(), s2)
        assert torch.equal(bm.cpu(), b2)
        rows.append(bm)
        key0.append(k)
        k += len(sp) + 1000
    for r in (0, world - 1):
        cat = torch.cat([b[r] for b in rows])
        nw = [int(b.shape[1]) for b in rows]
        nk = int(sum(bin(int(v) & (2**64 - 1)).count("1") for b in rows for v in b[r].cpu().tolist()))
        keys = HipShardOps.keys_from_bitmaps(ops, cat, nw, key0, nk)
        assert torch.equal(keys.cpu(), ref.keys_from_bitmaps(cat, nw, key0, nk))
        with pytest.raises(pcconv.PccError):   # a receive count that disagrees with the bits
            HipShardOps.keys_from_bitmaps(ops, cat, nw, key0, nk + 1)


@pytest.mark.parametrize("slabs,world,n", [(False, 2, 1), (False, 8, 4096), (False, 8, 1_000_003),
                                           (True, 16, 300_007), (True, 64, 2_500_001)])
def test_route_bitmaps_one_pass_matches_two_pass(slabs, world, n):
    """pcc_shard_route_bitmaps_hist (histogram totals + decoupled look-back
    between tiles, one read of the points) == pcc_shard_route_bitmaps and the
    numpy restatement: points in order, counts, every bitmap word; a histogram
    of other points is rejected."""
    ref = NumpyShardOps("/nonexistent")
    sp = synth(41 + world, 1 + int(slabs), n, lo=-2500.0, ext=5000.0)
    pts = as_tensor(sp).to(DEV)
    gmin, gmax = ref.bbox(as_tensor(sp))
    g = pcconv.shard_grid_from_bbox(gmin, gmax)
    dim = int(ref.cfg_full()["sub_grid_dimension"])
    nu = g.ncells * (pcconv.SHARD_LAYERS if slabs else 1)
    table = torch.from_numpy((np.arange(nu) * 13 % world).astype(np.int32))
    td = table.to(DEV)
    h = torch.empty(nu, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    if slabs:
        pcconv.shard_slab_histogram(pts.data_ptr(), n, g, dim, h.data_ptr())
    else:
        pcconv.shard_histogram(pts.data_ptr(), n, g, h.data_ptr())
    ops = HipShardOps.__new__(HipShardOps)
    ops.dev, ops.cfg = 0, {}
    s1, b1, c1 = ops.route_bitmaps(pts, g, td, world, slabs, hist=h)
    s2, b2, c2 = ops.route_bitmaps(pts, g, td, world, slabs)
    assert c1 == c2 and sum(c1) == n
    assert torch.equal(s1, s2)
    assert torch.equal(b1, b2)
    if n < 400_000:
        s3, b3, c3 = ref.route_bitmaps(as_tensor(sp), g, table, world, slabs)
        assert c1 == c3
        assert torch.equal(s1.cpu(), s3)
        assert torch.equal(b1.cpu(), b3)
    hb = h.clone()
    hb[int(torch.argmax(hb))] -= 1   # one point missing from the histogram
    with pytest.raises(pcconv.PccError):
        ops.route_bitmaps(pts, g, td, world, slabs, hist=hb)


@pytest.mark.parametrize("limit,batch", [(50, 7), (64, 64), (1, 1000), (300, 13)])
def test_device_bucket_resolution_matches_numpy(limit, batch):
    """pcc_shard_resolve_buckets (HipShardOps.resolve_level1) == the numpy
    statement (dist.resolve_level1): bucket states, spill batches, the kept lists
    in key order, the spilled buckets' rows in segment order.  Buckets of 0..4
    segments (empty ones included; each several sorted runs, as a cell's slabs)
    with totals around the limit, over a file structure with an empty file and a
    short last batch."""
    from pcconv.dist import resolve_level1
    rng = np.random.default_rng(limit * 7 + batch)
    files = [3 * batch + 5, 0, 40 * batch + 1, 2 * batch]
    n_keys = sum(files)
    rows, segs = [], []
    for b in range(60):
        cell = (int(rng.integers(-5, 5)), int(rng.integers(-5, 5)), b)
        tot = int(rng.choice([0, 1, limit - 1, limit, limit + 1, 2 * limit + 3, int(rng.integers(1, 3 * limit + 2))]))
        tot = max(0, min(tot, n_keys))
        keys = np.sort(rng.choice(n_keys, size=tot, replace=False))
        if b % 5 == 0 and tot:   # all in one batch when it fits
            k0 = int(rng.integers(0, max(1, n_keys - tot)))
            keys = np.arange(k0, k0 + tot)
        nseg = int(rng.integers(1, 5))
        owner = rng.integers(0, nseg, size=tot)
        for s in range(nseg):
            k = keys[owner == s]
            # a segment is a cell's arrivals from one rank: sorted runs (slabs), not sorted as a whole
            runs = rng.integers(0, 3, size=len(k))
            segs.append((cell, np.concatenate([k[runs == q] for q in (2, 0, 1)])))
    order = rng.permutation(len(segs))   # segments of a bucket interleave with others
    meta, kk = [], []
    for i in order:
        cell, k = segs[i]
        meta.append([*cell, len(k)])
        kk.append(k)
    meta = np.array(meta, dtype=np.int64)
    keys = np.concatenate(kk).astype(np.uint32)
    pts = np.zeros((len(keys), 4), np.int32)
    pts[:, 0] = np.arange(len(keys))
    pts[:, 1] = keys.view(np.int32)
    pts[:, 3] = rng.integers(-2**31, 2**31 - 1, size=len(keys), dtype=np.int64).astype(np.int32)
    kt = torch.from_numpy(keys.view(np.int32).copy())
    ref = resolve_level1(meta, torch.from_numpy(pts), kt, files, batch, limit)
    ops = HipShardOps.__new__(HipShardOps)
    ops.dev, ops.cfg, ops.batch_size = 0, {"cell_point_overflow_limit": limit}, batch
    got = ops.resolve_level1(meta, torch.from_numpy(pts).to(DEV), kt.to(DEV), files)
    assert np.array_equal(got["bucket_rows"], ref["bucket_rows"])
    assert set(got["bucket_rows"][:, 3]) == {1, 2}, "both states must occur"
    assert np.array_equal(got["roots_xyz"], ref["roots_xyz"])
    assert np.array_equal(got["roots_sb"], ref["roots_sb"])
    for k in ("kept_pts", "sub_pts", "sub_keys"):
        assert torch.equal(got[k].cpu(), ref[k]), k


def test_export_grid_equals_visited_cells():
    """pcc_export_grid (a raw level-0 lead build's partial cells on the device)
    == the cells pcc_visit_cells walks: same cells, order, grid points."""
    from pcconv.dist import key_range
    n = 300_000
    pts = as_tensor(synth(71, 2, n)).to(DEV)
    a, b = key_range(n, 1, 3)
    keys = torch.arange(a, b, dtype=torch.int32, device=DEV)
    ops = HipShardOps(0, batch_size=5000, config=SKEW_CFG)
    try:
        ops.begin_step()
        _, _, (pxyz, pn, G) = ops.lead_build_raw([n], pts[a:b], keys)
        seen = []

        def grab(vp):
            v = pcconv.CellView.from_address(vp)
            seen.append(((v.x, v.y, v.z), v.grid_points().view(np.int32).reshape(-1, 4)))
            return 0
        ops.conv_lead.visit_cells(grab)
        assert len(seen) == len(pxyz) > 0
        assert [s[0] for s in seen] == [tuple(int(q) for q in r) for r in pxyz]
        assert [len(s[1]) for s in seen] == [int(q) for q in pn]
        assert np.array_equal(np.concatenate([s[1] for s in seen]), G.cpu().numpy())
    finally:
        ops.close()


def test_synth_device_matches_oracle_stream():
    p = torch.empty((77_777, 4), dtype=torch.int32, device=DEV)
    pcconv.synth_device(p.data_ptr(), 123_456, 77_777, 9, 1)
    assert (as_points(p.cpu()).view(np.uint8) == synth(9, 1, 77_777, first=123_456).view(np.uint8)).all()


def _run_threads(files, world, out, cfg=None, batch=10_000, merge=False):
    fp = [len(f) for f in files]
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            torch.cuda.set_device(DEV)
            pts, key0 = rank_slice(files, r, world)
            ops = HipShardOps(0, out_dir=out, batch_size=batch, config=cfg, merge=merge)
            t = as_tensor(pts).to(DEV)
            res[r] = shard_build(ThreadComm(grp, r, DEV), ops, t, key0, fp, write=True, merge=merge)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    return res


@pytest.mark.parametrize("case,world", [("uniform", 1), ("files", 1), ("uniform", 2), ("files", 3), ("clustered", 4),
                                        ("uniform", 8)])
def test_sharded_threads_match_oracle(tmp_path, case, world):
    files = make_input(case)
    out = str(tmp_path / "out")
    res = _run_threads(files, world, out)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, res[0].summary)


def test_sharded_threads_2m_multilevel(tmp_path):
    """2M uniform points, 32-slot sub-grid: several levels per shard, 4 octants per rank."""
    cfg = dict(sub_grid_dimension=32)
    files = [synth(31, 0, 2_000_000)]
    out = str(tmp_path / "out")
    res = _run_threads(files, 2, out, cfg=cfg)
    assert [r.owned_cells for r in res] == [4, 4]
    assert res[0].summary["hierarchies"] >= 2
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg)


def test_sharded_small_limit_deep(tmp_path):
    """Tiny overflow limit + clustered data: deep hierarchies per shard."""
    cfg = dict(cell_point_overflow_limit=64, sub_grid_dimension=8)
    files = [synth(32, 1, 60_000)]
    out = str(tmp_path / "out")
    res = _run_threads(files, 3, out, cfg=cfg, batch=777)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg, batch=777)


@pytest.mark.parametrize("case,world", [("uniform", 2), ("partial", 3), ("clustered", 4)])
def test_sharded_merge_threads_match_oracle(tmp_path, case, world):
    """Config 5 sharded: every rank opens the existing cloud for
    its own subtrees (pcc_open_subtrees), merges its routed points on the GPU and
    rewrites them == the oracle converting old and new files in one run."""
    old, new = make_merge_input(case)
    out = str(tmp_path / "out")
    assert run_oracle(out, old)[0] == 0
    res = _run_threads(new, world, out, merge=True)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in new)
    check_against_oracle(tmp_path, old + new, out, res[0].summary)


def test_sharded_merge_into_gpu_built_cloud_multilevel(tmp_path):
    """A GPU-built 1.5M cloud (several levels, spilled buckets) + 500k new points
    merged by 2 ranks."""
    cfg = dict(sub_grid_dimension=32, cell_point_overflow_limit=500)
    old, new = [synth(33, 1, 1_500_000)], [synth(34, 1, 500_000)]
    out = str(tmp_path / "out")
    run_gpu(out, old, cfg=cfg)
    res = _run_threads(new, 2, out, cfg=cfg, merge=True)
    assert res[0].summary["hierarchies"] >= 3
    check_against_oracle(tmp_path, old + new, out, res[0].summary, cfg=cfg)


def test_sharded_merge_takes_config_from_existing_cloud(tmp_path):
    """The existing cloud was built with a non-default config; the sharded merge
    is opened WITHOUT a config and must use the one in its metadata.json
    (lib.rs:86-101) for the shard grid and the engine alike."""
    cfg = dict(sub_grid_dimension=24, cell_point_overflow_limit=300, max_cell_size=400.0)
    old, new = [synth(35, 1, 400_000)], [synth(36, 0, 150_000)]
    out = str(tmp_path / "out")
    run_gpu(out, old, cfg=cfg)
    res = _run_threads(new, 3, out, cfg=None, merge=True)
    check_against_oracle(tmp_path, old + new, out, res[0].summary, cfg=cfg)


SKEW_CFG = {"sub_grid_dimension": 16, "cell_point_overflow_limit": 100, "max_cell_size": 1000.0}


@pytest.mark.parametrize("world", [4, 8])
def test_sharded_threads_split_cells_match_oracle(tmp_path, world):
    """Gaussian-mixture cloud: heavy level-0 cells are built by a leader (level 0,
    pcc_set_level_range(0, 1)) and the owners of their level-1 sub-trees
    (pcc_export_pending -> exchange -> pcc_set_level_range(1, 0)) == the oracle."""
    files = [synth(61, 2, 400_000), synth(62, 2, 50_001)]
    out = str(tmp_path / "out")
    res = _run_threads(files, world, out, cfg=SKEW_CFG)
    assert res[0].plan["split_cells"] > 0
    assert sum(r.local["phases"]["sub"] for r in res) > 0
    assert sum(r.recv_points for r in res) == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=SKEW_CFG)


def test_sharded_split_cells_kept_lists_above_lds(tmp_path):
    """Shared level-0 cells whose octant buckets stay Some with more than 8 192
    points (a limit of 13 056, above the LDS sort capacity; the randomised
    sweep's case 7, a plane of 88 099 points over 4 ranks): the device bucket
    resolution sorts those kept lists in global memory, == the oracle."""
    from fuzz_cases import mid_case
    files, cfg, batch, _ = mid_case(7)
    assert cfg["cell_point_overflow_limit"] > 8192
    out = str(tmp_path / "out")
    res = _run_threads(files, 4, out, cfg=cfg, batch=batch)
    assert res[0].plan["split_cells"] > 0
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg, batch=batch)


def test_sharded_threads_sparse_wide_cloud_coarse_grid(tmp_path):
    """Level-0 grid beyond the shard grid's 2^22 cells: ownership by blocks of
    level-0 cells (pcconv.dist.shard_grid), hashed level-0 grid per rank."""
    cfg = {"sub_grid_dimension": 4, "cell_point_overflow_limit": 8, "max_cell_size": 1.0}
    files = [synth(81, 0, 30_000, lo=-2000.0, ext=4000.0), synth(82, 1, 20_000, lo=-2000.0, ext=4000.0)]
    out = str(tmp_path / "out")
    res = _run_threads(files, 3, out, cfg=cfg)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg)


def _gloo_hip_worker(rank, world, port, case, out, res_dir):
    """One process per rank on the same GPU: gloo for the collectives (host
    tensors), the product's HIP ops for the local work (the N > 1 bench path
    with RCCL swapped for gloo, since RCCL refuses two ranks on one device)."""
    import json
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pcconv.dist import TorchComm
        if case == "gauss":
            files, cfg = [synth(61, 2, 300_000)], SKEW_CFG
        else:
            files, cfg = make_input(case), None
        pts, key0 = rank_slice(files, rank, world)
        ops = HipShardOps(0, out_dir=out, config=cfg)
        comm = TorchComm(torch.device("cpu"))
        comm.max_msg_bytes = 1 << 20
        r = shard_build(comm, ops, as_tensor(pts).to(DEV), key0, [len(f) for f in files], write=True)
        ops.close()
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"summary": r.summary, "recv": r.recv_points, "plan": r.plan}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("files", 2), ("gauss", 3)])
def test_gloo_processes_with_hip_ops_match_oracle(tmp_path, case, world):
    import json
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out, rd = str(tmp_path / "out"), str(tmp_path / "res")
    os.makedirs(rd)
    mp.spawn(_gloo_hip_worker, args=(world, port, case, out, rd), nprocs=world, join=True)
    r = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(world)]
    files, cfg = ([synth(61, 2, 300_000)], SKEW_CFG) if case == "gauss" else (make_input(case), None)
    assert all(x["summary"] == r[0]["summary"] for x in r)
    assert sum(x["recv"] for x in r) == sum(len(f) for f in files)
    if case == "gauss":
        assert r[0]["plan"]["split_cells"] > 0
    check_against_oracle(tmp_path, files, out, r[0]["summary"], cfg=cfg)


# NaN / +-inf coordinates through the sharded build (dist.shard_build's
# "nonfinite" path: the reference's box and the cell extent from
# pcc_shard_bbox_nonfinite, points with an infinite coordinate routed as unit 0,
# no shared cells) and through a sharded merge, against the oracle.
@pytest.mark.parametrize("world,kinds", [(2, "mixed"), (3, "nan"), (4, "mixed")])
def test_sharded_threads_nonfinite_match_oracle(tmp_path, world, kinds):
    from nonfinite_input import NONFINITE_CFG, nonfinite_files
    files = nonfinite_files(seed=41, n=100_000, kinds=kinds)
    out = str(tmp_path / "out")
    res = _run_threads(files, world, out, cfg=NONFINITE_CFG, batch=5000)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=NONFINITE_CFG, batch=5000)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_merge_nonfinite_match_oracle(tmp_path, world):
    from nonfinite_input import NONFINITE_CFG, nonfinite_files
    old = nonfinite_files(seed=42, n=80_000, kinds="nan")
    new = nonfinite_files(seed=43, n=50_000, kinds="mixed")
    out = str(tmp_path / "out")
    assert run_oracle(out, old, NONFINITE_CFG, 5000)[0] == 0
    res = _run_threads(new, world, out, batch=5000, merge=True)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in new)
    check_against_oracle(tmp_path, old + new, out, res[0].summary, cfg=NONFINITE_CFG, batch=5000)


def test_shard_ops_nonfinite_units():
    """pcc_shard_bbox* report NaN / inf input (-EDOM: None in the mirror),
    pcc_shard_bbox_nonfinite == the numpy statement, and the cell histogram /
    one-pass route send an infinite point as unit 0 (as the numpy double)."""
    from nonfinite_input import nonfinite_files
    p = np.concatenate(nonfinite_files(seed=44, n=50_000, kinds="mixed"))
    t = as_tensor(p).to(DEV)
    torch.cuda.synchronize()
    assert pcconv.shard_bbox(t.data_ptr(), len(p)) is None
    assert pcconv.shard_bbox_sample(t.data_ptr(), len(p)) is None or np.isfinite(p["x"][::97]).all()
    ref = NumpyShardOps(None)
    parts = pcconv.shard_bbox_nonfinite(t.data_ptr(), len(p))
    want = ref.bbox_nonfinite(as_tensor(p))
    assert [np.float32(v) for v in parts] == [np.float32(v) for v in want]
    from pcconv.dist import shard_grid
    g = shard_grid(parts[9:12], parts[12:15], 1000.0)
    h = torch.empty(g.ncells, dtype=torch.int32, device=DEV)
    pcconv.shard_histogram(t.data_ptr(), len(p), g, h.data_ptr())
    assert np.array_equal(h.cpu().numpy(), ref.histogram(as_tensor(p), g).numpy())
    world = 3
    owner = torch.from_numpy((np.arange(g.ncells) % world).astype(np.int32)).to(DEV)
    ops = HipShardOps.__new__(HipShardOps)
    ops.dev, ops.cfg = 0, {}
    s1, b1, c1 = ops.route_bitmaps(t, g, owner, world, False, hist=h)
    s2, b2, c2 = ref.route_bitmaps(as_tensor(p), g, owner.cpu(), world, False)
    assert c1 == c2
    assert torch.equal(s1.cpu(), s2) and torch.equal(b1.cpu(), b2)


# Rank-local keys (clouds of 2^32 points and more): the batch table of a rank
# from the exchange bitmaps with 64-bit global keys, and a build whose event
# batches lie beyond 2^32 / batch, against the oracle fed the same batches.
def test_shard_batch_starts_64bit_keys_match_numpy():
    rng = np.random.default_rng(5)
    key0 = [0, (1 << 32) + 7, (1 << 33) + 100_003, (1 << 34) + 1]   # sparse senders beyond 2^32
    nwords = [37, 0, 129, 64]
    words = [rng.integers(0, 2**63 - 1, size=n, dtype=np.int64) for n in nwords]
    bm = torch.from_numpy(np.concatenate(words)).to(DEV)
    gs = np.sort(np.concatenate([rng.integers(0, (1 << 34) + 10_000, size=2000, dtype=np.int64),
                                 np.array(key0, dtype=np.int64), np.array(key0, dtype=np.int64) + 64 * np.array(nwords),
                                 [0, (1 << 35)]])).astype(np.uint64)
    got = pcconv.shard_batch_starts(bm.data_ptr(), nwords, key0, gs)
    ref = NumpyShardOps(None).batch_starts(bm.cpu(), nwords, key0, gs)
    assert np.array_equal(got, ref)


def test_event_table_build_beyond_2p32_keys(tmp_path):
    """A rank's build with rank-local keys whose event batches are those of a
    cloud of more than 2^32 points (batch numbers near 5e5 of 10 000 points):
    the cells equal the oracle's when it is fed the same batch sequence."""
    from gpu_util import compare_dirs
    from oracle_ctypes import Oracle
    from pcconv.dist import event_table
    cfg = dict(cell_point_overflow_limit=40, sub_grid_dimension=8)
    p = synth(51, 1, 30_000)
    rng = np.random.default_rng(3)
    # 30 000 points spread over batches 430 000 .. 430 300 (keys > 4.3e9), some batches skipped
    eb = np.sort(rng.choice(np.arange(430_000, 430_300), size=len(p)))
    starts = np.flatnonzero(np.concatenate([[True], eb[1:] != eb[:-1]]))
    total = 430_400
    etab = event_table(starts, eb[starts], len(p), total)
    go, oo = str(tmp_path / "g"), str(tmp_path / "o")
    c = pcconv.Converter(go, batch_size=10_000, config=cfg)
    t = as_tensor(p).to(DEV)
    c.set_event_table(*etab)
    c.set_keyed_points_device(t.data_ptr(), 0, len(p))
    torch.cuda.synchronize()
    c.build()
    c.write()
    c.close()
    o = Oracle(cfg)
    NumpyShardOps(None)._feed_table(o, p, etab)
    assert o.error == 0
    o.write(oo)
    o.close()
    d, mg, mo = compare_dirs(go, oo)
    assert d == [], d[:5]
    assert mg == mo


# ---- exchange overlap: level-0 pass 1 on the groups of tiles whose points have
# landed (pcc_input_landed), the build running the rest
def _landed_build(out, p, cfg, ranges, stream=0):
    from pcconv.dist import event_table
    n = len(p)
    starts = np.arange(0, n, 10_000)
    etab = event_table(starts, np.arange(len(starts)), n, len(starts))
    c = pcconv.Converter(out, batch_size=10_000, config=cfg)
    t = as_tensor(p).to(DEV)
    torch.cuda.synchronize()
    c.set_event_table(*etab)
    c.set_keyed_points_device(t.data_ptr(), 0, n)
    for a, b in ranges:
        c.input_landed(a, b, stream)
    st = c.build()
    c.write()
    c.close()
    return st


@pytest.mark.parametrize("order", ["forward", "shuffled", "overlapping", "partial", "none", "nan", "wide"])
def test_input_landed_matches_oracle(tmp_path, order):
    """Ranges landed in any order (overlapping, some never: the build runs those
    groups) give the oracle's cloud; pass 1 ran early on the landed groups when
    the level-0 grid folds (at most two cells per axis)."""
    from gpu_util import compare_dirs
    cfg = dict(cell_point_overflow_limit=500, sub_grid_dimension=32)
    n = 700_001
    # "wide": ten level-0 cells per axis, no fold (pass 1 all inside the build)
    p = synth(71, 0, n) if order != "wide" else synth(72, 0, n, lo=-5000.0, ext=10000.0)
    if order == "nan":   # NaN coordinates in a late tile: the build redoes level 0 the non-finite way
        p["x"][n - 5_000:n - 4_990] = np.nan
    rng = np.random.default_rng(8)
    cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n, size=40)]))
    ranges = [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    if order == "shuffled" or order == "nan" or order == "wide":
        rng.shuffle(ranges)
    elif order == "overlapping":
        ranges = [(max(0, a - 5000), min(n, b + 7000)) for a, b in ranges]
        rng.shuffle(ranges)
    elif order == "partial":
        ranges = ranges[::3]
    elif order == "none":
        ranges = []
    go, oo = str(tmp_path / "g"), str(tmp_path / "o")
    st = _landed_build(go, p, cfg, ranges)
    assert run_oracle(oo, [p], cfg=cfg)[0] == 0
    d, mg, mo = compare_dirs(go, oo)
    assert d == [], d[:5]
    assert mg == mo
    if order in ("forward", "shuffled", "overlapping", "partial"):
        assert st["level0_early_tiles"] > 0, st
    else:
        assert st["level0_early_tiles"] == 0, st


def test_input_landed_behind_a_stream(tmp_path):
    """The points copied in on another stream, each piece's range handed over
    with that stream: the engine's pass 1 waits for the copy, not the host."""
    from gpu_util import compare_dirs
    from pcconv.dist import event_table
    cfg = dict(cell_point_overflow_limit=500, sub_grid_dimension=32)
    n = 500_000
    p = synth(73, 0, n)
    src = as_tensor(p).to(DEV)
    dst = torch.empty_like(src)
    starts = np.arange(0, n, 10_000)
    etab = event_table(starts, np.arange(len(starts)), n, len(starts))
    go, oo = str(tmp_path / "g"), str(tmp_path / "o")
    c = pcconv.Converter(go, batch_size=10_000, config=cfg)
    torch.cuda.synchronize()
    c.set_event_table(*etab)
    c.set_keyed_points_device(dst.data_ptr(), 0, n)
    s = torch.cuda.Stream(DEV)
    with torch.cuda.stream(s):
        for a in range(0, n, 100_000):
            b = min(n, a + 100_000)
            torch.cuda._sleep(2_000_000)   # the copy lands well after the call returns
            dst[a:b].copy_(src[a:b])
            c.input_landed(a, b, s.cuda_stream)
    st = c.build()
    c.write()
    c.close()
    assert st["level0_early_tiles"] > 0
    assert run_oracle(oo, [p], cfg=cfg)[0] == 0
    d, mg, mo = compare_dirs(go, oo)
    assert d == [], d[:5]
    assert mg == mo


def test_input_landed_refused_without_event_table(tmp_path):
    c = pcconv.Converter(str(tmp_path / "g"))
    t = as_tensor(synth(74, 0, 1000)).to(DEV)
    c.declare_files([1000])
    c.set_keyed_points_device(t.data_ptr(), 0, 1000)
    with pytest.raises(pcconv.PccError, match="event table"):
        c.input_landed(0, 1000)
    c.close()


@pytest.mark.parametrize("rounds", [0, 3])
def test_sharded_threads_exchange_rounds(tmp_path, rounds):
    """Thread ranks whose exchange lands in rounds with pass 1 behind each (the
    product default) or in one exchange: both equal the oracle; with rounds the
    ranks' level-0 pass 1 ran on landed tiles before the build."""
    files = [synth(75, 0, 1_200_000)]
    out = str(tmp_path / "out")
    fp = [len(f) for f in files]
    world = 2
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            torch.cuda.set_device(DEV)
            pts, key0 = rank_slice(files, r, world)
            ops = HipShardOps(0, out_dir=out, config=dict(sub_grid_dimension=32))
            ops.landing_rounds = rounds
            t = as_tensor(pts).to(DEV)
            res[r] = shard_build(ThreadComm(grp, r, DEV), ops, t, key0, fp, write=True)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    early = [int(r.local.get("level0_early_tiles", 0)) for r in res]
    assert all(e > 0 for e in early) if rounds > 1 else all(e == 0 for e in early), early
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=dict(sub_grid_dimension=32))


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_threads_keys_past_2p32(tmp_path, world):
    """Thread ranks with the HIP ops whose global keys start at 2^32 (a first
    file no rank holds: synthetic sparse keys), rank-local keys and event
    tables, the exchange in rounds: == the oracle fed the same batches."""
    from test_dist_cpu import check_phantom_against_oracle, phantom_case
    real, fp = phantom_case()
    out = str(tmp_path / "out")
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            torch.cuda.set_device(DEV)
            pts, key0 = rank_slice(real, r, world)
            ops = HipShardOps(0, out_dir=out)
            t = as_tensor(pts).to(DEV)
            res[r] = shard_build(ThreadComm(grp, r, DEV), ops, t, key0 + fp[0], fp, write=True)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert all(r.summary == res[0].summary for r in res)
    check_phantom_against_oracle(tmp_path, real, fp, out, res[0].summary)


def test_sharded_threads_wide_subgrid(tmp_path):
    """Thread ranks with the HIP ops at sub_grid_dimension 128 (the sequential
    replay per rank, rank-local keys and event tables): == the oracle."""
    cfg = dict(sub_grid_dimension=128, cell_point_overflow_limit=300)
    files = make_input("files")
    out = str(tmp_path / "out")
    res = _run_threads(files, 3, out, cfg=cfg)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg)


def test_input_landed_refused_for_merge_and_after_build(tmp_path):
    """pcc_input_landed is for a borrowed, event-table input before its build:
    a merge (its seeds come first) and a call after the build are refused."""
    from pcconv.dist import event_table
    p = synth(76, 0, 50_000)
    t = as_tensor(p).to(DEV)
    etab = event_table(np.arange(0, len(p), 10_000), np.arange(5), len(p), 5)
    c = pcconv.Converter(str(tmp_path / "g"))
    c.set_event_table(*etab)
    c.set_keyed_points_device(t.data_ptr(), 0, len(p))
    torch.cuda.synchronize()
    c.input_landed(0, 20_000)
    c.build()
    with pytest.raises(pcconv.PccError, match="after build"):
        c.input_landed(20_000, 50_000)
    c.write()
    c.close()
    m = pcconv.Converter(str(tmp_path / "g"))   # reopens the cloud just written: a merge
    m.set_event_table(*etab)
    m.set_keyed_points_device(t.data_ptr(), 0, len(p))
    with pytest.raises(pcconv.PccError, match="merge"):
        m.input_landed(0, len(p))
    m.close()
