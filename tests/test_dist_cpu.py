"""Sharded (multi-GPU) orchestration on CPU ranks — SURVEY.md §8e.

pcconv/dist.py runs unchanged over gloo (world size 2, separate processes) and
over in-process thread ranks, with the CPU test double tests/shard_np.py for the
local work.  The union of the ranks' cell files plus rank 0's metadata must equal
the single-process sequential oracle's output on the same input.
"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))

import canon  # noqa: E402
from gpu_util import run_oracle  # noqa: E402
from oracle_ctypes import synth  # noqa: E402
from pcconv.dist import ThreadComm, ThreadGroup, TorchComm, assign_owners, key_range, shard_build  # noqa: E402
from shard_np import NumpyShardOps, as_tensor  # noqa: E402


def make_input(case):
    """(list of per-file point arrays) for a named case."""
    if case == "uniform":
        return [synth(11, 0, 120_000)]
    if case == "files":     # ragged files incl. an empty one: batch structure crosses rank key ranges
        return [synth(12, 0, 33_333), synth(13, 0, 0), synth(14, 1, 47_001, lo=-1500.0, ext=3000.0)]
    if case == "clustered":
        return [synth(15, 1, 90_000)]
    raise KeyError(case)


def rank_slice(files, rank, world):
    allp = np.concatenate(files) if files else np.zeros(0)
    a, b = key_range(len(allp), rank, world)
    return allp[a:b], a


def check_against_oracle(tmp_path, files, out_dir, summary, cfg=None, batch=10_000):
    ref = str(tmp_path / "oracle")
    err, _ = run_oracle(ref, files, cfg, batch)
    assert err == 0
    ca, ma = canon.read_dir_fast(ref)
    cb, mb = canon.read_dir_fast(out_dir)
    d = canon.diff_fast(ca, cb)
    assert not d, d
    assert summary["number_of_points"] == ma["number_of_points"] == mb["number_of_points"]
    assert summary["hierarchies"] == ma["hierarchies"] == mb["hierarchies"]
    assert ma["bmin"] == mb["bmin"] and ma["bmax"] == mb["bmax"]


# ------------------------------------------------------------- owner table
def test_assign_owners_greedy_balanced_and_deterministic():
    h = np.array([0, 50, 10, 10, 0, 40, 30, 20], dtype=np.int64)
    o = assign_owners(h, 2)
    assert (assign_owners(h, 2) == o).all()
    load = [int(h[o == r].sum()) for r in range(2)]
    assert sorted(load) == [80, 80]
    assert (o[h == 0] == 0).all()
    assert (assign_owners(h, 1) == 0).all()


def test_assign_owners_eight_octants_one_per_rank():
    h = np.full(8, 125_000_000, dtype=np.int64)
    assert sorted(assign_owners(h, 8).tolist()) == list(range(8))
    o4 = assign_owners(h, 4)
    assert [int((o4 == r).sum()) for r in range(4)] == [2, 2, 2, 2]


def test_assign_owners_many_cells_prefix_split():
    rng = np.random.default_rng(0)
    h = rng.integers(0, 1000, size=20_000)
    o = assign_owners(h, 3, greedy_max=100)
    assert (np.diff(o[h > 0].astype(np.int64)) >= 0).all()   # contiguous ranges
    load = np.array([h[o == r].sum() for r in range(3)])
    assert load.max() - load.min() <= 2 * h.max()


# ------------------------------------------------------------- thread ranks
# bitmap: the exchange carries membership bitmaps (keys rebuilt by the receiver),
# else a 4-B key per routed point
# mode: "fused" bounding box + slab histogram in one pass over a guessed grid
# (the default), "miss" a guess that leaves points outside (histogram again on
# the true grid), "plain" the separate box and histogram passes
@pytest.mark.parametrize("case,world,bitmap,mode", [("uniform", 1, True, "fused"), ("uniform", 2, True, "fused"),
                                                    ("uniform", 2, False, "fused"), ("files", 3, True, "fused"),
                                                    ("files", 3, False, "fused"), ("clustered", 4, True, "fused"),
                                                    ("clustered", 3, True, "miss"), ("files", 2, True, "plain")])
def test_thread_ranks_match_oracle(tmp_path, case, world, bitmap, mode):
    import threading
    files = make_input(case)
    fp = [len(f) for f in files]
    out = str(tmp_path / "out")
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(files, r, world)
            ops = NumpyShardOps(out)
            ops.bitmap_keys = bitmap
            if mode == "plain":
                ops.fused_bbox_hist = False
            elif mode == "miss":   # a sample box of one point: the guessed grid misses the rest
                ops.bbox_sample = lambda p: ([float(v) for v in p[0, :3].view(torch.float32)],) * 2
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True)
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
    assert sum(r.recv_points for r in res) == sum(fp)
    assert all(r.summary == res[0].summary for r in res)
    check_against_oracle(tmp_path, files, out, res[0].summary)


@pytest.mark.parametrize("cells,expect", [(4, 4 ** 3), (6, 8 ** 3)])
def test_guess_grid_prefers_lds_histogram(tmp_path, cells, expect):
    """A sample box of 4 cells a side: with the one-cell margin the guess would be
    6^3 cells x 256 layers, past the fused kernel's LDS histogram, so the guess
    drops the margin (4^3); at 6 cells a side neither fits and the margin stays.
    Either way the result matches the oracle (points the guess misses are taken
    again on the true grid)."""
    import threading
    files = make_input("uniform")
    fp = [len(f) for f in files]
    out = str(tmp_path / "out")
    grp = ThreadGroup(2)
    res, errs, seen = [None] * 2, [], []

    def worker(r):
        try:
            pts, key0 = rank_slice(files, r, 2)
            ops = NumpyShardOps(out)
            cs = float(ops.cfg_full()["max_cell_size"])
            ops.bbox_sample = lambda p: ([0.25 * cs] * 3, [(cells - 0.75) * cs] * 3)
            fused = ops.bbox_slab_histogram

            def record(p, guess):
                seen.append(int(guess.ncells))
                return fused(p, guess)
            ops.bbox_slab_histogram = record
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, errs
    assert seen == [expect, expect]
    assert all(r.summary == res[0].summary for r in res)
    check_against_oracle(tmp_path, files, out, res[0].summary)


def test_thread_ranks_empty_input(tmp_path):
    import threading
    grp = ThreadGroup(2)
    res = [None, None]

    def worker(r):
        ops = NumpyShardOps(str(tmp_path / "out"))
        pts = as_tensor(np.zeros(0, dtype=synth(1, 0, 1).dtype))
        res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, pts, 0, [0], write=False)

    th = [threading.Thread(target=worker, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert res[0].summary == {"number_of_points": 0, "hierarchies": 1, "bbox_min": [0.0] * 3, "bbox_max": [0.0] * 3}


# ------------------------------------------------------------- gloo, 2 processes
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, case, out, res_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        files = make_input(case)
        pts, key0 = rank_slice(files, rank, world)
        ops = NumpyShardOps(out)
        r = shard_build(TorchComm(torch.device("cpu")), ops, as_tensor(pts), key0, [len(f) for f in files],
                        write=True)
        ops.close()
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"summary": r.summary, "recv": r.recv_points, "owned": r.owned_cells}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["uniform", "files"])
def test_gloo_world2_matches_oracle(tmp_path, case):
    import torch.multiprocessing as mp
    out, rd = str(tmp_path / "out"), str(tmp_path / "res")
    os.makedirs(rd)
    mp.spawn(_gloo_worker, args=(2, _free_port(), case, out, rd), nprocs=2, join=True)
    r = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(2)]
    files = make_input(case)
    assert r[0]["summary"] == r[1]["summary"]
    assert r[0]["recv"] + r[1]["recv"] == sum(len(f) for f in files)
    if case == "uniform":
        assert r[0]["owned"] == r[1]["owned"] == 4     # 8 level-0 octants, 4 per rank
    check_against_oracle(tmp_path, files, out, r[0]["summary"])


# ------------------------------------------------------------- sharded incremental merge (config 5)
def make_merge_input(case):
    """(existing files, new files) for a named merge case."""
    if case == "uniform":
        return [synth(21, 0, 80_000)], [synth(22, 0, 30_000)]
    if case == "partial":   # new points in one octant plus new level-0 cells beyond the old bbox
        return [synth(23, 0, 60_000)], [synth(24, 0, 20_000, lo=100.0, ext=800.0),
                                        synth(25, 0, 7_000, lo=-1900.0, ext=800.0)]
    if case == "clustered":
        return [synth(26, 1, 50_000)], [synth(27, 1, 40_000)]
    raise KeyError(case)


def _thread_merge(out, new_files, world):
    import threading
    fp = [len(f) for f in new_files]
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(new_files, r, world)
            ops = NumpyShardOps(out, merge=True)
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True,
                                 merge=True)
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


@pytest.mark.parametrize("case,world", [("uniform", 2), ("partial", 3), ("clustered", 4)])
def test_thread_ranks_merge_matches_oracle(tmp_path, case, world):
    """Existing cloud (oracle-written) + new points merged by `world` ranks, each
    rewriting only its subtrees, == the oracle converting old and new files in
    one run (the reference's incremental-merge semantics, converter.rs:187-207)."""
    old, new = make_merge_input(case)
    out = str(tmp_path / "out")
    err, _ = run_oracle(out, old)
    assert err == 0
    res = _thread_merge(out, new, world)
    assert all(r.summary == res[0].summary for r in res)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in new)
    check_against_oracle(tmp_path, old + new, out, res[0].summary)


def test_thread_ranks_merge_no_new_points(tmp_path):
    old, _ = make_merge_input("uniform")
    out = str(tmp_path / "out")
    assert run_oracle(out, old)[0] == 0
    res = _thread_merge(out, [np.zeros(0, dtype=old[0].dtype)], 2)
    assert res[0].summary["number_of_points"] == len(old[0])
    check_against_oracle(tmp_path, old + [np.zeros(0, dtype=old[0].dtype)], out, res[0].summary)


def _gloo_merge_worker(rank, world, port, case, out, res_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, new = make_merge_input(case)
        pts, key0 = rank_slice(new, rank, world)
        ops = NumpyShardOps(out, merge=True)
        r = shard_build(TorchComm(torch.device("cpu")), ops, as_tensor(pts), key0, [len(f) for f in new],
                        write=True, merge=True)
        ops.close()
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"summary": r.summary, "recv": r.recv_points}, f)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_merge_matches_oracle(tmp_path):
    import torch.multiprocessing as mp
    old, new = make_merge_input("partial")
    out, rd = str(tmp_path / "out"), str(tmp_path / "res")
    os.makedirs(rd)
    assert run_oracle(out, old)[0] == 0
    mp.spawn(_gloo_merge_worker, args=(2, _free_port(), "partial", out, rd), nprocs=2, join=True)
    r = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(2)]
    assert r[0]["summary"] == r[1]["summary"]
    check_against_oracle(tmp_path, old + new, out, r[0]["summary"])


def _gloo_chunked_worker(rank, world, port, out, res_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        files = make_input("files")
        pts, key0 = rank_slice(files, rank, world)
        comm = TorchComm(torch.device("cpu"))
        comm.max_msg_bytes = 1 << 16   # force every peer segment into many transfers
        ops = NumpyShardOps(out)
        r = shard_build(comm, ops, as_tensor(pts), key0, [len(f) for f in files], write=True)
        ops.close()
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"summary": r.summary, "recv": r.recv_points}, f)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_chunked_exchange_matches_oracle(tmp_path):
    """Peer segments split into many transfers (TorchComm.max_msg_bytes) give the same exchange."""
    import torch.multiprocessing as mp
    out, rd = str(tmp_path / "out"), str(tmp_path / "res")
    os.makedirs(rd)
    mp.spawn(_gloo_chunked_worker, args=(2, _free_port(), out, rd), nprocs=2, join=True)
    r = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(2)]
    files = make_input("files")
    assert r[0]["recv"] + r[1]["recv"] == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, r[0]["summary"])


# ------------------------------------------------------------- exchange in rounds (pass 1 behind each)
def test_round_pieces_and_landed_ranges_tile_the_receive_buffer():
    from pcconv.dist import landed_ranges, round_piece
    rng = np.random.default_rng(5)
    for _ in range(200):
        world, rounds = int(rng.integers(1, 9)), int(rng.integers(1, 9))
        rc = [int(v) for v in rng.integers(0, 40, size=world)]
        me = int(rng.integers(0, world))
        for cnt in rc:
            assert [round_piece(cnt, r, rounds) for r in range(rounds)][-1][1] == cnt
            assert all(round_piece(cnt, r, rounds)[1] == round_piece(cnt, r + 1, rounds)[0] for r in range(rounds - 1))
        got = sorted(x for r in range(rounds) for x in landed_ranges(rc, me, r, rounds))
        pos = 0
        for a, b in got:
            assert a == pos and b > a
            pos = b
        assert pos == sum(rc)
        assert sum(b - a for a, b in landed_ranges(rc, me, 0, rounds)) >= rc[me]   # the own segment first


@pytest.mark.parametrize("rounds,world", [(0, 3), (1, 2), (2, 3), (7, 4)])
def test_thread_ranks_landing_rounds_match_oracle(tmp_path, rounds, world):
    """The exchange in `rounds` rounds with the build's input borrowed before it
    (HipShardOps.begin_landing / landed / build_landed; 0: one exchange, then the
    build): every round reports its ranges, they tile the receive buffer, and
    the cloud equals the oracle's."""
    import threading
    files = make_input("files")
    fp = [len(f) for f in files]
    out = str(tmp_path / "out")
    grp = ThreadGroup(world)
    res, logs, errs = [None] * world, [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(files, r, world)
            ops = NumpyShardOps(out)
            ops.landing_rounds = rounds
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True)
            logs[r] = getattr(ops, "landed_log", None)
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
    for lg in logs:
        assert (lg is None) if rounds <= 1 else (len(lg) == rounds)
    assert all(r.summary == res[0].summary for r in res)
    check_against_oracle(tmp_path, files, out, res[0].summary)


def _gloo_rounds_worker(rank, world, port, out, res_dir, rounds):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        files = make_input("files")
        pts, key0 = rank_slice(files, rank, world)
        comm = TorchComm(torch.device("cpu"))
        comm.max_msg_bytes = 1 << 14   # pieces of rounds in several transfers too
        ops = NumpyShardOps(out)
        ops.landing_rounds = rounds
        r = shard_build(comm, ops, as_tensor(pts), key0, [len(f) for f in files], write=True)
        ops.close()
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"summary": r.summary, "recv": r.recv_points, "log": ops.landed_log}, f)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_exchange_rounds_match_oracle(tmp_path):
    """TorchComm.alltoallv_rounds over gloo: round r + 1 posted before round r is
    waited for, each round's ranges handed to the ops, the cloud == the oracle's."""
    import torch.multiprocessing as mp
    out, rd = str(tmp_path / "out"), str(tmp_path / "res")
    os.makedirs(rd)
    mp.spawn(_gloo_rounds_worker, args=(2, _free_port(), out, rd, 5), nprocs=2, join=True)
    r = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(2)]
    files = make_input("files")
    assert r[0]["recv"] + r[1]["recv"] == sum(len(f) for f in files)
    assert all(len(x["log"]) == 5 for x in r)
    check_against_oracle(tmp_path, files, out, r[0]["summary"])


def test_hip_shard_ops_config_and_fresh_dir_guards(tmp_path):
    """HipShardOps refuses (before any device work): a merge whose caller config
    differs from the existing cloud's metadata.json, and a non-merge run into a
    directory that already holds a cloud (pcc_open would merge on every rank)."""
    import json
    from pcconv.dist import HipShardOps
    d = tmp_path / "cloud"
    d.mkdir()
    meta = {"version": "1.0", "name": "Unknown", "number_of_points": 10, "hierarchies": 1,
            "bounding_box": {"min": [0.0, 0.0, 0.0], "max": [1.0, 1.0, 1.0]},
            "config": {"cell_point_overflow_limit": 5000, "sub_grid_dimension": 96, "max_cell_size": 500.0}}
    (d / "metadata.json").write_text(json.dumps(meta))
    with pytest.raises(ValueError, match="max_cell_size"):
        HipShardOps(0, out_dir=str(d), config=dict(max_cell_size=1000.0), merge=True)
    ops = HipShardOps(0, out_dir=str(d), merge=True)   # no converter opened yet
    assert ops.cfg["max_cell_size"] == 500.0 and ops.max_cell_size == 500.0
    with pytest.raises(ValueError, match="merge=True"):
        HipShardOps(0, out_dir=str(d))


# ------------------------------------------------------------- skewed clouds: heavy level-0 cells split at level 1
SKEW_CFG = {"sub_grid_dimension": 16, "cell_point_overflow_limit": 100, "max_cell_size": 1000.0}


def make_skewed(case):
    if case == "gauss":      # Gaussian mixture (config-3 generator): a few heavy level-0 cells
        return [synth(61, 2, 150_000)]
    if case == "gauss_files":
        return [synth(62, 2, 70_001), synth(63, 0, 0), synth(64, 2, 33_333)]
    raise KeyError(case)


@pytest.mark.parametrize("case,world,bitmap", [("gauss", 3, True), ("gauss", 3, False), ("gauss", 8, True),
                                               ("gauss_files", 5, True)])
def test_thread_ranks_split_cells_match_oracle(tmp_path, case, world, bitmap):
    """Heavy level-0 cells built by a leader (level 0) and the owners of their
    level-1 sub-trees (plan_split) == the sequential oracle."""
    import threading
    files = make_skewed(case)
    fp = [len(f) for f in files]
    out = str(tmp_path / "out")
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(files, r, world)
            ops = NumpyShardOps(out, config=SKEW_CFG)
            ops.bitmap_keys = bitmap
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True)
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
    assert res[0].plan["split_cells"] > 0
    assert all(r.plan == res[0].plan for r in res)
    assert sum(r.recv_points for r in res) == sum(fp)
    assert sum(r.local["phases"]["sub"] for r in res) > 0
    assert all(r.summary == res[0].summary for r in res)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=SKEW_CFG)


def _gloo_split_worker(rank, world, port, out, res_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        files = make_skewed("gauss")
        pts, key0 = rank_slice(files, rank, world)
        comm = TorchComm(torch.device("cpu"))
        comm.max_msg_bytes = 1 << 14   # many transfers per peer segment in both exchanges
        ops = NumpyShardOps(out, config=SKEW_CFG)
        r = shard_build(comm, ops, as_tensor(pts), key0, [len(f) for f in files], write=True)
        ops.close()
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"summary": r.summary, "recv": r.recv_points, "plan": r.plan, "phases": r.local["phases"]}, f)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_split_cells_match_oracle(tmp_path):
    import torch.multiprocessing as mp
    out, rd = str(tmp_path / "out"), str(tmp_path / "res")
    os.makedirs(rd)
    mp.spawn(_gloo_split_worker, args=(2, _free_port(), out, rd), nprocs=2, join=True)
    r = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(2)]
    files = make_skewed("gauss")
    assert r[0]["summary"] == r[1]["summary"]
    assert r[0]["plan"]["split_cells"] > 0
    assert r[0]["recv"] + r[1]["recv"] == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, r[0]["summary"], cfg=SKEW_CFG)


def test_plan_split_uniform_is_assign_owners():
    """Equal level-0 cells on as many ranks: nothing to gain, nothing split."""
    from pcconv.dist import plan_split
    h0 = np.full(8, 1000, dtype=np.int64)
    h1 = np.full(64, 125, dtype=np.int64)
    ch = np.arange(64).reshape(8, 8)
    sh = np.zeros((8, 256), np.int64)
    sh[:, 10:30] = 50
    p = plan_split(h0, h1, ch, 8, slab_hist=sh.reshape(-1))
    assert not p.split.any() and (p.owner0 == assign_owners(h0, 8)).all()
    # one heavy cell among light ones: shared, its 40 slabs spread over all ranks
    h0 = np.array([8000, 10, 10, 10], np.int64)
    sh = np.zeros((4, 256), np.int64)
    sh[0, 20:60] = 200
    sh[1:, 5] = 10
    p3 = plan_split(h0, np.concatenate([np.full(8, 1000), np.zeros(24)]).astype(np.int64), np.arange(32).reshape(4, 8), 4,
                    slab_hist=sh.reshape(-1))
    assert p3.split[0] and not p3.split[1:].any()
    assert sorted(set(p3.slab_owner[20:60].tolist())) == [0, 1, 2, 3]
    assert p3.est["ratio"] < 0.8 * plan_split(h0, None, None, 4, allow=False).est["ratio"]


def test_thread_ranks_sparse_wide_cloud_coarse_grid(tmp_path):
    """A cloud whose level-0 grid exceeds the shard grid's 2^22 cells (64e9 cells
    of size 1 here): ownership falls back to blocks of 2^k x 2^k x 2^k level-0
    cells (shard_grid), every level-0 sub-tree still on one rank == the oracle."""
    import threading
    from pcconv.dist import shard_grid
    cfg = {"sub_grid_dimension": 4, "cell_point_overflow_limit": 8, "max_cell_size": 1.0}
    files = [synth(81, 0, 30_000, lo=-2000.0, ext=4000.0), synth(82, 1, 20_000, lo=-2000.0, ext=4000.0)]
    g = shard_grid([-2000.0] * 3, [2000.0] * 3, 1.0)
    assert g.coarse > 0 and g.ncells <= (1 << 22)
    fp = [len(f) for f in files]
    out = str(tmp_path / "out")
    world = 3
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(files, r, world)
            ops = NumpyShardOps(out, config=cfg)
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True)
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
    assert sum(r.recv_points for r in res) == sum(fp)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg)


def test_lpt_matches_heap_restatement():
    """pcc_shard_lpt (the plan's C++ inner loop) == the heap formulation of
    largest-first greedy (heaviest first, ties by index, to the least loaded
    rank, ties by rank), owners and float64 loads alike."""
    import heapq
    import pcconv

    def lpt_py(w, world):
        own = np.zeros(len(w), dtype=np.uint32)
        load = np.zeros(world)
        heap = [(0.0, r) for r in range(world)]
        for i in np.lexsort((np.arange(len(w)), -w)).tolist():
            ld, r = heapq.heappop(heap)
            own[i] = r
            ld += float(w[i])
            load[r] = ld
            heapq.heappush(heap, (ld, r))
        return own, load
    rng = np.random.default_rng(1)
    for _ in range(200):
        n, world = int(rng.integers(0, 2000)), int(rng.integers(1, 17))
        w = rng.integers(0, 50, n).astype(np.float64) * rng.choice([1.0, 0.5, 3.0])
        a, b = lpt_py(w, world), pcconv.shard_lpt(w, world)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_plan_search_placement_equals_lpt_of_its_lists():
    """pcc_shard_plan_search's owners and loads for its best k (what plan_split
    uses) == pcc_shard_lpt over the two lists that k defines: phase 1 = the
    whole cells k.. then the slabs of cells ..k, phase 2 = those cells'
    children; and the best k minimises the estimate (a larger k only when more
    than 2 % lower)."""
    import pcconv
    rng = np.random.default_rng(5)
    for _ in range(120):
        world = int(rng.integers(2, 17))
        nc = int(rng.integers(1, 40))
        kmax = min(nc, 2 * world)
        whole = np.sort(rng.integers(1, 10_000, nc).astype(np.float64))[::-1].copy()
        whole[rng.random(nc) < 0.2] *= 20.0
        whole = np.sort(whole)[::-1].copy()
        ns = rng.integers(0, 30, kmax)
        nk = rng.integers(0, 9, kmax)
        so = np.concatenate([[0], np.cumsum(ns)]).astype(np.uint64)
        co = np.concatenate([[0], np.cumsum(nk)]).astype(np.uint64)
        sw = rng.integers(0, 500, int(so[-1])).astype(np.float64)
        cw = rng.integers(0, 2_000, int(co[-1])).astype(np.float64)
        k, t, ow, osl, och, l1, l2 = pcconv.shard_plan_search(whole, so, sw, co, cw, kmax, world, owners=True)
        assert (k, t) == pcconv.shard_plan_search(whole, so, sw, co, cw, kmax, world)
        s1 = int(so[k])
        o1, m1 = pcconv.shard_lpt(np.concatenate([whole[k:], sw[:s1]]), world)
        assert np.array_equal(np.concatenate([ow[k:], osl[:s1]]), o1) and np.array_equal(l1, m1)
        c1 = int(co[k])
        o2, m2 = pcconv.shard_lpt(cw[:c1], world)
        assert np.array_equal(och[:c1], o2) and np.array_equal(l2, m2)
        est = []
        for kk in range(kmax + 1):
            _, a = pcconv.shard_lpt(np.concatenate([whole[kk:], sw[:int(so[kk])]]), world)
            _, b = pcconv.shard_lpt(cw[:int(co[kk])], world)
            est.append(a.max() + (b.max() if int(co[kk]) else 0.0))
        best = 0
        for kk in range(1, kmax + 1):
            if est[kk] < est[best] * 0.98:
                best = kk
        assert k == best and t == est[best]


# ------------------------------------------------------------- NaN / infinite coordinates
# bounding-volume/src/lib.rs:23-31 (NaN skipped, infinities kept), metadata.rs:100-102
# (`as i32`: NaN -> cell 0, infinities saturate), cell.rs:77-80 (NaN never less).
# The ownership grid spans the cells of the points without an infinite
# coordinate (NaN as 0); the points with one travel as unit 0 (one rank builds
# them all); no cell is shared.
def _same_summary(a, b):
    return json.dumps(a, sort_keys=True) == json.dumps(b, sort_keys=True)   # NaN == NaN


def _thread_run(out, files, world, cfg, batch, merge=False, mode="fused"):
    import threading
    fp = [len(f) for f in files]
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(files, r, world)
            ops = NumpyShardOps(out, batch_size=batch, config=None if merge else cfg, merge=merge)
            if mode == "plain":
                ops.fused_bbox_hist = False
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True,
                                 merge=merge)
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
    assert all(_same_summary(r.summary, res[0].summary) for r in res)
    return res


@pytest.mark.parametrize("world,kinds,mode", [(2, "mixed", "fused"), (3, "mixed", "plain"), (4, "nan", "fused")])
def test_thread_ranks_nonfinite_match_oracle(tmp_path, world, kinds, mode):
    from nonfinite_input import NONFINITE_CFG, nonfinite_files
    files = nonfinite_files(seed=31, n=60_000, kinds=kinds)
    out = str(tmp_path / "out")
    res = _thread_run(out, files, world, NONFINITE_CFG, 5000, mode=mode)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=NONFINITE_CFG, batch=5000)


@pytest.mark.parametrize("world", [2, 3])
def test_thread_ranks_nonfinite_merge_matches_oracle(tmp_path, world):
    """NaN and +-inf points merged by `world` ranks into a cloud holding NaN points."""
    from nonfinite_input import NONFINITE_CFG, nonfinite_files
    old = nonfinite_files(seed=32, n=50_000, kinds="nan")
    new = nonfinite_files(seed=33, n=30_000, kinds="mixed")
    out = str(tmp_path / "out")
    assert run_oracle(out, old, NONFINITE_CFG, 5000)[0] == 0
    res = _thread_run(out, new, world, NONFINITE_CFG, 5000, merge=True)
    assert sum(r.recv_points for r in res) == sum(len(f) for f in new)
    check_against_oracle(tmp_path, old + new, out, res[0].summary, cfg=NONFINITE_CFG, batch=5000)


def _gloo_nonfinite_worker(rank, world, port, out, res_dir):
    import torch.distributed as dist
    from nonfinite_input import NONFINITE_CFG, nonfinite_files
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        files = nonfinite_files(seed=34, n=40_000, kinds="mixed")
        pts, key0 = rank_slice(files, rank, world)
        ops = NumpyShardOps(out, batch_size=5000, config=NONFINITE_CFG)
        r = shard_build(TorchComm(torch.device("cpu")), ops, as_tensor(pts), key0, [len(f) for f in files],
                        write=True)
        ops.close()
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"summary": r.summary, "recv": r.recv_points}, f)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_nonfinite_matches_oracle(tmp_path):
    import torch.multiprocessing as mp
    from nonfinite_input import NONFINITE_CFG, nonfinite_files
    out, rd = str(tmp_path / "out"), str(tmp_path / "res")
    os.makedirs(rd)
    mp.spawn(_gloo_nonfinite_worker, args=(2, _free_port(), out, rd), nprocs=2, join=True)
    r = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(2)]
    files = nonfinite_files(seed=34, n=40_000, kinds="mixed")
    assert _same_summary(r[0]["summary"], r[1]["summary"])
    assert r[0]["recv"] + r[1]["recv"] == sum(len(f) for f in files)
    check_against_oracle(tmp_path, files, out, r[0]["summary"], cfg=NONFINITE_CFG, batch=5000)


def test_global_batches_beyond_2p32_keys():
    """The batch table of a file structure of more than 2^32 points: 64-bit batch
    starts, an empty file one empty batch (lib.rs:31-52)."""
    from pcconv.dist import event_batches, global_batches
    fp = [(1 << 32) + 12_345, 0, 25_000]
    gs, gb, nbt = global_batches(fp, 10_000)
    n0 = ((1 << 32) + 12_345 + 9_999) // 10_000
    assert nbt == n0 + 1 + 3
    assert len(gs) == len(gb) == n0 + 3
    assert gs.dtype == np.uint64 and int(gs[n0 - 1]) == (n0 - 1) * 10_000
    assert int(gs[n0]) == (1 << 32) + 12_345 and int(gb[n0]) == n0 + 1   # after the empty file's batch
    k = np.array([0, 9_999, 10_000, (1 << 32) + 12_344, (1 << 32) + 12_345, (1 << 32) + 37_344], dtype=np.int64)
    assert list(event_batches(k, fp, 10_000)) == [0, 0, 1, n0 - 1, n0 + 1, n0 + 3]


# ------------------------------------------------------------- keys past 2^32 on thread ranks
def phantom_case():
    """Global keys past 2^32 with synthetic sparse keys: a first file of 2^32
    points that no rank holds (its batches are empty here), then the real
    files, whose keys therefore start at 2^32."""
    real = [synth(81, 0, 60_000), synth(82, 1, 25_001)]
    return real, [1 << 32] + [len(f) for f in real]


def check_phantom_against_oracle(tmp_path, real, fp, out, summary, cfg=None, batch=10_000):
    """The oracle fed the phantom file's batches empty, then the real files."""
    from oracle_ctypes import Oracle
    ref = str(tmp_path / "oracle")
    o = Oracle(cfg)
    empty = real[0][:0]
    for _ in range((fp[0] + batch - 1) // batch):
        o.add_batch(empty)
    for f in real:
        o.add_file(f, batch)
    assert o.error == 0
    o.write(ref)
    o.close()
    ca, ma = canon.read_dir_fast(ref)
    cb, mb = canon.read_dir_fast(out)
    d = canon.diff_fast(ca, cb)
    assert not d, d[:5]
    assert summary["number_of_points"] == sum(fp)
    assert summary["hierarchies"] == ma["hierarchies"] == mb["hierarchies"]
    assert ma["bmin"] == mb["bmin"] and ma["bmax"] == mb["bmax"]


@pytest.mark.parametrize("world", [2, 3])
def test_thread_ranks_keys_past_2p32_match_oracle(tmp_path, world):
    """Thread ranks whose global keys start at 2^32 (rank-local keys + event
    tables over 429 499 global batches) == the oracle fed the same batches."""
    import threading
    real, fp = phantom_case()
    out = str(tmp_path / "out")
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(real, r, world)
            ops = NumpyShardOps(out)
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0 + fp[0], fp,
                                 write=True)
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


@pytest.mark.parametrize("stage", ["bbox_sample", "bbox_slab_histogram", "bbox"])
def test_rank_failure_in_bbox_pass_raises_on_every_rank(tmp_path, stage):
    """One rank's local bounding-box pass raising: every rank raises after the
    collective (the failing rank its own error, the others a named one) instead
    of the others waiting in the all-reduce forever."""
    import threading
    files = make_input("files")
    fp = [len(f) for f in files]
    world = 3
    grp = ThreadGroup(world)
    errs = [None] * world

    def worker(r):
        pts, key0 = rank_slice(files, r, world)
        ops = NumpyShardOps(str(tmp_path / "out"))
        if stage == "bbox":
            ops.fused_bbox_hist = False
        if r == 1:
            def boom(*a, **k):
                raise ValueError("injected failure")
            setattr(ops, stage, boom)
        try:
            shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a rank is still waiting in a collective"
    assert isinstance(errs[1], ValueError) and "injected" in str(errs[1])
    for r in (0, 2):
        assert isinstance(errs[r], RuntimeError) and "another rank failed" in str(errs[r]), errs[r]


def test_thread_ranks_wide_subgrid_match_oracle(tmp_path):
    """sub_grid_dimension 128 (beyond the slab units): whole cells only, no fused
    slab histogram, against the oracle."""
    import threading
    cfg = dict(sub_grid_dimension=128, cell_point_overflow_limit=300)
    files = make_input("files")
    fp = [len(f) for f in files]
    out = str(tmp_path / "out")
    world = 3
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            pts, key0 = rank_slice(files, r, world)
            ops = NumpyShardOps(out, config=cfg)
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(pts), key0, fp, write=True)
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
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg)
