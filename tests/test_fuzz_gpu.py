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

from fuzz_cases import big_case, mid_case
from gpu_util import compare_dirs, run_gpu, run_oracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _shm():
    return "/dev/shm" if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK) else None


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
        assert d == [], (kind, cfg, batch, d)
        assert mg == mo
        assert st["arrivals"] == arrivals
        assert st["grid_points"] + st["kept_points"] == st["number_of_points"]


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


@pytest.mark.parametrize("seed", range(1, 48, 3))
def test_fuzz_sharded_threads_match_oracle(seed, tmp_path):
    """The sweep's cases sharded over 2-8 thread ranks on cuda:0 (pcconv.dist:
    level-0 cells or slabs owned per rank, the exchange in 0 or 2-5 rounds with
    level-0 pass 1 behind it), merged output against the oracle's one-process run."""
    import threading
    import numpy as np
    import torch
    from pcconv.dist import HipShardOps, ThreadComm, ThreadGroup, key_range, shard_build
    from test_dist_cpu import check_against_oracle
    from shard_np import as_tensor
    files, cfg, batch, kind = mid_case(seed)
    world = [2, 3, 4, 5, 8][seed % 5]
    rounds = [0, 2, 3, 5][seed % 4]
    fp = [len(f) for f in files]
    allp = np.concatenate(files)
    out = str(tmp_path / "out")
    dev = torch.device("cuda", 0)
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            torch.cuda.set_device(dev)
            a, b = key_range(len(allp), r, world)
            ops = HipShardOps(0, out_dir=out, batch_size=batch, config=cfg)
            ops.landing_rounds = rounds
            t = as_tensor(allp[a:b]).to(dev)
            res[r] = shard_build(ThreadComm(grp, r, dev), ops, t, a, fp, write=True)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, (kind, cfg, batch, world, errs)
    assert sum(r.recv_points for r in res) == len(allp)
    check_against_oracle(tmp_path, files, out, res[0].summary, cfg=cfg, batch=batch)
