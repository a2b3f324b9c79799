"""CPU side of the randomised sweep (tests/fuzz_cases.py): the case generator is
deterministic, and on each case's first 1 500 points the keyed restatement the
GPU build implements (oracle/pyref.py::convert_keyed) agrees with the sequential
C oracle (the reference's per-batch recursion), over the sweep's whole config
space: dimensions 1-96, limits 1-20 000, cell sizes 0.125-12 345, batches 1-50 000."""
import tempfile

import numpy as np
import pytest

import canon
import pyref
from fuzz_cases import mid_case
from oracle_ctypes import Oracle


def test_cases_deterministic():
    a, b = mid_case(5), mid_case(5)
    assert a[1:] == b[1:] and len(a[0]) == len(b[0])
    assert all(np.array_equal(x, y) for x, y in zip(a[0], b[0]))


@pytest.mark.parametrize("seed", range(0, 48, 3))
def test_keyed_restatement_agrees_with_oracle(seed):
    files, cfg, batch, _ = mid_case(seed)
    left, cut = 1500, []
    for f in files:
        cut.append(f[:max(0, min(len(f), left))])
        left -= len(cut[-1])
    py = [[(p["x"], p["y"], p["z"], tuple(int(c) for c in p["rgba"])) for p in f] for f in cut]
    key, mkey = pyref.convert_keyed(py, cfg, batch)
    with tempfile.TemporaryDirectory() as tmp:
        o = Oracle(cfg)
        for f in cut:
            o.add_file(f, batch)
        assert o.error == 0
        o.write(tmp)
        o.close()
        cells, meta = canon.read_dir(tmp)
    assert canon.diff(key, cells) == []
    assert meta == mkey


def _cpu_sharded(tmp_path, files, cfg, batch, world, merge=False, prior=None):
    """The sharding layer (pcconv.dist) on CPU thread ranks with the numpy shard
    ops, against the oracle: the same control flow the GPU sweep runs."""
    import threading
    import torch
    from gpu_util import run_oracle   # (puts the package on the path)
    from pcconv.dist import ThreadComm, ThreadGroup, key_range, shard_build
    from shard_np import NumpyShardOps, as_tensor
    from test_dist_cpu import check_against_oracle
    fp = [len(f) for f in files]
    allp = np.concatenate(files)
    out = str(tmp_path / "out")
    if merge:
        assert run_oracle(out, prior, cfg=cfg, batch=batch)[0] == 0
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            a, b = key_range(len(allp), r, world)
            ops = NumpyShardOps(out, batch_size=batch, config=cfg, merge=merge)   # (the numpy ops take no config from metadata.json)
            res[r] = shard_build(ThreadComm(grp, r, torch.device("cpu")), ops, as_tensor(allp[a:b]), a, fp,
                                 write=True, merge=merge)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs, errs
    check_against_oracle(tmp_path, (prior or []) + files, out, res[0].summary, cfg=cfg, batch=batch)


@pytest.mark.parametrize("seed", [7, 13, 19, 28, 31, 40])
def test_sharded_numpy_ops_match_oracle(seed, tmp_path):
    """Includes the sweep's cases that found a rank with no shared-cell
    segments (13, 19, 28) and kept lists above 8 192 points (7)."""
    files, cfg, batch, _ = mid_case(seed)
    _cpu_sharded(tmp_path, files, cfg, batch, [2, 3, 4, 5, 8][seed % 5])


@pytest.mark.parametrize("seed", [2, 10, 22])
def test_sharded_merge_numpy_ops_match_oracle(seed, tmp_path):
    from fuzz_cases import halves
    files, cfg, batch, _ = mid_case(seed)
    first, second = halves(files)
    _cpu_sharded(tmp_path, second, cfg, batch, 3, merge=True, prior=first)
