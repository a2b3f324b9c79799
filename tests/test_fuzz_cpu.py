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
