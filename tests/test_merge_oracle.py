"""Incremental merge (lib.rs:86-101 load_metadata + converter.rs:187-207
load_or_create_cell): CPU checks of the oracle's loader.

Converting files A into an empty directory and then files B into the same
directory must give exactly the cloud of converting A then B in one run: the
converter's whole state is its cells and metadata.json, both on disk between
runs, and FxHashMap orders do not change results (cells and buckets are
independent).  Pinned three ways on adversarial small cases: the C oracle's
loader, the independent Python sequential restatement seeded with the on-disk
state, and the one-run conversion.
"""
import os
import random
import shutil
import sys
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, HERE)

import canon  # noqa: E402
import pyref  # noqa: E402
from oracle_ctypes import Oracle  # noqa: E402
from test_oracle_xcheck import _case, _to_np  # noqa: E402


def _split(files, seed):
    rng = random.Random(1000 + seed)
    k = rng.randint(1, len(files)) if len(files) > 1 else 1
    if len(files) == 1:   # cut the single file in two
        f = files[0]
        c = rng.randint(1, max(1, len(f) - 1))
        return [f[:c]], [f[c:]]
    return files[:k], files[k:] or [files[-1][: len(files[-1]) // 2]]


@pytest.mark.parametrize("seed", range(40))
def test_oracle_merge_equals_one_run(seed):
    files, cfg, batch = _case(seed)
    first, second = _split(files, seed)
    with tempfile.TemporaryDirectory() as d1, tempfile.TemporaryDirectory() as d2:
        o = Oracle(cfg)
        for f in first:
            o.add_file(_to_np(f), batch)
        o.write(d1)
        o.close()
        prior = canon.read_dir(d1)
        # loader: state from disk + second files
        m = Oracle()
        m.load(d1)
        for f in second:
            m.add_file(_to_np(f), batch)
        assert m.error == 0
        m.write(d1)
        merged = canon.read_dir(d1)
        # one run over all files
        r = Oracle(cfg)
        for f in first + second:
            r.add_file(_to_np(f), batch)
        r.write(d2)
        one = canon.read_dir(d2)
        assert canon.diff(merged[0], one[0]) == []
        assert merged == one
        # independent restatement seeded with the on-disk state
        seq, mseq = pyref.convert_sequential(second, cfg, batch, prior=prior)
        assert canon.diff(seq, one[0]) == []
        assert seq == one[0]
        assert mseq == one[1]
