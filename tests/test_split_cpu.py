"""Level ranges on the CPU oracle (the test double of the split sharded build,
tests/shard_np.py): a hierarchy converted in pieces cut at level boundaries —
the points forwarded to the cut level recorded with their batch numbers, then
replayed batch by batch as the input of a converter rooted at that level —
gives exactly the cells of one whole run (converter.rs:114-139: a level-h cell
sees only the lists forwarded to it, one per batch).
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

from oracle_ctypes import Digest, Oracle, synth  # noqa: E402

SMALL = {"sub_grid_dimension": 16, "cell_point_overflow_limit": 100, "max_cell_size": 1000.0}


def whole_digest(files, cfg):
    o = Oracle(cfg)
    for f in files:
        o.add_file(f, 10_000)
    d = Digest()
    d.add_oracle(o)
    r = d.result()
    arr = o.arrivals
    d.close()
    o.close()
    return r, arr


def replay(o, pts, batch):
    """Recorded forwarded points as the batches of a rooted converter."""
    for e in np.unique(batch):
        o.add_batch(pts[batch == e])


@pytest.mark.parametrize("cuts", [[1], [2], [1, 2], [1, 3]])
def test_oracle_level_pieces_equal_whole(cuts):
    files = [synth(51, 1, 60_000), synth(52, 1, 9_999)]
    ref, arr = whole_digest(files, SMALL)
    d = Digest()
    bounds = [0] + cuts
    pend, total = None, 0
    for i, h0 in enumerate(bounds):
        m = bounds[i + 1] - h0 if i + 1 < len(bounds) else 0
        o = Oracle(SMALL)
        o.set_level_range(h0, m)
        if i == 0:
            for f in files:
                o.add_file(f, 10_000)
        else:
            replay(o, pend[0], pend[1])
        assert o.error == 0
        d.add_oracle(o)
        total += o.arrivals
        pend = o.pending()
        o.close()
        if len(pend[0]) == 0:
            break
    assert d.result() == ref
    assert total == arr
    d.close()
    assert max(s["levels"] for s in ref["subtrees"]) > max(cuts)


def test_oracle_pending_is_grouped_by_forwarding_batch():
    o = Oracle(SMALL)
    o.set_level_range(0, 1)
    o.add_file(synth(53, 1, 40_000), 10_000)
    p, b, xyz = o.pending()
    o.close()
    assert len(p) > 0
    assert (np.diff(b.astype(np.int64)) >= 0).all()   # recorded in batch order
    cs = 500.0   # level-1 cells (metadata.rs:91-93, 100-102)
    assert (np.floor(p["x"] / np.float32(cs)).astype(np.int32) == xyz[:, 0]).all()
