"""Level ranges of one build (pcc_set_level_range / pcc_export_pending): the
hierarchy split at a level boundary and built in pieces — levels 0..k-1 in one
converter, the exported level-k arrivals (with their parent buckets' spill
batches) as the roots of another — must give exactly the cells of one whole
build.  This is what lets several ranks share a heavy level-0 cell (SURVEY §8e,
§8f-4): a level-h cell's content depends only on the points forwarded to it and
their event batches (converter.rs:114-139, cell.rs:70-153).
"""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import pcconv  # noqa: E402
from gpu_util import gpu_digest  # noqa: E402
from oracle_ctypes import Digest, Oracle, synth  # noqa: E402

DEV = torch.device("cuda", 0)
SMALL = {"sub_grid_dimension": 16, "cell_point_overflow_limit": 100, "max_cell_size": 1000.0}


def piece(tmp, name, cfg, files, rng, roots=None, arrivals=None):
    """One converter over a level range; returns (converter, exported pending or None)."""
    c = pcconv.Converter(str(tmp / name), batch_size=10_000, device=0, config=cfg)
    c.set_level_range(*rng)
    if roots is None:
        for f in files:
            c.add_points(f)
    else:
        pts, keys = arrivals
        c.declare_files([len(f) for f in files])
        c.set_root_spill_batches(*roots)
        c.set_keyed_points_device(pts.data_ptr(), keys.data_ptr(), pts.shape[0])
    st = c.build()
    nc, npt = c.pending_cells()
    exp = None
    if rng[1]:
        P = torch.empty((npt, 4), dtype=torch.int32, device=DEV)
        K = torch.empty(npt, dtype=torch.int32, device=DEV)
        xyz, sb, cn = c.export_pending(P.data_ptr(), K.data_ptr())
        assert len(xyz) == nc and int(cn.sum()) == npt
        exp = ((xyz, sb), (P, K))
    return c, st, exp


@pytest.mark.gpu
@pytest.mark.parametrize("case,cfg,cuts", [
    ("clustered_small_grid", SMALL, [1]),
    ("clustered_small_grid", SMALL, [2]),
    ("clustered_small_grid", SMALL, [1, 3]),
    ("uniform_small_grid", SMALL, [1]),
    ("gauss_default", None, [1]),
])
def test_level_pieces_equal_whole_build(tmp_path, case, cfg, cuts):
    if case == "clustered_small_grid":
        files = [synth(41, 1, 250_000), synth(42, 1, 37_777)]
    elif case == "uniform_small_grid":
        files = [synth(43, 0, 200_000)]
    else:   # Gaussian mixture (config-3 generator), default config: level-0 spills
        files = [synth(44, 2, 3_000_000)]
    whole = pcconv.Converter(str(tmp_path / "whole"), batch_size=10_000, device=0, config=cfg)
    for f in files:
        whole.add_points(f)
    wst = whole.build()
    ref = gpu_digest(whole)
    whole.close()

    d = Digest()
    bounds = [0] + cuts
    exp, arrivals, convs = None, 0, []
    for i, h0 in enumerate(bounds):
        m = (bounds[i + 1] - h0) if i + 1 < len(bounds) else 0
        if exp is None and i > 0:
            break   # nothing reached this level
        c, st, exp = piece(tmp_path, f"p{i}", cfg, files, (h0, m), None if i == 0 else exp[0],
                           None if i == 0 else exp[1])
        convs.append(c)
        arrivals += st["arrivals"]
        c.visit_cells(lambda v: d.add_view(v) or 0)
        if exp is not None and exp[1][0].shape[0] == 0:
            exp = None
    got = d.result()
    d.close()
    for c in convs:
        c.close()
    assert got == ref
    assert arrivals == wst["arrivals"]
    assert max(s["levels"] for s in ref["subtrees"]) > max(cuts)   # the cut is inside the hierarchy


@pytest.mark.gpu
def test_level_pieces_match_oracle(tmp_path):
    files = [synth(45, 1, 120_000)]
    o = Oracle(SMALL)
    for f in files:
        o.add_file(f, 10_000)
    d0 = Digest()
    d0.add_oracle(o)
    ref = d0.result()
    o.close()
    d0.close()
    a, _, exp = piece(tmp_path, "a", SMALL, files, (0, 1))
    b, _, _ = piece(tmp_path, "b", SMALL, files, (1, 0), exp[0], exp[1])
    d = Digest()
    for c in (a, b):
        c.visit_cells(lambda v: d.add_view(v) or 0)
        c.close()
    assert d.result() == ref
    d.close()


@pytest.mark.gpu
def test_level_range_guards(tmp_path):
    c = pcconv.Converter(str(tmp_path / "g"), batch_size=10_000, device=0)
    c.set_level_range(1, 0)
    c.declare_files([10])
    c.set_root_spill_batches(np.array([[99, 99, 99]], np.int32), np.zeros(1, np.uint32))
    p = torch.from_numpy(synth(46, 0, 10).view(np.int32).reshape(-1, 4).copy()).to(DEV)
    k = torch.arange(10, dtype=torch.int32, device=DEV)
    c.set_keyed_points_device(p.data_ptr(), k.data_ptr(), 10)
    with pytest.raises(pcconv.PccError):   # a root cell without a spill batch: refused on the device
        c.build()
    c.close()
