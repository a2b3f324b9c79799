"""The oracle on inputs with NaN / +-inf coordinates (tests/nonfinite_input.py):
it converts them without error, the metadata bounding box follows f32::min/max
(NaN skipped, infinities kept, written as null like serde_json), and the cloud
holds cells with saturated indices and NaN grid points."""
import json
import os

import numpy as np

from gpu_util import run_oracle
from nonfinite_input import NONFINITE_CFG, nonfinite_files


def test_oracle_converts_nonfinite_points(tmp_path):
    files = nonfinite_files()
    out = str(tmp_path / "o")
    err, arrivals = run_oracle(out, files, cfg=NONFINITE_CFG, batch=5000)
    assert err == 0
    meta = json.load(open(os.path.join(out, "metadata.json")))
    allp = np.concatenate(files)
    for a, k in enumerate("xyz"):
        col = allp[k].astype(np.float64)
        if np.isinf(col).any():   # an infinite coordinate makes that bound infinite -> null
            assert meta["bounding_box"]["min"][a] is None or meta["bounding_box"]["max"][a] is None
    assert meta["number_of_points"] == len(allp)
    names = [n for h in os.listdir(out) if h.startswith("h_") for n in os.listdir(os.path.join(out, h))]
    assert any("2147483647" in n or "-2147483648" in n for n in names), "cells with saturated indices"
    assert int(meta["hierarchies"]) >= 3
