"""GPU parity on inputs with NaN / +-inf coordinates (tests/nonfinite_input.py)
against the oracle: same cells, grid points, overflow lists and metadata (the
bounding box follows f32::min/max, written as null where non-finite).  The
reference's semantics: bounding-volume/src/lib.rs:23-31 (NaN skipped),
metadata.rs:100-102 and hex.rs:67-85 (`as i32` saturates, NaN -> 0),
cell.rs:77-80 (a NaN distance is never less)."""

import numpy as np
import pytest

from gpu_util import compare_dirs, run_gpu, run_oracle
from nonfinite_input import NONFINITE_CFG, nonfinite_files

pytestmark = pytest.mark.gpu

CASES = {
    # small slabs (k_slab_small / k_slab_wave / k_bucket)
    "nan_small": (NONFINITE_CFG, dict(kinds="nan"), 5000),
    # one root cell of 32 layers: slabs of ~12k arrivals (the dense k_slab)
    "nan_dense": ({"sub_grid_dimension": 32, "cell_point_overflow_limit": 2000, "max_cell_size": 1000.0},
                  dict(kinds="nan", n=400_000), 50_000),
    "mixed_small": (NONFINITE_CFG, dict(kinds="mixed"), 5000),
    "mixed_dense": ({"sub_grid_dimension": 32, "cell_point_overflow_limit": 2000, "max_cell_size": 1000.0},
                    dict(kinds="mixed", n=400_000), 50_000),
}


@pytest.mark.parametrize("case", list(CASES))
def test_nonfinite_parity(tmp_path, case):
    cfg, kw, batch = CASES[case]
    files = nonfinite_files(**kw)
    go, oo = str(tmp_path / "g"), str(tmp_path / "o")
    err, _ = run_oracle(oo, files, cfg=cfg, batch=batch)
    assert err == 0
    run_gpu(go, files, cfg=cfg, batch=batch)
    diffs, mg, mo = compare_dirs(go, oo)
    assert not diffs, diffs[:10]
    assert mg == mo


# Merges (lib.rs:86-101 + converter.rs:187-207): the existing cloud holds NaN
# points (its bounding box stays finite, so its metadata.json reads back), the
# new files NaN and +-inf points.  The GPU merge must write what the oracle
# writes for all files in one run (the equivalence of tests/test_merge_oracle.py).
MERGE_CASES = {
    "small": (NONFINITE_CFG, 5000, 120_000),
    # dim 32, one root cell: dense slabs of the existing cloud's levels >= 1 (k_slab merge mode)
    "dense": ({"sub_grid_dimension": 32, "cell_point_overflow_limit": 2000, "max_cell_size": 1000.0}, 50_000, 400_000),
}


@pytest.mark.parametrize("prior_by", ["oracle", "gpu"])
@pytest.mark.parametrize("case", list(MERGE_CASES))
def test_nonfinite_merge_parity(tmp_path, case, prior_by):
    cfg, batch, n = MERGE_CASES[case]
    old = nonfinite_files(seed=11, n=n, kinds="nan")
    new = nonfinite_files(seed=12, n=n // 2, kinds="mixed")
    for f in old:   # the existing cloud's box is finite on every axis
        assert all(np.isfinite(f[a]).any() for a in ("x", "y", "z"))
    go, oo = str(tmp_path / "g"), str(tmp_path / "o")
    if prior_by == "oracle":
        err, _ = run_oracle(go, old, cfg=cfg, batch=batch)
        assert err == 0
    else:
        run_gpu(go, old, cfg=cfg, batch=batch)
    st = run_gpu(go, new, cfg=None, batch=batch)   # the config comes from the existing metadata.json
    err, _ = run_oracle(oo, old + new, cfg=cfg, batch=batch)
    assert err == 0
    diffs, mg, mo = compare_dirs(go, oo)
    assert not diffs, diffs[:10]
    assert mg == mo
    assert st["number_of_points"] == sum(len(f) for f in old + new)


def test_nonfinite_merge_of_finite_points_into_nan_cloud(tmp_path):
    """Finite new points into a cloud that holds NaN points: the
    existing NaN grid points keep their slots (nothing is less than NaN)."""
    cfg, batch = NONFINITE_CFG, 5000
    old = nonfinite_files(seed=13, n=80_000, kinds="nan")
    new = [f[np.isfinite(f["x"]) & np.isfinite(f["y"]) & np.isfinite(f["z"])] for f in
           nonfinite_files(seed=14, n=60_000, kinds="nan")]
    go, oo = str(tmp_path / "g"), str(tmp_path / "o")
    run_gpu(go, old, cfg=cfg, batch=batch)
    run_gpu(go, new, cfg=None, batch=batch)
    err, _ = run_oracle(oo, old + new, cfg=cfg, batch=batch)
    assert err == 0
    diffs, mg, mo = compare_dirs(go, oo)
    assert not diffs, diffs[:10]
    assert mg == mo
