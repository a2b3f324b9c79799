"""GPU parity on inputs with NaN / +-inf coordinates (tests/nonfinite_input.py)
against the oracle: same cells, grid points, overflow lists and metadata (the
bounding box follows f32::min/max, written as null where non-finite).  The
reference's semantics: bounding-volume/src/lib.rs:23-31 (NaN skipped),
metadata.rs:100-102 and hex.rs:67-85 (`as i32` saturates, NaN -> 0),
cell.rs:77-80 (a NaN distance is never less)."""
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
