"""C-ABI surface checks that need no GPU: libpcconv.so loads, exports every
function include/pcconv.h declares, and host-only entry points behave.  No
compute call is made here (those are the -m gpu tests)."""
import ctypes as C
import errno
import os
import re
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))

import pcconv  # noqa: E402

HEADER = os.path.join(ROOT, "include", "pcconv.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pcc_\w+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("pcc_open", "pcc_add_points", "pcc_build", "pcc_finish", "pcc_last_error",
                 "pcc_shard_route", "pcc_add_keyed_points_device"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = pcconv.lib()
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(pcconv.EXPORTS) == declared()
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.abspath(pcconv.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    dyn = set(re.findall(r" T (pcc_\w+)$", out, flags=re.M))
    assert set(declared()) <= dyn


def test_abi_version_and_defaults():
    lib = pcconv.lib()
    assert lib.pcc_abi_version() == 1
    o = pcconv.default_options()
    assert (o.batch_size, o.device, o.cell_point_overflow_limit, o.sub_grid_dimension, o.max_cell_size) == \
        (10_000, 0, 5000, 96, 1000.0)   # lib.rs:32, metadata.rs:80-88
    assert C.sizeof(pcconv.Options) == 24


def test_shard_grid_from_bbox_host_only():
    g = pcconv.shard_grid_from_bbox([-999.5, -0.25, 0.0], [999.9, 0.0, 2500.0])
    assert list(g.lo) == [-1, -1, 0] and list(g.dims) == [2, 2, 3] and g.cell_size == 1000.0
    assert g.ncells == 12
    with pytest.raises(pcconv.PccError) as e:
        pcconv.shard_grid_from_bbox([0, 0, 0], [1e9, 1e9, 1e9])
    assert e.value.code == -errno.EFBIG
    with pytest.raises(pcconv.PccError):
        pcconv.shard_grid_from_bbox([1, 0, 0], [0, 0, 0])


def test_null_arguments_rejected_without_device_work():
    lib = pcconv.lib()
    assert lib.pcc_add_points(None, None, 0) == -errno.EINVAL
    assert lib.pcc_build(None) == -errno.EINVAL
    assert b"null" in lib.pcc_last_error()


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="host has a GPU")
def test_open_fails_loudly_without_gpu(tmp_path):
    """No CPU fallback: without a HIP device the converter refuses to open."""
    with pytest.raises(pcconv.PccError) as e:
        pcconv.Converter(str(tmp_path / "o"))
    assert e.value.code == -errno.ENODEV
    assert "no CPU fallback" in str(e.value)


def test_cell_view_layout_matches_checker():
    """pcc_cell_view as the Python mirror declares it == the digest checker's copy."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_ctypes import lib as olib
    assert C.sizeof(pcconv.CellView) == olib().dg_view_size() == 256
