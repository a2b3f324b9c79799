"""Input readers through the CLI (lib.rs:62-84 dispatch by extension) on the GPU.

* LAS (converter/las.rs:23-46 over las 0.8.4 [dep]): coordinates are
  `scale * X + offset` in f64 then `as f32`, colour channels are u16 `as u8`
  (low byte), alpha 255, formats without colour give black.  The expected
  points are decoded here independently with numpy and run through the oracle.
  No LAS fixture ships with the reference: the files are written by this test.
* metadata.json of another cloud (converter/own.rs): its points in the fixed
  enumeration format.h documents (h order, sorted file names, grid then Some
  lists in file order), re-decoded here from the cell files.
"""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from gpu_util import compare_dirs  # noqa: E402
from oracle_ctypes import POINT_DTYPE, Oracle, synth  # noqa: E402

pytestmark = pytest.mark.gpu


def _exe():
    import pcconv
    return os.path.join(os.path.dirname(pcconv.LIB_PATH), "point_converter")


def write_las(path, X, Y, Z, scale, offset, fmt=3, rgb=None, minor=2):
    """Minimal uncompressed LAS writer (header + point records, no VLRs)."""
    n = len(X)
    color_off = {0: None, 1: None, 2: 20, 3: 28, 6: None, 7: 30, 8: 30}[fmt]
    rec = {0: 20, 1: 28, 2: 26, 3: 34, 6: 30, 7: 36, 8: 38}[fmt]
    hsize = 375 if minor >= 4 else 227
    h = bytearray(hsize)
    h[0:4] = b"LASF"
    h[24] = 1
    h[25] = minor
    struct.pack_into("<H", h, 94, hsize)
    struct.pack_into("<I", h, 96, hsize)
    struct.pack_into("<I", h, 100, 0)
    h[104] = fmt
    struct.pack_into("<H", h, 105, rec)
    struct.pack_into("<I", h, 107, n if (minor < 4 and n < 2**32) else 0)
    struct.pack_into("<3d", h, 131, *scale)
    struct.pack_into("<3d", h, 155, *offset)
    if minor >= 4:
        struct.pack_into("<Q", h, 247, n)
    body = np.zeros((n, rec), dtype=np.uint8)
    xyz = np.stack([X, Y, Z], axis=1).astype("<i4")
    body[:, 0:12] = xyz.view(np.uint8).reshape(n, 12)
    if color_off is not None:
        body[:, color_off:color_off + 6] = np.asarray(rgb, dtype="<u2").view(np.uint8).reshape(n, 6)
    with open(path, "wb") as f:
        f.write(bytes(h))
        f.write(body.tobytes())


def decode(X, Y, Z, scale, offset, rgb=None):
    """las Transform::direct + las.rs:34-41, restated with numpy."""
    p = np.zeros(len(X), dtype=POINT_DTYPE)
    p["x"] = (np.float64(scale[0]) * X.astype(np.float64) + np.float64(offset[0])).astype(np.float32)
    p["y"] = (np.float64(scale[1]) * Y.astype(np.float64) + np.float64(offset[1])).astype(np.float32)
    p["z"] = (np.float64(scale[2]) * Z.astype(np.float64) + np.float64(offset[2])).astype(np.float32)
    if rgb is not None:
        p["rgba"][:, :3] = (np.asarray(rgb) & 0xFF).astype(np.uint8)
    p["rgba"][:, 3] = 255
    return p


def test_las_cli_formats_and_colour_truncation():
    rng = np.random.default_rng(5)
    with tempfile.TemporaryDirectory() as td:
        files, decoded = [], []
        for k, (fmt, minor, n) in enumerate([(3, 2, 70_000), (1, 2, 15_000), (7, 4, 40_000)]):
            scale = (0.01, 0.02, 0.005)
            offset = (-500.25, 100.5, -3.0)
            X = rng.integers(-100_000, 100_000, n)
            Y = rng.integers(-60_000, 30_000, n)
            Z = rng.integers(-200_000, 200_000, n)
            rgb = rng.integers(0, 65536, (n, 3)) if fmt in (3, 7) else None
            path = os.path.join(td, f"f{k}.las")
            write_las(path, X, Y, Z, scale, offset, fmt=fmt, rgb=rgb, minor=minor)
            files.append(path)
            decoded.append(decode(X, Y, Z, scale, offset, rgb))
        out = os.path.join(td, "out")
        args = [_exe(), "-o", out]
        for f in files:
            args += ["-f", f]
        r = subprocess.run(args, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        ref = os.path.join(td, "ref")
        o = Oracle()
        for d in decoded:
            o.add_file(d)
        o.write(ref)
        o.close()
        d, mg, mo = compare_dirs(out, ref, fast=False)
        assert d == [] and mg == mo


def _enumerate_cloud(cloud_dir, hierarchies):
    """Points of a converted cloud in format.h's fixed enumeration."""
    chunks = []
    for h in range(hierarchies):
        hd = os.path.join(cloud_dir, f"h_{h}")
        if not os.path.isdir(hd):
            continue
        for name in sorted(os.listdir(hd)):
            with open(os.path.join(hd, name), "rb") as f:
                data = f.read()
            number = struct.unpack_from("<I", data, 20)[0]
            off = 48
            chunks.append(np.frombuffer(data, dtype=POINT_DTYPE, count=number, offset=off))
            off += 16 * number
            nb = data[off]
            off += 1
            for _ in range(nb):
                n = struct.unpack_from("<I", data, off + 12)[0]
                off += 16
                if n:
                    chunks.append(np.frombuffer(data, dtype=POINT_DTYPE, count=n, offset=off))
                    off += 16 * n
    return np.concatenate(chunks) if chunks else np.zeros(0, dtype=POINT_DTYPE)


def test_metadata_json_as_input():
    import json
    pts = synth(41, 1, 300_000)
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "src")
        o = Oracle(dict(cell_point_overflow_limit=200, sub_grid_dimension=8, max_cell_size=1000.0))
        o.add_file(pts)
        o.write(src)
        o.close()
        with open(os.path.join(src, "metadata.json")) as f:
            hier = json.load(f)["hierarchies"]
        out = os.path.join(td, "out")
        r = subprocess.run([_exe(), "-o", out, "-f", os.path.join(src, "metadata.json")],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        ref = os.path.join(td, "ref")
        o = Oracle()
        o.add_file(_enumerate_cloud(src, hier))
        o.write(ref)
        o.close()
        d, mg, mo = compare_dirs(out, ref, fast=True)
        assert d == [] and mg == mo
