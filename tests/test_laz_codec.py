"""LAZ codec (point-cloud_amd/csrc/laz.cpp: the LASzip pointwise-chunked format
for point formats 0-5, the LASzip 3 layered-chunked format for 6-10) through
laz_tool: LAS -> LAZ -> LAS restores the point records byte for byte, for every
item combination, chunk sizes from 1 point up, scanner-channel switches,
extreme coordinate jumps and GPS time jumps beyond 32-bit differences.
Parity unpinned: no .laz fixture in the reference and no LASzip here, so this
pins the codec's own round trip; las.rs:23-46 decoding of the points is
checked through the CLI in tests/test_inputs_gpu.py."""
import os
import subprocess

import numpy as np
import pytest

from las_util import REC, survey_records, survey_records14, write_las_records

HERE = os.path.dirname(os.path.abspath(__file__))
TOOL = os.path.join(HERE, "..", "point-cloud_amd", "build", "laz_tool")


def _roundtrip(tmp_path, body, fmt, chunk):
    a, z, b = str(tmp_path / "a.las"), str(tmp_path / "a.laz"), str(tmp_path / "b.las")
    write_las_records(a, body, fmt, len(body), (0.01, 0.01, 0.001), (100.0, 200.0, 0.0), minor=4 if fmt >= 6 else 2)
    subprocess.run([TOOL, "compress", a, z, str(chunk)], check=True)
    subprocess.run([TOOL, "decompress", z, b], check=True)
    ra, rb = open(a, "rb").read(), open(b, "rb").read()
    assert len(rb) == len(ra)
    assert ra == rb
    return os.path.getsize(z) / os.path.getsize(a)


@pytest.mark.parametrize("fmt,extra", [(0, 0), (1, 0), (2, 0), (3, 0), (1, 3), (3, 5), (4, 0), (5, 0), (5, 2)])
def test_laz_roundtrip_formats(tmp_path, fmt, extra):
    body = survey_records(60_000, fmt, seed=fmt * 10 + extra, extra=extra)
    ratio = _roundtrip(tmp_path, body, fmt, 50_000)
    assert ratio < 0.6   # it compresses


@pytest.mark.parametrize("chunk", [1, 2, 7, 1000])
def test_laz_roundtrip_chunk_sizes(tmp_path, chunk):
    body = survey_records(5_000, 3, seed=chunk)
    _roundtrip(tmp_path, body, 3, chunk)


def test_laz_roundtrip_extreme_values(tmp_path):
    rng = np.random.default_rng(7)
    n = 4_000
    body = np.zeros((n, REC[1]), dtype=np.uint8)
    xyz = rng.integers(-2**31, 2**31, (n, 3), dtype=np.int64).astype("<i4")   # full-range jumps
    xyz[::5] = np.iinfo(np.int32).min
    xyz[1::7] = np.iinfo(np.int32).max
    body[:, 0:12] = xyz.view(np.uint8).reshape(n, 12)
    body[:, 12:20] = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    g = rng.normal(0, 1e12, n).astype("<f8")
    body[:, 20:28] = g.view(np.uint8).reshape(n, 8)
    _roundtrip(tmp_path, body, 1, 333)


@pytest.mark.parametrize("fmt,extra,channels", [(6, 0, 1), (6, 0, 4), (7, 0, 2), (8, 0, 4), (6, 3, 3), (8, 2, 4),
                                                (9, 0, 1), (9, 0, 3), (10, 0, 4), (10, 3, 2)])
def test_laz_layered_roundtrip_formats(tmp_path, fmt, extra, channels):
    """Point formats 6-8 (LASzip 3 layered chunks): POINT14 + RGB14 / RGBNIR14 +
    BYTE14, points hopping between scanner channels (model contexts)."""
    body = survey_records14(60_000, fmt, seed=fmt * 10 + extra + channels, extra=extra, channels=channels)
    ratio = _roundtrip(tmp_path, body, fmt, 50_000)
    assert ratio < 0.6


@pytest.mark.parametrize("chunk", [1, 2, 7, 1000])
def test_laz_layered_chunk_sizes(tmp_path, chunk):
    body = survey_records14(5_000, 8, seed=chunk, extra=1)
    _roundtrip(tmp_path, body, 8, chunk)


def test_laz_layered_constant_layers(tmp_path):
    """Fields constant over a chunk store empty layers (Z, flags, angle, ...)."""
    body = survey_records14(3_000, 7, seed=5, extra=2, channels=1)
    body[:, 8:12] = body[0, 8:12]       # z
    body[:, 15:22] = body[0, 15:22]     # flags, class, user, angle, point source
    body[:, 30:36] = body[0, 30:36]     # colour
    body[:, 36:] = body[0, 36:]         # extra bytes
    _roundtrip(tmp_path, body, 7, 1000)


def test_laz_layered_extreme_values(tmp_path):
    rng = np.random.default_rng(8)
    n = 4_000
    body = rng.integers(0, 256, (n, REC[6]), dtype=np.uint8)   # every field random, all channels
    xyz = rng.integers(-2**31, 2**31, (n, 3), dtype=np.int64).astype("<i4")
    xyz[::5] = np.iinfo(np.int32).min
    body[:, 0:12] = xyz.view(np.uint8).reshape(n, 12)
    g = rng.normal(0, 1e12, n).astype("<f8")
    body[:, 22:30] = g.view(np.uint8).reshape(n, 8)
    _roundtrip(tmp_path, body, 6, 333)
