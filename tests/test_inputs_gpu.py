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

from gpu_util import compare_dirs, gpu_digest  # noqa: E402
from oracle_ctypes import POINT_DTYPE, Oracle, synth  # noqa: E402
from las_util import survey_records, survey_records14, write_las, write_las_records  # noqa: E402

pytestmark = pytest.mark.gpu


def _exe():
    import pcconv
    return os.path.join(os.path.dirname(pcconv.LIB_PATH), "point_converter")


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


def _write_ply_props(path, cols, enc="binary_little_endian", count=None, drop_bytes=0):
    """PLY with arbitrary vertex properties: cols = [(name, ply type, numpy array)].
    `count` overrides the declared vertex count; `drop_bytes` cuts the file short."""
    n = len(cols[0][2])
    np_t = {"double": "f8", "float": "f4", "uchar": "u1", "ushort": "u2", "int": "i4"}
    hdr = "ply\nformat %s 1.0\nelement vertex %d\n" % (enc, n if count is None else count)
    hdr += "".join("property %s %s\n" % (t, nm) for nm, t, _ in cols) + "end_header\n"
    with open(path, "wb") as f:
        f.write(hdr.encode())
        if enc == "ascii":
            for i in range(n):
                f.write((" ".join(repr(c[2][i].item()) for c in cols) + "\n").encode())
        else:
            bo = ">" if enc == "binary_big_endian" else "<"
            dt = np.dtype([(nm, bo + np_t[t]) for nm, t, _ in cols])
            rec = np.zeros(n, dtype=dt)
            for nm, _, a in cols:
                rec[nm] = a
            data = rec.tobytes()
            f.write(data[:len(data) - drop_bytes] if drop_bytes else data)


def _ply_expect(cols):
    """point.rs:61-130 restated: x/y/z Float or Double (`as f32`); red/green/blue/alpha
    UChar, or Float as `(v / 255.0) as u8` (f32 division, saturating cast)."""
    n = len(cols[0][2])
    p = np.zeros(n, dtype=POINT_DTYPE)
    p["rgba"][:, 3] = 255
    for nm, t, a in cols:
        if nm in ("x", "y", "z") and t in ("float", "double"):
            p[nm] = np.asarray(a).astype(np.float32)
        ch = {"red": 0, "green": 1, "blue": 2, "alpha": 3}.get(nm)
        if ch is not None:
            if t == "uchar":
                p["rgba"][:, ch] = a
            elif t == "float":
                v = np.asarray(a, dtype=np.float32) / np.float32(255.0)
                p["rgba"][:, ch] = np.nan_to_num(np.clip(v, 0, 255), nan=0.0).astype(np.uint8)
    return p


def _cli(files, out):
    args = [_exe(), "-o", out]
    for f in files:
        args += ["-f", f]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stderr


def _oracle_dir(path, files_pts, empty_batches=None):
    o = Oracle()
    for i, pts in enumerate(files_pts):
        if empty_batches and i in empty_batches:
            for _ in range(empty_batches[i]):
                o.add_batch(pts[:0])
        elif pts is not None:
            o.add_file(pts)
    o.write(path)
    o.close()


def test_ply_big_endian_double_coords_float_colours():
    """PLY binary big-endian, double coordinates, float colours, an ignored extra
    property (point.rs:61-130; ply.rs:54-61)."""
    rng = np.random.default_rng(8)
    n = 33_333
    cols = [("x", "double", rng.uniform(-900, 900, n)), ("y", "double", rng.uniform(-900, 900, n)),
            ("intensity", "ushort", rng.integers(0, 65535, n)), ("z", "double", rng.uniform(-900, 900, n)),
            ("red", "float", rng.uniform(0, 70_000, n).astype(np.float32)),
            ("green", "float", rng.uniform(-10, 300, n).astype(np.float32)),
            ("blue", "uchar", rng.integers(0, 256, n)), ("alpha", "float", np.full(n, 255.0 * 100, np.float32))]
    with tempfile.TemporaryDirectory() as td:
        a = os.path.join(td, "be.ply")
        _write_ply_props(a, cols, enc="binary_big_endian")
        out, ref = os.path.join(td, "out"), os.path.join(td, "ref")
        _cli([a], out)
        _oracle_dir(ref, [_ply_expect(cols)])
        d, mg, mo = compare_dirs(out, ref, fast=False)
        assert d == [] and mg == mo


def test_truncated_inputs_keep_complete_batches():
    """lib.rs:31-52: a get_batch error is logged and ends its file; the batches read
    before stay, the failing batch is lost, the next files are still converted.
    PLY (binary LE, truncated mid-batch), ASCII PLY (short of lines: its complete
    batches still count, ply.rs:43-51) and LAS (truncated point data)."""
    rng = np.random.default_rng(9)
    pts = synth(61, 0, 80_000)
    cols = [("x", "float", pts["x"]), ("y", "float", pts["y"]), ("z", "float", pts["z"]),
            ("red", "uchar", pts["rgba"][:, 0]), ("green", "uchar", pts["rgba"][:, 1]),
            ("blue", "uchar", pts["rgba"][:, 2]), ("alpha", "uchar", pts["rgba"][:, 3])]
    with tempfile.TemporaryDirectory() as td:
        f1 = os.path.join(td, "a.ply")   # 35 000 declared, 23 456 records present -> 2 batches
        _write_ply_props(f1, [(nm, t, a[:35_000]) for nm, t, a in cols], drop_bytes=16 * (35_000 - 23_456) + 5)
        f2 = os.path.join(td, "b.ply")   # ASCII, 25 000 declared, 12 345 lines -> 1 empty batch
        _write_ply_props(f2, [(nm, t, a[:12_345]) for nm, t, a in cols], enc="ascii", count=25_000)
        n3 = 27_000                      # LAS, 27 000 declared, 26 001 present -> 2 batches
        X = rng.integers(-100_000, 100_000, n3)
        Y = rng.integers(-100_000, 100_000, n3)
        Z = rng.integers(-100_000, 100_000, n3)
        rgb = rng.integers(0, 65536, (n3, 3))
        f3 = os.path.join(td, "c.las")
        write_las(f3, X, Y, Z, (0.01, 0.01, 0.01), (0.0, 0.0, 0.0), fmt=3, rgb=rgb)
        with open(f3, "r+b") as f:
            f.truncate(227 + 34 * 26_001 + 7)
        f4 = os.path.join(td, "d.ply")   # a complete file after the broken ones
        _write_ply_props(f4, [(nm, t, a[40_000:]) for nm, t, a in cols])
        out, ref = os.path.join(td, "out"), os.path.join(td, "ref")
        log = _cli([f1, f2, f3, f4], out)
        assert log.count("ERROR") == 3, log
        las = decode(X, Y, Z, (0.01, 0.01, 0.01), (0.0, 0.0, 0.0), rgb)
        _oracle_dir(ref, [pts[:20_000], pts[:0], las[:20_000], pts[40_000:]], empty_batches={1: 1})
        d, mg, mo = compare_dirs(out, ref, fast=False)
        assert d == [] and mg == mo


def test_file_in_pieces_equals_one_call(tmp_path):
    """pcc_begin_file / pcc_append_points / pcc_end_file (the pinned-ring
    upload the CLI uses) == one pcc_add_points call per file; pieces larger
    than one 4M-point staging buffer, a 1-point piece, keep < total (a reader
    error keeps the complete batches) and a cancelled file (no batch)."""
    import pcconv
    a, b = synth(91, 0, 9_000_001), synth(92, 1, 123_457)
    ref = pcconv.Converter(str(tmp_path / "ref"))
    ref.add_points(a)
    ref.add_points(b[:120_000])
    ref.build()
    dref = gpu_digest(ref)
    ref.close()
    c = pcconv.Converter(str(tmp_path / "pieces"))
    c.add_file_pieces([a[:5_000_000], a[5_000_000:5_000_001], a[5_000_001:]])
    lib = pcconv.lib()
    import ctypes as C
    assert lib.pcc_begin_file(c._h, 10) == 0
    assert lib.pcc_append_points(c._h, C.c_void_p(b.ctypes.data), 5) == 0
    assert lib.pcc_cancel_file(c._h) == 0
    c.add_file_pieces([b[:60_000], b[60_000:]], keep=120_000)
    c.build()
    assert gpu_digest(c) == dref
    c.close()


def test_file_in_pieces_beyond_its_expected_size():
    """A streamed file that outgrows the size announced to pcc_begin_file: the
    device input grows while the file is open and keeps the points already
    pushed (and their level-0 tile counts)."""
    import ctypes as C
    import pcconv
    a, b = synth(93, 0, 300_001), synth(94, 1, 6_000_007)
    ref = pcconv.Converter(tempfile.mkdtemp(prefix="pcc_ref_"))
    ref.add_points(a)
    ref.add_points(b)
    ref.build()
    dref = gpu_digest(ref)
    ref.close()
    c = pcconv.Converter(tempfile.mkdtemp(prefix="pcc_grow_"))
    c.add_points(a)
    lib = pcconv.lib()
    assert lib.pcc_begin_file(c._h, 1000) == 0
    for o in range(0, len(b), 1_500_000):
        p = np.ascontiguousarray(b[o:o + 1_500_000])
        assert lib.pcc_append_points(c._h, C.c_void_p(p.ctypes.data), len(p)) == 0
    assert lib.pcc_end_file(c._h, len(b)) == 0
    c.build()
    assert gpu_digest(c) == dref
    c.close()


def test_ply_vertex_not_first_element():
    """ply.rs:36-73 reads `vertex` records straight after the header, whatever
    element the header declares first: the bytes of a leading `extra` element
    (12-byte records: three finite floats) are read as vertex records (x, y, z
    float; red, green, blue, alpha uchar), and the last vertex records are never
    reached.  Parity unpinned: no reference fixture, the expected points come
    from reinterpreting the file's bytes here."""
    rng = np.random.default_rng(9)
    n, k = 40_000, 3_000
    extra = rng.uniform(-800, 800, (k, 3)).astype("<f4")
    vert = np.zeros(n, dtype=POINT_DTYPE)
    for a in "xyz":
        vert[a] = rng.uniform(-900, 900, n).astype(np.float32)
    vert["rgba"] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    hdr = ("ply\nformat binary_little_endian 1.0\nelement extra %d\nproperty float a\nproperty float b\n"
           "property float c\nelement vertex %d\nproperty float x\nproperty float y\nproperty float z\n"
           "property uchar red\nproperty uchar green\nproperty uchar blue\nproperty uchar alpha\n"
           "element face 0\nproperty list uchar int vertex_indices\nend_header\n") % (k, n)
    payload = extra.tobytes() + vert.tobytes()
    expect = np.frombuffer(payload[:16 * n], dtype=POINT_DTYPE).copy()
    with tempfile.TemporaryDirectory() as td:
        a = os.path.join(td, "x.ply")
        with open(a, "wb") as f:
            f.write(hdr.encode())
            f.write(payload)
        out, ref = os.path.join(td, "out"), os.path.join(td, "ref")
        _cli([a], out)
        _oracle_dir(ref, [expect])
        d, mg, mo = compare_dirs(out, ref, fast=False)
        assert d == [] and mg == mo


@pytest.mark.parametrize("formats", [(1, 3), (6, 8), (7,), (4, 5), (9, 10)])
def test_laz_cli_equals_las(tmp_path, formats):
    """LAZ input (las.rs:14-46 through laz [dep]): a .laz made by laz_tool from a
    .las converts to exactly the .las's cloud, for point formats 1 and 3 (GPS
    time, colour; pointwise chunks), 6, 7, 8 (LAS 1.4, layered chunks, colour
    from 7 / 8) and the wave-packet formats 4, 5 (pointwise) and 9, 10
    (layered), two files in one run.  Parity unpinned: the .laz files come
    from this repository's own encoder (no reference fixture, no LASzip here)."""
    tool = os.path.join(os.path.dirname(_exe()), "laz_tool")
    files_las, files_laz = [], []
    sizes = {1: 45_000, 3: 120_000, 6: 45_000, 8: 120_000, 7: 165_000,   # 165k points per run
             4: 45_000, 5: 120_000, 9: 45_000, 10: 120_000}
    for k, fmt in enumerate(formats):
        n = sizes[fmt]
        body = (survey_records(n, fmt, seed=40 + fmt) if fmt < 6 else survey_records14(n, fmt, seed=40 + fmt))
        a = str(tmp_path / f"f{k}.las")
        z = str(tmp_path / f"f{k}.laz")
        write_las_records(a, body, fmt, len(body), (0.001, 0.001, 0.0005), (-900.0, 1900.0, -20.0),
                          minor=4 if fmt >= 6 else 2)
        subprocess.run([tool, "compress", a, z, "50000"], check=True)
        files_las.append(a)
        files_laz.append(z)
    out_las, out_laz = str(tmp_path / "out_las"), str(tmp_path / "out_laz")
    _cli(files_las, out_las)
    log = _cli(files_laz, out_laz)
    assert "not supported" not in log
    d, ma, mb = compare_dirs(out_las, out_laz, fast=False)
    assert d == [] and ma == mb
    assert ma["number_of_points"] == 165_000


@pytest.mark.parametrize("seed", range(8))
def test_las_cli_random_transforms(seed):
    """Randomised LAS inputs through the CLI: point formats 0-10, LAS 1.2 / 1.4,
    scales 10^-4..10 with odd mantissas, offsets up to 10^6 with fractions,
    integer ranges up to the whole i32, 1-3 files (converter/las.rs:23-46:
    scale * X + offset in f64, then as f32), against the oracle on the numpy
    decoding."""
    from las_util import COLOR_OFF, REC
    rng = np.random.default_rng(900 + seed)
    with tempfile.TemporaryDirectory() as td:
        files, decoded = [], []
        for k in range(int(rng.integers(1, 4))):
            fmt = int(rng.choice(sorted(REC)))
            minor = 4 if fmt >= 6 else int(rng.choice([2, 4]))
            n = int(rng.integers(1, 60_000))
            scale = tuple(float(np.float64(rng.choice([1, 3, 7, 125, 333])) * 10.0 ** int(rng.integers(-6, 0)))
                          for _ in range(3))
            offset = tuple(float(rng.choice([0.0, rng.uniform(-1e6, 1e6), float(rng.integers(-500_000, 500_000)) + 0.5]))
                           for _ in range(3))
            span = int(rng.choice([1000, 100_000, 10_000_000, 2**31 - 1]))
            lim = [min(span, int(1000.0 / s)) + 1 for s in scale]   # (about +-1000 units around the offset)
            X, Y, Z = (rng.integers(-m, m, n) for m in lim)
            rgb = rng.integers(0, 65536, (n, 3)) if COLOR_OFF[fmt] is not None else None
            path = os.path.join(td, f"f{k}.las")
            write_las(path, X, Y, Z, scale, offset, fmt=fmt, rgb=rgb, minor=minor)
            files.append(path)
            decoded.append(decode(X, Y, Z, scale, offset, rgb))
        out = os.path.join(td, "out")
        _cli(files, out)
        ref = os.path.join(td, "ref")
        _oracle_dir(ref, decoded)
        d, mg, mo = compare_dirs(out, ref, fast=True)
        assert d == [] and mg == mo, d


@pytest.mark.parametrize("seed", range(8))
def test_ply_cli_random_layouts(seed):
    """Randomised binary PLY vertex layouts through the CLI: x/y/z as float or
    double, colours as uchar, float or absent, extra properties of other types
    interleaved in any order, little or big endian, 1-2 files
    (ply.rs:36-73, point.rs:61-130), against the oracle on the numpy decoding."""
    rng = np.random.default_rng(700 + seed)
    with tempfile.TemporaryDirectory() as td:
        files, expect = [], []
        for k in range(int(rng.integers(1, 3))):
            n = int(rng.integers(1, 50_000))
            lo, ext = float(rng.uniform(-3000, 1000)), float(rng.uniform(10, 4000))
            cols = [(a, str(rng.choice(["float", "double"])), rng.uniform(lo, lo + ext, n)) for a in "xyz"]
            for ch in ("red", "green", "blue", "alpha"):
                t = str(rng.choice(["uchar", "float", "none"]))
                if t == "uchar":
                    cols.append((ch, t, rng.integers(0, 256, n)))
                elif t == "float":
                    cols.append((ch, t, rng.uniform(-100, 70_000, n).astype(np.float32)))
            for e in range(int(rng.integers(0, 4))):
                t = str(rng.choice(["ushort", "int", "uchar", "double"]))
                cols.append((f"extra{e}", t, rng.integers(0, 200, n)))
            order = rng.permutation(len(cols))
            cols = [cols[i] for i in order]
            path = os.path.join(td, f"f{k}.ply")
            _write_ply_props(path, cols, enc=str(rng.choice(["binary_little_endian", "binary_big_endian"])))
            files.append(path)
            expect.append(_ply_expect(cols))
        out, ref = os.path.join(td, "out"), os.path.join(td, "ref")
        _cli(files, out)
        _oracle_dir(ref, expect)
        d, mg, mo = compare_dirs(out, ref, fast=True)
        assert d == [] and mg == mo, d
