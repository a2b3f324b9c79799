"""Known-answer tests of the hex / cell arithmetic.

Both restatements the parity rests on — the C oracle (oracle/pcc_oracle.c) and
the numpy one (oracle/pyref.py) — are checked against answers derived WITHOUT
float32 hardware arithmetic:

  * literal cases derived by hand below (each with its derivation), covering
    exact hex-edge ties, z truncation around 0 (hex.rs:83 `as i32` truncates, so
    z-slab 0 is 2r thick), negative coordinates and cell boundaries
    (metadata.rs:100-102 floor), cell sizes and centres (metadata.rs:91-106);
  * an exact-rational restatement (fractions.Fraction, every operation rounded
    to nearest-even float32 explicitly, in the op order of hex.rs:67-85 and
    metadata.rs:91-106) on boundary-heavy generated cases.
"""
import ctypes as C
import math
import os
import sys
from fractions import Fraction as Q

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import pyref  # noqa: E402
from oracle_ctypes import lib  # noqa: E402

F = np.float32


class IVec3(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("z", C.c_int32)]


class Cfg(C.Structure):
    _fields_ = [("cell_point_overflow_limit", C.c_uint32), ("sub_grid_dimension", C.c_uint32),
                ("max_cell_size", C.c_float)]


def _c():
    L = lib()
    L.orc_hex_from_world.restype = IVec3
    L.orc_hex_from_world.argtypes = [C.c_float] * 4
    L.orc_cell_index.restype = IVec3
    L.orc_cell_index.argtypes = [C.c_float] * 4
    L.orc_cell_size.restype = C.c_float
    L.orc_cell_size.argtypes = [C.POINTER(Cfg), C.c_uint32]
    L.orc_cell_pos.argtypes = [IVec3, C.c_float, C.POINTER(C.c_float)]
    return L


def c_hex(p, r):
    v = _c().orc_hex_from_world(F(p[0]), F(p[1]), F(p[2]), F(r))
    return (v.x, v.y, v.z)


def c_cell_index(p, cs):
    v = _c().orc_cell_index(F(p[0]), F(p[1]), F(p[2]), F(cs))
    return (v.x, v.y, v.z)


# ------------------------------------------------------------ exact-rational float32
def rn32(v: Q) -> Q:
    """Round a rational to the nearest float32 (ties to even), subnormals included."""
    if v == 0:
        return Q(0)
    s = -1 if v < 0 else 1
    a = abs(v)
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Q(2) ** e > a:
        e -= 1
    e = max(e, -126)
    ulp = Q(2) ** (e - 23)
    qv = a / ulp
    n = math.floor(qv)
    rem = qv - n
    if rem > Q(1, 2) or (rem == Q(1, 2) and n % 2 == 1):
        n += 1
    return s * n * ulp


def q32(x) -> Q:
    return Q(float(F(x)))


S3 = rn32(Q("1.73205080757"))   # hex.rs:3 `1.73205080757f32`


def sat_i32(v: Q) -> int:   # Rust `f32 as i32` on an already-integral or truncated value
    t = math.trunc(v)
    return max(-2 ** 31, min(2 ** 31 - 1, t))


def exact_hex(p, r):
    """hex.rs:67-85 AxialIndex::from_world + to_offset (hex.rs:45-51), each f32
    operation as an exact rational rounded to float32."""
    r = q32(r)
    px, py, pz = (q32(v) for v in p)
    x = rn32(px / rn32(r * S3))
    y = rn32(py / rn32(-r * S3))
    t = rn32(rn32(S3 * y) + 1)
    t1 = Q(math.floor(rn32(t + x)))
    t2 = rn32(t - x)
    t3 = rn32(rn32(2 * x) + 1)
    q = sat_i32(Q(math.floor(rn32(rn32(t1 + t3) / 3))))
    rr = -sat_i32(Q(math.floor(rn32(rn32(t1 + t2) / 3))))
    h = sat_i32(rn32(pz / r))
    return (q + (rr - (rr & 1)) // 2, rr, h)


def exact_cell_index(p, cs):   # metadata.rs:100-102
    cs = q32(cs)
    return tuple(sat_i32(Q(math.floor(rn32(q32(v) / cs)))) for v in p)


def exact_cell_size(mcs, h):   # metadata.rs:91-93
    return rn32(q32(mcs) / (2 ** h))


def exact_cell_pos(idx, cs):   # metadata.rs:104-106
    cs = q32(cs)
    return tuple(rn32(rn32(Q(i) * cs) + rn32(cs / 2)) for i in idx)


# ------------------------------------------------------------ hand-derived cases
# Radius r = 0.5 (sub_cell_size 1 = cell size 96 at dimension 96): r * S3 = S3/2
# exactly (halving is exact), so with R = S3/2 every x = p.x / R below is exact.
R = float(S3 / 2)
HAND_HEX = [
    # origin: x = 0, y = -0, t = 1, t1 = 1, t2 = 1, t3 = 1 -> q = floor(2/3) = 0, r = -floor(2/3) = 0
    ((0.0, 0.0, 0.0), 0.5, (0, 0, 0)),
    # two hex widths along +x: x = 2, t1 = 3, t2 = -1, t3 = 5 -> q = floor(8/3) = 2, r = 0
    ((2 * R, 0.0, 0.0), 0.5, (2, 0, 0)),
    # exactly on the edge between hexes 0 and 1: x = 0.5, t1 = floor(1.5) = 1, t3 = 2 ->
    # q = floor(3/3) = 1: the tie goes to the +x hex
    ((R / 2, 0.0, 0.0), 0.5, (1, 0, 0)),
    # the mirrored edge: x = -0.5, t1 = floor(0.5) = 0, t3 = 0 -> q = 0: again the +x hex
    ((-R / 2, 0.0, 0.0), 0.5, (0, 0, 0)),
    # one ulp below the edge still lands in hex 1: x = 0.5 - 2^-25, 2x + 1 = 2 - 2^-24 is a
    # float32 midpoint and rounds to even (2.0), t1 = floor(RN(1.49999997)) = floor(1.5) = 1,
    # so q = floor(3/3) = 1
    ((float(np.nextafter(F(R / 2), F(0))), 0.0, 0.0), 0.5, (1, 0, 0)),
    # p.y = -R: y = 1, t = RN(S3 + 1) = 2.7320508, x = 0: t1 = 2, t2 = t, t3 = 1 ->
    # q = floor(3/3) = 1, r = -floor(RN(4.7320508/3)) = -1; offset x = 1 + (-1 - 1)/2 = 0:
    # on the shared edge of axial (1, -1) and (0, -1) the +x hex wins again
    ((0.0, -R, 0.0), 0.5, (0, -1, 0)),
    # z truncates toward zero (hex.rs:83): z / r = 0.98 -> 0, -0.98 -> 0 (slab 0 spans
    # (-r, r), twice as thick as the others), 1.0 -> 1, -1.0 -> -1, 2.4 -> 2, -2.4 -> -2
    ((0.0, 0.0, 0.49), 0.5, (0, 0, 0)),
    ((0.0, 0.0, -0.49), 0.5, (0, 0, 0)),
    ((0.0, 0.0, 0.5), 0.5, (0, 0, 1)),
    ((0.0, 0.0, -0.5), 0.5, (0, 0, -1)),
    ((0.0, 0.0, 1.2), 0.5, (0, 0, 2)),
    ((0.0, 0.0, -1.2), 0.5, (0, 0, -2)),
    ((0.0, 0.0, -0.0), 0.5, (0, 0, 0)),
]

HAND_CELL = [
    # metadata.rs:100-102 floor(p / 1000): negative side and the boundaries
    ((-0.001, 0.0, 999.99994), 1000.0, (-1, 0, 0)),
    ((-1000.0, 1000.0, -0.0), 1000.0, (-1, 1, 0)),           # floor(-1) = -1, floor(1) = 1, -0 -> 0
    ((-1000.0001, 1999.9999, 0.0), 1000.0, (-2, 1, 0)),
    # a 2^-7-sized cell at level 17 of the default config: 1000 / 2^17 = 0.00762939453125
    ((0.00762939453125, -0.00762939453125, 0.0038), 0.00762939453125, (1, -1, 0)),
]


@pytest.mark.parametrize("p,r,want", HAND_HEX)
def test_hex_hand_derived(p, r, want):
    assert exact_hex(p, r) == want
    assert c_hex(p, r) == want
    assert pyref.hex_from_world(p, r) == want


@pytest.mark.parametrize("p,cs,want", HAND_CELL)
def test_cell_index_hand_derived(p, cs, want):
    assert exact_cell_index(p, cs) == want
    assert c_cell_index(p, cs) == want
    assert pyref.cell_index(p, cs) == want


def test_cell_size_and_pos_hand_derived():
    cfg = Cfg(5000, 96, 1000.0)
    L = _c()
    for h, want in [(0, 1000.0), (1, 500.0), (3, 125.0), (10, 0.9765625), (20, 1000.0 / 2 ** 20)]:
        assert float(exact_cell_size(1000.0, h)) == want
        assert L.orc_cell_size(C.byref(cfg), h) == want
        assert float(pyref.cell_size({"max_cell_size": 1000.0}, h)) == want
    # cell_pos = idx * cs + cs / 2: (-1, 0, 2) at cs 1000 -> (-500, 500, 2500)
    out = (C.c_float * 3)()
    L.orc_cell_pos(IVec3(-1, 0, 2), 1000.0, out)
    assert list(out) == [-500.0, 500.0, 2500.0]
    assert [float(v) for v in exact_cell_pos((-1, 0, 2), 1000.0)] == [-500.0, 500.0, 2500.0]
    assert [float(v) for v in pyref.cell_pos((-1, 0, 2), 1000.0)] == [-500.0, 500.0, 2500.0]
    # sub_cell_size(1000) = RN(1000 / 96) = RN(125 / 12); hex radius = half of it (exact)
    sub = rn32(Q(1000) / 96)
    assert float(sub) == float(F(1000.0) / F(96.0)) == 10.416666984558105


def _boundary_cases(rng, n):
    """Points on and next to hex edges, slot centres, z-slab and cell boundaries."""
    out = []
    for r in (0.5, float(F(1000.0) / F(96.0) / F(2.0)), float(F(125.0) / F(96.0) / F(2.0)), 0.001):
        r32 = F(r)
        for _ in range(n):
            q, rr, hz = (int(v) for v in rng.integers(-60, 60, 3))
            X, Y, Z = pyref.hex_to_world((q, rr, hz), r32)
            kind = rng.integers(0, 4)
            if kind == 0:      # the centre itself
                p = (X, Y, Z)
            elif kind == 1:    # a hex vertex / edge point: centre + r * unit direction
                ang = rng.integers(0, 12) * math.pi / 6
                p = (F(X + F(r32 * F(math.cos(ang)))), F(Y + F(r32 * F(math.sin(ang)))), Z)
            elif kind == 2:    # ulp neighbours of the edge midpoint along x
                p = (np.nextafter(F(X + F(r32 * F(0.8660254))), F(rng.choice([-1e9, 1e9]))), Y, Z)
            else:              # z-slab boundaries around 0 and negative coordinates
                p = (F(X), F(Y), F(F(hz) * r32) * F(rng.choice([1.0, -1.0])) + F(rng.choice([0.0, 1e-6, -1e-6])))
            out.append((tuple(float(v) for v in p), float(r32)))
    return out


def test_hex_exact_rational_restatement_boundaries():
    rng = np.random.default_rng(2024)
    for p, r in _boundary_cases(rng, 150):
        want = exact_hex(p, r)
        assert c_hex(p, r) == want, (p, r)
        assert pyref.hex_from_world(p, r) == want, (p, r)


def test_cell_index_exact_rational_restatement_boundaries():
    rng = np.random.default_rng(7)
    for h in (0, 1, 2, 5, 13):
        cs = float(exact_cell_size(1000.0, h))
        for _ in range(200):
            i = [int(v) for v in rng.integers(-40, 40, 3)]
            eps = [float(rng.choice([0.0, 1.0, -1.0])) for _ in range(3)]
            p = tuple(float(np.nextafter(F(F(i[a]) * F(cs)), F(eps[a] * 1e9))) if eps[a] else float(F(i[a]) * F(cs))
                      for a in range(3))
            want = exact_cell_index(p, cs)
            assert c_cell_index(p, cs) == want, (p, cs)
            assert pyref.cell_index(p, cs) == want, (p, cs)
