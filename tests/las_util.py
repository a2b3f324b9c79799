"""LAS writing helpers shared by the LAS/LAZ tests (the reference ships no LAS
or LAZ fixture: the tests write their own files)."""
import struct

import numpy as np

REC = {0: 20, 1: 28, 2: 26, 3: 34, 4: 57, 5: 63, 6: 30, 7: 36, 8: 38, 9: 59, 10: 67}
COLOR_OFF = {0: None, 1: None, 2: 20, 3: 28, 4: None, 5: 28, 6: None, 7: 30, 8: 30, 9: None, 10: 30}
GPS_OFF = {0: None, 1: 20, 2: None, 3: 20, 4: 20, 5: 20, 6: 22, 7: 22, 8: 22, 9: 22, 10: 22}
WAVE_OFF = {4: 28, 5: 34, 9: 30, 10: 38}   # the 29-byte wave packet record


def write_las_records(path, body, fmt, n, scale, offset, minor=2):
    """Header (no VLRs) + raw point records `body` (n x record bytes)."""
    rec = body.shape[1] if n else REC[fmt]
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
    with open(path, "wb") as f:
        f.write(bytes(h))
        f.write(np.ascontiguousarray(body).tobytes())


def write_las(path, X, Y, Z, scale, offset, fmt=3, rgb=None, minor=2):
    """Minimal uncompressed LAS writer (header + point records, no VLRs)."""
    n = len(X)
    rec = REC[fmt]
    body = np.zeros((n, rec), dtype=np.uint8)
    xyz = np.stack([X, Y, Z], axis=1).astype("<i4")
    body[:, 0:12] = xyz.view(np.uint8).reshape(n, 12)
    if COLOR_OFF[fmt] is not None:
        body[:, COLOR_OFF[fmt]:COLOR_OFF[fmt] + 6] = np.asarray(rgb, dtype="<u2").view(np.uint8).reshape(n, 6)
    write_las_records(path, body, fmt, n, scale, offset, minor)


def add_wave_packets(body, off, rng):
    """Wave packet records (LAS formats 4 / 5 / 9 / 10) at byte `off`: descriptor
    index, waveform data offset (mostly the previous offset + the previous
    packet size, sometimes repeated, sometimes a 32-bit jump, a few 64-bit
    jumps), packet size, return point location and x(t), y(t), z(t) floats."""
    n = body.shape[0]
    idx = rng.choice([1, 1, 1, 2, 3], n).astype(np.uint8)
    size = rng.choice([120, 240, 240, 480], n).astype(np.uint64)
    step = size.copy()
    r = rng.random(n)
    step[r < 0.1] = 0
    jump = (r >= 0.1) & (r < 0.15)
    step[jump] = rng.integers(1, 2**31, int(jump.sum())).astype(np.uint64)
    off64 = (np.uint64(60_000) + np.concatenate([[0], np.cumsum(step[:-1])])).astype(np.uint64)
    big = rng.random(n) < 0.003
    off64[big] += np.uint64(1 << 40)
    body[:, off] = idx
    body[:, off + 1:off + 9] = off64.astype("<u8").view(np.uint8).reshape(n, 8)
    body[:, off + 9:off + 13] = size.astype("<u4").view(np.uint8).reshape(n, 4)
    f = np.stack([rng.normal(1000, 50, n), rng.normal(0, 1e-4, n), rng.normal(0, 1e-4, n),
                  -np.abs(rng.normal(0.5, 0.01, n))], 1).astype("<f4")
    f[::97] = f[::97] * 3.0
    body[:, off + 13:off + 29] = f.view(np.uint8).reshape(n, 16)


def survey_records(n, fmt, seed, extra=0):
    """Point records shaped like an airborne survey (what LAZ is made for):
    coordinates along scan lines, multiple returns, increasing GPS time with
    repeats, correlated colour, flags, plus `extra` bytes per record."""
    rng = np.random.default_rng(seed)
    rec = REC[fmt] + extra
    body = np.zeros((n, rec), dtype=np.uint8)
    t = np.arange(n)
    x = (np.cumsum(rng.integers(-40, 120, n)) + 1_000_000).astype("<i4")
    y = (np.cumsum(rng.integers(-3, 4, n)) * 7 + (t // 500) * 900 - 2_000_000).astype("<i4")
    z = (50_000 + np.cumsum(rng.integers(-30, 31, n)) + rng.integers(-200, 200, n) * (rng.random(n) < 0.05)).astype("<i4")
    body[:, 0:12] = np.stack([x, y, z], 1).view(np.uint8).reshape(n, 12)
    inten = (rng.integers(0, 700, n) * (rng.random(n) < 0.9)).astype("<u2")
    body[:, 12:14] = inten.view(np.uint8).reshape(n, 2)
    nret = rng.integers(1, 5, n)
    ret = np.minimum(rng.integers(1, 5, n), nret)
    sdir = (t // 300) % 2
    edge = (t % 300 == 299).astype(np.int64)
    body[:, 14] = (ret | (nret << 3) | (sdir << 6) | (edge << 7)).astype(np.uint8)
    body[:, 15] = rng.choice([1, 2, 2, 2, 5, 6], n).astype(np.uint8)
    body[:, 16] = ((t // 40) % 60 - 30).astype(np.int8).view(np.uint8)
    body[:, 17] = (rng.random(n) < 0.02).astype(np.uint8) * rng.integers(0, 255, n).astype(np.uint8)
    psid = np.full(n, 17, dtype="<u2")
    psid[n // 2:] = 18
    body[:, 18:20] = psid.view(np.uint8).reshape(n, 2)
    if GPS_OFF.get(fmt) is not None:
        g = 250_000.0 + np.repeat(np.cumsum(rng.random((n + 1) // 2) * 1e-4), 2)[:n]
        g[n // 3] += 1e9   # a jump beyond 32-bit differences
        body[:, 20:28] = g.astype("<f8").view(np.uint8).reshape(n, 8)
    if fmt in WAVE_OFF:
        add_wave_packets(body, WAVE_OFF[fmt], rng)
    if COLOR_OFF.get(fmt) is not None:
        base = np.cumsum(rng.integers(-3, 4, n)) % 65536
        rgb = np.stack([base, (base + rng.integers(0, 300, n)) % 65536, (base * 3) % 65536], 1).astype("<u2")
        grey = rng.random(n) < 0.3
        rgb[grey, 1] = rgb[grey, 0]
        rgb[grey, 2] = rgb[grey, 0]
        co = COLOR_OFF[fmt]
        body[:, co:co + 6] = rgb.view(np.uint8).reshape(n, 6)
    if extra:
        body[:, REC[fmt]:] = (np.arange(n)[:, None] * np.arange(1, extra + 1)[None, :] % 251).astype(np.uint8)
    return body


def survey_records14(n, fmt, seed, extra=0, channels=4):
    """LAS 1.4 point records (formats 6-8) shaped like a multi-channel survey:
    scan lines whose points alternate between `channels` scanner channels in
    runs, up to 15 returns, classification flags, scan angle in 0.006 degree
    steps, increasing GPS time with repeats and one large jump, colour and NIR
    (formats 7 / 8), plus `extra` bytes."""
    rng = np.random.default_rng(seed)
    rec = REC[fmt] + extra
    body = np.zeros((n, rec), dtype=np.uint8)
    t = np.arange(n)
    ch = ((t // rng.integers(1, 40)) % channels) if channels > 1 else np.zeros(n, np.int64)
    x = (np.cumsum(rng.integers(-40, 120, n)) + 1_000_000 + ch * 5000).astype("<i4")
    y = (np.cumsum(rng.integers(-3, 4, n)) * 7 + (t // 500) * 900 - 2_000_000).astype("<i4")
    z = (50_000 + np.cumsum(rng.integers(-30, 31, n)) + rng.integers(-200, 200, n) * (rng.random(n) < 0.05)).astype("<i4")
    body[:, 0:12] = np.stack([x, y, z], 1).view(np.uint8).reshape(n, 12)
    inten = (rng.integers(0, 700, n) * (rng.random(n) < 0.9)).astype("<u2")
    body[:, 12:14] = inten.view(np.uint8).reshape(n, 2)
    nret = rng.choice([1, 1, 2, 3, 4, 7, 15], n)
    ret = np.minimum(rng.integers(1, 16, n), nret)
    body[:, 14] = (ret | (nret << 4)).astype(np.uint8)
    cflags = (rng.random(n) < 0.05) * rng.integers(0, 16, n)
    sdir = (t // 300) % 2
    edge = (t % 300 == 299).astype(np.int64)
    body[:, 15] = (cflags | (ch << 4) | (sdir << 6) | (edge << 7)).astype(np.uint8)
    body[:, 16] = rng.choice([1, 2, 2, 2, 5, 6, 40, 200], n).astype(np.uint8)
    body[:, 17] = (rng.random(n) < 0.02).astype(np.uint8) * rng.integers(0, 255, n).astype(np.uint8)
    ang = (((t // 40) % 600) - 300) * 10
    ang[rng.random(n) < 0.01] = -30000
    body[:, 18:20] = ang.astype("<i2").view(np.uint8).reshape(n, 2)
    psid = np.full(n, 17, dtype="<u2")
    psid[n // 2:] = 18
    body[:, 20:22] = psid.view(np.uint8).reshape(n, 2)
    g = 250_000.0 + np.repeat(np.cumsum(rng.random((n + 1) // 2) * 1e-4), 2)[:n]
    g[n // 3:] += 1e9   # a jump beyond 32-bit differences
    body[:, 22:30] = g.astype("<f8").view(np.uint8).reshape(n, 8)
    if fmt in WAVE_OFF:
        add_wave_packets(body, WAVE_OFF[fmt], rng)
    if fmt in (7, 8, 10):
        base = np.cumsum(rng.integers(-3, 4, n)) % 65536
        rgb = np.stack([base, (base + rng.integers(0, 300, n)) % 65536, (base * 3) % 65536], 1).astype("<u2")
        grey = rng.random(n) < 0.3
        rgb[grey, 1] = rgb[grey, 0]
        rgb[grey, 2] = rgb[grey, 0]
        body[:, 30:36] = rgb.view(np.uint8).reshape(n, 6)
    if fmt in (8, 10):
        nir = ((np.cumsum(rng.integers(-2, 3, n)) + 30000) % 65536).astype("<u2")
        body[:, 36:38] = nir.view(np.uint8).reshape(n, 2)
    if extra:
        body[:, REC[fmt]:] = (np.arange(n)[:, None] * np.arange(1, extra + 1)[None, :] % 251).astype(np.uint8)
    return body
