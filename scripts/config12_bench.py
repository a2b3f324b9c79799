#!/usr/bin/env python3
"""Configs 1 and 2 of BASELINE.md, measured once (GPU box; not the bench line).

config 1: 100k uniform points (seed 1) as a binary-LE PLY through the CLI
          (point-cloud_amd/build/point_converter -o OUT -f FILE): end-to-end wall
          time of the process (PLY decode, device init, build, files), plus the
          build alone through the C-ABI;
config 2: 10M uniform points (seed 2) generated in HBM, build time (5 steps).
CPU baseline of both: the sequential C restatement, full run, in memory (mode B),
1 thread.  Writes gpurun_out/config12.json.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
from oracle_ctypes import Oracle, synth  # noqa: E402


def write_ply(path, pts):
    hdr = ("ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
           "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nproperty uchar alpha\n"
           "end_header\n" % len(pts)).encode()
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(np.ascontiguousarray(pts).tobytes())


def cpu_mode_b(pts):
    o = Oracle()
    t0 = time.perf_counter()
    o.add_file(pts, 10_000)
    dt = time.perf_counter() - t0
    o.close()
    return len(pts) / dt


def main():
    import torch
    torch.cuda.init()
    import pcconv
    out = {}
    p1 = synth(1, 0, 100_000)
    with tempfile.TemporaryDirectory() as d:
        ply = os.path.join(d, "c1.ply")
        write_ply(ply, p1)
        exe = os.path.join(ROOT, "point-cloud_amd", "build", "point_converter")
        t0 = time.perf_counter()
        subprocess.run([exe, "-o", os.path.join(d, "out"), "-f", ply], check=True, capture_output=True)
        cli = time.perf_counter() - t0
        c = pcconv.Converter(os.path.join(d, "out2"))
        c.add_points(p1)
        c.build()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            c.build()
            ts.append(time.perf_counter() - t0)
        c.close()
    out["config1"] = {"cli_end_to_end_s": cli, "build_ms": 1e3 * min(ts), "gpu_build_points_per_s": 1e5 / min(ts),
                      "cpu_mode_b_points_per_s": cpu_mode_b(p1)}
    with tempfile.TemporaryDirectory() as d:
        c = pcconv.Converter(d)
        c.add_synthetic(2, 0, 10_000_000)
        st = c.build()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            st = c.build()
            ts.append(time.perf_counter() - t0)
        c.close()
    out["config2"] = {"build_ms": 1e3 * min(ts), "gpu_points_per_s": 1e7 / min(ts), "levels": st["levels"],
                      "cells": st["cells"], "arrivals_W": st["arrivals"],
                      "cpu_mode_b_points_per_s": cpu_mode_b(synth(2, 0, 10_000_000))}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "config12.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
