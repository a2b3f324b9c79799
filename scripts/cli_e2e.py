#!/usr/bin/env python3
"""CLI end-to-end timing (GPU box): N uniform points (seed 4) written as a
binary-LE PLY (x, y, z float; red, green, blue, alpha uchar), then
`point_converter -o OUT -f FILE` timed as a whole process, with PCC_VERBOSE
stage lines.  Usage: python scripts/cli_e2e.py N [tag]"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
from oracle_ctypes import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
tag = sys.argv[2] if len(sys.argv) > 2 else "cli"
d = tempfile.mkdtemp(prefix="pcc_cli_", dir="/tmp")
ply = os.path.join(d, "in.ply")
with open(ply, "wb") as f:
    f.write(("ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
             "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nproperty uchar alpha\n"
             "end_header\n" % n).encode())
    for a in range(0, n, 10_000_000):
        f.write(synth(4, 0, min(10_000_000, n - a), first=a).tobytes())
exe = os.path.join(ROOT, "point-cloud_amd", "build", "point_converter")
env = dict(os.environ, PCC_VERBOSE="1")
t0 = time.perf_counter()
r = subprocess.run([exe, "-o", os.path.join(d, "out"), "-f", ply], capture_output=True, text=True, env=env)
dt = time.perf_counter() - t0
lines = [ln for ln in (r.stdout + r.stderr).splitlines() if "[pcc]" in ln or "Finished" in ln or "ERROR" in ln]
rep = {"points": n, "file_bytes": os.path.getsize(ply), "rc": r.returncode, "wall_s": dt, "lines": lines[-40:]}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rep, open(os.path.join(ROOT, "gpurun_out", f"{tag}.json"), "w"), indent=1)
print(json.dumps({k: rep[k] for k in ("points", "rc", "wall_s")}))
subprocess.run(["rm", "-rf", d])
