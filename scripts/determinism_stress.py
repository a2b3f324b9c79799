"""Determinism stress: every randomised case (tests/fuzz_cases.py) built REPS
times on the GPU in one process; the canonical per-subtree digests
(pcc_visit_cells -> oracle/digest.c, the checker) must be identical across the
repeats.  Usage: determinism_stress.py REPS [nf]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import tempfile  # noqa: E402

from gpu_util import gpu_digest  # noqa: E402  (puts the package on the path)
import pcconv  # noqa: E402
from fuzz_cases import mid_case  # noqa: E402

reps = int(sys.argv[1])
nonfinite = len(sys.argv) > 2 and sys.argv[2] == "nf"
bad = 0
for seed in range(48 if not nonfinite else 24):
    files, cfg, batch, kind = mid_case(seed, nonfinite=nonfinite)
    ref = None
    for rep in range(reps):
        with tempfile.TemporaryDirectory(dir="/dev/shm") as d:
            conv = pcconv.Converter(d, batch_size=batch, config=cfg)
            for f in files:
                conv.add_points(f)
            conv.build()
            dg = gpu_digest(conv)
            conv.close()
        if ref is None:
            ref = dg
        elif dg != ref:
            bad += 1
            diff = [k for k in set(ref) | set(dg) if ref.get(k) != dg.get(k)]
            print("seed", seed, kind, cfg, batch, "rep", rep, "differs in", diff[:4], flush=True)
    if seed % 12 == 0:
        print("seed", seed, "done", flush=True)
print("nondeterministic builds:", bad)
