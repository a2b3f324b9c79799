"""Helpers for GPU parity tests: run the HIP build and the C oracle on the same input."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import canon  # noqa: E402
import pcconv  # noqa: E402
from oracle_ctypes import Oracle  # noqa: E402


def run_gpu(out_dir, files, cfg=None, batch=10_000, synth=None, empty_batches=()):
    """files: list of numpy POINT_DTYPE arrays (one per input file).
    synth: list of (seed, kind, n) synthetic files generated on the device instead."""
    conv = pcconv.Converter(out_dir, batch_size=batch, config=cfg)
    try:
        if synth:
            for seed, kind, n in synth:
                conv.add_synthetic(seed, kind, n)
        for i, f in enumerate(files):
            if i in empty_batches:
                conv.add_empty_batches(f)
            else:
                conv.add_points(f)
        st = conv.build()
        conv.write()
    finally:
        conv.close()
    return st


def run_oracle(out_dir, files, cfg=None, batch=10_000):
    o = Oracle(cfg)
    for f in files:
        o.add_file(f, batch)
    err = o.error
    if not err:
        o.write(out_dir)
    arr = o.arrivals
    o.close()
    return err, arr


def gpu_digest(conv) -> dict:
    """Canonical per-subtree digests of a built converter's cells, walked in
    memory through pcc_visit_cells (oracle/digest.c does the hashing)."""
    from oracle_ctypes import Digest
    d = Digest()
    try:
        conv.visit_cells(lambda view: d.add_view(view) or 0)
        return d.result()
    finally:
        d.close()


def compare_dirs(a, b, fast=True):
    if fast:
        ca, ma = canon.read_dir_fast(a)
        cb, mb = canon.read_dir_fast(b)
        return canon.diff_fast(ca, cb), ma, mb
    ca, ma = canon.read_dir(a)
    cb, mb = canon.read_dir(b)
    return canon.diff(ca, cb), ma, mb
