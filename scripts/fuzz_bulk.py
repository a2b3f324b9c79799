"""Bulk randomised comparison beyond the committed sweep: seeds [A, B) of the
sweep's generator (tests/fuzz_cases.py) as plain builds, builds with NaN/+-inf,
and merges, each against the oracle; with "sharded", each seed over 2-8 thread
ranks on cuda:0 instead.  Prints each mismatch or error and a summary.
Usage: fuzz_bulk.py A B [sharded]"""
import os
import shutil
import sys
import tempfile
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
from gpu_util import compare_dirs, run_gpu, run_oracle  # noqa: E402
import pcconv  # noqa: E402
from fuzz_cases import halves, mid_case  # noqa: E402

a, b = int(sys.argv[1]), int(sys.argv[2])
stats = {"ok": 0, "bad": 0, "both_refused": 0}


def one(tag, seed, files, cfg, batch, prior=None):
    tg, to = tempfile.mkdtemp(dir="/dev/shm"), tempfile.mkdtemp(dir="/dev/shm")
    try:
        if prior is not None:
            if run_oracle(tg, prior, cfg=cfg, batch=batch)[0]:
                stats["both_refused"] += 1
                return
        err, _ = run_oracle(to, (prior or []) + files, cfg=cfg, batch=batch)
        try:
            run_gpu(tg, files, cfg=None if prior is not None else cfg, batch=batch)
            gerr = None
        except pcconv.PccError as e:
            gerr = str(e)
        if err and gerr:
            stats["both_refused"] += 1
            return
        if err or gerr:
            stats["bad"] += 1
            print(tag, seed, cfg, batch, "oracle err", err, "gpu", gerr, flush=True)
            return
        d, mg, mo = compare_dirs(tg, to, fast=True)
        if d or mg != mo:
            stats["bad"] += 1
            print(tag, seed, cfg, batch, d[:2], flush=True)
        else:
            stats["ok"] += 1
    except Exception:  # noqa: BLE001
        stats["bad"] += 1
        print(tag, seed, traceback.format_exc()[-600:], flush=True)
    finally:
        shutil.rmtree(tg, ignore_errors=True)
        shutil.rmtree(to, ignore_errors=True)


def sharded(seed):
    import threading
    import numpy as np
    import torch
    from pcconv.dist import HipShardOps, ThreadComm, ThreadGroup, key_range, shard_build
    from shard_np import as_tensor
    import canon
    files, cfg, batch, _ = mid_case(seed, nonfinite=seed % 4 == 0)
    world = [2, 3, 4, 5, 8][seed % 5]
    fp = [len(f) for f in files]
    allp = np.concatenate(files)
    out, to = tempfile.mkdtemp(dir="/dev/shm"), tempfile.mkdtemp(dir="/dev/shm")
    dev = torch.device("cuda", 0)
    grp = ThreadGroup(world)
    res, errs = [None] * world, []

    def worker(r):
        try:
            torch.cuda.set_device(dev)
            lo, hi = key_range(len(allp), r, world)
            ops = HipShardOps(0, out_dir=out, batch_size=batch, config=cfg)
            ops.landing_rounds = [0, 2, 3, 5][seed % 4]
            res[r] = shard_build(ThreadComm(grp, r, dev), ops, as_tensor(allp[lo:hi]).to(dev), lo, fp, write=True)
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    try:
        err, _ = run_oracle(to, files, cfg=cfg, batch=batch)
        th = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
        [t.start() for t in th]
        [t.join() for t in th]
        if err and errs:
            stats["both_refused"] += 1
        elif err or errs:
            stats["bad"] += 1
            print("sharded", seed, cfg, batch, world, "oracle", err, "gpu", errs[:1], flush=True)
        else:
            ca, ma = canon.read_dir_fast(to)
            cb, mb = canon.read_dir_fast(out)
            d = canon.diff_fast(ca, cb)
            if d or ma["number_of_points"] != mb["number_of_points"] or ma["hierarchies"] != mb["hierarchies"]:
                stats["bad"] += 1
                print("sharded", seed, cfg, batch, world, d[:2], flush=True)
            else:
                stats["ok"] += 1
    finally:
        shutil.rmtree(out, ignore_errors=True)
        shutil.rmtree(to, ignore_errors=True)


for seed in range(a, b):
    if len(sys.argv) > 3 and sys.argv[3] == "sharded":
        sharded(seed)
        if seed % 25 == 0:
            print("at", seed, stats, flush=True)
        continue
    files, cfg, batch, _ = mid_case(seed)
    one("plain", seed, files, cfg, batch)
    if seed % 2 == 0:
        files, cfg, batch, _ = mid_case(seed, nonfinite=True)
        one("nonfinite", seed, files, cfg, batch)
    if seed % 3 == 0:
        files, cfg, batch, _ = mid_case(seed)
        first, second = halves(files)
        one("merge", seed, second, cfg, batch, prior=first)
    if seed % 50 == 0:
        print("at", seed, stats, flush=True)
print("summary", stats)
