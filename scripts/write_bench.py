"""Output path timing (SURVEY.md §8d reports it apart from the build): one
synthetic conversion, then pcc_write (per-level compacted D2H overlapped with
cell-file writes) with 1 writer thread and with the default pool.
Usage: python scripts/write_bench.py N [kind]"""
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))
import pcconv  # noqa: E402

n = int(sys.argv[1])
kind = int(sys.argv[2]) if len(sys.argv) > 2 else 0
res = {"points": n, "kind": kind}
for threads in ("1", ""):
    d = tempfile.mkdtemp(prefix="pcc_wb_", dir=os.environ.get("PCC_WB_DIR", "/tmp"))
    try:
        if threads:
            os.environ["PCC_WRITE_THREADS"] = threads
        else:
            os.environ.pop("PCC_WRITE_THREADS", None)
        c = pcconv.Converter(d)
        c.add_synthetic(4, kind, n)
        t0 = time.perf_counter()
        st = c.build()
        t1 = time.perf_counter()
        c.write()
        t2 = time.perf_counter()
        c.close()
        files = sum(len(fs) for _, _, fs in os.walk(d))
        nbytes = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(d) for f in fs)
        res["threads=" + (threads or "default")] = {"build_ms": round((t1 - t0) * 1e3, 1),
                                                    "write_ms": round((t2 - t1) * 1e3, 1), "files": files,
                                                    "bytes": nbytes, "GBps": round(nbytes / (t2 - t1) / 1e9, 2)}
    finally:
        shutil.rmtree(d, ignore_errors=True)
print(json.dumps(res), flush=True)
