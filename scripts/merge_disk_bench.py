"""Config 5 from disk (VERDICT r1 "next" item 4): the
1B-point config-4 cloud is converted and written as cell files, then a new
converter opens that directory (pcc_open: metadata.json + every cell file,
read_cloud + prior_from_cells + upload of the seeds) and merges the +100M
config-5 points.  Reports the on-disk load apart from the merge build and the
write of the touched cells.  The cell files were just written, so the load
reads them from the page cache (this user cannot drop it): a file-system read
rate, not a cold-disk one.
Usage: python scripts/merge_disk_bench.py [N_PRIOR] [N_NEW]"""
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))
import pcconv  # noqa: E402

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
n1 = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
d = tempfile.mkdtemp(prefix="pcc_md_", dir=os.environ.get("PCC_WB_DIR", "/tmp"))
res = {"prior_points": n0, "new_points": n1}
try:
    t0 = time.perf_counter()
    c = pcconv.Converter(d)
    c.add_synthetic(4, 0, n0)
    st = c.build()
    c.write()
    c.close()
    t1 = time.perf_counter()
    files = sum(len(fs) for _, _, fs in os.walk(d))
    nbytes = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(d) for f in fs)
    res["prior"] = {"cells": st["cells"], "files": files, "bytes": nbytes, "build_write_s": round(t1 - t0, 2)}
    print("prior written", res["prior"], file=sys.stderr, flush=True)
    for rep in range(2):
        t2 = time.perf_counter()
        m = pcconv.Converter(d)          # loads the existing cloud (merge mode)
        t3 = time.perf_counter()
        m.add_synthetic(5, 0, n1)
        t4 = time.perf_counter()
        sm = m.build()
        t5 = time.perf_counter()
        r = {"load_ms": round((t3 - t2) * 1e3, 1), "load_GBps": round(nbytes / (t3 - t2) / 1e9, 2),
             "new_points_ms": round((t4 - t3) * 1e3, 1), "merge_build_ms": round((t5 - t4) * 1e3, 1),
             "arrivals": sm["arrivals"], "number_of_points": sm["number_of_points"]}
        m.close()
        res[f"run{rep}"] = r
        print(r, file=sys.stderr, flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
print(json.dumps(res), flush=True)
