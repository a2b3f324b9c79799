"""Diagnostic: the first build of a second converter opened in the same process
(after the first one closed), with host or device input."""
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))
import pcconv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
mode = sys.argv[2] if len(sys.argv) > 2 else "synth"
host = None
if mode == "host":
    import torch
    dev = torch.empty((n, 4), dtype=torch.int32, device="cuda")
    pcconv.synth_device(dev.data_ptr(), 0, n, 4, 0, -1000.0, 2000.0, 0)
    torch.cuda.synchronize()
    host = dev.cpu().numpy().view(pcconv.POINT_DTYPE).reshape(-1)
    del dev
    torch.cuda.empty_cache()
for rep in range(3):
    c = pcconv.Converter(tempfile.mkdtemp(prefix="pcc_2c_"))
    t0 = time.perf_counter()
    if host is not None:
        c.add_points(host)
    else:
        c.add_synthetic(4, 0, n)
    t1 = time.perf_counter()
    st = c.build()
    t2 = time.perf_counter()
    c.build()
    t3 = time.perf_counter()
    c.close()
    print(mode, rep, "input %.1f ms, first build %.1f ms, rebuild %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3),
          {k: v for k, v in st.items() if "ms" in k}, flush=True)
