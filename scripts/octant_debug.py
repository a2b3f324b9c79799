#!/usr/bin/env python3
"""Debug: build one level-0 cell of uniform points several ways (synthetic on
device, device pointer input, repeated builds, fold on/off)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))
import torch  # noqa: E402
import pcconv  # noqa: E402


def run(tag, n, how, reps=2):
    c = pcconv.Converter("/tmp/pcc_octdbg", batch_size=10_000)
    res = {"tag": tag, "n": n, "how": how}
    try:
        if how == "synth":
            c.add_synthetic(4, 0, n, 0.0, 1000.0)
        else:
            pts = torch.empty((n, 4), dtype=torch.int32, device="cuda")
            pcconv.synth_device(pts.data_ptr(), 0, n, 4, 0, 0.0, 1000.0, 0)
            torch.cuda.synchronize()
            c.add_points_device(pts.data_ptr(), n)
        for r in range(reps):
            t0 = time.perf_counter()
            try:
                s = c.build()
                res[f"rep{r}"] = {"ms": round((time.perf_counter() - t0) * 1e3, 2), "levels": s["levels"],
                                  "cells": s["cells"], "arrivals": s["arrivals"]}
            except pcconv.PccError as e:
                res[f"rep{r}"] = {"error": str(e)}
    finally:
        c.close()
    print(json.dumps(res), flush=True)


for n in (2_000_000, 20_000_000, 125_000_000):
    for how in ("synth", "device"):
        for fold in ("1", "0"):
            if fold == "0":
                os.environ["PCC_NO_FOLD"] = "1"
            else:
                os.environ.pop("PCC_NO_FOLD", None)
            run(f"fold{fold}", n, how)
