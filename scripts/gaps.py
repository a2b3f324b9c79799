#!/usr/bin/env python3
"""Diagnostic: idle gaps between kernels of the last build in a rocprofv3 kernel trace."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(("pcc::k_l0_up0g(", "pcc::k_l0_up0_bbox("))]
b = rows[idx[-1]:]
t0, prev, tot, big = int(b[0]["Start_Timestamp"]), None, 0.0, []
for r in b:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev is not None:
        g = (s - prev) / 1e3
        tot += max(g, 0.0)
        if g > float(sys.argv[2] if len(sys.argv) > 2 else 60):
            big.append((round(g, 1), r["Kernel_Name"][:45]))
    prev = max(prev or 0, e)
print("gaps us", round(tot, 1), "span ms", round((prev - t0) / 1e6, 3))
for x in big:
    print(x)
