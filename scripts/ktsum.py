"""Per-launch durations of the last build in a rocprofv3 kernel trace (launches > 50 us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(("pcc::k_l0_up0g(", "pcc::k_l0_up0_bbox(", "pcc::k_bbox_sample("))]
tot = 0.0
for r in rows[idx[-1]:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot += d
    if d > 0.05:
        print(f"{d:8.3f} ms  grid={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):>8} wg={r['Workgroup_Size_X']:>4}  {r['Kernel_Name'][:60]}")
print(f"sum {tot:.2f} ms")
