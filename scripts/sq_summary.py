#!/usr/bin/env python3
"""Per-dispatch SQ counter summary of rocprofv3 --pmc passes (scripts/r3_sq.sh).
Usage: sq_summary.py OUTDIR [kernel-substring ...] -> JSON on stdout.
Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* and
SQ_BUSY_CYCLES count quad-cycles (x4 = cycles); SQ_INSTS_* count instructions."""
import csv
import glob
import json
import sys
from collections import OrderedDict


def main(out, subs):
    disp = OrderedDict()
    for f in sorted(glob.glob(out + "/*/*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if subs and not any(s in k for s in subs):
                continue
            key = (f.split("/")[-2], int(r["Dispatch_Id"]))
            e = disp.setdefault(key, {"kernel": k.split("(")[0], "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # align the passes by occurrence order of each kernel
    passes = OrderedDict()
    for (p, d), e in disp.items():
        passes.setdefault(p, []).append(e)
    rows = []
    for p, lst in passes.items():
        occ = {}
        for e in lst:
            i = occ.get(e["kernel"], 0)
            occ[e["kernel"]] = i + 1
            while len(rows) <= len([r for r in rows]) and False:
                pass
            match = [r for r in rows if r["kernel"] == e["kernel"] and r["_i"] == i]
            if match:
                r = match[0]
                r.update({k: v for k, v in e.items() if k not in ("kernel", "ns")})
                r["ns_" + p] = e["ns"]
            else:
                r = dict(e)
                r["_i"] = i
                r["ns_" + p] = e["ns"]
                rows.append(r)
    res = []
    for r in rows:
        d = {k: v for k, v in r.items() if k != "_i"}
        wc = r.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in r:
                    d["frac_" + c] = r[c] / wc
        ns = next((v for k, v in r.items() if k.startswith("ns_")), 0)
        if wc and ns:   # resident waves per CU over the kernel (quad-cycles x 4, 256 CUs, 2.4 GHz nominal clock)
            d["waves_per_cu"] = wc * 4.0 / (ns * 2.4 * 256)
        if r.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = r.get("SQ_LDS_BANK_CONFLICT", 0) / r["SQ_LDS_IDX_ACTIVE"]
        if r.get("SQ_INSTS_VALU") and r.get("SQ_INSTS_SALU"):
            d["salu_per_valu"] = r["SQ_INSTS_SALU"] / r["SQ_INSTS_VALU"]
        res.append(d)
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
