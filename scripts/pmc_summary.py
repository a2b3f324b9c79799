#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of scripts/pmc.sh into profiles/<name>.json.

HBM bytes per kernel follow MI355X_MICROARCH.md "HBM [CDNA4]": WRITE_SIZE (KB) is
exact; FETCH_SIZE (KB) reports half of the bytes of wide coalesced reads on
gfx950, so it is doubled.  Per-launch values are averages over the launches of
one build (bench.py --steps 1 --warmup 0)."""
import csv
import json
import re
import sys
from collections import OrderedDict


def load(path, counter):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            rows.append((r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0,
                         int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return rows


def main(out_dir, name, bench_json):
    fetch = load(f"{out_dir}/pmc_fetch/fetch_counter_collection.csv", "FETCH_SIZE")
    write = load(f"{out_dir}/pmc_write/write_counter_collection.csv", "WRITE_SIZE")
    k = OrderedDict()
    for nm, v, t in fetch:
        e = k.setdefault(nm, {"launches": 0, "fetch_bytes_raw": 0.0, "write_bytes": 0.0, "ns": 0})
        e["launches"] += 1
        e["fetch_bytes_raw"] += v
        e["ns"] += t
    for nm, v, t in write:
        k.setdefault(nm, {"launches": 0, "fetch_bytes_raw": 0.0, "write_bytes": 0.0, "ns": 0})["write_bytes"] += v
    for e in k.values():
        e["hbm_bytes"] = 2.0 * e["fetch_bytes_raw"] + e["write_bytes"]
        e["hbm_bytes_per_launch"] = e["hbm_bytes"] / max(e["launches"], 1)
    bench = json.load(open(bench_json))
    dense = next(v for n, v in k.items() if n.startswith(("pcc::k_slab(", "void pcc::k_slab<false>(", "void pcc::k_slab<false, false>(", "void pcc::k_slab<false, false, false>(",
                                                 "void pcc::k_slab<false, false, false, false>(")))
    # level-0 binning: every build kernel launched before the first slab kernel, against
    # one 16-B read and one 20-B write (point + key) per input point
    l0 = {"hbm_bytes": 0.0, "ns": 0, "kernels": []}
    for n, v in k.items():
        if "k_slab" in n:
            break
        if n.startswith(("pcc::k_synth", "__amd_rocclr")):   # bench input generation, runtime copies
            continue
        l0["hbm_bytes"] += v["hbm_bytes"]
        l0["ns"] += v["ns"]
        l0["kernels"].append(n.split("(")[0])
    npts = float(re.search(r"(\d+) ", bench["config"]["workload"]).group(1))
    arr = bench["stage_ms"]["dense_arrivals"]
    summary = {
        "workload": bench["config"]["workload"],
        "command": "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0",
        "correction": "hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM [CDNA4])",
        "dense_kernel": {"launches": dense["launches"], "hbm_bytes_per_launch": dense["hbm_bytes_per_launch"],
                         "alg_bytes_per_launch": 32.0 * arr / dense["launches"],
                         "traffic_over_alg": dense["hbm_bytes"] / (32.0 * arr)},
        "level0": {"kernels": l0["kernels"], "hbm_bytes": l0["hbm_bytes"], "alg_bytes": 36.0 * npts,
                   "traffic_over_alg": l0["hbm_bytes"] / (36.0 * npts), "ms": l0["ns"] / 1e6},
        "kernels": k,
    }
    # per launch of the dense kernel (one per level, in dispatch order), with the
    # level's arrivals from the engine's verbose log when the pass ran with PCC_VERBOSE=1
    lv_arr = []
    try:
        for line in open(f"{out_dir}/pmc_fetch.err"):
            m = re.search(r"\[pcc\] level (\d+): .*\(dense (\d+), small (\d+)\) arrivals (\d+)", line)
            if m:
                lv_arr.append((int(m.group(1)), int(m.group(2)), int(m.group(4))))
    except OSError:
        pass
    fd = [(t, v) for nm, v, t in fetch if "k_slab<" in nm and "k_slab_" not in nm]
    wd = [v for nm, v, t in write if "k_slab<" in nm and "k_slab_" not in nm]
    per = []
    dense_levels = [a for a in lv_arr if a[1] > 0]
    for i, ((t, f), w) in enumerate(zip(fd, wd)):
        e = {"launch": i, "ms": t / 1e6, "fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes": 2.0 * f + w}
        if i < len(dense_levels):
            lvl, _, arrivals = dense_levels[i]
            e.update({"level": lvl, "arrivals": arrivals, "alg_bytes": 32.0 * arrivals,
                      "traffic_over_alg": (2.0 * f + w) / (32.0 * arrivals),
                      "uncorrected_over_alg": (f + w) / (32.0 * arrivals),
                      "alg_GBps": 32.0 * arrivals / t})
        per.append(e)
    summary["dense_kernel"]["per_launch"] = per
    json.dump(summary, open(f"profiles/{name}.json", "w"), indent=1)
    for e in per:
        print(json.dumps(e))
    print(json.dumps(summary["dense_kernel"]))
    print(json.dumps({a: b for a, b in summary["level0"].items() if a != "kernels"}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
