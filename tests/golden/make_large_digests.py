#!/usr/bin/env python3
"""Full-size canonical digests of BASELINE configs 3, 4 and 5 from the C oracle
(TEST INFRASTRUCTURE; writes tests/golden/large_digests.json).

The sequential oracle (oracle/pcc_oracle.c) converts each configuration one part
of the level-0 cells at a time (oracle/digest_main.c): level-0 subtrees are
independent (converter.rs:32-47, 114-139), and each part keeps the global
10 000-point batch structure (lib.rs:31-52).  Digests are per level-0 subtree
(oracle/digest.c, canonical form of SURVEY.md Appendix B.3).

  config 3: 100M points, Gaussian mixture (synthetic kind 2), seed 3
  config 4: 1B uniform points in [-1000,1000)^3, seed 4
  config 5: config 4's cloud, then +100M uniform points, seed 5 (incremental merge:
            converting A then B into one directory == one run over A then B,
            tests/test_merge_oracle.py)

Run from the repo root:  python tests/golden/make_large_digests.py  [--jobs 8]
(about 10-20 minutes on 8 cores; peak memory about 4 GB per job).
"""
import argparse
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
EXE = os.path.join(ROOT, "oracle", "build", "orc_digest")

CONFIGS = {
    "config3": {"streams": [{"seed": 3, "kind": 2, "n": 100_000_000}]},
    # config 5 = phase 2 of the config-4 run
    "config4": {"streams": [{"seed": 4, "kind": 0, "n": 1_000_000_000}, {"seed": 5, "kind": 0, "n": 100_000_000}]},
}
PARTS = 8


def run_part(streams, part):
    args = [EXE, str(part), str(PARTS)]
    for s in streams:
        args += [str(s["seed"]), str(s["kind"]), str(s["n"])]
    out = subprocess.run(args, capture_output=True, text=True, check=True).stdout
    return [json.loads(line) for line in out.splitlines() if line.strip()]


def combine(lines, phase):
    subs = sorted((dict(ln) for ln in lines if ln["phase"] == phase and "subtree" in ln), key=lambda d: d["subtree"])
    sums = [ln for ln in lines if ln["phase"] == phase and ln.get("summary")]
    bb = {tuple(s["bbox_bits"]) for s in sums}
    assert len(bb) == 1, "parts disagree on the bounding box"
    assert all(s["error"] == 0 for s in sums)
    for d in subs:
        del d["phase"]
    return {
        "subtrees": subs,
        "input_points": sums[0]["input_points"],
        "arrivals": sum(s["arrivals"] for s in sums),
        "grid_points": sum(s["grid_points"] for s in sums),
        "kept_points": sum(s["kept_points"] for s in sums),
        "hierarchies": max(d["levels"] for d in subs),
        "bbox_bits": list(bb.pop()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    out_path = os.path.join(HERE, "large_digests.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for name, cfg in CONFIGS.items():
        if a.only and name != a.only:
            continue
        with ThreadPoolExecutor(a.jobs) as ex:
            lines = [ln for part in ex.map(lambda p: run_part(cfg["streams"], p), range(PARTS)) for ln in part]
        with open(os.path.join("/tmp", f"large_digests_{name}.jsonl"), "w") as f:   # raw lines, for re-combining
            f.write("".join(json.dumps(ln) + "\n" for ln in lines))
        s0 = cfg["streams"][0]
        res[name] = dict(combine(lines, 1), synth=s0)
        if len(cfg["streams"]) > 1:
            res["config5"] = dict(combine(lines, 2), synth=cfg["streams"][1], prior_synth=s0)
        print(name, "done", file=sys.stderr, flush=True)
    res["_generator"] = ("tests/golden/make_large_digests.py: oracle/digest_main.c (sequential C oracle, "
                         "per level-0 part, global 10 000-point batches), digests of oracle/digest.c")
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
