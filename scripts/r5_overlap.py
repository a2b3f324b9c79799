"""Exchange / level-0 overlap of a sharded step, measured on one GPU.

`world` thread ranks on cuda:0 (pcconv.dist.ThreadComm: the exchange is device
copies, on each rank's side stream) run shard_build with HipShardOps; with
--rounds R > 1 the exchange lands in R rounds and level-0 pass 1 (k_l0_tile6)
of the landed groups is queued behind each.  Run under
`rocprofv3 --kernel-trace --output-format csv -d DIR -o kt -- python3 scripts/r5_overlap.py ...`,
then `python3 scripts/r5_overlap.py --trace DIR/kt_kernel_trace.csv --stages FILE`
prints the per-stage JSON: the last step's exchange copies and pass-1 kernels
from the trace (GPU timestamps), and the ranks' stage times and early tiles.
"""
import argparse
import csv
import json
import os
import sys
import tempfile
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "point-cloud_amd"))


def run(args):
    import torch
    import pcconv
    from pcconv.dist import HipShardOps, ThreadComm, ThreadGroup, key_range, shard_build
    dev = torch.device("cuda", 0)
    grp = ThreadGroup(args.world)
    res, errs = [None] * args.world, []
    tmp = tempfile.mkdtemp(dir="/dev/shm" if os.path.isdir("/dev/shm") else None)

    def worker(r):
        try:
            torch.cuda.set_device(dev)
            a, b = key_range(args.points, r, args.world)
            pts = torch.empty((b - a, 4), dtype=torch.int32, device=dev)
            pcconv.synth_device(pts.data_ptr(), a, b - a, 4, 0)
            ops = HipShardOps(0, out_dir=os.path.join(tmp, "out"))
            ops.landing_rounds = args.rounds
            comm = ThreadComm(grp, r, dev)
            for s in range(args.steps):
                if s == args.steps - 1:
                    comm.barrier()
                    torch.cuda.synchronize()
                    if r == 0:
                        torch.cuda._sleep(1000)   # trace marker: the last step starts after it
                        torch.cuda.synchronize()
                    comm.barrier()
                out = shard_build(comm, ops, pts, a, [args.points], sync=torch.cuda.synchronize)
            res[r] = {"rank": r, "ms": {k: round(v, 3) for k, v in out.ms.items()}, "recv_points": out.recv_points,
                      "level0_early_tiles": int(out.local.get("level0_early_tiles", 0)),
                      "level0_tiles": (out.recv_points + 3071) // 3072}
            ops.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(args.world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    with open(args.stages, "w") as f:
        json.dump({"points": args.points, "world": args.world, "rounds": args.rounds, "ranks": res}, f)


def summarize(args):
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]))
    rows.sort()
    marks = [x[1] for x in rows if "sleep" in x[2].lower() or "spin" in x[2].lower()]
    t0 = marks[-1] if marks else rows[0][0]
    last = [x for x in rows if x[0] >= t0]
    tile6 = [x for x in last if "k_l0_tile6" in x[2]]
    slab = [x for x in last if "k_slab" in x[2]]
    route = [x for x in last if "k_route" in x[2]]
    st = json.load(open(args.stages))
    ms = lambda v: round(v / 1e6, 3)   # ns -> ms from the marker
    # the exchange: copy kernels after the routes on streams that run no library
    # kernel (the exchange's side streams, or torch's stream without rounds)
    lib_streams = {x[3] for x in last if "pcc::" in x[2]}
    r_end = max((x[1] for x in route), default=t0)
    s_end = slab[0][0] if slab else last[-1][1]
    ex = [x for x in last if "copy" in x[2].lower() and x[3] not in lib_streams and r_end <= x[0] < s_end]
    out = {"what": "last sharded step, GPU timestamps (ms after the step's start marker)",
           "rounds": st["rounds"], "world": st["world"], "points": st["points"],
           "exchange_copies": len(ex),
           "exchange_first_start_ms": ms(ex[0][0] - t0) if ex else None,
           "exchange_last_end_ms": ms(max(x[1] for x in ex) - t0) if ex else None,
           "tile6_kernels": len(tile6),
           "tile6_first_start_ms": ms(tile6[0][0] - t0) if tile6 else None,
           "tile6_started_before_exchange_end": sum(1 for x in tile6 if ex and x[0] < max(y[1] for y in ex)),
           "first_slab_start_ms": ms(slab[0][0] - t0) if slab else None,
           "ranks": st["ranks"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=400_000_000)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--stages", default="gpurun_out/r5_overlap_stages.json")
    ap.add_argument("--trace", default=None)
    a = ap.parse_args()
    summarize(a) if a.trace else run(a)
