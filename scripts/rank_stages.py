#!/usr/bin/env python3
"""Per-stage timing of the sharded step (pcconv/dist.py::shard_build) with ONE
PROCESS PER RANK, every rank on the box's single MI355X (gloo over the host for
the exchanges, the product HIP ops for everything else).

  python scripts/rank_stages.py --config 4 --world 8     # 1B uniform, 125M points per rank
  python scripts/rank_stages.py --config 3 --world 8     # 100M Gaussian mixture, shared cells

For each rank: the stage times of one step (shard_build's `ms`, device synced at
every stage boundary), measured with all ranks running at once, and the rank's
build stages timed again ALONE (ranks take turns, the others wait at a barrier),
which is what that rank's build costs on its own GPU.  The exchange stages run
over gloo through host memory here (RCCL over xGMI on an 8-GPU node), so they
are reported but are not representative.  Prints one JSON object."""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "point-cloud_amd"))

BUILD_STAGES = ("build", "lead", "subtrees")


class TimedComm:
    """The communicator with its calls timed (device synced first, so queued
    device work is not counted as communication); shard_build splits each
    stage into <stage>_comm (collectives) and the rest (local work)."""

    def __init__(self, comm):
        self.c = comm
        self.elapsed_ms = 0.0

    def move(self, t, dev):   # gloo's host staging of device tensors counts as communication
        import torch
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = t.to(dev)
        torch.cuda.synchronize()
        self.elapsed_ms += (time.perf_counter() - t0) * 1e3
        return r

    def __getattr__(self, name):
        import torch
        a = getattr(self.c, name)
        if not callable(a):
            return a

        def timed(*args, **kw):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = a(*args, **kw)
            self.elapsed_ms += (time.perf_counter() - t0) * 1e3
            return r
        return timed


class RecOps:
    """The ops with their local device calls recorded (stage, name, args), so a
    rank can replay them alone on the GPU after the step."""
    STAGE = {"bbox": "bbox", "bbox_sample": "bbox", "bbox_slab_histogram": "bbox", "slab_histogram": "hist", "histogram": "hist", "route_bitmaps": "route",
             "route_slabs": "route", "route": "route", "keys_from_bitmaps": "exchange", "batch_starts": "exchange",
             "resolve_level1": "resolve"}

    def __init__(self, ops):
        self.o = ops
        self.calls = []

    def __getattr__(self, name):
        a = getattr(self.o, name)
        if name not in self.STAGE or not callable(a):
            return a

        def rec(*args, **kw):
            self.calls.append((self.STAGE[name], a, args, kw))
            return a(*args, **kw)
        return rec


def worker(rank, world, port, args, res_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pcconv
        from pcconv.dist import HipShardOps, TorchComm, key_range, shard_build
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        a, b = key_range(args.points, rank, world)
        pts = torch.empty((b - a, 4), dtype=torch.int32, device=dev)
        pcconv.synth_device(pts.data_ptr(), a, b - a, args.seed, args.kind, -1000.0, 2000.0, 0)
        torch.cuda.synchronize()
        ops = RecOps(HipShardOps(0, batch_size=10_000))
        ops.o.record_inputs = True
        # the host-only pieces of the plan and assembly stages, recorded too so
        # they can be timed alone (measured inside the step they include waits
        # for a GPU the other ranks share)
        import pcconv.dist as D
        host_calls = []
        HOST = {"plan_split": "plan", "children_ids": "plan", "route_table": "plan"}

        def hrec(stage, fn):
            def f(*fa, **fk):
                host_calls.append((stage, fn, fa, fk))
                return fn(*fa, **fk)
            return f
        for name, stage in HOST.items():
            setattr(D, name, hrec(stage, getattr(D, name)))
        comm = TimedComm(TorchComm(torch.device("cpu")))
        files = [args.points]
        for _ in range(args.warmup):
            shard_build(comm, ops, pts, a, files)
        dist.barrier()
        ops.calls = []
        host_calls.clear()
        r = shard_build(comm, ops, pts, a, files, sync=torch.cuda.synchronize)
        # the same step again, this rank's build stages alone on the GPU: every
        # rank runs the step, but a rank's local builds wait for their turn
        alone = {}
        for turn in range(world):
            dist.barrier()
            if turn == rank:
                li = dict(ops.o.last_inputs)
                for stage, fn, fa, fk in ops.calls:   # the recorded local device calls
                    best = None
                    for _ in range(2):
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        fn(*fa, **fk)
                        torch.cuda.synchronize()
                        t = (time.perf_counter() - t0) * 1e3
                        best = t if best is None else min(best, t)
                    alone["dev_" + stage] = alone.get("dev_" + stage, 0.0) + best
                for stage, fn, fa, fk in host_calls:   # the recorded host-only calls (best of 3)
                    best = None
                    for _ in range(3):
                        t0 = time.perf_counter()
                        fn(*fa, **fk)
                        t = (time.perf_counter() - t0) * 1e3
                        best = t if best is None else min(best, t)
                    alone["host_" + stage] = alone.get("host_" + stage, 0.0) + best
                for name, fn, name_in in (("build", ops.build, "build"), ("lead", ops.lead_build_raw, "lead"),
                                          ("subtrees", ops.sub_build, "sub")):
                    if name_in not in li:
                        continue
                    best = None
                    for _ in range(2):   # the better of two runs (the first may grow buffers)
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        fn(*li[name_in])
                        torch.cuda.synchronize()
                        t = (time.perf_counter() - t0) * 1e3
                        best = t if best is None else min(best, t)
                    alone[name] = best
        dist.barrier()
        out = {"rank": rank, "ms": r.ms, "recv_points": r.recv_points, "owned_cells": r.owned_cells,
               "sub_points": r.sub_points, "assembled_cells": r.assembled_cells,
               "phases": r.local.get("phases"), "arrivals": int(r.local.get("arrivals", 0)),
               "alone": alone, "plan": r.plan}
        with open(os.path.join(res_dir, f"rank{rank}.json"), "w") as f:
            json.dump(out, f)
        ops.close()
    finally:
        dist.destroy_process_group()


def main():
    import tempfile
    import torch.multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4, choices=(3, 4))
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--points", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    args.kind, args.seed = (0, 4) if args.config == 4 else (2, 3)
    if not args.points:
        args.points = 1_000_000_000 if args.config == 4 else 100_000_000
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    rd = tempfile.mkdtemp(prefix="pcc_stages_")
    mp.spawn(worker, args=(args.world, port, args, rd), nprocs=args.world, join=True)
    ranks = [json.load(open(os.path.join(rd, f"rank{i}.json"))) for i in range(args.world)]
    for r in ranks:
        ms = r["ms"]
        stages = [k for k in ms if not k.endswith("_comm")]
        comm = {k: ms.get(k + "_comm", 0.0) for k in stages}
        local = {k: max(0.0, ms[k] - comm[k]) for k in stages}
        r["comm_ms_gloo"] = sum(comm.values())
        r["local_ms_concurrent"] = local
        ba = sum(r["alone"].get(k, 0.0) for k in BUILD_STAGES)
        r["build_ms_alone"] = ba
        # local non-build work: the device calls outside the builds replayed alone,
        # plus the host-only stages (ownership plan, assembly bookkeeping,
        # summary) as measured; the exchange stages' local part is gloo's host
        # staging (device <-> host copies), absent with RCCL, and left out
        dev = {k[4:]: v for k, v in r["alone"].items() if k.startswith("dev_") and k != "dev_exchange"}
        # plan: its host calls timed alone (plan_split, children_ids,
        # route_table: the stage's work, the rest is a few numpy lookups);
        # assembly (with its segment bookkeeping) and summary as measured in
        # the step, whose sync points may wait for the other ranks' kernels
        host = {"plan": r["alone"].get("host_plan", local.get("plan", 0.0)),
                "assemble": local.get("assemble", 0.0), "summary": local.get("summary", 0.0)}
        r["host_stage_ms_in_step"] = {k: local.get(k, 0.0) for k in ("plan", "assemble", "summary")}
        nb = sum(dev.values()) + sum(host.values()) + r["alone"].get("dev_exchange", 0.0)
        r["non_build_device_alone_ms"] = dev
        r["non_build_host_ms"] = host
        r["non_build_local_ms"] = nb
        r["non_build_over_build_alone"] = nb / ba if ba else None
    print(json.dumps({"config": args.config, "world": args.world, "points": args.points,
                      "note": "one process per rank on ONE MI355X; collectives over gloo (host), not RCCL/xGMI, "
                              "timed apart (<stage>_comm); 'alone' = the rank's builds and bucket resolution "
                              "re-run (best of 2) while the other ranks wait; the plan's host calls timed "
                              "alone too (best of 3)",
                      "ranks": ranks}))


if __name__ == "__main__":
    main()
