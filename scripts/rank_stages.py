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
EXCHANGE_STAGES = ("exchange", "exchange2")


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
        ops = HipShardOps(0, batch_size=10_000)
        comm = TorchComm(torch.device("cpu"))
        files = [args.points]
        for _ in range(args.warmup):
            shard_build(comm, ops, pts, a, files)
        dist.barrier()
        r = shard_build(comm, ops, pts, a, files, sync=torch.cuda.synchronize)
        # the same step again, this rank's build stages alone on the GPU: every
        # rank runs the step, but a rank's local builds wait for their turn
        alone = {}
        for turn in range(world):
            dist.barrier()
            if turn == rank:
                li = dict(ops.last_inputs)
                for name, fn in (("build", ops.build), ("lead", ops.lead_build_raw), ("subtrees", ops.sub_build)):
                    if name == "subtrees":
                        name_in = "sub"
                    else:
                        name_in = name
                    if name_in not in li:
                        continue
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    fn(*li[name_in])
                    torch.cuda.synchronize()
                    alone[name] = (time.perf_counter() - t0) * 1e3
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
        b = sum(ms.get(k, 0.0) for k in BUILD_STAGES)
        ex = sum(ms.get(k, 0.0) for k in EXCHANGE_STAGES)
        other = sum(v for k, v in ms.items() if k not in BUILD_STAGES and k not in EXCHANGE_STAGES)
        r["build_ms_concurrent"] = b
        r["exchange_ms_gloo"] = ex
        r["non_build_non_exchange_ms"] = other
        ba = sum(r["alone"].get(k, 0.0) for k in BUILD_STAGES)
        r["build_ms_alone"] = ba
        r["non_build_over_build_alone"] = other / ba if ba else None
    print(json.dumps({"config": args.config, "world": args.world, "points": args.points,
                      "note": "one process per rank on ONE MI355X; exchanges over gloo (host), not RCCL/xGMI; "
                              "'alone' = the rank's whole-cell build re-run while the other ranks wait",
                      "ranks": ranks}))


if __name__ == "__main__":
    main()
