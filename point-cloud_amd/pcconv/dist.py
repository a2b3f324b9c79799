"""Sharded multi-GPU build: one process per GPU, one conversion.

The reference converter is single-threaded (point-converter/src/converter.rs:72-139).
Its level-0 subtrees are independent, because every level-h cell has a unique
level-0 ancestor (converter.rs:32-47 groups a point of cell c at h+1 into a child
of c).  So the unit of ownership is the level-0 cell, and one step is:

  1. every rank holds a contiguous key range of the global input (keys = global
     input index, lib.rs:31-52 order) resident in HBM;
  2. local bbox -> all-reduce(max of [-min, max]) -> global bbox (the metadata
     bounding box, converter.rs:96-104) and the level-0 grid it spans;
  3. per-cell histogram -> all-reduce(sum) -> identical owner table on every
     rank (`assign_owners`, deterministic);
  4. stable partition by owner (HIP) -> all-to-all of counts, then one grouped
     batch of point-to-point transfers (RCCL over xGMI) of the 16-B points and
     the u32 keys straight into this rank's receive buffers, at most 2^30 bytes
     per transfer (larger ones corrupt on this stack, TorchComm.max_msg_bytes);
     the own segment is a device copy.  Segments land in source-rank order, so
     each rank's input stays in global key order.  With one rank the partition
     is the identity and nothing is routed;
  5. independent level-synchronous builds with the GLOBAL batch structure,
     reading the receive buffers in place (pcc_declare_files +
     pcc_set_keyed_points_device);
  6. all-reduce(max) of `hierarchies`; every rank writes its own (disjoint) cell
     files, rank 0 writes metadata.json after a barrier.

Incremental merge (config 5, `merge=True`): the output directory holds an
existing cloud.  After step 3 every rank opens it restricted to the level-0
subtrees it owns and that receive new points (pcc_open_subtrees: converter.rs:
187-207 for its own cells only), merges its routed points into them (its seeds
first, then its new points in global key order) and rewrites those subtrees;
the other subtrees stay as they are on disk.  The metadata values continue from
the existing metadata.json (lib.rs:86-101: counters, Aabb::extend_aabb).

The collectives go through a small communicator interface: `TorchComm`
(torch.distributed; backend "nccl" is RCCL on ROCm, "gloo" for the CPU tests) or
`ThreadComm` (ranks as threads of one process, used to run the exchange on a
single GPU in tests).  Local work goes through an ops object: `HipShardOps` is
the product (libpcconv.so, no fallback); tests inject CPU restatements.
"""
from __future__ import annotations

import os
import tempfile
import threading
import time
from dataclasses import dataclass, field

import numpy as np
import torch

import pcconv


# ----------------------------------------------------------------- communicators
class TorchComm:
    """torch.distributed process group (nccl == RCCL on ROCm, or gloo)."""

    def __init__(self, device: torch.device):
        import torch.distributed as dist
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.device = device

    def allreduce_(self, t: torch.Tensor, op: str) -> torch.Tensor:
        ops = {"sum": self.dist.ReduceOp.SUM, "max": self.dist.ReduceOp.MAX}
        self.dist.all_reduce(t, op=ops[op])
        return t

    def alltoall_counts(self, counts: list[int]) -> list[int]:
        s = torch.tensor(counts, dtype=torch.int64, device=self.device)
        r = torch.empty_like(s)
        self.dist.all_to_all_single(r, s)
        return [int(v) for v in r.tolist()]

    # bytes one RCCL point-to-point transfer may carry.  On this stack a single
    # send/recv of more than 2^30 bytes (all_to_all_single is built from the same
    # transfers) returns the second half of the message corrupted, for any dtype;
    # exactly 2^30 is fine (scripts/a2a_threshold.py, profiles/r2_rccl_threshold.log)
    max_msg_bytes = 1 << 30

    def alltoallv_into(self, send: torch.Tensor, send_counts: list[int], recv_counts: list[int],
                       out: torch.Tensor) -> torch.Tensor:
        """Rows send[so[p]:so[p]+send_counts[p]] go to rank p; rank p's rows land
        in out[ro[p]:ro[p]+recv_counts[p]] (source-rank order).  One grouped
        batch of point-to-point transfers straight into those slices, each at
        most `max_msg_bytes`; the own segment is a local device copy."""
        row = send.element_size() * max(1, int(np.prod(send.shape[1:])))
        mr = max(1, self.max_msg_bytes // row)
        so = np.concatenate([[0], np.cumsum(send_counts)]).astype(np.int64)
        ro = np.concatenate([[0], np.cumsum(recv_counts)]).astype(np.int64)
        me = self.rank
        if int(send_counts[me]) != int(recv_counts[me]):
            raise ValueError("own segment: send and receive counts differ")
        if send_counts[me]:
            out.narrow(0, int(ro[me]), int(recv_counts[me])).copy_(send.narrow(0, int(so[me]), int(send_counts[me])))
        ops = []
        for k in range(1, self.world):   # peers in ring order from this rank
            p_to, p_from = (me + k) % self.world, (me - k) % self.world
            for a in range(0, int(send_counts[p_to]), mr):
                ops.append(self.dist.P2POp(self.dist.isend, send.narrow(0, int(so[p_to]) + a,
                                                                        min(mr, int(send_counts[p_to]) - a)), p_to))
            for b in range(0, int(recv_counts[p_from]), mr):
                ops.append(self.dist.P2POp(self.dist.irecv, out.narrow(0, int(ro[p_from]) + b,
                                                                       min(mr, int(recv_counts[p_from]) - b)), p_from))
        if ops:
            for req in self.dist.batch_isend_irecv(ops):
                req.wait()
        return out

    def barrier(self):
        self.dist.barrier()


class ThreadGroup:
    """Shared state of `world` in-process ranks (one thread each)."""

    def __init__(self, world: int):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slot: list = [None] * world


class ThreadComm:
    """Collectives between threads of one process (same semantics as TorchComm)."""

    def __init__(self, group: ThreadGroup, rank: int, device: torch.device):
        self.g = group
        self.rank = rank
        self.world = group.world
        self.device = device

    def _exchange(self, obj):
        self.g.slot[self.rank] = obj
        self.g.bar.wait()
        allv = list(self.g.slot)
        self.g.bar.wait()   # nobody overwrites a slot before everyone has read it
        return allv

    def allreduce_(self, t: torch.Tensor, op: str) -> torch.Tensor:
        allv = self._exchange(t.clone())
        acc = allv[0].clone()
        for v in allv[1:]:
            acc = acc + v.to(acc.device) if op == "sum" else torch.maximum(acc, v.to(acc.device))
        t.copy_(acc)
        return t

    def alltoall_counts(self, counts: list[int]) -> list[int]:
        allv = self._exchange(list(counts))
        return [int(allv[src][self.rank]) for src in range(self.world)]

    def alltoallv_into(self, send: torch.Tensor, send_counts: list[int], recv_counts: list[int],
                       out: torch.Tensor) -> torch.Tensor:
        allv = self._exchange((send, list(send_counts)))
        o_out = 0
        for src in range(self.world):
            t, c = allv[src]
            o = sum(c[: self.rank])
            m = int(c[self.rank])
            if m != int(recv_counts[src]):
                raise ValueError("receive count differs from the sender's count")
            out.narrow(0, o_out, m).copy_(t.narrow(0, o, m))
            o_out += m
        self.g.bar.wait()   # senders may free/reuse their buffers only after every copy
        return out

    def barrier(self):
        self.g.bar.wait()


# ----------------------------------------------------------------- ownership
def assign_owners(hist: np.ndarray, world: int, greedy_max: int = 4096) -> np.ndarray:
    """Owner rank of every level-0 cell from the GLOBAL histogram (identical on
    every rank).  Up to `greedy_max` non-empty cells: LPT greedy (largest cell
    first, ties by cell id, to the least-loaded rank, ties by rank).  Beyond
    that: contiguous cell-id ranges split at equal point counts."""
    hist = np.asarray(hist, dtype=np.int64)
    owner = np.zeros(len(hist), dtype=np.uint32)
    nz = np.flatnonzero(hist)
    if world <= 1 or len(nz) == 0:
        return owner
    if len(nz) <= greedy_max:
        order = nz[np.lexsort((nz, -hist[nz]))]
        load = np.zeros(world, dtype=np.int64)
        for c in order:
            r = int(np.argmin(load))
            owner[c] = r
            load[r] += hist[c]
        return owner
    before = np.cumsum(hist) - hist
    owner[:] = np.minimum(world - 1, (before * world) // max(int(hist.sum()), 1)).astype(np.uint32)
    return owner


# ----------------------------------------------------------------- local ops (product)
class HipShardOps:
    """Local per-rank work on the GPU through libpcconv.so (no CPU fallback)."""

    def __init__(self, device_index: int, out_dir: str | None = None, batch_size: int = 10_000,
                 config: dict | None = None, merge: bool = False):
        self.dev = device_index
        self.cfg = dict(config or {})
        self.batch_size = batch_size
        self.merge = merge
        self._tmp = None
        self.subtrees = None
        if merge:   # the converter opens on the existing cloud once the owned subtrees are known
            if out_dir is None:
                raise ValueError("a sharded merge needs the directory of the existing cloud")
            # lib.rs:86-101: the existing metadata.json's config governs the merge;
            # the shard grid must be the engine's level-0 grid, so a caller config
            # that disagrees is an error rather than a silently split cell
            disk = read_prior_meta(out_dir)["config"]
            for k, v in self.cfg.items():
                if k in disk and float(disk[k]) != float(v):
                    raise ValueError(f"config {k}={v} differs from the existing cloud's {disk[k]}")
            self.cfg = {k: disk[k] for k in ("cell_point_overflow_limit", "sub_grid_dimension", "max_cell_size")}
            self.max_cell_size = float(self.cfg["max_cell_size"])
            self.out_dir = out_dir
            self.conv = None
            return
        self.max_cell_size = float(self.cfg.get("max_cell_size", 1000.0))
        if out_dir is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="pcc_shard_")
            out_dir = self._tmp.name
        elif os.path.exists(os.path.join(out_dir, "metadata.json")) and read_prior_meta(out_dir)["number_of_points"] > 0:
            # pcc_open would turn this into a merge on every rank (each loading and
            # rewriting the whole existing cloud): refuse, merge=True is the way
            raise ValueError(f"{out_dir} already holds a converted cloud; open it with merge=True")
        self.out_dir = out_dir
        self.conv = pcconv.Converter(out_dir, batch_size=batch_size, device=device_index, config=self.cfg)

    def prior_meta(self) -> dict:
        return read_prior_meta(self.out_dir)

    def set_subtrees(self, cells: np.ndarray):
        """Merge mode: (re)open the existing cloud restricted to these level-0 cells."""
        cells = np.asarray(cells, dtype=np.int32).reshape(-1, 3)
        if self.conv is not None and self.subtrees is not None and np.array_equal(cells, self.subtrees):
            return
        if self.conv is not None:
            self.conv.close()
        self.conv = pcconv.Converter(self.out_dir, batch_size=self.batch_size, device=self.dev, config=self.cfg,
                                     subtrees=cells)
        self.subtrees = cells

    def _ready(self):
        # inputs may come from torch kernels or RCCL on torch's streams; the
        # library runs on its own stream, so order them through the host
        torch.cuda.synchronize(self.dev)

    def bbox(self, pts: torch.Tensor):
        self._ready()
        return pcconv.shard_bbox(pts.data_ptr(), pts.shape[0], self.dev)

    def grid(self, gmin, gmax) -> pcconv.ShardGrid:
        return pcconv.shard_grid_from_bbox(gmin, gmax, self.max_cell_size)

    def histogram(self, pts: torch.Tensor, grid) -> torch.Tensor:
        h = torch.empty(grid.ncells, dtype=torch.int32, device=pts.device)
        self._ready()
        pcconv.shard_histogram(pts.data_ptr(), pts.shape[0], grid, h.data_ptr(), self.dev)
        return h

    def route(self, pts: torch.Tensor, key0: int, grid, owner: torch.Tensor, world: int):
        n = pts.shape[0]
        send = torch.empty_like(pts)
        keys = torch.empty(n, dtype=torch.int32, device=pts.device)
        self._ready()
        counts = pcconv.shard_route(pts.data_ptr(), n, key0, grid, owner.data_ptr(), world, send.data_ptr(),
                                    keys.data_ptr(), self.dev)
        return send, keys, counts

    def build(self, file_points, pts: torch.Tensor, keys: torch.Tensor | None) -> dict:
        """keys None: this rank holds the whole input in key order (keys 0..n-1).
        The build reads `pts`/`keys` in place (borrowed until it returns)."""
        c = self.conv
        self._ready()
        c.clear_input()
        c.declare_files(file_points)
        c.set_keyed_points_device(pts.data_ptr(), 0 if keys is None else keys.data_ptr(), pts.shape[0])
        return c.build()

    def write(self, summary: dict, cells: bool, metadata: bool):
        c = self.conv
        c.set_summary(summary["number_of_points"], summary["bbox_min"], summary["bbox_max"], summary["hierarchies"])
        if cells:
            c.write_cells()
        if metadata:
            c.write_metadata()

    def close(self):
        if self.conv is not None:
            self.conv.close()
        if self._tmp is not None:
            self._tmp.cleanup()


# ----------------------------------------------------------------- one sharded step
@dataclass
class ShardResult:
    summary: dict
    local: dict
    recv_points: int
    owned_cells: int
    ms: dict = field(default_factory=dict)


def read_prior_meta(out_dir: str) -> dict:
    """metadata.json of an existing cloud (lib.rs:86-101 load_metadata)."""
    import json
    with open(os.path.join(out_dir, "metadata.json")) as f:
        m = json.load(f)
    return {"number_of_points": int(m["number_of_points"]), "hierarchies": int(m["hierarchies"]),
            "bbox_min": [float(v) for v in m["bounding_box"]["min"]],
            "bbox_max": [float(v) for v in m["bounding_box"]["max"]],
            "config": {"cell_point_overflow_limit": int(m["config"]["cell_point_overflow_limit"]),
                       "sub_grid_dimension": int(m["config"]["sub_grid_dimension"]),
                       "max_cell_size": float(m["config"]["max_cell_size"])}}


def cell_triples(ids: np.ndarray, grid) -> np.ndarray:
    """Level-0 cell indices (x, y, z) of linear shard-grid ids ((x*dy + y)*dz + z)."""
    ids = np.asarray(ids, dtype=np.int64)
    d1, d2 = int(grid.dims[1]), int(grid.dims[2])
    out = np.stack([ids // (d1 * d2) + int(grid.lo[0]), (ids // d2) % d1 + int(grid.lo[1]), ids % d2 + int(grid.lo[2])],
                   axis=1)
    return out.astype(np.int32).reshape(-1, 3)


def shard_build(comm, ops, pts: torch.Tensor, key0: int, file_points, write: bool = False,
                sync=None, merge: bool = False) -> ShardResult:
    """One sharded conversion step.  `pts` is this rank's (n, 4) int32 view of
    16-B points with global keys key0 .. key0+n-1 (contiguous ranges in rank
    order).  `file_points` is the GLOBAL file structure.  `sync` (optional)
    synchronises the device for stage timing.  `merge`: incremental merge into
    the existing cloud of the ops' directory (module docstring)."""
    ms = {}
    t0 = time.perf_counter()

    def mark(name):
        nonlocal t0
        if sync is not None:
            sync()
        t1 = time.perf_counter()
        ms[name] = ms.get(name, 0.0) + (t1 - t0) * 1e3
        t0 = t1

    n_total = int(sum(int(v) for v in file_points))
    # 2. global bounding box (converter.rs:96-104: componentwise min/max)
    if pts.shape[0]:
        bmin, bmax = ops.bbox(pts)
    else:
        bmin, bmax = [float("inf")] * 3, [float("-inf")] * 3
    bb = torch.tensor([-bmin[0], -bmin[1], -bmin[2], bmax[0], bmax[1], bmax[2]], dtype=torch.float32,
                      device=comm.device)
    comm.allreduce_(bb, "max")
    bbh = bb.cpu().tolist()
    gmin, gmax = [-bbh[0], -bbh[1], -bbh[2]], bbh[3:]
    mark("bbox")
    if n_total == 0:
        recv = pts[:0]
        keys = torch.empty(0, dtype=torch.int32, device=pts.device)
        owned = 0
        if merge:
            ops.set_subtrees(np.zeros((0, 3), dtype=np.int32))
    else:
        # 3. level-0 ownership
        grid = ops.grid(gmin, gmax)
        hist = ops.histogram(pts, grid)
        hist = comm.allreduce_(hist.to(comm.device), "sum")
        hist_h = hist.cpu().numpy().astype(np.int64)
        owner_h = assign_owners(hist_h, comm.world)
        owned = int(np.count_nonzero((owner_h == comm.rank) & (hist_h > 0)))
        owner = torch.from_numpy(owner_h.astype(np.int32)).to(pts.device)
        if merge:   # the existing cells of the owned subtrees that receive new points
            ops.set_subtrees(cell_triples(np.flatnonzero((owner_h == comm.rank) & (hist_h > 0)), grid))
        mark("plan")
        # 4. route + exchange (grouped point-to-point transfers of points and keys)
        if comm.world == 1:   # one rank owns every cell: the partition is the identity
            recv, keys = pts, None
            mark("route")
        else:
            send, skeys, counts = ops.route(pts, key0, grid, owner, comm.world)
            mark("route")
            rcounts = comm.alltoall_counts(counts)
            nrecv = int(sum(rcounts))
            if comm.device == pts.device:   # receive straight into the build's input buffers
                recv = torch.empty((nrecv,) + tuple(pts.shape[1:]), dtype=pts.dtype, device=pts.device)
                keys = torch.empty(nrecv, dtype=torch.int32, device=pts.device)
                comm.alltoallv_into(send, counts, rcounts, recv)
                comm.alltoallv_into(skeys, counts, rcounts, keys)
            else:   # host communicator (gloo) driving device ops
                recv = torch.empty((nrecv,) + tuple(pts.shape[1:]), dtype=pts.dtype, device=comm.device)
                keys = torch.empty(nrecv, dtype=torch.int32, device=comm.device)
                comm.alltoallv_into(send.to(comm.device), counts, rcounts, recv)
                comm.alltoallv_into(skeys.to(comm.device), counts, rcounts, keys)
                recv, keys = recv.to(pts.device), keys.to(pts.device)
            del send, skeys
        mark("exchange")
    # 5. independent build of the owned level-0 subtrees
    local = ops.build(file_points, recv, keys)
    mark("build")
    # 6. global metadata values
    hz = torch.tensor([int(local["hierarchies"])], dtype=torch.int64, device=comm.device)
    comm.allreduce_(hz, "max")
    summary = {"number_of_points": n_total, "hierarchies": int(hz.item()),
               "bbox_min": gmin if n_total else [0.0, 0.0, 0.0], "bbox_max": gmax if n_total else [0.0, 0.0, 0.0]}
    if merge:   # lib.rs:86-101: counters continue; converter.rs:96-104 Aabb::extend_aabb
        pm = ops.prior_meta()
        if pm["number_of_points"] > 0:
            if n_total:
                summary["bbox_min"] = [min(a, b) for a, b in zip(gmin, pm["bbox_min"])]
                summary["bbox_max"] = [max(a, b) for a, b in zip(gmax, pm["bbox_max"])]
            else:
                summary["bbox_min"], summary["bbox_max"] = pm["bbox_min"], pm["bbox_max"]
        summary["number_of_points"] = n_total + pm["number_of_points"]
        summary["hierarchies"] = max(summary["hierarchies"], pm["hierarchies"])
    mark("summary")
    if write:
        ops.write(summary, cells=True, metadata=False)
        comm.barrier()
        if comm.rank == 0:
            ops.write(summary, cells=False, metadata=True)
        comm.barrier()
        mark("write")
    return ShardResult(summary=summary, local=local, recv_points=int(recv.shape[0]), owned_cells=owned, ms=ms)


def key_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous key range [a, b) of rank `rank` (input split evenly in order)."""
    return (n_total * rank) // world, (n_total * (rank + 1)) // world
