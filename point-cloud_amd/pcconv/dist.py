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

import ctypes as C

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
        ops = self._p2p_ops(send, send_counts, recv_counts, out)
        if ops:
            for req in self.dist.batch_isend_irecv(ops):
                req.wait()
        return out

    def _p2p_ops(self, send, send_counts, recv_counts, out, part=(0, 1)) -> list:
        """The own segment copied locally; the point-to-point ops of the rest.
        part (r, R): only piece r of R of every segment (round_piece); the own
        segment is copied whole in piece 0."""
        row = send.element_size() * max(1, int(np.prod(send.shape[1:])))
        mr = max(1, self.max_msg_bytes // row)
        so = np.concatenate([[0], np.cumsum(send_counts)]).astype(np.int64)
        ro = np.concatenate([[0], np.cumsum(recv_counts)]).astype(np.int64)
        me = self.rank
        if int(send_counts[me]) != int(recv_counts[me]):
            raise ValueError("own segment: send and receive counts differ")
        if send_counts[me] and part[0] == 0:
            out.narrow(0, int(ro[me]), int(recv_counts[me])).copy_(send.narrow(0, int(so[me]), int(send_counts[me])))
        ops = []
        for k in range(1, self.world):   # peers in ring order from this rank
            p_to, p_from = (me + k) % self.world, (me - k) % self.world
            a0, a1 = round_piece(int(send_counts[p_to]), *part)
            for a in range(a0, a1, mr):
                ops.append(self.dist.P2POp(self.dist.isend, send.narrow(0, int(so[p_to]) + a, min(mr, a1 - a)), p_to))
            b0, b1 = round_piece(int(recv_counts[p_from]), *part)
            for b in range(b0, b1, mr):
                ops.append(self.dist.P2POp(self.dist.irecv, out.narrow(0, int(ro[p_from]) + b, min(mr, b1 - b)),
                                           p_from))
        return ops

    def alltoallv_rounds(self, send: torch.Tensor, send_counts: list[int], recv_counts: list[int],
                         out: torch.Tensor, rounds: int, on_landed) -> torch.Tensor:
        """alltoallv_into in `rounds` grouped batches, piece r of every segment in
        round r (all peers at once: every xGMI link busy in every round).  Round
        r + 1 is posted before round r is waited for; after the wait (on the
        current stream: the host does not block on RCCL) on_landed(ranges,
        stream) gets round r's received row ranges, so the consumer's work on
        them queues behind that round while the next one is in flight."""
        pend = None
        for r in range(rounds + 1):
            reqs = None
            if r < rounds:
                ops = self._p2p_ops(send, send_counts, recv_counts, out, part=(r, rounds))
                reqs = self.dist.batch_isend_irecv(ops) if ops else []
            if pend is not None:
                for req in pend[0]:
                    req.wait()
                on_landed(landed_ranges(recv_counts, self.rank, pend[1], rounds), _stream_handle(out))
            pend = (reqs, r)
        return out

    def alltoallv_many(self, specs):
        """alltoallv_into for several (send, send_counts, recv_counts, out) in ONE
        grouped batch of point-to-point transfers (one round trip, not one each)."""
        ops = []
        for send, sc, rc, out in specs:
            ops.extend(self._p2p_ops(send, sc, rc, out))
        if ops:
            for req in self.dist.batch_isend_irecv(ops):
                req.wait()

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

    def alltoallv_rounds(self, send: torch.Tensor, send_counts: list[int], recv_counts: list[int],
                         out: torch.Tensor, rounds: int, on_landed) -> torch.Tensor:
        """TorchComm.alltoallv_rounds between threads: piece r of every segment in
        round r, then on_landed(round r's row ranges, stream of the copies)."""
        allv = self._exchange((send, list(send_counts)))
        ro = np.concatenate([[0], np.cumsum([int(v) for v in recv_counts])]).astype(np.int64)
        for src in range(self.world):
            if int(allv[src][1][self.rank]) != int(recv_counts[src]):
                raise ValueError("receive count differs from the sender's count")
        for r in range(rounds):
            for src in range(self.world):
                t, c = allv[src]
                o = sum(int(v) for v in c[: self.rank])
                m = int(c[self.rank])
                a, b = round_piece(m, r, rounds) if src != self.rank else ((0, m) if r == 0 else (0, 0))
                if b > a:
                    out.narrow(0, int(ro[src]) + a, b - a).copy_(t.narrow(0, o + a, b - a))
            on_landed(landed_ranges(recv_counts, self.rank, r, rounds), _stream_handle(out))
        if out.is_cuda:   # (the copies read the other threads' buffers)
            torch.cuda.current_stream(out.device).synchronize()
        self.g.bar.wait()   # senders may free/reuse their buffers only after every copy
        return out

    def barrier(self):
        self.g.bar.wait()


def round_piece(count: int, r: int, rounds: int) -> tuple[int, int]:
    """Rows [a, b) of a segment of `count` rows that round r of `rounds` carries."""
    return count * r // rounds, count * (r + 1) // rounds


def landed_ranges(recv_counts, me: int, r: int, rounds: int) -> list[tuple[int, int]]:
    """Row ranges of the receive buffer (segments in source-rank order) that round
    r of an alltoallv_rounds completes: piece r of every peer's segment, and the
    own segment (a local copy) in round 0."""
    ro = np.concatenate([[0], np.cumsum([int(v) for v in recv_counts])]).astype(np.int64)
    out = []
    for src, cnt in enumerate(recv_counts):
        a, b = round_piece(int(cnt), r, rounds) if src != me else ((0, int(cnt)) if r == 0 else (0, 0))
        if b > a:
            out.append((int(ro[src]) + a, int(ro[src]) + b))
    return out


_sides = threading.local()


def _side_stream(dev) -> "torch.cuda.Stream":
    """The calling thread's side stream on `dev` for the exchange rounds (made once:
    creating a stream per step cost milliseconds)."""
    d = getattr(_sides, "d", None)
    if d is None:
        d = _sides.d = {}
    key = torch.device(dev).index
    if key not in d:
        d[key] = torch.cuda.Stream(dev)
    return d[key]


def _stream_handle(t: torch.Tensor) -> int:
    """The current HIP stream of t's device (0 for host tensors).  The null
    stream cannot be handed to the library (NULL there means "nothing to wait
    for"), so work on it is waited for here (shard_build exchanges on a side
    stream instead)."""
    if not t.is_cuda:
        return 0
    s = torch.cuda.current_stream(t.device)
    if int(s.cuda_stream) == 0:
        s.synchronize()
    return int(s.cuda_stream)


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
    if len(nz) <= greedy_max:   # (counts < 2^53: exact in the float64 loads)
        owner[nz] = pcconv.shard_lpt(hist[nz].astype(np.float64), world)[0]
        return owner
    before = np.cumsum(hist) - hist
    owner[:] = np.minimum(world - 1, (before * world) // max(int(hist.sum()), 1)).astype(np.uint32)
    return owner


# ----------------------------------------------------------------- split plan (skewed clouds)
# Cost model of the plan (relative units per point): a level-0 arrival costs
# about twice a deeper one (it pays the level-0 binning: config 4 spends 36 ms on
# 1B level-0 arrivals and 38 ms on 2B deeper ones), and a point arrives at about
# DEPTH deeper levels.  Config 3 averages 3.3 (W / N = 4.3), but its heavy cells
# are the dense ones and go deeper (W / N of the four largest: 4.0-4.9), and an
# unsplit heavy cell is what sets the critical path, so the plan uses 4.
L0_COST, DEEP_COST, DEPTH = 2.0, 1.0, 4.0


def _lpt(w: np.ndarray, world: int):
    """Largest-first greedy: item i (weight w[i], ties by index) to the least
    loaded rank (ties by rank).  Deterministic on every rank."""
    return pcconv.shard_lpt(w, world)   # C++ (pcc_shard_lpt): the plan tries up to 2 * world + 1 of these


@dataclass
class SplitPlan:
    """Who builds what in one sharded step.

    Whole level-0 cells: owner0[c] builds the cell's sub-tree (phase 1).  A
    split cell c (split[c]) is shared: its level-0 slabs (cell, hex z-layer) go
    to slab_owner[c * SHARD_LAYERS + layer], which resolve their slots and
    forward every emission (phase 1, raw level 0); each level-1 cell c1 below
    it goes to owner1[c1], which resolves that overflow bucket (cell.rs:108-153)
    from all ranks' emissions and builds the sub-tree if it spilled (phase 2);
    writer[c] assembles the level-0 cell file from the pieces."""
    owner0: np.ndarray
    split: np.ndarray
    slab_owner: np.ndarray | None = None
    writer: np.ndarray | None = None
    owner1: np.ndarray | None = None
    est: dict = field(default_factory=dict)


def plan_split(hist0: np.ndarray, hist1: np.ndarray | None, children: np.ndarray | None, world: int,
               slab_hist: np.ndarray | None = None, allow: bool = True) -> SplitPlan:
    """Choose the level-0 cells to share (largest first) so that the estimated
    critical path max(phase 1) + max(phase 2) is smallest; without a gain of
    more than 2 % nothing is shared and this is `assign_owners`.  children[c]:
    the level-1 grid ids of cell c's 8 children (-1: outside the grid);
    slab_hist: points per (cell, layer), SHARD_LAYERS per cell."""
    from pcconv import SHARD_LAYERS as NL
    hist0 = np.asarray(hist0, dtype=np.int64)
    nz = np.flatnonzero(hist0)
    base = assign_owners(hist0, world)
    whole_w = hist0 * (L0_COST + DEEP_COST * DEPTH)
    total = float(whole_w.sum())
    mean = total / max(world, 1)
    no = SplitPlan(base, np.zeros(len(hist0), dtype=bool))
    lb = np.zeros(world)
    for c in nz:
        lb[base[c]] += whole_w[c]
    no.est = {"phase1_max": float(lb.max()) if world else 0.0, "phase2_max": 0.0,
              "ratio": float(lb.max() / mean) if mean else 1.0, "split_cells": 0}
    if not allow or world <= 1 or hist1 is None or slab_hist is None or len(nz) == 0 or len(nz) > 4096:
        return no
    sh = np.asarray(slab_hist, dtype=np.int64).reshape(len(hist0), NL)
    order = nz[np.lexsort((nz, -hist0[nz]))]
    kmax = min(len(order), 2 * world)
    # per candidate that may be shared (the kmax heaviest): its slabs (cell * NL
    # + layer, non-empty layers ascending) and its non-empty level-1 children
    # (octant order)
    slabs = [c * NL + np.flatnonzero(sh[c]) for c in order[:kmax]]
    kids = []
    for c in order[:kmax]:
        q = children[c]
        q = q[q >= 0]
        kids.append(q[hist1[q] > 0])
    slab_off = np.concatenate([[0], np.cumsum([len(a) for a in slabs])]).astype(np.uint64)
    child_off = np.concatenate([[0], np.cumsum([len(a) for a in kids])]).astype(np.uint64)
    sl_all = np.concatenate(slabs).astype(np.int64)
    ch_all = np.concatenate(kids).astype(np.int64) if kids else np.zeros(0, np.int64)
    # the search over k (C++, pcc_shard_plan_search): phase 1 = the whole cells
    # and the shared cells' level-0 slabs, phase 2 = the shared cells' level-1
    # sub-trees, both placed largest first
    # and the best k's placement, the LPT of its two lists
    k, best_t, ow, osl, och, l1, l2 = pcconv.shard_plan_search(
        whole_w[order].astype(np.float64), slab_off, sh.reshape(-1)[sl_all] * L0_COST, child_off,
        hist1[ch_all] * DEEP_COST * DEPTH, kmax, world, owners=True)
    if k == 0:
        return no
    sp, whole = order[:k], order[k:]
    sl = sl_all[:int(slab_off[k])]
    o1 = np.concatenate([ow[k:], osl[:len(sl)]])
    ch = ch_all[:int(child_off[k])]
    o2 = och[:len(ch)]
    owner0 = np.zeros(len(hist0), dtype=np.uint32)
    split = np.zeros(len(hist0), dtype=bool)
    split[sp] = True
    owner0[whole] = o1[:len(whole)]
    slab_owner = np.zeros(len(hist0) * NL, dtype=np.uint32)
    slab_owner[sl] = o1[len(whole):]
    writer = np.zeros(len(hist0), dtype=np.uint32)
    for c in sp:   # the rank holding most of the cell's points
        w = np.bincount(slab_owner[c * NL:(c + 1) * NL], weights=sh[c], minlength=world)
        writer[c] = int(np.argmax(w))
    owner1 = np.zeros(len(hist1), dtype=np.uint32)
    owner1[ch] = o2
    return SplitPlan(owner0, split, slab_owner, writer, owner1,
                     {"phase1_max": float(l1.max()), "phase2_max": float(l2.max()) if len(ch) else 0.0,
                      "ratio": best_t / mean, "split_cells": int(len(sp))})


def route_table(plan: SplitPlan, world: int) -> np.ndarray:
    """Destination of every level-0 slab for the route (SHARD_LAYERS per cell):
    rank r for a whole cell's points, r + world for a shared cell's slab."""
    from pcconv import SHARD_LAYERS as NL
    t = np.repeat(plan.owner0.astype(np.int64), NL)
    sp = np.repeat(plan.split, NL)
    t[sp] = plan.slab_owner.astype(np.int64)[sp] + world
    return t


# ----------------------------------------------------------------- shared cells: bucket resolution
def event_batches(keys: np.ndarray, file_points, batch: int) -> np.ndarray:
    """Event batch of each global key (lib.rs:31-52: files in CLI order, batches
    of `batch`, a file end is a batch boundary, an empty file one empty batch)."""
    fp = np.asarray([int(v) for v in file_points], dtype=np.int64)
    start = np.concatenate([[0], np.cumsum(fp)])[:-1]
    nb = np.maximum(1, (fp + batch - 1) // batch)
    eb0 = np.concatenate([[0], np.cumsum(nb)])[:-1]
    k = np.asarray(keys, dtype=np.int64)
    f = np.searchsorted(start, k, side="right") - 1   # last file whose start <= key
    return eb0[f] + (k - start[f]) // batch


def global_batches(file_points, batch: int):
    """(start key of every non-empty global batch, its event batch number, the
    global batch count): lib.rs:31-52, an empty file is one empty batch.  Keys
    are 64-bit: any cloud size."""
    fp = np.asarray([int(v) for v in file_points], dtype=np.int64)
    start = np.concatenate([[0], np.cumsum(fp)])[:-1]
    nb = np.maximum(1, (fp + batch - 1) // batch)
    eb0 = np.concatenate([[0], np.cumsum(nb)])[:-1]
    full = (fp + batch - 1) // batch   # batches holding points
    f = np.repeat(np.arange(len(fp)), full)
    b = np.arange(int(full.sum()), dtype=np.int64) - np.repeat(np.concatenate([[0], np.cumsum(full)])[:-1], full)
    return (start[f] + b * batch).astype(np.uint64), (eb0[f] + b).astype(np.int64), int(nb.sum())


def event_table(local_starts: np.ndarray, batch_no: np.ndarray, nrecv: int, total: int):
    """The rank-local event table (pcc_set_event_table) from the local start of
    every non-empty global batch: the batches with some of this rank's points."""
    ls = np.asarray(local_starts, dtype=np.int64)
    nxt = np.concatenate([ls[1:], [nrecv]])
    keep = ls < nxt
    return ls[keep].astype(np.uint64), np.asarray(batch_no)[keep].astype(np.uint32), int(total)


def resolve_bucket(keys: np.ndarray, file_points, batch: int, limit: int):
    """cell.rs:108-153 for one overflow bucket of a level-0 cell, from all its
    emissions (their causing keys, any order; level 0: event batch = eb0(key)).
    Returns (spilled, spill batch, key order).  Batch by batch: the first batch's
    list is kept if it has at most L points, later batches are appended while
    the list stays below L; otherwise the bucket turns None at that batch and
    everything is forwarded (the kept points at that batch)."""
    order = np.argsort(np.asarray(keys, dtype=np.int64), kind="stable")
    if len(order) == 0:
        return False, 0, order
    eb = event_batches(np.asarray(keys)[order], file_points, batch)
    tot = len(eb)
    spilled = tot > limit or (tot == limit and eb[0] != eb[-1])
    if not spilled:
        return False, 0, order
    first = int(np.count_nonzero(eb == eb[0]))
    thr = limit + (1 if first == limit else 0)
    return True, int(eb[max(thr, 1) - 1]), order


def children_ids(ids0: np.ndarray, grid0, grid1) -> np.ndarray:
    """(n, 8) level-1 grid ids of the children of level-0 cells (-1 outside grid1);
    the level-1 index of a point is 2 x its level-0 index + 0/1 per axis
    (metadata.rs:91-102: cell sizes are power-of-two scalings)."""
    t = cell_triples(ids0, grid0).astype(np.int64)
    lo1 = np.array([int(v) for v in grid1.lo], dtype=np.int64)
    d1 = np.array([int(v) for v in grid1.dims], dtype=np.int64)
    out = np.full((len(t), 8), -1, dtype=np.int64)
    for o in range(8):
        q = 2 * t + np.array([o & 1, (o >> 1) & 1, (o >> 2) & 1]) - lo1
        ok = ((q >= 0) & (q < d1)).all(axis=1)
        out[ok, o] = (q[ok, 0] * d1[1] + q[ok, 1]) * d1[2] + q[ok, 2]
    return out


def level1_ids(xyz: np.ndarray, grid1) -> np.ndarray:
    lo1 = np.array([int(v) for v in grid1.lo], dtype=np.int64)
    d1 = np.array([int(v) for v in grid1.dims], dtype=np.int64)
    q = np.asarray(xyz, dtype=np.int64).reshape(-1, 3) - lo1
    if not ((q >= 0) & (q < d1)).all():
        raise ValueError("exported level-1 cell outside the level-1 grid")
    return (q[:, 0] * d1[1] + q[:, 1]) * d1[2] + q[:, 2]


def cell_ids(xyz: np.ndarray, grid) -> np.ndarray:
    """Linear shard-grid ids of level-0 cells (x, y, z)."""
    lo = np.array([int(v) for v in grid.lo], dtype=np.int64)
    d = np.array([int(v) for v in grid.dims], dtype=np.int64)
    q = np.asarray(xyz, dtype=np.int64).reshape(-1, 3) - lo
    if not ((q >= 0) & (q < d)).all():
        raise ValueError("cell outside the shard grid")
    return (q[:, 0] * d[1] + q[:, 1]) * d[2] + q[:, 2]


def _exchange_segments(comm, dest: np.ndarray, meta: np.ndarray, lens: np.ndarray, tensors: list, dev):
    """Segment i (metadata row meta[i]; lens[i] rows of every tensor, the
    segments contiguous in order) to rank dest[i].  Returns the received
    metadata rows and tensors: source rank by source rank, each source's
    segments in its sending order, rows of a segment in their order."""
    W = comm.world
    dest = np.asarray(dest, dtype=np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    meta = np.asarray(meta, dtype=np.int64)
    k = meta.shape[1] if meta.ndim == 2 else (meta.size // len(dest) if len(dest) else 1)
    meta = meta.reshape(len(dest), k)   # (no segments: 0 rows of k, not reshape(0, -1))
    order = np.argsort(dest, kind="stable")
    if len(order) and not np.array_equal(order, np.arange(len(order))):
        starts = np.concatenate([[0], np.cumsum(lens)])[:-1]
        ls, ss = lens[order], starts[order]
        idx = torch.from_numpy(np.repeat(ss - (np.cumsum(ls) - ls), ls) + np.arange(int(ls.sum()), dtype=np.int64))
        tensors = [t.index_select(0, idx.to(t.device)) for t in tensors]
    nseg = [int(v) for v in np.bincount(dest, minlength=W)] if len(dest) else [0] * W
    nrow = [int(v) for v in np.bincount(dest, weights=lens, minlength=W).astype(np.int64)] if len(dest) else [0] * W
    mt = torch.from_numpy(np.ascontiguousarray(meta[order]).reshape(-1, k)).to(comm.device)
    rmeta = _exchange(comm, mt, nseg, comm.alltoall_counts(nseg), comm.device).cpu().numpy().reshape(-1, k)
    rr = comm.alltoall_counts(nrow)
    return rmeta, [_exchange(comm, t, nrow, rr, dev) for t in tensors]


def resolve_level1(rmeta: np.ndarray, pts: torch.Tensor, keys: torch.Tensor, file_points, batch: int, limit: int):
    """Owner side of a shared cell's overflow buckets.  rmeta rows (x, y, z, n):
    segments of emissions (pts/keys, in order) of level-1 cells; one cell can
    come in several segments (one per rank holding slabs of its parent).  Each
    cell is the bucket of its level-0 parent for that octant (converter.rs:67-68):
    resolve it over all its emissions (resolve_bucket).  Returns the spilled
    cells' emissions (the sub-tree input, roots with their spill batches), and
    per bucket a row (x, y, z, state 1 = Some / 2 = None, n) with the kept
    lists (key order) of the Some buckets."""
    rmeta = np.asarray(rmeta, dtype=np.int64).reshape(-1, 4)
    starts = np.concatenate([[0], np.cumsum(rmeta[:, 3])])[:-1]
    groups = {}
    for i, row in enumerate(rmeta):
        if row[3]:
            groups.setdefault(tuple(int(v) for v in row[:3]), []).append(i)
    kh = keys.cpu().numpy().view(np.uint32).astype(np.int64) if len(groups) else np.zeros(0, np.int64)
    sub_idx, roots, sbs, rows, kept_idx = [], [], [], [], []
    for c1 in sorted(groups):
        idx = np.concatenate([np.arange(starts[i], starts[i] + rmeta[i, 3]) for i in groups[c1]])
        spilled, sb, order = resolve_bucket(kh[idx], file_points, batch, limit)
        if spilled:
            sub_idx.append(idx)
            roots.append(c1)
            sbs.append(sb)
            rows.append([*c1, 2, len(idx)])
        else:
            kept_idx.append(idx[order])
            rows.append([*c1, 1, len(idx)])
    dev = pts.device

    def take(lst, t):
        if not lst:
            return t[:0]
        return t.index_select(0, torch.from_numpy(np.concatenate(lst)).to(dev))
    return {"sub_pts": take(sub_idx, pts), "sub_keys": take(sub_idx, keys),
            "roots_xyz": np.array(roots, dtype=np.int32).reshape(-1, 3), "roots_sb": np.array(sbs, dtype=np.uint32),
            "bucket_rows": np.array(rows, dtype=np.int64).reshape(-1, 5), "kept_pts": take(kept_idx, pts)}


def assemble_cells(rmw: np.ndarray, grid_pts: torch.Tensor, rmk: np.ndarray, kept_pts: torch.Tensor, cfg: dict):
    """Writer side: the level-0 cells this rank assembles from their pieces --
    grid winners of every rank's slabs (rmw rows (x, y, z, n) over grid_pts) and
    the bucket rows (x1, y1, z1, state, n) of their octants with the Some lists
    (kept_pts, in row order).  Header as cell.rs:43-49, 264-274: size =
    cell_size(0), sub = size / dim, pos = index * size + size / 2; number = grid
    points, overflow = kept points, total = their sum."""
    rmw = np.asarray(rmw, dtype=np.int64).reshape(-1, 4)
    rmk = np.asarray(rmk, dtype=np.int64).reshape(-1, 5)
    g = grid_pts.cpu().numpy().reshape(-1, 4).astype(np.int32, copy=False)
    kp = kept_pts.cpu().numpy().reshape(-1, 4).astype(np.int32, copy=False)
    cells = {}
    o = 0
    for x, y, z, n in rmw:
        c = cells.setdefault((int(x), int(y), int(z)), {"grid": [], "buckets": {}})
        c["grid"].append(g[o:o + n])
        o += int(n)
    o = 0
    for x1, y1, z1, st, n in rmk:
        cnt = int(n) if st == 1 else 0
        c = cells.setdefault((int(x1) >> 1, int(y1) >> 1, int(z1) >> 1), {"grid": [], "buckets": {}})
        c["buckets"][(int(x1), int(y1), int(z1))] = (int(st), kp[o:o + cnt])
        o += cnt
    f32 = np.float32
    size = f32(cfg["max_cell_size"]) / f32(1.0)
    sub = size / f32(cfg["sub_grid_dimension"])
    out = []
    for (x, y, z), c in sorted(cells.items()):
        entries = []
        for oc in range(8):   # octant order, as the engine's cells
            c1 = (2 * x + (oc & 1), 2 * y + ((oc >> 1) & 1), 2 * z + ((oc >> 2) & 1))
            if c1 in c["buckets"]:
                entries.append((c1,) + c["buckets"][c1])
        grid = np.concatenate(c["grid"]) if c["grid"] else np.zeros((0, 4), np.int32)
        out.append({"h": 0, "xyz": (x, y, z), "grid": np.ascontiguousarray(grid), "entries": entries,
                    "size": size, "sub": sub,
                    "pos": [f32(v) * size + size / f32(2.0) for v in (x, y, z)]})
    return out


class AssembledCells:
    """The level-0 cells a writer assembles (assemble_cells), kept as their
    pieces -- host rows of counts plus the received grid / kept tensors, on the
    device -- until the cells are walked or written; iterating materialises
    them once (one device-to-host copy of each tensor)."""

    def __init__(self, rmw, grid_pts: torch.Tensor, rmk, kept_pts: torch.Tensor, cfg: dict):
        self.rmw = np.asarray(rmw, dtype=np.int64).reshape(-1, 4)
        self.rmk = np.asarray(rmk, dtype=np.int64).reshape(-1, 5)
        self.grid_pts, self.kept_pts, self.cfg = grid_pts, kept_pts, cfg
        self._cells = None
        xyz = np.concatenate([self.rmw[:, :3], self.rmk[:, :3] >> 1])
        self._n = len(np.unique(xyz, axis=0)) if len(xyz) else 0

    def __len__(self):
        return self._n

    def __iter__(self):
        if self._cells is None:
            self._cells = assemble_cells(self.rmw, self.grid_pts, self.rmk, self.kept_pts, self.cfg)
            self.grid_pts = self.kept_pts = None
        return iter(self._cells)


def cell_view(c: dict):
    """pcc_cell_view of an assembled cell (the arrays must outlive the view)."""
    v = pcconv.CellView()
    v.hierarchy = c["h"]
    v.x, v.y, v.z = c["xyz"]
    v.number_of_points = len(c["grid"])
    over = sum(len(p) for _, st, p in c["entries"] if st == 1)
    v.number_of_overflow_points = over
    v.total_number_of_points = v.number_of_points + over
    v.size, v.sub_cell_size = float(c["size"]), float(c["sub"])
    for a in range(3):
        v.pos[a] = float(c["pos"][a])
    v.grid = c["grid"].ctypes.data if len(c["grid"]) else None
    v.entries = len(c["entries"])
    for i, (c1, st, p) in enumerate(c["entries"]):
        for a in range(3):
            v.child[i][a] = c1[a]
        v.count[i] = len(p) if st == 1 else 0
        v.list[i] = p.ctypes.data if (st == 1 and len(p)) else None
    return v


def shard_grid(gmin, gmax, max_cell_size: float, level: int = 0):
    """The unit grid of ownership.  Level 0: the level-0 cells spanned by the
    global bbox; when that grid exceeds the 2^22 cells pcc_shard_grid_from_bbox
    allows (a sparse, widely spread cloud), cells of 2^k x the size, k smallest
    that fits: floor(p / (cs 2^k)) = floor(p / cs) >> k exactly (power-of-two
    scaling), so a coarse cell is a block of whole level-0 cells and every
    level-0 sub-tree still has one owner (`grid.coarse` = k; cells are not
    shared then).  Level 1 (cell sharing): None when too large."""
    cs = max_cell_size / float(1 << level)
    if level > 0:
        try:
            g = pcconv.shard_grid_from_bbox(gmin, gmax, cs)
        except pcconv.PccError:
            return None
        g.coarse = 0
        return g
    for k in range(0, 24):
        try:
            g = pcconv.shard_grid_from_bbox(gmin, gmax, cs * float(1 << k))
        except pcconv.PccError as e:
            if e.code != -27:   # -EFBIG: grid too large, try coarser cells
                raise
            continue
        g.coarse = k
        return g
    raise ValueError("bounding box too large for the shard grid")


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
            self.conv_lead = self.conv_sub = None
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
        # split cells: level 0 as their leader, level-1 sub-trees as their owner
        self.conv_lead = pcconv.Converter(out_dir, batch_size=batch_size, device=device_index, config=self.cfg)
        self.conv_lead.set_level_range(0, 1, raw=True)
        self.conv_sub = pcconv.Converter(out_dir, batch_size=batch_size, device=device_index, config=self.cfg)
        self.conv_sub.set_level_range(1, 0)

    def prior_meta(self) -> dict:
        return read_prior_meta(self.out_dir)

    def set_subtrees(self, cells: np.ndarray):
        """Merge mode: (re)open the existing cloud restricted to these level-0 cells."""
        cells = np.asarray(cells, dtype=np.int32).reshape(-1, 3)
        if self.conv is not None and self.subtrees is not None and np.array_equal(cells, self.subtrees):
            return
        if self.conv is not None:
            self.conv.close()
            # the closed converter's buffers would sit in the library's device
            # cache, invisible to PyTorch's allocator and RCCL
            pcconv.release_device_cache()
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

    def bbox_nonfinite(self, pts: torch.Tensor) -> list:
        self._ready()
        return pcconv.shard_bbox_nonfinite(pts.data_ptr(), pts.shape[0], self.dev)

    def grid(self, gmin, gmax, level: int = 0):
        return shard_grid(gmin, gmax, self.max_cell_size, level)

    # the bounding box and the slab histogram in one pass over a guessed grid
    fused_bbox_hist = True

    def bbox_sample(self, pts: torch.Tensor):
        self._ready()
        return pcconv.shard_bbox_sample(pts.data_ptr(), pts.shape[0], self.dev)

    def bbox_slab_histogram(self, pts: torch.Tensor, guess):
        """(bmin, bmax, slab histogram over `guess`, points outside `guess`)."""
        h = torch.empty(guess.ncells * pcconv.SHARD_LAYERS, dtype=torch.int32, device=pts.device)
        self._ready()
        r = pcconv.shard_bbox_histogram(pts.data_ptr(), pts.shape[0], guess,
                                        int(self.cfg_full()["sub_grid_dimension"]), h.data_ptr(), self.dev)
        if r is None:   # NaN / infinite coordinates
            return None
        return r[0], r[1], h, r[2]

    def begin_step(self):
        self._built = []
        self.assembled = []

    def cfg_full(self) -> dict:
        d = dict(cell_point_overflow_limit=5000, sub_grid_dimension=96, max_cell_size=1000.0)
        d.update(self.cfg)
        return d

    @property
    def limit(self) -> int:
        return int(self.cfg_full()["cell_point_overflow_limit"])

    def set_assembled(self, cells: list):
        self.assembled = cells

    def slab_histogram(self, pts: torch.Tensor, grid) -> torch.Tensor:
        h = torch.empty(grid.ncells * pcconv.SHARD_LAYERS, dtype=torch.int32, device=pts.device)
        self._ready()
        pcconv.shard_slab_histogram(pts.data_ptr(), pts.shape[0], grid, int(self.cfg_full()["sub_grid_dimension"]),
                                    h.data_ptr(), self.dev)
        return h

    def route_slabs(self, pts: torch.Tensor, key0: int, grid, table: torch.Tensor, nranks: int):
        n = pts.shape[0]
        send = torch.empty_like(pts)
        keys = torch.empty(n, dtype=torch.int32, device=pts.device)
        self._ready()
        counts = pcconv.shard_route_slabs(pts.data_ptr(), n, key0, grid, int(self.cfg_full()["sub_grid_dimension"]),
                                          table.data_ptr(), nranks, send.data_ptr(), keys.data_ptr(), self.dev)
        return send, keys, counts

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

    # the exchange carries membership bitmaps instead of keys (route_bitmaps / keys_from_bitmaps)
    bitmap_keys = True
    # build() returns the bounding box of the points it built (pcc_get_stats)
    build_reports_bbox = True

    def route_bitmaps(self, pts: torch.Tensor, grid, table: torch.Tensor, nranks: int, slabs: bool,
                      hist: torch.Tensor | None = None):
        """(send, bitmaps (nranks, ceil(n/64)) int64, counts): pcc_shard_route_bitmaps
        on cell units (table = owner per cell) or slab units (table per slab).
        hist: this rank's points per unit of the same kind (the local histogram
        the plan was made from) -> the one-pass form, pcc_shard_route_bitmaps_hist."""
        n = pts.shape[0]
        send = torch.empty_like(pts)
        bm = torch.empty((nranks, (n + 63) // 64), dtype=torch.int64, device=pts.device)
        if hist is not None:
            hist = hist.to(device=pts.device, dtype=torch.int32).contiguous()
        self._ready()   # after every torch op on the inputs
        dim = int(self.cfg_full()["sub_grid_dimension"]) if slabs else 0
        if hist is not None:
            counts = pcconv.shard_route_bitmaps_hist(pts.data_ptr(), n, grid, dim, table.data_ptr(), nranks,
                                                     hist.data_ptr(), send.data_ptr(), bm.data_ptr(), self.dev)
        else:
            counts = pcconv.shard_route_bitmaps(pts.data_ptr(), n, grid, dim, table.data_ptr(), nranks,
                                                send.data_ptr(), bm.data_ptr(), self.dev)
        return send, bm, counts

    # builds with rank-local keys and an event table (shard_build, no shared cell)
    local_keys = True

    def batch_starts(self, bm: torch.Tensor, nwords, key0, gstarts) -> np.ndarray:
        self._ready()
        return pcconv.shard_batch_starts(bm.data_ptr(), nwords, key0, gstarts, self.dev)

    def keys_from_bitmaps(self, bm: torch.Tensor, nwords, key0, nkeys: int) -> torch.Tensor:
        keys = torch.empty(nkeys, dtype=torch.int32, device=bm.device)
        self._ready()
        pcconv.shard_keys_from_bitmaps(bm.data_ptr(), nwords, key0, keys.data_ptr(), nkeys, self.dev)
        return keys

    def build(self, file_points, pts: torch.Tensor, keys: torch.Tensor | None, etab=None) -> dict:
        """keys None: this rank holds the whole input in key order (keys 0..n-1),
        or, with etab (event_table), its points in global key order with
        rank-local keys.  The build reads `pts`/`keys` in place (borrowed until
        it returns)."""
        self.landing_active = False
        self._record("build", (file_points, pts, keys, etab), first=True)
        return self._keyed_build(self.conv, file_points, pts, keys, etab=etab)

    # the exchange lands the points in this many rounds, level-0 pass 1 running
    # behind each (pcc_input_landed); 0 or 1: one exchange, then the build
    landing_rounds = int(os.environ.get("PCC_LAND_ROUNDS", "4"))
    landing_active = False

    def begin_landing(self, file_points, recv: torch.Tensor, etab):
        """Borrow `recv` (rank-local keys, etab) before the exchange fills it."""
        self._ready()
        c = self.conv
        c.clear_input()
        c.set_event_table(*etab)
        c.set_keyed_points_device(recv.data_ptr(), 0, recv.shape[0])
        self.landing_active = True
        self._landing = (file_points, recv, etab, c)

    def landed(self, ranges, stream: int):
        """Row ranges of the borrowed input that the exchange's work queued on
        `stream` so far writes: pass 1 of the groups they complete queues behind."""
        c = self._landing[3]
        for a, b in ranges:
            c.input_landed(a, b, stream)

    def build_landed(self) -> dict:
        file_points, recv, etab, c = self._landing
        self._landing = None
        self.landing_active = False
        self._record("build", (file_points, recv, None, etab), first=True)
        self._ready()
        st = c.build()
        if c not in getattr(self, "_built", []):
            self._built = getattr(self, "_built", []) + [c]
        return st

    # Diagnostics only (scripts/rank_stages.py replays a step's local calls): with
    # record_inputs set, every stage's device inputs are kept in last_inputs until
    # the next step or close().  Off in the product: they would hold GBs of
    # device memory per rank into the next step's exchange.
    record_inputs = False

    def _record(self, stage, args, first=False):
        if not self.record_inputs:
            return
        if first or not hasattr(self, "last_inputs"):
            self.last_inputs = {}
        self.last_inputs[stage] = args

    def _keyed_build(self, c, file_points, pts, keys, roots=None, etab=None) -> dict:
        self._ready()
        c.clear_input()
        if etab is not None:
            c.set_event_table(*etab)
        else:
            c.declare_files(file_points)
        if roots is not None:
            c.set_root_spill_batches(*roots)
        c.set_keyed_points_device(pts.data_ptr(), 0 if keys is None else keys.data_ptr(), pts.shape[0])
        st = c.build()
        if c not in getattr(self, "_built", []):
            self._built = getattr(self, "_built", []) + [c]
        return st

    def lead_build_raw(self, file_points, pts: torch.Tensor, keys: torch.Tensor):
        """Level 0 of the shared cells' slabs this rank holds, raw (every emission
        forwarded).  Returns (stats, (level-1 cells (n,3), -, points per cell,
        their emissions (m,4), causing keys), partial level-0 cells [{xyz, grid}])."""
        c = self.conv_lead
        self._record("lead", (file_points, pts, keys))
        st = self._keyed_build(c, file_points, pts, keys)
        _, m = c.pending_cells()
        P = torch.empty((m, 4), dtype=torch.int32, device=pts.device)
        K = torch.empty(m, dtype=torch.int32, device=pts.device)
        xyz, sb, cn = c.export_pending(P.data_ptr(), K.data_ptr())
        # the partial level-0 cells' grid winners stay on the device (pcc_export_grid)
        _, ng = c.grid_cells()
        G = torch.empty((ng, 4), dtype=torch.int32, device=pts.device)
        self._ready()   # G's block may have been freed by pending torch work
        pxyz, pn = c.export_grid(G.data_ptr())
        return st, (xyz, sb, cn, P, K), (pxyz.astype(np.int64), pn.astype(np.int64), G)

    def resolve_level1(self, rmeta: np.ndarray, pts: torch.Tensor, keys: torch.Tensor, file_points) -> dict:
        """Module resolve_level1 on the device (pcc_shard_resolve_buckets): the
        same outputs, with only the segment table and the bucket states crossing
        to the host."""
        self._record("resolve", (rmeta, pts, keys, file_points))
        rmeta = np.asarray(rmeta, dtype=np.int64).reshape(-1, 4)
        rmeta = rmeta[rmeta[:, 3] > 0]   # empty segments carry no rows
        dev = pts.device
        if not len(rmeta):
            return {"sub_pts": pts[:0], "sub_keys": keys[:0], "roots_xyz": np.zeros((0, 3), np.int32),
                    "roots_sb": np.zeros(0, np.uint32), "bucket_rows": np.zeros((0, 5), np.int64),
                    "kept_pts": pts[:0]}
        cells, inv = np.unique(rmeta[:, :3], axis=0, return_inverse=True)   # sorted (x, y, z) as the numpy statement
        inv = inv.reshape(-1)
        nrow = int(rmeta[:, 3].sum())
        if nrow != int(pts.shape[0]) or nrow != int(keys.shape[0]):
            raise ValueError("segment rows do not match the received emissions")
        kept = torch.empty((nrow, 4), dtype=torch.int32, device=dev)
        sub = torch.empty((nrow, 4), dtype=torch.int32, device=dev)
        subk = torch.empty(nrow, dtype=torch.int32, device=dev)
        self._ready()
        st, sb, _, nk, ns = pcconv.shard_resolve_buckets(rmeta[:, 3], inv, len(cells), pts.data_ptr(),
                                                         keys.data_ptr(), file_points, self.batch_size, self.limit,
                                                         kept.data_ptr(), sub.data_ptr(), subk.data_ptr(), self.dev)
        tot = np.bincount(inv, weights=rmeta[:, 3], minlength=len(cells)).astype(np.int64)
        spilled = st == 2
        rows = np.column_stack([cells, st.astype(np.int64), tot]).astype(np.int64).reshape(-1, 5)
        return {"sub_pts": sub[:ns], "sub_keys": subk[:ns], "roots_xyz": cells[spilled].astype(np.int32).reshape(-1, 3),
                "roots_sb": sb[spilled].astype(np.uint32), "bucket_rows": rows, "kept_pts": kept[:nk]}

    def sub_build(self, file_points, pts: torch.Tensor, keys: torch.Tensor, cells_xyz, spill_batch) -> dict:
        """The level-1 sub-trees of split cells this rank owns (their arrivals, cell
        after cell, from the leaders' pcc_export_pending)."""
        self._record("sub", (file_points, pts, keys, cells_xyz, spill_batch))
        return self._keyed_build(self.conv_sub, file_points, pts, keys, roots=(cells_xyz, spill_batch))

    def _outputs(self):
        # the raw level-0 pieces of shared cells are written by their assemblers
        return [self.conv] + [c for c in getattr(self, "_built", []) if c is not self.conv and c is not self.conv_lead]

    def visit_cells(self, fn):
        """pcc_visit_cells over every converter built in the last step, then the
        shared level-0 cells this rank assembled."""
        for c in self._outputs():
            c.visit_cells(fn)
        for cell in getattr(self, "assembled", []):
            v = cell_view(cell)
            fn(C.addressof(v))

    def write(self, summary: dict, cells: bool, metadata: bool):
        convs = self._outputs()
        for c in convs:
            c.set_summary(summary["number_of_points"], summary["bbox_min"], summary["bbox_max"],
                          summary["hierarchies"])
        if cells:
            for c in convs:
                c.write_cells()
            for cell in getattr(self, "assembled", []):
                pcconv.write_cell_view(self.out_dir, cell_view(cell))
        if metadata:
            self.conv.write_metadata()

    def close(self):
        for c in (self.conv, getattr(self, "conv_lead", None), getattr(self, "conv_sub", None)):
            if c is not None:
                c.close()
        self.conv = self.conv_lead = self.conv_sub = None
        self.last_inputs = {}
        # the library's device cache is invisible to PyTorch's allocator and RCCL
        pcconv.release_device_cache()
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
    sub_points: int = 0          # level-1 arrivals received for split cells' sub-trees
    plan: dict = field(default_factory=dict)   # plan_split's estimate
    assembled_cells: int = 0     # shared level-0 cells this rank assembled and wrote


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


def _move(comm, t: torch.Tensor, dev) -> torch.Tensor:
    """t on `dev`; a communicator may do (and time) the staging copies itself."""
    return comm.move(t, dev) if hasattr(comm, "move") else t.to(dev)


def _exchange(comm, send: torch.Tensor, counts, rcounts, dev) -> torch.Tensor:
    """All-to-all-v of rows into a new tensor on `dev` (straight into it when the
    communicator works on that device, else through the communicator's device)."""
    n = int(sum(int(v) for v in rcounts))
    if comm.device == dev:
        out = torch.empty((n,) + tuple(send.shape[1:]), dtype=send.dtype, device=dev)
        return comm.alltoallv_into(send, counts, rcounts, out)
    out = torch.empty((n,) + tuple(send.shape[1:]), dtype=send.dtype, device=comm.device)
    comm.alltoallv_into(_move(comm, send, comm.device), counts, rcounts, out)
    return _move(comm, out, dev)


def _exchange_many(comm, specs, dev) -> list:
    """Several all-to-all-v exchanges (send, counts, recv counts) in one grouped
    batch when the communicator offers it (alltoallv_many), else one by one."""
    outs = []
    for send, counts, rcounts in specs:
        n = int(sum(int(v) for v in rcounts))
        outs.append(torch.empty((n,) + tuple(send.shape[1:]), dtype=send.dtype, device=comm.device))
    sends = [sp[0] if comm.device == dev else _move(comm, sp[0], comm.device) for sp in specs]
    if hasattr(comm, "alltoallv_many"):
        comm.alltoallv_many([(sd, sp[1], sp[2], o) for sd, sp, o in zip(sends, specs, outs)])
    else:
        for sd, sp, o in zip(sends, specs, outs):
            comm.alltoallv_into(sd, sp[1], sp[2], o)
    return [o if comm.device == dev else _move(comm, o, dev) for o in outs]


def _combine(parts: list[dict]) -> dict:
    out = dict(parts[-1])
    for k in ("arrivals", "cells", "slabs"):
        if all(k in p for p in parts):
            out[k] = sum(int(p[k]) for p in parts)
    for k in ("hierarchies", "levels"):
        if all(k in p for p in parts):
            out[k] = max(int(p[k]) for p in parts)
    return out


def _sub_grid_hist(h, guess, grid, nl: int):
    """The slab histogram over `guess` restricted to `grid` (a sub-box of it;
    cell id = ((ix - lo.x) dims.y + iy - lo.y) dims.z + iz - lo.z), or None when
    `grid` is not inside `guess`."""
    o = [int(grid.lo[a]) - int(guess.lo[a]) for a in range(3)]
    d, dg = [int(v) for v in grid.dims], [int(v) for v in guess.dims]
    if any(o[a] < 0 or o[a] + d[a] > dg[a] for a in range(3)):
        return None
    v = h.view(dg[0], dg[1], dg[2], nl)
    return v[o[0]:o[0] + d[0], o[1]:o[1] + d[1], o[2]:o[2] + d[2]].contiguous().view(-1)


def _attempt(fn, fallback):
    """(fn(), None), or (fallback, the exception) when this rank's local pass fails."""
    try:
        return fn(), None
    except Exception as e:  # noqa: BLE001 (re-raised by _raise_together after the collective)
        return fallback, e


def _raise_together(err, flag: float, stage: str):
    """After a collective carrying every rank's error flag: this rank's own error,
    or an error naming the stage another rank failed in."""
    if err is not None:
        raise err
    if flag > 0:
        raise RuntimeError(f"shard_build: another rank failed in its {stage} pass")


def _fmin(a: float, b: float) -> float:   # f32::min (glam Vec3::min): a NaN operand is skipped
    return b if a != a else (a if b != b else min(a, b))


def _fmax(a: float, b: float) -> float:
    return b if a != a else (a if b != b else max(a, b))


def shard_build(comm, ops, pts: torch.Tensor, key0: int, file_points, write: bool = False,
                sync=None, merge: bool = False, split: bool = True) -> ShardResult:
    """One sharded conversion step.  `pts` is this rank's (n, 4) int32 view of
    16-B points with global keys key0 .. key0+n-1 (contiguous ranges in rank
    order).  `file_points` is the GLOBAL file structure.  `sync` (optional)
    synchronises the device for stage timing.  `merge`: incremental merge into
    the existing cloud of the ops' directory (module docstring).  `split`: allow
    heavy level-0 cells to be shared at level 1 (plan_split; never for a merge)."""
    ms = {}
    t0 = time.perf_counter()

    c0 = getattr(comm, "elapsed_ms", None)   # a timing communicator (scripts/rank_stages.py) splits out its calls

    def mark(name):
        nonlocal t0, c0
        if sync is not None:
            sync()
        t1 = time.perf_counter()
        ms[name] = ms.get(name, 0.0) + (t1 - t0) * 1e3
        t0 = t1
        if c0 is not None:
            c1 = comm.elapsed_ms
            ms[name + "_comm"] = ms.get(name + "_comm", 0.0) + (c1 - c0)
            c0 = c1

    W, dev = comm.world, pts.device
    n_total = int(sum(int(v) for v in file_points))
    if W == 1 and not merge and getattr(ops, "build_reports_bbox", False):
        # One rank owns every level-0 cell: the ownership plan is the identity, so
        # neither the bounding-box all-reduce nor the cell histogram has anything
        # to decide.  The build reads the input in place and computes the bounding
        # box itself (its level-0 pass 0, converter.rs:96-104).
        ops.begin_step()
        mark("plan")
        local = ops.build(file_points, pts, None)
        mark("build")
        local = _combine([local])
        local["phases"] = {"lead": 0, "sub": 0, "whole": int(local.get("arrivals", 0))}
        summary = {"number_of_points": n_total, "hierarchies": int(local["hierarchies"]),
                   "bbox_min": list(local["bbox_min"]) if n_total else [0.0, 0.0, 0.0],
                   "bbox_max": list(local["bbox_max"]) if n_total else [0.0, 0.0, 0.0]}
        mark("summary")
        if write:
            ops.write(summary, cells=True, metadata=True)
            mark("write")
        return ShardResult(summary=summary, local=local, recv_points=int(pts.shape[0]),
                           owned_cells=int(local.get("level0_cells", -1)), ms=ms)
    # 2. global bounding box (converter.rs:96-104: componentwise min/max).  With
    # fused ops the same pass over the points also takes the slab histogram, over
    # a grid guessed from an all-reduced sample box with one cell of margin; if
    # a point falls outside it on any rank, the histogram is taken again (step 3).
    # NaN / infinite coordinates on any rank ("nonfinite"): the reference's box
    # skips NaN per axis and keeps infinities (bounding-volume/src/lib.rs:23-31),
    # the ownership grid spans the cells of the points without an infinite
    # coordinate (NaN as cell 0, metadata.rs:100-102), and the points with one
    # travel as unit 0 (one rank builds them all); no cell is shared.
    from pcconv import SHARD_LAYERS as NL, SHARD_LDS_UNITS
    inf3, ninf3 = [float("inf")] * 3, [float("-inf")] * 3
    guess, sh_guess, outside, nf_local = None, None, 0, 0
    # A rank whose local pass fails still joins the collective, with an error flag
    # in the reduced tensor, so that every rank raises instead of the others
    # waiting in it forever.
    # slab units (cell x hex layer) exist for sub-grids of at most 96 (the engine's
    # level-0 layer field); beyond that, whole cells only
    wide = int(ops.cfg_full()["sub_grid_dimension"]) > 96 if hasattr(ops, "cfg_full") else False
    if getattr(ops, "fused_bbox_hist", False) and not merge and n_total and not wide:
        sbox, err = _attempt(lambda: ops.bbox_sample(pts) if pts.shape[0] else (inf3, ninf3), (inf3, ninf3))
        if sbox is None:
            nf_local, sbox = 1, (inf3, ninf3)
        smin, smax = sbox
        sb = torch.tensor([-smin[0], -smin[1], -smin[2], smax[0], smax[1], smax[2], float(nf_local),
                           1.0 if err else 0.0], dtype=torch.float32, device=comm.device)
        comm.allreduce_(sb, "max")
        sbh = sb.cpu().tolist()
        _raise_together(err, sbh[7], "bounding-box sample")
        cs = float(ops.cfg_full()["max_cell_size"])
        if sbh[6] == 0:
            # a guess whose units fit the fused kernel's LDS histogram is preferred,
            # even without the margin: beyond it the counts go to global atomics,
            # which clustered points contend on (config 3: 3.4 ms against 0.3 ms
            # for the two-pass fallback).  The margin-less guess may miss points
            # (step 3 then takes the histogram again).
            def sample_grid(m):
                g = ops.grid([-sbh[0] - m, -sbh[1] - m, -sbh[2] - m], [sbh[3] + m, sbh[4] + m, sbh[5] + m])
                return None if int(getattr(g, "coarse", 0)) else g
            units = lambda g: int(g.ncells) * NL
            g_m = sample_grid(cs)
            if g_m is not None and units(g_m) > SHARD_LDS_UNITS:
                g_0 = sample_grid(0.0)
                if g_0 is not None and units(g_0) <= SHARD_LDS_UNITS:
                    g_m = g_0
            if g_m is not None and units(g_m) <= (1 << 24):
                guess = g_m
    bmin, bmax, err = inf3, ninf3, None
    if guess is not None:
        r, err = _attempt(lambda: ops.bbox_slab_histogram(pts, guess), (inf3, ninf3, None, 0))
        if r is None:
            nf_local = 1
        else:
            bmin, bmax, sh_guess, outside = r
    elif pts.shape[0]:
        r, err = _attempt(lambda: ops.bbox(pts), (inf3, ninf3))
        if r is None:
            nf_local = 1
        else:
            bmin, bmax = r
    bb = torch.tensor([-bmin[0], -bmin[1], -bmin[2], bmax[0], bmax[1], bmax[2], 1.0 if outside else 0.0,
                       float(nf_local), 1.0 if err else 0.0], dtype=torch.float32, device=comm.device)
    comm.allreduce_(bb, "max")
    bbh = bb.cpu().tolist()
    _raise_together(err, bbh[8], "bounding box")
    gmin, gmax = [-bbh[0], -bbh[1], -bbh[2]], bbh[3:6]
    emin, emax = gmin, gmax   # the extent the ownership grid spans
    nonfinite = bbh[7] > 0
    if bbh[6] > 0 or nonfinite:   # the guess missed some point on some rank
        guess, sh_guess = None, None
    if nonfinite:
        empty_parts = inf3 + ninf3 + [0.0] * 3 + inf3 + ninf3
        parts, err = _attempt(lambda: ops.bbox_nonfinite(pts) if pts.shape[0] else empty_parts, empty_parts)
        v = torch.tensor([-x if (k < 3 or 9 <= k < 12) else x for k, x in enumerate(parts)] + [1.0 if err else 0.0],
                         dtype=torch.float32, device=comm.device)
        comm.allreduce_(v, "max")
        vh = v.cpu().tolist()
        _raise_together(err, vh[15], "non-finite bounding box")
        gmin = [-vh[a] if vh[6 + a] > 0 else float("nan") for a in range(3)]
        gmax = [vh[3 + a] if vh[6 + a] > 0 else float("nan") for a in range(3)]
        emin, emax = [-vh[9 + a] for a in range(3)], [vh[12 + a] for a in range(3)]
        if not all(a <= b for a, b in zip(emin, emax)):   # every point has an infinite coordinate
            emin, emax = [0.0] * 3, [0.0] * 3
    mark("bbox")
    plan, etab = None, None
    if n_total == 0:
        recv = pts[:0]
        keys = torch.empty(0, dtype=torch.int32, device=dev)
        owned = 0
        if merge:
            ops.set_subtrees(np.zeros((0, 3), dtype=np.int32))
    else:
        # 3. ownership: level-0 cells; heavy ones shared slab by slab
        grid = ops.grid(emin, emax)
        # this rank's slab histogram over the true grid from the fused pass
        sh_local = (_sub_grid_hist(sh_guess, guess, grid, NL)
                    if sh_guess is not None and not int(getattr(grid, "coarse", 0)) else None)
        coarse = int(getattr(grid, "coarse", 0))
        if merge and coarse:
            raise ValueError("sharded merge: the existing cloud's bounding box spans more than 2^22 level-0 cells")
        # (shared cells exchange global u32 keys: none beyond 2^32 points)
        grid1 = (ops.grid(emin, emax, level=1)
                 if (split and not merge and W > 1 and not coarse and not nonfinite and not wide and n_total < (1 << 32))
                 else None)
        if grid1 is not None and (int(grid1.ncells) > (1 << 22) or int(grid.ncells) * NL > (1 << 24)):
            grid1 = None
        if grid1 is not None:
            sh = sh_local if sh_local is not None else ops.slab_histogram(pts, grid)
            lhist = {"slab": sh}   # this rank's own counts: the one-pass route's totals
            sh_h = comm.allreduce_(sh.to(comm.device).to(torch.int64), "sum").cpu().numpy()
            mark("hist")
            hist_h = sh_h.reshape(-1, NL).sum(axis=1)
            plan = plan_split(hist_h, None, None, W, allow=False)
            if plan.est["ratio"] > 1.02:   # whole cells unbalanced: consider sharing (level-1 histogram)
                mark("plan")
                h1 = ops.histogram(pts, grid1)
                hist1_h = comm.allreduce_(h1.to(comm.device).to(torch.int64), "sum").cpu().numpy()
                mark("hist")
                ch = np.full((len(hist_h), 8), -1, dtype=np.int64)
                nz = np.flatnonzero(hist_h)
                ch[nz] = children_ids(nz, grid, grid1)
                plan = plan_split(hist_h, hist1_h, ch, W, slab_hist=sh_h)
        else:
            hist = (sh_local.view(-1, NL).sum(dim=1, dtype=torch.int32) if sh_local is not None
                    else ops.histogram(pts, grid))
            lhist = {"cell": hist}
            hist_h = comm.allreduce_(hist.to(comm.device).to(torch.int64), "sum").cpu().numpy()
            mark("hist")
            plan = plan_split(hist_h, None, None, W, allow=False)
        owner_h = plan.owner0
        owned = int(np.count_nonzero((owner_h == comm.rank) & (hist_h > 0) & ~plan.split))
        if merge:   # the existing cells of the owned subtrees that receive new points
            ops.set_subtrees(cell_triples(np.flatnonzero((owner_h == comm.rank) & (hist_h > 0)), grid))
        mark("plan")
        # 4. route + exchange (grouped point-to-point transfers of points and keys).
        # A shared cell's slabs travel as a second stream: destination "rank + W".
        nsplit = bool(plan.split.any())
        if W == 1:   # one rank owns every cell: the partition is the identity
            recv, keys = pts, None
            mark("route")
        elif getattr(ops, "bitmap_keys", False):
            # the points travel with one membership bit per sender point instead
            # of a 4-B key each; every receiver rebuilds its keys in rank order
            nd = 2 * W if nsplit else W
            # rank-local keys (no shared cell): the receiver's points keep their
            # key order, their keys are their indices, and the event batches come
            # from a table of the batches' local starts (any cloud size)
            local_keys = getattr(ops, "local_keys", False) and not nsplit
            tab = torch.from_numpy((route_table(plan, W) if nsplit else owner_h).astype(np.int32)).to(dev)
            if nsplit:
                lh = lhist.get("slab")
            else:
                lh = lhist.get("cell")
                if lh is None:   # cells from the slab histogram
                    lh = lhist["slab"].view(-1, NL).sum(dim=1)
            send, bm, counts = ops.route_bitmaps(pts, grid, tab, nd, nsplit, hist=lh)
            mark("route")
            nwl = int(bm.shape[1])
            rw = comm.alltoall_counts([nwl] * W)
            k0 = comm.alltoall_counts([int(key0)] * W)
            streams = [(0, [int(v) for v in counts[:W]], 0)]
            if nsplit:
                streams.append((sum(int(v) for v in counts[:W]), [int(v) for v in counts[W:]], W))
            got = []
            # the points land in rounds while level-0 pass 1 runs on the groups
            # of tiles each round completes (exchange overlap)
            rounds = int(getattr(ops, "landing_rounds", 0)) if local_keys and not merge else 0
            if rounds > 1 and hasattr(comm, "alltoallv_rounds") and comm.device == dev:
                cw = streams[0][1]
                rc = comm.alltoall_counts(cw)
                rbm = _exchange_many(comm, [(bm.narrow(0, 0, W).reshape(-1), [nwl] * W, rw)], dev)[0]
                gs, gb, nbt = global_batches(file_points, ops.batch_size)
                etab = event_table(ops.batch_starts(rbm, rw, k0, gs), gb, sum(rc), nbt)
                recv = torch.empty((sum(rc),) + tuple(send.shape[1:]), dtype=send.dtype, device=dev)
                ops.begin_landing(file_points, recv, etab)
                side = _side_stream(dev) if recv.is_cuda else None   # (named to the library per round)
                if side is not None:
                    side.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(side):
                        comm.alltoallv_rounds(send.narrow(0, 0, sum(cw)), cw, rc, recv, rounds, ops.landed)
                    torch.cuda.current_stream(dev).wait_stream(side)
                else:
                    comm.alltoallv_rounds(send.narrow(0, 0, sum(cw)), cw, rc, recv, rounds, ops.landed)
                streams = []
                got.append((recv, None))
            for off, cw, row in streams:
                rc = comm.alltoall_counts(cw)
                rp, rbm = _exchange_many(comm, [(send.narrow(0, off, sum(cw)), cw, rc),
                                                (bm.narrow(0, row, W).reshape(-1), [nwl] * W, rw)], dev)
                if local_keys:
                    gs, gb, nbt = global_batches(file_points, ops.batch_size)
                    etab = event_table(ops.batch_starts(rbm, rw, k0, gs), gb, sum(rc), nbt)
                    got.append((rp, None))
                else:
                    got.append((rp, ops.keys_from_bitmaps(rbm, rw, k0, sum(rc))))
            recv, keys = got[0]
            if nsplit:
                lrecv, lkeys = got[1]
            del send, bm
        else:
            if nsplit:
                tab = torch.from_numpy(route_table(plan, W).astype(np.int32)).to(dev)
                send, skeys, counts = ops.route_slabs(pts, key0, grid, tab, 2 * W)
            else:
                owner = torch.from_numpy(owner_h.astype(np.int32)).to(dev)
                send, skeys, counts = ops.route(pts, key0, grid, owner, W)
            mark("route")
            cw = [int(v) for v in counts[:W]]
            rc = comm.alltoall_counts(cw)
            nw = sum(cw)
            recv = _exchange(comm, send.narrow(0, 0, nw), cw, rc, dev)
            keys = _exchange(comm, skeys.narrow(0, 0, nw), cw, rc, dev)
            if nsplit:
                cs = [int(v) for v in counts[W:]]
                rcs = comm.alltoall_counts(cs)
                lrecv = _exchange(comm, send.narrow(0, nw, sum(cs)), cs, rcs, dev)
                lkeys = _exchange(comm, skeys.narrow(0, nw, sum(cs)), cs, rcs, dev)
            del send, skeys
        mark("exchange")
    ops.begin_step()
    phases = {"lead": 0, "sub": 0, "whole": 0}
    sub_points = 0
    # 5a. phase 1: the whole level-0 sub-trees this rank owns ...
    if getattr(ops, "landing_active", False):   # the input already borrowed, pass 1 partly run
        local = ops.build_landed()
    else:
        local = (ops.build(file_points, recv, keys, etab=etab) if etab is not None
                 else ops.build(file_points, recv, keys))
    parts = [local]
    phases["whole"] = int(local.get("arrivals", 0))
    mark("build")
    assembled = []
    if plan is not None and plan.split.any() and W > 1:
        # ... and the slots of the shared cells' slabs it holds (raw level 0:
        # every emission forwarded with the key of the arrival that caused it)
        lst, (xyz, _, cn, P, K), (pxyz, pn, gpts) = ops.lead_build_raw(file_points, lrecv, lkeys)
        parts.append(lst)
        phases["lead"] = int(lst["arrivals"])
        mark("lead")
        # 5b. emissions to the owners of their level-1 cells; the partial
        # level-0 cells (grid winners of these slabs) to their writers
        xyz = np.asarray(xyz, np.int64).reshape(-1, 3)
        cn = np.asarray(cn, np.int64)
        d1 = plan.owner1[level1_ids(xyz, grid1)].astype(np.int64) if len(xyz) else np.zeros(0, np.int64)
        rm1, (rP, rK) = _exchange_segments(comm, d1, np.column_stack([xyz, cn]), cn, [P, K], dev)
        del P, K
        pxyz = np.asarray(pxyz, dtype=np.int64).reshape(-1, 3)
        pn = np.asarray(pn, dtype=np.int64).reshape(-1)
        dw = plan.writer[cell_ids(pxyz, grid)].astype(np.int64) if len(pxyz) else np.zeros(0, np.int64)
        rmw, (rG,) = _exchange_segments(comm, dw, np.column_stack([pxyz, pn]), pn, [gpts.to(dev)], dev)
        del gpts
        mark("exchange2")
        # 5c. phase 2: resolve each received level-1 cell's bucket (all ranks'
        # emissions; on the device when the ops offer it), build the spilled ones'
        # sub-trees
        if hasattr(ops, "resolve_level1"):
            res = ops.resolve_level1(rm1, rP, rK, file_points)
        else:
            res = resolve_level1(rm1, rP, rK, file_points, ops.batch_size, ops.limit)
        mark("resolve")
        sub_points = int(res["sub_pts"].shape[0])
        sst = ops.sub_build(file_points, res["sub_pts"], res["sub_keys"], res["roots_xyz"], res["roots_sb"])
        parts.append(sst)
        phases["sub"] = int(sst["arrivals"])
        mark("subtrees")
        # 5d. bucket states and kept lists to the writers, who assemble the cells
        bx = res["bucket_rows"]
        dk = (plan.writer[cell_ids(bx[:, :3] >> 1, grid)].astype(np.int64) if len(bx) else np.zeros(0, np.int64))
        rmk, (rKP,) = _exchange_segments(comm, dk, bx, bx[:, 4] * (bx[:, 3] == 1), [res["kept_pts"]], dev)
        # the pieces stay where they arrived (device) until the cells are
        # walked or written (AssembledCells)
        assembled = AssembledCells(rmw, rG, rmk, rKP, ops.cfg_full())
        ops.set_assembled(assembled)
        mark("assemble")
    local = _combine(parts)
    local["phases"] = phases
    # 6. global metadata values
    hz = torch.tensor([int(local["hierarchies"])], dtype=torch.int64, device=comm.device)
    comm.allreduce_(hz, "max")
    summary = {"number_of_points": n_total, "hierarchies": int(hz.item()),
               "bbox_min": gmin if n_total else [0.0, 0.0, 0.0], "bbox_max": gmax if n_total else [0.0, 0.0, 0.0]}
    if merge:   # lib.rs:86-101: counters continue; converter.rs:96-104 Aabb::extend_aabb
        pm = ops.prior_meta()
        if pm["number_of_points"] > 0:
            if n_total:   # f32::min / max: NaN skipped
                summary["bbox_min"] = [_fmin(a, b) for a, b in zip(gmin, pm["bbox_min"])]
                summary["bbox_max"] = [_fmax(a, b) for a, b in zip(gmax, pm["bbox_max"])]
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
    nrecv = int(recv.shape[0]) + (int(lrecv.shape[0]) if plan is not None and plan.split.any() and W > 1 else 0)
    return ShardResult(summary=summary, local=local, recv_points=nrecv, owned_cells=owned, ms=ms,
                       sub_points=sub_points, plan=(plan.est if plan is not None else {}),
                       assembled_cells=len(assembled))


def key_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous key range [a, b) of rank `rank` (input split evenly in order)."""
    return (n_total * rank) // world, (n_total * (rank + 1)) // world
