"""One event sharded across GPUs: receiver ranges, per-pass state exchange.

Every stage after message passing reduces over one receiver's in-slot segment, so
cutting the receiver-major slot array at node boundaries keeps all of that work
local. Rank r owns receivers [node_lo, node_hi) -- chosen so every rank holds about
S / P slots -- and every rank keeps a replica of the whole graph (a pileup-200 event
is ~0.35 GB; HBM holds hundreds). Per pass, rank r:

1. scans the out-edges of its ``senders`` (every sender with an edge into an owned
   receiver, plus its own senders, whose cumulative merged_cov[1,1] it publishes);
2. extrapolates its owned slots and runs the node kernels on its owned receivers
   (``gtf_pass_shard``);
3. publishes its owned nodes' merged state and its owned slots' activation:
   ``gtf_shard_pack`` -> one all-gather of equal-size chunks (RCCL over xGMI, or gloo
   through host memory) -> ``gtf_shard_unpack``. The bytes travel unchanged, so the
   replicas stay bit-identical and the sharded pass equals the one-GPU pass exactly.

The plan (ranges, sender lists, schedules) is host logic (:class:`ShardPlan`).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat
from .graph import BUCKETS, TrackGraph


class ShardPlan:
    """Receiver ranges balanced by slot count, and each rank's sender list and schedule."""

    def __init__(self, g: TrackGraph, world: int):
        if world < 1:
            raise ValueError("world must be >= 1")
        sp = g.slot_ptr.astype(np.int64)
        S = int(sp[-1])
        targets = [(r * S + world // 2) // world for r in range(world + 1)]
        cuts = [0] + [int(np.searchsorted(sp, t, side="left")) for t in targets[1:-1]] + [g.n_nodes]
        cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts, np.int64), g.n_nodes))
        self.world = world
        self.node_lo = cuts[:-1].astype(np.int32)
        self.node_hi = cuts[1:].astype(np.int32)
        self.slot_lo = sp[self.node_lo].astype(np.int32)
        self.slot_hi = sp[self.node_hi].astype(np.int32)
        self.cap_nodes = int((self.node_hi - self.node_lo).max(initial=0))
        self.cap_slots = int((self.slot_hi - self.slot_lo).max(initial=0))
        self._g = g

    def ranges(self) -> np.ndarray:
        """int32 [4 * world]: node_lo, node_hi, slot_lo, slot_hi per rank"""
        return np.stack([self.node_lo, self.node_hi, self.slot_lo, self.slot_hi], 1).reshape(-1).astype(np.int32)

    def senders(self, r: int) -> np.ndarray:
        g = self._g
        lo, hi = int(self.slot_lo[r]), int(self.slot_hi[r])
        src = g.slot["slot_src"][lo:hi]
        ise = g.slot["is_edge"][lo:hi].astype(bool)
        halo = src[ise & (src >= 0)]
        own = np.arange(self.node_lo[r], self.node_hi[r])
        own = own[np.diff(g.out_ptr.astype(np.int64))[own] > 0]
        return np.unique(np.concatenate([halo.astype(np.int64), own])).astype(np.int32)

    def schedule(self, r: int):
        """(sched, [n_g4, n_g8, n_g16, n_g32, n_g64], n_big) of the owned receivers"""
        deg = np.diff(self._g.slot_ptr.astype(np.int64))
        idx = np.arange(self.node_lo[r], self.node_hi[r], dtype=np.int32)
        d = deg[idx]
        buckets = [idx[(d >= lo) & (d <= hi)] for lo, hi in BUCKETS]
        big = idx[d > 64]
        return np.concatenate(buckets + [big]).astype(np.int32), [int(b.size) for b in buckets], int(big.size)


def allgather_bytes(chunk, out, backend: str, group=None):
    """all-gather equal-size uint8 chunks into ``out`` (world x chunk bytes). RCCL
    ("nccl") gathers device buffers directly over xGMI; gloo stages through host memory."""
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        dist.all_gather_into_tensor(out, chunk, group=group)
        return out
    world = dist.get_world_size(group)
    host = [torch.empty(chunk.numel(), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(host, chunk.cpu(), group=group)
    out.copy_(torch.cat(host).to(out.device))
    return out


class ShardedDeviceGraph:
    """A DeviceGraph replica on this rank's GPU that runs the pass for its receivers
    and exchanges the published state with the other ranks after each pass."""

    def __init__(self, g: TrackGraph, rank: int, world: int, device="cuda", backend="nccl", group=None):
        import torch
        from .device import DeviceGraph, sched_segments
        self.torch = torch
        self.rank, self.world, self.backend, self.group = rank, world, backend, group
        self.plan = ShardPlan(g, world)
        self.d = DeviceGraph(g, device)
        d = self.d
        dev = d.device
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.senders = up(self.plan.senders(rank))
        sched, n_g, n_big = self.plan.schedule(rank)
        self.sched = up(sched)
        self.sched_seg = up(sched_segments(g.slot_ptr, sched))
        self.ranges = up(self.plan.ranges())
        p = d.ptr
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t.numel() else 0)  # noqa: E731
        self.cg = nat.GtfGraph(n_nodes=d.n_nodes, n_slots=d.n_slots, n_edges=d.n_edges, n_big=n_big,
                               slot_ptr=p("slot_ptr"), slot_src=p("slot_src"), slot_dst=p("slot_dst"),
                               out_ptr=p("out_ptr"), out_slot=p("out_slot"), slot_outpos=p("slot_outpos"),
                               is_edge=p("is_edge"), rev_edge=p("rev_edge"), solo=p("solo"), gnn=p("gnn"),
                               xyzr=p("xyzr"), layer=p("layer"), sched=vp(self.sched), n_g4=n_g[0], n_g8=n_g[1],
                               n_g16=n_g[2], n_g32=n_g[3], n_g64=n_g[4], out_dst=p("out_dst"),
                               slot_layer=p("slot_layer"), sched_seg=vp(self.sched_seg))
        pl = self.plan
        self.shard = nat.GtfShard(vp(self.senders), int(self.senders.numel()), int(pl.node_lo[rank]),
                                  int(pl.node_hi[rank]), int(pl.slot_lo[rank]), int(pl.slot_hi[rank]))
        self.chunk_bytes = int(d.lib.gtf_shard_chunk_bytes(pl.cap_nodes, pl.cap_slots))
        self.chunk = torch.zeros(self.chunk_bytes, dtype=torch.uint8, device=dev)
        self.gathered = torch.zeros(self.chunk_bytes * world, dtype=torch.uint8, device=dev)

    def pass_(self, p, events=None):
        """the pass for the owned receivers (events: optional 5 hipEvent_t handles)"""
        d = self.d
        cp = d.cparams(p)
        ev = (ctypes.c_void_p * 5)(*events) if events is not None else None
        nat.check(d.lib.gtf_pass_shard(ctypes.byref(self.cg), ctypes.byref(d.cn), ctypes.byref(d.ctse),
                                       ctypes.byref(d.cuts), ctypes.byref(d.ce), ctypes.byref(cp),
                                       ctypes.byref(self.shard), d.ptr("ws"), d.stream, ev))

    def exchange(self):
        """publish the owned merged states and activations; take the other ranks'"""
        d = self.d
        pl = self.plan
        nat.check(d.lib.gtf_shard_pack(ctypes.byref(d.cn), ctypes.byref(d.ce), ctypes.byref(self.shard),
                                       pl.cap_nodes, pl.cap_slots, ctypes.c_void_p(self.chunk.data_ptr()), d.stream))
        if self.world > 1:
            allgather_bytes(self.chunk, self.gathered, self.backend, self.group)
            nat.check(d.lib.gtf_shard_unpack(ctypes.byref(d.cn), ctypes.byref(d.ce),
                                             ctypes.c_void_p(self.gathered.data_ptr()), self.world, self.rank,
                                             ctypes.c_void_p(self.ranges.data_ptr()), pl.cap_nodes, pl.cap_slots,
                                             d.stream))

    def step(self, p, events=None):
        self.pass_(p, events)
        self.exchange()
