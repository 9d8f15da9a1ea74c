"""One event sharded across GPUs: receiver ranges, per-pass halo exchange.

Every stage after message passing reduces over one receiver's in-slot segment, so
cutting the receiver-major slot array at node boundaries keeps all of that work
local. Rank r owns receivers [node_lo, node_hi) and every rank keeps a replica of the
whole graph (a pileup-200 event is ~0.35 GB; HBM holds hundreds).

Node order. With more than one rank the event is renumbered before upload so that the
contiguous ranges are azimuthal wedges (``sector_order``: φ cut at slot-weighted
quantiles, original (layer, φ) order inside a wedge): tracks are nearly radial and an
edge spans at most ~0.06 rad, so few edges cross a wedge boundary. Inside every rank's
range the nodes are then bucketed by slot count tile by tile (the 1-GPU "tiled" layout,
``gtf.device.schedule_order``); the pass is equivariant under renumbering, and
``download`` maps results back to the host order.

Per pass, rank r (``gtf_pass_shard``):

1. scans the out-edges of its ``senders`` (every sender with an edge into an owned
   receiver, plus its own senders) on an out-degree-bucketed schedule (``out_sched``,
   as the 1-GPU pass);
2. extrapolates its owned slots and runs the fused node kernel on its owned receivers
   (their slot-count schedule, 2-lane groups included);
3. exchanges the halo (:class:`HaloPlan`): each rank sends every other rank the merged
   states of that rank's senders it owns and the activations of those senders'
   out-edges whose receivers it owns -- exactly what the other rank's next sender scan
   reads -- through per-destination segments of ONE all-to-all (RCCL over xGMI; gloo
   through host memory on CPU). Values travel as bytes, so the pass equals the one-GPU
   pass bit for bit.

``sync`` makes every replica complete (all-gather of every owned state, the round-1
exchange) before results are read back.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _native as nat
from .graph import BUCKETS, TrackGraph, renumber


def sector_order(g: TrackGraph, world: int):
    """(order, cuts): node order with each of `world` azimuthal wedges contiguous (wedges
    balanced by slots + nodes, original order inside a wedge) and the wedges' node
    boundaries (cuts[r]..cuts[r+1] is wedge r)."""
    N = g.n_nodes
    if world <= 1 or N == 0:
        return np.arange(N, dtype=np.int64), np.array([0, N], np.int64)
    phi = np.arctan2(g.node["gnn"][:, 1], g.node["gnn"][:, 0])
    w = np.diff(g.slot_ptr.astype(np.int64)) + 1
    o = np.argsort(phi, kind="stable")
    cw = np.cumsum(w[o])
    tot = cw[-1]
    k = np.searchsorted(cw, [tot * r / world for r in range(1, world)], side="left")
    cuts_phi = phi[o[np.minimum(k, N - 1)]]
    sector = np.searchsorted(cuts_phi, phi, side="right")
    order = np.lexsort((np.arange(N), sector))
    cuts = np.concatenate([[0], np.cumsum(np.bincount(sector, minlength=world))]).astype(np.int64)
    return order.astype(np.int64), cuts


def shard_layout(g: TrackGraph, world: int, tile: int):
    """The device node order of a sharded event and its rank cuts: wedges (world > 1),
    then the tiled slot-count bucketing inside each rank's range. Returns
    (device graph, order, slot_perm, cuts); device node i is host node order[i]."""
    from .device import schedule_order
    o1, cuts = sector_order(g, world)
    g1, sp1 = renumber(g, o1)
    sp = g1.slot_ptr.astype(np.int64)
    parts = []
    for r in range(len(cuts) - 1):
        lo, hi = int(cuts[r]), int(cuts[r + 1])
        parts.append(lo + schedule_order(sp[lo:hi + 1] - sp[lo], tile))
    o2 = np.concatenate(parts) if parts else np.zeros(0, np.int64)
    g2, sp2 = renumber(g1, o2)
    return g2, o1[o2], sp1[sp2], cuts


class ShardPlan:
    """Receiver ranges (given cuts, or balanced by slot count), and each rank's sender
    list and schedules."""

    def __init__(self, g: TrackGraph, world: int, cuts=None):
        if world < 1:
            raise ValueError("world must be >= 1")
        sp = g.slot_ptr.astype(np.int64)
        S = int(sp[-1])
        if cuts is None:
            targets = [(r * S + world // 2) // world for r in range(world + 1)]
            cuts = [0] + [int(np.searchsorted(sp, t, side="left")) for t in targets[1:-1]] + [g.n_nodes]
            cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts, np.int64), g.n_nodes))
        cuts = np.asarray(cuts, np.int64)
        if cuts.size != world + 1 or cuts[0] != 0 or cuts[-1] != g.n_nodes or (np.diff(cuts) < 0).any():
            raise ValueError("cuts must be world + 1 non-decreasing node boundaries from 0 to n_nodes")
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

    def owner_of_nodes(self) -> np.ndarray:
        return np.repeat(np.arange(self.world, dtype=np.int32), self.node_hi - self.node_lo)

    def senders(self, r: int) -> np.ndarray:
        g = self._g
        lo, hi = int(self.slot_lo[r]), int(self.slot_hi[r])
        src = g.slot["slot_src"][lo:hi]
        ise = g.slot["is_edge"][lo:hi].astype(bool)
        halo = src[ise & (src >= 0)]
        own = np.arange(self.node_lo[r], self.node_hi[r])
        own = own[np.diff(g.out_ptr.astype(np.int64))[own] > 0]
        return np.unique(np.concatenate([halo.astype(np.int64), own])).astype(np.int32)

    def split(self, r: int):
        """rank r's pass in two edge phases (gtf_shard.phases, SURVEY §8e overlap): the
        INTERIOR senders -- owned by r with every out-edge receiver owned by r, so their
        merged state and every activation their scan reads are r's own after its pass --
        with the owned slots they send to (and the owned keys without an edge), and the
        other senders with their owned edges (halo-dependent: what the exchange brings).
        Returns (interior senders, other senders, interior slots, other slots), int32,
        ascending; every sender of senders(r) and every owned slot in exactly one part."""
        g = self._g
        s = self.senders(r).astype(np.int64)
        on = self.owner_of_nodes()
        op = g.out_ptr.astype(np.int64)
        dst = g.slot_dst()[g.out_slot.astype(np.int64)] if g.n_slots else np.zeros(0, np.int64)
        foreign = (on[dst] != r).astype(np.int64) if dst.size else np.zeros(0, np.int64)
        cf = np.concatenate([[0], np.cumsum(foreign)])
        interior = (on[s] == r) & (cf[op[s + 1]] == cf[op[s]])
        is_in = np.zeros(g.n_nodes, bool)
        is_in[s[interior]] = True
        lo, hi = int(self.slot_lo[r]), int(self.slot_hi[r])
        src = g.slot["slot_src"][lo:hi].astype(np.int64)
        ise = g.slot["is_edge"][lo:hi].astype(bool)
        # the other part = exactly the owned edges of the other senders (their out-edges into
        # the rank's receivers: the fused sender-major phase 1b reaches them through the
        # senders' out-lists); keys without an edge and orphans need nothing from anyone
        k_in = ~(ise & (src >= 0) & ~is_in[np.maximum(src, 0)])
        ks = np.arange(lo, hi, dtype=np.int64)
        return (s[interior].astype(np.int32), s[~interior].astype(np.int32), ks[k_in].astype(np.int32),
                ks[~k_in].astype(np.int32))

    def schedule(self, r: int, widen: int = 0):
        """(sched, [n_g4, n_g8, n_g16, n_g32, n_g64], n_big, n_g2) of the owned receivers:
        slot-count buckets in node order, the <= 2-slot nodes first in the <= 4 bucket.
        widen = k > 0: every node in the bucket k sizes up (2**k times the lanes, capped at
        64; no 2-lane groups) -- a rank's small share then runs each node's op chain on more
        lanes (fewer pair rounds) where the GPU has lanes to spare"""
        deg = np.diff(self._g.slot_ptr.astype(np.int64))
        idx = np.arange(self.node_lo[r], self.node_hi[r], dtype=np.int32)
        d = deg[idx]
        q = np.full(d.size, -1, np.int64)
        for j, (lo, hi) in enumerate(BUCKETS):
            q[(d >= lo) & (d <= hi)] = j
        q = np.where(q >= 0, np.minimum(q + widen, len(BUCKETS) - 1), -1)
        buckets = [idx[q == j] for j in range(len(BUCKETS))]
        d0 = deg[buckets[0]]
        n2 = int((d0 <= 2).sum()) if widen == 0 else 0
        if widen == 0:
            buckets[0] = np.concatenate([buckets[0][d0 <= 2], buckets[0][d0 > 2]])
        big = idx[d > 64]
        return (np.concatenate(buckets + [big]).astype(np.int32), [int(b.size) for b in buckets], int(big.size), n2)

    def sender_schedule(self, r: int):
        """the rank's senders as (u, out_ptr[u], out_ptr[u+1], 0) quadruples bucketed by
        out-degree (gtf_graph.out_sched) and the bucket sizes [n_o4, n_o8, n_o16]"""
        from .device import sender_schedule
        g = self._g
        u = self.senders(r).astype(np.int64)
        op = g.out_ptr.astype(np.int64)
        return sender_schedule(op, u)


class HaloPlan:
    """What each rank's next pass reads from the others: for rank r, the merged states
    of its senders owned elsewhere and the activations of its senders' out-edges whose
    receivers are owned elsewhere. A message q -> r is one segment
    [node records (GTF_HALO_NODE_BYTES each) | activation bytes], padded to 8 bytes."""

    def __init__(self, plan: ShardPlan):
        g = plan._g
        W = plan.world
        self.world = W
        on = plan.owner_of_nodes()
        slot_dst = g.slot_dst() if g.n_slots else np.zeros(0, np.int64)
        os_ = on[slot_dst] if g.n_slots else np.zeros(0, np.int32)
        op = g.out_ptr.astype(np.int64)
        self.need_nodes, self.need_slots = [], []
        for r in range(W):
            s = plan.senders(r).astype(np.int64)
            self.need_nodes.append(np.sort(s[on[s] != r]).astype(np.int32))
            cnt = op[s + 1] - op[s]
            first = np.repeat(op[s], cnt)
            pos = np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(np.cumsum(cnt) - cnt, cnt)
            sl = g.out_slot.astype(np.int64)[first + pos] if cnt.sum() else np.zeros(0, np.int64)
            self.need_slots.append(np.unique(sl[os_[sl] != r]).astype(np.int32))
        self._on, self._os = on, os_

    @staticmethod
    def _seg_bytes(n_nodes, n_slots):
        return (nat.HALO_NODE_BYTES * n_nodes + n_slots + 7) // 8 * 8

    def message(self, q: int, r: int):
        """(nodes, slots) rank q sends rank r"""
        nn, ns = self.need_nodes[r], self.need_slots[r]
        return nn[self._on[nn] == q], ns[self._os[ns] == q]

    def lists(self, rank: int, send: bool):
        """node / slot indices with their byte offsets in this rank's send (or receive)
        buffer, and the per-peer segment sizes (all_to_all split sizes)"""
        idx_n, off_n, idx_s, off_s, sizes = [], [], [], [], []
        base = 0
        for peer in range(self.world):
            if peer == rank:
                sizes.append(0)
                continue
            nodes, slots = self.message(rank, peer) if send else self.message(peer, rank)
            idx_n.append(nodes)
            off_n.append(base + nat.HALO_NODE_BYTES * np.arange(nodes.size, dtype=np.int64))
            idx_s.append(slots)
            off_s.append(base + nat.HALO_NODE_BYTES * nodes.size + np.arange(slots.size, dtype=np.int64))
            b = self._seg_bytes(nodes.size, slots.size)
            sizes.append(b)
            base += b
        cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
        return cat(idx_n, np.int32), cat(off_n, np.int64), cat(idx_s, np.int32), cat(off_s, np.int64), sizes

    def bytes_sent(self, rank: int) -> int:
        return int(sum(self.lists(rank, True)[4]))


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


def alltoall_bytes(send, recv, send_sizes, recv_sizes, backend: str, group=None):
    """one all-to-all of variable-size uint8 segments (split sizes in bytes). RCCL moves
    device buffers over xGMI; gloo stages through host memory."""
    import torch.distributed as dist
    if backend == "nccl":
        dist.all_to_all_single(recv, send, recv_sizes, send_sizes, group=group)
        return recv
    h = recv.cpu()
    dist.all_to_all_single(h, send.cpu(), recv_sizes, send_sizes, group=group)
    recv.copy_(h.to(recv.device))
    return recv


def allreduce_max_i64(buf, backend: str, group=None):
    """element-wise MAX all-reduce of an int64 buffer (the sharded tag sweep's exchange).
    RCCL reduces the device buffer over xGMI; gloo stages through host memory."""
    import torch.distributed as dist
    if backend == "nccl":
        dist.all_reduce(buf, op=dist.ReduceOp.MAX, group=group)
        return buf
    h = buf.cpu()
    dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
    if h is not buf:
        buf.copy_(h.to(buf.device))
    return buf


class ShardedDeviceGraph:
    """A DeviceGraph replica on this rank's GPU (wedge + tiled node order) that runs the
    pass for its receivers and exchanges the halo with the other ranks after each pass."""

    def __init__(self, g: TrackGraph, rank: int, world: int, device="cuda", backend="nccl", group=None,
                 tile: int = None, widen: int = None, comm=None):
        """backend: "nccl" (torch.distributed over RCCL), "gloo" (torch.distributed staged through
        host memory), "native" (libgtf's own RCCL communicator, gtf.comm.NativeComm: `comm`,
        else one made from `group` when torch.distributed runs, else a world of one), or
        "local" (no collective: SplitDeviceGraph)."""
        import torch
        from .device import DeviceGraph, TILE, sched_segments, sender_lanes
        from .device import sender_schedule as sender_schedule_of
        self.torch = torch
        self.rank, self.world, self.backend, self.group = rank, world, backend, group
        gd, order, slot_perm, cuts = shard_layout(g, world, TILE if tile is None else tile)
        self.plan = ShardPlan(gd, world, cuts)
        self.halo = HaloPlan(self.plan)
        self.d = DeviceGraph(gd, device)
        d = self.d
        d.order, d.slot_perm, d.layout = order, slot_perm, "sharded"   # download() maps back to host order
        dev = d.device
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t.numel() else 0)  # noqa: E731
        pl = self.plan
        self.senders = up(pl.senders(rank))
        if widen is None:
            widen = int(os.environ.get("GTF_SHARD_WIDEN", "0"))
        sched, n_g, n_big, n_g2 = pl.schedule(rank, widen)
        self.sched = up(sched)
        self.sched_seg = up(sched_segments(gd.slot_ptr, sched))
        osched, n_o = pl.sender_schedule(rank)
        self.out_sched = up(osched)
        self.out_lanes = up(sender_lanes(d.t["out_slot"].cpu().numpy(), d.t["out_dst"].cpu().numpy(), osched, n_o))
        self.ranges = up(pl.ranges())
        p = d.ptr
        self.cg = nat.GtfGraph(n_nodes=d.n_nodes, n_slots=d.n_slots, n_edges=d.n_edges, n_big=n_big,
                               slot_ptr=p("slot_ptr"), slot_src=p("slot_src"), slot_dst=p("slot_dst"),
                               out_ptr=p("out_ptr"), out_slot=p("out_slot"), slot_outpos=p("slot_outpos"),
                               is_edge=p("is_edge"), rev_edge=p("rev_edge"), solo=p("solo"), gnn=p("gnn"),
                               xyzr=p("xyzr"), layer=p("layer"), sched=vp(self.sched), n_g4=n_g[0], n_g8=n_g[1],
                               n_g16=n_g[2], n_g32=n_g[3], n_g64=n_g[4], out_dst=p("out_dst"),
                               slot_layer=p("slot_layer"), sched_seg=vp(self.sched_seg),
                               out_sched=vp(self.out_sched), n_o4=n_o[0], n_o8=n_o[1], n_o16=n_o[2], n_g2=n_g2,
                               out_lanes=vp(self.out_lanes),
                               slot_outidx=p("slot_outidx") if d.use_outidx else ctypes.c_void_p(0),
                               slot_class=p("slot_class") if d.use_classes else ctypes.c_void_p(0),
                               slot_sflags=p("slot_sflags") if d.use_classes else ctypes.c_void_p(0),
                               slot_sxzr=p("slot_sxzr") if d.use_sxzr else ctypes.c_void_p(0),
                               slot_static=p("slot_static") if d.use_static32 else ctypes.c_void_p(0),
                               slot_xclass=p("slot_xclass") if d.use_classes else ctypes.c_void_p(0))
        self.shard = nat.GtfShard(vp(self.senders), int(self.senders.numel()), int(pl.node_lo[rank]),
                                  int(pl.node_hi[rank]), int(pl.slot_lo[rank]), int(pl.slot_hi[rank]))
        # the pass in phases (ShardPlan.split): 1a the interior senders and their slots, 1b the
        # rest after the halo exchange, 2 the node kernels -- so the exchange of one pass's
        # halo overlaps the next pass's phase 1a (step)
        self._phase_t = []
        self.cg_phase, self.shard_phase = [], []
        self._part_slots = []
        for part_s, part_k in (lambda x: ((x[0], x[2]), (x[1], x[3])))(pl.split(rank)):
            z1 = np.zeros(1, np.int32)
            ts, tk = up(np.concatenate([part_s, z1])), up(np.concatenate([part_k, z1]))   # int32, never empty
            osch, n_o_ = sender_schedule_of(gd.out_ptr, part_s)
            t_os = up(osch if osch.size else np.zeros(4, np.int32))
            t_ol = up(sender_lanes(d.t["out_slot"].cpu().numpy(), d.t["out_dst"].cpu().numpy(), osch, n_o_))
            self._phase_t += [ts, tk, t_os, t_ol]
            cgp = type(self.cg).from_buffer_copy(self.cg)
            cgp.out_sched, cgp.out_lanes = vp(t_os), vp(t_ol)
            cgp.n_o4, cgp.n_o8, cgp.n_o16 = n_o_
            self.cg_phase.append(cgp)
            # phase 1b (the second part): the halo senders' scan, then their owned slots; or
            # fused (GTF_SHARD_FUSED_1B=1, gtf_shard.phases bit 4: the scan's lanes extrapolate
            # their owned out-edges, one launch) -- measured slower on the box (N = 8: 18.0 vs
            # 14.7 us; the fused kernel runs 3 waves per SIMD at 145 VGPRs)
            ph = 5 if (self.shard_phase and os.environ.get("GTF_SHARD_FUSED_1B", "0") == "1") else 1
            self._part_slots.append(int(part_k.size))
            # (the fused form extrapolates the senders' owned out-edges itself: no slot list)
            self.shard_phase.append(nat.GtfShard(vp(ts), int(part_s.size), int(pl.node_lo[rank]), int(pl.node_hi[rank]),
                                                 int(pl.slot_lo[rank]), int(pl.slot_hi[rank]),
                                                 ph, vp(tk) if ph != 5 else ctypes.c_void_p(0),
                                                 int(part_k.size) if ph != 5 else 0, 0))
        self.shard_node = nat.GtfShard(vp(self.senders), int(self.senders.numel()), int(pl.node_lo[rank]),
                                       int(pl.node_hi[rank]), int(pl.slot_lo[rank]), int(pl.slot_hi[rank]), 2)
        self.split_sizes = {"interior_senders": int(self.shard_phase[0].n_senders),
                            "halo_senders": int(self.shard_phase[1].n_senders),
                            "interior_slots": int(self.shard_phase[0].n_slot_list),
                            "halo_slots": int(self._part_slots[1])}
        self.overlap = True        # step(): the halo exchange beside the next pass's phase 1a
        self._pending = False      # a pass's halo not yet exchanged
        # halo exchange buffers and lists (fixed per plan)
        self._halo_t = {}
        self.halo_send, self.halo_recv = self._halo(True), self._halo(False)
        self.send_buf = torch.zeros(max(sum(self.send_sizes), 8), dtype=torch.uint8, device=dev)
        self.recv_buf = torch.zeros(max(sum(self.recv_sizes), 8), dtype=torch.uint8, device=dev)
        # full sync (every owned state, all-gather) before results are read back
        self.chunk_bytes = int(d.lib.gtf_shard_chunk_bytes(pl.cap_nodes, pl.cap_slots))
        self.chunk = torch.zeros(self.chunk_bytes, dtype=torch.uint8, device=dev)
        self.gathered = torch.zeros(self.chunk_bytes * world, dtype=torch.uint8, device=dev)
        self.comm = None
        if backend == "native":
            from .comm import NativeComm
            if comm is None:
                import torch.distributed as dist
                # gtf_comm_init binds RCCL to the CURRENT HIP device: make this rank's current
                with torch.cuda.device(torch.device(dev)):
                    if dist.is_available() and dist.is_initialized():
                        comm = NativeComm.from_torch(group, lib=d.lib)
                    elif world == 1:
                        comm = NativeComm.single(lib=d.lib)
                    else:
                        raise ValueError("backend 'native' with world > 1 needs a NativeComm (gtf.comm) or "
                                         "torch.distributed")
            if comm.world != world or comm.rank != rank:
                raise ValueError("NativeComm is rank %d of %d, the shard rank %d of %d" % (comm.rank, comm.world, rank, world))
            self.comm = comm
            self._sizes_c = ((ctypes.c_int64 * world)(*self.send_sizes), (ctypes.c_int64 * world)(*self.recv_sizes))

    def _halo(self, send):
        torch = self.torch
        idx_n, off_n, idx_s, off_s, sizes = self.halo.lists(self.rank, send)
        ts = [torch.from_numpy(a).to(self.d.device) for a in (idx_n, off_n, idx_s, off_s)]
        self._halo_t[send] = ts     # keep the device lists alive
        if send:
            self.send_sizes = sizes
        else:
            self.recv_sizes = sizes
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t.numel() else 0)  # noqa: E731
        return nat.GtfHalo(vp(ts[0]), vp(ts[1]), int(idx_n.size), 0, vp(ts[2]), vp(ts[3]), int(idx_s.size), 0)

    @property
    def halo_bytes(self) -> int:
        """bytes this rank sends per pass"""
        return int(sum(self.send_sizes))

    # Per-pass host work is kept to the calls themselves: at N = 8 a rank's pass is ~40 us
    # of GPU time, so the parameter struct, workspace / buffer pointers, the stream handle
    # and the exchange's tensor views are built once (the stream current at the first call
    # is used for every later one).
    def _io(self):
        io = getattr(self, "_io_c", None)
        if io is None:
            d = self.d
            io = self._io_c = (d.ptr("ws"), d.stream, ctypes.c_void_p(self.send_buf.data_ptr()),
                               ctypes.c_void_p(self.recv_buf.data_ptr()), self.send_buf[:sum(self.send_sizes)],
                               self.recv_buf[:sum(self.recv_sizes)])
        return io

    def _tstream(self):
        """the cached pass stream (_io) as a torch stream: the exchange's events, asynchronous
        collectives and host copies are ordered against THIS stream, on which halo_pack /
        halo_unpack and the phases run, whatever stream is current at a later call"""
        ts = getattr(self, "_ts_c", None)
        if ts is None:
            torch = self.torch
            h = self._io()[1].value or 0
            dev = torch.device(self.d.device)
            ts = self._ts_c = (torch.cuda.ExternalStream(h, device=dev) if h else torch.cuda.default_stream(dev))
        return ts

    def _cparams(self, p):
        key = (p.sigma0xy, p.sigma0rz, p.sigma0rz2, p.endcap_boundary, p.chi2_cut, p.reweight_threshold,
               p.cluster_chi2, p.cluster_kl)
        c = getattr(self, "_cp_c", None)
        if c is None or c[0] != key:
            c = self._cp_c = (key, self.d.cparams(p))
        return c[1]

    def pass_(self, p, events=None):
        """the pass for the owned receivers (events: optional 5 hipEvent_t handles); a halo
        an overlapped step left pending is exchanged first"""
        self.flush()
        d = self.d
        ws, st = self._io()[:2]
        ev = (ctypes.c_void_p * 5)(*events) if events is not None else None
        nat.check(d.lib.gtf_pass_shard(ctypes.byref(self.cg), ctypes.byref(d.cn), ctypes.byref(d.ctse),
                                       ctypes.byref(d.cuts), ctypes.byref(d.ce), ctypes.byref(self._cparams(p)),
                                       ctypes.byref(self.shard), ws, st, ev))

    def exchange(self):
        """the halo: what the other ranks' next pass reads, one all-to-all"""
        self.flush()
        if self.comm is not None:   # pack, all-to-all and unpack inside libgtf (gtf_halo_exchange)
            d = self.d
            _, st, sbuf, rbuf = self._io()[:4]
            nat.check(d.lib.gtf_halo_exchange(self.comm.ptr, ctypes.byref(d.cn), ctypes.byref(d.ce),
                                              ctypes.byref(self.halo_send), ctypes.byref(self.halo_recv), sbuf, rbuf,
                                              ctypes.cast(self._sizes_c[0], ctypes.c_void_p),
                                              ctypes.cast(self._sizes_c[1], ctypes.c_void_p), st))
            return
        if self.world == 1:
            return
        _, st, sbuf, rbuf, sview, rview = self._io()
        self.halo_pack()
        with self.torch.cuda.stream(self._tstream()):   # ordered after the pack, before the unpack
            alltoall_bytes(sview, rview, self.send_sizes, self.recv_sizes, self.backend, self.group)
        self.halo_unpack(rbuf)

    def halo_pack(self):
        """this rank's halo segments into its send buffer (on its stream)"""
        d = self.d
        _, st, sbuf = self._io()[:3]
        nat.check(d.lib.gtf_halo_pack(ctypes.byref(d.cn), ctypes.byref(d.ce), ctypes.byref(self.halo_send), sbuf, st))

    def halo_unpack(self, buf, stream=None):
        """the received halo segments (device buffer address `buf`, receive layout) into this
        rank's replica (on its stream, or on `stream`: a torch stream)"""
        d = self.d
        st = self._io()[1] if stream is None else ctypes.c_void_p(stream.cuda_stream)
        nat.check(d.lib.gtf_halo_unpack(ctypes.byref(d.cn), ctypes.byref(d.ce), ctypes.byref(self.halo_recv), buf,
                                        st))

    def sync(self):
        """every owned merged state and activation to every replica (all-gather), so the
        whole graph can be read back from any rank (a pending halo is part of it)"""
        self._pending = False
        d = self.d
        pl = self.plan
        nat.check(d.lib.gtf_shard_pack(ctypes.byref(d.cn), ctypes.byref(d.ce), ctypes.byref(self.shard),
                                       pl.cap_nodes, pl.cap_slots, ctypes.c_void_p(self.chunk.data_ptr()), d.stream))
        if self.comm is not None:
            self.comm.allgather_bytes(self.chunk, self.gathered, d.stream)
        if self.world > 1:
            if self.comm is None:
                allgather_bytes(self.chunk, self.gathered, self.backend, self.group)
            nat.check(d.lib.gtf_shard_unpack(ctypes.byref(d.cn), ctypes.byref(d.ce),
                                             ctypes.c_void_p(self.gathered.data_ptr()), self.world, self.rank,
                                             ctypes.c_void_p(self.ranges.data_ptr()), pl.cap_nodes, pl.cap_slots,
                                             d.stream))

    def _phase(self, p, which):
        """one phase of the pass: 0 = 1a (interior senders and their slots), 1 = 1b (the rest),
        2 = the node kernels"""
        d = self.d
        ws, st = self._io()[:2]
        cg, sh = (self.cg_phase[which], self.shard_phase[which]) if which < 2 else (self.cg, self.shard_node)
        nat.check(d.lib.gtf_pass_shard(ctypes.byref(cg), ctypes.byref(d.cn), ctypes.byref(d.ctse),
                                       ctypes.byref(d.cuts), ctypes.byref(d.ce), ctypes.byref(self._cparams(p)),
                                       ctypes.byref(sh), ws, st, None))

    def _exchange_begin(self, pack=True):
        """(pack this rank's halo segments and) start the all-to-all; returns what
        _exchange_end needs. The pack is stream-ordered before anything the caller enqueues
        next, so the next pass's phase 1a can run while the segments travel. step() packs at
        the end of its own pass (pack=False here): the halo is that pass's outputs whatever
        the caller does between two steps (e.g. bench's use_inputs)."""
        if self.world == 1 and self.comm is None:
            return None
        if pack:
            self.halo_pack()
        _, st, sbuf, rbuf, sview, rview = self._io()
        if self.comm is not None:   # libgtf's RCCL group on a stream of its own
            torch = self.torch
            if getattr(self, "_xs", None) is None:
                self._xs = torch.cuda.Stream(device=self.d.device)
                self._xev = (torch.cuda.Event(), torch.cuda.Event())
            self._xev[0].record(self._tstream())   # after the pack (on the pass stream)
            self._xs.wait_event(self._xev[0])
            nat.check(self.d.lib.gtf_halo_alltoall(self.comm.ptr, sbuf, rbuf,
                                                   ctypes.cast(self._sizes_c[0], ctypes.c_void_p),
                                                   ctypes.cast(self._sizes_c[1], ctypes.c_void_p),
                                                   ctypes.c_void_p(self._xs.cuda_stream)))
            self._xev[1].record(self._xs)
            return "native"
        if self.backend == "nccl":   # torch.distributed over RCCL, asynchronous
            import torch.distributed as dist
            # the collective's stream waits on the CURRENT stream: make it the pass stream
            with self.torch.cuda.stream(self._tstream()):
                return dist.all_to_all_single(rview, sview, self.recv_sizes, self.send_sizes, group=self.group,
                                              async_op=True)
        return "host"   # gloo: through host memory at _exchange_end

    def _exchange_end(self, h):
        if h is None:
            return
        _, st, sbuf, rbuf, sview, rview = self._io()
        ts = self._tstream()   # the unpack runs on the pass stream: that stream waits
        if h == "native":
            ts.wait_event(self._xev[1])
        else:
            with self.torch.cuda.stream(ts):
                if h == "host":
                    alltoall_bytes(sview, rview, self.send_sizes, self.recv_sizes, self.backend, self.group)
                else:
                    h.wait()
        self.halo_unpack(rbuf)

    def step(self, p, events=None, overlap=None, phase_events=None):
        """one pass of the owned receivers. overlap (default self.overlap = True): the pass
        in phases -- the previous pass's halo exchange (pending) starts, phase 1a (interior
        senders and their slots, which read nothing the exchange brings) runs while it
        travels, then the halo is unpacked and phase 1b and the node kernels follow; this
        pass's own halo stays pending until the next step (or flush / sync). Bit-equal to
        overlap=False (the one-call pass, then the exchange). phase_events (diagnostics):
        5 torch events recorded on the pass stream before phase 1a, after it, after the
        exchange's wait and unpack, after phase 1b, after the node kernels and the pack."""
        if overlap is None:
            overlap = self.overlap
        if not overlap or events is not None:
            self.flush()
            self.pass_(p, events)
            self.exchange()
            return
        pe = phase_events
        ts = self._tstream() if pe is not None else None
        if pe is not None:
            pe[0].record(ts)
        h = self._exchange_begin(pack=False) if self._pending else None
        self._pending = False
        self._phase(p, 0)
        if pe is not None:
            pe[1].record(ts)
        self._exchange_end(h)
        if pe is not None:
            pe[2].record(ts)
        self._phase(p, 1)
        if pe is not None:
            pe[3].record(ts)
        self._phase(p, 2)
        if self.world > 1 or self.comm is not None:   # (native: RCCL even at world 1)
            self.halo_pack()        # this pass's halo, packed now; sent by the next step / flush
            self._pending = True
        if pe is not None:
            pe[4].record(ts)

    def flush(self):
        """the pending halo exchange (a step's last pass, already packed), now"""
        if self._pending:
            self._pending = False
            self._exchange_end(self._exchange_begin(pack=False))

    def tag_propagation(self, tags, radius, threshold=0.1, max_sweeps=100000):
        """Tag propagation (tag_propagation/tag_propagation.py:97-164) on the edge-sharded
        event: the keep mask and the processed count come from the replica
        (gtf_tag_prepare over the whole event, no exchange); per sweep every rank computes
        its owned nodes' next tags (gtf_tag_sweep_shard) and ONE all-reduce(MAX) of the
        n_nodes + world int64 words gives every replica the whole next tag array and every
        rank's flip count. Same stop rule (flips / processed <= threshold), sweeps and tags
        as DeviceGraph.tag_propagation, bit for bit. Returns (tags in host node order,
        flips per sweep) on every rank; tags / radius are host-order arrays."""
        torch = self.torch
        d = self.d
        N, W = d.n_nodes, self.world
        dev = d.device
        vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        if self.comm is not None:   # the whole stage inside libgtf (gtf_tag_propagate_shard)
            r = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(radius), dtype=np.float64)).to(dev)
            ta = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(tags), dtype=np.int64)).to(dev)
            nb = int(d.lib.gtf_tag_shard_workspace_bytes(N, d.n_edges, W))
            ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
            hf = np.zeros(max(int(max_sweeps), 1), np.int32)
            n = ctypes.c_int32(0)
            nat.check(d.lib.gtf_tag_propagate_shard(self.comm.ptr, ctypes.byref(self.cg), ctypes.byref(self.shard),
                                                    vp(r), vp(ta), float(threshold), int(max_sweeps),
                                                    ctypes.c_void_p(hf.ctypes.data), ctypes.byref(n), vp(ws),
                                                    ctypes.c_size_t(nb), d.stream))
            out = ta.cpu().numpy()
            h = np.empty_like(out)
            h[d.order] = out
            return h, [int(x) for x in hf[:n.value]]
        keep = torch.zeros(max(d.n_edges, 1), dtype=torch.uint8, device=dev)
        proc = torch.zeros(max(N, 1), dtype=torch.uint8, device=dev)
        cnt = torch.zeros(2, dtype=torch.int32, device=dev)
        r = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(radius), dtype=np.float64)).to(dev)
        ta = torch.zeros(N + W, dtype=torch.int64, device=dev)
        ta[:N] = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(tags), dtype=np.int64)).to(dev)
        tb = torch.zeros(N + W, dtype=torch.int64, device=dev)
        st = d.stream
        # the replica's whole-event graph (d.cg: its sender schedule lists every sender); self.cg's
        # schedule holds only this rank's senders
        nat.check(d.lib.gtf_tag_prepare(ctypes.byref(d.cg), vp(r), vp(keep), vp(proc), vp(cnt), st))
        total = int(cnt[0].item())
        hist = []
        frac = 1.0
        while frac > threshold and len(hist) < max_sweeps:
            nat.check(d.lib.gtf_tag_sweep_shard(ctypes.byref(self.cg), vp(keep), vp(proc), vp(ta), vp(tb),
                                                ctypes.byref(self.shard), self.rank, W, st))
            allreduce_max_i64(tb, self.backend, self.group)
            f = int(tb[N:].sum().item())
            hist.append(f)
            frac = f / total if total else 0.0
            ta, tb = tb, ta
        out = ta[:N].cpu().numpy()
        h = np.empty_like(out)
        h[d.order] = out
        return h, hist

    def owned_host_nodes(self) -> np.ndarray:
        """host indices of this rank's receivers (their results are final on this rank)"""
        r = self.rank
        return self.d.order[self.plan.node_lo[r]:self.plan.node_hi[r]]

    def owned_host_slots(self) -> np.ndarray:
        r = self.rank
        return self.d.slot_perm[self.plan.slot_lo[r]:self.plan.slot_hi[r]]


class SplitDeviceGraph:
    """One event's pass on ONE GPU as two receiver wedges run concurrently on two HIP
    streams (the tail of each half's kernels overlaps the other's): two replicas of the
    sharded layout (ShardedDeviceGraph with world 2) in this process, each on its own
    stream; after both halves, each half's halo goes to the other through device memory
    (the sender's halo_pack buffer is the receiver's unpack input -- for two parts the
    send layout of one is the receive layout of the other), and the streams join. The
    results equal the one-stream pass bit for bit (tests/test_gpu_split.py); each half's
    owned receivers are final in its own replica (download() merges them).

    Measured on C4 (tools/overlap_probe.py): two halves on two streams 129-136 us against
    147-152 us for the one-stream pass; three parts no better, four slower."""

    PARTS = 2

    def __init__(self, g: TrackGraph, device="cuda"):
        import torch
        self.torch = torch
        self.streams = [torch.cuda.Stream(device) for _ in range(self.PARTS)]
        self.parts = []
        for r in range(self.PARTS):
            with torch.cuda.stream(self.streams[r]):
                sd = ShardedDeviceGraph(g, r, self.PARTS, device, backend="local")
                sd._io()                        # fixes the part's stream: streams[r]
                self.parts.append(sd)
        self._ev = [[torch.cuda.Event() for _ in range(self.PARTS)] for _ in range(2)]   # packed, done
        self.n_edges, self.n_nodes = g.n_edges, g.n_nodes

    # ------------------------------------------------------------------ staging
    def snapshot(self):
        from .device import DeviceGraph
        return [sd.d.snapshot(DeviceGraph.PASS_INPUTS) for sd in self.parts]

    def stage_inputs(self, k: int):
        for r, sd in enumerate(self.parts):
            with self.torch.cuda.stream(self.streams[r]):
                sd.d.stage_inputs(k)

    def fill_inputs(self, snaps):
        for r, sd in enumerate(self.parts):
            with self.torch.cuda.stream(self.streams[r]):
                sd.d.fill_inputs(snaps[r])

    def use_inputs(self, i):
        for sd in self.parts:
            sd.d.use_inputs(i)

    def clear_errors(self):
        for r, sd in enumerate(self.parts):
            with self.torch.cuda.stream(self.streams[r]):
                sd.d.clear_errors()

    def errors(self) -> int:
        f = 0
        for r, sd in enumerate(self.parts):
            with self.torch.cuda.stream(self.streams[r]):
                f |= sd.d.errors()
        return f

    # ------------------------------------------------------------------ the pass
    def step(self, p, exchange=True, join=True, linear=False):
        """the pass of the whole event: both halves concurrently, then the halo exchange
        through device memory, then the two streams join (every later call on either
        stream sees the whole pass). exchange / join False: diagnostics timings only.
        linear: the exchange joined into the first stream instead -- it waits for the second
        half's pack and runs both unpacks, and the second stream then waits for it -- one
        cross-stream dependency at a time (the mutual mid-capture waits of the default form
        crash hipStreamEndCapture on this stack, profiles/r04/capture/)."""
        if not linear and self.torch.cuda.is_current_stream_capturing():
            # the joined form's mutual mid-capture waits crash hipStreamEndCapture on this stack:
            # a capture always records the one-way (linear) form, which replays bit-equal
            linear = True
        (a, b), (sa, sb) = self.parts, self.streams
        packed, done = self._ev
        for r, sd in enumerate(self.parts):
            sd.pass_(p)
            if exchange:
                sd.halo_pack()
                packed[r].record(self.streams[r])
        if exchange and linear:
            sa.wait_event(packed[1])
            a.halo_unpack(ctypes.c_void_p(b.send_buf.data_ptr()))
            b.halo_unpack(ctypes.c_void_p(a.send_buf.data_ptr()), stream=sa)
            if join:
                done[0].record(sa)
                sb.wait_event(done[0])
            return
        if exchange:
            sa.wait_event(packed[1])
            a.halo_unpack(ctypes.c_void_p(b.send_buf.data_ptr()))
            sb.wait_event(packed[0])
            b.halo_unpack(ctypes.c_void_p(a.send_buf.data_ptr()))
        if join:
            for r in range(self.PARTS):
                done[r].record(self.streams[r])
            sa.wait_event(done[1])   # the next pack on one stream must not overwrite a buffer the
            sb.wait_event(done[0])   # other is still unpacking

    def join(self, stream=None):
        """make `stream` (default: the current one) wait for both halves"""
        torch = self.torch
        s = stream or torch.cuda.current_stream()
        for r in range(self.PARTS):
            e = torch.cuda.Event()
            e.record(self.streams[r])
            s.wait_event(e)

    def download(self, g: TrackGraph) -> TrackGraph:
        """every half's owned receivers (and their slots) from its replica, host order"""
        from .graph import SLOT_FIELDS
        from .device import MUTABLE_NODE, STATIC_SLOT
        self.torch.cuda.synchronize()
        for sd in self.parts:
            h = sd.d.download(g.copy())
            nodes, slots = sd.owned_host_nodes(), sd.owned_host_slots()
            for f in MUTABLE_NODE:
                g.node[f][nodes] = h.node[f][nodes]
            for f in SLOT_FIELDS:
                if f in STATIC_SLOT or f == "slot_key":
                    continue
                g.slot[f][slots] = h.slot[f][slots]
        return g
