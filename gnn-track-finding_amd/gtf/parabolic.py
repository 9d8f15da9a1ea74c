"""Parabolic-model edge states and pairwise KL distances on the GPU.

Host side of ``gtf_parabolic_kl`` (include/gtf.h). It mirrors the reference's
training-data generator in learn_KL_parabolic_model/src/generate_training_data:

* ``compute_track_state_estimates`` (utils.py:221-289): per in-edge parabolic
  state ``edge_state_vector`` (3,) / ``edge_covariance`` (3, 3) and the node's
  ``xy_edge_gradient_mean_var``;
* ``calc_pairwise_distances`` + the row loop of
  extract_metadata_trackml_parabolic_model.py:15-99: one ``(kl_dist, emp_var,
  truth)`` row per pair i > j of the in-edges of every node with >= 2 in-edges.

Pairs are laid out node by node (node order), row-major lower triangle over the
node's in-slots (slot order = sender index order); ``ParabolicKL.pair_index``
gives each row's node and slot positions. The reference orders its rows by glob()
file order and dict order, which carry no meaning; the row
multiset is what parity is checked on.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _native as nat
from .graph import TrackGraph

BUCKETS = ((1, 2), (3, 4), (5, 8), (9, 1 << 30))   # in-degree ranges of the 1/4/8/64-lane groups
TILE_MAX = 256   # bucket-0 nodes per tile of the tiled layout (one per thread of a gtf_kl.hip WBLOCK)
WIN_NODES = 1024   # LDS window of a tile (gtf_kl.hip WWIN)
WIN_MARGIN = 128   # window nodes either side of a tile (99 % of the vol-7 neighbours lie within 73)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def in_edge_csr(g: TrackGraph):
    """(slot_ptr, slot_src) of the graph's in-edges (slots that are edges)."""
    ise = g.slot["is_edge"].astype(bool)
    if ise.all():
        return g.slot_ptr.astype(np.int32), g.slot["slot_src"].astype(np.int32)
    dst = g.slot_dst()
    cnt = np.bincount(dst[ise], minlength=g.n_nodes)
    ptr = np.zeros(g.n_nodes + 1, np.int32)
    np.cumsum(cnt, out=ptr[1:])
    return ptr, g.slot["slot_src"][ise].astype(np.int32)


class ParabolicKL:
    """Device-resident KL graph of one or many events (events concatenated into one CSR).

    ordered: the nodes are renumbered on upload so that each in-degree bucket is one node
    range -- one-edge nodes, two-edge nodes, then the 3..4, 5..8 and > 8 buckets, then the
    unlisted nodes -- with slots and pairs following node order (gtf_kl_graph's ordered
    layout: the kernel reaches the two-edge bucket by arithmetic). Device outputs are then
    in that order: ``node_of`` maps a device node to the caller's, pair_index() returns the
    caller's node ids, and ``host_nodes`` / ``host_slots`` reorder per-node / per-slot
    outputs; pairs keep the caller's (node, i, j) rows through pair_index().

    tile = T > 0 (T <= 256): the nodes azimuth-sorted inside sort windows (an event of a
    batch), then cut into tiles of T one- / two-edge (bucket-0) nodes and whatever lies
    between them, each tile with its bucket-0 nodes first: one 256-thread block per tile
    record (gtf_kl_graph.blk) loads its nodes' sender lists and the coordinates of a window
    of consecutive nodes around the tile -- where a hit's neighbours lie -- in one round,
    and reads the neighbours from LDS. The 3..4, 5..8 and > 8 buckets go by node list."""

    def __init__(self, slot_ptr, slot_src, gnn, truth=None, device="cuda", with_single=False, ordered=False,
                 tile=0, sort_window=8192, tile_b1=True):
        slot_ptr = np.ascontiguousarray(slot_ptr, np.int32)
        self.n_nodes = int(slot_ptr.shape[0] - 1)
        self.n_slots = int(slot_ptr[-1])
        d = np.diff(slot_ptr).astype(np.int64)
        lo = 1 if with_single else 2
        self.node_of = self.slot_of = None
        self.tile = int(tile)
        ordered = ordered or self.tile > 0
        if ordered:
            sp = slot_ptr.astype(np.int64)
            # buckets 1 and 2 as runs of one in-degree each (3, 4 | 5, 6, 7, 8), then the > 8 bucket
            keys = [d == 1 if lo == 1 else np.zeros(d.size, bool)] + [d == q for q in range(2, 9)] + [d > 8]
            rank = np.full(d.size, len(keys), np.int64)
            for q in reversed(range(len(keys))):
                rank[keys[q]] = q
            if self.tile > 0:   # azimuth order in sort windows, cut into tiles of T bucket-0 nodes
                if not 0 < self.tile <= TILE_MAX:
                    raise ValueError("tile must be in 1..%d" % TILE_MAX)
                xy = np.asarray(gnn, np.float64).reshape(-1, 4)
                phi = np.arctan2(xy[:, 1], xy[:, 0])
                idx = np.arange(d.size, dtype=np.int64)
                o1 = np.lexsort((idx, phi, idx // sort_window))
                self.tile_b1 = bool(tile_b1)
                b0 = rank[o1] < (4 if self.tile_b1 else 2)          # the nodes a tile's threads take
                tid = np.empty(d.size, np.int64)
                tid[o1] = (np.cumsum(b0) - b0) // self.tile         # a tile: T such nodes and the rest between
                order = np.lexsort((np.argsort(o1), rank, tid))
                self._tiles = (tid[order], rank[order])
            else:
                order = np.argsort(rank, kind="stable")
            nd = d[order]
            new_ptr = np.zeros(self.n_nodes + 1, np.int64)
            np.cumsum(nd, out=new_ptr[1:])
            owner = np.repeat(np.arange(self.n_nodes), nd)
            slot_of = sp[order][owner] + (np.arange(self.n_slots) - new_ptr[owner])
            inv = np.empty(self.n_nodes, np.int64)
            inv[order] = np.arange(self.n_nodes)
            slot_src = inv[np.asarray(slot_src, np.int64)[slot_of]]
            gnn = np.asarray(gnn, np.float64).reshape(-1, 4)[order]
            truth = np.asarray(truth, np.int64)[order] if truth is not None else None
            slot_ptr = new_ptr.astype(np.int32)
            d = nd
            self.node_of, self.slot_of = order, slot_of
            self._ranges = [int(k.sum()) for k in keys]
        self.slot_ptr_host = np.asarray(slot_ptr, np.int64)
        npair = np.where(d >= 2, d * (d - 1) // 2, 0)
        pair_ptr = np.zeros(self.n_nodes + 1, np.int64)
        np.cumsum(npair, out=pair_ptr[1:])
        self.n_pairs = int(pair_ptr[-1])
        lists = [np.nonzero((d >= max(a, lo)) & (d <= b))[0].astype(np.int32) for a, b in BUCKETS]
        self.n_listed = int(sum(x.size for x in lists))
        self.degree = d
        self.pair_ptr_host = pair_ptr
        dev = torch.device(device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.slot_ptr = t(slot_ptr)
        self.slot_src = t(np.asarray(slot_src, np.int32))
        # the kernel reads GNN_Measurement x and y only: a compact [N, 2] copy (gnn_stride 2)
        # halves the bytes of the node and neighbour coordinate gathers
        self.gnn = t(np.asarray(gnn, np.float64).reshape(-1, 4)[:, :2])
        self.truth = t(np.asarray(truth, np.int64)) if truth is not None else None
        self.pair_ptr = t(pair_ptr)
        self.lists = [t(x) for x in lists]
        self.device = dev
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        if self.tile > 0:   # one block record per tile (gtf_kl_graph.blk); buckets 1..3 by list
            blk = self._block_table(d, pair_ptr)
            self.blk = t(blk)
            self.n_blk = int(blk.size // 12)
            by_list = [q >= (2 if self.tile_b1 else 1) and self.lists[q].numel() > 0 for q in range(4)]
            self._g = nat.GtfKlGraph(self.n_nodes, self.n_slots, _ptr(self.slot_ptr), _ptr(self.slot_src),
                                     _ptr(self.gnn), _ptr(self.truth), _ptr(self.pair_ptr),
                                     (ctypes.c_void_p * 4)(*[x.data_ptr() if b else None
                                                             for x, b in zip(self.lists, by_list)]),
                                     (ctypes.c_int32 * 4)(*[x.numel() if b else 0 for x, b in zip(self.lists, by_list)]),
                                     (ctypes.c_int32 * 4)(), 0, 2, 0, 0, _ptr(self.blk), self.n_blk)
        elif ordered:   # bucket ranges, no lists
            n1, n2 = self._ranges[0], self._ranges[1]
            counts = [n1 + n2] + [int(x.size) for x in lists[1:]]
            first = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
            self._g = nat.GtfKlGraph(self.n_nodes, self.n_slots, _ptr(self.slot_ptr), _ptr(self.slot_src),
                                     _ptr(self.gnn), _ptr(self.truth), _ptr(self.pair_ptr),
                                     (ctypes.c_void_p * 4)(), (ctypes.c_int32 * 4)(*counts),
                                     (ctypes.c_int32 * 4)(*first.tolist()), n1, 2, 0, 0)
            if os.environ.get("GTF_KL_DEG_RUNS", "1") != "0":   # degree runs (0: the round-3 ordered form)
                self._g.deg_runs = 1
                for q in range(6):
                    self._g.n_deg[q] = self._ranges[2 + q]
        else:
            self._g = nat.GtfKlGraph(self.n_nodes, self.n_slots, _ptr(self.slot_ptr), _ptr(self.slot_src),
                                     _ptr(self.gnn), _ptr(self.truth), _ptr(self.pair_ptr),
                                     (ctypes.c_void_p * 4)(*[x.data_ptr() if x.numel() else None for x in self.lists]),
                                     (ctypes.c_int32 * 4)(*[x.numel() for x in self.lists]), gnn_stride=2)

    def _block_table(self, d, pair_ptr, margin=WIN_MARGIN):   # (rank < 16: 10 keys)
        """gtf_kl_graph.blk of the tiled layout: one record of 12 int32 per tile (first node,
        bucket-0 count, its one-edge count, the three- and four-edge counts that follow (0 and
        0 unless tile_b1), 0, bucket 0's first slot, its first pair lo / hi, the window
        [lo, hi) -- the tile's nodes and `margin` nodes either side, at most WIN_NODES -- 0)"""
        tid, rank = self._tiles
        sp = self.slot_ptr_host
        n = tid.size
        nt = int(tid.max()) + 1 if n else 0
        bounds = np.searchsorted(tid, np.arange(nt + 1))
        a, b = bounds[:-1], bounds[1:]
        n1 = np.searchsorted(tid * 16 + rank, tid[a] * 16 + 1) - a if nt else a   # rank-0 run at the tile head
        n0 = np.searchsorted(tid * 16 + rank, tid[a] * 16 + 2) - a if nt else a
        z = np.zeros(nt, np.int64)
        n3 = n4 = z
        if self.tile_b1 and nt:
            n3 = np.searchsorted(tid * 16 + rank, tid[a] * 16 + 3) - a - n0
            n4 = np.searchsorted(tid * 16 + rank, tid[a] * 16 + 4) - a - n0 - n3
        pr = pair_ptr[a]   # (one-edge nodes have no pairs: the first two-edge node's, then the 3- / 4-edge nodes')
        span = b - a
        m = np.clip((WIN_NODES - span) // 2, 0, margin)
        wlo = np.maximum(a - m, 0)
        whi = np.minimum(np.minimum(b + m, n), wlo + WIN_NODES)
        # one thread per node of the tile's bucket 0 and its in-tile 3- / 4-edge nodes: a
        # 256-thread block (gtf_kl.hip) would skip any beyond 256 without an error
        if nt and int((n0 + n3 + n4).max()) > 256:
            raise ValueError("KL tile with %d one- to four-edge nodes (the block handles at most 256)"
                             % int((n0 + n3 + n4).max()))
        recs = np.stack([a, n0, n1, n3, n4, z, sp[a], pr & 0xFFFFFFFF, pr >> 32, wlo, whi, z], 1)
        recs = np.where(recs >= 2**31, recs - 2**32, recs)   # low words as int32 bits
        return recs.astype(np.int32).reshape(-1)

    def replica(self, gnn=None):
        """An independent copy of this batch in its own device buffers (same structure):
        ``gnn`` (caller's node order, [N, 4] or [N, 2]) replaces the coordinates, e.g. a
        batch jittered with another seed. Used to rotate launches over several resident
        batches so that no launch finds its inputs in the caches (bench.py, config 5)."""
        import copy
        r = copy.copy(self)
        cl = lambda t: t.clone() if t is not None else None  # noqa: E731
        r.slot_ptr, r.slot_src, r.pair_ptr = cl(self.slot_ptr), cl(self.slot_src), cl(self.pair_ptr)
        r.truth = cl(self.truth)
        r.lists = [cl(x) for x in self.lists]
        if getattr(self, "blk", None) is not None:
            r.blk = cl(self.blk)
        r.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        if gnn is None:
            r.gnn = cl(self.gnn)
        else:
            gh = np.asarray(gnn, np.float64)[:, :2]
            if self.node_of is not None:
                gh = gh[self.node_of]
            r.gnn = torch.from_numpy(np.ascontiguousarray(gh)).to(self.device)
        g = nat.GtfKlGraph.from_buffer_copy(self._g)
        g.slot_ptr, g.slot_src, g.gnn = _ptr(r.slot_ptr), _ptr(r.slot_src), _ptr(r.gnn)
        g.truth, g.pair_ptr = _ptr(r.truth), _ptr(r.pair_ptr)
        if getattr(r, "blk", None) is not None:
            g.blk = _ptr(r.blk)
        for q in range(4):
            if g.list[q]:
                g.list[q] = r.lists[q].data_ptr() if r.lists[q].numel() else None
        r._g = g
        return r

    def footprint_bytes(self, out) -> int:
        """device bytes of this batch's inputs and the outputs in ``out``"""
        ts = [self.slot_ptr, self.slot_src, self.gnn, self.truth, self.pair_ptr] + list(self.lists)
        ts += [v for k, v in out.items() if k not in ("kl", "truth")]   # (views of _kl / _truth)
        seen, tot = set(), 0
        for t in ts:
            if t is None or t.data_ptr() in seen:
                continue
            seen.add(t.data_ptr())
            tot += t.numel() * t.element_size()
        return tot

    @classmethod
    def from_graph(cls, g: TrackGraph, truth=None, device="cuda", with_single=False):
        ptr, src = in_edge_csr(g)
        return cls(ptr, src, g.node["gnn"], truth, device, with_single)

    def alloc(self, dtype="f64", truth=True, emp=True, states=False):
        f = torch.float64 if dtype == "f64" else torch.float32
        # pair buffers hold >= 1 element so their pointers are never null, even with no
        # pairs (the C-ABI rejects null outputs); "kl"/"truth" are views of the pair count
        z = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=self.device)  # noqa: E731
        out = {"_kl": z(self.n_pairs, f)}
        out["kl"] = out["_kl"][:self.n_pairs]
        if truth and self.truth is not None:
            out["_truth"] = z(self.n_pairs, torch.int8)
            out["truth"] = out["_truth"][:self.n_pairs]
        if emp:     # True: gradient mean and variance; "var": variance only (the training rows)
            out["emp_var"] = torch.full((self.n_nodes,), float("nan"), dtype=torch.float64, device=self.device)
            if emp is True:
                out["emp_mean"] = torch.full((self.n_nodes,), float("nan"), dtype=torch.float64,
                                             device=self.device)
        if states:
            out["sv"] = torch.full((self.n_slots, 3), float("nan"), dtype=torch.float64, device=self.device)
            out["cov"] = torch.full((self.n_slots, 3, 3), float("nan"), dtype=torch.float64, device=self.device)
        return out

    def run(self, out, dtype="f64", stream=None):
        """launch gtf_parabolic_kl into the buffers of ``alloc`` (stream-ordered)."""
        o = nat.GtfKlOut(_ptr(out["_kl"]), _ptr(out.get("_truth")), _ptr(out.get("emp_var")),
                         _ptr(out.get("emp_mean")), _ptr(out.get("sv")), _ptr(out.get("cov")), _ptr(self.err))
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        nat.check(nat.lib().gtf_parabolic_kl(ctypes.byref(self._g), nat.GTF_F64 if dtype == "f64" else nat.GTF_F32,
                                             ctypes.byref(o), ctypes.c_void_p(s.cuda_stream)))
        return out

    def errors(self):
        return int(self.err.item())

    def pair_index(self, device_nodes=False):
        """(node, i, j) of every pair row (host); node in the caller's numbering unless
        device_nodes (the ordered layout's own)."""
        d = self.degree
        nodes = np.nonzero(d >= 2)[0]
        node = np.repeat(nodes, (d[nodes] * (d[nodes] - 1) // 2))
        t = np.arange(self.n_pairs, dtype=np.int64) - self.pair_ptr_host[node]
        i = np.floor((1 + np.sqrt(1 + 8 * t.astype(np.float64))) / 2).astype(np.int64)
        i -= (i * (i - 1) // 2 > t)
        i += ((i + 1) * i // 2 <= t)
        if self.node_of is not None and not device_nodes:
            node = self.node_of[node]
        return node, i, t - i * (i - 1) // 2

    def host_nodes(self, a):
        """a per-node device output (array, first axis = node) in the caller's node order"""
        a = np.asarray(a)
        if self.node_of is None:
            return a
        out = np.empty_like(a)
        out[self.node_of] = a
        return out

    def host_slots(self, a):
        """a per-slot device output in the caller's slot order"""
        a = np.asarray(a)
        if self.slot_of is None:
            return a
        out = np.empty_like(a)
        out[self.slot_of] = a
        return out


def training_rows(g: TrackGraph, truth=None, dtype="f64", device="cuda"):
    """(node, i, j, kl_dist, emp_var, truth) rows of extract_metadata_trackml_parabolic_model.py
    for one event graph, computed on the GPU."""
    ptr, src = in_edge_csr(g)
    return training_rows_csr(ptr, src, g.node["gnn"], truth, dtype, device)


def training_rows_csr(slot_ptr, slot_src, gnn, truth=None, dtype="f64", device="cuda"):
    k = ParabolicKL(slot_ptr, slot_src, gnn, truth, device)
    out = k.run(k.alloc(dtype, truth=truth is not None, emp="var"), dtype)
    node, i, j = k.pair_index()
    ev = out["emp_var"].cpu().numpy()[node]
    tr = out["truth"].cpu().numpy() if "truth" in out else np.zeros(k.n_pairs, np.int8)
    flags = k.errors()
    if flags:
        raise np.linalg.LinAlgError(nat.ERR_FLAGS[128])
    return node, i, j, out["kl"].cpu().numpy(), ev, tr


def compute_track_state_estimates(g: TrackGraph, device="cuda"):
    """Per in-edge parabolic states and per-node gradient (mean, var) of one graph
    (utils.py:221-289): returns (sv [S,3], cov [S,3,3], grad_mean [N], grad_var [N]),
    slots in the graph's in-edge order."""
    k = ParabolicKL.from_graph(g, None, device, with_single=True)
    out = k.run(k.alloc("f64", truth=False, emp=True, states=True), "f64")
    if k.errors():
        raise np.linalg.LinAlgError(nat.ERR_FLAGS[128])
    return (out["sv"].cpu().numpy(), out["cov"].cpu().numpy(), out["emp_mean"].cpu().numpy(),
            out["emp_var"].cpu().numpy())


def batch(slot_ptr, slot_src, gnn, truth, n_events, jitter=1e-3, seed=0):
    """n_events copies of one event concatenated into one CSR (the config-5 batch):
    copy e > 0 has every hit moved by a seeded N(0, jitter) mm in x and y, so the
    events differ. Truth ids repeat per copy (pairs never span copies)."""
    rng = np.random.default_rng(seed)
    n, s = gnn.shape[0], slot_src.shape[0]
    ptrs = [np.asarray(slot_ptr[:-1], np.int64) + e * s for e in range(n_events)] + [np.array([n_events * s])]
    src = np.concatenate([np.asarray(slot_src, np.int64) + e * n for e in range(n_events)])
    g = np.tile(np.asarray(gnn, np.float64), (n_events, 1))
    g[n:, :2] += rng.normal(0.0, jitter, (g.shape[0] - n, 2))
    tr = np.tile(np.asarray(truth, np.int64), n_events) if truth is not None else None
    return np.concatenate(ptrs).astype(np.int32), src.astype(np.int32), g, tr
