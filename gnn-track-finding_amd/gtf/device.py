"""Device-resident TrackGraph and the stage entry points (host side of the C-ABI).

``DeviceGraph`` uploads a :class:`gtf.graph.TrackGraph` into HBM once (torch
tensors are used only as device allocations; every computation runs in
libgtf.so's HIP kernels), then the stage methods call the C-ABI on the current
HIP stream. ``download`` copies the mutable arrays back for unpacking.

Stage methods mirror the reference's stage bodies:
  extrapolate() -> src/extrapolate/extrapolate_merged_states.py:552-566
  update()      -> src/update/remove_state_metadata.py:29-53
  cluster()     -> src/clustering/clustering.py:181-373
  full_pass()   -> the three in run_gnn_trackml_mod.sh order (extrapolate,
                   update, cluster on updated_track_states), fused
  tag_propagation() -> tag_propagation/tag_propagation.py:97-164
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat
from .graph import BUCKETS, TrackGraph, NODE_FIELDS, SLOT_FIELDS, padded, renumber
from .params import Params

STATIC_SLOT = ("slot_src", "is_edge", "rev_edge", "send_mw")
MUTABLE_NODE = ("has_merged", "merged_state", "merged_cov", "merged_prior", "has_tse", "has_uts", "degree")
STATE_FIELDS = ("rank", "sv", "tau", "cov", "xyzr", "lik", "mw", "prior", "lr", "side", "fresh")


def sched_segments(slot_ptr, sched):
    """gtf_graph.sched_seg: (slot_ptr[v], slot_ptr[v + 1]) of every schedule entry v"""
    sp = np.asarray(slot_ptr, dtype=np.int64)
    v = np.asarray(sched, dtype=np.int64)
    return np.stack([sp[v], sp[v + 1]], axis=1).astype(np.int32).reshape(-1)


def sender_schedule(out_ptr, nodes=None):
    """gtf_graph.out_sched: (sender, out begin, out end, 0) of every node with an
    out-edge (or of the given nodes: a shard's senders), bucketed by out-degree 1..4 /
    5..8 / more; returns (array, counts)"""
    op = np.asarray(out_ptr, dtype=np.int64)
    idx = np.arange(op.size - 1, dtype=np.int64) if nodes is None else np.asarray(nodes, dtype=np.int64)
    od = op[idx + 1] - op[idx]
    parts = [idx[(od >= 1) & (od <= 4)], idx[(od >= 5) & (od <= 8)], idx[od > 8]]
    u = np.concatenate(parts).astype(np.int64)
    q = np.stack([u, op[u], op[u + 1], np.zeros_like(u)], axis=1).astype(np.int32).reshape(-1)
    return q, [int(x.size) for x in parts]


def sender_lanes(out_slot, out_dst, q, counts):
    """gtf_graph.out_lanes: for every lane of the 4- and 8-lane entries of the sender
    schedule `q` (sender_schedule), (slot, receiver) of the lane's out-edge or (-1, 0)"""
    q = np.asarray(q, dtype=np.int64).reshape(-1, 4)
    os_ = np.asarray(out_slot, dtype=np.int64)
    od = np.asarray(out_dst, dtype=np.int64)
    parts, at = [], 0
    for G, n in ((4, counts[0]), (8, counts[1])):
        e = q[at:at + n]
        at += n
        idx = e[:, 1:2] + np.arange(G)[None, :]
        ok = idx < e[:, 2:3]
        safe = np.minimum(idx, max(os_.size - 1, 0))
        k = np.where(ok, os_[safe] if os_.size else -1, -1)
        v = np.where(ok, od[safe] if od.size else 0, 0)
        parts.append(np.stack([k, v], axis=2).reshape(-1))
    return np.concatenate(parts).astype(np.int32) if parts else np.zeros(0, np.int32)


def pack_schedule(slot_ptr):
    """gtf_graph.pack_ent / pack_wave: the nodes with <= 64 slots, largest first, packed
    greedily into wavefronts of 64 lanes (one lane per slot, one for a slot-free node);
    returns (entries [4*n] int32 (v, lo, hi, first lane), wave_ptr [W+1] int32)"""
    sp = np.asarray(slot_ptr, dtype=np.int64)
    deg = np.diff(sp)
    idx = np.nonzero(deg <= 64)[0]
    order = idx[np.argsort(-deg[idx], kind="stable")]
    size = np.maximum(deg[order], 1)
    off = np.empty(order.size, np.int64)
    starts = [0]
    used = 0
    for i, z in enumerate(size.tolist()):
        if used + z > 64:
            starts.append(i)
            used = 0
        off[i] = used
        used += z
    starts.append(order.size)
    ent = np.stack([order, sp[order], sp[order + 1], off], axis=1).astype(np.int32).reshape(-1)
    wave = np.asarray(starts if order.size else [0], dtype=np.int32)
    return ent, wave


CLASS_MAX = 32   # segments of up to this many slots get graph-static classes (gtf_graph.slot_class)
XCLASS_MAX = 64  # 33..64-slot segments: the layer classes in slot_class, the x ones in slot_xclass (ABI v7)
CLASS_MIN_SLOTS = 1 << 16   # graphs this large get them by default (the host pass: ~4 ms on 15k slots)


def slot_classes(g: TrackGraph):
    """gtf_graph.slot_class / slot_sflags (ABI v5) / slot_xclass (v7): for every slot of a receiver segment of
    d <= 32 slots, bits 0..31 = the segment positions whose sender has this slot's sender
    layer (compute_prior_probabilities' groups, helper.py:30-63), bits 32..63 = the positions
    whose sender's GNN x equals this slot's sender's (the side norm's distinct-x classes,
    helper.py:111-139, for entries holding their sender's live coordinates); a NaN (orphan
    key) equals only itself. sflags bit 0 = sender GNN x < receiver GNN x (the side,
    helper.py:116-121). Segments of 33..64 slots (v7): all 64 bits of slot_class are the
    layer positions and slot_xclass holds the x positions. Larger segments get 0 (the kernel
    builds their classes)."""
    S = g.n_slots
    cls = np.zeros(S, np.uint64)
    src = g.slot["slot_src"].astype(np.int64)
    ok = src >= 0
    layer = np.full(S, np.nan)
    sx = np.full(S, np.nan)
    if g.n_nodes:
        layer[ok] = g.node["layer"][src[ok]]
        sx[ok] = g.node["gnn"][src[ok], 0]
    rx = g.node["gnn"][g.slot_dst(), 0] if S else np.zeros(0)
    with np.errstate(invalid="ignore"):
        sfl = (sx < rx).astype(np.uint8)
    sp = g.slot_ptr.astype(np.int64)
    deg = np.diff(sp)
    xcls = np.zeros(S, np.uint64)
    for d in range(1, XCLASS_MAX + 1):
        v = np.nonzero(deg == d)[0]
        if v.size == 0:
            continue
        idx = sp[v][:, None] + np.arange(d)[None, :]                 # [n, d] slots
        own = np.eye(d, dtype=bool)[None, :, :]
        bits = (np.uint64(1) << np.arange(d, dtype=np.uint64))[None, None, :]
        masks = []
        for val in (layer, sx):
            a = val[idx]
            eq = (a[:, :, None] == a[:, None, :]) | own              # [n, i, j]
            masks.append(np.bitwise_or.reduce(np.where(eq, bits, np.uint64(0)), axis=2))
        if d <= CLASS_MAX:   # both in one word
            cls[idx.reshape(-1)] = (masks[0] | (masks[1] << np.uint64(32))).reshape(-1)
        else:                # 33..64 slots: the layer positions in slot_class, the x ones in slot_xclass
            cls[idx.reshape(-1)] = masks[0].reshape(-1)
            xcls[idx.reshape(-1)] = masks[1].reshape(-1)
    return cls, sfl, xcls


STATIC_MAX = 8   # segments of up to this many slots get gtf_graph.slot_static words


def slot_static_words(g: TrackGraph, cls: np.ndarray, sfl: np.ndarray) -> np.ndarray:
    """gtf_graph.slot_static (ABI v7): for a slot of a segment of d <= 8 slots, its class bits
    (same layer: bits 0..7, same x: bits 8..15), is_edge (16), rev_edge (17) and side flag
    (18) in one uint32; 0 for larger segments"""
    deg = np.diff(g.slot_ptr.astype(np.int64))
    small = np.repeat(deg <= STATIC_MAX, deg)
    c = cls.astype(np.uint64)
    w = (c & np.uint64(0xff)) | (((c >> np.uint64(32)) & np.uint64(0xff)) << np.uint64(8))
    w = w.astype(np.uint32)
    w |= (g.slot["is_edge"].astype(np.uint32) & 1) << 16
    w |= (g.slot["rev_edge"].astype(np.uint32) & 1) << 17
    w |= (sfl.astype(np.uint32) & 1) << 18
    return np.where(small, w, np.uint32(0)).astype(np.uint32)


def slot_sender_xzr(g: TrackGraph) -> np.ndarray:
    """gtf_graph.slot_sxzr (ABI v7): per slot its sender's GNN_Measurement x, z, r
    (gnn[slot_src][0, 2, 3]), NaN rows for orphan keys; [S, 3] float64"""
    src = g.slot["slot_src"].astype(np.int64)
    out = np.full((g.n_slots, 3), np.nan)
    ok = src >= 0
    if g.n_nodes and ok.any():
        out[ok] = g.node["gnn"][src[ok]][:, [0, 2, 3]]
    return out


def live_coordinates(g: TrackGraph) -> np.ndarray:
    """gtf_states.fresh bit 1 for an uploaded graph: the updated_track_states entries whose
    stored 'xyzr' is bit for bit their sender's current GNN_Measurement coordinates (what
    extrapolate_merged_states.py:377 stores; a close-proximity merge of the sender since,
    extract_track_candidates.py:111-118, breaks it). Those entries' xyzr is read from gnn."""
    src = g.slot["slot_src"].astype(np.int64)
    ok = (src >= 0) & (g.slot["uts_rank"] >= 0)
    live = np.zeros(g.n_slots, bool)
    if ok.any():
        a = np.ascontiguousarray(g.slot["uts_xyzr"][ok]).view(np.int64)
        b = np.ascontiguousarray(g.node["gnn"][src[ok]]).view(np.int64)
        live[ok] = (a == b).all(axis=1)
    return live


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("gtf needs a HIP device (MI355X); torch.cuda.is_available() is False")
    return torch


def schedule_order(slot_ptr, tile=0):
    """node indices bucketed by slot count as the node-kernel schedule takes them
    (BUCKETS, then the nodes beyond 64 slots), node order inside a bucket. tile > 0:
    the same inside every run of `tile` consecutive nodes, tile after tile, so a bucket's
    nodes stay contiguous within a tile and spatially close nodes stay close"""
    deg = np.diff(np.asarray(slot_ptr, dtype=np.int64))
    idx = np.arange(deg.size, dtype=np.int64)
    bucket = np.full(deg.size, len(BUCKETS), np.int64)
    for q, (lo, hi) in reversed(list(enumerate(BUCKETS))):
        bucket[(deg >= lo) & (deg <= hi)] = q
    t = idx // tile if tile > 0 else np.zeros_like(idx)
    return np.lexsort((idx, bucket, t))


TILE = 4096   # nodes per tile of the "tiled" layout


class DeviceGraph:
    """pack: the fused pass's node kernel on packed variable-size lane segments
    (gtf_graph.pack_ent) instead of power-of-two lane groups -- same results, same speed
    on C4, kept as an option.
    layout "natural": the host graph's node and slot order. layout "schedule": nodes
    renumbered into schedule order (graph.renumber), so the lane groups of one
    wavefront take adjacent slot segments and every slot load of the node kernel is
    one contiguous run; download() maps the results back to the host order. The
    stage methods are layout-independent (the pass is equivariant under renumber)."""

    def __init__(self, g: TrackGraph, device: str = "cuda", schedule: bool = True, layout: str = "natural",
                 pack: bool = False, tile: int = TILE, mem: str = "torch", classes=None):
        """mem "torch": the arrays are torch tensors (every method). mem "hip": plain
        allocations from libgtf (gtf.devmem, no torch in the process): the stage methods,
        clear_errors / errors and download only -- the drop-in CLIs' path. classes: upload
        the graph-static slot classes (gtf_graph.slot_class); None = on graphs of at least
        CLASS_MIN_SLOTS slots."""
        if mem not in ("torch", "hip"):
            raise ValueError("mem must be 'torch' or 'hip'")
        self.mem = mem
        torch = _torch() if mem == "torch" else None
        self.layout = layout
        self.order = self.slot_perm = None
        self.pad_plan = None
        if layout in ("schedule", "tiled"):
            self.order = schedule_order(g.slot_ptr, tile if layout == "tiled" else 0)
            g, self.slot_perm = renumber(g, self.order)
        elif layout == "padded":   # padded tiles (graph.padded): dummy nodes / padding slots map to -1
            g, self.order, self.slot_perm, self.pad_plan = padded(g, tile)
        elif layout != "natural":
            raise ValueError("layout must be 'natural', 'schedule', 'tiled' or 'padded'")
        self.slot_ptr_host = g.slot_ptr
        self.torch = torch
        if torch is not None:
            self.device = torch.device(device)
            self.lib = nat.lib()
        else:
            self.device = device
            self.lib = nat.lib(lean=True)
            nat.check(self.lib.gtf_device_init(int(device.split(":")[1]) if ":" in device else 0))
        self.n_nodes, self.n_slots, self.n_edges = g.n_nodes, g.n_slots, g.n_edges
        self.t = {}
        up = self._up
        up("slot_ptr", g.slot_ptr.astype(np.int32))
        up("out_ptr", g.out_ptr.astype(np.int32))
        up("out_slot", g.out_slot.astype(np.int32))
        up("slot_dst", g.slot_dst().astype(np.int32))
        out_dst = g.slot_dst()[g.out_slot].astype(np.int32) if g.n_edges else np.zeros(0, np.int32)
        up("out_dst", out_dst)
        src = g.slot["slot_src"].astype(np.int64)
        up("slot_layer", np.where(src >= 0, g.node["layer"][np.maximum(src, 0)] if g.n_nodes else np.nan,
                                  np.nan).astype(np.float64))
        outpos = np.full(g.n_slots, -1, np.int32)
        if g.n_edges:
            owner = np.repeat(np.arange(g.n_nodes, dtype=np.int64), np.diff(g.out_ptr.astype(np.int64)))
            outpos[g.out_slot] = (np.arange(g.n_edges) - g.out_ptr[owner]).astype(np.int32)
        up("slot_outpos", outpos)
        # global out-edge index of every slot's edge (gtf_graph.slot_outidx): the sender scan
        # stores its running values in out-edge order (GTF_NO_OUTIDX=1: by slot, for A/B)
        import os
        self.use_outidx = os.environ.get("GTF_NO_OUTIDX", "0") != "1"
        # graph-static slot classes for the node kernel on graphs of >= CLASS_MIN_SLOTS slots
        # (smaller ones -- a drop-in stage's directory -- have the kernel build them: the host
        # pass would cost more than it saves); classes=True / False forces either way,
        # GTF_NO_CLASSES=1 turns them off (A/B)
        self.use_classes = (classes if classes is not None else g.n_slots >= CLASS_MIN_SLOTS) and \
            os.environ.get("GTF_NO_CLASSES", "0") != "1"
        oidx = np.full(g.n_slots, -1, np.int32)
        if g.n_edges:
            oidx[g.out_slot] = np.arange(g.n_edges, dtype=np.int32)
        up("slot_outidx", oidx)
        if self.use_classes:
            cls, sfl, xcls = slot_classes(g)
            up("slot_class", cls.view(np.int64))
            up("slot_sflags", sfl)
            up("slot_xclass", xcls.view(np.int64))
        # the senders' GNN x, z, r per slot (gtf_graph.slot_sxzr): a live UTS entry's stored
        # coordinates, read contiguously by the clustering instead of gathered per state
        # (GTF_NO_SXZR=1: gathered, for A/B)
        self.use_sxzr = self.use_classes and os.environ.get("GTF_NO_SXZR", "0") != "1"
        if self.use_sxzr:
            up("slot_sxzr", slot_sender_xzr(g))
        # the static slot fields of <= 8-slot segments in one word (gtf_graph.slot_static;
        # GTF_NO_STATIC32=1: the separate arrays, for A/B)
        self.use_static32 = self.use_classes and os.environ.get("GTF_NO_STATIC32", "0") != "1"
        if self.use_static32:
            up("slot_static", slot_static_words(g, cls, sfl).view(np.int32))
        sub = g.node["sub_id"].astype(np.int64)
        if g.n_nodes:
            sizes = np.bincount(sub - sub.min())
            solo = (sizes[sub - sub.min()] == 1).astype(np.uint8)
        else:
            solo = np.zeros(0, np.uint8)
        up("solo", solo)
        # slot-count-bucketed node schedule for the node-local kernels (G lanes per node)
        deg = np.diff(g.slot_ptr.astype(np.int64))
        idx = np.arange(g.n_nodes, dtype=np.int32)
        buckets = [idx[(deg >= lo) & (deg <= hi)] for lo, hi in BUCKETS]
        # the <= 2-slot nodes first in the <= 4-slot bucket: they run on 2 lanes (gtf_graph.n_g2)
        buckets[0] = np.concatenate([buckets[0][deg[buckets[0]] <= 2], buckets[0][deg[buckets[0]] > 2]])
        self.n_g2 = int((deg[buckets[0]] <= 2).sum())
        rest = idx[deg > 64]
        sched = np.concatenate(buckets + [rest]).astype(np.int32)
        up("sched", sched)
        up("sched_seg", sched_segments(g.slot_ptr, sched))
        osched, self.n_o = sender_schedule(g.out_ptr)
        up("out_sched", osched)
        up("out_lanes", sender_lanes(g.out_slot, out_dst, osched, self.n_o))
        self.n_pack_waves = 0
        if pack:   # the packed lane segments are built only when asked for
            pent, pwave = pack_schedule(g.slot_ptr)
            up("pack_ent", pent)
            up("pack_wave", pwave)
            self.n_pack_waves = int(pwave.size - 1)
        self.n_g_all = [int(b.size) for b in buckets]
        self.n_big = int(rest.size)
        self.n_g = self.n_g_all if schedule else [0] * len(BUCKETS)
        self.use_sched = schedule
        for f in ("gnn", "xyzr", "layer") + MUTABLE_NODE:
            up(f, g.node[f])
        for f in SLOT_FIELDS:
            if f in ("slot_key",):
                continue
            if f == "uts_fresh":   # bit 0: fresh; bit 1: the entry's xyzr is its sender's live gnn
                up(f, ((g.slot[f] != 0).astype(np.uint8) | (live_coordinates(g).astype(np.uint8) << 1)))
                continue
            up(f, g.slot[f])
        self._staged, self._resident = [], None   # stage_inputs() copies
        ws_bytes = int(self.lib.gtf_workspace_bytes(g.n_nodes, g.n_slots))
        if torch is not None:
            self._make_arena(self.PASS_INPUTS)
            self.t["ws"] = torch.zeros(ws_bytes, dtype=torch.uint8, device=self.device)
        else:   # (no arena: snapshots and staged inputs are benchmark tools, torch only)
            from .devmem import HipArray
            self.arena = None
            self.t["ws"] = HipArray.zeros(ws_bytes, np.uint8)
            nat.check(self.lib.gtf_stream_synchronize(None))   # the uploads' host buffers may go
            for t in self.t.values():
                t._pending = None
        self._build_structs(pack)

    # ---------------------------------------------------------------- memory
    def _make_arena(self, names):
        """place the arrays a pass mutates in one contiguous allocation, so a
        benchmark restore of the pass input is a single device copy"""
        torch = self.torch
        offs, total = {}, 0
        for k in names:
            nb = self.t[k].numel() * self.t[k].element_size()
            offs[k] = total
            total += (nb + 255) // 256 * 256
        arena = torch.zeros(max(total, 256), dtype=torch.uint8, device=self.device)
        for k in names:
            t = self.t[k]
            nb = t.numel() * t.element_size()
            view = arena[offs[k]:offs[k] + nb].view(t.dtype)
            view.copy_(t)
            self.t[k] = view
        self.arena = arena


    def _up(self, name, arr):
        arr = np.ascontiguousarray(arr)
        if self.torch is None:
            from .devmem import HipArray
            self.t[name] = HipArray.from_numpy(arr)
            return
        t = self.torch.from_numpy(arr.reshape(-1) if arr.size else arr.reshape(0)).to(self.device)
        self.t[name] = t

    def _np(self, t):
        """host copy of a device array (synchronises)"""
        return t.numpy() if self.torch is None else t.cpu().numpy()

    def _need_torch(self, what):
        if self.torch is None:
            raise NotImplementedError("%s needs DeviceGraph(mem='torch'); mem='hip' carries the stage methods, "
                                      "errors and download only" % what)

    def ptr(self, name):
        t = self.t[name]
        return ctypes.c_void_p(t.data_ptr() if t.numel() else 0)

    def _build_structs(self, pack=True):
        p = self.ptr
        base = dict(n_nodes=self.n_nodes, n_slots=self.n_slots, n_edges=self.n_edges,
                    slot_ptr=p("slot_ptr"), slot_src=p("slot_src"), slot_dst=p("slot_dst"), out_ptr=p("out_ptr"),
                    out_slot=p("out_slot"), slot_outpos=p("slot_outpos"), is_edge=p("is_edge"),
                    rev_edge=p("rev_edge"), solo=p("solo"), gnn=p("gnn"), xyzr=p("xyzr"), layer=p("layer"),
                    out_dst=p("out_dst"), slot_layer=p("slot_layer"),
                    slot_outidx=p("slot_outidx") if self.use_outidx else ctypes.c_void_p(0),
                    slot_class=p("slot_class") if self.use_classes else ctypes.c_void_p(0),
                    slot_sflags=p("slot_sflags") if self.use_classes else ctypes.c_void_p(0),
                    slot_sxzr=p("slot_sxzr") if self.use_sxzr else ctypes.c_void_p(0),
                    slot_static=p("slot_static") if self.use_static32 else ctypes.c_void_p(0),
                    slot_xclass=p("slot_xclass") if self.use_classes else ctypes.c_void_p(0))
        # with the node schedule (lane groups) and the sender schedule
        sched = dict(n_big=self.n_big, sched=p("sched"), n_g4=self.n_g_all[0], n_g8=self.n_g_all[1],
                     n_g16=self.n_g_all[2], n_g32=self.n_g_all[3], n_g64=self.n_g_all[4], sched_seg=p("sched_seg"),
                     out_sched=p("out_sched"), n_o4=self.n_o[0], n_o8=self.n_o[1], n_o16=self.n_o[2],
                     n_g2=self.n_g2, out_lanes=p("out_lanes"))
        if self.pad_plan is not None and self.pad_plan["tile_nodes"] > 0:   # (an empty graph has no tiles)
            pl = self.pad_plan
            sched.update(pad_tiles=pl["tiles"], pad_tile_nodes=pl["tile_nodes"], pad_tile_slots=pl["tile_slots"],
                         pad_count=(ctypes.c_int32 * 6)(*pl["count"]))
        if not self.use_sched:   # thread per node, 8-lane sender scan
            self.cg = nat.GtfGraph(**base)
        elif pack and self.n_pack_waves:
            self.cg = nat.GtfGraph(**base, **sched, pack_ent=p("pack_ent"), pack_wave=p("pack_wave"),
                                   n_pack_waves=self.n_pack_waves)
        else:
            self.cg = nat.GtfGraph(**base, **sched)
        self.cg_sched = nat.GtfGraph(**base, **sched)
        self.cn = nat.GtfNodes(*[p(f) for f in MUTABLE_NODE])
        self.cuts = nat.GtfStates(p("uts_rank"), p("uts_sv"), p("uts_tau"), p("uts_cov"), p("uts_xyzr"),
                                  p("uts_lik"), p("uts_mw"), p("uts_prior"), p("uts_lr"), p("uts_side"),
                                  p("uts_fresh"))
        self.ctse = nat.GtfStates(p("tse_rank"), p("tse_sv"), p("tse_tau"), p("tse_cov"), p("tse_xyzr"),
                                  ctypes.c_void_p(0), p("tse_mw"), p("tse_prior"), ctypes.c_void_p(0),
                                  ctypes.c_void_p(0), ctypes.c_void_p(0))
        self.ce = nat.GtfEdges(p("act"), p("edge_mw"), p("send_mw"))

    @property
    def stream(self):
        if self.torch is None:
            return ctypes.c_void_p(0)   # mem "hip": the default stream
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def cparams(p: Params) -> nat.GtfParams:
        return nat.GtfParams(p.sigma0xy, p.sigma0rz, p.sigma0rz2, p.endcap_boundary, p.chi2_cut,
                             p.reweight_threshold, p.cluster_chi2, p.cluster_kl)

    # ---------------------------------------------------------------- stages
    def clear_errors(self):
        nat.check(self.lib.gtf_clear_errors(self.ptr("ws"), self.stream))

    def errors(self) -> int:
        f = ctypes.c_uint32(0)
        nat.check(self.lib.gtf_read_errors(self.ptr("ws"), ctypes.byref(f), self.stream))
        return int(f.value)

    def raise_errors(self, ignore=0):
        f = self.errors() & ~ignore
        if f:
            msgs = [m for b, m in nat.ERR_FLAGS.items() if f & b]
            raise ValueError("reference exception reproduced on device: " + "; ".join(msgs))

    def extrapolate(self, p: Params):
        cp = self.cparams(p)
        nat.check(self.lib.gtf_extrapolate(ctypes.byref(self.cg), ctypes.byref(self.cn), ctypes.byref(self.cuts),
                                           ctypes.byref(self.ce), ctypes.byref(cp), self.ptr("ws"), self.stream))

    def message_passing(self, p: Params):
        cp = self.cparams(p)
        nat.check(self.lib.gtf_message_passing(ctypes.byref(self.cg), ctypes.byref(self.cn),
                                               ctypes.byref(self.cuts), ctypes.byref(self.ce), ctypes.byref(cp),
                                               self.ptr("ws"), self.stream))

    def node_ops(self, ops, p: Params, chi2=0.0, kl=0.0):
        """run named node-local ops (gtf._native.OPS) in order, one launch"""
        codes = [nat.OPS[o] for o in ops]
        arr = (ctypes.c_int8 * len(codes))(*codes)
        cp = self.cparams(p)
        nat.check(self.lib.gtf_node_ops(ctypes.byref(self.cg), ctypes.byref(self.cn), ctypes.byref(self.ctse),
                                        ctypes.byref(self.cuts), ctypes.byref(self.ce), ctypes.byref(cp), arr,
                                        len(codes), float(chi2), float(kl), self.ptr("ws"), self.stream))

    def update(self, p: Params):
        cp = self.cparams(p)
        nat.check(self.lib.gtf_update(ctypes.byref(self.cg), ctypes.byref(self.cn), ctypes.byref(self.ctse),
                                      ctypes.byref(self.cuts), ctypes.byref(self.ce), ctypes.byref(cp),
                                      self.ptr("ws"), self.stream))

    def cluster(self, key: str, chi2: float, kl: float, p: Params):
        cp = self.cparams(p)
        st = self.cuts if key in ("uts", "updated_track_states") else self.ctse
        k = 1 if st is self.cuts else 0
        nat.check(self.lib.gtf_cluster(ctypes.byref(self.cg), ctypes.byref(self.cn), ctypes.byref(st),
                                       ctypes.byref(self.ce), k, float(chi2), float(kl), ctypes.byref(cp),
                                       self.ptr("ws"), self.stream))

    def full_pass(self, p: Params, events=None):
        """events: optional 5 raw hipEvent_t handles (per-kernel timing)"""
        cp = self.cparams(p)
        if events is None:
            nat.check(self.lib.gtf_pass(ctypes.byref(self.cg), ctypes.byref(self.cn), ctypes.byref(self.ctse),
                                        ctypes.byref(self.cuts), ctypes.byref(self.ce), ctypes.byref(cp),
                                        self.ptr("ws"), self.stream))
        else:
            arr = (ctypes.c_void_p * 5)(*events)
            nat.check(self.lib.gtf_pass_ev(ctypes.byref(self.cg), ctypes.byref(self.cn), ctypes.byref(self.ctse),
                                           ctypes.byref(self.cuts), ctypes.byref(self.ce), ctypes.byref(cp),
                                           self.ptr("ws"), self.stream, arr))

    def track_state_estimates(self, p: Params, host_order: bool = True):
        """helper.compute_track_state_estimates (helper.py:238-452) for every key of the
        nodes' track_state_estimates dicts (tse_rank >= 0, dict order as given): writes
        tse_sv / tse_cov / tse_tau / tse_xyzr / tse_theta / tse_var_ms on the device and
        returns the per-node attributes (xy/zr_edge_gradient_mean_var,
        angle_of_rotation, translation) as device tensors -- in host node order, or with
        host_order=False in the device layout's order (no gathers: what a caller that keeps
        the event on the device consumes)."""
        self._natural_only("track_state_estimates")
        if self.torch is None:
            return self._track_state_estimates_hip(p, host_order)
        torch = self.torch
        N = self.n_nodes
        nan = float("nan")
        x = {"xy_mean_var": torch.full((N, 2), nan, dtype=torch.float64, device=self.device),
             "zr_mean_var": torch.full((N, 2), nan, dtype=torch.float64, device=self.device),
             "angle_of_rotation": torch.full((N,), nan, dtype=torch.float64, device=self.device),
             "translation": torch.full((N, 2), nan, dtype=torch.float64, device=self.device)}
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t.numel() else 0)  # noqa: E731
        ex = nat.GtfTseExtra(self.ptr("tse_theta"), self.ptr("tse_var_ms"), vp(x["xy_mean_var"]),
                             vp(x["zr_mean_var"]), vp(x["angle_of_rotation"]), vp(x["translation"]))
        cp = self.cparams(p)
        nat.check(self.lib.gtf_track_state_estimates(ctypes.byref(self.cg_sched), ctypes.byref(self.ctse),
                                                     ctypes.byref(ex), ctypes.byref(cp), self.stream))
        if self.order is not None and host_order:   # per-node outputs in host node order
            inv = self._inv_order()
            x = {k: v[inv] for k, v in x.items()}
        return x

    def _track_state_estimates_hip(self, p: Params, host_order: bool):
        """mem "hip": the same call on gtf.devmem arrays; the per-node attributes come back
        as host arrays"""
        from .devmem import HipArray
        N = self.n_nodes
        shapes = {"xy_mean_var": (N, 2), "zr_mean_var": (N, 2), "angle_of_rotation": (N,), "translation": (N, 2)}
        x = {k: HipArray.from_numpy(np.full(int(np.prod(sh)), np.nan)) for k, sh in shapes.items()}
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t.numel() else 0)  # noqa: E731
        ex = nat.GtfTseExtra(self.ptr("tse_theta"), self.ptr("tse_var_ms"), vp(x["xy_mean_var"]),
                             vp(x["zr_mean_var"]), vp(x["angle_of_rotation"]), vp(x["translation"]))
        cp = self.cparams(p)
        nat.check(self.lib.gtf_track_state_estimates(ctypes.byref(self.cg_sched), ctypes.byref(self.ctse),
                                                     ctypes.byref(ex), ctypes.byref(cp), self.stream))
        out = {k: v.numpy().reshape(shapes[k]) for k, v in x.items()}
        if self.order is not None and host_order:
            inv = np.empty(self.order.size, np.int64)
            inv[self.order] = np.arange(self.order.size)
            out = {k: v[inv] for k, v in out.items()}
        return out

    # ------------------------------------------ a15: distances between updated states
    def updated_state_distances(self, truth=None, host_order: bool = True):
        """calculate_distance_between_updated_track_states.py (:27-104 over the pair loop
        :134-195) on the current updated_track_states: every pair i > j of the dict entries
        of each node with the dict and more than one active in-edge. Returns (pair_ptr [N+1]
        int64, {"chi2", "avg_tau", "avg_theta", "delta_theta"[, "truth"]}) as device
        tensors, pairs of node v at [pair_ptr[v], pair_ptr[v+1]) in the reference's loop
        order. truth: [N] truth_particle per node (host or device), or None. host_order=False:
        the node segments in the device layout's node order (no reordering gathers)."""
        self._natural_only("updated_state_distances")
        self._need_torch("updated_state_distances")
        torch = self.torch
        dev = self.device
        N = self.n_nodes
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None and t.numel() else 0)  # noqa: E731
        counts = torch.zeros(max(N, 1), dtype=torch.int64, device=dev)
        nat.check(self.lib.gtf_updated_state_pair_counts(ctypes.byref(self.cg_sched), ctypes.byref(self.cn),
                                                         ctypes.byref(self.cuts), ctypes.byref(self.ce), vp(counts),
                                                         self.stream))
        pair_ptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
        if N:
            torch.cumsum(counts[:N], 0, out=pair_ptr[1:])
        P = int(pair_ptr[-1].item())
        out = {k: torch.empty(max(P, 1), dtype=torch.float64, device=dev)
               for k in ("chi2", "avg_tau", "avg_theta", "delta_theta")}
        tr = None
        if truth is not None:
            tr = torch.as_tensor(np.asarray(truth, dtype=np.int64) if not torch.is_tensor(truth) else truth,
                                 device=dev).to(torch.int64).contiguous()
            out["truth"] = torch.empty(max(P, 1), dtype=torch.int8, device=dev)
        if tr is not None and self.order is not None:
            tr = tr[torch.from_numpy(self.order).to(dev)].contiguous()   # device node order
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        po = nat.GtfPairOut(vp(out["chi2"]), vp(out["avg_tau"]), vp(out["avg_theta"]), vp(out["delta_theta"]),
                            vp(out.get("truth")), vp(err))
        nat.check(self.lib.gtf_updated_state_distances(ctypes.byref(self.cg_sched), ctypes.byref(self.cn),
                                                       ctypes.byref(self.cuts), ctypes.byref(self.ce), vp(tr),
                                                       vp(pair_ptr), ctypes.byref(po), self.stream))
        f = int(err.item())
        if f:
            raise ValueError("updated-state distances: " +
                             "; ".join(m for b, m in nat.ERR_FLAGS.items() if f & b))
        cols = {k: v[:P] for k, v in out.items()}
        if self.order is not None and N and host_order:   # node segments of pairs in host node order
            inv = self._inv_order()
            cnt = counts[:N][inv]
            hptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
            torch.cumsum(cnt, 0, out=hptr[1:])
            first = torch.repeat_interleave(pair_ptr[:N][inv], cnt, output_size=P)
            idx = first + (torch.arange(P, device=dev) - torch.repeat_interleave(hptr[:N], cnt, output_size=P))
            cols = {k: v[idx] for k, v in cols.items()}
            pair_ptr = hptr
        return pair_ptr, cols

    # ------------------------------------------------------- tag propagation
    def tag_propagation(self, tags, radius, threshold=0.1, max_sweeps=100000):
        """Jacobi sweeps until flips / processed <= threshold (tag_propagation.py:97-164), the
        whole stage in one gtf_tag_propagate call (stop rule on the device, one host read per
        batch of sweeps). tags / radius in host node order; returns (tags, flips per sweep)."""
        self._natural_only("tag_propagation")
        r = self._dev_from(np.ascontiguousarray(self._to_dev_nodes(radius), dtype=np.float64))
        ta = self._dev_from(np.ascontiguousarray(self._to_dev_nodes(tags), dtype=np.int64))
        flips = self.tag_propagation_dev(ta, r, threshold, max_sweeps)
        out = self._np(ta)[:self.n_nodes]
        if self.order is not None:
            h = np.empty_like(out)
            h[self.order] = out
            out = h
        return out, flips

    def tag_propagation_dev(self, tags, radius, threshold=0.1, max_sweeps=100000):
        """gtf_tag_propagate on device arrays in this graph's node order: `tags` (int64 [N]) is
        replaced by the final tags; returns the flip count of every sweep"""
        nb = int(self.lib.gtf_tag_workspace_bytes(self.n_nodes, self.n_edges))
        ws = getattr(self, "_tag_ws", None)
        if ws is None or ws.numel() < nb:
            ws = self._tag_ws = self._dev_zeros(nb, np.uint8)
        hf = getattr(self, "_tag_flips", None)
        if hf is None or hf.size < max(max_sweeps, 1):
            hf = self._tag_flips = np.zeros(max(max_sweeps, 1), np.int32)
        n = ctypes.c_int32(0)
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t.numel() else 0)  # noqa: E731
        nat.check(self.lib.gtf_tag_propagate(ctypes.byref(self.cg), vp(radius), vp(tags), float(threshold),
                                             int(max_sweeps), ctypes.c_void_p(hf.ctypes.data), ctypes.byref(n),
                                             vp(ws), ctypes.c_size_t(nb), self.stream))
        return [int(x) for x in hf[:n.value]]

    def _dev_zeros(self, n, dtype):
        """a zeroed device array of this graph's allocator"""
        if self.torch is None:
            from .devmem import HipArray
            return HipArray.zeros(n, dtype)
        return self.torch.zeros(n, dtype=getattr(self.torch, np.dtype(dtype).name), device=self.device)

    def _dev_from(self, a):
        """a host array on the device (this graph's allocator)"""
        a = np.ascontiguousarray(a).reshape(-1)
        if self.torch is None:
            from .devmem import HipArray
            return HipArray.from_numpy(a)
        return self.torch.from_numpy(a).to(self.device)

    # ------------------------------------------------------------ diagnostics
    def set_diagnostics(self, node_err: bool = True, edge_chi2: bool = True, slot_cluster: bool = False):
        """SURVEY §5's optional diagnostic outputs (gtf_set_diagnostics), written by the stage
        kernels from now on: the GTF_ERR_* bits of every reference exception per node (which
        node, so which subgraph, would make the reference raise) and the chi2 of every
        extrapolated edge (the values extrapolate_merged_states.py:134-172 prints to CSV).
        Off by default and never on the benchmark's path; set_diagnostics(False, False)
        unregisters them."""
        self._need_torch("set_diagnostics")
        torch = self.torch
        self.diag_t = {}
        if node_err:
            self.diag_t["node_err"] = torch.zeros(max(self.n_nodes, 1), dtype=torch.int32, device=self.device)
        if edge_chi2:
            self.diag_t["edge_chi2"] = torch.full((max(self.n_slots, 1),), float("nan"), dtype=torch.float64,
                                                  device=self.device)
        if slot_cluster:
            self.diag_t["slot_cluster"] = torch.zeros(max(self.n_slots, 1), dtype=torch.uint8, device=self.device)
        vp = lambda k: ctypes.c_void_p(self.diag_t[k].data_ptr()) if k in self.diag_t else ctypes.c_void_p(0)  # noqa: E731
        d = nat.GtfDiag(vp("node_err"), vp("edge_chi2"), vp("slot_cluster"))
        nat.check(self.lib.gtf_set_diagnostics(self.ptr("ws"), ctypes.byref(d), self.stream))

    def diagnostics(self) -> dict:
        """the registered diagnostics in host order: node_err [N] uint32, edge_chi2 [S]
        (NaN where no extrapolation ran), slot_cluster [S] uint8"""
        out = {}
        for k, v in getattr(self, "diag_t", {}).items():
            if k == "node_err":
                a = v.cpu().numpy()[:self.n_nodes].astype(np.uint32)
                out[k] = a if self.order is None else self._host_nodes(a)
            else:
                a = v.cpu().numpy()[:self.n_slots]
                out[k] = a if self.slot_perm is None else self._host_slots(a, np.nan if a.dtype.kind == "f" else 0)
        return out

    def clear_diagnostics(self):
        """zero node_err / slot_cluster and NaN-fill edge_chi2 (stream-ordered)"""
        for k, v in getattr(self, "diag_t", {}).items():
            v.fill_(float("nan") if k == "edge_chi2" else 0)

    def _host_nodes(self, a, fill=0):
        nm = self.order >= 0
        h = np.full(int(nm.sum()), fill, a.dtype)
        h[self.order[nm]] = a[nm]
        return h

    def _host_slots(self, a, fill=0):
        sm = self.slot_perm >= 0
        h = np.full(int(sm.sum()), fill, a.dtype)
        h[self.slot_perm[sm]] = a[sm]
        return h

    # ---------------------------------------------------------------- results
    def materialize(self):
        """write the live updated_track_states coordinates (gtf_states.fresh bit 1) into
        uts_xyzr on the device (gtf_uts_materialize): before reading them back"""
        nat.check(self.lib.gtf_uts_materialize(ctypes.byref(self.cg_sched), ctypes.byref(self.cuts), self.stream))

    def download(self, g: TrackGraph) -> TrackGraph:
        """copy the mutable arrays back into the host TrackGraph (in place, host order)"""
        self.materialize()
        nm = None if self.order is None else self.order >= 0          # (padded: not a dummy node)
        sm = None if self.slot_perm is None else self.slot_perm >= 0  # (padded: not a padding slot)
        for f in MUTABLE_NODE:
            a = self._np(self.t[f]).reshape((-1,) + g.node[f].shape[1:])
            if self.order is None:
                g.node[f][...] = a
            else:
                g.node[f][self.order[nm]] = a[nm]
        for f in SLOT_FIELDS:
            if f in STATIC_SLOT or f == "slot_key":
                continue
            a = self._np(self.t[f]).reshape((-1,) + g.slot[f].shape[1:])
            if f == "uts_fresh":
                a = a & 1   # (bit 1 is cleared by materialize())
            if self.slot_perm is None:
                g.slot[f][...] = a
            else:
                g.slot[f][self.slot_perm[sm]] = a[sm]
        return g

    def _natural_only(self, what):
        """node-indexed arrays cross these methods in host order: every layout whose node order
        is a permutation of the host's maps them (the padded layout's dummy nodes do not)"""
        if self.layout == "padded":
            raise NotImplementedError("%s takes node-indexed host arrays: not with layout='padded'" % what)

    def _to_dev_nodes(self, a):
        """a host-order per-node array (numpy) in device node order"""
        a = np.asarray(a)
        return a if self.order is None else a[self.order]

    def _inv_order(self):
        """device tensor: host node h -> device node"""
        if getattr(self, "_inv_t", None) is None:
            inv = np.empty(self.order.size, np.int64)
            inv[self.order] = np.arange(self.order.size)
            self._inv_t = self.torch.from_numpy(inv).to(self.device)
        return self._inv_t

    # arrays whose values decide how much work the next pass does: restoring
    # them makes every benchmark step process the same input
    PASS_INPUTS = ("act", "uts_rank", "has_uts", "has_merged", "merged_state", "merged_cov", "merged_prior")

    def snapshot(self, names=None):
        """device-side copy of mutable arrays (default: every one). The pass inputs
        (PASS_INPUTS) live in one arena and snapshot as a single buffer."""
        self._need_torch("snapshot")
        if names is not None and tuple(names) == tuple(self.PASS_INPUTS):
            return {"__arena__": self.arena.clone()}
        names = names or [k for k in self.t if k in MUTABLE_NODE or
                          (k in SLOT_FIELDS and k not in STATIC_SLOT and k != "slot_key")]
        return {k: self.t[k].clone() for k in names}

    def restore(self, snap):
        """copy a snapshot back (the pass-input arena is one device copy)"""
        if "__arena__" in snap:
            self.arena.copy_(snap["__arena__"], non_blocking=True)
            return
        for k, v in snap.items():
            self.t[k].copy_(v, non_blocking=True)

    # ------------------------------------------------ staged copies of the pass input
    def stage_inputs(self, k: int):
        """k device copies of the pass-input arena (PASS_INPUTS), each with its own C structs,
        for a benchmark whose steps each run one pass over a resident, identical input without
        a restore copy between them: use_inputs(i) points every stage method at copy i
        (None: the arrays of this graph). The arrays outside the arena (state values,
        degree) are shared: a pass overwrites every value it reads back."""
        self._need_torch("stage_inputs")
        if self._resident is None:
            self._resident = (self.cn, self.cuts, self.ctse, self.ce)
        self.use_inputs(None)
        lo = self.arena.data_ptr()
        hi = lo + self.arena.numel()

        def rebase(st, off):
            vals = []
            for name, typ in st._fields_:
                v = getattr(st, name)
                if typ is ctypes.c_void_p and v is not None and lo <= v < hi:
                    v = v + off
                vals.append(v)
            return type(st)(*vals)

        self._staged = []   # (a second call replaces the copies)
        for _ in range(k):
            a = self.torch.empty_like(self.arena)
            off = a.data_ptr() - lo
            self._staged.append((a, tuple(rebase(s, off) for s in self._resident)))

    def fill_inputs(self, snap):
        """copy the pass-input snapshot (snapshot(PASS_INPUTS)) into every staged copy"""
        if "__arena__" not in snap:
            raise ValueError("fill_inputs takes snapshot(DeviceGraph.PASS_INPUTS)")
        for a, _ in self._staged:
            a.copy_(snap["__arena__"], non_blocking=True)

    def use_inputs(self, i):
        """point the stage methods at staged copy i, or back at this graph's arrays (None)"""
        if i is None:
            if self._resident is not None:
                self.cn, self.cuts, self.ctse, self.ce = self._resident
            return
        self.cn, self.cuts, self.ctse, self.ce = self._staged[i][1]
