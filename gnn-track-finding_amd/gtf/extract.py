"""Track-candidate extraction on the GPU: host side of ``gtf_extract_candidates``.

Mirrors src/extract/extract_track_candidates.py (:349-467): CCA over the activated
edges, close-proximity merging, the one-hit-per-layer check and the xy / rz Kalman
fits with chi-square p-values, per candidate on the device. This module turns the
per-candidate device results into the stage's outputs (extracted candidates in the
reference's order with their p-values, the remaining and fragment subgraphs) and, in
:func:`extract_graphs`, into the reference's networkx objects.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat
from .graph import TrackGraph

FRAGMENT, BAD, REJECTED, EXTRACTED = 0, 1, 2, 3


class Params:
    """extract_track_candidates.py flags -p -n -s -t -e -z -b (run_gnn_trackml_mod.sh defaults)."""

    def __init__(self, pval=0.01, numhits=4, separation_3d_threshold=10.0, threshold_distance_node_merging=8.0,
                 sigma0xy=0.3, sigma0rz=0.4, endcap_boundary=550.0):
        self.pval, self.numhits = float(pval), int(numhits)
        self.separation = float(separation_3d_threshold)
        self.merge = float(threshold_distance_node_merging)
        self.sigma0xy, self.sigma0rz, self.endcap = float(sigma0xy), float(sigma0rz), float(endcap_boundary)

    def c(self):
        return nat.GtfExtractParams(self.pval, self.numhits, 0, self.separation, self.merge, self.sigma0xy,
                                    self.sigma0rz, self.endcap)


def run(g: TrackGraph, vivl, params: Params, order_key=None, device="cuda", d=None):
    """Run the extraction on the device for a packed graph (the pass's output).
    vivl: [N, 2] (volume_id, in_volume_layer_id); order_key: optional [N] member order
    inside a candidate (default node order); d: the DeviceGraph of ``g`` already in HBM
    (a stage just ran on it: its activation mask is read in place), else ``g`` is
    uploaded. Returns a dict of host arrays."""
    from .device import DeviceGraph
    if params.numhits < 3:
        raise ValueError("numhits must be >= 3 (rotate_track reads three hits)")
    if d is None:
        from .devmem import default_mem
        d = DeviceGraph(g, device, mem=default_mem())
    elif d.n_nodes != g.n_nodes or d.n_slots != g.n_slots:
        raise ValueError("DeviceGraph does not hold this graph")
    N = g.n_nodes
    sub = g.node["sub_id"].astype(np.int32)
    if N and (np.any(np.diff(sub) < 0) or sub[0] != 0 or np.any(np.diff(sub) > 1)):
        raise ValueError("extraction needs nodes grouped by subgraph (sub_id 0, 1, 2, ... non-decreasing), "
                         "as pack() numbers them")
    n_sub = int(sub.max()) + 1 if N else 0
    sub_ptr = np.searchsorted(sub, np.arange(n_sub + 1)).astype(np.int32)
    n1 = max(N, 1)
    up = lambda a, dt=None: _up(d, np.asarray(a) if dt is None else np.asarray(a).astype(dt))  # noqa: E731
    t = {"xyzr": up(g.node["xyzr"], np.float64), "vivl": up(np.asarray(vivl), np.float64), "sub": up(sub),
         "sub_ptr": up(sub_ptr), "gnn": up(g.node["gnn"], np.float64),
         "order": up(np.asarray(order_key), np.int32) if order_key is not None else None,
         "label": up(np.zeros(n1, np.int32)),
         "status": up(np.full(n1, -1, np.int8)),
         "pxy": up(np.full(n1, np.nan)),
         "pzr": up(np.full(n1, np.nan)),
         "ext": up(np.zeros(n1, np.uint8)),
         "ncand": up(np.zeros(1, np.int32))}
    ws = _zeros(d, int(d.lib.gtf_extract_workspace_bytes(N, n_sub)))
    vp = lambda x: ctypes.c_void_p(x.data_ptr() if x is not None and x.numel() else 0)  # noqa: E731
    io = nat.GtfExtractIO(vp(t["xyzr"]), vp(t["vivl"]), vp(t["sub"]), vp(t["sub_ptr"]), n_sub, 0, vp(t["order"]),
                          vp(t["gnn"]), vp(t["label"]), vp(t["status"]), vp(t["pxy"]), vp(t["pzr"]),
                          vp(t["ext"]), vp(t["ncand"]))
    cp = params.c()
    nat.check(d.lib.gtf_extract_candidates(ctypes.byref(d.cg), ctypes.byref(d.ce), ctypes.byref(io),
                                           ctypes.byref(cp), vp(ws), d.stream))
    out = {k: d._np(t[k])[:N] for k in ("label", "status", "pxy", "pzr", "ext")}
    out["gnn"] = d._np(t["gnn"]).reshape(-1, 4)[:N]
    out["n_candidates"] = int(d._np(t["ncand"])[0])
    return out


def _up(d, a):
    """a host array as a device array of d's allocator (torch tensor or gtf.devmem)"""
    a = np.ascontiguousarray(a).reshape(-1)
    if d.torch is None:
        from .devmem import HipArray
        return HipArray.from_numpy(a)
    return d.torch.from_numpy(a).to(d.device)


def _zeros(d, nbytes):
    if d.torch is None:
        from .devmem import HipArray
        return HipArray.zeros(nbytes, np.uint8)
    return d.torch.zeros(nbytes, dtype=d.torch.uint8, device=d.device)


def candidate_order(g: TrackGraph) -> np.ndarray:
    """Each node's position inside its candidate in the reference's member order
    (gtf_candidate_order: networkx CCA + subgraph-copy orders, :332-346), for run()'s
    order_key. Host function on the packed graph's activation mask."""
    N = g.n_nodes
    a = {k: np.ascontiguousarray(v) for k, v in (
        ("slot_ptr", g.slot_ptr.astype(np.int32)), ("slot_src", g.slot["slot_src"].astype(np.int32)),
        ("is_edge", g.slot["is_edge"].astype(np.uint8)), ("act", g.slot["act"].astype(np.uint8)),
        ("out_ptr", g.out_ptr.astype(np.int32)), ("out_slot", g.out_slot.astype(np.int32)),
        ("sub_id", g.node["sub_id"].astype(np.int32)), ("node_id", g.node["node_id"].astype(np.int64)))}
    vp = lambda x: ctypes.c_void_p(x.ctypes.data if x.size else 0)  # noqa: E731
    cg = nat.GtfCandidateGraph(N, g.n_slots, g.n_edges, 0, vp(a["slot_ptr"]), vp(a["slot_src"]), vp(a["is_edge"]),
                               vp(a["act"]), vp(a["out_ptr"]), vp(a["out_slot"]), vp(a["sub_id"]), vp(a["node_id"]))
    out = np.zeros(max(N, 1), np.int32)
    nat.check(nat.lib(lean=True).gtf_candidate_order(ctypes.byref(cg), vp(out)))   # host code: no torch needed
    return out[:N]


def outputs(g: TrackGraph, res, fragment, order_key=None):
    """The stage's outputs from the device results: extracted candidates (node index
    arrays, in the reference's order), their p-values, remaining and fragment node
    sets per subgraph (:423-430). order_key: member order inside each candidate (as
    given to run()); default node order."""
    label, status, ext = res["label"], res["status"], res["ext"].astype(bool)
    roots = np.unique(label)                          # candidate order = first-node order
    extracted = [np.nonzero(label == r)[0] for r in roots if status[r] == EXTRACTED]
    if order_key is not None:
        extracted = [c[np.argsort(order_key[c], kind="stable")] for c in extracted]
    pxy = np.array([res["pxy"][r] for r in roots if status[r] == EXTRACTED])
    pzr = np.array([res["pzr"][r] for r in roots if status[r] == EXTRACTED])
    sub = g.node["sub_id"]
    remaining, fragments = [], []
    for s in range(int(sub.max()) + 1 if g.n_nodes else 0):
        left = np.nonzero((sub == s) & ~ext)[0]
        if 0 < len(left) < fragment:
            fragments.append(left)
        elif len(left) >= fragment:
            remaining.append(left)
    return {"extracted": extracted, "pval_xy": pxy, "pval_zr": pzr, "remaining": remaining,
            "fragments": fragments}
