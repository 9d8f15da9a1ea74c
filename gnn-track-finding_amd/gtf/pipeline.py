"""The track-finding loop of run_gnn_trackml_mod.sh (:61-146) on the device.

Reference flow (one process per stage, gpickle directories in between):

    event_conversion  ->  it 1: clustering(track_state_estimates, -c 1.0 -k 2.0) -> extract
                          it 2: extrapolate(-c 2.0) -> extract -> remove_state_metadata(remaining)
                          it 3: clustering(updated_track_states, -c 1000 -k 100) -> extract
                          ... (even: as 2, odd: as 3); each iteration starts from the
                          previous iteration's remaining subgraphs (:140)

Here every stage runs in HBM through the C-ABI on one packed graph per iteration:
the stage and the extraction share one DeviceGraph (the extraction reads the stage's
activation mask in place), and the host only builds the next iteration's graph from
the extraction's verdict (:func:`gtf.graph.subset`, the packed form of
``remove_nodes_from`` + dropping fragments) with the extraction's GNN_Measurement
coordinate mutation (close-proximity merging, extract_track_candidates.py:91-118)
carried over.

Event conversion (:func:`build_event`, event_conversion.py:53-101): the packed graph
and its orders come from gtf_build_event_csr (csrc/gtf_build.cpp: the reference's
node, successor and weakly-connected-component orders and the set order of the
track_state_estimates keys, helper.py:277,350-351, without networkx); the states,
priors, mixture weights and degrees are computed on the device
(gtf_track_state_estimates + gtf_node_ops).
"""
from __future__ import annotations

import dataclasses
import time
from typing import List, Optional

import numpy as np

from . import extract
from .graph import TrackGraph, pack, refresh_send_mw, subset
from .params import Params

CLUSTER_FIRST = (1.0, 2.0)        # run_gnn_trackml_mod.sh:89  -d track_state_estimates -c 1.0 -k 2.0
CLUSTER_LATER = (1000.0, 100.0)   # run_gnn_trackml_mod.sh:112 -d updated_track_states -c 1000 -k 100


@dataclasses.dataclass
class Iteration:
    """One iteration's outputs as node ids (the reference's candidates/, remaining/,
    fragments/ directories and candidates/pvals.csv)."""
    index: int
    stage: str
    candidates: List[np.ndarray]
    pval_xy: np.ndarray
    pval_zr: np.ndarray
    remaining: List[np.ndarray]
    fragments: List[np.ndarray]
    seconds: dict
    network: Optional[TrackGraph] = None      # the stage's output graph (keep_graphs=True)
    remaining_graph: Optional[TrackGraph] = None    # next iteration's input
    remaining_vivl: Optional[np.ndarray] = None


def event_layout(event_prefix: str, min_volume: int, max_volume: int, builder: str = "native", device="cuda"):
    """Host half of event conversion: the packed network in the reference's orders,
    with empty track_state_estimates dicts keyed in their set order and every edge
    active (helper.initialize_edge_activation). Returns (graph, vivl[N, 2]).

    builder "native": gtf_build_event_csr (C++, CSV rows -> CSR, CPython set orders
    reproduced); "device": gtf_build_event_csr_device (the same build on the GPU, the
    same arrays); "networkx": the reference's own construction through networkx and
    pack() (gtf.io.build_networkx) -- the slow path the native one is tested against."""
    from . import io
    if builder == "native":
        return io.build_event_csr(event_prefix, min_volume, max_volume)
    if builder == "device":
        return io.build_event_csr(event_prefix, min_volume, max_volume, device=device)
    if builder != "networkx":
        raise ValueError("builder must be 'native', 'device' or 'networkx'")
    import networkx as nx
    subs = io.build_networkx(event_prefix, min_volume, max_volume)
    for G in subs:
        for node in G.nodes():
            keys = list(set(nx.all_neighbors(G, node)))
            keys.reverse()
            G.nodes[node]["track_state_estimates"] = {k: {} for k in keys}
    g = pack(subs)
    vivl = np.array([(G.nodes[n]["volume_id"], G.nodes[n]["in_volume_layer_id"]) for G in subs for n in G.nodes],
                    dtype=np.float64).reshape(-1, 2)
    return g, vivl


def build_event(event_prefix: str, min_volume: int, max_volume: int, p: Params = None, device="cuda",
                builder: str = "device"):
    """event_conversion.py:53-101: CSVs -> packed network with track_state_estimates,
    activation 1, priors, mixture weights and degrees, all on the GPU (the graph build by
    gtf_build_event_csr_device; builder "native" for the host C++ one, the same arrays).
    Returns (graph, vivl[N, 2])."""
    from .device import DeviceGraph
    p = p or Params()
    g, vivl = event_layout(event_prefix, min_volume, max_volume, builder, device)
    if g.n_nodes == 0:
        return g, vivl
    d = DeviceGraph(g, device)
    d.clear_errors()
    d.track_state_estimates(p)
    d.node_ops(["priors_tse", "mw_tse", "degree"], p)
    d.raise_errors()
    d.download(g)
    refresh_send_mw(g)
    return g, vivl


def _ids(g: TrackGraph, groups):
    return [g.node["node_id"][np.asarray(x, np.int64)] for x in groups]


def run(g: TrackGraph, vivl, iterations: int = 3, p: Params = None, ex: extract.Params = None,
        device="cuda", first: int = 1, keep_graphs: bool = False) -> List[Iteration]:
    """Iterations ``first`` .. ``first + iterations - 1`` of the loop, starting from
    the stage input ``g`` (the event network for iteration 1). Stops early when
    nothing remains. keep_graphs: also return each iteration's stage output and
    remaining graphs (for saving, gtf.store)."""
    from .device import DeviceGraph
    p = p or Params()
    ex = ex or extract.Params()
    vivl = np.asarray(vivl, np.float64).reshape(-1, 2)
    if vivl.shape[0] != g.n_nodes:
        raise ValueError("vivl must have one row per node")
    out = []
    torch = None
    for it in range(first, first + iterations):
        if g.n_nodes == 0:
            break
        t0 = time.perf_counter()
        d = DeviceGraph(g, device)
        torch = d.torch
        d.clear_errors()
        if it == 1:
            stage = "clustering(track_state_estimates)"
            d.cluster("tse", CLUSTER_FIRST[0], CLUSTER_FIRST[1], p)
        elif it % 2 == 0:
            stage = "extrapolation"
            d.extrapolate(p)
        else:
            stage = "clustering(updated_track_states)"
            d.cluster("uts", CLUSTER_LATER[0], CLUSTER_LATER[1], p)
        d.raise_errors()
        torch.cuda.synchronize(d.device)
        t1 = time.perf_counter()
        d.download(g)
        order = extract.candidate_order(g)            # members in the reference's candidate order
        res = extract.run(g, vivl, ex, order_key=order, d=d)
        t2 = time.perf_counter()
        o = extract.outputs(g, res, ex.numhits, order)
        net = g.copy() if keep_graphs else None       # the stage's output, before the merging mutation
        keep = np.zeros(g.n_nodes, bool)
        for r in o["remaining"]:
            keep[r] = True
        g.node["gnn"] = res["gnn"]                 # GNN_Measurement mutated in place by merging
        nxt = subset(g, keep)
        refresh_send_mw(nxt)
        if it % 2 == 0 and nxt.n_nodes:
            # remove_state_metadata.py on the remaining directory (run_gnn_trackml_mod.sh:137-139)
            du = DeviceGraph(nxt, device)
            du.clear_errors()
            du.update(p)
            du.raise_errors()
            du.download(nxt)
        t3 = time.perf_counter()
        rec = Iteration(it, stage, _ids(g, o["extracted"]), o["pval_xy"], o["pval_zr"],
                        _ids(g, o["remaining"]), _ids(g, o["fragments"]),
                        {"stage": t1 - t0, "extract": t2 - t1, "next": t3 - t2})
        if keep_graphs:
            rec.network, rec.remaining_graph, rec.remaining_vivl = net, nxt, vivl[keep]
        out.append(rec)
        g, vivl = nxt, vivl[keep]
    return out
