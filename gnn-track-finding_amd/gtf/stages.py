"""Graph-level stage API: list[nx.DiGraph] in, the same graphs mutated out.

This is the layer the drop-in modules (utilities/helper.py,
extrapolate/extrapolate_merged_states.py, clustering/clustering.py,
update/remove_state_metadata.py, tag_propagation/) call. Each call packs the
graphs (gtf.graph.pack), uploads them, runs the HIP stage through the C-ABI,
and writes the results back with the reference's attribute schema
(gtf.graph.unpack). Reference exceptions detected on the device are raised as
the same Python exception class the reference raises.
"""
from __future__ import annotations

import glob
import os
import pickle
from typing import List

from .graph import pack, unpack
from .params import Params

SUBGRAPH_SUFFIX = "_subgraph.gpickle"

_EXC = {1: KeyError, 2: KeyError, 4: ValueError, 8: ValueError, 16: ZeroDivisionError, 32: ValueError, 64: KeyError}


def _raise_flags(flags: int):
    from ._native import ERR_FLAGS
    for bit, msg in ERR_FLAGS.items():
        if flags & bit:
            raise _EXC[bit](msg)


def _run(subGraphs, body, states=("tse", "uts"), merged=True):
    """pack -> device -> body(DeviceGraph) -> check flags -> unpack"""
    from .device import DeviceGraph
    from .devmem import default_mem
    g = pack(subGraphs)
    if g.n_nodes == 0:
        return subGraphs
    d = DeviceGraph(g, mem=default_mem())
    d.clear_errors()
    body(d)
    flags = d.errors()
    d.download(g)
    if flags:
        _raise_flags(flags)
    unpack(g, subGraphs, states=states, merged=merged)
    return subGraphs


def _key(k: str) -> str:
    if k in ("track_state_estimates", "tse"):
        return "tse"
    if k in ("updated_track_states", "uts"):
        return "uts"
    raise KeyError(k)


# ------------------------------------------------------------------ helpers
def compute_track_state_estimates(GraphList, sigma0xy, sigma0rz, sigma0rz2, endcap_boundary):
    """helper.compute_track_state_estimates (helper.py:238-452) on the GPU.

    The dict order is the reference's: reversed(set(nx.all_neighbors(G, node)))
    (:277, :350-351), taken from this interpreter's own set() on the same neighbour
    sequence; the states themselves come from gtf_track_state_estimates. Writes the
    same node attributes and dict entries as the reference (``edge_covariance is
    joint_vector_covariance``, :417-425)."""
    import networkx as nx
    import numpy as np
    from .device import DeviceGraph
    from .graph import mat_from_cov5
    for G in GraphList:
        for node in G.nodes():
            keys = list(set(nx.all_neighbors(G, node)))
            keys.reverse()
            G.nodes[node]["track_state_estimates"] = {k: {} for k in keys}
    g = pack(GraphList)
    if g.n_nodes == 0:
        return GraphList
    p = Params(sigma0xy=sigma0xy, sigma0rz=sigma0rz, sigma0rz2=sigma0rz2, endcap_boundary=endcap_boundary)
    from .devmem import default_mem
    d = DeviceGraph(g, mem=default_mem())
    x = {k: v if isinstance(v, np.ndarray) else v.cpu().numpy() for k, v in d.track_state_estimates(p).items()}
    d.download(g)
    S = g.slot
    vi = 0
    for G in GraphList:
        for node in G.nodes():
            attr = G.nodes[node]
            lo, hi = int(g.slot_ptr[vi]), int(g.slot_ptr[vi + 1])
            ranked = sorted((int(S["tse_rank"][k]), k) for k in range(lo, hi) if S["tse_rank"][k] >= 0)
            keys = list(attr["track_state_estimates"].keys())
            tse = {}
            for (_, k), key in zip(ranked, keys):
                sv = S["tse_sv"][k].copy()
                cov = mat_from_cov5(S["tse_cov"][k])
                th = S["tse_theta"][k]
                xyzr = S["tse_xyzr"][k]
                tse[key] = {"xyzr": (xyzr[0], xyzr[1], xyzr[2], xyzr[3]),
                            "edge_state_vector": sv,
                            "edge_covariance": cov,
                            "joint_vector": [sv[0], sv[1], S["tse_tau"][k]],
                            "joint_vector_covariance": cov,
                            "theta": th[0], "theta2": th[1], "variance_theta": th[2],
                            "var_ms_node": S["tse_var_ms"][k]}
            attr["track_state_estimates"] = tse
            attr["xy_edge_gradient_mean_var"] = tuple(np.float64(v) for v in x["xy_mean_var"][vi])
            attr["zr_edge_gradient_mean_var"] = tuple(np.float64(v) for v in x["zr_mean_var"][vi])
            attr["angle_of_rotation"] = float(x["angle_of_rotation"][vi])
            attr["translation"] = (x["translation"][vi][0], x["translation"][vi][1])
            vi += 1
    return GraphList


def compute_prior_probabilities(GraphList, track_state_key):
    """helper.compute_prior_probabilities (helper.py:30-63)"""
    k = _key(track_state_key)
    p = Params()
    return _run(GraphList, lambda d: d.node_ops(["priors_" + k], p))


def compute_mixture_weights(GraphList, TRACK_STATE_KEY):
    """helper.compute_mixture_weights (helper.py:76-96)"""
    k = _key(TRACK_STATE_KEY)
    p = Params()
    return _run(GraphList, lambda d: d.node_ops(["mw_" + k], p))


def reweight(subGraphs, track_state_estimates_key, reweight_threshold=0.1):
    """helper.reweight incl. calculate_side_norm_factor (helper.py:99-225)"""
    if _key(track_state_estimates_key) != "uts":
        raise KeyError("likelihood")     # the reference reads 'likelihood', absent from TSE entries
    p = Params(reweight_threshold=reweight_threshold)
    return _run(subGraphs, lambda d: d.node_ops(["reweight_uts"], p))


def node_degrees(subGraphs):
    """set node attr 'degree' = active in-edges for every node (the loops around
    helper.query_node_degree_in_edges in every stage main)"""
    return _run(subGraphs, lambda d: d.node_ops(["degree"], Params()))


# ------------------------------------------------------------------- stages
def message_passing(subGraphs, chi2CutFactor, sigma0xy, sigma0rz, sigma0rz2, endcap_boundary):
    """extrapolate_merged_states.message_passing (:406-451)"""
    p = Params(sigma0xy=sigma0xy, sigma0rz=sigma0rz, sigma0rz2=sigma0rz2, endcap_boundary=endcap_boundary,
               chi2_cut=chi2CutFactor)
    return _run(subGraphs, lambda d: d.message_passing(p))


def extrapolate_stage(subGraphs, p: Params):
    """extrapolate_merged_states.main body (:552-566), one fused device call"""
    return _run(subGraphs, lambda d: d.extrapolate(p))


def update_stage(subGraphs, p: Params = None):
    """remove_state_metadata.main body (:29-53)"""
    p = p or Params()
    return _run(subGraphs, lambda d: d.update(p))


def cluster_graphs(subGraphs, track_state_key, chi2_threshold, KL_threshold, p: Params):
    """clustering.cluster body after loading (clustering.py:181-373)"""
    k = _key(track_state_key)
    return _run(subGraphs, lambda d: d.cluster(k, chi2_threshold, KL_threshold, p))


def full_pass(subGraphs, p: Params):
    """extrapolate -> update -> cluster(updated_track_states), fused"""
    return _run(subGraphs, lambda d: d.full_pass(p))


def tag_propagation(G, threshold=0.1):
    """tag_propagation.py:64-164 on one graph: returns (node -> final tag, flips per sweep).
    Tags are written to the node attribute 'tags' (appended, as the script does)."""
    g = pack([G])
    from .device import DeviceGraph
    from .devmem import default_mem
    d = DeviceGraph(g, mem=default_mem())
    radius = [G.nodes[n]["zr"][1] if "zr" in G.nodes[n] else G.nodes[n]["xyzr"][3] for n in G.nodes]
    tags, flips = d.tag_propagation(g.node["tag"], radius, threshold)
    out = {}
    for i, n in enumerate(G.nodes):
        out[n] = int(tags[i])
    return out, flips


# ---------------------------------------------------------------------- I/O
def updated_state_distances(subGraphs):
    """calculate_distance_between_updated_track_states.py (:27-104, pair loop :134-195) on
    the GPU: for every node with an updated_track_states dict and more than one active
    in-edge, every pair i > j of its entries in dict order. Returns one dict per subgraph,
    {node: rows}, rows = [(chi2, <tau>, <theta>, delta_theta, truth, neighbour_i,
    neighbour_j), ...] in the reference's loop order (truth per :190-193 from the nodes'
    'truth_particle')."""
    import numpy as np
    from .device import DeviceGraph
    g = pack(subGraphs)
    out = [dict() for _ in subGraphs]
    if g.n_nodes == 0:
        return out
    truth = np.array([G.nodes[n].get("truth_particle", -1) for G in subGraphs for n in G.nodes()], dtype=np.int64)
    d = DeviceGraph(g)
    ptr, cols = d.updated_state_distances(truth)
    ptr = ptr.cpu().numpy()
    c = {k: v.cpu().numpy() for k, v in cols.items()}
    S = g.slot
    node_of = [(si, n) for si, G in enumerate(subGraphs) for n in G.nodes()]
    for v in np.nonzero(np.diff(ptr) > 0)[0]:
        lo, hi = int(g.slot_ptr[v]), int(g.slot_ptr[v + 1])
        keys = sorted((k for k in range(lo, hi) if S["uts_rank"][k] >= 0), key=lambda k: S["uts_rank"][k])
        si, n = node_of[v]
        rows = []
        t = int(ptr[v])
        for i in range(len(keys)):
            for j in range(i):
                rows.append((float(c["chi2"][t]), float(c["avg_tau"][t]), float(c["avg_theta"][t]),
                             float(c["delta_theta"][t]), int(c["truth"][t]), S["slot_key"][keys[i]],
                             S["slot_key"][keys[j]]))
                t += 1
        out[si][n] = rows
    return out


def read_subgraphs(inputDir: str) -> List:
    """the stages' loader: glob order, pickled nx.DiGraph (== nx.read_gpickle)"""
    out = []
    for f in glob.glob(inputDir + "*" + SUBGRAPH_SUFFIX):
        with open(f, "rb") as fh:
            out.append(pickle.load(fh))
    return out


def save_network(directory, i, subGraph):
    """helper.save_network (helper.py:585-587): nx.write_gpickle == pickle HIGHEST_PROTOCOL"""
    with open(directory + str(i) + SUBGRAPH_SUFFIX, "wb") as fh:
        pickle.dump(subGraph, fh, pickle.HIGHEST_PROTOCOL)
