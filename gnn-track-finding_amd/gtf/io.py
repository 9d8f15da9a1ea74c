"""Event CSV -> packed TrackGraph, directly (no networkx, no pandas row loops).

The reference builds its graph with O(N*H) pandas lookups
(helper.load_nodes_edges + construct_graph, helper.py:465-545; 34 s of a 35 s
stage for one volume). Here the CSVs are read with numpy and the CSR
is assembled vectorised. Semantics kept:

* nodes: ``layer_id`` in [min_volume*1000, (max_volume+1)*1000] (helper.py:526-531,
  pandas ``between`` is inclusive), r = sqrt(x^2 + y^2), in_volume_layer_id =
  layer_id % 100, node order = CSV order;
* edges: ``edges.csv`` has a "<N> <E>" first line, then node2,node1,weight
  (helper.py:537-543); both directions are added when both ends are kept
  (helper.py:512-518).

Truth joins (particle ids, module ids) are not on the packed path; build_networkx adds
them to the networkx graph the drop-in event conversion writes.
"""
from __future__ import annotations

import numpy as np

from .graph import TrackGraph


def read_nodes(path: str, min_volume: int, max_volume: int):
    """the reference's pandas parser (helper.load_nodes_edges, helper.py:524-531)"""
    import pandas as pd
    a = pd.read_csv(path)
    lo, hi = min_volume * 1000, (max_volume + 1) * 1000
    lid = a["layer_id"].to_numpy()
    keep = (lid >= lo) & (lid <= hi)
    x, y, z = (a[c].to_numpy(np.float64)[keep] for c in ("x", "y", "z"))
    return (a["node_idx"].to_numpy(np.int64)[keep], x, y, z, edge_length_xy(x, y), lid[keep].astype(np.int64))


def edge_length_xy(x, y):
    """helper.edge_length_xy (helper.py:12-13) as the reference evaluates it, on numpy
    float64 scalars of a DataFrame row: ``row.x**2`` is the C library's pow(x, 2), which
    differs from x * x in the last bit for some x (6 of the 8,748 vol-7 hits), where numpy's
    array power squares; so the squares go through math.pow (the same pow)."""
    import math
    sq = np.frompyfunc(math.pow, 2, 1)
    x2 = sq(np.asarray(x, np.float64), 2.0).astype(np.float64)
    y2 = sq(np.asarray(y, np.float64), 2.0).astype(np.float64)
    return np.sqrt(x2 + y2)


def read_edges(path: str):
    with open(path) as f:
        f.readline()                      # "<N> <E>"
        f.readline()                      # node2,node1,weight
        e = np.loadtxt(f, delimiter=",", dtype=np.float64, ndmin=2)
    return e[:, 0].astype(np.int64), e[:, 1].astype(np.int64)


def load_event(event_prefix: str, min_volume: int, max_volume: int, params=None) -> TrackGraph:
    """``event_prefix`` like ``.../event_1_filtered_graph_`` (nodes.csv / edges.csv appended)."""
    from .synth import _assemble
    from .params import Params
    ids, x, y, z, r, layer = read_nodes(event_prefix + "nodes.csv", min_volume, max_volume)
    n2, n1 = read_edges(event_prefix + "edges.csv")
    pos = {int(v): i for i, v in enumerate(ids)}
    idx = np.full(int(max(ids.max(), n1.max(), n2.max())) + 1 if ids.size else 1, -1, np.int64)
    idx[ids] = np.arange(ids.size)
    a, b = idx[n1], idx[n2]
    ok = (a >= 0) & (b >= 0)
    a, b = a[ok], b[ok]
    # add_edge(node1, node2) then add_edge(node2, node1); duplicates collapse
    src = np.concatenate([np.stack([a, b], 1), np.stack([b, a], 1)], 1).reshape(-1, 2)
    _, first = np.unique(src[:, 0] * ids.size + src[:, 1], return_index=True)
    src = src[np.sort(first)]
    g = _assemble(ids.size, src[:, 0], src[:, 1], x, y, z, r, layer, params or Params())
    g.node["node_id"] = ids.copy()
    del pos
    return g


def read_truth(path: str, node_ids: np.ndarray) -> np.ndarray:
    """truth_particle per node, aligned with ``node_ids`` (-1 where absent).

    ``path`` is a hit->particle mapping CSV with ``node_idx`` and ``particle_id``
    columns (the reference's event_truth/*-full-mapping-*.csv, or a two-column
    extract of it). A node's truth is the particle of its first row -- the first of
    ``unique()`` in helper.construct_graph (helper.py:468-471, 493)."""
    a = np.genfromtxt(path, delimiter=",", names=True, dtype=None, encoding=None)
    nid = a["node_idx"].astype(np.int64)
    pid = a["particle_id"].astype(np.int64)
    u, first = np.unique(nid, return_index=True)
    out = np.full(node_ids.shape[0], -1, np.int64)
    pos = np.searchsorted(u, node_ids)
    ok = (pos < u.size) & (u[np.minimum(pos, u.size - 1)] == node_ids)
    out[ok] = pid[first[pos[ok]]]
    return out


def aggregate_truth(event_path: str, truth_event_path: str, truth_event_file: str) -> None:
    """helper.load_save_truth (helper.py:548-582) without its per-row pandas lookups: one
    row per nodes_to_hits row (its order), with the hit's particle (truth.csv) and its
    volume / layer / module (hits.csv) -- each hit must occur exactly once in those files,
    where the reference's ``.item()`` raises ValueError otherwise -- and the particle's
    nhits from particles.csv, 0.0 where the particle is absent or listed twice (the
    reference's ``except ValueError``). Written as the reference writes it (nhits float)."""
    import pandas as pd
    hits_particles = pd.read_csv(truth_event_path + "truth.csv")
    particles_nhits = pd.read_csv(truth_event_path + "particles.csv")
    hits_module_id = pd.read_csv(truth_event_path + "hits.csv")
    nodes_hits = pd.read_csv(event_path + "nodes_to_hits.csv")
    hit = nodes_hits["hit_id"]

    def lookup(df, col):
        cnt = hit.map(df["hit_id"].value_counts()).fillna(0)
        if (cnt != 1).any():
            raise ValueError("can only convert an array of size 1 to a Python scalar (hit_id %d)"
                             % int(hit[cnt != 1].iloc[0]))
        return hit.map(df.drop_duplicates("hit_id").set_index("hit_id")[col])

    truth = pd.DataFrame({"node_idx": nodes_hits["node_idx"], "hit_id": hit,
                          "particle_id": lookup(hits_particles, "particle_id"),
                          "volume_id": lookup(hits_module_id, "volume_id"),
                          "layer_id": lookup(hits_module_id, "layer_id"),
                          "module_id": lookup(hits_module_id, "module_id")})
    pid = truth["particle_id"]
    once = pid.map(particles_nhits["particle_id"].value_counts()).fillna(0) == 1
    nh = pid.map(particles_nhits.drop_duplicates("particle_id").set_index("particle_id")["nhits"])
    truth["nhits"] = np.where(once, nh, 0).astype(np.float64)
    truth.to_csv(truth_event_file, index=False)


def truth_joins(truth):
    """construct_graph's truth joins (helper.py:468-481) on the mapping DataFrame: per
    node_idx, its particles (first = truth_particle), hits and modules, each distinct in
    row order, and every hit's particle (a hit listed twice makes the reference's
    ``.item()`` raise ValueError). Returns {node_idx: (truth_particle, module_ids,
    hit_ids, [particle per hit])}. Vectorised: the distinct (node, value) pairs in row
    order, grouped by node with a stable sort."""
    import pandas as pd
    node = truth["node_idx"].to_numpy(np.int64)
    hit = truth["hit_id"].to_numpy(np.int64)
    pid = truth["particle_id"].to_numpy(np.int64)
    uh, first, cnt = np.unique(hit, return_index=True, return_counts=True)
    if (cnt != 1).any():
        raise ValueError("can only convert an array of size 1 to a Python scalar (hit_id %d)" % int(uh[cnt != 1][0]))

    def distinct(col):
        d = pd.DataFrame({"n": node, "v": truth[col].to_numpy(np.int64)}).drop_duplicates()
        n, v = d["n"].to_numpy(), d["v"].to_numpy()
        o = np.argsort(n, kind="stable")
        un, start = np.unique(n[o], return_index=True)
        return un, np.split(v[o], start[1:])

    nodes, pids = distinct("particle_id")
    _, modules = distinct("module_id")
    _, hits = distinct("hit_id")
    pid_of_hit = pid[first]                      # hits are unique: every hit's one row
    out = {}
    for n, p, m, h in zip(nodes.tolist(), pids, modules, hits):
        out[n] = (int(p[0]), m, h, pid_of_hit[np.searchsorted(uh, h)].tolist())
    return out


def build_networkx(event_prefix: str, min_volume: int, max_volume: int, truth_csv: str = None, truth=None):
    """The reference's event_conversion graph (event_conversion.py:53-88): construct_graph
    (helper.py:465-521) -- nodes in CSV order with GNN_Measurement, xy, zr, xyzr,
    volume/layer ids, module_id, truth_particle, hit_dissociation and tags, with the
    reference's value types (numpy float64 coordinates and ids from its row Series); both
    directions of every CSV edge in row order -- then nx.DiGraph and the weakly connected
    subgraphs, copied. Returns the list of subgraphs (no state estimates yet).
    truth: the full mapping DataFrame (node_idx, hit_id, particle_id, ..., module_id), as
    event_conversion reads it: every construct_graph attribute. truth_csv: a two-column
    node_idx -> particle_id extract instead (truth_particle only; no module_id /
    hit_dissociation, which only extraction's node merging and the efficiency read)."""
    import networkx as nx
    from GNN_Measurement.GNN_Measurement import GNN_Measurement
    ids, x, y, z, r, layer = read_nodes(event_prefix + "nodes.csv", min_volume, max_volume)
    joins = truth_joins(truth) if truth is not None else None
    tp = read_truth(truth_csv, ids) if truth_csv else np.full(ids.size, -1, np.int64)
    G = nx.DiGraph()
    for i in range(ids.size):
        n = int(ids[i])
        xi, yi, zi, ri = x[i], y[i], z[i], r[i]
        vol, lay = np.float64(int(layer[i] / 1000)), np.float64(int(layer[i] % 100))
        if joins is not None:
            if n not in joins:   # grouped_pid.loc[...].item() of no row
                raise ValueError("can only convert an array of size 1 to a Python scalar (node %d)" % n)
            t, modules, hits, hit_pids = joins[n]
            G.add_node(n, GNN_Measurement=GNN_Measurement(xi, yi, zi, ri, truth_particle=t, n=n),
                       xy=(xi, yi), zr=(zi, ri), xyzr=(xi, yi, zi, ri), volume_id=vol, in_volume_layer_id=lay,
                       vivl_id=(vol, lay), module_id=modules, truth_particle=t,
                       hit_dissociation={"hit_id": hits, "particle_id": hit_pids}, tags=[n])
        else:
            t = int(tp[i])
            G.add_node(n, GNN_Measurement=GNN_Measurement(xi, yi, zi, ri, truth_particle=t, n=n),
                       xy=(xi, yi), zr=(zi, ri), xyzr=(xi, yi, zi, ri), volume_id=vol, in_volume_layer_id=lay,
                       vivl_id=(vol, lay), truth_particle=t, tags=[n])
    n2, n1 = read_edges(event_prefix + "edges.csv")
    for a, b in zip(n1.tolist(), n2.tolist()):
        if a in G and b in G:
            G.add_edge(a, b)
            G.add_edge(b, a)
    G = nx.DiGraph(G)
    return [G.subgraph(c).copy() for c in nx.weakly_connected_components(G)]


def csr_from_rows(ids, a, b, device=None):
    """The packed CSR of an event from its columns (node ids in CSV order; edge rows
    add_edge(a, b) then add_edge(b, a)): gtf_build_event_csr on the host, or
    gtf_build_event_csr_device on ``device`` (the build on the GPU, the same arrays bit
    for bit). Returns (outputs dict of host arrays, n_edges, n_subgraphs)."""
    import ctypes
    from . import _native as nat
    N, R = int(ids.size), int(a.size)
    ids = np.ascontiguousarray(ids, np.int64)
    a, b = np.ascontiguousarray(a, np.int64), np.ascontiguousarray(b, np.int64)
    shapes = {"order": max(N, 1), "sub_id": max(N, 1), "slot_ptr": N + 1, "out_ptr": N + 1,
              "slot_src": max(2 * R, 1), "tse_rank": max(2 * R, 1), "out_slot": max(2 * R, 1)}
    names = ("order", "sub_id", "slot_ptr", "slot_src", "tse_rank", "out_ptr", "out_slot")
    if device is None:
        o = {k: np.zeros(n, np.int32) for k, n in shapes.items()}
        vp = lambda t: ctypes.c_void_p(t.ctypes.data)  # noqa: E731
        ev = nat.GtfEventCsr(N, R, vp(ids) if N else None, vp(a) if R else None, vp(b) if R else None,
                             *[vp(o[k]) for k in names], 0, 0, 0)
        nat.check(nat.lib().gtf_build_event_csr(ctypes.byref(ev)))
        return o, int(ev.n_edges), int(ev.n_subgraphs)
    import torch
    L = nat.lib()
    t_ids, t_a, t_b = (torch.from_numpy(x).to(device) for x in (ids, a, b))
    o = {k: torch.zeros(n, dtype=torch.int32, device=device) for k, n in shapes.items()}
    ws_bytes = int(L.gtf_build_event_device_workspace_bytes(N, R))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ev = nat.GtfEventCsr(N, R, vp(t_ids) if N else None, vp(t_a) if R else None, vp(t_b) if R else None,
                         *[vp(o[k]) for k in names], 0, 0, 0)
    stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    nat.check(L.gtf_build_event_csr_device(ctypes.byref(ev), vp(ws), ws_bytes, stream))
    return {k: v.cpu().numpy() for k, v in o.items()}, int(ev.n_edges), int(ev.n_subgraphs)


def build_event_csr(event_prefix: str, min_volume: int, max_volume: int, device=None):
    """Event conversion's graph straight to the packed CSR (gtf_build_event_csr, or on
    the GPU with ``device``: gtf_build_event_csr_device): the same TrackGraph as pack()
    of build_networkx's subgraphs with their track_state_estimates keys in the
    reference's set order, without networkx. Returns (graph with empty states -- every
    edge active, has_tse set, tse_rank in dict order -- and vivl [N, 2] = (volume_id,
    in_volume_layer_id))."""
    from .graph import NODE_FIELDS, SLOT_FIELDS, check_layout, empty_arrays
    ids, x, y, z, r, layer = read_nodes(event_prefix + "nodes.csv", min_volume, max_volume)
    n2, n1 = read_edges(event_prefix + "edges.csv")
    N = int(ids.size)
    ids = np.ascontiguousarray(ids, np.int64)
    o, E, n_sub = csr_from_rows(ids, n1, n2, device)
    order = o["order"][:N].astype(np.int64)
    node, slot = empty_arrays(NODE_FIELDS, N), empty_arrays(SLOT_FIELDS, E)
    gnn = np.stack([x, y, z, r], axis=1)[order]
    node["gnn"] = gnn
    node["xyzr"] = gnn.copy()
    node["layer"] = (layer[order] % 100).astype(np.float64)
    node["has_tse"][:] = 1
    node["tag"] = ids[order]
    node["node_id"] = ids[order]
    node["sub_id"] = o["sub_id"][:N].copy()
    src = o["slot_src"][:E].copy()
    slot["slot_src"] = src
    slot["slot_key"] = ids[order][src] if E else np.zeros(0, np.int64)
    slot["is_edge"][:] = 1
    slot["rev_edge"][:] = 1
    slot["act"][:] = 1
    slot["tse_rank"] = o["tse_rank"][:E].copy()
    g = TrackGraph(N, E, o["slot_ptr"].copy(), o["out_ptr"].copy(), o["out_slot"][:E].copy(), node, slot, n_sub)
    check_layout(g)
    lay = layer[order]
    vivl = np.stack([(lay / 1000).astype(np.int64), lay % 100], 1).astype(np.float64)
    return g, vivl
