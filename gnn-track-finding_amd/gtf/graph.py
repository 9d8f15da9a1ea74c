"""Packed CSR layout of a list of reference subgraphs (host side).

The reference keeps every subgraph as a networkx ``DiGraph`` whose nodes carry
attribute dicts (SURVEY.md §8b "Node attributes"). The hot path needs them as
flat structure-of-arrays so one HIP launch can cover every subgraph of every
event. ``pack`` turns ``list[nx.DiGraph]`` into a :class:`TrackGraph`;
``unpack`` writes the results back into the same graph objects with the
reference's attribute schema (key order, aliasing and mutation semantics of
src/extrapolate/extrapolate_merged_states.py:375-385,443-447,
src/clustering/clustering.py:291-293, src/utilities/helper.py:30-225).

Layout (see DESIGN.md "Data layout in HBM"):

* nodes are numbered 0..N-1 in subgraph-list order, then in each subgraph's
  node-iteration order (the order every reference stage loops in);
* a node's *slots* are the union of its in-edge senders and the keys of its
  ``track_state_estimates`` (TSE) / ``updated_track_states`` (UTS) dicts,
  sorted by sender node index (orphan keys whose node left the subgraph go
  last). Slot ``k`` of node ``v`` describes the directed edge
  ``slot_src[k] -> v`` and the state ``v`` holds for that sender;
* the dict order of a state dict is carried explicitly as a per-slot rank
  (``tse_rank`` / ``uts_rank``; -1 = key absent) -- never re-sorted;
* per-edge flags (``activated``, edge ``mixture_weight``) are stored per slot,
  i.e. receiver-major. The out-view ``out_ptr``/``out_slot`` lists each
  node's successors in ``G.neighbors`` order (the order message passing walks
  them, extrapolate_merged_states.py:430).

Every state covariance on the path is block diagonal after the reference's
aliasing (helper.py:422-425, extrapolate_merged_states.py:362-365), so a
covariance is stored as 5 numbers ``c00 c01 c10 c11 c22``.
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional

import numpy as np

F64 = np.float64
NAN = float("nan")

# slot-count buckets of the node-kernel schedule (gtf_graph.sched): 4, 8, 16, 32, 64 lanes
# per node; nodes with more slots run one thread each (n_big)
BUCKETS = ((0, 4), (5, 8), (9, 16), (17, 32), (33, 64))

# covariance packing order
COV5 = ((0, 0), (0, 1), (1, 0), (1, 1), (2, 2))


def cov5_from_mat(m) -> np.ndarray:
    m = np.asarray(m, dtype=F64)
    return np.array([m[0, 0], m[0, 1], m[1, 0], m[1, 1], m[2, 2]], dtype=F64)


def mat_from_cov5(c) -> np.ndarray:
    m = np.zeros((3, 3), dtype=F64)
    m[0, 0], m[0, 1], m[1, 0], m[1, 1], m[2, 2] = c[0], c[1], c[2], c[3], c[4]
    return m


# --------------------------------------------------------------------------
# container
# --------------------------------------------------------------------------
NODE_FIELDS = {
    # name: (dtype, trailing shape, fill)
    "gnn": (F64, (4,), NAN),          # GNN_Measurement x, y, z, r
    "xyzr": (F64, (4,), NAN),         # node attr 'xyzr' (clustering reads this one)
    "layer": (F64, (), NAN),          # 'in_volume_layer_id'
    "has_merged": (np.uint8, (), 0),
    "merged_state": (F64, (3,), NAN),
    "merged_cov": (F64, (5,), NAN),
    "merged_prior": (F64, (), NAN),
    "has_tse": (np.uint8, (), 0),     # node has a 'track_state_estimates' key
    "has_uts": (np.uint8, (), 0),     # node has an 'updated_track_states' key
    "degree": (np.int32, (), -1),
    "tag": (np.int64, (), -1),        # tags[-1]
    "node_id": (np.int64, (), -1),    # original networkx node id
    "sub_id": (np.int32, (), -1),     # index of the subgraph the node came from
}

SLOT_FIELDS = {
    "slot_src": (np.int32, (), -1),   # sender node index, -1 = orphan key
    "slot_key": (np.int64, (), -1),   # sender's original id (dict key)
    "is_edge": (np.uint8, (), 0),     # edge sender -> receiver exists
    "rev_edge": (np.uint8, (), 0),    # edge receiver -> sender exists
    "act": (np.uint8, (), 0),         # edge attr 'activated'
    "edge_mw": (F64, (), NAN),        # edge attr 'mixture_weight' (NaN = absent)
    "send_mw": (F64, (), NAN),        # sender's TSE[receiver]['mixture_weight']
    # track_state_estimates entry (at the receiver, keyed by sender)
    "tse_rank": (np.int32, (), -1),
    "tse_sv": (F64, (3,), NAN),       # edge_state_vector a, b, c
    "tse_tau": (F64, (), NAN),        # joint_vector[2]
    "tse_cov": (F64, (5,), NAN),
    "tse_xyzr": (F64, (4,), NAN),
    "tse_prior": (F64, (), NAN),
    "tse_mw": (F64, (), NAN),
    "tse_theta": (F64, (3,), NAN),    # theta, theta2, variance_theta
    "tse_var_ms": (F64, (), NAN),     # var_ms_node
    # updated_track_states entry
    "uts_rank": (np.int32, (), -1),
    "uts_sv": (F64, (3,), NAN),
    "uts_tau": (F64, (), NAN),
    "uts_cov": (F64, (5,), NAN),
    "uts_xyzr": (F64, (4,), NAN),
    "uts_lik": (F64, (), NAN),
    "uts_mw": (F64, (), NAN),
    "uts_prior": (F64, (), NAN),
    "uts_lr": (F64, (), NAN),         # lr_layer_norm (int in the reference)
    "uts_side": (np.int8, (), -1),    # 0 left, 1 right, -1 absent
    "uts_fresh": (np.uint8, (), 0),   # entry (re)created by the last message passing
}


@dataclasses.dataclass
class TrackGraph:
    """Structure-of-arrays CSR view of a list of subgraphs (or events)."""

    n_nodes: int
    n_slots: int
    slot_ptr: np.ndarray          # int32 [N+1]
    out_ptr: np.ndarray           # int32 [N+1]
    out_slot: np.ndarray          # int32 [E] slot index of each out-edge, successor order
    node: dict                    # name -> array [N, ...]
    slot: dict                    # name -> array [S, ...]
    n_subgraphs: int = 1

    @property
    def n_edges(self) -> int:
        return int(self.out_slot.shape[0])

    def copy(self) -> "TrackGraph":
        return TrackGraph(self.n_nodes, self.n_slots, self.slot_ptr.copy(), self.out_ptr.copy(),
                          self.out_slot.copy(), {k: v.copy() for k, v in self.node.items()},
                          {k: v.copy() for k, v in self.slot.items()}, self.n_subgraphs)

    # convenience accessors -------------------------------------------------
    def __getattr__(self, name):
        d = self.__dict__
        if "node" in d and name in d["node"]:
            return d["node"][name]
        if "slot" in d and name in d["slot"]:
            return d["slot"][name]
        raise AttributeError(name)

    def slot_dst(self) -> np.ndarray:
        """receiver node index of every slot"""
        return np.repeat(np.arange(self.n_nodes, dtype=np.int32), np.diff(self.slot_ptr))


def empty_arrays(fields: dict, n: int) -> dict:
    out = {}
    for name, (dt, shape, fill) in fields.items():
        out[name] = np.full((n,) + shape, fill, dtype=dt)
    return out


def check_layout(g: TrackGraph) -> None:
    """Validate every index the HIP kernels will dereference (host-side guard)."""
    N, S = g.n_nodes, g.n_slots
    sp, op = g.slot_ptr, g.out_ptr
    assert sp.shape == (N + 1,) and op.shape == (N + 1,)
    assert sp[0] == 0 and sp[-1] == S and np.all(np.diff(sp) >= 0)
    assert op[0] == 0 and op[-1] == g.n_edges and np.all(np.diff(op) >= 0)
    src = g.slot["slot_src"]
    assert src.shape == (S,)
    assert np.all((src >= -1) & (src < N))
    assert np.all(g.slot["is_edge"][src < 0] == 0), "orphan slot flagged as an edge"
    if g.n_edges:
        os_ = g.out_slot
        assert np.all((os_ >= 0) & (os_ < S))
        assert np.all(g.slot["is_edge"][os_] == 1)
        # every out-edge must point at a slot whose sender is the source node
        owner = np.repeat(np.arange(N, dtype=np.int32), np.diff(op))
        assert np.array_equal(src[os_], owner), "out_slot does not match slot_src"
    for name, (dt, shape, _) in NODE_FIELDS.items():
        assert g.node[name].shape == (N,) + shape and g.node[name].dtype == dt, name
    for name, (dt, shape, _) in SLOT_FIELDS.items():
        assert g.slot[name].shape == (S,) + shape and g.slot[name].dtype == dt, name


def renumber(g: TrackGraph, order) -> tuple:
    """The same graph with node i' = order[i'] of g: node arrays permuted, every
    receiver's slot segment moved along unchanged (its slots keep their order, so
    dict insertion order and the reference's per-receiver orders are untouched),
    slot_src remapped, every sender's out-list kept in successor order. The pass is
    equivariant under this relabelling (its semantics reach node order only through
    slot order, out-list order and explicit dict ranks). Returns (graph, slot_perm)
    with new slot s' = old slot slot_perm[s']; g.node[f][order] and
    g.slot[f][slot_perm] give the new arrays, and the inverse scatters them back."""
    order = np.asarray(order, dtype=np.int64)
    N = g.n_nodes
    if order.shape != (N,) or (N and not np.array_equal(np.sort(order), np.arange(N))):
        raise ValueError("order must be a permutation of the %d nodes" % N)
    sp = g.slot_ptr.astype(np.int64)
    deg = np.diff(sp)
    new_sp = np.zeros(N + 1, np.int64)
    np.cumsum(deg[order], out=new_sp[1:])
    # new slot s' of new node i' (offset j in its segment) = old slot sp[order[i']] + j
    owner = np.repeat(np.arange(N, dtype=np.int64), deg[order])
    slot_perm = sp[order][owner] + (np.arange(new_sp[-1]) - new_sp[owner]) if N else np.zeros(0, np.int64)
    new_of_old_node = np.empty(N, np.int64)
    new_of_old_node[order] = np.arange(N)
    new_of_old_slot = np.empty(g.n_slots, np.int64)
    new_of_old_slot[slot_perm] = np.arange(g.n_slots)
    node = {k: v[order].copy() for k, v in g.node.items()}
    slot = {k: v[slot_perm].copy() for k, v in g.slot.items()}
    src = slot["slot_src"].astype(np.int64)
    slot["slot_src"] = np.where(src >= 0, new_of_old_node[np.maximum(src, 0)], -1).astype(g.slot["slot_src"].dtype)
    op = g.out_ptr.astype(np.int64)
    odeg = np.diff(op)
    new_op = np.zeros(N + 1, np.int64)
    np.cumsum(odeg[order], out=new_op[1:])
    oown = np.repeat(np.arange(N, dtype=np.int64), odeg[order])
    old_pos = op[order][oown] + (np.arange(new_op[-1]) - new_op[oown]) if N else np.zeros(0, np.int64)
    out_slot = new_of_old_slot[g.out_slot.astype(np.int64)[old_pos]] if g.n_edges else g.out_slot.copy()
    h = TrackGraph(N, g.n_slots, new_sp.astype(np.int32), new_op.astype(np.int32), out_slot.astype(np.int32),
                   node, slot, g.n_subgraphs)
    check_layout(h)
    return h, slot_perm


GROUPS = ((2, 0, 2), (4, 3, 4), (8, 5, 8), (16, 9, 16), (32, 17, 32), (64, 33, 64))   # (lanes, min, max slots)


def padded(g: TrackGraph, tile: int = 4096) -> tuple:
    """The padded tile layout of the node kernel (gtf_graph.pad_*): nodes grouped by the
    lane-group size G of their slot count (GROUPS), every node of group G owning exactly G
    slots -- its own, then inert padding slots (orphan, no edge, no key in either dict,
    which every op treats as an absent key) -- and T tiles that each hold the same number
    c_G of group-G nodes (the group's nodes in host order, cut into T runs; the few
    missing ones are dummy nodes: no slots of their own, an empty TSE dict, alone in their
    subgraph). Node (t, G, i) is t * TN + off_G + i and its slots start at t * TS + soff_G
    + i * G, so the node kernel finds every node and slot by arithmetic. Nodes with more
    than 64 slots follow the tiles unpadded. Returns (graph, node_of_new, slot_of_new,
    plan): old node / slot of every new one (-1 = dummy / padding) and the tile plan
    {"tiles", "tile_nodes", "tile_slots", "count" (c_G per GROUPS entry)}."""
    N, S = g.n_nodes, g.n_slots
    sp = g.slot_ptr.astype(np.int64)
    deg = np.diff(sp)
    T = max(1, -(-N // tile))
    lists = [np.nonzero((deg >= lo) & (deg <= hi))[0] for _, lo, hi in GROUPS]
    big = np.nonzero(deg > 64)[0]
    cnt = [-(-len(L) // T) for L in lists]
    TN = int(sum(cnt))
    TS = int(sum(c * G for c, (G, _, _) in zip(cnt, GROUPS)))
    n_new = T * TN + len(big)
    node_of_new = np.full(n_new, -1, np.int64)
    start_new = np.zeros(n_new + 1, np.int64)   # slot_ptr of the new graph
    cap_new = np.zeros(n_new, np.int64)
    off = soff = 0
    for L, c, (G, _, _) in zip(lists, cnt, GROUPS):
        j = np.arange(T * c)
        t, i = j // max(c, 1), j % max(c, 1)
        v = t * TN + off + i
        if c:
            node_of_new[v[:len(L)]] = L
            start_new[v] = t * TS + soff + i * G
            cap_new[v] = G
        off += c
        soff += c * G
    vb = T * TN + np.arange(len(big))
    node_of_new[vb] = big
    cap_new[vb] = deg[big]
    start_new[vb] = T * TS + np.concatenate([[0], np.cumsum(deg[big])[:-1]]) if len(big) else 0
    S_new = int(T * TS + deg[big].sum())
    start_new[n_new] = S_new
    assert np.all(np.diff(start_new) == cap_new)
    real = node_of_new >= 0
    new_of_old = np.empty(N, np.int64)
    new_of_old[node_of_new[real]] = np.nonzero(real)[0]
    # slots: the old segment of each real node at the start of its new one
    slot_of_new = np.full(S_new, -1, np.int64)
    if S:
        owner_old = np.repeat(np.arange(N), deg)
        new_slot = start_new[new_of_old[owner_old]] + (np.arange(S) - sp[owner_old])
        slot_of_new[new_slot] = np.arange(S)
    new_of_old_slot = np.empty(S, np.int64)
    new_of_old_slot[slot_of_new[slot_of_new >= 0]] = np.nonzero(slot_of_new >= 0)[0]
    node = empty_arrays(NODE_FIELDS, n_new)
    for k in NODE_FIELDS:
        node[k][real] = g.node[k][node_of_new[real]]
    dummy = ~real
    node["has_tse"][dummy] = 1   # an empty dict: pruning and priors find no key
    sub0 = int(g.node["sub_id"].max()) + 1 if N else 0
    node["sub_id"][dummy] = sub0 + np.arange(int(dummy.sum()))   # alone in its subgraph
    slot = empty_arrays(SLOT_FIELDS, S_new)
    rs = slot_of_new >= 0
    for k in SLOT_FIELDS:
        slot[k][rs] = g.slot[k][slot_of_new[rs]]
    src = slot["slot_src"].astype(np.int64)
    slot["slot_src"] = np.where(src >= 0, new_of_old[np.maximum(src, 0)], -1).astype(np.int32)
    # out-lists in the new node order, successor order kept
    op = g.out_ptr.astype(np.int64)
    odeg_new = np.zeros(n_new, np.int64)
    odeg_new[real] = np.diff(op)[node_of_new[real]]
    new_op = np.zeros(n_new + 1, np.int64)
    np.cumsum(odeg_new, out=new_op[1:])
    E = g.n_edges
    out_slot = np.zeros(E, np.int64)
    if E:
        owner_o = np.repeat(np.arange(N), np.diff(op))
        pos = new_op[new_of_old[owner_o]] + (np.arange(E) - op[owner_o])
        out_slot[pos] = new_of_old_slot[g.out_slot.astype(np.int64)]
    h = TrackGraph(n_new, S_new, start_new.astype(np.int32), new_op.astype(np.int32), out_slot.astype(np.int32),
                   node, slot, g.n_subgraphs)
    check_layout(h)
    plan = {"tiles": T, "tile_nodes": TN, "tile_slots": TS, "count": [int(c) for c in cnt]}
    return h, node_of_new, slot_of_new, plan


# --------------------------------------------------------------------------
# pack: list[nx.DiGraph] -> TrackGraph
# --------------------------------------------------------------------------
def _f(x) -> float:
    return float(x)


def pack(subgraphs, like: Optional[TrackGraph] = None) -> TrackGraph:
    """Pack reference subgraphs (list of ``nx.DiGraph``) into a TrackGraph.

    ``like``: reuse the slot layout of an earlier pack of the same nodes (a
    stage that removes state keys, e.g. remove_state_metadata, then still
    packs onto the slots of its input so arrays compare index for index).
    """
    # global node numbering ------------------------------------------------
    node_ids: List = []
    sub_of: List[int] = []
    local_maps: List[dict] = []
    for si, G in enumerate(subgraphs):
        m = {}
        for n in G.nodes:
            m[n] = len(node_ids)
            node_ids.append(n)
            sub_of.append(si)
        local_maps.append(m)
    N = len(node_ids)
    nodeA = empty_arrays(NODE_FIELDS, N)

    slot_rows = []           # per node: list of (sender_idx or -1, key)
    slot_ptr = np.zeros(N + 1, dtype=np.int64)
    gi = 0
    for si, G in enumerate(subgraphs):
        lm = local_maps[si]
        for v in G.nodes:
            attr = G.nodes[v]
            keys = []
            seen = set()
            for u in G.predecessors(v):
                if u not in seen:
                    seen.add(u)
                    keys.append(u)
            for dk in ("track_state_estimates", "updated_track_states"):
                d = attr.get(dk)
                if d is not None:
                    for u in d.keys():
                        if u not in seen:
                            seen.add(u)
                            keys.append(u)
            if like is not None:
                lo_, hi_ = int(like.slot_ptr[gi]), int(like.slot_ptr[gi + 1])
                row = [(int(like.slot["slot_src"][k]), int(like.slot["slot_key"][k])) for k in range(lo_, hi_)]
                rk = set(r[1] for r in row)
                assert all(int(u) in rk for u in keys), "pack(like=...): new state key not in layout"
            else:
                inside = sorted((lm[u], u) for u in keys if u in lm)
                orphans = [(-1, u) for u in keys if u not in lm]
                row = inside + orphans
            slot_rows.append(row)
            slot_ptr[gi + 1] = slot_ptr[gi] + len(row)
            gi += 1
    S = int(slot_ptr[-1])
    slotA = empty_arrays(SLOT_FIELDS, S)

    # lookup (receiver idx, sender key) -> slot
    slot_of = {}
    for vi, row in enumerate(slot_rows):
        base = int(slot_ptr[vi])
        for j, (ui, key) in enumerate(row):
            slot_of[(vi, key)] = base + j
            slot_of[(vi, int(key))] = base + j
            slotA["slot_src"][base + j] = ui
            slotA["slot_key"][base + j] = int(key)

    out_ptr = np.zeros(N + 1, dtype=np.int64)
    out_slot = []

    gi = 0
    for si, G in enumerate(subgraphs):
        lm = local_maps[si]
        for v in G.nodes:
            attr = G.nodes[v]
            vi = gi
            gm = attr.get("GNN_Measurement")
            if gm is not None:
                nodeA["gnn"][vi] = (_f(gm.x), _f(gm.y), _f(gm.z), _f(gm.r))
            if "xyzr" in attr:
                nodeA["xyzr"][vi] = [_f(c) for c in attr["xyzr"]]
            if "in_volume_layer_id" in attr:
                nodeA["layer"][vi] = _f(attr["in_volume_layer_id"])
            if "merged_state" in attr:
                nodeA["has_merged"][vi] = 1
                nodeA["merged_state"][vi] = np.asarray(attr["merged_state"], dtype=F64)
                nodeA["merged_cov"][vi] = cov5_from_mat(attr["merged_cov"])
                nodeA["merged_prior"][vi] = _f(attr.get("merged_prior", NAN))
            if "degree" in attr:
                nodeA["degree"][vi] = int(attr["degree"])
            tags = attr.get("tags")
            nodeA["tag"][vi] = int(tags[-1]) if tags else int(v)
            nodeA["node_id"][vi] = int(v)
            nodeA["sub_id"][vi] = si

            # in-edges
            for u in G.predecessors(v):
                k = slot_of[(vi, u)]
                slotA["is_edge"][k] = 1
                ed = G[u][v]
                slotA["act"][k] = int(ed.get("activated", 1))
                if "mixture_weight" in ed:
                    slotA["edge_mw"][k] = _f(ed["mixture_weight"])
                # sender's TSE entry keyed by this receiver (read by message passing)
                tse_u = G.nodes[u].get("track_state_estimates")
                if tse_u is not None and v in tse_u and "mixture_weight" in tse_u[v]:
                    slotA["send_mw"][k] = _f(tse_u[v]["mixture_weight"])
            for ui_key in [r[1] for r in slot_rows[vi]]:
                if ui_key in lm:
                    k = slot_of[(vi, ui_key)]
                    slotA["rev_edge"][k] = 1 if G.has_edge(v, ui_key) else 0

            d = attr.get("track_state_estimates")
            if d is not None:
                nodeA["has_tse"][vi] = 1
                for rank, (u, st) in enumerate(d.items()):
                    k = slot_of[(vi, u)]
                    slotA["tse_rank"][k] = rank
                    _fill_state(slotA, "tse", k, st)
                    if "theta" in st:
                        slotA["tse_theta"][k] = (_f(st["theta"]), _f(st["theta2"]), _f(st["variance_theta"]))
                    if "var_ms_node" in st:
                        slotA["tse_var_ms"][k] = _f(st["var_ms_node"])
            d = attr.get("updated_track_states")
            if d is not None:
                nodeA["has_uts"][vi] = 1
                for rank, (u, st) in enumerate(d.items()):
                    k = slot_of[(vi, u)]
                    slotA["uts_rank"][k] = rank
                    _fill_state(slotA, "uts", k, st)
                    if "likelihood" in st:
                        slotA["uts_lik"][k] = _f(st["likelihood"])
                    if "lr_layer_norm" in st:
                        slotA["uts_lr"][k] = _f(st["lr_layer_norm"])
                    if "side" in st:
                        slotA["uts_side"][k] = 0 if st["side"] == "left" else 1

            # out-edges in successor order
            for w in G.successors(v):
                out_slot.append(slot_of[(lm[w], v)])
            out_ptr[vi + 1] = out_ptr[vi] + G.out_degree(v)
            gi += 1

    g = TrackGraph(N, S, slot_ptr.astype(np.int32), out_ptr.astype(np.int32),
                   np.asarray(out_slot, dtype=np.int32), nodeA, slotA, len(subgraphs))
    check_layout(g)
    return g


def _fill_state(slotA, pfx, k, st):
    if "edge_state_vector" in st:
        slotA[pfx + "_sv"][k] = np.asarray(st["edge_state_vector"], dtype=F64)[:3]
    if "joint_vector" in st:
        slotA[pfx + "_tau"][k] = _f(st["joint_vector"][2])
    cov = st.get("joint_vector_covariance", st.get("edge_covariance"))
    if cov is not None:
        slotA[pfx + "_cov"][k] = cov5_from_mat(cov)
    if "xyzr" in st:
        slotA[pfx + "_xyzr"][k] = [_f(c) for c in st["xyzr"]]
    if "prior" in st:
        slotA[pfx + "_prior"][k] = _f(st["prior"])
    if "mixture_weight" in st:
        slotA[pfx + "_mw"][k] = _f(st["mixture_weight"])


# --------------------------------------------------------------------------
# unpack: write TrackGraph results back into the reference graphs
# --------------------------------------------------------------------------
def unpack(g: TrackGraph, subgraphs, *, states=("tse", "uts"), merged=True,
           degree=True, edges=True) -> None:
    """Write packed results back into ``subgraphs`` (the objects given to pack).

    Mirrors the reference's in-place mutations: activation and edge mixture
    weight per directed edge, node ``degree``, ``merged_state/cov/prior``,
    and the state dicts rebuilt in rank (dict) order. A freshly created UTS
    entry gets the key order of extrapolate_merged_states.py:375-385 and
    ``edge_covariance is joint_vector_covariance`` (aliasing, :362-365).
    """
    sp = g.slot_ptr
    gi = 0
    for si, G in enumerate(subgraphs):
        for v in G.nodes:
            vi = gi
            gi += 1
            attr = G.nodes[v]
            lo, hi = int(sp[vi]), int(sp[vi + 1])
            if edges:
                for k in range(lo, hi):
                    if g.slot["is_edge"][k]:
                        u = _key(G, g.slot["slot_key"][k])
                        ed = G[u][v]
                        ed["activated"] = int(g.slot["act"][k])
                        mw = g.slot["edge_mw"][k]
                        if not np.isnan(mw):
                            ed["mixture_weight"] = mw
            if degree and g.node["degree"][vi] >= 0:
                attr["degree"] = int(g.node["degree"][vi])
            if merged and g.node["has_merged"][vi]:
                ms, mc = g.node["merged_state"][vi], mat_from_cov5(g.node["merged_cov"][vi])
                old_ms, old_mc = attr.get("merged_state"), attr.get("merged_cov")
                # message passing mutates the stored arrays in place (extrapolate_merged_states.py:128);
                # keep the objects, so aliases held elsewhere see the same values
                if isinstance(old_ms, np.ndarray) and old_ms.shape == (3,) and old_ms.dtype == F64:
                    old_ms[...] = ms
                else:
                    attr["merged_state"] = ms.copy()
                if isinstance(old_mc, np.ndarray) and old_mc.shape == (3, 3) and old_mc.dtype == F64:
                    old_mc[...] = mc
                else:
                    attr["merged_cov"] = mc
                attr["merged_prior"] = g.node["merged_prior"][vi]
            if "tse" in states and g.node["has_tse"][vi]:
                _write_dict(g, "tse", attr, "track_state_estimates", lo, hi, G)
            if "uts" in states and g.node["has_uts"][vi]:
                _write_dict(g, "uts", attr, "updated_track_states", lo, hi, G)


def _key(G, key):
    # node ids may be python ints or numpy ints; compare by value
    return key if key in G else int(key)


def _write_dict(g, pfx, attr, dname, lo, hi, G):
    S = g.slot
    old = attr.get(dname) or {}
    ranked = sorted((int(S[pfx + "_rank"][k]), k) for k in range(lo, hi) if S[pfx + "_rank"][k] >= 0)
    new = {}
    for _, k in ranked:
        key = int(S["slot_key"][k])
        okey = next((ok for ok in old.keys() if ok == key), key)
        st = old.get(okey)
        fresh = pfx == "uts" and (st is None or bool(S["uts_fresh"][k]))
        if st is None or fresh:
            st = _fresh_uts(g, k) if pfx == "uts" else {}
        else:
            _update_state(g, pfx, k, st)
        new[okey] = st
    attr[dname] = new


def _fresh_uts(g, k) -> dict:
    S = g.slot
    xyzr = tuple(S["uts_xyzr"][k])
    sv = S["uts_sv"][k].copy()
    cov = mat_from_cov5(S["uts_cov"][k])
    st = {
        "xy": (xyzr[0], xyzr[1]),
        "zr": (xyzr[2], xyzr[3]),
        "xyzr": xyzr,
        "edge_state_vector": sv,
        "edge_covariance": cov,
        "joint_vector": [sv[0], sv[1], S["uts_tau"][k]],
        "joint_vector_covariance": cov,
        "likelihood": S["uts_lik"][k],
        "mixture_weight": S["uts_mw"][k],
    }
    _update_state(g, "uts", k, st)
    return st


def _update_state(g, pfx, k, st):
    S = g.slot
    if not np.isnan(S[pfx + "_prior"][k]):
        st["prior"] = S[pfx + "_prior"][k]
    if not np.isnan(S[pfx + "_mw"][k]):
        st["mixture_weight"] = S[pfx + "_mw"][k]
    if pfx == "uts":
        if S["uts_side"][k] >= 0:
            st["side"] = "left" if S["uts_side"][k] == 0 else "right"
        if not np.isnan(S["uts_lr"][k]):
            st["lr_layer_norm"] = int(S["uts_lr"][k])


def concat(graphs: List[TrackGraph]) -> TrackGraph:
    """Fuse several TrackGraphs (events) into one CSR with node-index offsets."""
    node = {k: np.concatenate([g.node[k] for g in graphs]) for k in NODE_FIELDS}
    slot = {k: np.concatenate([g.slot[k] for g in graphs]) for k in SLOT_FIELDS}
    noff = np.cumsum([0] + [g.n_nodes for g in graphs])
    soff = np.cumsum([0] + [g.n_slots for g in graphs])
    eoff = np.cumsum([0] + [g.n_edges for g in graphs])
    sub_off = np.cumsum([0] + [g.n_subgraphs for g in graphs])
    slot_ptr = np.concatenate([[0]] + [g.slot_ptr[1:] + soff[i] for i, g in enumerate(graphs)])
    out_ptr = np.concatenate([[0]] + [g.out_ptr[1:] + eoff[i] for i, g in enumerate(graphs)])
    out_slot = np.concatenate([g.out_slot + soff[i] for i, g in enumerate(graphs)])
    src = []
    for i, g in enumerate(graphs):
        s = g.slot["slot_src"].astype(np.int64)
        src.append(np.where(s >= 0, s + noff[i], -1))
    slot["slot_src"] = np.concatenate(src).astype(np.int32)
    node["sub_id"] = np.concatenate([g.node["sub_id"] + sub_off[i] for i, g in enumerate(graphs)]).astype(np.int32)
    out = TrackGraph(int(noff[-1]), int(soff[-1]), slot_ptr.astype(np.int32), out_ptr.astype(np.int32),
                     out_slot.astype(np.int32), node, slot, int(sub_off[-1]))
    check_layout(out)
    return out


# --------------------------------------------------------------------------
# subset: the graph a stage saves after removing nodes (extraction)
# --------------------------------------------------------------------------
def subset(g: TrackGraph, keep) -> TrackGraph:
    """The packed form of the reference's ``subGraph.remove_nodes_from(extracted)``
    (extract_track_candidates.py:459-467) followed by dropping the fragment
    subgraphs: nodes with ``keep`` set survive, in order. Equal to ``pack()`` of the
    reduced networkx graphs, array for array:

    * a kept receiver keeps a slot per remaining dict key: senders still in the
      graph first (by node index), then the removed senders whose keys stay in its
      state dicts as orphans (slot_src = -1, no edge), in the key order pack()
      discovers them -- track_state_estimates order, then updated_track_states;
    * slots whose key was neither an edge nor a dict entry disappear;
    * successor order of the out view is kept; ``sub_id`` is renumbered densely
      (the saved subgraphs are numbered 0..k-1).
    """
    keep = np.asarray(keep, dtype=bool)
    N, S = g.n_nodes, g.n_slots
    if keep.shape != (N,):
        raise ValueError("keep must be a bool mask over the %d nodes" % N)
    new_idx = np.full(N, -1, np.int64)
    new_idx[keep] = np.arange(int(keep.sum()))
    dst = g.slot_dst().astype(np.int64)
    src = g.slot["slot_src"].astype(np.int64)
    kr = keep[dst] if S else np.zeros(0, bool)
    inside = kr & (src >= 0) & keep[np.maximum(src, 0)]
    edge = inside & g.slot["is_edge"].astype(bool)
    tr, ur = g.slot["tse_rank"].astype(np.int64), g.slot["uts_rank"].astype(np.int64)
    orphan = kr & ~inside & ((tr >= 0) | (ur >= 0))
    ks = np.nonzero(edge | (inside & ((tr >= 0) | (ur >= 0))) | orphan)[0]
    big = np.int64(1) << 40
    minor = np.where(inside[ks], new_idx[np.maximum(src[ks], 0)],
                     big + np.where(tr[ks] >= 0, tr[ks], big + ur[ks]))
    ks = ks[np.lexsort((minor, new_idx[dst[ks]]))]
    n2 = int(keep.sum())
    s2 = ks.size
    slot_ptr = np.zeros(n2 + 1, np.int64)
    np.add.at(slot_ptr, new_idx[dst[ks]] + 1, 1)
    slot_ptr = np.cumsum(slot_ptr)
    slot = {k: v[ks].copy() for k, v in g.slot.items()}
    orph = ~inside[ks]
    slot["slot_src"] = np.where(orph, -1, new_idx[np.maximum(src[ks], 0)]).astype(np.int32)
    for name in ("is_edge", "rev_edge", "act"):
        slot[name][orph] = 0
    slot["is_edge"][~orph] = g.slot["is_edge"][ks][~orph]
    for name in ("edge_mw", "send_mw"):
        slot[name][orph] = NAN
    slot["uts_fresh"][:] = 0
    # out view: successors still in the graph, order kept
    old2new = np.full(S, -1, np.int64)
    old2new[ks] = np.arange(s2)
    osl = g.out_slot.astype(np.int64)
    owner = np.repeat(np.arange(N, dtype=np.int64), np.diff(g.out_ptr.astype(np.int64)))
    ok = keep[owner] & (old2new[osl] >= 0) if osl.size else np.zeros(0, bool)
    ok &= edge[osl] if osl.size else ok
    out_slot = old2new[osl[ok]].astype(np.int32)
    out_ptr = np.zeros(n2 + 1, np.int64)
    np.add.at(out_ptr, new_idx[owner[ok]] + 1, 1)
    out_ptr = np.cumsum(out_ptr)
    node = {k: v[keep].copy() for k, v in g.node.items()}
    if n2:
        _, node["sub_id"] = np.unique(node["sub_id"], return_inverse=True)
        node["sub_id"] = node["sub_id"].astype(np.int32)
    out = TrackGraph(n2, s2, slot_ptr.astype(np.int32), out_ptr.astype(np.int32), out_slot, node, slot,
                     int(node["sub_id"].max()) + 1 if n2 else 0)
    check_layout(out)
    return out


def refresh_send_mw(g: TrackGraph) -> TrackGraph:
    """send_mw[k] of the edge u -> v = u's track_state_estimates[v]['mixture_weight'],
    read from the slot (receiver u, key v) -- after a device stage rewrote tse_mw
    (compute_mixture_weights, helper.py:76-96). Absent entry -> NaN (as pack())."""
    S = g.n_slots
    dst = g.slot_dst().astype(np.int64)
    src = g.slot["slot_src"].astype(np.int64)
    N = max(g.n_nodes, 1)
    ins = np.nonzero(src >= 0)[0]
    code = dst[ins] * N + src[ins]                 # slot (receiver, sender)
    order = np.argsort(code, kind="stable")
    sc = code[order]
    e = np.nonzero(g.slot["is_edge"].astype(bool))[0]
    want = src[e] * N + dst[e]                     # reverse slot (receiver u, sender v)
    pos = np.searchsorted(sc, want)
    pos_c = np.minimum(pos, max(sc.size - 1, 0))
    hit = (pos < sc.size) & (sc[pos_c] == want) if sc.size else np.zeros(e.size, bool)
    mw = np.full(S, NAN)
    rk = ins[order[pos_c[hit]]]
    vals = np.where(g.slot["tse_rank"][rk] >= 0, g.slot["tse_mw"][rk], NAN)
    mw[e[hit]] = vals
    g.slot["send_mw"] = mw
    return g
