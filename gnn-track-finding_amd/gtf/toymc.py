"""Config C1 (BASELINE configs[0]): the reference's toy Monte Carlo event, in 3-D.

The reference's toy (src/toyMC_model/track_simulation_xy.py:36-188) draws 88 straight
tracks from the origin (11 end points x 8 octant reflections, :43-54), 10 hits each
at x = linspace(0, x_end, 10) with y = slope * x + N(0, 0.05) (:71-85), proposes hit
pairs between hits 1 or 2 layers apart that lie within 3 of each other and whose line
has |y-intercept| <= 1.8 and |x-intercept| <= 1.8 (:102-121), removes the hits at the
origin (:130-131) and every hit of a pair with |dx| > 0.75 (:148-152), makes the graph
directed and splits it into weakly connected subgraphs (:159, :175).

Its hits have z = r = 0, and the track-finding pass divides by dr, so SURVEY §8d
defines C1 with one addition: per track a polar angle, z = cot(theta) * r with
r = sqrt(x^2 + y^2) (cot theta = sinh(eta), eta uniform in [-1, 1], drawn from a
separate seeded stream so the x-y event is the reference's own for the same seed:
its smearing draws come from np.random.seed(seed)'s legacy stream in the reference's
order, pinned by tests/golden/make_golden_toymc.py).

``subgraphs(seed)`` returns the reference-schema networkx subgraphs (the node
attributes of helper.construct_graph, helper.py:465-521, which the stage CLIs read);
``event(seed)`` the packed TrackGraph. Both carry no state estimates yet: the pass
needs the initial track-state estimates (a2) and a full-load merged state
(``full_load``), as for the other configs.
"""
from __future__ import annotations

import numpy as np

from .graph import TrackGraph, pack

ANGLES = (0.5, 1, 2, 3, 4, 5, 6, 7, 8, 9, 9.5)   # :43
RADIUS = 10.0                                     # :40
NUM_HITS = 10                                     # :39
SIGMA0 = 0.05                                     # :65
VOLUME_ID = 0                                     # the toy has no detector volumes


def end_points() -> np.ndarray:
    """[88, 2] track end points in the reference's order (:44-56)."""
    c = []
    for i in ANGLES:
        y = np.sqrt(RADIUS**2 - i**2)
        c += [i, y, y, i, -i, -y, -y, -i, i, -y, -y, i, -i, y, y, -i]
    return np.array(c, dtype=np.float64).reshape(-1, 2)


def hits(seed: int = 0):
    """x, y, layer, track of every hit, node id = position (:68-94): the smearing is
    drawn track by track, layer by layer, from np.random.seed(seed)'s stream."""
    rs = np.random.RandomState(seed)
    ends = end_points()
    xs, ys = [], []
    for n in range(ends.shape[0]):
        gradient = ends[n, 1] / ends[n, 0]               # start = (0, 0)
        x = np.linspace(0.0, ends[n, 0], NUM_HITS)
        for xi in x:
            nu = SIGMA0 * rs.normal(0.0, 1.0)
            xs.append(xi)
            ys.append(gradient * xi + nu)
    n_tr = ends.shape[0]
    layer = np.tile(np.arange(NUM_HITS), n_tr)
    track = np.repeat(np.arange(n_tr), NUM_HITS)
    return np.array(xs), np.array(ys), layer, track


def hit_pairs(x, y, layer):
    """The reference's pair rule over every ordered node pair in node order (:102-121),
    vectorised. Returns (node1, node2, dx) in the loop's order."""
    n = x.size
    a, b = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    a, b = a.ravel(), b.ravel()
    diff = np.abs(layer[b] - layer[a])
    keep = (diff > 0) & (diff <= 2) & (a != b)
    a, b = a[keep], b[keep]
    dx = x[b] - x[a]
    dy = y[b] - y[a]
    near = np.sqrt(dx**2 + dy**2) <= 3
    a, b, dx, dy = a[near], b[near], dx[near], dy[near]
    with np.errstate(divide="ignore", invalid="ignore"):
        m = dy / dx
        c = y[b] - (m * x[b])
        x_int = -1 * c / m
        ok = (np.abs(c) <= 1.8) & (np.abs(x_int) <= 1.8)
    return a[ok], b[ok], dx[ok]


def cot_theta(seed: int, n_tracks: int) -> np.ndarray:
    eta = np.random.default_rng([seed, 1]).uniform(-1.0, 1.0, n_tracks)
    return np.sinh(eta)


def subgraphs(seed: int = 0):
    """The toy event as the reference builds it (:59-175), with z added, as a list of
    nx.DiGraph in the construct_graph node schema."""
    import networkx as nx
    from GNN_Measurement.GNN_Measurement import GNN_Measurement
    x, y, layer, track = hits(seed)
    n_tr = int(track.max()) + 1
    r = np.sqrt(x**2 + y**2)
    z = cot_theta(seed, n_tr)[track] * r
    G = nx.Graph()
    for i in range(x.size):
        xi, yi, zi, ri = float(x[i]), float(y[i]), float(z[i]), float(r[i])
        lay = int(layer[i])
        G.add_node(i, GNN_Measurement=GNN_Measurement(xi, yi, zi, ri, truth_particle=int(track[i]), n=i),
                   xy=(xi, yi), zr=(zi, ri), xyzr=(xi, yi, zi, ri), volume_id=VOLUME_ID,
                   in_volume_layer_id=lay, vivl_id=(VOLUME_ID, lay), truth_particle=int(track[i]), tags=[i])
    a, b, dx = hit_pairs(x, y, layer)
    for u, v, d in zip(a.tolist(), b.tolist(), dx.tolist()):
        G.add_edge(u, v, dx=d)                                                   # :121
    for i in range(n_tr):                                                        # :130-131
        G.remove_node(i * NUM_HITS)
    copyG = G.copy()                                                             # :148-152
    for u, v, data in copyG.edges(data=True):
        if np.abs(data["dx"]) > 0.75:
            if u in G:
                G.remove_node(u)
            if v in G:
                G.remove_node(v)
    G = nx.to_directed(G)                                                        # :159
    for _, _, data in G.edges(data=True):
        data.pop("dx", None)
    return [G.subgraph(c).copy() for c in nx.weakly_connected_components(G)]   # :175


def event(seed: int = 0) -> TrackGraph:
    """C1 packed (node order = subgraph order, then node order inside each), with the
    track_state_estimates keys of a fresh network in the reference's dict order,
    reversed(set(nx.all_neighbors)) (helper.py:277, :350-351, this interpreter's own
    set as in gtf.stages.compute_track_state_estimates); the entries' values come from
    the TSE kernel (or the oracle in the tests)."""
    import networkx as nx
    sgs = subgraphs(seed)
    for G in sgs:
        for node in G.nodes():
            keys = list(set(nx.all_neighbors(G, node)))
            keys.reverse()
            G.nodes[node]["track_state_estimates"] = {k: {} for k in keys}
    g = pack(sgs)
    g.node["has_tse"][:] = 1       # every node gets a (possibly empty) dict (helper.py:444)
    g.slot["act"][g.slot["is_edge"] == 1] = 1   # initialize_edge_activation (helper.py:24-27)
    return g


def full_load(g: TrackGraph) -> TrackGraph:
    """Every node with a track_state_estimates entry starts the pass with its first
    entry (dict order) as merged state, prior 1 (SURVEY §8d "full load"). In place."""
    r = g.slot["tse_rank"]
    sp = g.slot_ptr.astype(np.int64)
    owner = np.repeat(np.arange(g.n_nodes), np.diff(sp))
    first = np.nonzero(r == 0)[0]
    v = owner[first]
    g.node["has_merged"][v] = 1
    g.node["merged_state"][v] = g.slot["tse_sv"][first]
    g.node["merged_cov"][v] = g.slot["tse_cov"][first]
    g.node["merged_prior"][v] = 1.0
    return g
