"""Golden fixture for the np.where tie semantics of clustering, made by
the REFERENCE's own clustering.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_tie.py        # writes tests/golden/cluster_tie.npz

Ties in the pairwise chi2 matrix come from neighbours with identical coordinates
(double-sided strip modules): 17 nodes of the 800' and 28 of the 134 all-volume graphs,
where some of them empty the state list and crash the reference's stage (clustering.py
:116). The configured volume-7 run has none. This script makes ties that do NOT empty
the list, on the volume-7 network of make_golden.py:

  * for a node v whose smallest nonzero pairwise chi2 (clustering.py:114-124) involves
    in-neighbour u, and whose dict keeps >= 3 other states, a clone hit u' with u's
    coordinates (a fresh node id) joined to v in both directions (construct_graph adds
    both, helper.py:513-518) is added BEFORE the reference's own
    compute_track_state_estimates / activation / priors / weights / degree
    (event_conversion.py:84-101), so u' carries at v the same state as u:
    chi2(u, X) == chi2(u', X) for every X, and v's minimum is a tie;
  * the reference's clustering on track_state_estimates (-c 1.0 -k 2.0,
    run_gnn_trackml_mod.sh:89) runs on the result, with get_smallest_dist_idx wrapped to
    record every call that returns more than two indices (the tie) and its node.

The fixture holds the packed input and output (pick/save of make_golden.py) and the
tied nodes; tests/test_oracle_golden.py and tests/test_gpu_parity.py compare the
oracle and the HIP path with it.
"""
import copy
import inspect
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as M  # noqa: E402  (shims, reference imports, pack/save helpers)
import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

h, ref_cluster = M.h, M.ref_cluster
P = M.P
CHI2, KL = 1.0, 2.0


def _graph():
    nodes, edges = h.load_nodes_edges(M.EV134, 7, 7)
    truth = pd.read_csv(M.TRUTH134)
    G = nx.DiGraph()
    G = h.construct_graph(G, nodes, edges, truth)
    return nx.DiGraph(G)


def _states(G):
    subs = [G.subgraph(c).copy() for c in nx.weakly_connected_components(G)]
    subs = h.compute_track_state_estimates(subs, P["sigma0xy"], P["sigma0rz"], P["sigma0rz2"], P["endcap_boundary"])
    h.initialize_edge_activation(subs)
    h.compute_prior_probabilities(subs, "track_state_estimates")
    h.compute_mixture_weights(subs, "track_state_estimates")
    for s in subs:
        for n, _ in s.nodes(data=True):
            s.nodes[n]["degree"] = h.query_node_degree_in_edges(s, n)
    return subs


def _min_pair(s, v):
    """the reference's pairwise chi2 of v's dict and its smallest nonzero entry's keys"""
    attr = s.nodes[v]
    tse = attr["track_state_estimates"]
    keys = list(tse.keys())
    n = len(keys)
    D = np.zeros((n, n))
    for i in range(n):
        for j in range(i):
            a, b = tse[keys[i]], tse[keys[j]]
            D[i][j] = ref_cluster.mahalanobis_distance(np.array(a["joint_vector"]), a["joint_vector_covariance"],
                                                       np.array(b["joint_vector"]), b["joint_vector_covariance"],
                                                       attr["xyzr"], s.nodes[keys[i]]["xyzr"],
                                                       s.nodes[keys[j]]["xyzr"], P["sigma0rz"], P["sigma0rz2"],
                                                       P["endcap_boundary"])
    if not np.any(D):
        return None
    nz = D[np.nonzero(D)]
    r, c = np.where(D == nz.min())
    return keys[r[0]], keys[c[0]]


def main():
    G = _graph()
    with M._Quiet():
        base = _states(G.copy())
    # candidate receivers: 5..13 keys (room for one clone, >= 3 states left after the
    # tie removes u, u' and X), every key an in-neighbour inside the subgraph
    picks = []
    for s in base:
        for v in s.nodes:
            tse = s.nodes[v]["track_state_estimates"]
            if 5 <= len(tse) <= 13:
                mp = _min_pair(s, v)
                if mp is not None:
                    picks.append((v, mp[0]))
    rng = np.random.default_rng(11)
    rng.shuffle(picks)
    used = set()
    chosen = []
    for v, u in picks:          # receivers far apart: one clone per neighbourhood
        if v in used or u in used or any(w in used for w in G.neighbors(v)):
            continue
        chosen.append((v, u))
        used.update([v, u])
        used.update(G.neighbors(v))
        if len(chosen) == 40:
            break
    next_id = max(G.nodes) + 1
    for v, u in chosen:
        a = dict(G.nodes[u])
        gm = a["GNN_Measurement"]
        a["GNN_Measurement"] = copy.copy(gm)
        a["GNN_Measurement"].node = next_id
        a["tags"] = [next_id]
        G.add_node(next_id, **a)
        G.add_edge(next_id, v)
        G.add_edge(v, next_id)
        next_id += 1
    with M._Quiet():
        net = _states(G)
    # the configured subgraph set of make_golden.py would drop most receivers: keep every
    # subgraph holding a clone, plus the first ~2000 nodes of the rest
    clones = set(range(max(G.nodes) - len(chosen) + 1, max(G.nodes) + 1))
    keep, tot = [], 0
    for s in net:
        if any(n in clones for n in s.nodes):
            keep.append(s)
        elif tot < 2000:
            keep.append(s)
            tot += len(s)
    ties = []
    orig = ref_cluster.get_smallest_dist_idx

    def rec(distances):
        sm, idx = orig(distances)
        if not isinstance(distances, list) and np.size(idx) > 2:
            fr = inspect.currentframe().f_back
            ties.append((int(fr.f_locals["node_num"]), int(np.size(idx))))
        return sm, idx
    ref_cluster.get_smallest_dist_idx = rec
    out = M.run_cluster(keep, "track_state_estimates", CHI2, KL)
    ref_cluster.get_smallest_dist_idx = orig
    gin, gout = M.pack(keep), M.pack(out)
    tie_nodes = np.array(sorted(set(t[0] for t in ties)), np.int64)
    print("clones %d, tied receivers %d, index counts %s" % (len(chosen), tie_nodes.size,
                                                           sorted(set(t[1] for t in ties))))
    assert tie_nodes.size >= 10
    M.save("cluster_tie", gin, gout, extra={"tie_nodes": tie_nodes},
           meta=dict(key="track_state_estimates", chi2=CHI2, kl=KL, **P))


if __name__ == "__main__":
    main()
