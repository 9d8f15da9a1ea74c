"""Golden fixtures on real multi-volume data: the committed 800' all-volume event
(learn_KL_parabolic_model/.../minCurv_0.3_800, SURVEY §8a "C2": 29,590 nodes / 89,028
directed edges, volumes 7-14), made by the REFERENCE's own functions.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_800.py     # writes tests/golden/c2_800_*.npz

The reference crashes its clustering stage on this event: where neighbours share
identical coordinates (double-sided strip modules) a distance tie can remove every state
and ``np.min([])`` raises ValueError (clustering.py:114-124). A stage
processes all subgraphs in one loop, so one raising subgraph loses the stage's whole
output. Here every stage runs subgraph by subgraph, the ValueError is caught per
subgraph, and the subgraphs that raise are recorded; every other subgraph's outputs are
pinned.

* network: event_conversion.py:53-101 with the committed truth mapping (make_golden.py's
  recipe on this event, volumes 7..14);
* c2_800_cluster_tse.npz -- iteration 1 of run_gnn_trackml_mod.sh: clustering on
  track_state_estimates with -c 1.0 -k 2.0 (:89);
* c2_800_pass.npz -- the benchmarked pass chain on the full load (every node's merged
  state = its first TSE entry): extrapolation (extrapolate_merged_states.py
  :552-566, -c 2.0), update (remove_state_metadata.py), clustering on
  updated_track_states (-c 1000 -k 100, run_gnn_trackml_mod.sh:112).

Stored in the packed node / slot order of gtf.graph.pack (= gtf_build_event_csr's order;
a structure digest pins it): masks and flags exactly, merged states of merged nodes (every 2nd one on the full load), the
updated states' dict order, and the updated-state floats of every 4th present slot
(fixture size). raised[sub] = 1 where the reference raised in that subgraph (its outputs
are then not pinned), tie_nodes = the receivers whose get_smallest_dist_idx returned a
tie. Inputs are NOT stored: the test rebuilds them from tests/golden/kat800 (the same
committed CSVs) with the GPU's event conversion and initial states.
"""
import copy
import hashlib
import inspect
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as M  # noqa: E402  (shims, reference imports, pack helpers)
import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

h, ref_cluster = M.h, M.ref_cluster
P = M.P
REF800 = os.path.join(M.REF, "learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/minCurv_0.3_800")
EV800 = os.path.join(REF800, "event_network/event_1_filtered_graph_")
TRUTH800 = os.path.join(REF800, "event_truth/event000001000-full-mapping-minCurv-0.3-800.csv")
VOLS = (7, 14)


def structure_digest(g):
    """SHA-256 of the packed structure (node ids, slot segments, senders, successor order)"""
    hh = hashlib.sha256()
    for a in (g.node["node_id"].astype(np.int64), g.slot_ptr.astype(np.int64), g.slot["slot_src"].astype(np.int64),
              g.out_ptr.astype(np.int64), g.out_slot.astype(np.int64), g.slot["tse_rank"].astype(np.int64)):
        hh.update(np.ascontiguousarray(a).tobytes())
    return hh.hexdigest()


def build_network():
    nodes, edges = h.load_nodes_edges(EV800, *VOLS)
    truth = pd.read_csv(TRUTH800)
    G = nx.DiGraph()
    G = h.construct_graph(G, nodes, edges, truth)
    G = nx.DiGraph(G)
    subs = [G.subgraph(c).copy() for c in nx.weakly_connected_components(G)]
    subs = h.compute_track_state_estimates(subs, P["sigma0xy"], P["sigma0rz"], P["sigma0rz2"], P["endcap_boundary"])
    h.initialize_edge_activation(subs)
    h.compute_prior_probabilities(subs, "track_state_estimates")
    h.compute_mixture_weights(subs, "track_state_estimates")
    for s in subs:
        for n, _ in s.nodes(data=True):
            s.nodes[n]["degree"] = h.query_node_degree_in_edges(s, n)
    return subs


class TieRecorder:
    """wraps the reference's get_smallest_dist_idx: receivers whose matrix minimum is a tie"""

    def __init__(self):
        self.nodes = set()
        self.orig = ref_cluster.get_smallest_dist_idx

    def __enter__(self):
        def rec(distances):
            sm, idx = self.orig(distances)
            if not isinstance(distances, list) and np.size(idx) > 2:
                self.nodes.add(int(inspect.currentframe().f_back.f_locals["node_num"]))
            return sm, idx
        ref_cluster.get_smallest_dist_idx = rec
        return self

    def __exit__(self, *a):
        ref_cluster.get_smallest_dist_idx = self.orig


def run_cluster(subs, key, chi2, kl):
    """make_golden.run_cluster for ONE subgraph. The reference's confusion-matrix printout
    after the subgraph loop (clustering.py:342-369) divides by zero when the stage's totals
    are zero -- in a whole-event run they never are, subgraph by subgraph they can be --
    and it runs before the stage's last two calls (:372-373). On that ZeroDivisionError the
    stage's own subgraph list is taken from the raising frame and those two calls
    (compute_mixture_weights, compute_prior_probabilities on the stage key) are made here:
    the outputs the stage would have saved. A ValueError (the tie, :114-124) propagates."""
    import glob
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        ind, outd = os.path.join(d, "in") + "/", os.path.join(d, "out") + "/"
        os.makedirs(ind), os.makedirs(outd)
        for i, s in enumerate(subs):
            h.save_network(ind, i, s)
        try:
            with M._Quiet():
                ref_cluster.cluster(ind, outd, key, chi2, kl, None, 1, False, P["sigma0rz"], P["sigma0rz2"],
                                    P["endcap_boundary"])
            out = [M._read_gpickle(f) for f in glob.glob(outd + "*_subgraph.gpickle")]
        except ZeroDivisionError as e:
            tb, fr = e.__traceback__, None
            while tb is not None:
                if tb.tb_frame.f_code is ref_cluster.cluster.__code__:
                    fr = tb.tb_frame
                tb = tb.tb_next
            assert fr is not None and fr.f_lineno >= 342, "ZeroDivisionError outside the diagnostics"
            out = fr.f_locals["subGraphs"]
            with M._Quiet():
                h.compute_mixture_weights(out, key)
                h.compute_prior_probabilities(out, key)
    return M._canon(subs, out)


def per_subgraph(subs, stage):
    """stage([s]) -> [s'] for every subgraph on its own; (outputs, raised) with the input
    subgraph kept where the reference raised ValueError (not pinned)"""
    outs, raised = [], np.zeros(len(subs), np.uint8)
    for i, s in enumerate(subs):
        try:
            outs.append(stage([s])[0])
        except ValueError:
            raised[i] = 1
            outs.append(s)
    return outs, raised


def node_sub(g):
    return g.node["sub_id"].astype(np.int64)


def save(name, g_in, g_out, raised, ties, uts):
    mm = g_out.node["has_merged"].astype(bool)
    arrs = {
        "structure_sha": np.array(structure_digest(g_in)),
        "n_nodes": np.array(g_in.n_nodes), "n_slots": np.array(g_in.n_slots),
        "raised": raised, "tie_nodes": np.array(sorted(ties), np.int64),
        "act_bits": np.packbits(g_out.slot["act"].astype(np.uint8)),
        "has_merged_bits": np.packbits(mm.astype(np.uint8)),
        "degree": g_out.node["degree"].astype(np.int16),
    }
    # merged floats of every merged node, or of every 2nd one when all of them are (the full
    # load: every node starts with a merged state; fixture size)
    sn = np.nonzero(mm)[0]
    sn = sn[::2] if sn.size > 10000 else sn
    arrs.update({"sample_node": sn.astype(np.int32), "merged_state": g_out.node["merged_state"][sn],
                 "merged_cov": g_out.node["merged_cov"][sn], "merged_prior": g_out.node["merged_prior"][sn]})
    if uts:
        from compare import dense_ranks
        arrs["has_uts_bits"] = np.packbits(g_out.node["has_uts"].astype(np.uint8))
        arrs["uts_dense_rank"] = dense_ranks(g_out, "uts_rank").astype(np.int8)
        pres = np.nonzero(g_out.slot["uts_rank"] >= 0)[0]
        smp = pres[::4]
        arrs["sample_slot"] = smp.astype(np.int32)
        for f in ("uts_sv", "uts_cov", "uts_tau", "uts_lik", "uts_mw", "uts_prior", "edge_mw"):
            arrs["slot__" + f] = g_out.slot[f][smp]
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print("wrote %s %.1f KB: %d subgraphs, %d raised, %d tie receivers, %d merged" % (
        name, os.path.getsize(path) / 1024, raised.size, int(raised.sum()), len(ties), int(mm.sum())))


def main():
    sys.path.insert(0, os.path.dirname(HERE))     # tests/ (compare.dense_ranks)
    t0 = time.time()
    with M._Quiet():
        net = build_network()
    print("800' network: %d subgraphs, %d nodes, %d edges (%.0f s)" % (
        len(net), sum(len(s) for s in net), sum(s.number_of_edges() for s in net), time.time() - t0))
    g0 = M.pack(net)
    assert g0.n_nodes == 29590 and g0.n_edges == 89028, (g0.n_nodes, g0.n_edges)

    # iteration 1: clustering on track_state_estimates, -c 1.0 -k 2.0
    with TieRecorder() as tr:
        c1, raised1 = per_subgraph(net, lambda s: run_cluster(s, "track_state_estimates", 1.0, 2.0))
    save("c2_800_cluster_tse", g0, M.pack(c1, like=g0), raised1, tr.nodes, uts=False)
    print("  (%.0f s)" % (time.time() - t0))

    # the pass chain on the full load: extrapolate -> update -> cluster UTS (-c 1000 -k 100)
    fl = M.full_load(net)

    def chain(s):
        x = M.run_extrapolate(s)
        u = M.run_update(x)
        return run_cluster(u, "updated_track_states", 1000.0, 100.0)
    with TieRecorder() as tr:
        c2, raised2 = per_subgraph(fl, chain)
    gfl = M.pack(fl)
    assert structure_digest(gfl) == structure_digest(g0)
    save("c2_800_pass", gfl, M.pack(c2, like=gfl), raised2, tr.nodes, uts=True)
    print("done in %.0f s" % (time.time() - t0))


if __name__ == "__main__":
    main()
