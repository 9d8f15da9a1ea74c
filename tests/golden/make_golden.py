"""Generate golden fixtures by running the REFERENCE's own functions.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

What it does (SURVEY.md §8c "Generated fixtures"):

* builds the committed volume-7 event of minCurv_0.3_134 with the reference's
  ``helper.load_nodes_edges`` / ``construct_graph`` (truth = the committed
  full-mapping CSV, because the raw TrackML hits/truth files are absent), splits
  it into weakly connected subgraphs and runs the reference's TSE, activation,
  prior, mixture-weight and degree functions (mirrors
  src/trackml_mod/event_conversion.py:53-101);
* runs, on copies of that network, the reference stages whose outputs the
  fixtures pin: clustering on track_state_estimates (run_gnn_trackml_mod.sh:89
  flags), extrapolation (extrapolate_merged_states.py:552-566, flags of :101),
  remove_state_metadata after a simulated extraction (random node removal ->
  orphan state keys), clustering on updated_track_states (:112 flags), a
  "full-load" extrapolation (every node's merged state = its first TSE entry),
  the fused pass chain and tag propagation (tag_propagation.py run whole);
* packs inputs and reference outputs with ``gtf.graph.pack`` and stores the
  arrays the GPU path and the oracle are compared on.

Shims (this container only): ``shims/filterpy`` restates filterpy 1.4.5;
``nx.read_gpickle/write_gpickle`` (removed in networkx 3) are bound to pickle.
Reference sources are imported from /root/reference and never copied.
"""
import copy
import glob
import os
import pickle
import random
import runpy
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [os.path.join(HERE, "shims"), os.path.join(REF, "src"),
                os.path.join(REPO, "gnn-track-finding_amd")]
os.environ.setdefault("MPLBACKEND", "Agg")
sys.dont_write_bytecode = True

import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402


def _read_gpickle(path):
    with open(path, "rb") as f:
        return pickle.load(f)


def _write_gpickle(G, path):
    with open(path, "wb") as f:
        pickle.dump(G, f, pickle.HIGHEST_PROTOCOL)


nx.read_gpickle = _read_gpickle
nx.write_gpickle = _write_gpickle

from utilities import helper as h  # noqa: E402  (reference)
from clustering import clustering as ref_cluster  # noqa: E402  (reference)
from extrapolate import extrapolate_merged_states as ref_extrap  # noqa: E402  (reference)


def _diagnostics_safe(fn):
    """The reference's confusion-matrix printout divides by zero when no
    outlier was a true outlier (helper.py:216-217, message_passing :509-510,
    with the '=1' counter bug of helper.py:199-200). It runs AFTER every
    mutation of the stage is done, so the stage outputs are complete; the
    exception is swallowed here so the outputs can be recorded."""
    def wrapped(*a, **k):
        try:
            return fn(*a, **k)
        except ZeroDivisionError:
            return None
    return wrapped


h.reweight = _diagnostics_safe(h.reweight)
ref_extrap.message_passing = _diagnostics_safe(ref_extrap.message_passing)
from gtf.graph import pack, NODE_FIELDS, SLOT_FIELDS  # noqa: E402  (ours: container only)

EV134 = os.path.join(REF, "src/trackml_mod/event_network/minCurv_0.3_134/event_1_filtered_graph_")
TRUTH134 = os.path.join(REF, "learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/"
                        "minCurv_0.3_134/event_truth/event000001000-full-mapping-minCurv-0.3-134.csv")
P = dict(sigma0xy=0.3, sigma0rz=0.4, sigma0rz2=0.6, endcap_boundary=550.0, chi2_cut=2.0)


class _Quiet:
    def __enter__(self):
        self._o = sys.stdout
        sys.stdout = open(os.devnull, "w")

    def __exit__(self, *a):
        sys.stdout.close()
        sys.stdout = self._o


def build_network(min_volume=7, max_volume=7):
    """event_conversion.py:53-101 with the committed truth mapping."""
    nodes, edges = h.load_nodes_edges(EV134, min_volume, max_volume)
    truth = pd.read_csv(TRUTH134)
    G = nx.DiGraph()
    G = h.construct_graph(G, nodes, edges, truth)
    G = nx.DiGraph(G)
    subs = [G.subgraph(c).copy() for c in nx.weakly_connected_components(G)]
    subs = h.compute_track_state_estimates(subs, P["sigma0xy"], P["sigma0rz"], P["sigma0rz2"],
                                           P["endcap_boundary"])
    h.initialize_edge_activation(subs)
    h.compute_prior_probabilities(subs, "track_state_estimates")
    h.compute_mixture_weights(subs, "track_state_estimates")
    for s in subs:
        for n, _ in s.nodes(data=True):
            s.nodes[n]["degree"] = h.query_node_degree_in_edges(s, n)
    return subs


def _canon(subs_in, subs_out):
    """reorder stage outputs (glob order) back to input subgraph order"""
    key = {min(s.nodes): i for i, s in enumerate(subs_in) if len(s)}
    out = [None] * len(subs_in)
    for s in subs_out:
        out[key[min(s.nodes)]] = s
    return out


def run_cluster(subs, key, chi2, kl):
    with tempfile.TemporaryDirectory() as d:
        ind, outd = os.path.join(d, "in") + "/", os.path.join(d, "out") + "/"
        os.makedirs(ind), os.makedirs(outd)
        for i, s in enumerate(subs):
            h.save_network(ind, i, s)
        with _Quiet():
            ref_cluster.cluster(ind, outd, key, chi2, kl, None, 1, False, P["sigma0rz"], P["sigma0rz2"],
                                P["endcap_boundary"])
        out = [_read_gpickle(f) for f in glob.glob(outd + "*_subgraph.gpickle")]
    return _canon(subs, out)


def run_extrapolate(subs):
    """extrapolate_merged_states.main body (:552-566) in-process."""
    subs = copy.deepcopy(subs)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)  # the stage appends diagnostic CSVs to the CWD
        try:
            with _Quiet():
                ref_extrap.message_passing(subs, P["chi2_cut"], P["sigma0xy"], P["sigma0rz"], P["sigma0rz2"],
                                           P["endcap_boundary"])
                h.compute_prior_probabilities(subs, "updated_track_states")
                h.reweight(subs, "updated_track_states")
                h.compute_prior_probabilities(subs, "updated_track_states")
                h.reweight(subs, "updated_track_states")
                for s in subs:
                    for n, _ in s.nodes(data=True):
                        s.nodes[n]["degree"] = h.query_node_degree_in_edges(s, n)
        finally:
            os.chdir(cwd)
    return subs


def run_update(subs):
    """src/update/remove_state_metadata.py main() via its CLI entry point."""
    with tempfile.TemporaryDirectory() as d:
        rem = os.path.join(d, "rem") + "/"
        os.makedirs(rem)
        for i, s in enumerate(subs):
            h.save_network(rem, i, s)
        argv = sys.argv
        sys.argv = ["remove_state_metadata.py", "-r", rem]
        try:
            with _Quiet():
                runpy.run_path(os.path.join(REF, "src/update/remove_state_metadata.py"), run_name="__main__")
        finally:
            sys.argv = argv
        out = [_read_gpickle(f) for f in glob.glob(rem + "*_subgraph.gpickle")]
    return _canon(subs, out)


def run_tags(subs):
    """tag_propagation.py executed whole on the composed network; returns
    (node id -> final tag, flips per sweep)."""
    G = nx.DiGraph()
    for s in subs:
        G = nx.compose(G, s)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        _write_gpickle(G, os.path.join(d, "0_subgraph.gpickle"))
        os.chdir(d)
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
            plt.savefig = lambda *a, **k: None          # plots only; skip writing PNGs
            with _Quiet():
                glb = runpy.run_path(os.path.join(REF, "tag_propagation/tag_propagation.py"))
            plt.close("all")
        finally:
            os.chdir(cwd)
    fin = glb["current_endcap_graph"]
    return G, {n: fin.nodes[n]["tags"][-1] for n in fin.nodes}, list(glb["num_tags_flipped"])


def full_load(subs):
    """every node's merged state = a copy of its first TSE entry."""
    subs = copy.deepcopy(subs)
    for s in subs:
        for n in s.nodes:
            tse = s.nodes[n]["track_state_estimates"]
            if tse:
                first = next(iter(tse.values()))
                s.nodes[n]["merged_state"] = np.array(first["edge_state_vector"], dtype=float).copy()
                s.nodes[n]["merged_cov"] = np.array(first["edge_covariance"], dtype=float).copy()
                s.nodes[n]["merged_prior"] = first.get("prior", 1.0)
    return subs


def simulate_extraction(subs, frac=0.08, seed=7):
    """remove a seeded random node subset (as extraction does) -> orphan keys"""
    rng = random.Random(seed)
    subs = copy.deepcopy(subs)
    for s in subs:
        drop = [n for n in s.nodes if rng.random() < frac]
        s.remove_nodes_from(drop)
    return [s for s in subs if len(s)]


def pick(g, fields):
    out = {"slot_ptr": g.slot_ptr, "out_ptr": g.out_ptr, "out_slot": g.out_slot}
    for f in fields:
        if f in NODE_FIELDS:
            out["node__" + f] = g.node[f]
        elif f in SLOT_FIELDS:
            out["slot__" + f] = g.slot[f]
        else:
            raise KeyError(f)
    return out


IN_FIELDS = ["gnn", "xyzr", "layer", "has_merged", "merged_state", "merged_cov", "merged_prior", "has_tse",
             "has_uts", "degree", "tag", "node_id", "sub_id", "slot_src", "slot_key", "is_edge", "rev_edge",
             "act", "edge_mw", "send_mw", "tse_rank", "tse_sv", "tse_tau", "tse_cov", "tse_xyzr",
             "tse_prior", "tse_mw", "uts_rank", "uts_sv", "uts_tau", "uts_cov", "uts_xyzr", "uts_lik",
             "uts_mw", "uts_prior", "uts_lr", "uts_side"]
OUT_FIELDS = ["has_merged", "merged_state", "merged_cov", "merged_prior", "has_uts", "degree", "act",
              "edge_mw", "tse_rank", "tse_prior", "tse_mw", "uts_rank", "uts_sv", "uts_tau", "uts_cov",
              "uts_xyzr", "uts_lik", "uts_mw", "uts_prior", "uts_lr", "uts_side"]


def save(name, gin, gout, extra=None, meta=None):
    arrs = {}
    for k, v in pick(gin, IN_FIELDS).items():
        arrs["in__" + k] = v
    if gout is not None:
        for k, v in pick(gout, OUT_FIELDS).items():
            if k.startswith(("node__", "slot__")):
                arrs["out__" + k] = v
        assert np.array_equal(gin.slot_ptr, gout.slot_ptr) and np.array_equal(gin.out_slot, gout.out_slot), \
            "stage changed the graph structure"
        assert np.array_equal(gin.slot["slot_key"], gout.slot["slot_key"])
    for k, v in (extra or {}).items():
        arrs["x__" + k] = np.asarray(v)
    arrs["meta"] = np.array(repr(meta or {}))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print("wrote %-28s %7.1f KB  N=%d S=%d E=%d" % (name + ".npz", os.path.getsize(path) / 1024,
                                                      gin.n_nodes, gin.n_slots, gin.n_edges))


def main():
    t0 = time.time()
    with _Quiet():
        net0 = build_network()
    print("network built in %.1fs: %d subgraphs, %d nodes, %d edges" % (
        time.time() - t0, len(net0), sum(len(s) for s in net0), sum(s.number_of_edges() for s in net0)))
    # keep fixtures small (< 2 MB): the first ~third of the subgraphs by node count,
    # plus the largest one (it holds the densest neighbourhoods)
    order = sorted(range(len(net0)), key=lambda i: -len(net0[i]))
    keep = set(order[:1])
    tot = 0
    for i in range(len(net0)):
        if tot > 3000:
            break
        keep.add(i)
        tot += len(net0[i])
    net = [net0[i] for i in sorted(keep)]
    g0 = pack(net)
    save("tse_network", g0, None, meta=dict(src="event_conversion (vol 7, minCurv_0.3_134)", **P))

    # iteration 1: clustering on track_state_estimates, -c 1.0 -k 2.0
    it1 = run_cluster(net, "track_state_estimates", 1.0, 2.0)
    save("cluster_tse", g0, pack(it1), meta=dict(key="track_state_estimates", chi2=1.0, kl=2.0, **P))

    # iteration 2: extrapolation of the merged states
    it2 = run_extrapolate(it1)
    save("extrapolate_it2", pack(it1), pack(it2), meta=dict(**P))

    # update after a simulated extraction (orphans + pruning)
    rem = simulate_extraction(it2)
    upd = run_update(rem)
    grem = pack(rem)
    save("update_it2", grem, pack(upd, like=grem), meta=dict(**P))

    # iteration 3: clustering on updated_track_states, -c 1000 -k 100
    # (clustering input = update of the un-thinned it2 network: after random
    #  thinning some nodes keep an empty UTS dict and the reference's
    #  compute_mixture_weights divides by zero, helper.py:90)
    upd2 = run_update(it2)
    it3 = run_cluster(upd2, "updated_track_states", 1000.0, 100.0)
    gupd = pack(upd2)
    save("cluster_uts", gupd, pack(it3, like=gupd), meta=dict(key="updated_track_states", chi2=1000.0, kl=100.0, **P))

    # full-load extrapolation and the benchmarked pass chain (extrapolate -> update -> cluster uts)
    fl = full_load(net)
    fx = run_extrapolate(fl)
    save("extrapolate_full", pack(fl), pack(fx), meta=dict(**P))
    fu = run_update(fx)
    fc = run_cluster(fu, "updated_track_states", 1000.0, 100.0)
    gfl = pack(fl)
    save("pass_full", gfl, pack(fc, like=gfl), meta=dict(chi2=1000.0, kl=100.0, **P))

    # tag propagation on the whole volume-7 network
    G, tags, flips = run_tags(net0)
    gt = pack([G])
    tag_out = np.array([tags.get(int(n), -1) for n in gt.node["node_id"]], dtype=np.int64)
    save("tags_vol7", gt, None, extra=dict(tags=tag_out, flips=np.array(flips)), meta=dict(threshold=0.1))
    print("done in %.1fs" % (time.time() - t0))


if __name__ == "__main__":
    main()
