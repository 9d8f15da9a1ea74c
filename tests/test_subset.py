"""gtf.graph.subset (the packed form of extraction's node removal) against pack() of
the reduced networkx graphs, on reference stage graphs (CPU)."""
import copy
import os
import pickle
import random

import numpy as np
import pytest

from fixtures import GOLDEN
from gtf.graph import NODE_FIELDS, SLOT_FIELDS, pack, refresh_send_mw, subset


def _load(name):
    with open(os.path.join(GOLDEN, "dropin_%s.pkl" % name), "rb") as f:
        return pickle.load(f)


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        return bool(np.array_equal(a, b, equal_nan=True))
    return bool(np.array_equal(a, b))


def _assert_graphs_equal(got, exp):
    assert got.n_nodes == exp.n_nodes and got.n_slots == exp.n_slots
    for k in ("slot_ptr", "out_ptr", "out_slot"):
        assert _same(getattr(got, k), getattr(exp, k)), k
    for k in NODE_FIELDS:
        assert _same(got.node[k], exp.node[k]), k
    for k in SLOT_FIELDS:
        assert _same(got.slot[k], exp.slot[k]), k


@pytest.mark.parametrize("name,key,seed", [("extract", "input", 1), ("extrapolate", "out", 2),
                                           ("update", "in", 3), ("update", "out", 4)])
def test_subset_matches_pack_of_reduced_graphs(name, key, seed):
    subs = copy.deepcopy(_load(name)[key])
    rng = random.Random(seed)
    g = pack(subs)
    keep = np.zeros(g.n_nodes, bool)
    reduced = []
    i = 0
    for G in subs:
        whole = rng.random() < 0.1            # a fragment / fully extracted subgraph
        drop = []
        for n in G.nodes:
            k = not whole and rng.random() > 0.2
            keep[i] = k
            if not k:
                drop.append(n)
            i += 1
        H = copy.deepcopy(G)
        H.remove_nodes_from(drop)
        if len(H):
            reduced.append(H)
    assert 0 < keep.sum() < g.n_nodes
    _assert_graphs_equal(subset(g, keep), pack(reduced))


def test_subset_keep_all_and_none():
    subs = copy.deepcopy(_load("extrapolate")["out"])
    g = pack(subs)
    _assert_graphs_equal(subset(g, np.ones(g.n_nodes, bool)), g)
    e = subset(g, np.zeros(g.n_nodes, bool))
    assert e.n_nodes == 0 and e.n_slots == 0 and e.n_edges == 0


def test_refresh_send_mw_matches_pack():
    g = pack(copy.deepcopy(_load("extract")["input"]))
    exp = g.slot["send_mw"].copy()
    g.slot["send_mw"][:] = np.nan
    refresh_send_mw(g)
    assert _same(g.slot["send_mw"], exp)


@pytest.mark.parametrize("name,key", [("extract", "input"), ("extract", "remaining"), ("extrapolate", "out"),
                                      ("update", "in")])
def test_candidate_order_matches_networkx_cca(name, key):
    """gtf_candidate_order (native) == the reference CCA's candidate node orders
    (networkx weakly connected components + subgraph copies), on reference graphs"""
    import sys
    from fixtures import GOLDEN as _G  # noqa: F401
    from gtf.extract import candidate_order
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "gnn-track-finding_amd"))
    from extract.extract_track_candidates import candidates_nx
    subs = _load(name)[key]
    g = pack(subs)
    got = candidate_order(g)
    exp = np.zeros(g.n_nodes, np.int32)
    pos, vi = {}, 0
    for s in subs:
        for n in s.nodes:
            pos[(id(s), n)] = vi
            vi += 1
    n_multi = 0
    for s in subs:
        cs = candidates_nx(s)
        n_multi += len(cs) > 1
        for c in cs:
            for k, n in enumerate(c.nodes):
                exp[pos[(id(s), n)]] = k
    assert n_multi > 0 or key == "remaining"
    assert np.array_equal(got, exp)
