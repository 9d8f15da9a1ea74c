"""The diagnostics counting (gtf.diagnostics) on the CPU: fed with the CPU
checker's stage outputs split into the reference's calls, the block functions reproduce the
outlier-masking numbers the reference printed on the volume-7 network
(tests/golden/diag_vol7.json, captured from its stdout by make_golden_diag.py). The GPU
test (test_gpu_diagnostics.py) feeds them the device's outputs instead."""
import json
import os

import numpy as np

import gtf_oracle as O
from fixtures import GOLDEN, load
from gtf.diagnostics import cluster_block, message_passing_block, reweight_block
from gtf.params import Params


def _truth(g):
    t = json.load(open(os.path.join(GOLDEN, "diag_vol7.json")))["truth"]
    return np.array([t[str(int(n))] for n in g.node["node_id"]], dtype=np.int64)


def _expected(name):
    return json.load(open(os.path.join(GOLDEN, "diag_vol7.json")))[name]


def _params(meta):
    return Params(sigma0xy=meta["sigma0xy"], sigma0rz=meta["sigma0rz"], sigma0rz2=meta["sigma0rz2"],
                  endcap_boundary=meta["endcap_boundary"], chi2_cut=meta["chi2_cut"])


def test_cluster_counts_match_reference_print():
    g, _, _, meta = load("cluster_tse")
    p = _params(meta)
    sc = np.zeros(g.n_slots, np.uint8)
    for v in range(g.n_nodes):
        if not g.node["has_tse"][v]:
            continue
        left = O.cluster_node(g, "tse", v, meta["chi2"], meta["kl"], p, tie_policy="raise")
        if left is not None:
            for k in O._dict_order(g, "tse", v):
                sc[k] = 2 if k in left else 1
    assert [cluster_block(g, sc, _truth(g))] == _expected("cluster_tse")


def test_extrapolate_counts_match_reference_print():
    g, _, _, meta = load("extrapolate_it2")
    p = _params(meta)
    t = _truth(g)
    h = g.copy()
    O.message_passing(h, p)
    blocks = [message_passing_block(g, h.slot["uts_fresh"], t)]
    for _ in range(2):
        O.compute_prior_probabilities(h, "uts")
        a0 = h.slot["act"].copy()
        O.reweight(h, "uts", p.reweight_threshold)
        blocks.append(reweight_block(h, a0, h.slot["act"], t))
    assert blocks == _expected("extrapolate")


def test_update_counts_match_reference_print():
    g, _, _, meta = load("update_it2")
    t = _truth(g)
    h = g.copy()
    O.prune_states(h)
    O.compute_prior_probabilities(h, "tse")
    O.compute_prior_probabilities(h, "uts")
    a0 = h.slot["act"].copy()
    O.reweight(h, "uts", 0.1)
    assert [reweight_block(h, a0, h.slot["act"], t)] == _expected("update")
