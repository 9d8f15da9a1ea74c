"""Config C1 (BASELINE configs[0]): the reference's toy Monte Carlo event in 3-D.

* The x-y event of gtf.toymc equals the reference's own simulate_event
  (src/toyMC_model/track_simulation_xy.py:36-188) run with np.random.seed(0)
  (tests/golden/toymc_c1.npz, tests/golden/make_golden_toymc.py): node ids and order
  of every subgraph, x / y bit for bit, layer, truth, directed edges in G.edges order.
* The CPU path of C1 (the reference's NumPy / networkx arithmetic, restated by the
  oracle): initial track-state estimates, priors, mixture weights, degree, full load,
  then the fused pass; it runs without a reference exception and is deterministic.
* On the GPU: the same chain through libgtf (gtf_track_state_estimates, the node ops,
  gtf_pass) equals the oracle (masks, ranks, flags exact; floats within 1e-6).
"""
import os

import numpy as np
import pytest

import gtf_oracle as O
from compare import compare
from fixtures import GOLDEN
from gtf import toymc
from gtf.graph import refresh_send_mw
from gtf.params import Params


def test_toy_xy_event_is_the_references():
    z = np.load(os.path.join(GOLDEN, "toymc_c1.npz"), allow_pickle=False)
    sgs = toymc.subgraphs(0)
    assert len(sgs) == int(z["n_subgraphs"])
    for i, G in enumerate(sgs):
        lo, hi = z["sub_ptr"][i], z["sub_ptr"][i + 1]
        assert list(G.nodes()) == z["nodes"][lo:hi].tolist()
        for j, n in enumerate(G.nodes()):
            a = G.nodes[n]
            assert a["xy"][0] == z["x"][lo + j] and a["xy"][1] == z["y"][lo + j]
            assert a["in_volume_layer_id"] == z["layer"][lo + j]
            assert a["truth_particle"] == z["truth"][lo + j]
        e0, e1 = z["edge_ptr"][i], z["edge_ptr"][i + 1]
        assert [tuple(e) for e in G.edges()] == list(zip(z["edge_src"][e0:e1].tolist(),
                                                         z["edge_dst"][e0:e1].tolist()))


def test_toy_z_is_cot_theta_r():
    for G in toymc.subgraphs(0):
        for n in G.nodes():
            x, y, zz, r = G.nodes[n]["xyzr"]
            assert r == np.sqrt(x * x + y * y) and r > 0
            t = G.nodes[n]["truth_particle"]
            assert zz == toymc.cot_theta(0, 88)[t] * r


def cpu_c1(p=None):
    """C1 on the CPU path: a2 -> a3 / a4 / a5 -> full load -> the fused pass."""
    p = p or Params()
    g = toymc.event(0)
    O.compute_track_state_estimates(g, p)
    O.compute_prior_probabilities(g, "tse")
    O.compute_mixture_weights(g, "tse")
    O.query_node_degree_in_edges(g)
    refresh_send_mw(g)
    toymc.full_load(g)
    start = g.copy()
    info = O.full_pass(g, p, tie_policy="raise")
    return start, g, info


def test_c1_cpu_path_runs_and_is_deterministic():
    start, g, info = cpu_c1()
    assert g.n_nodes == 110 and g.n_edges == 300
    assert start.node["has_merged"].sum() == (np.diff(g.slot_ptr) > 0).sum() == 100   # 10 isolated hits
    assert info["merged_nodes"] > 0
    assert (g.slot["uts_rank"] >= 0).sum() > 0
    assert 0 < g.slot["act"].sum() < g.n_edges
    _, g2, _ = cpu_c1()
    assert compare(g2, g, rtol=0.0) == []


@pytest.mark.gpu
def test_c1_gpu_matches_cpu_path():
    from gtf.device import DeviceGraph
    p = Params()
    start, ref, _ = cpu_c1(p)
    g = toymc.event(0)
    d = DeviceGraph(g)
    d.clear_errors()
    d.track_state_estimates(p)
    d.node_ops(["priors_tse", "mw_tse", "degree"], p)
    d.raise_errors()
    d.download(g)
    refresh_send_mw(g)
    toymc.full_load(g)
    errs = compare(g, start, rtol=1e-6)
    assert errs == [], "\n".join(errs)
    d = DeviceGraph(g)
    d.clear_errors()
    d.full_pass(p)
    d.raise_errors()
    got = d.download(g.copy())
    errs = compare(got, ref, rtol=1e-6)
    assert errs == [], "\n".join(errs)
