"""The real multi-volume event on the CPU side (SURVEY §8a "C2", the committed 800'
all-volume event; tests/golden/make_golden_800.py):

* the native event conversion (gtf_build_event_csr, host C++) reproduces the
  reference's packed network -- node order, successor order, subgraphs and the set
  order of every track_state_estimates dict -- on all 8 volumes (the structure digest
  the fixtures were made on);
* the oracle (the CPU checker) reproduces the reference's per-subgraph clustering of
  iteration 1, including which subgraphs raise (tie empties the list), from its own
  restatement of the initial states.
"""
import numpy as np
import pytest

import gtf_oracle as O
import real800 as R
from gtf import io
from gtf.params import Params


def test_native_event_conversion_matches_reference_structure():
    g, vivl = io.build_event_csr(R.PREFIX, *R.VOLS)
    assert g.n_nodes == 29590 and g.n_edges == 89028
    for name in ("cluster_tse", "pass"):
        assert R.structure_digest(g) == str(R.fixture(name)["structure_sha"]), name
    z = R.fixture("cluster_tse")
    assert z["raised"].size == int(g.node["sub_id"].max()) + 1


@pytest.mark.slow
def test_oracle_cluster_tse_matches_reference_per_subgraph():
    p = Params()
    g, _ = io.build_event_csr(R.PREFIX, *R.VOLS)
    O.compute_track_state_estimates(g, p)
    O.compute_prior_probabilities(g, "tse")
    O.compute_mixture_weights(g, "tse")
    O.query_node_degree_in_edges(g)
    # clustering.cluster subgraph by subgraph: a node whose tie empties its list makes
    # the reference raise (ValueError) for its whole subgraph
    node_err = np.zeros(g.n_nodes, np.uint32)
    deact = []
    for v in range(g.n_nodes):
        if not g.node["has_tse"][v]:
            continue
        try:
            r = O.cluster_node(g, "tse", v, R.CLUSTER_TSE["chi2"], R.CLUSTER_TSE["kl"], p, tie_policy="raise")
        except O.ReferenceError_:
            node_err[v] = 8
            continue
        if r is not None:
            deact.extend(r)
    for k in deact:
        if g.slot["is_edge"][k]:
            g.slot["act"][k] = 0
    O.query_node_degree_in_edges(g)
    errs, stats = R.compare(g, R.fixture("cluster_tse"), node_err)
    print(stats)
    assert errs == [], "\n".join(errs)
