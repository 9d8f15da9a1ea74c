"""The CPU oracle reproduces the reference's outputs on the golden fixtures.

Fixtures come from tests/golden/make_golden.py, which ran the reference's own
functions on the committed volume-7 event. This pins the oracle before it is
used to check the HIP path.
"""
import numpy as np
import pytest

import gtf_oracle as O
from compare import compare
from fixtures import load, expected_graph
from gtf.params import Params


def _params(meta):
    return Params(sigma0xy=meta["sigma0xy"], sigma0rz=meta["sigma0rz"], sigma0rz2=meta["sigma0rz2"],
                  endcap_boundary=meta["endcap_boundary"], chi2_cut=meta.get("chi2_cut", 2.0),
                  cluster_chi2=meta.get("chi2", 1000.0), cluster_kl=meta.get("kl", 100.0))


RTOL = 1e-12   # oracle vs reference: same NumPy calls, so (near) bit-exact


def test_extrapolate_it2():
    g, out, _, meta = load("extrapolate_it2")
    exp = expected_graph(g, out)
    O.extrapolate_stage(g, _params(meta))
    assert compare(g, exp, rtol=RTOL) == []


def test_extrapolate_full_load():
    g, out, _, meta = load("extrapolate_full")
    exp = expected_graph(g, out)
    O.extrapolate_stage(g, _params(meta))
    assert compare(g, exp, rtol=RTOL) == []


def test_update_with_orphans():
    g, out, _, meta = load("update_it2")
    assert (g.slot["slot_src"] < 0).any(), "fixture should carry orphan state keys"
    exp = expected_graph(g, out)
    O.update_stage(g, _params(meta))
    assert compare(g, exp, rtol=RTOL) == []


def test_cluster_tse():
    g, out, _, meta = load("cluster_tse")
    exp = expected_graph(g, out)
    O.cluster_stage(g, "tse", meta["chi2"], meta["kl"], _params(meta))
    assert compare(g, exp, rtol=RTOL) == []


def test_cluster_tie():
    """non-emptying np.where ties, made and clustered by the reference (make_golden_tie.py):
    the merged pair is (rows[0], rows[1]) and every listed index is removed"""
    g, out, extra, meta = load("cluster_tie")
    exp = expected_graph(g, out)
    assert extra["tie_nodes"].size >= 20
    O.cluster_stage(g, "tse", meta["chi2"], meta["kl"], _params(meta))
    assert compare(g, exp, rtol=RTOL) == []
    ids = g.node["node_id"]
    tied = np.isin(ids, extra["tie_nodes"])
    # a tie whose chi2 is above the threshold (-c 1.0) merges nothing (clustering.py:228)
    assert tied.sum() == extra["tie_nodes"].size and g.node["has_merged"][tied].sum() >= 15


def test_cluster_uts():
    g, out, _, meta = load("cluster_uts")
    exp = expected_graph(g, out)
    O.cluster_stage(g, "uts", meta["chi2"], meta["kl"], _params(meta))
    assert compare(g, exp, rtol=RTOL) == []


def test_full_pass():
    g, out, _, meta = load("pass_full")
    exp = expected_graph(g, out)
    O.full_pass(g, _params(meta))
    assert compare(g, exp, rtol=RTOL) == []


def test_tag_propagation():
    g, _, extra, _ = load("tags_vol7")
    tags, flips = O.tag_propagation(g)
    assert list(flips) == list(extra["flips"])
    kept = extra["tags"] >= 0          # isolated nodes are dropped by the script (:75-92)
    assert kept.sum() > 0.7 * len(kept)
    assert np.array_equal(tags[kept], extra["tags"][kept])
    assert np.array_equal(tags[~kept], g.node["tag"][~kept])


TSE_FIELDS = ("tse_sv", "tse_tau", "tse_cov", "tse_xyzr", "tse_theta", "tse_var_ms")


def test_track_state_estimates_full_vol7():
    """helper.compute_track_state_estimates (§8 a2) on the whole volume-7 network"""
    g, _, extra, meta = load("tse_full")
    exp = {f: g.slot[f].copy() for f in TSE_FIELDS}
    for f in TSE_FIELDS:
        g.slot[f][:] = np.nan
    node = O.compute_track_state_estimates(g, _params(meta))
    has = g.slot["tse_rank"] >= 0
    assert has.sum() == 14766
    for f in TSE_FIELDS:
        a, b = g.slot[f][has], exp[f][has]
        assert np.allclose(a, b, rtol=RTOL, atol=0, equal_nan=True), f
    for k in ("xy_mean_var", "zr_mean_var", "angle_of_rotation", "translation"):
        assert np.allclose(node[k], extra[k], rtol=RTOL, atol=0, equal_nan=True), k


@pytest.mark.parametrize("name", ["extrapolate_full", "pass_full"])
def test_updated_state_pairs_a15(name):
    """a15 (calculate_distance_between_updated_track_states.py:27-104, pair loop :134-195)
    against the reference's own function run on the same states (make_golden_a15.py)"""
    import os
    from fixtures import GOLDEN
    z = np.load(os.path.join(GOLDEN, "a15_pairs.npz"), allow_pickle=False)
    g, out, _, _ = load(name)
    e = expected_graph(g, out)
    ptr, got = O.updated_state_pairs(e, z[name + "__node_truth"])
    assert np.array_equal(ptr, z[name + "__pair_ptr"])
    assert ptr[-1] > 1000
    for c in ("chi2", "avg_tau", "avg_theta", "delta_theta"):
        np.testing.assert_allclose(got[c], z[name + "__" + c], rtol=RTOL, atol=1e-300, err_msg=c)
    assert np.array_equal(got["truth"], z[name + "__truth"])
