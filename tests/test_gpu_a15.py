"""a15 on the GPU: gtf_updated_state_distances (calculate_distance_between_updated_track_
states.py:27-104 over the pair loop :134-195) against

  * the reference's own mahalanobis_distance run on the committed volume-7 states
    (tests/golden/a15_pairs.npz, tests/golden/make_golden_a15.py): pair layout and truth
    flags exact, floats within 1e-6 relative;
  * the oracle (oracle.updated_state_pairs) on the states the HIP extrapolation leaves on
    a seeded synthetic event whose hub nodes carry > 64 dict entries (the one-wavefront
    path): same inputs, so within 1e-12.
"""
import os

import numpy as np
import pytest

import gtf_oracle as O
from fixtures import GOLDEN, load, expected_graph
from gtf.params import Params

pytestmark = pytest.mark.gpu

COLS = ("chi2", "avg_tau", "avg_theta", "delta_theta")


def _gpu(g, truth):
    from gtf.device import DeviceGraph
    d = DeviceGraph(g)
    ptr, out = d.updated_state_distances(truth)
    return ptr.cpu().numpy(), {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("name", ["extrapolate_full", "pass_full"])
def test_a15_matches_reference_pairs(name):
    z = np.load(os.path.join(GOLDEN, "a15_pairs.npz"), allow_pickle=False)
    g, out, _, _ = load(name)
    e = expected_graph(g, out)
    ptr, got = _gpu(e, z[name + "__node_truth"])
    assert np.array_equal(ptr, z[name + "__pair_ptr"])
    for c in COLS:
        ref = z[name + "__" + c]
        # <theta> is a mean of two angles: absolute floor where it cancels to ~0
        atol = 1e-12 if c in ("avg_theta", "delta_theta", "avg_tau") else 0.0
        np.testing.assert_allclose(got[c], ref, rtol=1e-6, atol=atol, err_msg=c)
    assert np.array_equal(got["truth"], z[name + "__truth"])


def _hub_states(seed=5):
    """a synthetic event with 4 hub hits (> 64 slots each) after the HIP extrapolation
    stage, with every slot of each hub turned into an active edge holding an
    updated_track_states entry (random dict order, states drawn around the event's own
    entries, SPD covariances): > 64 dict entries per hub, so the pair kernel's
    one-wavefront path and its dict-position map carry thousands of pairs."""
    from gtf.device import DeviceGraph
    from test_gpu_edges import hub_event
    g = hub_event(seed=seed, n_tracks=1500, n_hubs=4)
    d = DeviceGraph(g)
    d.extrapolate(Params())
    g = d.download(g.copy())
    rng = np.random.default_rng(seed)
    S = g.slot
    have = np.nonzero(S["uts_rank"] >= 0)[0]
    hubs = np.nonzero(np.diff(g.slot_ptr) > 64)[0]
    assert hubs.size >= 3 and have.size > 100
    for v in hubs:
        lo, hi = int(g.slot_ptr[v]), int(g.slot_ptr[v + 1])
        ks = np.arange(lo, hi)[S["slot_src"][lo:hi] >= 0]
        S["is_edge"][ks] = 1
        S["act"][ks] = 1
        S["uts_rank"][lo:hi] = -1
        S["uts_rank"][ks] = rng.permutation(ks.size)
        src = rng.choice(have, ks.size)
        S["uts_sv"][ks] = S["uts_sv"][src] * (1 + 1e-3 * rng.standard_normal((ks.size, 3)))
        S["uts_tau"][ks] = S["uts_tau"][src] + 1e-3 * rng.standard_normal(ks.size)
        a, c = rng.uniform(1e-4, 1e-2, (2, ks.size))
        b = rng.uniform(-0.5, 0.5, ks.size) * np.sqrt(a * c)
        S["uts_cov"][ks] = np.stack([a, b, b, c, rng.uniform(1e-4, 1e-2, ks.size)], axis=1)
        g.node["has_uts"][v] = 1
    return g, hubs


def test_a15_matches_oracle_with_hubs():
    g, hubs = _hub_states()
    truth = np.random.default_rng(0).integers(0, 3, g.n_nodes)
    ptr, got = _gpu(g, truth)
    ref_ptr, ref = O.updated_state_pairs(g, truth)
    assert np.array_equal(ptr, ref_ptr)
    per_node = np.diff(ptr)
    assert per_node[hubs].min() > 64 * 63 // 2 and ptr[-1] > 10000
    for c in COLS:
        np.testing.assert_allclose(got[c], ref[c], rtol=1e-10, atol=1e-15, err_msg=c)
    assert np.array_equal(got["truth"], ref["truth"])
    assert got["truth"].sum() > 0


def test_a15_dropin_cli(tmp_path):
    """the drop-in script on the reference's own extrapolation output (gpickles): every
    row equals the oracle's mahalanobis_distance_updated on the same networkx attributes"""
    import csv
    from test_dropin import _load, _run_cli, _write
    d = _load("extrapolate")
    _write(d["out"], str(tmp_path / "in"))
    _run_cli("calculate_distance_between_updated_states/calculate_distance_between_updated_track_states.py",
             ["-i", str(tmp_path / "in") + "/", "-o", str(tmp_path / "pairs.csv")], str(tmp_path))
    got = {}
    with open(tmp_path / "pairs.csv") as f:
        for r in csv.DictReader(f):
            got[(int(r["node"]), int(r["neighbour1"]), int(r["neighbour2"]))] = (
                float(r["chi2"]), float(r["tau_average"]), float(r["theta_average"]), float(r["delta_theta"]),
                int(r["truth"]))
    exp = {}
    for G in d["out"]:
        for node, attr in G.nodes(data=True):
            nact = sum(1 for u, _ in G.in_edges(node) if G[u][node]["activated"] == 1)
            if nact <= 1 or "updated_track_states" not in attr:
                continue
            uts = attr["updated_track_states"]
            keys = list(uts.keys())
            for i in range(len(keys)):
                for j in range(i):
                    a, b = uts[keys[i]], uts[keys[j]]
                    r = O.mahalanobis_distance_updated(np.asarray(a["joint_vector"]), a["joint_vector_covariance"],
                                                       np.asarray(b["joint_vector"]), b["joint_vector_covariance"],
                                                       attr["xyzr"], G.nodes[keys[i]]["xyzr"],
                                                       G.nodes[keys[j]]["xyzr"])
                    t = [G.nodes[n]["truth_particle"] for n in (node, keys[i], keys[j])]
                    exp[(int(node), int(keys[i]), int(keys[j]))] = tuple(r) + (int(t[0] == t[1] == t[2]),)
    assert len(exp) >= 5 and got.keys() == exp.keys()
    for k, e in exp.items():
        np.testing.assert_allclose(got[k][:4], e[:4], rtol=1e-6, atol=1e-12, err_msg=str(k))
        assert got[k][4] == e[4], k
