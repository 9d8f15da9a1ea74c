"""Edge cases of the fused pass on the GPU (through the C-ABI), against the oracle:

  * hub hits with more than 64 slots (receivers beyond the lane-group buckets run one
    thread per node, k_node; senders with > 8 out-edges take several k_sender chunks),
    built by wiring a few hits of a seeded synthetic event to ~100 neighbours each;
  * an empty graph and a graph of isolated hits (no slots): the pass is a no-op;
  * a graph with every edge deactivated: nothing is extrapolated, no state appears.

Same bar as test_gpu_synthetic.py (masks exact except ulp-undetermined decisions,
floats within 1e-6 relative plus the oracle's own perturbation noise); the hub graph
is also run through the thread-per-node implementation, bit for bit.
"""
import numpy as np
import pytest

import gtf_oracle as O
from compare import compare_noise, noise_envelope
from gtf import graph, synth
from gtf.params import Params

pytestmark = pytest.mark.gpu


def hub_event(seed=7, n_tracks=400, n_hubs=3, fan=110):
    """a synthetic event plus n_hubs hits joined (both directions) to the `fan` hits
    closest in azimuth on the two neighbouring layers"""
    p = Params()
    g = synth.event(seed=seed, n_tracks=n_tracks, fake_mean=synth.C4_FAKE)
    x, y, z, r = (g.node["gnn"][:, i].copy() for i in range(4))
    layer = g.node["layer"].copy()
    owner = np.repeat(np.arange(g.n_nodes), np.diff(g.out_ptr.astype(np.int64)))
    src = owner.astype(np.int64)
    dst = g.slot_dst()[g.out_slot].astype(np.int64)
    phi = np.arctan2(y, x)
    rng = np.random.default_rng(seed)
    levels = np.unique(layer)
    mid = np.nonzero((layer > levels[0]) & (layer < levels[-1]))[0]
    have = set(zip(src.tolist(), dst.tolist()))
    add_s, add_d = [], []
    for h in rng.choice(mid, n_hubs, replace=False):
        li = np.searchsorted(levels, layer[h])
        near = np.nonzero((layer == levels[li - 1]) | (layer == levels[li + 1]))[0]
        dphi = np.abs(np.angle(np.exp(1j * (phi[near] - phi[h]))))
        for v in near[np.argsort(dphi)[:fan]]:
            if (h, v) not in have:
                have.add((h, v)); have.add((v, h))
                add_s += [h, v]; add_d += [v, h]
    src = np.concatenate([src, np.array(add_s, np.int64)])
    dst = np.concatenate([dst, np.array(add_d, np.int64)])
    return synth._assemble(g.n_nodes, src, dst, x, y, z, r, layer, p)


def _gpu(g, p, schedule=True, layout="natural"):
    from gtf.device import DeviceGraph
    d = DeviceGraph(g, schedule=schedule, layout=layout)
    d.clear_errors()
    d.full_pass(p)
    flags = d.errors()
    return d, d.download(g.copy()), flags


def test_hub_nodes_beyond_64_slots_match_oracle():
    g = hub_event()
    deg = np.diff(g.slot_ptr)
    outdeg = np.diff(g.out_ptr)
    assert (deg > 64).sum() >= 3 and outdeg.max() > 64
    p = Params()

    def run(x):
        O.full_pass(x, p, tie_policy="stop")
        return x

    ref, noise, flips = noise_envelope(run, g)
    d, got, flags = _gpu(g, p)
    assert d.n_big >= 3
    errs, stats = compare_noise(got, ref, noise, flips)
    print("hub event: %d edges, max slots %d, %s, device flags %d" % (g.n_edges, deg.max(), stats, flags))
    assert errs == [], "\n".join(errs)
    # the same pass one thread per node everywhere, and in the tiled and padded layouts
    # (the > 64-slot nodes after the padded tiles): bit for bit
    for kw in ({"schedule": False}, {"layout": "tiled"}, {"layout": "padded"}):
        _, got1, flags1 = _gpu(g, p, **kw)
        assert flags1 == flags, kw
        for k in ("act", "uts_rank", "uts_sv", "uts_cov", "uts_mw", "uts_prior", "edge_mw"):
            a, b = got.slot[k], got1.slot[k]
            assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), (kw, k)
        for k in ("has_merged", "merged_state", "merged_cov", "degree"):
            a, b = got.node[k], got1.node[k]
            assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), (kw, k)


@pytest.mark.parametrize("layout", ["natural", "padded"])
@pytest.mark.parametrize("keep", ["none", "isolated"])
def test_graph_without_slots_is_a_no_op(keep, layout):
    g = synth.event(seed=3, n_tracks=60)
    if keep == "none":
        h = graph.subset(g, np.zeros(g.n_nodes, bool))
        assert h.n_nodes == 0
    else:
        iso = np.diff(g.slot_ptr) == 0
        if not iso.any():
            pytest.skip("no isolated hit in this seed")
        h = graph.subset(g, iso)
        assert h.n_slots == 0 and h.n_nodes > 0
    p = Params()
    O.full_pass(h.copy(), p)   # the oracle takes it too
    d, got, flags = _gpu(h, p, layout=layout)
    assert flags == 0
    for k in ("has_merged", "merged_state", "merged_cov", "degree", "has_uts"):
        a, b = got.node[k], h.node[k]
        assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), k


def test_all_edges_inactive():
    g = synth.event(seed=4, n_tracks=200)
    g.slot["act"][:] = 0
    p = Params()
    exp = g.copy()
    O.full_pass(exp, p)
    d, got, flags = _gpu(g, p)
    assert flags == 0
    assert got.slot["act"].sum() == 0
    assert (got.slot["uts_rank"] < 0).all() and got.node["has_uts"].sum() == 0
    assert np.array_equal(got.node["degree"], exp.node["degree"])
    assert np.array_equal(got.node["has_merged"], exp.node["has_merged"])
