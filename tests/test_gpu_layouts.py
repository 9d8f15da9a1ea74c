"""The node-indexed stages -- initial track-state estimates (a2), updated-state distances
(a15), tag propagation (a16) -- on the renumbered device layouts ("tiled", "schedule"): the
host-order inputs are mapped to device order and the outputs back, and the results equal
the natural layout's bit for bit (the kernels are equivariant under node renumbering)."""
import numpy as np
import pytest
import torch

from gtf import synth
from gtf.device import DeviceGraph
from gtf.params import Params

pytestmark = pytest.mark.gpu

LAYOUTS = ["tiled", "schedule"]


def _event():
    return synth.event(seed=21, n_tracks=1500, fake_mean=synth.C4_FAKE)


@pytest.mark.parametrize("layout", LAYOUTS)
def test_track_state_estimates_layout_equivariant(layout):
    g = _event()
    res = []
    for lay in ("natural", layout):
        h = g.copy()
        d = DeviceGraph(h, layout=lay, tile=512)
        x = {k: v.cpu().numpy() for k, v in d.track_state_estimates(Params()).items()}
        d.node_ops(["priors_tse", "mw_tse", "degree"], Params())
        d.download(h)
        res.append((h, x))
    (a, xa), (b, xb) = res
    for f in ("tse_sv", "tse_cov", "tse_tau", "tse_xyzr", "tse_theta", "tse_var_ms", "tse_prior", "tse_mw"):
        assert np.array_equal(a.slot[f], b.slot[f], equal_nan=True), f
    assert np.array_equal(a.node["degree"], b.node["degree"])
    for k in xa:
        assert np.array_equal(xa[k], xb[k], equal_nan=True), k


@pytest.mark.parametrize("layout", LAYOUTS)
def test_updated_state_distances_layout_equivariant(layout):
    g = _event()
    truth = np.random.default_rng(1).integers(0, 40, g.n_nodes)
    res = []
    for lay in ("natural", layout):
        d = DeviceGraph(g.copy(), layout=lay, tile=512)
        d.full_pass(Params())
        ptr, cols = d.updated_state_distances(truth)
        res.append((ptr.cpu().numpy(), {k: v.cpu().numpy() for k, v in cols.items()}))
    (pa, ca), (pb, cb) = res
    assert np.array_equal(pa, pb) and pa[-1] > 0
    for k in ca:
        assert np.array_equal(ca[k], cb[k], equal_nan=True), k


@pytest.mark.parametrize("layout", LAYOUTS)
def test_tag_propagation_layout_equivariant(layout):
    g = _event()
    tags = np.arange(g.n_nodes, dtype=np.int64)
    radius = g.node["xyzr"][:, 3].copy()
    res = [DeviceGraph(g.copy(), layout=lay, tile=512).tag_propagation(tags, radius) for lay in ("natural", layout)]
    (ta, fa), (tb, fb) = res
    assert np.array_equal(ta, tb) and fa == fb and len(fa) >= 1
    torch.cuda.synchronize()
