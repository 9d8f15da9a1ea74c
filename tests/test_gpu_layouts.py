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


def test_device_order_outputs_are_the_host_order_ones_renumbered():
    """host_order=False (the bench's device-resident timing): the same a2 node attributes
    and a15 pair segments, in the tiled layout's node order"""
    g = _event()
    d = DeviceGraph(g.copy(), layout="tiled", tile=512)
    xh = {k: v.cpu().numpy() for k, v in d.track_state_estimates(Params()).items()}
    xd = {k: v.cpu().numpy() for k, v in d.track_state_estimates(Params(), host_order=False).items()}
    order = d.order   # device node i is host node order[i]
    for k in xh:
        assert np.array_equal(xd[k], xh[k][order], equal_nan=True), k
    d.full_pass(Params())
    ph, ch = d.updated_state_distances()
    pd_, cd = d.updated_state_distances(host_order=False)
    ph, pd_ = ph.cpu().numpy(), pd_.cpu().numpy()
    ch, cd = {k: v.cpu().numpy() for k, v in ch.items()}, {k: v.cpu().numpy() for k, v in cd.items()}
    assert ph[-1] == pd_[-1] > 0
    seg = np.concatenate([np.arange(ph[h], ph[h + 1]) for h in order])
    for k in ch:
        assert np.array_equal(cd[k], ch[k][seg], equal_nan=True), k
