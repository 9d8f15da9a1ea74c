"""gtf_track_state_estimates (§8 a2) on the GPU vs the reference's own output.

tests/golden/tse_full.npz holds helper.compute_track_state_estimates run by the
reference on the whole volume-7 network of the committed 134 event
(make_golden_tse.py). The GPU recomputes every TSE field from the coordinates and
the dict order alone; floats must agree within 1e-6 relative (the north-star bar)
-- element-wise, with an absolute floor of 1e-12 of the row's largest entry for
entries that are exact zeros in one and rounding residue in the other (the
reference's np.linalg.inv leaves ~1e-17 where the closed form has 0). A synthetic
event checks the same against the oracle.
"""
import numpy as np
import pytest

import gtf_oracle as O
from fixtures import load
from gtf import synth
from gtf.params import Params

pytestmark = pytest.mark.gpu

FIELDS = ("tse_sv", "tse_tau", "tse_cov", "tse_xyzr", "tse_theta", "tse_var_ms")


def _params(meta):
    return Params(sigma0xy=meta["sigma0xy"], sigma0rz=meta["sigma0rz"], sigma0rz2=meta["sigma0rz2"],
                  endcap_boundary=meta["endcap_boundary"])


def _gpu_tse(g, p):
    from gtf.device import DeviceGraph
    h = g.copy()
    for f in FIELDS:
        h.slot[f][:] = np.nan
    d = DeviceGraph(h)
    x = d.track_state_estimates(p)
    d.download(h)
    return h, {k: v.cpu().numpy() for k, v in x.items()}


def _check(got, exp, has, name):
    a, b = got[has], exp[has]
    if a.ndim == 1:
        a, b = a[:, None], b[:, None]
    scale = np.nanmax(np.abs(b), axis=1, keepdims=True)
    ok = (np.abs(a - b) <= 1e-6 * np.abs(b) + 1e-12 * scale) | (np.isnan(a) & np.isnan(b))
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    print("%s: max rel %.3g (entries beyond 1e-6 rel: %d)" % (name, np.nanmax(np.where(np.abs(b) > 1e-12 * scale, rel, 0)),
                                                             int((~ok).sum())))
    assert ok.all(), (name, np.argwhere(~ok)[:5])


def test_gpu_tse_matches_reference_vol7():
    g, _, extra, meta = load("tse_full")
    got, x = _gpu_tse(g, _params(meta))
    has = g.slot["tse_rank"] >= 0
    for f in FIELDS:
        _check(got.slot[f], g.slot[f], has, f)
    allnodes = np.ones(g.n_nodes, bool)
    for k in ("xy_mean_var", "zr_mean_var", "angle_of_rotation", "translation"):
        _check(x[k], extra[k], allnodes, k)


def test_gpu_tse_matches_oracle_synthetic():
    g = synth.event(seed=7, n_tracks=600, fake_mean=synth.C4_FAKE)
    rng = np.random.default_rng(7)   # arbitrary dict orders (the reference's are set orders)
    for v in range(g.n_nodes):
        lo, hi = g.slot_ptr[v], g.slot_ptr[v + 1]
        g.slot["tse_rank"][lo:hi] = rng.permutation(hi - lo) * 3 + 1    # sparse ranks too
    p = Params()
    ref = g.copy()
    node = O.compute_track_state_estimates(ref, p)
    got, x = _gpu_tse(g, p)
    has = g.slot["tse_rank"] >= 0
    assert has.any()
    for f in FIELDS:
        _check(got.slot[f], ref.slot[f], has, f)
    for k in node:
        _check(x[k], node[k], np.ones(g.n_nodes, bool), k)


def test_gpu_tse_beyond_64_slots():
    """a node with 70 neighbours (the 64-lane group loops over its slots; the
    position -> neighbour table is not staged)"""
    rng = np.random.default_rng(11)
    n = 71
    phi = rng.uniform(0.1, 0.5, n)
    r = np.concatenate([[300.0], rng.uniform(100, 600, n - 1)])
    z = np.concatenate([[100.0], rng.uniform(-800, 800, n - 1)])
    x, y = r * np.cos(phi), r * np.sin(phi)
    a = np.concatenate([np.zeros(n - 1, np.int64), np.arange(1, n)])
    b = np.concatenate([np.arange(1, n), np.zeros(n - 1, np.int64)])
    g = synth._assemble(n, a, b, x, y, z, r, (np.arange(n) % 5).astype(np.float64), Params())
    assert np.diff(g.slot_ptr).max() == 70
    p = Params()
    ref = g.copy()
    node = O.compute_track_state_estimates(ref, p)
    got, xx = _gpu_tse(g, p)
    has = g.slot["tse_rank"] >= 0
    for f in FIELDS:
        _check(got.slot[f], ref.slot[f], has, f)
    for k in node:
        _check(xx[k], node[k], np.ones(g.n_nodes, bool), k)
