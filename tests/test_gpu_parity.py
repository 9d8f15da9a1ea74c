"""HIP path (through the C-ABI) vs the pinned oracle and the reference fixtures.

Bar: activation masks, dict membership/order (ranks), merged flags and degree
bit-exact; floats within 1e-6 relative (north star tolerance).
"""
import numpy as np
import pytest

import gtf_oracle as O
from compare import compare
from fixtures import load, expected_graph
from gtf.params import Params

pytestmark = pytest.mark.gpu
RTOL = 1e-6


def _params(meta):
    return Params(sigma0xy=meta["sigma0xy"], sigma0rz=meta["sigma0rz"], sigma0rz2=meta["sigma0rz2"],
                  endcap_boundary=meta["endcap_boundary"], chi2_cut=meta.get("chi2_cut", 2.0),
                  cluster_chi2=meta.get("chi2", 1000.0), cluster_kl=meta.get("kl", 100.0))


def _dev(g):
    from gtf.device import DeviceGraph
    return DeviceGraph(g)


def _run(name, fn, rtol=RTOL):
    g, out, extra, meta = load(name)
    exp = expected_graph(g, out)
    p = _params(meta)
    d = _dev(g)
    d.clear_errors()
    fn(d, p, meta)
    d.raise_errors()
    got = d.download(g.copy())
    errs = compare(got, exp, rtol=rtol, atol=0.0 if rtol == 0.0 else 1e-12)
    assert errs == [], "\n".join(errs)
    return got


def test_extrapolate_it2():
    _run("extrapolate_it2", lambda d, p, m: d.extrapolate(p))


def test_extrapolate_full_load():
    _run("extrapolate_full", lambda d, p, m: d.extrapolate(p))


def test_update_with_orphans():
    _run("update_it2", lambda d, p, m: d.update(p))


# clustering from the reference's own states: numpy's BLAS rounding is restated
# (csrc/gtf_math.h, tests/test_numpy_rounding.py), so every output is bit for bit the
# reference's (rtol 0)
def test_cluster_tse():
    _run("cluster_tse", lambda d, p, m: d.cluster("tse", m["chi2"], m["kl"], p), rtol=0.0)


def test_cluster_tie():
    """the reference's own clustering on non-emptying ties (make_golden_tie.py)"""
    got = _run("cluster_tie", lambda d, p, m: d.cluster("tse", m["chi2"], m["kl"], p), rtol=0.0)
    _, _, extra, _ = load("cluster_tie")
    tied = np.isin(got.node["node_id"], extra["tie_nodes"])
    assert tied.sum() >= 20 and got.node["has_merged"][tied].sum() >= 15


def test_cluster_uts():
    _run("cluster_uts", lambda d, p, m: d.cluster("uts", m["chi2"], m["kl"], p), rtol=0.0)


def test_full_pass_fused():
    _run("pass_full", lambda d, p, m: d.full_pass(p))


def test_tag_propagation():
    g, _, extra, _ = load("tags_vol7")
    d = _dev(g)
    tags, flips = d.tag_propagation(g.node["tag"], g.node["xyzr"][:, 3])
    assert list(flips) == list(extra["flips"])
    kept = extra["tags"] >= 0
    assert np.array_equal(tags[kept], extra["tags"][kept])


def test_tag_propagate_one_call():
    """gtf_tag_propagate (the whole stage behind one C-ABI call, caller workspace) against
    the reference's tags and flip vector, through ctypes with no Python sweep loop"""
    import ctypes
    import torch
    from gtf import _native as nat
    g, _, extra, _ = load("tags_vol7")
    d = _dev(g)
    L = d.lib
    tags = torch.from_numpy(np.ascontiguousarray(g.node["tag"], dtype=np.int64)).to(d.device)
    radius = torch.from_numpy(np.ascontiguousarray(g.node["xyzr"][:, 3], dtype=np.float64)).to(d.device)
    nb = L.gtf_tag_workspace_bytes(g.n_nodes, g.n_edges)
    ws = torch.zeros(nb, dtype=torch.uint8, device=d.device)
    flips = (ctypes.c_int32 * 64)()
    sweeps = ctypes.c_int32(0)
    nat.check(L.gtf_tag_propagate(ctypes.byref(d.cg), ctypes.c_void_p(radius.data_ptr()),
                                  ctypes.c_void_p(tags.data_ptr()), 0.1, 64, ctypes.cast(flips, ctypes.c_void_p), ctypes.byref(sweeps),
                                  ctypes.c_void_p(ws.data_ptr()), nb, d.stream))
    torch.cuda.synchronize()
    assert list(flips[:sweeps.value]) == list(extra["flips"])
    out = tags.cpu().numpy()
    kept = extra["tags"] >= 0
    assert np.array_equal(out[kept], extra["tags"][kept])
    # too small a workspace is refused, not overrun
    assert L.gtf_tag_propagate(ctypes.byref(d.cg), ctypes.c_void_p(radius.data_ptr()),
                               ctypes.c_void_p(tags.data_ptr()), 0.1, 64, ctypes.cast(flips, ctypes.c_void_p), ctypes.byref(sweeps),
                               ctypes.c_void_p(ws.data_ptr()), nb - 1, d.stream) != 0
