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


@pytest.fixture(params=[False, True], ids=["kernel_classes", "static_classes"], autouse=True)
def _classes(request):
    """every test with the node kernel building its slot classes (the default at this size)
    and with the graph-static classes uploaded (gtf_graph.slot_class, the large-graph default)"""
    global CLASSES
    CLASSES = request.param
    yield


def _dev(g):
    from gtf.device import DeviceGraph
    return DeviceGraph(g, classes=CLASSES)


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


# gtf_tag_propagate's forms (environment; unset: the default)
_CSR_MODES = {
    "default": {},
    "packed_n1": {"GTF_TAG_NPT": "1"},
    "packed_n2": {"GTF_TAG_NPT": "2", "GTF_TAG_PREP_NPT": "2", "GTF_TAG_R": "2"},
    "packed_n2_r4": {"GTF_TAG_NPT": "2", "GTF_TAG_PREP_NPT": "0", "GTF_TAG_R": "4"},
    "packed_n4": {"GTF_TAG_NPT": "4", "GTF_TAG_PREP_NPT": "4", "GTF_TAG_R": "4", "GTF_TAG_COOP": "0"},
    "packed_n2_lanes": {"GTF_TAG_NPT": "2", "GTF_TAG_PREP_NPT": "2", "GTF_TAG_COOP": "0"},
    "coop1": {"GTF_TAG_NPT": "2", "GTF_TAG_PREP_NPT": "1", "GTF_TAG_COOP": "1"},
    "coop4": {"GTF_TAG_NPT": "2", "GTF_TAG_PREP_NPT": "1", "GTF_TAG_COOP": "4"},
    "packed_prep1": {"GTF_TAG_PREP_NPT": "1"},
    "unpacked_n2": {"GTF_TAG_NPT": "2", "GTF_TAG_PREP_NPT": "2", "GTF_TAG_PACK": "0"},
    "counts_thread_prep": {"GTF_TAG_KWORD": "0", "GTF_TAG_NPT": "1", "GTF_TAG_PREP_NPT": "1"},
    "counts_group_prep": {"GTF_TAG_KWORD": "0", "GTF_TAG_NPT": "2", "GTF_TAG_PREP_NPT": "0"},
    "mask": {"GTF_TAG_CSR": "0"},
}
_TAG_ENV = ("GTF_TAG_CSR", "GTF_TAG_KWORD", "GTF_TAG_NPT", "GTF_TAG_PREP_NPT", "GTF_TAG_R", "GTF_TAG_PACK", "GTF_TAG_COOP")


def _csr_env(monkeypatch, mode):
    """gtf_tag_propagate's sweep form: compact kept lists with one packed word per node (1, 2 or
    4 nodes per thread in the prepare and the sweeps, 2 or 4 kept indices per node in a sweep's
    second round; the thread prepare's lists back to back per run of 256 nodes, or at the front
    of each node's out-range with GTF_TAG_PACK=0; on packed lists the 2-node sweep is the
    wave-cooperative one, 1 / 2 / 4 groups of 64 nodes per wave, or GTF_TAG_COOP=0 the per-lane
    one) or a count and an offset per node, built by the
    one-node-per-thread or the lane-group prepare, or the keep-mask sweeps (GTF_TAG_CSR=0)"""
    for k in _TAG_ENV:
        monkeypatch.setenv(k, _CSR_MODES[mode].get(k, ""))


@pytest.mark.parametrize("csr", list(_CSR_MODES))
@pytest.mark.parametrize("poll", ["1", "0"])
@pytest.mark.parametrize("schedule", [True, False])
@pytest.mark.parametrize("max_sweeps", [64, 3, 0])
def test_tag_propagate_stop_rule_and_cap(schedule, max_sweeps, poll, csr, monkeypatch):
    """the stop rule evaluated on the device (gtf_tag_propagate's batched sweeps): the
    reference's flip vector, cut at max_sweeps, on the sender-schedule and the thread-per-node
    prepare kernels, over the compact kept lists with int32 tags or the keep mask (GTF_TAG_CSR),
    with the batch report polled in mapped memory or copied back (GTF_TAG_POLL); the tags equal
    the host loop of single sweeps run that many times"""
    monkeypatch.setenv("GTF_TAG_POLL", poll)
    _csr_env(monkeypatch, csr)
    import ctypes
    import torch
    from gtf import _native as nat
    from gtf.device import DeviceGraph
    g, _, extra, _ = load("tags_vol7")
    d = DeviceGraph(g, schedule=schedule)
    L = d.lib
    t0 = np.ascontiguousarray(g.node["tag"], dtype=np.int64)
    tags = torch.from_numpy(t0).to(d.device)
    radius = torch.from_numpy(np.ascontiguousarray(g.node["xyzr"][:, 3], dtype=np.float64)).to(d.device)
    nb = L.gtf_tag_workspace_bytes(g.n_nodes, g.n_edges)
    ws = torch.full((nb,), 0xFF, dtype=torch.uint8, device=d.device)   # no zeroing needed
    flips = (ctypes.c_int32 * 64)()
    sweeps = ctypes.c_int32(-1)
    nat.check(L.gtf_tag_propagate(ctypes.byref(d.cg), ctypes.c_void_p(radius.data_ptr()),
                                  ctypes.c_void_p(tags.data_ptr()), 0.1, max_sweeps,
                                  ctypes.cast(flips, ctypes.c_void_p), ctypes.byref(sweeps),
                                  ctypes.c_void_p(ws.data_ptr()), nb, d.stream))
    torch.cuda.synchronize()
    want = list(extra["flips"])[:max_sweeps]
    assert sweeps.value == len(want) and list(flips[:sweeps.value]) == want
    # the same number of single sweeps (gtf_tag_sweep), host loop
    keep = torch.zeros(max(g.n_edges, 1), dtype=torch.uint8, device=d.device)
    proc = torch.zeros(max(g.n_nodes, 1), dtype=torch.uint8, device=d.device)
    cnt = torch.zeros(2, dtype=torch.int32, device=d.device)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    ta, tb = torch.from_numpy(t0).to(d.device), torch.empty(g.n_nodes, dtype=torch.int64, device=d.device)
    nat.check(L.gtf_tag_prepare(ctypes.byref(d.cg), vp(radius), vp(keep), vp(proc), vp(cnt), d.stream))
    for _ in range(len(want)):
        nat.check(L.gtf_tag_sweep(ctypes.byref(d.cg), vp(keep), vp(proc), vp(ta), vp(tb), vp(cnt[1:2]), d.stream))
        ta, tb = tb, ta
    torch.cuda.synchronize()
    assert torch.equal(tags, ta)


def _chain_graph(n):
    """n nodes, edges u -> u + 1, radius falling along the chain and tag[u] = u: every sweep
    carries the largest tag one hop down, so the stage runs n sweeps with flips n-1, ..., 1, 0
    (flip threshold 0)"""
    from gtf.graph import TrackGraph, NODE_FIELDS, SLOT_FIELDS, empty_arrays
    node = empty_arrays(NODE_FIELDS, n)
    slot = empty_arrays(SLOT_FIELDS, n - 1)
    node["gnn"][:] = 1.0
    node["xyzr"][:] = 1.0
    node["xyzr"][:, 3] = np.arange(n, 0, -1, dtype=np.float64)
    node["tag"][:] = np.arange(n)
    node["layer"][:] = np.arange(n) % 7
    slot["slot_src"][:] = np.arange(n - 1)
    slot["slot_key"][:] = np.arange(n - 1)
    slot["is_edge"][:] = 1
    slot["act"][:] = 1
    slot_ptr = np.concatenate([[0], np.arange(n - 1)]).astype(np.int32)
    slot_ptr = np.concatenate([slot_ptr, [n - 1]]).astype(np.int32)
    out_ptr = np.concatenate([np.arange(n), [n - 1]]).astype(np.int32)
    return TrackGraph(n, n - 1, slot_ptr, out_ptr, np.arange(n - 1, dtype=np.int32), node, slot)


@pytest.mark.parametrize("csr", list(_CSR_MODES))
@pytest.mark.parametrize("poll", ["1", "0"])
@pytest.mark.parametrize("schedule", [True, False])
def test_tag_propagate_long_run(schedule, poll, csr, monkeypatch):
    """300 sweeps in one gtf_tag_propagate call: batches of 2 .. 64 launches, the flip-counter
    ring (128 sweeps) wrapped twice with every sweep zeroing the next one's counters"""
    monkeypatch.setenv("GTF_TAG_POLL", poll)
    _csr_env(monkeypatch, csr)
    import ctypes
    import torch
    from gtf import _native as nat
    from gtf.device import DeviceGraph
    n = 300
    g = _chain_graph(n)
    d = DeviceGraph(g, schedule=schedule)
    L = d.lib
    tags = torch.arange(n, dtype=torch.int64, device=d.device)
    radius = torch.from_numpy(np.ascontiguousarray(g.node["xyzr"][:, 3])).to(d.device)
    nb = L.gtf_tag_workspace_bytes(g.n_nodes, g.n_edges)
    ws = torch.full((nb,), 0xFF, dtype=torch.uint8, device=d.device)
    flips = (ctypes.c_int32 * 512)()
    sweeps = ctypes.c_int32(-1)
    nat.check(L.gtf_tag_propagate(ctypes.byref(d.cg), ctypes.c_void_p(radius.data_ptr()),
                                  ctypes.c_void_p(tags.data_ptr()), 0.0, 512,
                                  ctypes.cast(flips, ctypes.c_void_p), ctypes.byref(sweeps),
                                  ctypes.c_void_p(ws.data_ptr()), nb, d.stream))
    torch.cuda.synchronize()
    want_tags, want_flips = O.tag_propagation(g, 0.0)
    assert want_flips == list(range(n - 1, -1, -1))
    assert sweeps.value == len(want_flips) and list(flips[:sweeps.value]) == want_flips
    assert np.array_equal(tags.cpu().numpy(), want_tags)


@pytest.mark.parametrize("shape", ["all_wide", "one_wide", "negative"])
def test_tag_propagate_tags_beyond_int32(shape, monkeypatch):
    """tags that do not fit 32 bits (the int64 of the reference's tag arrays): the compact-list
    sweeps carry int32 tags only while every value fits, so a shift by 2^40 of every tag, one
    wide tag alone (its kept predecessors take it from the first sweep on) and tags shifted
    below -2^31 give the keep-mask sweeps' (GTF_TAG_CSR=0) flips and tags word for word, and
    the shifted ones the reference's flips and shifted tags"""
    import ctypes
    import torch
    from gtf import _native as nat
    g, _, extra, _ = load("tags_vol7")
    d = _dev(g)
    L = d.lib
    t0 = np.ascontiguousarray(g.node["tag"], dtype=np.int64)
    if shape == "all_wide":
        t0 = t0 + (1 << 40)
    elif shape == "negative":
        t0 = t0 - (1 << 40)
    else:
        t0 = t0.copy()
        t0[int(np.argmax(t0))] = 1 << 40
    radius = torch.from_numpy(np.ascontiguousarray(g.node["xyzr"][:, 3], dtype=np.float64)).to(d.device)
    nb = L.gtf_tag_workspace_bytes(g.n_nodes, g.n_edges)
    res = {}
    for csr, mode in (("1", "default"), ("n2", "packed_n2"), ("n4", "packed_n4"), ("p1", "packed_prep1"),
                      ("u2", "unpacked_n2"), ("l2", "packed_n2_lanes"), ("c1", "coop1"), ("c4", "coop4"),
                      ("ct", "counts_thread_prep"), ("0", "mask")):
        _csr_env(monkeypatch, mode)
        tags = torch.from_numpy(t0).to(d.device)
        ws = torch.full((nb,), 0xFF, dtype=torch.uint8, device=d.device)
        flips = (ctypes.c_int32 * 64)()
        sweeps = ctypes.c_int32(-1)
        nat.check(L.gtf_tag_propagate(ctypes.byref(d.cg), ctypes.c_void_p(radius.data_ptr()),
                                      ctypes.c_void_p(tags.data_ptr()), 0.1, 64,
                                      ctypes.cast(flips, ctypes.c_void_p), ctypes.byref(sweeps),
                                      ctypes.c_void_p(ws.data_ptr()), nb, d.stream))
        torch.cuda.synchronize()
        res[csr] = (list(flips[:sweeps.value]), tags.cpu().numpy())
    for m in ("1", "n2", "n4", "p1", "u2", "l2", "c1", "c4", "ct"):   # (every compact-list form, its int64 fallback included)
        assert res[m][0] == res["0"][0]
        assert np.array_equal(res[m][1], res["0"][1])
    if shape != "one_wide":   # (a shift changes no comparison)
        assert res["1"][0] == list(extra["flips"])
        off = (1 << 40) if shape == "all_wide" else -(1 << 40)
        kept = extra["tags"] >= 0
        assert np.array_equal(res["1"][1][kept], extra["tags"][kept] + off)


_ORACLE_CACHE = {}


def _star_graph(k, r0):
    """node 0 sends to nodes 1..k (one slot each), receiver radius 1..k against node 0's r0:
    the receivers at or inside r0 are kept; receiver v also sends to v + 1 (a chain behind the
    star, so the maximum travels several sweeps)"""
    from gtf.graph import TrackGraph, NODE_FIELDS, SLOT_FIELDS, empty_arrays
    n = k + 1
    src = np.concatenate([np.zeros(k, np.int64), np.arange(1, k)])        # star, then chain v -> v + 1
    dst = np.concatenate([np.arange(1, k + 1), np.arange(2, k + 1)])
    order = np.lexsort((src, dst))   # slots grouped by receiver
    src, dst = src[order], dst[order]
    ns = src.size
    node = empty_arrays(NODE_FIELDS, n)
    slot = empty_arrays(SLOT_FIELDS, ns)
    node["gnn"][:] = 1.0
    node["xyzr"][:] = 1.0
    node["xyzr"][1:, 3] = np.arange(k, 0, -1, dtype=np.float64)   # v -> v + 1 kept: radius falls
    node["xyzr"][0, 3] = r0
    node["tag"][:] = np.random.default_rng(5).permutation(n)
    node["layer"][:] = np.arange(n) % 7
    slot["slot_src"][:] = src
    slot["slot_key"][:] = np.arange(ns)
    slot["is_edge"][:] = 1
    slot["act"][:] = 1
    slot_ptr = np.searchsorted(dst, np.arange(n + 1)).astype(np.int32)
    eo = np.lexsort((dst, src))      # out-edges grouped by sender
    out_ptr = np.searchsorted(src[eo], np.arange(n + 1)).astype(np.int32)
    return TrackGraph(n, ns, slot_ptr, out_ptr, eo.astype(np.int32), node, slot)


@pytest.mark.parametrize("csr", list(_CSR_MODES))
@pytest.mark.parametrize("schedule", [True, False])
@pytest.mark.parametrize("kept", [700, 300])
def test_tag_propagate_saturated_kept_count(schedule, csr, kept, monkeypatch):
    """a node with 1,200 out-edges, 700 of them kept: past the packed word's 511 (the count then
    read from its own word), or 300: more than the cooperative sweep stages for one 64-node group
    (its per-lane loop); on the lane-group and thread-per-node prepare kernels; the tags and flips
    equal the oracle's"""
    _csr_env(monkeypatch, csr)
    import torch
    from gtf.device import DeviceGraph
    g = _star_graph(1200, kept + 0.5)
    d = DeviceGraph(g, schedule=schedule)
    tags = torch.from_numpy(np.ascontiguousarray(g.node["tag"], dtype=np.int64)).to(d.device)
    radius = torch.from_numpy(np.ascontiguousarray(g.node["xyzr"][:, 3])).to(d.device)
    flips = d.tag_propagation_dev(tags, radius, threshold=0.0, max_sweeps=5000)
    if kept not in _ORACLE_CACHE:   # (~1,000 sweeps of the Python oracle: once per module and size)
        _ORACLE_CACHE[kept] = O.tag_propagation(g, 0.0)
    want_tags, want_flips = _ORACLE_CACHE[kept]
    assert flips == list(want_flips) and len(flips) > 2
    assert np.array_equal(tags.cpu().numpy(), want_tags)


def test_workspace_init_contract():
    """a workspace that was not allocated zeroed (filled with 0xFF here: every gtf_diag
    pointer garbage) is usable after gtf_workspace_init, as include/gtf.h documents"""
    import ctypes
    import torch
    from gtf import _native as nat
    g, out, extra, meta = load("pass_full")
    exp = expected_graph(g, out)
    p = _params(meta)
    d = _dev(g)
    d.t["ws"].fill_(0xFF)
    nat.check(d.lib.gtf_workspace_init(d.ptr("ws"), d.stream))
    d.full_pass(p)
    d.raise_errors()
    got = d.download(g.copy())
    errs = compare(got, exp, rtol=RTOL, atol=1e-12)
    assert errs == [], "\n".join(errs)
    ws = d.t["ws"][:256].cpu().numpy()
    assert not ws[nat.DIAG_OFFSET:nat.DIAG_OFFSET + ctypes.sizeof(nat.GtfDiag)].any()


def test_live_coordinates_equal_stored():
    """the updated states' 'xyzr' kept live in gnn (gtf_states.fresh bit 1: k_extrapolate
    does not write the snapshot) against the same passes with the snapshot materialised
    between them (download -> gtf_uts_materialize, the stored path of every reader): two
    fused passes, bit for bit, and the downloaded xyzr equal to the senders' coordinates"""
    g, out, extra, meta = load("pass_full")
    p = _params(meta)
    a, b = _dev(g), _dev(g)
    for d in (a, b):
        d.clear_errors()
    a.full_pass(p)
    a.full_pass(p)                        # pass 2 reads pass 1's entries live
    b.full_pass(p)
    b.download(g.copy())                  # materialises: pass 2 reads them stored
    b.full_pass(p)
    ga, gb = a.download(g.copy()), b.download(g.copy())
    assert a.errors() == 0 and b.errors() == 0
    errs = compare(ga, gb, rtol=0.0, atol=0.0)
    assert errs == [], "\n".join(errs)
    pres = (ga.slot["uts_rank"] >= 0) & (ga.slot["slot_src"] >= 0)
    src = ga.slot["slot_src"][pres]
    assert pres.sum() > 100
    assert np.array_equal(ga.slot["uts_xyzr"][pres], ga.node["gnn"][src])
