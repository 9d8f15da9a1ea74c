"""Full-size checks on the benchmark workload (BASELINE configs[3], C4: ~180k hits,
~1.0M directed edges) through size-independent properties -- the oracle takes
minutes per pass at this size, so parity there is pinned at smaller sizes
(test_gpu_synthetic.py, test_gpu_parity.py) and these tests hold the full-size path
to the same results by construction:

  * the fused pass (gtf_pass: one node launch for every node-local op) equals the
    three stage entry points run one after the other (gtf_extrapolate -> gtf_update
    -> gtf_cluster, one launch per stage), bit for bit;
  * both equal the run-time op interpreter (gtf_node_ops, k_node_group), the
    thread-per-node implementation (no schedule, k_node), the packed variable-size lane
    segments (k_node_pack) and the pass on nodes renumbered into schedule order, which
    restate the same reference functions with different code or data order;
  * a pass is deterministic (two runs from the same input, bit-identical);
  * activations only switch off (reweight and clustering never re-activate an edge).
"""
import numpy as np
import pytest

from gtf import synth
from gtf.params import Params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c4():
    return synth.workload("c4", seed=0)


def _state(d):
    """every array a pass may write (DeviceGraph.snapshot's default set), with the live state
    coordinates materialised as download() does (gtf_uts_materialize; fresh bit 0)"""
    d.materialize()
    out = {k: v.cpu().numpy().reshape(-1) for k, v in d.snapshot().items()}
    out["uts_fresh"] = out["uts_fresh"] & 1
    return out


def _state_keys(g):
    from gtf.device import MUTABLE_NODE, STATIC_SLOT
    return set(MUTABLE_NODE) | {k for k in g.slot if k not in STATIC_SLOT and k != "slot_key"}


def _same(a, b, what):
    assert a.keys() == b.keys()
    for k in a:
        x, y = np.asarray(a[k]).reshape(-1), np.asarray(b[k]).reshape(-1)
        if x.dtype.kind == "f":
            eq = (x == y) | (np.isnan(x) & np.isnan(y))
        else:
            eq = x == y
        assert eq.all(), "%s: %s differs in %d of %d entries" % (what, k, int((~eq).sum()), eq.size)


def _run(g, how, p):
    from gtf.device import DeviceGraph
    if how in ("schedule_layout", "tiled_layout", "padded_layout", "packed"):   # renumbered nodes (results mapped back) / packed
        d = (DeviceGraph(g, layout=how.split("_")[0]) if how.endswith("_layout") else DeviceGraph(g, pack=True))
        d.clear_errors()
        d.full_pass(p)
        got = d.download(g.copy())
        return ({k: v for k, v in list(got.node.items()) + list(got.slot.items()) if k in _state_keys(g)},
                d.errors())
    d = DeviceGraph(g, schedule=(how != "thread_per_node"))
    d.clear_errors()
    if how in ("fused", "thread_per_node"):
        d.full_pass(p)
    elif how == "stages":
        d.extrapolate(p)
        d.update(p)
        d.cluster("uts", p.cluster_chi2, p.cluster_kl, p)
    elif how == "interpreter":
        d.message_passing(p)
        # "fresh" and "ranks" again: both are idempotent right after message passing, and this
        # runs the interpreter's own OP_FRESH / OP_RANKS code
        d.node_ops(["fresh", "ranks", "priors_uts", "reweight_uts", "priors_uts", "reweight_uts", "degree", "prune", "priors_tse",
                    "priors_uts", "reweight_uts"], p)
        d.node_ops(["cluster_uts", "degree", "mw_uts", "priors_uts"], p, p.cluster_chi2, p.cluster_kl)
    d.torch.cuda.synchronize()
    return _state(d), d.errors()


def test_fused_pass_equals_stagewise_and_other_implementations(c4):
    p = Params()
    ref, ref_flags = _run(c4, "fused", p)
    assert ref["act"].sum() > 0 and ref["has_merged"].sum() > 0
    for how in ("stages", "interpreter", "thread_per_node", "schedule_layout", "tiled_layout", "padded_layout", "packed"):
        got, flags = _run(c4, how, p)
        assert flags == ref_flags, how
        _same(got, ref, how)


def test_pass_is_deterministic_and_only_deactivates(c4):
    from gtf.device import DeviceGraph
    p = Params()
    d = DeviceGraph(c4)
    act0 = d.t["act"].cpu().numpy().copy()
    snap = d.snapshot(DeviceGraph.PASS_INPUTS)
    d.full_pass(p)
    first = _state(d)
    d.restore(snap)
    d.full_pass(p)
    _same(_state(d), first, "second run")
    assert np.all(first["act"] <= act0), "an edge was re-activated"


def test_staged_input_copies_equal_the_resident_pass(c4):
    """bench.py's steps run on staged copies of the pass-input arena (DeviceGraph.stage_inputs):
    a pass on copy i leaves copy i exactly as a pass on the resident arrays leaves them,
    and the other copies untouched"""
    from gtf.device import DeviceGraph
    p = Params()
    d = DeviceGraph(c4, layout="tiled")
    snap = d.snapshot(DeviceGraph.PASS_INPUTS)
    d.stage_inputs(3)
    d.fill_inputs(snap)
    d.clear_errors()
    d.use_inputs(1)
    d.full_pass(p)
    d.use_inputs(None)
    d.full_pass(p)
    assert d.errors() == 0
    import torch
    assert torch.equal(d._staged[1][0], d.arena)
    assert torch.equal(d._staged[0][0], snap["__arena__"]) and torch.equal(d._staged[2][0], snap["__arena__"])
    assert not torch.equal(d.arena, snap["__arena__"])


@pytest.mark.parametrize("variant", ["no_sxzr", "no_static32", "no_classes"])
def test_slot_tables_do_not_change_the_pass(c4, variant, monkeypatch):
    """the graph-static slot tables (gtf_graph.slot_class / slot_xclass / slot_static /
    slot_sxzr, ABI v5 / v7) only move where the node kernel reads things from: the C4 pass
    without each of them (the kernel then gathers the senders' coordinates, reads the four
    static fields, or builds every class itself) equals the default pass bit for bit"""
    from gtf.device import DeviceGraph
    p = Params()
    d = DeviceGraph(c4, layout="tiled")
    assert d.use_sxzr and d.use_static32 and d.use_classes
    d.clear_errors()
    d.full_pass(p)
    h = d.download(c4.copy())
    ref = {k: v for k, v in list(h.node.items()) + list(h.slot.items()) if k in _state_keys(c4)}
    flags = d.errors()
    if variant == "no_sxzr":
        monkeypatch.setenv("GTF_NO_SXZR", "1")
    elif variant == "no_static32":
        monkeypatch.setenv("GTF_NO_STATIC32", "1")
    e = DeviceGraph(c4, layout="tiled", classes=(False if variant == "no_classes" else None))
    assert (e.use_sxzr, e.use_static32, e.use_classes) == {"no_sxzr": (False, True, True),
                                                           "no_static32": (True, False, True),
                                                           "no_classes": (False, False, False)}[variant]
    e.clear_errors()
    e.full_pass(p)
    h = e.download(c4.copy())
    got = {k: v for k, v in list(h.node.items()) + list(h.slot.items()) if k in _state_keys(c4)}
    assert e.errors() == flags
    _same(got, ref, variant)


@pytest.mark.parametrize("order", ["ascending", "descending"])
def test_c3_tag_stage_forms_agree(order, monkeypatch):
    """gtf_tag_propagate on configs[2] (C3: 64 C2-like events fused, 2.0 M nodes / 5.9 M edges,
    after one pass) -- the size where the stage's defaults are the packed kept lists and the
    wave-cooperative sweep (two 64-node groups per wave) -- against the per-lane sweep on the
    same packed lists (GTF_TAG_COOP=0), the lists at the out-range fronts (GTF_TAG_PACK=0) and
    the keep-mask sweeps of gtf_tag_sweep (GTF_TAG_CSR=0): the same flips, sweep count and tags
    word for word, from ascending (one sweep) and descending (several) initial tags"""
    import torch
    from gtf.device import DeviceGraph
    g = synth.workload("c3", seed=0)
    d = DeviceGraph(g, layout="tiled")
    d.full_pass(Params())
    rad = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(g.node["xyzr"][:, 3]))).to(d.device)
    t = np.arange(g.n_nodes, dtype=np.int64)
    if order == "descending":
        t = t[::-1].copy()
    t0 = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(t))).to(d.device)
    res = {}
    for name, env in (("default", {}), ("lanes", {"GTF_TAG_COOP": "0"}), ("unpacked", {"GTF_TAG_PACK": "0"}),
                      ("mask", {"GTF_TAG_CSR": "0"})):
        for k in ("GTF_TAG_CSR", "GTF_TAG_PACK", "GTF_TAG_COOP"):
            monkeypatch.setenv(k, env.get(k, ""))
        ta = t0.clone()
        flips = d.tag_propagation_dev(ta, rad)
        torch.cuda.synchronize()
        res[name] = (list(flips), ta.cpu())
    assert len(res["default"][0]) >= (2 if order == "descending" else 1)
    for name in ("lanes", "unpacked", "mask"):
        assert res[name][0] == res["default"][0], name
        assert torch.equal(res[name][1], res["default"][1]), name
