"""The batched benchmark configs on the GPU (BASELINE configs[2] and configs[4]).

C3: 64 C2-like events fused into one CSR (gtf.graph.concat, node / slot offsets). The
fused pass must equal the 64 per-event passes bit for bit (events never share an edge,
so the fusion is a pure relabelling), and two of the events must match the oracle
(masks exact except perturbation-undetermined decisions, floats within 1e-6 + 100x noise,
tests/compare.py).

C5: 256 copies of the committed volume-7 134 event (gtf.parabolic.batch) through
gtf_parabolic_kl. Every copy's rows must equal the single-event path's rows for that
copy bit for bit, and copy 0 (unjittered) must reproduce the reference's committed
training CSV (kl within 1e-8, emp_var 1e-9, truth exact).
"""
import numpy as np
import pytest

import gtf_oracle as O
from compare import compare_noise, noise_envelope
from gtf import synth
from gtf.graph import concat
from gtf.params import Params

pytestmark = pytest.mark.gpu

N_C3 = 64


def _state_arrays(g):
    from test_gpu_fullsize import _state_keys
    return {k: v for k, v in list(g.node.items()) + list(g.slot.items()) if k in _state_keys(g)}


def _pass(g, p, layout="natural"):
    from gtf.device import DeviceGraph
    d = DeviceGraph(g, layout=layout)
    d.clear_errors()
    d.full_pass(p)
    return d.download(g.copy()), d.errors()


@pytest.fixture(scope="module")
def c3_events():
    return [synth.event(s, synth.C2_TRACKS, synth.C2_FAKE) for s in range(N_C3)]


def test_c3_fused_equals_per_event(c3_events):
    p = Params()
    events = c3_events
    fused = concat(events)
    assert fused.n_edges > 5_000_000
    got, flags = _pass(fused, p, layout="tiled")
    assert flags == 0
    noff = np.cumsum([0] + [e.n_nodes for e in events])
    soff = np.cumsum([0] + [e.n_slots for e in events])
    a = _state_arrays(got)
    for i, ev in enumerate(events):
        one, f1 = _pass(ev, p)
        assert f1 == 0
        b = _state_arrays(one)
        for k in b:
            part = a[k][noff[i]:noff[i + 1]] if k in got.node else a[k][soff[i]:soff[i + 1]]
            x, y = np.asarray(part).reshape(-1), np.asarray(b[k]).reshape(-1)
            same = (x == y) | ((x != x) & (y != y)) if x.dtype.kind == "f" else x == y
            assert same.all(), "event %d: %s differs in %d entries" % (i, k, int((~same).sum()))


@pytest.mark.parametrize("i", [0, 37])
def test_c3_event_matches_oracle(c3_events, i):
    p = Params()
    ev = c3_events[i]
    one, flags = _pass(ev, p)
    assert flags == 0

    def run(x):
        O.full_pass(x, p, tie_policy="stop")
        return x
    ref, noise, fl = noise_envelope(run, ev)
    errs, stats = compare_noise(one, ref, noise, fl)
    print("C3 event %d: %d edges, %s" % (i, ev.n_edges, stats))
    assert errs == [], "\n".join(errs)
    assert stats["mask_undetermined"] <= 0.001 * ev.n_edges


def test_c5_batch_equals_single_event_rows_and_kat():
    from gtf import parabolic
    from test_kat_parabolic import kat_event, kat_rows, sorted_rows
    g, truth = kat_event()
    ptr, src = parabolic.in_edge_csr(g)
    n_ev = 256
    bptr, bsrc, bgnn, btr = parabolic.batch(ptr, src, g.node["gnn"], truth, n_ev)
    node, i, j, kl, ev, tr = parabolic.training_rows_csr(bptr, bsrc, bgnn, btr)
    N = g.n_nodes
    per = kl.size // n_ev
    assert per * n_ev == kl.size == 256 * 7574
    for e in (0, 1, 100, 255):
        one = parabolic.training_rows_csr(ptr, src, bgnn[e * N:(e + 1) * N], truth)
        sl = slice(e * per, (e + 1) * per)
        assert np.array_equal(node[sl] - e * N, one[0])
        assert np.array_equal(kl[sl], one[3]) and np.array_equal(ev[sl], one[4]) and np.array_equal(tr[sl], one[5])
    kat = kat_rows()
    a = sorted_rows(kl[:per], ev[:per], tr[:per].astype(np.float64))
    b = sorted_rows(kat["kl_dist"], kat["emp_var"], kat["truth"])
    assert (np.abs(a[0] - b[0]) <= 1e-8 * np.abs(b[0])).all()
    assert (np.abs(a[1] - b[1]) <= 1e-9 * np.abs(b[1])).all()
    assert (a[2] == b[2]).all()


def test_c5_fp32_envelope_256_events():
    """config 5's fp32 mode on the whole 256-event batch (the fp64-vs-fp32
    tolerance sweep): against the fp64 kernel, median relative KL error < 1e-5, 99th
    percentile < 1e-3, no decision flip at k in {1, 2, 10, 100} and identical pair truth
    flags. (The largest relative errors sit on near-zero distances, where fp32's absolute
    error is what a threshold sees: the flip counts are the bar there, not the maximum.)"""
    import torch
    from gtf import parabolic
    from test_kat_parabolic import kat_event
    g, truth = kat_event()
    ptr, src = parabolic.in_edge_csr(g)
    bptr, bsrc, bgnn, btr = parabolic.batch(ptr, src, g.node["gnn"], truth, 256)
    k = parabolic.ParabolicKL(bptr, bsrc, bgnn, btr, "cuda", ordered=True)
    o64, o32 = k.alloc("f64", emp="var"), k.alloc("f32", emp="var")
    k.run(o64, "f64")
    k.run(o32, "f32")
    torch.cuda.synchronize()
    assert k.errors() == 0
    a = o64["kl"].double().cpu().numpy()
    b = o32["kl"].double().cpu().numpy()
    assert a.size == 256 * 7574
    rel = np.abs(b - a) / np.maximum(np.abs(a), 1e-300)
    p50, p99 = np.percentile(rel, 50), np.percentile(rel, 99)
    flips = {t: int(((a < t) != (b < t)).sum()) for t in (1.0, 2.0, 10.0, 100.0)}
    print("fp32 vs fp64 over %d pairs: median %.3g, p99 %.3g, max %.3g, flips %s" % (a.size, p50, p99, rel.max(), flips))
    assert p50 < 1e-5 and p99 < 1e-3
    assert all(v == 0 for v in flips.values()), flips
    assert torch.equal(o64["truth"], o32["truth"])
