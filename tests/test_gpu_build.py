"""gtf_build_event_csr_device -- event conversion's graph build on the GPU (SURVEY §8f
#2) -- against the host builder gtf_build_event_csr, which tests/test_build.py pins to
the reference's networkx construction and tests/test_real800.py to the reference's own
packed 800' network (structure digest). The device build must give the same arrays bit
for bit: node order (CPython set order for components under half the graph), subgraph
ids, slots, successor order and the track_state_estimates key order.

Inputs: the committed vol-7 134 event, the 800' all-volume event, the synthetic CSV
events of test_build.py (duplicates, self loops, unknown ends, a component over half the
graph, a dense id space) and a C4-sized edge list (1M directed edges) from the synthetic
generator's graph."""
import os

import numpy as np
import pytest

import real800 as R
from fixtures import GOLDEN
from gtf import io, synth
from test_build import _equal, _write_event

pytestmark = pytest.mark.gpu

KEYS = ("order", "sub_id", "slot_ptr", "slot_src", "tse_rank", "out_ptr", "out_slot")


def _both_builders(prefix, lo, hi):
    return io.build_event_csr(prefix, lo, hi) + io.build_event_csr(prefix, lo, hi, device="cuda")


def test_device_build_vol7():
    _equal(*_both_builders(os.path.join(GOLDEN, "kat134", "event_1_filtered_graph_"), 7, 7))


def test_device_build_800_all_volumes():
    g, v = io.build_event_csr(R.PREFIX, *R.VOLS, device="cuda")
    assert g.n_nodes == 29590 and g.n_edges == 89028
    assert R.structure_digest(g) == str(R.fixture("pass")["structure_sha"])
    _equal(g, v, *io.build_event_csr(R.PREFIX, *R.VOLS))


@pytest.mark.parametrize("seed,n,rows,space,chain", [(0, 400, 300, 10 ** 6, 0.0), (1, 3000, 4000, 5000, 0.0),
                                                     (2, 2000, 1500, 10 ** 6, 0.7), (3, 5000, 9000, 2 ** 40, 0.3)])
def test_device_build_synthetic(tmp_path, seed, n, rows, space, chain):
    _equal(*_both_builders(_write_event(str(tmp_path), seed, n, rows, space, chain), 7, 8))


def _rows_of(g, seed):
    """the undirected edges of a packed graph as shuffled CSV rows, random node ids"""
    rng = np.random.default_rng(seed)
    dst = np.repeat(np.arange(g.n_nodes), np.diff(g.slot_ptr))
    src = g.slot["slot_src"]
    keep = (src >= 0) & (src < dst)
    a, b = src[keep], dst[keep]
    perm = rng.permutation(a.size)
    flip = rng.random(a.size) < 0.5
    a, b = np.where(flip, b, a)[perm], np.where(flip, a, b)[perm]
    ids = rng.choice(2 ** 40, size=g.n_nodes, replace=False).astype(np.int64)
    return ids, ids[a], ids[b]


@pytest.mark.parametrize("workload", ["c2", "c4"])
def test_device_build_generator_sized(workload):
    g = synth.workload(workload, seed=3)
    ids, a, b = _rows_of(g, 5)
    oh, eh, sh = io.csr_from_rows(ids, a, b)
    od, ed, sd = io.csr_from_rows(ids, a, b, device="cuda")
    assert (eh, sh) == (ed, sd) and eh == 2 * a.size
    for k in KEYS:
        n = {"slot_src": eh, "tse_rank": eh, "out_slot": eh}.get(k, oh[k].size)
        assert np.array_equal(oh[k][:n], od[k][:n]), k


def test_device_build_rejects_duplicate_ids():
    ids = np.array([5, 7, 5], np.int64)
    with pytest.raises(RuntimeError, match="duplicate"):
        io.csr_from_rows(ids, np.array([5], np.int64), np.array([7], np.int64), device="cuda")


def test_device_build_no_edges():
    ids = np.array([9, 3, 4], np.int64)
    o, e, s = io.csr_from_rows(ids, np.zeros(0, np.int64), np.zeros(0, np.int64), device="cuda")
    oh, eh, sh = io.csr_from_rows(ids, np.zeros(0, np.int64), np.zeros(0, np.int64))
    assert (e, s) == (eh, sh) == (0, 3)
    for k in ("order", "sub_id", "slot_ptr", "out_ptr"):
        assert np.array_equal(o[k], oh[k]), k
