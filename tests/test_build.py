"""gtf_build_event_csr (native event conversion) against the
reference's construction through networkx + pack() (CPU; host code, no GPU).

The native builder must reproduce every order networkx produces -- component order,
node order inside each subgraph copy (CPython set order for components smaller than
half the graph), successor order, and the track_state_estimates key order
reversed(set(all_neighbors)) -- so the packed arrays are compared for equality."""
import os

import numpy as np
import pytest

from fixtures import GOLDEN
from gtf.graph import NODE_FIELDS, SLOT_FIELDS


def _equal(g1, v1, g2, v2):
    assert (g1.n_nodes, g1.n_slots, g1.n_edges, g1.n_subgraphs) == (g2.n_nodes, g2.n_slots, g2.n_edges,
                                                                      g2.n_subgraphs)
    for k in ("slot_ptr", "out_ptr", "out_slot"):
        assert np.array_equal(getattr(g1, k), getattr(g2, k)), k
    for fields, a, b in ((NODE_FIELDS, g1.node, g2.node), (SLOT_FIELDS, g1.slot, g2.slot)):
        for k in fields:
            assert np.array_equal(a[k], b[k], equal_nan=a[k].dtype.kind == "f"), k
    assert np.array_equal(v1, v2)


def _both(prefix, lo, hi):
    from gtf.pipeline import event_layout
    return event_layout(prefix, lo, hi, "native") + event_layout(prefix, lo, hi, "networkx")


def test_native_build_matches_networkx_vol7():
    _equal(*_both(os.path.join(GOLDEN, "kat134", "event_1_filtered_graph_"), 7, 7))


def _write_event(d, seed, n, rows, id_space, chain_frac):
    rng = np.random.default_rng(seed)
    ids = rng.choice(id_space, size=n, replace=False).astype(np.int64)
    layer = rng.integers(7, 10, n) * 1000 + rng.integers(2, 14, n)
    xyz = rng.normal(0, 300, (n, 3)).round(4)
    with open(os.path.join(d, "ev_nodes.csv"), "w") as f:
        f.write("node_idx,layer_id,x,y,z\n")
        for i in range(n):
            f.write("%d,%d,%r,%r,%r\n" % (ids[i], layer[i], float(xyz[i, 0]), float(xyz[i, 1]), float(xyz[i, 2])))
    # a long chain (one big component) plus random local edges, duplicates, self loops
    # and rows naming nodes outside the node file
    m = int(n * chain_frac)
    e = [(ids[i], ids[i + 1]) for i in range(m - 1)]
    for _ in range(rows):
        i = int(rng.integers(0, n))
        j = int(min(n - 1, max(0, i + rng.integers(-6, 7))))
        e.append((ids[i], ids[j]))
    e += e[:: max(1, len(e) // 50)]                          # duplicate rows
    e += [(ids[0], 10 ** 7 + 5), (10 ** 7 + 6, ids[1])]      # unknown ends are dropped
    order = rng.permutation(len(e))
    with open(os.path.join(d, "ev_edges.csv"), "w") as f:
        f.write("%d %d\n" % (n, len(e)))
        f.write("node2,node1,weight\n")
        for k in order:
            f.write("%d,%d,1.0\n" % (e[k][1], e[k][0]))
    return os.path.join(d, "ev_")


@pytest.mark.parametrize("seed,n,rows,space,chain", [(0, 400, 300, 10 ** 6, 0.0), (1, 3000, 4000, 5000, 0.0),
                                                     (2, 2000, 1500, 10 ** 6, 0.7), (3, 5000, 9000, 2 ** 40, 0.3)])
def test_native_build_matches_networkx_synthetic(tmp_path, seed, n, rows, space, chain):
    prefix = _write_event(str(tmp_path), seed, n, rows, space, chain)
    _equal(*_both(prefix, 7, 8))


def test_native_build_empty(tmp_path):
    prefix = _write_event(str(tmp_path), 4, 50, 40, 1000, 0.0)
    from gtf import io
    g, v = io.build_event_csr(prefix, 20, 21)          # no node in the volume window
    assert g.n_nodes == 0 and g.n_slots == 0 and v.shape == (0, 2)
