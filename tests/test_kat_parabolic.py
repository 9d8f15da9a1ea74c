"""Known-answer test of the parabolic-model state + pairwise KL distance (§8 a17).

The reference's committed training file
learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/
minCurv_0.3_134/event_graph_data/1_events_training_data.csv holds 7,574 KL
distances its own code computed on the volume-7 graph of the committed
minCurv_0.3_134 event (extract_metadata_trackml_parabolic_model.py:15-99). The
CSV and the event graph are copied into tests/golden/ (data files, not source).
The oracle's restatement must reproduce the sorted distance list.
"""
import os

import numpy as np
import pytest

import gtf_oracle as O
from fixtures import GOLDEN
from gtf import io


def _event():
    return io.load_event(os.path.join(GOLDEN, "kat134", "event_1_filtered_graph_"), 7, 7)


def _oracle_pairs(g):
    gnn = g.node["gnn"]
    src = g.slot["slot_src"]
    out = []
    for v in range(g.n_nodes):
        lo, hi = g.slot_ptr[v], g.slot_ptr[v + 1]
        if hi - lo <= 1:                 # query_node_degree_in_edges <= 1 -> skipped (:61-62)
            continue
        st = O.parabolic_states(gnn[v], gnn[src[lo:hi]])
        out.extend(O.parabolic_kl_pairs([s for s, _ in st], [c for _, c in st]))
    return np.asarray(out)


def test_parabolic_kl_matches_committed_training_csv():
    kat = np.genfromtxt(os.path.join(GOLDEN, "kat134", "1_events_training_data.csv"), delimiter=",",
                        names=True)["kl_dist"]
    got = _oracle_pairs(_event())
    assert got.size == kat.size == 7574
    a, b = np.sort(got), np.sort(kat)
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    assert rel.max() < 1e-8, rel.max()
