"""Known-answer test of the parabolic-model state + pairwise KL distance (§8 a17).

The reference's committed training file
learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/
minCurv_0.3_134/event_graph_data/1_events_training_data.csv holds 7,574
(kl_dist, emp_var, truth) rows its own code computed on the volume-7 graph of the
committed minCurv_0.3_134 event (extract_metadata_trackml_parabolic_model.py:15-99).
tests/golden/make_kat134.py copies the CSV, the volume-7 node/edge rows and the
node truth into tests/golden/kat134/ (data files, not source). The oracle's
restatement must reproduce the rows as a multiset (the reference's row order
follows glob() file order).
"""
import os

import numpy as np

import gtf_oracle as O
from fixtures import GOLDEN
from gtf import io

KAT = os.path.join(GOLDEN, "kat134")


def kat_event():
    g = io.load_event(os.path.join(KAT, "event_1_filtered_graph_"), 7, 7)
    truth = io.read_truth(os.path.join(KAT, "truth_vol7.csv"), g.node["node_id"])
    return g, truth


def kat_rows():
    return np.genfromtxt(os.path.join(KAT, "1_events_training_data.csv"), delimiter=",", names=True)


def sorted_rows(kl, ev, tr):
    o = np.lexsort((tr, ev, kl))
    return kl[o], ev[o], tr[o]


def test_parabolic_rows_match_committed_training_csv():
    g, truth = kat_event()
    assert (truth >= 0).all()
    _, _, _, kl, ev, tr = O.parabolic_training_rows(g, truth)
    kat = kat_rows()
    assert kl.size == kat.size == 7574
    a = sorted_rows(kl, ev, tr.astype(np.float64))
    b = sorted_rows(kat["kl_dist"], kat["emp_var"], kat["truth"])
    assert np.abs(a[0] - b[0]).max() / 1.0 < 1e-8 * np.abs(b[0]).max()
    assert (np.abs(a[0] - b[0]) / np.abs(b[0])).max() < 1e-8
    assert (np.abs(a[1] - b[1]) <= 1e-9 * np.abs(b[1])).all()
    assert (a[2] == b[2]).all()
    assert int(tr.sum()) == 5231
