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


# ---------------------------------------------------------------- KAT-2
KAT800 = os.path.join(GOLDEN, "kat800")


def kat2_event():
    """volume 7 of the committed minCurv_0.3_800 event: the graph of the rows of event 1 in
    the reference's 3_events_training_data.csv (its other two events are not committed)"""
    g = io.load_event(os.path.join(KAT800, "event_1_filtered_graph_"), 7, 7)
    truth = io.read_truth(os.path.join(KAT800, "truth.csv"), g.node["node_id"])
    return g, truth


def kat2_match(kl, ev, tr):
    """rows found in KAT-2: a CSV row with kl within 1e-8, emp_var within 1e-9 relative and
    the same truth flag (each CSV row used once); returns the indices not found"""
    kat = np.genfromtxt(os.path.join(KAT800, "3_events_training_data.csv"), delimiter=",", names=True)
    assert kat.size == 6163
    o = np.argsort(kat["kl_dist"])
    ks, ke, kt = kat["kl_dist"][o], kat["emp_var"][o], kat["truth"][o]
    used = np.zeros(ks.size, bool)
    missing = []
    for n in range(kl.size):
        lo = np.searchsorted(ks, kl[n] - 1e-8 * abs(kl[n]))
        hi = np.searchsorted(ks, kl[n] + 1e-8 * abs(kl[n]), side="right")
        c = [m for m in range(lo, hi) if not used[m] and abs(ke[m] - ev[n]) <= 1e-9 * abs(ev[n]) and kt[m] == tr[n]]
        if c:
            used[c[0]] = True
        else:
            missing.append(n)
    return missing


def test_parabolic_rows_match_kat2():
    """1,054 of the 1,055 volume-7 pairs of the 800' event are rows of the reference's
    KAT-2 CSV (kl 1e-8, emp_var 1e-9, truth exact). The one that is not (node 1635, kl
    276.24, emp_var 1.1e-3) has no CSV row within 1.7 % -- its emp_var differs 5x from
    every candidate, i.e. that node's neighbourhood differed in the run that wrote the
    CSV (the survey's probe found the same 1,054 / 1,055)."""
    g, truth = kat2_event()
    node, _, _, kl, ev, tr = O.parabolic_training_rows(g, truth)
    assert kl.size == 1055
    missing = kat2_match(kl, ev, tr.astype(np.float64))
    assert len(missing) == 1 and g.node["node_id"][node[missing[0]]] == 1635, missing
