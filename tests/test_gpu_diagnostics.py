"""Diagnostics outputs: the truth-based outlier-masking counts the reference's
stages print, reproduced from the device's diagnostics (gtf_set_diagnostics: per-slot
clustering membership, the stage split into the reference's calls) and compared with the
reference's own printed numbers on the volume-7 network (tests/golden/diag_vol7.json, made
by tests/golden/make_golden_diag.py from its stdout):

* clustering on track_state_estimates (-c 1.0 -k 2.0): clustering.py:342-369;
* the extrapolation stage: message_passing (extrapolate_merged_states.py:496-518) and the
  two reweights (helper.py:203-225, with its '= 1' counter bug);
* the update stage's reweight.

The stage outputs of the split runs equal the fused stages' (the same node-op sequences).
"""
import json
import os

import numpy as np
import pytest

from fixtures import GOLDEN, load
from compare import compare
from gtf.params import Params

pytestmark = pytest.mark.gpu


def _truth(g):
    t = json.load(open(os.path.join(GOLDEN, "diag_vol7.json")))["truth"]
    return np.array([t[str(int(n))] for n in g.node["node_id"]], dtype=np.int64)


def _expected(name):
    return json.load(open(os.path.join(GOLDEN, "diag_vol7.json")))[name]


def test_diagnostics_cluster_tse():
    from gtf.diagnostics import stage_diagnostics
    g, out, _, meta = load("cluster_tse")
    h, blocks = stage_diagnostics(g, "cluster", _truth(g), Params(), chi2=meta["chi2"], kl=meta["kl"], key="tse")
    assert blocks == _expected("cluster_tse"), blocks


def test_diagnostics_extrapolate():
    from gtf.device import DeviceGraph
    from gtf.diagnostics import stage_diagnostics
    g, out, _, meta = load("extrapolate_it2")
    p = Params(sigma0xy=meta["sigma0xy"], sigma0rz=meta["sigma0rz"], sigma0rz2=meta["sigma0rz2"],
               endcap_boundary=meta["endcap_boundary"], chi2_cut=meta["chi2_cut"])
    h, blocks = stage_diagnostics(g, "extrapolate", _truth(g), p)
    assert blocks == _expected("extrapolate"), blocks
    # the split run's outputs are the fused stage's
    f = g.copy()
    d = DeviceGraph(f)
    d.extrapolate(p)
    d.download(f)
    errs = compare(h, f, rtol=0.0, atol=0.0)
    assert errs == [], errs


def test_diagnostics_update():
    from gtf.diagnostics import stage_diagnostics
    g, out, _, meta = load("update_it2")
    h, blocks = stage_diagnostics(g, "update", _truth(g), Params())
    assert blocks == _expected("update"), blocks
