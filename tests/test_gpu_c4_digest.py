"""The benchmark workload itself (C4, BASELINE configs[3]: 179,788 hits / 1,027,548
directed edges) against the oracle at full size.

tests/golden/make_c4_digest.py ran the oracle's fused pass on this event (plus three
ulp-perturbed runs for the noise envelope) and committed a digest: every activation,
every has_merged / has_uts flag, every degree and every slot's dense
updated_track_states position, plus floats at a 1 % sample. The HIP pass, uploaded in
the bench's tiled node order, must reproduce:

  * every mask / flag / degree / dict position exactly, except the positions the
    digest marks undetermined (the decision flips under a 2^-46 relative perturbation
    of the inputs, or reads a state whose own perturbation noise exceeds 1e-6);
  * the sampled floats within 1e-6 relative plus 100x their perturbation noise;
  * no reference-exception flag (the reference raises on none of these nodes).
"""
import ast
import os

import numpy as np
import pytest

from compare import dense_ranks, input_sha
from fixtures import GOLDEN
from gtf import synth
from gtf.params import Params

pytestmark = pytest.mark.gpu

RTOL = 1e-6
K_NOISE = 100.0


def _digest():
    return np.load(os.path.join(GOLDEN, "c4_digest.npz"), allow_pickle=False)


def test_c4_generator_matches_digest():
    z = _digest()
    g = synth.workload("c4", seed=0)
    assert input_sha(g) == str(z["input_sha"]), "gtf.synth changed: regenerate tests/golden/c4_digest.npz"


def digest_errors(got, z):
    """mismatches of a pass's output `got` (host order) against the digest, and the count
    of undetermined positions that differ"""
    S, N = got.n_slots, got.n_nodes
    und_s = np.unpackbits(z["und_slot_bits"], count=S).astype(bool)
    und_n = np.unpackbits(z["und_node_bits"], count=N).astype(bool)
    errs = []

    def exact(name, a, b, und):
        bad = np.nonzero((a != b) & ~und)[0]
        if bad.size:
            errs.append("%s: %d mismatches, e.g. %s got %s exp %s" % (name, bad.size, bad[:6], a[bad[:6]], b[bad[:6]]))
        return int(np.sum((a != b) & und))

    diff_und = 0
    diff_und += exact("act", got.slot["act"].astype(np.uint8),
                      np.unpackbits(z["act_bits"], count=S), und_s)
    diff_und += exact("has_merged", got.node["has_merged"].astype(np.uint8),
                      np.unpackbits(z["has_merged_bits"], count=N), und_n)
    diff_und += exact("has_uts", got.node["has_uts"].astype(np.uint8),
                      np.unpackbits(z["has_uts_bits"], count=N), und_n)
    diff_und += exact("degree", got.node["degree"].astype(np.int64), z["degree"].astype(np.int64), und_n)
    diff_und += exact("uts_rank", dense_ranks(got, "uts_rank").astype(np.int64),
                      z["uts_dense_rank"].astype(np.int64), und_s)
    for kind, idx, fields in (("slot", z["sample_slot"], ["uts_sv", "uts_cov", "uts_tau", "uts_lik", "uts_mw",
                                                           "uts_prior", "edge_mw"]),
                              ("node", z["sample_node"], ["merged_state", "merged_cov", "merged_prior"])):
        for f in fields:
            a = getattr(got, kind)[f][idx]
            b = z[kind + "__" + f]
            nz = z["noise__" + f]
            tol = RTOL * np.abs(b) + K_NOISE * nz + 1e-300
            if f == "uts_sv":   # receiver-frame offset c ~ 0: rounding level of the predicted state
                tol[:, 2] += 8 * 2.0 ** -52 * np.max(np.abs(b[:, :2]), axis=1)
            ok = (np.abs(a - b) <= tol) | (np.isnan(a) & np.isnan(b))
            ok = ok.reshape(ok.shape[0], -1).all(axis=1)
            bad = np.nonzero(~ok)[0]
            if bad.size:
                errs.append("%s.%s: %d of %d sampled beyond rtol+noise, e.g. %d got %s exp %s" % (
                    kind, f, bad.size, idx.size, idx[bad[0]], a[bad[0]], b[bad[0]]))
    return errs, diff_und


@pytest.mark.parametrize("layout", ["tiled", "natural"])
def test_c4_pass_matches_oracle_digest(layout):
    from gtf.device import DeviceGraph
    z = _digest()
    stats = ast.literal_eval(str(z["stats"]))
    g = synth.workload("c4", seed=0)
    d = DeviceGraph(g, layout=layout)
    d.clear_errors()
    d.full_pass(Params())
    flags = d.errors()
    got = d.download(g.copy())
    errs, diff_und = digest_errors(got, z)
    print("C4 %s layout: %s; undetermined positions that differ: %d; device flags %d" % (
        layout, stats, diff_und, flags))
    assert errs == [], "\n".join(errs)
    assert flags == 0, flags
    # the undetermined class stays small (a few per mille of the slots)
    assert stats["undetermined_slots"] <= 0.01 * g.n_slots
