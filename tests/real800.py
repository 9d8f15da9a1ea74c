"""Helpers of the real multi-volume parity tests (test_real800.py, test_gpu_real800.py):
the committed 800' all-volume event (tests/golden/kat800, SURVEY §8a "C2") and the
reference's per-subgraph outputs (tests/golden/make_golden_800.py)."""
import hashlib
import os

import numpy as np

from fixtures import GOLDEN

KAT800 = os.path.join(GOLDEN, "kat800")
PREFIX = os.path.join(KAT800, "event_1_filtered_graph_")
VOLS = (7, 14)
CLUSTER_TSE = dict(chi2=1.0, kl=2.0)          # run_gnn_trackml_mod.sh:89
RAISING = 4 | 8 | 32                          # GTF_ERR_ALL_ZERO_DIST | _TIE_EMPTIED | _NAN_KL: ValueError


def fixture(name):
    return np.load(os.path.join(GOLDEN, "c2_800_%s.npz" % name), allow_pickle=False)


def structure_digest(g):
    """make_golden_800.structure_digest: node ids, slot segments, senders, successor order,
    TSE dict order"""
    hh = hashlib.sha256()
    for a in (g.node["node_id"].astype(np.int64), g.slot_ptr.astype(np.int64), g.slot["slot_src"].astype(np.int64),
              g.out_ptr.astype(np.int64), g.out_slot.astype(np.int64), g.slot["tse_rank"].astype(np.int64)):
        hh.update(np.ascontiguousarray(a).tobytes())
    return hh.hexdigest()


def full_load(g):
    """every node's merged state = a copy of its first TSE entry (make_golden.full_load,
    SURVEY §8d), on a packed graph"""
    h = g.copy()
    first = np.nonzero(h.slot["tse_rank"] == 0)[0]
    v = h.slot_dst()[first]
    h.node["has_merged"][:] = 0
    h.node["has_merged"][v] = 1
    h.node["merged_state"][v] = h.slot["tse_sv"][first]
    h.node["merged_cov"][v] = h.slot["tse_cov"][first]
    h.node["merged_prior"][v] = h.slot["tse_prior"][first]
    return h


def compare(got, z, node_err=None, rtol=1e-6):
    """mismatches of a stage output (host order) against a per-subgraph reference fixture:
    every subgraph the reference did not raise in matches exactly on masks / flags /
    degree / dict order and within rtol on the pinned floats; with node_err, the
    subgraphs where the device flags a ValueError of the reference are exactly the
    raising ones. Returns (errors, stats)."""
    errs = []
    sub = got.node["sub_id"].astype(np.int64)
    raised = z["raised"].astype(bool)
    ok_n = ~raised[sub]
    ok_s = ok_n[got.slot_dst()]
    N, S = got.n_nodes, got.n_slots

    def exact(name, a, b, m):
        bad = np.nonzero((a != b) & m)[0]
        if bad.size:
            errs.append("%s: %d mismatches, e.g. %s got %s exp %s" % (name, bad.size, bad[:6], a[bad[:6]], b[bad[:6]]))

    exact("act", got.slot["act"].astype(np.uint8), np.unpackbits(z["act_bits"], count=S), ok_s)
    exact("has_merged", got.node["has_merged"].astype(np.uint8), np.unpackbits(z["has_merged_bits"], count=N), ok_n)
    exact("degree", got.node["degree"].astype(np.int64), z["degree"].astype(np.int64), ok_n)
    if "has_uts_bits" in z:
        from compare import dense_ranks
        exact("has_uts", got.node["has_uts"].astype(np.uint8), np.unpackbits(z["has_uts_bits"], count=N), ok_n)
        exact("uts_rank", dense_ranks(got, "uts_rank").astype(np.int64), z["uts_dense_rank"].astype(np.int64), ok_s)
        smp = z["sample_slot"].astype(np.int64)
        for f in ("uts_sv", "uts_cov", "uts_tau", "uts_lik", "uts_mw", "uts_prior", "edge_mw"):
            a, b = got.slot[f][smp], z["slot__" + f]
            tol = rtol * np.abs(b) + 1e-300
            if f == "uts_sv":   # receiver-frame offset c ~ 0: rounding level of the predicted state
                tol[:, 2] += 8 * 2.0 ** -52 * np.max(np.abs(b[:, :2]), axis=1)
            good = ((np.abs(a - b) <= tol) | (np.isnan(a) & np.isnan(b))).reshape(smp.size, -1).all(1) | ~ok_s[smp]
            if not good.all():
                i = np.nonzero(~good)[0][0]
                errs.append("%s: %d of %d sampled beyond rtol, e.g. slot %d got %s exp %s" % (
                    f, int((~good).sum()), smp.size, smp[i], a[i], b[i]))
    sn = z["sample_node"].astype(np.int64)
    for f in ("merged_state", "merged_cov", "merged_prior"):
        a, b = got.node[f][sn], z[f]
        good = (np.abs(a - b) <= rtol * np.abs(b) + 1e-300).reshape(sn.size, -1).all(1) | ~ok_n[sn]
        if not good.all():
            i = np.nonzero(~good)[0][0]
            errs.append("%s: %d of %d beyond rtol, e.g. node %d got %s exp %s" % (
                f, int((~good).sum()), sn.size, sn[i], a[i], b[i]))
    stats = {"subgraphs": int(raised.size), "raised": np.nonzero(raised)[0].tolist()}
    if node_err is not None:
        flagged = np.zeros(raised.size, bool)
        np.logical_or.at(flagged, sub, (node_err & RAISING) != 0)
        if not np.array_equal(flagged, raised):
            errs.append("ValueError subgraphs: device %s, reference %s" % (
                np.nonzero(flagged)[0].tolist(), np.nonzero(raised)[0].tolist()))
        stats["flag_nodes"] = {int(v): int(node_err[v]) for v in np.nonzero(node_err)[0]}
    return errs, stats
