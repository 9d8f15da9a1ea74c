"""Field-by-field comparison of TrackGraph outputs (test helper).

Integer / flag / index outputs must match exactly (activation masks, ranks =
dict membership and order, degree, merged flags). Floats are compared with a
relative tolerance, only where the entry exists (rank >= 0 / has_merged).
"""
import numpy as np

INT_NODE = ["has_merged", "has_uts", "degree"]
INT_SLOT = ["act", "tse_rank", "uts_rank", "uts_side"]
FLOAT_NODE = ["merged_state", "merged_cov", "merged_prior"]
FLOAT_SLOT_UTS = ["uts_sv", "uts_tau", "uts_cov", "uts_xyzr", "uts_lik", "uts_mw", "uts_prior", "uts_lr"]
FLOAT_SLOT_TSE = ["tse_prior", "tse_mw"]


def _close(a, b, rtol, atol):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    ok = np.isclose(a, b, rtol=rtol, atol=atol) | both_nan
    return ok


def dense_ranks(g, field):
    """per-node dict order as 0..n-1 (ranks may have gaps after pruning)"""
    r = g.slot[field].astype(np.int64)
    out = np.full_like(r, -1)
    sp = g.slot_ptr
    for v in range(g.n_nodes):
        lo, hi = sp[v], sp[v + 1]
        seg = r[lo:hi]
        pres = np.nonzero(seg >= 0)[0]
        if pres.size:
            order = pres[np.argsort(seg[pres], kind="stable")]
            out[lo + order] = np.arange(order.size)
    return out


def compare(got, exp, rtol=1e-6, atol=1e-12, fields=None, report=8):
    """Returns a list of human-readable mismatch descriptions (empty = equal)."""
    errs = []
    want = set(fields) if fields else None

    def use(f):
        return want is None or f in want

    for f in INT_NODE:
        if use(f) and f in exp.node:
            bad = np.nonzero(got.node[f] != exp.node[f])[0]
            if bad.size:
                errs.append("node.%s: %d mismatches, e.g. %s got %s exp %s" % (
                    f, bad.size, bad[:report], got.node[f][bad[:report]], exp.node[f][bad[:report]]))
    for f in INT_SLOT:
        if use(f):
            if f == "uts_side":
                m = exp.slot["uts_rank"] >= 0
            else:
                m = np.ones(exp.n_slots, bool)
            if f == "act":
                m = exp.slot["is_edge"] == 1
            gv, ev = got.slot[f], exp.slot[f]
            if f.endswith("_rank"):
                gv, ev = dense_ranks(got, f), dense_ranks(exp, f)
            bad = np.nonzero((gv != ev) & m)[0]
            if bad.size:
                errs.append("slot.%s: %d mismatches, e.g. %s got %s exp %s" % (
                    f, bad.size, bad[:report], gv[bad[:report]], ev[bad[:report]]))
    mm = exp.node["has_merged"] == 1
    for f in FLOAT_NODE:
        if use(f):
            ok = _close(got.node[f], exp.node[f], rtol, atol)
            ok = ok.reshape(ok.shape[0], -1).all(axis=1) | ~mm
            bad = np.nonzero(~ok)[0]
            if bad.size:
                errs.append("node.%s: %d mismatches, e.g. node %d got %s exp %s" % (
                    f, bad.size, bad[0], got.node[f][bad[0]], exp.node[f][bad[0]]))
    for pfx, flist in (("uts", FLOAT_SLOT_UTS), ("tse", FLOAT_SLOT_TSE)):
        present = exp.slot[pfx + "_rank"] >= 0
        for f in flist:
            if use(f):
                ok = _close(got.slot[f], exp.slot[f], rtol, atol)
                ok = ok.reshape(ok.shape[0], -1).all(axis=1) | ~present
                bad = np.nonzero(~ok)[0]
                if bad.size:
                    errs.append("slot.%s: %d mismatches, e.g. slot %d got %s exp %s" % (
                        f, bad.size, bad[0], got.slot[f][bad[0]], exp.slot[f][bad[0]]))
    if use("edge_mw"):
        m = exp.slot["is_edge"] == 1
        ok = _close(got.slot["edge_mw"], exp.slot["edge_mw"], rtol, atol) | ~m
        bad = np.nonzero(~ok)[0]
        if bad.size:
            errs.append("slot.edge_mw: %d mismatches, e.g. slot %d got %s exp %s" % (
                bad.size, bad[0], got.slot["edge_mw"][bad[0]], exp.slot["edge_mw"][bad[0]]))
    return errs
