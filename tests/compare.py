"""Field-by-field comparison of TrackGraph outputs (test helper).

Integer / flag / index outputs must match exactly (activation masks, ranks =
dict membership and order, degree, merged flags). Floats are compared with a
relative tolerance, only where the entry exists (rank >= 0 / has_merged).
"""
import hashlib

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


# ---------------------------------------------------------------------------
# conditioning-aware float comparison (DESIGN.md "Parity bar")
# ---------------------------------------------------------------------------
def cov_defect(c5):
    """symmetry defect |c01 - c10| / sqrt(|c00 c11|) of stored covariances: the exact
    result is symmetric, so this is a lower bound on the relative rounding error the
    value already carries in fp64 (in whichever implementation produced it)."""
    c5 = np.asarray(c5, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = np.abs(c5[:, 1] - c5[:, 2]) / np.sqrt(np.abs(c5[:, 0] * c5[:, 3]))
    return np.where(np.isfinite(d), d, np.inf)


def compare_cond(got, exp, rtol=1e-6, report=8):
    """Masks / ranks / flags exactly; floats within rtol, except that a value whose
    computation is ill-conditioned is compared within rtol + 10 x its measured
    defect (normalised covariance units). Returns (errors, n_relaxed)."""
    errs = compare(got, exp, rtol=rtol, fields=INT_NODE + INT_SLOT + ["tse_prior", "tse_mw", "edge_mw",
                                                                      "uts_tau", "uts_xyzr", "uts_lr"])
    S, G = exp.slot, got.slot
    pres = S["uts_rank"] >= 0
    dk = np.maximum(cov_defect(S["uts_cov"]), cov_defect(G["uts_cov"]))
    tol = rtol + 10.0 * np.where(dk > 1e-9, dk, 0.0)
    relaxed = int(np.sum(pres & (dk > 1e-9)))
    # covariance 2x2 block in normalised units, c22 relative
    c_e, c_g = S["uts_cov"], G["uts_cov"]
    with np.errstate(divide="ignore", invalid="ignore"):
        sc = np.sqrt(np.abs(np.stack([c_e[:, 0] * c_e[:, 0], c_e[:, 0] * c_e[:, 3], c_e[:, 0] * c_e[:, 3],
                                      c_e[:, 3] * c_e[:, 3]], axis=1)))
        dn = np.abs(c_g[:, :4] - c_e[:, :4]) / sc
    ok = ((dn <= tol[:, None]) | np.isclose(c_g[:, :4], c_e[:, :4], rtol=rtol, atol=0)).all(1)
    ok &= np.isclose(c_g[:, 4], c_e[:, 4], rtol=rtol, atol=0)
    bad = np.nonzero(pres & ~ok)[0]
    if bad.size:
        errs.append("slot.uts_cov: %d beyond tolerance, e.g. slot %d got %s exp %s" % (
            bad.size, bad[0], c_g[bad[0]], c_e[bad[0]]))
    # state vector: a, b relative (+ defect); c (receiver-frame offset, ~0 by construction)
    # absolute at the rounding level of the predicted offset
    sv_e, sv_g = S["uts_sv"], G["uts_sv"]
    ab_ok = (np.abs(sv_g[:, :2] - sv_e[:, :2]) <= tol[:, None] * np.abs(sv_e[:, :2]) + 1e-12).all(1)
    c_ok = np.abs(sv_g[:, 2] - sv_e[:, 2]) <= rtol * np.abs(sv_e[:, 2]) + 1e-14 * np.max(
        np.abs(sv_e[:, :2]), axis=1) + 1e-12
    bad = np.nonzero(pres & ~(ab_ok & c_ok))[0]
    if bad.size:
        errs.append("slot.uts_sv: %d beyond tolerance, e.g. slot %d got %s exp %s" % (
            bad.size, bad[0], sv_g[bad[0]], sv_e[bad[0]]))
    for f in ("uts_lik", "uts_mw", "uts_prior"):
        t = tol
        ok = np.abs(G[f] - S[f]) <= t * np.abs(S[f]) + 1e-12
        ok |= np.isnan(G[f]) & np.isnan(S[f])
        bad = np.nonzero(pres & ~ok)[0]
        if bad.size:
            errs.append("slot.%s: %d beyond tolerance, e.g. slot %d got %s exp %s" % (f, bad.size, bad[0],
                                                                                  G[f][bad[0]], S[f][bad[0]]))
    # merged outputs: tolerance from the worst defect among the node's states
    dst = exp.slot_dst()
    dv = np.zeros(exp.n_nodes)
    np.maximum.at(dv, dst[pres], np.where(dk[pres] > 1e-9, dk[pres], 0.0))
    tv = rtol + 1e3 * dv
    relaxed += int(np.sum((exp.node["has_merged"] == 1) & (dv > 0)))
    mm = exp.node["has_merged"] == 1
    ms_e, ms_g = exp.node["merged_state"], got.node["merged_state"]
    okm = (np.abs(ms_g - ms_e) <= tv[:, None] * np.abs(ms_e) + 1e-14 * np.max(np.abs(ms_e), axis=1,
                                                                                  keepdims=True)).all(1)
    mc_e, mc_g = exp.node["merged_cov"], got.node["merged_cov"]
    with np.errstate(divide="ignore", invalid="ignore"):
        scm = np.sqrt(np.abs(np.stack([mc_e[:, 0] * mc_e[:, 0], mc_e[:, 0] * mc_e[:, 3], mc_e[:, 0] * mc_e[:, 3],
                                       mc_e[:, 3] * mc_e[:, 3]], axis=1)))
        dnm = np.abs(mc_g[:, :4] - mc_e[:, :4]) / scm
    okc = ((dnm <= tv[:, None]) | np.isclose(mc_g[:, :4], mc_e[:, :4], rtol=rtol, atol=0)).all(1)
    okc &= np.abs(mc_g[:, 4] - mc_e[:, 4]) <= tv * np.abs(mc_e[:, 4])
    okp = np.abs(got.node["merged_prior"] - exp.node["merged_prior"]) <= tv * np.abs(exp.node["merged_prior"])
    bad = np.nonzero(mm & ~(okm & okc & okp))[0]
    if bad.size:
        errs.append("node.merged_*: %d beyond tolerance, e.g. node %d got %s / %s exp %s / %s (defect %.2e)" % (
            bad.size, bad[0], ms_g[bad[0]], mc_g[bad[0]], ms_e[bad[0]], mc_e[bad[0]], dv[bad[0]]))
    return errs, relaxed


# ---------------------------------------------------------------------------
# intrinsic numerical noise, estimated by perturbing the inputs at the ulp level
# ---------------------------------------------------------------------------
FLOAT_OUT_NODE = ["merged_state", "merged_cov", "merged_prior"]
FLOAT_OUT_SLOT = ["uts_sv", "uts_tau", "uts_cov", "uts_lik", "uts_mw", "uts_prior", "edge_mw", "tse_prior",
                  "tse_mw"]
MASK_OUT = [("node", "has_merged"), ("node", "has_uts"), ("node", "degree"), ("slot", "act"),
            ("slot", "uts_rank")]


PERTURB_NODE = ("gnn", "merged_state", "merged_cov")


def perturbed(g, rel, seed):
    """copy of g with the continuous physical inputs (hit coordinates, merged
    states and covariances) scaled by (1 + U(-rel, rel)); keys such as the layer
    id and exact weights are left alone"""
    rng = np.random.default_rng(seed)
    p = g.copy()
    same = np.array_equal(g.node["gnn"], g.node["xyzr"], equal_nan=True)
    for k in PERTURB_NODE:
        v = p.node[k]
        p.node[k] = v * (1.0 + rng.uniform(-rel, rel, v.shape))
    if same:
        p.node["xyzr"] = p.node["gnn"].copy()
    return p


def noise_envelope(run, g, n=3, rel=2.0 ** -46):
    """run(g) -> output TrackGraph. Returns (reference output, per-field noise arrays,
    per-field set of mask positions that flip under the perturbation)."""
    ref = run(g.copy())
    noise = {("node", f): np.zeros_like(ref.node[f]) for f in FLOAT_OUT_NODE}
    noise.update({("slot", f): np.zeros_like(ref.slot[f]) for f in FLOAT_OUT_SLOT})
    flips = {m: np.zeros(getattr(ref, m[0])[m[1]].shape, bool) for m in MASK_OUT}
    for i in range(n):
        o = run(perturbed(g, rel, 1000 + i))
        for (kind, f), arr in noise.items():
            a, b = getattr(o, kind)[f], getattr(ref, kind)[f]
            dif = np.abs(a - b)
            dif = np.where(np.isnan(a) & np.isnan(b), 0.0, dif)
            dif = np.where(np.isnan(dif), np.inf, dif)
            np.maximum(arr, dif, out=arr)
        for (kind, f) in MASK_OUT:
            flips[(kind, f)] |= getattr(o, kind)[f] != getattr(ref, kind)[f]
    return ref, noise, flips


def compare_noise(got, ref, noise, flips, rtol=1e-6, k=100.0):
    """masks exact except positions that flip under ulp perturbation of the inputs;
    floats within rtol*|ref| + k*noise. Returns (errors, stats)."""
    errs = []
    stats = {"mask_undetermined": 0, "float_ill": 0, "float_checked": 0}
    present_uts = ref.slot["uts_rank"] >= 0
    present_tse = ref.slot["tse_rank"] >= 0
    # a state whose value is numerically undetermined (its own perturbation noise exceeds
    # rtol) makes every decision its node takes from it undetermined too: the node's
    # merged outputs and the masks of its in-slots are not held to exact equality
    ill_slot = np.zeros(ref.n_slots, bool)
    for f in ("uts_sv", "uts_cov"):
        nz, b = noise[("slot", f)], ref.slot[f]
        ill_slot |= (nz > rtol * np.abs(b)).any(axis=1) & present_uts
    dst = ref.slot_dst()
    ill_node = np.zeros(ref.n_nodes, bool)
    ill_node[dst[ill_slot]] = True
    ill_slot_all = ill_node[dst]
    stats["ill_nodes"] = int(ill_node.sum())
    for (kind, f), fl in flips.items():
        a, b = getattr(got, kind)[f], getattr(ref, kind)[f]
        m = ref.slot["is_edge"] == 1 if f == "act" else np.ones(a.shape, bool)
        if f == "uts_rank":
            a, b = dense_ranks(got, f), dense_ranks(ref, f)
        und = fl | (ill_slot_all if kind == "slot" else ill_node)
        bad = np.nonzero((a != b) & m & ~und)[0]
        stats["mask_undetermined"] += int(np.sum(fl & m))
        stats["mask_ill_differs"] = stats.get("mask_ill_differs", 0) + int(np.sum((a != b) & m & und & ~fl))
        if bad.size:
            errs.append("%s.%s: %d mismatches (not perturbation-sensitive), e.g. %s got %s exp %s" % (
                kind, f, bad.size, bad[:6], a[bad[:6]], b[bad[:6]]))
    for (kind, f), nz in noise.items():
        a, b = getattr(got, kind)[f], getattr(ref, kind)[f]
        if kind == "node":
            m = ref.node["has_merged"] == 1
        elif f.startswith("uts"):
            m = present_uts
        elif f.startswith("tse"):
            m = present_tse
        else:
            m = ref.slot["is_edge"] == 1
        # a state whose dict membership is perturbation-sensitive is not compared
        if kind == "slot":
            m = m & ~flips[("slot", "uts_rank")] & ~flips[("slot", "act")]
            if f in ("uts_mw", "uts_prior", "edge_mw", "tse_prior", "tse_mw"):
                m = m & ~ill_slot_all      # weights downstream of an undetermined decision
        else:
            m = m & ~flips[("node", "has_merged")] & ~ill_node
        tol = rtol * np.abs(b) + k * nz + 1e-300
        if f == "uts_sv":   # receiver-frame offset c ~ 0: rounding level of the predicted state
            scale = ref.slot.get("xp_scale", np.max(np.abs(b[:, :2]), axis=1))
            tol[:, 2] += 8 * 2.0 ** -52 * scale
        ok = (np.abs(a - b) <= tol) | (np.isnan(a) & np.isnan(b))
        ok = ok.reshape(ok.shape[0], -1).all(axis=1)
        ill = (nz > rtol * np.abs(b)).reshape(nz.shape[0], -1).any(axis=1)
        stats["float_ill"] += int(np.sum(ill & m))
        stats["float_checked"] += int(np.sum(m))
        bad = np.nonzero(m & ~ok)[0]
        if bad.size:
            errs.append("%s.%s: %d beyond rtol+noise, e.g. %d got %s exp %s noise %s" % (
                kind, f, bad.size, bad[0], a[bad[0]], b[bad[0]], nz[bad[0]]))
    return errs, stats


def input_sha(g):
    """SHA-256 of a generated event's structure and of the inputs the pass reads (pins a
    full-size digest to the generator output it was made from)"""
    h = hashlib.sha256()
    for a in (g.slot_ptr, g.out_ptr, g.out_slot, g.slot["slot_src"], g.node["gnn"], g.node["xyzr"],
              g.node["merged_state"], g.node["merged_cov"], g.node["has_merged"], g.slot["send_mw"],
              g.slot["tse_rank"], g.node["layer"]):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
