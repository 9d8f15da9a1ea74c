"""CPU oracle: NumPy restatement of the reference's hot-path algorithm.

TEST INFRASTRUCTURE ONLY. Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker (or, in bench.py,
as the timed CPU baseline). The product path (``gtf``) never falls back to it.

Every function restates one reference function, op for op with the same NumPy
calls (``np.linalg.inv``, ``dot``, filterpy's predict/update sequence), on the
packed :class:`gtf.graph.TrackGraph` layout instead of networkx dicts, so its
results match the reference bit for bit on the same inputs. Citations are
``file:line`` in ``/root/reference``.

Pinning (see DESIGN.md "Oracle"): the restatement is checked against
``tests/golden/*.npz`` -- fixtures produced by running the reference's own
functions on its committed event data (tests/golden/make_golden.py) -- and the
parabolic-model KL (a17) against the reference's committed training CSV
(known-answer test). filterpy (third-party, unpinned, not vendored; SURVEY
§8c) is restated from its 1.4.5 release; parity for that piece is pinned only
to that restatement.
"""
from __future__ import annotations

import math
from math import atan2

import numpy as np

from gtf.graph import TrackGraph, mat_from_cov5, cov5_from_mat  # container only


class ReferenceError_(ValueError):
    """Raised where the reference itself raises (KeyError / ValueError paths)."""


# ---------------------------------------------------------------------------
# helpers over the packed layout
# ---------------------------------------------------------------------------
def _dict_order(g: TrackGraph, pfx: str, v: int):
    """slots of node v holding a key of the given state dict, in dict order"""
    lo, hi = int(g.slot_ptr[v]), int(g.slot_ptr[v + 1])
    r = g.slot[pfx + "_rank"][lo:hi]
    ks = [lo + j for j in range(hi - lo) if r[j] >= 0]
    ks.sort(key=lambda k: int(g.slot[pfx + "_rank"][k]))
    return ks


def _has(g, pfx, v):
    return bool(g.node["has_" + pfx][v])


def _edge_active(g, k):
    return bool(g.slot["is_edge"][k]) and g.slot["act"][k] == 1


# ---------------------------------------------------------------------------
# filterpy 1.4.5 KalmanFilter restated (third-party; not in /root/reference)
# call sites: src/extrapolate/extrapolate_merged_states.py:307-323
# ---------------------------------------------------------------------------
def _kf_predict_update(x, P, F, H, R, Q, z):
    dot = np.dot
    # predict(): x = Fx ; P = alpha_sq * FPF' + Q  (alpha_sq = 1.0)
    x = dot(F, x)
    P = 1.0 * dot(dot(F, P), F.T) + Q
    # update(z): reshape_z(z, dim_z=1, ndim=x.ndim=1) -> shape (1,)
    z = np.atleast_2d(z)
    if z.shape[1] == 1:
        z = z.T
    z = z[:, 0]
    y = z - dot(H, x)
    PHT = dot(P, H.T)
    S = dot(H, PHT) + R
    SI = np.linalg.inv(S)
    K = dot(PHT, SI)
    x = x + dot(K, y)
    I_KH = np.eye(3) - dot(K, H)
    P = dot(dot(I_KH, P), I_KH.T) + dot(dot(K, R), K.T)
    return x.copy(), P.copy()


# ---------------------------------------------------------------------------
# a7: extrapolate_validate  (extrapolate_merged_states.py:26-402)
# ---------------------------------------------------------------------------
def extrapolate_validate(node_gnn, nb_gnn, merged_state, merged_cov, chi2_cut, sigma0xy,
                         sigma0rz, sigma0rz2, endcap_boundary):
    """Returns (accepted, payload, chi2). ``merged_cov`` is mutated in place
    (merged_cov[1,1] += var_ms, :127-128) exactly like the reference."""
    node_x, node_y, node_z, node_r = node_gnn
    neighbour_x, neighbour_y, neighbour_z, neighbour_r = nb_gnn
    angle_of_rotation_C = atan2(node_y, node_x)                                   # :41
    x_A = (neighbour_x - node_x) * np.cos(angle_of_rotation_C) + (neighbour_y - node_y) * np.sin(angle_of_rotation_C)   # :52
    y_A = -(neighbour_x - node_x) * np.sin(angle_of_rotation_C) + (neighbour_y - node_y) * np.cos(angle_of_rotation_C)  # :53
    a, b, c = merged_state[0], merged_state[1], merged_state[2]                   # :58
    phi = atan2((node_x * neighbour_y) - (node_y * neighbour_x), (node_x * neighbour_x) + (node_y * neighbour_y))  # :59
    x_prime = x_A + (c * np.sin(phi))                                             # :63
    Vx_prime = np.cos(phi) + (b * np.sin(phi))
    Ax_prime = a * np.sin(phi)
    s_star = (- x_prime * ((2 * Vx_prime**2) + (Ax_prime * x_prime))) / (2 * Vx_prime**3)   # :68
    # :71-79 (y_c, b_c, a_c are computed by the reference but never used)
    numer = x_A + c * np.sin(phi)                                                 # :82
    denom = np.cos(phi) + b * np.sin(phi)
    ds_da = - (np.sin(phi) * numer**2) / denom**3
    ds_db = ((np.sin(phi) * numer) * (1 + ((3 * a * np.sin(phi) * numer) / denom**2))) / denom**2
    ds_dc = - np.sin(phi) * (1 + ((2 * a * np.sin(phi) * numer) / denom**2)) / denom
    denom = np.cos(phi) + ((2 * a + b) * np.sin(phi))                             # :89
    da_da = (1 / denom**3) * (1 - ((6 * a * np.sin(phi)) * (s_star + a * ds_da) / denom))
    da_db = (-3 * a * np.sin(phi) * ((2 * a * ds_db) + 1)) / denom**4
    da_dc = (-6 * np.sin(phi) * ds_dc * a**2) / denom**4
    denom = np.cos(phi) + ((2 * a * s_star + b) * np.sin(phi))                    # :95
    bracket = np.cos(phi) - ((np.sin(phi) * (-np.sin(phi) + ((2 * a * s_star + b) * np.cos(phi)))) / denom)
    db_da = (2 * (s_star + a * ds_da) * bracket) / denom
    db_db = ((1 + (2 * a * ds_da)) * bracket) / denom
    db_dc = (2 * a * ds_dc * bracket) / denom
    bracket = (np.cos(phi) * (2 * a + b)) - np.sin(phi)                           # :102
    dc_da = (ds_da * bracket) + (s_star**2 * np.cos(phi))
    dc_db = (ds_db * bracket) + (s_star * np.cos(phi))
    dc_dc = (ds_dc * bracket) + np.cos(phi)
    F = np.array([[da_da, da_db, da_dc],
                  [db_da, db_db, db_dc],
                  [dc_da, dc_db, dc_dc]])                                          # :108
    dr = neighbour_r - node_r                                                     # :114
    dz = neighbour_z - node_z
    hyp = np.sqrt(dr**2 + dz**2)
    sin_t = np.abs(dr) / hyp
    kappa = (2 * a) / (1 + ((2 * a * neighbour_x) + b)**2)**1.5
    var_ms = sin_t * ((13.6 * 1e-3 * np.sqrt(0.02) * kappa) / 0.3)**2              # :120
    if np.abs(node_z) >= endcap_boundary:
        tan_t = np.abs(dr) / np.abs(dz)
        var_ms = var_ms * tan_t
    merged_cov[1, 1] += var_ms                                                    # :128 (in place)
    extrp_state = F.dot(merged_state)
    extrp_cov = F.dot(merged_cov).dot(F.T)
    H = np.array([[0., 0., 1.]])
    residual = .0 - H.dot(extrp_state)                                           # :137
    S = H.dot(extrp_cov).dot(H.T) + sigma0xy**2
    inv_S = np.linalg.inv(S)
    chi2 = residual.T.dot(inv_S).dot(residual)                                   # :140
    # :143-295 rz-plane chi2 / CSV appends: diagnostics only, no effect on outputs
    if chi2 <= chi2_cut:                                                          # :298
        factor = 2 * math.pi * np.abs(S)
        norm_factor = math.pow(float(factor[0, 0]), -0.5)
        likelihood = norm_factor * np.exp(-0.5 * chi2)                            # :304
        Q = np.array([[0., 0., 0.], [0., var_ms, 0.], [0., 0., 0.]])
        updated_state, updated_cov = _kf_predict_update(extrp_state, extrp_cov, F, H,
                                                        sigma0xy**2, Q, .0)       # :307-323
        tau = dz / dr                                                             # :326
        sigma_r, sigma_z = sigma0rz, sigma0rz2
        if np.abs(node_z) >= endcap_boundary:
            sigma_z, sigma_r = sigma0rz, sigma0rz2
        sigma_r_neighbour, sigma_z_neighbour = sigma0rz, sigma0rz2
        if np.abs(neighbour_z) >= endcap_boundary:
            sigma_z_neighbour, sigma_r_neighbour = sigma0rz, sigma0rz2
        J = np.array([1 / dr, -1 / dr, - dz / dr**2, dz / dr**2])                  # :344-348
        S2 = np.array([[sigma_z**2, 0, 0, 0],
                       [0, sigma_z_neighbour**2, 0, 0],
                       [0, 0, sigma_r**2, 0],
                       [0, 0, 0, sigma_r_neighbour**2]])
        variance_tau = J.dot(S2).dot(J.T)                                         # :357-358
        jcov = updated_cov                                                        # alias :362
        jcov[:, 2] = 0.0
        jcov[2, :] = 0.0
        jcov[2, 2] = variance_tau + var_ms
        return True, dict(sv=updated_state, tau=tau, cov=jcov, lik=likelihood,
                          xp_scale=max(np.max(np.abs(extrp_state)), np.max(np.abs(F.dot(extrp_state))))), chi2
    return False, None, chi2


# ---------------------------------------------------------------------------
# a6: message_passing  (extrapolate_merged_states.py:406-451)
# ---------------------------------------------------------------------------
def message_passing(g: TrackGraph, p) -> dict:
    N, S = g.node, g.slot
    dst = g.slot_dst()
    S["uts_fresh"][:] = 0
    next_rank = np.full(g.n_nodes, 0, dtype=np.int64)
    for v in range(g.n_nodes):
        lo, hi = g.slot_ptr[v], g.slot_ptr[v + 1]
        r = S["uts_rank"][lo:hi]
        next_rank[v] = (int(r.max()) + 1) if (hi > lo and r.max() >= 0) else 0
    chi2_all = np.full(g.n_slots, np.nan)
    # diagnostic (tests only): magnitude of the predicted state, the rounding scale of
    # the updated receiver-frame offset c, which cancels to ~0 by construction
    S["xp_scale"] = np.zeros(g.n_slots)
    for u in range(g.n_nodes):                                                    # :419
        if not N["has_merged"][u]:
            continue
        state = N["merged_state"][u].copy()
        cov = mat_from_cov5(N["merged_cov"][u])                                   # stored array, mutated
        for e in range(g.out_ptr[u], g.out_ptr[u + 1]):                           # :430 successors
            k = int(g.out_slot[e])
            if S["act"][k] != 1:                                                  # :431
                continue
            v = int(dst[k])
            ok, res, chi2 = extrapolate_validate(N["gnn"][u], N["gnn"][v], state, cov, p.chi2_cut,
                                                 p.sigma0xy, p.sigma0rz, p.sigma0rz2, p.endcap_boundary)
            chi2_all[k] = chi2
            if ok:                                                                # :441-447
                if not N["has_uts"][v]:
                    N["has_uts"][v] = 1
                if S["uts_rank"][k] < 0:
                    S["uts_rank"][k] = next_rank[v]
                    next_rank[v] += 1
                S["uts_fresh"][k] = 1
                S["uts_sv"][k] = res["sv"]
                S["uts_tau"][k] = res["tau"]
                S["uts_cov"][k] = cov5_from_mat(res["cov"])
                S["uts_xyzr"][k] = N["gnn"][u]                                    # sender coords :377
                S["uts_lik"][k] = res["lik"]
                S["xp_scale"][k] = res["xp_scale"]
                if np.isnan(S["send_mw"][k]):
                    raise ReferenceError_("KeyError: sender TSE has no entry for receiver (:384)")
                S["uts_mw"][k] = S["send_mw"][k]                                  # :384
                S["uts_prior"][k] = np.nan                                        # fresh dict: no prior yet
                S["uts_lr"][k] = np.nan
                S["uts_side"][k] = -1
            else:
                S["act"][k] = 0                                                   # :393
        N["merged_cov"][u] = cov5_from_mat(cov)                                   # in-place mutation persisted
    return {"chi2": chi2_all}


# ---------------------------------------------------------------------------
# a3 / a4 / a5  (helper.py:30-96)
# ---------------------------------------------------------------------------
def compute_prior_probabilities(g: TrackGraph, pfx: str) -> None:                # helper.py:30-63
    S = g.slot
    for v in range(g.n_nodes):
        if not _has(g, pfx, v):
            continue
        groups = {}
        for k in _dict_order(g, pfx, v):
            if _edge_active(g, k):
                layer = g.node["layer"][S["slot_src"][k]]
                groups.setdefault(layer, []).append(k)
        for ks in groups.values():
            prior = 1 / len(ks)
            for k in ks:
                S[pfx + "_prior"][k] = prior


def compute_mixture_weights(g: TrackGraph, pfx: str) -> None:                    # helper.py:76-96
    for v in range(g.n_nodes):
        if not _has(g, pfx, v):
            continue
        ks = _dict_order(g, pfx, v)
        if not ks:
            # single-node subgraphs are skipped (helper.py:79); elsewhere 1/0 raises (:90)
            if np.count_nonzero(g.node["sub_id"] == g.node["sub_id"][v]) == 1:
                continue
            raise ReferenceError_("ZeroDivisionError: empty state dict (helper.py:90)")
        mw = 1 / len(ks)
        for k in ks:
            g.slot[pfx + "_mw"][k] = mw


def query_node_degree_in_edges(g: TrackGraph) -> None:                           # helper.py:67-73
    S = g.slot
    for v in range(g.n_nodes):
        lo, hi = g.slot_ptr[v], g.slot_ptr[v + 1]
        g.node["degree"][v] = int(np.sum((S["is_edge"][lo:hi] == 1) & (S["act"][lo:hi] == 1)))


# ---------------------------------------------------------------------------
# a9 + a10: calculate_side_norm_factor + reweight  (helper.py:99-225)
# ---------------------------------------------------------------------------
def reweight(g: TrackGraph, pfx: str = "uts", threshold: float = 0.1) -> None:
    S, N = g.slot, g.node
    for v in range(g.n_nodes):
        if not _has(g, pfx, v):
            continue
        order = _dict_order(g, pfx, v)
        # --- calculate_side_norm_factor (helper.py:99-139)
        node_x = N["gnn"][v][0]
        left, right, lc, rc = [], [], [], []
        for k in order:
            nx_ = S[pfx + "_xyzr"][k][0]
            if _edge_active(g, k):
                if nx_ < node_x:
                    left.append(k); lc.append(nx_)
                else:
                    right.append(k); rc.append(nx_)
        last = order[-1] if order else None           # stale loop variable (helper.py:131,138)
        if (left or right) and not S["is_edge"][last]:
            raise ReferenceError_("KeyError: stale neighbour_num has no edge (helper.py:131)")
        left_norm = len(list(set(lc)))
        for k in left:
            S["uts_side"][k] = 0
            S["uts_lr"][k] = 1
            if S["act"][last] == 1:
                S["uts_lr"][k] = left_norm
        right_norm = len(list(set(rc)))
        for k in right:
            S["uts_side"][k] = 1
            S["uts_lr"][k] = 1
            if S["act"][last] == 1:
                S["uts_lr"][k] = right_norm
        # --- reweight (helper.py:164-200)
        denom = 0
        for k in order:
            if _edge_active(g, k):
                denom += (S[pfx + "_mw"][k] * S[pfx + "_lik"][k]) if pfx == "uts" else np.nan
        for k in order:
            if _edge_active(g, k):
                w = (S["uts_mw"][k] * S["uts_lik"][k] * S["uts_prior"][k]) / denom
                w /= S["uts_lr"][k]
                S["uts_mw"][k] = w
                S["edge_mw"][k] = w
                S["act"][k] = 0 if w < threshold else 1


# ---------------------------------------------------------------------------
# a11: remove_state_metadata  (src/update/remove_state_metadata.py:29-53)
# ---------------------------------------------------------------------------
def prune_states(g: TrackGraph) -> None:
    S = g.slot
    for v in range(g.n_nodes):
        pfx = "uts" if g.node["has_uts"][v] else "tse"
        if not _has(g, pfx, v):
            raise ReferenceError_("KeyError: node has no state dict (remove_state_metadata.py:39)")
        for k in _dict_order(g, pfx, v):
            if not S["rev_edge"][k]:          # sender not in graph.neighbors(node)
                S[pfx + "_rank"][k] = -1


def update_stage(g: TrackGraph, p) -> None:
    prune_states(g)
    compute_prior_probabilities(g, "tse")                                        # :51
    compute_prior_probabilities(g, "uts")                                        # :52
    reweight(g, "uts", p.reweight_threshold)                                     # :53


def extrapolate_stage(g: TrackGraph, p) -> dict:
    info = message_passing(g, p)                                                 # :552
    compute_prior_probabilities(g, "uts")                                        # :554
    reweight(g, "uts", p.reweight_threshold)
    compute_prior_probabilities(g, "uts")                                        # :558
    reweight(g, "uts", p.reweight_threshold)
    query_node_degree_in_edges(g)                                                # :562-566
    return info


# ---------------------------------------------------------------------------
# a12-a14: clustering  (src/clustering/clustering.py:11-124,181-327,372-373)
# ---------------------------------------------------------------------------
def mahalanobis_distance(mean1, cov1, mean2, cov2, node_coords, n1, n2, sigma0rz, sigma0rz2,
                         endcap_boundary):                                        # clustering.py:11-78
    residual = mean1[:2] - mean2[:2]
    covariance_delta_ab = cov1[0:2, 0:2] + cov2[0:2, 0:2]
    inv_covariance_delta_ab = np.linalg.inv(covariance_delta_ab)
    distance1 = residual.T.dot(inv_covariance_delta_ab).dot(residual)
    x_a, x_b, x_c = node_coords[0], n1[0], n2[0]
    z_a, r_a = node_coords[2], node_coords[3]
    z_b, r_b = n1[2], n1[3]
    z_c, r_c = n2[2], n2[3]
    j2 = 1 / (r_b - r_a)
    j3 = -1 / (r_c - r_a)
    j1 = - j3 - j2
    j5 = -(z_b - z_a) / (r_b - r_a)**2
    j6 = (z_c - z_a) / (r_c - r_a)**2
    j4 = - j5 - j6
    J = np.array([j1, j2, j3, j4, j5, j6])
    sza = szb = szc = sigma0rz2
    sra = srb = src = sigma0rz
    if np.abs(x_a) >= endcap_boundary:
        sza, sra = sigma0rz, sigma0rz2
    if np.abs(x_b) >= endcap_boundary:
        szb, srb = sigma0rz, sigma0rz2
    if np.abs(x_c) >= endcap_boundary:
        szc, src = sigma0rz, sigma0rz2
    Sm = np.diag([sza**2, szb**2, szc**2, sra**2, srb**2, src**2]).astype(float)
    cov_delta_tau = J.dot(Sm).dot(J.T)
    inv_cov_delta_tau = 1 / cov_delta_tau
    tau1 = (z_b - z_a) / (r_b - r_a)
    tau2 = (z_c - z_a) / (r_c - r_a)
    residual = tau1 - tau2
    distance2 = residual**2 * inv_cov_delta_tau
    return distance1 + distance2


def mahalanobis_distance_updated(mean1, cov1, mean2, cov2, node_coords, n1, n2):
    """a15: calculate_distance_between_updated_track_states.py:27-104 (hard-coded
    sigmas, |x| >= 600 endcap test). Returns (chi2, <tau>, <theta>, dtheta)."""
    residual = mean1[:2] - mean2[:2]
    inv = np.linalg.inv(cov1[0:2, 0:2] + cov2[0:2, 0:2])
    distance1 = residual.T.dot(inv).dot(residual)
    x_a, x_b, x_c = node_coords[0], n1[0], n2[0]
    z_a, r_a = node_coords[2], node_coords[3]
    z_b, r_b = n1[2], n1[3]
    z_c, r_c = n2[2], n2[3]
    j2 = 1 / (r_b - r_a)
    j3 = -1 / (r_c - r_a)
    j1 = - j3 - j2
    j5 = -(z_b - z_a) / (r_b - r_a)**2
    j6 = (z_c - z_a) / (r_c - r_a)**2
    j4 = - j5 - j6
    J = np.array([j1, j2, j3, j4, j5, j6])
    sza = szb = szc = 0.5
    sra = srb = src = 0.1
    if np.abs(x_a) >= 600.0:
        sza, sra = 0.1, 0.5
    if np.abs(x_b) >= 600.0:
        szb, srb = 0.1, 0.5
    if np.abs(x_c) >= 600.0:
        szc, src = 0.1, 0.5
    Sm = np.diag([sza**2, szb**2, szc**2, sra**2, srb**2, src**2]).astype(float)
    inv_cov_delta_tau = 1 / J.dot(Sm).dot(J.T)
    dz1, dr1 = z_b - z_a, r_b - r_a
    dz2, dr2 = z_c - z_a, r_c - r_a
    tau1, tau2 = dz1 / dr1, dz2 / dr2
    theta1, theta2 = atan2(dz1, dr1), atan2(dz2, dr2)
    distance2 = (tau1 - tau2)**2 * inv_cov_delta_tau
    return distance1 + distance2, (tau1 + tau2) / 2, (theta1 + theta2) / 2, theta1 - theta2


def updated_state_pairs(g: TrackGraph, truth=None):
    """a15 pair loop (calculate_distance_between_updated_track_states.py:134-195): for every
    node with an updated_track_states dict (:143) and more than one active in-edge
    (:139-140), every pair i > j of the dict's entries in dict order (:174-176), with the
    node's and the neighbours' node attribute xyzr (:162-163, :182-183) and the pair truth
    flag (:190-193). Returns pair_ptr [N+1] and a dict of per-pair arrays."""
    S = g.slot
    sp = g.slot_ptr
    ptr = np.zeros(g.n_nodes + 1, np.int64)
    cols = {"chi2": [], "avg_tau": [], "avg_theta": [], "delta_theta": [], "truth": []}
    for v in range(g.n_nodes):
        lo, hi = sp[v], sp[v + 1]
        nact = int(np.sum((S["is_edge"][lo:hi] == 1) & (S["act"][lo:hi] == 1)))
        n = 0
        if g.node["has_uts"][v] == 1 and nact > 1:
            keys = _dict_order(g, "uts", v)
            for i in range(len(keys)):
                for j in range(i):
                    ki, kj = keys[i], keys[j]
                    ui, uj = S["slot_src"][ki], S["slot_src"][kj]
                    if ui < 0 or uj < 0:
                        raise ReferenceError_("KeyError: neighbour not in the subgraph (:182-183)")
                    mi = np.array([S["uts_sv"][ki][0], S["uts_sv"][ki][1], S["uts_tau"][ki]])
                    mj = np.array([S["uts_sv"][kj][0], S["uts_sv"][kj][1], S["uts_tau"][kj]])
                    r = mahalanobis_distance_updated(mi, mat_from_cov5(S["uts_cov"][ki]), mj,
                                                     mat_from_cov5(S["uts_cov"][kj]), g.node["xyzr"][v],
                                                     g.node["xyzr"][ui], g.node["xyzr"][uj])
                    for c, x in zip(("chi2", "avg_tau", "avg_theta", "delta_theta"), r):
                        cols[c].append(x)
                    t = 0
                    if truth is not None:
                        t = int(truth[v] == truth[ui] and truth[ui] == truth[uj] and truth[v] == truth[uj])
                    cols["truth"].append(t)
                    n += 1
        ptr[v + 1] = ptr[v] + n
    out = {k: np.array(x, np.float64) for k, x in cols.items() if k != "truth"}
    out["truth"] = np.array(cols["truth"], np.int8)
    return ptr, out


def KLDistance(mean1, cov1, mean2, cov2):                                        # clustering.py:90-94
    inv1 = np.linalg.inv(cov1)
    inv2 = np.linalg.inv(cov2)
    trace = np.trace((cov1 - cov2) * (inv2 - inv1))
    return trace + (mean1 - mean2).T.dot(inv1 + inv2).dot(mean1 - mean2)


def merge_states(mean1, cov1, mean2, cov2):                                      # clustering.py:97-105
    inv1 = np.linalg.inv(cov1)
    inv2 = np.linalg.inv(cov2)
    merged_cov = np.linalg.inv(inv1 + inv2)
    merged_mean = inv1.dot(mean1) + inv2.dot(mean2)
    merged_mean = merged_cov.dot(merged_mean)
    return merged_mean, merged_cov


def get_smallest_dist_idx(distances):                                            # clustering.py:114-124
    if isinstance(distances, list):
        smallest = np.min(distances)
        return smallest, distances.index(smallest)
    nonzero = distances[np.nonzero(distances)]
    smallest = np.min(nonzero)
    row, column = np.where(distances == smallest)
    return smallest, np.concatenate((row, column), axis=None)


def cluster_node(g, pfx, v, chi2_threshold, KL_threshold, p, tie_policy="raise"):
    """One node of clustering.cluster (clustering.py:197-307). Returns the list
    of slots whose in-edge gets deactivated, or None when no merge happened."""
    S = g.slot
    order = _dict_order(g, pfx, v)
    num = len(order)
    if num <= 2 or num >= 16:                                                     # :207
        return None
    nbrs = np.array(order)
    psv = np.array([S[pfx + "_sv"][k] for k in order])
    pcov = np.array([mat_from_cov5(S[pfx + "_cov"][k]) for k in order])       # edge_covariance is the joint cov
    priors = np.array([S[pfx + "_prior"][k] for k in order])
    node_coords = g.node["xyzr"][v]
    nb_coords = np.array([S[pfx + "_xyzr"][k] for k in order])
    jsv = np.array([[S[pfx + "_sv"][k][0], S[pfx + "_sv"][k][1], S[pfx + "_tau"][k]] for k in order])
    jcov = pcov.copy()
    D = np.zeros((num, num))
    for i in range(num):                                                          # :80-86
        for j in range(i):
            D[i][j] = mahalanobis_distance(jsv[i], jcov[i], jsv[j], jcov[j], node_coords, nb_coords[i],
                                           nb_coords[j], p.sigma0rz, p.sigma0rz2, p.endcap_boundary)
    if not np.any(D):
        raise ReferenceError_("ValueError: all pairwise distances are zero (clustering.py:120)")
    smallest, idx = get_smallest_dist_idx(D)
    if not (smallest < chi2_threshold):                                          # :228
        return None
    pm, pc = merge_states(psv[idx[0]], pcov[idx[0]], psv[idx[1]], pcov[idx[1]])
    jm, jc = merge_states(jsv[idx[0]], jcov[idx[0]], jsv[idx[1]], jcov[idx[1]])
    mprior = priors[idx[0]] + priors[idx[1]]
    psv = np.delete(psv, idx, axis=0); pcov = np.delete(pcov, idx, axis=0)
    jsv = np.delete(jsv, idx, axis=0); jcov = np.delete(jcov, idx, axis=0)
    priors = np.delete(priors, idx)
    nbrs = np.delete(nbrs, idx, axis=0)
    num = psv.shape[0]
    tie_stop = False
    if num == 0:
        if tie_policy == "raise":
            raise ReferenceError_("ValueError: tie emptied the state list (clustering.py:116)")
        tie_stop = True
    if not tie_stop:
        dists = [KLDistance(jsv[i], jcov[i], jm, jc) for i in range(num)]
        smallest, idx = get_smallest_dist_idx(dists)
        while smallest < KL_threshold:                                            # :261
            pm, pc = merge_states(psv[idx], pcov[idx], pm, pc)
            jm, jc = merge_states(jsv[idx], jcov[idx], jm, jc)
            mprior = priors[idx] + mprior
            psv = np.delete(psv, idx, axis=0); pcov = np.delete(pcov, idx, axis=0)
            jsv = np.delete(jsv, idx, axis=0); jcov = np.delete(jcov, idx, axis=0)
            priors = np.delete(priors, idx)
            nbrs = np.delete(nbrs, idx, axis=0)
            num = psv.shape[0]
            if len(nbrs) == 0:
                break
            dists = [KLDistance(jsv[i], jcov[i], jm, jc) for i in range(num)]
            smallest, idx = get_smallest_dist_idx(dists)
    g.node["has_merged"][v] = 1                                                   # :291-293
    g.node["merged_state"][v] = pm
    g.node["merged_cov"][v] = cov5_from_mat(pc)
    g.node["merged_prior"][v] = mprior
    return [int(k) for k in nbrs]


def cluster_stage(g: TrackGraph, pfx: str, chi2_threshold: float, KL_threshold: float, p,
                  tie_policy="raise") -> dict:
    """clustering.cluster body after loading (clustering.py:181-373)."""
    deact = []
    merged = 0
    for v in range(g.n_nodes):
        if not _has(g, pfx, v):
            continue
        r = cluster_node(g, pfx, v, chi2_threshold, KL_threshold, p, tie_policy)
        if r is not None:
            merged += 1
            deact.extend(r)
    for k in deact:                                                               # :311-321
        if g.slot["is_edge"][k]:
            g.slot["act"][k] = 0
    query_node_degree_in_edges(g)                                                 # :324-327
    compute_mixture_weights(g, pfx)                                               # :372
    compute_prior_probabilities(g, pfx)                                           # :373
    return {"merged_nodes": merged}


def full_pass(g: TrackGraph, p, tie_policy="stop") -> dict:
    """The benchmarked pass: extrapolate stage -> update stage -> clustering on
    updated_track_states (run_gnn_trackml_mod.sh:101,138,112 order)."""
    info = extrapolate_stage(g, p)
    update_stage(g, p)
    info.update(cluster_stage(g, "uts", p.cluster_chi2, p.cluster_kl, p, tie_policy))
    return info


# ---------------------------------------------------------------------------
# a16: tag propagation  (tag_propagation/tag_propagation.py:64-164)
# ---------------------------------------------------------------------------
def tag_propagation(g: TrackGraph, threshold: float = 0.1):
    """Returns (final tags [N], number of tags flipped per sweep)."""
    N = g.n_nodes
    r = g.node["gnn"][:, 3] if np.all(np.isnan(g.node["xyzr"][:, 3])) else g.node["xyzr"][:, 3]
    # A = to_dict_of_dicts: successors (:67); keep neighbours with r_nbr <= r_node (:99-110)
    dst = g.slot_dst()
    proc = {}
    for u in range(N):
        nb = []
        for e in range(g.out_ptr[u], g.out_ptr[u + 1]):
            w = int(dst[g.out_slot[e]])
            if not (r[w] > r[u]):
                nb.append(w)
        if nb:
            proc[u] = nb
    tags = g.node["tag"].copy()
    flips_hist = []
    total = len(proc)
    frac = 1.0
    while frac > threshold:                                                       # :137
        new = tags.copy()
        flips = 0
        for u, nb in proc.items():
            t = max([tags[u]] + [tags[w] for w in nb])                            # :148 max
            new[u] = t
            if tags[u] != t:
                flips += 1
        flips_hist.append(flips)
        frac = flips / total if total else 0.0
        tags = new
    return tags, flips_hist


# ---------------------------------------------------------------------------
# a17: parabolic 3-parameter state + pairwise KL
# learn_KL_parabolic_model/src/generate_training_data/utils.py:221-299,
# extract_metadata_trackml_parabolic_model.py:15-99
# ---------------------------------------------------------------------------
def parabolic_states(gnn_node, gnn_nbrs):
    """track_state_estimates of one node for its neighbours (utils.py:221-289)."""
    S = np.array([[4.0**2, 0, 0], [0, 0.1**2, 0], [0, 0, 0.1**2]])
    coords = [(0.0, 0.0), (gnn_node[0], gnn_node[1])] + [(c[0], c[1]) for c in gnn_nbrs]
    coords.reverse()
    # rotate_track (utils.py:197-218): p1 = origin, p2 = node
    p1, p2 = coords[-1], coords[-2]
    a = atan2(p2[1] - p1[1], p2[0] - p1[0])
    while a < 0.0:
        a += math.pi * 2
    angle = 2 * math.pi - a
    rotated = []
    for c in coords:
        x, y = c[0], c[1]
        rotated.append((x * np.cos(angle) - y * np.sin(angle), x * np.sin(angle) + y * np.cos(angle)))
    xt, yt = rotated[-2][0], rotated[-2][1]
    tc = [(rc[0] - xt, rc[1] - yt) for rc in rotated]
    x_0 = tc[-1][0]
    out = []
    for tnc in tc[:-2]:
        x_B, m_B = tnc[0], tnc[1]
        H = np.array([[x_0**2, x_0, 1], [0, 0, 1], [x_B**2, x_B, 1]])
        H_inv = np.linalg.inv(H)
        sv = H_inv.dot([0.0, 0.0, m_B])
        cov = H_inv.dot(S).dot(H_inv.T)
        out.append((sv, cov))
    out.reverse()          # back to neighbour order (keys were reversed too)
    return out


def parabolic_kl_pairs(svs, covs):
    """calc_pairwise_distances (extract_metadata_trackml_parabolic_model.py:15-25):
    lower triangle i > j, row-major."""
    inv = np.linalg.inv(np.asarray(covs))
    out = []
    for i in range(len(svs)):
        for j in range(i):
            trace = np.trace((covs[i] - covs[j]) * (inv[j] - inv[i]))
            out.append(trace + (svs[i] - svs[j]).T.dot(inv[i] + inv[j]).dot(svs[i] - svs[j]))
    return out


def parabolic_training_rows(g: TrackGraph, truth=None):
    """(kl_dist, emp_var, truth) rows of extract_metadata_trackml_parabolic_model.py:56-99
    for every node with >= 2 in-edges (:61-62), pairs i > j in slot order per node.

    States: utils.py:221-289 (parabolic_states above). emp_var: np.var of the
    gradients dy/dx over nx.all_neighbors = predecessors then successors
    (utils.py:240-254, :286), here the in-slot list then the out-list.
    truth: 1 iff node, neighbour i and neighbour j share truth_particle (:82-95).
    Returns (node, i, j, kl, emp_var, truth) arrays."""
    gnn = g.node["gnn"]
    src = g.slot["slot_src"]
    dst = g.slot_dst()
    rows = []
    for v in range(g.n_nodes):
        lo, hi = int(g.slot_ptr[v]), int(g.slot_ptr[v + 1])
        d = hi - lo
        if d <= 1:
            continue
        nb = list(src[lo:hi]) + list(dst[g.out_slot[g.out_ptr[v]:g.out_ptr[v + 1]]])
        grads = [(gnn[v][1] - gnn[u][1]) / (gnn[v][0] - gnn[u][0]) for u in nb]
        with np.errstate(all="ignore"):
            emp_var = float(np.var(grads))
        st = parabolic_states(gnn[v], gnn[src[lo:hi]])
        kl = parabolic_kl_pairs([s for s, _ in st], [c for _, c in st])
        t = 0
        for i in range(d):
            for j in range(i):
                tr = 0
                if truth is not None:
                    tn, ti, tj = truth[v], truth[src[lo + i]], truth[src[lo + j]]
                    tr = int(tn == ti and ti == tj and tn == tj)
                rows.append((v, i, j, kl[t], emp_var, tr))
                t += 1
    if not rows:
        z = np.zeros(0)
        return z.astype(np.int64), z.astype(np.int64), z.astype(np.int64), z, z, z.astype(np.int8)
    a = list(zip(*rows))
    return (np.asarray(a[0], np.int64), np.asarray(a[1], np.int64), np.asarray(a[2], np.int64),
            np.asarray(a[3], np.float64), np.asarray(a[4], np.float64), np.asarray(a[5], np.int8))


def compute_track_state_estimates(g: TrackGraph, p):
    """helper.compute_track_state_estimates (helper.py:238-452) on the packed layout.

    The dict order of each node's track_state_estimates is the INPUT ``tse_rank``
    (the reference's reversed(set(nx.all_neighbors)) order); the
    set order is its reverse. Writes tse_sv, tse_cov (aliased, :417-425), tse_tau,
    tse_xyzr, tse_theta (theta, theta2, variance_theta), tse_var_ms per slot and
    returns the node arrays (xy_mean_var, zr_mean_var, angle_of_rotation,
    translation). The per-neighbour lists gradients_zr / del_tau / theta are
    filled in set order but read with the dict-order index (:384, :419-431) --
    reproduced as is."""
    S = np.array([[4.0**2, 0, 0], [0, p.sigma0xy**2, 0], [0, 0, p.sigma0xy**2]])
    gnn = g.node["gnn"]
    N = g.n_nodes
    xy_mv = np.full((N, 2), np.nan)
    zr_mv = np.full((N, 2), np.nan)
    ang = np.full(N, np.nan)
    trans = np.full((N, 2), np.nan)
    sl = g.slot
    for v in range(N):
        dict_order = _dict_order(g, "tse", v)
        set_order = dict_order[::-1]
        xA, yA, zA, rA = gnn[v]
        sigma_r, sigma_z = p.sigma0rz, p.sigma0rz2                                    # :269-274
        if np.abs(zA) >= p.endcap_boundary:
            sigma_z, sigma_r = p.sigma0rz, p.sigma0rz2
        gxy, gzr, del_tau, th, th2, del_th = [], [], [], [], [], []
        for k in set_order:                                                          # :277-338
            u = sl["slot_src"][k]
            x2, y2, z2, r2 = gnn[u]
            gxy.append((y2 - yA) / (x2 - xA))
            r1, z1 = rA, zA
            gzr.append((z2 - z1) / (r2 - r1))
            szn, srn = p.sigma0rz2, p.sigma0rz
            if np.abs(z2) >= p.endcap_boundary:
                szn, srn = p.sigma0rz, p.sigma0rz2
            J = np.array([1 / (r1 - r2), -1 / (r1 - r2), -(z1 - z2) / (r1 - r2)**2, (z1 - z2) / (r1 - r2)**2])
            S2 = np.diag([sigma_z**2, szn**2, sigma_r**2, srn**2])
            del_tau.append(J.dot(S2).dot(J.T))
            tau = gzr[-1]
            th.append(np.arctan(1 / tau))
            th2.append(np.arctan2(r2 - r1, z2 - z1))
            pre = -1 / (1 + tau**2)
            J = np.array([pre / (r1 - r2), -pre / (r1 - r2), (-pre * (z1 - z2)) / (r1 - r2)**2,
                          (pre * (z1 - z2)) / (r1 - r2)**2])
            del_th.append(J.dot(S2).dot(J.T))
        azimuth = atan2(yA, xA)                                                      # :352-365
        ca, sa = np.cos(azimuth), np.sin(azimuth)
        x_0 = (0.0 - xA) * ca + (0.0 - yA) * sa
        for i, k in enumerate(dict_order):                                           # :371-437
            u = sl["slot_src"][k]
            xk, yk, zk, rk = gnn[u]
            x_B = (xk - xA) * ca + (yk - yA) * sa
            m_B = -(xk - xA) * sa + (yk - yA) * ca
            H = np.array([[0.5 * x_0**2, x_0, 1], [0.0, 0.0, 1], [0.5 * x_B**2, x_B, 1]])
            H_inv = np.linalg.inv(H)
            sv = H_inv.dot([0.0, 0.0, m_B])
            a, b = sv[0], sv[1]
            dr, dz = rA - rk, zA - zk
            hyp = np.sqrt(dr**2 + dz**2)
            sin_t = np.abs(dr) / hyp
            kappa = (2 * a) / (1 + ((2 * a * xk) + b)**2)**1.5
            var_ms = sin_t * ((13.6 * 1e-3 * np.sqrt(0.02) * kappa) / 0.3)**2
            if np.abs(zA) >= p.endcap_boundary:
                var_ms = var_ms * np.abs(dr / dz)
            cov = H_inv.dot(S).dot(H_inv.T)
            cov[1, 1] += var_ms
            sl["tse_sv"][k] = sv
            sl["tse_tau"][k] = gzr[i]
            sl["tse_cov"][k] = (cov[0, 0], cov[0, 1], cov[1, 0], cov[1, 1], del_tau[i]**2 + var_ms)
            sl["tse_xyzr"][k] = (xk, yk, zk, rk)
            sl["tse_theta"][k] = (th[i], th2[i], del_th[i]**2 + var_ms)
            sl["tse_var_ms"][k] = var_ms
        with np.errstate(all="ignore"):
            xy_mv[v] = (np.mean(gxy), np.var(gxy))
            zr_mv[v] = (np.mean(gzr), np.var(gzr))
        ang[v] = azimuth
        trans[v] = (xA, yA)
    return {"xy_mean_var": xy_mv, "zr_mean_var": zr_mv, "angle_of_rotation": ang, "translation": trans}


# ---------------------------------------------------------------------------
# candidate extraction (src/extract/extract_track_candidates.py, §8f next #1)
# ---------------------------------------------------------------------------
def active_components(g: TrackGraph):
    """CCA (extract_track_candidates.py:332-346) per subgraph: weakly connected
    components over the activated edges, in nx.weakly_connected_components order
    (by first node), nodes ascending; a subgraph with no deactivated edge stays one
    candidate (:342-343), connected or not. Returns a list of (subgraph, nodes)."""
    N = g.n_nodes
    sub = g.node["sub_id"]
    parent = np.arange(N)

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a
    dst = g.slot_dst()
    ise = g.slot["is_edge"].astype(bool)
    act = g.slot["act"] == 1
    src = g.slot["slot_src"]
    inactive_sub = np.zeros(int(sub.max()) + 1 if N else 0, bool)
    for k in np.nonzero(ise)[0]:
        u, v = int(src[k]), int(dst[k])
        if act[k]:
            ru, rv = find(u), find(v)
            if ru != rv:
                parent[max(ru, rv)] = min(ru, rv)
        else:
            inactive_sub[sub[v]] = True
    out = []
    starts = np.r_[0, np.nonzero(np.diff(sub))[0] + 1, N] if N else np.zeros(1, np.int64)
    for a, b in zip(starts[:-1], starts[1:]):
        s = int(sub[a])
        nodes = np.arange(a, b)
        if not inactive_sub[s]:
            out.append((s, nodes))
            continue
        roots = np.array([find(v) for v in nodes])
        seen = {}
        for v, r in zip(nodes, roots):
            seen.setdefault(r, []).append(v)
        for r in sorted(seen, key=lambda r: seen[r][0]):
            out.append((s, np.asarray(seen[r])))
    return out


def check_close_proximity_nodes(nodes, vivl, xyzr, gnn, threshold):
    """extract_track_candidates.py:56-152 on one candidate (nodes in candidate order).
    Mutates gnn (the shared GNN_Measurement objects) like the reference; returns
    (assess_nodes, assess_xyzr, merged) -- the merged copy's nodes and coordinates, or
    the candidate's own when no merge copy survives."""
    ids = [tuple(vivl[v]) for v in nodes]
    freq = {}
    for x in ids:
        freq[x] = freq.get(x, 0) + 1
    fc = list(freq.values())
    coords = {int(v): tuple(xyzr[v]) for v in nodes}
    merged = False
    copied = None
    if 2 in fc:
        rest = [c for c in fc if c != 2]
        if len(fc) - len(rest) <= 2 and not any(c != 1 for c in rest):
            dups = list(set([t for t in ids if ids.count(t) > 1]))
            copied = (list(int(v) for v in nodes), dict(coords))
            for dup in dups:
                idx = [i for i, x in enumerate(ids) if x == dup]
                noi = [int(nodes[i]) for i in idx]
                if len(noi) == 2:
                    n1, n2 = noi
                    c1, c2 = copied[1][n1], copied[1][n2]
                    dist = np.sqrt((c1[0] - c2[0])**2 + (c1[1] - c2[1])**2 + (c1[2] - c2[2])**2)
                    if dist <= threshold:
                        xm, ym, zm = (c1[0] + c2[0]) / 2, (c1[1] + c2[1]) / 2, (c1[2] + c2[2]) / 2
                        rm = np.sqrt(xm**2 + ym**2)
                        gnn[n1] = (xm, ym, zm, rm)
                        copied[1][n1] = (xm, ym, zm, rm)
                        copied[0].remove(n2)
                        merged = True
                    else:
                        copied = None
                        break
                else:
                    copied = None
                    break
    if copied is None:
        return [int(v) for v in nodes], coords, merged
    return copied[0], copied[1], merged


def rotate_track(coords, separation_3d_threshold):                            # :176-195
    p1, p2 = coords[-1], coords[-2]
    d = np.sqrt((p1[0] - p2[0])**2 + (p1[1] - p2[1])**2 + (p1[2] - p2[2])**2)
    if d < separation_3d_threshold:
        p2 = coords[-3]
    axy = atan2(p2[1] - p1[1], p2[0] - p1[0])
    azr = atan2(p2[2] - p1[2], p2[3] - p1[3])
    out = []
    for c in coords:
        x, y, z, r = c[0], c[1], c[2], c[3]
        out.append((x * np.cos(axy) + y * np.sin(axy), -x * np.sin(axy) + y * np.cos(axy),
                    -z * np.sin(azr) + z * np.cos(azr), r * np.cos(azr) + r * np.sin(azr)))
    return out


def _kf_step(x, P, F, Q, H, R, z):
    """filterpy 1.4.5 predict() then update(z) (Q may be a scalar: broadcast, as filterpy)."""
    x = F.dot(x)
    P = F.dot(P).dot(F.T) + Q
    y = z - H.dot(x)
    PHT = P.dot(H.T)
    S = H.dot(PHT) + R
    K = PHT.dot(np.linalg.inv(S))
    x = x + K.dot(y)
    IKH = np.eye(len(x)) - K.dot(H)
    P = IKH.dot(P).dot(IKH.T) + K.dot(R).dot(K.T)
    return x, P


def kf_track_fit_moliere(sigma0xy, sigma0rz, coords, endcap_boundary):         # :209-327
    from scipy.stats import distributions
    f_x = np.array([coords[0][1], 0., 0.])
    f_P = np.array([[sigma0xy**2, 0., 0.], [0., 1., 0.], [0., 0., 1.]])
    f_H = np.array([[1., 0., 0.]])
    f_R = sigma0xy**2
    g_x = np.array([coords[0][3], 0.])
    g_P = np.array([[sigma0rz**2, 0.], [0., 1000.]])
    g_H = np.array([[1., 0.]])
    g_R = sigma0rz**2
    c2xy, c2zr = [], []
    for i in range(len(coords) - 1):
        x2, y2 = coords[i][0], coords[i][1]
        x3, y3 = coords[i + 1][0], coords[i + 1][1]
        x1, y1 = .0, .0
        denom = (x1 - x2) * (x1 - x3) * (x2 - x3)                              # calc_parabola_params
        a = ((x3 * (y2 - y1)) + (x2 * (y1 - y3)) + (x1 * (y3 - y2))) / denom
        b = ((x3**2 * (y1 - y2)) + (x2**2 * (y3 - y1)) + (x1**2 * (y2 - y3))) / denom
        z2, r2 = coords[i][2], coords[i][3]
        z3, r3 = coords[i + 1][2], coords[i + 1][3]
        dr, dz = r3 - r2, z3 - z2
        hyp = np.sqrt(dr**2 + dz**2)
        sin_t = np.abs(dr) / hyp
        kappa = (2 * a) / (1 + ((2 * a * x3) + b)**2)**1.5
        var_ms = sin_t * ((13.6 * 1e-3 * np.sqrt(0.02) * kappa) / 0.3)**2
        if np.abs(z3) >= endcap_boundary:
            var_ms = var_ms * np.abs(dr / dz)
        dx = x3 - x2
        alpha = 0.1
        e1 = np.exp(-np.abs(dx) * alpha)
        f1 = (1.0 - e1) / alpha
        g1 = (np.abs(dx) - f1) / alpha
        sw2 = 0.00001**2
        st2 = var_ms
        dx2 = dx**2
        dxw2 = dx2 * sw2
        Q02 = 0.5 * dxw2
        Q01 = dx * (st2 + Q02)
        Q12 = dx * sw2
        F = np.array([[1., dx, g1], [0., 1., f1], [0., 0., e1]])
        Q = np.array([[dx2 * (st2 + 0.25 * dxw2), Q01, Q02], [Q01, st2 + dxw2, Q12], [Q02, Q12, sw2]])
        f_x, f_P = _kf_step(f_x, f_P, F, Q, f_H, f_R, y3)
        res = y3 - f_H.dot(f_x)
        S = f_H.dot(f_P).dot(f_H.T) + f_R
        c2xy.append(res.T.dot(np.linalg.inv(S)).dot(res))
        G = np.array([[1., dz], [0., 1.]])
        g_x, g_P = _kf_step(g_x, g_P, G, var_ms, g_H, g_R, r3)
        res = r3 - g_H.dot(g_x)
        S = g_H.dot(g_P).dot(g_H.T) + g_R
        c2zr.append(res.T.dot(np.linalg.inv(S)).dot(res))
    dof = len(coords) - 2
    return (float(distributions.chi2.sf(sum(c2xy), dof)), float(distributions.chi2.sf(sum(c2zr), dof)))


def extract_candidates(g: TrackGraph, vivl, p_accept, fragment, separation, merge_threshold, sigma0xy,
                       sigma0rz, endcap_boundary):
    """extract_track_candidates.main (:349-467) on the packed graph. vivl: [N,2]
    (volume_id, in_volume_layer_id). Candidate node order is ascending node index
    (the reference iterates networkx subgraph views, whose order can follow a Python
    set for small components). Returns extracted candidates (node
    index arrays) with p-values in extraction order, remaining and fragment node
    sets, the mutated GNN coordinates, and per-candidate records."""
    gnn = g.node["gnn"].copy()
    xyzr = g.node["xyzr"]
    comps = active_components(g)
    extracted, pxy, pzr, records = [], [], [], []
    removed = np.zeros(g.n_nodes, bool)
    for s, nodes in comps:
        rec = {"sub": s, "nodes": nodes, "status": "fragment", "pval_xy": np.nan, "pval_zr": np.nan}
        records.append(rec)
        if len(nodes) < fragment:
            continue
        an, ac, merged = check_close_proximity_nodes(nodes, vivl, xyzr, gnn, merge_threshold)
        rec["merged"] = merged
        ids = [tuple(vivl[v]) for v in an]
        if not (len(ids) == len(set(ids)) and len(set(ids)) >= fragment):
            rec["status"] = "bad"
            continue
        coords = sorted([ac[v] for v in an], key=lambda c: c[3], reverse=True)
        coords = rotate_track(coords, separation)
        pv, pz = kf_track_fit_moliere(sigma0xy, sigma0rz, coords, endcap_boundary)
        rec["pval_xy"], rec["pval_zr"] = pv, pz
        if pv >= p_accept and pz >= p_accept:
            rec["status"] = "extracted"
            extracted.append(np.asarray(nodes))
            pxy.append(pv)
            pzr.append(pz)
            removed[nodes] = True
        else:
            rec["status"] = "rejected"
    sub = g.node["sub_id"]
    remaining, fragments = [], []
    for s in range(int(sub.max()) + 1 if g.n_nodes else 0):
        left = np.nonzero((sub == s) & ~removed)[0]
        if 0 < len(left) < fragment:
            fragments.append(left)
        elif len(left) >= fragment:
            remaining.append(left)
    return {"extracted": extracted, "pval_xy": np.asarray(pxy), "pval_zr": np.asarray(pzr),
            "remaining": remaining, "fragments": fragments, "gnn_after": gnn, "records": records}
