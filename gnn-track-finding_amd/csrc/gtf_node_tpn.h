// gtf_node_tpn.h -- the node-local op sequence with ONE THREAD per receiver node, for nodes of
// at most D slots (the fused node kernel's smallest bucket: D = 2).
//
// Why: a lane group of G lanes per node (gtf_node_group.h) turns every per-node reduction
// into ballots, shuffles and LDS round trips. For a node of one or two slots those chains
// are the whole cost of the op (the 2-lane bucket's waves lived 19k cycles on C4 with the
// loads and stores ~7k of it, profiles/r05/diag/op_timing.json), and a wave holds only 32
// nodes. Here a thread holds its node's D slots in registers and every reduction is a few
// register operations; a wave holds 64 nodes. The slot loads stay coalesced: consecutive
// threads take consecutive nodes of the tiled schedule, whose slot segments are adjacent.
//
// The arithmetic is the group form's, term for term (the same products and quotients, the
// same dict-order sums, the same LDS table of correctly rounded reciprocals), so the two
// forms give the same bits; tests/test_gpu_c4_digest.py and the parity fixtures hold both.
// A node with more than two present keys never reaches this path (clustering needs >= 3,
// clustering.py:207), so the op set needs no clustering here.
#pragma once

template <int D>
struct TCtx {
    static_assert(D >= 1 && D <= 8, "a handful of slots per thread");
    int v, lo, d;
    unsigned valid;                       // bit j: slot lo + j exists (j < d)
    unsigned edge, rev, act, act0;        // is_edge, rev_edge, activated (now / at load)
    unsigned fresh, live;                 // gtf_states.fresh bits 0 / 1 of the UTS entry
    bool use_cls;                         // graph-static classes (gtf_graph.slot_class)
    uint64_t cls[D];                      // the slot's class word (bits over the segment)
    unsigned sfl;                         // bit j: slot_sflags bit 0 (sender x < receiver x)
    double layer[D];                      // sender layer (without the static classes)
    uint64_t slm;                         // same-layer masks (lazy): slot j's at bits [j D, j D + D)
    bool sl_ok;
    uint64_t sxm;                         // same-x masks of the UTS entries (lazy), packed alike
    unsigned left;                        // bit j: the entry's x < the receiver's x (with sx)
    bool sx_ok;
    int rt[D], ru[D];                     // TSE / UTS dict ranks (-1 absent)
    double prt[D];                        // TSE prior
    double mwu[D], pru[D], lik[D], smw[D];
    double emw[D];                        // edge mixture weight
    int lri[D];                           // side-norm divisor (-1: lr = NaN, a fresh entry)
    int8_t side[D];
    unsigned dt_rank, dt_prior;           // dirty: TSE rank / prior
    unsigned du_rank, du_mw, du_prior;    // dirty: UTS rank / mw / prior
    unsigned d_lr, d_emw;                 // dirty: UTS lr + side / edge weight
    int degree;
    bool degree_set;
    uint8_t solo;
};

__device__ __forceinline__ bool tbit(unsigned m, int j) { return (m >> j) & 1u; }
// slot j's mask of a packed per-slot mask word (D bits each)
template <int D>
__device__ __forceinline__ unsigned tmask(uint64_t w, int j) { return (unsigned)(w >> (j * D)) & ((1u << D) - 1u); }

// the dict positions of the present keys: pos[j] = number of present keys with a smaller
// rank (the rank is the dict insertion order); -1 absent
template <int D>
__device__ __forceinline__ void t_dict_order(const TCtx<D>& c, const int* r, int* pos) {
#pragma unroll
    for (int j = 0; j < D; j++) {
        int q = 0;
#pragma unroll
        for (int i = 0; i < D; i++) q += (tbit(c.valid, i) && r[i] >= 0 && r[i] < r[j]) ? 1 : 0;
        pos[j] = (tbit(c.valid, j) && r[j] >= 0) ? q : -1;
    }
}

template <int D>
__device__ __forceinline__ unsigned t_present(const TCtx<D>& c, const int* r) {
    unsigned m = 0;
#pragma unroll
    for (int j = 0; j < D; j++) m |= (tbit(c.valid, j) && r[j] >= 0) ? (1u << j) : 0u;
    return m;
}

// lane_active: present, an edge, activated
template <int D>
__device__ __forceinline__ unsigned t_active(const TCtx<D>& c, const int* r) {
    return t_present(c, r) & c.edge & c.act;
}

// mask of the valid slots whose value equals slot j's (a NaN equals only itself)
template <int D>
__device__ __forceinline__ unsigned t_equal(const TCtx<D>& c, const double* val, int j) {
    unsigned m = 1u << j;
#pragma unroll
    for (int i = 0; i < D; i++) m |= (tbit(c.valid, i) && val[i] == val[j]) ? (1u << i) : 0u;
    return m;
}

// compute_prior_probabilities (helper.py:30-63), as g_priors
template <int D>
__device__ __forceinline__ void t_priors(TCtx<D>& c, const int* r, double* pr, unsigned& dirty) {
    if (!c.sl_ok) {
        c.slm = 0;
#pragma unroll
        for (int j = 0; j < D; j++) {
            const unsigned m = !tbit(c.valid, j) ? 0u : (c.use_cls ? (unsigned)(c.cls[j] & 0xffffffffull) : t_equal(c, c.layer, j));
            c.slm |= (uint64_t)(m & ((1u << D) - 1u)) << (j * D);
        }
        c.sl_ok = true;
    }
    const unsigned A = t_active(c, r);
#pragma unroll
    for (int j = 0; j < D; j++)
        if (tbit(A, j)) {
            pr[j] = g_rcp_lds[__popc(A & tmask<D>(c.slm, j))];
            dirty |= 1u << j;
        }
}

// calculate_side_norm_factor + reweight (helper.py:99-200), as g_reweight
template <int D>
__device__ __forceinline__ void t_reweight(TCtx<D>& c, const gtf_graph& g, const gtf_states& uts, double thr,
                                           uint32_t* err) {
    const unsigned P = t_present(c, c.ru);
    const unsigned A = P & c.edge & c.act;
    // last dict key = the present key with the largest rank (slot 0 when none)
    int last = 0, maxr = -1;
#pragma unroll
    for (int j = 0; j < D; j++)
        if (tbit(P, j) && c.ru[j] > maxr) { maxr = c.ru[j]; last = j; }
    const bool last_is_edge = tbit(c.edge, last), last_act = tbit(c.act, last);
    if (!c.sx_ok) {
        if (c.use_cls && (P & ~c.live) == 0u) {
            c.sxm = 0;
#pragma unroll
            for (int j = 0; j < D; j++)
                c.sxm |= (uint64_t)(tbit(c.valid, j) ? (unsigned)(c.cls[j] >> 32) & ((1u << D) - 1u) : 0u) << (j * D);
            c.left = c.sfl;
        } else {
            double x0[D];
            const double xr = g.gnn[4 * (int64_t)c.v];
            c.left = 0;
#pragma unroll
            for (int j = 0; j < D; j++) {
                const int64_t k = c.lo + j;
                x0[j] = !tbit(c.valid, j) ? 0.0
                        : (tbit(c.live, j) ? (g.slot_sxzr ? g.slot_sxzr[3 * k] : g.gnn[4 * (int64_t)g.slot_src[k]])
                                           : uts.xyzr[4 * k]);
                c.left |= (tbit(c.valid, j) && x0[j] < xr) ? (1u << j) : 0u;
            }
            c.sxm = 0;
#pragma unroll
            for (int j = 0; j < D; j++)
                c.sxm |= (uint64_t)(tbit(c.valid, j) ? t_equal(c, x0, j) & ((1u << D) - 1u) : 0u) << (j * D);
        }
        c.sx_ok = true;
    }
    // first active key of its distinct-x class (equal x, same side), counted per side
    int dl = 0, dr = 0;
#pragma unroll
    for (int j = 0; j < D; j++) {
        const bool first = tbit(A, j) && (tmask<D>(c.sxm, j) & A & ((1u << j) - 1u)) == 0u;
        if (first) {
            if (tbit(c.left, j)) dl++;
            else dr++;
        }
    }
    if (A != 0u) {
        if (!last_is_edge) raise_node(err, c.v, GTF_ERR_STALE_KEY_NO_EDGE);
#pragma unroll
        for (int j = 0; j < D; j++)
            if (tbit(A, j)) {
                const bool lj = tbit(c.left, j);
                c.side[j] = lj ? 0 : 1;
                c.lri[j] = (last_is_edge && last_act) ? (lj ? dl : dr) : 1;
                c.d_lr |= 1u << j;
            }
    }
    // denominator: the dict-order sum over the present keys, inactive ones adding +0.0
    int pos[D];
    t_dict_order(c, c.ru, pos);
    double term[D];
#pragma unroll
    for (int i = 0; i < D; i++) term[i] = 0.0;
#pragma unroll
    for (int j = 0; j < D; j++)
        if (pos[j] >= 0) {
            const double t = tbit(A, j) ? c.mwu[j] * c.lik[j] : 0.0;
#pragma unroll
            for (int i = 0; i < D; i++)
                if (pos[j] == i) term[i] = t;
        }
    double denom = 0.0;
    const int npres = __popc(P);
#pragma unroll
    for (int i = 0; i < D; i++)
        if (i < npres) denom = denom + term[i];
#pragma unroll
    for (int j = 0; j < D; j++)
        if (tbit(A, j)) {
            double wgt = (c.mwu[j] * c.lik[j] * c.pru[j]) / denom;
            wgt = qdiv(wgt, (double)c.lri[j], g_rcp_lds[c.lri[j]]);   // (lr = lri exactly)
            c.mwu[j] = wgt;
            c.du_mw |= 1u << j;
            c.emw[j] = wgt;
            c.d_emw |= 1u << j;
            if (wgt < thr) c.act &= ~(1u << j);
            else c.act |= 1u << j;
        }
}

template <int D>
__device__ __forceinline__ void t_fresh(TCtx<D>& c) {
#pragma unroll
    for (int j = 0; j < D; j++)
        if (tbit(c.valid & c.fresh, j)) {
            if (!GTF_MW_IN_EXTRAP) {   // (else k_extrapolate stored it)
                c.mwu[j] = c.smw[j];
                c.du_mw |= 1u << j;
            }
            c.pru[j] = NAN;
            c.du_prior |= 1u << j;
            c.lri[j] = -1;   // lr = NaN
            c.side[j] = -1;
            c.d_lr |= 1u << j;
        }
}

template <int D>
__device__ __forceinline__ void t_ranks(TCtx<D>& c) {
    int maxr = -1;
#pragma unroll
    for (int j = 0; j < D; j++)
        if (tbit(c.valid, j)) maxr = max(maxr, c.ru[j]);
    int next = maxr + 1;
#pragma unroll
    for (int j = 0; j < D; j++)
        if (tbit(c.valid & c.fresh, j) && c.ru[j] < 0) {
            c.ru[j] = next++;
            c.du_rank |= 1u << j;
        }
}

template <int D>
__device__ __forceinline__ void t_degree(TCtx<D>& c) {
    c.degree = __popc(c.valid & c.edge & c.act);
    c.degree_set = true;
}

template <int D>
__device__ __forceinline__ void t_prune(TCtx<D>& c, bool has_tse, bool has_uts, uint32_t* err) {
    if (!has_uts && !has_tse) {
        raise_node(err, c.v, GTF_ERR_NO_STATE_DICT);
        return;
    }
    // (two loops, not a pointer to either array: the arrays stay in registers)
    if (has_uts) {
#pragma unroll
        for (int j = 0; j < D; j++)
            if (tbit(c.valid, j) && c.ru[j] >= 0 && !tbit(c.rev, j)) {
                c.ru[j] = -1;
                c.du_rank |= 1u << j;
            }
    } else {
#pragma unroll
        for (int j = 0; j < D; j++)
            if (tbit(c.valid, j) && c.rt[j] >= 0 && !tbit(c.rev, j)) {
                c.rt[j] = -1;
                c.dt_rank |= 1u << j;
            }
    }
}

template <int D>
__device__ __forceinline__ void t_mixture_weights(TCtx<D>& c, uint32_t* err) {   // UTS (the pass's)
    const unsigned P = t_present(c, c.ru);
    const int cnt = __popc(P);
    if (cnt == 0) {
        if (!c.solo) raise_node(err, c.v, GTF_ERR_EMPTY_DICT_MW);
        return;
    }
#pragma unroll
    for (int j = 0; j < D; j++)
        if (tbit(P, j)) {
            c.mwu[j] = g_rcp_lds[cnt];
            c.du_mw |= 1u << j;
        }
}

// the TSE mixture weights are not in the thread form (no fused sequence updates them)
template <int... OPS>
struct TpnOk {
    static constexpr bool value = !((OPS == OP_MW_TSE || OPS == OP_CLUSTER_TSE) || ...);
};

template <int D>
__device__ __forceinline__ void t_store(TCtx<D>& c, gtf_nodes& n, gtf_states& tse, gtf_states& uts, gtf_edges& e,
                                        bool flush_only) {
#pragma unroll
    for (int j = 0; j < D; j++) {
        if (!tbit(c.valid, j)) continue;
        const int64_t k = c.lo + j;
        if (!flush_only && tbit(c.act ^ c.act0, j)) e.act[k] = tbit(c.act, j) ? 1 : 0;
        if (tbit(c.d_emw, j)) e.edge_mw[k] = c.emw[j];
        if (tbit(c.dt_rank, j)) tse.rank[k] = c.rt[j];
        if (tbit(c.dt_prior, j)) tse.prior[k] = c.prt[j];
        if (tbit(c.du_rank, j)) uts.rank[k] = c.ru[j];
        if (!flush_only && tbit(c.du_mw, j)) uts.mw[k] = c.mwu[j];
        if (!flush_only && tbit(c.du_prior, j)) uts.prior[k] = c.pru[j];
        if (tbit(c.d_lr, j)) {
            uts.lr[k] = c.lri[j] < 0 ? (double)NAN : (double)c.lri[j];
            uts.side[k] = c.side[j];
        }
    }
    // (OP_FLUSH: the fields no later op changes; node_flush's set)
    c.d_emw = 0u;
    c.dt_rank = c.dt_prior = 0u;
    c.du_rank = 0u;
    c.d_lr = 0u;
    if (!flush_only && c.degree_set) n.degree[c.v] = c.degree;
}

template <int D, int OP>
__device__ __forceinline__ void t_op(TCtx<D>& c, const gtf_graph& g, gtf_nodes& n, gtf_states& tse,
                                     gtf_states& uts, gtf_edges& e, const gtf_params& p, const Ws& w, bool has_tse,
                                     bool has_uts) {
    if constexpr (OP == OP_FLUSH) t_store(c, n, tse, uts, e, true);
    if constexpr (OP == OP_FRESH) t_fresh(c);
    if constexpr (OP == OP_RANKS) t_ranks(c);
    if constexpr (OP == OP_PRIORS_TSE) { if (has_tse) t_priors(c, c.rt, c.prt, c.dt_prior); }
    if constexpr (OP == OP_PRIORS_UTS) { if (has_uts) t_priors(c, c.ru, c.pru, c.du_prior); }
    if constexpr (OP == OP_REWEIGHT_UTS) { if (has_uts) t_reweight(c, g, uts, p.reweight_threshold, w.err); }
    if constexpr (OP == OP_DEGREE) t_degree(c);
    if constexpr (OP == OP_PRUNE) t_prune(c, has_tse, has_uts, w.err);
    if constexpr (OP == OP_MW_UTS) { if (has_uts) t_mixture_weights(c, w.err); }
    // OP_CLUSTER_UTS: a node of <= 2 slots has <= 2 keys: no clustering (clustering.py:207)
    static_assert(OP != OP_CLUSTER_UTS || D <= 2, "thread-per-node clustering needs <= 2 slots");
}

// one thread per node of the bucket (list / seg as the group kernels'); `bid` = the block
// index inside the bucket's range of the launch
template <int D, int... OPS>
__device__ __forceinline__ void tpn_body(const gtf_graph& g, gtf_nodes& n, gtf_states& tse, gtf_states& uts,
                                         gtf_edges& e, const gtf_params& p, const Ws& w, const int32_t* list,
                                         const int32_t* seg, int count, int bid) {
    using Q = OpSeq<OPS...>;
    constexpr Need nd = Q::need;
    const int gi = bid * NBLOCK + (int)threadIdx.x;
#if GTF_OP_TIMING
    // (diagnostics) the group kernels' per-wave stamps, word 23 = 1 for a thread-per-node wave
    const uint64_t t_start = __builtin_readcyclecounter();
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
    const int wave = (int)((blockIdx.x * NBLOCK + threadIdx.x) / 64);
    uint64_t* tb = ((threadIdx.x & 63) == 0 && wave < GTF_OP_TIMING_WAVES) ? g_op_time + 24 * (int64_t)wave : nullptr;
    int ti = 2;
#endif
    if (gi >= count) return;
    TCtx<D> c;
    c.v = list[gi];
    if (seg) {
        const int2 sg = reinterpret_cast<const int2*>(seg)[gi];
        c.lo = sg.x;
        c.d = sg.y - sg.x;
    } else {
        c.lo = g.slot_ptr[c.v];
        c.d = g.slot_ptr[c.v + 1] - c.lo;
    }
    c.valid = c.d >= D ? (1u << D) - 1u : (1u << c.d) - 1u;
    c.use_cls = g.slot_class != nullptr;
    const bool st32 = D <= 8 && g.slot_static != nullptr;   // the static fields in one word per slot
    c.use_cls = c.use_cls || st32;
    c.edge = c.rev = c.act = c.fresh = c.live = c.sfl = 0u;
    c.sl_ok = c.sx_ok = false;
    c.left = 0u;
    c.dt_rank = c.dt_prior = c.du_rank = c.du_mw = c.du_prior = c.d_lr = c.d_emw = 0u;
    c.degree = 0;
    c.degree_set = false;
    c.solo = nd.solo ? g.solo[c.v] : 0;
#pragma unroll
    for (int j = 0; j < D; j++) {
        const bool ok = tbit(c.valid, j);
        const int64_t k = c.lo + j;
        c.cls[j] = 0;
        c.layer[j] = NAN;
        c.rt[j] = c.ru[j] = -1;
        c.prt[j] = c.mwu[j] = c.pru[j] = c.lik[j] = c.smw[j] = c.emw[j] = 0.0;
        c.lri[j] = 1;
        c.side[j] = -1;
        if (!ok) continue;
        c.act |= e.act[k] == 1 ? (1u << j) : 0u;
        if (st32) {
            const uint32_t sw = g.slot_static[k];
            c.edge |= ((sw >> 16) & 1u) << j;
            c.rev |= ((sw >> 17) & 1u) << j;
            c.sfl |= ((sw >> 18) & 1u) << j;
            c.cls[j] = (uint64_t)(sw & 0xffu) | ((uint64_t)((sw >> 8) & 0xffu) << 32);
        } else {
            c.edge |= g.is_edge[k] ? (1u << j) : 0u;
            c.rev |= g.rev_edge[k] ? (1u << j) : 0u;
        }
        if (st32) {
        } else if (c.use_cls) {
            c.cls[j] = g.slot_class[k];
            c.sfl |= (g.slot_sflags[k] & 1) ? (1u << j) : 0u;
        } else if (g.slot_layer) {
            c.layer[j] = g.slot_layer[k];
        } else {
            const int src = g.slot_src[k];
            c.layer[j] = src >= 0 ? g.layer[src] : NAN;
        }
        if (nd.tse_rank) c.rt[j] = tse.rank[k];
        if (nd.tse_prior) c.prt[j] = tse.prior[k];
        if (nd.uts_rank) c.ru[j] = uts.rank[k];
        if (nd.uts_mw) c.mwu[j] = uts.mw[k];
        if (nd.uts_prior) c.pru[j] = uts.prior[k];
        if (nd.uts_lik) c.lik[j] = uts.lik[k];
        if (nd.uts_fresh || nd.uts_live) {
            const uint8_t f = uts.fresh[k];
            c.fresh |= (f & 1) ? (1u << j) : 0u;
            c.live |= (f & 2) ? (1u << j) : 0u;
        }
        if (nd.send_mw) c.smw[j] = e.send_mw[k];
    }
    c.act0 = c.act;
    // the act byte is 0 / 1 in every graph (activated, extrapolate_merged_states.py:393); a
    // value that is neither is kept as "inactive" by the group form too (act == 1 tests)
    const bool has_tse = n.has_tse[c.v];
    bool has_uts = n.has_uts[c.v];
    if (Q::fresh && !has_uts && (c.valid & c.fresh) != 0u) {   // fresh_has_uts
        has_uts = true;
        n.has_uts[c.v] = 1;
    }
#if GTF_OP_TIMING
    {
        const uint64_t t = __builtin_readcyclecounter();
        if (tb) { tb[0] = t_start; tb[1] = t; tb[20] = rt_start; tb[23] = 1; }
    }
    (
        [&] {
            t_op<D, OPS>(c, g, n, tse, uts, e, p, w, has_tse, has_uts);
            const uint64_t t = __builtin_readcyclecounter();
            if (tb && ti < 20) tb[ti] = t;
            ti++;
        }(),
        ...);
#else
    (t_op<D, OPS>(c, g, n, tse, uts, e, p, w, has_tse, has_uts), ...);
#endif
    t_store(c, n, tse, uts, e, false);
#if GTF_OP_TIMING
    {
        const uint64_t t = __builtin_readcyclecounter();
        const uint64_t rt = __builtin_amdgcn_s_memrealtime();
        if (tb && ti < 20) tb[ti] = t;
        if (tb) tb[21] = rt;
    }
#endif
}
