// gtf_node_group.h -- the node-local op sequence with G lanes per receiver node
// (G = 16 for nodes with <= 16 slots, G = 64 for <= 64), one slot per lane.
//
// Why: every stage after message passing reduces over one node's in-edge slot
// segment. One thread per node serialises O(d^2) loops over
// uncoalesced global memory; here each lane loads ITS slot once (consecutive
// lanes = consecutive slots = coalesced), keeps the mutable fields in registers
// across the whole op sequence, and the per-node reductions (prior counts,
// side-norm distinct counts, the reweight denominator, pairwise chi2 minimum,
// KL argmin) run as group shuffles / ballots. Ordered sums (dict order) go
// through a per-group LDS line so the addition order stays the reference's
// sequential Python order. Writes happen once, at the end.
//
// Control flow that contains a shuffle is group-uniform: every branch around a
// shuffle depends only on group-reduced values, so all G lanes of the group are
// active at each shuffle.
#pragma once

template <int G>
struct Grp {
    int gl;     // lane within the group
    int gbase;  // first wave lane of the group
    __device__ __forceinline__ Grp() {
        const int lane = threadIdx.x & 63;
        gl = lane & (G - 1);
        gbase = lane & ~(G - 1);
    }
    __device__ __forceinline__ unsigned long long bits(bool pred) const {
        const unsigned long long b = __ballot(pred);
        return G == 64 ? b : ((b >> gbase) & ((1ull << G) - 1ull));
    }
    __device__ __forceinline__ int count(bool pred) const { return __popcll(bits(pred)); }
    __device__ __forceinline__ bool any(bool pred) const { return bits(pred) != 0ull; }
    template <typename T>
    __device__ __forceinline__ T shfl(T x, int src) const { return __shfl(x, src, G); }
    __device__ __forceinline__ int max_i(int x) const {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, G));
        return x;
    }
    __device__ __forceinline__ int min_i(int x) const {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, G));
        return x;
    }
    __device__ __forceinline__ double min_d(double x) const {  // NaN-free inputs
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o, G));
        return x;
    }
    __device__ __forceinline__ unsigned or_u(unsigned x) const {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x |= __shfl_xor(x, o, G);
        return x;
    }
};

// per-lane (per-slot) registers of one state dict
struct LaneDict {
    int rank;
    double mw, prior;
    bool dirty;
};

template <int G>
struct NodeCtx {
    Grp<G> grp;
    int v, lo, d, k;
    bool valid;
    uint8_t is_edge, rev_edge, act, act0;
    int src;
    double layer;
    LaneDict tse, uts;
    double lik, lr, x0, edge_mw;
    int8_t side;
    uint8_t fresh;
    bool uts_dirty_lr, edge_mw_dirty;
    int degree;
    bool degree_set;
};

// position of this lane's key in the dict order (number of present keys with a smaller rank)
template <int G>
__device__ __forceinline__ int dict_pos(const NodeCtx<G>& c, int rank) {
    int pos = 0;
    for (int j = 0; j < G; j++) {
        const int rj = c.grp.shfl(rank, j);
        pos += (rj >= 0 && rj < rank) ? 1 : 0;
    }
    return rank >= 0 ? pos : -1;
}

// sequential (dict-order) sum of `term` over lanes where `take`, every lane gets the
// sum. Lanes write their term at their dict position in a per-group LDS line and
// every lane adds the line in order; skipped entries add +0.0, which leaves the
// running sum unchanged (it starts from the integer 0 of helper.py:165).
template <int G>
__device__ __forceinline__ double ordered_sum(const NodeCtx<G>& c, volatile double* sval, int rank, bool take,
                                             double term) {
    const int pos = dict_pos(c, rank);
    const int npres = c.grp.count(rank >= 0);
    if (rank >= 0) sval[c.grp.gbase + pos] = take ? term : 0.0;
    __builtin_amdgcn_wave_barrier();
    double s = 0.0;
    for (int i = 0; i < npres; i++) s = s + sval[c.grp.gbase + i];
    __builtin_amdgcn_wave_barrier();
    return s;
}

template <int G>
__device__ __forceinline__ bool lane_active(const NodeCtx<G>& c, int rank) {
    return c.valid && rank >= 0 && c.is_edge && c.act == 1;
}

// compute_prior_probabilities (helper.py:30-63)
template <int G>
__device__ __forceinline__ void g_priors(NodeCtx<G>& c, LaneDict& st) {
    const bool act = lane_active(c, st.rank);
    int cnt = 0;
    for (int j = 0; j < G; j++) {
        const double lj = c.grp.shfl(c.layer, j);
        const int aj = c.grp.shfl((int)act, j);
        cnt += (aj && lj == c.layer) ? 1 : 0;
    }
    if (act) {
        st.prior = 1.0 / (double)cnt;
        st.dirty = true;
    }
}

// calculate_side_norm_factor + reweight (helper.py:99-200), UTS only
template <int G>
__device__ __forceinline__ void g_reweight(NodeCtx<G>& c, volatile double* sval, const double* gnn, double thr,
                                           uint32_t* err) {
    LaneDict& st = c.uts;
    const bool act = lane_active(c, st.rank);
    // last dict key = the present key with the largest rank (stale loop variable, :131,138)
    const int maxr = c.grp.max_i(c.valid ? st.rank : -1);
    const unsigned long long lastb = c.grp.bits(c.valid && st.rank == maxr && maxr >= 0);
    const int last = lastb ? __ffsll((long long)lastb) - 1 : 0;
    const int last_is_edge = c.grp.shfl((int)c.is_edge, last);
    const int last_act = c.grp.shfl((int)c.act, last);
    const double node_x = gnn[4 * (int64_t)c.v];
    const bool left = c.x0 < node_x;
    bool dup = false;
    for (int j = 0; j < G; j++) {
        const double xj = c.grp.shfl(c.x0, j);
        const int aj = c.grp.shfl((int)act, j);
        if (j < c.grp.gl && aj && ((xj < node_x) == left) && xj == c.x0) dup = true;
    }
    const int nact = c.grp.count(act);
    const int dl = c.grp.count(act && left && !dup);
    const int dr = c.grp.count(act && !left && !dup);
    if (nact > 0) {
        if (!last_is_edge && c.grp.gl == 0) atomicOr(err, (uint32_t)GTF_ERR_STALE_KEY_NO_EDGE);
        if (act) {
            c.side = left ? 0 : 1;
            c.lr = (last_is_edge && last_act == 1) ? (double)(left ? dl : dr) : 1.0;
            c.uts_dirty_lr = true;
        }
    }
    const double denom = ordered_sum(c, sval, st.rank, act, st.mw * c.lik);
    if (act) {
        double wgt = (st.mw * c.lik * st.prior) / denom;
        wgt = wgt / c.lr;
        st.mw = wgt;
        st.dirty = true;
        c.edge_mw = wgt;
        c.edge_mw_dirty = true;
        c.act = (wgt < thr) ? 0 : 1;
    }
}

template <int G>
__device__ __forceinline__ void g_degree(NodeCtx<G>& c) {
    c.degree = c.grp.count(c.valid && c.is_edge && c.act == 1);
    c.degree_set = true;
}

// remove_state_metadata pruning (:31-48)
template <int G>
__device__ __forceinline__ void g_prune(NodeCtx<G>& c, bool has_tse, bool has_uts, uint32_t* err) {
    if (!has_uts && !has_tse) {
        if (c.grp.gl == 0) atomicOr(err, (uint32_t)GTF_ERR_NO_STATE_DICT);
        return;
    }
    LaneDict& st = has_uts ? c.uts : c.tse;
    if (c.valid && st.rank >= 0 && !c.rev_edge) {
        st.rank = -1;
        st.dirty = true;
    }
}

template <int G>
__device__ __forceinline__ void g_mixture_weights(NodeCtx<G>& c, LaneDict& st, bool solo, uint32_t* err) {
    const int cnt = c.grp.count(c.valid && st.rank >= 0);
    if (cnt == 0) {
        if (!solo && c.grp.gl == 0) atomicOr(err, (uint32_t)GTF_ERR_EMPTY_DICT_MW);
        return;
    }
    if (c.valid && st.rank >= 0) {
        st.mw = 1.0 / (double)cnt;
        st.dirty = true;
    }
}

template <int G>
__device__ __forceinline__ void g_ranks(NodeCtx<G>& c) {
    LaneDict& st = c.uts;
    const int maxr = c.grp.max_i(c.valid ? st.rank : -1);
    const bool isnew = c.valid && c.fresh && st.rank < 0;
    const unsigned long long nb = c.grp.bits(isnew);
    if (isnew) {
        const unsigned long long below = nb & ((1ull << c.grp.gl) - 1ull);
        st.rank = maxr + 1 + __popcll(below);
        st.dirty = true;
    }
}

// pairwise chi2 + greedy KL merging of one node (clustering.py:197-307)
template <int G>
__device__ __forceinline__ void g_cluster(NodeCtx<G>& c, gtf_nodes& n, const gtf_states& S, LaneDict& st,
                                          volatile int* slane, const double* xyzr_node, double chi2_thr,
                                          double kl_thr, const gtf_params& p, uint32_t* err) {
    const bool pres = c.valid && st.rank >= 0;
    const int d = c.grp.count(pres);
    if (d <= 2 || d >= 16) return;                                                 // :207
    const int pos = dict_pos(c, st.rank);
    if (pres) slane[c.grp.gbase + pos] = c.grp.gl;
    __builtin_amdgcn_wave_barrier();
    // this lane's state (joint vector a, b, tau; parabolic c; covariance; sender coords)
    double a = 0, b = 0, cc = 0, tau = 0, x = 0, z = 0, r = 0, prior = 0;
    Cov5 cv{1, 0, 0, 1, 1};
    if (pres) {
        a = S.sv[3 * (int64_t)c.k];
        b = S.sv[3 * (int64_t)c.k + 1];
        cc = S.sv[3 * (int64_t)c.k + 2];
        tau = S.tau[c.k];
        cv = load_cov5(S.cov, c.k);
        x = S.xyzr[4 * (int64_t)c.k];
        z = S.xyzr[4 * (int64_t)c.k + 2];
        r = S.xyzr[4 * (int64_t)c.k + 3];
        prior = st.prior;
    }
    const double na[4] = {xyzr_node[0], xyzr_node[1], xyzr_node[2], xyzr_node[3]};
    const double mine[4] = {x, 0.0, z, r};
    // row `pos` of the lower triangle: D[pos][j], j < pos
    double rmin = INFINITY;
    int rj0 = -1, rties = 0;
    unsigned rmask = 0;
    bool rnan = false, rnz = false;
    for (int j = 0; j < d - 1; j++) {
        const int lj = slane[c.grp.gbase + j];
        const double aj = c.grp.shfl(a, lj), bj = c.grp.shfl(b, lj);
        const Cov5 cj{c.grp.shfl(cv.c00, lj), c.grp.shfl(cv.c01, lj), c.grp.shfl(cv.c10, lj),
                      c.grp.shfl(cv.c11, lj), c.grp.shfl(cv.c22, lj)};
        const double oth[4] = {c.grp.shfl(x, lj), 0.0, c.grp.shfl(z, lj), c.grp.shfl(r, lj)};
        if (pres && j < pos) {
            const double D = mahalanobis(a, b, cv, aj, bj, cj, na, mine, oth, p.sigma0rz2, p.sigma0rz, p.sigma0rz,
                                         p.sigma0rz2, p.endcap_boundary);
            if (D != 0.0) {
                rnz = true;
                if (isnan(D)) {
                    rnan = true;
                } else if (D < rmin) {
                    rmin = D; rj0 = j; rties = 1; rmask = 1u << j;
                } else if (D == rmin) {
                    rties++; rmask |= 1u << j;
                }
            }
        }
    }
    if (!c.grp.any(rnz)) {
        if (c.grp.gl == 0) atomicOr(err, (uint32_t)GTF_ERR_ALL_ZERO_DIST);
        return;
    }
    if (c.grp.any(rnan)) return;                       // np.min over a NaN -> no merge (:228)
    const double best = c.grp.min_d(rmin);
    if (!(best < chi2_thr)) return;
    // np.where(D == best) in row-major order: rows ascend with pos
    const bool tie_row = pres && rmin == best;
    const unsigned long long trb = c.grp.bits(tie_row);
    // row index (dict position) of each tie row, found via the lane map
    int ti0 = 99, tj0 = -1, ti1 = 99, t0ties = 0;
    {
        // first tie row = smallest pos among tie rows
        const int mypos_if = tie_row ? pos : 99;
        ti0 = c.grp.min_i(mypos_if);
        const int l0 = slane[c.grp.gbase + ti0];
        tj0 = c.grp.shfl(rj0, l0);
        t0ties = c.grp.shfl(rties, l0);
        const int second = (tie_row && pos != ti0) ? pos : 99;
        ti1 = (t0ties >= 2) ? ti0 : c.grp.min_i(second);
    }
    (void)trb;
    unsigned tiemask = tie_row ? (rmask | (1u << pos)) : 0u;
    tiemask = c.grp.or_u(tiemask);
    const int p0 = ti0, p1 = (ti1 < 99) ? ti1 : tj0;
    // merge the pair (every lane computes the same merge: uniform work)
    const int l0 = slane[c.grp.gbase + p0], l1 = slane[c.grp.gbase + p1];
    double ps0[3] = {c.grp.shfl(a, l0), c.grp.shfl(b, l0), c.grp.shfl(cc, l0)};
    double ps1[3] = {c.grp.shfl(a, l1), c.grp.shfl(b, l1), c.grp.shfl(cc, l1)};
    const double t0 = c.grp.shfl(tau, l0), t1 = c.grp.shfl(tau, l1);
    const Cov5 c0{c.grp.shfl(cv.c00, l0), c.grp.shfl(cv.c01, l0), c.grp.shfl(cv.c10, l0), c.grp.shfl(cv.c11, l0),
                  c.grp.shfl(cv.c22, l0)};
    const Cov5 c1{c.grp.shfl(cv.c00, l1), c.grp.shfl(cv.c01, l1), c.grp.shfl(cv.c10, l1), c.grp.shfl(cv.c11, l1),
                  c.grp.shfl(cv.c22, l1)};
    double pm[3], jm[3];
    Cov5 pc, jc;
    {
        const double js0[3] = {ps0[0], ps0[1], t0};
        const double js1[3] = {ps1[0], ps1[1], t1};
        merge_states(ps0, c0, ps1, c1, pm, pc);
        merge_states(js0, c0, js1, c1, jm, jc);
    }
    double mprior = c.grp.shfl(prior, l0) + c.grp.shfl(prior, l1);
    unsigned alive = ((1u << d) - 1u) & ~tiemask;
    bool my_alive = pres && (alive >> pos & 1u);
    if (alive == 0) {
        if (c.grp.gl == 0) atomicOr(err, (uint32_t)GTF_ERR_TIE_EMPTIED);
    } else {
        const double js_me[3] = {a, b, tau};
        while (true) {                                                             // :251-287
            double D = INFINITY;
            bool dn = false;
            if (my_alive) {
                D = kl_distance(js_me, cv, jm, jc);
                if (isnan(D)) { dn = true; D = INFINITY; }
            }
            if (c.grp.any(dn)) {
                if (c.grp.gl == 0) atomicOr(err, (uint32_t)GTF_ERR_NAN_KL);
                break;
            }
            const double mind = c.grp.min_d(D);
            if (!(mind < kl_thr)) break;
            // first minimum in dict order
            const int mpos = c.grp.min_i((my_alive && D == mind) ? pos : 99);
            const int lm = slane[c.grp.gbase + mpos];
            const double ps[3] = {c.grp.shfl(a, lm), c.grp.shfl(b, lm), c.grp.shfl(cc, lm)};
            const double js[3] = {ps[0], ps[1], c.grp.shfl(tau, lm)};
            const Cov5 ci{c.grp.shfl(cv.c00, lm), c.grp.shfl(cv.c01, lm), c.grp.shfl(cv.c10, lm),
                          c.grp.shfl(cv.c11, lm), c.grp.shfl(cv.c22, lm)};
            double npm[3], njm[3];
            Cov5 npc, njc;
            merge_states(ps, ci, pm, pc, npm, npc);
            merge_states(js, ci, jm, jc, njm, njc);
            pm[0] = npm[0]; pm[1] = npm[1]; pm[2] = npm[2]; pc = npc;
            jm[0] = njm[0]; jm[1] = njm[1]; jm[2] = njm[2]; jc = njc;
            mprior = c.grp.shfl(prior, lm) + mprior;
            alive &= ~(1u << mpos);
            my_alive = pres && (alive >> pos & 1u);
            if (alive == 0) break;
        }
    }
    if (c.grp.gl == 0) {                                                           // :291-293
        n.has_merged[c.v] = 1;
        n.merged_state[3 * (int64_t)c.v + 0] = pm[0];
        n.merged_state[3 * (int64_t)c.v + 1] = pm[1];
        n.merged_state[3 * (int64_t)c.v + 2] = pm[2];
        store_cov5(n.merged_cov, c.v, pc);
        n.merged_prior[c.v] = mprior;
    }
    if (my_alive && c.is_edge) c.act = 0;                                          // :311-321
}

template <int G>
__global__ void __launch_bounds__(BLOCK) k_node_group(gtf_graph g, gtf_nodes n, gtf_states tse, gtf_states uts,
                                                      gtf_edges e, gtf_params p, Ws w, NodeOps ops,
                                                      double chi2_thr, double kl_thr, const int32_t* list,
                                                      int count) {
    __shared__ volatile double s_val[BLOCK];
    __shared__ volatile int s_lane[BLOCK];
    const int gi = (blockIdx.x * BLOCK + (int)threadIdx.x) / G;
    if (gi >= count) return;  // group-uniform
    NodeCtx<G> c;
    volatile double* sval = s_val + (threadIdx.x & ~63);
    volatile int* slane = s_lane + (threadIdx.x & ~63);
    c.v = list[gi];
    c.lo = g.slot_ptr[c.v];
    c.d = g.slot_ptr[c.v + 1] - c.lo;
    c.k = c.lo + c.grp.gl;
    c.valid = c.grp.gl < c.d;
    const int k = c.k;
    c.is_edge = c.valid ? g.is_edge[k] : 0;
    c.rev_edge = c.valid ? g.rev_edge[k] : 0;
    c.act = c.valid ? e.act[k] : 0;
    c.act0 = c.act;
    c.src = c.valid ? g.slot_src[k] : -1;
    c.layer = c.src >= 0 ? g.layer[c.src] : NAN;
    const bool has_tse = n.has_tse[c.v], has_uts_in = n.has_uts[c.v];
    c.tse = LaneDict{-1, 0.0, 0.0, false};
    c.uts = LaneDict{-1, 0.0, 0.0, false};
    c.lik = 0; c.lr = 0; c.x0 = 0; c.edge_mw = 0; c.side = -1; c.fresh = 0;
    c.uts_dirty_lr = false; c.edge_mw_dirty = false; c.degree = 0; c.degree_set = false;
    if (ops.uses_tse && c.valid) {
        c.tse.rank = tse.rank[k];
        c.tse.mw = tse.mw[k];
        c.tse.prior = tse.prior[k];
    }
    if (ops.uses_uts && c.valid) {
        c.uts.rank = uts.rank[k];
        c.uts.mw = uts.mw[k];
        c.uts.prior = uts.prior[k];
        c.lik = uts.lik[k];
        c.lr = uts.lr[k];
        c.side = uts.side[k];
        c.x0 = uts.xyzr[4 * (int64_t)k];
        c.fresh = uts.fresh[k];
    }
    bool has_uts = has_uts_in;
    for (int i = 0; i < ops.n; i++) {
        switch (ops.op[i]) {
            case OP_RANKS: g_ranks(c); break;
            case OP_PRIORS_TSE: if (has_tse) g_priors(c, c.tse); break;
            case OP_PRIORS_UTS: if (has_uts) g_priors(c, c.uts); break;
            case OP_REWEIGHT_UTS: if (has_uts) g_reweight(c, sval, g.gnn, p.reweight_threshold, w.err); break;
            case OP_DEGREE: g_degree(c); break;
            case OP_PRUNE: g_prune(c, has_tse, has_uts, w.err); break;
            case OP_MW_TSE: if (has_tse) g_mixture_weights(c, c.tse, g.solo[c.v], w.err); break;
            case OP_MW_UTS: if (has_uts) g_mixture_weights(c, c.uts, g.solo[c.v], w.err); break;
            case OP_CLUSTER_TSE:
                if (has_tse) g_cluster(c, n, tse, c.tse, slane, g.xyzr + 4 * (int64_t)c.v, chi2_thr, kl_thr, p, w.err);
                break;
            case OP_CLUSTER_UTS:
                if (has_uts) g_cluster(c, n, uts, c.uts, slane, g.xyzr + 4 * (int64_t)c.v, chi2_thr, kl_thr, p, w.err);
                break;
            default: break;
        }
    }
    // write back what changed
    if (c.valid) {
        if (c.act != c.act0) e.act[k] = c.act;
        if (c.edge_mw_dirty) e.edge_mw[k] = c.edge_mw;
        if (c.tse.dirty) { tse.rank[k] = c.tse.rank; tse.mw[k] = c.tse.mw; tse.prior[k] = c.tse.prior; }
        if (c.uts.dirty) { uts.rank[k] = c.uts.rank; uts.mw[k] = c.uts.mw; uts.prior[k] = c.uts.prior; }
        if (c.uts_dirty_lr) { uts.lr[k] = c.lr; uts.side[k] = c.side; }
    }
    if (c.degree_set && c.grp.gl == 0) n.degree[c.v] = c.degree;
}
