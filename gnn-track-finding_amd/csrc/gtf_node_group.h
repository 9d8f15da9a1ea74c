// gtf_node_group.h -- the node-local op sequence with G lanes per receiver node
// (G = 4, 8, 16, 32, 64 for nodes with <= 4, 8, 16, 32, 64 slots), one slot per lane.
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

#ifndef GTF_ABLATE
#define GTF_ABLATE 0  // diagnostics builds only (tools/ablate_build.sh)
#endif
#ifndef GTF_HOIST
#define GTF_HOIST 1   // the node's own scalars (x, xyzr, solo) loaded with the slot fields
#endif
#ifndef GTF_KL_LEAN
#define GTF_KL_LEAN 1   // the clustering's merged means as one 4-vector, KL operands re-read per iteration
#endif
#ifndef GTF_EARLY_STAGE
#define GTF_EARLY_STAGE 0   // clustering operands loaded into LDS with the slot fields
#endif

// Lane exchanges inside one wavefront through ds_bpermute with byte addresses computed
// once per lane: a power-of-two group's lanes are [gbase, gbase + G), so a shuffle from
// group lane src reads wave lane gbase + src and an xor-butterfly step with o < G stays in
// the group by itself -- none of the lane-id and bounds arithmetic of the generic __shfl /
// __shfl_xor (which recomputes the lane id on every call)
#ifndef GTF_FAST_SHFL
#define GTF_FAST_SHFL 0   // measured neutral in instruction count; its lane register costs a spill at 5 waves
#endif
__device__ __forceinline__ int bperm32(int addr, int v) { return __builtin_amdgcn_ds_bpermute(addr, v); }
template <typename T>
__device__ __forceinline__ T bperm(int addr, T x) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit lane values");
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, bperm32(addr, __builtin_bit_cast(int, x)));
    } else {
        const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
        const unsigned lo = (unsigned)bperm32(addr, (int)(unsigned)u);
        const unsigned hi = (unsigned)bperm32(addr, (int)(unsigned)(u >> 32));
        return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
    }
}

template <int G>
struct Grp {
    int gl;     // lane within the group
    int gbase;  // first wave lane of the group
    int lane4;  // 4 x the wave lane (ds_bpermute byte address of this lane)
    __device__ __forceinline__ Grp() {
        int tid = (int)threadIdx.x;
        const int lane = tid & 63;
        gl = lane & (G - 1);
        gbase = lane & ~(G - 1);
        lane4 = lane << 2;
    }
    __device__ __forceinline__ unsigned long long bits(bool pred) const {
        const unsigned long long b = __ballot(pred);
        if constexpr (G == 64) return b;
        else return (b >> gbase) & ((1ull << G) - 1ull);
    }
    __device__ __forceinline__ int count(bool pred) const { return __popcll(bits(pred)); }
    __device__ __forceinline__ bool any(bool pred) const { return bits(pred) != 0ull; }
#if GTF_FAST_SHFL
    template <typename T>
    __device__ __forceinline__ T shfl(T x, int src) const { return bperm<T>((gbase + src) << 2, x); }
    template <typename T>
    __device__ __forceinline__ T xshfl(T x, int o) const { return bperm<T>(lane4 ^ (o << 2), x); }
#else
    template <typename T>
    __device__ __forceinline__ T shfl(T x, int src) const { return __shfl(x, src, G); }
    template <typename T>
    __device__ __forceinline__ T xshfl(T x, int o) const { return __shfl_xor(x, o, G); }
#endif
    __device__ __forceinline__ int max_i(int x) const {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x = max(x, xshfl(x, o));
        return x;
    }
    __device__ __forceinline__ int min_i(int x) const {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x = min(x, xshfl(x, o));
        return x;
    }
    __device__ __forceinline__ double min_d(double x) const {  // NaN-free inputs
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x = fmin(x, xshfl(x, o));
        return x;
    }
    __device__ __forceinline__ unsigned or_u(unsigned x) const {
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) x |= xshfl(x, o);
        return x;
    }
    __device__ __forceinline__ int size() const { return G; }
    __device__ __forceinline__ int stage_base() const { return 0; }  // one stage struct per group
};

// G = 0: variable-size lane segments packed back to back in a wavefront (gtf_graph.pack_ent):
// the group is lanes [gbase, gbase + gsize) of the wave. Reductions are segmented
// shuffle-down steps (wmax = the wave's largest segment, wave-uniform) followed by a
// broadcast from the segment's first lane; the clustering stage is one per wavefront,
// the group's states at [gbase + i].
template <>
struct Grp<0> {
    int gl, gbase, gsize, wmax;
    unsigned long long lowmask;
    __device__ __forceinline__ Grp() {}
    __device__ __forceinline__ unsigned long long bits(bool pred) const { return (__ballot(pred) >> gbase) & lowmask; }
    __device__ __forceinline__ int count(bool pred) const { return __popcll(bits(pred)); }
    __device__ __forceinline__ bool any(bool pred) const { return bits(pred) != 0ull; }
    template <typename T>
    __device__ __forceinline__ T shfl(T x, int src) const { return __shfl(x, gbase + src); }
    template <typename T, typename Op>
    __device__ __forceinline__ T reduce(T x, Op op) const {
        for (int o = 1; o < wmax; o <<= 1) {
            const T y = __shfl_down(x, o);
            if (gl + o < gsize) x = op(x, y);
        }
        return __shfl(x, gbase);
    }
    __device__ __forceinline__ int max_i(int x) const { return reduce(x, [](int a, int b) { return max(a, b); }); }
    __device__ __forceinline__ int min_i(int x) const { return reduce(x, [](int a, int b) { return min(a, b); }); }
    __device__ __forceinline__ double min_d(double x) const {  // NaN-free inputs
        return reduce(x, [](double a, double b) { return fmin(a, b); });
    }
    __device__ __forceinline__ unsigned or_u(unsigned x) const {
        return reduce(x, [](unsigned a, unsigned b) { return a | b; });
    }
    __device__ __forceinline__ int size() const { return gsize; }
    __device__ __forceinline__ int stage_base() const { return gbase; }
};

// Correctly rounded reciprocals 1/n (n = 1..64) in LDS: every node kernel block fills the
// table at its start, and the ops' integer reciprocals (priors 1/count, mixture weights
// 1/count, the side norm's divisor through qdiv) read it instead of running an fp64 division
// (~10 VALU instructions each) -- the same bits (the table holds 1.0 / n itself)
#ifndef GTF_RCP_TABLE
#define GTF_RCP_TABLE 1
#endif
__shared__ double g_rcp_lds[65];
// (i, j) of lower-triangle pair t (pair_ij) for t < 120 (15 states: 105 pairs), i | j << 8:
// the clustering's pair loop reads its pairs here instead of solving t = i (i - 1) / 2 + j
// (a float square root and two correction loops, ~40 VALU instructions per pair)
__shared__ uint16_t g_pair_lds[120];
// every node kernel fills both tables at its start, before its block barrier
__device__ __forceinline__ void node_tables_init() {
#if GTF_RCP_TABLE
    // (strided: blocks of fewer than 120 threads fill every entry too)
    for (int t = (int)threadIdx.x; t < 120; t += (int)blockDim.x) {
        if (t < 65) g_rcp_lds[t] = t ? 1.0 / (double)t : 0.0;
        int i, j;
        pair_ij(t, i, j);
        g_pair_lds[t] = (uint16_t)(i | (j << 8));
    }
#endif
}
__device__ __forceinline__ void pair_of(int t, int& i, int& j) {
#if GTF_RCP_TABLE
    const int e = g_pair_lds[t];
    i = e & 0xff;
    j = e >> 8;
#else
    pair_ij(t, i, j);
#endif
}

// per-lane (per-slot) registers of one state dict
enum : uint8_t { D_RANK = 1, D_MW = 2, D_PRIOR = 4 };  // LaneDict.dirty: fields to store

struct LaneDict {
    int rank;
    double mw, prior;
    uint8_t dirty;   // D_* bits of the fields an op changed
    int pos;         // cached dict position (-1 absent), valid while pos_ok
    bool pos_ok;
    int last;        // group lane of the last dict key (largest rank), valid while last_ok
    bool last_ok;
};

template <int G>
struct NodeCtx {
    Grp<G> grp;
    int v, lo, d, k;
    bool valid;
    uint8_t is_edge, rev_edge, act, act0;
    double layer;                   // sender layer (without the static classes)
    uint64_t cls;                   // gtf_graph.slot_class of the slot (0 without)
    uint64_t xcls;                  // G = 64: gtf_graph.slot_xclass of the slot (its same-x positions)
    uint8_t sfl;                    // gtf_graph.slot_sflags of the slot
    bool use_cls;                   // the static classes cover this group (group-uniform)
    bool live;                      // UTS entry's xyzr = gnn[slot_src] (gtf_states.fresh bit 1)
    bool left;                      // side of the UTS entry (x < node x), with same_x
    int src;                        // slot_src (read for the UTS clustering's coordinates)
    unsigned long long same_layer;  // lanes whose sender has this lane's layer (lazy)
    bool same_layer_ok;
    unsigned long long same_x;      // lanes whose stored UTS x equals this lane's (lazy; NaN: itself)
    bool same_x_ok;
    LaneDict tse, uts;
    double lik, lr, edge_mw, smw;
    int8_t side;
    uint8_t fresh;
    bool uts_dirty_lr, edge_mw_dirty;
    int degree;
    bool degree_set;
    double xa, za, ra;         // node attribute xyzr x, z, r (clustering tau geometry)
    uint8_t solo;              // node alone in its subgraph (mixture weights)
    bool staged;               // clustering operands already in the group's LDS stage (slot lanes)
    int lri;                   // the side norm's divisor as an integer (1 for lr = 1.0)
};

// 1.0 / n for a count n >= 1 (<= 64): the LDS table or a division
template <int G>
__device__ __forceinline__ double rcp_count(const NodeCtx<G>& c, int n) {
    (void)c;
    return GTF_RCP_TABLE ? g_rcp_lds[n] : 1.0 / (double)n;
}

// highest set bit index of m (m != 0)
__device__ __forceinline__ int hibit(unsigned long long m) { return 63 - __clzll((long long)m); }

// dict position of this lane's key = number of present keys with a smaller rank.
// Fast path: ranks ascending in slot order (fresh UTS dicts) -> popcount.
template <int G>
__device__ __forceinline__ int dict_pos(const NodeCtx<G>& c, LaneDict& st) {
    if (st.pos_ok) return st.pos;
    const bool pres = c.valid && st.rank >= 0;
    const unsigned long long P = c.grp.bits(pres);
    const unsigned long long below = P & ((1ull << c.grp.gl) - 1ull);
    const int prev = below ? hibit(below) : c.grp.gl;
    const int rprev = c.grp.shfl(st.rank, prev);
    const bool mono = !pres || !below || rprev < st.rank;
    int pos;
    if (!c.grp.any(!mono)) {
        pos = __popcll(below);
    } else {
        pos = 0;
        for (int j = 0; j < c.grp.size(); j++) {
            const int rj = c.grp.shfl(st.rank, j);
            pos += (rj >= 0 && rj < st.rank) ? 1 : 0;
        }
    }
    st.pos = pres ? pos : -1;
    st.pos_ok = true;
    return st.pos;
}

// sequential (dict-order) sum of `term` over lanes where `take`; every lane gets the
// sum. Lanes write their term at their dict position in a per-group LDS line and
// every lane adds the line in order; skipped entries add +0.0, which leaves the
// running sum unchanged (it starts from the integer 0 of helper.py:165).
#ifndef GTF_CHUNKED_SUM
#define GTF_CHUNKED_SUM 1
#endif
#ifndef GTF_SUM_ZFILL
#define GTF_SUM_ZFILL 1
#endif
template <int G>
__device__ __forceinline__ double ordered_sum(NodeCtx<G>& c, double* sval, LaneDict& st, bool take,
                                             double term) {
    const int pos = dict_pos(c, st);
    const int npres = c.grp.count(c.valid && st.rank >= 0);
#if GTF_SUM_ZFILL
    // the group's line zeroed first (every lane its own entry), then the terms at their dict
    // positions (the same wave's LDS stores land in issue order): the entries past the last
    // key read +0.0, so the chunked sum needs no per-entry select
    if constexpr (G > 0) sval[c.grp.gbase + c.grp.gl] = 0.0;
#endif
    if (pos >= 0) sval[c.grp.gbase + pos] = take ? term : 0.0;
    wave_lds_sync();
    double s = 0.0;
#if GTF_CHUNKED_SUM
    // the line is read CH entries at a time (independent LDS reads, one wait) and added in
    // order; entries past the last key add +0.0, which leaves the sum unchanged (it is never
    // -0.0: it starts at +0.0 and round-to-nearest cancellation gives +0.0)
    constexpr int CH = G == 0 ? 1 : (G < 8 ? G : 8);   // chunks stay inside the group's line
    for (int i = 0; i < npres; i += CH) {
        double v[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) v[j] = sval[c.grp.gbase + i + j];
#pragma unroll
        for (int j = 0; j < CH; j++) s = s + ((GTF_SUM_ZFILL && G > 0) || i + j < npres ? v[j] : 0.0);
    }
#else
    for (int i = 0; i < npres; i++) s = s + sval[c.grp.gbase + i];
#endif
    wave_lds_sync();
    return s;
}

#ifndef GTF_PAIRWISE_CLASSES
#define GTF_PAIRWISE_CLASSES 1   // 1: groups of up to 16 lanes, 2: every group size
#endif
constexpr int PAIRWISE_MAX_G = GTF_PAIRWISE_CLASSES >= 2 ? 64 : 16;
// mask of the group's valid lanes whose value equals this lane's (a NaN equals nothing;
// the caller adds the lane itself): every lane puts its value on the group's LDS line and
// compares with all G entries -- independent reads instead of a leader-election chain of
// ballots and shuffles (groups of up to 16 lanes)
template <int G>
__device__ __forceinline__ unsigned long long equal_lanes(const NodeCtx<G>& c, double* sval, double mine) {
    sval[c.grp.gbase + c.grp.gl] = c.valid ? mine : NAN;
    wave_lds_sync();
    unsigned long long m = 0ull;
    constexpr int CH = G < 16 ? G : 16;
#pragma unroll
    for (int i = 0; i < G; i += CH) {
        double v[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) v[j] = sval[c.grp.gbase + i + j];
#pragma unroll
        for (int j = 0; j < CH; j++) m |= (v[j] == mine) ? (1ull << (i + j)) : 0ull;
    }
    wave_lds_sync();
    return c.valid ? m : 0ull;
}

template <int G>
__device__ __forceinline__ bool lane_active(const NodeCtx<G>& c, int rank) {
    return c.valid && rank >= 0 && c.is_edge && c.act == 1;
}

// compute_prior_probabilities (helper.py:30-63): prior = 1 / #active keys whose sender
// shares this key's layer. The same-layer masks are built once per node, one
// iteration per distinct layer value (leader election with a ballot).
template <int G>
__device__ __forceinline__ void g_priors(NodeCtx<G>& c, LaneDict& st, double* sval) {
    if constexpr (G > 0 && G <= 64) {
        if (!c.same_layer_ok && c.use_cls) {   // the graph-static classes (gtf_graph.slot_class)
            // (33..64-slot segments: all 64 bits of slot_class are the same-layer positions)
            c.same_layer = c.valid ? (G == 64 ? c.cls : (c.cls & 0xffffffffull)) : 0ull;
            c.same_layer_ok = true;
        }
    }
#if GTF_PAIRWISE_CLASSES
    if constexpr (G > 0 && G <= PAIRWISE_MAX_G) {
        if (!c.same_layer_ok) {
            c.same_layer = equal_lanes(c, sval, c.layer) | (c.valid ? (1ull << c.grp.gl) : 0ull);
            c.same_layer_ok = true;
        }
    }
#endif
    if (!c.same_layer_ok) {
        bool done = !c.valid || c.layer != c.layer;  // NaN layers (orphans) never match
        c.same_layer = c.valid ? (1ull << c.grp.gl) : 0ull;
        while (true) {
            const unsigned long long todo = c.grp.bits(!done);
            if (!todo) break;
            const int leader = __ffsll((long long)todo) - 1;
            const double L = c.grp.shfl(c.layer, leader);
            const bool mine = !done && c.layer == L;
            const unsigned long long m = c.grp.bits(mine);
            if (mine) { c.same_layer = m; done = true; }
        }
        c.same_layer_ok = true;
    }
    const bool act = lane_active(c, st.rank);
    const unsigned long long A = c.grp.bits(act);
    if (act) {
        st.prior = rcp_count(c, __popcll(A & c.same_layer));
        st.dirty |= D_PRIOR;
    }
}

// calculate_side_norm_factor + reweight (helper.py:99-200), UTS only
// the x of a UTS entry's stored coordinates: its sender's live GNN x (gtf_states.fresh bit 1,
// extrapolate_merged_states.py:377) or the stored snapshot
template <int G>
__device__ __forceinline__ double uts_x(const NodeCtx<G>& c, const gtf_graph& g, const gtf_states& uts) {
    if (!c.valid) return 0.0;
    if (c.live) return g.slot_sxzr ? g.slot_sxzr[3 * (int64_t)c.k] : g.gnn[4 * (int64_t)g.slot_src[c.k]];
    return uts.xyzr[4 * (int64_t)c.k];
}

template <int G>
__device__ __forceinline__ void g_reweight(NodeCtx<G>& c, double* sval, const gtf_graph& g, const gtf_states& uts,
                                           double thr, uint32_t* err) {
    LaneDict& st = c.uts;
    const bool act = lane_active(c, st.rank);
    // last dict key = the present key with the largest rank (stale loop variable, :131,138);
    // kept until the key set changes (ranks / prune)
    if (!st.last_ok) {
        const int maxr = c.grp.max_i(c.valid ? st.rank : -1);
        const unsigned long long lastb = c.grp.bits(c.valid && st.rank == maxr && maxr >= 0);
        st.last = lastb ? __ffsll((long long)lastb) - 1 : 0;
        st.last_ok = true;
    }
    const int last = st.last;
    const int last_is_edge = c.grp.shfl((int)c.is_edge, last);
    const int last_act = c.grp.shfl((int)c.act, last);
    // distinct x values per side (len(set(coords))): the classes of equal stored x, built
    // once per node (a NaN is only equal to itself, as set() keeps every NaN object); a key
    // counts if it is the first active key of its class -- equal x, same side. When every
    // present key's x is its sender's live GNN x (the entries message passing wrote), the
    // classes and sides are graph-static (gtf_graph.slot_class / slot_sflags); the present
    // keys only shrink after this point (pruning), so they stay valid for the pass.
    if constexpr (G > 0 && G <= 64) {
        if (!c.same_x_ok && c.use_cls && !c.grp.any(c.valid && st.rank >= 0 && !c.live)) {
            c.same_x = c.valid ? (G == 64 ? c.xcls : (c.cls >> 32)) : 0ull;
            c.left = (c.sfl & 1) != 0;
            c.same_x_ok = true;
        }
    }
    if (!c.same_x_ok) {
        const double x0 = uts_x(c, g, uts);
        c.left = x0 < g.gnn[4 * (int64_t)c.v];
#if GTF_PAIRWISE_CLASSES
        if constexpr (G > 0 && G <= PAIRWISE_MAX_G) {
            c.same_x = equal_lanes(c, sval, x0) | (c.valid ? (1ull << c.grp.gl) : 0ull);
            c.same_x_ok = true;
        }
#endif
        if (!c.same_x_ok) {
            bool done = !c.valid || x0 != x0;
            c.same_x = c.valid ? (1ull << c.grp.gl) : 0ull;
            while (true) {
                const unsigned long long todo = c.grp.bits(!done);
                if (!todo) break;
                const int leader = __ffsll((long long)todo) - 1;
                const double X = c.grp.shfl(x0, leader);
                const bool mine = !done && x0 == X;
                const unsigned long long m = c.grp.bits(mine);
                if (mine) { c.same_x = m; done = true; }
            }
            c.same_x_ok = true;
        }
    }
    const bool left = c.left;
    const unsigned long long A = c.grp.bits(act);
    const bool first = act && (c.same_x & A & ((1ull << c.grp.gl) - 1ull)) == 0ull;
    const int dl = c.grp.count(first && left);
    const int dr = c.grp.count(first && !left);
    const int nact = c.grp.count(act);
    if (nact > 0) {
        if (!last_is_edge && c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_STALE_KEY_NO_EDGE);
        if (act) {
            c.side = left ? 0 : 1;
            c.lri = (last_is_edge && last_act == 1) ? (left ? dl : dr) : 1;
            c.lr = (last_is_edge && last_act == 1) ? (double)(left ? dl : dr) : 1.0;
            c.uts_dirty_lr = true;
        }
    }
    const double denom = ordered_sum(c, sval, st, act, st.mw * c.lik);
    if (act) {
        double wgt = (st.mw * c.lik * st.prior) / denom;
        wgt = GTF_RCP_TABLE ? qdiv(wgt, c.lr, g_rcp_lds[c.lri]) : wgt / c.lr;   // (lr = lri exactly)
        st.mw = wgt;
        st.dirty |= D_MW;
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
        if (c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_NO_STATE_DICT);
        return;
    }
    LaneDict& st = has_uts ? c.uts : c.tse;
    if (c.valid && st.rank >= 0 && !c.rev_edge) {
        st.rank = -1;
        st.dirty |= D_RANK;
    }
    st.pos_ok = false;
    st.last_ok = false;
}

template <int G>
__device__ __forceinline__ void g_mixture_weights(NodeCtx<G>& c, LaneDict& st, bool solo, uint32_t* err) {
    const int cnt = c.grp.count(c.valid && st.rank >= 0);
    if (cnt == 0) {
        if (!solo && c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_EMPTY_DICT_MW);
        return;
    }
    if (c.valid && st.rank >= 0) {
        st.mw = rcp_count(c, cnt);
        st.dirty |= D_MW;
    }
}

// the entries the last message passing (re)wrote carry the sender's TSE mixture weight
// (extrapolate_merged_states.py:384) and no prior, lr or side yet (a fresh dict entry
// the priors / side norm have not reached); set here with the node's other slot stores
// instead of by k_extrapolate
template <int G>
__device__ __forceinline__ void g_fresh(NodeCtx<G>& c) {
    if (c.valid && c.fresh) {
        if (!GTF_MW_IN_EXTRAP) {   // (else k_extrapolate stored it)
            c.uts.mw = c.smw;
            c.uts.dirty |= D_MW;
        }
        c.uts.prior = NAN;
        c.uts.dirty |= D_PRIOR;
        c.lr = NAN;
        c.side = -1;
        c.uts_dirty_lr = true;
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
        st.dirty |= D_RANK;
    }
    st.pos_ok = false;
    st.last_ok = false;
}

// per-group LDS staging of up to 15 states (structure of arrays): the state, its
// covariance and inverse (computed once per state: np.linalg.inv of a state's
// covariance is the same value every time the reference recomputes it), and the
// per-neighbour tau geometry of the pairwise chi2
// Entries sit at the state's SLOT lane (its lane in the group), ord[dict position] maps a
// dict position to it: the operands can then be staged before the ops have settled
// which keys are present and in what order (GTF_EARLY_STAGE).
template <int CAP>
#ifndef GTF_MERGE_SHFL
#define GTF_MERGE_SHFL 0   // 1: the greedy merge takes the chosen key's inverse from its lane (below); measured +1.5 us (3 VGPRs spill), profiles/r06/shfl/
#endif
#ifndef GTF_STAGE_NOINV
#define GTF_STAGE_NOINV 2   // (with GTF_KL_LEAN) 3 = 2x2-block inverses staged after the pair loop (below;
                            // one division per merge instead of three, but 3 VGPRs spill: 3.5 us slower);
                            // no inverses in LDS: 1 = in the owning lane's registers,
                            // 2 = recomputed from the staged covariances where used
#endif
struct StageT {
    double a[CAP], b[CAP], c[CAP], tau[CAP];
    double c00[CAP], c01[CAP], c10[CAP], c11[CAP], c22[CAP];
#if !GTF_STAGE_NOINV
    double i00[CAP], i01[CAP], i10[CAP], i11[CAP], i22[CAP];
#endif
    double q[CAP], w[CAP], tg[CAP], prior[CAP];   // (early staging parks x, z, r in q, w, tg)
#if GTF_STAGE_NOINV == 3
    double x4[CAP];   // with q, w, tg after the pair loop: the state's 2x2-block inverse
#endif
    uint8_t ec[CAP];  // neighbour in the endcap (|x| >= boundary): picks its sigma_z / sigma_r pair
    uint8_t ord[CAP]; // slot lane of the state at each dict position
};

// the clustering operands of this lane's state, raw, at its slot lane
template <typename Stage>
__device__ __forceinline__ void stage_raw(Stage* stg, int li, const gtf_states& S, int64_t k, const double* gnn,
                                          bool live, int src, const double* sxzr) {
    stg->a[li] = S.sv[3 * k];
    stg->b[li] = S.sv[3 * k + 1];
    stg->c[li] = S.sv[3 * k + 2];
    stg->tau[li] = S.tau[k];
    const double* cv = S.cov + 5 * k;
    stg->c00[li] = cv[0]; stg->c01[li] = cv[1]; stg->c10[li] = cv[2]; stg->c11[li] = cv[3]; stg->c22[li] = cv[4];
    // the state's stored sender coordinates: the sender's live GNN ones for an entry message
    // passing wrote (gtf_states.fresh bit 1) -- from the slot's own copy (gtf_graph.slot_sxzr,
    // contiguous) or gathered from the sender's gnn row --, else the snapshot
    if (live && sxzr) {
        const double* xp = sxzr + 3 * k;
        stg->q[li] = xp[0];
        stg->w[li] = xp[1];
        stg->tg[li] = xp[2];
        return;
    }
    const double* xp = live ? gnn + 4 * (int64_t)src : S.xyzr + 4 * k;
    stg->q[li] = xp[0];
    stg->w[li] = xp[2];
    stg->tg[li] = xp[3];
}

template <typename Stage>
__device__ __forceinline__ Cov5 stage_cov(const Stage* s, int i) {
    return Cov5{s->c00[i], s->c01[i], s->c10[i], s->c11[i], s->c22[i]};
}
#if !GTF_STAGE_NOINV
template <typename Stage>
__device__ __forceinline__ Cov5 stage_inv(const Stage* s, int i) {
    return Cov5{s->i00[i], s->i01[i], s->i10[i], s->i11[i], s->i22[i]};
}
#elif !GTF_KL_LEAN
#error "GTF_STAGE_NOINV needs GTF_KL_LEAN"
#endif
template <typename Stage>
__device__ __forceinline__ TauGeo stage_geo(const Stage* s, int i, double szb2, double srb2) {
    TauGeo t;
    t.q = s->q[i]; t.w = s->w[i]; t.tau = s->tg[i];
    const bool ec = s->ec[i];   // endcap swaps the barrel pair (tau_geo)
    t.sz2 = ec ? srb2 : szb2;
    t.sr2 = ec ? szb2 : srb2;
    return t;
}

#ifndef GTF_OP_TIMING
#define GTF_OP_TIMING 0
#endif
#if GTF_OP_TIMING
#define GTF_OP_TIMING_WAVES 65536
__device__ uint64_t g_op_time[GTF_OP_TIMING_WAVES * 24];
// a stamp inside an op (words 19 and 22 of the wave's row), lane 0 only
#define GTF_SUBSTAMP(word)                                                                        \
    do {                                                                                          \
        const int wv_ = (int)((blockIdx.x * blockDim.x + threadIdx.x) / 64);                      \
        if ((threadIdx.x & 63) == 0 && wv_ < GTF_OP_TIMING_WAVES)                                 \
            g_op_time[24 * (int64_t)wv_ + (word)] = __builtin_readcyclecounter();                  \
    } while (0)
#else
#define GTF_SUBSTAMP(word) \
    do {                   \
    } while (0)
#endif

// pairwise chi2 + greedy KL merging of one node (clustering.py:197-307). The
// d(d-1)/2 pairs are dealt round-robin over the G lanes (row-major pair index t),
// so the np.where tie order is the order of t. The parabolic and the joint merge
// share their covariance (both merge the same aliased covariances), so one
// (I1 + I2)^-1 serves both means.
template <int G, typename Stage>
__device__ __forceinline__ void g_cluster(NodeCtx<G>& c, gtf_nodes& n, const gtf_states& S, LaneDict& st,
                                          Stage* stg, const double* xyzr_node, const double* gnn, bool live,
                                          double chi2_thr, double kl_thr, const gtf_params& p, uint32_t* err,
                                          const double* sxzr, bool prior_known) {
#if GTF_ABLATE == 1
    return;  // diagnostics build (tools/ablate_build.sh): no clustering work
#endif
    const bool pres = c.valid && st.rank >= 0;
    const int d = c.grp.count(pres);
    if (d <= 2 || d >= 16) return;                                                 // :207
    const int pos = dict_pos(c, st);
    const int sb = c.grp.stage_base();   // this group's first entry in the stage arrays
    const int me_l = sb + c.grp.gl;      // this lane's entry (its slot lane)
#if GTF_HOIST
    (void)xyzr_node;
    const double xa = c.xa, za = c.za, ra = c.ra;
#else
    const double xa = xyzr_node[0], za = xyzr_node[2], ra = xyzr_node[3];
#endif
    if (pres) {
        if (!c.staged) stage_raw(stg, me_l, S, c.k, gnn, live, c.src, sxzr);
        const double x = stg->q[me_l], z = stg->w[me_l], r = stg->tg[me_l];
#if !GTF_STAGE_NOINV
        const Cov5 I = inv_cov5(stage_cov(stg, me_l));
        stg->i00[me_l] = I.c00; stg->i01[me_l] = I.c01; stg->i10[me_l] = I.c10; stg->i11[me_l] = I.c11;
        stg->i22[me_l] = I.c22;
#endif
        const TauGeo t = tau_geo(x, z, r, za, ra, p.sigma0rz2, p.sigma0rz, p.sigma0rz, p.sigma0rz2, p.endcap_boundary);
        stg->q[me_l] = t.q; stg->w[me_l] = t.w; stg->tg[me_l] = t.tau;
        stg->ec[me_l] = fabs(x) >= p.endcap_boundary;
        // the key's prior: as an op of the sequence set it (or it was loaded), else the stored one
        stg->prior[me_l] = (prior_known || (st.dirty & D_PRIOR)) ? st.prior : S.prior[c.k];
        stg->ord[sb + pos] = (uint8_t)c.grp.gl;
    }
    wave_lds_sync();
    GTF_SUBSTAMP(22);   // (diagnostics) the states staged
    const double szb2 = p.sigma0rz2 * p.sigma0rz2, srb2 = p.sigma0rz * p.sigma0rz;   // barrel sigma_z^2, sigma_r^2
    const bool ec = fabs(xa) >= p.endcap_boundary;
    const double sza = ec ? p.sigma0rz : p.sigma0rz2, sra = ec ? p.sigma0rz2 : p.sigma0rz;
    const double sza2 = sza * sza, sra2 = sra * sra;
    const int npairs = d * (d - 1) / 2;
    double lmin = INFINITY;
    int lt0 = 1 << 20, lt1 = 1 << 20;
    unsigned lmask = 0;
    bool lnan = false, lnz = false;
    // a lane's pairs in ascending t (the np.where order of its ties): fold one distance
    auto fold = [&](double D, int t, int i, int j) {
        if (D == 0.0) return;  // zeros are excluded (np.nonzero)
        lnz = true;
        if (D != D) { lnan = true; return; }
        if (D < lmin) {
            lmin = D; lt0 = t; lt1 = 1 << 20; lmask = (1u << i) | (1u << j);
        } else if (D == lmin) {
            if (lt1 == (1 << 20)) lt1 = t;
            lmask |= (1u << i) | (1u << j);
        }
    };
#ifndef GTF_PAIR_SPLIT
#define GTF_PAIR_SPLIT 0   // the [a, b] term's operands, then the tau term's (fewer LDS values live at once)
#endif
    auto pair_d = [&](int i, int j) {
        const int li = sb + stg->ord[sb + i], lj = sb + stg->ord[sb + j];
#if GTF_PAIR_SPLIT
        const double d1 = maha_d1(stg->a[li], stg->b[li], stage_cov(stg, li), stg->a[lj], stg->b[lj], stage_cov(stg, lj));
        __builtin_amdgcn_sched_barrier(0);
        const double d2 = maha_d2(sza2, sra2, stage_geo(stg, li, szb2, srb2), stage_geo(stg, lj, szb2, srb2));
        return d1 + d2;
#else
        return mahalanobis_geo(stg->a[li], stg->b[li], stage_cov(stg, li), stg->a[lj], stg->b[lj],
                               stage_cov(stg, lj), sza2, sra2, stage_geo(stg, li, szb2, srb2),
                               stage_geo(stg, lj, szb2, srb2));
#endif
    };
#ifndef GTF_PAIR_UNROLL
#define GTF_PAIR_UNROLL 1
#endif
#if GTF_PAIR_UNROLL > 1
    // GTF_PAIR_UNROLL of the lane's pairs per iteration: their division chains (the 2x2
    // inverse of the summed covariances, the tau term) are independent and overlap; folded
    // in t order
    constexpr int U = GTF_PAIR_UNROLL;
    const int step = c.grp.size();
    for (int t = c.grp.gl; t < npairs; t += U * step) {
        double Dv[U];
        int iv[U], jv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int tu = t + u * step;
            pair_of(tu < npairs ? tu : t, iv[u], jv[u]);
            Dv[u] = pair_d(iv[u], jv[u]);
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if (t + u * step < npairs) fold(Dv[u], t + u * step, iv[u], jv[u]);
    }
#else
    for (int t = c.grp.gl; t < npairs; t += c.grp.size()) {
        int i, j;
        pair_of(t, i, j);
        fold(pair_d(i, j), t, i, j);
    }
#endif
    GTF_SUBSTAMP(19);   // (diagnostics) the pair loop done
    if (!c.grp.any(lnz)) {
        if (c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_ALL_ZERO_DIST);
        return;
    }
    if (c.grp.any(lnan)) return;                       // np.min over a NaN -> no merge (:228)
#if GTF_ABLATE == 2
    if (c.grp.min_d(lmin) > -1.0) return;  // diagnostics build: staging + pair distances only
#endif
    const double best = c.grp.min_d(lmin);
    if (!(best < chi2_thr)) return;
    const bool tl = lmin == best;
    const int t0 = c.grp.min_i(tl ? lt0 : (1 << 20));
    const int t1 = c.grp.min_i(tl ? (lt0 == t0 ? lt1 : lt0) : (1 << 20));
    const unsigned tiemask = c.grp.or_u(tl ? lmask : 0u);
    int ti0, tj0, ti1 = 0, tj1;
    pair_of(t0, ti0, tj0);
    if (t1 < (1 << 20)) pair_of(t1, ti1, tj1);
    // merged pair = (idx[0], idx[1]) of concatenate((rows, cols)) (:231-233)
    const int p0 = ti0, p1 = (t1 < (1 << 20)) ? ti1 : tj0;
#if GTF_KL_LEAN
    // the parabolic and the joint merged means share components 0 and 1 bit for bit (the same
    // a, b through the same block-diagonal products: merge_with_inv), so one 4-vector
    // (a, b, c, tau) carries both; the per-lane KL operands are re-read from LDS every
    // iteration instead of held in registers across the loop (fewer live registers)
    double mm[4];
    Cov5 mc;
    const int l0 = sb + stg->ord[sb + p0], l1 = sb + stg->ord[sb + p1];
#if GTF_STAGE_NOINV == 3
    // every present state's 2x2-block inverse (np.linalg.inv of its covariance: the same value
    // wherever the reference recomputes it) computed once and staged in the tau-geometry
    // entries the pair loop has finished with (q, w, tg) and x4; only its (2, 2) entry
    // 1 / c22 is recomputed where used: one division instead of three per use
    wave_lds_sync();   // (every lane's pair loop has read its q, w, tg)
    if (pres) {
        double i00, i01, i10, i11;
        inv2(stg->c00[me_l], stg->c01[me_l], stg->c10[me_l], stg->c11[me_l], i00, i01, i10, i11);
        stg->q[me_l] = i00; stg->w[me_l] = i01; stg->tg[me_l] = i10; stg->x4[me_l] = i11;
    }
    wave_lds_sync();
    auto inv_of = [&](int l) { return Cov5{stg->q[l], stg->w[l], stg->tg[l], stg->x4[l], 1.0 / stg->c22[l]}; };
#elif GTF_STAGE_NOINV == 2
    // inverses recomputed from the staged covariances where they are used (np.linalg.inv of a
    // state's covariance is the same value wherever the reference recomputes it): no register
    // holds one across the loop
    auto inv_of = [&](int l) { return inv_cov5(stage_cov(stg, l)); };
#elif GTF_STAGE_NOINV
    // every present state's inverse in its own lane (np.linalg.inv of its covariance, the same
    // value wherever the reference recomputes it); a merge takes it from the owner by shuffles
    Cov5 myI{0.0, 0.0, 0.0, 0.0, 0.0};
    if (pres) myI = inv_cov5(stage_cov(stg, me_l));
    auto inv_of = [&](int l) {
        const int src = l - sb;
        return Cov5{c.grp.shfl(myI.c00, src), c.grp.shfl(myI.c01, src), c.grp.shfl(myI.c10, src),
                    c.grp.shfl(myI.c11, src), c.grp.shfl(myI.c22, src)};
    };
#else
    auto inv_of = [&](int l) { return stage_inv(stg, l); };
#endif
    {
        const Cov5 i0 = inv_of(l0), i1 = inv_of(l1);
        mc = inv_cov5(add_cov5(i0, i1));
        const double x0[4] = {stg->a[l0], stg->b[l0], stg->c[l0], stg->tau[l0]};
        const double x1[4] = {stg->a[l1], stg->b[l1], stg->c[l1], stg->tau[l1]};
        merge4_with_inv(x0, i0, x1, i1, mc, mm);
    }
    double mprior = stg->prior[l0] + stg->prior[l1];
    unsigned alive = ((1u << d) - 1u) & ~tiemask;
    if (alive == 0) {
        if (c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_TIE_EMPTIED);
    } else {
        while (GTF_ABLATE != 3) {                                                  // :251-287
            asm volatile("" ::: "memory");
            const Cov5 im = inv_cov5(mc);   // the merged state's inverse, shared by KL and the next merge
            const bool me = pres && (alive >> pos & 1u);
            double D = INFINITY;
            bool dn = false;
#if GTF_STAGE_NOINV == 2 && GTF_MERGE_SHFL
            Cov5 ime{0.0, 0.0, 0.0, 0.0, 0.0};   // this lane's state's inverse (the KL's), handed to the merge
#endif
            if (me) {
                const double js_me[3] = {stg->a[me_l], stg->b[me_l], stg->tau[me_l]};
                const double jm[3] = {mm[0], mm[1], mm[3]};
#if GTF_STAGE_NOINV == 3
                D = kl_with_inv(js_me, stage_cov(stg, me_l), inv_of(me_l), jm, mc, im);
#elif GTF_STAGE_NOINV == 2 && GTF_MERGE_SHFL
                const Cov5 cme = stage_cov(stg, me_l);
                ime = inv_cov5(cme);
                D = kl_with_inv(js_me, cme, ime, jm, mc, im);
#elif GTF_STAGE_NOINV == 2
                const Cov5 cme = stage_cov(stg, me_l);
                D = kl_with_inv(js_me, cme, inv_cov5(cme), jm, mc, im);
#elif GTF_STAGE_NOINV
                D = kl_with_inv(js_me, stage_cov(stg, me_l), myI, jm, mc, im);
#else
                D = kl_with_inv(js_me, stage_cov(stg, me_l), stage_inv(stg, me_l), jm, mc, im);
#endif
                if (D != D) { dn = true; D = INFINITY; }
            }
            if (c.grp.any(dn)) {
                if (c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_NAN_KL);
                break;
            }
            const double mind = c.grp.min_d(D);
            if (!(mind < kl_thr)) break;
            const int m = c.grp.min_i((me && D == mind) ? pos : 99);  // first minimum (list.index)
#if GTF_STAGE_NOINV == 2 && GTF_MERGE_SHFL
            // the merged key's inverse from the lane that holds it (it computed that inverse for
            // its KL term: np.linalg.inv of one covariance is one value), by shuffles, instead of
            // recomputed from the stage (two divisions on the loop's dependent chain)
            const unsigned long long wb = c.grp.bits(me && pos == m);
            const int wl = wb ? __ffsll((long long)wb) - 1 : 0;
            const int lm = sb + wl;
            const Cov5 ii{c.grp.shfl(ime.c00, wl), c.grp.shfl(ime.c01, wl), c.grp.shfl(ime.c10, wl),
                          c.grp.shfl(ime.c11, wl), c.grp.shfl(ime.c22, wl)};
#else
            const int lm = sb + stg->ord[sb + m];
            const Cov5 ii = inv_of(lm);
#endif
            const Cov5 nmc = inv_cov5(add_cov5(ii, im));
            const double x[4] = {stg->a[lm], stg->b[lm], stg->c[lm], stg->tau[lm]};
            double nm[4];
            merge4_with_inv(x, ii, mm, im, nmc, nm);
            mm[0] = nm[0]; mm[1] = nm[1]; mm[2] = nm[2]; mm[3] = nm[3];
            mc = nmc;
            mprior = stg->prior[lm] + mprior;
            alive &= ~(1u << m);
            if (alive == 0) break;
        }
    }
    const double pm[3] = {mm[0], mm[1], mm[2]};
#else
    double pm[3], jm[3];
    Cov5 mc;
    const int l0 = sb + stg->ord[sb + p0], l1 = sb + stg->ord[sb + p1];
    {
        const Cov5 i0 = stage_inv(stg, l0), i1 = stage_inv(stg, l1);
        mc = inv_cov5(add_cov5(i0, i1));
        const double ps0[3] = {stg->a[l0], stg->b[l0], stg->c[l0]};
        const double ps1[3] = {stg->a[l1], stg->b[l1], stg->c[l1]};
        const double js0[3] = {ps0[0], ps0[1], stg->tau[l0]};
        const double js1[3] = {ps1[0], ps1[1], stg->tau[l1]};
        merge_with_inv(ps0, i0, ps1, i1, mc, pm);
        merge_with_inv(js0, i0, js1, i1, mc, jm);
    }
    double mprior = stg->prior[l0] + stg->prior[l1];
    unsigned alive = ((1u << d) - 1u) & ~tiemask;
    if (alive == 0) {
        if (c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_TIE_EMPTIED);
    } else {
        while (GTF_ABLATE != 3) {                                                  // :251-287
            const Cov5 im = inv_cov5(mc);   // the merged state's inverse, shared by KL and the next merge
            const bool me = pres && (alive >> pos & 1u);
            double D = INFINITY;
            bool dn = false;
            if (me) {
                const double js_me[3] = {stg->a[me_l], stg->b[me_l], stg->tau[me_l]};
                D = kl_with_inv(js_me, stage_cov(stg, me_l), stage_inv(stg, me_l), jm, mc, im);
                if (D != D) { dn = true; D = INFINITY; }
            }
            if (c.grp.any(dn)) {
                if (c.grp.gl == 0) raise_node(err, c.v, GTF_ERR_NAN_KL);
                break;
            }
            const double mind = c.grp.min_d(D);
            if (!(mind < kl_thr)) break;
            const int m = c.grp.min_i((me && D == mind) ? pos : 99);  // first minimum (list.index)
            const int lm = sb + stg->ord[sb + m];
            const Cov5 ii = stage_inv(stg, lm);
            const Cov5 nmc = inv_cov5(add_cov5(ii, im));
            const double ps[3] = {stg->a[lm], stg->b[lm], stg->c[lm]};
            const double js[3] = {ps[0], ps[1], stg->tau[lm]};
            double npm[3], njm[3];
            merge_with_inv(ps, ii, pm, im, nmc, npm);
            merge_with_inv(js, ii, jm, im, nmc, njm);
            pm[0] = npm[0]; pm[1] = npm[1]; pm[2] = npm[2];
            jm[0] = njm[0]; jm[1] = njm[1]; jm[2] = njm[2];
            mc = nmc;
            mprior = stg->prior[lm] + mprior;
            alive &= ~(1u << m);
            if (alive == 0) break;
        }
    }
#endif
    wave_lds_sync();
    if (c.grp.gl == 0) {                                                           // :291-293
        n.has_merged[c.v] = 1;
        n.merged_state[3 * (int64_t)c.v + 0] = pm[0];
        n.merged_state[3 * (int64_t)c.v + 1] = pm[1];
        n.merged_state[3 * (int64_t)c.v + 2] = pm[2];
        store_cov5(n.merged_cov, c.v, mc);
        n.merged_prior[c.v] = mprior;
    }
    if (pres && (alive >> pos & 1u) && c.is_edge) c.act = 0;                       // :311-321
    uint8_t* sc = reinterpret_cast<const gtf_diag*>(reinterpret_cast<const char*>(err) + GTF_DIAG_OFFSET)->slot_cluster;
    if (sc && pres) sc[c.k] = (alive >> pos & 1u) ? 2 : 1;   // diagnostics: merged (1) or left (2)
}

// LDS of one wavefront's clustering stages: the largest (64 / G) x sizeof(StageT<G>) over the
// group sizes (G = 2: 32 stages of 216 bytes; every other G: 6,784 bytes). Every wave's stages
// start at a multiple of this span whatever its G, so waves of one block that run different
// group sizes can never overlap each other's stages (round-5 verdict item 1).
template <int G>
constexpr size_t wave_stage_bytes() { return (size_t)(64 / G) * sizeof(StageT<G>); }
constexpr size_t max_sz(size_t a, size_t b) { return a > b ? a : b; }
constexpr size_t WAVE_STAGE_BYTES =
    max_sz(max_sz(max_sz(wave_stage_bytes<2>(), wave_stage_bytes<4>()), max_sz(wave_stage_bytes<8>(), wave_stage_bytes<16>())),
           max_sz(wave_stage_bytes<32>(), wave_stage_bytes<64>()));
static_assert(WAVE_STAGE_BYTES % 8 == 0, "stage spans keep 8-byte alignment");
constexpr size_t node_smem_bytes() { return NBLOCK * sizeof(double) + (NBLOCK / 64) * WAVE_STAGE_BYTES; }
// this lane's group's stage: the wave's own span, then the group's entry in it
template <typename Stage, int G>
__device__ __forceinline__ Stage* wave_stage(char* smem) {
    const int t = (int)threadIdx.x;
    return (Stage*)(smem + NBLOCK * sizeof(double) + (size_t)(t >> 6) * WAVE_STAGE_BYTES) + ((t & 63) / (G > 0 ? G : 64));
}

// ---------------------------------------------------------------------------
// kernels: load a node's slots into lane registers, run the ops, write back
// ---------------------------------------------------------------------------
// the per-slot fields an op sequence reads from memory (the others it only writes)
struct Need {
    bool tse_rank, tse_prior, uts_rank, uts_mw, uts_prior, uts_lik, uts_live, uts_fresh, send_mw;
    bool src, node_xyzr, solo;   // slot_src (UTS clustering), the node's own scalars an op reads
};

template <int G>
__device__ __forceinline__ bool node_fields(NodeCtx<G>& c, const gtf_graph& g, const gtf_states& tse,
                                            const gtf_states& uts, const gtf_edges& e, const Need& nd);

// the padded tile layout (gtf_graph.pad_*) of one lane-group size: c nodes per tile
struct Arith {
    int32_t c, node_off, slot_off, tn, ts;
};

template <int G>
__device__ __forceinline__ bool node_load(NodeCtx<G>& c, const gtf_graph& g, const gtf_nodes& n,
                                          const gtf_states& tse, const gtf_states& uts, const gtf_edges& e,
                                          const int32_t* list, const int32_t* seg, int count, int gi,
                                          const Need& nd, const Arith ar = Arith{0, 0, 0, 0, 0}) {
    if (gi >= count) return false;  // group-uniform
#ifndef GTF_PAD_ARITH   // the padded layout's arithmetic addressing (diagnostics builds): its
#define GTF_PAD_ARITH 0    // arguments raise the fused kernel's SGPR spills 64 -> 120, +2-4 us on tiled
#endif
    if (GTF_PAD_ARITH && G > 0 && ar.c > 0) {   // padded tiles: node and slots by arithmetic, no schedule loads
        const int t = gi / ar.c, i = gi - t * ar.c;
        c.v = t * ar.tn + ar.node_off + i;
        c.lo = t * ar.ts + ar.slot_off + i * G;
        c.d = G;
        return node_fields(c, g, tse, uts, e, nd);
    }
    c.v = list[gi];
    if (seg) {  // the slot segment stored beside the schedule entry: no dependent slot_ptr gather
        const int2 sg = reinterpret_cast<const int2*>(seg)[gi];
        c.lo = sg.x;
        c.d = sg.y - sg.x;
    } else {
        c.lo = g.slot_ptr[c.v];
        c.d = g.slot_ptr[c.v + 1] - c.lo;
    }
    return node_fields(c, g, tse, uts, e, nd);
}

// the per-slot fields of the lane's slot (c.v, c.lo, c.d and the group set)
template <int G>
__device__ __forceinline__ bool node_fields(NodeCtx<G>& c, const gtf_graph& g, const gtf_states& tse,
                                            const gtf_states& uts, const gtf_edges& e, const Need& nd) {
    c.k = c.lo + c.grp.gl;
    c.valid = c.grp.gl < c.d;
    const int k = c.k;
    c.act = c.valid ? e.act[k] : 0;
    c.act0 = c.act;
    // the graph-static classes of the slot (gtf_graph.slot_class) where they cover the group,
    // else the sender layer the priors build them from
    c.use_cls = G > 0 && ((G <= 32 && g.slot_class != nullptr) || (G == 64 && g.slot_xclass != nullptr));
    c.cls = 0;
    c.xcls = 0;
    c.sfl = 0;
    c.layer = NAN;
    // groups of <= 8 lanes: the slot's static fields in one word (gtf_graph.slot_static)
    const bool st32 = G > 0 && G <= 8 && g.slot_static != nullptr;
    if (st32) {
        const uint32_t sw = c.valid ? g.slot_static[k] : 0u;
        c.is_edge = (sw >> 16) & 1u;
        c.rev_edge = (sw >> 17) & 1u;
        c.sfl = (sw >> 18) & 1u;
        c.cls = (uint64_t)(sw & 0xffu) | ((uint64_t)((sw >> 8) & 0xffu) << 32);
        c.use_cls = true;
    } else {
        c.is_edge = c.valid ? g.is_edge[k] : 0;
        c.rev_edge = c.valid ? g.rev_edge[k] : 0;
    }
    if (st32) {
    } else if (c.use_cls) {
        if (c.valid) {
            c.cls = g.slot_class[k];
            c.sfl = g.slot_sflags[k];
            if (G == 64) c.xcls = g.slot_xclass[k];
        }
    } else if (g.slot_layer) {
        c.layer = c.valid ? g.slot_layer[k] : NAN;
    } else {
        const int src = c.valid ? g.slot_src[k] : -1;
        c.layer = src >= 0 ? g.layer[src] : NAN;
    }
    // the sender index: the clustering's coordinate gather of a live entry, not needed with
    // the slots' own copy (gtf_graph.slot_sxzr)
    c.src = (nd.src && c.valid && !g.slot_sxzr) ? g.slot_src[k] : -1;
    c.live = false;
    c.left = false;
    c.same_layer = 0;
    c.same_layer_ok = false;
    c.same_x = 0;
    c.same_x_ok = false;
    c.tse = LaneDict{-1, 0.0, 0.0, 0, -1, false, 0, false};
    c.uts = LaneDict{-1, 0.0, 0.0, 0, -1, false, 0, false};
    c.lik = 0; c.lr = 0; c.edge_mw = 0; c.side = -1; c.fresh = 0;
    c.uts_dirty_lr = false; c.edge_mw_dirty = false; c.degree = 0; c.degree_set = false;
    c.staged = false;
    c.lri = 1;
#if GTF_HOIST
    // the node's own scalars, in the same round of loads as the slot fields (loaded inside
    // an op, after its LDS fences, each one's latency would add to every wave's life)
    if (nd.node_xyzr && c.d >= 3) {   // (read by the clustering only: >= 3 keys, clustering.py:207)
        const double* xn = g.xyzr + 4 * (int64_t)c.v;
        c.xa = xn[0]; c.za = xn[2]; c.ra = xn[3];
    }
    if (nd.solo) c.solo = g.solo[c.v];
#endif
    // only what an op reads: mw of the TSE dict, lr and side are written, never read
    // (the reweight sets lr / side of every key it weighs before using them)
    if (c.valid) {
        if (nd.tse_rank) c.tse.rank = tse.rank[k];
        if (nd.tse_prior) c.tse.prior = tse.prior[k];
        if (nd.uts_rank) c.uts.rank = uts.rank[k];
        if (nd.uts_mw) c.uts.mw = uts.mw[k];
        if (nd.uts_prior) c.uts.prior = uts.prior[k];
        if (nd.uts_lik) c.lik = uts.lik[k];
        if (nd.uts_fresh || nd.uts_live) {
            const uint8_t f = uts.fresh[k];
            c.fresh = f & 1;          // written by the last message passing
            c.live = (f & 2) != 0;    // its xyzr = gnn[slot_src]
        }
        if (nd.send_mw) c.smw = e.send_mw[k];
    }
    return true;
}

#ifndef GTF_FULL_STORES
#define GTF_FULL_STORES 0   // 1 (A/B): the loaded fields (activation, ranks, UTS weight) stored for every valid slot, so a
                            // wave's stores cover whole lines instead of the dirty slots only
#endif
template <int G>
__device__ __forceinline__ void node_store(NodeCtx<G>& c, gtf_nodes& n, gtf_states& tse, gtf_states& uts,
                                           gtf_edges& e, const Need& nd) {
    const int k = c.k;
    if (GTF_FULL_STORES && c.valid) {
        e.act[k] = c.act;
        if (nd.tse_rank) tse.rank[k] = c.tse.rank;
        if (nd.uts_rank) uts.rank[k] = c.uts.rank;
        if (nd.uts_mw) uts.mw[k] = c.uts.mw;
        c.act0 = c.act;
        c.tse.dirty &= (uint8_t)~D_RANK;
        c.uts.dirty &= (uint8_t)~(D_RANK | (nd.uts_mw ? D_MW : 0));
    }
#if GTF_ABLATE == 6
    if (c.valid && c.act != c.act0) e.act[k] = c.act;   // diagnostics build: the activation store only
    return;
#endif
    if (c.valid) {
        if (c.act != c.act0) e.act[k] = c.act;
        if (c.edge_mw_dirty) e.edge_mw[k] = c.edge_mw;
        if (c.tse.dirty & D_RANK) tse.rank[k] = c.tse.rank;
        if (c.tse.dirty & D_MW) tse.mw[k] = c.tse.mw;
        if (c.tse.dirty & D_PRIOR) tse.prior[k] = c.tse.prior;
        if (c.uts.dirty & D_RANK) uts.rank[k] = c.uts.rank;
        if (c.uts.dirty & D_MW) uts.mw[k] = c.uts.mw;
        if (c.uts.dirty & D_PRIOR) uts.prior[k] = c.uts.prior;
        if (c.uts_dirty_lr) { uts.lr[k] = c.lr; uts.side[k] = c.side; }
    }
    if (c.degree_set && c.grp.gl == 0) n.degree[c.v] = c.degree;
}

// OP_FLUSH: the fields no later op of a compile-time sequence changes (the TSE dict, the UTS
// ranks, lr / side and the edge weight once the last reweight ran), stored before the
// clustering so their registers are free there; node_store then skips them
template <int G>
__device__ __forceinline__ void node_flush(NodeCtx<G>& c, gtf_states& tse, gtf_states& uts, gtf_edges& e) {
    const int k = c.k;
    if (c.valid) {
        if (c.edge_mw_dirty) e.edge_mw[k] = c.edge_mw;
        if (c.tse.dirty & D_RANK) tse.rank[k] = c.tse.rank;
        if (c.tse.dirty & D_MW) tse.mw[k] = c.tse.mw;
        if (c.tse.dirty & D_PRIOR) tse.prior[k] = c.tse.prior;
        if (c.uts.dirty & D_RANK) uts.rank[k] = c.uts.rank;
        if (c.uts_dirty_lr) { uts.lr[k] = c.lr; uts.side[k] = c.side; }
    }
    c.edge_mw_dirty = false;
    c.tse.dirty = 0;
    c.uts.dirty &= (uint8_t)~D_RANK;
    c.uts_dirty_lr = false;
}

#ifndef GTF_ASM_MARK
#define GTF_ASM_MARK 0   // assembly-listing builds only: a comment line before every op (tools/asm_ops.py)
#endif
template <int G, int OP, typename Stage>
__device__ __forceinline__ void node_op(NodeCtx<G>& c, const gtf_graph& g, gtf_nodes& n, gtf_states& tse,
                                        gtf_states& uts, gtf_edges& e, const gtf_params& p, const Ws& w,
                                        double* sval, Stage* stg, double chi2_thr, double kl_thr, bool has_tse,
                                        bool has_uts, const Need& nd) {
#if GTF_ASM_MARK
    asm volatile("; GTF_OP_MARK G=%0 OP=%1" ::"i"(G), "i"(OP));
#endif
    if constexpr (OP == OP_FLUSH) node_flush(c, tse, uts, e);
    if constexpr (OP == OP_FRESH) g_fresh(c);
    if constexpr (OP == OP_RANKS) g_ranks(c);
    if constexpr (OP == OP_PRIORS_TSE) { if (has_tse) g_priors(c, c.tse, sval); }
    if constexpr (OP == OP_PRIORS_UTS) { if (has_uts) g_priors(c, c.uts, sval); }
    if constexpr (OP == OP_REWEIGHT_UTS) { if (has_uts) g_reweight(c, sval, g, uts, p.reweight_threshold, w.err); }
    if constexpr (OP == OP_DEGREE) g_degree(c);
    if constexpr (OP == OP_PRUNE) g_prune(c, has_tse, has_uts, w.err);
#if GTF_HOIST
    if constexpr (OP == OP_MW_TSE) { if (has_tse) g_mixture_weights(c, c.tse, c.solo, w.err); }
    if constexpr (OP == OP_MW_UTS) { if (has_uts) g_mixture_weights(c, c.uts, c.solo, w.err); }
#else
    if constexpr (OP == OP_MW_TSE) { if (has_tse) g_mixture_weights(c, c.tse, g.solo[c.v], w.err); }
    if constexpr (OP == OP_MW_UTS) { if (has_uts) g_mixture_weights(c, c.uts, g.solo[c.v], w.err); }
#endif
    // (a 2-lane group holds <= 2 keys: the clustering returns before doing anything,
    // clustering.py:207, so it is not compiled in there)
    if constexpr (OP == OP_CLUSTER_TSE && G != 2) {
        if (has_tse)
            g_cluster(c, n, tse, c.tse, stg, g.xyzr + 4 * (int64_t)c.v, g.gnn, false, chi2_thr, kl_thr, p, w.err,
                      g.slot_sxzr, nd.tse_prior);
    }
    if constexpr (OP == OP_CLUSTER_UTS && G != 2) {
        if (has_uts)
            g_cluster(c, n, uts, c.uts, stg, g.xyzr + 4 * (int64_t)c.v, g.gnn, c.live, chi2_thr, kl_thr, p, w.err,
                      g.slot_sxzr, nd.uts_prior);
    }
}

// true when every OP_REWEIGHT_UTS of the sequence follows an OP_PRIORS_UTS with no op between
// them that adds keys (OP_RANKS / OP_FRESH): the reweight then reads only priors the sequence
// itself set (every active key's, helper.py:30-63), and the stored UTS priors need not be
// loaded up front -- the clustering reads a key's stored prior where no op set it
#ifndef GTF_LAZY_PRIOR
#define GTF_LAZY_PRIOR 1   // 0 (A/B): the UTS priors loaded up front whenever a reweight runs
#endif
template <int... OPS>
constexpr bool priors_before_reweights() {
    if (!GTF_LAZY_PRIOR) return false;
    constexpr int ops[] = {OPS..., -1};
    bool fresh_priors = false;
    for (int i = 0; ops[i] >= 0; i++) {
        if (ops[i] == OP_PRIORS_UTS) fresh_priors = true;
        if (ops[i] == OP_RANKS || ops[i] == OP_FRESH) fresh_priors = false;
        if (ops[i] == OP_REWEIGHT_UTS && !fresh_priors) return false;
    }
    return true;
}

template <int... OPS>
struct OpSeq {
    static constexpr bool uses_tse =
        ((OPS == OP_PRIORS_TSE || OPS == OP_MW_TSE || OPS == OP_CLUSTER_TSE || OPS == OP_PRUNE) || ...);
    static constexpr bool uses_uts = ((OPS == OP_FRESH || OPS == OP_RANKS || OPS == OP_PRIORS_UTS || OPS == OP_REWEIGHT_UTS ||
                                       OPS == OP_MW_UTS || OPS == OP_CLUSTER_UTS || OPS == OP_PRUNE) || ...);
    static constexpr bool cluster = ((OPS == OP_CLUSTER_TSE || OPS == OP_CLUSTER_UTS) || ...);
    static constexpr bool reweight = ((OPS == OP_REWEIGHT_UTS) || ...);
    static constexpr bool fresh = ((OPS == OP_FRESH) || ...);
    static constexpr bool cluster_uts = ((OPS == OP_CLUSTER_UTS) || ...);
    static constexpr Need need{uses_tse, ((OPS == OP_CLUSTER_TSE) || ...), uses_uts, reweight,
                               reweight && !priors_before_reweights<OPS...>(), reweight, reweight || cluster_uts,
                               ((OPS == OP_RANKS) || ...) || fresh, fresh && !GTF_MW_IN_EXTRAP,
                               cluster_uts, cluster, ((OPS == OP_MW_TSE || OPS == OP_MW_UTS) || ...)};
};

// has_uts of the node; where the sequence finishes message passing (OP_FRESH) a node that
// received an entry gets its updated_track_states dict here (extrapolate_merged_states.py
// :441-447), one store by the group's first lane instead of one per accepted slot
template <int G>
__device__ __forceinline__ bool fresh_has_uts(const NodeCtx<G>& c, gtf_nodes& n, bool with_fresh) {
    bool h = n.has_uts[c.v];
    if (with_fresh && !h && c.grp.any(c.valid && c.fresh)) {
        h = true;
        if (c.grp.gl == 0) n.has_uts[c.v] = 1;
    }
    return h;
}

__device__ __forceinline__ bool ops_have_fresh(const NodeOps& ops) {
    for (int i = 0; i < ops.n; i++)
        if (ops.op[i] == OP_FRESH) return true;
    return false;
}

// Diagnostics build GTF_OP_TIMING=1: lane 0 of every wavefront (up to
// GTF_OP_TIMING_WAVES) records the shader clock at its start, after its loads, after every
// op of the sequence and after its stores (row of 24 words per wave; word 23 = G), read
// back by gtf_op_timing (tools/op_timing.py); words 20 / 21 = the chip-wide real-time
// clock at the start / end (the shader clocks of different XCDs are not aligned)
#if GTF_OP_TIMING
template <int G, int OP, typename Stage>
__device__ __forceinline__ void node_op_timed(NodeCtx<G>& c, const gtf_graph& g, gtf_nodes& n, gtf_states& tse,
                                              gtf_states& uts, gtf_edges& e, const gtf_params& p, const Ws& w, double* sval,
                                              Stage* stg, double chi2_thr, double kl_thr, bool has_tse, bool has_uts,
                                              const Need& nd, uint64_t* tb, int& ti) {
    node_op<G, OP, Stage>(c, g, n, tse, uts, e, p, w, sval, stg, chi2_thr, kl_thr, has_tse, has_uts, nd);
    const uint64_t t = __builtin_readcyclecounter();
    if (tb && ti < 20) tb[ti] = t;
    ti++;
}
#endif

// compile-time op sequence for one group size: dead ops are compiled out.
// `bid` is the block index inside this bucket's range of the launch.
template <int G, int... OPS>
__device__ __forceinline__ void node_seq_body(const gtf_graph& g, gtf_nodes& n, gtf_states& tse, gtf_states& uts,
                                              gtf_edges& e, const gtf_params& p, const Ws& w, double chi2_thr,
                                              double kl_thr, const int32_t* list, const int32_t* seg, int count,
                                              int bid, char* smem, const Arith ar) {
    using Q = OpSeq<OPS...>;
    using Stage = StageT<G>;
    NodeCtx<G> c;
    const int gi = (bid * NBLOCK + (int)threadIdx.x) / G;
#if GTF_OP_TIMING
    const uint64_t t_start = __builtin_readcyclecounter();
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();   // chip-wide constant-rate clock
    const int wave = (int)((blockIdx.x * NBLOCK + threadIdx.x) / 64);
    uint64_t* tb = ((threadIdx.x & 63) == 0 && wave < GTF_OP_TIMING_WAVES) ? g_op_time + 24 * (int64_t)wave : nullptr;
    int ti = 2;
#endif
    if (!node_load(c, g, n, tse, uts, e, list, seg, count, gi, Q::need, ar)) return;
#if GTF_OP_TIMING
    {
        const uint64_t t = __builtin_readcyclecounter();
        if (tb) { tb[0] = t_start; tb[1] = t; tb[20] = rt_start; tb[23] = (uint64_t)G; }
    }
#endif
    double* sval = (double*)smem + (threadIdx.x & ~63);
    Stage* stg = Q::cluster ? wave_stage<Stage, G>(smem) : (Stage*)(smem + NBLOCK * sizeof(double));
#if GTF_EARLY_STAGE
    // the clustering operands of every slot of a node that may cluster (>= 3 slots), read
    // with the slot fields and parked in the group's LDS stage at the slot lane
    if constexpr (Q::cluster && G > 2) {
        c.staged = c.d >= 3;   // group-uniform
#if GTF_EARLY_STAGE == 2
        const bool maybe = c.valid && (Q::cluster_uts ? (c.uts.rank >= 0 || c.fresh) : c.tse.rank >= 0);
#else
        const bool maybe = c.valid;
#endif
        if (c.staged && maybe)
            stage_raw(stg, c.grp.gl, Q::cluster_uts ? uts : tse, c.k, g.gnn, Q::cluster_uts && c.live, c.src, g.slot_sxzr);
    }
#endif
    const bool has_tse = n.has_tse[c.v];
    const bool has_uts = fresh_has_uts(c, n, Q::fresh);
#if GTF_ABLATE == 4
    // diagnostics build: the node's loads and stores only (every field marked dirty)
    if (has_tse || has_uts) { c.uts.dirty = c.tse.dirty = D_RANK | D_MW | D_PRIOR; c.uts_dirty_lr = true; c.edge_mw_dirty = true; }
#elif GTF_OP_TIMING
    (node_op_timed<G, OPS, Stage>(c, g, n, tse, uts, e, p, w, sval, stg, chi2_thr, kl_thr, has_tse, has_uts, Q::need,
                                  tb, ti),
     ...);
#else
    (node_op<G, OPS, Stage>(c, g, n, tse, uts, e, p, w, sval, stg, chi2_thr, kl_thr, has_tse, has_uts, Q::need), ...);
#endif
#if GTF_ASM_MARK
    asm volatile("; GTF_OP_MARK G=%0 OP=99" ::"i"(G));
#endif
    node_store(c, n, tse, uts, e, Q::need);
#if GTF_ASM_MARK
    asm volatile("; GTF_OP_MARK G=%0 OP=100" ::"i"(G));
#endif
#if GTF_OP_TIMING
    {
        const uint64_t t = __builtin_readcyclecounter();
        const uint64_t rt = __builtin_amdgcn_s_memrealtime();
        if (tb && ti < 20) tb[ti] = t;
        if (tb) tb[21] = rt;
    }
#endif
}

struct Buckets {
    const int32_t* list[6];  // node lists for G = 64, 32, 16, 8, 4, 2 (slowest first)
    const int32_t* seg[6];   // their slot segments (gtf_graph.sched_seg) or NULL
    int32_t count[6];
    int32_t blocks[6];
    Arith ar[6];             // padded tile layout (ar[q].c > 0: addresses by arithmetic)
};

// All arguments of k_node_multi in one by-value struct (the kernarg segment).
struct NodeKArgs {
    gtf_graph g;
    gtf_nodes n;
    gtf_states tse, uts;
    gtf_edges e;
    gtf_params p;
    Ws w;
    double chi2_thr, kl_thr;
    Buckets bk;
};
typedef const __attribute__((address_space(4))) NodeKArgs* KArgPtr;

// The kernarg segment through an opaque copy of its address: the compiler cannot hoist the
// argument loads of the six bucket bodies into the kernel's entry (they are speculatable
// kernarg loads otherwise), where their union -- ~90 SGPRs of pointers live across the
// whole op sequence -- spilled 64 SGPRs into VGPR lanes on every wave. Each body now loads
// only its own arguments, where it uses them (scalar loads from the constant segment).
#ifndef GTF_KARG_LAUNDER
#define GTF_KARG_LAUNDER 1
#endif
__device__ __forceinline__ KArgPtr node_kargs() {
    uint64_t a = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
#if GTF_KARG_LAUNDER
    asm volatile("" : "+s"(a));
#endif
    return (KArgPtr)a;
}

template <int G, int... OPS>
__device__ __forceinline__ void node_bucket(int q, int b, char* smem) {
    const KArgPtr A = node_kargs();
    node_seq_body<G, OPS...>(*(const gtf_graph*)&A->g, *(gtf_nodes*)&A->n, *(gtf_states*)&A->tse,
                             *(gtf_states*)&A->uts, *(gtf_edges*)&A->e, *(const gtf_params*)&A->p,
                             *(const Ws*)&A->w, A->chi2_thr, A->kl_thr, A->bk.list[q], A->bk.seg[q],
                             A->bk.count[q], b, smem, *(const Arith*)&A->bk.ar[q]);
}

// one launch over every bucket: blocks of the long-running buckets (many slots per node)
// are dealt first so they overlap the bulk of small nodes instead of trailing it
#ifndef GTF_NODE_WAVES
#define GTF_NODE_WAVES 5   // > 0: amdgpu_waves_per_eu lower bound for the fused node kernel (register budget)
#endif
#if GTF_NODE_WAVES > 0
#define GTF_NODE_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(GTF_NODE_WAVES)))
#else
#define GTF_NODE_WAVES_ATTR
#endif
#ifndef GTF_NODE_XCD_CHUNK
#define GTF_NODE_XCD_CHUNK 4   // runs of this many consecutive blocks on one XCD (node_block_map; 1 = dispatch order)
#endif
// Dispatch block b (on XCD b % 8, round-robin) -> the block of work it runs: runs of C
// consecutive work blocks share an XCD, the runs of the 8 XCDs interleaved, so neighbouring
// nodes' slot lines meet in one L2 while every XCD still draws from every part of the
// launch (an XCD-contiguous remap of the whole launch, gtf::xcd_local, unbalanced the XCDs).
// C = 1 is the identity (gtf::block_map).
template <int C>
__device__ __forceinline__ int node_block_map(int b, int n) {
    return gtf::block_map<C < 1 ? 1 : C>(b, n);
}

template <int... OPS>
__global__ void __launch_bounds__(NBLOCK) GTF_NODE_WAVES_ATTR k_node_multi(NodeKArgs args) {
    (void)args;   // read through node_kargs()
    using Q = OpSeq<OPS...>;
    __shared__ __attribute__((aligned(16))) char smem[Q::cluster ? node_smem_bytes() : NBLOCK * sizeof(double)];
    // Blocks stay in dispatch order (round-robin over the XCDs): per-node cost varies
    // with the node's state count and clustering work, and an XCD-contiguous remap
    // (gtf::xcd_local) made this kernel 35 % slower on config 4, presumably by putting
    // the costly nodes of a node range on one XCD.
    const KArgPtr A = node_kargs();
    node_tables_init();
    __syncthreads();
    int b = node_block_map<GTF_NODE_XCD_CHUNK>((int)blockIdx.x, (int)gridDim.x);
#ifndef GTF_NODE_ORDER
#define GTF_NODE_ORDER 0   // 1 (diagnostics): the buckets by measured wave life, longest first (16, 32, 8, 64, 4, 2)
#endif
#if GTF_NODE_ORDER == 1
    if (b < A->bk.blocks[2]) { node_bucket<16, OPS...>(2, b, smem); return; }
    b -= A->bk.blocks[2];
    if (b < A->bk.blocks[1]) { node_bucket<32, OPS...>(1, b, smem); return; }
    b -= A->bk.blocks[1];
    if (b < A->bk.blocks[3]) { node_bucket<8, OPS...>(3, b, smem); return; }
    b -= A->bk.blocks[3];
    if (b < A->bk.blocks[0]) { node_bucket<64, OPS...>(0, b, smem); return; }
    b -= A->bk.blocks[0];
#else
    if (b < A->bk.blocks[0]) { node_bucket<64, OPS...>(0, b, smem); return; }
    b -= A->bk.blocks[0];
    if (b < A->bk.blocks[1]) { node_bucket<32, OPS...>(1, b, smem); return; }
    b -= A->bk.blocks[1];
    if (b < A->bk.blocks[2]) { node_bucket<16, OPS...>(2, b, smem); return; }
    b -= A->bk.blocks[2];
    if (b < A->bk.blocks[3]) { node_bucket<8, OPS...>(3, b, smem); return; }
    b -= A->bk.blocks[3];
#endif
    if (b < A->bk.blocks[4]) { node_bucket<4, OPS...>(4, b, smem); return; }
    b -= A->bk.blocks[4];
    node_bucket<2, OPS...>(5, b, smem);
}

// GTF_SPLIT_G2 (A/B): the <= 2-slot bucket in a launch of its own after the others, at
// GTF_G2_WAVES waves per SIMD (no clustering there, so far fewer registers, and no stage LDS)
#ifndef GTF_SPLIT_G2
#define GTF_SPLIT_G2 0
#endif
#ifndef GTF_G2_WAVES
#define GTF_G2_WAVES 8
#endif
template <int... OPS>
__global__ void __launch_bounds__(NBLOCK) __attribute__((amdgpu_waves_per_eu(GTF_G2_WAVES))) k_node_g2(NodeKArgs args) {
    (void)args;   // read through node_kargs()
    __shared__ __attribute__((aligned(16))) char smem[NBLOCK * sizeof(double)];
    node_tables_init();
    __syncthreads();
    node_bucket<2, OPS...>(5, node_block_map<GTF_NODE_XCD_CHUNK>((int)blockIdx.x, (int)gridDim.x), smem);
}

// Packed lane segments (gtf_graph.pack_ent / pack_wave): wavefront wv takes the entries
// [pack_wave[wv], pack_wave[wv + 1]), each (v, slot_ptr[v], slot_ptr[v+1], first lane),
// one lane per slot (one for a slot-free node) back to back, so 90+ % of the lanes hold a
// slot instead of the 59-88 % of power-of-two groups. Same op code as the groups (G = 0).
template <int... OPS>
__global__ void __launch_bounds__(NBLOCK) k_node_pack(gtf_graph g, gtf_nodes n, gtf_states tse, gtf_states uts,
                                                     gtf_edges e, gtf_params p, Ws w, double chi2_thr, double kl_thr) {
    using Q = OpSeq<OPS...>;
    using Stage = StageT<64>;   // one per wavefront, a group's states at [gbase + i]
    __shared__ __attribute__((aligned(16))) char smem[NBLOCK * sizeof(double) +
                                                      (Q::cluster ? (NBLOCK / 64) * sizeof(Stage) : 0)];
    __shared__ uint8_t s_start[NBLOCK];
    node_tables_init();
    __syncthreads();
    const int wv = blockIdx.x * (NBLOCK / 64) + (int)threadIdx.x / 64;
    if (wv >= g.n_pack_waves) return;  // wavefront-uniform
    const int lane = threadIdx.x & 63;
    const int e0 = g.pack_wave[wv], ne = g.pack_wave[wv + 1] - e0;
    int4 en = make_int4(0, 0, 0, 0);
    if (lane < ne) en = reinterpret_cast<const int4*>(g.pack_ent)[e0 + lane];
    uint8_t* st = s_start + (threadIdx.x & ~63);
    st[lane] = 0;
    wave_lds_sync();
    if (lane < ne) st[en.w] = 1;
    wave_lds_sync();
    const unsigned long long M = __ballot(st[lane] != 0);
    const int idx = __popcll(lane == 63 ? M : (M & ((2ull << lane) - 1ull))) - 1;  // my entry
    NodeCtx<0> c;
    c.v = __shfl(en.x, idx);
    c.lo = __shfl(en.y, idx);
    c.d = __shfl(en.z, idx) - c.lo;
    c.grp.gbase = __shfl(en.w, idx);
    c.grp.gsize = c.d > 0 ? c.d : 1;
    c.grp.gl = lane - c.grp.gbase;
    c.grp.lowmask = c.grp.gsize >= 64 ? ~0ull : ((1ull << c.grp.gsize) - 1ull);
    int mx = c.grp.gsize;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
    c.grp.wmax = mx;
    if (c.grp.gl >= c.grp.gsize) return;  // past the last segment
    if (!node_fields(c, g, tse, uts, e, Q::need)) return;
    double* sval = (double*)smem + (threadIdx.x & ~63);
    Stage* stg = (Stage*)(smem + NBLOCK * sizeof(double)) + (Q::cluster ? (int)threadIdx.x / 64 : 0);
    const bool has_tse = n.has_tse[c.v];
    const bool has_uts = fresh_has_uts(c, n, Q::fresh);
    (node_op<0, OPS, Stage>(c, g, n, tse, uts, e, p, w, sval, stg, chi2_thr, kl_thr, has_tse, has_uts, Q::need), ...);
    node_store(c, n, tse, uts, e, Q::need);
}

// run-time op sequence (gtf_node_ops): any order of any ops
template <int G>
__global__ void __launch_bounds__(NBLOCK) k_node_group(gtf_graph g, gtf_nodes n, gtf_states tse, gtf_states uts,
                                                      gtf_edges e, gtf_params p, Ws w, NodeOps ops,
                                                      double chi2_thr, double kl_thr, const int32_t* list,
                                                      const int32_t* seg, int count) {
    using Stage = StageT<G>;
    __shared__ double s_val[NBLOCK];
    __shared__ Stage s_stage[NBLOCK / G];
    node_tables_init();
    __syncthreads();
    NodeCtx<G> c;
    const int gi = (blockIdx.x * NBLOCK + (int)threadIdx.x) / G;
    const Need nd{(bool)ops.uses_tse, (bool)ops.uses_tse, (bool)ops.uses_uts, (bool)ops.uses_uts,
                  (bool)ops.uses_uts, (bool)ops.uses_uts, (bool)ops.uses_uts, (bool)ops.uses_uts,
                  (bool)ops.uses_uts, (bool)ops.uses_uts, true, true};
    if (!node_load(c, g, n, tse, uts, e, list, seg, count, gi, nd)) return;
    double* sval = s_val + (threadIdx.x & ~63);
    Stage* stg = s_stage + (int)threadIdx.x / G;
    const bool has_tse = n.has_tse[c.v];
    const bool has_uts = fresh_has_uts(c, n, ops_have_fresh(ops));
    for (int i = 0; i < ops.n; i++) {
        switch (ops.op[i]) {
#define GTF_CASE(OPC) \
    case OPC: node_op<G, OPC, Stage>(c, g, n, tse, uts, e, p, w, sval, stg, chi2_thr, kl_thr, has_tse, has_uts, nd); break;
            GTF_CASE(OP_FRESH)
            GTF_CASE(OP_RANKS)
            GTF_CASE(OP_PRIORS_TSE)
            GTF_CASE(OP_PRIORS_UTS)
            GTF_CASE(OP_REWEIGHT_UTS)
            GTF_CASE(OP_DEGREE)
            GTF_CASE(OP_PRUNE)
            GTF_CASE(OP_MW_TSE)
            GTF_CASE(OP_MW_UTS)
            GTF_CASE(OP_CLUSTER_TSE)
            GTF_CASE(OP_CLUSTER_UTS)
#undef GTF_CASE
            default: break;
        }
    }
    node_store(c, n, tse, uts, e, nd);
}
