// gtf_a15.hip -- pairwise distances between a node's updated track states (SURVEY §8
// a15): calculate_distance_between_updated_states/
// calculate_distance_between_updated_track_states.py, function mahalanobis_distance
// (:27-104) over the pair loop of :134-195, for gfx950.
//
// For every node with an updated_track_states dict (:143) and more than one active
// in-edge (:139-140), every pair i > j of the dict's entries in dict order (:174-176):
//   chi2 = [a,b] Mahalanobis term with (C_i + C_j)[:2,:2]^-1  +  delta-tau term with the
//          hard-coded sigma_z = 0.5 / sigma_r = 0.1, swapped to 0.1 / 0.5 where
//          |x| >= 600 (the x coordinate, as the reference tests it, :62-74);
//   <tau> = (tau_1 + tau_2) / 2, <theta> = (theta_1 + theta_2) / 2, dtheta = theta_1 - theta_2
//          with theta = atan2(dz, dr) (:89-99);
//   truth = node, neighbour 1 and neighbour 2 share a particle (:190-193).
// Coordinates are the node attribute xyzr of the node and of each neighbour (:162-163,
// :182-183).
//
// Work decomposition: one group of G lanes per node from the node schedule (gtf_graph.sched:
// G = 2 .. 64 by slot count), one slot per lane. Each lane turns its entry into the
// per-state pair operands once -- [a, b], the 2x2 covariance block, 1/dr, dz/dr^2, tau,
// theta, the endcap flag -- and stages them in LDS at its dict position; the group then
// deals the node's d(d-1)/2 pairs round-robin over its lanes (row-major t = i(i-1)/2 + j,
// the reference's loop order), so consecutive lanes write consecutive pairs. Nodes with
// more than 64 slots run one wavefront each, with a dict-position -> slot map in LDS and
// the operands read from HBM per pair.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/gtf.h"
#include "gtf_math.h"

using namespace gtf;

namespace {

constexpr int BLOCK = 256;
constexpr double SZ_BARREL = 0.5, SR_BARREL = 0.1;   // :63-64
constexpr double SZ_ENDCAP = 0.1, SR_ENDCAP = 0.5;   // :66-74
constexpr double ENDCAP_X = 600.0;                   // |x| >= 600.0 (:66, :69, :72)
constexpr int BIG_CAP = 2048;                        // dict entries of a > 64-slot node

struct PairOps {   // per-state operands of the pair terms
    double a, b, c00, c01, c10, c11, q, w, tau, theta;
    long long tr;
    uint8_t ec;
};

template <int CAP>
struct PairStage {
    double a[CAP], b[CAP], c00[CAP], c01[CAP], c10[CAP], c11[CAP], q[CAP], w[CAP], tau[CAP], theta[CAP];
    long long tr[CAP];
    uint8_t ec[CAP];
};

struct Args {
    gtf_graph g;
    gtf_nodes n;
    gtf_states uts;
    gtf_edges e;
    const int64_t* truth;
    const int64_t* pair_ptr;
    gtf_pair_out o;
};

__device__ __forceinline__ void flag(const Args& A, uint32_t f) {
    if (A.o.err) atomicOr(A.o.err, f);
}

// operands of the entry at slot k (sender u) for a node at (za, ra)
__device__ __forceinline__ PairOps pair_ops(const Args& A, int k, int u, double za, double ra) {
    PairOps s;
    s.a = A.uts.sv[3 * (int64_t)k];
    s.b = A.uts.sv[3 * (int64_t)k + 1];
    const double* cv = A.uts.cov + 5 * (int64_t)k;
    s.c00 = cv[0]; s.c01 = cv[1]; s.c10 = cv[2]; s.c11 = cv[3];
    const double* nb = A.g.xyzr + 4 * (int64_t)u;
    const TauGeo t = tau_geo(nb[0], nb[2], nb[3], za, ra, SZ_BARREL, SR_BARREL, SZ_ENDCAP, SR_ENDCAP, ENDCAP_X);
    s.q = t.q; s.w = t.w; s.tau = t.tau;
    s.theta = atan2(nb[2] - za, nb[3] - ra);                                       // :95-96
    s.ec = fabs(nb[0]) >= ENDCAP_X;
    s.tr = A.truth ? A.truth[u] : 0;
    return s;
}

__device__ __forceinline__ TauGeo geo_of(const PairOps& s) {
    TauGeo t;
    t.q = s.q; t.w = s.w; t.tau = s.tau;
    t.sz2 = s.ec ? SZ_ENDCAP * SZ_ENDCAP : SZ_BARREL * SZ_BARREL;
    t.sr2 = s.ec ? SR_ENDCAP * SR_ENDCAP : SR_BARREL * SR_BARREL;
    return t;
}

// one pair (i > j): chi2, <tau>, <theta>, dtheta, truth at out index t
__device__ __forceinline__ void write_pair(const Args& A, int64_t t, const PairOps& si, const PairOps& sj, double sza2,
                                           double sra2, long long tv) {
    const Cov5 ci{si.c00, si.c01, si.c10, si.c11, 0.0}, cj{sj.c00, sj.c01, sj.c10, sj.c11, 0.0};
    A.o.chi2[t] = mahalanobis_geo(si.a, si.b, ci, sj.a, sj.b, cj, sza2, sra2, geo_of(si), geo_of(sj));
    if (A.o.avg_tau) A.o.avg_tau[t] = (si.tau + sj.tau) / 2.0;                     // :97
    if (A.o.avg_theta) A.o.avg_theta[t] = (si.theta + sj.theta) / 2.0;             // :98
    if (A.o.delta_theta) A.o.delta_theta[t] = si.theta - sj.theta;                 // :99
    if (A.o.truth) A.o.truth[t] = (int8_t)(tv == si.tr && si.tr == sj.tr && tv == sj.tr);   // :192-193
}

template <typename St>
__device__ __forceinline__ void put(St* s, int i, const PairOps& p) {
    s->a[i] = p.a; s->b[i] = p.b; s->c00[i] = p.c00; s->c01[i] = p.c01; s->c10[i] = p.c10; s->c11[i] = p.c11;
    s->q[i] = p.q; s->w[i] = p.w; s->tau[i] = p.tau; s->theta[i] = p.theta; s->tr[i] = p.tr; s->ec[i] = p.ec;
}
template <typename St>
__device__ __forceinline__ PairOps get(const St* s, int i) {
    PairOps p;
    p.a = s->a[i]; p.b = s->b[i]; p.c00 = s->c00[i]; p.c01 = s->c01[i]; p.c10 = s->c10[i]; p.c11 = s->c11[i];
    p.q = s->q[i]; p.w = s->w[i]; p.tau = s->tau[i]; p.theta = s->theta[i]; p.tr = s->tr[i]; p.ec = s->ec[i];
    return p;
}

// the node's sigma pair (:62-67, tested on the node's x)
__device__ __forceinline__ void node_sigmas(const double* na, double& sza2, double& sra2) {
    const bool ec = fabs(na[0]) >= ENDCAP_X;
    const double sza = ec ? SZ_ENDCAP : SZ_BARREL, sra = ec ? SR_ENDCAP : SR_BARREL;
    sza2 = sza * sza;
    sra2 = sra * sra;
}

// pairs the node must have: d(d-1)/2 for a node the loop visits, else 0
__device__ __forceinline__ int64_t want_pairs(bool visit, int d) { return visit ? (int64_t)d * (d - 1) / 2 : 0; }

// this group's lanes of a wave-wide ballot
template <int G>
__device__ __forceinline__ unsigned long long group_bits(bool pred) {
    const unsigned long long b = __ballot(pred);
    if constexpr (G == 64) return b;
    else return (b >> (threadIdx.x & 63 & ~(G - 1))) & ((1ull << G) - 1ull);
}

// one node on G lanes (slots <= G)
template <int G>
__device__ __forceinline__ void group_node(const Args& A, const int32_t* list, const int32_t* seg, int count, int b,
                                           char* smem) {
    using Stage = PairStage<G>;
    const int gi = (b * BLOCK + (int)threadIdx.x) / G;
    if (gi >= count) return;  // group-uniform
    const int gl = threadIdx.x & (G - 1);
    const int v = list[gi];
    int lo, hi;
    if (seg) { lo = seg[2 * gi]; hi = seg[2 * gi + 1]; }
    else { lo = A.g.slot_ptr[v]; hi = A.g.slot_ptr[v + 1]; }
    const int k = lo + gl;
    const bool valid = k < hi;
    const int rank = valid ? A.uts.rank[k] : -1;
    const bool pres = rank >= 0;
    const bool act = valid && A.g.is_edge[k] && A.e.act[k] == 1;
    const int nact = __popcll(group_bits<G>(act));
    // dict position = present keys with a smaller rank
    int pos = 0, d = 0;
    for (int j = 0; j < G; j++) {
        const int rj = __shfl(rank, j, G);
        d += rj >= 0;
        pos += (rj >= 0 && rj < rank) ? 1 : 0;
    }
    const bool visit = A.n.has_uts[v] && nact > 1;                                 // :139-143
    const int64_t base = A.pair_ptr[v];
    if (A.pair_ptr[v + 1] - base != want_pairs(visit, d)) {
        if (gl == 0) flag(A, GTF_ERR_PAIR_COUNT);
        return;
    }
    if (!visit || d < 2) return;
    const double* na = A.g.xyzr + 4 * (int64_t)v;
    const double za = na[2], ra = na[3];
    const int src = valid ? A.g.slot_src[k] : -1;
    if (group_bits<G>(pres && src < 0)) {
        if (gl == 0) flag(A, GTF_ERR_NEIGHBOUR_MISSING);                           // KeyError :182-183
        return;
    }
    Stage* stg = (Stage*)smem + (int)threadIdx.x / G;
    if (pres) put(stg, pos, pair_ops(A, k, src, za, ra));
    wave_lds_sync();
    double sza2, sra2;
    node_sigmas(na, sza2, sra2);
    const long long tv = A.truth ? A.truth[v] : 0;
    const int np = d * (d - 1) / 2;
    for (int t = gl; t < np; t += G) {
        int i, j;
        pair_ij(t, i, j);
        write_pair(A, base + t, get(stg, i), get(stg, j), sza2, sra2, tv);
    }
}

struct Buckets {
    const int32_t* list[6];  // G = 64, 32, 16, 8, 4, 2
    const int32_t* seg[6];
    int32_t count[6];
    int32_t blocks[6];
};

template <int G>
constexpr size_t stage_bytes() { return (size_t)(BLOCK / G) * sizeof(PairStage<G>); }
constexpr size_t cmax(size_t a, size_t b) { return a > b ? a : b; }
constexpr size_t group_smem() {
    return cmax(cmax(cmax(stage_bytes<64>(), stage_bytes<32>()), cmax(stage_bytes<16>(), stage_bytes<8>())),
                cmax(stage_bytes<4>(), stage_bytes<2>()));
}

__global__ void __launch_bounds__(BLOCK) k_pairs_groups(Args A, Buckets bk) {
    __shared__ __attribute__((aligned(16))) char smem[group_smem()];
    int b = blockIdx.x;
    if (b < bk.blocks[0]) { group_node<64>(A, bk.list[0], bk.seg[0], bk.count[0], b, smem); return; }
    b -= bk.blocks[0];
    if (b < bk.blocks[1]) { group_node<32>(A, bk.list[1], bk.seg[1], bk.count[1], b, smem); return; }
    b -= bk.blocks[1];
    if (b < bk.blocks[2]) { group_node<16>(A, bk.list[2], bk.seg[2], bk.count[2], b, smem); return; }
    b -= bk.blocks[2];
    if (b < bk.blocks[3]) { group_node<8>(A, bk.list[3], bk.seg[3], bk.count[3], b, smem); return; }
    b -= bk.blocks[3];
    if (b < bk.blocks[4]) { group_node<4>(A, bk.list[4], bk.seg[4], bk.count[4], b, smem); return; }
    b -= bk.blocks[4];
    group_node<2>(A, bk.list[5], bk.seg[5], bk.count[5], b, smem);
}

// nodes with more than 64 slots (or every node without a schedule): one wavefront each
__global__ void __launch_bounds__(64) k_pairs_wave(Args A, const int32_t* list, int count) {
    __shared__ int32_t s_slot[BIG_CAP];
    const int gi = blockIdx.x;
    if (gi >= count) return;
    const int lane = threadIdx.x;
    const int v = list ? list[gi] : gi;
    const int lo = A.g.slot_ptr[v], hi = A.g.slot_ptr[v + 1];
    int d = 0, nact = 0;
    bool orphan = false;
    for (int k = lo + lane; k < hi; k += 64) {
        const int r = A.uts.rank[k];
        d += r >= 0;
        nact += (A.g.is_edge[k] && A.e.act[k] == 1) ? 1 : 0;
        orphan |= r >= 0 && A.g.slot_src[k] < 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        d += __shfl_xor(d, o);
        nact += __shfl_xor(nact, o);
    }
    const bool visit = A.n.has_uts[v] && nact > 1;
    const int64_t base = A.pair_ptr[v];
    if (A.pair_ptr[v + 1] - base != want_pairs(visit, d)) {
        if (lane == 0) flag(A, GTF_ERR_PAIR_COUNT);
        return;
    }
    if (!visit || d < 2) return;
    if (d > BIG_CAP) {
        if (lane == 0) flag(A, GTF_ERR_TOO_MANY_STATES);
        return;
    }
    if (__ballot(orphan)) {
        if (lane == 0) flag(A, GTF_ERR_NEIGHBOUR_MISSING);
        return;
    }
    // dict position of every present key (ranks may be out of slot order after pruning)
    for (int k = lo + lane; k < hi; k += 64) {
        const int r = A.uts.rank[k];
        if (r < 0) continue;
        int pos = 0;
        for (int j = lo; j < hi; j++) {
            const int rj = A.uts.rank[j];
            pos += (rj >= 0 && rj < r) ? 1 : 0;
        }
        s_slot[pos] = k;
    }
    __syncthreads();
    const double* na = A.g.xyzr + 4 * (int64_t)v;
    double sza2, sra2;
    node_sigmas(na, sza2, sra2);
    const long long tv = A.truth ? A.truth[v] : 0;
    const int64_t np = (int64_t)d * (d - 1) / 2;
    for (int64_t t = lane; t < np; t += 64) {
        int i, j;
        pair_ij((int)t, i, j);
        const int ki = s_slot[i], kj = s_slot[j];
        write_pair(A, base + t, pair_ops(A, ki, A.g.slot_src[ki], na[2], na[3]),
                   pair_ops(A, kj, A.g.slot_src[kj], na[2], na[3]), sza2, sra2, tv);
    }
}

// pairs per node (0 or d(d-1)/2): one thread per node
__global__ void __launch_bounds__(BLOCK) k_pair_counts(Args A, int64_t* counts) {
    const int v = blockIdx.x * BLOCK + threadIdx.x;
    if (v >= A.g.n_nodes) return;
    const int lo = A.g.slot_ptr[v], hi = A.g.slot_ptr[v + 1];
    int d = 0, nact = 0;
    for (int k = lo; k < hi; k++) {
        d += A.uts.rank[k] >= 0;
        nact += (A.g.is_edge[k] && A.e.act[k] == 1) ? 1 : 0;
    }
    counts[v] = want_pairs(A.n.has_uts[v] && nact > 1, d);
}

int check_args(const gtf_graph* g, const gtf_nodes* n, const gtf_states* uts, const gtf_edges* e) {
    if (int rc = gtf::check_abi(g, "gtf_updated_state_distances")) return rc;
    if (!n || !uts || !e) { gtf::set_error("a15: null argument"); return -2; }
    if (g->n_nodes < 0 || g->n_slots < 0) { gtf::set_error("a15: negative sizes"); return -2; }
    if (g->n_nodes > 0 && (!g->slot_ptr || !g->xyzr || !n->has_uts)) { gtf::set_error("a15: missing arrays"); return -2; }
    if (g->n_slots > 0 && (!g->slot_src || !g->is_edge || !uts->rank || !uts->sv || !uts->cov || !e->act)) {
        gtf::set_error("a15: missing slot arrays");
        return -2;
    }
    return 0;
}

int done() {
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        gtf::set_error(hipGetErrorString(err));
        return -1;
    }
    return 0;
}

}  // namespace

extern "C" int gtf_updated_state_pair_counts(const gtf_graph* g, const gtf_nodes* n, const gtf_states* uts,
                                             const gtf_edges* e, int64_t* counts, gtf_stream_t stream) {
    int rc = check_args(g, n, uts, e);
    if (rc) return rc;
    if (g->n_nodes == 0) return 0;
    if (!counts) { gtf::set_error("a15: null counts"); return -2; }
    Args A{*g, *n, *uts, *e, nullptr, nullptr, gtf_pair_out{}};
    hipLaunchKernelGGL(k_pair_counts, dim3((g->n_nodes + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, (hipStream_t)stream, A,
                       counts);
    return done();
}

extern "C" int gtf_updated_state_distances(const gtf_graph* g, const gtf_nodes* n, const gtf_states* uts,
                                           const gtf_edges* e, const int64_t* truth, const int64_t* pair_ptr,
                                           const gtf_pair_out* out, gtf_stream_t stream) {
    int rc = check_args(g, n, uts, e);
    if (rc) return rc;
    if (!out || !pair_ptr || !out->chi2) { gtf::set_error("a15: missing pair_ptr / chi2 output"); return -2; }
    if (out->truth && !truth) { gtf::set_error("a15: truth output needs node truth"); return -2; }
    if (g->n_nodes == 0) return 0;
    Args A{*g, *n, *uts, *e, truth, pair_ptr, *out};
    hipStream_t st = (hipStream_t)stream;
    if (g->sched) {
        Buckets bk;
        const int n2 = g->n_g2 > 0 && g->n_g2 <= g->n_g4 ? g->n_g2 : 0;
        const int cnt[6] = {g->n_g64, g->n_g32, g->n_g16, g->n_g8, g->n_g4 - n2, n2};
        const int gs[6] = {64, 32, 16, 8, 4, 2};
        const int32_t* s8 = g->sched + g->n_g4;
        const int32_t* starts[6] = {s8 + g->n_g8 + g->n_g16 + g->n_g32, s8 + g->n_g8 + g->n_g16, s8 + g->n_g8, s8,
                                    g->sched + n2, g->sched};
        int total = 0;
        for (int q = 0; q < 6; q++) {
            bk.list[q] = starts[q];
            bk.seg[q] = g->sched_seg ? g->sched_seg + 2 * (starts[q] - g->sched) : nullptr;
            bk.count[q] = cnt[q];
            bk.blocks[q] = (cnt[q] + BLOCK / gs[q] - 1) / (BLOCK / gs[q]);
            total += bk.blocks[q];
        }
        if (total > 0) hipLaunchKernelGGL(k_pairs_groups, dim3(total), dim3(BLOCK), 0, st, A, bk);
        const int ng = g->n_g4 + g->n_g8 + g->n_g16 + g->n_g32 + g->n_g64;
        if (g->n_big > 0) hipLaunchKernelGGL(k_pairs_wave, dim3(g->n_big), dim3(64), 0, st, A, g->sched + ng, g->n_big);
    } else {
        hipLaunchKernelGGL(k_pairs_wave, dim3(g->n_nodes), dim3(64), 0, st, A, (const int32_t*)nullptr, g->n_nodes);
    }
    return done();
}
