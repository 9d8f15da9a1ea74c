// gtf_pass.hip -- the extrapolate -> update -> cluster pass as HIP kernels for
// gfx950 (MI355X), behind the C-ABI of include/gtf.h.
//
// Work decomposition (DESIGN.md "Kernels"):
//   k_sender         8 lanes / sender node over its out-edges (successor order): Highland
//                     var_ms per edge and the running merged_cov[1,1] += var_ms each
//                     extrapolation sees -- the in-place mutation of
//                     extrapolate_merged_states.py:127-128 -- as a sequential scan.
//   k_extrapolate     1 thread / slot (receiver-major, coalesced writes of the new
//                     updated_track_states entry): parabolic extrapolation, chi2 gate,
//                     Kalman predict + update (extrapolate_merged_states.py:26-402).
//   k_node_*          1 thread / receiver node over its slot segment: everything after
//                     message passing only reads/writes the node's own in-edge segment
//                     (priors, side norm, reweight, degree, pruning, KL clustering), so
//                     these stages fuse into one launch with no inter-node traffic.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gtf.h"
#include "gtf_math.h"

using namespace gtf;

namespace {

// block sizes (diagnostics knobs): 64- or 128-thread blocks for every pass kernel, or
// for the node kernels alone, measured within noise of 256 or slower
#ifndef GTF_PASS_BLOCK
#define GTF_PASS_BLOCK 256
#endif
constexpr int BLOCK = GTF_PASS_BLOCK;
constexpr int MAX_CLUSTER = 15;  // clustering.py:207 (2 < d < 16)

struct Ws {
    uint32_t* err;    // error word (the workspace's first bytes; gtf_diag at GTF_DIAG_OFFSET)
    double* vc;       // [S] per active edge, by SLOT: the merged_cov[1,1] its extrapolation sees
    const gtf_diag* diag;   // optional diagnostics outputs (gtf_set_diagnostics), in the workspace
};

__host__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// workspace header: [0, 256) error word + gtf_diag
constexpr size_t WS_HEAD = 256;

__host__ inline Ws carve(void* base, int32_t n_nodes, int32_t n_slots) {
    (void)n_nodes;
    char* p = (char*)base;
    Ws w;
    w.err = (uint32_t*)p;
    w.diag = (const gtf_diag*)(p + GTF_DIAG_OFFSET);
    w.vc = (double*)(p + WS_HEAD);
    return w;
}

// a reference exception at node v: the workspace error word, and v's entry of the optional
// per-node diagnostics array (gtf_diag.node_err, read from the workspace only on this path)
__device__ __forceinline__ void raise_node(uint32_t* err, int v, uint32_t f) {
    atomicOr(err, f);
    uint32_t* ne = reinterpret_cast<const gtf_diag*>(reinterpret_cast<const char*>(err) + GTF_DIAG_OFFSET)->node_err;
    if (ne) atomicOr(ne + v, f);
}

__device__ __forceinline__ Cov5 load_cov5(const double* c, int64_t i) {
    const double* p = c + 5 * i;
    return Cov5{p[0], p[1], p[2], p[3], p[4]};
}
__device__ __forceinline__ void store_cov5(double* c, int64_t i, const Cov5& v) {
    double* p = c + 5 * i;
    p[0] = v.c00; p[1] = v.c01; p[2] = v.c10; p[3] = v.c11; p[4] = v.c22;
}

// The extrapolation's quotients by a divisor used more than once: qdiv (the correctly
// rounded quotient, the same bits as dividing) or, with GTF_EXTRAP_FAST (A/B builds), the
// product with the reciprocal (within 1.5 ulp). The extrapolation is compared within a
// tolerance (numpy's vectorised cos / sin / exp are not reproducible bit for bit anyway).
#ifndef GTF_EXTRAP_FAST
#define GTF_EXTRAP_FAST 0
#endif
__device__ __forceinline__ double xdiv(double x, double d, double r) {
    if (GTF_EXTRAP_FAST) return x * r;
    return qdiv(x, d, r);
}

// a fresh UTS entry's mixture weight (extrapolate_merged_states.py:384): stored by the
// extrapolation, which loads the sender's TSE weight anyway (1), or set by the node kernel's
// OP_FRESH from its own load of send_mw (0, the round-5 form)
#ifndef GTF_MW_IN_EXTRAP
#define GTF_MW_IN_EXTRAP 0   // 1 measured: node kernel -1 us, k_extrapolate +3.5 us on C4 (profiles/r06/v3/)
#endif

// ---------------------------------------------------------------------------
// var_ms: Highland multiple scattering term (extrapolate_merged_states.py:114-124)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double highland_var_ms(double a, double b, const double* ng, const double* nb,
                                                  double boundary) {
    double dr = nb[3] - ng[3];
    double dz = nb[2] - ng[2];
    double hyp = sqrt(dr * dr + dz * dz);
    double sin_t = fabs(dr) / hyp;
    double q = (2.0 * a * nb[0]) + b;
    const double t15 = 1.0 + q * q;
    double kappa = (2.0 * a) / (t15 * sqrt(t15));  // (1 + q^2)**1.5
    double t = xdiv((13.6 * 1e-3 * sqrt(0.02)) * kappa, 0.3, 1.0 / 0.3);   // (a constant reciprocal)
    double var_ms = sin_t * (t * t);
    if (fabs(ng[2]) >= boundary) {
        double tan_t = fabs(dr) / fabs(dz);
        var_ms = var_ms * tan_t;
    }
    return var_ms;
}

// ---------------------------------------------------------------------------
// k_sender: one 8-lane group per sender node, lanes over its out-edges in
// successor order (chunks of 8). Each lane computes the Highland var_ms of its
// out-edge (extrapolate_merged_states.py:114-124); then every lane forms the
// running "merged_cov[1, 1] += var_ms" its extrapolation sees (:127-128) as the
// sequential sum over the lanes before it (shuffles, the reference's addition
// order), and the last value is the array the stage saves. Inactive out-edges do
// not take part (:431). Out-list reads are contiguous per sender; each active edge's
// running value (8 bytes) goes to the edge's slot, where k_extrapolate reads it
// coalesced instead of gathering it through the sender's out-list (and recomputes the
// edge's own var_ms from operands it loads anyway).
// ---------------------------------------------------------------------------
// the fused sender-major form (gtf_shard.phases bit 4, a shard's halo-dependent senders):
// every scanned edge into the owned slots [lo, hi) is extrapolated by its lane right after
// the scan, with the running value in a register instead of the workspace
#ifndef GTF_EXTRAP_MAP
#define GTF_EXTRAP_MAP 0   // gtf::block_map of k_extrapolate: 0 one slot range per XCD, 1 dispatch order, C > 1 runs of C
#endif
#ifndef GTF_SEND_MAP
#define GTF_SEND_MAP 0     // the same for each bucket of k_sender_sched
#endif
#ifndef GTF_SEND_CHUNKS
#define GTF_SEND_CHUNKS 2   // out-edge chunks per round of loads in the chunked sender scan (> 8 out-edges)
#endif
#ifndef GTF_SEND_KEEP_CARRY
#define GTF_SEND_KEEP_CARRY 1   // 1: a sender's merged_cov[1, 1] stored only when an out-edge changed it
#endif
struct Fuse {
    gtf_states uts;
    int32_t lo, hi;
};
// what the fused sender-major scan already holds of an out-edge when it extrapolates it: the
// sender's state and coordinates, the receiver's coordinates, the activation and var_ms
struct ExKnown {
    int u, v;
    uint8_t act;
    double a, b, c, mc00, mc01, mc10, mc22, vm;
    double ng[4], nb[4];
};
template <bool KNOWN = false>
__device__ __forceinline__ void extrap_slot(const gtf_graph& g, gtf_nodes& n, gtf_states& uts, gtf_edges& e,
                                            const gtf_params& p, const Ws& w, int k, bool have_vc, double vc_given,
                                            const ExKnown* kn = nullptr);

// one sender u over its out-list [ob, oe) with SG lanes (lane gl), chunks of SG
template <int SG, bool FUSED = false>
__device__ __forceinline__ void sender_scan(const gtf_graph& g, gtf_nodes& n, const gtf_edges& e,
                                            const gtf_params& p, const Ws& w, int u, int ob, int oe, int gl,
                                            const Fuse* fu = nullptr) {
    // the sender's flag, state and coordinates in one round of loads
    const uint8_t hm = n.has_merged[u];
    const double a = n.merged_state[3 * (int64_t)u + 0];
    const double b = n.merged_state[3 * (int64_t)u + 1];
    const double ngl[4] = {g.gnn[4 * (int64_t)u], g.gnn[4 * (int64_t)u + 1], g.gnn[4 * (int64_t)u + 2],
                           g.gnn[4 * (int64_t)u + 3]};
    const double* ng = ngl;
    double carry = n.merged_cov[5 * (int64_t)u + 3];
    const double carry0 = carry;
    // (the fused form) the rest of the sender's state, in the same round: the extrapolation
    // reads it from here instead of gathering it again per out-edge
    double c3 = 0.0, m00 = 0.0, m01 = 0.0, m10 = 0.0, m22 = 0.0;
    if constexpr (FUSED) {
        c3 = n.merged_state[3 * (int64_t)u + 2];
        m00 = n.merged_cov[5 * (int64_t)u + 0]; m01 = n.merged_cov[5 * (int64_t)u + 1];
        m10 = n.merged_cov[5 * (int64_t)u + 2]; m22 = n.merged_cov[5 * (int64_t)u + 4];
    }
    if constexpr (FUSED) {
        if (!hm) {   // no state to extrapolate: the owned slots still end their message passing
            for (int i = ob + gl; i < oe; i += SG) {
                const int k = g.out_slot[i];
                if (k >= fu->lo && k < fu->hi) extrap_slot(g, n, *(gtf_states*)&fu->uts, *(gtf_edges*)&e, p, w, k,
                                                            false, 0.0);
            }
            return;
        }
    }
    if (!hm || ob == oe) return;
    // NC chunks of SG out-edges per round of loads: their slot / receiver indices first, then
    // the receivers' coordinates and activations, so a sender with up to NC * SG out-edges
    // waits on two rounds instead of two per chunk (clamped indices past the end: loads of
    // an address the group reads anyway)
    constexpr int NC = FUSED ? 1 : GTF_SEND_CHUNKS;   // (the fused form: one extrapolation body)
    for (int base = ob; base < oe; base += NC * SG) {
        int kk[NC], vv[NC];
#pragma unroll
        for (int j = 0; j < NC; j++) {
            const int i = min(base + j * SG + gl, oe - 1);
            kk[j] = g.out_slot[i];
            vv[j] = g.out_dst ? g.out_dst[i] : -1;
        }
        double nbv[NC][4];
        uint8_t ac[NC];
        int vr[NC];   // the receivers (the fused form's extrapolation)
#pragma unroll
        for (int j = 0; j < NC; j++) {
            const int v = g.out_dst ? vv[j] : g.slot_dst[kk[j]];
            vr[j] = v;
#pragma unroll
            for (int q = 0; q < 4; q++) nbv[j][q] = g.gnn[4 * (int64_t)v + q];
            ac[j] = e.act[kk[j]];
        }
#pragma unroll
        for (int j = 0; j < NC; j++) {
            if (base + j * SG >= oe) break;   // group-uniform
            const int i = base + j * SG + gl;
            const int k = i < oe ? kk[j] : -1;
            double vm = -1.0;
            if (k >= 0 && ac[j] == 1) vm = highland_var_ms(a, b, ng, nbv[j], p.endcap_boundary);
            double c = carry;
            for (int m = 0; m < SG; m++) {
                const double vmm = __shfl(vm, m, SG);
                if (m <= gl && vmm != -1.0) c = c + vmm;
            }
            // the running value of each active edge, stored in out-edge order (contiguous per
            // sender: coalesced stores) when the graph has slot_outidx, else at its slot
            if constexpr (FUSED) {
                if (k >= fu->lo && k < fu->hi) {
                    const ExKnown kn{u, vr[j], ac[j], a, b, c3, m00, m01, m10, m22, vm,
                                     {ng[0], ng[1], ng[2], ng[3]}, {nbv[j][0], nbv[j][1], nbv[j][2], nbv[j][3]}};
                    extrap_slot<true>(g, n, *(gtf_states*)&fu->uts, *(gtf_edges*)&e, p, w, k, true, c, &kn);
                }
            } else {
                if (vm != -1.0) w.vc[g.slot_outidx ? i : k] = c;
            }
            carry = __shfl(c, SG - 1, SG);  // lanes past the end carry the full sum
        }
    }
    // the aliased merged_cov[1, 1] (:127-128) only where an active out-edge added to it
    // (compared as bits: -0.0 + 0.0 is +0.0)
    if (gl == 0 && (!GTF_SEND_KEEP_CARRY || __double_as_longlong(carry) != __double_as_longlong(carry0)))
        n.merged_cov[5 * (int64_t)u + 3] = carry;
}

// one sender u whose out-edges fit the group (<= G), lane gl holding out-edge slot k
// (-1 past the end) with receiver v from gtf_graph.out_lanes: every load of the scan
// is issued in one round, beside the sender's own fields
template <int G, bool FUSED = false>
__device__ __forceinline__ void sender_scan_lane(const gtf_graph& g, gtf_nodes& n, const gtf_edges& e,
                                                 const gtf_params& p, const Ws& w, int u, int ob, int k, int v,
                                                 int gl, const Fuse* fu = nullptr) {
    const uint8_t hm = n.has_merged[u];
    const double a = n.merged_state[3 * (int64_t)u + 0];
    const double b = n.merged_state[3 * (int64_t)u + 1];
    const double ng[4] = {g.gnn[4 * (int64_t)u], g.gnn[4 * (int64_t)u + 1], g.gnn[4 * (int64_t)u + 2],
                          g.gnn[4 * (int64_t)u + 3]};
    const double carry = n.merged_cov[5 * (int64_t)u + 3];
    double c3 = 0.0, m00 = 0.0, m01 = 0.0, m10 = 0.0, m22 = 0.0;   // (the fused form, as in sender_scan)
    if constexpr (FUSED) {
        c3 = n.merged_state[3 * (int64_t)u + 2];
        m00 = n.merged_cov[5 * (int64_t)u + 0]; m01 = n.merged_cov[5 * (int64_t)u + 1];
        m10 = n.merged_cov[5 * (int64_t)u + 2]; m22 = n.merged_cov[5 * (int64_t)u + 4];
    }
    const int kk = k >= 0 ? k : 0;
    const double nb[4] = {g.gnn[4 * (int64_t)v], g.gnn[4 * (int64_t)v + 1], g.gnn[4 * (int64_t)v + 2],
                          g.gnn[4 * (int64_t)v + 3]};
    const uint8_t act = e.act[kk];
    if constexpr (FUSED) {
        if (!hm) {   // no state to extrapolate: the owned slots still end their message passing
            if (k >= fu->lo && k < fu->hi) extrap_slot(g, n, *(gtf_states*)&fu->uts, *(gtf_edges*)&e, p, w, k, false,
                                                        0.0);
            return;
        }
    }
    if (!hm) return;   // group-uniform
    double vm = -1.0;
    if (k >= 0 && act == 1) vm = highland_var_ms(a, b, ng, nb, p.endcap_boundary);
    double c = carry;
    for (int m = 0; m < G; m++) {
        const double vmm = __shfl(vm, m, G);
        if (m <= gl && vmm != -1.0) c = c + vmm;
    }
    if (!FUSED && vm != -1.0) w.vc[g.slot_outidx ? ob + gl : k] = c;
    const double fin = __shfl(c, G - 1, G);   // the last lane has every active edge's term
    if (gl == 0 && (!GTF_SEND_KEEP_CARRY || __double_as_longlong(fin) != __double_as_longlong(carry)))
        n.merged_cov[5 * (int64_t)u + 3] = fin;
    if constexpr (FUSED) {
        if (k >= fu->lo && k < fu->hi) {
            const ExKnown kn{u, v, act, a, b, c3, m00, m01, m10, m22, vm, {ng[0], ng[1], ng[2], ng[3]},
                             {nb[0], nb[1], nb[2], nb[3]}};
            extrap_slot<true>(g, n, *(gtf_states*)&fu->uts, *(gtf_edges*)&e, p, w, k, true, c, &kn);
        }
    }
}

// every node (list NULL) or a list of senders (a shard's), 8 lanes per sender
constexpr int SG = 8;
__global__ void __launch_bounds__(BLOCK) k_sender(gtf_graph g, gtf_nodes n, gtf_edges e, gtf_params p, Ws w,
                                                  const int32_t* list, int count) {
    const int gi = (xcd_local(blockIdx.x, gridDim.x) * BLOCK + (int)threadIdx.x) / SG;
    if (gi >= count) return;  // group-uniform
    const int u = list ? list[gi] : gi;
    sender_scan<SG>(g, n, e, p, w, u, g.out_ptr[u], g.out_ptr[u + 1], threadIdx.x & (SG - 1));
}

// the sender schedule (gtf_graph.out_sched): senders with 1..4 out-edges on 4 lanes,
// 5..8 on 8, more on 16, each entry carrying the sender's out-range (no dependent
// out_ptr gather). One launch; each bucket's blocks form a range padded to a multiple
// of 8, XCD-contiguous inside the range (neighbouring senders' receivers share an L2).
struct SendBuckets {
    const int4* list[3];
    int32_t count[3];
    int32_t blocks[3];  // padded to multiples of 8
    const int2* lanes[2];  // gtf_graph.out_lanes of the 4- and 8-lane buckets, or NULL
};

template <int G, bool FUSED = false>
__device__ __forceinline__ void sender_bucket(const gtf_graph& g, gtf_nodes& n, const gtf_edges& e,
                                              const gtf_params& p, const Ws& w, const int4* list, int count,
                                              int b, int nb, const Fuse* fu = nullptr) {
    const int gi = (gtf::block_map<GTF_SEND_MAP>(b, nb) * BLOCK + (int)threadIdx.x) / G;
    if (gi >= count) return;  // group-uniform
    const int4 en = list[gi];
    sender_scan<G, FUSED>(g, n, e, p, w, en.x, en.y, en.z, threadIdx.x & (G - 1), fu);
}

template <int G, bool FUSED = false>
__device__ __forceinline__ void sender_bucket_lanes(const gtf_graph& g, gtf_nodes& n, const gtf_edges& e,
                                                    const gtf_params& p, const Ws& w, const int4* list,
                                                    const int2* lanes, int count, int b, int nb,
                                                    const Fuse* fu = nullptr) {
    const int t = gtf::block_map<GTF_SEND_MAP>(b, nb) * BLOCK + (int)threadIdx.x;
    const int gi = t / G;
    if (gi >= count) return;  // group-uniform
    const int4 en = list[gi];
    const int2 kv = lanes[t];  // lane t of the bucket = lane (t % G) of entry gi
    sender_scan_lane<G, FUSED>(g, n, e, p, w, en.x, en.y, kv.x, kv.y, t & (G - 1), fu);
}

// All arguments of k_sender_sched in one by-value struct, read through a laundered copy of
// the kernarg-segment address (as the node kernel's NodeKArgs, gtf_node_group.h): each
// bucket path loads only the pointers it uses. Passed as separate structs the scan kept
// ~100 SGPRs live, which admits 6 blocks of 256 threads per CU (SGPR budget 800 /
// (ceil(sgpr / 16) * 16 + 16)) where its 58 VGPRs allow 8.
struct SendKArgs {
    gtf_graph g;
    gtf_nodes n;
    gtf_edges e;
    gtf_params p;
    Ws w;
    SendBuckets sb;
    Fuse fu;   // (the fused form only)
};
typedef const __attribute__((address_space(4))) SendKArgs* SendKArgPtr;
__device__ __forceinline__ SendKArgPtr send_kargs() {
    uint64_t a = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(a));
    return (SendKArgPtr)a;
}

#ifndef GTF_SEND_KARGS
#define GTF_SEND_KARGS 1
#endif
#ifndef GTF_SEND_NUM_SGPR
#define GTF_SEND_NUM_SGPR 72
#endif
template <bool FUSED>
#ifndef GTF_SEND_WAVES
#define GTF_SEND_WAVES 0   // > 0: amdgpu_waves_per_eu lower bound of the (unfused) sender scan
#endif
#if GTF_SEND_WAVES > 0
#define GTF_SEND_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(FUSED ? 1 : GTF_SEND_WAVES)))
#else
#define GTF_SEND_WAVES_ATTR
#endif
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(GTF_SEND_NUM_SGPR))) GTF_SEND_WAVES_ATTR
k_sender_sched(SendKArgs args) {
#if GTF_SEND_KARGS
    (void)args;
    const SendKArgPtr A = send_kargs();
#define GTF_SA(f) (*(decltype(args.f)*)&A->f)
#else
#define GTF_SA(f) (args.f)
#endif
    int b = blockIdx.x;
    const int b0 = GTF_SA(sb).blocks[0];
    if (b < b0) {
        const SendBuckets& sb = GTF_SA(sb);
        if (sb.lanes[0])
            sender_bucket_lanes<4, FUSED>(GTF_SA(g), GTF_SA(n), GTF_SA(e), GTF_SA(p), GTF_SA(w), sb.list[0],
                                          sb.lanes[0], sb.count[0], b, b0, &GTF_SA(fu));
        else sender_bucket<4, FUSED>(GTF_SA(g), GTF_SA(n), GTF_SA(e), GTF_SA(p), GTF_SA(w), sb.list[0], sb.count[0], b,
                                     b0, &GTF_SA(fu));
        return;
    }
    b -= b0;
    const int b1 = GTF_SA(sb).blocks[1];
    if (b < b1) {
        const SendBuckets& sb = GTF_SA(sb);
        if (sb.lanes[1])
            sender_bucket_lanes<8, FUSED>(GTF_SA(g), GTF_SA(n), GTF_SA(e), GTF_SA(p), GTF_SA(w), sb.list[1],
                                          sb.lanes[1], sb.count[1], b, b1, &GTF_SA(fu));
        else sender_bucket<8, FUSED>(GTF_SA(g), GTF_SA(n), GTF_SA(e), GTF_SA(p), GTF_SA(w), sb.list[1], sb.count[1], b,
                                     b1, &GTF_SA(fu));
        return;
    }
    b -= b1;
    const SendBuckets& sb = GTF_SA(sb);
    sender_bucket<16, FUSED>(GTF_SA(g), GTF_SA(n), GTF_SA(e), GTF_SA(p), GTF_SA(w), sb.list[2], sb.count[2], b,
                             sb.blocks[2], &GTF_SA(fu));
#undef GTF_SA
}

// ---------------------------------------------------------------------------
// k_extrapolate: one slot (edge u -> v) per thread
// ---------------------------------------------------------------------------
#ifndef GTF_EXTRAP_PRED
#define GTF_EXTRAP_PRED 1   // 1: k_extrapolate's gathers predicated on an active edge with a sender
#endif
#ifndef GTF_EXTRAP_WAVES
#define GTF_EXTRAP_WAVES 0   // > 0: amdgpu_waves_per_eu lower bound (register budget) of k_extrapolate
#endif
#if GTF_EXTRAP_WAVES > 0
#define GTF_EXTRAP_ATTR __attribute__((amdgpu_waves_per_eu(GTF_EXTRAP_WAVES)))
#else
#define GTF_EXTRAP_ATTR
#endif
// the extrapolation of slot k (edge u -> v), k_extrapolate's per-slot body; have_vc: the
// running merged_cov[1,1] of the edge comes from the caller (the fused sender-major form)
// instead of the workspace
// extrapolate_validate's arithmetic and the slot's stores (extrapolate_merged_states.py:41-402)
// for an active edge of a merged sender, from its loaded operands
template <bool KNOWN>
__device__ __forceinline__ void extrap_math(const gtf_graph& g, gtf_states& uts, gtf_edges& e, const gtf_params& p,
                                            const Ws& w, int k, int v, uint8_t f_old, double smw, double vc,
                                            double node_x, double node_y, double node_z, double node_r, double nbx,
                                            double nby, double nbz, double nbr, double a, double b, double c,
                                            double mc00, double mc01, double mc10, double mc22, double vm_known) {
    (void)g;
    // cos/sin of atan2(y, x) as x/h, y/h (h = |(x, y)|): the same angles as the
    // reference's atan2 -> cos/sin round trips, to a couple of ulps, without fp64 libm
    // (divisors used more than once: one correctly rounded reciprocal, then xdiv() -- the
    // same bits as dividing each time)
    const double rA = sqrt(node_x * node_x + node_y * node_y);
    const double irA = 1.0 / rA;
    const double ca = rA > 0.0 ? xdiv(node_x, rA, irA) : 1.0, sa = rA > 0.0 ? xdiv(node_y, rA, irA) : 0.0;  // :41
    const double x_A = (nbx - node_x) * ca + (nby - node_y) * sa;                              // :52
    const double py = (node_x * nby) - (node_y * nbx), px = (node_x * nbx) + (node_y * nby);  // :59
    const double hp = sqrt(px * px + py * py);
    const double ihp = 1.0 / hp;
    const double sp = hp > 0.0 ? xdiv(py, hp, ihp) : 0.0, cp = hp > 0.0 ? xdiv(px, hp, ihp) : 1.0;
    const double x_prime = x_A + (c * sp);                                        // :63
    const double Vx = cp + (b * sp);
    const double Ax = a * sp;
    const double s_star = (-x_prime * ((2.0 * (Vx * Vx)) + (Ax * x_prime))) / (2.0 * (Vx * Vx * Vx));  // :68

    double numer = x_A + c * sp;                                                  // :82
    double denom = cp + b * sp;
    const double d2 = denom * denom;
    const double id2 = 1.0 / d2;
    const double ds_da = -(sp * (numer * numer)) / (d2 * denom);
    const double ds_db = xdiv((sp * numer) * (1.0 + xdiv(3.0 * a * sp * numer, d2, id2)), d2, id2);
    const double ds_dc = (-sp * (1.0 + xdiv(2.0 * a * sp * numer, d2, id2))) / denom;
    denom = cp + ((2.0 * a + b) * sp);                                             // :89
    const double e2 = denom * denom;
    const double da_da = (1.0 / (e2 * denom)) * (1.0 - ((6.0 * a * sp) * (s_star + a * ds_da) / denom));
    const double e4 = e2 * e2, ie4 = 1.0 / e4;
    const double da_db = xdiv(-3.0 * a * sp * ((2.0 * a * ds_db) + 1.0), e4, ie4);
    const double da_dc = xdiv(-6.0 * sp * ds_dc * (a * a), e4, ie4);
    denom = cp + ((2.0 * a * s_star + b) * sp);                                    // :95
    const double idn = 1.0 / denom;
    double bracket = cp - xdiv(sp * (-sp + ((2.0 * a * s_star + b) * cp)), denom, idn);
    const double db_da = xdiv(2.0 * (s_star + a * ds_da) * bracket, denom, idn);
    const double db_db = xdiv((1.0 + (2.0 * a * ds_da)) * bracket, denom, idn);
    const double db_dc = xdiv(2.0 * a * ds_dc * bracket, denom, idn);
    bracket = (cp * (2.0 * a + b)) - sp;                                           // :102
    const double dc_da = (ds_da * bracket) + ((s_star * s_star) * cp);
    const double dc_db = (ds_db * bracket) + (s_star * cp);
    const double dc_dc = (ds_dc * bracket) + cp;
    const Mat3 F = {{{da_da, da_db, da_dc}, {db_da, db_db, db_dc}, {dc_da, dc_db, dc_dc}}};

    // var_ms again from the operands k_sender used (the same bits): 8 bytes per slot
    // cross the two kernels instead of 16
    double var_ms = vm_known;   // (the fused scan: the value it computed from the same operands)
    if constexpr (!KNOWN) {
        const double ngv[4] = {node_x, node_y, node_z, node_r}, nbv[4] = {nbx, nby, nbz, nbr};
        var_ms = highland_var_ms(a, b, ngv, nbv, p.endcap_boundary);
    }
    const Mat3 C = {{{mc00, mc01, 0.0}, {mc10, vc, 0.0}, {0.0, 0.0, mc22}}};  // :128
    const double m[3] = {a, b, c};
    double xe[3];
    mv3(F, m, xe);                                                                 // :129
    const Mat3 Pe = mm3t(mul_block(F, C), F);                                      // :130
    const double sig2 = p.sigma0xy * p.sigma0xy;
    const double S = Pe.m[2][2] + sig2;                                            // :138
    const double invS = 1.0 / S;
    const double resid = 0.0 - xe[2];
    const double chi2 = (resid * invS) * resid;                                    // :140
    if (w.diag->edge_chi2) w.diag->edge_chi2[k] = chi2;   // diagnostics (gtf_set_diagnostics), off by default
    if (!(chi2 <= p.chi2_cut)) {                                                   // :298
        e.act[k] = 0;                                                              // :393
        if (f_old & 1) uts.fresh[k] = f_old & 2;
        return;
    }
    const double lik = (1.0 / sqrt((2.0 * M_PI) * fabs(S))) * exp(-0.5 * chi2);  // :302-304

    // filterpy 1.4.5 predict() + update(0)  (:307-323): F applied a second time
    double xp[3];
    mv3(F, xe, xp);
    Mat3 Pp = mm3t(mm3(F, Pe), F);
    Pp.m[1][1] = Pp.m[1][1] + var_ms;                                              // + Q
    const double y = 0.0 - xp[2];
    const double S2 = Pp.m[2][2] + sig2;
    const double SI = 1.0 / S2;
    const double K0 = Pp.m[0][2] * SI, K1 = Pp.m[1][2] * SI, K2 = Pp.m[2][2] * SI;
    const double xu0 = xp[0] + K0 * y, xu1 = xp[1] + K1 * y, xu2 = xp[2] + K2 * y;
    const Mat3 IKH = {{{1.0, 0.0, 0.0 - K0}, {0.0, 1.0, 0.0 - K1}, {0.0, 0.0, 1.0 - K2}}};
    // A = (I - K H) Pp, rows 0 and 1 (the only ones the aliased [a, b] block reads); the
    // identity's exact zero / one entries contribute nothing to the reference's sums
    Mat3 A;
    // (numpy gemm: the 1 * P0j and 0 * P1j terms are exact, the last one is fused)
#pragma unroll
    for (int j = 0; j < 3; j++) {
        A.m[0][j] = fma(IKH.m[0][2], Pp.m[2][j], Pp.m[0][j]);
        A.m[1][j] = fma(IKH.m[1][2], Pp.m[2][j], Pp.m[1][j]);
    }
    // P = A IKH^T + (K R) K^T, only the [a,b] block survives the aliasing (:362-365)
    double P00 = fma(A.m[0][2], IKH.m[0][2], A.m[0][0]);
    double P01 = fma(A.m[0][2], IKH.m[1][2], A.m[0][1]);
    double P10 = fma(A.m[1][2], IKH.m[0][2], A.m[1][0]);
    double P11 = fma(A.m[1][2], IKH.m[1][2], A.m[1][1]);
    P00 = P00 + (K0 * sig2) * K0;
    P01 = P01 + (K0 * sig2) * K1;
    P10 = P10 + (K1 * sig2) * K0;
    P11 = P11 + (K1 * sig2) * K1;

    // tau and its variance (:326-358) -- NOT squared here, unlike helper.py:421
    const double dr = nbr - node_r;
    const double dz = nbz - node_z;
    const double J0 = 1.0 / dr;
    const double tau = xdiv(dz, dr, J0);
    double sigma_r = p.sigma0rz, sigma_z = p.sigma0rz2;
    if (fabs(node_z) >= p.endcap_boundary) { sigma_z = p.sigma0rz; sigma_r = p.sigma0rz2; }
    double sigma_rn = p.sigma0rz, sigma_zn = p.sigma0rz2;
    if (fabs(nbz) >= p.endcap_boundary) { sigma_zn = p.sigma0rz; sigma_rn = p.sigma0rz2; }
    // -1 / dr == -(1 / dr) and (-dz) / q == -(dz / q) exactly (round to nearest is symmetric)
    const double J1 = -J0, J3 = dz / (dr * dr), J2 = -J3;
    double vt = (J0 * (sigma_z * sigma_z)) * J0;      // J @ S2 @ J.T (numpy ddot)
    vt = fma(J1 * (sigma_zn * sigma_zn), J1, vt);
    vt = fma(J2 * (sigma_r * sigma_r), J2, vt);
    vt = fma(J3 * (sigma_rn * sigma_rn), J3, vt);

    if (isnan(smw)) raise_node(w.err, v, GTF_ERR_SEND_MW_MISSING);
#if GTF_MW_IN_EXTRAP
    uts.mw[k] = smw;   // mixture_weight = the sender's TSE weight for this receiver (:384)
#endif
#ifndef GTF_DIAG_NOSTORE
#define GTF_DIAG_NOSTORE 0   // diagnostics builds only (wrong results): 1 no covariance store, 2 no state / tau, 3 neither
#endif
    if (!(GTF_DIAG_NOSTORE & 2)) {
        uts.sv[3 * (int64_t)k + 0] = xu0;
        uts.sv[3 * (int64_t)k + 1] = xu1;
        uts.sv[3 * (int64_t)k + 2] = xu2;
        uts.tau[k] = tau;
    } else {
        asm volatile("" ::"v"(xu0), "v"(xu1), "v"(xu2), "v"(tau));
    }
    if (!(GTF_DIAG_NOSTORE & 1)) {
        store_cov5(uts.cov, k, Cov5{P00, P01, P10, P11, vt + var_ms});
    } else {
        const double c22 = vt + var_ms;
        asm volatile("" ::"v"(P00), "v"(P01), "v"(P10), "v"(P11), "v"(c22));
    }
    uts.lik[k] = lik;
    // The empty prior / lr / side of a fresh entry are set by the node kernel's OP_FRESH,
    // merged with its own stores of those fields (its mixture weight is stored here: this
    // kernel loads send_mw anyway, and the node kernel then reads no send_mw of its own). The entry's
    // 'xyzr' (:377) is the sender's GNN coordinates, which stay resident in g.gnn: bit 1
    // marks it live instead of writing a 32-byte copy per accepted edge (gtf_uts_materialize
    // writes it when it is read back or before g.gnn changes)
    uts.fresh[k] = 3;   // the receiver's has_uts flag follows in the node kernel (OP_FRESH)
}

template <bool KNOWN>
__device__ __forceinline__ void extrap_slot(const gtf_graph& g, gtf_nodes& n, gtf_states& uts, gtf_edges& e,
                                            const gtf_params& p, const Ws& w, int k, bool have_vc, double vc_given,
                                            const ExKnown* kn) {
    if constexpr (KNOWN) {
        // (the fused scan) only the slot's own fields are loaded; everything else is the scan's
        const uint8_t is_edge = g.is_edge[k];
        const uint8_t f_old = uts.fresh[k];
        const double smw = e.send_mw[k];
        if (!is_edge || kn->act != 1) {
            if (f_old & 1) uts.fresh[k] = f_old & 2;
            return;
        }
        extrap_math<true>(g, uts, e, p, w, k, kn->v, f_old, smw, vc_given, kn->ng[0], kn->ng[1], kn->ng[2], kn->ng[3],
                          kn->nb[0], kn->nb[1], kn->nb[2], kn->nb[3], kn->a, kn->b, kn->c, kn->mc00, kn->mc01,
                          kn->mc10, kn->mc22, kn->vm);
        return;
    }
    // Two levels of loads instead of a chain: everything indexed by the slot, then
    // everything indexed by its sender / receiver, issued before any early exit (the
    // exits would otherwise serialise each load behind the previous one's branch).
    const uint8_t is_edge = g.is_edge[k], act = e.act[k];
    const uint8_t f_old = uts.fresh[k];   // bit 1 (live coordinates) survives a rejected extrapolation
    const int src = g.slot_src[k], v = g.slot_dst[k];
    // written by k_sender for active edges of merged senders: in out-edge order through
    // slot_outidx (one gather beside the sender's), or by slot
    const int oi = (have_vc || !g.slot_outidx) ? k : g.slot_outidx[k];
    const double smw = e.send_mw[k];
#if GTF_EXTRAP_PRED
    // the sender / receiver gathers only for the slots that can extrapolate (an active edge
    // with a sender): the same second level of loads, without the ~170 bytes per slot the
    // keys without an edge and the deactivated edges would fetch for nothing
    const bool go = is_edge && src >= 0 && act == 1;
    double vc = 0.0, node_x = 0.0, node_y = 0.0, node_z = 0.0, node_r = 0.0, nbx = 0.0, nby = 0.0, nbz = 0.0,
           nbr = 0.0, a = 0.0, b = 0.0, c = 0.0, mc00 = 0.0, mc01 = 0.0, mc10 = 0.0, mc22 = 0.0;
    uint8_t hm = 0;
    if (go) {
        vc = have_vc ? vc_given : w.vc[oi >= 0 ? oi : 0];
        const double* ng = g.gnn + 4 * (int64_t)src;  // sender ("node" in the reference)
        const double* nb = g.gnn + 4 * (int64_t)v;    // receiver ("neighbour")
        hm = n.has_merged[src];
        node_x = ng[0]; node_y = ng[1]; node_z = ng[2]; node_r = ng[3];
        nbx = nb[0]; nby = nb[1]; nbz = nb[2]; nbr = nb[3];
        a = n.merged_state[3 * src + 0]; b = n.merged_state[3 * src + 1]; c = n.merged_state[3 * src + 2];
        const double* mcp = n.merged_cov + 5 * (int64_t)src;
        mc00 = mcp[0]; mc01 = mcp[1]; mc10 = mcp[2]; mc22 = mcp[4];
    }
    if (!go || !hm) {
#else
    const double vc = have_vc ? vc_given : w.vc[oi >= 0 ? oi : 0];
    const int u = src >= 0 ? src : 0;   // orphan keys have no sender
    const double* ng = g.gnn + 4 * (int64_t)u;  // sender ("node" in the reference)
    const double* nb = g.gnn + 4 * (int64_t)v;  // receiver ("neighbour")
    const uint8_t hm = n.has_merged[u];
    const double node_x = ng[0], node_y = ng[1], node_z = ng[2], node_r = ng[3];
    const double nbx = nb[0], nby = nb[1], nbz = nb[2], nbr = nb[3];
    const double a = n.merged_state[3 * u + 0], b = n.merged_state[3 * u + 1], c = n.merged_state[3 * u + 2];
    const double* mcp = n.merged_cov + 5 * (int64_t)u;
    const double mc00 = mcp[0], mc01 = mcp[1], mc10 = mcp[2], mc22 = mcp[4];
    if (!is_edge || src < 0 || !hm || act != 1) {
#endif
        if (f_old & 1) uts.fresh[k] = f_old & 2;
        return;
    }

    extrap_math<false>(g, uts, e, p, w, k, v, f_old, smw, vc, node_x, node_y, node_z, node_r, nbx, nby, nbz, nbr, a, b,
                       c, mc00, mc01, mc10, mc22, 0.0);
}

// slots [slot_lo, slot_hi), or (list) the slot_hi - slot_lo listed slots list[0, ...)
__global__ void __launch_bounds__(BLOCK) GTF_EXTRAP_ATTR k_extrapolate(gtf_graph g, gtf_nodes n, gtf_states uts,
                                                                       gtf_edges e, gtf_params p, Ws w, int slot_lo,
                                                                       int slot_hi, const int32_t* list) {
    const int i = gtf::block_map<GTF_EXTRAP_MAP>(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
    if (slot_lo + i >= slot_hi) return;
    extrap_slot(g, n, uts, e, p, w, list ? list[i] : slot_lo + i, false, 0.0);
}

// gtf_uts_materialize: the stored 'xyzr' snapshot (extrapolate_merged_states.py:377) of every
// entry whose coordinates are live (fresh bit 1)
__global__ void __launch_bounds__(BLOCK) k_uts_materialize(gtf_graph g, gtf_states uts) {
    const int k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= g.n_slots) return;
    const uint8_t f = uts.fresh[k];
    if (!(f & 2)) return;
    const int u = g.slot_src[k];
    if (u >= 0) {
        const double* x = g.gnn + 4 * (int64_t)u;
        double* y = uts.xyzr + 4 * (int64_t)k;
        y[0] = x[0]; y[1] = x[1]; y[2] = x[2]; y[3] = x[3];
    }
    uts.fresh[k] = f & 1;
}

// ---------------------------------------------------------------------------
// node-local stages (1 thread per receiver node)
// ---------------------------------------------------------------------------
#define EXTRAP_OPS OP_FRESH, OP_RANKS, OP_PRIORS_UTS, OP_REWEIGHT_UTS, OP_PRIORS_UTS, OP_REWEIGHT_UTS, OP_DEGREE
#define UPDATE_OPS OP_PRUNE, OP_PRIORS_TSE, OP_PRIORS_UTS, OP_REWEIGHT_UTS
#define CLUSTER_UTS_OPS OP_CLUSTER_UTS, OP_DEGREE, OP_MW_UTS, OP_PRIORS_UTS
#ifndef GTF_SPLIT_NODE
#define GTF_SPLIT_NODE 0  // diagnostics build only: update and clustering in two launches
#endif
#define CLUSTER_TSE_OPS OP_CLUSTER_TSE, OP_DEGREE, OP_MW_TSE, OP_PRIORS_TSE

struct Seg {
    int lo, hi;
};

// iterate the slots of a dict in rank order: calls f(slot) for each present key
template <typename Fn>
__device__ __forceinline__ void for_dict(const int32_t* rank, Seg s, bool monotone, Fn f) {
    if (monotone) {
        for (int k = s.lo; k < s.hi; k++)
            if (rank[k] >= 0) f(k);
        return;
    }
    int prev = -1;
    while (true) {
        int best = -1, br = 0x7fffffff;
        for (int k = s.lo; k < s.hi; k++) {
            const int r = rank[k];
            if (r > prev && r < br) { br = r; best = k; }
        }
        if (best < 0) break;
        f(best);
        prev = br;
    }
}

__device__ __forceinline__ bool ranks_monotone(const int32_t* rank, Seg s) {
    int prev = -1;
    for (int k = s.lo; k < s.hi; k++) {
        const int r = rank[k];
        if (r >= 0) {
            if (r <= prev) return false;
            prev = r;
        }
    }
    return true;
}

__device__ __forceinline__ bool edge_active(const gtf_graph& g, const gtf_edges& e, int k) {
    return g.is_edge[k] && e.act[k] == 1;
}

// the stored sender coordinates of state k: the sender's live GNN ones (gtf_states.fresh
// bit 1, UTS only) or the snapshot
__device__ __forceinline__ const double* state_xyzr(const gtf_graph& g, const gtf_states& st, int k) {
    if (st.fresh && (st.fresh[k] & 2)) return g.gnn + 4 * (int64_t)g.slot_src[k];
    return st.xyzr + 4 * (int64_t)k;
}

// compute_prior_probabilities for one node (helper.py:30-63)
__device__ void node_priors(const gtf_graph& g, const gtf_edges& e, const gtf_states& st, Seg s) {
    for (int k = s.lo; k < s.hi; k++) {
        if (st.rank[k] < 0 || !edge_active(g, e, k)) continue;
        const double lk = g.layer[g.slot_src[k]];
        int cnt = 0;
        for (int j = s.lo; j < s.hi; j++)
            if (st.rank[j] >= 0 && edge_active(g, e, j) && g.layer[g.slot_src[j]] == lk) cnt++;
        st.prior[k] = 1.0 / (double)cnt;
    }
}

// calculate_side_norm_factor + reweight for one node (helper.py:99-200)
__device__ void node_reweight(const gtf_graph& g, gtf_edges& e, gtf_states& st, Seg s, int v, double thr,
                              uint32_t* err) {
    const bool mono = ranks_monotone(st.rank, s);
    // the stale loop variable after the side-norm loop is the LAST dict key (helper.py:131,138)
    int last = -1, lastr = -1;
    for (int k = s.lo; k < s.hi; k++)
        if (st.rank[k] > lastr) { lastr = st.rank[k]; last = k; }
    const double node_x = g.gnn[4 * (int64_t)v];
    int nl = 0, nr = 0, dl = 0, dr = 0;
    for (int k = s.lo; k < s.hi; k++) {
        if (st.rank[k] < 0 || !edge_active(g, e, k)) continue;
        const double xk = state_xyzr(g, st, k)[0];
        const bool left = xk < node_x;
        bool dup = false;  // distinct x values per side: len(set(coords))
        for (int j = s.lo; j < k; j++) {
            if (st.rank[j] < 0 || !edge_active(g, e, j)) continue;
            const double xj = state_xyzr(g, st, j)[0];
            if ((xj < node_x) == left && xj == xk) { dup = true; break; }
        }
        if (left) { nl++; if (!dup) dl++; } else { nr++; if (!dup) dr++; }
    }
    if (nl + nr > 0) {
        if (!g.is_edge[last]) raise_node(err, v, GTF_ERR_STALE_KEY_NO_EDGE);
        const bool last_act = g.is_edge[last] && e.act[last] == 1;
        for (int k = s.lo; k < s.hi; k++) {
            if (st.rank[k] < 0 || !edge_active(g, e, k)) continue;
            const bool left = state_xyzr(g, st, k)[0] < node_x;
            st.side[k] = left ? 0 : 1;
            st.lr[k] = last_act ? (double)(left ? dl : dr) : 1.0;
        }
    }
    double denom = 0.0;  // sequential sum in dict order (:165-169)
    for_dict(st.rank, s, mono, [&](int k) {
        if (edge_active(g, e, k)) denom = denom + (st.mw[k] * st.lik[k]);
    });
    for (int k = s.lo; k < s.hi; k++) {  // :172-200 (order-independent)
        if (st.rank[k] < 0 || !edge_active(g, e, k)) continue;
        double wgt = (st.mw[k] * st.lik[k] * st.prior[k]) / denom;
        wgt = wgt / st.lr[k];
        st.mw[k] = wgt;
        e.edge_mw[k] = wgt;
        e.act[k] = (wgt < thr) ? 0 : 1;
    }
}

__device__ __forceinline__ int node_degree(const gtf_graph& g, const gtf_edges& e, Seg s) {
    int d = 0;
    for (int k = s.lo; k < s.hi; k++) d += edge_active(g, e, k) ? 1 : 0;
    return d;
}

// compute_mixture_weights for one node (helper.py:76-96)
__device__ void node_mixture_weights(const gtf_graph& g, gtf_states& st, Seg s, int v, uint32_t* err) {
    int cnt = 0;
    for (int k = s.lo; k < s.hi; k++) cnt += st.rank[k] >= 0 ? 1 : 0;
    if (cnt == 0) {
        if (!g.solo[v]) raise_node(err, v, GTF_ERR_EMPTY_DICT_MW);
        return;
    }
    const double mw = 1.0 / (double)cnt;
    for (int k = s.lo; k < s.hi; k++)
        if (st.rank[k] >= 0) st.mw[k] = mw;
}

// the fields of the entries message passing (re)wrote (g_fresh, thread-per-node form)
__device__ void node_fresh(gtf_nodes& n, gtf_states& uts, const gtf_edges& e, Seg s, int v) {
    for (int k = s.lo; k < s.hi; k++)
        if (uts.fresh[k] & 1) {
            n.has_uts[v] = 1;
            if (!GTF_MW_IN_EXTRAP) uts.mw[k] = e.send_mw[k];
            uts.prior[k] = NAN;
            uts.lr[k] = NAN;
            uts.side[k] = -1;
        }
}

// new UTS keys created by this message passing are appended after the existing
// ones in sender order (dict insertion, extrapolate_merged_states.py:443-447)
__device__ void node_assign_ranks(gtf_states& uts, Seg s) {
    int next = -1;
    for (int k = s.lo; k < s.hi; k++) next = max(next, uts.rank[k]);
    next += 1;
    for (int k = s.lo; k < s.hi; k++)
        if ((uts.fresh[k] & 1) && uts.rank[k] < 0) uts.rank[k] = next++;
}

// remove_state_metadata pruning (remove_state_metadata.py:31-48)
__device__ void node_prune(const gtf_graph& g, const gtf_nodes& n, gtf_states& tse, gtf_states& uts, Seg s, int v,
                           uint32_t* err) {
    gtf_states& st = n.has_uts[v] ? uts : tse;
    if (!n.has_uts[v] && !n.has_tse[v]) {
        raise_node(err, v, GTF_ERR_NO_STATE_DICT);
        return;
    }
    for (int k = s.lo; k < s.hi; k++)
        if (st.rank[k] >= 0 && !g.rev_edge[k]) st.rank[k] = -1;
}

// clustering of one node (clustering.py:197-307)
__device__ void node_cluster(const gtf_graph& g, gtf_nodes& n, const gtf_states& st, gtf_edges& e, Seg s, int v,
                             double chi2_thr, double kl_thr, const gtf_params& p, uint32_t* err) {
    int d = 0;
    for (int k = s.lo; k < s.hi; k++) d += st.rank[k] >= 0 ? 1 : 0;
    if (d <= 2 || d >= 16) return;                                                 // :207
    int ord[MAX_CLUSTER];
    {
        int i = 0;
        for_dict(st.rank, s, ranks_monotone(st.rank, s), [&](int k) { ord[i++] = k; });
    }
    const double* na = g.xyzr + 4 * (int64_t)v;
    // pairwise chi2 over the lower triangle, np.where semantics on ties (:114-124)
    double best = INFINITY;
    bool any_nonzero = false, has_nan = false;
    int ti0 = -1, tj0 = -1, ti1 = -1;
    uint32_t tiemask = 0;
    for (int i = 1; i < d; i++) {
        const int ki = ord[i];
        const Cov5 ci = load_cov5(st.cov, ki);
        const double ai = st.sv[3 * (int64_t)ki], bi = st.sv[3 * (int64_t)ki + 1];
        for (int j = 0; j < i; j++) {
            const int kj = ord[j];
            const Cov5 cj = load_cov5(st.cov, kj);
            const double D = mahalanobis(ai, bi, ci, st.sv[3 * (int64_t)kj], st.sv[3 * (int64_t)kj + 1], cj, na,
                                         state_xyzr(g, st, ki), state_xyzr(g, st, kj), p.sigma0rz2,
                                         p.sigma0rz, p.sigma0rz, p.sigma0rz2, p.endcap_boundary);
            if (D == 0.0) continue;  // zeros are excluded (np.nonzero)
            any_nonzero = true;
            if (isnan(D)) { has_nan = true; continue; }
            if (D < best) {
                best = D; ti0 = i; tj0 = j; ti1 = -1;
                tiemask = (1u << i) | (1u << j);
            } else if (D == best) {
                if (ti1 < 0) ti1 = i;
                tiemask |= (1u << i) | (1u << j);
            }
        }
    }
    if (!any_nonzero) { raise_node(err, v, GTF_ERR_ALL_ZERO_DIST); return; }
    if (has_nan || !(best < chi2_thr)) return;                                     // :228
    // merge pair = (idx[0], idx[1]) of concatenate((rows, cols))
    const int p0 = ti0, p1 = (ti1 >= 0) ? ti1 : tj0;
    double pm[3], jm[3];
    Cov5 pc, jc;
    {
        const int k0 = ord[p0], k1 = ord[p1];
        const double ps0[3] = {st.sv[3 * (int64_t)k0], st.sv[3 * (int64_t)k0 + 1], st.sv[3 * (int64_t)k0 + 2]};
        const double ps1[3] = {st.sv[3 * (int64_t)k1], st.sv[3 * (int64_t)k1 + 1], st.sv[3 * (int64_t)k1 + 2]};
        const double js0[3] = {ps0[0], ps0[1], st.tau[k0]};
        const double js1[3] = {ps1[0], ps1[1], st.tau[k1]};
        const Cov5 c0 = load_cov5(st.cov, k0), c1 = load_cov5(st.cov, k1);
        merge_states(ps0, c0, ps1, c1, pm, pc);
        merge_states(js0, c0, js1, c1, jm, jc);
    }
    double mprior = st.prior[ord[p0]] + st.prior[ord[p1]];
    uint32_t alive = ((1u << d) - 1u) & ~tiemask;
    if (alive == 0) {
        raise_node(err, v, GTF_ERR_TIE_EMPTIED);
    } else {
        while (true) {                                                             // :251-287
            double mind = 0.0;
            int mi = -1;
            bool nan_seen = false;
            for (int i = 0; i < d; i++) {
                if (!(alive & (1u << i))) continue;
                const int ki = ord[i];
                const double js[3] = {st.sv[3 * (int64_t)ki], st.sv[3 * (int64_t)ki + 1], st.tau[ki]};
                const double D = kl_distance(js, load_cov5(st.cov, ki), jm, jc);
                if (isnan(D)) nan_seen = true;
                if (mi < 0 || D < mind) { mind = D; mi = i; }  // first minimum (list.index)
            }
            if (nan_seen) { raise_node(err, v, GTF_ERR_NAN_KL); break; }
            if (!(mind < kl_thr)) break;
            const int ki = ord[mi];
            const double ps[3] = {st.sv[3 * (int64_t)ki], st.sv[3 * (int64_t)ki + 1], st.sv[3 * (int64_t)ki + 2]};
            const double js[3] = {ps[0], ps[1], st.tau[ki]};
            const Cov5 ci = load_cov5(st.cov, ki);
            double npm[3], njm[3];
            Cov5 npc, njc;
            merge_states(ps, ci, pm, pc, npm, npc);
            merge_states(js, ci, jm, jc, njm, njc);
            pm[0] = npm[0]; pm[1] = npm[1]; pm[2] = npm[2]; pc = npc;
            jm[0] = njm[0]; jm[1] = njm[1]; jm[2] = njm[2]; jc = njc;
            mprior = st.prior[ki] + mprior;
            alive &= ~(1u << mi);
            if (alive == 0) break;
        }
    }
    n.has_merged[v] = 1;                                                           // :291-293
    n.merged_state[3 * (int64_t)v + 0] = pm[0];
    n.merged_state[3 * (int64_t)v + 1] = pm[1];
    n.merged_state[3 * (int64_t)v + 2] = pm[2];
    store_cov5(n.merged_cov, v, pc);
    n.merged_prior[v] = mprior;
    for (int i = 0; i < d; i++)                                                    // :311-321 deactivation
        if (alive & (1u << i)) {
            const int ki = ord[i];
            if (g.is_edge[ki]) e.act[ki] = 0;
        }
    uint8_t* sc = reinterpret_cast<const gtf_diag*>(reinterpret_cast<const char*>(err) + GTF_DIAG_OFFSET)->slot_cluster;
    if (sc)   // diagnostics: merged (1) or left (2)
        for (int i = 0; i < d; i++) sc[ord[i]] = (alive & (1u << i)) ? 2 : 1;
}

// node-local operations, executed in sequence per node by k_node
enum : int8_t {
    OP_RANKS = 1,        // append fresh UTS keys to the dict (extrapolate_merged_states.py:443-447)
    OP_PRIORS_TSE = 2,   // compute_prior_probabilities(.., 'track_state_estimates') helper.py:30-63
    OP_PRIORS_UTS = 3,   // compute_prior_probabilities(.., 'updated_track_states')
    OP_REWEIGHT_UTS = 4, // reweight(.., 'updated_track_states') helper.py:143-225
    OP_DEGREE = 5,       // degree = active in-edges (helper.py:67-73)
    OP_PRUNE = 6,        // remove_state_metadata.py:31-48
    OP_MW_TSE = 7,       // compute_mixture_weights helper.py:76-96
    OP_MW_UTS = 8,
    OP_CLUSTER_TSE = 9,  // clustering.py:197-321 on track_state_estimates
    OP_CLUSTER_UTS = 10, // ... on updated_track_states
    OP_FRESH = 11,       // finish the entries k_extrapolate wrote (weight = sender's, no prior/lr/side)
    OP_FLUSH = 12,       // (internal, compile-time sequences) store the slot fields no later op changes
};

struct NodeOps {
    int8_t op[24];
    int32_t n;
    int32_t uses_tse, uses_uts;
};

__global__ void __launch_bounds__(BLOCK) k_node(gtf_graph g, gtf_nodes n, gtf_states tse, gtf_states uts,
                                                gtf_edges e, gtf_params p, Ws w, NodeOps ops, double chi2_thr,
                                                double kl_thr, const int32_t* list, int count) {
    const int t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= count) return;
    const int v = list ? list[t] : t;
    const Seg s{g.slot_ptr[v], g.slot_ptr[v + 1]};
    for (int i = 0; i < ops.n; i++) {
        switch (ops.op[i]) {
            case OP_FRESH: node_fresh(n, uts, e, s, v); break;
            case OP_RANKS: node_assign_ranks(uts, s); break;
            case OP_PRIORS_TSE: if (n.has_tse[v]) node_priors(g, e, tse, s); break;
            case OP_PRIORS_UTS: if (n.has_uts[v]) node_priors(g, e, uts, s); break;
            case OP_REWEIGHT_UTS:
                if (n.has_uts[v]) node_reweight(g, e, uts, s, v, p.reweight_threshold, w.err);
                break;
            case OP_DEGREE: n.degree[v] = node_degree(g, e, s); break;
            case OP_PRUNE: node_prune(g, n, tse, uts, s, v, w.err); break;
            case OP_MW_TSE: if (n.has_tse[v]) node_mixture_weights(g, tse, s, v, w.err); break;
            case OP_MW_UTS: if (n.has_uts[v]) node_mixture_weights(g, uts, s, v, w.err); break;
            case OP_CLUSTER_TSE:
                if (n.has_tse[v]) {
                    gtf_states t = tse;
                    t.fresh = nullptr;   // TSE coordinates are always the stored ones
                    node_cluster(g, n, t, e, s, v, chi2_thr, kl_thr, p, w.err);
                }
                break;
            case OP_CLUSTER_UTS:
                if (n.has_uts[v]) node_cluster(g, n, uts, e, s, v, chi2_thr, kl_thr, p, w.err);
                break;
            default: break;
        }
    }
}

// node kernels' block size (k_node_multi / k_node_group / k_node_pack)
#ifndef GTF_NODE_BLOCK
#define GTF_NODE_BLOCK 256
#endif
constexpr int NBLOCK = GTF_NODE_BLOCK;
#include "gtf_node_group.h"

thread_local char g_err[512] = "";

int fail(const char* what, hipError_t e) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -1;
}

int check_graph(const gtf_graph* g) {
    if (int rc = check_abi(g, "gtf_pass")) return rc;
    if (g->n_nodes < 0 || g->n_slots < 0 || g->n_edges < 0) {
        snprintf(g_err, sizeof(g_err), "negative sizes"); return -2;
    }
    if (g->n_nodes > 0 && (!g->slot_ptr || !g->out_ptr || !g->gnn)) {
        snprintf(g_err, sizeof(g_err), "missing graph arrays"); return -2;
    }
    if (g->pad_tiles != 0) {   // the padded tile layout must stay inside the arrays
        long long tn = 0, ts = 0;
        bool ok = g->pad_tiles > 0 && g->sched;
        for (int j = 0; j < 6; j++) {
            ok = ok && g->pad_count[j] >= 0;
            tn += g->pad_count[j];
            ts += (long long)g->pad_count[j] * (2 << j);
        }
        ok = ok && tn == g->pad_tile_nodes && ts == g->pad_tile_slots &&
             (long long)g->pad_tiles * tn <= g->n_nodes && (long long)g->pad_tiles * ts <= g->n_slots;
        if (!ok) { snprintf(g_err, sizeof(g_err), "bad padded tile layout"); return -2; }
    }
    return 0;
}

inline int grid(int n) { return (n + BLOCK - 1) / BLOCK; }

// sender scan over `senders` (NULL = every node) and extrapolation of slots [slot_lo,
// slot_hi); events (may be NULL) are recorded before, between and after the two
int launch_extrap_edges(const gtf_graph* g, gtf_nodes* n, gtf_states* uts, gtf_edges* e, const gtf_params* p,
                        Ws w, hipStream_t st, const gtf_shard* sh = nullptr, void* const* events = nullptr) {
    const int32_t* list = sh ? sh->senders : nullptr;
    const int count = sh ? sh->n_senders : g->n_nodes;
    // phases bit 4: the fused sender-major form (the senders' owned out-edges extrapolated
    // by the scan's lanes; needs the sender schedule), no slot-parallel extrapolation
    const bool fused = sh && (sh->phases & 4) && g->out_sched;
    const int32_t* slots = sh ? sh->slot_list : nullptr;   // (a phase-1 call's listed slots)
    const int slot_lo = slots ? 0 : (sh ? sh->slot_lo : 0);
    const int slot_hi = slots ? sh->n_slot_list : (sh ? sh->slot_hi : g->n_slots);
    if (events) (void)hipEventRecord((hipEvent_t)events[0], st);
    if (g->n_slots > 0 && count > 0) {
        if (g->out_sched) {   // (a shard's graph view carries its own senders' schedule)
            SendBuckets sb;
            const int cnt[3] = {g->n_o4, g->n_o8, g->n_o16}, gs[3] = {4, 8, 16};
            const int4* l = reinterpret_cast<const int4*>(g->out_sched);
            int total = 0;
#ifdef GTF_NO_OUT_LANES   // diagnostics build: the scan without the per-lane table
            const int2* ln = nullptr;
#else
            const int2* ln = reinterpret_cast<const int2*>(g->out_lanes);
#endif
            sb.lanes[0] = ln;
            sb.lanes[1] = ln ? ln + 4 * g->n_o4 : nullptr;
            for (int q = 0; q < 3; q++) {
                sb.list[q] = l;
                l += cnt[q];
                sb.count[q] = cnt[q];
                sb.blocks[q] = pad8((cnt[q] + BLOCK / gs[q] - 1) / (BLOCK / gs[q]));
                total += sb.blocks[q];
            }
            if (total > 0 && fused)
                hipLaunchKernelGGL(k_sender_sched<true>, dim3(total), dim3(BLOCK), 0, st,
                                   SendKArgs{*g, *n, *e, *p, w, sb, Fuse{*uts, sh->slot_lo, sh->slot_hi}});
            else if (total > 0)
                hipLaunchKernelGGL(k_sender_sched<false>, dim3(total), dim3(BLOCK), 0, st,
                                   SendKArgs{*g, *n, *e, *p, w, sb, Fuse{}});
        } else {
            hipLaunchKernelGGL(k_sender, dim3((count + BLOCK / SG - 1) / (BLOCK / SG)), dim3(BLOCK), 0, st, *g, *n,
                               *e, *p, w, list, count);
        }
    }
    if (events) (void)hipEventRecord((hipEvent_t)events[1], st);
    if (slot_hi > slot_lo && !fused)
        hipLaunchKernelGGL(k_extrapolate, dim3(grid(slot_hi - slot_lo)), dim3(BLOCK), 0, st, *g, *n, *uts, *e, *p,
                           w, slot_lo, slot_hi, slots);
    if (events) (void)hipEventRecord((hipEvent_t)events[2], st);
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? 0 : fail("extrapolate launch", err);
}


void finish_ops(NodeOps& ops, const gtf_states* tse, const gtf_states* uts) {
    for (int i = 0; i < ops.n; i++) {
        const int o = ops.op[i];
        if (o == OP_PRIORS_TSE || o == OP_MW_TSE || o == OP_CLUSTER_TSE || o == OP_PRUNE) ops.uses_tse = 1;
        if (o == OP_FRESH || o == OP_RANKS || o == OP_PRIORS_UTS || o == OP_REWEIGHT_UTS || o == OP_MW_UTS || o == OP_CLUSTER_UTS ||
            o == OP_PRUNE)
            ops.uses_uts = 1;
    }
    if (!tse) ops.uses_tse = 0;
    if (!uts) ops.uses_uts = 0;
}

// nodes the group kernels do not cover (> 64 slots, or no schedule) run one thread per node
void launch_serial_rest(const gtf_graph* g, gtf_nodes* n, const gtf_states& T, const gtf_states& U, gtf_edges* e,
                        const gtf_params* p, Ws w, const NodeOps& ops, double chi2, double kl, hipStream_t st) {
    if (g->sched) {
        const int ng = g->n_g4 + g->n_g8 + g->n_g16 + g->n_g32 + g->n_g64;
        const int nbig = g->n_big;
        if (nbig > 0)
            hipLaunchKernelGGL(k_node, dim3(grid(nbig)), dim3(BLOCK), 0, st, *g, *n, T, U, *e, *p, w, ops, chi2, kl,
                               g->sched + ng, nbig);
    } else if (g->n_nodes > 0) {
        hipLaunchKernelGGL(k_node, dim3(grid(g->n_nodes)), dim3(BLOCK), 0, st, *g, *n, T, U, *e, *p, w, ops, chi2, kl,
                           (const int32_t*)nullptr, g->n_nodes);
    }
}

// run-time op list (gtf_node_ops)
int launch_ops(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
               const gtf_params* p, Ws w, const int8_t* const* seqs, const int* lens, int nseq, double chi2,
               double kl, hipStream_t st) {
    NodeOps ops;
    memset(&ops, 0, sizeof(ops));
    for (int q = 0; q < nseq; q++)
        for (int i = 0; i < lens[q]; i++) {
            if (ops.n >= (int)sizeof(ops.op)) {
                snprintf(g_err, sizeof(g_err), "too many node ops");
                return -2;
            }
            ops.op[ops.n++] = seqs[q][i];
        }
    finish_ops(ops, tse, uts);
    gtf_states dummy;
    memset(&dummy, 0, sizeof(dummy));
    const gtf_states T = tse ? *tse : dummy, U = uts ? *uts : dummy;
    if (g->n_nodes > 0 && ops.n > 0) {
        if (g->sched) {
            const int32_t* l = g->sched;
            // slot segments of the schedule entries from l on (NULL without sched_seg)
            auto seg = [&](const int32_t* at) { return g->sched_seg ? g->sched_seg + 2 * (at - g->sched) : nullptr; };
            const int n2 = g->n_g2 > 0 && g->n_g2 <= g->n_g4 ? g->n_g2 : 0, n4 = g->n_g4 - n2;
            if (n2 > 0)
                hipLaunchKernelGGL(k_node_group<2>, dim3((n2 + NBLOCK / 2 - 1) / (NBLOCK / 2)), dim3(NBLOCK), 0, st,
                                   *g, *n, T, U, *e, *p, w, ops, chi2, kl, l, seg(l), n2);
            l += n2;
            if (n4 > 0)
                hipLaunchKernelGGL(k_node_group<4>, dim3((n4 + NBLOCK / 4 - 1) / (NBLOCK / 4)), dim3(NBLOCK), 0, st,
                                   *g, *n, T, U, *e, *p, w, ops, chi2, kl, l, seg(l), n4);
            l += n4;
            if (g->n_g8 > 0)
                hipLaunchKernelGGL(k_node_group<8>, dim3((g->n_g8 + NBLOCK / 8 - 1) / (NBLOCK / 8)), dim3(NBLOCK), 0, st,
                                   *g, *n, T, U, *e, *p, w, ops, chi2, kl, l, seg(l), g->n_g8);
            l += g->n_g8;
            if (g->n_g16 > 0)
                hipLaunchKernelGGL(k_node_group<16>, dim3((g->n_g16 + NBLOCK / 16 - 1) / (NBLOCK / 16)), dim3(NBLOCK), 0,
                                   st, *g, *n, T, U, *e, *p, w, ops, chi2, kl, l, seg(l), g->n_g16);
            l += g->n_g16;
            if (g->n_g32 > 0)
                hipLaunchKernelGGL(k_node_group<32>, dim3((g->n_g32 + NBLOCK / 32 - 1) / (NBLOCK / 32)), dim3(NBLOCK), 0,
                                   st, *g, *n, T, U, *e, *p, w, ops, chi2, kl, l, seg(l), g->n_g32);
            l += g->n_g32;
            if (g->n_g64 > 0)
                hipLaunchKernelGGL(k_node_group<64>, dim3((g->n_g64 + NBLOCK / 64 - 1) / (NBLOCK / 64)), dim3(NBLOCK), 0,
                                   st, *g, *n, T, U, *e, *p, w, ops, chi2, kl, l, seg(l), g->n_g64);
        }
        launch_serial_rest(g, n, T, U, e, p, w, ops, chi2, kl, st);
    }
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? 0 : fail("node kernel launch", err);
}

// compile-time op sequence (the stage entry points)
template <int... OPS>
int launch_seq(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e, const gtf_params* p,
               Ws w, double chi2, double kl, hipStream_t st) {
    NodeOps ops;
    memset(&ops, 0, sizeof(ops));
    const int8_t list[] = {(int8_t)OPS...};
    for (int8_t o : list) ops.op[ops.n++] = o;
    finish_ops(ops, tse, uts);
    gtf_states dummy;
    memset(&dummy, 0, sizeof(dummy));
    const gtf_states T = tse ? *tse : dummy, U = uts ? *uts : dummy;
    if (g->n_nodes > 0) {
        if (g->sched) {
            Buckets bk;
            // the first n_g2 entries of the <= 4-slot bucket have <= 2 slots: 2 lanes each
            const int n2 = g->n_g2 > 0 && g->n_g2 <= g->n_g4 ? g->n_g2 : 0;
            const int cnt[6] = {g->n_g64, g->n_g32, g->n_g16, g->n_g8, g->n_g4 - n2, n2};
            const int gs[6] = {64, 32, 16, 8, 4, 2};
            const int32_t* s8 = g->sched + g->n_g4;
            const int32_t* starts[6] = {s8 + g->n_g8 + g->n_g16 + g->n_g32, s8 + g->n_g8 + g->n_g16, s8 + g->n_g8,
                                        s8, g->sched + n2, g->sched};
            int total = 0;
            // padded tile layout: tile offsets of the groups G = 2, 4, 8, 16, 32, 64 (in that order)
            int noff[6] = {0}, soff[6] = {0};
            for (int j = 1; j < 6; j++) {
                noff[j] = noff[j - 1] + g->pad_count[j - 1];
                soff[j] = soff[j - 1] + g->pad_count[j - 1] * (2 << (j - 1));
            }
            for (int q = 0; q < 6; q++) {
                bk.list[q] = starts[q];
                bk.seg[q] = g->sched_seg ? g->sched_seg + 2 * (starts[q] - g->sched) : nullptr;
                bk.count[q] = cnt[q];
                bk.ar[q] = Arith{0, 0, 0, 0, 0};
                if (g->pad_tiles > 0) {   // every node of the group, in tile order, by arithmetic
                    const int j = 5 - q;
                    bk.ar[q] = Arith{g->pad_count[j], noff[j], soff[j], g->pad_tile_nodes, g->pad_tile_slots};
                    bk.count[q] = g->pad_tiles * g->pad_count[j];
                }
                bk.blocks[q] = (bk.count[q] + NBLOCK / gs[q] - 1) / (NBLOCK / gs[q]);
                total += bk.blocks[q];
            }
            if (g->pack_ent && g->pack_wave && g->n_pack_waves > 0)   // every <= 64-slot node, packed
                hipLaunchKernelGGL((k_node_pack<OPS...>), dim3((g->n_pack_waves + NBLOCK / 64 - 1) / (NBLOCK / 64)),
                                   dim3(NBLOCK), 0, st, *g, *n, T, U, *e, *p, w, chi2, kl);
            else if (GTF_SPLIT_G2 && bk.blocks[5] > 0) {   // (A/B) the <= 2-slot bucket in a launch of its own
                const int b5 = bk.blocks[5];
                bk.blocks[5] = 0;
                if (total - b5 > 0)
                    hipLaunchKernelGGL((k_node_multi<OPS...>), dim3(total - b5), dim3(NBLOCK), 0, st,
                                       NodeKArgs{*g, *n, T, U, *e, *p, w, chi2, kl, bk});
                bk.blocks[5] = b5;
                hipLaunchKernelGGL((k_node_g2<OPS...>), dim3(b5), dim3(NBLOCK), 0, st,
                                   NodeKArgs{*g, *n, T, U, *e, *p, w, chi2, kl, bk});
            } else if (total > 0)
                hipLaunchKernelGGL((k_node_multi<OPS...>), dim3(total), dim3(NBLOCK), 0, st,
                                   NodeKArgs{*g, *n, T, U, *e, *p, w, chi2, kl, bk});
        }
        launch_serial_rest(g, n, T, U, e, p, w, ops, chi2, kl, st);
    }
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? 0 : fail("node kernel launch", err);
}


#define SEQ(x) x, (int)sizeof(x)

// the fused pass: message passing, then every node-local op (extrapolation's priors and
// reweights, the update, KL clustering) in ONE node launch: each receiver's ops read and
// write only its own slot segment (plus static coordinates), so there is no inter-node
// dependency between the update and the clustering and one load/store round of the slot
// state serves both. (GTF_SPLIT_NODE=1 builds the earlier two-launch variant for A/B.)
int run_pass(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
             const gtf_params* p, const gtf_shard* sh, void* ws, hipStream_t st, void* const* events) {
    Ws w = carve(ws, g->n_nodes, g->n_slots);
    const int phases = (sh && sh->phases) ? sh->phases : 3;   // (gtf_shard.phases: 1 edges, 2 nodes, 4 fused)
    int rc = 0;
    if (phases & 1) rc = launch_extrap_edges(g, n, uts, e, p, w, st, sh, events);
    if (rc || !(phases & 2)) return rc;
#if GTF_SPLIT_NODE
    rc = launch_seq<EXTRAP_OPS, UPDATE_OPS>(g, n, tse, uts, e, p, w, 0.0, 0.0, st);
    if (rc) return rc;
    if (events) (void)hipEventRecord((hipEvent_t)events[3], st);
    rc = launch_seq<CLUSTER_UTS_OPS>(g, n, tse, uts, e, p, w, p->cluster_chi2, p->cluster_kl, st);
#else
#ifndef GTF_SEQ_VARIANT
#define GTF_SEQ_VARIANT 0  // diagnostics builds: 1..4 = a prefix of the op sequence only
#endif
#if GTF_SEQ_VARIANT == 1
    rc = launch_seq<OP_RANKS, OP_PRIORS_UTS>(g, n, tse, uts, e, p, w, 0.0, 0.0, st);
#elif GTF_SEQ_VARIANT == 2
    rc = launch_seq<OP_RANKS, OP_PRIORS_UTS, OP_REWEIGHT_UTS>(g, n, tse, uts, e, p, w, 0.0, 0.0, st);
#elif GTF_SEQ_VARIANT == 3
    rc = launch_seq<EXTRAP_OPS>(g, n, tse, uts, e, p, w, 0.0, 0.0, st);
#elif GTF_SEQ_VARIANT == 4
    rc = launch_seq<EXTRAP_OPS, UPDATE_OPS>(g, n, tse, uts, e, p, w, 0.0, 0.0, st);
#else
#ifndef GTF_EARLY_STORE
#define GTF_EARLY_STORE 1   // store the update's final slot fields before the clustering (shorter live ranges)
#endif
#if GTF_EARLY_STORE
    rc = launch_seq<EXTRAP_OPS, UPDATE_OPS, OP_FLUSH, CLUSTER_UTS_OPS>(g, n, tse, uts, e, p, w, p->cluster_chi2,
                                                                       p->cluster_kl, st);
    if (false)
#endif
    rc = launch_seq<EXTRAP_OPS, UPDATE_OPS, CLUSTER_UTS_OPS>(g, n, tse, uts, e, p, w, p->cluster_chi2,
                                                             p->cluster_kl, st);
#endif
    if (events) (void)hipEventRecord((hipEvent_t)events[3], st);
#endif
    if (events) (void)hipEventRecord((hipEvent_t)events[4], st);
    return rc;
}

}  // namespace

namespace gtf {
// error text for gtf_last_error from the other translation units (gtf_kl.hip)
void set_error(const char* msg) { snprintf(g_err, sizeof(g_err), "%s", msg); }
}  // namespace gtf

extern "C" {

size_t gtf_workspace_bytes(int32_t n_nodes, int32_t n_slots) {
    (void)n_nodes;
    return WS_HEAD + align256(sizeof(double) * (size_t)(n_slots > 0 ? n_slots : 1));
}

int gtf_workspace_init(void* ws, gtf_stream_t stream) {
    // error word + gtf_diag (no diagnostics)
    hipError_t e = hipMemsetAsync(ws, 0, WS_HEAD, (hipStream_t)stream);
    return e == hipSuccess ? 0 : fail("workspace init", e);
}

int gtf_uts_materialize(const gtf_graph* g, gtf_states* uts, gtf_stream_t stream) {
    int rc = check_graph(g);
    if (rc) return rc;
    if (!uts) { snprintf(g_err, sizeof(g_err), "gtf_uts_materialize: null states"); return -2; }
    if (g->n_slots > 0 && (!uts->fresh || !uts->xyzr || !g->slot_src || !g->gnn)) {
        snprintf(g_err, sizeof(g_err), "gtf_uts_materialize: needs uts->fresh, uts->xyzr, g->slot_src and g->gnn");
        return -2;
    }
    if (g->n_slots > 0)
        hipLaunchKernelGGL(k_uts_materialize, dim3(grid(g->n_slots)), dim3(BLOCK), 0, (hipStream_t)stream, *g, *uts);
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? 0 : fail("materialize launch", err);
}

int gtf_clear_errors(void* ws, gtf_stream_t stream) {
    hipError_t e = hipMemsetAsync(ws, 0, GTF_DIAG_OFFSET, (hipStream_t)stream);   // (keeps gtf_diag)
    return e == hipSuccess ? 0 : fail("clear errors", e);
}

int gtf_set_diagnostics(void* ws, const gtf_diag* d, gtf_stream_t stream) {
    gtf_diag z;
    memset(&z, 0, sizeof(z));
    hipError_t e = hipMemcpyAsync((char*)ws + GTF_DIAG_OFFSET, d ? d : &z, sizeof(gtf_diag), hipMemcpyHostToDevice,
                                  (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);   // (d / z are host stack memory)
    return e == hipSuccess ? 0 : fail("set diagnostics", e);
}

int gtf_read_errors(void* ws, uint32_t* flags, gtf_stream_t stream) {
    hipError_t e = hipMemcpyAsync(flags, ws, sizeof(uint32_t), hipMemcpyDeviceToHost, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? 0 : fail("read errors", e);
}

int gtf_message_passing(const gtf_graph* g, gtf_nodes* n, gtf_states* uts, gtf_edges* e, const gtf_params* p,
                        void* ws, gtf_stream_t stream) {
    int rc = check_graph(g);
    if (rc) return rc;
    Ws w = carve(ws, g->n_nodes, g->n_slots);
    rc = launch_extrap_edges(g, n, uts, e, p, w, (hipStream_t)stream);
    if (rc) return rc;
    return launch_seq<OP_FRESH, OP_RANKS>(g, n, nullptr, uts, e, p, w, 0.0, 0.0, (hipStream_t)stream);
}

int gtf_node_ops(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
                 const gtf_params* p, const int8_t* ops, int32_t n_ops, double chi2_threshold,
                 double kl_threshold, void* ws, gtf_stream_t stream) {
    int rc = check_graph(g);
    if (rc) return rc;
    for (int i = 0; i < n_ops; i++)
        if (ops[i] < OP_RANKS || ops[i] > OP_FRESH) {
            snprintf(g_err, sizeof(g_err), "unknown node op %d", (int)ops[i]);
            return -2;
        }
    Ws w = carve(ws, g->n_nodes, g->n_slots);
    const int8_t* seqs[] = {ops};
    const int lens[] = {n_ops};
    return launch_ops(g, n, tse, uts, e, p, w, seqs, lens, 1, chi2_threshold, kl_threshold, (hipStream_t)stream);
}

int gtf_extrapolate(const gtf_graph* g, gtf_nodes* n, gtf_states* uts, gtf_edges* e, const gtf_params* p,
                    void* ws, gtf_stream_t stream) {
    int rc = check_graph(g);
    if (rc) return rc;
    Ws w = carve(ws, g->n_nodes, g->n_slots);
    rc = launch_extrap_edges(g, n, uts, e, p, w, (hipStream_t)stream);
    if (rc) return rc;
    return launch_seq<EXTRAP_OPS>(g, n, nullptr, uts, e, p, w, 0.0, 0.0, (hipStream_t)stream);
}

int gtf_update(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
               const gtf_params* p, void* ws, gtf_stream_t stream) {
    int rc = check_graph(g);
    if (rc) return rc;
    Ws w = carve(ws, g->n_nodes, g->n_slots);
    return launch_seq<UPDATE_OPS>(g, n, tse, uts, e, p, w, 0.0, 0.0, (hipStream_t)stream);
}

int gtf_cluster(const gtf_graph* g, gtf_nodes* n, gtf_states* states, gtf_edges* e, int32_t key,
                double chi2_threshold, double kl_threshold, const gtf_params* p, void* ws, gtf_stream_t stream) {
    int rc = check_graph(g);
    if (rc) return rc;
    Ws w = carve(ws, g->n_nodes, g->n_slots);
    if (key)
        return launch_seq<CLUSTER_UTS_OPS>(g, n, nullptr, states, e, p, w, chi2_threshold, kl_threshold,
                                           (hipStream_t)stream);
    return launch_seq<CLUSTER_TSE_OPS>(g, n, states, nullptr, e, p, w, chi2_threshold, kl_threshold,
                                       (hipStream_t)stream);
}

int gtf_pass_ev(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
                const gtf_params* p, void* ws, gtf_stream_t stream, void* const* events) {
    int rc = check_graph(g);
    if (rc) return rc;
    return run_pass(g, n, tse, uts, e, p, nullptr, ws, (hipStream_t)stream, events);
}

int gtf_pass_shard(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
                   const gtf_params* p, const gtf_shard* sh, void* ws, gtf_stream_t stream, void* const* events) {
    int rc = check_graph(g);
    if (rc) return rc;
    if (!sh || sh->n_senders < 0 || (sh->n_senders > 0 && !sh->senders) || sh->slot_lo < 0 ||
        sh->slot_hi < sh->slot_lo || sh->slot_hi > g->n_slots || sh->node_lo < 0 || sh->node_hi < sh->node_lo ||
        sh->node_hi > g->n_nodes || sh->phases < 0 || sh->phases > 7 || sh->n_slot_list < 0 ||
        (sh->n_slot_list > 0 && !sh->slot_list)) {
        snprintf(g_err, sizeof(g_err), "gtf_pass_shard: bad shard");
        return -2;
    }
    if (!g->sched) {
        snprintf(g_err, sizeof(g_err), "gtf_pass_shard: needs the owned receivers' schedule in g->sched");
        return -2;
    }
    // bit 4 (fused sender-major phase 1) only with bit 1, the sender schedule and no slot list:
    // phases 4 / 6 would skip the edge phase silently, and the fused form ignores slot_list
    if ((sh->phases & 4) && (!(sh->phases & 1) || !g->out_sched || sh->slot_list || sh->n_slot_list > 0)) {
        snprintf(g_err, sizeof(g_err),
                 "gtf_pass_shard: phases bit 4 needs bit 1, g->out_sched and no slot_list (phases %d)", sh->phases);
        return -2;
    }
    return run_pass(g, n, tse, uts, e, p, sh, ws, (hipStream_t)stream, events);
}

int gtf_pass(const gtf_graph* g, gtf_nodes* n, gtf_states* tse, gtf_states* uts, gtf_edges* e,
             const gtf_params* p, void* ws, gtf_stream_t stream) {
    return gtf_pass_ev(g, n, tse, uts, e, p, ws, stream, nullptr);
}

#if GTF_OP_TIMING
// diagnostics build only: the node kernel's per-wave op timestamps (g_op_time), reset / read
int gtf_op_timing(uint64_t* host, int32_t n_words, int32_t reset) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_op_time)) != hipSuccess) return -1;
    const size_t cap = sizeof(uint64_t) * (size_t)GTF_OP_TIMING_WAVES * 24;
    const size_t nb = n_words < 0 ? 0 : (size_t)n_words * sizeof(uint64_t);
    if (reset) return hipMemset(a, 0, cap) == hipSuccess ? 0 : -1;
    return hipMemcpy(host, a, nb < cap ? nb : cap, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

const char* gtf_last_error(void) { return g_err; }
const char* gtf_version(void) { return "gtf 0.1.0 (gfx950)"; }

}  // extern "C"
