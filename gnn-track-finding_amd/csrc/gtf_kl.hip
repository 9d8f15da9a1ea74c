// gtf_kl.hip -- parabolic-model edge states and pairwise KL distances (SURVEY §8
// a17) for gfx950: the training-data generator of learn_KL_parabolic_model
// (utils.py:221-289 states, extract_metadata_trackml_parabolic_model.py:15-99 pairs).
//
// Nodes by in-degree bucket, all buckets in one launch: one thread per node for d <= 4
// (the states in registers, the pairs written back to back); beyond, one group of G
// lanes per node (8 lanes for d <= 8, a 64-lane wavefront above), one in-edge per
// lane: each lane forms its neighbour's parabolic state in closed form and stages it
// in LDS, and the group deals the node's d(d-1)/2 pairs round-robin over its lanes,
// writing them to the node's contiguous pair range (consecutive lanes, consecutive
// pairs).
//
// Closed form. The reference inverts H = [[x0^2, x0, 1], [0, 0, 1], [xB^2, xB, 1]]
// with np.linalg.inv. H maps parabola coefficients (a, b, c) to the parabola's
// values at x0, 0 and xB, so the columns of H^-1 are the Lagrange basis
// polynomials on {x0, 0, xB}:
//   L0 = (1, -xB, 0) / (x0 (x0 - xB))   L1 = (1, -(x0 + xB), x0 xB) / (x0 xB)
//   L2 = (1, -x0, 0) / (xB (xB - x0))
// so sv = m_B L2, cov = H^-1 S H^-T = sum_k s_k L_k L_k^T and
// cov^-1 = H^T S^-1 H = sum_k h_k h_k^T / s_k (h_k = rows of H) -- no 3x3 inverse at
// all, and no loss of accuracy where H is ill-conditioned. Against the reference's
// committed training CSV this matches to 8e-11 relative (tests/test_kat_parabolic.py).
// sv[2] = 0 and cov[2][2] = s1 for every state, so the KL terms of component 2
// vanish and a state is 7 numbers in LDS: sv0, sv1, c00, c11, i00, i01, i11.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/gtf.h"
#include "gtf_math.h"

namespace gtf {
void set_error(const char* msg);
}

namespace {

// one-wavefront blocks: config 5 fp64 25.9-26.1 us at 256 threads, 25.5-25.6 at 128,
// 25.1-25.4 at 64 (finer-grained dispatch of the mixed buckets), 29.3-29.5 at 512
#ifndef GTF_KL_BLOCK
#define GTF_KL_BLOCK 64
#endif
constexpr int BLOCK = GTF_KL_BLOCK;
#ifndef GTF_KL_NPT
#define GTF_KL_NPT 1
#endif

// node frame: rotation by 2 pi - atan2(y, x) (rotate_track, utils.py:197-218, with
// cos/sin of the angle as x/h, -y/h), then translation to the node (:262-270)
struct Frame {
    double ca, sa, xt, yt, x0, x, y;
};

__device__ __forceinline__ Frame node_frame_xy(double x, double y) {
    Frame f;
    f.x = x;
    f.y = y;
    const double h = sqrt(f.x * f.x + f.y * f.y);
    const double rh = 1.0 / h;   // one reciprocal for both
    f.ca = h > 0.0 ? f.x * rh : 1.0;
    f.sa = h > 0.0 ? -f.y * rh : 0.0;
    f.xt = f.x * f.ca - f.y * f.sa;
    f.yt = f.x * f.sa + f.y * f.ca;
    f.x0 = 0.0 - f.xt;  // the old origin (0, 0) rotates to (0, 0)
    return f;
}

// GNN_Measurement x / y of node v: rows of gnn_stride doubles (4: x, y, z, r; 2: the
// compact x, y copy, half the bytes of the four-field rows)
__device__ __forceinline__ int64_t gnn_row(const gtf_kl_graph& g, int v) {
    return (int64_t)(g.gnn_stride ? g.gnn_stride : 4) * v;
}
__device__ __forceinline__ double gx(const gtf_kl_graph& g, int v) { return g.gnn[gnn_row(g, v)]; }
__device__ __forceinline__ double gy(const gtf_kl_graph& g, int v) { return g.gnn[gnn_row(g, v) + 1]; }

// cache policy of the once-touched streams (GTF_KL_NT bits, diagnostics builds): 1 the
// outputs stored non-temporal, 2 the in-edge sender lists loaded non-temporal, 4 the node's
// own coordinates and truth id too (they are also other nodes' sender gathers)
#ifndef GTF_KL_NT
#define GTF_KL_NT 0
#endif
template <typename T>
__device__ __forceinline__ void st_out(T* p, T v) {
    if (GTF_KL_NT & 1) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <typename T>
__device__ __forceinline__ T ld_list(const T* p) {
    if (GTF_KL_NT & 2) return __builtin_nontemporal_load(p);
    return *p;
}
template <typename T>
__device__ __forceinline__ T ld_own(const T* p) {
    if (GTF_KL_NT & 4) return __builtin_nontemporal_load(p);
    return *p;
}

// where a kernel reads neighbour coordinates and truth ids: global memory, or a block's
// LDS window of consecutive nodes [lo, hi) with global memory beyond it
struct GSrc {   // the fields themselves, not a pointer to the kernel-argument struct
    const double* gnn;
    int64_t stride;
    const int64_t* truth;
    __device__ __forceinline__ explicit GSrc(const gtf_kl_graph& g)
        : gnn(g.gnn), stride(g.gnn_stride ? g.gnn_stride : 4), truth(g.truth) {}
    __device__ __forceinline__ double x(int u) const { return gnn[stride * u]; }
    __device__ __forceinline__ double y(int u) const { return gnn[stride * u + 1]; }
    __device__ __forceinline__ long long t(int u) const { return truth[u]; }
};
struct WSrc {
    const gtf_kl_graph* g;
    const double* sx;
    const double* sy;
    const long long* st;
    int lo, hi;
    __device__ __forceinline__ bool in(int u) const { return u >= lo && u < hi; }
    // the LDS read at a clamped index always, the global one only outside the window: a
    // select of values (a select of an LDS and a global address miscompiles on gfx950)
    __device__ __forceinline__ int at(int u) const { return min(max(u - lo, 0), max(hi - lo - 1, 0)); }
    __device__ __forceinline__ double x(int u) const {
        const double a = sx[at(u)];
        return in(u) ? a : gx(*g, u);
    }
    __device__ __forceinline__ double y(int u) const {
        const double a = sy[at(u)];
        return in(u) ? a : gy(*g, u);
    }
    __device__ __forceinline__ long long t(int u) const {
        const long long a = st[at(u)];
        return in(u) ? a : g->truth[u];
    }
};

template <typename T>
struct PState {
    T s0, s1, c00, c11, i00, i01, i11;
};

// parabolic state of the edge from neighbour (xb, yb) in the node's frame
// (utils.py:273-283); optional full fp64 outputs
// the Lagrange denominator D = x0 xB (x0 - xB) of the state from neighbour (xb, yb), as
// pstate forms it in type T
template <typename T>
__device__ __forceinline__ T pstate_den(const Frame& f, double xb, double yb) {
    const T X0 = (T)f.x0, XB = (T)((xb * f.ca - yb * f.sa) - f.xt);
    return X0 * XB * (X0 - XB);
}

template <typename T>
__device__ __forceinline__ PState<T> pstate(const Frame& f, double xb, double yb, bool& singular, double* sv_out,
                                            double* cov_out, const T* rd_given = nullptr) {
    const double xB = (xb * f.ca - yb * f.sa) - f.xt;
    const double mB = (xb * f.sa + yb * f.ca) - f.yt;
    const double x0 = f.x0;
    singular = (xB == 0.0) || (xB == x0) || (x0 == 0.0);
    const double s0d = 4.0 * 4.0, s1d = 0.1 * 0.1;   // sigma0**2, sigmaA**2 = sigmaB**2 (:223-229)
    if (sv_out || cov_out) {
        const double rD = 1.0 / (x0 * xB * (x0 - xB));
        const double r0 = xB * rD, r1 = (x0 - xB) * rD, r2 = -x0 * rD;
        const double L0[3] = {r0, -xB * r0, 0.0};
        const double L1[3] = {r1, -(x0 + xB) * r1, 1.0};
        const double L2[3] = {r2, -x0 * r2, 0.0};
        if (sv_out) { sv_out[0] = mB * L2[0]; sv_out[1] = mB * L2[1]; sv_out[2] = 0.0; }
        if (cov_out)
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++)
                    cov_out[3 * i + j] = s0d * L0[i] * L0[j] + s1d * L1[i] * L1[j] + s1d * L2[i] * L2[j];
    }
    const T X0 = (T)x0, XB = (T)xB, MB = (T)mB;
    const T s0 = (T)s0d, s1 = (T)s1d;
    // the three Lagrange denominators share one reciprocal: D = x0 xB (x0 - xB)
    const T rD = rd_given ? *rd_given : T(1) / (X0 * XB * (X0 - XB));
    const T r0 = XB * rD, r1 = (X0 - XB) * rD, r2 = -X0 * rD;
    const T a0 = r0, b0 = -XB * r0;
    const T a1 = r1, b1 = -(X0 + XB) * r1;
    const T a2 = r2, b2 = -X0 * r2;
    PState<T> p;
    p.s0 = MB * a2;
    p.s1 = MB * b2;
    p.c00 = s0 * a0 * a0 + s1 * a1 * a1 + s1 * a2 * a2;
    p.c11 = s0 * b0 * b0 + s1 * b1 * b1 + s1 * b2 * b2;
    const T w0 = T(1) / s0, w2 = T(1) / s1;  // h1 = (0, 0, 1) adds nothing to the [a, b] block
    const T X02 = X0 * X0, XB2 = XB * XB;
    p.i00 = w0 * X02 * X02 + w2 * XB2 * XB2;
    p.i01 = w0 * X02 * X0 + w2 * XB2 * XB;
    p.i11 = w0 * X02 + w2 * XB2;
    return p;
}

// KLDistance(mean_i, cov_i, inv_i, mean_j, cov_j, inv_j) (:15-17): the trace of the
// element-wise product is the sum of the diagonal products
template <typename T>
__device__ __forceinline__ T pkl(const PState<T>& a, const PState<T>& b) {
    const T tr = (a.c00 - b.c00) * (b.i00 - a.i00) + (a.c11 - b.c11) * (b.i11 - a.i11);
    const T d0 = a.s0 - b.s0, d1 = a.s1 - b.s1;
    const T S00 = a.i00 + b.i00, S01 = a.i01 + b.i01, S11 = a.i11 + b.i11;
    return tr + (d0 * (d0 * S00 + d1 * S01) + d1 * (d0 * S01 + d1 * S11));
}

template <typename T, int CAP>
struct KlStage {
    T s0[CAP], s1[CAP], c00[CAP], c11[CAP], i00[CAP], i01[CAP], i11[CAP];
    long long tr[CAP];  // neighbour truth ids (pair truth flags without re-gathering)
};

template <typename T, typename St>
__device__ __forceinline__ void put(St* s, int i, const PState<T>& p) {
    s->s0[i] = p.s0; s->s1[i] = p.s1; s->c00[i] = p.c00; s->c11[i] = p.c11;
    s->i00[i] = p.i00; s->i01[i] = p.i01; s->i11[i] = p.i11;
}
template <typename T, typename St>
__device__ __forceinline__ PState<T> get(const St* s, int i) {
    return PState<T>{s->s0[i], s->s1[i], s->c00[i], s->c11[i], s->i00[i], s->i01[i], s->i11[i]};
}

template <int G>
__device__ __forceinline__ double grp_sum(double x) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, G);
    return x;
}

// group sizes of the four degree buckets of gtf_kl_graph.list (d <= 2, <= 4, <= 8, > 8)
constexpr int BG[4] = {1, 4, 8, 64};
constexpr size_t stage_bytes(int G, size_t t) { return (size_t)(BLOCK / G) * G * (7 * t + 8); }

// one node per group of G lanes; states staged in LDS when d <= G (always, except in
// the wavefront bucket beyond 64 in-edges, where pair lanes recompute both states)
// node v on G lanes (lane gl), its states staged at stg
// (i, j) of pair t < 120 (i | j << 8) in LDS, filled by the block of a lane-group bucket
// (pair_table_fill): read instead of solved per pair (a float square root and two
// correction loops, ~40 VALU instructions)
constexpr int PTAB = 120;
__device__ __forceinline__ void pair_table_fill(uint16_t* tab) {
    for (int t = (int)threadIdx.x; t < PTAB; t += BLOCK) {
        int i, j;
        gtf::pair_ij(t, i, j);
        tab[t] = (uint16_t)(i | (j << 8));
    }
    if (BLOCK == 64) gtf::wave_lds_sync();
    else __syncthreads();
}

template <typename T, int G, bool STATES, typename S>
__device__ __forceinline__ void pkl_node_core(const gtf_kl_graph& g, const gtf_kl_out& o, const S& src, int v, int lo,
                                              int d, int64_t base, int gl, KlStage<T, G>* stg,
                                              const uint16_t* ptab = nullptr) {
    if (d < 1) return;
    const Frame f = node_frame_xy(src.x(v), src.y(v));

    // states of the node's in-edges and the gradients dy/dx (utils.py:249-254, 273-283)
    double gsum = 0.0, gr0 = 0.0;
    bool sing = false;
    for (int q = gl; q < d; q += G) {
        const int k = lo + q;
        const int u = g.slot_src[k];
        const double xb = src.x(u), yb = src.y(u);
        bool s;
        const PState<T> p = pstate<T>(f, xb, yb, s, STATES ? o.sv + 3 * (int64_t)k : nullptr,
                                      STATES ? o.cov + 9 * (int64_t)k : nullptr);
        sing |= s;
        if (d <= G) {
            put<T>(stg, q, p);
            if (g.truth) stg->tr[q] = src.t(u);
        }
        const double gr = (f.y - yb) / (f.x - xb);
        if (q == gl) gr0 = gr;
        gsum += gr;
    }
    if (sing && o.err) atomicOr(o.err, (uint32_t)GTF_ERR_SINGULAR_H);
    if (o.emp_var || o.emp_mean) {  // np.mean / np.var over the neighbours (:286)
        const double mean = grp_sum<G>(gsum) / (double)d;
        double vs = 0.0;
        for (int q = gl; q < d; q += G) {
            double gr = gr0;
            if (q != gl) {
                const int u = g.slot_src[lo + q];
                gr = (f.y - src.y(u)) / (f.x - src.x(u));
            }
            vs += (gr - mean) * (gr - mean);
        }
        vs = grp_sum<G>(vs);
        if (gl == 0) {
            if (o.emp_var) st_out(o.emp_var + (v), (double)(vs / (double)d));
            if (o.emp_mean) st_out(o.emp_mean + (v), (double)(mean));
        }
    }
    gtf::wave_lds_sync();

    // pairs i > j, row-major, round-robin over the lanes: consecutive lanes write
    // consecutive distances (calc_pairwise_distances, :19-25)
    const int np = d * (d - 1) / 2;
    const long long tv = g.truth ? src.t(v) : 0;
    T* kl = (T*)o.kl;
    for (int t = gl; t < np; t += G) {
        int i, j;
        if (ptab && np <= PTAB) {   // (np: group-uniform)
            const int e = ptab[t];
            i = e & 0xff;
            j = e >> 8;
        } else {
            gtf::pair_ij(t, i, j);
        }
        PState<T> a, b;
        long long ti = 0, tj = 0;
        if (d <= G) {
            a = get<T>(stg, i);
            b = get<T>(stg, j);
            if (o.truth) { ti = stg->tr[i]; tj = stg->tr[j]; }
        } else {  // beyond the LDS stage (wavefront bucket, d > 64): recompute both states
            bool s;
            const int ui = g.slot_src[lo + i], uj = g.slot_src[lo + j];
            a = pstate<T>(f, src.x(ui), src.y(ui), s, nullptr, nullptr);
            b = pstate<T>(f, src.x(uj), src.y(uj), s, nullptr, nullptr);
            if (o.truth) { ti = src.t(ui); tj = src.t(uj); }
        }
        st_out(kl + (base + t), (T)(pkl<T>(a, b)));
        if (o.truth) st_out(o.truth + (base + t), (int8_t)(tv == ti && ti == tj && tv == tj));  // (:84-95)
    }
}

template <typename T, int G, bool STATES, typename S>
__device__ __forceinline__ void pkl_node_body(const gtf_kl_graph& g, const gtf_kl_out& o, const S& src, int v, int gl,
                                              KlStage<T, G>* stg, const uint16_t* ptab = nullptr) {
    const int lo = g.slot_ptr[v], d = g.slot_ptr[v + 1] - lo;
    if (d < 1) return;
    pkl_node_core<T, G, STATES>(g, o, src, v, lo, d, g.pair_ptr[v], gl, stg, ptab);
}

template <typename T, int G, bool STATES>
__device__ __forceinline__ void pkl_node(const gtf_kl_graph& g, const gtf_kl_out& o, const int32_t* list, int count,
                                         int bid, char* smem, int first = 0, int tid = -1,
                                         const uint16_t* ptab = nullptr) {
    if (tid < 0) tid = (int)threadIdx.x;   // (tid: the thread in a BLOCK-thread (sub)block)
    const int gi = (bid * BLOCK + tid) / G;
    if (gi >= count) return;  // group-uniform
    const int v = list ? list[gi] : first + gi;   // (ordered layout: the bucket is a node range)
    pkl_node_body<T, G, STATES>(g, o, GSrc(g), v, tid & (G - 1), (KlStage<T, G>*)smem + tid / G, ptab);
}

// d <= 2: one thread per node, both states in registers (the bulk of a TrackML
// volume: 88 % of the listed nodes of the vol-7 134 event). A thread may take NPT
// nodes and issue their loads phase by phase (node -> its slots -> the neighbours),
// NPT independent gather chains in flight per lane. Measured on config 5: NPT = 1 48 us, 2 58 us, 4 90 us -- more
// resident waves beat more chains per wave, so the default is 1.
constexpr int NPT = GTF_KL_NPT;

// ordered layout (gtf_kl_graph.first / n_d1 / slot0 / pair0): node, slots and pair of
// bucket-0 entry gi by arithmetic, so the node's own fields and its in-edges' senders are
// one round of independent loads and the senders' coordinates the second. A thread takes
// NPT_ORD entries (gi = (bid * NPT_ORD + j) * BLOCK + lane), their loads issued round by
// round, so NPT_ORD gather chains per lane are in flight at once.
#ifndef GTF_KL_NPT_ORD
#define GTF_KL_NPT_ORD 1
#endif
constexpr int NPT_ORD = GTF_KL_NPT_ORD;
struct B0Node {
    int v, u0, u1;
    bool ok, two;
    int64_t l, pp;
    double xv, yv, x0, y0, x1, y1;
    long long tv, t0, t1;
};

// GTF_KL_RCP (fp64): the node's two Lagrange denominators and two gradient run lengths share
// ONE division -- R = 1 / (Da Db E0 E1), each reciprocal R times the product of the other
// three -- instead of four; within a few ulp of the divisions (the a17 outputs stay within
// the tests' tolerances of the reference's), and the divisions themselves wherever the
// product is zero, subnormal or not finite (a singular state or a zero run, whose infinities
// must stay the reference's)
#ifndef GTF_KL_RCP
#define GTF_KL_RCP 0
#endif
template <typename T, bool STATES>
__device__ __forceinline__ void pkl_b0_finish(const gtf_kl_out& o, const B0Node& n) {
    const Frame f = node_frame_xy(n.xv, n.yv);
    bool s0, s1 = false;
    const double e0 = f.x - n.x0, e1 = n.two ? f.x - n.x1 : 1.0;
    double re0 = 0.0, re1 = 0.0;
    T rda = T(0), rdb = T(0);
    bool shared = false;
    if constexpr (GTF_KL_RCP && sizeof(T) == 8 && !STATES) {
        const double da = pstate_den<double>(f, n.x0, n.y0), db = n.two ? pstate_den<double>(f, n.x1, n.y1) : 1.0;
        const double p1 = da * db, p2 = p1 * e0, P = p2 * e1;
        shared = fabs(P) >= 2.2250738585072014e-308 && fabs(P) <= 1.7976931348623157e308;
        if (shared) {
            const double R = 1.0 / P;
            re1 = R * p2;
            const double t1 = R * e1;
            re0 = t1 * p1;
            const double t2 = t1 * e0;
            rdb = t2 * da;
            rda = t2 * db;
        }
    }
    const PState<T> a = pstate<T>(f, n.x0, n.y0, s0, STATES ? o.sv + 3 * n.l : nullptr, STATES ? o.cov + 9 * n.l : nullptr,
                                  shared ? &rda : nullptr);
    PState<T> b = a;
    if (n.two)
        b = pstate<T>(f, n.x1, n.y1, s1, STATES ? o.sv + 3 * (n.l + 1) : nullptr, STATES ? o.cov + 9 * (n.l + 1) : nullptr,
                      shared ? &rdb : nullptr);
    if ((s0 || s1) && o.err) atomicOr(o.err, (uint32_t)GTF_ERR_SINGULAR_H);
    const double g0 = shared ? (f.y - n.y0) * re0 : (f.y - n.y0) / e0;
    const double g1 = n.two ? (shared ? (f.y - n.y1) * re1 : (f.y - n.y1) / e1) : g0;
    // / 2 and / 1 as exact scalings
    const double mean = n.two ? (g0 + g1) * 0.5 : g0;
    if (o.emp_var)
        st_out(o.emp_var + (n.v), (double)(n.two ? ((g0 - mean) * (g0 - mean) + (g1 - mean) * (g1 - mean)) * 0.5
                                                 : 0.0 * (g0 - mean)));
    if (o.emp_mean) st_out(o.emp_mean + (n.v), (double)(mean));
    if (n.two) {
        st_out((T*)o.kl + (n.pp), (T)(pkl<T>(b, a)));   // pair (i, j) = (1, 0)
        if (o.truth) st_out(o.truth + (n.pp), (int8_t)(n.tv == n.t1 && n.t1 == n.t0 && n.tv == n.t0));
    }
}

template <typename T, bool STATES>
__device__ __forceinline__ void pkl_node1_ordered(const gtf_kl_graph& g, const gtf_kl_out& o, int bid) {
    B0Node n[NPT_ORD];
    const bool tr = o.truth && g.truth;
#pragma unroll
    for (int j = 0; j < NPT_ORD; j++) {   // round 1: own fields and sender lists
        const int gi = (bid * NPT_ORD + j) * BLOCK + (int)threadIdx.x;
        n[j].ok = gi < g.count[0];
        if (!n[j].ok) continue;
        n[j].v = g.first[0] + gi;
        n[j].two = gi >= g.n_d1;
        n[j].l = g.slot0 + (n[j].two ? g.n_d1 + 2 * (int64_t)(gi - g.n_d1) : gi);
        n[j].pp = g.pair0 + (gi - g.n_d1);
        n[j].xv = ld_own(g.gnn + gnn_row(g, n[j].v));
        n[j].yv = ld_own(g.gnn + gnn_row(g, n[j].v) + 1);
        n[j].tv = tr ? ld_own(g.truth + n[j].v) : 0;
        n[j].u0 = ld_list(g.slot_src + n[j].l);
        n[j].u1 = n[j].two ? ld_list(g.slot_src + n[j].l + 1) : n[j].u0;
    }
#pragma unroll
    for (int j = 0; j < NPT_ORD; j++) {   // round 2: the senders' coordinates
        if (!n[j].ok) continue;
#ifdef GTF_KL_DIAG_NODEP   // diagnostics (wrong results): neighbours v -+ 1, no dependent round
        const int w0 = max(n[j].v - 1, 0), w1 = min(n[j].v + 1, g.n_nodes - 1);
#else
        const int w0 = n[j].u0, w1 = n[j].u1;
#endif
        n[j].x0 = gx(g, w0);
        n[j].y0 = gy(g, w0);
        n[j].x1 = gx(g, w1);
        n[j].y1 = gy(g, w1);
        n[j].t0 = tr ? g.truth[w0] : 0;
        n[j].t1 = tr ? g.truth[w1] : 0;
    }
#pragma unroll
    for (int j = 0; j < NPT_ORD; j++)
        if (n[j].ok) {
            pkl_b0_finish<T, STATES>(o, n[j]);
#ifdef GTF_KL_DIAG_NODEP
            asm volatile("" ::"v"(n[j].u0), "v"(n[j].u1));   // (the sender-list loads stay)
#endif
        }
}

// one- or two-edge node v (two: its slots l, l + 1 with senders u0, u1 and pair pp; else
// slot l, sender u0): both states in registers
template <typename T, bool STATES, typename S>
__device__ __forceinline__ void pkl_b0_body(const gtf_kl_graph& g, const gtf_kl_out& o, const S& src, int v, bool two,
                                            int64_t l, int64_t pp, int u0, int u1) {
    const bool tr = o.truth && g.truth;
    B0Node n;
    n.ok = true;
    n.v = v, n.two = two, n.l = l, n.pp = pp, n.u0 = u0, n.u1 = u1;
    n.xv = src.x(v), n.yv = src.y(v);
    n.tv = tr ? src.t(v) : 0;
    n.x0 = src.x(u0), n.y0 = src.y(u0);
    n.x1 = src.x(u1), n.y1 = src.y(u1);
    n.t0 = tr ? src.t(u0) : 0;
    n.t1 = tr ? src.t(u1) : 0;
    pkl_b0_finish<T, STATES>(o, n);
}

template <typename T, bool STATES>
__device__ __forceinline__ void pkl_node1(const gtf_kl_graph& g, const gtf_kl_out& o, const int32_t* list, int count,
                                          int bid) {
    int v[NPT], lo[NPT], d[NPT], u0[NPT], u1[NPT];
    double xv[NPT], yv[NPT], x0[NPT], y0[NPT], x1[NPT], y1[NPT];
    int64_t pp[NPT];
    long long tv[NPT], t0[NPT], t1[NPT];
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        const int gi = (bid * NPT + j) * BLOCK + (int)threadIdx.x;
        v[j] = gi < count ? list[gi] : -1;
    }
#pragma unroll
    for (int j = 0; j < NPT; j++) {
        d[j] = 0;
        if (v[j] >= 0) {
            lo[j] = g.slot_ptr[v[j]];
            d[j] = g.slot_ptr[v[j] + 1] - lo[j];
            xv[j] = gx(g, v[j]);
            yv[j] = gy(g, v[j]);
            pp[j] = g.pair_ptr[v[j]];
            tv[j] = (o.truth && g.truth) ? g.truth[v[j]] : 0;
        }
        if (d[j] < 1 || d[j] > 2) d[j] = 0;
    }
#pragma unroll
    for (int j = 0; j < NPT; j++)
        if (d[j]) {
            u0[j] = g.slot_src[lo[j]];
            u1[j] = d[j] == 2 ? g.slot_src[lo[j] + 1] : u0[j];
        }
#pragma unroll
    for (int j = 0; j < NPT; j++)
        if (d[j]) {
            x0[j] = gx(g, u0[j]);
            y0[j] = gy(g, u0[j]);
            x1[j] = gx(g, u1[j]);
            y1[j] = gy(g, u1[j]);
            if (o.truth && g.truth) {
                t0[j] = g.truth[u0[j]];
                t1[j] = g.truth[u1[j]];
            }
        }
#pragma unroll
    for (int j = 0; j < NPT; j++) {   // (the ordered and tiled layouts' bucket-0 arithmetic, bit for bit)
        if (!d[j]) continue;
        B0Node n;
        n.ok = true;
        n.v = v[j], n.two = d[j] == 2, n.l = lo[j], n.pp = pp[j], n.u0 = u0[j], n.u1 = u1[j];
        n.xv = xv[j], n.yv = yv[j], n.x0 = x0[j], n.y0 = y0[j], n.x1 = x1[j], n.y1 = y1[j];
        n.tv = tv[j];
        n.t0 = (o.truth && g.truth) ? t0[j] : 0;
        n.t1 = (o.truth && g.truth) ? t1[j] : 0;
        pkl_b0_finish<T, STATES>(o, n);
    }
}

// 3 <= d <= 4: one thread per node as well, its <= 4 states in registers and its <= 6
// pairs written back to back (no LDS stage, no group shuffles, every lane busy; the
// gradient moments summed in neighbour order, numpy's order). GTF_KL_B1_LANES=1: the
// 4-lane groups of pkl_node instead.
#ifndef GTF_KL_B1_LANES
#define GTF_KL_B1_LANES 0
#endif
// node v with d in 1..4 in-edges from slot lo (senders u[0..d)) and pairs from base
template <typename T, bool STATES, typename S>
__device__ __forceinline__ void pkl_node4_core(const gtf_kl_graph& g, const gtf_kl_out& o, const S& src, int v, int lo,
                                               int d, int64_t base, const int (&u)[4]) {
    const double xv = src.x(v), yv = src.y(v);
    const long long tv = (o.truth && g.truth) ? src.t(v) : 0;
    double xb[4], yb[4];
    long long tu[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        xb[q] = q < d ? src.x(u[q]) : 0.0;
        yb[q] = q < d ? src.y(u[q]) : 0.0;
        tu[q] = (q < d && o.truth && g.truth) ? src.t(u[q]) : 0;
    }
    const Frame f = node_frame_xy(xv, yv);
    PState<T> st[4];
    double gr[4];
    bool sing = false;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q < d) {
            bool s;
            st[q] = pstate<T>(f, xb[q], yb[q], s, STATES ? o.sv + 3 * (int64_t)(lo + q) : nullptr,
                              STATES ? o.cov + 9 * (int64_t)(lo + q) : nullptr);
            sing |= s;
            gr[q] = (f.y - yb[q]) / (f.x - xb[q]);
        }
    }
    if (sing && o.err) atomicOr(o.err, (uint32_t)GTF_ERR_SINGULAR_H);
    if (o.emp_var || o.emp_mean) {
        double sm = gr[0];
#pragma unroll
        for (int q = 1; q < 4; q++)
            if (q < d) sm = sm + gr[q];
        const double mean = sm / (double)d;
        double vs = (gr[0] - mean) * (gr[0] - mean);
#pragma unroll
        for (int q = 1; q < 4; q++)
            if (q < d) vs = vs + (gr[q] - mean) * (gr[q] - mean);
        if (o.emp_var) st_out(o.emp_var + (v), (double)(vs / (double)d));
        if (o.emp_mean) st_out(o.emp_mean + (v), (double)(mean));
    }
    T* kl = (T*)o.kl;
    int t = 0;
#pragma unroll
    for (int i = 1; i < 4; i++)
#pragma unroll
        for (int j = 0; j < i; j++)
            if (i < d) {
                st_out(kl + (base + t), (T)(pkl<T>(st[i], st[j])));
                if (o.truth) st_out(o.truth + (base + t), (int8_t)(tv == tu[i] && tu[i] == tu[j] && tv == tu[j]));
                t++;
            }
}

template <typename T, bool STATES, typename S>
__device__ __forceinline__ void pkl_node4_body(const gtf_kl_graph& g, const gtf_kl_out& o, const S& src, int v) {
    const int lo = g.slot_ptr[v], d = g.slot_ptr[v + 1] - lo;
    const int64_t base = g.pair_ptr[v];
    if (d < 1 || d > 4) return;
    int u[4];
#pragma unroll
    for (int q = 0; q < 4; q++) u[q] = q < d ? g.slot_src[lo + q] : 0;
    pkl_node4_core<T, STATES>(g, o, src, v, lo, d, base, u);
}

template <typename T, bool STATES>
__device__ __forceinline__ void pkl_node4(const gtf_kl_graph& g, const gtf_kl_out& o, const int32_t* list, int count,
                                          int bid, int first, int tid = -1) {
    if (tid < 0) tid = (int)threadIdx.x;
    const int gi = bid * BLOCK + tid;
    if (gi >= count) return;
    pkl_node4_body<T, STATES>(g, o, GSrc(g), list ? list[gi] : first + gi);
}

struct KlBuckets {
    int32_t blocks[4];
    int32_t ordered;   // gtf_kl_graph's ordered layout (every list NULL)
    int32_t runs;      // ... with degree runs (gtf_kl_graph.deg_runs): buckets 1 / 2 by arithmetic
    int32_t n3;        // bucket 1's three-edge nodes (its first run)
    int32_t r2[4];     // bucket 2's runs of 5..8 in-edges: first entry of each
    int64_t slot1, pair1;        // bucket 1's first slot / pair
    int64_t slot2[4], pair2[4];  // each bucket-2 run's first slot / pair
};

// ordered layout with degree runs: bucket-1 entry gi (three- then four-edge nodes), its
// slots, senders and pairs by arithmetic -- the node's own fields and its sender list are
// one round of independent loads, the senders' coordinates the second
template <typename T, bool STATES>
__device__ __forceinline__ void pkl_node4_runs(const gtf_kl_graph& g, const gtf_kl_out& o, const KlBuckets& bk, int bid) {
    const int gi = bid * BLOCK + (int)threadIdx.x;
    if (gi >= g.count[1]) return;
    const bool three = gi < bk.n3;
    const int d = three ? 3 : 4;
    const int64_t lo = bk.slot1 + (three ? 3 * (int64_t)gi : 3 * (int64_t)bk.n3 + 4 * (int64_t)(gi - bk.n3));
    const int64_t pp = bk.pair1 + (three ? 3 * (int64_t)gi : 3 * (int64_t)bk.n3 + 6 * (int64_t)(gi - bk.n3));
    int u[4];
#pragma unroll
    for (int q = 0; q < 4; q++) u[q] = q < d ? ld_list(g.slot_src + lo + q) : 0;
    pkl_node4_core<T, STATES>(g, o, GSrc(g), g.first[1] + gi, (int)lo, d, pp, u);
}

// ... bucket-1 entry gi on a 4-lane group (GTF_KL_B1_LANES: the LDS-staged form, fewer
// registers than the thread-per-node one)
template <typename T, bool STATES>
__device__ __forceinline__ void pkl_node4l_runs(const gtf_kl_graph& g, const gtf_kl_out& o, const KlBuckets& bk, int bid,
                                                char* smem) {
    const int gi = (bid * BLOCK + (int)threadIdx.x) / 4;
    if (gi >= g.count[1]) return;   // group-uniform
    const bool three = gi < bk.n3;
    const int d = three ? 3 : 4;
    const int64_t lo = bk.slot1 + (three ? 3 * (int64_t)gi : 3 * (int64_t)bk.n3 + 4 * (int64_t)(gi - bk.n3));
    const int64_t pp = bk.pair1 + (three ? 3 * (int64_t)gi : 3 * (int64_t)bk.n3 + 6 * (int64_t)(gi - bk.n3));
    pkl_node_core<T, 4, STATES>(g, o, GSrc(g), g.first[1] + gi, (int)lo, d, pp, (int)threadIdx.x & 3,
                                (KlStage<T, 4>*)smem + (int)threadIdx.x / 4);
}

// ... and bucket-2 group gi (runs of 5, 6, 7, 8 in-edges) on G = 8 lanes
template <typename T, bool STATES>
__device__ __forceinline__ void pkl_node8_runs(const gtf_kl_graph& g, const gtf_kl_out& o, const KlBuckets& bk, int bid,
                                               char* smem, const uint16_t* ptab = nullptr) {
    const int gi = (bid * BLOCK + (int)threadIdx.x) / 8;
    if (gi >= g.count[2]) return;   // group-uniform
    const int k = gi >= bk.r2[3] ? 3 : gi >= bk.r2[2] ? 2 : gi >= bk.r2[1] ? 1 : 0;
    const int d = 5 + k, i = gi - bk.r2[k];
    pkl_node_core<T, 8, STATES>(g, o, GSrc(g), g.first[2] + gi, (int)(bk.slot2[k] + (int64_t)i * d), d,
                                bk.pair2[k] + (int64_t)i * (d * (d - 1) / 2), (int)threadIdx.x & 7,
                                (KlStage<T, 8>*)smem + (int)threadIdx.x / 8, ptab);
}

// one launch over the four buckets; wavefront-bucket blocks first (longest-running)
// 5 waves per SIMD (96 VGPRs, 6 spilled in the fp64 kernel): the compiler's default pick
// takes more registers and fewer waves; at 6 waves (80 VGPRs) the 3-4-edge bucket's
// register-resident states spill 32 (config 5 fp64: 4 waves 26.6 us, 5 waves 25.7 us,
// 6 waves 28.1 us, 8 waves 44.7 us)
#ifndef GTF_KL_WAVES
#define GTF_KL_WAVES 5
#endif
#define KL_ATTR __attribute__((amdgpu_waves_per_eu(GTF_KL_WAVES)))
template <typename T, bool STATES>
__global__ void __launch_bounds__(BLOCK) KL_ATTR k_parabolic_kl(gtf_kl_graph g, gtf_kl_out o, KlBuckets bk) {
    __shared__ __attribute__((aligned(16))) char smem[stage_bytes(4, sizeof(T)) > stage_bytes(64, sizeof(T))
                                                          ? stage_bytes(4, sizeof(T))
                                                          : stage_bytes(64, sizeof(T))];
    // bucket block ranges are multiples of 8, each remapped XCD-contiguous on its own:
    // neighbouring nodes (one event's hits) share an L2. GTF_KL_ORDER: 0 the
    // > 8, 5..8, 3..4-edge buckets' blocks first, then bucket 0; 1 bucket 0 first; 2 the
    // other buckets' blocks spread evenly among bucket 0's; 3 the same in chunks of 8 blocks
    int b = blockIdx.x;
#ifndef GTF_KL_ORDER
#define GTF_KL_ORDER 3
#endif
#ifndef GTF_KL_MIX
#define GTF_KL_MIX 100
#endif
    if (GTF_KL_ORDER == 1 && bk.ordered) {
        if (b < bk.blocks[0]) {
            pkl_node1_ordered<T, STATES>(g, o, gtf::xcd_local(b, bk.blocks[0]));
            return;
        }
        b -= bk.blocks[0];
    } else if (GTF_KL_ORDER == 2 && bk.ordered) {
        const int64_t rest = (int64_t)bk.blocks[3] + bk.blocks[2] + bk.blocks[1];
        const int64_t tot = rest + bk.blocks[0];
        const int upto = (int)(((int64_t)b + 1) * rest / tot);   // other-bucket blocks among [0, b]
        if (upto == (int)((int64_t)b * rest / tot)) {           // b is a bucket-0 block
            pkl_node1_ordered<T, STATES>(g, o, b - upto);
            return;
        }
        b = upto - 1;
    } else if (GTF_KL_ORDER == 3 && bk.ordered) {   // as 2 in chunks of 8 blocks (one per XCD): the
        // XCD-contiguous maps stay intact; the other buckets' chunks spread over the first
        // GTF_KL_MIX % of bucket 0's
        const int64_t rest = ((int64_t)bk.blocks[3] + bk.blocks[2] + bk.blocks[1]) / 8;
        const int64_t tot = rest + (int64_t)bk.blocks[0] / 8 * GTF_KL_MIX / 100;
        const int ch = b / 8, x = b % 8;
        const int upto = ch >= tot ? (int)rest : (int)(((int64_t)ch + 1) * rest / tot);
        if (ch >= tot || upto == (int)((int64_t)ch * rest / tot)) {
            pkl_node1_ordered<T, STATES>(g, o, gtf::xcd_local((ch - upto) * 8 + x, bk.blocks[0]));
            return;
        }
        b = (upto - 1) * 8 + x;
    }
    __shared__ uint16_t s_pair[PTAB];   // (filled by the lane-group buckets' blocks only)
    if (b < bk.blocks[3]) {
        pair_table_fill(s_pair);
        pkl_node<T, 64, STATES>(g, o, g.list[3], g.count[3], gtf::xcd_local(b, bk.blocks[3]), smem, g.first[3], -1,
                                s_pair);
        return;
    }
    b -= bk.blocks[3];
    if (b < bk.blocks[2]) {
        pair_table_fill(s_pair);
        if (bk.runs) pkl_node8_runs<T, STATES>(g, o, bk, gtf::xcd_local(b, bk.blocks[2]), smem, s_pair);
        else pkl_node<T, 8, STATES>(g, o, g.list[2], g.count[2], gtf::xcd_local(b, bk.blocks[2]), smem, g.first[2],
                                    -1, s_pair);
        return;
    }
    b -= bk.blocks[2];
    if (b < bk.blocks[1]) {
        if (GTF_KL_B1_LANES && bk.runs) pkl_node4l_runs<T, STATES>(g, o, bk, gtf::xcd_local(b, bk.blocks[1]), smem);
        else if (GTF_KL_B1_LANES) pkl_node<T, 4, STATES>(g, o, g.list[1], g.count[1], gtf::xcd_local(b, bk.blocks[1]), smem, g.first[1]);
        else if (bk.runs) pkl_node4_runs<T, STATES>(g, o, bk, gtf::xcd_local(b, bk.blocks[1]));
        else pkl_node4<T, STATES>(g, o, g.list[1], g.count[1], gtf::xcd_local(b, bk.blocks[1]), g.first[1]);
        return;
    }
    b -= bk.blocks[1];
    if (GTF_KL_ORDER != 0 && bk.ordered) return;   // (bucket 0 taken above)
    if (bk.ordered) pkl_node1_ordered<T, STATES>(g, o, gtf::xcd_local(b, bk.blocks[0]));
    else pkl_node1<T, STATES>(g, o, g.list[0], g.count[0], gtf::xcd_local(b, bk.blocks[0]));
}

// GTF_KL_SPLIT_B0 (ordered layout): the one-/two-edge bucket in a launch of its own at
// GTF_KL_B0_WAVES waves per SIMD (its path needs far fewer registers than the 3..4-edge
// bucket's register-resident states, which set the one-launch kernel's budget), after the
// launch of the other buckets on the same stream
#ifndef GTF_KL_SPLIT_B0
#define GTF_KL_SPLIT_B0 0
#endif
#ifndef GTF_KL_B0_WAVES
#define GTF_KL_B0_WAVES 8
#endif
template <typename T, bool STATES>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(GTF_KL_B0_WAVES)))
k_parabolic_kl_b0(gtf_kl_graph g, gtf_kl_out o, int nblk) {
    pkl_node1_ordered<T, STATES>(g, o, gtf::xcd_local(blockIdx.x, nblk));
}

// Tiled layout (gtf_kl_graph.blk, gtf.parabolic.ParabolicKL(tile=T)): the nodes
// azimuth-sorted per event and cut into tiles of <= 256 one- / two-edge (bucket-0) nodes
// and the other nodes between them, bucket 0 first inside a tile. One block of WBLOCK
// threads per tile, one bucket-0 node per thread: in ONE round of independent loads it
// reads its thread's sender list and the x, y and truth ids of the tile's window -- the
// tile and up to 128 nodes either side, where a hit's neighbours lie -- into LDS, then
// every node reads its own coordinates and its neighbours' there (global memory outside
// the window). The ordered layout needs two dependent rounds (the sender list, then the
// gathers). Record per tile (12 int32): first node, bucket-0 count, its one-edge count,
// 0, 0, 0, bucket 0's first slot, its first pair (lo, hi), window [lo, hi), 0. The 3..4,
// 5..8 and > 8 buckets run from gtf_kl_graph.list in the same launch, ahead of the tiles,
// each 256-thread block as WBLOCK / BLOCK sub-blocks of the list kernel's.
constexpr int WBLOCK = 256;
#ifndef GTF_KL_WWIN
#define GTF_KL_WWIN 1024
#endif
constexpr int WWIN = GTF_KL_WWIN;          // window nodes (gtf.parabolic.WIN_NODES)
constexpr int WPT = (WWIN + WBLOCK - 1) / WBLOCK;
constexpr int SUBS = WBLOCK / BLOCK;
constexpr size_t sub_stage_bytes(size_t t) {
    return stage_bytes(4, t) > stage_bytes(64, t) ? stage_bytes(4, t) : stage_bytes(64, t);
}
constexpr size_t win_lds_bytes(size_t t) {
    return WWIN * 24 > SUBS * sub_stage_bytes(t) ? WWIN * 24 : SUBS * sub_stage_bytes(t);
}
#ifndef GTF_KL_WIN_WAVES
#define GTF_KL_WIN_WAVES 5
#endif
struct WinBuckets {
    int32_t blocks[4];   // [0] tile blocks (n_blk padded to 8), [1..3] list blocks
};

template <typename T, bool STATES>
__device__ __forceinline__ void pkl_tile(const gtf_kl_graph& g, const gtf_kl_out& o, int tile, char* lds) {
    double* sx = (double*)lds;
    double* sy = sx + WWIN;
    long long* st = (long long*)(sy + WWIN);
    const int32_t* r = g.blk + 12 * (int64_t)tile;
    const int node_lo = r[0], n0 = r[1], n1 = r[2], n3 = r[3], n4 = r[4];
    const int64_t slot_lo = (int64_t)(uint32_t)r[6];
    const int64_t pair_lo = (int64_t)(uint32_t)r[7] | ((int64_t)r[8] << 32);
    const int wlo = r[9], wn = min(r[10], r[9] + WWIN) - r[9];
    const int t = (int)threadIdx.x;
    // one round: the thread's senders, then the window (all independent of each other)
    const bool mine = t < n0, two = t >= n1;
    const int64_t l = slot_lo + (two ? n1 + 2 * (int64_t)(t - n1) : t);
    int u0 = 0, u1 = 0;
    if (mine) {
        u0 = ld_list(g.slot_src + l);
        u1 = two ? ld_list(g.slot_src + l + 1) : u0;
    }
    // threads n0 .. n0 + n3 + n4: the tile's three-, then four-edge nodes (tile_b1), their
    // slots and pairs by arithmetic after bucket 0's
    const int i4 = t - n0;
    const bool mine4 = i4 >= 0 && i4 < n3 + n4;
    const int d4 = i4 < n3 ? 3 : 4;
    const int64_t l4 = slot_lo + n1 + 2 * (int64_t)(n0 - n1) + (i4 < n3 ? 3 * (int64_t)i4 : 3 * (int64_t)n3 + 4 * (int64_t)(i4 - n3));
    const int64_t p4 = pair_lo + (n0 - n1) + (i4 < n3 ? 3 * (int64_t)i4 : 3 * (int64_t)n3 + 6 * (int64_t)(i4 - n3));
    int u4[4] = {0, 0, 0, 0};
    if (mine4) {
#pragma unroll
        for (int q = 0; q < 4; q++) u4[q] = q < d4 ? ld_list(g.slot_src + l4 + q) : 0;
    }
    double wx[WPT], wy[WPT];
    long long wt[WPT];
#pragma unroll
    for (int j = 0; j < WPT; j++) {
        const int i = t + j * WBLOCK;
        if (i < wn) {
            wx[j] = gx(g, wlo + i);
            wy[j] = gy(g, wlo + i);
            wt[j] = g.truth ? g.truth[wlo + i] : 0;
        }
    }
#pragma unroll
    for (int j = 0; j < WPT; j++) {
        const int i = t + j * WBLOCK;
        if (i < wn) {
            sx[i] = wx[j];
            sy[i] = wy[j];
            st[i] = wt[j];
        }
    }
    __syncthreads();
    const WSrc src{&g, sx, sy, st, wlo, wlo + wn};
    if (mine) pkl_b0_body<T, STATES>(g, o, src, node_lo + t, two, l, pair_lo + (t - n1), u0, u1);
    else if (mine4) pkl_node4_core<T, STATES>(g, o, src, node_lo + t, (int)l4, d4, p4, u4);
}

template <typename T, bool STATES>
__global__ void __launch_bounds__(WBLOCK) __attribute__((amdgpu_waves_per_eu(GTF_KL_WIN_WAVES)))
k_parabolic_kl_win(gtf_kl_graph g, gtf_kl_out o, WinBuckets bk) {
    __shared__ __attribute__((aligned(16))) char lds[win_lds_bytes(sizeof(T))];
    int b = blockIdx.x;
    const int sub = (int)threadIdx.x / BLOCK, tid = (int)threadIdx.x % BLOCK;
    char* stage = lds + sub * sub_stage_bytes(sizeof(T));
    if (b < bk.blocks[3]) {   // > 8 in-edges: a wavefront per node (longest-running first)
        pkl_node<T, 64, STATES>(g, o, g.list[3], g.count[3], gtf::xcd_local(b, bk.blocks[3]) * SUBS + sub, stage, 0, tid);
        return;
    }
    b -= bk.blocks[3];
    if (b < bk.blocks[2]) {
        pkl_node<T, 8, STATES>(g, o, g.list[2], g.count[2], gtf::xcd_local(b, bk.blocks[2]) * SUBS + sub, stage, 0, tid);
        return;
    }
    b -= bk.blocks[2];
    if (b < bk.blocks[1]) {
        pkl_node4<T, STATES>(g, o, g.list[1], g.count[1], gtf::xcd_local(b, bk.blocks[1]) * SUBS + sub, 0, tid);
        return;
    }
    b -= bk.blocks[1];
    const int tile = gtf::xcd_local(b, bk.blocks[0]);
    if (tile >= g.n_blk) return;   // (block-uniform: the padding to 8)
    pkl_tile<T, STATES>(g, o, tile, lds);
}

template <typename T>
int launch(const gtf_kl_graph* g, const gtf_kl_out* o, hipStream_t st) {
    if (g->blk) {   // tiled layout: one block per tile record, buckets 1..3 by list
        WinBuckets wb;
        wb.blocks[0] = gtf::pad8(g->n_blk);
        int total = wb.blocks[0];
        for (int i = 1; i < 4; i++) {
            const int per_block = i == 1 ? WBLOCK : WBLOCK / BG[i];   // nodes per 256-thread block
            wb.blocks[i] = gtf::pad8((g->count[i] + per_block - 1) / per_block);
            total += wb.blocks[i];
        }
        if (g->n_blk == 0) total -= wb.blocks[0], wb.blocks[0] = 0;
        if (total > 0) {
            if (o->sv || o->cov)
                hipLaunchKernelGGL((k_parabolic_kl_win<T, true>), dim3(total), dim3(WBLOCK), 0, st, *g, *o, wb);
            else
                hipLaunchKernelGGL((k_parabolic_kl_win<T, false>), dim3(total), dim3(WBLOCK), 0, st, *g, *o, wb);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            gtf::set_error(hipGetErrorString(e));
            return -1;
        }
        return 0;
    }
    KlBuckets bk;
    bk.ordered = !g->list[0] && !g->list[1] && !g->list[2] && !g->list[3];
    bk.runs = bk.ordered && g->deg_runs == 1;
    bk.n3 = g->n_deg[0];
    bk.slot1 = g->slot0 + g->n_d1 + 2 * (int64_t)(g->count[0] - g->n_d1);
    bk.pair1 = g->pair0 + (g->count[0] - g->n_d1);
    bk.r2[0] = 0;
    bk.slot2[0] = bk.slot1 + 3 * (int64_t)g->n_deg[0] + 4 * (int64_t)g->n_deg[1];
    bk.pair2[0] = bk.pair1 + 3 * (int64_t)g->n_deg[0] + 6 * (int64_t)g->n_deg[1];
    for (int k = 1; k < 4; k++) {
        const int dp = 4 + k;   // the previous run's in-degree
        bk.r2[k] = bk.r2[k - 1] + g->n_deg[1 + k];
        bk.slot2[k] = bk.slot2[k - 1] + (int64_t)dp * g->n_deg[1 + k];
        bk.pair2[k] = bk.pair2[k - 1] + (int64_t)(dp * (dp - 1) / 2) * g->n_deg[1 + k];
    }
    int total = 0;
    for (int i = 0; i < 4; i++) {
        int per_block = i == 0 ? (bk.ordered ? BLOCK * NPT_ORD : BLOCK * NPT) : BLOCK / BG[i];   // nodes per block
        if (i == 1 && !GTF_KL_B1_LANES) per_block = BLOCK;
        bk.blocks[i] = gtf::pad8((g->count[i] + per_block - 1) / per_block);
        total += bk.blocks[i];
    }
    int b0_blocks = 0;
    if (GTF_KL_SPLIT_B0 && bk.ordered && bk.blocks[0] > 0) {   // bucket 0 in its own launch, after the others
        b0_blocks = bk.blocks[0];
        total -= b0_blocks;
        bk.blocks[0] = 0;
    }
    if (total > 0) {
        if (o->sv || o->cov)
            hipLaunchKernelGGL((k_parabolic_kl<T, true>), dim3(total), dim3(BLOCK), 0, st, *g, *o, bk);
        else
            hipLaunchKernelGGL((k_parabolic_kl<T, false>), dim3(total), dim3(BLOCK), 0, st, *g, *o, bk);
    }
    if (b0_blocks > 0) {
        if (o->sv || o->cov)
            hipLaunchKernelGGL((k_parabolic_kl_b0<T, true>), dim3(b0_blocks), dim3(BLOCK), 0, st, *g, *o, b0_blocks);
        else
            hipLaunchKernelGGL((k_parabolic_kl_b0<T, false>), dim3(b0_blocks), dim3(BLOCK), 0, st, *g, *o, b0_blocks);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        gtf::set_error(hipGetErrorString(e));
        return -1;
    }
    return 0;
}

}  // namespace

extern "C" int gtf_parabolic_kl(const gtf_kl_graph* g, int32_t dtype, const gtf_kl_out* out, gtf_stream_t stream) {
    if (!g || !out) { gtf::set_error("gtf_parabolic_kl: null argument"); return -2; }
    if (g->n_nodes < 0 || g->n_slots < 0) { gtf::set_error("gtf_parabolic_kl: negative sizes"); return -2; }
    if (g->blk && g->n_blk < 0) { gtf::set_error("gtf_parabolic_kl: bad block table"); return -2; }
    int listed = 0;
    const bool ordered = !g->blk && !g->list[0] && !g->list[1] && !g->list[2] && !g->list[3];
    for (int i = g->blk ? 1 : 0; i < 4; i++) {
        if (g->count[i] < 0 || (g->count[i] > 0 && !g->list[i] && !ordered)) {
            gtf::set_error("gtf_parabolic_kl: bad node list");
            return -2;
        }
        listed += g->count[i];
    }
    if (ordered) {   // every address the ordered layout implies stays inside the arrays
        bool ok = g->n_d1 >= 0 && g->n_d1 <= g->count[0] && g->slot0 >= 0 && g->pair0 >= 0 &&
                  g->slot0 + g->n_d1 + 2 * (int64_t)(g->count[0] - g->n_d1) <= g->n_slots;
        for (int i = 0; i < 4; i++)
            ok = ok && g->first[i] >= 0 && (int64_t)g->first[i] + g->count[i] <= g->n_nodes;
        if (ok && g->deg_runs == 1) {   // the runs add up to buckets 1 and 2 and stay inside the slots / pairs
            int64_t slots = g->slot0 + g->n_d1 + 2 * (int64_t)(g->count[0] - g->n_d1), c1 = 0, c2 = 0;
            for (int k = 0; k < 6; k++) {
                ok = ok && g->n_deg[k] >= 0;
                slots += (int64_t)(3 + k) * g->n_deg[k];
                (k < 2 ? c1 : c2) += g->n_deg[k];
            }
            // (a bucket left out -- count 0 -- launches nothing; the runs still place the next one)
            ok = ok && (c1 == g->count[1] || g->count[1] == 0) && (c2 == g->count[2] || g->count[2] == 0) &&
                 slots <= g->n_slots;
        } else if (g->deg_runs != 0) {
            ok = false;
        }
        if (!ok) { gtf::set_error("gtf_parabolic_kl: bad ordered layout"); return -2; }
    }
    if (g->gnn_stride != 0 && g->gnn_stride != 2 && g->gnn_stride != 4) {
        gtf::set_error("gtf_parabolic_kl: gnn_stride must be 0, 2 or 4");
        return -2;
    }
    if ((listed || (g->blk && g->n_blk > 0)) && (!g->slot_ptr || !g->slot_src || !g->gnn || !g->pair_ptr || !out->kl)) {
        gtf::set_error("gtf_parabolic_kl: missing arrays");
        return -2;
    }
    if ((out->sv == nullptr) != (out->cov == nullptr)) {
        gtf::set_error("gtf_parabolic_kl: sv and cov outputs go together");
        return -2;
    }
    if (out->truth && !g->truth) { gtf::set_error("gtf_parabolic_kl: truth output needs graph truth"); return -2; }
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GTF_F64) return launch<double>(g, out, st);
    if (dtype == GTF_F32) return launch<float>(g, out, st);
    gtf::set_error("gtf_parabolic_kl: dtype must be GTF_F64 or GTF_F32");
    return -2;
}
