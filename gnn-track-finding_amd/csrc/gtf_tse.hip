// gtf_tse.hip -- initial track-state estimates for gfx950:
// helper.compute_track_state_estimates (helper.py:238-452), one state per
// (node, neighbour) key of the node's track_state_estimates dict.
//
// One group of G lanes per node (G from the graph's slot-count schedule, 8..64;
// nodes beyond 64 slots run on a 64-lane group that loops over its slots), one
// slot per lane. Per key the lane forms, in closed form (see gtf_kl.hip for the
// Lagrange-basis inverse of H; here H's first column carries the reference's 1/2):
//   edge_state_vector (a, b, c) = m_B H^-1[:, 2], the Highland var_ms (:398-415),
//   covariance = H^-1 S H^-T with [1,1] += var_ms, aliased with the joint covariance
//   (row/col 2 zeroed, [2,2] = del_tau^2 + var_ms, :417-425), theta, theta2 and
//   variance_theta (:333-346, :427-429).
// The reference fills gradients_zr / del_tau / theta lists in SET order and reads
// them back with the DICT position (the dict order is the reversed set order), so
// the key at dict position i takes those values from the key at dict position
// n - 1 - i (:384, :419-431). The lane computes them for its partner's neighbour
// (the position -> neighbour table is staged in LDS), which is the reference's
// value without a second pass.
// The node's gradient mean/variance (np.mean / np.var over the set-order lists,
// :440-441) is summed by lane 0 in numpy's pairwise order (sequential below 8
// terms, 8 partial sums up to 128).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/gtf.h"
#include "gtf_math.h"

namespace gtf {
void set_error(const char* msg);
}

namespace {

constexpr int BLOCK = 256;

struct NodeGeo {
    double x, y, z, r;  // GNN_Measurement of the node
    double ca, sa;      // cos / sin of the azimuth atan2(y, x) (:352-355) as x/h, y/h
    double x0;          // the origin in the node frame (:369)
    double sz2, sr2;    // node sigma_z^2, sigma_r^2 (endcap swap on |z|, :269-274)
};

// tau, del_tau, theta, theta2, del_theta of the edge node -> neighbour (:283-338)
struct ZrTerms {
    double tau, del_tau, theta, theta2, del_theta, grad_xy;
};

__device__ __forceinline__ ZrTerms zr_terms(const NodeGeo& n, const double* nb, const gtf_params& p) {
    ZrTerms t;
    const double x2 = nb[0], y2 = nb[1], z2 = nb[2], r2 = nb[3];
    t.grad_xy = (y2 - n.y) / (x2 - n.x);
    const double r1 = n.r, z1 = n.z;
    t.tau = (z2 - z1) / (r2 - r1);
    double szn = p.sigma0rz2, srn = p.sigma0rz;
    if (fabs(z2) >= p.endcap_boundary) { szn = p.sigma0rz; srn = p.sigma0rz2; }
    const double dr = r1 - r2, dzz = z1 - z2;
    const double j1 = 1.0 / dr, j2 = -1.0 / dr, j3 = -dzz / (dr * dr), j4 = dzz / (dr * dr);
    // J S2 J^T with S2 = diag(sz^2, szn^2, sr^2, srn^2): the dot products' order
    double v = (j1 * n.sz2) * j1;
    v = v + (j2 * (szn * szn)) * j2;
    v = v + (j3 * n.sr2) * j3;
    v = v + (j4 * (srn * srn)) * j4;
    t.del_tau = v;
    t.theta = atan(1.0 / t.tau);
    t.theta2 = atan2(r2 - r1, z2 - z1);
    const double pre = -1.0 / (1.0 + t.tau * t.tau);
    const double k1 = pre / dr, k2 = -pre / dr, k3 = (-pre * dzz) / (dr * dr), k4 = (pre * dzz) / (dr * dr);
    double w = (k1 * n.sz2) * k1;
    w = w + (k2 * (szn * szn)) * k2;
    w = w + (k3 * n.sr2) * k3;
    w = w + (k4 * (srn * srn)) * k4;
    t.del_theta = w;
    return t;
}

__device__ __forceinline__ NodeGeo node_geo(const double* gnn, int v, const gtf_params& p) {
    NodeGeo n;
    n.x = gnn[4 * (int64_t)v];
    n.y = gnn[4 * (int64_t)v + 1];
    n.z = gnn[4 * (int64_t)v + 2];
    n.r = gnn[4 * (int64_t)v + 3];
    const double h = sqrt(n.x * n.x + n.y * n.y);
    n.ca = h > 0.0 ? n.x / h : 1.0;
    n.sa = h > 0.0 ? n.y / h : 0.0;
    n.x0 = (0.0 - n.x) * n.ca + (0.0 - n.y) * n.sa;
    double sr = p.sigma0rz, sz = p.sigma0rz2;
    if (fabs(n.z) >= p.endcap_boundary) { sz = p.sigma0rz; sr = p.sigma0rz2; }
    n.sz2 = sz * sz;
    n.sr2 = sr * sr;
    return n;
}

// numpy add.reduce over a contiguous float64 array (pairwise_sum): sequential below 8
// terms, otherwise 8 interleaved partial sums combined pairwise, then the tail
template <typename Get>
__device__ __forceinline__ double np_sum(int n, Get a) {
    if (n < 8) {
        double s = 0.0;
        for (int i = 0; i < n; i++) s += a(i);
        return s;
    }
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = a(j);
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += a(i + j);
    double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) s += a(i);
    return s;
}

template <int G>
struct TseStage {
    int u[G];            // neighbour of each dict position
    double gxy[G], gzr[G];
};

template <int G>
__device__ __forceinline__ void tse_node(const gtf_graph& g, gtf_states& tse, const gtf_tse_extra& x,
                                         const gtf_params& p, const int32_t* list, int count, int bid, char* smem) {
    const int gi = (bid * BLOCK + (int)threadIdx.x) / G;
    const int gl = threadIdx.x & (G - 1);
    if (gi >= count) return;  // group-uniform
    const int v = list[gi];
    const int lo = g.slot_ptr[v], d = g.slot_ptr[v + 1] - lo;
    TseStage<G>* stg = (TseStage<G>*)smem + (int)threadIdx.x / G;
    const NodeGeo ng = node_geo(g.gnn, v, p);
    const bool staged = d <= G;
    // number of keys and each key's dict position (ranks need not be dense)
    int n = 0;
    for (int b = 0; b < d; b += G) {
        const int k = lo + b + gl;
        const bool pres = (b + gl < d) && tse.rank[k] >= 0;
        n += __popcll(__ballot(pres) >> (threadIdx.x & 63 & ~(G - 1)) & (G >= 64 ? ~0ull : ((1ull << (G & 63)) - 1)));
    }
    auto dict_pos = [&](int k) {  // keys of v with a smaller rank
        const int rk = tse.rank[k];
        int pos = 0;
        for (int j = lo; j < lo + d; j++) {
            const int rj = tse.rank[j];
            pos += (rj >= 0 && rj < rk) ? 1 : 0;
        }
        return pos;
    };
    if (staged) {
        const int k = lo + gl;
        if (gl < d && tse.rank[k] >= 0) {
            const int pos = dict_pos(k);
            const int u = g.slot_src[k];
            stg->u[pos] = u;
            const ZrTerms t = zr_terms(ng, g.gnn + 4 * (int64_t)u, p);
            stg->gxy[n - 1 - pos] = t.grad_xy;   // set order = reversed dict order
            stg->gzr[n - 1 - pos] = t.tau;
        }
        gtf::wave_lds_sync();
    }
    for (int b = 0; b < d; b += G) {
        const int k = lo + b + gl;
        if (b + gl >= d || tse.rank[k] < 0) continue;
        const int pos = dict_pos(k);
        const int u = g.slot_src[k];
        const double* nb = g.gnn + 4 * (int64_t)u;
        const double xk = nb[0], yk = nb[1], zk = nb[2], rk = nb[3];
        // partner: the key at set position pos = dict position n - 1 - pos
        int up;
        if (staged) {
            up = stg->u[n - 1 - pos];
        } else {
            up = -1;
            for (int j = lo; j < lo + d && up < 0; j++)
                if (tse.rank[j] >= 0 && dict_pos(j) == n - 1 - pos) up = g.slot_src[j];
        }
        const ZrTerms t = zr_terms(ng, g.gnn + 4 * (int64_t)up, p);

        // parabola through (x0, 0), (0, 0), (x_B, m_B) in the node frame (:356-380)
        const double xB = (xk - ng.x) * ng.ca + (yk - ng.y) * ng.sa;
        const double mB = -(xk - ng.x) * ng.sa + (yk - ng.y) * ng.ca;
        const double x0 = ng.x0;
        const double r0 = 1.0 / (x0 * (x0 - xB)), r1 = 1.0 / (x0 * xB), r2 = 1.0 / (xB * (xB - x0));
        // columns of H^-1 (coefficients a = 2 alpha, b, c of the Lagrange basis)
        const double A0 = 2.0 * r0, B0 = -xB * r0;
        const double A1 = 2.0 * r1, B1 = -(x0 + xB) * r1;
        const double A2 = 2.0 * r2, B2 = -x0 * r2;
        const double a = mB * A2, bb = mB * B2;
        const double s0 = 4.0 * 4.0, s1 = p.sigma0xy * p.sigma0xy;
        double c00 = s0 * A0 * A0 + s1 * A1 * A1 + s1 * A2 * A2;
        double c01 = s0 * A0 * B0 + s1 * A1 * B1 + s1 * A2 * B2;
        double c11 = s0 * B0 * B0 + s1 * B1 * B1 + s1 * B2 * B2;
        // Highland multiple scattering with the neighbour's global x (:398-415)
        const double dr = ng.r - rk, dz = ng.z - zk;
        const double hyp = sqrt(dr * dr + dz * dz);
        const double sin_t = fabs(dr) / hyp;
        const double q = (2.0 * a * xk) + bb;
        const double t15 = 1.0 + q * q;
        const double kappa = (2.0 * a) / (t15 * sqrt(t15));
        const double hl = ((13.6 * 1e-3 * sqrt(0.02)) * kappa) / 0.3;
        double var_ms = sin_t * (hl * hl);
        if (fabs(ng.z) >= p.endcap_boundary) var_ms = var_ms * fabs(dr / dz);
        c11 = c11 + var_ms;
        tse.sv[3 * (int64_t)k] = a;
        tse.sv[3 * (int64_t)k + 1] = bb;
        tse.sv[3 * (int64_t)k + 2] = 0.0;  // c = m_A = 0
        tse.tau[k] = t.tau;
        double* cv = tse.cov + 5 * (int64_t)k;
        cv[0] = c00; cv[1] = c01; cv[2] = c01; cv[3] = c11;
        cv[4] = t.del_tau * t.del_tau + var_ms;
        double* sx = tse.xyzr + 4 * (int64_t)k;
        sx[0] = xk; sx[1] = yk; sx[2] = zk; sx[3] = rk;
        if (x.theta) {
            double* th = x.theta + 3 * (int64_t)k;
            th[0] = t.theta; th[1] = t.theta2; th[2] = t.del_theta * t.del_theta + var_ms;
        }
        if (x.var_ms) x.var_ms[k] = var_ms;
    }
    if (gl == 0) {
        if (x.xy_mean_var || x.zr_mean_var) {
            double gx[2], gz[2];
            for (int w = 0; w < 2; w++) {
                // w = 0: the gradients; w = 1: squared deviations from their mean
                auto getx = [&](int i) -> double {
                    double val;
                    if (staged) val = stg->gxy[i];
                    else {
                        int uu = -1;
                        for (int j = lo; j < lo + d && uu < 0; j++)
                            if (tse.rank[j] >= 0 && dict_pos(j) == n - 1 - i) uu = g.slot_src[j];
                        val = zr_terms(ng, g.gnn + 4 * (int64_t)uu, p).grad_xy;
                    }
                    return w == 0 ? val : (val - gx[0]) * (val - gx[0]);
                };
                auto getz = [&](int i) -> double {
                    double val;
                    if (staged) val = stg->gzr[i];
                    else {
                        int uu = -1;
                        for (int j = lo; j < lo + d && uu < 0; j++)
                            if (tse.rank[j] >= 0 && dict_pos(j) == n - 1 - i) uu = g.slot_src[j];
                        val = zr_terms(ng, g.gnn + 4 * (int64_t)uu, p).tau;
                    }
                    return w == 0 ? val : (val - gz[0]) * (val - gz[0]);
                };
                gx[w] = np_sum(n, getx) / (double)n;   // n = 0 -> NaN, like np.mean([])
                gz[w] = np_sum(n, getz) / (double)n;
            }
            if (x.xy_mean_var) { x.xy_mean_var[2 * (int64_t)v] = gx[0]; x.xy_mean_var[2 * (int64_t)v + 1] = gx[1]; }
            if (x.zr_mean_var) { x.zr_mean_var[2 * (int64_t)v] = gz[0]; x.zr_mean_var[2 * (int64_t)v + 1] = gz[1]; }
        }
        if (x.angle) x.angle[v] = atan2(ng.y, ng.x);
        if (x.translation) { x.translation[2 * (int64_t)v] = ng.x; x.translation[2 * (int64_t)v + 1] = ng.y; }
    }
}

struct TseBuckets {
    const int32_t* list[5];
    int32_t count[5];
    int32_t blocks[5];
};

constexpr size_t tse_smem() {
    return (size_t)(BLOCK / 8) * sizeof(TseStage<8>) > (size_t)(BLOCK / 64) * sizeof(TseStage<64>)
               ? (size_t)(BLOCK / 8) * sizeof(TseStage<8>)
               : (size_t)(BLOCK / 64) * sizeof(TseStage<64>);
}

// one launch over the slot-count buckets, long-running ones first
__global__ void __launch_bounds__(BLOCK) k_tse(gtf_graph g, gtf_states tse, gtf_tse_extra x, gtf_params p,
                                               TseBuckets bk) {
    __shared__ __attribute__((aligned(16))) char smem[tse_smem() > (size_t)(BLOCK / 16) * sizeof(TseStage<16>)
                                                          ? tse_smem()
                                                          : (size_t)(BLOCK / 16) * sizeof(TseStage<16>)];
    int b = blockIdx.x;
    if (b < bk.blocks[0]) { tse_node<64>(g, tse, x, p, bk.list[0], bk.count[0], b, smem); return; }  // > 64 slots
    b -= bk.blocks[0];
    if (b < bk.blocks[1]) { tse_node<64>(g, tse, x, p, bk.list[1], bk.count[1], b, smem); return; }
    b -= bk.blocks[1];
    if (b < bk.blocks[2]) { tse_node<32>(g, tse, x, p, bk.list[2], bk.count[2], b, smem); return; }
    b -= bk.blocks[2];
    if (b < bk.blocks[3]) { tse_node<16>(g, tse, x, p, bk.list[3], bk.count[3], b, smem); return; }
    b -= bk.blocks[3];
    tse_node<8>(g, tse, x, p, bk.list[4], bk.count[4], b, smem);
}

}  // namespace

extern "C" int gtf_track_state_estimates(const gtf_graph* g, gtf_states* tse, const gtf_tse_extra* x,
                                         const gtf_params* p, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_track_state_estimates")) return rc;
    if (!tse || !x || !p) { gtf::set_error("gtf_track_state_estimates: null argument"); return -2; }
    if (g->n_nodes < 0 || g->n_slots < 0) { gtf::set_error("gtf_track_state_estimates: negative sizes"); return -2; }
    if (g->n_nodes == 0) return 0;
    if (!g->sched || !g->slot_ptr || !g->slot_src || !g->gnn || !tse->rank || !tse->sv || !tse->tau || !tse->cov ||
        !tse->xyzr) {
        gtf::set_error("gtf_track_state_estimates: needs the node schedule, graph arrays and TSE outputs");
        return -2;
    }
    // nodes with <= 4 slots (n_g4, scheduled first) take the 8-lane path
    const int n8 = g->n_g4 + g->n_g8, n16 = g->n_g16, n32 = g->n_g32, n64 = g->n_g64;
    const int rest = g->n_big;
    if (rest < 0 || g->n_g4 < 0 || g->n_g8 < 0 || n16 < 0 || n32 < 0 || n64 < 0) {
        gtf::set_error("gtf_track_state_estimates: bad schedule counts");
        return -2;
    }
    TseBuckets bk;
    bk.list[0] = g->sched + n8 + n16 + n32 + n64; bk.count[0] = rest;
    bk.list[1] = g->sched + n8 + n16 + n32;       bk.count[1] = n64;
    bk.list[2] = g->sched + n8 + n16;             bk.count[2] = n32;
    bk.list[3] = g->sched + n8;                   bk.count[3] = n16;
    bk.list[4] = g->sched;                        bk.count[4] = n8;
    const int gs[5] = {64, 64, 32, 16, 8};
    int total = 0;
    for (int i = 0; i < 5; i++) {
        bk.blocks[i] = (bk.count[i] + BLOCK / gs[i] - 1) / (BLOCK / gs[i]);
        total += bk.blocks[i];
    }
    hipLaunchKernelGGL(k_tse, dim3(total), dim3(BLOCK), 0, (hipStream_t)stream, *g, *tse, *x, *p, bk);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { gtf::set_error(hipGetErrorString(e)); return -1; }
    return 0;
}
