// gtf_extract.hip -- track-candidate extraction on the GPU:
// src/extract/extract_track_candidates.py main (:349-467) after the hot path.
//
//  1. CCA (:332-346): connected components over the ACTIVATED edges of each subgraph
//     (undirected), by min-label hooking + pointer jumping; a subgraph with no
//     deactivated edge is one candidate whatever its connectivity (:342-343). A
//     candidate's id is its first node (min index), so ids sort in the reference's
//     candidate order (subgraph order, then weakly_connected_components order).
//  2. Members grouped per candidate by one radix sort of (candidate, order key).
//  3. One thread per candidate (a candidate is a handful of hits): fragment check,
//     close-proximity merging with the reference's in-place GNN_Measurement mutation
//     (:56-152), the one-hit-per-layer check (:407), the stable sort by radius (:411),
//     rotate_track (:176-195), the xy (3-state OU) and rz (2-state) Kalman fits with
//     filterpy 1.4.5 predict/update (:209-327) and the chi-square p-values
//     (scipy.stats.chi2.sf = the regularized upper incomplete gamma, cephes igamc).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <stdint.h>

#include "../../include/gtf.h"
#include "gtf_math.h"

namespace gtf {
void set_error(const char* msg);
}

namespace {

constexpr int BLOCK = 256;
inline int grid(int n) { return (n + BLOCK - 1) / BLOCK; }

// ------------------------------------------------------------------ CCA
__global__ void __launch_bounds__(BLOCK) k_ex_init(int n, int n_sub, int32_t* label, uint8_t* inactive,
                                                   int32_t* flag) {
    const int t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n) label[t] = t;
    if (t < n_sub) inactive[t] = 0;
    if (t == 0) *flag = 0;
}

__global__ void __launch_bounds__(BLOCK) k_ex_inactive(gtf_graph g, gtf_edges e, const int32_t* sub,
                                                       uint8_t* inactive) {
    const int k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= g.n_slots || !g.is_edge[k]) return;
    if (e.act[k] == 0) inactive[sub[g.slot_dst[k]]] = 1;   // :335-336 (activated == 0)
}

__device__ __forceinline__ int find_root(const int32_t* label, int x) {
    int p = label[x];
    while (p != x) {
        x = p;
        p = label[x];
    }
    return x;
}

// hook the larger root under the smaller one for every active edge
__global__ void __launch_bounds__(BLOCK) k_ex_hook(gtf_graph g, gtf_edges e, int32_t* label, int32_t* flag) {
    const int k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= g.n_slots || !g.is_edge[k] || e.act[k] != 1) return;
    const int u = g.slot_src[k], v = g.slot_dst[k];
    const int ru = find_root(label, u), rv = find_root(label, v);
    if (ru == rv) return;
    const int hi = ru > rv ? ru : rv, lo = ru > rv ? rv : ru;
    atomicMin(&label[hi], lo);
    *flag = 1;
}

__global__ void __launch_bounds__(BLOCK) k_ex_compress(int n, int32_t* label) {
    const int v = blockIdx.x * BLOCK + threadIdx.x;
    if (v < n) label[v] = find_root(label, v);
}

// subgraphs without a deactivated edge stay whole; then the sort keys
__global__ void __launch_bounds__(BLOCK) k_ex_keys(int n, const int32_t* sub, const int32_t* sub_ptr,
                                                   const uint8_t* inactive, const int32_t* order_key,
                                                   int32_t* label, uint64_t* keys, int32_t* vals) {
    const int v = blockIdx.x * BLOCK + threadIdx.x;
    if (v >= n) return;
    const int s = sub[v];
    int l = label[v];
    if (!inactive[s]) l = sub_ptr[s];
    label[v] = l;
    keys[v] = ((uint64_t)(uint32_t)l << 32) | (uint32_t)(order_key ? order_key[v] : v);
    vals[v] = v;
}

__global__ void __launch_bounds__(BLOCK) k_ex_starts(int n, const uint64_t* keys, int32_t* is_start) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) is_start[i] = (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32)) ? 1 : 0;
}

__global__ void __launch_bounds__(BLOCK) k_ex_ptr(int n, const int32_t* is_start, const int32_t* cidx,
                                                  int32_t* cand_ptr, int32_t* n_cand) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n && is_start[i]) cand_ptr[cidx[i]] = i;
    if (i == n - 1) {
        const int nc = cidx[i] + is_start[i];
        *n_cand = nc;
        cand_ptr[nc] = n;
    }
}

// ------------------------------------------------------------------ chi2.sf
constexpr double MACHEP = 1.11022302462515654042e-16;
constexpr double MAXLOG = 7.09782712893383996843e2;
constexpr double BIG = 4.503599627370496e15;
constexpr double BIGINV = 2.22044604925031308085e-16;

__device__ double igamc(double a, double x);

__device__ double igam(double a, double x) {
    if (x <= 0.0 || a <= 0.0) return 0.0;
    if (x > 1.0 && x > a) return 1.0 - igamc(a, x);
    double ax = a * log(x) - x - lgamma(a);
    if (ax < -MAXLOG) return 0.0;
    ax = exp(ax);
    double r = a, c = 1.0, ans = 1.0;
    do {
        r += 1.0;
        c *= x / r;
        ans += c;
    } while (c / ans > MACHEP);
    return ans * ax / a;
}

__device__ double igamc(double a, double x) {
    if (x < 0.0 || a <= 0.0) return NAN;
    if (x < 1.0 || x < a) return 1.0 - igam(a, x);
    double ax = a * log(x) - x - lgamma(a);
    if (ax < -MAXLOG) return 0.0;
    ax = exp(ax);
    double y = 1.0 - a, z = x + y + 1.0, c = 0.0;
    double pkm2 = 1.0, qkm2 = x, pkm1 = x + 1.0, qkm1 = z * x;
    double ans = pkm1 / qkm1, t;
    do {
        c += 1.0;
        y += 1.0;
        z += 2.0;
        const double yc = y * c;
        const double pk = pkm1 * z - pkm2 * yc;
        const double qk = qkm1 * z - qkm2 * yc;
        if (qk != 0.0) {
            const double r = pk / qk;
            t = fabs((ans - r) / r);
            ans = r;
        } else {
            t = 1.0;
        }
        pkm2 = pkm1; pkm1 = pk; qkm2 = qkm1; qkm1 = qk;
        if (fabs(pk) > BIG) { pkm2 *= BIGINV; pkm1 *= BIGINV; qkm2 *= BIGINV; qkm1 *= BIGINV; }
    } while (t > MACHEP);
    return ans * ax;
}

__device__ __forceinline__ double chi2_sf(double x, int dof) {
    if (x != x) return NAN;
    return igamc(0.5 * dof, 0.5 * x);
}

// ------------------------------------------------------------------ CPython set order
// Iteration order of set() over the <= 2 duplicated (volume_id, in_volume_layer_id)
// tuples (:96): CPython 3.10 tuple hash (xxHash lanes of the item hashes; an integral
// float hashes to its integer) and set insertion into the minimum 8-slot table.
__device__ __forceinline__ uint64_t py_tuple_hash2(double a, double b) {
    const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P5 = 2870177450012600261ull;
    uint64_t acc = P5;
    const double it[2] = {a, b};
    for (int i = 0; i < 2; i++) {
        const int64_t hv = (int64_t)it[i];          // integral, small, non-negative
        const uint64_t lane = (uint64_t)(hv == -1 ? -2 : hv);
        acc += lane * P2;
        acc = (acc << 31) | (acc >> 33);
        acc *= P1;
    }
    acc += 2ull ^ (P5 ^ 3527539ull);
    if (acc == ~0ull) return 1546275796ull;
    return acc;
}

__device__ __forceinline__ int py_set_slot(uint64_t h, int occupied) {
    uint64_t i = h & 7ull, perturb = h;
    while ((int)i == occupied) {
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & 7ull;
    }
    return (int)i;
}

// ------------------------------------------------------------------ per candidate
struct Hit {
    double x, y, z, r;
};

struct KfState3 {
    double x[3], P[3][3];
};

// filterpy predict (x = F x, P = F P F^T + Q) and update with H = [1 0 0], scalar R
__device__ void kf3_step(KfState3& s, const double F[3][3], const double Q[3][3], double R, double z) {
    double x[3], FP[3][3], P[3][3];
    for (int i = 0; i < 3; i++) {
        double v = F[i][0] * s.x[0];
        v = v + F[i][1] * s.x[1];
        v = v + F[i][2] * s.x[2];
        x[i] = v;
    }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double v = F[i][0] * s.P[0][j];
            v = v + F[i][1] * s.P[1][j];
            v = v + F[i][2] * s.P[2][j];
            FP[i][j] = v;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double v = FP[i][0] * F[j][0];
            v = v + FP[i][1] * F[j][1];
            v = v + FP[i][2] * F[j][2];
            P[i][j] = v + Q[i][j];
        }
    const double y = z - x[0];
    const double S = P[0][0] + R;
    const double SI = 1.0 / S;
    const double K[3] = {P[0][0] * SI, P[1][0] * SI, P[2][0] * SI};
    for (int i = 0; i < 3; i++) s.x[i] = x[i] + K[i] * y;
    // Joseph form: (I - K H) P (I - K H)^T + K R K^T
    double IKH[3][3] = {{1.0 - K[0], 0.0, 0.0}, {0.0 - K[1], 1.0, 0.0}, {0.0 - K[2], 0.0, 1.0}};
    double A[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double v = IKH[i][0] * P[0][j];
            v = v + IKH[i][1] * P[1][j];
            v = v + IKH[i][2] * P[2][j];
            A[i][j] = v;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double v = A[i][0] * IKH[j][0];
            v = v + A[i][1] * IKH[j][1];
            v = v + A[i][2] * IKH[j][2];
            s.P[i][j] = v + (K[i] * R) * K[j];
        }
}

struct KfState2 {
    double x[2], P[2][2];
};

// F = [[1, dz], [0, 1]], scalar Q added to every entry of P (filterpy keeps a scalar Q
// as is, so F P F^T + Q broadcasts), H = [1 0], scalar R
__device__ void kf2_step(KfState2& s, double dz, double Q, double R, double z) {
    const double x0 = s.x[0] + dz * s.x[1], x1 = s.x[1];
    double FP[2][2];
    FP[0][0] = s.P[0][0] + dz * s.P[1][0];
    FP[0][1] = s.P[0][1] + dz * s.P[1][1];
    FP[1][0] = 0.0 * s.P[0][0] + 1.0 * s.P[1][0];
    FP[1][1] = 0.0 * s.P[0][1] + 1.0 * s.P[1][1];
    double P[2][2];
    P[0][0] = (FP[0][0] * 1.0 + FP[0][1] * dz) + Q;
    P[0][1] = (FP[0][0] * 0.0 + FP[0][1] * 1.0) + Q;
    P[1][0] = (FP[1][0] * 1.0 + FP[1][1] * dz) + Q;
    P[1][1] = (FP[1][0] * 0.0 + FP[1][1] * 1.0) + Q;
    const double y = z - x0;
    const double S = P[0][0] + R;
    const double SI = 1.0 / S;
    const double K[2] = {P[0][0] * SI, P[1][0] * SI};
    s.x[0] = x0 + K[0] * y;
    s.x[1] = x1 + K[1] * y;
    const double IKH[2][2] = {{1.0 - K[0], 0.0}, {0.0 - K[1], 1.0}};
    double A[2][2];
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++) A[i][j] = IKH[i][0] * P[0][j] + IKH[i][1] * P[1][j];
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++) s.P[i][j] = (A[i][0] * IKH[j][0] + A[i][1] * IKH[j][1]) + (K[i] * R) * K[j];
}

enum { EX_FRAGMENT = 0, EX_BAD = 1, EX_REJECTED = 2, EX_EXTRACTED = 3 };

__global__ void __launch_bounds__(BLOCK) k_ex_candidate(gtf_extract_io io, gtf_extract_params p,
                                                        const int32_t* members, const int32_t* cand_ptr,
                                                        const int32_t* n_cand_dev) {
    const int c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= *n_cand_dev) return;
    const int lo = cand_ptr[c], n = cand_ptr[c + 1] - lo;
    const int32_t* m = members + lo;
    const int root = io.label[m[0]];
    io.status[root] = EX_FRAGMENT;
    io.pval_xy[root] = NAN;
    io.pval_zr[root] = NAN;
    if (n < p.fragment) return;                                                   // :398
    auto vv = [&](int i, int comp) { return io.vivl[2 * (int64_t)m[i] + comp]; };
    auto same = [&](int i, int j) { return vv(i, 0) == vv(j, 0) && vv(i, 1) == vv(j, 1); };

    // ---- check_close_proximity_nodes (:56-152)
    int n2count = 0, bad_other = 0;
    int dup_first[2] = {-1, -1};
    for (int i = 0; i < n; i++) {
        bool first = true;
        int cnt = 0;
        for (int j = 0; j < n; j++) {
            if (same(i, j)) {
                cnt++;
                if (j < i) first = false;
            }
        }
        if (!first) continue;
        if (cnt == 2) {
            if (n2count < 2) dup_first[n2count] = i;
            n2count++;
        } else if (cnt != 1) {
            bad_other = 1;
        }
    }
    int removed[2] = {-1, -1}, mnode[2] = {-1, -1};
    Hit mid[2];
    bool copied = false;
    if (n2count >= 1 && n2count <= 2 && !bad_other) {
        copied = true;
        // set() iteration order of the duplicated tuples
        int order[2] = {0, 1};
        if (n2count == 2) {
            const uint64_t hA = py_tuple_hash2(vv(dup_first[0], 0), vv(dup_first[0], 1));
            const uint64_t hB = py_tuple_hash2(vv(dup_first[1], 0), vv(dup_first[1], 1));
            const int sA = py_set_slot(hA, -1);
            const int sB = py_set_slot(hB, sA);
            if (sB < sA) { order[0] = 1; order[1] = 0; }
        }
        int nm = 0;
        for (int q = 0; q < n2count; q++) {
            const int i1 = dup_first[order[q]];
            int i2 = -1;
            for (int j = i1 + 1; j < n && i2 < 0; j++)
                if (same(i1, j)) i2 = j;
            const double* c1 = io.xyzr + 4 * (int64_t)m[i1];
            const double* c2 = io.xyzr + 4 * (int64_t)m[i2];
            const double dx = c1[0] - c2[0], dy = c1[1] - c2[1], dz = c1[2] - c2[2];
            const double dist = sqrt(((dx * dx) + (dy * dy)) + (dz * dz));
            if (dist <= p.merge_distance) {
                Hit h;
                h.x = (c1[0] + c2[0]) / 2;
                h.y = (c1[1] + c2[1]) / 2;
                h.z = (c1[2] + c2[2]) / 2;
                h.r = sqrt(h.x * h.x + h.y * h.y);
                double* gm = io.gnn + 4 * (int64_t)m[i1];            // shared GNN_Measurement (:111-114)
                gm[0] = h.x; gm[1] = h.y; gm[2] = h.z; gm[3] = h.r;
                mnode[nm] = i1;
                mid[nm] = h;
                removed[nm] = i2;
                nm++;
            } else {
                copied = false;                                                  // :143-145
                break;
            }
        }
    }
    if (!copied) { removed[0] = removed[1] = -1; mnode[0] = mnode[1] = -1; }
    auto alive = [&](int i) { return i != removed[0] && i != removed[1]; };
    auto hit = [&](int i) {
        if (i == mnode[0]) return mid[0];
        if (i == mnode[1]) return mid[1];
        const double* c = io.xyzr + 4 * (int64_t)m[i];
        return Hit{c[0], c[1], c[2], c[3]};
    };

    // ---- one hit per layer (:405-407)
    int na = 0;
    bool unique = true;
    for (int i = 0; i < n; i++) {
        if (!alive(i)) continue;
        na++;
        for (int j = 0; j < i && unique; j++)
            if (alive(j) && same(i, j)) unique = false;
    }
    if (!unique || na < p.fragment) { io.status[root] = EX_BAD; return; }

    // ---- coordinates by radius, largest first, stable (:409-411): walk the order
    // with (r, position) cursors instead of sorting
    auto before = [&](int i, int j) {      // does i come before j in the sorted order?
        const double ri = hit(i).r, rj = hit(j).r;
        return ri > rj || (ri == rj && i < j);
    };
    auto next_after = [&](int last) {      // the element right after `last` (-1 = first)
        int best = -1;
        for (int i = 0; i < n; i++) {
            if (!alive(i)) continue;
            if (last >= 0 && !before(last, i)) continue;
            if (best < 0 || before(i, best)) best = i;
        }
        return best;
    };
    // the innermost three (coords[-1], [-2], [-3]) for rotate_track
    int last3[3] = {-1, -1, -1};
    for (int i = 0; i < n; i++) {
        if (!alive(i)) continue;
        // keep the 3 latest in order: last3[0] = last element, [1] = second last ...
        if (last3[0] < 0 || before(last3[0], i)) { last3[2] = last3[1]; last3[1] = last3[0]; last3[0] = i; }
        else if (last3[1] < 0 || before(last3[1], i)) { last3[2] = last3[1]; last3[1] = i; }
        else if (last3[2] < 0 || before(last3[2], i)) { last3[2] = i; }
    }
    const Hit p1 = hit(last3[0]);
    Hit p2 = hit(last3[1]);
    {
        const double dx = p1.x - p2.x, dy = p1.y - p2.y, dz = p1.z - p2.z;
        if (sqrt(((dx * dx) + (dy * dy)) + (dz * dz)) < p.separation_3d) p2 = hit(last3[2]);   // :181-183
    }
    const double axy = atan2(p2.y - p1.y, p2.x - p1.x), azr = atan2(p2.z - p1.z, p2.r - p1.r);
    const double cxy = cos(axy), sxy = sin(axy), czr = cos(azr), szr = sin(azr);
    auto rot = [&](const Hit& h) {
        return Hit{h.x * cxy + h.y * sxy, -h.x * sxy + h.y * cxy, -h.z * szr + h.z * czr, h.r * czr + h.r * szr};
    };

    // ---- KF_track_fit_moliere (:209-327)
    int cur = next_after(-1);
    Hit h2 = rot(hit(cur));
    KfState3 f;
    f.x[0] = h2.y; f.x[1] = 0.0; f.x[2] = 0.0;
    const double s2xy = p.sigma0xy * p.sigma0xy, s2rz = p.sigma0rz * p.sigma0rz;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) f.P[i][j] = 0.0;
    f.P[0][0] = s2xy; f.P[1][1] = 1.0; f.P[2][2] = 1.0;
    KfState2 gk;
    gk.x[0] = h2.r; gk.x[1] = 0.0;
    gk.P[0][0] = s2rz; gk.P[0][1] = 0.0; gk.P[1][0] = 0.0; gk.P[1][1] = 1000.0;
    double c2xy = 0.0, c2zr = 0.0;
    for (int step = 0; step < na - 1; step++) {
        cur = next_after(cur);
        const Hit h3 = rot(hit(cur));
        const double x1 = 0.0, y1 = 0.0;
        const double x2 = h2.x, y2 = h2.y, x3 = h3.x, y3 = h3.y;
        const double denom = (x1 - x2) * (x1 - x3) * (x2 - x3);
        const double a = ((x3 * (y2 - y1)) + (x2 * (y1 - y3)) + (x1 * (y3 - y2))) / denom;
        const double b = ((x3 * x3 * (y1 - y2)) + (x2 * x2 * (y3 - y1)) + (x1 * x1 * (y2 - y3))) / denom;
        const double dr = h3.r - h2.r, dz = h3.z - h2.z;
        const double hyp = sqrt(dr * dr + dz * dz);
        const double sin_t = fabs(dr) / hyp;
        const double q = (2.0 * a * x3) + b;
        const double t15 = 1.0 + q * q;
        const double kappa = (2.0 * a) / (t15 * sqrt(t15));
        const double hl = (13.6 * 1e-3 * sqrt(0.02) * kappa) / 0.3;
        double var_ms = sin_t * (hl * hl);
        if (fabs(h3.z) >= p.endcap_boundary) var_ms = var_ms * fabs(dr / dz);
        const double dx = x3 - x2;
        const double alpha = 0.1;
        const double e1 = exp(-fabs(dx) * alpha);
        const double f1 = (1.0 - e1) / alpha;
        const double g1 = (fabs(dx) - f1) / alpha;
        const double sw2 = 0.00001 * 0.00001, st2 = var_ms;
        const double dx2 = dx * dx, dxw2 = dx2 * sw2;
        const double Q02 = 0.5 * dxw2, Q01 = dx * (st2 + Q02), Q12 = dx * sw2;
        const double F[3][3] = {{1.0, dx, g1}, {0.0, 1.0, f1}, {0.0, 0.0, e1}};
        const double Q[3][3] = {{dx2 * (st2 + 0.25 * dxw2), Q01, Q02}, {Q01, st2 + dxw2, Q12}, {Q02, Q12, sw2}};
        kf3_step(f, F, Q, s2xy, y3);
        {
            const double res = y3 - f.x[0];
            const double S = f.P[0][0] + s2xy;
            c2xy = c2xy + (res * (1.0 / S)) * res;
        }
        kf2_step(gk, dz, var_ms, s2rz, h3.r);
        {
            const double res = h3.r - gk.x[0];
            const double S = gk.P[0][0] + s2rz;
            c2zr = c2zr + (res * (1.0 / S)) * res;
        }
        h2 = h3;
    }
    const double pv = chi2_sf(c2xy, na - 2), pz = chi2_sf(c2zr, na - 2);
    io.pval_xy[root] = pv;
    io.pval_zr[root] = pz;
    io.status[root] = (pv >= p.p_accept && pz >= p.p_accept) ? EX_EXTRACTED : EX_REJECTED;     // :416
}

__global__ void __launch_bounds__(BLOCK) k_ex_flags(int n, gtf_extract_io io) {
    const int v = blockIdx.x * BLOCK + threadIdx.x;
    if (v < n) io.extracted[v] = io.status[io.label[v]] == EX_EXTRACTED ? 1 : 0;
}

struct ExWs {
    uint64_t *keys_in, *keys_out;
    int32_t *vals_in, *vals_out, *is_start, *cidx, *cand_ptr, *flag;
    uint8_t* inactive;
    void* cub;
    size_t cub_bytes;
};

size_t al(size_t x) { return (x + 255) & ~size_t(255); }

size_t cub_bytes(int n) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (int32_t*)nullptr, (int32_t*)nullptr, n);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr, n);
    return a > b ? a : b;
}

ExWs carve_ex(void* base, int n, int n_sub) {
    char* p = (char*)base;
    ExWs w;
    w.keys_in = (uint64_t*)p; p += al(8 * (size_t)n);
    w.keys_out = (uint64_t*)p; p += al(8 * (size_t)n);
    w.vals_in = (int32_t*)p; p += al(4 * (size_t)n);
    w.vals_out = (int32_t*)p; p += al(4 * (size_t)n);
    w.is_start = (int32_t*)p; p += al(4 * (size_t)n);
    w.cidx = (int32_t*)p; p += al(4 * (size_t)n);
    w.cand_ptr = (int32_t*)p; p += al(4 * ((size_t)n + 1));
    w.flag = (int32_t*)p; p += 256;
    w.inactive = (uint8_t*)p; p += al((size_t)(n_sub > 0 ? n_sub : 1));
    w.cub_bytes = cub_bytes(n);
    w.cub = p;
    return w;
}

}  // namespace

extern "C" {

size_t gtf_extract_workspace_bytes(int32_t n_nodes, int32_t n_sub) {
    const int n = n_nodes > 0 ? n_nodes : 1;
    return 6 * al(8 * (size_t)n) + al(4 * ((size_t)n + 1)) + 256 + al((size_t)(n_sub > 0 ? n_sub : 1)) +
           cub_bytes(n) + 256;
}

int gtf_extract_candidates(const gtf_graph* g, const gtf_edges* e, const gtf_extract_io* io,
                           const gtf_extract_params* p, void* workspace, gtf_stream_t stream) {
    if (int rc = gtf::check_abi(g, "gtf_extract_candidates")) return rc;
    if (!e || !io || !p || !workspace) { gtf::set_error("gtf_extract_candidates: null argument"); return -2; }
    const int n = g->n_nodes;
    if (n <= 0) return 0;
    if (!io->xyzr || !io->vivl || !io->sub_id || !io->sub_ptr || !io->gnn || !io->label || !io->status ||
        !io->pval_xy || !io->pval_zr || !io->extracted || !io->n_candidates || p->fragment < 3) {
        gtf::set_error("gtf_extract_candidates: missing arrays or fragment < 3");
        return -2;
    }
    hipStream_t st = (hipStream_t)stream;
    ExWs w = carve_ex(workspace, n, io->n_sub);
    const int nb = grid(n > io->n_sub ? n : io->n_sub);
    hipLaunchKernelGGL(k_ex_init, dim3(nb), dim3(BLOCK), 0, st, n, io->n_sub, io->label, w.inactive, w.flag);
    if (g->n_slots > 0)
        hipLaunchKernelGGL(k_ex_inactive, dim3(grid(g->n_slots)), dim3(BLOCK), 0, st, *g, *e, io->sub_id,
                           w.inactive);
    // hook + compress until no root changes (candidates are short: a few rounds)
    for (int round = 0; round < 64; round++) {
        int32_t zero = 0, changed = 0;
        if (hipMemcpyAsync(w.flag, &zero, sizeof(int32_t), hipMemcpyHostToDevice, st) != hipSuccess) return -1;
        if (g->n_slots > 0)
            hipLaunchKernelGGL(k_ex_hook, dim3(grid(g->n_slots)), dim3(BLOCK), 0, st, *g, *e, io->label, w.flag);
        hipLaunchKernelGGL(k_ex_compress, dim3(grid(n)), dim3(BLOCK), 0, st, n, io->label);
        if (hipMemcpyAsync(&changed, w.flag, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            gtf::set_error("gtf_extract_candidates: CCA round failed");
            return -1;
        }
        if (!changed) break;
    }
    hipLaunchKernelGGL(k_ex_keys, dim3(grid(n)), dim3(BLOCK), 0, st, n, io->sub_id, io->sub_ptr, w.inactive,
                       io->order_key, io->label, w.keys_in, w.vals_in);
    size_t cb = w.cub_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.keys_in, w.keys_out, w.vals_in, w.vals_out, n, 0, 64, st) !=
        hipSuccess) {
        gtf::set_error("gtf_extract_candidates: sort failed");
        return -1;
    }
    hipLaunchKernelGGL(k_ex_starts, dim3(grid(n)), dim3(BLOCK), 0, st, n, w.keys_out, w.is_start);
    cb = w.cub_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.is_start, w.cidx, n, st) != hipSuccess) {
        gtf::set_error("gtf_extract_candidates: scan failed");
        return -1;
    }
    hipLaunchKernelGGL(k_ex_ptr, dim3(grid(n)), dim3(BLOCK), 0, st, n, w.is_start, w.cidx, w.cand_ptr,
                       io->n_candidates);
    hipLaunchKernelGGL(k_ex_candidate, dim3(grid(n)), dim3(BLOCK), 0, st, *io, *p, w.vals_out, w.cand_ptr,
                       io->n_candidates);
    hipLaunchKernelGGL(k_ex_flags, dim3(grid(n)), dim3(BLOCK), 0, st, n, *io);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) { gtf::set_error(hipGetErrorString(err)); return -1; }
    return 0;
}

}  // extern "C"
