// gtf_math.h -- fp64 small-matrix arithmetic of the track-finding pass, written
// in the operation order of the reference's NumPy expressions so that results
// track the CPU path to the last few ulps (built with -ffp-contract=off: no
// fused multiply-add where the reference has separate roundings, and an explicit
// fma() exactly where numpy's BLAS / LAPACK kernels fuse, see below).
//
// Covariances on the path are block diagonal [[c00 c01 0][c10 c11 0][0 0 c22]]
// (the reference zeroes row/col 2 of every stored state covariance:
// helper.py:422-425, extrapolate_merged_states.py:362-365), carried as 5 numbers.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/gtf.h"

namespace gtf {

void set_error(const char* msg);   // gtf_last_error() text (gtf_pass.hip)

// A gtf_graph built against another layout of include/gtf.h: refused with status -3
// instead of read with shifted fields. Host side, every entry point taking a gtf_graph.
inline int check_abi(const gtf_graph* g, const char* who) {
    if (!g) {
        char m[160];
        snprintf(m, sizeof(m), "%s: null graph", who);
        set_error(m);
        return -2;
    }
    if (g->struct_size != (uint32_t)sizeof(gtf_graph) || g->abi_version != GTF_ABI_VERSION) {
        char m[200];
        snprintf(m, sizeof(m), "%s: gtf_graph ABI mismatch (caller struct_size %u, abi_version %u; library %u, %u)",
                 who, g->struct_size, g->abi_version, (unsigned)sizeof(gtf_graph), (unsigned)GTF_ABI_VERSION);
        set_error(m);
        return -3;
    }
    return 0;
}

// XCD-aware block index. MI355X deals workgroups round-robin over its 8 XCDs, each with
// its own 4 MiB L2 (MI355X_MICROARCH.md, workgroup dispatch), so consecutive blocks --
// which gather the same nodes' data -- would fill eight L2s with the same lines. This
// bijective remap (cdna_hip_programming.md T1) gives the blocks that share an XCD one
// contiguous range of work instead. `b` indexes a range of n blocks that starts at a
// multiple of 8 in the grid; speed only, never correctness.
__device__ __forceinline__ int xcd_local(int b, int n) {
    const int q = n / 8, r = n % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}
__host__ __device__ __forceinline__ int pad8(int n) { return (n + 7) & ~7; }
// the same family by one parameter: C = 0 xcd_local (one contiguous range per XCD), C = 1
// dispatch order, C > 1 runs of C consecutive blocks per XCD interleaved over the 8 XCDs
// (the last partial round of 8 C blocks in dispatch order); a bijection of [0, n) each
template <int C>
__device__ __forceinline__ int block_map(int b, int n) {
    if constexpr (C == 0) {
        return xcd_local(b, n);
    } else if constexpr (C == 1) {
        return b;
    } else {
        const int full = n / (8 * C) * (8 * C);
        if (b >= full) return b;
        const int x = b % 8, r = b / 8;
        return (r / C) * 8 * C + x * C + r % C;
    }
}

// Lanes of ONE wavefront hand values to each other through LDS. A wave's LDS
// instructions execute in issue order, so only the compiler has to be kept from
// moving loads above the other lanes' stores: wavefront-scope fences around a
// wave barrier. (Plain, not volatile, LDS pointers: a volatile access makes the
// compiler wait for each LDS load on its own instead of batching them.)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// row i and column j of lower-triangle pair t in row-major order
// ((1,0) (2,0) (2,1) (3,0) ...): t = i (i - 1) / 2 + j. Arithmetic, not a table: a
// lane-varying index into a __constant__ table is a vector memory load per pair.
__device__ __forceinline__ void pair_ij(int t, int& i, int& j) {
    int r = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)t)) * 0.5f);
    while (r * (r - 1) / 2 > t) r--;
    while ((r + 1) * r / 2 <= t) r++;
    i = r;
    j = t - r * (r - 1) / 2;
}

// x / d given r = 1.0 / d (correctly rounded): one product and two fused corrections give
// the correctly rounded quotient, the same bits as x / d (Markstein's theorem: r = RN(1/d),
// q = RN(x r), e = x - d q exactly, RN(q + e r) = RN(x / d); quotients near the ends of
// the exponent range, zeros and non-finite operands take the division; checked on random,
// adversarial and special operands in tests/test_numpy_rounding.py). A divisor
// used k times then costs one division and k * 3 instructions instead of k divisions.
__device__ __forceinline__ double qdiv(double x, double d, double r) {
    const double q = x * r;
    const double m = fabs(q);
    if (m >= 0x1p-960 && m <= 0x1p+1000) return fma(fma(-q, d, x), r, q);
    return x / d;   // zero, subnormal, huge, inf / NaN quotients (or d = 0, inf, NaN): divide
}

struct Cov5 {
    double c00, c01, c10, c11, c22;
};

// numpy's small products go through OpenBLAS (0.3.29, x86-64 FMA kernels), whose
// rounding the reference's values carry; these helpers reproduce it bit for bit
// (checked against numpy on random operands, tests/test_numpy_rounding.py):
//   x @ y (1-D, ddot)           s = x0*y0; s = fma(x1, y1, s); s = fma(x2, y2, s) ...
//   A @ x (gemv_n, 3x3)         s = A_i1*x1; s = fma(A_i0, x0, s); s = fma(A_i2, x2, s)
//   x @ A (gemv_t)              s = x0*A_0j; s = fma(x1, A_1j, s); s = fma(x2, A_2j, s)
//   A @ B, A @ B.T (gemm, 3x3)  s = A_i0*B_0j; s = fma(A_i1, B_1j, s); s = fma(A_i2, B_2j, s)
// Exact zeros of block-diagonal operands add exact zeros and are skipped.

// 2x2 inverse the way np.linalg.inv gets it from OpenBLAS (dgesv = getf2 LU with
// partial pivoting, then triangular solves): the pivot and u22 are inverted once and
// multiplied (getf2 scales by 1/pivot, the trsm kernels store the inverted diagonal),
// and the back substitution's update is one fused multiply-add (trsm kernel
// c -= b * a), so each inverse costs two divisions.
__device__ __forceinline__ void inv2(double a, double b, double c, double d, double& i00, double& i01,
                                     double& i10, double& i11) {
    const bool sw = fabs(c) > fabs(a);
    const double p0 = sw ? c : a, p1 = sw ? d : b;   // pivot row
    const double q0 = sw ? a : c, q1 = sw ? b : d;   // other row
    const double rp = 1.0 / p0;
    const double l = q0 * rp;
    const double u22 = q1 - l * p1;
    const double ru = 1.0 / u22;
    // columns of P*I: e0 -> (sw ? (0,1) : (1,0)), e1 -> (sw ? (1,0) : (0,1))
    const double y0a = sw ? 0.0 : 1.0, y1a = (sw ? 1.0 : 0.0) - l * y0a;
    const double x1a = y1a * ru, x0a = fma(-x1a, p1, y0a) * rp;
    const double y0b = sw ? 1.0 : 0.0, y1b = (sw ? 0.0 : 1.0) - l * y0b;
    const double x1b = y1b * ru, x0b = fma(-x1b, p1, y0b) * rp;
    i00 = x0a; i10 = x1a; i01 = x0b; i11 = x1b;
}

__device__ __forceinline__ Cov5 inv_cov5(const Cov5& m) {
    Cov5 r;
    inv2(m.c00, m.c01, m.c10, m.c11, r.c00, r.c01, r.c10, r.c11);
    r.c22 = 1.0 / m.c22;
    return r;
}

__device__ __forceinline__ Cov5 add_cov5(const Cov5& a, const Cov5& b) {
    return Cov5{a.c00 + b.c00, a.c01 + b.c01, a.c10 + b.c10, a.c11 + b.c11, a.c22 + b.c22};
}

// y = M x (numpy gemv_n) for a block-diagonal M (zeros contribute exact zeros)
__device__ __forceinline__ void mv_cov5(const Cov5& m, const double x[3], double y[3]) {
    y[0] = fma(m.c00, x[0], m.c01 * x[1]);
    y[1] = fma(m.c10, x[0], m.c11 * x[1]);
    y[2] = m.c22 * x[2];
}

// merge_states (clustering.py:97-105) given the two inverses already computed:
// merged_cov = (I1 + I2)^-1, merged_mean = merged_cov (I1 m1 + I2 m2)
__device__ __forceinline__ void merge_with_inv(const double m1[3], const Cov5& i1, const double m2[3], const Cov5& i2,
                                               const Cov5& co, double mo[3]) {
    double a[3], b[3], t[3];
    mv_cov5(i1, m1, a);
    mv_cov5(i2, m2, b);
    t[0] = a[0] + b[0];
    t[1] = a[1] + b[1];
    t[2] = a[2] + b[2];
    mv_cov5(co, t, mo);
}

// merge_with_inv of the parabolic (a, b, c) and the joint (a, b, tau) means at once, as one
// 4-vector (a, b, c, tau): components 0 and 1 of the two merges are the same operations on
// the same operands, so they are formed once
__device__ __forceinline__ void merge4_with_inv(const double m1[4], const Cov5& i1, const double m2[4], const Cov5& i2,
                                                const Cov5& co, double mo[4]) {
    const double a0 = fma(i1.c00, m1[0], i1.c01 * m1[1]), a1 = fma(i1.c10, m1[0], i1.c11 * m1[1]);
    const double b0 = fma(i2.c00, m2[0], i2.c01 * m2[1]), b1 = fma(i2.c10, m2[0], i2.c11 * m2[1]);
    const double t0 = a0 + b0, t1 = a1 + b1;
    const double tc = i1.c22 * m1[2] + i2.c22 * m2[2];
    const double tt = i1.c22 * m1[3] + i2.c22 * m2[3];
    mo[0] = fma(co.c00, t0, co.c01 * t1);
    mo[1] = fma(co.c10, t0, co.c11 * t1);
    mo[2] = co.c22 * tc;
    mo[3] = co.c22 * tt;
}

__device__ __forceinline__ void merge_states(const double m1[3], const Cov5& c1, const double m2[3], const Cov5& c2,
                                             double mo[3], Cov5& co) {
    const Cov5 i1 = inv_cov5(c1);
    const Cov5 i2 = inv_cov5(c2);
    co = inv_cov5(add_cov5(i1, i2));
    merge_with_inv(m1, i1, m2, i2, co, mo);
}

// KLDistance (clustering.py:90-94) given both inverses:
// trace((C1-C2) .* (I2-I1)) + dm' (I1+I2) dm
__device__ __forceinline__ double kl_with_inv(const double m1[3], const Cov5& c1, const Cov5& i1, const double m2[3],
                                              const Cov5& c2, const Cov5& i2) {
    double tr = (c1.c00 - c2.c00) * (i2.c00 - i1.c00);
    tr = tr + (c1.c11 - c2.c11) * (i2.c11 - i1.c11);
    tr = tr + (c1.c22 - c2.c22) * (i2.c22 - i1.c22);
    const Cov5 s = add_cov5(i1, i2);
    const double d0 = m1[0] - m2[0], d1 = m1[1] - m2[1], d2 = m1[2] - m2[2];
    // dm @ (I1 + I2) (gemv_t), then @ dm (ddot)
    const double w0 = fma(d1, s.c10, d0 * s.c00);
    const double w1 = fma(d1, s.c11, d0 * s.c01);
    const double w2 = d2 * s.c22;
    double q = fma(w1, d1, w0 * d0);
    q = fma(w2, d2, q);
    return tr + q;
}

__device__ __forceinline__ double kl_distance(const double m1[3], const Cov5& c1, const double m2[3], const Cov5& c2) {
    return kl_with_inv(m1, c1, inv_cov5(c1), m2, c2, inv_cov5(c2));
}

// Per-neighbour geometry of the tau term of mahalanobis_distance (clustering.py:37-75),
// computed once per state instead of once per pair; every pair value is built from
// these with the reference's operation order (j1 = -j3 - j2 = q_j - q_i, j4 = -j5 - j6).
struct TauGeo {
    double q;    // 1 / (r - r_a)             (j2 of the pair's first state, -j3 of its second)
    double w;    // (z - z_a) / (r - r_a)**2  (-j5 / j6)
    double tau;  // (z - z_a) / (r - r_a)
    double sz2, sr2;  // sigma_z**2, sigma_r**2 of this hit (endcap swap on |x|)
};

__device__ __forceinline__ TauGeo tau_geo(double x, double z, double r, double za, double ra, double sz_barrel,
                                          double sr_barrel, double sz_endcap, double sr_endcap, double boundary) {
    TauGeo t;
    const double dr = r - ra, dz = z - za;
    t.q = 1.0 / dr;
    t.w = dz / (dr * dr);
    t.tau = dz / dr;
    const bool ec = fabs(x) >= boundary;
    const double sz = ec ? sz_endcap : sz_barrel, sr = ec ? sr_endcap : sr_barrel;
    t.sz2 = sz * sz;
    t.sr2 = sr * sr;
    return t;
}

// mahalanobis_distance (clustering.py:11-78) from [a, b], the 2x2 covariance blocks,
// the node's sigma pair and the two neighbours' TauGeo.
// its [a, b] term (d1) and its tau term (d2), separately
__device__ __forceinline__ double maha_d1(double a1, double b1, const Cov5& c1, double a2, double b2, const Cov5& c2) {
    const double r0 = a1 - a2, r1 = b1 - b2;
    double i00, i01, i10, i11;
    inv2(c1.c00 + c2.c00, c1.c01 + c2.c01, c1.c10 + c2.c10, c1.c11 + c2.c11, i00, i01, i10, i11);
    // residual @ inv (gemv_t), then @ residual (ddot)
    const double t0 = fma(r1, i10, r0 * i00);
    const double t1 = fma(r1, i11, r0 * i01);
    return fma(t1, r1, t0 * r0);
}

__device__ __forceinline__ double maha_d2(double sza2, double sra2, const TauGeo& gb, const TauGeo& gc) {
    const double j2 = gb.q, j3 = -gc.q;
    const double j1 = -j3 - j2;
    const double j5 = -gb.w, j6 = gc.w;
    const double j4 = -j5 - j6;
    // J @ diag(S) (exact products), then @ J (ddot)
    double cdt = (j1 * sza2) * j1;
    cdt = fma(j2 * gb.sz2, j2, cdt);
    cdt = fma(j3 * gc.sz2, j3, cdt);
    cdt = fma(j4 * sra2, j4, cdt);
    cdt = fma(j5 * gb.sr2, j5, cdt);
    cdt = fma(j6 * gc.sr2, j6, cdt);
    const double res = gb.tau - gc.tau;
    return (res * res) * (1.0 / cdt);
}

__device__ __forceinline__ double mahalanobis_geo(double a1, double b1, const Cov5& c1, double a2, double b2,
                                                  const Cov5& c2, double sza2, double sra2, const TauGeo& gb,
                                                  const TauGeo& gc) {
    const double d1 = maha_d1(a1, b1, c1, a2, b2, c2);
    const double d2 = maha_d2(sza2, sra2, gb, gc);
    return d1 + d2;
}

// mahalanobis from raw coordinates (thread-per-node path)
__device__ __forceinline__ double mahalanobis(double a1, double b1, const Cov5& c1, double a2, double b2,
                                              const Cov5& c2, const double* na, const double* nb,
                                              const double* nc, double sz_barrel, double sr_barrel,
                                              double sz_endcap, double sr_endcap, double boundary) {
    const TauGeo gb = tau_geo(nb[0], nb[2], nb[3], na[2], na[3], sz_barrel, sr_barrel, sz_endcap, sr_endcap, boundary);
    const TauGeo gc = tau_geo(nc[0], nc[2], nc[3], na[2], na[3], sz_barrel, sr_barrel, sz_endcap, sr_endcap, boundary);
    const bool ec = fabs(na[0]) >= boundary;
    const double sza = ec ? sz_endcap : sz_barrel, sra = ec ? sr_endcap : sr_barrel;
    return mahalanobis_geo(a1, b1, c1, a2, b2, c2, sza * sza, sra * sra, gb, gc);
}

struct Mat3 {
    double m[3][3];
};

// A @ B (numpy gemm)
__device__ __forceinline__ Mat3 mm3(const Mat3& A, const Mat3& B) {
    Mat3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double s = A.m[i][0] * B.m[0][j];
            s = fma(A.m[i][1], B.m[1][j], s);
            s = fma(A.m[i][2], B.m[2][j], s);
            C.m[i][j] = s;
        }
    return C;
}

// A @ B.T (numpy gemm)
__device__ __forceinline__ Mat3 mm3t(const Mat3& A, const Mat3& B) {
    Mat3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double s = A.m[i][0] * B.m[j][0];
            s = fma(A.m[i][1], B.m[j][1], s);
            s = fma(A.m[i][2], B.m[j][2], s);
            C.m[i][j] = s;
        }
    return C;
}

// A @ C for a block-diagonal C ([[c00 c01 0] [c10 c11 0] [0 0 c22]]): the products with
// C's exact zeros, which add nothing to the reference's sums, are skipped
__device__ __forceinline__ Mat3 mul_block(const Mat3& A, const Mat3& C) {
    Mat3 R;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        R.m[i][0] = fma(A.m[i][1], C.m[1][0], A.m[i][0] * C.m[0][0]);
        R.m[i][1] = fma(A.m[i][1], C.m[1][1], A.m[i][0] * C.m[0][1]);
        R.m[i][2] = A.m[i][2] * C.m[2][2];
    }
    return R;
}

// A @ x (numpy gemv_n: column 1 first, then 0, then 2)
__device__ __forceinline__ void mv3(const Mat3& A, const double x[3], double y[3]) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double s = A.m[i][1] * x[1];
        s = fma(A.m[i][0], x[0], s);
        s = fma(A.m[i][2], x[2], s);
        y[i] = s;
    }
}

}  // namespace gtf
