// gtf_math.h -- fp64 small-matrix arithmetic of the track-finding pass, written
// in the operation order of the reference's NumPy expressions so that results
// track the CPU path to the last few ulps (built with -ffp-contract=off: no
// fused multiply-add where the reference has separate roundings).
//
// Covariances on the path are block diagonal [[c00 c01 0][c10 c11 0][0 0 c22]]
// (the reference zeroes row/col 2 of every stored state covariance:
// helper.py:422-425, extrapolate_merged_states.py:362-365), carried as 5 numbers.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace gtf {

struct Cov5 {
    double c00, c01, c10, c11, c22;
};

// LAPACK-style 2x2 inverse (dgetrf partial pivoting, then solve A X = I), the
// path np.linalg.inv takes; keeps the result close to the reference's bits.
__device__ __forceinline__ void inv2(double a, double b, double c, double d, double& i00, double& i01,
                                     double& i10, double& i11) {
    if (fabs(c) > fabs(a)) {
        // rows swapped: P A = [[c d][a b]]
        double l = a / c;
        double u22 = b - l * d;
        // solve for columns of P^-1 ... P A X = P I ; P I = [[0 1][1 0]]
        // column 0 of X: rhs (0, 1)
        double y1 = 1.0 - l * 0.0;
        double x1 = y1 / u22;
        double x0 = (0.0 - d * x1) / c;
        // column 1 of X: rhs (1, 0)
        double z1 = 0.0 - l * 1.0;
        double w1 = z1 / u22;
        double w0 = (1.0 - d * w1) / c;
        i00 = x0; i10 = x1; i01 = w0; i11 = w1;
    } else {
        double l = c / a;
        double u22 = d - l * b;
        double y1 = 0.0 - l * 1.0;
        double x1 = y1 / u22;
        double x0 = (1.0 - b * x1) / a;
        double z1 = 1.0 - l * 0.0;
        double w1 = z1 / u22;
        double w0 = (0.0 - b * w1) / a;
        i00 = x0; i10 = x1; i01 = w0; i11 = w1;
    }
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

// y = M x for a block-diagonal M (zeros contribute exact zeros)
__device__ __forceinline__ void mv_cov5(const Cov5& m, const double x[3], double y[3]) {
    y[0] = m.c00 * x[0] + m.c01 * x[1];
    y[1] = m.c10 * x[0] + m.c11 * x[1];
    y[2] = m.c22 * x[2];
}

// merge_states (clustering.py:97-105): inverse-variance weighted mean
__device__ __forceinline__ void merge_states(const double m1[3], const Cov5& c1, const double m2[3], const Cov5& c2,
                                             double mo[3], Cov5& co) {
    Cov5 i1 = inv_cov5(c1);
    Cov5 i2 = inv_cov5(c2);
    Cov5 s = add_cov5(i1, i2);
    co = inv_cov5(s);
    double a[3], b[3], t[3];
    mv_cov5(i1, m1, a);
    mv_cov5(i2, m2, b);
    t[0] = a[0] + b[0];
    t[1] = a[1] + b[1];
    t[2] = a[2] + b[2];
    mv_cov5(co, t, mo);
}

// KLDistance (clustering.py:90-94): trace((C1-C2) .* (I2-I1)) + dm' (I1+I2) dm
__device__ __forceinline__ double kl_distance(const double m1[3], const Cov5& c1, const double m2[3], const Cov5& c2) {
    Cov5 i1 = inv_cov5(c1);
    Cov5 i2 = inv_cov5(c2);
    double tr = (c1.c00 - c2.c00) * (i2.c00 - i1.c00);
    tr = tr + (c1.c11 - c2.c11) * (i2.c11 - i1.c11);
    tr = tr + (c1.c22 - c2.c22) * (i2.c22 - i1.c22);
    Cov5 s = add_cov5(i1, i2);
    double d0 = m1[0] - m2[0], d1 = m1[1] - m2[1], d2 = m1[2] - m2[2];
    double w0 = d0 * s.c00 + d1 * s.c10;
    double w1 = d0 * s.c01 + d1 * s.c11;
    double w2 = d2 * s.c22;
    double q = w0 * d0 + w1 * d1;
    q = q + w2 * d2;
    return tr + q;
}

// mahalanobis_distance (clustering.py:11-78); variant=1 is the updated-state
// flavour of calculate_distance_between_updated_track_states.py:27-104.
__device__ __forceinline__ double mahalanobis(double a1, double b1, const Cov5& c1, double a2, double b2,
                                              const Cov5& c2, const double* na, const double* nb,
                                              const double* nc, double sz_barrel, double sr_barrel,
                                              double sz_endcap, double sr_endcap, double boundary) {
    double r0 = a1 - a2, r1 = b1 - b2;
    double i00, i01, i10, i11;
    inv2(c1.c00 + c2.c00, c1.c01 + c2.c01, c1.c10 + c2.c10, c1.c11 + c2.c11, i00, i01, i10, i11);
    double t0 = r0 * i00 + r1 * i10;
    double t1 = r0 * i01 + r1 * i11;
    double d1 = t0 * r0 + t1 * r1;
    double x_a = na[0], x_b = nb[0], x_c = nc[0];
    double z_a = na[2], r_a = na[3], z_b = nb[2], r_b = nb[3], z_c = nc[2], r_c = nc[3];
    double j2 = 1.0 / (r_b - r_a);
    double j3 = -1.0 / (r_c - r_a);
    double j1 = -j3 - j2;
    double drb = r_b - r_a, drc = r_c - r_a;
    double j5 = -(z_b - z_a) / (drb * drb);
    double j6 = (z_c - z_a) / (drc * drc);
    double j4 = -j5 - j6;
    double sza = sz_barrel, szb = sz_barrel, szc = sz_barrel;
    double sra = sr_barrel, srb = sr_barrel, src = sr_barrel;
    if (fabs(x_a) >= boundary) { sza = sz_endcap; sra = sr_endcap; }
    if (fabs(x_b) >= boundary) { szb = sz_endcap; srb = sr_endcap; }
    if (fabs(x_c) >= boundary) { szc = sz_endcap; src = sr_endcap; }
    double cdt = (j1 * (sza * sza)) * j1;
    cdt = cdt + (j2 * (szb * szb)) * j2;
    cdt = cdt + (j3 * (szc * szc)) * j3;
    cdt = cdt + (j4 * (sra * sra)) * j4;
    cdt = cdt + (j5 * (srb * srb)) * j5;
    cdt = cdt + (j6 * (src * src)) * j6;
    double inv_cdt = 1.0 / cdt;
    double tau1 = (z_b - z_a) / drb;
    double tau2 = (z_c - z_a) / drc;
    double res = tau1 - tau2;
    double d2 = (res * res) * inv_cdt;
    return d1 + d2;
}

struct Mat3 {
    double m[3][3];
};

__device__ __forceinline__ Mat3 mm3(const Mat3& A, const Mat3& B) {
    Mat3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double s = A.m[i][0] * B.m[0][j];
            s = s + A.m[i][1] * B.m[1][j];
            s = s + A.m[i][2] * B.m[2][j];
            C.m[i][j] = s;
        }
    return C;
}

// A * B^T
__device__ __forceinline__ Mat3 mm3t(const Mat3& A, const Mat3& B) {
    Mat3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double s = A.m[i][0] * B.m[j][0];
            s = s + A.m[i][1] * B.m[j][1];
            s = s + A.m[i][2] * B.m[j][2];
            C.m[i][j] = s;
        }
    return C;
}

__device__ __forceinline__ void mv3(const Mat3& A, const double x[3], double y[3]) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double s = A.m[i][0] * x[0];
        s = s + A.m[i][1] * x[1];
        s = s + A.m[i][2] * x[2];
        y[i] = s;
    }
}

}  // namespace gtf
