// cpu_ref.cpp -- fp64 C++ restatement of the reference's hot-path pass, OpenMP over
// senders (message passing) and receivers (every node-local stage).
//
// TEST INFRASTRUCTURE / CPU BASELINE ONLY (oracle/): the all-cores CPU denominator of
// bench.py's cpu_baseline and a second CPU check of the fixtures
// (tests/test_cpu_ref.py). The product path never links or calls it.
//
// The pass is oracle.full_pass (gtf_oracle.py:564) = run_gnn_trackml_mod.sh:101,138,112:
//   extrapolate stage  extrapolate_merged_states.py:552-566
//     message_passing :406-451 with extrapolate_validate :26-402 and filterpy 1.4.5's
//     KalmanFilter.predict / update (third party, restated as in the oracle),
//     compute_prior_probabilities + reweight twice (helper.py:30-63, :99-225), degree (:67-73)
//   update stage       remove_state_metadata.py:29-53
//   clustering         clustering.py:11-124, 181-373 on updated_track_states
// on the packed layout of gtf.graph.TrackGraph (host arrays, structure of arrays).
//
// Arithmetic follows the reference's expressions in its operation order; numpy's small
// BLAS / LAPACK calls are restated with OpenBLAS 0.3.29's rounding (fused multiply-adds
// exactly where its x86-64 kernels fuse, none elsewhere: -ffp-contract=off; matrix
// inverses as its getf2 / trsm LU), so the clustering arithmetic equals numpy's bit for
// bit (tests/test_numpy_rounding.py) and the rest agrees to a few ulp (libm trig / exp).
//
// Everything after message passing reads and writes only the receiver's own slot
// segment, so one parallel loop over receivers runs the whole node-local op chain
// (the reference's per-stage loops over all nodes commute with it).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include <omp.h>

extern "C" {

struct cr_graph {
    int32_t n_nodes, n_slots;
    const int32_t* slot_ptr;   // [N+1]
    const int32_t* slot_src;   // [S] sender, -1 orphan key
    const int32_t* out_ptr;    // [N+1]
    const int32_t* out_slot;   // [E] successor order
    const uint8_t* is_edge;    // [S]
    const uint8_t* rev_edge;   // [S]
    const uint8_t* solo;       // [N] alone in its subgraph
    const double* gnn;         // [N*4]
    const double* xyzr;        // [N*4]
    const double* layer;       // [N]
    // node state
    uint8_t* has_merged;
    double* merged_state;      // [N*3]
    double* merged_cov;        // [N*5]
    double* merged_prior;
    uint8_t* has_tse;
    uint8_t* has_uts;
    int32_t* degree;
    // slot state
    uint8_t* act;
    double* edge_mw;
    const double* send_mw;
    int32_t* tse_rank;
    double* tse_prior;
    double* tse_sv;            // [S*3]
    double* tse_tau;
    double* tse_cov;           // [S*5]
    double* tse_xyzr;          // [S*4]
    double* tse_mw;
    int32_t* uts_rank;
    double* uts_sv;            // [S*3]
    double* uts_tau;
    double* uts_cov;           // [S*5]
    double* uts_xyzr;          // [S*4]
    double* uts_lik;
    double* uts_mw;
    double* uts_prior;
    double* uts_lr;
    int8_t* uts_side;
    uint8_t* uts_fresh;
};

struct cr_params {
    double sigma0xy, sigma0rz, sigma0rz2, endcap_boundary, chi2_cut, reweight_threshold, cluster_chi2, cluster_kl;
};

}  // extern "C"

namespace {

// flags = include/gtf.h GTF_ERR_* (the reference raises there)
enum : uint32_t {
    E_SEND_MW = 1, E_STALE_KEY = 2, E_ALL_ZERO = 4, E_TIE_EMPTIED = 8, E_EMPTY_MW = 16, E_NAN_KL = 32,
    E_NO_DICT = 64
};

struct M3 {
    double m[3][3];
};

M3 mul(const M3& a, const M3& b) {
    M3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = a.m[i][0] * b.m[0][j];       // numpy gemm (OpenBLAS: fused)
            s = fma(a.m[i][1], b.m[1][j], s);
            s = fma(a.m[i][2], b.m[2][j], s);
            r.m[i][j] = s;
        }
    return r;
}

M3 tr(const M3& a) {
    M3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.m[i][j] = a.m[j][i];
    return r;
}

void mv(const M3& a, const double x[3], double y[3]) {
    for (int i = 0; i < 3; i++) {
        double s = a.m[i][1] * x[1];                // numpy gemv_n: column 1, 0, 2, fused
        s = fma(a.m[i][0], x[0], s);
        s = fma(a.m[i][2], x[2], s);
        y[i] = s;
    }
}

// covariances of the state dicts are block diagonal (the reference's joint-cov alias,
// SURVEY a2/a7): c00 c01 c10 c11 c22
struct C5 {
    double c00, c01, c10, c11, c22;
};

C5 load5(const double* p) { return C5{p[0], p[1], p[2], p[3], p[4]}; }
void store5(double* p, const C5& c) { p[0] = c.c00; p[1] = c.c01; p[2] = c.c10; p[3] = c.c11; p[4] = c.c22; }

// np.linalg.inv of a 2x2 (OpenBLAS dgesv: getf2 LU with partial pivoting, trsm solves
// with inverted diagonals and a fused back-substitution update)
void inv2(double a, double b, double c, double d, double& i00, double& i01, double& i10, double& i11) {
    const bool sw = fabs(c) > fabs(a);
    const double p0 = sw ? c : a, p1 = sw ? d : b;
    const double q0 = sw ? a : c, q1 = sw ? b : d;
    const double rp = 1.0 / p0;                     // getf2 scales by 1 / pivot
    const double l = q0 * rp;
    const double u22 = q1 - l * p1;
    const double ru = 1.0 / u22;                    // trsm stores inverted diagonals
    // solve P A X = P I column by column
    const double e0a = sw ? 0.0 : 1.0, e1a = sw ? 1.0 : 0.0;
    const double y1a = e1a - l * e0a;
    const double x1a = y1a * ru, x0a = fma(-x1a, p1, e0a) * rp;
    const double e0b = sw ? 1.0 : 0.0, e1b = sw ? 0.0 : 1.0;
    const double y1b = e1b - l * e0b;
    const double x1b = y1b * ru, x0b = fma(-x1b, p1, e0b) * rp;
    i00 = x0a; i10 = x1a; i01 = x0b; i11 = x1b;
}

C5 inv5(const C5& m) {
    C5 r;
    inv2(m.c00, m.c01, m.c10, m.c11, r.c00, r.c01, r.c10, r.c11);
    r.c22 = 1.0 / m.c22;
    return r;
}

C5 add5(const C5& a, const C5& b) { return C5{a.c00 + b.c00, a.c01 + b.c01, a.c10 + b.c10, a.c11 + b.c11, a.c22 + b.c22}; }

void mv5(const C5& m, const double x[3], double y[3]) {
    y[0] = fma(m.c00, x[0], m.c01 * x[1]);          // numpy gemv_n
    y[1] = fma(m.c10, x[0], m.c11 * x[1]);
    y[2] = m.c22 * x[2];
}

// merge_states (clustering.py:97-105)
void merge(const double m1[3], const C5& c1, const double m2[3], const C5& c2, double mo[3], C5& co) {
    const C5 i1 = inv5(c1), i2 = inv5(c2);
    co = inv5(add5(i1, i2));
    double a[3], b[3], t[3];
    mv5(i1, m1, a);
    mv5(i2, m2, b);
    for (int i = 0; i < 3; i++) t[i] = a[i] + b[i];
    mv5(co, t, mo);
}

// KLDistance (clustering.py:90-94): trace((C1 - C2) * (I2 - I1)) + dm' (I1 + I2) dm
double kl(const double m1[3], const C5& c1, const double m2[3], const C5& c2) {
    const C5 i1 = inv5(c1), i2 = inv5(c2);
    double t = (c1.c00 - c2.c00) * (i2.c00 - i1.c00);
    t = t + (c1.c11 - c2.c11) * (i2.c11 - i1.c11);
    t = t + (c1.c22 - c2.c22) * (i2.c22 - i1.c22);
    const C5 s = add5(i1, i2);
    const double d0 = m1[0] - m2[0], d1 = m1[1] - m2[1], d2 = m1[2] - m2[2];
    const double w0 = fma(d1, s.c10, d0 * s.c00), w1 = fma(d1, s.c11, d0 * s.c01), w2 = d2 * s.c22;   // gemv_t
    double q = fma(w1, d1, w0 * d0);                                                                 // ddot
    q = fma(w2, d2, q);
    return t + q;
}

// mahalanobis_distance (clustering.py:11-78)
double mahalanobis(const double m1[3], const C5& c1, const double m2[3], const C5& c2, const double* na,
                   const double* nb, const double* nc, const cr_params& p) {
    const double r0 = m1[0] - m2[0], r1 = m1[1] - m2[1];
    double i00, i01, i10, i11;
    inv2(c1.c00 + c2.c00, c1.c01 + c2.c01, c1.c10 + c2.c10, c1.c11 + c2.c11, i00, i01, i10, i11);
    const double t0 = fma(r1, i10, r0 * i00), t1 = fma(r1, i11, r0 * i01);   // gemv_t
    const double d1 = fma(t1, r1, t0 * r0);                                  // ddot
    const double xa = na[0], xb = nb[0], xc = nc[0];
    const double za = na[2], ra = na[3], zb = nb[2], rb = nb[3], zc = nc[2], rc = nc[3];
    const double j2 = 1 / (rb - ra);
    const double j3 = -1 / (rc - ra);
    const double j1 = -j3 - j2;
    const double j5 = -(zb - za) / ((rb - ra) * (rb - ra));
    const double j6 = (zc - za) / ((rc - ra) * (rc - ra));
    const double j4 = -j5 - j6;
    double sza = p.sigma0rz2, szb = p.sigma0rz2, szc = p.sigma0rz2, sra = p.sigma0rz, srb = p.sigma0rz, src = p.sigma0rz;
    if (fabs(xa) >= p.endcap_boundary) { sza = p.sigma0rz; sra = p.sigma0rz2; }
    if (fabs(xb) >= p.endcap_boundary) { szb = p.sigma0rz; srb = p.sigma0rz2; }
    if (fabs(xc) >= p.endcap_boundary) { szc = p.sigma0rz; src = p.sigma0rz2; }
    double cdt = (j1 * (sza * sza)) * j1;             // J @ Sm (exact products) @ J (ddot)
    cdt = fma(j2 * (szb * szb), j2, cdt);
    cdt = fma(j3 * (szc * szc), j3, cdt);
    cdt = fma(j4 * (sra * sra), j4, cdt);
    cdt = fma(j5 * (srb * srb), j5, cdt);
    cdt = fma(j6 * (src * src), j6, cdt);
    const double inv_cdt = 1 / cdt;
    const double tau1 = (zb - za) / (rb - ra), tau2 = (zc - za) / (rc - ra);
    const double res = tau1 - tau2;
    return d1 + (res * res) * inv_cdt;
}

// extrapolate_validate (extrapolate_merged_states.py:26-402); cov is the sender's stored
// merged_cov, mutated in place (:127-128). Returns accepted.
bool extrapolate(const double* ng, const double* nb, const double st[3], M3& cov, const cr_params& p,
                 double out_sv[3], C5& out_cov, double& out_tau, double& out_lik) {
    const double nx = ng[0], ny = ng[1], nz = ng[2], nr = ng[3];
    const double bx = nb[0], by = nb[1], bz = nb[2], br = nb[3];
    const double ang = atan2(ny, nx);                                                 // :41
    const double ca = cos(ang), sa = sin(ang);
    const double xA = (bx - nx) * ca + (by - ny) * sa;                                // :52
    const double a = st[0], b = st[1], c = st[2];
    const double phi = atan2((nx * by) - (ny * bx), (nx * bx) + (ny * by));           // :59
    const double sp = sin(phi), cp = cos(phi);
    const double x_prime = xA + (c * sp);                                             // :63
    const double Vx = cp + (b * sp);
    const double Ax = a * sp;
    const double s_star = (-x_prime * ((2 * (Vx * Vx)) + (Ax * x_prime))) / (2 * (Vx * Vx * Vx));   // :68
    const double numer = xA + c * sp;                                                 // :82
    double den = cp + b * sp;
    const double den2 = den * den, den3 = den2 * den;
    const double ds_da = -(sp * (numer * numer)) / den3;
    const double ds_db = ((sp * numer) * (1 + ((3 * a * sp * numer) / den2))) / den2;
    const double ds_dc = -sp * (1 + ((2 * a * sp * numer) / den2)) / den;
    den = cp + ((2 * a + b) * sp);                                                    // :89
    const double d3 = den * den * den, d4 = d3 * den;
    const double da_da = (1 / d3) * (1 - ((6 * a * sp) * (s_star + a * ds_da) / den));
    const double da_db = (-3 * a * sp * ((2 * a * ds_db) + 1)) / d4;
    const double da_dc = (-6 * sp * ds_dc * (a * a)) / d4;
    den = cp + ((2 * a * s_star + b) * sp);                                           // :95
    double bracket = cp - ((sp * (-sp + ((2 * a * s_star + b) * cp))) / den);
    const double db_da = (2 * (s_star + a * ds_da) * bracket) / den;
    const double db_db = ((1 + (2 * a * ds_da)) * bracket) / den;
    const double db_dc = (2 * a * ds_dc * bracket) / den;
    bracket = (cp * (2 * a + b)) - sp;                                                // :102
    const double dc_da = (ds_da * bracket) + ((s_star * s_star) * cp);
    const double dc_db = (ds_db * bracket) + (s_star * cp);
    const double dc_dc = (ds_dc * bracket) + cp;
    const M3 F{{{da_da, da_db, da_dc}, {db_da, db_db, db_dc}, {dc_da, dc_db, dc_dc}}};
    const double dr = br - nr, dz = bz - nz;                                          // :114
    const double hyp = sqrt(dr * dr + dz * dz);
    const double sin_t = fabs(dr) / hyp;
    const double kb = (2 * a * bx) + b;
    const double kappa = (2 * a) / pow(1 + kb * kb, 1.5);
    const double ms = (13.6 * 1e-3 * sqrt(0.02) * kappa) / 0.3;
    double var_ms = sin_t * (ms * ms);                                                // :120
    if (fabs(nz) >= p.endcap_boundary) var_ms = var_ms * (fabs(dr) / fabs(dz));
    cov.m[1][1] += var_ms;                                                            // :128
    double xe[3];
    mv(F, st, xe);
    const M3 Pe = mul(mul(F, cov), tr(F));
    const double residual = 0.0 - xe[2];                                              // :137
    const double S = Pe.m[2][2] + p.sigma0xy * p.sigma0xy;
    const double inv_S = 1.0 / S;
    const double chi2 = (residual * inv_S) * residual;                                // :140
    if (!(chi2 <= p.chi2_cut)) return false;                                          // :298
    const double factor = 2 * M_PI * fabs(S);
    const double lik = pow(factor, -0.5) * exp(-0.5 * chi2);                          // :302-304
    // filterpy predict(): x = F x, P = F P F' + Q
    double x[3];
    mv(F, xe, x);
    M3 P = mul(mul(F, Pe), tr(F));
    P.m[1][1] = P.m[1][1] + var_ms;
    // update(0): y = z - H x, S = H P H' + R, K = P H' / S, x += K y,
    // P = (I - K H) P (I - K H)' + K R K'
    const double R = p.sigma0xy * p.sigma0xy;
    const double y = 0.0 - x[2];
    const double PHT[3] = {P.m[0][2], P.m[1][2], P.m[2][2]};
    const double S2 = PHT[2] + R;
    const double SI = 1.0 / S2;
    const double K[3] = {PHT[0] * SI, PHT[1] * SI, PHT[2] * SI};
    for (int i = 0; i < 3; i++) x[i] = x[i] + K[i] * y;
    M3 IKH{{{1, 0, -K[0]}, {0, 1, -K[1]}, {0, 0, 1 - K[2]}}};
    M3 KRK;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) KRK.m[i][j] = (K[i] * R) * K[j];
    M3 Pn = mul(mul(IKH, P), tr(IKH));
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Pn.m[i][j] = Pn.m[i][j] + KRK.m[i][j];
    const double tau = dz / dr;                                                       // :326
    double sr = p.sigma0rz, sz = p.sigma0rz2;
    if (fabs(nz) >= p.endcap_boundary) { sz = p.sigma0rz; sr = p.sigma0rz2; }
    double srn = p.sigma0rz, szn = p.sigma0rz2;
    if (fabs(bz) >= p.endcap_boundary) { szn = p.sigma0rz; srn = p.sigma0rz2; }
    const double J0 = 1 / dr, J1 = -1 / dr, J2 = -dz / (dr * dr), J3 = dz / (dr * dr);   // :344-348
    double vt = (J0 * (sz * sz)) * J0;                                                // :357-358 (ddot)
    vt = fma(J1 * (szn * szn), J1, vt);
    vt = fma(J2 * (sr * sr), J2, vt);
    vt = fma(J3 * (srn * srn), J3, vt);
    out_sv[0] = x[0]; out_sv[1] = x[1]; out_sv[2] = x[2];
    out_cov = C5{Pn.m[0][0], Pn.m[0][1], Pn.m[1][0], Pn.m[1][1], vt + var_ms};        // :361-365
    out_tau = tau;
    out_lik = lik;
    return true;
}

struct Seg {
    int lo, hi;
};

// slots of node v holding a key of the dict, in dict order
void dict_order(const int32_t* rank, int lo, int hi, std::vector<int>& out) {
    out.clear();
    for (int k = lo; k < hi; k++)
        if (rank[k] >= 0) out.push_back(k);
    std::sort(out.begin(), out.end(), [&](int x, int y) { return rank[x] < rank[y]; });
}

inline bool active(const cr_graph& g, int k) { return g.is_edge[k] && g.act[k] == 1; }

// one state dict's per-slot arrays
struct Dict {
    int32_t* rank;
    double *sv, *tau, *cov, *xyzr, *prior, *mw;
};

Dict uts_dict(const cr_graph& g) { return Dict{g.uts_rank, g.uts_sv, g.uts_tau, g.uts_cov, g.uts_xyzr, g.uts_prior, g.uts_mw}; }
Dict tse_dict(const cr_graph& g) { return Dict{g.tse_rank, g.tse_sv, g.tse_tau, g.tse_cov, g.tse_xyzr, g.tse_prior, g.tse_mw}; }

// compute_prior_probabilities (helper.py:30-63)
void priors(const cr_graph& g, const std::vector<int>& ord, double* prior) {
    for (int k : ord) {
        if (!active(g, k)) continue;
        const double L = g.layer[g.slot_src[k]];
        int n = 0;
        for (int q : ord)
            if (active(g, q) && g.layer[g.slot_src[q]] == L) n++;
        prior[k] = 1.0 / n;
    }
}

// calculate_side_norm_factor + reweight (helper.py:99-225), updated_track_states
void reweight(const cr_graph& g, int v, const std::vector<int>& ord, double thr, uint32_t& err) {
    const double node_x = g.gnn[4 * (int64_t)v];
    std::vector<double> lc, rc;
    bool any = false;
    for (int k : ord)
        if (active(g, k)) {
            any = true;
            const double x = g.uts_xyzr[4 * (int64_t)k];
            (x < node_x ? lc : rc).push_back(x);
        }
    const int last = ord.empty() ? -1 : ord.back();   // stale neighbour_num (helper.py:131,138)
    if (any && !g.is_edge[last]) { err |= E_STALE_KEY; return; }
    std::sort(lc.begin(), lc.end());
    std::sort(rc.begin(), rc.end());
    const double ln = (double)(std::unique(lc.begin(), lc.end()) - lc.begin());
    const double rn = (double)(std::unique(rc.begin(), rc.end()) - rc.begin());
    for (int k : ord)
        if (active(g, k)) {
            const bool left = g.uts_xyzr[4 * (int64_t)k] < node_x;
            g.uts_side[k] = left ? 0 : 1;
            g.uts_lr[k] = 1;
            if (g.act[last] == 1) g.uts_lr[k] = left ? ln : rn;
        }
    double denom = 0;
    for (int k : ord)
        if (active(g, k)) denom += g.uts_mw[k] * g.uts_lik[k];
    for (int k : ord)
        if (active(g, k)) {
            double w = (g.uts_mw[k] * g.uts_lik[k] * g.uts_prior[k]) / denom;
            w /= g.uts_lr[k];
            g.uts_mw[k] = w;
            g.edge_mw[k] = w;
            g.act[k] = w < thr ? 0 : 1;
        }
}

void degree(const cr_graph& g, int v) {
    int d = 0;
    for (int k = g.slot_ptr[v]; k < g.slot_ptr[v + 1]; k++) d += active(g, k);
    g.degree[v] = d;
}

// clustering.cluster body for one node (clustering.py:197-307) on one state dict
void cluster(const cr_graph& g, const Dict& dc, int v, const std::vector<int>& ord, const cr_params& p,
             double chi2_thr, double kl_thr, uint32_t& err) {
    const int num0 = (int)ord.size();
    if (num0 <= 2 || num0 >= 16) return;                                              // :207
    struct St {
        double ps[3], js[3];
        C5 c;
        double prior;
        int k;
    };
    std::vector<St> s(num0);
    for (int i = 0; i < num0; i++) {
        const int k = ord[i];
        for (int j = 0; j < 3; j++) s[i].ps[j] = dc.sv[3 * (int64_t)k + j];
        s[i].js[0] = s[i].ps[0]; s[i].js[1] = s[i].ps[1]; s[i].js[2] = dc.tau[k];
        s[i].c = load5(dc.cov + 5 * (int64_t)k);
        s[i].prior = dc.prior[k];
        s[i].k = k;
    }
    const double* na = g.xyzr + 4 * (int64_t)v;
    std::vector<double> D(num0 * num0, 0.0);
    bool any = false;
    for (int i = 0; i < num0; i++)
        for (int j = 0; j < i; j++) {
            const double d = mahalanobis(s[i].js, s[i].c, s[j].js, s[j].c, na, dc.xyzr + 4 * (int64_t)s[i].k,
                                         dc.xyzr + 4 * (int64_t)s[j].k, p);
            D[i * num0 + j] = d;
            any |= d != 0.0;
        }
    if (!any) { err |= E_ALL_ZERO; return; }                                          // :120
    // np.min over the nonzero entries: NaN if any of them is NaN
    double sm = INFINITY;
    for (double d : D)
        if (d != 0.0) sm = (d != d || sm != sm) ? NAN : (d < sm ? d : sm);
    // np.where(D == smallest): row-major positions, idx = concat(rows, cols)
    std::vector<int> rows, cols;
    for (int i = 0; i < num0; i++)
        for (int j = 0; j < num0; j++)
            if (D[i * num0 + j] == sm) { rows.push_back(i); cols.push_back(j); }
    if (!(sm < chi2_thr)) return;                                                     // :228
    std::vector<int> idx(rows);
    idx.insert(idx.end(), cols.begin(), cols.end());
    double pm[3], jm[3];
    C5 pc, jc;
    merge(s[idx[0]].ps, s[idx[0]].c, s[idx[1]].ps, s[idx[1]].c, pm, pc);
    merge(s[idx[0]].js, s[idx[0]].c, s[idx[1]].js, s[idx[1]].c, jm, jc);
    double mprior = s[idx[0]].prior + s[idx[1]].prior;
    std::vector<bool> drop(num0, false);
    for (int i : idx) drop[i] = true;
    std::vector<St> rest;
    for (int i = 0; i < num0; i++)
        if (!drop[i]) rest.push_back(s[i]);
    bool stop = false;
    if (rest.empty()) { err |= E_TIE_EMPTIED; stop = true; }                          // :116
    while (!stop) {
        int bi = 0;
        double bd = 0;
        for (int i = 0; i < (int)rest.size(); i++) {
            const double d = kl(rest[i].js, rest[i].c, jm, jc);
            if (d != d) { err |= E_NAN_KL; stop = true; break; }                      // :117
            if (i == 0 || d < bd) { bd = d; bi = i; }
        }
        if (stop || !(bd < kl_thr)) break;                                            // :261
        double pm2[3], jm2[3];
        C5 pc2, jc2;
        merge(rest[bi].ps, rest[bi].c, pm, pc, pm2, pc2);
        merge(rest[bi].js, rest[bi].c, jm, jc, jm2, jc2);
        memcpy(pm, pm2, sizeof pm); memcpy(jm, jm2, sizeof jm);
        pc = pc2; jc = jc2;
        mprior = rest[bi].prior + mprior;
        rest.erase(rest.begin() + bi);
        if (rest.empty()) break;
    }
    g.has_merged[v] = 1;                                                              // :291-293
    for (int j = 0; j < 3; j++) g.merged_state[3 * (int64_t)v + j] = pm[j];
    store5(g.merged_cov + 5 * (int64_t)v, pc);
    g.merged_prior[v] = mprior;
    for (const St& r : rest)                                                          // :311-321
        if (g.is_edge[r.k]) g.act[r.k] = 0;
}

// compute_mixture_weights (helper.py:76-96)
void mixture_weights(const cr_graph& g, int v, const std::vector<int>& ord, double* mwp, uint32_t& err) {
    if (ord.empty()) {
        if (!g.solo[v]) err |= E_EMPTY_MW;
        return;
    }
    const double mw = 1.0 / (double)ord.size();
    for (int k : ord) mwp[k] = mw;
}

}  // namespace

extern "C" {

// the fused pass of gtf_pass on host arrays; threads <= 0: OpenMP default.
// Returns the GTF_ERR_* flags of the places where the reference raises.
uint32_t cr_full_pass(const cr_graph* gp, const cr_params* pp, int threads) {
    const cr_graph& g = *gp;
    const cr_params& p = *pp;
    if (threads > 0) omp_set_num_threads(threads);
    uint32_t err = 0;
    const int N = g.n_nodes;
    memset(g.uts_fresh, 0, (size_t)g.n_slots);
    // ---- message passing (extrapolate_merged_states.py:406-451): one sender per task;
    // every out-slot belongs to one sender, so the writes never collide
#pragma omp parallel for schedule(dynamic, 64) reduction(| : err)
    for (int u = 0; u < N; u++) {
        if (!g.has_merged[u]) continue;
        const double st[3] = {g.merged_state[3 * (int64_t)u], g.merged_state[3 * (int64_t)u + 1],
                              g.merged_state[3 * (int64_t)u + 2]};
        const double* mc = g.merged_cov + 5 * (int64_t)u;
        M3 cov{{{mc[0], mc[1], 0.0}, {mc[2], mc[3], 0.0}, {0.0, 0.0, mc[4]}}};
        for (int e = g.out_ptr[u]; e < g.out_ptr[u + 1]; e++) {
            const int k = g.out_slot[e];
            if (g.act[k] != 1) continue;                                              // :431
            // receiver of slot k: the node whose slot segment holds it
            const int v = (int)(std::upper_bound(g.slot_ptr, g.slot_ptr + N + 1, k) - g.slot_ptr) - 1;
            double sv[3], tau, lik;
            C5 c5;
            if (extrapolate(g.gnn + 4 * (int64_t)u, g.gnn + 4 * (int64_t)v, st, cov, p, sv, c5, tau, lik)) {
                g.uts_fresh[k] = 1;
                for (int j = 0; j < 3; j++) g.uts_sv[3 * (int64_t)k + j] = sv[j];
                g.uts_tau[k] = tau;
                store5(g.uts_cov + 5 * (int64_t)k, c5);
                for (int j = 0; j < 4; j++) g.uts_xyzr[4 * (int64_t)k + j] = g.gnn[4 * (int64_t)u + j];
                g.uts_lik[k] = lik;
                if (g.send_mw[k] != g.send_mw[k]) err |= E_SEND_MW;                   // :384
                g.uts_mw[k] = g.send_mw[k];
                g.uts_prior[k] = NAN;
                g.uts_lr[k] = NAN;
                g.uts_side[k] = -1;
            } else {
                g.act[k] = 0;                                                         // :393
            }
        }
        double* m = g.merged_cov + 5 * (int64_t)u;                                   // in place (:128)
        m[0] = cov.m[0][0]; m[1] = cov.m[0][1]; m[2] = cov.m[1][0]; m[3] = cov.m[1][1]; m[4] = cov.m[2][2];
    }
    // ---- every node-local stage, one receiver per task
#pragma omp parallel reduction(| : err)
    {
        std::vector<int> ord, tord;
#pragma omp for schedule(dynamic, 256)
        for (int v = 0; v < N; v++) {
            const int lo = g.slot_ptr[v], hi = g.slot_ptr[v + 1];
            // new keys of message passing appended in sender order (:443-447)
            int next = 0;
            bool fresh = false;
            for (int k = lo; k < hi; k++) next = std::max(next, g.uts_rank[k] + 1);
            for (int k = lo; k < hi; k++)
                if (g.uts_fresh[k]) {
                    fresh = true;
                    if (g.uts_rank[k] < 0) g.uts_rank[k] = next++;
                }
            if (fresh) g.has_uts[v] = 1;
            // extrapolate stage tail (:554-566)
            if (g.has_uts[v]) {
                dict_order(g.uts_rank, lo, hi, ord);
                priors(g, ord, g.uts_prior);
                reweight(g, v, ord, p.reweight_threshold, err);
                priors(g, ord, g.uts_prior);
                reweight(g, v, ord, p.reweight_threshold, err);
            }
            degree(g, v);
            // update stage (remove_state_metadata.py:31-53)
            const bool u_ = g.has_uts[v];
            if (!u_ && !g.has_tse[v]) { err |= E_NO_DICT; continue; }
            int32_t* rk = u_ ? g.uts_rank : g.tse_rank;
            for (int k = lo; k < hi; k++)
                if (rk[k] >= 0 && !g.rev_edge[k]) rk[k] = -1;
            if (g.has_tse[v]) {
                dict_order(g.tse_rank, lo, hi, tord);
                priors(g, tord, g.tse_prior);
            }
            if (u_) {
                dict_order(g.uts_rank, lo, hi, ord);
                priors(g, ord, g.uts_prior);
                reweight(g, v, ord, p.reweight_threshold, err);
                // clustering on updated_track_states (clustering.py:181-373)
                cluster(g, uts_dict(g), v, ord, p, p.cluster_chi2, p.cluster_kl, err);
            }
            degree(g, v);                                                             // :324-327
            if (u_) {
                mixture_weights(g, v, ord, g.uts_mw, err);                            // :372
                priors(g, ord, g.uts_prior);                                          // :373
            }
        }
    }
    return err;
}

// clustering.cluster's body alone (clustering.py:181-373) on track_state_estimates
// (uts == 0) or updated_track_states (uts == 1): every node with that dict, the deferred
// deactivations, degree, mixture weights and priors of that dict.
uint32_t cr_cluster(const cr_graph* gp, const cr_params* pp, int uts, double chi2_thr, double kl_thr, int threads) {
    const cr_graph& g = *gp;
    const cr_params& p = *pp;
    if (threads > 0) omp_set_num_threads(threads);
    uint32_t err = 0;
    const Dict dc = uts ? uts_dict(g) : tse_dict(g);
    const uint8_t* has = uts ? g.has_uts : g.has_tse;
#pragma omp parallel reduction(| : err)
    {
        std::vector<int> ord;
#pragma omp for schedule(dynamic, 256)
        for (int v = 0; v < g.n_nodes; v++) {
            const int lo = g.slot_ptr[v], hi = g.slot_ptr[v + 1];
            if (has[v]) {
                dict_order(dc.rank, lo, hi, ord);
                cluster(g, dc, v, ord, p, chi2_thr, kl_thr, err);
            }
            degree(g, v);
            if (has[v]) {
                mixture_weights(g, v, ord, dc.mw, err);
                priors(g, ord, dc.prior);
            }
        }
    }
    return err;
}

}  // extern "C"
