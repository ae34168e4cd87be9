// mpcc_oracle.cpp — CPU restatement of the reference MPCC per-control-step solve.
//
// TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).  See oracle_api.h for the rules and
// for how this restatement is pinned.  Every function cites the reference file:line it restates
// (paths relative to the reference's cpp/ directory).  Written in plain C++17 with fixed-size
// arrays; no Eigen/RBDL/OSQP.  Deliberately scalar and layout-faithful: it mirrors the reference's
// data flow (AoS State/Input, dense QP layout) rather than the GPU engine's SoA/stage layout.
#include "oracle_api.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <sstream>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

// Robot dimensions: ORC_DOF = 7 is the reference's Franka Panda (config.h:29-38); ORC_DOF = 10 builds the
// same restatement for the Husky+Panda mobile manipulator (BASELINE configs[3]): planar base
// joints (x, y, theta) followed by the seven Panda joints.  State [q(DOF), s, vs], input [dq(DOF), dVs].
constexpr int DOF = ORC_DOF, NX = DOF + 2, NU = DOF + 1, NXU = NX + NU, NPC = 11, NLINK = 9;
constexpr int IS = DOF, IVS = DOF + 1, IDVS = DOF;  // indices of s, vs in the state and of dVs in the input
constexpr int NARM = 7, NBASE = DOF - NARM;       // the Panda joints follow the base joints
constexpr double INF = 1e30;                 // config.h:37
constexpr int N_SPLINE = 100;                // config.h:38
// RobotData layout (robot_data.h:13-31): pos 3, R 9, J 6 x DOF, mu, dmu DOF, d_self, dd_self DOF, obs_r,
// d_env 9, dd_env 9 x DOF (143 doubles for the Panda)
constexpr int R_POS = 0, R_ROT = 3, R_J = 12, R_MU = R_J + 6 * DOF, R_DMU = R_MU + 1, R_SEL = R_DMU + DOF,
              R_DSEL = R_SEL + 1, R_OBSR = R_DSEL + DOF, R_ENV = R_OBSR + 1, R_DENV = R_ENV + 9;
constexpr int REC = R_DENV + 9 * DOF;

enum Status {  // solver_interface.h:28-42
    SOLVED, MAX_ITER_EXCEEDED, QP_DualInfeasibleInaccurate, QP_PrimalInfeasibleInaccurate,
    QP_SolvedInaccurate, QP_MaxIterReached, QP_PrimalInfeasible, QP_DualInfeasible, Sigint,
    INVALID_SETTINGS, NAN_HESSIAN, NON_PD_HESSIAN
};

// ------------------------------------------------------------------------------------------------
// small dense helpers (row-major)
// ------------------------------------------------------------------------------------------------
static inline void mat3_mul(const double* A, const double* B, double* C) {
    double T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += A[3 * i + k] * B[3 * k + j];
            T[3 * i + j] = s;
        }
    std::memcpy(C, T, sizeof T);
}
static inline void mat3_mul_tn(const double* A, const double* B, double* C) {  // A^T B
    double T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += A[3 * k + i] * B[3 * k + j];
            T[3 * i + j] = s;
        }
    std::memcpy(C, T, sizeof T);
}
static inline void mat3_vec(const double* A, const double* v, double* o) {
    double t[3];
    for (int i = 0; i < 3; i++) t[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
    o[0] = t[0]; o[1] = t[1]; o[2] = t[2];
}
static inline void skew(const double* v, double* S) {  // cubic_spline_rot.cpp:25-35
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
static inline void invskew(const double* S, double* v) {  // cubic_spline_rot.cpp:37-42
    v[0] = S[7]; v[1] = S[2]; v[2] = S[3];
}

// 3x3 symmetric eigen-decomposition (cyclic Jacobi) on the LOWER triangle, as Eigen's
// SelfAdjointEigenSolver reads it.  Eigenvalues ascending.  Used only by LogMatrix's theta=pi
// branch; eigenvector signs follow this routine (parity unpinned in that branch).
static void sym_eig3(const double* Rin, double* w, double* V) {
    double A[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) A[3 * i + j] = (i >= j) ? Rin[3 * i + j] : Rin[3 * j + i];
    for (int i = 0; i < 9; i++) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; sweep++) {
        double off = std::fabs(A[1]) + std::fabs(A[2]) + std::fabs(A[5]);
        if (off < 1e-300) break;
        for (int p = 0; p < 2; p++)
            for (int q = p + 1; q < 3; q++) {
                double apq = A[3 * p + q];
                if (std::fabs(apq) < 1e-300) continue;
                double theta = (A[3 * q + q] - A[3 * p + p]) / (2 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < 3; k++) {
                    double akp = A[3 * k + p], akq = A[3 * k + q];
                    A[3 * k + p] = c * akp - s * akq;
                    A[3 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; k++) {
                    double apk = A[3 * p + k], aqk = A[3 * q + k];
                    A[3 * p + k] = c * apk - s * aqk;
                    A[3 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; k++) {
                    double vkp = V[3 * k + p], vkq = V[3 * k + q];
                    V[3 * k + p] = c * vkp - s * vkq;
                    V[3 * k + q] = s * vkp + c * vkq;
                }
            }
    }
    int idx[3] = {0, 1, 2};
    std::sort(idx, idx + 3, [&](int a, int b) { return A[4 * a] < A[4 * b]; });
    double Vs[9];
    for (int j = 0; j < 3; j++) {
        w[j] = A[4 * idx[j]];
        for (int i = 0; i < 3; i++) Vs[3 * i + j] = V[3 * i + idx[j]];
    }
    std::memcpy(V, Vs, sizeof Vs);
}

// LogMatrix — cubic_spline_rot.cpp:44-79 (quirk Q10)
static void log_matrix(const double* R, double* out) {
    double tr = R[0] + R[4] + R[8];
    for (int i = 0; i < 9; i++) out[i] = 0;
    if (std::fabs(tr + 1.0) < 1e-6) {
        double w[3], V[9];
        sym_eig3(R, w, V);
        for (int i = 0; i < 3; i++) {
            if (std::fabs(w[i] - 1.0) < 1e-4) {
                double v[3] = {V[i], V[3 + i], V[6 + i]};
                double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                for (int k = 0; k < 3; k++) v[k] /= n;
                double S[9];
                skew(v, S);
                for (int k = 0; k < 9; k++) out[k] = -S[k] * M_PI;
            }
        }
    } else if (std::fabs(tr - 3.0) < 1e-6) {
        // zero
    } else {
        double th = std::acos((tr - 1.0) / 2.0);
        double f = 1.0 / 2.0 * th / std::sin(th);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) out[3 * i + j] = f * (R[3 * i + j] - R[3 * j + i]);
    }
}

// ExpMatrix — cubic_spline_rot.cpp:81-95 (quirk Q11: integer 1/2 == 0)
static void exp_matrix(const double* sk, double* out) {
    double sym = 0, dg = 0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double t = sk[3 * j + i] + sk[3 * i + j];
            sym += t * t;
        }
    for (int i = 0; i < 3; i++) dg += sk[4 * i] * sk[4 * i];
    if (std::sqrt(sym) >= 1e-8 || std::sqrt(dg) >= 1e-8) {
        for (int i = 0; i < 9; i++) out[i] = 0;
        return;
    }
    double v[3];
    invskew(sk, v);
    double vn = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    double sk2[9];
    mat3_mul(sk, sk, sk2);
    if (vn <= 1e-8) {
        for (int i = 0; i < 9; i++) out[i] = (i % 4 == 0 ? 1.0 : 0.0) + std::cos(vn) * sk[i] + 0 * sk2[i];
        return;
    }
    double a = std::sin(vn) / vn, b = (1 - std::cos(vn)) / (vn * vn);
    for (int i = 0; i < 9; i++) out[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * sk[i] + b * sk2[i];
}

// ------------------------------------------------------------------------------------------------
// Splines — cubic_spline.cpp:25-246, cubic_spline_rot.cpp:97-259, arc_length_spline.cpp:33-379
// ------------------------------------------------------------------------------------------------
struct CubicSpline {
    std::vector<double> x, y, a, b, c, d;
    bool regular = false;
    double dx = 0;
    std::map<double, int> xmap;

    void gen(const std::vector<double>& xin, const std::vector<double>& yin, bool is_regular) {  // :162-183
        x = xin; y = yin; regular = is_regular;
        int n = (int)x.size();
        if (is_regular) dx = x[1] - x[0];
        else { dx = 0; xmap.clear(); for (int i = 0; i < n; i++) xmap[x[i]] = i; }
        // compSplineParams :65-124
        a = y; b.assign(n - 1, 0); c.assign(n, 0); d.assign(n - 1, 0);
        std::vector<double> mu(n - 1, 0), h(n - 1, 0), alpha(n - 1, 0), l(n, 0), z(n, 0);
        for (int i = 0; i < n - 1; i++) h[i] = x[i + 1] - x[i];
        for (int i = 1; i < n - 1; i++)
            alpha[i] = 3.0 / h[i] * (a[i + 1] - a[i]) - 3.0 / h[i - 1] * (a[i] - a[i - 1]);
        l[0] = 1.0; mu[0] = 0.0; z[0] = 0.0;
        for (int i = 1; i < n - 1; i++) {
            l[i] = 2.0 * (x[i + 1] - x[i - 1]) - h[i - 1] * mu[i - 1];
            mu[i] = h[i] / l[i];
            z[i] = (alpha[i] - h[i - 1] * z[i - 1]) / l[i];
        }
        l[n - 1] = 1.0; z[n - 1] = 0.0;
        c[n - 1] = 0.0;
        for (int i = n - 2; i >= 0; i--) {
            c[i] = z[i] - mu[i] * c[i + 1];
            b[i] = (a[i + 1] - a[i]) / h[i] - (h[i] * (c[i + 1] + 2.0 * c[i])) / 3.0;
            d[i] = (c[i + 1] - c[i]) / (3.0 * h[i]);
        }
    }
    int index(double xx) const {  // :126-153
        int n = (int)x.size();
        if (xx == x[n - 1]) return n - 1;
        if (regular) return int(std::floor(xx / dx));
        auto it = xmap.upper_bound(xx);
        if (it == xmap.end()) return -1;
        return it->second - 1;
    }
    double unwrap(double xx) const { return std::max(0., std::min(xx, x.back())); }
    double point(double xx) const {  // :185-207
        xx = unwrap(xx);
        int i = index(xx);
        double d1 = xx - x[i], d2 = d1 * d1, d3 = d1 * d2;
        if (i == (int)x.size() - 1) return y.back();
        return a[i] + b[i] * d1 + c[i] * d2 + d[i] * d3;
    }
    double deriv(double xx) const {  // :209-227
        xx = unwrap(xx);
        int i = index(xx);
        double d1 = xx - x[i], d2 = d1 * d1;
        if (i == (int)x.size() - 1) return 0.;
        return b[i] + 2.0 * c[i] * d1 + 3.0 * d[i] * d2;
    }
    double deriv2(double xx) const {  // :229-246
        xx = unwrap(xx);
        int i = index(xx);
        double d1 = xx - x[i];
        if (i == (int)x.size() - 1) return 2.0 * c[i];
        return 2.0 * c[i] + 6.0 * d[i] * d1;
    }
};

struct CubicSplineRot {
    std::vector<double> x, c, d;
    std::vector<std::array<double, 9>> R;
    bool regular = false;
    double dx = 0;
    std::map<double, int> xmap;
    void gen(const std::vector<double>& xin, const std::vector<std::array<double, 9>>& Rin, bool is_regular) {
        x = xin; R = Rin; regular = is_regular;
        int n = (int)x.size();
        if (is_regular) dx = x[1] - x[0];
        else { dx = 0; xmap.clear(); for (int i = 0; i < n; i++) xmap[x[i]] = i; }
        c.assign(n - 1, 0); d.assign(n - 1, 0);  // compSplineRotParams :137-155
        for (int i = 0; i < n - 1; i++) {
            c[i] = 3.0 / std::pow(x[i + 1] - x[i], 2);
            d[i] = -2.0 / std::pow(x[i + 1] - x[i], 3);
        }
    }
    int index(double xx) const {
        int n = (int)x.size();
        if (xx == x[n - 1]) return n - 1;
        if (regular) return int(std::floor(xx / dx));
        auto it = xmap.upper_bound(xx);
        if (it == xmap.end()) return -1;
        return it->second - 1;
    }
    double unwrap(double xx) const { return std::max(0., std::min(xx, x.back())); }
    void point(double xx, double* out) const {  // :216-238
        xx = unwrap(xx);
        int i = index(xx);
        if (i == (int)x.size() - 1) { std::memcpy(out, R.back().data(), 72); return; }
        double d1 = xx - x[i], d2 = d1 * d1, d3 = d1 * d2;
        double RtR[9], L[9], E[9];
        mat3_mul_tn(R[i].data(), R[i + 1].data(), RtR);
        log_matrix(RtR, L);
        double f = c[i] * d2 + d[i] * d3;
        for (int k = 0; k < 9; k++) L[k] *= f;
        exp_matrix(L, E);
        mat3_mul(R[i].data(), E, out);
    }
    void deriv(double xx, double* out) const {  // :240-259
        xx = unwrap(xx);
        int i = index(xx);
        if (i == (int)x.size() - 1) { out[0] = out[1] = out[2] = 0; return; }
        double d1 = xx - x[i], d2 = d1 * d1;
        double RtR[9], L[9], v[3];
        mat3_mul_tn(R[i].data(), R[i + 1].data(), RtR);
        log_matrix(RtR, L);
        invskew(L, v);
        double f = 2.0 * c[i] * d1 + 3.0 * d[i] * d2;
        for (int k = 0; k < 3; k++) out[k] = v[k] * f;
    }
};

struct ArcLengthSpline {
    std::vector<double> s, X, Y, Z;
    std::vector<std::array<double, 9>> R;
    CubicSpline sx, sy, sz;
    CubicSplineRot sr;
    double proj_max_dist = 0.03;
    bool set = false;

    static std::vector<double> arc_length(const std::vector<double>& X, const std::vector<double>& Y,
                                          const std::vector<double>& Z) {  // :66-87
        int n = (int)X.size();
        std::vector<double> s(n, 0.0);
        for (int i = 0; i < n - 1; i++) {
            double dx = X[i + 1] - X[i], dy = Y[i + 1] - Y[i], dz = Z[i + 1] - Z[i];
            s[i + 1] = s[i] + std::sqrt(dx * dx + dy * dy + dz * dz);
        }
        return s;
    }
    static std::vector<double> linspaced(int n, double lo, double hi) {  // Eigen LinSpaced (no flip for lo=0)
        std::vector<double> v(n);
        double step = (hi - lo) / double(n - 1);
        bool flip = std::fabs(hi) < std::fabs(lo);
        for (int i = 0; i < n; i++) {
            if (flip) v[i] = (i == 0) ? lo : hi - double(n - 1 - i) * step;
            else v[i] = (i == n - 1) ? hi : lo + double(i) * step;
        }
        return v;
    }
    void resample(const CubicSpline& fx, const CubicSpline& fy, const CubicSpline& fz, const CubicSplineRot& fr,
                  double total, std::vector<double>& rs, std::vector<double>& rx, std::vector<double>& ry,
                  std::vector<double>& rz, std::vector<std::array<double, 9>>& rR) const {  // :89-119
        rs = linspaced(N_SPLINE, 0, total);
        rx.assign(N_SPLINE, 0); ry.assign(N_SPLINE, 0); rz.assign(N_SPLINE, 0); rR.assign(N_SPLINE, {});
        for (int i = 0; i < N_SPLINE; i++) {
            rx[i] = fx.point(rs[i]);
            ry[i] = fy.point(rs[i]);
            rz[i] = fz.point(rs[i]);
            fr.point(rs[i], rR[i].data());
        }
    }
    void fit(const std::vector<double>& X0, const std::vector<double>& Y0, const std::vector<double>& Z0,
             const std::vector<std::array<double, 9>>& R0) {  // fitSpline :213-253
        std::vector<double> sa = arc_length(X0, Y0, Z0);
        double total = sa.back();
        CubicSpline f1x, f1y, f1z; CubicSplineRot f1r;
        f1x.gen(sa, X0, false); f1y.gen(sa, Y0, false); f1z.gen(sa, Z0, false); f1r.gen(sa, R0, false);
        std::vector<double> s1, x1, y1, z1; std::vector<std::array<double, 9>> R1;
        resample(f1x, f1y, f1z, f1r, total, s1, x1, y1, z1, R1);
        sa = arc_length(x1, y1, z1);
        total = sa.back();
        CubicSpline f2x, f2y, f2z; CubicSplineRot f2r;
        f2x.gen(sa, x1, false); f2y.gen(sa, y1, false); f2z.gen(sa, z1, false); f2r.gen(sa, R1, false);
        std::vector<double> s2, x2, y2, z2; std::vector<std::array<double, 9>> R2;
        resample(f2x, f2y, f2z, f2r, total, s2, x2, y2, z2, R2);
        s = s2; X = x2; Y = y2; Z = z2; R = R2;  // setRegularData
        sx.gen(s, X, true); sy.gen(s, Y, true); sz.gen(s, Z, true); sr.gen(s, R, true);
        set = true;
    }
    double length() const { return s.back(); }
    double unwrap(double x) const { return std::max(0., std::min(x, length())); }
    void pos(double t, double* o) const { o[0] = sx.point(t); o[1] = sy.point(t); o[2] = sz.point(t); }
    void dpos(double t, double* o) const { o[0] = sx.deriv(t); o[1] = sy.deriv(t); o[2] = sz.deriv(t); }
    void ddpos(double t, double* o) const { o[0] = sx.deriv2(t); o[1] = sy.deriv2(t); o[2] = sz.deriv2(t); }
    void rot(double t, double* o) const { sr.point(t, o); }
    void drot(double t, double* o) const { sr.deriv(t, o); }

    // projectOnSpline — arc_length_spline.cpp:318-379 (quirk Q12 in the far branch)
    double project(double s_guess, const double* ee) const {
        double pp[3];
        pos(s_guess, pp);
        double s_opt = s_guess;
        double dist = std::sqrt((ee[0] - pp[0]) * (ee[0] - pp[0]) + (ee[1] - pp[1]) * (ee[1] - pp[1]) +
                                (ee[2] - pp[2]) * (ee[2] - pp[2]));
        if (dist >= proj_max_dist) {
            int n = (int)s.size();
            std::vector<double> d2(n), filt(n);
            bool any = false;
            for (int i = 0; i < n; i++) {
                double dx = X[i] - ee[0], dy = Y[i] - ee[1], dz = Z[i] - ee[2];
                d2[i] = dx * dx + dy * dy + dz * dz;
                bool valid = std::fabs(s[i] - s_guess) <= proj_max_dist;
                any |= valid;
                double m = valid ? 1.0 : 0.0;
                filt[i] = d2[i] * m + (1.0 - m) * std::numeric_limits<double>::infinity();  // NaN for valid
            }
            // Eigen minCoeff, scalar semantics: first index, replaced only by strictly smaller.
            int mi = 0;
            double mv = filt[0];
            for (int i = 1; i < n; i++)
                if (filt[i] < mv) { mv = filt[i]; mi = i; }
            if (!any) {
                int mj = (int)(std::min_element(d2.begin(), d2.end()) - d2.begin());
                s_opt = s[mj];
            } else {
                s_opt = s[mi];
            }
        }
        if (s_opt >= s.back()) return s.back();
        double s_old = s_opt;
        for (int i = 0; i < 20; i++) {
            double p[3], dp[3], ddp[3];
            pos(s_opt, p); dpos(s_opt, dp); ddpos(s_opt, ddp);
            double df[3] = {p[0] - ee[0], p[1] - ee[1], p[2] - ee[2]};
            double jac = 2.0 * df[0] * dp[0] + 2.0 * df[1] * dp[1] + 2.0 * df[2] * dp[2];
            double hes = 2.0 * dp[0] * dp[0] + 2.0 * df[0] * ddp[0] + 2.0 * dp[1] * dp[1] + 2.0 * df[1] * ddp[1] +
                         2.0 * dp[2] * dp[2] + 2.0 * df[2] * ddp[2];
            s_opt -= jac / hes;
            s_opt = unwrap(s_opt);
            if (std::fabs(s_old - s_opt) <= 1e-5) return s_opt;
            s_old = s_opt;
        }
        return s_guess;
    }
};

// ------------------------------------------------------------------------------------------------
// Robot kinematics — RBDL restatement of robot_model.cpp:68-319 (Panda chain) and :366-450
// RBDL SpatialTransform(E, r): E maps parent to child coordinates, so the child frame's rotation
// in the parent is E^T; a revolute-z joint contributes Rz(q).
// ------------------------------------------------------------------------------------------------
static const double JOINT_E[9][9] = {
    {1, 0, 0, 0, 1, 0, 0, 0, 1},                 // [0] world->link0 (base rotation = I)
    {1, 0, 0, 0, 1, 0, 0, 0, 1},                 // [1] link0->link1   :189-193
    {1, 0, 0, 0, 0, -1, 0, 1, 0},                // [2] link1->link2   :196-200
    {1, 0, 0, 0, 0, 1, 0, -1, 0},                // [3]                :203-207
    {1, 0, 0, 0, 0, 1, 0, -1, 0},                // [4]                :210-214
    {1, 0, 0, 0, 0, -1, 0, 1, 0},                // [5]                :217-221
    {1, 0, 0, 0, 0, 1, 0, -1, 0},                // [6]                :224-228
    {1, 0, 0, 0, 0, 1, 0, -1, 0},                // [7]                :231-235
    {0.707107, -0.707107, 0., 0.707107, 0.707107, 0., 0., 0., 1.},  // [8] link7->hand :238-242 (Q19)
};
static const double JOINT_R[9][3] = {
    {0, 0, 0}, {0, 0, 0.333}, {0, 0, 0}, {0, -0.316, 0}, {0.0825, 0, 0},
    {-0.0825, 0.384, 0}, {0, 0, 0}, {0.088, 0, 0}, {0, 0, 0.107}};  // :171-179
static const double TCP_R[3] = {0, 0, 0.1034};                      // :182

// FK + geometric Jacobian of panda_hand_tcp for the 7 Panda joints.  J 6x7: rows 0-2 = Jv, 3-5 = Jw
// (robot_model.cpp:372-375)
static void fk_arm(const double* q, double* pos, double* Rout, double* J) {
    double Rc[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, pc[3] = {0, 0, 0};
    double z[7][3], o[7][3];
    for (int i = 1; i <= 7; i++) {
        double t[3];
        mat3_vec(Rc, JOINT_R[i], t);
        pc[0] += t[0]; pc[1] += t[1]; pc[2] += t[2];
        double Et[9], Rt[9];
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) Et[3 * a + b] = JOINT_E[i][3 * b + a];
        mat3_mul(Rc, Et, Rt);
        z[i - 1][0] = Rt[2]; z[i - 1][1] = Rt[5]; z[i - 1][2] = Rt[8];
        o[i - 1][0] = pc[0]; o[i - 1][1] = pc[1]; o[i - 1][2] = pc[2];
        double c = std::cos(q[i - 1]), s = std::sin(q[i - 1]);
        double Rz[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
        mat3_mul(Rt, Rz, Rc);
    }
    {   // hand (fixed)
        double t[3];
        mat3_vec(Rc, JOINT_R[8], t);
        pc[0] += t[0]; pc[1] += t[1]; pc[2] += t[2];
        double Et[9], Rt[9];
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) Et[3 * a + b] = JOINT_E[8][3 * b + a];
        mat3_mul(Rc, Et, Rt);
        std::memcpy(Rc, Rt, sizeof Rt);
        mat3_vec(Rc, TCP_R, t);  // tcp (fixed, identity rotation)
        pc[0] += t[0]; pc[1] += t[1]; pc[2] += t[2];
    }
    if (pos) { pos[0] = pc[0]; pos[1] = pc[1]; pos[2] = pc[2]; }
    if (Rout) std::memcpy(Rout, Rc, 72);
    if (J) {
        for (int i = 0; i < 7; i++) {
            double r[3] = {pc[0] - o[i][0], pc[1] - o[i][1], pc[2] - o[i][2]};
            J[0 * 7 + i] = z[i][1] * r[2] - z[i][2] * r[1];
            J[1 * 7 + i] = z[i][2] * r[0] - z[i][0] * r[2];
            J[2 * 7 + i] = z[i][0] * r[1] - z[i][1] * r[0];
            J[3 * 7 + i] = z[i][0];
            J[4 * 7 + i] = z[i][1];
            J[5 * 7 + i] = z[i][2];
        }
    }
}

// Frame f of RobotModel::getPosition/getOrientation/getJacobian(frame_id) (robot_model.cpp:354-398; body_id_
// :310-319): 1 = panda_link0, 2..8 = panda_link1..7 (RBDL body origin after joint f-1), 9 = panda_hand_tcp.
// CalcPointJacobian6D at the body origin: joints after the frame give zero columns.
static void fk_frame(const double* q, int frame, double* pos, double* Rout, double* J) {
    if (frame >= 9) { fk_arm(q, pos, Rout, J); return; }
    double Rc[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, pc[3] = {0, 0, 0};
    double z[7][3], o[7][3];
    const int nj = frame - 1;
    for (int i = 1; i <= nj; i++) {
        double t[3];
        mat3_vec(Rc, JOINT_R[i], t);
        pc[0] += t[0]; pc[1] += t[1]; pc[2] += t[2];
        double Et[9], Rt[9];
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) Et[3 * a + b] = JOINT_E[i][3 * b + a];
        mat3_mul(Rc, Et, Rt);
        z[i - 1][0] = Rt[2]; z[i - 1][1] = Rt[5]; z[i - 1][2] = Rt[8];
        o[i - 1][0] = pc[0]; o[i - 1][1] = pc[1]; o[i - 1][2] = pc[2];
        double c = std::cos(q[i - 1]), s = std::sin(q[i - 1]);
        double Rz[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
        mat3_mul(Rt, Rz, Rc);
    }
    if (pos) { pos[0] = pc[0]; pos[1] = pc[1]; pos[2] = pc[2]; }
    if (Rout) std::memcpy(Rout, Rc, 72);
    if (J) {
        for (int i = 0; i < 7; i++) {
            if (i >= nj) {
                for (int a = 0; a < 6; a++) J[a * 7 + i] = 0.0;
                continue;
            }
            double r[3] = {pc[0] - o[i][0], pc[1] - o[i][1], pc[2] - o[i][2]};
            J[0 * 7 + i] = z[i][1] * r[2] - z[i][2] * r[1];
            J[1 * 7 + i] = z[i][2] * r[0] - z[i][0] * r[2];
            J[2 * 7 + i] = z[i][0] * r[1] - z[i][1] * r[0];
            J[3 * 7 + i] = z[i][0];
            J[4 * 7 + i] = z[i][1];
            J[5 * 7 + i] = z[i][2];
        }
    }
}

// det via partial-pivot LU (Eigen MatrixXd::determinant for n>4 -> PartialPivLU)
static double det_lu(double* A, int n) {
    double det = 1.0;
    for (int k = 0; k < n; k++) {
        int p = k;
        double mx = std::fabs(A[k * n + k]);
        for (int i = k + 1; i < n; i++)
            if (std::fabs(A[i * n + k]) > mx) { mx = std::fabs(A[i * n + k]); p = i; }
        if (p != k) {
            for (int j = 0; j < n; j++) std::swap(A[k * n + j], A[p * n + j]);
            det = -det;
        }
        double piv = A[k * n + k];
        det *= piv;
        if (piv == 0.0) continue;
        for (int i = k + 1; i < n; i++) {
            double f = A[i * n + k] / piv;
            for (int j = k + 1; j < n; j++) A[i * n + j] -= f * A[k * n + j];
        }
    }
    return det;
}

// Mobile base of the Husky+Panda (ORC_DOF = 10; robot_model.cpp:321-352 setHusky: prismatic x, prismatic y,
// revolute theta about z, then the fixed husky_base).  The reference never mounts the Panda on it
// (setRobot appends only setPanda, :58-66); this build mounts panda_link0 at MOBILE_MOUNT in the base
// frame with identity rotation (setPanda(base_id, base_position, I), :68) — our definition, DESIGN.md §11.
static const double MOBILE_MOUNT[3] = {0.0, 0.0, 0.35};

// FK + geometric Jacobian of panda_hand_tcp for the robot of this build: J 6 x DOF, rows Jv; Jw.  With the
// base: p = [x, y, 0] + Rz(th) (mount + p_arm), R = Rz(th) R_arm; base columns e_x, e_y and
// (e_z x (p - [x, y, 0]), e_z); arm columns rotated by Rz(th) — CalcPointJacobian6D of that chain.
static void fk(const double* q, double* pos, double* Rout, double* J) {
    if (NBASE == 0) { fk_arm(q, pos, Rout, J); return; }
    double pa[3], Ra[9], Ja[42];
    fk_arm(q + NBASE, pa, Ra, J ? Ja : nullptr);
    const double c = std::cos(q[2]), sn = std::sin(q[2]);
    const double Rz[9] = {c, -sn, 0, sn, c, 0, 0, 0, 1};
    const double pl[3] = {MOBILE_MOUNT[0] + pa[0], MOBILE_MOUNT[1] + pa[1], MOBILE_MOUNT[2] + pa[2]};
    double pw[3];
    mat3_vec(Rz, pl, pw);
    const double p3[3] = {q[0] + pw[0], q[1] + pw[1], 0.0 + pw[2]};
    if (pos) { pos[0] = p3[0]; pos[1] = p3[1]; pos[2] = p3[2]; }
    if (Rout) mat3_mul(Rz, Ra, Rout);
    if (J) {
        for (int i = 0; i < 6 * DOF; i++) J[i] = 0.0;
        J[0 * DOF + 0] = 1.0;                      // x
        J[1 * DOF + 1] = 1.0;                      // y
        J[0 * DOF + 2] = -(p3[1] - q[1]);          // theta: e_z x (p - base)
        J[1 * DOF + 2] = p3[0] - q[0];
        J[5 * DOF + 2] = 1.0;
        for (int j = 0; j < NARM; j++) {
            const double v[3] = {Ja[0 * 7 + j], Ja[1 * 7 + j], Ja[2 * 7 + j]}, w[3] = {Ja[3 * 7 + j], Ja[4 * 7 + j], Ja[5 * 7 + j]};
            double rv[3], rw[3];
            mat3_vec(Rz, v, rv);
            mat3_vec(Rz, w, rw);
            for (int a = 0; a < 3; a++) { J[a * DOF + NBASE + j] = rv[a]; J[(3 + a) * DOF + NBASE + j] = rw[a]; }
        }
    }
}

// sqrt(det(J J^T)) of a 6 x DOF Jacobian — robot_model.cpp:431-435
static double manip_of_J(const double* J) {
    double JJ[36];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) {
            double s = 0;
            for (int k = 0; k < DOF; k++) s += J[DOF * i + k] * J[DOF * j + k];
            JJ[6 * i + j] = s;
        }
    return std::sqrt(det_lu(JJ, 6));
}
// Manipulability — robot_model.cpp:431-435
static double manipulability(const double* q) {
    double J[6 * DOF];
    fk(q, nullptr, nullptr, J);
    return manip_of_J(J);
}
// dManipulability — robot_model.cpp:437-450 (central FD, delta = 1e-4)
static void dmanipulability(const double* q, double* d) {
    const double delta = 1e-4;
    for (int i = 0; i < DOF; i++) {
        double qp[DOF], qm[DOF];
        for (int k = 0; k < DOF; k++) { qp[k] = q[k] + (k == i ? delta : 0.0); qm[k] = q[k] - (k == i ? delta : 0.0); }
        double m1 = manipulability(qp), m2 = manipulability(qm);
        d[i] = (m1 - m2) / (2 * delta);
    }
}

// ------------------------------------------------------------------------------------------------
// NeRF MLP with forward-mode input Jacobian — SelfCollisionModel.cpp:140-250 (Env identical)
// Every dot product is an fma chain in ascending k (s = fma(W[i][k], x[k], s)), bitwise the
// accumulation of v_mfma_f64_16x16x4f64 k-step by k-step (tools/probes/mfma_f64_probe.hip); the
// reference's own order is Eigen-internal, so this is the restatement's choice.
// ------------------------------------------------------------------------------------------------
struct MLP {
    int n_in = 0, n_out = 0;
    std::vector<int> dims;                 // [3*n_in, hidden..., n_out]
    std::vector<std::vector<double>> W, b; // W[l] rows=dims[l+1], cols=dims[l]
    bool ok = false;

    bool load(const std::string& dir, int nin, int nout, const std::vector<int>& hidden) {
        n_in = nin; n_out = nout;
        dims.clear(); dims.push_back(3 * nin);
        for (int h : hidden) dims.push_back(h);
        dims.push_back(nout);
        W.assign(dims.size() - 1, {}); b.assign(dims.size() - 1, {});
        for (size_t l = 0; l + 1 < dims.size(); l++) {
            size_t nw = (size_t)dims[l + 1] * dims[l], nb = dims[l + 1];
            W[l].resize(nw); b[l].resize(nb);
            std::ifstream fw(dir + "/weight_" + std::to_string(l) + ".f64", std::ios::binary);
            std::ifstream fb(dir + "/bias_" + std::to_string(l) + ".f64", std::ios::binary);
            if (!fw || !fb) return false;
            fw.read((char*)W[l].data(), nw * 8);
            fb.read((char*)b[l].data(), nb * 8);
            if (!fw || !fb) return false;
        }
        ok = true;
        return true;
    }
    // out [n_out], jac [n_out * n_in] row-major
    void eval(const double* in, double* out, double* jac) const {
        int L = (int)dims.size() - 1;
        int n0 = dims[0];
        std::vector<double> nerf(n0);
        for (int i = 0; i < n_in; i++) {
            nerf[i] = in[i];
            nerf[n_in + i] = std::sin(in[i]);
            nerf[2 * n_in + i] = std::cos(in[i]);
        }
        std::vector<double> hid, hprev;
        std::vector<double> temp;  // current derivative (rows = layer width, cols = n_in)
        for (int l = 0; l < L; l++) {
            int r = dims[l + 1], c = dims[l];
            const std::vector<double>& x = (l == 0) ? nerf : hprev;
            hid.assign(r, 0.0);
            for (int i = 0; i < r; i++) {
                double s = 0;
                for (int k = 0; k < c; k++) s = std::fma(W[l][(size_t)i * c + k], x[k], s);
                hid[i] = s + b[l][i];
            }
            if (l == L - 1) {  // output layer :194-203
                for (int i = 0; i < r; i++) out[i] = hid[i];
                for (int i = 0; i < r; i++)
                    for (int j = 0; j < n_in; j++) {
                        double s = 0;
                        for (int k = 0; k < c; k++) s = std::fma(W[l][(size_t)i * c + k], temp[(size_t)k * n_in + j], s);
                        jac[i * n_in + j] = s;
                    }
                break;
            }
            // hidden_derivative.row(h) = ReLU'(h) * W.row(h); then chain
            std::vector<double> nt((size_t)r * n_in, 0.0);
            if (l == 0) {
                // temp = hd0 * nerf_jac, nerf_jac = [I; diag(cos x); diag(-sin x)]  :177-188
                // (the fma chain over the full nerf_jac column: its zero entries leave the sum unchanged)
                for (int i = 0; i < r; i++) {
                    const bool g = hid[i] > 0;
                    for (int j = 0; j < n_in; j++) {
                        const double* w = &W[0][(size_t)i * c];
                        double s = std::fma(w[j], 1.0, 0.0);
                        s = std::fma(w[n_in + j], std::cos(in[j]), s);
                        s = std::fma(w[2 * n_in + j], -std::sin(in[j]), s);
                        nt[(size_t)i * n_in + j] = g ? s : 0.0;
                    }
                }
            } else {
                for (int i = 0; i < r; i++) {
                    const bool g = hid[i] > 0;
                    for (int j = 0; j < n_in; j++) {
                        double s = 0;
                        for (int k = 0; k < c; k++) s = std::fma(W[l][(size_t)i * c + k], temp[(size_t)k * n_in + j], s);
                        nt[(size_t)i * n_in + j] = g ? s : 0.0;
                    }
                }
            }
            for (int i = 0; i < r; i++) hid[i] = std::max(0.0, hid[i]);
            temp.swap(nt);
            hprev = hid;
        }
    }
};

// ------------------------------------------------------------------------------------------------
// Oracle state
// ------------------------------------------------------------------------------------------------
struct Oracle {
    OracleParams p;
    OracleOptions opt;
    MLP self_nn, env_nn;
    ArcLengthSpline track;
    // discretized LTI model (model.cpp:47-91): A = I + Ts e_s e_vs^T, B closed form of expm
    double A[NX * NX], B[NX * NU];

    void set_params(const OracleParams* pp) {
        p = *pp;
        track.proj_max_dist = p.proj_max_dist;
        for (int i = 0; i < NX * NX; i++) A[i] = (i % (NX + 1) == 0) ? 1.0 : 0.0;
        for (int i = 0; i < NX * NU; i++) B[i] = 0.0;
        A[IS * NX + IVS] = p.Ts;                       // s <- vs
        for (int j = 0; j < DOF; j++) B[j * NU + j] = p.Ts;  // q <- dq
        B[IS * NU + IDVS] = p.Ts * p.Ts / 2.0;         // s <- dVs
        B[IVS * NU + IDVS] = p.Ts;                     // vs <- dVs
    }
    int N() const { return p.N; }
    int nvar() const { return (N() + 1) * NX + N() * NU; }
    int nconstr() const { return (N() + 1) * NX + ((N() + 1) * NX + N() * NU + N() * NU) + (N() + 1) * NPC; }
};

static void robot_record(const Oracle& o, const double* q, const double* obs, double obs_r, double* rec) {
    // RobotData::update (robot_data.h:55-71)
    for (int i = 0; i < REC; i++) rec[i] = 0;
    fk(q, rec + R_POS, rec + R_ROT, rec + R_J);
    rec[R_MU] = manipulability(q);
    dmanipulability(q, rec + R_DMU);
    // The Panda-trained networks see the arm: joints q[NBASE..] (self: the base moves no arm link relative to
    // another, so its columns are zero) and the obstacle in the panda_link0 frame (env, below).
    const double* qa = q + NBASE;
    if ((o.p.constraint_mask & 1) && o.self_nn.ok) {
        o.self_nn.eval(qa, rec + R_SEL, rec + R_DSEL + NBASE);
    } else {
        rec[R_SEL] = std::numeric_limits<double>::infinity();  // masked: no self-collision data
    }
    // RobotData::updateEnv (robot_data.h:74-88)
    rec[R_OBSR] = obs_r;
    if ((o.p.constraint_mask & 4) && o.env_nn.ok) {
        double oa[3] = {obs[0], obs[1], obs[2]};
        double dO[3][3] = {};  // d o_arm / d (x, y, theta)
        if (NBASE > 0) {       // o_arm = Rz(th)^T (obs - [x, y, 0]) - mount
            const double c = std::cos(q[2]), sn = std::sin(q[2]);
            const double dx = obs[0] - q[0], dy = obs[1] - q[1], dz = obs[2];
            oa[0] = (c * dx + sn * dy) - MOBILE_MOUNT[0];
            oa[1] = (-sn * dx + c * dy) - MOBILE_MOUNT[1];
            oa[2] = dz - MOBILE_MOUNT[2];
            dO[0][0] = -c;  dO[1][0] = sn;  dO[2][0] = 0.0;   // d/dx
            dO[0][1] = -sn; dO[1][1] = -c;  dO[2][1] = 0.0;   // d/dy
            dO[0][2] = -sn * dx + c * dy; dO[1][2] = -c * dx - sn * dy; dO[2][2] = 0.0;  // d/dtheta
        }
        double in[10] = {qa[0], qa[1], qa[2], qa[3], qa[4], qa[5], qa[6], oa[0], oa[1], oa[2]};
        double out[9], jac[90];
        o.env_nn.eval(in, out, jac);
        for (int i = 0; i < 9; i++) {
            rec[R_ENV + i] = out[i];
            for (int j = 0; j < 7; j++) rec[R_DENV + DOF * i + NBASE + j] = jac[10 * i + j];  // 9x7 arm block (Q17)
            for (int b = 0; b < NBASE; b++)
                rec[R_DENV + DOF * i + b] = jac[10 * i + 7] * dO[0][b] + jac[10 * i + 8] * dO[1][b] + jac[10 * i + 9] * dO[2][b];
        }
    } else {
        for (int i = 0; i < 9; i++) rec[R_ENV + i] = std::numeric_limits<double>::infinity();
    }
}

// ------------------------------------------------------------------------------------------------
// Cost — cost.cpp:36-357
// ------------------------------------------------------------------------------------------------
static double cubic_blend(double x, double x0, double xf, double y0, double yf) {  // :36-43
    double t = (x - x0) / (xf - x0);
    double t2 = std::pow(t, 2), t3 = std::pow(t, 3);
    return y0 + (yf - y0) * (3 * t2 - 2 * t3);
}

struct CostOut {
    double obj;
    double fx[NX], fu[NU], fxx[NX * NX], fuu[NU * NU], fxu[NX * NU];
};

static void stage_cost(const Oracle& o, const double* x, const double* u, const double* rec, int k, bool want_grad,
                       CostOut& out) {
    const OracleParams& p = o.p;
    const int N = p.N;
    // weight schedule :293-308
    double ratio = std::min(rec[R_SEL] / (p.cost_tol_selcol * 2.0), rec[R_MU] / (p.cost_tol_sing * 2.0));
    double qc, ql, qo;
    if (ratio <= 1.0) {
        qc = p.q_c * cubic_blend(ratio, 0.5, 1.0, p.q_c_red_ratio, 1.0);
        ql = p.q_l * cubic_blend(ratio, 0.5, 1.0, p.q_l_inc_ratio, 1.0);
        qo = p.q_ori * cubic_blend(ratio, 0.5, 1.0, p.q_ori_red_ratio, 1.0);
    } else {
        qc = p.q_c; ql = p.q_l; qo = p.q_ori;
    }
    const double s = x[IS], vs = x[IVS];
    // getRefPoint :46-68 (Q2: ddz_ref = ddpos(1))
    double pr[3], dpr[3], ddp[3];
    o.track.pos(s, pr);
    o.track.dpos(s, dpr);
    o.track.ddpos(s, ddp);
    double ddr[3] = {ddp[0], ddp[1], ddp[1]};

    // ---- contouring + lag + vs (getContouringCost :119-162, getErrorInfo :82-117)
    const double* pos = rec + R_POS;
    double et[3] = {pos[0] - pr[0], pos[1] - pr[1], pos[2] - pr[2]};
    const double* T = dpr;
    double Te = T[0] * et[0] + T[1] * et[1] + T[2] * et[2];
    double el[3] = {Te * T[0], Te * T[1], Te * T[2]};
    double ec[3] = {et[0] - el[0], et[1] - el[1], et[2] - el[2]};
    // d_total (3x9): q cols = Jv, s col = -T
    double dt[3][NX] = {};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < DOF; j++) dt[i][j] = rec[R_J + DOF * i + j];
        dt[i][IS] = -T[i];
    }
    double nel = std::sqrt(el[0] * el[0] + el[1] * el[1] + el[2] * el[2]);
    // d_lag = (T T^T) d_total + (T e^T + |e_l| I) d_T, d_T only in s col = ddr  (Q3)
    double dl[3][NX], dc[3][NX];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < NX; j++) {
            double a = T[i] * T[0] * dt[0][j] + T[i] * T[1] * dt[1][j] + T[i] * T[2] * dt[2][j];
            double b = 0;
            if (j == IS) {
                for (int m = 0; m < 3; m++) b += (T[i] * et[m] + (i == m ? nel : 0.0)) * ddr[m];
            }
            dl[i][j] = a + b;
            dc[i][j] = dt[i][j] - dl[i][j];
        }
    double CC0 = (k < N) ? qc : p.q_c_N_mult * qc;
    double CC1 = ql;
    double s_max = o.track.length();
    double des = (s < s_max * p.deacc_ratio) ? p.desired_ee_velocity
                                             : -p.desired_ee_velocity / (s_max * p.deacc_ratio) * (s - s_max);
    double obj_c = CC0 * (ec[0] * ec[0] + ec[1] * ec[1] + ec[2] * ec[2]) +
                   CC1 * (el[0] * el[0] + el[1] * el[1] + el[2] * el[2]) + p.q_vs * std::pow(vs - des, 2);

    // ---- heading (getHeadingCost :164-207)
    double Rref[9], dRref[3];
    o.track.rot(s, Rref);
    o.track.drot(s, dRref);
    const double* Rcur = rec + R_ROT;
    double Rbar[9], Lm[9], w[3];
    mat3_mul_tn(Rref, Rcur, Rbar);
    log_matrix(Rbar, Lm);
    invskew(Lm, w);
    double wn2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double obj_h = qo * wn2;

    // ---- input (getInputCost :209-270)
    double obj_i = 0;
    if (k != N) {
        double dq2 = 0;
        for (int j = 0; j < DOF; j++) dq2 += u[j] * u[j];
        obj_i = p.r_dq * dq2 + p.r_dVs * std::pow(u[IDVS], 2);
    }
    // ---- singularity (:272-288)
    double obj_s = -p.q_sing * rec[R_MU];
    out.obj = obj_c + obj_h + obj_i + obj_s;
    if (!want_grad) return;

    // gradients / Hessians
    double gxc[NX] = {}, hxc[NX * NX] = {};
    for (int j = 0; j < NX; j++) {
        double s1 = 0, s2 = 0;
        for (int i = 0; i < 3; i++) { s1 += dc[i][j] * ec[i]; s2 += dl[i][j] * el[i]; }
        gxc[j] = 2.0 * CC0 * s1 + 2.0 * CC1 * s2;
    }
    gxc[IVS] += 2.0 * p.q_vs * (vs - des);
    for (int a = 0; a < NX; a++)
        for (int b = 0; b < NX; b++) {
            double s1 = 0, s2 = 0;
            for (int i = 0; i < 3; i++) { s1 += dc[i][a] * dc[i][b]; s2 += dl[i][a] * dl[i][b]; }
            hxc[a * NX + b] = 2.0 * CC0 * s1 + 2.0 * CC1 * s2;
        }
    hxc[IVS * NX + IVS] += 2.0 * p.q_vs;

    // heading linearization :183-205 (Q23: '+' sign in the J_r^{-1} coefficient, as written)
    double Jri[9];
    double wn = std::sqrt(wn2);
    if (wn < 1e-8) {
        for (int i = 0; i < 9; i++) Jri[i] = (i % 4 == 0) ? 1.0 : 0.0;
    } else {
        double S[9], S2[9];
        skew(w, S);
        mat3_mul(S, S, S2);
        double coef = 1. / wn2 + (1. + std::cos(wn)) / (2. * wn * std::sin(wn));
        for (int i = 0; i < 9; i++) Jri[i] = ((i % 4 == 0) ? 1.0 : 0.0) + 1. / 2. * S[i] + coef * S2[i];
    }
    double JRt[9];  // J_r_inv * cur_R^T
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double sacc = 0;
            for (int m = 0; m < 3; m++) sacc += Jri[3 * i + m] * Rcur[3 * j + m];
            JRt[3 * i + j] = sacc;
        }
    double dL[3][NX] = {};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < DOF; j++) {
            double sacc = 0;
            for (int m = 0; m < 3; m++) sacc += JRt[3 * i + m] * rec[R_J + DOF * (3 + m) + j];
            dL[i][j] = sacc;
        }
        double sacc = 0;
        for (int m = 0; m < 3; m++) sacc += JRt[3 * i + m] * dRref[m];
        dL[i][IS] = -sacc;
    }
    double gxh[NX], hxh[NX * NX];
    for (int j = 0; j < NX; j++) {
        double sacc = 0;
        for (int i = 0; i < 3; i++) sacc += dL[i][j] * w[i];
        gxh[j] = 2.0 * qo * sacc;
    }
    for (int a = 0; a < NX; a++)
        for (int b = 0; b < NX; b++) {
            double sacc = 0;
            for (int i = 0; i < 3; i++) sacc += dL[i][a] * dL[i][b];
            hxh[a * NX + b] = 2.0 * qo * sacc;
        }
    // input grads
    double gui[NU] = {}, huu[NU * NU] = {};
    if (k != N) {
        for (int j = 0; j < DOF; j++) gui[j] = 2.0 * p.r_dq * u[j];
        gui[IDVS] = 2.0 * p.r_dVs * u[IDVS];
        for (int j = 0; j < DOF; j++) huu[j * NU + j] = 2.0 * p.r_dq;
        huu[IDVS * NU + IDVS] = 2.0 * p.r_dVs;
    }
    double gxs[NX] = {};
    for (int j = 0; j < DOF; j++) gxs[j] = -p.q_sing * rec[R_DMU + j];

    for (int j = 0; j < NX; j++) out.fx[j] = gxc[j] + gxh[j] + 0.0 + gxs[j];
    for (int j = 0; j < NU; j++) out.fu[j] = 0.0 + 0.0 + gui[j] + 0.0;
    for (int i = 0; i < NX * NX; i++) out.fxx[i] = hxc[i] + hxh[i] + 0.0 + 0.0;
    for (int i = 0; i < NU * NU; i++) out.fuu[i] = 0.0 + 0.0 + huu[i] + 0.0;
    for (int i = 0; i < NX * NU; i++) out.fxu[i] = 0.0;
    for (int i = 0; i < NX; i++) out.fxx[i * NX + i] += 1e-6;  // :353-354
    for (int i = 0; i < NU; i++) out.fuu[i * NU + i] += 1e-6;
}

// ------------------------------------------------------------------------------------------------
// Constraints — constraints.cpp:34-243
// ------------------------------------------------------------------------------------------------
static double rbf(double delta, double h) {  // :34-43
    if (h >= delta) return -std::log(h + 1);
    return -std::log(delta + 1) - 1 / (delta + 1) * (h - delta) + 1 / (2 * std::pow(delta + 1, 2)) * std::pow(h - delta, 2);
}
static double drbf(double delta, double h) {  // :52-61
    if (h >= delta) return -1 / (h + 1);
    return -1 / (delta + 1) + 1 / (std::pow(delta + 1, 2)) * (h - delta);
}

struct ConOut {
    double c[NPC], l[NPC], u[NPC];
    double cx[NPC * NX], cu[NPC * NU];
};

static void stage_constraints(const Oracle& o, const double* x, const double* u, const double* rec, int k, bool want_jac,
                              ConOut& out) {
    const OracleParams& p = o.p;
    const int N = p.N;
    std::memset(&out, 0, sizeof out);
    const double delta = -0.5;
    auto masked = [&](int r) { out.c[r] = 0; out.l[r] = -INF; out.u[r] = INF; };
    // self collision :70-108
    if (p.constraint_mask & 1) {
        double md = 0.01 * rec[R_SEL];
        double dmd[DOF];
        for (int j = 0; j < DOF; j++) dmd[j] = 0.01 * rec[R_DSEL + j];
        double r = p.con_tol_selcol * 0.01;
        double R = rbf(delta, md - r);
        if (k != N) {
            double dot = 0;
            for (int j = 0; j < DOF; j++) dot += dmd[j] * u[j];
            out.l[0] = -INF; out.u[0] = 0.0; out.c[0] = -dot + R;
            if (want_jac) {
                double dR = drbf(delta, md - r);
                for (int j = 0; j < DOF; j++) { out.cx[0 * NX + j] = dR * dmd[j]; out.cu[0 * NU + j] = -dmd[j]; }
            }
        }
    } else if (k != N) masked(0);
    // singularity :110-147
    if (p.constraint_mask & 2) {
        double mu = rec[R_MU];
        double eps = p.con_tol_sing;
        double R = rbf(delta, mu - eps);
        if (k != N) {
            double dot = 0;
            for (int j = 0; j < DOF; j++) dot += rec[R_DMU + j] * u[j];
            out.l[1] = -INF; out.u[1] = 0.0; out.c[1] = -dot + R;
            if (want_jac) {
                double dR = drbf(delta, mu - eps);
                for (int j = 0; j < DOF; j++) { out.cx[1 * NX + j] = dR * rec[R_DMU + j]; out.cu[1 * NU + j] = -rec[R_DMU + j]; }
            }
        }
    } else if (k != N) masked(1);
    // env collision :149-190
    if (p.constraint_mask & 4) {
        double r = 0.01 * p.con_tol_envcol;
        for (int m = 0; m < NLINK; m++) {
            double md = 0.01 * (rec[R_ENV + m] - rec[R_OBSR] * 1.2);
            double R = rbf(delta, md - r);
            if (k != N) {
                double dot = 0;
                for (int j = 0; j < DOF; j++) dot += (0.01 * rec[R_DENV + DOF * m + j]) * u[j];
                out.l[2 + m] = -INF; out.u[2 + m] = 0.0; out.c[2 + m] = -dot + R;
                if (want_jac) {
                    double dR = drbf(delta, md - r);
                    for (int j = 0; j < DOF; j++) {
                        double g = 0.01 * rec[R_DENV + DOF * m + j];
                        out.cx[(2 + m) * NX + j] = dR * g;
                        out.cu[(2 + m) * NU + j] = -g;
                    }
                }
            }
        }
    } else if (k != N) for (int m = 0; m < NLINK; m++) masked(2 + m);
}

// ------------------------------------------------------------------------------------------------
// Dense QP assembly in the reference layout — osqp_interface.cpp:129-396
// guess layout here: (N+1) x [x(9), u(8)]  (u of stage N is zero/unused)
// ------------------------------------------------------------------------------------------------
struct DenseQP {
    int nv, nc;
    double obj;
    std::vector<double> P, g, A, c, l, u;
};

static inline const double* gx(const double* guess, int i) { return guess + NXU * i; }
static inline const double* gu(const double* guess, int i) { return guess + NXU * i + NX; }

// setCost (:129-219) + setConstraints (:221-389).  want: 0 = obj/constr/l/u only, 1 = full.
static void set_qp(const Oracle& o, const double* guess, const double* recs, const double* ucur, bool full, DenseQP& q) {
    const OracleParams& p = o.p;
    const int N = p.N;
    const double* Tx = p.Tx; const double* Tu = p.Tu;
    q.nv = o.nvar(); q.nc = o.nconstr();
    const int nv = q.nv, nc = q.nc;
    const int Neq = (N + 1) * NX, Nib = nv + N * NU;
    q.obj = 0;
    if (full) { q.P.assign((size_t)nv * nv, 0.0); q.g.assign(nv, 0.0); q.A.assign((size_t)nc * nv, 0.0); }
    q.c.assign(nc, 0.0); q.l.assign(nc, 0.0); q.u.assign(nc, 0.0);
    auto P = [&](int i, int j) -> double& { return q.P[(size_t)i * nv + j]; };
    auto A = [&](int i, int j) -> double& { return q.A[(size_t)i * nv + j]; };
    const double rddq = p.qp_r_ddq;
    // ---- cost
    for (int i = 0; i <= N; i++) {
        CostOut co;
        stage_cost(o, gx(guess, i), gu(guess, i), recs + (size_t)REC * i, i, full, co);
        q.obj += co.obj;
        if (full) {
            for (int a = 0; a < NX; a++) q.g[NX * i + a] = Tx[a] * co.fx[a];
            for (int a = 0; a < NX; a++)
                for (int b = 0; b < NX; b++) P(NX * i + a, NX * i + b) = Tx[a] * co.fxx[a * NX + b] * Tx[b];
            if (i != N) {
                int u0 = NX * (N + 1) + NU * i;
                for (int a = 0; a < NU; a++) q.g[u0 + a] = Tu[a] * co.fu[a];
                for (int a = 0; a < NU; a++)
                    for (int b = 0; b < NU; b++) P(u0 + a, u0 + b) = Tu[a] * co.fuu[a * NU + b] * Tu[b];
                for (int a = 0; a < NX; a++)
                    for (int b = 0; b < NU; b++) {
                        double v = Tx[a] * co.fxu[a * NU + b] * Tu[b];
                        P(NX * i + a, u0 + b) = v;
                        P(u0 + b, NX * i + a) = v;
                    }
            }
        }
        if (i != N) {  // ddq cost :166-217
            const double* ui = gu(guess, i);
            if (i != N - 1) {
                const double* un = gu(guess, i + 1);
                double sq = 0;
                for (int j = 0; j < DOF; j++) sq += (un[j] - ui[j]) * (un[j] - ui[j]);
                q.obj += rddq * sq;
            }
            if (full) {
                int u0 = NX * (N + 1) + NU * i;
                for (int j = 0; j < DOF; j++) {
                    double gg;
                    if (i == 0) gg = 2. * rddq * (ui[j] - gu(guess, i + 1)[j]);
                    else if (i == N - 1) gg = 2. * rddq * (ui[j] - gu(guess, i - 1)[j]);
                    else gg = 2. * rddq * (2. * ui[j] - gu(guess, i + 1)[j] - gu(guess, i - 1)[j]);
                    q.g[u0 + j] += Tu[j] * gg;
                }
                double cii, cij;
                if (i == 0) { cii = 2. * rddq; cij = -2. * rddq; }
                else if (i == N - 1) { cii = 2. * rddq; cij = 0; }
                else { cii = 4. * rddq; cij = -2. * rddq; }
                for (int j = 0; j < DOF; j++) {
                    P(u0 + j, u0 + j) += Tu[j] * cii * Tu[j];
                    if (i != N - 1) {
                        P(u0 + j, u0 + NU + j) += Tu[j] * cij * Tu[j];
                        P(u0 + NU + j, u0 + j) += Tu[j] * cij * Tu[j];
                    }
                }
            }
        }
    }
    // ---- dynamics (setDynamics :221-252)
    for (int i = 0; i <= N; i++) {
        if (i == 0) {
            if (full) for (int a = 0; a < NX; a++) A(a, a) = 1.0;
            continue;
        }
        const double* xp = gx(guess, i - 1); const double* up = gu(guess, i - 1); const double* xi = gx(guess, i);
        double pred[NX];
        for (int a = 0; a < NX; a++) {
            double s1 = 0, s2 = 0;
            for (int b = 0; b < NX; b++) s1 += o.A[a * NX + b] * xp[b];
            for (int b = 0; b < NU; b++) s2 += o.B[a * NU + b] * up[b];
            pred[a] = s1 + s2 + 0.0;
        }
        for (int a = 0; a < NX; a++) q.c[NX * i + a] = (1.0 / Tx[a]) * (xi[a] - pred[a]);
        if (full) {
            for (int a = 0; a < NX; a++) {
                for (int b = 0; b < NX; b++) A(NX * i + a, NX * (i - 1) + b) = -(1.0 / Tx[a]) * o.A[a * NX + b] * Tx[b];
                A(NX * i + a, NX * i + a) = 1.0;
                for (int b = 0; b < NU; b++)
                    A(NX * i + a, NX * (N + 1) + NU * (i - 1) + b) = -(1.0 / Tx[a]) * o.B[a * NU + b] * Tu[b];
            }
        }
    }
    // ---- bounds (setBounds :254-300, Bounds::getBounds* bounds.cpp:85-128)
    const double L = o.track.length();
    for (int i = 0; i <= N; i++) {
        const double* xi = gx(guess, i);
        int r0 = Neq + NX * i;
        for (int a = 0; a < NX; a++) {
            if (full) A(r0 + a, NX * i + a) = Tx[a];
            q.c[r0 + a] = xi[a];
            q.l[r0 + a] = p.lx[a];
            q.u[r0 + a] = p.ux[a];
        }
        q.l[r0 + IS] = std::max(xi[IS] - p.s_trust_region, 0.);
        q.u[r0 + IS] = std::min(xi[IS] + p.s_trust_region, L);
        if (i != N) {
            const double* ui = gu(guess, i);
            int r1 = Neq + NX * (N + 1) + NU * i;  // input bounds, Q1: columns NU*i (state columns)
            for (int a = 0; a < NU; a++) {
                if (full) A(r1 + a, NU * i + a) = Tu[a];
                q.c[r1 + a] = ui[a];
                q.l[r1 + a] = p.lu[a];
                q.u[r1 + a] = p.uu[a];
            }
            int r2 = Neq + NX * (N + 1) + NU * N + NU * i;  // ddq rows (8th row zero: Q15)
            for (int j = 0; j < DOF; j++) {
                if (i == 0) {
                    if (full) A(r2 + j, NX * (N + 1) + NU * i + j) = 1. / p.Ts * Tu[j];
                    q.c[r2 + j] = 1. / p.Ts * ui[j];
                    q.l[r2 + j] = p.lddq[j] + 1. / p.Ts * ucur[j];
                    q.u[r2 + j] = p.uddq[j] + 1. / p.Ts * ucur[j];
                } else {
                    if (full) {
                        A(r2 + j, NX * (N + 1) + NU * i + j) = 1. / p.Ts * Tu[j];
                        A(r2 + j, NX * (N + 1) + NU * (i - 1) + j) = -1. / p.Ts * Tu[j];
                    }
                    q.c[r2 + j] = 1. / p.Ts * (ui[j] - gu(guess, i - 1)[j]);
                    q.l[r2 + j] = p.lddq[j];
                    q.u[r2 + j] = p.uddq[j];
                }
            }
        }
    }
    // ---- polytopic (setPolytopicConstraints :302-344)
    for (int i = 0; i <= N; i++) {
        ConOut co;
        stage_constraints(o, gx(guess, i), gu(guess, i), recs + (size_t)REC * i, i, full, co);
        int r0 = Neq + Nib + NPC * i;
        for (int r = 0; r < NPC; r++) {
            q.c[r0 + r] = co.c[r]; q.l[r0 + r] = co.l[r]; q.u[r0 + r] = co.u[r];
            if (full) {
                for (int a = 0; a < NX; a++) A(r0 + r, NX * i + a) = co.cx[r * NX + a] * Tx[a];
                if (i != N)
                    for (int b = 0; b < NU; b++) A(r0 + r, NX * (N + 1) + NU * i + b) = co.cu[r * NU + b] * Tu[b];
            }
        }
    }
}

// constraint_norm — osqp_interface.cpp:824-833, with parity policy P1: per-row violations at or below
// vio_floor (rounding noise of an exactly solved QP step) count as zero.
static double constraint_norm(const DenseQP& q, double floor_) {
    double a = 0, b = 0;
    for (int i = 0; i < q.nc; i++) { double v = std::max(q.l[i] - q.c[i], 0.0); a += (v > floor_) ? v : 0.0; }
    for (int i = 0; i < q.nc; i++) { double v = std::max(q.c[i] - q.u[i], 0.0); b += (v > floor_) ? v : 0.0; }
    return a + b;
}

// ------------------------------------------------------------------------------------------------
// QP solvers (replacing OSQP, osqp_interface.cpp:592-656)
// ------------------------------------------------------------------------------------------------
constexpr double BIG = 1e20;  // |bound| >= BIG is treated as infinite (OSQP_INFTY semantics)
constexpr int IPM_MAX_IT = 60;
// Round 6: mu 1e-13 -> 1e-12 and the step test 1e-11 -> 3e-9: the QP is still solved to ~2e-10 in
// u (max |du0| against the tight tolerances over 4096 configs[1] and 2048 default-rows instances: 1.8e-10 / 1.7e-10),
// 5000x inside the north star's 1e-6 and far inside OSQP's eps_abs 1e-4 (osqp_interface.cpp:623), in ~0.4 fewer IPM
// iterations per QP (configs[1]: 6.82 -> 6.46 per instance, slowest wave 8.04 -> 7.66 on average).  k_sqp applies the
// same rule.
constexpr double IPM_TOL_MU = 1e-12, IPM_TOL_P = 1e-11, IPM_TOL_STEP = 3e-9;
// Step test: the last Newton step max|dz| is below IPM_TOL_STEP, or the last two steps contract
// quadratically enough that the remaining error estimate dz_k^2 / dz_{k-1} is (the final phase of
// Mehrotra's method converges quadratically; without the estimate every QP spends one more iteration
// only to observe a step of ~1e-15).  On the configs[1] workload: 9.19 -> 8.59 mean IPM iterations,
// slowest wave 21 -> 20, max |du0| vs the plain step test 6e-13.  k_ipm applies the
// same rule.
static inline bool step_converged(double dz, double dz_prev) {
    return dz < IPM_TOL_STEP || dz * dz < IPM_TOL_STEP * dz_prev;
}
constexpr double IPM_TOL_FB = 1e-9;  // P2: accept a converged iterate when the Riccati factor breaks down
constexpr double IPM_DIV = 1e6;      // P3: mu > IPM_DIV * mu_0 -> primal infeasible (divergent multipliers)
constexpr double IPM_TAU = 0.995;    // fraction-to-boundary floor
constexpr double FEAS_TOL = 1e-9;

// ---------------- stage-structured primal-dual IPM with a Riccati factorization ----------------
// Stage vector z_k = [y(9) | w(7) | v(8)] (normalized step of x_k; w_k = previous joint-input step
// v_{k-1}[0:7]; v_k = normalized step of u_k).  Dynamics: y_{k+1} = M y_k + G v_k, w_{k+1} = E v_k
// with M = Tx^-1 A Tx, G = Tx^-1 B Tu.  y_0 = 0, w_0 = 0 (dynamics row block 0, osqp_interface.cpp:231-237).
constexpr int NXA = NX + DOF, NZ = NXA + NU;  // y | w | v

struct SRow { double c[NZ]; double lb, ub; };
struct SStage {
    double H[NZ * NZ];
    double h[NZ];
    double b[NX];            // y_{k+1} = M y_k + G v_k + b_k  (b_k = -c_{k+1})
    std::vector<SRow> rows;
};

struct StructQP {
    int N;
    double M[NX * NX], G[NX * NU];
    std::vector<SStage> st;  // N+1 stages (stage N has no v)
    bool infeasible = false;
};

// Build the stage-structured QP equivalent to the dense layout (same primal solution).
// zshift (SecondOrderCorrection, osqp_interface.cpp:658-681): a QP step in the reference layout
// [x_0..x_N (9 each) | u_0..u_{N-1} (8 each)].  Each row's bounds then become l - d with d = c - A step,
// i.e. the bounds at this guess shifted by the row's A step, written out per row kind below (the
// engine's soc_stage, dev_sqp.h, uses the same formulas in the same order).
static void build_struct_qp(const Oracle& o, const double* guess, const double* recs, const double* ucur, StructQP& S,
                            const double* zshift = nullptr) {
    const OracleParams& p = o.p;
    const int N = p.N;
    const double* Tx = p.Tx; const double* Tu = p.Tu;
    S.N = N;
    S.st.assign(N + 1, SStage());
    S.infeasible = false;
    for (int a = 0; a < NX; a++) {
        for (int b = 0; b < NX; b++) S.M[a * NX + b] = (1.0 / Tx[a]) * o.A[a * NX + b] * Tx[b];
        for (int b = 0; b < NU; b++) S.G[a * NU + b] = (1.0 / Tx[a]) * o.B[a * NU + b] * Tu[b];
    }
    const double rddq = p.qp_r_ddq;
    const double L = o.track.length();
    auto ysh = [&](int k, int a) { return zshift[(size_t)NX * k + a]; };
    auto vsh = [&](int k, int b) { return (k < N) ? zshift[(size_t)NX * (N + 1) + (size_t)NU * k + b] : 0.0; };
    // Box bounds on y (state bounds + Q1 rows), accumulated as intersections in y-units.
    std::vector<double> ylb((N + 1) * NX, -INF), yub((N + 1) * NX, INF);
    auto add_box = [&](int k, int m, double lo, double hi) {
        if (lo > -BIG) ylb[k * NX + m] = std::max(ylb[k * NX + m], lo);
        if (hi < BIG) yub[k * NX + m] = std::min(yub[k * NX + m], hi);
    };
    for (int k = 0; k <= N; k++) {
        SStage& s = S.st[k];
        std::memset(s.H, 0, sizeof s.H); std::memset(s.h, 0, sizeof s.h); std::memset(s.b, 0, sizeof s.b);
        const double* xk = gx(guess, k); const double* uk = gu(guess, k);
        CostOut co;
        stage_cost(o, xk, uk, recs + (size_t)REC * k, k, true, co);
        for (int a = 0; a < NX; a++) {
            s.h[a] = Tx[a] * co.fx[a];
            for (int b = 0; b < NX; b++) s.H[a * NZ + b] = Tx[a] * co.fxx[a * NX + b] * Tx[b];
        }
        if (k != N) {
            for (int a = 0; a < NU; a++) {
                s.h[NXA + a] = Tu[a] * co.fu[a];
                for (int b = 0; b < NU; b++) s.H[(NXA + a) * NZ + NXA + b] = Tu[a] * co.fuu[a * NU + b] * Tu[b];
                for (int b = 0; b < NX; b++) {
                    double v = Tx[b] * co.fxu[b * NU + a] * Tu[a];
                    s.H[(NXA + a) * NZ + b] = v; s.H[b * NZ + NXA + a] = v;
                }
            }
            // ddq cost gradient + diagonal, coupling to v_{k-1} via w_k
            for (int j = 0; j < DOF; j++) {
                double gg;
                if (k == 0) gg = 2. * rddq * (uk[j] - gu(guess, k + 1)[j]);
                else if (k == N - 1) gg = 2. * rddq * (uk[j] - gu(guess, k - 1)[j]);
                else gg = 2. * rddq * (2. * uk[j] - gu(guess, k + 1)[j] - gu(guess, k - 1)[j]);
                s.h[NXA + j] += Tu[j] * gg;
                double cii = (k == 0 || k == N - 1) ? 2. * rddq : 4. * rddq;
                s.H[(NXA + j) * NZ + NXA + j] += Tu[j] * cii * Tu[j];
                if (k >= 1) {  // coupling between v_{k-1} (= w_k) and v_k, present when k-1 != N-1
                    double cij = -2. * rddq;
                    double v = Tu[j] * cij * Tu[j];
                    s.H[(NXA + j) * NZ + NX + j] += v;
                    s.H[(NX + j) * NZ + NXA + j] += v;
                }
            }
        }
        // dynamics offset b_k = -c_{k+1}
        if (k < N) {
            const double* xn = gx(guess, k + 1);
            for (int a = 0; a < NX; a++) {
                double s1 = 0, s2 = 0;
                for (int b = 0; b < NX; b++) s1 += o.A[a * NX + b] * xk[b];
                for (int b = 0; b < NU; b++) s2 += o.B[a * NU + b] * uk[b];
                double pred = s1 + s2 + 0.0;
                s.b[a] = -((1.0 / Tx[a]) * (xn[a] - pred));
                if (zshift) {  // + (y_{k+1} - M y_k - G v_k) of the step
                    double ay = 0, gv = 0;
                    for (int m = 0; m < NX; m++) ay += S.M[a * NX + m] * ysh(k, m);
                    for (int m = 0; m < NU; m++) gv += S.G[a * NU + m] * vsh(k, m);
                    s.b[a] = s.b[a] + (ysh(k + 1, a) - ay - gv);
                }
            }
        }
        // state bounds
        for (int a = 0; a < NX; a++) {
            double lo = p.lx[a], hi = p.ux[a];
            if (a == IS) { lo = std::max(xk[IS] - p.s_trust_region, 0.); hi = std::min(xk[IS] + p.s_trust_region, L); }
            add_box(k, a, (lo - xk[a]) / Tx[a], (hi - xk[a]) / Tx[a]);
        }
        if (k != N) {
            // Q1 input-bound rows: variable index NU*k + a of the stacked state-step vector
            for (int a = 0; a < NU; a++) {
                int idx = NU * k + a;
                int kk = idx / NX, m = idx % NX;
                add_box(kk, m, (p.lu[a] - uk[a]) / Tu[a], (p.uu[a] - uk[a]) / Tu[a]);
            }
            // ddq rows
            for (int j = 0; j < DOF; j++) {
                double coef = 1. / p.Ts * Tu[j];
                SRow r; std::memset(r.c, 0, sizeof r.c);
                double c, lo, hi;
                if (k == 0) {
                    c = 1. / p.Ts * uk[j];
                    lo = p.lddq[j] + 1. / p.Ts * ucur[j];
                    hi = p.uddq[j] + 1. / p.Ts * ucur[j];
                    r.c[NXA + j] = 1.0;
                } else {
                    c = 1. / p.Ts * (uk[j] - gu(guess, k - 1)[j]);
                    lo = p.lddq[j]; hi = p.uddq[j];
                    r.c[NXA + j] = 1.0; r.c[NX + j] = -1.0;
                }
                r.lb = (lo - c) / coef; r.ub = (hi - c) / coef;
                if (zshift) {  // + v_k[j] - v_{k-1}[j] (k = 0: v_0[j]) of the step
                    const double sh = (k == 0) ? vsh(0, j) : vsh(k, j) - vsh(k - 1, j);
                    r.lb = r.lb + sh; r.ub = r.ub + sh;
                }
                s.rows.push_back(r);
            }
            // polytopic rows
            ConOut cn;
            stage_constraints(o, xk, uk, recs + (size_t)REC * k, k, true, cn);
            for (int r = 0; r < NPC; r++) {
                double lo = cn.l[r] - cn.c[r], hi = cn.u[r] - cn.c[r];
                bool lo_inf = cn.l[r] <= -BIG, hi_inf = cn.u[r] >= BIG;
                if (lo_inf && hi_inf) continue;
                SRow row; std::memset(row.c, 0, sizeof row.c);
                for (int a = 0; a < NX; a++) row.c[a] = cn.cx[r * NX + a] * Tx[a];
                for (int b = 0; b < NU; b++) row.c[NXA + b] = cn.cu[r * NU + b] * Tu[b];
                row.lb = lo_inf ? -INF : lo;
                row.ub = hi_inf ? INF : hi;
                if (zshift) {  // + a . y_k[0:7] + bv . v_k[0:7] of the step (the row's other entries are 0)
                    double sh = 0;
                    for (int a = 0; a < DOF; a++) sh += row.c[a] * ysh(k, a);
                    for (int b = 0; b < DOF; b++) sh += row.c[NXA + b] * vsh(k, b);
                    if (!lo_inf) row.lb = lo + sh;
                    if (!hi_inf) row.ub = hi + sh;
                }
                s.rows.push_back(row);
            }
        }
    }
    // box rows: + y_k[m] of the step (state rows and Q1 rows alike; finite bounds only)
    if (zshift)
        for (int k = 0; k <= N; k++)
            for (int m = 0; m < NX; m++) {
                if (ylb[k * NX + m] > -BIG) ylb[k * NX + m] = ylb[k * NX + m] + ysh(k, m);
                if (yub[k * NX + m] < BIG) yub[k * NX + m] = yub[k * NX + m] + ysh(k, m);
            }
    // stage-0 y rows are constants (y_0 = 0): feasibility check only
    for (int m = 0; m < NX; m++) {
        if (ylb[m] > FEAS_TOL || yub[m] < -FEAS_TOL) S.infeasible = true;
    }
    for (int k = 1; k <= N; k++)
        for (int m = 0; m < NX; m++) {
            double lo = ylb[k * NX + m], hi = yub[k * NX + m];
            if (lo > hi) { S.infeasible = true; continue; }
            if (lo <= -BIG && hi >= BIG) continue;
            SRow r; std::memset(r.c, 0, sizeof r.c);
            r.c[m] = 1.0; r.lb = lo; r.ub = hi;
            S.st[k].rows.push_back(r);
        }
}

// Cholesky in place (lower), returns false if not PD
static bool chol(double* F, int n) {
    for (int j = 0; j < n; j++) {
        double d = F[j * n + j];
        for (int k = 0; k < j; k++) d -= F[j * n + k] * F[j * n + k];
        if (!(d > 0)) return false;
        d = std::sqrt(d);
        F[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = F[i * n + j];
            for (int k = 0; k < j; k++) s -= F[i * n + k] * F[j * n + k];
            F[i * n + j] = s / d;
        }
        for (int i = 0; i < j; i++) F[i * n + j] = 0;
    }
    return true;
}
static void chol_solve(const double* L, int n, double* x) {
    for (int i = 0; i < n; i++) {
        double s = x[i];
        for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
        x[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = x[i];
        for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
        x[i] = s / L[i * n + i];
    }
}

struct Ineq { int k; int row; double sgn; double bnd; };  // sgn*(c^T z_k) <= sgn*bnd

// Riccati factorization of the step system with stage Hessians Hk (NZ x NZ) and the solve for gk.
struct Riccati {
    int N;
    std::vector<double> K, kff, LF, Gm;   // per stage: K 8x16, kff 8, LF 8x8, Gm 8x16
    bool factor(const StructQP& S, const std::vector<double>& Hs) {
        N = S.N;
        K.assign((size_t)N * NU * NXA, 0); kff.assign((size_t)N * NU, 0);
        LF.assign((size_t)N * NU * NU, 0); Gm.assign((size_t)N * NU * NXA, 0);
        // A~ = [[M,0],[0,0]], B~ = [[G],[E]]
        double At[NXA * NXA] = {}, Bt[NXA * NU] = {};
        for (int a = 0; a < NX; a++) {
            for (int b = 0; b < NX; b++) At[a * NXA + b] = S.M[a * NX + b];
            for (int b = 0; b < NU; b++) Bt[a * NU + b] = S.G[a * NU + b];
        }
        for (int j = 0; j < DOF; j++) Bt[(NX + j) * NU + j] = 1.0;
        double P[NXA * NXA];
        const double* HN = &Hs[(size_t)N * NZ * NZ];
        for (int a = 0; a < NXA; a++)
            for (int b = 0; b < NXA; b++) P[a * NXA + b] = HN[a * NZ + b];
        for (int k = N - 1; k >= 0; k--) {
            const double* H = &Hs[(size_t)k * NZ * NZ];
            double PB[NXA * NU], PA[NXA * NXA];
            for (int a = 0; a < NXA; a++) {
                for (int j = 0; j < NU; j++) { double s = 0; for (int m = 0; m < NXA; m++) s += P[a * NXA + m] * Bt[m * NU + j]; PB[a * NU + j] = s; }
                for (int j = 0; j < NXA; j++) { double s = 0; for (int m = 0; m < NXA; m++) s += P[a * NXA + m] * At[m * NXA + j]; PA[a * NXA + j] = s; }
            }
            double F[NU * NU], Gk[NU * NXA], Hb[NXA * NXA];
            for (int i = 0; i < NU; i++)
                for (int j = 0; j < NU; j++) {
                    double s = 0; for (int m = 0; m < NXA; m++) s += Bt[m * NU + i] * PB[m * NU + j];
                    F[i * NU + j] = H[(NXA + i) * NZ + NXA + j] + s;
                }
            for (int i = 0; i < NU; i++)
                for (int j = 0; j < NXA; j++) {
                    double s = 0; for (int m = 0; m < NXA; m++) s += Bt[m * NU + i] * PA[m * NXA + j];
                    Gk[i * NXA + j] = H[(NXA + i) * NZ + j] + s;
                }
            for (int i = 0; i < NXA; i++)
                for (int j = 0; j < NXA; j++) {
                    double s = 0; for (int m = 0; m < NXA; m++) s += At[m * NXA + i] * PA[m * NXA + j];
                    Hb[i * NXA + j] = H[i * NZ + j] + s;
                }
            if (!chol(F, NU)) return false;
            double* Kk = &K[(size_t)k * NU * NXA];
            for (int j = 0; j < NXA; j++) {
                double col[NU];
                for (int i = 0; i < NU; i++) col[i] = Gk[i * NXA + j];
                chol_solve(F, NU, col);
                for (int i = 0; i < NU; i++) Kk[i * NXA + j] = -col[i];
            }
            std::memcpy(&LF[(size_t)k * NU * NU], F, sizeof F);
            std::memcpy(&Gm[(size_t)k * NU * NXA], Gk, sizeof Gk);
            for (int i = 0; i < NXA; i++)
                for (int j = 0; j < NXA; j++) {
                    double s = 0; for (int m = 0; m < NU; m++) s += Gk[m * NXA + i] * Kk[m * NXA + j];
                    P[i * NXA + j] = Hb[i * NXA + j] + s;
                }
            for (int i = 0; i < NXA; i++)  // symmetrize
                for (int j = i + 1; j < NXA; j++) { double v = 0.5 * (P[i * NXA + j] + P[j * NXA + i]); P[i * NXA + j] = P[j * NXA + i] = v; }
        }
        return true;
    }
    // solve for gradient gs (per stage NZ) -> dz (per stage NZ); dynamics homogeneous, z~_0 = 0
    void solve(const StructQP& S, const std::vector<double>& gs, std::vector<double>& dz) const {
        double At[NXA * NXA] = {}, Bt[NXA * NU] = {};
        for (int a = 0; a < NX; a++) {
            for (int b = 0; b < NX; b++) At[a * NXA + b] = S.M[a * NX + b];
            for (int b = 0; b < NU; b++) Bt[a * NU + b] = S.G[a * NU + b];
        }
        for (int j = 0; j < DOF; j++) Bt[(NX + j) * NU + j] = 1.0;
        std::vector<double> kf((size_t)N * NU);
        double pv[NXA];
        for (int a = 0; a < NXA; a++) pv[a] = gs[(size_t)N * NZ + a];
        for (int k = N - 1; k >= 0; k--) {
            const double* g = &gs[(size_t)k * NZ];
            double f[NU];
            for (int i = 0; i < NU; i++) { double s = 0; for (int m = 0; m < NXA; m++) s += Bt[m * NU + i] * pv[m]; f[i] = g[NXA + i] + s; }
            chol_solve(&LF[(size_t)k * NU * NU], NU, f);
            for (int i = 0; i < NU; i++) kf[(size_t)k * NU + i] = -f[i];
            const double* Gk = &Gm[(size_t)k * NU * NXA];
            double np[NXA];
            for (int i = 0; i < NXA; i++) {
                double s = 0; for (int m = 0; m < NXA; m++) s += At[m * NXA + i] * pv[m];
                double t = 0; for (int m = 0; m < NU; m++) t += Gk[m * NXA + i] * kf[(size_t)k * NU + m];
                np[i] = g[i] + s + t;
            }
            std::memcpy(pv, np, sizeof np);
        }
        dz.assign((size_t)(N + 1) * NZ, 0.0);
        double x[NXA] = {};
        for (int k = 0; k < N; k++) {
            double* z = &dz[(size_t)k * NZ];
            for (int a = 0; a < NXA; a++) z[a] = x[a];
            const double* Kk = &K[(size_t)k * NU * NXA];
            for (int i = 0; i < NU; i++) { double s = 0; for (int m = 0; m < NXA; m++) s += Kk[i * NXA + m] * x[m]; z[NXA + i] = s + kf[(size_t)k * NU + i]; }
            double xn[NXA];
            for (int a = 0; a < NXA; a++) {
                double s = 0; for (int m = 0; m < NXA; m++) s += At[a * NXA + m] * x[m];
                for (int m = 0; m < NU; m++) s += Bt[a * NU + m] * z[NXA + m];
                xn[a] = s;
            }
            std::memcpy(x, xn, sizeof xn);
        }
        for (int a = 0; a < NXA; a++) dz[(size_t)N * NZ + a] = x[a];
    }
};

// ---------------- damped BFGS (SQPParam use_BFGS, osqp_interface.cpp:437-453, 683-715) ----------------
// After SQP iteration 0 the reference keeps its QP Hessian and updates it by damped BFGS (setQP is called
// without the Hessian, :441-442).  Held as the structured Hessian H_0 of iteration 0 plus low-rank terms,
// B = H_0 + sum_j c_j u_j u_j^T, u_j in the stage layout (y and v parts, w = 0).  The interior point solves
// with B through the Sherman-Morrison-Woodbury identity around each Riccati solve.
// Gaussian elimination with partial pivoting of a small n x n system (the Woodbury capacitance matrix)
static void lu_solve_small(std::vector<double>& A, int n, std::vector<double>& b) {
    for (int k = 0; k < n; k++) {
        int p = k;
        for (int i = k + 1; i < n; i++) if (std::fabs(A[(size_t)i * n + k]) > std::fabs(A[(size_t)p * n + k])) p = i;
        if (p != k) { for (int j = 0; j < n; j++) std::swap(A[(size_t)k * n + j], A[(size_t)p * n + j]); std::swap(b[k], b[p]); }
        for (int i = k + 1; i < n; i++) {
            const double f = A[(size_t)i * n + k] / A[(size_t)k * n + k];
            for (int j = k; j < n; j++) A[(size_t)i * n + j] -= f * A[(size_t)k * n + j];
            b[i] -= f * b[k];
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        double s2 = b[i];
        for (int j = i + 1; j < n; j++) s2 -= A[(size_t)i * n + j] * b[j];
        b[i] = s2 / A[(size_t)i * n + i];
    }
}
constexpr int BFGS_MAX_TERMS = 28;  // low-rank terms held at most (the engine's LRX, kernels.h)
struct LowRank {
    std::vector<std::vector<double>> u;  // (N+1)*NZ each
    std::vector<double> c;
    int r() const { return (int)c.size(); }
};
static double vdot(const std::vector<double>& a, const std::vector<double>& b) {
    double s = 0;
    for (size_t i = 0; i < a.size(); i++) s += a[i] * b[i];
    return s;
}
// reference layout [x_0..x_N | u_0..u_{N-1}] <-> stage layout z_k = [y_k | w_k | v_k] (w_k left 0)
static void dense_to_stage(int N, const double* d, std::vector<double>& z) {
    z.assign((size_t)(N + 1) * NZ, 0.0);
    for (int k = 0; k <= N; k++) {
        for (int a = 0; a < NX; a++) z[(size_t)k * NZ + a] = d[(size_t)NX * k + a];
        if (k < N)
            for (int b = 0; b < NU; b++) z[(size_t)k * NZ + NXA + b] = d[(size_t)NX * (N + 1) + NU * k + b];
    }
}
// B s in the reference layout: the stage Hessians act on z_k = [x_k | u_{k-1}[0:DOF] | u_k] (the ddq
// coupling of u_k and u_{k-1} sits in stage k's (v, w) block), plus the low-rank terms
static void bfgs_hess_mul(const StructQP& S, const LowRank& lr, const std::vector<double>& sd, std::vector<double>& out) {
    const int N = S.N;
    const size_t ou = (size_t)NX * (N + 1);
    out.assign(sd.size(), 0.0);
    for (int k = 0; k <= N; k++) {
        double z[NZ] = {};
        for (int a = 0; a < NX; a++) z[a] = sd[(size_t)NX * k + a];
        if (k >= 1)
            for (int j = 0; j < DOF; j++) z[NX + j] = sd[ou + (size_t)NU * (k - 1) + j];
        if (k < N)
            for (int b = 0; b < NU; b++) z[NXA + b] = sd[ou + (size_t)NU * k + b];
        for (int a = 0; a < NZ; a++) {
            double t = 0;
            for (int b = 0; b < NZ; b++) t += S.st[k].H[a * NZ + b] * z[b];
            if (a < NX) out[(size_t)NX * k + a] += t;
            else if (a < NXA) { if (k >= 1) out[ou + (size_t)NU * (k - 1) + (a - NX)] += t; }
            else if (k < N) out[ou + (size_t)NU * k + (a - NXA)] += t;
        }
    }
    std::vector<double> ud;
    for (int j = 0; j < lr.r(); j++) {  // + c_j u_j (u_j^T s), u_j back in the reference layout
        ud.assign(sd.size(), 0.0);
        for (int k = 0; k <= N; k++) {
            for (int a = 0; a < NX; a++) ud[(size_t)NX * k + a] = lr.u[j][(size_t)k * NZ + a];
            if (k < N)
                for (int b = 0; b < NU; b++) ud[ou + (size_t)NU * k + b] = lr.u[j][(size_t)k * NZ + NXA + b];
        }
        const double f = lr.c[j] * vdot(ud, sd);
        for (size_t i = 0; i < sd.size(); i++) out[i] += f * ud[i];
    }
}
// BFGSUpdate (osqp_interface.cpp:683-715): B' = B - Bs Bs^T / sBs + r r^T / sr (damped; unchanged if
// sr < eps).  Returns false if the update makes the Hessian NaN (sBs = 0 with sr >= eps, as the reference's
// division would), which the caller reports as NAN_HESSIAN (isNan, :474-477).
static bool bfgs_update(const StructQP& S0, LowRank& lr, const std::vector<double>& sp, const std::vector<double>& dg) {
    const int N = S0.N;
    std::vector<double> Bs;
    bfgs_hess_mul(S0, lr, sp, Bs);
    const double sBs = vdot(sp, Bs), sy = vdot(sp, dg);
    std::vector<double> r(sp.size());
    double sr;
    if (sy < 0.2 * sBs) {
        const double theta = 0.8 * sBs / (sBs - sy);
        for (size_t i = 0; i < r.size(); i++) r[i] = theta * dg[i] + (1 - theta) * Bs[i];
        sr = theta * sy + (1 - theta) * sBs;
    } else {
        r = dg;
        sr = sy;
    }
    if (sr < std::numeric_limits<double>::epsilon()) return true;
    if (!(sBs != 0.0) || !std::isfinite(sBs) || !std::isfinite(sr)) return false;
    std::vector<double> zs;
    dense_to_stage(N, Bs.data(), zs);
    lr.u.push_back(zs); lr.c.push_back(-1.0 / sBs);
    dense_to_stage(N, r.data(), zs);
    lr.u.push_back(zs); lr.c.push_back(1.0 / sr);
    return true;
}

// qp_mode 2: BFGSUpdate (osqp_interface.cpp:683-715) verbatim on one dense Hess_ that is updated in place at every
// SQP iteration, with no cap on the number of updates (the engine and qp_modes 0/1 restart past BFGS_MAX_TERMS
// low-rank terms: deviation 7).  Same operation order as the Eigen expression
// Hess - Bs * Bs^T / sBs + r * r^T / sr.
static void bfgs_update_dense(std::vector<double>& H, int nv, const std::vector<double>& s, const std::vector<double>& dg) {
    std::vector<double> Bs(nv, 0.0), r(nv);
    for (int a = 0; a < nv; a++) {
        double t = 0;
        for (int b = 0; b < nv; b++) t += H[(size_t)a * nv + b] * s[b];
        Bs[a] = t;
    }
    const double sBs = vdot(s, Bs), sy = vdot(s, dg);
    double sr;
    if (sy < 0.2 * sBs) {
        const double theta = 0.8 * sBs / (sBs - sy);
        for (int i = 0; i < nv; i++) r[i] = theta * dg[i] + (1 - theta) * Bs[i];
        sr = theta * sy + (1 - theta) * sBs;
    } else {
        r = dg;
        sr = sy;
    }
    if (sr < std::numeric_limits<double>::epsilon()) return;
    for (int a = 0; a < nv; a++)
        for (int b = 0; b < nv; b++)
            H[(size_t)a * nv + b] = H[(size_t)a * nv + b] - Bs[a] * Bs[b] / sBs + r[a] * r[b] / sr;
}

// Returns 0 on success (step filled in reference layout: [y_0..y_N | v_0..v_{N-1}]), else Status.
static const bool g_ipm_debug = std::getenv("MPCC_ORACLE_IPM_DEBUG") != nullptr;  // per-iteration log (debug)

// debug statistics of the last attempt on this thread (MPCC_ORACLE_IPM_STATS): max mu / mu_0 over iterations >= 1 and
// the first iteration at which it exceeded each threshold (-1: never)
static thread_local double g_ipm_rmax = 0;
static thread_local int g_ipm_cross[4] = {-1, -1, -1, -1};
static const double g_ipm_thr[4] = {1e2, 1e3, 1e4, 1e5};
static int solve_struct_ipm_from(const StructQP& S, std::vector<double>& step, int* iters_out, double s_floor,
                                 double lam_scale, int max_it, const LowRank* lr = nullptr) {
    const int N = S.N;
    if (S.infeasible) return QP_PrimalInfeasible;
    std::vector<Ineq> I;
    for (int k = 0; k <= N; k++)
        for (int r = 0; r < (int)S.st[k].rows.size(); r++) {
            const SRow& row = S.st[k].rows[r];
            if (row.lb > -BIG) I.push_back({k, r, -1.0, row.lb});
            if (row.ub < BIG) I.push_back({k, r, 1.0, row.ub});
        }
    const int m = (int)I.size();
    // initial primal: dynamics rollout with v = 0
    std::vector<double> z((size_t)(N + 1) * NZ, 0.0);
    for (int k = 0; k < N; k++) {
        const double* zk = &z[(size_t)k * NZ];
        double* zn = &z[(size_t)(k + 1) * NZ];
        for (int a = 0; a < NX; a++) {
            double s = 0; for (int b = 0; b < NX; b++) s += S.M[a * NX + b] * zk[b];
            zn[a] = s + S.st[k].b[a];
        }
    }
    auto rowdot = [&](const Ineq& q, const std::vector<double>& zz) {
        const SRow& row = S.st[q.k].rows[q.row];
        const double* zk = &zz[(size_t)q.k * NZ];
        double s = 0; for (int a = 0; a < NZ; a++) s += row.c[a] * zk[a];
        return s;
    };
    std::vector<double> sl(m), lam(m, 1.0), rp(m), W(m), dsa(m), dla(m), ds(m), dl(m), rc(m);
    for (int i = 0; i < m; i++) {
        double g = I[i].sgn * rowdot(I[i], z) - I[i].sgn * I[i].bnd;
        sl[i] = std::max(-g, s_floor);
        if (lam_scale > 0) lam[i] = lam_scale / sl[i];
    }
    std::vector<double> Hs((size_t)(N + 1) * NZ * NZ), gs((size_t)(N + 1) * NZ), dz, dza;
    Riccati R;
    int it;
    bool conv = false, diverged = false;
    double last_dz = 1e30, prev_dz = 1e30, mu0 = 0.0;
    for (it = 0; it < max_it; it++) {
        double mu = 0, rpmax = 0;
        for (int i = 0; i < m; i++) {
            rp[i] = I[i].sgn * rowdot(I[i], z) - I[i].sgn * I[i].bnd + sl[i];
            mu += sl[i] * lam[i];
            rpmax = std::max(rpmax, std::fabs(rp[i]));
        }
        mu = (m > 0) ? mu / m : 0.0;
        if (g_ipm_debug) {
            double lmax = 0, smin = 1e300;
            for (int i = 0; i < m; i++) { lmax = std::max(lmax, lam[i]); smin = std::min(smin, sl[i]); }
            std::fprintf(stderr, "ipm it %2d mu %.3e rp %.3e dz %.3e lam_max %.3e s_min %.3e\n", it, mu, rpmax,
                         last_dz, lmax, smin);
        }
        if (it > 0 && mu < IPM_TOL_MU && rpmax < IPM_TOL_P && step_converged(last_dz, prev_dz)) {
            conv = true;
            break;
        }
        // P3: the complementarity of a primal-infeasible QP grows without bound while rp
        // stalls; OSQP reports such a QP PrimalInfeasible (osqp_interface.cpp:497-499).  Converged
        // solves never exceed ~1.1 mu_0, so 1e6 mu_0 cannot cut a solve that would converge.
        if (it == 0) mu0 = mu;
        else {
            const double r = mu / mu0;  // debug statistics (MPCC_ORACLE_IPM_STATS)
            if (r > g_ipm_rmax) g_ipm_rmax = r;
            for (int q = 0; q < 4; q++)
                if (g_ipm_cross[q] < 0 && r > g_ipm_thr[q]) g_ipm_cross[q] = it;
        }
        if (it > 0 && mu > IPM_DIV * mu0) {
            diverged = true;
            break;
        }
        for (int i = 0; i < m; i++) W[i] = lam[i] / sl[i];
        // H~ = H + sum W c c^T ; base gradient Hz + h
        for (int k = 0; k <= N; k++) {
            std::memcpy(&Hs[(size_t)k * NZ * NZ], S.st[k].H, sizeof(double) * NZ * NZ);
            const double* zk = &z[(size_t)k * NZ];
            for (int a = 0; a < NZ; a++) {
                double s = 0; for (int b = 0; b < NZ; b++) s += S.st[k].H[a * NZ + b] * zk[b];
                gs[(size_t)k * NZ + a] = s + S.st[k].h[a];
            }
        }
        if (lr)  // + sum_j c_j u_j (u_j^T z)
            for (int j = 0; j < lr->r(); j++) {
                const double f = lr->c[j] * vdot(lr->u[j], z);
                for (size_t a = 0; a < gs.size(); a++) gs[a] += f * lr->u[j][a];
            }
        for (int i = 0; i < m; i++) {
            const SRow& row = S.st[I[i].k].rows[I[i].row];
            double* H = &Hs[(size_t)I[i].k * NZ * NZ];
            for (int a = 0; a < NZ; a++) {
                if (row.c[a] == 0) continue;
                for (int b = 0; b < NZ; b++) H[a * NZ + b] += W[i] * row.c[a] * row.c[b];
            }
        }
        if (!R.factor(S, Hs)) {
            // Riccati breakdown (chol(F) loses definiteness at extreme barrier weights near the end of the
            // solve): an iterate that is already converged to IPM_TOL_FB is the QP solution
            if (it > 0 && mu < IPM_TOL_FB && rpmax < IPM_TOL_FB) conv = true;
            break;
        }
        // low-rank Hessian terms (BFGS): Q_j = M u_j = -solve(u_j), Smat = C^-1 + U^T Q; every Riccati solve
        // dz_s = -M g is corrected to -(M - Q Smat^-1 Q^T) g = dz_s - Q Smat^-1 (U^T dz_s)
        const int nr = lr ? lr->r() : 0;
        std::vector<std::vector<double>> Q(nr);
        std::vector<double> Smat((size_t)nr * nr);
        for (int j = 0; j < nr; j++) {
            R.solve(S, lr->u[j], Q[j]);
            for (double& v : Q[j]) v = -v;
        }
        for (int i = 0; i < nr; i++)
            for (int j = 0; j < nr; j++) Smat[(size_t)i * nr + j] = (i == j ? 1.0 / lr->c[i] : 0.0) + vdot(lr->u[i], Q[j]);
        auto lr_solve = [&](const std::vector<double>& g, std::vector<double>& d) {
            R.solve(S, g, d);
            if (!nr) return;
            std::vector<double> t(nr), Mc = Smat;
            for (int j = 0; j < nr; j++) t[j] = vdot(lr->u[j], d);
            lu_solve_small(Mc, nr, t);
            for (int j = 0; j < nr; j++)
                for (size_t a = 0; a < d.size(); a++) d[a] -= t[j] * Q[j][a];
        };
        std::vector<double> g0 = gs;
        auto add_rows = [&](std::vector<double>& g, const std::vector<double>& coef) {
            for (int i = 0; i < m; i++) {
                const SRow& row = S.st[I[i].k].rows[I[i].row];
                double* gk = &g[(size_t)I[i].k * NZ];
                double cf = I[i].sgn * coef[i];
                for (int a = 0; a < NZ; a++) gk[a] += cf * row.c[a];
            }
        };
        auto recover = [&](const std::vector<double>& d, std::vector<double>& dS, std::vector<double>& dL) {
            for (int i = 0; i < m; i++) {
                double cd = I[i].sgn * rowdot(I[i], d);
                dS[i] = -rp[i] - cd;
                dL[i] = W[i] * (cd + rp[i]) - rc[i] / sl[i];
            }
        };
        auto max_step = [&](const std::vector<double>& dS, const std::vector<double>& dL, double cap) {
            double a = cap;
            for (int i = 0; i < m; i++) {
                if (dS[i] < 0) a = std::min(a, -sl[i] / dS[i]);
                if (dL[i] < 0) a = std::min(a, -lam[i] / dL[i]);
            }
            return a;
        };
        // predictor
        std::vector<double> coef(m);
        for (int i = 0; i < m; i++) { rc[i] = sl[i] * lam[i]; coef[i] = lam[i] + W[i] * rp[i] - rc[i] / sl[i]; }
        gs = g0; add_rows(gs, coef);
        lr_solve(gs, dza);
        recover(dza, dsa, dla);
        double aa = max_step(dsa, dla, 1.0);
        double mua = 0;
        for (int i = 0; i < m; i++) mua += (sl[i] + aa * dsa[i]) * (lam[i] + aa * dla[i]);
        mua = (m > 0) ? mua / m : 0.0;
        double sigma = (mu > 0) ? std::pow(mua / mu, 3) : 0.0;
        // corrector
        for (int i = 0; i < m; i++) { rc[i] = sl[i] * lam[i] + dsa[i] * dla[i] - sigma * mu; coef[i] = lam[i] + W[i] * rp[i] - rc[i] / sl[i]; }
        gs = g0; add_rows(gs, coef);
        lr_solve(gs, dz);
        recover(dz, ds, dl);
        // fraction to the boundary: tau = max(0.995, 1 - sqrt(mu)) lets the step approach the boundary as
        // mu -> 0 (superlinear final phase; 10.4 -> 9.2 mean IPM iterations on the configs[1] workload,
        // DESIGN.md §3.2); k_ipm applies the same rule
        const double tau = std::max(IPM_TAU, 1.0 - std::sqrt(mu));
        double a = std::min(1.0, tau * max_step(ds, dl, 1e30));
        if (g_ipm_debug) {
            double uz0 = 0, t0 = 0, S0 = 0;
            if (nr) {
                uz0 = vdot(lr->u[0], z);
                S0 = Smat[0];
            }
            std::fprintf(stderr, "orc it %2d mu %.6e amax %.6e sig %.6e alpha %.6e uz0 %.9e S0 %.9e\n", it, mu, aa, sigma, a,
                         uz0, S0);
            (void)t0;
        }
        double dzmax = 0;
        for (size_t i = 0; i < z.size(); i++) { z[i] += a * dz[i]; dzmax = std::max(dzmax, std::fabs(dz[i])); }
        for (int i = 0; i < m; i++) { sl[i] += a * ds[i]; lam[i] += a * dl[i]; }
        prev_dz = last_dz;
        last_dz = dzmax;
    }
    if (iters_out) *iters_out = it;
    if (g_ipm_debug) std::fprintf(stderr, "ipm end conv %d it %d div %d\n", conv ? 1 : 0, it, diverged ? 1 : 0);
    if (diverged) return QP_PrimalInfeasible;
    if (!conv) return QP_MaxIterReached;
    // export in reference layout
    step.assign((size_t)(N + 1) * NX + N * NU, 0.0);
    for (int k = 0; k <= N; k++) {
        for (int a = 0; a < NX; a++) step[(size_t)NX * k + a] = z[(size_t)k * NZ + a];
        if (k < N)
            for (int b = 0; b < NU; b++) step[(size_t)NX * (N + 1) + NU * k + b] = z[(size_t)k * NZ + NXA + b];
    }
    return 0;
}

// Start point: first from slacks floored at IPM_S0 with complementary multipliers
// lambda = IPM_L0 / s (mu_0 = IPM_L0: close to the central path and scaled to the bounds), at most
// IPM_MAX_IT_SCALED iterations; a solve that does not converge from there (max iterations, P3) restarts
// from the unit start point s = max(-g, 1), lambda = 1 with the full IPM_MAX_IT.  The restart is
// exactly the solve without the scaled attempt, so the scaled start can only change which iterate a
// converging QP ends on (~1e-12), never a failure into a different failure.
constexpr double IPM_S0 = 0.02, IPM_L0 = 0.002;
constexpr int IPM_MAX_IT_SCALED = 24;  // round 6: 30 -> 24
static int solve_struct_ipm(const StructQP& S, std::vector<double>& step, int* iters_out, const LowRank* lr = nullptr) {
    int it1 = 0, it2 = 0;
    static const bool stats = std::getenv("MPCC_ORACLE_IPM_STATS") != nullptr;  // debug: one line per QP solve
    auto reset = [] { g_ipm_rmax = 0; for (int q = 0; q < 4; q++) g_ipm_cross[q] = -1; };
    reset();
    // debug: start-point experiments (MPCC_ORACLE_IPM_S0 / _L0 / _CAP override the scaled start and its iteration
    // cap; never set in tests)
    static const double s0 = std::getenv("MPCC_ORACLE_IPM_S0") ? std::atof(std::getenv("MPCC_ORACLE_IPM_S0")) : IPM_S0;
    static const double l0 = std::getenv("MPCC_ORACLE_IPM_L0") ? std::atof(std::getenv("MPCC_ORACLE_IPM_L0")) : IPM_L0;
    static const int cap = std::getenv("MPCC_ORACLE_IPM_CAP") ? std::atoi(std::getenv("MPCC_ORACLE_IPM_CAP")) : IPM_MAX_IT_SCALED;
    int rc = solve_struct_ipm_from(S, step, &it1, s0, l0, cap, lr);
    const int rc1 = rc;
    const double r1 = g_ipm_rmax;
    int c1[4];
    for (int q = 0; q < 4; q++) c1[q] = g_ipm_cross[q];
    reset();
    // the restart from the unit start point follows a scaled attempt that hit its cap or broke down
    // (QP_MaxIterReached); a P3 divergence (QP_PrimalInfeasible) is final
    if (rc == QP_MaxIterReached) rc = solve_struct_ipm_from(S, step, &it2, 1.0, 0.0, IPM_MAX_IT, lr);
    if (stats)
        std::fprintf(stderr, "ipmstat %d %d %d %d %.4g %d %d %d %d %.4g %d %d %d %d\n", it1, rc1, it2, rc, r1, c1[0], c1[1],
                     c1[2], c1[3], g_ipm_rmax, g_ipm_cross[0], g_ipm_cross[1], g_ipm_cross[2], g_ipm_cross[3]);
    if (iters_out) *iters_out = it1 + it2;
    return rc;
}

// ---------------- dense-layout primal-dual IPM (validation; solves the reference QP verbatim) ---
static bool lu_solve_dense(std::vector<double>& M, int n, std::vector<double>& rhs) {
    std::vector<int> piv(n);
    for (int k = 0; k < n; k++) {
        int p = k;
        double mx = std::fabs(M[(size_t)k * n + k]);
        for (int i = k + 1; i < n; i++) if (std::fabs(M[(size_t)i * n + k]) > mx) { mx = std::fabs(M[(size_t)i * n + k]); p = i; }
        if (mx == 0) return false;
        piv[k] = p;
        if (p != k) { for (int j = 0; j < n; j++) std::swap(M[(size_t)k * n + j], M[(size_t)p * n + j]); std::swap(rhs[k], rhs[p]); }
        double d = M[(size_t)k * n + k];
        for (int i = k + 1; i < n; i++) {
            double f = M[(size_t)i * n + k] / d;
            if (f == 0) continue;
            M[(size_t)i * n + k] = f;
            for (int j = k + 1; j < n; j++) M[(size_t)i * n + j] -= f * M[(size_t)k * n + j];
            rhs[i] -= f * rhs[k];
        }
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = rhs[i];
        for (int j = i + 1; j < n; j++) s -= M[(size_t)i * n + j] * rhs[j];
        rhs[i] = s / M[(size_t)i * n + i];
    }
    return true;
}

static int solve_dense_ipm(const DenseQP& q, std::vector<double>& step, int* iters_out) {
    const int nv = q.nv, nc = q.nc;
    // classify rows
    std::vector<int> eq, in;
    std::vector<double> beq;
    struct DI { int row; double sgn, bnd; };
    std::vector<DI> I;
    // variables fixed to zero by the stage-0 dynamics rows (identity on y_0, rhs 0)
    auto fixed0 = [&](int col) { return col < NX; };
    for (int r = 0; r < nc; r++) {
        const double* a = &q.A[(size_t)r * nv];
        bool nz = false, only_fixed = true;
        for (int j = 0; j < nv; j++) if (a[j] != 0) { nz = true; if (!fixed0(j)) only_fixed = false; }
        double lo = q.l[r] - q.c[r], hi = q.u[r] - q.c[r];
        if (!nz) { if (lo > FEAS_TOL || hi < -FEAS_TOL) return QP_PrimalInfeasible; continue; }
        if (r < NX) { eq.push_back(r); beq.push_back(lo); continue; }  // y_0 = 0 (dynamics block 0)
        if (only_fixed) { if (lo > FEAS_TOL || hi < -FEAS_TOL) return QP_PrimalInfeasible; continue; }
        if (q.l[r] == q.u[r]) { eq.push_back(r); beq.push_back(lo); continue; }
        if (q.l[r] > -BIG) I.push_back({r, -1.0, lo});
        if (q.u[r] < BIG) I.push_back({r, 1.0, hi});
    }
    const int ne = (int)eq.size(), m = (int)I.size();
    std::vector<double> x(nv, 0.0), nu(ne, 0.0), s(m), lam(m, 1.0), rp(m), W(m), rc(m);
    auto Arow = [&](int r) { return &q.A[(size_t)r * nv]; };
    auto rowdot = [&](int r, const std::vector<double>& v) { const double* a = Arow(r); double t = 0; for (int j = 0; j < nv; j++) t += a[j] * v[j]; return t; };
    for (int i = 0; i < m; i++) s[i] = std::max(-(I[i].sgn * rowdot(I[i].row, x) - I[i].sgn * I[i].bnd), 1.0);
    int n = nv + ne;
    int it; bool conv = false, diverged = false;
    double last_dx = 1e30, prev_dx = 1e30, mu0 = 0.0;
    for (it = 0; it < IPM_MAX_IT; it++) {
        double mu = 0, rpmax = 0;
        for (int i = 0; i < m; i++) { rp[i] = I[i].sgn * rowdot(I[i].row, x) - I[i].sgn * I[i].bnd + s[i]; mu += s[i] * lam[i]; rpmax = std::max(rpmax, std::fabs(rp[i])); }
        mu = m ? mu / m : 0;
        std::vector<double> re(ne);
        double remax = 0;
        for (int e = 0; e < ne; e++) { re[e] = rowdot(eq[e], x) - beq[e]; remax = std::max(remax, std::fabs(re[e])); }
        if (it > 0 && mu < IPM_TOL_MU && rpmax < IPM_TOL_P && remax < IPM_TOL_P && step_converged(last_dx, prev_dx)) { conv = true; break; }
        if (it == 0) mu0 = mu;
        else if (mu > IPM_DIV * mu0) { diverged = true; break; }  // P3
        for (int i = 0; i < m; i++) W[i] = lam[i] / s[i];
        std::vector<double> K((size_t)n * n, 0.0);
        for (int i = 0; i < nv; i++) for (int j = 0; j < nv; j++) K[(size_t)i * n + j] = q.P[(size_t)i * nv + j];
        for (int i = 0; i < m; i++) {
            const double* a = Arow(I[i].row);
            for (int u = 0; u < nv; u++) { if (a[u] == 0) continue; for (int v = 0; v < nv; v++) if (a[v] != 0) K[(size_t)u * n + v] += W[i] * a[u] * a[v]; }
        }
        for (int e = 0; e < ne; e++) { const double* a = Arow(eq[e]); for (int j = 0; j < nv; j++) { K[(size_t)(nv + e) * n + j] = a[j]; K[(size_t)j * n + nv + e] = a[j]; } }
        // rd0 = P x + g + A_e^T nu  (inequality part added per solve)
        std::vector<double> rd0(nv);
        for (int i = 0; i < nv; i++) { double t = q.g[i]; for (int j = 0; j < nv; j++) t += q.P[(size_t)i * nv + j] * x[j]; rd0[i] = t; }
        for (int e = 0; e < ne; e++) { const double* a = Arow(eq[e]); for (int j = 0; j < nv; j++) rd0[j] += a[j] * nu[e]; }
        auto do_solve = [&](const std::vector<double>& rcv, std::vector<double>& dx, std::vector<double>& dnu, std::vector<double>& dS, std::vector<double>& dL) {
            std::vector<double> rhs(n, 0.0);
            for (int i = 0; i < nv; i++) rhs[i] = -rd0[i];
            for (int i = 0; i < m; i++) {
                const double* a = Arow(I[i].row);
                double cf = I[i].sgn * (lam[i] + W[i] * rp[i] - rcv[i] / s[i]);
                for (int j = 0; j < nv; j++) rhs[j] -= cf * a[j];
            }
            for (int e = 0; e < ne; e++) rhs[nv + e] = -re[e];
            std::vector<double> Kc = K;
            if (!lu_solve_dense(Kc, n, rhs)) return false;
            dx.assign(rhs.begin(), rhs.begin() + nv);
            dnu.assign(rhs.begin() + nv, rhs.end());
            dS.resize(m); dL.resize(m);
            for (int i = 0; i < m; i++) { double cd = I[i].sgn * rowdot(I[i].row, dx); dS[i] = -rp[i] - cd; dL[i] = W[i] * (cd + rp[i]) - rcv[i] / s[i]; }
            return true;
        };
        auto max_step = [&](const std::vector<double>& dS, const std::vector<double>& dL, double cap) {
            double a = cap;
            for (int i = 0; i < m; i++) { if (dS[i] < 0) a = std::min(a, -s[i] / dS[i]); if (dL[i] < 0) a = std::min(a, -lam[i] / dL[i]); }
            return a;
        };
        for (int i = 0; i < m; i++) rc[i] = s[i] * lam[i];
        std::vector<double> dxa, dnua, dsa, dla;
        if (!do_solve(rc, dxa, dnua, dsa, dla)) break;
        double aa = max_step(dsa, dla, 1.0);
        double mua = 0; for (int i = 0; i < m; i++) mua += (s[i] + aa * dsa[i]) * (lam[i] + aa * dla[i]);
        mua = m ? mua / m : 0;
        double sigma = mu > 0 ? std::pow(mua / mu, 3) : 0;
        for (int i = 0; i < m; i++) rc[i] = s[i] * lam[i] + dsa[i] * dla[i] - sigma * mu;
        std::vector<double> dx, dnu, dS, dL;
        if (!do_solve(rc, dx, dnu, dS, dL)) break;
        double a = std::min(1.0, std::max(IPM_TAU, 1.0 - std::sqrt(mu)) * max_step(dS, dL, 1e30));
        double dxmax = 0;
        for (int j = 0; j < nv; j++) { x[j] += a * dx[j]; dxmax = std::max(dxmax, std::fabs(dx[j])); }
        prev_dx = last_dx;
        last_dx = dxmax;
        for (int e = 0; e < ne; e++) nu[e] += dnu[e];  // equality multipliers: full step
        for (int i = 0; i < m; i++) { s[i] += a * dS[i]; lam[i] += a * dL[i]; }
    }
    if (iters_out) *iters_out = it;
    if (g_ipm_debug) std::fprintf(stderr, "ipm end conv %d it %d div %d\n", conv ? 1 : 0, it, diverged ? 1 : 0);
    if (diverged) return QP_PrimalInfeasible;
    if (!conv) return QP_MaxIterReached;
    step = x;
    return 0;
}

// ------------------------------------------------------------------------------------------------
// SQP — OsqpInterface::solveOCP (osqp_interface.cpp:398-590) with filterLineSearch (:759-808)
// ------------------------------------------------------------------------------------------------
struct Filter { double obj, vio; };

static void denorm_add(const Oracle& o, const double* base, const std::vector<double>& step, double alpha, double* out) {
    // out = base + alpha * deNormalizeStep(step)  (:859-869), base/out in (N+1)x17 layout
    const int N = o.p.N;
    for (int i = 0; i <= N; i++) {
        for (int a = 0; a < NX; a++) out[NXU * i + a] = base[NXU * i + a] + alpha * (o.p.Tx[a] * step[(size_t)NX * i + a]);
        for (int b = 0; b < NU; b++)
            out[NXU * i + NX + b] = (i != N) ? base[NXU * i + NX + b] + alpha * (o.p.Tu[b] * step[(size_t)NX * (N + 1) + NU * i + b]) : base[NXU * i + NX + b];
    }
}

// optional per-instance SQP trace (test instrumentation): 4 iterations x 8 doubles, same fields as
// the engine's mpcc_debug_trace_get
static thread_local double* g_trace = nullptr;

// SecondOrderCorrection (osqp_interface.cpp:658-681).  The correction point is
// vectorToOptvar(OptvarToVector(initial_guess) + step): the normalized QP step added as is, without
// deNormalizeStep (:661).  The QP keeps the first QP's P, q and A; its bounds are l(x') - d and
// u(x') - d with d = c(x') - A step (:676-678).  Returns the QP status; `out` is the new step on success.
static void soc_point(const Oracle& o, const double* guess, const std::vector<double>& step, std::vector<double>& xs) {
    const int N = o.p.N;
    xs.assign(guess, guess + (size_t)(N + 1) * NXU);
    for (int k = 0; k <= N; k++) {
        for (int a = 0; a < NX; a++) xs[NXU * k + a] = guess[NXU * k + a] + step[(size_t)NX * k + a];
        if (k < N)
            for (int b = 0; b < NU; b++) xs[NXU * k + NX + b] = guess[NXU * k + NX + b] + step[(size_t)NX * (N + 1) + NU * k + b];
    }
}
static int soc_dense(const Oracle& o, const DenseQP& q, const double* guess, const double* recs, const double* ucur,
                     const std::vector<double>& step, std::vector<double>& out, int* iters) {
    std::vector<double> xs;
    soc_point(o, guess, step, xs);
    DenseQP q2;
    set_qp(o, xs.data(), recs, ucur, false, q2);  // setConstraints(updates_initial_guess, NULL, ...) (:668)
    DenseQP qc = q;
    for (int r = 0; r < q.nc; r++) {
        double as = 0;
        for (int j = 0; j < q.nv; j++) as += q.A[(size_t)r * q.nv + j] * step[j];
        qc.c[r] = q2.c[r] - as;  // d; the solver takes l - d <= A s <= u - d
    }
    qc.l = q2.l;
    qc.u = q2.u;
    return solve_dense_ipm(qc, out, iters);
}
static int soc_struct(const Oracle& o, const StructQP& S, const double* guess, const double* recs, const double* ucur,
                      const std::vector<double>& step, std::vector<double>& out, int* iters, const LowRank* lr = nullptr) {
    std::vector<double> xs;
    soc_point(o, guess, step, xs);
    StructQP S2;
    build_struct_qp(o, xs.data(), recs, ucur, S2, step.data());
    for (int k = 0; k <= S.N; k++) {  // objective of the first QP (P, q)
        std::memcpy(S2.st[k].H, S.st[k].H, sizeof S.st[k].H);
        std::memcpy(S2.st[k].h, S.st[k].h, sizeof S.st[k].h);
    }
    return solve_struct_ipm(S2, out, iters, lr);
}

static int solve_ocp(const Oracle& o, double* guess, const double* recs, const double* ucur, double* opt_sol, int* iters_out) {
    const OracleParams& p = o.p;
    const int N = p.N;
    const int nv = o.nvar();
    std::vector<double> step(nv, 0.0);
    std::vector<Filter> filter;
    std::vector<double> zero((size_t)(N + 1) * NXU, 0.0);
    for (int i = 0; i <= N; i++) for (int a = 0; a < NX; a++) zero[NXU * i + a] = guess[a];
    int status = MAX_ITER_EXCEEDED;
    bool status_set = false;
    int it;
    std::vector<double> trial((size_t)(N + 1) * NXU);
    // damped BFGS state (use_BFGS, osqp_interface.cpp:403-453, 540-555): Hessian of iteration 0 (H0 / P0) and
    // its low-rank updates, grad_L_prev, A^T lambda and step_prev = alpha * step, all normalized, in the
    // reference layout.  A^T y of an exact QP solution is -(B step + q) (its KKT stationarity), so the
    // multiplier update lambda += alpha (y - lambda) is carried as A^T lambda (the constraint Jacobian does
    // not change within a solve: frozen records, Q4) — DESIGN.md §4.2.
    const bool bfgs = p.use_BFGS != 0;
    // At most BFGS_MAX_TERMS low-rank terms are held (the engine's LRX).  An update that would need more restarts
    // the quasi-Newton matrix instead: that SQP iteration's Hessian is the exact one of setQP (as in iteration 0,
    // :440), the terms are dropped, and later iterations update from it.  Below 1 + BFGS_MAX_TERMS / 2 = 15 SQP
    // iterations no restart can happen, so the reference's update is reproduced verbatim there.
    bool bfgs_restart = false;
    LowRank lr;
    StructQP S0;
    std::vector<double> P0, grad_L_prev(nv, 0.0), g_lam(nv, 0.0), step_prev(nv, 0.0), qd(nv, 0.0);
    bool bfgs_nan = false;
    auto bfgs_grad = [&](int iter) {  // grad_L = q + A^T lambda; Hess_ = BFGSUpdate(Hess_, step_prev, dgrad_L)
        std::vector<double> gl(nv);
        for (int i = 0; i < nv; i++) gl[i] = qd[i] + g_lam[i];
        if (iter > 0 && !bfgs_restart) {
            std::vector<double> dg(nv);
            for (int i = 0; i < nv; i++) dg[i] = gl[i] - grad_L_prev[i];
            if (!bfgs_update(S0, lr, step_prev, dg)) bfgs_nan = true;
        }
        grad_L_prev = gl;
    };
    const bool verbatim = o.opt.qp_mode == 2;  // the reference's dense in-place BFGSUpdate, no restart
    std::vector<double> Hd;                    // its Hess_ (qp_mode 2)
    for (it = 0; it < p.max_iter; it++) {
        // setQP + PD / NaN checks of the normalized Hessian (:445-473)
        bool nan = false, pd = true;
        bfgs_restart = bfgs && !verbatim && it > 0 && lr.r() + 2 > BFGS_MAX_TERMS;
        if (bfgs_restart) { lr.u.clear(); lr.c.clear(); }
        if (o.opt.qp_mode == 1 || verbatim) {
            DenseQP q;
            set_qp(o, guess, recs, ucur, true, q);
            if (bfgs && verbatim) {  // :438-453: Hess_ of setQP at iteration 0, then BFGSUpdate(Hess_, step_prev_, dgrad_L)
                if (it == 0) Hd = q.P;
                qd = q.g;
                std::vector<double> gl(nv);
                for (int i = 0; i < nv; i++) gl[i] = qd[i] + g_lam[i];
                if (it > 0) {
                    std::vector<double> dg(nv);
                    for (int i = 0; i < nv; i++) dg[i] = gl[i] - grad_L_prev[i];
                    bfgs_update_dense(Hd, nv, step_prev, dg);
                }
                grad_L_prev = gl;
                q.P = Hd;
            } else if (bfgs) {  // dense form of the same BFGS matrix: P0 + sum_j c_j u_j u_j^T
                if (it == 0 || bfgs_restart) { P0 = q.P; build_struct_qp(o, guess, recs, ucur, S0); }
                qd = q.g;
                bfgs_grad(it);
                q.P = P0;
                std::vector<double> ud(nv);
                for (int j = 0; j < lr.r(); j++) {
                    for (int k = 0; k <= N; k++) {
                        for (int a = 0; a < NX; a++) ud[(size_t)NX * k + a] = lr.u[j][(size_t)k * NZ + a];
                        if (k < N) for (int b = 0; b < NU; b++) ud[(size_t)NX * (N + 1) + NU * k + b] = lr.u[j][(size_t)k * NZ + NXA + b];
                    }
                    for (int a = 0; a < nv; a++)
                        for (int b = 0; b < nv; b++) q.P[(size_t)a * nv + b] += lr.c[j] * ud[a] * ud[b];
                }
                if (bfgs_nan) q.P[0] = std::numeric_limits<double>::quiet_NaN();
            }
            for (double v : q.P) if (std::isnan(v)) nan = true;
            std::vector<double> Pc = q.P;
            // Eigen LLT semantics: fails only on pivot <= 0 (NaN pivots pass)
            for (int j = 0; j < nv && pd; j++) {
                double d = Pc[(size_t)j * nv + j];
                for (int k = 0; k < j; k++) d -= Pc[(size_t)j * nv + k] * Pc[(size_t)j * nv + k];
                if (d <= 0) { pd = false; break; }
                d = std::sqrt(d);
                Pc[(size_t)j * nv + j] = d;
                for (int i = j + 1; i < nv; i++) {
                    double s = Pc[(size_t)i * nv + j];
                    for (int k = 0; k < j; k++) s -= Pc[(size_t)i * nv + k] * Pc[(size_t)j * nv + k];
                    Pc[(size_t)i * nv + j] = s / d;
                }
            }
            if (!pd) { status = NON_PD_HESSIAN; status_set = true; break; }
            if (nan) { status = NAN_HESSIAN; status_set = true; break; }
            std::vector<double> st;
            int qit = 0;
            int qs = solve_dense_ipm(q, st, &qit);
            if (g_trace && it < 4) { g_trace[8 * it] = qs; g_trace[8 * it + 1] = qit; }
            if (qs == 0) step = st; else { status = qs; status_set = true; }  // Q6: keep old step
            if (p.do_SOC) {  // :506-535, on whatever step_ holds, even after a failed QP
                int sit = 0;
                const int ss = soc_dense(o, q, guess, recs, ucur, step, st, &sit);
                if (ss == 0) step = st; else { status = ss; status_set = true; }
            }
            if (bfgs) {  // A^T y = -(B step + q) of the QP just solved (dense product)
                std::vector<double> Bs(nv, 0.0);
                for (int a = 0; a < nv; a++) {
                    double t = 0;
                    for (int b = 0; b < nv; b++) t += q.P[(size_t)a * nv + b] * step[b];
                    Bs[a] = t;
                }
                for (int i = 0; i < nv; i++) qd[i] = -(Bs[i] + q.g[i]);  // reused below as A^T y
            }
        } else {
            StructQP S;
            build_struct_qp(o, guess, recs, ucur, S);
            if (bfgs) {  // the QP keeps the Hessian of iteration 0 (setQP without Hess_, :441-442)
                if (it == 0 || bfgs_restart) S0 = S;
                else for (int k = 0; k <= N; k++) std::memcpy(S.st[k].H, S0.st[k].H, sizeof S.st[k].H);
                for (int k = 0; k <= N; k++) {
                    for (int a = 0; a < NX; a++) qd[(size_t)NX * k + a] = S.st[k].h[a];
                    if (k < N) for (int b = 0; b < NU; b++) qd[(size_t)NX * (N + 1) + NU * k + b] = S.st[k].h[NXA + b];
                }
                bfgs_grad(it);
                if (bfgs_nan) nan = true;
            }
            // PD check on the block structure: state blocks and the per-component tridiagonal input blocks
            for (int k = 0; k <= N && pd; k++) {
                double Q[NX * NX];
                for (int a = 0; a < NX; a++) for (int b = 0; b < NX; b++) { Q[a * NX + b] = S.st[k].H[a * NZ + b]; if (std::isnan(Q[a * NX + b])) nan = true; }
                bool ok = true;
                for (int j = 0; j < NX && ok; j++) {  // LLT pivots (NaN passes, as Eigen)
                    double d = Q[j * NX + j];
                    for (int kk = 0; kk < j; kk++) d -= Q[j * NX + kk] * Q[j * NX + kk];
                    if (d <= 0) { ok = false; break; }
                    d = std::sqrt(d); Q[j * NX + j] = d;
                    for (int i = j + 1; i < NX; i++) { double s = Q[i * NX + j]; for (int kk = 0; kk < j; kk++) s -= Q[i * NX + kk] * Q[j * NX + kk]; Q[i * NX + j] = s / d; }
                }
                if (!ok) pd = false;
            }
            for (int b = 0; b < NU && pd; b++) {
                double prev_l = 0;  // L_{k,k-1}
                double prev_d = 0;
                for (int k = 0; k < N; k++) {
                    double dk = S.st[k].H[(NXA + b) * NZ + NXA + b];
                    if (std::isnan(dk)) nan = true;
                    double off = (k >= 1 && b < DOF) ? S.st[k].H[(NXA + b) * NZ + NX + b] : 0.0;
                    double l = (k >= 1) ? off / prev_d : 0.0;
                    double d = dk - l * l;
                    if (d <= 0) { pd = false; break; }
                    prev_d = std::sqrt(d);
                    prev_l = l;
                }
                (void)prev_l;
            }
            if (!pd) { status = NON_PD_HESSIAN; status_set = true; break; }
            if (nan) { status = NAN_HESSIAN; status_set = true; break; }
            std::vector<double> st;
            int qit = 0;
            int qs = solve_struct_ipm(S, st, &qit, bfgs ? &lr : nullptr);
            if (g_trace && it < 4) { g_trace[8 * it] = qs; g_trace[8 * it + 1] = qit; }
            if (qs == 0) step = st; else { status = qs; status_set = true; }
            if (p.do_SOC) {  // :506-535
                int sit = 0;
                const int ss = soc_struct(o, S, guess, recs, ucur, step, st, &sit, bfgs ? &lr : nullptr);
                if (ss == 0) step = st; else { status = ss; status_set = true; }
            }
            if (bfgs) {  // A^T y = -(B step + q)
                std::vector<double> Bs;
                bfgs_hess_mul(S0, lr, step, Bs);
                for (int i = 0; i < nv; i++) qd[i] = -(Bs[i] + qd[i]);
            }
        }
        // filterLineSearch :759-808
        bool accepted = true;
        double alpha = 1.0;
        for (int ls = 0; ls < p.line_search_max_iter; ls++) {
            if (!accepted) { alpha *= p.line_search_tau; continue; }  // later trials cannot be accepted (Q5)
            denorm_add(o, guess, step, alpha, trial.data());
            DenseQP q;
            set_qp(o, trial.data(), recs, ucur, false, q);
            Filter f{q.obj, constraint_norm(q, p.vio_floor)};
            if (g_trace && it < 4 && ls == 0) { g_trace[8 * it + 2] = f.obj; g_trace[8 * it + 3] = f.vio; }
            for (size_t j = 0; j < filter.size(); j++)
                if (f.obj >= filter[j].obj && f.vio >= filter[j].vio) { accepted = false; break; }
            if (accepted) {
                std::vector<Filter> nf;
                for (size_t j = 0; j < filter.size(); j++)
                    if (f.obj > filter[j].obj || f.vio > filter[j].vio) nf.push_back(filter[j]);
                nf.push_back(f);
                filter = nf;
                break;
            } else {
                alpha *= p.line_search_tau;
            }
        }
        // take step :549-551
        if (bfgs) {  // lambda += alpha (y - lambda) as A^T lambda; step_prev = alpha step (:550-555)
            for (int i = 0; i < nv; i++) {
                g_lam[i] = g_lam[i] + alpha * (qd[i] - g_lam[i]);
                step_prev[i] = alpha * step[i];
            }
        }
        denorm_add(o, guess, step, alpha, trial.data());
        std::memcpy(guess, trial.data(), sizeof(double) * (N + 1) * NXU);
        double nrm = 0;
        for (int i = 0; i < nv; i++) nrm = std::max(nrm, std::fabs(step[i]));
        double pn = alpha * nrm;
        if (g_trace && it < 4) { g_trace[8 * it + 4] = (alpha == 1.0) ? 1 : 0; g_trace[8 * it + 5] = nrm; g_trace[8 * it + 6] = alpha; g_trace[8 * it + 7] = pn; }
        if (pn < p.eps_prim) { status = SOLVED; status_set = true; break; }
    }
    if (it == p.max_iter) status = MAX_ITER_EXCEEDED;
    (void)status_set;
    if (iters_out) *iters_out = it;
    if (status == SOLVED) std::memcpy(opt_sol, guess, sizeof(double) * (N + 1) * NXU);
    else std::memcpy(opt_sol, zero.data(), sizeof(double) * (N + 1) * NXU);
    return status;
}

// integrator.cpp:29-43
static void rk4(const double* x, const double* u, double ts, double* out) {
    auto f = [&](const double* xx, double* o) {
        for (int j = 0; j < DOF; j++) o[j] = u[j];
        o[IS] = xx[IVS]; o[IVS] = u[IDVS];
    };
    double k1[NX], k2[NX], k3[NX], k4[NX], t[NX];
    f(x, k1);
    for (int i = 0; i < NX; i++) t[i] = x[i] + ts / 2. * k1[i];
    f(t, k2);
    for (int i = 0; i < NX; i++) t[i] = x[i] + ts / 2. * k2[i];
    f(t, k3);
    for (int i = 0; i < NX; i++) t[i] = x[i] + ts * k3[i];
    f(t, k4);
    for (int i = 0; i < NX; i++) out[i] = x[i] + ts * (k1[i] / 6. + k2[i] / 3. + k3[i] / 3. + k4[i] / 6.);
}

// MPC::runMPC_ — mpc.cpp:104-190 for one instance
// runMPC_ up to the solve (mpc.cpp:104-130): projection, warm start, frozen robot records (Q4)
static void prepare_one(const Oracle& o, double* x0, const double* u0, const double* obs, double* guess, int* valid,
                        int* fails, double* recs) {
    const OracleParams& p = o.p;
    const int N = p.N;
    double last_s = x0[IS];
    double ee[3], J[6 * DOF];
    fk(x0, ee, nullptr, nullptr);
    x0[IS] = o.track.project(last_s, ee);
    fk(x0, nullptr, nullptr, J);
    double ev[3] = {0, 0, 0};
    for (int i = 0; i < 3; i++) { double s = 0; for (int j = 0; j < DOF; j++) s += J[DOF * i + j] * u0[j]; ev[i] = s; }
    double dir[3];
    o.track.dpos(x0[IS], dir);
    x0[IVS] = ev[0] * dir[0] + ev[1] * dir[1] + ev[2] * dir[2];
    if (std::fabs(last_s - x0[IS]) > p.guess_max_dist) { *valid = 0; (*fails)++; }
    const double L = o.track.length();
    if (*valid) {  // updateInitialGuess :54-68
        for (int i = 1; i < N; i++) std::memcpy(guess + NXU * (i - 1), guess + NXU * i, sizeof(double) * NXU);
        std::memcpy(guess, x0, sizeof(double) * NX);
        if (N >= 2) std::memcpy(guess + NXU * (N - 1), guess + NXU * (N - 2), sizeof(double) * NXU);  // N = 1: g[-1] in the reference
        rk4(guess + NXU * (N - 1), guess + NXU * (N - 1) + NX, p.Ts, guess + NXU * N);
        for (int b = 0; b < NU; b++) guess[NXU * N + NX + b] = 0.0;
    } else {  // generateNewInitialGuess :79-89
        for (int i = 0; i <= N; i++) {
            std::memcpy(guess + NXU * i, x0, sizeof(double) * NX);
            for (int b = 0; b < NU; b++) guess[NXU * i + NX + b] = 0.0;
        }
        *valid = 1;
    }
    for (int i = 1; i <= N; i++) guess[NXU * i + IS] = std::min(guess[NXU * i + IS], L);  // unwrapInitialGuess
    // setInitialGuess + setEnvData: robot records at the warm start (Q4)
    for (int i = 0; i <= N; i++) robot_record(o, guess + NXU * i, obs, obs[3], &recs[(size_t)REC * i]);
}

static int run_mpc_one(const Oracle& o, double* x0, const double* u0, const double* obs, double* guess, int* valid,
                       int* fails, double* u0_out, double* horizon, int* ok, int* iters) {
    const OracleParams& p = o.p;
    const int N = p.N;
    std::vector<double> recs((size_t)REC * (N + 1));
    prepare_one(o, x0, u0, obs, guess, valid, fails, recs.data());
    std::vector<double> sol((size_t)(N + 1) * NXU);
    int status = solve_ocp(o, guess, recs.data(), u0, sol.data(), iters);
    std::memcpy(guess, sol.data(), sizeof(double) * NXU * (N + 1));  // initial_guess_ = opt_sol
    if (status == SOLVED) { *valid = 1; *fails = 0; }
    else { *valid = 0; (*fails)++; }
    std::memcpy(u0_out, guess + NX, sizeof(double) * NU);
    std::memcpy(horizon, guess, sizeof(double) * NXU * (N + 1));
    *ok = (status == SOLVED || (status == MAX_ITER_EXCEEDED && *fails < 5)) ? 1 : 0;
    return status;
}

}  // namespace orc

using namespace orc;

extern "C" {

void* oracle_create(const OracleParams* p, const char* nn_dir, OracleOptions opt) {
    Oracle* o = new Oracle();
    o->opt = opt;
    o->set_params(p);
    if (nn_dir) {
        std::string d(nn_dir);
        o->self_nn.load(d + "/self", 7, 1, {256, 64});
        o->env_nn.load(d + "/env", 10, 9, {256, 256, 256, 256});
    }
    return o;
}
void oracle_destroy(void* h) { delete (Oracle*)h; }
void oracle_set_params(void* h, const OracleParams* p) { ((Oracle*)h)->set_params(p); }
void oracle_set_track(void* h, int n, const double* X, const double* Y, const double* Z, const double* R9) {
    Oracle* o = (Oracle*)h;
    std::vector<double> x(X, X + n), y(Y, Y + n), z(Z, Z + n);
    std::vector<std::array<double, 9>> R(n);
    for (int i = 0; i < n; i++) std::memcpy(R[i].data(), R9 + 9 * i, 72);
    o->track.fit(x, y, z, R);
}
double oracle_track_length(void* h) { return ((Oracle*)h)->track.length(); }
void oracle_track_path(void* h, double* s, double* X, double* Y, double* Z, double* R9) {
    Oracle* o = (Oracle*)h;
    for (int i = 0; i < N_SPLINE; i++) {
        s[i] = o->track.s[i]; X[i] = o->track.X[i]; Y[i] = o->track.Y[i]; Z[i] = o->track.Z[i];
        std::memcpy(R9 + 9 * i, o->track.R[i].data(), 72);
    }
}
void oracle_fk(const double* q, double* pos3, double* R9, double* J42) { fk(q, pos3, R9, J42); }
double oracle_manipulability(const double* q) { return manipulability(q); }
void oracle_fk_frame(const double* q, int frame, double* pos3, double* R9, double* J42) { fk_frame(q, frame, pos3, R9, J42); }
double oracle_manip_from_J(const double* J) { return manip_of_J(J); }  // robot_model.cpp:431-435, J 6 x DOF
void oracle_dmanipulability(const double* q, double* d7) { dmanipulability(q, d7); }
void oracle_self_mlp(void* h, const double* q7, double* d, double* grad7) { ((Oracle*)h)->self_nn.eval(q7, d, grad7); }
void oracle_env_mlp(void* h, const double* in10, double* d9, double* jac90) { ((Oracle*)h)->env_nn.eval(in10, d9, jac90); }
void oracle_spline_eval(void* h, double s, double* pos, double* d, double* dd, double* R9, double* dR) {
    Oracle* o = (Oracle*)h;
    o->track.pos(s, pos); o->track.dpos(s, d); o->track.ddpos(s, dd); o->track.rot(s, R9); o->track.drot(s, dR);
}
double oracle_project(void* h, double s, const double* ee3) { return ((Oracle*)h)->track.project(s, ee3); }
void oracle_robot_record(void* h, const double* q7, const double* obs3, double obs_r, double* rec) {
    robot_record(*(Oracle*)h, q7, obs3, obs_r, rec);
}
void oracle_stage_cost(void* h, const double* x9, const double* u8, const double* rec, int k, double* obj, double* fx,
                       double* fu, double* fxx, double* fuu, double* fxu) {
    CostOut c;
    stage_cost(*(Oracle*)h, x9, u8, rec, k, true, c);
    *obj = c.obj;
    std::memcpy(fx, c.fx, sizeof c.fx); std::memcpy(fu, c.fu, sizeof c.fu);
    std::memcpy(fxx, c.fxx, sizeof c.fxx); std::memcpy(fuu, c.fuu, sizeof c.fuu); std::memcpy(fxu, c.fxu, sizeof c.fxu);
}
void oracle_stage_constraints(void* h, const double* x9, const double* u8, const double* rec, int k, double* c, double* l,
                              double* u, double* cx, double* cu) {
    ConOut co;
    stage_constraints(*(Oracle*)h, x9, u8, rec, k, true, co);
    std::memcpy(c, co.c, sizeof co.c); std::memcpy(l, co.l, sizeof co.l); std::memcpy(u, co.u, sizeof co.u);
    std::memcpy(cx, co.cx, sizeof co.cx); std::memcpy(cu, co.cu, sizeof co.cu);
}
double oracle_dense_qp(void* h, const double* guess, const double* recs, const double* u_current, double* P, double* g,
                       double* A, double* c, double* l, double* u) {
    Oracle* o = (Oracle*)h;
    DenseQP q;
    set_qp(*o, guess, recs, u_current, true, q);
    std::memcpy(P, q.P.data(), q.P.size() * 8); std::memcpy(g, q.g.data(), q.g.size() * 8);
    std::memcpy(A, q.A.data(), q.A.size() * 8); std::memcpy(c, q.c.data(), q.c.size() * 8);
    std::memcpy(l, q.l.data(), q.l.size() * 8); std::memcpy(u, q.u.data(), q.u.size() * 8);
    return q.obj;
}
int oracle_solve_qp(void* h, int mode, const double* guess, const double* recs, const double* u_current, double* step,
                    int* iters) {
    Oracle* o = (Oracle*)h;
    std::vector<double> st;
    int rc;
    if (mode == 1) {
        DenseQP q;
        set_qp(*o, guess, recs, u_current, true, q);
        rc = solve_dense_ipm(q, st, iters);
    } else {
        StructQP S;
        build_struct_qp(*o, guess, recs, u_current, S);
        rc = solve_struct_ipm(S, st, iters);
    }
    if (rc == 0) std::memcpy(step, st.data(), st.size() * 8);
    return rc;
}
// One QP with low-rank Hessian terms B = H + sum_j lrc_j u_j u_j^T (u_j in the horizon layout [(N+1)][x | u],
// u_N = 0): the damped-BFGS QP form.  mode 0: Riccati + Woodbury, 1: dense Hessian.
int oracle_solve_qp_lr(void* h, int mode, const double* guess, const double* recs, const double* u_current, int nlr,
                       const double* lr, const double* lrc, double* step, int* iters) {
    Oracle* o = (Oracle*)h;
    const int N = o->N(), nv = o->nvar();
    std::vector<double> st;
    int rc;
    std::vector<std::vector<double>> ud(nlr, std::vector<double>(nv, 0.0));
    for (int j = 0; j < nlr; j++)
        for (int k = 0; k <= N; k++) {
            for (int a = 0; a < NX; a++) ud[j][(size_t)NX * k + a] = lr[((size_t)j * (N + 1) + k) * NXU + a];
            if (k < N)
                for (int b = 0; b < NU; b++) ud[j][(size_t)NX * (N + 1) + NU * k + b] = lr[((size_t)j * (N + 1) + k) * NXU + NX + b];
        }
    if (mode == 1) {
        DenseQP q;
        set_qp(*o, guess, recs, u_current, true, q);
        for (int j = 0; j < nlr; j++)
            for (int a = 0; a < nv; a++)
                for (int b = 0; b < nv; b++) q.P[(size_t)a * nv + b] += lrc[j] * ud[j][a] * ud[j][b];
        rc = solve_dense_ipm(q, st, iters);
    } else {
        StructQP S;
        build_struct_qp(*o, guess, recs, u_current, S);
        LowRank L;
        for (int j = 0; j < nlr; j++) {
            std::vector<double> z;
            dense_to_stage(N, ud[j].data(), z);
            L.u.push_back(z);
            L.c.push_back(lrc[j]);
        }
        rc = solve_struct_ipm(S, st, iters, &L);
    }
    if (rc == 0) std::memcpy(step, st.data(), st.size() * 8);
    return rc;
}
// SecondOrderCorrection QP (osqp_interface.cpp:658-681) after a first step step_in: mode 0 structured, 1 dense
int oracle_solve_soc(void* h, int mode, const double* guess, const double* recs, const double* u_current,
                     const double* step_in, double* step_out, int* iters) {
    Oracle* o = (Oracle*)h;
    std::vector<double> step(step_in, step_in + o->nvar()), st;
    int rc;
    if (mode == 1) {
        DenseQP q;
        set_qp(*o, guess, recs, u_current, true, q);
        rc = soc_dense(*o, q, guess, recs, u_current, step, st, iters);
    } else {
        StructQP S;
        build_struct_qp(*o, guess, recs, u_current, S);
        rc = soc_struct(*o, S, guess, recs, u_current, step, st, iters);
    }
    if (rc == 0) std::memcpy(step_out, st.data(), st.size() * 8);
    return rc;
}
void oracle_rk4(const double* x9, const double* u8, double ts, double* out9) { rk4(x9, u8, ts, out9); }
void oracle_sim_time_step(const double* x9, const double* u8, double ts, double* out9) {  // integrator.cpp:55-68
    const double fine = 0.001;
    int steps = (int)(ts / fine);
    double x[NX];
    std::memcpy(x, x9, sizeof(double) * NX);
    for (int i = 0; i < steps; i++) { double t[NX]; rk4(x, u8, fine, t); std::memcpy(x, t, sizeof(double) * NX); }
    std::memcpy(out9, x, sizeof(double) * NX);
}
int oracle_run_mpc_trace(void* h, int B, double* x0, const double* u0, const double* obs, double* guess, int* valid,
                         int* fails, double* u0_out, double* horizon, int* status, int* ok, int* sqp_iters, double* trace) {
    Oracle* o = (Oracle*)h;
    const int N = o->p.N;
#ifdef _OPENMP
    int nt = o->opt.nthreads > 0 ? o->opt.nthreads : 1;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 4)
#endif
    for (int b = 0; b < B; b++) {
        int it = 0;
        g_trace = trace ? trace + (size_t)32 * b : nullptr;
        if (g_trace) for (int i = 0; i < 32; i++) g_trace[i] = 0.0;
        status[b] = run_mpc_one(*o, x0 + NX * b, u0 + NU * b, obs + 4 * b, guess + (size_t)NXU * (N + 1) * b, valid + b,
                                fails + b, u0_out + NU * b, horizon + (size_t)NXU * (N + 1) * b, ok + b, &it);
        if (sqp_iters) sqp_iters[b] = it;
        g_trace = nullptr;
    }
    return 0;
}
int oracle_run_mpc(void* h, int B, double* x0, const double* u0, const double* obs, double* guess, int* valid, int* fails,
                   double* u0_out, double* horizon, int* status, int* ok, int* sqp_iters) {
    return oracle_run_mpc_trace(h, B, x0, u0, obs, guess, valid, fails, u0_out, horizon, status, ok, sqp_iters, nullptr);
}
int oracle_rec_size(void) { return REC; }
int oracle_dof(void) { return DOF; }
// CubicSpline (cubic_spline.cpp:126-246) on (x, y): value, first and second derivative at xq
void oracle_cubic_spline(int n, const double* x, const double* y, int regular, int m, const double* xq, double* out3) {
    CubicSpline sp;
    sp.gen(std::vector<double>(x, x + n), std::vector<double>(y, y + n), regular != 0);
    for (int i = 0; i < m; i++) {
        out3[3 * i] = sp.point(xq[i]);
        out3[3 * i + 1] = sp.deriv(xq[i]);
        out3[3 * i + 2] = sp.deriv2(xq[i]);
    }
}
int oracle_prepare(void* h, int B, double* x0, const double* u0, const double* obs, double* guess, int* valid, int* fails,
                   double* recs) {
    Oracle* o = (Oracle*)h;
    const int N = o->p.N;
    for (int b = 0; b < B; b++)
        prepare_one(*o, x0 + NX * b, u0 + NU * b, obs + 4 * b, guess + (size_t)NXU * (N + 1) * b, valid + b, fails + b,
                    recs + (size_t)REC * (N + 1) * b);
    return 0;
}

}  // extern "C"
