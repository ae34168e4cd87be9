// host_spline.cpp — see host_spline.h.
#include "host_spline.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <stdexcept>

namespace mpcc {

namespace {

constexpr int NSPLINE = 100;  // N_SPLINE, config.h:38
using Mat3 = std::array<double, 9>;

Mat3 mul(const Mat3& A, const Mat3& B) {
    Mat3 C{};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    return C;
}
Mat3 mul_tn(const Mat3& A, const Mat3& B) {
    Mat3 C{};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[3 * i + j] = A[i] * B[j] + A[3 + i] * B[3 + j] + A[6 + i] * B[6 + j];
    return C;
}

// symmetric eigen decomposition of the lower triangle (Jacobi), ascending eigenvalues
void sym_eig3(const double* Rin, double* w, double* V) {
    double A[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) A[3 * i + j] = (i >= j) ? Rin[3 * i + j] : Rin[3 * j + i];
    for (int i = 0; i < 9; i++) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; sweep++) {
        if (std::fabs(A[1]) + std::fabs(A[2]) + std::fabs(A[5]) < 1e-300) break;
        for (int pq = 0; pq < 3; pq++) {
            int p = (pq == 2) ? 1 : 0, q = (pq == 0) ? 1 : 2;
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

void exp_skew(const double* v, double* E) {  // ExpMatrix(skew(v)), Q11
    double sk[9] = {0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0};
    double sk2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) sk2[3 * i + j] = sk[3 * i] * sk[j] + sk[3 * i + 1] * sk[3 + j] + sk[3 * i + 2] * sk[6 + j];
    double vn = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (vn <= 1e-8) {
        for (int i = 0; i < 9; i++) E[i] = ((i % 4 == 0) ? 1.0 : 0.0) + std::cos(vn) * sk[i];
        return;
    }
    double a = std::sin(vn) / vn, b = (1 - std::cos(vn)) / (vn * vn);
    for (int i = 0; i < 9; i++) E[i] = ((i % 4 == 0) ? 1.0 : 0.0) + a * sk[i] + b * sk2[i];
}

struct Cubic {  // CubicSpline (cubic_spline.cpp)
    std::vector<double> x, y, a, b, c, d;
    bool regular = false;
    double dx = 0;
    std::map<double, int> xmap;
    void gen(const std::vector<double>& xin, const std::vector<double>& yin, bool reg) {
        x = xin; y = yin; regular = reg;
        const int n = (int)x.size();
        if (reg) dx = x[1] - x[0];
        else { xmap.clear(); for (int i = 0; i < n; i++) xmap[x[i]] = i; }
        a = y; b.assign(n, 0.0); c.assign(n, 0.0); d.assign(n, 0.0);
        std::vector<double> mu(n, 0.0), h(n, 0.0), alpha(n, 0.0), l(n, 0.0), z(n, 0.0);
        for (int i = 0; i < n - 1; i++) h[i] = x[i + 1] - x[i];
        for (int i = 1; i < n - 1; i++) alpha[i] = 3.0 / h[i] * (a[i + 1] - a[i]) - 3.0 / h[i - 1] * (a[i] - a[i - 1]);
        l[0] = 1.0;
        for (int i = 1; i < n - 1; i++) {
            l[i] = 2.0 * (x[i + 1] - x[i - 1]) - h[i - 1] * mu[i - 1];
            mu[i] = h[i] / l[i];
            z[i] = (alpha[i] - h[i - 1] * z[i - 1]) / l[i];
        }
        for (int i = n - 2; i >= 0; i--) {
            c[i] = z[i] - mu[i] * c[i + 1];
            b[i] = (a[i + 1] - a[i]) / h[i] - (h[i] * (c[i + 1] + 2.0 * c[i])) / 3.0;
            d[i] = (c[i + 1] - c[i]) / (3.0 * h[i]);
        }
    }
    int index(double xx) const {
        if (xx == x.back()) return (int)x.size() - 1;
        if (regular) return (int)std::floor(xx / dx);
        auto it = xmap.upper_bound(xx);
        return (it == xmap.end()) ? -1 : it->second - 1;
    }
    double point(double xx) const {
        xx = std::max(0., std::min(xx, x.back()));
        int i = index(xx);
        double d1 = xx - x[i], d2 = d1 * d1, d3 = d1 * d2;
        if (i == (int)x.size() - 1) return y.back();
        return a[i] + b[i] * d1 + c[i] * d2 + d[i] * d3;
    }
    double deriv(double xx) const {  // getDerivative (cubic_spline.cpp)
        xx = std::max(0., std::min(xx, x.back()));
        int i = index(xx);
        double d1 = xx - x[i], d2 = d1 * d1;
        if (i == (int)x.size() - 1) return 0.;
        return b[i] + 2.0 * c[i] * d1 + 3.0 * d[i] * d2;
    }
    double deriv2(double xx) const {  // getSecondDerivative
        xx = std::max(0., std::min(xx, x.back()));
        int i = index(xx);
        double d1 = xx - x[i];
        if (i == (int)x.size() - 1) return 2.0 * c[i];
        return 2.0 * c[i] + 6.0 * d[i] * d1;
    }
};

struct CubicRot {  // CubicSplineRot (cubic_spline_rot.cpp)
    std::vector<double> x, c, d;
    std::vector<Mat3> R;
    std::vector<std::array<double, 3>> lv;
    bool regular = false;
    double dx = 0;
    std::map<double, int> xmap;
    void gen(const std::vector<double>& xin, const std::vector<Mat3>& Rin, bool reg) {
        x = xin; R = Rin; regular = reg;
        const int n = (int)x.size();
        if (reg) dx = x[1] - x[0];
        else { xmap.clear(); for (int i = 0; i < n; i++) xmap[x[i]] = i; }
        c.assign(n, 0.0); d.assign(n, 0.0); lv.assign(n, {0, 0, 0});
        for (int i = 0; i < n - 1; i++) {
            c[i] = 3.0 / std::pow(x[i + 1] - x[i], 2);
            d[i] = -2.0 / std::pow(x[i + 1] - x[i], 3);
            Mat3 RtR = mul_tn(R[i], R[i + 1]);
            host_log_vec(RtR.data(), lv[i].data());
        }
    }
    int index(double xx) const {
        if (xx == x.back()) return (int)x.size() - 1;
        if (regular) return (int)std::floor(xx / dx);
        auto it = xmap.upper_bound(xx);
        return (it == xmap.end()) ? -1 : it->second - 1;
    }
    Mat3 point(double xx) const {
        xx = std::max(0., std::min(xx, x.back()));
        int i = index(xx);
        if (i == (int)x.size() - 1) return R.back();
        double d1 = xx - x[i], d2 = d1 * d1, d3 = d1 * d2;
        double f = c[i] * d2 + d[i] * d3;
        double v[3] = {lv[i][0] * f, lv[i][1] * f, lv[i][2] * f};
        Mat3 E;
        exp_skew(v, E.data());
        return mul(R[i], E);
    }
    std::array<double, 3> deriv(double xx) const {  // getDerivative (cubic_spline_rot.cpp:239-259)
        xx = std::max(0., std::min(xx, x.back()));
        int i = index(xx);
        if (i == (int)x.size() - 1) return {0, 0, 0};
        double d1 = xx - x[i], d2 = d1 * d1;
        double f = 2.0 * c[i] * d1 + 3.0 * d[i] * d2;
        return {lv[i][0] * f, lv[i][1] * f, lv[i][2] * f};
    }
};

std::vector<double> arc_length(const std::vector<double>& X, const std::vector<double>& Y, const std::vector<double>& Z) {
    const int n = (int)X.size();
    std::vector<double> s(n, 0.0);
    for (int i = 0; i < n - 1; i++) {
        double dx = X[i + 1] - X[i], dy = Y[i + 1] - Y[i], dz = Z[i + 1] - Z[i];
        s[i + 1] = s[i] + std::sqrt(dx * dx + dy * dy + dz * dz);
    }
    return s;
}

std::vector<double> lin_spaced(int n, double lo, double hi) {  // Eigen::VectorXd::LinSpaced
    std::vector<double> v(n);
    const double step = (hi - lo) / double(n - 1);
    const bool flip = std::fabs(hi) < std::fabs(lo);
    for (int i = 0; i < n; i++) {
        if (flip) v[i] = (i == 0) ? lo : hi - double(n - 1 - i) * step;
        else v[i] = (i == n - 1) ? hi : lo + double(i) * step;
    }
    return v;
}

struct Path {
    std::vector<double> s, X, Y, Z;
    std::vector<Mat3> R;
};

Path resample(const Cubic& fx, const Cubic& fy, const Cubic& fz, const CubicRot& fr, double total) {  // :89-119
    Path p;
    p.s = lin_spaced(NSPLINE, 0, total);
    p.X.resize(NSPLINE); p.Y.resize(NSPLINE); p.Z.resize(NSPLINE); p.R.resize(NSPLINE);
    for (int i = 0; i < NSPLINE; i++) {
        p.X[i] = fx.point(p.s[i]);
        p.Y[i] = fy.point(p.s[i]);
        p.Z[i] = fz.point(p.s[i]);
        p.R[i] = fr.point(p.s[i]);
    }
    return p;
}

}  // namespace

void host_log_vec(const double* R, double* v) {  // invskew(LogMatrix(R)), Q10
    const double tr = R[0] + R[4] + R[8];
    v[0] = v[1] = v[2] = 0.0;
    if (std::fabs(tr + 1.0) < 1e-6) {
        double w[3], V[9];
        sym_eig3(R, w, V);
        for (int i = 0; i < 3; i++) {
            if (std::fabs(w[i] - 1.0) < 1e-4) {
                double e0 = V[i], e1 = V[3 + i], e2 = V[6 + i];
                double n = std::sqrt(e0 * e0 + e1 * e1 + e2 * e2);
                v[0] = -(e0 / n) * M_PI; v[1] = -(e1 / n) * M_PI; v[2] = -(e2 / n) * M_PI;
            }
        }
    } else if (std::fabs(tr - 3.0) < 1e-6) {
        // zero
    } else {
        const double th = std::acos((tr - 1.0) / 2.0);
        const double f = 1.0 / 2.0 * th / std::sin(th);
        v[0] = f * (R[7] - R[5]);
        v[1] = f * (R[2] - R[6]);
        v[2] = f * (R[3] - R[1]);
    }
}

void quat_to_rot(double qx, double qy, double qz, double qw, double* R) {
    const double n = std::sqrt(qx * qx + qy * qy + qz * qz + qw * qw);
    const double x = qx / n, y = qy / n, z = qz / n, w = qw / n;
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

SplineTables build_track_spline(int n, const double* X, const double* Y, const double* Z, const double* R9) {
    std::vector<double> x0(X, X + n), y0(Y, Y + n), z0(Z, Z + n);
    std::vector<Mat3> r0(n);
    for (int i = 0; i < n; i++) std::memcpy(r0[i].data(), R9 + 9 * i, sizeof(double) * 9);
    // fitSpline (arc_length_spline.cpp:213-253): two irregular fit/resample passes, final regular fit
    std::vector<double> sa = arc_length(x0, y0, z0);
    double total = sa.back();
    Cubic f1x, f1y, f1z;
    CubicRot f1r;
    f1x.gen(sa, x0, false); f1y.gen(sa, y0, false); f1z.gen(sa, z0, false); f1r.gen(sa, r0, false);
    Path p1 = resample(f1x, f1y, f1z, f1r, total);
    sa = arc_length(p1.X, p1.Y, p1.Z);
    total = sa.back();
    Cubic f2x, f2y, f2z;
    CubicRot f2r;
    f2x.gen(sa, p1.X, false); f2y.gen(sa, p1.Y, false); f2z.gen(sa, p1.Z, false); f2r.gen(sa, p1.R, false);
    Path p2 = resample(f2x, f2y, f2z, f2r, total);
    std::vector<double> R2((size_t)NSPLINE * 9);
    for (int i = 0; i < NSPLINE; i++) std::memcpy(&R2[(size_t)9 * i], p2.R[i].data(), sizeof(double) * 9);
    return build_track_from_path(NSPLINE, p2.s.data(), p2.X.data(), p2.Y.data(), p2.Z.data(), R2.data());
}

SplineTables build_track_from_path(int n, const double* s, const double* X, const double* Y, const double* Z,
                                   const double* R9) {
    if (n != NSPLINE) throw std::invalid_argument("path data must have N_SPLINE = 100 points (config.h:38)");
    for (int i = 1; i < n; i++)
        if (!(s[i] > s[i - 1])) throw std::invalid_argument("path data s must be strictly increasing");
    Path p2;
    p2.s.assign(s, s + n); p2.X.assign(X, X + n); p2.Y.assign(Y, Y + n); p2.Z.assign(Z, Z + n);
    p2.R.resize(n);
    for (int i = 0; i < n; i++) std::memcpy(p2.R[i].data(), R9 + 9 * i, sizeof(double) * 9);
    // final spline fit with fixed delta s (arc_length_spline.cpp:245-252)
    Cubic fx, fy, fz;
    CubicRot fr;
    fx.gen(p2.s, p2.X, true); fy.gen(p2.s, p2.Y, true); fz.gen(p2.s, p2.Z, true); fr.gen(p2.s, p2.R, true);

    SplineTables t;
    t.n = NSPLINE;
    t.delta = p2.s[1] - p2.s[0];
    t.s = p2.s; t.X = p2.X; t.Y = p2.Y; t.Z = p2.Z;
    const Cubic* ax[3] = {&fx, &fy, &fz};
    for (int a = 0; a < 3; a++) { t.a[a] = ax[a]->a; t.b[a] = ax[a]->b; t.c[a] = ax[a]->c; t.d[a] = ax[a]->d; }
    t.R.resize((size_t)NSPLINE * 9);
    for (int i = 0; i < NSPLINE; i++) std::memcpy(&t.R[(size_t)9 * i], p2.R[i].data(), sizeof(double) * 9);
    t.cr = fr.c; t.dr = fr.d;
    t.logv.resize((size_t)NSPLINE * 3);
    for (int i = 0; i < NSPLINE; i++)
        for (int a = 0; a < 3; a++) t.logv[(size_t)3 * i + a] = fr.lv[i][a];
    return t;
}

// ---- host evaluation of the final tables: the device's spline_pos3 / spline_rot / project_on_spline
//      (dev_model.h), i.e. cubic_spline.cpp:126-246, cubic_spline_rot.cpp:216-259, arc_length_spline.cpp:318-379
namespace {
double tab_unwrap(const SplineTables& t, double x) {
    const double L = t.length();
    const double m = (L < x) ? L : x;
    return (0. < m) ? m : 0.;
}
int tab_index(const SplineTables& t, double x) {
    if (x == t.length()) return t.n - 1;
    return (int)std::floor(x / t.delta);
}
}  // namespace

void eval_tables(const SplineTables& t, double s, double* p, double* dp, double* ddp, double* R9, double* dR) {
    const double x = tab_unwrap(t, s);
    const int i = tab_index(t, x);
    const int n = t.n;
    const double d1 = x - t.s[i], d2 = d1 * d1, d3 = d1 * d2;
    for (int a = 0; a < 3; a++) {
        if (i == n - 1) {
            if (p) p[a] = t.a[a][n - 1];
            if (dp) dp[a] = 0.;
            if (ddp) ddp[a] = 2.0 * t.c[a][n - 1];
        } else {
            const double A = t.a[a][i], B = t.b[a][i], C = t.c[a][i], D = t.d[a][i];
            if (p) p[a] = A + B * d1 + C * d2 + D * d3;
            if (dp) dp[a] = B + 2.0 * C * d1 + 3.0 * D * d2;
            if (ddp) ddp[a] = 2.0 * C + 6.0 * D * d1;
        }
    }
    if (i == n - 1) {
        if (R9) for (int a = 0; a < 9; a++) R9[a] = t.R[(size_t)9 * (n - 1) + a];
        if (dR) dR[0] = dR[1] = dR[2] = 0.;
        return;
    }
    const double* lv = &t.logv[(size_t)3 * i];
    const double cr = t.cr[i], dr = t.dr[i];
    if (R9) {
        const double f = cr * d2 + dr * d3;
        double v[3] = {lv[0] * f, lv[1] * f, lv[2] * f}, E[9];
        exp_skew(v, E);
        const double* Ri = &t.R[(size_t)9 * i];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double acc = 0;
                for (int k = 0; k < 3; k++) acc += Ri[3 * r + k] * E[3 * k + c];
                R9[3 * r + c] = acc;
            }
    }
    if (dR) {
        const double f = 2.0 * cr * d1 + 3.0 * dr * d2;
        dR[0] = lv[0] * f; dR[1] = lv[1] * f; dR[2] = lv[2] * f;
    }
}

double project_tables(const SplineTables& t, double proj_max_dist, double s_guess, const double* ee) {
    double pp[3];
    eval_tables(t, s_guess, pp, nullptr, nullptr, nullptr, nullptr);
    double s_opt = s_guess;
    const double dx = ee[0] - pp[0], dy = ee[1] - pp[1], dz = ee[2] - pp[2];
    if (std::sqrt(dx * dx + dy * dy + dz * dz) >= proj_max_dist) {  // far branch (Q12), as the device
        bool any = false;
        double best = 0;
        int bi = 0;
        for (int i = 0; i < t.n; i++) {
            any |= std::fabs(t.s[i] - s_guess) <= proj_max_dist;
            const double ex = t.a[0][i] - ee[0], ey = t.a[1][i] - ee[1], ez = t.a[2][i] - ee[2];
            const double d2 = ex * ex + ey * ey + ez * ez;
            if (i == 0 || d2 < best) { best = d2; bi = i; }
        }
        s_opt = any ? t.s[0] : t.s[bi];
    }
    if (s_opt >= t.length()) return t.length();
    double s_old = s_opt;
    for (int it = 0; it < 20; it++) {
        double p[3], dp[3], ddp[3];
        eval_tables(t, s_opt, p, dp, ddp, nullptr, nullptr);
        const double d0 = p[0] - ee[0], d1 = p[1] - ee[1], d2 = p[2] - ee[2];
        const double jac = 2.0 * d0 * dp[0] + 2.0 * d1 * dp[1] + 2.0 * d2 * dp[2];
        const double hes = 2.0 * dp[0] * dp[0] + 2.0 * d0 * ddp[0] + 2.0 * dp[1] * dp[1] + 2.0 * d1 * ddp[1] +
                           2.0 * dp[2] * dp[2] + 2.0 * d2 * ddp[2];
        s_opt -= jac / hes;
        s_opt = tab_unwrap(t, s_opt);
        if (std::fabs(s_old - s_opt) <= 1e-5) return s_opt;
        s_old = s_opt;
    }
    return s_guess;
}

// CubicSpline / CubicSplineRot fitted to n points and evaluated at m abscissas (host, for tests and the
// C ABI): value, first and second derivative; rotation and its derivative vector
void host_cubic_spline(int n, const double* x, const double* y, bool regular, int m, const double* xq, double* out3) {
    Cubic c;
    c.gen(std::vector<double>(x, x + n), std::vector<double>(y, y + n), regular);
    for (int i = 0; i < m; i++) {
        out3[3 * i] = c.point(xq[i]);
        out3[3 * i + 1] = c.deriv(xq[i]);
        out3[3 * i + 2] = c.deriv2(xq[i]);
    }
}
void host_rot_spline(int n, const double* x, const double* R9, bool regular, int m, const double* xq, double* Rq, double* dRq) {
    std::vector<Mat3> R(n);
    for (int i = 0; i < n; i++) std::copy(R9 + 9 * i, R9 + 9 * i + 9, R[i].begin());
    CubicRot c;
    c.gen(std::vector<double>(x, x + n), R, regular);
    for (int i = 0; i < m; i++) {
        if (Rq) {
            const Mat3 r = c.point(xq[i]);
            std::copy(r.begin(), r.end(), Rq + 9 * i);
        }
        if (dRq) {
            const auto d = c.deriv(xq[i]);
            std::copy(d.begin(), d.end(), dRq + 3 * i);
        }
    }
}

// ExpMatrix(sk) (cubic_spline_rot.cpp:81-95): a zero matrix when sk is not skew-symmetric (the reference
// prints an error and returns Zero), else Exp of invskew(sk) with quirk Q11
void host_exp_matrix(const double* sk, double* E) {
    double n1 = 0, n2 = 0;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) {
            const double a = sk[3 * j + i] + sk[3 * i + j];
            n1 += a * a;
        }
        n2 += sk[4 * i] * sk[4 * i];
    }
    if (std::sqrt(n1) >= 1e-8 || std::sqrt(n2) >= 1e-8) {
        for (int i = 0; i < 9; i++) E[i] = 0.0;
        return;
    }
    const double v[3] = {sk[7], sk[2], sk[3]};  // getInverseSkewVector: (R21, R02, R10)
    exp_skew(v, E);
}

}  // namespace mpcc
