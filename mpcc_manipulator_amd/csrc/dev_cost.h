// dev_cost.h — per-stage cost and polytopic constraints (one lane = one horizon stage).
//
// Restates Cost::getCost (cost.cpp:290-357 with getErrorInfo :82-117, getContouringCost :119-162,
// getHeadingCost :164-207, getInputCost :209-270, getSingularityCost :272-288) and
// Constraints::getConstraints (constraints.cpp:34-243).  q-dependent quantities come from the robot
// record frozen at the warm start (quirk Q4).  f_xu is identically zero in the reference (all four
// terms setZero it), so no x-u cross block is produced.
#pragma once
#include "dev_model.h"

namespace mpcc {

__device__ __forceinline__ double cubic_blend(double x, double x0, double xf, double y0, double yf) {  // cost.cpp:36-43
    double t = (x - x0) / (xf - x0);
    double t2 = t * t, t3 = t2 * t;
    return y0 + (yf - y0) * (3 * t2 - 2 * t3);
}

struct RecView {  // strided view of one stage's robot record (SoA)
    const double* base;
    int stride;
    __device__ __forceinline__ double operator[](int f) const { return base[(size_t)f * stride]; }
};

// Stage cost.  want: 0 = objective only (line-search trials), 1 = objective + gradient + Hessian.
// fx[NX], fu[NU], fxx[NX*NX] (row-major), fuu_diag[NU]
__device__ inline double stage_cost(const DevConst& c, const SplineView& sp, const double* x, const double* u, const RecView& rec, int k,
                                    bool want, double* fx, double* fu, double* fxx, double* fuu_diag) {
    const mpcc_params& p = c.p;
    const int N = c.N;
    const double mu = rec[R_MU];
    double ratio = fmin(rec[R_SEL] / (p.cost_tol_selcol * 2.0), mu / (p.cost_tol_sing * 2.0));
    double qc = p.q_c, ql = p.q_l, qo = p.q_ori;
    if (ratio <= 1.0) {
        qc = p.q_c * cubic_blend(ratio, 0.5, 1.0, p.q_c_red_ratio, 1.0);
        ql = p.q_l * cubic_blend(ratio, 0.5, 1.0, p.q_l_inc_ratio, 1.0);
        qo = p.q_ori * cubic_blend(ratio, 0.5, 1.0, p.q_ori_red_ratio, 1.0);
    }
    const double s = x[XS], vs = x[XVS];
    double pr[3], T[3], dd[3];
    spline_pos3(sp, s, pr, T, dd);
    const double ddr[3] = {dd[0], dd[1], dd[1]};  // Q2: ddz_ref = ddpos(1)
    double pos[3] = {rec[R_POS], rec[R_POS + 1], rec[R_POS + 2]};
    double et[3] = {pos[0] - pr[0], pos[1] - pr[1], pos[2] - pr[2]};
    double Te = T[0] * et[0] + T[1] * et[1] + T[2] * et[2];
    double el[3] = {Te * T[0], Te * T[1], Te * T[2]};
    double ec[3] = {et[0] - el[0], et[1] - el[1], et[2] - el[2]};
    const double CC0 = (k < N) ? qc : p.q_c_N_mult * qc;
    const double CC1 = ql;
    const double smax = sp.L;
    const double des = (s < smax * p.deacc_ratio) ? p.desired_ee_velocity
                                                  : -p.desired_ee_velocity / (smax * p.deacc_ratio) * (s - smax);
    double obj_c = CC0 * (ec[0] * ec[0] + ec[1] * ec[1] + ec[2] * ec[2]) +
                   CC1 * (el[0] * el[0] + el[1] * el[1] + el[2] * el[2]) + p.q_vs * ((vs - des) * (vs - des));
    // heading (rotation error Log(R_ref^T R_ee))
    double Rref[9], dRref[3], Rcur[9], Rbar[9], w[3];
    spline_rot(sp, s, Rref, want ? dRref : nullptr);
#pragma unroll
    for (int a = 0; a < 9; a++) Rcur[a] = rec[R_ROT + a];
    m3mul_tn(Rref, Rcur, Rbar);
    log_vec(Rbar, w);
    const double wn2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double obj_h = qo * wn2;
    double obj_i = 0;
    if (k != N) {
        double dq2 = 0;
#pragma unroll
        for (int j = 0; j < DOF; j++) dq2 += u[j] * u[j];
        obj_i = p.r_dq * dq2 + p.r_dVs * (u[UVS] * u[UVS]);
    }
    double obj_s = -p.q_sing * mu;
    double obj = obj_c + obj_h + obj_i + obj_s;
    if (!want) return obj;

    // ---- contouring / lag linearization: d_total, d_lag (Q3: |e_l| I), d_cont
    double nel = sqrt(el[0] * el[0] + el[1] * el[1] + el[2] * el[2]);
    double dc[3][NX], dl[3][NX];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        // d_lag = T T^T d_total + (T e^T + |e_l| I) d_T ; d_total q-cols = Jv, s-col = -T ; d_T s-col = ddr
#pragma unroll
        for (int j = 0; j < NX; j++) {
            double dt0 = (j < DOF) ? rec[R_J + 0 * DOF + j] : (j == XS ? -T[0] : 0.0);
            double dt1 = (j < DOF) ? rec[R_J + 1 * DOF + j] : (j == XS ? -T[1] : 0.0);
            double dt2 = (j < DOF) ? rec[R_J + 2 * DOF + j] : (j == XS ? -T[2] : 0.0);
            double dti = (i == 0) ? dt0 : (i == 1 ? dt1 : dt2);
            double a = T[i] * T[0] * dt0 + T[i] * T[1] * dt1 + T[i] * T[2] * dt2;
            double b = 0;
            if (j == XS) {
#pragma unroll
                for (int m = 0; m < 3; m++) b += (T[i] * et[m] + (i == m ? nel : 0.0)) * ddr[m];
            }
            dl[i][j] = a + b;
            dc[i][j] = dti - dl[i][j];
        }
    }
    // ---- heading linearization (Q23: '+' in the J_r^-1 coefficient as written in cost.cpp:188)
    double Jri[9];
    double wn = sqrt(wn2);
    if (wn < 1e-8) {
#pragma unroll
        for (int a = 0; a < 9; a++) Jri[a] = (a % 4 == 0) ? 1.0 : 0.0;
    } else {
        double S[9], S2[9];
        skew3(w, S);
        m3mul(S, S, S2);
        double coef = 1. / wn2 + (1. + cos(wn)) / (2. * wn * sin(wn));
#pragma unroll
        for (int a = 0; a < 9; a++) Jri[a] = ((a % 4 == 0) ? 1.0 : 0.0) + 1. / 2. * S[a] + coef * S2[a];
    }
    double JRt[9];  // J_r^-1 R_cur^T
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            JRt[3 * i + j] = Jri[3 * i] * Rcur[3 * j] + Jri[3 * i + 1] * Rcur[3 * j + 1] + Jri[3 * i + 2] * Rcur[3 * j + 2];
    double dL[3][NX];
#pragma unroll
    for (int i = 0; i < 3; i++) {
#pragma unroll
        for (int j = 0; j < DOF; j++)
            dL[i][j] = JRt[3 * i] * rec[R_J + 3 * DOF + j] + JRt[3 * i + 1] * rec[R_J + 4 * DOF + j] +
                       JRt[3 * i + 2] * rec[R_J + 5 * DOF + j];
        dL[i][XS] = -(JRt[3 * i] * dRref[0] + JRt[3 * i + 1] * dRref[1] + JRt[3 * i + 2] * dRref[2]);
        dL[i][XVS] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < NX; j++) {
        double s1 = dc[0][j] * ec[0] + dc[1][j] * ec[1] + dc[2][j] * ec[2];
        double s2 = dl[0][j] * el[0] + dl[1][j] * el[1] + dl[2][j] * el[2];
        double g = 2.0 * CC0 * s1 + 2.0 * CC1 * s2;
        if (j == XVS) g += 2.0 * p.q_vs * (vs - des);
        double gh = 2.0 * qo * (dL[0][j] * w[0] + dL[1][j] * w[1] + dL[2][j] * w[2]);
        double gs = (j < DOF) ? -p.q_sing * rec[R_DMU + j] : 0.0;
        fx[j] = g + gh + 0.0 + gs;
    }
#pragma unroll
    for (int a = 0; a < NX; a++)
#pragma unroll
        for (int b = a; b < NX; b++) {
            double s1 = dc[0][a] * dc[0][b] + dc[1][a] * dc[1][b] + dc[2][a] * dc[2][b];
            double s2 = dl[0][a] * dl[0][b] + dl[1][a] * dl[1][b] + dl[2][a] * dl[2][b];
            double h = 2.0 * CC0 * s1 + 2.0 * CC1 * s2;
            if (a == XVS && b == XVS) h += 2.0 * p.q_vs;
            double hh = 2.0 * qo * (dL[0][a] * dL[0][b] + dL[1][a] * dL[1][b] + dL[2][a] * dL[2][b]);
            double v = h + hh + 0.0 + 0.0;
            if (a == b) v += 1e-6;
            fxx[a * NX + b] = v;
            fxx[b * NX + a] = v;
        }
#pragma unroll
    for (int j = 0; j < NU; j++) {
        double gi = 0, hi = 0;
        if (k != N) {
            gi = (j < DOF) ? 2.0 * p.r_dq * u[j] : 2.0 * p.r_dVs * u[UVS];
            hi = (j < DOF) ? 2.0 * p.r_dq : 2.0 * p.r_dVs;
        }
        fu[j] = 0.0 + 0.0 + gi + 0.0;
        fuu_diag[j] = 0.0 + 0.0 + hi + 0.0 + 1e-6;
    }
    return obj;
}

// RBF relaxed barrier (constraints.cpp:34-61)
__device__ __forceinline__ double rbf(double delta, double h) {
    if (h >= delta) return -log(h + 1);
    double d1 = delta + 1;
    return -log(d1) - 1 / d1 * (h - delta) + 1 / (2 * (d1 * d1)) * ((h - delta) * (h - delta));
}
__device__ __forceinline__ double drbf(double delta, double h) {
    if (h >= delta) return -1 / (h + 1);
    double d1 = delta + 1;
    return -1 / d1 + 1 / (d1 * d1) * (h - delta);
}

// One polytopic row r of stage k < N: value c(u) and, if want, the normalized linearization
// a[DOF] = c_x[q] * Tx, bv[DOF] = c_u[dq] * Tu.  Returns false if the row is masked (l=-INF,u=+INF).
// Row order: 0 self-collision, 1 singularity, 2..10 env links (config.h:64-74).
__device__ inline bool poly_row(const DevConst& c, const double* u, const RecView& rec, int r, double* val, bool want,
                                double* a, double* bv) {
    const mpcc_params& p = c.p;
    const double delta = -0.5;
    double grad[DOF], h, cu_scale;
    if (r == 0) {
        if (!(p.constraint_mask & MPCC_CON_SELFCOL)) return false;
        double md = 0.01 * rec[R_SEL];
#pragma unroll
        for (int j = 0; j < DOF; j++) grad[j] = 0.01 * rec[R_DSEL + j];
        h = md - p.con_tol_selcol * 0.01;
        cu_scale = 1.0;
    } else if (r == 1) {
        if (!(p.constraint_mask & MPCC_CON_SING)) return false;
#pragma unroll
        for (int j = 0; j < DOF; j++) grad[j] = rec[R_DMU + j];
        h = rec[R_MU] - p.con_tol_sing;
        cu_scale = 1.0;
    } else {
        if (!(p.constraint_mask & MPCC_CON_ENVCOL)) return false;
        int m = r - 2;
        double md = 0.01 * (rec[R_ENV + m] - rec[R_OBSR] * 1.2);
#pragma unroll
        for (int j = 0; j < DOF; j++) grad[j] = 0.01 * rec[R_DENV + DOF * m + j];
        h = md - 0.01 * p.con_tol_envcol;
        cu_scale = 1.0;
    }
    (void)cu_scale;
    double dot = 0;
#pragma unroll
    for (int j = 0; j < DOF; j++) dot += grad[j] * u[j];
    *val = -dot + rbf(delta, h);
    if (want) {
        double dR = drbf(delta, h);
#pragma unroll
        for (int j = 0; j < DOF; j++) {
            a[j] = (dR * grad[j]) * c.p.Tx[j];
            bv[j] = (-grad[j]) * c.p.Tu[j];
        }
    }
    return true;
}

}  // namespace mpcc
