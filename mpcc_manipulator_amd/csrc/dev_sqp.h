// dev_sqp.h — the per-stage and per-instance pieces of one SQP iteration (osqp_interface.cpp:431-574)
// that run around the QP solve: QP assembly of a stage, the filter line-search trial of a stage, the
// filter decision and the step/termination of an instance.
//
// Shared by the lane-per-stage kernels of kernels.hip and the fused per-instance SQP kernel k_sqp
// (ipm.hip).  All of it follows the oracle's operation order without FP contraction, so the discrete
// decisions (filter comparisons, termination) see the same values as the CPU oracle: kernels.hip is
// built with -ffp-contract=off, and ipm.hip includes this header under #pragma clang fp contract(off).
#pragma once
#include "dev_cost.h"
#include "kernels.h"

namespace mpcc {

// ------------------------------------------------------------------------------------------------
// k_setqp: stage QP record (setCost + setDynamics + setBounds + setPolytopicConstraints,
// osqp_interface.cpp:129-344) in the stage-structured normalized form.
// ------------------------------------------------------------------------------------------------
// keep_hess (damped BFGS, SQP iteration >= 1): the state Hessian block and its NaN / PD flags stay those of
// SQP iteration 0 (setQP is called without the Hessian, osqp_interface.cpp:441-442); the input diagonal is
// constant and is rewritten unchanged.
#ifndef MPCC_SETQP_PRELOAD
#define MPCC_SETQP_PRELOAD (DOF == 7)  // the mobile build's larger arrays cost its fused kernels scratch
#endif
__device__ inline void setqp_stage(const DevConst& c, const SplineView& sp, const double* __restrict__ gb, const RecView& rv, int k,
                                   const double* __restrict__ ucur, double* __restrict__ q, bool keep_hess = false) {
    const mpcc_params& p = c.p;
    const int N = c.N;
    const double* Tx = p.Tx;
    const double* Tu = p.Tu;
    const double* xk = gb + NXU * k;
    const double* uk = gb + NXU * k + NX;
    double fx[NX], fu[NU], fxx[NX * NX], fuu[NU];
    double obj = stage_cost(c, sp, xk, uk, rv, k, true, fx, fu, fxx, fuu);
    // Every guess value the record needs after the cost, loaded before the record's first store: gfx9 counts stores
    // in vmcnt, so a load issued after a store waits for it too (the y-box, ddq and dynamics loops below loaded from
    // the guess between their stores: ~90 of the kernel's 109 full vmcnt waits).  The values and every operation on
    // them are the same.  Addresses past the horizon are clamped to a valid stage and the value is not used.
#if MPCC_SETQP_PRELOAD
    const int kn = k < N ? k + 1 : k, kp = k > 0 ? k - 1 : k;
    double xkv[NX], ukv[NU], xnv[NX], unv[DOF], upv[DOF], ucv[DOF], uib[NX], lub[NX], uub[NX], tub[NX];
#pragma unroll
    for (int a = 0; a < NX; a++) { xkv[a] = xk[a]; xnv[a] = gb[NXU * kn + a]; }
#pragma unroll
    for (int j = 0; j < NU; j++) ukv[j] = uk[j];
#pragma unroll
    for (int j = 0; j < DOF; j++) { unv[j] = gb[NXU * kn + NX + j]; upv[j] = gb[NXU * kp + NX + j]; ucv[j] = ucur[j]; }
#pragma unroll
    for (int m = 0; m < NX; m++) {
        const int idx = NX * k + m, i = idx / NU, j = idx % NU;
        uib[m] = gb[NXU * (i < N ? i : 0) + NX + j];
        lub[m] = p.lu[j];  // kernel-argument loads at a lane-dependent index: loads like the guess's
        uub[m] = p.uu[j];
        tub[m] = Tu[j];
    }
#define XK(a) xkv[a]
#define UK(j) ukv[j]
#define UN(j) unv[j]
#define UP(j) upv[j]
#define XN(a) xnv[a]
#define UC(j) ucv[j]
#define UI(m, i, j) uib[m]
#define LU(m, j) lub[m]
#define UU(m, j) uub[m]
#define TU(m, j) tub[m]
#else
#define XK(a) xk[a]
#define UK(j) uk[j]
#define UN(j) gb[NXU * (k + 1) + NX + (j)]
#define UP(j) gb[NXU * (k - 1) + NX + (j)]
#define XN(a) gb[NXU * (k + 1) + (a)]
#define UC(j) ucur[j]
#define UI(m, i, j) gb[NXU * (i) + NX + (j)]
#define LU(m, j) p.lu[j]
#define UU(m, j) p.uu[j]
#define TU(m, j) Tu[j]
#endif
    int flag = keep_hess ? ((int)q[QS_FLAG] & 3) : 0;
    for (int a = 0; a < NX; a++) {
        q[QS_q + a] = Tx[a] * fx[a];
        if (keep_hess) continue;
        for (int bb = 0; bb < NX; bb++) {
            double v = Tx[a] * fxx[a * NX + bb] * Tx[bb];
            q[QS_Q + a * NX + bb] = v;
            if (isnan(v)) flag |= 1;
        }
    }
    // PD check of the state block (LLT pivots; NaN pivots pass as in Eigen)
    if (!keep_hess) {
        double L[NX * (NX + 1) / 2];
        int idx = 0;
        for (int i = 0; i < NX; i++)
            for (int j = 0; j <= i; j++) L[idx++] = q[QS_Q + i * NX + j];
        for (int j = 0; j < NX; j++) {
            int jj = j * (j + 1) / 2;
            double dgn = L[jj + j];
            for (int m = 0; m < j; m++) dgn -= L[jj + m] * L[jj + m];
            if (dgn <= 0) { flag |= 2; break; }
            dgn = sqrt(dgn);
            L[jj + j] = dgn;
            for (int i = j + 1; i < NX; i++) {
                int ii = i * (i + 1) / 2;
                double s = L[ii + j];
                for (int m = 0; m < j; m++) s -= L[ii + m] * L[jj + m];
                L[ii + j] = s / dgn;
            }
        }
    }
    const double rddq = p.qp_r_ddq;
    double objd = 0.0;
    if (k < N) {
        for (int j = 0; j < NU; j++) {
            q[QS_r + j] = Tu[j] * fu[j];
            q[QS_R + j] = Tu[j] * fuu[j] * Tu[j];
        }
        // ddq cost (osqp_interface.cpp:166-217)
        if (k != N - 1) {
            double sq = 0;
            for (int j = 0; j < DOF; j++) sq += (UN(j) - UK(j)) * (UN(j) - UK(j));
            objd = rddq * sq;
        }
        for (int j = 0; j < DOF; j++) {
            double gg;
            if (k == 0) gg = 2. * rddq * (UK(j) - UN(j));
            else if (k == N - 1) gg = 2. * rddq * (UK(j) - UP(j));
            else gg = 2. * rddq * (2. * UK(j) - UN(j) - UP(j));
            q[QS_r + j] += Tu[j] * gg;
            double cii = (k == 0 || k == N - 1) ? 2. * rddq : 4. * rddq;
            q[QS_R + j] += Tu[j] * cii * Tu[j];
        }
        for (int j = 0; j < NU; j++) if (isnan(q[QS_R + j])) flag |= 1;
        // dynamics offset b_k = -c_{k+1} = -Tx^-1 (x_{k+1} - (A x_k + B u_k + g))   (:247)
        for (int a = 0; a < NX; a++) {
            double s1 = 0, s2 = 0;
            for (int m = 0; m < NX; m++) s1 += c.A[a * NX + m] * XK(m);
            for (int m = 0; m < NU; m++) s2 += c.B[a * NU + m] * UK(m);
            double pred = s1 + s2 + 0.0;
            q[QS_B + a] = -((1.0 / Tx[a]) * (XN(a) - pred));
        }
        // ddq rows (setBounds :279-297): v_0[j] (k=0) or v_k[j]-v_{k-1}[j] within (l - c) / coef
        for (int j = 0; j < DOF; j++) {
            double coef = 1. / p.Ts * Tu[j];
            double cc, lo, hi;
            if (k == 0) {
                cc = 1. / p.Ts * UK(j);
                lo = p.lddq[j] + 1. / p.Ts * UC(j);
                hi = p.uddq[j] + 1. / p.Ts * UC(j);
            } else {
                cc = 1. / p.Ts * (UK(j) - UP(j));
                lo = p.lddq[j];
                hi = p.uddq[j];
            }
            q[QS_DLB + j] = (lo - cc) / coef;
            q[QS_DUB + j] = (hi - cc) / coef;
        }
        // polytopic rows (setPolytopicConstraints :302-344); upper bound 0 - c, lower -INF
        int np = 0;
        for (int r = 0; r < NPC; r++) {
            double val, a[DOF], bv[DOF];
#if MPCC_SETQP_PRELOAD
            if (!poly_row(c, ukv, rv, r, &val, true, a, bv)) continue;
#else
            if (!poly_row(c, uk, rv, r, &val, true, a, bv)) continue;
#endif
            double* row = q + QS_POLY + POLY_W * np;
            for (int j = 0; j < DOF; j++) { row[j] = a[j]; row[DOF + j] = bv[j]; }
            row[2 * DOF] = 0.0 - val;
            np++;
        }
        q[QS_NPOLY] = (double)np;
    } else {
        for (int j = 0; j < NU; j++) { q[QS_r + j] = 0.0; q[QS_R + j] = 0.0; }
        for (int a = 0; a < NX; a++) q[QS_B + a] = 0.0;
        for (int j = 0; j < DOF; j++) { q[QS_DLB + j] = -INF; q[QS_DUB + j] = INF; }
        q[QS_NPOLY] = 0.0;
    }
    // box on y_k: state bounds (bounds.cpp:85-103, s trust region) intersected with the Q1 rows
    // (input bounds placed on stacked-state columns NU*i, osqp_interface.cpp:273)
    const double L = sp.L;
    for (int m = 0; m < NX; m++) {
        double lo = p.lx[m], hi = p.ux[m];
        bool lo_inf = lo <= -BIG, hi_inf = hi >= BIG;
        if (m == XS) { lo = fmax(XK(XS) - p.s_trust_region, 0.); hi = fmin(XK(XS) + p.s_trust_region, L); lo_inf = hi_inf = false; }
        double ylo = lo_inf ? -INF : (lo - XK(m)) / Tx[m];
        double yhi = hi_inf ? INF : (hi - XK(m)) / Tx[m];
        const int idx = NX * k + m;
        const int i = idx / NU, j = idx % NU;
        if (i < N) {
            const double ui = UI(m, i, j);
            if (LU(m, j) > -BIG) ylo = fmax(ylo, (LU(m, j) - ui) / TU(m, j));
            if (UU(m, j) < BIG) yhi = fmin(yhi, (UU(m, j) - ui) / TU(m, j));
        }
        q[QS_YLB + m] = ylo;
        q[QS_YUB + m] = yhi;
        const double FEAS = 1e-9;
        if (k == 0) {
            if (ylo > FEAS || yhi < -FEAS) flag |= 4;  // constant rows on y_0 = 0
        } else if (ylo > yhi) {
            flag |= 4;
        }
    }
    q[QS_FLAG] = (double)flag;
    q[QS_OBJ] = obj + objd;
#undef XK
#undef UK
#undef UN
#undef UP
#undef XN
#undef UC
#undef UI
#undef LU
#undef UU
#undef TU
}

// ------------------------------------------------------------------------------------------------
// SecondOrderCorrection (osqp_interface.cpp:506-535, 658-681) of stage k: the QP is solved again with
// the first QP's P, q and A, and the bounds l(x') - d, u(x') - d with d = c(x') - A step at
// x' = OptvarToVector(initial_guess) + step — the normalized step added as is, before any
// deNormalizeStep (:661).  Only the bound fields of the stage record change: dynamics offset, ddq box,
// polytopic upper bounds and the y box with its feasibility flag.  Same formulas and order as the
// oracle's build_struct_qp(zshift).
// ------------------------------------------------------------------------------------------------
__device__ inline void soc_stage(const DevConst& c, const SplineView& sp, const double* __restrict__ gb,
                                 const double* __restrict__ sb, const RecView& rv, int k, const double* __restrict__ ucur,
                                 double* __restrict__ q) {
    const mpcc_params& p = c.p;
    const int N = c.N;
    const double* Tx = p.Tx;
    const double* Tu = p.Tu;
    auto X = [&](int i, int a) { return gb[NXU * i + a] + sb[NXU * i + a]; };
    auto U = [&](int i, int a) { return gb[NXU * i + NX + a] + sb[NXU * i + NX + a]; };  // the step's u_N is 0
    auto Y = [&](int i, int a) { return sb[NXU * i + a]; };
    auto V = [&](int i, int a) { return sb[NXU * i + NX + a]; };
    double xk[NX], uk[NU];
    for (int a = 0; a < NX; a++) xk[a] = X(k, a);
    for (int a = 0; a < NU; a++) uk[a] = U(k, a);
    int flag = ((int)q[QS_FLAG]) & 3;  // the Hessian bits of the first QP stay
    if (k < N) {
        for (int a = 0; a < NX; a++) {  // b' = -c_{k+1}(x') + (y_{k+1} - M y_k - G v_k)
            double s1 = 0, s2 = 0;
            for (int m = 0; m < NX; m++) s1 += c.A[a * NX + m] * xk[m];
            for (int m = 0; m < NU; m++) s2 += c.B[a * NU + m] * uk[m];
            double pred = s1 + s2 + 0.0;
            const double bk = -((1.0 / Tx[a]) * (X(k + 1, a) - pred));
            double ay = 0, gv = 0;
            for (int m = 0; m < NX; m++) ay += c.M[a * NX + m] * Y(k, m);
            for (int m = 0; m < NU; m++) gv += c.G[a * NU + m] * V(k, m);
            q[QS_B + a] = bk + (Y(k + 1, a) - ay - gv);
        }
        for (int j = 0; j < DOF; j++) {  // ddq rows: + v_k[j] - v_{k-1}[j] (k = 0: v_0[j])
            double coef = 1. / p.Ts * Tu[j];
            double cc, lo, hi;
            if (k == 0) {
                cc = 1. / p.Ts * uk[j];
                lo = p.lddq[j] + 1. / p.Ts * ucur[j];
                hi = p.uddq[j] + 1. / p.Ts * ucur[j];
            } else {
                cc = 1. / p.Ts * (uk[j] - U(k - 1, j));
                lo = p.lddq[j];
                hi = p.uddq[j];
            }
            const double sh = (k == 0) ? V(0, j) : V(k, j) - V(k - 1, j);
            q[QS_DLB + j] = (lo - cc) / coef + sh;
            q[QS_DUB + j] = (hi - cc) / coef + sh;
        }
        int np = 0;  // polytopic rows: + a . y_k[0:DOF] + bv . v_k[0:DOF]
        for (int r = 0; r < NPC; r++) {
            double val;
            if (!poly_row(c, uk, rv, r, &val, false, nullptr, nullptr)) continue;
            double* row = q + QS_POLY + POLY_W * np;
            double sh = 0;
            for (int j = 0; j < DOF; j++) sh += row[j] * Y(k, j);
            for (int j = 0; j < DOF; j++) sh += row[DOF + j] * V(k, j);
            row[2 * DOF] = (0.0 - val) + sh;
            np++;
        }
    }
    const double L = sp.L;  // y box at x', + y_k[m] (finite bounds only)
    for (int m = 0; m < NX; m++) {
        double lo = p.lx[m], hi = p.ux[m];
        bool lo_inf = lo <= -BIG, hi_inf = hi >= BIG;
        if (m == XS) { lo = fmax(xk[XS] - p.s_trust_region, 0.); hi = fmin(xk[XS] + p.s_trust_region, L); lo_inf = hi_inf = false; }
        double ylo = lo_inf ? -INF : (lo - xk[m]) / Tx[m];
        double yhi = hi_inf ? INF : (hi - xk[m]) / Tx[m];
        const int idx = NX * k + m;
        const int i = idx / NU, j = idx % NU;
        if (i < N) {
            const double ui = U(i, j);
            if (p.lu[j] > -BIG) ylo = fmax(ylo, (p.lu[j] - ui) / Tu[j]);
            if (p.uu[j] < BIG) yhi = fmin(yhi, (p.uu[j] - ui) / Tu[j]);
        }
        if (ylo > -BIG) ylo = ylo + Y(k, m);
        if (yhi < BIG) yhi = yhi + Y(k, m);
        q[QS_YLB + m] = ylo;
        q[QS_YUB + m] = yhi;
        const double FEAS = 1e-9;
        if (k == 0) {
            if (ylo > FEAS || yhi < -FEAS) flag |= 4;
        } else if (ylo > yhi) {
            flag |= 4;
        }
    }
    q[QS_FLAG] = (double)flag;
}

// ------------------------------------------------------------------------------------------------
// filterLineSearch trial (osqp_interface.cpp:759-808) of stage k of instance b: objective and l1
// constraint violation (:824-833) of setQP(obj, constr) at guess + alpha * T * step, with the frozen
// robot record (Q4).  Rows owned by stage k: dynamics block k, state bounds k, input bounds (Q1) k,
// ddq block k, polytopic block k.  out = {obj, ddq objective, sum (l - c)^+, sum (c - u)^+}.
// ------------------------------------------------------------------------------------------------
__device__ inline void trial_stage(const DevConst& c, const DevBuffers& d, int b, int k, double alpha,
                                   const double* __restrict__ ucur, double* out) {
    const int N = c.N;
    const mpcc_params& p = c.p;
    const SplineView sp = spl_of(c.spl, b);
    const double* gb = d.guess + (size_t)b * (N + 1) * NXU;
    const double* sb = d.step + (size_t)b * (N + 1) * NXU;
    auto tx = [&](int i, int a) { return gb[NXU * i + a] + alpha * (p.Tx[a] * sb[NXU * i + a]); };
    auto tu = [&](int i, int a) {
        return (i < N) ? gb[NXU * i + NX + a] + alpha * (p.Tu[a] * sb[NXU * i + NX + a]) : gb[NXU * i + NX + a];
    };
    double x[NX], u[NU];
    for (int a = 0; a < NX; a++) x[a] = tx(k, a);
    for (int a = 0; a < NU; a++) u[a] = tu(k, a);
    RecView rv{d.rec + (size_t)b * (N + 1) + k, c.S};
    double fdum[NX], udum[NU], hdum[NX * NX], rdum[NU];
    double obj = stage_cost(c, sp, x, u, rv, k, false, fdum, udum, hdum, rdum);
    double objd = 0;
    if (k < N && k != N - 1) {
        double sq = 0;
        for (int j = 0; j < DOF; j++) { double dlt = tu(k + 1, j) - u[j]; sq += dlt * dlt; }
        objd = p.qp_r_ddq * sq;
    }
    double lo = 0, up = 0;  // sum (l - c)^+ and sum (c - u)^+ (parity policy P1: noise floor per row)
    const double vf = p.vio_floor;
    auto vfloor = [](double v, double f) { return (v > f) ? v : 0.0; };
    if (k >= 1) {  // dynamics rows, l = u = 0
        double xp[NX], up_[NU];
        for (int a = 0; a < NX; a++) xp[a] = tx(k - 1, a);
        for (int a = 0; a < NU; a++) up_[a] = tu(k - 1, a);
        for (int a = 0; a < NX; a++) {
            double s1 = 0, s2 = 0;
            for (int m = 0; m < NX; m++) s1 += c.A[a * NX + m] * xp[m];
            for (int m = 0; m < NU; m++) s2 += c.B[a * NU + m] * up_[m];
            double cv = (1.0 / p.Tx[a]) * (x[a] - (s1 + s2 + 0.0));
            lo += vfloor(fmax(0.0 - cv, 0.0), vf);
            up += vfloor(fmax(cv - 0.0, 0.0), vf);
        }
    }
    for (int a = 0; a < NX; a++) {  // state bounds
        double l = p.lx[a], h = p.ux[a];
        if (a == XS) { l = fmax(x[XS] - p.s_trust_region, 0.); h = fmin(x[XS] + p.s_trust_region, sp.L); }
        lo += vfloor(fmax(l - x[a], 0.0), vf);
        up += vfloor(fmax(x[a] - h, 0.0), vf);
    }
    if (k < N) {
        for (int a = 0; a < NU; a++) {  // input bounds (constr = u, :274)
            lo += vfloor(fmax(p.lu[a] - u[a], 0.0), vf);
            up += vfloor(fmax(u[a] - p.uu[a], 0.0), vf);
        }
        for (int j = 0; j < DOF; j++) {  // ddq rows
            double cv, l, h;
            if (k == 0) {
                cv = 1. / p.Ts * u[j];
                l = p.lddq[j] + 1. / p.Ts * ucur[j];
                h = p.uddq[j] + 1. / p.Ts * ucur[j];
            } else {
                cv = 1. / p.Ts * (u[j] - tu(k - 1, j));
                l = p.lddq[j];
                h = p.uddq[j];
            }
            lo += vfloor(fmax(l - cv, 0.0), vf);
            up += vfloor(fmax(cv - h, 0.0), vf);
        }
        for (int r = 0; r < NPC; r++) {  // polytopic: l = -INF, u = 0
            double val;
            if (!poly_row(c, u, rv, r, &val, false, nullptr, nullptr)) continue;
            lo += vfloor(fmax(-INF - val, 0.0), vf);
            up += vfloor(fmax(val - 0.0, 0.0), vf);
        }
    }
    out[0] = obj;
    out[1] = objd;
    out[2] = lo;
    out[3] = up;
}

// ------------------------------------------------------------------------------------------------
// filter decision, step length, filter update (osqp_interface.cpp:540-574, 759-808) of instance b from
// the per-stage trial records (summed in stage order, as the oracle does)
// ------------------------------------------------------------------------------------------------
__device__ inline void accept_instance(const DevConst& c, const DevBuffers& d, int b) {
    int32_t* si = d.sqi + (size_t)b * SQI;
    const int N = c.N;
    const mpcc_params& p = c.p;
    const double* tr = d.trial + (size_t)b * (N + 1) * 4;
    double obj = 0, lo = 0, up = 0;
    for (int k = 0; k <= N; k++) {
        obj += tr[4 * k];
        obj += tr[4 * k + 1];
        lo += tr[4 * k + 2];
        up += tr[4 * k + 3];
    }
    const double vio = lo + up;
    double* sd = d.sqd + (size_t)b * SQ;
    int nf = si[SQ_NFILT];
    bool accepted = true;
    for (int j = 0; j < nf; j++)
        if (obj >= sd[SQ_FILT + 2 * j] && vio >= sd[SQ_FILT + 2 * j + 1]) { accepted = false; break; }
    double alpha = 1.0;
    if (accepted) {
        int m = 0;
        for (int j = 0; j < nf; j++) {
            double fo = sd[SQ_FILT + 2 * j], fv = sd[SQ_FILT + 2 * j + 1];
            if (obj > fo || vio > fv) { sd[SQ_FILT + 2 * m] = fo; sd[SQ_FILT + 2 * m + 1] = fv; m++; }
        }
        if (m < MAX_FILT) { sd[SQ_FILT + 2 * m] = obj; sd[SQ_FILT + 2 * m + 1] = vio; m++; }
        si[SQ_NFILT] = m;
    } else {
        for (int i = 0; i < p.line_search_max_iter; i++) alpha *= p.line_search_tau;
    }
    sd[SQ_ALPHA] = alpha;
    si[SQ_REJECT] = accepted ? 0 : 1;
    if (d.dbg_trace && si[SQ_ITER] < TRACE_IT) {
        double* trc = d.dbg_trace + ((size_t)b * TRACE_IT + si[SQ_ITER]) * TRACE_W;
        trc[0] = si[SQ_QPSTAT]; trc[1] = si[SQ_IPMIT]; trc[2] = obj; trc[3] = vio; trc[4] = accepted ? 1 : 0;
    }
}

// guess += alpha * deNormalizeStep(step) for element e of the (N+1) x NXU horizon of instance b
// (osqp_interface.cpp:549-552, 859-869); returns |step_e| for the termination norm (0 for u_N)
__device__ __forceinline__ double apply_elem(const DevConst& c, const DevBuffers& d, int b, int e, double alpha) {
    const int N = c.N;
    const int k = e / NXU, a = e - NXU * k;
    if (k == N && a >= NX) return 0.0;
    double* g = d.guess + (size_t)b * (N + 1) * NXU;
    const double* st = d.step + (size_t)b * (N + 1) * NXU;
    const double T = (a < NX) ? c.p.Tx[a] : c.p.Tu[a - NX];
    g[e] = g[e] + alpha * (T * st[e]);
    return fabs(st[e]);
}

// apply_elem over elements e0, e0 + stride, ... of instance b, APB at a time: every load of a batch is issued before
// its stores (gfx9 counts stores in vmcnt, so a load after a store waited for it: one HBM round trip per element);
// returns max |step_e| over them
template <int APB>
__device__ inline double apply_range(const DevConst& c, const DevBuffers& d, int b, int e0, int stride, double alpha) {
    const int N = c.N, n = (N + 1) * NXU;
    double* g = d.guess + (size_t)b * n;
    const double* st = d.step + (size_t)b * n;
    double nrm = 0.0;
    for (int base = e0; base < n; base += APB * stride) {
        double gv[APB], sv[APB];
#pragma unroll
        for (int j = 0; j < APB; j++) {
            const int e = min(base + j * stride, n - 1);
            gv[j] = g[e];
            sv[j] = st[e];
        }
#pragma unroll
        for (int j = 0; j < APB; j++) {
            const int e = base + j * stride;
            if (e >= n) break;
            const int k = e / NXU, a = e - NXU * k;
            if (k == N && a >= NX) continue;
            const double T = (a < NX) ? c.p.Tx[a] : c.p.Tu[a - NX];
            g[e] = gv[j] + alpha * (T * sv[j]);
            nrm = fmax(nrm, fabs(sv[j]));
        }
    }
    return nrm;
}

// termination test after the step (osqp_interface.cpp:553-574); nrm = max |step| (order-free)
__device__ inline void finish_iteration(const DevConst& c, const DevBuffers& d, int b, double nrm) {
    int32_t* si = d.sqi + (size_t)b * SQI;
    const double alpha = d.sqd[(size_t)b * SQ + SQ_ALPHA];
    const double pn = alpha * nrm;
    int iter = si[SQ_ITER];
    if (d.dbg_trace && iter < TRACE_IT) {
        double* tr = d.dbg_trace + ((size_t)b * TRACE_IT + iter) * TRACE_W;
        tr[5] = nrm; tr[6] = alpha; tr[7] = pn;
    }
    if (pn < c.p.eps_prim) {
        si[SQ_STATUS] = MPCC_SOLVED;
        si[SQ_ACTIVE] = 0;
        si[SQ_ITER] = iter;
        return;
    }
    iter++;
    si[SQ_ITER] = iter;
    if (iter >= c.p.max_iter) {
        si[SQ_STATUS] = MPCC_MAX_ITER_EXCEEDED;
        si[SQ_ACTIVE] = 0;
    }
}

}  // namespace mpcc
