// dev_common.h — shared constants, layouts and small device helpers of the MI355X MPCC engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpcc_engine.h"

namespace mpcc {

constexpr int NX = 9, NU = 8, NPC = 11, DOF = 7, NLINK = 9;   // config.h:29-38
constexpr int NSPL = 100;                                      // N_SPLINE, config.h:38
constexpr double INF = 1e30;                                   // config.h:37
constexpr double BIG = 1e20;   // |bound| >= BIG is an infinite bound (OSQP_INFTY semantics)
constexpr int NMAX = 64;       // largest supported horizon (one lane per stage in the record kernels)

// ---- robot record (RobotData, robot_data.h:13-31) — SoA: rec[field * S + b*(N+1) + k] ----
constexpr int REC = MPCC_REC_SIZE;
constexpr int R_POS = 0, R_ROT = 3, R_J = 12, R_MU = 54, R_DMU = 55, R_SEL = 62, R_DSEL = 63,
              R_OBSR = 70, R_ENV = 71, R_DENV = 80;

// ---- per (instance, stage) QP record, AoS per instance: qs[(b*(N+1)+k)*QS + field] ----
// Stage-structured normalized QP: y = Tx^-1 dx, v = Tu^-1 du.
constexpr int QS_Q = 0;        // 81  Tx f_xx Tx               (osqp_interface.cpp:158)
constexpr int QS_q = 81;       // 9   Tx f_x                   (:157)
constexpr int QS_R = 90;       // 8   diag(Tu f_uu Tu) + ddq diag (:162, :210)
constexpr int QS_r = 98;       // 8   Tu f_u + Tu ddq_grad     (:161, :191)
constexpr int QS_B = 106;      // 9   y_{k+1} = M y_k + G v_k + b_k, b_k = -c_{k+1} (:247)
constexpr int QS_YLB = 115;    // 9   box on y_k (state bounds ∩ Q1 rows)
constexpr int QS_YUB = 124;    // 9
constexpr int QS_DLB = 133;    // 7   ddq rows: v_0[j] (k=0) or v_k[j]-v_{k-1}[j] in [lb, ub]
constexpr int QS_DUB = 140;    // 7
constexpr int QS_NPOLY = 147;  // 1   number of live polytopic rows
constexpr int QS_POLY = 148;   // 11 x 15: a[7] (on y[0:7]), bv[7] (on v[0:7]), ub
constexpr int QS_FLAG = 313;   // 1   bit0: NaN in stage Hessian, bit1: non-PD state block, bit2: infeasible constant rows
constexpr int QS_OBJ = 314;    // 1   stage objective (cost + ddq term)
constexpr int QS = 320;
constexpr int POLY_W = 15;

// ---- IPM state per (instance, stage), AoS: is[(b*(N+1)+k)*IS + field] ----
constexpr int NSLOT = 43;      // 9 y-lower, 9 y-upper, 7 ddq-lower, 7 ddq-upper, 11 poly
constexpr int SL_YL = 0, SL_YU = 9, SL_DL = 18, SL_DU = 25, SL_P = 32;
constexpr int IS_S = 0, IS_L = 43, IS_W = 86, IS_RP = 129, IS_DSA = 172, IS_DLA = 215, IS_COEF = 258,
              IS_RC = 301, IS_DS = 344, IS_DL = 387, IS_BND = 430, IS_ACT = 473;
constexpr int IS_Z = 516;      // 24: y(9) w(7) v(8)
constexpr int IS_DZ = 540;     // 24
constexpr int IS_G0 = 564;     // 24 objective gradient H z + h
constexpr int IS_G = 588;      // 24 step-system gradient
constexpr int IS_U = 612;      // 8x16  U = LF^-1 Gm
constexpr int IS_LF = 740;     // 8x8   chol(F)
constexpr int IS_T = 804;      // 8     LF^-1 f
constexpr int IS = 816;

// ---- per-instance SQP bookkeeping (sqp[b*SQ + field]) ----
constexpr int SQ_STATUS = 0, SQ_ACTIVE = 1, SQ_ITER = 2, SQ_NFILT = 3, SQ_QPSTAT = 4, SQ_IPMIT = 5;
constexpr int SQ_ALPHA = 6;    // double slots start here (stored as double)
constexpr int SQ_FILT = 8;     // filter (obj, vio) pairs
constexpr int MAX_FILT = 64;
constexpr int SQ = SQ_FILT + 2 * MAX_FILT;

// spline table (host-built, arc_length_spline.cpp:213-265): n points, regular grid
// Track spline tables.  One track = 27 n + 2 doubles (n = NSPL): s[n] | a0 b0 c0 d0 | a1 .. | a2 .. |
// R[9n] | cr[n] | dr[n] | logv[3n] | delta | L, padded to SPL_STRIDE.  Instance b uses the track at
// base + b * stride: stride 0 = one shared track (MPC::setTrack), SPL_STRIDE = a track per instance.
constexpr int SPL_A = NSPL, SPL_R = 13 * NSPL, SPL_CR = 22 * NSPL, SPL_DR = 23 * NSPL, SPL_LOGV = 24 * NSPL,
              SPL_DELTA = 27 * NSPL, SPL_L = 27 * NSPL + 1, SPL_STRIDE = 27 * NSPL + 8;
struct SplineDev {
    const double* base;
    long stride;
};
// one track (cubic_spline.cpp / cubic_spline_rot.cpp tables of the final regular fit)
struct SplineView {
    const double* t;
    double delta, L;
    __device__ __forceinline__ double s(int i) const { return t[i]; }
    __device__ __forceinline__ double a(int ax, int i) const { return t[SPL_A + 4 * NSPL * ax + i]; }
    __device__ __forceinline__ double b(int ax, int i) const { return t[SPL_A + 4 * NSPL * ax + NSPL + i]; }
    __device__ __forceinline__ double c(int ax, int i) const { return t[SPL_A + 4 * NSPL * ax + 2 * NSPL + i]; }
    __device__ __forceinline__ double d(int ax, int i) const { return t[SPL_A + 4 * NSPL * ax + 3 * NSPL + i]; }
    __device__ __forceinline__ const double* R(int i) const { return t + SPL_R + 9 * i; }
    __device__ __forceinline__ double cr(int i) const { return t[SPL_CR + i]; }
    __device__ __forceinline__ double dr(int i) const { return t[SPL_DR + i]; }
    __device__ __forceinline__ const double* logv(int i) const { return t + SPL_LOGV + 3 * i; }
};
__device__ __forceinline__ SplineView spl_of(const SplineDev& sp, int b) {
    const double* t = sp.base + (size_t)b * sp.stride;
    return {t, t[SPL_DELTA], t[SPL_L]};
}

// Everything a kernel needs that is constant over a batch call (passed by value).
struct DevConst {
    mpcc_params p;
    double A[NX * NX], B[NX * NU];   // discretized kinematic model (model.cpp:47-91)
    double M[NX * NX], G[NX * NU];   // Tx^-1 A Tx, Tx^-1 B Tu
    SplineDev spl;
    int N;
    int S;                           // record stride = B*(N+1) of this call
    int Bn;                          // batch size of this call
    int faithful_dead_trials;
    int ocp;                         // 1: SolverInterface::solveOCP only (mpcc_solve_ocp), no MPC bookkeeping
};

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ void m3mul(const double* A, const double* B, double* C) {
    double T[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
    for (int i = 0; i < 9; i++) C[i] = T[i];
}
__device__ __forceinline__ void m3mul_tn(const double* A, const double* B, double* C) {  // A^T B
    double T[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) T[3 * i + j] = A[i] * B[j] + A[3 + i] * B[3 + j] + A[6 + i] * B[6 + j];
#pragma unroll
    for (int i = 0; i < 9; i++) C[i] = T[i];
}
__device__ __forceinline__ void skew3(const double* v, double* S) {  // cubic_spline_rot.cpp:25-35
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}

}  // namespace mpcc
