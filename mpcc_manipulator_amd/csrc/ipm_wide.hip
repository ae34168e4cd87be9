// ipm_wide.hip — the QP solve (replacing OSQP, osqp_interface.cpp:592-656) and the fused SQP kernel k_sqp of
// the Husky+Panda mobile manipulator build (MPCC_DOF = 10; BASELINE configs[3]).
//
// Same method, start point, tolerances and parity policies as ipm.hip and the oracle's solve_struct_ipm:
// Mehrotra predictor-corrector on the stage-structured normalized QP, Riccati recursion over the augmented
// stage state x~ = [y(NX), w(DOF)] (w_k = v_{k-1}[0:DOF] carries the ddq coupling) with input v(NU).  For
// this robot x~ has 22 components and a stage 22 box/ddq rows, more than one 16-lane DPP row holds, so:
//  * one 32-lane group per instance, 2 instances per wavefront.  Lane t owns box row t (t < NX: y_t; NX <= t
//    < NX + DOF: ddq row t - NX), poly row t, component t of x~ and of v (t < NU) and column t of P.
//  * broadcasts inside the group: v_permlane16_swap (gfx950) duplicates each 16-lane half over both halves,
//    then a DPP row_newbcast picks the lane (no LDS); shifts t <- t +- n across the half boundary combine
//    the same duplicate with a DPP row shift.  Group sums are a DPP row reduction plus one swap.
//  * F, U = LF^-1 Gm and K of the current stage pass through the instance's LDS block (broadcast reads).
//  * the forward sweeps form v = K x~ + kff as group reductions over the K column layout (lane c holds
//    K[i][c]), so the workspace keeps one K layout; F^-1 rows serve the corrector's kff = -F^-1 f.
//  * per-stage slacks, multipliers, iterate, steps and gains stream through a [field][32 lanes] global
//    workspace, one stage ahead.  The predictor backward solve is fused into the factorization sweep and the
//    iterate update applied lazily by the next one, as in ipm.hip.
// QP assembly and line-search pieces of k_sqp: oracle operation order, no FP contraction, the shared headers'
// helpers included (bitwise kernels.hip's k_setqp / k_trial, as in ipm.hip)
#pragma clang fp contract(off)
#include "dev_common.h"
#include "dev_dpp.h"
#include "kernels.h"
#include "dev_sqp.h"
#pragma clang fp contract(fast)

namespace mpcc {

// The mobile build's QP solver; both builds run the damped-BFGS option on it (the Panda's x~ fills half the
// group there).

constexpr int IPM_MAX_IT = 60;
#ifndef MPCC_TOL_MU
#define MPCC_TOL_MU 1e-12  // round 6: 1e-13 -> 1e-12, the oracle's (solve_struct_ipm_from)
#endif
#ifndef MPCC_TOL_STEP
#define MPCC_TOL_STEP 3e-9  // round 6: 1e-11 -> 3e-9, the oracle's
#endif
constexpr double IPM_TOL_MU = MPCC_TOL_MU, IPM_TOL_P = 1e-11, IPM_TOL_STEP = MPCC_TOL_STEP;
constexpr double IPM_TOL_FB = 1e-9;  // P2
constexpr double IPM_DIV = 1e6;      // P3
constexpr double IPM_S0 = 0.02, IPM_L0 = 0.002;
constexpr int IPM_MAX_IT_SCALED = 24;  // the oracle's (round 6: 30 -> 24)
constexpr double IPM_TAU = 0.995;
typedef __attribute__((address_space(1))) double gdouble;
typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int GW = 32;               // lanes per instance
constexpr int IPW = 64 / GW;         // instances per wavefront
constexpr int NXA = NX + DOF;        // augmented stage state [y, w]
static_assert(NXA <= GW && NU <= 16, "stage dimensions of the 32-lane group");

// workspace fields, ws[(b*(N+1) + k)*ISW + field*GW + lane]
enum : int {
    WF_SL = 0, WF_LL, WF_SU, WF_LU, WF_SP, WF_LP,  // slack / multiplier of the lower, upper and poly slot of row t
    WF_ZX, WF_ZV,                                 // iterate: lane c -> x~_c; lane j < NU -> v_j
    WF_DX, WF_DV,                                 // corrector step
    WF_AX, WF_AV,                                 // predictor step
    WF_GX, WF_GV,                                 // objective gradient H z + h
    WF_KFF,                                       // kff (lanes < NU)
    WF_KC,                                        // NU fields: field i, lane c = K[i][c]
    WF_FI = WF_KC + NU,                           // NU fields: field m, lane i = F^-1[i][m]
    WF_KFJ = WF_FI + NU,                          // LRM fields: kff of the low-rank solves Q_j (BFGS)
    WF_QX = WF_KFJ + LRM,                         // LRM fields: Q_j = M u_j, x~ part
    WF_QV = WF_QX + LRM,                          // LRM fields: Q_j, v part
    WF_PZ = WF_QV + LRM, WF_PA, WF_PD,            // PCACHE: lane p -> c_p^T z, c_p^T dza, c_p^T dz of poly row p
    NWF
};
static_assert(NWF * GW <= ISW, "IPM workspace must fit the per-stage ISW allocation");

// per-instance LDS block (doubles): F [i*16 + j], U [i*32 + c], model constants diag(M) [L_C + a], diag(G) [L_C + 16 + j]
constexpr int L_F = 0, L_U = 16 * 16, L_C = L_U + NU * GW;
constexpr int GRP_LDS = L_C + 32 + 16;  // + 16 doubles: the two instances of a wave start 16 banks apart

// Many-poly-row variants (NPM >= 9): the factorization's rank-NPM poly blocks sum_p W_p bv_p bv_p^T,
// sum_p W_p bv_p a_p^T and sum_p W_p a_p a_p^T of both instances on v_mfma_f64_16x16x4f64 (ipm.hip's Gram form;
// here bv_p and a_p have DOF = 10 entries each, so the three blocks are separate 16x16 products).  Per wavefront
// after the per-instance blocks: the operands [inst][24 rows: bv_p (p < 12, zero past NPM), a_p][16 lanes] and
// the weights [inst][16], then, in the same place, the 6 products [3 inst + {bb, ba, aa}][16][16].
#ifndef MPCC_WIDE_GRAM
#define MPCC_WIDE_GRAM 1
#endif
constexpr int G_ROWS = 24, G_OPW = IPW * G_ROWS * 16, GRAM_LDS = 6 * 256;
static_assert(G_OPW + IPW * 16 <= GRAM_LDS, "Gram operands inside the product area");
__host__ __device__ constexpr bool wide_gram(int npm) { return MPCC_WIDE_GRAM && npm >= 9; }

// extended low-rank path (nlr > LRM): per instance the capacitance matrix S = C^-1 + U^T Q (LU in place) and
// the per-term scalars u_j^T z, t = S^-1 U^T dz_s, u_j^T dz, the row pivots and c_j (doubles)
constexpr int XL_S = 0, XL_UZ = LRX * LRX, XL_TT = XL_UZ + LRX, XL_UD = XL_TT + LRX, XL_PIV = XL_UD + LRX,
              XL_C = XL_PIV + LRX, XL_LDS = XL_C + LRX;
static_assert(LRX <= GW && LRX % 4 == 0, "extended low-rank path: one lane per term, terms in chunks of 4");
size_t ipm_wide_lds_bytes(int npm, bool lr) {
    return (size_t)(IPW * GRP_LDS + (wide_gram(npm) ? GRAM_LDS : 0) + (lr ? IPW * XL_LDS : 0)) * sizeof(double);
}

namespace {

using namespace dpp;

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---- 32-lane group exchange ---------------------------------------------------------------------------
// halves(v): .lo = the group's lower 16 lanes' values in both halves, .hi = the upper 16 lanes' values.
// v_permlane16_swap swaps the odd rows of its first operand with the even rows of its second; with both
// operands v the two results are the even and the odd row duplicated over the row pair.  Evaluated with the
// whole wave active (like DPP) and pinned against sinking into divergent code.
struct Halves {
    double lo, hi;
};
__device__ __forceinline__ Halves halves(double v) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(v);
    const unsigned l = (unsigned)x, h = (unsigned)(x >> 32);
    const auto a = __builtin_amdgcn_permlane16_swap(l, l, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(h, h, false, false);
    long long lo = (long long)(((unsigned long long)b[0] << 32) | a[0]);
    long long hi = (long long)(((unsigned long long)b[1] << 32) | a[1]);
    asm volatile("" : "+v"(lo), "+v"(hi));
    return {__longlong_as_double(lo), __longlong_as_double(hi)};
}
// lane i of the group (i a constant after unrolling)
__device__ __forceinline__ double bch(const Halves& h, int i) { return bcn(i < 16 ? h.lo : h.hi, i & 15); }
// lane t <- t + n / t - n inside the group (0 < n < 16); lanes whose source is outside the group get junk
template <int n>
__device__ __forceinline__ double up32(double v, const Halves& h, int t) {
    const double a = from_up<n>(v), b = from_down<16 - n>(h.hi);
    return ((t & 15) + n < 16) ? a : b;
}
template <int n>
__device__ __forceinline__ double down32(double v, const Halves& h, int t) {
    const double a = from_down<n>(v), b = from_up<16 - n>(h.lo);
    return ((t & 15) >= n) ? a : b;
}
// lane t <- t + NX / t - NX (NX = 12)
__device__ __forceinline__ double up_nx(double v, int t) { return up32<NX>(v, halves(v), t); }
__device__ __forceinline__ double down_nx(double v, int t) { return down32<NX>(v, halves(v), t); }
__device__ __forceinline__ double up1(double v, int t) { return up32<1>(v, halves(v), t); }
__device__ __forceinline__ double down1(double v, int t) { return down32<1>(v, halves(v), t); }
__device__ __forceinline__ double g_sum32(double v) {
    const Halves h = halves(g_sum(v));
    return h.lo + h.hi;
}
__device__ __forceinline__ double g_max32(double v) {
    const Halves h = halves(g_max(v));
    return fmax(h.lo, h.hi);
}
__device__ __forceinline__ double g_min32(double v) {
    const Halves h = halves(g_min(v));
    return fmin(h.lo, h.hi);
}

// ---- slot algebra (oracle solve_struct_ipm), slot: sgn*(c^T z) <= sgn*bnd (as ipm.hip) -----------------
struct SlotStep {
    double ds, dl;
};
__device__ __forceinline__ double slot_rp(double sgn, double cz, double bnd, double s) { return sgn * cz - sgn * bnd + s; }
__device__ __forceinline__ SlotStep slot_recover(double ri, double l, double rp, double cd, double rc) {
    const double W = l * ri;
    return {-rp - cd, W * (cd + rp) - rc * ri};
}
__device__ __forceinline__ double slot_coef(double ri, double l, double rp, double rc) { return l + (l * ri) * rp - rc * ri; }
struct MinRatio {
    double num, den;
    __device__ __forceinline__ explicit MinRatio(double cap) : num(cap), den(1.0) {}
    __device__ __forceinline__ void add(double n, double dneg) {
        const double d = -dneg;
        const bool take = dneg < 0 && n * den < num * d;
        num = take ? n : num;
        den = take ? d : den;
    }
    __device__ __forceinline__ double value() const { return num / den; }
};
__device__ __forceinline__ void step_bound(MinRatio& a, double s, double l, SlotStep d) {
    a.add(s, d.ds);
    a.add(l, d.dl);
}
__device__ __forceinline__ double rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    return fma(fma(-x, r, 1.0), r, r);
}
__device__ __forceinline__ SlotStep slot_corr(double sgn, double bnd, double cz, double ca, double cd, double s, double l,
                                              double smu, double* rp_out) {
    const double ri = rcp(s);
    const double rp = slot_rp(sgn, cz, bnd, s);
    const SlotStep pa = slot_recover(ri, l, rp, sgn * ca, s * l);
    const double rc = s * l + pa.ds * pa.dl - smu;
    *rp_out = rp;
    return slot_recover(ri, l, rp, sgn * cd, rc);
}

// 1/sqrt(x) for x > 0: v_rsq_f64 refined by two Newton steps (ipm.hip rsqrt_pos)
__device__ __forceinline__ double rsqrt_pos(double x) {
    const double h = 0.5 * x;
    double r = __builtin_amdgcn_rsq(x);
    r = r * fma(-h * r, r, 1.5);
    return r * fma(-h * r, r, 1.5);
}

// Cholesky of the NU x NU stage F (packed lower triangle), reciprocal pivots (the diagonal of L is not
// formed: the solves read dinv and the strict lower triangle); forward / backward solves
__device__ __forceinline__ bool cholN(double* L, double* dinv) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NU; j++) {
        const int jj = j * (j + 1) / 2;
        double d = L[jj + j];
#pragma unroll
        for (int m = 0; m < j; m++) d -= L[jj + m] * L[jj + m];
        ok = ok && (d > 0);
        const double inv = rsqrt_pos(d);
        dinv[j] = inv;
#pragma unroll
        for (int i = j + 1; i < NU; i++) {
            const int ii = i * (i + 1) / 2;
            double s = L[ii + j];
#pragma unroll
            for (int m = 0; m < j; m++) s -= L[ii + m] * L[jj + m];
            L[ii + j] = s * inv;
        }
    }
    return ok;
}
__device__ __forceinline__ void fwdN(const double* L, const double* dinv, double* x) {
#pragma unroll
    for (int i = 0; i < NU; i++) {
        const int ii = i * (i + 1) / 2;
        double s = x[i];
#pragma unroll
        for (int m = 0; m < i; m++) s -= L[ii + m] * x[m];
        x[i] = s * dinv[i];
    }
}
__device__ __forceinline__ void bwdN(const double* L, const double* dinv, double* x) {
#pragma unroll
    for (int i = NU - 1; i >= 0; i--) {
        double s = x[i];
#pragma unroll
        for (int m = i + 1; m < NU; m++) s -= L[m * (m + 1) / 2 + i] * x[m];
        x[i] = s * dinv[i];
    }
}

// x = A^-1 b for the LRM x LRM Woodbury capacitance matrix (partial pivoting, the oracle's lu_solve_small),
// redundantly per lane; indices are constants after unrolling, pivot rows are moved by selects
__device__ __forceinline__ void solve_small(double (&A)[LRM * LRM], double (&b)[LRM]) {
#pragma unroll
    for (int k = 0; k < LRM; k++) {
        int p = k;
        double mx = fabs(A[k * LRM + k]);
#pragma unroll
        for (int i = k + 1; i < LRM; i++) {
            const bool take = fabs(A[i * LRM + k]) > mx;
            mx = take ? fabs(A[i * LRM + k]) : mx;
            p = take ? i : p;
        }
#pragma unroll
        for (int i = k + 1; i < LRM; i++) {  // swap rows k and p
            const bool sw = (i == p);
#pragma unroll
            for (int j = 0; j < LRM; j++) {
                const double a = A[k * LRM + j], c2 = A[i * LRM + j];
                A[k * LRM + j] = sw ? c2 : a;
                A[i * LRM + j] = sw ? a : c2;
            }
            const double bk = b[k], bi = b[i];
            b[k] = sw ? bi : bk;
            b[i] = sw ? bk : bi;
        }
#pragma unroll
        for (int i = k + 1; i < LRM; i++) {
            const double f = A[i * LRM + k] / A[k * LRM + k];
#pragma unroll
            for (int j = k; j < LRM; j++) A[i * LRM + j] -= f * A[k * LRM + j];
            b[i] -= f * b[k];
        }
    }
#pragma unroll
    for (int i = LRM - 1; i >= 0; i--) {
        double s = b[i];
#pragma unroll
        for (int j = i + 1; j < LRM; j++) s -= A[i * LRM + j] * b[j];
        b[i] = s / A[i * LRM + i];
    }
}

// per-stage inputs of one lane, loaded one stage ahead of their use
template <int NPE>
struct StageIn {
    double lb, ub, np;
    double pa[NPE], pb[NPE];      // poly rows p: a_p[t], bv_p[t] (t < DOF)
    double pub;                   // upper bound of poly row t (t < npmax)
    double sL, lL, sU, lU, sP, lP, zx, zv;
    double pz, pca, pcd;          // PCACHE: c_p^T z, c_p^T dza, c_p^T dz of poly row t
    double x0, x1, x2, x3;        // sweep-specific pairs (dz, dza, g0)
    double m[2 * NU];             // sweep-specific: Q row (NX) + q, R, r | K column (NU) + kff | K column + F^-1 row
};

// Light sweeps of the many-poly-row variants without the prefetch buffer: measured slower here (mobile
// configs[3] k_sqp<11> 348.7 ms against 341.7 ms with it, profiles/r02f_c3*.json), unlike ipm.hip, so off
#ifndef MPCC_WIDE_LIGHT_NOPF
#define MPCC_WIDE_LIGHT_NOPF 0
#endif
// stage sweep i = 0..N in order s(i) with the next stage prefetched (copy-based double buffer)
template <class In, class LoadF, class BodyF>
__device__ __forceinline__ void sweep(int N, bool backward, In& b0, In& b1, LoadF load, BodyF body) {
    auto s = [&](int i) { return backward ? N - i : i; };
    load(s(0), b0);
    for (int i = 0; i <= N; i++) {
        load(s(i + 1 <= N ? i + 1 : N), b1);
        body(s(i), b0);
        b0 = b1;
    }
}

// The same sweep without the prefetch buffer: each stage's loads are issued at the top of its body.
template <class In, class LoadF, class BodyF>
__device__ __forceinline__ void sweep_noprefetch(int N, bool backward, In& b0, LoadF load, BodyF body) {
    for (int i = 0; i <= N; i++) {
        const int k = backward ? N - i : i;
        load(k, b0);
        body(k, b0);
    }
}

}  // namespace

// The QP solve of the 2 instances of this wavefront (32 lanes each).  Writes the step (d.step), QP status
// and IPM iteration count (d.sqi).  LR: the Hessian carries the damped-BFGS low-rank terms.
template <int NPM, bool LR>
__device__ __forceinline__ void ipm_group(const DevConst& c, const DevBuffers& d, double* smem) {
    constexpr int NPE = NPM > 0 ? NPM : 1;
    using In = StageIn<NPE>;
    const int lane = threadIdx.x;
    const int grp = lane / GW;
    const int t = lane % GW;
    const int b = blockIdx.x * IPW + grp;
    const int N = c.N;
    const int NS = N + 1;
    double* const S = smem + grp * GRP_LDS;

    const bool valid = b < c.Bn;
    int32_t* si = d.sqi + (size_t)(valid ? b : 0) * SQI;
    bool run = valid && si[SQ_ACTIVE] != 0;
    if (__ballot(run) == 0) return;

    const gdouble* QSb = (const gdouble*)(d.qs + (size_t)MPCC_BCHK(c.bchk, valid ? b : 0, c.Bn, BC_INSTANCE) * NS * QS);
    gdouble* WSb = (gdouble*)(d.isw + (size_t)(valid ? b : 0) * NS * ISW);
    gdouble* const WSt = WSb + t;
    auto ws = [&](int k, int f) -> gdouble* {
        gdouble* wk = WSt + (size_t)MPCC_BCHK(c.bchk, k, NS, BC_WS_STAGE) * ISW;
        asm("" : "+v"(wk));
        return wk + MPCC_BCHK(c.bchk, f, NWF, BC_WS_FIELD) * GW;
    };
    auto qs_stage = [&](int k) -> const gdouble* {
        const gdouble* qk = QSb + (size_t)MPCC_BCHK(c.bchk, k, NS, BC_QS_STAGE) * QS;
        asm("" : "+v"(qk));
        return qk;
    };

    // ---- model constants of this lane: M = diag(m) + m_sv e_s e_vs^T, G = diag(g) + g_v e_vs e_dVs^T
    const double msv = c.M[XS * NX + XVS], mss = c.M[XS * (NX + 1)];
    const double gs = c.G[XS * NU + UVS], gv = c.G[XVS * NU + UVS];
    double mt = 0.0, gt = 0.0, Hct = 0.0;
    const double HcB = -2. * c.p.qp_r_ddq;
#pragma unroll
    for (int a = 0; a < NX; a++)
        if (t == a) mt = c.M[a * (NX + 1)];
#pragma unroll
    for (int a = 0; a < DOF; a++) {
        if (t == a) gt = c.G[a * (NU + 1)];
        if (t == a || t == NX + a) Hct = c.p.Tu[a] * HcB * c.p.Tu[a];
    }
    if (t == UVS) gt = gs;
    // diag(M), diag(G) for the factor body's Y = B~^T P and Hb products: read there per stage, from LDS
    if (t < NX) S[L_C + t] = c.M[t * (NX + 1)];
    if (t < DOF) S[L_C + 16 + t] = c.G[t * (NU + 1)];
    lds_sync();
    const bool rowY = t < NX;
    const bool rowD = t >= NX && t < NXA;
    const int j9 = t - NX;
    const int jc = rowD ? j9 : 0;  // clamped ddq row (addresses stay inside the record)
    constexpr double sgnL = -1.0, sgnU = 1.0;

    // ---- Hessian checks (osqp_interface.cpp:454-473): stage flags + tridiagonal input blocks
    int fl = 0;
    if (run) {
        for (int k = t; k < NS; k += GW) fl |= (int)QSb[(size_t)k * QS + QS_FLAG];
        if (t < NU) {
            // diagonals read 8 stages at a time ahead of the recursion (ipm.hip: no HBM round trip per stage)
            double prev_d = 0;
            bool bad = false;
            for (int k0 = 0; k0 < N && !bad; k0 += 8) {
                double dk8[8];
#pragma unroll
                for (int q = 0; q < 8; q++) dk8[q] = QSb[(size_t)min(k0 + q, N - 1) * QS + QS_R + t];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const int k = k0 + q;
                    if (bad || k >= N) break;
                    const double dk = dk8[q];
                    const double off = (k >= 1 && t < DOF) ? Hct : 0.0;
                    const double l = (k >= 1) ? off / prev_d : 0.0;
                    const double dd = dk - l * l;
                    if (dd <= 0) { fl |= 2; bad = true; break; }
                    prev_d = sqrt(dd);
                }
            }
        }
    }
    {
        int o = 0;
#pragma unroll
        for (int bit = 0; bit < 3; bit++)
            if (g_max32((double)((fl >> bit) & 1)) > 0.5) o |= 1 << bit;
        fl = o;
    }
    if (run && (fl & 2)) { if (t == 0) { si[SQ_STATUS] = MPCC_NON_PD_HESSIAN; si[SQ_ACTIVE] = 0; } run = false; }
    if (run && (fl & 1)) { if (t == 0) { si[SQ_STATUS] = MPCC_NAN_HESSIAN; si[SQ_ACTIVE] = 0; } run = false; }
    if (run && (fl & 4)) { if (t == 0) si[SQ_QPSTAT] = MPCC_QP_PrimalInfeasible; run = false; }  // keep old step (Q6)
    if constexpr (LR) {  // more than LRM terms need the extended path's columns (d.lrq, allocated by the engine
                         // whenever d.lrs > LRM): without them the instance stops with INVALID_SETTINGS, never a stray write
        if (run && si[SQ_NLR] > LRM && d.lrq == nullptr) {
            if (t == 0) { si[SQ_STATUS] = MPCC_INVALID_SETTINGS; si[SQ_ACTIVE] = 0; }
            run = false;
        }
    }
    const bool entered = run;

    // ---- low-rank Hessian terms of the damped-BFGS option: B = H_0 + sum_j c_j u_j u_j^T, u_j per stage as
    //      [x (NX) | u (NU)] (d.lr).  Every Riccati solve dz_s = -M g is corrected by the Woodbury identity,
    //      dz = dz_s - Q S^-1 (U^T dz_s) with Q_j = M u_j = -solve(u_j) (backward recursion in the factorization
    //      sweep, forward in the predictor forward sweep) and S = C^-1 + U^T Q (the oracle's lr_solve).
    int nlr = 0;
    double lrc[LRM];
    const gdouble* LRb = (const gdouble*)d.step;  // any valid address when !LR
#pragma unroll
    for (int j = 0; j < LRM; j++) lrc[j] = 0.0;
    if constexpr (LR) {
        nlr = si[SQ_NLR];
#pragma unroll
        for (int j = 0; j < LRM; j++) lrc[j] = (j < nlr) ? d.lrc[(size_t)(valid ? b : 0) * d.lrs + j] : 0.0;
        LRb = (const gdouble*)(d.lr + (size_t)(valid ? b : 0) * d.lrs * NS * NXU);
    }
    // more terms than the fused sweeps carry: the wave runs the extended path (both instances; nlr_w = the larger
    // count, the other instance's extra terms are zero vectors with unit capacitance)
    const bool xlw = LR && __ballot(entered && nlr > LRM) != 0;
    const int nlr_w = xlw ? max(__shfl(entered ? nlr : 0, 0), __shfl(entered ? nlr : 0, GW)) : 0;
    const bool lrw = LR && !xlw && __ballot(entered && nlr > 0) != 0;  // this wave runs the split (Woodbury) sweeps
    auto u_y = [&](int j, int k) -> double {  // u_j, y part of stage k (lanes < NX)
        const double v = LRb[((size_t)MPCC_BCHK(c.bchk, j, d.lrs, BC_LR) * NS + MPCC_BCHK(c.bchk, k, NS, BC_LR)) * NXU + (rowY ? t : 0)];
        return (LR && rowY && j < nlr) ? v : 0.0;
    };
    auto u_v = [&](int j, int k) -> double {  // u_j, v part of stage k (lanes < NU, k < N)
        const double v = LRb[((size_t)MPCC_BCHK(c.bchk, j, d.lrs, BC_LR) * NS + MPCC_BCHK(c.bchk, k, NS, BC_LR)) * NXU + NX + (t < NU ? t : 0)];
        return (LR && t < NU && k < N && j < nlr) ? v : 0.0;
    };
    double uz[LRM];  // u_j^T z of the current iterate
#pragma unroll
    for (int j = 0; j < LRM; j++) uz[j] = 0.0;

    // ---- extended low-rank path (xlw): the Woodbury correction of the fused sweeps for any nlr <= LRX, with the
    //      columns Q_j in memory (d.lrq, per lane) and S, its LU and the per-term scalars in the instance's LDS
    //      (XL_*), the terms taken 4 at a time.  Same formulas as the fused path and the oracle's lr_solve.
    double* const XL = smem + IPW * GRP_LDS + (wide_gram(NPM) ? GRAM_LDS : 0) + grp * XL_LDS;
    // xlw implies d.lrq (the INVALID_SETTINGS guard above); the null base is never dereferenced otherwise
    gdouble* const XQb = (gdouble*)(d.lrq + (d.lrq ? (size_t)(valid ? b : 0) * d.lrs * NS * 3 * GW : 0));
    auto xq = [&](int j, int k, int f) -> gdouble* {  // f: 0 Q_j x~ part, 1 Q_j v part, 2 kff of the solve of u_j
        return XQb + (((size_t)MPCC_BCHK(c.bchk, j, d.lrs, BC_LR) * NS + MPCC_BCHK(c.bchk, k, NS, BC_LR)) * 3 + f) * GW + t;
    };
    const int xlt = t < LRX ? t : LRX - 1;  // this lane's term / row of S (clamped address)
    if (xlw && t < LRX) XL[XL_C + t] = (t < nlr) ? d.lrc[(size_t)(valid ? b : 0) * d.lrs + t] : 0.0;
    // dst[j] = u_j^T [ws fx | ws fv] over the horizon, all j < nlr_w
    auto xl_dots = [&](int dst, int fx, int fv) {
        for (int j0 = 0; j0 < nlr_w; j0 += 4) {
            double pq[4] = {0.0, 0.0, 0.0, 0.0};
            for (int k = 0; k <= N; k++) {
                const double x = *ws(k, fx), v = *ws(k, fv);
#pragma unroll
                for (int q = 0; q < 4; q++) pq[q] += u_y(j0 + q, k) * x + u_v(j0 + q, k) * v;
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const double sm = g_sum32(pq[q]);
                if (t == 0) XL[dst + j0 + q] = sm;
            }
        }
        lds_sync();
    };

    // Many poly rows (without the low-rank terms): c_p^T z, c_p^T dza and c_p^T dz are formed once per iteration
    // where z, dza and dz are made and kept in the workspace (WF_PZ, WF_PA, WF_PD) for the other sweeps, which
    // recomputed them from the same stored vectors (ipm.hip PCACHE)
    constexpr bool PCACHE = NPM >= 9 && !LR;
    // Gram variants: the factorization sweep runs on the whole wave (the matrix cores need every lane); lanes of an
    // instance that is done re-read stage N and store nothing
    constexpr bool GRAM = wide_gram(NPM);
    double* const GM = smem + IPW * GRP_LDS;
    // ---- stage loaders (unconditional loads, lane/stage conditions as selects)
    auto load_common = [&](int k, In& o) {
        const gdouble* q = qs_stage(k);
        const double ylb = q[QS_YLB + (rowY ? t : 0)], yub = q[QS_YUB + (rowY ? t : 0)];
        const double dlb = q[QS_DLB + jc], dub = q[QS_DUB + jc];
        o.lb = rowY ? ylb : (rowD ? dlb : -INF);
        o.ub = rowY ? yub : (rowD ? dub : INF);
        o.np = q[QS_NPOLY];
        const int tp = t < DOF ? t : 0;
#pragma unroll
        for (int p = 0; p < NPE; p++) {
            const double a = q[QS_POLY + POLY_W * p + tp], bv = q[QS_POLY + POLY_W * p + DOF + tp];
            o.pa[p] = (NPM > 0 && t < DOF) ? a : 0.0;
            o.pb[p] = (NPM > 0 && t < DOF) ? bv : 0.0;
        }
        const double pu = q[QS_POLY + POLY_W * (t < NPE ? t : 0) + 2 * DOF];
        o.pub = (t < NPM) ? pu : INF;
        o.sL = *ws(k, WF_SL); o.lL = *ws(k, WF_LL); o.sU = *ws(k, WF_SU); o.lU = *ws(k, WF_LU);
        o.sP = *ws(k, WF_SP); o.lP = *ws(k, WF_LP);
        o.zx = *ws(k, WF_ZX); o.zv = *ws(k, WF_ZV);
        if constexpr (PCACHE) { o.pz = *ws(k, WF_PZ); o.pca = *ws(k, WF_PA); o.pcd = *ws(k, WF_PD); }
    };
    auto load_factor = [&](int k, In& o, bool upd) {
        load_common(k, o);
        const gdouble* q = qs_stage(k);
        const int tr = rowY ? t : 0;
#pragma unroll
        for (int m = 0; m < NX; m++) {
            const double v = q[QS_Q + tr * NX + m];
            o.m[m] = rowY ? v : 0.0;
        }
        const int tu = t < NU ? t : 0;
        const double qv = q[QS_q + tr], rv = q[QS_R + tu], rr = q[QS_r + tu];
        o.m[NX] = rowY ? qv : 0.0;
        o.m[NX + 1] = (t < NU && k < N) ? rv : 0.0;
        o.m[NX + 2] = (t < NU && k < N) ? rr : 0.0;
        const double x0 = *ws(k, WF_DX), x1 = *ws(k, WF_DV), x2 = *ws(k, WF_AX), x3 = *ws(k, WF_AV);
        o.x0 = upd ? x0 : 0.0; o.x1 = upd ? x1 : 0.0; o.x2 = upd ? x2 : 0.0; o.x3 = upd ? x3 : 0.0;
    };
    auto load_fwd = [&](int k, In& o, bool corr) {
        load_common(k, o);
#pragma unroll
        for (int i = 0; i < NU; i++) {
            const double v = *ws(k, WF_KC + i);
            o.m[i] = (k < N) ? v : 0.0;
        }
        const double kf = *ws(k, WF_KFF);
        o.m[NU] = (k < N) ? kf : 0.0;
        if (corr) { o.x0 = *ws(k, WF_AX); o.x1 = *ws(k, WF_AV); } else { o.x0 = o.x1 = 0.0; }
    };
    auto load_bwd = [&](int k, In& o) {
        load_common(k, o);
        o.x0 = *ws(k, WF_AX); o.x1 = *ws(k, WF_AV); o.x2 = *ws(k, WF_GX); o.x3 = *ws(k, WF_GV);
#pragma unroll
        for (int i = 0; i < NU; i++) {
            const double v = *ws(k, WF_KC + i);
            o.m[i] = (k < N) ? v : 0.0;
        }
#pragma unroll
        for (int m = 0; m < NU; m++) {
            const double v = *ws(k, WF_FI + m);
            o.m[NU + m] = (k < N) ? v : 0.0;
        }
    };

    // ---- stage-local helpers
    auto row_active = [&](int k, double bnd) { return (rowY ? (k >= 1) : (rowD && k < N)) && fabs(bnd) < BIG; };
    // unsigned c^T z of this lane's box / ddq row; (x, v) = lane components of a stage vector
    auto row_cz = [&](int k, double x, double v) -> double {
        const double vj = down_nx(v, t);  // lane NX+j <- v_j
        if (rowY) return x;
        return (k == 0) ? vj : vj - x;
    };
    // c^T z of poly row t (= p), reduced over the group: sum_m a_p[m] y_m + bv_p[m] v_m
    auto poly_cz = [&](const In& in, int k, double x, double v) -> double {
        double r = 0.0;
#pragma unroll
        for (int p = 0; p < NPM; p++) {
            const bool live = (double)p < in.np && k < N;
            const double term = live ? in.pa[p] * x + in.pb[p] * v : 0.0;
            const double s = g_sum32(term);
            if (t == p) r = s;
        }
        return r;
    };
    auto poly_slot_active = [&](const In& in, int k) {
        return t < NPM && (double)t < in.np && k < N && fabs(in.pub) < BIG;
    };
    // step-system gradient g = g0 + sum_i sgn_i coef_i c_i (dvr: signed coefficient of row t, cP: poly row t)
    auto assemble_grad = [&](const In& in, int k, double g0x, double g0v, double dvr, double cP, double& gx, double& gvv) {
        gx = g0x;
        if (rowY) gx += dvr;
        else if (rowD && k >= 1) gx -= dvr;
        gvv = g0v;
        const double dv_up = up_nx(dvr, t);  // lane j <- ddq row j
        if (t < DOF && k < N) gvv += dv_up;
        const Halves hc = halves(cP);
#pragma unroll
        for (int p = 0; p < NPM; p++) {
            const double cp = bch(hc, p);
            const bool live = (double)p < in.np && k < N;
            if (live) {
                gx += cp * in.pa[p];  // zero for lanes >= DOF
                gvv += cp * in.pb[p];
            }
        }
    };
    // forward step: v = K x~ + kff (group sums over the K column layout; result on lanes < NU) and
    // x~' = A~ x~ + B~ v (all lanes)
    auto fwd_step_k = [&](const In& in, double xt, double kff, double& v, double& xn) {
        double vv = 0.0;
#pragma unroll
        for (int i = 0; i < NU; i++) {
            const double s = g_sum32(in.m[i] * xt);
            if (t == i) vv = s;
        }
        v = vv + kff;
        const Halves hx = halves(xt), hv = halves(v);
        const double xvs = bch(hx, XVS);
        const double vprev = down32<1>(v, hv, t);   // lane XVS <- v_dVs (lane XS)
        const double vj = down32<NX>(v, hv, t);     // lane NX + j <- v_j
        if (t < DOF) xn = mt * xt + gt * v;
        else if (t == XS) xn = (mss * xt + msv * xvs) + gs * v;
        else if (t == XVS) xn = mt * xt + gv * vprev;
        else xn = rowD ? vj : 0.0;
    };
    auto fwd_step = [&](const In& in, double xt, double& v, double& xn) { fwd_step_k(in, xt, in.m[NU], v, xn); };

    // ---- extended low-rank path: Q_j = M u_j = -solve(u_j) from the stored gains, 4 terms per backward +
    //      forward pass (the fused path's recursions, ipm_group factorization / predictor sweeps)
    auto xl_q = [&]() {
        for (int j0 = 0; j0 < nlr_w; j0 += 4) {
            double pj[4];
            for (int k = N; k >= 0; k--) {
                if (k == N) {
#pragma unroll
                    for (int q = 0; q < 4; q++) pj[q] = u_y(j0 + q, k);
                    continue;
                }
                double kc[NU], fi[NU];
#pragma unroll
                for (int i = 0; i < NU; i++) { kc[i] = *ws(k, WF_KC + i); fi[i] = *ws(k, WF_FI + i); }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const Halves hq = halves(pj[q]);
                    const double qu = up32<NX>(pj[q], hq, t), qu1 = up32<1>(pj[q], hq, t);
                    const double fvj = u_v(j0 + q, k) + gt * pj[q] + ((t < DOF) ? qu : gv * qu1);
                    const Halves hfj = halves(fvj);
                    double kffj = 0.0, ktfj = 0.0;
#pragma unroll
                    for (int m = 0; m < NU; m++) {
                        const double fbm = bch(hfj, m);
                        kffj -= fi[m] * fbm;
                        ktfj += kc[m] * fbm;
                    }
                    *xq(j0 + q, k, 2) = (t < NU) ? kffj : 0.0;
                    double atpj = 0.0;
                    const double pq7 = down32<1>(pj[q], hq, t);
                    if (rowY) {
                        atpj = mt * pj[q];
                        if (t == XVS) atpj += msv * pq7;
                    }
                    pj[q] = u_y(j0 + q, k) + atpj + ktfj;
                }
            }
            double xqv[4] = {0.0, 0.0, 0.0, 0.0};
            for (int k = 0; k <= N; k++) {
                In kin;
#pragma unroll
                for (int i = 0; i < NU; i++) {
                    const double v = *ws(k, WF_KC + i);
                    kin.m[i] = (k < N) ? v : 0.0;
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const double kfj = *xq(j0 + q, k, 2);
                    double vq = 0.0, xqn = 0.0;
                    fwd_step_k(kin, xqv[q], (k < N) ? kfj : 0.0, vq, xqn);
                    *xq(j0 + q, k, 0) = (t < NXA) ? -xqv[q] : 0.0;
                    *xq(j0 + q, k, 1) = (t < NU && k < N) ? -vq : 0.0;
                    xqv[q] = (k < N) ? xqn : 0.0;
                }
            }
        }
    };
    // S = C^-1 + U^T Q over 4 x 4 blocks of terms (the upper blocks, mirrored), then its LU with partial pivoting
    // in place: lane c works on column c (< nlr_w), row swaps as the oracle's lu_solve_small (the first largest
    // |pivot| candidate), multipliers below the diagonal, pivot rows in XL_PIV
    auto xl_smat_lu = [&]() {
        double* const Sm = XL + XL_S;
        for (int i0 = 0; i0 < nlr_w; i0 += 4)
            for (int j0 = i0; j0 < nlr_w; j0 += 4) {
                double pq[4][4];
#pragma unroll
                for (int q = 0; q < 4; q++)
#pragma unroll
                    for (int r = 0; r < 4; r++) pq[q][r] = 0.0;
                for (int k = 0; k <= N; k++) {
                    double qx[4], qv[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) { qx[r] = *xq(j0 + r, k, 0); qv[r] = *xq(j0 + r, k, 1); }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const double uy = u_y(i0 + q, k), uv = u_v(i0 + q, k);
#pragma unroll
                        for (int r = 0; r < 4; r++) pq[q][r] += uy * qx[r] + uv * qv[r];
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; q++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int i = i0 + q, j = j0 + r;
                        const double uq = g_sum32(pq[q][r]);
                        if (t == 0) {
                            const double ci = (i < nlr) ? 1.0 / XL[XL_C + i] : 1.0;
                            Sm[i * LRX + j] = (i == j ? ci : 0.0) + uq;
                            if (j0 > i0) Sm[j * LRX + i] = uq;
                        }
                    }
            }
        lds_sync();
        for (int kk = 0; kk < nlr_w; kk++) {
            const double a = (t >= kk && t < nlr_w) ? fabs(Sm[xlt * LRX + kk]) : -1.0;
            const double mx = g_max32(a);
            const unsigned gb = (unsigned)(__ballot(a == mx) >> (grp * GW));
            const int p = gb ? __ffs(gb) - 1 : kk;
            if (t == 0) XL[XL_PIV + kk] = (double)p;
            if (p != kk && t < nlr_w) {
                const double x = Sm[kk * LRX + xlt], y = Sm[p * LRX + xlt];
                Sm[kk * LRX + xlt] = y;
                Sm[p * LRX + xlt] = x;
            }
            lds_sync();
            const double rp = 1.0 / Sm[kk * LRX + kk];
            const double ukt = Sm[kk * LRX + xlt];
            for (int i = kk + 1; i < nlr_w; i++) {
                const double l = Sm[i * LRX + kk] * rp;  // read by every lane before lane kk stores it (in order)
                if (t > kk && t < nlr_w) Sm[i * LRX + xlt] -= l * ukt;
                if (t == kk) Sm[i * LRX + kk] = l;
            }
            lds_sync();
        }
    };
    // XL[slot + j] <- S^-1 XL[slot + j]: the row swaps in order (the multipliers were swapped with their rows),
    // the unit lower solve, the upper solve; lane j holds entry j, the pivot entry is broadcast by a lane shuffle
    auto xl_solve = [&](int slot) {
        const double* const Sm = XL + XL_S;
        const int base = grp * GW;
        double v = (t < nlr_w) ? XL[slot + xlt] : 0.0;
        for (int kk = 0; kk < nlr_w; kk++) {
            const int p = (int)XL[XL_PIV + kk];
            const int src = (t == kk) ? p : ((t == p) ? kk : t);
            v = __shfl(v, base + src);
        }
        for (int kk = 0; kk < nlr_w; kk++) {
            const double vk = __shfl(v, base + kk);
            if (t > kk && t < nlr_w) v -= Sm[xlt * LRX + kk] * vk;
        }
        for (int kk = nlr_w - 1; kk >= 0; kk--) {
            if (t == kk) v = v / Sm[kk * LRX + kk];
            const double xk = __shfl(v, base + kk);
            if (t < kk) v -= Sm[xlt * LRX + kk] * xk;
        }
        if (t < nlr_w) XL[slot + t] = v;
        lds_sync();
    };
    // dz = dz_s - sum_j t_j Q_j of stage k (t = XL_TT)
    auto xl_fix = [&](int k, double& x, double& v) {
        for (int j = 0; j < nlr_w; j++) {
            const double tj = XL[XL_TT + j];
            x -= tj * *xq(j, k, 0);
            v -= tj * *xq(j, k, 1);
        }
    };

    In cur, nxt;
    // light sweeps (no factorization), optionally without the prefetch buffer (MPCC_WIDE_LIGHT_NOPF)
    auto light_sweep = [&](bool backward, auto load, auto body) {
        if constexpr (NPM > 2 && MPCC_WIDE_LIGHT_NOPF) sweep_noprefetch(N, backward, cur, load, body);
        else sweep(N, backward, cur, nxt, load, body);
    };
    int it = 0, it_total = 0;
    bool conv = false, diverged = false;
    double alpha = 0.0;
#pragma unroll 1
    for (int attempt = 0; attempt < 2; attempt++) {
        const double s_floor = (attempt == 0) ? IPM_S0 : 1.0;
        const double lam_scale = (attempt == 0) ? IPM_L0 : 0.0;
        const int max_it = (attempt == 0) ? IPM_MAX_IT_SCALED : IPM_MAX_IT;
        if (attempt == 1) {
            run = entered && !conv && !diverged;  // a P3 divergence is final (solve_struct_ipm)
            if (__ballot(run) == 0) break;
            if (run) diverged = false;
        }
        // ---- start point: dynamics rollout with v = 0; slacks / multipliers (solve_struct_ipm)
        double mcount = 0.0;
        double uzp[LRM];
#pragma unroll
        for (int j = 0; j < LRM; j++) uzp[j] = 0.0;
        if (run) {
            double y = 0.0;  // lane a < NX: y_a of stage k
            for (int k = 0; k <= N; k++) {
                load_common(k, cur);
                const double bk = (k < N && rowY) ? QSb[(size_t)k * QS + QS_B + (rowY ? t : 0)] : 0.0;
                const double yx = rowY ? y : 0.0;
                const double cz = row_cz(k, yx, 0.0);
                const double pcz = poly_cz(cur, k, yx, 0.0);
                if constexpr (PCACHE) *ws(k, WF_PZ) = pcz;
                const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                double sL = 1, lL = 0, sU = 1, lU = 0, sP = 1, lP = 0;
                if (aL) { sL = fmax(-(sgnL * cz - sgnL * cur.lb), s_floor); lL = (lam_scale > 0) ? lam_scale / sL : 1.0; }
                if (aU) { sU = fmax(-(sgnU * cz - sgnU * cur.ub), s_floor); lU = (lam_scale > 0) ? lam_scale / sU : 1.0; }
                if (aP) { sP = fmax(-(sgnU * pcz - sgnU * cur.pub), s_floor); lP = (lam_scale > 0) ? lam_scale / sP : 1.0; }
                mcount += (aL ? 1.0 : 0.0) + (aU ? 1.0 : 0.0) + (aP ? 1.0 : 0.0);
                *ws(k, WF_SL) = sL; *ws(k, WF_LL) = lL; *ws(k, WF_SU) = sU; *ws(k, WF_LU) = lU;
                *ws(k, WF_SP) = sP; *ws(k, WF_LP) = lP;
                *ws(k, WF_ZX) = yx;
                *ws(k, WF_ZV) = 0.0;
                if (lrw)
#pragma unroll
                    for (int j = 0; j < LRM; j++) uzp[j] += u_y(j, k) * yx;
                // y_{k+1} = M y_k + b_k (oracle order: sum_b M[a][b] y_b, then + b_a)
                const double yvs = up1(y, t);  // lane XS <- y_vs
                const double yn = (t == XS) ? mss * y + msv * yvs : mt * y;
                y = rowY ? yn + bk : 0.0;
            }
        }
        mcount = g_sum32(mcount);
        if (lrw)
#pragma unroll
            for (int j = 0; j < LRM; j++) uz[j] = g_sum32(uzp[j]);
        if (xlw && run) xl_dots(XL_UZ, WF_ZX, WF_ZV);  // u_j^T z of the start point (v = 0)

        it = 0;
        double mu0 = 0.0, dz_prev = 1e30, sigma_mu = 0.0, mu_cur = 1e30, rp_cur = 1e30;
        bool pending = false;
        if (run) alpha = 0.0;
        while (true) {
            if (__ballot(run) == 0) break;
            if (run || GRAM) {
                // ================= factorization sweep k = N..0 (lazy update, g0, predictor backward solve)
                double Pc[NXA];  // column t of P_{k+1}
                double pv = 0.0; // p_{k+1}, component t
                double pj[LRM];  // p of the low-rank solves Q_j
#pragma unroll
                for (int j = 0; j < LRM; j++) pj[j] = 0.0;
                bool chol_ok = true;
                auto factor_sweep = [&](auto load, auto body) {
                    // the factorization body holds the most registers: with many poly rows a prefetched stage
                    // buffer pushes it deep into scratch (regalloc: 109 spills + 172 reloads per stage against
                    // 52 + 115 without it), so those variants load each stage at the top of its body
                    if constexpr (NPM > 2) sweep_noprefetch(N, true, cur, load, body);
                    else sweep(N, true, cur, nxt, load, body);
                };
                // global stores of the sweep: only a running instance's (the Gram variants run it on the whole wave)
                auto wst = [&](int k, int f, double v) {
                    if (!GRAM || run) *ws(k, f) = v;
                };
                // the Gram products of this stage (GRAM): operands through the wave's LDS area into the MFMA layouts
                // (A lane l -> A[l & 15][l >> 4], B lane l -> B[l >> 4][l & 15], k = poly row 4 q + (l >> 4)), the
                // products back into it (C lane l, reg r -> C[(l >> 4) + 4 r][l & 15]), read there by column
                auto gram = [&](const In& in, double wp) {
                    if constexpr (GRAM) {
                        double* const O = GM + grp * (G_ROWS * 16);
                        if (t < 16) {
#pragma unroll
                            for (int p = 0; p < 12; p++) {
                                O[p * 16 + t] = (p < NPM) ? in.pb[p] : 0.0;          // bv_p[t] (zero for t >= DOF)
                                O[(12 + p) * 16 + t] = (p < NPM) ? in.pa[p] : 0.0;   // a_p[t]
                            }
                            if (t < 12) GM[G_OPW + grp * 16 + t] = (t < NPM) ? wp : 0.0;  // W_p (zero unless live)
                        }
                        lds_sync();
                        const int g = lane >> 4, cc = lane & 15;
                        d4 acc[6];
#pragma unroll
                        for (int m = 0; m < 6; m++) acc[m] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int q = 0; q < (NPM + 3) / 4; q++)
#pragma unroll
                            for (int j = 0; j < IPW; j++) {
                                const double* Oj = GM + j * (G_ROWS * 16);
                                const double bv = Oj[(4 * q + g) * 16 + cc], a = Oj[(12 + 4 * q + g) * 16 + cc];
                                const double w = GM[G_OPW + j * 16 + 4 * q + g];
                                const double wb = w * bv, wa = w * a;
                                acc[3 * j] = __builtin_amdgcn_mfma_f64_16x16x4f64(wb, bv, acc[3 * j], 0, 0, 0);
                                acc[3 * j + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(wb, a, acc[3 * j + 1], 0, 0, 0);
                                acc[3 * j + 2] = __builtin_amdgcn_mfma_f64_16x16x4f64(wa, a, acc[3 * j + 2], 0, 0, 0);
                            }
                        // the products overwrite the operands: LDS executes a wave's operations in program order
#pragma unroll
                        for (int m = 0; m < 6; m++)
#pragma unroll
                            for (int r = 0; r < 4; r++) GM[m * 256 + (g + 4 * r) * 16 + cc] = acc[m][r];
                        lds_sync();
                    }
                };
                factor_sweep([&](int k, In& o) { load_factor((GRAM && !run) ? N : k, o, pending); }, [&](int k, const In& cur) {
                    const double lb = cur.lb, ub = cur.ub;
                    const double* Qr = cur.m;
                    const double qt = cur.m[NX], Rt = cur.m[NX + 1], rt = cur.m[NX + 2];
                    double sL = cur.sL, lL = cur.lL, sU = cur.sU, lU = cur.lU, sP = cur.sP, lP = cur.lP;
                    double zx = cur.zx, zv = cur.zv;
                    const bool aL = row_active(k, lb), aU = row_active(k, ub), aP = poly_slot_active(cur, k);
                    if (pending) {
                        const double dx = cur.x0, dv = cur.x1, ax = cur.x2, av = cur.x3;
                        const double cz = row_cz(k, zx, zv), cd = row_cz(k, dx, dv), ca = row_cz(k, ax, av);
                        double pcz, pcd, pca;
                        if constexpr (PCACHE) {
                            pcz = cur.pz; pcd = cur.pcd; pca = cur.pca;
                        } else {
                            pcz = poly_cz(cur, k, zx, zv); pcd = poly_cz(cur, k, dx, dv); pca = poly_cz(cur, k, ax, av);
                        }
                        double rpd;
                        if (aL) { const SlotStep st = slot_corr(sgnL, lb, cz, ca, cd, sL, lL, sigma_mu, &rpd); sL += alpha * st.ds; lL += alpha * st.dl; }
                        if (aU) { const SlotStep st = slot_corr(sgnU, ub, cz, ca, cd, sU, lU, sigma_mu, &rpd); sU += alpha * st.ds; lU += alpha * st.dl; }
                        if (aP) { const SlotStep st = slot_corr(sgnU, cur.pub, pcz, pca, pcd, sP, lP, sigma_mu, &rpd); sP += alpha * st.ds; lP += alpha * st.dl; }
                        zx += alpha * dx;
                        zv += alpha * dv;
                        wst(k, WF_SL, sL); wst(k, WF_LL, lL); wst(k, WF_SU, sU); wst(k, WF_LU, lU);
                        wst(k, WF_SP, sP); wst(k, WF_LP, lP);
                        wst(k, WF_ZX, zx); wst(k, WF_ZV, zv);
                    }
                    // ---- slots: barrier weights and predictor coefficients (rc = s l)
                    const double cz = row_cz(k, zx, zv);
                    const double pcz = poly_cz(cur, k, zx, zv);
                    if constexpr (PCACHE) wst(k, WF_PZ, pcz);
                    double WL = 0, WU = 0, WP = 0, cL = 0, cU = 0, cP = 0;
                    if (aL) { const double rp = slot_rp(sgnL, cz, lb, sL); const double ri = rcp(sL); WL = lL * ri; cL = slot_coef(ri, lL, rp, sL * lL); }
                    if (aU) { const double rp = slot_rp(sgnU, cz, ub, sU); const double ri = rcp(sU); WU = lU * ri; cU = slot_coef(ri, lU, rp, sU * lU); }
                    if (aP) { const double rp = slot_rp(sgnU, pcz, cur.pub, sP); const double ri = rcp(sP); WP = lP * ri; cP = slot_coef(ri, lP, rp, sP * lP); }
                    const double wd = WL + WU;
                    const double dvr = sgnL * cL + sgnU * cU;
                    // ---- objective gradient g0 = H z + h
                    double g0x, g0v = 0.0;
                    {
                        const Halves hz = halves(zx);
                        const double vj = down_nx(zv, t);  // lane NX+j <- v_j
                        const double wj = up32<NX>(zx, hz, t);  // lane j <- w_j
                        if (rowY) {
                            double s = 0;
#pragma unroll
                            for (int m = 0; m < NX; m++) s += Qr[m] * bch(hz, m);
                            g0x = s + qt;
                        } else {
                            g0x = (rowD && k >= 1 && k < N) ? Hct * vj : 0.0;
                        }
                        if (t < NU && k < N) {
                            double s = (k >= 1 && t < DOF) ? Hct * wj : 0.0;
                            s += Rt * zv;
                            g0v = s + rt;
                        }
                    }
                    if (lrw)  // + sum_j c_j u_j (u_j^T z)
#pragma unroll
                        for (int j = 0; j < LRM; j++) {
                            const double f = lrc[j] * uz[j];
                            g0x += f * u_y(j, k);
                            g0v += f * u_v(j, k);
                        }
                    if (xlw)
                        for (int j = 0; j < nlr_w; j++) {
                            const double f = XL[XL_C + j] * XL[XL_UZ + j];
                            g0x += f * u_y(j, k);
                            g0v += f * u_v(j, k);
                        }
                    wst(k, WF_GX, g0x);
                    wst(k, WF_GV, g0v);
                    double gx, gvv;
                    assemble_grad(cur, k, g0x, g0v, dvr, cP, gx, gvv);
                    if (k == N) {
                        // terminal stage: P = Hb_N (y block; Q row t used as column t), p = g_x~
#pragma unroll
                        for (int a = 0; a < NXA; a++) {
                            double v = 0.0;
                            if (rowY && a < NX) {
                                v = Qr[a];
                                if (a == t) v += wd;
                            }
                            Pc[a] = v;
                        }
                        pv = gx;
                        if (lrw)
#pragma unroll
                            for (int j = 0; j < LRM; j++) pj[j] = u_y(j, k);
                        return;
                    }
                    // ---- (1) Y = B~^T P (column t), f = g_v + B~^T p (lanes < NU)
                    double Y[NU];
#pragma unroll
                    for (int i = 0; i < DOF; i++) Y[i] = S[L_C + 16 + i] * Pc[i] + Pc[NX + i];
                    Y[UVS] = gs * Pc[XS] + gv * Pc[XVS];
                    const Halves hp = halves(pv);
                    const double pu = up32<NX>(pv, hp, t), pu1 = up32<1>(pv, hp, t);
                    const double fv = gvv + gt * pv + ((t < DOF) ? pu : gv * pu1);
                    // ---- (2) F column t (t < NU), Gm column t (t < NX); poly terms W_p bv_p bv_p^T, W_p bv_p a_p^T
                    //          (accumulated over p ascending per entry, as ipm.hip)
                    const double wdv = up_nx(wd, t);  // lane j <- ddq row j weight
                    const Halves hw = GRAM ? Halves{0.0, 0.0} : halves(WP);  // the VALU poly terms' broadcasts
                    double Fc[NU], gm[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        Fc[i] = (i == t) ? Rt + ((t < DOF) ? wdv : 0.0) : 0.0;
                        gm[i] = 0.0;
                    }
                    gram(cur, WP);
                    const double* const Dg = GM + (3 * grp) * 256 + (t & 15);  // column t of this instance's products
                    if constexpr (GRAM) {
#pragma unroll
                        for (int i = 0; i < DOF; i++) {
                            const double dbb = Dg[i * 16], dba = Dg[256 + i * 16];
                            Fc[i] += (t < DOF) ? dbb : 0.0;
                            gm[i] += (t < DOF) ? dba : 0.0;
                        }
                    }
#pragma unroll
                    for (int p = 0; p < (GRAM ? 0 : NPM); p++) {
                        const bool live = (double)p < cur.np && k < N;
                        const double wp = bch(hw, p);
                        const double Wp = live ? wp : 0.0;
                        const Halves hb = halves(cur.pb[p]);
#pragma unroll
                        for (int i = 0; i < DOF; i++) {
                            const double bvi = bch(hb, i);
                            Fc[i] += Wp * (bvi * cur.pb[p]);   // bv_p[t]: zero for lanes >= DOF
                            gm[i] += Wp * (bvi * cur.pa[p]);   // a_p[t]: zero for lanes >= DOF
                        }
                    }
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        const Halves hy = halves(Y[i]);
                        const double yu = up32<NX>(Y[i], hy, t);
                        const double yu1 = up32<1>(Y[i], hy, t);
                        const double yd = down32<1>(Y[i], hy, t);
                        Fc[i] = Fc[i] + (gt * Y[i] + ((t < DOF) ? yu : gv * yu1));
                        gm[i] = gm[i] + (mt * Y[i] + ((t == XVS) ? msv * yd : 0.0));
                    }
                    // ---- (3) chol(F) from the LDS copy of F; U = LF^-1 Gm; K = -LF^-T U; F^-1 row t;
                    //          kff = -F^-1 f; p = g_x~ + A~^T p + K^T f
                    if (t < NU)
#pragma unroll
                        for (int i = 0; i < NU; i++) S[MPCC_BCHK(c.bchk, L_F + i * 16 + t, L_U, BC_LDS)] = Fc[i];
                    lds_sync();
                    double LF[NU * (NU + 1) / 2], dinv[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        const double2* row = reinterpret_cast<const double2*>(S + L_F + i * 16);
#pragma unroll
                        for (int q2 = 0; q2 < (NU + 1) / 2; q2++) {
                            const double2 w = row[q2];
                            if (2 * q2 <= i) LF[i * (i + 1) / 2 + 2 * q2] = w.x;
                            if (2 * q2 + 1 <= i) LF[i * (i + 1) / 2 + 2 * q2 + 1] = w.y;
                        }
                    }
                    const bool cok = cholN(LF, dinv);
                    chol_ok = (cok || (GRAM && !run)) && chol_ok;
                    double u[NU];
                    const double gw = (k >= 1) ? Hct - wd : 0.0;
#pragma unroll
                    for (int i = 0; i < NU; i++) u[i] = rowY ? gm[i] : ((rowD && i == j9) ? gw : 0.0);
                    fwdN(LF, dinv, u);
                    double kc[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) kc[i] = u[i];
                    bwdN(LF, dinv, kc);
#pragma unroll
                    for (int i = 0; i < NU; i++) kc[i] = -kc[i];
                    double fi[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) fi[i] = (i == t) ? 1.0 : 0.0;
                    fwdN(LF, dinv, fi);
                    bwdN(LF, dinv, fi);
                    const Halves hf = halves(fv);
                    double fb[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) fb[i] = bch(hf, i);
                    double kff = 0.0;
#pragma unroll
                    for (int m = 0; m < NU; m++) kff -= fi[m] * fb[m];
                    double pnew;
                    {
                        double atp = 0.0;
                        const double p7 = down32<1>(pv, hp, t);  // lane XVS <- p_s
                        if (rowY) {
                            atp = mt * pv;
                            if (t == XVS) atp += msv * p7;
                        }
                        double ktf = 0.0;
#pragma unroll
                        for (int i = 0; i < NU; i++) ktf += kc[i] * fb[i];
                        pnew = gx + atp + ktf;
                    }
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        S[MPCC_BCHK(c.bchk, L_U + i * GW + t, L_C, BC_LDS)] = u[i];
                        wst(k, WF_KC + i, kc[i]);
                        wst(k, WF_FI + i, fi[i]);
                    }
                    wst(k, WF_KFF, (t < NU) ? kff : 0.0);
                    if (lrw)  // backward recursion of the low-rank solves, gradient u_j (y and v parts)
#pragma unroll
                        for (int j = 0; j < LRM; j++) {
                            const Halves hq = halves(pj[j]);
                            // both shifts unconditionally: a DPP read inside a divergent branch sees masked lanes as 0
                            const double qu = up32<NX>(pj[j], hq, t), qu1 = up32<1>(pj[j], hq, t);
                            const double fvj = u_v(j, k) + gt * pj[j] + ((t < DOF) ? qu : gv * qu1);
                            const Halves hfj = halves(fvj);
                            double kffj = 0.0, ktfj = 0.0;
#pragma unroll
                            for (int m = 0; m < NU; m++) {
                                const double fbm = bch(hfj, m);
                                kffj -= fi[m] * fbm;
                                ktfj += kc[m] * fbm;
                            }
                            wst(k, WF_KFJ + j, (t < NU) ? kffj : 0.0);
                            double atpj = 0.0;
                            const double pq7 = down32<1>(pj[j], hq, t);
                            if (rowY) {
                                atpj = mt * pj[j];
                                if (t == XVS) atpj += msv * pq7;
                            }
                            pj[j] = u_y(j, k) + atpj + ktfj;
                        }
                    // ---- (4) Hb column t and P = Hb - U^T U (column t); U rows are broadcast LDS reads
                    double hbv[NXA];
                    {
                        double Pc7[NX];
                        const double zero = 0.0;
#pragma unroll
                        for (int a = 0; a < NX; a++) Pc7[a] = down1(Pc[a], t);  // lane XVS <- P[a][XS]
#pragma unroll
                        for (int a = 0; a < NXA; a++) {
                            double v = 0.0;
                            if (a < NX) {
                                if (rowY) {
                                    v = Qr[a];
                                    if (a == t) v += wd;
                                }
                            } else if (a == t) {
                                v = wd;
                            }
                            hbv[a] = v;
                        }
                        if constexpr (GRAM) {
#pragma unroll
                            for (int a = 0; a < DOF; a++) {
                                const double daa = Dg[512 + a * 16];
                                hbv[a] += (t < DOF) ? daa : 0.0;
                            }
                        }
#pragma unroll
                        for (int p = 0; p < (GRAM ? 0 : NPM); p++) {
                            const bool live = (double)p < cur.np && k < N;
                            const double wpb = bch(hw, p);  // DPP outside the select
                            const double Wp = live ? wpb : zero;
                            const Halves ha = halves(cur.pa[p]);
#pragma unroll
                            for (int a = 0; a < DOF; a++) {
                                const double pab = bch(ha, a);
                                if (rowY) hbv[a] += Wp * (pab * cur.pa[p]);
                            }
                        }
                        if (rowY) {
#pragma unroll
                            for (int a = 0; a < NX; a++) {
                                const double ma = S[L_C + a];
                                double mp = (ma * mt) * Pc[a];
                                if (t == XVS) mp += (ma * msv) * Pc7[a];
                                if (a == XVS) mp += (msv * mt) * Pc[XS];
                                if (a == XVS && t == XVS) mp += (msv * msv) * Pc7[XS];
                                hbv[a] += mp;
                            }
                        }
                    }
                    lds_sync();
                    if (k > 0) {
#pragma unroll
                        for (int i = 0; i < NU; i++) {
                            const double2* row = reinterpret_cast<const double2*>(S + L_U + i * GW);
                            double ur[NXA];
#pragma unroll
                            for (int q2 = 0; q2 < NXA / 2; q2++) {
                                const double2 w = row[q2];
                                ur[2 * q2] = w.x;
                                ur[2 * q2 + 1] = w.y;
                            }
#pragma unroll
                            for (int a = 0; a < NXA; a++) hbv[a] -= ur[a] * u[i];
                        }
#pragma unroll
                        for (int a = 0; a < NXA; a++) Pc[a] = hbv[a];
                    }
                    pv = pnew;
                    lds_sync();
                });
                if (run && !chol_ok) {
                    conv = it > 0 && mu_cur < IPM_TOL_FB && rp_cur < IPM_TOL_FB;  // P2
                    alpha = 0.0;
                    run = false;
                }
            }
            if (run) {
                // ---- predictor forward: x~_0 = 0; recover dsa, dla; max step; mu(alpha) sums
                double S0 = 0, S1 = 0, S2 = 0;
                MinRatio amr(1.0);
                double xt = 0.0;
                auto pred_rec = [&](int k, const In& cur, double xs, double dvv) {
                    const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                    *ws(k, WF_AX) = xs;
                    *ws(k, WF_AV) = dvv;
                    const double cz = row_cz(k, cur.zx, cur.zv), ca = row_cz(k, xs, dvv);
                    const double pcz = PCACHE ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv), pca = poly_cz(cur, k, xs, dvv);
                    if constexpr (PCACHE) *ws(k, WF_PA) = pca;
                    auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l) {
                        if (!a) return;
                        const double rp = slot_rp(sgn, czz, bnd, s);
                        const SlotStep st = slot_recover(rcp(s), l, rp, sgn * caa, s * l);
                        step_bound(amr, s, l, st);
                        S0 += s * l;
                        S1 += s * st.dl + l * st.ds;
                        S2 += st.ds * st.dl;
                    };
                    rec(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL);
                    rec(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU);
                    rec(aP, sgnU, cur.pub, pcz, pca, cur.sP, cur.lP);
                };
                // Woodbury pieces of this factorization (low-rank option): Q_j, S = C^-1 + U^T Q
                double Smat[LRM * LRM];
#ifdef MPCC_IPM_TRACE
                double trc_t0 = 0.0, trc_S0 = 0.0;
#endif
                auto load_fix = [&](int k, In& o, bool corr) {  // stored dz_s (and predictor step) with the Q_j
                    load_common(k, o);
                    o.x0 = *ws(k, WF_AX); o.x1 = *ws(k, WF_AV);
                    o.x2 = corr ? *ws(k, WF_DX) : 0.0; o.x3 = corr ? *ws(k, WF_DV) : 0.0;
#pragma unroll
                    for (int j = 0; j < LRM; j++) { o.m[j] = *ws(k, WF_QX + j); o.m[LRM + j] = *ws(k, WF_QV + j); }
                };
                auto load_xfix = [&](int k, In& o, bool corr) {  // the stored dz_s (and predictor step)
                    load_common(k, o);
                    o.x0 = *ws(k, WF_AX); o.x1 = *ws(k, WF_AV);
                    o.x2 = corr ? *ws(k, WF_DX) : 0.0; o.x3 = corr ? *ws(k, WF_DV) : 0.0;
                };
                if (xlw) {
                    xl_q();
                    xl_smat_lu();
#ifdef MPCC_IPM_TRACE
                    trc_S0 = XL[XL_S];  // U[0][0] after the pivoting
#endif
                    light_sweep(false, [&](int k, In& o) { load_fwd(k, o, false); }, [&](int k, const In& cur) {
                        double v = 0.0, xn = 0.0;
                        fwd_step(cur, xt, v, xn);
                        *ws(k, WF_AX) = xt;  // dz_s
                        *ws(k, WF_AV) = (t < NU && k < N) ? v : 0.0;
                        xt = (k < N) ? xn : 0.0;
                    });
                    xl_dots(XL_TT, WF_AX, WF_AV);
                    xl_solve(XL_TT);
#ifdef MPCC_IPM_TRACE
                    trc_t0 = XL[XL_TT];
#endif
                    light_sweep(false, [&](int k, In& o) { load_xfix(k, o, false); }, [&](int k, const In& cur) {
                        double xs = cur.x0, dvv = cur.x1;
                        xl_fix(k, xs, dvv);
                        pred_rec(k, cur, xs, dvv);
                    });
                } else if (!lrw) {
                    light_sweep(false, [&](int k, In& o) { load_fwd(k, o, false); }, [&](int k, const In& cur) {
                        double v = 0.0, xn = 0.0;
                        fwd_step(cur, xt, v, xn);
                        pred_rec(k, cur, xt, (t < NU && k < N) ? v : 0.0);
                        xt = (k < N) ? xn : 0.0;
                    });
                } else {
                    double xq[LRM], udp[LRM], uqp[LRM * LRM];
#pragma unroll
                    for (int j = 0; j < LRM; j++) { xq[j] = 0.0; udp[j] = 0.0; }
#pragma unroll
                    for (int j = 0; j < LRM * LRM; j++) uqp[j] = 0.0;
                    light_sweep(false, [&](int k, In& o) { load_fwd(k, o, false); }, [&](int k, const In& cur) {
                        double v = 0.0, xn = 0.0;
                        fwd_step(cur, xt, v, xn);
                        const double dvv = (t < NU && k < N) ? v : 0.0;
                        *ws(k, WF_AX) = xt;  // dz_s
                        *ws(k, WF_AV) = dvv;
                        double uyk[LRM], uvk[LRM];
#pragma unroll
                        for (int j = 0; j < LRM; j++) {
                            uyk[j] = u_y(j, k);
                            uvk[j] = u_v(j, k);
                            udp[j] += uyk[j] * xt + uvk[j] * dvv;
                        }
#pragma unroll
                        for (int j = 0; j < LRM; j++) {  // Q_j = -solve(u_j), forward recursion
                            const double kfj = *ws(k, WF_KFJ + j);
                            double vq = 0.0, xqn = 0.0;
                            fwd_step_k(cur, xq[j], (k < N) ? kfj : 0.0, vq, xqn);
                            const double qx = (t < NXA) ? -xq[j] : 0.0, qv = (t < NU && k < N) ? -vq : 0.0;
                            *ws(k, WF_QX + j) = qx;
                            *ws(k, WF_QV + j) = qv;
#pragma unroll
                            for (int i = 0; i < LRM; i++) uqp[i * LRM + j] += uyk[i] * qx + uvk[i] * qv;
                            xq[j] = (k < N) ? xqn : 0.0;
                        }
                        xt = (k < N) ? xn : 0.0;
                    });
                    double tt[LRM], Sm[LRM * LRM];
#pragma unroll
                    for (int i = 0; i < LRM; i++) {
                        tt[i] = g_sum32(udp[i]);
#pragma unroll
                        for (int j = 0; j < LRM; j++) {
                            const double uq = g_sum32(uqp[i * LRM + j]);
                            Smat[i * LRM + j] = (i == j ? (i < nlr ? 1.0 / lrc[i] : 1.0) : 0.0) + uq;
                            Sm[i * LRM + j] = Smat[i * LRM + j];
                        }
                    }
                    solve_small(Sm, tt);
#ifdef MPCC_IPM_TRACE
                    trc_t0 = tt[0]; trc_S0 = Smat[0];
#endif
                    // dz = dz_s - Q S^-1 U^T dz_s, then the recovery of the predictor step
                    light_sweep(false, [&](int k, In& o) { load_fix(k, o, false); }, [&](int k, const In& cur) {
                        double xs = cur.x0, dvv = cur.x1;
#pragma unroll
                        for (int j = 0; j < LRM; j++) { xs -= tt[j] * cur.m[j]; dvv -= tt[j] * cur.m[LRM + j]; }
                        pred_rec(k, cur, xs, dvv);
                    });
                }
                const double amax = g_min32(amr.value());
                S0 = g_sum32(S0); S1 = g_sum32(S1); S2 = g_sum32(S2);
                const double mu = (mcount > 0) ? S0 / mcount : 0.0;
                if (it == 0) mu0 = mu;
                double mua = S0 + amax * S1 + amax * amax * S2;
                mua = (mcount > 0) ? mua / mcount : 0.0;
                const double ratio = (mu > 0) ? mua / mu : 0.0;
                const double sigma = (mu > 0) ? ratio * ratio * ratio : 0.0;
                const double smu = sigma * mu;

                // ---- corrector backward: coef with rc = s l + dsa dla - sigma mu; f = g_v + B~^T p;
                //      kff = -F^-1 f; p = g_x~ + A~^T p + K^T f
                double pv = 0.0;
                light_sweep(true, [&](int k, In& o) { load_bwd(k, o); }, [&](int k, const In& cur) {
                    const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                    const double cz = row_cz(k, cur.zx, cur.zv), ca = row_cz(k, cur.x0, cur.x1);
                    const double pcz = PCACHE ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv);
                    const double pca = PCACHE ? cur.pca : poly_cz(cur, k, cur.x0, cur.x1);
                    auto coef = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l) -> double {
                        if (!a) return 0.0;
                        const double rp = slot_rp(sgn, czz, bnd, s);
                        const double ri = rcp(s);
                        const SlotStep pa = slot_recover(ri, l, rp, sgn * caa, s * l);
                        const double rc = s * l + pa.ds * pa.dl - smu;
                        return slot_coef(ri, l, rp, rc);
                    };
                    const double cL = coef(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL);
                    const double cU = coef(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU);
                    const double cP = coef(aP, sgnU, cur.pub, pcz, pca, cur.sP, cur.lP);
                    const double dvr = sgnL * cL + sgnU * cU;
                    double gx, gvv;
                    assemble_grad(cur, k, cur.x2, cur.x3, dvr, cP, gx, gvv);
                    const Halves hp = halves(pv);
                    const double pu = up32<NX>(pv, hp, t), pu1 = up32<1>(pv, hp, t);
                    const double fv = gvv + gt * pv + ((t < DOF) ? pu : gv * pu1);
                    const Halves hf = halves(fv);
                    double fb[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) fb[i] = bch(hf, i);
                    double kff = 0.0;
#pragma unroll
                    for (int m = 0; m < NU; m++) kff -= cur.m[NU + m] * fb[m];
                    *ws(k, WF_KFF) = (t < NU && k < N) ? kff : 0.0;
                    double atp = 0.0;
                    const double p7 = down32<1>(pv, hp, t);
                    if (rowY) {
                        atp = mt * pv;
                        if (t == XVS) atp += msv * p7;
                    }
                    double ktf = 0.0;
#pragma unroll
                    for (int i = 0; i < NU; i++) ktf += cur.m[i] * fb[i];
                    pv = (k == N) ? gx : gx + atp + ktf;
                });

                // ---- corrector forward: dz, ds, dl, max step, mu(alpha) sums, max |rp|, max |dz|
                double T0 = 0, T1 = 0, T2 = 0, rpm = 0, dzm = 0;
                MinRatio amc(1e30);
                double uzd[LRM], uzdp[LRM];  // u_j^T dz of the corrector step
#pragma unroll
                for (int j = 0; j < LRM; j++) { uzd[j] = 0.0; uzdp[j] = 0.0; }
                auto corr_rec = [&](int k, const In& cur, double xtt, double dvv, double ax, double av) {
                    const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                    *ws(k, WF_DX) = xtt;
                    *ws(k, WF_DV) = dvv;
                    dzm = fmax(dzm, fmax(fabs(xtt), fabs(dvv)));
                    const double cz = row_cz(k, cur.zx, cur.zv), cd = row_cz(k, xtt, dvv), ca = row_cz(k, ax, av);
                    const double pcz = PCACHE ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv), pcd = poly_cz(cur, k, xtt, dvv);
                    const double pca = PCACHE ? cur.pca : poly_cz(cur, k, ax, av);
                    if constexpr (PCACHE) *ws(k, WF_PD) = pcd;
                    auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double cdd, double s, double l) {
                        if (!a) return;
                        double rp;
                        const SlotStep st = slot_corr(sgn, bnd, czz, caa, cdd, s, l, smu, &rp);
                        step_bound(amc, s, l, st);
                        T0 += s * l;
                        T1 += s * st.dl + l * st.ds;
                        T2 += st.ds * st.dl;
                        rpm = fmax(rpm, fabs(rp));
                    };
                    rec(aL, sgnL, cur.lb, cz, ca, cd, cur.sL, cur.lL);
                    rec(aU, sgnU, cur.ub, cz, ca, cd, cur.sU, cur.lU);
                    rec(aP, sgnU, cur.pub, pcz, pca, pcd, cur.sP, cur.lP);
                };
                xt = 0.0;
                if (xlw) {
                    light_sweep(false, [&](int k, In& o) { load_fwd(k, o, false); }, [&](int k, const In& cur) {
                        double v = 0.0, xn = 0.0;
                        fwd_step(cur, xt, v, xn);
                        *ws(k, WF_DX) = (t < NXA) ? xt : 0.0;  // dz_s
                        *ws(k, WF_DV) = (t < NU && k < N) ? v : 0.0;
                        xt = (k < N) ? xn : 0.0;
                    });
                    xl_dots(XL_TT, WF_DX, WF_DV);
                    xl_solve(XL_TT);
                    light_sweep(false, [&](int k, In& o) { load_xfix(k, o, true); }, [&](int k, const In& cur) {
                        double xtt = cur.x2, dvv = cur.x3;
                        xl_fix(k, xtt, dvv);
                        corr_rec(k, cur, xtt, dvv, cur.x0, cur.x1);
                    });
                    xl_dots(XL_UD, WF_DX, WF_DV);  // u_j^T dz of the corrector step
                } else if (!lrw) {
                    light_sweep(false, [&](int k, In& o) { load_fwd(k, o, true); }, [&](int k, const In& cur) {
                        double v = 0.0, xn = 0.0;
                        fwd_step(cur, xt, v, xn);
                        corr_rec(k, cur, (t < NXA) ? xt : 0.0, (t < NU && k < N) ? v : 0.0, cur.x0, cur.x1);
                        xt = (k < N) ? xn : 0.0;
                    });
                } else {
                    double udp[LRM];
#pragma unroll
                    for (int j = 0; j < LRM; j++) udp[j] = 0.0;
                    light_sweep(false, [&](int k, In& o) { load_fwd(k, o, false); }, [&](int k, const In& cur) {
                        double v = 0.0, xn = 0.0;
                        fwd_step(cur, xt, v, xn);
                        const double xtt = (t < NXA) ? xt : 0.0, dvv = (t < NU && k < N) ? v : 0.0;
                        *ws(k, WF_DX) = xtt;  // dz_s
                        *ws(k, WF_DV) = dvv;
#pragma unroll
                        for (int j = 0; j < LRM; j++) udp[j] += u_y(j, k) * xtt + u_v(j, k) * dvv;
                        xt = (k < N) ? xn : 0.0;
                    });
                    double tt[LRM], Sm[LRM * LRM];
#pragma unroll
                    for (int i = 0; i < LRM; i++) tt[i] = g_sum32(udp[i]);
#pragma unroll
                    for (int i = 0; i < LRM * LRM; i++) Sm[i] = Smat[i];
                    solve_small(Sm, tt);
                    light_sweep(false, [&](int k, In& o) { load_fix(k, o, true); }, [&](int k, const In& cur) {
                        double xtt = cur.x2, dvv = cur.x3;
#pragma unroll
                        for (int j = 0; j < LRM; j++) { xtt -= tt[j] * cur.m[j]; dvv -= tt[j] * cur.m[LRM + j]; }
                        corr_rec(k, cur, xtt, dvv, cur.x0, cur.x1);
#pragma unroll
                        for (int j = 0; j < LRM; j++) uzdp[j] += u_y(j, k) * xtt + u_v(j, k) * dvv;
                    });
#pragma unroll
                    for (int j = 0; j < LRM; j++) uzd[j] = g_sum32(uzdp[j]);
                }
                const double amx = g_min32(amc.value());
                T0 = g_sum32(T0); T1 = g_sum32(T1); T2 = g_sum32(T2);
                rpm = g_max32(rpm);
                dzm = g_max32(dzm);
                alpha = fmin(1.0, fmax(IPM_TAU, 1.0 - sqrt(mu)) * amx);
#pragma unroll
                for (int j = 0; j < LRM; j++) uz[j] += alpha * uzd[j];  // u_j^T z of the next iterate
#ifdef MPCC_IPM_TRACE
                const double trc_uz0 = xlw ? XL[XL_UZ] : uz[0] - alpha * uzd[0];
#endif
                if (xlw) {
                    if (t < nlr_w) XL[XL_UZ + t] += alpha * XL[XL_UD + t];
                    lds_sync();
                }
#ifdef MPCC_IPM_TRACE
                if (b == 0 && t == 0)
                    printf("gpu it %2d mu %.6e amax %.6e sig %.6e amx %.6e alpha %.6e rp %.6e dz %.6e uz0 %.9e t0 %.9e S0 %.9e\n",
                           it, mu, amax, sigma, amx, alpha, rpm, dzm, trc_uz0, trc_t0, trc_S0);
#endif
                sigma_mu = smu;
                pending = true;
                it++;
                if (it < max_it) {
                    double mun = T0 + alpha * T1 + alpha * alpha * T2;
                    mun = (mcount > 0) ? mun / mcount : 0.0;
                    const double rpn = (1.0 - alpha) * rpm;
                    mu_cur = mun;
                    rp_cur = rpn;
                    const bool step_ok = dzm < IPM_TOL_STEP || dzm * dzm < IPM_TOL_STEP * dz_prev;
                    dz_prev = dzm;
                    if (mun < IPM_TOL_MU && rpn < IPM_TOL_P && step_ok) {
                        conv = true;
                        run = false;
                    } else if (mun > IPM_DIV * mu0) {
                        diverged = true;
                        run = false;
                    }
                } else {
                    run = false;
                }
            }
        }
        it_total += it;
    }  // attempt

    if (!entered) return;
    if (t == 0) si[SQ_IPMIT] = it_total;
    if (!conv) {  // keep the previous step (Q6)
        if (t == 0) si[SQ_QPSTAT] = diverged ? MPCC_QP_PrimalInfeasible : MPCC_QP_MaxIterReached;
        return;
    }
    if (t == 0) si[SQ_QPSTAT] = 0;
    gdouble* stp = (gdouble*)(d.step + (size_t)b * NS * NXU);
    for (int k = 0; k <= N; k++) {
        const double zx = *ws(k, WF_ZX) + alpha * *ws(k, WF_DX);
        const double zv = *ws(k, WF_ZV) + alpha * *ws(k, WF_DV);
        if (t < NX) stp[k * NXU + t] = zx;
        if (t < NU) stp[k * NXU + NX + t] = (k < N) ? zv : 0.0;
    }
}

template <int NPM, bool LR>
__global__ void __launch_bounds__(64) k_ipm(DevConst c, DevBuffers d) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    ipm_group<NPM, LR>(c, d, smem);
}
template <int NPM, bool LR>
static void launch_ipm_t(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL((k_ipm<NPM, LR>), dim3((c.Bn + IPW - 1) / IPW), dim3(64), ipm_wide_lds_bytes(NPM, LR), s, c, d);
}
// one QP solve per active instance on the 32-lane interior point (lr: with the instances' low-rank terms)
void launch_ipm_wide(const DevConst& c, const DevBuffers& d, int npmax, int lr, hipStream_t s) {
    if (lr) {
        switch (npmax) {
            case 0: launch_ipm_t<0, true>(c, d, s); break;
            case 1: launch_ipm_t<1, true>(c, d, s); break;
            case 2: launch_ipm_t<2, true>(c, d, s); break;
            default: launch_ipm_t<11, true>(c, d, s); break;
        }
        return;
    }
    switch (npmax) {
        case 0: launch_ipm_t<0, false>(c, d, s); break;
        case 1: launch_ipm_t<1, false>(c, d, s); break;
        case 2: launch_ipm_t<2, false>(c, d, s); break;
        default: launch_ipm_t<11, false>(c, d, s); break;
    }
}

// ------------------------------------------------------------------------------------------------
// k_sqp: the SQP loop of solveOCP (osqp_interface.cpp:431-574) per instance, one 32-lane group per instance
// (as ipm.hip's k_sqp: QP solve, line-search trial lane = stage, filter decision, step, next QP assembly)
// ------------------------------------------------------------------------------------------------
__device__ __attribute__((noinline)) void sqp_setqp_phase(const DevConst& c, const DevBuffers& d, int b, int t,
                                                          const double* __restrict__ ucur, bool keep_hess) {
    const int N = c.N, NS = N + 1;
    const SplineView sp = spl_of(c.spl, b);
    const double* gb = d.guess + (size_t)b * NS * NXU;
    for (int k = t; k <= N; k += GW)
        setqp_stage(c, sp, gb, RecView{d.rec + (size_t)b * NS + k, c.S}, k, ucur, d.qs + ((size_t)b * NS + k) * QS,
                    keep_hess);
}
#ifndef MPCC_TRIAL_INLINE
#define MPCC_TRIAL_INLINE 1  // the trial inlined into the wave loop (ipm.hip: no callee-saved spills per call)
#endif
#if MPCC_TRIAL_INLINE
__device__ __forceinline__ void sqp_trial_phase(const DevConst& c, const DevBuffers& d, int b, int t,
#else
__device__ __attribute__((noinline)) void sqp_trial_phase(const DevConst& c, const DevBuffers& d, int b, int t,
#endif
                                                          const double* __restrict__ ucur, double alpha, bool keep) {
    const int N = c.N, NS = N + 1;
    for (int k = t; k <= N; k += GW) {
        double out[4];
        trial_stage(c, d, b, k, alpha, ucur, out);
        if (keep) {
            double* tr = d.trial + ((size_t)b * NS + k) * 4;
            for (int i = 0; i < 4; i++) tr[i] = out[i];
        }
    }
}
__device__ __attribute__((noinline)) void sqp_soc_phase(const DevConst& c, const DevBuffers& d, int b, int t,
                                                        const double* __restrict__ ucur) {
    const int N = c.N, NS = N + 1;
    const SplineView sp = spl_of(c.spl, b);
    const size_t o = (size_t)b * NS * NXU;
    for (int k = t; k <= N; k += GW)
        soc_stage(c, sp, d.guess + o, d.step + o, RecView{d.rec + (size_t)b * NS + k, c.S}, k, ucur,
                  d.qs + ((size_t)b * NS + k) * QS);
}
template <int NPM, bool LR>
__device__ __attribute__((noinline)) void sqp_ipm_phase(const DevConst& c, const DevBuffers& d, double* smem) {
    ipm_group<NPM, LR>(c, d, smem);
}

// ---- damped BFGS bookkeeping (osqp_interface.cpp:403-453, 540-555, 683-715), one 32-lane group per instance.
//      Vectors in the horizon layout [(N+1)][x (NX) | u (NU)] (u_N = 0), normalized as the QP; the oracle's
//      solve_ocp / bfgs_update.
// element e of B s: the stage Hessians of SQP iteration 0 (QS_Q, QS_R and the ddq coupling Hct between u_k and
// u_{k-1}, k in [1, N-1]) plus the low-rank terms sum_j c_j (u_j^T s) u_j (us[j] = u_j^T s)
__device__ __forceinline__ double bfgs_hmul_elem(const DevConst& c, const double* __restrict__ qsb, const double* __restrict__ sv,
                                                 const double* __restrict__ lrb, const double* __restrict__ lrcb, const double* us,
                                                 int nlr, int N, int e) {
    const int NS = N + 1;
    const int k = e / NXU, a = e - NXU * k;
    const double* q = qsb + (size_t)k * QS;
    double v = 0.0;
    if (a < NX) {
        for (int m = 0; m < NX; m++) v += q[QS_Q + a * NX + m] * sv[NXU * k + m];
    } else if (k < N) {
        const int i = a - NX;
        v = q[QS_R + i] * sv[e];
        if (i < DOF) {
            const double hct = c.p.Tu[i] * (-2. * c.p.qp_r_ddq) * c.p.Tu[i];
            if (k >= 1) v += hct * sv[e - NXU];
            if (k + 1 <= N - 1) v += hct * sv[e + NXU];
        }
    }
#pragma unroll
    for (int j = 0; j < LRX; j++)
        if (j < nlr) v += (lrcb[j] * us[j]) * lrb[(size_t)j * NS * NXU + e];
    return v;
}
// the QP gradient (normalized grad_obj) of element e: Tx f_x / Tu f_u + ddq gradient (QS_q / QS_r)
__device__ __forceinline__ double bfgs_q_elem(const double* __restrict__ qsb, int N, int e) {
    const int k = e / NXU, a = e - NXU * k;
    const double* q = qsb + (size_t)k * QS;
    return (a < NX) ? q[QS_q + a] : ((k < N) ? q[QS_r + a - NX] : 0.0);
}
// u_j^T s over the horizon for the instance's low-rank terms (group reductions)
__device__ __forceinline__ void bfgs_us(const double* __restrict__ lrb, const double* __restrict__ sv, int nlr, int NE, int t,
                                        double (&us)[LRX]) {
#pragma unroll
    for (int j = 0; j < LRX; j++) {
        double p = 0.0;
        if (j < nlr)
            for (int e = t; e < NE; e += GW) p += lrb[(size_t)j * NE + e] * sv[e];
        us[j] = g_sum32(p);
    }
}
// SQP iteration it (after setQP): grad_L = q + A^T lambda; for it > 0, dgrad_L = grad_L - grad_L_prev and
// Hess_ = BFGSUpdate(Hess_, step_prev, dgrad_L) appends -Bs Bs^T / sBs + r r^T / sr to the low-rank terms.
// Returns false when the update makes the Hessian NaN (sBs = 0 with sr >= eps): NAN_HESSIAN (:474-477).
// restart (the instance holds LRX - 1 or more terms, so the update would not fit): this iteration's exact
// Hessian (setQP with keep_hess off) becomes the new iteration-0 Hessian and the terms are dropped, as the
// oracle's solve_ocp (BFGS_MAX_TERMS); grad_L is recorded as in iteration 0.
__device__ __attribute__((noinline)) bool bfgs_pre(const DevConst& c, const DevBuffers& d, int b, int t, int it,
                                                   bool restart) {
    const int N = c.N, NS = N + 1, NE = NS * NXU;
    int32_t* si = d.sqi + (size_t)b * SQI;
    const int nlr = si[SQ_NLR];
    const double* qsb = d.qs + (size_t)b * NS * QS;
    double* lrb = d.lr + (size_t)b * d.lrs * NE;
    const double* lrcb = d.lrc + (size_t)b * d.lrs;
    double* glam = d.glam + (size_t)b * NE;
    double* gprev = d.gprev + (size_t)b * NE;
    const double* sp = d.sp + (size_t)b * NE;
    if (it == 0 || restart) {
        for (int e = t; e < NE; e += GW) gprev[e] = bfgs_q_elem(qsb, N, e) + glam[e];
        if (restart && t == 0) si[SQ_NLR] = 0;
        return true;
    }
    // dgrad_L into slot nlr + 1, B step_prev into slot nlr (B of the previous iteration)
    double* bsv = lrb + (size_t)nlr * NE;
    double* dgv = lrb + (size_t)(nlr + 1) * NE;
    double us[LRX];
    bfgs_us(lrb, sp, nlr, NE, t, us);
    double sbs = 0.0, sy = 0.0;
    for (int e = t; e < NE; e += GW) {
        const double gl = bfgs_q_elem(qsb, N, e) + glam[e];
        const double dg = gl - gprev[e];
        gprev[e] = gl;
        const double bs = bfgs_hmul_elem(c, qsb, sp, lrb, lrcb, us, nlr, N, e);  // reads slots < nlr only
        bsv[e] = bs;
        dgv[e] = dg;
        sbs += sp[e] * bs;
        sy += sp[e] * dg;
    }
    sbs = g_sum32(sbs);
    sy = g_sum32(sy);
    double theta = 1.0, sr = sy;
    const bool damp = sy < 0.2 * sbs;
    if (damp) {
        theta = 0.8 * sbs / (sbs - sy);
        sr = theta * sy + (1 - theta) * sbs;
    }
    if (sr < 2.220446049250313e-16) return true;  // unchanged Hessian (std::numeric_limits<double>::epsilon())
    if (!(sbs != 0.0) || !isfinite(sbs) || !isfinite(sr)) return false;
    for (int e = t; e < NE; e += GW) {
        const double dg = dgv[e];
        dgv[e] = damp ? theta * dg + (1 - theta) * bsv[e] : dg;  // r
    }
    if (t == 0) {
        double* lc = d.lrc + (size_t)b * d.lrs;
        lc[nlr] = -1.0 / sbs;
        lc[nlr + 1] = 1.0 / sr;
        si[SQ_NLR] = nlr + 2;
    }
    return true;
}
// after the QP (and the correction): A^T y = -(B step + q) of the exact QP solution (its stationarity)
__device__ __attribute__((noinline)) void bfgs_post_qp(const DevConst& c, const DevBuffers& d, int b, int t) {
    const int N = c.N, NS = N + 1, NE = NS * NXU;
    const int nlr = d.sqi[(size_t)b * SQI + SQ_NLR];
    const double* qsb = d.qs + (size_t)b * NS * QS;
    const double* lrb = d.lr + (size_t)b * d.lrs * NE;
    const double* lrcb = d.lrc + (size_t)b * d.lrs;
    const double* stp = d.step + (size_t)b * NE;
    double* aty = d.aty + (size_t)b * NE;
    double us[LRX];
    bfgs_us(lrb, stp, nlr, NE, t, us);
    for (int e = t; e < NE; e += GW) aty[e] = -(bfgs_hmul_elem(c, qsb, stp, lrb, lrcb, us, nlr, N, e) + bfgs_q_elem(qsb, N, e));
}
// after the line search: lambda += alpha (y - lambda) as A^T lambda, step_prev = alpha step (:540-555)
__device__ __attribute__((noinline)) void bfgs_post_step(const DevConst& c, const DevBuffers& d, int b, int t, double alpha) {
    const int NE = (c.N + 1) * NXU;
    double* glam = d.glam + (size_t)b * NE;
    double* sp = d.sp + (size_t)b * NE;
    const double* aty = d.aty + (size_t)b * NE;
    const double* stp = d.step + (size_t)b * NE;
    for (int e = t; e < NE; e += GW) {
        glam[e] = glam[e] + alpha * (aty[e] - glam[e]);
        sp[e] = alpha * stp[e];
    }
}

template <int NPM, bool LR>
__global__ void __launch_bounds__(64) k_sqp(DevConst, DevBuffers, const double* __restrict__ ucur_all) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const DevConst& c = kernarg_const();     // the arguments in place (kernels.h kernarg_const)
    const DevBuffers& d = kernarg_buffers();
    const int t = threadIdx.x % GW;
    const int b = blockIdx.x * IPW + threadIdx.x / GW;
    const bool valid = b < c.Bn;
    const int N = c.N, NS = N + 1;
    const int bb = valid ? b : 0;
    int32_t* si = d.sqi + (size_t)bb * SQI;
    const double* ucur = ucur_all + NU * bb;
    if constexpr (LR) {  // fresh BFGS state per solveOCP (:403-408)
        if (valid)
            for (int e = t; e < NS * NXU; e += GW) d.glam[(size_t)b * NS * NXU + e] = 0.0;
    }
    PhaseClock ph(d.phase_cyc);  // the ComputeTime split (mpcc_timing): set_qp / solve_qp / get_alpha / step
    for (int it = 0; it < c.p.max_iter; it++) {
        bool act = valid && si[SQ_ACTIVE] != 0;
        if (__ballot(act) == 0) break;
        ph.mark(PH_STEP);
        // damped BFGS past LRX terms: restart from this iteration's exact Hessian (bfgs_pre)
        const bool restart = LR && it > 0 && act && si[SQ_NLR] + 2 > LRX;
        if (it > 0) {
            if (act) sqp_setqp_phase(c, d, b, t, ucur, LR && !restart);
            __syncthreads();
        }
        if constexpr (LR) {
            if (act && !bfgs_pre(c, d, b, t, it, restart) && t == 0) { si[SQ_STATUS] = MPCC_NAN_HESSIAN; si[SQ_ACTIVE] = 0; }
            __syncthreads();
        }
        ph.mark(PH_SETQP);  // setQP and the Hessian update (osqp_interface.cpp:435-475)
        sqp_ipm_phase<NPM, LR>(c, d, smem);
        __syncthreads();
        if (c.p.do_SOC) {  // SecondOrderCorrection (osqp_interface.cpp:506-535)
            act = valid && si[SQ_ACTIVE] != 0;
            if (act) sqp_soc_phase(c, d, b, t, ucur);
            __syncthreads();
            sqp_ipm_phase<NPM, LR>(c, d, smem);
            __syncthreads();
        }
        act = valid && si[SQ_ACTIVE] != 0;
        if constexpr (LR) {
            if (act) bfgs_post_qp(c, d, b, t);
            __syncthreads();
        }
        ph.mark(PH_SOLVE);
        if (act) sqp_trial_phase(c, d, b, t, ucur, 1.0, true);
        __syncthreads();
        if (act && t == 0) accept_instance(c, d, b);
        __syncthreads();
        if (act && c.faithful_dead_trials && si[SQ_REJECT]) {
            double alpha = 1.0;
            for (int l = 1; l < c.p.line_search_max_iter; l++) {
                alpha *= c.p.line_search_tau;
                sqp_trial_phase(c, d, b, t, ucur, alpha, false);
            }
        }
        ph.mark(PH_ALPHA);
        double nrm = 0.0;
        if (act) {
            const double alpha = d.sqd[(size_t)b * SQ + SQ_ALPHA];
            if constexpr (LR) bfgs_post_step(c, d, b, t, alpha);
            nrm = apply_range<8>(c, d, b, t, GW, alpha);
        }
        nrm = g_max32(nrm);
        if (act && t == 0) finish_iteration(c, d, b, nrm);
        __syncthreads();
    }
    ph.mark(PH_STEP);
    ph.flush(threadIdx.x == 0);
}

template <int NPM, bool LR>
static void launch_sqp_t(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s) {
    hipLaunchKernelGGL((k_sqp<NPM, LR>), dim3((c.Bn + IPW - 1) / IPW), dim3(64), ipm_wide_lds_bytes(NPM, LR), s, c, d, u_cur);
}

void launch_sqp_wide(const DevConst& c, const DevBuffers& d, const double* u_cur, int npmax, int bfgs, hipStream_t s) {
    if (bfgs) {
        switch (npmax) {
            case 0: launch_sqp_t<0, true>(c, d, u_cur, s); break;
            case 1: launch_sqp_t<1, true>(c, d, u_cur, s); break;
            case 2: launch_sqp_t<2, true>(c, d, u_cur, s); break;
            default: launch_sqp_t<11, true>(c, d, u_cur, s); break;
        }
        return;
    }
    switch (npmax) {
        case 0: launch_sqp_t<0, false>(c, d, u_cur, s); break;
        case 1: launch_sqp_t<1, false>(c, d, u_cur, s); break;
        case 2: launch_sqp_t<2, false>(c, d, u_cur, s); break;
        default: launch_sqp_t<11, false>(c, d, u_cur, s); break;
    }
}

#if MPCC_DOF != 7
// the mobile build's QP solver (the Panda build's is ipm.hip)
size_t ipm_lds_bytes(int /*N*/, int npmax) { return ipm_wide_lds_bytes(npmax > 2 ? 11 : npmax, true); }
void launch_ipm(const DevConst& c, const DevBuffers& d, int npmax, hipStream_t s) { launch_ipm_wide(c, d, npmax, 0, s); }
bool launch_sqp_solo(const DevConst&, const DevBuffers&, const double*, int, hipStream_t) { return false; }
void launch_sqp(const DevConst& c, const DevBuffers& d, const double* u_cur, int npmax, hipStream_t s) {
    launch_sqp_wide(c, d, u_cur, npmax, c.p.use_BFGS, s);
}
#endif

}  // namespace mpcc
