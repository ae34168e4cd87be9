// ipm.hip — k_ipm: the per-instance QP solve that replaces OSQP (osqp_interface.cpp:592-656).
//
// Mehrotra predictor-corrector interior point on the stage-structured normalized QP;
// same start point, tolerances, step rule and iteration-count rule as oracle/mpcc_oracle.cpp
// solve_struct_ipm.  Step systems are solved by a Riccati recursion over the augmented stage state
// x~ = [y(9), w(7)] (w_k = v_{k-1}[0:7] carries the ddq coupling) with input v(8).
//
// MI355X mapping:
//  * one 16-lane DPP row per instance, 4 instances per wavefront.  Lane t owns row t of the stage
//    (t < 9: box row on y_t, t >= 9: ddq row j = t-9), poly row t, column t of the 16x16 Riccati
//    matrices and component t of the stage vectors.  Cross-lane traffic inside an instance uses DPP
//    row shifts / rotations or the instance's private LDS block; there are no workgroup barriers.
//  * the dynamics are sparse (M = diag(m) + m78 e7 e8^T, G = diag(g) + g87 e8 e7^T, checked on the
//    host): the Riccati products are written out structurally; the dense work per stage is chol(F)
//    (8x8, redundant per lane), U = LF^-1 Gm and K = -F^-1 Gm (lane = column) and P = Hb - U^T U
//    (lane = row).
//  * per-stage state (slacks, multipliers, iterate, steps, gains) streams through a coalesced
//    [field][16 lanes] global workspace.  Backward solves are mat-vecs (p = g + A~^T p + K^T f,
//    kff = -F^-1 f) and so are forward solves (v = K x~ + kff): no division chains outside chol(F).
//  * the predictor backward solve is fused into the factorization sweep, and the iterate update of
//    iteration i is applied lazily by the factorization sweep of iteration i+1.  The convergence test
//    uses mu(alpha) = (S0 + alpha S1 + alpha^2 S2)/m and rp(alpha) = (1 - alpha) rp, accumulated by
//    the corrector forward sweep (exact identities of the oracle's update, rounding aside).
#include "dev_common.h"
#include "kernels.h"

namespace mpcc {

constexpr int IPM_MAX_IT = 60;
constexpr double IPM_TOL_MU = 1e-13, IPM_TOL_P = 1e-11, IPM_TOL_STEP = 1e-11;
constexpr double IPM_TOL_FB = 1e-9;  // P2: a converged iterate is accepted when the Riccati factor breaks down
constexpr int IPW = 4;  // instances per wavefront (16 lanes each)

// workspace fields, ws[((b*(N+1) + k)*IS + field*16 + lane]
enum : int {
    WF_SL = 0, WF_LL, WF_SU, WF_LU, WF_SP, WF_LP,  // slack / multiplier of the lower, upper and poly slot of row t
    WF_ZX, WF_ZV,                                 // iterate: lane c -> x~_c (y, w); lane j < 8 -> v_j
    WF_DX, WF_DV,                                 // corrector step (same layout)
    WF_AX, WF_AV,                                 // predictor step
    WF_GX, WF_GV,                                 // objective gradient H z + h
    WF_KFF,                                       // kff (lanes 0..7)
    WF_KC,                                        // 8 fields: K column layout, field i lane c = K[i][c]
    WF_KR = WF_KC + 8,                            // 8 fields: K row halves, field m: lane i -> K[i][m], lane 8+i -> K[i][8+m]
    WF_FI = WF_KR + 8,                            // 4 fields: F^-1 row halves, field m: lane i -> Fi[i][m], lane 8+i -> Fi[i][4+m]
    NWF = WF_FI + 4
};
static_assert(NWF * 16 <= IS, "IPM workspace must fit the per-stage IS allocation");

// per-instance LDS block (doubles)
constexpr int L_P = 0;      // 16x16 Riccati P (full, symmetric)
constexpr int L_U = 256;    // 8x16  Y = B~^T P scratch, then U = LF^-1 Gm, [i*16 + c]
constexpr int L_K = 384;    // 8x16  K, [i*16 + c]
constexpr int L_F = 512;    // 8x8   F, [i*8 + j]
constexpr int L_Z = 576;    // 24    stage iterate z = [y, w, v]
constexpr int L_DZ = 600;   // 24    corrector step
constexpr int L_DA = 624;   // 24    predictor step
constexpr int L_X = 648;    // 2x16  forward x~ (ping-pong)
constexpr int L_PV = 680;   // 2x16  backward p (ping-pong)
constexpr int L_FV = 712;   // 8     f
constexpr int L_WD = 720;   // 16    row barrier weights W_lo + W_up
constexpr int L_PC = 736;   // 16    poly coefficients
constexpr int L_POLY = 752; // npmax x 16: a[7], bv[7], ub, W
__host__ __device__ constexpr int grp_lds(int npmax) { return L_POLY + 16 * (npmax > 0 ? npmax : 1); }

size_t ipm_lds_bytes(int /*N*/, int npmax) { return (size_t)IPW * grp_lds(npmax) * sizeof(double); }

#ifdef MPCC_IPM_PROF
// cycle accounting per k_ipm section (profiling build only, see _build.py / tools/ipm_prof.py)
__device__ unsigned long long g_ipm_prof[16];
#define PMARK(i) do { const long long t_ = clock64(); prof_acc[i] += t_ - prof_t; prof_t = t_; } while (0)
#else
#define PMARK(i) do { } while (0)
#endif

namespace {

// ---- 16-lane row primitives (DPP rows coincide with instances) ---------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(v);
    int lo = (int)(unsigned)(x & 0xffffffffull), hi = (int)(unsigned)(x >> 32);
    lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xF, 0xF, true);
    hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int n> __device__ __forceinline__ double from_up(double v) { return dpp_d<0x100 + n>(v); }    // row_shl: lane t <- t+n
template <int n> __device__ __forceinline__ double from_down(double v) { return dpp_d<0x110 + n>(v); } // row_shr: lane t <- t-n
template <int n> __device__ __forceinline__ double rot16(double v) { return dpp_d<0x120 + n>(v); }     // row_ror
__device__ __forceinline__ double g_sum(double v) {
    v += rot16<8>(v); v += rot16<4>(v); v += rot16<2>(v); v += rot16<1>(v);
    return v;
}
__device__ __forceinline__ double g_max(double v) {
    v = fmax(v, rot16<8>(v)); v = fmax(v, rot16<4>(v)); v = fmax(v, rot16<2>(v)); v = fmax(v, rot16<1>(v));
    return v;
}
__device__ __forceinline__ double g_min(double v) {
    v = fmin(v, rot16<8>(v)); v = fmin(v, rot16<4>(v)); v = fmin(v, rot16<2>(v)); v = fmin(v, rot16<1>(v));
    return v;
}

// One wavefront per workgroup: cross-lane LDS hand-offs only need this wave's LDS operations retired
// and a compiler barrier; __syncthreads() would also drain outstanding global loads (vmcnt(0)).
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---- slot algebra (oracle solve_struct_ipm), slot: sgn*(c^T z) <= sgn*bnd ----------------------
struct SlotStep {
    double ds, dl;
};
__device__ __forceinline__ double slot_rp(double sgn, double cz, double bnd, double s) { return sgn * cz - sgn * bnd + s; }
__device__ __forceinline__ SlotStep slot_recover(double s, double l, double rp, double cd, double rc) {
    const double W = l / s;
    return {-rp - cd, W * (cd + rp) - rc / s};
}
__device__ __forceinline__ double slot_coef(double s, double l, double rp, double rc) { return l + (l / s) * rp - rc / s; }
__device__ __forceinline__ double step_bound(double a, double s, double l, SlotStep d) {
    if (d.ds < 0) a = fmin(a, -s / d.ds);
    if (d.dl < 0) a = fmin(a, -l / d.dl);
    return a;
}
// corrector step of a slot given the iterate (cz), the predictor step (ca) and the corrector step (cd)
__device__ __forceinline__ SlotStep slot_corr(double sgn, double bnd, double cz, double ca, double cd, double s, double l,
                                              double smu, double* rp_out) {
    const double rp = slot_rp(sgn, cz, bnd, s);
    const SlotStep pa = slot_recover(s, l, rp, sgn * ca, s * l);
    const double rc = s * l + pa.ds * pa.dl - smu;
    *rp_out = rp;
    return slot_recover(s, l, rp, sgn * cd, rc);
}

// Cholesky of the 8x8 stage F (lower triangle read from LDS), packed; reciprocal pivots
__device__ __forceinline__ bool chol8(const double* F, double* L, double* dinv) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) L[i * (i + 1) / 2 + j] = F[i * 8 + j];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int jj = j * (j + 1) / 2;
        double d = L[jj + j];
#pragma unroll
        for (int m = 0; m < j; m++) d -= L[jj + m] * L[jj + m];
        ok = ok && (d > 0);
        d = sqrt(d);
        L[jj + j] = d;
        const double inv = 1.0 / d;
        dinv[j] = inv;
#pragma unroll
        for (int i = j + 1; i < 8; i++) {
            const int ii = i * (i + 1) / 2;
            double s = L[ii + j];
#pragma unroll
            for (int m = 0; m < j; m++) s -= L[ii + m] * L[jj + m];
            L[ii + j] = s * inv;
        }
    }
    return ok;
}
__device__ __forceinline__ void fwd8(const double* L, const double* dinv, double* x) {  // x = LF^-1 x
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int ii = i * (i + 1) / 2;
        double s = x[i];
#pragma unroll
        for (int m = 0; m < i; m++) s -= L[ii + m] * x[m];
        x[i] = s * dinv[i];
    }
}
__device__ __forceinline__ void bwd8(const double* L, const double* dinv, double* x) {  // x = LF^-T x
#pragma unroll
    for (int i = 7; i >= 0; i--) {
        double s = x[i];
#pragma unroll
        for (int m = i + 1; m < 8; m++) s -= L[m * (m + 1) / 2 + i] * x[m];
        x[i] = s * dinv[i];
    }
}

}  // namespace

template <int NPM>
__global__ void __launch_bounds__(64) k_ipm(DevConst c, DevBuffers d) {
    constexpr int NPE = NPM > 0 ? NPM : 1;      // poly rows held in LDS (row 0 stays zero when NPM = 0)
    constexpr int PFP = (15 * NPM + 15) / 16;   // poly prefetch registers per lane
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int lane = threadIdx.x;
    const int grp = lane >> 4;
    const int t = lane & 15;
    const int b = blockIdx.x * IPW + grp;
    const int N = c.N;
    const int NS = N + 1;
    double* const S = smem + grp * grp_lds(NPM);
#ifdef MPCC_IPM_PROF
    long long prof_acc[16] = {0};
    long long prof_t = clock64();
#endif

    const bool valid = b < c.Bn;
    int32_t* si = d.sqi + (size_t)(valid ? b : 0) * SQI;
    bool run = valid && si[SQ_ACTIVE] != 0;
    if (__ballot(run) == 0) return;

    const double* QSb = d.qs + (size_t)(valid ? b : 0) * NS * QS;
    double* WSb = d.is + (size_t)(valid ? b : 0) * NS * IS;
    auto ws = [&](int k, int f) -> double* { return WSb + (size_t)k * IS + f * 16 + t; };

    // ---- model constants of this lane (sparse M, G; selects keep the kernel-argument reads scalar)
    const double m78 = c.M[7 * 9 + 8], m77 = c.M[7 * 10], m88 = c.M[8 * 10];
    const double g77 = c.G[7 * 8 + 7], g87 = c.G[8 * 8 + 7];
    double mt = 0.0, gt = 0.0, Hct = 0.0;
    const double HcB = -2. * c.p.qp_r_ddq;
#pragma unroll
    for (int a = 0; a < 9; a++)
        if (t == a) mt = c.M[a * 10];
#pragma unroll
    for (int a = 0; a < 7; a++)
        if (t == a || t == 9 + a) {
            gt = (t < 7) ? c.G[a * 9] : 0.0;
            Hct = c.p.Tu[a] * HcB * c.p.Tu[a];
        }
    if (t == 7) gt = g77;
    const bool rowY = t < 9;
    const int j9 = t - 9;
    constexpr double sgnL = -1.0, sgnU = 1.0;

    // ---- Hessian checks (osqp_interface.cpp:454-473): stage flags from k_setqp + tridiagonal input blocks
    int fl = 0;
    if (run) {
        for (int k = t; k < NS; k += 16) fl |= (int)QSb[(size_t)k * QS + QS_FLAG];
        if (t < 8) {
            double prev_d = 0;
            for (int k = 0; k < N; k++) {
                const double dk = QSb[(size_t)k * QS + QS_R + t];
                const double off = (k >= 1 && t < DOF) ? Hct : 0.0;
                const double l = (k >= 1) ? off / prev_d : 0.0;
                const double dd = dk - l * l;
                if (dd <= 0) { fl |= 2; break; }
                prev_d = sqrt(dd);
            }
        }
    }
    {
        int o = 0;
#pragma unroll
        for (int bit = 0; bit < 3; bit++)
            if (g_max((double)((fl >> bit) & 1)) > 0.5) o |= 1 << bit;
        fl = o;
    }
    if (run && (fl & 2)) { if (t == 0) { si[SQ_STATUS] = MPCC_NON_PD_HESSIAN; si[SQ_ACTIVE] = 0; } run = false; }
    if (run && (fl & 1)) { if (t == 0) { si[SQ_STATUS] = MPCC_NAN_HESSIAN; si[SQ_ACTIVE] = 0; } run = false; }
    if (run && (fl & 4)) { if (t == 0) si[SQ_QPSTAT] = MPCC_QP_PrimalInfeasible; run = false; }  // keep old step (Q6)
    const bool entered = run;

    // ---- per-stage inputs, loaded one stage ahead of their use (software pipelining of the sweeps)
    struct StageIn {
        double lb, ub;          // bounds of row t
        int np;                 // live poly rows
        double pv[PFP > 0 ? PFP : 1];
        double sL, lL, sU, lU, sP, lP, zx, zv;
        double x0, x1, x2, x3;  // sweep-specific pairs (dz / dza / g0)
        double m[12];           // sweep-specific: Q row + q,R,r | K rows + kff | K column + Finv half
    };
    auto load_common = [&](int k, StageIn& o) {
        const double* q = QSb + (size_t)k * QS;
        o.lb = q[rowY ? QS_YLB + t : QS_DLB + j9];
        o.ub = q[rowY ? QS_YUB + t : QS_DUB + j9];
        o.np = (int)q[QS_NPOLY];
#pragma unroll
        for (int i = 0; i < PFP; i++) {
            const int e = t + 16 * i;
            o.pv[i] = (e < 15 * NPM) ? q[QS_POLY + e] : 0.0;
        }
        o.sL = *ws(k, WF_SL); o.lL = *ws(k, WF_LL); o.sU = *ws(k, WF_SU); o.lU = *ws(k, WF_LU);
        o.sP = *ws(k, WF_SP); o.lP = *ws(k, WF_LP);
        o.zx = *ws(k, WF_ZX); o.zv = *ws(k, WF_ZV);
    };
    auto load_bounds = [&](int k, double& lb, double& ub, int& np) {
        const double* q = QSb + (size_t)k * QS;
        lb = q[rowY ? QS_YLB + t : QS_DLB + j9];
        ub = q[rowY ? QS_YUB + t : QS_DUB + j9];
        np = (int)q[QS_NPOLY];
    };
    auto load_poly = [&](int k, double* r) {
        const double* q = QSb + (size_t)k * QS + QS_POLY;
#pragma unroll
        for (int i = 0; i < PFP; i++) {
            const int e = t + 16 * i;
            r[i] = (e < 15 * NPM) ? q[e] : 0.0;
        }
    };
    // stage the poly rows (rows >= np zeroed); returns this lane's poly bound (INF: no live row t)
    auto stage_poly = [&](const double* r, int np, int k) -> double {
#pragma unroll
        for (int i = 0; i < PFP; i++) {
            const int e = t + 16 * i;
            if (e < 15 * NPM) {
                const int p = e / 15, m = e - 15 * p;
                S[L_POLY + p * 16 + m] = (p < np && k < N) ? r[i] : 0.0;
            }
        }
        lds_sync();
        return (t < np && t < NPM && k < N) ? S[L_POLY + t * 16 + 14] : INF;
    };
    auto row_active = [&](int k, double bnd) { return (rowY ? (k >= 1) : (k < N)) && fabs(bnd) < BIG; };
    // unsigned c^T z of this lane's box/ddq row and of poly row t; z = stage vector in LDS at off
    auto row_cz = [&](int k, int off) -> double {
        if (rowY) return S[off + t];
        const double v = S[off + 16 + j9];
        return (k == 0) ? v : v - S[off + 9 + j9];
    };
    auto poly_cz = [&](int off) -> double {
        if (t >= NPM) return 0.0;
        const double* row = S + L_POLY + t * 16;
        double s = 0;
#pragma unroll
        for (int m = 0; m < 7; m++) s += row[m] * S[off + m];
#pragma unroll
        for (int m = 0; m < 7; m++) s += row[7 + m] * S[off + 16 + m];
        return s;
    };
    auto put_vec = [&](int off, double x, double v) {  // lane c: x~_c, lane j < 8: v_j
        S[off + t] = x;
        if (t < 8) S[off + 16 + t] = v;
    };
    auto load_factor = [&](int k, StageIn& o, bool upd) {
        load_common(k, o);
        const double* q = QSb + (size_t)k * QS;
#pragma unroll
        for (int m = 0; m < 9; m++) o.m[m] = (t < 9) ? q[QS_Q + t * 9 + m] : 0.0;
        o.m[9] = (t < 9) ? q[QS_q + t] : 0.0;
        o.m[10] = (t < 8 && k < N) ? q[QS_R + t] : 0.0;
        o.m[11] = (t < 8 && k < N) ? q[QS_r + t] : 0.0;
        if (upd) {
            o.x0 = *ws(k, WF_DX); o.x1 = *ws(k, WF_DV); o.x2 = *ws(k, WF_AX); o.x3 = *ws(k, WF_AV);
        } else {
            o.x0 = o.x1 = o.x2 = o.x3 = 0.0;
        }
    };
    auto load_fwd = [&](int k, StageIn& o, bool corr) {
        load_common(k, o);
        if (k < N) {
#pragma unroll
            for (int m = 0; m < 8; m++) o.m[m] = *ws(k, WF_KR + m);
            o.m[8] = *ws(k, WF_KFF);
        } else {
#pragma unroll
            for (int m = 0; m < 9; m++) o.m[m] = 0.0;
        }
        if (corr) { o.x0 = *ws(k, WF_AX); o.x1 = *ws(k, WF_AV); } else { o.x0 = o.x1 = 0.0; }
    };
    auto load_bwd = [&](int k, StageIn& o) {
        load_common(k, o);
        o.x0 = *ws(k, WF_AX); o.x1 = *ws(k, WF_AV); o.x2 = *ws(k, WF_GX); o.x3 = *ws(k, WF_GV);
        if (k < N) {
#pragma unroll
            for (int i = 0; i < 8; i++) o.m[i] = *ws(k, WF_KC + i);
#pragma unroll
            for (int m = 0; m < 4; m++) o.m[8 + m] = *ws(k, WF_FI + m);
        } else {
#pragma unroll
            for (int m = 0; m < 12; m++) o.m[m] = 0.0;
        }
    };

    // ---- start point: dynamics rollout with v = 0, s = max(-g, 1), lambda = 1
    double mcount = 0.0;
    if (run) {
        double y = 0.0;  // lane a < 9: y_a of stage k
        double lb, ub, bk; int np;
        double pv[PFP > 0 ? PFP : 1];
        auto load_start = [&](int k, double& lb_, double& ub_, int& np_, double* pv_, double& bk_) {
            load_bounds(k, lb_, ub_, np_);
            load_poly(k, pv_);
            bk_ = (k < N && t < 9) ? QSb[(size_t)k * QS + QS_B + t] : 0.0;
        };
        load_start(0, lb, ub, np, pv, bk);
        for (int k = 0; k <= N; k++) {
            double lbn = 0, ubn = 0, bkn = 0; int npn = 0;
            double pvn[PFP > 0 ? PFP : 1];
            if (k < N) load_start(k + 1, lbn, ubn, npn, pvn, bkn);
            put_vec(L_Z, rowY ? y : 0.0, 0.0);
            const double pb = stage_poly(pv, np, k);
            const double cz = row_cz(k, L_Z);
            const double pcz = poly_cz(L_Z);
            const bool aL = row_active(k, lb), aU = row_active(k, ub), aP = fabs(pb) < BIG;
            double sL = 1, lL = 0, sU = 1, lU = 0, sP = 1, lP = 0;
            if (aL) { sL = fmax(-(sgnL * cz - sgnL * lb), 1.0); lL = 1.0; }
            if (aU) { sU = fmax(-(sgnU * cz - sgnU * ub), 1.0); lU = 1.0; }
            if (aP) { sP = fmax(-(sgnU * pcz - sgnU * pb), 1.0); lP = 1.0; }
            mcount += (aL ? 1.0 : 0.0) + (aU ? 1.0 : 0.0) + (aP ? 1.0 : 0.0);
            *ws(k, WF_SL) = sL; *ws(k, WF_LL) = lL; *ws(k, WF_SU) = sU; *ws(k, WF_LU) = lU;
            *ws(k, WF_SP) = sP; *ws(k, WF_LP) = lP;
            *ws(k, WF_ZX) = rowY ? y : 0.0;
            *ws(k, WF_ZV) = 0.0;
            // y_{k+1} = M y_k + b_k (oracle order: sum_b M[a][b] y_b, then + b_a)
            const double y8 = from_up<1>(y);  // lane 7 <- y_8
            const double yn = (t == 7) ? m77 * y + m78 * y8 : mt * y;
            y = (t < 9) ? yn + bk : 0.0;
            lb = lbn; ub = ubn; np = npn; bk = bkn;
#pragma unroll
            for (int i = 0; i < PFP; i++) pv[i] = pvn[i];
            lds_sync();
        }
    }
    mcount = g_sum(mcount);
    PMARK(0);

    int it = 0;
    bool conv = false;
    double alpha = 0.0, sigma_mu = 0.0;  // previous iteration's step length and sigma*mu (lazy update)
    double mu_cur = 1e30, rp_cur = 1e30; // mu and max |rp| of the current iterate (known for it > 0)
    bool pending = false;
    StageIn cur, nxt;
    while (true) {
        if (__ballot(run) == 0) break;
        if (run) {
            // ================= factorization sweep k = N..0 with the lazy update of the previous step,
            // the objective gradient g0 = H z + h and the predictor backward solve
            int pcur = 0;  // p ping-pong slot holding p_{k+1}
            bool chol_ok = true;
            load_factor(N, cur, pending);
            PMARK(1);
            for (int k = N; k >= 0; k--) {
                if (k > 0) load_factor(k - 1, nxt, pending);
                const double lb = cur.lb, ub = cur.ub;
                const double* Qr = cur.m;
                const double qt = cur.m[9], Rt = cur.m[10], rt = cur.m[11];
                double sL = cur.sL, lL = cur.lL, sU = cur.sU, lU = cur.lU, sP = cur.sP, lP = cur.lP;
                double zx = cur.zx, zv = cur.zv;
                const double pb = stage_poly(cur.pv, cur.np, k);
                const bool aL = row_active(k, lb), aU = row_active(k, ub), aP = fabs(pb) < BIG;
                if (pending) {
                    // previous iteration's update at this stage (oracle: z += a dz, s += a ds, l += a dl)
                    const double dx = cur.x0, dv = cur.x1, ax = cur.x2, av = cur.x3;
                    put_vec(L_Z, zx, zv); put_vec(L_DZ, dx, dv); put_vec(L_DA, ax, av);
                    lds_sync();
                    const double cz = row_cz(k, L_Z), cd = row_cz(k, L_DZ), ca = row_cz(k, L_DA);
                    const double pcz = poly_cz(L_Z), pcd = poly_cz(L_DZ), pca = poly_cz(L_DA);
                    double rpd;
                    if (aL) { const SlotStep st = slot_corr(sgnL, lb, cz, ca, cd, sL, lL, sigma_mu, &rpd); sL += alpha * st.ds; lL += alpha * st.dl; }
                    if (aU) { const SlotStep st = slot_corr(sgnU, ub, cz, ca, cd, sU, lU, sigma_mu, &rpd); sU += alpha * st.ds; lU += alpha * st.dl; }
                    if (aP) { const SlotStep st = slot_corr(sgnU, pb, pcz, pca, pcd, sP, lP, sigma_mu, &rpd); sP += alpha * st.ds; lP += alpha * st.dl; }
                    zx += alpha * dx;
                    zv += alpha * dv;
                    *ws(k, WF_SL) = sL; *ws(k, WF_LL) = lL; *ws(k, WF_SU) = sU; *ws(k, WF_LU) = lU;
                    *ws(k, WF_SP) = sP; *ws(k, WF_LP) = lP;
                    *ws(k, WF_ZX) = zx; *ws(k, WF_ZV) = zv;
                    lds_sync();
                }
                PMARK(8);
                put_vec(L_Z, zx, zv);
                lds_sync();
                // ---- slots: barrier weights and predictor coefficients (rc = s l)
                const double cz = row_cz(k, L_Z);
                const double pcz = poly_cz(L_Z);
                double WL = 0, WU = 0, WP = 0, cL = 0, cU = 0, cP = 0;
                if (aL) { const double rp = slot_rp(sgnL, cz, lb, sL); WL = lL / sL; cL = slot_coef(sL, lL, rp, sL * lL); }
                if (aU) { const double rp = slot_rp(sgnU, cz, ub, sU); WU = lU / sU; cU = slot_coef(sU, lU, rp, sU * lU); }
                if (aP) { const double rp = slot_rp(sgnU, pcz, pb, sP); WP = lP / sP; cP = slot_coef(sP, lP, rp, sP * lP); }
                const double wd = WL + WU;                 // diagonal weight of row t
                const double dvr = sgnL * cL + sgnU * cU;  // signed coefficient of row t
                S[L_PC + t] = cP;
                if (t < NPE) S[L_POLY + t * 16 + 15] = WP;
                // ---- objective gradient g0 = H z + h (f_xu = 0; oracle order: sum over z, then + h)
                double g0x, g0v = 0.0;
                if (t < 9) {
                    double s = 0;
#pragma unroll
                    for (int m = 0; m < 9; m++) s += Qr[m] * S[L_Z + m];
                    g0x = s + qt;
                } else {
                    g0x = (k >= 1 && k < N) ? Hct * S[L_Z + 16 + j9] : 0.0;
                }
                if (t < 8 && k < N) {
                    double s = (k >= 1 && t < DOF) ? Hct * S[L_Z + 9 + t] : 0.0;
                    s += Rt * zv;
                    g0v = s + rt;
                }
                *ws(k, WF_GX) = g0x;
                *ws(k, WF_GV) = g0v;
                lds_sync();
                // ---- step-system gradient (predictor): g = g0 + sum_i sgn_i coef_i c_i
                double gx = g0x, gv = g0v;
                if (t < 9) {
                    gx += dvr;
                    if (t < 7)
#pragma unroll
                        for (int p = 0; p < NPM; p++) gx += S[L_PC + p] * S[L_POLY + p * 16 + t];
                } else if (k >= 1) {
                    gx -= dvr;
                }
                const double dv_up = from_up<9>(dvr);  // lane j <- ddq row j
                if (t < 7 && k < N) {
                    gv += dv_up;
#pragma unroll
                    for (int p = 0; p < NPM; p++) gv += S[L_PC + p] * S[L_POLY + p * 16 + 7 + t];
                }
                if (k == N) {
                    // terminal stage: P = Hb_N (y block only), p = g_x~ (upper triangle mirrored, lane = row)
#pragma unroll
                    for (int cc = 0; cc < 16; cc++) {
                        double v = 0.0;
                        if (t < 9 && cc < 9) {
                            v = Qr[cc];
                            if (cc == t) v += wd;
                        }
                        if (cc >= t) { S[L_P + t * 16 + cc] = v; S[L_P + cc * 16 + t] = v; }
                    }
                    S[L_PV + t] = gx;
                    pcur = 0;
                    lds_sync();
                    cur = nxt;
                    continue;
                }
                PMARK(9);
                // ---- (1) Y = B~^T P (lane n: column n of Y from column n of P), f = g_v + B~^T p
                double Pc[16];
#pragma unroll
                for (int i = 0; i < 16; i++) Pc[i] = S[L_P + i * 16 + t];
                {
                    double Y[8];
#pragma unroll
                    for (int i = 0; i < 7; i++) Y[i] = c.G[i * 9] * Pc[i] + Pc[9 + i];
                    Y[7] = g77 * Pc[7] + g87 * Pc[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) S[L_U + i * 16 + t] = Y[i];
                }
                const double* pn = S + L_PV + 16 * pcur;
                if (t < 8) {
                    const double bp = (t < 7) ? gt * pn[t] + pn[9 + t] : g77 * pn[7] + g87 * pn[8];
                    S[L_FV + t] = gv + bp;
                }
                lds_sync();
                // ---- (2) Hb_yy row t, F column t (t < 8), Gm column t (t < 9)
                double Hb[9];
                {
                    const double P77 = S[L_P + 7 * 16 + 7];
#pragma unroll
                    for (int cc = 0; cc < 9; cc++) {
                        const double mc = c.M[cc * 10];
                        double v = Qr[cc];
                        if (cc == t) v += wd;
                        if (t < 7 && cc < 7)
#pragma unroll
                            for (int p = 0; p < NPM; p++) {
                                const double* row = S + L_POLY + p * 16;
                                v += row[15] * (row[t] * row[cc]);
                            }
                        double mp = (mt * mc) * Pc[cc];
                        if (cc == 8) mp += (mt * m78) * Pc[7];
                        if (t == 8) mp += (m78 * mc) * S[L_P + 7 * 16 + cc];
                        if (t == 8 && cc == 8) mp += (m78 * m78) * P77;
                        Hb[cc] = v + mp;
                    }
                }
                double gm[8];
                {
                    // F[:, t] = H_vv[:, t] + (Y B~)[:, t];  B~ column j = g_j e_j + e_{9+j} (j < 7), g77 e7 + g87 e8
                    const bool fj = t < 7;
                    const int c1 = fj ? t : 7, c2 = fj ? 9 + t : 8;
                    const double w2 = fj ? 1.0 : g87;
                    const double wdv = from_up<9>(wd);  // lane j <- ddq row j weight
                    double Fc[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const double v = gt * S[L_U + i * 16 + c1] + w2 * S[L_U + i * 16 + c2];
                        double h = 0.0;
                        if (i == t) {
                            h = Rt;
                            if (fj) h += wdv;
                        }
                        if (i < 7 && fj)
#pragma unroll
                            for (int p = 0; p < NPM; p++) {
                                const double* row = S + L_POLY + p * 16;
                                h += row[15] * (row[7 + i] * row[7 + t]);
                            }
                        Fc[i] = h + v;
                    }
                    if (t < 8)
#pragma unroll
                        for (int i = 0; i < 8; i++) S[L_F + i * 8 + t] = Fc[i];
                    // Gm[:, t] = H_vy[:, t] + (Y M)[:, t] (t < 9); w columns are diag(Hc - W_ddq) (k >= 1)
                    const int ct = (t < 9) ? t : 0;
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        double v = mt * S[L_U + i * 16 + ct];
                        if (t == 8) v += m78 * S[L_U + i * 16 + 7];
                        double h = 0.0;
                        if (i < 7 && t < 7)
#pragma unroll
                            for (int p = 0; p < NPM; p++) {
                                const double* row = S + L_POLY + p * 16;
                                h += row[15] * (row[7 + i] * row[ct]);
                            }
                        gm[i] = h + v;
                    }
                }
                lds_sync();
                PMARK(10);
                // ---- (3) chol(F); U = LF^-1 Gm; K = -LF^-T U; Finv column (t & 7); kff = -F^-1 f;
                //          p = g_x~ + A~^T p + K^T f
                double LF[36], dinv[8];
                chol_ok = chol8(S + L_F, LF, dinv) && chol_ok;
                double u[8];
                const double gw = (k >= 1) ? Hct - wd : 0.0;
#pragma unroll
                for (int i = 0; i < 8; i++) u[i] = (t < 9) ? gm[i] : ((i == j9) ? gw : 0.0);
                fwd8(LF, dinv, u);
                double kc[8];
#pragma unroll
                for (int i = 0; i < 8; i++) kc[i] = u[i];
                bwd8(LF, dinv, kc);
#pragma unroll
                for (int i = 0; i < 8; i++) kc[i] = -kc[i];
                double fi[8];
#pragma unroll
                for (int i = 0; i < 8; i++) fi[i] = (i == (t & 7)) ? 1.0 : 0.0;
                fwd8(LF, dinv, fi);
                bwd8(LF, dinv, fi);
                double f[8];
#pragma unroll
                for (int i = 0; i < 8; i++) f[i] = S[L_FV + i];
                double kff = 0.0;
#pragma unroll
                for (int m = 0; m < 8; m++) kff -= fi[m] * f[m];
                {
                    double atp = 0.0;
                    if (t < 9) {
                        atp = mt * pn[t];
                        if (t == 8) atp += m78 * pn[7];
                    }
                    double ktf = 0.0;
#pragma unroll
                    for (int i = 0; i < 8; i++) ktf += kc[i] * f[i];
                    S[L_PV + 16 * (pcur ^ 1) + t] = gx + atp + ktf;
                }
                PMARK(11);
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    S[L_U + i * 16 + t] = u[i];
                    S[L_K + i * 16 + t] = kc[i];
                    *ws(k, WF_KC + i) = kc[i];
                }
                *ws(k, WF_KFF) = (t < 8) ? kff : 0.0;
#pragma unroll
                for (int m = 0; m < 4; m++) *ws(k, WF_FI + m) = (t < 8) ? fi[m] : fi[4 + m];
                lds_sync();
                {
                    const int ri = t & 7, hoff = (t < 8) ? 0 : 8;
#pragma unroll
                    for (int m = 0; m < 8; m++) *ws(k, WF_KR + m) = S[L_K + ri * 16 + hoff + m];
                }
                PMARK(12);
                // ---- (4) P = Hb - U^T U (lane = row t, upper triangle mirrored)
                if (k > 0) {
#pragma unroll
                    for (int cc = 0; cc < 16; cc++) {
                        if (cc < t) continue;
                        double v = 0.0;
                        if (t < 9 && cc < 9) v = Hb[cc];
                        else if (t >= 9 && cc == t) v = wd;
#pragma unroll
                        for (int i = 0; i < 8; i++) v -= u[i] * S[L_U + i * 16 + cc];
                        S[L_P + t * 16 + cc] = v;
                        S[L_P + cc * 16 + t] = v;
                    }
                }
                pcur ^= 1;
                lds_sync();
                cur = nxt;
                PMARK(13);
            }
            if (!chol_ok) {
                // Riccati breakdown: MaxIterReached unless the current iterate is converged to IPM_TOL_FB (P2);
                // the sweep has already applied the pending update, so the iterate is the stored z
                conv = it > 0 && mu_cur < IPM_TOL_FB && rp_cur < IPM_TOL_FB;
                alpha = 0.0;
                run = false;
            }
        }
        PMARK(2);
        if (run) {
            // forward sweep body shared by the predictor and the corrector:
            // x~_0 = 0; v = K x~ + kff; x~' = A~ x~ + B~ v; returns (x~_k, v_k) of stage k
            auto fwd_step = [&](int k, const StageIn& in, int xc, double& xt, double& vv) {
                const double* xs = S + L_X + 16 * xc;
                xt = xs[t];
                double v = 0.0;
                if (k < N) {
                    const int hoff = (t < 8) ? 0 : 8;
                    double part = 0.0;
#pragma unroll
                    for (int m = 0; m < 8; m++) part += in.m[m] * xs[hoff + m];
                    v = part + from_up<8>(part) + in.m[8];
                    const double x8 = xs[8];
                    const double v7 = from_down<1>(v);
                    const double vj = from_down<9>(v);
                    double xn;
                    if (t < 7) xn = mt * xt + gt * v;
                    else if (t == 7) xn = (m77 * xt + m78 * x8) + g77 * v;
                    else if (t == 8) xn = m88 * xt + g87 * v7;
                    else xn = vj;
                    S[L_X + 16 * (xc ^ 1) + t] = xn;
                }
                vv = (t < 8 && k < N) ? v : 0.0;
            };
            // ---- predictor forward: recover dsa, dla; max step; mu(alpha) sums
            double S0 = 0, S1 = 0, S2 = 0, amax = 1.0;
            int xc = 0;
            S[L_X + t] = 0.0;
            load_fwd(0, cur, false);
            lds_sync();
            for (int k = 0; k <= N; k++) {
                if (k < N) load_fwd(k + 1, nxt, false);
                const double pb = stage_poly(cur.pv, cur.np, k);
                const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = fabs(pb) < BIG;
                double xt, dvv;
                fwd_step(k, cur, xc, xt, dvv);
                *ws(k, WF_AX) = xt;
                *ws(k, WF_AV) = dvv;
                put_vec(L_Z, cur.zx, cur.zv);
                put_vec(L_DA, xt, dvv);
                lds_sync();
                const double cz = row_cz(k, L_Z), ca = row_cz(k, L_DA);
                const double pcz = poly_cz(L_Z), pca = poly_cz(L_DA);
                auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l) {
                    if (!a) return;
                    const double rp = slot_rp(sgn, czz, bnd, s);
                    const SlotStep st = slot_recover(s, l, rp, sgn * caa, s * l);
                    amax = step_bound(amax, s, l, st);
                    S0 += s * l;
                    S1 += s * st.dl + l * st.ds;
                    S2 += st.ds * st.dl;
                };
                rec(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL);
                rec(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU);
                rec(aP, sgnU, pb, pcz, pca, cur.sP, cur.lP);
                xc ^= 1;
                lds_sync();
                cur = nxt;
            }
            amax = g_min(amax);
            S0 = g_sum(S0); S1 = g_sum(S1); S2 = g_sum(S2);
            const double mu = (mcount > 0) ? S0 / mcount : 0.0;
            double mua = S0 + amax * S1 + amax * amax * S2;
            mua = (mcount > 0) ? mua / mcount : 0.0;
            const double ratio = (mu > 0) ? mua / mu : 0.0;
            const double sigma = (mu > 0) ? ratio * ratio * ratio : 0.0;
            const double smu = sigma * mu;
            PMARK(3);

            // ---- corrector backward: coef with rc = s l + dsa dla - sigma mu; f = g_v + B~^T p;
            //      kff = -F^-1 f; p = g_x~ + A~^T p + K^T f
            int pcur = 0;
            load_bwd(N, cur);
            for (int k = N; k >= 0; k--) {
                if (k > 0) load_bwd(k - 1, nxt);
                const double pb = stage_poly(cur.pv, cur.np, k);
                const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = fabs(pb) < BIG;
                put_vec(L_Z, cur.zx, cur.zv);
                put_vec(L_DA, cur.x0, cur.x1);
                lds_sync();
                const double cz = row_cz(k, L_Z), ca = row_cz(k, L_DA);
                const double pcz = poly_cz(L_Z), pca = poly_cz(L_DA);
                auto coef = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l) -> double {
                    if (!a) return 0.0;
                    const double rp = slot_rp(sgn, czz, bnd, s);
                    const SlotStep pa = slot_recover(s, l, rp, sgn * caa, s * l);
                    const double rc = s * l + pa.ds * pa.dl - smu;
                    return slot_coef(s, l, rp, rc);
                };
                const double cL = coef(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL);
                const double cU = coef(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU);
                const double cP = coef(aP, sgnU, pb, pcz, pca, cur.sP, cur.lP);
                const double dvr = sgnL * cL + sgnU * cU;
                S[L_PC + t] = cP;
                lds_sync();
                double gx = cur.x2, gv = cur.x3;
                if (t < 9) {
                    gx += dvr;
                    if (t < 7)
#pragma unroll
                        for (int p = 0; p < NPM; p++) gx += S[L_PC + p] * S[L_POLY + p * 16 + t];
                } else if (k >= 1) {
                    gx -= dvr;
                }
                const double dv_up = from_up<9>(dvr);
                if (t < 7 && k < N) {
                    gv += dv_up;
#pragma unroll
                    for (int p = 0; p < NPM; p++) gv += S[L_PC + p] * S[L_POLY + p * 16 + 7 + t];
                }
                if (k == N) {
                    S[L_PV + t] = gx;
                    pcur = 0;
                    lds_sync();
                    cur = nxt;
                    continue;
                }
                const double* pn = S + L_PV + 16 * pcur;
                if (t < 8) {
                    const double bp = (t < 7) ? gt * pn[t] + pn[9 + t] : g77 * pn[7] + g87 * pn[8];
                    S[L_FV + t] = gv + bp;
                }
                lds_sync();
                double f[8];
#pragma unroll
                for (int i = 0; i < 8; i++) f[i] = S[L_FV + i];
                const int hoff = (t < 8) ? 0 : 4;
                double part = 0.0;
#pragma unroll
                for (int m = 0; m < 4; m++) part -= cur.m[8 + m] * f[hoff + m];
                const double kff = part + from_up<8>(part);
                *ws(k, WF_KFF) = (t < 8) ? kff : 0.0;
                if (k > 0) {
                    double atp = 0.0;
                    if (t < 9) {
                        atp = mt * pn[t];
                        if (t == 8) atp += m78 * pn[7];
                    }
                    double ktf = 0.0;
#pragma unroll
                    for (int i = 0; i < 8; i++) ktf += cur.m[i] * f[i];
                    S[L_PV + 16 * (pcur ^ 1) + t] = gx + atp + ktf;
                }
                pcur ^= 1;
                lds_sync();
                cur = nxt;
            }
            PMARK(4);

            // ---- corrector forward: dz, ds, dl, max step, mu(alpha) sums, max |rp|, max |dz|
            double T0 = 0, T1 = 0, T2 = 0, amx = 1e30, rpm = 0, dzm = 0;
            xc = 0;
            S[L_X + t] = 0.0;
            load_fwd(0, cur, true);
            lds_sync();
            for (int k = 0; k <= N; k++) {
                if (k < N) load_fwd(k + 1, nxt, true);
                const double pb = stage_poly(cur.pv, cur.np, k);
                const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = fabs(pb) < BIG;
                double xt, dvv;
                fwd_step(k, cur, xc, xt, dvv);
                *ws(k, WF_DX) = xt;
                *ws(k, WF_DV) = dvv;
                dzm = fmax(dzm, fmax(fabs(xt), fabs(dvv)));
                put_vec(L_Z, cur.zx, cur.zv);
                put_vec(L_DZ, xt, dvv);
                put_vec(L_DA, cur.x0, cur.x1);
                lds_sync();
                const double cz = row_cz(k, L_Z), cd = row_cz(k, L_DZ), ca = row_cz(k, L_DA);
                const double pcz = poly_cz(L_Z), pcd = poly_cz(L_DZ), pca = poly_cz(L_DA);
                auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double cdd, double s, double l) {
                    if (!a) return;
                    double rp;
                    const SlotStep st = slot_corr(sgn, bnd, czz, caa, cdd, s, l, smu, &rp);
                    amx = step_bound(amx, s, l, st);
                    T0 += s * l;
                    T1 += s * st.dl + l * st.ds;
                    T2 += st.ds * st.dl;
                    rpm = fmax(rpm, fabs(rp));
                };
                rec(aL, sgnL, cur.lb, cz, ca, cd, cur.sL, cur.lL);
                rec(aU, sgnU, cur.ub, cz, ca, cd, cur.sU, cur.lU);
                rec(aP, sgnU, pb, pcz, pca, pcd, cur.sP, cur.lP);
                xc ^= 1;
                lds_sync();
                cur = nxt;
            }
            amx = g_min(amx);
            T0 = g_sum(T0); T1 = g_sum(T1); T2 = g_sum(T2);
            rpm = g_max(rpm);
            dzm = g_max(dzm);
            alpha = fmin(1.0, 0.995 * amx);
            sigma_mu = smu;
            pending = true;
            it++;
            PMARK(5);
            // convergence test at the start of the next iteration (oracle: only while it < IPM_MAX_IT)
            if (it < IPM_MAX_IT) {
                double mun = T0 + alpha * T1 + alpha * alpha * T2;
                mun = (mcount > 0) ? mun / mcount : 0.0;
                const double rpn = (1.0 - alpha) * rpm;
                mu_cur = mun;
                rp_cur = rpn;
                if (mun < IPM_TOL_MU && rpn < IPM_TOL_P && dzm < IPM_TOL_STEP) {
                    conv = true;
                    run = false;
                }
            } else {
                run = false;
            }
        }
    }

#ifdef MPCC_IPM_PROF
    if (entered && t == 0) {
        for (int i = 0; i < 16; i++) if (i != 6 && i != 7) atomicAdd(&g_ipm_prof[i], (unsigned long long)prof_acc[i]);
        atomicAdd(&g_ipm_prof[6], (unsigned long long)it);
        atomicAdd(&g_ipm_prof[7], 1ull);
    }
#endif
    if (!entered) return;
    if (t == 0) si[SQ_IPMIT] = it;
    if (!conv) {
        if (t == 0) si[SQ_QPSTAT] = MPCC_QP_MaxIterReached;  // keep the previous step (Q6)
        return;
    }
    if (t == 0) si[SQ_QPSTAT] = 0;
    double* stp = d.step + (size_t)b * NS * 17;
    for (int k = 0; k <= N; k++) {
        const double zx = *ws(k, WF_ZX) + alpha * *ws(k, WF_DX);
        const double zv = *ws(k, WF_ZV) + alpha * *ws(k, WF_DV);
        if (t < 9) stp[k * 17 + t] = zx;
        if (t < 8) stp[k * 17 + 9 + t] = (k < N) ? zv : 0.0;
    }
}

#ifdef MPCC_IPM_PROF
extern "C" int mpcc_debug_ipm_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ipm_prof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ipm_prof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif

template <int NPM>
static void launch_ipm_t(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    const size_t lds = ipm_lds_bytes(c.N, NPM);
    static bool configured = false;
    if (!configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ipm<NPM>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        configured = true;
    }
    hipLaunchKernelGGL(k_ipm<NPM>, dim3((c.Bn + IPW - 1) / IPW), dim3(64), lds, s, c, d);
}

void launch_ipm(const DevConst& c, const DevBuffers& d, int npmax, hipStream_t s) {
    switch (npmax) {
        case 0: launch_ipm_t<0>(c, d, s); break;
        case 1: launch_ipm_t<1>(c, d, s); break;
        case 2: launch_ipm_t<2>(c, d, s); break;
        case 9: launch_ipm_t<9>(c, d, s); break;
        case 10: launch_ipm_t<10>(c, d, s); break;
        default: launch_ipm_t<11>(c, d, s); break;
    }
}

}  // namespace mpcc
