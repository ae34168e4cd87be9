// ipm.hip — k_ipm: the per-instance QP solve that replaces OSQP (osqp_interface.cpp:592-656).
//
// Mehrotra predictor-corrector interior point on the stage-structured normalized QP;
// same start point, tolerances, step rule and iteration-count rule as oracle/mpcc_oracle.cpp
// solve_struct_ipm.  Step systems are solved by a Riccati recursion over the augmented stage state
// x~ = [y(9), w(7)] (w_k = v_{k-1}[0:7] carries the ddq coupling) with input v(8).
//
// MI355X mapping:
//  * one 16-lane DPP row per instance, 4 instances per wavefront.  Lane t owns row t of the stage
//    (t < 9: box row on y_t, t >= 9: ddq row j = t-9), poly row t, component t of every stage vector
//    and column t of every 16x16 / 8x16 stage matrix.  All of it lives in registers: P is carried
//    from stage to stage as one column per lane, and every exchange inside an instance is a DPP row
//    broadcast (row_newbcast) or row shift — no LDS round trip, so no lgkmcnt waits on the chain.
//    The only LDS traffic is U (8x16) for P = Hb - U^T U (broadcast ds_read_b128 of U's rows) and
//    the K transpose for the forward-solve layout.
//  * the dynamics are sparse (M = diag(m) + m78 e7 e8^T, G = diag(g) + g87 e8 e7^T, checked on the
//    host): the Riccati products are written out structurally; the dense work per stage is chol(F)
//    (8x8, redundant per lane), U = LF^-1 Gm, K = -F^-1 Gm (lane = column) and P = Hb - U^T U.
//  * per-stage state (slacks, multipliers, iterate, steps, gains) streams through a coalesced
//    [field][16 lanes] global workspace, prefetched one stage ahead.  Backward solves are mat-vecs
//    (p = g + A~^T p + K^T f, kff = -F^-1 f) and so are forward solves (v = K x~ + kff).
//  * the predictor backward solve is fused into the factorization sweep, and the iterate update of
//    iteration i is applied lazily by the factorization sweep of iteration i+1.  The convergence test
//    uses mu(alpha) = (S0 + alpha S1 + alpha^2 S2)/m and rp(alpha) = (1 - alpha) rp, accumulated by
//    the corrector forward sweep (exact identities of the oracle's update, rounding aside).
#include <type_traits>

// QP assembly, records and line-search pieces of k_sqp: oracle operation order, no FP contraction, exactly as
// kernels.hip (-ffp-contract=off) builds them; the shared headers' helpers (dev_common.h's 3x3 products of the
// kinematics and the spline frames) are parsed under the same setting, so the in-kernel records and QP records are
// bitwise k_records' and k_setqp's
#pragma clang fp contract(off)
#include "dev_common.h"
#include "dev_dpp.h"
#include "kernels.h"
#include "dev_sqp.h"
#include "dev_records.h"
#pragma clang fp contract(fast)

namespace mpcc {

static_assert(DOF == 7, "ipm.hip is the Panda's 16-lane interior point (x~ = [y(9), w(7)] fills a DPP row); "
                        "the mobile manipulator builds ipm_wide.hip");

#ifndef MPCC_IPM_MAXIT
#define MPCC_IPM_MAXIT 60
#endif
constexpr int IPM_MAX_IT = MPCC_IPM_MAXIT;  // 60 (oracle); a debug build may cap it
#ifndef MPCC_TOL_MU
#define MPCC_TOL_MU 1e-12  // round 6: 1e-13 -> 1e-12, the oracle's (solve_struct_ipm_from)
#endif
#ifndef MPCC_TOL_STEP
#define MPCC_TOL_STEP 3e-9  // round 6: 1e-11 -> 3e-9, the oracle's
#endif
constexpr double IPM_TOL_MU = MPCC_TOL_MU, IPM_TOL_P = 1e-11, IPM_TOL_STEP = MPCC_TOL_STEP;
constexpr double IPM_TOL_FB = 1e-9;  // P2: a converged iterate is accepted when the Riccati factor breaks down
constexpr double IPM_DIV = 1e6;      // P3: mu > IPM_DIV * mu_0 -> primal infeasible (divergent multipliers)
constexpr double IPM_S0 = 0.02, IPM_L0 = 0.002;  // scaled start point (oracle: solve_struct_ipm)
#ifdef MPCC_DBG_IPM_STOP  // debug builds (tools/tail_ws_diff.py): stop every QP after that many iterations, no restart
constexpr int IPM_MAX_IT_SCALED = MPCC_DBG_IPM_STOP, IPM_ATTEMPTS = 1;
#else
constexpr int IPM_MAX_IT_SCALED = 24, IPM_ATTEMPTS = 2;  // the oracle's (round 6: 30 -> 24)
#endif
constexpr double IPM_TAU = 0.995;    // fraction-to-boundary floor: tau = max(IPM_TAU, 1 - sqrt(mu))
typedef __attribute__((address_space(1))) double gdouble;  // global-memory double (global_* loads/stores)
constexpr int IPW = 4;               // instances per wavefront (16 lanes each)

// workspace fields, ws[(b*(N+1) + k)*IS + field*16 + lane].  Ordered so that what each light sweep reads is
// one run of fields from WF_SL: predictor forward [0, LF_PRED), corrector forward [0, LF_CFWD), corrector
// backward [0, LF_CBWD) (the LDS ring of those sweeps copies whole runs, see glds_stage).
enum : int {
    WF_SL = 0, WF_LL, WF_SU, WF_LU,               // slack / multiplier of the lower and upper slot of row t
    WF_ZX, WF_ZV,                                 // iterate: lane c -> x~_c (y, w); lane j < 8 -> v_j; with <= 4
                                                  // poly rows (PACKP) lanes 8 + p / 12 + p hold s / lambda of poly
                                                  // slot p, and WF_SP / WF_LP are not used
    WF_KR,                                        // 8 fields: K row halves, field m: lane i -> K[i][m], lane 8+i -> K[i][8+m]
    WF_GVK = WF_KR + 8,                           // lanes 0..7: objective gradient (H z + h)_v; lanes 8+i: kff_i
    WF_AX, WF_AV,                                 // predictor step (x~ on all lanes, v on lanes 0..7)
    WF_GX,                                        // objective gradient (H z + h)_x~
    WF_FI,                                        // 4 fields: F^-1 row halves, field m: lane i -> Fi[i][m], lane 8+i -> Fi[i][4+m]
    WF_SP = WF_FI + 4, WF_LP,                     // slack / multiplier of poly slot t (more than 4 poly rows)
    WF_PZ, WF_PA, WF_PD,                          // wide-poly variants (PCACHE): lane p -> c_p^T z, c_p^T dza, c_p^T dz
                                                  // of poly row p, each formed once per iteration (poly_cz)
    WF_DX, WF_DV,                                 // corrector step (same layout as the predictor step)
    NWF
};
constexpr int LF_PRED = WF_GVK + 1, LF_CFWD = WF_AV + 1, LF_CBWD = WF_FI + 4;
static_assert(NWF * 16 <= IS, "IPM workspace must fit the per-stage IS allocation");

// per-instance LDS block (doubles): U and K of the current stage, [i*16 + c]
constexpr int L_U = 0, L_K = 128;
constexpr int GRP_LDS = 256 + 16;  // 16 mod 32 doubles: the two instances of a half-wave start 32 banks apart
#ifndef MPCC_P_LDS
#define MPCC_P_LDS 0  // 1: the factorization's P update moves Hb, U and P through LDS instead of permlane butterflies
#endif
constexpr int P_LDS_BASE = 1152;  // doubles from the wave's LDS base: past the groups' U/K areas (IPW * GRP_LDS)

// LDS ring of the light sweeps (NPM <= 2): LRING slots, each holding one stage of the 4 instances of the
// wave: the 4-line bound block of the QP record, then the sweep's workspace fields.  One global_load_lds
// (16 B per lane) fills 2 lines of each instance, so a slot is LG(nf) KiB; the ring aliases U / K of the
// factorization sweep (the phases never overlap).
constexpr int LRING = 3;                              // stages s(i), s(i+1), s(i+2): two in flight
constexpr int QLINES = 4;                             // QS_YLB .. QS_YLB + 63: bounds, NPOLY, 2 poly rows
__host__ __device__ constexpr int LG(int nf, int ql = QLINES) { return (ql + nf + 1) / 2; }
static_assert(QS_POLY + 2 * 15 <= QS_YLB + 16 * QLINES, "bound block of <= 2 poly rows in QLINES lines");
// The wide-poly variants (NPM >= 9, MPCC_WIDE_RING): a 2-slot ring (one stage in flight) of a 14-line
// bound block (11 poly rows) and the fields up to the unpacked poly slot state; 19 KiB per slot, so 4 waves
// of 38 KiB fit a CU's 160 KiB.
#ifndef MPCC_GRAM_MFMA
#define MPCC_GRAM_MFMA 1
#endif
#ifndef MPCC_PIN
#define MPCC_PIN 0  // 1: settle the prefetched stage before the late stores: 3.43 ms against 3.31 (r03ae_ab_pin.log)
#endif
#ifndef MPCC_KR_EARLY
#define MPCC_KR_EARLY 1
#endif
#ifndef MPCC_PCN
#define MPCC_PCN 0  // 1: cached c_p^T (z, dza, dz) in spare lanes for 1 or 2 poly rows: 1% slower (profiles/r03w_ab_pcn.log)
#endif
#ifndef MPCC_WIDE_RING
#define MPCC_WIDE_RING 1
#endif
#ifndef MPCC_SLOT_SELECT
#define MPCC_SLOT_SELECT 0  // 1: the slot algebra without divergent branches (selects): 0.4% slower at configs[1] (r05g A/B)
#endif
#ifndef MPCC_ROLL_RING
#define MPCC_ROLL_RING 1  // the start-point rollout through a register ring of record-only loads (sweep_ring)
#endif
#ifndef MPCC_WIDE_TAIL
#define MPCC_WIDE_TAIL 1  // tail mode for the wide-poly variants (ipm_tail.h, round 5)
#endif
#ifndef MPCC_RING_KIB
#define MPCC_RING_KIB 39  // LDS ring of the narrow light sweeps per wave; each sweep keeps RING_KIB / LG(run) slots
#endif
constexpr int RING_KIB = MPCC_RING_KIB;
static_assert(RING_KIB >= LRING * LG(LF_CBWD) && RING_KIB <= 40, "3 slots of the longest run; 4 waves inside 160 KiB");
constexpr int LRING_W = 2, QLINES_W = 14;
static_assert(QS_POLY + NPC * 15 <= QS_YLB + 16 * QLINES_W, "bound block of all poly rows in QLINES_W lines");
__host__ __device__ constexpr bool use_ring(int npm) { return npm <= 2 || (MPCC_WIDE_RING && npm >= 9); }
__host__ __device__ constexpr int ring_q(int npm) { return npm <= 2 ? QLINES : QLINES_W; }
__host__ __device__ constexpr int ring_d(int npm) { return npm <= 2 ? LRING : LRING_W; }
static_assert(LF_CBWD + 1 <= NWF, "the odd last line of a ring slot reads one field past the run");

// doubles of LDS per k_sqp wave
__host__ __device__ constexpr int ipm_wave_lds(int npmax) {
    const int uk = IPW * GRP_LDS;
    const int ring = (npmax <= 2)     ? RING_KIB * 128
                     : use_ring(npmax) ? LRING_W * LG(WF_PD, QLINES_W) * 128
                                       : 0;
    return ring > uk ? ring : uk;
}
static_assert(P_LDS_BASE >= IPW * GRP_LDS, "P exchange past the groups' U/K areas");
static_assert(P_LDS_BASE + 64 * 28 <= ipm_wave_lds(0) && P_LDS_BASE + 64 * 28 <= ipm_wave_lds(11),
              "P exchange inside the wave's LDS");
size_t ipm_lds_bytes(int /*N*/, int npmax) {
    const size_t uk = (size_t)IPW * GRP_LDS * sizeof(double);
    const size_t ring = (npmax <= 2)          ? (size_t)RING_KIB * 1024
                        : use_ring(npmax)       ? (size_t)LRING_W * LG(WF_PD, QLINES_W) * 1024  // longest wide run: 26 fields
                                                : 0;
    return ring > uk ? ring : uk;
}

#ifdef MPCC_IPM_PROF
// cycle accounting per k_ipm section (profiling build only, see _build.py / tools/ipm_prof.py)
__device__ unsigned long long g_ipm_prof[16];
// per-wave start / end of the last k_sqp launch (s_memrealtime, 100 MHz), indexed by workgroup (one wave each),
// and the IPM iterations of all QPs of each instance (tools/wave_times.py)
constexpr int PROF_WAVES = 1 << 16;
__device__ unsigned long long g_wave_t[2 * PROF_WAVES];
__device__ int g_inst_its[4 * PROF_WAVES];
__device__ unsigned long long g_tail_prof[16];  // tail mode: factor A, B, C, D, predictor fwd, corrector bwd, fwd; iterations; B sub-sections
__device__ unsigned long long g_solo_prof[8];   // solo waves of k_sqp: cycles in setqp, QP solve, trial, accept, step; waves, SQP iterations
#define TMARK(i) do { const long long t_ = clock64(); tprof[i] += t_ - tprof_t; tprof_t = t_; } while (0)
#define PMARK(i) do { const long long t_ = clock64(); prof_acc[i] += t_ - prof_t; prof_t = t_; } while (0)
#else
#define TMARK(i) do { } while (0)
#define PMARK(i) do { } while (0)
#endif

namespace {

using namespace dpp;

// One wavefront per workgroup: cross-lane LDS hand-offs only need this wave's LDS operations retired
// and a compiler barrier; __syncthreads() would also drain outstanding global loads (vmcnt(0)).
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// global_load_lds_dwordx4: 16 bytes per lane from src + OFF into LDS at lds_dst + 16 * lane (lds_dst
// wave-uniform, through M0, which the statement saves and restores).  The immediate offset applies to the
// LDS address as well, so M0 = lds_dst - OFF.  hipcc does not count asm memory operations, so completion
// is waited for explicitly (s_waitcnt vmcnt).
template <int OFF>
__device__ __forceinline__ void glds16(const void* src, unsigned lds_dst) {
    lds_dst -= OFF;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off offset:%3\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_dst), "n"(OFF) : "memory");
}
// one ring slot: instruction i copies 2 lines of each instance (i < QL2: the QP record's bound block at qk,
// then the workspace fields at wk), immediate offsets from the two per-lane bases
#ifndef MPCC_GLDS_ONE
#define MPCC_GLDS_ONE 1
#endif
#if MPCC_GLDS_ONE
// The whole slot in ONE statement: M0 saved once, then stepped between copies (copy i of a run writes LDS at
// dst + 1024 i through M0 = dst + 1024 i - OFF_i, OFF_i = 256 x its index in the run: +768 per copy, +256 QL2 + 768
// from the record's run to the workspace's).  A statement per copy (glds16) spent 6 instructions on each (M0 saved,
// set from a fresh SGPR sum, nop, load, M0 restored); at one wave per SIMD every instruction is an issue slot of the
// light sweeps.  s_add_u32 sets SCC (clobbered); the nop after each M0 write is the LDS-DMA M0 hazard.
#define GL_ADD(n) "s_add_u32 m0, m0, " #n "\n\ts_nop 0\n\t"
#define GL_Q(o) "global_load_lds_dwordx4 %1, off offset:" #o "\n\t"
#define GL_W(o) "global_load_lds_dwordx4 %2, off offset:" #o "\n\t"
#define GL_WN(o) GL_ADD(768) GL_W(o)
#define GL_QN(o) GL_ADD(768) GL_Q(o)
#define GL_W7 GL_WN(256) GL_WN(512) GL_WN(768) GL_WN(1024) GL_WN(1280) GL_WN(1536) GL_WN(1792)
#define GL_W8 GL_W7 GL_WN(2048)
#define GL_W9 GL_W8 GL_WN(2304)
#define GL_W10 GL_W9 GL_WN(2560)
#define GL_W11 GL_W10 GL_WN(2816)
#define GL_W12 GL_W11 GL_WN(3072)
#define GL_HEAD "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t" GL_Q(0)
#define GL_Q2 GL_HEAD GL_QN(256) GL_ADD(1280) GL_W(0)
#define GL_Q7 GL_HEAD GL_QN(256) GL_QN(512) GL_QN(768) GL_QN(1024) GL_QN(1280) GL_QN(1536) GL_ADD(2560) GL_W(0)
#define GL_TAIL "s_mov_b32 m0, %0"
#define GL_STMT(text) asm volatile(text : "=&s"(keep) : "v"(qk), "v"(wk), "s"(dst) : "memory", "scc")
template <int G, int QL2>
__device__ __forceinline__ void glds_slot(const char* qk, const char* wk, unsigned dst) {
    unsigned keep;
    if constexpr (QL2 == 2 && G == 10) GL_STMT(GL_Q2 GL_W7 GL_TAIL);
    else if constexpr (QL2 == 2 && G == 11) GL_STMT(GL_Q2 GL_W8 GL_TAIL);
    else if constexpr (QL2 == 2 && G == 13) GL_STMT(GL_Q2 GL_W10 GL_TAIL);
    else if constexpr (QL2 == 7 && G == 15) GL_STMT(GL_Q7 GL_W7 GL_TAIL);
    else if constexpr (QL2 == 7 && G == 16) GL_STMT(GL_Q7 GL_W8 GL_TAIL);
    else if constexpr (QL2 == 7 && G == 17) GL_STMT(GL_Q7 GL_W9 GL_TAIL);
    else if constexpr (QL2 == 7 && G == 18) GL_STMT(GL_Q7 GL_W10 GL_TAIL);
    else if constexpr (QL2 == 7 && G == 19) GL_STMT(GL_Q7 GL_W11 GL_TAIL);
    else if constexpr (QL2 == 7 && G == 20) GL_STMT(GL_Q7 GL_W12 GL_TAIL);
    else static_assert(G < 0, "glds_slot: no statement for this slot shape");
}
#undef GL_STMT
#endif
template <int I, int G, int QL2>
struct GldsBatch {
    __device__ __forceinline__ static void run(const char* qk, const char* wk, unsigned dst) {
        if constexpr (I < G) {
            if constexpr (I < QL2) glds16<I * 256>(qk, dst + I * 1024u);
            else glds16<(I - QL2) * 256>(wk, dst + I * 1024u);
            GldsBatch<I + 1, G, QL2>::run(qk, wk, dst);
        }
    }
};

// ---- slot algebra (oracle solve_struct_ipm), slot: sgn*(c^T z) <= sgn*bnd ----------------------
struct SlotStep {
    double ds, dl;
};
__device__ __forceinline__ double slot_rp(double sgn, double cz, double bnd, double s) { return sgn * cz - sgn * bnd + s; }
// ri = 1/s is formed once per slot and sweep (W = l/s, rc/s become products)
__device__ __forceinline__ SlotStep slot_recover(double ri, double l, double rp, double cd, double rc) {
    const double W = l * ri;
    return {-rp - cd, fma(W, cd + rp, -(rc * ri))};
}
__device__ __forceinline__ double slot_coef(double ri, double l, double rp, double rc) { return l + (l * ri) * rp - rc * ri; }
// Fraction-to-boundary ratio test min(a, -s/ds, -l/dl) without a division per slot: the running
// minimum is kept as a ratio num/den (den > 0) and candidates are compared by cross-multiplication;
// value() divides once.  It is the oracle's min over the same quotients (max_step, solve_struct_ipm),
// exact unless two candidates tie to within rounding of the products.
struct MinRatio {
    double num, den;
    __device__ __forceinline__ explicit MinRatio(double cap) : num(cap), den(1.0) {}
    __device__ __forceinline__ void add(double n, double dneg) {  // candidate n / (-dneg), dneg < 0
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
// 1/x for x > 0: v_rcp_f64 refined by two Newton steps (vs the ~10-instruction IEEE division sequence)
__device__ __forceinline__ double rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    return fma(fma(-x, r, 1.0), r, r);
}
// mu(alpha) sums of one slot, S0 += s l, S1 += s dl + l ds, S2 += ds dl, with the fused forms written out: the
// contraction the compiler would choose depends on whether s l is also used elsewhere, and tail mode (ipm_tail.h)
// accumulates the same terms in another function, which must come out bitwise the same
__device__ __forceinline__ void mu_acc(double& S0, double& S1, double& S2, double s, double l, double ds, double dl) {
    S0 = fma(s, l, S0);
    S1 = S1 + fma(s, dl, l * ds);
    S2 = fma(ds, dl, S2);
}
// a b + c d with the product a b fused: every two-product form of the recursions and the dynamics is written out for
// the reason of mu_acc (which product the compiler fuses depends on the surrounding code, and tail mode evaluates the
// same expressions in another function)
__device__ __forceinline__ double fma2(double a, double b, double c, double d) { return fma(a, b, c * d); }
// instance of 16-lane group slot `slot` of the launch: k_sqp with solo waves maps slots through d.order (k_order),
// every other launch is the identity; an empty slot is c.Bn (not valid)
__device__ __forceinline__ int inst_of(const DevConst& c, const DevBuffers& d, int slot) {
    if (!c.solo) return slot;
    const int v = d.order[slot];
    return v < 0 ? c.Bn : v;
}
// corrector step of a slot given the iterate (cz), the predictor step (ca) and the corrector step (cd)
__device__ __forceinline__ SlotStep slot_corr(double sgn, double bnd, double cz, double ca, double cd, double s, double l,
                                              double smu, double* rp_out) {
    const double ri = rcp(s);
    const double rp = slot_rp(sgn, cz, bnd, s);
    const SlotStep pa = slot_recover(ri, l, rp, sgn * ca, s * l);
    const double rc = fma(s, l, pa.ds * pa.dl) - smu;
    *rp_out = rp;
    return slot_recover(ri, l, rp, sgn * cd, rc);
}

// 1/sqrt(x) for x > 0: v_rsq_f64 refined by two Newton steps, r <- r (1.5 - x/2 r^2).  On the Cholesky's
// pivot chain this is 7 dependent instructions where sqrt (the ~12-instruction IEEE sequence) and then
// rcp were 17; the solves only use the reciprocal pivots.
__device__ __forceinline__ double rsqrt_pos(double x) {
    const double h = 0.5 * x;
    double r = __builtin_amdgcn_rsq(x);
    r = r * fma(-h * r, r, 1.5);
    return r * fma(-h * r, r, 1.5);
}

// Cholesky of the 8x8 stage F (lower triangle, packed row-major in L on entry); reciprocal pivots in dinv
// (the diagonal of L itself is not formed: fwd8 / bwd8 only read dinv and the strict lower triangle)
__device__ __forceinline__ bool chol8(double* L, double* dinv) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int jj = j * (j + 1) / 2;
        double d = L[jj + j];
#pragma unroll
        for (int m = 0; m < j; m++) d -= L[jj + m] * L[jj + m];
        ok = ok && (d > 0);
        const double inv = rsqrt_pos(d);
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

typedef double d4 __attribute__((ext_vector_type(4)));

// ---- 4x4 transpose of the wave's 16-lane groups: afterwards lane (g, c) holds in x[j][r] what lane (j, c) held
//      in x[g][r].  Two butterflies, on the group bit 1 (v_permlane32_swap: the first operand's upper 32
//      lanes <-> the second's lower 32) and the group bit 0 (v_permlane16_swap: the first operand's odd rows <->
//      the second's even rows), each on both dwords of a double.  Needs the whole wave active.
__device__ __forceinline__ void swap_rows32(double& a, double& b) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(a), y = (unsigned long long)__double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)y, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
    a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ void swap_rows16(double& a, double& b) {
    const unsigned long long x = (unsigned long long)__double_as_longlong(a), y = (unsigned long long)__double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)y, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
    a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
template <int R>
__device__ __forceinline__ void group_transpose(double (&x)[4][R]) {
#pragma unroll
    for (int r = 0; r < R; r++) {
        swap_rows32(x[0][r], x[2][r]);
        swap_rows32(x[1][r], x[3][r]);
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        swap_rows16(x[0][r], x[1][r]);
        swap_rows16(x[2][r], x[3][r]);
    }
}

// per-stage inputs of one lane, loaded one stage ahead of their use
template <int NPE>
struct StageIn {
    double lb, ub, np;            // bounds of row t, live poly rows
    double pa[NPE], pb[NPE];      // poly rows p: a_p[t], bv_p[t] (t < 7)
    double pub;                   // upper bound of poly row t (t < npmax)
    double sL, lL, sU, lU, sP, lP, zx, zv;
    double pz, pca, pcd;          // PCACHE: c_p^T z, c_p^T dza, c_p^T dz of poly row t (WF_PZ, WF_PA, WF_PD)
    double x0, x1, x2, x3;        // sweep-specific pairs (dz, dza, g0)
    double m[12];                 // sweep-specific: Q row + q, R, r | K row halves + kff | K column + F^-1 half
};

// Stage sweep i = 0..N in the order s(i) (forward or backward) with the next stage prefetched into the
// other of two buffers.  Unrolled by two so that the buffers swap roles instead of being copied (a copy
// of an in-flight buffer waits for its loads), and every load is issued unconditionally (the last one
// re-reads stage s(N)): loads behind branches make the waitcnt pass drain all loads at the join.
template <bool PINGPONG, class In, class LoadF, class BodyF>
__device__ __forceinline__ void sweep(int N, bool backward, In& b0, In& b1, LoadF load, BodyF body) {
    auto s = [&](int i) { return backward ? N - i : i; };
    load(s(0), b0);
    if constexpr (!PINGPONG) {  // wide-poly variants: the unrolled factor body doubles their spills
        for (int i = 0; i <= N; i++) {
            load(s(i + 1 <= N ? i + 1 : N), b1);
            body(s(i), b0);
            b0 = b1;
        }
        return;
    }
    for (int i = 0; i <= N; i += 2) {
        load(s(i + 1 <= N ? i + 1 : N), b1);
        body(s(i), b0, b1);  // the body may settle the prefetched buffer (pin) before its late stores
        if (i + 1 > N) break;
        load(s(i + 2 <= N ? i + 2 : N), b0);
        body(s(i + 1), b1, b0);
    }
}

// The same sweep without a prefetch buffer: each stage's loads are issued at the top of its body (the
// factorization sweep of the wide-poly variants, whose body already holds most of the registers).
template <class In, class LoadF, class BodyF>
__device__ __forceinline__ void sweep_noprefetch(int N, bool backward, In& b0, LoadF load, BodyF body) {
    for (int i = 0; i <= N; i++) {
        const int k = backward ? N - i : i;
        load(k, b0);
        body(k, b0);
    }
}

// Stage sweep with a ring of D stage buffers: stage s(i + D - 1) is loaded while stage s(i) is processed,
// so D - 1 stages of loads are in flight.  Loads are unconditional (the stages past the end re-read
// s(N)); the ring index is a constant after unrolling, so the buffers stay in registers.
// D = 2 since the stage addresses stopped spilling: same box, configs[1], k_sqp
// 3.83 ms at D = 2, 3.88 ms at D = 3, 4.14 ms at D = 4 (tools/bench_variants.sh).
// Sweeps of the wide-poly variants (NPM >= 9), whose stage buffers hold 11 poly rows: register pressure
// costs them more than load latency.  Same box, reference default rows (bench --config 1-all-rows), k_sqp<11>:
// light sweeps with the copy-based prefetch 15.72 ms, without it 14.57 ms (the default); the factorization
// sweep with that prefetch 16.63 ms (it stays without).  profiles/r02e_c1all_*.json
#ifndef MPCC_WIDE_FACTOR_PF
#define MPCC_WIDE_FACTOR_PF 0
#endif
#ifndef MPCC_WIDE_LIGHT_NOPF
#define MPCC_WIDE_LIGHT_NOPF 1
#endif
#ifndef MPCC_LIGHT_DEPTH
#define MPCC_LIGHT_DEPTH 2
#endif
#ifndef MPCC_LIGHT_UNROLL  // unroll factor of the LDS-ring light sweeps (A/B switch)
#define MPCC_LIGHT_UNROLL 1
#endif
template <int D, class In, class LoadF, class BodyF>
__device__ __forceinline__ void sweep_ring(int N, bool backward, In (&b)[D], LoadF load, BodyF body) {
    auto s = [&](int i) { return backward ? N - i : i; };
    auto cl = [&](int i) { return s(i <= N ? i : N); };
#pragma unroll
    for (int j = 0; j < D - 1; j++) load(cl(j), b[j]);
    for (int i = 0; i <= N; i += D) {
#pragma unroll
        for (int j = 0; j < D; j++) {
            load(cl(i + j + D - 1), b[(j + D - 1) % D]);
            body(s(i + j), b[j]);
            if (i + j + 1 > N) return;
        }
    }
}

// Workspace field indices of the NPM variant (ipm_group and tail mode).  The wide-poly variants (NPM >= 9) order
// their fields so that each light sweep's LDS-ring image is the shortest run from field 0: the poly slot state and
// c_p^T z right after the iterate, then K and kff (predictor forward), the predictor step and c_p^T dza (corrector
// forward), the gradient and F^-1 (corrector backward); c_p^T dz and the corrector step are read by the
// factorization only.  The narrow variants keep the enum order (their poly slot state is packed into WF_ZV).
template <int NPM>
struct WsF {
    static constexpr bool WLAY = NPM >= 9;
    static constexpr int SL = WF_SL, LL = WF_LL, SU = WF_SU, LU = WF_LU, ZX = WF_ZX, ZV = WF_ZV;
    static constexpr int SP = WLAY ? 6 : WF_SP, LP = WLAY ? 7 : WF_LP, PZ = WLAY ? 8 : WF_PZ;
    static constexpr int KR = WLAY ? 9 : WF_KR, GVK = KR + 8, AX = GVK + 1, AV = AX + 1;
    static constexpr int PA = WLAY ? AV + 1 : WF_PA, GX = WLAY ? PA + 1 : WF_GX, FI = GX + 1;
    static constexpr int PD = WLAY ? FI + 4 : WF_PD, DX = WF_DX, DV = WF_DV;
    static_assert(WLAY || (GVK == WF_GVK && AX == WF_AX && AV == WF_AV && FI == WF_FI), "narrow layout = enum");
    static_assert(!WLAY || (PD == WF_PD && PD + 1 == DX), "wide layout: a permutation of the enum's fields");
    // poly slot state packed into the upper lanes of the v field (<= 4 poly rows); c_p^T z, dza, dz cached in the
    // workspace (wide-poly variants)
    static constexpr bool PACKP = NPM <= 4, PCACHE = NPM >= 9;
};

#include "ipm_tail.h"

}  // namespace

// The QP solve of the 4 instances of this wavefront (16 lanes each); instances whose SQP is inactive
// idle through it.  Writes the step (d.step), QP status and IPM iteration count (d.sqi).
template <int NPM>
__device__ __forceinline__ bool ipm_group(const DevConst& c, const DevBuffers& d, double* smem) {
    // Workspace field indices of this variant (WsF)
    using L = WsF<NPM>;
    constexpr int F_SL = L::SL, F_LL = L::LL, F_SU = L::SU, F_LU = L::LU, F_ZX = L::ZX, F_ZV = L::ZV;
    constexpr int F_SP = L::SP, F_LP = L::LP, F_PZ = L::PZ;
    constexpr int F_KR = L::KR, F_GVK = L::GVK, F_AX = L::AX, F_AV = L::AV;
    constexpr int F_PA = L::PA, F_GX = L::GX, F_FI = L::FI;
    constexpr int F_PD = L::PD, F_DX = L::DX, F_DV = L::DV;
    constexpr int NPE = NPM > 0 ? NPM : 1;
    using In = StageIn<NPE>;
    const int lane = threadIdx.x;
    const int grp = lane >> 4;
    const int t = lane & 15;
    const int b = inst_of(c, d, blockIdx.x * IPW + grp);
    const int N = c.N;
    const int NS = N + 1;
    double* const S = smem + grp * GRP_LDS;
#ifdef MPCC_IPM_PROF
    long long prof_acc[16] = {0};
    long long prof_t = clock64();
#endif

    const bool valid = b < c.Bn;
    int32_t* si = d.sqi + (size_t)(valid ? b : 0) * SQI;
    bool run = valid && si[SQ_ACTIVE] != 0;
    if (__ballot(run) == 0) return false;

    // QP records and the workspace through global-address-space pointers: their loads and stores compile
    // to global_* instructions, which count only in vmcnt.  Through the generic pointers of DevBuffers they
    // were flat_*, which also count in lgkmcnt, so every LDS wait (lgkmcnt(0), the U/K reads of the factor
    // sweep) drained the in-flight stage prefetch as well.
    const gdouble* QSb = (const gdouble*)(d.qs + (size_t)MPCC_BCHK(c.bchk, valid ? b : 0, c.Bn, BC_INSTANCE) * NS * QS);
    gdouble* WSb = (gdouble*)(d.is + (size_t)(valid ? b : 0) * NS * IS);
    // Stage base addresses pass through an empty asm: the optimizer cannot strength-reduce every
    // (field, stage) address into its own 64-bit induction variable.  It did, ran out of registers,
    // spilled the addresses to scratch, and each scratch reload (s_waitcnt vmcnt(0)) drained the stage
    // prefetch.  Fields are then immediate offsets from one stage pointer.
    gdouble* const WSt = WSb + t;
    auto ws = [&](int k, int f) -> gdouble* {
        gdouble* wk = WSt + (size_t)MPCC_BCHK(c.bchk, k, NS, BC_WS_STAGE) * IS;
        asm("" : "+v"(wk));
        return wk + MPCC_BCHK(c.bchk, f, NWF, BC_WS_FIELD) * 16;
    };
    auto qs_stage = [&](int k) -> const gdouble* {
        const gdouble* qk = QSb + (size_t)MPCC_BCHK(c.bchk, k, NS, BC_QS_STAGE) * QS;
        asm("" : "+v"(qk));
        return qk;
    };

    // ---- model constants of this lane (sparse M, G; selects keep the kernel-argument reads scalar)
    const double m78 = c.M[7 * 9 + 8], m77 = c.M[7 * 10], m88 = c.M[8 * 10];
    const double g77 = c.G[7 * 8 + 7], g87 = c.G[8 * 8 + 7];
    double mt = 0.0, gt = 0.0, Hct = 0.0;
    const double HcB = -2. * c.p.qp_r_ddq;
    double mdiag[9], gdiag[7];
#pragma unroll
    for (int a = 0; a < 9; a++) {
        mdiag[a] = c.M[a * 10];
        if (t == a) mt = mdiag[a];
    }
#pragma unroll
    for (int a = 0; a < 7; a++) {
        gdiag[a] = c.G[a * 9];
        if (t == a || t == 9 + a) {
            gt = (t < 7) ? gdiag[a] : 0.0;
            Hct = c.p.Tu[a] * HcB * c.p.Tu[a];
        }
    }
    if (t == 7) gt = g77;
    const bool rowY = t < 9;
    const int j9 = t - 9;
    constexpr double sgnL = -1.0, sgnU = 1.0;
    // Hb[a][t] (a, t < 9) = base + (A~^T P A~)[a][t] for the sparse A~ (diagonal + the (7, 8) entry); Pc7: lane 8 <- P[a][7]
    auto hb_mp = [&](double v, int a, const double (&Pc)[16], const double (&Pc7)[9]) -> double {
        v = fma(mdiag[a] * mt, Pc[a], v);
        if (t == 8) v = fma(mdiag[a] * m78, Pc7[a], v);
        if (a == 8) v = fma(m78 * mt, Pc[7], v);
        if (a == 8 && t == 8) v = fma(m78 * m78, Pc7[7], v);
        return v;
    };

    // ---- Hessian checks (osqp_interface.cpp:454-473): stage flags from k_setqp + tridiagonal input blocks
    int fl = 0;
    if (run) {
        for (int k = t; k < NS; k += 16) fl |= (int)QSb[(size_t)k * QS + QS_FLAG];
        if (t < 8) {
            // the input-block diagonals are read 8 stages at a time before the recursion uses them: loaded inside
            // the loop (behind its early exit) they were 20 dependent HBM round trips at the start of every QP
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
            if (g_max((double)((fl >> bit) & 1)) > 0.5) o |= 1 << bit;
        fl = o;
    }
    if (run && (fl & 2)) { if (t == 0) { si[SQ_STATUS] = MPCC_NON_PD_HESSIAN; si[SQ_ACTIVE] = 0; } run = false; }
    if (run && (fl & 1)) { if (t == 0) { si[SQ_STATUS] = MPCC_NAN_HESSIAN; si[SQ_ACTIVE] = 0; } run = false; }
    if (run && (fl & 4)) { if (t == 0) si[SQ_QPSTAT] = MPCC_QP_PrimalInfeasible; run = false; }  // keep old step (Q6)
    const bool entered = run;

    // Poly slot state packed into the upper lanes of the v field (<= 4 poly rows): every sweep then loads
    // 6 workspace lines of slot and iterate state per stage instead of 8.
    constexpr bool PACKP = L::PACKP;
    // Wide-poly variants: c_p^T z, c_p^T dza and c_p^T dz (11 reductions over the row's 16 lanes each) are formed
    // once per iteration where z, dza, dz are made, kept in the workspace (F_PZ, F_PA, F_PD) and read by the
    // other sweeps, which recomputed them from the same stored vectors (the same values: 3 evaluations per stage
    // and iteration instead of 11)
    constexpr bool PCACHE = L::PCACHE;
    // The same for 1 or 2 poly rows at no extra traffic: c_p^T z rides in the free lanes 10 + p of the packed F_ZV,
    // c_p^T dza and c_p^T dz in lanes 8 + p of F_AV and F_DV (whose v occupies lanes 0..7; readers mask them)
    constexpr bool PCN = MPCC_PCN && NPM >= 1 && NPM <= 2;
    constexpr bool PCV = PCACHE || PCN;
    constexpr bool GRAM_MFMA = MPCC_GRAM_MFMA && NPM >= 9;  // poly Gram terms of the factorization on MFMA
    auto zv_pack = [&](double zv, double sP, double lP, double pz) -> double {
        if constexpr (PCN) {
            const double s8 = from_down<8>(sP), l12 = from_down<12>(lP), z10 = from_down<10>(pz);  // whole row active
            return (t < 8) ? zv : ((t < 10) ? s8 : ((t < 12) ? z10 : l12));
        } else if constexpr (PACKP) {
            const double s8 = from_down<8>(sP), l12 = from_down<12>(lP);  // DPP with the whole row active
            return (t < 8) ? zv : ((t < 12) ? s8 : l12);
        } else {
            return zv;
        }
    };
    auto store_slots = [&](int k, double sL, double lL, double sU, double lU, double sP, double lP, double zx,
                           double zv, double pz) {
        *ws(k, F_SL) = sL; *ws(k, F_LL) = lL; *ws(k, F_SU) = sU; *ws(k, F_LU) = lU;
        if constexpr (!PACKP) { *ws(k, F_SP) = sP; *ws(k, F_LP) = lP; }
        *ws(k, F_ZX) = zx;
        *ws(k, F_ZV) = zv_pack(zv, sP, lP, pz);
    };

    // ---- stage loaders: every load unconditional (addresses clamped inside the stage record), the
    //      lane/stage conditions applied as selects afterwards (see sweep())
    auto load_common = [&](int k, In& o) {
        const gdouble* q = qs_stage(k);
        o.lb = q[rowY ? QS_YLB + t : QS_DLB + j9];
        o.ub = q[rowY ? QS_YUB + t : QS_DUB + j9];
        o.np = q[QS_NPOLY];
        const int tp = t < 7 ? t : 0;  // keep the address inside row p (15 p + 7 + t would leave the record)
#pragma unroll
        for (int p = 0; p < NPE; p++) {
            const double a = q[QS_POLY + 15 * p + tp], bv = q[QS_POLY + 15 * p + 7 + tp];
            o.pa[p] = (NPM > 0 && t < 7) ? a : 0.0;
            o.pb[p] = (NPM > 0 && t < 7) ? bv : 0.0;
        }
        const double pu = q[QS_POLY + 15 * (t < NPE ? t : 0) + 14];
        o.pub = (t < NPM) ? pu : INF;
        o.sL = *ws(k, F_SL); o.lL = *ws(k, F_LL); o.sU = *ws(k, F_SU); o.lU = *ws(k, F_LU);
        o.zx = *ws(k, F_ZX);
        if constexpr (PCACHE) { o.pz = *ws(k, F_PZ); o.pca = *ws(k, F_PA); o.pcd = *ws(k, F_PD); }
        const double zraw = *ws(k, F_ZV);
        if constexpr (PACKP) {
            o.sP = from_up<8>(zraw);   // lane p <- lane 8 + p
            o.lP = from_up<12>(zraw);  // lane p <- lane 12 + p
            if constexpr (PCN) o.pz = from_up<10>(zraw);  // lane p <- lane 10 + p
            o.zv = (t < 8) ? zraw : 0.0;
        } else {
            o.sP = *ws(k, F_SP); o.lP = *ws(k, F_LP);
            o.zv = zraw;
        }
    };
    auto load_factor = [&](int k, In& o, bool upd) {
        load_common(k, o);
        const gdouble* q = qs_stage(k);
#pragma unroll
        for (int m = 0; m < 9; m++) {
            const double v = q[QS_Q + t * 9 + m];
            o.m[m] = (t < 9) ? v : 0.0;
        }
        const double qv = q[QS_q + t], rv = q[QS_R + t], rr = q[QS_r + t];
        o.m[9] = (t < 9) ? qv : 0.0;
        o.m[10] = (t < 8 && k < N) ? rv : 0.0;
        o.m[11] = (t < 8 && k < N) ? rr : 0.0;
        const double x0 = *ws(k, F_DX), x1 = *ws(k, F_DV), x2 = *ws(k, F_AX), x3 = *ws(k, F_AV);
        const bool vl = !PCN || t < 8;  // PCN: lanes 8.. of DV / AV carry c_p^T dz / c_p^T dza
        o.x0 = upd ? x0 : 0.0; o.x1 = (upd && vl) ? x1 : 0.0; o.x2 = upd ? x2 : 0.0; o.x3 = (upd && vl) ? x3 : 0.0;
        if constexpr (PCN) { o.pcd = from_up<8>(x1); o.pca = from_up<8>(x3); }  // lane p <- lane 8 + p
    };
    auto load_fwd = [&](int k, In& o, bool corr) {
        load_common(k, o);
#pragma unroll
        for (int m = 0; m < 8; m++) o.m[m] = *ws(k, F_KR + m);  // zero at k = N (factor sweep)
        o.m[8] = from_up<8>(*ws(k, F_GVK));  // lane i <- kff_i (lanes 8..15: 0)
        if (corr) {  // corr: constant
            o.x0 = *ws(k, F_AX);
            const double av = *ws(k, F_AV);
            o.x1 = (!PCN || t < 8) ? av : 0.0;
            if constexpr (PCN) o.pca = from_up<8>(av);
        } else {
            o.x0 = o.x1 = 0.0;
        }
    };
    auto load_bwd = [&](int k, In& o) {
        load_common(k, o);
        o.x0 = *ws(k, F_AX); o.x2 = *ws(k, F_GX);
        const double av = *ws(k, F_AV);
        o.x1 = (!PCN || t < 8) ? av : 0.0;
        if constexpr (PCN) o.pca = from_up<8>(av);
        const double gvk = *ws(k, F_GVK);
        o.x3 = (t < 8) ? gvk : 0.0;
#pragma unroll
        for (int m = 0; m < 8; m++) o.m[m] = *ws(k, F_KR + m);  // zero at k = N (factor sweep)
#pragma unroll
        for (int m = 0; m < 4; m++) o.m[8 + m] = *ws(k, F_FI + m);
    };

    // ---- the light sweeps of NPM <= 2 (and of NPM >= 9 with MPCC_WIDE_RING: 2 slots, 14 record lines from
    //      QS_YLB - 16, fields 0..F_LP) read their stages from an LDS ring filled by global_load_lds:
    //      LRING - 1 = 2 stages in flight at no register cost (a register ring that deep spilled, and
    //      every scratch reload waited for all loads in flight).  Slot image of one instance: line j at
    //      (j >> 1) * 128 + (j & 1) * 16 doubles from the instance's base (grp * 32), lines 0..3 = the QP
    //      record's bound block (QS_YLB ..), lines 4.. = workspace fields 0.. .  Lane (grp, t) copies chunk
    //      t & 7 of lines 2i + (t >> 3) of its own instance, so groups that are not running load nothing
    //      and read nothing.
    const unsigned lds_base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)smem;
    auto img_at = [](int j) { return (j >> 1) * 128 + (j & 1) * 16; };
    constexpr int QL = ring_q(NPM), RD = ring_d(NPM);
    // first record line of the slot image: the bound block; the wide ring starts one line earlier so that its
    // 14 lines end with the stage record (a line past it would leave the buffer at the last stage)
    constexpr int QB = (NPM <= 2) ? QS_YLB : QS_YLB - 16;
    static_assert(QB + 16 * QL <= QS, "ring image inside the stage record");
    auto qoff = [&](int r) { const int x = r - QB; return img_at(x >> 4) + (x & 15); };
    const int o_lb = qoff(rowY ? QS_YLB + t : QS_DLB + j9), o_ub = qoff(rowY ? QS_YUB + t : QS_DUB + j9);
    const int o_np = qoff(QS_NPOLY), o_pub = qoff(QS_POLY + 15 * (t < NPE ? t : 0) + 14);
    int o_pa[NPE], o_pb[NPE];  // a_p[t], bv_p[t] (t < 7); NPM <= 2 only
#pragma unroll
    for (int p = 0; p < (NPM <= 2 ? NPE : 0); p++) {
        o_pa[p] = qoff(QS_POLY + 15 * p + (t < 7 ? t : 0));
        o_pb[p] = qoff(QS_POLY + 15 * p + 7 + (t < 7 ? t : 0));
    }
    // fields in a slot image: the sweep's run; the wide ring also needs the unpacked poly slot state
    // fields in a slot image: the sweep's run (the wide layout's runs: through kff, through c_p^T dza, through F^-1)
    auto ring_nf = [](auto nfc) {
        constexpr int nf = decltype(nfc)::value;
        if constexpr (NPM <= 2) return nf;
        else return nf == LF_PRED ? F_GVK + 1 : (nf == LF_CFWD ? F_PA + 1 : F_FI + 4);
    };
    // slots of a sweep's ring: as many as the wave's ring LDS holds (narrow), RD (wide)
    auto ring_depth = [](auto nfc) {
        if constexpr (NPM <= 2) return RING_KIB / LG(decltype(nfc)::value);
        else return ring_d(NPM);
    };
    auto glds_stage = [&](int k, int slot, auto nfc) {
        constexpr int G = LG(ring_nf(nfc), QL);
        // the image's last record line and workspace line stay inside the stage (static), the stage inside the
        // instance and the slot inside the ring (checked build)
        static_assert(QB + 16 * 2 * (G > QL / 2 ? QL / 2 : G) <= QS, "ring record lines inside the stage record");
        static_assert(16 * 2 * (G - QL / 2) <= IS, "ring workspace lines inside the stage workspace");
        k = MPCC_BCHK(c.bchk, k, NS, BC_RING);
        slot = MPCC_BCHK(c.bchk, slot, ring_depth(nfc), BC_RING);
        const char* qk = (const char*)(QSb + (size_t)k * QS + QB) + (t & 7) * 16 + (t >> 3) * 128;
        const char* wk = (const char*)(WSb + (size_t)k * IS) + (t & 7) * 16 + (t >> 3) * 128;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of the slot's previous stage retired
        const unsigned dst = lds_base + (unsigned)(slot * G) * 1024u;
#if MPCC_GLDS_ONE
        glds_slot<G, QL / 2>(qk, wk, dst);
#else
        GldsBatch<0, G, QL / 2>::run(qk, wk, dst);
#endif
    };
    auto lds_common = [&](const double* im, In& o) {
        o.lb = im[o_lb];
        o.ub = im[o_ub];
        o.np = im[o_np];
#pragma unroll
        for (int p = 0; p < NPE; p++) {
            // the wide ring computes the offsets per use (22 offsets held through the solve spilled)
            const int opa = (NPM <= 2) ? o_pa[p] : qoff(QS_POLY + 15 * p + (t < 7 ? t : 0));
            const int opb = (NPM <= 2) ? o_pb[p] : qoff(QS_POLY + 15 * p + 7 + (t < 7 ? t : 0));
            const double a = im[opa], bv = im[opb];
            o.pa[p] = (NPM > 0 && t < 7) ? a : 0.0;
            o.pb[p] = (NPM > 0 && t < 7) ? bv : 0.0;
        }
        const double pu = im[o_pub];
        o.pub = (t < NPM) ? pu : INF;
        auto f = [&](int field) { return im[img_at(QL + field) + t]; };
        o.sL = f(F_SL); o.lL = f(F_LL); o.sU = f(F_SU); o.lU = f(F_LU);
        o.zx = f(F_ZX);
        if constexpr (PCACHE) { o.pz = f(F_PZ); o.pca = f(F_PA); o.pcd = f(F_PD); }
        const double zraw = f(F_ZV);
        if constexpr (PACKP) {
            o.sP = from_up<8>(zraw);   // lane p <- lane 8 + p
            o.lP = from_up<12>(zraw);  // lane p <- lane 12 + p
            if constexpr (PCN) o.pz = from_up<10>(zraw);
            o.zv = (t < 8) ? zraw : 0.0;
        } else {
            o.sP = f(F_SP); o.lP = f(F_LP);
            o.zv = zraw;
        }
    };
    auto fld = [&](const double* im, int field) { return im[img_at(QL + field) + t]; };
    auto lds_fwd = [&](const double* im, In& o, bool corr) {
        lds_common(im, o);
#pragma unroll
        for (int m = 0; m < 8; m++) o.m[m] = fld(im, F_KR + m);
        o.m[8] = from_up<8>(fld(im, F_GVK));
        if (corr) {
            o.x0 = fld(im, F_AX);
            const double av = fld(im, F_AV);
            o.x1 = (!PCN || t < 8) ? av : 0.0;
            if constexpr (PCN) o.pca = from_up<8>(av);
        } else {
            o.x0 = o.x1 = 0.0;
        }
    };
    auto lds_bwd = [&](const double* im, In& o) {
        lds_common(im, o);
        o.x0 = fld(im, F_AX); o.x2 = fld(im, F_GX);
        const double av = fld(im, F_AV);
        o.x1 = (!PCN || t < 8) ? av : 0.0;
        if constexpr (PCN) o.pca = from_up<8>(av);
        const double gvk = fld(im, F_GVK);
        o.x3 = (t < 8) ? gvk : 0.0;
#pragma unroll
        for (int m = 0; m < 8; m++) o.m[m] = fld(im, F_KR + m);
#pragma unroll
        for (int m = 0; m < 4; m++) o.m[8 + m] = fld(im, F_FI + m);
    };
    // stage sweep over the ring: stage s(i + 2) is issued while s(i) is read and processed; every issue
    // is unconditional (the stages past the end re-read s(N)), so the wait count is fixed: after issuing
    // s(i + 2), stage s(i) has landed once at most 2 G memory operations are outstanding (the bodies'
    // stores only make that wait stricter).  The extra loads are drained before the ring's LDS is reused.
    auto lds_sweep = [&](bool backward, auto nfc, auto read, auto body) {
        constexpr int G = LG(ring_nf(nfc), QL);
        constexpr int RD = ring_depth(nfc);
        auto s = [&](int i) { return backward ? N - i : i; };
        auto cl = [&](int i) { return s(i <= N ? i : N); };
#pragma unroll
        for (int j = 0; j < RD - 1; j++) glds_stage(cl(j), j, nfc);
        int slot = 0;
#pragma unroll MPCC_LIGHT_UNROLL
        for (int i = 0; i <= N; i++) {
            glds_stage(cl(i + RD - 1), slot == 0 ? RD - 1 : slot - 1, nfc);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((RD - 1) * G) : "memory");
            In o;
            // the slot's image of this instance (last line of the slot: (G - 1) * 128 + grp * 32 + 16 + 15)
            static_assert((size_t)RD * G * 1024 <= 160 * 1024, "ring inside the LDS of a CU");
            read(smem + MPCC_BCHK(c.bchk, slot * G * 128, RD * G * 128 - G * 128 + 1, BC_LDS) + grp * 32, o);
            body(s(i), o);
            slot = slot == RD - 1 ? 0 : slot + 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };

    // ---- stage-local helpers (registers + DPP only)
    auto row_active = [&](int k, double bnd) { return (rowY ? (k >= 1) : (k < N)) && fabs(bnd) < BIG; };
    // unsigned c^T z of this lane's box / ddq row; (x, v) = lane components of a stage vector
    auto row_cz = [&](int k, double x, double v) -> double {
        const double vj = from_down<9>(v);  // lane 9+j <- v_j
        if (rowY) return x;
        return (k == 0) ? vj : vj - x;
    };
    // c^T z of poly row t (= p), reduced over the row's 16 lanes: sum_m a_p[m] y_m + bv_p[m] v_m
    auto poly_cz = [&](const In& in, int k, double x, double v) -> double {
        double r = 0.0;
#pragma unroll
        for (int p = 0; p < NPM; p++) {
            const bool live = (double)p < in.np && k < N;
            const double term = live ? fma2(in.pa[p], x, in.pb[p], v) : 0.0;
            const double s = g_sum(term);
            if (t == p) r = s;
        }
        return r;
    };
    auto poly_slot_active = [&](const In& in, int k) {
        return t < NPM && (double)t < in.np && k < N && fabs(in.pub) < BIG;
    };
    // gradient of the step system: g = g0 + sum_i sgn_i coef_i c_i (dvr: signed coefficient of row t,
    // cP: coefficient of poly row t)
    auto assemble_grad = [&](const In& in, int k, double g0x, double g0v, double dvr, double cP, double& gx, double& gv) {
        gx = g0x;
        if (t < 9) gx += dvr;
        else if (k >= 1) gx -= dvr;
        gv = g0v;
        const double dv_up = from_up<9>(dvr);  // lane j <- ddq row j
        if (t < 7 && k < N) gv += dv_up;
#pragma unroll
        for (int p = 0; p < NPM; p++) {
            const double cp = bcn(cP, p);
            const bool live = (double)p < in.np && k < N;
            if (live) {
                gx += cp * in.pa[p];  // zero for lanes >= 7
                gv += cp * in.pb[p];
            }
        }
    };
    // forward step: v = K x~ + kff (lanes 0..7) and x~' = A~ x~ + B~ v (all lanes)
    auto fwd_step = [&](const In& in, double xt, double& v, double& xn) {
        double part = 0.0;
        double xb[16];
#pragma unroll
        for (int m = 0; m < 16; m++) xb[m] = bcn(xt, m);
#pragma unroll
        for (int m = 0; m < 8; m++) part += in.m[m] * ((t < 8) ? xb[m] : xb[8 + m]);
        const double xb8 = xb[8];
        v = part + from_up<8>(part) + in.m[8];
        const double v7 = from_down<1>(v);
        const double vj = from_down<9>(v);
        if (t < 7) xn = fma2(mt, xt, gt, v);
        else if (t == 7) xn = fma(g77, v, fma2(m77, xt, m78, xb8));
        else if (t == 8) xn = fma2(m88, xt, g87, v7);
        else xn = vj;
    };

    // ---- start point: dynamics rollout with v = 0; slacks s = max(-g, IPM_S0), lambda = IPM_L0 / s, at most
    //      IPM_MAX_IT_SCALED iterations; a solve that does not converge from there restarts from
    //      s = max(-g, 1), lambda = 1 with IPM_MAX_IT (the oracle's solve_struct_ipm)
    In cur, nxt;
    // the three sweeps without the factorization (predictor forward, corrector backward and forward)
    // are short bodies that wait on their stage loads: they keep MPCC_LIGHT_DEPTH - 1 stages in flight
    In ring[MPCC_LIGHT_DEPTH];
    auto light_sweep = [&](bool backward, auto nfc, auto load, auto read, auto body) {
        if constexpr (use_ring(NPM)) lds_sweep(backward, nfc, read, body);
        else if constexpr (MPCC_WIDE_LIGHT_NOPF) sweep_noprefetch(N, backward, cur, load, body);
        else sweep<false>(N, backward, cur, nxt, load, body);
    };
    int it = 0, it_total = 0;
    bool conv = false, diverged = false;
    bool tail_req = false;  // tail mode requested for instance tail_gs of this wave (NPM <= 2)
    int tail_gs = 0;
    double alpha = 0.0;  // step length of the last iteration (the final iterate is z + alpha dz)
#pragma unroll 1
    for (int attempt = 0; attempt < IPM_ATTEMPTS; attempt++) {
    const double s_floor = (attempt == 0) ? IPM_S0 : 1.0;
    const double lam_scale = (attempt == 0) ? IPM_L0 : 0.0;
    const int max_it = (attempt == 0) ? IPM_MAX_IT_SCALED : IPM_MAX_IT;
    if (attempt == 1) {
        // restart only the solves that hit the cap or broke down from the scaled start; a P3 divergence is final
        // (the oracle's solve_struct_ipm)
        run = entered && !conv && !diverged;
        if (__ballot(run) == 0) break;
        if (run) diverged = false;
    }
    double mcount = 0.0;
    if (run) {
        double y = 0.0;  // lane a < 9: y_a of stage k
#if MPCC_ROLL_RING
        // the rollout reads only the QP record (bounds, poly rows, b_k in x0), RD_ROLL - 1 stages ahead in a
        // register ring (sweep_ring): with one stage ahead and the workspace fields of load_common besides, each
        // stage waited on its loads
        auto load_roll = [&](int k, In& o) {
            const gdouble* q = qs_stage(k);
            o.lb = q[rowY ? QS_YLB + t : QS_DLB + j9];
            o.ub = q[rowY ? QS_YUB + t : QS_DUB + j9];
            o.np = q[QS_NPOLY];
            const int tp = t < 7 ? t : 0;
#pragma unroll
            for (int p = 0; p < NPE; p++) {
                const double a = q[QS_POLY + 15 * p + tp], bv = q[QS_POLY + 15 * p + 7 + tp];
                o.pa[p] = (NPM > 0 && t < 7) ? a : 0.0;
                o.pb[p] = (NPM > 0 && t < 7) ? bv : 0.0;
            }
            const double pu = q[QS_POLY + 15 * (t < NPE ? t : 0) + 14];
            o.pub = (t < NPM) ? pu : INF;
            const double braw = q[QS_B + (t < 9 ? t : 0)];
            o.x0 = (k < N && t < 9) ? braw : 0.0;
        };
        constexpr int RD_ROLL = (NPM <= 2) ? 4 : 2;
        In rb[RD_ROLL];
        sweep_ring<RD_ROLL>(N, false, rb, load_roll, [&](int k, In& cur) {
            const double bk = cur.x0;
#else
        double bk = 0, bkn = 0;
        load_common(0, cur);
        bk = (N > 0 && t < 9) ? QSb[QS_B + t] : 0.0;
        for (int k = 0; k <= N; k++) {
            if (k < N) {
                load_common(k + 1, nxt);
                bkn = (k + 1 < N && t < 9) ? QSb[(size_t)(k + 1) * QS + QS_B + t] : 0.0;
            }
#endif
            const double yx = rowY ? y : 0.0;
            const double cz = row_cz(k, yx, 0.0);
            const double pcz = poly_cz(cur, k, yx, 0.0);
            if constexpr (PCACHE) *ws(k, F_PZ) = pcz;
            const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
            double sL = 1, lL = 0, sU = 1, lU = 0, sP = 1, lP = 0;
            if (aL) { sL = fmax(-(sgnL * cz - sgnL * cur.lb), s_floor); lL = (lam_scale > 0) ? lam_scale / sL : 1.0; }
            if (aU) { sU = fmax(-(sgnU * cz - sgnU * cur.ub), s_floor); lU = (lam_scale > 0) ? lam_scale / sU : 1.0; }
            if (aP) { sP = fmax(-(sgnU * pcz - sgnU * cur.pub), s_floor); lP = (lam_scale > 0) ? lam_scale / sP : 1.0; }
            mcount += (aL ? 1.0 : 0.0) + (aU ? 1.0 : 0.0) + (aP ? 1.0 : 0.0);
            store_slots(k, sL, lL, sU, lU, sP, lP, yx, 0.0, pcz);
            // y_{k+1} = M y_k + b_k (oracle order: sum_b M[a][b] y_b, then + b_a)
            const double y8 = from_up<1>(y);  // lane 7 <- y_8
            const double yn = (t == 7) ? fma2(m77, y, m78, y8) + bk : fma(mt, y, bk);
            y = (t < 9) ? yn : 0.0;
#if MPCC_ROLL_RING
        });
#else
            cur = nxt;
            bk = bkn;
        }
#endif
    }
    mcount = g_sum(mcount);
    PMARK(0);

    it = 0;
    double mu0 = 0.0;                    // mu of the starting point (P3)
    double dz_prev = 1e30;               // max |dz| of the previous iteration (step test)
    double sigma_mu = 0.0;               // previous iteration's sigma*mu (lazy update)
    double mu_cur = 1e30, rp_cur = 1e30; // mu and max |rp| of the current iterate (known for it > 0)
    bool pending = false;
    if (run) alpha = 0.0;
    while (true) {
        if (__ballot(run) == 0) break;
        if constexpr (NPM <= 2 || (MPCC_WIDE_TAIL && NPM >= 9)) {
            // Tail mode (ipm_tail.h): the wave's last running instance takes all four groups for the rest of its
            // solve.  Its iteration state goes to LDS and the solve continues in ipm_tail_solve after this function
            // returns (a call from here would change this function's register allocation); the wave's other
            // instances are done with this QP, and none of them waits for the restart of attempt 1.
            const unsigned long long lead = __ballot(run && t == 0);
            if (c.tail && __popcll(lead) == 1 &&
                __ballot(t == 0 && !run && entered && !conv && !diverged && attempt == 0) == 0) {
                tail_gs = (__ffsll((long long)lead) - 1) >> 4;
                tail_req = true;
                if (lane == tail_gs * 16) {
                    double* st = smem + TL_STATE;
                    st[0] = it; st[1] = max_it; st[2] = pending ? 1.0 : 0.0; st[3] = attempt; st[4] = it_total;
                    st[5] = mu0; st[6] = dz_prev; st[7] = sigma_mu; st[8] = mu_cur; st[9] = rp_cur; st[10] = alpha;
                    st[11] = mcount; st[12] = tail_gs;
                }
                run = false;
                break;
            }
        }
        {
            // ================= factorization sweep k = N..0 with the lazy update of the previous step,
            // the objective gradient g0 = H z + h and the predictor backward solve.  The whole wave runs it,
            // the instances that are done included (their lanes re-read stage N and store nothing): P's update
            // U^T U runs on the matrix cores over the wave's 4 instances, which needs every lane (see (4)).
            double Pc[16];   // column t of P_{k+1}
            double pv = 0.0; // p_{k+1}, component t
            bool chol_ok = true;
            auto factor_sweep = [&](auto load, auto body) {
                if constexpr (NPM <= 2) sweep<true>(N, true, cur, nxt, load, body);
                else if constexpr (MPCC_WIDE_FACTOR_PF) sweep<false>(N, true, cur, nxt, load, body);
                else sweep_noprefetch(N, true, cur, load, body);
            };
            // pin(nx): the next stage's prefetched fields, settled in registers before the body's late stores.  A
            // load's first use waits (vmcnt) for every store issued before it as well (gfx9 counts stores in
            // vmcnt); settled here, a body's stores no longer delay the next body's start.
            auto pin = [&](In& x) {
                asm volatile("" : "+v"(x.lb), "+v"(x.ub), "+v"(x.np), "+v"(x.pub), "+v"(x.zx), "+v"(x.zv));
                asm volatile("" : "+v"(x.sL), "+v"(x.lL), "+v"(x.sU), "+v"(x.lU), "+v"(x.sP), "+v"(x.lP));
                asm volatile("" : "+v"(x.x0), "+v"(x.x1), "+v"(x.x2), "+v"(x.x3));
#pragma unroll
                for (int q = 0; q < 12; q++) asm volatile("" : "+v"(x.m[q]));
#pragma unroll
                for (int q = 0; q < NPE; q++) asm volatile("" : "+v"(x.pa[q]), "+v"(x.pb[q]));
            };
            factor_sweep([&](int k, In& o) { load_factor(run ? k : N, o, pending); }, [&](int k, const In& cur, auto&... nx) {
                const double lb = cur.lb, ub = cur.ub;
                const double* Qr = cur.m;
                const double qt = cur.m[9], Rt = cur.m[10], rt = cur.m[11];
                double sL = cur.sL, lL = cur.lL, sU = cur.sU, lU = cur.lU, sP = cur.sP, lP = cur.lP;
                double zx = cur.zx, zv = cur.zv;
                const bool aL = row_active(k, lb), aU = row_active(k, ub), aP = poly_slot_active(cur, k);
                if (pending) {
                    // previous iteration's update at this stage (oracle: z += a dz, s += a ds, l += a dl)
                    const double dx = cur.x0, dv = cur.x1, ax = cur.x2, av = cur.x3;
                    const double cz = row_cz(k, zx, zv), cd = row_cz(k, dx, dv), ca = row_cz(k, ax, av);
                    double pcz, pcd, pca;
                    if constexpr (PCV) {
                        pcz = cur.pz; pcd = cur.pcd; pca = cur.pca;
                    } else {
                        pcz = poly_cz(cur, k, zx, zv); pcd = poly_cz(cur, k, dx, dv); pca = poly_cz(cur, k, ax, av);
                    }
                    double rpd;
                    if constexpr (MPCC_SLOT_SELECT) {  // every slot computed, inactive ones kept by selects (no branches)
                        auto upd = [&](bool a, double sgn, double bnd, double czz, double caa, double cdd, double& sv, double& lv) {
                            const SlotStep st = slot_corr(sgn, bnd, czz, caa, cdd, sv, lv, sigma_mu, &rpd);
                            const double sn = sv + alpha * st.ds, ln = lv + alpha * st.dl;
                            sv = a ? sn : sv;
                            lv = a ? ln : lv;
                        };
                        upd(aL, sgnL, lb, cz, ca, cd, sL, lL);
                        upd(aU, sgnU, ub, cz, ca, cd, sU, lU);
                        upd(aP, sgnU, cur.pub, pcz, pca, pcd, sP, lP);
                    } else {
                    if (aL) { const SlotStep st = slot_corr(sgnL, lb, cz, ca, cd, sL, lL, sigma_mu, &rpd); sL += alpha * st.ds; lL += alpha * st.dl; }
                    if (aU) { const SlotStep st = slot_corr(sgnU, ub, cz, ca, cd, sU, lU, sigma_mu, &rpd); sU += alpha * st.ds; lU += alpha * st.dl; }
                    if (aP) { const SlotStep st = slot_corr(sgnU, cur.pub, pcz, pca, pcd, sP, lP, sigma_mu, &rpd); sP += alpha * st.ds; lP += alpha * st.dl; }
                    }
                    zx += alpha * dx;
                    zv += alpha * dv;
                    if constexpr (!PCN) {
                        if (run) store_slots(k, sL, lL, sU, lU, sP, lP, zx, zv, 0.0);
                    }
                }
                PMARK(8);
                // ---- slots: barrier weights and predictor coefficients (rc = s l)
                const double cz = row_cz(k, zx, zv);
                const double pcz = poly_cz(cur, k, zx, zv);
                if constexpr (PCACHE) {
                    if (run) *ws(k, F_PZ) = pcz;
                }
                if constexpr (PCN) {  // the updated iterate with its c_p^T z (unchanged iterate: stored as it is)
                    if (run && pending) store_slots(k, sL, lL, sU, lU, sP, lP, zx, zv, pcz);
                }
                double WL = 0, WU = 0, WP = 0, cL = 0, cU = 0, cP = 0;
                if constexpr (MPCC_SLOT_SELECT) {
                    auto wc = [&](bool a, double sgn, double czz, double bnd, double sv, double lv, double& W, double& cf) {
                        const double rp = slot_rp(sgn, czz, bnd, sv);
                        const double ri = rcp(sv);
                        const double w = lv * ri, cc = slot_coef(ri, lv, rp, sv * lv);
                        W = a ? w : 0.0;
                        cf = a ? cc : 0.0;
                    };
                    wc(aL, sgnL, cz, lb, sL, lL, WL, cL);
                    wc(aU, sgnU, cz, ub, sU, lU, WU, cU);
                    wc(aP, sgnU, pcz, cur.pub, sP, lP, WP, cP);
                } else {
                if (aL) { const double rp = slot_rp(sgnL, cz, lb, sL); const double ri = rcp(sL); WL = lL * ri; cL = slot_coef(ri, lL, rp, sL * lL); }
                if (aU) { const double rp = slot_rp(sgnU, cz, ub, sU); const double ri = rcp(sU); WU = lU * ri; cU = slot_coef(ri, lU, rp, sU * lU); }
                if (aP) { const double rp = slot_rp(sgnU, pcz, cur.pub, sP); const double ri = rcp(sP); WP = lP * ri; cP = slot_coef(ri, lP, rp, sP * lP); }
                }
                const double wd = WL + WU;                 // diagonal weight of row t
                const double dvr = sgnL * cL + sgnU * cU;  // signed coefficient of row t
                // ---- objective gradient g0 = H z + h (f_xu = 0; oracle order: sum over z, then + h)
                double g0x, g0v = 0.0;
                {
                    double zb[9];
#pragma unroll
                    for (int m = 0; m < 9; m++) zb[m] = bcn(zx, m);
                    const double vj = from_down<9>(zv);  // lane 9+j <- v_j
                    const double wj = from_up<9>(zx);    // lane j <- w_j
                    if (t < 9) {
                        double s = 0;
#pragma unroll
                        for (int m = 0; m < 9; m++) s += Qr[m] * zb[m];
                        g0x = s + qt;
                    } else {
                        g0x = (k >= 1 && k < N) ? Hct * vj : 0.0;
                    }
                    if (t < 8 && k < N) {
                        double s = (k >= 1 && t < DOF) ? Hct * wj : 0.0;
                        s += Rt * zv;
                        g0v = s + rt;
                    }
                }
                if (run) *ws(k, F_GX) = g0x;
                double gx, gv;
                assemble_grad(cur, k, g0x, g0v, dvr, cP, gx, gv);
                PMARK(9);
                if (k == N) {
                    // terminal stage: P = Hb_N (y block only; Q row t used as column t), p = g_x~
#pragma unroll
                    for (int a = 0; a < 16; a++) {
                        double v = 0.0;
                        if (t < 9 && a < 9) {
                            v = Qr[a];
                            if (a == t) v += wd;
                        }
                        Pc[a] = v;
                    }
                    pv = gx;
                    // no gains at the terminal stage: zeros, so the light sweeps' loads need no stage select
                    if (run) {
#pragma unroll
                        for (int m = 0; m < 8; m++) *ws(k, F_KR + m) = 0.0;
                        *ws(k, F_GVK) = (t < 8) ? g0v : 0.0;
#pragma unroll
                        for (int m = 0; m < 4; m++) *ws(k, F_FI + m) = 0.0;
                    }
                    return;
                }
                // ---- (1) Y = B~^T P (column t), f = g_v + B~^T p (lanes 0..7)
                double Y[8];
#pragma unroll
                for (int i = 0; i < 7; i++) Y[i] = gdiag[i] * Pc[i] + Pc[9 + i];
                Y[7] = fma2(g77, Pc[7], g87, Pc[8]);
                const double pu9 = from_up<9>(pv), pu1 = from_up<1>(pv);  // DPP in uniform control flow
                const double fg = fma(gt, pv, gv);
                const double fv = (t < 7) ? fg + pu9 : fma(g87, pu1, fg);
                // ---- (2) F column t (t < 8), Gm column t (t < 9); poly terms W_p bv_p bv_p^T, W_p bv_p a_p^T
                // The rank-NPM poly terms accumulate row p by row p: each broadcast bv_p[i] is consumed as
                // soon as it is made (DPP results are pinned in program order, so broadcasting every
                // bv_p[i] first kept 8 NPM values live; at NPM = 11 that spilled).  Per accumulator the
                // operations and their order are those of the oracle's sum over p.
                const double wdv = from_up<9>(wd);  // lane j <- ddq row j weight
                double hF[8], hG[8];
                double hq[7];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    hF[i] = (i == t) ? Rt + ((t < 7) ? wdv : 0.0) : 0.0;
                    hG[i] = 0.0;
                }
                auto hq_base = [&]() {
#pragma unroll
                    for (int a = 0; a < 7; a++) {
                        hq[a] = Qr[a];
                        if (a == t) hq[a] += wd;
                    }
                };
                if constexpr (GRAM_MFMA) {
                    // Wide-poly variants: the three rank-NPM blocks as one Gram matrix on the matrix cores.  With
                    // r_p = [bv_p (lanes 0..6), 0, a_p (lanes 8..14), 0] and w_p the barrier weight of live poly row
                    // p, D = sum_p w_p r_p r_p^T holds sum_p W_p bv_p bv_p^T (rows, columns 0..6), W_p bv_p a_p^T
                    // (rows 0..6, columns 8..14) and W_p a_p a_p^T (rows, columns 8..14): per instance
                    // ceil(NPM / 4) v_mfma_f64_16x16x4f64 over k = p, operands and products moved between the
                    // instance layout and the MFMA layout by the 16-lane-group transposes of (4).  Replaced ~100
                    // broadcasts and multiply-adds per poly row and stage.
                    constexpr int KS = (NPM + 3) / 4;
                    double xs[KS][4][1], as[KS][4][1];
#pragma unroll
                    for (int q = 0; q < KS; q++)
#pragma unroll
                        for (int g = 0; g < 4; g++) {
                            const int pp = 4 * q + g;
                            double x = 0.0, w = 0.0;
                            if (pp < NPM) {
                                const double a8 = from_down<8>(cur.pa[pp]);  // lane 8 + i <- a_p[i]
                                x = (t < 8) ? cur.pb[pp] : a8;
                                const bool live = (double)pp < cur.np && k < N;
                                const double wp = bcn(WP, pp);
                                w = live ? wp : 0.0;
                            }
                            xs[q][g][0] = x;
                            as[q][g][0] = w * x;
                        }
#pragma unroll
                    for (int q = 0; q < KS; q++) {
                        group_transpose(xs[q]);
                        group_transpose(as[q]);
                    }
                    double dg[4][4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int q = 0; q < KS; q++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(as[q][j][0], xs[q][j][0], acc, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 4; r++) dg[j][r] = acc[r];
                    }
                    group_transpose(dg);  // lane (j, t): column t of D_j, row g + 4 r in dg[g][r]
                    const bool q7 = t < 7;
#pragma unroll
                    for (int i = 0; i < 7; i++) {
                        const double dF = dg[i & 3][i >> 2];                       // D[i][t]
                        const double dG = from_up<8>(dg[i & 3][i >> 2]);           // D[i][8 + t]
                        hF[i] += q7 ? dF : 0.0;
                        hG[i] += q7 ? dG : 0.0;
                    }
                    hq_base();
#pragma unroll
                    for (int a = 0; a < 7; a++) {
                        const double dq = from_up<8>(dg[(8 + a) & 3][(8 + a) >> 2]);  // D[8 + a][8 + t]
                        hq[a] += q7 ? dq : 0.0;
                    }
                } else {
                // The rank-NPM poly terms accumulate row p by row p: each broadcast bv_p[i] is consumed as
                // soon as it is made (DPP results are pinned in program order, so broadcasting every
                // bv_p[i] first kept 8 NPM values live; at NPM = 11 that spilled).  Per accumulator the
                // operations and their order are those of the oracle's sum over p.
                double Wb[NPE];
#pragma unroll
                for (int p = 0; p < NPM; p++) {
                    const bool live = (double)p < cur.np && k < N;
                    const double wp = bcn(WP, p);
                    Wb[p] = live ? wp : 0.0;
#pragma unroll
                    for (int i = 0; i < 7; i++) {
                        const double bv = bcn(cur.pb[p], i);
                        hF[i] += Wb[p] * (bv * cur.pb[p]);  // bv_p[t]: zero for lanes >= 7
                        hG[i] += Wb[p] * (bv * cur.pa[p]);  // a_p[t]: zero for lanes >= 7
                    }
                }
                }
                // Hb's poly terms (q block, rows a < 7), row p by row p as for F above.  The wide-poly variants
                // without the Gram MFMA form them here, so that a_p (NPM values per lane) dies before the Cholesky
                // instead of living through it into the Hb section (it spilled there); <= 2 rows keep the late
                // placement, where the 7 sums would be the longer live range.  Same terms in the same order.
                auto poly_hq = [&]() {
                    hq_base();
#pragma unroll
                    for (int p = 0; p < NPM; p++) {
                        const bool live = (double)p < cur.np && k < N;
                        const double wp = bcn(WP, p);
                        const double wb = live ? wp : 0.0;
#pragma unroll
                        for (int a = 0; a < 7; a++) {
                            const double pa_ = bcn(cur.pa[p], a);
                            hq[a] += wb * (pa_ * cur.pa[p]);
                        }
                    }
                };
                if constexpr (!GRAM_MFMA && NPM > 2) poly_hq();
                double Fc[8], gm[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const double yu9 = from_up<9>(Y[i]);
                    const double yu1 = from_up<1>(Y[i]);
                    const double yd = from_down<1>(Y[i]);
                    Fc[i] = hF[i] + fma(gt, Y[i], (t < 7) ? yu9 : g87 * yu1);
                    gm[i] = hG[i] + fma(mt, Y[i], (t == 8) ? m78 * yd : 0.0);
                }
                PMARK(10);
                // ---- (3) chol(F) from the broadcast columns; U = LF^-1 Gm; K = -LF^-T U; Finv column (t & 7);
                //          kff = -F^-1 f; p = g_x~ + A~^T p + K^T f
                double LF[36], dinv[8];
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) LF[i * (i + 1) / 2 + j] = bcn(Fc[i], j);
                chol_ok = chol8(LF, dinv) && chol_ok;
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
                double fb[8];
#pragma unroll
                for (int i = 0; i < 8; i++) fb[i] = bcn(fv, i);
                double kff = 0.0;
#pragma unroll
                for (int m = 0; m < 8; m++) kff -= fi[m] * fb[m];
                double pnew;
                {
                    const double p7 = from_down<1>(pv);
                    double gxa = gx;  // g_x~ + A~^T p
                    if (t < 9) gxa = fma(mt, pv, gxa);
                    if (t == 8) gxa = fma(m78, p7, gxa);
                    double ktf = 0.0;
#pragma unroll
                    for (int i = 0; i < 8; i++) ktf += kc[i] * fb[i];
                    pnew = gxa + ktf;
                }
                PMARK(11);
#ifdef MPCC_IPM_DBGF2  // tools/tail_ws_diff.py --dbg2: L, 1/L_jj (lane 0, fields 29..31), U and K columns (32..47)
                if (run) {
                    if (t == 0) {
                        for (int i = 0; i < 36; i++) WSb[(size_t)k * IS + 29 * 16 + i] = LF[i];
                        for (int i = 0; i < 8; i++) WSb[(size_t)k * IS + 29 * 16 + 36 + i] = dinv[i];
                    }
                    double uu[8];
                    for (int i = 0; i < 8; i++) uu[i] = u[i];
                    for (int i = 0; i < 8; i++) { *ws(k, 32 + i) = uu[i]; *ws(k, 40 + i) = kc[i]; }
                }
#endif
#ifdef MPCC_IPM_DBGF
                if (run) { *ws(k, 35) = gx; *ws(k, 36) = gv; *ws(k, 37) = pv; *ws(k, 38) = fv; *ws(k, 39) = dvr; *ws(k, 40) = cP;
                *ws(k, 41) = wd; *ws(k, 42) = pnew; *ws(k, 43) = kff; *ws(k, 44) = Pc[0]; *ws(k, 45) = LF[35];
                *ws(k, 46) = dinv[7]; *ws(k, 47) = u[0]; *ws(k, 48) = kc[0]; *ws(k, 49) = Y[0]; *ws(k, 50) = Fc[0]; }
#endif
#pragma unroll
                for (int i = 0; i < 8; i++) S[L_K + i * 16 + t] = kc[i];
                if constexpr (MPCC_PIN) (pin(nx), ...);
                // K row halves to the workspace (LDS transpose), early: a store's completion is waited for by the
                // next vmcnt wait on a load (gfx9 counts stores in vmcnt), and the next stage's first use of its
                // prefetched fields comes right at the top of the next body; issued here, the P update below
                // covers their latency
                if constexpr (MPCC_KR_EARLY) {
                lds_sync();
                {
                    const int ri = t & 7, hoff = (t < 8) ? 0 : 8;
                    const double2* row = reinterpret_cast<const double2*>(S + L_K + ri * 16 + hoff);
#pragma unroll
                    for (int q2 = 0; q2 < 4; q2++) {
                        const double2 w = row[q2];
                        if (run) {
                            *ws(k, F_KR + 2 * q2) = w.x;
                            *ws(k, F_KR + 2 * q2 + 1) = w.y;
                        }
                    }
                }
                }
                {
                    const double kffd = from_down<8>(kff);  // lane 8+i <- kff_i
                    if (run) *ws(k, F_GVK) = (t < 8) ? g0v : kffd;
                }
                if (run) {
#pragma unroll
                    for (int m = 0; m < 4; m++) *ws(k, F_FI + m) = (t < 8) ? fi[m] : fi[4 + m];
                }
                // ---- (4) Hb column t and P = Hb - U^T U (column t)
                double hb[16];
                {
                    double Pc7[9];
#pragma unroll
                    for (int a = 0; a < 9; a++) Pc7[a] = from_down<1>(Pc[a]);  // lane 8 <- P[a][7]
                    if constexpr (NPM <= 2) poly_hq();
#pragma unroll
                    for (int a = 0; a < 16; a++) {
                        double v = 0.0;
                        if (a < 9) {
                            if (t < 9) {
                                if (a < 7) {
                                    v = hq[a];
                                } else {
                                    v = Qr[a];
                                    if (a == t) v += wd;
                                }
                                v = hb_mp(v, a, Pc, Pc7);
                            }
                        } else if (a == t) {
                            v = wd;
                        }
                        hb[a] = v;
                    }
                }
                if (k > 0) {
                    // On the matrix cores, per instance j of the wave: P_j = Hb_j - U_j^T U_j as two
                    // v_mfma_f64_16x16x4f64 (rows 0..3, then 4..7 of U_j) with C = Hb_j.  The instruction is
                    // bitwise an ascending fma chain over k (tools/probes/mfma_f64_probe.hip), so every entry
                    // is fma(-U[7][a], U[7][t], ... fma(-U[0][a], U[0][t], Hb[a][t])), the VALU form's order.
                    // Operand maps (A lane (g, c) -> A[c][g], B -> B[g][c], C/D register r -> [g + 4r][c]) from
                    // the instance layout (lane (j, t): column t of instance j) by 4x4 transposes of the
                    // wave's 16-lane groups: lane (g, c) gets U_j[g][c], U_j[4 + g][c] and Hb_j[g + 4r][c]
                    // of every instance j, and the products go back the same way.  (U^T U issued from C = 0
                    // right after U is formed, to overlap the solves, held its 16 results through them: more
                    // spills, k_sqp 3.40 ms against 3.31 ms; profiles/r03m_*.)
#if MPCC_P_LDS
                    // The instance <-> MFMA layout moves through the wave's LDS (free during the factorization
                    // sweep: the light sweeps' ring is drained) instead of permlane butterflies: lane (j, c) stores
                    // its Hb column in the order p(a) = 4 (a & 3) + (a >> 2) and its U column as [u0 u4 u1 u5 ..];
                    // lane (g, c) then reads Hb_j[g + 4r][c] (r = 0..3) and U_j[g][c], U_j[4 + g][c] of every
                    // instance j as three 16-byte reads, and the products return the same way.  Same MFMAs on the
                    // same operands: bitwise the butterfly form.
                    {
                        double* const PX = smem + P_LDS_BASE;            // [64 lanes][18]: Hb, then the products
                        double* const PU = smem + P_LDS_BASE + 64 * 18;  // [64 lanes][10]: U
                        double2* const h2 = reinterpret_cast<double2*>(PX + lane * 18);
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            const int p0 = 2 * q, p1 = 2 * q + 1;
                            h2[q] = make_double2(hb[(p0 & 3) * 4 + (p0 >> 2)], hb[(p1 & 3) * 4 + (p1 >> 2)]);
                        }
                        double2* const u2 = reinterpret_cast<double2*>(PU + lane * 10);
#pragma unroll
                        for (int q = 0; q < 4; q++) u2[q] = make_double2(u[q], u[4 + q]);
                        lds_sync();
                        d4 acc[4];
                        double2 uu[4];
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const int src = j * 16 + t;
                            const double2* hs = reinterpret_cast<const double2*>(PX + src * 18 + grp * 4);
                            const double2 h01 = hs[0], h23 = hs[1];
                            acc[j] = d4{h01.x, h01.y, h23.x, h23.y};
                            uu[j] = reinterpret_cast<const double2*>(PU + src * 10)[grp];
                        }
                        lds_sync();
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(-uu[j].x, uu[j].x, acc[j], 0, 0, 0);
                            acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(-uu[j].y, uu[j].y, acc[j], 0, 0, 0);
                        }
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            double2* const rs = reinterpret_cast<double2*>(PX + (j * 16 + t) * 18 + grp * 4);
                            rs[0] = make_double2(acc[j][0], acc[j][1]);
                            rs[1] = make_double2(acc[j][2], acc[j][3]);
                        }
                        lds_sync();
                        double pp[16];
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            const double2 v = h2[q];
                            pp[2 * q] = v.x;
                            pp[2 * q + 1] = v.y;
                        }
#pragma unroll
                        for (int a = 0; a < 16; a++) Pc[a] = pp[(a & 3) * 4 + (a >> 2)];
                    }
#else
                    double x[4][4], ua[4][1], ub[4][1];
#pragma unroll
                    for (int g = 0; g < 4; g++) {
#pragma unroll
                        for (int r = 0; r < 4; r++) x[g][r] = hb[g + 4 * r];
                        ua[g][0] = u[g];
                        ub[g][0] = u[4 + g];
                    }
                    group_transpose(x);
                    group_transpose(ua);
                    group_transpose(ub);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        d4 acc = {x[j][0], x[j][1], x[j][2], x[j][3]};
                        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ua[j][0], ua[j][0], acc, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ub[j][0], ub[j][0], acc, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 4; r++) x[j][r] = acc[r];
                    }
                    group_transpose(x);
#pragma unroll
                    for (int g = 0; g < 4; g++)
#pragma unroll
                        for (int r = 0; r < 4; r++) Pc[g + 4 * r] = x[g][r];
#endif
                }
                if constexpr (!MPCC_KR_EARLY) {
                lds_sync();
                {
                    const int ri = t & 7, hoff = (t < 8) ? 0 : 8;
                    const double2* row = reinterpret_cast<const double2*>(S + L_K + ri * 16 + hoff);
#pragma unroll
                    for (int q2 = 0; q2 < 4; q2++) {
                        const double2 w = row[q2];
                        if (run) {
                            *ws(k, F_KR + 2 * q2) = w.x;
                            *ws(k, F_KR + 2 * q2 + 1) = w.y;
                        }
                    }
                }
                }
                pv = pnew;
                lds_sync();
                PMARK(13);
            });
            if (run && !chol_ok) {
                // Riccati breakdown: MaxIterReached unless the current iterate is converged to IPM_TOL_FB (P2);
                // the sweep has already applied the pending update, so the iterate is the stored z
                conv = it > 0 && mu_cur < IPM_TOL_FB && rp_cur < IPM_TOL_FB;
                alpha = 0.0;
                run = false;
            }
        }
        PMARK(2);
        if (run) {
            // ---- predictor forward: x~_0 = 0; recover dsa, dla; max step; mu(alpha) sums
            double S0 = 0, S1 = 0, S2 = 0;
            MinRatio amr(1.0);
            double xt = 0.0;
            light_sweep(false, std::integral_constant<int, LF_PRED>{}, [&](int k, In& o) { load_fwd(k, o, false); },
                        [&](const double* im, In& o) { lds_fwd(im, o, false); }, [&](int k, const In& cur) {
                const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                double v = 0.0, xn = 0.0;
                if (k < N) fwd_step(cur, xt, v, xn);
                const double dvv = (t < 8 && k < N) ? v : 0.0;
                *ws(k, F_AX) = xt;
                const double cz = row_cz(k, cur.zx, cur.zv), ca = row_cz(k, xt, dvv);
                const double pcz = PCV ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv), pca = poly_cz(cur, k, xt, dvv);
                if constexpr (PCACHE) *ws(k, F_PA) = pca;
                if constexpr (PCN) {
                    const double pa8 = from_down<8>(pca);  // lane 8 + p <- c_p^T dza
                    *ws(k, F_AV) = (t < 8) ? dvv : pa8;
                } else {
                    *ws(k, F_AV) = dvv;
                }
                auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l) {
                    if (!MPCC_SLOT_SELECT && !a) return;
                    const double rp = slot_rp(sgn, czz, bnd, s);
                    SlotStep st = slot_recover(rcp(s), l, rp, sgn * caa, s * l);
                    if constexpr (MPCC_SLOT_SELECT) {  // an inactive slot adds exact zeros (as tail mode's D phase)
                        st.ds = a ? st.ds : 0.0;
                        st.dl = a ? st.dl : 0.0;
                        s = a ? s : 0.0;
                        l = a ? l : 0.0;
                    }
                    step_bound(amr, s, l, st);
                    mu_acc(S0, S1, S2, s, l, st.ds, st.dl);
                };
                rec(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL);
                rec(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU);
                rec(aP, sgnU, cur.pub, pcz, pca, cur.sP, cur.lP);
                xt = xn;
            });
            const double amax = g_min(amr.value());
            S0 = g_sum(S0); S1 = g_sum(S1); S2 = g_sum(S2);
            const double mu = (mcount > 0) ? S0 / mcount : 0.0;
            if (it == 0) mu0 = mu;
            double mua = S0 + amax * S1 + amax * amax * S2;
            mua = (mcount > 0) ? mua / mcount : 0.0;
            const double ratio = (mu > 0) ? mua / mu : 0.0;
            const double sigma = (mu > 0) ? ratio * ratio * ratio : 0.0;
            const double smu = sigma * mu;
            PMARK(3);

            // ---- corrector backward: coef with rc = s l + dsa dla - sigma mu; f = g_v + B~^T p;
            //      kff = -F^-1 f; p = g_x~ + A~^T p + K^T f
            double pv = 0.0;
            light_sweep(true, std::integral_constant<int, LF_CBWD>{}, [&](int k, In& o) { load_bwd(k, o); },
                        [&](const double* im, In& o) { lds_bwd(im, o); }, [&](int k, const In& cur) {
                const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                const double cz = row_cz(k, cur.zx, cur.zv), ca = row_cz(k, cur.x0, cur.x1);
                const double pcz = PCV ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv);
                const double pca = PCV ? cur.pca : poly_cz(cur, k, cur.x0, cur.x1);
                auto coef = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l) -> double {
                    if (!MPCC_SLOT_SELECT && !a) return 0.0;
                    const double rp = slot_rp(sgn, czz, bnd, s);
                    const double ri = rcp(s);
                    const SlotStep pa = slot_recover(ri, l, rp, sgn * caa, s * l);
                    const double rc = fma(s, l, pa.ds * pa.dl) - smu;
                    const double cf = slot_coef(ri, l, rp, rc);
                    return a ? cf : 0.0;
                };
                const double cL = coef(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL);
                const double cU = coef(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU);
                const double cP = coef(aP, sgnU, cur.pub, pcz, pca, cur.sP, cur.lP);
                const double dvr = sgnL * cL + sgnU * cU;
                double gx, gv;
                assemble_grad(cur, k, cur.x2, cur.x3, dvr, cP, gx, gv);
                if (k == N) {
                    pv = gx;
                    return;
                }
                const double pu9 = from_up<9>(pv), pu1 = from_up<1>(pv);  // DPP in uniform control flow
                const double fg = fma(gt, pv, gv);
                const double fv = (t < 7) ? fg + pu9 : fma(g87, pu1, fg);
                double part = 0.0;
                double fb[8];
#pragma unroll
                for (int i = 0; i < 8; i++) fb[i] = bcn(fv, i);
#pragma unroll
                for (int m = 0; m < 4; m++) part -= cur.m[8 + m] * ((t < 8) ? fb[m] : fb[4 + m]);
                const double kff = part + from_up<8>(part);
                const double kffd = from_down<8>(kff);  // lane 8+i <- kff_i
                if (t >= 8) *ws(k, F_GVK) = kffd;
                const double p7 = from_down<1>(pv);
                double gxa = gx;  // g_x~ + A~^T p
                if (t < 9) gxa = fma(mt, pv, gxa);
                if (t == 8) gxa = fma(m78, p7, gxa);
                // K^T f from the K row halves: column sums over each 8-lane half by a transpose-reduce
                // butterfly (lane j <-> 7-j, j^2, j^1); lane c ends with column c (c < 8) or 8 + (c & 7)
                const double f8 = rot16<8>(fv);  // lane 8+i <- f_i (unconditional: DPP in uniform control flow)
                const double fh = (t < 8) ? fv : f8;
                double r1[4], r2[2];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const bool lo = (t & 4) == 0;
                    const double mk = lo ? cur.m[q] : cur.m[4 + q], mo = lo ? cur.m[4 + q] : cur.m[q];
                    r1[q] = fma(mk, fh, half_mirror(mo * fh));
                }
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const bool lo = (t & 2) == 0;
                    r2[q] = (lo ? r1[q] : r1[2 + q]) + quad_swap2(lo ? r1[2 + q] : r1[q]);
                }
                const bool lo1 = (t & 1) == 0;
                const double ktf = (lo1 ? r2[0] : r2[1]) + quad_swap1(lo1 ? r2[1] : r2[0]);
                pv = gxa + ktf;
            });
            PMARK(4);

            // ---- corrector forward: dz, ds, dl, max step, mu(alpha) sums, max |rp|, max |dz|
            double T0 = 0, T1 = 0, T2 = 0, rpm = 0, dzm = 0;
            MinRatio amc(1e30);
            xt = 0.0;
            light_sweep(false, std::integral_constant<int, LF_CFWD>{}, [&](int k, In& o) { load_fwd(k, o, true); },
                        [&](const double* im, In& o) { lds_fwd(im, o, true); }, [&](int k, const In& cur) {
                const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                double v = 0.0, xn = 0.0;
                if (k < N) fwd_step(cur, xt, v, xn);
                const double dvv = (t < 8 && k < N) ? v : 0.0;
                *ws(k, F_DX) = xt;
                dzm = fmax(dzm, fmax(fabs(xt), fabs(dvv)));
                const double cz = row_cz(k, cur.zx, cur.zv), cd = row_cz(k, xt, dvv), ca = row_cz(k, cur.x0, cur.x1);
                const double pcz = PCV ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv), pcd = poly_cz(cur, k, xt, dvv);
                const double pca = PCV ? cur.pca : poly_cz(cur, k, cur.x0, cur.x1);
                if constexpr (PCACHE) *ws(k, F_PD) = pcd;
                if constexpr (PCN) {
                    const double pd8 = from_down<8>(pcd);  // lane 8 + p <- c_p^T dz
                    *ws(k, F_DV) = (t < 8) ? dvv : pd8;
                } else {
                    *ws(k, F_DV) = dvv;
                }
                auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double cdd, double s, double l) {
                    if (!MPCC_SLOT_SELECT && !a) return;
                    double rp;
                    SlotStep st = slot_corr(sgn, bnd, czz, caa, cdd, s, l, smu, &rp);
                    if constexpr (MPCC_SLOT_SELECT) {
                        st.ds = a ? st.ds : 0.0;
                        st.dl = a ? st.dl : 0.0;
                        s = a ? s : 0.0;
                        l = a ? l : 0.0;
                        rp = a ? rp : 0.0;
                    }
                    step_bound(amc, s, l, st);
                    mu_acc(T0, T1, T2, s, l, st.ds, st.dl);
                    rpm = fmax(rpm, fabs(rp));
                };
                rec(aL, sgnL, cur.lb, cz, ca, cd, cur.sL, cur.lL);
                rec(aU, sgnU, cur.ub, cz, ca, cd, cur.sU, cur.lU);
                rec(aP, sgnU, cur.pub, pcz, pca, pcd, cur.sP, cur.lP);
                xt = xn;
            });
            const double amx = g_min(amc.value());
            T0 = g_sum(T0); T1 = g_sum(T1); T2 = g_sum(T2);
            rpm = g_max(rpm);
            dzm = g_max(dzm);
            alpha = fmin(1.0, fmax(IPM_TAU, 1.0 - sqrt(mu)) * amx);  // adaptive fraction to the boundary (oracle)
            sigma_mu = smu;
            pending = true;
            it++;
            PMARK(5);
            // convergence test at the start of the next iteration (oracle: only while it < max_it)
            if (it < max_it) {
                double mun = T0 + alpha * T1 + alpha * alpha * T2;
                mun = (mcount > 0) ? mun / mcount : 0.0;
                const double rpn = (1.0 - alpha) * rpm;
                mu_cur = mun;
                rp_cur = rpn;
                // step test: |dz| below tolerance, or quadratic contraction dz^2 / dz_prev below it
                // (the oracle's step_converged, mpcc_oracle.cpp)
                const bool step_ok = dzm < IPM_TOL_STEP || dzm * dzm < IPM_TOL_STEP * dz_prev;
                dz_prev = dzm;
                if (mun < IPM_TOL_MU && rpn < IPM_TOL_P && step_ok) {
                    conv = true;
                    run = false;
                } else if (mun > IPM_DIV * mu0) {  // P3: divergent multipliers, primal infeasible
                    diverged = true;
                    run = false;
                }
            } else {
                run = false;
            }
        }
    }
    it_total += it;
    if (tail_req) break;  // no other instance of the wave needs the restart (checked at the hand-over)
    }  // attempt

#ifdef MPCC_IPM_PROF
    if (entered && t == 0) {
        for (int i = 0; i < 16; i++) if (i != 6 && i != 7) atomicAdd(&g_ipm_prof[i], (unsigned long long)prof_acc[i]);
        atomicAdd(&g_ipm_prof[6], (unsigned long long)it_total);
        atomicAdd(&g_ipm_prof[7], 1ull);
    }
#endif
    if (!entered || (tail_req && grp == tail_gs)) return tail_req;
#ifdef MPCC_IPM_PROF
    if (t == 0 && b < 4 * PROF_WAVES) g_inst_its[b] += it_total;
#endif
    if (t == 0) si[SQ_IPMIT] = it_total;
    if (!conv) {  // keep the previous step (Q6)
        if (t == 0) si[SQ_QPSTAT] = diverged ? MPCC_QP_PrimalInfeasible : MPCC_QP_MaxIterReached;
        return tail_req;
    }
    if (t == 0) si[SQ_QPSTAT] = 0;
    gdouble* stp = (gdouble*)(d.step + (size_t)b * NS * 17);
    for (int k = 0; k <= N; k++) {
        const double zx = *ws(k, F_ZX) + alpha * *ws(k, F_DX);
        const double zv = *ws(k, F_ZV) + alpha * *ws(k, F_DV);  // lanes < 8
        if (t < 9) stp[k * 17 + t] = zx;
        if (t < 8) stp[k * 17 + 9 + t] = (k < N) ? zv : 0.0;
    }
    return tail_req;
}

#ifdef MPCC_IPM_PROF
extern "C" int mpcc_debug_wave_times(unsigned long long* out, int n) {
    if (n > PROF_WAVES) n = PROF_WAVES;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), sizeof(unsigned long long) * n) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + n, HIP_SYMBOL(g_wave_t), sizeof(unsigned long long) * n,
                            sizeof(unsigned long long) * PROF_WAVES) != hipSuccess) return -1;
    return n;
}
extern "C" int mpcc_debug_tail_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tail_prof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tail_prof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
extern "C" int mpcc_debug_inst_ipm_iters(int* out, int n) {  // IPM iterations of every QP of the last k_sqp launch
    if (n > 4 * PROF_WAVES) n = 4 * PROF_WAVES;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_inst_its), sizeof(int) * n) == hipSuccess ? n : -1;
}
extern "C" int mpcc_debug_solo_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solo_prof), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_solo_prof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
extern "C" int mpcc_debug_ipm_prof(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ipm_prof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ipm_prof), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif


// ------------------------------------------------------------------------------------------------
// k_sqp: the whole SQP loop of solveOCP (osqp_interface.cpp:431-574) per instance, one 16-lane group
// per instance: QP solve, filter line-search trial (lane = stage), filter decision, step and
// termination, then the next iteration's QP assembly (lane = stage) — without leaving the kernel.
// An instance that needs another SQP iteration starts it as soon as its own line search is done, so
// its second QP overlaps the first QPs of the rest of the batch instead of running as a separate,
// nearly empty launch.  The first iteration's QP records come from k_setqp.  Arithmetic is that of
// k_setqp / k_trial / k_accept / k_apply (dev_sqp.h, no FP contraction).
// ------------------------------------------------------------------------------------------------
// Phases of k_sqp as separate (non-inlined) functions: each has its own register allocation, so the
// QP assembly and trial code does not add live ranges to the register-resident interior point.
// the per-stage phases of k_sqp: lane t of st lanes works on stages t, t + st, ... (st = 16, a solo wave: 64)
// MPCC_TRIAL_INLINE (default 1): the line-search trial inlined into the wave loop.  As a call it saved and restored
// 256 callee-saved registers through scratch around every trial (its first loads queued behind those stores):
// get_alpha 5.5% -> 3.7% of k_sqp, configs[1] 1.650-1.653M -> 1.663-1.672M (profiles/r05ab_ab_trial_inline.log).
// MPCC_SETQP_INLINE: the same for the second and later QP assemblies.
#ifndef MPCC_TRIAL_INLINE
#define MPCC_TRIAL_INLINE 1
#endif
#ifndef MPCC_SETQP_INLINE
#define MPCC_SETQP_INLINE 0
#endif
#if MPCC_SETQP_INLINE
__device__ __forceinline__ void sqp_setqp_phase(const DevConst& c, const DevBuffers& d, int b, int t, int st,
#else
__device__ __attribute__((noinline)) void sqp_setqp_phase(const DevConst& c, const DevBuffers& d, int b, int t, int st,
#endif
                                                          const double* __restrict__ ucur) {
    const int N = c.N, NS = N + 1;
    const SplineView sp = spl_of(c.spl, b);
    const double* gb = d.guess + (size_t)b * NS * 17;
    for (int k = t; k <= N; k += st)
        setqp_stage(c, sp, gb, RecView{d.rec + (size_t)b * NS + k, c.S}, k, ucur, d.qs + ((size_t)b * NS + k) * QS);
}
#if MPCC_TRIAL_INLINE
__device__ __forceinline__ void sqp_trial_phase(const DevConst& c, const DevBuffers& d, int b, int t, int st,
#else
__device__ __attribute__((noinline)) void sqp_trial_phase(const DevConst& c, const DevBuffers& d, int b, int t, int st,
#endif
                                                          const double* __restrict__ ucur, double alpha, bool keep) {
    const int N = c.N, NS = N + 1;
    for (int k = t; k <= N; k += st) {
        double out[4];
        trial_stage(c, d, b, k, alpha, ucur, out);
        if (keep) {
            double* tr = d.trial + ((size_t)b * NS + k) * 4;
            for (int i = 0; i < 4; i++) tr[i] = out[i];
        }
    }
}
__device__ __attribute__((noinline)) void sqp_soc_phase(const DevConst& c, const DevBuffers& d, int b, int t, int st,
                                                        const double* __restrict__ ucur) {
    const int N = c.N, NS = N + 1;
    const SplineView sp = spl_of(c.spl, b);
    const size_t o = (size_t)b * NS * 17;
    for (int k = t; k <= N; k += st)
        soc_stage(c, sp, d.guess + o, d.step + o, RecView{d.rec + (size_t)b * NS + k, c.S}, k, ucur,
                  d.qs + ((size_t)b * NS + k) * QS);
}
// returns true when the wave's last running instance is handed to tail mode (ipm_tail_solve, called by the kernel:
// a call inside this function would change the interior point's register allocation)
template <int NPM>
__device__ __attribute__((noinline)) bool sqp_ipm_phase(const DevConst& c, const DevBuffers& d, double* smem) {
    return ipm_group<NPM>(c, d, smem);
}
// Solo blocks (k_sqp_solo): wave 0 runs a cold-started instance's SQP, wave 1 helps in each of its
// tail-mode QP solves.  The helper waits at the block barrier for wave 0's post: 1 = a solve (ipm_tail_solve on all
// SB_GB groups), 0 = the end.  Wave 0 meets the block's barriers only at its posts and inside ipm_tail_solve.
template <int NPM>
__device__ __attribute__((noinline)) void solo_helper(const DevConst& c, const DevBuffers& d, double* smem) {
    while (true) {
        __syncthreads();
        const double cmd = smem[sb_cmd<NPM>()];
        if (cmd == 0.0) break;
        ipm_tail_solve<NPM, SB_GB>(c, d, smem);
    }
}
template <int NPM>
__device__ __forceinline__ void solo_post(double* smem, double cmd) {
    if (threadIdx.x == 0) smem[sb_cmd<NPM>()] = cmd;
    __syncthreads();
}
template <int NPM, bool SB = false>
__device__ __forceinline__ void sqp_qp_solve(const DevConst& c, const DevBuffers& d, double* smem) {
    if (sqp_ipm_phase<NPM>(c, d, smem)) {
        if constexpr (NPM <= 2 || (MPCC_WIDE_TAIL && NPM >= 9)) {
            if constexpr (SB) {
                solo_post<NPM>(smem, 1.0);
                ipm_tail_solve<NPM, SB_GB>(c, d, smem);
            } else {
                ipm_tail_solve<NPM>(c, d, smem);
            }
        }
    }
}
// wave 0 of a solo block: the ordering of the SQP phases within the wave (some lanes' global stores before other
// lanes' loads) without the barrier of __syncthreads, which the helper wave does not meet there
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// k_ipm: one QP solve per active instance (the staged SQP loop of run_batch and the debug QP entry); its arguments
// read in place like k_sqp's (kernels.h kernarg_const)
template <int NPM>
__global__ void __launch_bounds__(64) k_ipm(DevConst, DevBuffers) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    sqp_qp_solve<NPM>(kernarg_const(), kernarg_buffers(), smem);
}

#ifdef MPCC_SOLO_TS  // timeline of the solo blocks (tools/solo_ts.py): s_memrealtime (100 MHz) per block at entry, after the
                     // first QP records, and after the QP records / QP solve / step of SQP iterations 0 and 1
__device__ unsigned long long g_solo_ts[64 * 8];
#define SOLO_TS(i) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_solo_ts[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
}  // namespace mpcc
extern "C" int mpcc_debug_solo_ts(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mpcc::g_solo_ts), sizeof(unsigned long long) * 64 * 8) == hipSuccess ? 0 : -1;
}
namespace mpcc {
#else
#define SOLO_TS(i) do { } while (0)
#endif
// the SQP loop of one wave (k_sqp: each wave; k_sqp_solo: wave 0 of a solo block, SB)
template <int NPM, bool SB>
__device__ __forceinline__ void sqp_waves(const DevConst& c, const DevBuffers& d, const double* __restrict__ ucur_all,
                                          double* smem) {
    auto bar = [] {
        if constexpr (SB) wave_sync();
        else __syncthreads();
    };
    const int t = threadIdx.x & 15;
    const int b = inst_of(c, d, blockIdx.x * IPW + (threadIdx.x >> 4));
    const bool valid = b < c.Bn;
    const int N = c.N, NS = N + 1;
    const int bb = valid ? b : 0;
    int32_t* si = d.sqi + (size_t)bb * SQI;
    const double* ucur = ucur_all + 8 * bb;
    // a wave holding one instance (a solo wave, or the batch's last) runs that instance's per-stage phases (QP
    // assembly, line-search trial, correction bounds) on all 64 lanes, one stage per lane
    const unsigned long long lead = __ballot(valid && t == 0);
    const bool one = __popcll(lead) == 1;
    const int pb = one ? __shfl(b, __ffsll((long long)lead) - 1) : b;  // the instance of this lane's stage phases
    const int pt = one ? (int)threadIdx.x : t, pst = one ? 64 : 16;
    const int pbb = pb < c.Bn ? pb : 0;
    const int32_t* psi = d.sqi + (size_t)pbb * SQI;
    const double* pucur = ucur_all + 8 * pbb;
#ifdef MPCC_IPM_PROF
    if (threadIdx.x == 0 && blockIdx.x < PROF_WAVES) g_wave_t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    if (t == 0 && b < 4 * PROF_WAVES) g_inst_its[b] = 0;
    const bool solo_w = __popcll(__ballot(valid && t == 0)) == 1;
    long long sp_t = clock64(), sp_acc[5] = {0, 0, 0, 0, 0};
    int sp_it = 0;
#define SPMARK(i) do { const long long t_ = clock64(); sp_acc[i] += t_ - sp_t; sp_t = t_; } while (0)
#else
#define SPMARK(i) do { } while (0)
#endif
    PhaseClock ph(d.phase_cyc);  // the ComputeTime split (mpcc_timing): set_qp / solve_qp / get_alpha / step
    for (int it = 0; it < c.p.max_iter; it++) {
        bool act = valid && si[SQ_ACTIVE] != 0;
        if (__ballot(act) == 0) break;
#ifdef MPCC_IPM_PROF
        sp_it++;
#endif
        SPMARK(4);
        ph.mark(PH_STEP);
        if (it > 0) {
            if (pb < c.Bn && psi[SQ_ACTIVE] != 0) sqp_setqp_phase(c, d, pb, pt, pst, pucur);
            bar();
        }
        SPMARK(0);
        ph.mark(PH_SETQP);
        if constexpr (SB) if (it < 2) SOLO_TS(2 + 3 * it);
        sqp_qp_solve<NPM, SB>(c, d, smem);
        bar();
        if constexpr (SB) if (it < 2) SOLO_TS(3 + 3 * it);
        SPMARK(1);
        if (c.p.do_SOC) {  // SecondOrderCorrection (osqp_interface.cpp:506-535): same P, q, A, shifted bounds
            if (pb < c.Bn && psi[SQ_ACTIVE] != 0) sqp_soc_phase(c, d, pb, pt, pst, pucur);
            bar();
            sqp_qp_solve<NPM, SB>(c, d, smem);  // a failed correction keeps the step (Q6)
            bar();
        }
        ph.mark(PH_SOLVE);
        act = valid && si[SQ_ACTIVE] != 0;
        const bool pact = pb < c.Bn && psi[SQ_ACTIVE] != 0;
        if (pact) sqp_trial_phase(c, d, pb, pt, pst, pucur, 1.0, true);
        bar();
        SPMARK(2);
        if (act && t == 0) accept_instance(c, d, b);
        bar();
        SPMARK(3);
        if (pact && c.faithful_dead_trials && psi[SQ_REJECT]) {  // discarded trials (Q5), evaluated for timing fidelity
            double alpha = 1.0;
            for (int l = 1; l < c.p.line_search_max_iter; l++) {
                alpha *= c.p.line_search_tau;
                sqp_trial_phase(c, d, pb, pt, pst, pucur, alpha, false);
            }
        }
        ph.mark(PH_ALPHA);
        double nrm = 0.0;
        if (act) {
            const double alpha = d.sqd[(size_t)b * SQ + SQ_ALPHA];
            nrm = apply_range<8>(c, d, b, t, 16, alpha);
        }
        nrm = g_max(nrm);  // DPP: whole row active
        if (act && t == 0) finish_iteration(c, d, b, nrm);
        bar();
        if constexpr (SB) if (it < 2) SOLO_TS(4 + 3 * it);
    }
    ph.mark(PH_STEP);
    ph.flush(threadIdx.x == 0);
    if constexpr (SB) solo_post<NPM>(smem, 0.0);  // the helper leaves
#ifdef MPCC_IPM_PROF
    SPMARK(4);
    if (threadIdx.x == 0 && blockIdx.x < PROF_WAVES) g_wave_t[PROF_WAVES + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    if (solo_w && threadIdx.x == 0) {
        for (int i = 0; i < 5; i++) atomicAdd(&g_solo_prof[i], (unsigned long long)sp_acc[i]);
        atomicAdd(&g_solo_prof[5], 1ull);
        atomicAdd(&g_solo_prof[6], (unsigned long long)sp_it);
    }
#endif
#undef SPMARK
}

// k_sqp: every wave its slots' instances.  With solo blocks (c.solo 2) the first NSOLO waves (k_order's solo waves)
// are k_sqp_solo's and return at once.
template <int NPM>
__global__ void __launch_bounds__(64) k_sqp(DevConst, DevBuffers, const double* __restrict__ ucur_all) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const DevConst& c = kernarg_const();     // the arguments in place (kernels.h kernarg_const)
    const DevBuffers& d = kernarg_buffers();
    if (c.solo == 2 && blockIdx.x < NSOLO) return;
    sqp_waves<NPM, false>(c, d, ucur_all, smem);
}
// k_sqp_solo (c.solo 2, launched beside k_sqp on a second stream): block r holds solo wave r's cold-started instance
// (k_order's slot 4 r); wave 0 runs its SQP, wave 1 joins its tail-mode QP solves (solo_helper).  A block without a
// cold instance returns at once.
// Early solo blocks (engine.cpp run_batch, c.subset 1): the block builds its instance's first QP records itself
// before the SQP loop (k_setqp's setqp_stage, the same arithmetic: fp-contract off as in kernels.hip), on the two SIMDs
// it holds, instead of in a launch that waits for SIMDs the other instances' launches occupy.  The records come from
// k_records over the solo instances (subset 1) before this launch.  Both waves take part.
__device__ __attribute__((noinline)) void solo_prep(const DevConst& c, const DevBuffers& d, int b,
                                                    const double* __restrict__ ucur_all) {
    sqp_setqp_phase(c, d, b, (int)threadIdx.x, (int)blockDim.x, ucur_all + NU * b);
    __syncthreads();  // the QP records before the SQP loop
}
template <int NPM>
__global__ void __launch_bounds__(64 * SB_WAVES) k_sqp_solo(DevConst, DevBuffers, const double* __restrict__ ucur_all) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const DevConst& c = kernarg_const();
    const DevBuffers& d = kernarg_buffers();
    if (d.order[blockIdx.x * IPW] < 0) return;
    SOLO_TS(0);
    if (c.subset == 1) solo_prep(c, d, d.order[blockIdx.x * IPW], ucur_all);
    SOLO_TS(1);
    if (threadIdx.x >= 64) {
        solo_helper<NPM>(c, d, smem);
        return;
    }
    sqp_waves<NPM, true>(c, d, ucur_all, smem);
}

}  // namespace mpcc
// QP solves finished in tail mode (ipm_tail.h) since the last reset, over all engines of the process
extern "C" int mpcc_debug_tail_solves(long long* out, int reset) {
    unsigned long long v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(mpcc::g_tail_solves), sizeof v) != hipSuccess) return -1;
    if (out) *out = (long long)v;
    if (reset) {
        const unsigned long long z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(mpcc::g_tail_solves), &z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
namespace mpcc {

template <int NPM>
static void launch_ipm_t(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_ipm<NPM>, dim3((c.Bn + IPW - 1) / IPW), dim3(64), ipm_lds_bytes(c.N, NPM), s, c, d);
}
template <int NPM>
static void launch_sqp_t(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s) {
    const int waves = c.solo ? order_slots(c.Bn) / IPW : (c.Bn + IPW - 1) / IPW;
    hipLaunchKernelGGL(k_sqp<NPM>, dim3(waves), dim3(64), ipm_lds_bytes(c.N, NPM), s, c, d, u_cur);
}
template <int NPM>
static void launch_sqp_solo_t(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s) {
    hipLaunchKernelGGL(k_sqp_solo<NPM>, dim3(NSOLO), dim3(64 * SB_WAVES), SB_WAVES * ipm_lds_bytes(c.N, NPM), s, c, d,
                       u_cur);
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
bool launch_sqp_solo(const DevConst& c, const DevBuffers& d, const double* u_cur, int npmax, hipStream_t s) {
    switch (npmax) {
        case 0: launch_sqp_solo_t<0>(c, d, u_cur, s); return true;
        case 1: launch_sqp_solo_t<1>(c, d, u_cur, s); return true;
        case 2: launch_sqp_solo_t<2>(c, d, u_cur, s); return true;
#if MPCC_WIDE_TAIL
        case 9: launch_sqp_solo_t<9>(c, d, u_cur, s); return true;
        case 10: launch_sqp_solo_t<10>(c, d, u_cur, s); return true;
        case 11: launch_sqp_solo_t<11>(c, d, u_cur, s); return true;
#endif
        default: return false;  // tail mode (and so solo blocks) exists for these variants only
    }
}
void launch_sqp(const DevConst& c, const DevBuffers& d, const double* u_cur, int npmax, hipStream_t s) {
    switch (npmax) {
        case 0: launch_sqp_t<0>(c, d, u_cur, s); break;
        case 1: launch_sqp_t<1>(c, d, u_cur, s); break;
        case 2: launch_sqp_t<2>(c, d, u_cur, s); break;
        case 9: launch_sqp_t<9>(c, d, u_cur, s); break;
        case 10: launch_sqp_t<10>(c, d, u_cur, s); break;
        default: launch_sqp_t<11>(c, d, u_cur, s); break;
    }
}

}  // namespace mpcc
