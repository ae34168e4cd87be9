// ipm_tail.h — tail mode of the 16-lane interior point (included by ipm.hip inside namespace mpcc, after its
// stage helpers).  DESIGN.md §3.5.
//
// A k_sqp launch lasts as long as its slowest wave, and a wave as long as its slowest instance: at configs[1] the
// bulk of a 2048-instance launch is done after ~1.9 ms while 1-5 waves with a cold-started instance (two QPs,
// 16-17 IPM iterations) run on alone to ~3 ms (tools/wave_times.py, profiles/r04a_wave_times.json).  Such a wave
// has three idle 16-lane groups.  Tail mode gives them to the last instance: the remaining IPM iterations of the
// QP run with all four groups on the one instance, each sweep over the horizon in blocks of four stages:
//   A  group g works on stage kb -/+ g: its stage loads and everything of the stage that does not depend on the
//      sweep's recursion (the lazy update, slot weights and coefficients, gradients, the P-independent parts of
//      F, Gm and Hb; in the light sweeps the slot algebra);
//   B  the recursion itself, stage after stage, redundantly on all four groups (P_k from P_{k+1} through chol(F)
//      and U; the forward rollout x~_{k+1}; the backward costate p_k);
//   C  again four stages at once: what needs the recursion's output (K, F^-1, the slot steps and bounds);
//   D  the order-dependent accumulations (p chain of the factorization, the mu(alpha) sums) in stage order.
// Stage data move between the phases through the wave's LDS (the ring of the light sweeps is idle in tail mode).
// Every value is computed by the same expressions as in ipm_group, in the same order; the accumulations of D run
// in stage order, so a tail-mode solve is bitwise the normal one (tests/test_tail_mode.py checks it on the GPU;
// only a tie of the fraction-to-boundary candidates within product rounding could pick the other candidate).
//
// Narrow variants (NPM <= 2: the poly slot state packed into WF_ZV) and, since round 5, the wide-poly variants
// (NPM >= 9: the workspace layout WsF, the poly slot state in its own fields, c_p^T z / dza / dz cached in the
// workspace, the poly Gram blocks of F, Gm and Hb on the matrix cores in phase A: the group transposes of ipm_group
// act on four stages of one instance here instead of four instances).

#ifndef MPCC_TAIL_P1
#define MPCC_TAIL_P1 1  // phase B's P update without the instance transposes (0: ipm_group's form)
#endif

__device__ unsigned long long g_tail_solves;  // QP solves finished in tail mode since the last reset

struct TailIO {
    int it, max_it, pending, conv, diverged, restart;
    double mu0, dz_prev, sigma_mu, mu_cur, rp_cur, alpha, mcount;
};

// LDS layout of tail mode (doubles from the wave's base): per-stage exchange slots [slot j][lane t][field],
// row strides = 2 mod 4 doubles so that the 16 lanes' 16-byte accesses fall on distinct bank groups
constexpr int TL_SA = 30;                       // factorization A -> B, D: 28 + 2 fields
constexpr int TL_A = 0;                         // 4 * 16 * TL_SA
constexpr int TL_LF = TL_A + 4 * 16 * TL_SA;    // 4 * 48: L of chol(F) (36) and its reciprocal pivots (8), per stage
constexpr int TL_U = TL_LF + 4 * 48;            // 4 * 16 * 10: U column (8)
constexpr int TL_K = TL_U + 4 * 16 * 10;        // 4 * 144: K transpose area per group (8 x 16, +16 pad); in B the P exchange
constexpr int TL_C = TL_K + 4 * 144;            // 4 * 16 * 18: K column (8) and F^-1 column (8)
constexpr int TL_END = TL_C + 4 * 16 * 18;
constexpr int TL_STATE = TL_END;                // 16: iteration state handed over by ipm_group
// light sweeps (alias the factorization's areas)
constexpr int TL_LA = 0;                        // A -> B: 14 fields, stride 18
constexpr int TL_LB = TL_LA + 4 * 16 * 18;      // B -> C: x~_k, v_k, stride 2
constexpr int TL_LC = TL_LB + 4 * 16 * 2;       // C -> D: per slot row (L, U, P): s, l, ds, dl; stride 14
constexpr int TL_LM = TL_LC + 4 * 16 * 14;      // per-group combine scratch: 64 lanes x 4
static_assert((TL_STATE + 16) * 8 <= LRING * LG(LF_CBWD) * 1024, "tail-mode LDS inside the narrow variants' ring");
static_assert((TL_LM + 64 * 4) * 8 <= LRING * LG(LF_CBWD) * 1024, "tail-mode LDS inside the narrow variants' ring");
static_assert((TL_STATE + 16) * 8 <= LRING_W * LG(WF_PD, QLINES_W) * 1024, "tail-mode LDS inside the wide variants' ring");
// The same layout for GB 16-lane groups (GB / 4 waves of one workgroup: solo blocks); GB = 4 is the
// layout above.  Phase B's P exchange uses the K area of the wave's first group.
template <int GB>
struct TailLayout {
    static constexpr int A = 0, LF = A + GB * 16 * TL_SA, U = LF + GB * 48, K = U + GB * 16 * 10, C = K + GB * 144;
    static constexpr int END = C + GB * 16 * 18;
    static constexpr int LA = 0, LB = LA + GB * 16 * 18, LC = LB + GB * 16 * 2, LM = LC + GB * 16 * 14;
    static constexpr int LEND = LM + GB * 16 * 4;
    static constexpr int SIZE = END > LEND ? END : LEND;
};
static_assert(TailLayout<4>::END == TL_END && TailLayout<4>::LM == TL_LM && TailLayout<4>::K == TL_K, "GB = 4 layout");
// a solo block: SB_WAVES waves on one instance; the command word (wave 0 -> helper waves) is the last double of the
// block's ring slices, past the SB_GB-group layout
#ifndef MPCC_SB_WAVES
#define MPCC_SB_WAVES 2
#endif
constexpr int SB_WAVES = MPCC_SB_WAVES, SB_GB = 4 * SB_WAVES;
// doubles of LDS per k_sqp wave of the NPM variant (ipm_wave_lds: the light sweeps' ring) and the command word's index
template <int NPM>
__host__ __device__ constexpr int sb_cmd() { return SB_WAVES * ipm_wave_lds(NPM) - 1; }
static_assert(TailLayout<SB_GB>::SIZE <= sb_cmd<0>() && TL_STATE + 16 <= sb_cmd<0>(), "solo-block LDS (narrow)");
static_assert(TailLayout<SB_GB>::SIZE <= sb_cmd<11>() && TL_STATE + 16 <= sb_cmd<11>(), "solo-block LDS (wide-poly)");

template <int NPM, int GB>
__device__ __attribute__((noinline)) void ipm_tail(const DevConst& c, const DevBuffers& d, double* smem, int b, TailIO& io) {
    static_assert(NPM <= 2 || NPM >= 9, "tail mode: narrow and wide-poly variants");
    static_assert(!(MPCC_PCN && NPM >= 1 && NPM <= 2), "tail mode does not carry the MPCC_PCN lane cache");
    static_assert(GB % 4 == 0, "whole waves");
    using L = WsF<NPM>;
    constexpr bool PACKP = L::PACKP, PCACHE = L::PCACHE, GRAM_MFMA = MPCC_GRAM_MFMA && NPM >= 9;
    using namespace dpp;
    using TLy = TailLayout<GB>;
    constexpr int NWV = GB / 4;  // waves on the instance
    constexpr int TL_A = TLy::A, TL_LF = TLy::LF, TL_U = TLy::U, TL_K = TLy::K, TL_C = TLy::C;
    constexpr int TL_LA = TLy::LA, TL_LB = TLy::LB, TL_LC = TLy::LC, TL_LM = TLy::LM;
    constexpr int NPE = NPM > 0 ? NPM : 1;
    using In = StageIn<NPE>;
    const int lane = threadIdx.x & 63;
    const int wv = NWV > 1 ? (int)(threadIdx.x >> 6) : 0;
    const int g = lane >> 4;      // group in the wave (phase B's MFMA operand selects)
    const int G = wv * 4 + g;     // group on the instance: its stage in phases A and C
    const int t = lane & 15;
    const int N = c.N;
    const int NS = N + 1;

    const gdouble* QSb = (const gdouble*)(d.qs + (size_t)MPCC_BCHK(c.bchk, b, c.Bn, BC_INSTANCE) * NS * QS);
    gdouble* WSb = (gdouble*)(d.is + (size_t)b * NS * IS);
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
    auto lds = [&](int off) -> double* { return smem + MPCC_BCHK(c.bchk, off, TLy::SIZE, BC_LDS); };

    // ---- model constants of this lane (as ipm_group)
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
    auto hb_mp = [&](double v, int a, const double (&Pc)[16], const double (&Pc7)[9]) -> double {  // as ipm_group
        v = fma(mdiag[a] * mt, Pc[a], v);
        if (t == 8) v = fma(mdiag[a] * m78, Pc7[a], v);
        if (a == 8) v = fma(m78 * mt, Pc[7], v);
        if (a == 8 && t == 8) v = fma(m78 * m78, Pc7[7], v);
        return v;
    };
    const bool own = G == 0;  // the group that stores what all groups computed redundantly (phases B, D)

    // ---- stage loaders (ipm_group's)
    auto load_common = [&](int k, In& o) {
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
        o.sL = *ws(k, L::SL); o.lL = *ws(k, L::LL); o.sU = *ws(k, L::SU); o.lU = *ws(k, L::LU);
        o.zx = *ws(k, L::ZX);
        if constexpr (PCACHE) { o.pz = *ws(k, L::PZ); o.pca = *ws(k, L::PA); o.pcd = *ws(k, L::PD); }
        const double zraw = *ws(k, L::ZV);
        if constexpr (PACKP) {
            o.sP = from_up<8>(zraw);
            o.lP = from_up<12>(zraw);
            o.zv = (t < 8) ? zraw : 0.0;
        } else {
            o.sP = *ws(k, L::SP); o.lP = *ws(k, L::LP);
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
        const double x0 = *ws(k, L::DX), x1 = *ws(k, L::DV), x2 = *ws(k, L::AX), x3 = *ws(k, L::AV);
        o.x0 = upd ? x0 : 0.0; o.x1 = upd ? x1 : 0.0; o.x2 = upd ? x2 : 0.0; o.x3 = upd ? x3 : 0.0;
    };
    auto load_fwd = [&](int k, In& o, bool corr) {
        load_common(k, o);
#pragma unroll
        for (int m = 0; m < 8; m++) o.m[m] = *ws(k, L::KR + m);
        o.m[8] = from_up<8>(*ws(k, L::GVK));
        if (corr) {
            o.x0 = *ws(k, L::AX);
            o.x1 = *ws(k, L::AV);
        } else {
            o.x0 = o.x1 = 0.0;
        }
    };
    auto load_bwd = [&](int k, In& o) {
        load_common(k, o);
        o.x0 = *ws(k, L::AX); o.x2 = *ws(k, L::GX);
        o.x1 = *ws(k, L::AV);
        const double gvk = *ws(k, L::GVK);
        o.x3 = (t < 8) ? gvk : 0.0;
#pragma unroll
        for (int m = 0; m < 8; m++) o.m[m] = *ws(k, L::KR + m);
#pragma unroll
        for (int m = 0; m < 4; m++) o.m[8 + m] = *ws(k, L::FI + m);
    };
    // DPP with the whole row active: called unconditionally, the store itself under the caller's condition
    auto store_slots = [&](bool st, int k, double sL, double lL, double sU, double lU, double sP, double lP, double zx,
                           double zv) {
        if constexpr (PACKP) {
            const double s8 = from_down<8>(sP), l12 = from_down<12>(lP);
            zv = (t < 8) ? zv : ((t < 12) ? s8 : l12);
        }
        if (!st) return;
        *ws(k, L::SL) = sL; *ws(k, L::LL) = lL; *ws(k, L::SU) = sU; *ws(k, L::LU) = lU;
        if constexpr (!PACKP) { *ws(k, L::SP) = sP; *ws(k, L::LP) = lP; }
        *ws(k, L::ZX) = zx;
        *ws(k, L::ZV) = zv;
    };

    // ---- stage-local helpers (ipm_group's)
    auto row_active = [&](int k, double bnd) { return (rowY ? (k >= 1) : (k < N)) && fabs(bnd) < BIG; };
    auto row_cz = [&](int k, double x, double v) -> double {
        const double vj = from_down<9>(v);
        if (rowY) return x;
        return (k == 0) ? vj : vj - x;
    };
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
    auto assemble_grad = [&](const In& in, int k, double g0x, double g0v, double dvr, double cP, double& gx, double& gv) {
        gx = g0x;
        if (t < 9) gx += dvr;
        else if (k >= 1) gx -= dvr;
        gv = g0v;
        const double dv_up = from_up<9>(dvr);
        if (t < 7 && k < N) gv += dv_up;
#pragma unroll
        for (int p = 0; p < NPM; p++) {
            const double cp = bcn(cP, p);
            const bool live = (double)p < in.np && k < N;
            if (live) {
                gx += cp * in.pa[p];
                gv += cp * in.pb[p];
            }
        }
    };
    // forward step of the rollout from the K row halves + kff (m[0..8])
    auto fwd_step = [&](const double* m, double xt, double& v, double& xn) {
        double part = 0.0;
        double xb[16];
#pragma unroll
        for (int q = 0; q < 16; q++) xb[q] = bcn(xt, q);
#pragma unroll
        for (int q = 0; q < 8; q++) part += m[q] * ((t < 8) ? xb[q] : xb[8 + q]);
        const double xb8 = xb[8];
        v = part + from_up<8>(part) + m[8];
        const double v7 = from_down<1>(v);
        const double vj = from_down<9>(v);
        if (t < 7) xn = fma2(mt, xt, gt, v);
        else if (t == 7) xn = fma(g77, v, fma2(m77, xt, m78, xb8));
        else if (t == 8) xn = fma2(m88, xt, g87, v7);
        else xn = vj;
    };
    auto sync = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    // between phases: the wave's LDS order, or with more than one wave a workgroup barrier (its fences also order
    // one wave's workspace stores before the other's loads)
    auto bsync = [] {
        if constexpr (NWV == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        else __syncthreads();
    };
    // slot j of an exchange area: lane t's fields at base + (j * 16 + t) * stride
    auto xs = [&](int base, int j, int stride) -> double* { return lds(base + (j * 16 + t) * stride); };
    // max of per-group values over the GB groups (every lane gets the max over the groups of its t)
    auto maxG = [&](double v) {
        sync();
        *lds(TL_LM + wv * 64 + lane) = v;
        bsync();
        double o[GB];
#pragma unroll
        for (int q = 0; q < GB; q++) o[q] = *lds(TL_LM + q * 16 + t);
        bsync();
        double m = o[0];
#pragma unroll
        for (int q = 1; q < GB; q++) m = fmax(m, o[q]);
        return m;
    };

#ifdef MPCC_IPM_PROF
    long long tprof[16] = {0};
    long long tprof_t = clock64();
    const int it_in = io.it;
#endif
    int it = io.it;
    const int max_it = io.max_it;
    double mu0 = io.mu0, dz_prev = io.dz_prev, sigma_mu = io.sigma_mu, mu_cur = io.mu_cur, rp_cur = io.rp_cur;
    double alpha = io.alpha;
    double mcount = io.mcount;
    bool pending = io.pending != 0, conv = false, diverged = false;
    if (io.restart) {
        // restart from the unit start point (attempt 1 of ipm_group): dynamics rollout with v = 0, s = max(-g, 1),
        // lambda = 1, on all groups (the stores by one)
        In cur, nxt;
        double y = 0.0, bk = 0, bkn = 0;
        mcount = 0.0;
        load_common(0, cur);
        bk = (N > 0 && t < 9) ? QSb[QS_B + t] : 0.0;
        for (int k = 0; k <= N; k++) {
            if (k < N) {
                load_common(k + 1, nxt);
                bkn = (k + 1 < N && t < 9) ? QSb[(size_t)(k + 1) * QS + QS_B + t] : 0.0;
            }
            const double yx = rowY ? y : 0.0;
            const double cz = row_cz(k, yx, 0.0);
            const double pcz = poly_cz(cur, k, yx, 0.0);
            if constexpr (PCACHE) { if (own) *ws(k, L::PZ) = pcz; }
            const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
            double sL = 1, lL = 0, sU = 1, lU = 0, sP = 1, lP = 0;
            if (aL) { sL = fmax(-(sgnL * cz - sgnL * cur.lb), 1.0); lL = 1.0; }
            if (aU) { sU = fmax(-(sgnU * cz - sgnU * cur.ub), 1.0); lU = 1.0; }
            if (aP) { sP = fmax(-(sgnU * pcz - sgnU * cur.pub), 1.0); lP = 1.0; }
            mcount += (aL ? 1.0 : 0.0) + (aU ? 1.0 : 0.0) + (aP ? 1.0 : 0.0);
            store_slots(own, k, sL, lL, sU, lU, sP, lP, yx, 0.0);
            const double y8 = from_up<1>(y);
            const double yn = (t == 7) ? fma2(m77, y, m78, y8) + bk : fma(mt, y, bk);
            y = (t < 9) ? yn : 0.0;
            cur = nxt;
            bk = bkn;
        }
        mcount = g_sum(mcount);
        if constexpr (NWV > 1) bsync();  // the start point's stores before any group's loads
    }

    while (true) {
        // ================= factorization sweep k = N..0 (blocks of 4 stages: kb, kb - 1, kb - 2, kb - 3)
        double Pc[16];
        double pv = 0.0;
        bool chol_ok = true;
#pragma unroll
        for (int a = 0; a < 16; a++) Pc[a] = 0.0;
        for (int kb = N; kb >= 0; kb -= GB) {
            // ---- A: group g, stage kb - g: lazy update, slots, gradient, P-independent parts of F, Gm, Hb
            {
                const int kg = kb - G;
                const bool vA = kg >= 0;
                const int k = vA ? kg : 0;
                In cur;
                load_factor(k, cur, pending);
                const double lb = cur.lb, ub = cur.ub;
                const double* Qr = cur.m;
                const double qt = cur.m[9], Rt = cur.m[10], rt = cur.m[11];
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
                    store_slots(vA, k, sL, lL, sU, lU, sP, lP, zx, zv);
                }
                const double cz = row_cz(k, zx, zv);
                const double pcz = poly_cz(cur, k, zx, zv);
                if constexpr (PCACHE) { if (vA) *ws(k, L::PZ) = pcz; }
                double WL = 0, WU = 0, WP = 0, cL = 0, cU = 0, cP = 0;
                if (aL) { const double rp = slot_rp(sgnL, cz, lb, sL); const double ri = rcp(sL); WL = lL * ri; cL = slot_coef(ri, lL, rp, sL * lL); }
                if (aU) { const double rp = slot_rp(sgnU, cz, ub, sU); const double ri = rcp(sU); WU = lU * ri; cU = slot_coef(ri, lU, rp, sU * lU); }
                if (aP) { const double rp = slot_rp(sgnU, pcz, cur.pub, sP); const double ri = rcp(sP); WP = lP * ri; cP = slot_coef(ri, lP, rp, sP * lP); }
                const double wd = WL + WU;
                const double dvr = sgnL * cL + sgnU * cU;
                double g0x, g0v = 0.0;
                {
                    double zb[9];
#pragma unroll
                    for (int m = 0; m < 9; m++) zb[m] = bcn(zx, m);
                    const double vj = from_down<9>(zv);
                    const double wj = from_up<9>(zx);
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
                if (vA) *ws(k, L::GX) = g0x;
                double gx, gv;
                assemble_grad(cur, k, g0x, g0v, dvr, cP, gx, gv);
                const double wdv = from_up<9>(wd);
                double hF[8], hG[8], hb9[9];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    hF[i] = (i == t) ? Rt + ((t < 7) ? wdv : 0.0) : 0.0;
                    hG[i] = 0.0;
                }
                double dq[7];  // Gram: D[8 + a][8 + t], the poly terms of Hb's q block
                if constexpr (GRAM_MFMA) {
                    // ipm_group's Gram MFMA (D = sum_p w_p r_p r_p^T, r_p = [bv_p, 0, a_p, 0]), the wave's four groups
                    // on their four stages: the same operands per group, so bitwise the normal path's blocks
                    constexpr int KS = (NPM + 3) / 4;
                    double xs_[KS][4][1], as_[KS][4][1];
#pragma unroll
                    for (int q = 0; q < KS; q++)
#pragma unroll
                        for (int gg = 0; gg < 4; gg++) {
                            const int pp = 4 * q + gg;
                            double x = 0.0, w = 0.0;
                            if (pp < NPM) {
                                const double a8 = from_down<8>(cur.pa[pp]);  // lane 8 + i <- a_p[i]
                                x = (t < 8) ? cur.pb[pp] : a8;
                                const bool live = (double)pp < cur.np && k < N;
                                const double wp = bcn(WP, pp);
                                w = live ? wp : 0.0;
                            }
                            xs_[q][gg][0] = x;
                            as_[q][gg][0] = w * x;
                        }
#pragma unroll
                    for (int q = 0; q < KS; q++) {
                        group_transpose(xs_[q]);
                        group_transpose(as_[q]);
                    }
                    double dg[4][4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int q = 0; q < KS; q++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(as_[q][j][0], xs_[q][j][0], acc, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 4; r++) dg[j][r] = acc[r];
                    }
                    group_transpose(dg);
                    const bool q7 = t < 7;
#pragma unroll
                    for (int i = 0; i < 7; i++) {
                        const double dF = dg[i & 3][i >> 2];
                        const double dG = from_up<8>(dg[i & 3][i >> 2]);
                        hF[i] += q7 ? dF : 0.0;
                        hG[i] += q7 ? dG : 0.0;
                    }
#pragma unroll
                    for (int a = 0; a < 7; a++) {
                        const double dd = from_up<8>(dg[(8 + a) & 3][(8 + a) >> 2]);
                        dq[a] = q7 ? dd : 0.0;
                    }
                } else {
                    double Wb[NPE];
#pragma unroll
                    for (int p = 0; p < NPM; p++) {
                        const bool live = (double)p < cur.np && k < N;
                        const double wp = bcn(WP, p);
                        Wb[p] = live ? wp : 0.0;
#pragma unroll
                        for (int i = 0; i < 7; i++) {
                            const double bv = bcn(cur.pb[p], i);
                            hF[i] += Wb[p] * (bv * cur.pb[p]);
                            hG[i] += Wb[p] * (bv * cur.pa[p]);
                        }
                    }
                }
                if (k == N) {
                    // terminal stage: P = Hb_N (y block; Q row t as column t) into the hb9 slot; no gains
#pragma unroll
                    for (int a = 0; a < 9; a++) {
                        double v = 0.0;
                        if (t < 9) {
                            v = Qr[a];
                            if (a == t) v += wd;
                        }
                        hb9[a] = v;
                    }
                    if (vA) {
#pragma unroll
                        for (int m = 0; m < 8; m++) *ws(k, L::KR + m) = 0.0;
                        *ws(k, L::GVK) = (t < 8) ? g0v : 0.0;
#pragma unroll
                        for (int m = 0; m < 4; m++) *ws(k, L::FI + m) = 0.0;
                    }
                } else {
                    // Hb base of rows a < 9: the q block with its poly terms (poly_hq), Q rows 7, 8 + the diagonal weight
                    double hq[7];
#pragma unroll
                    for (int a = 0; a < 7; a++) {
                        hq[a] = Qr[a];
                        if (a == t) hq[a] += wd;
                    }
                    if constexpr (GRAM_MFMA) {
#pragma unroll
                        for (int a = 0; a < 7; a++) hq[a] += dq[a];
                    } else {
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
                    }
#pragma unroll
                    for (int a = 0; a < 9; a++) {
                        double v;
                        if (a < 7) {
                            v = hq[a];
                        } else {
                            v = Qr[a];
                            if (a == t) v += wd;
                        }
                        hb9[a] = v;
                    }
                }
                const double gw = (k >= 1) ? Hct - wd : 0.0;
#ifdef MPCC_IPM_DBGF
                if (vA && k < N) { *ws(k, 35) = gx; *ws(k, 36) = gv; *ws(k, 39) = dvr; *ws(k, 40) = cP; *ws(k, 41) = wd; }
#endif
                double* o = xs(TL_A, G, TL_SA);
                double2* o2 = reinterpret_cast<double2*>(o);
                o2[0] = make_double2(gx, gv);
                o2[1] = make_double2(g0v, wd);
                o2[2] = make_double2(gw, hb9[8]);
#pragma unroll
                for (int i = 0; i < 4; i++) o2[3 + i] = make_double2(hF[2 * i], hF[2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 4; i++) o2[7 + i] = make_double2(hG[2 * i], hG[2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 4; i++) o2[11 + i] = make_double2(hb9[2 * i], hb9[2 * i + 1]);
            }
            bsync();
            TMARK(0);
            // ---- B: the P recursion, stage after stage on all groups
            for (int j = 0; j < GB; j++) {
                const int k = kb - j;
                if (k < 0) break;
                const double2* a2 = reinterpret_cast<const double2*>(xs(TL_A, j, TL_SA));
                const double2 x01 = a2[0], x23 = a2[1], x45 = a2[2];
                const double gx = x01.x, wd = x23.y, gw = x45.x;
                double hF[8], hG[8], hb9[9];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const double2 f = a2[3 + i], gg = a2[7 + i], h = a2[11 + i];
                    hF[2 * i] = f.x; hF[2 * i + 1] = f.y;
                    hG[2 * i] = gg.x; hG[2 * i + 1] = gg.y;
                    hb9[2 * i] = h.x; hb9[2 * i + 1] = h.y;
                }
                hb9[8] = x45.y;
                if (k == N) {
#pragma unroll
                    for (int a = 0; a < 16; a++) Pc[a] = (t < 9 && a < 9) ? hb9[a < 9 ? a : 0] : 0.0;
                    pv = gx;
                    continue;
                }
                // (1) Y = B~^T P (column t)
                double Y[8];
#pragma unroll
                for (int i = 0; i < 7; i++) Y[i] = gdiag[i] * Pc[i] + Pc[9 + i];
                Y[7] = fma2(g77, Pc[7], g87, Pc[8]);
                // (2) F column t, Gm column t
                double Fc[8], gm[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const double yu9 = from_up<9>(Y[i]);
                    const double yu1 = from_up<1>(Y[i]);
                    const double yd = from_down<1>(Y[i]);
                    Fc[i] = hF[i] + fma(gt, Y[i], (t < 7) ? yu9 : g87 * yu1);
                    gm[i] = hG[i] + fma(mt, Y[i], (t == 8) ? m78 * yd : 0.0);
                }
                TMARK(8);
                // (3) chol(F), U = LF^-1 Gm
                double LF[36], dinv[8];
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int jj = 0; jj <= i; jj++) LF[i * (i + 1) / 2 + jj] = bcn(Fc[i], jj);
                chol_ok = chol8(LF, dinv) && chol_ok;
                TMARK(9);
                double u[8];
#pragma unroll
                for (int i = 0; i < 8; i++) u[i] = (t < 9) ? gm[i] : ((i == j9) ? gw : 0.0);
                fwd8(LF, dinv, u);
#ifdef MPCC_IPM_DBGF2
                if (own) {
                    if (t == 0) {
                        for (int i = 0; i < 36; i++) WSb[(size_t)k * IS + 29 * 16 + i] = LF[i];
                        for (int i = 0; i < 8; i++) WSb[(size_t)k * IS + 29 * 16 + 36 + i] = dinv[i];
                    }
                    for (int i = 0; i < 8; i++) *ws(k, 32 + i) = u[i];
                }
#endif
#ifdef MPCC_IPM_DBGF
                if (own) { *ws(k, 44) = Pc[0]; *ws(k, 45) = LF[35]; *ws(k, 46) = dinv[7]; *ws(k, 47) = u[0]; *ws(k, 49) = Y[0]; *ws(k, 50) = Fc[0]; }
#endif
                // hand L, its pivots and U to phase C
                if (lane == 0 && wv == 0) {
                    double2* lf = reinterpret_cast<double2*>(lds(TL_LF + j * 48));
#pragma unroll
                    for (int q = 0; q < 18; q++) lf[q] = make_double2(LF[2 * q], LF[2 * q + 1]);
#pragma unroll
                    for (int q = 0; q < 4; q++) lf[18 + q] = make_double2(dinv[2 * q], dinv[2 * q + 1]);
                }
                {
                    double2* uo = reinterpret_cast<double2*>(xs(TL_U, j, 10));
#pragma unroll
                    for (int q = 0; q < 4; q++) uo[q] = make_double2(u[2 * q], u[2 * q + 1]);
                }
                TMARK(10);
                // (4) Hb column t and P = Hb - U^T U (column t), as ipm_group
                double hb[16];
                {
                    double Pc7[9];
#pragma unroll
                    for (int a = 0; a < 9; a++) Pc7[a] = from_down<1>(Pc[a]);
#pragma unroll
                    for (int a = 0; a < 16; a++) {
                        double v = 0.0;
                        if (a < 9) {
                            if (t < 9) {
                                v = hb9[a];
                                v = hb_mp(v, a, Pc, Pc7);
                            }
                        } else if (a == t) {
                            v = wd;
                        }
                        hb[a] = v;
                    }
                }
                TMARK(11);
                if (k > 0) {
#if MPCC_TAIL_P1
                    // One instance on all four groups: the operands of its two MFMAs are already in every lane (lane
                    // (g, t) holds U[g][t], U[4 + g][t] and Hb[g + 4r][t]: selects by g instead of ipm_group's
                    // transposes between instances), and the products P[g + 4r][t] go back to the column layout
                    // (every group: P[a][t]) through LDS.  Same MFMAs on the same operands: bitwise ipm_group's P.
                    double ua = u[0], ub = u[4];
                    d4 acc = {hb[0], hb[4], hb[8], hb[12]};
#pragma unroll
                    for (int q = 1; q < 4; q++)
                        if (g == q) {
                            ua = u[q];
                            ub = u[4 + q];
                            acc = d4{hb[q], hb[q + 4], hb[q + 8], hb[q + 12]};
                        }
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ua, ua, acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ub, ub, acc, 0, 0, 0);
                    double* Sp = lds(TL_K + wv * 576 + t * 18);  // row t: P[0..15][t] (stride 18: conflict-free, 16-byte aligned)
#pragma unroll
                    for (int r = 0; r < 4; r++) Sp[g + 4 * r] = acc[r];
                    sync();
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const double2 v = reinterpret_cast<const double2*>(Sp)[q];
                        Pc[2 * q] = v.x;
                        Pc[2 * q + 1] = v.y;
                    }
                    sync();
#else
                    double x[4][4], ua[4][1], ub[4][1];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
#pragma unroll
                        for (int r = 0; r < 4; r++) x[q][r] = hb[q + 4 * r];
                        ua[q][0] = u[q];
                        ub[q][0] = u[4 + q];
                    }
                    group_transpose(x);
                    group_transpose(ua);
                    group_transpose(ub);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        d4 acc = {x[q][0], x[q][1], x[q][2], x[q][3]};
                        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ua[q][0], ua[q][0], acc, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ub[q][0], ub[q][0], acc, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 4; r++) x[q][r] = acc[r];
                    }
                    group_transpose(x);
#pragma unroll
                    for (int q = 0; q < 4; q++)
#pragma unroll
                        for (int r = 0; r < 4; r++) Pc[q + 4 * r] = x[q][r];
#endif
                }
                TMARK(12);
            }
            bsync();
            TMARK(1);
            // ---- C: group g, stage kb - g (< N): K = -LF^-T U, F^-1 column, the gain stores
            {
                const int kg = kb - G;
                const bool vC = kg >= 0 && kg < N;
                const double2* lf = reinterpret_cast<const double2*>(lds(TL_LF + G * 48));
                double LF[36], dinv[8];
#pragma unroll
                for (int q = 0; q < 18; q++) { const double2 v = lf[q]; LF[2 * q] = v.x; LF[2 * q + 1] = v.y; }
#pragma unroll
                for (int q = 0; q < 4; q++) { const double2 v = lf[18 + q]; dinv[2 * q] = v.x; dinv[2 * q + 1] = v.y; }
                double kc[8];
                {
                    const double2* ui = reinterpret_cast<const double2*>(xs(TL_U, G, 10));
#pragma unroll
                    for (int q = 0; q < 4; q++) { const double2 v = ui[q]; kc[2 * q] = v.x; kc[2 * q + 1] = v.y; }
                }
                bwd8(LF, dinv, kc);
#pragma unroll
                for (int i = 0; i < 8; i++) kc[i] = -kc[i];
#ifdef MPCC_IPM_DBGF
                if (vC) *ws(kg, 48) = kc[0];
#endif
#ifdef MPCC_IPM_DBGF2
                if (vC) for (int i = 0; i < 8; i++) *ws(kg, 40 + i) = kc[i];
#endif
                double fi[8];
#pragma unroll
                for (int i = 0; i < 8; i++) fi[i] = (i == (t & 7)) ? 1.0 : 0.0;
                fwd8(LF, dinv, fi);
                bwd8(LF, dinv, fi);
                double* Sk = lds(TL_K + G * 144);
#pragma unroll
                for (int i = 0; i < 8; i++) Sk[i * 16 + t] = kc[i];
                {
                    double2* co = reinterpret_cast<double2*>(xs(TL_C, G, 18));
#pragma unroll
                    for (int q = 0; q < 4; q++) co[q] = make_double2(kc[2 * q], kc[2 * q + 1]);
#pragma unroll
                    for (int q = 0; q < 4; q++) co[4 + q] = make_double2(fi[2 * q], fi[2 * q + 1]);
                }
                sync();
                const int ri = t & 7, hoff = (t < 8) ? 0 : 8;
                const double2* row = reinterpret_cast<const double2*>(Sk + ri * 16 + hoff);
#pragma unroll
                for (int q2 = 0; q2 < 4; q2++) {
                    const double2 w = row[q2];
                    if (vC) {
                        *ws(kg, L::KR + 2 * q2) = w.x;
                        *ws(kg, L::KR + 2 * q2 + 1) = w.y;
                    }
                }
                if (vC) {
#pragma unroll
                    for (int m = 0; m < 4; m++) *ws(kg, L::FI + m) = (t < 8) ? fi[m] : fi[4 + m];
                }
            }
            bsync();
            TMARK(2);
            // ---- D: the p recursion, stage after stage (f = g_v + B~^T p, kff = -F^-1 f, p = g_x~ + A~^T p + K^T f)
            for (int j = 0; j < GB; j++) {
                const int k = kb - j;
                if (k < 0) break;
                if (k == N) continue;  // p_N = g_x~ (phase B)
                const double2* a2 = reinterpret_cast<const double2*>(xs(TL_A, j, TL_SA));
                const double2 x01 = a2[0], x23 = a2[1];
                const double gx = x01.x, gv = x01.y, g0v = x23.x;
                const double2* ci = reinterpret_cast<const double2*>(xs(TL_C, j, 18));
                double kc[8], fi[8];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const double2 a = ci[q], f = ci[4 + q];
                    kc[2 * q] = a.x; kc[2 * q + 1] = a.y;
                    fi[2 * q] = f.x; fi[2 * q + 1] = f.y;
                }
                const double pu9 = from_up<9>(pv), pu1 = from_up<1>(pv);
                const double fg = fma(gt, pv, gv);
                const double fv = (t < 7) ? fg + pu9 : fma(g87, pu1, fg);
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
                const double kffd = from_down<8>(kff);
                if (own) *ws(k, L::GVK) = (t < 8) ? g0v : kffd;
#ifdef MPCC_IPM_DBGF
                if (own) { *ws(k, 37) = pv; *ws(k, 38) = fv; *ws(k, 42) = pnew; *ws(k, 43) = kff; }
#endif
                pv = pnew;
            }
            bsync();
            TMARK(3);
        }
        if (!chol_ok) {
            conv = it > 0 && mu_cur < IPM_TOL_FB && rp_cur < IPM_TOL_FB;
            alpha = 0.0;
            break;
        }

        // ================= predictor forward: x~_0 = 0; recover dsa, dla; max step; mu(alpha) sums
        double S0 = 0, S1 = 0, S2 = 0;
        MinRatio amr(1.0);
        double xt = 0.0;
        // forward light sweep in blocks k = kb + j: A loads (and exports the gains), B rolls x~ out, C does the slot
        // algebra of its stage (body), D accumulates the sums in stage order (acc)
        auto fwd_sweep = [&](bool corr, auto body, auto acc) {
            for (int kb = 0; kb <= N; kb += GB) {
                const int kg = kb + G;
                const bool vA = kg <= N;
                const int k = vA ? kg : N;
                In cur;
                load_fwd(k, cur, corr);
                {
                    double* o = xs(TL_LA, G, 18);
                    double2* o2 = reinterpret_cast<double2*>(o);
#pragma unroll
                    for (int q = 0; q < 4; q++) o2[q] = make_double2(cur.m[2 * q], cur.m[2 * q + 1]);
                    o[8] = cur.m[8];
                }
                bsync();
                if (!corr) TMARK(13);
                for (int j = 0; j < GB; j++) {
                    const int kk = kb + j;
                    if (kk > N) break;
                    const double* mi = xs(TL_LA, j, 18);
                    double m[9];
#pragma unroll
                    for (int q = 0; q < 9; q++) m[q] = mi[q];
                    double v = 0.0, xn = 0.0;
                    if (kk < N) fwd_step(m, xt, v, xn);
                    const double dvv = (t < 8 && kk < N) ? v : 0.0;
                    *reinterpret_cast<double2*>(xs(TL_LB, j, 2)) = make_double2(xt, dvv);
                    xt = xn;
                }
                bsync();
                if (!corr) TMARK(14);
                {
                    const double2 xv = *reinterpret_cast<const double2*>(xs(TL_LB, G, 2));
                    double rr[14];
                    body(k, vA, cur, xv.x, xv.y, rr);
                    double2* o2 = reinterpret_cast<double2*>(xs(TL_LC, G, 14));
#pragma unroll
                    for (int q = 0; q < 7; q++) o2[q] = make_double2(rr[2 * q], rr[2 * q + 1]);
                }
                bsync();
                if (!corr) TMARK(15);
                for (int j = 0; j < GB; j++) {
                    if (kb + j > N) break;
                    const double2* r2 = reinterpret_cast<const double2*>(xs(TL_LC, j, 14));
                    double rr[14];
#pragma unroll
                    for (int q = 0; q < 7; q++) { const double2 v = r2[q]; rr[2 * q] = v.x; rr[2 * q + 1] = v.y; }
                    acc(rr);
                }
                bsync();
            }
        };
        fwd_sweep(false, [&](int k, bool vA, const In& cur, double xt_k, double dvv, double (&rr)[14]) {
            const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
            if (vA) { *ws(k, L::AX) = xt_k; *ws(k, L::AV) = dvv; }
            const double cz = row_cz(k, cur.zx, cur.zv), ca = row_cz(k, xt_k, dvv);
            const double pcz = PCACHE ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv), pca = poly_cz(cur, k, xt_k, dvv);
            if constexpr (PCACHE) { if (vA) *ws(k, L::PA) = pca; }
            MinRatio loc(1.0);  // this stage's candidates; merged in stage order in D (strict <: the sequential scan)
            auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l, int r) {
                double ds = 0.0, dl = 0.0, sv = 0.0, lv = 0.0;
                if (a && vA) {
                    const double rp = slot_rp(sgn, czz, bnd, s);
                    const SlotStep st = slot_recover(rcp(s), l, rp, sgn * caa, s * l);
                    step_bound(loc, s, l, st);
                    sv = s; lv = l; ds = st.ds; dl = st.dl;
                }
                rr[4 * r] = sv; rr[4 * r + 1] = lv; rr[4 * r + 2] = ds; rr[4 * r + 3] = dl;
            };
            rec(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL, 0);
            rec(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU, 1);
            rec(aP, sgnU, cur.pub, pcz, pca, cur.sP, cur.lP, 2);
            rr[12] = loc.num;
            rr[13] = loc.den;
        }, [&](const double (&rr)[14]) {
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const double s = rr[4 * r], l = rr[4 * r + 1], ds = rr[4 * r + 2], dl = rr[4 * r + 3];
                mu_acc(S0, S1, S2, s, l, ds, dl);
            }
            amr.add(rr[12], -rr[13]);
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
        TMARK(4);

        // ================= corrector backward: A coefficients and gradients (4 stages), B the p recursion
        {
            double pvc = 0.0;
            for (int kb = N; kb >= 0; kb -= GB) {
                {
                    const int kg = kb - G;
                    const bool vA = kg >= 0;
                    const int k = vA ? kg : 0;
                    In cur;
                    load_bwd(k, cur);
                    const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
                    const double cz = row_cz(k, cur.zx, cur.zv), ca = row_cz(k, cur.x0, cur.x1);
                    const double pcz = PCACHE ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv);
                    const double pca = PCACHE ? cur.pca : poly_cz(cur, k, cur.x0, cur.x1);
                    auto coef = [&](bool a, double sgn, double bnd, double czz, double caa, double s, double l) -> double {
                        if (!a) return 0.0;
                        const double rp = slot_rp(sgn, czz, bnd, s);
                        const double ri = rcp(s);
                        const SlotStep pa = slot_recover(ri, l, rp, sgn * caa, s * l);
                        const double rc = fma(s, l, pa.ds * pa.dl) - smu;
                        return slot_coef(ri, l, rp, rc);
                    };
                    const double cL = coef(aL, sgnL, cur.lb, cz, ca, cur.sL, cur.lL);
                    const double cU = coef(aU, sgnU, cur.ub, cz, ca, cur.sU, cur.lU);
                    const double cP = coef(aP, sgnU, cur.pub, pcz, pca, cur.sP, cur.lP);
                    const double dvr = sgnL * cL + sgnU * cU;
                    double gx, gv;
                    assemble_grad(cur, k, cur.x2, cur.x3, dvr, cP, gx, gv);
                    double2* o2 = reinterpret_cast<double2*>(xs(TL_LA, G, 18));
                    o2[0] = make_double2(gx, gv);
#pragma unroll
                    for (int q = 0; q < 6; q++) o2[1 + q] = make_double2(cur.m[2 * q], cur.m[2 * q + 1]);
                }
                bsync();
                for (int j = 0; j < GB; j++) {
                    const int k = kb - j;
                    if (k < 0) break;
                    const double2* a2 = reinterpret_cast<const double2*>(xs(TL_LA, j, 18));
                    const double2 gg = a2[0];
                    const double gx = gg.x, gv = gg.y;
                    if (k == N) {
                        pvc = gx;
                        continue;
                    }
                    double m[12];
#pragma unroll
                    for (int q = 0; q < 6; q++) { const double2 v = a2[1 + q]; m[2 * q] = v.x; m[2 * q + 1] = v.y; }
                    const double pu9 = from_up<9>(pvc), pu1 = from_up<1>(pvc);
                    const double fg = fma(gt, pvc, gv);
                    const double fv = (t < 7) ? fg + pu9 : fma(g87, pu1, fg);
                    double part = 0.0;
                    double fb[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) fb[i] = bcn(fv, i);
#pragma unroll
                    for (int q = 0; q < 4; q++) part -= m[8 + q] * ((t < 8) ? fb[q] : fb[4 + q]);
                    const double kff = part + from_up<8>(part);
                    const double kffd = from_down<8>(kff);
                    if (own && t >= 8) *ws(k, L::GVK) = kffd;
                    const double p7 = from_down<1>(pvc);
                    double gxa = gx;  // g_x~ + A~^T p
                    if (t < 9) gxa = fma(mt, pvc, gxa);
                    if (t == 8) gxa = fma(m78, p7, gxa);
                    const double f8 = rot16<8>(fv);
                    const double fh = (t < 8) ? fv : f8;
                    double r1[4], r2[2];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const bool lo = (t & 4) == 0;
                        const double mk = lo ? m[q] : m[4 + q], mo = lo ? m[4 + q] : m[q];
                        r1[q] = fma(mk, fh, half_mirror(mo * fh));
                    }
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const bool lo = (t & 2) == 0;
                        r2[q] = (lo ? r1[q] : r1[2 + q]) + quad_swap2(lo ? r1[2 + q] : r1[q]);
                    }
                    const bool lo1 = (t & 1) == 0;
                    const double ktf = (lo1 ? r2[0] : r2[1]) + quad_swap1(lo1 ? r2[1] : r2[0]);
                    pvc = gxa + ktf;
                }
                bsync();
            }
        }

        TMARK(5);
        // ================= corrector forward: dz, ds, dl, max step, mu(alpha) sums, max |rp|, max |dz|
        double T0 = 0, T1 = 0, T2 = 0, rpm = 0, dzm = 0;
        MinRatio amc(1e30);
        xt = 0.0;
        fwd_sweep(true, [&](int k, bool vA, const In& cur, double xt_k, double dvv, double (&rr)[14]) {
            const bool aL = row_active(k, cur.lb), aU = row_active(k, cur.ub), aP = poly_slot_active(cur, k);
            if (vA) {
                *ws(k, L::DX) = xt_k;
                *ws(k, L::DV) = dvv;
                dzm = fmax(dzm, fmax(fabs(xt_k), fabs(dvv)));
            }
            const double cz = row_cz(k, cur.zx, cur.zv), cd = row_cz(k, xt_k, dvv), ca = row_cz(k, cur.x0, cur.x1);
            const double pcz = PCACHE ? cur.pz : poly_cz(cur, k, cur.zx, cur.zv), pcd = poly_cz(cur, k, xt_k, dvv);
            const double pca = PCACHE ? cur.pca : poly_cz(cur, k, cur.x0, cur.x1);
            if constexpr (PCACHE) { if (vA) *ws(k, L::PD) = pcd; }
            MinRatio loc(1e30);
            auto rec = [&](bool a, double sgn, double bnd, double czz, double caa, double cdd, double s, double l, int r) {
                double ds = 0.0, dl = 0.0, sv = 0.0, lv = 0.0;
                if (a && vA) {
                    double rp;
                    const SlotStep st = slot_corr(sgn, bnd, czz, caa, cdd, s, l, smu, &rp);
                    step_bound(loc, s, l, st);
                    rpm = fmax(rpm, fabs(rp));
                    sv = s; lv = l; ds = st.ds; dl = st.dl;
                }
                rr[4 * r] = sv; rr[4 * r + 1] = lv; rr[4 * r + 2] = ds; rr[4 * r + 3] = dl;
            };
            rec(aL, sgnL, cur.lb, cz, ca, cd, cur.sL, cur.lL, 0);
            rec(aU, sgnU, cur.ub, cz, ca, cd, cur.sU, cur.lU, 1);
            rec(aP, sgnU, cur.pub, pcz, pca, pcd, cur.sP, cur.lP, 2);
            rr[12] = loc.num;
            rr[13] = loc.den;
        }, [&](const double (&rr)[14]) {
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const double s = rr[4 * r], l = rr[4 * r + 1], ds = rr[4 * r + 2], dl = rr[4 * r + 3];
                mu_acc(T0, T1, T2, s, l, ds, dl);
            }
            amc.add(rr[12], -rr[13]);
        });
        rpm = maxG(rpm);
        dzm = maxG(dzm);
        const double amx = g_min(amc.value());
        T0 = g_sum(T0); T1 = g_sum(T1); T2 = g_sum(T2);
        rpm = g_max(rpm);
        dzm = g_max(dzm);
        alpha = fmin(1.0, fmax(IPM_TAU, 1.0 - sqrt(mu)) * amx);
        sigma_mu = smu;
        pending = true;
        it++;
        TMARK(6);
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
                break;
            } else if (mun > IPM_DIV * mu0) {
                diverged = true;
                break;
            }
        } else {
            break;
        }
    }
#ifdef MPCC_IPM_PROF
    if (lane == 0 && wv == 0) {
        for (int i = 0; i < 16; i++) if (i != 7) atomicAdd(&g_tail_prof[i], (unsigned long long)tprof[i]);
        atomicAdd(&g_tail_prof[7], (unsigned long long)(it - it_in));
    }
#endif
    io.it = it;
    io.conv = conv ? 1 : 0;
    io.diverged = diverged ? 1 : 0;
    io.alpha = alpha;
}

// The rest of a QP solve handed over by ipm_group (its iteration state in LDS at TL_STATE): the remaining
// iterations of the current attempt, the restart from the unit start point if that attempt fails, and ipm_group's
// epilogue (iteration count, QP status, step).  GB = 4: the handing wave alone; GB > 4: every wave of a solo block
// (wave 0 handed over, the others are its helpers, solo_helper), the instance that of wave 0.
template <int NPM, int GB = 4>
__device__ __attribute__((noinline)) void ipm_tail_solve(const DevConst& c, const DevBuffers& d, double* smem) {
    constexpr int NWV = GB / 4;
    const int lane = threadIdx.x & 63, t = lane & 15;
    const int wv = NWV > 1 ? (int)(threadIdx.x >> 6) : 0;
    if (lane == 0 && wv == 0) atomicAdd(&g_tail_solves, 1ull);  // tail-mode hand-overs (mpcc_debug_tail_solves)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const double* st = smem + TL_STATE;
    TailIO io;
    io.it = (int)st[0];
    io.max_it = (int)st[1];
    io.pending = (int)st[2];
    const int attempt = (int)st[3];
    int it_total = (int)st[4];
    io.mu0 = st[5]; io.dz_prev = st[6]; io.sigma_mu = st[7]; io.mu_cur = st[8]; io.rp_cur = st[9]; io.alpha = st[10];
    io.mcount = st[11];
    const int gs = (int)st[12];
    io.conv = io.diverged = io.restart = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int b = inst_of(c, d, blockIdx.x * IPW + gs);
    if constexpr (NWV > 1) __syncthreads();  // every wave has the state before the layout reuses its LDS
    ipm_tail<NPM, GB>(c, d, smem, b, io);
    it_total += io.it;
    if (!io.conv && !io.diverged && attempt == 0 && IPM_ATTEMPTS > 1) {  // a P3 divergence is final
        io.it = 0; io.max_it = IPM_MAX_IT; io.pending = 0; io.conv = 0; io.diverged = 0; io.restart = 1;
        io.mu0 = 0.0; io.dz_prev = 1e30; io.sigma_mu = 0.0; io.mu_cur = 1e30; io.rp_cur = 1e30; io.alpha = 0.0;
        io.mcount = 0.0;
        ipm_tail<NPM, GB>(c, d, smem, b, io);
        it_total += io.it;
    }
    if constexpr (NWV > 1) {
        __syncthreads();  // the helpers are done with the LDS and the workspace
        if (wv != 0) return;
    }
    const int N = c.N, NS = N + 1;
    int32_t* si = d.sqi + (size_t)b * SQI;
#ifdef MPCC_IPM_PROF
    if (lane == 0 && b < 4 * PROF_WAVES) g_inst_its[b] += it_total;
#endif
    if (lane == 0) si[SQ_IPMIT] = it_total;
    if (!io.conv) {  // keep the previous step (Q6)
        if (lane == 0) si[SQ_QPSTAT] = io.diverged ? MPCC_QP_PrimalInfeasible : MPCC_QP_MaxIterReached;
        return;
    }
    if (lane == 0) si[SQ_QPSTAT] = 0;
    if (lane >= 16) return;
    const gdouble* W = (const gdouble*)(d.is + (size_t)b * NS * IS) + t;
    gdouble* stp = (gdouble*)(d.step + (size_t)b * NS * 17);
    const double alpha = io.alpha;
    for (int k = 0; k <= N; k++) {
        const gdouble* wk = W + (size_t)k * IS;
        const double zx = wk[WsF<NPM>::ZX * 16] + alpha * wk[WsF<NPM>::DX * 16];
        const double zv = wk[WsF<NPM>::ZV * 16] + alpha * wk[WsF<NPM>::DV * 16];  // lanes < 8
        if (t < 9) stp[k * 17 + t] = zx;
        if (t < 8) stp[k * 17 + 9 + t] = (k < N) ? zv : 0.0;
    }
}
