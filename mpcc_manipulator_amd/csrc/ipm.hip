// ipm.hip — k_ipm: the per-instance QP solve that replaces OSQP (osqp_interface.cpp:592-656).
//
// Mehrotra predictor-corrector interior point on the stage-structured normalized QP,
// one wavefront per instance.  Step systems are solved by a Riccati recursion over the augmented stage
// state z~ = [y(9), w(7)] (w_k = v_{k-1}[0:7] carries the ddq rate coupling) with input v(8).
// Same algorithm, tolerances and iteration rule as oracle/mpcc_oracle.cpp solve_struct_ipm.
//
// MI355X design: everything the sequential sweeps touch repeatedly lives in LDS (slot slacks and
// multipliers, primal iterate and directions, gradients, Riccati work matrices); per-stage read-only
// QP records and the Riccati factors (U, LF) stream from global memory through double-buffered LDS
// staging, issued one stage ahead so their latency hides under the current stage's arithmetic.
// Backward solves compute the stage gradient on the fly and forward solves recover the slack /
// multiplier steps of the stage they just produced (fused sweeps, no whole-horizon passes between).
#include "dev_common.h"
#include "kernels.h"

namespace mpcc {

constexpr int IPM_MAX_IT = 60;
constexpr double IPM_TOL_MU = 1e-13, IPM_TOL_P = 1e-11, IPM_TOL_STEP = 1e-11;
constexpr int BND_U = 0, BND_LF = 128, BND_POLY = 164;  // stage bundle: U(8x16) | LF(36) | poly rows
constexpr int BND_SZ = 336;
constexpr int PF_QS = (QS + 63) / 64, PF_BND = (BND_SZ + 63) / 64;  // prefetch registers per lane

struct IpmLayout {
    int NS, ns, npmax;
    int oM, oG, oP, oPB, oPM, oF, oGm, oHb, oU, oSt, oBd, oW, oCf, oVec;
    int oS, oL, oDSA, oDLA, oDS, oDL, oBND, oZ, oDZ, oG0, oT, total;
};

__host__ __device__ inline IpmLayout ipm_layout(int N, int npmax) {
    IpmLayout L;
    L.NS = N + 1;
    L.npmax = npmax;
    L.ns = SL_P + npmax;
    int o = 0;
    auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };  // keep 16-B alignment
    L.oM = take(81); L.oG = take(72);
    L.oP = take(256); L.oPB = take(128); L.oPM = take(81); L.oF = take(64); L.oGm = take(128); L.oHb = take(81);
    L.oU = take(128);
    L.oSt = take(2 * QS);
    L.oBd = take(2 * BND_SZ);
    L.oW = take(64); L.oCf = take(64);
    L.oVec = take(96);
    const int nsl = L.NS * L.ns;
    L.oS = take(nsl); L.oL = take(nsl); L.oDSA = take(nsl); L.oDLA = take(nsl); L.oDS = take(nsl); L.oDL = take(nsl);
    L.oBND = take(nsl);
    L.oZ = take(L.NS * 24); L.oDZ = take(L.NS * 24); L.oG0 = take(L.NS * 24);
    L.oT = take(L.NS * 8);
    L.total = o;
    return L;
}

size_t ipm_lds_bytes(int N, int npmax) { return (size_t)ipm_layout(N, npmax).total * sizeof(double); }

// The workgroup is ONE wavefront: lanes run in lockstep, so cross-lane LDS hand-offs only need this
// wave's LDS operations retired (lgkmcnt) and a compiler memory barrier.  __syncthreads() would also
// wait vmcnt(0) and drain the global prefetches the sweeps keep in flight (cdna_hip_programming.md §5).
__device__ __forceinline__ void wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double slot_sgn(int i) { return (i < SL_YU || (i >= SL_DL && i < SL_DU)) ? -1.0 : 1.0; }

// c_i^T z for slot i of stage k (unsigned); z = [y(9) w(7) v(8)]; poly = the stage's poly rows
__device__ __forceinline__ double slot_cz(int i, int k, const double* z, const double* poly) {
    if (i < SL_DL) return z[(i < SL_YU) ? i : i - SL_YU];
    if (i < SL_P) {
        const int j = (i < SL_DU) ? i - SL_DL : i - SL_DU;
        return (k == 0) ? z[16 + j] : z[16 + j] - z[9 + j];
    }
    const double* row = poly + POLY_W * (i - SL_P);
    double s = 0;
#pragma unroll
    for (int j = 0; j < 7; j++) s += row[j] * z[j] + row[7 + j] * z[16 + j];
    return s;
}

__global__ void __launch_bounds__(64) k_ipm(DevConst c, DevBuffers d, int npmax) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    int32_t* si = d.sqi + (size_t)b * SQI;
    if (!si[SQ_ACTIVE]) return;
    const int N = c.N;
    const IpmLayout Ly = ipm_layout(N, npmax);
    const int NS = Ly.NS, ns = Ly.ns;
    double* sM = smem + Ly.oM;   double* sG = smem + Ly.oG;
    double* sP = smem + Ly.oP;   double* sPB = smem + Ly.oPB; double* sPM = smem + Ly.oPM;
    double* sF = smem + Ly.oF;   double* sGm = smem + Ly.oGm; double* sHb = smem + Ly.oHb;
    double* sU = smem + Ly.oU;
    double* sSt = smem + Ly.oSt;  // 2 x QS
    double* sBd = smem + Ly.oBd;  // 2 x BND_SZ
    double* sW = smem + Ly.oW;   double* sCf = smem + Ly.oCf;
    double* sVec = smem + Ly.oVec;
    double* pv0 = sVec;      double* pv1 = sVec + 16;  // backward p (ping-pong)
    double* xv0 = sVec + 32; double* xv1 = sVec + 48;  // forward x~ (ping-pong)
    double* sFv = sVec + 64; double* sH = sVec + 72; double* sGx = sVec + 80;
    double* sS = smem + Ly.oS;   double* sL = smem + Ly.oL;
    double* sDSA = smem + Ly.oDSA; double* sDLA = smem + Ly.oDLA;
    double* sDS = smem + Ly.oDS; double* sDL = smem + Ly.oDL;
    double* sBND = smem + Ly.oBND;
    double* sZ = smem + Ly.oZ;   double* sDZ = smem + Ly.oDZ; double* sG0 = smem + Ly.oG0;
    double* sT = smem + Ly.oT;

    const double* QSb = d.qs + (size_t)b * NS * QS;
    double* ISb = d.is + (size_t)b * NS * IS;
    const double* Tu = c.p.Tu;
    const double HcB = -2. * c.p.qp_r_ddq;
    auto Hc = [&](int j) { return Tu[j] * HcB * Tu[j]; };

    for (int e = lane; e < 81; e += 64) sM[e] = c.M[e];
    for (int e = lane; e < 72; e += 64) sG[e] = c.G[e];

    // ---- Hessian checks (osqp_interface.cpp:454-473): state blocks (k_setqp flags) + tridiagonal input blocks
    int fl = 0;
    for (int k = lane; k < NS; k += 64) fl |= (int)QSb[(size_t)k * QS + QS_FLAG];
    if (lane < 8) {
        const int j = lane;
        double prev_d = 0;
        for (int k = 0; k < N; k++) {
            const double dk = QSb[(size_t)k * QS + QS_R + j];
            const double off = (k >= 1 && j < DOF) ? Hc(j) : 0.0;
            const double l = (k >= 1) ? off / prev_d : 0.0;
            const double dd = dk - l * l;
            if (dd <= 0) { fl |= 2; break; }
            prev_d = sqrt(dd);
        }
    }
    fl = wave_or(fl);
    if (fl & 2) { if (lane == 0) { si[SQ_STATUS] = MPCC_NON_PD_HESSIAN; si[SQ_ACTIVE] = 0; } return; }
    if (fl & 1) { if (lane == 0) { si[SQ_STATUS] = MPCC_NAN_HESSIAN; si[SQ_ACTIVE] = 0; } return; }
    if (fl & 4) { if (lane == 0) si[SQ_QPSTAT] = MPCC_QP_PrimalInfeasible; return; }  // keep old step (Q6)

    // ---- global -> LDS staging helpers (issue into registers, commit later)
    auto qs_issue = [&](int k, double* r) {
        const double* src = QSb + (size_t)k * QS;
#pragma unroll
        for (int t = 0; t < PF_QS; t++) { const int e = lane + 64 * t; r[t] = (e < QS) ? src[e] : 0.0; }
    };
    auto qs_commit = [&](double* dst, const double* r) {
#pragma unroll
        for (int t = 0; t < PF_QS; t++) { const int e = lane + 64 * t; if (e < QS) dst[e] = r[t]; }
    };
    const int npw = POLY_W * npmax;
    auto bd_issue = [&](int k, double* r) {
        const double* is = ISb + (size_t)k * IS;
        const double* q = QSb + (size_t)k * QS;
#pragma unroll
        for (int t = 0; t < PF_BND; t++) {
            const int e = lane + 64 * t;
            double v = 0.0;
            if (e >= BND_SZ) v = 0.0;
            else if (e < 128) v = is[IS_U + e];
            else if (e < 164) v = is[IS_LF + e - 128];
            else if (e < 164 + npw) v = q[QS_POLY + e - 164];
            r[t] = v;
        }
    };
    auto bd_commit = [&](double* dst, const double* r) {
#pragma unroll
        for (int t = 0; t < PF_BND; t++) { const int e = lane + 64 * t; if (e < BND_SZ) dst[e] = r[t]; }
    };

    // ---- slots: bounds / activity
    const int nsl = NS * ns;
    double mcount = 0;
    for (int e = lane; e < nsl; e += 64) {
        const int k = e / ns, i = e - k * ns;
        const double* q = QSb + (size_t)k * QS;
        double bnd;
        bool act;
        if (i < SL_DL) {
            bnd = (i < SL_YU) ? q[QS_YLB + i] : q[QS_YUB + i - SL_YU];
            act = (k >= 1) && fabs(bnd) < BIG;
        } else if (i < SL_P) {
            bnd = (i < SL_DU) ? q[QS_DLB + i - SL_DL] : q[QS_DUB + i - SL_DU];
            act = (k < N) && fabs(bnd) < BIG;
        } else {
            const int r = i - SL_P;
            const int np = (int)q[QS_NPOLY];
            bnd = (r < np) ? q[QS_POLY + POLY_W * r + 14] : INF;
            act = (k < N) && (r < np) && fabs(bnd) < BIG;
        }
        sBND[e] = act ? bnd : INF;
        mcount += act ? 1.0 : 0.0;
    }
    mcount = wave_sum(mcount);
    // ---- primal start: dynamics rollout with v = 0
    for (int e = lane; e < NS * 24; e += 64) sZ[e] = 0.0;
    wave_sync();
    for (int k = 0; k < N; k++) {
        double yn = 0;
        if (lane < 9) {
            double s = 0;
            for (int m = 0; m < 9; m++) s += sM[lane * 9 + m] * sZ[k * 24 + m];
            yn = s + QSb[(size_t)k * QS + QS_B + lane];
        }
        if (lane < 9) sZ[(k + 1) * 24 + lane] = yn;
        wave_sync();
    }
    for (int e = lane; e < nsl; e += 64) {
        const int k = e / ns, i = e - k * ns;
        if (fabs(sBND[e]) < BIG) {
            const double sg = slot_sgn(i);
            const double g = sg * slot_cz(i, k, sZ + 24 * k, QSb + (size_t)k * QS + QS_POLY) - sg * sBND[e];
            sS[e] = fmax(-g, 1.0);
            sL[e] = 1.0;
        } else {
            sS[e] = 1.0;
            sL[e] = 0.0;
        }
        sDSA[e] = 0.0; sDLA[e] = 0.0;
    }
    wave_sync();

    // per-slot residual / complementarity helpers for stage k, slot i (uses staged poly rows)
    auto rp_of = [&](int k, int i, int e, const double* poly) {
        const double sg = slot_sgn(i);
        return sg * slot_cz(i, k, sZ + 24 * k, poly) - sg * sBND[e] + sS[e];
    };

    double last_dz = 1e30;
    bool conv = false;
    int it;
    double rq[PF_QS > PF_BND ? PF_QS : PF_BND];
    for (it = 0; it < IPM_MAX_IT; it++) {
        // ---- pass A: complementarity and primal residual
        double mus = 0, rpm = 0;
        for (int e = lane; e < nsl; e += 64) {
            const int k = e / ns, i = e - k * ns;
            if (fabs(sBND[e]) >= BIG) continue;
            const double rp = rp_of(k, i, e, QSb + (size_t)k * QS + QS_POLY);
            mus += sS[e] * sL[e];
            rpm = fmax(rpm, fabs(rp));
        }
        mus = wave_sum(mus);
        rpm = wave_max(rpm);
        const double mu = (mcount > 0) ? mus / mcount : 0.0;
        if (it > 0 && mu < IPM_TOL_MU && rpm < IPM_TOL_P && last_dz < IPM_TOL_STEP) { conv = true; break; }

        // ================= Riccati factorization sweep (k = N .. 0), fused with g0 = H z + h
        qs_issue(N, rq);
        qs_commit(sSt + (N & 1) * QS, rq);
        if (N >= 1) qs_issue(N - 1, rq);
        wave_sync();
        {
            const double* st = sSt + (N & 1) * QS;
            if (lane < ns) {
                const int e = N * ns + lane;
                sW[lane] = (fabs(sBND[e]) < BIG) ? sL[e] / sS[e] : 0.0;
            }
            if (lane < 24) {  // g0 of the terminal stage: y part only
                double g = 0;
                if (lane < 9) {
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += st[QS_Q + lane * 9 + m] * sZ[N * 24 + m];
                    g = s + st[QS_q + lane];
                }
                sG0[N * 24 + lane] = g;
            }
            wave_sync();
            for (int e = lane; e < 256; e += 64) {
                const int a = e >> 4, cc = e & 15;
                double v = 0;
                if (a < 9 && cc < 9) {
                    v = st[QS_Q + a * 9 + cc];
                    if (a == cc) v += sW[SL_YL + a] + sW[SL_YU + a];
                }
                sP[e] = v;
            }
        }
        for (int k = N - 1; k >= 0; k--) {
            double* st = sSt + (k & 1) * QS;
            qs_commit(st, rq);
            if (k >= 1) qs_issue(k - 1, rq);
            wave_sync();
            double* is = ISb + (size_t)k * IS;
            // (a) barrier weights, g0, PB = P B~, PM = P_yy M
            if (lane < ns) {
                const int e = k * ns + lane;
                sW[lane] = (fabs(sBND[e]) < BIG) ? sL[e] / sS[e] : 0.0;
            }
            if (lane < 24) {
                const double* z = sZ + 24 * k;
                const int a = lane;
                double g;
                if (a < 9) {
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += st[QS_Q + a * 9 + m] * z[m];
                    g = s + st[QS_q + a];
                } else if (a < 16) {
                    const int j = a - 9;
                    g = (k >= 1) ? Hc(j) * z[16 + j] : 0.0;
                } else {
                    const int j = a - 16;
                    g = st[QS_R + j] * z[a] + st[QS_r + j];
                    if (k >= 1 && j < DOF) g += Hc(j) * z[9 + j];
                }
                sG0[k * 24 + a] = g;
            }
            for (int e = lane; e < 128 + 81; e += 64) {
                if (e < 128) {
                    const int a = e >> 3, j = e & 7;
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sP[a * 16 + m] * sG[m * 8 + j];
                    if (j < 7) s += sP[a * 16 + 9 + j];
                    sPB[e] = s;
                } else {
                    const int e2 = e - 128, a = e2 / 9, cc = e2 - a * 9;
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sP[a * 16 + m] * sM[m * 9 + cc];
                    sPM[e2] = s;
                }
            }
            wave_sync();
            const int np = (int)st[QS_NPOLY];
            // (b) F = R~ + B~^T P B~, Gm = S~ + B~^T P A~, Hb_yy = Q~_yy + M^T P_yy M
            for (int e = lane; e < 64 + 128 + 81; e += 64) {
                if (e < 64) {
                    const int i = e >> 3, j = e & 7;
                    double rt = 0;
                    if (i == j) {
                        rt = st[QS_R + i];
                        if (i < 7) rt += sW[SL_DL + i] + sW[SL_DU + i];
                    }
                    if (i < 7 && j < 7)
                        for (int r = 0; r < np; r++) {
                            const double* row = st + QS_POLY + POLY_W * r;
                            rt += sW[SL_P + r] * row[7 + i] * row[7 + j];
                        }
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sG[m * 8 + i] * sPB[m * 8 + j];
                    if (i < 7) s += sPB[(9 + i) * 8 + j];
                    sF[e] = rt + s;
                } else if (e < 192) {
                    const int e2 = e - 64, i = e2 >> 4, cc = e2 & 15;
                    double v;
                    if (cc < 9) {
                        double st_ = 0;
                        if (i < 7 && cc < 7)
                            for (int r = 0; r < np; r++) {
                                const double* row = st + QS_POLY + POLY_W * r;
                                st_ += sW[SL_P + r] * row[7 + i] * row[cc];
                            }
                        double s = 0;
                        for (int m = 0; m < 9; m++) s += sPB[m * 8 + i] * sM[m * 9 + cc];
                        v = st_ + s;
                    } else {
                        const int j = cc - 9;
                        v = (i == j && k >= 1) ? Hc(j) - (sW[SL_DL + j] + sW[SL_DU + j]) : 0.0;
                    }
                    sGm[e2] = v;
                } else {
                    const int e2 = e - 192, a = e2 / 9, cc = e2 - a * 9;
                    double v = st[QS_Q + a * 9 + cc];
                    if (a == cc) v += sW[SL_YL + a] + sW[SL_YU + a];
                    if (a < 7 && cc < 7)
                        for (int r = 0; r < np; r++) {
                            const double* row = st + QS_POLY + POLY_W * r;
                            v += sW[SL_P + r] * row[a] * row[cc];
                        }
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sM[m * 9 + a] * sPM[m * 9 + cc];
                    sHb[e2] = v + s;
                }
            }
            wave_sync();
            // (c) LF = chol(F) in every lane (registers); U = LF^-1 Gm, lane = column
            double Lf[36];
            {
                int idx = 0;
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) Lf[idx++] = sF[i * 8 + j];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int jj = j * (j + 1) / 2;
                    double dg = Lf[jj + j];
#pragma unroll
                    for (int m = 0; m < j; m++) dg -= Lf[jj + m] * Lf[jj + m];
                    dg = sqrt(dg);
                    Lf[jj + j] = dg;
                    const double inv = 1.0 / dg;
#pragma unroll
                    for (int i = j + 1; i < 8; i++) {
                        const int ii = i * (i + 1) / 2;
                        double s = Lf[ii + j];
#pragma unroll
                        for (int m = 0; m < j; m++) s -= Lf[ii + m] * Lf[jj + m];
                        Lf[ii + j] = s * inv;
                    }
                }
            }
            if (lane < 16) {
                double u[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int ii = i * (i + 1) / 2;
                    double s = sGm[i * 16 + lane];
#pragma unroll
                    for (int m = 0; m < i; m++) s -= Lf[ii + m] * u[m];
                    u[i] = s / Lf[ii + i];
                }
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    sU[i * 16 + lane] = u[i];
                    is[IS_U + i * 16 + lane] = u[i];
                }
            } else if (lane < 16 + 36) {
                const int e = lane - 16;
                double v = 0;
#pragma unroll
                for (int m = 0; m < 36; m++) v = (m == e) ? Lf[m] : v;
                is[IS_LF + e] = v;
            }
            wave_sync();
            // (d) P = Hb - U^T U
            if (k > 0) {
                for (int e = lane; e < 256; e += 64) {
                    const int a = e >> 4, cc = e & 15;
                    double v = 0;
                    if (a < 9 && cc < 9) v = sHb[a * 9 + cc];
                    else if (a >= 9 && a == cc) v = sW[SL_DL + a - 9] + sW[SL_DU + a - 9];
                    double s = 0;
#pragma unroll
                    for (int i = 0; i < 8; i++) s += sU[i * 16 + a] * sU[i * 16 + cc];
                    sP[e] = v - s;
                }
            }
        }
        // U / LF stores of the sweep must be performed before the solves load them back
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_sync();

        // ================= two solves (predictor, corrector) with the same factorization
        double sigma_mu = 0.0, alpha = 0.0, dzmax = 0.0;
        for (int phase = 0; phase < 2; phase++) {
            // slot coefficient of stage k slot i: sgn * (l + W rp - rc / s)
            auto coef_of = [&](int k, int i, const double* poly) -> double {
                const int e = k * ns + i;
                if (fabs(sBND[e]) >= BIG) return 0.0;
                const double s = sS[e], l = sL[e];
                const double rp = rp_of(k, i, e, poly);
                const double rc = (phase == 0) ? s * l : s * l + sDSA[e] * sDLA[e] - sigma_mu;
                return slot_sgn(i) * (l + (l / s) * rp - rc / s);
            };
            // ---- backward sweep: p_N = g_x~(N); per stage f = g_v + B~^T p, t = LF^-1 f, p = g_x~ + A~^T p - U^T t
            {
                const double* poly = QSb + (size_t)N * QS + QS_POLY;  // unused at N (no poly slots)
                if (lane < ns) sCf[lane] = coef_of(N, lane, poly);
                bd_issue(N - 1, rq);
                wave_sync();
                if (lane < 16) {
                    double g = sG0[N * 24 + lane];
                    if (lane < 9) g += sCf[SL_YL + lane] + sCf[SL_YU + lane];
                    pv0[lane] = g;  // p of stage N lives in pv[N & 1]; use pv0/pv1 by parity below
                    if (N & 1) pv1[lane] = g;
                }
                wave_sync();
            }
            for (int k = N - 1; k >= 0; k--) {
                double* bd = sBd + (k & 1) * BND_SZ;
                bd_commit(bd, rq);
                if (k >= 1) bd_issue(k - 1, rq);
                wave_sync();
                const double* pn = ((k + 1) & 1) ? pv1 : pv0;
                double* pc = (k & 1) ? pv1 : pv0;
                const double* poly = bd + BND_POLY;
                if (lane < ns) sCf[lane] = coef_of(k, lane, poly);
                wave_sync();
                const int np = (int)QSb[(size_t)k * QS + QS_NPOLY];
                if (lane < 24) {
                    const int a = lane;
                    double g = sG0[k * 24 + a];
                    if (a < 9) {
                        g += sCf[SL_YL + a] + sCf[SL_YU + a];
                        if (a < 7)
                            for (int r = 0; r < np; r++) g += sCf[SL_P + r] * poly[POLY_W * r + a];
                        sGx[a] = g;
                    } else if (a < 16) {
                        const int j = a - 9;
                        if (k >= 1) g -= sCf[SL_DL + j] + sCf[SL_DU + j];
                        sGx[a] = g;
                    } else {
                        const int j = a - 16;
                        if (j < 7) {
                            g += sCf[SL_DL + j] + sCf[SL_DU + j];
                            for (int r = 0; r < np; r++) g += sCf[SL_P + r] * poly[POLY_W * r + 7 + j];
                        }
                        double s = 0;
                        for (int m = 0; m < 9; m++) s += sG[m * 8 + j] * pn[m];
                        if (j < 7) s += pn[9 + j];
                        sFv[j] = g + s;
                    }
                }
                wave_sync();
                double t[8];
                {
                    const double* Lf = bd + BND_LF;
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const int ii = i * (i + 1) / 2;
                        double s = sFv[i];
#pragma unroll
                        for (int m = 0; m < i; m++) s -= Lf[ii + m] * t[m];
                        t[i] = s / Lf[ii + i];
                    }
                }
                if (lane < 8) {
                    double tv = 0;
#pragma unroll
                    for (int m = 0; m < 8; m++) tv = (m == lane) ? t[m] : tv;
                    sT[k * 8 + lane] = tv;
                }
                if (k > 0 && lane < 16) {
                    double s = sGx[lane];
                    if (lane < 9)
                        for (int m = 0; m < 9; m++) s += sM[m * 9 + lane] * pn[m];
                    const double* U = bd + BND_U;
#pragma unroll
                    for (int i = 0; i < 8; i++) s -= U[i * 16 + lane] * t[i];
                    pc[lane] = s;
                }
                wave_sync();
            }
            // ---- forward sweep: x~_0 = 0; v = -LF^-T (U x~ + t); x~_{k+1} = A~ x~ + B~ v; recover ds, dl
            double amax = (phase == 0) ? 1.0 : 1e30;
            double dzm = 0.0;
            if (lane < 16) xv0[lane] = 0.0;
            bd_issue(0, rq);
            wave_sync();
            double* sDSx = (phase == 0) ? sDSA : sDS;
            double* sDLx = (phase == 0) ? sDLA : sDL;
            auto recover = [&](int k, const double* poly) {
                if (lane < ns) {
                    const int i = lane, e = k * ns + i;
                    if (fabs(sBND[e]) < BIG) {
                        const double cd = slot_sgn(i) * slot_cz(i, k, sDZ + 24 * k, poly);
                        const double s = sS[e], l = sL[e];
                        const double rp = rp_of(k, i, e, poly);
                        const double rc = (phase == 0) ? s * l : s * l + sDSA[e] * sDLA[e] - sigma_mu;
                        const double ds = -rp - cd;
                        const double dl = (l / s) * (cd + rp) - rc / s;
                        sDSx[e] = ds;
                        sDLx[e] = dl;
                        if (ds < 0) amax = fmin(amax, -s / ds);
                        if (dl < 0) amax = fmin(amax, -l / dl);
                    }
                }
            };
            for (int k = 0; k < N; k++) {
                double* bd = sBd + (k & 1) * BND_SZ;
                bd_commit(bd, rq);
                if (k + 1 < N) bd_issue(k + 1, rq);
                wave_sync();
                const double* xc = (k & 1) ? xv1 : xv0;
                double* xn_ = (k & 1) ? xv0 : xv1;
                if (lane < 8) {
                    double s = sT[k * 8 + lane];
                    const double* U = bd + BND_U;
                    for (int a = 0; a < 16; a++) s += U[lane * 16 + a] * xc[a];
                    sH[lane] = s;
                }
                wave_sync();
                double v[8];
                {
                    const double* Lf = bd + BND_LF;
#pragma unroll
                    for (int i = 7; i >= 0; i--) {
                        double s = sH[i];
#pragma unroll
                        for (int m = i + 1; m < 8; m++) s -= Lf[m * (m + 1) / 2 + i] * v[m];
                        v[i] = s / Lf[i * (i + 1) / 2 + i];
                    }
#pragma unroll
                    for (int i = 0; i < 8; i++) v[i] = -v[i];
                }
                if (lane < 16) {
                    double xn;
                    if (lane < 9) {
                        double s = 0;
                        for (int m = 0; m < 9; m++) s += sM[lane * 9 + m] * xc[m];
#pragma unroll
                        for (int j = 0; j < 8; j++) s += sG[lane * 8 + j] * v[j];
                        xn = s;
                    } else {
                        double vv = 0;
#pragma unroll
                        for (int j = 0; j < 7; j++) vv = (j == lane - 9) ? v[j] : vv;
                        xn = vv;
                    }
                    xn_[lane] = xn;
                    sDZ[k * 24 + lane] = xc[lane];
                    dzm = fmax(dzm, fabs(xc[lane]));
                } else if (lane < 24) {
                    double vv = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) vv = (j == lane - 16) ? v[j] : vv;
                    sDZ[k * 24 + lane] = vv;
                    dzm = fmax(dzm, fabs(vv));
                }
                wave_sync();
                recover(k, bd + BND_POLY);
            }
            if (lane < 24) {
                const double* xl = (N & 1) ? xv1 : xv0;
                const double v = (lane < 16) ? xl[lane] : 0.0;
                sDZ[N * 24 + lane] = v;
                dzm = fmax(dzm, fabs(v));
            }
            wave_sync();
            recover(N, QSb + (size_t)N * QS + QS_POLY);
            amax = wave_min(amax);
            wave_sync();
            if (phase == 0) {
                double mua = 0;
                for (int e = lane; e < nsl; e += 64) {
                    if (fabs(sBND[e]) >= BIG) continue;
                    mua += (sS[e] + amax * sDSA[e]) * (sL[e] + amax * sDLA[e]);
                }
                mua = wave_sum(mua);
                mua = (mcount > 0) ? mua / mcount : 0.0;
                const double ratio = (mu > 0) ? mua / mu : 0.0;
                const double sigma = (mu > 0) ? ratio * ratio * ratio : 0.0;
                sigma_mu = sigma * mu;
            } else {
                alpha = fmin(1.0, 0.995 * amax);
                dzmax = wave_max(dzm);
            }
        }
        // ---- update
        for (int e = lane; e < NS * 24; e += 64) sZ[e] += alpha * sDZ[e];
        for (int e = lane; e < nsl; e += 64) {
            if (fabs(sBND[e]) >= BIG) continue;
            sS[e] += alpha * sDS[e];
            sL[e] += alpha * sDL[e];
        }
        last_dz = dzmax;
        wave_sync();
    }
    if (lane == 0) si[SQ_IPMIT] = it;
    if (!conv) {
        if (lane == 0) si[SQ_QPSTAT] = MPCC_QP_MaxIterReached;  // keep the previous step (Q6)
        return;
    }
    if (lane == 0) si[SQ_QPSTAT] = 0;
    double* stp = d.step + (size_t)b * NS * 17;
    for (int e = lane; e < NS * 17; e += 64) {
        const int k = e / 17, a = e - k * 17;
        const double* z = sZ + 24 * k;
        stp[e] = (a < 9) ? z[a] : ((k < N) ? z[16 + a - 9] : 0.0);
    }
}

void launch_ipm(const DevConst& c, const DevBuffers& d, int npmax, hipStream_t s) {
    const size_t lds = ipm_lds_bytes(c.N, npmax);
    static size_t configured = 0;
    if (lds > configured) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ipm), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        configured = lds;
    }
    hipLaunchKernelGGL(k_ipm, dim3(c.Bn), dim3(64), lds, s, c, d, npmax);
}

}  // namespace mpcc
