// kernels.hip — HIP kernels of the MI355X batched MPCC solve engine (gfx950, FP64).
//
// One batch call = one MPC::runMPC_ (cpp/src/MPC/mpc.cpp:104-190) for each of B independent
// controllers.  Kernel sequence:
//   k_prepare      thread / instance        projection, vs estimate, warm-start shift  (mpc.cpp:104-124, 54-89)
//   k_records      thread / (instance,stage) RobotData::update: FK, J, manipulability + FD gradient (robot_data.h:55-71)
//   k_nn           wave / (instance,stage)  self / env collision MLPs + input Jacobians (SelfCollisionModel.cpp:140-250)
//   per SQP iteration (osqp_interface.cpp:431-574):
//     k_setqp      thread / (instance,stage) stage QP record: cost, constraint rows, bounds, dynamics residual
//     k_ipm        wave / instance           Mehrotra interior point, Riccati factorization (replaces OSQP)
//     k_trial      thread / (instance,stage) filter line-search trial at alpha = 1 (objective, violation)
//     k_accept     thread / instance         filter, step, termination
//   k_finalize     thread / instance         Status -> warm start / outputs (osqp_interface.cpp:575-589, mpc.cpp:140-189)
#include "dev_cost.h"
#include "kernels.h"

namespace mpcc {

// ------------------------------------------------------------------------------------------------
// k_prepare
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_prepare(DevConst c, DevBuffers d) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= c.Bn) return;
    const int N = c.N;
    double x[9], u[8];
#pragma unroll
    for (int i = 0; i < 9; i++) x[i] = d.x0[9 * b + i];
#pragma unroll
    for (int i = 0; i < 8; i++) u[i] = d.u0[8 * b + i];
    const double last_s = x[7];
    double ee[3], J[42];
    panda_fk(x, ee, nullptr, J, true);
    x[7] = project_on_spline(c.spl, c.p.proj_max_dist, last_s, ee);
    double ev[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double s = 0;
#pragma unroll
        for (int j = 0; j < DOF; j++) s += J[7 * i + j] * u[j];
        ev[i] = s;
    }
    double dir[3];
    spline_pos3(c.spl, x[7], nullptr, dir, nullptr);
    x[8] = ev[0] * dir[0] + ev[1] * dir[1] + ev[2] * dir[2];
    int valid = d.valid[b], fails = d.fails[b];
    if (fabs(last_s - x[7]) > c.p.guess_max_dist) { valid = 0; fails++; }
    double* g = d.guess + (size_t)b * (N + 1) * 17;
    if (valid) {  // updateInitialGuess (mpc.cpp:54-68)
        for (int i = 1; i < N; i++)
            for (int a = 0; a < 17; a++) g[17 * (i - 1) + a] = g[17 * i + a];
        for (int a = 0; a < 9; a++) g[a] = x[a];
        for (int a = 0; a < 17; a++) g[17 * (N - 1) + a] = g[17 * (N - 2) + a];
        rk4_step(g + 17 * (N - 1), g + 17 * (N - 1) + 9, c.p.Ts, g + 17 * N);
        for (int a = 0; a < 8; a++) g[17 * N + 9 + a] = 0.0;
    } else {  // generateNewInitialGuess (mpc.cpp:79-89)
        for (int i = 0; i <= N; i++) {
            for (int a = 0; a < 9; a++) g[17 * i + a] = x[a];
            for (int a = 0; a < 8; a++) g[17 * i + 9 + a] = 0.0;
        }
        valid = 1;
    }
    for (int i = 1; i <= N; i++) g[17 * i + 7] = fmin(g[17 * i + 7], c.spl.L);  // unwrapInitialGuess
#pragma unroll
    for (int i = 0; i < 9; i++) d.x0[9 * b + i] = x[i];
    d.valid[b] = valid;
    d.fails[b] = fails;
    int32_t* si = d.sqi + (size_t)b * SQI;
    si[SQ_STATUS] = MPCC_MAX_ITER_EXCEEDED;
    si[SQ_ACTIVE] = 1;
    si[SQ_ITER] = 0;
    si[SQ_NFILT] = 0;
    si[SQ_QPSTAT] = 0;
    si[SQ_IPMIT] = 0;
    double* st = d.step + (size_t)b * (N + 1) * 17;
    for (int i = 0; i < (N + 1) * 17; i++) st[i] = 0.0;  // step_.setZero (osqp_interface.cpp:404)
}

// ------------------------------------------------------------------------------------------------
// k_records: FK, Jacobian, manipulability and its central-difference gradient (15 Jacobians).
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_records(DevConst c, DevBuffers d) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int S = c.S;
    if (t >= S) return;
    const int N = c.N;
    const int b = t / (N + 1), k = t - b * (N + 1);
    const double* g = d.guess + ((size_t)b * (N + 1) + k) * 17;
    double q[7];
#pragma unroll
    for (int j = 0; j < 7; j++) q[j] = g[j];
    double pos[3], R[9], J[42];
    panda_fk(q, pos, R, J, true);
    double* rec = d.rec + t;
#pragma unroll
    for (int a = 0; a < 3; a++) rec[(size_t)(R_POS + a) * S] = pos[a];
#pragma unroll
    for (int a = 0; a < 9; a++) rec[(size_t)(R_ROT + a) * S] = R[a];
#pragma unroll
    for (int a = 0; a < 42; a++) rec[(size_t)(R_J + a) * S] = J[a];
    rec[(size_t)R_MU * S] = manip_from_J(J);
    const double delta = 1e-4;  // robot_model.cpp:439
    for (int i = 0; i < 7; i++) {
        double qp[7], qm[7];
#pragma unroll
        for (int j = 0; j < 7; j++) { qp[j] = q[j] + (j == i ? delta : 0.0); qm[j] = q[j] - (j == i ? delta : 0.0); }
        double m1 = manipulability(qp), m2 = manipulability(qm);
        rec[(size_t)(R_DMU + i) * S] = (m1 - m2) / (2 * delta);
    }
    const double inf = __longlong_as_double(0x7ff0000000000000LL);
    if (!(c.p.constraint_mask & MPCC_CON_SELFCOL)) {
        rec[(size_t)R_SEL * S] = inf;
#pragma unroll
        for (int j = 0; j < 7; j++) rec[(size_t)(R_DSEL + j) * S] = 0.0;
    }
    rec[(size_t)R_OBSR * S] = d.obs[4 * b + 3];
    if (!(c.p.constraint_mask & MPCC_CON_ENVCOL)) {
        for (int m = 0; m < 9; m++) rec[(size_t)(R_ENV + m) * S] = inf;
        for (int m = 0; m < 63; m++) rec[(size_t)(R_DENV + m) * S] = 0.0;
    }
}

// ------------------------------------------------------------------------------------------------
// k_nn: NeRF MLP value + 7-column forward-mode input Jacobian, one wave per (instance, stage).
// Weights are stored transposed per layer (W^T[k][r]) so that a wave's lanes read consecutive
// output rows.  Activations [width][8] (value + 7 tangents) live in LDS.
// ------------------------------------------------------------------------------------------------


template <int MAXW>
__device__ inline void nn_eval_wave(const NNDesc& nd, const double* __restrict__ W, const double* in, double* lds_a,
                                    double* lds_b, double* out_val, double* out_jac /* nout x 7 */) {
    const int lane = threadIdx.x;
    const int nin = nd.nin;
    // layer 0 (NeRF input [x, sin x, cos x]; SelfCollisionModel.cpp:143-151, 162-188)
    {
        const int R = nd.dims[1], C = nd.dims[0];
        const double* WT = W + nd.offW[0];
        const double* bb = W + nd.offb[0];
        for (int r = lane; r < R; r += 64) {
            double h = 0;
            for (int k = 0; k < C; k++) {
                int kk = k % nin, part = k / nin;
                double xk = in[kk];
                double f = (part == 0) ? xk : (part == 1 ? sin(xk) : cos(xk));
                h += WT[(size_t)k * R + r] * f;
            }
            h += bb[r];
            double gsw = h > 0 ? 1.0 : 0.0;
            lds_a[r * 8] = fmax(0.0, h);
#pragma unroll
            for (int j = 0; j < 7; j++) {
                double w0 = gsw * WT[(size_t)j * R + r];
                double w1 = gsw * WT[(size_t)(nin + j) * R + r];
                double w2 = gsw * WT[(size_t)(2 * nin + j) * R + r];
                lds_a[r * 8 + 1 + j] = w0 * 1.0 + w1 * cos(in[j]) + w2 * (-sin(in[j]));
            }
        }
    }
    __syncthreads();
    double* src = lds_a;
    double* dst = lds_b;
    for (int l = 1; l < nd.L; l++) {
        const int R = nd.dims[l + 1], C = nd.dims[l];
        const double* WT = W + nd.offW[l];
        const double* bb = W + nd.offb[l];
        const bool last = (l == nd.L - 1);
        for (int r = lane; r < R; r += 64) {
            double acc[8];
#pragma unroll
            for (int j = 0; j < 8; j++) acc[j] = 0.0;
            for (int k = 0; k < C; k++) {
                double w = WT[(size_t)k * R + r];
#pragma unroll
                for (int j = 0; j < 8; j++) acc[j] += w * src[k * 8 + j];
            }
            double h = acc[0] + bb[r];
            if (last) {
                out_val[r] = h;
#pragma unroll
                for (int j = 0; j < 7; j++) out_jac[r * 7 + j] = acc[1 + j];
            } else {
                double gsw = h > 0 ? 1.0 : 0.0;
                dst[r * 8] = fmax(0.0, h);
#pragma unroll
                for (int j = 0; j < 7; j++) dst[r * 8 + 1 + j] = gsw * acc[1 + j];
            }
        }
        __syncthreads();
        double* t = src; src = dst; dst = t;
    }
}

__global__ void __launch_bounds__(64) k_nn(DevConst c, DevBuffers d, NNDesc nd, const double* __restrict__ W, int which,
                                          int M, const double* __restrict__ qin, const double* __restrict__ obsin,
                                          double* __restrict__ recout, int rec_stride) {
    __shared__ double lds[2 * 256 * 8];
    const int t = blockIdx.x;
    if (t >= M) return;
    __shared__ double outv[16], outj[16 * 7];
    double in[10];
    int S = rec_stride;
    const double* obs;
    if (qin) {  // debug path: explicit q / obs lists
        for (int j = 0; j < 7; j++) in[j] = qin[7 * t + j];
        obs = obsin + 4 * t;
    } else {
        const int N = c.N;
        const int b = t / (N + 1), k = t - b * (N + 1);
        const double* g = d.guess + ((size_t)b * (N + 1) + k) * 17;
        for (int j = 0; j < 7; j++) in[j] = g[j];
        obs = d.obs + 4 * b;
    }
    if (which == 1) { in[7] = obs[0]; in[8] = obs[1]; in[9] = obs[2]; }
    nn_eval_wave<256>(nd, W, in, lds, lds + 256 * 8, outv, outj);
    __syncthreads();
    double* rec = recout + t;
    const int lane = threadIdx.x;
    if (which == 0) {
        if (lane == 0) rec[(size_t)R_SEL * S] = outv[0];
        if (lane < 7) rec[(size_t)(R_DSEL + lane) * S] = outj[lane];
    } else {
        if (lane < 9) rec[(size_t)(R_ENV + lane) * S] = outv[lane];
        if (lane < 63) rec[(size_t)(R_DENV + lane) * S] = outj[lane];
    }
}

// ------------------------------------------------------------------------------------------------
// k_setqp: stage QP record (setCost + setDynamics + setBounds + setPolytopicConstraints,
// osqp_interface.cpp:129-344) in the stage-structured normalized form.
// ------------------------------------------------------------------------------------------------
__device__ inline void setqp_stage(const DevConst& c, const double* __restrict__ gb, const RecView& rv, int k,
                                   const double* __restrict__ ucur, double* __restrict__ q) {
    const mpcc_params& p = c.p;
    const int N = c.N;
    const double* Tx = p.Tx;
    const double* Tu = p.Tu;
    const double* xk = gb + 17 * k;
    const double* uk = gb + 17 * k + 9;
    double fx[9], fu[8], fxx[81], fuu[8];
    double obj = stage_cost(c, xk, uk, rv, k, true, fx, fu, fxx, fuu);
    int flag = 0;
    for (int a = 0; a < 9; a++) {
        q[QS_q + a] = Tx[a] * fx[a];
        for (int bb = 0; bb < 9; bb++) {
            double v = Tx[a] * fxx[a * 9 + bb] * Tx[bb];
            q[QS_Q + a * 9 + bb] = v;
            if (isnan(v)) flag |= 1;
        }
    }
    // PD check of the state block (LLT pivots; NaN pivots pass as in Eigen)
    {
        double L[45];
        int idx = 0;
        for (int i = 0; i < 9; i++)
            for (int j = 0; j <= i; j++) L[idx++] = q[QS_Q + i * 9 + j];
        for (int j = 0; j < 9; j++) {
            int jj = j * (j + 1) / 2;
            double dgn = L[jj + j];
            for (int m = 0; m < j; m++) dgn -= L[jj + m] * L[jj + m];
            if (dgn <= 0) { flag |= 2; break; }
            dgn = sqrt(dgn);
            L[jj + j] = dgn;
            for (int i = j + 1; i < 9; i++) {
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
        for (int j = 0; j < 8; j++) {
            q[QS_r + j] = Tu[j] * fu[j];
            q[QS_R + j] = Tu[j] * fuu[j] * Tu[j];
        }
        // ddq cost (osqp_interface.cpp:166-217)
        if (k != N - 1) {
            const double* un = gb + 17 * (k + 1) + 9;
            double sq = 0;
            for (int j = 0; j < DOF; j++) sq += (un[j] - uk[j]) * (un[j] - uk[j]);
            objd = rddq * sq;
        }
        for (int j = 0; j < DOF; j++) {
            double gg;
            if (k == 0) gg = 2. * rddq * (uk[j] - gb[17 * (k + 1) + 9 + j]);
            else if (k == N - 1) gg = 2. * rddq * (uk[j] - gb[17 * (k - 1) + 9 + j]);
            else gg = 2. * rddq * (2. * uk[j] - gb[17 * (k + 1) + 9 + j] - gb[17 * (k - 1) + 9 + j]);
            q[QS_r + j] += Tu[j] * gg;
            double cii = (k == 0 || k == N - 1) ? 2. * rddq : 4. * rddq;
            q[QS_R + j] += Tu[j] * cii * Tu[j];
        }
        for (int j = 0; j < 8; j++) if (isnan(q[QS_R + j])) flag |= 1;
        // dynamics offset b_k = -c_{k+1} = -Tx^-1 (x_{k+1} - (A x_k + B u_k + g))   (:247)
        const double* xn = gb + 17 * (k + 1);
        for (int a = 0; a < 9; a++) {
            double s1 = 0, s2 = 0;
            for (int m = 0; m < 9; m++) s1 += c.A[a * 9 + m] * xk[m];
            for (int m = 0; m < 8; m++) s2 += c.B[a * 8 + m] * uk[m];
            double pred = s1 + s2 + 0.0;
            q[QS_B + a] = -((1.0 / Tx[a]) * (xn[a] - pred));
        }
        // ddq rows (setBounds :279-297): v_0[j] (k=0) or v_k[j]-v_{k-1}[j] within (l - c) / coef
        for (int j = 0; j < DOF; j++) {
            double coef = 1. / p.Ts * Tu[j];
            double cc, lo, hi;
            if (k == 0) {
                cc = 1. / p.Ts * uk[j];
                lo = p.lddq[j] + 1. / p.Ts * ucur[j];
                hi = p.uddq[j] + 1. / p.Ts * ucur[j];
            } else {
                cc = 1. / p.Ts * (uk[j] - gb[17 * (k - 1) + 9 + j]);
                lo = p.lddq[j];
                hi = p.uddq[j];
            }
            q[QS_DLB + j] = (lo - cc) / coef;
            q[QS_DUB + j] = (hi - cc) / coef;
        }
        // polytopic rows (setPolytopicConstraints :302-344); upper bound 0 - c, lower -INF
        int np = 0;
        for (int r = 0; r < NPC; r++) {
            double val, a[7], bv[7];
            if (!poly_row(c, uk, rv, r, &val, true, a, bv)) continue;
            double* row = q + QS_POLY + POLY_W * np;
            for (int j = 0; j < 7; j++) { row[j] = a[j]; row[7 + j] = bv[j]; }
            row[14] = 0.0 - val;
            np++;
        }
        q[QS_NPOLY] = (double)np;
    } else {
        for (int j = 0; j < 8; j++) { q[QS_r + j] = 0.0; q[QS_R + j] = 0.0; }
        for (int a = 0; a < 9; a++) q[QS_B + a] = 0.0;
        for (int j = 0; j < 7; j++) { q[QS_DLB + j] = -INF; q[QS_DUB + j] = INF; }
        q[QS_NPOLY] = 0.0;
    }
    // box on y_k: state bounds (bounds.cpp:85-103, s trust region) intersected with the Q1 rows
    // (input bounds placed on stacked-state columns NU*i, osqp_interface.cpp:273)
    const double L = c.spl.L;
    for (int m = 0; m < 9; m++) {
        double lo = p.lx[m], hi = p.ux[m];
        bool lo_inf = lo <= -BIG, hi_inf = hi >= BIG;
        if (m == 7) { lo = fmax(xk[7] - p.s_trust_region, 0.); hi = fmin(xk[7] + p.s_trust_region, L); lo_inf = hi_inf = false; }
        double ylo = lo_inf ? -INF : (lo - xk[m]) / Tx[m];
        double yhi = hi_inf ? INF : (hi - xk[m]) / Tx[m];
        const int idx = 9 * k + m;
        const int i = idx / 8, j = idx % 8;
        if (i < N) {
            const double ui = gb[17 * i + 9 + j];
            if (p.lu[j] > -BIG) ylo = fmax(ylo, (p.lu[j] - ui) / Tu[j]);
            if (p.uu[j] < BIG) yhi = fmin(yhi, (p.uu[j] - ui) / Tu[j]);
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
}

__global__ void __launch_bounds__(64) k_setqp(DevConst c, DevBuffers d, const double* __restrict__ ucur_all) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c.S) return;
    const int N = c.N;
    const int b = t / (N + 1), k = t - b * (N + 1);
    if (!d.sqi[(size_t)b * SQI + SQ_ACTIVE]) return;
    const double* gb = d.guess + (size_t)b * (N + 1) * 17;
    RecView rv{d.rec + t, c.S};
    double* q = d.qs + (size_t)t * QS;
    setqp_stage(c, gb, rv, k, ucur_all + 8 * b, q);
}

// ------------------------------------------------------------------------------------------------
// k_ipm: Mehrotra predictor-corrector interior point for the stage-structured QP of one instance,
// one wavefront per instance.  Step systems are solved by a Riccati recursion over the augmented
// stage state z~ = [y(9), w(7)] (w_k = v_{k-1}[0:7] carries the ddq coupling) with input v(8).
// Matches oracle/mpcc_oracle.cpp solve_struct_ipm (same algorithm, tolerances and iteration rule).
// ------------------------------------------------------------------------------------------------
constexpr int IPM_MAX_IT = 60;
constexpr double IPM_TOL_MU = 1e-13, IPM_TOL_P = 1e-11, IPM_TOL_STEP = 1e-11;

struct IpmShared {
    double M[81], G[72];
    double P[256], PB[128], PM[81], F[64], Gm[128], Hb[81], U[128];
    double st[QS];                 // staged stage record
    double W[NSLOT];
    double pv[2][16];              // backward vector recursion
    double fv[8];
    double xv[2][16];              // forward rollout
    double hv[8];
    double red[4];
};

// c_i^T z_k for slot i (unsigned) — z points at the stage's 24-vector [y, w, v]
__device__ __forceinline__ double slot_cz(int i, int k, const double* z, const double* qsk) {
    if (i < 9) return z[i];
    if (i < 18) return z[i - 9];
    if (i < 32) {
        int j = (i < 25) ? i - 18 : i - 25;
        return (k == 0) ? z[16 + j] : z[16 + j] - z[9 + j];
    }
    const double* row = qsk + QS_POLY + POLY_W * (i - 32);
    double s = 0;
#pragma unroll
    for (int j = 0; j < 7; j++) s += row[j] * z[j] + row[7 + j] * z[16 + j];
    return s;
}
__device__ __forceinline__ double slot_sgn(int i) { return (i < 9 || (i >= 18 && i < 25)) ? -1.0 : 1.0; }

__global__ void __launch_bounds__(64) k_ipm(DevConst c, DevBuffers d) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    int32_t* si = d.sqi + (size_t)b * SQI;
    if (!si[SQ_ACTIVE]) return;
    __shared__ IpmShared sh;
    const int N = c.N, NS = N + 1;
    const double* QSb = d.qs + (size_t)b * NS * QS;
    double* ISb = d.is + (size_t)b * NS * IS;
    for (int e = lane; e < 81; e += 64) sh.M[e] = c.M[e];
    for (int e = lane; e < 72; e += 64) sh.G[e] = c.G[e];
    const double* Tu = c.p.Tu;
    const double rddq = c.p.qp_r_ddq;

    // ---- Hessian checks (osqp_interface.cpp:454-473): state blocks (flags from k_setqp) and the
    // per-component tridiagonal input blocks.
    int fl = 0;
    for (int k = lane; k < NS; k += 64) fl |= (int)QSb[(size_t)k * QS + QS_FLAG];
    if (lane < 8) {
        const int j = lane;
        double prev_d = 0;
        for (int k = 0; k < N; k++) {
            double dk = QSb[(size_t)k * QS + QS_R + j];
            double off = (k >= 1 && j < DOF) ? (Tu[j] * (-2. * rddq) * Tu[j]) : 0.0;
            double l = (k >= 1) ? off / prev_d : 0.0;
            double dd = dk - l * l;
            if (dd <= 0) { fl |= 2; break; }
            prev_d = sqrt(dd);
        }
    }
    fl = wave_or(fl);
    if (fl & 2) {
        if (lane == 0) { si[SQ_STATUS] = MPCC_NON_PD_HESSIAN; si[SQ_ACTIVE] = 0; }
        return;
    }
    if (fl & 1) {
        if (lane == 0) { si[SQ_STATUS] = MPCC_NAN_HESSIAN; si[SQ_ACTIVE] = 0; }
        return;
    }
    if (fl & 4) {  // constant rows violated / empty box: OSQP reports primal infeasibility; keep step (Q6)
        if (lane == 0) si[SQ_QPSTAT] = MPCC_QP_PrimalInfeasible;
        return;
    }

    // ---- slot setup: bounds, active flags; z = dynamics rollout with v = 0; s, lambda
    const int nslots = NS * NSLOT;
    double mcount = 0;
    for (int e = lane; e < nslots; e += 64) {
        const int k = e / NSLOT, i = e - k * NSLOT;
        const double* q = QSb + (size_t)k * QS;
        double bnd;
        bool act;
        if (i < 18) {
            bnd = (i < 9) ? q[QS_YLB + i] : q[QS_YUB + i - 9];
            act = (k >= 1) && fabs(bnd) < BIG;
        } else if (i < 32) {
            bnd = (i < 25) ? q[QS_DLB + i - 18] : q[QS_DUB + i - 25];
            act = (k < N) && fabs(bnd) < BIG;
        } else {
            int r = i - 32;
            int np = (int)q[QS_NPOLY];
            bnd = (r < np) ? q[QS_POLY + POLY_W * r + 14] : INF;
            act = (k < N) && (r < np) && fabs(bnd) < BIG;
        }
        double* is = ISb + (size_t)k * IS;
        is[IS_BND + i] = bnd;
        is[IS_ACT + i] = act ? 1.0 : 0.0;
        mcount += act ? 1.0 : 0.0;
    }
    mcount = wave_sum(mcount);
    // rollout
    if (lane < 16) sh.xv[0][lane] = 0.0;
    for (int e = lane; e < NS * 24; e += 64) ISb[(size_t)(e / 24) * IS + IS_Z + (e % 24)] = 0.0;
    __syncthreads();
    for (int k = 0; k < N; k++) {
        const double* q = QSb + (size_t)k * QS;
        double yn = 0;
        if (lane < 9) {
            double s = 0;
            for (int m = 0; m < 9; m++) s += sh.M[lane * 9 + m] * sh.xv[k & 1][m];
            yn = s + q[QS_B + lane];
        }
        __syncthreads();
        if (lane < 9) {
            sh.xv[(k + 1) & 1][lane] = yn;
            ISb[(size_t)(k + 1) * IS + IS_Z + lane] = yn;
        }
        __syncthreads();
    }
    for (int e = lane; e < nslots; e += 64) {
        const int k = e / NSLOT, i = e - k * NSLOT;
        double* is = ISb + (size_t)k * IS;
        if (is[IS_ACT + i] != 0.0) {
            double g = slot_sgn(i) * slot_cz(i, k, is + IS_Z, QSb + (size_t)k * QS) - slot_sgn(i) * is[IS_BND + i];
            is[IS_S + i] = fmax(-g, 1.0);
            is[IS_L + i] = 1.0;
        } else {
            is[IS_S + i] = 1.0;
            is[IS_L + i] = 0.0;
        }
    }
    __syncthreads();

    double last_dz = 1e30;
    bool conv = false;
    int it;
    const double HcBase = -2. * rddq;
    for (it = 0; it < IPM_MAX_IT; it++) {
        // ---- pass A: primal residuals, complementarity, barrier weights
        double mus = 0, rpm = 0;
        for (int e = lane; e < nslots; e += 64) {
            const int k = e / NSLOT, i = e - k * NSLOT;
            double* is = ISb + (size_t)k * IS;
            if (is[IS_ACT + i] == 0.0) { is[IS_W + i] = 0.0; continue; }
            double sg = slot_sgn(i);
            double rp = sg * slot_cz(i, k, is + IS_Z, QSb + (size_t)k * QS) - sg * is[IS_BND + i] + is[IS_S + i];
            is[IS_RP + i] = rp;
            mus += is[IS_S + i] * is[IS_L + i];
            rpm = fmax(rpm, fabs(rp));
            is[IS_W + i] = is[IS_L + i] / is[IS_S + i];
        }
        mus = wave_sum(mus);
        rpm = wave_max(rpm);
        const double mu = (mcount > 0) ? mus / mcount : 0.0;
        if (it > 0 && mu < IPM_TOL_MU && rpm < IPM_TOL_P && last_dz < IPM_TOL_STEP) { conv = true; break; }
        // ---- objective gradient g0 = H z + h (per stage component)
        for (int e = lane; e < NS * 24; e += 64) {
            const int k = e / 24, a = e - k * 24;
            const double* q = QSb + (size_t)k * QS;
            double* is = ISb + (size_t)k * IS;
            const double* z = is + IS_Z;
            double g = 0;
            if (a < 9) {
                double s = 0;
                for (int m = 0; m < 9; m++) s += q[QS_Q + a * 9 + m] * z[m];
                g = s + q[QS_q + a];
            } else if (a < 16) {
                int j = a - 9;
                g = (k >= 1 && k <= N - 1) ? (Tu[j] * HcBase * Tu[j]) * z[16 + j] : 0.0;
            } else if (k < N) {
                int j = a - 16;
                g = q[QS_R + j] * z[a] + q[QS_r + j];
                if (k >= 1 && j < DOF) g += (Tu[j] * HcBase * Tu[j]) * z[9 + j];
            }
            is[IS_G0 + a] = g;
        }
        __syncthreads();

        // ---- Riccati factorization with barrier-augmented stage Hessians
        // terminal stage: P = [[Q_N + diag(W_y), 0], [0, 0]]
        {
            const double* q = QSb + (size_t)N * QS;
            const double* is = ISb + (size_t)N * IS;
            for (int e = lane; e < 256; e += 64) {
                int a = e >> 4, cc = e & 15;
                double v = 0;
                if (a < 9 && cc < 9) {
                    v = q[QS_Q + a * 9 + cc];
                    if (a == cc) v += is[IS_W + SL_YL + a] + is[IS_W + SL_YU + a];
                }
                sh.P[e] = v;
            }
        }
        __syncthreads();
        for (int k = N - 1; k >= 0; k--) {
            const double* q = QSb + (size_t)k * QS;
            double* is = ISb + (size_t)k * IS;
            for (int e = lane; e < QS; e += 64) sh.st[e] = q[e];
            if (lane < NSLOT) sh.W[lane] = is[IS_W + lane];
            // (1) PB = P B~ (16x8), PM = P_yy M (9x9)
            for (int e = lane; e < 128 + 81; e += 64) {
                if (e < 128) {
                    int a = e >> 3, j = e & 7;
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sh.P[a * 16 + m] * sh.G[m * 8 + j];
                    if (j < 7) s += sh.P[a * 16 + 9 + j];
                    sh.PB[e] = s;
                } else {
                    int e2 = e - 128, a = e2 / 9, cc = e2 - a * 9;
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sh.P[a * 16 + m] * sh.M[m * 9 + cc];
                    sh.PM[e2] = s;
                }
            }
            __syncthreads();
            const int np = (int)sh.st[QS_NPOLY];
            // (2) F = R~ + B~^T P B~, Gm = S~ + B~^T P A~, Hb_yy = Q~_yy + M^T P_yy M
            for (int e = lane; e < 64 + 128 + 81; e += 64) {
                if (e < 64) {
                    int i = e >> 3, j = e & 7;
                    double rt = 0;
                    if (i == j) {
                        rt = sh.st[QS_R + i];
                        if (i < 7) rt += sh.W[SL_DL + i] + sh.W[SL_DU + i];
                    }
                    if (i < 7 && j < 7)
                        for (int r = 0; r < np; r++) {
                            const double* row = sh.st + QS_POLY + POLY_W * r;
                            rt += sh.W[SL_P + r] * row[7 + i] * row[7 + j];
                        }
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sh.G[m * 8 + i] * sh.PB[m * 8 + j];
                    if (i < 7) s += sh.PB[(9 + i) * 8 + j];
                    sh.F[e] = rt + s;
                } else if (e < 192) {
                    int e2 = e - 64, i = e2 >> 4, cc = e2 & 15;
                    double v;
                    if (cc < 9) {
                        double st_ = 0;
                        if (i < 7 && cc < 7)
                            for (int r = 0; r < np; r++) {
                                const double* row = sh.st + QS_POLY + POLY_W * r;
                                st_ += sh.W[SL_P + r] * row[7 + i] * row[cc];
                            }
                        double s = 0;
                        for (int m = 0; m < 9; m++) s += sh.PB[m * 8 + i] * sh.M[m * 9 + cc];
                        v = st_ + s;
                    } else {
                        int j = cc - 9;
                        v = 0;
                        if (i == j && k >= 1) v = Tu[j] * HcBase * Tu[j] - (sh.W[SL_DL + j] + sh.W[SL_DU + j]);
                    }
                    sh.Gm[e2] = v;
                } else {
                    int e2 = e - 192, a = e2 / 9, cc = e2 - a * 9;
                    double v = sh.st[QS_Q + a * 9 + cc];
                    if (a == cc) v += sh.W[SL_YL + a] + sh.W[SL_YU + a];
                    if (a < 7 && cc < 7)
                        for (int r = 0; r < np; r++) {
                            const double* row = sh.st + QS_POLY + POLY_W * r;
                            v += sh.W[SL_P + r] * row[a] * row[cc];
                        }
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sh.M[m * 9 + a] * sh.PM[m * 9 + cc];
                    sh.Hb[e2] = v + s;
                }
            }
            __syncthreads();
            // (3) LF = chol(F) (every lane, registers); U = LF^-1 Gm (lane = column)
            double Lf[36];
            {
                int idx = 0;
#pragma unroll
                for (int i = 0; i < 8; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) Lf[idx++] = sh.F[i * 8 + j];
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
                    double s = sh.Gm[i * 16 + lane];
#pragma unroll
                    for (int m = 0; m < i; m++) s -= Lf[ii + m] * u[m];
                    u[i] = s / Lf[ii + i];
                }
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    sh.U[i * 16 + lane] = u[i];
                    is[IS_U + i * 16 + lane] = u[i];
                }
            } else if (lane < 16 + 36) {
                // spread the packed factor to global (one entry per lane, select from registers)
                const int e = lane - 16;
                double v = 0;
#pragma unroll
                for (int m = 0; m < 36; m++) v = (m == e) ? Lf[m] : v;
                is[IS_LF + e] = v;
            }
            __syncthreads();
            // (4) P = Hb - U^T U  (not needed at k = 0)
            if (k > 0) {
                for (int e = lane; e < 256; e += 64) {
                    int a = e >> 4, cc = e & 15;
                    double v = 0;
                    if (a < 9 && cc < 9) v = sh.Hb[a * 9 + cc];
                    else if (a >= 9 && a == cc) v = (sh.W[SL_DL + a - 9] + sh.W[SL_DU + a - 9]);
                    double s = 0;
#pragma unroll
                    for (int i = 0; i < 8; i++) s += sh.U[i * 16 + a] * sh.U[i * 16 + cc];
                    sh.P[e] = v - s;
                }
            }
            __syncthreads();
        }

        // ---- two solves (predictor, corrector) with the same factorization
        double sigma_mu = 0.0;
        double alpha = 0.0, dzmax = 0.0;
        for (int phase = 0; phase < 2; phase++) {
            // slot pass: rc, signed coefficient for the gradient
            for (int e = lane; e < nslots; e += 64) {
                const int k = e / NSLOT, i = e - k * NSLOT;
                double* is = ISb + (size_t)k * IS;
                if (is[IS_ACT + i] == 0.0) { is[IS_COEF + i] = 0.0; continue; }
                double s = is[IS_S + i], l = is[IS_L + i];
                double rc = (phase == 0) ? s * l : s * l + is[IS_DSA + i] * is[IS_DLA + i] - sigma_mu;
                is[IS_RC + i] = rc;
                double coef = l + is[IS_W + i] * is[IS_RP + i] - rc / s;
                is[IS_COEF + i] = slot_sgn(i) * coef;
            }
            __syncthreads();
            // gradient of the step system
            for (int e = lane; e < NS * 24; e += 64) {
                const int k = e / 24, a = e - k * 24;
                const double* q = QSb + (size_t)k * QS;
                double* is = ISb + (size_t)k * IS;
                double g = is[IS_G0 + a];
                const double* sc = is + IS_COEF;
                const int np = (k < N) ? (int)q[QS_NPOLY] : 0;
                if (a < 9) {
                    g += sc[SL_YL + a] + sc[SL_YU + a];
                    if (a < 7)
                        for (int r = 0; r < np; r++) g += sc[SL_P + r] * q[QS_POLY + POLY_W * r + a];
                } else if (a < 16) {
                    int j = a - 9;
                    if (k >= 1 && k < N) g -= sc[SL_DL + j] + sc[SL_DU + j];
                } else if (k < N) {
                    int j = a - 16;
                    if (j < 7) {
                        g += sc[SL_DL + j] + sc[SL_DU + j];
                        for (int r = 0; r < np; r++) g += sc[SL_P + r] * q[QS_POLY + POLY_W * r + 7 + j];
                    }
                }
                is[IS_G + a] = g;
            }
            __syncthreads();
            // backward vector recursion: p_N = g_x~(N); f = g_v + B~^T p; t = LF^-1 f; p = g_x~ + A~^T p - U^T t
            if (lane < 16) sh.pv[N & 1][lane] = ISb[(size_t)N * IS + IS_G + lane];
            __syncthreads();
            for (int k = N - 1; k >= 0; k--) {
                double* is = ISb + (size_t)k * IS;
                const double* pn = sh.pv[(k + 1) & 1];
                if (lane < 8) {
                    double s = 0;
                    for (int m = 0; m < 9; m++) s += sh.G[m * 8 + lane] * pn[m];
                    if (lane < 7) s += pn[9 + lane];
                    sh.fv[lane] = is[IS_G + 16 + lane] + s;
                }
                __syncthreads();
                double Lf[36], t[8];
#pragma unroll
                for (int m = 0; m < 36; m++) Lf[m] = is[IS_LF + m];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int ii = i * (i + 1) / 2;
                    double s = sh.fv[i];
#pragma unroll
                    for (int m = 0; m < i; m++) s -= Lf[ii + m] * t[m];
                    t[i] = s / Lf[ii + i];
                }
                if (lane < 8) {
                    double tv = 0;
#pragma unroll
                    for (int m = 0; m < 8; m++) tv = (m == lane) ? t[m] : tv;
                    is[IS_T + lane] = tv;
                }
                if (k > 0 && lane < 16) {
                    double s = is[IS_G + lane];
                    if (lane < 9)
                        for (int m = 0; m < 9; m++) s += sh.M[m * 9 + lane] * pn[m];
#pragma unroll
                    for (int i = 0; i < 8; i++) s -= is[IS_U + i * 16 + lane] * t[i];
                    sh.pv[k & 1][lane] = s;
                }
                __syncthreads();
            }
            // forward rollout: x~_0 = 0; v = -LF^-T (U x~ + t); x~_{k+1} = A~ x~ + B~ v
            if (lane < 16) sh.xv[0][lane] = 0.0;
            __syncthreads();
            double dzm = 0.0;
            for (int k = 0; k < N; k++) {
                double* is = ISb + (size_t)k * IS;
                const double* xc = sh.xv[k & 1];
                if (lane < 8) {
                    double s = is[IS_T + lane];
                    for (int a = 0; a < 16; a++) s += is[IS_U + lane * 16 + a] * xc[a];
                    sh.hv[lane] = s;
                }
                __syncthreads();
                double Lf[36], v[8];
#pragma unroll
                for (int m = 0; m < 36; m++) Lf[m] = is[IS_LF + m];
#pragma unroll
                for (int i = 7; i >= 0; i--) {
                    double s = sh.hv[i];
#pragma unroll
                    for (int m = i + 1; m < 8; m++) s -= Lf[m * (m + 1) / 2 + i] * v[m];
                    v[i] = s / Lf[i * (i + 1) / 2 + i];
                }
#pragma unroll
                for (int i = 0; i < 8; i++) v[i] = -v[i];
                if (lane < 16) {
                    double xn;
                    if (lane < 9) {
                        double s = 0;
                        for (int m = 0; m < 9; m++) s += sh.M[lane * 9 + m] * xc[m];
                        for (int j = 0; j < 8; j++) s += sh.G[lane * 8 + j] * v[j];
                        xn = s;
                    } else {
                        double vv = 0;
#pragma unroll
                        for (int j = 0; j < 7; j++) vv = (j == lane - 9) ? v[j] : vv;
                        xn = vv;
                    }
                    sh.xv[(k + 1) & 1][lane] = xn;
                    is[IS_DZ + lane] = xc[lane];
                    dzm = fmax(dzm, fabs(xc[lane]));
                } else if (lane < 24) {
                    double vv = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) vv = (j == lane - 16) ? v[j] : vv;
                    is[IS_DZ + lane] = vv;
                    dzm = fmax(dzm, fabs(vv));
                }
                __syncthreads();
            }
            if (lane < 24) {
                double v = (lane < 16) ? sh.xv[N & 1][lane] : 0.0;
                ISb[(size_t)N * IS + IS_DZ + lane] = v;
                dzm = fmax(dzm, fabs(v));
            }
            __syncthreads();
            // slot pass: recover ds, dl; step length
            double amax = (phase == 0) ? 1.0 : 1e30;
            for (int e = lane; e < nslots; e += 64) {
                const int k = e / NSLOT, i = e - k * NSLOT;
                double* is = ISb + (size_t)k * IS;
                if (is[IS_ACT + i] == 0.0) continue;
                double cd = slot_sgn(i) * slot_cz(i, k, is + IS_DZ, QSb + (size_t)k * QS);
                double rp = is[IS_RP + i];
                double s = is[IS_S + i], l = is[IS_L + i];
                double ds = -rp - cd;
                double dl = is[IS_W + i] * (cd + rp) - is[IS_RC + i] / s;
                if (phase == 0) { is[IS_DSA + i] = ds; is[IS_DLA + i] = dl; }
                else { is[IS_DS + i] = ds; is[IS_DL + i] = dl; }
                if (ds < 0) amax = fmin(amax, -s / ds);
                if (dl < 0) amax = fmin(amax, -l / dl);
            }
            amax = wave_min(amax);
            if (phase == 0) {
                double mua = 0;
                for (int e = lane; e < nslots; e += 64) {
                    const int k = e / NSLOT, i = e - k * NSLOT;
                    const double* is = ISb + (size_t)k * IS;
                    if (is[IS_ACT + i] == 0.0) continue;
                    mua += (is[IS_S + i] + amax * is[IS_DSA + i]) * (is[IS_L + i] + amax * is[IS_DLA + i]);
                }
                mua = wave_sum(mua);
                mua = (mcount > 0) ? mua / mcount : 0.0;
                double ratio = (mu > 0) ? mua / mu : 0.0;
                double sigma = (mu > 0) ? ratio * ratio * ratio : 0.0;
                sigma_mu = sigma * mu;
            } else {
                alpha = fmin(1.0, 0.995 * amax);
                dzmax = wave_max(dzm);
            }
            __syncthreads();
        }
        // ---- update
        for (int e = lane; e < NS * 24; e += 64) {
            const int k = e / 24, a = e - k * 24;
            double* is = ISb + (size_t)k * IS;
            is[IS_Z + a] += alpha * is[IS_DZ + a];
        }
        for (int e = lane; e < nslots; e += 64) {
            const int k = e / NSLOT, i = e - k * NSLOT;
            double* is = ISb + (size_t)k * IS;
            if (is[IS_ACT + i] == 0.0) continue;
            is[IS_S + i] += alpha * is[IS_DS + i];
            is[IS_L + i] += alpha * is[IS_DL + i];
        }
        last_dz = dzmax;
        __syncthreads();
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
        const double* z = ISb + (size_t)k * IS + IS_Z;
        stp[e] = (a < 9) ? z[a] : ((k < N) ? z[16 + a - 9] : 0.0);
    }
}

// ------------------------------------------------------------------------------------------------
// k_trial: filterLineSearch trial (osqp_interface.cpp:759-808) — objective and l1 constraint
// violation (:824-833) of setQP(obj, constr) at guess + alpha * T * step, one lane per stage.
// Rows owned by stage k: dynamics block k, state bounds k, input bounds (Q1) k, ddq block k,
// polytopic block k.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_trial(DevConst c, DevBuffers d, const double* __restrict__ ucur_all,
                                             double alpha, int dead) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c.S) return;
    const int N = c.N;
    const int b = t / (N + 1), k = t - b * (N + 1);
    const int32_t* si = d.sqi + (size_t)b * SQI;
    if (!si[SQ_ACTIVE]) return;
    if (dead && !si[SQ_REJECT]) return;  // dead trials only follow a rejected alpha = 1
    const mpcc_params& p = c.p;
    const double* gb = d.guess + (size_t)b * (N + 1) * 17;
    const double* sb = d.step + (size_t)b * (N + 1) * 17;
    auto tx = [&](int i, int a) { return gb[17 * i + a] + alpha * (p.Tx[a] * sb[17 * i + a]); };
    auto tu = [&](int i, int a) { return (i < N) ? gb[17 * i + 9 + a] + alpha * (p.Tu[a] * sb[17 * i + 9 + a]) : gb[17 * i + 9 + a]; };
    double x[9], u[8];
    for (int a = 0; a < 9; a++) x[a] = tx(k, a);
    for (int a = 0; a < 8; a++) u[a] = tu(k, a);
    RecView rv{d.rec + t, c.S};
    double fdum[9], udum[8], hdum[81], rdum[8];
    double obj = stage_cost(c, x, u, rv, k, false, fdum, udum, hdum, rdum);
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
        double xp[9], up_[8];
        for (int a = 0; a < 9; a++) xp[a] = tx(k - 1, a);
        for (int a = 0; a < 8; a++) up_[a] = tu(k - 1, a);
        for (int a = 0; a < 9; a++) {
            double s1 = 0, s2 = 0;
            for (int m = 0; m < 9; m++) s1 += c.A[a * 9 + m] * xp[m];
            for (int m = 0; m < 8; m++) s2 += c.B[a * 8 + m] * up_[m];
            double cv = (1.0 / p.Tx[a]) * (x[a] - (s1 + s2 + 0.0));
            lo += vfloor(fmax(0.0 - cv, 0.0), vf);
            up += vfloor(fmax(cv - 0.0, 0.0), vf);
        }
    }
    for (int a = 0; a < 9; a++) {  // state bounds
        double l = p.lx[a], h = p.ux[a];
        if (a == 7) { l = fmax(x[7] - p.s_trust_region, 0.); h = fmin(x[7] + p.s_trust_region, c.spl.L); }
        lo += vfloor(fmax(l - x[a], 0.0), vf);
        up += vfloor(fmax(x[a] - h, 0.0), vf);
    }
    if (k < N) {
        for (int a = 0; a < 8; a++) {  // input bounds (constr = u, :274)
            lo += vfloor(fmax(p.lu[a] - u[a], 0.0), vf);
            up += vfloor(fmax(u[a] - p.uu[a], 0.0), vf);
        }
        for (int j = 0; j < DOF; j++) {  // ddq rows
            double cv, l, h;
            if (k == 0) {
                cv = 1. / p.Ts * u[j];
                l = p.lddq[j] + 1. / p.Ts * ucur_all[8 * b + j];
                h = p.uddq[j] + 1. / p.Ts * ucur_all[8 * b + j];
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
    if (dead) return;  // faithful evaluation of a discarded trial: results are not used
    double* tr = d.trial + (size_t)t * 4;
    tr[0] = obj;
    tr[1] = objd;
    tr[2] = lo;
    tr[3] = up;
}

// ------------------------------------------------------------------------------------------------
// k_accept: filter decision, step, termination (osqp_interface.cpp:540-574, 759-808)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_accept(DevConst c, DevBuffers d) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= c.Bn) return;
    int32_t* si = d.sqi + (size_t)b * SQI;
    if (!si[SQ_ACTIVE]) return;
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
}

// take step (osqp_interface.cpp:549-573): guess += alpha * deNormalizeStep(step); termination test
__global__ void __launch_bounds__(64) k_apply(DevConst c, DevBuffers d) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= c.Bn) return;
    int32_t* si = d.sqi + (size_t)b * SQI;
    if (!si[SQ_ACTIVE]) return;
    const int N = c.N;
    const mpcc_params& p = c.p;
    double* sd = d.sqd + (size_t)b * SQ;
    const double alpha = sd[SQ_ALPHA];
    double* g = d.guess + (size_t)b * (N + 1) * 17;
    const double* st = d.step + (size_t)b * (N + 1) * 17;
    double nrm = 0;
    for (int k = 0; k <= N; k++) {
        for (int a = 0; a < 9; a++) {
            g[17 * k + a] = g[17 * k + a] + alpha * (p.Tx[a] * st[17 * k + a]);
            nrm = fmax(nrm, fabs(st[17 * k + a]));
        }
        if (k < N)
            for (int a = 0; a < 8; a++) {
                g[17 * k + 9 + a] = g[17 * k + 9 + a] + alpha * (p.Tu[a] * st[17 * k + 9 + a]);
                nrm = fmax(nrm, fabs(st[17 * k + 9 + a]));
            }
    }
    const double pn = alpha * nrm;
    int iter = si[SQ_ITER];
    if (pn < p.eps_prim) {
        si[SQ_STATUS] = MPCC_SOLVED;
        si[SQ_ACTIVE] = 0;
        si[SQ_ITER] = iter;
        return;
    }
    iter++;
    si[SQ_ITER] = iter;
    if (iter >= p.max_iter) {
        si[SQ_STATUS] = MPCC_MAX_ITER_EXCEEDED;
        si[SQ_ACTIVE] = 0;
    }
}

// ------------------------------------------------------------------------------------------------
// k_finalize: opt_sol / zero_guess, controller bookkeeping and outputs (osqp_interface.cpp:575-589,
// mpc.cpp:136-189)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_finalize(DevConst c, DevBuffers d) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= c.Bn) return;
    const int N = c.N;
    int32_t* si = d.sqi + (size_t)b * SQI;
    const int status = si[SQ_STATUS];
    double* g = d.guess + (size_t)b * (N + 1) * 17;
    if (status != MPCC_SOLVED) {  // zero_guess: x_0 repeated, u = 0
        double x0[9];
        for (int a = 0; a < 9; a++) x0[a] = g[a];
        for (int k = 0; k <= N; k++) {
            for (int a = 0; a < 9; a++) g[17 * k + a] = x0[a];
            for (int a = 0; a < 8; a++) g[17 * k + 9 + a] = 0.0;
        }
    } else {
        for (int a = 0; a < 8; a++) g[17 * N + 9 + a] = 0.0;
    }
    int fails = d.fails[b];
    if (status == MPCC_SOLVED) { d.valid[b] = 1; fails = 0; }
    else { d.valid[b] = 0; fails++; }
    d.fails[b] = fails;
    if (d.status) d.status[b] = status;
    if (d.ok) d.ok[b] = (status == MPCC_SOLVED || (status == MPCC_MAX_ITER_EXCEEDED && fails < 5)) ? 1 : 0;
    if (d.u0_out)
        for (int a = 0; a < 8; a++) d.u0_out[8 * b + a] = g[9 + a];
    if (d.horizon)
        for (int e = 0; e < (N + 1) * 17; e++) d.horizon[(size_t)b * (N + 1) * 17 + e] = g[e];
}

// ------------------------------------------------------------------------------------------------
// closed-loop simulator step (Integrator::simTimeStep, integrator.cpp:55-68: 10 x RK4 at 1 ms)
// ------------------------------------------------------------------------------------------------
__global__ void k_sim_step(int B, const double* __restrict__ x, const double* __restrict__ u, double ts, double* __restrict__ xn) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xc[9], uu[8];
    for (int a = 0; a < 9; a++) xc[a] = x[9 * b + a];
    for (int a = 0; a < 8; a++) uu[a] = u[8 * b + a];
    const double fine = 0.001;
    int steps = (int)(ts / fine);
    for (int i = 0; i < steps; i++) {
        double t[9];
        rk4_step(xc, uu, fine, t);
        for (int a = 0; a < 9; a++) xc[a] = t[a];
    }
    for (int a = 0; a < 9; a++) xn[9 * b + a] = xc[a];
}

// ---- debug kernels (stage-level parity) ----
__global__ void k_debug_records(DevConst c, int M, const double* __restrict__ qin, const double* __restrict__ obsin,
                                double* __restrict__ rec) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M) return;
    double q[7], pos[3], R[9], J[42];
    for (int j = 0; j < 7; j++) q[j] = qin[7 * t + j];
    panda_fk(q, pos, R, J, true);
    for (int a = 0; a < 3; a++) rec[(size_t)(R_POS + a) * M + t] = pos[a];
    for (int a = 0; a < 9; a++) rec[(size_t)(R_ROT + a) * M + t] = R[a];
    for (int a = 0; a < 42; a++) rec[(size_t)(R_J + a) * M + t] = J[a];
    rec[(size_t)R_MU * M + t] = manip_from_J(J);
    const double delta = 1e-4;
    for (int i = 0; i < 7; i++) {
        double qp[7], qm[7];
        for (int j = 0; j < 7; j++) { qp[j] = q[j] + (j == i ? delta : 0.0); qm[j] = q[j] - (j == i ? delta : 0.0); }
        rec[(size_t)(R_DMU + i) * M + t] = (manipulability(qp) - manipulability(qm)) / (2 * delta);
    }
    const double inf = __longlong_as_double(0x7ff0000000000000LL);
    if (!(c.p.constraint_mask & MPCC_CON_SELFCOL)) {
        rec[(size_t)R_SEL * M + t] = inf;
        for (int j = 0; j < 7; j++) rec[(size_t)(R_DSEL + j) * M + t] = 0.0;
    }
    rec[(size_t)R_OBSR * M + t] = obsin[4 * t + 3];
    if (!(c.p.constraint_mask & MPCC_CON_ENVCOL)) {
        for (int m = 0; m < 9; m++) rec[(size_t)(R_ENV + m) * M + t] = inf;
        for (int m = 0; m < 63; m++) rec[(size_t)(R_DENV + m) * M + t] = 0.0;
    }
}

__global__ void k_debug_spline(DevConst c, int M, const double* __restrict__ sv, double* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M) return;
    double* o = out + (size_t)t * 21;
    spline_pos3(c.spl, sv[t], o, o + 3, o + 6);
    spline_rot(c.spl, sv[t], o + 9, o + 18);
}

__global__ void k_debug_cost(DevConst c, int M, const double* __restrict__ x, const double* __restrict__ u,
                             const double* __restrict__ rec, const int32_t* __restrict__ kk, double* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M) return;
    RecView rv{rec + t, M};
    double* o = out + (size_t)t * (1 + 9 + 8 + 81 + 64);
    double fuu[8];
    o[0] = stage_cost(c, x + 9 * t, u + 8 * t, rv, kk[t], true, o + 1, o + 10, o + 18, fuu);
    for (int i = 0; i < 64; i++) o[99 + i] = 0.0;
    for (int i = 0; i < 8; i++) o[99 + 9 * i] = fuu[i];
}

// ------------------------------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------------------------------
static inline int nblk(long n, int t) { return (int)((n + t - 1) / t); }

void launch_prepare(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_prepare, dim3(nblk(c.Bn, 64)), dim3(64), 0, s, c, d);
}
void launch_stage_records(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_records, dim3(nblk(c.S, 64)), dim3(64), 0, s, c, d);
}
void launch_setqp(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s) {
    hipLaunchKernelGGL(k_setqp, dim3(nblk(c.S, 64)), dim3(64), 0, s, c, d, u_cur);
}
void launch_ipm(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_ipm, dim3(c.Bn), dim3(64), 0, s, c, d);
}
void launch_trial(const DevConst& c, const DevBuffers& d, const double* u_cur, double alpha, int dead, hipStream_t s) {
    hipLaunchKernelGGL(k_trial, dim3(nblk(c.S, 64)), dim3(64), 0, s, c, d, u_cur, alpha, dead);
}
void launch_accept(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_accept, dim3(nblk(c.Bn, 64)), dim3(64), 0, s, c, d);
}
void launch_apply(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_apply, dim3(nblk(c.Bn, 64)), dim3(64), 0, s, c, d);
}
void launch_nn(const DevConst& c, const DevBuffers& d, const NNDesc& nd, const double* W, int which, int M,
               const double* q, const double* obs, double* rec, int rec_stride, hipStream_t s) {
    hipLaunchKernelGGL(k_nn, dim3(M), dim3(64), 0, s, c, d, nd, W, which, M, q, obs, rec, rec_stride);
}
void launch_debug_records(const DevConst& c, int M, const double* q, const double* obs, double* rec, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_records, dim3(nblk(M, 64)), dim3(64), 0, s, c, M, q, obs, rec);
}
void launch_finalize(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3(nblk(c.Bn, 64)), dim3(64), 0, s, c, d);
}
void launch_sim_step(int B, const double* x, const double* u, double ts, double* xn, hipStream_t s) {
    hipLaunchKernelGGL(k_sim_step, dim3(nblk(B, 64)), dim3(64), 0, s, B, x, u, ts, xn);
}
void launch_debug_spline(const DevConst& c, int M, const double* sv, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_spline, dim3(nblk(M, 64)), dim3(64), 0, s, c, M, sv, out);
}
void launch_debug_cost(const DevConst& c, int M, const double* x, const double* u, const double* rec, const int32_t* k,
                       double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_cost, dim3(nblk(M, 64)), dim3(64), 0, s, c, M, x, u, rec, k, out);
}

}  // namespace mpcc
