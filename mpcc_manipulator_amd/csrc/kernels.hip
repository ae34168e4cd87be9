// kernels.hip — HIP kernels of the MI355X batched MPCC solve engine (gfx950, FP64).
//
// One batch call = one MPC::runMPC_ (cpp/src/MPC/mpc.cpp:104-190) for each of B independent
// controllers.  Kernel sequence:
//   k_prepare      thread / instance        projection, vs estimate, warm-start shift  (mpc.cpp:104-124, 54-89)
//   k_records      RPT threads / (instance,stage) RobotData::update: FK, J, manipulability + FD gradient (robot_data.h:55-71)
//   k_mlp_*        (mlp.hip) 2 samples / wave, FP64 MFMA: self / env collision MLPs + input Jacobians
//   per SQP iteration (osqp_interface.cpp:431-574):
//     k_setqp      thread / (instance,stage) stage QP record: cost, constraint rows, bounds, dynamics residual
//     k_ipm        wave / instance           Mehrotra interior point, Riccati factorization (replaces OSQP)
//     k_trial      thread / (instance,stage) filter line-search trial at alpha = 1 (objective, violation)
//     k_accept     thread / instance         filter, step, termination
//   k_finalize     thread / horizon element  Status -> warm start / outputs (osqp_interface.cpp:575-589, mpc.cpp:140-189)
#include <algorithm>

#include "dev_sqp.h"
#include "dev_records.h"

namespace mpcc {

// ------------------------------------------------------------------------------------------------
// k_prepare
// ------------------------------------------------------------------------------------------------
// MPC::runMPC_ before solveOCP (mpc.cpp:104-124, 54-89): projection, vs estimate, guess shift.  PL lanes per
// instance: every lane of the group evaluates the projection and the vs estimate (the same values), then the group
// writes the new guess element-parallel.  One lane per instance spent most of the kernel on dependent memory round
// trips: the stage-by-stage shift (a load, wait and store per stage) and the unwrap re-reading what the shift had
// just stored.
constexpr int PL = 16;          // lanes per instance (one DPP row, in lockstep within the wave)
constexpr int PREP_BATCH = 16;  // guess elements per lane loaded before any is stored
__device__ inline void prepare_mpc(const DevConst& c, const DevBuffers& d, int b, int j) {
    const int N = c.N;
    double x[NX], u[NU];
#pragma unroll
    for (int i = 0; i < NX; i++) x[i] = d.x0[NX * b + i];
#pragma unroll
    for (int i = 0; i < NU; i++) u[i] = d.u0[NU * b + i];
    const double last_s = x[XS];
    double ee[3], J[6 * DOF];
    robot_fk(x, ee, nullptr, J, true);
    const SplineView sp = spl_of(c.spl, b);
    x[XS] = project_on_spline(sp, c.p.proj_max_dist, last_s, ee);
    double ev[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double s = 0;
#pragma unroll
        for (int jj = 0; jj < DOF; jj++) s += J[DOF * i + jj] * u[jj];
        ev[i] = s;
    }
    double dir[3];
    spline_pos3(sp, x[XS], nullptr, dir, nullptr);
    x[XVS] = ev[0] * dir[0] + ev[1] * dir[1] + ev[2] * dir[2];
    int valid = d.valid[b], fails = d.fails[b];
    if (fabs(last_s - x[XS]) > c.p.guess_max_dist) { valid = 0; fails++; }
    if (j == 0 && d.order) d.order[order_slots(c.Bn) + b] = valid ? 0 : 1;  // cold start this step (k_order)
    double* g = d.guess + (size_t)b * (N + 1) * NXU;
    // updateInitialGuess (mpc.cpp:54-68) element by element: stage i < N takes old stage min(i, N - 2) + 1 (the shift,
    // then g[N-1] = g[N-2]) with the state of stage 0 replaced by x; stage N is RK4 of the new stage N - 1 with a zero
    // input.  generateNewInitialGuess (:79-89): every stage [x, 0].  unwrapInitialGuess: s of stages >= 1 clamped to
    // the track length.  N = 1 keeps stage 0's input (the reference's g[N-1] = g[N-2] reads g[-1] there).
    double xN[NX];
    {
        double gN[NXU];  // the new stage N - 1, read before any store
#pragma unroll
        for (int a = 0; a < NXU; a++) gN[a] = g[NXU * (N - 1) + a];
        if (N <= 2) {
#pragma unroll
            for (int a = 0; a < NX; a++) gN[a] = x[a];
        }
        rk4_step(gN, gN + NX, c.p.Ts, xN);
    }
    const int NE = (N + 1) * NXU;
    for (int e0 = 0; e0 < NE; e0 += PL * PREP_BATCH) {
        double v[PREP_BATCH];
#pragma unroll
        for (int r = 0; r < PREP_BATCH; r++) {
            const int e = e0 + PL * r + j;
            const int i = e / NXU, a = e - i * NXU;
            const int ii = i < N - 2 ? i : N - 2;  // source stage - 1 (-1 when N = 1)
            const int src = (e < NE && i < N) ? (ii + 1) * NXU + a : 0;
            double w = g[src];
            double xa = 0.0;
#pragma unroll
            for (int q = 0; q < NX; q++) xa = (a == q) ? x[q] : xa;
            double xna = 0.0;
#pragma unroll
            for (int q = 0; q < NX; q++) xna = (a == q) ? xN[q] : xna;
            if (valid) {
                if (i == N) w = (a < NX) ? xna : 0.0;
                else if (ii <= 0 && a < NX) w = xa;
            } else {
                w = (a < NX) ? xa : 0.0;
            }
            if (i >= 1 && a == XS) w = fmin(w, sp.L);
            v[r] = w;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every old element of the batch read before the stores
#pragma unroll
        for (int r = 0; r < PREP_BATCH; r++) {
            const int e = e0 + PL * r + j;
            if (e < NE) g[e] = v[r];
        }
    }
    if (!valid) valid = 1;
    if (j == 0) {
#pragma unroll
        for (int i = 0; i < NX; i++) d.x0[NX * b + i] = x[i];
        d.valid[b] = valid;
        d.fails[b] = fails;
    }
}

__global__ void __launch_bounds__(64) k_prepare(DevConst c, DevBuffers d) {
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = gt / PL, j = gt % PL;
    if (b >= c.Bn) return;  // whole groups
    const int N = c.N;
    if (!c.ocp) prepare_mpc(c, d, b, j);
    int32_t* si = d.sqi + (size_t)b * SQI;
    if (j == 0) {
        si[SQ_STATUS] = MPCC_MAX_ITER_EXCEEDED;
        si[SQ_ACTIVE] = 1;
        si[SQ_ITER] = 0;
        si[SQ_NFILT] = 0;
        si[SQ_QPSTAT] = 0;
        si[SQ_IPMIT] = 0;
        si[SQ_NLR] = 0;
    }
    double* st = d.step + (size_t)b * (N + 1) * NXU;
    for (int i = j; i < (N + 1) * NXU; i += PL) st[i] = 0.0;  // step_.setZero (osqp_interface.cpp:404)
}

// ------------------------------------------------------------------------------------------------
// k_records: FK, Jacobian, manipulability and its central-difference gradient (15 Jacobians).
// ------------------------------------------------------------------------------------------------
// The instance of record group t0 of a launch over c.subset (early solo blocks, engine.cpp run_batch): 0 record t0,
// 1 stage t0 mod (N+1) of solo block t0 / (N+1)'s instance (d.order slot 4 r; -1 when the block has none), 2 record t0
// unless its instance is in a solo block (k_order marks those 2 in the cold flags).  Returns the record index or -1;
// the whole group of a record returns together.
__device__ __forceinline__ int subset_record(const DevConst& c, const DevBuffers& d, int t0) {
    const int NS = c.N + 1;
    if (c.subset == 1) {
        const int r = t0 / NS;
        const int b = r < NSOLO ? d.order[4 * r] : -1;
        return b < 0 ? -1 : b * NS + (t0 - r * NS);
    }
    if (t0 >= c.S) return -1;
    if (c.subset == 2 && d.order[order_slots(c.Bn) + t0 / NS] == 2) return -1;
    return t0;
}
__host__ __device__ inline long subset_records(const DevConst& c) { return c.subset == 1 ? (long)NSOLO * (c.N + 1) : c.S; }
__global__ void __launch_bounds__(64) k_records(DevConst c, DevBuffers d) {
    const long g_t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int S = c.S;
    const int t0 = (int)(g_t / RPT), u = (int)(g_t % RPT);
    bool live = t0 < S;
    int tr = t0;
    if (c.subset) {  // whole record groups of 16 (RPT) lanes leave together
        tr = subset_record(c, d, t0);
        if (tr < 0) return;
        live = true;
    }
    const int t = live ? tr : S - 1;  // every lane of a record group evaluates (the split form exchanges values)
    record_group(c, d, t, u, live);
}

// ------------------------------------------------------------------------------------------------
// k_setqp: stage QP record (setqp_stage, dev_sqp.h), one lane per (instance, stage)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_setqp(DevConst, DevBuffers, const double* __restrict__ ucur_all) {
    // the arguments read in place (kernels.h kernarg_const): setqp_stage indexes the params' bound arrays at a
    // lane-dependent position, which on a by-value parameter made the compiler copy it into the private segment
    const DevConst& c = kernarg_const();
    const DevBuffers& d = kernarg_buffers();
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (c.subset) {
        t = subset_record(c, d, t);
        if (t < 0) return;
    } else if (t >= c.S) {
        return;
    }
    const int N = c.N;
    const int b = t / (N + 1), k = t - b * (N + 1);
    if (!d.sqi[(size_t)b * SQI + SQ_ACTIVE]) return;
    const double* gb = d.guess + (size_t)b * (N + 1) * NXU;
    RecView rv{d.rec + t, c.S};
    double* q = d.qs + (size_t)t * QS;
    setqp_stage(c, spl_of(c.spl, b), gb, rv, k, ucur_all + NU * b, q);
}

// k_soc: the SecondOrderCorrection bounds of each (instance, stage) record (soc_stage, dev_sqp.h)
__global__ void __launch_bounds__(64) k_soc(DevConst c, DevBuffers d, const double* __restrict__ ucur_all) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c.S) return;
    const int N = c.N;
    const int b = t / (N + 1), k = t - b * (N + 1);
    if (!d.sqi[(size_t)b * SQI + SQ_ACTIVE]) return;
    const size_t o = (size_t)b * (N + 1) * NXU;
    soc_stage(c, spl_of(c.spl, b), d.guess + o, d.step + o, RecView{d.rec + t, c.S}, k, ucur_all + NU * b,
              d.qs + (size_t)t * QS);
}

// ------------------------------------------------------------------------------------------------
// k_trial / k_accept / k_apply: filter line search and step (dev_sqp.h) as lane-per-stage and
// lane-per-instance kernels; k_sqp (ipm.hip) runs the same pieces per instance inside the QP kernel.
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
    double out[4];
    trial_stage(c, d, b, k, alpha, ucur_all + NU * b, out);
    if (dead) return;  // faithful evaluation of a discarded trial: results are not used
    double* tr = d.trial + (size_t)t * 4;
    for (int i = 0; i < 4; i++) tr[i] = out[i];
}

__global__ void __launch_bounds__(64) k_accept(DevConst c, DevBuffers d) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= c.Bn) return;
    if (!d.sqi[(size_t)b * SQI + SQ_ACTIVE]) return;
    accept_instance(c, d, b);
}

__global__ void __launch_bounds__(64) k_apply(DevConst c, DevBuffers d) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= c.Bn) return;
    if (!d.sqi[(size_t)b * SQI + SQ_ACTIVE]) return;
    const double alpha = d.sqd[(size_t)b * SQ + SQ_ALPHA];
    double nrm = 0;
    for (int e = 0; e < (c.N + 1) * NXU; e++) nrm = fmax(nrm, apply_elem(c, d, b, e, alpha));
    finish_iteration(c, d, b, nrm);
}

// ------------------------------------------------------------------------------------------------
// k_finalize: opt_sol / zero_guess, controller bookkeeping and outputs (osqp_interface.cpp:575-589,
// mpc.cpp:136-189)
// ------------------------------------------------------------------------------------------------
// opt_sol / zero_guess element-wise (thread per horizon element, coalesced): a non-SOLVED instance gets
// x_0 repeated with u = 0 (osqp_interface.cpp:422-428), a SOLVED one u_N = 0; the horizon output is the
// result.  x_0 itself (k = 0, a < NX) is never rewritten, so the threads that read it do not race.  One launch per solve: thread (instance b, element r of the opt_sol / zero_guess horizon).  The element
// threads of stage 0's inputs also write u0 (the value they store); thread r = 0 writes the status and the MPC
// bookkeeping (mpc.cpp:143-189).
__global__ void __launch_bounds__(64) k_finalize(DevConst c, DevBuffers d) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int W = (c.N + 1) * NXU;
    if (e >= (long)c.Bn * W) return;
    const int b = (int)(e / W), r = (int)(e - (long)b * W);
    const int k = r / NXU, a = r - NXU * k;
    double* g = d.guess + (size_t)b * W;
    const int status = d.sqi[(size_t)b * SQI + SQ_STATUS];
    const bool solved = status == MPCC_SOLVED;
    double v = g[r];
    if (!solved) v = (a < NX) ? g[a] : 0.0;
    else if (k == c.N && a >= NX) v = 0.0;
    if (!(k == 0 && a < NX)) g[r] = v;
    if (d.horizon) d.horizon[(size_t)b * W + r] = v;
    if (k == 0 && a >= NX && d.u0_out) d.u0_out[(size_t)NU * b + (a - NX)] = v;
    if (r != 0) return;
    if (d.status) d.status[b] = status;
    if (c.ocp) {  // solveOCP's return value only; the MPC bookkeeping belongs to the caller
        if (d.ok) d.ok[b] = solved ? 1 : 0;
    } else {
        int fails = d.fails[b];
        if (solved) { d.valid[b] = 1; fails = 0; }
        else { d.valid[b] = 0; fails++; }
        d.fails[b] = fails;
        if (d.ok) d.ok[b] = (solved || (status == MPCC_MAX_ITER_EXCEEDED && fails < 5)) ? 1 : 0;
    }
}

// ------------------------------------------------------------------------------------------------
// closed-loop simulator step (Integrator::simTimeStep, integrator.cpp:55-68: 10 x RK4 at 1 ms)
// ------------------------------------------------------------------------------------------------
__global__ void k_sim_step(int B, const double* __restrict__ x, const double* __restrict__ u, double ts, double* __restrict__ xn) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xc[NX], uu[NU];
    for (int a = 0; a < NX; a++) xc[a] = x[NX * b + a];
    for (int a = 0; a < NU; a++) uu[a] = u[NU * b + a];
    const double fine = 0.001;
    int steps = (int)(ts / fine);
    for (int i = 0; i < steps; i++) {
        double t[NX];
        rk4_step(xc, uu, fine, t);
        for (int a = 0; a < NX; a++) xc[a] = t[a];
    }
    for (int a = 0; a < NX; a++) xn[NX * b + a] = xc[a];
}

// ---- device closed loop (main.cpp:100-114; mpcc_closed_loop).  The step index lives in device memory
//      so that one captured control step (hipGraph) can be replayed: k_loop_tick advances it.
__global__ void k_loop_pre(int B, const double* __restrict__ x, double* __restrict__ xtraj, const int* __restrict__ kstep) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const size_t o = ((size_t)*kstep * B + b) * NX;
    for (int a = 0; a < NX; a++) xtraj[o + a] = x[NX * b + a];
}
// after runMPC_: a live instance takes u0 and integrates the state runMPC_ updated (simTimeStep); an
// instance whose runMPC_ returned false stops (main.cpp:108-112) — its state is frozen at the state
// that entered the failing step and later steps report status -1
__global__ void k_loop_post(int B, double ts, double* __restrict__ x, double* __restrict__ u,
                            const double* __restrict__ xtraj, const double* __restrict__ u0out,
                            const int32_t* __restrict__ status, const int32_t* __restrict__ ok, int32_t* __restrict__ alive,
                            double* __restrict__ utraj, int32_t* __restrict__ straj, const int* __restrict__ kstep) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int k = *kstep;
    const bool live = alive[b] != 0;
    const bool go = live && ok[b] != 0;
    if (go) {
        double xc[NX], uu[NU];
        for (int a = 0; a < NU; a++) uu[a] = u0out[NU * b + a];
        for (int a = 0; a < NX; a++) xc[a] = x[NX * b + a];
        const int steps = (int)(ts / 0.001);
        for (int i = 0; i < steps; i++) {
            double t[NX];
            rk4_step(xc, uu, 0.001, t);
            for (int a = 0; a < NX; a++) xc[a] = t[a];
        }
        for (int a = 0; a < NX; a++) x[NX * b + a] = xc[a];
        for (int a = 0; a < NU; a++) u[NU * b + a] = uu[a];
    } else {
        for (int a = 0; a < NX; a++) x[NX * b + a] = xtraj[((size_t)k * B + b) * NX + a];
    }
    if (live && !go) alive[b] = 0;
    straj[(size_t)k * B + b] = live ? status[b] : -1;
    for (int a = 0; a < NU; a++) utraj[((size_t)k * B + b) * NU + a] = u[NU * b + a];
}
__global__ void k_loop_tick(int* kstep) { *kstep += 1; }

// ---- debug kernels (stage-level parity) ----
__global__ void k_debug_records(DevConst c, int M, const double* __restrict__ qin, const double* __restrict__ obsin,
                                double* __restrict__ rec) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M) return;
    double q[DOF];
    for (int j = 0; j < DOF; j++) q[j] = qin[DOF * t + j];
    robot_record(c, q, obsin[4 * t + 3], rec + t, (size_t)M);
}

__global__ void k_debug_spline(DevConst c, int M, const double* __restrict__ sv, double* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M) return;
    double* o = out + (size_t)t * 21;
    const SplineView sp = spl_of(c.spl, 0);
    spline_pos3(sp, sv[t], o, o + 3, o + 6);
    spline_rot(sp, sv[t], o + 9, o + 18);
}

__global__ void k_debug_project(DevConst c, int M, const double* __restrict__ sg, const double* __restrict__ ee,
                                double* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M) return;
    out[t] = project_on_spline(spl_of(c.spl, 0), c.p.proj_max_dist, sg[t], ee + 3 * t);
}

__global__ void k_debug_cost(DevConst c, int M, const double* __restrict__ x, const double* __restrict__ u,
                             const double* __restrict__ rec, const int32_t* __restrict__ kk, double* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= M) return;
    RecView rv{rec + t, M};
    double* o = out + (size_t)t * (1 + NX + NU + NX * NX + NU * NU);
    double fuu[NU];
    double* fuuo = o + 1 + NX + NU + NX * NX;
    o[0] = stage_cost(c, spl_of(c.spl, 0), x + NX * t, u + NU * t, rv, kk[t], true, o + 1, o + 1 + NX, o + 1 + NX + NU, fuu);
    for (int i = 0; i < NU * NU; i++) fuuo[i] = 0.0;
    for (int i = 0; i < NU; i++) fuuo[(NU + 1) * i] = fuu[i];
}

// ------------------------------------------------------------------------------------------------
// k_order: k_sqp's group slots.  The first NSOLO cold-started instances (ascending) get slot 4 r of wave r, alone in
// it; every other instance (ascending) is packed 4 per wave after them; unused slots hold -1.  One wave: it runs
// between the other controller group's k_sqp waves, which hold every VGPR of their SIMDs (a 1024-thread block had
// to wait for a whole CU to drain: up to 1.1 ms, profiles/r04z_kernel_stats.csv).  Chunks of 64 instances, the cold
// count before each lane by ballot, 8 chunks' flags loaded ahead.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_order(DevConst c, DevBuffers d) {
    const int Bn = c.Bn, NSL = order_slots(Bn);
    int32_t* slot = d.order;
    int32_t* cold = d.order + NSL;
    const int lane = threadIdx.x;
    for (int i = lane; i < NSL; i += 64) slot[i] = -1;
    __syncthreads();  // the -1 stores land before any slot's instance
    const unsigned long long below = (1ull << lane) - 1;
    int cb = 0;  // cold instances before the chunk
    for (int base = 0; base < Bn; base += 8 * 64) {
        int fl[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int b = base + q * 64 + lane;
            fl[q] = b < Bn ? cold[b] : 0;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int b = base + q * 64 + lane;
            const bool cd = fl[q] != 0;
            const unsigned long long m = __ballot(cd);
            const int before = cb + __popcll(m & below);
            if (b < Bn) {
                if (cd && before < NSOLO) {
                    slot[4 * before] = b;
                    cold[b] = 2;  // in a solo block (k_records / k_setqp subsets)
                }
                else slot[4 * NSOLO + b - min(before, NSOLO)] = b;
            }
            cb += __popcll(m);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------------------------------
static inline int nblk(long n, int t) { return (int)((n + t - 1) / t); }

void launch_prepare(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_prepare, dim3(nblk((long)c.Bn * PL, 64)), dim3(64), 0, s, c, d);
}
void launch_order(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_order, dim3(1), dim3(64), 0, s, c, d);
}
void launch_stage_records(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    hipLaunchKernelGGL(k_records, dim3(nblk(subset_records(c) * RPT, 64)), dim3(64), 0, s, c, d);
}
void launch_setqp(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s) {
    hipLaunchKernelGGL(k_setqp, dim3(nblk(subset_records(c), 64)), dim3(64), 0, s, c, d, u_cur);
}
void launch_soc(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s) {
    hipLaunchKernelGGL(k_soc, dim3(nblk(c.S, 64)), dim3(64), 0, s, c, d, u_cur);
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
void launch_debug_records(const DevConst& c, int M, const double* q, const double* obs, double* rec, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_records, dim3(nblk(M, 64)), dim3(64), 0, s, c, M, q, obs, rec);
}
void launch_finalize(const DevConst& c, const DevBuffers& d, hipStream_t s) {
    // one-wave workgroups: a multi-wave workgroup waits for room on every SIMD of a CU, which the concurrent
    // controller groups' k_sqp waves (a whole SIMD's registers each) do not leave until they finish: 256-thread
    // blocks of this kernel ran 0.5-1.3 ms behind another group's interior point (profiles/r03aj trace)
    hipLaunchKernelGGL(k_finalize, dim3(nblk((long)c.Bn * (c.N + 1) * NXU, 64)), dim3(64), 0, s, c, d);
}
__global__ void __launch_bounds__(64) k_warmstart_copy(long ng, const double* __restrict__ g, double* __restrict__ gd, int B,
                                                         const int32_t* __restrict__ v, int32_t* __restrict__ vd,
                                                         const int32_t* __restrict__ f, int32_t* __restrict__ fd) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g)
        for (long e = i; e < ng; e += (long)gridDim.x * blockDim.x) gd[e] = g[e];
    if (i < B) {
        if (v) vd[i] = v[i];
        if (f) fd[i] = f[i];
    }
}
void launch_warmstart_copy(long ng, const double* g, double* gd, int B, const int32_t* v, int32_t* vd, const int32_t* f,
                           int32_t* fd, hipStream_t s) {
    const long n = ng > B ? ng : B;
    if (n <= 0) return;
    // grid-stride over the guess; valid / fails one element per thread, so at least ceil(B / 64) one-wave blocks
    const long cap = std::max(16384L, ((long)B + 63) / 64);
    const long blocks = std::min((n + 63) / 64, cap);
    hipLaunchKernelGGL(k_warmstart_copy, dim3((int)blocks), dim3(64), 0, s, ng, g, gd, B, v, vd, f, fd);
}
void launch_sim_step(int B, const double* x, const double* u, double ts, double* xn, hipStream_t s) {
    hipLaunchKernelGGL(k_sim_step, dim3(nblk(B, 64)), dim3(64), 0, s, B, x, u, ts, xn);
}
void launch_loop_pre(int B, const double* x, double* xtraj, const int* kstep, hipStream_t s) {
    hipLaunchKernelGGL(k_loop_pre, dim3(nblk(B, 64)), dim3(64), 0, s, B, x, xtraj, kstep);
}
void launch_loop_post(int B, double ts, double* x, double* u, const double* xtraj, const double* u0out,
                      const int32_t* status, const int32_t* ok, int32_t* alive, double* utraj, int32_t* straj,
                      int* kstep, hipStream_t s) {
    hipLaunchKernelGGL(k_loop_post, dim3(nblk(B, 64)), dim3(64), 0, s, B, ts, x, u, xtraj, u0out, status, ok, alive,
                       utraj, straj, kstep);
    hipLaunchKernelGGL(k_loop_tick, dim3(1), dim3(1), 0, s, kstep);
}
void launch_debug_project(const DevConst& c, int M, const double* sg, const double* ee, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_project, dim3(nblk(M, 64)), dim3(64), 0, s, c, M, sg, ee, out);
}
void launch_debug_spline(const DevConst& c, int M, const double* sv, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_spline, dim3(nblk(M, 64)), dim3(64), 0, s, c, M, sv, out);
}
void launch_debug_cost(const DevConst& c, int M, const double* x, const double* u, const double* rec, const int32_t* k,
                       double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_cost, dim3(nblk(M, 64)), dim3(64), 0, s, c, M, x, u, rec, k, out);
}

}  // namespace mpcc
