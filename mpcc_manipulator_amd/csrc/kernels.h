// kernels.h — host-side launch wrappers of the engine's HIP kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "dev_common.h"

namespace mpcc {

// host: one layer of a collision network from disk (engine.cpp), and the thread's last-error message
bool nn_read_layer(const std::string& dir, int l, int R, int C, std::vector<double>& W, std::vector<double>& b);
void set_last_error(const std::string& m);

struct DevBuffers {
    // per-call I/O (device)
    double* x0;        // [B*9]  in/out
    const double* u0;  // [B*8]
    const double* obs; // [B*4]
    double* u0_out;    // [B*8]
    double* horizon;   // [B*(N+1)*17]
    int32_t* status;   // [B]
    int32_t* ok;       // [B]
    // persistent controller state
    double* guess;     // [maxB*(N+1)*17]
    int32_t* valid;    // [maxB]
    int32_t* fails;    // [maxB]
    // workspaces
    double* rec;       // [REC * maxB*(N+1)]  SoA
    double* qs;        // [maxB*(N+1)*QS]
    double* is;        // [maxB*(N+1)*IS]
    double* step;      // [maxB*(N+1)*17]
    double* trial;     // [maxB*(N+1)*4]  per stage: obj, vio_lo, vio_up, spare
    int32_t* sqi;      // [maxB*SQI]
    double* sqd;       // [maxB*SQ]
    // NN weights (device)
    const double* nn_self;  // packed W0,b0,W1,b1,W2,b2
    const double* nn_env;   // packed W0,b0,...,W4,b4
    // debug: per-instance SQP trace (null unless mpcc_debug_trace_enable), TRACE_W doubles per iteration
    double* dbg_trace;
    // 32-lane interior point (ipm_wide.hip): workspace [maxB*(N+1)*ISW] — the mobile build's QP solver, and the
    // damped-BFGS option of either build
    double* isw;
    // damped BFGS (use_BFGS, osqp_interface.cpp:437-453, 683-715), per instance, horizon layout [(N+1)][NXU]:
    // low-rank vectors lr [lrs][(N+1)*NXU] and coefficients lrc [lrs], A^T lambda (glam), grad_L of the previous
    // iteration (gprev), A^T y of the last QP (aty), step_prev = alpha * step (sp)
    double *lr, *lrc, *glam, *gprev, *aty, *sp;
    // more than LRM low-rank terms (max_iter > 1 + LRM / 2): per term and stage the Woodbury column Q_j = M u_j (x~
    // and v parts) and the kff of its backward solve, [lrs][(N+1)][3][32 lanes]; null unless lrs > LRM
    double* lrq;
    // k_sqp's instance of each 16-lane group slot ([4 * (ceil(Bn / 4) + NSOLO)], -1: none) followed by the per-instance
    // cold-start flags of this step ([Bn], written by k_prepare); k_order builds the slots (solo waves)
    int32_t* order;
    // ComputeTime split of the fused SQP kernels (mpcc_timing; osqp_interface.cpp:435-564): per-phase wave cycles
    // summed over a launch's waves, [PH_SETQP, PH_SOLVE, PH_ALPHA, PH_STEP]; null unless timing is on
    unsigned long long* phase_cyc;
    // low-rank terms allocated per instance (the stride of lr / lrc / lrq): the terms max_iter can produce,
    // min(LRX, 2 (max_iter - 1)), rounded up to a multiple of 4 (>= LRM); 0 without use_BFGS
    int lrs;
};
constexpr int PH_SETQP = 0, PH_SOLVE = 1, PH_ALPHA = 2, PH_STEP = 3, PH_N = 4;
// per-wave phase clock of the fused SQP kernels: mark(i) books the cycles since the previous mark to phase i; one
// atomic add per phase and wave at the end (lane 0); nothing when timing is off
struct PhaseClock {
    unsigned long long* const out;
    long long t0 = 0, acc[PH_N] = {0, 0, 0, 0};
    __device__ explicit PhaseClock(unsigned long long* o) : out(o) {
        if (out) t0 = clock64();
    }
    __device__ __forceinline__ void mark(int i) {
        if (!out) return;
        const long long t = clock64();
        acc[i] += t - t0;
        t0 = t;
    }
    __device__ __forceinline__ void flush(bool lane0) {
        if (!out || !lane0) return;
        for (int i = 0; i < PH_N; i++) atomicAdd(&out[i], (unsigned long long)acc[i]);
    }
};
// Cold-started controllers (a regenerated initial guess) are the ones that take a second SQP iteration; k_sqp
// gives each of the first NSOLO of them a wave of its own (tail mode from its first IPM iteration), so that they do
// not set the launch's length from inside a 4-instance wave; with solo blocks (DevConst::solo 2)
// k_sqp_solo runs those waves instead, each as a block of two waves (§3.7)
constexpr int NSOLO = 64;
__host__ __device__ inline int order_slots(int Bn) { return 4 * ((Bn + 3) / 4 + NSOLO); }
// The fused SQP kernels (k_sqp of ipm.hip / ipm_wide.hip) are declared (DevConst c, DevBuffers d, const double*)
// and hand c and d to their non-inlined phases by reference into the kernel-argument segment: a reference to the
// by-value parameter itself makes the compiler copy the 5.4 KB DevConst into every lane's private segment (a
// 5.8 KB per-lane stack frame) and read it back through flat private-aperture loads in the interior point.
static_assert(sizeof(DevConst) % alignof(DevBuffers) == 0, "DevBuffers follows DevConst in the kernel arguments");
__device__ __forceinline__ const DevConst& kernarg_const() {
    return *(const DevConst*)__builtin_amdgcn_kernarg_segment_ptr();
}
__device__ __forceinline__ const DevBuffers& kernarg_buffers() {
    return *(const DevBuffers*)((const char*)__builtin_amdgcn_kernarg_segment_ptr() + sizeof(DevConst));
}

constexpr int TRACE_W = 8, TRACE_IT = 4;  // qp status, ipm iters, obj, vio, accepted, |step|_inf, alpha, alpha*|step|

constexpr int SQI = 8;  // int bookkeeping per instance: status, active, iter, nfilt, qp_status, ipm_iters, reject, nlr
constexpr int SQ_REJECT = 6;
constexpr int SQ_NLR = 7;  // low-rank BFGS terms held (2 per update)
constexpr int LRM = 4;     // low-rank terms carried in registers through the fused sweeps (use_BFGS, max_iter <= 3)
constexpr int LRX = 28;    // low-rank terms held at most (ipm_wide.hip xl_*); an update past them restarts the
                           // quasi-Newton matrix from that iteration's exact Hessian (bfgs_pre)
// low-rank terms an instance can hold with max_iter SQP iterations (2 per update), as allocated (DevBuffers::lrs)
inline int bfgs_terms(int max_iter) {
    const int n = max_iter > 1 ? 2 * (max_iter - 1) : 0;
    const int r = ((n < LRX ? n : LRX) + 3) / 4 * 4;
    return r < LRM ? LRM : r;
}
constexpr int ISW = 2048;  // doubles per stage of the 32-lane interior point's workspace (64 fields x 32 lanes)

struct NNDesc {
    int L;              // number of layers
    int nin;            // raw input size (7 self, 10 env)
    int dims[6];        // dims[0] = 3*nin ... dims[L] = nout
    long offW[5], offb[5];
};

void launch_prepare(const DevConst& c, const DevBuffers& d, hipStream_t s);
// k_sqp's slot -> instance map from k_prepare's cold-start flags (c.solo launches)
void launch_order(const DevConst& c, const DevBuffers& d, hipStream_t s);
void launch_stage_records(const DevConst& c, const DevBuffers& d, hipStream_t s);
void launch_nn(const DevConst& c, const DevBuffers& d, const NNDesc& nd, const double* W, int which, int M,
               const double* q, const double* obs, double* rec, int rec_stride, hipStream_t s);
void launch_setqp(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s);
void launch_ipm(const DevConst& c, const DevBuffers& d, int npmax, hipStream_t s);
// SecondOrderCorrection bounds (osqp_interface.cpp:658-681) of the stage records, before a second k_ipm
void launch_soc(const DevConst& c, const DevBuffers& d, const double* u_cur, hipStream_t s);
// the fused SQP loop (QP solve, line search, step, next QP assembly) after the first k_setqp
void launch_sqp(const DevConst& c, const DevBuffers& d, const double* u_cur, int npmax, hipStream_t s);
// solo blocks: k_sqp_solo beside a k_sqp launch with c.solo 2; false (nothing launched) where the
// variant has no tail mode
bool launch_sqp_solo(const DevConst& c, const DevBuffers& d, const double* u_cur, int npmax, hipStream_t s);
// the fused SQP loop on the 32-lane interior point (ipm_wide.hip); bfgs = 1: damped BFGS Hessian updates
void launch_sqp_wide(const DevConst& c, const DevBuffers& d, const double* u_cur, int npmax, int bfgs, hipStream_t s);
size_t ipm_wide_lds_bytes(int npmax, bool lr);
void launch_ipm_wide(const DevConst& c, const DevBuffers& d, int npmax, int lr, hipStream_t s);
size_t ipm_lds_bytes(int N, int npmax);
inline int poly_rows_max(int mask) {
    return ((mask & MPCC_CON_SELFCOL) ? 1 : 0) + ((mask & MPCC_CON_SING) ? 1 : 0) + ((mask & MPCC_CON_ENVCOL) ? 9 : 0);
}
void launch_trial(const DevConst& c, const DevBuffers& d, const double* u_cur, double alpha_scale, int dead, hipStream_t s);
void launch_accept(const DevConst& c, const DevBuffers& d, hipStream_t s);
void launch_apply(const DevConst& c, const DevBuffers& d, hipStream_t s);
void launch_finalize(const DevConst& c, const DevBuffers& d, hipStream_t s);
void launch_sim_step(int B, const double* x, const double* u, double ts, double* xn, hipStream_t s);
// device-to-device warm start (guess, valid, fails) in one launch; null sources are skipped
void launch_warmstart_copy(long ng, const double* g, double* gd, int B, const int32_t* v, int32_t* vd, const int32_t* f,
                           int32_t* fd, hipStream_t s);
void launch_loop_pre(int B, const double* x, double* xtraj, const int* kstep, hipStream_t s);
void launch_loop_post(int B, double ts, double* x, double* u, const double* xtraj, const double* u0out,
                      const int32_t* status, const int32_t* ok, int32_t* alive, double* utraj, int32_t* straj,
                      int* kstep, hipStream_t s);
void launch_debug_records(const DevConst& c, int M, const double* q, const double* obs, double* rec, hipStream_t s);
void launch_debug_spline(const DevConst& c, int M, const double* sv, double* out, hipStream_t s);
void launch_debug_project(const DevConst& c, int M, const double* sg, const double* ee, double* out, hipStream_t s);
void launch_debug_cost(const DevConst& c, int M, const double* x, const double* u, const double* rec, const int32_t* k,
                       double* out, hipStream_t s);

}  // namespace mpcc
