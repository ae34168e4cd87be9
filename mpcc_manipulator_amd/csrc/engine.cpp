// engine.cpp — C-ABI implementation (include/mpcc_engine.h): engine object, device memory,
// track upload and the batched runMPC_ launch sequence.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "host_json.h"
#include "host_spline.h"
#include "kernels.h"
#include "mpcc_engine.h"

namespace mpcc {

static thread_local std::string g_last_error;
void set_last_error(const std::string& m) { g_last_error = m; }

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
#define HIPCHK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) throw HipError(std::string(#x) + ": " + hipGetErrorString(e_));              \
    } while (0)

template <class T>
static T* dmalloc(size_t n) {
    void* p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) throw std::bad_alloc();
    return (T*)p;
}

struct NNWeights {
    double* d = nullptr;
    NNDesc desc{};
    bool loaded = false;
};

}  // namespace mpcc

using namespace mpcc;

struct mpcc_engine {
    mpcc_config cfg{};
    // SQP loop: fused per-instance kernel k_sqp (default) or one launch per stage of each iteration
    // (MPCC_STAGED_SQP=1; same arithmetic, kept for A/B timing and debugging)
    bool staged_sqp = false;
    bool wide_sqp = false;  // MPCC_WIDE_SQP=1: the 32-lane fused kernel for the Panda build too (experiment)
    int tail_mode = 1;      // MPCC_TAIL=0: no tail mode in k_sqp (A/B switch; results are bitwise the same)
    int solo_mode = 2;      // MPCC_SOLO: 0 no solo waves for cold starts in k_sqp, 1 solo waves, 2 (default) solo blocks
    int early_solo = 1;     // MPCC_EARLY_SOLO=0: the solo blocks start after every instance's QP records (run_batch)
                            // (narrow variants; A/B switch, bitwise the same)
    bool last_wide = DOF != 7;  // the last solve's interior point ran on the 32-lane workspace (d.isw)
    uint32_t* bchk = nullptr;  // bounds-checked build: per-lane violation bits (dev_common.h MPCC_BCHK)
    mpcc_params params{};
    int N = 0, maxB = 0;
    hipStream_t stream = nullptr;
    hipStream_t solo_stream = nullptr;  // k_sqp_solo (solo blocks), forked from and joined to `stream` per launch
    int simds = 1024;                   // SIMDs of the device (4 per CU)
    hipEvent_t solo_fork = nullptr, solo_join = nullptr;
    hipEvent_t nn_fork = nullptr, nn_join = nullptr;  // the self network on the side stream beside the env network
    int nn_par = 0;  // MPCC_NN_PAR=1: the self network on the side stream beside the env network (A/B; slower)
    SplineTables track;
    bool has_track = false;
    double* d_spl = nullptr;
    SplineDev spl{};
    int n_tracks = 0;  // 1: shared track (stride 0); B: one per instance (mpcc_set_tracks)
    bool ext_async = false;  // a device call was queued on a caller stream since the last quiesce()
    DevBuffers d{};
    // host-API staging
    double *s_x0 = nullptr, *s_u0 = nullptr, *s_obs = nullptr, *s_u0out = nullptr, *s_hor = nullptr;
    int32_t *s_status = nullptr, *s_ok = nullptr;
    NNWeights nn_self, nn_env;
    double A[NX * NX], B[NX * NU], M[NX * NX], G[NX * NU];
    std::vector<hipEvent_t> events;
    // live timing (mpcc_timing_begin/end): event pairs per phase over many calls
    bool live = false;
    std::vector<hipEvent_t> live_pool;
    size_t live_used = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> lv_env, lv_setqp, lv_ipm, lv_alpha, lv_total;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> lv_mlp_self, lv_mlp_env;  // the collision-MLP launches alone
    double last_mlp_self_s = 0, last_mlp_env_s = 0;                         // totals of the last timing window
    int last_mlp_self_n = 0, last_mlp_env_n = 0;
    int live_calls = 0;
    // ComputeTime split of the fused SQP kernel (DevBuffers::phase_cyc): per-phase wave cycles on the device, the
    // k_sqp spans of the last window and their split (mpcc_timing_sqp)
    unsigned long long* d_phase = nullptr;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> lv_sqp;
    double last_sqp_s = 0, last_frac[PH_N] = {0, 0, 0, 0};
    int last_sqp_n = 0;
    // phase fractions from the counters (reset afterwards on stream st); false if nothing was counted
    bool phase_fracs(double (&f)[PH_N], hipStream_t st) {
        unsigned long long h[PH_N];
        HIPCHK(hipMemcpy(h, d_phase, sizeof h, hipMemcpyDeviceToHost));
        HIPCHK(hipMemsetAsync(d_phase, 0, sizeof h, st));
        double sum = 0;
        for (int i = 0; i < PH_N; i++) sum += (double)h[i];
        for (int i = 0; i < PH_N; i++) f[i] = sum > 0 ? (double)h[i] / sum : 0.0;
        return sum > 0;
    }
    hipEvent_t live_ev() {
        if (live_used == live_pool.size()) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            live_pool.push_back(e);
        }
        return live_pool[live_used++];
    }

    ~mpcc_engine() {
        auto f = [](void* p) { if (p) (void)hipFree(p); };
        f(d_spl);
        f(d.guess); f(d.valid); f(d.fails); f(d.rec); f(d.qs); f(d.is); f(d.step); f(d.trial); f(d.sqi); f(d.sqd); f(d.order);
        if (d.isw != d.is) f(d.isw);
        f(d.lr); f(d.lrc); f(d.glam); f(d.gprev); f(d.aty); f(d.sp); f(d.lrq);
        f(d.dbg_trace);
        f(d_phase);
        f(bchk);
        f(s_x0); f(s_u0); f(s_obs); f(s_u0out); f(s_hor); f(s_status); f(s_ok);
        f(nn_self.d); f(nn_env.d);
        for (auto ev : events) (void)hipEventDestroy(ev);
        for (auto ev : live_pool) (void)hipEventDestroy(ev);
        if (stream) (void)hipStreamDestroy(stream);
        if (solo_stream) (void)hipStreamDestroy(solo_stream);
        if (solo_fork) (void)hipEventDestroy(solo_fork);
        if (solo_join) (void)hipEventDestroy(solo_join);
        if (nn_fork) (void)hipEventDestroy(nn_fork);
        if (nn_join) (void)hipEventDestroy(nn_join);
    }

    void set_model() {
        const mpcc_params& p = params;
        // ZOH of the kinematic model (model.cpp:47-91); the (NX+NU)^2 expm is exact in closed form because
        // the continuous A is nilpotent: A = I + Ts e_s e_vs^T, B = Ts [I_DOF 0; 0 Ts/2; 0 1] (dVs column).
        for (int i = 0; i < NX * NX; i++) A[i] = (i % (NX + 1) == 0) ? 1.0 : 0.0;
        for (int i = 0; i < NX * NU; i++) B[i] = 0.0;
        A[XS * NX + XVS] = p.Ts;
        for (int j = 0; j < DOF; j++) B[j * NU + j] = p.Ts;
        B[XS * NU + UVS] = p.Ts * p.Ts / 2.0;
        B[XVS * NU + UVS] = p.Ts;
        for (int a = 0; a < NX; a++) {
            for (int b = 0; b < NX; b++) M[a * NX + b] = (1.0 / p.Tx[a]) * A[a * NX + b] * p.Tx[b];
            for (int b = 0; b < NU; b++) G[a * NU + b] = (1.0 / p.Tx[a]) * B[a * NU + b] * p.Tu[b];
        }
        // the interior point writes the Riccati products for M = diag(m) + m_sv e_s e_vs^T and
        // G = diag(g) + g_v e_vs e_dVs^T (the s row's dVs entry is G's diagonal, XS == UVS)
        for (int a = 0; a < NX; a++) {
            for (int b = 0; b < NX; b++)
                if (M[a * NX + b] != 0.0 && a != b && !(a == XS && b == XVS))
                    throw std::logic_error("discrete model outside the structure k_ipm assumes (M)");
            for (int b = 0; b < NU; b++)
                if (G[a * NU + b] != 0.0 && a != b && !(a == XVS && b == UVS))
                    throw std::logic_error("discrete model outside the structure k_ipm assumes (G)");
        }
    }

    // Buffers of the 32-lane interior point (use_BFGS, MPCC_WIDE_SQP): its workspace (the mobile build's regular
    // one) and, with use_BFGS, the per-instance BFGS state for the low-rank terms max_iter can produce
    // (bfgs_terms: 2 per update, at most LRX; above LRM the Woodbury columns go to memory, d.lrq).  Reallocated
    // when a larger max_iter needs more terms (the stride d.lrs changes; the state is per solve).
    void ensure_wide_buffers(bool bfgs, int max_iter) {
        const size_t B = (size_t)maxB, NE = ((size_t)N + 1) * NXU;
        if (!d.isw) d.isw = dmalloc<double>(B * (N + 1) * ISW);
        if (!bfgs) return;
        // every set is allocated whole before it replaces the engine's pointers: a failed hipMalloc (thrown out of
        // mpcc_set_params, which restores the old params) leaves the previous, consistent buffers in place
        auto fr = [](double*& p) { if (p) (void)hipFree(p); p = nullptr; };
        auto alloc_all = [&](std::initializer_list<std::pair<double**, size_t>> want) {
            std::vector<double*> got;
            try {
                for (const auto& w : want) got.push_back(w.second ? dmalloc<double>(w.second) : nullptr);
            } catch (...) {
                for (double* p : got) fr(p);
                throw;
            }
            size_t i = 0;
            for (const auto& w : want) { fr(*w.first); *w.first = got[i++]; }
        };
        if (!d.glam || !d.gprev || !d.aty || !d.sp)
            alloc_all({{&d.glam, B * NE}, {&d.gprev, B * NE}, {&d.aty, B * NE}, {&d.sp, B * NE}});
        const int lrs = bfgs_terms(max_iter);
        if (lrs > d.lrs) {
            alloc_all({{&d.lr, B * lrs * NE}, {&d.lrc, B * lrs},
                       {&d.lrq, lrs > LRM ? B * lrs * (N + 1) * 3 * 32 : 0}});
            d.lrs = lrs;
        }
    }

    DevConst make_const(int Bn) const {
        DevConst c;
        std::memset(&c, 0, sizeof c);
        c.p = params;
        std::memcpy(c.A, A, sizeof A);
        std::memcpy(c.B, B, sizeof B);
        std::memcpy(c.M, M, sizeof M);
        std::memcpy(c.G, G, sizeof G);
        c.spl = spl;
        c.bchk = bchk;
#ifdef MPCC_BOUNDS_CHECK
        c.spl.err = bchk;
#endif
        c.N = N;
        c.Bn = Bn;
        c.S = Bn * (N + 1);
        c.faithful_dead_trials = cfg.faithful_dead_trials;
        c.tail = tail_mode;
        return c;
    }

    // the solo blocks' side stream, created at their first launch (each stream takes one of the process's few
    // hardware queues); MPCC_SOLO_PRIO=h / l: at the highest / lowest stream priority (A/B)
    hipStream_t side_stream() {
        if (solo_stream) return solo_stream;
        const char* sp = std::getenv("MPCC_SOLO_PRIO");
        if (sp && (sp[0] == 'h' || sp[0] == 'l')) {
            int least = 0, greatest = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIPCHK(hipStreamCreateWithPriority(&solo_stream, hipStreamNonBlocking, sp[0] == 'h' ? greatest : least));
        } else {
            HIPCHK(hipStreamCreateWithFlags(&solo_stream, hipStreamNonBlocking));
        }
        return solo_stream;
    }

    hipEvent_t ev(size_t i) {
        while (events.size() <= i) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            events.push_back(e);
        }
        return events[i];
    }
};

namespace {

// ---- NN weights: binary (manifest.json + *.f64, this repo's data/nn) or the reference's text files
bool read_doubles_bin(const std::string& path, std::vector<double>& out, size_t n) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f || (size_t)f.tellg() != n * sizeof(double)) return false;  // exactly rows x cols values
    f.seekg(0);
    out.resize(n);
    f.read((char*)out.data(), (std::streamsize)(n * sizeof(double)));
    return (bool)f;
}
bool read_doubles_txt(const std::string& path, std::vector<double>& out, size_t n) {
    std::ifstream f(path);
    if (!f) return false;
    out.resize(n);
    for (size_t i = 0; i < n; i++)
        if (!(f >> out[i])) return false;  // operator>> as SelfCollisionModel.cpp:29
    return true;
}

}  // namespace

// Layer l (R x C row-major W, b[R]) of a network under dir: <dir>/weight_l.f64 (this repo's binary
// form), else the reference's text files <dir>/parameter/weight_l.txt or <dir>/weight_l.txt
// (SelfCollisionModel.cpp:19-73).
bool mpcc::nn_read_layer(const std::string& dir, int l, int R, int C, std::vector<double>& W, std::vector<double>& b) {
    const std::string base = dir + "/", tb = base + "parameter/", ls = std::to_string(l);
    return (read_doubles_bin(base + "weight_" + ls + ".f64", W, (size_t)R * C) &&
            read_doubles_bin(base + "bias_" + ls + ".f64", b, R)) ||
           (read_doubles_txt(tb + "weight_" + ls + ".txt", W, (size_t)R * C) &&
            read_doubles_txt(tb + "bias_" + ls + ".txt", b, R)) ||
           (read_doubles_txt(base + "weight_" + ls + ".txt", W, (size_t)R * C) &&
            read_doubles_txt(base + "bias_" + ls + ".txt", b, R));
}

namespace {

void load_nn(mpcc_engine* e, const std::string& dir, int nin, int nout, std::vector<int> hidden, NNWeights& w) {
    // k_mlp_self / k_mlp_env are specialized for the reference architectures (osqp_interface.cpp:35-43)
    const bool self_arch = nin == 7 && nout == 1 && hidden == std::vector<int>{256, 64};
    const bool env_arch = nin == 10 && nout == 9 && hidden == std::vector<int>{256, 256, 256, 256};
    if (!self_arch && !env_arch) throw std::runtime_error("unsupported MLP architecture under " + dir);
    std::vector<int> dims;
    dims.push_back(3 * nin);
    for (int h : hidden) dims.push_back(h);
    dims.push_back(nout);
    const int L = (int)dims.size() - 1;
    NNDesc nd{};
    nd.L = L;
    nd.nin = nin;
    for (int i = 0; i <= L; i++) nd.dims[i] = dims[i];
    std::vector<double> packed;
    for (int l = 0; l < L; l++) {
        const int R = dims[l + 1], C = dims[l];
        std::vector<double> W, b;
        if (!nn_read_layer(dir, l, R, C, W, b)) throw std::runtime_error("cannot read MLP layer " + std::to_string(l) + " under " + dir);
        // MFMA fragment order (mlp.hip): [row tile t][k-step s][lane l] = W[16t + (l & 15)][4s + (l >> 4)],
        // zero-padded to 16-row tiles and 16-deep k-tiles; bias zero-padded to the row tiles
        const int RT = (R + 15) / 16, KS = 4 * ((C + 15) / 16);
        nd.offW[l] = (long)packed.size();
        for (int t = 0; t < RT; t++)
            for (int s = 0; s < KS; s++)
                for (int ln = 0; ln < 64; ln++) {
                    const int r = 16 * t + (ln & 15), k = 4 * s + (ln >> 4);
                    packed.push_back((r < R && k < C) ? W[(size_t)r * C + k] : 0.0);
                }
        nd.offb[l] = (long)packed.size();
        for (int r = 0; r < 16 * RT; r++) packed.push_back(r < R ? b[r] : 0.0);
        while (packed.size() % 8) packed.push_back(0.0);  // 64-byte aligned layers
    }
    w.d = dmalloc<double>(packed.size());
    HIPCHK(hipMemcpy(w.d, packed.data(), packed.size() * sizeof(double), hipMemcpyHostToDevice));
    w.desc = nd;
    w.loaded = true;
    (void)e;
}

int fail(int code, const std::string& m) {
    set_last_error(m);
    return code;
}

void validate_params(const mpcc_params& p) {
    if (p.N < 1 || p.N > NMAX) throw std::invalid_argument("N out of range [1, 64]");
    if (ipm_lds_bytes(p.N, poly_rows_max(p.constraint_mask)) > 160 * 1024)
        throw std::invalid_argument("too many constraint rows for the interior-point LDS block");
    if (!(p.Ts > 0)) throw std::invalid_argument("Ts must be > 0");
    for (int i = 0; i < NX; i++) if (!(p.Tx[i] > 0)) throw std::invalid_argument("T_x must be > 0");
    for (int i = 0; i < NU; i++) if (!(p.Tu[i] > 0)) throw std::invalid_argument("T_u must be > 0");
    if (p.max_iter < 0 || p.line_search_max_iter < 0) throw std::invalid_argument("negative iteration limit");
    // Damped BFGS (osqp_interface.cpp:683-715) takes any max_iter: the QP Hessian is the structured Hessian of
    // SQP iteration 0 plus 2 low-rank terms per update, solved with the Woodbury identity around the Riccati
    // recursion; an update past LRX terms restarts from that iteration's exact Hessian.
}

// one track's tables in the device layout (dev_common.h SplineDev): SPL_STRIDE doubles
void pack_track(const SplineTables& t, double* out) {
    const int n = t.n;
    if (n != NSPL) throw std::logic_error("spline tables must have N_SPLINE points");
    size_t o = 0;
    auto push = [&](const std::vector<double>& v, size_t len) {
        if (v.size() != len) throw std::logic_error("spline table size");
        std::memcpy(out + o, v.data(), len * sizeof(double));
        o += len;
    };
    push(t.s, n);
    for (int a = 0; a < 3; a++) { push(t.a[a], n); push(t.b[a], n); push(t.c[a], n); push(t.d[a], n); }
    push(t.R, (size_t)9 * n); push(t.cr, n); push(t.dr, n); push(t.logv, (size_t)3 * n);
    out[SPL_DELTA] = t.delta;
    out[SPL_L] = t.length();
    for (int i = SPL_L + 1; i < SPL_STRIDE; i++) out[i] = 0.0;
}

// tables of B tracks (B = 1 and stride 0: one track shared by every instance)
void upload_tracks(mpcc_engine* e, const std::vector<SplineTables>& tracks, bool per_instance) {
    std::vector<double> buf(tracks.size() * (size_t)SPL_STRIDE);
    for (size_t i = 0; i < tracks.size(); i++) pack_track(tracks[i], buf.data() + i * SPL_STRIDE);
    if (e->d_spl) HIPCHK(hipFree(e->d_spl));
    e->d_spl = nullptr;
    e->d_spl = dmalloc<double>(buf.size());
    HIPCHK(hipMemcpy(e->d_spl, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice));
    e->spl.base = e->d_spl;
    e->spl.stride = per_instance ? SPL_STRIDE : 0;
    e->track = tracks[0];
    e->n_tracks = (int)tracks.size();
}

void upload_track(mpcc_engine* e) { upload_tracks(e, {e->track}, false); }

// Every entry point runs on the engine's device, whatever device the calling thread has current
// (a process may hold engines on several GPUs); the caller's current device is restored on return.
struct DevGuard {
    int prev = -1, dev = -1;
    explicit DevGuard(const mpcc_engine* e) : dev(e->cfg.device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DevGuard() {
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
};

// Host-side accessors of engine state (warm start, tracks, params, debug entries) first wait for every
// asynchronous call that may still use that state: the engine stream, and — when a device call ran
// on a caller stream (mpcc_solve_device / mpcc_set_warmstart_device with stream != NULL, which the
// engine's non-blocking stream does not order against) — the whole device.
void quiesce(mpcc_engine* e) {
    HIPCHK(hipStreamSynchronize(e->stream));
    if (e->ext_async) {
        HIPCHK(hipDeviceSynchronize());
        e->ext_async = false;
    }
}

// the fused kernel's span T over the ComputeTime fields by its waves' phase fractions: set_qp gets the in-kernel QP
// assembly on top of k_setqp's launch, solve_qp the QP solves, get_alpha the line search; the step update's share
// stays in total only (the reference times it in none of the four, osqp_interface.cpp:548-564).  t.solve_qp holds T
// plus any staged k_ipm spans of the same window (MPCC_STAGED_SQP calls mixed with fused ones): only T is split.
void split_sqp(mpcc_timing& t, double T, const double (&f)[PH_N]) {
    t.set_qp += T * f[PH_SETQP];
    t.solve_qp = (t.solve_qp - T) + T * f[PH_SOLVE];
    t.get_alpha += T * f[PH_ALPHA];
}

constexpr int IPW_SQP = 4;  // instances per k_sqp wave (ipm.hip IPW)
void run_batch(mpcc_engine* e, int B, hipStream_t st, mpcc_timing* timing, bool ocp = false) {
    DevConst c = e->make_const(B);
    c.ocp = ocp ? 1 : 0;
    DevBuffers& d = e->d;
    // Event recording: 'timing' (one synchronous call) or live mode (pairs kept until timing_end).
    const bool tm = timing != nullptr || e->live;
    std::vector<hipEvent_t> evs;
    int ei = 0;
    // a boundary with no launch since the previous one reuses its event: every event record is a marker packet
    // on the stream, and a chain of them between two kernels (the MLP and phase brackets of a configuration
    // that runs no MLP) widened that gap to ~25 us per step
    bool launched = true;
    auto mark = [&]() -> int {
        if (!launched && !evs.empty()) return (int)evs.size() - 1;
        hipEvent_t ev = e->live ? e->live_ev() : e->ev(ei);
        ei++;
        HIPCHK(hipEventRecord(ev, st));
        evs.push_back(ev);
        launched = false;
        return (int)evs.size() - 1;
    };
    std::vector<std::pair<int, int>> set_qp, solve_qp, get_alpha;
    int t0 = -1, t_env0 = -1, t_env1 = -1, t_end = -1;
    const bool fused = !e->staged_sqp || c.p.use_BFGS;
    d.phase_cyc = (tm && fused) ? e->d_phase : nullptr;  // the fused kernels' ComputeTime split (PhaseClock)
    bool sqp_timed = false;
    if (tm) t0 = mark();
    if (d.dbg_trace) HIPCHK(hipMemsetAsync(d.dbg_trace, 0, sizeof(double) * B * TRACE_IT * TRACE_W, st));
    launched = true;
    launch_prepare(c, d, st);
    launched = true;
    // Early solo blocks (configurations without collision networks): the cold starts that get solo blocks are the
    // launch's critical path (k_sqp_solo ~0.15 ms longer than the packed k_sqp at configs[1]).  After k_order and the
    // records of the solo instances alone (DevConst::subset 1), k_sqp_solo starts on the side stream and builds their
    // first QP records itself (ipm.hip solo_prep), while the other instances' records and QP records are built on the
    // group's stream (subset 2: k_order marks the solo instances) and the packed k_sqp follows them.  Every
    // instance's arithmetic is unchanged.
    const int npm_c = poly_rows_max(c.p.constraint_mask);
    const bool early_solo = fused && !(c.p.use_BFGS || e->wide_sqp) && DOF == 7 && e->solo_mode == 2 && e->tail_mode &&
                            e->early_solo && !c.ocp && !(c.p.constraint_mask & (MPCC_CON_SELFCOL | MPCC_CON_ENVCOL)) &&
                            (npm_c <= 2 || npm_c >= 9) && (c.Bn + IPW_SQP - 1) / IPW_SQP <= e->simds;
    DevConst cs = c;  // the fused k_sqp's launch constants (solo slots)
    hipStream_t side = nullptr;
    if (early_solo) {
        cs.solo = 2;
        launch_order(cs, d, st);
        if (tm) t_env0 = mark();
        // the solo instances' records, then the solo blocks on the side stream (they build their first QP records
        // themselves), beside the other instances' records and QP records on the group's stream
        DevConst c1 = c;
        c1.subset = 1;
        launch_stage_records(c1, d, st);
        side = e->side_stream();
        HIPCHK(hipEventRecord(e->solo_fork, st));
        HIPCHK(hipStreamWaitEvent(side, e->solo_fork, 0));
        DevConst cso = cs;
        cso.subset = 1;  // k_sqp_solo builds its instances' first QP records (ipm.hip solo_prep)
        if (!launch_sqp_solo(cso, d, d.u0, npm_c, side)) throw std::logic_error("early solo blocks without tail mode");
        HIPCHK(hipEventRecord(e->solo_join, side));
        c.subset = 2;  // the remaining launches of the records and the first QP records: every other instance
    } else if (tm) {
        t_env0 = mark();
    }
    launch_stage_records(c, d, st);
    launched = true;
    int m0 = -1, m1 = -1, m2 = -1;
    const bool nn_both = (c.p.constraint_mask & MPCC_CON_SELFCOL) && (c.p.constraint_mask & MPCC_CON_ENVCOL);
    if (nn_both && e->nn_par && !early_solo) {
        // The two collision networks (SelfCollisionModel / EnvCollisionModel, RobotData's update order) read the same
        // stage records and write disjoint record fields: the self network runs on the side stream beside the env
        // network, joined before the QP records.  Same kernels, same outputs.
        hipStream_t sd = e->side_stream();
        HIPCHK(hipEventRecord(e->nn_fork, st));
        HIPCHK(hipStreamWaitEvent(sd, e->nn_fork, 0));
        hipEvent_t s0 = nullptr, s1 = nullptr;
        if (e->live) {
            s0 = e->live_ev();
            HIPCHK(hipEventRecord(s0, sd));
        }
        launch_nn(c, d, e->nn_self.desc, e->nn_self.d, 0, c.S, nullptr, nullptr, d.rec, c.S, sd);
        if (e->live) {
            s1 = e->live_ev();
            HIPCHK(hipEventRecord(s1, sd));
        }
        HIPCHK(hipEventRecord(e->nn_join, sd));
        if (e->live) m1 = mark();
        launch_nn(c, d, e->nn_env.desc, e->nn_env.d, 1, c.S, nullptr, nullptr, d.rec, c.S, st);
        launched = true;
        if (e->live) {
            m2 = mark();
            e->lv_mlp_self.push_back({s0, s1});
            e->lv_mlp_env.push_back({evs[m1], evs[m2]});
        }
        HIPCHK(hipStreamWaitEvent(st, e->nn_join, 0));
    } else {
    if (e->live) m0 = mark();
    if (c.p.constraint_mask & MPCC_CON_SELFCOL)
    {
        launch_nn(c, d, e->nn_self.desc, e->nn_self.d, 0, c.S, nullptr, nullptr, d.rec, c.S, st);
        launched = true;
    }
    if (e->live) m1 = mark();
    if (c.p.constraint_mask & MPCC_CON_ENVCOL)
    {
        launch_nn(c, d, e->nn_env.desc, e->nn_env.d, 1, c.S, nullptr, nullptr, d.rec, c.S, st);
        launched = true;
    }
    if (e->live) {
        m2 = mark();
        if (c.p.constraint_mask & MPCC_CON_SELFCOL) e->lv_mlp_self.push_back({evs[m0], evs[m1]});
        if (c.p.constraint_mask & MPCC_CON_ENVCOL) e->lv_mlp_env.push_back({evs[m1], evs[m2]});
    }
    }
    if (tm) t_env1 = mark();
    const double* ucur = d.u0;
    if (fused) {
        // first QP assembly lane-per-stage, then the whole SQP loop per instance in one kernel (the damped-BFGS
        // option always on the fused 32-lane kernel)
        int a0 = -1, a1 = -1, b1 = -1;
        if (tm) a0 = mark();
        launch_setqp(c, d, ucur, st);
        c.subset = 0;
        launched = true;
        if (tm) a1 = mark();
        e->last_wide = DOF != 7 || c.p.use_BFGS || e->wide_sqp;
        if (early_solo) {
            launch_sqp(cs, d, ucur, npm_c, st);
            HIPCHK(hipStreamWaitEvent(st, e->solo_join, 0));
        } else if (c.p.use_BFGS || e->wide_sqp) launch_sqp_wide(c, d, ucur, poly_rows_max(c.p.constraint_mask), c.p.use_BFGS ? 1 : 0, st);
        else if (DOF == 7 && e->solo_mode && e->tail_mode && !c.ocp) {  // cold starts alone in a wave / block (k_prepare flags
                                                                       // them; the 16-lane interior point's tail mode)
            cs = c;
            const int npm = npm_c;
            cs.solo = 1;
            launch_order(cs, d, st);
            // solo blocks where the packed launch is one round of waves (at most one per SIMD): beyond that the
            // cold starts' time is spread over several rounds (B = 65,536: 2.078M with, 2.092M without, r04ah)
            if (e->solo_mode == 2 && DOF == 7 && (npm <= 2 || npm >= 9) && (c.Bn + IPW_SQP - 1) / IPW_SQP <= e->simds) {
                // solo blocks: k_sqp_solo on the side stream beside k_sqp (which leaves the solo waves to it), joined
                // before anything after k_sqp
                // The kernel on the forked stream starts ≈30 µs after the one that follows k_order in its own stream
                // (the cross-queue wait): k_sqp_solo, which ends last, goes on the group's stream, the packed k_sqp
                // on the side stream (MPCC_SOLO_SIDE=1: the other way round, A/B).
                cs.solo = 2;
                const char* ss = std::getenv("MPCC_SOLO_SIDE");
                const bool solo_side = ss && ss[0] == '1';
                hipStream_t side = e->side_stream();
                HIPCHK(hipEventRecord(e->solo_fork, st));
                HIPCHK(hipStreamWaitEvent(side, e->solo_fork, 0));
                // k_sqp with solo 2 leaves its first NSOLO waves to k_sqp_solo: if that cannot launch (a variant
                // without tail mode), k_sqp runs them itself as solo waves (solo 1)
                if (!launch_sqp_solo(cs, d, ucur, npm, solo_side ? side : st)) cs.solo = 1;
                launch_sqp(cs, d, ucur, npm, solo_side ? st : side);
                HIPCHK(hipEventRecord(e->solo_join, side));
                HIPCHK(hipStreamWaitEvent(st, e->solo_join, 0));
            } else {
                launch_sqp(cs, d, ucur, npm, st);
            }
        } else {
            launch_sqp(c, d, ucur, poly_rows_max(c.p.constraint_mask), st);
        }
        launched = true;
        if (tm) {
            b1 = mark();
            set_qp.push_back({a0, a1});
            solve_qp.push_back({a1, b1});
            sqp_timed = true;
        }
    } else {
    e->last_wide = DOF != 7;  // the staged loop's k_ipm: 16 lanes for the Panda (a wide debug QP before must not stick)
    for (int it = 0; it < c.p.max_iter; it++) {
        int a0 = -1, a1 = -1, b1 = -1, c1 = -1;
        if (tm) a0 = mark();
        launch_setqp(c, d, ucur, st);
        launched = true;
        if (tm) a1 = mark();
        launch_ipm(c, d, poly_rows_max(c.p.constraint_mask), st);
        launched = true;
        if (c.p.do_SOC) {  // SecondOrderCorrection (osqp_interface.cpp:506-535)
            launch_soc(c, d, ucur, st);
            launch_ipm(c, d, poly_rows_max(c.p.constraint_mask), st);
        }
        if (tm) b1 = mark();
        launch_trial(c, d, ucur, 1.0, 0, st);
        launch_accept(c, d, st);
        if (c.faithful_dead_trials) {
            double alpha = 1.0;
            for (int l = 1; l < c.p.line_search_max_iter; l++) {
                alpha *= c.p.line_search_tau;
                launch_trial(c, d, ucur, alpha, 1, st);
            }
        }
        launch_apply(c, d, st);
        launched = true;
        if (tm) {
            c1 = mark();
            set_qp.push_back({a0, a1});
            solve_qp.push_back({a1, b1});
            get_alpha.push_back({b1, c1});
        }
    }
    }
    launch_finalize(c, d, st);
    launched = true;
    HIPCHK(hipGetLastError());
    if (!tm) return;
    t_end = mark();
    if (e->live) {
        e->lv_total.push_back({evs[t0], evs[t_end]});
        e->lv_env.push_back({evs[t_env0], evs[t_env1]});
        for (auto& pr : set_qp) e->lv_setqp.push_back({evs[pr.first], evs[pr.second]});
        for (auto& pr : solve_qp) e->lv_ipm.push_back({evs[pr.first], evs[pr.second]});
        for (auto& pr : get_alpha) e->lv_alpha.push_back({evs[pr.first], evs[pr.second]});
        if (sqp_timed)
            for (auto& pr : solve_qp) e->lv_sqp.push_back({evs[pr.first], evs[pr.second]});
        e->live_calls++;
    }
    if (timing) {
        HIPCHK(hipEventSynchronize(evs[t_end]));
        auto el = [&](int a, int b) { float ms = 0; (void)hipEventElapsedTime(&ms, evs[a], evs[b]); return ms * 1e-3; };
        timing->set_env = el(t_env0, t_env1);
        timing->set_qp = 0; timing->solve_qp = 0; timing->get_alpha = 0;
        for (auto& pr : set_qp) timing->set_qp += el(pr.first, pr.second);
        for (auto& pr : solve_qp) timing->solve_qp += el(pr.first, pr.second);
        for (auto& pr : get_alpha) timing->get_alpha += el(pr.first, pr.second);
        timing->total = el(t0, t_end);
        double f[PH_N];
        if (sqp_timed && !e->live && e->phase_fracs(f, st)) split_sqp(*timing, timing->solve_qp, f);
    }
}

}  // namespace

extern "C" {

int mpcc_abi_version(void) { return MPCC_ABI_VERSION; }

int mpcc_robot_dof(void) { return DOF; }

int mpcc_cubic_spline_host(int n, const double* x, const double* y, int regular, int m, const double* xq, double* out3) {
    if (n < 2 || m < 0 || !x || !y || (m && (!xq || !out3))) return fail(MPCC_E_INVALID, "mpcc_cubic_spline_host: invalid argument");
    host_cubic_spline(n, x, y, regular != 0, m, xq, out3);
    return MPCC_OK;
}

int mpcc_rot_spline_host(int n, const double* x, const double* R9, int regular, int m, const double* xq, double* Rq,
                         double* dRq) {
    if (n < 2 || m < 0 || !x || !R9 || (m && !xq)) return fail(MPCC_E_INVALID, "mpcc_rot_spline_host: invalid argument");
    host_rot_spline(n, x, R9, regular != 0, m, xq, Rq, dRq);
    return MPCC_OK;
}

int mpcc_so3_log(const double* R9, double* S9) {
    if (!R9 || !S9) return fail(MPCC_E_INVALID, "mpcc_so3_log: null argument");
    double v[3];
    host_log_vec(R9, v);
    const double S[9] = {0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0};
    std::memcpy(S9, S, sizeof S);
    return MPCC_OK;
}

int mpcc_so3_exp(const double* S9, double* R9) {
    if (!S9 || !R9) return fail(MPCC_E_INVALID, "mpcc_so3_exp: null argument");
    host_exp_matrix(S9, R9);
    return MPCC_OK;
}
const char* mpcc_last_error(void) { return g_last_error.c_str(); }
#if MPCC_DOF != 7
// the mobile build's interior point (ipm_wide.hip) has no tail mode (ipm_tail.h is the Panda's 16-lane form)
int mpcc_debug_tail_solves(long long* out, int /*reset*/) {
    if (out) *out = 0;
    return MPCC_OK;
}
#endif

int mpcc_debug_order(mpcc_engine* e, int32_t* out, int n) {
    if (!e || !out || n < 0) return fail(MPCC_E_INVALID, "mpcc_debug_order: invalid argument");
    n = std::min(n, order_slots(e->maxB) + e->maxB);
    try {
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipMemcpy(out, e->d.order, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
    } catch (const std::exception& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_debug_order: ") + x.what());
    }
    return n;
}

int mpcc_create(const mpcc_config* cfg, const mpcc_params* params, const char* nn_dir, mpcc_engine** out) {
    if (!cfg || !params || !out) return fail(MPCC_E_INVALID, "mpcc_create: null argument");
    std::unique_ptr<mpcc_engine> e(new mpcc_engine());
    try {
        e->cfg = *cfg;
        const char* st = std::getenv("MPCC_STAGED_SQP");
        e->staged_sqp = st && st[0] == '1';
        const char* wd = std::getenv("MPCC_WIDE_SQP");
        e->wide_sqp = wd && wd[0] == '1';
        const char* tl = std::getenv("MPCC_TAIL");
        e->tail_mode = (tl && tl[0] == '0') ? 0 : 1;
        const char* so = std::getenv("MPCC_SOLO");
        e->solo_mode = (so && so[0] == '0') ? 0 : (so && so[0] == '1') ? 1 : 2;
        const char* es = std::getenv("MPCC_EARLY_SOLO");
        e->early_solo = (es && es[0] == '0') ? 0 : 1;
        const char* np = std::getenv("MPCC_NN_PAR");
        e->nn_par = (np && np[0] == '1') ? 1 : 0;
        e->params = *params;
        e->params.N = cfg->N;
        e->params.Ts = cfg->Ts;
        if (cfg->constraint_mask >= 0) e->params.constraint_mask = cfg->constraint_mask;
        validate_params(e->params);
        if (cfg->max_batch < 1) throw std::invalid_argument("max_batch must be >= 1");
        e->N = cfg->N;
        e->maxB = cfg->max_batch;
        HIPCHK(hipSetDevice(cfg->device));
        // A blocking stream: work a caller queues on the legacy default stream (torch's default
        // stream, or any NULL-stream copy of the inputs) is ordered before and after the engine's
        // kernels, as the ABI's "NULL = engine stream" would otherwise race with it.
        HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamDefault));
        {
            int ncu = 0;
            if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess && ncu > 0)
                e->simds = 4 * ncu;
        }
        HIPCHK(hipEventCreateWithFlags(&e->solo_fork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&e->solo_join, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&e->nn_fork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&e->nn_join, hipEventDisableTiming));
        const size_t B = (size_t)e->maxB, NS = (size_t)e->N + 1;
        DevBuffers& d = e->d;
        d.guess = dmalloc<double>(B * NS * NXU);
        d.valid = dmalloc<int32_t>(B);
        d.fails = dmalloc<int32_t>(B);
        d.rec = dmalloc<double>((size_t)REC * B * NS);
        d.qs = dmalloc<double>(B * NS * QS);
        d.is = dmalloc<double>(B * NS * IS);
        d.step = dmalloc<double>(B * NS * NXU);
        d.trial = dmalloc<double>(B * NS * 4);
        d.sqi = dmalloc<int32_t>(B * SQI);
        d.sqd = dmalloc<double>(B * SQ);
        d.order = dmalloc<int32_t>((size_t)order_slots((int)B) + B);
        e->d_phase = dmalloc<unsigned long long>(PH_N);
        HIPCHK(hipMemset(e->d_phase, 0, PH_N * sizeof(unsigned long long)));
        HIPCHK(hipMemset(d.guess, 0, B * NS * NXU * sizeof(double)));
        HIPCHK(hipMemset(d.valid, 0, B * sizeof(int32_t)));
        HIPCHK(hipMemset(d.fails, 0, B * sizeof(int32_t)));
        HIPCHK(hipMemset(d.sqi, 0, B * SQI * sizeof(int32_t)));
        if (DOF != 7) d.isw = d.is;  // the mobile build's interior point is the 32-lane one
#ifdef MPCC_BOUNDS_CHECK
        e->bchk = dmalloc<uint32_t>(64);
        HIPCHK(hipMemset(e->bchk, 0, 64 * sizeof(uint32_t)));
#endif
        if (e->params.use_BFGS || e->wide_sqp) e->ensure_wide_buffers(e->params.use_BFGS, e->params.max_iter);
        e->s_x0 = dmalloc<double>(B * NX);
        e->s_u0 = dmalloc<double>(B * NU);
        e->s_obs = dmalloc<double>(B * 4);
        e->s_u0out = dmalloc<double>(B * NU);
        e->s_hor = dmalloc<double>(B * NS * NXU);
        e->s_status = dmalloc<int32_t>(B);
        e->s_ok = dmalloc<int32_t>(B);
        e->set_model();
        const int mask = e->params.constraint_mask;
        if (mask & (MPCC_CON_SELFCOL | MPCC_CON_ENVCOL)) {
            if (!nn_dir) throw std::invalid_argument("nn_dir required when collision rows are enabled");
            std::string dir(nn_dir);
            load_nn(e.get(), dir + "/self", 7, 1, {256, 64}, e->nn_self);      // osqp_interface.cpp:35-38
            load_nn(e.get(), dir + "/env", 10, 9, {256, 256, 256, 256}, e->nn_env);  // :40-43
        }
    } catch (const std::bad_alloc&) {
        return fail(MPCC_E_OOM, "mpcc_create: device allocation failed");
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_create: ") + x.what());
    } catch (const std::invalid_argument& x) {
        return fail(MPCC_E_INVALID, std::string("mpcc_create: ") + x.what());
    } catch (const std::exception& x) {
        return fail(MPCC_E_IO, std::string("mpcc_create: ") + x.what());
    }
    *out = e.release();
    return MPCC_OK;
}

void mpcc_destroy(mpcc_engine* e) {
    if (!e) return;
    DevGuard dg_(e);
    (void)hipDeviceSynchronize();  // no kernel may still use the buffers being freed
    delete e;
}

int mpcc_set_params(mpcc_engine* e, const mpcc_params* p) {
    if (!e || !p) return fail(MPCC_E_INVALID, "mpcc_set_params: null argument");
    DevGuard dg_(e);
    mpcc_params np = *p;
    np.N = e->N;  // horizon and Ts are fixed at creation (device buffers, model)
    np.Ts = e->params.Ts;
    if ((np.constraint_mask & (MPCC_CON_SELFCOL | MPCC_CON_ENVCOL)) && !(e->nn_self.loaded && e->nn_env.loaded))
        return fail(MPCC_E_INVALID, "mpcc_set_params: collision rows need NN weights loaded at create");
    const mpcc_params old = e->params;
    try {
        quiesce(e);
        validate_params(np);
        e->params = np;
        e->set_model();
        if (np.use_BFGS) e->ensure_wide_buffers(true, np.max_iter);
    } catch (const std::exception& x) {
        e->params = old;
        e->set_model();
        return fail(MPCC_E_INVALID, std::string("mpcc_set_params: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_get_params(mpcc_engine* e, mpcc_params* out) {
    if (!e || !out) return fail(MPCC_E_INVALID, "mpcc_get_params: null argument");
    DevGuard dg_(e);
    *out = e->params;
    return MPCC_OK;
}

int mpcc_set_track(mpcc_engine* e, int n, const double* X, const double* Y, const double* Z, const double* R9) {
    if (!e || n < 3 || !X || !Y || !Z || !R9) return fail(MPCC_E_INVALID, "mpcc_set_track: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        e->track = build_track_spline(n, X, Y, Z, R9);
        upload_track(e);
        e->has_track = true;
        HIPCHK(hipMemset(e->d.valid, 0, (size_t)e->maxB * sizeof(int32_t)));  // valid_initial_guess_ = false
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_set_track: ") + x.what());
    } catch (const std::exception& x) {
        return fail(MPCC_E_INVALID, std::string("mpcc_set_track: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_set_track_path(mpcc_engine* e, int n, const double* s, const double* X, const double* Y, const double* Z,
                        const double* R9) {
    if (!e || !s || !X || !Y || !Z || !R9) return fail(MPCC_E_INVALID, "mpcc_set_track_path: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        e->track = build_track_from_path(n, s, X, Y, Z, R9);
        upload_track(e);
        e->has_track = true;
        HIPCHK(hipMemset(e->d.valid, 0, (size_t)e->maxB * sizeof(int32_t)));
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_set_track_path: ") + x.what());
    } catch (const std::exception& x) {
        return fail(MPCC_E_INVALID, std::string("mpcc_set_track_path: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_set_tracks(mpcc_engine* e, int B, int n, const double* X, const double* Y, const double* Z, const double* R9) {
    if (!e || B < 1 || B > e->maxB || n < 3 || !X || !Y || !Z || !R9)
        return fail(MPCC_E_INVALID, "mpcc_set_tracks: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        std::vector<SplineTables> tr(B);
        const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> pool;
        std::vector<std::string> err(nt);
        for (unsigned w = 0; w < nt; w++)
            pool.emplace_back([&, w]() {
                try {
                    for (int b = (int)w; b < B; b += (int)nt) {
                        const size_t o = (size_t)b * n;
                        tr[b] = build_track_spline(n, X + o, Y + o, Z + o, R9 + 9 * o);
                    }
                } catch (const std::exception& x) {
                    err[w] = x.what();
                }
            });
        for (auto& th : pool) th.join();
        for (auto& m : err)
            if (!m.empty()) throw std::invalid_argument(m);
        upload_tracks(e, tr, true);
        e->has_track = true;
        HIPCHK(hipMemset(e->d.valid, 0, (size_t)e->maxB * sizeof(int32_t)));  // valid_initial_guess_ = false
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_set_tracks: ") + x.what());
    } catch (const std::exception& x) {
        return fail(MPCC_E_INVALID, std::string("mpcc_set_tracks: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_track_eval_host(int n, const double* X, const double* Y, const double* Z, const double* R9, int M,
                         const double* s, double* pos, double* d1, double* d2, double* R, double* dR) {
    if (n < 3 || M < 0 || !X || !Y || !Z || !R9 || (M && !s)) return fail(MPCC_E_INVALID, "mpcc_track_eval_host: invalid argument");
    try {
        const SplineTables t = build_track_spline(n, X, Y, Z, R9);
        for (int i = 0; i < M; i++)
            eval_tables(t, s[i], pos ? pos + 3 * i : nullptr, d1 ? d1 + 3 * i : nullptr, d2 ? d2 + 3 * i : nullptr,
                        R ? R + 9 * i : nullptr, dR ? dR + 3 * i : nullptr);
    } catch (const std::exception& x) {
        return fail(MPCC_E_INVALID, std::string("mpcc_track_eval_host: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_track_project_host(int n, const double* X, const double* Y, const double* Z, const double* R9, int M,
                            double proj_max_dist, const double* s_guess, const double* ee, double* s_out) {
    if (n < 3 || M < 0 || !X || !Y || !Z || !R9 || (M && (!s_guess || !ee || !s_out)))
        return fail(MPCC_E_INVALID, "mpcc_track_project_host: invalid argument");
    try {
        const SplineTables t = build_track_spline(n, X, Y, Z, R9);
        for (int i = 0; i < M; i++) s_out[i] = project_tables(t, proj_max_dist, s_guess[i], ee + 3 * i);
    } catch (const std::exception& x) {
        return fail(MPCC_E_INVALID, std::string("mpcc_track_project_host: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_track_build_host(int n, const double* X, const double* Y, const double* Z, const double* R9, double* s,
                          double* Xo, double* Yo, double* Zo, double* Ro9, double* length) {
    if (n < 3 || !X || !Y || !Z || !R9) return fail(MPCC_E_INVALID, "mpcc_track_build_host: invalid argument");
    try {
        SplineTables t = build_track_spline(n, X, Y, Z, R9);
        if (s) std::memcpy(s, t.s.data(), t.n * sizeof(double));
        if (Xo) std::memcpy(Xo, t.X.data(), t.n * sizeof(double));
        if (Yo) std::memcpy(Yo, t.Y.data(), t.n * sizeof(double));
        if (Zo) std::memcpy(Zo, t.Z.data(), t.n * sizeof(double));
        if (Ro9) std::memcpy(Ro9, t.R.data(), (size_t)t.n * 9 * sizeof(double));
        if (length) *length = t.length();
    } catch (const std::exception& x) {
        return fail(MPCC_E_INVALID, std::string("mpcc_track_build_host: ") + x.what());
    }
    return MPCC_OK;
}

double mpcc_track_length(mpcc_engine* e) { return (e && e->has_track) ? e->track.length() : 0.0; }

int mpcc_get_track_path(mpcc_engine* e, double* s, double* X, double* Y, double* Z, double* R9) {
    if (!e || !e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_get_track_path: no track");
    DevGuard dg_(e);
    const SplineTables& t = e->track;
    if (s) std::memcpy(s, t.s.data(), t.n * sizeof(double));
    if (X) std::memcpy(X, t.X.data(), t.n * sizeof(double));
    if (Y) std::memcpy(Y, t.Y.data(), t.n * sizeof(double));
    if (Z) std::memcpy(Z, t.Z.data(), t.n * sizeof(double));
    if (R9) std::memcpy(R9, t.R.data(), (size_t)t.n * 9 * sizeof(double));
    return MPCC_OK;
}

int mpcc_set_warmstart(mpcc_engine* e, int B, const double* guess, const int32_t* valid, const int32_t* fails) {
    if (!e || B < 0 || B > e->maxB) return fail(MPCC_E_INVALID, "mpcc_set_warmstart: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        const size_t NS = e->N + 1;
        if (guess) HIPCHK(hipMemcpy(e->d.guess, guess, (size_t)B * NS * NXU * sizeof(double), hipMemcpyHostToDevice));
        if (valid) HIPCHK(hipMemcpy(e->d.valid, valid, (size_t)B * sizeof(int32_t), hipMemcpyHostToDevice));
        if (fails) HIPCHK(hipMemcpy(e->d.fails, fails, (size_t)B * sizeof(int32_t), hipMemcpyHostToDevice));
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_get_warmstart(mpcc_engine* e, int B, double* guess, int32_t* valid, int32_t* fails) {
    if (!e || B < 0 || B > e->maxB) return fail(MPCC_E_INVALID, "mpcc_get_warmstart: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        const size_t NS = e->N + 1;
        if (guess) HIPCHK(hipMemcpy(guess, e->d.guess, (size_t)B * NS * NXU * sizeof(double), hipMemcpyDeviceToHost));
        if (valid) HIPCHK(hipMemcpy(valid, e->d.valid, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToHost));
        if (fails) HIPCHK(hipMemcpy(fails, e->d.fails, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToHost));
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_reset_warmstart(mpcc_engine* e, int B, const uint8_t* mask) {
    if (!e || B < 0 || B > e->maxB) return fail(MPCC_E_INVALID, "mpcc_reset_warmstart: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        if (!mask) {
            HIPCHK(hipMemset(e->d.valid, 0, (size_t)B * sizeof(int32_t)));
            HIPCHK(hipMemset(e->d.fails, 0, (size_t)B * sizeof(int32_t)));
            return MPCC_OK;
        }
        std::vector<int32_t> v(B), f(B);
        HIPCHK(hipMemcpy(v.data(), e->d.valid, B * sizeof(int32_t), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(f.data(), e->d.fails, B * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (int i = 0; i < B; i++) if (mask[i]) { v[i] = 0; f[i] = 0; }
        HIPCHK(hipMemcpy(e->d.valid, v.data(), B * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->d.fails, f.data(), B * sizeof(int32_t), hipMemcpyHostToDevice));
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_solve_device(mpcc_engine* e, int B, double* d_x0, const double* d_u0, const double* d_obs, double* d_u0_out,
                      double* d_horizon, int32_t* d_status, int32_t* d_ok, void* stream) {
    if (!e || B < 1 || B > e->maxB || !d_x0 || !d_u0 || !d_obs)
        return fail(MPCC_E_INVALID, "mpcc_solve_device: invalid argument");
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_solve_device: set_track first");
    DevGuard dg_(e);
    if (e->spl.stride && B > e->n_tracks) return fail(MPCC_E_INVALID, "mpcc_solve_device: more instances than per-instance tracks");
    try {
        hipStream_t st = stream ? (hipStream_t)stream : e->stream;
        if (st != e->stream) e->ext_async = true;
        e->d.x0 = d_x0; e->d.u0 = d_u0; e->d.obs = d_obs;
        e->d.u0_out = d_u0_out; e->d.horizon = d_horizon; e->d.status = d_status; e->d.ok = d_ok;
        run_batch(e, B, st, nullptr);
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_solve_device: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_set_warmstart_device(mpcc_engine* e, int B, const double* d_guess, const int32_t* d_valid,
                              const int32_t* d_fails, void* stream) {
    if (!e || B < 0 || B > e->maxB) return fail(MPCC_E_INVALID, "mpcc_set_warmstart_device: invalid argument");
    DevGuard dg_(e);
    try {
        hipStream_t st = stream ? (hipStream_t)stream : e->stream;
        if (st != e->stream) e->ext_async = true;
        const size_t NS = e->N + 1;
        // one launch for the three arrays (three blits were three launches and their gaps on the step's chain)
        launch_warmstart_copy(d_guess ? (long)B * NS * NXU : 0, d_guess, e->d.guess, B, d_valid, e->d.valid, d_fails,
                              e->d.fails, st);
        HIPCHK(hipGetLastError());
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_timing_begin(mpcc_engine* e) {
    if (!e) return fail(MPCC_E_INVALID, "mpcc_timing_begin: null engine");
    DevGuard dg_(e);
    e->live = true;
    e->live_used = 0;
    e->live_calls = 0;
    e->lv_env.clear(); e->lv_setqp.clear(); e->lv_ipm.clear(); e->lv_alpha.clear(); e->lv_total.clear();
    e->lv_mlp_self.clear(); e->lv_mlp_env.clear(); e->lv_sqp.clear();
    try {
        HIPCHK(hipMemsetAsync(e->d_phase, 0, PH_N * sizeof(unsigned long long), e->stream));
    } catch (const HipError& x) {
        e->live = false;
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_timing_end(mpcc_engine* e, mpcc_timing* sum, int32_t* n_calls, int32_t* n_ipm) {
    if (!e || !e->live) return fail(MPCC_E_INVALID, "mpcc_timing_end: timing not active");
    DevGuard dg_(e);
    try {
        mpcc_timing t{};
        auto acc = [&](const std::vector<std::pair<hipEvent_t, hipEvent_t>>& v) {
            double s = 0;
            for (auto& pr : v) {
                HIPCHK(hipEventSynchronize(pr.second));
                float ms = 0;
                HIPCHK(hipEventElapsedTime(&ms, pr.first, pr.second));
                s += ms * 1e-3;
            }
            return s;
        };
        t.total = acc(e->lv_total);
        t.set_env = acc(e->lv_env);
        t.set_qp = acc(e->lv_setqp);
        t.solve_qp = acc(e->lv_ipm);
        t.get_alpha = acc(e->lv_alpha);
        e->last_mlp_self_s = acc(e->lv_mlp_self);
        e->last_mlp_env_s = acc(e->lv_mlp_env);
        e->last_mlp_self_n = (int)e->lv_mlp_self.size();
        e->last_mlp_env_n = (int)e->lv_mlp_env.size();
        e->last_sqp_s = acc(e->lv_sqp);
        e->last_sqp_n = (int)e->lv_sqp.size();
        double f[PH_N] = {0, 0, 0, 0};
        HIPCHK(hipDeviceSynchronize());  // the counters of launches on caller streams too
        if (e->phase_fracs(f, e->stream) && e->last_sqp_n) split_sqp(t, e->last_sqp_s, f);
        for (int i = 0; i < PH_N; i++) e->last_frac[i] = f[i];
        if (sum) *sum = t;
        if (n_calls) *n_calls = e->live_calls;
        if (n_ipm) *n_ipm = (int32_t)e->lv_ipm.size();
    } catch (const HipError& x) {
        e->live = false;
        return fail(MPCC_E_HIP, x.what());
    }
    e->live = false;
    return MPCC_OK;
}

int mpcc_get_solve_stats(mpcc_engine* e, int B, int32_t* sqp_iter, int32_t* ipm_iters, int32_t* qp_status) {
    if (!e || B < 1 || B > e->maxB) return fail(MPCC_E_INVALID, "mpcc_get_solve_stats: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        HIPCHK(hipDeviceSynchronize());  // the stats of the last solve, whichever stream it ran on
        std::vector<int32_t> sqi((size_t)B * SQI);
        HIPCHK(hipMemcpy(sqi.data(), e->d.sqi, sqi.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (int b = 0; b < B; b++) {
            if (sqp_iter) sqp_iter[b] = sqi[(size_t)b * SQI + SQ_ITER];
            if (ipm_iters) ipm_iters[b] = sqi[(size_t)b * SQI + SQ_IPMIT];
            if (qp_status) qp_status[b] = sqi[(size_t)b * SQI + SQ_QPSTAT];
        }
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_solve(mpcc_engine* e, int B, double* x0, const double* u0, const double* obs, double* u0_out, double* horizon_out,
               int32_t* status, int32_t* ok, mpcc_timing* timing) {
    if (!e || B < 1 || B > e->maxB || !x0 || !u0 || !obs) return fail(MPCC_E_INVALID, "mpcc_solve: invalid argument");
    DevGuard dg_(e);
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_solve: set_track first");
    if (e->spl.stride && B > e->n_tracks) return fail(MPCC_E_INVALID, "mpcc_solve: more instances than per-instance tracks");
    try {
        quiesce(e);
        hipStream_t st = e->stream;
        const size_t NS = e->N + 1;
        HIPCHK(hipMemcpyAsync(e->s_x0, x0, B * NX * sizeof(double), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->s_u0, u0, B * NU * sizeof(double), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->s_obs, obs, B * 4 * sizeof(double), hipMemcpyHostToDevice, st));
        e->d.x0 = e->s_x0; e->d.u0 = e->s_u0; e->d.obs = e->s_obs;
        e->d.u0_out = e->s_u0out; e->d.horizon = e->s_hor; e->d.status = e->s_status; e->d.ok = e->s_ok;
        run_batch(e, B, st, timing);
        HIPCHK(hipMemcpyAsync(x0, e->s_x0, B * NX * sizeof(double), hipMemcpyDeviceToHost, st));
        if (u0_out) HIPCHK(hipMemcpyAsync(u0_out, e->s_u0out, B * NU * sizeof(double), hipMemcpyDeviceToHost, st));
        if (horizon_out)
            HIPCHK(hipMemcpyAsync(horizon_out, e->s_hor, B * NS * NXU * sizeof(double), hipMemcpyDeviceToHost, st));
        if (status) HIPCHK(hipMemcpyAsync(status, e->s_status, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        if (ok) HIPCHK(hipMemcpyAsync(ok, e->s_ok, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_solve: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_solve_ocp(mpcc_engine* e, int B, const double* guess, const double* u_cur, const double* obs,
                   double* opt_sol, int32_t* status, int32_t* solved, mpcc_timing* timing) {
    if (!e || B < 1 || B > e->maxB || !guess || !u_cur || !obs || !opt_sol)
        return fail(MPCC_E_INVALID, "mpcc_solve_ocp: invalid argument");
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_solve_ocp: set_track first");
    DevGuard dg_(e);
    if (e->spl.stride && B > e->n_tracks) return fail(MPCC_E_INVALID, "mpcc_solve_ocp: more instances than per-instance tracks");
    try {
        quiesce(e);
        hipStream_t st = e->stream;
        const size_t NS = e->N + 1;
        HIPCHK(hipMemcpyAsync(e->d.guess, guess, B * NS * NXU * sizeof(double), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->s_u0, u_cur, B * NU * sizeof(double), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->s_obs, obs, B * 4 * sizeof(double), hipMemcpyHostToDevice, st));
        e->d.x0 = e->s_x0; e->d.u0 = e->s_u0; e->d.obs = e->s_obs;
        e->d.u0_out = e->s_u0out; e->d.horizon = e->s_hor; e->d.status = e->s_status; e->d.ok = e->s_ok;
        run_batch(e, B, st, timing, true);
        HIPCHK(hipMemcpyAsync(opt_sol, e->s_hor, B * NS * NXU * sizeof(double), hipMemcpyDeviceToHost, st));
        if (status) HIPCHK(hipMemcpyAsync(status, e->s_status, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        if (solved) HIPCHK(hipMemcpyAsync(solved, e->s_ok, B * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_solve_ocp: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_closed_loop(mpcc_engine* e, int B, int steps, double* x0, double* u0, const double* obs, double* x_traj,
                     double* u_traj, int32_t* status_traj, int use_graph) {
    if (!e || B < 1 || B > e->maxB || steps < 0 || !x0 || !u0 || !obs)
        return fail(MPCC_E_INVALID, "mpcc_closed_loop: invalid argument");
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_closed_loop: set_track first");
    DevGuard dg_(e);
    if (e->spl.stride && B > e->n_tracks) return fail(MPCC_E_INVALID, "mpcc_closed_loop: more instances than per-instance tracks");
    std::vector<void*> owned;
    auto dev = [&](size_t bytes) { void* p = dmalloc<char>(bytes ? bytes : 1); owned.push_back(p); return p; };
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    int rc = MPCC_OK;
    try {
        quiesce(e);
        hipStream_t st = e->stream;
        double* dx = (double*)dev((size_t)B * NX * 8);
        double* du = (double*)dev((size_t)B * NU * 8);
        double* dobs = (double*)dev((size_t)B * 4 * 8);
        int32_t* alive = (int32_t*)dev((size_t)B * 4);
        int* kstep = (int*)dev(sizeof(int));
        double* xtraj = (double*)dev((size_t)(steps + 1) * B * NX * 8);
        double* utraj = (double*)dev((size_t)steps * B * NU * 8);
        int32_t* straj = (int32_t*)dev((size_t)steps * B * 4);
        HIPCHK(hipMemcpyAsync(dx, x0, (size_t)B * NX * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(du, u0, (size_t)B * NU * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(dobs, obs, (size_t)B * 4 * 8, hipMemcpyHostToDevice, st));
        std::vector<int32_t> ones(B, 1);
        HIPCHK(hipMemcpyAsync(alive, ones.data(), (size_t)B * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemsetAsync(kstep, 0, sizeof(int), st));
        DevBuffers& d = e->d;
        d.x0 = dx; d.u0 = du; d.obs = dobs;
        d.u0_out = e->s_u0out; d.horizon = nullptr; d.status = e->s_status; d.ok = e->s_ok;
        const double ts = e->params.Ts;
        auto step = [&]() {
            launch_loop_pre(B, dx, xtraj, kstep, st);
            run_batch(e, B, st, nullptr);
            launch_loop_post(B, ts, dx, du, xtraj, e->s_u0out, e->s_status, e->s_ok, alive, utraj, straj, kstep, st);
        };
        if (use_graph && steps > 0) {
            HIPCHK(hipStreamSynchronize(st));
            (void)e->side_stream();  // created outside the capture (the solo blocks and the self network fork onto it)
            HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            step();
            HIPCHK(hipStreamEndCapture(st, &graph));
            HIPCHK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
            for (int k = 0; k < steps; k++) HIPCHK(hipGraphLaunch(exec, st));
        } else {
            for (int k = 0; k < steps; k++) step();
        }
        launch_loop_pre(B, dx, xtraj, kstep, st);  // x_traj[steps] = final state
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(x0, dx, (size_t)B * NX * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(u0, du, (size_t)B * NU * 8, hipMemcpyDeviceToHost, st));
        if (x_traj) HIPCHK(hipMemcpyAsync(x_traj, xtraj, (size_t)(steps + 1) * B * NX * 8, hipMemcpyDeviceToHost, st));
        if (u_traj && steps) HIPCHK(hipMemcpyAsync(u_traj, utraj, (size_t)steps * B * NU * 8, hipMemcpyDeviceToHost, st));
        if (status_traj && steps)
            HIPCHK(hipMemcpyAsync(status_traj, straj, (size_t)steps * B * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    } catch (const HipError& x) {
        rc = fail(MPCC_E_HIP, std::string("mpcc_closed_loop: ") + x.what());
    }
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    for (void* p : owned) (void)hipFree(p);
    return rc;
}

int mpcc_sim_time_step(mpcc_engine* e, int B, const double* x, const double* u, double ts, double* x_next) {
    if (!e || B < 1 || !x || !u || !x_next) return fail(MPCC_E_INVALID, "mpcc_sim_time_step: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        double* dx = dmalloc<double>((size_t)B * NX);
        double* du = dmalloc<double>((size_t)B * NU);
        double* dn = dmalloc<double>((size_t)B * NX);
        HIPCHK(hipMemcpy(dx, x, B * NX * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(du, u, B * NU * sizeof(double), hipMemcpyHostToDevice));
        launch_sim_step(B, dx, du, ts, dn, e->stream);
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipMemcpy(x_next, dn, B * NX * sizeof(double), hipMemcpyDeviceToHost));
        (void)hipFree(dx); (void)hipFree(du); (void)hipFree(dn);
    } catch (const std::bad_alloc&) {
        return fail(MPCC_E_OOM, "mpcc_sim_time_step: allocation failed");
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_debug_robot_records(mpcc_engine* e, int M, const double* q, const double* obs, double* rec) {
    if (!e || M < 1 || !q || !obs || !rec) return fail(MPCC_E_INVALID, "mpcc_debug_robot_records: invalid argument");
    DevGuard dg_(e);
    try {
        quiesce(e);
        double* dq = dmalloc<double>((size_t)M * DOF);
        double* dob = dmalloc<double>((size_t)M * 4);
        double* drec = dmalloc<double>((size_t)M * REC);
        HIPCHK(hipMemcpy(dq, q, M * DOF * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dob, obs, M * 4 * sizeof(double), hipMemcpyHostToDevice));
        DevConst c = e->make_const(1);
        launch_debug_records(c, M, dq, dob, drec, e->stream);
        if (c.p.constraint_mask & MPCC_CON_SELFCOL)
            launch_nn(c, e->d, e->nn_self.desc, e->nn_self.d, 0, M, dq, dob, drec, M, e->stream);
        if (c.p.constraint_mask & MPCC_CON_ENVCOL)
            launch_nn(c, e->d, e->nn_env.desc, e->nn_env.d, 1, M, dq, dob, drec, M, e->stream);
        HIPCHK(hipStreamSynchronize(e->stream));
        std::vector<double> soa((size_t)M * REC);
        HIPCHK(hipMemcpy(soa.data(), drec, soa.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int t = 0; t < M; t++)
            for (int f = 0; f < REC; f++) rec[(size_t)t * REC + f] = soa[(size_t)f * M + t];
        (void)hipFree(dq); (void)hipFree(dob); (void)hipFree(drec);
    } catch (const std::bad_alloc&) {
        return fail(MPCC_E_OOM, "allocation failed");
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_debug_project(mpcc_engine* e, int M, const double* s_guess, const double* ee, double* s_out) {
    if (!e || M < 1 || !s_guess || !ee || !s_out) return fail(MPCC_E_INVALID, "mpcc_debug_project: invalid argument");
    DevGuard dg_(e);
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_debug_project: no track");
    double *dg = nullptr, *de = nullptr, *dout = nullptr;
    try {
        quiesce(e);
        dg = dmalloc<double>(M);
        de = dmalloc<double>((size_t)M * 3);
        dout = dmalloc<double>(M);
        HIPCHK(hipMemcpy(dg, s_guess, M * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(de, ee, (size_t)M * 3 * sizeof(double), hipMemcpyHostToDevice));
        DevConst c = e->make_const(1);
        launch_debug_project(c, M, dg, de, dout, e->stream);
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipMemcpy(s_out, dout, M * sizeof(double), hipMemcpyDeviceToHost));
    } catch (const std::exception& x) {
        (void)hipFree(dg); (void)hipFree(de); (void)hipFree(dout);
        return fail(MPCC_E_HIP, std::string("mpcc_debug_project: ") + x.what());
    }
    (void)hipFree(dg); (void)hipFree(de); (void)hipFree(dout);
    return MPCC_OK;
}

int mpcc_debug_spline(mpcc_engine* e, int M, const double* s, double* pos, double* dd1, double* dd2, double* R, double* dR) {
    if (!e || M < 1 || !s) return fail(MPCC_E_INVALID, "mpcc_debug_spline: invalid argument");
    DevGuard dg_(e);
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_debug_spline: no track");
    try {
        quiesce(e);
        double* ds = dmalloc<double>(M);
        double* dout = dmalloc<double>((size_t)M * 21);
        HIPCHK(hipMemcpy(ds, s, M * sizeof(double), hipMemcpyHostToDevice));
        DevConst c = e->make_const(1);
        launch_debug_spline(c, M, ds, dout, e->stream);
        HIPCHK(hipStreamSynchronize(e->stream));
        std::vector<double> o((size_t)M * 21);
        HIPCHK(hipMemcpy(o.data(), dout, o.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int t = 0; t < M; t++) {
            const double* r = &o[(size_t)t * 21];
            for (int a = 0; a < 3; a++) {
                if (pos) pos[3 * t + a] = r[a];
                if (dd1) dd1[3 * t + a] = r[3 + a];
                if (dd2) dd2[3 * t + a] = r[6 + a];
                if (dR) dR[3 * t + a] = r[18 + a];
            }
            if (R) for (int a = 0; a < 9; a++) R[9 * t + a] = r[9 + a];
        }
        (void)hipFree(ds); (void)hipFree(dout);
    } catch (const std::bad_alloc&) {
        return fail(MPCC_E_OOM, "allocation failed");
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

int mpcc_debug_stage_cost(mpcc_engine* e, int M, const double* x, const double* u, const double* rec, const int32_t* k,
                          double* obj, double* fx, double* fu, double* fxx, double* fuu) {
    if (!e || M < 1 || !x || !u || !rec || !k) return fail(MPCC_E_INVALID, "mpcc_debug_stage_cost: invalid argument");
    DevGuard dg_(e);
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_debug_stage_cost: no track");
    try {
        quiesce(e);
        const int W = 1 + NX + NU + NX * NX + NU * NU;
        double* dx = dmalloc<double>((size_t)M * NX);
        double* du = dmalloc<double>((size_t)M * NU);
        double* dr = dmalloc<double>((size_t)M * REC);
        int32_t* dk = dmalloc<int32_t>(M);
        double* dout = dmalloc<double>((size_t)M * W);
        std::vector<double> soa((size_t)M * REC);
        for (int t = 0; t < M; t++)
            for (int f = 0; f < REC; f++) soa[(size_t)f * M + t] = rec[(size_t)t * REC + f];
        HIPCHK(hipMemcpy(dx, x, M * NX * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(du, u, M * NU * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dr, soa.data(), soa.size() * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dk, k, M * sizeof(int32_t), hipMemcpyHostToDevice));
        DevConst c = e->make_const(1);
        launch_debug_cost(c, M, dx, du, dr, dk, dout, e->stream);
        HIPCHK(hipStreamSynchronize(e->stream));
        std::vector<double> o((size_t)M * W);
        HIPCHK(hipMemcpy(o.data(), dout, o.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int t = 0; t < M; t++) {
            const double* r = &o[(size_t)t * W];
            if (obj) obj[t] = r[0];
            if (fx) std::memcpy(fx + NX * t, r + 1, NX * sizeof(double));
            if (fu) std::memcpy(fu + NU * t, r + 1 + NX, NU * sizeof(double));
            if (fxx) std::memcpy(fxx + NX * NX * t, r + 1 + NX + NU, NX * NX * sizeof(double));
            if (fuu) std::memcpy(fuu + NU * NU * t, r + 1 + NX + NU + NX * NX, NU * NU * sizeof(double));
        }
        (void)hipFree(dx); (void)hipFree(du); (void)hipFree(dr); (void)hipFree(dk); (void)hipFree(dout);
    } catch (const std::bad_alloc&) {
        return fail(MPCC_E_OOM, "allocation failed");
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}

}  // extern "C"
static int debug_solve_qp(mpcc_engine* e, int B, const double* guess, const double* rec, const double* u_cur, int nlr,
                          const double* lr, const double* lrc, double* step, int32_t* qp_status, int32_t* ipm_iters);
extern "C" {

int mpcc_debug_solve_qp(mpcc_engine* e, int B, const double* guess, const double* rec, const double* u_cur, double* step,
                        int32_t* qp_status, int32_t* ipm_iters) {
    return debug_solve_qp(e, B, guess, rec, u_cur, -1, nullptr, nullptr, step, qp_status, ipm_iters);
}

int mpcc_debug_solve_qp_lr(mpcc_engine* e, int B, const double* guess, const double* rec, const double* u_cur, int nlr,
                           const double* lr, const double* lrc, double* step, int32_t* qp_status, int32_t* ipm_iters) {
    if (nlr < 0 || nlr > LRX || (nlr && (!lr || !lrc))) return fail(MPCC_E_INVALID, "mpcc_debug_solve_qp_lr: invalid argument");
    return debug_solve_qp(e, B, guess, rec, u_cur, nlr, lr, lrc, step, qp_status, ipm_iters);
}

}  // extern "C"

// nlr < 0: the build's regular QP solver; nlr >= 0: the 32-lane interior point with nlr low-rank terms
static int debug_solve_qp(mpcc_engine* e, int B, const double* guess, const double* rec, const double* u_cur, int nlr,
                          const double* lr, const double* lrc, double* step, int32_t* qp_status, int32_t* ipm_iters) {
    if (!e || B < 1 || B > e->maxB || !guess || !rec || !u_cur)
        return fail(MPCC_E_INVALID, "mpcc_debug_solve_qp: invalid argument");
    if (!e->has_track) return fail(MPCC_E_NOTRACK, "mpcc_debug_solve_qp: no track");
    DevGuard dg_(e);
    if (e->spl.stride && B > e->n_tracks) return fail(MPCC_E_INVALID, "mpcc_debug_solve_qp: more instances than per-instance tracks");
    try {
        quiesce(e);
        hipStream_t st = e->stream;
        const int N = e->N;
        const size_t NS = N + 1, S = (size_t)B * NS;
        DevConst c = e->make_const(B);
        std::vector<double> soa((size_t)REC * S);
        for (size_t t = 0; t < S; t++)
            for (int f = 0; f < REC; f++) soa[(size_t)f * S + t] = rec[t * REC + f];
        HIPCHK(hipMemcpy(e->d.guess, guess, S * NXU * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->d.rec, soa.data(), soa.size() * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->s_u0, u_cur, B * NU * sizeof(double), hipMemcpyHostToDevice));
        std::vector<int32_t> sqi((size_t)B * SQI, 0);
        for (int b = 0; b < B; b++) sqi[(size_t)b * SQI + SQ_ACTIVE] = 1;
        HIPCHK(hipMemcpy(e->d.sqi, sqi.data(), sqi.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(hipMemset(e->d.step, 0, S * NXU * sizeof(double)));
        if (nlr >= 0) {  // low-rank terms of every instance, then the 32-lane solver
            e->ensure_wide_buffers(true, (nlr + 1) / 2 + 1);  // room for nlr terms
            const size_t NE = S * NXU / B, L = (size_t)e->d.lrs;
            std::vector<double> l((size_t)B * L * NE, 0.0), lc((size_t)B * L, 0.0);
            for (int b = 0; b < B; b++)
                for (int j = 0; j < nlr; j++) {
                    std::memcpy(&l[((size_t)b * L + j) * NE], lr + (size_t)j * NE, NE * sizeof(double));
                    lc[(size_t)b * L + j] = lrc[j];
                }
            HIPCHK(hipMemcpy(e->d.lr, l.data(), l.size() * sizeof(double), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(e->d.lrc, lc.data(), lc.size() * sizeof(double), hipMemcpyHostToDevice));
            for (int b = 0; b < B; b++) sqi[(size_t)b * SQI + SQ_NLR] = nlr;
            HIPCHK(hipMemcpy(e->d.sqi, sqi.data(), sqi.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        }
        launch_setqp(c, e->d, e->s_u0, st);
        e->last_wide = DOF != 7 || nlr >= 0;
        if (nlr >= 0) launch_ipm_wide(c, e->d, poly_rows_max(c.p.constraint_mask), 1, st);
        else launch_ipm(c, e->d, poly_rows_max(c.p.constraint_mask), st);
        HIPCHK(hipStreamSynchronize(st));
        std::vector<double> stp(S * NXU);
        HIPCHK(hipMemcpy(stp.data(), e->d.step, stp.size() * sizeof(double), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(sqi.data(), e->d.sqi, sqi.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
        const size_t nv = NS * NX + (size_t)N * NU;
        for (int b = 0; b < B; b++) {
            for (size_t k = 0; k < NS; k++) {
                for (int a = 0; a < NX; a++) step[b * nv + NX * k + a] = stp[(b * NS + k) * NXU + a];
                if ((int)k < N)
                    for (int a = 0; a < NU; a++) step[b * nv + NX * NS + NU * k + a] = stp[(b * NS + k) * NXU + NX + a];
            }
            int active = sqi[(size_t)b * SQI + SQ_ACTIVE];
            int qs = sqi[(size_t)b * SQI + SQ_QPSTAT];
            if (qp_status) qp_status[b] = active ? qs : sqi[(size_t)b * SQI + SQ_STATUS];
            if (ipm_iters) ipm_iters[b] = sqi[(size_t)b * SQI + SQ_IPMIT];
        }
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}


int mpcc_debug_trace_enable(mpcc_engine* e, int enable) {
    if (!e) return fail(MPCC_E_INVALID, "mpcc_debug_trace_enable: null engine");
    DevGuard dg_(e);
    try {
        quiesce(e);
        if (enable && !e->d.dbg_trace) e->d.dbg_trace = dmalloc<double>((size_t)e->cfg.max_batch * TRACE_IT * TRACE_W);
        if (!enable && e->d.dbg_trace) { HIPCHK(hipFree(e->d.dbg_trace)); e->d.dbg_trace = nullptr; }
    } catch (const std::exception& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_debug_trace_enable: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_debug_trace_get(mpcc_engine* e, int B, double* out) {
    if (!e || !out || B < 1 || B > e->cfg.max_batch || !e->d.dbg_trace)
        return fail(MPCC_E_INVALID, "mpcc_debug_trace_get: invalid argument or trace disabled");
    DevGuard dg_(e);
    try {
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy(out, e->d.dbg_trace, sizeof(double) * B * TRACE_IT * TRACE_W, hipMemcpyDeviceToHost));
    } catch (const std::exception& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_debug_trace_get: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_debug_workspace(mpcc_engine* e, int B, double* out) {
    if (!e || !out || B < 1 || B > e->cfg.max_batch) return fail(MPCC_E_INVALID, "mpcc_debug_workspace: invalid argument");
    // the Panda library's BFGS / MPCC_WIDE_SQP solves use the 32-lane workspace (ISW doubles per stage), which
    // does not fit the caller's [B*(N+1)*MPCC_IPM_WS] buffer: refused rather than returning the stale 16-lane one
    if (DOF == 7 && e->last_wide)
        return fail(MPCC_E_INVALID, "mpcc_debug_workspace: the last solve used the 32-lane interior point (use_BFGS / "
                                    "MPCC_WIDE_SQP); its workspace is not in the 16-lane layout");
    DevGuard dg_(e);
    try {
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy(out, e->d.is, sizeof(double) * (size_t)B * (e->N + 1) * IS, hipMemcpyDeviceToHost));
    } catch (const std::exception& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_debug_workspace: ") + x.what());
    }
    return MPCC_OK;
}

int mpcc_debug_bounds(mpcc_engine* e, uint32_t* flags, int clear) {
    if (!e || !flags) return fail(MPCC_E_INVALID, "mpcc_debug_bounds: null argument");
    if (!e->bchk) return fail(MPCC_E_INVALID, "mpcc_debug_bounds: not a bounds-checked build (MPCC_BOUNDS_CHECK)");
    DevGuard dg_(e);
    try {
        HIPCHK(hipDeviceSynchronize());
        uint32_t w[64];
        HIPCHK(hipMemcpy(w, e->bchk, sizeof w, hipMemcpyDeviceToHost));
        uint32_t o = 0;
        for (uint32_t x : w) o |= x;
        *flags = o;
        if (clear) HIPCHK(hipMemset(e->bchk, 0, sizeof w));
    } catch (const std::exception& x) {
        return fail(MPCC_E_HIP, std::string("mpcc_debug_bounds: ") + x.what());
    }
    return MPCC_OK;
}

#ifndef MPCC_BUILD_ID
#define MPCC_BUILD_ID "unknown"
#endif
const char* mpcc_build_id(void) { return MPCC_BUILD_ID; }
int mpcc_build_flags(void) {
    int f = 0;
#ifdef MPCC_BOUNDS_CHECK
    f |= MPCC_BUILD_BOUNDS_CHECK;
#endif
#ifdef MPCC_IPM_PROF
    f |= MPCC_BUILD_PROF;
#endif
    return f;
}

int mpcc_timing_sqp(mpcc_engine* e, double* span_s, int32_t* n, double* frac4) {
    if (!e) return fail(MPCC_E_INVALID, "mpcc_timing_sqp: null engine");
    if (span_s) *span_s = e->last_sqp_s;
    if (n) *n = e->last_sqp_n;
    if (frac4)
        for (int i = 0; i < PH_N; i++) frac4[i] = e->last_frac[i];
    return MPCC_OK;
}

int mpcc_timing_mlp(mpcc_engine* e, double* self_s, int32_t* self_n, double* env_s, int32_t* env_n) {
    if (!e) return fail(MPCC_E_INVALID, "mpcc_timing_mlp: null engine");
    if (self_s) *self_s = e->last_mlp_self_s;
    if (self_n) *self_n = e->last_mlp_self_n;
    if (env_s) *env_s = e->last_mlp_env_s;
    if (env_n) *env_n = e->last_mlp_env_n;
    return MPCC_OK;
}

int mpcc_timing_intervals(mpcc_engine* e, mpcc_engine* anchor, int kind, int max, double* start_ms, double* end_ms,
                          int32_t* n) {
    if (!e || !anchor || !n || max < 0 || (max && (!start_ms || !end_ms)) || kind < 0 || kind > 2)
        return fail(MPCC_E_INVALID, "mpcc_timing_intervals: invalid argument");
    if (anchor->lv_total.empty() || e->cfg.device != anchor->cfg.device)
        return fail(MPCC_E_INVALID, "mpcc_timing_intervals: the anchor engine has no timing window on this device");
    const auto& lv = kind == MPCC_TIMING_QP ? e->lv_ipm : (kind == MPCC_TIMING_MLP_SELF ? e->lv_mlp_self : e->lv_mlp_env);
    DevGuard dg_(e);
    try {
        const hipEvent_t a0 = anchor->lv_total.front().first;
        HIPCHK(hipEventSynchronize(a0));
        int k = 0;
        for (auto& pr : lv) {
            if (k >= max) break;
            HIPCHK(hipEventSynchronize(pr.second));
            float s = 0, t = 0;
            HIPCHK(hipEventElapsedTime(&s, a0, pr.first));
            HIPCHK(hipEventElapsedTime(&t, a0, pr.second));
            start_ms[k] = s;
            end_ms[k] = t;
            k++;
        }
        // the number of intervals recorded, which may exceed max (only the first max were written): a caller that
        // sized its buffers too small sees n > max instead of a silently truncated list
        *n = (int32_t)lv.size();
    } catch (const HipError& x) {
        return fail(MPCC_E_HIP, x.what());
    }
    return MPCC_OK;
}
