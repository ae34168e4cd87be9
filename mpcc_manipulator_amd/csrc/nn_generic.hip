// nn_generic.hip — the reference's stand-alone network and kinematics objects on the GPU, for the
// MPCC_WRAPPER surface:
//   * SelCollNNmodel / EnvCollNNmodel::setNeuralNetwork + calculateMlpOutput (SelfCollisionModel.cpp /
//     EnvCollisionModel.cpp:75-250) for any architecture the reference accepts (n_input, n_output, hidden
//     sizes, NeRF encoding on or off): the output and its full Jacobian with respect to every input, the
//     10-column env Jacobian included (quirk Q17: the solve itself only uses its 9x7 block);
//   * RobotModel frame queries (robot_model.cpp:354-450): position, orientation and Jacobian of any frame
//     1..9 (panda_link0..link7, panda_hand_tcp), its manipulability and the central-difference gradient.
// The solve path does not use these: its MLPs are the FP64-MFMA kernels of mlp.hip and its kinematics
// the record kernel.  Here one workgroup evaluates one sample, rows of a layer spread over its 256
// threads, value and tangent columns in LDS; weights are stored transposed ([k][row]) so the threads of
// a layer read each k-slice of W coalesced.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "dev_model.h"
#include "kernels.h"
#include "mpcc_engine.h"

namespace mpcc {

constexpr int GMLP_MAXL = 8;     // layers (hidden + output)
constexpr int GMLP_MAXIN = 16;   // raw inputs (Jacobian columns)
constexpr int GMLP_THREADS = 256;

struct GMlpDesc {
    int L, nin, nout, nerf, maxw, enc;  // enc = width of the first layer's input (3 nin with NeRF)
    int rows[GMLP_MAXL], cols[GMLP_MAXL];
    long offW[GMLP_MAXL], offb[GMLP_MAXL];
};

namespace {

// value column 0 and tangent columns 1..nin of one layer's activations: act[c * maxw + k]
__global__ void __launch_bounds__(GMLP_THREADS) k_mlp_generic(GMlpDesc g, const double* __restrict__ W, int M,
                                                             const double* __restrict__ in, double* __restrict__ out,
                                                             double* __restrict__ jac) {
    extern __shared__ double sm[];
    const int m = blockIdx.x;
    if (m >= M) return;
    const int C1 = 1 + g.nin, n = g.nin;
    double* enc = sm;                    // encoded input [enc]
    double* A = sm + g.enc;              // activations of the previous layer [C1][maxw]
    double* Bf = A + (size_t)C1 * g.maxw;
    const double* x = in + (size_t)m * n;
    for (int k = threadIdx.x; k < g.enc; k += blockDim.x) {
        const int j = k % n, part = k / n;
        const double v = x[j];
        enc[k] = g.nerf ? (part == 0 ? v : (part == 1 ? sin(v) : cos(v))) : v;
    }
    __syncthreads();
    for (int l = 0; l < g.L; l++) {
        const int R = g.rows[l], K = g.cols[l];
        const double* Wl = W + g.offW[l];  // transposed: Wl[k * R + r]
        const double* bl = W + g.offb[l];
        const bool last = l == g.L - 1;
        for (int r = threadIdx.x; r < R; r += blockDim.x) {
            double acc[GMLP_MAXIN + 1];
#pragma unroll
            for (int c = 0; c <= GMLP_MAXIN; c++) acc[c] = 0.0;
            if (l == 0) {
                // hidden = W0 * input (+ b); d hidden / d input = relu' * W0 * nerf_jac (SelfCollisionModel.cpp:163-186)
                for (int k = 0; k < K; k++) acc[0] += Wl[(size_t)k * R + r] * enc[k];
#pragma unroll
                for (int c = 0; c < GMLP_MAXIN; c++) {
                    if (c >= n) break;
                    double t = Wl[(size_t)c * R + r];
                    if (g.nerf) {
                        const double v = x[c];
                        t += Wl[(size_t)(n + c) * R + r] * cos(v);
                        t += Wl[(size_t)(2 * n + c) * R + r] * (-sin(v));
                    }
                    acc[1 + c] = t;
                }
            } else {
                for (int k = 0; k < K; k++) {
                    const double w = Wl[(size_t)k * R + r];
#pragma unroll
                    for (int c = 0; c <= GMLP_MAXIN; c++)
                        if (c < C1) acc[c] += w * A[(size_t)c * g.maxw + k];
                }
            }
            const double z = acc[0] + bl[r];
            if (last) {
                out[(size_t)m * g.nout + r] = z;
#pragma unroll
                for (int c = 0; c < GMLP_MAXIN; c++)
                    if (c < n) jac[((size_t)m * g.nout + r) * n + c] = acc[1 + c];
            } else {
                const double gate = (z > 0) ? 1.0 : 0.0;  // ReLU_derivative (SelfCollisionModel.h:66-69)
                Bf[r] = fmax(0.0, z);
#pragma unroll
                for (int c = 0; c < GMLP_MAXIN; c++)
                    if (c < n) Bf[(size_t)(1 + c) * g.maxw + r] = gate * acc[1 + c];
            }
        }
        __syncthreads();
        double* t = A; A = Bf; Bf = t;
    }
}

// RobotModel frame record: pos(3) R(9) J(42) mani(1) dmani(7) = 62 doubles per query
constexpr int FREC = 62;
__global__ void __launch_bounds__(64) k_robot_frames(int M, const double* __restrict__ q, int frame, double* __restrict__ o) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    double qq[7];
    for (int j = 0; j < 7; j++) qq[j] = q[7 * i + j];
    double* r = o + (size_t)i * FREC;
    double J[42];
    panda_frame(qq, frame, r, r + 3, J);
    for (int a = 0; a < 42; a++) r[12 + a] = J[a];
    r[54] = manip_from_J<7>(J);
    const double delta = 1e-4;  // robot_model.cpp:439
    for (int j = 0; j < 7; j++) {
        double qp[7], qm[7], Jp[42], Jm[42];
        for (int a = 0; a < 7; a++) { qp[a] = qq[a] + (a == j ? delta : 0.0); qm[a] = qq[a] - (a == j ? delta : 0.0); }
        panda_frame(qp, frame, nullptr, nullptr, Jp);
        panda_frame(qm, frame, nullptr, nullptr, Jm);
        r[55 + j] = (manip_from_J<7>(Jp) - manip_from_J<7>(Jm)) / (2 * delta);
    }
}

}  // namespace
}  // namespace mpcc

using namespace mpcc;

struct mpcc_mlp {
    int device = 0;
    GMlpDesc desc{};
    double* d_w = nullptr;
    double* d_in = nullptr;
    double* d_out = nullptr;
    int cap = 0;  // samples the I/O buffers hold
    ~mpcc_mlp() {
        for (double* p : {d_w, d_in, d_out})
            if (p) (void)hipFree(p);
    }
};

namespace {
struct GuardDev {
    int prev = -1, dev;
    explicit GuardDev(int d) : dev(d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~GuardDev() {
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
};
size_t gmlp_lds(const GMlpDesc& g) { return sizeof(double) * ((size_t)g.enc + 2 * (size_t)(1 + g.nin) * g.maxw); }
int gfail(int code, const std::string& m) {
    set_last_error(m);
    return code;
}
}  // namespace

extern "C" {

int mpcc_mlp_create(int device, const char* dir, int n_input, int n_output, const int32_t* n_hidden, int n_layers_hidden,
                    int is_nerf, mpcc_mlp** out) {
    if (!dir || !out || n_input < 1 || n_input > GMLP_MAXIN || n_output < 1 || n_layers_hidden < 0 ||
        n_layers_hidden + 1 > GMLP_MAXL || (n_layers_hidden && !n_hidden))
        return gfail(MPCC_E_INVALID, "mpcc_mlp_create: invalid architecture (1..16 inputs, <= 7 hidden layers)");
    std::unique_ptr<mpcc_mlp> m(new mpcc_mlp());
    m->device = device;
    GMlpDesc& g = m->desc;
    g.L = n_layers_hidden + 1;
    g.nin = n_input;
    g.nout = n_output;
    g.nerf = is_nerf ? 1 : 0;
    g.enc = (is_nerf ? 3 : 1) * n_input;
    g.maxw = 1;
    std::vector<double> packed;
    try {
        for (int l = 0; l < g.L; l++) {
            const int R = (l == g.L - 1) ? n_output : n_hidden[l];
            const int K = (l == 0) ? g.enc : n_hidden[l - 1];
            if (R < 1) throw std::invalid_argument("layer width must be >= 1");
            if (l < g.L - 1) g.maxw = std::max(g.maxw, R);
            std::vector<double> Wv, bv;
            if (!nn_read_layer(dir, l, R, K, Wv, bv))
                throw std::runtime_error("cannot read layer " + std::to_string(l) + " (" + std::to_string(R) + "x" +
                                         std::to_string(K) + ") under " + std::string(dir));
            g.rows[l] = R;
            g.cols[l] = K;
            g.offW[l] = (long)packed.size();
            for (int k = 0; k < K; k++)
                for (int r = 0; r < R; r++) packed.push_back(Wv[(size_t)r * K + k]);
            g.offb[l] = (long)packed.size();
            packed.insert(packed.end(), bv.begin(), bv.end());
        }
        if (gmlp_lds(g) > 64 * 1024) throw std::invalid_argument("network too wide for the LDS of one workgroup");
        GuardDev gd(device);
        if (hipMalloc(&m->d_w, packed.size() * sizeof(double)) != hipSuccess) return gfail(MPCC_E_OOM, "mpcc_mlp_create: hipMalloc");
        if (hipMemcpy(m->d_w, packed.data(), packed.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
            return gfail(MPCC_E_HIP, "mpcc_mlp_create: hipMemcpy");
    } catch (const std::invalid_argument& x) {
        return gfail(MPCC_E_INVALID, std::string("mpcc_mlp_create: ") + x.what());
    } catch (const std::exception& x) {
        return gfail(MPCC_E_IO, std::string("mpcc_mlp_create: ") + x.what());
    }
    *out = m.release();
    return MPCC_OK;
}

int mpcc_mlp_eval(mpcc_mlp* m, int M, const double* in, double* out, double* jac) {
    if (!m || M < 0 || (M && (!in || !out))) return gfail(MPCC_E_INVALID, "mpcc_mlp_eval: invalid argument");
    if (M == 0) return MPCC_OK;
    GuardDev gd(m->device);
    const GMlpDesc& g = m->desc;
    const size_t nin = (size_t)M * g.nin, nout = (size_t)M * g.nout, nj = nout * g.nin;
    if (M > m->cap) {
        for (double** p : {&m->d_in, &m->d_out}) {
            if (*p) (void)hipFree(*p);
            *p = nullptr;
        }
        if (hipMalloc(&m->d_in, nin * sizeof(double)) != hipSuccess ||
            hipMalloc(&m->d_out, (nout + nj) * sizeof(double)) != hipSuccess) {
            m->cap = 0;
            return gfail(MPCC_E_OOM, "mpcc_mlp_eval: hipMalloc");
        }
        m->cap = M;
    }
    if (hipMemcpy(m->d_in, in, nin * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
        return gfail(MPCC_E_HIP, "mpcc_mlp_eval: hipMemcpy");
    hipLaunchKernelGGL(k_mlp_generic, dim3(M), dim3(GMLP_THREADS), gmlp_lds(g), 0, g, m->d_w, M, m->d_in, m->d_out,
                       m->d_out + nout);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return gfail(MPCC_E_HIP, "mpcc_mlp_eval: kernel failed");
    if (hipMemcpy(out, m->d_out, nout * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
        (jac && hipMemcpy(jac, m->d_out + nout, nj * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess))
        return gfail(MPCC_E_HIP, "mpcc_mlp_eval: hipMemcpy");
    return MPCC_OK;
}

void mpcc_mlp_destroy(mpcc_mlp* m) {
    if (!m) return;
    GuardDev gd(m->device);
    (void)hipDeviceSynchronize();
    delete m;
}

int mpcc_mlp_dims(mpcc_mlp* m, int32_t* n_input, int32_t* n_output) {
    if (!m) return gfail(MPCC_E_INVALID, "mpcc_mlp_dims: null");
    if (n_input) *n_input = m->desc.nin;
    if (n_output) *n_output = m->desc.nout;
    return MPCC_OK;
}

int mpcc_robot_frames(int device, int M, const double* q, int frame_id, double* pos, double* R, double* J, double* mani,
                      double* dmani) {
    if (M < 0 || (M && !q) || frame_id < 1 || frame_id > 9)
        return gfail(MPCC_E_INVALID, "mpcc_robot_frames: invalid argument (frame_id 1..9)");
    if (M == 0) return MPCC_OK;
    GuardDev gd(device);
    double *dq = nullptr, *dout = nullptr;
    if (hipMalloc(&dq, (size_t)M * 7 * sizeof(double)) != hipSuccess ||
        hipMalloc(&dout, (size_t)M * FREC * sizeof(double)) != hipSuccess) {
        if (dq) (void)hipFree(dq);
        return gfail(MPCC_E_OOM, "mpcc_robot_frames: hipMalloc");
    }
    std::vector<double> o((size_t)M * FREC);
    bool ok = hipMemcpy(dq, q, (size_t)M * 7 * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_robot_frames, dim3((M + 63) / 64), dim3(64), 0, 0, M, dq, frame_id, dout);
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpy(o.data(), dout, o.size() * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(dq);
    (void)hipFree(dout);
    if (!ok) return gfail(MPCC_E_HIP, "mpcc_robot_frames: HIP error");
    for (int i = 0; i < M; i++) {
        const double* r = o.data() + (size_t)i * FREC;
        if (pos) std::memcpy(pos + 3 * i, r, 3 * sizeof(double));
        if (R) std::memcpy(R + 9 * i, r + 3, 9 * sizeof(double));
        if (J) std::memcpy(J + 42 * i, r + 12, 42 * sizeof(double));
        if (mani) mani[i] = r[54];
        if (dmani) std::memcpy(dmani + 7 * i, r + 55, 7 * sizeof(double));
    }
    return MPCC_OK;
}

}  // extern "C"
