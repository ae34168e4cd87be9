// mlp.hip — k_mlp: the collision MLPs (SelCollNNmodel / EnvCollNNmodel::calculateMlpOutput,
// SelfCollisionModel.cpp:140-250, EnvCollisionModel.cpp:137-247) with their forward-mode input
// Jacobian, as FP64 MFMA GEMMs over (instance, stage) samples.
//
// One wave carries 2 samples x 8 columns (value + 7 tangent directions dq_0..dq_6) = one 16-column
// tile through every layer: Z = W X is v_mfma_f64_16x16x4f64 over 16-row tiles of W and 4-deep k-steps.
//  * The f64 C/D layout (lane l, reg r -> row (l>>4) + 4r of the tile, column l&15) is exactly the
//    B-operand layout of the next layer's k-step 4t + r, so activations stay in registers from layer
//    to layer — no LDS.  Bias, ReLU (value columns) and ReLU' gating (tangent columns, the value of
//    the same sample broadcast over the 16-lane row by DPP) are applied in place between layers.
//  * W is packed on the host in fragment order ([row tile][k-step][lane]), zero-padded to 16-row /
//    4-column multiples: every A fragment is one coalesced 512-byte line.  Both networks' weights
//    (1.84 MB) stay L2-resident.  The 256-row layers (both input layers, the env hidden layers)
//    stage each k-tile of W through LDS for the block's 4 waves (mfma_layer_lds), so a weight element
//    loaded from L2 feeds 4 x 16 columns = 8 samples: k_mlp_env 51.5 -> 23.7 ms on 335,872 samples,
//    27% -> 58% of the FP64 roof; k_mlp_self 5.9 -> 4.8 ms.
//  * v_mfma_f64_16x16x4f64 accumulates as an ascending fma chain over k (bitwise,
//    tools/probes/mfma_f64_probe.hip); the oracle's MLP uses the same chain.
#include <type_traits>

#include "dev_model.h"
#include "dev_dpp.h"
#include "kernels.h"

namespace mpcc {
namespace {

using namespace dpp;
typedef double d4 __attribute__((ext_vector_type(4)));

// out[t] = sum_k W[16t + row][k] in[k] over KT k-tiles (4 k-steps of 4 each), RT 16-row output tiles
template <int KT, int RT>
__device__ __forceinline__ void mfma_layer(const double* __restrict__ Wp, const d4 (&in)[KT], d4 (&out)[RT],
                                           int lane) {
    constexpr int KS = 4 * KT;
#pragma unroll
    for (int t = 0; t < RT; t++) out[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kt = 0; kt < KT; kt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int s = 4 * kt + r;
#pragma unroll
            for (int t = 0; t < RT; t++)
                out[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(Wp[((size_t)t * KS + s) * 64 + lane], in[kt][r], out[t], 0,
                                                              0, 0);
        }
}

// The same layer with the weights staged through LDS for the block's 4 waves: k-tile kt of every row
// tile (RT x 4 k-steps x 64 lanes = RT x 2 KB) is loaded once per block, cooperatively and coalesced,
// into one of two LDS buffers while the MFMAs of k-tile kt - 1 run from the other.  Every A fragment
// then comes from L2 once per 4 waves (8 samples) instead of once per wave, and the per-MFMA operand
// latency is an LDS read.  Same fragments, same ascending k order per row tile: bitwise the result
// of mfma_layer.  All 256 threads of the block must call it (it contains barriers).
template <int KT, int RT>
__device__ __forceinline__ void mfma_layer_lds(const double* __restrict__ Wp, const d4 (&in)[KT], d4 (&out)[RT],
                                               int lane, double* __restrict__ lds /* 2 x RT*256 */) {
    constexpr int KS = 4 * KT;
    constexpr int CH = RT * 256;       // doubles per k-tile chunk
    constexpr int PT = CH / 256 / 2;   // double2 per thread per chunk
    static_assert(RT % 2 == 0, "mfma_layer_lds: RT must be even");
    const int tid = threadIdx.x;
    double2 st[PT];
    auto fetch = [&](int kt) {
#pragma unroll
        for (int j = 0; j < PT; j++) {
            const int idx = 2 * (tid + 256 * j);           // chunk element: [t][r][lane]
            const int t = idx >> 8, w = idx & 255;
            st[j] = *reinterpret_cast<const double2*>(Wp + ((size_t)t * KS + 4 * kt) * 64 + w);
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int j = 0; j < PT; j++) reinterpret_cast<double2*>(lds + buf * CH)[tid + 256 * j] = st[j];
    };
#pragma unroll
    for (int t = 0; t < RT; t++) out[t] = d4{0.0, 0.0, 0.0, 0.0};
    fetch(0);
    stash(0);
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < KT; kt++) {
        if (kt + 1 < KT) fetch(kt + 1);
        const double* L = lds + (kt & 1) * CH;
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int t = 0; t < RT; t++)
                out[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(L[(t * 4 + r) * 64 + lane], in[kt][r], out[t], 0, 0, 0);
        if (kt + 1 < KT) stash((kt + 1) & 1);
        __syncthreads();
    }
}

// The same layer with the k-tiles of W streamed into a 3-slot LDS ring by global_load_lds_dwordx4 (16 bytes per
// lane straight to LDS, no register staging), two k-tiles ahead: the block's 4 waves each copy a quarter of a
// tile, wait for their own copies (vmcnt), then one barrier per k-tile makes the tile visible to all and retires
// the slot read two tiles ago, which the next copy overwrites.  The register-staged double buffer (mfma_layer_lds)
// waited on the L2 latency of the tile it had just fetched at every stash.  Same fragments, same ascending k
// order per row tile: bitwise the result of mfma_layer.  All 256 threads of the block must call it.
constexpr int RING_SLOTS = 3;
__device__ __forceinline__ void glds16_to(const void* src, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}
template <int KT, int RT, int NW = 4>
__device__ __forceinline__ void mfma_layer_ring(const double* __restrict__ Wp, const d4 (&in)[KT], d4 (&out)[RT],
                                                int lane, double* __restrict__ ring /* RING_SLOTS x RT*256 */) {
    constexpr int KS = 4 * KT;
    constexpr int CH = RT * 256;          // doubles per k-tile
    constexpr int PT = CH / 2 / (64 * NW);  // 16-byte copies per thread per k-tile
    static_assert(CH % (128 * NW) == 0, "mfma_layer_ring: whole 16-byte copies per thread");
    const int tid = threadIdx.x, w = tid >> 6;
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)ring;
    auto issue = [&](int kt) {  // k-tile kt into slot kt % RING_SLOTS; copy j of wave w: 1 KB at NW KB j + 1 KB w
        const unsigned slot = base + (unsigned)((kt % RING_SLOTS) * CH * 8);
#pragma unroll
        for (int j = 0; j < PT; j++) {
            const int e = tid + 64 * NW * j;  // 16-byte element of the tile: double 2e = [t][r][lane]
            const int t = e >> 7;
            glds16_to(Wp + ((size_t)t * KS + 4 * kt) * 64 + 2 * (e & 127),
                      __builtin_amdgcn_readfirstlane(slot + 1024u * (NW * j + w)));
        }
    };
#pragma unroll
    for (int t = 0; t < RT; t++) out[t] = d4{0.0, 0.0, 0.0, 0.0};
    issue(0);
    if (KT > 1) issue(1);
#pragma unroll
    for (int kt = 0; kt < KT; kt++) {
        // this wave's copies of tile kt have landed once at most those of tile kt + 1 are outstanding
        if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PT) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kt + 2 < KT) issue(kt + 2);
        const double* L = ring + (kt % RING_SLOTS) * CH;
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int t = 0; t < RT; t++)
                out[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(L[(t * 4 + r) * 64 + lane], in[kt][r], out[t], 0, 0, 0);
    }
    __syncthreads();  // the ring is free for the next layer's first copies
}

// mfma_layer_ring with the A fragments read one k-step ahead: the fragment of row tile t is reloaded right after
// its MFMA issues, with the next k-step's, so each LDS read has the other RT - 1 MFMAs of the k-step to land
// (mfma_layer_ring read each fragment just before its MFMA: with one wave per SIMD the matrix core waited on the
// LDS latency, profiles/r03bg_cfg2_env_k_mlp_env_pmc.json 65% SQ_WAIT_INST_ANY).  The next tile's first
// fragments are read during the tile's last k-step, so its barrier (own copies landed, tile visible to the
// block) moves to that k-step; the copy two tiles ahead is issued right after it, into the slot of the tile
// every wave has finished reading.  Same MFMAs in the same order per row tile: bitwise mfma_layer.
#ifndef MPCC_MLP_PF
#define MPCC_MLP_PF 1
#endif
// RS ring slots: the barrier of tile kt sits in its last k-step, after which no wave reads tile kt's slot again, so the
// copy of tile kt + 2 may go into it: two slots suffice (RS = 2; three keep one more tile of slack)
template <int KT, int RT, int NW = 4, int RS = RING_SLOTS>
__device__ __forceinline__ void mfma_layer_ring_pf(const double* __restrict__ Wp, const d4 (&in)[KT], d4 (&out)[RT],
                                                   int lane, double* __restrict__ ring /* RS x RT*256 */) {
    constexpr int KS = 4 * KT;
    constexpr int CH = RT * 256;
    constexpr int PT = CH / 2 / (64 * NW);
    static_assert(CH % (128 * NW) == 0, "mfma_layer_ring_pf: whole 16-byte copies per thread");
    static_assert(RS >= 2, "two ring slots at least");
    const int tid = threadIdx.x, w = tid >> 6;
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)ring;
    auto issue = [&](int kt) {
        const unsigned slot = base + (unsigned)((kt % RS) * CH * 8);
#pragma unroll
        for (int j = 0; j < PT; j++) {
            const int e = tid + 64 * NW * j;
            const int t = e >> 7;
            glds16_to(Wp + ((size_t)t * KS + 4 * kt) * 64 + 2 * (e & 127),
                      __builtin_amdgcn_readfirstlane(slot + 1024u * (NW * j + w)));
        }
    };
#pragma unroll
    for (int t = 0; t < RT; t++) out[t] = d4{0.0, 0.0, 0.0, 0.0};
    issue(0);
    if (KT > 1) {
        issue(1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PT) : "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    double fr[RT];
#pragma unroll
    for (int t = 0; t < RT; t++) fr[t] = ring[(t * 4) * 64 + lane];
#pragma unroll
    for (int kt = 0; kt < KT; kt++) {
        const double* L = ring + (kt % RS) * CH;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if (r == 3 && kt + 1 < KT) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of tile kt + 1
                __syncthreads();
                if (kt + 2 < KT) issue(kt + 2);
            }
            const bool nxt = r < 3 || kt + 1 < KT;
            const double* Ln = (r < 3) ? L : ring + ((kt + 1) % RS) * CH;
            const int rn = (r < 3) ? r + 1 : 0;
#pragma unroll
            for (int t = 0; t < RT; t++) {
                out[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[t], in[kt][r], out[t], 0, 0, 0);
                if (nxt) fr[t] = Ln[(t * 4 + rn) * 64 + lane];
            }
        }
    }
    __syncthreads();  // the ring is free for the next layer's first copies
}

// relu_gate on one 16-row output tile (bias_t = the layer's bias from row 16 t): the same operations per element
template <int CPS>
__device__ __forceinline__ void relu_tile(d4& a, const double* __restrict__ bias_t, int lane) {
    const bool isv = (lane & (CPS - 1)) == 0;
    const bool hi = CPS == 8 && (lane & 8) != 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const double z = a[r] + bias_t[(lane >> 4) + 4 * r];
        double zs;
        if constexpr (CPS == 4) {
            zs = dpp_d<0x00>(z);
        } else {
            const double z0 = bc<0>(z), z8 = bc<8>(z);
            zs = hi ? z8 : z0;
        }
        const bool on = zs > 0.0;
        a[r] = isv ? (z > 0.0 ? z : 0.0) : (on ? a[r] : 0.0);
    }
}

// The layers of one network as ONE stream of weight k-tiles through the LDS ring (mfma_layer_ring_pf per layer
// started every layer with an empty ring: the first tile's L2 latency, a barrier and the previous layer's ReLU
// epilogue with the matrix core idle).  Stream tile g goes to slot g % RS; a layer's last two k-steps issue the
// next layer's first two tiles and read its first fragments, and the ReLU of the layer's input tile kt + 1 (the
// previous layer's output, pre-activation, when bias_in is set) is formed during the MFMAs of tile kt.  Entry:
// stream tiles g0 and g0 + 1 issued, g0 visible to the block, fr = its k-step-0 fragments; exit (KTN > 0): the
// same for the next layer (KTN k-tiles at Wn).  Same fragments, same ascending k order per row tile and the
// same ReLU arithmetic: bitwise mfma_layer_ring_pf + relu_gate.  All threads of the block must call it.
template <int KT, int RT, int NW, int RS, int KTN, int CPS>
__device__ __forceinline__ void mfma_layer_chain(const double* __restrict__ Wp, const double* __restrict__ Wn, int g0,
                                                 d4 (&in)[KT], const double* __restrict__ bias_in, d4 (&out)[RT],
                                                 double (&fr)[RT], int lane, double* __restrict__ ring) {
    constexpr int KS = 4 * KT, KSN = 4 * KTN;
    constexpr int CH = RT * 256;
    constexpr int PT = CH / 2 / (64 * NW);
    static_assert(CH % (128 * NW) == 0, "mfma_layer_chain: whole 16-byte copies per thread");
    static_assert(RS >= 2 && KT >= 2 && (KTN == 0 || KTN >= 2), "two slots; two tiles per layer");
    const int tid = threadIdx.x, w = tid >> 6;
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)ring;
    auto issue = [&](const double* Wsrc, int ks, int j, int g) {
        const unsigned slot = base + (unsigned)((g % RS) * CH * 8);
#pragma unroll
        for (int q = 0; q < PT; q++) {
            const int e = tid + 64 * NW * q;
            const int t = e >> 7;
            glds16_to(Wsrc + ((size_t)t * ks + 4 * j) * 64 + 2 * (e & 127),
                      __builtin_amdgcn_readfirstlane(slot + 1024u * (NW * q + w)));
        }
    };
#pragma unroll
    for (int t = 0; t < RT; t++) out[t] = d4{0.0, 0.0, 0.0, 0.0};
    if (bias_in) relu_tile<CPS>(in[0], bias_in, lane);
#pragma unroll
    for (int kt = 0; kt < KT; kt++) {
        const double* L = ring + ((g0 + kt) % RS) * CH;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const bool more = kt + 1 < KT || KTN > 0;  // a next tile in the stream
            if (r == 3 && more) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of stream tile g0 + kt + 1
                __syncthreads();
                if (kt + 2 < KT) issue(Wp, KS, kt + 2, g0 + kt + 2);
                else if (KTN > 0) issue(Wn, KSN, kt + 2 - KT, g0 + kt + 2);
            }
            const bool nxt = r < 3 || more;
            const double* Ln = (r < 3) ? L : ring + ((g0 + kt + 1) % RS) * CH;
            const int rn = (r < 3) ? r + 1 : 0;
#pragma unroll
            for (int t = 0; t < RT; t++) {
                out[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fr[t], in[kt][r], out[t], 0, 0, 0);
                if (nxt) fr[t] = Ln[(t * 4 + rn) * 64 + lane];
            }
            if (r == 0 && bias_in && kt + 1 < KT) {
                // keep the ReLU of tile kt + 1 (and its bias reads) in this k-step: hoisted to the layer's start, the
                // bias operands of all tiles held 128 more registers and spilled
                __builtin_amdgcn_sched_barrier(0);
                relu_tile<CPS>(in[kt + 1], bias_in + 16 * (kt + 1), lane);
            }
        }
    }
    if (KTN == 0) __syncthreads();  // end of the stream: the ring is free
}

// hidden-layer epilogue: value columns h = relu(z + b); tangent columns dh = (z + b > 0) ? dz : 0.
// CPS = columns per sample: 8 (value + 7 tangents, 2 samples per 16-column tile), 4 (value + 3 tangents, 4 samples
// per tile: the mobile env network's obstacle directions) or 16 (value + up to 15 tangents, one sample per tile).
template <int RT, int CPS = 8>
__device__ __forceinline__ void relu_gate(d4 (&a)[RT], const double* __restrict__ bias, int lane) {
    const bool isv = (lane & (CPS - 1)) == 0;
    const bool hi = CPS == 8 && (lane & 8) != 0;
#pragma unroll
    for (int t = 0; t < RT; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const double z = a[t][r] + bias[16 * t + (lane >> 4) + 4 * r];
            double zs;  // the value of this lane's sample in this row
            if constexpr (CPS == 4) {
                zs = dpp_d<0x00>(z);  // quad_perm [0,0,0,0]: the quad's lane 0
            } else {
                const double z0 = bc<0>(z), z8 = bc<8>(z);  // this row's value of sample 0 / sample 1
                zs = hi ? z8 : z0;
            }
            const bool on = zs > 0.0;
            a[t][r] = isv ? (z > 0.0 ? z : 0.0) : (on ? a[t][r] : 0.0);  // std::max(0., h) of the oracle
        }
}

// NeRF input [x, sin x, cos x] (3 NIN rows, zero-padded to 32) with its Jacobian columns for the input
// directions D0..D0+CPS-2 (nerf_jac = [I; diag(cos x); diag(-sin x)], SelfCollisionModel.cpp:143-151, 177-188)
template <int NIN, int CPS = 8, int D0 = 0>
__device__ __forceinline__ void nerf_input(const double (&x)[NIN], d4 (&in)[2], int lane) {
    double sx[NIN], cx[NIN];
#pragma unroll
    for (int i = 0; i < NIN; i++) {
        sx[i] = sin(x[i]);
        cx[i] = cos(x[i]);
    }
    const int j = lane & (CPS - 1);  // 0: value column, 1 + d - D0: tangent of input d
    const int d = j - 1 + D0;
#pragma unroll
    for (int kt = 0; kt < 2; kt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int k = 16 * kt + 4 * r + (lane >> 4);
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < NIN; i++) {
                if (j == 0) {
                    if (k == i) v = x[i];
                    if (k == NIN + i) v = sx[i];
                    if (k == 2 * NIN + i) v = cx[i];
                } else if (d == i) {
                    if (k == i) v = 1.0;
                    if (k == NIN + i) v = cx[i];
                    if (k == 2 * NIN + i) v = -sx[i];
                }
            }
            in[kt][r] = v;
        }
}

// output tile: rows i < NOUT; value column -> out_i + b_i, tangent column 1 + d -> J[i][d] at the record's
// Jacobian column NBASE + d (the arm joints)
template <int NOUT>
__device__ __forceinline__ void write_out(const d4& o, const double* __restrict__ bias, int lane, int m, int M,
                                          double* __restrict__ rec, int S, int r_val, int r_jac) {
    if (m >= M) return;
    const int j = lane & 7;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int i = (lane >> 4) + 4 * r;
        if (i >= NOUT) continue;
        if (j == 0) rec[(size_t)(r_val + i) * S + m] = o[r] + bias[i];
        else rec[(size_t)(r_jac + DOF * i + NBASE + (j - 1)) * S + m] = o[r];
    }
}

// Arm-frame obstacle of the mobile manipulator (the oracle's robot_record): o_arm = Rz(th)^T (obs - [x, y, 0])
// - mount, and dO[a][b] = d o_arm[a] / d (x, y, theta)[b].  The Panda-trained env network sees the obstacle
// in the panda_link0 frame.
__device__ __forceinline__ void arm_frame_obstacle(const double* q, const double* obs, double* oa, double (&dO)[3][3]) {
    double sn, cs;
    sincos(q[2], &sn, &cs);
    const double dx = obs[0] - q[0], dy = obs[1] - q[1], dz = obs[2];
    oa[0] = (cs * dx + sn * dy) - 0.0;
    oa[1] = (-sn * dx + cs * dy) - 0.0;
    oa[2] = dz - MOBILE_MOUNT_Z;
    dO[0][0] = -cs; dO[1][0] = sn; dO[2][0] = 0.0;
    dO[0][1] = -sn; dO[1][1] = -cs; dO[2][1] = 0.0;
    dO[0][2] = -sn * dx + cs * dy; dO[1][2] = -cs * dx - sn * dy; dO[2][2] = 0.0;
}

// output tile of the mobile env network (CPS = 16, one sample per tile): value column 0, arm tangents 1..7,
// obstacle tangents 8..10.  The base columns of the record are the chain rule through the arm-frame obstacle,
// sum_a J[i][7 + a] dO[a][b] (the oracle's order), formed on lanes 11..13 of each row from DPP broadcasts.
template <int NOUT>
__device__ __forceinline__ void write_out_mobile(const d4& o, const double* __restrict__ bias, int lane, int m, int M,
                                                 double* __restrict__ rec, int S, const double (&dO)[3][3]) {
    const int j = lane & 15;
    const int bb = j - 11;  // base column of lanes 11..13
    double d0 = 0.0, d1 = 0.0, d2 = 0.0;
#pragma unroll
    for (int b = 0; b < NBASE; b++)
        if (bb == b) { d0 = dO[0][b]; d1 = dO[1][b]; d2 = dO[2][b]; }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const double j8 = bc<8>(o[r]), j9 = bc<9>(o[r]), j10 = bc<10>(o[r]);  // whole row active
        const int i = (lane >> 4) + 4 * r;
        if (m >= M || i >= NOUT) continue;
        if (j == 0) rec[(size_t)(R_ENV + i) * S + m] = o[r] + bias[i];
        else if (j <= NARM) rec[(size_t)(R_DENV + DOF * i + NBASE + (j - 1)) * S + m] = o[r];
        else if (bb >= 0 && bb < NBASE) rec[(size_t)(R_DENV + DOF * i + bb) * S + m] = j8 * d0 + j9 * d1 + j10 * d2;
    }
}

// mobile env network, obstacle pass (CPS = 4, 4 samples per tile): tangents of the 3 arm-frame obstacle coordinates
// on lanes 1..3 of each quad; the record's base columns are the chain rule sum_a J[i][7 + a] dO[a][b] (the
// oracle's order), formed on lane 1 + b from quad broadcasts.  The value and arm columns come from the arm pass.
template <int NOUT>
__device__ __forceinline__ void write_out_obs(const d4& o, int lane, int m, int M, double* __restrict__ rec, int S,
                                              const double (&dO)[3][3]) {
    const int bb = (lane & 3) - 1;  // base column of lanes 1..3 of a quad
    double d0 = 0.0, d1 = 0.0, d2 = 0.0;
#pragma unroll
    for (int b = 0; b < 3; b++)
        if (bb == b) { d0 = dO[0][b]; d1 = dO[1][b]; d2 = dO[2][b]; }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const double j7 = dpp_d<0x55>(o[r]), j8 = dpp_d<0xAA>(o[r]), j9 = dpp_d<0xFF>(o[r]);  // whole row active
        const int i = (lane >> 4) + 4 * r;
        if (m >= M || i >= NOUT || bb < 0 || bb >= NBASE) continue;
        rec[(size_t)(R_DENV + DOF * i + bb) * S + m] = j7 * d0 + j8 * d1 + j9 * d2;
    }
}

// sample m of the call: the robot's joints q (DOF) and the obstacle (x, y, z)
__device__ __forceinline__ void sample_input(const DevConst& c, const DevBuffers& d, int m, int M, const double* qin,
                                             const double* obsin, double* q /* DOF */, double* obs /* 3 */) {
    const int mm = m < M ? m : 0;
    const double* qs;
    const double* os;
    if (qin) {  // debug path: explicit q / obs lists
        qs = qin + DOF * mm;
        os = obsin + 4 * mm;
    } else {
        const int b = mm / (c.N + 1), k = mm - b * (c.N + 1);
        qs = d.guess + ((size_t)b * (c.N + 1) + k) * NXU;
        os = d.obs + 4 * b;
    }
#pragma unroll
    for (int i = 0; i < DOF; i++) q[i] = qs[i];
    obs[0] = os[0]; obs[1] = os[1]; obs[2] = os[2];
}

}  // namespace

// self network 21 -> 256 -> 64 -> 1 (osqp_interface.cpp:35-38) on the Panda joints.  The input layer's 16-row
// output tiles are consumed as they are made: tile t (after bias + ReLU gating) is k-tile t of the 256 -> 64
// layer, so the 256-wide hidden activation never exists as a whole — a fraction of the registers of the
// layer-by-layer form (336), several waves per SIMD, and the weights are read straight from L2 (the wave count
// hides their latency; no LDS, no barriers).  A wave carries SELF_CT 16-column tiles (2 samples each), so every
// weight fragment it loads feeds SELF_CT MFMAs.  Per output the same fragments in the same ascending k order:
// bitwise the layer-by-layer form.
#ifndef MPCC_SELF_CT
#define MPCC_SELF_CT 2
#endif
constexpr int SELF_CT = MPCC_SELF_CT;
#ifndef MPCC_SELF_WAVES
#define MPCC_SELF_WAVES 4  // waves per k_mlp_self block: 2, 4, or 0 = two for launches of at most ENV_SMALL samples
#endif
#ifndef MPCC_SELF_RING
#define MPCC_SELF_RING 1
#endif
constexpr int SELF_RS = 3, SELF_SLOT = 512 + 4 * 256;  // ring slots; doubles per slot (W1 row tile + W2 k-tile)
template <int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) k_mlp_self(DevConst c, DevBuffers d, NNDesc nd, const double* __restrict__ W, int M,
                                                  const double* __restrict__ qin, const double* __restrict__ obsin,
                                                  double* __restrict__ rec, int S) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * NW + (threadIdx.x >> 6);
    int m[SELF_CT];
    d4 a0[SELF_CT][2], a2[SELF_CT][4], o[SELF_CT][1];
#pragma unroll
    for (int ct = 0; ct < SELF_CT; ct++) {
        m[ct] = 2 * (SELF_CT * wave + ct) + ((lane >> 3) & 1);
        double q[DOF], obs[3];
        sample_input(c, d, m[ct], M, qin, obsin, q, obs);
        double x[7];
#pragma unroll
        for (int i = 0; i < 7; i++) x[i] = q[NBASE + i];
        nerf_input<7>(x, a0[ct], lane);
#pragma unroll
        for (int u = 0; u < 4; u++) a2[ct][u] = d4{0.0, 0.0, 0.0, 0.0};
    }
    const double* __restrict__ W1 = W + nd.offW[0];  // [16 row tiles][8 k-steps][64]
    const double* __restrict__ W2 = W + nd.offW[1];  // [4 row tiles][64 k-steps][64]
    // the biases in LDS: the epilogues read 64 of them per lane in a lane-dependent order, which as global loads
    // the allocator could only issue one at a time (one register pair free, a full wait each)
    __shared__ double sb[256 + 64 + 16];
    for (int i = threadIdx.x; i < 256; i += 64 * NW) sb[i] = W[nd.offb[0] + i];
    if (threadIdx.x < 64) sb[256 + threadIdx.x] = W[nd.offb[1] + threadIdx.x];
    if (threadIdx.x < 1) sb[320] = W[nd.offb[2]];
    __syncthreads();
#ifndef MPCC_SELF_UNROLL
#define MPCC_SELF_UNROLL 1
#endif
#if MPCC_SELF_RING
    // the weights of tile t (W1 row tile t: 8 k-steps x 64 lanes, 4 KiB; W2 k-steps 4t..4t+3 of its 4 row tiles, 8 KiB)
    // staged by the block into a 3-slot LDS ring, two tiles ahead (global_load_lds, no registers): 3 copies of 16 bytes
    // per thread per tile; the fragments are then LDS reads instead of one L2 round trip per MFMA group
    __shared__ __attribute__((aligned(16))) double ring[SELF_RS * SELF_SLOT];
    const int tid = threadIdx.x, w = tid >> 6;
    const unsigned rbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)ring;
    static_assert(12 % NW == 0, "whole 16-byte copies per thread");
    constexpr int SPT = 12 / NW;  // 16-byte copies per thread and tile (768 per slot)
    auto issue = [&](int t) {
        const unsigned slot = rbase + (unsigned)((t % SELF_RS) * SELF_SLOT * 8);
#pragma unroll
        for (int j = 0; j < SPT; j++) {
            const int e = tid + 64 * NW * j;  // 16-byte chunk of the slot: [W1 tile t: 256][W2 u = 0..3: 128 each]
            const double* src = (e < 256) ? W1 + (size_t)t * 512 + 2 * e
                                          : W2 + ((size_t)((e - 256) >> 7) * 64 + 4 * t) * 64 + 2 * ((e - 256) & 127);
            glds16_to(src, __builtin_amdgcn_readfirstlane(slot + 1024u * (NW * j + w)));
        }
    };
    issue(0);
    issue(1);
#endif
#pragma unroll MPCC_SELF_UNROLL
    for (int t = 0; t < 16; t++) {
#if MPCC_SELF_RING
        // this wave's copies of tile t have landed once at most those of tile t + 1 are outstanding; the barrier
        // publishes tile t and retires the slot of tile t - 1, which the copy of tile t + 2 overwrites
        if (t + 1 < 16) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SPT) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t + 2 < 16) issue(t + 2);
        const double* L = ring + (t % SELF_RS) * SELF_SLOT;
#endif
        d4 z[SELF_CT][1];
#pragma unroll
        for (int ct = 0; ct < SELF_CT; ct++) z[ct][0] = d4{0.0, 0.0, 0.0, 0.0};
        // k-steps 6 and 7 of the input layer hold the zero padding of the 21 NeRF rows to 32 (weights and inputs
        // both zero): skipped, an fma with two zero factors leaves the accumulator as it is
#pragma unroll
        for (int s = 0; s < 6; s++) {
#if MPCC_SELF_RING
            const double w = L[s * 64 + lane];
#else
            const double w = W1[((size_t)t * 8 + s) * 64 + lane];
#endif
#pragma unroll
            for (int ct = 0; ct < SELF_CT; ct++)
                z[ct][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(w, a0[ct][s >> 2][s & 3], z[ct][0], 0, 0, 0);
        }
#pragma unroll
        for (int ct = 0; ct < SELF_CT; ct++) relu_gate<1>(z[ct], sb + 16 * t, lane);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int u = 0; u < 4; u++) {
#if MPCC_SELF_RING
                const double w = L[512 + u * 256 + r * 64 + lane];
#else
                const double w = W2[((size_t)u * 64 + 4 * t + r) * 64 + lane];
#endif
#pragma unroll
                for (int ct = 0; ct < SELF_CT; ct++)
                    a2[ct][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(w, z[ct][0][r], a2[ct][u], 0, 0, 0);
            }
    }
#pragma unroll
    for (int ct = 0; ct < SELF_CT; ct++) {
        relu_gate<4>(a2[ct], sb + 256, lane);
        mfma_layer<4, 1>(W + nd.offW[2], a2[ct], o[ct], lane);
        write_out<1>(o[ct][0], sb + 320, lane, m[ct], M, rec, S, R_SEL, R_DSEL);
    }
}

// env network 30 -> 256 -> 256 -> 256 -> 256 -> 9 (osqp_interface.cpp:40-43).  Panda: 2 samples per wave,
// tangents of q_0..q_6.  Mobile manipulator (input directions: 7 arm joints + 3 arm-frame obstacle coordinates, the
// base columns by the chain rule): two passes, the Panda's (CPS = 8, the arm tangents, D0 = 0) and an obstacle pass
// (CPS = 4, D0 = 7: 4 samples per tile), 12 columns per sample instead of one 16-column tile with 11 used
// (MPCC_ENV_SPLIT = 0: that form, CPS = 16).  A column's MFMA chain does not depend on the other columns of its
// tile, so every output is bitwise that of the one-tile form.
// Blocks of ENV_WAVES waves around one LDS weight ring of ENV_SLOTS k-tiles (32 KiB each).  Two waves and two slots
// (72 KiB with the biases) fit on a CU beside two one-wave-per-SIMD k_sqp waves of the other controller group (40 KiB
// of LDS each); a four-wave block with three slots (104 KiB, four free SIMDs) could only start on a CU without any,
// so with two groups the env network mostly waited for the other group's QP launch to drain (round 5 trace,
// DESIGN.md §3.3).  The waves of a block share each tile's copy; the MFMAs per output are the same in any case.
// Long launches (configs[2]: 1.3M samples) run mostly without the other group's QP launch beside them, and the
// four-wave form streams half the weight bytes per sample: 214k against 212k solves/s; the two-wave form wins where
// the launch is short (the reference's default rows at configs[1]'s batch: 324k -> 367k, profiles/r05h_*).  Launches of
// at most ENV_SMALL samples take the two-wave blocks (MPCC_ENV_WAVES = 2 or 4 forces one form).
#ifndef MPCC_ENV_WAVES
#define MPCC_ENV_WAVES 0
#endif
#ifndef MPCC_ENV_CHAIN
// 1: the layers' weight k-tiles as one ring stream (mfma_layer_chain); bitwise, but slower: configs[2] 209.7k against
// 212.5-212.9k, default rows 361k against 367k (profiles/r05o_ab_env_chain_REJECTED.log)
#define MPCC_ENV_CHAIN 0
#endif
#ifndef MPCC_ENV_CHAIN_LAZY
#define MPCC_ENV_CHAIN_LAZY 0  // 1: the ReLU of a layer's input tiles inside its k-steps (spills: 208k, 331k)
#endif
constexpr int ENV_SMALL = 262144;
template <int NW>
constexpr int env_slots() { return (MPCC_MLP_PF && NW < 4) ? 2 : RING_SLOTS; }
template <int CPS, int D0 = 0, int NW = 4>
__device__ __forceinline__ void mlp_env_body(const DevConst& c, const DevBuffers& d, const NNDesc& nd, const double* __restrict__ W,
                                             int M, const double* __restrict__ qin, const double* __restrict__ obsin,
                                             double* __restrict__ rec, int S, double* wl, double* bl) {
    constexpr int ENV_SLOTS = env_slots<NW>();
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * NW + (threadIdx.x >> 6);
    const int m = (16 / CPS) * wave + (lane & 15) / CPS;
    double q[DOF], obs[3];
    sample_input(c, d, m, M, qin, obsin, q, obs);
    double x[10];
    double dO[3][3] = {};
#pragma unroll
    for (int i = 0; i < 7; i++) x[i] = q[NBASE + i];
    if constexpr (NBASE > 0) {
        double oa[3];
        arm_frame_obstacle(q, obs, oa, dO);
        x[7] = oa[0]; x[8] = oa[1]; x[9] = oa[2];
    } else {
        x[7] = obs[0]; x[8] = obs[1]; x[9] = obs[2];
    }
    // the biases in LDS (see k_mlp_self); the first ring barrier publishes them
    for (int l = 0; l < 4; l++)
        for (int i = threadIdx.x; i < 256; i += 64 * NW) bl[l * 256 + i] = W[nd.offb[l] + i];
    if (threadIdx.x < 9) bl[1024 + threadIdx.x] = W[nd.offb[4] + threadIdx.x];
    d4 a0[2], a[16], h[16], o[1];
    nerf_input<10, CPS, D0>(x, a0, lane);
#if MPCC_ENV_CHAIN
    {
        // prologue of the weight stream: the input layer's two k-tiles (stream tiles 0, 1); the barrier also
        // publishes the biases
        constexpr int CH = 16 * 256, PT = CH / 2 / (64 * NW);
        const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)wl;
        const int tid = threadIdx.x, w = tid >> 6;
        const double* W0 = W + nd.offW[0];
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int q = 0; q < PT; q++) {
                const int e = tid + 64 * NW * q;
                const int t = e >> 7;
                glds16_to(W0 + ((size_t)t * 8 + 4 * j) * 64 + 2 * (e & 127),
                          __builtin_amdgcn_readfirstlane(base + (unsigned)((j % ENV_SLOTS) * CH * 8) + 1024u * (NW * q + w)));
            }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PT) : "memory");
        __syncthreads();
        double fr[16];
#pragma unroll
        for (int t = 0; t < 16; t++) fr[t] = wl[(t * 4) * 64 + lane];
        mfma_layer_chain<2, 16, NW, ENV_SLOTS, 16, CPS>(W0, W + nd.offW[1], 0, a0, nullptr, a, fr, lane, wl);
#if MPCC_ENV_CHAIN_LAZY
        for (int l = 1; l <= 2; l++) {  // hidden layers 1 and 2 share one unrolled body; layer 3 ends the stream
            mfma_layer_chain<16, 16, NW, ENV_SLOTS, 16, CPS>(W + nd.offW[l], W + nd.offW[l + 1], 2 + 16 * (l - 1), a,
                                                             bl + 256 * (l - 1), h, fr, lane, wl);
#pragma unroll
            for (int t = 0; t < 16; t++) a[t] = h[t];
        }
        mfma_layer_chain<16, 16, NW, ENV_SLOTS, 0, CPS>(W + nd.offW[3], nullptr, 34, a, bl + 512, h, fr, lane, wl);
#else
        relu_gate<16, CPS>(a, bl, lane);
        for (int l = 1; l <= 2; l++) {
            mfma_layer_chain<16, 16, NW, ENV_SLOTS, 16, CPS>(W + nd.offW[l], W + nd.offW[l + 1], 2 + 16 * (l - 1), a,
                                                             nullptr, h, fr, lane, wl);
            relu_gate<16, CPS>(h, bl + 256 * l, lane);
#pragma unroll
            for (int t = 0; t < 16; t++) a[t] = h[t];
        }
        mfma_layer_chain<16, 16, NW, ENV_SLOTS, 0, CPS>(W + nd.offW[3], nullptr, 34, a, nullptr, h, fr, lane, wl);
#endif
        relu_gate<16, CPS>(h, bl + 768, lane);
#pragma unroll
        for (int t = 0; t < 16; t++) a[t] = h[t];
    }
#else
#if MPCC_MLP_PF
    mfma_layer_ring_pf<2, 16, NW, ENV_SLOTS>(W + nd.offW[0], a0, a, lane, wl);
#else
    mfma_layer_ring<2, 16, NW>(W + nd.offW[0], a0, a, lane, wl);
#endif
    relu_gate<16, CPS>(a, bl, lane);
    for (int l = 1; l <= 3; l++) {  // three 256 x 256 hidden layers share one unrolled body
#if MPCC_MLP_PF
        mfma_layer_ring_pf<16, 16, NW, ENV_SLOTS>(W + nd.offW[l], a, h, lane, wl);
#else
        mfma_layer_ring<16, 16, NW>(W + nd.offW[l], a, h, lane, wl);
#endif
        relu_gate<16, CPS>(h, bl + 256 * l, lane);
#pragma unroll
        for (int t = 0; t < 16; t++) a[t] = h[t];
    }
#endif
    mfma_layer<16, 1>(W + nd.offW[4], a, o, lane);
    if constexpr (CPS == 8) write_out<9>(o[0], bl + 1024, lane, m, M, rec, S, R_ENV, R_DENV);
    else if constexpr (CPS == 4) write_out_obs<9>(o[0], lane, m, M, rec, S, dO);
    else write_out_mobile<9>(o[0], bl + 1024, lane, m, M, rec, S, dO);
}

#ifndef MPCC_ENV_SPLIT
#define MPCC_ENV_SPLIT 1
#endif
constexpr bool ENV_SPLIT = MPCC_ENV_SPLIT && NBASE > 0;      // the mobile build's two passes
constexpr int ENV_CPS = (NBASE > 0 && !ENV_SPLIT) ? 16 : 8;  // columns per sample of k_mlp_env
constexpr int ENV_SPW = 16 / ENV_CPS;                        // samples per wave

template <int NW>
__global__ void __launch_bounds__(64 * NW) k_mlp_env(DevConst c, DevBuffers d, NNDesc nd, const double* __restrict__ W, int M,
                                                    const double* __restrict__ qin, const double* __restrict__ obsin,
                                                    double* __restrict__ rec, int S) {
    // no early exit: the hidden layers synchronize the block (a wave past M computes on a clamped
    // sample and write_out drops its result)
    __shared__ __attribute__((aligned(16))) double wl[env_slots<NW>() * 16 * 256];
    __shared__ double bl[4 * 256 + 16];
    mlp_env_body<ENV_CPS, 0, NW>(c, d, nd, W, M, qin, obsin, rec, S, wl, bl);
}
#if MPCC_DOF != 7
// the mobile build's obstacle pass (ENV_SPLIT)
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_mlp_env_obs(DevConst c, DevBuffers d, NNDesc nd, const double* __restrict__ W,
                                                        int M, const double* __restrict__ qin,
                                                        const double* __restrict__ obsin, double* __restrict__ rec, int S) {
    __shared__ __attribute__((aligned(16))) double wl[env_slots<NW>() * 16 * 256];
    __shared__ double bl[4 * 256 + 16];
    mlp_env_body<4, 7, NW>(c, d, nd, W, M, qin, obsin, rec, S, wl, bl);
}
#endif

void launch_nn(const DevConst& c, const DevBuffers& d, const NNDesc& nd, const double* W, int which, int M,
               const double* q, const double* obs, double* rec, int rec_stride, hipStream_t s) {
    if (M <= 0) return;
    if (which == 0) {  // NW waves x SELF_CT tiles x 2 samples
        const bool two = MPCC_SELF_WAVES == 2 || (MPCC_SELF_WAVES == 0 && M <= ENV_SMALL);
        auto go = [&](auto nwc) {
            constexpr int NW = decltype(nwc)::value;
            hipLaunchKernelGGL(k_mlp_self<NW>, dim3((M + 2 * NW * SELF_CT - 1) / (2 * NW * SELF_CT)), dim3(64 * NW), 0, s, c,
                               d, nd, W, M, q, obs, rec, rec_stride);
        };
        if (two) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 4>{});
    } else {
        const bool two = MPCC_ENV_WAVES == 2 || (MPCC_ENV_WAVES == 0 && M <= ENV_SMALL);
        auto go = [&](auto nwc) {
            constexpr int NW = decltype(nwc)::value;
            hipLaunchKernelGGL(k_mlp_env<NW>, dim3((M + NW * ENV_SPW - 1) / (NW * ENV_SPW)), dim3(64 * NW), 0, s, c, d, nd, W,
                               M, q, obs, rec, rec_stride);
#if MPCC_DOF != 7
            if constexpr (ENV_SPLIT)  // NW waves x 4 samples
                hipLaunchKernelGGL(k_mlp_env_obs<NW>, dim3((M + 4 * NW - 1) / (4 * NW)), dim3(64 * NW), 0, s, c, d, nd, W, M, q,
                                   obs, rec, rec_stride);
#endif
        };
        if (MPCC_ENV_WAVES == 1) go(std::integral_constant<int, 1>{});  // A/B only: 243k against 377k at the default rows
        else if (two) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 4>{});
    }
}

}  // namespace mpcc
