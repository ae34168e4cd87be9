// mfma_f64_probe.hip — is v_mfma_f64_16x16x4_f64 bitwise a sequential fma chain over k?
// C[16x16] = A[16xK] B[Kx16] by K/4 MFMA k-steps; compared with CPU fma chains in several orders.
// Operand maps (cdna_hip_programming.md §3): A lane l -> A[l&15][4s + (l>>4)], B lane l -> B[4s + (l>>4)][l&15],
// C lane l reg r -> C[(l>>4) + 4r][l&15].
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_probe(const double* A, const double* B, double* C, int K) {
    const int l = threadIdx.x;
    d4 acc = {0, 0, 0, 0};
    for (int s = 0; s < K / 4; s++) {
        const double a = A[(l & 15) * K + 4 * s + (l >> 4)];
        const double b = B[(4 * s + (l >> 4)) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; r++) C[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

int main() {
    const int K = 256;
    std::mt19937_64 g(7);
    std::normal_distribution<double> nd(0.0, 1.0);
    double *A = new double[16 * K], *B = new double[K * 16], *C = new double[256];
    for (int i = 0; i < 16 * K; i++) A[i] = nd(g) * std::exp(nd(g));
    for (int i = 0; i < K * 16; i++) B[i] = nd(g) * std::exp(nd(g));
    double *dA, *dB, *dC;
    hipMalloc(&dA, 16 * K * 8); hipMalloc(&dB, K * 16 * 8); hipMalloc(&dC, 256 * 8);
    hipMemcpy(dA, A, 16 * K * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, K * 16 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, K);
    hipMemcpy(C, dC, 256 * 8, hipMemcpyDeviceToHost);
    int eq_chain = 0, eq_unfused = 0, eq_rev = 0, eq_pair = 0;
    double maxrel = 0;
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) {
            double c1 = 0, c2 = 0, c3 = 0, c4 = 0;
            for (int k = 0; k < K; k++) c1 = std::fma(A[i * K + k], B[k * 16 + j], c1);        // ascending fma chain
            for (int k = 0; k < K; k++) c2 = c2 + A[i * K + k] * B[k * 16 + j];                 // unfused
            for (int s = 0; s < K / 4; s++)                                                        // fma chain, k descending in step
                for (int q = 3; q >= 0; q--) c3 = std::fma(A[i * K + 4 * s + q], B[(4 * s + q) * 16 + j], c3);
            for (int s = 0; s < K / 4; s++) {                                                      // exact 4-term sum, one rounding
                long double t = c4;
                for (int q = 0; q < 4; q++) t += (long double)A[i * K + 4 * s + q] * B[(4 * s + q) * 16 + j];
                c4 = (double)t;
            }
            const double c = C[i * 16 + j];
            eq_chain += (c == c1); eq_unfused += (c == c2); eq_rev += (c == c3); eq_pair += (c == c4);
            maxrel = std::fmax(maxrel, std::fabs(c - c1) / std::fabs(c1));
        }
    std::printf("of 256: fma-chain-asc %d  unfused %d  fma-chain-desc-in-step %d  one-rounding-per-step %d  maxrel-vs-chain %.3e\n",
                eq_chain, eq_unfused, eq_rev, eq_pair, maxrel);
    return 0;
}
