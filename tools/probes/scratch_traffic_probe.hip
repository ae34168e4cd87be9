// scratch_traffic_probe.hip — does rocprofv3's FETCH_SIZE need the x2 correction for scratch (spill) traffic?
// (the MI355X guide calibrates the x2 only for 16-byte-per-lane streaming reads.)
//
// Two kernels with a known byte count, each far past the 256 MiB Infinity Cache so that the bytes reach HBM:
//   k_stream8   global_load_dwordx2 streaming read, 8 bytes per lane (the width of a spill reload), 1 GiB
//   k_scratch   a per-lane private array of NP doubles indexed by a runtime value (so it lives in scratch): written
//               once (NP x 8 B per lane), then read R times in a wave-uniform, data-dependent order — the access
//               pattern of the IPM's spill reloads (scratch_load_dwordx2 at one offset for the whole wave)
// Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE in a separate pass); the program prints the algorithmic
// bytes of each dispatch for the comparison (tools/probes/scratch_traffic_summary.py).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NP = 512;  // private doubles per lane: 4 KiB per lane, 256 KiB per wave

__global__ void __launch_bounds__(64) k_stream8(const double* __restrict__ src, double* __restrict__ out, long n) {
    double acc = 0.0;
    for (long i = (long)blockIdx.x * 64 + threadIdx.x; i < n; i += (long)gridDim.x * 64) acc += src[i];
    out[(long)blockIdx.x * 64 + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(64) k_scratch(int R, int seed, double* __restrict__ out) {
    double buf[NP];
    const int lane = threadIdx.x;
#pragma unroll 1
    for (int i = 0; i < NP; i++) buf[(i * 5 + seed) & (NP - 1)] = (double)(i + lane);
    double acc = 0.0;
#pragma unroll 1
    for (int r = 0; r < R; r++)
#pragma unroll 1
        for (int i = 0; i < NP; i++) acc += buf[(i * 7 + r + seed) & (NP - 1)];
    out[(long)blockIdx.x * 64 + lane] = acc;
}

int main() {
    const long n = 1L << 27;  // 1 GiB of doubles
    double *src, *out;
    CHECK(hipMalloc(&src, n * sizeof(double)));
    CHECK(hipMemset(src, 0, n * sizeof(double)));
    const int blocks = 16384;
    CHECK(hipMalloc(&out, (long)blocks * 64 * sizeof(double)));
    hipLaunchKernelGGL(k_stream8, dim3(blocks), dim3(64), 0, 0, src, out, n);
    CHECK(hipDeviceSynchronize());
    printf("{\"kernel\": \"k_stream8\", \"read_bytes\": %ld, \"write_bytes\": %ld}\n", n * 8, (long)blocks * 64 * 8);
    const int R = 4, sb = 4096;  // 4096 waves x 256 KiB = 1 GiB of scratch
    hipLaunchKernelGGL(k_scratch, dim3(sb), dim3(64), 0, 0, R, 3, out);
    CHECK(hipDeviceSynchronize());
    const long lanes = (long)sb * 64;
    printf("{\"kernel\": \"k_scratch\", \"read_bytes\": %ld, \"write_bytes\": %ld, \"scratch_read_bytes\": %ld, "
           "\"scratch_write_bytes\": %ld}\n", lanes * NP * 8 * R, lanes * NP * 8 + lanes * 8, lanes * NP * 8 * R, lanes * NP * 8);
    CHECK(hipFree(src));
    CHECK(hipFree(out));
    return 0;
}
