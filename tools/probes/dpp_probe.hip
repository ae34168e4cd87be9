// DPP semantics probe on gfx950: row_shl / row_shr / row_ror / row_newbcast on 16-lane rows.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int C> __device__ int dpp(int v) { return __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, true); }
__global__ void k(int* o) {
    int l = threadIdx.x;
    int v = 100 + l;
    o[0 * 64 + l] = dpp<0x101>(v);  // row_shl:1
    o[1 * 64 + l] = dpp<0x119>(v);  // row_shr:9
    o[2 * 64 + l] = dpp<0x153>(v);  // row_newbcast:3
    o[3 * 64 + l] = dpp<0x15F>(v);  // row_newbcast:15
    o[4 * 64 + l] = dpp<0x128>(v);  // row_ror:8
}
int main() {
    int* d; hipMalloc(&d, 5 * 64 * sizeof(int));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[320]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char* nm[5] = {"row_shl:1", "row_shr:9", "row_newbcast:3", "row_newbcast:15", "row_ror:8"};
    for (int r = 0; r < 5; r++) { printf("%-16s", nm[r]); for (int l = 0; l < 32; l++) printf(" %d", h[r * 64 + l]); printf("\n"); }
    return 0;
}
