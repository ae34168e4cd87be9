// permlane_probe.hip — checks the v_permlane16_swap semantics ipm_wide.hip's 32-lane exchange relies on:
// with both operands v, result[0] = v's even 16-lane row duplicated over the row pair, result[1] = the odd row.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
    const unsigned v = threadIdx.x;
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    out[threadIdx.x] = r[0];
    out[64 + threadIdx.x] = r[1];
}
int main() {
    unsigned* d;
    unsigned h[128];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int l = 0; l < 64; l++) {
        const unsigned pair = l / 32, col = l % 16;
        const unsigned lo = 32 * pair + col, hi = 32 * pair + 16 + col;
        if (h[l] != lo || h[64 + l] != hi) bad++;
    }
    for (int l = 0; l < 64; l++) printf("%u/%u%c", h[l], h[64 + l], l % 16 == 15 ? '\n' : ' ');
    printf("permlane16_swap probe: %s\n", bad ? "MISMATCH" : "ok");
    (void)hipFree(d);
    return bad ? 1 : 0;
}
