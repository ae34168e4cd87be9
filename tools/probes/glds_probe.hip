// Probe: where does global_load_lds_dwordx4 with an immediate offset write in LDS?  (M0 = 0; offset 256)
// Prints which LDS byte offset holds the first 16 bytes of src + 256.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const double* src, double* out) {
    __shared__ double lds[512];
    for (int i = threadIdx.x; i < 512; i += 64) lds[i] = -1.0;
    __syncthreads();
    const char* p = (const char*)src + threadIdx.x * 16;
    unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)lds, keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off offset:256\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(p), "s"(base) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}
int main() {
    double h[1024], *s, *o, r[512];
    for (int i = 0; i < 1024; i++) h[i] = i;
    hipMalloc(&s, sizeof h); hipMalloc(&o, sizeof r);
    hipMemcpy(s, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 64>>>(s, o);
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    int first = -1;
    for (int i = 0; i < 512; i++) if (r[i] >= 0) { first = i; break; }
    printf("first written LDS double %d holds src double %g (offset applied to LDS: %s)\n", first, first >= 0 ? r[first] : -1,
           first == 32 ? "yes" : (first == 0 ? "no" : "?"));
    return 0;
}
