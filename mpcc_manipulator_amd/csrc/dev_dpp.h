// dev_dpp.h — 16-lane DPP row primitives shared by the register-resident kernels (k_ipm, k_mlp).
#pragma once
#include <hip/hip_runtime.h>

namespace mpcc {
namespace dpp {

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    // One 64-bit DPP move: gfx950 executes row_newbcast on 64-bit operands as a single v_mov_b64_dpp
    // (the DP-ALU DPP form); the other row controls are split into two v_mov_b32_dpp by the backend.
    long long x = __builtin_amdgcn_update_dpp(0LL, (long long)__double_as_longlong(v), CTRL, 0xF, 0xF, true);
    // Pin the DPP where it is written: the optimizer may otherwise sink it into a lane-divergent branch
    // of its only consumer (e.g. the t >= 9 side of a select), where the source lanes are masked off
    // and read as 0.  An empty volatile asm on the result cannot be moved across control flow.
    asm volatile("" : "+v"(x));
    return __longlong_as_double(x);
}
template <int n> __device__ __forceinline__ double from_up(double v) { return dpp_d<0x100 + n>(v); }    // row_shl: lane t <- t+n
template <int n> __device__ __forceinline__ double from_down(double v) { return dpp_d<0x110 + n>(v); } // row_shr: lane t <- t-n
template <int n> __device__ __forceinline__ double rot16(double v) { return dpp_d<0x120 + n>(v); }     // row_ror
template <int n> __device__ __forceinline__ double bc(double v) { return dpp_d<0x150 + n>(v); }        // row_newbcast: lane n
__device__ __forceinline__ double half_mirror(double v) { return dpp_d<0x141>(v); }  // lane j <- 7 - j in each 8-lane half
__device__ __forceinline__ double quad_swap2(double v) { return dpp_d<0x4E>(v); }   // quad_perm [2,3,0,1]: lane j <- j ^ 2
__device__ __forceinline__ double quad_swap1(double v) { return dpp_d<0xB1>(v); }   // quad_perm [1,0,3,2]: lane j <- j ^ 1
// lane n of the row for an n that is a constant after unrolling
__device__ __forceinline__ double bcn(double v, int n) {
    switch (n) {
        case 0: return bc<0>(v);   case 1: return bc<1>(v);   case 2: return bc<2>(v);   case 3: return bc<3>(v);
        case 4: return bc<4>(v);   case 5: return bc<5>(v);   case 6: return bc<6>(v);   case 7: return bc<7>(v);
        case 8: return bc<8>(v);   case 9: return bc<9>(v);   case 10: return bc<10>(v); case 11: return bc<11>(v);
        case 12: return bc<12>(v); case 13: return bc<13>(v); case 14: return bc<14>(v); default: return bc<15>(v);
    }
}
__device__ __forceinline__ double g_sum(double v) {
    v += rot16<8>(v); v += rot16<4>(v); v += rot16<2>(v); v += rot16<1>(v);
    return v;
}
__device__ __forceinline__ double g_max(double v) {
    v = fmax(v, rot16<8>(v)); v = fmax(v, rot16<4>(v)); v = fmax(v, rot16<2>(v)); v = fmax(v, rot16<1>(v));
    return v;
}
__device__ __forceinline__ double g_min(double v) {
    v = fmin(v, rot16<8>(v)); v = fmin(v, rot16<4>(v)); v = fmin(v, rot16<2>(v)); v = fmin(v, rot16<1>(v));
    return v;
}

// NOTE: every DPP read must execute with the whole 16-lane row active — a lane reading from a lane that
// is masked off at that instruction gets 0.  Shifts/broadcasts are therefore evaluated unconditionally
// and consumed through selects.

}  // namespace dpp
}  // namespace mpcc
