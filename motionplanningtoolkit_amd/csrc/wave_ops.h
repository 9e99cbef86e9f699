// wave_ops.h -- whole-wave reductions from DPP row operations and the gfx950 permlane swaps:
// no LDS round trip (ds_bpermute, what __shfl_xor compiles to, waits on the LDS pipe at every
// level), every level a VALU exchange plus the operation.  For uniform control flow with every
// lane of the wave active.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpt {

// the value of the lane in the other half of this lane's 2L-lane block (after the levels below
// L every lane of a block holds the block's value, so a mirror is as good as an xor)
template <int L>
__device__ __forceinline__ uint32_t wave_xchg(uint32_t v) {
    if constexpr (L == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
    else if constexpr (L == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, true);  // quad_perm [2,3,0,1]
    else if constexpr (L == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, true);  // row_half_mirror
    else if constexpr (L == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, true);  // row_mirror
    else if constexpr (L == 16) {  // rows 0 <-> 1, 2 <-> 3
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (threadIdx.x & 16) ? r[0] : r[1];
    } else {  // lanes 0..31 <-> 32..63
        static_assert(L == 32, "wave_xchg level");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
}

template <class Op>
__device__ __forceinline__ float wave_reduce_f32(float v, Op op) {
    v = op(v, __uint_as_float(wave_xchg<1>(__float_as_uint(v))));
    v = op(v, __uint_as_float(wave_xchg<2>(__float_as_uint(v))));
    v = op(v, __uint_as_float(wave_xchg<4>(__float_as_uint(v))));
    v = op(v, __uint_as_float(wave_xchg<8>(__float_as_uint(v))));
    v = op(v, __uint_as_float(wave_xchg<16>(__float_as_uint(v))));
    v = op(v, __uint_as_float(wave_xchg<32>(__float_as_uint(v))));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// the least / greatest float of the wave, uniform
__device__ __forceinline__ float wave_min_dpp(float v) {
    return wave_reduce_f32(v, [](float a, float b) { return fminf(a, b); });
}
__device__ __forceinline__ float wave_max_dpp(float v) {
    return wave_reduce_f32(v, [](float a, float b) { return fmaxf(a, b); });
}

template <int L>
__device__ __forceinline__ double wave_xchg_f64(double x) {
    const uint32_t lo = (uint32_t)__double2loint(x), hi = (uint32_t)__double2hiint(x);
    return __hiloint2double((int)wave_xchg<L>(hi), (int)wave_xchg<L>(lo));
}

template <class Op>
__device__ __forceinline__ double wave_reduce_f64(double v, Op op) {
    v = op(v, wave_xchg_f64<1>(v));
    v = op(v, wave_xchg_f64<2>(v));
    v = op(v, wave_xchg_f64<4>(v));
    v = op(v, wave_xchg_f64<8>(v));
    v = op(v, wave_xchg_f64<16>(v));
    v = op(v, wave_xchg_f64<32>(v));
    return v;  // the same in every lane
}
__device__ __forceinline__ double wave_min_f64_dpp(double v) {
    return wave_reduce_f64(v, [](double a, double b) { return fmin(a, b); });
}
__device__ __forceinline__ double wave_max_f64_dpp(double v) {
    return wave_reduce_f64(v, [](double a, double b) { return fmax(a, b); });
}

// (v, idx) of the least v, ties to the least idx, in every lane
template <int L>
__device__ __forceinline__ void argmin_level(float &v, int &idx) {
    const float ov = __uint_as_float(wave_xchg<L>(__float_as_uint(v)));
    const int oi = (int)wave_xchg<L>((uint32_t)idx);
    const bool t = ov < v || (ov == v && oi < idx);
    v = t ? ov : v;
    idx = t ? oi : idx;
}
__device__ __forceinline__ void wave_argmin_f32_dpp(float &v, int &idx) {
    argmin_level<1>(v, idx);
    argmin_level<2>(v, idx);
    argmin_level<4>(v, idx);
    argmin_level<8>(v, idx);
    argmin_level<16>(v, idx);
    argmin_level<32>(v, idx);
}

}  // namespace mpt
