// MFMA operand helpers shared by the GEMM-shaped kernels (gfx950).
#pragma once

#include "common.hpp"

namespace cai {

template <typename T> struct OpT;
template <> struct OpT<bf16> { static constexpr int VEC = 8; };
template <> struct OpT<float> { static constexpr int VEC = 4; };

template <typename T>
using gptr = const T __attribute__((address_space(1)))*;
template <typename T>
__device__ __forceinline__ gptr<T> to_global(const void* p) {
    return (gptr<T>)(reinterpret_cast<uintptr_t>(p));
}

__device__ __forceinline__ u32x4 abs_chunk(u32x4 v, int elem_bytes) {
    const unsigned m = elem_bytes == 2 ? 0x7FFF7FFFu : 0x7FFFFFFFu;
    v.x &= m; v.y &= m; v.z &= m; v.w &= m;
    return v;
}

template <typename T>
__device__ __forceinline__ u32x4 sq_chunk(u32x4 v);
template <> __device__ __forceinline__ u32x4 sq_chunk<bf16>(u32x4 v) {
    bf16x8 h = __builtin_bit_cast(bf16x8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float f = (float)h[e];
        h[e] = (bf16)(f * f);
    }
    return __builtin_bit_cast(u32x4, h);
}
template <> __device__ __forceinline__ u32x4 sq_chunk<float>(u32x4 v) {
    f32x4 h = __builtin_bit_cast(f32x4, v);
    h = h * h;
    return __builtin_bit_cast(u32x4, h);
}

template <typename T>
__device__ __forceinline__ f32x4 mma16(u32x4 a, u32x4 b, f32x4 c);
template <> __device__ __forceinline__ f32x4 mma16<bf16>(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                   0, 0);
}
template <> __device__ __forceinline__ f32x4 mma16<float>(u32x4 a, u32x4 b, f32x4 c) {
    // the four k-values of a 16-byte slot go to four MFMAs; A and B use the
    // same permutation of k so the sum is unchanged
    const f32x4 av = __builtin_bit_cast(f32x4, a), bv = __builtin_bit_cast(f32x4, b);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], c, 0, 0, 0);
    return c;
}

}  // namespace cai
