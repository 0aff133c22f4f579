// Shared helpers for the libcai HIP sources (gfx950 / CDNA4 only).
#pragma once
#include <type_traits>

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "cai.h"

namespace cai {

// ---------------------------------------------------------------------------
// error handling: thread-local message, no global mutable state
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);

#define CAI_CHECK_ARG(cond, ...)            \
    do {                                    \
        if (!(cond)) {                      \
            ::cai::set_error(__VA_ARGS__);  \
            return CAI_EINVAL;              \
        }                                   \
    } while (0)

#define CAI_LAUNCH_CHECK(what)                                                          \
    do {                                                                                \
        hipError_t e_ = hipGetLastError();                                              \
        if (e_ != hipSuccess) {                                                         \
            ::cai::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));     \
            return CAI_EDEVICE;                                                         \
        }                                                                               \
    } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------------------
// vector types
// ---------------------------------------------------------------------------
typedef __bf16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
// native 16-byte vector (HIP's uint4 is a struct: selects on it lower through scratch)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

// generic scalar load/store by runtime dtype code
__device__ __forceinline__ float ld_any(const void* p, int dtype, int64_t i) {
    return dtype == CAI_BF16 ? (float)reinterpret_cast<const bf16*>(p)[i] : reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void st_any(void* p, int dtype, int64_t i, float v) {
    if (dtype == CAI_BF16)
        reinterpret_cast<bf16*>(p)[i] = (bf16)v;
    else
        reinterpret_cast<float*>(p)[i] = v;
}

static inline int dtype_size(int dtype) { return dtype == CAI_BF16 ? 2 : 4; }

// ---------------------------------------------------------------------------
// wave / block reductions (wave = 64 lanes)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// Sum over the 64 lanes on the VALU (no LDS): DPP butterflies inside each 16-lane row, then the four row
// sums read into scalars and added in a fixed order.  The result is wave-uniform and deterministic.
__device__ __forceinline__ float wave_sum_dpp(float v) {
    auto dpp = [](float x, auto ctrl) {
        return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), decltype(ctrl)::value,
                                                                      0xF, 0xF, false));
    };
    v += dpp(v, std::integral_constant<int, 0xB1>{});    // quad_perm [1,0,3,2]
    v += dpp(v, std::integral_constant<int, 0x4E>{});    // quad_perm [2,3,0,1]
    v += dpp(v, std::integral_constant<int, 0x124>{});   // row_ror:4
    v += dpp(v, std::integral_constant<int, 0x128>{});   // row_ror:8
    const int b = __builtin_bit_cast(int, v);
    const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0));
    const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16));
    const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32));
    const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
    return (r0 + r1) + (r2 + r3);
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block of NT threads -> value valid in thread 0
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* smem) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) smem[w] = v;
    __syncthreads();
    float r = 0.f;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) r += smem[i];
    }
    __syncthreads();
    return r;
}

// the same sum in every thread (each adds the wave partials in thread 0's order: the same float)
template <int NT>
__device__ __forceinline__ float block_sum_all(float v, float* smem) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) smem[w] = v;
    __syncthreads();
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) r += smem[i];
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------------------
// counted waits as compiler builtins (gfx9 s_waitcnt encoding: vmcnt[3:0] + [15:14], expcnt[6:4],
// lgkmcnt[11:8]).  Unlike inline asm these are visible to the waitcnt pass, which otherwise falls
// back to lgkmcnt(0) before every later LDS-fragment use.
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}
__device__ __forceinline__ void wait_lgkmcnt0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
__device__ __forceinline__ void wait_vmcnt_n(int n) {    // n folds to a constant after unrolling
    switch (n) {
        case 0: wait_vmcnt<0>(); break;
        case 1: wait_vmcnt<1>(); break;
        case 2: wait_vmcnt<2>(); break;
        case 3: wait_vmcnt<3>(); break;
        case 4: wait_vmcnt<4>(); break;
        case 5: wait_vmcnt<5>(); break;
        case 6: wait_vmcnt<6>(); break;
        case 7: wait_vmcnt<7>(); break;
        case 8: wait_vmcnt<8>(); break;
        case 9: wait_vmcnt<9>(); break;
        case 10: wait_vmcnt<10>(); break;
        case 11: wait_vmcnt<11>(); break;
        case 12: wait_vmcnt<12>(); break;
        case 13: wait_vmcnt<13>(); break;
        case 14: wait_vmcnt<14>(); break;
        case 15: wait_vmcnt<15>(); break;
        case 16: wait_vmcnt<16>(); break;
        case 17: wait_vmcnt<17>(); break;
        case 18: wait_vmcnt<18>(); break;
        case 19: wait_vmcnt<19>(); break;
        case 20: wait_vmcnt<20>(); break;
        case 21: wait_vmcnt<21>(); break;
        case 22: wait_vmcnt<22>(); break;
        case 23: wait_vmcnt<23>(); break;
        default: wait_vmcnt<24>(); break;
    }
}

// The LDS DMA (global_load_lds_dwordx4) issued from inline asm.  The waitcnt pass books the builtin
// (__builtin_amdgcn_global_load_lds) as an LDS write of unknown order: with one in flight every later fragment
// read waits for lgkmcnt(0) and vmcnt(0) -- every DMA, prefetches included (the weight-gradient kernels measured
// 97 -> 81 us once their DMAs moved here).  Issued from asm it is invisible; every ring counts its DMAs with
// explicit vmcnt waits.  M0 carries the wave's LDS base and is restored after the DMA (the compiler reserves it).
__device__ __forceinline__ void glds16_asm(const void* g, const char* lds_wave_base) {
    const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds_wave_base));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}


}  // namespace cai
