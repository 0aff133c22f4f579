// Convolution / transposed convolution as implicit GEMM on CDNA4 MFMA.
//
// Replaces the nn.Conv2d / nn.ConvTranspose2d modules built by
// compressai/models/utils.py:128-146 (conv k5 s2 p2, deconv k5 s2 p2 op1,
// conv k3 s1 p1) and the 1x1 / masked 5x5 convs of google.py:467-478.
//
// One kernel family, two row-addressing modes:
//   gather  : out[b,j,i]  = sum_{kh,kw,c} in[b, j*s-p+kh, i*s-p+kw, c] * W[n,kh,kw,c]
//             (Conv2d forward, ConvTranspose2d input-gradient)
//   phase   : the transposed (adjoint) op, decomposed by output phase
//             (py,px) = (oy mod s, ox mod s) so every output row of a phase
//             has the same tap list: taps kh = kh0 + s*a, input row
//             iy = j + dy0 - a.  (Conv2d input-gradient, ConvTranspose2d forward)
// Operands: activations pixel-major (NHWC) bf16 or fp32, weights pre-packed
// per phase as [n][tap][c] rows (K contiguous).  A tile = BM output pixels x
// 128 bytes of K, B tile = BN output channels x 128 bytes of K, both staged
// global -> registers -> LDS (XOR-swizzled 16-byte slots, double buffered,
// one barrier per K-tile).  MFMA: v_mfma_f32_16x16x32_bf16, or four
// v_mfma_f32_16x16x4_f32 per 16-byte slot for the exact-fp32 parity path.
// Epilogue: bias + ReLU/LeakyReLU or a gradient mask from an aux tensor,
// staged through LDS as fp32 and stored 16 bytes per lane.
//
// wgrad: dW[n][tap][q] = sum_m G[m][n] * X[pix(m,tap)][q] with the pixel
// dimension as K, split over workgroups (fp32 partial slabs + a fixed-order
// reduce: deterministic).  Both operands arrive [pixel][channel]; bf16 MFMA
// fragments are read with ds_read_b64_tr_b16 (hardware transpose).
#include "common.hpp"

#include <type_traits>
#include "edge_frag.hpp"
#include "mfma.hpp"
#include "reduce_jobs.hpp"
#include "conv_args.hpp"

#include <algorithm>
#include <vector>

namespace cai {

constexpr int NT = 256;


__device__ __forceinline__ int swz(int row, int slot) { return slot ^ ((row >> 1) & 7); }

__device__ __forceinline__ float apply_act(float v, int act, float prm) {
    if (act == CAI_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == CAI_ACT_LEAKY) return v > 0.f ? v : v * prm;
    return v;
}
// the activation as the epilogue applies it before the store: deferred to the store when a residual is added
// first (store_out_chunk / store_out_scalar add res, then activate)
__device__ __forceinline__ float act_pre(const ConvArgs& a, float v) {
    return a.res ? v : apply_act(v, a.act, a.act_param);
}
__device__ __forceinline__ float mask_val(int mode, float a, float prm) {
    if (mode == CAI_MASK_POS) return a > 0.f ? 1.f : 0.f;
    if (mode == CAI_MASK_LEAKY) return a > 0.f ? 1.f : prm;
    if (mode == CAI_MASK_SIGN) return a > 0.f ? 1.f : (a < 0.f ? -1.f : 0.f);
    return 1.f;
}

template <int BM_, int BN_, int WM_, int WN_>
struct Cfg {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
};

template <typename T, typename C>
struct ConvSmem {
    static constexpr int PIPE = 2 * (C::BM + C::BN) * 128;
    static constexpr int EPI_STRIDE = C::BN + 4;
    static constexpr int EPI = C::BM * EPI_STRIDE * 4;
    static constexpr int BYTES = PIPE > EPI ? PIPE : EPI;
};

template <int N>
struct U4 {
    u32x4 v[N];
};

// output-mapping helpers shared by the fused epilogue and the split-K reduce
template <typename T>
__device__ __forceinline__ void out_pixel(const ConvArgs& a, const PhaseDesc& P, int plane, int m, int& b, int& oy,
                                          int& ox) {
    b = m / plane;
    const int r = m - b * plane;
    const int j = r / P.OWg;
    oy = P.oy0 + a.out_step * j;
    ox = P.ox0 + a.out_step * (r - j * P.OWg);
}

// EXTRA = false: the caller has checked that there is no residual and no mask (no loads at all: a load here sits
// behind the earlier iterations' stores on the shared vmcnt, and its wait serialized a whole epilogue's stores --
// 38 % of the phase kernel's block time).  POST = false: a.res_post is not supported (the halo kernels: its
// registers spill their main loops; the host rejects it there)
template <typename T, bool EXTRA = true, bool POST = true>
__device__ __forceinline__ void store_out_chunk(const ConvArgs& a, const PhaseDesc& P, int plane, int m, int n,
                                                float (&v)[8], int VO) {
    int b, oy, ox;
    out_pixel<T>(a, P, plane, m, b, oy, ox);
    auto mask = [&]() {
        const T* AUX = reinterpret_cast<const T*>(a.aux);
        const int64_t pa = (((int64_t)b * a.out_h + oy) * a.out_w + ox) * a.aux_ld + n;
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (e < VO) v[e] *= mask_val(a.mask_mode, to_f32(AUX[pa + e]), a.mask_param);
    };
    if (EXTRA && POST && a.mask_mode && a.res_post) mask();
    if (EXTRA && a.res) {
        const int64_t px = ((int64_t)b * a.out_h + oy) * a.out_w + ox;
        const bf16* R = a.res + px * a.res_ld + n;
        const bf16* R2 = a.res2 ? a.res2 + px * a.res2_ld + n : nullptr;
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (e < VO) v[e] = apply_act(v[e] + (float)R[e] + (R2 ? (float)R2[e] : 0.f), a.act, a.act_param);
    }
    if (EXTRA && a.mask_mode && !(POST && a.res_post)) mask();
    const int64_t off = (int64_t)b * a.ysb + (int64_t)oy * a.ysy + (int64_t)ox * a.ysx + n;
    if (a.y_dtype == CAI_BF16) {
        bf16x8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
        *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.y) + off) = h;
    } else {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.y) + off) = f32x4{v[0], v[1], v[2], v[3]};
    }
}

template <typename T, bool POST = true>
__device__ __forceinline__ void store_out_scalar(const ConvArgs& a, const PhaseDesc& P, int plane, int m, int n,
                                                 float v) {
    int b, oy, ox;
    out_pixel<T>(a, P, plane, m, b, oy, ox);
    const float mk = a.mask_mode ? mask_val(a.mask_mode, to_f32(reinterpret_cast<const T*>(a.aux)[
                                                 (((int64_t)b * a.out_h + oy) * a.out_w + ox) * a.aux_ld + n]),
                                             a.mask_param)
                                 : 1.f;
    if (POST && a.res_post) v *= mk;
    if (a.res) {
        const int64_t px = ((int64_t)b * a.out_h + oy) * a.out_w + ox;
        v += (float)a.res[px * a.res_ld + n];
        if (a.res2) v += (float)a.res2[px * a.res2_ld + n];
        v = apply_act(v, a.act, a.act_param);
    }
    if (!(POST && a.res_post)) v *= mk;
    st_any(a.y, a.y_dtype, (int64_t)b * a.ysb + (int64_t)n * a.ysc + (int64_t)oy * a.ysy + (int64_t)ox * a.ysx, v);
}

// Epilogue shared by the conv kernels: the wave accumulators go through LDS as
// fp32 [BM][BN+4]; split-K writes the raw partial tile to ws[z][m][n] (bias /
// act / mask applied by the reduce), otherwise bias + act (+ mask) and 16-byte
// stores.  `E` must hold BM*(BN+4) floats and may alias the operand stages.
// rowm(row): the GEMM row m of tile row `row`, or -1 outside the phase
// slab: the split-K partial slab this block writes (-1: blockIdx.z, the phase * ksplit + split of the
// phase-major grids)
template <typename T, int BM, int BN, int WM, int WN, int NTH, class RowMap, bool POST = true>
__device__ __forceinline__ void conv_epilogue_rows(const ConvArgs& a, const PhaseDesc& P, int plane, int n0, float* E,
                                                   const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], RowMap rowm,
                                                   int slab = -1) {
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int ES = BN + 4;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    if (a.ksplit > 1) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = wn * WTN + tn * 16 + (lane & 15);
#pragma unroll
                for (int r = 0; r < 4; ++r) E[(wm * WTM + tm * 16 + (lane >> 4) * 4 + r) * ES + col] = acc[tm][tn][r];
            }
        __syncthreads();
        const int sb = slab >= 0 ? slab : (int)blockIdx.z;
        float* dst = a.ws + (int64_t)sb * a.ws_rows * a.ws_ld;
        constexpr int cpr = BN / 4;
        for (int id = tid; id < BM * cpr; id += NTH) {
            const int row = id / cpr, cc = id - (id / cpr) * cpr;
            const int m = rowm(row), n = n0 + cc * 4;
            if (m < 0 || n >= a.ws_ld) continue;
            *reinterpret_cast<f32x4*>(dst + (int64_t)m * a.ws_ld + n) =
                *reinterpret_cast<const f32x4*>(E + row * ES + cc * 4);
        }
        return;
    }
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = wn * WTN + tn * 16 + (lane & 15);
            const int n = n0 + col;
            const float bv = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = wm * WTM + tm * 16 + (lane >> 4) * 4 + r;
                E[row * ES + col] = act_pre(a, acc[tm][tn][r] + bv);
            }
        }
    __syncthreads();
    if (a.y_vec) {
        const int VO = a.y_dtype == CAI_BF16 ? 8 : 4;
        const int cpr = BN / VO;
        auto run = [&](auto extra) {
            for (int id = tid; id < BM * cpr; id += NTH) {
                const int row = id / cpr, cc = id - (id / cpr) * cpr;
                const int m = rowm(row), n = n0 + cc * VO;
                if (m < 0 || n >= a.Cout) continue;
                float v[8];
                const f32x4 lo = *reinterpret_cast<const f32x4*>(E + row * ES + cc * VO);
                f32x4 hi = f32x4{0.f, 0.f, 0.f, 0.f};
                if (VO == 8) hi = *reinterpret_cast<const f32x4*>(E + row * ES + cc * VO + 4);
                v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
                v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
                store_out_chunk<T, decltype(extra)::value, POST>(a, P, plane, m, n, v, VO);
            }
        };
        if (a.res || a.mask_mode)
            run(std::true_type{});
        else
            run(std::false_type{});
    } else {
        for (int id = tid; id < BM * BN; id += NTH) {
            const int col = id / BM, row = id - (id / BM) * BM;
            const int m = rowm(row), n = n0 + col;
            if (m < 0 || n >= a.Cout) continue;
            store_out_scalar<T, POST>(a, P, plane, m, n, E[row * ES + col]);
        }
    }
}

#ifndef CAI_WG_BIAS_AFTER
#define CAI_WG_BIAS_AFTER 1   // A/B: 0 = the halo weight gradient's bias sums ahead of each fragment's MFMAs
#endif
#ifndef CAI_EPI_MASK_PREFETCH
#define CAI_EPI_MASK_PREFETCH 2   // A/B: 0 = the per-chunk masked epilogue, 1 = staged through LDS with prefetch
#endif

// Epilogue for TRANSPOSED accumulators (weights as the MFMA's A operand): lane (i16, g_) of tile (tm, tn)
// holds output channels wn*WTN + tn*16 + 4*g_ + 0..3 of tile row wm*WTM + tm*16 + i16, so the common cases
// store straight from registers: split-K partials as 16-byte fp32 stores into the slab, bf16 outputs
// (bias + act) as 8-byte stores.  Masked or non-bf16 / scalar outputs go through LDS as in
// conv_epilogue_rows (E must then hold BM*(BN+4) floats; NOLDS tiles have no such buffer and are only
// launched where epi_t_direct holds or K is split).
__host__ __device__ __forceinline__ bool epi_t_direct(const ConvArgs& a) {
    return a.y_vec && a.y_dtype == CAI_BF16 && (a.Cout & 3) == 0 &&
           (!a.mask_mode || ((a.aux_ld & 3) == 0 && (reinterpret_cast<uintptr_t>(a.aux) & 7) == 0));
}

// MPF: the mask-prefetch forms below -- instantiated by the stride-1 input-gradient halo kernels only (in the
// stride-2 gather / phase kernels the extra live registers pushed conv_halo_kernel<5> into 128 bytes of spills)
template <typename T, int BM, int BN, int WM, int WN, int NTH, class RowMap, bool NOLDS = false, bool POST = true,
          bool MPF = false>
__device__ __forceinline__ void conv_epilogue_rows_t(const ConvArgs& a, const PhaseDesc& P, int plane, int n0,
                                                     float* E, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                                     RowMap rowm, int slab) {
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int ES = BN + 4;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int g_ = lane >> 4, i16 = lane & 15;
    if (a.ksplit > 1) {
        float* dst = a.ws + (int64_t)slab * a.ws_rows * a.ws_ld;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int m = rowm(wm * WTM + tm * 16 + i16);
            if (m < 0) continue;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * WTN + tn * 16 + 4 * g_;
                if (n < a.ws_ld) *reinterpret_cast<f32x4*>(dst + (int64_t)m * a.ws_ld + n) = acc[tm][tn];
            }
        }
        return;
    }
    // gradient mask without residual (the input gradients of LeakyReLU / ReLU-fed convs), any tile: straight from the
    // registers, every mask load (and bias load) issued before the first store -- the loads-behind-stores rule of
    // section 6; the accumulators' 64 VGPRs + 2 per (tm, tn) mask chunk stay far below the main loop's pressure
    if (MPF && CAI_EPI_MASK_PREFETCH == 2 && std::is_same<T, bf16>::value && epi_t_direct(a) && a.mask_mode && !a.res) {
        const bf16* AUX = reinterpret_cast<const bf16*>(a.aux);
        bf16x4 mv[TM][TN];
        f32x4 bv[TN];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int m = rowm(wm * WTM + tm * 16 + i16);
            int b, oy, ox;
            out_pixel<T>(a, P, plane, m < 0 ? 0 : m, b, oy, ox);
            const bf16* arow = AUX + (((int64_t)b * a.out_h + oy) * a.out_w + ox) * a.aux_ld;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * WTN + tn * 16 + 4 * g_;
                mv[tm][tn] = (m >= 0 && n < a.Cout) ? *reinterpret_cast<const bf16x4*>(arow + n) : bf16x4{};
            }
        }
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * WTN + tn * 16 + 4 * g_;
#pragma unroll
            for (int r = 0; r < 4; ++r) bv[tn][r] = (a.bias && n + r < a.Cout) ? a.bias[n + r] : 0.f;
        }
        wait_vmcnt<0>();
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int m = rowm(wm * WTM + tm * 16 + i16);
            int b, oy, ox;
            out_pixel<T>(a, P, plane, m < 0 ? 0 : m, b, oy, ox);
            bf16* Y = reinterpret_cast<bf16*>(a.y) + (int64_t)b * a.ysb + (int64_t)oy * a.ysy + (int64_t)ox * a.ysx;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * WTN + tn * 16 + 4 * g_;
                bf16x4 h;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    h[r] = (bf16)(apply_act(acc[tm][tn][r] + bv[tn][r], a.act, a.act_param) *
                                  mask_val(a.mask_mode, (float)mv[tm][tn][r], a.mask_param));
                if (m >= 0 && n < a.Cout) *reinterpret_cast<bf16x4*>(Y + n) = h;
            }
        }
        return;
    }
    // (the general mask variant only in the NOLDS tiles: in the 128-channel halo kernels its registers spill the loop)
    if (NOLDS ? epi_t_direct(a)
              : (a.y_vec && a.y_dtype == CAI_BF16 && !a.mask_mode && (a.Cout & 3) == 0)) {
        f32x4 bv[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int n = n0 + wn * WTN + tn * 16 + 4 * g_;
#pragma unroll
            for (int r = 0; r < 4; ++r) bv[tn][r] = (a.bias && n + r < a.Cout) ? a.bias[n + r] : 0.f;
        }
        if (!a.res && !(NOLDS && a.mask_mode)) {
            // no residual, no mask: stores only.  The bias loads are retired here once: a wait at their first use
            // inside the store loop (the compiler's, behind divergent control flow) was a vmcnt(0) that also
            // drained every store issued before it -- the epilogue ran at ~1.3 TB/s, 38 % of the phase kernel's
            // block time (CAI_PH_PROBE).
            wait_vmcnt<0>();
            // the activation as one branch-free select: v > 0 ? v : v * neg (neg = 0 / slope / 1; the ReLU's
            // negative side stays +0)
            const float neg = a.act == CAI_ACT_RELU ? 0.f : (a.act == CAI_ACT_LEAKY ? a.act_param : 1.f);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const int m = rowm(wm * WTM + tm * 16 + i16);
                int b, oy, ox;
                out_pixel<T>(a, P, plane, m < 0 ? 0 : m, b, oy, ox);
                bf16* Y = reinterpret_cast<bf16*>(a.y) + (int64_t)b * a.ysb + (int64_t)oy * a.ysy + (int64_t)ox * a.ysx;
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    const int n = n0 + wn * WTN + tn * 16 + 4 * g_;
                    bf16x4 h;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float v = acc[tm][tn][r] + bv[tn][r];
                        h[r] = (bf16)(v > 0.f ? v : (neg == 0.f ? 0.f : v * neg));
                    }
                    if (m >= 0 && n < a.Cout) *reinterpret_cast<bf16x4*>(Y + n) = h;
                }
            }
            return;
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int m = rowm(wm * WTM + tm * 16 + i16);
            if (m < 0) continue;
            int b, oy, ox;
            out_pixel<T>(a, P, plane, m, b, oy, ox);
            bf16* Y = reinterpret_cast<bf16*>(a.y) + (int64_t)b * a.ysb + (int64_t)oy * a.ysy + (int64_t)ox * a.ysx;
            // gradient mask (dgrad): the aux tensor at the same pixel, 4 channels per lane as in store_out_chunk
            const bf16* AUX = (NOLDS && a.mask_mode) ? reinterpret_cast<const bf16*>(a.aux) +
                                                           (((int64_t)b * a.out_h + oy) * a.out_w + ox) * a.aux_ld
                                                     : nullptr;
            const int64_t rpx = ((int64_t)b * a.out_h + oy) * a.out_w + ox;
            const bf16* RS = a.res ? a.res + rpx * a.res_ld : nullptr;
            const bf16* RS2 = a.res2 ? a.res2 + rpx * a.res2_ld : nullptr;
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int n = n0 + wn * WTN + tn * 16 + 4 * g_;
                if (n >= a.Cout) continue;
                f32x4 v;
                f32x4 rf = f32x4{0.f, 0.f, 0.f, 0.f};
                if (RS) {
                    const bf16x4 rv = *reinterpret_cast<const bf16x4*>(RS + n);
#pragma unroll
                    for (int r = 0; r < 4; ++r) rf[r] = (float)rv[r];
                    if (RS2) {
                        const bf16x4 rv2 = *reinterpret_cast<const bf16x4*>(RS2 + n);
#pragma unroll
                        for (int r = 0; r < 4; ++r) rf[r] += (float)rv2[r];
                    }
                }
                f32x4 mk = f32x4{1.f, 1.f, 1.f, 1.f};
                if (NOLDS && AUX) {
                    const bf16x4 mv = *reinterpret_cast<const bf16x4*>(AUX + n);
#pragma unroll
                    for (int r = 0; r < 4; ++r) mk[r] = mask_val(a.mask_mode, (float)mv[r], a.mask_param);
                }
                // res_post (dgrad): mask(aux) * (conv input gradient) + res; else mask(aux) * act(... + res)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    v[r] = (POST && a.res_post) ? (acc[tm][tn][r] + bv[tn][r]) * mk[r] + rf[r]
                                      : apply_act(acc[tm][tn][r] + bv[tn][r] + rf[r], a.act, a.act_param) * mk[r];
                bf16x4 h;
#pragma unroll
                for (int r = 0; r < 4; ++r) h[r] = (bf16)v[r];
                *reinterpret_cast<bf16x4*>(Y + n) = h;
            }
        }
        return;
    }
    if constexpr (NOLDS) return;    // host guarantees epi_t_direct (or split-K) for these tiles
    else {
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int row = wm * WTM + tm * 16 + i16, col = wn * WTN + tn * 16 + 4 * g_;
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + col + r;
                const float bvr = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
                v[r] = act_pre(a, acc[tm][tn][r] + bvr);
            }
            *reinterpret_cast<f32x4*>(E + row * ES + col) = v;
        }
    // gradient mask, no residual, bf16 output and aux (the input gradients of LeakyReLU-fed convs): every aux chunk of
    // this thread's output chunks is loaded up front, before the staging barrier.  In the per-chunk form each aux load
    // waited behind the previous chunk's store on the shared vmcnt -- one exposed load latency per chunk, the
    // multimodal trunk's 256-channel input gradients ran 1.4x their forwards' time (-DCAI_EPI_MASK_PREFETCH=0: that form)
    constexpr int CPR8 = BN / 8, NIT = (BM * CPR8 + NTH - 1) / NTH;
    const bool mfast = MPF && std::is_same<T, bf16>::value && CAI_EPI_MASK_PREFETCH == 1 && a.y_vec && a.mask_mode && !a.res &&
                       a.y_dtype == CAI_BF16 && (a.Cout & 7) == 0 && (a.aux_ld & 7) == 0 &&
                       (reinterpret_cast<uintptr_t>(a.aux) & 15) == 0;
    bf16x8 mreg[NIT];
    if (mfast) {
        const bf16* AUX = reinterpret_cast<const bf16*>(a.aux);
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int id = tid + it * NTH, row = id / CPR8, n = n0 + (id - row * CPR8) * 8;
            const int m = id < BM * CPR8 ? rowm(row) : -1;
            mreg[it] = bf16x8{};
            if (m >= 0 && n < a.Cout) {
                int b, oy, ox;
                out_pixel<T>(a, P, plane, m, b, oy, ox);
                mreg[it] = *reinterpret_cast<const bf16x8*>(AUX + (((int64_t)b * a.out_h + oy) * a.out_w + ox) * a.aux_ld + n);
            }
        }
    }
    __syncthreads();
    if (mfast) {
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int id = tid + it * NTH, row = id / CPR8, cc = id - row * CPR8, n = n0 + cc * 8;
            const int m = id < BM * CPR8 ? rowm(row) : -1;
            if (m < 0 || n >= a.Cout) continue;
            const f32x4 lo = *reinterpret_cast<const f32x4*>(E + row * ES + cc * 8);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(E + row * ES + cc * 8 + 4);
            const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            bf16x8 h;
#pragma unroll
            for (int e = 0; e < 8; ++e) h[e] = (bf16)(v[e] * mask_val(a.mask_mode, (float)mreg[it][e], a.mask_param));
            int b, oy, ox;
            out_pixel<T>(a, P, plane, m, b, oy, ox);
            *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.y) + (int64_t)b * a.ysb + (int64_t)oy * a.ysy +
                                       (int64_t)ox * a.ysx + n) = h;
        }
        return;
    }
    if (a.y_vec) {
        const int VO = a.y_dtype == CAI_BF16 ? 8 : 4;
        const int cpr = BN / VO;
        auto run = [&](auto extra) {
            for (int id = tid; id < BM * cpr; id += NTH) {
                const int row = id / cpr, cc = id - (id / cpr) * cpr;
                const int m = rowm(row), n = n0 + cc * VO;
                if (m < 0 || n >= a.Cout) continue;
                float v[8];
                const f32x4 lo = *reinterpret_cast<const f32x4*>(E + row * ES + cc * VO);
                f32x4 hi = f32x4{0.f, 0.f, 0.f, 0.f};
                if (VO == 8) hi = *reinterpret_cast<const f32x4*>(E + row * ES + cc * VO + 4);
                v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
                v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
                store_out_chunk<T, decltype(extra)::value, POST>(a, P, plane, m, n, v, VO);
            }
        };
        if (a.res || a.mask_mode)
            run(std::true_type{});
        else
            run(std::false_type{});
    } else {
        for (int id = tid; id < BM * BN; id += NTH) {
            const int col = id / BM, row = id - (id / BM) * BM;
            const int m = rowm(row), n = n0 + col;
            if (m < 0 || n >= a.Cout) continue;
            store_out_scalar<T, POST>(a, P, plane, m, n, E[row * ES + col]);
        }
    }
    }
}

template <typename T, int BM, int BN, int WM, int WN, int NTH>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const PhaseDesc& P, int plane, int Mph, int m0,
                                              int n0, float* E, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16]) {
    conv_epilogue_rows<T, BM, BN, WM, WN, NTH>(a, P, plane, n0, E, acc, [=](int row) {
        const int m = m0 + row;
        return m < Mph ? m : -1;
    });
}

template <typename T, typename C>
__global__ __launch_bounds__(NT, 2) void conv_gemm_kernel(const ConvArgs a) {
    constexpr int BM = C::BM, BN = C::BN, WM = C::WM, WN = C::WN;
    constexpr int VEC = OpT<T>::VEC;
    constexpr int BK = 128 / (int)sizeof(T);
    constexpr int A_CH = BM * 8 / NT;
    constexpr int B_CH = (BN * 8 + NT - 1) / NT;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    static_assert(BM % 32 == 0 && WM * WN == 4 && WTM % 16 == 0 && WTN % 16 == 0, "bad tile");
    using SM = ConvSmem<T, C>;
    __shared__ __attribute__((aligned(16))) char smem[SM::BYTES];

    // grid.z = phase * ksplit + split.  The phase descriptor is selected with
    // uniform branches (a dynamic index into the by-value kernarg struct would
    // be copied to scratch).
    const int ph = blockIdx.z / a.ksplit, split = blockIdx.z - ph * a.ksplit;
    const PhaseDesc P = ph == 0 ? a.ph[0] : (ph == 1 ? a.ph[1] : (ph == 2 ? a.ph[2] : a.ph[3]));
    const int plane = P.OHg * P.OWg;
    const int Mph = a.B * plane;
    const int m0 = blockIdx.x * BM;
    if (m0 >= Mph) return;
    const int n0 = blockIdx.y * BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int slot = tid & 7;

    // ---- per-row gather state of this thread's A chunks (rows i*32 + tid/8) ----
    int rbase[A_CH], ry[A_CH], rx[A_CH];
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
        const int m = m0 + i * (NT / 8) + (tid >> 3);
        if (m < Mph) {
            const int b = m / plane;
            const int r = m - b * plane;
            const int j = r / P.OWg;
            rbase[i] = b * a.IH;
            ry[i] = j * a.row_stride;
            rx[i] = (r - j * P.OWg) * a.row_stride;
        } else {
            rbase[i] = 0;
            ry[i] = -(1 << 28);   // forces the bounds test to fail
            rx[i] = 0;
        }
    }
    const gptr<T> X = to_global<T>(a.x);
    const gptr<T> W = to_global<T>(a.w) + P.w_off + slot * VEC;
    int woff[B_CH];
    bool wok[B_CH];
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
        const int row = (i * NT + tid) >> 3;
        wok[i] = row < BN && n0 + row < a.Npad;
        woff[i] = wok[i] ? (n0 + row) * a.Kp : 0;
    }
    // K-tile range of this split
    const int nk_all = (P.K + BK - 1) / BK;
    const int per = (nk_all + a.ksplit - 1) / a.ksplit;
    const int kt0 = split * per;
    const int kt1 = min(nk_all, kt0 + per);
    const int nk = max(0, kt1 - kt0);
    const u32x4 zero = u32x4{0u, 0u, 0u, 0u};
    U4<A_CH> ra0, ra1;
    U4<B_CH> rw0, rw1;

#define CONV_LOAD_TILE(KT, RA, RW)                                                                           \
    {                                                                                                        \
        const int kg_ = kt0 + (KT);                                                                          \
        const int k_ = kg_ * BK + slot * VEC;                                                                \
        const int t_ = k_ / a.Cin_pad;                                                                       \
        const int ci_ = k_ - t_ * a.Cin_pad;                                                                 \
        const int ty_ = t_ / P.ntx;                                                                          \
        int dy_ = P.dy0 + a.tap_sy * ty_;                                                                    \
        const int dx_ = P.dx0 + a.tap_sx * (t_ - ty_ * P.ntx);                                               \
        if (t_ >= P.ntaps) dy_ = -(1 << 28);                                                                 \
        _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                                                   \
            const int iy = ry[i] + dy_, ix = rx[i] + dx_;                                                    \
            const bool ok = (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;                 \
            const int64_t off = ok ? ((int64_t)(rbase[i] + iy) * a.IW + ix) * a.x_ld + ci_ : 0;             \
            u32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(X + off);            \
            if (a.in_abs) v = abs_chunk(v, sizeof(T));                                                       \
            RA.v[i] = ok ? v : zero;                                                                         \
        }                                                                                                    \
        _Pragma("unroll") for (int i = 0; i < B_CH; ++i) {                                                   \
            const u32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(              \
                W + woff[i] + kg_ * BK);                                                                     \
            RW.v[i] = wok[i] ? v : zero;                                                                     \
        }                                                                                                    \
    }

#define CONV_STORE_TILE(BUF, RA, RW)                                                                         \
    {                                                                                                        \
        char* As_ = smem + (BUF) * (BM + BN) * 128;                                                          \
        char* Bs_ = As_ + BM * 128;                                                                          \
        _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                                                   \
            const int row = i * (NT / 8) + (tid >> 3);                                                       \
            *reinterpret_cast<u32x4*>(As_ + row * 128 + swz(row, slot) * 16) = RA.v[i];                      \
        }                                                                                                    \
        _Pragma("unroll") for (int i = 0; i < B_CH; ++i) {                                                   \
            const int row = (i * NT + tid) >> 3;                                                             \
            if (row < BN) *reinterpret_cast<u32x4*>(Bs_ + row * 128 + swz(row, slot) * 16) = RW.v[i];        \
        }                                                                                                    \
    }

#define CONV_COMPUTE(BUF)                                                                                    \
    {                                                                                                        \
        const char* As = smem + (BUF) * (BM + BN) * 128;                                                     \
        const char* Bs = As + BM * 128;                                                                      \
        _Pragma("unroll") for (int c = 0; c < 2; ++c) {                                                      \
            const int ls = c * 4 + (lane >> 4);                                                              \
            u32x4 fa[TM], fb[TN];                                                                            \
            _Pragma("unroll") for (int tm = 0; tm < TM; ++tm) {                                              \
                const int row = wm * WTM + tm * 16 + (lane & 15);                                            \
                fa[tm] = *reinterpret_cast<const u32x4*>(As + row * 128 + swz(row, ls) * 16);                \
            }                                                                                                \
            _Pragma("unroll") for (int tn = 0; tn < TN; ++tn) {                                              \
                const int row = wn * WTN + tn * 16 + (lane & 15);                                            \
                fb[tn] = *reinterpret_cast<const u32x4*>(Bs + row * 128 + swz(row, ls) * 16);                \
            }                                                                                                \
            _Pragma("unroll") for (int tm = 0; tm < TM; ++tm)                                                \
                _Pragma("unroll") for (int tn = 0; tn < TN; ++tn)                                            \
                    acc[tm][tn] = mma16<T>(fa[tm], fb[tn], acc[tm][tn]);                                     \
        }                                                                                                    \
    }

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // 2-deep register prefetch: tile t+2 is in flight while tile t is
    // computed and tile t+1 is written to the other LDS buffer.
    if (nk > 0) {
        CONV_LOAD_TILE(0, ra0, rw0);
        CONV_STORE_TILE(0, ra0, rw0);
        if (nk > 1) CONV_LOAD_TILE(1, ra1, rw1);
        __syncthreads();
        for (int kt = 0; kt < nk; kt += 2) {
            if (kt + 2 < nk) CONV_LOAD_TILE(kt + 2, ra0, rw0);
            CONV_COMPUTE(0);
            if (kt + 1 < nk) CONV_STORE_TILE(1, ra1, rw1);
            __syncthreads();
            if (kt + 1 >= nk) break;
            if (kt + 3 < nk) CONV_LOAD_TILE(kt + 3, ra1, rw1);
            CONV_COMPUTE(1);
            if (kt + 2 < nk) CONV_STORE_TILE(0, ra0, rw0);
            __syncthreads();
        }
    }
#undef CONV_LOAD_TILE
#undef CONV_STORE_TILE
#undef CONV_COMPUTE

    conv_epilogue<T, BM, BN, WM, WN, NT>(a, P, plane, Mph, m0, n0, reinterpret_cast<float*>(smem), acc);
}

// ---------------------------------------------------------------------------
// bf16 implicit GEMM with LDS-DMA staging (global_load_lds_dwordx4) and a
// 3-stage ring: tile kt+2 streams into LDS while tile kt is multiplied, one
// raw barrier per K-tile behind a counted vmcnt (cdna_hip_programming.md §5
// "Pipelining across barriers").  512 threads = 8 waves.  With
// Cin_pad % 64 == 0 every 64-channel K-tile lies inside one tap (Cin_pad % 64 == 32: each 32-channel half
// of a K-tile lies inside one tap and is addressed on its own): the tap's
// (dy, dx) shift is uniform per tile and the per-lane gather is one add + a
// bounds test.  Padding taps read a zero page.  The LDS image is lane-linear
// (DMA), so the XOR swizzle that keeps the fragment reads conflict-free is
// applied to the per-lane SOURCE slot (both-sides rule).
// ---------------------------------------------------------------------------
__device__ __attribute__((aligned(64))) unsigned cai_zero_page[64];

template <int BM_, int BN_, int WM_, int WN_>
struct Cfg2 {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
    static constexpr int NTH = 512, STAGES = 3;
    static constexpr int STAGE = (BM + BN) * 128;
    static constexpr int EPI = BM * (BN + 4) * 4;
    static constexpr int BYTES = (STAGES * STAGE > EPI) ? STAGES * STAGE : EPI;
};

typedef const void __attribute__((address_space(1)))* gvoid_ptr;
typedef void __attribute__((address_space(3)))* lvoid_ptr;

#define GLDS glds16_asm

template <typename C>
__global__ __launch_bounds__(512, 1) void conv_glds_kernel(const ConvArgs a) {
    constexpr int BM = C::BM, BN = C::BN, WM = C::WM, WN = C::WN;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int AG = BM / 64, BG = BN / 64;     // DMA instructions per thread per K-tile
    constexpr int G = AG + BG;
    static_assert(WM * WN == 8 && BM % 64 == 0 && BN % 64 == 0, "bad tile");
    __shared__ __attribute__((aligned(16))) char smem[C::BYTES];

    const int ph = blockIdx.z / a.ksplit, split = blockIdx.z - ph * a.ksplit;
    const PhaseDesc P = ph == 0 ? a.ph[0] : (ph == 1 ? a.ph[1] : (ph == 2 ? a.ph[2] : a.ph[3]));
    const int plane = P.OHg * P.OWg;
    const int Mph = a.B * plane;
    const int m0 = blockIdx.x * BM;
    if (m0 >= Mph) return;
    const int n0 = blockIdx.y * BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;

    // this thread's DMA rows: i*64 + wid*8 + lane/8; all share one logical slot
    const int rsub = wid * 8 + (lane >> 3);
    const int ls = (lane & 7) ^ ((rsub >> 1) & 7);
    // Cin_pad % 64 == 32 (96-, 160-channel inputs): a 64-element K-tile may straddle two taps; slots 0-3 and
    // 4-7 are then addressed separately (half = the 32-element half this lane's slot belongs to), and
    // elements past K (the packed rows' zero padding) read the zero page
    const bool halves = (a.Cin_pad & 63) != 0;
    const int hsel = ls >> 2;
    const char* X = reinterpret_cast<const char*>(a.x);
    const int ld_b = a.x_ld * 2;                 // bytes per pixel row
    int abase[AG], ay[AG], ax[AG];
#pragma unroll
    for (int i = 0; i < AG; ++i) {
        const int m = m0 + i * 64 + rsub;
        if (m < Mph) {
            const int b = m / plane;
            const int r = m - b * plane;
            const int j = r / P.OWg;
            ay[i] = j * a.row_stride;
            ax[i] = (r - j * P.OWg) * a.row_stride;
            abase[i] = ((b * a.IH + ay[i]) * a.IW + ax[i]) * ld_b + (halves ? (ls & 3) : ls) * 16;
        } else {
            ay[i] = -(1 << 28);
            ax[i] = 0;
            abase[i] = 0;
        }
    }
    const char* Wb = reinterpret_cast<const char*>(a.w) + P.w_off * 2 + ls * 16;
    int boff[BG];
#pragma unroll
    for (int i = 0; i < BG; ++i) {
        const int row = n0 + i * 64 + rsub;
        boff[i] = row < a.Npad ? row * a.Kp * 2 : -1;
    }
    const int nk_all = (P.K + 63) / 64;
    const int per = (nk_all + a.ksplit - 1) / a.ksplit;
    const int kt0 = split * per;
    const int nk = max(0, min(nk_all, kt0 + per) - kt0);

    auto issue = [&](int kt, int stage) {
        const int kg = kt0 + kt;
        // the K element this lane's slot starts its 32-element half at (whole tile when !halves)
        const int k0 = kg * 64 + (halves ? hsel * 32 : 0);
        const int t = k0 / a.Cin_pad;
        const int ci0 = k0 - t * a.Cin_pad;
        const int ty = t / P.ntx;
        const int dy = P.dy0 + a.tap_sy * ty, dx = P.dx0 + a.tap_sx * (t - ty * P.ntx);
        const int delta = (dy * a.IW + dx) * ld_b + ci0 * 2;
        const bool kin = k0 < P.K;
        char* sbase = smem + stage * C::STAGE + wid * 8 * 128;
#pragma unroll
        for (int i = 0; i < AG; ++i) {
            const int iy = ay[i] + dy, ix = ax[i] + dx;
            const bool ok = kin && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
            const void* src = ok ? (const void*)(X + abase[i] + delta) : (const void*)cai_zero_page;
            GLDS(src, sbase + i * 64 * 128);
        }
#pragma unroll
        for (int i = 0; i < BG; ++i) {
            const void* src = boff[i] >= 0 ? (const void*)(Wb + boff[i] + kg * 128) : (const void*)cai_zero_page;
            GLDS(src, sbase + BM * 128 + i * 64 * 128);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (nk > 0) issue(0, 0);
    if (nk > 1) issue(1, 1);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk)
            wait_vmcnt<G>();
        else
            wait_vmcnt<0>();
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const char* As = smem + (kt % 3) * C::STAGE;
        const char* Bs = As + BM * 128;
        // every fragment of the K-tile is requested up front; the second half's reads and the next
        // DMA issue overlap the first half's MFMAs (one exposed LDS latency per K-tile, not four)
        u32x4 fa[2][TM], fb[2][TN];
        auto rd_a = [&](int c) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const int row = wm * WTM + tm * 16 + (lane & 15);
                fa[c][tm] = *reinterpret_cast<const u32x4*>(As + row * 128 + swz(row, c * 4 + (lane >> 4)) * 16);
            }
        };
        auto rd_b = [&](int c) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int row = wn * WTN + tn * 16 + (lane & 15);
                fb[c][tn] = *reinterpret_cast<const u32x4*>(Bs + row * 128 + swz(row, c * 4 + (lane >> 4)) * 16);
            }
        };
        // lgkmcnt holds 15 reads: the first half's fragments and the second half's A go out first, the
        // second half's B behind the first 16 MFMAs
        rd_a(0);
        rd_b(0);
        rd_a(1);
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * TM + TN, 0);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mma16<bf16>(fa[0][tm], fb[0][tn], acc[tm][tn]);
        __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
        rd_b(1);
        __builtin_amdgcn_sched_group_barrier(0x100, TN, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 2 < nk) issue(kt + 2, (kt + 2) % 3);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mma16<bf16>(fa[1][tm], fb[1][tn], acc[tm][tn]);
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    conv_epilogue<bf16, BM, BN, WM, WN, 512>(a, P, plane, Mph, m0, n0, reinterpret_cast<float*>(smem), acc);
}

// ---------------------------------------------------------------------------
// Latent-size convolutions (the hyper branch and the latent ends of g_a / g_s: 4x4 .. 16x16 latents at the
// training batch): the whole K reduction in ONE launch, no split-K partial slabs and no reduce launch.
// These GEMMs have M = B*H*W of a few hundred to a few thousand rows against K = taps*Cin = 1-3 thousand:
// a tile grid cannot fill the chip, and the split-K path paid a second launch for the combine.  Here a
// block owns a small BM x BN output tile (16..32 x 32..64) and its 8 waves split K eight ways inside the
// block; each wave loads its MFMA fragments straight from global memory into registers (no operand is
// shared between the waves, so there is nothing to stage in LDS), D K-steps ahead, every load issued as
// a buffer load whose out-of-range lanes (padding taps, rows past M, K-steps past the wave's range) carry
// an offset beyond the buffer and read 0 -- no branch around any load, so the compiler's counted waits
// never see a shorter path.  The 8 partial tiles meet in LDS and are summed in wave order (deterministic), then the usual
// epilogue (bias, ReLU / LeakyReLU, gradient mask, 16-byte stores).  Gather and phase modes as above;
// K steps of 32 channels inside one tap (Cin_pad % 32 == 0), bf16, |x| on load for h_a's first conv.
// ---------------------------------------------------------------------------
constexpr int SMALL_NW = 8, SMALL_D = 4;

template <int RT, int CT>
struct SmallCfg {
    static constexpr int BM = 16 * RT, BN = 16 * CT, ES = BN + 4;
    static constexpr int BYTES = SMALL_NW * BM * ES * 4;
};

template <int RT, int CT>
__global__ __launch_bounds__(512, 1) void conv_small_kernel(const ConvArgs a) {
    using SC = SmallCfg<RT, CT>;
    constexpr int BM = SC::BM, BN = SC::BN, ES = SC::ES, D = SMALL_D;
    __shared__ __attribute__((aligned(16))) float red[SMALL_NW * BM * ES];

    const int ph = blockIdx.z;
    const PhaseDesc P = ph == 0 ? a.ph[0] : (ph == 1 ? a.ph[1] : (ph == 2 ? a.ph[2] : a.ph[3]));
    const int plane = P.OHg * P.OWg;
    const int Mph = a.B * plane;
    const int m0 = blockIdx.x * BM;
    if (m0 >= Mph) return;
    const int n0 = blockIdx.y * BN;
    // wave-uniform as a scalar: the K-step bookkeeping below stays on the SALU
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kq = 8 * (lane >> 4);               // this lane's 8 K elements of a 32-wide step

    constexpr unsigned OOB = 0x80000000u;          // beyond every buffer: the load returns 0
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(a.x), (short)0, (int)((int64_t)a.B * a.IH * a.IW * a.x_ld * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(a.w), (short)0, (int)((int64_t)a.nphase * a.Npad * a.Kp * 2), 0x00020000);
    int abase[RT];                                 // element offsets (inputs < 2 GiB: checked by run_conv)
    int ay[RT], ax[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int m = m0 + rt * 16 + (lane & 15);
        if (m < Mph) {
            const int b = m / plane;
            const int r = m - b * plane;
            const int j = r / P.OWg;
            ay[rt] = j * a.row_stride;
            ax[rt] = (r - j * P.OWg) * a.row_stride;
            abase[rt] = ((b * a.IH + ay[rt]) * a.IW + ax[rt]) * a.x_ld + kq;
        } else {
            ay[rt] = -(1 << 28);
            ax[rt] = 0;
            abase[rt] = 0;
        }
    }
    int boff[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        const int n = n0 + ct * 16 + (lane & 15);
        boff[ct] = n < a.Npad ? (int)P.w_off + n * a.Kp + kq : -1;
    }
    // this wave's K steps: [k0, k0 + per), padded to whole groups of D (the padding reads the zero page)
    const int nk = P.K / 32;
    const int per = (nk + SMALL_NW - 1) / SMALL_NW;
    const int k0 = wave * per, k1 = min(nk, k0 + per);
    const int ngroups = (per + D - 1) / D;

    // the tap / channel position of the next K step to load: loads are issued for consecutive K steps (k0,
    // k0 + 1, ...), so it advances by one 32-channel step per load instead of being re-derived with two integer
    // divisions (~50 VALU instructions per load: the kernels were VALU-issue bound, 1,400 VALU per wave for 56
    // MFMAs on C2's h_a[0])
    int st_kg = k0 * 32, st_t = st_kg / a.Cin_pad;
    int st_ci = st_kg - st_t * a.Cin_pad, st_ty = st_t / P.ntx;
    int st_tx = st_t - st_ty * P.ntx;
    auto load = [&](int ks, u32x4 (&fa)[RT], u32x4 (&fb)[CT]) {
        const bool kok = ks < k1;
        const int kg = st_kg;
        const int dy = P.dy0 + a.tap_sy * st_ty, dx = P.dx0 + a.tap_sx * st_tx;
        const int delta = (dy * a.IW + dx) * a.x_ld + st_ci;
        st_kg += 32;
        st_ci += 32;
        const bool w1 = st_ci == a.Cin_pad;
        st_ci = w1 ? 0 : st_ci;
        st_tx += w1 ? 1 : 0;
        const bool w2 = st_tx == P.ntx;
        st_tx = w2 ? 0 : st_tx;
        st_ty += w2 ? 1 : 0;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            // bitwise tests and an unconditional offset: a short-circuit && here becomes a branch
            const int iy = ay[rt] + dy, ix = ax[rt] + dx;
            const bool ok = kok & ((unsigned)iy < (unsigned)a.IH) & ((unsigned)ix < (unsigned)a.IW);
            const unsigned off = (unsigned)(abase[rt] + delta) * 2u;
            fa[rt] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? off : OOB, 0, 0));
        }
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const unsigned off = (unsigned)(boff[ct] + kg) * 2u;
            const bool ok = kok & (boff[ct] >= 0);
            fb[ct] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, ok ? off : OOB, 0, 0));
        }
    };

    f32x4 acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 fa[D][RT], fb[D][CT];
#pragma unroll
    for (int d = 0; d < D; ++d) load(k0 + d, fa[d], fb[d]);
    for (int g = 0; g < ngroups; ++g) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            u32x4 ca[RT], cb[CT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) ca[rt] = a.in_abs ? abs_chunk(fa[d][rt], 2) : fa[d][rt];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) cb[ct] = fb[d][ct];
            load(k0 + (g + 1) * D + d, fa[d], fb[d]);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = mma16<bf16>(ca[rt], cb[ct], acc[rt][ct]);
        }
    }
    // the 8 partial tiles -> LDS, summed in wave order by the epilogue threads
    float* mine = red + wave * BM * ES;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int r = 0; r < 4; ++r) mine[(rt * 16 + (lane >> 4) * 4 + r) * ES + ct * 16 + (lane & 15)] = acc[rt][ct][r];
    __syncthreads();
    const int VO = a.y_dtype == CAI_BF16 ? 8 : 4;
    const int cpr = BN / VO;
    for (int id = tid; id < BM * cpr; id += 512) {
        const int row = id / cpr, cc = id - (id / cpr) * cpr;
        const int m = m0 + row, nb = n0 + cc * VO;
        if (m >= Mph || nb >= a.Cout) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
        for (int w = 0; w < SMALL_NW; ++w) {
            const float* src = red + (w * BM + row) * ES + cc * VO;
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (e < VO) v[e] += src[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int n = nb + e;
            const float bv = (a.bias && e < VO && n < a.Cout) ? a.bias[n] : 0.f;
            v[e] = act_pre(a, v[e] + bv);
        }
        if (a.y_vec && !a.res && !a.mask_mode) {
            store_out_chunk<bf16, false>(a, P, plane, m, nb, v, VO);
        } else if (a.y_vec) {
            store_out_chunk<bf16>(a, P, plane, m, nb, v, VO);
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (e < VO && nb + e < a.Cout) store_out_scalar<bf16>(a, P, plane, m, nb + e, v[e]);
        }
    }
}

// ---------------------------------------------------------------------------
// Halo-staged implicit GEMM for the stride-2 gather convolutions (Conv2d k3/k5 s2 p=k/2 forward and the
// matching ConvTranspose2d input gradient), bf16.  The tap-gather kernel above fetches every input pixel
// once per tap (25 times for k5), and its speed is set by how fast a CU can pull bytes into LDS, not by
// the MFMAs (a no-MFMA build of it runs within 1 % of the real one).  Here a block owns an 8 x 32 output
// tile and all 128 output channels; per 32-channel chunk it stages the tile's input footprint
// ((2*7+k) x (2*31+k) pixels) in LDS once, and the k*k taps read their A fragments from that patch at a
// per-tap offset: the A bytes fetched per block drop ~4.5x.  The weights stream through a 4-stage
// LDS-DMA ring (one 16-byte DMA per lane per tap, three taps ahead).
//
// Patch layout: four planes (8 channels each) of 16-byte cells; inside a plane, patch row r, column c
// sits at r*PW + (c&1)*PWE + c/2 (even columns, then odd), so the 16 lanes of one A fragment (16
// consecutive output columns, stride-2 input columns) read 16 consecutive cells.  PLANE = 4 (mod 16)
// keeps the staging writes (4 pixels x 4 planes per 16 lanes) conflict-free too.  The next chunk's
// patch is loaded into registers while the current one is consumed.
// ---------------------------------------------------------------------------
// loads issued after weight tap t+1 that step t's wait leaves in flight: taps t+2 .. t+NSTB-1, the patch
// cells issued at steps j in [t+1-NSTB, t-1] (j < NPI), and the four fence loads that follow cell NPI-1
__host__ __device__ constexpr int halo_younger(int t, int nstb, int npi) {
    const int lo = t + 1 - nstb > 0 ? t + 1 - nstb : 0;
    const int hi = t - 1 < npi - 1 ? t - 1 : npi - 1;
    const int cells = hi >= lo ? hi - lo + 1 : 0;
    const int fences = (npi - 1 >= t + 1 - nstb && npi - 1 <= t - 1) ? 4 : 0;
    return nstb - 2 + cells + fences;
}

// the same count when footprint cell i is issued at step i * csp (fences after the last cell)
__host__ __device__ constexpr int halo_younger_sp(int t, int nstb, int npi, int csp) {
    const int lo = t + 1 - nstb > 0 ? t + 1 - nstb : 0;
    int cells = 0;
    for (int j = lo; j <= t - 1; ++j)
        if (j % csp == 0 && j / csp < npi) ++cells;
    const int last = (npi - 1) * csp;
    return nstb - 2 + cells + ((last >= lo && last <= t - 1) ? 4 : 0);
}


// transposed accumulators + register-direct epilogue (conv_epilogue_rows_t) in the halo kernels: the
// phase kernel's launches 57.8 vs 59.7 us average in the C2 step (profiles/r02_edge_s2d_ab.log, r02af)

template <int KS>
struct HaloCfg {
    static constexpr int TH = 8, TW = 32, BM = TH * TW, BN = 128, WM = 4, WN = 2, CK = 32;
    static constexpr int PH = 2 * (TH - 1) + KS, PW = 2 * (TW - 1) + KS;
    static constexpr int ODD = ((PW + 1) / 2 + 3) / 8 * 8 + 4;   // first odd-column cell of a row: = 4 (mod 8)
    static constexpr int PWR = ODD + PW / 2;                      // cells per patch row
    static constexpr int NPOS = PH * PW;
    static constexpr int PLANE = (PH * PWR + 15) / 16 * 16;       // = 0 (mod 16)
    static constexpr int PATCH = 4 * PLANE * 16;
    static constexpr int NPI = (4 * NPOS + 511) / 512;
    static constexpr int NTAP = KS * KS;
    // NTAP % NSTB == 0: a tap's stage is t % NSTB.  (A 9-deep ring, stage tracked at run time, measured 6 %
    // slower for k5: the compiler's wait before the footprint store then drains taps still in flight.)
    static constexpr int BSTAGE = BN * CK * 2, NSTB = KS;
    // footprint cells are spread over the chunk, one every CSP steps: issued back to back, the next chunk's
    // footprint is requested by all blocks at once and the burst queues at HBM
    static constexpr int CSP = (NTAP - 1) / NPI > 1 ? (NTAP - 1) / NPI : 1;
    static constexpr int EPI = BM * (BN + 4) * 4;
    static constexpr int BYTES = (PATCH + NSTB * BSTAGE > EPI) ? PATCH + NSTB * BSTAGE : EPI;
};

template <int KS>
__global__ __launch_bounds__(512, 1) void conv_halo_kernel(const ConvArgs a, int tiles_x, int tiles_y) {
    using H = HaloCfg<KS>;
    constexpr int BM = H::BM, BN = H::BN, WM = H::WM, WN = H::WN;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int NPI = H::NPI, NTAP = H::NTAP, NSTB = H::NSTB, CSP = H::CSP;
    static_assert(WM * WN == 8 && WTM == 2 * H::TW && H::BYTES <= 160 * 1024 && NPI <= NTAP &&
                  NTAP % NSTB == 0 && (NPI - 1) * CSP <= NTAP - 1, "halo tile");
    __shared__ __attribute__((aligned(16))) char smem[H::BYTES];
    char* const patch = smem;
    char* const bring = smem + H::PATCH;

    const PhaseDesc& P = a.ph[0];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    // consecutive tiles of an image on one XCD: their halos overlap in its L2
    const int ntiles = gridDim.x;
    const int bid = (ntiles & 7) == 0 ? (blockIdx.x & 7) * (ntiles >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const int per_img = tiles_x * tiles_y;
    const int b = bid / per_img;
    const int rt = bid - b * per_img;
    const int ty0 = (rt / tiles_x) * H::TH, tx0 = (rt % tiles_x) * H::TW;
    const int nch = a.Cin_pad / H::CK;
    const int per = (nch + a.ksplit - 1) / a.ksplit;
    const int c0 = blockIdx.z * per;
    const int nc = max(0, min(nch, c0 + per) - c0);
    const char* X = reinterpret_cast<const char*>(a.x);
    const int ld_b = a.x_ld * 2;

    // this thread's patch cells (8 pixels x 4 planes per 32 lanes), recomputed per chunk to keep them out
    // of the loop's registers.  Chunk indices past the block's range load the zero page (the pipeline
    // issues a patch batch after every chunk, so its wait counts stay fixed).
    const int iyb = ty0 * 2 + P.dy0, ixb = tx0 * 2 + P.dx0;
    u32x4 pr_[NPI];
    unsigned fence_[4] = {0u, 0u, 0u, 0u};
    auto load_cell = [&](int ci, int i) {
        const bool real = ci < nc;
        const int cc = c0 + ci;
        const int q4 = tid + 512 * i, g = (q4 >> 3) & 3, q = ((q4 >> 5) << 3) | (q4 & 7);
        const int pr = q / H::PW, pc = q - (q / H::PW) * H::PW;
        const int iy = iyb + pr, ix = ixb + pc;
        const bool in = real && q < H::NPOS && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
        const void* src = in ? (const void*)(X + ((b * a.IH + iy) * a.IW + ix) * ld_b + g * 16 + cc * (H::CK * 2))
                             : (const void*)cai_zero_page;
        pr_[i] = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(reinterpret_cast<uintptr_t>(src));
    };
    // four compiler-visible loads behind a patch batch: the compiler's waits before the patch store then
    // leave the (invisible) weight DMAs issued since in flight instead of draining them
    auto fence_loads = [&]() {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            asm volatile("" ::"v"(fence_[j]));
            fence_[j] = *reinterpret_cast<const __attribute__((address_space(1))) unsigned*>(
                reinterpret_cast<uintptr_t>(cai_zero_page + 16 * j));
        }
    };
    auto store_patch = [&]() {
#pragma unroll
        for (int i = 0; i < NPI; ++i) {
            const int q4 = tid + 512 * i, g = (q4 >> 3) & 3, q = ((q4 >> 5) << 3) | (q4 & 7);
            const int pr = q / H::PW, pc = q - (q / H::PW) * H::PW;
            if (q < H::NPOS)
                *reinterpret_cast<u32x4*>(patch + (g * H::PLANE + pr * H::PWR + (pc & 1) * H::ODD + (pc >> 1)) * 16) =
                    pr_[i];
        }
    };

    // weight ring: LDS cell p of a stage holds (n = p/4, 16-byte slot s) at p = 4n + (s ^ 3*((n/8) & 1)),
    // conflict-free for ds_read_b128's lane groups.  Taps past the block's range read the zero page.
    const int bp = wid * 64 + lane;
    const int bn_ = bp >> 2, bs_ = (bp & 3) ^ (((bn_ >> 3) & 1) * 3);
    const char* Wrow = bn_ < a.Npad ? reinterpret_cast<const char*>(a.w) + bn_ * a.Kp * 2 + bs_ * 16 : nullptr;
    auto issue_b = [&](int ci, int t, int stage) {    // tap t of chunk ci into `stage` (= t % NSTB)
        const void* src = (Wrow && ci < nc) ? (const void*)(Wrow + (t * a.Cin_pad + (c0 + ci) * H::CK) * 2)
                                            : (const void*)cai_zero_page;
        glds16_asm(src, bring + stage * H::BSTAGE + wid * 1024);
    };

    // per-lane fragment cells
    const int g_ = lane >> 4, i16 = lane & 15;
    int apos[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * WTM + tm * 16 + i16;
        apos[tm] = (g_ * H::PLANE + 2 * (r / H::TW) * H::PWR + (r % H::TW)) * 16;
    }
    int bpos[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
        const int n = wn * WTN + tn * 16 + i16;
        bpos[tn] = H::PATCH + (4 * n + (g_ ^ (((n >> 3) & 1) * 3))) * 16;
    }
    auto read_frags = [&](int t, int stage, u32x4 (&fa)[TM], u32x4 (&fb)[TN]) {
        const int ty = t / KS, tx = t % KS;
        const int toff = (ty * H::PWR + (tx & 1) * H::ODD + (tx >> 1)) * 16;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) fa[tm] = *reinterpret_cast<const u32x4*>(smem + apos[tm] + toff);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
            fb[tn] = *reinterpret_cast<const u32x4*>(smem + bpos[tn] + stage * H::BSTAGE);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Step (ci, t) multiplies the fragments read during the previous step while the next step's are read.
    // Its wait retires weight tap t+1; tap t+NSTB then streams into the stage tap t has left.  The next
    // chunk's patch is loaded one cell per step over the first NPI steps (a batch would hold up the taps
    // issued after it: vmcnt retires in issue order), and stored at the chunk's last step.  Every step
    // issues one tap and every chunk one patch (zero page past the block's range), so the number of
    // loads younger than tap t+1 depends on t alone (halo_younger).
    u32x4 fa[TM], fb[TN];
    if (nc > 0) {
#pragma unroll
        for (int i = 0; i < NPI; ++i) load_cell(0, i);
#pragma unroll
        for (int t = 0; t < NSTB; ++t) issue_b(0, t, t);
        store_patch();
        wait_vmcnt<NSTB - 1>();
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();
        read_frags(0, 0, fa, fb);
    }
    for (int ci = 0; ci < nc; ++ci) {
#pragma unroll
        for (int t = 0; t < NTAP; ++t) {
            wait_vmcnt_n(halo_younger_sp(t, NSTB, NPI, CSP));
            wait_lgkmcnt0();
            __builtin_amdgcn_s_barrier();
            if (t == NTAP - 1) {
                // every wave has read its last fragment of this chunk: stage the next chunk's patch (when the
                // footprint needs a cell per step of the chunk (k3: NPI == NTAP), the last one is loaded here)
                if (NPI == NTAP) load_cell(ci + 1, NTAP - 1);
                store_patch();
                wait_lgkmcnt0();
                __builtin_amdgcn_s_barrier();
            }
            __builtin_amdgcn_sched_barrier(0);
            // step g + NSTB reuses the stage of step g (read during the previous step, so free after the barrier)
            if (t + NSTB < NTAP)
                issue_b(ci, t + NSTB, t % NSTB);
            else
                issue_b(ci + 1, t + NSTB - NTAP, t % NSTB);
            // the next chunk's patch, one cell every CSP steps
            if (t % CSP == 0 && t / CSP < NPI && t < NTAP - 1) load_cell(ci + 1, t / CSP);
            if (t == (NPI - 1) * CSP) fence_loads();
            u32x4 na[TM], nb[TN];
            read_frags(t + 1 == NTAP ? 0 : t + 1, (t + 1) % NSTB, na, nb);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    acc[tm][tn] = mma16<bf16>(fb[tn], fa[tm], acc[tm][tn]);   // transposed accumulators
                }
            // the next step's reads (separate registers) alternate with this step's first MFMAs (measured:
            // a read burst ahead of the MFMAs, or reads every other MFMA, ran 2-6 % slower)
#pragma unroll
            for (int i = 0; i < TM + TN; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - (TM + TN), 0);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) fa[tm] = na[tm];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) fb[tn] = nb[tn];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    wait_vmcnt<0>();
    asm volatile("" ::"v"(fence_[0]), "v"(fence_[1]), "v"(fence_[2]), "v"(fence_[3]));
    __syncthreads();
    const int plane = P.OHg * P.OWg;
    auto rowm = [=](int row) {
        const int oy = ty0 + row / H::TW, ox = tx0 + row % H::TW;
        return (oy < P.OHg && ox < P.OWg) ? b * plane + oy * P.OWg + ox : -1;
    };
    conv_epilogue_rows_t<bf16, BM, BN, WM, WN, 512, decltype(rowm), false, false>(
        a, P, plane, 0, reinterpret_cast<float*>(smem), acc, rowm, (int)blockIdx.z);
}

// Halo-staged s^2-phase implicit GEMM for the stride-2 k5 transposed convolutions (ConvTranspose2d k5 s2 p2
// op1 forward and the matching Conv2d k5 s2 p2 input gradient), bf16.  Output phase (py, px) is a stride-1
// convolution of the input with NA x NC taps (3x3, 3x2, 2x3, 2x2 for the four phases), and all of a phase's
// taps read inside the input footprint of its output tile.  A block owns an 8 x 32 tile of one phase's
// output grid and all 128 output channels; per 64-channel chunk it stages the footprint ((8+NA-1) x
// (32+NC-1) pixels, eight planes of 8 channels, rows contiguous so one A fragment reads 16 consecutive
// cells) in LDS once and runs the NA*NC taps x two 32-channel halves out of it.  The weights stream through
// the same hand-ordered LDS-DMA ring as conv_halo_kernel (one 16-byte DMA per lane per step, NSTB-1 steps
// ahead); the next chunk's footprint is loaded into registers while the current one is consumed.
// (Variants measured slower and removed in round 5 -- one barrier per two steps, a ping-pong wave schedule,
// the four phases of a tile interleaved on one XCD, the 256-thread form, a 6-stage ring: DESIGN.md section 8,
// the round-4 tree of this file.)  conv_halo_quad_kernel (conv_quad.hip) runs all four phases of a tile from
// one staged footprint for the large 128-channel layers.
template <int NA, int NC, int BN_ = 128>
struct HaloPhCfg {
    static constexpr int TH = 8, TW = 32, BM = TH * TW, BN = BN_, WM = 4, WN = 2, CK = 64;
    static constexpr int NT = 512;
    // 16-byte weight DMAs per lane per step: NT lanes stage NT / 4 rows x 64 bytes per round; DPS rounds cover
    // the BN rows (BN = 192 on 512 lanes: rows 128..255 of the second round past the tile read the zero page
    // into unread cells)
    static constexpr int DPS = (4 * BN + NT - 1) / NT;
    static constexpr int PH = TH + NA - 1, PW = TW + NC - 1;
    static constexpr int NPOS = PH * PW;
    static constexpr int PLANE = (NPOS + 15) / 16 * 16;       // = 0 (mod 16): conflict-free fragment reads
    static constexpr int PATCH = 8 * PLANE * 16;
    static constexpr int NPI = (8 * NPOS + NT - 1) / NT;
    static constexpr int NTAP = NA * NC, NST = 2 * NTAP;       // steps per chunk: (half, tap)
    // NST % NSTB == 0: a step's stage is t % NSTB (a 6-stage ring measured slower: C2 8180 vs 8430 patches/s)
    static constexpr int NSTB = NST % 3 == 0 ? 3 : 2;
    static constexpr int BSTAGE = DPS * NT * 16;
    // BN > 128: register-direct epilogue only (no LDS staging buffer), see conv_epilogue_rows_t
    static constexpr int EPI = BN > 128 ? 0 : BM * (BN + 4) * 4;
    static constexpr int BYTES = (PATCH + NSTB * BSTAGE > EPI) ? PATCH + NSTB * BSTAGE : EPI;
    static_assert(NPI <= NST - NSTB, "the next chunk's footprint must retire before the chunk's last step");
};


// GATHER = false: the s^2-phase form (tap (ty, tx) reads footprint cell (NA-1-ty, NC-1-tx) from an origin
// NA-1 / NC-1 before dy0 / dx0).  GATHER = true: a stride-1 gather convolution (Conv2d k3 s1 forward): tap
// (ty, tx) = kernel (kh, kw) reads cell (ty, tx) from the origin dy0 = -pad.  n0: the tile's first output
// channel (grid y).
template <int NA, int NC, int BN_ = 128, bool GATHER = false, bool MPF = false>
__device__ __forceinline__ void conv_halo_phase_body(const ConvArgs& a, char* smem, int ph, int split, int bid,
                                                     int tiles_x, int tiles_y, int n0 = 0) {
    using H = HaloPhCfg<NA, NC, BN_>;
    constexpr int BM = H::BM, BN = H::BN, WM = H::WM, WN = H::WN, DPS = H::DPS, NT = H::NT;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int NPI = H::NPI, NTAP = H::NTAP, NST = H::NST, NSTB = H::NSTB;
    static_assert(WM * WN == NT / 64 && WTM == 2 * H::TW && H::BYTES <= 160 * 1024, "halo phase tile");
    char* const patch = smem;
    char* const bring = smem + H::PATCH;

    const PhaseDesc& P = a.ph[ph];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int per_img = tiles_x * tiles_y;
    const int b = bid / per_img;
    const int rt = bid - b * per_img;
    const int ty0 = (rt / tiles_x) * H::TH, tx0 = (rt % tiles_x) * H::TW;
    const int nch = a.Cin_pad / H::CK;
    const int per = (nch + a.ksplit - 1) / a.ksplit;
    const int c0 = split * per;
    const int nc = max(0, min(nch, c0 + per) - c0);
    const char* X = reinterpret_cast<const char*>(a.x);
    const int ld_b = a.x_ld * 2;

    // tap (ty, tx) reads input (qy + dy0 - ty, qx + dx0 - tx): the footprint starts NA-1 rows / NC-1 columns
    // before the tile's dy0/dx0 offset
    const int iyb = GATHER ? ty0 + P.dy0 : ty0 + P.dy0 - (NA - 1), ixb = GATHER ? tx0 + P.dx0 : tx0 + P.dx0 - (NC - 1);
    u32x4 pr_[NPI];
    unsigned fence_[4] = {0u, 0u, 0u, 0u};
    auto load_cell = [&](int ci, int i) {
        const bool real = ci < nc;
        const int cc = c0 + ci;
        const int q8 = tid + NT * i, g = (q8 >> 3) & 7, q = ((q8 >> 6) << 3) | (q8 & 7);
        const int pr = q / H::PW, pc = q - (q / H::PW) * H::PW;
        const int iy = iyb + pr, ix = ixb + pc;
        const bool in = real && q < H::NPOS && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
        const void* src = in ? (const void*)(X + ((b * a.IH + iy) * a.IW + ix) * ld_b + g * 16 + cc * (H::CK * 2))
                             : (const void*)cai_zero_page;
        pr_[i] = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(reinterpret_cast<uintptr_t>(src));
    };
    auto fence_loads = [&]() {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            asm volatile("" ::"v"(fence_[j]));
            fence_[j] = *reinterpret_cast<const __attribute__((address_space(1))) unsigned*>(
                reinterpret_cast<uintptr_t>(cai_zero_page + 16 * j));
        }
    };
    auto store_patch = [&]() {
#pragma unroll
        for (int i = 0; i < NPI; ++i) {
            const int q8 = tid + NT * i, g = (q8 >> 3) & 7, q = ((q8 >> 6) << 3) | (q8 & 7);
            if (q < H::NPOS) *reinterpret_cast<u32x4*>(patch + (g * H::PLANE + q) * 16) = pr_[i];
        }
    };

    const int bp = wid * 64 + lane;
    const int bn_ = bp >> 2, bs_ = (bp & 3) ^ (((bn_ >> 3) & 1) * 3);
    const char* Wrow = n0 + bn_ < a.Npad
                           ? reinterpret_cast<const char*>(a.w) + (P.w_off + (int64_t)(n0 + bn_) * a.Kp) * 2 + bs_ * 16
                           : nullptr;
    const char* Wrow2 = (DPS == 2 && n0 + NT / 4 + bn_ < a.Npad)
                            ? reinterpret_cast<const char*>(a.w) + (P.w_off + (int64_t)(n0 + NT / 4 + bn_) * a.Kp) * 2 +
                                  bs_ * 16
                            : nullptr;
    auto issue_b = [&](int ci, int t) {    // step t = (half t / NTAP, tap t % NTAP) of chunk ci into stage t % NSTB
        const int hf = t / NTAP, tap = t - hf * NTAP;
        const int koff = (tap * a.Cin_pad + (c0 + ci) * H::CK + hf * 32) * 2;
        const void* src = (Wrow && ci < nc) ? (const void*)(Wrow + koff) : (const void*)cai_zero_page;
        glds16_asm(src, bring + (t % NSTB) * H::BSTAGE + wid * 1024);
        if constexpr (DPS == 2) {
            const void* src2 = (Wrow2 && ci < nc) ? (const void*)(Wrow2 + koff) : (const void*)cai_zero_page;
            glds16_asm(src2, bring + (t % NSTB) * H::BSTAGE + NT * 16 + wid * 1024);
        }
    };

    const int g_ = lane >> 4, i16 = lane & 15;
    int apos[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * WTM + tm * 16 + i16;
        apos[tm] = (g_ * H::PLANE + (r / H::TW) * H::PW + (r % H::TW)) * 16;
    }
    int bpos[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
        const int n = wn * WTN + tn * 16 + i16;
        bpos[tn] = H::PATCH + (4 * n + (g_ ^ (((n >> 3) & 1) * 3))) * 16;
    }
    auto read_frags = [&](int t, u32x4 (&fa)[TM], u32x4 (&fb)[TN]) {
        const int hf = t / NTAP, tap = t - hf * NTAP;
        const int ty = tap / NC, tx = tap - (tap / NC) * NC;
        const int toff = GATHER ? (hf * 4 * H::PLANE + ty * H::PW + tx) * 16
                                : (hf * 4 * H::PLANE + (NA - 1 - ty) * H::PW + (NC - 1 - tx)) * 16;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) fa[tm] = *reinterpret_cast<const u32x4*>(smem + apos[tm] + toff);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
            fb[tn] = *reinterpret_cast<const u32x4*>(smem + bpos[tn] + (t % NSTB) * H::BSTAGE);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 fa[TM], fb[TN];
    // the step pipeline of conv_halo_kernel, NST steps per chunk
    if (nc > 0) {
#pragma unroll
        for (int i = 0; i < NPI; ++i) load_cell(0, i);
#pragma unroll
        for (int t = 0; t < NSTB; ++t) issue_b(0, t);
        store_patch();
        wait_vmcnt<DPS * (NSTB - 1)>();
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();
        read_frags(0, fa, fb);
    }
    for (int ci = 0; ci < nc; ++ci) {
#pragma unroll
        for (int t = 0; t < NST; ++t) {
            // halo_younger counts one DMA per younger step; DPS DMAs per step add (DPS - 1) per younger tap
            wait_vmcnt_n(halo_younger(t, NSTB, NPI) + (DPS - 1) * (NSTB - 2));
            wait_lgkmcnt0();
            __builtin_amdgcn_s_barrier();
            if (t == NST - 1) {
                store_patch();
                wait_lgkmcnt0();
                __builtin_amdgcn_s_barrier();
            }
            __builtin_amdgcn_sched_barrier(0);
            if (t + NSTB < NST)
                issue_b(ci, t + NSTB);
            else
                issue_b(ci + 1, t + NSTB - NST);
            if (t < NPI) load_cell(ci + 1, t);
            if (t == NPI - 1) fence_loads();
            u32x4 na[TM], nb[TN];
            read_frags(t + 1 == NST ? 0 : t + 1, na, nb);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = mma16<bf16>(fb[tn], fa[tm], acc[tm][tn]);   // transposed accumulators
#pragma unroll
            for (int i = 0; i < TM + TN; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - (TM + TN), 0);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) fa[tm] = na[tm];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) fb[tn] = nb[tn];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    wait_vmcnt<0>();
    asm volatile("" ::"v"(fence_[0]), "v"(fence_[1]), "v"(fence_[2]), "v"(fence_[3]));
    __syncthreads();
    const int plane = P.OHg * P.OWg;
    auto rowm = [=](int row) {
        const int oy = ty0 + row / H::TW, ox = tx0 + row % H::TW;
        return (oy < P.OHg && ox < P.OWg) ? b * plane + oy * P.OWg + ox : -1;
    };
    conv_epilogue_rows_t<bf16, BM, BN, WM, WN, NT, decltype(rowm), (BN > 128), false, MPF>(
        a, P, plane, n0, reinterpret_cast<float*>(smem), acc, rowm, ph * a.ksplit + split);
}


// grid: x = 4 x the output tiles of one phase, z = split (the split-K slab index of the epilogue).  Block
// order: phase-major, tiles XCD-remapped within a phase.
// 256 x 192 tiles of the halo phase / stride-1 kernels (192-, 384-, 768-channel layers).  The 96 accumulator
// registers leave no room for register-staged footprint cells or a second B fragment set, so:
//  * the next chunk's footprint goes global -> LDS by DMA into the other half of a double-buffered patch
//    (wave w owns plane w, one 64-pixel run per step of the chunk's first RUNS steps; pixels outside the
//    image or past the footprint read the zero page), no footprint store, no fence loads;
//  * the weight stage holds 256 rows (two DMAs per lane per step; rows past the layer read the zero page);
//  * MFMAs go column by column: the next step's A set is read during the first column, B fragment tn of the
//    next step is read into fb[tn] once column tn's MFMAs are issued.
// Waits: before step t reads step t+1's operands, the loads younger than tap t+1 are the 2 (NSTB - 2) tap
// DMAs of steps t+2-NSTB .. t-1 and the footprint runs of steps t+1-NSTB .. t-1.
template <int NA, int NC, int BN_ = 192>
struct HaloWideCfg {
    static constexpr int TH = 8, TW = 32, BM = TH * TW, BN = BN_, WM = 4, WN = 2, CK = 64;
    static constexpr int DPS = BN > 128 ? 2 : 1;               // weight DMAs per lane per step
    static constexpr int PH = TH + NA - 1, PW = TW + NC - 1;
    static constexpr int NPOS = PH * PW;
    static constexpr int PLANE = (NPOS + 63) / 64 * 64;      // whole 64-cell runs per plane, = 0 (mod 16)
    static constexpr int RUNS = PLANE / 64;
    static constexpr int PATCH = 8 * PLANE * 16;
    static constexpr int NTAP = NA * NC, NST = 2 * NTAP;
    static constexpr int NSTB = NST % 3 == 0 ? 3 : 2;
    static constexpr int BSTAGE = DPS * 128 * 32 * 2;
    static constexpr int EPI = BN > 128 ? 0 : BM * (BN + 4) * 4;   // BN = 128: LDS epilogue fallback
    static constexpr int BYTES = 2 * PATCH + NSTB * BSTAGE > EPI ? 2 * PATCH + NSTB * BSTAGE : EPI;
    static_assert(RUNS <= NST - NSTB, "the next chunk's footprint must retire before the chunk's last step");
};

__host__ __device__ constexpr int wide_younger(int t, int nstb, int runs, int dps) {
    const int lo = t + 1 - nstb > 0 ? t + 1 - nstb : 0;
    const int hi = t - 1 < runs - 1 ? t - 1 : runs - 1;
    return dps * (nstb - 2) + (hi >= lo ? hi - lo + 1 : 0);
}

template <int NA, int NC, bool GATHER, int BN_ = 192, bool MPF = false>
__device__ __forceinline__ void conv_halo_wide_body(const ConvArgs& a, char* smem, int ph, int split, int bid,
                                                    int tiles_x, int tiles_y, int n0) {
    using H = HaloWideCfg<NA, NC, BN_>;
    constexpr int BM = H::BM, BN = H::BN, WM = H::WM, WN = H::WN, DPS = H::DPS;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int RUNS = H::RUNS, NTAP = H::NTAP, NST = H::NST, NSTB = H::NSTB;
    static_assert(WM * WN == 8 && WTM == 2 * H::TW && H::BYTES <= 160 * 1024, "halo wide tile");
    char* const bring = smem + 2 * H::PATCH;

    const PhaseDesc& P = a.ph[ph];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int per_img = tiles_x * tiles_y;
    const int b = bid / per_img;
    const int rt = bid - b * per_img;
    const int ty0 = (rt / tiles_x) * H::TH, tx0 = (rt % tiles_x) * H::TW;
    const int nch = a.Cin_pad / H::CK;
    const int per = (nch + a.ksplit - 1) / a.ksplit;
    const int c0 = split * per;
    const int nc = max(0, min(nch, c0 + per) - c0);
    const char* X = reinterpret_cast<const char*>(a.x);
    const int ld_b = a.x_ld * 2;

    const int iyb = GATHER ? ty0 + P.dy0 : ty0 + P.dy0 - (NA - 1), ixb = GATHER ? tx0 + P.dx0 : tx0 + P.dx0 - (NC - 1);
    // footprint run j of this wave: plane wid (channels 8 wid .. 8 wid + 7 of the chunk), pixels 64 j + lane
    auto dma_run = [&](int ci, int j) {
        int q = j * 64 + lane;
        asm volatile("" : "+v"(q));    // recomputed per run: hoisted run addresses would spill
        const int pr = q / H::PW, pc = q - (q / H::PW) * H::PW;
        const int iy = iyb + pr, ix = ixb + pc;
        const bool in = ci < nc && q < H::NPOS && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
        const void* src = in ? (const void*)(X + ((b * a.IH + iy) * a.IW + ix) * ld_b + wid * 16 + (c0 + ci) * 128)
                             : (const void*)cai_zero_page;
        glds16_asm(src, smem + (ci & 1) * H::PATCH + (wid * H::PLANE + j * 64) * 16);
    };

    const int bp = wid * 64 + lane;
    const int bn_ = bp >> 2, bs_ = (bp & 3) ^ (((bn_ >> 3) & 1) * 3);
    const char* W0 = reinterpret_cast<const char*>(a.w) + P.w_off * 2 + bs_ * 16;
    const char* Wrow = n0 + bn_ < a.Npad ? W0 + (int64_t)(n0 + bn_) * a.Kp * 2 : nullptr;
    const char* Wrow2 = n0 + 128 + bn_ < a.Npad ? W0 + (int64_t)(n0 + 128 + bn_) * a.Kp * 2 : nullptr;
    auto issue_b = [&](int ci, int t) {    // step t = (half t / NTAP, tap t % NTAP) of chunk ci into stage t % NSTB
        const int hf = t / NTAP, tap = t - hf * NTAP;
        const int koff = (tap * a.Cin_pad + (c0 + ci) * H::CK + hf * 32) * 2;
        const bool real = ci < nc;
        glds16_asm((Wrow && real) ? (const void*)(Wrow + koff) : (const void*)cai_zero_page,
                   bring + (t % NSTB) * H::BSTAGE + wid * 1024);
        if constexpr (DPS == 2)
            glds16_asm((Wrow2 && real) ? (const void*)(Wrow2 + koff) : (const void*)cai_zero_page,
                       bring + (t % NSTB) * H::BSTAGE + 8192 + wid * 1024);
    };

    const int g_ = lane >> 4, i16 = lane & 15;
    int apos[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
        const int r = wm * WTM + tm * 16 + i16;
        apos[tm] = (g_ * H::PLANE + (r / H::TW) * H::PW + (r % H::TW)) * 16;
    }
    int bpos[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
        const int n = wn * WTN + tn * 16 + i16;
        bpos[tn] = (4 * n + (g_ ^ (((n >> 3) & 1) * 3))) * 16;
    }
    auto toff_of = [&](int t) {
        const int hf = t / NTAP, tap = t - hf * NTAP;
        const int ty = tap / NC, tx = tap - (tap / NC) * NC;
        return GATHER ? (hf * 4 * H::PLANE + ty * H::PW + tx) * 16
                      : (hf * 4 * H::PLANE + (NA - 1 - ty) * H::PW + (NC - 1 - tx)) * 16;
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    u32x4 fa[TM], fb[TN];
    if (nc > 0) {
#pragma unroll
        for (int j = 0; j < RUNS; ++j) dma_run(0, j);
#pragma unroll
        for (int t = 0; t < NSTB; ++t) issue_b(0, t);
        wait_vmcnt<DPS * (NSTB - 1)>();
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) fa[tm] = *reinterpret_cast<const u32x4*>(smem + apos[tm] + toff_of(0));
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) fb[tn] = *reinterpret_cast<const u32x4*>(bring + bpos[tn]);
    }
    for (int ci = 0; ci < nc; ++ci) {
        const char* cur = smem + (ci & 1) * H::PATCH;
        const char* nxt = smem + ((ci + 1) & 1) * H::PATCH;
#pragma unroll
        for (int t = 0; t < NST; ++t) {
            wait_vmcnt_n(wide_younger(t, NSTB, RUNS, DPS));
            wait_lgkmcnt0();
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (t + NSTB < NST)
                issue_b(ci, t + NSTB);
            else
                issue_b(ci + 1, t + NSTB - NST);
            if (t < RUNS) dma_run(ci + 1, t);
            const int t1 = t + 1 == NST ? 0 : t + 1;
            const char* abase = (t + 1 == NST ? nxt : cur) + toff_of(t1);
            const char* bst = bring + (t1 % NSTB) * H::BSTAGE;
            u32x4 na[TM];
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    acc[tm][tn] = mma16<bf16>(fb[tn], fa[tm], acc[tm][tn]);
                    if (tn == 0) na[tm] = *reinterpret_cast<const u32x4*>(abase + apos[tm]);
                }
                fb[tn] = *reinterpret_cast<const u32x4*>(bst + bpos[tn]);
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
            for (int tn = 1; tn < TN; ++tn) {
                __builtin_amdgcn_sched_group_barrier(0x008, TM, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) fa[tm] = na[tm];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    wait_vmcnt<0>();
    __syncthreads();
    const int plane = P.OHg * P.OWg;
    auto rowm = [=](int row) {
        const int oy = ty0 + row / H::TW, ox = tx0 + row % H::TW;
        return (oy < P.OHg && ox < P.OWg) ? b * plane + oy * P.OWg + ox : -1;
    };
    conv_epilogue_rows_t<bf16, BM, BN, WM, WN, 512, decltype(rowm), (BN > 128), false, MPF>(
        a, P, plane, n0, reinterpret_cast<float*>(smem), acc, rowm, ph * a.ksplit + split);
}


// grid y: output-channel tiles of BN (192-channel layers: BN = 192, one tile per 192 channels).
template <int BN>
__global__ __launch_bounds__(512, 1) void conv_halo_phase_kernel(const ConvArgs a, int tiles_x, int tiles_y) {
    constexpr bool DMA = BN > 128;
    constexpr int BYTES =
        DMA ? HaloWideCfg<3, 3, BN>::BYTES
            : (HaloPhCfg<3, 3>::BYTES > HaloPhCfg<2, 2>::BYTES ? HaloPhCfg<3, 3>::BYTES : HaloPhCfg<2, 2>::BYTES);
    static_assert(DMA ? (BYTES >= HaloWideCfg<3, 2, BN>::BYTES && BYTES >= HaloWideCfg<2, 3, BN>::BYTES &&
                         BYTES >= HaloWideCfg<2, 2, BN>::BYTES)
                      : (BYTES >= HaloPhCfg<3, 2>::BYTES && BYTES >= HaloPhCfg<2, 3>::BYTES),
                  "halo phase LDS");
    __shared__ __attribute__((aligned(16))) char smem[BYTES];
    const int n0 = blockIdx.y * BN;
    const int nt = gridDim.x >> 2;
    const int ph = blockIdx.x / nt;
    const int t = blockIdx.x - ph * nt;
    const int bid = (nt & 7) == 0 ? (t & 7) * (nt >> 3) + (t >> 3) : t;
    const int split = blockIdx.z;
    if constexpr (DMA) {
        switch (ph) {
            case 0: conv_halo_wide_body<3, 3, false, BN>(a, smem, 0, split, bid, tiles_x, tiles_y, n0); break;
            case 1: conv_halo_wide_body<3, 2, false, BN>(a, smem, 1, split, bid, tiles_x, tiles_y, n0); break;
            case 2: conv_halo_wide_body<2, 3, false, BN>(a, smem, 2, split, bid, tiles_x, tiles_y, n0); break;
            default: conv_halo_wide_body<2, 2, false, BN>(a, smem, 3, split, bid, tiles_x, tiles_y, n0); break;
        }
    } else {
        switch (ph) {    // k5 s2 p2 phases: (py, px) = (0,0) 3x3, (0,1) 3x2, (1,0) 2x3, (1,1) 2x2 taps
            case 0: conv_halo_phase_body<3, 3>(a, smem, 0, split, bid, tiles_x, tiles_y, n0); break;
            case 1: conv_halo_phase_body<3, 2>(a, smem, 1, split, bid, tiles_x, tiles_y, n0); break;
            case 2: conv_halo_phase_body<2, 3>(a, smem, 2, split, bid, tiles_x, tiles_y, n0); break;
            default: conv_halo_phase_body<2, 2>(a, smem, 3, split, bid, tiles_x, tiles_y, n0); break;
        }
    }
}


// Halo-staged stride-1 k3 p1 convolution (the 3x3 convs of cheng2020's residual / attention blocks and
// sub-pixel convs, conv3x3 layers/layers.py:38-49 / 86-91): the phase body with one phase of 3x3 taps.
// GATHER: Conv2d forward (tap = kernel (kh, kw), footprint origin -pad); otherwise the input gradient in the
// phase form of make_plan (flipped taps).  grid: x = output tiles (XCD-remapped), y = BN-channel tiles,
// z = split.
template <int BN, bool GATHER>
__global__ __launch_bounds__(512, 1) void conv_halo_s1_kernel(const ConvArgs a, int tiles_x, int tiles_y) {
    constexpr bool DMA = BN > 128;
    __shared__ __attribute__((aligned(16))) char smem[DMA ? HaloWideCfg<3, 3, BN>::BYTES : HaloPhCfg<3, 3, BN>::BYTES];
    const int nt = gridDim.x, t = blockIdx.x;
    const int bid = (nt & 7) == 0 ? (t & 7) * (nt >> 3) + (t >> 3) : t;
    if constexpr (DMA)
        conv_halo_wide_body<3, 3, GATHER, BN, !GATHER>(a, smem, 0, blockIdx.z, bid, tiles_x, tiles_y, blockIdx.y * BN);
    else
        conv_halo_phase_body<3, 3, BN, GATHER, !GATHER>(a, smem, 0, blockIdx.z, bid, tiles_x, tiles_y, blockIdx.y * BN);
}

// split-K reduce: out = epilogue(sum_s ws[ph*S + s][m][n]) in a fixed order
template <typename T>
__global__ __launch_bounds__(256) void conv_splitk_reduce_kernel(const ConvArgs a) {
    const int ph = blockIdx.y;
    const PhaseDesc P = ph == 0 ? a.ph[0] : (ph == 1 ? a.ph[1] : (ph == 2 ? a.ph[2] : a.ph[3]));
    const int plane = P.OHg * P.OWg;
    const int Mph = a.B * plane;
    const int VO = (a.y_vec && a.y_dtype == CAI_BF16) ? 8 : 4;
    const int cpr = (a.Cout + VO - 1) / VO;
    const int64_t total = (int64_t)Mph * cpr;
    const int64_t slab = (int64_t)a.ws_rows * a.ws_ld;
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(id / cpr);
        const int n = (int)(id - (int64_t)m * cpr) * VO;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const float* src = a.ws + ((int64_t)ph * a.ksplit) * slab + (int64_t)m * a.ws_ld + n;
        // split order fixed; loads in batches of 4 independent requests
        int s = 0;
        for (; s + 4 <= a.ksplit; s += 4) {
            f32x4 lo[4], hi[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                lo[j] = *reinterpret_cast<const f32x4*>(src + (s + j) * slab);
                hi[j] = VO == 8 ? *reinterpret_cast<const f32x4*>(src + (s + j) * slab + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[0] += lo[j][0]; v[1] += lo[j][1]; v[2] += lo[j][2]; v[3] += lo[j][3];
                v[4] += hi[j][0]; v[5] += hi[j][1]; v[6] += hi[j][2]; v[7] += hi[j][3];
            }
        }
        for (; s < a.ksplit; ++s) {
            const f32x4 lo = *reinterpret_cast<const f32x4*>(src + s * slab);
            v[0] += lo[0]; v[1] += lo[1]; v[2] += lo[2]; v[3] += lo[3];
            if (VO == 8) {
                const f32x4 hi = *reinterpret_cast<const f32x4*>(src + s * slab + 4);
                v[4] += hi[0]; v[5] += hi[1]; v[6] += hi[2]; v[7] += hi[3];
            }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int nn = n + e;
            const float bv = (a.bias && nn < a.Cout) ? a.bias[nn] : 0.f;
            v[e] = act_pre(a, v[e] + bv);
        }
        if (a.y_vec && !a.res && !a.mask_mode) {
            store_out_chunk<T, false>(a, P, plane, m, n, v, VO);
        } else if (a.y_vec) {
            store_out_chunk<T>(a, P, plane, m, n, v, VO);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (n + e < a.Cout) store_out_scalar<T>(a, P, plane, m, n + e, v[e]);
        }
    }
}

// ---------------------------------------------------------------------------
// weight packing: source [D0][D1][k][k] fp32 -> packed[ph][n][tap][c] (T)
// ---------------------------------------------------------------------------
struct PackArgs {
    const float* w;
    const float* mask;
    void* out;
    int D1, k;
    int n_is_d0;
    int Nreal, Creal, Cpad, Npad, Kp;
    int nphase;
    int ntaps[4], ntx[4], kh0[4], kw0[4], step;   // step = tap stride inside the kernel (s for phase, 1 for gather)
    int64_t off[4];
    int64_t item_begin;    // pack_many: first global 8-element item of this descriptor (item-mode descriptors)
    int items_pp;          // pack_many: 8-element items per phase (Npad * Kp / 8)
    int64_t row_begin;     // pack_many: first global row of this descriptor (row-mode conv descriptors)
    int64_t rows_total;    // pack_many: rows of the whole table (the same in every descriptor)
    int rowmode;           // 1: packed output rows (all phases) per block from an LDS copy of their sources
    int rpu;               // row mode: consecutive rows per work unit (as many as the LDS copy holds, <= 8)
    int edge;              // 1: edge-layer MFMA fragments (edge_frag.hpp), one item per fragment
    EdgeFragSpec es;
    int gdn;               // 1: GDN reparametrisation (w = gamma_raw, mask = beta_raw, out = gamma_op, D1 = C)
    float* gdn_beta;       //    beta output (C floats)
    float gdn_bb, gdn_gb, gdn_ped;
    // pack_many tile mode: 1 = this descriptor owns source tiles (and, pair = 1, also writes the next descriptor:
    // the other direction of the same weight, from the same LDS tile); 2 = written by the previous one's tiles
    int tilemode, pair;
    int td0, td1, tdp;     // tile: source dim-0 x dim-1 entries (k*k taps each); LDS row pitch (floats)
    int tstride;           // LDS floats per tap plane: td0 * tdp + 4 (planes start on different banks)
    int d0real, d1real;    // source extents (torch dims 0 / 1)
    int tn1;               // tiles along dim 1
    uint32_t mrl, mkk;     // ceil(2^32 / (td1 * k * k)), ceil(2^32 / (k * k)) (k > 1): divisions by multiply-high
    int64_t tile_begin;    // first global tile of this descriptor (non-decreasing over the table)
    int64_t tiles_total;   // tiles of the whole table (the same in every descriptor)
};

template <typename T>
__device__ __forceinline__ void pack_weight_body(const PackArgs& a, int ph) {
    const int64_t total = (int64_t)a.Npad * a.Kp;
    T* out = reinterpret_cast<T*>(a.out) + a.off[ph];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int n = (int)(i / a.Kp);
        const int kk = (int)(i - (int64_t)n * a.Kp);
        const int t = kk / a.Cpad, c = kk - t * a.Cpad;
        float v = 0.f;
        if (n < a.Nreal && c < a.Creal && t < a.ntaps[ph]) {
            const int kh = a.kh0[ph] + a.step * (t / a.ntx[ph]);
            const int kw = a.kw0[ph] + a.step * (t % a.ntx[ph]);
            const int d0 = a.n_is_d0 ? n : c, d1 = a.n_is_d0 ? c : n;
            const int64_t src = (((int64_t)d0 * a.D1 + d1) * a.k + kh) * a.k + kw;
            v = a.w[src];
            if (a.mask) v *= a.mask[src];
        }
        out[i] = from_f32<T>(v);
    }
}

template <typename T>
__global__ void pack_weight_kernel(const PackArgs a) {
    pack_weight_body<T>(a, blockIdx.z);
}

// all the convs of a model in one launch.  Conv descriptors go row by row: a block copies the fp32 source
// row of one output channel n (all input channels x k*k taps: contiguous for the forward direction, k*k
// runs for the transposed one) into LDS with coalesced loads, then writes the packed row of every phase
// with 16-byte stores.  Edge-fragment and GDN descriptors (and conv rows too long for the LDS copy) go by
// 8-element items, a thread per item.  Work units: rows_total row blocks, then blocks of 256 items.
#ifndef CAI_PACK_ROW_MAX
#define CAI_PACK_ROW_MAX 6144   // 24 KB: A/B 12288 / 6144 / 4096 / item-only -> 47 / 33 / 35 / 47 us (C2)
#endif
constexpr int PACK_ROW_MAX = CAI_PACK_ROW_MAX;   // source floats per row that fit the LDS copy
#ifndef CAI_PACK_ROWS_PER_UNIT
#define CAI_PACK_ROWS_PER_UNIT 8   // A/B: 1 = one row per work unit (the round-3 form)
#endif
constexpr int PACK_ROWS_PER_UNIT = CAI_PACK_ROWS_PER_UNIT;
#ifndef CAI_PACK_TILES
#define CAI_PACK_TILES 1   // A/B: 0 = row / item modes only (each direction reads its fp32 source itself)
#endif
constexpr bool PACK_TILES = CAI_PACK_TILES != 0;

template <typename T>
__device__ __forceinline__ void pack_item(const PackArgs* __restrict__ descs, int n, int64_t gi) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (descs[mid].item_begin <= gi) lo = mid; else hi = mid - 1;
    }
    const PackArgs& a = descs[lo];
    const int local = (int)(gi - a.item_begin);
    if constexpr (sizeof(T) == 2) {
        if (a.edge) {
            float v[8];
            edge_frag_values(a.w, a.es.C, a.es.N, a.es.k, a.es.p, a.es.emode, local, v);
            bf16x8 h;
#pragma unroll
            for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
            *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.out) + (int64_t)local * 8) = h;
            return;
        }
    }
    if (a.gdn) {
        // gdn_reparam_kernel's element rule for 8 consecutive gamma entries (and beta for i < C)
        const int C = a.D1;
        const int64_t CC = (int64_t)C * C;
        T* gop = reinterpret_cast<T*>(a.out);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int64_t i = (int64_t)local * 8 + e;
            if (i >= CC) break;
            const int r = (int)(i / C), c = (int)(i - (int64_t)r * C);
            const float lb = fmaxf(a.w[i], a.gdn_gb);
            const float v = lb * lb - a.gdn_ped;
            gop[i] = from_f32<T>(v);
            gop[CC + (int64_t)c * C + r] = from_f32<T>(v);
            if (i < C) {
                const float lbb = fmaxf(a.mask[i], a.gdn_bb);
                a.gdn_beta[i] = lbb * lbb - a.gdn_ped;
            }
        }
        return;
    }
    const int ph = local / a.items_pp;
    const int e0 = (local - ph * a.items_pp) * 8;
    const int nrow = e0 / a.Kp;
    const int kk0 = e0 - nrow * a.Kp;
    int t = kk0 / a.Cpad, c = kk0 - t * a.Cpad;
    const int ntaps = ph == 0 ? a.ntaps[0] : (ph == 1 ? a.ntaps[1] : (ph == 2 ? a.ntaps[2] : a.ntaps[3]));
    const int ntx = ph == 0 ? a.ntx[0] : (ph == 1 ? a.ntx[1] : (ph == 2 ? a.ntx[2] : a.ntx[3]));
    const int kh0 = ph == 0 ? a.kh0[0] : (ph == 1 ? a.kh0[1] : (ph == 2 ? a.kh0[2] : a.kh0[3]));
    const int kw0 = ph == 0 ? a.kw0[0] : (ph == 1 ? a.kw0[1] : (ph == 2 ? a.kw0[2] : a.kw0[3]));
    const int64_t off = ph == 0 ? a.off[0] : (ph == 1 ? a.off[1] : (ph == 2 ? a.off[2] : a.off[3]));
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float x = 0.f;
        if (nrow < a.Nreal && c < a.Creal && t < ntaps) {
            const int ty = t / ntx;
            const int kh = kh0 + a.step * ty, kw = kw0 + a.step * (t - ty * ntx);
            const int d0 = a.n_is_d0 ? nrow : c, d1 = a.n_is_d0 ? c : nrow;
            const int64_t src = (((int64_t)d0 * a.D1 + d1) * a.k + kh) * a.k + kw;
            x = a.w[src];
            if (a.mask) x *= a.mask[src];
        }
        v[e] = x;
        if (++c == a.Cpad) { c = 0; ++t; }
    }
    T* out = reinterpret_cast<T*>(a.out) + off + e0;
    if constexpr (sizeof(T) == 2) {
        bf16x8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
        *reinterpret_cast<bf16x8*>(out) = h;
    } else {
        *reinterpret_cast<f32x4*>(out) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(out + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
}

// TO[ph * 64 + t]: the source tap (kernel offset kh * k + kw) of packed tap t of phase ph, filled once per unit
// (k <= 7: <= 49 taps) so the packing loop reads S without an integer division per element.  A unit is `cnt`
// consecutive output rows n0 .. n0 + cnt - 1 (a.rpu of them): their sources go to LDS in one round of loads and
// one barrier -- a unit per row left cheng2020's 1728-float rows latency-bound (267 us per C4 step).
template <typename T>
__device__ __forceinline__ void pack_rows(const PackArgs& a, int n0, int cnt, float* S, int* TO) {
    const int KK = a.k * a.k;
    const int nsrc = a.Creal * KK;
    const int tot = cnt * nsrc;
    {
        // PACK_LD independent loads in flight per thread
        constexpr int PACK_LD = 16;
        for (int i0 = threadIdx.x; i0 < tot; i0 += PACK_LD * blockDim.x) {
            float v[PACK_LD];
#pragma unroll
            for (int j = 0; j < PACK_LD; ++j) {
                const int i = min(i0 + j * (int)blockDim.x, tot - 1);
                const int r = i / nsrc, ii = i - r * nsrc;
                const int n = n0 + r;
                const int c = ii / KK, tap = ii - c * KK;
                const int64_t src = a.n_is_d0 ? (int64_t)n * a.D1 * KK + ii : ((int64_t)c * a.D1 + n) * KK + tap;
                v[j] = n < a.Nreal ? a.w[src] : 0.f;
                if (a.mask && n < a.Nreal) v[j] *= a.mask[src];
            }
#pragma unroll
            for (int j = 0; j < PACK_LD; ++j)
                if (i0 + j * (int)blockDim.x < tot) S[i0 + j * blockDim.x] = v[j];
        }
    }
    for (int idx = threadIdx.x; idx < a.nphase * 64; idx += blockDim.x) {
        const int ph = idx >> 6, t = idx & 63;
        const int ntx = ph == 0 ? a.ntx[0] : (ph == 1 ? a.ntx[1] : (ph == 2 ? a.ntx[2] : a.ntx[3]));
        const int kh0 = ph == 0 ? a.kh0[0] : (ph == 1 ? a.kh0[1] : (ph == 2 ? a.kh0[2] : a.kh0[3]));
        const int kw0 = ph == 0 ? a.kw0[0] : (ph == 1 ? a.kw0[1] : (ph == 2 ? a.kw0[2] : a.kw0[3]));
        const int ty = t / ntx;
        TO[idx] = (kh0 + a.step * ty) * a.k + kw0 + a.step * (t - ty * ntx);
    }
    __syncthreads();
    const int nch = a.Kp / 8;
    for (int ph = 0; ph < a.nphase; ++ph) {
        const int ntaps = ph == 0 ? a.ntaps[0] : (ph == 1 ? a.ntaps[1] : (ph == 2 ? a.ntaps[2] : a.ntaps[3]));
        const int64_t off = ph == 0 ? a.off[0] : (ph == 1 ? a.off[1] : (ph == 2 ? a.off[2] : a.off[3]));
        const int* TOp = TO + ph * 64;
        for (int idx = threadIdx.x; idx < cnt * nch; idx += blockDim.x) {
            const int r = idx / nch, ch = idx - r * nch;
            const int n = n0 + r;
            T* out = reinterpret_cast<T*>(a.out) + off + (int64_t)n * a.Kp;
            const float* Sr = S + r * nsrc;
            const int e0 = ch * 8;
            int t = e0 / a.Cpad, c = e0 - t * a.Cpad;   // fp32 (Cpad % 4 == 0): the 8 may span two taps
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float x = 0.f;
                if (n < a.Nreal && c < a.Creal && t < ntaps) x = Sr[c * KK + TOp[t]];
                v[e] = x;
                if (++c == a.Cpad) { c = 0; ++t; }
            }
            if constexpr (sizeof(T) == 2) {
                bf16x8 h;
#pragma unroll
                for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
                *reinterpret_cast<bf16x8*>(out + e0) = h;
            } else {
                *reinterpret_cast<f32x4*>(out + e0) = f32x4{v[0], v[1], v[2], v[3]};
                *reinterpret_cast<f32x4*>(out + e0 + 4) = f32x4{v[4], v[5], v[6], v[7]};
            }
        }
    }
    __syncthreads();   // the next unit reuses S
}

// Tile mode (round 4): a unit is a td0 x td1 tile of the SOURCE [D0][D1][k*k], loaded once with coalesced runs
// of td1*k*k floats (16-byte loads where the rows allow) and kept in LDS tap-major, S[tap][a][b] (row pitch
// tdp = td1 + 4, plane stride td0 * tdp + 4).  Both packed directions of the
// weight are written from it: the one whose rows are dim 0 (rows a, 16-byte channel chunks read as vectors along
// b) and the one whose rows are dim 1 (rows b, chunks gathered along a).  Every packed element of a tile's rows
// and channels is written, padding included: rows < Npad, and each row as ceil(Kp / Cpad) slots of Cpad channels
// (slot t < ntaps[ph] holds source tap TO[ph][t]; the rest, and channels >= Creal, are zero).  The row mode read
// the source once per direction, a unit of <= 8 rows at a time (a third of cheng2020's step in the pack launch
// ran at 1.8 TB/s).
constexpr int PACK_TILE_FLOATS = 10404;   // 41.6 KB: 32 x 32 tiles of 3x3, 16 x 16 of 5x5, 128 x 64 of 1x1
constexpr int PACK_LDS_FLOATS = PACK_TILE_FLOATS > PACK_ROW_MAX ? PACK_TILE_FLOATS : PACK_ROW_MAX;

__device__ __forceinline__ void pack_taps(const PackArgs& a, int* TO) {
    for (int idx = threadIdx.x; idx < a.nphase * 64; idx += blockDim.x) {
        const int ph = idx >> 6, t = idx & 63;
        const int ntx = ph == 0 ? a.ntx[0] : (ph == 1 ? a.ntx[1] : (ph == 2 ? a.ntx[2] : a.ntx[3]));
        const int kh0 = ph == 0 ? a.kh0[0] : (ph == 1 ? a.kh0[1] : (ph == 2 ? a.kh0[2] : a.kh0[3]));
        const int kw0 = ph == 0 ? a.kw0[0] : (ph == 1 ? a.kw0[1] : (ph == 2 ? a.kw0[2] : a.kw0[3]));
        const int ty = t / ntx;
        TO[idx] = (kh0 + a.step * ty) * a.k + kw0 + a.step * (t - ty * ntx);
    }
}

template <typename T>
__device__ __forceinline__ void pack_tile_store(const PackArgs& X, int ph, int n, int e0, const float (&v)[16 / sizeof(T)]) {
    const int64_t off = ph == 0 ? X.off[0] : (ph == 1 ? X.off[1] : (ph == 2 ? X.off[2] : X.off[3]));
    T* out = reinterpret_cast<T*>(X.out) + off + (int64_t)n * X.Kp + e0;
    if constexpr (sizeof(T) == 2) {
        bf16x8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
        *reinterpret_cast<bf16x8*>(out) = h;
    } else {
        *reinterpret_cast<f32x4*>(out) = f32x4{v[0], v[1], v[2], v[3]};
    }
}

// rows = source dim 0 (n = d0, channel c = d1): chunk reads are 16-byte LDS vectors along b
template <typename T>
__device__ __forceinline__ void pack_tile_rows0(const PackArgs& X, int d0_0, int d1_0, const PackArgs& G, const float* S,
                                                const int* TO) {
    constexpr int VW = 16 / sizeof(T);
    const int td0 = G.td0, tdp = G.tdp, nch = G.td1 / VW;
    const int nslot = (X.Kp + X.Cpad - 1) / X.Cpad;
    const int cnt = X.nphase * td0 * nslot * nch;
    for (int w = threadIdx.x; w < cnt; w += blockDim.x) {
        const int ch = w % nch, r1 = w / nch, t = r1 % nslot, r2 = r1 / nslot, a = r2 % td0, ph = r2 / td0;
        const int n = d0_0 + a, c0 = d1_0 + ch * VW, e0 = t * X.Cpad + c0;
        if (n >= X.Npad || c0 >= X.Cpad || e0 >= X.Kp) continue;
        const int ntaps = ph == 0 ? X.ntaps[0] : (ph == 1 ? X.ntaps[1] : (ph == 2 ? X.ntaps[2] : X.ntaps[3]));
        float v[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) v[e] = 0.f;
        if (n < X.Nreal && t < ntaps) {
            const float* s = S + TO[ph * 64 + t] * G.tstride + a * tdp + ch * VW;
#pragma unroll
            for (int q = 0; q < VW / 4; ++q) {
                const f32x4 f = *reinterpret_cast<const f32x4*>(s + 4 * q);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[4 * q + e] = c0 + 4 * q + e < X.Creal ? f[e] : 0.f;
            }
        }
        pack_tile_store<T>(X, ph, n, e0, v);
    }
}

// rows = source dim 1 (n = d1, channel c = d0): consecutive lanes take a row's consecutive chunks, then rows
template <typename T>
__device__ __forceinline__ void pack_tile_rows1(const PackArgs& X, int d0_0, int d1_0, const PackArgs& G, const float* S,
                                                const int* TO) {
    constexpr int VW = 16 / sizeof(T);
    const int td0 = G.td0, td1 = G.td1, tdp = G.tdp, nch = td0 / VW;
    const int nslot = (X.Kp + X.Cpad - 1) / X.Cpad;
    const int cnt = X.nphase * nslot * td1 * nch;
    for (int w = threadIdx.x; w < cnt; w += blockDim.x) {
        const int ch = w % nch, r1 = w / nch, b = r1 % td1, r2 = r1 / td1, t = r2 % nslot, ph = r2 / nslot;
        const int n = d1_0 + b, c0 = d0_0 + ch * VW, e0 = t * X.Cpad + c0;
        if (n >= X.Npad || c0 >= X.Cpad || e0 >= X.Kp) continue;
        const int ntaps = ph == 0 ? X.ntaps[0] : (ph == 1 ? X.ntaps[1] : (ph == 2 ? X.ntaps[2] : X.ntaps[3]));
        float v[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) v[e] = 0.f;
        if (n < X.Nreal && t < ntaps) {
            const float* s = S + TO[ph * 64 + t] * G.tstride + ch * VW * tdp + b;
#pragma unroll
            for (int e = 0; e < VW; ++e) v[e] = c0 + e < X.Creal ? s[e * tdp] : 0.f;
        }
        pack_tile_store<T>(X, ph, n, e0, v);
    }
}

template <typename T>
__device__ __forceinline__ void pack_tile(const PackArgs* __restrict__ descs, int lo, int64_t tl, float* S, int* TO) {
    const PackArgs& A = descs[lo];
    const int i0 = (int)(tl / A.tn1), i1 = (int)(tl - (int64_t)i0 * A.tn1);
    const int td0 = A.td0, td1 = A.td1, tdp = A.tdp;
    const int d0_0 = i0 * td0, d1_0 = i1 * td1;
    const int KK = A.k * A.k, RL = td1 * KK, tot = td0 * RL;
    pack_taps(A, TO);
    if (A.pair) pack_taps(descs[lo + 1], TO + 256);
    const int TS = A.tstride;
    const int lim = (A.d1real - d1_0) * KK;   // valid source floats of a tile row
    if (((A.D1 * KK) & 3) == 0 && (((uintptr_t)A.w | (uintptr_t)A.mask) & 15) == 0) {
        // 16-byte loads: a tile row is td1*k*k floats (a multiple of 4) starting 16-byte aligned
        constexpr int LD = 8;   // independent 16-byte loads in flight per thread
        const int tot4 = tot >> 2;
        for (int q0 = threadIdx.x; q0 < tot4; q0 += LD * blockDim.x) {
            f32x4 v[LD];
            int aa[LD], rr[LD];
#pragma unroll
            for (int j = 0; j < LD; ++j) {
                const int q = q0 + j * (int)blockDim.x, l = 4 * q;
                const int a = (int)__umulhi((unsigned)l, A.mrl), r = l - a * RL;
                aa[j] = q < tot4 ? a : -1;
                rr[j] = r;
                v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (q >= tot4 || d0_0 + a >= A.d0real) continue;
                const int64_t src = ((int64_t)(d0_0 + a) * A.D1 + d1_0) * KK + r;
                if (r + 4 <= lim) {
                    v[j] = *reinterpret_cast<const f32x4*>(A.w + src);
                    if (A.mask) v[j] *= *reinterpret_cast<const f32x4*>(A.mask + src);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (r + e < lim) v[j][e] = A.mask ? A.w[src + e] * A.mask[src + e] : A.w[src + e];
                }
            }
#pragma unroll
            for (int j = 0; j < LD; ++j) {
                if (aa[j] < 0) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = rr[j] + e;
                    const int b = KK == 1 ? r : (int)__umulhi((unsigned)r, A.mkk), tap = r - b * KK;
                    S[tap * TS + aa[j] * tdp + b] = v[j][e];
                }
            }
        }
    } else {
        constexpr int LD = 8;   // independent loads in flight per thread
        for (int l0 = threadIdx.x; l0 < tot; l0 += LD * blockDim.x) {
            float v[LD];
            int dst[LD];
#pragma unroll
            for (int j = 0; j < LD; ++j) {
                const int l = l0 + j * (int)blockDim.x;
                const int a = (int)__umulhi((unsigned)l, A.mrl), r = l - a * RL;
                const int b = KK == 1 ? r : (int)__umulhi((unsigned)r, A.mkk), tap = r - b * KK;   // 2^32 / 1 overflows
                const bool ok = l < tot && d0_0 + a < A.d0real && r < lim;
                const int64_t src = ((int64_t)(d0_0 + a) * A.D1 + d1_0) * KK + r;
                float x = ok ? A.w[src] : 0.f;
                if (A.mask && ok) x *= A.mask[src];
                v[j] = x;
                dst[j] = l < tot ? tap * TS + a * tdp + b : -1;
            }
#pragma unroll
            for (int j = 0; j < LD; ++j)
                if (dst[j] >= 0) S[dst[j]] = v[j];
        }
    }
    __syncthreads();
    if (A.n_is_d0)
        pack_tile_rows0<T>(A, d0_0, d1_0, A, S, TO);
    else
        pack_tile_rows1<T>(A, d0_0, d1_0, A, S, TO);
    if (A.pair) {
        const PackArgs& B = descs[lo + 1];
        if (B.n_is_d0)
            pack_tile_rows0<T>(B, d0_0, d1_0, A, S, TO + 256);
        else
            pack_tile_rows1<T>(B, d0_0, d1_0, A, S, TO + 256);
    }
    __syncthreads();   // the next unit reuses S and TO
}

template <typename T>
__global__ __launch_bounds__(256) void pack_many_kernel(const PackArgs* __restrict__ descs, int n, int64_t total) {
    __shared__ __attribute__((aligned(16))) float S[PACK_LDS_FLOATS];
    __shared__ int TO[2 * 4 * 64];
    const int64_t Tt = descs[0].tiles_total;
    const int64_t R = descs[0].rows_total;
    const int64_t I = total - Tt - R;
    const int64_t units = Tt + R + (I + 255) / 256;
    for (int64_t u0 = blockIdx.x; u0 < units; u0 += gridDim.x) {
        if (u0 < Tt) {
            int lo = 0, hi = n - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (descs[mid].tile_begin <= u0) lo = mid; else hi = mid - 1;
            }
            pack_tile<T>(descs, lo, u0 - descs[lo].tile_begin, S, TO);
            continue;
        }
        const int64_t u = u0 - Tt;
        if (u < R) {
            int lo = 0, hi = n - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (descs[mid].row_begin <= u) lo = mid; else hi = mid - 1;
            }
            const PackArgs& d = descs[lo];
            const int n0 = (int)(u - d.row_begin) * d.rpu;
            pack_rows<T>(d, n0, min(d.rpu, d.Npad - n0), S, TO);
        } else {
            const int64_t gi = (u - R) * 256 + threadIdx.x;
            if (gi < I) pack_item<T>(descs, n, gi);
        }
    }
}

template <typename T>
__global__ void pack_nchw_kernel(const float* __restrict__ x, int B, int C, int HW, T* __restrict__ out, int ld) {
    const int64_t total = (int64_t)B * HW * ld;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / ld;
        const int c = (int)(i - p * ld);
        const int64_t b = p / HW, s = p - b * HW;
        out[i] = from_f32<T>(c < C ? x[(b * C + c) * HW + s] : 0.f);
    }
}

// ---------------------------------------------------------------------------
// wgrad
// ---------------------------------------------------------------------------
struct WgradArgs {
    const void* g;
    int g_ld, Ng;
    const void* x;
    int x_ld, Cq_pad, in_abs, in_sq;
    int B, Hg, Wg, Hx, Wx;
    int k, s, p;
    int ncols;
    int64_t M;
    int64_t split_len;
    float* ws;
    int ctiles, rtiles, nsub, grp_len, chunk;
    int nsplit;        // glds kernel: pixel splits (split_len pixels each)
    float* bws;        // glds kernel: per-split bias partials [nsplit][Ng] (NULL: none)
    // ConvTranspose2d bias gradient from the X operand (WG_TBIAS): the column sums of the taps
    // (tb_kh0 + a, tb_kw0 + b), a, b < tb_s, which together visit every output pixel exactly once;
    // partials [nsplit * tb_s^2][nbias]
    int tb_kh0, tb_kw0, tb_s, nbias;
};

constexpr int WG_CHUNK = 1024;   // max pixels per L2-resident wgrad chunk (multiple of 64)

// bijective XCD remap (cdna_hip_programming.md T1): physical workgroup id ->
// logical id such that logical ids [x*q, (x+1)*q) run on one XCD
__device__ __forceinline__ int xcd_remap(int wgid, int nwg) {
    const int xcd = wgid & 7, idx = wgid >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// LDS byte offset of 16-byte slot `slot` of row `row` in a [32][256 B] bf16 image
// read by ds_read_b64_tr_b16 (rows 8g+q of a half-wave land on distinct slots)
__device__ __forceinline__ int trswz(int row, int slot) {
    return row * 256 + ((slot ^ (((row & 3) << 1) | (((row >> 3) & 1) << 3))) << 4);
}

typedef short __attribute__((address_space(3))) * lds_s16_ptr;

__device__ __forceinline__ s16x4 ds_tr16(const char* base, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(base + byte_off));
}

template <typename T>
__global__ __launch_bounds__(NT, 2) void wgrad_kernel(const WgradArgs a) {
    constexpr int VEC = OpT<T>::VEC;
    constexpr int BKP = sizeof(T) == 2 ? 64 : 32;  // pixels per K-step
    constexpr int ROWB = 128 * (int)sizeof(T);    // bytes per LDS row (128 channels)
    constexpr int CPR = ROWB / 16;                // 16-byte chunks per row
    constexpr int CH = BKP * CPR / NT;            // chunks per thread per operand
    constexpr int OPB = BKP * ROWB;               // bytes per operand tile
    __shared__ __attribute__((aligned(16))) char smem[4 * OPB];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    // Pixel partition (speed only -- any placement is correct): workgroups
    // b and b+8 share an XCD, so group g = b % 8 owns pixel range g of 8; its
    // workgroups (all tap/channel tiles x nsub) walk that range in 1024-pixel
    // chunks, sub k taking chunks k, k+nsub, ...  The tiles working on one
    // chunk gather the same pixels at about the same time from one L2.
    const int grp = (int)(blockIdx.x & 7);
    const int w = (int)(blockIdx.x >> 3);
    const int ctile = w % a.ctiles;
    const int rtile = (w / a.ctiles) % a.rtiles;
    const int sub = w / (a.ctiles * a.rtiles);
    const int split = grp * a.nsub + sub;
    const int c0 = ctile * 128;        // column tile (tap, q)
    const int r0 = rtile * 128;        // row tile (G channel)
    // pixel indices fit in 32 bits (M < 2^31 is checked on the host)
    const int gbeg = min((int)a.M, grp * a.grp_len);
    const int gend = min((int)a.M, gbeg + a.grp_len);
    const int CHK = a.chunk;
    const int nchunk = (gend - gbeg + CHK - 1) / CHK;
    int nsteps = 0;   // 64-pixel steps of this workgroup
    for (int c = sub; c < nchunk; c += a.nsub)
        nsteps += (min(gend, gbeg + (c + 1) * CHK) - (gbeg + c * CHK) + BKP - 1) / BKP;
    if (nsteps == 0) {
        // empty split: still write zeros so the reduce reads defined data
        for (int id = tid; id < 128 * 128; id += NT) {
            const int rr = r0 + id / 128, cc = c0 + (id & 127);
            if (rr < a.Ng && cc < a.ncols) a.ws[((int64_t)split * a.Ng + rr) * a.ncols + cc] = 0.f;
        }
        return;
    }
    const int SPC = CHK / BKP;   // steps per chunk
    // first pixel of step st (this sub's chunks in order; the last chunk may be short)
    auto step_base = [&](int st) { return gbeg + (sub + (st / SPC) * a.nsub) * CHK + (st % SPC) * BKP; };

    // this thread's fixed chunk column
    const int cc = tid % CPR;
    const int gcol = r0 + cc * VEC;                 // G channel of the chunk
    const int xcol = c0 + cc * VEC;                 // X (tap, q) column of the chunk
    const int xt = xcol / a.Cq_pad, xq = xcol - xt * a.Cq_pad;
    const int xkh = xt / a.k, xkw = xt - xkh * a.k;
    const bool xvalid = xcol < a.ncols;
    const bool gvalid = gcol < a.Ng;
    const int plane = a.Hg * a.Wg;
    const gptr<T> G = to_global<T>(a.g);
    const gptr<T> X = to_global<T>(a.x);
    const u32x4 zero = u32x4{0u, 0u, 0u, 0u};
    U4<CH> rg0, rx0;

#define WG_LOAD(MB, RG, RX)                                                                                  \
    {                                                                                                        \
        _Pragma("unroll") for (int i = 0; i < CH; ++i) {                                                     \
            const int row = i * (NT / CPR) + tid / CPR;                                                      \
            const int m = (MB) + row;                                                                        \
            const bool mok = m < gend && (m - gbeg) / CHK == ((MB) - gbeg) / CHK;                            \
            const int mm = mok ? m : gbeg;                                                                   \
            const u32x4 gv = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(              \
                G + (int64_t)mm * a.g_ld + (gvalid ? gcol : 0));                                             \
            RG.v[i] = (mok && gvalid) ? gv : zero;                                                           \
            const int b = mm / plane;                                                                        \
            const int r = mm - b * plane;                                                                    \
            const int j = r / a.Wg;                                                                          \
            const int iy = j * a.s - a.p + xkh, ix = (r - j * a.Wg) * a.s - a.p + xkw;                       \
            const bool ok = mok && xvalid && (unsigned)iy < (unsigned)a.Hx && (unsigned)ix < (unsigned)a.Wx; \
            const int64_t off = ok ? (((int64_t)b * a.Hx + iy) * a.Wx + ix) * a.x_ld + xq : 0;               \
            u32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(X + off);            \
            if (a.in_abs) v = abs_chunk(v, sizeof(T));                                                       \
            if (a.in_sq) v = sq_chunk<T>(v);                                                                 \
            RX.v[i] = ok ? v : zero;                                                                         \
        }                                                                                                    \
    }
#define WG_STORE(BUF, RG, RX)                                                                                \
    {                                                                                                        \
        char* Gs_ = smem + (BUF) * 2 * OPB;                                                                  \
        char* Xs_ = Gs_ + OPB;                                                                               \
        _Pragma("unroll") for (int i = 0; i < CH; ++i) {                                                     \
            const int row = i * (NT / CPR) + tid / CPR;                                                      \
            const int off = (sizeof(T) == 2) ? trswz(row, cc) : row * ROWB + cc * 16;                        \
            *reinterpret_cast<u32x4*>(Gs_ + off) = RG.v[i];                                                  \
            *reinterpret_cast<u32x4*>(Xs_ + off) = RX.v[i];                                                  \
        }                                                                                                    \
    }

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#define WG_COMPUTE(BUF)                                                                                      \
    {                                                                                                        \
        const char* Gs = smem + (BUF) * 2 * OPB;                                                             \
        const char* Xs = Gs + OPB;                                                                           \
        if constexpr (sizeof(T) == 2) {                                                                      \
            const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;                          \
            _Pragma("unroll") for (int ks = 0; ks < BKP / 32; ++ks) {                                        \
                const int r0_ = 32 * ks + 8 * g_ + q_;                                                       \
                u32x4 fb[4];                                                                                 \
                _Pragma("unroll") for (int t = 0; t < 4; ++t) {                                              \
                    const int colB = wn * 64 + t * 16 + 4 * p4;                                              \
                    s16x4 b0 = ds_tr16(Xs, trswz(r0_, colB >> 3) + ((colB & 7) << 1));                      \
                    s16x4 b1 = ds_tr16(Xs, trswz(r0_ + 4, colB >> 3) + ((colB & 7) << 1));                  \
                    s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};                     \
                    fb[t] = __builtin_bit_cast(u32x4, bv);                                                   \
                }                                                                                            \
                _Pragma("unroll") for (int tm = 0; tm < 4; ++tm) {                                           \
                    const int colA = wm * 64 + tm * 16 + 4 * p4;                                             \
                    s16x4 a0 = ds_tr16(Gs, trswz(r0_, colA >> 3) + ((colA & 7) << 1));                      \
                    s16x4 a1 = ds_tr16(Gs, trswz(r0_ + 4, colA >> 3) + ((colA & 7) << 1));                  \
                    s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};                     \
                    const u32x4 fa = __builtin_bit_cast(u32x4, av);                                          \
                    _Pragma("unroll") for (int tn = 0; tn < 4; ++tn)                                         \
                        acc[tm][tn] = mma16<bf16>(fa, fb[tn], acc[tm][tn]);                                  \
                }                                                                                            \
            }                                                                                                \
        } else {                                                                                             \
            const float* Gf = reinterpret_cast<const float*>(Gs);                                            \
            const float* Xf = reinterpret_cast<const float*>(Xs);                                           \
            _Pragma("unroll") for (int ks = 0; ks < BKP / 4; ++ks) {                                         \
                const int row = ks * 4 + (lane >> 4);                                                        \
                float fa[4], fb[4];                                                                          \
                _Pragma("unroll") for (int t = 0; t < 4; ++t) {                                              \
                    fa[t] = Gf[row * 128 + wm * 64 + t * 16 + (lane & 15)];                                  \
                    fb[t] = Xf[row * 128 + wn * 64 + t * 16 + (lane & 15)];                                  \
                }                                                                                            \
                _Pragma("unroll") for (int tm = 0; tm < 4; ++tm)                                             \
                    _Pragma("unroll") for (int tn = 0; tn < 4; ++tn)                                         \
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[tm], fb[tn], acc[tm][tn], 0, 0, 0); \
            }                                                                                                \
        }                                                                                                    \
    }

    // one register set in flight: tile st+1 loads while tile st is computed
    // (64-pixel steps keep 32 MFMAs per wave between barriers)
    WG_LOAD(step_base(0), rg0, rx0);
    WG_STORE(0, rg0, rx0);
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
        const bool more = st + 1 < nsteps;
        if (more) WG_LOAD(step_base(st + 1), rg0, rx0);
        WG_COMPUTE(st & 1);
        if (more) WG_STORE((st + 1) & 1, rg0, rx0);
        __syncthreads();
    }
#undef WG_LOAD
#undef WG_STORE
#undef WG_COMPUTE

    float* out = a.ws + (int64_t)split * a.Ng * a.ncols;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) {
            const int col = c0 + wn * 64 + tn * 16 + (lane & 15);
            if (col >= a.ncols) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = r0 + wm * 64 + tm * 16 + (lane >> 4) * 4 + r;
                if (row < a.Ng) out[(int64_t)row * a.ncols + col] = acc[tm][tn][r];
            }
        }
}

// ---------------------------------------------------------------------------
// Latent-size weight gradients (M = B*H*W <= 1024 G pixels: the hyper branch's 4x4 / 8x8 latents): one
// launch writing dW (and the bias gradient) in torch layout -- no pixel-split partial
// slabs and no reduce launch.  dW has few rows of K here (a few thousand pixels) but many output columns
// (taps x channels), so the output is tiled finely instead: a block owns 64 G channels x 64 X columns of
// one tap, and its 8 waves split the pixels eight ways.  Per 32-pixel step a wave stages its own G and X
// tiles ([32 px][64 ch] bf16, XOR-swizzled 16-byte slots) in a private LDS region -- no block barrier in
// the loop -- and reads the MFMA fragments (pixels as K) with ds_read_b64_tr_b16, the next step's loads
// already in flight (two register sets; buffer loads: padding taps and pixels past M read 0).  The 8
// partial tiles are summed in wave order in LDS (deterministic).  Bias gradient: Conv2d's is the column
// sums of G, accumulated by the (tap 0, q 0) blocks from the chunks they stage; ConvTranspose2d's (column
// sums of dy = X, 4x the pixels) is taken by trailing blocks (blockIdx.x == ncb), 64 channels each.
// ---------------------------------------------------------------------------
struct SwArgs {
    const void* g;
    int g_ld, Ng;
    const void* x;
    int x_ld, Cq, Cq_pad, in_abs, in_sq;
    int B, Hg, Wg, Hx, Wx, k, s, p;
    int M;            // G pixels
    int ncb;          // 64-wide column blocks: k*k*cbt
    int cbt;          // column blocks per tap: ceil(Cq_pad / 64) (the last one masked when Cq_pad % 64 == 32)
    float* dw;
    int accumulate;
    const void* bsrc; // bias: column sums of bsrc [bnpix][bc] (ld bsrc_ld) -> db; db == NULL: none
    int bsrc_ld, bnpix, bc;
    float* db;
    int bias_from_g;  // Conv2d: db = column sums of G, taken by the main blocks; else by trailing blocks
    float inv_plane, inv_wg;   // 1 / (Hg * Wg), 1 / Wg: the per-row pixel decomposition without integer division
    float* slab;      // non-NULL: dW goes to the [Ng][k*k*Cq_pad] slab (coalesced rows; a WGRAD reduce job transposes it)
};

// n / d for 0 <= n < 2^23 from a float reciprocal and one correction each way (n * inv is off by at most one);
// a 32-bit integer division is ~25 VALU instructions
__device__ __forceinline__ int div_small(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    const int r = n - q * d;
    q += (r >= d ? 1 : 0) - (r < 0 ? 1 : 0);
    return q;
}

constexpr int SW_NW = 8, SW_STEPS = 4;   // waves; 32-pixel steps per wave (M <= SW_NW * SW_STEPS * 32)
// 16-byte slot swizzle of a [32][128 B] tile read by ds_read_b64_tr_b16: the 8 rows one half-wave reads
// (4 per 16-lane group, groups 8 rows apart) land on distinct bank groups
__device__ __forceinline__ int swz_sw(int row, int slot) {
    return row * 128 + ((slot ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2))) << 4);
}

// 8 x (64 x 68 fp32) partial tiles (the loop's staging uses the first 64 KB) + 512 x 8 bias partials
constexpr int SW_SMEM = SW_NW * 64 * 68 * 4 + 512 * 8 * 4;

// One block of the latent-size weight gradient: block (bx, by) of a (ncb [+ 1]) x gy grid.
// LONG: more than SW_STEPS steps per wave (M up to small_wgrad_mmax()): the step pairs in a loop
template <int XT, bool LONG>   // X transform on load: 0 none, 1 |x| (h_a's first conv), 2 x^2 (GDN's gamma gradient)
__device__ __forceinline__ void wgrad_small_block(const SwArgs& a, int bx, int by, int gy, char* smem) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr unsigned OOB = 0x80000000u;
    if (bx == a.ncb) {
        // bias: 64 channels per block, pixels over 64 row groups of 8 threads (8 channels each)
        if (!a.db || a.bias_from_g) return;
        float* red = reinterpret_cast<float*>(smem);
        const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<void*>(a.bsrc), (short)0, (int)((int64_t)a.bnpix * a.bsrc_ld * 2), 0x00020000);
        for (int c0 = by * 64; c0 < a.bc; c0 += gy * 64) {
            const int slot = tid & 7, r = tid >> 3;
            const int c = c0 + slot * 8;
            float sacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            // 8 rows (512 pixels apart) per batch, all loads issued before the adds
            for (int pb = r; pb < a.bnpix; pb += 512) {
                u32x4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int pp = pb + u * 64;
                    const unsigned off = (unsigned)(pp * a.bsrc_ld + c) * 2u;
                    v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                          br, ((pp < a.bnpix) & (c < a.bc)) ? off : OOB, 0, 0));
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const bf16x8 h = __builtin_bit_cast(bf16x8, v[u]);
#pragma unroll
                    for (int e = 0; e < 8; ++e) sacc[e] += (float)h[e];
                }
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < 8; ++e) red[r * 64 + slot * 8 + e] = sacc[e];
            __syncthreads();
            if (tid < 64 && c0 + tid < a.bc) {
                float v = 0.f;
                for (int rr = 0; rr < 64; ++rr) v += red[rr * 64 + tid];
                float* d = a.db + c0 + tid;
                *d = a.accumulate ? *d + v : v;
            }
        }
        return;
    }
    const int n0 = by * 64;
    const int t = bx / a.cbt, q0 = (bx - t * a.cbt) * 64;
    const int kh = t / a.k, kw = t - kh * a.k;
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(a.g), (short)0, (int)((int64_t)a.M * a.g_ld * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(a.x), (short)0, (int)((int64_t)a.B * a.Hx * a.Wx * a.x_ld * 2), 0x00020000);
    char* const Gs = smem + wave * 8192;
    char* const Xs = Gs + 4096;
    const int nsteps = (a.M + 31) / 32;
    const int per = (nsteps + SW_NW - 1) / SW_NW;
    const int s0 = wave * per, s1 = min(nsteps, s0 + per);
    const int plane = a.Hg * a.Wg;
    const int slot = lane & 7;
    // Conv2d: the bias gradient is the column sums of G -- taken by the (tap 0, q 0) blocks from the G
    // chunks they stage anyway (the pixel rows each thread loads: 8 channels, summed over its rows)
    const bool gsum = a.db && a.bias_from_g && t == 0 && q0 == 0;
    const float gsf = gsum ? 1.f : 0.f;
    float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    u32x4 rga[4], rxa[4], rgb[4], rxb[4];
    auto load = [&](int st, u32x4 (&rg)[4], u32x4 (&rx)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = i * 8 + (lane >> 3);
            const int m = st * 32 + row;
            const bool okm = (st < s1) & (m < a.M);
            // 32-multiple widths: the channel slots past Ng / Cq_pad of the last row / column block read 0
            const bool okg = okm & (n0 + slot * 8 < a.Ng);
            const unsigned goff = (unsigned)(m * a.g_ld + n0 + slot * 8) * 2u;
            rg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(gr, okg ? goff : OOB, 0, 0));
            const int b = div_small(m, plane, a.inv_plane);
            const int r = m - b * plane;
            const int j = div_small(r, a.Wg, a.inv_wg);
            const int iy = j * a.s - a.p + kh, ix = (r - j * a.Wg) * a.s - a.p + kw;
            const bool okx = okm & ((unsigned)iy < (unsigned)a.Hx) & ((unsigned)ix < (unsigned)a.Wx) &
                             (q0 + slot * 8 < a.Cq_pad);
            const unsigned xoff = (unsigned)(((b * a.Hx + iy) * a.Wx + ix) * a.x_ld + q0 + slot * 8) * 2u;
            rx[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, okx ? xoff : OOB, 0, 0));
        }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    const int r0 = 8 * g_ + q_;
    // two steps in flight (register sets A / B, straight-line pair loop; steps past s1 read zeros)
    load(s0, rga, rxa);
    load(s0 + 1, rgb, rxb);
    auto step = [&](int st, u32x4 (&rg)[4], u32x4 (&rx)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = i * 8 + (lane >> 3);
            u32x4 xv = rx[i];
            if constexpr (XT == 1) xv = abs_chunk(xv, 2);
            if constexpr (XT == 2) xv = sq_chunk<bf16>(xv);
            *reinterpret_cast<u32x4*>(Gs + swz_sw(row, slot)) = rg[i];
            *reinterpret_cast<u32x4*>(Xs + swz_sw(row, slot)) = xv;
            // branch-free (a branch here costs the counted waits): scaled by 0 outside the bias blocks
            const bf16x8 h = __builtin_bit_cast(bf16x8, rg[i]);
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum[e] += gsf * (float)h[e];
        }
        load(st + 2, rg, rx);
        u32x4 fb[4];
#pragma unroll
        for (int tn = 0; tn < 4; ++tn) {
            const int c = tn * 16 + 4 * p4;
            const s16x4 b0 = ds_tr16(Xs, swz_sw(r0, c >> 3) + ((c & 7) << 1));
            const s16x4 b1 = ds_tr16(Xs, swz_sw(r0 + 4, c >> 3) + ((c & 7) << 1));
            const s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
            fb[tn] = __builtin_bit_cast(u32x4, bv);
        }
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) {
            const int c = tm * 16 + 4 * p4;
            const s16x4 a0 = ds_tr16(Gs, swz_sw(r0, c >> 3) + ((c & 7) << 1));
            const s16x4 a1 = ds_tr16(Gs, swz_sw(r0 + 4, c >> 3) + ((c & 7) << 1));
            const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
            const u32x4 fa = __builtin_bit_cast(u32x4, av);
#pragma unroll
            for (int tn = 0; tn < 4; ++tn) acc[tm][tn] = mma16<bf16>(fa, fb[tn], acc[tm][tn]);
        }
    };
    // M <= 1024 (host check): at most SW_STEPS steps per wave, straight-line code (no loop-carried
    // register sets, whose back-edge copies would wait for the prefetch); steps past s1 multiply zeros
    static_assert(SW_STEPS % 2 == 0, "pairs");
    if constexpr (LONG) {
        // the two register sets keep fixed roles in the pair body: no back-edge copies
        const int npairs = s1 > s0 ? (s1 - s0 + 1) / 2 : 0;
        for (int it = 0; it < npairs; ++it) {
            step(s0 + 2 * it, rga, rxa);
            step(s0 + 2 * it + 1, rgb, rxb);
        }
    } else {
#pragma unroll
        for (int it = 0; it < SW_STEPS / 2; ++it) {
            step(s0 + 2 * it, rga, rxa);
            step(s0 + 2 * it + 1, rgb, rxb);
        }
    }
    // partial tiles: wave w -> fp32 [64][68] at w * 17 KB (the staging regions are dead past this barrier)
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    float* mine = red + wave * 64 * 68;
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn)
#pragma unroll
            for (int r = 0; r < 4; ++r) mine[(tm * 16 + (lane >> 4) * 4 + r) * 68 + tn * 16 + (lane & 15)] = acc[tm][tn][r];
    __syncthreads();
    float* bred = red + SW_NW * 64 * 68;
    if (gsum) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bred[tid * 8 + e] = bsum[e];
    }
    __syncthreads();
    if (gsum && tid < 64 && n0 + tid < a.Ng) {
        // channel n0 + tid: slot tid / 8, element tid % 8, summed over (wave, row group) in fixed order
        float v = 0.f;
        for (int w = 0; w < SW_NW; ++w)
#pragma unroll
            for (int lr = 0; lr < 8; ++lr) v += bred[(w * 64 + lr * 8 + (tid >> 3)) * 8 + (tid & 7)];
        float* d = a.db + n0 + tid;
        *d = a.accumulate ? *d + v : v;
    }
    if (a.slab) {
        // slab row n: [tap][Cq_pad] -- this block's 64 columns are one contiguous 256-byte run per row (the torch
        // layout's stride-k*k scatter cost one L2 request per element: 819 K requests per C2 h-layer launch)
        const int ncols = a.k * a.k * a.Cq_pad;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int id = u * 512 + tid;
            const int nl = id >> 6, ql = id & 63;
            const int n = n0 + nl, q = q0 + ql;
            float s_ = 0.f;
#pragma unroll
            for (int w = 0; w < SW_NW; ++w) s_ += red[(w * 64 + nl) * 68 + ql];
            if (n < a.Ng && q < a.Cq_pad) a.slab[(int64_t)n * ncols + t * a.Cq_pad + q] = s_;
        }
        return;
    }
    // torch layout dw[n][q][kh][kw]: 8 elements per thread, their old values (accumulate) loaded together
    // before any store -- one dependent round trip instead of eight
    const int kk = a.k * a.k;
    float v[8];
    float* d[8];
    bool ok[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int id = u * 512 + tid;
        const int nl = id >> 6, ql = id & 63;
        const int n = n0 + nl, q = q0 + ql;
        ok[u] = n < a.Ng && q < a.Cq;
        d[u] = a.dw + ((int64_t)(ok[u] ? n : 0) * a.Cq + (ok[u] ? q : 0)) * kk + t;
        float s_ = 0.f;
#pragma unroll
        for (int w = 0; w < SW_NW; ++w) s_ += red[(w * 64 + nl) * 68 + ql];
        v[u] = s_;
    }
    if (a.accumulate) {
        float old[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) old[u] = *d[u];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] += old[u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (ok[u]) *d[u] = v[u];
}

template <int XT, bool LONG = false>
__global__ __launch_bounds__(512, 1) void wgrad_small_kernel(const SwArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[SW_SMEM];
    wgrad_small_block<XT, LONG>(a, (int)blockIdx.x, (int)blockIdx.y, (int)gridDim.y, smem);
}

// Several latent-size weight gradients in ONE launch (cai_conv_wgrad_batch): job j owns blocks
// [start[j], start[j + 1]) of a 1-D grid, laid out as its own gx x gy grid.  They are independent (each writes
// its own slab; bias gradients written in place never repeat within a batch: host check), so a batch costs one
// launch and fills the chip with blocks that one layer alone leaves idle.
constexpr int SW_BATCH_MAX = 16;
struct SwBatch {
    SwArgs job[SW_BATCH_MAX];
    int start[SW_BATCH_MAX + 1];
    int gx[SW_BATCH_MAX], gy[SW_BATCH_MAX];
    int n;
};

template <int XT, bool LONG>
__global__ __launch_bounds__(512, 1) void wgrad_small_batch_kernel(const SwBatch b) {
    __shared__ __attribute__((aligned(16))) char smem[SW_SMEM];
    const int L = (int)blockIdx.x;
    int j = 0;
    while (j + 1 < b.n && L >= b.start[j + 1]) ++j;
    const int l = L - b.start[j], gx = b.gx[j];
    wgrad_small_block<XT, LONG>(b.job[j], l % gx, l / gx, b.gy[j], smem);
}

// dw[n][q][kh][kw] (+)= sum_s ws[s][n][(kh*k+kw)*Cq_pad + q]
// Block = 16 float4 column groups x 16 split groups: reads walk the slabs in
// memory order (256-byte runs), the 16 split partials meet in LDS in a fixed
// order (deterministic); the transposed writes are 1/S of the bytes.
// ---------------------------------------------------------------------------
// bf16 wgrad with LDS-DMA staging: block tile 128 G-channels (rows n) x 256
// (tap, q) columns, 64-pixel K-steps, 3-stage ring, 8 waves (2 x 4, each
// 64 x 64).  The G tile [64 px][128 ch] and the two X half-tiles
// [64 px][128 cols] are 256-byte-row images filled lane-linearly by
// global_load_lds (4 rows per wave-instruction); the tr-read swizzle trswz()
// goes on the per-lane source slot.  A lane's column chunk (tap, q) is fixed
// for the whole launch, so its X gather is one bounds test per pixel row.
// Block b works on pixel split (xcd-remapped index / tiles): the tiles of one
// pixel range share an XCD's L2.
// ---------------------------------------------------------------------------
enum { WG_ABS = 1, WG_SQ = 2, WG_BIAS = 4, WG_TBIAS = 8 };

__device__ __forceinline__ float sum8_bf16(u32x4 v) {
    const bf16x8 h = __builtin_bit_cast(bf16x8, v);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (float)h[e];
    return s;
}

// index of tap (kh, kw) in the transposed-bias tap set, or -1
__device__ __forceinline__ int tbias_sel(const WgradArgs& a, int kh, int kw) {
    const int dh = kh - a.tb_kh0, dw = kw - a.tb_kw0;
    return ((unsigned)dh < (unsigned)a.tb_s && (unsigned)dw < (unsigned)a.tb_s) ? dh * a.tb_s + dw : -1;
}

template <int CT>
constexpr int wgrad_glds_smem() { return 3 * (1 + CT / 128) * 64 * 256; }

// block wgid of an nwg-block grid (its XCD: wgid & 7, as the hardware dispatches a grid of its own)
template <int CT, int FLAGS>
__device__ __forceinline__ void wgrad_glds_block(const WgradArgs& a, int wgid, int nwg, char* smem) {
    constexpr int OPB = 64 * 256;                 // one [64][256 B] image
    constexpr int NX = CT / 128;                  // X images (128 columns each)
    constexpr int STAGE = (1 + NX) * OPB;         // G, X_0 [, X_1]
    constexpr int WCOL = CT / 4;                  // columns per wave
    constexpr int TN = WCOL / 16;
    constexpr int G = 2 * (1 + NX);               // DMA instructions per thread per step
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;        // 2 (rows) x 4 (cols) waves
    const int ntile = a.ctiles * a.rtiles;
    const int L = xcd_remap(wgid, nwg);
    const int split = L / ntile;
    const int tl = L - split * ntile;
    const int ctile = tl % a.ctiles, rtile = tl / a.ctiles;
    const int c0 = ctile * CT, r0 = rtile * 128;
    const int pbeg = min((int)a.M, (int)(split * a.split_len));
    const int pend = min((int)a.M, (int)(pbeg + a.split_len));
    const int nsteps = (pend - pbeg + 63) / 64;
    float* out = a.ws + (int64_t)split * a.Ng * a.ncols;

    // DMA rows of this lane: (i*8 + wid)*4 + lane/16 for i = 0, 1; the source
    // slot is the physical slot lane%16 XOR the tr-read swizzle of that row
    const int prow0 = wid * 4 + (lane >> 4);      // i = 0; i = 1 adds 32
    const int sl = (lane & 15) ^ ((((lane >> 4) & 3) << 1) | (((wid >> 1) & 1) << 3));
    const char* Gp = reinterpret_cast<const char*>(a.g);
    const char* Xp = reinterpret_cast<const char*>(a.x);
    const int gch = r0 + sl * 8;
    const bool gvalid = gch < a.Ng;
    int xoff[NX], xkh[NX], xkw[NX];
    bool xvalid[NX];
#pragma unroll
    for (int h = 0; h < NX; ++h) {
        const int col = c0 + h * 128 + sl * 8;
        xvalid[h] = col < a.ncols;
        const int t = xvalid[h] ? col / a.Cq_pad : 0;
        const int q = xvalid[h] ? col - t * a.Cq_pad : 0;
        xkh[h] = t / a.k;
        xkw[h] = t - xkh[h] * a.k;
        // byte offset of this lane's tap / channel slot from the tap-(0,0) pixel of its row
        xoff[h] = ((xkh[h] * a.Wx + xkw[h]) * a.x_ld + q) * 2;
    }
    const int plane = a.Hg * a.Wg;
    // pixel coordinates (image, row, column) of this thread's two DMA rows for the next step to issue:
    // steps are issued in order and advance the pixel index by 64, so the coordinates advance by
    // carries instead of two integer divisions per row and step
    int cb[2], cj[2], cx[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int m = pbeg + prow0 + i * 32;
        cb[i] = m / plane;
        const int r = m - cb[i] * plane;
        cj[i] = r / a.Wg;
        cx[i] = r - cj[i] * a.Wg;
    }

    auto issue = [&](int st, int stage) {
        char* sb = smem + stage * STAGE + wid * 4 * 256;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = pbeg + st * 64 + prow0 + i * 32;
            const bool mok = m < pend;
            const void* gs = (mok && gvalid) ? (const void*)(Gp + ((int64_t)m * a.g_ld + gch) * 2)
                                             : (const void*)cai_zero_page;
            glds16_asm(gs, sb + i * 32 * 256);
            const int b = cb[i], j = cj[i];
            const int yb = j * a.s - a.p, xb = cx[i] * a.s - a.p;
            cx[i] += 64;
            while (cx[i] >= a.Wg) {
                cx[i] -= a.Wg;
                if (++cj[i] == a.Hg) {
                    cj[i] = 0;
                    ++cb[i];
                }
            }
            // tap-(0,0) pixel of this row (may lie in the padding; only in-range taps are read)
            const char* xrow = Xp + (((int64_t)b * a.Hx + yb) * a.Wx + xb) * a.x_ld * 2;
#pragma unroll
            for (int h = 0; h < NX; ++h) {
                const int iy = yb + xkh[h], ix = xb + xkw[h];
                const bool ok = mok && xvalid[h] && (unsigned)iy < (unsigned)a.Hx && (unsigned)ix < (unsigned)a.Wx;
                const void* xs = ok ? (const void*)(xrow + xoff[h]) : (const void*)cai_zero_page;
                glds16_asm(xs, sb + (1 + h) * OPB + i * 32 * 256);
            }
        }
    };

    f32x4 acc[4][TN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    // bias gradient (column sums of G) from the A fragments: the wc == 0 waves
    // of the ctile-0 blocks hold every G value of the tile exactly once
    // (the four column waves of a row pair share the A fragments: wave wc sums tm == wc)
    const bool do_bias = (FLAGS & WG_BIAS) && ctile == 0;
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    const int wcol = wc * WCOL;
    const int ximg = 1 + wcol / 128, xcb = wcol % 128;
    // transposed bias: this lane's column (tap, q) of each column block, if its tap is in the set
    int tsel[TN], tq[TN];
    float tsum[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) {
        tsum[t] = 0.f;
        tsel[t] = -1;
        tq[t] = 0;
        if constexpr ((FLAGS & WG_TBIAS) != 0) {
            const int col = c0 + wcol + t * 16 + (lane & 15);
            const int tap = col / a.Cq_pad, q = col - tap * a.Cq_pad;
            if (col < a.ncols && q < a.nbias && rtile == 0 && wr == 0) tsel[t] = tbias_sel(a, tap / a.k, tap % a.k);
            tq[t] = q;
        }
    }
    if (nsteps > 0) issue(0, 0);
    if (nsteps > 1) issue(1, 1);
    for (int st = 0; st < nsteps; ++st) {
        if (st + 1 < nsteps)
            wait_vmcnt<G>();
        else
            wait_vmcnt<0>();
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (st + 2 < nsteps) issue(st + 2, (st + 2) % 3);
        const char* Gs = smem + (st % 3) * STAGE;
        const char* Xs = Gs + OPB * ximg;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int rr = 32 * ks + 8 * g_ + q_;
            u32x4 fb[TN];
#pragma unroll
            for (int t = 0; t < TN; ++t) {
                const int colB = xcb + t * 16 + 4 * p4;
                s16x4 b0 = ds_tr16(Xs, trswz(rr, colB >> 3) + ((colB & 7) << 1));
                s16x4 b1 = ds_tr16(Xs, trswz(rr + 4, colB >> 3) + ((colB & 7) << 1));
                s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
                fb[t] = __builtin_bit_cast(u32x4, bv);
                if constexpr ((FLAGS & WG_ABS) != 0) fb[t] = abs_chunk(fb[t], 2);
                if constexpr ((FLAGS & WG_SQ) != 0) fb[t] = sq_chunk<bf16>(fb[t]);
            }
#pragma unroll
            for (int tm = 0; tm < 4; ++tm) {
                const int colA = wr * 64 + tm * 16 + 4 * p4;
                s16x4 a0 = ds_tr16(Gs, trswz(rr, colA >> 3) + ((colA & 7) << 1));
                s16x4 a1 = ds_tr16(Gs, trswz(rr + 4, colA >> 3) + ((colA & 7) << 1));
                s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                const u32x4 fa = __builtin_bit_cast(u32x4, av);
                if constexpr ((FLAGS & WG_BIAS) != 0) {
                    if (do_bias && tm == wc) {
                        const bf16x8 h = __builtin_bit_cast(bf16x8, fa);
                        float sacc = 0.f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) sacc += (float)h[e];
                        bsum[tm] += sacc;
                    }
                }
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mma16<bf16>(fa, fb[tn], acc[tm][tn]);
            }
            // transposed bias sums after the MFMAs: inside the read loop they made each B read wait
            if constexpr ((FLAGS & WG_TBIAS) != 0) {
#pragma unroll
                for (int t = 0; t < TN; ++t)
                    if (tsel[t] >= 0) tsum[t] += sum8_bf16(fb[t]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr ((FLAGS & WG_BIAS) != 0) {
        if (do_bias) {
            // an A fragment lane holds channel (lane & 15) of its 16-row group
            // over 8 pixels (8 * (lane >> 4)): fold the four pixel groups
            float v = bsum[0] + bsum[1] + bsum[2] + bsum[3];   // only bsum[wc] is non-zero
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            const int n = r0 + wr * 64 + wc * 16 + lane;
            if (lane < 16 && n < a.Ng) a.bws[(int64_t)split * a.Ng + n] = v;
        }
    }
    if constexpr ((FLAGS & WG_TBIAS) != 0) {
        // a column's 4 lane groups (lane >> 4) hold disjoint pixels: fold them, one lane writes
#pragma unroll
        for (int t = 0; t < TN; ++t) {
            float v = tsum[t];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane < 16 && tsel[t] >= 0)
                a.bws[((int64_t)split * a.tb_s * a.tb_s + tsel[t]) * a.nbias + tq[t]] = v;
        }
    }
#pragma unroll
    for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = c0 + wcol + tn * 16 + (lane & 15);
            if (col >= a.ncols) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = r0 + wr * 64 + tm * 16 + (lane >> 4) * 4 + r;
                if (row < a.Ng) out[(int64_t)row * a.ncols + col] = acc[tm][tn][r];
            }
        }
}

template <int CT, int FLAGS>
__global__ __launch_bounds__(512, 1) void wgrad_glds_kernel(const WgradArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[wgrad_glds_smem<CT>()];
    wgrad_glds_block<CT, FLAGS>(a, (int)blockIdx.x, (int)gridDim.x, smem);
}

// Several pixel-split weight gradients of one kernel variant in one launch (cai_conv_wgrad_batch): job j owns
// blocks [start[j], start[j + 1]) of a 1-D grid -- its nwg[j] blocks, then padding blocks that exit; starts are
// multiples of 8, so every block keeps the XCD of its launch-of-its-own index.  Each job writes only its slabs.
constexpr int WG_BATCH_MAX = 16;
struct WgBatch {
    WgradArgs job[WG_BATCH_MAX];
    int start[WG_BATCH_MAX + 1];
    int nwg[WG_BATCH_MAX];
    int n;
};
static_assert(sizeof(WgBatch) <= 4096, "kernel argument block");

__device__ __forceinline__ int wg_batch_job(const WgBatch& b, int L) {
    int j = 0;
    while (j + 1 < b.n && L >= b.start[j + 1]) ++j;
    return j;
}

template <int CT, int FLAGS>
__global__ __launch_bounds__(512, 1) void wgrad_glds_batch_kernel(const WgBatch b) {
    __shared__ __attribute__((aligned(16))) char smem[wgrad_glds_smem<CT>()];
    const int L = (int)blockIdx.x, j = wg_batch_job(b, L), l = L - b.start[j];
    if (l < b.nwg[j]) wgrad_glds_block<CT, FLAGS>(b.job[j], l, b.nwg[j], smem);
}

// ---------------------------------------------------------------------------
// Halo-staged weight gradient of the stride-2 gather convolutions (Conv2d k3/k5 s2 p=k/2, and the
// ConvTranspose2d of that geometry, whose wgrad gathers its output gradient the same way), bf16, for
// G maps whose width is a multiple of 64.  wgrad_glds_kernel gathers the X operand per (pixel, tap)
// column: for a 256-column tile (two taps) every step pulls 32 KB of X plus 16 KB of G through LDS, and
// the kernel runs at the rate L2 / MALL deliver those bytes (45 % of wave time parked on the DMA waits,
// profiles/r02_*).  Here a block owns one KERNEL ROW kh, all KS taps of it and 64 channels (KS*64
// columns), and a K-step is one 64-pixel strip of a G row: the strip's whole X footprint for that kernel
// row -- input row 2j-p+kh, x offsets 0 .. 2*63+KS-1 from 2*i0-p, 64 channels -- is ONE LDS image of
// 2*63+KS cells (16.8 KB for k5) that all KS taps read at a per-tap offset.  Bytes per step drop to
// 33 KB for 1.25x the MFMA work, so a 4-stage ring (3 strips in flight) fits in LDS.
//
// Footprint layout: x offset t -> plane t&1 (even offsets first, then odd), cell t>>1, so tap kw reads
// pixel p at cell p + kw/2 of plane kw&1: 16 consecutive pixels = 16 consecutive cells.  A cell is 64
// channels (128 B = four 32-B groups of 16 channels); the group of a 16-channel block is XOR-swizzled
// by h(cell) = bit1 | bit3<<1 of the cell index, which puts the 8 cells a half-wave's
// ds_read_b64_tr_b16 touches (p..p+3, p+8..p+11) on 8 distinct 32-B bank groups.  The DMA writes LDS
// lane-linearly, so the swizzle is applied to the per-lane SOURCE slot (both-sides rule).
// Partials leave through the same [split][Ng][ncols] slab as wgrad_glds_kernel (same reduce).
// ---------------------------------------------------------------------------
// R > 1 (G width 64 / R = 32 or 16): a strip is R whole G rows of 64 / R pixels (still 64 consecutive G
// pixels); each row has its own footprint row image of NCR cells (even / odd planes), rows stacked.
// GR = 192 (192-row tiles): the G strip is three [64 px][64 ch] images of 128-byte rows (swz_sw slots), 24 KB.
template <int KS, int S = 2, int R = 1, int GR = 128>
struct WhCfg {
    static constexpr int WR = 64 / R;                 // pixels per strip row
    static constexpr int NCR = S * (WR - 1) + KS;     // footprint cells of one strip row
    static constexpr int NE = S == 2 ? (NCR + 1) / 2 : NCR;   // even-offset plane of a row (stride 1: one plane)
    static constexpr int NCELL = R * NCR;             // footprint cells of one strip
    static constexpr int XSLOTS = NCELL * 8;          // 16-byte pieces of the footprint
    static constexpr int XGRP = (XSLOTS + 63) / 64;   // wave-instructions that fill it
    static constexpr int NXI = (XGRP + 7) / 8;        // per thread (8 waves); spare instructions hit a sink
    static constexpr int NST = 4;                     // ring stages (3 strips in flight)
    static constexpr int GIMG = 64 * 2 * GR;          // G strip [64 px][128 ch]; the 4 G images first ...
    static constexpr int XBASE = NST * GIMG;          // ... then the 4 footprints (GR = 128: every stage offset < 64 KB)
    static constexpr int XSTRIDE = XGRP * 1024 + 1024;   // footprint + a 1 KB sink for the spare DMAs
    static constexpr int BYTES = XBASE + NST * XSTRIDE;
    static_assert(BYTES <= 160 * 1024, "LDS");
    static constexpr int NLOAD = (GR == 192 ? 3 : 2) + NXI;   // DMA instructions per thread per step
    static constexpr int CT = KS * 64;                // tile columns
    static constexpr int WCOL = CT / 4;               // columns per column-wave
    static constexpr int TN = WCOL / 16;
};


__device__ __forceinline__ int wh_h(int cell) { return ((cell >> 1) & 1) | (((cell >> 3) & 1) << 1); }

// keep a per-lane value opaque to the optimiser: it stays one materialised VGPR instead of being
// re-derived from its parts at every use
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// S = 1: the stride-1 k3 p1 Conv2d (cheng2020's 3x3 convs): one footprint plane, tap kw at cell p + kw.
// TMR: row fragments per wave -- 4 (128-row tiles), 2 (64-row tiles, for Ng a multiple of 64 but not of 128:
// C2's g_a[6] / g_s[0]; the 128-row tiles left a third of their rows empty) or 6 (192-row tiles, stride-1 k3 with
// Ng = 192: cheng2020's 3x3 convs -- X read once per tile and no empty rows, against 64-row tiles' three passes
// over X and half the MFMA work per step)
template <int KS, int S, int FLAGS, int R, int TMR>
__device__ __forceinline__ void wgrad_halo_block(const WgradArgs& a, int wgid, int nwg, char* smem) {
    static_assert(TMR == 4 || TMR == 2 || TMR == 6, "128-, 64- or 192-row tiles");
    using W = WhCfg<KS, S, R, TMR == 6 ? 192 : 128>;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;            // 2 (rows) x 4 (cols) waves
    const int nqc = a.Cq_pad / 64;
    const int ntile = KS * nqc * a.rtiles;
    const int L = xcd_remap(wgid, nwg);
    const int split = L / ntile;
    const int tl = L - split * ntile;
    const int ctile = tl % (KS * nqc), rtile = tl / (KS * nqc);
    const int kh = ctile / nqc, q0 = (ctile - kh * nqc) * 64, r0 = rtile * (32 * TMR);
    const int nsr = R == 1 ? a.Wg / 64 : 1;           // strips per G row (R > 1: one strip spans R rows)
    const int nrg = a.Hg / R;                         // strip rows per image
    const int nstrip = a.B * nrg * nsr;
    const int sbeg = min(nstrip, split * a.nsplit), send = min(nstrip, sbeg + a.nsplit);   // a.nsplit: strips per split
    const int nsteps = send - sbeg;
    float* out = a.ws + (int64_t)split * a.Ng * a.ncols;

    // G DMA: rows prow0 + 32 i of the strip, source slot sl (the tr-read swizzle of that row)
    const int prow0 = wid * 4 + (lane >> 4);
    const int sl = (lane & 15) ^ ((((lane >> 4) & 3) << 1) | (((wid >> 1) & 1) << 3));
    const char* Gp = reinterpret_cast<const char*>(a.g);
    const char* Xp = reinterpret_cast<const char*>(a.x);
    const int gch = r0 + sl * 8;
    const bool gvalid = gch < a.Ng && (TMR == 4 || sl < 8);   // 64-row tiles: the strip's first 64 channels
    // 192-row tiles: wave w fills rows 8w .. 8w + 7 of each 64-channel image, one instruction per image; a lane's
    // source slot is the swz_sw slot of its lane-linear LDS position
    const int grow6 = wid * 8 + (lane >> 3);
    const int gsl6 = (lane & 7) ^ ((((grow6 >> 1) & 1) << 1) | (((grow6 >> 3) & 1) << 2));
    // X DMA: this lane's footprint piece of each instruction (x offset t, channel byte offset), or the sink
    int xt[W::NXI];
    int xr[W::NXI];                                   // strip row of the piece (R > 1)
    bool xin[W::NXI];
    int64_t xlane[W::NXI];                            // byte offset of the piece inside a strip's footprint row
    const int64_t xpix = (int64_t)a.x_ld * 2;         // bytes per X pixel
#pragma unroll
    for (int n = 0; n < W::NXI; ++n) {
        const int grp = n * 8 + wid;
        const int Ls = grp * 64 + lane;
        xin[n] = grp < W::XGRP && Ls < W::XSLOTS;
        const int pc = xin[n] ? Ls >> 3 : 0, ps = Ls & 7;
        const int rc = pc % W::NCR;                   // cell inside its row image
        xr[n] = pc / W::NCR;
        xt[n] = S == 1 ? rc : (rc < W::NE ? 2 * rc : 2 * (rc - W::NE) + 1);
        const int ls = (((ps >> 1) ^ wh_h(pc)) << 1) | (ps & 1);
        xlane[n] = xt[n] * xpix + (q0 + ls * 8) * 2;
    }
    // strip coordinates (column block, row, image) of the next strip to issue: strips are issued in order,
    // so they advance by carries instead of integer divisions per step
    int cib = sbeg % nsr, cj = ((sbeg / nsr) % nrg) * R, cb = (sbeg / nsr) / nrg;
    const char* gsrc = TMR == 6 ? Gp + ((int64_t)(sbeg * 64 + grow6) * a.g_ld + r0 + gsl6 * 8) * 2
                                : Gp + ((int64_t)(sbeg * 64 + prow0) * a.g_ld + gch) * 2;   // strips are 64 G pixels
    const int64_t gstep = (int64_t)64 * a.g_ld * 2, ghalf = (int64_t)32 * a.g_ld * 2;

    auto issue = [&](int stage) {
        char* gb = smem + stage * W::GIMG;
        char* xb = smem + W::XBASE + stage * W::XSTRIDE;
        if constexpr (TMR == 6) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
                glds16_asm(r0 + i * 64 + gsl6 * 8 < a.Ng ? (const void*)(gsrc + i * 128) : (const void*)cai_zero_page,
                           gb + i * 8192 + wid * 1024);
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
                glds16_asm(gvalid ? (const void*)(gsrc + i * ghalf) : (const void*)cai_zero_page,
                       gb + wid * 4 * 256 + i * 32 * 256);
        }
        gsrc += gstep;
        const int y = cj * S - a.p + kh;
        const int x0 = cib * (64 * S) - a.p;
        const bool yok = (unsigned)y < (unsigned)a.Hx;
        const char* xrow = Xp + (((int64_t)cb * a.Hx + (yok ? y : 0)) * a.Wx + x0) * xpix;
#pragma unroll
        for (int n = 0; n < W::NXI; ++n) {
            const int grp = n * 8 + wid;
            if constexpr (R == 1) {
                const bool ok = xin[n] && yok && (unsigned)(x0 + xt[n]) < (unsigned)a.Wx;
                glds16_asm(ok ? (const void*)(xrow + xlane[n]) : (const void*)cai_zero_page,
                       xb + (grp < W::XGRP ? grp * 1024 : W::XGRP * 1024));
            } else {
                const int yr = y + S * xr[n];            // input row of the piece's strip row
                const bool ok = xin[n] && (unsigned)yr < (unsigned)a.Hx && (unsigned)(x0 + xt[n]) < (unsigned)a.Wx;
                const char* src = Xp + (((int64_t)cb * a.Hx + yr) * a.Wx + x0) * xpix + xlane[n];
                glds16_asm(ok ? (const void*)src : (const void*)cai_zero_page,
                       xb + (grp < W::XGRP ? grp * 1024 : W::XGRP * 1024));
            }
        }
        if (++cib == nsr) {
            cib = 0;
            cj += R;
            if (cj == a.Hg) {
                cj = 0;
                ++cb;
            }
        }
    };

    f32x4 acc[TMR][W::TN];
#pragma unroll
    for (int i = 0; i < TMR; ++i)
#pragma unroll
        for (int j = 0; j < W::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    const bool do_bias = (FLAGS & WG_BIAS) && ctile == 0;
    float bsum[TMR];
#pragma unroll
    for (int i = 0; i < TMR; ++i) bsum[i] = 0.f;
    const int wcol = wc * W::WCOL;
    int tsel[W::TN];
    float tsum[W::TN];
#pragma unroll
    for (int t = 0; t < W::TN; ++t) {
        tsum[t] = 0.f;
        tsel[t] = -1;
        if constexpr ((FLAGS & WG_TBIAS) != 0) {
            const int col = wcol + t * 16 + (lane & 15);
            if (q0 + col % 64 < a.nbias && rtile == 0 && wr == 0) tsel[t] = tbias_sel(a, kh, col / 64);
        }
    }
    // LDS byte offsets of every fragment read, fixed for the launch (stage 0; the other stages add a
    // compile-time immediate): B (footprint) per (ks, column block, pixel half) -- the tap's plane / cell
    // shift and the block's swizzled 32-B group -- and A (G strip)
    int boff[2][W::TN][2], aoff[2][TMR][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const int rr = 32 * ks + 8 * g_ + q_;
        const int row0 = (rr / W::WR) * W::NCR, px = rr % W::WR;   // strip row image, pixel in the row
#pragma unroll
        for (int tn = 0; tn < W::TN; ++tn) {
            const int col = wcol + tn * 16, kw = col / 64, cg = (col % 64) / 16;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = row0 + (S == 1 ? kw : (kw & 1) * W::NE + (kw >> 1)) + px + 4 * h;
                boff[ks][tn][h] = opaque(W::XBASE + c * 128 + (((cg ^ wh_h(c)) << 1) | (p4 >> 1)) * 16 + (p4 & 1) * 8);
            }
        }
#pragma unroll
        for (int tm = 0; tm < TMR; ++tm) {
            const int colA = wr * (16 * TMR) + tm * 16 + 4 * p4;
#pragma unroll
            for (int h = 0; h < 2; ++h)
                aoff[ks][tm][h] = opaque(TMR == 6 ? (colA >> 6) * 8192 + swz_sw(rr + 4 * h, (colA & 63) >> 3) + ((colA & 7) << 1)
                                                  : trswz(rr + 4 * h, colA >> 3) + ((colA & 7) << 1));
        }
    }

    // fragment reads of one K-half (ks) of a ring stage, and the MFMAs (+ bias sums) on them
    auto rd = [&](auto ustage, auto kc, u32x4 (&fa)[TMR], u32x4 (&fb)[W::TN]) {
        constexpr int U = decltype(ustage)::value, ks = decltype(kc)::value;
        const char* Gs = smem + U * W::GIMG;
        const char* Xs = smem + U * W::XSTRIDE;      // boff carries XBASE
#pragma unroll
        for (int t = 0; t < W::TN; ++t) {
            s16x4 b0 = ds_tr16(Xs, boff[ks][t][0]);
            s16x4 b1 = ds_tr16(Xs, boff[ks][t][1]);
            s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
            fb[t] = __builtin_bit_cast(u32x4, bv);
        }
#pragma unroll
        for (int tm = 0; tm < TMR; ++tm) {
            s16x4 a0 = ds_tr16(Gs, aoff[ks][tm][0]);
            s16x4 a1 = ds_tr16(Gs, aoff[ks][tm][1]);
            s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
            fa[tm] = __builtin_bit_cast(u32x4, av);
        }
    };
    constexpr bool BIAS_AFTER = CAI_WG_BIAS_AFTER && TMR <= 4;
    auto mm = [&](const u32x4 (&fa)[TMR], const u32x4 (&fb)[W::TN]) {
#pragma unroll
        for (int tm = 0; tm < TMR; ++tm) {
            if constexpr ((FLAGS & WG_BIAS) != 0 && !BIAS_AFTER) {
                if (do_bias && (tm & 3) == wc) {   // fragment tm's sums: column-wave tm % 4
                    const bf16x8 h = __builtin_bit_cast(bf16x8, fa[tm]);
                    float sacc = 0.f;
#pragma unroll
                    for (int e = 0; e < 8; ++e) sacc += (float)h[e];
                    bsum[tm] += sacc;
                }
            }
#pragma unroll
            for (int tn = 0; tn < W::TN; ++tn) acc[tm][tn] = mma16<bf16>(fa[tm], fb[tn], acc[tm][tn]);
        }
        // the bias sums behind the step's MFMAs (CAI_WG_BIAS_AFTER): ahead of them they delayed each fragment's issue
        // (not the 192-row tiles: six A fragments held to the end spill)
        if constexpr ((FLAGS & WG_BIAS) != 0 && BIAS_AFTER) {
            if (do_bias) {
#pragma unroll
                for (int tm = 0; tm < TMR; ++tm)
                    if ((tm & 3) == wc) bsum[tm] += sum8_bf16(fa[tm]);
            }
        }
        // transposed bias sums after the MFMAs: inside the read loop they made each B read wait
        if constexpr ((FLAGS & WG_TBIAS) != 0) {
#pragma unroll
            for (int t = 0; t < W::TN; ++t)
                if (tsel[t] >= 0) tsum[t] += sum8_bf16(fb[t]);
        }
    };
    using K0 = std::integral_constant<int, 0>;
    using K1 = std::integral_constant<int, 1>;

#pragma unroll
    for (int s = 0; s < W::NST - 1; ++s)
        if (s < nsteps) issue(s);
    // the ring position is a compile-time constant: the loop runs NST strips per trip
    for (int st0 = 0; st0 < nsteps; st0 += W::NST) {
        auto one = [&](auto ustage) {
            constexpr int U = decltype(ustage)::value;
            const int st = st0 + U;
            if (st >= nsteps) return;
            const int ahead = min(W::NST - 2, nsteps - 1 - st);   // later strips already issued
            if (ahead >= 2)
                wait_vmcnt<2 * W::NLOAD>();
            else if (ahead == 1)
                wait_vmcnt<W::NLOAD>();
            else
                wait_vmcnt<0>();
            wait_lgkmcnt0();
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (st + W::NST - 1 < nsteps) issue((U + W::NST - 1) % W::NST);
            u32x4 fa[TMR], fb[W::TN];
            rd(ustage, K0(), fa, fb);
            mm(fa, fb);
            rd(ustage, K1(), fa, fb);
            mm(fa, fb);
            __builtin_amdgcn_sched_barrier(0);
        };
        one(std::integral_constant<int, 0>());
        one(std::integral_constant<int, 1>());
        one(std::integral_constant<int, 2>());
        one(std::integral_constant<int, 3>());
    }
    if constexpr ((FLAGS & WG_BIAS) != 0) {
        if (do_bias) {   // wave (wr, wc) summed fragments wc, wc + 4 of its rows
#pragma unroll
            for (int tm = 0; tm < TMR; ++tm) {
                if ((tm & 3) != wc) continue;
                float v = bsum[tm];
                v += __shfl_xor(v, 16);
                v += __shfl_xor(v, 32);
                const int n = r0 + wr * (16 * TMR) + tm * 16 + lane;
                if (lane < 16 && n < a.Ng) a.bws[(int64_t)split * a.Ng + n] = v;
            }
        }
    }
    if constexpr ((FLAGS & WG_TBIAS) != 0) {
#pragma unroll
        for (int t = 0; t < W::TN; ++t) {
            float v = tsum[t];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            const int col = wcol + t * 16 + (lane & 15);
            if (lane < 16 && tsel[t] >= 0)
                a.bws[((int64_t)split * a.tb_s * a.tb_s + tsel[t]) * a.nbias + q0 + col % 64] = v;
        }
    }
#pragma unroll
    for (int tn = 0; tn < W::TN; ++tn) {
        const int col = wcol + tn * 16 + (lane & 15), kw = col / 64;
        const int gcol = (kh * KS + kw) * a.Cq_pad + q0 + col % 64;
#pragma unroll
        for (int tm = 0; tm < TMR; ++tm)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = r0 + wr * (16 * TMR) + tm * 16 + (lane >> 4) * 4 + r;
                if (row < a.Ng) out[(int64_t)row * a.ncols + gcol] = acc[tm][tn][r];
            }
    }
}

template <int KS, int S, int FLAGS, int R = 1, int TMR = 4>
__global__ __launch_bounds__(512, 1) void wgrad_halo_kernel(const WgradArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[WhCfg<KS, S, R, TMR == 6 ? 192 : 128>::BYTES];
    wgrad_halo_block<KS, S, FLAGS, R, TMR>(a, (int)blockIdx.x, (int)gridDim.x, smem);
}

template <int KS, int S, int FLAGS, int R = 1, int TMR = 4>
__global__ __launch_bounds__(512, 1) void wgrad_halo_batch_kernel(const WgBatch b) {
    __shared__ __attribute__((aligned(16))) char smem[WhCfg<KS, S, R, TMR == 6 ? 192 : 128>::BYTES];
    const int L = (int)blockIdx.x, j = wg_batch_job(b, L), l = L - b.start[j];
    if (l < b.nwg[j]) wgrad_halo_block<KS, S, FLAGS, R, TMR>(b.job[j], l, b.nwg[j], smem);
}

template <int KS, int S, int R = 1, int TMR = 4>
static void launch_wgrad_halo(const WgradArgs& a, int nblocks, int bias, hipStream_t st) {
    if (bias == WG_BIAS)
        hipLaunchKernelGGL((wgrad_halo_kernel<KS, S, WG_BIAS, R, TMR>), dim3(nblocks), dim3(512), 0, st, a);
    else if (S == 2 && bias == WG_TBIAS)
        hipLaunchKernelGGL((wgrad_halo_kernel<KS, S, WG_TBIAS, R, TMR>), dim3(nblocks), dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((wgrad_halo_kernel<KS, S, 0, R, TMR>), dim3(nblocks), dim3(512), 0, st, a);
}

template <int KS, int S, int R = 1, int TMR = 4>
static void launch_wgrad_halo_batch(const WgBatch& b, int bias, hipStream_t st) {
    const dim3 grid(b.start[b.n]);
    if (bias == WG_BIAS)
        hipLaunchKernelGGL((wgrad_halo_batch_kernel<KS, S, WG_BIAS, R, TMR>), grid, dim3(512), 0, st, b);
    else if (S == 2 && bias == WG_TBIAS)
        hipLaunchKernelGGL((wgrad_halo_batch_kernel<KS, S, WG_TBIAS, R, TMR>), grid, dim3(512), 0, st, b);
    else
        hipLaunchKernelGGL((wgrad_halo_batch_kernel<KS, S, 0, R, TMR>), grid, dim3(512), 0, st, b);
}

template <int CT>
static void launch_wgrad_glds_batch(const WgBatch& b, int f, hipStream_t st) {
    const dim3 grid(b.start[b.n]);
    switch (f) {
        case WG_TBIAS: hipLaunchKernelGGL((wgrad_glds_batch_kernel<CT, WG_TBIAS>), grid, dim3(512), 0, st, b); break;
        case 0: hipLaunchKernelGGL((wgrad_glds_batch_kernel<CT, 0>), grid, dim3(512), 0, st, b); break;
        case WG_ABS: hipLaunchKernelGGL((wgrad_glds_batch_kernel<CT, WG_ABS>), grid, dim3(512), 0, st, b); break;
        case WG_SQ: hipLaunchKernelGGL((wgrad_glds_batch_kernel<CT, WG_SQ>), grid, dim3(512), 0, st, b); break;
        case WG_BIAS: hipLaunchKernelGGL((wgrad_glds_batch_kernel<CT, WG_BIAS>), grid, dim3(512), 0, st, b); break;
        case WG_ABS | WG_BIAS:
            hipLaunchKernelGGL((wgrad_glds_batch_kernel<CT, WG_ABS | WG_BIAS>), grid, dim3(512), 0, st, b);
            break;
        default:
            hipLaunchKernelGGL((wgrad_glds_batch_kernel<CT, WG_SQ | WG_BIAS>), grid, dim3(512), 0, st, b);
            break;
    }
}

template <int CT>
static void launch_wgrad_glds(const WgradArgs& a, int nblocks, int in_abs, int in_sq, int bias, hipStream_t st) {
    const int f = (in_abs ? WG_ABS : 0) | (in_sq ? WG_SQ : 0) | bias;
    switch (f) {
        case WG_TBIAS: hipLaunchKernelGGL((wgrad_glds_kernel<CT, WG_TBIAS>), dim3(nblocks), dim3(512), 0, st, a); break;
        case 0: hipLaunchKernelGGL((wgrad_glds_kernel<CT, 0>), dim3(nblocks), dim3(512), 0, st, a); break;
        case WG_ABS: hipLaunchKernelGGL((wgrad_glds_kernel<CT, WG_ABS>), dim3(nblocks), dim3(512), 0, st, a); break;
        case WG_SQ: hipLaunchKernelGGL((wgrad_glds_kernel<CT, WG_SQ>), dim3(nblocks), dim3(512), 0, st, a); break;
        case WG_BIAS: hipLaunchKernelGGL((wgrad_glds_kernel<CT, WG_BIAS>), dim3(nblocks), dim3(512), 0, st, a); break;
        case WG_ABS | WG_BIAS:
            hipLaunchKernelGGL((wgrad_glds_kernel<CT, WG_ABS | WG_BIAS>), dim3(nblocks), dim3(512), 0, st, a);
            break;
        default:   // WG_SQ | WG_BIAS (GDN), WG_ABS | WG_SQ never requested
            hipLaunchKernelGGL((wgrad_glds_kernel<CT, WG_SQ | WG_BIAS>), dim3(nblocks), dim3(512), 0, st, a);
            break;
    }
}

// Column sums of a pixel-major tensor (bias gradients, GDN dbeta).
// stage 1: a block takes a pixel chunk and all channels: each thread owns one
// 16-byte channel group and strides over rows (vector loads, fp32 sums), then
// the rows reduce through LDS -> part[chunk][C].  stage 2: one block per 64
// channels, 16 waves over the chunks, fixed-order tree: deterministic.
constexpr int COLSUM_MAXC = 1 << 16;
template <typename T>
__global__ __launch_bounds__(256) void colsum_stage1(const T* __restrict__ g, int64_t npix, int C, int ld,
                                                     int64_t chunk, float* __restrict__ part) {
    constexpr int VEC = OpT<T>::VEC;
    __shared__ float red[256 * VEC];
    // blockIdx.y picks a slice of <= 256 channel groups (any C)
    const int cg0 = blockIdx.y * 256;
    const int cpt = min(256, (C + VEC - 1) / VEC - cg0);   // channel groups of this slice
    const int rows = 256 / cpt;               // rows in flight per pass
    const int tid = threadIdx.x;
    const int r = tid / cpt, cg = cg0 + tid - (tid / cpt) * cpt;
    const int64_t pb = blockIdx.x * chunk;
    int64_t pe = pb + chunk;
    if (pe > npix) pe = npix;
    float s[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) s[e] = 0.f;
    if (r < rows) {
        for (int64_t p = pb + r; p < pe; p += rows) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(g + p * ld + cg * VEC);
            if constexpr (VEC == 8) {
                const bf16x8 h = __builtin_bit_cast(bf16x8, v);
#pragma unroll
                for (int e = 0; e < 8; ++e) s[e] += (float)h[e];
            } else {
                const f32x4 f = __builtin_bit_cast(f32x4, v);
#pragma unroll
                for (int e = 0; e < 4; ++e) s[e] += f[e];
            }
        }
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) red[tid * VEC + e] = (r < rows) ? s[e] : 0.f;
    __syncthreads();
    for (int cl = tid; cl < cpt * VEC; cl += 256) {
        const int c = cg0 * VEC + cl;
        if (c >= C) break;
        const int g0 = cl / VEC, e = cl - (cl / VEC) * VEC;
        float acc = 0.f;
        for (int rr = 0; rr < rows; ++rr) acc += red[(rr * cpt + g0) * VEC + e];
        part[(int64_t)c * gridDim.x + blockIdx.x] = acc;
    }
}
__global__ __launch_bounds__(256) void colsum_stage2(const float* __restrict__ part, int nchunk, int C,
                                                     float* __restrict__ out, int accumulate) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= C) return;
    float s = 0.f;
    for (int i = lane; i < nchunk; i += 64) s += part[(int64_t)c * nchunk + i];
    s = wave_sum(s);
    if (lane == 0) out[c] = accumulate ? out[c] + s : s;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int round_up(int v, int m) { return (v + m - 1) / m * m; }

struct Plan {
    bool phase;      // phase (transposed) mode vs gather mode
    int nphase;
    int kin_c;       // channels of the kernel input (K channels)
    int kout_c;      // channels of the kernel output (N)
    int in_h, in_w, out_h, out_w;
    int Cin_pad, Npad, Kp;
    int ntaps[4], ntx[4], kh0[4], kw0[4], dy0[4], dx0[4], oy0[4], ox0[4], OHg[4], OWg[4];
    int step;
};

static int check_geom(const cai_conv_geom* g) {
    CAI_CHECK_ARG(g, "conv: null geometry");
    CAI_CHECK_ARG(g->batch > 0 && g->in_c > 0 && g->out_c > 0 && g->in_h > 0 && g->in_w > 0, "conv: bad sizes");
    CAI_CHECK_ARG(g->kernel >= 1 && g->kernel <= 7 && g->stride >= 1 && g->stride <= 2 && g->pad >= 0,
                  "conv: unsupported kernel %d stride %d pad %d", g->kernel, g->stride, g->pad);
    int oh, ow;
    if (g->transposed) {
        oh = (g->in_h - 1) * g->stride - 2 * g->pad + g->kernel + g->output_padding;
        ow = (g->in_w - 1) * g->stride - 2 * g->pad + g->kernel + g->output_padding;
    } else {
        CAI_CHECK_ARG(g->output_padding == 0, "conv: output_padding only for transposed");
        oh = (g->in_h + 2 * g->pad - g->kernel) / g->stride + 1;
        ow = (g->in_w + 2 * g->pad - g->kernel) / g->stride + 1;
    }
    CAI_CHECK_ARG(oh == g->out_h && ow == g->out_w, "conv: output size %dx%d != expected %dx%d", g->out_h, g->out_w, oh,
                  ow);
    CAI_CHECK_ARG(oh > 0 && ow > 0, "conv: empty output (%dx%d): input smaller than the kernel", oh, ow);
    return CAI_OK;
}

// direction 0 = forward, 1 = input gradient
static Plan make_plan(const cai_conv_geom* g, int dtype, int direction) {
    Plan P{};
    const int VEC = dtype == CAI_BF16 ? 8 : 4;
    const int BK = 128 / dtype_size(dtype);
    const int k = g->kernel, s = g->stride, p = g->pad;
    P.phase = (g->transposed != direction);
    if (direction == 0) {
        P.kin_c = g->in_c; P.kout_c = g->out_c;
        P.in_h = g->in_h; P.in_w = g->in_w; P.out_h = g->out_h; P.out_w = g->out_w;
    } else {
        P.kin_c = g->out_c; P.kout_c = g->in_c;
        P.in_h = g->out_h; P.in_w = g->out_w; P.out_h = g->in_h; P.out_w = g->in_w;
    }
    P.Cin_pad = round_up(P.kin_c, VEC);
    P.Npad = round_up(P.kout_c, 16);
    int kmax = 0;
    if (!P.phase) {
        P.nphase = 1;
        P.ntaps[0] = k * k; P.ntx[0] = k; P.kh0[0] = P.kw0[0] = 0;
        P.dy0[0] = P.dx0[0] = -p; P.oy0[0] = P.ox0[0] = 0;
        P.OHg[0] = P.out_h; P.OWg[0] = P.out_w;
        P.step = 1;
        kmax = k * k * P.Cin_pad;
    } else {
        P.nphase = s * s;
        P.step = s;
        for (int py = 0; py < s; ++py)
            for (int px = 0; px < s; ++px) {
                const int ph = py * s + px;
                const int kh0 = ((py + p) % s + s) % s, kw0 = ((px + p) % s + s) % s;
                const int na = kh0 < k ? (k - kh0 + s - 1) / s : 0;
                const int nc = kw0 < k ? (k - kw0 + s - 1) / s : 0;
                P.kh0[ph] = kh0; P.kw0[ph] = kw0;
                P.ntaps[ph] = na * nc; P.ntx[ph] = nc > 0 ? nc : 1;
                P.dy0[ph] = (py + p - kh0) / s; P.dx0[ph] = (px + p - kw0) / s;
                P.oy0[ph] = py; P.ox0[ph] = px;
                P.OHg[ph] = P.out_h > py ? (P.out_h - py + s - 1) / s : 0;
                P.OWg[ph] = P.out_w > px ? (P.out_w - px + s - 1) / s : 0;
                kmax = std::max(kmax, na * nc * P.Cin_pad);
            }
    }
    P.Kp = round_up(std::max(kmax, 1), BK);
    return P;
}

using CfgL = Cfg<128, 128, 2, 2>;
using CfgW = Cfg<64, 192, 1, 4>;
using CfgM = Cfg<128, 64, 2, 2>;
using CfgS = Cfg<256, 16, 4, 1>;

enum { CFG_L, CFG_W, CFG_M, CFG_S };

static int pick_cfg(int C, int& BM, int& BN) {
    int id;
    if (C <= 16) id = CFG_S;
    else if (C <= 64) id = CFG_M;
    else if (C % 128 != 0 && (C % 192 == 0 || C % 192 > 128 || (C > 128 && C <= 192))) id = CFG_W;
    else id = CFG_L;
    static const int bm[] = {128, 64, 128, 256}, bn[] = {128, 192, 64, 16};
    BM = bm[id];
    BN = bn[id];
    return id;
}

using CfgG1 = Cfg2<256, 128, 4, 2>;
using CfgG2 = Cfg2<128, 192, 2, 4>;
using CfgG3 = Cfg2<256, 64, 4, 2>;
using CfgG4 = Cfg2<128, 128, 2, 4>;
using CfgG5 = Cfg2<64, 128, 2, 4>;
using CfgG6 = Cfg2<64, 192, 2, 4>;
enum { CFG_G1 = 10, CFG_G2, CFG_G3, CFG_G4, CFG_G5, CFG_G6 };

// 64-row tiles for mid-size maps (cheng2020's attention units at 64x64, B = 4: M = 16384): where the 256 / 128-row
// grid would split K to fill the chip, the 64-row grid reaches >= 128 tiles without a split (no partial slab, no
// reduce launch).  A/B knob CAI_GLDS_M64=0.
static bool glds_m64_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_GLDS_M64");
        return e && *e == '0';
    }();
    return off;
}

static int pick_cfg_glds(int C, int nphase, int& BM, int& BN) {
    if (C <= 64) { BM = 256; BN = 64; return CFG_G3; }
    // phase mode: the s*s phases carry different tap counts (9/6/6/4 for k5 s2);
    // half-height tiles give the dispatcher enough blocks to balance them
    (void)nphase;
    if (C % 128 != 0 && (C % 192 == 0 || C % 192 > 128 || (C > 128 && C <= 192))) { BM = 128; BN = 192; return CFG_G2; }
    BM = 256; BN = 128;
    return CFG_G1;
}

// the LDS-DMA kernel needs bf16 operands read as stored (no |x| on load) and
// 64-channel K-tiles inside one tap
static bool glds_off32() {    // A/B knob: CAI_GLDS32_OFF=1 keeps 32-mod-64 input widths on conv_gemm_kernel
    static const bool off = [] {
        const char* e = getenv("CAI_GLDS32_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
static bool glds_eligible(const Plan& P, int dtype, int in_abs) {
    return dtype == CAI_BF16 && !in_abs && (P.Cin_pad % 64 == 0 || (P.Cin_pad % 32 == 0 && !glds_off32()));
}

// Launch geometry of one conv call: tiles, split-K factor and its workspace.
struct ConvLaunch {
    int cfg, BM, BN, mtiles, ntiles, mmax, ksplit, ws_ld;
    bool glds;
    int halo, tiles_x, tiles_y;    // halo: kernel size of the halo-staged path (0: not taken)
    bool halo_ph;                  // the halo-staged s^2-phase path (k5 s2 p2 transposed direction)
    bool halo_s1;                  // the halo-staged stride-1 k3 path
    int hbn;                       // output-channel tile of the halo phase / s1 paths (128 / 192)
    int small;                     // conv_small_kernel tile (SMALL_*; 0: not taken)
    size_t ws_bytes;
};

// latent-size problems: conv_small_kernel instead of split-K + reduce (A/B knob CAI_SMALL_CONV_OFF)
enum { SMALL_NONE = 0, SMALL_16x32, SMALL_32x32, SMALL_32x64 };
static bool small_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_SMALL_CONV_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
// Taken where it measured faster than split-K + reduce on MI355X (B=16 hyperprior, per-launch trace):
// M <= 512 rows (4x4 latents), or K <= 2048 with either <= 256 blocks or M <= 1024 (h_a[0] k3 192->128 at
// 16x16: 16.4 vs 22.8 us; h_s[0] 4->8: 9.3 vs 15.5).  At K = 3200 with M >= 1024 the per-wave K loop is
// latency-bound and the small tiles re-read the weights too often (g_a[6] 48.9 vs 22.6 us): split-K stays.
// Also taken where the big-tile grid has fewer than 64 blocks and K is too short to split (cheng2020's attention
// units at 16x16, B = 4: 1x1 96 <-> 192 on 4 blocks of 256 x 128 ran 16-25 us).
// A/B knob CAI_SMALL_CONV_KMAX (default 2048): the K bound of the second rule
static int small_kmax() {
    static const int v = [] {
        const char* e = getenv("CAI_SMALL_CONV_KMAX");
        return (e && *e) ? atoi(e) : 2048;
    }();
    return v;
}
// A/B knob CAI_SMALL_CONV_MMAX (default 1024): the row bound that lifts the 256-block limit of the second rule
static int small_mmax() {
    static const int v = [] {
        const char* e = getenv("CAI_SMALL_CONV_MMAX");
        return (e && *e) ? atoi(e) : 1024;
    }();
    return v;
}
// A/B knob CAI_SMALL_CONV_KMAX512 (default: no bound): the K bound of the first rule (M <= 512)
static int small_kmax512() {
    static const int v = [] {
        const char* e = getenv("CAI_SMALL_CONV_KMAX512");
        return (e && *e) ? atoi(e) : (1 << 30);
    }();
    return v;
}
static int pick_small(const Plan& P, int dtype, int mmax, int big_ksplit, int big_blocks) {
    if (small_off() || dtype != CAI_BF16 || P.Cin_pad % 32 != 0 || (big_ksplit <= 1 && big_blocks >= 64) ||
        mmax > 8192)
        return SMALL_NONE;
    int kmax = 0;
    for (int ph = 0; ph < P.nphase; ++ph) kmax = std::max(kmax, P.ntaps[ph] * P.Cin_pad);
    const int cfg = mmax <= 512 ? SMALL_16x32 : (mmax <= 2048 ? SMALL_32x32 : SMALL_32x64);
    static const int bm[] = {0, 16, 32, 32}, bn[] = {0, 32, 32, 64};
    const int blocks = (mmax + bm[cfg] - 1) / bm[cfg] * ((P.kout_c + bn[cfg] - 1) / bn[cfg]) * P.nphase;
    if ((mmax <= 512 && kmax <= small_kmax512()) || (kmax <= small_kmax() && (blocks <= 256 || mmax <= small_mmax())))
        return cfg;
    return SMALL_NONE;
}

// the halo-staged kernel: stride-2 gather convolutions with k in {3, 5}, pad k/2, <= 128 output channels
static bool halo_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_HALO_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
// A/B knob CAI_HALO_MIN_TILES (default 0): below this many 8 x 32 output tiles the gather layer goes to the
// LDS-DMA kernel (64-row tiles, no split-K) instead of the split-K halo kernel + reduce
static int halo_min_tiles() {
    static const int v = [] {
        const char* e = getenv("CAI_HALO_MIN_TILES");
        return (e && *e) ? atoi(e) : 0;
    }();
    return v;
}
static int halo_ks(const cai_conv_geom* g, const Plan& P, bool glds) {
    if (!glds || P.phase || halo_off() || g->stride != 2 || (g->kernel != 3 && g->kernel != 5) ||
        g->pad != g->kernel / 2 || P.Cin_pad % 32 != 0 || P.kout_c > 128 || P.OHg[0] < 8 || P.OWg[0] < 32)
        return 0;
    if (halo_min_tiles() > 0 &&
        (int64_t)g->batch * ((P.OWg[0] + 31) / 32) * ((P.OHg[0] + 7) / 8) < halo_min_tiles())
        return 0;
    return g->kernel;
}

// the halo-staged phase kernel: the s^2-phase direction of k5 s2 p2 (phase taps 3x3, 3x2, 2x3, 2x2),
// 64-channel input chunks, <= 128 output channels
static bool halo_phase_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_HALO_PH_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
// output-channel tile of the halo phase / s1 kernels: 128 up to 128 channels, else 192 unless the width
// is a multiple of 128 but not of 192 (256, 512: no padded columns)
static int halo_bn(int cout) { return (cout <= 128 || (cout % 128 == 0 && cout % 192 != 0)) ? 128 : 192; }
// 192-channel tiles only with >= 512 blocks: on C2' / C3' (B = 16) the 64x64 -> 128x128 layers gain (203 ->
// 176 us, 193 -> 176 us against conv_glds_kernel<128x192>) but the 32x32 -> 64x64 ones (256 blocks) lose
// (57 -> 61 us)
static bool halo_phase_ok(const cai_conv_geom* g, const Plan& P, bool glds, bool wide) {
    static const int nt[4] = {9, 6, 6, 4}, nx[4] = {3, 2, 3, 2};
    const int bn = halo_bn(P.kout_c);
    const int64_t blocks = 4ll * g->batch * ((P.OWg[0] + 31) / 32) * ((P.OHg[0] + 7) / 8) * ((P.kout_c + bn - 1) / bn);
    if (!glds || !P.phase || halo_off() || halo_phase_off() || P.nphase != 4 || g->stride != 2 || g->kernel != 5 || g->pad != 2 ||
        P.Cin_pad % 64 != 0 || (bn > 128 && (!wide || blocks < 512)) || P.OHg[0] < 8 || P.OWg[0] < 32)
        return false;
    for (int ph = 0; ph < 4; ++ph)
        if (P.ntaps[ph] != nt[ph] || P.ntx[ph] != nx[ph]) return false;
    return true;
}

// the halo-staged stride-1 k3 p1 kernel (both directions), 64-channel input chunks, any output width in
// BN-channel tiles; A/B knob CAI_HALO_S1_OFF
static bool halo_s1_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_HALO_S1_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
// Taken with >= 128 tiles: at B = 4 the 64x64 / 32x32 maps (16-64 tiles, split K) measured slower than
// conv_glds_kernel (192->192 64x64: 43 vs 38 us, 32x32: 31 vs 24 us; 128x128: 58 vs 73 us fwd, 71 vs 94 dgrad),
// and with > 64 output channels: 64-channel outputs fill half the 128-channel tile (multimodal 64->64 at
// 512x640 input gradient 200 vs 157 us on conv_glds_kernel<256x64>)
// Also taken with >= 64 tiles when the input is wide (Cin_pad >= CAI_HALO_S1_SPLIT_CIN, default 512; 0 = off): K
// splits at least four ways into chunks as long as a 192-channel layer's whole K, so the split blocks run the
// forward's per-block work (cheng2020's sub-pixel conv 192 -> 768 at 64x64, B = 4: its input gradient, K = 6912,
// ran 256 blocks of conv_glds_kernel<64x192> at 102 us)
static int halo_s1_split_cin() {
    static const int v = [] {
        const char* e = getenv("CAI_HALO_S1_SPLIT_CIN");
        return (e && *e) ? atoi(e) : 512;
    }();
    return v;
}
// 64-channel outputs on 256 x 64 halo tiles (conv_halo_s1_kernel<64>: the multimodal trunks' ResidualBlock(64, 64)
// 3x3 convs at 512x640, 17 each of forward / input gradient per step on conv_glds_kernel<256x64> at 0.10-0.12 of
// the bf16 peak, re-gathering the input per tap); A/B knob CAI_HALO_S1_BN64=0 keeps them there
static bool halo_s1_bn64() {
    static const bool on = [] {
        const char* e = getenv("CAI_HALO_S1_BN64");
        return !(e && *e == '0');
    }();
    return on;
}
static bool halo_s1_ok(const cai_conv_geom* g, const Plan& P, bool glds, bool wide) {
    const int bn = halo_bn(P.kout_c);
    const int64_t tiles = (int64_t)g->batch * ((P.OWg[0] + 31) / 32) * ((P.OHg[0] + 7) / 8) * ((P.kout_c + bn - 1) / bn);
    const bool split_wide = halo_s1_split_cin() > 0 && P.Cin_pad >= halo_s1_split_cin() && tiles >= 64;
    return glds && !halo_off() && !halo_s1_off() && g->stride == 1 && g->kernel == 3 && g->pad == 1 &&
           P.nphase == 1 && P.ntaps[0] == 9 && P.Cin_pad % 64 == 0 && (bn == 128 || wide) && P.OHg[0] >= 8 &&
           P.OWg[0] >= 32 && (tiles >= 128 || split_wide) && (P.kout_c > 64 || (P.kout_c == 64 && halo_s1_bn64()));
}


// A/B knob: an upper bound on the split-K factor of every conv launch (CAI_KSPLIT_MAX, read once; 0 = none)
static int ksplit_cap() {
    static const int cap = [] {
        const char* e = getenv("CAI_KSPLIT_MAX");
        return (e && *e) ? std::max(0, atoi(e)) : 0;
    }();
    return cap;
}
static int capped(int ks) { return ksplit_cap() > 0 ? std::max(1, std::min(ks, ksplit_cap())) : ks; }

// wide: the 192-channel halo tiles may be taken (their epilogue has no LDS path: the caller's output must
// satisfy epi_t_direct, or K must be split)
static ConvLaunch conv_launch(const cai_conv_geom* g, int dtype, int direction, int in_abs, bool wide = true) {
    const Plan P = make_plan(g, dtype, direction);
    ConvLaunch L{};
    L.glds = glds_eligible(P, dtype, in_abs);
    L.halo = halo_ks(g, P, L.glds);
    L.halo_ph = !L.halo && halo_phase_ok(g, P, L.glds, wide);
    L.halo_s1 = !L.halo && !L.halo_ph && halo_s1_ok(g, P, L.glds, wide);
    if (L.halo_ph || L.halo_s1) {
        const int np = L.halo_ph ? 4 : 1;
        L.hbn = (L.halo_s1 && P.kout_c == 64) ? 64 : halo_bn(P.kout_c);
        L.BM = 256;
        L.BN = L.hbn;
        L.tiles_x = (P.OWg[0] + 31) / 32;
        L.tiles_y = (P.OHg[0] + 7) / 8;
        for (int ph = 0; ph < np; ++ph) L.mmax = std::max(L.mmax, g->batch * P.OHg[ph] * P.OWg[ph]);
        L.mtiles = g->batch * L.tiles_x * L.tiles_y;
        L.ntiles = (P.kout_c + L.hbn - 1) / L.hbn;
        const int nch = P.Cin_pad / 64, blocks = np * L.mtiles * L.ntiles;
        L.ksplit = capped(blocks >= 256 ? 1 : std::min(nch, (256 + blocks - 1) / blocks));
        while (L.ksplit > 1 && (L.ksplit - 1) * ((nch + L.ksplit - 1) / L.ksplit) >= nch) --L.ksplit;
        L.ws_ld = L.ntiles * L.hbn;
        L.ws_bytes = L.ksplit > 1 ? (size_t)np * L.ksplit * L.mmax * L.ws_ld * sizeof(float) : 0;
        return L;
    }
    if (L.halo) {
        L.BM = 256;
        L.BN = 128;
        L.tiles_x = (P.OWg[0] + 31) / 32;
        L.tiles_y = (P.OHg[0] + 7) / 8;
        L.mmax = g->batch * P.OHg[0] * P.OWg[0];
        L.mtiles = g->batch * L.tiles_x * L.tiles_y;
        L.ntiles = 1;
        const int nch = P.Cin_pad / 32;
        L.ksplit = capped(L.mtiles >= 256 ? 1 : std::min(nch, (256 + L.mtiles - 1) / L.mtiles));
        // every split gets a chunk: per = ceil(nch / ks) must leave no empty split
        while (L.ksplit > 1 && (L.ksplit - 1) * ((nch + L.ksplit - 1) / L.ksplit) >= nch) --L.ksplit;
        L.ws_ld = 128;
        L.ws_bytes = L.ksplit > 1 ? (size_t)L.ksplit * L.mmax * L.ws_ld * sizeof(float) : 0;
        return L;
    }
    L.cfg = L.glds ? pick_cfg_glds(P.kout_c, P.nphase, L.BM, L.BN) : pick_cfg(P.kout_c, L.BM, L.BN);
    int kmax = 0;
    for (int ph = 0; ph < P.nphase; ++ph) {
        L.mmax = std::max(L.mmax, g->batch * P.OHg[ph] * P.OWg[ph]);
        kmax = std::max(kmax, P.ntaps[ph] * P.Cin_pad);
    }
    if (L.glds && !glds_m64_off() && (L.cfg == CFG_G1 || L.cfg == CFG_G2)) {
        const int nt = (P.kout_c + L.BN - 1) / L.BN;
        const int big = (L.mmax + L.BM - 1) / L.BM * nt * P.nphase;
        const int m64 = (L.mmax + 63) / 64 * nt * P.nphase;
        if (big < 256 && m64 >= 128) {
            L.cfg = L.cfg == CFG_G1 ? CFG_G5 : CFG_G6;
            L.BM = 64;
        }
    }
    L.mtiles = (L.mmax + L.BM - 1) / L.BM;
    L.ntiles = (P.kout_c + L.BN - 1) / L.BN;
    const int tiles = L.mtiles * L.ntiles * P.nphase;
    const int nk = (kmax + 128 / dtype_size(dtype) - 1) / (128 / dtype_size(dtype));
    // split K when the tile grid cannot fill the 256 CUs (small spatial layers);
    // each split keeps >= 4 K-tiles so the 2-deep prefetch still has work to hide
    int ks = 1;
    const int target = L.glds ? 256 : 512;    // one 512-thread block per CU vs two 256-thread ones
    if (tiles < 256) ks = std::min({(target + tiles - 1) / tiles, std::max(1, nk / 4), 16});
    L.ksplit = capped(std::max(1, ks));
    L.small = pick_small(P, dtype, L.mmax, L.ksplit, tiles * L.ksplit);
    if (L.small) {
        static const int bm[] = {0, 16, 32, 32}, bn[] = {0, 32, 32, 64};
        L.BM = bm[L.small];
        L.BN = bn[L.small];
        L.mtiles = (L.mmax + L.BM - 1) / L.BM;
        L.ntiles = (P.kout_c + L.BN - 1) / L.BN;
        L.ksplit = 1;
    }
    L.ws_ld = L.ntiles * L.BN;
    L.ws_bytes = L.ksplit > 1 ? (size_t)P.nphase * L.ksplit * L.mmax * L.ws_ld * sizeof(float) : 0;
    return L;
}

template <typename T, typename C>
static void launch_conv(const ConvArgs& a, const ConvLaunch& L, hipStream_t st) {
    dim3 grid(L.mtiles, L.ntiles, a.nphase * a.ksplit);
    hipLaunchKernelGGL((conv_gemm_kernel<T, C>), grid, dim3(NT), 0, st, a);
    if (a.ksplit > 1) {
        const int VO = (a.y_vec && a.y_dtype == CAI_BF16) ? 8 : 4;
        const int64_t total = (int64_t)L.mmax * ((a.Cout + VO - 1) / VO);
        const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (total + 255) / 256));
        hipLaunchKernelGGL((conv_splitk_reduce_kernel<T>), dim3(gx, a.nphase), dim3(256), 0, st, a);
    }
}

template <typename C>
static void launch_conv_glds(const ConvArgs& a, const ConvLaunch& L, hipStream_t st) {
    dim3 grid(L.mtiles, L.ntiles, a.nphase * a.ksplit);
    hipLaunchKernelGGL((conv_glds_kernel<C>), grid, dim3(512), 0, st, a);
    if (a.ksplit > 1) {
        const int VO = (a.y_vec && a.y_dtype == CAI_BF16) ? 8 : 4;
        const int64_t total = (int64_t)L.mmax * ((a.Cout + VO - 1) / VO);
        const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (total + 255) / 256));
        hipLaunchKernelGGL((conv_splitk_reduce_kernel<bf16>), dim3(gx, a.nphase), dim3(256), 0, st, a);
    }
}

static void launch_conv_halo(const ConvArgs& a, const ConvLaunch& L, hipStream_t st) {
    dim3 grid(L.mtiles, 1, a.ksplit);
    if (L.halo == 5)
        hipLaunchKernelGGL(conv_halo_kernel<5>, grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
    else
        hipLaunchKernelGGL(conv_halo_kernel<3>, grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
    if (a.ksplit > 1) {
        const int VO = (a.y_vec && a.y_dtype == CAI_BF16) ? 8 : 4;
        const int64_t total = (int64_t)L.mmax * ((a.Cout + VO - 1) / VO);
        const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (total + 255) / 256));
        hipLaunchKernelGGL((conv_splitk_reduce_kernel<bf16>), dim3(gx, 1), dim3(256), 0, st, a);
    }
}

// the four-phase kernel (conv_quad.hip) where every block of it gets a CU: >= 256 tiles, no split
static bool quad_grid(const ConvLaunch& L) { return L.halo_ph && L.hbn == 128 && L.ksplit == 1 && L.mtiles >= 256; }

static void launch_conv_halo_phase(const ConvArgs& a, const ConvLaunch& L, hipStream_t st) {
    const dim3 grid(L.halo_ph ? 4 * L.mtiles : L.mtiles, L.ntiles, a.ksplit);
    if (L.halo_ph) {
        if (quad_grid(L) && conv_quad_ok(a))
            launch_conv_halo_quad(a, L.tiles_x, L.tiles_y, L.mtiles, st);
        else if (L.hbn == 192)
            hipLaunchKernelGGL(conv_halo_phase_kernel<192>, grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
        else
            hipLaunchKernelGGL(conv_halo_phase_kernel<128>, grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
    } else {
        const bool gather = a.tap_sy > 0;
        if (L.hbn == 192) {
            if (gather)
                hipLaunchKernelGGL((conv_halo_s1_kernel<192, true>), grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
            else
                hipLaunchKernelGGL((conv_halo_s1_kernel<192, false>), grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
        } else if (L.hbn == 64) {
            if (gather)
                hipLaunchKernelGGL((conv_halo_s1_kernel<64, true>), grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
            else
                hipLaunchKernelGGL((conv_halo_s1_kernel<64, false>), grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
        } else {
            if (gather)
                hipLaunchKernelGGL((conv_halo_s1_kernel<128, true>), grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
            else
                hipLaunchKernelGGL((conv_halo_s1_kernel<128, false>), grid, dim3(512), 0, st, a, L.tiles_x, L.tiles_y);
        }
    }
    if (a.ksplit > 1) {
        const int VO = (a.y_vec && a.y_dtype == CAI_BF16) ? 8 : 4;
        const int64_t total = (int64_t)L.mmax * ((a.Cout + VO - 1) / VO);
        const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (total + 255) / 256));
        hipLaunchKernelGGL((conv_splitk_reduce_kernel<bf16>), dim3(gx, a.nphase), dim3(256), 0, st, a);
    }
}

static void launch_conv_small(const ConvArgs& a, const ConvLaunch& L, hipStream_t st) {
    const dim3 grid(L.mtiles, L.ntiles, a.nphase);
    if (L.small == SMALL_16x32)
        hipLaunchKernelGGL((conv_small_kernel<1, 2>), grid, dim3(512), 0, st, a);
    else if (L.small == SMALL_32x32)
        hipLaunchKernelGGL((conv_small_kernel<2, 2>), grid, dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((conv_small_kernel<2, 4>), grid, dim3(512), 0, st, a);
}

template <typename T>
static void dispatch_conv(const ConvArgs& a, const ConvLaunch& L, hipStream_t st) {
    if constexpr (sizeof(T) == 2) {
        if (L.small) {
            launch_conv_small(a, L, st);
            return;
        }
        if (L.halo) {
            launch_conv_halo(a, L, st);
            return;
        }
        if (L.halo_ph || L.halo_s1) {
            launch_conv_halo_phase(a, L, st);
            return;
        }
        switch (L.cfg) {
            case CFG_G1: launch_conv_glds<CfgG1>(a, L, st); return;
            case CFG_G2: launch_conv_glds<CfgG2>(a, L, st); return;
            case CFG_G3: launch_conv_glds<CfgG3>(a, L, st); return;
            case CFG_G4: launch_conv_glds<CfgG4>(a, L, st); return;
            case CFG_G5: launch_conv_glds<CfgG5>(a, L, st); return;
            case CFG_G6: launch_conv_glds<CfgG6>(a, L, st); return;
            default: break;
        }
    }
    switch (L.cfg) {
        case CFG_S: launch_conv<T, CfgS>(a, L, st); break;
        case CFG_M: launch_conv<T, CfgM>(a, L, st); break;
        case CFG_W: launch_conv<T, CfgW>(a, L, st); break;
        default: launch_conv<T, CfgL>(a, L, st); break;
    }
}

// (A split-K "fold" -- the last-arriving block of a tile sums the slabs, no reduce launch -- was measured and
// removed: C2 7530 vs 8594 patches/s, every agent-scope release writes back and every acquire invalidates the
// XCD's L2, and it needed a library-global device counter pool; profiles/r02_splitk_fold_ab.log.)
static int run_conv(const cai_conv_geom* g, int dtype, int direction, const void* x, int x_ld, int in_abs,
                    const void* w, const float* bias, int act, float act_param, void* y, int y_dtype, int64_t ysb,
                    int64_t ysc, int64_t ysy, int64_t ysx, const void* aux, int aux_ld, int mask_mode,
                    float mask_param, void* workspace, size_t ws_bytes, void* stream, const char* name,
                    const void* res = nullptr, int res_ld = 0, const void* res2 = nullptr, int res2_ld = 0) {
    int rc = check_geom(g);
    if (rc) return rc;
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "%s: bad dtype", name);
    CAI_CHECK_ARG(x && w && y, "%s: null pointer", name);
    const Plan P = make_plan(g, dtype, direction);
    ConvLaunch L = conv_launch(g, dtype, direction, in_abs);
    const int VEC = dtype == CAI_BF16 ? 8 : 4;
    CAI_CHECK_ARG(x_ld >= P.Cin_pad && x_ld % VEC == 0, "%s: input ld %d must be >= %d and a multiple of %d", name,
                  x_ld, P.Cin_pad, VEC);
    CAI_CHECK_ARG(((uintptr_t)x & 15) == 0, "%s: input not 16-byte aligned", name);
    CAI_CHECK_ARG((int64_t)g->batch * P.in_h * P.in_w * x_ld * dtype_size(dtype) < (1ll << 31),
                  "%s: input larger than 2 GiB", name);
    const int res_post = (mask_mode & CAI_MASK_BEFORE_RES) != 0;
    mask_mode &= ~CAI_MASK_BEFORE_RES;
    CAI_CHECK_ARG(mask_mode >= CAI_MASK_NONE && mask_mode <= CAI_MASK_SIGN, "%s: bad mask mode", name);
    CAI_CHECK_ARG(!res_post || (res && direction == 1 && mask_mode != CAI_MASK_NONE),
                  "%s: CAI_MASK_BEFORE_RES needs a residual, a mask and the dgrad direction", name);
    CAI_CHECK_ARG(!mask_mode || (aux && aux_ld >= P.kout_c), "%s: mask needs aux", name);
    CAI_CHECK_ARG(L.ws_bytes == 0 || (workspace && ws_bytes >= L.ws_bytes && ((uintptr_t)workspace & 15) == 0),
                  "%s: workspace of %zu bytes required", name, L.ws_bytes);
    ConvArgs a{};
    a.x = x; a.B = g->batch; a.IH = P.in_h; a.IW = P.in_w; a.x_ld = x_ld; a.Cin_pad = P.Cin_pad; a.in_abs = in_abs;
    a.w = w; a.Kp = P.Kp; a.Npad = P.Npad; a.nphase = P.nphase;
    a.tap_sy = P.phase ? -1 : 1; a.tap_sx = a.tap_sy;
    a.row_stride = P.phase ? 1 : g->stride;
    a.out_step = P.phase ? g->stride : 1;
    a.out_h = P.out_h; a.out_w = P.out_w; a.Cout = P.kout_c;
    a.y = y; a.y_dtype = y_dtype; a.ysb = ysb; a.ysc = ysc; a.ysy = ysy; a.ysx = ysx;
    const int VO = y_dtype == CAI_BF16 ? 8 : 4;
    a.y_vec = (ysc == 1 && ysx % VO == 0 && ysy % VO == 0 && ysb % VO == 0 && P.kout_c % VO == 0 &&
               ((uintptr_t)y & 15) == 0);
    a.bias = bias; a.act = act; a.act_param = act_param;
    a.aux = aux; a.aux_ld = aux_ld; a.mask_mode = mask_mode; a.mask_param = mask_param;
    // residual: bf16 pixel-major, 8-byte aligned 4-channel groups, added before the activation (forward) or to
    // the input gradient before its mask (dgrad)
    CAI_CHECK_ARG(!res || (direction != 2 && dtype == CAI_BF16 && a.y_vec && y_dtype == CAI_BF16 &&
                           (!mask_mode || direction == 1) &&
                           res_ld >= P.kout_c && res_ld % 4 == 0 && ((uintptr_t)res & 7) == 0),
                  "%s: residual needs a bf16 pixel-major output and res_ld >= Cout, a multiple of 4", name);
    CAI_CHECK_ARG(!res2 || (res && direction == 1 && res2_ld >= P.kout_c && res2_ld % 4 == 0 &&
                            ((uintptr_t)res2 & 7) == 0),
                  "%s: a second residual needs the first, the dgrad direction and res2_ld >= Cout, a multiple of 4",
                  name);
    a.res = reinterpret_cast<const bf16*>(res); a.res_ld = res_ld;
    a.res2 = reinterpret_cast<const bf16*>(res2); a.res2_ld = res2_ld;
    a.res_post = res_post;
    if ((L.halo_ph || L.halo_s1) && L.hbn > 128 && L.ksplit == 1 && !epi_t_direct(a))
        L = conv_launch(g, dtype, direction, in_abs, false);    // the 192-channel tiles store from registers only
    CAI_CHECK_ARG(!res_post || !(L.halo || L.halo_ph || L.halo_s1),
                  "%s: CAI_MASK_BEFORE_RES is not supported by the halo-staged tiles (%s)", name,
                  "check cai_conv_kernel_name first");
    CAI_CHECK_ARG(L.ws_bytes == 0 || (workspace && ws_bytes >= L.ws_bytes && ((uintptr_t)workspace & 15) == 0),
                  "%s: workspace of %zu bytes required", name, L.ws_bytes);
    a.ksplit = L.ksplit; a.ws = reinterpret_cast<float*>(workspace); a.ws_rows = L.mmax; a.ws_ld = L.ws_ld;
    for (int ph = 0; ph < P.nphase; ++ph) {
        PhaseDesc& d = a.ph[ph];
        d.oy0 = P.oy0[ph]; d.ox0 = P.ox0[ph]; d.OHg = P.OHg[ph]; d.OWg = P.OWg[ph];
        d.ntaps = P.ntaps[ph]; d.ntx = P.ntx[ph]; d.dy0 = P.dy0[ph]; d.dx0 = P.dx0[ph];
        d.K = P.ntaps[ph] * P.Cin_pad;
        d.w_off = (int64_t)ph * P.Npad * P.Kp;
    }
    if (L.mmax == 0) return CAI_OK;
    if (dtype == CAI_BF16)
        dispatch_conv<bf16>(a, L, as_stream(stream));
    else
        dispatch_conv<float>(a, L, as_stream(stream));
    CAI_LAUNCH_CHECK(name);
    return CAI_OK;
}

struct WgradPlan {
    int halo;        // kernel size of the halo-staged kernel (0: not taken); S then counts strip ranges
    int tbias, tb_kh0, tb_kw0;   // ConvTranspose2d bias from the X operand's tap set (WG_TBIAS)
    int Sb, nbias;               // bias partial slabs and their length
    int strips_per_split;
    int hrows;                   // halo kernel: rows (output channels) per tile, 128, 64 or 192
    bool glds, fused_bias;
    int ct;
    size_t ws_bias;
    int tiles;
    int Ng, Cq, Cq_pad, ncols, S, nsub, grp_len, px_chunk;
    int64_t M, split_len;
    int nchunk;
    int64_t chunk;
    size_t ws_slab, ws_col;
};

// the halo-staged wgrad: stride-2 gather geometry with k in {3, 5}, pad k/2, G width a multiple of 64,
// 64-channel X chunks (G channels beyond 128 take more row tiles)
static bool halo_wgrad_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_HALO_WGRAD_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
// A/B knob CAI_HALO_WGRAD_S1_OFF=1.  Measured before the weight-gradient DMAs moved to asm, the stride-1 form
// only tied wgrad_glds_kernel (117 vs 120 us); with both kernels' rings overlapping it wins: cheng2020-attn q6
// 192->192 at 128x128 122 -> 100 us, 64x64 44 -> 39 us (390 -> 397.6 patches/s); multimodal 256->256 at
// 512x640 1124 -> 976 us, 64->64 188 -> 123 us (profiles/r02_halo_wgrad_s1_ab.log)
static bool halo_wgrad_s1_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_HALO_WGRAD_S1_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
// G rows per 64-pixel strip: 1 for G widths that are multiples of 64, 2 / 4 for widths 32 / 16 (stride 2
// only, whole rows; A/B knob CAI_HALO_WGRAD_ROWS_OFF), 0: not taken
static bool halo_wgrad_rows_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_HALO_WGRAD_ROWS_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
static int halo_wgrad_rows(const cai_conv_geom* g) {
    const int Wg = g->transposed ? g->in_w : g->out_w, Hg = g->transposed ? g->in_h : g->out_h;
    if (Wg % 64 == 0) return 1;
    if (g->stride != 2 || halo_wgrad_rows_off()) return 0;
    const int R = Wg == 32 ? 2 : (Wg == 16 ? 4 : 0);
    return (R && Hg % R == 0) ? R : 0;
}
// stride 2 (k3/k5, pad k/2, both conv kinds) or the stride-1 k3 p1 Conv2d
static bool halo_wgrad_ks(const cai_conv_geom* g, const WgradPlan& W) {
    const bool s2 = g->stride == 2 && (g->kernel == 3 || g->kernel == 5) && g->pad == g->kernel / 2;
    const bool s1 = g->stride == 1 && g->kernel == 3 && g->pad == 1 && !g->transposed && !halo_wgrad_s1_off();
    return !halo_wgrad_off() && (s1 || s2) && halo_wgrad_rows(g) > 0 && W.Cq_pad % 64 == 0;
}

// ConvTranspose2d: an s x s block of taps (kh0 + a, kw0 + b) such that every output pixel is reached
// from exactly one (input pixel, tap) pair -- the bias gradient is then the sum of those taps' X columns
static bool tbias_axis(int k, int s, int p, int in, int out, int& k0) {
    for (k0 = 0; k0 + s <= k; ++k0) {
        bool ok = true;
        for (int o = 0; o < out && ok; ++o) {
            int cnt = 0;
            for (int kk = k0; kk < k0 + s; ++kk) {
                const int t = o + p - kk;
                if (t >= 0 && t % s == 0 && t / s < in) ++cnt;
            }
            ok = cnt == 1;
        }
        if (ok) return true;
    }
    return false;
}
static bool tbias_taps(const cai_conv_geom* g, int& kh0, int& kw0) {
    return g->transposed && tbias_axis(g->kernel, g->stride, g->pad, g->in_h, g->out_h, kh0) &&
           tbias_axis(g->kernel, g->stride, g->pad, g->in_w, g->out_w, kw0);
}

static int colsum_nchunk(int64_t npix) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(1024, (npix + 255) / 256));
}

// A/B knobs of the weight-gradient pixel splits (read once): CAI_WG_BLOCKS = target blocks per launch (default
// 256), CAI_WG_MIN_STRIPS = minimum 64-pixel strips per split of the halo kernels (default 4).  Fewer, larger
// splits shrink the fp32 partial slabs (S x Ng x k*k*Cq floats, summed by the reduce job).
static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e && *e) ? std::max(1, atoi(e)) : dflt;
}
static int wg_blocks() {
    static const int v = env_int("CAI_WG_BLOCKS", 256);
    return v;
}
static int wg_min_strips() {
    static const int v = env_int("CAI_WG_MIN_STRIPS", 4);
    return v;
}

// 64-row weight-gradient tiles for the k3 layers with Ng = 64 too (the 128-row tiles left half their rows empty:
// the multimodal trunks' 64 -> 64 3x3 convs); A/B knob CAI_HALO_WGRAD_K3_ROWS64=0 keeps 128
static bool halo_wgrad_rows64_k3() {
    static const bool on = [] {
        const char* e = getenv("CAI_HALO_WGRAD_K3_ROWS64");
        return !(e && *e == '0');
    }();
    return on;
}

static WgradPlan make_wgrad_plan(const cai_conv_geom* g, int dtype, bool glds, bool in_tf = false) {
    WgradPlan W{};
    W.glds = glds && dtype == CAI_BF16;
    const int VEC = dtype == CAI_BF16 ? 8 : 4;
    if (!g->transposed) {
        W.Ng = g->out_c; W.Cq = g->in_c;
        W.M = (int64_t)g->batch * g->out_h * g->out_w;
    } else {
        W.Ng = g->in_c; W.Cq = g->out_c;
        W.M = (int64_t)g->batch * g->in_h * g->in_w;
    }
    W.Cq_pad = round_up(W.Cq, VEC);
    W.ncols = g->kernel * g->kernel * W.Cq_pad;
    const int tiles = ((W.ncols + 127) / 128) * ((W.Ng + 127) / 128);
    // 8 pixel groups (one per XCD) x nsub workgroups per tile and group:
    // >= ~512 workgroups, >= 8 steps of 64 pixels per workgroup
    const int64_t per_grp = (W.M + 7) / 8;
    int nsub = std::max(1, (512 + 8 * tiles - 1) / (8 * tiles));
    nsub = (int)std::max<int64_t>(1, std::min<int64_t>(nsub, per_grp / 256));
    W.nsub = nsub;
    // chunk: at most WG_CHUNK, small enough that every sub gets one
    W.px_chunk = (int)std::min<int64_t>(WG_CHUNK, ((per_grp + nsub - 1) / nsub + 63) / 64 * 64);
    W.grp_len = (int)((per_grp + 63) / 64 * 64);
    W.S = 8 * nsub;
    W.split_len = 0;
    if (W.glds) {
        // one 512-thread block per CU: ~256 blocks of (256-col tile, pixel split)
        W.ct = W.ncols <= 128 ? 128 : 256;      // 1x1 layers (GDN, small deconv): half-width tile
        W.tiles = ((W.ncols + W.ct - 1) / W.ct) * ((W.Ng + 127) / 128);
        int S = std::max(1, wg_blocks() / W.tiles);
        S = (int)std::max<int64_t>(1, std::min<int64_t>(S, W.M / 256));
        W.split_len = ((W.M + S - 1) / S + 63) / 64 * 64;
        W.S = (int)((W.M + W.split_len - 1) / W.split_len);
    }
    if (W.glds && !in_tf && halo_wgrad_ks(g, W)) {
        W.halo = g->kernel;
        const int Wg = g->transposed ? g->in_w : g->out_w;
        const int Hg = g->transposed ? g->in_h : g->out_h;
        const int64_t nstrip = (int64_t)g->batch * Hg * Wg / 64;    // 64-pixel strips (R rows each)
        // 64-row tiles where 128 would leave rows empty (Ng = 192: a third of the MFMA work) -- for the k5 kernel
        // only: C2's g_a[6] / g_s[0] weight gradients 10198 -> 10265 patches/s, while cheng2020's k3 layers lost
        // 0.9 % (688 -> 682: half the MFMA work per step against the same per-step DMA and barrier, and more steps
        // per block; profiles/r05_halo_wgrad_64_rows_ab.log).  A/B knob CAI_HALO_WGRAD_ROWS128=1 keeps 128.
        static const bool rows128 = [] {
            const char* e = getenv("CAI_HALO_WGRAD_ROWS128");
            return e && *e == '1';
        }();
        W.hrows = (!rows128 && (W.halo == 5 || (W.Ng == 64 && halo_wgrad_rows64_k3())) && W.Ng % 128 != 0 &&
                   W.Ng % 64 == 0) ? 64 : 128;
        // 192-row tiles for the stride-1 k3 kernel at Ng = 192 k (cheng2020's 3x3 convs).  A/B knob
        // CAI_HALO_WGRAD_ROWS192=0 keeps 128.
        static const bool rows192 = [] {
            const char* e = getenv("CAI_HALO_WGRAD_ROWS192");
            return !(e && *e == '0');
        }();
        if (rows192 && !rows128 && W.halo == 3 && g->stride == 1 && halo_wgrad_rows(g) == 1 && W.Ng % 192 == 0 &&
            W.Ng % 128 != 0)
            W.hrows = 192;
        W.tiles = W.halo * (W.Cq_pad / 64) * ((W.Ng + W.hrows - 1) / W.hrows);
        // 192-row tiles: half the 256-block target by default (CAI_WG_BLOCKS_R192) -- the same pixel splits as the
        // 128-row tiles had, so the fp32 slab the reduce reads back does not double (cheng2020's 192-channel layers:
        // 9 tiles, 14 splits of 18.6 MB instead of 28 of 37 MB)
        static const int blocks192 = env_int("CAI_WG_BLOCKS_R192", 128);
        int S = std::max(1, (W.hrows == 192 ? blocks192 : wg_blocks()) / W.tiles);
        S = (int)std::max<int64_t>(1, std::min<int64_t>(S, nstrip / wg_min_strips()));   // >= 4 strips per split
        W.strips_per_split = (int)((nstrip + S - 1) / S);
        W.S = (int)((nstrip + W.strips_per_split - 1) / W.strips_per_split);
    }
    W.ws_slab = (size_t)W.S * W.Ng * W.ncols * sizeof(float);
    W.fused_bias = W.glds && !g->transposed;
    W.tbias = W.glds && g->transposed && !in_tf && tbias_taps(g, W.tb_kh0, W.tb_kw0);
    W.Sb = W.fused_bias ? W.S : (W.tbias ? W.S * g->stride * g->stride : 0);
    W.nbias = W.fused_bias ? W.Ng : W.Cq;
    W.ws_bias = W.Sb ? ((size_t)W.Sb * W.nbias * sizeof(float) + 255) / 256 * 256 : 0;
    // bias grad: columns of the module output gradient
    const int64_t npix_out = (int64_t)g->batch * g->out_h * g->out_w;
    W.nchunk = colsum_nchunk(npix_out);
    W.chunk = (npix_out + W.nchunk - 1) / W.nchunk;
    W.ws_col = (size_t)W.nchunk * g->out_c * sizeof(float);
    return W;
}

// the latent-size weight-gradient kernel: bf16, <= 1024 G pixels (8x8 latents at B = 16; at 4096 the
// pixel-split glds kernel + reduce measured faster: 21-34 vs 31-75 us), 64-channel tiles on both sides
static bool small_wgrad_off() {
    static const bool off = [] {
        const char* e = getenv("CAI_SMALL_WGRAD_OFF");
        return e && *e && *e != '0';
    }();
    return off;
}
// ... and with at most 2^20 weights: wider outputs (cheng2020 q6 at B = 4: 192->384 k5 and 192->768 k3 at 16x16,
// 192->768 k3 at 4x4) measured slower than the pixel-split kernel + reduce (134 / 71 / 91 vs 60 / 56 / 54 us,
// profiles/r03_cheng2020_dispatch_ab.log)
// G pixels up to which the latent-size weight gradient is taken: SW_NW * SW_STEPS * 32 = 1024 (straight-line
// steps); A/B knob CAI_SMALL_WGRAD_MMAX (e.g. 4096: C2's g_a[6] / g_s[0], 16 x 16 x 16 pixels, on the looped form)
static int64_t small_wgrad_mmax() {
    static const int64_t v = [] {
        const char* e = getenv("CAI_SMALL_WGRAD_MMAX");
        return (e && *e) ? (int64_t)atoi(e) : (int64_t)(SW_NW * SW_STEPS * 32);
    }();
    return v;
}
static bool small_wgrad_ok(const cai_conv_geom* g, int dtype) {
    const WgradPlan W = make_wgrad_plan(g, dtype, true);
    // 32-multiple channel counts take partial 64-wide tiles (cheng2020's 96 / 160 / 288-channel latent layers:
    // 127 us for the 8x8 288 -> 1152 sub-pixel conv's weight gradient on split slabs + reduce)
    // (A/B knob CAI_SMALL_WGRAD_W64=1: the round-3 rule, 64-multiples and <= 2^20 weights)
    static const bool w64 = [] {
        const char* e = getenv("CAI_SMALL_WGRAD_W64");
        return e && *e == '1';
    }();
    // at most 2^20 weights (A/B knob CAI_SMALL_WGRAD_WMAX = log2 of the bound): cheng2020's 288 -> 1152 k3 at 8x8
    // (3 M weights, 810 blocks of one K step per wave) ran faster on the pixel-split kernel, both deferred and
    // batched (C4 676.7 -> 680.4 patches/s, profiles/r05_small_wgrad_wmax_ab.log)
    static const int wmax = [] {
        const char* e = getenv("CAI_SMALL_WGRAD_WMAX");
        return (e && *e) ? atoi(e) : 20;
    }();
    const int gran = w64 ? 64 : 32;
    return !small_wgrad_off() && dtype == CAI_BF16 && W.M <= small_wgrad_mmax() && W.Ng % gran == 0 &&
           W.Cq_pad % gran == 0 && (int64_t)W.Ng * W.ncols <= ((int64_t)1 << wmax);
}


template <typename T>
static void launch_colsum(const void* g, int64_t npix, int C, int ld, int nchunk, int64_t chunk, float* part,
                          float* out, int accumulate, hipStream_t st) {
    const int nslice = ((C + OpT<T>::VEC - 1) / OpT<T>::VEC + 255) / 256;
    hipLaunchKernelGGL(colsum_stage1<T>, dim3(nchunk, nslice), dim3(256), 0, st, reinterpret_cast<const T*>(g), npix, C, ld,
                       chunk, part);
    hipLaunchKernelGGL(colsum_stage2, dim3((C + 3) / 4), dim3(256), 0, st, part, nchunk, C, out, accumulate);
}

}  // namespace cai

using namespace cai;

extern "C" {

size_t cai_conv_packed_weight_bytes(const cai_conv_geom* g, int dtype, int direction) {
    if (check_geom(g)) return 0;
    const Plan P = make_plan(g, dtype, direction);
    return (size_t)P.nphase * P.Npad * P.Kp * dtype_size(dtype);
}

static int fill_pack_args(const cai_conv_geom* g, int dtype, int direction, const float* w, const float* mask,
                          void* packed, PackArgs& a) {
    int rc = check_geom(g);
    if (rc) return rc;
    CAI_CHECK_ARG(direction == 0 || direction == 1, "pack_weight: bad direction");
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "pack_weight: bad dtype");
    CAI_CHECK_ARG(w && packed, "pack_weight: null pointer");
    const Plan P = make_plan(g, dtype, direction);
    a = PackArgs{};
    a.w = w; a.mask = mask; a.out = packed;
    a.k = g->kernel;
    // torch layout: Conv2d [out][in][k][k], ConvTranspose2d [in][out][k][k]
    a.D1 = g->transposed ? g->out_c : g->in_c;
    a.n_is_d0 = (g->transposed == direction);
    a.Nreal = P.kout_c; a.Creal = P.kin_c; a.Cpad = P.Cin_pad; a.Npad = P.Npad; a.Kp = P.Kp;
    a.nphase = P.nphase; a.step = P.step;
    for (int ph = 0; ph < P.nphase; ++ph) {
        a.ntaps[ph] = P.ntaps[ph]; a.ntx[ph] = P.ntx[ph]; a.kh0[ph] = P.kh0[ph]; a.kw0[ph] = P.kw0[ph];
        a.off[ph] = (int64_t)ph * P.Npad * P.Kp;
    }
    return CAI_OK;
}

int cai_conv_pack_weight(const cai_conv_geom* g, int dtype, int direction, const float* w, const float* mask,
                         void* packed, void* stream) {
    PackArgs a;
    const int rc = fill_pack_args(g, dtype, direction, w, mask, packed, a);
    if (rc) return rc;
    const int64_t total = (int64_t)a.Npad * a.Kp;
    const int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(pack_weight_kernel<bf16>, dim3(blocks, 1, a.nphase), dim3(256), 0, as_stream(stream), a);
    else
        hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(blocks, 1, a.nphase), dim3(256), 0, as_stream(stream), a);
    CAI_LAUNCH_CHECK("pack_weight");
    return CAI_OK;
}

size_t cai_conv_pack_desc_bytes(void) { return sizeof(PackArgs); }

int cai_conv_pack_describe(const cai_conv_geom* g, int dtype, int direction, const float* w, const float* mask,
                           void* packed, void* desc) {
    CAI_CHECK_ARG(desc, "pack_describe: null descriptor");
    PackArgs a;
    const int rc = fill_pack_args(g, dtype, direction, w, mask, packed, a);
    if (rc) return rc;
    memcpy(desc, &a, sizeof(a));
    return CAI_OK;
}

int cai_edge_pack_describe(const cai_conv_geom* g, int dtype, int direction, const float* w, void* frag, void* desc) {
    CAI_CHECK_ARG(desc && w && frag, "edge_pack_describe: null pointer");
    PackArgs a{};
    CAI_CHECK_ARG(edge_frag_spec(g, dtype, direction, a.es), "edge_pack_describe: unsupported geometry / direction");
    a.w = w;
    a.out = frag;
    a.edge = 1;
    a.nphase = 1;
    a.Npad = a.es.nfrag * 8;   // finalize: items_pp = Npad * Kp / 8 = one item per fragment
    a.Kp = 1;
    memcpy(desc, &a, sizeof(a));
    return CAI_OK;
}

int cai_gdn_reparam_describe(const float* beta_raw, const float* gamma_raw, int32_t C, float beta_min,
                             float reparam_offset, float* beta, void* gamma_op, void* desc) {
    CAI_CHECK_ARG(desc && beta_raw && gamma_raw && beta && gamma_op && C > 0, "gdn_reparam_describe: bad arguments");
    PackArgs a{};
    const float ped = reparam_offset * reparam_offset;
    a.gdn = 1;
    a.w = gamma_raw;
    a.mask = beta_raw;
    a.out = gamma_op;
    a.D1 = C;
    a.gdn_beta = beta;
    a.gdn_bb = sqrtf(beta_min + ped);
    a.gdn_gb = sqrtf(0.f + ped);
    a.gdn_ped = ped;
    a.nphase = 1;
    a.Npad = (int)(((int64_t)C * C + 7) / 8 * 8);   // finalize: one item per 8 gamma entries
    a.Kp = 1;
    memcpy(desc, &a, sizeof(a));
    return CAI_OK;
}

int64_t cai_conv_pack_finalize(void* descs, int32_t n) {
    if (!descs || n <= 0) return -1;
    PackArgs* d = reinterpret_cast<PackArgs*>(descs);
    // tile mode for conv descriptors with k*k <= 25 (the two directions of one weight, consecutive in the table,
    // share their tiles), row mode for the other conv descriptors whose source row fits the LDS copy; zero-size
    // entries in the other numberings keep every begin array non-decreasing (a unit's descriptor is the LAST one
    // at or below it)
    int64_t items = 0, rows = 0, tiles = 0;
    auto conv_desc = [&](int i) { return !d[i].edge && !d[i].gdn; };
    auto src_ext = [&](const PackArgs& x, int& e0, int& e1) {   // source entries the tiles cover (padding included)
        e0 = x.n_is_d0 ? x.Npad : x.Cpad;
        e1 = x.n_is_d0 ? x.Cpad : x.Npad;
    };
    for (int i = 0; i < n; ++i) {
        d[i].tilemode = d[i].pair = 0;
        d[i].tile_begin = tiles;
        if (!conv_desc(i) || d[i].k * d[i].k > 25 || !PACK_TILES) continue;
        if (i > 0 && d[i - 1].tilemode == 1 && d[i - 1].pair) {
            d[i].tilemode = 2;
            continue;
        }
        PackArgs& x = d[i];
        const int kk = x.k * x.k;
        static const int cand[][2] = {{128, 64}, {64, 64}, {32, 64}, {32, 32}, {16, 32}, {16, 16}, {8, 16}, {8, 8}};
        x.td0 = x.td1 = 0;
        for (const auto& c : cand)
            if ((int64_t)kk * (c[0] * (c[1] + 4) + 4) <= PACK_TILE_FLOATS) {
                x.td0 = c[0];
                x.td1 = c[1];
                break;
            }
        x.tdp = x.td1 + 4;
        x.tstride = x.td0 * x.tdp + 4;
        x.d0real = x.n_is_d0 ? x.Nreal : x.Creal;
        x.d1real = x.n_is_d0 ? x.Creal : x.Nreal;
        x.mrl = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)(x.td1 * kk) - 1) / (uint64_t)(x.td1 * kk));
        x.mkk = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)kk - 1) / (uint64_t)kk);
        int e0, e1;
        src_ext(x, e0, e1);
        if (i + 1 < n && conv_desc(i + 1)) {
            const PackArgs& y = d[i + 1];
            if (y.w == x.w && y.mask == x.mask && y.k == x.k && y.D1 == x.D1 && y.n_is_d0 != x.n_is_d0 &&
                (y.n_is_d0 ? y.Nreal : y.Creal) == x.d0real && (y.n_is_d0 ? y.Creal : y.Nreal) == x.d1real) {
                int f0, f1;
                src_ext(y, f0, f1);
                e0 = std::max(e0, f0);
                e1 = std::max(e1, f1);
                x.pair = 1;
            }
        }
        x.tilemode = 1;
        x.tn1 = (e1 + x.td1 - 1) / x.td1;
        tiles += (int64_t)((e0 + x.td0 - 1) / x.td0) * x.tn1;
    }
    for (int i = 0; i < n; ++i) {
        d[i].items_pp = (int)((int64_t)d[i].Npad * d[i].Kp / 8);
        d[i].rowmode = !d[i].tilemode && !d[i].edge && !d[i].gdn && d[i].Creal * d[i].k * d[i].k <= PACK_ROW_MAX;
        d[i].rpu = d[i].rowmode ? std::max(1, std::min(PACK_ROWS_PER_UNIT, PACK_ROW_MAX / (d[i].Creal * d[i].k * d[i].k)))
                                : 1;
        d[i].item_begin = items;
        d[i].row_begin = rows;
        if (d[i].tilemode)
            continue;
        if (d[i].rowmode)
            rows += (d[i].Npad + d[i].rpu - 1) / d[i].rpu;
        else
            items += (int64_t)d[i].items_pp * d[i].nphase;
    }
    for (int i = 0; i < n; ++i) {
        d[i].rows_total = rows;
        d[i].tiles_total = tiles;
    }
    return tiles + rows + items;
}

int cai_conv_pack_many(const void* descs, int32_t n, int dtype, int64_t total_items, void* stream) {
    CAI_CHECK_ARG(descs && n > 0 && total_items > 0, "pack_many: bad arguments");
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "pack_many: bad dtype");
    CAI_CHECK_ARG(((uintptr_t)descs & 7) == 0, "pack_many: descriptor table not 8-byte aligned");
    // work units: one block per row-mode row, one per 256 items; total_items = rows + items bounds them
    const int blocks = (int)std::min<int64_t>(8192, total_items);
    const PackArgs* d = reinterpret_cast<const PackArgs*>(descs);
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(pack_many_kernel<bf16>, dim3(blocks), dim3(256), 0, as_stream(stream), d, n, total_items);
    else
        hipLaunchKernelGGL(pack_many_kernel<float>, dim3(blocks), dim3(256), 0, as_stream(stream), d, n, total_items);
    CAI_LAUNCH_CHECK("pack_many");
    return CAI_OK;
}

int cai_pack_nchw(const float* x, int32_t B, int32_t C, int32_t H, int32_t W, int dtype, void* out, int32_t ld,
                  void* stream) {
    CAI_CHECK_ARG(x && out && B > 0 && C > 0 && H > 0 && W > 0 && ld >= C && ld % 8 == 0, "pack_nchw: bad arguments");
    const int64_t total = (int64_t)B * H * W * ld;
    const int blocks = (int)std::min<int64_t>(8192, (total + 255) / 256);
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(pack_nchw_kernel<bf16>, dim3(blocks), dim3(256), 0, as_stream(stream), x, B, C, H * W,
                           reinterpret_cast<bf16*>(out), ld);
    else
        hipLaunchKernelGGL(pack_nchw_kernel<float>, dim3(blocks), dim3(256), 0, as_stream(stream), x, B, C, H * W,
                           reinterpret_cast<float*>(out), ld);
    CAI_LAUNCH_CHECK("pack_nchw");
    return CAI_OK;
}

size_t cai_conv_workspace_bytes(const cai_conv_geom* g, int dtype, int direction) {
    if (check_geom(g)) return 0;
    // the kernel choice may depend on in_abs (not known here): cover both
    // and on whether the output allows the 192-channel halo tiles (run_conv falls back)
    return std::max({conv_launch(g, dtype, direction, 0).ws_bytes, conv_launch(g, dtype, direction, 1).ws_bytes,
                     conv_launch(g, dtype, direction, 0, false).ws_bytes});
}

int cai_conv_fwd(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, int32_t in_abs, const void* packed_w,
                 const float* bias, int32_t act, float act_param, void* y, int y_dtype, int64_t ysb, int64_t ysc,
                 int64_t ysy, int64_t ysx, void* workspace, size_t ws_bytes, void* stream) {
    return run_conv(g, dtype, 0, x, x_ld, in_abs, packed_w, bias, act, act_param, y, y_dtype, ysb, ysc, ysy, ysx,
                    nullptr, 0, CAI_MASK_NONE, 0.f, workspace, ws_bytes, stream, "conv_fwd");
}

int cai_conv_fwd_res(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, int32_t in_abs,
                     const void* packed_w, const float* bias, int32_t act, float act_param, const void* res,
                     int32_t res_ld, void* y, int y_dtype, int64_t ysb, int64_t ysc, int64_t ysy, int64_t ysx,
                     void* workspace, size_t ws_bytes, void* stream) {
    CAI_CHECK_ARG(res, "conv_fwd_res: null residual");
    return run_conv(g, dtype, 0, x, x_ld, in_abs, packed_w, bias, act, act_param, y, y_dtype, ysb, ysc, ysy, ysx,
                    nullptr, 0, CAI_MASK_NONE, 0.f, workspace, ws_bytes, stream, "conv_fwd_res", res, res_ld);
}

int cai_conv_dgrad(const cai_conv_geom* g, int dtype, const void* dy, int32_t dy_ld, const void* packed_wt, void* dx,
                   int32_t dx_ld, int32_t mask_mode, float mask_param, const void* aux, int32_t aux_ld,
                   void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_geom(g);
    if (rc) return rc;
    const int64_t ld = dx_ld;
    return run_conv(g, dtype, 1, dy, dy_ld, 0, packed_wt, nullptr, CAI_ACT_NONE, 0.f, dx, dtype,
                    (int64_t)g->in_h * g->in_w * ld, 1, (int64_t)g->in_w * ld, ld, aux, aux_ld, mask_mode,
                    mask_param, workspace, ws_bytes, stream, "conv_dgrad");
}

int cai_conv_dgrad_res(const cai_conv_geom* g, int dtype, const void* dy, int32_t dy_ld, const void* packed_wt,
                       const void* res, int32_t res_ld, void* dx, int32_t dx_ld, int32_t mask_mode, float mask_param,
                       const void* aux, int32_t aux_ld, void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_geom(g);
    if (rc) return rc;
    CAI_CHECK_ARG(res, "conv_dgrad_res: null residual");
    const int64_t ld = dx_ld;
    return run_conv(g, dtype, 1, dy, dy_ld, 0, packed_wt, nullptr, CAI_ACT_NONE, 0.f, dx, dtype,
                    (int64_t)g->in_h * g->in_w * ld, 1, (int64_t)g->in_w * ld, ld, aux, aux_ld, mask_mode, mask_param,
                    workspace, ws_bytes, stream, "conv_dgrad_res", res, res_ld);
}

int cai_conv_dgrad_res2(const cai_conv_geom* g, int dtype, const void* dy, int32_t dy_ld, const void* packed_wt,
                        const void* res, int32_t res_ld, const void* res2, int32_t res2_ld, void* dx, int32_t dx_ld,
                        int32_t mask_mode, float mask_param, const void* aux, int32_t aux_ld, void* workspace,
                        size_t ws_bytes, void* stream) {
    int rc = check_geom(g);
    if (rc) return rc;
    CAI_CHECK_ARG(res && res2, "conv_dgrad_res2: null residual");
    const int64_t ld = dx_ld;
    return run_conv(g, dtype, 1, dy, dy_ld, 0, packed_wt, nullptr, CAI_ACT_NONE, 0.f, dx, dtype,
                    (int64_t)g->in_h * g->in_w * ld, 1, (int64_t)g->in_w * ld, ld, aux, aux_ld, mask_mode, mask_param,
                    workspace, ws_bytes, stream, "conv_dgrad_res2", res, res_ld, res2, res2_ld);
}

const char* cai_conv_kernel_name(const cai_conv_geom* g, int dtype, int direction, int32_t in_abs) {
    if (check_geom(g) || (dtype != CAI_BF16 && dtype != CAI_F32) || direction < 0 || direction > 2) return "";
    if (direction == 2) {
        if (small_wgrad_ok(g, dtype)) return "wgrad_small_kernel";
        const WgradPlan W = make_wgrad_plan(g, dtype, true, in_abs != 0);
        if (!W.glds) return dtype == CAI_BF16 ? "wgrad_kernel<bf16>" : "wgrad_kernel<float>";
        if (W.halo) {
            static const char* const nm[2][5] = {{"", "wgrad_halo_kernel<3>", "wgrad_halo_kernel<3,r2>", "",
                                                  "wgrad_halo_kernel<3,r4>"},
                                                 {"", "wgrad_halo_kernel<5>", "wgrad_halo_kernel<5,r2>", "",
                                                  "wgrad_halo_kernel<5,r4>"}};
            if (g->stride == 1) return "wgrad_halo_kernel<3,s1>";
            return nm[W.halo == 5][halo_wgrad_rows(g)];
        }
        return W.ct == 256 ? "wgrad_glds_kernel<256>" : "wgrad_glds_kernel<128>";
    }
    const ConvLaunch L = conv_launch(g, dtype, direction, in_abs);
    if (L.halo) return L.halo == 5 ? "conv_halo_kernel<5>" : "conv_halo_kernel<3>";
    if (L.halo_ph) {
        if (quad_grid(L) && dtype == CAI_BF16) {
            // the four-phase kernel when the output takes the register-direct epilogue (bf16, no mask / residual)
            const Plan P = make_plan(g, dtype, direction);
            ConvArgs a{};
            a.nphase = P.nphase; a.Cin_pad = P.Cin_pad; a.Cout = P.kout_c; a.Npad = P.Npad; a.ksplit = L.ksplit;
            a.out_step = P.phase ? g->stride : 1; a.in_abs = in_abs; a.y_vec = 1; a.y_dtype = CAI_BF16;
            a.x_ld = P.Cin_pad;
            for (int ph = 0; ph < P.nphase; ++ph) {
                a.ph[ph].ntaps = P.ntaps[ph]; a.ph[ph].ntx = P.ntx[ph]; a.ph[ph].dy0 = P.dy0[ph];
                a.ph[ph].dx0 = P.dx0[ph]; a.ph[ph].oy0 = P.oy0[ph]; a.ph[ph].ox0 = P.ox0[ph];
            }
            if (conv_quad_ok(a)) return "conv_halo_quad_kernel";
        }
        return L.hbn == 192 ? "conv_halo_phase_kernel<192>" : "conv_halo_phase_kernel";
    }
    if (L.halo_s1)
        return L.hbn == 192 ? "conv_halo_s1_kernel<192>" : (L.hbn == 64 ? "conv_halo_s1_kernel<64>" : "conv_halo_s1_kernel<128>");
    if (L.small) return L.small == SMALL_16x32 ? "conv_small_kernel<16x32>"
                        : (L.small == SMALL_32x32 ? "conv_small_kernel<32x32>" : "conv_small_kernel<32x64>");
    switch (L.cfg) {
        case CFG_G1: return "conv_glds_kernel<256x128>";
        case CFG_G2: return "conv_glds_kernel<128x192>";
        case CFG_G3: return "conv_glds_kernel<256x64>";
        case CFG_G4: return "conv_glds_kernel<128x128>";
        case CFG_G5: return "conv_glds_kernel<64x128>";
        case CFG_G6: return "conv_glds_kernel<64x192>";
        case CFG_S: return dtype == CAI_BF16 ? "conv_gemm_kernel<bf16,256x16>" : "conv_gemm_kernel<float,256x16>";
        case CFG_M: return dtype == CAI_BF16 ? "conv_gemm_kernel<bf16,128x64>" : "conv_gemm_kernel<float,128x64>";
        case CFG_W: return dtype == CAI_BF16 ? "conv_gemm_kernel<bf16,64x192>" : "conv_gemm_kernel<float,64x192>";
        default: return dtype == CAI_BF16 ? "conv_gemm_kernel<bf16,128x128>" : "conv_gemm_kernel<float,128x128>";
    }
}

int32_t cai_conv_split_factor(const cai_conv_geom* g, int dtype, int direction, int32_t in_abs) {
    if (check_geom(g) || (dtype != CAI_BF16 && dtype != CAI_F32) || direction < 0 || direction > 2) return 0;
    if (direction == 2) return make_wgrad_plan(g, dtype, true, in_abs != 0).S;
    return conv_launch(g, dtype, direction, in_abs).ksplit;
}

size_t cai_conv_wgrad_workspace_bytes(const cai_conv_geom* g, int dtype) {
    if (check_geom(g)) return 0;
    // the plan depends on whether the input is transformed (|x|, x^2): cover every variant
    const WgradPlan W0 = make_wgrad_plan(g, dtype, false), W1 = make_wgrad_plan(g, dtype, true),
                    W2 = make_wgrad_plan(g, dtype, true, true);
    return std::max({W0.ws_slab + W0.ws_col, W1.ws_slab + W1.ws_bias + W1.ws_col,
                     W2.ws_slab + W2.ws_bias + W2.ws_col}) + 256;
}

// The latent-size weight gradient's arguments, grid and (slab -> torch layout) reduce job; `a` carries the
// operand roles run_conv_wgrad set up (Conv2d: G = dy, X = x; ConvTranspose2d: the other way round).
static int small_wgrad_setup(const cai_conv_geom* g, const WgradPlan& W, const WgradArgs& a, const void* dy,
                             int32_t dy_ld, float* dw, float* db, int32_t accumulate, float* slab, SwArgs& sa,
                             dim3& grid, cai_reduce_job& J) {
    sa = SwArgs{};
    sa.g = a.g; sa.g_ld = a.g_ld; sa.Ng = W.Ng;
    sa.x = a.x; sa.x_ld = a.x_ld; sa.Cq = W.Cq; sa.Cq_pad = W.Cq_pad; sa.in_abs = a.in_abs; sa.in_sq = a.in_sq;
    sa.B = g->batch; sa.Hg = a.Hg; sa.Wg = a.Wg; sa.Hx = a.Hx; sa.Wx = a.Wx;
    sa.k = g->kernel; sa.s = g->stride; sa.p = g->pad;
    sa.M = (int)W.M; sa.cbt = (W.Cq_pad + 63) / 64; sa.ncb = g->kernel * g->kernel * sa.cbt;
    sa.dw = dw; sa.accumulate = accumulate;
    sa.bsrc = dy; sa.bsrc_ld = dy_ld; sa.bnpix = g->batch * g->out_h * g->out_w; sa.bc = g->out_c; sa.db = db;
    sa.bias_from_g = !g->transposed;
    sa.inv_plane = 1.f / (float)(a.Hg * a.Wg);
    sa.inv_wg = 1.f / (float)a.Wg;
    CAI_CHECK_ARG((int64_t)sa.bnpix * dy_ld * 2 < (1ll << 31) && (int64_t)a.B * a.Hx * a.Wx * a.x_ld * 2 < (1ll << 31),
                  "conv_wgrad: operand larger than 2 GiB");
    // dW through a one-split slab and a WGRAD job (deferred: joins the backward's batched reduce launch);
    // A/B knob CAI_SMALL_WGRAD_DIRECT=1: straight into the torch layout (scattered stores)
    static const bool direct_out = [] {
        const char* e = getenv("CAI_SMALL_WGRAD_DIRECT");
        return e && *e == '1';
    }();
    sa.slab = direct_out ? nullptr : slab;
    grid = dim3(sa.ncb + ((db && g->transposed) ? 1 : 0), (W.Ng + 63) / 64);
    J = cai_reduce_job{};
    if (direct_out) return CAI_OK;
    J.kind = CAI_JOB_WGRAD;
    J.nblocks = wgrad_job_blocks(W.Ng, W.Cq_pad, g->kernel, 0);
    J.p[0] = slab; J.p[1] = dw;
    J.i[0] = 1; J.i[1] = W.Ng; J.i[2] = W.ncols; J.i[3] = W.Cq; J.i[4] = W.Cq_pad; J.i[5] = g->kernel;
    J.i[6] = accumulate;
    return CAI_OK;
}

static void launch_wgrad_small(const SwArgs& sa, dim3 grid, bool lng, hipStream_t st) {
    if (sa.in_abs && lng)
        hipLaunchKernelGGL((wgrad_small_kernel<1, true>), grid, dim3(512), 0, st, sa);
    else if (sa.in_abs)
        hipLaunchKernelGGL((wgrad_small_kernel<1, false>), grid, dim3(512), 0, st, sa);
    else if (sa.in_sq && lng)
        hipLaunchKernelGGL((wgrad_small_kernel<2, true>), grid, dim3(512), 0, st, sa);
    else if (sa.in_sq)
        hipLaunchKernelGGL((wgrad_small_kernel<2, false>), grid, dim3(512), 0, st, sa);
    else if (lng)
        hipLaunchKernelGGL((wgrad_small_kernel<0, true>), grid, dim3(512), 0, st, sa);
    else
        hipLaunchKernelGGL((wgrad_small_kernel<0, false>), grid, dim3(512), 0, st, sa);
}

static void launch_wgrad_small_batch(const SwBatch& b, int cls, hipStream_t st) {
    const dim3 grid(b.start[b.n]);
    switch (cls) {
        case 1: hipLaunchKernelGGL((wgrad_small_batch_kernel<1, false>), grid, dim3(512), 0, st, b); break;
        case 2: hipLaunchKernelGGL((wgrad_small_batch_kernel<2, false>), grid, dim3(512), 0, st, b); break;
        case 3: hipLaunchKernelGGL((wgrad_small_batch_kernel<0, true>), grid, dim3(512), 0, st, b); break;
        case 4: hipLaunchKernelGGL((wgrad_small_batch_kernel<1, true>), grid, dim3(512), 0, st, b); break;
        case 5: hipLaunchKernelGGL((wgrad_small_batch_kernel<2, true>), grid, dim3(512), 0, st, b); break;
        default: hipLaunchKernelGGL((wgrad_small_batch_kernel<0, false>), grid, dim3(512), 0, st, b); break;
    }
}

// the argument checks and operand roles of a weight-gradient call (run_conv_wgrad, cai_conv_wgrad_batch)
static int wgrad_prepare(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, int32_t in_abs,
                         int32_t in_sq, const void* dy, int32_t dy_ld, const float* dw, const float* db,
                         const void* workspace, size_t ws_bytes, WgradPlan& W, WgradArgs& a) {
    int rc = check_geom(g);
    if (rc) return rc;
    CAI_CHECK_ARG(x && dy && dw, "conv_wgrad: null pointer");
    W = make_wgrad_plan(g, dtype, true, in_abs || in_sq);
    CAI_CHECK_ARG(workspace && ws_bytes >= W.ws_slab + W.ws_bias + W.ws_col + 256, "conv_wgrad: workspace too small");
    const int VEC = dtype == CAI_BF16 ? 8 : 4;
    a = WgradArgs{};
    if (!g->transposed) {
        a.g = dy; a.g_ld = dy_ld; a.x = x; a.x_ld = x_ld;
        a.Hg = g->out_h; a.Wg = g->out_w; a.Hx = g->in_h; a.Wx = g->in_w;
        a.in_abs = in_abs; a.in_sq = in_sq;
    } else {
        a.g = x; a.g_ld = x_ld; a.x = dy; a.x_ld = dy_ld;
        a.Hg = g->in_h; a.Wg = g->in_w; a.Hx = g->out_h; a.Wx = g->out_w;
        CAI_CHECK_ARG(!in_abs && !in_sq, "conv_wgrad: input transforms only for Conv2d");
    }
    // gradient rows are read in VEC-channel chunks: rows past Ng (inside g_ld) only
    // feed output rows that are never stored
    CAI_CHECK_ARG(W.M < (1ll << 31), "conv_wgrad: too many pixels");
    CAI_CHECK_ARG(a.g_ld % VEC == 0 && a.x_ld % VEC == 0 && a.x_ld >= W.Cq_pad && a.g_ld >= round_up(W.Ng, VEC),
                  "conv_wgrad: bad leading dimensions (g_ld %d for %d rows, x_ld %d for %d columns)", a.g_ld, W.Ng,
                  a.x_ld, W.Cq_pad);
    CAI_CHECK_ARG(!db || (dy_ld % VEC == 0 && g->out_c <= COLSUM_MAXC), "conv_wgrad: bad bias-gradient layout");
    a.Ng = W.Ng; a.Cq_pad = W.Cq_pad; a.B = g->batch;
    a.k = g->kernel; a.s = g->stride; a.p = g->pad; a.ncols = W.ncols; a.M = W.M; a.split_len = W.split_len;
    a.ws = reinterpret_cast<float*>(const_cast<void*>(workspace));
    return CAI_OK;
}

// The pixel-split weight gradient (LDS-DMA glds / halo kernels): the remaining kernel arguments, the kernel variant
// (key: halo KS, S, R and bias flag, or glds CT and input / bias flags) and the block count.
static void wgrad_split_setup(const cai_conv_geom* g, const WgradPlan& W, WgradArgs& a, void* workspace, float* db,
                              int in_abs, int in_sq, int& key, int& nblocks) {
    a.ctiles = (W.ncols + W.ct - 1) / W.ct;
    a.rtiles = (W.Ng + 127) / 128;
    a.nsub = W.nsub; a.grp_len = W.grp_len; a.chunk = W.px_chunk;
    a.split_len = W.split_len;
    a.nsplit = W.S;
    float* bws = nullptr;
    if ((W.fused_bias || W.tbias) && db) bws = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + W.ws_slab);
    a.bws = bws;
    a.tb_kh0 = W.tb_kh0; a.tb_kw0 = W.tb_kw0; a.tb_s = g->stride; a.nbias = W.nbias;
    const int bflag = !bws ? 0 : (W.tbias ? WG_TBIAS : WG_BIAS);
    nblocks = W.S * W.tiles;
    if (W.halo) {
        a.nsplit = W.strips_per_split;
        a.rtiles = (W.Ng + W.hrows - 1) / W.hrows;
        // row mode (bits 4-5): 0 = 128-row tiles, 1 = 64, 2 = 192
        key = (((((W.halo * 10 + g->stride) * 10 + halo_wgrad_rows(g)) << 2) | (W.hrows == 64 ? 1 : W.hrows == 192 ? 2 : 0)) << 4) | bflag;
    } else {
        key = (1 << 20) | (W.ct << 4) | (in_abs ? WG_ABS : 0) | (in_sq ? WG_SQ : 0) | bflag;
    }
}

// the fixed-order slab reduce of a pixel-split weight gradient (slab a.ws, bias partials a.bws) into torch layout
static cai_reduce_job wgrad_split_job(const cai_conv_geom* g, const WgradPlan& W, const WgradArgs& a, float* dw,
                                      float* db, int accumulate) {
    cai_reduce_job J{};
    J.kind = CAI_JOB_WGRAD;
    J.nblocks = wgrad_job_blocks(W.Ng, W.Cq_pad, g->kernel, a.bws ? (W.nbias + 255) / 256 : 0);
    J.p[0] = a.ws; J.p[1] = dw; J.p[2] = a.bws; J.p[3] = db;
    J.i[0] = W.S; J.i[1] = W.Ng; J.i[2] = W.ncols; J.i[3] = W.Cq; J.i[4] = W.Cq_pad; J.i[5] = g->kernel;
    J.i[6] = accumulate; J.i[7] = W.Sb; J.i[8] = W.nbias;
    return J;
}

static void launch_wgrad_split(const WgradArgs& a, int key, int nblocks, hipStream_t st) {
    const int f = key & 15;
    if (key >> 20) {
        const int in_abs = (f & WG_ABS) != 0, in_sq = (f & WG_SQ) != 0, bflag = f & (WG_BIAS | WG_TBIAS);
        if (((key >> 4) & 0xffff) == 256)
            launch_wgrad_glds<256>(a, nblocks, in_abs, in_sq, bflag, st);
        else
            launch_wgrad_glds<128>(a, nblocks, in_abs, in_sq, bflag, st);
        return;
    }
    const int rmode = (key >> 4) & 3;
    const bool r64 = rmode == 1;
    switch (key >> 6) {
        case 521: r64 ? launch_wgrad_halo<5, 2, 1, 2>(a, nblocks, f, st) : launch_wgrad_halo<5, 2>(a, nblocks, f, st); break;
        case 522: r64 ? launch_wgrad_halo<5, 2, 2, 2>(a, nblocks, f, st) : launch_wgrad_halo<5, 2, 2>(a, nblocks, f, st); break;
        case 524: r64 ? launch_wgrad_halo<5, 2, 4, 2>(a, nblocks, f, st) : launch_wgrad_halo<5, 2, 4>(a, nblocks, f, st); break;
        case 322: r64 ? launch_wgrad_halo<3, 2, 2, 2>(a, nblocks, f, st) : launch_wgrad_halo<3, 2, 2>(a, nblocks, f, st); break;
        case 324: r64 ? launch_wgrad_halo<3, 2, 4, 2>(a, nblocks, f, st) : launch_wgrad_halo<3, 2, 4>(a, nblocks, f, st); break;
        case 311:
            if (rmode == 2) launch_wgrad_halo<3, 1, 1, 6>(a, nblocks, f, st);
            else r64 ? launch_wgrad_halo<3, 1, 1, 2>(a, nblocks, f, st) : launch_wgrad_halo<3, 1>(a, nblocks, f, st);
            break;
        default: r64 ? launch_wgrad_halo<3, 2, 1, 2>(a, nblocks, f, st) : launch_wgrad_halo<3, 2>(a, nblocks, f, st); break;
    }
}

static void launch_wgrad_split_batch(const WgBatch& b, int key, hipStream_t st) {
    const int f = key & 15;
    if (key >> 20) {
        if (((key >> 4) & 0xffff) == 256)
            launch_wgrad_glds_batch<256>(b, f, st);
        else
            launch_wgrad_glds_batch<128>(b, f, st);
        return;
    }
    const int rmode = (key >> 4) & 3;
    const bool r64 = rmode == 1;
    switch (key >> 6) {
        case 521: r64 ? launch_wgrad_halo_batch<5, 2, 1, 2>(b, f, st) : launch_wgrad_halo_batch<5, 2>(b, f, st); break;
        case 522: r64 ? launch_wgrad_halo_batch<5, 2, 2, 2>(b, f, st) : launch_wgrad_halo_batch<5, 2, 2>(b, f, st); break;
        case 524: r64 ? launch_wgrad_halo_batch<5, 2, 4, 2>(b, f, st) : launch_wgrad_halo_batch<5, 2, 4>(b, f, st); break;
        case 322: r64 ? launch_wgrad_halo_batch<3, 2, 2, 2>(b, f, st) : launch_wgrad_halo_batch<3, 2, 2>(b, f, st); break;
        case 324: r64 ? launch_wgrad_halo_batch<3, 2, 4, 2>(b, f, st) : launch_wgrad_halo_batch<3, 2, 4>(b, f, st); break;
        case 311:
            if (rmode == 2) launch_wgrad_halo_batch<3, 1, 1, 6>(b, f, st);
            else r64 ? launch_wgrad_halo_batch<3, 1, 1, 2>(b, f, st) : launch_wgrad_halo_batch<3, 1>(b, f, st);
            break;
        default: r64 ? launch_wgrad_halo_batch<3, 2, 1, 2>(b, f, st) : launch_wgrad_halo_batch<3, 2>(b, f, st); break;
    }
}

static int run_conv_wgrad(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, int32_t in_abs,
                          int32_t in_sq, const void* dy, int32_t dy_ld, float* dw, float* db, int32_t accumulate,
                          void* workspace, size_t ws_bytes, void* stream, cai_reduce_job* job) {
    if (job) *job = cai_reduce_job{};
    WgradPlan W;
    WgradArgs a;
    int rc = wgrad_prepare(g, dtype, x, x_ld, in_abs, in_sq, dy, dy_ld, dw, db, workspace, ws_bytes, W, a);
    if (rc) return rc;
    float* slab = a.ws;
    a.ctiles = (W.ncols + 127) / 128;
    a.rtiles = (W.Ng + 127) / 128;
    a.nsub = W.nsub;
    a.grp_len = W.grp_len;
    a.chunk = W.px_chunk;
    hipStream_t st = as_stream(stream);
    if (small_wgrad_ok(g, dtype)) {
        SwArgs sa;
        dim3 grid;
        cai_reduce_job J;
        rc = small_wgrad_setup(g, W, a, dy, dy_ld, dw, db, accumulate, slab, sa, grid, J);
        if (rc) return rc;
        launch_wgrad_small(sa, grid, W.M > SW_NW * SW_STEPS * 32, st);
        CAI_LAUNCH_CHECK("conv_wgrad");
        if (J.kind == CAI_JOB_NONE) return CAI_OK;
        if (job) {
            *job = J;
            return CAI_OK;
        }
        return launch_reduce_jobs(&J, 1, st);
    }
    float* bws = nullptr;
    if (W.glds) {
        int key, nblocks;
        wgrad_split_setup(g, W, a, workspace, db, in_abs, in_sq, key, nblocks);
        bws = a.bws;
        launch_wgrad_split(a, key, nblocks, st);
    } else {
        dim3 grid(8 * a.ctiles * a.rtiles * a.nsub);
        if (dtype == CAI_BF16)
            hipLaunchKernelGGL(wgrad_kernel<bf16>, grid, dim3(NT), 0, st, a);
        else
            hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(NT), 0, st, a);
    }
    // the fixed-order slab reduce into torch layout: a job (reduce_jobs.hip), returned to a deferring caller or
    // run now
    a.bws = bws;
    const cai_reduce_job J = wgrad_split_job(g, W, a, dw, db, accumulate);
    (void)slab;
    if (job) {
        *job = J;
    } else {
        rc = launch_reduce_jobs(&J, 1, st);
        if (rc) return rc;
    }
    if (db && !bws) {
        float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + W.ws_slab + W.ws_bias);
        const int64_t npix = (int64_t)g->batch * g->out_h * g->out_w;
        if (dtype == CAI_BF16)
            launch_colsum<bf16>(dy, npix, g->out_c, dy_ld, W.nchunk, W.chunk, part, db, accumulate, st);
        else
            launch_colsum<float>(dy, npix, g->out_c, dy_ld, W.nchunk, W.chunk, part, db, accumulate, st);
    }
    CAI_LAUNCH_CHECK("conv_wgrad");
    return CAI_OK;
}

int cai_conv_wgrad(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, int32_t in_abs, int32_t in_sq,
                   const void* dy, int32_t dy_ld, float* dw, float* db, int32_t accumulate, void* workspace,
                   size_t ws_bytes, void* stream) {
    return run_conv_wgrad(g, dtype, x, x_ld, in_abs, in_sq, dy, dy_ld, dw, db, accumulate, workspace, ws_bytes, stream,
                          nullptr);
}

int cai_conv_wgrad_deferred(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, int32_t in_abs,
                            int32_t in_sq, const void* dy, int32_t dy_ld, float* dw, float* db, int32_t accumulate,
                            void* workspace, size_t ws_bytes, void* stream, cai_reduce_job* job) {
    CAI_CHECK_ARG(job, "conv_wgrad_deferred: null job");
    return run_conv_wgrad(g, dtype, x, x_ld, in_abs, in_sq, dy, dy_ld, dw, db, accumulate, workspace, ws_bytes, stream,
                          job);
}

int cai_conv_wgrad_batch(const cai_wgrad_call* calls, int32_t n, void* stream, cai_reduce_job* jobs) {
    CAI_CHECK_ARG(n >= 0 && (n == 0 || (calls && jobs)), "conv_wgrad_batch: bad arguments");
    hipStream_t st = as_stream(stream);
    // the latent-size calls, grouped by kernel variant (input transform, long form): one launch per group of up to
    // SW_BATCH_MAX calls; a call whose bias gradient (written in place) another call of the open group also
    // writes starts a new group, so no launch holds two writers of one bias
    SwBatch b[6];
    for (int c = 0; c < 6; ++c) b[c].n = 0, b[c].start[0] = 0;
    // the pixel-split calls (glds / halo kernels) grouped by kernel variant, up to WG_BATCH_MAX per launch
    std::vector<std::pair<int, WgBatch>> groups;
    for (int i = 0; i < n; ++i) {
        const cai_wgrad_call& c = calls[i];
        jobs[i] = cai_reduce_job{};
        if (!small_wgrad_ok(&c.geom, c.dtype)) {
            WgradPlan W;
            WgradArgs a;
            int rc = wgrad_prepare(&c.geom, c.dtype, c.x, c.x_ld, c.in_abs, c.in_sq, c.dy, c.dy_ld, c.dw, c.db,
                                   c.workspace, c.ws_bytes, W, a);
            if (rc) return rc;
            const bool fused_bias = !c.db || ((W.fused_bias || W.tbias));
            if (!W.glds || !fused_bias) {   // other kernels, or a bias gradient by separate column sums: as usual
                rc = run_conv_wgrad(&c.geom, c.dtype, c.x, c.x_ld, c.in_abs, c.in_sq, c.dy, c.dy_ld, c.dw, c.db,
                                    c.accumulate, c.workspace, c.ws_bytes, stream, &jobs[i]);
                if (rc) return rc;
                continue;
            }
            int key, nblocks;
            wgrad_split_setup(&c.geom, W, a, c.workspace, c.db, c.in_abs, c.in_sq, key, nblocks);
            jobs[i] = wgrad_split_job(&c.geom, W, a, c.dw, c.db, c.accumulate);
            size_t gi = 0;
            while (gi < groups.size() && groups[gi].first != key) ++gi;
            if (gi == groups.size()) {
                groups.emplace_back(key, WgBatch{});
                groups[gi].second.n = 0;
                groups[gi].second.start[0] = 0;
            }
            WgBatch& B = groups[gi].second;
            if (B.n == WG_BATCH_MAX) {
                launch_wgrad_split_batch(B, key, st);
                B.n = 0;
            }
            B.job[B.n] = a;
            B.nwg[B.n] = nblocks;
            B.start[B.n + 1] = B.start[B.n] + (nblocks + 7) / 8 * 8;
            ++B.n;
            continue;
        }
        WgradPlan W;
        WgradArgs a;
        int rc = wgrad_prepare(&c.geom, c.dtype, c.x, c.x_ld, c.in_abs, c.in_sq, c.dy, c.dy_ld, c.dw, c.db,
                               c.workspace, c.ws_bytes, W, a);
        if (rc) return rc;
        SwArgs sa;
        dim3 grid;
        rc = small_wgrad_setup(&c.geom, W, a, c.dy, c.dy_ld, c.dw, c.db, c.accumulate, a.ws, sa, grid, jobs[i]);
        if (rc) return rc;
        const bool lng = W.M > SW_NW * SW_STEPS * 32;
        const int cls = (sa.in_abs ? 1 : (sa.in_sq ? 2 : 0)) + (lng ? 3 : 0);
        SwBatch& B = b[cls];
        bool clash = false;
        for (int j = 0; j < B.n; ++j) clash |= sa.db && B.job[j].db == sa.db;
        if (clash || B.n == SW_BATCH_MAX) {
            launch_wgrad_small_batch(B, cls, st);
            B.n = 0;
        }
        B.job[B.n] = sa;
        B.gx[B.n] = (int)grid.x;
        B.gy[B.n] = (int)grid.y;
        B.start[B.n + 1] = B.start[B.n] + (int)(grid.x * grid.y);
        ++B.n;
    }
    for (int c = 0; c < 6; ++c)
        if (b[c].n) launch_wgrad_small_batch(b[c], c, st);
    for (auto& kv : groups)
        if (kv.second.n) launch_wgrad_split_batch(kv.second, kv.first, st);
    CAI_LAUNCH_CHECK("conv_wgrad_batch");
    return CAI_OK;
}

}  // extern "C"

// exported for gdn.hip (1x1 wgrad on u and x^2, column sums)
namespace cai {
int colsum_any(int dtype, const void* g, int64_t npix, int C, int ld, float* out, int accumulate, void* ws,
               size_t wsb, hipStream_t st) {
    const int nchunk = colsum_nchunk(npix);
    const int64_t chunk = (npix + nchunk - 1) / nchunk;
    CAI_CHECK_ARG(wsb >= (size_t)nchunk * C * sizeof(float), "colsum: workspace too small");
    CAI_CHECK_ARG(C <= COLSUM_MAXC && ld % (dtype == CAI_BF16 ? 8 : 4) == 0, "colsum: bad layout");
    if (dtype == CAI_BF16)
        launch_colsum<bf16>(g, npix, C, ld, nchunk, chunk, reinterpret_cast<float*>(ws), out, accumulate, st);
    else
        launch_colsum<float>(g, npix, C, ld, nchunk, chunk, reinterpret_cast<float*>(ws), out, accumulate, st);
    return CAI_OK;
}
size_t colsum_ws_bytes(int64_t npix, int C) { return (size_t)colsum_nchunk(npix) * C * sizeof(float); }
}  // namespace cai
