// Lane-local GDN / IGDN kernels (bf16; compressai/layers/gdn.py:41-92): the per-pixel C x C contractions with
// NO LDS tile and no workgroup barrier in the pixel path.
//
// Operand layout.  A wave owns 16 pixels at a time.  x (and dy) arrive straight from global memory in the
// v_mfma_f32_16x16x32_bf16 B-operand layout: lane l holds pixel l & 15, channels 32 kb + 8 (l >> 4) .. +8 of
// K block kb (one 16-byte buffer load per K block: 16 pixels x 64 contiguous bytes per wave instruction).  The
// A operand (gamma, and gamma^T in the backward) is held in registers for the wave's lifetime with its rows
// PERMUTED: row m of output block cb is channel
//     ch(cb, m) = 32 (cb >> 1) + 8 (m >> 2) + 4 (cb & 1) + (m & 3).
// The MFMA leaves D row 4 (l >> 4) + r of column l & 15 in lane l, i.e. channel 32 (cb >> 1) + 8 (l >> 4) +
// 4 (cb & 1) + r of the lane's own pixel: element 4 (cb & 1) + r of the chunk the lane loaded for K block
// cb >> 1.  Every elementwise stage is therefore lane-local, the backward's u is already in the B layout of the
// dx GEMM (dx^T = gamma^T u^T), and outputs leave as the same 16-byte chunks the inputs came in.  The norm / dx
// dot products run the same K-block sequence as gdn_fwd_kernel / gdn_bwd_fused_kernel (each 32-channel K block
// in lane order 8 (l >> 4) + e, blocks in order): the forward is bit-identical to gdn_fwd_kernel.
//
// Backward (gdn_bwd_lane_kernel): the same operand layout, with the work of a 64-pixel step split between two
// wave roles that share each SIMD: norm waves (gamma in registers: x^2, norm, the lane-local u / t1 stage, fp32
// dbeta) and dx waves (gamma^T and the dgamma accumulators in registers: dx GEMM, dx, dgamma = u^T x^2 with
// pixels as K through ds_read_b64_tr_b16).  u, t1, x and x^2 pass from one role to the other through a
// double-buffered LDS image, one barrier per step.  Per-block partials (dgamma, dbeta) go to the same
// [block][C*C + C] slab as the fused kernel's, reduced by the GDN reduce job (reduce_jobs.hip).
// Pixels past npix load as 0 (buffer loads out of range): x = dy = 0 gives u = 0, so they add nothing.
#include "common.hpp"
#include "mfma.hpp"

#include <stdlib.h>

#include <algorithm>

namespace cai {

namespace {

#ifndef CAI_GDN_FWD_NSET
#define CAI_GDN_FWD_NSET 2   // 16-pixel tiles of loads in flight per wave of the C = 128 forward (A/B: 1 measured 3.7 us slower per C2 step, profiles/r03_gdn_fwd_nset_ab.log)
#endif

constexpr unsigned LANE_OOB = 0x80000000u;   // beyond every buffer: loads return 0, stores are dropped

__device__ __forceinline__ int perm_ch(int cb, int m) { return 32 * (cb >> 1) + 8 * (m >> 2) + 4 * (cb & 1) + (m & 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// the KB 16-byte chunks of pixel pix (row stride ld elements) in the B-operand layout
template <int KB>
__device__ __forceinline__ void chunk_load(u32x4 (&r)[KB], __amdgpu_buffer_rsrc_t rs, int64_t pix, int64_t npix, int ld,
                                           int g) {
    const bool ok = pix < npix;
    const unsigned base = (unsigned)(pix * ld + 8 * g) * 2u;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
        r[kb] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? base + 64u * kb : LANE_OOB, 0, 0));
}
template <int KB>
__device__ __forceinline__ void chunk_store(const u32x4 (&r)[KB], __amdgpu_buffer_rsrc_t rs, int64_t pix, int64_t npix,
                                            int ld, int g) {
    const bool ok = pix < npix;
    const unsigned base = (unsigned)(pix * ld + 8 * g) * 2u;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
        __builtin_amdgcn_raw_buffer_store_b128(r[kb], rs, ok ? base + 64u * kb : LANE_OOB, 0, 0);
}

// gamma-shaped A fragments (rows permuted as above) of a row-major [C][C] bf16 matrix
template <int C>
__device__ __forceinline__ void afrag_load(u32x4 (&a)[C / 16][C / 32], const bf16* mat, int p, int g) {
#pragma unroll
    for (int cb = 0; cb < C / 16; ++cb) {
        const bf16* row = mat + (int64_t)perm_ch(cb, p) * C + 8 * g;
#pragma unroll
        for (int kb = 0; kb < C / 32; ++kb) a[cb][kb] = *reinterpret_cast<const u32x4*>(row + 32 * kb);
    }
}

// The workgroup's copy of NM consecutive [C][C] bf16 matrices in LDS (rows padded by 16 bytes: the fragment reads
// of 16 rows at one column spread over the banks): one coalesced global read per workgroup instead of one
// fragment gather per wave.  Ends with a barrier.
template <int C, int NM, int NT>
__device__ __forceinline__ void stage_mats(char* lds, const bf16* mat) {
    constexpr int RSG = 2 * C + 16, CH = 2 * C / 16;   // row stride (bytes), 16-byte chunks per row
    for (int i = threadIdx.x; i < NM * C * CH; i += NT) {
        const int row = i / CH, ch = i - (i / CH) * CH;
        *reinterpret_cast<u32x4*>(lds + row * RSG + ch * 16) = *reinterpret_cast<const u32x4*>(mat + (int64_t)row * C + ch * 8);
    }
    __syncthreads();
}
template <int C>
__device__ __forceinline__ void afrag_lds(u32x4 (&a)[C / 16][C / 32], const char* img, int p, int g) {
    constexpr int RSG = 2 * C + 16;
#pragma unroll
    for (int cb = 0; cb < C / 16; ++cb) {
        const char* row = img + perm_ch(cb, p) * RSG + 16 * g;
#pragma unroll
        for (int kb = 0; kb < C / 32; ++kb) a[cb][kb] = *reinterpret_cast<const u32x4*>(row + 64 * kb);
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// forward: persistent waves, two 16-pixel tiles of loads in flight per wave
// ---------------------------------------------------------------------------
// OCC = resident waves per SIMD; NSET = 16-pixel tiles of loads in flight per wave (register sets)
template <int C, bool INV, int OCC, int NSET = (OCC == 1 ? 2 : 1)>
__global__ __launch_bounds__(256, OCC) void gdn_fwd_lane_kernel(const bf16* __restrict__ x, int x_ld,
                                                                             int64_t npix, const bf16* __restrict__ gamma,
                                                                             const float* __restrict__ beta,
                                                                             bf16* __restrict__ y, int y_ld) {
    constexpr int KB = C / 32, NB = C / 16;
    __shared__ __attribute__((aligned(16))) char Lg[C * (2 * C + 16)];
    __shared__ __attribute__((aligned(16))) float Lb[C];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, p = lane & 15;
    for (int c = threadIdx.x; c < C; c += 256) Lb[c] = beta[c];
    stage_mats<C, 1, 256>(Lg, gamma);
    u32x4 ga[NB][KB];
    afrag_lds<C>(ga, Lg, p, g);

    const __amdgpu_buffer_rsrc_t xr = rsrc(x, npix * x_ld * 2), yr = rsrc(y, npix * y_ld * 2);
    const int64_t ntiles = (npix + 15) / 16;
    const int64_t nw = (int64_t)gridDim.x * 4;
    int64_t t = (int64_t)blockIdx.x * 4 + wave;
    const int64_t mine = t < ntiles ? (ntiles - t + nw - 1) / nw : 0;
    u32x4 ra[KB], rb[KB];
    chunk_load<KB>(ra, xr, t * 16 + p, npix, x_ld, g);
    if constexpr (NSET == 2) chunk_load<KB>(rb, xr, (t + nw) * 16 + p, npix, x_ld, g);

    auto step = [&](u32x4 (&rx)[KB], int64_t cur, int64_t nxt) {
        u32x4 xc[KB], q[KB];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            xc[kb] = rx[kb];
            q[kb] = sq_chunk<bf16>(xc[kb]);
        }
        chunk_load<KB>(rx, xr, nxt * 16 + p, npix, x_ld, g);
        u32x4 yv[KB];
#pragma unroll
        for (int kx = 0; kx < KB; ++kx) {
            const bf16x8 xv = __builtin_bit_cast(bf16x8, xc[kx]);
            bf16x8 yy;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kb = 0; kb < KB; ++kb) acc = mma16<bf16>(ga[2 * kx + h][kb], q[kb], acc);
                const f32x4 bq = *reinterpret_cast<const f32x4*>(Lb + 32 * kx + 8 * g + 4 * h);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float nv = acc[r] + bq[r];
                    const float rs = rsqrtf(nv);
                    yy[4 * h + r] = (bf16)((float)xv[4 * h + r] * (INV ? nv * rs : rs));
                }
            }
            yv[kx] = __builtin_bit_cast(u32x4, yy);
            if constexpr (OCC == 2) __builtin_amdgcn_sched_barrier(0);   // bound the live accumulators
        }
        chunk_store<KB>(yv, yr, cur * 16 + p, npix, y_ld, g);
    };
    if constexpr (NSET == 2) {
        for (int64_t it = 0; it < mine / 2; ++it, t += 2 * nw) {
            step(ra, t, t + 2 * nw);
            step(rb, t + nw, t + 3 * nw);
        }
        if (mine & 1) step(ra, t, t + 2 * nw);
    } else {
        for (int64_t it = 0; it < mine; ++it, t += nw) step(ra, t, t + nw);
    }
}

// ---------------------------------------------------------------------------
// backward: one 512-thread workgroup per CU, two roles per SIMD (waves w and w + 4 share a SIMD)
//   norm waves 0-3 (gamma fragments in registers): per 64-pixel step each loads x, dy of its 16 pixels (next
//     step's chunks issued as the current ones retire), forms x^2, runs norm^T = gamma (x^2)^T, the lane-local
//     u / t1 stage and the fp32 dbeta sums, and writes x^2, x, u, t1 to the step's LDS buffer;
//   dx waves 4-7 (gamma^T fragments and the dgamma accumulators in registers): after the step's barrier each
//     reads its partner's u chunks as B operands, runs dx^T = gamma^T u^T, forms dx = t1 + 2 x (gamma^T u) and
//     stores it, then accumulates dgamma rows [C/4 d, C/4 (d+1)) += u^T x^2 over the step's 64 pixels.
// The vector-heavy and the matrix-heavy halves of the step share each SIMD; the norm waves of step s + 1 run
// while the dx waves finish step s (double-buffered LDS, one barrier per step).
// ---------------------------------------------------------------------------
template <int C>
struct SplitBwdGeo {
    static constexpr int KB = C / 32, NB = C / 16;
    static constexpr int BP = 64;                      // pixels per step (4 norm waves x 16)
    static constexpr int RS = 2 * C + 16;              // LDS row stride: conflict-free 16-byte row writes
    static constexpr int IMG = BP * RS;                // one [64 px][C] bf16 image
    static constexpr int BUF = 4 * IMG;                // x^2, u, t1, x of one step
    static constexpr int IB = NB / 4;                  // dgamma row blocks per dx wave
    static constexpr int LDS = 2 * BUF + C * 4 + 4 * C * 4;   // two buffers, beta, dbeta per norm wave
};

template <int C, bool INV>
__global__ __launch_bounds__(512, 1) void gdn_bwd_lane_kernel(const bf16* __restrict__ x, int x_ld,
                                                              const bf16* __restrict__ dy, int dy_ld, int64_t npix,
                                                              const bf16* __restrict__ gamma_op,
                                                              const float* __restrict__ beta,
                                                              bf16* __restrict__ dx, int dx_ld,
                                                              float* __restrict__ part) {
    using G = SplitBwdGeo<C>;
    constexpr int KB = G::KB, NB = G::NB, IB = G::IB;
    __shared__ __attribute__((aligned(16))) char lds[G::LDS];
    float* const Lb = reinterpret_cast<float*>(lds + 2 * G::BUF);
    float* const Ldb = Lb + C;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, p = lane & 15;
    const bool norm_role = wave < 4;
    const int d = wave & 3;                 // the 16-pixel slot of the step (dx wave d serves norm wave d)
    const int prow = d * 16 + p;            // this lane's pixel row inside a step
    for (int c = threadIdx.x; c < C; c += 512) Lb[c] = beta[c];
    static_assert(2 * C * (2 * C + 16) <= 2 * G::BUF, "gamma staging");
    stage_mats<C, 2, 512>(lds, gamma_op);   // gamma, gamma^T: staged in the step buffers before their first use
    u32x4 gf[NB][KB];                       // gamma (norm waves) or gamma^T (dx waves) A fragments
    afrag_lds<C>(gf, lds + (norm_role ? 0 : C * (2 * C + 16)), p, g);
    __syncthreads();

    const int64_t nsteps = (npix + G::BP - 1) / G::BP;
    const int64_t stride = gridDim.x;
    const int64_t s0 = blockIdx.x;
    const int64_t mine = s0 < nsteps ? (nsteps - s0 + stride - 1) / stride : 0;
    float* const pb = part + (int64_t)blockIdx.x * ((int64_t)C * C + C);

    if (norm_role) {
        const __amdgpu_buffer_rsrc_t xr = rsrc(x, npix * x_ld * 2), gr = rsrc(dy, npix * dy_ld * 2);
        float dbeta[KB][8];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int e = 0; e < 8; ++e) dbeta[kb][e] = 0.f;
        // one step: consume (rx, rg) = step s; as each chunk retires, that chunk of step `pf` goes out into its
        // registers (pf = the next step, or the one after it with two register sets in flight)
        auto nstep = [&](u32x4 (&rx)[KB], u32x4 (&rg)[KB], int64_t it, int64_t pf) {
            char* const Lq = lds + (it & 1) * G::BUF;
            char* const Lu = Lq + G::IMG;
            char* const Lt = Lu + G::IMG;
            char* const Lx = Lt + G::IMG;
            const int64_t npx = pf * G::BP + prow;
            const bool nok = npx < npix;
            u32x4 q[KB];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                q[kb] = sq_chunk<bf16>(rx[kb]);
                *reinterpret_cast<u32x4*>(Lq + prow * G::RS + (32 * kb + 8 * g) * 2) = q[kb];
                *reinterpret_cast<u32x4*>(Lx + prow * G::RS + (32 * kb + 8 * g) * 2) = rx[kb];
            }
#pragma unroll
            for (int kx = 0; kx < KB; ++kx) {
                const bf16x8 xv = __builtin_bit_cast(bf16x8, rx[kx]);
                const bf16x8 gv = __builtin_bit_cast(bf16x8, rg[kx]);
                bf16x8 uu, tt;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int kb = 0; kb < KB; ++kb) acc = mma16<bf16>(gf[2 * kx + h][kb], q[kb], acc);
                    const f32x4 bq = *reinterpret_cast<const f32x4*>(Lb + 32 * kx + 8 * g + 4 * h);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int e = 4 * h + r;
                        const float xf = (float)xv[e], gv_ = (float)gv[e];
                        const float nv = acc[r] + bq[r];
                        const float rs = rsqrtf(nv);
                        float uv, tv;
                        if constexpr (INV) {
                            tv = gv_ * nv * rs;
                            uv = 0.5f * gv_ * xf * rs;
                        } else {
                            tv = gv_ * rs;
                            uv = -0.5f * gv_ * xf * rs * rs * rs;
                        }
                        dbeta[kx][e] += uv;
                        tt[e] = (bf16)tv;   // t1 rounded to bf16 as in the fused kernel
                        uu[e] = (bf16)uv;
                    }
                }
                *reinterpret_cast<bf16x8*>(Lu + prow * G::RS + (32 * kx + 8 * g) * 2) = uu;
                *reinterpret_cast<bf16x8*>(Lt + prow * G::RS + (32 * kx + 8 * g) * 2) = tt;
                const unsigned off = nok ? (unsigned)(npx * x_ld + 8 * g) * 2u + 64u * kx : LANE_OOB;
                const unsigned offg = nok ? (unsigned)(npx * dy_ld + 8 * g) * 2u + 64u * kx : LANE_OOB;
                rx[kx] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
                rg[kx] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(gr, offg, 0, 0));
                __builtin_amdgcn_sched_barrier(0);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        };
        u32x4 rx[KB], rg[KB];
        chunk_load<KB>(rx, xr, s0 * G::BP + prow, npix, x_ld, g);
        chunk_load<KB>(rg, gr, s0 * G::BP + prow, npix, dy_ld, g);
        int64_t s = s0;
        for (int64_t it = 0; it < mine; ++it, s += stride) nstep(rx, rg, it, s + stride);
        // dbeta: the 16 pixel lanes of each channel, then the four norm waves in order
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float v = dbeta[kb][e];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
                if (p == 0) Ldb[d * C + 32 * kb + 8 * g + e] = v;
            }
    } else {
        const __amdgpu_buffer_rsrc_t dr = rsrc(dx, npix * dx_ld * 2);
        const int q_ = p >> 2, p4 = p & 3;
        f32x4 dg[IB][NB];
#pragma unroll
        for (int i = 0; i < IB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) dg[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        int64_t s = s0;
        for (int64_t it = 0; it < mine; ++it, s += stride) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            const char* const Lq = lds + (it & 1) * G::BUF;
            const char* const Lu = Lq + G::IMG;
            const char* const Lt = Lu + G::IMG;
            const char* const Lx = Lt + G::IMG;
            const int64_t pix = s * G::BP + prow;
            u32x4 uf[KB];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb)
                uf[kb] = *reinterpret_cast<const u32x4*>(Lu + prow * G::RS + (32 * kb + 8 * g) * 2);
            // ---- dx^T = gamma^T u^T; dx = t1 + 2 x (gamma^T u), 16 bytes out per K block ----
            const bool ok = pix < npix;
            const unsigned base = (unsigned)(pix * dx_ld + 8 * g) * 2u;
#pragma unroll
            for (int kx = 0; kx < KB; ++kx) {
                const bf16x8 xv = *reinterpret_cast<const bf16x8*>(Lx + prow * G::RS + (32 * kx + 8 * g) * 2);
                const bf16x8 tt = *reinterpret_cast<const bf16x8*>(Lt + prow * G::RS + (32 * kx + 8 * g) * 2);
                bf16x8 dd;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int kb = 0; kb < KB; ++kb) acc = mma16<bf16>(gf[2 * kx + h][kb], uf[kb], acc);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int e = 4 * h + r;
                        dd[e] = (bf16)((float)tt[e] + 2.f * (float)xv[e] * acc[r]);
                    }
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dd), dr, ok ? base + 64u * kx : LANE_OOB,
                                                       0, 0);
            }
            // ---- dgamma rows of this wave += u^T x^2 over the step's 64 pixels ----
#pragma unroll
            for (int ks = 0; ks < G::BP / 32; ++ks) {
                const int rr = 32 * ks + 8 * g + q_;
                u32x4 afr[IB];
#pragma unroll
                for (int i = 0; i < IB; ++i) {
                    const int col = (d * IB + i) * 16 + 4 * p4;
                    const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) s16x4*)(Lu + rr * G::RS + col * 2));
                    const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) s16x4*)(Lu + (rr + 4) * G::RS + col * 2));
                    const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                    afr[i] = __builtin_bit_cast(u32x4, av);
                }
#pragma unroll
                for (int jb = 0; jb < NB; ++jb) {
                    const int col = jb * 16 + 4 * p4;
                    const s16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) s16x4*)(Lq + rr * G::RS + col * 2));
                    const s16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) s16x4*)(Lq + (rr + 4) * G::RS + col * 2));
                    const s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
                    const u32x4 bfr = __builtin_bit_cast(u32x4, bv);
#pragma unroll
                    for (int i = 0; i < IB; ++i) dg[i][jb] = mma16<bf16>(afr[i], bfr, dg[i][jb]);
                }
            }
        }
        // dgamma partial rows of this wave
#pragma unroll
        for (int i = 0; i < IB; ++i)
#pragma unroll
            for (int jb = 0; jb < NB; ++jb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = (d * IB + i) * 16 + 4 * g + r, col = jb * 16 + p;
                    pb[(int64_t)row * C + col] = dg[i][jb][r];
                }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 512) pb[(int64_t)C * C + c] = ((Ldb[c] + Ldb[C + c]) + Ldb[2 * C + c]) + Ldb[3 * C + c];
}

// ---------------------------------------------------------------------------
// launchers (gdn.hip dispatches here)
// ---------------------------------------------------------------------------
// Taken from 32768 pixels up: below, the per-workgroup prologue (gamma staging, first loads) outweighs the
// per-pixel gain (C2's 16 x 32 x 32 layers: lane 7.6 / 9.4 us vs 5.8 / 6.5 us for gdn_fwd_kernel; 16 x 64 x 64:
// 10.2 / 11.8 vs 12.2 / 12.4; 16 x 128 x 128: 25.5 / 28.7 vs 30.8 / 30.6, profiles/r03_gdn_lane_kprof.txt)
constexpr int64_t LANE_MIN_NPIX = 32768;

bool gdn_lane_fwd_ok(int C, int64_t npix, int x_ld, int y_ld) {
    return (C == 64 || C == 128 || C == 192) && npix >= LANE_MIN_NPIX &&
           npix * (int64_t)std::max(x_ld, y_ld) * 2 < (1ll << 31);
}

void launch_gdn_fwd_lane(const void* x, int x_ld, int64_t npix, int C, const void* g, const float* b, int inv, void* y,
                         int y_ld, hipStream_t st) {
    const int64_t ntiles = (npix + 15) / 16;
    const int occ = C <= 128 ? 2 : 1;
    // whole waves of resident blocks, at least two tiles per wave
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(256 * occ, (ntiles + 7) / 8));
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, reinterpret_cast<const bf16*>(x), x_ld, npix,
                           reinterpret_cast<const bf16*>(g), b, reinterpret_cast<bf16*>(y), y_ld);
    };
    if (C == 64)
        inv ? go(gdn_fwd_lane_kernel<64, true, 2>) : go(gdn_fwd_lane_kernel<64, false, 2>);
    else if (C == 128)
        inv ? go(gdn_fwd_lane_kernel<128, true, 2, CAI_GDN_FWD_NSET>) : go(gdn_fwd_lane_kernel<128, false, 2, CAI_GDN_FWD_NSET>);
    else
        inv ? go(gdn_fwd_lane_kernel<192, true, 1>) : go(gdn_fwd_lane_kernel<192, false, 1>);
}

// (backward at 16 x 32 x 32: 15.2 / 16.5 us vs 12.4 / 11.6 for gdn_bwd_fused_kernel; 16 x 64 x 64: 21.6 / 22.2 vs
// 24.2 / 23.9; 16 x 128 x 128: 57.2 / 55.5 vs 65.4 / 63.1)
bool gdn_lane_bwd_ok(int C, int64_t npix, int x_ld, int dy_ld, int dx_ld) {
    return (C == 64 || C == 128) && npix >= LANE_MIN_NPIX &&
           npix * (int64_t)std::max(x_ld, std::max(dy_ld, dx_ld)) * 2 < (1ll << 31);
}

// blocks of the lane backward: one per CU, at least CAI_GDN_LANE_MIN_STEPS (default 2) 64-pixel steps per block
// (the [block][C*C + C] fp32 partials of a block outweigh one step's pixels)
int gdn_lane_bwd_blocks(int64_t npix) {
    static const int min_steps = [] {
        const char* e = getenv("CAI_GDN_LANE_MIN_STEPS");
        return (e && *e) ? std::max(1, atoi(e)) : 2;
    }();
    const int64_t steps = (npix + 63) / 64;
    return (int)std::max<int64_t>(1, std::min<int64_t>(256, (steps + min_steps - 1) / min_steps));
}

void launch_gdn_bwd_lane(const void* x, int x_ld, const void* dy, int dy_ld, int64_t npix, int C, const void* gop,
                         const float* beta, int inv, void* dx, int dx_ld, float* part, int nblk, hipStream_t st) {
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(nblk), dim3(512), 0, st, reinterpret_cast<const bf16*>(x), x_ld,
                           reinterpret_cast<const bf16*>(dy), dy_ld, npix, reinterpret_cast<const bf16*>(gop), beta,
                           reinterpret_cast<bf16*>(dx), dx_ld, part);
    };
    if (C == 64)
        inv ? go(gdn_bwd_lane_kernel<64, true>) : go(gdn_bwd_lane_kernel<64, false>);
    else
        inv ? go(gdn_bwd_lane_kernel<128, true>) : go(gdn_bwd_lane_kernel<128, false>);
}

}  // namespace cai
