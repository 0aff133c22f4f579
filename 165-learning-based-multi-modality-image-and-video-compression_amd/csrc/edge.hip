// The stride-2 "edge" layers of the transforms through the space-to-depth view.
//
//   analysis first layer   Conv2d(C, N, k, stride 2, pad k/2)                models/utils.py conv()
//   synthesis last layer   ConvTranspose2d(N, C, k, stride 2, pad k/2, op 1) models/utils.py deconv()
//   (google.py:96-112 / 145-170 and every model built on them), C <= 3 image channels, k odd <= 5.
//
// Viewing the image as a grid of 2x2 superpixels (S: 4C channels at half resolution, read straight
// from the NCHW fp32 tensor) turns both layers into a 3x3 stride-1 convolution between S and the
// pixel-major bf16 feature map P on the same Hs x Ws grid:
//   conv fwd     P[p][n]   = sum_t sum_ch S[p + off(t)][ch] W1[t][ch][n]            (edge_s2d_kernel)
//   deconv dgrad dX[p][n]  = same form, W1'[t][ch][n] = W2[8 - t][n][ch]            (edge_s2d_kernel)
//   deconv fwd   S[q][c16] = sum_t sum_ci P[q + off(t)][ci] W2[t][ci][c16]          (edge_d2s_kernel)
//   wgrads       G[t][ch][n] = sum_p S[p + off(t)][ch] P[p][n]                       (edge_wgrad_kernel)
//                conv: dW1 = G (+ bias grad from a constant-1 channel); deconv: dW2[t] = G[8 - t]^T
// with W1[t=(dy,dx)][(py,px,ci)][n] = W[n][ci][2dy+py+k/2][2dx+px+k/2] and
// W2[t][ci][(py,px,co)] = W[ci][co][py-2dy+k/2][px-2dx+k/2] (zero where the tap falls outside k x k).
//
// This replaces, for these layers, the image-side pack + 16x-padded implicit GEMM (first layer) and the
// per-pixel GEMM + col2im / im2col pipeline of deconv_small.hip (last layer): every kernel reads its
// HBM operands once, coalesced, stages the 3-row halo in LDS and runs v_mfma_f32_16x16x32_bf16 with
// the weights gathered from the fp32 torch tensors into registers once per (persistent) block.  The
// weight-gradient partials are reduced in a fixed order (no float atomics) straight into the torch
// layout of dW / db.
#include "common.hpp"
#include "reduce_jobs.hpp"
#include "edge_frag.hpp"
#include "mfma.hpp"

#include <algorithm>
#include <cstdlib>

namespace cai {
namespace {

constexpr int TB = 64;            // superpixel columns per tile
constexpr int TBH = TB + 2;       // plus the 3x3 halo
constexpr int SROW = TBH * 32;    // bytes of one staged superpixel row (16 bf16 channels)
constexpr int NT = 256;           // threads of the s2d / wgrad kernels
constexpr int ONES = 12;          // constant-1 superpixel channel (bias gradient of the conv)

struct EdgeArgs {
    const float* img;     // NCHW fp32 [B, C, 2Hs, 2Ws] (x of the conv, dy of the deconv)
    const bf16* feat;     // pixel-major bf16 [B, Hs, Ws, N] (dy of the conv, x of the deconv)
    int feat_ld;
    const u32x4* frag;    // packed weight fragments (edge_frag.hpp)
    const float* bias;
    bf16* out_feat;       // s2d output, pixel-major
    int out_ld;
    float* out_img;       // d2s output, NCHW fp32
    float* part;          // wgrad partials [units][9*16*N + 16]
    int B, C, Hs, Ws, N, k, p;
    int mode;             // 0: conv weights, 1: deconv weights
    int ncb;              // column blocks of TB superpixels
    int rch;              // rows per work unit (d2s / wgrad)
    int units;
    bf16* sbf;            // packed superpixels [B][Hs][Ws][16] bf16 (wgrad DMA path)
    float* cs_part;       // per-pack-block fp32 column sums of the image side [npack][16]
    int npack, ipb;       // pack blocks, superpixels per pack block
};

// s2d A/B knobs, measured on MI355X (the C2 g_a[0] forward / g_s[6] input gradient, 16 x 128 x 128 x 128
// bf16 out, profiles/r02_edge_s2d_ab.log): one tile per block with an LDS-staged epilogue 27.6 us;
// persistent + 8-byte register stores 31.6; 16-byte register stores 27.2; + grid-stride tile order 23.3
// (the default); prefetch distance 2 23.4; nt stores 28.5 / 26.9 (grid-stride).  Timing probes (results
// invalid): stores skipped at run time 12.9, no in-loop image loads 18.8 -- the kernel is issue-bound
// (MFMA + VALU per tile) with the stores on top, against 11.3 us for a torch fill of the same bytes.
#ifndef CAI_EDGE_S2D_PD
#define CAI_EDGE_S2D_PD 1     // prefetch distance in tiles (1 or 2)
#endif
#ifndef CAI_EDGE_S2D_GS
#define CAI_EDGE_S2D_GS 1     // tile order: 1 grid-stride (one output window sweeping), 0 contiguous runs
#endif
#ifndef CAI_EDGE_ST_AUX
#define CAI_EDGE_ST_AUX 0     // cache-policy bits of the output stores (2: nt)
#endif

__device__ __attribute__((aligned(64))) unsigned edge_zero_page[64];
// float stride of one superpixel's 16 partial outputs in the d2s cross-wave sum: 17 (not 16) spreads the
// per-pixel reads of neighbouring threads over the banks (16 put every other pixel on one bank group:
// SQ_LDS_BANK_CONFLICT 0.60 of the LDS cycles, profiles/r03_pmc_c2_kernels.txt)
#ifndef CAI_D2S_RS
#define CAI_D2S_RS 17
#endif
constexpr int D2S_RS = CAI_D2S_RS;

typedef const void __attribute__((address_space(1)))* gvoid_ptr;
typedef void __attribute__((address_space(3)))* lvoid_ptr;

// The LDS DMA issued from inline asm: the builtin is booked by the compiler's waitcnt pass as an LDS write
// of unknown order, so every later fragment read waited for vmcnt(0) -- the ring's prefetches included.
// The kernels here count their DMAs themselves (wait_vmcnt<N> before each step's barrier).  M0 carries the
// wave's LDS base and is restored after the DMA (the compiler reserves it).
__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
    const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds_wave_base));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}

// LDS byte offset of 16-byte slot `slot` of row `row` in a [rows][256 B] bf16 image read by
// ds_read_b64_tr_b16 (the rows 8g+q of a half-wave land on distinct slots)
__device__ __forceinline__ int trswz(int row, int slot) {
    return row * 256 + ((slot ^ (((row & 3) << 1) | (((row >> 3) & 1) << 3))) << 4);
}

// bijective XCD remap: logical ids [x*q, (x+1)*q) run on XCD x (dispatch is round-robin over 8 XCDs)
__device__ __forceinline__ int xcd_remap_e(int wgid, int nwg) {
    const int xcd = wgid & 7, idx = wgid >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ s16x4 ds_tr16(const char* base, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + byte_off));
}
__device__ __forceinline__ u32x4 tr_frag(const char* base, int off0, int off4) {
    const s16x4 a = ds_tr16(base, off0), b = ds_tr16(base, off4);
    const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(u32x4, v);
}

// Ss[dyi][j][16] <- superpixel (a - 1 + dyi, b0 - 1 + j) of image n as bf16, channel (py*2+px)*C + ci,
// channel ONES = 1, zero outside the image.  want_cs: the centre row's fp32 values are added to the
// calling thread's cs[] (each superpixel column of the tile is owned by one fixed thread).
template <int C>
__device__ __forceinline__ void stage_s(const EdgeArgs& A, int n, int a, int b0, char* Ss, float (&cs)[12],
                                        bool want_cs) {
    const int it = threadIdx.x;
    if (it >= 3 * TBH) return;
    const int dyi = it / TBH, j = it - dyi * TBH;
    const int sa = a - 1 + dyi, sb = b0 - 1 + j;
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = 0.f;
    v[ONES] = 1.f;
    if (sa >= 0 && sa < A.Hs && sb >= 0 && sb < A.Ws) {
        const int64_t W2 = 2 * (int64_t)A.Ws;
#pragma unroll
        for (int ci = 0; ci < C; ++ci) {
            const float* base = A.img + ((int64_t)(n * C + ci) * (2 * A.Hs) + 2 * sa) * W2 + 2 * sb;
            const float2 q0 = *reinterpret_cast<const float2*>(base);
            const float2 q1 = *reinterpret_cast<const float2*>(base + W2);
            v[0 * C + ci] = q0.x;
            v[1 * C + ci] = q0.y;
            v[2 * C + ci] = q1.x;
            v[3 * C + ci] = q1.y;
        }
    }
    if (want_cs && dyi == 1 && j >= 1 && j <= TB) {
#pragma unroll
        for (int e = 0; e < 4 * C; ++e) cs[e] += v[e];
    }
    bf16x8 lo, hi;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        lo[e] = (bf16)v[e];
        hi[e] = (bf16)v[8 + e];
    }
    *reinterpret_cast<u32x4*>(Ss + dyi * SROW + j * 32) = __builtin_bit_cast(u32x4, lo);
    *reinterpret_cast<u32x4*>(Ss + dyi * SROW + j * 32 + 16) = __builtin_bit_cast(u32x4, hi);
}

// stage_s split in two for software pipelining: the loads of the next tile (branch-free, clamped
// addresses) are in flight while the current tile is computed.
template <int C>
struct SPre {
    float2 q[2 * C];
    bool ok;
};

template <int C>
__device__ __forceinline__ void s_load(const EdgeArgs& A, int n, int a, int b0, SPre<C>& L) {
    const int it = min((int)threadIdx.x, 3 * TBH - 1);
    const int dyi = it / TBH, j = it - dyi * TBH;
    const int sa = a - 1 + dyi, sb = b0 - 1 + j;
    L.ok = threadIdx.x < 3 * TBH && sa >= 0 && sa < A.Hs && sb >= 0 && sb < A.Ws;
    const int64_t W2 = 2 * (int64_t)A.Ws;
#pragma unroll
    for (int ci = 0; ci < C; ++ci) {
        const float* base =
            L.ok ? A.img + ((int64_t)(n * C + ci) * (2 * A.Hs) + 2 * sa) * W2 + 2 * sb : A.img;
        L.q[2 * ci] = *reinterpret_cast<const float2*>(base);
        L.q[2 * ci + 1] = *reinterpret_cast<const float2*>(base + (L.ok ? W2 : 0));
    }
}

template <int C>
__device__ __forceinline__ void s_store(const SPre<C>& L, char* Ss) {
    const int it = threadIdx.x;
    if (it >= 3 * TBH) return;
    const int dyi = it / TBH, j = it - dyi * TBH;
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = 0.f;
    v[ONES] = 1.f;
    if (L.ok) {
#pragma unroll
        for (int ci = 0; ci < C; ++ci) {
            v[0 * C + ci] = L.q[2 * ci].x;
            v[1 * C + ci] = L.q[2 * ci].y;
            v[2 * C + ci] = L.q[2 * ci + 1].x;
            v[3 * C + ci] = L.q[2 * ci + 1].y;
        }
    }
    bf16x8 lo, hi;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        lo[e] = (bf16)v[e];
        hi[e] = (bf16)v[8 + e];
    }
    *reinterpret_cast<u32x4*>(Ss + dyi * SROW + j * 32) = __builtin_bit_cast(u32x4, lo);
    *reinterpret_cast<u32x4*>(Ss + dyi * SROW + j * 32 + 16) = __builtin_bit_cast(u32x4, hi);
}

// ---------------------------------------------------------------------------
// S (image side) -> P (feature side): conv forward, deconv input gradient.
// Tile = 64 superpixels of one row x all N channels; wave w owns the n-tiles [w*NPW, (w+1)*NPW).
// K = 9 taps x 16 channels in 5 k-steps of two taps (the 10th tap is zero).  Persistent, tiles in
// grid-stride order (the tiles in flight form one contiguous window of the output); the weight fragments
// are loaded once per block and the next tile's image loads are in flight while the current tile is
// computed.  The GEMM is the transposed one
// (weights as A, superpixels as B): each lane holds 4 consecutive channels of one pixel and writes
// them as one 8-byte store, no LDS round trip for the output.
// ---------------------------------------------------------------------------
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned EOOB = 0x80000000u;   // beyond every buffer: loads return 0, stores are dropped

// the 2C float2 image loads of one staged superpixel (s_load as branch-free buffer loads; every
// thread issues all of them, so the waitcnt pass can count them past the tile's stores)
template <int C>
struct SPreB {
    u32x2 q[2 * C];
};

template <int C>
__device__ __forceinline__ void s_load_b(const EdgeArgs& A, __amdgpu_buffer_rsrc_t ir, int n, int a, int b0,
                                         SPreB<C>& L) {
    const int it = min((int)threadIdx.x, 3 * TBH - 1);
    const int dyi = it / TBH, j = it - dyi * TBH;
    const int sa = a - 1 + dyi, sb = b0 - 1 + j;
    const bool ok = ((int)threadIdx.x < 3 * TBH) & (sa >= 0) & (sa < A.Hs) & (sb >= 0) & (sb < A.Ws);
    const int W2 = 2 * A.Ws;
#pragma unroll
    for (int ci = 0; ci < C; ++ci) {
        const unsigned off = (unsigned)((((n * C + ci) * (2 * A.Hs) + 2 * sa) * W2 + 2 * sb) * 4);
        L.q[2 * ci] = __builtin_amdgcn_raw_buffer_load_b64(ir, ok ? off : EOOB, 0, 0);
        L.q[2 * ci + 1] = __builtin_amdgcn_raw_buffer_load_b64(ir, ok ? off + (unsigned)W2 * 4u : EOOB, 0, 0);
    }
}

// out-of-image superpixels arrive as zeros; the constant-1 channel is 1 everywhere (its weights are 0
// in the forward fragments)
template <int C>
__device__ __forceinline__ void s_store_b(const SPreB<C>& L, char* Ss) {
    const int it = threadIdx.x;
    if (it >= 3 * TBH) return;
    const int dyi = it / TBH, j = it - dyi * TBH;
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = 0.f;
    v[ONES] = 1.f;
#pragma unroll
    for (int ci = 0; ci < C; ++ci) {
        const float2 q0 = __builtin_bit_cast(float2, L.q[2 * ci]), q1 = __builtin_bit_cast(float2, L.q[2 * ci + 1]);
        v[0 * C + ci] = q0.x;
        v[1 * C + ci] = q0.y;
        v[2 * C + ci] = q1.x;
        v[3 * C + ci] = q1.y;
    }
    bf16x8 lo, hi;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        lo[e] = (bf16)v[e];
        hi[e] = (bf16)v[8 + e];
    }
    *reinterpret_cast<u32x4*>(Ss + dyi * SROW + j * 32) = __builtin_bit_cast(u32x4, lo);
    *reinterpret_cast<u32x4*>(Ss + dyi * SROW + j * 32 + 16) = __builtin_bit_cast(u32x4, hi);
}

template <int C, int NPW, int PD>
__global__ __launch_bounds__(NT) void edge_s2d_kernel(const EdgeArgs A) {
    constexpr int N = 64 * NPW, NTL = N / 16;
    __shared__ __attribute__((aligned(16))) char Ss[2][3 * SROW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g_ = lane >> 4, i16 = lane & 15;
    const int tiles = A.B * A.Hs * A.ncb;
#if CAI_EDGE_S2D_GS
    // grid-stride: the blocks' current tiles form one contiguous window of the output sweeping through it
    const int t0 = (int)blockIdx.x, t1 = tiles, TS = (int)gridDim.x;
#else
    const int lb = xcd_remap_e((int)blockIdx.x, (int)gridDim.x);
    const int per = tiles / (int)gridDim.x, extra = tiles % (int)gridDim.x;
    const int t0 = lb * per + min(lb, extra), t1 = t0 + per + (lb < extra ? 1 : 0), TS = 1;
#endif
    if (t0 >= t1) return;
    // byte sizes < 2 GiB: launch_s2d splits the batch
    const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(A.img), (short)0, A.B * A.C * 16 * A.Hs * A.Ws, 0x00020000);
    const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
        A.out_feat, (short)0, A.B * A.Hs * A.Ws * A.out_ld * 2, 0x00020000);
    auto decode = [&](int t, int& n, int& a, int& b0) {
        if (t >= t1) t -= TS;   // past the run: reload the last tile (harmless, keeps the load count fixed)
        a = t % A.Hs;
        const int rest = t / A.Hs;
        b0 = (rest % A.ncb) * TB;
        n = rest / A.ncb;
    };
    int n0, a0, b00, n1 = 0, a1 = 0, b01 = 0;
    SPreB<C> pre0, pre1;
    decode(t0, n0, a0, b00);
    s_load_b<C>(A, ir, n0, a0, b00, pre0);
    if (PD == 2) {
        decode(t0 + TS, n1, a1, b01);
        s_load_b<C>(A, ir, n1, a1, b01, pre1);
    }
    // A-operand rows of the first two n-tiles of a wave are permuted so that lane (i16, g_) ends up with
    // channels 8*g_ .. 8*g_ + 7 of the wave's first 32 (row 4*g_ + r of tile j <-> channel 8*g_ + 4*j + r):
    // one 16-byte store per pixel and lane.  A third tile (N = 192) keeps the natural order.
    u32x4 bw[5][NPW];
    f32x4 bias[NPW];
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
        int fnt, flane;   // fragment holding this lane's A row
        if (j < 2) {
            const int c = wave * NPW * 16 + 8 * (i16 >> 2) + 4 * j + (i16 & 3);
            fnt = c >> 4;
            flane = g_ * 16 + (c & 15);
        } else {
            fnt = wave * NPW + j;
            flane = lane;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = j < 2 ? wave * NPW * 16 + 8 * g_ + 4 * j + r : (wave * NPW + j) * 16 + 4 * g_ + r;
            bias[j][r] = A.bias ? A.bias[c] : 0.f;
        }
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) bw[ks][j] = A.frag[(ks * NTL + fnt) * 64 + flane];
    }
    // weights and first tiles landed: inside the loop the only outstanding operations are the next
    // tiles' loads and the stores (the loop-header merge would otherwise wait for them all)
    wait_vmcnt<0>();
    // one tile: stage its superpixels, put the load of tile t + PD in flight, MFMAs, 8-byte stores
    auto tile = [&](char* S, SPreB<C>& P, int& n, int& a, int& b0, int t) {
        s_store_b<C>(P, S);
        __syncthreads();
        const int tn = n, ta = a, tb0 = b0;
        decode(t + PD * TS, n, a, b0);
        s_load_b<C>(A, ir, n, a, b0, P);
        f32x4 acc[4][NPW];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int j = 0; j < NPW; ++j) acc[m][j] = bias[j];
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            const int tap = 2 * ks + (g_ >> 1);
            const int tt = tap < 9 ? tap : 4;
            const int off = (tt / 3) * SROW + (tt % 3) * 32 + 16 * (g_ & 1);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                u32x4 av = *reinterpret_cast<const u32x4*>(S + off + (16 * m + i16) * 32);
                if (tap > 8) av = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                for (int j = 0; j < NPW; ++j) acc[m][j] = mma16<bf16>(bw[ks][j], av, acc[m][j]);
            }
        }
        const int rowoff = ((tn * A.Hs + ta) * A.Ws + tb0) * A.out_ld;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int px = 16 * m + i16;
            const bool ok = tb0 + px < A.Ws;
            {
                bf16x8 h;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    h[r] = (bf16)acc[m][0][r];
                    h[4 + r] = (bf16)acc[m][1][r];
                }
                const unsigned off = (unsigned)((rowoff + px * A.out_ld + wave * NPW * 16 + 8 * g_) * 2);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), orr, ok ? off : EOOB, 0, CAI_EDGE_ST_AUX);
            }
            if (NPW == 3) {
                bf16x4 h;
#pragma unroll
                for (int r = 0; r < 4; ++r) h[r] = (bf16)acc[m][NPW - 1][r];
                const unsigned off =
                    (unsigned)((rowoff + px * A.out_ld + (wave * NPW + NPW - 1) * 16 + 4 * g_) * 2);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), orr, ok ? off : EOOB, 0, CAI_EDGE_ST_AUX);
            }
        }
    };
    for (int t = t0; t < t1; t += PD * TS) {
        tile(Ss[0], pre0, n0, a0, b00, t);
        if (PD == 2 && t + TS < t1) tile(Ss[1], pre1, n1, a1, b01, t + TS);
        if (PD == 1 && t + TS < t1) {   // alternate the staging buffer
            tile(Ss[1], pre0, n0, a0, b00, t + TS);
            t += TS;
        }
    }
}

// ---------------------------------------------------------------------------
// P (feature side) -> S (image side): deconv forward.  NW = N / 32 waves; wave w owns input channels
// [32w, 32w + 32) (one k-step per tap, its 9 weight fragments in registers).  A unit streams the
// feature rows a0 - 1 .. a1 of a 64-superpixel column block through LDS; each staged 16-pixel fragment
// feeds the three output rows it touches (dy = -1, 0, 1) from three rotating accumulator slots, and
// output row r - 1 is complete once row r has been consumed: its per-wave partials meet in LDS, are
// summed in wave order, biased and written as 2 x 128 contiguous fp32 per channel.
// ---------------------------------------------------------------------------
// one feature row (64 + 2 halo superpixels x N channels) in registers: KP 16-byte chunks per thread
template <int NW>
struct RowPre {
    static constexpr int N = 32 * NW, NTH = NW * 64, CH = TBH * (N / 8), KP = (CH + NTH - 1) / NTH;
    u32x4 v[KP];
    unsigned ok;   // bit i: chunk i is inside the image (zero otherwise), applied when stored
};

template <int NW>
__device__ __forceinline__ void row_load(const EdgeArgs& A, int n, int r, int b0, RowPre<NW>& P) {
    using R = RowPre<NW>;
    const bool live = r >= 0 && r < A.Hs;
    const bf16* src = A.feat + ((int64_t)n * A.Hs + (live ? r : 0)) * A.Ws * A.feat_ld;
    P.ok = 0u;
#pragma unroll
    for (int i = 0; i < R::KP; ++i) {
        const int c = threadIdx.x + i * R::NTH;
        const int j = c / (R::N / 8), part = c - j * (R::N / 8);
        const int sb = b0 - 1 + j;
        const bool ok = live && c < R::CH && sb >= 0 && sb < A.Ws;
        P.v[i] = *reinterpret_cast<const u32x4*>(src + (ok ? (int64_t)sb * A.feat_ld + part * 8 : 0));
        P.ok |= (ok ? 1u : 0u) << i;
    }
}

template <int C, int NW, int U>
__device__ __forceinline__ void d2s_row(const EdgeArgs& A, int n, int b0, int a0, int a1, int rr, char* Px,
                                        float* red, const u32x4 (&bw)[9], f32x4 (&acc)[3][4], RowPre<NW>& pre,
                                        const float (&bC)[3]) {
    constexpr int N = 32 * NW, RS = N * 2 + 16, NTH = NW * 64;
    using R = RowPre<NW>;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g_ = lane >> 4, i16 = lane & 15;
    const int r = a0 - 1 + rr;
    const bool live = r >= 0 && r < A.Hs;
    __syncthreads();   // readers of Px / red from the previous row are done
#pragma unroll
    for (int i = 0; i < R::KP; ++i) {
        const int c = threadIdx.x + i * NTH;
        if (c < R::CH) {
            const int j = c / (N / 8), part = c - j * (N / 8);
            *reinterpret_cast<u32x4*>(Px + j * RS + part * 16) =
                ((pre.ok >> i) & 1u) ? pre.v[i] : u32x4{0u, 0u, 0u, 0u};
        }
    }
    __syncthreads();
    if (r + 1 <= a1) row_load<NW>(A, n, r + 1, b0, pre);   // next row in flight during this one
    if (live) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int dxi = 0; dxi < 3; ++dxi) {
                const u32x4 av =
                    *reinterpret_cast<const u32x4*>(Px + (16 * m + i16 + dxi) * RS + (32 * wave + 8 * g_) * 2);
                // feature row r feeds output row r - dy: dy = -1 -> slot U+1, 0 -> U, +1 -> U-1 (mod 3)
                acc[(U + 1) % 3][m] = mma16<bf16>(av, bw[0 + dxi], acc[(U + 1) % 3][m]);
                acc[U % 3][m] = mma16<bf16>(av, bw[3 + dxi], acc[U % 3][m]);
                acc[(U + 2) % 3][m] = mma16<bf16>(av, bw[6 + dxi], acc[(U + 2) % 3][m]);
            }
    }
    constexpr int SL = (U + 2) % 3;   // output row r - 1
    const int a = r - 1;
    if (a >= a0 && a < a1) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[(wave * TB + 16 * m + 4 * g_ + q) * D2S_RS + i16] = acc[SL][m][q];
        __syncthreads();
        const int64_t W2 = 2 * (int64_t)A.Ws;
        const int xw = min(2 * TB, (int)(W2 - 2 * b0));
#pragma unroll
        for (int co = 0; co < C; ++co)
            for (int rem = threadIdx.x; rem < 4 * TB; rem += NTH) {
                const int py = rem / (2 * TB), x = rem - py * (2 * TB);
                const int c16 = (py * 2 + (x & 1)) * C + co;
                float s = bC[co];
#pragma unroll
                for (int w = 0; w < NW; ++w) s += red[(w * TB + (x >> 1)) * D2S_RS + c16];
                if (x < xw) A.out_img[((int64_t)(n * C + co) * (2 * A.Hs) + 2 * a + py) * W2 + 2 * b0 + x] = s;
            }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[SL][m] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int C, int NW>
__global__ __launch_bounds__(NW * 64) void edge_d2s_kernel(const EdgeArgs A) {
    constexpr int N = 32 * NW, RS = N * 2 + 16;
    __shared__ __attribute__((aligned(16))) char smem[TBH * RS + NW * TB * D2S_RS * 4];
    char* Px = smem;
    float* red = reinterpret_cast<float*>(smem + TBH * RS);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float bC[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) bC[c] = (c < C && A.bias) ? A.bias[c] : 0.f;
    u32x4 bw[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) bw[t] = A.frag[(t * NW + wave) * 64 + lane];
    const int nch = (A.Hs + A.rch - 1) / A.rch;
    for (int unit = blockIdx.x; unit < A.units; unit += gridDim.x) {
        const int cb = unit % A.ncb, rest = unit / A.ncb;
        const int ch = rest % nch, n = rest / nch;
        const int a0 = ch * A.rch, a1 = min(a0 + A.rch, A.Hs);
        const int b0 = cb * TB;
        f32x4 acc[3][4];
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[s][m] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int nrows = a1 - a0 + 2;   // feature rows a0 - 1 .. a1
        RowPre<NW> pre;
        row_load<NW>(A, n, a0 - 1, b0, pre);
        for (int i = 0; i < nrows; i += 3) {
            d2s_row<C, NW, 0>(A, n, b0, a0, a1, i, Px, red, bw, acc, pre, bC);
            if (i + 1 < nrows) d2s_row<C, NW, 1>(A, n, b0, a0, a1, i + 1, Px, red, bw, acc, pre, bC);
            if (i + 2 < nrows) d2s_row<C, NW, 2>(A, n, b0, a0, a1, i + 2, Px, red, bw, acc, pre, bC);
        }
    }
}

// ---------------------------------------------------------------------------
// Weight gradient: G[t][ch][n] = sum_p S[p + off(t)][ch] P[p][n] over a unit of rows (all columns),
// K = pixels: both operands come out of pixel-major LDS tiles by ds_read_b64_tr_b16.  Wave w owns
// n-tiles [w*NPW, (w+1)*NPW) and all 9 taps (36*NPW accumulator registers).  The partial of a unit
// and the fp32 column sums of the image side (the deconv's bias gradient) go to the workspace.
// ---------------------------------------------------------------------------
template <int C, int NPW>
__global__ __launch_bounds__(NT) void edge_wgrad_kernel(const EdgeArgs A) {
    constexpr int N = 64 * NPW, RS = N * 2 + 16;
    __shared__ __attribute__((aligned(16))) char Ss[3 * SROW];
    __shared__ __attribute__((aligned(16))) char Pf[TB * RS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    f32x4 acc[9][NPW];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < NPW; ++j) acc[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float cs[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) cs[e] = 0.f;

    const int nch = (A.Hs + A.rch - 1) / A.rch;
    const int unit = blockIdx.x;
    const int ch = unit % nch, n = unit / nch;
    const int a0 = ch * A.rch, a1 = min(a0 + A.rch, A.Hs);
    for (int a = a0; a < a1; ++a)
        for (int cb = 0; cb < A.ncb; ++cb) {
            const int b0 = cb * TB;
            __syncthreads();
            stage_s<C>(A, n, a, b0, Ss, cs, true);
            const bf16* src = A.feat + ((int64_t)n * A.Hs + a) * A.Ws * A.feat_ld;
            for (int c = threadIdx.x; c < TB * (N / 8); c += NT) {
                const int px = c / (N / 8), part = c - px * (N / 8);
                u32x4 v = u32x4{0u, 0u, 0u, 0u};
                if (b0 + px < A.Ws)
                    v = *reinterpret_cast<const u32x4*>(src + (int64_t)(b0 + px) * A.feat_ld + part * 8);
                *reinterpret_cast<u32x4*>(Pf + px * RS + part * 16) = v;
            }
            __syncthreads();
#pragma unroll
            for (int ks = 0; ks < TB / 32; ++ks) {
                const int rr = 32 * ks + 8 * g_ + q_;
                u32x4 bv[NPW];
#pragma unroll
                for (int j = 0; j < NPW; ++j) {
                    const int col = (wave * NPW + j) * 16 + 4 * p4;
                    bv[j] = tr_frag(Pf, rr * RS + col * 2, (rr + 4) * RS + col * 2);
                }
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const char* base = Ss + (t / 3) * SROW + (t % 3) * 32;
                    const u32x4 av = tr_frag(base, rr * 32 + 8 * p4, (rr + 4) * 32 + 8 * p4);
#pragma unroll
                    for (int j = 0; j < NPW; ++j) acc[t][j] = mma16<bf16>(av, bv[j], acc[t][j]);
                }
            }
        }
    const int O = 9 * 16 * N + 16;
    float* P = A.part + (int64_t)unit * O;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < NPW; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) P[(t * 16 + 4 * g_ + q) * N + (wave * NPW + j) * 16 + i16] = acc[t][j][q];
    // image-side column sums: the centre-row owners are threads TBH + 1 .. TBH + TB
    __syncthreads();
    float* red = reinterpret_cast<float*>(Pf);
    const int own = threadIdx.x - (TBH + 1);
    if (own >= 0 && own < TB)
#pragma unroll
        for (int e = 0; e < 12; ++e) red[own * 12 + e] = cs[e];
    __syncthreads();
    if (threadIdx.x < 16) {
        float s = 0.f;
        if (threadIdx.x < 4 * C)
            for (int i = 0; i < TB; ++i) s += red[i * 12 + threadIdx.x];
        P[9 * 16 * N + threadIdx.x] = s;
    }
}

// Image side -> packed bf16 superpixels S[B][Hs][Ws][16] (the constant-1 channel set), and the fp32
// column sums of the image side per pack block (the deconv's bias gradient).  Block b owns the A.ipb
// consecutive superpixels [b*ipb, (b+1)*ipb) of the flattened (n, a, b) order, one per thread and pass
// (coalesced float2 reads of the two image rows, 32-byte contiguous writes); fixed order throughout.
template <int C>
__global__ __launch_bounds__(256) void edge_pack_s_kernel(const EdgeArgs A) {
    float cs[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) cs[e] = 0.f;
    const int64_t items = (int64_t)A.B * A.Hs * A.Ws;
    const int64_t i0 = (int64_t)blockIdx.x * A.ipb, i1 = min(items, i0 + A.ipb);
    const int64_t W2 = 2 * (int64_t)A.Ws;
    for (int64_t it = i0 + threadIdx.x; it < i1; it += 256) {
        const int64_t row = it / A.Ws;
        const int sb = (int)(it - row * A.Ws);
        const int n = (int)(row / A.Hs), a = (int)(row - (int64_t)n * A.Hs);
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = 0.f;
        v[ONES] = 1.f;
#pragma unroll
        for (int ci = 0; ci < C; ++ci) {
            const float* base = A.img + ((int64_t)(n * C + ci) * (2 * A.Hs) + 2 * a) * W2 + 2 * sb;
            const float2 q0 = *reinterpret_cast<const float2*>(base);
            const float2 q1 = *reinterpret_cast<const float2*>(base + W2);
            v[0 * C + ci] = q0.x;
            v[1 * C + ci] = q0.y;
            v[2 * C + ci] = q1.x;
            v[3 * C + ci] = q1.y;
        }
#pragma unroll
        for (int e = 0; e < 4 * C; ++e) cs[e] += v[e];
        bf16x8 lo, hi;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            lo[e] = (bf16)v[e];
            hi[e] = (bf16)v[8 + e];
        }
        bf16* dst = A.sbf + it * 16;
        *reinterpret_cast<u32x4*>(dst) = __builtin_bit_cast(u32x4, lo);
        *reinterpret_cast<u32x4*>(dst + 8) = __builtin_bit_cast(u32x4, hi);
    }
    // wave sums by DPP, then the four waves' partials in order
    __shared__ float red[4][12];
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int e = 0; e < 4 * C; ++e) {
        const float t = wave_sum_dpp(cs[e]);
        if ((threadIdx.x & 63) == 0) red[wave][e] = t;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        float s = 0.f;
        if (threadIdx.x < 4 * C) s = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        A.cs_part[blockIdx.x * 16 + threadIdx.x] = s;
    }
}

// ---------------------------------------------------------------------------
// Weight gradient, N = 128, LDS-DMA staging: one step = one superpixel row a x 128 columns; the
// feature tile [128 px][256 B] (tr-read swizzled) and the three packed superpixel rows a-1..a+1
// [3][132][32 B] arrive by global_load_lds into a 3-stage ring (12 DMA instructions per wave and
// step behind a counted vmcnt), so two steps are in flight while one is consumed.  Wave w owns the
// n-tiles 2w, 2w+1 and all 9 taps: per 32-pixel k-step 2 + 9 fragments feed 18 MFMAs.
// ---------------------------------------------------------------------------
constexpr int WTB = 128;                  // columns per step
constexpr int WPB = WTB * 256;            // feature image bytes
constexpr int WSR = 132 * 32;             // one packed superpixel row (130 used)
constexpr int WSB = 16 * 1024;            // S region: 3 rows, padded to 16 DMA instructions
constexpr int WSTAGE = WPB + WSB;
constexpr int WG = 12;                    // DMA instructions per wave and step

// slot of superpixel j in a packed superpixel row: odd groups of 8 rotated by 4 slots, so the half-wave's
// ds_read_b64_tr_b16 rows j and j+8 land on disjoint banks (linear slots: 2-way conflicts on every S read)
__device__ __forceinline__ int sswz(int j) { return j ^ ((j >> 1) & 4); }

__global__ __launch_bounds__(NT, 1) void edge_wgrad_dma_kernel(const EdgeArgs A) {
    __shared__ __attribute__((aligned(16))) char smem[3 * WSTAGE];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    const int ncb = (A.Ws + WTB - 1) / WTB;
    const int nch = (A.Hs + A.rch - 1) / A.rch;
    const int unit = blockIdx.x;
    const int ch = unit % nch, n = unit / nch;
    const int a0 = ch * A.rch, a1 = min(a0 + A.rch, A.Hs);
    const int nsteps = (a1 - a0) * ncb;
    const char* Pg = reinterpret_cast<const char*>(A.feat);
    const char* Sg = reinterpret_cast<const char*>(A.sbf);

    auto issue = [&](int st, int stage) {
        const int a = a0 + st / ncb, b0 = (st % ncb) * WTB;
        char* base = smem + stage * WSTAGE;
#pragma unroll
        for (int i = 0; i < 8; ++i) {            // feature tile: 32 instructions, 8 per wave
            const int k = i * 4 + wave;
            const int row = k * 4 + (lane >> 4);
            const int sl = (lane & 15) ^ ((((lane >> 4) & 3) << 1) | (((k >> 1) & 1) << 3));
            const int px = b0 + row;
            const void* src = px < A.Ws
                                  ? (const void*)(Pg + ((((int64_t)n * A.Hs + a) * A.Ws + px) * A.feat_ld + sl * 8) * 2)
                                  : (const void*)edge_zero_page;
            glds16(src, base + k * 1024);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {            // superpixel rows: 16 instructions, 4 per wave
            const int k = i * 4 + wave;
            const int off = k * 1024 + lane * 16;
            const void* src = (const void*)edge_zero_page;
            if (off < 3 * WSR) {
                const int sr = off / WSR, rem = off - sr * WSR;
                const int j = sswz(rem / 32);    // the superpixel whose slot this is (sswz is an involution)
                const int sa = a - 1 + sr, sb = b0 - 1 + j;
                if (sa >= 0 && sa < A.Hs && sb >= 0 && sb < A.Ws && j < WTB + 2)
                    src = (const void*)(Sg + ((((int64_t)n * A.Hs + sa) * A.Ws + sb) * 16) * 2 + (rem & 31));
            }
            glds16(src, base + WPB + k * 1024);
        }
    };

    f32x4 acc[9][2];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // superpixel-row read offsets for column shift dx and the +4 half (independent of ks: 32*ks leaves bits 0-3)
    int soff[3][2];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int h = 0; h < 2; ++h) soff[dx][h] = sswz(8 * g_ + q_ + dx + 4 * h) * 32 + 8 * p4;
    if (nsteps > 0) issue(0, 0);
    if (nsteps > 1) issue(1, 1);
    for (int st = 0; st < nsteps; ++st) {
        if (st + 1 < nsteps)
            wait_vmcnt<WG>();
        else
            wait_vmcnt<0>();
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (st + 2 < nsteps) issue(st + 2, (st + 2) % 3);
        const char* Pst = smem + (st % 3) * WSTAGE;
        const char* Sst = Pst + WPB;
#pragma unroll
        for (int ks = 0; ks < WTB / 32; ++ks) {
            const int rr = 32 * ks + 8 * g_ + q_;
            u32x4 bv[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int col = (wave * 2 + j) * 16 + 4 * p4;
                bv[j] = tr_frag(Pst, trswz(rr, col >> 3) + ((col & 7) << 1),
                                trswz(rr + 4, col >> 3) + ((col & 7) << 1));
            }
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const char* sbase = Sst + (t / 3) * WSR + ks * 1024;
                const u32x4 av = tr_frag(sbase, soff[t % 3][0], soff[t % 3][1]);
                acc[t][0] = mma16<bf16>(av, bv[0], acc[t][0]);
                acc[t][1] = mma16<bf16>(av, bv[1], acc[t][1]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const int O = 9 * 16 * 128 + 16;
    float* P = A.part + (int64_t)unit * O;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) P[(t * 16 + 4 * g_ + q) * 128 + (wave * 2 + j) * 16 + i16] = acc[t][j][q];
}

// Weight gradient, N = 192, the same LDS-DMA ring on 64-column steps (three 40 KB stages): the feature tile as
// channels 0-127 in the swizzled [64 px][256 B] image and channels 128-191 in a plain [64 px][128 B] one, the three
// packed superpixel rows [3][68][32 B]; wave w owns the n-tiles 3w .. 3w + 2 (4 + 2 + 2 DMA instructions per wave
// and step).  (The general kernel below ran the C2' / mbt2018 first layers at ~87 us, 3.5x the N = 128 DMA kernel.)
constexpr int W2TB = 64;                  // columns per step
constexpr int W2P0 = W2TB * 256;          // channels 0-127
constexpr int W2P1 = W2TB * 128;          // channels 128-191
constexpr int W2SR = (W2TB + 4) * 32;     // one packed superpixel row (66 used)
constexpr int W2SB = 8 * 1024;            // S region: 3 rows, padded to 8 DMA instructions
constexpr int W2STAGE = W2P0 + W2P1 + W2SB;
constexpr int W2G = 8;                    // DMA instructions per wave and step

__global__ __launch_bounds__(NT, 1) void edge_wgrad_dma192_kernel(const EdgeArgs A) {
    __shared__ __attribute__((aligned(16))) char smem[3 * W2STAGE];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    const int ncb = (A.Ws + W2TB - 1) / W2TB;
    const int nch = (A.Hs + A.rch - 1) / A.rch;
    const int unit = blockIdx.x;
    const int ch = unit % nch, n = unit / nch;
    const int a0 = ch * A.rch, a1 = min(a0 + A.rch, A.Hs);
    const int nsteps = (a1 - a0) * ncb;
    const char* Pg = reinterpret_cast<const char*>(A.feat);
    const char* Sg = reinterpret_cast<const char*>(A.sbf);

    auto issue = [&](int st, int stage) {
        const int a = a0 + st / ncb, b0 = (st % ncb) * W2TB;
        char* base = smem + stage * W2STAGE;
        const char* prow = Pg + (((int64_t)n * A.Hs + a) * A.Ws) * A.feat_ld * 2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {            // channels 0-127: 16 instructions of 4 rows, 4 per wave
            const int k = i * 4 + wave;
            const int row = k * 4 + (lane >> 4);
            const int sl = (lane & 15) ^ ((((lane >> 4) & 3) << 1) | (((k >> 1) & 1) << 3));
            const int px = b0 + row;
            glds16(px < A.Ws ? (const void*)(prow + ((int64_t)px * A.feat_ld + sl * 8) * 2) : (const void*)edge_zero_page,
                   base + k * 1024);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {            // channels 128-191: 8 instructions of 8 rows, 2 per wave
            const int k = i * 4 + wave;
            const int row = k * 8 + (lane >> 3);
            const int px = b0 + row;
            glds16(px < A.Ws ? (const void*)(prow + ((int64_t)px * A.feat_ld + 128 + (lane & 7) * 8) * 2)
                             : (const void*)edge_zero_page,
                   base + W2P0 + k * 1024);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {            // superpixel rows: 8 instructions, 2 per wave
            const int k = i * 4 + wave;
            const int off = k * 1024 + lane * 16;
            const void* src = (const void*)edge_zero_page;
            if (off < 3 * W2SR) {
                const int sr = off / W2SR, rem = off - sr * W2SR;
                const int j = sswz(rem / 32);
                const int sa = a - 1 + sr, sb = b0 - 1 + j;
                if (sa >= 0 && sa < A.Hs && sb >= 0 && sb < A.Ws && j < W2TB + 2)
                    src = (const void*)(Sg + ((((int64_t)n * A.Hs + sa) * A.Ws + sb) * 16) * 2 + (rem & 31));
            }
            glds16(src, base + W2P0 + W2P1 + k * 1024);
        }
    };

    f32x4 acc[9][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = acc[t][2] = f32x4{0.f, 0.f, 0.f, 0.f};
    int soff[3][2];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int h = 0; h < 2; ++h) soff[dx][h] = sswz(8 * g_ + q_ + dx + 4 * h) * 32 + 8 * p4;
    if (nsteps > 0) issue(0, 0);
    if (nsteps > 1) issue(1, 1);
    for (int st = 0; st < nsteps; ++st) {
        if (st + 1 < nsteps)
            wait_vmcnt<W2G>();
        else
            wait_vmcnt<0>();
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (st + 2 < nsteps) issue(st + 2, (st + 2) % 3);
        const char* P0 = smem + (st % 3) * W2STAGE;
        const char* P1 = P0 + W2P0;
        const char* Sst = P1 + W2P1;
#pragma unroll
        for (int ks = 0; ks < W2TB / 32; ++ks) {
            const int rr = 32 * ks + 8 * g_ + q_;
            u32x4 bv[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int nt = wave * 3 + j;
                if (nt < 8) {
                    const int col = nt * 16 + 4 * p4;
                    bv[j] = tr_frag(P0, trswz(rr, col >> 3) + ((col & 7) << 1),
                                    trswz(rr + 4, col >> 3) + ((col & 7) << 1));
                } else {
                    const int col = (nt - 8) * 16 + 4 * p4;
                    bv[j] = tr_frag(P1, rr * 128 + col * 2, (rr + 4) * 128 + col * 2);
                }
            }
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const char* sbase = Sst + (t / 3) * W2SR + ks * 1024;
                const u32x4 av = tr_frag(sbase, soff[t % 3][0], soff[t % 3][1]);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[t][j] = mma16<bf16>(av, bv[j], acc[t][j]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const int O = 9 * 16 * 192 + 16;
    float* P = A.part + (int64_t)unit * O;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) P[(t * 16 + 4 * g_ + q) * 192 + (wave * 3 + j) * 16 + i16] = acc[t][j][q];
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
bool edge_geo(const cai_conv_geom* g, int dtype, EdgeArgs& A) {
    if (!g || dtype != CAI_BF16 || g->batch < 1 || g->stride != 2 || g->kernel % 2 == 0 || g->kernel > 5 ||
        g->pad != g->kernel / 2)
        return false;
    A = EdgeArgs{};
    A.B = g->batch;
    A.k = g->kernel;
    A.p = g->pad;
    if (!g->transposed) {
        if (g->output_padding != 0 || g->in_h != 2 * g->out_h || g->in_w != 2 * g->out_w) return false;
        A.C = g->in_c;
        A.N = g->out_c;
        A.Hs = g->out_h;
        A.Ws = g->out_w;
        A.mode = 0;
    } else {
        if (g->out_h != 2 * g->in_h || g->out_w != 2 * g->in_w) return false;
        A.C = g->out_c;
        A.N = g->in_c;
        A.Hs = g->in_h;
        A.Ws = g->in_w;
        A.mode = 1;
    }
    if (A.C < 1 || A.C > 3 || (A.N != 128 && A.N != 192) || A.Hs < 1 || A.Ws < 1) return false;
    A.ncb = (A.Ws + TB - 1) / TB;
    return true;
}

int wgrad_units(const EdgeArgs& A, int* rch) {
    const int64_t rows = (int64_t)A.B * A.Hs;
    const int r = (int)std::max<int64_t>(1, (rows + 255) / 256);
    *rch = r;
    return A.B * ((A.Hs + r - 1) / r);
}

// the LDS-DMA weight-gradient kernels: N = 128, and N = 192 (A/B knob CAI_EDGE_WGRAD_DMA192=0: the general kernel)
bool edge_wgrad_dma(const EdgeArgs& A) {
    static const bool dma192 = [] {
        const char* e = std::getenv("CAI_EDGE_WGRAD_DMA192");
        return !(e && *e == '0');
    }();
    return A.N == 128 || (A.N == 192 && dma192);
}

// workspace of the wgrad: [unit partials][packed superpixels (DMA kernels)][pack column sums]
struct WgradWs {
    size_t off_sbf, off_cs, total;
    int npack, ipb;
};
WgradWs wgrad_ws(const EdgeArgs& A) {
    WgradWs W{};
    int rch;
    const int units = wgrad_units(A, &rch);
    const int64_t rows = (int64_t)A.B * A.Hs;
    // about 1024 pack blocks of 256 threads, one superpixel per thread and pass
    const int64_t items = rows * A.Ws;
    W.ipb = (int)(256 * std::max<int64_t>(1, (items + 256 * 1024 - 1) / (256 * 1024)));
    W.npack = (int)((items + W.ipb - 1) / W.ipb);
    auto up = [](size_t v) { return (v + 255) / 256 * 256; };
    W.off_sbf = up((size_t)units * (9 * 16 * A.N + 16) * sizeof(float));
    W.off_cs = W.off_sbf + (edge_wgrad_dma(A) ? up((size_t)rows * A.Ws * 32) : 0);
    W.total = W.off_cs + up((size_t)W.npack * 16 * sizeof(float));
    return W;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// persistent blocks per CU of the s2d kernel (A/B knob CAI_EDGE_S2D_BPC, read once; 0: one tile per block)
int s2d_blocks_per_cu() {
    static const int v = [] {
        const char* e = std::getenv("CAI_EDGE_S2D_BPC");
        return e ? std::max(0, std::atoi(e)) : 3;
    }();
    return v;
}

template <int C>
void launch_s2d(const EdgeArgs& A, hipStream_t st) {
    const int bpc = s2d_blocks_per_cu();
    // the kernel addresses image and output with 32-bit byte offsets: batches of < 2 GiB each
    const int64_t per_img = std::max<int64_t>((int64_t)A.C * 16 * A.Hs * A.Ws, (int64_t)A.Hs * A.Ws * A.out_ld * 2);
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(A.B, ((int64_t)1 << 31) / 2 / per_img));
    for (int b = 0; b < A.B; b += nb) {
        EdgeArgs P = A;
        P.B = std::min(nb, A.B - b);
        P.img = A.img + (int64_t)b * A.C * 4 * A.Hs * A.Ws;
        P.out_feat = A.out_feat + (int64_t)b * A.Hs * A.Ws * A.out_ld;
        const int pt = P.B * P.Hs * P.ncb;
        const int grid = bpc == 0 ? pt : std::min(pt, 256 * bpc);
        if (CAI_EDGE_S2D_PD == 2) {
            if (A.N == 128)
                edge_s2d_kernel<C, 2, 2><<<grid, NT, 0, st>>>(P);
            else
                edge_s2d_kernel<C, 3, 2><<<grid, NT, 0, st>>>(P);
        } else {
            if (A.N == 128)
                edge_s2d_kernel<C, 2, 1><<<grid, NT, 0, st>>>(P);
            else
                edge_s2d_kernel<C, 3, 1><<<grid, NT, 0, st>>>(P);
        }
    }
}

template <int C>
void launch_d2s(EdgeArgs A, hipStream_t st) {
    int rch = 8;
    auto units = [&](int r) { return A.B * A.ncb * ((A.Hs + r - 1) / r); };
    while (rch > 2 && units(rch) < 1024) rch /= 2;
    A.rch = rch;
    A.units = units(rch);
    const int grid = std::min(A.units, 2048);
    if (A.N == 128)
        edge_d2s_kernel<C, 4><<<grid, 256, 0, st>>>(A);
    else
        edge_d2s_kernel<C, 6><<<grid, 384, 0, st>>>(A);
}

// the weight-gradient kernels, then their fixed-order reduce as a job (reduce_jobs.hip): returned to a
// deferring caller or run now
template <int C>
void launch_wgrad(EdgeArgs A, char* ws, float* dw, float* db, int accumulate, hipStream_t st, cai_reduce_job* J) {
    const int O = 9 * 16 * A.N + 16;
    *J = cai_reduce_job{};
    J->kind = CAI_JOB_EDGE;
    J->nblocks = O / 16;
    J->p[0] = A.part; J->p[2] = dw; J->p[3] = db;
    J->i[0] = A.N; J->i[1] = A.units; J->i[2] = A.mode; J->i[3] = A.k; J->i[4] = A.p; J->i[5] = C;
    J->i[8] = accumulate;
    if (edge_wgrad_dma(A)) {   // packed superpixels + LDS-DMA ring
        const WgradWs W = wgrad_ws(A);
        A.sbf = reinterpret_cast<bf16*>(ws + W.off_sbf);
        A.cs_part = reinterpret_cast<float*>(ws + W.off_cs);
        A.npack = W.npack;
        A.ipb = W.ipb;
        edge_pack_s_kernel<C><<<W.npack, 256, 0, st>>>(A);
        if (A.N == 128)
            edge_wgrad_dma_kernel<<<A.units, NT, 0, st>>>(A);
        else
            edge_wgrad_dma192_kernel<<<A.units, NT, 0, st>>>(A);
        J->p[1] = A.cs_part; J->i[6] = W.npack; J->i[7] = 16;
    } else {
        edge_wgrad_kernel<C, 3><<<A.units, NT, 0, st>>>(A);
        J->p[1] = A.part + 9 * 16 * A.N; J->i[6] = A.units; J->i[7] = O;
    }
}

__global__ __launch_bounds__(256) void edge_pack_frag_kernel(const float* __restrict__ w, EdgeFragSpec s,
                                                             u32x4* __restrict__ out) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f >= s.nfrag) return;
    float v[8];
    edge_frag_values(w, s.C, s.N, s.k, s.p, s.emode, f, v);
    bf16x8 h;
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
    out[f] = __builtin_bit_cast(u32x4, h);
}

#define EDGE_BY_C(fn, ...)                  \
    switch (A.C) {                          \
        case 1: fn<1>(__VA_ARGS__); break;  \
        case 2: fn<2>(__VA_ARGS__); break;  \
        default: fn<3>(__VA_ARGS__); break; \
    }

}  // namespace

// direction 0: the forward (s2d for the conv, d2s for the deconv); 1: the deconv's input gradient
bool edge_frag_spec(const cai_conv_geom* g, int dtype, int direction, EdgeFragSpec& s) {
    EdgeArgs A;
    if (!edge_geo(g, dtype, A) || direction < 0 || direction > 1 || (direction == 1 && A.mode == 0)) return false;
    s.C = A.C;
    s.N = A.N;
    s.k = A.k;
    s.p = A.p;
    s.emode = A.mode == 0 ? 0 : (direction == 0 ? 2 : 1);
    s.nfrag = s.emode == 2 ? 9 * (A.N / 32) * 64 : 5 * (A.N / 16) * 64;
    return true;
}

}  // namespace cai

using namespace cai;

extern "C" {

int cai_edge_supported(const cai_conv_geom* g, int dtype) {
    EdgeArgs A;
    return edge_geo(g, dtype, A) ? 1 : 0;
}

size_t cai_edge_workspace_bytes(const cai_conv_geom* g, int dtype) {
    EdgeArgs A;
    if (!edge_geo(g, dtype, A)) return 0;
    return wgrad_ws(A).total;
}

size_t cai_edge_frag_bytes(const cai_conv_geom* g, int dtype, int direction) {
    EdgeFragSpec s;
    return edge_frag_spec(g, dtype, direction, s) ? (size_t)s.nfrag * 16 : 0;
}

int cai_edge_pack_weights(const cai_conv_geom* g, int dtype, int direction, const float* w, void* frag,
                          void* stream) {
    EdgeFragSpec s;
    CAI_CHECK_ARG(edge_frag_spec(g, dtype, direction, s), "edge_pack_weights: unsupported geometry / direction");
    CAI_CHECK_ARG(w && frag && aligned16(frag), "edge_pack_weights: null or misaligned pointer");
    edge_pack_frag_kernel<<<(s.nfrag + 255) / 256, 256, 0, as_stream(stream)>>>(w, s, static_cast<u32x4*>(frag));
    CAI_LAUNCH_CHECK("edge_pack_weights");
    return CAI_OK;
}

int cai_edge_conv_fwd(const cai_conv_geom* g, const float* x, const void* frag, const float* bias, void* y,
                      int32_t y_ld, void* stream) {
    EdgeArgs A;
    CAI_CHECK_ARG(g && !g->transposed && edge_geo(g, CAI_BF16, A), "edge_conv_fwd: unsupported geometry");
    CAI_CHECK_ARG(x && frag && y && aligned16(y) && aligned16(frag) && ((uintptr_t)x & 7) == 0,
                  "edge_conv_fwd: null or misaligned pointer");
    CAI_CHECK_ARG(y_ld >= A.N && y_ld % 8 == 0, "edge_conv_fwd: y_ld %d", y_ld);
    A.img = x;
    A.frag = static_cast<const u32x4*>(frag);
    A.bias = bias;
    A.out_feat = static_cast<bf16*>(y);
    A.out_ld = y_ld;
    EDGE_BY_C(launch_s2d, A, as_stream(stream));
    CAI_LAUNCH_CHECK("edge_conv_fwd");
    return CAI_OK;
}

int cai_edge_deconv_fwd(const cai_conv_geom* g, const void* x, int32_t x_ld, const void* frag, const float* bias,
                        float* y, void* stream) {
    EdgeArgs A;
    CAI_CHECK_ARG(g && g->transposed && edge_geo(g, CAI_BF16, A), "edge_deconv_fwd: unsupported geometry");
    CAI_CHECK_ARG(x && frag && y && aligned16(x) && aligned16(frag), "edge_deconv_fwd: null or misaligned pointer");
    CAI_CHECK_ARG(x_ld >= A.N && x_ld % 8 == 0, "edge_deconv_fwd: x_ld %d", x_ld);
    A.feat = static_cast<const bf16*>(x);
    A.feat_ld = x_ld;
    A.frag = static_cast<const u32x4*>(frag);
    A.bias = bias;
    A.out_img = y;
    EDGE_BY_C(launch_d2s, A, as_stream(stream));
    CAI_LAUNCH_CHECK("edge_deconv_fwd");
    return CAI_OK;
}

int cai_edge_deconv_dgrad(const cai_conv_geom* g, const float* dy, const void* frag, void* dx, int32_t dx_ld,
                          void* stream) {
    EdgeArgs A;
    CAI_CHECK_ARG(g && g->transposed && edge_geo(g, CAI_BF16, A), "edge_deconv_dgrad: unsupported geometry");
    CAI_CHECK_ARG(dy && frag && dx && aligned16(dx) && aligned16(frag) && ((uintptr_t)dy & 7) == 0,
                  "edge_deconv_dgrad: null or misaligned pointer");
    CAI_CHECK_ARG(dx_ld >= A.N && dx_ld % 8 == 0, "edge_deconv_dgrad: dx_ld %d", dx_ld);
    A.img = dy;
    A.frag = static_cast<const u32x4*>(frag);
    A.out_feat = static_cast<bf16*>(dx);
    A.out_ld = dx_ld;
    EDGE_BY_C(launch_s2d, A, as_stream(stream));
    CAI_LAUNCH_CHECK("edge_deconv_dgrad");
    return CAI_OK;
}

static int run_edge_wgrad(const cai_conv_geom* g, const float* img, const void* feat, int32_t feat_ld, float* dw,
                          float* db, int32_t accumulate, void* workspace, size_t ws_bytes, void* stream,
                          cai_reduce_job* job) {
    EdgeArgs A;
    CAI_CHECK_ARG(edge_geo(g, CAI_BF16, A), "edge_wgrad: unsupported geometry");
    CAI_CHECK_ARG(img && feat && dw && aligned16(feat) && ((uintptr_t)img & 7) == 0,
                  "edge_wgrad: null or misaligned pointer");
    CAI_CHECK_ARG(feat_ld >= A.N && feat_ld % 8 == 0, "edge_wgrad: feat_ld %d", feat_ld);
    CAI_CHECK_ARG(workspace && ws_bytes >= cai_edge_workspace_bytes(g, CAI_BF16), "edge_wgrad: workspace too small");
    A.img = img;
    A.feat = static_cast<const bf16*>(feat);
    A.feat_ld = feat_ld;
    A.part = static_cast<float*>(workspace);
    A.units = wgrad_units(A, &A.rch);
    cai_reduce_job J{};
    EDGE_BY_C(launch_wgrad, A, static_cast<char*>(workspace), dw, db, accumulate, as_stream(stream), &J);
    CAI_LAUNCH_CHECK("edge_wgrad");
    if (job) {
        *job = J;
        return CAI_OK;
    }
    return launch_reduce_jobs(&J, 1, as_stream(stream));
}

int cai_edge_wgrad(const cai_conv_geom* g, const float* img, const void* feat, int32_t feat_ld, float* dw, float* db,
                   int32_t accumulate, void* workspace, size_t ws_bytes, void* stream) {
    return run_edge_wgrad(g, img, feat, feat_ld, dw, db, accumulate, workspace, ws_bytes, stream, nullptr);
}

int cai_edge_wgrad_deferred(const cai_conv_geom* g, const float* img, const void* feat, int32_t feat_ld, float* dw,
                            float* db, int32_t accumulate, void* workspace, size_t ws_bytes, void* stream,
                            cai_reduce_job* job) {
    CAI_CHECK_ARG(job, "edge_wgrad_deferred: null job");
    return run_edge_wgrad(g, img, feat, feat_ld, dw, db, accumulate, workspace, ws_bytes, stream, job);
}

}  // extern "C"
