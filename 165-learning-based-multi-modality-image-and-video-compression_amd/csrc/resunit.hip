// cheng2020's ResidualUnit (compressai/layers/layers.py:211-226: AttentionBlock's conv_a / conv_b units,
// :225-236) in ONE launch per direction:
//     h1 = relu(conv1x1_a(x) + ba)        N -> N/2
//     h2 = relu(conv3x3_b(h1) + bb)       N/2 -> N/2, pad 1
//     y  = relu(conv1x1_c(h2) + bc + x)   N/2 -> N
// Unfused, a unit is three conv launches per direction (nine per training step with the weight gradients); at the
// per-GPU batch of C4 (4 x 64 x 64 and 4 x 16 x 16 latents) each is a small-grid, launch- and latency-bound GEMM.
//
// A 512-thread block owns an 8 x 8 tile of output pixels and all channels.  Three MFMA phases, all operands in LDS:
//   A  1x1 over the tile's 10 x 10 halo (the 3x3's input footprint): the halo's N-channel pixels and the layer's
//      weights staged in MFMA fragment order (16 x 32 bf16 operands, lane-linear 1 KiB pieces: conflict-free reads;
//      weights by LDS DMA, activations by register loads);  the N/2-channel result goes to an LDS image, zero
//      outside the image (the 3x3's zero padding);
//   B  3x3 over that image: 9 taps x N/2 channels, the tap weights streamed through a 4-deep LDS-DMA ring (one
//      barrier per tap); result to a second LDS image;
//   C  1x1 back to N channels, the epilogue adds the residual and stores 8 bytes per lane (transposed MFMA
//      accumulators: each lane holds 4 consecutive channels of one pixel).
// The halo costs phase A 100 / 64 of its pixels: 6 % of the unit's MACs at N = 192.
//
// Backward (input gradient; the weight gradients stay GEMMs over all pixels, compressai/_ops.py): the same three
// phases on the transposed weights (direction-1 packs of c, b, a) --
//     gc = gy * (y > 0)                          (unless the consumer already masked gy)
//     gb = (gc Wc^T) * (h2 > 0)                  on the halo
//     ga = conv3x3^T(gb) * (h1 > 0)              taps read (r + 2 - ty, c + 2 - tx) of the halo
//     dx = (ga Wa^T + gc [+ res2]) [* (xmask > 0)]
// and writes gc / gb / ga for the weight gradients.  Arithmetic: bf16 operands, fp32 accumulation, bf16 results
// -- the unfused chain's, with the MFMA K order of this kernel.
#include "common.hpp"
#include "mfma.hpp"
#include "reduce_jobs.hpp"

#include <algorithm>
#include <cstdlib>

namespace cai {
namespace {

template <int NC>
struct RuCfg {
    static constexpr int NH = NC / 2;
    static constexpr int TH = 8, TW = 8, HW = TW + 2, HPX = (TH + 2) * HW;   // 100 halo pixels
    static constexpr int MTA = (HPX + 15) / 16;             // 7 M tiles over the halo
    static constexpr int KA = NC / 32, NTA = NH / 16;       // phase A: K steps, N tiles (also phase B's N tiles)
    static constexpr int KB = NH / 32;                      // phase B: K steps per tap
    static constexpr int NTC = NC / 16, KC = NH / 32;       // phase C
    static constexpr int FRAG = 1024;                       // one 16 x 32 bf16 operand, lane-linear
    static constexpr int XA = MTA * KA * FRAG, WA = NTA * KA * FRAG;
    static constexpr int TAPB = NTA * KB * FRAG, NSTB = 4;  // one tap of the 3x3 weights; ring depth
    static constexpr int R1 = (XA + WA > NSTB * TAPB) ? XA + WA : NSTB * TAPB;
    // hidden-image row stride: 240 B keeps the tap-shifted 16-byte fragment reads and the 8-byte epilogue stores
    // at most 2-way on the banks for N/2 = 64 and 96 (a 192-B stride is 8-way on the stores)
    static constexpr int SH = 240;
    static constexpr int H1B = MTA * 16 * SH, H2B = 64 * SH;
    static constexpr int WC = NTC * KC * FRAG;
    static constexpr int BYTES = R1 + H1B + WC + H2B;
    static_assert(SH >= 2 * NH && BYTES <= 160 * 1024, "resunit LDS");
    static_assert(NTA % 2 == 0 && NTC % 2 == 0, "two wave columns");
};

struct RuArgs {
    const bf16* x;                   // forward: x; backward: gy
    const bf16* y;                   // backward: y (its ReLU mask when !gy_masked)
    const bf16 *wa, *wb, *wc;        // packed: forward a, b, c (direction 0); backward c, b, a (direction 1)
    const float *ba, *bb, *bc;       // forward biases
    bf16 *h1, *h2;                   // forward outputs / backward masks (ld N/2)
    bf16* out;                       // y / dx
    bf16 *gc, *gb, *ga;              // backward outputs (ld N, N/2, N/2); gc unused when gy_masked
    const bf16* res2;                // backward: one more gradient of x, added to dx (NULL: none)
    const bf16* xmask;               // backward: dx *= (xmask > 0) (NULL: none)
    int x_ld, y_ld, out_ld, res2_ld, xmask_ld;
    int kpa, kpb, kpc;
    int B, H, W, tiles_x, tiles_y;
    int gy_masked;
};

__device__ __forceinline__ u32x4 keep_pos(u32x4 v, u32x4 m) {   // v where m > 0 (bf16 lanes), else 0
    const bf16x8 mv = __builtin_bit_cast(bf16x8, m);
    bf16x8 vv = __builtin_bit_cast(bf16x8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) vv[e] = (float)mv[e] > 0.f ? vv[e] : (bf16)0.f;
    return __builtin_bit_cast(u32x4, vv);
}

template <int NC, bool BWD>
__global__ __launch_bounds__(512, 1) void resunit_kernel(const RuArgs a) {
    using R = RuCfg<NC>;
    constexpr int NH = R::NH, KA = R::KA, NTA = R::NTA, KB = R::KB, NTC = R::NTC, KC = R::KC, MTA = R::MTA;
    constexpr int FRAG = R::FRAG, SH = R::SH, NSTB = R::NSTB;
    constexpr int NJA = NTA / 2, NJC = NTC / 2;
    __shared__ __attribute__((aligned(16))) char smem[R::BYTES];
    char* const sXA = smem;
    char* const sWA = smem + R::XA;
    char* const ring = smem;                       // phase B reuses phase A's region
    char* const sH1 = smem + R::R1;
    char* const sWC = sH1 + R::H1B;
    char* const sH2 = sWC + R::WC;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l16 = lane & 15, lg = lane >> 4;
    const int per_img = a.tiles_x * a.tiles_y;
    const int b = blockIdx.x / per_img, rt = blockIdx.x - (blockIdx.x / per_img) * per_img;
    const int y0 = (rt / a.tiles_x) * R::TH, x0 = (rt - (rt / a.tiles_x) * a.tiles_x) * R::TW;
    auto pix = [&](int yy, int xx) -> int64_t { return ((int64_t)b * a.H + yy) * a.W + xx; };
    // weight fragment (N tile nt, K elements kofs ..): lane -> packed row nt * 16 + l16, 8 elements from 8 lg
    auto wsrc = [&](const bf16* w, int kp, int nt, int kofs) -> const void* {
        return w + (int64_t)(nt * 16 + l16) * kp + kofs + 8 * lg;
    };

    // ---- staging: phase A weights (DMA), phase A activations (registers -> LDS), phase C weights (DMA) ----
    for (int f = wave; f < NTA * KA; f += 8) {
        const int nt = f / KA, ks = f - (f / KA) * KA;
        glds16_asm(wsrc(a.wa, a.kpa, nt, ks * 32), sWA + f * FRAG);
    }
    for (int f = wave; f < MTA * KA; f += 8) {
        const int mt = f / KA, ks = f - (f / KA) * KA;
        const int q = mt * 16 + l16, hy = q / R::HW, hx = q - (q / R::HW) * R::HW;
        const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
        const bool in = q < R::HPX && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (in) {
            const int64_t p = pix(yy, xx);
            v = *reinterpret_cast<const u32x4*>(a.x + p * a.x_ld + ks * 32 + 8 * lg);
            if (BWD && !a.gy_masked) {
                v = keep_pos(v, *reinterpret_cast<const u32x4*>(a.y + p * a.y_ld + ks * 32 + 8 * lg));
                if (hy >= 1 && hy <= R::TH && hx >= 1 && hx <= R::TW)
                    *reinterpret_cast<u32x4*>(a.gc + p * NC + ks * 32 + 8 * lg) = v;
            }
        }
        *reinterpret_cast<u32x4*>(sXA + f * FRAG + lane * 16) = v;
    }
    int nwc = 0;
    for (int f = wave; f < NTC * KC; f += 8, ++nwc) {
        const int nt = f / KC, ks = f - (f / KC) * KC;
        glds16_asm(wsrc(a.wc, a.kpc, nt, ks * 32), sWC + f * FRAG);
    }
    wait_vmcnt_n(nwc);      // this wave's phase A weights landed (only its phase C DMAs may be in flight)
    wait_lgkmcnt0();
    __builtin_amdgcn_s_barrier();

    // ---- phase A: [112 halo px x N] . [N x N/2]; wave (mg, nh): M tiles mg, mg + 4; N tiles nh * NJA .. ----
    const int mg = wave & 3, nh = wave >> 2;
    {
        f32x4 acc[2][NJA];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < NJA; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        const bool two = mg + 4 < MTA;
#pragma unroll
        for (int ks = 0; ks < KA; ++ks) {
            u32x4 fa[2];
            fa[0] = *reinterpret_cast<const u32x4*>(sXA + (mg * KA + ks) * FRAG + lane * 16);
            fa[1] = two ? *reinterpret_cast<const u32x4*>(sXA + ((mg + 4) * KA + ks) * FRAG + lane * 16) : fa[0];
#pragma unroll
            for (int j = 0; j < NJA; ++j) {
                const u32x4 fb = *reinterpret_cast<const u32x4*>(sWA + ((nh * NJA + j) * KA + ks) * FRAG + lane * 16);
                acc[0][j] = mma16<bf16>(fb, fa[0], acc[0][j]);
                if (two) acc[1][j] = mma16<bf16>(fb, fa[1], acc[1][j]);
            }
        }
        // epilogue A: lane = halo pixel q, channels c0 .. c0 + 3.  Every load (bias / mask) is issued before the
        // first store: a load behind a store waits for it on the shared vmcnt, and the per-j load -> store chain
        // serialized the epilogues (the same for B and C below)
        int qv[2], pv[2];
        bool inv[2], intv[2];
        f32x4 bA[NJA];
        bf16x4 mA[2][NJA];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = (mg + 4 * i) * 16 + l16, hy = q / R::HW, hx = q - (q / R::HW) * R::HW;
            const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
            inv[i] = (i == 0 || two) && q < R::HPX && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
            intv[i] = inv[i] && hy >= 1 && hy <= R::TH && hx >= 1 && hx <= R::TW;
            qv[i] = q;
            pv[i] = inv[i] ? (int)pix(yy, xx) : 0;
        }
#pragma unroll
        for (int j = 0; j < NJA; ++j) {
            const int c0 = (nh * NJA + j) * 16 + 4 * lg;
            if (!BWD) {
#pragma unroll
                for (int r = 0; r < 4; ++r) bA[j][r] = a.ba[c0 + r];
            } else {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    mA[i][j] = bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
                    if (inv[i]) mA[i][j] = *reinterpret_cast<const bf16x4*>(a.h2 + (int64_t)pv[i] * NH + c0);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i == 1 && !two) break;
            const int q = qv[i];
            const bool in = inv[i], interior = intv[i];
            const int64_t p = pv[i];
#pragma unroll
            for (int j = 0; j < NJA; ++j) {
                const int c0 = (nh * NJA + j) * 16 + 4 * lg;
                bf16x4 hv;
                if (!BWD) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) hv[r] = (bf16)(in ? fmaxf(acc[i][j][r] + bA[j][r], 0.f) : 0.f);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) hv[r] = (bf16)((float)mA[i][j][r] > 0.f ? acc[i][j][r] : 0.f);
                }
                *reinterpret_cast<bf16x4*>(sH1 + q * SH + c0 * 2) = hv;
                if (interior) *reinterpret_cast<bf16x4*>((BWD ? a.gb : a.h1) + p * NH + c0) = hv;
            }
        }
    }
    wait_lgkmcnt0();
    __builtin_amdgcn_s_barrier();      // the halo image is complete; phase A's operands are dead (ring may refill)

    // ---- phase B: 3x3 over the halo image, tap weights through the DMA ring ----
    constexpr int FB = NTA * KB;       // weight fragments per tap
    const int nd = wave < FB ? (FB - 1 - wave) / 8 + 1 : 0;   // this wave's DMAs per tap
    auto issue_tap = [&](int t) {
        if (t >= 9) return;
        for (int f = wave; f < FB; f += 8) {
            const int nt = f / KB, ks = f - (f / KB) * KB;
            glds16_asm(wsrc(a.wb, a.kpb, nt, t * NH + ks * 32), ring + (t % NSTB) * R::TAPB + f * FRAG);
        }
    };
    issue_tap(0);
    issue_tap(1);
    issue_tap(2);
    const int mb = mg;                              // output rows 2 mb, 2 mb + 1 of the tile
    const int orow = 2 * mb + (l16 >> 3), ocol = l16 & 7;
    f32x4 accb[NJA];
#pragma unroll
    for (int j = 0; j < NJA; ++j) accb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        // taps t + 1, t + 2 (when they exist) were issued after tap t: everything older has landed
        wait_vmcnt_n((t + 2 <= 8 ? 2 : 8 - t) * nd);
        __builtin_amdgcn_s_barrier();   // every wave's tap-t DMAs landed, every wave done with tap t - 1's stage
        issue_tap(t + 3);               // into stage (t + 3) % 4 = (t - 1) % 4
        const int ty = t / 3, tx = t - (t / 3) * 3;
        const int hr = BWD ? orow + 2 - ty : orow + ty, hc = BWD ? ocol + 2 - tx : ocol + tx;
        const char* arow = sH1 + (hr * R::HW + hc) * SH + 16 * lg;
        const char* wst = ring + (t % NSTB) * R::TAPB + lane * 16;
#pragma unroll
        for (int ks = 0; ks < KB; ++ks) {
            const u32x4 fa = *reinterpret_cast<const u32x4*>(arow + 64 * ks);
#pragma unroll
            for (int j = 0; j < NJA; ++j) {
                const u32x4 fb = *reinterpret_cast<const u32x4*>(wst + ((nh * NJA + j) * KB + ks) * FRAG);
                accb[j] = mma16<bf16>(fb, fa, accb[j]);
            }
        }
    }
    // epilogue B: lane = output pixel (orow, ocol) of the tile
    const int oy = y0 + orow, ox = x0 + ocol;
    const bool oin = oy < a.H && ox < a.W;
    const int64_t op = oin ? pix(oy, ox) : 0;
    f32x4 bB[NJA];
    bf16x4 mB[NJA];
#pragma unroll
    for (int j = 0; j < NJA; ++j) {   // loads first (see epilogue A)
        const int c0 = (nh * NJA + j) * 16 + 4 * lg;
        if (!BWD) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bB[j][r] = a.bb[c0 + r];
        } else {
            mB[j] = bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
            if (oin) mB[j] = *reinterpret_cast<const bf16x4*>(a.h1 + op * NH + c0);
        }
    }
#pragma unroll
    for (int j = 0; j < NJA; ++j) {
        const int c0 = (nh * NJA + j) * 16 + 4 * lg;
        bf16x4 hv;
        if (!BWD) {
#pragma unroll
            for (int r = 0; r < 4; ++r) hv[r] = (bf16)fmaxf(accb[j][r] + bB[j][r], 0.f);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) hv[r] = (bf16)((float)mB[j][r] > 0.f ? accb[j][r] : 0.f);
        }
        *reinterpret_cast<bf16x4*>(sH2 + (mb * 16 + l16) * SH + c0 * 2) = hv;
        if (oin) *reinterpret_cast<bf16x4*>((BWD ? a.ga : a.h2) + op * NH + c0) = hv;
    }
    wait_lgkmcnt0();
    __builtin_amdgcn_s_barrier();      // (the last tap's wait drained every DMA, phase C's weights included)

    // ---- phase C: [64 px x N/2] . [N/2 x N] + residual ----
    f32x4 accc[NJC];
#pragma unroll
    for (int j = 0; j < NJC; ++j) accc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* arow = sH2 + (mb * 16 + l16) * SH + 16 * lg;
#pragma unroll
    for (int ks = 0; ks < KC; ++ks) {
        const u32x4 fa = *reinterpret_cast<const u32x4*>(arow + 64 * ks);
#pragma unroll
        for (int j = 0; j < NJC; ++j) {
            const u32x4 fb = *reinterpret_cast<const u32x4*>(sWC + ((nh * NJC + j) * KC + ks) * FRAG + lane * 16);
            accc[j] = mma16<bf16>(fb, fa, accc[j]);
        }
    }
    if (!oin) return;
    // every load of the epilogue before its first store (see epilogue A)
    bf16x4 xrC[NJC], ymC[NJC], r2C[NJC], xmC[NJC];
    f32x4 bC[NJC];
    const bf16x4 z4 = bf16x4{(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
#pragma unroll
    for (int j = 0; j < NJC; ++j) {
        const int c0 = (nh * NJC + j) * 16 + 4 * lg;
        xrC[j] = *reinterpret_cast<const bf16x4*>(a.x + op * a.x_ld + c0);
        if (!BWD) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bC[j][r] = a.bc[c0 + r];
        } else {
            ymC[j] = !a.gy_masked ? *reinterpret_cast<const bf16x4*>(a.y + op * a.y_ld + c0) : z4;
            r2C[j] = a.res2 ? *reinterpret_cast<const bf16x4*>(a.res2 + op * a.res2_ld + c0) : z4;
            xmC[j] = a.xmask ? *reinterpret_cast<const bf16x4*>(a.xmask + op * a.xmask_ld + c0) : z4;
        }
    }
#pragma unroll
    for (int j = 0; j < NJC; ++j) {
        const int c0 = (nh * NJC + j) * 16 + 4 * lg;
        const bf16x4 xr = xrC[j];
        bf16x4 ov;
        if (!BWD) {
#pragma unroll
            for (int r = 0; r < 4; ++r) ov[r] = (bf16)fmaxf(accc[j][r] + bC[j][r] + (float)xr[r], 0.f);
        } else {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (float)xr[r];
            if (!a.gy_masked) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = (float)ymC[j][r] > 0.f ? v[r] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += accc[j][r];
            if (a.res2) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += (float)r2C[j][r];
            }
            if (a.xmask) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = (float)xmC[j][r] > 0.f ? v[r] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) ov[r] = (bf16)v[r];
        }
        *reinterpret_cast<bf16x4*>(a.out + op * a.out_ld + c0) = ov;
    }
}


// ---------------------------------------------------------------------------
// The unit's three weight (+ bias) gradients in ONE launch (cai_resunit_wgrad), from the tensors the backward
// kernel leaves behind:
//     dWa[o][c]         = sum_p ga[p][o] x[p][c]                 (N/2 x N,  bias: sum_p ga)
//     dWb[o][c][ty][tx] = sum_p gb[p][o] h1[p + (ty-1, tx-1)][c]  (N/2 x N/2 x 9, zero outside the image)
//     dWc[o][c]         = sum_p gc[p][o] h2[p][c]                 (N x N/2,  bias: sum_p gc)
// Unfused these are three latency-bound weight-gradient launches per unit (C4's 16 x 16 / 64 x 64 units: 16-25
// us each for 38 MFLOP - 2.7 GFLOP).  Here the pixels are split S ways and every split has 13 blocks of one
// (N/2 x N/2) output tile each: the 9 taps of dWb, the two column halves of dWa, the two row halves of dWc.
// The 13 blocks of a split are consecutive in their XCD's dispatch order (xcd remap), so the split's operand
// chunks are read from HBM about once and shared through that XCD's L2.  A block walks its split in 64-pixel
// steps: G and X tiles [64 px][N/2] bf16 by 16-byte buffer loads (pixels past the split or shifted outside the
// image read 0) into a double-buffered LDS stage (XOR-swizzled slots: conflict-free writes and
// ds_read_b64_tr_b16 reads, one barrier per step), the next step's loads in flight during the MFMAs.  Wave w
// takes the 32-pixel half w >> 1 of each step and the column half w & 1 of the tile (all N/2 rows); the two
// halves are summed in LDS and written as fp32 slabs [S][rows][taps x channels] -- the conv weight-gradient
// slab format -- so the final sums are ordinary WGRAD reduce jobs (deferred to the end of the backward with the
// others).  Bias gradients: the column sums of the G tiles, accumulated from the loaded registers by the
// blocks of tiles 0 (gb), 9 (ga), 11 and 12 (gc), summed in pixel order.  Deterministic throughout.
// ---------------------------------------------------------------------------
struct RwArgs {
    const bf16 *x, *h1, *h2, *ga, *gb, *gc;
    int x_ld, gc_ld;                 // h1 / h2 / ga / gb: ld N/2
    int B, H, W, P;                  // P = B * H * W pixels
    int S, chunk;                    // pixel splits, pixels per split (a multiple of 64)
    float inv_plane, inv_w;          // 1 / (H * W), 1 / W
    float *slab_a, *slab_b, *slab_c; // [S][N/2][N], [S][N/2][9 * N/2], [S][N][N/2]
    float *bias_a, *bias_b, *bias_c; // [S][N/2], [S][N/2], [S][N]
};

template <int NH>
struct RwCfg {
    static constexpr int SLOTS = NH / 8;               // 16-byte slots per pixel row
    static constexpr int RB = NH * 2;                  // LDS row bytes
    static constexpr int STEP = 64;                    // pixels per step
    static constexpr int TILEB = STEP * RB;            // one operand tile
    static constexpr int LPT = STEP * SLOTS / 256;     // 16-byte loads per thread and operand (3 / 2)
    static constexpr int TM = NH / 16, TN = NH / 32;   // wave tile: all NH rows x NH / 2 columns
    static constexpr int EP = NH + 4;                  // epilogue partial row pitch (floats)
    static constexpr int EPI = NH * EP * 4;
    static constexpr int RED = 256 * LPT * 8 * 4;      // per-thread bias partials
    static constexpr int BYTES = (4 * TILEB > EPI + RED) ? 4 * TILEB : EPI + RED;
    static_assert(STEP * SLOTS % 256 == 0, "whole loads per thread");
    static_assert(BYTES <= 64 * 1024, "two blocks per CU");
};

// slot swizzle of a [64][NH] bf16 tile read by ds_read_b64_tr_b16 (rows 8g + q of a half-wave, g in {0, 1})
template <int NH>
__device__ __forceinline__ int rw_swz(int row, int slot) {
    if constexpr (NH == 96)
        return row * 192 + ((slot ^ (((row >> 3) & 1) << 1)) << 4);
    else
        return row * 128 + ((slot ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2))) << 4);
}

__device__ __forceinline__ s16x4 rw_tr16(const char* base, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + byte_off));
}

// n / d for 0 <= n < 2^23 from a float reciprocal and one correction each way
__device__ __forceinline__ int rw_div(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    const int r = n - q * d;
    q += (r >= d ? 1 : 0) - (r < 0 ? 1 : 0);
    return q;
}

// bijective XCD remap: logical ids [x*q, (x+1)*q) run on XCD x (dispatch is round-robin over 8 XCDs)
__device__ __forceinline__ int rw_xcd_remap(int wgid, int nwg) {
    const int xcd = wgid & 7, idx = wgid >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// block wgid of a 13 x S grid of nwg blocks (wgid's XCD: wgid & 7, as the hardware dispatches a grid)
template <int NH>
__device__ __forceinline__ void resunit_wgrad_block(const RwArgs& a, int wgid, int nwg, char* smem) {
    using R = RwCfg<NH>;
    constexpr int NC = 2 * NH, SLOTS = R::SLOTS, LPT = R::LPT, TM = R::TM, TN = R::TN, EP = R::EP;
    constexpr unsigned OOB = 0x80000000u;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int L = rw_xcd_remap(wgid, nwg);
    const int s = L / 13, t = L - (L / 13) * 13;

    // this block's GEMM: G (output rows) and X (columns) operands, tap shift, slab placement, bias role
    const bf16* G;
    const bf16* X;
    int g_ld = NH, x_ld = NH, dy = 0, dx = 0;
    float* slab;
    float* bias = nullptr;
    int ng, ncols, row0 = 0, col0 = 0;
    if (t < 9) {
        G = a.gb; X = a.h1; dy = t / 3 - 1; dx = t % 3 - 1;
        slab = a.slab_b; ng = NH; ncols = 9 * NH; col0 = t * NH;
        if (t == 0) bias = a.bias_b + (int64_t)s * NH;
    } else if (t < 11) {
        G = a.ga; X = a.x + (t - 9) * NH; x_ld = a.x_ld;
        slab = a.slab_a; ng = NH; ncols = NC; col0 = (t - 9) * NH;
        if (t == 9) bias = a.bias_a + (int64_t)s * NH;
    } else {
        row0 = (t - 11) * NH;
        G = a.gc + row0; g_ld = a.gc_ld; X = a.h2;
        slab = a.slab_c; ng = NC; ncols = NH;
        bias = a.bias_c + (int64_t)s * NC + row0;
    }
    const __amdgpu_buffer_rsrc_t gr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(G), (short)0, (int)((int64_t)a.P * g_ld * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(X), (short)0, (int)((int64_t)a.P * x_ld * 2), 0x00020000);
    const int p0 = s * a.chunk, p1 = min(a.P, p0 + a.chunk);
    const int nsteps = (p1 - p0 + R::STEP - 1) / R::STEP;
    const int plane = a.H * a.W;
    const float gsf = bias ? 1.f : 0.f;

    // per-thread load slots (fixed across steps): chunk e = u * 256 + tid -> pixel row e / SLOTS, slot e % SLOTS
    int lrow[LPT], lslot[LPT];
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
        const int e = u * 256 + tid;
        lrow[u] = e / SLOTS;
        lslot[u] = e - (e / SLOTS) * SLOTS;
    }
    u32x4 rg[LPT], rx[LPT];
    auto load = [&](int st) {
#pragma unroll
        for (int u = 0; u < LPT; ++u) {
            const int m = p0 + st * R::STEP + lrow[u];
            const bool okm = (st < nsteps) & (m < p1);
            rg[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  gr, okm ? (unsigned)(m * g_ld + lslot[u] * 8) * 2u : OOB, 0, 0));
            const int b = rw_div(m, plane, a.inv_plane);
            const int r = m - b * plane;
            const int i = rw_div(r, a.W, a.inv_w);
            const int j = r - i * a.W;
            const bool okx = okm & ((unsigned)(i + dy) < (unsigned)a.H) & ((unsigned)(j + dx) < (unsigned)a.W);
            const int xm = m + dy * a.W + dx;
            rx[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xr, okx ? (unsigned)(xm * x_ld + lslot[u] * 8) * 2u : OOB, 0, 0));
        }
    };
    float bsum[LPT][8];
#pragma unroll
    for (int u = 0; u < LPT; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[u][e] = 0.f;
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int kh = wave >> 1, wn = wave & 1;
    const int g_ = lane >> 4, q_ = (lane >> 2) & 3, p4 = lane & 3;
    const int r0 = 32 * kh + 8 * g_ + q_;
    load(0);
    for (int st = 0; st < nsteps; ++st) {
        char* const Gs = smem + (st & 1) * 2 * R::TILEB;
        char* const Xs = Gs + R::TILEB;
#pragma unroll
        for (int u = 0; u < LPT; ++u) {
            *reinterpret_cast<u32x4*>(Gs + rw_swz<NH>(lrow[u], lslot[u])) = rg[u];
            *reinterpret_cast<u32x4*>(Xs + rw_swz<NH>(lrow[u], lslot[u])) = rx[u];
            const bf16x8 h = __builtin_bit_cast(bf16x8, rg[u]);   // branch-free: scaled by 0 off the bias blocks
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum[u][e] += gsf * (float)h[e];
        }
        __syncthreads();
        load(st + 1);    // past the last step: every load reads 0 (no memory touched)
        u32x4 fb[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int c = wn * (NH / 2) + tn * 16 + 4 * p4;
            const s16x4 b0 = rw_tr16(Xs, rw_swz<NH>(r0, c >> 3) + ((c & 7) << 1));
            const s16x4 b1 = rw_tr16(Xs, rw_swz<NH>(r0 + 4, c >> 3) + ((c & 7) << 1));
            const s16x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
            fb[tn] = __builtin_bit_cast(u32x4, bv);
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            const int c = tm * 16 + 4 * p4;
            const s16x4 a0 = rw_tr16(Gs, rw_swz<NH>(r0, c >> 3) + ((c & 7) << 1));
            const s16x4 a1 = rw_tr16(Gs, rw_swz<NH>(r0 + 4, c >> 3) + ((c & 7) << 1));
            const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
            const u32x4 fa = __builtin_bit_cast(u32x4, av);
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mma16<bf16>(fa, fb[tn], acc[tm][tn]);
        }
    }
    // the two pixel halves summed through LDS, then the slab rows; bias partials in pixel order
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    float* bred = reinterpret_cast<float*>(smem + R::EPI);
    if (kh == 1) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    red[(tm * 16 + 4 * g_ + r) * EP + wn * (NH / 2) + tn * 16 + (lane & 15)] = acc[tm][tn][r];
    }
    if (bias) {
#pragma unroll
        for (int u = 0; u < LPT; ++u)
#pragma unroll
            for (int e = 0; e < 8; ++e) bred[(tid * LPT + u) * 8 + e] = bsum[u][e];
    }
    __syncthreads();
    if (kh == 0) {
        float* out = slab + ((int64_t)s * ng + row0) * ncols + col0;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = tm * 16 + 4 * g_ + r, col = wn * (NH / 2) + tn * 16 + (lane & 15);
                    out[(int64_t)row * ncols + col] = acc[tm][tn][r] + red[row * EP + col];
                }
    }
    if (bias && tid < NH) {
        const int sl = tid >> 3, el = tid & 7;
        float v = 0.f;
        for (int px = 0; px < R::STEP; ++px) {
            const int e = px * SLOTS + sl;
            const int u = e >> 8, th = e & 255;
            v += bred[(th * LPT + u) * 8 + el];
        }
        bias[tid] = v;
    }
}

template <int NH>
__global__ __launch_bounds__(256, 2) void resunit_wgrad_kernel(const RwArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[RwCfg<NH>::BYTES];
    resunit_wgrad_block<NH>(a, (int)blockIdx.x, (int)gridDim.x, smem);
}

// Several units' weight gradients in one launch (cai_resunit_wgrad_batch): job j owns blocks [start[j], start[j + 1])
// of a 1-D grid, its 13 * S blocks first (starts are multiples of 8, so a block's XCD is its local id's, as in a
// launch of its own), then padding blocks that exit.  Each job writes only its own slabs.
constexpr int RW_BATCH_MAX = 24;
struct RwBatch {
    RwArgs job[RW_BATCH_MAX];
    int start[RW_BATCH_MAX + 1];
    int n;
};

template <int NH>
__global__ __launch_bounds__(256, 2) void resunit_wgrad_batch_kernel(const RwBatch b) {
    __shared__ __attribute__((aligned(16))) char smem[RwCfg<NH>::BYTES];
    const int L = (int)blockIdx.x;
    int j = 0;
    while (j + 1 < b.n && L >= b.start[j + 1]) ++j;
    const int l = L - b.start[j], nwg = 13 * b.job[j].S;
    if (l >= nwg) return;
    resunit_wgrad_block<NH>(b.job[j], l, nwg, smem);
}

}  // namespace
}  // namespace cai

using namespace cai;

extern "C" int cai_resunit(const cai_resunit_args* p, int32_t direction, void* stream) {
    CAI_CHECK_ARG(p && (direction == 0 || direction == 1), "resunit: bad arguments");
    const int n = p->n;
    CAI_CHECK_ARG(n == 128 || n == 192, "resunit: N = %d (128 or 192 supported)", n);
    CAI_CHECK_ARG(p->batch > 0 && p->h > 0 && p->w > 0, "resunit: bad sizes");
    CAI_CHECK_ARG(p->x && p->wa && p->wb && p->wc && p->h1 && p->h2 && p->out, "resunit: null pointer");
    CAI_CHECK_ARG(p->x_ld >= n && p->x_ld % 8 == 0 && ((uintptr_t)p->x & 15) == 0, "resunit: x needs ld %% 8 == 0");
    CAI_CHECK_ARG(p->out_ld >= n && p->out_ld % 4 == 0, "resunit: out_ld");
    CAI_CHECK_ARG(p->kpa >= n && p->kpb >= 9 * (n / 2) && p->kpc >= n / 2 && p->kpa % 8 == 0 &&
                      p->kpb % 8 == 0 && p->kpc % 8 == 0,
                  "resunit: packed weight rows");
    if (direction == 0) {
        CAI_CHECK_ARG(p->ba && p->bb && p->bc, "resunit: forward needs the biases");
    } else {
        CAI_CHECK_ARG(p->ga && p->gb && (p->gy_masked || (p->y && p->gc && p->y_ld >= n && p->y_ld % 8 == 0)),
                      "resunit: backward outputs / y");
        CAI_CHECK_ARG(!p->res2 || (p->res2_ld >= n && p->res2_ld % 4 == 0), "resunit: res2_ld");
        CAI_CHECK_ARG(!p->xmask || (p->xmask_ld >= n && p->xmask_ld % 4 == 0), "resunit: xmask_ld");
    }
    const int64_t npix = (int64_t)p->batch * p->h * p->w;
    CAI_CHECK_ARG(npix * std::max(p->x_ld, p->out_ld) * 2 < (1ll << 31), "resunit: tensor too large");
    RuArgs a{};
    a.x = static_cast<const bf16*>(p->x);
    a.y = static_cast<const bf16*>(p->y);
    a.wa = static_cast<const bf16*>(p->wa);
    a.wb = static_cast<const bf16*>(p->wb);
    a.wc = static_cast<const bf16*>(p->wc);
    a.ba = p->ba; a.bb = p->bb; a.bc = p->bc;
    a.h1 = static_cast<bf16*>(p->h1);
    a.h2 = static_cast<bf16*>(p->h2);
    a.out = static_cast<bf16*>(p->out);
    a.gc = static_cast<bf16*>(p->gc);
    a.gb = static_cast<bf16*>(p->gb);
    a.ga = static_cast<bf16*>(p->ga);
    a.res2 = static_cast<const bf16*>(p->res2);
    a.xmask = static_cast<const bf16*>(p->xmask);
    a.x_ld = p->x_ld; a.y_ld = p->y_ld; a.out_ld = p->out_ld; a.res2_ld = p->res2_ld; a.xmask_ld = p->xmask_ld;
    a.kpa = p->kpa; a.kpb = p->kpb; a.kpc = p->kpc;
    a.B = p->batch; a.H = p->h; a.W = p->w;
    a.tiles_x = (p->w + 7) / 8;
    a.tiles_y = (p->h + 7) / 8;
    a.gy_masked = p->gy_masked;
    const dim3 grid((unsigned)(p->batch * a.tiles_x * a.tiles_y));
    hipStream_t st = as_stream(stream);
    if (n == 192 && direction)
        hipLaunchKernelGGL((resunit_kernel<192, true>), grid, dim3(512), 0, st, a);
    else if (n == 192)
        hipLaunchKernelGGL((resunit_kernel<192, false>), grid, dim3(512), 0, st, a);
    else if (direction)
        hipLaunchKernelGGL((resunit_kernel<128, true>), grid, dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((resunit_kernel<128, false>), grid, dim3(512), 0, st, a);
    CAI_LAUNCH_CHECK("resunit");
    return CAI_OK;
}

namespace {

// pixel splits of cai_resunit_wgrad: about 400 blocks (13 per split) from 8192 pixels, 4-16 steps per block
// below; A/B knob CAI_RW_SPLITS (fixed count)
int rw_splits(int64_t P) {
    static const int knob = [] {
        const char* e = std::getenv("CAI_RW_SPLITS");
        return (e && *e) ? std::max(0, std::atoi(e)) : 0;
    }();
    int S = knob > 0 ? knob : (int)std::min<int64_t>(32, std::max<int64_t>(1, P / 256));
    const int64_t chunk = ((P + S - 1) / S + 63) / 64 * 64;
    return (int)((P + chunk - 1) / chunk);
}

struct RwWs {
    int S, chunk;
    size_t off_a, off_b, off_c, off_ba, off_bb, off_bc, total;
};
bool rw_ws(const cai_resunit_wgrad_args* p, RwWs& w) {
    if (!p || (p->n != 128 && p->n != 192) || p->batch <= 0 || p->h <= 0 || p->w <= 0) return false;
    const int64_t P = (int64_t)p->batch * p->h * p->w;
    const int64_t nh = p->n / 2, n = p->n;
    w.S = rw_splits(P);
    w.chunk = (int)(((P + w.S - 1) / w.S + 63) / 64 * 64);
    auto up = [](size_t v) { return (v + 255) / 256 * 256; };
    size_t o = 0;
    w.off_a = o; o += up((size_t)w.S * nh * n * 4);
    w.off_b = o; o += up((size_t)w.S * nh * 9 * nh * 4);
    w.off_c = o; o += up((size_t)w.S * n * nh * 4);
    w.off_ba = o; o += up((size_t)w.S * nh * 4);
    w.off_bb = o; o += up((size_t)w.S * nh * 4);
    w.off_bc = o; o += up((size_t)w.S * n * 4);
    w.total = o;
    return true;
}

}  // namespace

extern "C" size_t cai_resunit_wgrad_workspace_bytes(const cai_resunit_wgrad_args* p) {
    RwWs w;
    return rw_ws(p, w) ? w.total : 0;
}

// the checks, kernel arguments and the three WGRAD reduce jobs of one call
static int rw_prepare(const cai_resunit_wgrad_args* p, void* workspace, size_t ws_bytes, RwArgs& a,
                      cai_reduce_job (&J)[3]) {
    RwWs w;
    CAI_CHECK_ARG(rw_ws(p, w), "resunit_wgrad: N = %d (128 or 192) and positive sizes", p ? p->n : -1);
    const int n = p->n, nh = n / 2;
    CAI_CHECK_ARG(p->x && p->h1 && p->h2 && p->ga && p->gb && p->gc, "resunit_wgrad: null operand");
    CAI_CHECK_ARG(p->dwa && p->dwb && p->dwc && p->dba && p->dbb && p->dbc, "resunit_wgrad: null gradient");
    CAI_CHECK_ARG(p->x_ld >= n && p->x_ld % 8 == 0 && p->gc_ld >= n && p->gc_ld % 8 == 0,
                  "resunit_wgrad: x_ld / gc_ld must be >= N and multiples of 8");
    for (const void* q : {p->x, p->h1, p->h2, p->ga, p->gb, p->gc})
        CAI_CHECK_ARG(((uintptr_t)q & 15) == 0, "resunit_wgrad: operands must be 16-byte aligned");
    CAI_CHECK_ARG(workspace && ws_bytes >= w.total, "resunit_wgrad: workspace %zu < %zu", ws_bytes, w.total);
    const int64_t P = (int64_t)p->batch * p->h * p->w;
    CAI_CHECK_ARG(P * std::max(p->x_ld, p->gc_ld) * 2 < (1ll << 31) && P < (1 << 23), "resunit_wgrad: tensor too large");
    char* ws = static_cast<char*>(workspace);
    a = RwArgs{};
    a.x = static_cast<const bf16*>(p->x);
    a.h1 = static_cast<const bf16*>(p->h1);
    a.h2 = static_cast<const bf16*>(p->h2);
    a.ga = static_cast<const bf16*>(p->ga);
    a.gb = static_cast<const bf16*>(p->gb);
    a.gc = static_cast<const bf16*>(p->gc);
    a.x_ld = p->x_ld; a.gc_ld = p->gc_ld;
    a.B = p->batch; a.H = p->h; a.W = p->w; a.P = (int)P;
    a.S = w.S; a.chunk = w.chunk;
    a.inv_plane = 1.f / (float)(p->h * p->w);
    a.inv_w = 1.f / (float)p->w;
    a.slab_a = reinterpret_cast<float*>(ws + w.off_a);
    a.slab_b = reinterpret_cast<float*>(ws + w.off_b);
    a.slab_c = reinterpret_cast<float*>(ws + w.off_c);
    a.bias_a = reinterpret_cast<float*>(ws + w.off_ba);
    a.bias_b = reinterpret_cast<float*>(ws + w.off_bb);
    a.bias_c = reinterpret_cast<float*>(ws + w.off_bc);
    // the final sums: three WGRAD reduce jobs over the slabs (reduce_jobs.hip)
    for (auto& j : J) j = cai_reduce_job{};
    auto fill = [&](cai_reduce_job& j, float* slab, float* dw, float* bws, float* db, int ng, int cq, int k) {
        j.kind = CAI_JOB_WGRAD;
        j.nblocks = wgrad_job_blocks(ng, cq, k, (ng + 255) / 256);
        j.p[0] = slab; j.p[1] = dw; j.p[2] = bws; j.p[3] = db;
        j.i[0] = w.S; j.i[1] = ng; j.i[2] = k * k * cq; j.i[3] = cq; j.i[4] = cq; j.i[5] = k;
        j.i[6] = p->accumulate ? 1 : 0; j.i[7] = w.S; j.i[8] = ng;
    };
    fill(J[0], a.slab_a, p->dwa, a.bias_a, p->dba, nh, n, 1);
    fill(J[1], a.slab_b, p->dwb, a.bias_b, p->dbb, nh, nh, 3);
    fill(J[2], a.slab_c, p->dwc, a.bias_c, p->dbc, n, nh, 1);
    return CAI_OK;
}

extern "C" int cai_resunit_wgrad(const cai_resunit_wgrad_args* p, void* workspace, size_t ws_bytes, void* stream,
                                 cai_reduce_job* jobs) {
    RwArgs a;
    cai_reduce_job J[3];
    const int rc = rw_prepare(p, workspace, ws_bytes, a, J);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)(13 * a.S));
    if (p->n == 192)
        hipLaunchKernelGGL(resunit_wgrad_kernel<96>, grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(resunit_wgrad_kernel<64>, grid, dim3(256), 0, st, a);
    CAI_LAUNCH_CHECK("resunit_wgrad");
    if (jobs) {
        for (int i = 0; i < 3; ++i) jobs[i] = J[i];
        return CAI_OK;
    }
    return launch_reduce_jobs(J, 3, st);
}

extern "C" int cai_resunit_wgrad_batch(const cai_resunit_wgrad_args* args, void* const* workspaces,
                                       const size_t* ws_bytes, int32_t n, void* stream, cai_reduce_job* jobs) {
    CAI_CHECK_ARG(n >= 0 && (n == 0 || (args && workspaces && ws_bytes && jobs)), "resunit_wgrad_batch: bad arguments");
    hipStream_t st = as_stream(stream);
    RwBatch b[2];     // N = 192 (NH 96), N = 128 (NH 64)
    b[0].n = b[1].n = 0;
    b[0].start[0] = b[1].start[0] = 0;
    auto flush = [&](int c) {
        if (!b[c].n) return;
        const dim3 grid((unsigned)b[c].start[b[c].n]);
        if (c == 0)
            hipLaunchKernelGGL(resunit_wgrad_batch_kernel<96>, grid, dim3(256), 0, st, b[c]);
        else
            hipLaunchKernelGGL(resunit_wgrad_batch_kernel<64>, grid, dim3(256), 0, st, b[c]);
        b[c].n = 0;
    };
    for (int i = 0; i < n; ++i) {
        RwArgs a;
        cai_reduce_job J[3];
        const int rc = rw_prepare(&args[i], workspaces[i], ws_bytes[i], a, J);
        if (rc) return rc;
        for (int k = 0; k < 3; ++k) jobs[3 * i + k] = J[k];
        const int c = args[i].n == 192 ? 0 : 1;
        if (b[c].n == RW_BATCH_MAX) flush(c);
        RwBatch& B = b[c];
        B.job[B.n] = a;
        B.start[B.n + 1] = B.start[B.n] + (13 * a.S + 7) / 8 * 8;
        ++B.n;
    }
    flush(0);
    flush(1);
    CAI_LAUNCH_CHECK("resunit_wgrad_batch");
    return CAI_OK;
}

