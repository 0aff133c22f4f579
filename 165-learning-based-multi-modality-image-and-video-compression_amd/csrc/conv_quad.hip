// Four-phase halo kernel: the 128-channel k5 s2 p2 layers in their s^2-phase direction, bf16 --
// ConvTranspose2d k5 s2 p2 op1 forward (deconv(), /root/reference/CompressAI/compressai/models/utils.py:138-146,
// g_s at google.py:244-252) and the input gradient of Conv2d k5 s2 p2 (conv(), utils.py:128-136, g_a).
//
// The s^2-phase decomposition turns such a layer into four stride-1 convolutions of the same input: output
// phase (py, px) has (3 - py) x (3 - px) taps, and tap (ty, tx) of it reads input (qy + 1 - ty, qx + 1 - tx)
// for phase-grid pixel (qy, qx).  Every phase of an 8 x 32 phase-grid tile therefore reads inside ONE
// (8 + 2) x (32 + 2) input footprint.  conv_halo_phase_kernel gives each phase its own block, so each CU
// stages that footprint four times and pays four prologues and four exposed epilogues (round-4 counters:
// 2.96x the algorithmic input fetched, waves parked 46 % of their cycles).  Here one 512-thread block owns
// the tile for all four phases:
//  * the footprint of all 128 input channels is staged in LDS once (two 64-channel chunks, eight planes of
//    8 channels each, 16-byte cells, rows contiguous so an A fragment reads 16 consecutive cells); chunk 0
//    before the first step, chunk 1 through registers under phase 0's first steps;
//  * the 100 steps of the tile (phase, chunk, 32-channel half, tap: 36 + 24 + 24 + 16) run back to back as
//    one unrolled pipeline: one weight stage (128 output channels x 32 input channels) per step through an
//    NSTB-deep LDS-DMA ring, the next step's fragments read while the current step's 16 MFMAs per wave issue,
//    one barrier per step;
//  * a phase's epilogue (bias + activation, bf16) stores straight from the accumulators, the four channel
//    groups of a 16-channel column pair exchanged by v_permlane16_swap so every lane writes 16 contiguous
//    bytes (8 stores per wave instead of 16); the stores stay in flight under the next phase's steps (every
//    wait below is counted, no vmcnt(0) between phases).
// The accumulation order of every output (chunk, half, tap) is conv_halo_phase_kernel's, so the results are
// bit-identical to it (tests/test_kernels_gpu.py).
#include "common.hpp"
#include "conv_args.hpp"
#include "mfma.hpp"

#include <type_traits>

namespace cai {

namespace {

__device__ __attribute__((aligned(64))) unsigned quad_zero_page[64];

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int Q_TH = 8, Q_TW = 32, Q_WM = 4, Q_WN = 2, Q_NT = 512;
constexpr int Q_TM = Q_TH * Q_TW / Q_WM / 16, Q_TN = 128 / Q_WN / 16;   // 4 x 4 fragments per wave
constexpr int Q_PW = Q_TW + 2, Q_NPOS = (Q_TH + 2) * Q_PW;                 // 10 x 34 footprint
constexpr int Q_PLANE = (Q_NPOS + 15) / 16 * 16;                          // = 0 (mod 16): conflict-free reads
constexpr int Q_PATCH = 8 * Q_PLANE * 16;                                 // one 64-channel chunk
constexpr int Q_NPI = (8 * Q_NPOS + Q_NT - 1) / Q_NT;                     // footprint cells per thread and chunk
// ring depth: 3 .. 8 stages and one barrier per two steps measured equal (profiles/r05_quad_variants.log)
#ifndef CAI_QUAD_NSTB
#define CAI_QUAD_NSTB 4
#endif
constexpr int Q_NSTB = CAI_QUAD_NSTB;                                     // weight ring depth
constexpr int Q_BSTAGE = Q_NT * 16;                                       // 128 rows x 64 bytes
constexpr int Q_RING = 2 * Q_PATCH, Q_BIASO = Q_RING + Q_NSTB * Q_BSTAGE;
constexpr int Q_BYTES = Q_BIASO + 128 * 4;
constexpr int Q_TOTAL = 100;                                              // steps per tile
constexpr int Q_STORE1 = 16;                                              // chunk 1's footprint -> LDS
constexpr int Q_NSTORE = Q_TM * Q_TN / 2;                                 // 16-byte stores per wave and phase
// a phase's 8 output stores per wave go out at the end of its last step, all at once (spreading them over the next
// phase's steps, one every 1 or 2 steps, measured equal: profiles/r05_quad_variants.log)
static_assert(Q_BYTES <= 160 * 1024 && Q_NPI + Q_NSTB <= Q_STORE1 && Q_STORE1 < 17, "quad tile");

__host__ __device__ constexpr int q_start(int p) { return p <= 0 ? 0 : p == 1 ? 36 : p == 2 ? 60 : p == 3 ? 84 : 100; }
__host__ __device__ constexpr int q_phase(int s) { return s < 36 ? 0 : s < 60 ? 1 : s < 84 ? 2 : 3; }
__host__ __device__ constexpr int q_ntap(int p) { return p == 0 ? 9 : p == 3 ? 4 : 6; }
__host__ __device__ constexpr int q_ncol(int p) { return (p & 1) ? 2 : 3; }
__host__ __device__ constexpr bool q_last(int s) { return s == 35 || s == 59 || s == 83 || s == 99; }
// step s = (phase, chunk, half, tap): byte offset of its weights inside the phase's packed row ([tap][c], 128
// input channels), and of its A operand inside the footprint (chunk patch, half's planes, tap cell)
__host__ __device__ constexpr int q_koff(int s) {
    const int p = q_phase(s), l = s - q_start(p), nst = 2 * q_ntap(p);
    const int c = l / nst, t = l % nst, hf = t / q_ntap(p), tap = t % q_ntap(p);
    return (tap * 128 + c * 64 + hf * 32) * 2;
}
__host__ __device__ constexpr int q_toff(int s) {
    const int p = q_phase(s), l = s - q_start(p), nst = 2 * q_ntap(p);
    const int c = l / nst, t = l % nst, hf = t / q_ntap(p), tap = t % q_ntap(p);
    const int ty = tap / q_ncol(p), tx = tap % q_ncol(p);
    return c * Q_PATCH + (hf * 4 * Q_PLANE + (2 - ty) * Q_PW + (2 - tx)) * 16;
}
// vector-memory operations a wave issues inside step j after that step's weight DMA: the next chunk's
// footprint cell (steps < NPI), the four fence loads behind the last one, and a finished phase's output
// stores (issued at the end of the phase's last step)
__host__ __device__ constexpr int q_after_dma(int j) {
    return (j < Q_NPI ? 1 : 0) + (j == Q_NPI - 1 ? 4 : 0) + (q_last(j) ? Q_NSTORE : 0);
}
__host__ __device__ constexpr int q_ops(int j) { return (j + Q_NSTB < Q_TOTAL ? 1 : 0) + q_after_dma(j); }
// operations issued after step s + 1's weight DMA when step s starts (the prologue drained everything)
__host__ __device__ constexpr int q_younger(int s) {
    const int i = s + 1 - Q_NSTB;   // the step that issued step s + 1's DMA
    int n = 0;
    if (i >= 0) n += q_after_dma(i);
    for (int j = (i >= 0 ? i + 1 : 0); j < s; ++j) n += q_ops(j);
    return n;
}

template <int I, int N, class F>
__device__ __forceinline__ void q_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        q_for<I + 1, N>(f);
    }
}

}  // namespace

// ACT: the output takes an activation (ReLU / LeakyReLU); false: bias only
template <bool ACT>
__global__ __launch_bounds__(512, 1) void conv_halo_quad_kernel(const ConvArgs a, int tiles_x, int tiles_y) {
    __shared__ __attribute__((aligned(16))) char smem[Q_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / Q_WN, wn = wid % Q_WN;
    const int g_ = lane >> 4, i16 = lane & 15;
    // consecutive tiles of an image on one XCD: their footprints overlap in its L2
    const int nt = gridDim.x, t = blockIdx.x;
    const int bid = (nt & 7) == 0 ? (t & 7) * (nt >> 3) + (t >> 3) : t;
    const int per_img = tiles_x * tiles_y;
    const int b = bid / per_img;
    const int rt = bid - b * per_img;
    const int ty0 = (rt / tiles_x) * Q_TH, tx0 = (rt % tiles_x) * Q_TW;
    const char* X = reinterpret_cast<const char*>(a.x);
    const int ld_b = a.x_ld * 2;

    // footprint cells: thread tid's i-th cell of a chunk is (plane g, position q), 8 lanes per plane-row so a
    // wave reads 8 pixels x 128 contiguous bytes.  Footprint origin: input (ty0 - 1, tx0 - 1).
    const int iyb = ty0 - 1, ixb = tx0 - 1;
    u32x4 pr_[Q_NPI];
    unsigned fence_[4] = {0u, 0u, 0u, 0u};
    auto load_cell = [&](int c, int i) {
        const int q8 = tid + Q_NT * i, g = (q8 >> 3) & 7, q = ((q8 >> 6) << 3) | (q8 & 7);
        const int pr = q / Q_PW, pc = q - (q / Q_PW) * Q_PW;
        const int iy = iyb + pr, ix = ixb + pc;
        const bool in = q < Q_NPOS && (unsigned)iy < (unsigned)a.IH && (unsigned)ix < (unsigned)a.IW;
        const void* src = in ? (const void*)(X + ((b * a.IH + iy) * a.IW + ix) * ld_b + g * 16 + c * 128)
                             : (const void*)quad_zero_page;
        pr_[i] = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(reinterpret_cast<uintptr_t>(src));
    };
    auto store_patch = [&](int c) {
#pragma unroll
        for (int i = 0; i < Q_NPI; ++i) {
            const int q8 = tid + Q_NT * i, g = (q8 >> 3) & 7, q = ((q8 >> 6) << 3) | (q8 & 7);
            if (q < Q_NPOS) *reinterpret_cast<u32x4*>(smem + c * Q_PATCH + (g * Q_PLANE + q) * 16) = pr_[i];
        }
    };
    // compiler-visible loads behind the last cell: the compiler's wait for the cells then leaves the (invisible)
    // weight DMAs issued after them in flight
    auto fence_loads = [&]() {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            asm volatile("" ::"v"(fence_[j]));
            fence_[j] = *reinterpret_cast<const __attribute__((address_space(1))) unsigned*>(
                reinterpret_cast<uintptr_t>(quad_zero_page + 16 * j));
        }
    };

    // weight ring: lane bp stages 16-byte slot bs_ of output channel bn_ (cell 4 n + (s ^ 3 ((n / 8) & 1))), one
    // DMA per lane and step; step s lands in stage s % NSTB
    const int bp = wid * 64 + lane;
    const int bn_ = bp >> 2, bs_ = (bp & 3) ^ (((bn_ >> 3) & 1) * 3);
    const char* Wlane = bn_ < a.Npad ? reinterpret_cast<const char*>(a.w) + (int64_t)bn_ * a.Kp * 2 + bs_ * 16 : nullptr;
    auto issue_b = [&](auto sc) {
        constexpr int s = decltype(sc)::value;
        const void* src = Wlane ? (const void*)(Wlane + a.ph[q_phase(s)].w_off * 2 + q_koff(s))
                                : (const void*)quad_zero_page;
        glds16_asm(src, smem + Q_RING + (s % Q_NSTB) * Q_BSTAGE + wid * 1024);
    };

    int apos[Q_TM];
#pragma unroll
    for (int tm = 0; tm < Q_TM; ++tm) {
        const int r = wm * (Q_TM * 16) + tm * 16 + i16;
        apos[tm] = (g_ * Q_PLANE + (r / Q_TW) * Q_PW + (r % Q_TW)) * 16;
    }
    int bpos[Q_TN];
#pragma unroll
    for (int tn = 0; tn < Q_TN; ++tn) {
        const int n = wn * (Q_TN * 16) + tn * 16 + i16;
        bpos[tn] = Q_RING + (4 * n + (g_ ^ (((n >> 3) & 1) * 3))) * 16;
    }
    auto read_frags = [&](auto sc, u32x4 (&fa)[Q_TM], u32x4 (&fb)[Q_TN]) {
        constexpr int s = decltype(sc)::value;
#pragma unroll
        for (int tm = 0; tm < Q_TM; ++tm) fa[tm] = *reinterpret_cast<const u32x4*>(smem + apos[tm] + q_toff(s));
#pragma unroll
        for (int tn = 0; tn < Q_TN; ++tn)
            fb[tn] = *reinterpret_cast<const u32x4*>(smem + bpos[tn] + (s % Q_NSTB) * Q_BSTAGE);
    };

    f32x4 acc[Q_TM][Q_TN];
#pragma unroll
    for (int i = 0; i < Q_TM; ++i)
#pragma unroll
        for (int j = 0; j < Q_TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // phase p's epilogue: bias + activation, bf16, 16-byte stores (lane group g of column pair (2pp, 2pp+1)
    // writes channels (2pp + (g & 1)) * 16 + (g >> 1) * 8 .. + 7 after the swap)
    const float neg = a.act == CAI_ACT_RELU ? 0.f : (a.act == CAI_ACT_LEAKY ? a.act_param : 1.f);
    const unsigned keep = a.act == CAI_ACT_RELU ? 0u : ~0u;
    // phase p's results: bias + activation, bf16, the column pairs (2pp, 2pp+1) exchanged so lane group g holds
    // channels (2pp + (g & 1)) * 16 + (g >> 1) * 8 .. + 7 of its pixel; accumulators cleared for the next phase
    u32x2 pend[Q_TM][Q_TN];
    auto finish = [&]() {
        f32x4 bv[Q_TN];
#pragma unroll
        for (int tn = 0; tn < Q_TN; ++tn)
            bv[tn] = *reinterpret_cast<const f32x4*>(smem + Q_BIASO + (wn * 64 + tn * 16 + 4 * g_) * 4);
#pragma unroll
        for (int tm = 0; tm < Q_TM; ++tm) {
#pragma unroll
            for (int tn = 0; tn < Q_TN; ++tn) {
                bf16x4 h;
                if constexpr (!ACT) {    // no activation: the add and the conversion only
#pragma unroll
                    for (int r = 0; r < 4; ++r) h[r] = (bf16)(acc[tm][tn][r] + bv[tn][r]);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        // v > 0 ? v : (ReLU ? +0 : v * neg), branch-free (keep: 0 for ReLU, all ones otherwise)
                        const float v = acc[tm][tn][r] + bv[tn][r];
                        const float m = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, v * neg) & keep);
                        h[r] = (bf16)(v > 0.f ? v : m);
                    }
                }
                pend[tm][tn] = __builtin_bit_cast(u32x2, h);
                acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int pp = 0; pp < Q_TN / 2; ++pp)
#pragma unroll
                for (int d = 0; d < 2; ++d) {
                    const auto sw = __builtin_amdgcn_permlane16_swap(pend[tm][2 * pp][d], pend[tm][2 * pp + 1][d],
                                                                      false, false);
                    pend[tm][2 * pp][d] = sw[0];
                    pend[tm][2 * pp + 1][d] = sw[1];
                }
        }
    };
    // store k = (row fragment tm = k / 2, column pair pp = k % 2) of phase p's results
    auto store_k = [&](auto pc, int k) {
        constexpr int p = decltype(pc)::value;
        const PhaseDesc& P = a.ph[p];
        const int tm = k >> 1, pp = k & 1;
        const int r = wm * (Q_TM * 16) + tm * 16 + i16;
        const int qy = ty0 + r / Q_TW, qx = tx0 + r % Q_TW;
        const int n = wn * 64 + (2 * pp + (g_ & 1)) * 16 + (g_ >> 1) * 8;
        const bool ok = qy < P.OHg && qx < P.OWg && n < a.Cout;
        bf16* Y = reinterpret_cast<bf16*>(a.y) + (int64_t)b * a.ysb + (int64_t)(P.oy0 + 2 * qy) * a.ysy +
                  (int64_t)(P.ox0 + 2 * qx) * a.ysx + n;
        if (ok)
            *reinterpret_cast<u32x4*>(Y) = u32x4{pend[tm][2 * pp][0], pend[tm][2 * pp][1], pend[tm][2 * pp + 1][0],
                                                 pend[tm][2 * pp + 1][1]};
    };

    // prologue: the first weight stages (lockstep NSTB, pairs NSTB - 1), the bias, chunk 0's footprint; everything
    // drained once
    q_for<0, Q_NSTB>([&](auto sc) { issue_b(sc); });
    const int nb = tid & 127;
    const float* bsrc = (a.bias && nb < a.Cout) ? a.bias + nb : reinterpret_cast<const float*>(quad_zero_page);
    const float bval = *reinterpret_cast<const __attribute__((address_space(1))) float*>(reinterpret_cast<uintptr_t>(bsrc));
#pragma unroll
    for (int i = 0; i < Q_NPI; ++i) load_cell(0, i);
    wait_vmcnt<0>();
    if (tid < 128) *reinterpret_cast<float*>(smem + Q_BIASO + tid * 4) = bval;
    store_patch(0);
    wait_lgkmcnt0();
    __builtin_amdgcn_s_barrier();
    u32x4 fa[Q_TM], fb[Q_TN];
    read_frags(std::integral_constant<int, 0>{}, fa, fb);

    q_for<0, Q_TOTAL>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        constexpr int yg = q_younger(s);
        static_assert(yg >= 0 && yg < 64, "vmcnt range");
        wait_vmcnt<yg>();    // step s + 1's weights have landed (this wave's share)
        wait_lgkmcnt0();
        __builtin_amdgcn_s_barrier();   // ... every wave's share; stage s % NSTB is free
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (s + Q_NSTB < Q_TOTAL) issue_b(std::integral_constant<int, s + Q_NSTB>{});
        if constexpr (s < Q_NPI) load_cell(1, s);
        if constexpr (s == Q_NPI - 1) fence_loads();
        // read from step 18 on (its fragments are read in step 17, after the next barrier)
        if constexpr (s == Q_STORE1) store_patch(1);
        u32x4 na[Q_TM], nb2[Q_TN];
        if constexpr (s + 1 < Q_TOTAL) read_frags(std::integral_constant<int, s + 1>{}, na, nb2);
#pragma unroll
        for (int tm = 0; tm < Q_TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < Q_TN; ++tn) acc[tm][tn] = mma16<bf16>(fb[tn], fa[tm], acc[tm][tn]);
        if constexpr (s + 1 < Q_TOTAL) {
            // the next step's reads (separate registers) alternate with this step's first MFMAs
#pragma unroll
            for (int i = 0; i < Q_TM + Q_TN; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, Q_TM * Q_TN - (Q_TM + Q_TN), 0);
#pragma unroll
            for (int tm = 0; tm < Q_TM; ++tm) fa[tm] = na[tm];
#pragma unroll
            for (int tn = 0; tn < Q_TN; ++tn) fb[tn] = nb2[tn];
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (q_last(s)) {
            finish();
#pragma unroll
            for (int k = 0; k < Q_NSTORE; ++k) store_k(std::integral_constant<int, q_phase(s)>{}, k);
        }
    });
    asm volatile("" ::"v"(fence_[0]), "v"(fence_[1]), "v"(fence_[2]), "v"(fence_[3]));
}

bool conv_quad_ok(const ConvArgs& a) {
    static const bool off = [] {
        const char* e = getenv("CAI_QUAD_OFF");
        return e && *e && *e != '0';
    }();
    if (off || a.nphase != 4 || a.Cin_pad != 128 || a.Cout > 128 || a.Npad > 128 || a.ksplit != 1 ||
        a.out_step != 2 || a.in_abs || !a.y_vec || a.y_dtype != CAI_BF16 || a.mask_mode || a.res || a.res2 ||
        (a.Cout & 7) != 0 || (a.x_ld & 7) != 0 || (reinterpret_cast<uintptr_t>(a.x) & 15) != 0)
        return false;
    static const int nt[4] = {9, 6, 6, 4}, nx[4] = {3, 2, 3, 2};
    for (int p = 0; p < 4; ++p) {
        const PhaseDesc& P = a.ph[p];
        if (P.ntaps != nt[p] || P.ntx != nx[p] || P.dy0 != 1 || P.dx0 != 1 || P.oy0 != (p >> 1) || P.ox0 != (p & 1))
            return false;
    }
    return true;
}

void launch_conv_halo_quad(const ConvArgs& a, int tiles_x, int tiles_y, int mtiles, hipStream_t st) {
    if (a.act == CAI_ACT_RELU || a.act == CAI_ACT_LEAKY)
        hipLaunchKernelGGL(conv_halo_quad_kernel<true>, dim3(mtiles), dim3(512), 0, st, a, tiles_x, tiles_y);
    else
        hipLaunchKernelGGL(conv_halo_quad_kernel<false>, dim3(mtiles), dim3(512), 0, st, a, tiles_x, tiles_y);
}

}  // namespace cai
