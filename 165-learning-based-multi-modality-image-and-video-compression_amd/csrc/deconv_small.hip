// ConvTranspose2d with few output channels (the synthesis transform's last
// layer, deconv(N, 3), models/utils.py:138-146 / google.py:244-252).
//
// Output-stationary implicit GEMM is a poor fit here (N = 3 of a 16-wide MFMA
// tile, and every output pixel re-gathers its input taps).  Instead:
//   forward : P = x W'    one dense GEMM per input pixel with N = k*k*Cout
//                         (75 -> 80) columns, W'[(kh,kw,c)][ci]
//             out = bias + col2im(P)   each output pixel sums its <= ceil(k/s)^2
//                         contributions; written as fp32 NCHW (x_hat)
//   backward: Q = im2col(dOut)         [input pixel][(kh,kw,c)]
//             dx  = Q W'^T              (K = 80)
//             dW' = Q^T x               (pixel-reduction wgrad of conv.hip),
//                                       scattered back to [ci][c][kh][kw]
//             db  = per-channel sums of dOut
// The two per-pixel GEMMs have short K (<= 256) and N (<= 256): rows_gemm
// keeps the whole weight matrix in LDS and streams activation rows straight
// from HBM into MFMA B-fragments (no LDS round trip), one register prefetch
// deep.  col2im / im2col stage their input window in LDS so the HBM side is
// read once, coalesced.
#include "common.hpp"
#include "mfma.hpp"

#include <algorithm>

namespace cai {

static int rup(int v, int m) { return (v + m - 1) / m * m; }
static int ntile_inst(int nt) { return nt <= 8 ? nt : (nt <= 12 ? 12 : 16); }

constexpr int C2I_TH = 8, C2I_TW = 32;     // col2im output tile
constexpr int I2C_TH = 4, I2C_TW = 32;     // im2col input-pixel tile

struct SmallPlan {
    int B, Cin, Cout, H, W, OH, OW, k, s, p, kk, Np;
    int ks;                   // k-span of one 16-byte MFMA operand slot
    int NTf, Kpf, NTb, Kpb;   // forward (W') / backward (W'^T) GEMM weight tiles
    int c2i_r, c2i_c, i2c_r, i2c_c;
    cai_conv_geom g_w;        // 1x1 Conv2d Cin -> Np: the dW' wgrad
    size_t off_wf, off_wb, off_pq, off_wg, off_dwt, off_col, total;
};

static SmallPlan small_plan(const cai_conv_geom* g, int dtype) {
    SmallPlan L{};
    L.B = g->batch; L.Cin = g->in_c; L.Cout = g->out_c; L.H = g->in_h; L.W = g->in_w;
    L.OH = g->out_h; L.OW = g->out_w; L.k = g->kernel; L.s = g->stride; L.p = g->pad;
    L.kk = L.k * L.k;
    L.Np = rup(L.kk * L.Cout, 16);
    const int es = dtype_size(dtype);
    L.ks = 4 * (16 / es);
    L.NTf = ntile_inst(L.Np / 16);
    L.Kpf = rup(L.Cin, L.ks);
    L.NTb = ntile_inst((L.Cin + 15) / 16);
    L.Kpb = rup(L.Np, L.ks);
    L.c2i_r = (C2I_TH - 1 + L.k - 1) / L.s + 2;
    L.c2i_c = (C2I_TW - 1 + L.k - 1) / L.s + 2;
    L.i2c_r = (I2C_TH - 1) * L.s + L.k;
    L.i2c_c = (I2C_TW - 1) * L.s + L.k;
    L.g_w = cai_conv_geom{L.B, L.Cin, L.H, L.W, L.Np, L.H, L.W, 1, 1, 0, 0, 0};
    const int64_t npix = (int64_t)L.B * L.H * L.W;
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o += (n + 255) / 256 * 256; return r; };
    L.off_wf = take((size_t)L.NTf * 16 * L.Kpf * es);
    L.off_wb = take((size_t)L.NTb * 16 * L.Kpb * es);
    L.off_pq = take((size_t)npix * L.Np * es);     // P (forward) / Q (backward)
    L.off_wg = take(cai_conv_wgrad_workspace_bytes(&L.g_w, dtype));
    L.off_dwt = take((size_t)L.Np * L.Cin * 4);
    L.off_col = take((size_t)1024 * L.Cout * 4);
    L.total = o;
    return L;
}

static size_t rows_gemm_lds(int nti, int kp, int es) { return (size_t)nti * 16 * (kp * es + 16); }
static size_t col2im_lds(const SmallPlan& L, int es) { return (size_t)L.c2i_r * L.c2i_c * L.Np * es; }
static size_t im2col_lds(const SmallPlan& L) { return (size_t)L.Cout * L.i2c_r * L.i2c_c * 4 + (size_t)L.Np * 4; }

__device__ __forceinline__ int floordiv(int a, int s) { return a >= 0 ? a / s : -((-a + s - 1) / s); }

// Wf[n][ci] = Wb[ci][n] = W[ci][c][kh][kw], n = (kh*k + kw)*Cout + c, zero padded
template <typename T>
__global__ void small_prep_kernel(const float* __restrict__ w, int Cin, int Cout, int kk, T* __restrict__ wf,
                                  int rows_f, int kpf, T* __restrict__ wb, int rows_b, int kpb) {
    const int nf = wf ? rows_f * kpf : 0, nb = wb ? rows_b * kpb : 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nf + nb; i += gridDim.x * blockDim.x) {
        int n, ci;
        if (i < nf) { n = i / kpf; ci = i - n * kpf; }
        else { ci = (i - nf) / kpb; n = (i - nf) - ci * kpb; }
        float v = 0.f;
        if (n < kk * Cout && ci < Cin) {
            const int t = n / Cout, c = n - (n / Cout) * Cout;
            v = w[((int64_t)ci * Cout + c) * kk + t];
        }
        if (i < nf) wf[i] = from_f32<T>(v);
        else wb[i - nf] = from_f32<T>(v);
    }
}

// C[m][n] = sum_k A[m][k] * Bw[n][k]   (m < M pixels, n < N <= NTI*16, k < K <= Kp)
// Bw [NTI*16][Kp] is staged in LDS; each wave owns PT*16 consecutive rows of A
// and computes C^T tiles (MFMA A-operand = weights, B-operand = pixels), so a
// lane's accumulator holds 4 consecutive n of one pixel.
template <typename T, int NTI, int PT>
__global__ __launch_bounds__(256) void rows_gemm_kernel(const T* __restrict__ A, int lda, int M, int K,
                                                        const T* __restrict__ Bw, int Kp, T* __restrict__ C, int ldc,
                                                        int N) {
    constexpr int VEC = OpT<T>::VEC;
    constexpr int KS = 4 * VEC;
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const int rs = Kp * (int)sizeof(T) + 16;
    const int tid = threadIdx.x;
    const int cpr = Kp * (int)sizeof(T) / 16;
    for (int i = tid; i < NTI * 16 * cpr; i += 256) {
        const int r = i / cpr, c = i - (i / cpr) * cpr;
        *reinterpret_cast<u32x4*>(sm + r * rs + c * 16) =
            *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(Bw) + (int64_t)r * Kp * sizeof(T) + c * 16);
    }
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6;
    const int pl = lane & 15, kq = lane >> 4;
    const gptr<T> Ag = to_global<T>(A);
    const u32x4 zero = u32x4{0u, 0u, 0u, 0u};
    const int ntiles = (M + 64 * PT - 1) / (64 * PT);
    // grid-stride over 64*PT-row tiles: the LDS weight copy is amortised
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int m0 = (tile * 4 + wave) * (PT * 16);
    if (m0 >= M) continue;
    f32x4 acc[NTI][PT];
#pragma unroll
    for (int i = 0; i < NTI; ++i)
#pragma unroll
        for (int j = 0; j < PT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 cur[PT], nxt[PT];
#define RG_LOAD(KSTEP, DST)                                                                              \
    _Pragma("unroll") for (int pt = 0; pt < PT; ++pt) {                                                  \
        const int m = m0 + pt * 16 + pl, kx = (KSTEP) * KS + kq * VEC;                                   \
        const bool ok = m < M && kx < K;                                                                 \
        const u32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(              \
            Ag + (ok ? (int64_t)m * lda + kx : 0));                                                      \
        DST[pt] = ok ? v : zero;                                                                         \
    }
    const int nsteps = Kp / KS;
    RG_LOAD(0, cur);
    for (int st = 0; st < nsteps; ++st) {
        if (st + 1 < nsteps) { RG_LOAD(st + 1, nxt); }
        const char* wrow = sm + pl * rs + (st * KS + kq * VEC) * (int)sizeof(T);
#pragma unroll
        for (int nt = 0; nt < NTI; ++nt) {
            const u32x4 wv = *reinterpret_cast<const u32x4*>(wrow + nt * 16 * rs);
#pragma unroll
            for (int pt = 0; pt < PT; ++pt) acc[nt][pt] = mma16<T>(wv, cur[pt], acc[nt][pt]);
        }
#pragma unroll
        for (int pt = 0; pt < PT; ++pt) cur[pt] = nxt[pt];
    }
#undef RG_LOAD
#pragma unroll
    for (int pt = 0; pt < PT; ++pt) {
        const int m = m0 + pt * 16 + pl;
        if (m >= M) continue;
        T* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int nt = 0; nt < NTI; ++nt) {
            const int n = nt * 16 + kq * 4;
            if (n >= N) continue;
            const f32x4 v = acc[nt][pt];
            if constexpr (sizeof(T) == 2) {
                bf16x4 h = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
                *reinterpret_cast<bf16x4*>(crow + n) = h;
            } else {
                *reinterpret_cast<f32x4*>(crow + n) = v;
            }
        }
    }
    }
}

template <typename T, int NTI>
static void launch_rows_gemm_nt(const T* A, int lda, int M, int K, const T* Bw, int Kp, T* C, int ldc, int N,
                                hipStream_t st) {
    constexpr int PT = NTI <= 4 ? 4 : (NTI <= 8 ? 2 : 1);
    const int rows_per_block = 4 * PT * 16;
    const size_t lds = rows_gemm_lds(NTI, Kp, (int)sizeof(T));
    const int ntiles = (M + rows_per_block - 1) / rows_per_block;
    // ~4 workgroups per CU resident, each walking several row tiles
    const int grid = std::min(ntiles, 1024);
    hipLaunchKernelGGL((rows_gemm_kernel<T, NTI, PT>), dim3(grid), dim3(256), lds, st, A, lda, M, K, Bw, Kp, C, ldc,
                       N);
}

template <typename T>
static void launch_rows_gemm(int nti, const T* A, int lda, int M, int K, const T* Bw, int Kp, T* C, int ldc, int N,
                             hipStream_t st) {
    switch (nti) {
        case 1: launch_rows_gemm_nt<T, 1>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 2: launch_rows_gemm_nt<T, 2>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 3: launch_rows_gemm_nt<T, 3>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 4: launch_rows_gemm_nt<T, 4>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 5: launch_rows_gemm_nt<T, 5>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 6: launch_rows_gemm_nt<T, 6>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 7: launch_rows_gemm_nt<T, 7>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 8: launch_rows_gemm_nt<T, 8>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        case 12: launch_rows_gemm_nt<T, 12>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
        default: launch_rows_gemm_nt<T, 16>(A, lda, M, K, Bw, Kp, C, ldc, N, st); break;
    }
}

// out[b][c][oy][ox] = bias[c] + sum_{kh,kw: oy = iy*s - p + kh} P[b][iy][ix][(kh*k+kw)*Cout + c]
// block = C2I_TH x C2I_TW output pixels (all channels); the P window it reads
// (IR x IC input pixels x Np) is staged in LDS first.  grid (OW/TW, OH/TH, B)
template <typename T>
__global__ __launch_bounds__(256) void col2im_kernel(const T* __restrict__ P, int H, int W, int Np, int Cout, int OH,
                                                     int OW, int k, int s, int p, const float* __restrict__ bias,
                                                     float* __restrict__ out, int IR, int IC) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const int tid = threadIdx.x;
    const int ox0 = blockIdx.x * C2I_TW, oy0 = blockIdx.y * C2I_TH, b = blockIdx.z;
    const int iy_lo = floordiv(oy0 + p - (k - 1), s), ix_lo = floordiv(ox0 + p - (k - 1), s);
    const int cpp = Np * (int)sizeof(T) / 16;
    const T* Pb = P + (int64_t)b * H * W * Np;
    for (int i = tid; i < IR * IC * cpp; i += 256) {
        const int pix = i / cpp, c = i - (i / cpp) * cpp;
        const int r = pix / IC, cc = pix - (pix / IC) * IC;
        const int iy = iy_lo + r, ix = ix_lo + cc;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (iy >= 0 && iy < H && ix >= 0 && ix < W)
            v = *reinterpret_cast<const u32x4*>(Pb + ((int64_t)iy * W + ix) * Np + c * (16 / (int)sizeof(T)));
        *reinterpret_cast<u32x4*>(sm + (size_t)i * 16) = v;
    }
    __syncthreads();
    const int oy = oy0 + (tid / C2I_TW), ox = ox0 + (tid % C2I_TW);
    if (oy >= OH || ox >= OW) return;
    const T* S = reinterpret_cast<const T*>(sm);
    float acc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = (c < Cout && bias) ? bias[c] : 0.f;
    const int ry = (oy + p) % s, rx = (ox + p) % s;
    for (int kh = ry; kh < k; kh += s) {
        const int iy = (oy + p - kh) / s;
        if (iy < 0 || iy >= H) continue;
        for (int kw = rx; kw < k; kw += s) {
            const int ix = (ox + p - kw) / s;
            if (ix < 0 || ix >= W) continue;
            const T* src = S + ((iy - iy_lo) * IC + (ix - ix_lo)) * Np + (kh * k + kw) * Cout;
#pragma unroll
            for (int c = 0; c < 16; ++c)
                if (c < Cout) acc[c] += to_f32(src[c]);
        }
    }
    const int plane = OH * OW;
    float* o = out + (int64_t)b * Cout * plane + oy * OW + ox;
#pragma unroll
    for (int c = 0; c < 16; ++c)
        if (c < Cout) o[(int64_t)c * plane] = acc[c];
}

// Q[b][iy][ix][n] = dOut[b][c][iy*s - p + kh][ix*s - p + kw], n = (kh*k + kw)*Cout + c
// block = I2C_TH x I2C_TW input pixels; the dOut window (Cout x R x Cc) is
// staged in LDS, then each thread writes 8-column chunks of Q rows.
template <typename T>
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ dy, int H, int W, int Np, int Cout,
                                                     int OH, int OW, int k, int s, int p, T* __restrict__ Q, int R,
                                                     int Cc) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    float* S = reinterpret_cast<float*>(sm);
    const int tid = threadIdx.x;
    const int ix0 = blockIdx.x * I2C_TW, iy0 = blockIdx.y * I2C_TH, b = blockIdx.z;
    const int oy_lo = iy0 * s - p, ox_lo = ix0 * s - p;
    const float* src = dy + (int64_t)b * Cout * OH * OW;
    for (int i = tid; i < Cout * R * Cc; i += 256) {
        const int cc = i % Cc, rr = i / Cc;
        const int r = rr % R, c = rr / R;
        const int oy = oy_lo + r, ox = ox_lo + cc;
        S[i] = (oy >= 0 && oy < OH && ox >= 0 && ox < OW) ? src[((int64_t)c * OH + oy) * OW + ox] : 0.f;
    }
    // column n -> window offset (c*R + kh)*Cc + kw, or -1 for the pad columns
    int* off = reinterpret_cast<int*>(sm + (size_t)Cout * R * Cc * 4);
    const int kk = k * k;
    for (int n = tid; n < Np; n += 256) {
        int o = -1;
        if (n < kk * Cout) {
            const int t = n / Cout, c = n - (n / Cout) * Cout;
            const int kh = t / k, kw = t - (t / k) * k;
            o = (c * R + kh) * Cc + kw;
        }
        off[n] = o;
    }
    __syncthreads();
    const int nch = Np / 8;
    for (int i = tid; i < I2C_TH * I2C_TW * nch; i += 256) {
        const int pix = i / nch, ch = i - (i / nch) * nch;
        const int ly = pix / I2C_TW, lx = pix - (pix / I2C_TW) * I2C_TW;
        const int iy = iy0 + ly, ix = ix0 + lx;
        if (iy >= H || ix >= W) continue;
        const int base = ly * s * Cc + lx * s;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int o = off[ch * 8 + e];
            v[e] = o >= 0 ? S[base + o] : 0.f;
        }
        T* dst = Q + (((int64_t)b * H + iy) * W + ix) * Np + ch * 8;
        if constexpr (sizeof(T) == 2) {
            bf16x8 h;
#pragma unroll
            for (int e = 0; e < 8; ++e) h[e] = (bf16)v[e];
            *reinterpret_cast<bf16x8*>(dst) = h;
        } else {
            *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
            *reinterpret_cast<f32x4*>(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
        }
    }
}

// dW[ci][c][kh][kw] (+)= dWt[(kh*k+kw)*Cout + c][ci]
__global__ void small_dw_scatter_kernel(const float* __restrict__ dwt, int Cin, int Cout, int kk,
                                        float* __restrict__ dw, int accumulate) {
    const int total = Cin * Cout * kk;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int t = i % kk;
        const int ci_c = i / kk;
        const int c = ci_c % Cout, ci = ci_c / Cout;
        const float v = dwt[(int64_t)(t * Cout + c) * Cin + ci];
        dw[i] = accumulate ? dw[i] + v : v;
    }
}

// per-channel sums of an NCHW fp32 tensor: stage 1 partials [chunk][c], stage 2
// one wave per channel, fixed order (deterministic)
__global__ __launch_bounds__(256) void nchw_sum_stage1(const float* __restrict__ x, int B, int C, int64_t HW,
                                                        int nchunk, float* __restrict__ part) {
    __shared__ float red[4];
    const int c = blockIdx.y, chunk = blockIdx.x;
    const int64_t per = (HW + nchunk - 1) / nchunk;
    const int64_t s0 = chunk * per, s1 = std::min<int64_t>(HW, s0 + per);
    float acc = 0.f;
    for (int b = 0; b < B; ++b) {
        const float* src = x + ((int64_t)b * C + c) * HW;
        for (int64_t i = s0 + threadIdx.x; i < s1; i += 256) acc += src[i];
    }
    const float r = block_sum<256>(acc, red);
    if (threadIdx.x == 0) part[(int64_t)chunk * C + c] = r;
}
__global__ __launch_bounds__(64) void nchw_sum_stage2(const float* __restrict__ part, int nchunk, int C,
                                                       float* __restrict__ out, int accumulate) {
    const int c = blockIdx.x, lane = threadIdx.x;
    float s = 0.f;
    for (int i = lane; i < nchunk; i += 64) s += part[(int64_t)i * C + c];
    s = wave_sum(s);
    if (lane == 0) out[c] = accumulate ? out[c] + s : s;
}

static int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256)); }

static int check_small(const cai_conv_geom* g, int dtype, int x_ld) {
    CAI_CHECK_ARG(g && g->transposed, "deconv_small: needs a ConvTranspose2d geometry");
    CAI_CHECK_ARG(g->out_c >= 1 && g->out_c <= 16, "deconv_small: out_c %d not in [1, 16]", g->out_c);
    CAI_CHECK_ARG(g->kernel * g->kernel * g->out_c <= 256, "deconv_small: k*k*out_c > 256");
    CAI_CHECK_ARG(g->in_c % 8 == 0 && g->in_c <= 256, "deconv_small: in_c must be a multiple of 8, <= 256");
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "deconv_small: bad dtype");
    CAI_CHECK_ARG(x_ld >= g->in_c && x_ld % 8 == 0, "deconv_small: bad input layout");
    CAI_CHECK_ARG(g->stride >= 1 && g->pad >= 0 && g->kernel >= 1, "deconv_small: bad geometry");
    const int oh = (g->in_h - 1) * g->stride - 2 * g->pad + g->kernel + g->output_padding;
    const int ow = (g->in_w - 1) * g->stride - 2 * g->pad + g->kernel + g->output_padding;
    CAI_CHECK_ARG(oh == g->out_h && ow == g->out_w, "deconv_small: output size mismatch");
    const int64_t np = rup(g->kernel * g->kernel * g->out_c, 16);
    CAI_CHECK_ARG((int64_t)g->batch * g->in_h * g->in_w * std::max<int64_t>(np, x_ld) < (1ll << 31) &&
                      (int64_t)oh * ow * g->out_c < (1ll << 31),
                  "deconv_small: tensor too large for 32-bit indexing");
    const SmallPlan L = small_plan(g, dtype);
    const int es = dtype_size(dtype);
    constexpr size_t kLds = 64 * 1024;
    CAI_CHECK_ARG(rows_gemm_lds(L.NTf, L.Kpf, es) <= kLds && rows_gemm_lds(L.NTb, L.Kpb, es) <= kLds &&
                      col2im_lds(L, es) <= kLds && im2col_lds(L) <= kLds,
                  "deconv_small: geometry needs more than 64 KB of LDS per workgroup");
    return CAI_OK;
}

template <typename T>
static void small_fwd_t(const SmallPlan& L, const void* x, int x_ld, const float* w, const float* bias, float* y,
                        char* ws, hipStream_t st) {
    T* wf = reinterpret_cast<T*>(ws + L.off_wf);
    T* P = reinterpret_cast<T*>(ws + L.off_pq);
    const int nf = L.NTf * 16 * L.Kpf;
    hipLaunchKernelGGL(small_prep_kernel<T>, dim3(grid_for(nf)), dim3(256), 0, st, w, L.Cin, L.Cout, L.kk, wf,
                       L.NTf * 16, L.Kpf, (T*)nullptr, 0, 0);
    const int M = L.B * L.H * L.W;
    launch_rows_gemm<T>(L.NTf, reinterpret_cast<const T*>(x), x_ld, M, L.Cin, wf, L.Kpf, P, L.Np, L.Np, st);
    const dim3 grid((L.OW + C2I_TW - 1) / C2I_TW, (L.OH + C2I_TH - 1) / C2I_TH, L.B);
    hipLaunchKernelGGL(col2im_kernel<T>, grid, dim3(256), col2im_lds(L, sizeof(T)), st, P, L.H, L.W, L.Np, L.Cout,
                       L.OH, L.OW, L.k, L.s, L.p, bias, y, L.c2i_r, L.c2i_c);
}

template <typename T>
static int small_bwd_t(const SmallPlan& L, int dtype, const void* x, int x_ld, const float* w, const float* dy,
                       void* dx, int dx_ld, float* dw, float* db, int accumulate, char* ws, void* stream) {
    hipStream_t st = as_stream(stream);
    T* Q = reinterpret_cast<T*>(ws + L.off_pq);
    const dim3 qgrid((L.W + I2C_TW - 1) / I2C_TW, (L.H + I2C_TH - 1) / I2C_TH, L.B);
    hipLaunchKernelGGL(im2col_kernel<T>, qgrid, dim3(256), im2col_lds(L), st, dy, L.H, L.W, L.Np, L.Cout, L.OH, L.OW,
                       L.k, L.s, L.p, Q, L.i2c_r, L.i2c_c);
    if (dx) {
        T* wb = reinterpret_cast<T*>(ws + L.off_wb);
        const int nb = L.NTb * 16 * L.Kpb;
        hipLaunchKernelGGL(small_prep_kernel<T>, dim3(grid_for(nb)), dim3(256), 0, st, w, L.Cin, L.Cout, L.kk,
                           (T*)nullptr, 0, 0, wb, L.NTb * 16, L.Kpb);
        const int M = L.B * L.H * L.W;
        launch_rows_gemm<T>(L.NTb, Q, L.Np, M, L.Np, wb, L.Kpb, reinterpret_cast<T*>(dx), dx_ld, L.Cin, st);
    }
    if (dw) {
        float* dwt = reinterpret_cast<float*>(ws + L.off_dwt);
        const int rc = cai_conv_wgrad(&L.g_w, dtype, x, x_ld, 0, 0, Q, L.Np, dwt, nullptr, 0, ws + L.off_wg,
                                      cai_conv_wgrad_workspace_bytes(&L.g_w, dtype), stream);
        if (rc) return rc;
        hipLaunchKernelGGL(small_dw_scatter_kernel, dim3(grid_for((int64_t)L.Cin * L.Cout * L.kk)), dim3(256), 0, st,
                           dwt, L.Cin, L.Cout, L.kk, dw, accumulate);
    }
    if (db) {
        float* part = reinterpret_cast<float*>(ws + L.off_col);
        const int nchunk = 256;
        hipLaunchKernelGGL(nchw_sum_stage1, dim3(nchunk, L.Cout), dim3(256), 0, st, dy, L.B, L.Cout,
                           (int64_t)L.OH * L.OW, nchunk, part);
        hipLaunchKernelGGL(nchw_sum_stage2, dim3(L.Cout), dim3(64), 0, st, part, nchunk, L.Cout, db, accumulate);
    }
    return CAI_OK;
}

}  // namespace cai

using namespace cai;

extern "C" {

size_t cai_deconv_small_workspace_bytes(const cai_conv_geom* g, int dtype) {
    if (!g || check_small(g, dtype, g->in_c) != CAI_OK) return 0;
    return small_plan(g, dtype).total;
}

int cai_deconv_small_fwd(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, const float* w,
                         const float* bias, float* y, void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_small(g, dtype, x_ld);
    if (rc) return rc;
    const SmallPlan L = small_plan(g, dtype);
    CAI_CHECK_ARG(x && w && y, "deconv_small_fwd: null pointer");
    CAI_CHECK_ARG(workspace && ws_bytes >= L.total, "deconv_small_fwd: workspace too small (%zu < %zu)", ws_bytes,
                  L.total);
    char* ws = reinterpret_cast<char*>(workspace);
    if (dtype == CAI_BF16)
        small_fwd_t<bf16>(L, x, x_ld, w, bias, y, ws, as_stream(stream));
    else
        small_fwd_t<float>(L, x, x_ld, w, bias, y, ws, as_stream(stream));
    CAI_LAUNCH_CHECK("deconv_small_fwd");
    return CAI_OK;
}

int cai_deconv_small_bwd(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, const float* w,
                         const float* dy, void* dx, int32_t dx_ld, float* dw, float* db, int32_t accumulate,
                         void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_small(g, dtype, x_ld);
    if (rc) return rc;
    const SmallPlan L = small_plan(g, dtype);
    CAI_CHECK_ARG(x && w && dy, "deconv_small_bwd: null pointer");
    CAI_CHECK_ARG(!dx || (dx_ld >= g->in_c && dx_ld % 4 == 0), "deconv_small_bwd: bad dx layout");
    CAI_CHECK_ARG(workspace && ws_bytes >= L.total, "deconv_small_bwd: workspace too small (%zu < %zu)", ws_bytes,
                  L.total);
    char* ws = reinterpret_cast<char*>(workspace);
    rc = dtype == CAI_BF16 ? small_bwd_t<bf16>(L, dtype, x, x_ld, w, dy, dx, dx_ld, dw, db, accumulate, ws, stream)
                           : small_bwd_t<float>(L, dtype, x, x_ld, w, dy, dx, dx_ld, dw, db, accumulate, ws, stream);
    if (rc) return rc;
    CAI_LAUNCH_CHECK("deconv_small_bwd");
    return CAI_OK;
}

}  // extern "C"
