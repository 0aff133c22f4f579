// ConvTranspose2d with few output channels (the synthesis transform's last
// layer, deconv(N, 3 or 1), models/utils.py:138-146 / google.py:244-252).
//
// Output-stationary implicit GEMM is a poor fit here (N = 3 of a 16-wide MFMA
// tile, and every output pixel re-gathers its input taps).  Instead:
//   forward : P = x * W'   -- one dense 1x1 GEMM per input pixel with
//             N = k*k*Cout (75 -> 80 padded) columns, W'[(kh,kw,c)][ci]
//             out = bias + col2im(P)  -- each output pixel sums its <= 9
//             (stride 2) contributions, written as fp32 NCHW (x_hat)
//   backward: Q = im2col(dOut)  ([input pixel][(kh,kw,c)])
//             dx  = Q * W'^T (1x1 GEMM, K = 80)
//             dW' = Q^T x    (1x1 wgrad), scattered back to [ci][c][kh][kw]
//             db  = per-channel sums of dOut
// The GEMMs run on the implicit-GEMM / wgrad kernels of conv.hip.
#include "common.hpp"

#include <algorithm>

namespace cai {

static int rup(int v, int m) { return (v + m - 1) / m * m; }

struct SmallPlan {
    int B, Cin, Cout, H, W, OH, OW, k, s, p, kk, Np;
    cai_conv_geom g_fwd;    // 1x1 Conv2d: Cin -> Np       (P = x W')
    cai_conv_geom g_dx;     // 1x1 ConvTranspose2d: Np -> Cin (dx = Q W'^T), weight layout [Np][Cin]
    size_t off_wt, off_pk, off_pm, off_q, off_cw, off_wg, off_dwt, off_col, total;
};

static SmallPlan small_plan(const cai_conv_geom* g, int dtype) {
    SmallPlan L{};
    L.B = g->batch; L.Cin = g->in_c; L.Cout = g->out_c; L.H = g->in_h; L.W = g->in_w;
    L.OH = g->out_h; L.OW = g->out_w; L.k = g->kernel; L.s = g->stride; L.p = g->pad;
    L.kk = L.k * L.k;
    L.Np = rup(L.kk * L.Cout, 8);
    L.g_fwd = cai_conv_geom{L.B, L.Cin, L.H, L.W, L.Np, L.H, L.W, 1, 1, 0, 0, 0};
    L.g_dx = cai_conv_geom{L.B, L.Np, L.H, L.W, L.Cin, L.H, L.W, 1, 1, 0, 0, 1};
    const int es = dtype_size(dtype);
    const int64_t npix = (int64_t)L.B * L.H * L.W;
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o += (n + 255) / 256 * 256; return r; };
    L.off_wt = take((size_t)L.Np * L.Cin * 4);
    const size_t pk = std::max(cai_conv_packed_weight_bytes(&L.g_fwd, dtype, 0),
                               cai_conv_packed_weight_bytes(&L.g_dx, dtype, 0));
    L.off_pk = take(pk);
    L.off_pm = take((size_t)npix * L.Np * es);     // P (forward) / Q (backward) share the slot
    L.off_q = L.off_pm;
    const size_t cw = std::max(cai_conv_workspace_bytes(&L.g_fwd, dtype, 0), cai_conv_workspace_bytes(&L.g_dx, dtype, 0));
    L.off_cw = take(std::max<size_t>(cw, 16));
    L.off_wg = take(cai_conv_wgrad_workspace_bytes(&L.g_fwd, dtype));
    L.off_dwt = take((size_t)L.Np * L.Cin * 4);
    L.off_col = take((size_t)1024 * L.Cout * 4);
    L.total = o;
    return L;
}

// Wt[n][ci] = W[ci][c][kh][kw], n = (kh*k + kw)*Cout + c  (0 for the pad rows)
__global__ void small_wt_kernel(const float* __restrict__ w, int Cin, int Cout, int kk, int Np, float* __restrict__ wt) {
    const int total = Np * Cin;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int n = i / Cin, ci = i - (i / Cin) * Cin;
        float v = 0.f;
        if (n < kk * Cout) {
            const int t = n / Cout, c = n - (n / Cout) * Cout;
            v = w[((int64_t)ci * Cout + c) * kk + t];
        }
        wt[i] = v;
    }
}

// out[b][c][oy][ox] = bias[c] + sum_{kh,kw: oy = iy*s - p + kh} P[b][iy][ix][(kh*k+kw)*Cout + c]
template <typename T>
__global__ void col2im_kernel(const T* __restrict__ P, int B, int H, int W, int Np, int Cout, int OH, int OW, int k,
                              int s, int p, const float* __restrict__ bias, float* __restrict__ out) {
    const int64_t total = (int64_t)B * Cout * OH * OW;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int ox = (int)(i % OW);
        int64_t r = i / OW;
        const int oy = (int)(r % OH);
        r /= OH;
        const int c = (int)(r % Cout);
        const int b = (int)(r / Cout);
        float acc = bias ? bias[c] : 0.f;
        const int ry = (oy + p) % s, rx = (ox + p) % s;
        for (int kh = ry; kh < k; kh += s) {
            const int iy = (oy + p - kh) / s;
            if (iy < 0 || iy >= H) continue;
            for (int kw = rx; kw < k; kw += s) {
                const int ix = (ox + p - kw) / s;
                if (ix < 0 || ix >= W) continue;
                acc += to_f32(P[(((int64_t)b * H + iy) * W + ix) * Np + (kh * k + kw) * Cout + c]);
            }
        }
        out[i] = acc;
    }
}

// Q[b][iy][ix][n] = dOut[b][c][iy*s - p + kh][ix*s - p + kw], n = (kh*k + kw)*Cout + c
template <typename T>
__global__ void im2col_kernel(const float* __restrict__ dy, int B, int H, int W, int Np, int Cout, int OH, int OW,
                              int k, int s, int p, T* __restrict__ Q) {
    const int64_t total = (int64_t)B * H * W * Np;
    const int kk = k * k;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int n = (int)(i % Np);
        const int64_t pix = i / Np;
        const int ix = (int)(pix % W);
        const int64_t r = pix / W;
        const int iy = (int)(r % H);
        const int b = (int)(r / H);
        float v = 0.f;
        if (n < kk * Cout) {
            const int t = n / Cout, c = n - (n / Cout) * Cout;
            const int kh = t / k, kw = t - (t / k) * k;
            const int oy = iy * s - p + kh, ox = ix * s - p + kw;
            if (oy >= 0 && oy < OH && ox >= 0 && ox < OW) v = dy[(((int64_t)b * Cout + c) * OH + oy) * OW + ox];
        }
        Q[i] = from_f32<T>(v);
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

// per-channel sums of an NCHW fp32 tensor: stage 1 partials [chunk][c], stage 2 fixed order
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
__global__ void nchw_sum_stage2(const float* __restrict__ part, int nchunk, int C, float* __restrict__ out,
                                int accumulate) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float s = 0.f;
    for (int i = 0; i < nchunk; ++i) s += part[(int64_t)i * C + c];
    out[c] = accumulate ? out[c] + s : s;
}

static int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256)); }

static int check_small(const cai_conv_geom* g, int dtype, int x_ld) {
    CAI_CHECK_ARG(g && g->transposed, "deconv_small: needs a ConvTranspose2d geometry");
    CAI_CHECK_ARG(g->out_c <= 16, "deconv_small: out_c %d > 16", g->out_c);
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "deconv_small: bad dtype");
    CAI_CHECK_ARG(x_ld >= g->in_c && x_ld % 8 == 0 && g->in_c % 8 == 0, "deconv_small: bad input layout");
    const int oh = (g->in_h - 1) * g->stride - 2 * g->pad + g->kernel + g->output_padding;
    const int ow = (g->in_w - 1) * g->stride - 2 * g->pad + g->kernel + g->output_padding;
    CAI_CHECK_ARG(oh == g->out_h && ow == g->out_w, "deconv_small: output size mismatch");
    return CAI_OK;
}

}  // namespace cai

using namespace cai;

extern "C" {

size_t cai_deconv_small_workspace_bytes(const cai_conv_geom* g, int dtype) {
    if (!g || !g->transposed || g->out_c > 16) return 0;
    return small_plan(g, dtype).total;
}

int cai_deconv_small_fwd(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, const float* w,
                         const float* bias, float* y, void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_small(g, dtype, x_ld);
    if (rc) return rc;
    const SmallPlan L = small_plan(g, dtype);
    CAI_CHECK_ARG(workspace && ws_bytes >= L.total && w && y, "deconv_small_fwd: bad arguments / workspace");
    char* ws = reinterpret_cast<char*>(workspace);
    hipStream_t st = as_stream(stream);
    float* wt = reinterpret_cast<float*>(ws + L.off_wt);
    hipLaunchKernelGGL(small_wt_kernel, dim3(grid_for((int64_t)L.Np * L.Cin)), dim3(256), 0, st, w, L.Cin, L.Cout,
                       L.kk, L.Np, wt);
    rc = cai_conv_pack_weight(&L.g_fwd, dtype, 0, wt, nullptr, ws + L.off_pk, stream);
    if (rc) return rc;
    const int64_t ld = L.Np;
    rc = cai_conv_fwd(&L.g_fwd, dtype, x, x_ld, 0, ws + L.off_pk, nullptr, CAI_ACT_NONE, 0.f, ws + L.off_pm, dtype,
                      (int64_t)L.H * L.W * ld, 1, (int64_t)L.W * ld, ld, ws + L.off_cw,
                      cai_conv_workspace_bytes(&L.g_fwd, dtype, 0), stream);
    if (rc) return rc;
    const int64_t tot = (int64_t)L.B * L.Cout * L.OH * L.OW;
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(col2im_kernel<bf16>, dim3(grid_for(tot)), dim3(256), 0, st,
                           reinterpret_cast<const bf16*>(ws + L.off_pm), L.B, L.H, L.W, L.Np, L.Cout, L.OH, L.OW, L.k,
                           L.s, L.p, bias, y);
    else
        hipLaunchKernelGGL(col2im_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, st,
                           reinterpret_cast<const float*>(ws + L.off_pm), L.B, L.H, L.W, L.Np, L.Cout, L.OH, L.OW,
                           L.k, L.s, L.p, bias, y);
    CAI_LAUNCH_CHECK("deconv_small_fwd");
    return CAI_OK;
}

int cai_deconv_small_bwd(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld, const float* w,
                         const float* dy, void* dx, int32_t dx_ld, float* dw, float* db, int32_t accumulate,
                         void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_small(g, dtype, x_ld);
    if (rc) return rc;
    const SmallPlan L = small_plan(g, dtype);
    CAI_CHECK_ARG(workspace && ws_bytes >= L.total && w && dy, "deconv_small_bwd: bad arguments / workspace");
    char* ws = reinterpret_cast<char*>(workspace);
    hipStream_t st = as_stream(stream);
    const int64_t npix = (int64_t)L.B * L.H * L.W;
    // Q = im2col(dOut)
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(im2col_kernel<bf16>, dim3(grid_for(npix * L.Np)), dim3(256), 0, st, dy, L.B, L.H, L.W,
                           L.Np, L.Cout, L.OH, L.OW, L.k, L.s, L.p, reinterpret_cast<bf16*>(ws + L.off_q));
    else
        hipLaunchKernelGGL(im2col_kernel<float>, dim3(grid_for(npix * L.Np)), dim3(256), 0, st, dy, L.B, L.H, L.W,
                           L.Np, L.Cout, L.OH, L.OW, L.k, L.s, L.p, reinterpret_cast<float*>(ws + L.off_q));
    float* wt = reinterpret_cast<float*>(ws + L.off_wt);
    if (dx) {
        hipLaunchKernelGGL(small_wt_kernel, dim3(grid_for((int64_t)L.Np * L.Cin)), dim3(256), 0, st, w, L.Cin, L.Cout,
                           L.kk, L.Np, wt);
        rc = cai_conv_pack_weight(&L.g_dx, dtype, 0, wt, nullptr, ws + L.off_pk, stream);
        if (rc) return rc;
        const int64_t ld = dx_ld;
        rc = cai_conv_fwd(&L.g_dx, dtype, ws + L.off_q, L.Np, 0, ws + L.off_pk, nullptr, CAI_ACT_NONE, 0.f, dx, dtype,
                          (int64_t)L.H * L.W * ld, 1, (int64_t)L.W * ld, ld, ws + L.off_cw,
                          cai_conv_workspace_bytes(&L.g_dx, dtype, 0), stream);
        if (rc) return rc;
    }
    if (dw) {
        float* dwt = reinterpret_cast<float*>(ws + L.off_dwt);
        rc = cai_conv_wgrad(&L.g_fwd, dtype, x, x_ld, 0, 0, ws + L.off_q, L.Np, dwt, nullptr, 0, ws + L.off_wg,
                            cai_conv_wgrad_workspace_bytes(&L.g_fwd, dtype), stream);
        if (rc) return rc;
        hipLaunchKernelGGL(small_dw_scatter_kernel, dim3(grid_for((int64_t)L.Cin * L.Cout * L.kk)), dim3(256), 0, st,
                           dwt, L.Cin, L.Cout, L.kk, dw, accumulate);
    }
    if (db) {
        float* part = reinterpret_cast<float*>(ws + L.off_col);
        const int nchunk = 256;
        hipLaunchKernelGGL(nchw_sum_stage1, dim3(nchunk, L.Cout), dim3(256), 0, st, dy, L.B, L.Cout,
                           (int64_t)L.OH * L.OW, nchunk, part);
        hipLaunchKernelGGL(nchw_sum_stage2, dim3(1), dim3(64), 0, st, part, nchunk, L.Cout, db, accumulate);
    }
    CAI_LAUNCH_CHECK("deconv_small_bwd");
    return CAI_OK;
}

}  // extern "C"
