// Kernels of the multi-modal codec's alignment modules
// (compressai/models/master.py):
//   * LayerNorm over the channel dim of pixel-major tokens (SwinTransformerBlock
//     norm1 / norm2, master.py:603-606,657-660)            fwd / bwd
//   * exact-erf GELU (Mlp.act, master.py:465-482)          fwd / bwd
//   * shifted-window cross attention (WindowAttention.forward, master.py:534-568,
//     with the cyclic shift + window partition / reverse of
//     SwinTransformerBlock.forward, master.py:665-695, folded into the
//     token addressing): one wave per (window, head), 16 tokens x 32 dims,
//     scores / softmax / P.V in fp32 registers + LDS; the backward recomputes P
//     (flash style) and reduces the relative-position-bias gradient in a fixed
//     order
//   * Channel_aligner pooling + affine (master.py:179-210): per-(image,
//     channel) spatial means and y = gamma * x + beta broadcast      fwd / bwd
// Tokens are pixel-major rows: token l of image b is row b*L + l.
#include "common.hpp"

#include <algorithm>
#include <initializer_list>

namespace cai {

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i) { return to_f32(p[i]); }

// --------------------------------------------------------------------------
// LayerNorm: one wave per token, C <= 1024
// --------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const T* __restrict__ x, int xld, int ntok, int C,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            float eps, T* __restrict__ y, int yld,
                                                            float* __restrict__ mean, float* __restrict__ rstd) {
    const int lane = threadIdx.x & 63;
    const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tok >= ntok) return;
    const T* xr = x + (int64_t)tok * xld;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += ldf(xr, c);
    const float mu = wave_sum(s) / C;
    float v = 0.f;
    for (int c = lane; c < C; c += 64) {
        const float d = ldf(xr, c) - mu;
        v += d * d;
    }
    const float rs = rsqrtf(wave_sum(v) / C + eps);
    T* yr = y + (int64_t)tok * yld;
    for (int c = lane; c < C; c += 64) yr[c] = from_f32<T>((ldf(xr, c) - mu) * rs * w[c] + b[c]);
    if (lane == 0) {
        mean[tok] = mu;
        rstd[tok] = rs;
    }
}

// dx = rstd * (dyw - mean(dyw) - xhat * mean(dyw * xhat)), dyw = dy * w;
// per-block partials of dw = sum dy * xhat and db = sum dy: part[blk][2][C]
template <typename T>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* __restrict__ x, int xld, const T* __restrict__ dy,
                                                            int dyld, int ntok, int C, const float* __restrict__ w,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, T* __restrict__ dx,
                                                            int dxld, float* __restrict__ part, int tok_per_block) {
    extern __shared__ float sm[];   // [4 waves][2][C]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* pw = sm + wv * 2 * C;
    for (int c = lane; c < 2 * C; c += 64) pw[c] = 0.f;
    const int t0 = blockIdx.x * tok_per_block;
    const int t1 = min(ntok, t0 + tok_per_block);
    for (int tok = t0 + wv; tok < t1; tok += 4) {
        const T* xr = x + (int64_t)tok * xld;
        const T* gr = dy + (int64_t)tok * dyld;
        const float mu = mean[tok], rs = rstd[tok];
        float a = 0.f, bsum = 0.f;
        for (int c = lane; c < C; c += 64) {
            const float xh = (ldf(xr, c) - mu) * rs;
            const float g = ldf(gr, c);
            a += g * w[c];
            bsum += g * w[c] * xh;
            pw[c] += g * xh;
            pw[C + c] += g;
        }
        const float ma = wave_sum(a) / C, mb = wave_sum(bsum) / C;
        T* dr = dx + (int64_t)tok * dxld;
        for (int c = lane; c < C; c += 64) {
            const float xh = (ldf(xr, c) - mu) * rs;
            dr[c] = from_f32<T>(rs * (ldf(gr, c) * w[c] - ma - xh * mb));
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * C; c += 256) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) s += sm[k * 2 * C + c];
        part[(int64_t)blockIdx.x * 2 * C + c] = s;
    }
}

// C <= 128 (the Swin blocks' 96 channels): a lane's <= 2 channels of x / dy stay in registers between the two passes
// and the dw / db partials accumulate in registers, written to LDS once -- the general kernel above reloads x / dy
// for the dx pass and read-modify-writes LDS per token (31 us per call on the multimodal 40960 x 96 tokens)
template <typename T>
__global__ __launch_bounds__(256) void layernorm_bwd_reg_kernel(const T* __restrict__ x, int xld, const T* __restrict__ dy,
                                                                int dyld, int ntok, int C, const float* __restrict__ w,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd, T* __restrict__ dx,
                                                                int dxld, float* __restrict__ part, int tok_per_block) {
    extern __shared__ float sm[];   // [4 waves][2][C]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int c0 = lane, c1 = lane + 64;
    const bool h0 = c0 < C, h1 = c1 < C;
    const float w0 = h0 ? w[c0] : 0.f, w1 = h1 ? w[c1] : 0.f;
    float pw0 = 0.f, pw1 = 0.f, pb0 = 0.f, pb1 = 0.f;
    const int t0 = blockIdx.x * tok_per_block;
    const int t1 = min(ntok, t0 + tok_per_block);
    for (int tok = t0 + wv; tok < t1; tok += 4) {
        const T* xr = x + (int64_t)tok * xld;
        const T* gr = dy + (int64_t)tok * dyld;
        const float mu = mean[tok], rs = rstd[tok];
        const float x0 = h0 ? ldf(xr, c0) : 0.f, x1 = h1 ? ldf(xr, c1) : 0.f;
        const float g0 = h0 ? ldf(gr, c0) : 0.f, g1 = h1 ? ldf(gr, c1) : 0.f;
        const float xh0 = (x0 - mu) * rs, xh1 = (x1 - mu) * rs;
        const float a = wave_sum(g0 * w0 + g1 * w1);
        const float bs = wave_sum(g0 * w0 * xh0 + g1 * w1 * xh1);
        pw0 += g0 * xh0;
        pw1 += g1 * xh1;
        pb0 += g0;
        pb1 += g1;
        const float ma = a / C, mb = bs / C;
        T* dr = dx + (int64_t)tok * dxld;
        if (h0) dr[c0] = from_f32<T>(rs * (g0 * w0 - ma - xh0 * mb));
        if (h1) dr[c1] = from_f32<T>(rs * (g1 * w1 - ma - xh1 * mb));
    }
    float* pw = sm + wv * 2 * C;
    if (h0) { pw[c0] = pw0; pw[C + c0] = pb0; }
    if (h1) { pw[c1] = pw1; pw[C + c1] = pb1; }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * C; c += 256) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) s += sm[k * 2 * C + c];
        part[(int64_t)blockIdx.x * 2 * C + c] = s;
    }
}

// [nblk][2C] partials -> dw / db: a block per 32 columns, 32 row groups of 32 threads (row group g sums rows g,
// g + 32, ... in order, eight loads in flight), the 32 group sums combined in group order through LDS -- a fixed
// order, so the result is deterministic.  (One 192-thread block walking all 1024 rows serially took ~65 us per
// call: 18 calls, 1.2 ms of the multimodal step.)
constexpr int LNR_COLS = 32, LNR_GROUPS = 32;
__global__ __launch_bounds__(LNR_COLS * LNR_GROUPS) void layernorm_param_reduce(const float* __restrict__ part,
                                                                                int nblk, int C, float* __restrict__ dw,
                                                                                float* __restrict__ db, int accumulate) {
    __shared__ float red[LNR_GROUPS][LNR_COLS + 1];
    const int col = threadIdx.x % LNR_COLS, grp = threadIdx.x / LNR_COLS;
    const int c = blockIdx.x * LNR_COLS + col;
    float s = 0.f;
    if (c < 2 * C) {
        int i = grp;
        for (; i + 7 * LNR_GROUPS < nblk; i += 8 * LNR_GROUPS) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = part[(int64_t)(i + j * LNR_GROUPS) * 2 * C + c];
#pragma unroll
            for (int j = 0; j < 8; ++j) s += v[j];
        }
        for (; i < nblk; i += LNR_GROUPS) s += part[(int64_t)i * 2 * C + c];
    }
    red[grp][col] = s;
    __syncthreads();
    if (grp != 0 || c >= 2 * C) return;
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < LNR_GROUPS; ++g) t += red[g][col];
    float* base = c < C ? dw : db;
    if (base == nullptr) return;
    float* d = base + (c < C ? c : c - C);
    *d = accumulate ? *d + t : t;
}

// --------------------------------------------------------------------------
// GELU (exact): y = x * Phi(x)
// --------------------------------------------------------------------------
template <typename T>
__global__ void gelu_fwd_kernel(const T* __restrict__ x, int xld, T* __restrict__ y, int yld, int ntok, int C) {
    const int64_t total = (int64_t)ntok * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(i / C), c = (int)(i - (int64_t)t * C);
        const float v = ldf(x, (int64_t)t * xld + c);
        y[(int64_t)t * yld + c] = from_f32<T>(0.5f * v * (1.f + erff(v * 0.70710678118654752f)));
    }
}

template <typename T>
__global__ void gelu_bwd_kernel(const T* __restrict__ x, int xld, const T* __restrict__ g, int gld,
                                T* __restrict__ dx, int dxld, int ntok, int C) {
    const int64_t total = (int64_t)ntok * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(i / C), c = (int)(i - (int64_t)t * C);
        const float v = ldf(x, (int64_t)t * xld + c);
        const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
        const float pdf = 0.3989422804014327f * __expf(-0.5f * v * v);
        dx[(int64_t)t * dxld + c] = from_f32<T>(ldf(g, (int64_t)t * gld + c) * (cdf + v * pdf));
    }
}

// --------------------------------------------------------------------------
// Window cross attention.  Window size WS = 4 (N = 16 tokens), head dim 32.
// --------------------------------------------------------------------------
constexpr int WS = 4, WN = WS * WS, HD = 32;

struct AttnArgs {
    const void* q;  int q_ld;        // [B*L][>= heads*32]: q = qkv1(x)
    const void* kv; int kv_ld;       // [B*L][>= 2*heads*32]: k = cols [0, C), v = cols [C, 2C)
    void* o; int o_ld;               // output rows (token order), heads*32 columns
    const float* bias_table;         // [(2WS-1)^2][heads]
    const int* rel_index;            // [WN][WN]
    const float* mask;               // [nW][WN][WN] or NULL
    int B, Hr, Wr, heads, shift;
    float scale;
    // backward
    const void* dout; int dout_ld;
    void* dq; int dq_ld;
    void* dkv; int dkv_ld;
    float* dbias_part;               // [gridDim.x][heads][WN][WN]
};

// token row of window position (wy, wx, iy, ix) after the cyclic shift
__device__ __forceinline__ int64_t win_row(const AttnArgs& a, int b, int wy, int wx, int i) {
    const int iy = i / WS, ix = i % WS;
    int r = wy * WS + iy + a.shift, c = wx * WS + ix + a.shift;
    if (r >= a.Hr) r -= a.Hr;
    if (c >= a.Wr) c -= a.Wr;
    return (int64_t)b * a.Hr * a.Wr + (int64_t)r * a.Wr + c;
}

// one wave per (window, head); block = 4 waves
template <typename T>
__global__ __launch_bounds__(256) void window_attn_fwd_kernel(const AttnArgs a) {
    __shared__ float sq[4][WN][HD + 1], sk[4][WN][HD + 1], sv[4][WN][HD + 1], sp[4][WN][WN + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nWy = a.Hr / WS, nWx = a.Wr / WS, nW = nWy * nWx;
    const int item0 = blockIdx.x * 4 + wv;
    const int total = a.B * nW * a.heads;
    // waves past the end repeat the last item (no early exit before the barriers)
    const int item = min(item0, total - 1);
    const bool live = item0 < total;
    const int h = item % a.heads;
    const int wglob = item / a.heads;
    const int b = wglob / nW, w = wglob - b * nW;
    const int wy = w / nWx, wx = w - wy * nWx;
    const int C = a.heads * HD;
    const T* Q = reinterpret_cast<const T*>(a.q);
    const T* KV = reinterpret_cast<const T*>(a.kv);
    // load 16 tokens x 32 dims of q, k, v: lane -> (token lane/4, dims (lane%4)*8 .. +8)
    {
        const int i = lane >> 2, d0 = (lane & 3) * 8;
        const int64_t row = win_row(a, b, wy, wx, i);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            sq[wv][i][d0 + e] = ldf(Q, row * a.q_ld + h * HD + d0 + e) * a.scale;
            sk[wv][i][d0 + e] = ldf(KV, row * a.kv_ld + h * HD + d0 + e);
            sv[wv][i][d0 + e] = ldf(KV, row * a.kv_ld + C + h * HD + d0 + e);
        }
    }
    __syncthreads();
    // scores: lane -> row i = lane/4, columns j = (lane%4)*4 .. +4
    const int i = lane >> 2, j0 = (lane & 3) * 4;
    float s[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        const int j = j0 + jj;
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < HD; ++d) acc += sq[wv][i][d] * sk[wv][j][d];
        acc += a.bias_table[a.rel_index[i * WN + j] * a.heads + h];
        if (a.mask) acc += a.mask[((int64_t)w * WN + i) * WN + j];
        s[jj] = acc;
    }
    float m = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
    m = fmaxf(m, __shfl_xor(m, 1));
    m = fmaxf(m, __shfl_xor(m, 2));
    float e[4], sum = 0.f;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        e[jj] = __expf(s[jj] - m);
        sum += e[jj];
    }
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    const float inv = 1.f / sum;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) sp[wv][i][j0 + jj] = e[jj] * inv;
    __syncthreads();
    // O[i][d] = sum_j P[i][j] v[j][d]: lane -> row i, dims (lane%4)*8 .. +8
    T* Out = reinterpret_cast<T*>(a.o);
    const int64_t row = win_row(a, b, wy, wx, i);
    const int d0 = (lane & 3) * 8;
    if (!live) return;
#pragma unroll
    for (int dd = 0; dd < 8; ++dd) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < WN; ++j) acc += sp[wv][i][j] * sv[wv][j][d0 + dd];
        Out[row * a.o_ld + h * HD + d0 + dd] = from_f32<T>(acc);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void window_attn_bwd_kernel(const AttnArgs a) {
    __shared__ float sq[4][WN][HD + 1], sk[4][WN][HD + 1], sv[4][WN][HD + 1], sdo[4][WN][HD + 1];
    __shared__ float sp[4][WN][WN + 1], sds[4][WN][WN + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nWy = a.Hr / WS, nWx = a.Wr / WS, nW = nWy * nWx;
    const int item = blockIdx.x * 4 + wv;
    const int total = a.B * nW * a.heads;
    const bool live = item < total;
    const int h = live ? item % a.heads : 0;
    const int wglob = item / a.heads;
    const int b = wglob / nW, w = wglob - b * nW;
    const int wy = w / nWx, wx = w - wy * nWx;
    const int C = a.heads * HD;
    const T* Q = reinterpret_cast<const T*>(a.q);
    const T* KV = reinterpret_cast<const T*>(a.kv);
    const T* DO = reinterpret_cast<const T*>(a.dout);
    const int i = lane >> 2, j0 = (lane & 3) * 4, d0 = (lane & 3) * 8;
    const int64_t row = live ? win_row(a, b, wy, wx, i) : 0;
    if (live) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            sq[wv][i][d0 + e] = ldf(Q, row * a.q_ld + h * HD + d0 + e) * a.scale;
            sk[wv][i][d0 + e] = ldf(KV, row * a.kv_ld + h * HD + d0 + e);
            sv[wv][i][d0 + e] = ldf(KV, row * a.kv_ld + C + h * HD + d0 + e);
            sdo[wv][i][d0 + e] = ldf(DO, row * a.dout_ld + h * HD + d0 + e);
        }
    }
    __syncthreads();
    float ds[4] = {0.f, 0.f, 0.f, 0.f};
    if (live) {
        float s[4], dp[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = j0 + jj;
            float acc = 0.f, accp = 0.f;
#pragma unroll
            for (int d = 0; d < HD; ++d) {
                acc += sq[wv][i][d] * sk[wv][j][d];
                accp += sdo[wv][i][d] * sv[wv][j][d];
            }
            acc += a.bias_table[a.rel_index[i * WN + j] * a.heads + h];
            if (a.mask) acc += a.mask[((int64_t)w * WN + i) * WN + j];
            s[jj] = acc;
            dp[jj] = accp;
        }
        float m = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
        m = fmaxf(m, __shfl_xor(m, 1));
        m = fmaxf(m, __shfl_xor(m, 2));
        float e[4], sum = 0.f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            e[jj] = __expf(s[jj] - m);
            sum += e[jj];
        }
        sum += __shfl_xor(sum, 1);
        sum += __shfl_xor(sum, 2);
        const float inv = 1.f / sum;
        float p[4], pdp = 0.f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            p[jj] = e[jj] * inv;
            pdp += p[jj] * dp[jj];
        }
        pdp += __shfl_xor(pdp, 1);
        pdp += __shfl_xor(pdp, 2);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            ds[jj] = p[jj] * (dp[jj] - pdp);
            sp[wv][i][j0 + jj] = p[jj];
            sds[wv][i][j0 + jj] = ds[jj];
        }
    }
    __syncthreads();
    if (live) {
        T* DQ = reinterpret_cast<T*>(a.dq);
        T* DKV = reinterpret_cast<T*>(a.dkv);
        // lane -> token t = lane/4 (as query i for dq, as key j for dk / dv), dims d0 .. +8
        const int t = i;
#pragma unroll
        for (int dd = 0; dd < 8; ++dd) {
            const int d = d0 + dd;
            float dq = 0.f, dk = 0.f, dv = 0.f;
#pragma unroll
            for (int u = 0; u < WN; ++u) {
                dq += sds[wv][t][u] * sk[wv][u][d];
                dk += sds[wv][u][t] * sq[wv][u][d];
                dv += sp[wv][u][t] * sdo[wv][u][d];
            }
            DQ[row * a.dq_ld + h * HD + d] = from_f32<T>(dq * a.scale);
            DKV[row * a.dkv_ld + h * HD + d] = from_f32<T>(dk);
            DKV[row * a.dkv_ld + C + h * HD + d] = from_f32<T>(dv);
        }
    }
    // relative-position-bias gradient: this block's sum of dS per (head, i, j)
    // (waves of one block may hold different heads: accumulate per head in LDS)
    __syncthreads();
    float* acc = &sq[0][0][0];   // reuse: heads * WN * WN floats (heads <= 8)
    for (int k = threadIdx.x; k < a.heads * WN * WN; k += 256) acc[k] = 0.f;
    __syncthreads();
    for (int k = 0; k < 4; ++k) {
        const int it = blockIdx.x * 4 + k;
        if (it >= total) break;
        const int hh = it % a.heads;
        if (wv == 0) {   // one wave folds the 4 waves' dS in a fixed order
            for (int q = lane; q < WN * WN; q += 64) acc[hh * WN * WN + q] += sds[k][q / WN][q % WN];
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < a.heads * WN * WN; k += 256) a.dbias_part[(int64_t)blockIdx.x * a.heads * WN * WN + k] = acc[k];
}

// dtable[idx[i][j]][h] (+)= sum_blocks part[blk][h][i][j], in a fixed order and
// in three stages, so that every stage has plenty of threads:
//   1. part[blk][e] -> part2[split][e]   (e = h*WN*WN + ij: coalesced rows, a block range per split)
//   2. part2[split][e] -> tot[e]
//   3. dtable[r][h] = sum over ij with rel_index[ij] == r of tot[h][ij]
constexpr int ATTN_SPLITS = 64;
__global__ __launch_bounds__(256) void attn_bias_sum_splits(const float* __restrict__ part, int nblk, int E,
                                                            float* __restrict__ part2) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    const int per = (nblk + ATTN_SPLITS - 1) / ATTN_SPLITS;
    const int b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
    float s = 0.f;
    for (int blk = b0; blk < b1; ++blk) s += part[(int64_t)blk * E + e];
    part2[blockIdx.y * E + e] = s;
}
__global__ __launch_bounds__(256) void attn_bias_sum_total(const float* __restrict__ part2, int E,
                                                           float* __restrict__ tot) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    float s = 0.f;
    for (int sp = 0; sp < ATTN_SPLITS; ++sp) s += part2[sp * E + e];
    tot[e] = s;
}
__global__ void attn_bias_grad_reduce(const float* __restrict__ tot, int heads, const int* __restrict__ rel_index,
                                      int table_rows, float* __restrict__ dtable, int accumulate) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= table_rows * heads) return;
    const int r = e / heads, h = e - (e / heads) * heads;
    float s = 0.f;
    for (int ij = 0; ij < WN * WN; ++ij)
        if (rel_index[ij] == r) s += tot[h * WN * WN + ij];
    dtable[e] = accumulate ? dtable[e] + s : s;
}

// --------------------------------------------------------------------------
// Channel aligner: per-(image, channel) means, y = gamma[b][c] * x + beta[b][c]
// --------------------------------------------------------------------------
// out[b][c] = scale * sum_p x[b][p][c] (* x2[b][p][c]), two stages, fixed order.
// Stage 1: block (chunk, b) sums a pixel chunk of image b for every channel:
// thread = (16-byte channel group, pixel row), rows in flight = 256 / groups.
template <typename T>
__global__ __launch_bounds__(256) void channel_mean_stage1(const T* __restrict__ x, int xld,
                                                           const T* __restrict__ x2, int x2ld, int HW, int C,
                                                           int chunk, float* __restrict__ part) {
    constexpr int VEC = 16 / sizeof(T);
    __shared__ float red[256 * VEC];
    const int ngrp = (C + VEC - 1) / VEC;
    const int rows = 256 / ngrp;
    const int tid = threadIdx.x, r = tid / ngrp, grp = tid - (tid / ngrp) * ngrp;
    const int b = blockIdx.y;
    const int64_t pb = (int64_t)blockIdx.x * chunk, pe = min((int64_t)HW, pb + chunk);
    float s[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) s[e] = 0.f;
    if (r < rows) {
        const T* xb = x + (int64_t)b * HW * xld + grp * VEC;
        const T* x2b = x2 ? x2 + (int64_t)b * HW * x2ld + grp * VEC : nullptr;
        for (int64_t p = pb + r; p < pe; p += rows) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(xb + p * xld);
            float f[VEC];
            if constexpr (VEC == 8) {
                const bf16x8 h = __builtin_bit_cast(bf16x8, v);
#pragma unroll
                for (int e = 0; e < 8; ++e) f[e] = (float)h[e];
            } else {
                const f32x4 h = __builtin_bit_cast(f32x4, v);
#pragma unroll
                for (int e = 0; e < 4; ++e) f[e] = h[e];
            }
            if (x2b) {
                const u32x4 v2 = *reinterpret_cast<const u32x4*>(x2b + p * x2ld);
                if constexpr (VEC == 8) {
                    const bf16x8 h = __builtin_bit_cast(bf16x8, v2);
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] *= (float)h[e];
                } else {
                    const f32x4 h = __builtin_bit_cast(f32x4, v2);
#pragma unroll
                    for (int e = 0; e < 4; ++e) f[e] *= h[e];
                }
            }
#pragma unroll
            for (int e = 0; e < VEC; ++e) s[e] += f[e];
        }
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) red[tid * VEC + e] = (r < rows) ? s[e] : 0.f;
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        const int g0 = c / VEC, e = c - g0 * VEC;
        float acc = 0.f;
        for (int rr = 0; rr < rows; ++rr) acc += red[(rr * ngrp + g0) * VEC + e];
        part[((int64_t)b * gridDim.x + blockIdx.x) * C + c] = acc;
    }
}
// stage 2: one wave per (b, c): the chunk partials, fixed xor tree
__global__ __launch_bounds__(256) void channel_mean_stage2(const float* __restrict__ part, int nchunk, int B, int C,
                                                           float* __restrict__ out, float scale) {
    const int lane = threadIdx.x & 63;
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= B * C) return;
    const int b = o / C, c = o - (o / C) * C;
    float s = 0.f;
    for (int i = lane; i < nchunk; i += 64) s += part[((int64_t)b * nchunk + i) * C + c];
    s = wave_sum(s);
    if (lane == 0) out[o] = s * scale;
}

static int mean_chunk(int B, int64_t HW) {
    const int64_t target = std::max(1, 1024 / B);                 // ~1024 stage-1 blocks in all
    return (int)std::max<int64_t>(256, (HW + target - 1) / target);
}

template <typename T>
__global__ void channel_affine_kernel(const T* __restrict__ x, int xld, const float* __restrict__ gamma,
                                      const float* __restrict__ beta, T* __restrict__ y, int yld, int B, int HW,
                                      int C, float beta_scale) {
    // y = gamma * x + beta * beta_scale (gamma may be NULL: y = beta * beta_scale broadcast)
    const int64_t total = (int64_t)B * HW * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const int64_t p = i / C;
        const int b = (int)(p / HW);
        float v = beta ? beta[(int64_t)b * C + c] * beta_scale : 0.f;
        if (gamma) v += gamma[(int64_t)b * C + c] * ldf(x, p * xld + c);
        y[p * yld + c] = from_f32<T>(v);
    }
}

static int grid256(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(16384, (n + 255) / 256)); }

// bf16 forms over 8-channel (16-byte) chunks, 32-bit index arithmetic once per chunk: the element-per-thread kernels
// above spend two 64-bit divisions and a 2-byte access per element (channel_affine on the multimodal aligner's 84 MB
// maps ran at ~2 TB/s).  Taken when C, the row pitches and the pointers allow 16-byte chunks.
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void st8(bf16* p, const bf16x8& v) { *reinterpret_cast<bf16x8*>(p) = v; }

__global__ void channel_affine_vec_kernel(const bf16* __restrict__ x, int xld, const float* __restrict__ gamma,
                                          const float* __restrict__ beta, bf16* __restrict__ y, int yld, int B, int HW,
                                          int C, float beta_scale) {
    const int cg = C >> 3;
    const int64_t total = (int64_t)B * HW * cg;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / cg;
        const int c = (int)(i - p * cg) * 8;
        const int b = (int)(p / HW);
        const bf16x8 xv = gamma ? ld8(x + p * xld + c) : bf16x8{};
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float v = beta ? beta[(int64_t)b * C + c + e] * beta_scale : 0.f;
            if (gamma) v += gamma[(int64_t)b * C + c + e] * (float)xv[e];
            o[e] = (bf16)v;
        }
        st8(y + p * yld + c, o);
    }
}

__global__ void gelu_fwd_vec_kernel(const bf16* __restrict__ x, int xld, bf16* __restrict__ y, int yld, int ntok, int C) {
    const int cg = C >> 3;
    const int64_t total = (int64_t)ntok * cg;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = i / cg;
        const int c = (int)(i - t * cg) * 8;
        const bf16x8 xv = ld8(x + t * xld + c);
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float v = (float)xv[e];
            o[e] = (bf16)(0.5f * v * (1.f + erff(v * 0.70710678118654752f)));
        }
        st8(y + t * yld + c, o);
    }
}

__global__ void gelu_bwd_vec_kernel(const bf16* __restrict__ x, int xld, const bf16* __restrict__ g, int gld,
                                    bf16* __restrict__ dx, int dxld, int ntok, int C) {
    const int cg = C >> 3;
    const int64_t total = (int64_t)ntok * cg;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = i / cg;
        const int c = (int)(i - t * cg) * 8;
        const bf16x8 xv = ld8(x + t * xld + c), gv = ld8(g + t * gld + c);
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float v = (float)xv[e];
            const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
            const float pdf = 0.3989422804014327f * __expf(-0.5f * v * v);
            o[e] = (bf16)((float)gv[e] * (cdf + v * pdf));
        }
        st8(dx + t * dxld + c, o);
    }
}

static bool vec8_ok(int C, std::initializer_list<int> lds, std::initializer_list<const void*> ptrs) {
    if (C % 8) return false;
    for (int l : lds)
        if (l % 8) return false;
    for (const void* q : ptrs)
        if (q && (reinterpret_cast<uintptr_t>(q) & 15)) return false;
    return true;
}

}  // namespace cai

using namespace cai;

#define DISPATCH_T(dtype, ...)                       \
    do {                                             \
        if ((dtype) == CAI_BF16) {                   \
            using T = bf16;                          \
            __VA_ARGS__;                             \
        } else {                                     \
            using T = float;                         \
            __VA_ARGS__;                             \
        }                                            \
    } while (0)

extern "C" {

int cai_layernorm_fwd(int dtype, const void* x, int32_t x_ld, int64_t ntok, int32_t C, const float* w, const float* b,
                      float eps, void* y, int32_t y_ld, float* mean, float* rstd, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "layernorm_fwd: bad dtype");
    CAI_CHECK_ARG(x && w && b && y && mean && rstd && C > 0 && C <= 1024 && x_ld >= C && y_ld >= C &&
                      ntok < (1ll << 31), "layernorm_fwd: bad arguments");
    if (ntok == 0) return CAI_OK;
    DISPATCH_T(dtype, hipLaunchKernelGGL(layernorm_fwd_kernel<T>, dim3((unsigned)((ntok + 3) / 4)), dim3(256), 0,
                                         as_stream(stream), (const T*)x, x_ld, (int)ntok, C, w, b, eps, (T*)y, y_ld,
                                         mean, rstd));
    CAI_LAUNCH_CHECK("layernorm_fwd");
    return CAI_OK;
}

// A/B knob CAI_LN_BWD_REG=0: the general LayerNorm backward for C <= 128 too
static bool layernorm_bwd_reg() {
    static const bool on = [] {
        const char* e = getenv("CAI_LN_BWD_REG");
        return !(e && *e == '0');
    }();
    return on;
}

size_t cai_layernorm_bwd_workspace_bytes(int64_t ntok, int32_t C) {
    const int64_t nblk = std::min<int64_t>(1024, (ntok + 63) / 64);
    return (size_t)std::max<int64_t>(nblk, 1) * 2 * C * sizeof(float);
}

int cai_layernorm_bwd(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t ntok, int32_t C,
                      const float* w, const float* mean, const float* rstd, void* dx, int32_t dx_ld, float* dw,
                      float* db, int32_t accumulate, void* workspace, size_t ws_bytes, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "layernorm_bwd: bad dtype");
    CAI_CHECK_ARG(x && dy && w && mean && rstd && dx && C > 0 && C <= 1024 && ntok < (1ll << 31),
                  "layernorm_bwd: bad arguments");
    CAI_CHECK_ARG(workspace && ws_bytes >= cai_layernorm_bwd_workspace_bytes(ntok, C), "layernorm_bwd: workspace");
    if (ntok == 0) return CAI_OK;
    const int nblk = (int)std::min<int64_t>(1024, (ntok + 63) / 64);
    const int per = (int)((ntok + nblk - 1) / nblk);
    float* part = reinterpret_cast<float*>(workspace);
    hipStream_t st = as_stream(stream);
    if (C <= 128 && layernorm_bwd_reg())
        DISPATCH_T(dtype, hipLaunchKernelGGL(layernorm_bwd_reg_kernel<T>, dim3(nblk), dim3(256), 4 * 2 * C * sizeof(float),
                                             st, (const T*)x, x_ld, (const T*)dy, dy_ld, (int)ntok, C, w, mean, rstd,
                                             (T*)dx, dx_ld, part, per));
    else
        DISPATCH_T(dtype, hipLaunchKernelGGL(layernorm_bwd_kernel<T>, dim3(nblk), dim3(256), 4 * 2 * C * sizeof(float),
                                             st, (const T*)x, x_ld, (const T*)dy, dy_ld, (int)ntok, C, w, mean, rstd,
                                             (T*)dx, dx_ld, part, per));
    if (dw || db)
        hipLaunchKernelGGL(layernorm_param_reduce, dim3((2 * C + LNR_COLS - 1) / LNR_COLS), dim3(LNR_COLS * LNR_GROUPS),
                           0, st, part, nblk, C, dw, db, accumulate);
    CAI_LAUNCH_CHECK("layernorm_bwd");
    return CAI_OK;
}

int cai_gelu_fwd(int dtype, const void* x, int32_t x_ld, void* y, int32_t y_ld, int64_t ntok, int32_t C, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "gelu_fwd: bad dtype");
    CAI_CHECK_ARG(x && y && x_ld >= C && y_ld >= C && ntok < (1ll << 31), "gelu_fwd: bad arguments");
    if (dtype == CAI_BF16 && vec8_ok(C, {x_ld, y_ld}, {x, y})) {
        hipLaunchKernelGGL(gelu_fwd_vec_kernel, dim3(grid256(ntok * C / 8)), dim3(256), 0, as_stream(stream),
                           (const bf16*)x, x_ld, (bf16*)y, y_ld, (int)ntok, C);
        CAI_LAUNCH_CHECK("gelu_fwd");
        return CAI_OK;
    }
    DISPATCH_T(dtype, hipLaunchKernelGGL(gelu_fwd_kernel<T>, dim3(grid256(ntok * C)), dim3(256), 0, as_stream(stream),
                                         (const T*)x, x_ld, (T*)y, y_ld, (int)ntok, C));
    CAI_LAUNCH_CHECK("gelu_fwd");
    return CAI_OK;
}

int cai_gelu_bwd(int dtype, const void* x, int32_t x_ld, const void* g, int32_t g_ld, void* dx, int32_t dx_ld,
                 int64_t ntok, int32_t C, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "gelu_bwd: bad dtype");
    CAI_CHECK_ARG(x && g && dx && ntok < (1ll << 31), "gelu_bwd: bad arguments");
    if (dtype == CAI_BF16 && vec8_ok(C, {x_ld, g_ld, dx_ld}, {x, g, dx})) {
        hipLaunchKernelGGL(gelu_bwd_vec_kernel, dim3(grid256(ntok * C / 8)), dim3(256), 0, as_stream(stream),
                           (const bf16*)x, x_ld, (const bf16*)g, g_ld, (bf16*)dx, dx_ld, (int)ntok, C);
        CAI_LAUNCH_CHECK("gelu_bwd");
        return CAI_OK;
    }
    DISPATCH_T(dtype, hipLaunchKernelGGL(gelu_bwd_kernel<T>, dim3(grid256(ntok * C)), dim3(256), 0, as_stream(stream),
                                         (const T*)x, x_ld, (const T*)g, g_ld, (T*)dx, dx_ld, (int)ntok, C));
    CAI_LAUNCH_CHECK("gelu_bwd");
    return CAI_OK;
}

static int check_attn(const cai_window_attn* p) {
    CAI_CHECK_ARG(p, "window_attn: null descriptor");
    CAI_CHECK_ARG(p->window == WS && p->head_dim == HD, "window_attn: only window 4 and head_dim 32 are built");
    CAI_CHECK_ARG(p->heads >= 1 && p->heads <= 8, "window_attn: 1..8 heads");
    CAI_CHECK_ARG(p->Hr % WS == 0 && p->Wr % WS == 0 && p->B > 0, "window_attn: resolution must be a multiple of 4");
    CAI_CHECK_ARG(p->shift >= 0 && p->shift < WS, "window_attn: bad shift");
    CAI_CHECK_ARG(p->q && p->kv && p->bias_table && p->rel_index, "window_attn: null pointer");
    return CAI_OK;
}

static AttnArgs attn_args(const cai_window_attn* p) {
    AttnArgs a{};
    a.q = p->q; a.q_ld = p->q_ld; a.kv = p->kv; a.kv_ld = p->kv_ld;
    a.bias_table = p->bias_table; a.rel_index = p->rel_index; a.mask = p->mask;
    a.B = p->B; a.Hr = p->Hr; a.Wr = p->Wr; a.heads = p->heads; a.shift = p->shift; a.scale = p->scale;
    return a;
}

static int attn_blocks(const cai_window_attn* p) {
    const int64_t items = (int64_t)p->B * (p->Hr / WS) * (p->Wr / WS) * p->heads;
    return (int)((items + 3) / 4);
}

int cai_window_attn_fwd(int dtype, const cai_window_attn* p, void* out, int32_t out_ld, void* stream) {
    int rc = check_attn(p);
    if (rc) return rc;
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "window_attn_fwd: bad dtype");
    CAI_CHECK_ARG(out, "window_attn_fwd: null output");
    AttnArgs a = attn_args(p);
    a.o = out; a.o_ld = out_ld;
    DISPATCH_T(dtype, hipLaunchKernelGGL(window_attn_fwd_kernel<T>, dim3(attn_blocks(p)), dim3(256), 0,
                                         as_stream(stream), a));
    CAI_LAUNCH_CHECK("window_attn_fwd");
    return CAI_OK;
}

size_t cai_window_attn_bwd_workspace_bytes(const cai_window_attn* p) {
    if (check_attn(p)) return 0;
    // per-block partials, ATTN_SPLITS split sums, the totals
    return ((size_t)attn_blocks(p) + ATTN_SPLITS + 1) * p->heads * WN * WN * sizeof(float);
}

int cai_window_attn_bwd(int dtype, const cai_window_attn* p, const void* dout, int32_t dout_ld, void* dq,
                        int32_t dq_ld, void* dkv, int32_t dkv_ld, float* dbias_table, int32_t accumulate,
                        void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_attn(p);
    if (rc) return rc;
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "window_attn_bwd: bad dtype");
    CAI_CHECK_ARG(dout && dq && dkv && dbias_table, "window_attn_bwd: null pointer");
    CAI_CHECK_ARG(workspace && ws_bytes >= cai_window_attn_bwd_workspace_bytes(p), "window_attn_bwd: workspace");
    AttnArgs a = attn_args(p);
    a.dout = dout; a.dout_ld = dout_ld; a.dq = dq; a.dq_ld = dq_ld; a.dkv = dkv; a.dkv_ld = dkv_ld;
    a.dbias_part = reinterpret_cast<float*>(workspace);
    const int nblk = attn_blocks(p);
    hipStream_t st = as_stream(stream);
    DISPATCH_T(dtype, hipLaunchKernelGGL(window_attn_bwd_kernel<T>, dim3(nblk), dim3(256), 0, st, a));
    const int rows = (2 * WS - 1) * (2 * WS - 1);
    const int E = p->heads * WN * WN;
    float* part2 = a.dbias_part + (int64_t)nblk * E;
    float* tot = part2 + (int64_t)ATTN_SPLITS * E;
    hipLaunchKernelGGL(attn_bias_sum_splits, dim3((E + 255) / 256, ATTN_SPLITS), dim3(256), 0, st, a.dbias_part, nblk,
                       E, part2);
    hipLaunchKernelGGL(attn_bias_sum_total, dim3((E + 255) / 256), dim3(256), 0, st, part2, E, tot);
    hipLaunchKernelGGL(attn_bias_grad_reduce, dim3((rows * p->heads + 63) / 64), dim3(64), 0, st, tot, p->heads,
                       p->rel_index, rows, dbias_table, accumulate);
    CAI_LAUNCH_CHECK("window_attn_bwd");
    return CAI_OK;
}

size_t cai_channel_mean_workspace_bytes(int32_t B, int64_t HW, int32_t C) {
    if (B <= 0 || HW <= 0 || C <= 0) return 0;
    const int64_t nchunk = (HW + mean_chunk(B, HW) - 1) / mean_chunk(B, HW);
    return (size_t)B * nchunk * C * sizeof(float);
}

int cai_channel_mean(int dtype, const void* x, int32_t x_ld, const void* x2, int32_t x2_ld, int32_t B, int64_t HW,
                     int32_t C, float* out, float scale, void* workspace, size_t ws_bytes, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "channel_mean: bad dtype");
    CAI_CHECK_ARG(x && out && B > 0 && HW > 0 && HW < (1ll << 31) && C > 0, "channel_mean: bad arguments");
    const int vec = dtype == CAI_BF16 ? 8 : 4;
    CAI_CHECK_ARG(C <= 256 * vec && x_ld % vec == 0 && ((uintptr_t)x & 15) == 0 &&
                      (!x2 || (x2_ld % vec == 0 && ((uintptr_t)x2 & 15) == 0)),
                  "channel_mean: operands must be 16-byte aligned with ld %% %d == 0 and C <= %d", vec, 256 * vec);
    CAI_CHECK_ARG(workspace && ws_bytes >= cai_channel_mean_workspace_bytes(B, HW, C),
                  "channel_mean: workspace of %zu bytes required", cai_channel_mean_workspace_bytes(B, HW, C));
    const int chunk = mean_chunk(B, HW);
    const int nchunk = (int)((HW + chunk - 1) / chunk);
    float* part = reinterpret_cast<float*>(workspace);
    hipStream_t st = as_stream(stream);
    DISPATCH_T(dtype, hipLaunchKernelGGL(channel_mean_stage1<T>, dim3(nchunk, B), dim3(256), 0, st, (const T*)x, x_ld,
                                         (const T*)x2, x2_ld, (int)HW, C, chunk, part));
    hipLaunchKernelGGL(channel_mean_stage2, dim3((B * C + 3) / 4), dim3(256), 0, st, part, nchunk, B, C, out, scale);
    CAI_LAUNCH_CHECK("channel_mean");
    return CAI_OK;
}

int cai_channel_affine(int dtype, const void* x, int32_t x_ld, const float* gamma, const float* beta, float beta_scale,
                       void* y, int32_t y_ld, int32_t B, int64_t HW, int32_t C, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "channel_affine: bad dtype");
    CAI_CHECK_ARG(y && B > 0 && HW > 0 && C > 0 && (!gamma || x), "channel_affine: bad arguments");
    if (dtype == CAI_BF16 && vec8_ok(C, {gamma ? x_ld : 8, y_ld}, {gamma ? x : nullptr, y})) {
        hipLaunchKernelGGL(channel_affine_vec_kernel, dim3(grid256((int64_t)B * HW * C / 8)), dim3(256), 0,
                           as_stream(stream), (const bf16*)x, x_ld, gamma, beta, (bf16*)y, y_ld, B, (int)HW, C,
                           beta_scale);
        CAI_LAUNCH_CHECK("channel_affine");
        return CAI_OK;
    }
    DISPATCH_T(dtype, hipLaunchKernelGGL(channel_affine_kernel<T>, dim3(grid256((int64_t)B * HW * C)), dim3(256), 0,
                                         as_stream(stream), (const T*)x, x_ld, gamma, beta, (T*)y, y_ld, B, (int)HW,
                                         C, beta_scale));
    CAI_LAUNCH_CHECK("channel_affine");
    return CAI_OK;
}

}  // extern "C"
