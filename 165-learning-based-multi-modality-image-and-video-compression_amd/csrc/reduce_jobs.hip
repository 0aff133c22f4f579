// Parameter-gradient reduces as jobs (cai_reduce_jobs): the fixed-order sums that turn a weight-gradient
// kernel's per-split fp32 slabs (conv) or per-block partials (fused GDN backward) into the torch-layout
// gradient.  One kernel runs any list of jobs -- each job owns a contiguous range of 256-thread blocks -- so
// the reduces of a whole backward pass can go out as ONE launch before the optimizer reads the gradients,
// instead of one launch after every layer (the per-layer launches were 14 of the 100 kernels of a C2 step).
// The immediate paths (cai_conv_wgrad, cai_gdn_backward) run their single job through the same kernel, so
// deferred and immediate reduces are bit-identical.
//
// Job bodies (the order and arithmetic of every sum is fixed: deterministic):
//   WGRAD  one block per output row n of the [Ng][ncols] slab: each 16-byte column chunk summed over the S
//          splits in split order (loads in batches of 8), the row transposed through LDS from [tap][q] to the
//          torch layout dw[n][q][tap] and stored contiguously (rows wider than 8192 columns: one thread per
//          chunk, scattered stores); trailing blocks: the bias partials [Sb][nbias] -> db, one thread per channel
//   EDGE   the image-side layers' weight gradient (edge.hip): unit partials summed in unit order, scattered
//          into dW / db (and the image-side column sums)
//   GDN    16 element columns x 16 partial-block groups per block (4 consecutive elements per thread), the
//          groups combined through LDS in a fixed tree, then the NonNegativeParametrizer / LowerBound backward
//          rule (ops/parametrizers.py:47-64, ops/bound_ops.py:36-80) into dgamma_raw / dbeta_raw
#include "common.hpp"
#include "reduce_jobs.hpp"

namespace cai {

// rows of the weight-gradient slab small enough to transpose through LDS (floats)
constexpr int WG_ROW_LDS = 8192;

__device__ __forceinline__ void wgrad_bias_body(const cai_reduce_job& J, int bid) {
    const float* __restrict__ bws = static_cast<const float*>(J.p[2]);
    float* __restrict__ db = static_cast<float*>(const_cast<void*>(J.p[3]));
    const int accumulate = J.i[6], Sb = J.i[7], nbias = J.i[8];
    const int n = bid * 256 + threadIdx.x;
    if (n >= nbias) return;
    float v = 0.f;
    int sp = 0;
    for (; sp + 8 <= Sb; sp += 8) {
        float b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = bws[(int64_t)(sp + j) * nbias + n];
#pragma unroll
        for (int j = 0; j < 8; ++j) v += b[j];
    }
    for (; sp < Sb; ++sp) v += bws[(int64_t)sp * nbias + n];
    db[n] = accumulate ? db[n] + v : v;
}

// one output row n per block: the row's ncols = k*k*Cq_pad columns (slab layout [tap][q]) summed over the S
// splits in split order (16-byte loads, 8 splits in flight), transposed through LDS and written to dw[n][q][tap]
// (the torch layout is contiguous over (q, tap) for a fixed n): coalesced read-modify-write stores instead of
// one 4-byte access per k*k-strided element
__device__ __forceinline__ void wgrad_row_body(const cai_reduce_job& J, int n, float* row) {
    const float* __restrict__ ws = static_cast<const float*>(J.p[0]);
    float* __restrict__ dw = static_cast<float*>(const_cast<void*>(J.p[1]));
    const int S = J.i[0], Ng = J.i[1], ncols = J.i[2], Cq = J.i[3], Cq_pad = J.i[4], k = J.i[5];
    const int accumulate = J.i[6];
    const int c4 = ncols >> 2;
    const int64_t slab4 = ((int64_t)Ng * ncols) >> 2;
    const f32x4* src = reinterpret_cast<const f32x4*>(ws) + (int64_t)n * c4;
    // RC column chunks per thread at once, RB splits per batch: RC * RB loads in flight per thread (one chunk at
    // a time left a thread waiting S / 8 + 1 round trips per chunk).  Every chunk still sums its splits in split
    // order: the same floats as one chunk at a time.
    constexpr int RC = 4, RB = 4;
    for (int cb = threadIdx.x; cb < c4; cb += 256 * RC) {
        bool ok[RC];
        f32x4 acc[RC];
#pragma unroll
        for (int q = 0; q < RC; ++q) {
            ok[q] = cb + 256 * q < c4;
            acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        int sp = 0;
        for (; sp + RB <= S; sp += RB) {
            f32x4 v[RB][RC];
#pragma unroll
            for (int j = 0; j < RB; ++j)
#pragma unroll
                for (int q = 0; q < RC; ++q)
                    v[j][q] = ok[q] ? src[(int64_t)(sp + j) * slab4 + cb + 256 * q] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < RB; ++j)
#pragma unroll
                for (int q = 0; q < RC; ++q) acc[q] += v[j][q];
        }
        for (; sp < S; ++sp)
#pragma unroll
            for (int q = 0; q < RC; ++q)
                if (ok[q]) acc[q] += src[(int64_t)sp * slab4 + cb + 256 * q];
#pragma unroll
        for (int q = 0; q < RC; ++q)
            if (ok[q]) *reinterpret_cast<f32x4*>(row + 4 * (cb + 256 * q)) = acc[q];
    }
    __syncthreads();
    const int kk = k * k, nout = Cq * kk;
    float* d = dw + (int64_t)n * nout;
    for (int i = threadIdx.x; i < nout; i += 256) {
        const int q = i / kk, t = i - (i / kk) * kk;
        const float v = row[t * Cq_pad + q];
        d[i] = accumulate ? d[i] + v : v;
    }
}

// the same sums for rows too wide for LDS: one thread per 16-byte column chunk, scattered 4-byte stores
__device__ __forceinline__ void wgrad_scatter_body(const cai_reduce_job& J, int bid) {
    const float* __restrict__ ws = static_cast<const float*>(J.p[0]);
    float* __restrict__ dw = static_cast<float*>(const_cast<void*>(J.p[1]));
    const int S = J.i[0], Ng = J.i[1], ncols = J.i[2], Cq = J.i[3], Cq_pad = J.i[4], k = J.i[5];
    const int accumulate = J.i[6];
    const int c4 = ncols >> 2;
    const int64_t total = (int64_t)Ng * c4;
    const int64_t i = (int64_t)bid * 256 + threadIdx.x;
    if (i >= total) return;
    const int64_t slab4 = ((int64_t)Ng * ncols) >> 2;
    const f32x4* src = reinterpret_cast<const f32x4*>(ws) + i;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    int sp = 0;
    for (; sp + 8 <= S; sp += 8) {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = src[(int64_t)(sp + j) * slab4];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += v[j];
    }
    for (; sp < S; ++sp) acc += src[(int64_t)sp * slab4];
    const int n = (int)(i / c4);
    const int col = (int)(i - (int64_t)n * c4) * 4;
    const int kk = k * k;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int cc = col + e;
        const int t = cc / Cq_pad, q = cc - (cc / Cq_pad) * Cq_pad;
        if (q >= Cq) continue;
        float* d = dw + ((int64_t)n * Cq + q) * kk + t;
        *d = accumulate ? *d + acc[e] : acc[e];
    }
}

// blocks [0, wblocks): the weight rows (LDS-transposed: one row per block; else scattered chunks); then the
// bias blocks
__device__ __forceinline__ void wgrad_reduce_body(const cai_reduce_job& J, int bid, float* row) {
    const int Ng = J.i[1], ncols = J.i[2];
    const bool lds = ncols <= WG_ROW_LDS;
    const int wblocks = lds ? Ng : (int)(((int64_t)Ng * (ncols >> 2) + 255) / 256);
    if (bid >= wblocks) {
        wgrad_bias_body(J, bid - wblocks);
        return;
    }
    if (lds)
        wgrad_row_body(J, bid, row);
    else
        wgrad_scatter_body(J, bid);
}

int wgrad_job_blocks(int Ng, int ncols, int nbias_blocks) {
    const int wblocks = ncols <= WG_ROW_LDS ? Ng : (int)(((int64_t)Ng * (ncols >> 2) + 255) / 256);
    return wblocks + nbias_blocks;
}

__device__ __forceinline__ void gdn_reduce_body(const cai_reduce_job& J, int bid, f32x4 (*red)[17]) {
    const float* __restrict__ part = static_cast<const float*>(J.p[0]);
    const float* __restrict__ beta_raw = static_cast<const float*>(J.p[1]);
    const float* __restrict__ gamma_raw = static_cast<const float*>(J.p[2]);
    float* __restrict__ dbeta_raw = static_cast<float*>(const_cast<void*>(J.p[3]));
    float* __restrict__ dgamma_raw = static_cast<float*>(const_cast<void*>(J.p[4]));
    const int nblk = J.i[0], C = J.i[1], accumulate = J.i[2];
    const float bbound = J.f[0], gbound = J.f[1];
    const int64_t CC = (int64_t)C * C, stride = CC + C;
    const int cg = threadIdx.x & 15, bg = threadIdx.x >> 4;
    const int64_t i0 = ((int64_t)bid * 16 + cg) * 4;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (i0 < stride) {
        int b = bg;
        for (; b + 16 * 7 < nblk; b += 16 * 8) {
            f32x4 t[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) t[j] = *reinterpret_cast<const f32x4*>(part + (int64_t)(b + 16 * j) * stride + i0);
#pragma unroll
            for (int j = 0; j < 8; ++j) v += t[j];
        }
        for (; b < nblk; b += 16) v += *reinterpret_cast<const f32x4*>(part + (int64_t)b * stride + i0);
    }
    red[bg][cg] = v;
    __syncthreads();
    if (bg != 0 || i0 >= stride) return;
#pragma unroll
    for (int j = 1; j < 16; ++j) v += red[j][cg];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int64_t i = i0 + e;
        if (i < CC) {
            const float gr = gamma_raw[i];
            const float d = 2.f * fmaxf(gr, gbound) * v[e];
            const float vg = (gr >= gbound || d < 0.f) ? d : 0.f;
            dgamma_raw[i] = accumulate ? dgamma_raw[i] + vg : vg;
        } else if (i < stride) {
            const int64_t c = i - CC;
            const float br = beta_raw[c];
            const float db = 2.f * fmaxf(br, bbound) * v[e];
            const float vb = (br >= bbound || db < 0.f) ? db : 0.f;
            dbeta_raw[c] = accumulate ? dbeta_raw[c] + vb : vb;
        }
    }
}

// EDGE: the image-side layers' weight gradient (edge.hip): unit partials [units][9*16*N + 16] summed in unit
// order (16 outputs x 16 unit groups per block, groups combined through LDS), scattered into the torch layout
// of dW / db; the 16 image-side column sums come from cs_src[count][stride]
constexpr int EDGE_ONES = 12;   // edge.hip's constant-1 superpixel channel
__device__ __forceinline__ void edge_reduce_body(const cai_reduce_job& J, int bid, float (*red)[16], float* tot) {
    const float* __restrict__ part = static_cast<const float*>(J.p[0]);
    const float* __restrict__ cs_src = static_cast<const float*>(J.p[1]);
    float* __restrict__ dw = static_cast<float*>(const_cast<void*>(J.p[2]));
    float* __restrict__ db = static_cast<float*>(const_cast<void*>(J.p[3]));
    const int N = J.i[0], units = J.i[1], mode = J.i[2], k = J.i[3], pad = J.i[4], C = J.i[5];
    const int cs_count = J.i[6], cs_stride = J.i[7], accumulate = J.i[8];
    const int G = 9 * 16 * N, O = G + 16;
    const int l = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int o = bid * 16 + l;
    const float* src;
    int cnt;
    int64_t stride;
    if (o < G) {
        src = part + o;
        cnt = units;
        stride = O;
    } else {
        src = cs_src + (o - G);
        cnt = cs_count;
        stride = cs_stride;
    }
    float s = 0.f;
    int u = grp;
    for (; u + 16 * 7 < cnt; u += 16 * 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = src[(int64_t)(u + 16 * i) * stride];
#pragma unroll
        for (int i = 0; i < 8; ++i) s += v[i];
    }
    for (; u < cnt; u += 16) s += src[(int64_t)u * stride];
    red[grp][l] = s;
    __syncthreads();
    if (grp == 0) {
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) v += red[i][l];
        tot[l] = v;
    }
    __syncthreads();
    if (grp != 0) return;
    s = tot[l];
    if (o >= G) {   // G is a multiple of 16: this block holds exactly the 16 column sums
        const int co = o - G;
        if (mode == 1 && db && co < C) {
            float v = 0.f;
#pragma unroll
            for (int sp = 0; sp < 4; ++sp) v += tot[sp * C + co];
            db[co] = accumulate ? db[co] + v : v;
        }
        return;
    }
    const int nn = o % N, tc = o / N, t = tc / 16, chn = tc % 16;
    int dst = -1;
    if (mode == 0) {
        if (chn == EDGE_ONES) {
            if (t == 4 && db) db[nn] = accumulate ? db[nn] + s : s;
            return;
        }
        if (chn >= 4 * C) return;
        const int sp = chn / C, ci = chn - sp * C;
        const int ky = 2 * (t / 3 - 1) + (sp >> 1) + pad, kx = 2 * (t % 3 - 1) + (sp & 1) + pad;
        if (ky >= 0 && ky < k && kx >= 0 && kx < k) dst = ((nn * C + ci) * k + ky) * k + kx;
    } else {
        if (chn >= 4 * C) return;
        const int sp = chn / C, co = chn - sp * C, tf = 8 - t;
        const int ky = (sp >> 1) - 2 * (tf / 3 - 1) + pad, kx = (sp & 1) - 2 * (tf % 3 - 1) + pad;
        if (ky >= 0 && ky < k && kx >= 0 && kx < k) dst = ((nn * C + co) * k + ky) * k + kx;
    }
    if (dst >= 0) dw[dst] = accumulate ? dw[dst] + s : s;
}

__global__ __launch_bounds__(256) void reduce_jobs_kernel(const ReduceBatch B) {
    __shared__ f32x4 red[16][17];
    __shared__ __attribute__((aligned(16))) float row[WG_ROW_LDS];
    __shared__ float ered[16][16];
    __shared__ float etot[16];
    // the job owning this block (block-uniform linear scan over <= CAI_REDUCE_BATCH entries)
    const int b = blockIdx.x;
    int j = 0;
    while (j + 1 < B.n && b >= B.start[j + 1]) ++j;
    const cai_reduce_job& J = B.jobs[j];
    const int bid = b - B.start[j];
    if (J.kind == CAI_JOB_WGRAD)
        wgrad_reduce_body(J, bid, row);
    else if (J.kind == CAI_JOB_GDN)
        gdn_reduce_body(J, bid, red);
    else if (J.kind == CAI_JOB_EDGE)
        edge_reduce_body(J, bid, ered, etot);
}

int launch_reduce_jobs(const cai_reduce_job* jobs, int n, hipStream_t st) {
    for (int j0 = 0; j0 < n;) {
        ReduceBatch B{};
        int blocks = 0;
        for (; j0 < n && B.n < CAI_REDUCE_BATCH; ++j0) {
            const cai_reduce_job& J = jobs[j0];
            if (J.kind == CAI_JOB_NONE || J.nblocks <= 0) continue;
            CAI_CHECK_ARG(J.kind == CAI_JOB_WGRAD || J.kind == CAI_JOB_GDN || J.kind == CAI_JOB_EDGE,
                          "reduce_jobs: unknown job kind %d", J.kind);
            B.jobs[B.n] = J;
            B.start[B.n] = blocks;
            blocks += J.nblocks;
            ++B.n;
        }
        if (B.n == 0) continue;
        hipLaunchKernelGGL(reduce_jobs_kernel, dim3((unsigned)blocks), dim3(256), 0, st, B);
        CAI_LAUNCH_CHECK("reduce_jobs");
    }
    return CAI_OK;
}

}  // namespace cai

extern "C" int cai_reduce_jobs(const cai_reduce_job* jobs, int32_t n, void* stream) {
    CAI_CHECK_ARG(n >= 0 && (n == 0 || jobs), "reduce_jobs: bad arguments");
    return cai::launch_reduce_jobs(jobs, n, cai::as_stream(stream));
}
