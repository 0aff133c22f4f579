// Parameter-gradient reduces as jobs (cai_reduce_jobs): the fixed-order sums that turn a weight-gradient
// kernel's per-split fp32 slabs (conv) or per-block partials (fused GDN backward) into the torch-layout
// gradient.  One kernel runs any list of jobs -- each job owns a contiguous range of 256-thread blocks -- so
// the reduces of a whole backward pass can go out as ONE launch before the optimizer reads the gradients,
// instead of one launch after every layer (the per-layer launches were 14 of the 100 kernels of a C2 step).
// The immediate paths (cai_conv_wgrad, cai_gdn_backward) run their single job through the same kernel, so
// deferred and immediate reduces are bit-identical.
//
// Job bodies (the order and arithmetic of every sum is fixed: deterministic):
//   WGRAD  one block per (output row n, slice of input channels) of the [Ng][ncols] slab: each 16-byte column
//          chunk summed over the S splits in split order (loads in batches of 8), the slice transposed through
//          LDS from [tap][q] to the torch layout dw[n][q][tap] and stored contiguously; trailing blocks: the
//          bias partials [Sb][nbias] -> db, one thread per channel
//   EDGE   the image-side layers' weight gradient (edge.hip): unit partials summed in unit order, scattered
//          into dW / db (and the image-side column sums)
//   GDN    16 element columns x 16 partial-block groups per block (4 consecutive elements per thread), the
//          groups combined through LDS in a fixed tree, then the NonNegativeParametrizer / LowerBound backward
//          rule (ops/parametrizers.py:47-64, ops/bound_ops.py:36-80) into dgamma_raw / dbeta_raw
#include "common.hpp"
#include "reduce_jobs.hpp"

namespace cai {

// WGRAD job layout: one block per (rpb output rows n .. n + rpb - 1, slice of input channels q).  The slab row of n
// is [tap][Cq_pad] (16-byte chunks of 4 channels); a block takes q4 chunks of every tap of each of its rows
// (rpb * q4 * k*k <= 256 threads, one chunk per thread), sums them over the S splits in split order (loads in
// batches of 16), transposes the slice through LDS from [tap][q] to the torch layout dw[n][q][tap] and writes it
// -- contiguous runs of the torch layout.  (One block per whole row kept 129-193 blocks per job: ~20 us per C2
// halo layer on its own, the batched launch load-imbalanced; power-of-two slices left 44 % of a 3x3 block's
// threads and most of a 1x1 block's idle.)
__host__ __device__ __forceinline__ void wg_shape(int kk, int cq4, int& q4, int& rpb) {
    int qmax = 256 / kk;
    if (qmax < 1) qmax = 1;
    const int nsl = (cq4 + qmax - 1) / qmax;
    q4 = (cq4 + nsl - 1) / nsl;   // equal slices: 5x5 at 128 channels 8 + 8 + 8 + 8, not 10 + 10 + 10 + 2
    rpb = 256 / (q4 * kk);
    if (rpb < 1) rpb = 1;
}
constexpr int WG_TR_FLOATS = 2048;   // rpb * 4 * q4 * (kk + 1) <= 4 * (256 + 256)

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

__device__ __forceinline__ void wgrad_slice_body(const cai_reduce_job& J, int bid, float* tr) {
    const float* __restrict__ ws = static_cast<const float*>(J.p[0]);
    float* __restrict__ dw = static_cast<float*>(const_cast<void*>(J.p[1]));
    const int S = J.i[0], Ng = J.i[1], ncols = J.i[2], Cq = J.i[3], Cq_pad = J.i[4], k = J.i[5];
    const int accumulate = J.i[6];
    const int kk = k * k, cq4 = Cq_pad >> 2, c4 = ncols >> 2;
    int q4, rpb;
    wg_shape(kk, cq4, q4, rpb);
    const int nsl = (cq4 + q4 - 1) / q4;
    const int nb = bid / nsl, c0 = (bid - nb * nsl) * q4, n0 = nb * rpb;
    const int per = q4 * kk, r = threadIdx.x / per, rem = threadIdx.x - r * per;
    const int t = rem / q4, j = rem - t * q4, c = c0 + j, n = n0 + r;
    const bool active = r < rpb && n < Ng && c < cq4;
    const int64_t slab4 = ((int64_t)Ng * ncols) >> 2;
    const int rpitch = 4 * q4 * (kk + 1);
    if (active) {
        const f32x4* src = reinterpret_cast<const f32x4*>(ws) + (int64_t)n * c4 + t * cq4 + c;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        int sp = 0;
        for (; sp + 16 <= S; sp += 16) {
            f32x4 v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = src[(int64_t)(sp + i) * slab4];
#pragma unroll
            for (int i = 0; i < 16; ++i) acc += v[i];
        }
        for (; sp + 4 <= S; sp += 4) {
            f32x4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = src[(int64_t)(sp + i) * slab4];
#pragma unroll
            for (int i = 0; i < 4; ++i) acc += v[i];
        }
        for (; sp < S; ++sp) acc += src[(int64_t)sp * slab4];
#pragma unroll
        for (int e = 0; e < 4; ++e) tr[r * rpitch + (4 * j + e) * (kk + 1) + t] = acc[e];
    }
    __syncthreads();
    const int qa = 4 * c0, qb = min(Cq, 4 * (c0 + q4));
    const int len = (qb - qa) * kk;
    const int rows = min(rpb, Ng - n0);
    for (int i = threadIdx.x; i < rows * len; i += 256) {
        const int rr = i / len, ii = i - rr * len;
        const int ql = ii / kk, tt = ii - ql * kk;
        const float v = tr[rr * rpitch + ql * (kk + 1) + tt];
        float* d = dw + ((int64_t)(n0 + rr) * Cq + qa) * kk + ii;
        *d = accumulate ? *d + v : v;
    }
}

// blocks [0, wblocks): the (rows, channel-slice) weight blocks; then the bias blocks
__device__ __forceinline__ void wgrad_reduce_body(const cai_reduce_job& J, int bid, float* tr) {
    const int Ng = J.i[1], Cq_pad = J.i[4], k = J.i[5];
    int q4, rpb;
    wg_shape(k * k, Cq_pad >> 2, q4, rpb);
    const int wblocks = (Ng + rpb - 1) / rpb * ((Cq_pad / 4 + q4 - 1) / q4);
    if (bid >= wblocks) {
        wgrad_bias_body(J, bid - wblocks);
        return;
    }
    wgrad_slice_body(J, bid, tr);
}

int wgrad_job_blocks(int Ng, int Cq_pad, int k, int nbias_blocks) {
    int q4, rpb;
    wg_shape(k * k, Cq_pad >> 2, q4, rpb);
    return (Ng + rpb - 1) / rpb * ((Cq_pad / 4 + q4 - 1) / q4) + nbias_blocks;
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

__device__ __forceinline__ void reduce_block(const ReduceBatch& B, int b, int& j, f32x4 (*red)[17], float* tr,
                                             float (*ered)[16], float* etot) {
    // the job owning block b (block-uniform linear scan over <= CAI_REDUCE_BATCH entries, from job j on)
    while (j + 1 < B.n && b >= B.start[j + 1]) ++j;
    const cai_reduce_job& J = B.jobs[j];
    const int bid = b - B.start[j];
    if (J.kind == CAI_JOB_WGRAD)
        wgrad_reduce_body(J, bid, tr);
    else if (J.kind == CAI_JOB_GDN)
        gdn_reduce_body(J, bid, red);
    else if (J.kind == CAI_JOB_EDGE)
        edge_reduce_body(J, bid, ered, etot);
}

// LOOP: a capped grid walks the batch's blocks in order (cai_reduce_jobs_grid: a reduce that runs beside other
// work on a side stream holds at most that many CUs' worth of blocks); each block's arithmetic is the same
template <bool LOOP>
__global__ __launch_bounds__(256) void reduce_jobs_kernel(const ReduceBatch B) {
    __shared__ f32x4 red[16][17];
    __shared__ __attribute__((aligned(16))) float tr[WG_TR_FLOATS];
    __shared__ float ered[16][16];
    __shared__ float etot[16];
    int j = 0;
    if constexpr (!LOOP) {
        reduce_block(B, (int)blockIdx.x, j, red, tr, ered, etot);
    } else {
        for (int b = (int)blockIdx.x; b < B.total; b += (int)gridDim.x) {
            __syncthreads();    // the previous block's LDS readers are done
            reduce_block(B, b, j, red, tr, ered, etot);
        }
    }
}

// The gradient buffers a job writes (read-modify-write when it accumulates).
static inline void job_dests(const cai_reduce_job& J, const void* d[2]) {
    d[0] = d[1] = nullptr;
    if (J.kind == CAI_JOB_WGRAD) {
        d[0] = J.p[1];
        d[1] = J.p[3];
    } else if (J.kind == CAI_JOB_GDN) {
        d[0] = J.p[3];
        d[1] = J.p[4];
    } else if (J.kind == CAI_JOB_EDGE) {
        d[0] = J.p[2];
        d[1] = J.p[3];
    }
}

static bool shares_dest(const ReduceBatch& B, const cai_reduce_job& J) {
    const void* a[2];
    job_dests(J, a);
    for (int q = 0; q < B.n; ++q) {
        const void* b[2];
        job_dests(B.jobs[q], b);
        for (int u = 0; u < 2; ++u)
            for (int v = 0; v < 2; ++v)
                if (a[u] && a[u] == b[v]) return true;
    }
    return false;
}

// Jobs run in list order across launches; within one launch their blocks run concurrently, so two jobs that
// write the same gradient (a module called twice in one forward, e.g. Channel_aligner's shared trunk,
// models/master.py:293-304: the second job accumulates onto the first) never share a launch -- the batch is
// closed before the second and it runs in the next launch, after the first on the stream.
int launch_reduce_jobs(const cai_reduce_job* jobs, int n, hipStream_t st, int max_grid) {
    for (int j0 = 0; j0 < n;) {
        ReduceBatch B{};
        int blocks = 0;
        for (; j0 < n && B.n < CAI_REDUCE_BATCH; ++j0) {
            const cai_reduce_job& J = jobs[j0];
            if (J.kind == CAI_JOB_NONE || J.nblocks <= 0) continue;
            CAI_CHECK_ARG(J.kind == CAI_JOB_WGRAD || J.kind == CAI_JOB_GDN || J.kind == CAI_JOB_EDGE,
                          "reduce_jobs: unknown job kind %d", J.kind);
            if (shares_dest(B, J)) break;
            B.jobs[B.n] = J;
            B.start[B.n] = blocks;
            blocks += J.nblocks;
            ++B.n;
        }
        if (B.n == 0) continue;
        B.total = blocks;
        if (max_grid > 0 && blocks > max_grid)
            hipLaunchKernelGGL(reduce_jobs_kernel<true>, dim3((unsigned)max_grid), dim3(256), 0, st, B);
        else
            hipLaunchKernelGGL(reduce_jobs_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, B);
        CAI_LAUNCH_CHECK("reduce_jobs");
    }
    return CAI_OK;
}

}  // namespace cai

extern "C" int cai_reduce_jobs(const cai_reduce_job* jobs, int32_t n, void* stream) {
    CAI_CHECK_ARG(n >= 0 && (n == 0 || jobs), "reduce_jobs: bad arguments");
    return cai::launch_reduce_jobs(jobs, n, cai::as_stream(stream), 0);
}

extern "C" int cai_reduce_jobs_grid(const cai_reduce_job* jobs, int32_t n, int32_t max_blocks, void* stream) {
    CAI_CHECK_ARG(n >= 0 && (n == 0 || jobs) && max_blocks >= 0, "reduce_jobs_grid: bad arguments");
    return cai::launch_reduce_jobs(jobs, n, cai::as_stream(stream), max_blocks);
}
