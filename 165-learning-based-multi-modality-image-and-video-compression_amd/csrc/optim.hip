// Optimiser step over flat fp32 buffers + library misc (errors, version).
//
// Adam follows torch.optim.Adam (no weight decay, no amsgrad), as used by
// examples/train.py:134-141:  m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ;
// p -= (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps).
// clip_grad_norm_(max_norm) (train.py:178) is folded in: the kernel scales g
// by min(1, max_norm/(||g|| + 1e-6)) read from the device-side squared norm,
// so the whole step stays on the stream (graph-capturable, no host sync).
// A non-finite squared norm skips the whole update, step counter included:
// what GradScaler.step does when unscale_ found inf/NaN gradients
// (train.py:176-179).
#include "common.hpp"

#include <stdarg.h>

namespace cai {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                            const float* __restrict__ step, const float* __restrict__ sqnorm, float max_norm) {
    // *step holds the number of steps already taken; this step is t = *step + 1
    if (sqnorm && !isfinite(*sqnorm)) return;
    const float t = *step + 1.f;
    const float bc1 = 1.f - powf(b1, t);
    const float bc2s = sqrtf(1.f - powf(b2, t));
    const float step_size = lr / bc1;
    float scale = 1.f;
    if (sqnorm) {
        const float coef = max_norm / (sqrtf(*sqnorm) + 1e-6f);
        scale = coef < 1.f ? coef : 1.f;
    }
    const int64_t n4 = n / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
        f32x4 gv = reinterpret_cast<const f32x4*>(g)[i] * scale;
        f32x4 mv = reinterpret_cast<f32x4*>(m)[i];
        f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
        f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            mv[e] = b1 * mv[e] + (1.f - b1) * gv[e];
            vv[e] = b2 * vv[e] + (1.f - b2) * gv[e] * gv[e];
            pv[e] -= step_size * mv[e] / (sqrtf(vv[e]) / bc2s + eps);
        }
        reinterpret_cast<f32x4*>(m)[i] = mv;
        reinterpret_cast<f32x4*>(v)[i] = vv;
        reinterpret_cast<f32x4*>(p)[i] = pv;
    }
    for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const float gv = g[i] * scale;
        m[i] = b1 * m[i] + (1.f - b1) * gv;
        v[i] = b2 * v[i] + (1.f - b2) * gv * gv;
        p[i] -= step_size * m[i] / (sqrtf(v[i]) / bc2s + eps);
    }
}

__global__ void step_incr_kernel(float* step, const float* __restrict__ sqnorm) {
    if (sqnorm && !isfinite(*sqnorm)) return;
    *step += 1.f;
}

// ---------------------------------------------------------------------------
// cai_adam_step: the whole clip + Adam step in two launches (one for small buffers) instead of four
// (sqnorm stage 1, stage 2, Adam, step increment): each launch past the first costs a kernel boundary.
//   large n:  sq_part_kernel  -- per-block partial sums of g^2 (as cai_sqnorm's stage 1); block 0 also
//                                counts the step (t = step + 1)
//             adam_fused_kernel -- every block reduces the partials itself, in cai_sqnorm's stage-2 order
//                                (the same float in every block), then clips and updates; a non-finite
//                                norm makes every block return and block 0 take the count back
//   small n:  adam_small_kernel -- one block: norm, finiteness, update, step count
// ---------------------------------------------------------------------------
constexpr int ADAM_SMALL_N = 1 << 16;
constexpr int SQ_PART_MAX = 1024;

static int sq_parts(int64_t n) {
    int64_t b = (n + 1023) / 1024;
    if (b > SQ_PART_MAX) b = SQ_PART_MAX;
    return b < 1 ? 1 : (int)b;
}

__global__ __launch_bounds__(256) void sq_part_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part,
                                                      float* __restrict__ step) {
    __shared__ float red[4];
    // 16-byte loads, U of them in flight per thread (the one-float loop ran at ~1.9 TB/s on C4's 26M gradients)
    constexpr int U = 4;
    const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * 256;
    f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
    for (int64_t ib = blockIdx.x * 256 + threadIdx.x; ib < n4; ib += U * stride) {
        f32x4 gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * stride;
            gv[u] = i < n4 ? reinterpret_cast<const f32x4*>(g)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) a4 += gv[u] * gv[u];
    }
    float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += stride) acc += g[i] * g[i];
    const float r = block_sum<256>(acc, red);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = r;
        if (blockIdx.x == 0) *step += 1.f;
    }
}

// zero_g: the gradient buffer is consumed -- each element is overwritten with 0 once read (CAI_ADAM_ZERO_GRAD:
// the next backward then needs no zero-fill launch)
__device__ __forceinline__ void zero_range(float* __restrict__ g, int64_t n, int64_t i0, int64_t stride) {
    const int64_t n4 = n / 4;
    for (int64_t i = i0; i < n4; i += stride) reinterpret_cast<f32x4*>(g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int64_t i = n4 * 4 + i0; i < n; i += stride) g[i] = 0.f;
}

__device__ __forceinline__ void adam_range(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                           float* __restrict__ v, int64_t n, int64_t i0, int64_t stride, float scale,
                                           float b1, float b2, float eps, float step_size, float bc2s, bool zero_g) {
    const int64_t n4 = n / 4;
    // U chunks per thread and round, all loaded before any store: a load issued behind a store waits for it (one
    // vmcnt for both), so the one-chunk loop was a chain of dependent round trips (14 per thread on C4)
    constexpr int U = 4;
    for (int64_t ib = i0; ib < n4; ib += U * stride) {
        f32x4 gv[U], mv[U], vv[U], pv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * stride;
            if (i < n4) {
                gv[u] = reinterpret_cast<const f32x4*>(g)[i] * scale;
                mv[u] = reinterpret_cast<f32x4*>(m)[i];
                vv[u] = reinterpret_cast<f32x4*>(v)[i];
                pv[u] = reinterpret_cast<f32x4*>(p)[i];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * stride;
            if (i >= n4) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                mv[u][e] = b1 * mv[u][e] + (1.f - b1) * gv[u][e];
                vv[u][e] = b2 * vv[u][e] + (1.f - b2) * gv[u][e] * gv[u][e];
                pv[u][e] -= step_size * mv[u][e] / (sqrtf(vv[u][e]) / bc2s + eps);
            }
            if (zero_g) reinterpret_cast<f32x4*>(g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            reinterpret_cast<f32x4*>(m)[i] = mv[u];
            reinterpret_cast<f32x4*>(v)[i] = vv[u];
            reinterpret_cast<f32x4*>(p)[i] = pv[u];
        }
    }
    for (int64_t i = n4 * 4 + i0; i < n; i += stride) {
        const float gv = g[i] * scale;
        if (zero_g) g[i] = 0.f;
        m[i] = b1 * m[i] + (1.f - b1) * gv;
        v[i] = b2 * v[i] + (1.f - b2) * gv * gv;
        p[i] -= step_size * m[i] / (sqrtf(v[i]) / bc2s + eps);
    }
}

__global__ __launch_bounds__(256) void adam_fused_kernel(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                         float lr, float b1, float b2, float eps, float* step,
                                                         const float* __restrict__ part, int nparts,
                                                         float* __restrict__ sqnorm_out, float max_norm, int zero_g) {
    __shared__ float red[4];
    float acc = 0.f;
    for (int i = threadIdx.x; i < nparts; i += 256) acc += part[i];
    const float sq = block_sum_all<256>(acc, red);
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    if (lead && sqnorm_out) *sqnorm_out = sq;
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    if (!isfinite(sq)) {
        if (lead) *step -= 1.f;   // no block reads the count on this path
        if (zero_g) zero_range(g, n, i0, stride);
        return;
    }
    const float t = *step;       // counted by sq_part_kernel
    const float coef = max_norm / (sqrtf(sq) + 1e-6f);
    adam_range(p, g, m, v, n, i0, stride, coef < 1.f ? coef : 1.f, b1, b2, eps, lr / (1.f - powf(b1, t)),
               sqrtf(1.f - powf(b2, t)), zero_g != 0);
}

__global__ __launch_bounds__(1024) void adam_small_kernel(float* __restrict__ p, float* __restrict__ g,
                                                          float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                          float lr, float b1, float b2, float eps, float* step,
                                                          float* __restrict__ sqnorm_out, float max_norm,
                                                          int use_norm, int zero_g) {
    __shared__ float red[16];
    float scale = 1.f;
    if (use_norm) {
        float acc = 0.f;
        for (int64_t i = threadIdx.x; i < n; i += 1024) acc += g[i] * g[i];
        const float sq = block_sum_all<1024>(acc, red);
        if (threadIdx.x == 0 && sqnorm_out) *sqnorm_out = sq;
        if (!isfinite(sq)) {
            if (zero_g) zero_range(g, n, threadIdx.x, 1024);   // the norm pass read g: block_sum_all synced
            return;
        }
        const float coef = max_norm / (sqrtf(sq) + 1e-6f);
        scale = coef < 1.f ? coef : 1.f;
    }
    const float t = *step + 1.f;
    __syncthreads();             // every thread has read the count before thread 0 advances it
    adam_range(p, g, m, v, n, threadIdx.x, 1024, scale, b1, b2, eps, lr / (1.f - powf(b1, t)),
               sqrtf(1.f - powf(b2, t)), zero_g != 0);
    if (threadIdx.x == 0) *step = t;
}

}  // namespace cai

using namespace cai;

extern "C" {

const char* cai_last_error(void) { return g_err; }
int cai_version(void) { return 1; }
int cai_abi_count(void) { return 92; }

int cai_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps,
             float* step, const float* sqnorm, float max_norm, void* stream) {
    CAI_CHECK_ARG(p && g && m && v && step, "adam: null pointer");
    CAI_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0, "adam: buffers must be 16-byte aligned");
    if (n > 0) {
        int64_t blocks = (n / 4 + 255) / 256;
        if (blocks > 2048) blocks = 2048;
        if (blocks < 1) blocks = 1;
        hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p, g, m, v, n, lr,
                           beta1, beta2, eps, step, sqnorm, max_norm);
    }
    hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(1), 0, as_stream(stream), step, sqnorm);
    CAI_LAUNCH_CHECK("adam");
    return CAI_OK;
}

size_t cai_adam_step_workspace_bytes(int64_t n) { return (size_t)sq_parts(n) * sizeof(float); }

int cai_adam_step(float* p, float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                  float eps, float* step, float* sqnorm, float max_norm, int32_t flags, void* workspace,
                  size_t ws_bytes, void* stream) {
    CAI_CHECK_ARG(p && g && m && v && step && n >= 0, "adam_step: bad arguments");
    CAI_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                  "adam_step: buffers must be 16-byte aligned");
    const bool clip = (flags & CAI_ADAM_CLIP) != 0, use_norm = clip || (flags & CAI_ADAM_SKIP_NONFINITE);
    const int zero_g = (flags & CAI_ADAM_ZERO_GRAD) ? 1 : 0;
    const float mn = clip ? max_norm : INFINITY;
    hipStream_t st = as_stream(stream);
    if (n <= ADAM_SMALL_N) {
        hipLaunchKernelGGL(adam_small_kernel, dim3(1), dim3(1024), 0, st, p, g, m, v, n, lr, beta1, beta2, eps, step,
                           sqnorm, mn, (int)use_norm, zero_g);
    } else if (!use_norm) {
        CAI_CHECK_ARG(!zero_g, "adam_step: ZERO_GRAD needs CLIP or SKIP_NONFINITE above the one-block size");
        return cai_adam(p, g, m, v, n, lr, beta1, beta2, eps, step, nullptr, INFINITY, stream);
    } else {
        CAI_CHECK_ARG(workspace && ws_bytes >= cai_adam_step_workspace_bytes(n), "adam_step: workspace too small");
        const int np = sq_parts(n);
        float* part = reinterpret_cast<float*>(workspace);
        hipLaunchKernelGGL(sq_part_kernel, dim3(np), dim3(256), 0, st, g, n, part, step);
        int64_t blocks = (n / 4 + 255) / 256;
        blocks = blocks > 2048 ? 2048 : (blocks < 1 ? 1 : blocks);
        hipLaunchKernelGGL(adam_fused_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, lr, beta1,
                           beta2, eps, step, part, np, sqnorm, mn, zero_g);
    }
    CAI_LAUNCH_CHECK("adam_step");
    return CAI_OK;
}

}  // extern "C"
