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

}  // namespace cai

using namespace cai;

extern "C" {

const char* cai_last_error(void) { return g_err; }
int cai_version(void) { return 1; }
int cai_abi_count(void) { return 73; }

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

}  // extern "C"
