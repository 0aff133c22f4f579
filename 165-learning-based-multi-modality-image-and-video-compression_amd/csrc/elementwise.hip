// Pointwise glue of the residual / attention / sub-pixel blocks
// (compressai/layers/layers.py:81-244: ResidualBlockWithStride,
// ResidualBlockUpsample, ResidualBlock, AttentionBlock, subpel_conv3x3) on
// pixel-major activations.  All kernels move 16-byte chunks (8 bf16 / 4 fp32)
// when the channel count allows it, and are HBM-bound by construction:
//   add_act      y = act(a + b)                       12 B/elem (bf16: 6)
//   act          y = act(x)                           (used when no conv epilogue can take it)
//   gate fwd     y = a * sigmoid(b) + x               AttentionBlock.forward, layers.py:236-243
//   gate bwd     da = g * s(b), db = g * a * s(b)(1 - s(b))
//   pixel shuffle / its inverse (torch.nn.PixelShuffle channel order c*r^2 + i*r + j)
//   gdn1 out     y = x / norm  (inverse: x * norm)    GDN1.forward after its |x| 1x1 conv, gdn.py:111-121
//   gdn1 bwd     dx = g / norm, dnorm = -g x / norm^2  (inverse: g norm, g x)
#include "common.hpp"

#include <algorithm>
#include <initializer_list>

namespace cai {

__device__ __forceinline__ float act_f(float v, int act, float prm) {
    if (act == CAI_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == CAI_ACT_LEAKY) return v > 0.f ? v : v * prm;
    return v;
}

template <typename T>
struct Vec;
template <>
struct Vec<bf16> {
    static constexpr int N = 8;
    typedef bf16x8 V;
};
template <>
struct Vec<float> {
    static constexpr int N = 4;
    typedef f32x4 V;
};

// one thread per (pixel, chunk of N channels); `vec` chunks when C % N == 0
template <typename T>
__global__ void add_act_kernel(const T* __restrict__ a, int ald, const T* __restrict__ b, int bld, T* __restrict__ y,
                               int yld, int npix, int C, int act, float prm) {
    constexpr int N = Vec<T>::N;
    const int nch = (C + N - 1) / N;
    const int64_t total = (int64_t)npix * nch;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i / nch), c0 = (int)(i - (int64_t)p * nch) * N;
        if (c0 + N <= C) {
            const typename Vec<T>::V va = *reinterpret_cast<const typename Vec<T>::V*>(a + (int64_t)p * ald + c0);
            const typename Vec<T>::V vb = *reinterpret_cast<const typename Vec<T>::V*>(b + (int64_t)p * bld + c0);
            typename Vec<T>::V vy;
#pragma unroll
            for (int e = 0; e < N; ++e) vy[e] = from_f32<T>(act_f(to_f32(va[e]) + to_f32(vb[e]), act, prm));
            *reinterpret_cast<typename Vec<T>::V*>(y + (int64_t)p * yld + c0) = vy;
        } else {
            for (int c = c0; c < C; ++c)
                y[(int64_t)p * yld + c] =
                    from_f32<T>(act_f(to_f32(a[(int64_t)p * ald + c]) + to_f32(b[(int64_t)p * bld + c]), act, prm));
        }
    }
}

template <typename T>
__global__ void act_kernel(const T* __restrict__ x, int xld, T* __restrict__ y, int yld, int npix, int C, int act,
                           float prm) {
    constexpr int N = Vec<T>::N;
    const int nch = (C + N - 1) / N;
    const int64_t total = (int64_t)npix * nch;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i / nch), c0 = (int)(i - (int64_t)p * nch) * N;
        if (c0 + N <= C) {
            const typename Vec<T>::V vx = *reinterpret_cast<const typename Vec<T>::V*>(x + (int64_t)p * xld + c0);
            typename Vec<T>::V vy;
#pragma unroll
            for (int e = 0; e < N; ++e) vy[e] = from_f32<T>(act_f(to_f32(vx[e]), act, prm));
            *reinterpret_cast<typename Vec<T>::V*>(y + (int64_t)p * yld + c0) = vy;
        } else {
            for (int c = c0; c < C; ++c) y[(int64_t)p * yld + c] = from_f32<T>(act_f(to_f32(x[(int64_t)p * xld + c]), act, prm));
        }
    }
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + __expf(-v)); }

// y = a * sigmoid(b) + x
template <typename T>
__global__ void gate_fwd_kernel(const T* __restrict__ a, const T* __restrict__ b, const T* __restrict__ x,
                                T* __restrict__ y, int ld, int npix, int C) {
    const int64_t total = (int64_t)npix * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i / C), c = (int)(i - (int64_t)p * C);
        const int64_t o = (int64_t)p * ld + c;
        y[o] = from_f32<T>(to_f32(a[o]) * sigmoidf_(to_f32(b[o])) + to_f32(x[o]));
    }
}

template <typename T>
__global__ void gate_bwd_kernel(const T* __restrict__ a, const T* __restrict__ b, const T* __restrict__ g, int gld,
                                T* __restrict__ da, T* __restrict__ db, int ld, int npix, int C, int relu_a) {
    const int64_t total = (int64_t)npix * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i / C), c = (int)(i - (int64_t)p * C);
        const int64_t o = (int64_t)p * ld + c;
        const float s = sigmoidf_(to_f32(b[o]));
        const float gv = to_f32(g[(int64_t)p * gld + c]);
        const float av = to_f32(a[o]);
        // relu_a: a is a ReLU output (AttentionBlock's conv_a chain): its mask applied here, not in a launch of its own
        da[o] = from_f32<T>(relu_a && !(av > 0.f) ? 0.f : gv * s);
        db[o] = from_f32<T>(gv * av * s * (1.f - s));
    }
}

// bf16 forms with one 8-channel chunk (16 bytes) per thread: C % 8 == 0, ld % 8 == 0, 16-byte aligned rows
__global__ void gate_fwd_vec_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, const bf16* __restrict__ x,
                                    bf16* __restrict__ y, int ld, int64_t npix, int nch) {
    const int64_t total = npix * nch;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / nch;
        const int64_t o = p * ld + (int)(i - p * nch) * 8;
        const bf16x8 va = *reinterpret_cast<const bf16x8*>(a + o), vb = *reinterpret_cast<const bf16x8*>(b + o),
                     vx = *reinterpret_cast<const bf16x8*>(x + o);
        bf16x8 vy;
#pragma unroll
        for (int e = 0; e < 8; ++e) vy[e] = (bf16)((float)va[e] * sigmoidf_((float)vb[e]) + (float)vx[e]);
        *reinterpret_cast<bf16x8*>(y + o) = vy;
    }
}

__global__ void gate_bwd_vec_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, const bf16* __restrict__ g,
                                    int gld, bf16* __restrict__ da, bf16* __restrict__ db, int ld, int64_t npix, int nch,
                                    int relu_a) {
    const int64_t total = npix * nch;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / nch;
        const int c0 = (int)(i - p * nch) * 8;
        const int64_t o = p * ld + c0;
        const bf16x8 va = *reinterpret_cast<const bf16x8*>(a + o), vb = *reinterpret_cast<const bf16x8*>(b + o),
                     vg = *reinterpret_cast<const bf16x8*>(g + p * gld + c0);
        bf16x8 oa, ob;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float sg = sigmoidf_((float)vb[e]), gv = (float)vg[e], av = (float)va[e];
            oa[e] = (bf16)(relu_a && !(av > 0.f) ? 0.f : gv * sg);
            ob[e] = (bf16)(gv * av * sg * (1.f - sg));
        }
        *reinterpret_cast<bf16x8*>(da + o) = oa;
        *reinterpret_cast<bf16x8*>(db + o) = ob;
    }
}

__host__ __forceinline__ bool vec8_ok(int C, std::initializer_list<int> lds, std::initializer_list<const void*> ptrs) {
    if (C % 8) return false;
    for (int l : lds)
        if (l % 8) return false;
    for (const void* q : ptrs)
        if (reinterpret_cast<uintptr_t>(q) & 15) return false;
    return true;
}

// Pixel shuffle between x [B][H][W][C*r*r] (channel n = c*r*r + i*r + j) and
// y [B][H*r][W*r][C], both given by element strides (b, row, col, channel) so
// either side may be pixel-major or NCHW.  inverse = 0: y <- x; 1: x <- y.
struct ShuffleArgs {
    const void* src;
    void* dst;
    int64_t xs[4], ys[4];
    int B, H, W, C, r, inverse;
};

template <typename T>
__global__ void pixel_shuffle_kernel(const ShuffleArgs s) {
    const int OH = s.H * s.r, OW = s.W * s.r;
    const int64_t total = (int64_t)s.B * OH * OW * s.C;
    const T* src = reinterpret_cast<const T*>(s.src);
    T* dst = reinterpret_cast<T*>(s.dst);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        // y-major order: channel fastest (coalesced on the pixel-major side)
        const int c = (int)(i % s.C);
        int64_t r = i / s.C;
        const int ox = (int)(r % OW);
        r /= OW;
        const int oy = (int)(r % OH);
        const int b = (int)(r / OH);
        const int h = oy / s.r, ii = oy - h * s.r, w = ox / s.r, jj = ox - w * s.r;
        const int n = (c * s.r + ii) * s.r + jj;
        const int64_t xo = b * s.xs[0] + h * s.xs[1] + w * s.xs[2] + n * s.xs[3];
        const int64_t yo = b * s.ys[0] + oy * s.ys[1] + ox * s.ys[2] + c * s.ys[3];
        if (s.inverse)
            dst[xo] = src[yo];
        else
            dst[yo] = src[xo];
    }
}

// The same shuffle for bf16 with channel-contiguous sides (xs[3] == ys[3] == 1, 16-byte aligned pixel rows,
// C % 8 == 0): one thread per (input pixel, 8 output channels) reads the R*R*8 contiguous input channels those
// outputs come from (R*R 16-byte loads) and writes R*R output pixels x 8 channels (R*R 16-byte stores) -- the
// scalar kernel above moves 2 bytes per thread with 64-bit divisions per element (20.9 us per cheng2020 launch).
template <int R>
__global__ void pixel_shuffle_vec_kernel(const ShuffleArgs s) {
    const int CG = s.C / 8;
    const int64_t total = (int64_t)s.B * s.H * s.W * CG;
    const bf16* src = reinterpret_cast<const bf16*>(s.src);
    bf16* dst = reinterpret_cast<bf16*>(s.dst);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int cg = (int)(i % CG);
        int64_t p = i / CG;
        const int w = (int)(p % s.W);
        p /= s.W;
        const int h = (int)(p % s.H);
        const int b = (int)(p / s.H);
        const int64_t xo = b * s.xs[0] + h * s.xs[1] + w * s.xs[2] + (int64_t)cg * 8 * R * R;
        bf16x8 xv[R * R];    // input channels cg*8*R*R .. +8*R*R: element e = c_local*R*R + ii*R + jj
        if (!s.inverse) {
#pragma unroll
            for (int q = 0; q < R * R; ++q) xv[q] = *reinterpret_cast<const bf16x8*>(src + xo + 8 * q);
        }
#pragma unroll
        for (int ii = 0; ii < R; ++ii)
#pragma unroll
            for (int jj = 0; jj < R; ++jj) {
                const int64_t yo = b * s.ys[0] + (int64_t)(h * R + ii) * s.ys[1] + (int64_t)(w * R + jj) * s.ys[2] +
                                   cg * 8;
                if (!s.inverse) {
                    bf16x8 o;
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        const int e = c * R * R + ii * R + jj;
                        o[c] = xv[e / 8][e % 8];
                    }
                    *reinterpret_cast<bf16x8*>(dst + yo) = o;
                } else {
                    const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + yo);
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        const int e = c * R * R + ii * R + jj;
                        xv[e / 8][e % 8] = v[c];
                    }
                }
            }
        if (s.inverse) {
#pragma unroll
            for (int q = 0; q < R * R; ++q) *reinterpret_cast<bf16x8*>(dst + xo + 8 * q) = xv[q];
        }
    }
}

// GDN1 (layers/gdn.py:95-121): norm = beta + gamma |x| comes from a 1x1 conv on |x|; this is the
// remaining  out = x * (1 / norm)  (inverse: x * norm)  and its backward
template <typename T>
__global__ void gdn1_out_kernel(const T* __restrict__ x, int xld, const T* __restrict__ nrm, int nld,
                                T* __restrict__ y, int yld, int npix, int C, int inverse) {
    const int64_t total = (int64_t)npix * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i / C), c = (int)(i - (int64_t)p * C);
        const float xv = to_f32(x[(int64_t)p * xld + c]), nv = to_f32(nrm[(int64_t)p * nld + c]);
        y[(int64_t)p * yld + c] = from_f32<T>(inverse ? xv * nv : xv * (1.f / nv));
    }
}

template <typename T>
__global__ void gdn1_out_bwd_kernel(const T* __restrict__ x, int xld, const T* __restrict__ nrm, int nld,
                                    const T* __restrict__ g, int gld, T* __restrict__ dx, int dxld,
                                    T* __restrict__ dn, int dnld, int npix, int C, int inverse) {
    const int64_t total = (int64_t)npix * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i / C), c = (int)(i - (int64_t)p * C);
        const float xv = to_f32(x[(int64_t)p * xld + c]), nv = to_f32(nrm[(int64_t)p * nld + c]);
        const float gv = to_f32(g[(int64_t)p * gld + c]);
        float a, b;
        if (inverse) {
            a = gv * nv;
            b = gv * xv;
        } else {
            const float r = 1.f / nv;
            a = gv * r;
            b = -gv * xv * r * r;
        }
        dx[(int64_t)p * dxld + c] = from_f32<T>(a);
        dn[(int64_t)p * dnld + c] = from_f32<T>(b);
    }
}

// y += x * g[0] with g a device scalar: the aux loss's parameter gradient scaled by its upstream gradient,
// accumulated into the optimizer's flat buffer (BottleneckAuxFn.backward)
__global__ void axpy_dev_kernel(int64_t n, const float* __restrict__ x, const float* __restrict__ g,
                                float* __restrict__ y) {
    const float s = g[0];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] += x[i] * s;
}

static int ew_grid2(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(16384, (n + 255) / 256)); }

}  // namespace cai

using namespace cai;

extern "C" {

int cai_add_act(int dtype, const void* a, int32_t a_ld, const void* b, int32_t b_ld, void* y, int32_t y_ld,
                int64_t npix, int32_t C, int32_t act, float act_param, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "add_act: bad dtype");
    CAI_CHECK_ARG(a && b && y && a_ld >= C && b_ld >= C && y_ld >= C, "add_act: bad arguments");
    CAI_CHECK_ARG(npix < (1ll << 31), "add_act: too many pixels");
    const int N = dtype == CAI_BF16 ? 8 : 4;
    CAI_CHECK_ARG(a_ld % N == 0 && b_ld % N == 0 && y_ld % N == 0, "add_act: ld must be a multiple of %d", N);
    const int64_t n = npix * ((C + N - 1) / N);
    if (n == 0) return CAI_OK;
    hipStream_t st = as_stream(stream);
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(add_act_kernel<bf16>, dim3(ew_grid2(n)), dim3(256), 0, st, (const bf16*)a, a_ld,
                           (const bf16*)b, b_ld, (bf16*)y, y_ld, (int)npix, C, act, act_param);
    else
        hipLaunchKernelGGL(add_act_kernel<float>, dim3(ew_grid2(n)), dim3(256), 0, st, (const float*)a, a_ld,
                           (const float*)b, b_ld, (float*)y, y_ld, (int)npix, C, act, act_param);
    CAI_LAUNCH_CHECK("add_act");
    return CAI_OK;
}

int cai_axpy_dev(int64_t n, const float* x, const float* g, float* y, void* stream) {
    CAI_CHECK_ARG(n >= 0 && (n == 0 || (x && g && y)), "axpy_dev: bad arguments");
    if (n == 0) return CAI_OK;
    hipLaunchKernelGGL(axpy_dev_kernel, dim3(ew_grid2(n)), dim3(256), 0, as_stream(stream), n, x, g, y);
    CAI_LAUNCH_CHECK("axpy_dev");
    return CAI_OK;
}

int cai_act(int dtype, const void* x, int32_t x_ld, void* y, int32_t y_ld, int64_t npix, int32_t C, int32_t act,
            float act_param, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "act: bad dtype");
    CAI_CHECK_ARG(x && y && x_ld >= C && y_ld >= C && npix < (1ll << 31), "act: bad arguments");
    const int N = dtype == CAI_BF16 ? 8 : 4;
    CAI_CHECK_ARG(x_ld % N == 0 && y_ld % N == 0, "act: ld must be a multiple of %d", N);
    const int64_t n = npix * ((C + N - 1) / N);
    if (n == 0) return CAI_OK;
    hipStream_t st = as_stream(stream);
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(act_kernel<bf16>, dim3(ew_grid2(n)), dim3(256), 0, st, (const bf16*)x, x_ld, (bf16*)y, y_ld,
                           (int)npix, C, act, act_param);
    else
        hipLaunchKernelGGL(act_kernel<float>, dim3(ew_grid2(n)), dim3(256), 0, st, (const float*)x, x_ld, (float*)y,
                           y_ld, (int)npix, C, act, act_param);
    CAI_LAUNCH_CHECK("act");
    return CAI_OK;
}

int cai_gate_fwd(int dtype, const void* a, const void* b, const void* x, void* y, int32_t ld, int64_t npix, int32_t C,
                 void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "gate_fwd: bad dtype");
    CAI_CHECK_ARG(a && b && x && y && ld >= C && npix < (1ll << 31), "gate_fwd: bad arguments");
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipStream_t st = as_stream(stream);
    if (dtype == CAI_BF16 && vec8_ok(C, {ld}, {a, b, x, y}))
        hipLaunchKernelGGL(gate_fwd_vec_kernel, dim3(ew_grid2(n / 8)), dim3(256), 0, st, (const bf16*)a, (const bf16*)b,
                           (const bf16*)x, (bf16*)y, ld, npix, C / 8);
    else if (dtype == CAI_BF16)
        hipLaunchKernelGGL(gate_fwd_kernel<bf16>, dim3(ew_grid2(n)), dim3(256), 0, st, (const bf16*)a, (const bf16*)b,
                           (const bf16*)x, (bf16*)y, ld, (int)npix, C);
    else
        hipLaunchKernelGGL(gate_fwd_kernel<float>, dim3(ew_grid2(n)), dim3(256), 0, st, (const float*)a,
                           (const float*)b, (const float*)x, (float*)y, ld, (int)npix, C);
    CAI_LAUNCH_CHECK("gate_fwd");
    return CAI_OK;
}

int cai_gate_bwd(int dtype, const void* a, const void* b, const void* g, int32_t g_ld, void* da, void* db, int32_t ld,
                 int64_t npix, int32_t C, int32_t relu_a, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "gate_bwd: bad dtype");
    CAI_CHECK_ARG(a && b && g && da && db && ld >= C && g_ld >= C && npix < (1ll << 31), "gate_bwd: bad arguments");
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipStream_t st = as_stream(stream);
    if (dtype == CAI_BF16 && vec8_ok(C, {ld, g_ld}, {a, b, g, da, db}))
        hipLaunchKernelGGL(gate_bwd_vec_kernel, dim3(ew_grid2(n / 8)), dim3(256), 0, st, (const bf16*)a,
                           (const bf16*)b, (const bf16*)g, g_ld, (bf16*)da, (bf16*)db, ld, npix, C / 8, (int)relu_a);
    else if (dtype == CAI_BF16)
        hipLaunchKernelGGL(gate_bwd_kernel<bf16>, dim3(ew_grid2(n)), dim3(256), 0, st, (const bf16*)a, (const bf16*)b,
                           (const bf16*)g, g_ld, (bf16*)da, (bf16*)db, ld, (int)npix, C, (int)relu_a);
    else
        hipLaunchKernelGGL(gate_bwd_kernel<float>, dim3(ew_grid2(n)), dim3(256), 0, st, (const float*)a,
                           (const float*)b, (const float*)g, g_ld, (float*)da, (float*)db, ld, (int)npix, C,
                           (int)relu_a);
    CAI_LAUNCH_CHECK("gate_bwd");
    return CAI_OK;
}

int cai_gdn1_out(int dtype, const void* x, int32_t x_ld, const void* norm, int32_t n_ld, void* y, int32_t y_ld,
                 int64_t npix, int32_t C, int32_t inverse, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "gdn1_out: bad dtype");
    CAI_CHECK_ARG(x && norm && y && x_ld >= C && n_ld >= C && y_ld >= C && npix < (1ll << 31),
                  "gdn1_out: bad arguments");
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipStream_t st = as_stream(stream);
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(gdn1_out_kernel<bf16>, dim3(ew_grid2(n)), dim3(256), 0, st, (const bf16*)x, x_ld,
                           (const bf16*)norm, n_ld, (bf16*)y, y_ld, (int)npix, C, inverse);
    else
        hipLaunchKernelGGL(gdn1_out_kernel<float>, dim3(ew_grid2(n)), dim3(256), 0, st, (const float*)x, x_ld,
                           (const float*)norm, n_ld, (float*)y, y_ld, (int)npix, C, inverse);
    CAI_LAUNCH_CHECK("gdn1_out");
    return CAI_OK;
}

int cai_gdn1_out_bwd(int dtype, const void* x, int32_t x_ld, const void* norm, int32_t n_ld, const void* g,
                     int32_t g_ld, void* dx, int32_t dx_ld, void* dnorm, int32_t dn_ld, int64_t npix, int32_t C,
                     int32_t inverse, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "gdn1_out_bwd: bad dtype");
    CAI_CHECK_ARG(x && norm && g && dx && dnorm && x_ld >= C && n_ld >= C && g_ld >= C && dx_ld >= C && dn_ld >= C &&
                      npix < (1ll << 31),
                  "gdn1_out_bwd: bad arguments");
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipStream_t st = as_stream(stream);
    if (dtype == CAI_BF16)
        hipLaunchKernelGGL(gdn1_out_bwd_kernel<bf16>, dim3(ew_grid2(n)), dim3(256), 0, st, (const bf16*)x, x_ld,
                           (const bf16*)norm, n_ld, (const bf16*)g, g_ld, (bf16*)dx, dx_ld, (bf16*)dnorm, dn_ld,
                           (int)npix, C, inverse);
    else
        hipLaunchKernelGGL(gdn1_out_bwd_kernel<float>, dim3(ew_grid2(n)), dim3(256), 0, st, (const float*)x, x_ld,
                           (const float*)norm, n_ld, (const float*)g, g_ld, (float*)dx, dx_ld, (float*)dnorm, dn_ld,
                           (int)npix, C, inverse);
    CAI_LAUNCH_CHECK("gdn1_out_bwd");
    return CAI_OK;
}

int cai_pixel_shuffle(int dtype, const void* src, const int64_t* src_strides, void* dst, const int64_t* dst_strides,
                      int32_t B, int32_t H, int32_t W, int32_t C, int32_t r, int32_t inverse, void* stream) {
    CAI_CHECK_ARG(dtype == CAI_BF16 || dtype == CAI_F32, "pixel_shuffle: bad dtype");
    CAI_CHECK_ARG(src && dst && src_strides && dst_strides && r >= 1 && B > 0 && H > 0 && W > 0 && C > 0,
                  "pixel_shuffle: bad arguments");
    ShuffleArgs s{};
    s.src = src; s.dst = dst;
    // strides are given for the (source, destination) tensors; map them to x / y
    const int64_t* xs = inverse ? dst_strides : src_strides;
    const int64_t* ys = inverse ? src_strides : dst_strides;
    for (int i = 0; i < 4; ++i) { s.xs[i] = xs[i]; s.ys[i] = ys[i]; }
    s.B = B; s.H = H; s.W = W; s.C = C; s.r = r; s.inverse = inverse;
    const int64_t n = (int64_t)B * H * r * W * r * C;
    hipStream_t st = as_stream(stream);
    auto al16 = [](const void* p, int64_t off) { return ((reinterpret_cast<uintptr_t>(p) + off * 2) & 15) == 0; };
    const bool vec = dtype == CAI_BF16 && (r == 2 || r == 4) && C % 8 == 0 && s.xs[3] == 1 && s.ys[3] == 1 &&
                     s.xs[0] % 8 == 0 && s.xs[1] % 8 == 0 && s.xs[2] % 8 == 0 && s.ys[0] % 8 == 0 &&
                     s.ys[1] % 8 == 0 && s.ys[2] % 8 == 0 && al16(src, 0) && al16(dst, 0);
    if (vec) {
        const int64_t items = (int64_t)B * H * W * (C / 8);
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(16384, (items + 255) / 256));
        if (r == 2)
            hipLaunchKernelGGL(pixel_shuffle_vec_kernel<2>, dim3(grid), dim3(256), 0, st, s);
        else
            hipLaunchKernelGGL(pixel_shuffle_vec_kernel<4>, dim3(grid), dim3(256), 0, st, s);
    } else if (dtype == CAI_BF16)
        hipLaunchKernelGGL(pixel_shuffle_kernel<bf16>, dim3(ew_grid2(n)), dim3(256), 0, st, s);
    else
        hipLaunchKernelGGL(pixel_shuffle_kernel<float>, dim3(ew_grid2(n)), dim3(256), 0, st, s);
    CAI_LAUNCH_CHECK("pixel_shuffle");
    return CAI_OK;
}

}  // extern "C"
