// Entropy-model kernels: quantize, GaussianConditional and EntropyBottleneck
// likelihoods (fwd + bwd), EB aux loss, RD-loss reductions.
//
// Reference semantics (paths under /root/reference/CompressAI/compressai):
//   quantize ............ entropy_models/entropy_models.py:157-182 (torch.round = half-to-even -> rintf)
//   GC likelihood ....... entropy_models.py:629-635, 692-731
//   EB chain/likelihood . entropy_models.py:457-492, forward :495-540, loss :450-454
//   LowerBound bwd rule . ops/bound_ops.py:40-42 (grad passes iff x >= bound or grad < 0)
//
// All element-wise kernels are HBM-bound, pixel-major: element (p, c) at
// ptr[p*ld + c]; threads walk (p, c) in memory order so loads coalesce.
#include "common.hpp"

#include <algorithm>

namespace cai {

static constexpr float kNegInvSqrt2 = -0.70710678118654752440f;   // float(-(2**-0.5))
static constexpr float kTwoOverSqrtPi = 1.12837916709551257390f;

// ---------------------------------------------------------------------------
// training noise U(-1/2, 1/2) (entropy_models.py:170 `empty_like(x).uniform_(-0.5, 0.5)`) generated on the
// device from a counter in device memory, so a captured graph draws fresh noise on every replay without
// torch's generator (whose replays re-seed through extra fill launches).  Philox4x32-10 (Salmon et al.,
// SC'11): key = the 64-bit seed, counter = (element quad, draw index); the draw index lives in
// state[1] and is advanced by the last block of each launch to finish (state[2] is its arrival ticket,
// left at 0), so every launch -- and every replay -- uses a new counter range.  24-bit mantissas:
// u = (r >> 8) * 2^-24 - 1/2 in [-1/2, 1/2).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox_round(unsigned (&c)[4], const unsigned (&k)[2]) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c[0];
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c[2];
    const unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0, hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
    c[0] = hi1 ^ c[1] ^ k[0];
    c[1] = lo1;
    c[2] = hi0 ^ c[3] ^ k[1];
    c[3] = lo0;
}
__device__ __forceinline__ void philox4x32_10(unsigned (&c)[4], unsigned k0, unsigned k1) {
    unsigned k[2] = {k0, k1};
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        philox_round(c, k);
        k[0] += 0x9E3779B9u;
        k[1] += 0xBB67AE85u;
    }
}

__device__ __forceinline__ float philox_uniform(unsigned long long seed, unsigned long long draw, int64_t i) {
    const unsigned long long q = (unsigned long long)i >> 2;
    unsigned c[4] = {(unsigned)q, (unsigned)(q >> 32), (unsigned)draw, (unsigned)(draw >> 32)};
    philox4x32_10(c, (unsigned)seed, (unsigned)(seed >> 32));
    const unsigned e = (unsigned)i & 3u;
    const unsigned r = e == 0 ? c[0] : (e == 1 ? c[1] : (e == 2 ? c[2] : c[3]));
    return (float)(r >> 8) * 5.9604644775390625e-8f - 0.5f;
}

// The noise operand inside a kernel (cai_noise_src): a buffer, or the Philox draw {seed, draw} generated per
// element -- element (p, c) is element p*C + c of cai_uniform_noise's draw, so DRAW / REPLAY reproduce a
// BUF launch fed by cai_uniform_noise bit for bit.
struct NoiseView {
    const float* buf;
    int ld, gen;
    unsigned long long seed, draw;
    __device__ __forceinline__ float at(int64_t p, int c, int C) const {
        return gen ? philox_uniform(seed, draw, p * C + c) : buf[p * ld + c];
    }
};

// Every thread calls this before any early return.  DRAW: thread 0 of each block reads the generator (seed,
// draw index) and broadcasts it through LDS; block 0 records it in the slot for the REPLAY launches.
__device__ __forceinline__ NoiseView noise_open(const cai_noise_src& S) {
    NoiseView v{S.buf, S.ld, S.kind != CAI_NOISE_BUF, 0ull, 0ull};
    if (S.kind == CAI_NOISE_DRAW) {
        __shared__ unsigned long long sd[2];
        if (threadIdx.x == 0 && threadIdx.y == 0) {
            const unsigned long long seed = __hip_atomic_load(S.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long draw = __hip_atomic_load(S.state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sd[0] = seed;
            sd[1] = draw;
            if (blockIdx.x == 0 && blockIdx.y == 0) {
                __hip_atomic_store(S.slot, seed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(S.slot + 1, draw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        v.seed = sd[0];
        v.draw = sd[1];
    } else if (S.kind == CAI_NOISE_REPLAY) {
        v.seed = S.slot[0];
        v.draw = S.slot[1];
    }
    return v;
}

// DRAW: thread 0 of every block, after its noise_open (its state read is complete: the value went to LDS).
// The block arrives on its XCD shard's ticket (blocks go round-robin over the 8 XCDs, shard = linear block id
// mod 8; a fan-in on one word costs ~12 ns per arrival, MI355X_MICROARCH.md 'fanin'); the last arriver of each
// shard resets it and arrives on state[2]; the last of those advances the draw index and resets state[2].
// Relaxed: the next launch sees the new index across the kernel boundary.
__device__ __forceinline__ void noise_close(const cai_noise_src& S, const NoiseView& v) {
    if (S.kind != CAI_NOISE_DRAW || threadIdx.x != 0 || threadIdx.y != 0) return;
    const unsigned nb = gridDim.x * gridDim.y;
    const unsigned b = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned k = b & 7u;
    const unsigned nk = (nb - k + 7u) / 8u;
    unsigned long long* shard = S.state + CAI_NOISE_SHARD0 + 16 * k;
    if (__hip_atomic_fetch_add(shard, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nk - 1) return;
    __hip_atomic_store(shard, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned ns = nb < 8u ? nb : 8u;
    if (__hip_atomic_fetch_add(S.state + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ns - 1) return;
    __hip_atomic_store(S.state + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(S.state + 1, v.draw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// quantize
// ---------------------------------------------------------------------------
__global__ void quantize_kernel(int mode, int64_t n, int C, const void* __restrict__ x, int xdt, int xld,
                                const float* __restrict__ means, int mld, int means_pc,
                                const cai_noise_src ns, void* __restrict__ out, int odt, int old) {
    const NoiseView nv = noise_open(ns);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int c = (int)(i - p * C);
        const float v = ld_any(x, xdt, p * xld + c);
        if (mode == CAI_Q_NOISE) {
            st_any(out, odt, p * old + c, v + nv.at(p, c, C));
            continue;
        }
        float mu = 0.f;
        if (means) mu = means_pc ? means[c] : means[p * mld + c];
        float r = rintf(means ? v - mu : v);
        if (mode == CAI_Q_SYMBOLS) {
            reinterpret_cast<int32_t*>(out)[p * old + c] = (int32_t)r;
        } else {
            st_any(out, odt, p * old + c, means ? r + mu : r);
        }
    }
    noise_close(ns, nv);
}

static inline int ew_grid(int64_t n, int nt = 256) {
    int64_t b = (n + nt - 1) / nt;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

// ---------------------------------------------------------------------------
// GaussianConditional
// ---------------------------------------------------------------------------
__device__ __forceinline__ float std_cum(float t) {   // 0.5 * erfc(-(2^-0.5) * t)
    return 0.5f * erfcf(kNegInvSqrt2 * t);
}
// d/dt [0.5 erfc(c t)] following torch's erfc backward: -2/sqrt(pi) exp(-(ct)^2) * c * 0.5
__device__ __forceinline__ float std_cum_grad(float t) {
    const float a = kNegInvSqrt2 * t;
    return 0.5f * (-kTwoOverSqrtPi * expf(-a * a)) * kNegInvSqrt2;
}

__global__ void gc_fwd_kernel(int mode, int64_t n, int C, const void* __restrict__ x, int xdt, int xld,
                              const void* __restrict__ sc, int sld, const void* __restrict__ mu, int mld, int smdt,
                              const cai_noise_src ns, float sbound, float lbound,
                              void* __restrict__ q, int qdt, int qld, float* __restrict__ lik, int lld) {
    const NoiseView nv = noise_open(ns);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int c = (int)(i - p * C);
        const float xv = ld_any(x, xdt, p * xld + c);
        const float m = mu ? ld_any(mu, smdt, p * mld + c) : 0.f;
        float qv;
        if (mode == CAI_Q_NOISE)
            qv = xv + nv.at(p, c, C);
        else
            qv = mu ? rintf(xv - m) + m : rintf(xv);
        if (q) st_any(q, qdt, p * qld + c, qv);
        const float v = mu ? qv - m : qv;
        const float s = fmaxf(ld_any(sc, smdt, p * sld + c), sbound);
        const float av = fabsf(v);
        const float up = std_cum((0.5f - av) / s);
        const float lo = std_cum((-0.5f - av) / s);
        lik[p * lld + c] = fmaxf(up - lo, lbound);
    }
    noise_close(ns, nv);
}

// relu: the scales are a ReLU's output (ScaleHyperprior's h_s ends in nn.ReLU) and their gradient leaves here with
// that ReLU's backward mask (scales > 0) applied -- the conv before the ReLU then needs no act-backward launch
__global__ void gc_bwd_kernel(int mode, int relu, int64_t n, int C, const void* __restrict__ x, int xdt, int xld,
                              const void* __restrict__ sc, int sld, const void* __restrict__ mu, int mld, int smdt,
                              const cai_noise_src ns, float sbound, float lbound,
                              const float* __restrict__ glik, int glld, const void* __restrict__ gq, int gqdt,
                              int gqld, void* __restrict__ dx, int dxld, void* __restrict__ ds, int dsld,
                              void* __restrict__ dm, int dmld) {
    const NoiseView nv = noise_open(ns);   // BUF or REPLAY
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int c = (int)(i - p * C);
        const float xv = ld_any(x, xdt, p * xld + c);
        const float m = mu ? ld_any(mu, smdt, p * mld + c) : 0.f;
        const float qv = (mode == CAI_Q_NOISE) ? xv + nv.at(p, c, C) : (mu ? rintf(xv - m) + m : rintf(xv));
        const float v = mu ? qv - m : qv;
        const float sraw = ld_any(sc, smdt, p * sld + c);
        const float s = fmaxf(sraw, sbound);
        const float av = fabsf(v);
        const float tu = (0.5f - av) / s;
        const float tl = (-0.5f - av) / s;
        float g = glik ? glik[p * glld + c] : 0.f;
        const float lraw = std_cum(tu) - std_cum(tl);
        if (!(lraw >= lbound || g < 0.f)) g = 0.f;           // LowerBound(lik) backward
        const float dtu = g * std_cum_grad(tu);
        const float dtl = -g * std_cum_grad(tl);
        // t = a / s : da = dt / s ; ds = -dt * a / (s*s)
        const float dav = -(dtu + dtl) / s;
        float dsv = -dtu * (0.5f - av) / (s * s) - dtl * (-0.5f - av) / (s * s);
        if (!(sraw >= sbound || dsv < 0.f)) dsv = 0.f;      // LowerBound(scales) backward
        if (relu && !(sraw > 0.f)) dsv = 0.f;                // the ReLU before it
        const float sgn = (v > 0.f) ? 1.f : ((v < 0.f) ? -1.f : 0.f);
        const float dv = dav * sgn;
        const float gqv = gq ? ld_any(gq, gqdt, p * gqld + c) : 0.f;
        if (mode == CAI_Q_NOISE) {
            if (dx) st_any(dx, xdt, p * dxld + c, gqv + dv);
            if (dm) st_any(dm, smdt, p * dmld + c, -dv);
        } else {
            if (dx) st_any(dx, xdt, p * dxld + c, 0.f);
            if (dm) st_any(dm, smdt, p * dmld + c, (gqv + dv) - dv);
        }
        if (ds) st_any(ds, smdt, p * dsld + c, dsv);
    }
}

// ---------------------------------------------------------------------------
// EntropyBottleneck: per-channel monotone MLP 1->3->3->3->3->1
// ---------------------------------------------------------------------------
// per-channel table: softplus'd matrices (3 + 9 + 9 + 9 + 3 = 33), biases
// (3*4 + 1 = 13), tanh'd factors (12), median (1)
constexpr int EB_SP = 0, EB_B = 33, EB_TF = 46, EB_MED = 58, EB_NP = 60;

__device__ __forceinline__ float softplus_f(float v) {   // F.softplus(beta=1, threshold=20)
    return v > 20.f ? v : log1pf(expf(v));
}
__device__ __forceinline__ float softplus_grad(float v) {   // torch softplus backward
    if (v > 20.f) return 1.f;
    const float z = expf(v);
    return z / (z + 1.f);
}
// the division as v_rcp_f32 (1 ulp): the IEEE divide's scale / fmas / fixup sequence was ~10 instructions, two per
// chain pair in both EntropyBottleneck kernels
__device__ __forceinline__ float sigmoid_f(float v) { return __builtin_amdgcn_rcpf(1.f + expf(-v)); }

// Address of the raw parameter behind element k of channel c's table (layout
// above; k < EB_NP, always a valid address -- the pad slot reads the median).
__device__ __forceinline__ const float* eb_raw_ptr(int c, int k, const cai_eb_params& P) {
    if (k < 3) return P.matrix[0] + c * 3 + k;
    if (k < 30) {
        const int l = (k - 3) / 9, j = (k - 3) - 9 * ((k - 3) / 9);
        return (l == 0 ? P.matrix[1] : (l == 1 ? P.matrix[2] : P.matrix[3])) + c * 9 + j;
    }
    if (k < 33) return P.matrix[4] + c * 3 + (k - 30);
    if (k < 45) {
        const int l = (k - 33) / 3, j = (k - 33) - 3 * ((k - 33) / 3);
        return (l == 0 ? P.bias[0] : (l == 1 ? P.bias[1] : (l == 2 ? P.bias[2] : P.bias[3]))) + c * 3 + j;
    }
    if (k == 45) return P.bias[4] + c;
    if (k < 58) {
        const int l = (k - 46) / 3, j = (k - 46) - 3 * ((k - 46) / 3);
        return (l == 0 ? P.factor[0] : (l == 1 ? P.factor[1] : (l == 2 ? P.factor[2] : P.factor[3]))) + c * 3 + j;
    }
    return P.quantiles + c * 3 + 1;
}
__device__ __forceinline__ float eb_xform(int k, float v) {
    if (k < EB_B) return softplus_f(v);
    if (k >= EB_TF && k < EB_MED) return tanhf(v);
    return k <= EB_MED ? v : 0.f;
}

// Tables of channels [c0, c0 + nch) into tab[nch][EB_NP] (LDS); caller syncs.
// Filled cooperatively in two passes: every thread first issues all of its
// PT loads (unconditional, from clamped valid addresses, so they are in
// flight together), then transforms them -- one global-load latency per
// block instead of one per parameter.  PT >= nch * EB_NP / blockDim.x.
template <int PT>
__device__ __forceinline__ void eb_fill_tables(int c0, int nch, int C, const cai_eb_params& P, float* tab) {
    const int n = nch * EB_NP;
    float raw[PT];
#pragma unroll
    for (int r = 0; r < PT; ++r) {
        const int i = min((int)(threadIdx.x + r * blockDim.x), n - 1);
        const int cl = i / EB_NP, k = i - cl * EB_NP;
        raw[r] = *eb_raw_ptr(min(c0 + cl, C - 1), k, P);
    }
#pragma unroll
    for (int r = 0; r < PT; ++r) {
        const int i = threadIdx.x + r * blockDim.x;
        if (i < n) {
            const int cl = i / EB_NP, k = i - cl * EB_NP;
            tab[i] = (c0 + cl < C) ? eb_xform(k, raw[r]) : 0.f;
        }
    }
}

// tanh for the CDF chains: Cephes' single-precision tanhf (|x| < 0.625: odd polynomial, relative error
// 1.3e-7; else 1 - 2 / (e^{2|x|} + 1) with the hardware exp; |x| > 9: +-1), ~12 instructions against ~100 for
// the libm tanhf with its special-case branches -- the chains evaluate 12 per call and dominated the
// EntropyBottleneck kernels.  The forward and backward kernels share it, so the backward re-derives exactly the
// forward's values (sign, LowerBound mask) and reads tanh' = 1 - tanh^2 from the recorded values.
// Both branches are evaluated and selected (branch-free: a divergent if / else around 12 tanh per chain cost an
// exec-mask save / restore and a scalar branch each), the large-|x| branch with v_rcp_f32 (1 ulp).
__device__ __forceinline__ float eb_tanh(float x) {
    const float ax = fabsf(x);
    const float z = x * x;
    const float p = ((((-5.70498872745e-3f * z + 2.06390887954e-2f) * z - 5.37397155531e-2f) * z + 1.33314422036e-1f) *
                         z - 3.33332819422e-1f) * z * x + x;
    const float e = __expf(2.f * fminf(ax, 9.f));
    const float q = copysignf(1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f), x);
    return ax < 0.625f ? p : q;
}

// forward of one chain; records the tanh of every hidden pre-activation and every hidden output
struct EbTrace {
    float t[4][3];   // tanh(a[l][j])
    float h[4][3];
};

__device__ __forceinline__ float eb_chain(float x, const float* t, EbTrace* tr) {
    float h[3], hn[3];
    // layer 0: [3,1]
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float a = t[EB_SP + j] * x + t[EB_B + j];
        const float th = eb_tanh(a);
        if (tr) tr->t[0][j] = th;
        h[j] = a + t[EB_TF + j] * th;
        if (tr) tr->h[0][j] = h[j];
    }
#pragma unroll
    for (int l = 1; l < 4; ++l) {
        const float* M = t + EB_SP + 3 + (l - 1) * 9;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float a = M[j * 3 + 0] * h[0] + M[j * 3 + 1] * h[1] + M[j * 3 + 2] * h[2] + t[EB_B + l * 3 + j];
            const float th = eb_tanh(a);
            if (tr) tr->t[l][j] = th;
            hn[j] = a + t[EB_TF + l * 3 + j] * th;
            if (tr) tr->h[l][j] = hn[j];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) h[j] = hn[j];
    }
    const float* M4 = t + EB_SP + 30;
    return M4[0] * h[0] + M4[1] * h[1] + M4[2] * h[2] + t[EB_B + 12];
}

// backward of one chain with upstream gradient d; accumulates d(softplus'd matrix), d(bias), d(tanh'd factor)
// into g[] (same index layout as the table) and returns d input.
__device__ __forceinline__ float eb_chain_bwd(float x, float d, const float* t, const EbTrace& tr, float* g) {
    float dh[3];
    g[EB_B + 12] += d;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        g[EB_SP + 30 + k] += d * tr.h[3][k];
        dh[k] = d * t[EB_SP + 30 + k];
    }
#pragma unroll
    for (int l = 3; l >= 0; --l) {
        float da[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float th = tr.t[l][j];
            const float tf = t[EB_TF + l * 3 + j];
            g[EB_TF + l * 3 + j] += dh[j] * th;
            da[j] = dh[j] * (1.f + tf * (1.f - th * th));
            g[EB_B + l * 3 + j] += da[j];
        }
        if (l == 0) {
            float dx = 0.f;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                g[EB_SP + j] += da[j] * x;
                dx += t[EB_SP + j] * da[j];
            }
            return dx;
        }
        const float* M = t + EB_SP + 3 + (l - 1) * 9;
        float* gM = g + EB_SP + 3 + (l - 1) * 9;
        float dp[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                gM[j * 3 + k] += da[j] * tr.h[l - 1][k];
                dp[k] += M[j * 3 + k] * da[j];
            }
#pragma unroll
        for (int k = 0; k < 3; ++k) dh[k] = dp[k];
    }
    return 0.f;
}

// d input of one chain (no parameter gradients): the aux loss's quantiles grad
__device__ __forceinline__ float eb_chain_dx(float d, const float* t, const EbTrace& tr) {
    float dh[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) dh[k] = d * t[EB_SP + 30 + k];
#pragma unroll
    for (int l = 3; l >= 0; --l) {
        float da[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float th = tr.t[l][j];
            da[j] = dh[j] * (1.f + t[EB_TF + l * 3 + j] * (1.f - th * th));
        }
        if (l == 0) return t[EB_SP + 0] * da[0] + t[EB_SP + 1] * da[1] + t[EB_SP + 2] * da[2];
        const float* M = t + EB_SP + 3 + (l - 1) * 9;
#pragma unroll
        for (int k = 0; k < 3; ++k) dh[k] = M[0 * 3 + k] * da[0] + M[1 * 3 + k] * da[1] + M[2 * 3 + k] * da[2];
    }
    return 0.f;
}

#ifndef EB_FWD_PPL
#define EB_FWD_PPL 4
#endif
// fwd: block = 256 threads = 32 channels x 8 pixel rows
__global__ __launch_bounds__(256) void eb_fwd_kernel(int mode, int64_t npix, int C, cai_eb_params P,
                                                      const void* __restrict__ x, int xdt, int xld,
                                                      const cai_noise_src ns, float lbound,
                                                      void* __restrict__ q, int qdt, int qld,
                                                      float* __restrict__ lik, int lld) {
    __shared__ float tab[32][EB_NP];
    const NoiseView nv = noise_open(ns);
    const int cl = threadIdx.x & 31, pr = threadIdx.x >> 5;
    const int c0 = blockIdx.x * 32;
    eb_fill_tables<(32 * EB_NP + 255) / 256>(c0, 32, C, P, &tab[0][0]);
    __syncthreads();
    const int c = c0 + cl;
    if (c >= C) return;
    const float* t = tab[cl];
    for (int64_t p = blockIdx.y * 8 + pr; p < npix; p += (int64_t)gridDim.y * 8) {
        const float xv = ld_any(x, xdt, p * xld + c);
        float v;
        if (mode == CAI_Q_NOISE)
            v = xv + nv.at(p, c, C);
        else
            v = rintf(xv - t[EB_MED]) + t[EB_MED];
        if (q) st_any(q, qdt, p * qld + c, v);
        const float lo = eb_chain(v - 0.5f, t, nullptr);
        const float up = eb_chain(v + 0.5f, t, nullptr);
        const float sum = lo + up;
        const float sgn = -((sum > 0.f) ? 1.f : ((sum < 0.f) ? -1.f : 0.f));
        const float l = fabsf(sigmoid_f(sgn * up) - sigmoid_f(sgn * lo));
        lik[p * lld + c] = fmaxf(l, lbound);
    }
    noise_close(ns, nv);   // thread 0 (c = c0 < C) always gets here
}

#ifndef EB_BWD_PPL
#define EB_BWD_PPL 4
#endif
// bwd: grid (C, S): block (c, s) takes every S-th 256-pixel slice of channel c, one chain pair per thread and
// pass; its 60 per-channel parameter sums reduce in a fixed order (lanes by xor-shuffles, the 4 waves through
// LDS).  With S > 1 each block stores its 60 sums write-through (sc1) into part[c][s], and the block whose
// arrival on the channel's ticket comes last sums them in split order (sc1 loads) -- the hand-off of
// MI355X_MICROARCH.md's first hand-off row (every storing wave waits vmcnt(0), a workgroup barrier, one agent
// atomic add per block; the last arriver learns it from the returned value), no fences -- resets the ticket
// and applies the chain rule through softplus / tanh into the torch layout.  Deterministic.
__global__ __launch_bounds__(256) void eb_bwd_kernel(int mode, int64_t npix, int C, cai_eb_params P,
                                                       const void* __restrict__ x, int xdt, int xld,
                                                       const cai_noise_src ns, float lbound,
                                                       const float* __restrict__ glik, int glld,
                                                       const void* __restrict__ gq, int gqdt, int gqld,
                                                       void* __restrict__ dx, int dxld, cai_eb_grads G,
                                                       float* __restrict__ part, unsigned* __restrict__ tickets) {
    __shared__ float tab[EB_NP];
    __shared__ float red[4][EB_NP];
    __shared__ int s_last;
    const int c = blockIdx.x, S = gridDim.y, sp = blockIdx.y;
    const NoiseView nv = noise_open(ns);   // BUF or REPLAY
    eb_fill_tables<1>(c, 1, C, P, tab);
    __syncthreads();
    const float* t = tab;
    float g[EB_NP];
#pragma unroll
    for (int k = 0; k < EB_NP; ++k) g[k] = 0.f;
    for (int64_t p = (int64_t)sp * 256 + threadIdx.x; p < npix; p += (int64_t)S * 256) {
        const float xv = ld_any(x, xdt, p * xld + c);
        const float v = (mode == CAI_Q_NOISE) ? xv + nv.at(p, c, C) : rintf(xv - t[EB_MED]) + t[EB_MED];
        EbTrace tl, tu;
        const float lo = eb_chain(v - 0.5f, t, &tl);
        const float up = eb_chain(v + 0.5f, t, &tu);
        const float sum = lo + up;
        const float sgn = -((sum > 0.f) ? 1.f : ((sum < 0.f) ? -1.f : 0.f));
        const float su = sigmoid_f(sgn * up), sl = sigmoid_f(sgn * lo);
        const float D = su - sl;
        float gl = glik ? glik[p * glld + c] : 0.f;
        if (!(fabsf(D) >= lbound || gl < 0.f)) gl = 0.f;      // LowerBound(lik)
        const float dD = gl * ((D > 0.f) ? 1.f : ((D < 0.f) ? -1.f : 0.f));   // abs
        const float dup = dD * su * (1.f - su) * sgn;
        const float dlo = -dD * sl * (1.f - sl) * sgn;
        float dv = eb_chain_bwd(v + 0.5f, dup, t, tu, g) + eb_chain_bwd(v - 0.5f, dlo, t, tl, g);
        const float gqv = gq ? ld_any(gq, gqdt, p * gqld + c) : 0.f;
        if (mode == CAI_Q_NOISE) {
            if (dx) st_any(dx, xdt, p * dxld + c, gqv + dv);
        } else {
            if (dx) st_any(dx, xdt, p * dxld + c, 0.f);
            g[EB_MED] += gqv + dv;
        }
    }
    // reduce each accumulator: 64 lanes by shuffles, then the 4 waves in order
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < EB_NP; ++k) {
        const float v = wave_sum_dpp(g[k]);
        if (lane == 0) red[w][k] = v;
    }
    __syncthreads();
    const int k = threadIdx.x;
    float v = 0.f;
    if (k < EB_NP) v = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    if (S > 1) {
        float* mine = part + ((int64_t)c * S + sp) * EB_NP;
        if (k < EB_NP) __hip_atomic_store(mine + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned prev = __hip_atomic_fetch_add(tickets + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = prev == (unsigned)S - 1;
            if (s_last) __hip_atomic_store(tickets + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!s_last) return;
        if (k < EB_NP) {
            const float* all = part + (int64_t)c * S * EB_NP + k;
            v = 0.f;
            for (int s2 = 0; s2 < S; ++s2)
                v += __hip_atomic_load(all + (int64_t)s2 * EB_NP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // one thread per table element: chain rule through softplus / tanh and the store to torch layout
    if (k >= EB_NP || k == 59) return;
    float* dst;
    float val;
    if (k < EB_B) {                                   // matrices: d softplus(raw) = sigmoid(raw)
        const float* raw = eb_raw_ptr(c, k, P);
        val = v * softplus_grad(*raw);
        const int64_t off = raw - (k < 3 ? P.matrix[0] : (k < 12 ? P.matrix[1] : (k < 21 ? P.matrix[2] :
                                   (k < 30 ? P.matrix[3] : P.matrix[4]))));
        float* base = k < 3 ? G.matrix[0] : (k < 12 ? G.matrix[1] : (k < 21 ? G.matrix[2] :
                      (k < 30 ? G.matrix[3] : G.matrix[4])));
        dst = base + off;
    } else if (k < EB_TF) {                           // biases
        const int kb = k - EB_B;
        const int l = kb / 3, j = kb - 3 * (kb / 3);
        val = v;
        dst = kb == 12 ? G.bias[4] + c
                       : (l == 0 ? G.bias[0] : (l == 1 ? G.bias[1] : (l == 2 ? G.bias[2] : G.bias[3]))) + c * 3 + j;
    } else if (k < EB_MED) {                          // factors: d tanh(raw) = 1 - tanh^2
        const int kf = k - EB_TF;
        const int l = kf / 3, j = kf - 3 * (kf / 3);
        const float th = t[k];
        val = v * (1.f - th * th);
        dst = (l == 0 ? G.factor[0] : (l == 1 ? G.factor[1] : (l == 2 ? G.factor[2] : G.factor[3]))) + c * 3 + j;
    } else {                                          // k == EB_MED: the medians (quantiles[:, :, 1])
        if (!G.quantiles) return;
        G.quantiles[c * 3 + 0] = G.accumulate ? G.quantiles[c * 3 + 0] : 0.f;
        G.quantiles[c * 3 + 2] = G.accumulate ? G.quantiles[c * 3 + 2] : 0.f;
        val = (mode == CAI_Q_NOISE) ? 0.f : v;
        dst = G.quantiles + c * 3 + 1;
    }
    *dst = G.accumulate ? *dst + val : val;
}

// aux loss: blocks of 32 channels (96 (channel, k) threads, tables filled cooperatively into LDS).  Each block
// stores its loss partial write-through and takes a ticket; the last block sums the partials in block order
// (the eb_bwd hand-off) into *loss.  Deterministic.
constexpr int EB_AUX_CH = 32;
__global__ __launch_bounds__(256) void eb_aux_kernel(int C, cai_eb_params P, const float* __restrict__ target,
                                                      float* __restrict__ loss, const float* __restrict__ gloss,
                                                      float* __restrict__ dq, int accumulate,
                                                      float* __restrict__ part, unsigned* __restrict__ ticket) {
    __shared__ float red[4];
    __shared__ float tab[EB_AUX_CH * EB_NP];
    __shared__ int s_last;
    const int c0 = blockIdx.x * EB_AUX_CH;
    const int nch = min(EB_AUX_CH, C - c0);
    eb_fill_tables<(EB_AUX_CH * EB_NP + 255) / 256>(c0, nch, C, P, tab);
    __syncthreads();
    float acc = 0.f;
    const float gs = gloss ? *gloss : 0.f;
    const int i = threadIdx.x;
    if (i < 3 * nch) {
        const int cl = i / 3, k = i - 3 * (i / 3), c = c0 + cl;
        const float* t = tab + cl * EB_NP;
        const float qv = P.quantiles[c * 3 + k];
        EbTrace tr;
        const float f = eb_chain(qv, t, &tr);
        const float diff = f - target[k];
        acc = fabsf(diff);
        if (dq) {
            const float sg = (diff > 0.f) ? 1.f : ((diff < 0.f) ? -1.f : 0.f);
            const float v = eb_chain_dx(gs * sg, t, tr);
            dq[c * 3 + k] = accumulate ? dq[c * 3 + k] + v : v;
        }
    }
    const float r = block_sum<256>(acc, red);
    const int nb = gridDim.x;
    if (nb == 1) {
        if (threadIdx.x == 0 && loss) *loss = r;
        return;
    }
    if (threadIdx.x == 0) {
        __hip_atomic_store(part + blockIdx.x, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == (unsigned)nb - 1;
        if (s_last) {
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            float tot = 0.f;
            for (int b = 0; b < nb; ++b) tot += __hip_atomic_load(part + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (loss) *loss = tot;
        }
    }
}

// ---------------------------------------------------------------------------
// reductions (two-stage, deterministic)
// ---------------------------------------------------------------------------
constexpr int RED_BLOCKS = 1024;

template <int KIND>   // 0: sum log(a) over (p,c) with ld ; 1: sum (a-b)^2 contiguous ; 2: sum a^2 contiguous
__global__ __launch_bounds__(256) void reduce_stage1(const float* __restrict__ a, const float* __restrict__ b,
                                                      int64_t n, int C, int ld, float* __restrict__ part) {
    __shared__ float red[4];
    float acc = 0.f;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if (KIND == 0) {
            const int64_t p = i / C;
            acc += logf(a[p * ld + (i - p * C)]);
        } else if (KIND == 1) {
            const float d = a[i] - b[i];
            acc += d * d;
        } else {
            acc += a[i] * a[i];
        }
    }
    const float r = block_sum<256>(acc, red);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}

__global__ __launch_bounds__(256) void reduce_stage2(const float* __restrict__ part, int n, float* __restrict__ out) {
    __shared__ float red[4];
    float acc = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) acc += part[i];
    const float r = block_sum<256>(acc, red);
    if (threadIdx.x == 0) *out = r;
}

static int red_blocks(int64_t n) {
    int64_t b = (n + 1023) / 1024;
    if (b > RED_BLOCKS) b = RED_BLOCKS;
    return b < 1 ? 1 : (int)b;
}

template <int KIND>
static int run_reduce(const float* a, const float* b, int64_t n, int C, int ld, float* out, void* ws, size_t wsb,
                      void* stream, const char* name) {
    CAI_CHECK_ARG(n >= 0, "%s: negative size", name);
    CAI_CHECK_ARG(ws && wsb >= cai_reduce_workspace_bytes(n), "%s: workspace too small", name);
    const int nb = red_blocks(n);
    float* part = reinterpret_cast<float*>(ws);
    hipLaunchKernelGGL(reduce_stage1<KIND>, dim3(nb), dim3(256), 0, as_stream(stream), a, b, n, C, ld, part);
    hipLaunchKernelGGL(reduce_stage2, dim3(1), dim3(256), 0, as_stream(stream), part, nb, out);
    CAI_LAUNCH_CHECK(name);
    return CAI_OK;
}

__global__ void log_bwd_kernel(const float* __restrict__ lik, int64_t n, int C, int ld, const float* __restrict__ scale,
                               float coef, float* __restrict__ g) {
    const float s = *scale * coef;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int64_t o = p * ld + (i - p * C);
        g[o] = s / lik[o];
    }
}

__global__ void sqdiff_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                  const float* __restrict__ scale, float coef, float* __restrict__ ga) {
    const float s = *scale * coef;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        ga[i] = s * (a[i] - b[i]);
}

__global__ void act_bwd_kernel(int mode, float prm, const void* __restrict__ y, int yld, const void* __restrict__ g,
                               int gld, void* __restrict__ out, int old, int64_t n, int C, int dt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / C;
        const int c = (int)(i - p * C);
        const float yv = ld_any(y, dt, p * yld + c);
        const float gv = ld_any(g, dt, p * gld + c);
        float m = 1.f;
        if (mode == CAI_MASK_POS) m = yv > 0.f ? 1.f : 0.f;
        else if (mode == CAI_MASK_LEAKY) m = yv > 0.f ? 1.f : prm;
        else if (mode == CAI_MASK_SIGN) m = yv > 0.f ? 1.f : (yv < 0.f ? -1.f : 0.f);
        st_any(out, dt, p * old + c, gv * m);
    }
}

// bf16, C % 8 == 0, 16-byte rows: one 8-channel chunk per thread (the element form above is a scalar load /
// store per element and an int64 division: 1.9 TB/s on cheng2020's 128 x 128 x 192 maps)
__global__ void act_bwd_vec_kernel(int mode, float prm, const bf16* __restrict__ y, int yld, const bf16* __restrict__ g,
                                   int gld, bf16* __restrict__ out, int old, int64_t npix, int nch) {
    const int64_t total = npix * nch;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = i / nch;
        const int c0 = (int)(i - p * nch) * 8;
        const bf16x8 yv = *reinterpret_cast<const bf16x8*>(y + p * yld + c0);
        const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + p * gld + c0);
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float yy = (float)yv[e];
            float m = 1.f;
            if (mode == CAI_MASK_POS) m = yy > 0.f ? 1.f : 0.f;
            else if (mode == CAI_MASK_LEAKY) m = yy > 0.f ? 1.f : prm;
            else if (mode == CAI_MASK_SIGN) m = yy > 0.f ? 1.f : (yy < 0.f ? -1.f : 0.f);
            o[e] = (bf16)((float)gv[e] * m);
        }
        *reinterpret_cast<bf16x8*>(out + p * old + c0) = o;
    }
}

__global__ void cast_kernel(const void* __restrict__ x, int xdt, void* __restrict__ y, int ydt, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        st_any(y, ydt, i, ld_any(x, xdt, i));
}

__global__ __launch_bounds__(256) void uniform_noise_kernel(float* __restrict__ out, int64_t n,
                                                             unsigned long long* __restrict__ state) {
    const unsigned long long seed = __hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long draw = __hip_atomic_load(state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t nq = (n + 3) / 4;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
        unsigned c[4] = {(unsigned)q, (unsigned)((unsigned long long)q >> 32), (unsigned)draw, (unsigned)(draw >> 32)};
        philox4x32_10(c, (unsigned)seed, (unsigned)(seed >> 32));
        float u[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = (float)(c[e] >> 8) * 5.9604644775390625e-8f - 0.5f;
        const int64_t i = 4 * q;
        if (i + 3 < n && ((reinterpret_cast<uintptr_t>(out) & 15) == 0)) {
            *reinterpret_cast<f32x4*>(out + i) = f32x4{u[0], u[1], u[2], u[3]};
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (i + e < n) out[i + e] = u[e];
        }
    }
    // every block has consumed the draw index above before taking a ticket; the last one advances it.
    // Relaxed: nothing in this launch reads what the last block writes (the next launch sees it across
    // the kernel boundary), and an acq_rel ticket would write back / invalidate the L2 once per block
    // (measured 23.8 vs 4.8 us for the 786K-element draw).
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = __hip_atomic_fetch_add(state + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == (unsigned long long)gridDim.x - 1) {
            __hip_atomic_store(state + 1, draw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(state + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// DRAW launches take one arrival per block on the sharded tickets: at most this many blocks (grid-stride)
static constexpr int kDrawBlocks = 1024;

static inline int ew_grid_noise(int64_t n, const cai_noise_src& ns) {
    const int g = ew_grid(n);
    return ns.kind == CAI_NOISE_DRAW ? std::min(g, kDrawBlocks) : g;
}

// the kernels' copy of the noise operand (kind -1: invalid, the error is set); modes other than NOISE get an
// empty BUF operand the kernels never read
static cai_noise_src noise_arg(int mode, const cai_noise_src* n, int C, bool may_draw, const char* who) {
    cai_noise_src s{CAI_NOISE_BUF, 0, nullptr, nullptr, nullptr};
    if (mode != CAI_Q_NOISE) return s;
    bool ok = n != nullptr;
    if (ok) {
        switch (n->kind) {
            case CAI_NOISE_BUF: ok = n->buf && n->ld >= C; break;
            case CAI_NOISE_DRAW:
                ok = may_draw && n->state && n->slot && (reinterpret_cast<uintptr_t>(n->state) & 7) == 0 &&
                     (reinterpret_cast<uintptr_t>(n->slot) & 7) == 0;
                break;
            case CAI_NOISE_REPLAY: ok = n->slot && (reinterpret_cast<uintptr_t>(n->slot) & 7) == 0; break;
            default: ok = false;
        }
    }
    if (!ok) {
        set_error("%s: noise mode needs a valid noise operand (BUF with ld >= C, DRAW%s, REPLAY)", who,
                  may_draw ? "" : " not allowed here");
        s.kind = -1;
        return s;
    }
    return *n;
}

}  // namespace cai

using namespace cai;

extern "C" {

int cai_uniform_noise(float* out, int64_t n, unsigned long long* state, void* stream) {
    CAI_CHECK_ARG(n >= 0 && (n == 0 || out) && state && (reinterpret_cast<uintptr_t>(state) & 7) == 0,
                  "uniform_noise: bad arguments");
    if (n == 0) return CAI_OK;
    // ~8 quads per thread and at most 256 blocks: the arrival tickets of one launch all hit one word (768
    // one-quad blocks measured 12.2 us for 786K elements, the atomics serialised)
    const int64_t nq = (n + 3) / 4;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nq + 2047) / 2048, 256));
    hipLaunchKernelGGL(uniform_noise_kernel, dim3(grid), dim3(256), 0, as_stream(stream), out, n, state);
    CAI_LAUNCH_CHECK("uniform_noise");
    return CAI_OK;
}

int cai_quantize(int mode, int64_t npix, int32_t C, const void* x, int x_dtype, int32_t x_ld, const float* means,
                 int32_t means_ld, int32_t means_per_channel, const cai_noise_src* noise, void* out,
                 int out_dtype, int32_t out_ld, void* stream) {
    CAI_CHECK_ARG(mode == CAI_Q_NOISE || mode == CAI_Q_DEQUANTIZE || mode == CAI_Q_SYMBOLS,
                  "quantize: invalid mode %d", mode);
    CAI_CHECK_ARG(C > 0 && npix >= 0 && x_ld >= C && out_ld >= C, "quantize: bad shape");
    const cai_noise_src ns = noise_arg(mode, noise, C, true, "quantize");
    if (ns.kind < 0) return CAI_EINVAL;
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipLaunchKernelGGL(quantize_kernel, dim3(ew_grid_noise(n, ns)), dim3(256), 0, as_stream(stream), mode, n, C, x,
                       x_dtype, x_ld, means, means_ld, means_per_channel, ns, out, out_dtype, out_ld);
    CAI_LAUNCH_CHECK("quantize");
    return CAI_OK;
}

int cai_gc_fwd(int mode, int64_t npix, int32_t C, const void* x, int x_dtype, int32_t x_ld, const void* scales,
               int32_t s_ld, const void* means, int32_t m_ld, int sm_dtype, const cai_noise_src* noise,
               float scale_bound, float lik_bound, void* q, int q_dtype, int32_t q_ld, float* lik, int32_t lik_ld,
               void* stream) {
    CAI_CHECK_ARG(mode == CAI_Q_NOISE || mode == CAI_Q_DEQUANTIZE, "gc_fwd: invalid mode %d", mode);
    CAI_CHECK_ARG(C > 0 && npix >= 0 && lik, "gc_fwd: bad arguments");
    const cai_noise_src ns = noise_arg(mode, noise, C, true, "gc_fwd");
    if (ns.kind < 0) return CAI_EINVAL;
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipLaunchKernelGGL(gc_fwd_kernel, dim3(ew_grid_noise(n, ns)), dim3(256), 0, as_stream(stream), mode, n, C, x,
                       x_dtype, x_ld, scales, s_ld, means, m_ld, sm_dtype, ns, scale_bound, lik_bound, q, q_dtype,
                       q_ld, lik, lik_ld);
    CAI_LAUNCH_CHECK("gc_fwd");
    return CAI_OK;
}

int cai_gc_bwd(int mode, int64_t npix, int32_t C, const void* x, int x_dtype, int32_t x_ld, const void* scales,
               int32_t s_ld, const void* means, int32_t m_ld, int sm_dtype, const cai_noise_src* noise,
               float scale_bound, float lik_bound, const float* g_lik, int32_t gl_ld, const void* g_q, int gq_dtype,
               int32_t gq_ld, void* dx, int32_t dx_ld, void* dscales, int32_t ds_ld, void* dmeans, int32_t dm_ld,
               void* stream) {
    const int relu = (mode & CAI_GC_SCALES_RELU) != 0;
    mode &= ~CAI_GC_SCALES_RELU;
    CAI_CHECK_ARG(mode == CAI_Q_NOISE || mode == CAI_Q_DEQUANTIZE, "gc_bwd: invalid mode %d", mode);
    CAI_CHECK_ARG(C > 0 && npix >= 0, "gc_bwd: bad arguments");
    const cai_noise_src ns = noise_arg(mode, noise, C, false, "gc_bwd");
    if (ns.kind < 0) return CAI_EINVAL;
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipLaunchKernelGGL(gc_bwd_kernel, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream), mode, relu, n, C, x, x_dtype,
                       x_ld, scales, s_ld, means, m_ld, sm_dtype, ns, scale_bound, lik_bound, g_lik, gl_ld, g_q,
                       gq_dtype, gq_ld, dx, dx_ld, dscales, ds_ld, dmeans, dm_ld);
    CAI_LAUNCH_CHECK("gc_bwd");
    return CAI_OK;
}

int cai_eb_fwd(int mode, int64_t npix, int32_t C, const cai_eb_params* prm, const void* x, int x_dtype, int32_t x_ld,
               const cai_noise_src* noise, float lik_bound, void* q, int q_dtype, int32_t q_ld, float* lik,
               int32_t lik_ld, void* stream) {
    CAI_CHECK_ARG(prm, "eb_fwd: null params");
    CAI_CHECK_ARG(mode == CAI_Q_NOISE || mode == CAI_Q_DEQUANTIZE, "eb_fwd: invalid mode %d", mode);
    CAI_CHECK_ARG(C > 0 && npix >= 0 && lik, "eb_fwd: bad arguments");
    const cai_noise_src ns = noise_arg(mode, noise, C, true, "eb_fwd");
    if (ns.kind < 0) return CAI_EINVAL;
    if (npix * C == 0) return CAI_OK;
    const int gx = (C + 31) / 32;
    // up to EB_FWD_PPL pixel rows per thread (one row per block and pass each took its own table fill: 45 us on
    // C1's y), but never fewer than ~256 blocks where one row per thread gives them (C2's z, 256 pixels: 4 rows
    // per thread on 32 blocks measured 20.9 us against 16.9 on 128 blocks)
    const int64_t rows1 = (npix + 7) / 8;
    int64_t gy = std::min<int64_t>(rows1, std::max<int64_t>((npix + 8 * EB_FWD_PPL - 1) / (8 * EB_FWD_PPL),
                                                            (256 + gx - 1) / gx));
    if (gy > 1024) gy = 1024;
    if (ns.kind == CAI_NOISE_DRAW) gy = std::max<int64_t>(1, std::min<int64_t>(gy, kDrawBlocks / gx));
    hipLaunchKernelGGL(eb_fwd_kernel, dim3(gx, (unsigned)gy), dim3(256), 0, as_stream(stream), mode, npix, C,
                       *prm, x, x_dtype, x_ld, ns, lik_bound, q, q_dtype, q_ld, lik, lik_ld);
    CAI_LAUNCH_CHECK("eb_fwd");
    return CAI_OK;
}

static int eb_bwd_splits(int64_t npix) {
    // EB_BWD_PPL pixels per thread; the blocks of one channel hand their sums to the last arriver.  (One pixel
    // per thread, 64 blocks per channel, repeated every block's table fill, 60 wave sums and hand-off for a single
    // chain pair: C1's backward took 220 us.)
    const int64_t per_block = 256 * EB_BWD_PPL;
    return (int)std::max<int64_t>(1, std::min<int64_t>((npix + per_block - 1) / per_block, 64));
}
static int eb_aux_blocks(int C) { return (C + EB_AUX_CH - 1) / EB_AUX_CH; }

size_t cai_eb_scratch_bytes(int64_t npix, int32_t C) {
    if (npix < 0 || C <= 0) return 0;
    const size_t bwd = (size_t)C * eb_bwd_splits(npix) * EB_NP * sizeof(float);
    const size_t aux = (size_t)eb_aux_blocks(C) * sizeof(float);
    return std::max(bwd, aux) + 256;
}

int cai_eb_bwd(int mode, int64_t npix, int32_t C, const cai_eb_params* prm, const void* x, int x_dtype, int32_t x_ld,
               const cai_noise_src* noise, float lik_bound, const float* g_lik, int32_t gl_ld,
               const void* g_q, int gq_dtype, int32_t gq_ld, void* dx, int32_t dx_ld, const cai_eb_grads* grads,
               float* scratch, size_t scratch_bytes, uint32_t* tickets, void* stream) {
    CAI_CHECK_ARG(prm && grads, "eb_bwd: null params/grads");
    CAI_CHECK_ARG(mode == CAI_Q_NOISE || mode == CAI_Q_DEQUANTIZE, "eb_bwd: invalid mode %d", mode);
    CAI_CHECK_ARG(C >= 0 && npix >= 0, "eb_bwd: bad arguments");
    const cai_noise_src ns = noise_arg(mode, noise, C > 0 ? C : 1, false, "eb_bwd");
    if (ns.kind < 0) return CAI_EINVAL;
    for (int i = 0; i < 5; ++i) CAI_CHECK_ARG(grads->matrix[i] && grads->bias[i], "eb_bwd: null grad");
    for (int i = 0; i < 4; ++i) CAI_CHECK_ARG(grads->factor[i], "eb_bwd: null grad");
    if (C == 0) return CAI_OK;
    // without scratch / tickets: one block per channel (no hand-off)
    const bool split = scratch && tickets && scratch_bytes >= cai_eb_scratch_bytes(npix, C);
    const int S = split ? eb_bwd_splits(npix) : 1;
    hipLaunchKernelGGL(eb_bwd_kernel, dim3(C, S), dim3(256), 0, as_stream(stream), mode, npix, C, *prm, x,
                       x_dtype, x_ld, ns, lik_bound, g_lik, gl_ld, g_q, gq_dtype, gq_ld, dx, dx_ld,
                       *grads, scratch, tickets);
    CAI_LAUNCH_CHECK("eb_bwd");
    return CAI_OK;
}

int cai_eb_aux_loss(int32_t C, const cai_eb_params* prm, const float* target, float* loss, const float* g_loss,
                    float* dquantiles, int32_t accumulate, float* scratch, size_t scratch_bytes, uint32_t* ticket,
                    void* stream) {
    CAI_CHECK_ARG(prm && target && C > 0, "eb_aux_loss: bad arguments");
    CAI_CHECK_ARG(!dquantiles || g_loss, "eb_aux_loss: dquantiles needs g_loss");
    const int nb = eb_aux_blocks(C);
    CAI_CHECK_ARG(nb == 1 || (scratch && ticket && scratch_bytes >= (size_t)nb * sizeof(float)),
                  "eb_aux_loss: %d channels need scratch and a ticket", C);
    hipLaunchKernelGGL(eb_aux_kernel, dim3(nb), dim3(256), 0, as_stream(stream), C, *prm, target, loss, g_loss,
                       dquantiles, accumulate, scratch, ticket);
    CAI_LAUNCH_CHECK("eb_aux_loss");
    return CAI_OK;
}


// ---------------------------------------------------------------------------
// RD loss in two launches (examples/train.py:68-82): stage 1 sums log(lik) of
// every likelihood tensor and (x_hat - x)^2 as one grid (grid.y = segment),
// stage 2 (one block) folds the per-block partials in a fixed order and
// forms {loss, mse, bpp}.  The backward is one elementwise launch over all
// segments with the upstream scalars read on the device.
// ---------------------------------------------------------------------------
constexpr int RD_BLOCKS = 256;

// one segment's sum over a grid-stride range: 16-byte loads, four independent loads in flight per thread
// (a scalar loop over 3 M elements ran at ~1 TB/s, latency-bound on its loop-carried accumulator)
__device__ __forceinline__ float rd_sum(const float* __restrict__ a, const float* __restrict__ t, int64_t n, bool SQ) {
    const int64_t tid = blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t done = 0;
    if ((((uintptr_t)a | (SQ ? (uintptr_t)t : (uintptr_t)0)) & 15) == 0) {
        const int64_t n4 = n >> 2;
        const f32x4* a4 = reinterpret_cast<const f32x4*>(a);
        const f32x4* t4 = reinterpret_cast<const f32x4*>(t);
        int64_t i = tid;
        for (; i + 3 * stride < n4; i += 4 * stride) {
            f32x4 va[4], vt[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                va[j] = a4[i + j * stride];
                if (SQ) vt[j] = t4[i + j * stride];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (SQ) {
                        const float d = va[j][e] - vt[j][e];
                        acc[j] += d * d;
                    } else {
                        acc[j] += logf(va[j][e]);
                    }
                }
        }
        for (; i < n4; i += stride) {
            const f32x4 va = a4[i];
            const f32x4 vt = SQ ? t4[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (SQ) {
                    const float d = va[e] - vt[e];
                    acc[e] += d * d;
                } else {
                    acc[e] += logf(va[e]);
                }
            }
        }
        done = n4 << 2;
    }
    for (int64_t i = done + tid; i < n; i += stride) {
        if (SQ) {
            const float d = a[i] - t[i];
            acc[0] += d * d;
        } else {
            acc[0] += logf(a[i]);
        }
    }
    return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

__global__ __launch_bounds__(256) void rd_stage1(cai_rd_inputs in, float* __restrict__ part) {
    __shared__ float red[4];
    const int seg = blockIdx.y;
    const bool sq = seg == in.nlik;
    const float* a = sq ? in.x_hat : (seg == 0 ? in.lik[0] : (seg == 1 ? in.lik[1] : (seg == 2 ? in.lik[2] : in.lik[3])));
    const int64_t n = sq ? in.n : (seg == 0 ? in.lik_n[0] : (seg == 1 ? in.lik_n[1] : (seg == 2 ? in.lik_n[2] : in.lik_n[3])));
    const float acc = sq ? rd_sum(a, in.target, n, true) : rd_sum(a, nullptr, n, false);
    const float r = block_sum<256>(acc, red);
    if (threadIdx.x == 0) part[seg * RD_BLOCKS + blockIdx.x] = r;
}

__global__ __launch_bounds__(256) void rd_stage2(const float* __restrict__ part, int nlik, float lmbda, float bpp_coef,
                                                 float inv_n, float* __restrict__ out) {
    __shared__ float red[4];
    float bpp = 0.f, sse = 0.f;
    for (int seg = 0; seg <= nlik; ++seg) {
        const float v = block_sum<256>(part[seg * RD_BLOCKS + threadIdx.x], red);
        if (seg < nlik) bpp += v; else sse = v;
    }
    if (threadIdx.x == 0) {
        const float b = bpp * bpp_coef, m = sse * inv_n;
        out[0] = lmbda * m + b;
        out[1] = m;
        out[2] = b;
    }
}


__global__ __launch_bounds__(256) void rd_bwd_kernel(cai_rd_inputs in, float lmbda, float bpp_coef,
                                                     const float* __restrict__ g_loss, const float* __restrict__ g_mse,
                                                     const float* __restrict__ g_bpp, float* __restrict__ dxh,
                                                     cai_rd_grads out) {
    const int seg = blockIdx.y;
    const float gl = g_loss ? *g_loss : 0.f;
    if (seg == in.nlik) {   // d loss / d x_hat = (g_mse + lmbda g_loss) * 2 (x_hat - x) / n
        const float k = ((g_mse ? *g_mse : 0.f) + lmbda * gl) * (2.f / (float)in.n);
        for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < in.n; i += (int64_t)gridDim.x * 256)
            dxh[i] = k * (in.x_hat[i] - in.target[i]);
        return;
    }
    const float* l = seg == 0 ? in.lik[0] : (seg == 1 ? in.lik[1] : (seg == 2 ? in.lik[2] : in.lik[3]));
    float* d = seg == 0 ? out.dlik[0] : (seg == 1 ? out.dlik[1] : (seg == 2 ? out.dlik[2] : out.dlik[3]));
    const int64_t n = seg == 0 ? in.lik_n[0] : (seg == 1 ? in.lik_n[1] : (seg == 2 ? in.lik_n[2] : in.lik_n[3]));
    const float k = ((g_bpp ? *g_bpp : 0.f) + gl) * bpp_coef;   // d bpp / d lik = coef / lik
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = k / l[i];
}

size_t cai_reduce_workspace_bytes(int64_t n) { return (size_t)red_blocks(n) * sizeof(float); }

int cai_sum_log(const float* lik, int64_t npix, int32_t C, int32_t ld, float* out, void* workspace, size_t ws_bytes,
                void* stream) {
    CAI_CHECK_ARG(C > 0 && ld >= C, "sum_log: bad shape");
    return run_reduce<0>(lik, nullptr, npix * C, C, ld, out, workspace, ws_bytes, stream, "sum_log");
}

int cai_sum_sqdiff(const float* a, const float* b, int64_t n, float* out, void* workspace, size_t ws_bytes,
                   void* stream) {
    return run_reduce<1>(a, b, n, 1, 1, out, workspace, ws_bytes, stream, "sum_sqdiff");
}

int cai_sqnorm(const float* g, int64_t n, float* out, void* workspace, size_t ws_bytes, void* stream) {
    return run_reduce<2>(g, nullptr, n, 1, 1, out, workspace, ws_bytes, stream, "sqnorm");
}

int cai_log_bwd(const float* lik, int64_t npix, int32_t C, int32_t ld, const float* scale, float coef, float* g,
                void* stream) {
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    hipLaunchKernelGGL(log_bwd_kernel, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream), lik, n, C, ld, scale, coef, g);
    CAI_LAUNCH_CHECK("log_bwd");
    return CAI_OK;
}

int cai_sqdiff_bwd(const float* a, const float* b, int64_t n, const float* scale, float coef, float* ga,
                   void* stream) {
    if (n == 0) return CAI_OK;
    hipLaunchKernelGGL(sqdiff_bwd_kernel, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream), a, b, n, scale, coef, ga);
    CAI_LAUNCH_CHECK("sqdiff_bwd");
    return CAI_OK;
}

int cai_act_bwd(int mask_mode, float param, const void* y, int32_t y_ld, const void* g, int32_t g_ld, void* out,
                int32_t out_ld, int64_t npix, int32_t C, int dtype, void* stream) {
    const int64_t n = npix * C;
    if (n == 0) return CAI_OK;
    const bool a16 = ((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(out)) &
                      15) == 0;
    if (dtype == CAI_BF16 && C % 8 == 0 && y_ld % 8 == 0 && g_ld % 8 == 0 && out_ld % 8 == 0 && a16) {
        const int nch = C / 8;
        hipLaunchKernelGGL(act_bwd_vec_kernel, dim3(ew_grid(npix * nch)), dim3(256), 0, as_stream(stream), mask_mode,
                           param, static_cast<const bf16*>(y), y_ld, static_cast<const bf16*>(g), g_ld,
                           static_cast<bf16*>(out), out_ld, npix, nch);
    } else {
        hipLaunchKernelGGL(act_bwd_kernel, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream), mask_mode, param, y, y_ld,
                           g, g_ld, out, out_ld, n, C, dtype);
    }
    CAI_LAUNCH_CHECK("act_bwd");
    return CAI_OK;
}

int cai_cast(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, void* stream) {
    if (n == 0) return CAI_OK;
    hipLaunchKernelGGL(cast_kernel, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream), x, x_dtype, y, y_dtype, n);
    CAI_LAUNCH_CHECK("cast");
    return CAI_OK;
}


static int check_rd(const cai_rd_inputs* in) {
    CAI_CHECK_ARG(in && in->nlik >= 1 && in->nlik <= 4 && in->x_hat && in->target && in->n > 0, "rd_loss: bad inputs");
    for (int i = 0; i < in->nlik; ++i) CAI_CHECK_ARG(in->lik[i] && in->lik_n[i] > 0, "rd_loss: bad likelihood %d", i);
    return CAI_OK;
}

size_t cai_rd_loss_workspace_bytes(void) { return (size_t)5 * RD_BLOCKS * sizeof(float); }

int cai_rd_loss_fwd(const cai_rd_inputs* in, float lmbda, float bpp_coef, float* out, void* workspace,
                    size_t ws_bytes, void* stream) {
    int rc = check_rd(in);
    if (rc) return rc;
    CAI_CHECK_ARG(out && workspace && ws_bytes >= cai_rd_loss_workspace_bytes(), "rd_loss_fwd: bad output/workspace");
    float* part = reinterpret_cast<float*>(workspace);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(rd_stage1, dim3(RD_BLOCKS, in->nlik + 1), dim3(256), 0, st, *in, part);
    hipLaunchKernelGGL(rd_stage2, dim3(1), dim3(256), 0, st, part, in->nlik, lmbda, bpp_coef, 1.f / (float)in->n, out);
    CAI_LAUNCH_CHECK("rd_loss_fwd");
    return CAI_OK;
}

int cai_rd_loss_bwd(const cai_rd_inputs* in, float lmbda, float bpp_coef, const float* g_loss, const float* g_mse,
                    const float* g_bpp, float* dx_hat, const cai_rd_grads* grads, void* stream) {
    int rc = check_rd(in);
    if (rc) return rc;
    CAI_CHECK_ARG(dx_hat && grads, "rd_loss_bwd: null output");
    for (int i = 0; i < in->nlik; ++i) CAI_CHECK_ARG(grads->dlik[i], "rd_loss_bwd: null dlik[%d]", i);
    int64_t mx = in->n;
    for (int i = 0; i < in->nlik; ++i) mx = std::max(mx, in->lik_n[i]);
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (mx + 255) / 256));
    hipLaunchKernelGGL(rd_bwd_kernel, dim3(gx, in->nlik + 1), dim3(256), 0, as_stream(stream), *in, lmbda, bpp_coef,
                       g_loss, g_mse, g_bpp, dx_hat, *grads);
    CAI_LAUNCH_CHECK("rd_loss_bwd");
    return CAI_OK;
}

}  // extern "C"
