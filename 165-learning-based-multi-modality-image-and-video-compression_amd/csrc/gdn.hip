// GDN / IGDN (compressai/layers/gdn.py:41-92) on CDNA4 MFMA.
//
//   beta  = max(beta_raw,  sqrt(beta_min + ped))^2 - ped      (ops/parametrizers.py:61-64)
//   gamma = max(gamma_raw, sqrt(ped))^2 - ped                  (ped = reparam_offset^2)
//   norm[p,i] = beta_i + sum_j gamma[i,j] x[p,j]^2             (F.conv2d(x**2, gamma, beta))
//   out = x * rsqrt(norm)   (inverse: x * sqrt(norm))
//
// The C x C contraction is a small-K GEMM (K = C = 128/192): per 64-pixel tile
// the x tile sits in LDS (rows padded by 16 B: conflict-free ds_read_b128),
// x^2 is formed in registers on the way into v_mfma_f32_16x16x32_bf16 (or the
// exact-fp32 16x16x4 path), the normalisation is fused into the epilogue and
// the tile leaves through LDS as 16-byte stores.  HBM traffic per pixel is
// the algorithmic minimum: read x once, write y once (fwd); read x, dy once,
// write dx, u once (bwd).  The forward keeps its gamma fragments in registers
// for the whole (persistent) block.
//
// Backward (per pixel, u_i = dLoss/dnorm_i):
//   GDN : r = rsqrt(norm), u_i = -0.5 g_i x_i r_i^3, dx_j = g_j r_j + 2 x_j sum_i gamma[i,j] u_i
//   IGDN: s = sqrt(norm),  u_i =  0.5 g_i x_i / s_i, dx_j = g_j s_j + 2 x_j sum_i gamma[i,j] u_i
//   dgamma[i,j] = sum_p u_i x_j^2 ; dbeta_i = sum_p u_i   (cai_gdn_param_grad: split-K MFMA
//   through the 1x1 wgrad kernel + fixed-order column sums), then the LowerBound rule.
#include "common.hpp"
#include "mfma.hpp"
#include "reduce_jobs.hpp"

#include <algorithm>

namespace cai {

int colsum_any(int dtype, const void* g, int64_t npix, int C, int ld, float* out, int accumulate, void* ws, size_t wsb,
               hipStream_t st);
// lane-local kernels (gdn_lane.hip)
bool gdn_lane_fwd_ok(int C, int64_t npix, int x_ld, int y_ld);
void launch_gdn_fwd_lane(const void* x, int x_ld, int64_t npix, int C, const void* g, const float* b, int inv, void* y,
                         int y_ld, hipStream_t st);
bool gdn_lane_bwd_ok(int C, int64_t npix, int x_ld, int dy_ld, int dx_ld);
int gdn_lane_bwd_blocks(int64_t npix);
void launch_gdn_bwd_lane(const void* x, int x_ld, const void* dy, int dy_ld, int64_t npix, int C, const void* gop,
                         const float* beta, int inv, void* dx, int dx_ld, float* part, int nblk, hipStream_t st);
// A/B knob: CAI_GDN_LANE=0 keeps the LDS-tile kernels (gdn_fwd_kernel, gdn_bwd_fused_kernel); read at every
// call (host side, a few hundred ns) so the parity tests can compare both kernels in one process
static bool gdn_lane_on() {
    const char* e = getenv("CAI_GDN_LANE");
    return !(e && *e == '0');
}
size_t colsum_ws_bytes(int64_t npix, int C);

__device__ __forceinline__ s16x4 ds_tr16(const char* base, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + byte_off));
}

template <typename T>
__device__ __forceinline__ f32x4 mma_sq(u32x4 a, u32x4 b, f32x4 c, bool square);
template <>
__device__ __forceinline__ f32x4 mma_sq<bf16>(u32x4 a, u32x4 b, f32x4 c, bool square) {
    bf16x8 av = __builtin_bit_cast(bf16x8, a);
    if (square) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float f = (float)av[e];
            av[e] = (bf16)(f * f);
        }
    }
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mma_sq<float>(u32x4 a, u32x4 b, f32x4 c, bool square) {
    f32x4 av = __builtin_bit_cast(f32x4, a);
    if (square) av = av * av;
    const f32x4 bv = __builtin_bit_cast(f32x4, b);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], c, 0, 0, 0);
    return c;
}

constexpr int GBM = 64;    // pixels per tile

// Workgroup barrier for LDS hand-offs that leaves global loads in flight:
// __syncthreads() also waits for every outstanding vector-memory operation,
// which would drain the next tile's register prefetch at each barrier.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}
constexpr int GNT = 256;   // 4 waves, split over channels (1 x 4)

template <typename T, int C>
struct GdnGeo {
    static constexpr int RB = C * (int)sizeof(T);   // bytes of one pixel row
    static constexpr int RS = RB + 16;               // padded LDS row stride
    static constexpr int KB = RB / 64;               // 64-byte K blocks per row
    // 4 waves split WM (pixels) x WN (channels); every wave owns >= one 16-col tile
    static constexpr int WN = (C % 64 == 0) ? 4 : ((C % 32 == 0) ? 2 : 1);
    static constexpr int WM = 4 / WN;
    static constexpr int NW = C / WN;                // channels per wave
    static constexpr int TN = NW / 16;               // 16-col tiles per wave
    static constexpr int TM = GBM / (16 * WM);       // 16-row tiles per wave
    __device__ static int col0(int wave) { return (wave % WN) * NW; }
    __device__ static int row0(int wave) { return (wave / WN) * (GBM / WM); }
    static constexpr int CHR = RB / 16;              // 16-byte chunks per row
    static constexpr int TILE_CH = GBM * CHR;        // chunks per tile
    static constexpr int CPT = (TILE_CH + GNT - 1) / GNT;
    static constexpr int TILE_LDS = GBM * RS;
};

// Rows past the end are stored to a sink instead of being skipped: every store is issued, so the
// compiler's vmcnt bookkeeping never meets a path with fewer memory operations (a skipped store there
// turns the next wait on the register prefetch into vmcnt(0), draining the prefetched tiles).
__device__ __attribute__((aligned(64))) u32x4 cai_gdn_sink[16];

// CPT stores to distinct sink slots (identical stores to one address would be merged into one, and the
// prologue would no longer match the loop's per-iteration store count), pinned in issue order
template <int CPT>
__device__ __forceinline__ void sink_stores(int base) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < CPT; ++i) cai_gdn_sink[base + i] = u32x4{0u, 0u, 0u, 0u};
    __builtin_amdgcn_sched_barrier(0);
}

template <typename T, int C>
struct TileRegs {
    u32x4 v[GdnGeo<T, C>::CPT];
};
template <typename T, int C>
struct BFrags {
    u32x4 v[GdnGeo<T, C>::TN][GdnGeo<T, C>::KB];
};
template <typename T, int C>
struct Acc {
    f32x4 v[GdnGeo<T, C>::TM][GdnGeo<T, C>::TN];
};

// stage a [GBM][C] pixel-major tile (ld elements per pixel) into registers
template <typename T, int C>
__device__ __forceinline__ void tile_load(TileRegs<T, C>& R, const T* src, int ld, int64_t p0, int64_t npix) {
    auto& r = R.v;
    using G = GdnGeo<T, C>;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * GNT + threadIdx.x;
        const int row = id / G::CHR, ch = id - (id / G::CHR) * G::CHR;
        const int64_t p = p0 + row;
        if (id < G::TILE_CH && p < npix)
            r[i] = *reinterpret_cast<const u32x4*>(src + p * ld + ch * (16 / sizeof(T)));
        else
            r[i] = u32x4{0u, 0u, 0u, 0u};
    }
}
// the same with every load issued: rows past the end re-read the last pixel (the forward's rows are
// independent; those results go to the sink)
template <typename T, int C>
__device__ __forceinline__ void tile_load_all(TileRegs<T, C>& R, const T* src, int ld, int64_t p0, int64_t npix) {
    using G = GdnGeo<T, C>;
    static_assert(G::TILE_CH % GNT == 0, "tile chunks");
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * GNT + threadIdx.x;
        const int row = id / G::CHR, ch = id - (id / G::CHR) * G::CHR;
        const int64_t p = min(p0 + row, npix - 1);
        R.v[i] = *reinterpret_cast<const u32x4*>(src + p * ld + ch * (16 / sizeof(T)));
    }
}
template <typename T, int C>
__device__ __forceinline__ void lds_to_global_all(const char* lds, T* dst, int ld, int64_t p0, int64_t npix) {
    using G = GdnGeo<T, C>;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * GNT + threadIdx.x;
        const int row = id / G::CHR, ch = id - (id / G::CHR) * G::CHR;
        const int64_t p = p0 + row;
        u32x4* d = p < npix ? reinterpret_cast<u32x4*>(dst + p * ld + ch * (16 / sizeof(T))) : cai_gdn_sink;
        *d = *reinterpret_cast<const u32x4*>(lds + row * G::RS + ch * 16);
    }
}
template <typename T, int C>
__device__ __forceinline__ void tile_to_lds(const TileRegs<T, C>& R, char* lds) {
    using G = GdnGeo<T, C>;
    const auto& r = R.v;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * GNT + threadIdx.x;
        const int row = id / G::CHR, ch = id - (id / G::CHR) * G::CHR;
        if (G::TILE_CH % GNT == 0 || id < G::TILE_CH) *reinterpret_cast<u32x4*>(lds + row * G::RS + ch * 16) = r[i];
    }
}
template <typename T, int C>
__device__ __forceinline__ void lds_to_global(const char* lds, T* dst, int ld, int64_t p0, int64_t npix) {
    using G = GdnGeo<T, C>;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * GNT + threadIdx.x;
        const int row = id / G::CHR, ch = id - (id / G::CHR) * G::CHR;
        const int64_t p = p0 + row;
        if (id < G::TILE_CH && p < npix)
            *reinterpret_cast<u32x4*>(dst + p * ld + ch * (16 / sizeof(T))) =
                *reinterpret_cast<const u32x4*>(lds + row * G::RS + ch * 16);
    }
}

// B fragments of a [C][C] row-major matrix for this wave's column slice
template <typename T, int C>
__device__ __forceinline__ void load_bfrag(BFrags<T, C>& FB, const T* mat, int wave) {
    using G = GdnGeo<T, C>;
    auto& fb = FB.v;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn) {
        const int n = G::col0(wave) + tn * 16 + (lane & 15);
#pragma unroll
        for (int kb = 0; kb < G::KB; ++kb)
            fb[tn][kb] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(mat + (int64_t)n * C) + kb * 64 +
                                                         16 * (lane >> 4));
    }
}

template <typename T, int C>
__device__ __forceinline__ void tile_gemm(Acc<T, C>& ACC, const char* lds, const BFrags<T, C>& FB, bool square,
                                          int wave) {
    using G = GdnGeo<T, C>;
    auto& acc = ACC.v;
    const auto& fb = FB.v;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < G::TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < G::KB; ++kb) {
        u32x4 fa[G::TM];
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) {
            const int row = G::row0(wave) + tm * 16 + (lane & 15);
            fa[tm] = *reinterpret_cast<const u32x4*>(lds + row * G::RS + kb * 64 + 16 * (lane >> 4));
        }
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < G::TN; ++tn) acc[tm][tn] = mma_sq<T>(fa[tm], fb[tn][kb], acc[tm][tn], square);
    }
}

// The same product transposed, norm^T = gamma . (x^2)^T: gamma's fragments as the A operand, the x^2 tile as
// B.  Each lane then holds 4 CONSECUTIVE channels of one pixel (acc[tn][tm][r]: channel col0 + 16 tn +
// 4 (lane >> 4) + r, pixel row0 + 16 tm + (lane & 15)), so the elementwise stage reads x and writes y as one
// 8-byte (bf16) / 16-byte (fp32) LDS access per 4 elements -- conflict-free across the wave -- instead of
// four 2-byte accesses that share bank words.
template <typename T, int C>
struct AccT {
    f32x4 v[GdnGeo<T, C>::TN][GdnGeo<T, C>::TM];
};
template <typename T, int C>
__device__ __forceinline__ void tile_gemm_t(AccT<T, C>& ACC, const char* lds, const BFrags<T, C>& FB, int wave) {
    using G = GdnGeo<T, C>;
    auto& acc = ACC.v;
    const auto& fb = FB.v;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) acc[tn][tm] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < G::KB; ++kb) {
        u32x4 fx[G::TM];
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) {
            const int row = G::row0(wave) + tm * 16 + (lane & 15);
            fx[tm] = *reinterpret_cast<const u32x4*>(lds + row * G::RS + kb * 64 + 16 * (lane >> 4));
        }
#pragma unroll
        for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
            for (int tm = 0; tm < G::TM; ++tm) acc[tn][tm] = mma16<T>(fb[tn][kb], fx[tm], acc[tn][tm]);
    }
}

// 4 consecutive elements of a row at an element offset that is a multiple of 4
template <typename T>
struct Quad;
template <>
struct Quad<bf16> {
    typedef bf16x4 V;
};
template <>
struct Quad<float> {
    typedef f32x4 V;
};

template <typename T>
__device__ __forceinline__ T* lds_elem(char* lds, int rs, int row, int col) {
    return reinterpret_cast<T*>(lds + row * rs) + col;
}

template <typename T, int C>
__global__ __launch_bounds__(GNT, (sizeof(T) == 2 && C <= 192) ? 2 : 1) void gdn_fwd_kernel(const T* __restrict__ x, int x_ld, int64_t npix,
                                                         const T* __restrict__ gamma, const float* __restrict__ beta,
                                                         int inverse, T* __restrict__ y, int y_ld) {
    using G = GdnGeo<T, C>;
    __shared__ __attribute__((aligned(16))) char lds[2 * G::TILE_LDS];
    char* lsq = lds + G::TILE_LDS;   // x^2, squared once per tile (not by each wave that reads it)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    BFrags<T, C> fb;
    load_bfrag<T, C>(fb, gamma, wave);
    float bq[G::TN][4];   // beta of this lane's 4 channels per channel tile (transposed GEMM layout)
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
        for (int r = 0; r < 4; ++r) bq[tn][r] = beta[G::col0(wave) + tn * 16 + (lane >> 4) * 4 + r];

    // persistent blocks, two tiles in flight per block (register sets A / B), every load and store issued
    // (clamped rows, sink stores) and a counted loop over tile pairs: the straight-line body lets each
    // step wait for its own set only (see the fused backward below)
    const int64_t ntiles = (npix + GBM - 1) / GBM;
    const int64_t stride = gridDim.x;
    const int64_t last = ntiles - 1;
    // the widest tiles keep one set (a second one would spill: C = 160+ bf16, 128+ fp32)
    constexpr bool PAIR = sizeof(T) == 2 ? C <= 128 : C <= 96;
    TileRegs<T, C> ra, rb;
    int64_t tile = blockIdx.x;
    tile_load_all<T, C>(ra, x, x_ld, min(tile, last) * GBM, npix);
    sink_stores<G::CPT>(0);
    if constexpr (PAIR) {
        tile_load_all<T, C>(rb, x, x_ld, min(tile + stride, last) * GBM, npix);
        sink_stores<G::CPT>(8);
    }
    auto step = [&](TileRegs<T, C>& rx, int64_t cur, int64_t nxt) {
        lds_barrier();                       // the previous tile's store has read lds
        tile_to_lds<T, C>(rx, lds);
        {
            TileRegs<T, C> sq;
#pragma unroll
            for (int i = 0; i < G::CPT; ++i) sq.v[i] = sq_chunk<T>(rx.v[i]);
            tile_to_lds<T, C>(sq, lsq);
        }
        tile_load_all<T, C>(rx, x, x_ld, nxt * GBM, npix);
        lds_barrier();
        AccT<T, C> A;
        tile_gemm_t<T, C>(A, lsq, fb, wave);
        auto& acc = A.v;
        // normalise: out = x * rsqrt(norm)  (or sqrt); lane: 4 consecutive channels of one pixel
        typedef typename Quad<T>::V QV;
#pragma unroll
        for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
            for (int tm = 0; tm < G::TM; ++tm) {
                const int col = G::col0(wave) + tn * 16 + (lane >> 4) * 4;
                const int row = G::row0(wave) + tm * 16 + (lane & 15);
                const QV xq = *reinterpret_cast<const QV*>(lds + row * G::RS + col * (int)sizeof(T));
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float nv = acc[tn][tm][r] + bq[tn][r];
                    const float rs = rsqrtf(nv);
                    acc[tn][tm][r] = to_f32(xq[r]) * (inverse ? nv * rs : rs);
                }
            }
        lds_barrier();
#pragma unroll
        for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
            for (int tm = 0; tm < G::TM; ++tm) {
                const int col = G::col0(wave) + tn * 16 + (lane >> 4) * 4;
                const int row = G::row0(wave) + tm * 16 + (lane & 15);
                QV yq;
#pragma unroll
                for (int r = 0; r < 4; ++r) yq[r] = from_f32<T>(acc[tn][tm][r]);
                *reinterpret_cast<QV*>(lds + row * G::RS + col * (int)sizeof(T)) = yq;
            }
        lds_barrier();
        lds_to_global_all<T, C>(lds, y, y_ld, cur * GBM, npix);
    };
    const int64_t mine = tile < ntiles ? (ntiles - tile + stride - 1) / stride : 0;
    if constexpr (PAIR) {
        for (int64_t it = 0; it < mine / 2; ++it, tile += 2 * stride) {
            step(ra, tile, min(tile + 2 * stride, last));
            step(rb, tile + stride, min(tile + 3 * stride, last));
        }
        if (mine & 1) step(ra, tile, last);
    } else {
        for (int64_t it = 0; it < mine; ++it, tile += stride) step(ra, tile, min(tile + stride, last));
    }
}

template <typename T, int C>
__global__ __launch_bounds__(GNT, 1) void gdn_bwd_kernel(const T* __restrict__ x, int x_ld, const T* __restrict__ dy,
                                                         int dy_ld, int64_t npix, const T* __restrict__ gamma_op,
                                                         const float* __restrict__ beta, int inverse,
                                                         T* __restrict__ dx, int dx_ld, T* __restrict__ u) {
    using G = GdnGeo<T, C>;
    __shared__ __attribute__((aligned(16))) char lds[3 * G::TILE_LDS];
    char* Lx = lds;
    char* Lg = lds + G::TILE_LDS;
    char* Lu = lds + 2 * G::TILE_LDS;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const T* gammaT = gamma_op + (int64_t)C * C;
    float bv[G::TN];
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn) bv[tn] = beta[G::col0(wave) + tn * 16 + (lane & 15)];

    const int64_t p0 = (int64_t)blockIdx.x * GBM;
    {
        TileRegs<T, C> r;
        tile_load<T, C>(r, x, x_ld, p0, npix);
        tile_to_lds<T, C>(r, Lx);
        tile_load<T, C>(r, dy, dy_ld, p0, npix);
        tile_to_lds<T, C>(r, Lg);
    }
    __syncthreads();
    Acc<T, C> A;
    auto& acc = A.v;
    {
        BFrags<T, C> fb;
        load_bfrag<T, C>(fb, gamma_op, wave);
        tile_gemm<T, C>(A, Lx, fb, true, wave);
    }
    // u = dLoss/dnorm into LDS; t1 = g * r (or g * s) replaces g in LDS
#pragma unroll
    for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < G::TN; ++tn) {
            const int col = G::col0(wave) + tn * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = G::row0(wave) + tm * 16 + (lane >> 4) * 4 + r;
                const float xv = to_f32(*lds_elem<T>(Lx, G::RS, row, col));
                T* gp = lds_elem<T>(Lg, G::RS, row, col);
                const float gv = to_f32(*gp);
                const float nv = acc[tm][tn][r] + bv[tn];
                float uv, t1;
                if (inverse) {
                    const float s = sqrtf(nv);
                    t1 = gv * s;
                    uv = 0.5f * gv * xv / s;
                } else {
                    const float rr = rsqrtf(nv);
                    t1 = gv * rr;
                    uv = -0.5f * gv * xv * rr * rr * rr;
                }
                *gp = from_f32<T>(t1);
                *lds_elem<T>(Lu, G::RS, row, col) = from_f32<T>(uv);
            }
        }
    __syncthreads();
    lds_to_global<T, C>(Lu, u, C, p0, npix);
    {
        BFrags<T, C> fb;
        load_bfrag<T, C>(fb, gammaT, wave);
        tile_gemm<T, C>(A, Lu, fb, false, wave);
    }
    // dx = t1 + 2 x (u gamma)  -> written over t1 in LDS
#pragma unroll
    for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < G::TN; ++tn) {
            const int col = G::col0(wave) + tn * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = G::row0(wave) + tm * 16 + (lane >> 4) * 4 + r;
                const float xv = to_f32(*lds_elem<T>(Lx, G::RS, row, col));
                T* gp = lds_elem<T>(Lg, G::RS, row, col);
                *gp = from_f32<T>(to_f32(*gp) + 2.f * xv * acc[tm][tn][r]);
            }
        }
    __syncthreads();
    lds_to_global<T, C>(Lg, dx, dx_ld, p0, npix);
}

// ---------------------------------------------------------------------------
// Fused backward (bf16, C in {64, 128}): dx AND the parameter gradients in one
// pass over x and dy.  Per 64-pixel tile (persistent blocks, next tile's x / dy
// prefetched into registers while this one is computed):
//   norm = x^2 gamma^T + beta          (MFMA, gamma fragments held in registers)
//   u, t1 = g*r (g*s)                  (fp32, u kept as a bf16 LDS tile)
//   dx = t1 + 2 x (u gamma)            (MFMA, gamma^T fragments in registers)
//   dgamma += u^T x^2                  (MFMA with the pixels as K: operands are
//                                       columns of the [pixel][channel] tiles,
//                                       read with ds_read_b64_tr_b16)
//   dbeta  += column sums of u (fp32)
// Each block leaves its fp32 dgamma / dbeta partial in the workspace; a
// fixed-order reduce over blocks applies the LowerBound / reparametrization
// rule (deterministic).  HBM traffic per pixel: read x, dy, write dx (6C B)
// -- the two-kernel path also writes and re-reads u and re-reads x (+6C B)
// and runs a separate split-K weight-gradient GEMM.
// ---------------------------------------------------------------------------
constexpr int FNT = 512;   // 8 waves

#ifndef CAI_GDN_RS_PAD
#define CAI_GDN_RS_PAD 32       // bytes of padding per LDS row of the fused backward's tiles (A/B: 16 / 32 / 48 / 80 -> 32 best, -2 %)
#endif

template <int C>
struct FusedGeo {
    static constexpr int RS = 2 * C + CAI_GDN_RS_PAD;   // padded LDS row (bf16)
    static constexpr int KB = C / 32;               // 32-deep K blocks over channels
    static constexpr int NB = C / 16;               // 16-channel blocks
    static constexpr int WN = NB < 8 ? NB : 8;      // waves across channels (pixel GEMMs)
    static constexpr int WM = 8 / WN;               // waves across pixels
    static constexpr int TM = GBM / (16 * WM);      // 16-pixel blocks per wave
    static constexpr int WJ = 8 / NB;               // waves sharing one dgamma column block
    static constexpr int TI = NB / WJ;              // dgamma row blocks per wave
    static constexpr int CPT = GBM * (2 * C / 16) / FNT;   // 16-byte chunks per thread per tile
    static constexpr int TILE = GBM * RS;
    static_assert(WM * WN == 8 && TM >= 1 && CPT >= 1 && WJ * NB == 8, "unsupported C");
};

template <int C>
__device__ __forceinline__ void ftile_load(u32x4 (&r)[FusedGeo<C>::CPT], const bf16* src, int ld, int64_t p0,
                                           int64_t npix) {
    using G = FusedGeo<C>;
    constexpr int CHR = 2 * C / 16;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * FNT + threadIdx.x;
        const int row = id / CHR, ch = id - (id / CHR) * CHR;
        const int64_t p = min(p0 + row, npix - 1);   // clamped: every load is issued (rows >= npix unused)
        r[i] = *reinterpret_cast<const u32x4*>(src + p * ld + ch * 8);
    }
}
template <int C>
__device__ __forceinline__ void ftile_to_lds(const u32x4 (&r)[FusedGeo<C>::CPT], char* lds, int64_t p0, int64_t npix) {
    using G = FusedGeo<C>;
    constexpr int CHR = 2 * C / 16;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * FNT + threadIdx.x;
        const int row = id / CHR, ch = id - (id / CHR) * CHR;
        // rows past the end are zero: they contribute nothing to dgamma / dbeta
        *reinterpret_cast<u32x4*>(lds + row * G::RS + ch * 16) = (p0 + row < npix) ? r[i] : u32x4{0u, 0u, 0u, 0u};
    }
}

// x tile and its elementwise square (bf16-rounded, as the MFMA operand): squared once per tile here
// instead of by each of the 8 waves that read it as a GEMM operand
template <int C>
__device__ __forceinline__ void ftile_to_lds_sq(const u32x4 (&r)[FusedGeo<C>::CPT], char* lds, char* lds_sq,
                                                int64_t p0, int64_t npix) {
    using G = FusedGeo<C>;
    constexpr int CHR = 2 * C / 16;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * FNT + threadIdx.x;
        const int row = id / CHR, ch = id - (id / CHR) * CHR;
        const u32x4 v = (p0 + row < npix) ? r[i] : u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(lds + row * G::RS + ch * 16) = v;
        *reinterpret_cast<u32x4*>(lds_sq + row * G::RS + ch * 16) = sq_chunk<bf16>(v);
    }
}

template <int C>
__device__ __forceinline__ void lds_to_global_rows(const char* lds, bf16* dst, int ld, int64_t p0, int64_t npix) {
    using G = FusedGeo<C>;
    constexpr int CHR = 2 * C / 16;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * FNT + threadIdx.x;
        const int row = id / CHR, ch = id - (id / CHR) * CHR;
        if (p0 + row < npix)
            *reinterpret_cast<u32x4*>(dst + (p0 + row) * ld + ch * 8) =
                *reinterpret_cast<const u32x4*>(lds + row * G::RS + ch * 16);
    }
}

template <int C>
__device__ __forceinline__ void lds_to_global_rows_all(const char* lds, bf16* dst, int ld, int64_t p0, int64_t npix) {
    using G = FusedGeo<C>;
    constexpr int CHR = 2 * C / 16;
#pragma unroll
    for (int i = 0; i < G::CPT; ++i) {
        const int id = i * FNT + threadIdx.x;
        const int row = id / CHR, ch = id - (id / CHR) * CHR;
        u32x4* d = (p0 + row < npix) ? reinterpret_cast<u32x4*>(dst + (p0 + row) * ld + ch * 8) : cai_gdn_sink;
        *d = *reinterpret_cast<const u32x4*>(lds + row * G::RS + ch * 16);
    }
}

template <int C, bool INV>
__global__ __launch_bounds__(FNT, 1) void gdn_bwd_fused_kernel(const bf16* __restrict__ x, int x_ld,
                                                               const bf16* __restrict__ dy, int dy_ld, int64_t npix,
                                                               const bf16* __restrict__ gamma_op,
                                                               const float* __restrict__ beta, int inverse,
                                                               bf16* __restrict__ dx, int dx_ld,
                                                               float* __restrict__ part) {
    using G = FusedGeo<C>;
    __shared__ __attribute__((aligned(16))) char lds[4 * G::TILE + C * 4];
    char* Lx = lds;
    char* Lg = lds + G::TILE;
    char* Lu = lds + 2 * G::TILE;
    char* Lq = lds + 3 * G::TILE;   // x^2
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wn = wave % G::WN, wm = wave / G::WN;
    const int n0 = wn * 16, r0 = wm * (GBM / G::WM);
    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    // dgamma tiling: column block jb, row blocks [ib0, ib0 + TI)
    const int jb = wave % G::NB, ib0 = (wave / G::NB) * G::TI;
    const bf16* gammaT = gamma_op + (int64_t)C * C;

    // gamma / gamma^T B fragments of this wave's 16 channels
    u32x4 fb[G::KB], fbT[G::KB];
#pragma unroll
    for (int kb = 0; kb < G::KB; ++kb) {
        const int n = n0 + i16;
        fb[kb] = *reinterpret_cast<const u32x4*>(gamma_op + (int64_t)n * C + kb * 32 + 8 * g_);
        fbT[kb] = *reinterpret_cast<const u32x4*>(gammaT + (int64_t)n * C + kb * 32 + 8 * g_);
    }
    // transposed GEMM layout (as the forward): a lane owns channels n0 + 4 g_ + r (r < 4) of one pixel.
    // beta sits in LDS (one 16-byte read per tile) rather than in 4 more live registers
    float dbeta[4] = {0.f, 0.f, 0.f, 0.f};
    float* const Lb = reinterpret_cast<float*>(lds + 4 * G::TILE);
    for (int c = threadIdx.x; c < C; c += FNT) Lb[c] = beta[c];
    f32x4 dg[G::TI];
#pragma unroll
    for (int t = 0; t < G::TI; ++t) dg[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // two tiles in flight: register set A holds tile t + 2*stride while set B waits with t + stride.  The
    // loop body is the A step then the B step in straight-line code, every prefetch is issued (past the
    // end it re-reads the last tile, an L2 hit) and every store too (lds_to_global_rows_all): no path with
    // fewer memory operations, so each step waits only for its own set, not vmcnt(0).
    const int64_t ntiles = (npix + GBM - 1) / GBM;
    const int64_t stride = gridDim.x;
    const int64_t last = ntiles - 1;
    u32x4 rxa[G::CPT], rga[G::CPT], rxb[G::CPT], rgb[G::CPT];
    int64_t tile = blockIdx.x;
    // the prologue issues what a loop iteration leaves in flight: set A, CPT stores, set B, CPT stores
    // (to the sink), so the loop's first wait is the same counted wait as the steady state's
    ftile_load<C>(rxa, x, x_ld, min(tile, last) * GBM, npix);
    ftile_load<C>(rga, dy, dy_ld, min(tile, last) * GBM, npix);
    sink_stores<G::CPT>(0);
    ftile_load<C>(rxb, x, x_ld, min(tile + stride, last) * GBM, npix);
    ftile_load<C>(rgb, dy, dy_ld, min(tile + stride, last) * GBM, npix);
    sink_stores<G::CPT>(8);
    auto step = [&](u32x4 (&rx)[G::CPT], u32x4 (&rg)[G::CPT], int64_t cur, int64_t nxt) {
        const int64_t p0 = cur * GBM;
        lds_barrier();                       // previous tile's dx store has read Lg
        ftile_to_lds_sq<C>(rx, Lx, Lq, p0, npix);
        ftile_to_lds<C>(rg, Lg, p0, npix);
        ftile_load<C>(rx, x, x_ld, nxt * GBM, npix);
        ftile_load<C>(rg, dy, dy_ld, nxt * GBM, npix);
        lds_barrier();
        const int nvalid = (int)min((int64_t)GBM, npix - p0);
        // ---- norm^T = gamma (x^2)^T (+ beta): gamma's fragments as A, the x^2 tile as B ----
        f32x4 acc[G::TM];
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) acc[tm] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < G::KB; ++kb)
#pragma unroll
            for (int tm = 0; tm < G::TM; ++tm) {
                const int row = r0 + tm * 16 + i16;
                const u32x4 b = *reinterpret_cast<const u32x4*>(Lq + row * G::RS + kb * 64 + 16 * g_);
                acc[tm] = mma16<bf16>(fb[kb], b, acc[tm]);
            }
        // ---- u, t1: lane = pixel r0 + 16 tm + i16, channels n0 + 4 g_ + r: one 8-byte LDS access per
        // 4 elements (x, g in; u out), conflict-free across the wave ----
        bf16x4 t1q[G::TM];   // t1 rounded to bf16 (as the dx tile it feeds): half the registers
        const f32x4 bq = *reinterpret_cast<const f32x4*>(Lb + n0 + 4 * g_);
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) {
            const int row = r0 + tm * 16 + i16;
            const bf16x4 xq = *reinterpret_cast<const bf16x4*>(Lx + row * G::RS + (n0 + 4 * g_) * 2);
            const bf16x4 gq = *reinterpret_cast<const bf16x4*>(Lg + row * G::RS + (n0 + 4 * g_) * 2);
            bf16x4 uq;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float xv = (float)xq[r];
                const float gv = (float)gq[r];
                const float nv = acc[tm][r] + bq[r];
                // one v_rsq per element for both forms (no IEEE divide / sqrt sequences)
                const float rs = rsqrtf(nv);
                float uv, t1;
                if constexpr (INV) {
                    t1 = gv * nv * rs;                 // g sqrt(norm)
                    uv = 0.5f * gv * xv * rs;          // g x / (2 sqrt(norm))
                } else {
                    t1 = gv * rs;
                    uv = -0.5f * gv * xv * rs * rs * rs;
                }
                if (row >= nvalid) uv = 0.f;
                dbeta[r] += uv;
                t1q[tm][r] = (bf16)t1;   // t1 stays in registers for the dx phase
                uq[r] = (bf16)uv;
            }
            *reinterpret_cast<bf16x4*>(Lu + row * G::RS + (n0 + 4 * g_) * 2) = uq;
        }
        lds_barrier();
        // ---- dgamma += u^T x^2 (K = the tile's 64 pixels; column reads by hardware transpose) ----
#pragma unroll
        for (int ks = 0; ks < GBM / 32; ++ks) {
            const int rr = 32 * ks + 8 * g_ + q_;
            const int colB = jb * 16 + 4 * p4;
            const s16x4 b0 = ds_tr16(Lq, rr * G::RS + colB * 2);
            const s16x4 b1 = ds_tr16(Lq, (rr + 4) * G::RS + colB * 2);
            const s16x8 bvv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
            const u32x4 fbx = __builtin_bit_cast(u32x4, bvv);
#pragma unroll
            for (int t = 0; t < G::TI; ++t) {
                const int colA = (ib0 + t) * 16 + 4 * p4;
                const s16x4 a0 = ds_tr16(Lu, rr * G::RS + colA * 2);
                const s16x4 a1 = ds_tr16(Lu, (rr + 4) * G::RS + colA * 2);
                const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                dg[t] = mma16<bf16>(__builtin_bit_cast(u32x4, av), fbx, dg[t]);
            }
        }
        // ---- dx^T = gamma^T u^T: gamma^T's fragments as A, the u tile as B ----
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) acc[tm] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < G::KB; ++kb)
#pragma unroll
            for (int tm = 0; tm < G::TM; ++tm) {
                const int row = r0 + tm * 16 + i16;
                const u32x4 b = *reinterpret_cast<const u32x4*>(Lu + row * G::RS + kb * 64 + 16 * g_);
                acc[tm] = mma16<bf16>(fbT[kb], b, acc[tm]);
            }
        // dx = t1 + 2 x (u gamma): t1 still in registers, x re-read from its tile (8 bytes: cheaper than
        // keeping it live through the dgamma phase), the same 4 channels of the same pixel
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) {
            const int row = r0 + tm * 16 + i16;
            const bf16x4 xqq = *reinterpret_cast<const bf16x4*>(Lx + row * G::RS + (n0 + 4 * g_) * 2);
            bf16x4 dq;
#pragma unroll
            for (int r = 0; r < 4; ++r) dq[r] = (bf16)((float)t1q[tm][r] + 2.f * (float)xqq[r] * acc[tm][r]);
            *reinterpret_cast<bf16x4*>(Lg + row * G::RS + (n0 + 4 * g_) * 2) = dq;
        }
        lds_barrier();
        lds_to_global_rows_all<C>(Lg, dx, dx_ld, p0, npix);
    };
    // a counted loop over tile pairs (one path through the body), then the odd tile
    const int64_t mine = tile < ntiles ? (ntiles - tile + stride - 1) / stride : 0;
    for (int64_t it = 0; it < mine / 2; ++it, tile += 2 * stride) {
        step(rxa, rga, tile, min(tile + 2 * stride, last));
        step(rxb, rgb, tile + stride, min(tile + 3 * stride, last));
    }
    if (mine & 1) step(rxa, rga, tile, last);
    // ---- partials: dbeta (lanes of one channel quad: the 16 pixels i16, xor 1..8; waves of one column
    // block via LDS) ----
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) dbeta[r] += __shfl_xor(dbeta[r], o, 64);
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
    if (i16 == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wm * C + n0 + 4 * g_ + r] = dbeta[r];
    }
    __syncthreads();
    float* pb = part + (int64_t)blockIdx.x * (C * C + C);
    for (int c = threadIdx.x; c < C; c += FNT) {
        float v = 0.f;
        for (int m = 0; m < G::WM; ++m) v += red[m * C + c];
        pb[C * C + c] = v;
    }
#pragma unroll
    for (int t = 0; t < G::TI; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = (ib0 + t) * 16 + g_ * 4 + r, j = jb * 16 + i16;
            pb[(int64_t)i * C + j] = dg[t][r];
        }
}

// ---------------------------------------------------------------------------
// Fused backward for wide layers (bf16, C = 160 / 192: the q6-8 hyperpriors, mbt2018, cheng2020 at N=192).
// The C <= 128 kernel above holds gamma AND gamma^T fragments plus its dgamma tile in registers; at
// C = 192 that no longer fits (the dgamma partial alone is 144 16x16 tiles).  Here one wave owns 16
// channels (C / 16 waves: 12 at C = 192), gamma^T lives in LDS (C x C bf16, row reads for the dx GEMM),
// gamma fragments of the wave's 16 rows stay in registers (norm GEMM), tiles are 32 pixels, and
// each wave accumulates one 16-column block of dgamma (C / 16 tiles).  Per tile:
//   norm = x^2 gamma^T + beta (MFMA)  ->  u, t1 (fp32)  ->  dgamma += u^T x^2 (MFMA, pixels as K,
//   ds_read_b64_tr_b16)  ->  dx = t1 + 2 x (u gamma) (MFMA, gamma^T rows from LDS)
// HBM traffic per pixel: read x, dy, write dx (6C B) -- the two-pass path moves 12C B.
// ---------------------------------------------------------------------------
template <int C>
struct WideGeo {
    static constexpr int NW = C / 16;                 // waves = 16-channel blocks
    static constexpr int NT = NW * 64;
    static constexpr int GB = 32;                     // pixels per tile
    static constexpr int RS = 2 * C + 16;             // LDS row stride (bytes): 16 rows x 16 B conflict-free
    static constexpr int KB = C / 32;                 // 32-deep K blocks over channels
    static constexpr int TM = GB / 16;
    static constexpr int CPT = GB * (2 * C / 16) / NT;   // 16-byte chunks per thread per tile (= 1)
    static constexpr int TILE = GB * RS;
    static constexpr int GT = C * RS;                 // gamma^T image
    static constexpr int BYTES = GT + 4 * TILE;
    static_assert(C % 32 == 0 && NW <= 16 && CPT >= 1 && GB * (2 * C / 16) % NT == 0, "unsupported C");
};

template <int C, bool INV>
__global__ __launch_bounds__(WideGeo<C>::NT, 1) void gdn_bwd_wide_kernel(const bf16* __restrict__ x, int x_ld,
                                                                        const bf16* __restrict__ dy, int dy_ld,
                                                                        int64_t npix, const bf16* __restrict__ gamma_op,
                                                                        const float* __restrict__ beta,
                                                                        bf16* __restrict__ dx, int dx_ld,
                                                                        float* __restrict__ part) {
    using G = WideGeo<C>;
    __shared__ __attribute__((aligned(16))) char lds[G::BYTES];
    char* Lt = lds;                       // gamma^T [C][C]
    char* Lx = lds + G::GT;
    char* Lg = Lx + G::TILE;
    char* Lu = Lg + G::TILE;
    char* Lq = Lu + G::TILE;              // x^2
    constexpr int CHR = 2 * C / 16;       // 16-byte chunks per pixel row
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = wave * 16;
    const int g_ = lane >> 4, i16 = lane & 15, q_ = i16 >> 2, p4 = i16 & 3;
    const bf16* gammaT = gamma_op + (int64_t)C * C;

    // gamma^T into LDS (row j = column j of gamma), gamma fragments of this wave's rows into registers
    for (int id = threadIdx.x; id < C * CHR; id += G::NT) {
        const int r = id / CHR, ch = id - r * CHR;
        *reinterpret_cast<u32x4*>(Lt + r * G::RS + ch * 16) =
            *reinterpret_cast<const u32x4*>(gammaT + (int64_t)r * C + ch * 8);
    }
    u32x4 fb[G::KB];
#pragma unroll
    for (int kb = 0; kb < G::KB; ++kb)
        fb[kb] = *reinterpret_cast<const u32x4*>(gamma_op + (int64_t)(n0 + i16) * C + kb * 32 + 8 * g_);
    const float bv = beta[n0 + i16];
    f32x4 dg[G::NW];
#pragma unroll
    for (int t = 0; t < G::NW; ++t) dg[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dbeta = 0.f;

    // one tile in flight: the next tile's x / dy chunk (one 16-byte chunk per thread each) loads while
    // this tile is computed
    const int64_t ntiles = (npix + G::GB - 1) / G::GB;
    const int crow = threadIdx.x / CHR, cch = threadIdx.x - (threadIdx.x / CHR) * CHR;
    auto load = [&](int64_t t, u32x4& rx, u32x4& rg) {
        const int64_t p = min(t * G::GB + crow, npix - 1);   // clamped: every load is issued
        rx = *reinterpret_cast<const u32x4*>(x + p * x_ld + cch * 8);
        rg = *reinterpret_cast<const u32x4*>(dy + p * dy_ld + cch * 8);
    };
    u32x4 rx, rg;
    int64_t tile = blockIdx.x;
    if (tile < ntiles) load(tile, rx, rg);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = tile * G::GB;
        const int nvalid = (int)min((int64_t)G::GB, npix - p0);
        lds_barrier();                    // the previous tile's dx store has read Lg
        {
            const bool ok = crow < nvalid;   // rows past the end are zero: nothing reaches dgamma / dbeta
            const u32x4 vx = ok ? rx : u32x4{0u, 0u, 0u, 0u};
            const u32x4 vg = ok ? rg : u32x4{0u, 0u, 0u, 0u};
            *reinterpret_cast<u32x4*>(Lx + crow * G::RS + cch * 16) = vx;
            *reinterpret_cast<u32x4*>(Lq + crow * G::RS + cch * 16) = sq_chunk<bf16>(vx);
            *reinterpret_cast<u32x4*>(Lg + crow * G::RS + cch * 16) = vg;
        }
        if (tile + gridDim.x < ntiles) load(tile + gridDim.x, rx, rg);
        lds_barrier();
        // ---- norm = x^2 gamma^T (+ beta): rows = pixels, columns = this wave's 16 channels ----
        f32x4 acc[G::TM];
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) acc[tm] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < G::KB; ++kb)
#pragma unroll
            for (int tm = 0; tm < G::TM; ++tm) {
                const u32x4 a = *reinterpret_cast<const u32x4*>(Lq + (tm * 16 + i16) * G::RS + kb * 64 + 16 * g_);
                acc[tm] = mma16<bf16>(a, fb[kb], acc[tm]);
            }
        // ---- u, t1 (element rows tm*16 + 4 g_ + r, column n0 + i16) ----
        float xr[G::TM][4], tr[G::TM][4];
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = tm * 16 + g_ * 4 + r;
                xr[tm][r] = (float)*lds_elem<bf16>(Lx, G::RS, row, n0 + i16);
                tr[tm][r] = (float)*lds_elem<bf16>(Lg, G::RS, row, n0 + i16);
            }
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = tm * 16 + g_ * 4 + r;
                const float xv = xr[tm][r], gv = tr[tm][r];
                const float nv = acc[tm][r] + bv;
                const float rs = rsqrtf(nv);
                float uv, t1;
                if constexpr (INV) {
                    t1 = gv * nv * rs;
                    uv = 0.5f * gv * xv * rs;
                } else {
                    t1 = gv * rs;
                    uv = -0.5f * gv * xv * rs * rs * rs;
                }
                if (row >= nvalid) uv = 0.f;
                dbeta += uv;
                tr[tm][r] = (float)(bf16)t1;
                *lds_elem<bf16>(Lu, G::RS, row, n0 + i16) = (bf16)uv;
            }
        lds_barrier();
        // ---- dgamma[:, n0 .. n0+15] += u^T x^2 (K = the tile's 32 pixels) ----
        {
            const int rr = 8 * g_ + q_;
            const int colB = n0 + 4 * p4;
            const s16x4 b0 = ds_tr16(Lq, rr * G::RS + colB * 2);
            const s16x4 b1 = ds_tr16(Lq, (rr + 4) * G::RS + colB * 2);
            const s16x8 bvv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
            const u32x4 fbx = __builtin_bit_cast(u32x4, bvv);
#pragma unroll
            for (int t = 0; t < G::NW; ++t) {
                const int colA = t * 16 + 4 * p4;
                const s16x4 a0 = ds_tr16(Lu, rr * G::RS + colA * 2);
                const s16x4 a1 = ds_tr16(Lu, (rr + 4) * G::RS + colA * 2);
                const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
                dg[t] = mma16<bf16>(__builtin_bit_cast(u32x4, av), fbx, dg[t]);
            }
        }
        // ---- dx = t1 + 2 x (u gamma): B = gamma^T rows of this wave's channels ----
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm) acc[tm] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < G::KB; ++kb) {
            const u32x4 bt = *reinterpret_cast<const u32x4*>(Lt + (n0 + i16) * G::RS + kb * 64 + 16 * g_);
#pragma unroll
            for (int tm = 0; tm < G::TM; ++tm) {
                const u32x4 a = *reinterpret_cast<const u32x4*>(Lu + (tm * 16 + i16) * G::RS + kb * 64 + 16 * g_);
                acc[tm] = mma16<bf16>(a, bt, acc[tm]);
            }
        }
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = tm * 16 + g_ * 4 + r;
                *lds_elem<bf16>(Lg, G::RS, row, n0 + i16) = (bf16)(tr[tm][r] + 2.f * xr[tm][r] * acc[tm][r]);
            }
        lds_barrier();
        if (crow < nvalid)
            *reinterpret_cast<u32x4*>(dx + (p0 + crow) * dx_ld + cch * 8) =
                *reinterpret_cast<const u32x4*>(Lg + crow * G::RS + cch * 16);
    }
    // ---- partials: dbeta of this wave's channels (lanes of one column: xor 16, 32), dgamma column block ----
    dbeta += __shfl_xor(dbeta, 16, 64);
    dbeta += __shfl_xor(dbeta, 32, 64);
    float* pb = part + (int64_t)blockIdx.x * (C * C + C);
    if (lane < 16) pb[C * C + n0 + lane] = dbeta;
#pragma unroll
    for (int t = 0; t < G::NW; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = t * 16 + g_ * 4 + r, j = n0 + i16;
            pb[(int64_t)i * C + j] = dg[t][r];
        }
}

// Blocks of the fused / lane backward.  Each block writes one (C*C + C) fp32 partial (66 KB at C = 128) that the
// reduce job reads back: at 64 pixels per block a 32 x 32 x 16 layer's 256 partials (16.9 MB) outweigh its x / dy /
// dx (12.6 MB).  CAI_GDN_BWD_MIN_PX (A/B knob, 0 = off) caps the blocks at ceil(npix / MIN_PX).
static int64_t gdn_bwd_min_px() {
    static const int64_t v = [] {
        const char* e = getenv("CAI_GDN_BWD_MIN_PX");
        return (int64_t)((e && *e) ? std::max(0, atoi(e)) : 0);
    }();
    return v;
}
static int gdn_bwd_cap(int64_t npix, int64_t blocks) {
    const int64_t m = gdn_bwd_min_px();
    if (m > 0) blocks = std::min<int64_t>(blocks, (npix + m - 1) / m);
    return (int)std::max<int64_t>(1, blocks);
}
static int fused_blocks(int64_t npix) {
    const int64_t tiles = (npix + GBM - 1) / GBM;
    return gdn_bwd_cap(npix, std::min<int64_t>(256, tiles));
}

__global__ void gdn_reparam_kernel(const float* __restrict__ beta_raw, const float* __restrict__ gamma_raw, int C,
                                   float bbound, float gbound, float ped, int dtype, float* __restrict__ beta,
                                   void* __restrict__ gop) {
    const int64_t CC = (int64_t)C * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < CC; i += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / C), c = (int)(i - (int64_t)r * C);
        const float lb = fmaxf(gamma_raw[i], gbound);
        const float v = lb * lb - ped;
        st_any(gop, dtype, i, v);                        // gamma[i][j]
        st_any(gop, dtype, CC + (int64_t)c * C + r, v);  // gamma^T
        if (i < C) {
            const float lbb = fmaxf(beta_raw[i], bbound);
            beta[i] = lbb * lbb - ped;
        }
    }
}

// NonNegativeParametrizer / LowerBound backward: d raw = (raw >= bound || d < 0) ? d : 0, d = 2 lb dparam
__global__ void gdn_reparam_bwd_kernel(const float* __restrict__ beta_raw, const float* __restrict__ gamma_raw,
                                       const float* __restrict__ dbeta, const float* __restrict__ dgamma, int C,
                                       float bbound, float gbound, float* __restrict__ dbeta_raw,
                                       float* __restrict__ dgamma_raw, int accumulate) {
    const int64_t CC = (int64_t)C * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < CC; i += (int64_t)gridDim.x * blockDim.x) {
        const float gr = gamma_raw[i];
        const float d = 2.f * fmaxf(gr, gbound) * dgamma[i];
        const float vg = (gr >= gbound || d < 0.f) ? d : 0.f;
        dgamma_raw[i] = accumulate ? dgamma_raw[i] + vg : vg;
        if (i < C) {
            const float br = beta_raw[i];
            const float db = 2.f * fmaxf(br, bbound) * dbeta[i];
            const float vb = (br >= bbound || db < 0.f) ? db : 0.f;
            dbeta_raw[i] = accumulate ? dbeta_raw[i] + vb : vb;
        }
    }
}

template <typename T, int C>
static void launch_gdn_fwd(const void* x, int x_ld, int64_t npix, const void* g, const float* b, int inv, void* y,
                           int y_ld, hipStream_t st) {
    const int64_t ntiles = (npix + GBM - 1) / GBM;
    // persistent: one wave of resident blocks (2 per CU where the launch bounds allow it)
    const int occ = (sizeof(T) == 2 && C <= 192) ? 2 : 1;
    const int grid = (int)std::min<int64_t>(ntiles, 256 * occ);
    hipLaunchKernelGGL((gdn_fwd_kernel<T, C>), dim3(grid), dim3(GNT), 0, st, reinterpret_cast<const T*>(x), x_ld, npix,
                       reinterpret_cast<const T*>(g), b, inv, reinterpret_cast<T*>(y), y_ld);
}
template <typename T, int C>
static void launch_gdn_bwd(const void* x, int x_ld, const void* dy, int dy_ld, int64_t npix, const void* g,
                           const float* b, int inv, void* dx, int dx_ld, void* u, hipStream_t st) {
    const int64_t ntiles = (npix + GBM - 1) / GBM;
    hipLaunchKernelGGL((gdn_bwd_kernel<T, C>), dim3((unsigned)ntiles), dim3(GNT), 0, st,
                       reinterpret_cast<const T*>(x), x_ld, reinterpret_cast<const T*>(dy), dy_ld, npix,
                       reinterpret_cast<const T*>(g), b, inv, reinterpret_cast<T*>(dx), dx_ld, reinterpret_cast<T*>(u));
}

// every channel count that is a multiple of 32 up to 256 (bf16) / 192 (fp32: three fp32 tiles of the
// two-pass backward fill the LDS at 192); other counts are zero-padded by the caller (layers/gdn.py)
#define GDN_CASE(FN, T, CC, ...) \
    case CC: FN<T, CC>(__VA_ARGS__); break;
#define GDN_DISPATCH(FN, ...)                                                  \
    do {                                                                       \
        if (dtype == CAI_BF16) {                                               \
            switch (C) {                                                       \
                GDN_CASE(FN, bf16, 32, __VA_ARGS__)                            \
                GDN_CASE(FN, bf16, 64, __VA_ARGS__)                            \
                GDN_CASE(FN, bf16, 96, __VA_ARGS__)                            \
                GDN_CASE(FN, bf16, 128, __VA_ARGS__)                           \
                GDN_CASE(FN, bf16, 160, __VA_ARGS__)                           \
                GDN_CASE(FN, bf16, 192, __VA_ARGS__)                           \
                GDN_CASE(FN, bf16, 224, __VA_ARGS__)                           \
                GDN_CASE(FN, bf16, 256, __VA_ARGS__)                           \
            }                                                                  \
        } else {                                                               \
            switch (C) {                                                       \
                GDN_CASE(FN, float, 32, __VA_ARGS__)                           \
                GDN_CASE(FN, float, 64, __VA_ARGS__)                           \
                GDN_CASE(FN, float, 96, __VA_ARGS__)                           \
                GDN_CASE(FN, float, 128, __VA_ARGS__)                          \
                GDN_CASE(FN, float, 160, __VA_ARGS__)                          \
                GDN_CASE(FN, float, 192, __VA_ARGS__)                          \
            }                                                                  \
        }                                                                      \
    } while (0)

static bool gdn_c_ok(int C, int dtype) { return C % 32 == 0 && C >= 32 && C <= (dtype == CAI_BF16 ? 256 : 192); }

}  // namespace cai

using namespace cai;

extern "C" {

int cai_gdn_reparam(const float* beta_raw, const float* gamma_raw, int32_t C, float beta_min, float reparam_offset,
                    int dtype, float* beta, void* gamma_op, void* stream) {
    CAI_CHECK_ARG(beta_raw && gamma_raw && beta && gamma_op && C > 0, "gdn_reparam: bad arguments");
    const float ped = reparam_offset * reparam_offset;
    const float bbound = sqrtf(beta_min + ped), gbound = sqrtf(0.f + ped);
    const int64_t CC = (int64_t)C * C;
    hipLaunchKernelGGL(gdn_reparam_kernel, dim3((unsigned)std::min<int64_t>(1024, (CC + 255) / 256)), dim3(256), 0,
                       as_stream(stream), beta_raw, gamma_raw, C, bbound, gbound, ped, dtype, beta, gamma_op);
    CAI_LAUNCH_CHECK("gdn_reparam");
    return CAI_OK;
}

int cai_gdn_fwd(int dtype, const void* x, int32_t x_ld, int64_t npix, int32_t C, const void* gamma_op,
                const float* beta, int32_t inverse, void* y, int32_t y_ld, void* stream) {
    CAI_CHECK_ARG(gdn_c_ok(C, dtype), "gdn_fwd: unsupported channel count %d", C);
    CAI_CHECK_ARG(x && gamma_op && beta && y && x_ld >= C && y_ld >= C, "gdn_fwd: bad arguments");
    CAI_CHECK_ARG(x_ld % 8 == 0 && y_ld % 8 == 0, "gdn_fwd: ld must be a multiple of 8");
    if (npix == 0) return CAI_OK;
    if (dtype == CAI_BF16 && gdn_lane_on() && gdn_lane_fwd_ok(C, npix, x_ld, y_ld)) {
        launch_gdn_fwd_lane(x, x_ld, npix, C, gamma_op, beta, inverse, y, y_ld, as_stream(stream));
        CAI_LAUNCH_CHECK("gdn_fwd");
        return CAI_OK;
    }
    GDN_DISPATCH(launch_gdn_fwd, x, x_ld, npix, gamma_op, beta, inverse, y, y_ld, as_stream(stream));
    CAI_LAUNCH_CHECK("gdn_fwd");
    return CAI_OK;
}

int cai_gdn_bwd(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t npix, int32_t C,
                const void* gamma_op, const float* beta, int32_t inverse, void* dx, int32_t dx_ld, void* u,
                void* stream) {
    CAI_CHECK_ARG(gdn_c_ok(C, dtype), "gdn_bwd: unsupported channel count %d", C);
    CAI_CHECK_ARG(x && dy && gamma_op && beta && dx && u, "gdn_bwd: bad arguments");
    CAI_CHECK_ARG(x_ld % 8 == 0 && dy_ld % 8 == 0 && dx_ld % 8 == 0 && x_ld >= C && dy_ld >= C && dx_ld >= C,
                  "gdn_bwd: bad leading dimensions");
    if (npix == 0) return CAI_OK;
    GDN_DISPATCH(launch_gdn_bwd, x, x_ld, dy, dy_ld, npix, gamma_op, beta, inverse, dx, dx_ld, u, as_stream(stream));
    CAI_LAUNCH_CHECK("gdn_bwd");
    return CAI_OK;
}

static cai_conv_geom gdn_geom(int64_t npix, int C) {
    cai_conv_geom g{};
    g.batch = 1; g.in_c = C; g.out_c = C; g.in_h = (int)npix; g.in_w = 1; g.out_h = (int)npix; g.out_w = 1;
    g.kernel = 1; g.stride = 1; g.pad = 0; g.output_padding = 0; g.transposed = 0;
    return g;
}

size_t cai_gdn_param_grad_workspace_bytes(int64_t npix, int32_t C, int dtype) {
    const cai_conv_geom g = gdn_geom(npix, C);
    return cai_conv_wgrad_workspace_bytes(&g, dtype) + (size_t)C * C * 4 + (size_t)C * 4 + colsum_ws_bytes(npix, C) +
           512;
}

int cai_gdn_param_grad(int dtype, const void* x, int32_t x_ld, const void* u, int64_t npix, int32_t C,
                       const float* beta_raw, const float* gamma_raw, float beta_min, float reparam_offset,
                       float* dbeta_raw, float* dgamma_raw, int32_t accumulate, void* workspace, size_t ws_bytes,
                       void* stream) {
    CAI_CHECK_ARG(npix > 0 && npix < (1ll << 31), "gdn_param_grad: bad pixel count");
    CAI_CHECK_ARG(ws_bytes >= cai_gdn_param_grad_workspace_bytes(npix, C, dtype), "gdn_param_grad: workspace too small");
    const cai_conv_geom g = gdn_geom(npix, C);
    const size_t wgb = cai_conv_wgrad_workspace_bytes(&g, dtype);
    char* ws = reinterpret_cast<char*>(workspace);
    float* dgamma = reinterpret_cast<float*>(ws + wgb);
    float* dbeta = dgamma + (size_t)C * C;
    char* cws = reinterpret_cast<char*>(dbeta + C);
    // dgamma[i][j] = sum_p u[p][i] * x[p][j]^2   (G = u, X = x squared on load)
    // dbeta[i]     = sum_p u[p][i]                (the same call's bias gradient)
    (void)cws;
    int rc = cai_conv_wgrad(&g, dtype, x, x_ld, 0, 1, u, C, dgamma, dbeta, 0, ws, wgb, stream);
    if (rc) return rc;
    const float ped = reparam_offset * reparam_offset;
    const float bbound = sqrtf(beta_min + ped), gbound = sqrtf(ped);
    const int64_t CC = (int64_t)C * C;
    hipLaunchKernelGGL(gdn_reparam_bwd_kernel, dim3((unsigned)std::min<int64_t>(1024, (CC + 255) / 256)), dim3(256), 0,
                       as_stream(stream), beta_raw, gamma_raw, dbeta, dgamma, C, bbound, gbound, dbeta_raw, dgamma_raw,
                       accumulate);
    CAI_LAUNCH_CHECK("gdn_param_grad");
    return CAI_OK;
}


static bool fused_ok(int dtype, int C) { return dtype == CAI_BF16 && (C == 64 || C == 128 || C == 160 || C == 192); }

size_t cai_gdn_backward_workspace_bytes(int64_t npix, int32_t C, int dtype) {
    if (npix <= 0 || !gdn_c_ok(C, dtype)) return 0;
    if (fused_ok(dtype, C)) return (size_t)fused_blocks(npix) * ((size_t)C * C + C) * sizeof(float);
    const size_t ub = ((size_t)npix * C * dtype_size(dtype) + 255) / 256 * 256;
    return ub + cai_gdn_param_grad_workspace_bytes(npix, C, dtype);
}

static int run_gdn_backward(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t npix,
                            int32_t C, const void* gamma_op, const float* beta, int32_t inverse, void* dx,
                            int32_t dx_ld, const float* beta_raw, const float* gamma_raw, float beta_min,
                            float reparam_offset, float* dbeta_raw, float* dgamma_raw, int32_t accumulate,
                            void* workspace, size_t ws_bytes, void* stream, cai_reduce_job* job) {
    if (job) *job = cai_reduce_job{};
    CAI_CHECK_ARG(gdn_c_ok(C, dtype), "gdn_backward: unsupported channel count %d", C);
    CAI_CHECK_ARG(x && dy && gamma_op && beta && dx && beta_raw && gamma_raw && dbeta_raw && dgamma_raw,
                  "gdn_backward: null pointer");
    CAI_CHECK_ARG(x_ld % 8 == 0 && dy_ld % 8 == 0 && dx_ld % 8 == 0 && x_ld >= C && dy_ld >= C && dx_ld >= C,
                  "gdn_backward: bad leading dimensions");
    CAI_CHECK_ARG(npix > 0 && npix < (1ll << 31), "gdn_backward: bad pixel count");
    CAI_CHECK_ARG(workspace && ws_bytes >= cai_gdn_backward_workspace_bytes(npix, C, dtype) &&
                      ((uintptr_t)workspace & 255) == 0,
                  "gdn_backward: workspace of %zu bytes (256-byte aligned) required",
                  cai_gdn_backward_workspace_bytes(npix, C, dtype));
    hipStream_t st = as_stream(stream);
    if (!fused_ok(dtype, C)) {
        // two-kernel path: dx + u, then the split-K parameter gradient
        const size_t ub = ((size_t)npix * C * dtype_size(dtype) + 255) / 256 * 256;
        char* ws = reinterpret_cast<char*>(workspace);
        int rc = cai_gdn_bwd(dtype, x, x_ld, dy, dy_ld, npix, C, gamma_op, beta, inverse, dx, dx_ld, ws, stream);
        if (rc) return rc;
        return cai_gdn_param_grad(dtype, x, x_ld, ws, npix, C, beta_raw, gamma_raw, beta_min, reparam_offset,
                                  dbeta_raw, dgamma_raw, accumulate, ws + ub, ws_bytes - ub, stream);
    }
    const bool lane = gdn_lane_on() && gdn_lane_bwd_ok(C, npix, x_ld, dy_ld, dx_ld);
    // (the lane kernel's block count never exceeds fused_blocks: the workspace size holds for both)
    const int nblk = lane ? gdn_bwd_cap(npix, gdn_lane_bwd_blocks(npix)) : fused_blocks(npix);
    float* part = reinterpret_cast<float*>(workspace);
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(nblk), dim3(FNT), 0, st, reinterpret_cast<const bf16*>(x), x_ld,
                           reinterpret_cast<const bf16*>(dy), dy_ld, npix, reinterpret_cast<const bf16*>(gamma_op),
                           beta, inverse, reinterpret_cast<bf16*>(dx), dx_ld, part);
    };
    auto launch_wide = [&](auto kern, int nt) {
        hipLaunchKernelGGL(kern, dim3(nblk), dim3(nt), 0, st, reinterpret_cast<const bf16*>(x), x_ld,
                           reinterpret_cast<const bf16*>(dy), dy_ld, npix, reinterpret_cast<const bf16*>(gamma_op),
                           beta, reinterpret_cast<bf16*>(dx), dx_ld, part);
    };
    if (lane) {
        launch_gdn_bwd_lane(x, x_ld, dy, dy_ld, npix, C, gamma_op, beta, inverse, dx, dx_ld, part, nblk, st);
    } else
    if (C == 192)
        inverse ? launch_wide(gdn_bwd_wide_kernel<192, true>, WideGeo<192>::NT)
                : launch_wide(gdn_bwd_wide_kernel<192, false>, WideGeo<192>::NT);
    else if (C == 160)
        inverse ? launch_wide(gdn_bwd_wide_kernel<160, true>, WideGeo<160>::NT)
                : launch_wide(gdn_bwd_wide_kernel<160, false>, WideGeo<160>::NT);
    else if (C == 128)
        inverse ? launch(gdn_bwd_fused_kernel<128, true>) : launch(gdn_bwd_fused_kernel<128, false>);
    else
        inverse ? launch(gdn_bwd_fused_kernel<64, true>) : launch(gdn_bwd_fused_kernel<64, false>);
    CAI_LAUNCH_CHECK("gdn_backward");
    // the per-block partials -> dgamma_raw / dbeta_raw: a job (reduce_jobs.hip; C % 4 == 0 and the 256-byte
    // aligned workspace give every partial row 16-byte alignment), returned to a deferring caller or run now
    const float ped = reparam_offset * reparam_offset;
    const int64_t n = (int64_t)C * C + C;
    cai_reduce_job J{};
    J.kind = CAI_JOB_GDN;
    J.nblocks = (int)((n + 63) / 64);
    J.p[0] = part; J.p[1] = beta_raw; J.p[2] = gamma_raw; J.p[3] = dbeta_raw; J.p[4] = dgamma_raw;
    J.i[0] = nblk; J.i[1] = C; J.i[2] = accumulate;
    J.f[0] = sqrtf(beta_min + ped); J.f[1] = sqrtf(ped);
    if (job) {
        *job = J;
        return CAI_OK;
    }
    return launch_reduce_jobs(&J, 1, st);
}

int cai_gdn_backward(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t npix, int32_t C,
                     const void* gamma_op, const float* beta, int32_t inverse, void* dx, int32_t dx_ld,
                     const float* beta_raw, const float* gamma_raw, float beta_min, float reparam_offset,
                     float* dbeta_raw, float* dgamma_raw, int32_t accumulate, void* workspace, size_t ws_bytes,
                     void* stream) {
    return run_gdn_backward(dtype, x, x_ld, dy, dy_ld, npix, C, gamma_op, beta, inverse, dx, dx_ld, beta_raw,
                            gamma_raw, beta_min, reparam_offset, dbeta_raw, dgamma_raw, accumulate, workspace,
                            ws_bytes, stream, nullptr);
}

int cai_gdn_backward_deferred(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t npix,
                              int32_t C, const void* gamma_op, const float* beta, int32_t inverse, void* dx,
                              int32_t dx_ld, const float* beta_raw, const float* gamma_raw, float beta_min,
                              float reparam_offset, float* dbeta_raw, float* dgamma_raw, int32_t accumulate,
                              void* workspace, size_t ws_bytes, void* stream, cai_reduce_job* job) {
    CAI_CHECK_ARG(job, "gdn_backward_deferred: null job");
    return run_gdn_backward(dtype, x, x_ld, dy, dy_ld, npix, C, gamma_op, beta, inverse, dx, dx_ld, beta_raw,
                            gamma_raw, beta_min, reparam_offset, dbeta_raw, dgamma_raw, accumulate, workspace,
                            ws_bytes, stream, job);
}

// The kernel cai_gdn_fwd (direction 0) / cai_gdn_backward (direction 1) launches for these arguments, as
// rocprofv3 names it (the per-launch ledger and the model-level dispatch tests read it); "" for bad arguments.
const char* cai_gdn_kernel_name(int dtype, int64_t npix, int32_t C, int32_t in_ld, int32_t out_ld, int32_t direction) {
    static thread_local char buf[48];
    if (!gdn_c_ok(C, dtype) || npix <= 0 || (direction != 0 && direction != 1)) return "";
    const char* nm;
    if (direction == 0)
        nm = dtype == CAI_BF16 && gdn_lane_on() && gdn_lane_fwd_ok(C, npix, in_ld, out_ld) ? "gdn_fwd_lane_kernel"
                                                                                          : "gdn_fwd_kernel";
    else if (!fused_ok(dtype, C))
        nm = "gdn_bwd_kernel+param_grad";
    else if (gdn_lane_on() && gdn_lane_bwd_ok(C, npix, in_ld, in_ld, out_ld))
        nm = "gdn_bwd_lane_kernel";
    else
        nm = (C == 192 || C == 160) ? "gdn_bwd_wide_kernel" : "gdn_bwd_fused_kernel";
    snprintf(buf, sizeof(buf), "%s<%d>", nm, C);
    return buf;
}

}  // extern "C"
