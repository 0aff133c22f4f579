// Weight fragments of the space-to-depth edge layers (edge.hip), shared with the per-model weight
// packer (conv.hip pack_many): one 16-byte bf16 MFMA B-operand fragment per (k-step, n-tile, lane).
//
//   s2d (conv forward, emode 0; deconv input gradient, emode 1):
//     fragment f = (ks * N/16 + nt) * 64 + lane, element e:
//       tap t = 2 ks + (lane >> 5), superpixel channel ch = 8 ((lane >> 4) & 1) + e, n = 16 nt + (lane & 15)
//       value W1[t][ch][n] (emode 0) or W2[8 - t][n][ch] (emode 1)
//   d2s (deconv forward, emode 2):
//     fragment f = (t * N/32 + w) * 64 + lane, element e:
//       ci = 32 w + 8 (lane >> 4) + e, c16 = lane & 15, value W2[t][ci][c16]
// with W1[t=(dy,dx)][(py,px,ci)][n] = W[n][ci][2dy+py+k/2][2dx+px+k/2] (Conv2d [N][C][k][k]) and
// W2[t][ci][(py,px,co)] = W[ci][co][py-2dy+k/2][px-2dx+k/2] (ConvTranspose2d [N][C][k][k]),
// zero where the tap falls outside the k x k kernel (t = 9 is the zero padding tap of the s2d K).
#pragma once

#include "common.hpp"

namespace cai {

struct EdgeFragSpec {
    int C, N, k, p;
    int emode;    // 0: conv s2d, 1: deconv dgrad s2d, 2: deconv fwd d2s
    int nfrag;    // 16-byte fragments
};

// host: the fragment set of one direction of an edge layer (false: not an edge geometry / direction)
bool edge_frag_spec(const cai_conv_geom* g, int dtype, int direction, EdgeFragSpec& s);

__device__ __forceinline__ float edge_w2(const float* w, int C, int k, int p, int t, int ci, int c16) {
    const int sp = c16 / C, co = c16 - sp * C;
    const int ky = (sp >> 1) - 2 * (t / 3 - 1) + p, kx = (sp & 1) - 2 * (t % 3 - 1) + p;
    if (t < 0 || t > 8 || c16 >= 4 * C || ky < 0 || ky >= k || kx < 0 || kx >= k) return 0.f;
    return w[((ci * C + co) * k + ky) * k + kx];
}

__device__ __forceinline__ float edge_w1(const float* w, int C, int k, int p, int t, int ch, int n) {
    const int sp = ch / C, ci = ch - sp * C;
    const int ky = 2 * (t / 3 - 1) + (sp >> 1) + p, kx = 2 * (t % 3 - 1) + (sp & 1) + p;
    if (t > 8 || ch >= 4 * C || ky < 0 || ky >= k || kx < 0 || kx >= k) return 0.f;
    return w[((n * C + ci) * k + ky) * k + kx];
}

// the 8 elements of fragment f
__device__ __forceinline__ void edge_frag_values(const float* w, int C, int N, int k, int p, int emode, int f,
                                                 float (&v)[8]) {
    const int lane = f & 63, g = lane >> 4, i16 = lane & 15;
    if (emode == 2) {
        const int nw = N / 32, t = (f >> 6) / nw, wv = (f >> 6) - t * nw;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = edge_w2(w, C, k, p, t, 32 * wv + 8 * g + e, i16);
        return;
    }
    const int nt_all = N / 16, ks = (f >> 6) / nt_all, nt = (f >> 6) - ks * nt_all;
    const int t = 2 * ks + (g >> 1), ch0 = 8 * (g & 1), n = 16 * nt + i16;
#pragma unroll
    for (int e = 0; e < 8; ++e)
        v[e] = emode == 0 ? edge_w1(w, C, k, p, t, ch0 + e, n) : edge_w2(w, C, k, p, 8 - t, n, ch0 + e);
}

}  // namespace cai
