// Argument block of the implicit-GEMM conv kernels (conv.hip, conv_quad.hip).
#pragma once

#include "common.hpp"

namespace cai {

struct PhaseDesc {
    int oy0, ox0;     // output offset of this phase
    int OHg, OWg;     // GEMM row grid of this phase
    int ntaps, ntx;   // taps, taps per kernel row
    int dy0, dx0;     // input offset of tap 0
    int K;            // ntaps * Cin_pad
    int pad_;
    int64_t w_off;    // element offset of this phase's packed weights
};

struct ConvArgs {
    const void* x;
    int B, IH, IW, x_ld, Cin_pad, in_abs;
    const void* w;
    int Kp, Npad;
    int nphase;
    int tap_sy, tap_sx;
    int row_stride, out_step;
    int out_h, out_w, Cout;
    void* y;
    int y_dtype, y_vec;
    int64_t ysb, ysc, ysy, ysx;
    const float* bias;
    int act;
    float act_param;
    const void* aux;
    int aux_ld, mask_mode;
    float mask_param;
    const bf16* res;         // residual input (cai_conv_fwd_res): y = act(conv + bias + res), pixel-major bf16, NULL: none
    int res_ld;
    const bf16* res2;        // a second residual (dgrad only, cai_conv_dgrad_res2), same layout as res; NULL: none
    int res2_ld;
    int res_post;            // dgrad: the mask scales the conv's input gradient only, the residuals are added after it
    int ksplit;              // K splits per phase (grid.z = nphase * ksplit)
    float* ws;               // split-K partials [nphase*ksplit][ws_rows][ws_ld] fp32
    int ws_rows, ws_ld;
    PhaseDesc ph[4];
};

// The four-phase k5 s2 kernel (conv_quad.hip).  conv_quad_ok: the phase descriptors and the output take its
// path (128 input channels, <= 128 output channels, k5 s2 p2 phases, bf16 output by the register-direct
// epilogue without mask or residual); the caller has checked the grid (>= 256 tiles, no split).
bool conv_quad_ok(const ConvArgs& a);
void launch_conv_halo_quad(const ConvArgs& a, int tiles_x, int tiles_y, int mtiles, hipStream_t st);

}  // namespace cai
