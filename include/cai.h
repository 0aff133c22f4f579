/*
 * libcai -- C ABI of the MI355X (gfx950) learned-compression hot path.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t
 * (passed as void*), allocates nothing persistent (scratch comes in as a
 * caller-owned workspace), keeps no global mutable state and is reentrant:
 * one host thread per device (DataParallel-style) or one process per GPU
 * (DDP) may call it concurrently.  All launches go to the given stream, so a
 * caller may capture them into a hipGraph.
 *
 * Return value: 0 (CAI_OK) on success, otherwise a CAI_E* code; a
 * thread-local message is available from cai_last_error().
 *
 * Tensor convention ("pixel-major"): an activation of logical NCHW shape
 * [B,C,H,W] is stored channels-last: element (p, c) with p = (b*H + y)*W + x
 * lives at ptr[p*ld + c] (ld >= C: pixel stride in elements).  This is what a
 * torch tensor in torch.channels_last memory format is; channel slices of a
 * wider tensor (chunk(2, 1)) are expressed with ld > C and an offset pointer.
 *
 * Reference interfaces replaced (paths relative to /root/reference/CompressAI):
 *   conv / deconv factories ........ compressai/models/utils.py:128-146 (nn.Conv2d / nn.ConvTranspose2d)
 *   GDN / IGDN ...................... compressai/layers/gdn.py:41-92 (+ ops/parametrizers.py:47-64, ops/bound_ops.py:36-80)
 *   EntropyModel.quantize ........... compressai/entropy_models/entropy_models.py:157-182
 *   EntropyBottleneck ............... entropy_models.py:450-540 (_logits_cumulative :457-477, _likelihood :480-492, loss :450-454)
 *   GaussianConditional ............. entropy_models.py:629-635,692-731
 *   RateDistortionLoss .............. examples/train.py:59-82
 *   Adam step + clip_grad_norm_ ..... examples/train.py:111-142,176-186 (torch.optim.Adam, torch.nn.utils.clip_grad_norm_)
 */
#ifndef CAI_H
#define CAI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define CAI_OK 0
#define CAI_EINVAL 1      /* bad argument / shape (python shim raises ValueError) */
#define CAI_EDEVICE 2     /* HIP launch / runtime error (python shim raises RuntimeError) */
#define CAI_EWORKSPACE 3  /* workspace too small */

/* ---- element types ---------------------------------------------------- */
#define CAI_F32 0
#define CAI_BF16 1

/* ---- epilogue activations / gradient masks ---------------------------- */
#define CAI_ACT_NONE 0
#define CAI_ACT_RELU 1
#define CAI_ACT_LEAKY 2   /* LeakyReLU, negative_slope = act_param */

#define CAI_MASK_NONE 0
#define CAI_MASK_POS 1    /* dgrad epilogue: out *= (aux > 0)          (ReLU backward)      */
#define CAI_MASK_LEAKY 2  /* dgrad epilogue: out *= aux > 0 ? 1 : slope (LeakyReLU backward) */
#define CAI_MASK_SIGN 3   /* dgrad epilogue: out *= sign(aux)           (abs backward)       */
/* flag OR-ed into the mask mode of cai_conv_dgrad_res / _res2: the mask scales the conv's input gradient
 * only and the residual gradients are added after it -- dx = mask(aux) * conv_input_grad(dy) + res (+ res2):
 * a tensor read by a masked first layer (h_a's abs, google.py) and by a second consumer */
#define CAI_MASK_BEFORE_RES 16

/* ---- quantisation modes (entropy_models.py:157-182) -------------------- */
#define CAI_Q_NOISE 0
#define CAI_Q_DEQUANTIZE 1
#define CAI_Q_SYMBOLS 2

/* ---- misc ------------------------------------------------------------- */
const char* cai_last_error(void);
int cai_version(void);
/* number of entry points exported below (checked by the loader test) */
int cai_abi_count(void);

/* =======================================================================
 * Convolution (implicit GEMM on MFMA).  One geometry struct describes the
 * *module*: an nn.Conv2d (transposed = 0) or nn.ConvTranspose2d
 * (transposed = 1) with square kernel, symmetric padding and output_padding.
 * Spatial sizes are those of the module's input (in_h, in_w) and output
 * (out_h, out_w); the library checks them against the module formula.
 * ======================================================================= */
typedef struct cai_conv_geom {
    int32_t batch;
    int32_t in_c, in_h, in_w;
    int32_t out_c, out_h, out_w;
    int32_t kernel, stride, pad, output_padding;
    int32_t transposed;
} cai_conv_geom;

/* Bytes of the packed-weight buffer for one direction (0 = forward,
 * 1 = input-gradient) at element type dtype. */
size_t cai_conv_packed_weight_bytes(const cai_conv_geom* g, int dtype, int direction);

/* Repack the fp32 torch weight ([out,in,k,k] for Conv2d, [in,out,k,k] for
 * ConvTranspose2d) into the per-phase MFMA layout for `direction`;
 * mask (nullable, same shape as w) multiplies the weight (MaskedConv2d). */
int cai_conv_pack_weight(const cai_conv_geom* g, int dtype, int direction,
                         const float* w, const float* mask, void* packed, void* stream);

/* Batched packing (one launch per step for all convs of a model): the host
 * fills a cai_conv_pack_desc_bytes()-sized descriptor per (conv, direction)
 * with cai_conv_pack_describe() (pointers captured, nothing launched), copies
 * the table to device memory once, and each step calls cai_conv_pack_many()
 * on it. */
size_t cai_conv_pack_desc_bytes(void);
int cai_conv_pack_describe(const cai_conv_geom* g, int dtype, int direction, const float* w, const float* mask,
                           void* packed, void* desc);
/* host side, once: number the 8-element work items of a contiguous table of n
 * descriptors; returns the total item count (total_items of pack_many). */
int64_t cai_conv_pack_finalize(void* descs, int32_t n);
/* A GDN / IGDN reparametrisation (cai_gdn_reparam's outputs: beta, gamma_op in
 * the pack_many dtype) as one more pack_many descriptor, so a model's GDN layers
 * are reparametrised in the same launch as its conv weights are packed
 * (replaces the per-layer NonNegativeParametrizer calls, layers/gdn.py:77-92,
 * ops/parametrizers.py:47-64). */
int cai_gdn_reparam_describe(const float* beta_raw, const float* gamma_raw, int32_t C, float beta_min,
                             float reparam_offset, float* beta, void* gamma_op, void* desc);
int cai_conv_pack_many(const void* descs, int32_t n, int dtype, int64_t total_items, void* stream);

/* NCHW (fp32, contiguous) -> pixel-major [B*H*W][ld] of dtype with zero
 * padding of channels C..ld-1.  ld must be a multiple of 8. */
int cai_pack_nchw(const float* x, int32_t B, int32_t C, int32_t H, int32_t W,
                  int dtype, void* out, int32_t ld, void* stream);

/* Scratch for split-K (small spatial layers whose tile grid cannot fill the
 * GPU split the reduction dimension over workgroups and reduce the fp32
 * partials in a fixed order); 0 when the call does not split. */
size_t cai_conv_workspace_bytes(const cai_conv_geom* g, int dtype, int direction);

/* forward: y = act(conv(x) + bias).  x: pixel-major input with ld x_ld
 * (x_ld >= in_c, multiple of 8 elements);  in_abs != 0 reads |x|.
 * y is written at y_ptr[b*ysb + c*ysc + oy*ysy + ox*ysx] (element strides);
 * y_dtype may differ from dtype (the operand type). */
int cai_conv_fwd(const cai_conv_geom* g, int dtype,
                 const void* x, int32_t x_ld, int32_t in_abs,
                 const void* packed_w, const float* bias,
                 int32_t act, float act_param,
                 void* y, int y_dtype, int64_t ysb, int64_t ysc, int64_t ysy, int64_t ysx,
                 void* workspace, size_t ws_bytes, void* stream);

/* forward with a residual: y = act(conv(x) + bias + res), the ResidualUnit of
 * cheng2020-attn's attention blocks (CompressAI/compressai/layers/layers.py:
 * 211-226, `out = self.conv(x); out += identity; out = self.relu(out)`)
 * in the conv epilogue.  bf16 only; res pixel-major with ld res_ld (>= out_c,
 * multiple of 4, 8-byte aligned); y pixel-major bf16 (ysc == 1). */
int cai_conv_fwd_res(const cai_conv_geom* g, int dtype,
                     const void* x, int32_t x_ld, int32_t in_abs,
                     const void* packed_w, const float* bias,
                     int32_t act, float act_param, const void* res, int32_t res_ld,
                     void* y, int y_dtype, int64_t ysb, int64_t ysc, int64_t ysy, int64_t ysx,
                     void* workspace, size_t ws_bytes, void* stream);

/* input gradient: dx = mask(aux) * conv_input_grad(dy).  dy pixel-major
 * (ld dy_ld), dx pixel-major (ld dx_ld), aux pixel-major (ld aux_ld) or NULL. */
int cai_conv_dgrad(const cai_conv_geom* g, int dtype,
                   const void* dy, int32_t dy_ld, const void* packed_wt,
                   void* dx, int32_t dx_ld,
                   int32_t mask_mode, float mask_param, const void* aux, int32_t aux_ld,
                   void* workspace, size_t ws_bytes, void* stream);

/* input gradient plus a residual gradient: dx = mask(aux) * (conv_input_grad(dy)
 * + res) (bf16), the gradient of a ResidualUnit's input (layers.py:211-226: x
 * feeds the first conv and the `out += identity` add) in the first conv's dgrad
 * epilogue instead of a separate sum; the mask (MASK_POS on the unit's input)
 * is the previous unit's trailing ReLU.  res pixel-major as in cai_conv_fwd_res. */
int cai_conv_dgrad_res(const cai_conv_geom* g, int dtype,
                       const void* dy, int32_t dy_ld, const void* packed_wt,
                       const void* res, int32_t res_ld, void* dx, int32_t dx_ld,
                       int32_t mask_mode, float mask_param, const void* aux, int32_t aux_ld,
                       void* workspace, size_t ws_bytes, void* stream);

/* as cai_conv_dgrad_res with a second residual gradient: dx = mask(aux) *
 * (conv_input_grad(dy) + res + res2) -- AttentionBlock's input (layers.py:
 * 196-244) feeds both residual branches and the gate's `+ identity`. */
int cai_conv_dgrad_res2(const cai_conv_geom* g, int dtype,
                        const void* dy, int32_t dy_ld, const void* packed_wt,
                        const void* res, int32_t res_ld, const void* res2, int32_t res2_ld,
                        void* dx, int32_t dx_ld,
                        int32_t mask_mode, float mask_param, const void* aux, int32_t aux_ld,
                        void* workspace, size_t ws_bytes, void* stream);

/* cheng2020's ResidualUnit (layers.py:211-226; AttentionBlock's conv_a / conv_b units, :225-236) in ONE launch
 * per direction (csrc/resunit.hip): h1 = relu(conv1x1_a(x) + ba), h2 = relu(conv3x3_b(h1) + bb),
 * y = relu(conv1x1_c(h2) + bc + x); x / y with n in {128, 192} channels, h1 / h2 with n / 2 (ld n / 2), bf16
 * pixel-major.  Replaces the unit's three cai_conv_fwd(_res) calls (forward) and three cai_conv_dgrad(_res)
 * calls (backward); the weight gradients stay cai_conv_wgrad calls on the tensors this writes.
 *   direction 0: x = the unit input; wa / wb / wc = a, b, c packed for direction 0 (cai_conv_pack_weight) with
 *     row lengths kpa / kpb / kpc; writes h1, h2 and out = y.
 *   direction 1: x = gy (dLoss/dy; y = the forward output, its ReLU mask applied here unless gy_masked);
 *     wa / wb / wc = c, b, a packed for direction 1; h1 / h2 = the forward's; writes gc = gy * (y > 0) (when
 *     !gy_masked), gb = dLoss/d(b's pre-activation), ga = dLoss/d(a's pre-activation) and
 *     out = dx = (ga . Wa^T + gc [+ res2]) [* (xmask > 0)]. */
typedef struct cai_resunit_args {
    int32_t batch, h, w, n;
    const void* x;
    const void* y;
    const void* wa;
    const void* wb;
    const void* wc;
    const float* ba;
    const float* bb;
    const float* bc;
    void* h1;
    void* h2;
    void* out;
    void* gc;
    void* gb;
    void* ga;
    const void* res2;
    const void* xmask;
    int32_t x_ld, y_ld, out_ld, res2_ld, xmask_ld;
    int32_t kpa, kpb, kpc;
    int32_t gy_masked;
} cai_resunit_args;
int cai_resunit(const cai_resunit_args* args, int32_t direction, void* stream);

/* Diagnostics for measurement (bench.py's per-launch roofline):
 * the kernel a conv call would launch (direction 0 = forward, 1 = input
 * gradient, 2 = weight gradient) as the name rocprofv3 reports, "" for an
 * invalid call; and its split factor (split-K slabs / wgrad pixel splits). */
const char* cai_conv_kernel_name(const cai_conv_geom* g, int dtype, int direction, int32_t in_abs);
int32_t cai_conv_split_factor(const cai_conv_geom* g, int dtype, int direction, int32_t in_abs);

/* weight / bias gradient (fp32, torch layout; overwritten, or added to the
 * existing values when accumulate != 0 -- the .grad += semantics of autograd,
 * used to write straight into an optimizer's flat gradient buffer).
 * x: module input (pixel-major, ld x_ld, in_abs as in forward; in_sq != 0
 * squares it), dy: output gradient (pixel-major, ld dy_ld).  db may be NULL. */
size_t cai_conv_wgrad_workspace_bytes(const cai_conv_geom* g, int dtype);
int cai_conv_wgrad(const cai_conv_geom* g, int dtype,
                   const void* x, int32_t x_ld, int32_t in_abs, int32_t in_sq,
                   const void* dy, int32_t dy_ld,
                   float* dw, float* db, int32_t accumulate,
                   void* workspace, size_t ws_bytes, void* stream);

/* Deferred parameter-gradient reduces.  A weight-gradient call can leave its final fixed-order reduce
 * (split slabs -> torch layout) as a job instead of launching it; cai_reduce_jobs runs any number of jobs in
 * ceil(n / 16) launches, each job on its own range of blocks.  The caller keeps the job's workspace alive
 * and unmodified, and reads the gradient only after cai_reduce_jobs on the same stream (compressai._ops
 * queues the jobs of one backward pass and runs them in an autograd final callback).  Results are
 * bit-identical to the immediate calls, which run their one job through the same kernel.  Job fields are
 * the library's own (filled by the *_deferred calls); kind CAI_JOB_NONE: nothing left to reduce. */
#define CAI_JOB_NONE 0
#define CAI_JOB_WGRAD 1
#define CAI_JOB_GDN 2
#define CAI_JOB_EDGE 3
typedef struct cai_reduce_job {
    int32_t kind, nblocks;
    int32_t i[10];
    float f[2];
    const void* p[6];
} cai_reduce_job;
int cai_conv_wgrad_deferred(const cai_conv_geom* g, int dtype,
                            const void* x, int32_t x_ld, int32_t in_abs, int32_t in_sq,
                            const void* dy, int32_t dy_ld,
                            float* dw, float* db, int32_t accumulate,
                            void* workspace, size_t ws_bytes, void* stream, cai_reduce_job* job);
int cai_reduce_jobs(const cai_reduce_job* jobs, int32_t n, void* stream);
/* cai_reduce_jobs with the grid capped at max_blocks (0 = uncapped): each block walks the batch's blocks in order,
 * same arithmetic per output (bit-identical).  For a reduce launched on a side stream beside the backward's chain
 * (compressai/_ops.py early reduces), so it holds a bounded share of the CUs. */
int cai_reduce_jobs_grid(const cai_reduce_job* jobs, int32_t n, int32_t max_blocks, void* stream);
/* n weight-gradient calls, each as cai_conv_wgrad_deferred makes it (jobs[i]: call i's reduce job), grouped
 * into batched launches: the latent-size ones (the wgrad_small_kernel path, cai_conv_kernel_name(direction 2)
 * == "wgrad_small_kernel") one launch per input transform, and the pixel-split ones (wgrad_glds_kernel<128 /
 * 256>, wgrad_halo_kernel variants) one launch per kernel variant, up to 16 (WG_BATCH_MAX) calls per launch;
 * two calls that write one bias gradient go to separate launches, in call order, and a pixel-split call whose
 * bias gradient is not fused into its kernel runs on its own.  Replaces a backward's per-layer launches of
 * those weight gradients, deferred to its end (compressai/_ops.py conv_wgrad).
 * Operands as cai_conv_wgrad_deferred; every call's buffers must stay valid until its reduce job has run. */
typedef struct cai_wgrad_call {
    cai_conv_geom geom;
    int32_t dtype;
    const void* x;
    int32_t x_ld, in_abs, in_sq;
    const void* dy;
    int32_t dy_ld;
    float* dw;
    float* db;
    int32_t accumulate;
    void* workspace;
    size_t ws_bytes;
} cai_wgrad_call;
int cai_conv_wgrad_batch(const cai_wgrad_call* calls, int32_t n, void* stream, cai_reduce_job* jobs);

/* The three weight (+ bias) gradients of a ResidualUnit (layers.py:211-226) in one launch, from the
 * tensors cai_resunit's backward leaves: x (the unit input, ld x_ld), h1 / h2 (the hidden activations,
 * ld n/2), ga / gb (the pre-activation gradients of a and b, ld n/2), gc (of c, ld gc_ld), all pixel-major
 * bf16.  dwa [n/2][n][1][1], dwb [n/2][n/2][3][3], dwc [n][n/2][1][1] and the biases: torch layout fp32,
 * overwritten or accumulated.  Replaces the three cai_conv_wgrad calls of a unit (compressai/_ops.py
 * _resunit_bwd).  jobs != NULL: the final slab sums are returned as three CAI_JOB_WGRAD jobs (run later by
 * cai_reduce_jobs, workspace kept alive until then); NULL: run now.  n in {128, 192}. */
typedef struct cai_resunit_wgrad_args {
    int32_t batch, h, w, n;
    const void* x;
    const void* h1;
    const void* h2;
    const void* ga;
    const void* gb;
    const void* gc;
    int32_t x_ld, gc_ld;
    float* dwa;
    float* dba;
    float* dwb;
    float* dbb;
    float* dwc;
    float* dbc;
    int32_t accumulate;
} cai_resunit_wgrad_args;
size_t cai_resunit_wgrad_workspace_bytes(const cai_resunit_wgrad_args* args);
/* n cai_resunit_wgrad calls (each with its own workspace, kept valid until its jobs have run) in one launch per
 * width; jobs: 3 per call, in call order.  The backward's ResidualUnit weight gradients, deferred to its end
 * (compressai/_ops.py _resunit_wgrad): one launch instead of one per unit, the small units' grids filling the
 * chip together. */
int cai_resunit_wgrad_batch(const cai_resunit_wgrad_args* args, void* const* workspaces, const size_t* ws_bytes,
                            int32_t n, void* stream, cai_reduce_job* jobs);
int cai_resunit_wgrad(const cai_resunit_wgrad_args* args, void* workspace, size_t ws_bytes, void* stream,
                      cai_reduce_job* jobs);

/* ConvTranspose2d with out_c <= 16 (the synthesis transform's last layer,
 * models/utils.py:138-146, e.g. deconv(N, 3)): forward as one dense GEMM per
 * input pixel (N = k*k*out_c columns) + col2im, backward as im2col + two 1x1
 * GEMMs.  w / dw: torch layout [in_c][out_c][k][k] fp32 (dw overwritten or
 * accumulated); y / dy: fp32 NCHW contiguous (x_hat); x / dx pixel-major. */
size_t cai_deconv_small_workspace_bytes(const cai_conv_geom* g, int dtype);
int cai_deconv_small_fwd(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld,
                         const float* w, const float* bias, float* y,
                         void* workspace, size_t ws_bytes, void* stream);
int cai_deconv_small_bwd(const cai_conv_geom* g, int dtype, const void* x, int32_t x_ld,
                         const float* w, const float* dy, void* dx, int32_t dx_ld,
                         float* dw, float* db, int32_t accumulate,
                         void* workspace, size_t ws_bytes, void* stream);

/* =======================================================================
 * Stride-2 edge layers through the space-to-depth view (csrc/edge.hip):
 * the analysis transform's first Conv2d(C, N, k, 2, k/2) and the synthesis
 * transform's last ConvTranspose2d(N, C, k, 2, k/2, output_padding 1)
 * (models/utils.py:21-38, google.py:96-112 / 145-170), C <= 3, k odd <= 5,
 * N in {128, 192}, bf16 compute.  The image side is NCHW fp32
 * [B, C, 2Hs, 2Ws], the feature side pixel-major bf16 [B, Hs, Ws, N] (ld).
 * ======================================================================= */
/* 1 when the edge path takes this geometry and dtype, else 0. */
int cai_edge_supported(const cai_conv_geom* g, int dtype);
/* Workspace of cai_edge_wgrad (0 when unsupported). */
size_t cai_edge_workspace_bytes(const cai_conv_geom* g, int dtype);
/* Packed bf16 MFMA weight fragments of one direction (0: forward, 1: the
 * deconv's input gradient) from the fp32 torch weight; bytes 0 = unsupported.
 * cai_edge_pack_describe fills a cai_conv_pack_many descriptor instead (the
 * per-model one-launch packer). */
size_t cai_edge_frag_bytes(const cai_conv_geom* g, int dtype, int direction);
int cai_edge_pack_weights(const cai_conv_geom* g, int dtype, int direction, const float* w, void* frag,
                          void* stream);
int cai_edge_pack_describe(const cai_conv_geom* g, int dtype, int direction, const float* w, void* frag,
                           void* desc);
/* Conv forward: y = conv(x) + bias, x NCHW fp32, y pixel-major bf16. */
int cai_edge_conv_fwd(const cai_conv_geom* g, const float* x, const void* frag, const float* bias, void* y,
                      int32_t y_ld, void* stream);
/* ConvTranspose forward: y (NCHW fp32) = deconv(x) + bias, x pixel-major bf16. */
int cai_edge_deconv_fwd(const cai_conv_geom* g, const void* x, int32_t x_ld, const void* frag, const float* bias,
                        float* y, void* stream);
/* ConvTranspose input gradient: dx (pixel-major bf16) from dy (NCHW fp32). */
int cai_edge_deconv_dgrad(const cai_conv_geom* g, const float* dy, const void* frag, void* dx, int32_t dx_ld,
                          void* stream);
/* Weight / bias gradients of either layer into the torch layouts (accumulate: +=).
 * conv: img = x, feat = dy; deconv: img = dy, feat = x.  Fixed-order reduction. */
int cai_edge_wgrad(const cai_conv_geom* g, const float* img, const void* feat, int32_t feat_ld, float* dw, float* db,
                   int32_t accumulate, void* workspace, size_t ws_bytes, void* stream);
/* cai_edge_wgrad with its final reduce left as a job (cai_reduce_jobs). */
int cai_edge_wgrad_deferred(const cai_conv_geom* g, const float* img, const void* feat, int32_t feat_ld, float* dw,
                            float* db, int32_t accumulate, void* workspace, size_t ws_bytes, void* stream,
                            cai_reduce_job* job);

/* =======================================================================
 * Pointwise glue of the residual / attention / sub-pixel blocks
 * (layers/layers.py:81-244), pixel-major, ld a multiple of 8 (bf16) / 4 (fp32).
 * ======================================================================= */
/* y = act(a + b): `out += identity` (layers.py:124,177) with the trailing
 * ReLU of AttentionBlock's ResidualUnit (layers.py:222-226) folded in. */
int cai_add_act(int dtype, const void* a, int32_t a_ld, const void* b, int32_t b_ld, void* y, int32_t y_ld,
                int64_t npix, int32_t C, int32_t act, float act_param, void* stream);
/* y = act(x) for a ReLU / LeakyReLU that no conv epilogue can absorb. */
int cai_act(int dtype, const void* x, int32_t x_ld, void* y, int32_t y_ld, int64_t npix, int32_t C, int32_t act,
            float act_param, void* stream);
/* y[i] += x[i] * g[0] (fp32, g a device scalar): a gradient accumulated with its upstream gradient read on
 * the device (EntropyBottleneck.loss's backward into an optimizer's flat buffer, compressai/_ops.py). */
int cai_axpy_dev(int64_t n, const float* x, const float* g, float* y, void* stream);
/* AttentionBlock gate (layers.py:238-243): y = a * sigmoid(b) + x;
 * backward da = g * s(b), db = g * a * s(b) * (1 - s(b)) (dx = g). */
/* GDN1 (layers/gdn.py:95-121): y = x / norm (inverse: x * norm), norm from a 1x1 conv of |x|
 * (cai_conv_fwd with in_abs); backward dx = g / norm, dnorm = -g x / norm^2 (inverse: g norm, g x). */
int cai_gdn1_out(int dtype, const void* x, int32_t x_ld, const void* norm, int32_t n_ld, void* y, int32_t y_ld,
                 int64_t npix, int32_t C, int32_t inverse, void* stream);
int cai_gdn1_out_bwd(int dtype, const void* x, int32_t x_ld, const void* norm, int32_t n_ld, const void* g,
                     int32_t g_ld, void* dx, int32_t dx_ld, void* dnorm, int32_t dn_ld, int64_t npix, int32_t C,
                     int32_t inverse, void* stream);
int cai_gate_fwd(int dtype, const void* a, const void* b, const void* x, void* y, int32_t ld, int64_t npix, int32_t C,
                 void* stream);
/* relu_a != 0: a is a ReLU output and da carries its mask (da = g sigmoid(b) [a > 0]) */
int cai_gate_bwd(int dtype, const void* a, const void* b, const void* g, int32_t g_ld, void* da, void* db, int32_t ld,
                 int64_t npix, int32_t C, int32_t relu_a, void* stream);
/* nn.PixelShuffle(r) of subpel_conv3x3 (layers.py:86-91) between
 * x[B][H][W][C*r*r] and y[B][H*r][W*r][C], each side described by element
 * strides {batch, row, column, channel}; inverse != 0 maps y back to x
 * (the backward).  src/dst strides describe the source/destination. */
int cai_pixel_shuffle(int dtype, const void* src, const int64_t* src_strides, void* dst, const int64_t* dst_strides,
                      int32_t B, int32_t H, int32_t W, int32_t C, int32_t r, int32_t inverse, void* stream);

/* =======================================================================
 * Multi-modal codec alignment modules (models/master.py): LayerNorm, GELU,
 * shifted-window cross attention, Channel_aligner pooling + affine.
 * Tokens are pixel-major rows (row = b*L + l, l = r*Wr + c).
 * ======================================================================= */
/* nn.LayerNorm over C (SwinTransformerBlock.norm1/norm2, master.py:603-606).
 * mean / rstd (fp32, one per token) are saved for the backward. */
int cai_layernorm_fwd(int dtype, const void* x, int32_t x_ld, int64_t ntok, int32_t C, const float* w, const float* b,
                      float eps, void* y, int32_t y_ld, float* mean, float* rstd, void* stream);
size_t cai_layernorm_bwd_workspace_bytes(int64_t ntok, int32_t C);
int cai_layernorm_bwd(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t ntok, int32_t C,
                      const float* w, const float* mean, const float* rstd, void* dx, int32_t dx_ld, float* dw,
                      float* db, int32_t accumulate, void* workspace, size_t ws_bytes, void* stream);
/* exact (erf) GELU of Mlp.act (master.py:465-482). */
int cai_gelu_fwd(int dtype, const void* x, int32_t x_ld, void* y, int32_t y_ld, int64_t ntok, int32_t C, void* stream);
int cai_gelu_bwd(int dtype, const void* x, int32_t x_ld, const void* g, int32_t g_ld, void* dx, int32_t dx_ld,
                 int64_t ntok, int32_t C, void* stream);

/* WindowAttention.forward (master.py:534-568) with SwinTransformerBlock's
 * cyclic shift and window partition / reverse (master.py:665-695) folded into
 * the token addressing: q = qkv1(x) rows, kv = qkv2(guided) rows (k = columns
 * [0, C), v = [C, 2C), C = heads*head_dim); output rows in token order (before
 * the proj Linear).  window 4, head_dim 32 are built. */
typedef struct cai_window_attn {
    const void* q;
    int32_t q_ld;
    const void* kv;
    int32_t kv_ld;
    const float* bias_table;   /* relative_position_bias_table [(2w-1)^2][heads] */
    const int32_t* rel_index;  /* relative_position_index [w*w][w*w] */
    const float* mask;         /* attn_mask [nW][w*w][w*w] or NULL */
    int32_t B, Hr, Wr;         /* token grid (input_resolution) */
    int32_t heads, head_dim, window, shift;
    float scale;
} cai_window_attn;
int cai_window_attn_fwd(int dtype, const cai_window_attn* p, void* out, int32_t out_ld, void* stream);
size_t cai_window_attn_bwd_workspace_bytes(const cai_window_attn* p);
int cai_window_attn_bwd(int dtype, const cai_window_attn* p, const void* dout, int32_t dout_ld, void* dq,
                        int32_t dq_ld, void* dkv, int32_t dkv_ld, float* dbias_table, int32_t accumulate,
                        void* workspace, size_t ws_bytes, void* stream);

/* Channel_aligner (master.py:179-210): out[b][c] = scale * sum_p x[b,p,c] (* x2[b,p,c])
 * (AdaptiveAvgPool2d(1) with scale = 1/HW; with x2, the gamma gradient): pixel chunks in parallel, then
 * a fixed-order sum of the chunk partials (workspace: cai_channel_mean_workspace_bytes);
 * y = gamma[b][c] * x + beta_scale * beta[b][c] (gamma / beta nullable). */
size_t cai_channel_mean_workspace_bytes(int32_t B, int64_t HW, int32_t C);
int cai_channel_mean(int dtype, const void* x, int32_t x_ld, const void* x2, int32_t x2_ld, int32_t B, int64_t HW,
                     int32_t C, float* out, float scale, void* workspace, size_t ws_bytes, void* stream);
int cai_channel_affine(int dtype, const void* x, int32_t x_ld, const float* gamma, const float* beta, float beta_scale,
                       void* y, int32_t y_ld, int32_t B, int64_t HW, int32_t C, void* stream);

/* =======================================================================
 * GDN / IGDN (layers/gdn.py:41-92), C a multiple of 32 up to 256 (bf16) / 192 (fp32);
 * layers/gdn.py zero-pads other channel counts.
 * ======================================================================= */
/* beta = max(beta_raw, sqrt(beta_min + ped))^2 - ped ; gamma likewise with
 * bound sqrt(ped); gamma_op is written in the operand dtype in both the
 * [i][j] and the transposed [j][i] order (2*C*C elements). */
int cai_gdn_reparam(const float* beta_raw, const float* gamma_raw, int32_t C,
                    float beta_min, float reparam_offset, int dtype,
                    float* beta, void* gamma_op, void* stream);
int cai_gdn_fwd(int dtype, const void* x, int32_t x_ld, int64_t npix, int32_t C,
                const void* gamma_op, const float* beta, int32_t inverse,
                void* y, int32_t y_ld, void* stream);
/* dx and u (= dLoss/dnorm, pixel-major [npix][C], operand dtype); dgamma and
 * dbeta are produced afterwards by cai_gdn_param_grad. */
int cai_gdn_bwd(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld,
                int64_t npix, int32_t C, const void* gamma_op, const float* beta,
                int32_t inverse, void* dx, int32_t dx_ld, void* u, void* stream);
size_t cai_gdn_param_grad_workspace_bytes(int64_t npix, int32_t C, int dtype);
/* dgamma_raw/dbeta_raw (fp32; overwritten or, accumulate != 0, added) through
 * the NonNegativeParametrizer / LowerBound backward rule (bound_ops.py:40-42). */
int cai_gdn_param_grad(int dtype, const void* x, int32_t x_ld, const void* u, int64_t npix, int32_t C,
                       const float* beta_raw, const float* gamma_raw, float beta_min, float reparam_offset,
                       float* dbeta_raw, float* dgamma_raw, int32_t accumulate,
                       void* workspace, size_t ws_bytes, void* stream);

/* The whole GDN / IGDN backward in one call: dx plus dgamma_raw / dbeta_raw
 * (overwritten, or added with accumulate != 0).  bf16 with C in {64, 128}
 * runs one fused pass over x and dy (dgamma as an MFMA with the pixels as K,
 * per-block partials reduced in a fixed order); other cases run cai_gdn_bwd +
 * cai_gdn_param_grad.  workspace: 256-byte aligned. */
size_t cai_gdn_backward_workspace_bytes(int64_t npix, int32_t C, int dtype);
int cai_gdn_backward(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t npix, int32_t C,
                     const void* gamma_op, const float* beta, int32_t inverse, void* dx, int32_t dx_ld,
                     const float* beta_raw, const float* gamma_raw, float beta_min, float reparam_offset,
                     float* dbeta_raw, float* dgamma_raw, int32_t accumulate, void* workspace, size_t ws_bytes,
                     void* stream);

/* cai_gdn_backward with its parameter-gradient reduce left as a job (see cai_reduce_jobs); the fused
 * pass only (bf16, C in {64, 128, 160, 192}), other cases run immediately and return CAI_JOB_NONE. */
/* The kernel cai_gdn_fwd (direction 0) or cai_gdn_backward (direction 1) launches for these arguments
 * (in_ld: x / dy leading dimension, out_ld: y / dx), e.g. "gdn_fwd_lane_kernel<128>"; "" for bad arguments.
 * Diagnostics for the per-launch ledger and the dispatch tests (no reference counterpart). */
const char* cai_gdn_kernel_name(int dtype, int64_t npix, int32_t C, int32_t in_ld, int32_t out_ld, int32_t direction);
int cai_gdn_backward_deferred(int dtype, const void* x, int32_t x_ld, const void* dy, int32_t dy_ld, int64_t npix,
                              int32_t C, const void* gamma_op, const float* beta, int32_t inverse, void* dx,
                              int32_t dx_ld, const float* beta_raw, const float* gamma_raw, float beta_min,
                              float reparam_offset, float* dbeta_raw, float* dgamma_raw, int32_t accumulate,
                              void* workspace, size_t ws_bytes, void* stream, cai_reduce_job* job);

/* =======================================================================
 * Entropy models.  Element (p, c) of every operand at ptr[p*ld + c].
 * ======================================================================= */
/* Training noise: out[0..n) = U(-1/2, 1/2) (fp32, 24-bit mantissas), Philox4x32-10 keyed by state[0] (the
 * seed) with counter (element quad, state[1]).  state: 3 uint64 in device memory, caller-owned, state[2]
 * zero before the first call; every call advances state[1] by one on the device (its last block to finish),
 * so a captured graph draws fresh noise on each replay.  Replaces the reference's
 * torch.empty_like(x).uniform_(-0.5, 0.5) (entropy_models.py:170) -- same distribution, its own stream. */
int cai_uniform_noise(float* out, int64_t n, unsigned long long* state, void* stream);

/* Noise operand of the NOISE-mode entropy kernels (quantize, gc_fwd/bwd, eb_fwd/bwd):
 *   BUF     element (p, c) = buf[p*ld + c] (fp32), a draw the caller made (cai_uniform_noise, or injected);
 *   DRAW    the kernel draws it itself: element (p, c) = element p*C + c of what cai_uniform_noise would write
 *           into a dense [npix, C] buffer at the generator's current draw index; the kernel records
 *           {seed, draw index} in slot[0..1] and advances the index once (its last block to arrive, on
 *           per-XCD sharded tickets in state[CAI_NOISE_SHARD0 + 16 k], k < 8) -- no noise buffer, no draw launch;
 *   REPLAY  the draw recorded in slot by an earlier DRAW launch (the backward, or a second consumer).
 * state: the generator's CAI_NOISE_STATE_WORDS uint64 (cai_uniform_noise's state, extended by the shards),
 * zero past state[1] before the first call; slot: 2 uint64 in device memory.  DRAW launches that share a
 * state must be ordered (one stream), as cai_uniform_noise calls must. */
#define CAI_NOISE_BUF 0
#define CAI_NOISE_DRAW 1
#define CAI_NOISE_REPLAY 2
#define CAI_NOISE_SHARD0 16
#define CAI_NOISE_STATE_WORDS 144
typedef struct cai_noise_src {
    int32_t kind;
    int32_t ld;                   /* BUF: row stride of buf (>= C) */
    const float* buf;             /* BUF */
    unsigned long long* state;    /* DRAW */
    unsigned long long* slot;     /* DRAW (written) / REPLAY (read) */
} cai_noise_src;

/* quantize: NOISE  out = x + noise  (noise required)
 *           DEQUANTIZE out = rint(x - means) + means  (means nullable)
 *           SYMBOLS    out(int32) = (int)rint(x - means)
 * x_dtype / out_dtype in {CAI_F32, CAI_BF16} (out int32 for SYMBOLS). */
int cai_quantize(int mode, int64_t npix, int32_t C,
                 const void* x, int x_dtype, int32_t x_ld,
                 const float* means, int32_t means_ld, int32_t means_per_channel,
                 const cai_noise_src* noise,
                 void* out, int out_dtype, int32_t out_ld, void* stream);

/* GaussianConditional forward: q = quantize(x) (NOISE or DEQUANTIZE),
 * lik = max(Phi((0.5-|q-mu|)/s) - Phi((-0.5-|q-mu|)/s), lik_bound), s = max(scales, scale_bound).
 * scales/means (means nullable) in dtype sm_dtype.  q may be NULL. */
int cai_gc_fwd(int mode, int64_t npix, int32_t C,
               const void* x, int x_dtype, int32_t x_ld,
               const void* scales, int32_t s_ld, const void* means, int32_t m_ld, int sm_dtype,
               const cai_noise_src* noise,
               float scale_bound, float lik_bound,
               void* q, int q_dtype, int32_t q_ld, float* lik, int32_t lik_ld, void* stream);
/* backward: inputs the gradients wrt lik (fp32, nullable) and wrt q (nullable),
 * outputs dx (x_dtype layout, nullable), dscales, dmeans (sm_dtype, nullable).
 * mode | CAI_GC_SCALES_RELU: the scales are a ReLU's output (ScaleHyperprior's h_s ends in nn.ReLU,
 * models/google.py:282-283 of the reference) and dscales leaves with that ReLU's backward mask (scales > 0) applied. */
#define CAI_GC_SCALES_RELU 16
int cai_gc_bwd(int mode, int64_t npix, int32_t C,
               const void* x, int x_dtype, int32_t x_ld,
               const void* scales, int32_t s_ld, const void* means, int32_t m_ld, int sm_dtype,
               const cai_noise_src* noise,
               float scale_bound, float lik_bound,
               const float* g_lik, int32_t gl_ld, const void* g_q, int gq_dtype, int32_t gq_ld,
               void* dx, int32_t dx_ld, void* dscales, int32_t ds_ld, void* dmeans, int32_t dm_ld,
               void* stream);

/* EntropyBottleneck.  params: the 5 matrices, 5 biases, 4 factors and the
 * quantiles, each fp32 contiguous torch tensors ([C,3,1],[C,3,3]x3,[C,1,3]; bias
 * [C,w,1]; factor [C,3,1]; quantiles [C,1,3]). */
typedef struct cai_eb_params {
    const float* matrix[5];
    const float* bias[5];
    const float* factor[4];
    const float* quantiles;
} cai_eb_params;
typedef struct cai_eb_grads {
    float* matrix[5];
    float* bias[5];
    float* factor[4];
    float* quantiles;   /* medians gradient in DEQUANTIZE mode (nullable) */
    int32_t accumulate; /* 0: overwrite, 1: add to the existing values */
} cai_eb_grads;

int cai_eb_fwd(int mode, int64_t npix, int32_t C, const cai_eb_params* prm,
               const void* x, int x_dtype, int32_t x_ld,
               const cai_noise_src* noise, float lik_bound,
               void* q, int q_dtype, int32_t q_ld, float* lik, int32_t lik_ld, void* stream);
/* Scratch of the split backward / the multi-block aux loss (fp32 partial sums).  Their hand-offs also take
 * caller-owned uint32 tickets -- C for cai_eb_bwd, 1 for cai_eb_aux_loss -- zero before the first call; every
 * call leaves them at zero (the last block of a hand-off resets its ticket), so one zeroed buffer serves every
 * later call and graph replay on the same stream. */
size_t cai_eb_scratch_bytes(int64_t npix, int32_t C);
/* parameter gradients (fp32, torch layout) per grads->accumulate.  Each channel's pixels are split over up to
 * 64 blocks whose sums the last arriving block adds in split order (deterministic); with scratch or tickets
 * NULL (or scratch_bytes short) one block per channel. */
int cai_eb_bwd(int mode, int64_t npix, int32_t C, const cai_eb_params* prm,
               const void* x, int x_dtype, int32_t x_ld,
               const cai_noise_src* noise, float lik_bound,
               const float* g_lik, int32_t gl_ld, const void* g_q, int gq_dtype, int32_t gq_ld,
               void* dx, int32_t dx_ld, const cai_eb_grads* grads,
               float* scratch, size_t scratch_bytes, uint32_t* tickets, void* stream);
/* aux loss sum_c sum_k |F_c(quantiles[c,k]) - target[k]| -> *loss (fp32 scalar);
 * if dquantiles != NULL also writes d loss / d quantiles scaled by *g_loss.  One block per 32 channels; more
 * than 32 channels need scratch (cai_eb_scratch_bytes) and one ticket. */
int cai_eb_aux_loss(int32_t C, const cai_eb_params* prm, const float* target,
                    float* loss, const float* g_loss, float* dquantiles, int32_t accumulate,
                    float* scratch, size_t scratch_bytes, uint32_t* ticket, void* stream);

/* =======================================================================
 * Rate-distortion loss reductions (examples/train.py:68-82).
 * ======================================================================= */
/* The whole RD loss in two launches: out[3] = {loss, mse, bpp} with
 * bpp = bpp_coef * sum_k sum(log lik_k), mse = mean((x_hat - target)^2),
 * loss = lmbda * mse + bpp (fixed-order reductions).  Tensors are dense fp32
 * (likelihoods in any layout: the sums are order-independent per element). */
typedef struct cai_rd_inputs {
    const float* lik[4];
    int64_t lik_n[4];
    int32_t nlik;
    const float* x_hat;
    const float* target;
    int64_t n;
} cai_rd_inputs;
typedef struct cai_rd_grads {
    float* dlik[4];
} cai_rd_grads;
size_t cai_rd_loss_workspace_bytes(void);
int cai_rd_loss_fwd(const cai_rd_inputs* in, float lmbda, float bpp_coef, float* out, void* workspace,
                    size_t ws_bytes, void* stream);
/* one launch: dx_hat = (g_mse + lmbda g_loss) 2 (x_hat - target) / n, dlik_k = (g_bpp + g_loss) bpp_coef / lik_k;
 * the upstream gradients are device scalars (nullable = 0). */
int cai_rd_loss_bwd(const cai_rd_inputs* in, float lmbda, float bpp_coef, const float* g_loss, const float* g_mse,
                    const float* g_bpp, float* dx_hat, const cai_rd_grads* grads, void* stream);
/* out[0] += sum(log(lik)) over n elements (fp32, contiguous or strided by ld over C). */
int cai_sum_log(const float* lik, int64_t npix, int32_t C, int32_t ld, float* out, void* workspace,
                size_t ws_bytes, void* stream);
/* out[0] = sum((a-b)^2) over n contiguous fp32 elements */
int cai_sum_sqdiff(const float* a, const float* b, int64_t n, float* out, void* workspace,
                   size_t ws_bytes, void* stream);
size_t cai_reduce_workspace_bytes(int64_t n);
/* g[i] = (*scale) * coef / lik[i]  (bpp backward) */
int cai_log_bwd(const float* lik, int64_t npix, int32_t C, int32_t ld, const float* scale, float coef,
                float* g, void* stream);
/* ga[i] = (*scale) * coef * (a[i] - b[i])   (mse backward) */
int cai_sqdiff_bwd(const float* a, const float* b, int64_t n, const float* scale, float coef,
                   float* ga, void* stream);

/* =======================================================================
 * Optimiser over flat fp32 buffers (torch.optim.Adam semantics).
 * ======================================================================= */
/* state[0] = sum(g^2) (fp32); workspace >= cai_reduce_workspace_bytes(n) */
int cai_sqnorm(const float* g, int64_t n, float* out, void* workspace, size_t ws_bytes, void* stream);
/* One Adam step on n parameters; grads are first scaled by
 * min(1, max_norm / (sqrt(*sqnorm) + 1e-6)) when sqnorm != NULL (clip_grad_norm_;
 * max_norm = +inf: finiteness check only).  A non-finite *sqnorm skips the step
 * (parameters, moments and *step untouched), like GradScaler.step after
 * unscale_ found inf/NaN (examples/train.py:176-179).
 * *step (fp32, device) counts the steps taken. */
int cai_adam(float* p, const float* g, float* m, float* v, int64_t n,
             float lr, float beta1, float beta2, float eps,
             float* step, const float* sqnorm, float max_norm, void* stream);

/* The whole optimiser step of FusedAdam in as few launches as possible (2 for n > 65536, else 1):
 * flags CAI_ADAM_CLIP scales the grads by min(1, max_norm / (||g|| + 1e-6)) (clip_grad_norm_),
 * CAI_ADAM_SKIP_NONFINITE skips the step on a non-finite norm (either flag computes the norm; a
 * non-finite norm always skips, as cai_adam).  *sqnorm (nullable) receives sum(g^2).  Same update
 * and step counting as cai_sqnorm + cai_adam.  CAI_ADAM_ZERO_GRAD consumes the gradients: g is left
 * all zero (skipped step included), so the next backward needs no zero-fill (with n > 65536 it needs
 * CLIP or SKIP_NONFINITE).  Workspace >= cai_adam_step_workspace_bytes(n). */
#define CAI_ADAM_CLIP 1
#define CAI_ADAM_SKIP_NONFINITE 2
#define CAI_ADAM_ZERO_GRAD 4
size_t cai_adam_step_workspace_bytes(int64_t n);
int cai_adam_step(float* p, float* g, float* m, float* v, int64_t n,
                  float lr, float beta1, float beta2, float eps,
                  float* step, float* sqnorm, float max_norm, int32_t flags,
                  void* workspace, size_t ws_bytes, void* stream);

/* elementwise helpers */
int cai_act_bwd(int mask_mode, float param, const void* y, int32_t y_ld, const void* g, int32_t g_ld,
                void* out, int32_t out_ld, int64_t npix, int32_t C, int dtype, void* stream);
int cai_cast(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CAI_H */
