/*
 * expertsim_hip.h — C ABI of the MI355X (gfx950) kernels behind the expertsim GAN training step.
 *
 * The reference (patrick-bedkowski/Generative-DNN-for-Physics-Simulations-CERN) has no FFI: its
 * hot path is PyTorch ATen ops dispatched from Python.  This header is the boundary the build
 * puts underneath the reference's own Python API (expertsim.models.* forward signatures and
 * MoEWrapper.train_step); each entry point replaces the ATen ops named at it,
 * with the reference call site cited as file:line (paths relative to the reference root).
 *
 * Conventions
 *  - every pointer is a DEVICE pointer unless the comment says otherwise; kernels never allocate,
 *    free or synchronise; everything is enqueued on `stream` (a hipStream_t);
 *  - tensors are described logically as (n, c, h, w) with element strides s[4] — the device layout
 *    (NHWC for conv activations, [rows][features] for linear activations) is the caller's choice;
 *  - return 0 (ES_OK) or an error code; es_last_error() gives the message (thread-local);
 *  - dtypes: ES_F32 (fp32 parity mode) and ES_BF16 (bf16 operands, fp32 accumulation).
 */
#ifndef EXPERTSIM_HIP_H
#define EXPERTSIM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { ES_F32 = 0, ES_BF16 = 1 } es_dtype_t;
enum { ES_OK = 0, ES_ERR_ARG = 1, ES_ERR_HIP = 2, ES_ERR_UNSUPPORTED = 3 };
enum { ES_ACT_NONE = 0, ES_ACT_RELU = 1, ES_ACT_LRELU = 2 };
enum { ES_NORM_NONE = 0, ES_NORM_BN = 1, ES_NORM_GN = 2, ES_NORM_LN = 3 };

typedef void* es_stream_t; /* hipStream_t */

/* Logical 4-D view: element (n,c,h,w) lives at base + n*s[0] + c*s[1] + h*s[2] + w*s[3].
 * rows (optional, device int32): the LIVE batch count of a capacity-sized tensor.  A multi-expert
 * step keeps each expert's activations in buffers of n = capacity images and the expert's image
 * count on the device (es_expert_plan), so the step issues the same launches whatever the routing
 * (no host synchronisation, one captured graph): every kernel given a view / descriptor with rows
 * set works on images [0, min(rows[0], n)) only — images at or past it are neither read nor
 * written and take no part in any reduction (BatchNorm statistics, weight gradients, losses).
 * NULL: all n images (reference moe.py:121-207 runs each expert on exactly its B_e samples). */
typedef struct {
  int n, c, h, w;
  int64_t s[4];
  const int32_t* rows;
} es_view_t;

/* Counter-based dropout (expertsim/utils/philox.py).  keep(i) = (philox(seed, stream, i + index_offset)
 * >> 8) < threshold, i = NCHW-logical element index; kept values are multiplied by `scale` = 1/(1-p).
 * With step_ptr set, the stream used is stream + step_ptr[0] * step_mul, read on the device: a
 * captured HIP graph then draws fresh masks at every replay (the train step's step counter).
 * index_offset: logical index of this tensor's first element within the global batch (data-parallel
 * rank r holding samples [n0, n0 + n) of an expert's batch passes n0 * C*H*W), so every rank draws
 * exactly the single-device masks of its samples.  Must keep i + index_offset 4-aligned wherever i is
 * (a multiple of 8 for C % 8 == 0 layers). */
typedef struct {
  uint64_t seed;
  uint32_t stream;
  uint32_t threshold;
  float scale;
  int enabled;
  const int32_t* step_ptr; /* device int32 or NULL */
  int32_t step_mul;
  uint64_t index_offset;
  const int32_t* index_ptr; /* optional device int32: index_offset += index_ptr[0] * index_mul (a
                               data-parallel rank's first sample of the expert, known on the device) */
  int64_t index_mul;
} es_dropout_t;

const char* es_last_error(void);
int es_version(void);
int es_device_sync(void); /* hipDeviceSynchronize, for tests only */

/* ------------------------------------------------------------------------------------------
 * Convolution / linear as MFMA implicit GEMM.
 * Replaces aten::convolution / convolution_backward and aten::addmm / mm for nn.Conv2d and
 * nn.Linear (neutron/generator.py:11,17,24,29,33,37; neutron/discriminator.py:12,17,27,33,39;
 * neutron/aux_reg.py:13,20,27,34,45,68; proton/generator.py:14,19,27,33,38,41;
 * proton/discriminator.py:122,127,134,140,146; proton/aux_reg.py:20-30,61,104-117;
 * routers/router.py:12-19).  A Linear layer is the 1x1 convolution of a 1x1 image.
 * The nearest upsample feeding a generator conv (neutron/generator.py:23,29;
 * proton/generator.py:26,32) is folded into the input gather through hmap/wmap.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  int N, C, H, W;   /* conv input (before upsample): batch, in-channels, height, width      */
  int Hu, Wu;       /* conv input after nearest upsample (== H, W when hmap/wmap are NULL)   */
  int K, P, Q;      /* out-channels, output height, output width                             */
  int R, S;         /* kernel height, width                                                  */
  int stride, pad;
  const int32_t* hmap; /* device [Hu]: source row of upsampled row (torch nearest), or NULL  */
  const int32_t* wmap; /* device [Wu]                                                        */
  int up_h, up_w;      /* integer nearest-upsample factors (Hu = H*up_h), or 0 to use the maps.
                          With factors set, es_conv2d_dgrad folds the upsample backward: it
                          writes dx on the SOURCE grid (H x W) with dxs strides.               */
  int subpixel;        /* 1: the packed weights are the sub-pixel combination of a x2 upsample
                          conv (es_pack_conv_weight mode 2 for fwd, 3 for dgrad) and the conv runs
                          as 4 parity-class convs on the source grid (es_conv_subpixel_ok).      */
  const int32_t* rows; /* optional device int32: live images of the N-capacity batch (es_view_t) */
  int rows_px;         /* > 0: rows counts SAMPLES that are the P*Q == rows_px pixels of each image
                          (a linear over 16-sample pixel blocks, layers.ConvOp._pixel_view): image i
                          pixel p is live when i*rows_px + p < rows[0]                             */
} es_conv_desc_t;

/* y[n,k,p,q] = bias[k] + sum_{c,r,s} xu[n,c,p*stride-pad+r,q*stride-pad+s] * W[k,c,r,s]
 * wk: packed weights [K][R][S][C] of dtype dt (es_pack_conv_weight, mode 0). bias may be NULL. */
/* Select the bf16 FWD/DGRAD main loop: 1 = LDS-DMA staged kernel where eligible (default),
 * 0 = register-staged kernel.  Both accumulate in the same order (bit-identical results); the
 * switch exists for A/B measurement and tests.  Returns the previous setting. */
int es_conv_set_glds(int on);
/* Select the 8-wave LDS-DMA ring kernels (conv_mfma.hip) for the bf16 convs whose K-step is one tap
 * x 64 channels: 1 = on (default), 0 = use the 4-wave kernels.  Returns the previous setting. */
int es_conv_set_ring(int on);
/* 256 x 256 ring tiles with 32-deep K-steps for sub-pixel FWD and DGRAD with >= 256 output channels:
 * 1 = on (default), 0 = 256 x 128 tiles (same accumulation order: bit-identical results).
 * Returns the previous setting. */
int es_conv_set_ring256(int on);
/* Persistent short-K DGRAD kernel (conv_mfma.hip conv_persist_kernel: generator conv_layers.9's
 * dgrad, <= 8 K-steps of 64 channels, 64 or 128 output columns): 1 = on (default), 0 = the ring
 * kernel (same accumulation order: bit-identical outputs).  Returns the previous setting. */
int es_conv_set_persist(int on);
/* Persistent 256 x 256 kernel for the merged sub-pixel FWD (conv_mfma.hip conv_p256_kernel:
 * generator conv_layers.0 / .5): 1 = on (default), 0 = the per-tile ring kernel (same accumulation
 * order: bit-identical outputs).  Returns the previous setting. */
int es_conv_set_p256(int on);
/* Sub-pixel decomposition of stride-1 convs over a x2 nearest upsample (conv_mfma.hip): 1 = on
 * (default; wgrad uses it internally, fwd/dgrad when the caller packs mode 2/3 weights and sets
 * desc->subpixel), 0 = off.  Returns the previous setting. */
int es_conv_set_subpixel(int on);
/* 1 if es_conv2d_fwd / es_conv2d_dgrad can run this conv on the sub-pixel path (bf16, x2 integer
 * upsample, stride 1, channels % 64 == 0, tensors below 1 GiB, dense NHWC activations). */
int es_conv_subpixel_ok(const es_conv_desc_t* d, es_dtype_t dt);
/* Number of combined taps of the sub-pixel packing (16 for 3x3, 25 for 4x4): the packed weight
 * of mode 2 / 3 holds K * C * es_subpixel_taps(R, S) elements. */
int es_subpixel_taps(int R, int S);

int es_conv2d_fwd(const es_conv_desc_t* d, es_dtype_t dt, const void* x, const int64_t xs[4],
                  const void* wk, const float* bias, void* y, es_dtype_t ydt, const int64_t ys[4],
                  es_stream_t stream);
/* es_conv2d_fwd fused with the BatchNorm statistics of the stored y (torch batch_norm train mode,
 * neutron/generator.py:26,31,35): when the 8-wave ring kernel runs this conv, its epilogue also
 * writes per row tile and channel (count, mean, M2) partials to part [chunks][3][K] (part_floats
 * available) and *chunks > 0; es_norm_stats_finalize then merges them.  *chunks == 0 means y was
 * computed but no partials were written (use es_norm_stats). */
int es_conv2d_fwd_stats(const es_conv_desc_t* d, es_dtype_t dt, const void* x, const int64_t xs[4],
                        const void* wk, const float* bias, void* y, es_dtype_t ydt, const int64_t ys[4],
                        float* part, int64_t part_floats, int* chunks, es_stream_t stream);
/* dxu[n,c,hu,wu] = sum_{k,r,s} dy[n,k,p,q] * W[k,c,r,s] over (hu+pad-r) = p*stride, ...
 * (gradient w.r.t. the UPSAMPLED input; es_upsample_bwd folds it to the source grid).  With
 * integer factors d->up_h/up_w the fold happens inside the GEMM (K grows by up_h*up_w) and the
 * output is dx on the source grid.
 * wd: packed weights [C][R][S][K] (es_pack_conv_weight, mode 1).  beta=1 accumulates into dxu. */
int es_conv2d_dgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                    const void* wd, void* dxu, es_dtype_t dxdt, const int64_t dxs[4], float beta,
                    es_stream_t stream);
/* dw[k][r][s][c] += sum_{n,p,q} dy[n,k,p,q] * xu[n,c,...]   (fp32, split-K with atomics: the
 * caller zeroes dw first; es_unpack_conv_grad converts to torch's [K][C][R][S]). */
int es_conv2d_wgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                    const void* x, const int64_t xs[4], float* dw, es_stream_t stream);
/* Deterministic weight gradient (parity mode; replaces the same aten::convolution_backward weight
 * output as es_conv2d_wgrad): dw (torch layout [K][C][R][S], fp32) = beta * dw + dW, summed in a
 * fixed order.  The K splits store raw partials into ws (no float atomics), then one ordered reduce
 * (split, then sub-pixel class) writes dw; the result is bit-identical across runs and boxes.  fp32
 * ring shapes (channels % 64, dense NHWC) run the LDS-DMA ring kernel on v_mfma_f32_16x16x4_f32.
 * ws: es_conv2d_wgrad_det_ws_bytes(d, dt, ys, xs) bytes (-1: bad descriptor). */
int64_t es_conv2d_wgrad_det_ws_bytes(const es_conv_desc_t* d, es_dtype_t dt, const int64_t ys[4],
                                     const int64_t xs[4]);
int es_conv2d_wgrad_det(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                        const void* x, const int64_t xs[4], float* dw, float beta, void* ws, int64_t ws_bytes,
                        es_stream_t stream);
/* Deterministic split-K (parity mode) of es_conv2d_fwd / es_conv2d_dgrad (beta 0): when the GEMM
 * has few output tiles and a long K (the generators' fc2 dgrad, K = 21632 / 92160), the K splits
 * store partials into ws and one ordered sum writes y / dx (fp32, dense), instead of float
 * atomics.  ws: es_conv2d_splitk_ws_bytes(d, mode) bytes (mode 0 FWD, 1 DGRAD). */
int64_t es_conv2d_splitk_ws_bytes(const es_conv_desc_t* d, int mode);
int es_conv2d_fwd_det(const es_conv_desc_t* d, es_dtype_t dt, const void* x, const int64_t xs[4], const void* wk,
                      const float* bias, void* y, es_dtype_t ydt, const int64_t ys[4], void* ws, int64_t ws_bytes,
                      es_stream_t stream);
int es_conv2d_dgrad_det(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4], const void* wd,
                        void* dxu, es_dtype_t dxdt, const int64_t dxs[4], void* ws, int64_t ws_bytes,
                        es_stream_t stream);
/* split-fp32 WGRAD with 128-row tiles: 1 (default) the wave-specialised kernel (waves 0-3 MFMA only,
waves 4-7 load + split), 0 the cooperative kernel (every wave loads, splits and multiplies); the
two give bitwise equal weight gradients.  Returns the previous setting.  Replaces nothing in the
reference (a kernel choice for ATen convolution_backward's weight gradient). */
int es_conv_set_wgrad_ws(int on);
/* Deterministic mode on / off (returns the previous setting): fp32 FWD / DGRAD take no split-K
 * float atomics, the generic norm backward's conv-bias sums become an ordered column reduction.
 * MoEWrapper turns it on in the fp32 parity mode (train.deterministic, default on). */
int es_set_deterministic(int on);
/* Test knob: ring convolutions (fp32 and bf16) launch over chunks of at most `images` images (0: only
 * as the 1 GiB operand limit requires); returns the previous value. */
int es_conv_set_f32_chunk(int images);
/* fp32 MFMA arithmetic of the ring convolutions (returns the previous setting): 0 = exact fp32
 * (v_mfma_f32_16x16x4_f32), 1 = split-fp32: each fp32 operand is the exact sum of three bf16
 * planes and the six plane products with p + q <= 2 run on v_mfma_f32_16x16x32_bf16 into the fp32
 * accumulator (dropped terms < 2^-23 |a b| per product; deterministic, fixed order).  Replaces the
 * same fp32 conv2d / conv_transpose products as es_conv2d_fwd / _dgrad / _wgrad_det (neutron
 * generator.py:23-35, proton generator.py:26-38).  MoEWrapper sets it from train.fp32_mfma. */
int es_conv_set_f32_split(int on);
/* on = 2: as 1, and the FWD / DGRAD kernels read the packed weights' bf16 planes precomputed by
 * es_pack_weight_planes (the caller packs them whenever level 2 is set).
 * Byte offset of the planes behind an fp32 packing of n elements, and the planes themselves: each
 * 32-element block g of the packing -> 192 bytes at base + es_weight_planes_offset(n) + 192 g, three
 * planes of 32 bf16 (x0 = rne(x), x1 = rne(x - x0), x2 = x - x0 - x1), k-permuted as the ring
 * kernels' fragments.  Same weights as es_pack_conv_weight (neutron generator.py:24,29,33). */
int64_t es_weight_planes_offset(int64_t n);
int es_pack_weight_planes(const float* packed, int64_t n, void* base, es_stream_t stream);
/* Host-side count of MFMA conv kernels issued so far (ring / persistent / p256 / fp32 WGRAD).
 * Instrumentation only: lets a profiler state how many kernel launches one conv op was. */
int64_t es_conv_launch_count(void);
/* Host-side tally of the MFMA work the conv entry points (es_conv2d_fwd / _dgrad / _wgrad /
 * _wgrad_det and their _stats / _bnred / _det variants) issued, as executed FLOPs (2 per MAC):
 * out[0] on the bf16 pipe (bf16 operands, and split-fp32: 6 plane products per fp32 product),
 * out[1] on the fp32 MFMA (v_mfma_f32_16x16x4_f32), out[2] on the VALU (thin Cin/Cout = 1 convs).
 * A sub-pixel conv counts its 4 parity-class convs (es_subpixel_taps / (4 R S) of the reference's
 * MACs).  reset != 0 zeroes the tally after reading it.  Instrumentation only (bench.py's executed
 * step MFMA fraction); the same products as neutron generator.py:23-35 / proton generator.py:26-38. */
int es_conv_exec_flops(double out[3], int reset);

/* Weight packing for the implicit GEMM (fp32 master [K][C][R][S] -> dt).
 * mode 0: out[k][r][s][c] = w*scale ; mode 1: out[c][r][s][k] = w*scale.
 * mode 2 / 3 (sub-pixel, x2 upsample): for each parity class t = 2a + b the combined weights
 * W'_t[d][e] = sum of w[.][.][r][s] over r in {2d-a, 2d-a+1}, s in {2e-b, 2e-b+1} (within range),
 * d < ((a+R-1)>>1)+1, e < ((b+S-1)>>1)+1; mode 2: class blocks [K][d][e][C] one after another,
 * mode 3: out[c][tap][k] with tap = the classes' (d, e) taps in order.  col_perm must be NULL.
 * scale = (inv_scale ? 1/inv_scale[0] : 1)  — the spectral-norm division W/sigma
 * (torch.nn.utils.spectral_norm compute_weight) is folded here.
 * col_perm (optional, device [C*R*S] for R=S=1 linears): input column index permutation. */
int es_pack_conv_weight(const float* w, int K, int C, int R, int S, int mode,
                        const float* inv_scale, const int32_t* col_perm, void* out, es_dtype_t dt,
                        es_stream_t stream);
/* One weight packing of es_pack_conv_weight (scale 1, no column permutation), with the split-fp32
 * planes behind it when planes != 0 (es_pack_weight_planes); out is the packing's buffer. */
typedef struct {
  const float* w;
  int K, C, R, S, mode;
  int dt;     /* es_dtype_t of the packing */
  int planes; /* fp32 only: also write the bf16 planes at out + es_weight_planes_offset(n) */
  void* out;
} es_pack_job_t;
/* The packings of every layer of a module rebuilt after a weight update (MoE optimizer steps) in one
 * launch per 32 jobs instead of one or two per layout (jobs: host array).  Same values as
 * es_pack_conv_weight + es_pack_weight_planes per job; the large mode-1 transposes keep their
 * LDS-tiled kernel. */
int es_pack_conv_weights(const es_pack_job_t* jobs, int n, es_stream_t stream);
/* grad[k][c][r][s] = beta*grad + dw[k][r][s][c] * (inv_scale ? 1/inv_scale[0] : 1) */
int es_unpack_conv_grad(const float* dw, int K, int C, int R, int S, const int32_t* col_perm,
                        float* grad, float beta, es_stream_t stream);
/* as es_unpack_conv_grad (no permutation), then dw[] = 0: a persistent packed accumulator needs no
 * zero fill before the next es_conv2d_wgrad */
int es_unpack_conv_grad_clear(float* dw, int K, int C, int R, int S, float* grad, float beta,
                              es_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Normalisation + dropout + activation (aten::native_batch_norm / native_group_norm /
 * native_layer_norm, aten::bernoulli_ + mul (nn.Dropout), leaky_relu / relu and their
 * backward).  One fused elementwise pass forward, reductions + one pass backward.
 * Stats groups: BN -> channel c (count N*H*W), GN -> (n, c / (C/groups)), LN -> n (count C*H*W).
 * gamma/beta index: BN/GN -> c; LN -> (c*H + h)*W + w.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  int kind;            /* ES_NORM_*                                                       */
  int groups;          /* GN only                                                         */
  const float* mean;   /* per stats group                                                 */
  const float* invstd; /* per stats group                                                 */
  const float* gamma;  /* may be NULL (identity)                                          */
  const float* beta;   /* may be NULL                                                     */
} es_norm_t;

typedef struct {
  es_dropout_t drop;
  int dropout_first; /* 1: act(drop(norm(x)))  [generator.py:13-15]; 0: drop(act(norm(x))) [aux_reg.py:15-17] */
  int act;           /* ES_ACT_*                                                          */
  float slope;       /* LeakyReLU negative slope (0.1 everywhere in the reference)        */
  uint8_t* keep;     /* optional device dropout keep bits, layout [n*h*w][c/8] (bit c%8 of byte
                        (row, c/8)), c % 8 == 0 required: es_norm_act_fwd writes the mask it draws,
                        es_norm_act_bwd then reads it instead of re-running Philox (same mask)   */
  int keep_ready;    /* 1: keep already holds this chain's mask (es_dropout_keep_bits, e.g. drawn on a
                        side stream ahead of the forward): es_norm_act_fwd reads it instead of
                        drawing it                                                                */
} es_chain_t;

/* Batch statistics of x (train-mode BN / GN / LN), written to mean/invstd per stats group.
 * For BN, running_mean/var (may be NULL) are updated with `momentum` and the unbiased
 * variance, as torch does.  ws: workspace of es_norm_stats_ws_bytes() bytes. */
int64_t es_norm_stats_ws_bytes(const es_view_t* x, int kind, int groups);
int es_norm_stats(const es_view_t* x, es_dtype_t xdt, const void* xp, int kind, int groups,
                  float eps, float* mean, float* invstd, float* running_mean, float* running_var,
                  float momentum, void* ws, es_stream_t stream);
/* y = chain(norm(x) [+ addend]) ; addend may be NULL (residual add of proton/aux_reg.py:130) */
/* Merge BatchNorm partials [chunks][3][C] (count, mean, M2; es_conv2d_fwd_stats) into mean /
 * invstd and the running statistics (momentum, unbiased variance), as es_norm_stats does. */
int es_norm_stats_finalize(const float* part, int chunks, int C, float eps, float* mean, float* invstd,
                           float* running_mean, float* running_var, float momentum, es_stream_t stream);
int es_norm_act_fwd(const es_view_t* x, es_dtype_t xdt, const es_norm_t* nm, const es_chain_t* ch,
                    const es_view_t* addend, es_dtype_t adt, const void* addend_ptr, const void* xp,
                    const es_view_t* y, es_dtype_t ydt, void* yp, es_stream_t stream);
/* Backward of es_norm_act_fwd.  dy: gradient of y.  act_ref (optional): evaluate the activation
 * derivative on this stored tensor (the block output) instead of the recomputed pre-activation.
 * Writes dx (beta=1 accumulates), accumulates dgamma/dbeta (fp32, may be NULL) and, when dsum is
 * given (C <= 1024), the per-channel sum of dx (the gradient of a conv bias feeding the norm). */
int64_t es_norm_bwd_ws_bytes(const es_view_t* x, int kind, int groups);
int es_norm_act_bwd(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_norm_t* nm,
                    const es_chain_t* ch, const es_view_t* dy, es_dtype_t dydt, const void* dyp,
                    const es_view_t* act_ref, es_dtype_t rdt, const void* refp,
                    const es_view_t* dx, es_dtype_t dxdt, void* dxp, float beta, float* dgamma,
                    float* dbeta, float* dsum, void* ws, es_stream_t stream);
/* es_conv2d_dgrad (beta 0) fused with the REDUCTION pass of the BatchNorm backward that consumes dx
 * (aten::native_batch_norm_backward's sums, neutron/generator.py:30-33: conv_layers.9's dgrad feeds
 * BatchNorm2d conv_layers.6 -> Dropout -> LeakyReLU): x = that norm's input (dx's layout), nm its
 * statistics, ch its dropout / activation chain with the forward's keep bits.  When the
 * persistent DGRAD kernel runs this conv, its epilogue writes per workgroup the sums of dnorm and
 * dnorm * xhat over the stored dx to part [chunks][3][C] (slots 1, 2; part_floats available) and
 * *chunks > 0 (then es_norm_act_bwd_sums finishes the backward); *chunks == 0: dx was computed
 * but no sums were written (use es_norm_act_bwd). */
int es_conv2d_dgrad_bnred(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                          const void* wd, void* dx, es_dtype_t dxdt, const int64_t dxs[4], const void* x,
                          const es_norm_t* nm, const es_chain_t* ch, float* part, int64_t part_floats,
                          int* chunks, es_stream_t stream);

/* Rest of the BatchNorm backward after es_conv2d_dgrad_bnred produced its reduction sums
 * (sums_part [chunks][3][C], slots 1, 2): the finalize (a1, a2, dgamma += , dbeta +=) and the
 * apply pass of es_norm_act_bwd (dx, and dsum += sum(dx) per channel when dsum != NULL).  BN only,
 * dense NHWC x / dy / dx of one dtype; ws: es_norm_bwd_ws_bytes(x, BN, 1) bytes. */
int es_norm_act_bwd_sums(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_norm_t* nm,
                         const es_chain_t* ch, const es_view_t* dy, es_dtype_t dydt, const void* dyp,
                         const es_view_t* dx, es_dtype_t dxdt, void* dxp, const float* sums_part, int chunks,
                         float* dgamma, float* dbeta, float* dsum, void* ws, es_stream_t stream);


/* Data-parallel (synchronised) BatchNorm: the batch statistics of the neutron generator's and aux
 * regressor's BatchNorms (neutron/generator.py:13,19,26,31,35; neutron/aux_reg.py:15-47) over the
 * GLOBAL batch, as one device computes them for the reference.
 *   es_norm_stats_merge: [chunks][3][C] (count, mean, M2) partials -> one [3][C] partial;
 *   es_norm_stats_local: the rank's [3][C] partial straight from x (ws: es_norm_stats_ws_bytes);
 * the caller all-gathers the ranks' [3][C] partials and finalizes them with es_norm_stats_finalize
 * (world partials -> mean / invstd / running stats).
 *   es_norm_bwd_sync phase 0: raw per-channel sums [2][C] (sum dnorm, sum dnorm*xhat) of the rank
 *   into `sums`, and the rank's dgamma / dbeta accumulation; the caller all-reduces `sums`;
 *   phase 1: dx from the global sums and the global row count `cnt` (+ dsum as es_norm_act_bwd);
 *   with cnt_mul (device float, dynamic rows) the count is cnt_mul[0] * cnt (cnt: per sample).
 * ws: es_norm_bwd_ws_bytes(x, ES_NORM_BN, 1). */
int es_norm_stats_merge(const float* part, int chunks, int C, float* out, es_stream_t stream);
int es_norm_stats_local(const es_view_t* x, es_dtype_t xdt, const void* xp, void* ws, float* out,
                        es_stream_t stream);
int es_norm_bwd_sync(int phase, const es_view_t* x, es_dtype_t xdt, const void* xp, const es_norm_t* nm,
                     const es_chain_t* ch, const es_view_t* dy, es_dtype_t dydt, const void* dyp,
                     const es_view_t* dx, es_dtype_t dxdt, void* dxp, float* sums, float cnt,
                     const float* cnt_mul, float* dgamma, float* dbeta, float* dsum, void* ws,
                     es_stream_t stream);

/* Plain elementwise chain without normalisation (router LeakyReLU, final ReLU, casts):
 * y = chain(x). And its backward dx = beta*dx + dchain(dy) evaluated at x (or act_ref). */
/* Draw the dropout keep bits of chain ch over x's geometry (n, c, h, w; dynamic rows: the live
 * samples of x->rows) into ch->keep -- the mask es_norm_act_fwd would draw for the same chain.  A
 * forward given the chain with keep_ready = 1 then reads them (reference: the nn.Dropout masks of
 * neutron/generator.py:13-36, drawn ahead of their layer; bit-identical to the in-pass draw). */
int es_dropout_keep_bits(const es_view_t* x, const es_chain_t* ch, es_stream_t stream);
int es_act_fwd(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_chain_t* ch,
               const es_view_t* y, es_dtype_t ydt, void* yp, es_stream_t stream);

/* Per-channel sum over (n,h,w): out[c] = beta*out[c] + sum x (conv/linear bias gradients). */
int64_t es_channel_sum_ws_bytes(const es_view_t* x);
int es_channel_sum(const es_view_t* x, es_dtype_t xdt, const void* xp, float* out, float beta,
                   void* ws, es_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Pooling / resampling / layout (aten::max_pool2d_with_indices(+_backward),
 * upsample_nearest2d_backward, adaptive_avg_pool2d, cat, copy_)
 * ---------------------------------------------------------------------------------------- */
/* max pool, kernel (kh,kw), stride (sh,sw), no padding, floor mode; idx: uint8 window argmax
 * (first max in row-major window order, as torch). */
int es_maxpool_fwd(const es_view_t* x, es_dtype_t dt, const void* xp, int kh, int kw, int sh, int sw,
                   const es_view_t* y, void* yp, uint8_t* idx, es_stream_t stream);
int es_maxpool_bwd(const es_view_t* dy, es_dtype_t dt, const void* dyp, const uint8_t* idx, int kh,
                   int kw, int sh, int sw, const es_view_t* dx, void* dxp, float beta,
                   es_stream_t stream);
/* Fused discriminator front (neutron/discriminator.py:11-15, proton/discriminator.py:121-125):
 * SNconv3x3 1->32 (+bias, weight w * 1/sigma[0]) -> GroupNorm(8, 32) -> LeakyReLU(slope) ->
 * MaxPool 2x2, one workgroup per image, the 32-channel conv map recomputed from the image in LDS
 * instead of stored.  img: fp32 [N][1][H][W] (element strides is[4]); H-2 and W-2 even,
 * H*W <= 2048.  Forward writes pooled [N][(H-2)/2][(W-2)/2][32] fp32 (dense NHWC), idx (same
 * shape, uint8 window argmax as es_maxpool_fwd) and the GN mean / invstd [N][8]. */
int es_dfront_fwd(const float* img, const int64_t is[4], int N, int H, int W, const float* w,
                  const float* sigma, const float* bias, const float* gamma, const float* beta, float eps,
                  float slope, float* mean, float* invstd, float* pooled, uint8_t* idx, es_stream_t stream);
/* Backward from dpooled (dense NHWC like pooled).  dx (optional, fp32 [N][1][H][W], strides dxs):
 * image gradient, written.  part: workspace of es_dfront_part_floats(N) floats.  dw (gradient of
 * W/sigma, [32][1][3][3]) is written; dbias / dgamma / dbeta are accumulated; each may be NULL. */
int64_t es_dfront_part_floats(int N);
int es_dfront_bwd(const float* img, const int64_t is[4], int N, int H, int W, const float* w,
                  const float* sigma, const float* bias, const float* gamma, const float* beta, float eps,
                  float slope, const float* mean, const float* invstd, const uint8_t* idx,
                  const float* dpooled, float* dx, const int64_t dxs[4], float* part, float* dw,
                  float* dbias, float* dgamma, float* dbeta, es_stream_t stream);
/* Fused discriminator front, both conv blocks (neutron/discriminator.py:11-24,
 * proton/discriminator.py:121-134): SNconv3x3 1->32 -> GroupNorm(8, 32) -> LeakyReLU -> MaxPool 2x2
 * -> SNconv3x3 32->16 -> GroupNorm(8, 16) -> LeakyReLU -> MaxPool (ph, pw) -> flatten (NCHW order),
 * one workgroup per image: the pooled 32-channel map and the 16-channel conv map stay in LDS (the
 * second conv on v_mfma_f32_16x16x4_f32), only the flattened features leave the chip.  Replaces
 * es_dfront_* + es_conv2d_fwd/dgrad/wgrad of conv_layers.4 + the GroupNorm / pool passes after it.
 * Weights are used as w * (1/sigma[0]) (sigma may be NULL: 1). */
typedef struct {
    const float* w1; const float* sigma1; const float* b1; const float* g1; const float* be1;  /* [32][1][3][3], GN(8,32) */
    const float* w2; const float* sigma2; const float* b2; const float* g2; const float* be2;  /* [16][32][3][3], GN(8,16) */
    float eps1, eps2, slope;
    int ph, pw;                       /* second pool window = stride (neutron 2x2, proton 2x1) */
    const int32_t* rows;              /* optional device int32: live images of the N-image capacity */
} es_dfront2_params_t;
/* 1 when the fused path supports this geometry (H*W <= 2048, H-2 and W-2 even, pooled map <= 448
 * pixels, second conv map <= 368 pixels) */
int es_dfront2_ok(int H, int W, int ph, int pw);
/* Forward.  img fp32 [N][1][H][W] (strides is).  Writes feat[n*feat_stride + f], f < 16*Hq*Wq
 * (the reference's view(B, -1) order) and stats [N][32] = GN1 mean[8], invstd[8], GN2 mean[8],
 * invstd[8].  save (optional; required by the backward): [N][es_dfront2_save_floats] floats of
 * per-image activations the backward reads instead of recomputing them. */
int64_t es_dfront2_save_floats(int H, int W, int ph, int pw);
int es_dfront2_fwd(const float* img, const int64_t is[4], int N, int H, int W, const es_dfront2_params_t* p,
                   float* stats, float* feat, int64_t feat_stride, float* save, es_stream_t stream);
/* Backward from dfeat (the gradient of the features, same indexing as feat), with the forward's
 * stats and save.  dx (optional): fp32 image gradient [N][1][H][W] (strides dxs), written.  part
 * (optional, es_dfront2_part_floats(N) floats): per-image weight-gradient partials; when given,
 * dw1 / dw2 (gradients of W/sigma, torch layouts) are written and db*, dg*, dbe* (biases, GN
 * affines) accumulated; each may be NULL. */
int64_t es_dfront2_part_floats(int N);
int es_dfront2_bwd(const float* img, const int64_t is[4], int N, int H, int W, const es_dfront2_params_t* p,
                   const float* stats, const float* save, const float* dfeat, int64_t dfeat_stride, float* dx,
                   const int64_t dxs[4],
                   float* part, float* dw1, float* db1, float* dg1, float* dbe1, float* dw2, float* db2,
                   float* dg2, float* dbe2, es_stream_t stream);
/* Fused fc tail of the spectral-norm discriminator (neutron/discriminator.py:26-48,
 * proton/discriminator.py:136-158): SNLinear F->128 -> LayerNorm(128) -> LeakyReLU -> SNLinear
 * 128->64 -> LayerNorm(64) -> LeakyReLU (latent) -> SNLinear 64->1, 16 samples per workgroup, fp32
 * (v_mfma_f32_16x16x4_f32), weights used as w * (1/sigma[0]) (sigma may be NULL: 1).  Replaces the
 * es_conv2d_* / es_norm_* / es_pack_conv_weight launches of those layers. */
typedef struct {
    const float* w1; const float* sigma1; const float* b1; const float* g1; const float* be1;  /* [128][F], LN(128) */
    const float* w2; const float* sigma2; const float* b2; const float* g2; const float* be2;  /* [64][128], LN(64) */
    const float* w3; const float* sigma3; const float* b3;                                    /* [1][64] */
    float eps1, eps2, slope;
    const int32_t* rows;   /* optional device int32: live samples of the B-sample capacity */
} es_dmlp_params_t;
/* Forward over X [B][F] (row stride xs): writes h3 [B][128] (fc1 output), s3 [B][2] (LN1 mean,
 * invstd), h4 [B][64], s4 [B][2], lat [B][64] (the latent) and out [B] (the logit). */
int es_dmlp_fwd(const float* X, int64_t xs, int B, int F, const es_dmlp_params_t* p, float* h3, float* s3,
                float* h4, float* s4, float* lat, float* out, es_stream_t stream);
/* Backward from dout [B] and / or dlat [B][64] (either may be NULL) with the forward's saved
 * values.  dX (optional, row stride dxs): the fc1 input gradient, written.  part (optional,
 * es_dmlp_part_floats(B, F) floats): per-workgroup partials; when given, dw1 / dw2 / dw3 (gradients
 * of W/sigma, torch layouts) are written and the bias / LayerNorm-affine gradients accumulated;
 * any output may be NULL. */
int64_t es_dmlp_part_floats(int B, int F);
int es_dmlp_bwd(const float* X, int64_t xs, int B, int F, const es_dmlp_params_t* p, const float* h3,
                const float* s3, const float* h4, const float* s4, const float* lat, const float* dout,
                const float* dlat, float* dX, int64_t dxs, float* part, float* dw1, float* db1, float* dg1,
                float* dbe1, float* dw2, float* db2, float* dg2, float* dbe2, float* dw3, float* db3,
                es_stream_t stream);
/* Nearest resize gather y[n, :, hu, wu] = x[n, :, hmap[hu], wmap[wu]] (torch upsample_nearest2d's index
 * maps; dense NHWC, C % 4 == 0 fp32 / % 8 bf16): the proton generator's 35x19 -> 56x30 resize feeding
 * conv_layers.5 (proton/generator.py:33-34), materialised so that the conv runs on the ring kernels. */
int es_upsample_fwd(const es_view_t* x, es_dtype_t dt, const void* xp, const int32_t* hmap, const int32_t* wmap,
                    const es_view_t* y, void* yp, es_stream_t stream);
/* dx[n,c,h,w] = beta*dx + sum over upsampled positions mapping to (h,w).  hstart/hcount (device
 * [H]) and wstart/wcount (device [W]) describe the contiguous preimage of each source row/col.
 * Dense NHWC views with C % 4 == 0 take a vectorised kernel. */
int es_upsample_bwd(const es_view_t* dxu, es_dtype_t dt, const void* dxup, const int32_t* hstart,
                    const int32_t* hcount, const int32_t* wstart, const int32_t* wcount,
                    const es_view_t* dx, es_dtype_t dxdt, void* dxp, float beta, es_stream_t stream);
/* y = alpha*x (+ beta*y) elementwise between any two views of equal logical shape (also casts) */
int es_copy(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_view_t* y, es_dtype_t ydt,
            void* yp, float alpha, float beta, es_stream_t stream);
/* global average pool over (h,w): y[n,c] (view (N,C,1,1)) and its backward */
int es_avgpool_fwd(const es_view_t* x, es_dtype_t dt, const void* xp, const es_view_t* y, void* yp,
                   es_stream_t stream);
int es_avgpool_bwd(const es_view_t* dy, const void* dyp, const es_view_t* dx, es_dtype_t dxdt,
                   void* dxp, float beta, es_stream_t stream);
/* rows gathered by index: dst[i,:] = src[idx[i],:] (fp32 rows of `cols`); idx NULL = identity */
int es_gather_rows(const float* src, int64_t src_ld, const int32_t* idx, int rows, int cols,
                   float* dst, int64_t dst_ld, es_stream_t stream);
/* Same with idx = perm + start[0], start read on the device (es_router_dispatch's offsets): the
 * per-expert gather of a multi-expert step (moe.py:121-143).  live (optional, device int32): only the
 * first live[0] of the `rows` (capacity) rows are gathered, the rest are written as zeros. */
int es_gather_rows_at(const float* src, int64_t src_ld, const int32_t* perm, const int32_t* start, int rows,
                      int cols, float* dst, int64_t dst_ld, const int32_t* live, es_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Spectral norm (torch.nn.utils.spectral_norm, n_power_iterations=1, eps=1e-12) for every
 * discriminator layer (neutron/discriminator.py:12,17,27,33,39; proton/discriminator.py:122,
 * 127,134,140,146).  One power iteration updates u,v in place and writes sigma = u.(W v).
 * sigma points to 1 + 2*(h + wd) floats: sigma[0], scratch, then a snapshot of the u [h] and
 * v [wd] this call used (what es_sn_bwd needs once the next call has updated u, v in place).
 * ---------------------------------------------------------------------------------------- */
/* active (optional, device int32): with active[0] == 0 the call computes sigma from the stored u, v
 * and updates nothing (an expert that does not train this step, moe.py:126-135). */
int es_sn_power_iter(const float* w, int h, int wd, float* u, float* v, float* sigma, int update,
                     const int32_t* active, es_stream_t stream);
/* es_sn_power_iter for n <= ES_SN_BATCH_MAX small layers (h*wd < 16384 each) in ONE launch; the
 * arrays are host arrays of device pointers / sizes, buf[i] as es_sn_power_iter's sigma buffer. */
#define ES_SN_BATCH_MAX 8
int es_sn_power_iter_batch(int n, const float* const* w, const int* h, const int* wd, float* const* u,
                           float* const* v, float* const* buf, int update, const int32_t* active,
                           es_stream_t stream);
/* es_sn_bwd for n <= ES_SN_BATCH_MAX small layers in ONE launch (host arrays of device pointers). */
int es_sn_bwd_batch(int n, const float* const* w, const float* const* g, const int* h, const int* wd,
                    const float* const* u, const float* const* v, const float* const* sigma, float* const* dw,
                    float beta, es_stream_t stream);
/* dW_orig = beta*dW_orig + G/sigma - (<G, W>/sigma^2) u v^T   (G = grad of W/sigma).
 * sigma is the buffer es_sn_power_iter wrote (1 + h + wd floats); its tail is used as scratch. */
int es_sn_bwd(const float* w, const float* g, int h, int wd, const float* u, const float* v,
              const float* sigma, float* dw_orig, float beta, es_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Losses (moe.py:506-642, proton/aux_reg.py:42-45, train/utils.py:623-642) and their gradients.
 * ---------------------------------------------------------------------------------------- */
/* Discriminator hinge (moe.py:518-523): out[0] = w*(mean relu(1-ro) + mean relu(1+fo));
 * dro/dfo = gradients of out[0].  w is read from device memory (w_ptr[0]) to avoid host syncs.
 * rows (optional, device int32): the live count of the n-capacity batch (0: out[0] = 0). */
int es_hinge_d(const float* ro, const float* fo, int n, const int32_t* rows, const float* w_ptr, float* out,
               float* dro, float* dfo, es_stream_t stream);
/* per-sample photon sum s[b] = sum_{h,w} (exp(x)-1) of the generated image (moe.py:611-616) */
int es_image_expsum(const es_view_t* x, es_dtype_t dt, const void* xp, float* s, es_stream_t stream);
/* Generator-step losses (moe.py:544-563): gen hinge, SDI diversity, intensity L1, log-cosh aux,
 * weighted by w.  Writes out[0..7] = {total, gen_hinge, div, intensity, aux, std_int, mean_int, w}
 * and gradients: dfo[n], dl1/dl2 [n,L], dcoord [n,2], coef[n] (= d total / d s[b]). */
typedef struct {
  int n, latent, noise;
  float di_strength, in_strength, aux_strength;
  const float* std_mean; /* optional device scalar: mean(std) over the expert's GLOBAL batch (data
                            parallel, SDI prefactor); NULL: the mean over these n samples */
  const int32_t* rows;   /* optional device int32: live samples of the n-capacity batch (0: metrics 0) */
} es_gen_loss_t;
int es_gen_losses(const es_gen_loss_t* p, const float* fo, const float* l1, const float* l2,
                  const float* n1, const float* n2, const float* std_, const float* s,
                  const float* intensity, const float* coord, const float* pos, const float* w_ptr,
                  float* out, float* dfo, float* dl1, float* dl2, float* dcoord, float* coef,
                  es_stream_t stream);
/* dimg[b,..] = beta*dimg + coef[b]*exp(x)   (intensity-term gradient of the generated image) */
int es_image_expsum_bwd(const es_view_t* x, es_dtype_t dt, const void* xp, const float* coef,
                        const es_view_t* dx, void* dxp, float beta, es_stream_t stream);

/* Router tail (routers/router.py:23 gumbel_softmax, moe.py:97-103 argmax/bincount):
 * gates = softmax((logits - log(e))/tau); idx = argmax; counts[E] (int32) */
int es_router_gumbel(const float* logits, const float* expo, int B, int E, float tau, float* gates,
                     int32_t* idx, int32_t* counts, es_stream_t stream);
/* Router loss gradient w.r.t. logits for the ALB term (train/utils.py:623-642, moe.py:407,429)
 * and the loss value: out[0] = coef*mean_e exp(1/(S_e+1e-6)), S_e = sum_b gates[b,e]. */
int es_router_alb(const float* gates, int B, int E, float tau, float coef, float* out,
                  float* dlogits, es_stream_t stream);
/* All router-loss terms that carry gradient (moe.py:258-268,407-434; train/utils.py:372-395
 * calculate_expert_distribution_loss, 398-419 calculate_expert_utilization_entropy, 623-642 ALB):
 * out[0] = alb_coef*mean_e exp(1/(S_e+1e-6)); out[1] = util*sum_e avg_e*log(avg_e+1e-9)
 * (= -entropy*util, avg = S/B_total); out[2] = 0.1*ed/B_total*sum_{a,b: idx_a=idx_b} |feat_a - feat_b|
 * (cdist of the [B,1] per-sample photon sums, gated by the straight-through one-hot gates);
 * dlogits = d(sum of the three)/d logits through the Gumbel softmax, for the B rows of `gates`.
 * Data parallel: colsum = the all-reduced S_e (NULL: this call's rows), B_total = the global batch
 * (<= 0: B), feat_all / idx_all [B_all] = the all-gathered ED features (NULL: this call's rows); out
 * then holds this rank's share of the ED sum.  feat / idx may be NULL when ed_strength == 0. */
int es_router_loss(const float* gates, const int32_t* idx, const float* feat, int B, int E, float tau,
                   float alb_coef, float util_strength, float ed_strength, const float* colsum, int B_total,
                   const float* feat_all, const int32_t* idx_all, int B_all, float* out, float* dlogits,
                   es_stream_t stream);
/* Device-side expert dispatch (moe.py:121-123 `(idx == i).nonzero()` per expert, without the host
 * round trip): perm[B] = the batch rows grouped by expert, each group in batch order;
 * offs[E+1] = start of each group (offs[E] = B). */
int es_router_dispatch(const int32_t* idx, int B, int E, int32_t* perm, int32_t* offs, es_stream_t stream);
/* out[e] = sum_b gates[b, e] (the rank's share of the router's gate sums). */
int es_router_colsum(const float* gates, int B, int E, float* out, es_stream_t stream);
/* The train step's metric dict (moe.py:480-502) in one launch: out[11 + 8E] = gen, disc, div,
 * intensity, aux (means over the experts of mbuf [E][9] = per expert total, gen, div, int, aux,
 * std_int, mean_int, w, disc), router, ED, differentiation, entropy, ALB, gan (moe.py:255-434 from
 * rl = [ALB*dec_w, entropy, ED]), then per expert gen_i, disc_i, div_i, int_i, aux_i, std_int_i,
 * mean_int_i, n_i (counts int32 or countsf float).  flags: 1 router (E > 1), 2 router trained this
 * epoch, 4 ALB on, 8 entropy on, 16 ED on. */
int es_step_metrics(const float* mbuf, int E, const float* rl, const int32_t* counts, const float* countsf,
                    float gan_strength, float diff_strength, float dec_w, int flags, float* out,
                    es_stream_t stream);
/* Data-parallel merge of the per-expert metric rows: rows [world][E][10] (the 9 metric columns of
 * MoEWrapper's buffer + the rank's sample count, 0 = not run) -> out [E][9], global-batch values. */
int es_dp_metrics_merge(const float* rows, int world, int E, float* out, es_stream_t stream);
/* dst[rows[i]] = src[i] for i < n (rows NULL: identity) -- moe.py:196-198 scatter of the
 * per-sample photon sums into the batch-ordered ED features. */
int es_scatter_rows(const float* src, const int32_t* rows, int n, float* dst, es_stream_t stream);
/* Same with the rows read from a dispatch permutation at a DEVICE start position (perm + start[0]),
 * so a captured per-expert graph stays valid whatever the expert's offset in a later step. */
int es_scatter_rows_at(const float* src, const int32_t* perm, const int32_t* start, int n, const int32_t* live,
                       float* dst, es_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Optimizer (torch.optim.Adam, created at train/training_setup.py:20-40, stepped at
 * moe.py:439,526,565,566): one launch over a flat fp32 parameter buffer.
 * ---------------------------------------------------------------------------------------- */
int es_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
            float beta2, float eps, int step, float grad_scale, es_stream_t stream);
/* Same update with the (1-based) step read on the device from step_ptr[0]; bias corrections
 * computed in the kernel (for captured train steps).  active (optional, device int32): no update when
 * active[0] == 0 (an expert skipped this step, moe.py:126-135). */
int es_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                float beta2, float eps, const int32_t* step_ptr, float grad_scale, const int32_t* active,
                es_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Random numbers (torch.randn at moe.py:144,535; exponential_ inside F.gumbel_softmax):
 * Philox4x32-10 + Box-Muller, counter = element index.
 * ---------------------------------------------------------------------------------------- */
int es_randn(float* out, int64_t n, uint64_t seed, uint32_t stream_id, es_stream_t stream);
int es_rand_exponential(float* out, int64_t n, uint64_t seed, uint32_t stream_id,
                        es_stream_t stream);
/* Same draws with the stream id offset on the device: stream_id + step_ptr[0] * step_mul, and the
 * element counter starting at `offset` (out[i] = draw number offset + i; randn: offset even), so a
 * data-parallel rank draws exactly its rows of the single-device draw. */
int es_randn_dev(float* out, int64_t n, uint64_t seed, uint32_t stream_id, const int32_t* step_ptr,
                 int32_t step_mul, int64_t offset, es_stream_t stream);
int es_rand_exponential_dev(float* out, int64_t n, uint64_t seed, uint32_t stream_id,
                            const int32_t* step_ptr, int32_t step_mul, int64_t offset, es_stream_t stream);
/* es_randn_dev whose element offset adds off_ptr[0] * off_mul on the device (a data-parallel rank's
 * first sample of an expert, es_expert_plan n0; offsets even). */
int es_randn_dev_at(float* out, int64_t n, uint64_t seed, uint32_t stream_id, const int32_t* step_ptr,
                    int32_t step_mul, int64_t offset, const int32_t* off_ptr, int64_t off_mul, es_stream_t stream);
/* counter[0] += v on the device (step counters of a captured train step); the _if forms only when
 * flag[0] != 0 (flag NULL: always) -- an expert's optimizer steps and BatchNorm num_batches_tracked
 * counters advance only when it trains (moe.py:126-135). */
int es_counter_add(int32_t* counter, int32_t v, es_stream_t stream);
int es_counter_add_if(int32_t* counter, int32_t v, const int32_t* flag, es_stream_t stream);
int es_counter_add_i64_if(int64_t* counter, int64_t v, const int32_t* flag, es_stream_t stream);
/* es_counter_add_i64_if over n counters in one launch (host arrays of device pointers / addends): the
 * BatchNorm num_batches_tracked counts of one expert program (dynamic rows) applied together. */
int es_counters_add_i64_if(int64_t* const* counters, const int64_t* v, int n, const int32_t* flag,
                           es_stream_t stream);
/* Multi-expert step plan on the device (moe.py:97-135 without the host round trip): from counts [E]
 * (this rank's expert counts, es_router_gumbel) and, data parallel, counts_all [world][E] (all ranks'
 * counts, all-gathered on the device; NULL on one process), for each expert e: rows[e] = this rank's
 * live rows (its count if the expert trains -- global count > 1 -- and the count is >= min_local, else
 * 0), active[e] (the expert trains), n0[e] (this rank's first sample of the expert's global batch),
 * w[e] = float(count) / float(B) (class_counts_adjusted, moe.py:99-100), gcnt[e] (global count, float),
 * lcnt[e] (rows[e] as float). */
int es_expert_plan(const int32_t* counts, const int32_t* counts_all, int world, int rank, int E, int B,
                   int min_local, int32_t* rows, int32_t* active, int32_t* n0, float* w, float* gcnt,
                   float* lcnt, es_stream_t stream);
/* sizeof of the ABI structs (0 es_view_t, 1 es_dropout_t, 2 es_conv_desc_t, 3 es_norm_t, 4 es_chain_t,
 * 5 es_gen_loss_t, 6 es_dfront2_params_t, 7 es_dmlp_params_t; -1 unknown): the bindings check their
 * mirrors against it on load. */
int64_t es_struct_size(int which);
/* x[i] /= max(d[0], 1) for i < n (a sum over an expert's global batch -> its mean, d = the device count) */
int es_div_by(float* x, int n, const float* d, es_stream_t stream);
/* EMA of a flat parameter buffer — replaces EMAHelper.update (expertsim/train/loop.py:392-400):
 * shadow[i] = decay*shadow[i] + one_minus_decay*p[i], each product rounded, then one add. */
int es_ema_update(float* shadow, const float* p, int64_t n, float decay, float one_minus_decay,
                  es_stream_t stream);
/* dropout mask materialisation (tests): out[i] = keep(i) */
int es_dropout_mask(uint8_t* out, int64_t n, const es_dropout_t* d, es_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Evaluation (moe.py:644-692).
 * ---------------------------------------------------------------------------------------- */
/* 5-channel photon sums of x [n,1,h,w] (any strides): out[b*5 + k] (fp64) = sum over mask k+1 of
 * get_channel_masks (train/utils.py:18-59) as sum_channels_parallel (train/utils.py:62-78)
 * computes it; log_domain != 0 applies expm1 first (moe.py:646, train/utils.py:198). */
int es_channel_sums(const es_view_t* x, es_dtype_t dt, const void* xp, int log_domain, double* out,
                    es_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* EXPERTSIM_HIP_H */
