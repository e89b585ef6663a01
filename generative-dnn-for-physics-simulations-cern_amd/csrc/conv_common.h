// Shared host/device definitions of the implicit-GEMM convolution kernels (conv_igemm.hip: the
// generic / register-staged and first LDS-DMA kernels; conv_mfma.hip: the 8-wave LDS-DMA ring
// kernels).  ConvArgs is passed by value to every conv kernel, so both files see one definition.
#pragma once
#include "common.h"

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

// Unsigned division by a run-time constant (x < 2^31): q = (umulhi(x, m) + x) >> l.
struct FastDiv {
  uint32_t m;
  int l;
};
static inline FastDiv mkdiv(uint32_t d) {
  FastDiv f;
  f.l = 0;
  while ((1ull << f.l) < d) ++f.l;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << f.l) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ int fdiv(int x, FastDiv f) {
  return (int)((__umulhi((uint32_t)x, f.m) + (uint32_t)x) >> f.l);
}

// Sub-pixel decomposition of a stride-1 conv over a x2 nearest-upsampled input (conv_mfma.hip).
// Output pixels split into 4 parity classes c = 2a + b, (p - pad) mod 2 = a, (q - pad) mod 2 = b.
// Class c covers output rows p = p0[c] + 2u (u < ph[c]) and is a plain dh[c] x dw[c] conv on the
// SOURCE grid: y[p0 + 2u][q0 + 2v] = sum_{d,e} x[u + oh + d][v + ow + e] * W'_c[d][e] with
// W'_c[d][e] = sum of W[r][s] over r in {2d - a, 2d - a + 1}, s in {2e - b, 2e - b + 1} (in range).
struct SubPixel {
  int on;
  int ph[4], pw[4];      // class grid
  int p0[4], q0[4];      // first output row / column of the class
  int oh[4], ow[4];      // source row of (u, d) = u + oh + d
  int dh[4], dw[4];      // combined taps
  int tap0[5];           // prefix sums of dh*dw (packed weight blocks)
  int tile0[5];          // FWD: prefix sums of the classes' row tiles (per 8-image group)
};
void es_make_subpixel(const es_conv_desc_t& d, int row_tile, SubPixel& sp);

struct ConvArgs {
  FastDiv fC, fS, fK, fQ, fP, fWu, fHu, fUh, fUw, fRSK, fW, fH;
  int fold;            // DGRAD with integer upsample folded (rows on the source grid)
  es_conv_desc_t d;
  const void* a_src;
  const void* b_src;
  int64_t as[4];      // FWD: x strides;  DGRAD/WGRAD: dy strides
  int64_t bs[4];      // WGRAD: x strides
  void* out;
  int64_t os[4];      // FWD: y strides; DGRAD: dxu strides
  const float* bias;
  float beta;
  int out_bf16;
  int M, Ng, Kd;
  int k_per_split;
  int dense_f32_out;   // host: output is fp32, dense [M][Ng] and beta == 0 (split-K allowed)
  int splitk;          // FWD / DGRAD split over blockIdx.z: fp32 atomics into a zeroed dense output
  SubPixel sp;         // ring kernels: sub-pixel class geometry (sp.on)
  int ng;              // ring FWD/DGRAD: images per group of the row order (8, 16, 32 or 64)
  int vec_out;         // ring FWD/DGRAD: output rows channel-contiguous, 16-byte aligned, beta == 0
  float* stats_part;   // ring FWD: per-row-tile BatchNorm partials [tile][3][Ng] (count, mean, M2)
  int sp_tpc;          // ring SP FWD: 0 = class-major tile order; else class-interleaved with this
                       // many tiles per class (the 4 classes of the same source pixels adjacent)
  int sp_merge;        // ring SP FWD with 4 identical class geometries: ONE GEMM whose columns are
                       // (class, out-channel) (4*Ng columns; the classes share the source gather)
  // persistent DGRAD fused with the reduction pass of the BatchNorm backward that consumes its
  // output (es_conv2d_dgrad_bnred): x = the norm's input h (same layout as the dgrad output), its
  // dropout keep bits and statistics; per workgroup sums of dnorm and dnorm*xhat -> bnr_part
  const void* bnr_x;
  const uint8_t* bnr_keep;
  const float *bnr_mean, *bnr_invstd, *bnr_gamma, *bnr_beta;
  float bnr_scale, bnr_slope;   // dropout 1/(1-p) (1 without dropout), LeakyReLU slope
  int bnr_dfirst, bnr_drop;
  float* bnr_part;              // [workgroup][3][Ng] (slots 1, 2: the two sums)
  int det;                      // WGRAD (es_conv2d_wgrad_det): split z stores its raw tile into
                                // g_det_req.ws + z * M * Ng instead of atomics; split-K FWD / DGRAD
                                // (es_conv2d_*_det): into det_ws + z * M * Ng
  float* det_ws;
  int prio;                     // split-fp32 ring kernels: waves 4-7 at s_setprio 1 (VALU arbitration)
  int nbase;                    // dynamic rows: the launch's first image within d.rows' count (chunks)
  int mslot;                    // generic kernels (device-side): the launch's M, the split partials' stride
};

// Images of the launch that carry data: d.N, or with dynamic rows (es_conv_desc_t.rows, a device
// count of the batch's live images) the part of [nbase, nbase + d.N) below that count.  Kernels
// skip the tiles / K-steps past it and read its images as zeros (buffer num_records).
__device__ __forceinline__ int conv_live(const ConvArgs& a) {
  if (a.d.rows == nullptr) return a.d.N;
  const int px = a.d.rows_px > 0 ? a.d.rows_px : 1;
  const int v = __builtin_amdgcn_readfirstlane(a.d.rows[0]) - a.nbase * px;
  const int img = (v + px - 1) / px;       // (pixel rows: the images holding a live one)
  return v <= 0 ? 0 : (img < a.d.N ? img : a.d.N);
}
// rows_px > 0: the live pixel rows (samples) of the launch, image-major; else INT_MAX (whole images)
__device__ __forceinline__ int conv_live_px(const ConvArgs& a) {
  if (a.d.rows == nullptr || a.d.rows_px <= 0) return 0x7fffffff;
  const int v = __builtin_amdgcn_readfirstlane(a.d.rows[0]) - a.nbase * a.d.rows_px;
  return v < 0 ? 0 : v;
}

// The generic GEMM kernels (conv_igemm.hip) shrink their problem to the live images: M (FWD /
// DGRAD rows, image-major) or the K of a WGRAD (N*P*Q pixels).  mslot keeps the launch's M.
__device__ __forceinline__ void conv_live_gemm(ConvArgs& a, int mode) {
  a.mslot = a.M;
  if (a.d.rows == nullptr) return;
  const int nl = conv_live(a), npx = conv_live_px(a);
  if (mode == MODE_WGRAD) a.Kd = min(nl * (a.Kd / a.d.N), npx);
  else a.M = min(nl * (a.M / a.d.N), npx);
}


// es_conv2d_wgrad_det: the partial buffer offered to the generic (register-staged / thin) WGRAD
// kernels (host, per thread); the launch sets splits = partial slots written
struct DetRequest {
  float* ws;
  int64_t floats;
  int splits;
};
extern thread_local DetRequest g_det_req;

// es_conv2d_dgrad_bnred: the caller's request (host, per thread); the persistent DGRAD launch
// sets chunks when it wrote the sums
struct BnRedRequest {
  const void* x;
  const es_norm_t* nm;
  const es_chain_t* ch;
  float* part;
  int64_t floats;
  int chunks;
};
extern thread_local BnRedRequest g_bnr_req;



// es_conv2d_fwd_stats: the caller's request for fused BatchNorm partials (host, per thread); the
// ring FWD launch sets chunks when it writes them.
struct StatsRequest {
  float* part;
  int64_t floats;
  int chunks;
};
extern thread_local StatsRequest g_stats_req;

// which ring path the last conv launch took (host, per thread; es_conv_exec_flops accounting):
// bit 0 a ring kernel ran, bit 1 split-fp32 planes, bit 2 the sub-pixel decomposition
extern thread_local int g_ring_hit;

// split-fp32 weight planes: byte offset of the planes behind an fp32 packing of n elements
extern "C" int64_t es_weight_planes_offset(int64_t n);

// 8-wave LDS-DMA ring kernels (conv_mfma.hip).  Return 1 when the call was launched, 0 when the
// shape is not eligible (the caller falls back to the kernels of conv_igemm.hip), <0 on error.
int es_conv_ring_launch(ConvArgs& a, int mode, hipStream_t st);
// fp32 operands (parity mode): FWD / DGRAD ring kernels over image chunks (same return convention)
int es_conv_ring_launch_f32(ConvArgs& a, int mode, hipStream_t st);
// deterministic fp32 WGRAD on the ring (conv_mfma.hip): partial floats needed (-1: not eligible), and
// the launch (partials + ordered reduce into the torch-layout dW; 1 done, 0 not eligible, < 0 error)
int64_t es_wgrad_f32_ring_floats(const es_conv_desc_t& d, const int64_t ys[4], const int64_t xs[4]);
int es_wgrad_f32_ring(const es_conv_desc_t& d, const void* dy, const int64_t ys[4], const void* x,
                      const int64_t xs[4], float* dw, float beta, float* ws, int64_t ws_floats, hipStream_t st);
// the wave-specialised split-fp32 WGRAD partial kernel (conv_wgrad_ws.hip), 128 x bn tiles over grid
// (row tiles, column tiles, K splits); 1 launched, 0 not eligible
int es_wgrad_ws_launch(int bn, bool sp, dim3 grid, const ConvArgs& a, float* wsc, int ngt, hipStream_t st);
// ordered sum of per-split partials ws[split][K][R*S*C] into dW (torch layout [K][C][R][S])
void es_wgrad_reduce_plain(const float* ws, int splits, int K, int C, int R, int S, float* dw, float beta,
                           hipStream_t st);
