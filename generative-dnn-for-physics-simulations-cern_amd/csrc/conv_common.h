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
};


// 8-wave LDS-DMA ring kernels (conv_mfma.hip).  Return 1 when the call was launched, 0 when the
// shape is not eligible (the caller falls back to the kernels of conv_igemm.hip), <0 on error.
int es_conv_ring_launch(ConvArgs& a, int mode, hipStream_t st);
