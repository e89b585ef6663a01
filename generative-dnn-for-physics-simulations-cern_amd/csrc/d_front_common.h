// Shared pieces of the fused discriminator-front kernels (d_front.hip, d_front2.hip): the first
// conv block SNconv 3x3 1->32 -> GroupNorm(8, 32) -> LeakyReLU -> MaxPool 2x2 evaluated per pooling
// window from the image staged in LDS.
//
// Lane layout: thread t handles channel quad g = t & 7 (GroupNorm group g = channels 4g..4g+3)
// and pooling windows u = t >> 3, u + 64, ...  A window's 2x2 conv outputs come from its 4x4 image
// patch, read once from LDS and shared by the quad's 4 channels.
#pragma once
#include "common.h"

namespace dfront {

constexpr int FT = 512;                    // threads per image
constexpr int FK = 32, FG = 8, CPG = 4;    // conv channels, GN groups, channels per group
constexpr int TAPS = 9;                    // 3x3
constexpr int MAXPIX = 2048;               // image pixels held in LDS
constexpr int MAXOUT = 1792;               // conv outputs per image (e_rs planes in LDS)
constexpr int NW = FT / 64;                // waves per workgroup

struct Quad {                              // the thread's 4 channels: W/sigma, bias, gamma, beta
  float w[CPG][TAPS], b[CPG], gm[CPG], bt[CPG];
};

__device__ __forceinline__ void load_quad_p(const float* w, const float* sigma, const float* bias, const float* gamma,
                                            const float* beta, int g, Quad& q) {
  const float sc = sigma ? 1.f / sigma[0] : 1.f;     // as es_pack_conv_weight
#pragma unroll
  for (int c = 0; c < CPG; ++c) {
    const int k = g * CPG + c;
#pragma unroll
    for (int t = 0; t < TAPS; ++t) q.w[c][t] = w[k * TAPS + t] * sc;
    q.b[c] = bias ? bias[k] : 0.f;
    q.gm[c] = gamma ? gamma[k] : 1.f;
    q.bt[c] = beta ? beta[k] : 0.f;
  }
}

// image n ([N][1][H][W], element strides is) into LDS, row-major
__device__ __forceinline__ void stage_image_p(const float* img, const int64_t* is, int H, int W, int n, float* im) {
  const float* src = img + n * is[0];
  for (int i = threadIdx.x; i < H * W; i += FT) {
    const int h = i / W, x = i - h * W;
    im[i] = src[h * is[2] + x * is[3]];
  }
}

// The 4x4 image patch of pooling window (pi, pj) and its 2x2 conv outputs v[pos][c],
// pos = 2*dy + dx (row-major window order, as the pool's argmax byte).
__device__ __forceinline__ void window(const float* im, int W, int pi, int pj, const Quad& q,
                                       float (&x)[4][4], float (&v)[4][CPG]) {
  const float* p = im + 2 * pi * W + 2 * pj;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int s = 0; s < 4; ++s) x[r][s] = p[r * W + s];
#pragma unroll
  for (int pos = 0; pos < 4; ++pos)
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      float s = q.b[c];
#pragma unroll
      for (int t = 0; t < TAPS; ++t) s = fmaf(x[(pos >> 1) + t / 3][(pos & 1) + t % 3], q.w[c][t], s);
      v[pos][c] = s;
    }
}

// In place: v[i] <- sum of v[i] over the workgroup's threads with the same channel quad (t & 7).
// red holds NW * 8 * NV floats.
template <int NV>
__device__ __forceinline__ void quad_sum(float (&v)[NV], float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] += __shfl_xor(v[i], 8, 64);
    v[i] += __shfl_xor(v[i], 16, 64);
    v[i] += __shfl_xor(v[i], 32, 64);
  }
  __syncthreads();                                   // red may still be read by a previous use
  if (lane < 8) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[(wid * 8 + lane) * NV + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) t += red[(k * 8 + (lane & 7)) * NV + i];
    v[i] = t;
  }
}


}  // namespace dfront
