// Fused front of the spectral-norm discriminator (conv_layers.0 .. conv_layers.3 of
// neutron/discriminator.py:11-15 and proton/discriminator.py:121-125):
//
//   SNconv 3x3 1->32 (+bias) -> GroupNorm(8, 32) -> LeakyReLU(0.1) -> MaxPool 2x2
//
// Unfused (c1_fwd of conv_thin.hip + the GN passes of norm.hip + the pool of misc.hip), this
// block moves the largest activations of the fp32 discriminator: the 32-channel conv output
// (42x42 neutron, 54x28 proton) is written once, read by the GN reduction, read and written by the
// GN/LReLU pass and read by the pool; the backward reads / writes it again in the pool backward,
// both GN-backward passes, the conv wgrad and the conv dgrad (~0.6 GB per forward and ~1 GB per
// backward at B = 512).  Its arithmetic is tiny (9 MACs per conv output), so ONE workgroup owns
// ONE image: the image (<= 2048 pixels) is staged in LDS and every pass recomputes the conv
// outputs it needs from it — the 32-channel map never goes to HBM.
//
//   forward  reads the image; writes pooled [N][Hp][Wp][32] fp32, the pool argmax bytes
//            [N][Hp][Wp][32] (es_maxpool_fwd's format) and the GN mean / invstd [N][8].
//   backward reads the image, dpooled, the argmax bytes and the GN stats; writes the image
//            gradient (optional) and per-image partials of dW (of W/sigma), dbias, dgamma, dbeta,
//            which a second launch sums over the images (deterministic, no atomics).
//            Image gradient: dx[i][j] = sum_{r,s} e_rs[i-r][j-s] with e_rs[o] = sum_k dh[o][k] W[k][r][s]
//            built in LDS (9 x Ho*Wo floats), so dh itself is never stored.
//
// Lane layout and the per-window helpers: d_front_common.h.
#include "d_front_common.h"

namespace {

using namespace dfront;

constexpr int NPART = FK * TAPS + 3 * FK;  // per image: dW [32][9] | dbias | dgamma | dbeta

struct FrontArgs {
  const float* img; int64_t is[4];         // image [N][1][H][W] with element strides
  int H, W, Ho, Wo, Hp, Wp;
  const float* w; const float* sigma;      // weight_orig [32][1][3][3]; sigma[0] (or NULL)
  const float* bias; const float* gamma; const float* beta;
  float eps, slope;
  float* mean; float* invstd;              // [N][8]
  float* pooled; uint8_t* idx;             // [N][Hp][Wp][32]
  const float* dpooled;                    // [N][Hp][Wp][32]
  float* dx; int64_t dxs[4];               // image gradient [N][1][H][W] (or NULL)
  float* part;                             // [N][NPART]
};

__global__ void __launch_bounds__(FT) dfront_fwd_kernel(FrontArgs a) {
  __shared__ float im[MAXPIX];
  __shared__ float red[NW * 8];
  const int n = blockIdx.x, g = threadIdx.x & 7, u = threadIdx.x >> 3;
  Quad q;
  load_quad_p(a.w, a.sigma, a.bias, a.gamma, a.beta, g, q);
  stage_image_p(a.img, a.is, a.H, a.W, n, im);
  __syncthreads();
  const int NP = a.Hp * a.Wp;
  const float cnt = (float)(CPG * a.Ho * a.Wo);

  float s[1] = {0.f};
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
#pragma unroll
    for (int pos = 0; pos < 4; ++pos)
#pragma unroll
      for (int c = 0; c < CPG; ++c) s[0] += v[pos][c];
  }
  quad_sum(s, red);
  const float mu = s[0] / cnt;

  float m2[1] = {0.f};                               // two-pass variance (biased, as GroupNorm)
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
#pragma unroll
    for (int pos = 0; pos < 4; ++pos)
#pragma unroll
      for (int c = 0; c < CPG; ++c) {
        const float d = v[pos][c] - mu;
        m2[0] = fmaf(d, d, m2[0]);
      }
  }
  quad_sum(m2, red);
  const float istd = rsqrtf(m2[0] / cnt + a.eps);
  if (threadIdx.x < 8) { a.mean[n * FG + g] = mu; a.invstd[n * FG + g] = istd; }

  float* out = a.pooled + (int64_t)n * NP * FK + g * CPG;
  uint32_t* ix = (uint32_t*)(a.idx + (int64_t)n * NP * FK) + g;
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
    float best[CPG];
    uint32_t bits = 0;
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      best[c] = -INFINITY;
      int bi = 0;
#pragma unroll
      for (int pos = 0; pos < 4; ++pos) {
        const float y = lrelu(fmaf((v[pos][c] - mu) * istd, q.gm[c], q.bt[c]), a.slope);
        if (y > best[c] || (isnan(y) && !isnan(best[c]))) { best[c] = y; bi = pos; }
      }
      bits |= (uint32_t)bi << (8 * c);
    }
    *(float4*)(out + pp * FK) = make_float4(best[0], best[1], best[2], best[3]);
    ix[pp * FG] = bits;
  }
}

// WANT_DX is compile-time: without the image gradient (the D step) the e_rs sums are not computed
template <bool WANT_DX>
__global__ void __launch_bounds__(FT) dfront_bwd_kernel(FrontArgs a) {
  __shared__ float im[MAXPIX];
  __shared__ float ep[TAPS * MAXOUT];      // e_rs planes; also the reduction scratch
  const int n = blockIdx.x, g = threadIdx.x & 7, u = threadIdx.x >> 3;
  Quad q;
  load_quad_p(a.w, a.sigma, a.bias, a.gamma, a.beta, g, q);
  stage_image_p(a.img, a.is, a.H, a.W, n, im);
  __syncthreads();
  const int NP = a.Hp * a.Wp;
  const float cnt = (float)(CPG * a.Ho * a.Wo);
  const float mu = a.mean[n * FG + g], istd = a.invstd[n * FG + g];
  const float* dp = a.dpooled + (int64_t)n * NP * FK + g * CPG;
  const uint32_t* ix = (const uint32_t*)(a.idx + (int64_t)n * NP * FK) + g;
  float* part = a.part + (int64_t)n * NPART;

  // pass 1: the pool routes dpooled to its argmax; there d(act input) = dp * lrelu'(a).
  // r = {sum dn, sum dn*xhat (dn = gamma * dact), dgamma[4] = sum dact*xhat, dbeta[4] = sum dact}
  float r[2 + 2 * CPG];
#pragma unroll
  for (int i = 0; i < 2 + 2 * CPG; ++i) r[i] = 0.f;
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
    const float4 d4 = *(const float4*)(dp + pp * FK);
    const float dv[CPG] = {d4.x, d4.y, d4.z, d4.w};
    const uint32_t bits = ix[pp * FG];
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      const int bi = (bits >> (8 * c)) & 3;
      float hv = v[0][c];
#pragma unroll
      for (int pos = 1; pos < 4; ++pos) hv = bi == pos ? v[pos][c] : hv;
      const float xh = (hv - mu) * istd;
      const float av = fmaf(xh, q.gm[c], q.bt[c]);
      const float da = av > 0.f ? dv[c] : dv[c] * a.slope;
      const float dn = da * q.gm[c];
      r[0] += dn;
      r[1] = fmaf(dn, xh, r[1]);
      r[2 + c] = fmaf(da, xh, r[2 + c]);
      r[2 + CPG + c] += da;
    }
  }
  quad_sum(r, ep);
  if (u == 0) {
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      part[FK * TAPS + FK + g * CPG + c] = r[2 + c];
      part[FK * TAPS + 2 * FK + g * CPG + c] = r[2 + CPG + c];
    }
  }
  const float k1 = r[0] / cnt, k2 = r[1] / cnt;
  __syncthreads();                         // every thread has read ep's reduction scratch

  // pass 2: dh = istd * (dn - mean(dn) - xhat * mean(dn * xhat)) at every conv output;
  // acc = {dW[c][tap] = sum dh * image tap, dbias[c] = sum dh}; e_rs[o] = sum_c dh[o][c] W[c][rs]
  float acc[CPG * TAPS + CPG];
#pragma unroll
  for (int i = 0; i < CPG * TAPS + CPG; ++i) acc[i] = 0.f;
  constexpr bool want_dx = WANT_DX;
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
    const float4 d4 = *(const float4*)(dp + pp * FK);
    const float dv[CPG] = {d4.x, d4.y, d4.z, d4.w};
    const uint32_t bits = ix[pp * FG];
    float e[4][TAPS];
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
#pragma unroll
      for (int t = 0; t < TAPS; ++t) e[pos][t] = 0.f;
#pragma unroll
      for (int c = 0; c < CPG; ++c) {
        const float xh = (v[pos][c] - mu) * istd;
        float dn = 0.f;
        if ((int)((bits >> (8 * c)) & 3) == pos) {
          const float av = fmaf(xh, q.gm[c], q.bt[c]);
          dn = (av > 0.f ? dv[c] : dv[c] * a.slope) * q.gm[c];
        }
        const float dh = istd * (dn - k1 - xh * k2);
        acc[CPG * TAPS + c] += dh;
#pragma unroll
        for (int t = 0; t < TAPS; ++t) {
          acc[c * TAPS + t] = fmaf(dh, x[(pos >> 1) + t / 3][(pos & 1) + t % 3], acc[c * TAPS + t]);
          if constexpr (WANT_DX) e[pos][t] = fmaf(dh, q.w[c][t], e[pos][t]);
        }
      }
    }
    if constexpr (want_dx) {
      // sum e over the window's 8 lanes (all 32 channels), then lane g stores entries g, g+8, ...
#pragma unroll
      for (int pos = 0; pos < 4; ++pos)
#pragma unroll
        for (int t = 0; t < TAPS; ++t) {
          float s = e[pos][t];
          s += __shfl_xor(s, 1, 64);
          s += __shfl_xor(s, 2, 64);
          s += __shfl_xor(s, 4, 64);
          e[pos][t] = s;
        }
#pragma unroll
      for (int i = 0; i < 4 * TAPS; ++i) {
        const int pos = i / TAPS, t = i % TAPS;
        if ((i & 7) == g) {
          const int o = (2 * pi + (pos >> 1)) * a.Wo + 2 * pj + (pos & 1);
          ep[t * MAXOUT + o] = e[pos][t];
        }
      }
    }
  }
  if constexpr (want_dx) {
    __syncthreads();
    // pass 3: image gradient, dx[i][j] = sum over taps (r, s) of e_rs[i - r][j - s]
    float* dx = a.dx + n * a.dxs[0];
    for (int p = threadIdx.x; p < a.H * a.W; p += FT) {
      const int i = p / a.W, j = p - i * a.W;
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const int oh = i - t / 3, ow = j - t % 3;
        if (oh >= 0 && oh < a.Ho && ow >= 0 && ow < a.Wo) s += ep[t * MAXOUT + oh * a.Wo + ow];
      }
      dx[i * a.dxs[2] + j * a.dxs[3]] = s;
    }
  }
  quad_sum(acc, ep);                       // (its leading barrier orders pass 3's reads of ep)
  if (u == 0) {
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
#pragma unroll
      for (int t = 0; t < TAPS; ++t) part[(g * CPG + c) * TAPS + t] = acc[c * TAPS + t];
      part[FK * TAPS + g * CPG + c] = acc[CPG * TAPS + c];
    }
  }
}

// Sum the per-image partials: dw (= grad of W/sigma, torch layout [32][1][3][3]) is WRITTEN,
// dbias / dgamma / dbeta are ACCUMULATED (+=); any may be NULL.
__global__ void __launch_bounds__(1024) dfront_part_reduce(const float* __restrict__ part, int N, float* dw,
                                                           float* dbias, float* dgamma, float* dbeta) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6, col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < NPART)
    for (int n = sl; n < N; n += 16) s += part[(int64_t)n * NPART + col];
  red[sl][lane] = s;
  __syncthreads();
  if (sl != 0 || col >= NPART) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k][lane];
  if (col < FK * TAPS) { if (dw) dw[col] = t; }
  else if (col < FK * TAPS + FK) { if (dbias) dbias[col - FK * TAPS] += t; }
  else if (col < FK * TAPS + 2 * FK) { if (dgamma) dgamma[col - FK * TAPS - FK] += t; }
  else if (dbeta) dbeta[col - FK * TAPS - 2 * FK] += t;
}

int front_args(FrontArgs& a, const float* img, const int64_t is[4], int N, int H, int W, const float* w,
               const float* sigma, const float* bias, const float* gamma, const float* beta, float eps,
               float slope) {
  ES_CHECK_ARG(img && is && w && N > 0, "es_dfront: null argument");
  ES_CHECK_ARG(H >= 4 && W >= 4 && H * W <= MAXPIX && (H - 2) * (W - 2) <= MAXOUT && (H - 2) % 2 == 0 &&
                   (W - 2) % 2 == 0,
               "es_dfront: image %dx%d unsupported (H*W <= %d, H-2 and W-2 even)", H, W, MAXPIX);
  a = FrontArgs{};
  a.img = img;
  for (int i = 0; i < 4; ++i) a.is[i] = is[i];
  a.H = H; a.W = W; a.Ho = H - 2; a.Wo = W - 2; a.Hp = a.Ho / 2; a.Wp = a.Wo / 2;
  a.w = w; a.sigma = sigma; a.bias = bias; a.gamma = gamma; a.beta = beta;
  a.eps = eps; a.slope = slope;
  return ES_OK;
}

}  // namespace

extern "C" int64_t es_dfront_part_floats(int N) { return (int64_t)N * NPART; }

extern "C" int es_dfront_fwd(const float* img, const int64_t is[4], int N, int H, int W, const float* w,
                             const float* sigma, const float* bias, const float* gamma, const float* beta,
                             float eps, float slope, float* mean, float* invstd, float* pooled, uint8_t* idx,
                             es_stream_t stream) {
  FrontArgs a;
  if (int rc = front_args(a, img, is, N, H, W, w, sigma, bias, gamma, beta, eps, slope)) return rc;
  ES_CHECK_ARG(mean && invstd && pooled && idx, "es_dfront_fwd: null output");
  a.mean = mean; a.invstd = invstd; a.pooled = pooled; a.idx = idx;
  hipLaunchKernelGGL(dfront_fwd_kernel, dim3(N), dim3(FT), 0, (hipStream_t)stream, a);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_dfront_bwd(const float* img, const int64_t is[4], int N, int H, int W, const float* w,
                             const float* sigma, const float* bias, const float* gamma, const float* beta,
                             float eps, float slope, const float* mean, const float* invstd, const uint8_t* idx,
                             const float* dpooled, float* dx, const int64_t dxs[4], float* part, float* dw,
                             float* dbias, float* dgamma, float* dbeta, es_stream_t stream) {
  FrontArgs a;
  if (int rc = front_args(a, img, is, N, H, W, w, sigma, bias, gamma, beta, eps, slope)) return rc;
  ES_CHECK_ARG(mean && invstd && idx && dpooled && part, "es_dfront_bwd: null argument");
  ES_CHECK_ARG(!dx || dxs, "es_dfront_bwd: dx without strides");
  a.mean = (float*)mean; a.invstd = (float*)invstd; a.idx = (uint8_t*)idx;
  a.dpooled = dpooled; a.dx = dx; a.part = part;
  if (dx)
    for (int i = 0; i < 4; ++i) a.dxs[i] = dxs[i];
  if (a.dx) hipLaunchKernelGGL(dfront_bwd_kernel<true>, dim3(N), dim3(FT), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(dfront_bwd_kernel<false>, dim3(N), dim3(FT), 0, (hipStream_t)stream, a);
  ES_CHECK_LAUNCH();
  if (dw || dbias || dgamma || dbeta) {
    hipLaunchKernelGGL(dfront_part_reduce, dim3((NPART + 63) / 64), dim3(1024), 0, (hipStream_t)stream, part, N,
                       dw, dbias, dgamma, dbeta);
    ES_CHECK_LAUNCH();
  }
  return ES_OK;
}
