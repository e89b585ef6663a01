// Direct (non-GEMM) convolutions for the layers with ONE input or ONE output channel.
//
// These layers have almost no arithmetic (<= 0.3 GFLOP per launch at B = 512) but move the largest
// activations of the step, and as implicit GEMMs they waste >= 3/4 of every MFMA tile (N or K
// collapses to 1), so they run here as HBM-bound direct kernels:
//   Cin  == 1 : the discriminators' conv_layers.0 (neutron/discriminator.py:12, proton/
//               discriminator.py:122; 1->32, 3x3) and the neutron aux regressor conv1
//               (neutron/aux_reg.py:14; 1->32, 3x3)                       fwd / dgrad / wgrad
//   Cout == 1 : the generators' last conv (neutron/generator.py:34, proton/generator.py:42;
//               64->1, 2x2)                                               fwd / dgrad / wgrad
// Same operands as the GEMM path (conv_igemm.hip): packed weights (fwd [K][R][S][C], dgrad
// [C][R][S][K]) in the compute dtype, fp32 accumulation, wgrad accumulated into fp32 [K][R*S*C]
// with atomics.  Stride 1 (Cin == 1 also stride 2), any zero padding, no upsample.
#include <algorithm>
#include <type_traits>

#include "conv_common.h"

namespace {

constexpr int NT = 256;

template <typename T> struct V16;
template <> struct V16<float> { static constexpr int N = 4; };
template <> struct V16<bf16> { static constexpr int N = 8; };

// 8 consecutive elements <-> floats
template <typename T> __device__ __forceinline__ void ld8(const T* p, float* f);
template <> __device__ __forceinline__ void ld8<bf16>(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = (float)v[k];
}
template <> __device__ __forceinline__ void ld8<float>(const float* p, float* f) {
  const float4 a = ((const float4*)p)[0], b = ((const float4*)p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
template <typename T> __device__ __forceinline__ void st8(T* p, const float* f);
template <> __device__ __forceinline__ void st8<bf16>(bf16* p, const float* f) {
  bf16x8 v;
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = (bf16)f[k];
  *(bf16x8*)p = v;
}
template <> __device__ __forceinline__ void st8<float>(float* p, const float* f) {
  ((float4*)p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  ((float4*)p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

struct Thin {
  es_conv_desc_t d;
  const void* a; int64_t as[4];    // fwd: x;  dgrad / wgrad: dy
  const void* b; int64_t bs[4];    // wgrad: x
  const void* w;                   // packed weights (fwd / dgrad)
  const float* bias;
  void* out; int64_t os[4];        // fwd: y; dgrad: dx; wgrad: fp32 dw [K][R*S*C]
  float beta;
  int M;                           // output pixels (fwd, wgrad: N*P*Q; dgrad: N*H*W)
  int det;                         // wgrad: block b stores its sums into out + b * (K*R*S*C) (no atomics)
};

// pixels of the live images (es_conv_desc_t.rows: a device count of the live images; the rows are
// image-major, so they are a prefix of the M = N * pixels rows)
__device__ __forceinline__ int thin_m(const Thin& t) {
  if (t.d.rows == nullptr) return t.M;
  if (t.d.rows_px > 0) return min(t.M, max(__builtin_amdgcn_readfirstlane(t.d.rows[0]), 0));   // pixel rows
  return live_rows(t.d.rows, t.d.N) * (t.M / t.d.N);
}

__device__ __forceinline__ void pix3(int m, int A, int B, int& n, int& i, int& j) {
  j = m % B; const int t = m / B; i = t % A; n = t / A;
}

// ============================================================ Cin == 1
// fwd: LP = K / VO lanes per output pixel, each producing VO consecutive channels (one 16-byte
// store; a pixel's K outputs are one contiguous run written by consecutive lanes).
template <typename T, typename TO, int RS>
__global__ void __launch_bounds__(NT) c1_fwd(Thin t) {
  constexpr int VO = 16 / sizeof(TO);
  const es_conv_desc_t& d = t.d;
  t.M = thin_m(t);   // dynamic rows: the live images' pixels
  __shared__ float wf[64 * RS], bs[64];
  for (int i = threadIdx.x; i < d.K * RS; i += NT) wf[i] = to_f(((const T*)t.w)[i]);
  for (int i = threadIdx.x; i < d.K; i += NT) bs[i] = t.bias ? t.bias[i] : 0.f;
  __syncthreads();
  const int LP = d.K / VO, PPB = NT / LP;
  const int k0 = (threadIdx.x % LP) * VO;
  // grid-stride over the pixels, two per trip (a block per 32 pixels spent its time staging the
  // weights: 56 k blocks at B = 1024)
  constexpr int U = 2;
  const int stride = gridDim.x * PPB;
  for (int m0 = blockIdx.x * PPB + threadIdx.x / LP; m0 < t.M; m0 += U * stride) {
    float xv[U][RS];
    int nn[U], pp[U], qq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * stride;
      pix3(m < t.M ? m : m0, d.P, d.Q, nn[u], pp[u], qq[u]);
      const T* x = (const T*)t.a + nn[u] * t.as[0];
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const int hu = pp[u] * d.stride - d.pad + j / d.S, wu = qq[u] * d.stride - d.pad + j % d.S;
        const bool ok = hu >= 0 && hu < d.H && wu >= 0 && wu < d.W;
        const float v = to_f(x[ok ? hu * t.as[2] + wu * t.as[3] : 0]);   // clamped: loads issue together
        xv[u][j] = ok ? v : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (m0 + u * stride >= t.M) break;
      float o[8];
#pragma unroll
      for (int kk = 0; kk < VO; ++kk) {
        float sacc = bs[k0 + kk];
#pragma unroll
        for (int j = 0; j < RS; ++j) sacc += xv[u][j] * wf[(k0 + kk) * RS + j];
        o[kk] = sacc;
      }
      TO* y = (TO*)t.out + nn[u] * t.os[0] + pp[u] * t.os[2] + qq[u] * t.os[3] + k0;
      if constexpr (VO == 8) st8<TO>(y, o);
      else *(float4*)y = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

// dgrad: LP = K / VN lanes per input pixel; lane l dots its 16-byte chunk of each tap's dy row
// with the weights (coalesced row reads), then the LP partial sums are reduced by shuffles.
template <typename T, typename TO, int RS>
__global__ void __launch_bounds__(NT) c1_dgrad(Thin t) {
  constexpr int VN = V16<T>::N;
  const es_conv_desc_t& d = t.d;
  t.M = thin_m(t);   // dynamic rows: the live images' pixels
  __shared__ float wf[64 * RS];
  for (int i = threadIdx.x; i < d.K * RS; i += NT) wf[i] = to_f(((const T*)t.w)[i]);
  __syncthreads();
  const int LP = d.K / VN, PPB = NT / LP;
  const int m = blockIdx.x * PPB + threadIdx.x / LP, l = threadIdx.x % LP;
  const bool live = m < t.M;
  int n, h, w;
  pix3(live ? m : 0, d.H, d.W, n, h, w);
  const T* dy = (const T*)t.a + n * t.as[0] + l * VN;
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < RS; ++j) {
    int ph = h + d.pad - j / d.S, pw = w + d.pad - j % d.S;
    bool ok = live && ph >= 0 && pw >= 0;
    if (d.stride == 2) {
      ok = ok && !((ph | pw) & 1);
      ph >>= 1; pw >>= 1;
    }
    ok = ok && ph < d.P && pw < d.Q;
    // clamped tap (row 0) and a select instead of a branch: the taps' loads issue together
    const T* row = dy + (ok ? ph * t.as[2] + pw * t.as[3] : 0);
    const float* wr = wf + j * d.K + l * VN;
    if constexpr (VN == 8) {
      float v[8];
      ld8<T>(row, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += (ok ? v[e] : 0.f) * wr[e];
    } else {
      const float4 v = *(const float4*)row;
      if (ok) acc += v.x * wr[0] + v.y * wr[1] + v.z * wr[2] + v.w * wr[3];
    }
  }
  for (int o = LP >> 1; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (live && l == 0) {
    TO* o = (TO*)t.out + n * t.os[0] + h * t.os[2] + w * t.os[3];
    if (t.beta != 0.f) acc += t.beta * to_f(*o);
    *o = from_f<TO>(acc);
  }
}

// dgrad, workgroup per image: each dy pixel is read once; its RS partial dots t_j = <dy, w[:, j]>
// (reduced over the LP lanes of the pixel) go to LDS, then dx(h, w) = sum_j t_j(h + pad - r_j, w + pad - s_j)
// (stride 1).  The pixel-major kernel above re-read every dy row once per tap (9x).
constexpr int C1_TP_FLOATS = 16384;   // LDS floats of the per-tap partial dots (RS * P * Q)
template <typename T, typename TO, int RS>
__global__ void __launch_bounds__(NT) c1_dgrad_img(Thin t) {
  constexpr int VN = V16<T>::N;
  const es_conv_desc_t& d = t.d;
  const int n = blockIdx.x;
  if (n >= live_rows(d.rows, d.N)) return;   // dynamic rows: a padding image
  __shared__ float wf[64 * RS];              // [k][rs] (dgrad packing [C = 1][R][S][K] read as [rs][k])
  __shared__ float tp[C1_TP_FLOATS];         // [RS][P * Q]
  for (int i = threadIdx.x; i < d.K * RS; i += NT) {
    const int j = i / d.K, k = i - j * d.K;
    wf[k * RS + j] = to_f(((const T*)t.w)[i]);
  }
  __syncthreads();
  const int PQ = d.P * d.Q, LP = d.K / VN, PPB = NT / LP, l = threadIdx.x % LP;
  const T* dyn = (const T*)t.a + n * t.as[0] + l * VN;
  constexpr int U = 2;
  for (int m0 = 0; m0 < PQ; m0 += U * PPB) {
    float v[U][VN];
    int mm[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * PPB + threadIdx.x / LP;
      mm[u] = m;
      const int mc = m < PQ ? m : 0;
      const int p = mc / d.Q, q = mc - p * d.Q;
      const T* px = dyn + p * t.as[2] + q * t.as[3];
      if constexpr (VN == 8) {
        ld8<T>(px, v[u]);
      } else {
        const float4 q4 = *(const float4*)px;
        v[u][0] = q4.x; v[u][1] = q4.y; v[u][2] = q4.z; v[u][3] = q4.w;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float sj[RS];
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        float a = 0.f;
#pragma unroll
        for (int e = 0; e < VN; ++e) a += v[u][e] * wf[(l * VN + e) * RS + j];
        sj[j] = a;
      }
      for (int o = LP >> 1; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < RS; ++j) sj[j] += __shfl_xor(sj[j], o, 64);
      if (l == 0 && mm[u] < PQ)
#pragma unroll
        for (int j = 0; j < RS; ++j) tp[j * PQ + mm[u]] = sj[j];
    }
  }
  __syncthreads();
  TO* xo = (TO*)t.out + n * t.os[0];
  for (int o = threadIdx.x; o < d.H * d.W; o += NT) {
    const int h = o / d.W, w = o - h * d.W;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      const int ph = h + d.pad - j / d.S, pw = w + d.pad - j % d.S;
      if ((unsigned)ph < (unsigned)d.P && (unsigned)pw < (unsigned)d.Q) acc += tp[j * PQ + ph * d.Q + pw];
    }
    TO* dst = xo + h * t.os[2] + w * t.os[3];
    if (t.beta != 0.f) acc += t.beta * to_f(*dst);
    *dst = from_f<TO>(acc);
  }
}

// wgrad: thread = (pixel lane, 8-channel group); acc[8][RS] over a strided pixel range, then a
// shuffle + LDS reduction over the pixel lanes and one atomic per (k, tap) per block.
template <typename T, int RS>
__global__ void __launch_bounds__(NT) c1_wgrad(Thin t) {
  const es_conv_desc_t& d = t.d;
  t.M = thin_m(t);   // dynamic rows: the live images' pixels
  const int KO = d.K / 8;                 // 1..8, power of two (host-checked)
  const int ko = threadIdx.x % KO, pl = threadIdx.x / KO, PL = NT / KO;
  float acc[8][RS];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk)
#pragma unroll
    for (int j = 0; j < RS; ++j) acc[kk][j] = 0.f;
  // two pixels per trip, every load clamped and issued before the FMAs (the guarded per-tap
  // loads of one pixel at a time left each trip waiting on one round of global latency)
  const int stride = gridDim.x * PL;
  for (int m0 = blockIdx.x * PL + pl; m0 < t.M; m0 += 2 * stride) {
    float g[2][8], xv[2][RS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int mu = m0 + u * stride;
      const bool live = mu < t.M;
      int n, p, q;
      pix3(live ? mu : m0, d.P, d.Q, n, p, q);
      ld8<T>((const T*)t.a + n * t.as[0] + p * t.as[2] + q * t.as[3] + ko * 8, g[u]);
      const T* x = (const T*)t.b + n * t.bs[0];
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const int hu = p * d.stride - d.pad + j / d.S, wu = q * d.stride - d.pad + j % d.S;
        const bool ok = live && hu >= 0 && hu < d.H && wu >= 0 && wu < d.W;
        const float v = to_f(x[ok ? hu * t.bs[2] + wu * t.bs[3] : 0]);
        xv[u][j] = ok ? v : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < RS; ++j)
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) acc[kk][j] += g[u][kk] * xv[u][j];
  }
  // lanes l and l ^ (KO * 2^i) share the channel group inside a wave
#pragma unroll
  for (int kk = 0; kk < 8; ++kk)
#pragma unroll
    for (int j = 0; j < RS; ++j)
      for (int o = KO; o < 64; o <<= 1) acc[kk][j] += __shfl_xor(acc[kk][j], o, 64);
  __shared__ float red[4][64 * RS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < KO) {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int j = 0; j < RS; ++j) red[wid][(ko * 8 + kk) * RS + j] = acc[kk][j];
  }
  __syncthreads();
  float* dw = (float*)t.out;
  if (t.det) {
    for (int i = threadIdx.x; i < d.K * RS; i += NT)
      dw[(int64_t)blockIdx.x * d.K * RS + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  } else {
    for (int i = threadIdx.x; i < d.K * RS; i += NT)
      atomicAdd(&dw[i], red[0][i] + red[1][i] + red[2][i] + red[3][i]);
  }
}

// ============================================================ Cout == 1
// A pixel is served by LP = C/(VN*CH) lanes (CH 16-byte channel chunks each); 64/LP pixels per wave.
// fwd: y = bias + sum over taps of <x row chunks, w chunks>, reduced over the LP lanes.
template <typename T, typename TO, int RS, int CH = 1>
__global__ void __launch_bounds__(NT) k1_fwd(Thin t, int LP) {
  constexpr int VN = V16<T>::N;
  const es_conv_desc_t& d = t.d;
  t.M = thin_m(t);   // dynamic rows: the live images' pixels
  __shared__ float wf[1024];
  for (int i = threadIdx.x; i < RS * d.C; i += NT) wf[i] = to_f(((const T*)t.w)[i]);   // [R][S][C]
  __syncthreads();
  const int PPB = NT / LP;
  const int l = threadIdx.x % LP;
  // block-uniform grid-stride loop (the weights are staged once per block; the LP lanes of a
  // pixel stay in step for the shuffle reduction)
  for (int mb = blockIdx.x * PPB; mb < t.M; mb += gridDim.x * PPB) {
  const int m = mb + threadIdx.x / LP;
  const bool live = m < t.M;
  int n, p, q;
  pix3(live ? m : 0, d.P, d.Q, n, p, q);
  const T* x = (const T*)t.a + n * t.as[0] + l * VN * CH;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < RS; ++j) {
    const int hu = p - d.pad + j / d.S, wu = q - d.pad + j % d.S;
    const bool ok = live && hu >= 0 && hu < d.H && wu >= 0 && wu < d.W;
    const T* px = x + (ok ? hu * t.as[2] + wu * t.as[3] : 0);   // clamped: the taps' loads issue together
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const float* pw = wf + j * d.C + (l * CH + c) * VN;
      if constexpr (VN == 8) {
        float v[8];
        ld8<T>(px + c * VN, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (ok ? v[e] : 0.f) * pw[e];
      } else {
        const float4 v = *(const float4*)(px + c * VN);
        if (ok) s += v.x * pw[0] + v.y * pw[1] + v.z * pw[2] + v.w * pw[3];
      }
    }
  }
  for (int o = LP >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (live && l == 0) {
    TO* y = (TO*)t.out + n * t.os[0] + p * t.os[2] + q * t.os[3];
    *y = from_f<TO>(s + (t.bias ? t.bias[0] : 0.f));
  }
  }
}

// dgrad: dx[n,h,w,c] = sum over taps of dy[n, h+pad-r, w+pad-s] * w[c][r][s]   (wd = [C][R][S])
template <typename T, typename TO, int RS, int CH = 1>
__global__ void __launch_bounds__(NT) k1_dgrad(Thin t, int LP) {
  constexpr int VN = V16<T>::N;
  const es_conv_desc_t& d = t.d;
  t.M = thin_m(t);   // dynamic rows: the live images' pixels
  __shared__ float wf[1024];                                  // transposed to [R*S][C]
  for (int i = threadIdx.x; i < RS * d.C; i += NT) {
    const int c = i / RS, j = i % RS;
    wf[j * d.C + c] = to_f(((const T*)t.w)[i]);
  }
  __syncthreads();
  const int PPB = NT / LP;
  const int l = threadIdx.x % LP;
  for (int m = blockIdx.x * PPB + threadIdx.x / LP; m < t.M; m += gridDim.x * PPB) {
  int n, h, w;
  pix3(m, d.H, d.W, n, h, w);
  const T* dy = (const T*)t.a + n * t.as[0];
  float acc[CH][VN];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int e = 0; e < VN; ++e) acc[c][e] = 0.f;
#pragma unroll
  for (int j = 0; j < RS; ++j) {
    const int ph = h + d.pad - j / d.S, pw = w + d.pad - j % d.S;
    const bool ok = ph >= 0 && pw >= 0 && ph < d.P && pw < d.Q;
    const float gv = to_f(dy[ok ? ph * t.as[2] + pw * t.as[3] : 0]);   // clamped, then select
    const float g = ok ? gv : 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const float* wr = wf + j * d.C + (l * CH + c) * VN;
#pragma unroll
      for (int e = 0; e < VN; ++e) acc[c][e] += g * wr[e];
    }
  }
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    TO* o = (TO*)t.out + n * t.os[0] + h * t.os[2] + w * t.os[3] + (l * CH + c) * VN;
    if constexpr (VN == 8) {
      if (t.beta != 0.f) {
        float old[8];
        ld8<TO>(o, old);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[c][e] += t.beta * old[e];
      }
      st8<TO>(o, acc[c]);
    } else {
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        float v = acc[c][e];
        if (t.beta != 0.f) v += t.beta * to_f(o[e]);
        o[e] = from_f<TO>(v);
      }
    }
  }
  }
}

// k1_dgrad (bf16 in / out, beta 0, dense NHWC dx) fused with the REDUCTION pass of the BatchNorm
// backward that consumes dx (generator conv_layers.13's dgrad -> BatchNorm2d conv_layers.10 ->
// Dropout -> LeakyReLU, neutron/generator.py:33-37; es_conv2d_dgrad_bnred): each thread also folds
// its stored (bf16-rounded) dx values with the norm input h at the same position and the forward's
// keep bits into per-channel sums of dnorm and dnorm * xhat (the expressions of norm_fast.hip
// bn_reduce_fast); per block one [3][C] partial (slots 1, 2).
struct ThinBnr {
  const void* x;                    // the norm input h (the dgrad's dtype)
  const uint8_t* keep;
  const float *mean, *invstd, *gamma, *beta;
  float scale, slope;
  int dfirst, drop;
  float* part;
};

// T = bf16 or float (round 4: the fp32 parity mode too; a lane owns 8 channels either way)
template <typename T, int RS>
__global__ void __launch_bounds__(NT) k1_dgrad_bnred(Thin t, int LP, ThinBnr b) {
  const es_conv_desc_t& d = t.d;
  t.M = thin_m(t);   // dynamic rows: the live images' pixels
  __shared__ float wf[1024];                                  // transposed to [R*S][C]
  __shared__ float r1[NT * 8], r2[NT * 8];
  for (int i = threadIdx.x; i < RS * d.C; i += NT) {
    const int c = i / RS, j = i % RS;
    wf[j * d.C + c] = to_f(((const T*)t.w)[i]);
  }
  const int PPB = NT / LP;
  const int l = threadIdx.x % LP;
  float mu[8], is[8], sc[8], sh[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = l * 8 + e;
    mu[e] = b.mean[c];
    is[e] = b.invstd[c];
    sc[e] = (b.gamma ? b.gamma[c] : 1.f) * is[e];
    sh[e] = (b.beta ? b.beta[c] : 0.f) - mu[e] * sc[e];
    s1[e] = s2[e] = 0.f;
  }
  __syncthreads();
  const float dsc = b.drop ? b.scale : 1.f;
  // two pixels per trip (their h / keep / dy loads issue together; the bf16 form was latency-bound)
  constexpr int U = 2;
  const int stride = gridDim.x * PPB;
  for (int m0 = blockIdx.x * PPB + threadIdx.x / LP; m0 < t.M; m0 += U * stride) {
    float hv[U][8], acc[U][8];
    uint32_t kb[U];
    int64_t off[U];
    bool lv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * stride;
      lv[u] = m < t.M;
      const int mc = lv[u] ? m : m0;
      int n, h, w;
      pix3(mc, d.H, d.W, n, h, w);
      const T* dy = (const T*)t.a + n * t.as[0];
      off[u] = n * t.os[0] + h * t.os[2] + w * t.os[3] + l * 8;
      ld8<T>((const T*)b.x + off[u], hv[u]);                  // issued before the tap loads' FMAs
      kb[u] = b.drop ? (uint32_t)b.keep[(int64_t)mc * (d.C / 8) + l] : 0xFFu;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[u][e] = 0.f;
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const int ph = h + d.pad - j / d.S, pw = w + d.pad - j % d.S;
        const bool ok = ph >= 0 && pw >= 0 && ph < d.P && pw < d.Q;
        const float gv = to_f(dy[ok ? ph * t.as[2] + pw * t.as[3] : 0]);
        const float g = ok ? gv : 0.f;
        const float* wr = wf + j * d.C + l * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[u][e] += g * wr[e];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!lv[u]) continue;
      st8<T>((T*)t.out + off[u], acc[u]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dv = std::is_same<T, bf16>::value ? (float)(bf16)acc[u][e] : acc[u][e], v = hv[u][e];   // the stored dx
        const bool keep = (kb[u] >> e) & 1u;
        const float z = v * sc[e] + sh[e];
        const float zs = b.drop && b.dfirst ? z * b.scale : z;
        const float dn = keep ? dv * (zs > 0.f ? 1.f : b.slope) * dsc : 0.f;
        s1[e] += dn;
        s2[e] += dn * ((v - mu[e]) * is[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    r1[e * NT + threadIdx.x] = s1[e];
    r2[e * NT + threadIdx.x] = s2[e];
  }
  __syncthreads();
  if (threadIdx.x < LP) {
    float* p = b.part + (int64_t)blockIdx.x * 3 * d.C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float a1 = 0.f, a2 = 0.f;
      for (int q = 0; q < PPB; ++q) {
        a1 += r1[e * NT + q * LP + threadIdx.x];
        a2 += r2[e * NT + q * LP + threadIdx.x];
      }
      const int c = threadIdx.x * 8 + e;
      p[c] = 0.f;
      p[d.C + c] = a1;
      p[2 * d.C + c] = a2;
    }
  }
}

// Input-major forms of the Cout == 1 forward and weight gradient.  The output-major kernels above
// read every input pixel once per tap (4x for 2x2 taps, through L2 / MALL) and ran at ~2.4 TB/s of
// unique input; these read each input pixel ONCE.
// fwd: one workgroup per image.  Per input pixel, the RS partial dots t_j = <x, w_j> (reduced over the
// LP lanes of the pixel) go to LDS; then y(p, q) = bias + sum_j t_j(p - pad + r_j, q - pad + s_j).
constexpr int K1_TP_FLOATS = 9216;   // LDS floats of the per-tap partial dots (RS * H * W)
template <typename T, typename TO, int RS>
__global__ void __launch_bounds__(NT) k1_fwd_img(Thin t, int LP) {
  constexpr int VN = V16<T>::N;
  const es_conv_desc_t& d = t.d;
  const int n = blockIdx.x;
  if (n >= live_rows(d.rows, d.N)) return;   // dynamic rows: a padding image
  __shared__ float wf[1024];                 // [R][S][C]
  __shared__ float tp[K1_TP_FLOATS];         // [RS][H * W]
  for (int i = threadIdx.x; i < RS * d.C; i += NT) wf[i] = to_f(((const T*)t.w)[i]);
  __syncthreads();
  const int HW = d.H * d.W, PPB = NT / LP, l = threadIdx.x % LP;
  const T* xn = (const T*)t.a + n * t.as[0] + l * VN;
  constexpr int U = 4;                       // four pixels per trip: their loads issue together
  for (int m0 = 0; m0 < HW; m0 += U * PPB) {
    float v[U][VN];
    int mm[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = m0 + u * PPB + threadIdx.x / LP;
      mm[u] = m;
      const int mc = m < HW ? m : 0;
      const int h = mc / d.W, w = mc - h * d.W;
      const T* px = xn + h * t.as[2] + w * t.as[3];
      if constexpr (VN == 8) {
        ld8<T>(px, v[u]);
      } else {
        const float4 q4 = *(const float4*)px;
        v[u][0] = q4.x; v[u][1] = q4.y; v[u][2] = q4.z; v[u][3] = q4.w;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s[RS];
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const float* wr = wf + j * d.C + l * VN;
        float a = 0.f;
#pragma unroll
        for (int e = 0; e < VN; ++e) a += v[u][e] * wr[e];
        s[j] = a;
      }
      for (int o = LP >> 1; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < RS; ++j) s[j] += __shfl_xor(s[j], o, 64);
      if (l == 0 && mm[u] < HW)
#pragma unroll
        for (int j = 0; j < RS; ++j) tp[j * HW + mm[u]] = s[j];
    }
  }
  __syncthreads();
  const float b0 = t.bias ? t.bias[0] : 0.f;
  TO* yn = (TO*)t.out + n * t.os[0];
  for (int o = threadIdx.x; o < d.P * d.Q; o += NT) {
    const int p = o / d.Q, q = o - p * d.Q;
    float y = 0.f;
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      const int h = p - d.pad + j / d.S, w = q - d.pad + j % d.S;
      if ((unsigned)h < (unsigned)d.H && (unsigned)w < (unsigned)d.W) y += tp[j * HW + h * d.W + w];
    }
    yn[p * t.os[2] + q * t.os[3]] = from_f<TO>(y + b0);
  }
}

// wgrad: dw[r][s][c] = sum over input pixels (h, w) of x[h][w][c] * dy[h + pad - r][w + pad - s]
// (the dy values are 4-byte L2 hits; x is streamed once, 16-byte chunks)
template <typename T, int RS, int CH = 1>
__global__ void __launch_bounds__(NT) k1_wgrad_in(Thin t, int LP) {
  constexpr int VN = V16<T>::N, VC = VN * CH;
  const es_conv_desc_t& d = t.d;
  const int Mi = live_rows(d.rows, d.N) * d.H * d.W;   // the live images' input pixels
  const int PPB = NT / LP;
  const int l = threadIdx.x % LP;
  float acc[RS][VC];
#pragma unroll
  for (int j = 0; j < RS; ++j)
#pragma unroll
    for (int e = 0; e < VC; ++e) acc[j][e] = 0.f;
  constexpr int U = CH > 1 ? 2 : 4;
  const int stride = gridDim.x * PPB;
  for (int m0 = blockIdx.x * PPB + threadIdx.x / LP; m0 < Mi; m0 += U * stride) {
    float g[U][RS];
    float v[U][VC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int mu = m0 + u * stride;
      const bool live = mu < Mi;
      int n, h, w;
      pix3(live ? mu : m0, d.H, d.W, n, h, w);
      const T* px = (const T*)t.b + n * t.bs[0] + h * t.bs[2] + w * t.bs[3] + l * VC;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if constexpr (VN == 8) {
          ld8<T>(px + c * VN, &v[u][c * VN]);
        } else {
          const float4 q4 = *(const float4*)(px + c * VN);
          v[u][c * 4 + 0] = q4.x; v[u][c * 4 + 1] = q4.y; v[u][c * 4 + 2] = q4.z; v[u][c * 4 + 3] = q4.w;
        }
      }
      const T* dyn = (const T*)t.a + n * t.as[0];
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const int p = h + d.pad - j / d.S, q = w + d.pad - j % d.S;
        const bool ok = live && (unsigned)p < (unsigned)d.P && (unsigned)q < (unsigned)d.Q;
        const float gv = to_f(dyn[ok ? p * t.as[2] + q * t.as[3] : 0]);   // clamped: loads issue together
        g[u][j] = ok ? gv : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < RS; ++j)
#pragma unroll
        for (int e = 0; e < VC; ++e) acc[j][e] += g[u][j] * v[u][e];
  }
#pragma unroll
  for (int j = 0; j < RS; ++j)
#pragma unroll
    for (int e = 0; e < VC; ++e)
      for (int o = LP; o < 64; o <<= 1) acc[j][e] += __shfl_xor(acc[j][e], o, 64);
  __shared__ float red[4][1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane < LP) {
#pragma unroll
    for (int j = 0; j < RS; ++j)
#pragma unroll
      for (int e = 0; e < VC; ++e) red[wid][j * d.C + l * VC + e] = acc[j][e];
  }
  __syncthreads();
  float* dw = (float*)t.out;
  if (t.det) {
    for (int i = threadIdx.x; i < RS * d.C; i += NT)
      dw[(int64_t)blockIdx.x * RS * d.C + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  } else {
    for (int i = threadIdx.x; i < RS * d.C; i += NT)
      atomicAdd(&dw[i], red[0][i] + red[1][i] + red[2][i] + red[3][i]);
  }
}

// ============================================================ small fp32 convs (few channels)
// The discriminator's conv_layers.4 (32 -> 16, 3x3, fp32: neutron/discriminator.py:16): as a GEMM
// its N = 16 fills a quarter of every tile.  Direct forward: one thread per output pixel with KO
// accumulators, weights in LDS.  (A direct dgrad measured slower than the GEMM; not used.)
// CC > 0: the channel count is a compile-time constant, so each tap's CC/4 float4 loads are issued
// together before its FMAs (the runtime-C loop waited on one load per 4 channels: 72 dependent
// global round trips per thread, 69 us per call at B = 512; latency-bound, not FMA-bound).
template <int KO, int CC>
__global__ void __launch_bounds__(NT) small_fwd(Thin t) {
  const es_conv_desc_t& d = t.d;
  t.M = thin_m(t);   // dynamic rows: the live images' pixels
  const int RS = d.R * d.S, C = CC > 0 ? CC : d.C;
  __shared__ float wf[9 * 64 * KO];                       // [rs][c][k]
  __shared__ float bs[KO];
  for (int i = threadIdx.x; i < KO * RS * C; i += NT) {   // packed wk = [k][rs][c]
    const int k = i / (RS * C), rc = i - k * (RS * C);
    wf[rc * KO + k] = ((const float*)t.w)[i];
  }
  if (threadIdx.x < KO) bs[threadIdx.x] = t.bias ? t.bias[threadIdx.x] : 0.f;
  __syncthreads();
  const int m = blockIdx.x * NT + threadIdx.x;
  if (m >= t.M) return;
  int n, p, q;
  pix3(m, d.P, d.Q, n, p, q);
  float acc[KO];
#pragma unroll
  for (int k = 0; k < KO; ++k) acc[k] = bs[k];
  const float* x = (const float*)t.a + n * t.as[0];
  for (int r = 0; r < d.R; ++r) {
    const int hu = p - d.pad + r;
    if (hu < 0 || hu >= d.H) continue;
    for (int s_ = 0; s_ < d.S; ++s_) {
      const int wu = q - d.pad + s_;
      if (wu < 0 || wu >= d.W) continue;
      const float* px = x + hu * t.as[2] + wu * t.as[3];
      const float* wr = wf + (r * d.S + s_) * C * KO;
      if constexpr (CC > 0) {
        float4 xv[CC / 4];
#pragma unroll
        for (int c4 = 0; c4 < CC / 4; ++c4) xv[c4] = *(const float4*)(px + 4 * c4);
#pragma unroll
        for (int c4 = 0; c4 < CC / 4; ++c4) {
          const float xs[4] = {xv[c4].x, xv[c4].y, xv[c4].z, xv[c4].w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int k = 0; k < KO; ++k) acc[k] += xs[e] * wr[(4 * c4 + e) * KO + k];
        }
      } else {
        for (int c = 0; c < C; c += 4) {
          const float4 xv = *(const float4*)(px + c);
          const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int k = 0; k < KO; ++k) acc[k] += xs[e] * wr[(c + e) * KO + k];
        }
      }
    }
  }
  float* y = (float*)t.out + n * t.os[0] + p * t.os[2] + q * t.os[3];
#pragma unroll
  for (int k = 0; k < KO; k += 4) *(float4*)(y + k) = make_float4(acc[k], acc[k + 1], acc[k + 2], acc[k + 3]);
}

bool plain(const es_conv_desc_t* d) {
  return d->hmap == nullptr && d->up_h <= 0 && d->Hu == d->H && d->Wu == d->W;
}
bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }
// every row start of a channels-last view is a multiple of v elements (vector loads / stores)
bool aligned(const int64_t s[4], int v) { return s[0] % v == 0 && s[2] % v == 0 && s[3] % v == 0; }

// Cin == 1 path: K % 8 == 0, K <= 64, stride 1 or 2, R*S in {4, 9}
bool c1_ok(const es_conv_desc_t* d, int rs) {
  return plain(d) && d->C == 1 && d->K % 8 == 0 && pow2(d->K) && d->K <= 64 && (d->stride == 1 || d->stride == 2) &&
         (rs == 4 || rs == 9);
}
// Cout == 1 path: stride 1, C / VN lanes per pixel dividing 64, R*S in {4, 9}, R*S*C <= 4096
bool k1_ok(const es_conv_desc_t* d, int rs, int vn) {
  return plain(d) && d->K == 1 && d->stride == 1 && d->C % vn == 0 && pow2(d->C / vn) && d->C / vn <= 64 &&
         (rs == 4 || rs == 9) && rs * d->C <= 1024;
}

unsigned blocks(int64_t items, int per) { return (unsigned)((items + per - 1) / per); }
// grid caps of the grid-stride thin kernels (re-measured round 4, kept)
constexpr int K1_GRID = 2048, THIN_WGRID = 1024, C1_GRID = 2048;
unsigned capped(unsigned b, int cap) { return cap > 0 ? std::min<unsigned>(b, (unsigned)cap) : b; }

// channel chunks per lane of the Cout == 1 kernels: 1 = one 16-byte chunk per lane (C / VN lanes per
// pixel); 2 / 4 = fewer lanes per pixel, more loads in flight per lane, fewer shuffle rounds.  Measured
// on conv_layers.13 at B = 1024 fp32 (us, CH = 1 / 2 / 4): fwd 241 / 226 / 414, dgrad 218 / 323 / 586,
// wgrad 207 / 169 / 197 (output-major kernels) -> fwd 2 (the output-major fallback), dgrad 1, wgrad 2.
// The input-major kernels (round 5, conv_layers.13 at B = 1024, us fp32 / bf16): fwd 236 / 91 -> 156 / 82
// (one workgroup per image, 4 pixels per trip); wgrad 170 / 159 -> 132 / 87 at CH = 2 with 2 pixels
// per trip (CH = 1 with 4 pixels per trip: 171 / 106)
constexpr int K1_CH = 2, K1_CH_DG = 1, K1_CH_WG = 2;
// CH usable for C / VN chunks (LP = chunks / CH >= 1, a power of two)
int k1_ch(int chunks, int want) {
  int ch = want == 4 || want == 2 ? want : 1;
  while (ch > 1 && chunks % ch) ch >>= 1;
  return ch;
}
#define ES_K1_CH_DISPATCH(CHV, BODY)                                             \
  do {                                                                          \
    if ((CHV) == 4) { constexpr int CH = 4; BODY; }                             \
    else if ((CHV) == 2) { constexpr int CH = 2; BODY; }                        \
    else { constexpr int CH = 1; BODY; }                                        \
  } while (0)

template <typename T, typename TO>
void launch_fwd(const Thin& t, int rs, int LP, hipStream_t st) {
  const es_conv_desc_t& d = t.d;
  if (d.C == 1) {
    const dim3 grid(capped(blocks(t.M, NT / (d.K / (16 / (int)sizeof(TO)))), C1_GRID));
    if (rs == 4) hipLaunchKernelGGL((c1_fwd<T, TO, 4>), grid, dim3(NT), 0, st, t);
    else hipLaunchKernelGGL((c1_fwd<T, TO, 9>), grid, dim3(NT), 0, st, t);
  } else if (rs == 4 && rs * d.H * d.W <= K1_TP_FLOATS && pow2(LP) && LP <= 64) {
    hipLaunchKernelGGL((k1_fwd_img<T, TO, 4>), dim3(d.N), dim3(NT), 0, st, t, LP);
  } else {
    const int ch = k1_ch(LP, K1_CH), lp = LP / ch;
    const dim3 grid(capped(blocks(t.M, NT / lp), K1_GRID));
    ES_K1_CH_DISPATCH(ch, {
      if (rs == 4) hipLaunchKernelGGL((k1_fwd<T, TO, 4, CH>), grid, dim3(NT), 0, st, t, lp);
      else hipLaunchKernelGGL((k1_fwd<T, TO, 9, CH>), grid, dim3(NT), 0, st, t, lp);
    });
  }
}

template <typename T, typename TO>
void launch_dgrad(const Thin& t, int rs, int LP, hipStream_t st) {
  const es_conv_desc_t& d = t.d;
  if (d.C == 1 && d.stride == 1 && rs * d.P * d.Q <= C1_TP_FLOATS) {
    if (rs == 4) hipLaunchKernelGGL((c1_dgrad_img<T, TO, 4>), dim3(d.N), dim3(NT), 0, st, t);
    else hipLaunchKernelGGL((c1_dgrad_img<T, TO, 9>), dim3(d.N), dim3(NT), 0, st, t);
  } else if (d.C == 1) {
    const dim3 grid(blocks(t.M, NT / (d.K / V16<T>::N)));
    if (rs == 4) hipLaunchKernelGGL((c1_dgrad<T, TO, 4>), grid, dim3(NT), 0, st, t);
    else hipLaunchKernelGGL((c1_dgrad<T, TO, 9>), grid, dim3(NT), 0, st, t);
  } else {
    const int ch = k1_ch(LP, K1_CH_DG), lp = LP / ch;
    const dim3 grid(capped(blocks(t.M, NT / lp), K1_GRID));
    ES_K1_CH_DISPATCH(ch, {
      if (rs == 4) hipLaunchKernelGGL((k1_dgrad<T, TO, 4, CH>), grid, dim3(NT), 0, st, t, lp);
      else hipLaunchKernelGGL((k1_dgrad<T, TO, 9, CH>), grid, dim3(NT), 0, st, t, lp);
    });
  }
}

template <typename T>
void launch_wgrad(const Thin& t, int rs, int LP, hipStream_t st) {
  const es_conv_desc_t& d = t.d;
  const int ch = d.C == 1 ? 1 : k1_ch(LP, K1_CH_WG), lp = d.C == 1 ? LP : LP / ch;
  // ~4 blocks per CU, each reducing a strided slice of the pixels
  const int per = d.C == 1 ? NT / (d.K / 8) : NT / lp;
  dim3 grid(capped(blocks(t.M, per), THIN_WGRID));
  if (t.det) {   // deterministic mode: one partial slot per block within the caller's workspace
    const int64_t slot = (int64_t)d.K * rs * d.C;
    grid.x = (unsigned)std::max<int64_t>(1, std::min<int64_t>(grid.x, g_det_req.floats / slot));
    g_det_req.splits = (int)grid.x;
  }
  if (d.C == 1) {
    if (rs == 4) hipLaunchKernelGGL((c1_wgrad<T, 4>), grid, dim3(NT), 0, st, t);
    else hipLaunchKernelGGL((c1_wgrad<T, 9>), grid, dim3(NT), 0, st, t);
  } else {
    ES_K1_CH_DISPATCH(ch, {
      if (rs == 4) hipLaunchKernelGGL((k1_wgrad_in<T, 4, CH>), grid, dim3(NT), 0, st, t, lp);
      else hipLaunchKernelGGL((k1_wgrad_in<T, 9, CH>), grid, dim3(NT), 0, st, t, lp);
    });
  }
}

}  // namespace

// fp32, stride 1, no upsample, K in {4, 8, 16}, C % 8 == 0, C <= 64, R*S <= 9, dense NHWC rows
bool small_ok(const es_conv_desc_t* d, es_dtype_t dt) {
  return dt == ES_F32 && plain(d) && d->stride == 1 && (d->K == 4 || d->K == 8 || d->K == 16) && d->C % 8 == 0 &&
         d->C <= 64 && d->R * d->S <= 9 && d->C > 1;
}
template <typename F>
void small_dispatch(int K, F&& f) {
  if (K == 4) f(std::integral_constant<int, 4>{});
  else if (K == 8) f(std::integral_constant<int, 8>{});
  else f(std::integral_constant<int, 16>{});
}

// ------------------------------------------------------------------------------- entry points
// Each returns 1 if it launched (caller checks the launch), 0 if the shape is not a thin conv.
int es_thin_conv_fwd(const es_conv_desc_t* d, es_dtype_t dt, const void* x, const int64_t xs[4], const void* wk,
                     const float* bias, void* y, es_dtype_t ydt, const int64_t ys[4], hipStream_t st) {
  const int rs = d->R * d->S, vn = dt == ES_BF16 ? 8 : 4;
  const bool c1 = c1_ok(d, rs) && ys[1] == 1 && aligned(ys, 8);
  const bool k1 = k1_ok(d, rs, vn) && xs[1] == 1 && xs[3] == d->C && aligned(xs, vn);
  if (!c1 && !k1 && small_ok(d, dt) && ydt == ES_F32 && xs[1] == 1 && aligned(xs, 4) && ys[1] == 1 &&
      aligned(ys, 4)) {
    Thin t{};
    t.d = *d; t.a = x; t.w = wk; t.bias = bias; t.out = y;
    for (int i = 0; i < 4; ++i) { t.as[i] = xs[i]; t.os[i] = ys[i]; }
    t.M = d->N * d->P * d->Q;
    small_dispatch(d->K, [&](auto ko) {
      constexpr int KO = decltype(ko)::value;
      if (d->C == 32)
        hipLaunchKernelGGL((small_fwd<KO, 32>), dim3(blocks(t.M, NT)), dim3(NT), 0, st, t);
      else
        hipLaunchKernelGGL((small_fwd<KO, 0>), dim3(blocks(t.M, NT)), dim3(NT), 0, st, t);
    });
    return 1;
  }
  if (!c1 && !k1) return 0;
  Thin t{};
  t.d = *d; t.a = x; t.w = wk; t.bias = bias; t.out = y;
  for (int i = 0; i < 4; ++i) { t.as[i] = xs[i]; t.os[i] = ys[i]; }
  t.M = d->N * d->P * d->Q;
  const int LP = k1 ? d->C / vn : 1;
  if (dt == ES_BF16) {
    if (ydt == ES_BF16) launch_fwd<bf16, bf16>(t, rs, LP, st); else launch_fwd<bf16, float>(t, rs, LP, st);
  } else {
    if (ydt == ES_BF16) launch_fwd<float, bf16>(t, rs, LP, st); else launch_fwd<float, float>(t, rs, LP, st);
  }
  return 1;
}

int es_thin_conv_dgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                       const void* wd, void* dx, es_dtype_t dxdt, const int64_t dxs[4], float beta,
                       hipStream_t st) {
  const int rs = d->R * d->S, vn = dt == ES_BF16 ? 8 : 4;
  const bool c1 = c1_ok(d, rs) && ys[1] == 1 && aligned(ys, 8);
  const bool k1 = k1_ok(d, rs, vn) && dxs[1] == 1 && dxs[3] == d->C && aligned(dxs, vn);
  if (!c1 && !k1) return 0;
  Thin t{};
  t.d = *d; t.a = dy; t.w = wd; t.out = dx; t.beta = beta;
  for (int i = 0; i < 4; ++i) { t.as[i] = ys[i]; t.os[i] = dxs[i]; }
  t.M = d->N * d->H * d->W;
  const int LP = k1 ? d->C / vn : 1;
  const BnRedRequest& q = g_bnr_req;
  const int lp8 = d->C / 8;   // the fused kernel's lanes per pixel: 8 channels per lane in both dtypes
  if (k1 && q.part && q.x && q.nm && q.ch && dt == dxdt && beta == 0.f && (rs == 4 || rs == 9) &&
      pow2(lp8) && lp8 <= 64 && d->C % 8 == 0 &&
      dxs[3] == d->C && dxs[2] == (int64_t)d->W * d->C && dxs[0] == (int64_t)d->H * d->W * d->C &&
      ((uintptr_t)q.x & 15) == 0 && (q.ch->act == ES_ACT_LRELU || q.ch->act == ES_ACT_RELU) &&
      (!q.ch->drop.enabled || q.ch->keep)) {
    const dim3 grid(capped(blocks(t.M, NT / lp8), K1_GRID));
    if ((int64_t)grid.x * 3 * d->C <= q.floats) {
      ThinBnr b{};
      b.x = q.x; b.keep = q.ch->keep;
      b.mean = q.nm->mean; b.invstd = q.nm->invstd; b.gamma = q.nm->gamma; b.beta = q.nm->beta;
      b.drop = q.ch->drop.enabled != 0;
      b.scale = b.drop ? q.ch->drop.scale : 1.f;
      b.dfirst = q.ch->dropout_first;
      b.slope = q.ch->act == ES_ACT_LRELU ? q.ch->slope : 0.f;
      b.part = q.part;
      if (dt == ES_BF16) {
        if (rs == 4) hipLaunchKernelGGL((k1_dgrad_bnred<bf16, 4>), grid, dim3(NT), 0, st, t, lp8, b);
        else hipLaunchKernelGGL((k1_dgrad_bnred<bf16, 9>), grid, dim3(NT), 0, st, t, lp8, b);
      } else {
        if (rs == 4) hipLaunchKernelGGL((k1_dgrad_bnred<float, 4>), grid, dim3(NT), 0, st, t, lp8, b);
        else hipLaunchKernelGGL((k1_dgrad_bnred<float, 9>), grid, dim3(NT), 0, st, t, lp8, b);
      }
      g_bnr_req.chunks = (int)grid.x;
      return 1;
    }
  }
  if (dt == ES_BF16) {
    if (dxdt == ES_BF16) launch_dgrad<bf16, bf16>(t, rs, LP, st); else launch_dgrad<bf16, float>(t, rs, LP, st);
  } else {
    if (dxdt == ES_BF16) launch_dgrad<float, bf16>(t, rs, LP, st); else launch_dgrad<float, float>(t, rs, LP, st);
  }
  return 1;
}

int es_thin_conv_wgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4], const void* x,
                       const int64_t xs[4], float* dw, hipStream_t st) {
  const int rs = d->R * d->S, vn = dt == ES_BF16 ? 8 : 4;
  const bool c1 = c1_ok(d, rs) && ys[1] == 1 && aligned(ys, 8) && pow2(d->K / 8) && d->K / 8 <= 8;
  const bool k1 = k1_ok(d, rs, vn) && xs[1] == 1 && xs[3] == d->C && aligned(xs, vn);
  if (!c1 && !k1) return 0;
  Thin t{};
  t.d = *d; t.a = dy; t.b = x; t.out = dw;
  for (int i = 0; i < 4; ++i) { t.as[i] = ys[i]; t.bs[i] = xs[i]; }
  t.M = d->N * d->P * d->Q;
  t.det = g_det_req.ws != nullptr && (float*)dw == g_det_req.ws;
  const int LP = k1 ? d->C / vn : 1;
  if (dt == ES_BF16) launch_wgrad<bf16>(t, rs, LP, st);
  else launch_wgrad<float>(t, rs, LP, st);
  return 1;
}
