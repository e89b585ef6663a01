// Fast path of the BatchNorm / GroupNorm + dropout + activation pipeline for dense channels-last
// tensors.
//
// Covers every BatchNorm of the neutron generator and aux regressor (neutron/generator.py:13,19,
// 26,31,35; neutron/aux_reg.py:15,23,31,39,47) and the GroupNorms of the discriminators and the
// proton generator (neutron/discriminator.py:13,18; proton/generator.py:28,34,39) when x, y / dy,
// dx are NHWC-dense ([rows][C], rows = N*H*W) of one dtype and C % 8 == 0.  GroupNorm runs the
// same kernels with blockIdx.z = sample n: a block then covers the H*W rows of one sample, its
// statistics are indexed (n, c / (C/G)), and per-(n, c) partials are merged per group.  Layout of the work: a thread owns 8 consecutive
// channels (one 16-byte bf16 / 32-byte fp32 vector) of 4 consecutive rows, so
//   * no per-element index division (one division per 4 rows),
//   * 16-byte vector loads and stores,
//   * one Philox4x32 call serves the 4 rows of a channel when H*W % 4 == 0 (the 4 rows then hold
//     the 4 consecutive NCHW-logical indices that share a Philox counter), or 4 channels of a row
//     when H*W == 1 (linear BatchNorm1d) — instead of one call per element.
// Statistics / backward sums are reduced per block in LDS into [chunk][3][C] partials that the
// finalize kernels of norm.hip merge.
#include "common.h"

namespace {

typedef unsigned int nt_u32x4 __attribute__((ext_vector_type(4)));
template <typename T> __device__ __forceinline__ void ld8(const T* p, float* f);
template <> __device__ __forceinline__ void ld8<bf16>(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = (float)v[k];
}
// The backward passes stream x and dy once each: non-temporal loads (measured on the c5 BatchNorm,
// 277 MB bf16: reduce + apply 317 -> 292 us).  The Welford stats pass keeps temporal loads (its
// input is usually still partly cached from the producing conv; NT loads measured slower there).
template <typename T> __device__ __forceinline__ void ld8nt(const T* p, float* f) { ld8<T>(p, f); }
template <> __device__ __forceinline__ void ld8nt<bf16>(const bf16* p, float* f) {
  const nt_u32x4 w = __builtin_nontemporal_load((const nt_u32x4*)p);
#pragma unroll
  for (int k = 0; k < 4; ++k) {          // little-endian pairs: element 2k is the low half
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
  }
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
  __builtin_nontemporal_store(*(const nt_u32x4*)&v, (nt_u32x4*)p);   // outputs are not re-read soon
}
// (fp32: plain stores; non-temporal fp32 loads / stores measured 2-10 % slower)
template <> __device__ __forceinline__ void st8<float>(float* p, const float* f) {
  ((float4*)p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  ((float4*)p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

struct FastArgs {
  const void* x; const void* dy; void* out;   // out: y (fwd) or dx (bwd apply)
  int rows, C, HW;
  int G, cg, zrows;                           // GroupNorm: G groups of cg channels, zrows = HW; BN: G = 0
  const float *mean, *invstd, *gamma, *beta;
  const float *a1, *a2;                       // bwd apply: per-channel gamma*mean(dnorm), gamma*mean(dnorm*xhat)
  float* part;                                // [chunk][3][C] partials (stats / bwd sums)
  float* dsum;                                // bwd apply: per-channel sum of dx (conv-bias gradient)
  es_dropout_t drop;
  int dfirst, act;
  float slope;
  uint8_t* keep;                              // dropout keep bits [rows][C/8] (written fwd, read bwd)
  const int32_t* nrows;                       // dynamic rows: device count of the live samples (es_view_t.rows)
};

__device__ __forceinline__ float actf(const FastArgs& a, float v) {
  return a.act == ES_ACT_RELU ? fmaxf(v, 0.f) : (a.act == ES_ACT_LRELU ? lrelu(v, a.slope) : v);
}
__device__ __forceinline__ float dactf(const FastArgs& a, float v) {
  return a.act == ES_ACT_RELU ? (v > 0.f ? 1.f : 0.f) : (a.act == ES_ACT_LRELU ? (v > 0.f ? 1.f : a.slope) : 1.f);
}

// keep bits for rows r0..r0+3 (bit k = channel c0+k)
// KM (keep mode, chosen on the host): KM_NONE no dropout, KM_HW4 H*W % 4 == 0, KM_ROW H*W == 1 and
// C % 4 == 0, KM_GEN anything else.  One instantiation per mode keeps each kernel's code small.
// KM_BITS: read the bits a forward pass stored in a.keep (no Philox).
enum { KM_NONE = 0, KM_HW4 = 1, KM_ROW = 2, KM_GEN = 3, KM_BITS = 4 };

__device__ __forceinline__ uint32_t keep4(const u32x4 w, uint32_t thr) {
  return (uint32_t)((w.x >> 8) < thr) | ((uint32_t)((w.y >> 8) < thr) << 1) |
         ((uint32_t)((w.z >> 8) < thr) << 2) | ((uint32_t)((w.w >> 8) < thr) << 3);
}

// KM_GEN (H*W % 4 != 0) with the wave's counters shared, for C <= 64 (8 or more row groups per
// wave, e.g. conv_layers.9's 45 x 45 x 64 output).  The 4 rows of a lane's group span two Philox
// counters per channel when i0 % 4 != 0; the second one is the FIRST counter of the same channel in
// the next row group, which the lane TCV above computes anyway.  The wave's last row group has no
// such neighbour, so its 8 second counters are computed one per row group of the wave (channel k
// by row group k) and gathered by shuffles: 9 calls per lane for every lane, instead of 8 plus a
// second call per misaligned channel (1.75 per channel on average), which SIMT execution ran for
// the whole wave whenever one lane needed it.  Returns false (nothing written) when the layout does
// not apply; lanes whose 4 rows straddle a sample, or whose neighbour does, compute their own.
__device__ __forceinline__ bool keep_bits_gen_shared(const FastArgs& a, int r0, int c0, uint32_t thr,
                                                     uint32_t k0, uint32_t k1, uint32_t (&keep)[4]) {
#if defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
  return false;   // the row-group / shuffle arithmetic below is for 64-lane waves (gfx950)
#endif
  const int tcv = min(a.C >> 3, 64);
  if (64 % tcv != 0 || 64 / tcv < 8) return false;          // uniform over the launch
  const int lane = threadIdx.x & 63, rgw = lane / tcv, cvl = lane - rgw * tcv, RGW = 64 / tcv;
  const bool in1 = r0 - (r0 / a.HW) * a.HW + 3 < a.HW && r0 + 3 < a.rows;
  uint64_t i00 = ~0ull;          // logical index of (row r0, channel c0); sentinel: not in1
  uint32_t m0 = 0;               // first-counter bits, 4 per channel
  if (in1) {
    const int n = r0 / a.HW, hw0 = r0 - n * a.HW;
    i00 = ((uint64_t)n * a.C + c0) * (uint64_t)a.HW + hw0 + a.drop.index_offset;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t q = (i00 + (uint64_t)k * a.HW) >> 2;
      m0 |= keep4(philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), a.drop.stream, 0u, k0, k1), thr) << (4 * k);
    }
  }
  // the last row group's second counter of channel k = rgw (its index read from that lane; a
  // sentinel or stale index only feeds bits that lane does not use)
  const int last = (RGW - 1) * tcv + cvl;
  const uint64_t il = ((uint64_t)__shfl((uint32_t)(i00 >> 32), last, 64) << 32) | __shfl((uint32_t)i00, last, 64);
  uint32_t xb = 0;
  if (rgw < 8) {
    const uint64_t q = ((il + (uint64_t)rgw * a.HW) >> 2) + 1;
    xb = keep4(philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), a.drop.stream, 0u, k0, k1), thr);
  }
  uint32_t lx = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) lx |= (__shfl(xb, k * tcv + cvl, 64) & 15u) << (4 * k);
  // the next row group's first counters (lane + tcv), checked by its logical index
  const uint32_t nb_m = __shfl_down(m0, tcv, 64);
  const uint64_t inb = ((uint64_t)__shfl_down((uint32_t)(i00 >> 32), tcv, 64) << 32) |
                       __shfl_down((uint32_t)i00, tcv, 64);
  if (!in1) return false;
  const bool nb_ok = rgw < RGW - 1 && inb == i00 + 4;
  const bool last_ok = rgw == RGW - 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t i0 = i00 + (uint64_t)k * a.HW;
    const int off = (int)(i0 & 3);
    uint32_t m = (m0 >> (4 * k)) & 15u;
    if (off) {
      uint32_t m1;
      if (nb_ok) {
        m1 = (nb_m >> (4 * k)) & 15u;
      } else if (last_ok) {
        m1 = (lx >> (4 * k)) & 15u;
      } else {
        const uint64_t q1 = (i0 >> 2) + 1;
        m1 = keep4(philox4x32_10((uint32_t)q1, (uint32_t)(q1 >> 32), a.drop.stream, 0u, k0, k1), thr);
      }
      m |= m1 << 4;
    }
    m >>= off;
    keep[0] |= (m & 1u) << k;
    keep[1] |= ((m >> 1) & 1u) << k;
    keep[2] |= ((m >> 2) & 1u) << k;
    keep[3] |= ((m >> 3) & 1u) << k;
  }
  return true;
}

template <int KM>
__device__ __forceinline__ void keep_bits(const FastArgs& a, int r0, int c0, uint32_t (&keep)[4]) {
  if constexpr (KM == KM_NONE) { keep[0] = keep[1] = keep[2] = keep[3] = 0xFFu; return; }
  if constexpr (KM == KM_BITS) {
    const int cb = a.C >> 3, cv = c0 >> 3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // clamped row, unconditional load (the 4 loads issue together)
      const bool in = r0 + j < a.rows;
      const uint32_t b = a.keep[(int64_t)(in ? r0 + j : r0) * cb + cv];
      keep[j] = in ? b : 0u;
    }
    return;
  }
  keep[0] = keep[1] = keep[2] = keep[3] = 0u;
  const uint32_t thr = a.drop.threshold;
  const uint32_t k0 = (uint32_t)a.drop.seed, k1 = (uint32_t)(a.drop.seed >> 32);
  if constexpr (KM == KM_HW4) {
    const int n = r0 / a.HW, hw0 = r0 - n * a.HW;     // r0 % 4 == 0 -> same n for the 4 rows
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t base = ((uint64_t)n * a.C + c0 + k) * (uint64_t)a.HW + hw0 + a.drop.index_offset;
      const uint64_t q = base >> 2;
      const u32x4 w = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), a.drop.stream, 0u, k0, k1);
      keep[0] |= (uint32_t)((w.x >> 8) < thr) << k;
      keep[1] |= (uint32_t)((w.y >> 8) < thr) << k;
      keep[2] |= (uint32_t)((w.z >> 8) < thr) << k;
      keep[3] |= (uint32_t)((w.w >> 8) < thr) << k;
    }
  } else if constexpr (KM == KM_ROW) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + j;
      if (r >= a.rows) break;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint64_t q = ((uint64_t)r * a.C + c0 + 4 * h + a.drop.index_offset) >> 2;
        const u32x4 w = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), a.drop.stream, 0u, k0, k1);
        keep[j] |= ((uint32_t)((w.x >> 8) < thr) | ((uint32_t)((w.y >> 8) < thr) << 1) |
                    ((uint32_t)((w.z >> 8) < thr) << 2) | ((uint32_t)((w.w >> 8) < thr) << 3)) << (4 * h);
      }
    }
  } else if (keep_bits_gen_shared(a, r0, c0, thr, k0, k1, keep)) {   // KM_GEN, <= 64 channels
    return;
  } else if (r0 - (r0 / a.HW) * a.HW + 3 < a.HW && r0 + 3 < a.rows) {   // KM_GEN
    // the 4 rows lie in one sample: their logical indices i0..i0+3 are consecutive and span at
    // most two Philox counters per channel (2 calls instead of 4)
    const int n = r0 / a.HW, hw0 = r0 - n * a.HW;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t i0 = ((uint64_t)n * a.C + c0 + k) * (uint64_t)a.HW + hw0 + a.drop.index_offset;
      const uint64_t q = i0 >> 2;
      const int off = (int)(i0 & 3);
      const u32x4 w = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), a.drop.stream, 0u, k0, k1);
      uint32_t m = (uint32_t)((w.x >> 8) < thr) | ((uint32_t)((w.y >> 8) < thr) << 1) |
                   ((uint32_t)((w.z >> 8) < thr) << 2) | ((uint32_t)((w.w >> 8) < thr) << 3);
      if (off) {
        const uint64_t q1 = q + 1;
        const u32x4 v = philox4x32_10((uint32_t)q1, (uint32_t)(q1 >> 32), a.drop.stream, 0u, k0, k1);
        m |= ((uint32_t)((v.x >> 8) < thr) << 4) | ((uint32_t)((v.y >> 8) < thr) << 5) |
             ((uint32_t)((v.z >> 8) < thr) << 6) | ((uint32_t)((v.w >> 8) < thr) << 7);
      }
      m >>= off;
      keep[0] |= (m & 1u) << k;
      keep[1] |= ((m >> 1) & 1u) << k;
      keep[2] |= ((m >> 2) & 1u) << k;
      keep[3] |= ((m >> 3) & 1u) << k;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + j;
      if (r >= a.rows) break;
      const int n = r / a.HW, hw = r - n * a.HW;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t i = ((uint64_t)n * a.C + c0 + k) * (uint64_t)a.HW + hw;
        keep[j] |= (uint32_t)((philox_word(a.drop.seed, a.drop.stream, i + a.drop.index_offset) >> 8) < thr) << k;
      }
    }
  }
}

// forward chain on a normalised value z with keep bit
__device__ __forceinline__ float chain_fwd(const FastArgs& a, float z, bool keep) {
  if (!a.drop.enabled) return actf(a, z);
  if (a.dfirst) return actf(a, keep ? z * a.drop.scale : 0.f);
  return keep ? actf(a, z) * a.drop.scale : 0.f;
}
// d out / d z
__device__ __forceinline__ float chain_bwd(const FastArgs& a, float z, float dout, bool keep) {
  if (!a.drop.enabled) return dout * dactf(a, z);
  if (!keep) return 0.f;
  if (a.dfirst) return dout * dactf(a, z * a.drop.scale) * a.drop.scale;
  return dout * a.drop.scale * dactf(a, z);
}

// Chain specialised at compile time (CH, from the launch's KM template argument): the generic
// chain branches on a.act / a.dfirst / a.drop.enabled per element, which left the Philox forward
// with ~1100 basic blocks; the specialised forms are the same expressions without the branches.
enum { CH_GEN = 0, CH_LRELU_DFIRST = 1, CH_LRELU_DLAST = 2 };
template <int CH, bool DROP>
__device__ __forceinline__ float chain_fwd_t(const FastArgs& a, float z, bool keep) {
  if constexpr (CH == CH_GEN) {
    return chain_fwd(a, z, keep);
  } else if constexpr (!DROP) {
    return lrelu(z, a.slope);
  } else if constexpr (CH == CH_LRELU_DFIRST) {
    return lrelu(keep ? z * a.drop.scale : 0.f, a.slope);
  } else {
    return keep ? lrelu(z, a.slope) * a.drop.scale : 0.f;
  }
}
template <int CH, bool DROP>
__device__ __forceinline__ float chain_bwd_t(const FastArgs& a, float z, float dout, bool keep) {
  if constexpr (CH == CH_GEN) {
    return chain_bwd(a, z, dout, keep);
  } else if constexpr (!DROP) {
    return dout * (z > 0.f ? 1.f : a.slope);
  } else if constexpr (CH == CH_LRELU_DFIRST) {
    if (!keep) return 0.f;
    return dout * (z * a.drop.scale > 0.f ? 1.f : a.slope) * a.drop.scale;
  } else {
    if (!keep) return 0.f;
    return dout * a.drop.scale * (z > 0.f ? 1.f : a.slope);
  }
}

__device__ __forceinline__ int pow2_ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

struct Geo {
  int CV, TCV, RGB, cv, rg, c0;
  int rbase, rlim;                            // rows of this block's z slice
  bool active;
  // index of the statistics of channel c (per channel for BN, per (n, group) for GN)
  __device__ __forceinline__ int sidx(const FastArgs& a, int c) const {
    return a.G ? (int)blockIdx.z * a.G + c / a.cg : c;
  }
};
__device__ __forceinline__ Geo geo(const FastArgs& a) {
  Geo g;
  g.CV = a.C >> 3;
  g.TCV = min(g.CV, 64);
  g.RGB = 256 / g.TCV;
  g.cv = blockIdx.x * g.TCV + (int)(threadIdx.x % g.TCV);
  g.rg = threadIdx.x / g.TCV;
  g.active = g.rg < g.RGB && g.cv < g.CV;
  g.c0 = g.cv * 8;
  g.rbase = (int)blockIdx.z * a.zrows;
  // rows of the live samples (a prefix: rows are sample-major); GN slices past them are empty
  const int rl = a.nrows ? live_rows(a.nrows, a.rows / a.HW) * a.HW : a.rows;
  g.rlim = min(rl, g.rbase + a.zrows);
  return g;
}

template <typename T, int KMC>
__global__ void __launch_bounds__(256) bn_fwd_fast(FastArgs a) {
  constexpr int KM = KMC & 15, CH = KMC >> 4;
  resolve_stream(a.drop);
  const Geo g = geo(a);
  if (!g.active) return;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = g.c0 + k, si = g.sidx(a, c);
    const float s = (a.gamma ? a.gamma[c] : 1.f) * a.invstd[si];
    sc[k] = s;
    sh[k] = (a.beta ? a.beta[c] : 0.f) - a.mean[si] * s;
  }
  const T* __restrict__ x = (const T*)a.x;
  T* __restrict__ y = (T*)a.out;
  const int ngroups = (g.rlim - g.rbase + 3) >> 2;
  for (int grp = blockIdx.y * g.RGB + g.rg; grp < ngroups; grp += gridDim.y * g.RGB) {
    const int r0 = g.rbase + grp * 4;
    const int nr = min(4, g.rlim - r0);
    float v[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)            // issue every load of the group before any store
      ld8<T>(x + (int64_t)(r0 + (j < nr ? j : 0)) * a.C + g.c0, v[j]);   // clamped: no branch per row
    uint32_t keep[4];
    keep_bits<KM>(a, r0, g.c0, keep);
    if (KM != KM_NONE && KM != KM_BITS && a.keep) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < nr) a.keep[(int64_t)(r0 + j) * (a.C >> 3) + g.cv] = (uint8_t)keep[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= nr) break;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        v[j][k] = chain_fwd_t<CH, KM != KM_NONE>(a, v[j][k] * sc[k] + sh[k], (keep[j] >> k) & 1u);
      st8<T>(y + (int64_t)(r0 + j) * a.C + g.c0, v[j]);
    }
  }
}

// MODE 0: Welford stats of x.  MODE 1: backward sums (sum dnorm, sum dnorm*xhat).
template <typename T, int MODE, int KMC>
__global__ void __launch_bounds__(256) bn_reduce_fast(FastArgs a) {
  constexpr int KM = KMC & 15, CH = KMC >> 4;
  resolve_stream(a.drop);
  const Geo g = geo(a);
  float s0[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s0[k] = s1[k] = s2[k] = 0.f;
  float sc[8], sh[8], mu[8], is[8];
  if (g.active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = g.c0 + k, si = g.sidx(a, c);
      if (MODE == 1) {
        mu[k] = a.mean[si]; is[k] = a.invstd[si];
        const float s = (a.gamma ? a.gamma[c] : 1.f) * is[k];
        sc[k] = s; sh[k] = (a.beta ? a.beta[c] : 0.f) - mu[k] * s;
      }
    }
    const T* __restrict__ x = (const T*)a.x;
    const T* __restrict__ dy = (const T*)a.dy;
    const int ngroups = (g.rlim - g.rbase + 3) >> 2;
    for (int grp = blockIdx.y * g.RGB + g.rg; grp < ngroups; grp += gridDim.y * g.RGB) {
      const int r0 = g.rbase + grp * 4;
      uint32_t keep[4];
      if (MODE == 1) keep_bits<KM>(a, r0, g.c0, keep);
      // every load of the group first (clamped rows; rows past the end are masked below): the
      // per-row guarded loads were serialised by a wait per row (~4 TB/s -> 5+)
      const int nr = min(4, g.rlim - r0);
      float vv[4][8], dd[4][8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rr = r0 + (j < nr ? j : 0);
        if (MODE == 1) {
          ld8nt<T>(x + (int64_t)rr * a.C + g.c0, vv[j]);
          ld8nt<T>(dy + (int64_t)rr * a.C + g.c0, dd[j]);
        } else {
          ld8<T>(x + (int64_t)rr * a.C + g.c0, vv[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nr) break;
        const float* v = vv[j];
        if (MODE == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            s0[k] += 1.f;
            const float d = v[k] - s1[k];
            s1[k] += d / s0[k];
            s2[k] += d * (v[k] - s1[k]);
          }
        } else {
          const float* d = dd[j];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float dn = chain_bwd_t<CH, KM != KM_NONE>(a, v[k] * sc[k] + sh[k], d[k], (keep[j] >> k) & 1u);
            const float xh = (v[k] - mu[k]) * is[k];
            s1[k] += dn;
            s2[k] += dn * xh;
          }
        }
      }
    }
  }
  // tree merge across the row groups (same channels) through LDS, [k][thread] layout
  __shared__ float l0[8 * 256], l1[8 * 256], l2[8 * 256];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    l0[k * 256 + threadIdx.x] = s0[k]; l1[k * 256 + threadIdx.x] = s1[k]; l2[k * 256 + threadIdx.x] = s2[k];
  }
  __syncthreads();
  for (int h = pow2_ceil(g.RGB) >> 1; h > 0; h >>= 1) {
    if (g.active && g.rg < h && g.rg + h < g.RGB) {
      const int o = threadIdx.x + h * g.TCV;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (MODE == 0) {
          const float nb = l0[k * 256 + o];
          if (nb > 0.f) {
            const float mb = l1[k * 256 + o], Mb = l2[k * 256 + o];
            const float nt = s0[k] + nb, dl = mb - s1[k], f = nb / nt;
            s1[k] += dl * f;
            s2[k] += Mb + dl * dl * s0[k] * f;
            s0[k] = nt;
          }
        } else {
          s1[k] += l1[k * 256 + o];
          s2[k] += l2[k * 256 + o];
        }
        l0[k * 256 + threadIdx.x] = s0[k]; l1[k * 256 + threadIdx.x] = s1[k]; l2[k * 256 + threadIdx.x] = s2[k];
      }
    }
    __syncthreads();
  }
  if (g.active && g.rg == 0) {
    float* p = a.part + ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * 3 * a.C;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      p[g.c0 + k] = s0[k]; p[a.C + g.c0 + k] = s1[k]; p[2 * a.C + g.c0 + k] = s2[k];
    }
  }
}

template <typename T, int KMC>
__global__ void __launch_bounds__(256) bn_bwd_apply_fast(FastArgs a) {
  constexpr int KM = KMC & 15, CH = KMC >> 4;
  resolve_stream(a.drop);
  const Geo g = geo(a);
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  if (g.active) {
    float mu[8], is[8], ga[8], be[8], c1[8], c2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = g.c0 + k, si = g.sidx(a, c);
      mu[k] = a.mean[si]; is[k] = a.invstd[si];
      ga[k] = a.gamma ? a.gamma[c] : 1.f;
      be[k] = a.beta ? a.beta[c] : 0.f;
      c1[k] = a.a1[si]; c2[k] = a.a2[si];
    }
    const T* __restrict__ x = (const T*)a.x;
    const T* __restrict__ dy = (const T*)a.dy;
    T* __restrict__ dx = (T*)a.out;
    const int ngroups = (g.rlim - g.rbase + 3) >> 2;
    for (int grp = blockIdx.y * g.RGB + g.rg; grp < ngroups; grp += gridDim.y * g.RGB) {
      const int r0 = g.rbase + grp * 4;
      const int nr = min(4, g.rlim - r0);
      float v[4][8], d[4][8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {        // every load of the group, unconditionally (clamped rows)
        const int rr = r0 + (j < nr ? j : 0);
        ld8nt<T>(x + (int64_t)rr * a.C + g.c0, v[j]);
        ld8nt<T>(dy + (int64_t)rr * a.C + g.c0, d[j]);
      }
      uint32_t keep[4];
      keep_bits<KM>(a, r0, g.c0, keep);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nr) break;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = (v[j][k] - mu[k]) * is[k];
          const float dn = chain_bwd_t<CH, KM != KM_NONE>(a, xh * ga[k] + be[k], d[j][k], (keep[j] >> k) & 1u);
          d[j][k] = is[k] * (dn * ga[k] - c1[k] - xh * c2[k]);
          acc[k] += d[j][k];
        }
        st8<T>(dx + (int64_t)(r0 + j) * a.C + g.c0, d[j]);
      }
    }
  }
  if (a.dsum) {
    // per-block channel sums of dx -> partials (s1 slot of [z][chunk][3][C]); the host merges
    // them into dsum (no same-address atomics from every block)
    __shared__ float l1[8 * 256];
#pragma unroll
    for (int k = 0; k < 8; ++k) l1[k * 256 + threadIdx.x] = acc[k];
    __syncthreads();
    for (int h = pow2_ceil(g.RGB) >> 1; h > 0; h >>= 1) {
      if (g.active && g.rg < h && g.rg + h < g.RGB) {
        const int o = threadIdx.x + h * g.TCV;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          acc[k] += l1[k * 256 + o];
          l1[k * 256 + threadIdx.x] = acc[k];
        }
      }
      __syncthreads();
    }
    if (g.active && g.rg == 0) {
      float* p = a.part + ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * 3 * a.C + a.C;
#pragma unroll
      for (int k = 0; k < 8; ++k) p[g.c0 + k] = acc[k];
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------- host dispatch
// Returns true when the fast path applies to these views (dense NHWC, same dtype, C % 8 == 0).
bool es_fast_dense_nhwc(const es_view_t* v) {
  const int64_t C = v->c, W = v->w, H = v->h;
  return v->c % 8 == 0 && v->s[1] == 1 && (W == 1 || v->s[3] == C) && (H == 1 || v->s[2] == W * C) &&
         (v->n == 1 || v->s[0] == H * W * C);
}

// G = 0: BatchNorm (one z slice over all rows); G > 0: GroupNorm (z = sample)
static void fast_geometry(const es_view_t* v, int G, dim3& grid, int& chunks) {
  const int CV = v->c / 8;
  const int TCV = CV < 64 ? CV : 64;
  const int RGB = 256 / TCV;
  const int gx = (CV + TCV - 1) / TCV;
  const int gz = G ? v->n : 1;
  const int64_t zrows = G ? (int64_t)v->h * v->w : (int64_t)v->n * v->h * v->w;
  const int64_t ngroups = (zrows + 3) / 4;
  int64_t gy = std::max<int64_t>(1, 2048 / ((int64_t)gx * gz));
  gy = std::min<int64_t>(gy, (ngroups + RGB - 1) / RGB);
  grid = dim3(gx, (unsigned)gy, gz);
  chunks = (int)gy;
}

int64_t es_fast_part_floats(const es_view_t* v, int G) {
  dim3 g; int chunks;
  fast_geometry(v, G, g, chunks);
  return (int64_t)g.z * chunks * 3 * v->c;
}

static int keep_mode(const FastArgs& a, bool read_bits = false) {
  if (!a.drop.enabled) return KM_NONE;
  if (read_bits && a.keep) return KM_BITS;
  const bool al4 = (a.drop.index_offset & 3) == 0;   // both fast modes need 4-aligned global indices
  if ((a.HW & 3) == 0 && al4) return KM_HW4;
  if (a.HW == 1 && (a.C & 3) == 0 && al4) return KM_ROW;
  return KM_GEN;
}
static int chain_kind(const FastArgs& a) {
  if (a.act != ES_ACT_LRELU) return CH_GEN;
  return a.dfirst ? CH_LRELU_DFIRST : CH_LRELU_DLAST;
}
#define ES_KM_LAUNCH(K, T, KMV, grid, st, a)                                                   \
  do {                                                                                      \
    const int ch_ = chain_kind(a);                                                          \
    if (ch_ == CH_LRELU_DFIRST) hipLaunchKernelGGL((K<T, (KMV) | (CH_LRELU_DFIRST << 4)>), grid, dim3(256), 0, st, a); \
    else if (ch_ == CH_LRELU_DLAST) hipLaunchKernelGGL((K<T, (KMV) | (CH_LRELU_DLAST << 4)>), grid, dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((K<T, KMV>), grid, dim3(256), 0, st, a);                        \
  } while (0)
#define ES_KM_DISPATCH(a, K, dt, grid, st, RB)                                             \
  do {                                                                                    \
    const int km_ = keep_mode(a, RB);                                                     \
    if (dt == ES_BF16) {                                                                  \
      if (km_ == KM_NONE) ES_KM_LAUNCH(K, bf16, KM_NONE, grid, st, a);                    \
      else if (km_ == KM_BITS) ES_KM_LAUNCH(K, bf16, KM_BITS, grid, st, a);               \
      else if (km_ == KM_HW4) ES_KM_LAUNCH(K, bf16, KM_HW4, grid, st, a);                 \
      else if (km_ == KM_ROW) ES_KM_LAUNCH(K, bf16, KM_ROW, grid, st, a);                 \
      else ES_KM_LAUNCH(K, bf16, KM_GEN, grid, st, a);                                    \
    } else {                                                                              \
      if (km_ == KM_NONE) ES_KM_LAUNCH(K, float, KM_NONE, grid, st, a);                   \
      else if (km_ == KM_BITS) ES_KM_LAUNCH(K, float, KM_BITS, grid, st, a);              \
      else if (km_ == KM_HW4) ES_KM_LAUNCH(K, float, KM_HW4, grid, st, a);                \
      else if (km_ == KM_ROW) ES_KM_LAUNCH(K, float, KM_ROW, grid, st, a);                \
      else ES_KM_LAUNCH(K, float, KM_GEN, grid, st, a);                                   \
    }                                                                                     \
  } while (0)
#define ES_KM_LAUNCH1(K, T, KMV, grid, st, a)                                                  \
  do {                                                                                      \
    const int ch_ = chain_kind(a);                                                          \
    if (ch_ == CH_LRELU_DFIRST) hipLaunchKernelGGL((K<T, 1, (KMV) | (CH_LRELU_DFIRST << 4)>), grid, dim3(256), 0, st, a); \
    else if (ch_ == CH_LRELU_DLAST) hipLaunchKernelGGL((K<T, 1, (KMV) | (CH_LRELU_DLAST << 4)>), grid, dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((K<T, 1, KMV>), grid, dim3(256), 0, st, a);                     \
  } while (0)
#define ES_KM_DISPATCH1(a, K, dt, grid, st)                                                \
  do {                                                                                    \
    const int km_ = keep_mode(a, true);                                                   \
    if (dt == ES_BF16) {                                                                  \
      if (km_ == KM_NONE) ES_KM_LAUNCH1(K, bf16, KM_NONE, grid, st, a);                   \
      else if (km_ == KM_BITS) ES_KM_LAUNCH1(K, bf16, KM_BITS, grid, st, a);              \
      else if (km_ == KM_HW4) ES_KM_LAUNCH1(K, bf16, KM_HW4, grid, st, a);                \
      else if (km_ == KM_ROW) ES_KM_LAUNCH1(K, bf16, KM_ROW, grid, st, a);                \
      else ES_KM_LAUNCH1(K, bf16, KM_GEN, grid, st, a);                                   \
    } else {                                                                              \
      if (km_ == KM_NONE) ES_KM_LAUNCH1(K, float, KM_NONE, grid, st, a);                  \
      else if (km_ == KM_BITS) ES_KM_LAUNCH1(K, float, KM_BITS, grid, st, a);             \
      else if (km_ == KM_HW4) ES_KM_LAUNCH1(K, float, KM_HW4, grid, st, a);               \
      else if (km_ == KM_ROW) ES_KM_LAUNCH1(K, float, KM_ROW, grid, st, a);               \
      else ES_KM_LAUNCH1(K, float, KM_GEN, grid, st, a);                                  \
    }                                                                                     \
  } while (0)

static FastArgs mk(const es_view_t* v, const es_chain_t* ch, int G) {
  FastArgs a{};
  a.rows = v->n * v->h * v->w;
  a.C = v->c;
  a.HW = v->h * v->w;
  a.G = G;
  a.cg = G ? v->c / G : 1;
  a.zrows = G ? a.HW : a.rows;
  a.nrows = v->rows;
  if (ch) {
    a.drop = ch->drop; a.dfirst = ch->dropout_first; a.act = ch->act; a.slope = ch->slope;
    a.keep = ch->drop.enabled ? ch->keep : nullptr;
  }
  return a;
}

// stats -> partials [z][chunk][3][C] (caller runs the finalize); returns chunks per z
int es_fast_norm_stats(const es_view_t* v, int G, es_dtype_t dt, const void* xp, float* part, hipStream_t st) {
  dim3 grid; int chunks;
  fast_geometry(v, G, grid, chunks);
  FastArgs a = mk(v, nullptr, G);
  a.x = xp; a.part = part;
  if (dt == ES_BF16) hipLaunchKernelGGL((bn_reduce_fast<bf16, 0, KM_NONE>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((bn_reduce_fast<float, 0, KM_NONE>), grid, dim3(256), 0, st, a);
  return chunks;
}

// keep_ready: a.keep already holds the mask (es_dropout_keep_bits): KM_BITS reads it, no Philox
void es_fast_norm_fwd(const es_view_t* v, int G, es_dtype_t dt, const void* xp, void* yp, const es_norm_t* nm,
                      const es_chain_t* ch, bool keep_ready, hipStream_t st) {
  dim3 grid; int chunks;
  fast_geometry(v, G, grid, chunks);
  FastArgs a = mk(v, ch, G);
  a.x = xp; a.out = yp;
  a.mean = nm->mean; a.invstd = nm->invstd; a.gamma = nm->gamma; a.beta = nm->beta;
  ES_KM_DISPATCH(a, bn_fwd_fast, dt, grid, st, keep_ready);
}

// dropout keep bits alone (for a forward that did not run the fast kernels): same bits as
// bn_fwd_fast would store
template <int KM>
__global__ void __launch_bounds__(256) keep_bits_kernel(FastArgs a) {
  resolve_stream(a.drop);
  const Geo g = geo(a);
  if (!g.active) return;
  const int ngroups = (g.rlim - g.rbase + 3) >> 2;
  for (int grp = blockIdx.y * g.RGB + g.rg; grp < ngroups; grp += gridDim.y * g.RGB) {
    const int r0 = g.rbase + grp * 4;
    const int nr = min(4, g.rlim - r0);
    uint32_t keep[4];
    keep_bits<KM>(a, r0, g.c0, keep);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < nr) a.keep[(int64_t)(r0 + j) * (a.C >> 3) + g.cv] = (uint8_t)keep[j];
  }
}

void es_fast_keep_bits(const es_view_t* v, const es_chain_t* ch, hipStream_t st) {
  es_view_t d = *v;   // logical rows (n, h, w) x C: the geometry of a dense view of the same shape
  dim3 grid; int chunks;
  fast_geometry(&d, 0, grid, chunks);
  FastArgs a = mk(&d, ch, 0);
  switch (keep_mode(a)) {
    case KM_HW4: hipLaunchKernelGGL((keep_bits_kernel<KM_HW4>), grid, dim3(256), 0, st, a); break;
    case KM_ROW: hipLaunchKernelGGL((keep_bits_kernel<KM_ROW>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((keep_bits_kernel<KM_GEN>), grid, dim3(256), 0, st, a); break;
  }
}

int es_fast_norm_bwd_reduce(const es_view_t* v, int G, es_dtype_t dt, const void* xp, const void* dyp,
                            const es_norm_t* nm, const es_chain_t* ch, float* part, hipStream_t st) {
  dim3 grid; int chunks;
  fast_geometry(v, G, grid, chunks);
  FastArgs a = mk(v, ch, G);
  a.x = xp; a.dy = dyp; a.part = part;
  a.mean = nm->mean; a.invstd = nm->invstd; a.gamma = nm->gamma; a.beta = nm->beta;
  ES_KM_DISPATCH1(a, bn_reduce_fast, dt, grid, st);
  return chunks;
}

// returns the number of dsum partials written to part (z slices x chunks), 0 without dsum
int es_fast_norm_bwd_apply(const es_view_t* v, int G, es_dtype_t dt, const void* xp, const void* dyp, void* dxp,
                           const es_norm_t* nm, const es_chain_t* ch, const float* a1, const float* a2,
                           float* dsum, float* part, hipStream_t st) {
  dim3 grid; int chunks;
  fast_geometry(v, G, grid, chunks);
  FastArgs a = mk(v, ch, G);
  a.x = xp; a.dy = dyp; a.out = dxp; a.a1 = a1; a.a2 = a2; a.dsum = dsum; a.part = part;
  a.mean = nm->mean; a.invstd = nm->invstd; a.gamma = nm->gamma; a.beta = nm->beta;
  ES_KM_DISPATCH(a, bn_bwd_apply_fast, dt, grid, st, true);
  return dsum ? (int)(grid.z * grid.y) : 0;
}
