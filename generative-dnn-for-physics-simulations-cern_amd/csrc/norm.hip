// Normalisation (BatchNorm / GroupNorm / LayerNorm) + dropout + activation, forward and backward.
//
// Replaces aten::native_batch_norm(+_backward) (neutron/generator.py:13,19,26,31,35;
// neutron/aux_reg.py:15,23,31,39,47), native_group_norm(+_backward) (neutron/discriminator.py:13,
// 18; proton/generator.py:28,34,39; proton/discriminator.py:123,128; proton/aux_reg.py:22,48-53),
// native_layer_norm(+_backward) (neutron/discriminator.py:28,34; proton/generator.py:15,20;
// proton/discriminator.py:135,141; proton/aux_reg.py:21,25), bernoulli_/mul of nn.Dropout and
// leaky_relu / relu (+ backward), fused into: stats reduction -> one elementwise pass forward,
// and reductions -> one elementwise pass backward.  The dropout mask is never stored: it is
// regenerated from (seed, stream, NCHW-logical index) by Philox (common.h).
//
// Reduction shapes
//   colred : per channel c over (n,h,w)   — BN stats, BN backward sums, GN/LN dgamma/dbeta,
//            bias gradients.  Block = 64 channels x 4 row lanes, rows split over blockIdx.y,
//            partials merged by a finalize kernel (Chan's parallel variance for stats).
//   segred : per stats group (n, g) over (c in g, h, w) — GN/LN stats and backward sums.  One
//            block per group, two passes (mean, then centred sum of squares).
#include "common.h"

// fast path for dense channels-last BatchNorm / GroupNorm (norm_fast.hip); G = 0 means BN
bool es_fast_dense_nhwc(const es_view_t* v);
int64_t es_fast_part_floats(const es_view_t* v, int G);
int es_fast_norm_stats(const es_view_t* v, int G, es_dtype_t dt, const void* xp, float* part, hipStream_t st);
void es_fast_norm_fwd(const es_view_t* v, int G, es_dtype_t dt, const void* xp, void* yp, const es_norm_t* nm,
                      const es_chain_t* ch, bool keep_ready, hipStream_t st);
void es_fast_keep_bits(const es_view_t* v, const es_chain_t* ch, hipStream_t st);
int es_fast_norm_bwd_reduce(const es_view_t* v, int G, es_dtype_t dt, const void* xp, const void* dyp,
                            const es_norm_t* nm, const es_chain_t* ch, float* part, hipStream_t st);
int es_fast_norm_bwd_apply(const es_view_t* v, int G, es_dtype_t dt, const void* xp, const void* dyp, void* dxp,
                           const es_norm_t* nm, const es_chain_t* ch, const float* a1, const float* a2,
                           float* dsum, float* part, hipStream_t st);

// which fast variant serves a norm of this kind on this view: -1 none, 0 BN, G > 0 GroupNorm
static int fast_kind(const es_view_t* v, int kind, int groups) {
  if (!es_fast_dense_nhwc(v)) return -1;
  if (kind == ES_NORM_BN) return 0;
  if (kind == ES_NORM_GN && groups > 0 && v->c % groups == 0 && v->h * v->w > 1) return groups;
  return -1;
}

// same logical shape and the same element addresses (strides of size-1 dims are irrelevant)
static bool same_view(const es_view_t* a, const es_view_t* b) {
  if (a->n != b->n || a->c != b->c || a->h != b->h || a->w != b->w) return false;
  const int dims[4] = {a->n, a->c, a->h, a->w};
  for (int i = 0; i < 4; ++i)
    if (dims[i] > 1 && a->s[i] != b->s[i]) return false;
  return true;
}

namespace {

struct View {
  int n, c, h, w;
  int64_t s[4];
  const int32_t* rows;   // dynamic rows: device count of the live samples (es_view_t.rows)
  __device__ __forceinline__ int64_t off(int in, int ic, int ih, int iw) const {
    return in * s[0] + ic * s[1] + ih * s[2] + iw * s[3];
  }
  __device__ __forceinline__ int live() const { return live_rows(rows, n); }
};
View mkview(const es_view_t* v) {
  View r;
  r.n = v->n; r.c = v->c; r.h = v->h; r.w = v->w;
  for (int i = 0; i < 4; ++i) r.s[i] = v->s[i];
  r.rows = v->rows;
  return r;
}

// A reduction's element count: c, or with dynamic rows (rows != NULL) c scaled to the live
// samples of the n-sample capacity (c = n * per-sample count)
struct Cnt {
  float c;
  const int32_t* rows;
  int n;
  __device__ __forceinline__ float get() const {
    return rows ? (float)live_rows(rows, n) * (c / (float)n) : c;
  }
};
Cnt mkcnt(float c, const es_view_t* v = nullptr) { return Cnt{c, v ? v->rows : nullptr, v ? v->n : 1}; }

__device__ __forceinline__ float ldf(const void* p, int bf, int64_t i) {
  return bf ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ void stf(void* p, int bf, int64_t i, float v) {
  if (bf) ((bf16*)p)[i] = (bf16)v;
  else ((float*)p)[i] = v;
}

struct Norm {
  int kind, groups, cg;
  const float *mean, *invstd, *gamma, *beta;
  __device__ __forceinline__ int group(int n, int c) const {
    return kind == ES_NORM_BN ? c : (kind == ES_NORM_GN ? n * groups + c / cg : n);
  }
  __device__ __forceinline__ float xhat(int n, int c, float x) const {
    if (kind == ES_NORM_NONE) return x;
    const int g = group(n, c);
    return (x - mean[g]) * invstd[g];
  }
  // LN gamma is indexed by feature; LN views have h = w = 1 so feature == c.
  __device__ __forceinline__ float gam(int c) const { return gamma ? gamma[c] : 1.f; }
  __device__ __forceinline__ float bet(int c) const { return beta ? beta[c] : 0.f; }
};
Norm mknorm(const es_norm_t* nm, int C) {
  Norm r{};
  if (!nm) { r.kind = ES_NORM_NONE; return r; }
  r.kind = nm->kind; r.groups = nm->groups > 0 ? nm->groups : 1;
  r.cg = C / r.groups;
  r.mean = nm->mean; r.invstd = nm->invstd; r.gamma = nm->gamma; r.beta = nm->beta;
  return r;
}

struct Chain {
  es_dropout_t drop;
  int dfirst, act;
  float slope;
  __device__ __forceinline__ float actf(float v) const {
    return act == ES_ACT_RELU ? fmaxf(v, 0.f) : (act == ES_ACT_LRELU ? lrelu(v, slope) : v);
  }
  __device__ __forceinline__ float dact(float v) const {  // derivative evaluated at input v
    return act == ES_ACT_RELU ? (v > 0.f ? 1.f : 0.f) : (act == ES_ACT_LRELU ? (v > 0.f ? 1.f : slope) : 1.f);
  }
  __device__ __forceinline__ float fwd(float y, uint64_t li) const {
    if (!drop.enabled) return actf(y);
    const bool keep = dropout_keep(drop, li);
    if (dfirst) return actf(keep ? y * drop.scale : 0.f);
    const float u = actf(y);
    return keep ? u * drop.scale : 0.f;
  }
  // d out / d y given dout; `ref` (if has_ref) replaces the activation input for the derivative
  __device__ __forceinline__ float bwd(float y, float dout, uint64_t li, bool has_ref, float ref) const {
    if (!drop.enabled) return dout * dact(has_ref ? ref : y);
    const bool keep = dropout_keep(drop, li);
    if (!keep) return 0.f;
    if (dfirst) {
      const float u = y * drop.scale;
      return dout * dact(has_ref ? ref : u) * drop.scale;
    }
    return dout * drop.scale * dact(has_ref ? ref : y);
  }
};
Chain mkchain(const es_chain_t* ch) {
  Chain c{};
  if (ch) { c.drop = ch->drop; c.dfirst = ch->dropout_first; c.act = ch->act; c.slope = ch->slope; }
  else { c.drop.enabled = 0; c.act = ES_ACT_NONE; }
  return c;
}

__device__ __forceinline__ uint64_t logical_index(const View& v, int n, int c, int h, int w) {
  return (((uint64_t)n * v.c + c) * v.h + h) * v.w + w;
}

// element e of the logical tensor -> (n,c,h,w); channels-last order when the view says so
__device__ __forceinline__ void decompose(const View& v, bool cl, int64_t e, int& n, int& c, int& h, int& w) {
  if (e < 0x7fffffff) {   // 32-bit index math (64-bit division is a long software sequence)
    uint32_t t = (uint32_t)e;
    if (cl) {
      c = t % (uint32_t)v.c; t /= (uint32_t)v.c; w = t % (uint32_t)v.w; t /= (uint32_t)v.w;
      h = t % (uint32_t)v.h; n = t / (uint32_t)v.h;
    } else {
      w = t % (uint32_t)v.w; t /= (uint32_t)v.w; h = t % (uint32_t)v.h; t /= (uint32_t)v.h;
      c = t % (uint32_t)v.c; n = t / (uint32_t)v.c;
    }
    return;
  }
  if (cl) {
    c = e % v.c; int64_t t = e / v.c; w = t % v.w; t /= v.w; h = t % v.h; n = t / v.h;
  } else {
    w = e % v.w; int64_t t = e / v.w; h = t % v.h; t /= v.h; c = t % v.c; n = t / v.c;
  }
}

// ============================================================================ colred
enum { RED_STATS = 0, RED_BWD = 1, RED_SUM = 2 };

struct BwdIn {   // everything needed to evaluate dnorm and xhat per element
  View x; const void* xp; int xbf;
  View dy; const void* dyp; int dybf;
  View ref; const void* refp; int refbf;  // refp may be null
  View add; const void* addp; int addbf;  // addend (fwd residual) may be null
  Norm nm; Chain ch;
};

__device__ __forceinline__ void bwd_elem(const BwdIn& b, int n, int c, int h, int w, float& dnorm, float& xh) {
  const float x = ldf(b.xp, b.xbf, b.x.off(n, c, h, w));
  xh = b.nm.xhat(n, c, x);
  float y = xh * b.nm.gam(c) + b.nm.bet(c);
  if (b.addp) y += ldf(b.addp, b.addbf, b.add.off(n, c, h, w));
  const float dout = ldf(b.dyp, b.dybf, b.dy.off(n, c, h, w));
  const float ref = b.refp ? ldf(b.refp, b.refbf, b.ref.off(n, c, h, w)) : 0.f;
  dnorm = b.ch.bwd(y, dout, logical_index(b.x, n, c, h, w), b.refp != nullptr, ref);
}

template <int RED>
__global__ void __launch_bounds__(256) colred_kernel(BwdIn b, int64_t rows, int64_t rows_per_chunk, float* part) {
  resolve_stream(b.ch.drop);
  // part layout: [chunk][3][C]
  const View& v = b.x;
  const int C = v.c;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int64_t r0 = blockIdx.y * rows_per_chunk;
  if (v.rows) rows = (int64_t)v.live() * v.h * v.w;
  const int64_t r1 = min(rows, r0 + rows_per_chunk);
  float cnt = 0.f, a = 0.f, m2 = 0.f;   // STATS: Welford (cnt, mean, M2); BWD/SUM: (., s1, s2)
  if (c < C) {
    // row r -> (n, h, w), w fastest
    for (int64_t r = r0 + ty; r < r1; r += 4) {
      const uint32_t r32 = (uint32_t)r, t = r32 / (uint32_t)v.w;   // rows < 2^31 (host-checked sizes)
      const int w = r32 - t * v.w, h = t % (uint32_t)v.h, n = t / (uint32_t)v.h;
      if (RED == RED_STATS) {
        const float x = ldf(b.xp, b.xbf, v.off(n, c, h, w));
        cnt += 1.f;
        const float d = x - a;
        a += d / cnt;
        m2 += d * (x - a);
      } else if (RED == RED_SUM) {
        a += ldf(b.xp, b.xbf, v.off(n, c, h, w));
      } else {
        float dn, xh;
        bwd_elem(b, n, c, h, w, dn, xh);
        a += dn;
        m2 += dn * xh;
      }
    }
  }
  __shared__ float sh[3][4][64];
  sh[0][ty][tx] = cnt; sh[1][ty][tx] = a; sh[2][ty][tx] = m2;
  __syncthreads();
  if (ty == 0 && c < C) {
    if (RED == RED_STATS) {
      float n_ = sh[0][0][tx], mu = sh[1][0][tx], M = sh[2][0][tx];
      for (int k = 1; k < 4; ++k) {
        const float nb = sh[0][k][tx];
        if (nb == 0.f) continue;
        const float mb = sh[1][k][tx], Mb = sh[2][k][tx];
        const float nt = n_ + nb, dl = mb - mu;
        mu += dl * nb / nt;
        M += Mb + dl * dl * n_ * nb / nt;
        n_ = nt;
      }
      cnt = n_; a = mu; m2 = M;
    } else {
      a = sh[1][0][tx] + sh[1][1][tx] + sh[1][2][tx] + sh[1][3][tx];
      m2 = sh[2][0][tx] + sh[2][1][tx] + sh[2][2][tx] + sh[2][3][tx];
    }
    float* p = part + (int64_t)blockIdx.y * 3 * C;
    p[c] = cnt; p[C + c] = a; p[2 * C + c] = m2;
  }
}

// BN stats finalize: merge chunk partials -> mean/invstd, running stats (torch semantics).
__device__ __forceinline__ void bn_stats_store(int c, double n_, double s1, double s2, float eps, float* mean,
                                               float* invstd, float* rmean, float* rvar, float mom) {
  if (n_ <= 0.0) {   // no live sample (dynamic rows): finite statistics, running stats untouched
    mean[c] = 0.f;
    invstd[c] = (float)(1.0 / sqrt((double)eps));
    return;
  }
  const double mt = s1 / n_;
  const double Mt = fmax(s2 - n_ * mt * mt, 0.0);
  const double var = Mt / n_;
  mean[c] = (float)mt;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) rmean[c] = (1.f - mom) * rmean[c] + mom * (float)mt;
  if (rvar) rvar[c] = (1.f - mom) * rvar[c] + mom * (float)(n_ > 1.0 ? Mt / (n_ - 1.0) : var);
}

// (few chunks: the exact fp64 Welford merge; the gradient parity tests at B = 8 sit on
// LeakyReLU / dropout kinks that a last-bit change of the statistics can flip)
__global__ void bn_finalize_kernel(const float* part, int chunks, int C, float eps, float* mean,
                                   float* invstd, float* rmean, float* rvar, float mom) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double n_ = 0.0, mu = 0.0, M = 0.0;
  for (int k = 0; k < chunks; ++k) {
    const float* p = part + (int64_t)k * 3 * C;
    const double nb = p[c];
    if (nb == 0.0) continue;
    const double mb = p[C + c], Mb = p[2 * C + c];
    const double nt = n_ + nb, dl = mb - mu;
    mu += dl * nb / nt;
    M += Mb + dl * dl * n_ * nb / nt;
    n_ = nt;
  }
  if (n_ <= 0.0) {   // no live sample (dynamic rows): finite statistics, running stats untouched
    mean[c] = 0.f;
    invstd[c] = (float)(1.0 / sqrt((double)eps));
    return;
  }
  const double var = M / n_;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) rmean[c] = (1.f - mom) * rmean[c] + mom * (float)mu;
  if (rvar) rvar[c] = (1.f - mom) * rvar[c] + mom * (float)(n_ > 1.0 ? M / (n_ - 1.0) : var);
}

// Two-level merge for many chunks and few channels (a conv epilogue's per-row-tile partials, e.g.
// 16208 x 64 for generator conv_layers.9 at B = 1024): level 1, block b Chan-merges the chunk range
// [b R, (b+1) R) with coalesced reads (threads along the channels) and writes the result IN PLACE
// into chunk b R of that range (only its own range is touched: no cross-block hazard; the partials
// are consumed); level 2 merges the G range heads per channel.  (One block per channel reading
// every chunk with a stride of 3C floats requested one cache line per load: ~50 us.)
__global__ void __launch_bounds__(256) bn_merge_l1_kernel(float* part, int chunks, int C, int R) {
  const int k0 = blockIdx.x * R, k1 = min(chunks, k0 + R);
  const int TS = 256 / C > 0 ? 256 / C : 1;           // chunk streams (C <= 256)
  const int c = threadIdx.x % C, sidx = threadIdx.x / C;
  __shared__ double sh[3][256];
  double n_ = 0.0, s1 = 0.0, s2 = 0.0;
  if (sidx < TS) {
#pragma unroll 4
    for (int k = k0 + sidx; k < k1; k += TS) {
      const float* p = part + (int64_t)k * 3 * C;
      const double nb = p[c], mb = p[C + c], Mb = p[2 * C + c];
      const bool has = nb > 0.0;
      n_ += nb;
      s1 += has ? nb * mb : 0.0;
      s2 += has ? Mb + nb * mb * mb : 0.0;
    }
  }
  sh[0][threadIdx.x] = n_; sh[1][threadIdx.x] = s1; sh[2][threadIdx.x] = s2;
  __syncthreads();                                      // every read of the range is done
  if (threadIdx.x < C) {
    for (int t = 1; t < TS; ++t) {
      n_ += sh[0][t * C + c]; s1 += sh[1][t * C + c]; s2 += sh[2][t * C + c];
    }
    float* p = part + (int64_t)k0 * 3 * C;
    const double mt = n_ > 0.0 ? s1 / n_ : 0.0;
    p[c] = (float)n_;
    p[C + c] = (float)mt;
    p[2 * C + c] = (float)fmax(s2 - n_ * mt * mt, 0.0);
  }
}

__global__ void __launch_bounds__(256) bn_merge_l2_kernel(const float* part, int G, int R, int C, float eps,
                                                          float* mean, float* invstd, float* rmean, float* rvar,
                                                          float mom) {
  const int c = blockIdx.x;
  __shared__ double sh[8];
  double n_ = 0.0, s1 = 0.0, s2 = 0.0;
  for (int b = threadIdx.x; b < G; b += 256) {
    const float* p = part + (int64_t)b * R * 3 * C;
    const double nb = p[c], mb = p[C + c], Mb = p[2 * C + c];
    const bool has = nb > 0.0;
    n_ += nb;
    s1 += has ? nb * mb : 0.0;
    s2 += has ? Mb + nb * mb * mb : 0.0;
  }
  n_ = block_sum_d(n_, sh);
  s1 = block_sum_d(s1, sh);
  s2 = block_sum_d(s2, sh);
  if (threadIdx.x == 0) bn_stats_store(c, n_, s1, s2, eps, mean, invstd, rmean, rvar, mom);
}

// BN backward finalize: per channel A1 = gamma*s1/cnt, A2 = gamma*s2/cnt ; dgamma += s2, dbeta += s1
__global__ void bn_bwd_finalize_kernel(const float* part, int chunks, int C, float cnt, const float* gamma,
                                       float* a1, float* a2, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f, s2 = 0.f;
  for (int k = 0; k < chunks; ++k) {
    const float* p = part + (int64_t)k * 3 * C;
    s1 += p[C + c]; s2 += p[2 * C + c];
  }
  const float g = gamma ? gamma[c] : 1.f;
  if (a1) { a1[c] = g * s1 / cnt; a2[c] = g * s2 / cnt; }
  if (dgamma) dgamma[c] += s2;
  if (dbeta) dbeta[c] += s1;
}

__global__ void sum_finalize_kernel(const float* part, int chunks, int C, float* out, float beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < chunks; ++k) s += part[(int64_t)k * 3 * C + C + c];
  out[c] = (beta != 0.f ? beta * out[c] : 0.f) + s;
}

// Block-per-channel variants of the finalize kernels (many chunks, moderate C).  1024 threads,
// four independent partial loads in flight per thread: with 256 threads and one load chain per
// thread the merge of a conv epilogue's 16208 row-tile partials (generator conv_layers.9, B = 1024)
// took 76 us, latency-bound on 64 busy CUs.
constexpr int FIN_T = 1024;

__global__ void __launch_bounds__(FIN_T) bn_finalize_block_kernel(const float* part, int chunks, int C, float eps,
                                                                  float* mean, float* invstd, float* rmean,
                                                                  float* rvar, float mom) {
  // Plain fp64 sums n, sum n_b*m_b, sum (M_b + n_b*m_b^2) instead of a Welford merge per chunk: the
  // merge's fp64 division made every thread's loop one dependent chain; sums let the strided
  // partial loads issue back to back.  fp64 keeps the S2 - n*mean^2 subtraction exact far beyond
  // fp32 resolution for activation statistics.
  const int c = blockIdx.x;
  double n_ = 0.0, s1 = 0.0, s2 = 0.0;
  const int64_t st = (int64_t)3 * C;
  int k = threadIdx.x;
  for (; k + 3 * FIN_T < chunks; k += 4 * FIN_T) {
    float nb[4], mb[4], Mb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* p = part + (int64_t)(k + u * FIN_T) * st;
      nb[u] = p[c]; mb[u] = p[C + c]; Mb[u] = p[2 * C + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool has = nb[u] > 0.f;        // an empty chunk's mean / M2 may be 0/0: skip it
      const double nd = nb[u], md = mb[u];
      n_ += nd;
      s1 += has ? nd * md : 0.0;
      s2 += has ? (double)Mb[u] + nd * md * md : 0.0;
    }
  }
  for (; k < chunks; k += FIN_T) {
    const float* p = part + (int64_t)k * st;
    const double nb = p[c], mb = p[C + c], Mb = p[2 * C + c];
    const bool has = nb > 0.0;
    n_ += nb;
    s1 += has ? nb * mb : 0.0;
    s2 += has ? Mb + nb * mb * mb : 0.0;
  }
  __shared__ double sh[FIN_T / 64];
  n_ = block_sum_d(n_, sh);
  s1 = block_sum_d(s1, sh);
  s2 = block_sum_d(s2, sh);
  if (threadIdx.x == 0) bn_stats_store(c, n_, s1, s2, eps, mean, invstd, rmean, rvar, mom);
}

// out1 (+)= s1 (beta1: scale of old out1), out2 += s2; a1/a2 = gamma*s/cnt (BN backward)
__device__ __forceinline__ void sums_store(int c, float s1, float s2, Cnt cn, const float* gamma, float* a1,
                                           float* a2, float* out1, float* out2, float beta1) {
  const float g = gamma ? gamma[c] : 1.f;
  const float cnt = fmaxf(cn.get(), 1.f);
  if (a1) { a1[c] = g * s1 / cnt; a2[c] = g * s2 / cnt; }
  if (out1) out1[c] = (beta1 != 0.f ? beta1 * out1[c] : 0.f) + s1;
  if (out2) out2[c] += s2;
}

__global__ void __launch_bounds__(FIN_T) sums_finalize_block_kernel(const float* part, int chunks, int C, Cnt cnt,
                                                                    const float* gamma, float* a1, float* a2,
                                                                    float* out1, float* out2, float beta1) {
  const int c = blockIdx.x;
  __shared__ float sh[FIN_T / 64];
  float s1 = 0.f, s2 = 0.f;
  const int64_t st = (int64_t)3 * C;
  int k = threadIdx.x;
  for (; k + 3 * FIN_T < chunks; k += 4 * FIN_T) {
    float v1[4], v2[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* p = part + (int64_t)(k + u * FIN_T) * st;
      v1[u] = p[C + c]; v2[u] = p[2 * C + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { s1 += v1[u]; s2 += v2[u]; }
  }
  for (; k < chunks; k += FIN_T) {
    const float* p = part + (int64_t)k * st;
    s1 += p[C + c]; s2 += p[2 * C + c];
  }
  s1 = block_sum(s1, sh);
  s2 = block_sum(s2, sh);
  if (threadIdx.x == 0) sums_store(c, s1, s2, cnt, gamma, a1, a2, out1, out2, beta1);
}

// thread-per-channel form of the same (few chunks, or many channels: coalesced across channels)
__global__ void __launch_bounds__(256) sums_finalize_kernel(const float* part, int chunks, int C, Cnt cnt,
                                                            const float* gamma, float* a1, float* a2, float* out1,
                                                            float* out2, float beta1) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int k = 0; k < chunks; ++k) {
    const float* p = part + (int64_t)k * 3 * C;
    s1 += p[C + c]; s2 += p[2 * C + c];
  }
  sums_store(c, s1, s2, cnt, gamma, a1, a2, out1, out2, beta1);
}

// finalize dispatch: a block per channel while the chunks dominate, a thread per channel otherwise
bool fin_block(int chunks, int C) { return chunks > 32 && C < 4096; }
// two-level in-place merge of many chunk partials (measured faster than the block-per-channel kernel)

void launch_bn_finalize(hipStream_t st, const float* part, int chunks, int C, float eps, float* mean, float* invstd,
                        float* rmean, float* rvar, float mom) {
  if (chunks >= 1024 && C <= 256) {   // (consumes the partials: they are merged in place)
    const int G = std::min(256, chunks / 16), R = (chunks + G - 1) / G;
    const int Gr = (chunks + R - 1) / R;
    hipLaunchKernelGGL(bn_merge_l1_kernel, dim3(Gr), dim3(256), 0, st, const_cast<float*>(part), chunks, C, R);
    hipLaunchKernelGGL(bn_merge_l2_kernel, dim3(C), dim3(256), 0, st, part, Gr, R, C, eps, mean, invstd, rmean,
                       rvar, mom);
    return;
  }
  if (fin_block(chunks, C))
    hipLaunchKernelGGL(bn_finalize_block_kernel, dim3(C), dim3(FIN_T), 0, st, part, chunks, C, eps, mean, invstd,
                       rmean, rvar, mom);
  else
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, chunks, C, eps, mean,
                       invstd, rmean, rvar, mom);
}

void launch_sums_finalize(hipStream_t st, const float* part, int chunks, int C, Cnt cnt, const float* gamma,
                          float* a1, float* a2, float* out1, float* out2, float beta1) {
  if (fin_block(chunks, C))
    hipLaunchKernelGGL(sums_finalize_block_kernel, dim3(C), dim3(FIN_T), 0, st, part, chunks, C, cnt, gamma, a1, a2,
                       out1, out2, beta1);
  else
    hipLaunchKernelGGL(sums_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, chunks, C, cnt, gamma,
                       a1, a2, out1, out2, beta1);
}

// GroupNorm stats finalize from fast partials [n][chunk][3][C]: one thread per (n, g), Chan merge
// over the chunks and the cg channels of the group.
__global__ void gn_finalize_kernel(const float* part, int N, int chunks, int C, int G, float eps, float* mean,
                                   float* invstd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * G) return;
  const int n = i / G, g = i % G, cg = C / G;
  double n_ = 0.0, mu = 0.0, M = 0.0;
  for (int k = 0; k < chunks; ++k) {
    const float* p = part + ((int64_t)n * chunks + k) * 3 * C;
    for (int c = g * cg; c < (g + 1) * cg; ++c) {
      const double nb = p[c];
      if (nb == 0.0) continue;
      const double mb = p[C + c], Mb = p[2 * C + c];
      const double nt = n_ + nb, dl = mb - mu;
      mu += dl * nb / nt;
      M += Mb + dl * dl * n_ * nb / nt;
      n_ = nt;
    }
  }
  mean[i] = (float)mu;
  invstd[i] = (float)(1.0 / sqrt((n_ > 0.0 ? M / n_ : 0.0) + (double)eps));   // (padding samples: n_ = 0)
}

// GroupNorm backward finalize from fast partials: a1/a2[n, g] = mean over the group of gamma*s
__global__ void gn_bwd_finalize_kernel(const float* part, int N, int chunks, int C, int G, float cnt,
                                       const float* gamma, float* a1, float* a2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * G) return;
  const int n = i / G, g = i % G, cg = C / G;
  float s1 = 0.f, s2 = 0.f;
  for (int k = 0; k < chunks; ++k) {
    const float* p = part + ((int64_t)n * chunks + k) * 3 * C;
    for (int c = g * cg; c < (g + 1) * cg; ++c) {
      const float ga = gamma ? gamma[c] : 1.f;
      s1 += ga * p[C + c]; s2 += ga * p[2 * C + c];
    }
  }
  a1[i] = s1 / cnt; a2[i] = s2 / cnt;
}

void colred_geometry(const View& v, int& cblocks, int& chunks, int64_t& rows, int64_t& per) {
  rows = (int64_t)v.n * v.h * v.w;
  cblocks = (v.c + 63) / 64;
  int want = std::max(1, 1024 / cblocks);
  want = (int)std::min<int64_t>(want, std::max<int64_t>(1, rows / 64));
  per = (rows + want - 1) / want;
  chunks = (int)((rows + per - 1) / per);
}

// single-channel sum: block partials into the s1 slot of [chunk][3][1]
__global__ void __launch_bounds__(256) sum1_kernel(BwdIn b, int rows, float* part) {
  const View& v = b.x;
  __shared__ float sh[8];
  float s = 0.f;
  if (v.rows) rows = v.live() * v.h * v.w;
  for (int r = blockIdx.x * 256 + threadIdx.x; r < rows; r += gridDim.x * 256) {
    const uint32_t t = (uint32_t)r / (uint32_t)v.w;
    const int w = r - (int)t * v.w, h = t % (uint32_t)v.h, n = t / (uint32_t)v.h;
    s += ldf(b.xp, b.xbf, v.off(n, 0, h, w));
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x * 3 + 1] = s;
}

// ============================================================================ segred
// one block per stats group; RED_STATS writes mean/invstd, RED_BWD writes A1/A2 (means over group)
template <int RED>
__global__ void __launch_bounds__(256) segred_kernel(BwdIn b, float eps, float* o1, float* o2) {
  resolve_stream(b.ch.drop);
  const View& v = b.x;
  const int G = b.nm.kind == ES_NORM_GN ? b.nm.groups : 1;
  const int cg = v.c / G;
  const int n = blockIdx.x / G, g = blockIdx.x % G;
  if (n >= v.live()) {   // a padding sample (dynamic rows): finite statistics, zero sums
    if (threadIdx.x == 0) { o1[blockIdx.x] = 0.f; o2[blockIdx.x] = RED == RED_STATS ? rsqrtf(eps) : 0.f; }
    return;
  }
  const int64_t cnt = (int64_t)cg * v.h * v.w;
  const bool cl = v.s[1] == 1 && cg > 1;
  __shared__ float sh[8];
  auto coords = [&](int64_t j64, int& c, int& h, int& w) {
    const uint32_t j = (uint32_t)j64;   // j < cnt = cg*h*w (one sample)
    if (cl) { c = g * cg + j % cg; const uint32_t t = j / cg; w = t % v.w; h = t / v.w; }
    else { w = j % v.w; const uint32_t t = j / v.w; h = t % v.h; c = g * cg + t / v.h; }
  };
  if (RED == RED_STATS) {
    float s = 0.f;
    for (int64_t j = threadIdx.x; j < cnt; j += blockDim.x) {
      int c, h, w; coords(j, c, h, w);
      s += ldf(b.xp, b.xbf, v.off(n, c, h, w));
    }
    const float mu = block_sum(s, sh) / (float)cnt;
    float q = 0.f;
    for (int64_t j = threadIdx.x; j < cnt; j += blockDim.x) {
      int c, h, w; coords(j, c, h, w);
      const float d = ldf(b.xp, b.xbf, v.off(n, c, h, w)) - mu;
      q += d * d;
    }
    const float var = block_sum(q, sh) / (float)cnt;
    if (threadIdx.x == 0) { o1[blockIdx.x] = mu; o2[blockIdx.x] = rsqrtf(var + eps); }
  } else {
    float s1 = 0.f, s2 = 0.f;
    for (int64_t j = threadIdx.x; j < cnt; j += blockDim.x) {
      int c, h, w; coords(j, c, h, w);
      float dn, xh;
      bwd_elem(b, n, c, h, w, dn, xh);
      const float dxh = dn * b.nm.gam(c);
      s1 += dxh; s2 += dxh * xh;
    }
    s1 = block_sum(s1, sh);
    s2 = block_sum(s2, sh);
    if (threadIdx.x == 0) { o1[blockIdx.x] = s1 / (float)cnt; o2[blockIdx.x] = s2 / (float)cnt; }
  }
}

// ============================================================================ elementwise
struct FwdArgs {
  View x; const void* xp; int xbf;
  View add; const void* addp; int addbf;
  View y; void* yp; int ybf;
  Norm nm; Chain ch;
};

__global__ void __launch_bounds__(256) norm_fwd_kernel(FwdArgs a) {
  resolve_stream(a.ch.drop);
  // (both element orders have n slowest: the live samples' elements are a prefix)
  const int64_t total = (int64_t)a.x.live() * a.x.c * a.x.h * a.x.w;
  const bool cl = a.x.s[1] == 1 && a.x.c > 1;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int n, c, h, w;
    decompose(a.x, cl, e, n, c, h, w);
    const float x = ldf(a.xp, a.xbf, a.x.off(n, c, h, w));
    float y = a.nm.kind == ES_NORM_NONE ? x : a.nm.xhat(n, c, x) * a.nm.gam(c) + a.nm.bet(c);
    if (a.addp) y += ldf(a.addp, a.addbf, a.add.off(n, c, h, w));
    stf(a.yp, a.ybf, a.y.off(n, c, h, w), a.ch.fwd(y, logical_index(a.x, n, c, h, w)));
  }
}

struct BwdApply {
  BwdIn b;
  View dx; void* dxp; int dxbf;
  const float* a1; const float* a2;  // per stats group
  float beta;
  float* csum;                        // optional: per-channel sum of dx (conv-bias gradient), C <= 1024
};

__global__ void __launch_bounds__(256) norm_bwd_apply_kernel(BwdApply a) {
  resolve_stream(a.b.ch.drop);
  const View& v = a.b.x;
  const int64_t total = (int64_t)v.live() * v.c * v.h * v.w;
  const bool cl = v.s[1] == 1 && v.c > 1;
  __shared__ float sacc[1024];
  if (a.csum) {
    for (int i = threadIdx.x; i < v.c; i += blockDim.x) sacc[i] = 0.f;
    __syncthreads();
  }
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int n, c, h, w;
    decompose(v, cl, e, n, c, h, w);
    float dn, xh;
    bwd_elem(a.b, n, c, h, w, dn, xh);
    float dx;
    if (a.b.nm.kind == ES_NORM_NONE) {
      dx = dn;
    } else {
      const int g = a.b.nm.group(n, c);
      dx = a.b.nm.invstd[g] * (dn * a.b.nm.gam(c) - a.a1[g] - xh * a.a2[g]);
    }
    const int64_t o = a.dx.off(n, c, h, w);
    if (a.csum) atomicAdd(&sacc[c], dx);
    if (a.beta != 0.f) dx += a.beta * ldf(a.dxp, a.dxbf, o);
    stf(a.dxp, a.dxbf, o, dx);
  }
  if (a.csum) {
    __syncthreads();
    for (int i = threadIdx.x; i < v.c; i += blockDim.x)
      if (sacc[i] != 0.f) atomicAdd(&a.csum[i], sacc[i]);
  }
}

int grid_for(int64_t total) { return (int)std::min<int64_t>((total + 255) / 256, 8192); }

BwdIn mk_bwdin(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_norm_t* nm,
               const es_chain_t* ch) {
  BwdIn b{};
  b.x = mkview(x); b.xp = xp; b.xbf = xdt == ES_BF16;
  b.nm = mknorm(nm, x->c); b.ch = mkchain(ch);
  b.refp = nullptr; b.addp = nullptr; b.dyp = nullptr;
  return b;
}

// dsum += sum of the fast apply's per-block partials (s1 slot of [chunk][3][C])
void fast_dsum_finalize(int C, int chunks, const float* part, float* dsum, hipStream_t st) {
  if (chunks <= 0 || dsum == nullptr) return;
  launch_sums_finalize(st, part, chunks, C, mkcnt(1.f), nullptr, (float*)nullptr, (float*)nullptr, dsum, (float*)nullptr, 1.f);
}

int64_t stats_groups(const es_view_t* x, int kind, int groups) {
  if (kind == ES_NORM_BN) return x->c;
  if (kind == ES_NORM_GN) return (int64_t)x->n * groups;
  return x->n;
}

// ---- data-parallel (SyncBN) helpers
// merge [chunks][3][C] (count, mean, M2) partials into one [3][C] partial (fp64 sums, as
// bn_finalize_block_kernel): a rank's local BatchNorm statistics, all-gathered across ranks and
// finalized with es_norm_stats_finalize(world partials)
__global__ void __launch_bounds__(256) stats_merge_kernel(const float* part, int chunks, int C, float* out) {
  const int c = blockIdx.x;
  double n_ = 0.0, s1 = 0.0, s2 = 0.0;
  for (int k = threadIdx.x; k < chunks; k += blockDim.x) {
    const float* p = part + (int64_t)k * 3 * C;
    const double nb = p[c], mb = p[C + c], Mb = p[2 * C + c];
    const bool has = nb > 0.0;
    n_ += nb;
    s1 += has ? nb * mb : 0.0;
    s2 += has ? Mb + nb * mb * mb : 0.0;
  }
  __shared__ double sn[256], sm[256], sM[256];
  sn[threadIdx.x] = n_; sm[threadIdx.x] = s1; sM[threadIdx.x] = s2;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      sn[threadIdx.x] += sn[threadIdx.x + off];
      sm[threadIdx.x] += sm[threadIdx.x + off];
      sM[threadIdx.x] += sM[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double nt = sn[0], mt = nt > 0.0 ? sm[0] / nt : 0.0;
    out[c] = (float)nt;
    out[C + c] = (float)mt;
    out[2 * C + c] = (float)fmax(sM[0] - nt * mt * mt, 0.0);
  }
}

// a1 = gamma*s1/cnt, a2 = gamma*s2/cnt from (all-reduced) raw backward sums [2][C]
__global__ void bn_scale_sums_kernel(const float* sums, int C, float cnt, const float* cnt_mul, const float* gamma,
                                     float* a1, float* a2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (cnt_mul) cnt *= fmaxf(cnt_mul[0], 1.f);   // device sample count x per-sample elements
  const float g = gamma ? gamma[c] : 1.f;
  a1[c] = g * sums[c] / cnt;
  a2[c] = g * sums[C + c] / cnt;
}

}  // namespace

// ================================================================================ C ABI
extern "C" int64_t es_norm_stats_ws_bytes(const es_view_t* x, int kind, int groups) {
  const int fk = fast_kind(x, kind, groups);
  int64_t b = 0;
  if (kind == ES_NORM_BN) {
    View v = mkview(x);
    int cb, chunks; int64_t rows, per;
    colred_geometry(v, cb, chunks, rows, per);
    b = (int64_t)chunks * 3 * v.c * sizeof(float);
  }
  if (fk >= 0) b = std::max<int64_t>(b, es_fast_part_floats(x, fk) * (int64_t)sizeof(float));
  return b;
}

extern "C" int es_norm_stats(const es_view_t* x, es_dtype_t xdt, const void* xp, int kind,
                             int groups, float eps, float* mean, float* invstd, float* running_mean,
                             float* running_var, float momentum, void* ws, es_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  ES_CHECK_ARG(kind == ES_NORM_BN || kind == ES_NORM_GN || kind == ES_NORM_LN, "norm_stats: kind %d", kind);
  ES_CHECK_ARG(kind != ES_NORM_GN || (groups > 0 && x->c % groups == 0), "norm_stats: groups");
  ES_CHECK_ARG(kind != ES_NORM_LN || (x->h == 1 && x->w == 1), "norm_stats: LN needs (N,F,1,1) views");
  es_norm_t nm{kind, groups, nullptr, nullptr, nullptr, nullptr};
  BwdIn b = mk_bwdin(x, xdt, xp, &nm, nullptr);
  const int fk = fast_kind(x, kind, groups);
  if (fk > 0) {
    ES_CHECK_ARG(ws != nullptr, "norm_stats: fast GroupNorm needs workspace");
    const int chunks = es_fast_norm_stats(x, fk, xdt, xp, (float*)ws, st);
    const int ng = x->n * groups;
    hipLaunchKernelGGL(gn_finalize_kernel, dim3((ng + 255) / 256), dim3(256), 0, st, (const float*)ws, x->n,
                       chunks, x->c, groups, eps, mean, invstd);
  } else if (kind == ES_NORM_BN) {
    int cb, chunks; int64_t rows, per;
    colred_geometry(b.x, cb, chunks, rows, per);
    ES_CHECK_ARG(ws != nullptr, "norm_stats: BN needs workspace");
    if (fk == 0)
      chunks = es_fast_norm_stats(x, 0, xdt, xp, (float*)ws, st);
    else
      hipLaunchKernelGGL(colred_kernel<RED_STATS>, dim3(cb, chunks), dim3(256), 0, st, b, rows, per, (float*)ws);
    launch_bn_finalize(st, (const float*)ws, chunks, x->c, eps, mean, invstd, running_mean, running_var, momentum);
  } else {
    const int64_t ng = stats_groups(x, kind, groups);
    hipLaunchKernelGGL(segred_kernel<RED_STATS>, dim3((unsigned)ng), dim3(256), 0, st, b, eps, mean, invstd);
  }
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_norm_stats_finalize(const float* part, int chunks, int C, float eps, float* mean, float* invstd,
                                      float* running_mean, float* running_var, float momentum, es_stream_t stream) {
  ES_CHECK_ARG(part && chunks > 0 && C > 0, "norm_stats_finalize: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  launch_bn_finalize(st, part, chunks, C, eps, mean, invstd, running_mean, running_var, momentum);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_norm_act_fwd(const es_view_t* x, es_dtype_t xdt, const es_norm_t* nm,
                               const es_chain_t* ch, const es_view_t* addend, es_dtype_t adt,
                               const void* addend_ptr, const void* xp, const es_view_t* y,
                               es_dtype_t ydt, void* yp, es_stream_t stream) {
  ES_CHECK_ARG(x->n == y->n && x->c == y->c && x->h == y->h && x->w == y->w, "norm_act_fwd: shape");
  const int fk = nm ? fast_kind(x, nm->kind, nm->groups) : -1;
  const bool bits = ch && ch->keep && ch->drop.enabled;
  ES_CHECK_ARG(!bits || x->c % 8 == 0, "norm_act_fwd: dropout keep bits need C %% 8 == 0");
  const bool ready = bits && ch->keep_ready;
  if (fk >= 0 && !addend_ptr && xdt == ydt && same_view(x, y)) {
    es_fast_norm_fwd(x, fk, xdt, xp, yp, nm, ch, ready, (hipStream_t)stream);
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  // the generic kernel draws the same mask in the pass; the bits for the backward are stored here
  if (bits && !ready) es_fast_keep_bits(x, ch, (hipStream_t)stream);
  FwdArgs a{};
  a.x = mkview(x); a.xp = xp; a.xbf = xdt == ES_BF16;
  a.y = mkview(y); a.yp = yp; a.ybf = ydt == ES_BF16;
  a.addp = addend_ptr;
  if (addend_ptr) { a.add = mkview(addend); a.addbf = adt == ES_BF16; }
  a.nm = mknorm(nm, x->c); a.ch = mkchain(ch);
  const int64_t total = (int64_t)x->n * x->c * x->h * x->w;
  hipLaunchKernelGGL(norm_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, a);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_dropout_keep_bits(const es_view_t* x, const es_chain_t* ch, es_stream_t stream) {
  ES_CHECK_ARG(x && ch && ch->keep && ch->drop.enabled, "dropout_keep_bits: needs an enabled dropout with keep");
  ES_CHECK_ARG(x->c % 8 == 0, "dropout_keep_bits: C %% 8 == 0 required (C = %d)", x->c);
  es_fast_keep_bits(x, ch, (hipStream_t)stream);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_act_fwd(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_chain_t* ch,
                          const es_view_t* y, es_dtype_t ydt, void* yp, es_stream_t stream) {
  return es_norm_act_fwd(x, xdt, nullptr, ch, nullptr, ES_F32, nullptr, xp, y, ydt, yp, stream);
}

extern "C" int64_t es_norm_bwd_ws_bytes(const es_view_t* x, int kind, int groups) {
  View v = mkview(x);
  int cb, chunks; int64_t rows, per;
  colred_geometry(v, cb, chunks, rows, per);
  int64_t part = (int64_t)chunks * 3 * v.c * sizeof(float);
  const int fk = fast_kind(x, kind, groups);
  if (fk >= 0) part = std::max<int64_t>(part, es_fast_part_floats(x, fk) * (int64_t)sizeof(float));
  const int64_t ng = kind == ES_NORM_NONE ? 0 : stats_groups(x, kind, groups);
  return part + 2 * ng * (int64_t)sizeof(float) + 256;
}

extern "C" int es_norm_act_bwd(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_norm_t* nm,
                               const es_chain_t* ch, const es_view_t* dy, es_dtype_t dydt,
                               const void* dyp, const es_view_t* act_ref, es_dtype_t rdt,
                               const void* refp, const es_view_t* dx, es_dtype_t dxdt, void* dxp,
                               float beta, float* dgamma, float* dbeta, float* dsum, void* ws,
                               es_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  const int kind = nm ? nm->kind : ES_NORM_NONE;
  ES_CHECK_ARG(dsum == nullptr || x->c <= 1024, "norm_act_bwd: dsum needs C <= 1024");
  const int groups = nm ? nm->groups : 1;
  ES_CHECK_ARG(kind != ES_NORM_LN || (x->h == 1 && x->w == 1), "norm_act_bwd: LN needs (N,F,1,1) views");
  BwdIn b = mk_bwdin(x, xdt, xp, nm, ch);
  b.dy = mkview(dy); b.dyp = dyp; b.dybf = dydt == ES_BF16;
  if (refp) { b.ref = mkview(act_ref); b.refp = refp; b.refbf = rdt == ES_BF16; }
  BwdApply ap{};
  ap.b = b; ap.dx = mkview(dx); ap.dxp = dxp; ap.dxbf = dxdt == ES_BF16; ap.beta = beta; ap.csum = dsum;
  // deterministic mode: the generic apply's float-atomic channel sums are replaced by an ordered
  // column reduction of dx after the apply (below)
  float* det_dsum = nullptr;
  if (g_es_det && dsum) { det_dsum = dsum; ap.csum = nullptr; }
  const int64_t total = (int64_t)x->n * x->c * x->h * x->w;
  int cb, chunks; int64_t rows, per;
  colred_geometry(b.x, cb, chunks, rows, per);
  float* part = (float*)ws;
  int64_t part_floats = (int64_t)chunks * 3 * x->c;
  const int fk = fast_kind(x, kind, groups);
  const bool fast = fk >= 0 && !refp && beta == 0.f && xdt == dydt && dydt == dxdt && same_view(x, dy) &&
                    (dxp == nullptr || same_view(x, dx));
  if (fk >= 0) part_floats = std::max<int64_t>(part_floats, es_fast_part_floats(x, fk));
  float* g1 = part + part_floats;
  const int64_t ng = kind == ES_NORM_NONE ? 0 : stats_groups(x, kind, groups);
  float* g2 = g1 + ng;
  if (fast && fk > 0) {
    const int fchunks = es_fast_norm_bwd_reduce(x, fk, xdt, xp, dyp, nm, ch, part, st);
    hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3((unsigned)((ng + 255) / 256)), dim3(256), 0, st,
                       (const float*)part, x->n, fchunks, x->c, groups, (float)((x->c / groups) * x->h * x->w),
                       nm->gamma, g1, g2);
    if (dgamma || dbeta) {
      const int allc = x->n * fchunks;   // per-channel sums over every (n, chunk) partial
      launch_sums_finalize(st, (const float*)part, allc, x->c, mkcnt(1.f), nullptr, (float*)nullptr, (float*)nullptr, dbeta, dgamma, 1.f);
    }
    if (dxp) fast_dsum_finalize(x->c, es_fast_norm_bwd_apply(x, fk, xdt, xp, dyp, dxp, nm, ch, g1, g2, dsum, part, st),
                                part, dsum, st);
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  if (fast) {
    const int fchunks = es_fast_norm_bwd_reduce(x, 0, xdt, xp, dyp, nm, ch, part, st);
    launch_sums_finalize(st, (const float*)part, fchunks, x->c, mkcnt((float)rows, x), nm->gamma, g1, g2, dbeta, dgamma, 1.f);
    if (dxp) fast_dsum_finalize(x->c, es_fast_norm_bwd_apply(x, 0, xdt, xp, dyp, dxp, nm, ch, g1, g2, dsum, part, st),
                                part, dsum, st);
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  if (kind == ES_NORM_BN) {
    hipLaunchKernelGGL(colred_kernel<RED_BWD>, dim3(cb, chunks), dim3(256), 0, st, b, rows, per, part);
    launch_sums_finalize(st, (const float*)part, chunks, x->c, mkcnt((float)rows, x), nm->gamma, g1, g2, dbeta, dgamma, 1.f);
    ap.a1 = g1; ap.a2 = g2;
  } else if (kind == ES_NORM_GN || kind == ES_NORM_LN) {
    hipLaunchKernelGGL(segred_kernel<RED_BWD>, dim3((unsigned)ng), dim3(256), 0, st, b, 0.f, g1, g2);
    if (dgamma || dbeta) {
      hipLaunchKernelGGL(colred_kernel<RED_BWD>, dim3(cb, chunks), dim3(256), 0, st, b, rows, per, part);
      launch_sums_finalize(st, (const float*)part, chunks, x->c, mkcnt(1.f), nullptr, (float*)nullptr, (float*)nullptr, dbeta, dgamma, 1.f);
    }
    ap.a1 = g1; ap.a2 = g2;
  }
  if (dxp) hipLaunchKernelGGL(norm_bwd_apply_kernel, dim3(grid_for(total)), dim3(256), 0, st, ap);
  ES_CHECK_LAUNCH();
  if (det_dsum && dxp) return es_channel_sum(dx, dxdt, dxp, det_dsum, 1.f, part, stream);
  return ES_OK;
}

// BatchNorm backward whose reduction pass already ran in the producing dgrad's epilogue
// (es_conv2d_dgrad_bnred): finalize the sums partials, then the fast apply pass
extern "C" int es_norm_act_bwd_sums(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_norm_t* nm,
                                    const es_chain_t* ch, const es_view_t* dy, es_dtype_t dydt, const void* dyp,
                                    const es_view_t* dx, es_dtype_t dxdt, void* dxp, const float* sums_part,
                                    int chunks, float* dgamma, float* dbeta, float* dsum, void* ws,
                                    es_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  ES_CHECK_ARG(nm && nm->kind == ES_NORM_BN && sums_part && chunks > 0 && dxp, "norm_act_bwd_sums: bad args");
  ES_CHECK_ARG(dsum == nullptr || x->c <= 1024, "norm_act_bwd_sums: dsum needs C <= 1024");
  const int fk = fast_kind(x, ES_NORM_BN, 1);
  ES_CHECK_ARG(fk == 0 && xdt == dydt && dydt == dxdt && same_view(x, dy) && same_view(x, dx),
               "norm_act_bwd_sums: needs the dense NHWC fast path");
  View xv = mkview(x);
  int cb, cchunks; int64_t rows, per;
  colred_geometry(xv, cb, cchunks, rows, per);
  const int64_t part_floats = std::max<int64_t>((int64_t)cchunks * 3 * x->c, es_fast_part_floats(x, 0));
  float* part = (float*)ws;
  float* g1 = part + part_floats;
  float* g2 = g1 + x->c;
  launch_sums_finalize(st, sums_part, chunks, x->c, mkcnt((float)rows, x), nm->gamma, g1, g2, dbeta, dgamma, 1.f);
  fast_dsum_finalize(x->c, es_fast_norm_bwd_apply(x, 0, xdt, xp, dyp, dxp, nm, ch, g1, g2, dsum, part, st), part,
                     dsum, st);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int64_t es_channel_sum_ws_bytes(const es_view_t* x) {
  View v = mkview(x);
  int cb, chunks; int64_t rows, per;
  colred_geometry(v, cb, chunks, rows, per);
  return (int64_t)chunks * 3 * v.c * sizeof(float);
}

extern "C" int es_channel_sum(const es_view_t* x, es_dtype_t xdt, const void* xp, float* out,
                              float beta, void* ws, es_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  BwdIn b = mk_bwdin(x, xdt, xp, nullptr, nullptr);
  int cb, chunks; int64_t rows, per;
  colred_geometry(b.x, cb, chunks, rows, per);
  if (x->c == 1 && rows < (1ll << 31)) {
    // one channel (bias of a 1-output conv): every thread of the colred geometry's chunks sums
    // rows, instead of 63 of every 64 lanes idling
    const int nb = std::min<int>(chunks, (int)((rows + 255) / 256));
    hipLaunchKernelGGL(sum1_kernel, dim3(nb), dim3(256), 0, st, b, (int)rows, (float*)ws);
    // (a single thread summing thousands of partials took ~75 us: a block for nb > 32)
    launch_sums_finalize(st, (const float*)ws, nb, 1, mkcnt(1.f), nullptr, (float*)nullptr, (float*)nullptr, out,
                         (float*)nullptr, beta);
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  hipLaunchKernelGGL(colred_kernel<RED_SUM>, dim3(cb, chunks), dim3(256), 0, st, b, rows, per, (float*)ws);
  launch_sums_finalize(st, (const float*)ws, chunks, x->c, mkcnt(1.f), nullptr, (float*)nullptr, (float*)nullptr, out, (float*)nullptr, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

// ------------------------------------------------------------------------ data-parallel BatchNorm
extern "C" int es_norm_stats_merge(const float* part, int chunks, int C, float* out, es_stream_t stream) {
  ES_CHECK_ARG(part && out && chunks > 0 && C > 0, "norm_stats_merge: bad arguments");
  hipLaunchKernelGGL(stats_merge_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, part, chunks, C, out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_norm_stats_local(const es_view_t* x, es_dtype_t xdt, const void* xp, void* ws, float* out,
                                   es_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  ES_CHECK_ARG(ws != nullptr && out != nullptr, "norm_stats_local: workspace / out");
  es_norm_t nm{ES_NORM_BN, 1, nullptr, nullptr, nullptr, nullptr};
  BwdIn b = mk_bwdin(x, xdt, xp, &nm, nullptr);
  const int fk = fast_kind(x, ES_NORM_BN, 1);
  int cb, chunks; int64_t rows, per;
  colred_geometry(b.x, cb, chunks, rows, per);
  if (fk == 0)
    chunks = es_fast_norm_stats(x, 0, xdt, xp, (float*)ws, st);
  else
    hipLaunchKernelGGL(colred_kernel<RED_STATS>, dim3(cb, chunks), dim3(256), 0, st, b, rows, per, (float*)ws);
  hipLaunchKernelGGL(stats_merge_kernel, dim3(x->c), dim3(256), 0, st, (const float*)ws, chunks, x->c, out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_norm_bwd_sync(int phase, const es_view_t* x, es_dtype_t xdt, const void* xp, const es_norm_t* nm,
                                const es_chain_t* ch, const es_view_t* dy, es_dtype_t dydt, const void* dyp,
                                const es_view_t* dx, es_dtype_t dxdt, void* dxp, float* sums, float cnt,
                                const float* cnt_mul, float* dgamma, float* dbeta, float* dsum, void* ws,
                                es_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  ES_CHECK_ARG(nm && nm->kind == ES_NORM_BN, "norm_bwd_sync: BatchNorm only");
  ES_CHECK_ARG(phase == 0 || phase == 1, "norm_bwd_sync: phase 0 (sums) or 1 (apply)");
  ES_CHECK_ARG(sums && ws, "norm_bwd_sync: sums / workspace");
  ES_CHECK_ARG(dsum == nullptr || x->c <= 1024, "norm_bwd_sync: dsum needs C <= 1024");
  BwdIn b = mk_bwdin(x, xdt, xp, nm, ch);
  b.dy = mkview(dy); b.dyp = dyp; b.dybf = dydt == ES_BF16;
  int cb, chunks; int64_t rows, per;
  colred_geometry(b.x, cb, chunks, rows, per);
  float* part = (float*)ws;
  int64_t part_floats = (int64_t)chunks * 3 * x->c;
  const int fk = fast_kind(x, ES_NORM_BN, 1);
  const bool fast = fk == 0 && xdt == dydt && dydt == dxdt && same_view(x, dy) && (dxp == nullptr || same_view(x, dx));
  if (fk >= 0) part_floats = std::max<int64_t>(part_floats, es_fast_part_floats(x, fk));
  float* g1 = part + part_floats;
  float* g2 = g1 + x->c;
  if (phase == 0) {
    int nchunks = chunks;
    if (fast)
      nchunks = es_fast_norm_bwd_reduce(x, 0, xdt, xp, dyp, nm, ch, part, st);
    else
      hipLaunchKernelGGL(colred_kernel<RED_BWD>, dim3(cb, chunks), dim3(256), 0, st, b, rows, per, part);
    // raw per-channel sums s1 = sum dnorm, s2 = sum dnorm*xhat (+ the local dbeta / dgamma)
    launch_sums_finalize(st, (const float*)part, nchunks, x->c, mkcnt(1.f), nullptr, sums, sums + x->c, dbeta, dgamma, 1.f);
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  ES_CHECK_ARG(cnt > 0.f && dxp != nullptr, "norm_bwd_sync: apply needs cnt > 0 and dx");
  hipLaunchKernelGGL(bn_scale_sums_kernel, dim3((x->c + 255) / 256), dim3(256), 0, st, (const float*)sums, x->c,
                     cnt, cnt_mul, nm->gamma, g1, g2);
  if (fast) {
    fast_dsum_finalize(x->c, es_fast_norm_bwd_apply(x, 0, xdt, xp, dyp, dxp, nm, ch, g1, g2, dsum, part, st),
                       part, dsum, st);
  } else {
    BwdApply ap{};
    ap.b = b; ap.dx = mkview(dx); ap.dxp = dxp; ap.dxbf = dxdt == ES_BF16; ap.beta = 0.f; ap.csum = dsum;
    ap.a1 = g1; ap.a2 = g2;
    // deterministic mode: as in es_norm_act_bwd, the apply's float-atomic channel sums are replaced
    // by an ordered column reduction of dx after the apply
    if (g_es_det && dsum) ap.csum = nullptr;
    const int64_t total = (int64_t)x->n * x->c * x->h * x->w;
    hipLaunchKernelGGL(norm_bwd_apply_kernel, dim3(grid_for(total)), dim3(256), 0, st, ap);
    ES_CHECK_LAUNCH();
    if (g_es_det && dsum) return es_channel_sum(dx, dxdt, dxp, dsum, 1.f, part, stream);
  }
  ES_CHECK_LAUNCH();
  return ES_OK;
}
