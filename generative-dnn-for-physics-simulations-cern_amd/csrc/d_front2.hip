// Fused discriminator front, BOTH conv blocks (conv_layers.0 .. conv_layers.7 of
// neutron/discriminator.py:11-24 and proton/discriminator.py:121-134), one workgroup per image:
//
//   block 1  SNconv 3x3 1->32 -> GroupNorm(8, 32) -> LeakyReLU -> MaxPool 2x2        (VALU)
//   block 2  SNconv 3x3 32->16 -> GroupNorm(8, 16) -> LeakyReLU -> MaxPool (ph, pw)  (MFMA)
//   -> flattened in the reference's view(B, -1) (NCHW) order straight into the fc1 input rows.
//
// Unfused, block 2 was five launches per forward (the 32->16 conv, GN statistics, GN apply, pool,
// the copy into the fc1 rows) and eight per backward (pool / GN backward passes, the conv's dgrad
// and wgrad, the bias and GN-affine reductions), each a few-GFLOP or few-MB kernel far below any
// roofline (conv_layers.4 wgrad: 217 us for 3.4 GFLOP at B = 1024).  Here the pooled block-1 map
// (<= 448 pixels x 32 channels) and the block-2 conv map (<= 384 x 16) live in LDS; the 32->16 conv
// is an implicit GEMM from LDS on v_mfma_f32_16x16x4_f32 (exact fp32 products):
//   forward  M = conv-2 pixels, N = 16, K = (tap, channel) = 288 in 72 steps of 4
//   wgrad    M = 16 (out channel), N = (tap, channel) = 288, K = conv-2 pixels
//   dgrad    M = pooled block-1 pixels, N = 32, K = (tap, out channel) = 144
// A fragments are 16-byte LDS reads (4 consecutive k) feeding four MFMAs (the B registers use
// the same k permutation); the operand images use pixel strides of 36 / 20 floats, so the 16 rows
// of one ds_read_b128 cover distinct banks.
//
//   forward  reads the image; writes the features, the GN statistics [N][32] (GN1 mean / invstd,
//            GN2 mean / invstd) and (training) a per-image save of the pooled block-1 map, the
//            block-1 conv values at the pool argmaxes and the block-2 conv map (es_dfront2_save_floats)
//   backward reads the image, the save, the feature gradient and the statistics (the block-1 conv
//            map is recomputed from the image in LDS: 9 MACs per value, cheaper than its HBM round
//            trip; the argmaxes with the forward's code); writes the image gradient
//            (optional: the generator step) and per-image partials of every weight gradient
//            (optional: the discriminator step), summed over the images by a second launch
//            (deterministic, no atomics).
// GroupNorm statistics and backward sums are reduced in a fixed order (shuffles, then waves), so
// results are run-to-run deterministic.
#include "d_front_common.h"

namespace {

using namespace dfront;

constexpr int K2 = 16;                      // block-2 conv output channels
constexpr int G2 = 8;                       // block-2 GroupNorm groups (channel pairs)
constexpr int MAXP1 = 448;                  // pooled block-1 pixels (neutron 21x21, proton 27x14)
constexpr int P1S = FK + 4;                 // p1 pixel stride (floats): 16-byte rows, b128 reads conflict-free
constexpr int MAXH2 = 384;                  // block-2 conv pixels (neutron 19x19, proton 25x12)
constexpr int H2S = K2 + 4;                 // h2 pixel stride (floats), likewise
constexpr int NWT2 = K2 * FK * TAPS;        // 4608 block-2 weights
// per-image partials: dW2 [16][32][9] | db2 | dg2 | dbe2 | dW1 [32][9] | db1 | dg1 | dbe1
constexpr int O_DB2 = NWT2, O_DG2 = O_DB2 + K2, O_DBE2 = O_DG2 + K2, O_W1 = O_DBE2 + K2;
constexpr int O_DB1 = O_W1 + FK * TAPS, O_DG1 = O_DB1 + FK, O_DBE1 = O_DG1 + FK;
constexpr int NPART2 = O_DBE1 + FK;         // 5040
constexpr int RFL = TAPS * MAXOUT;          // LDS region R (floats): h2 | dn, later e_rs planes
static_assert(2 * MAXH2 * H2S <= RFL, "h2 + dn must fit in R");
static_assert(NW * 8 * (CPG * TAPS + CPG) <= RFL, "quad_sum scratch must fit in R");

struct F2Args {
  const float* img; int64_t is[4];
  int H, W, Ho, Wo, Hp, Wp;                 // image, block-1 conv map, pooled block-1 map
  int Ho2, Wo2, Hq, Wq;                     // block-2 conv map, pooled block-2 map
  es_dfront2_params_t p;
  float* stats;                             // [N][32]
  float* feat; int64_t fs;                  // forward output
  const float* dfeat; int64_t dfs;          // backward input
  float* dx; int64_t dxs[4];                // image gradient (or NULL)
  float* part;                              // [N][NPART2] (or NULL)
  float* save; int64_t sv;                  // [N][sv]: p1 [NP1][32] | hv1 [NP1][32] | h2 [NO2][16]
  long long* probe;                         // phase timestamps of workgroup 0 (ES_DF2_PROBE builds)
};

long long* g_probe = nullptr;   // host: es_dfront2_set_probe

#ifdef ES_DF2_PROBE
#define PROBE(a, i) do { if ((a).probe && blockIdx.x == 0 && threadIdx.x == 0) (a).probe[i] = wall_clock64(); } while (0)
#else
#define PROBE(a, i) do { } while (0)
#endif

// Chan merge of (count, mean, M2) triples
__device__ __forceinline__ void chan_merge(float& n, float& m, float& M, float nb, float mb, float Mb) {
  const float nt = n + nb;
  if (nt > 0.f) {
    const float d = mb - m, f = nb / nt;
    m += d * f;
    M += Mb + d * d * n * f;
  }
  n = nt;
}

// GroupNorm(8, 32) statistics of the image's block-1 conv map in ONE pass: per window the 16
// values (4 positions x the quad's 4 channels) give (16, mean, M2), Chan-merged over the thread's
// windows, the 64 window streams of the group (shuffles) and the 8 waves (fixed order)
__device__ __forceinline__ void block1_stats(const F2Args& a, const float* im, const Quad& q, int u, float* red,
                                             float& mu, float& istd) {
  const int NP = a.Hp * a.Wp;
  const int g = threadIdx.x & 7, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float n_ = 0.f, m_ = 0.f, M_ = 0.f;
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
    float s = 0.f;
#pragma unroll
    for (int pos = 0; pos < 4; ++pos)
#pragma unroll
      for (int c = 0; c < CPG; ++c) s += v[pos][c];
    const float wm = s * (1.f / 16.f);
    float wq = 0.f;
#pragma unroll
    for (int pos = 0; pos < 4; ++pos)
#pragma unroll
      for (int c = 0; c < CPG; ++c) {
        const float d = v[pos][c] - wm;
        wq = fmaf(d, d, wq);
      }
    chan_merge(n_, m_, M_, 16.f, wm, wq);
  }
#pragma unroll
  for (int o = 8; o < 64; o <<= 1)
    chan_merge(n_, m_, M_, __shfl_xor(n_, o, 64), __shfl_xor(m_, o, 64), __shfl_xor(M_, o, 64));
  __syncthreads();                                   // red may still be read by a previous use
  if (lane < 8) {
    red[(wid * 8 + lane) * 3 + 0] = n_;
    red[(wid * 8 + lane) * 3 + 1] = m_;
    red[(wid * 8 + lane) * 3 + 2] = M_;
  }
  __syncthreads();
  n_ = red[g * 3];
  m_ = red[g * 3 + 1];
  M_ = red[g * 3 + 2];
#pragma unroll
  for (int w = 1; w < NW; ++w) chan_merge(n_, m_, M_, red[(w * 8 + g) * 3], red[(w * 8 + g) * 3 + 1], red[(w * 8 + g) * 3 + 2]);
  mu = m_;
  istd = rsqrtf(M_ / n_ + a.p.eps1);
}

// window argmax of the block-1 pool (first max in row-major window order, NaN wins, as torch)
__device__ __forceinline__ int block1_argmax(const float (&v)[4][CPG], int c, const Quad& q, float mu, float istd,
                                             float slope, float& best) {
  int bi = 0;
  best = lrelu(fmaf((v[0][c] - mu) * istd, q.gm[c], q.bt[c]), slope);
#pragma unroll
  for (int pos = 1; pos < 4; ++pos) {
    const float y = lrelu(fmaf((v[pos][c] - mu) * istd, q.gm[c], q.bt[c]), slope);
    if (y > best || (isnan(y) && !isnan(best))) { best = y; bi = pos; }
  }
  return bi;
}

// block-1 output into LDS (p1[pix * P1S + channel], one 16-byte store per window and quad) and,
// when saving, to the image's save: p1 and the conv values at the argmaxes (hv1)
__device__ __forceinline__ void block1_out(const F2Args& a, const float* im, const Quad& q, int g, int u, float mu,
                                           float istd, float* p1, float* sp1, float* shv) {
  const int NP = a.Hp * a.Wp;
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
    float best[CPG], hv[CPG];
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      const int bi = block1_argmax(v, c, q, mu, istd, a.p.slope, best[c]);
      hv[c] = v[0][c];
#pragma unroll
      for (int pos = 1; pos < 4; ++pos) hv[c] = bi == pos ? v[pos][c] : hv[c];
    }
    const float4 b4 = make_float4(best[0], best[1], best[2], best[3]);
    *(float4*)(p1 + pp * P1S + g * CPG) = b4;
    if (sp1) {
      *(float4*)(sp1 + pp * FK + g * CPG) = b4;
      *(float4*)(shv + pp * FK + g * CPG) = make_float4(hv[0], hv[1], hv[2], hv[3]);
    }
  }
}

// ---------------------------------------------------------------------------- block-2 conv
// h2[p][k] = b2[k] + sum_{tap, c} p1[(oy + tr, ox + ts)][c] * W2[k][c][tap] / sigma2 for the wave's
// row tiles rt0, rt0 + 8, ... (J of them, independent accumulators).  Per (tap, 16-channel block)
// lane (row r16 = pixel, kq) reads channels 4 kq .. 4 kq + 3 with one 16-byte LDS read and feeds
// four MFMAs (MFMA t: k = 4 kq + t); B: the lane's weight registers in the same order.
constexpr int NB2 = TAPS * 2;               // (tap, 16-channel block) steps of the block-2 forward
template <int J>
__device__ __forceinline__ void conv2_tiles(const F2Args& a, const float* p1, float* h2, const float (&bw)[NB2 * 4],
                                            int rt0) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  const int NO2 = a.Ho2 * a.Wo2;
  int base[J];
  f32x4 acc[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int p = min((rt0 + j * NW) * 16 + r16, NO2 - 1);
    const int oy = p / a.Wo2, ox = p - oy * a.Wo2;
    base[j] = (oy * a.Wp + ox) * P1S + kq * 4;
    acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int blk = 0; blk < NB2; ++blk) {
    const int tap = blk >> 1;
    const int off = ((tap / 3) * a.Wp + tap % 3) * P1S + (blk & 1) * 16;
    float4 av[J];
#pragma unroll
    for (int j = 0; j < J; ++j) av[j] = *(const float4*)(p1 + base[j] + off);
    // tiles innermost: consecutive MFMAs write different accumulators (no dependent issue)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].x, bw[blk * 4 + 0], acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].y, bw[blk * 4 + 1], acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].z, bw[blk * 4 + 2], acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].w, bw[blk * 4 + 3], acc[j], 0, 0, 0);
  }
  // D layout: lane holds rows kq*4 + i, column r16
  const float bias = a.p.b2 ? a.p.b2[r16] : 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = (rt0 + j * NW) * 16 + kq * 4 + i;
      if (p < NO2) h2[p * H2S + r16] = acc[j][i] + bias;
    }
}

__device__ __forceinline__ void block2_conv(const F2Args& a, const float* p1, float* h2) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float inv = a.p.sigma2 ? 1.f / a.p.sigma2[0] : 1.f;   // as es_pack_conv_weight
  float bw[NB2 * 4];
#pragma unroll
  for (int blk = 0; blk < NB2; ++blk)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int tap = blk >> 1, ch = (blk & 1) * 16 + (lane >> 4) * 4 + t;
      bw[blk * 4 + t] = a.p.w2[((lane & 15) * FK + ch) * TAPS + tap] * inv;
    }
  const int NT = (a.Ho2 * a.Wo2 + 15) >> 4;                    // <= 24 (host check)
  const int nj = wid < NT ? (NT - wid + NW - 1) / NW : 0;        // wave-uniform
  if (nj >= 3) conv2_tiles<3>(a, p1, h2, bw, wid);
  else if (nj == 2) conv2_tiles<2>(a, p1, h2, bw, wid);
  else if (nj == 1) conv2_tiles<1>(a, p1, h2, bw, wid);
}

// GroupNorm(8, 16) statistics of the block-2 map (groups = channel pairs), two passes.  Thread t:
// channel c = t & 15, pixel stream t >> 4 (32 streams); every thread returns its group's values.
__device__ __forceinline__ void block2_stats(const F2Args& a, const float* h2, float* red, float& mu, float& istd) {
  const int c = threadIdx.x & 15, s = threadIdx.x >> 4, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int NO2 = a.Ho2 * a.Wo2;
  const float cnt = 2.f * NO2;
  float v = 0.f;
  for (int p = s; p < NO2; p += 32) v += h2[p * H2S + c];
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  __syncthreads();
  if (lane < 16) red[wid * 16 + lane] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += red[w * 16 + c];
  mu = t / cnt;
  float m2 = 0.f;
  for (int p = s; p < NO2; p += 32) {
    const float d = h2[p * H2S + c] - mu;
    m2 = fmaf(d, d, m2);
  }
  m2 += __shfl_xor(m2, 1, 64);
  m2 += __shfl_xor(m2, 16, 64);
  m2 += __shfl_xor(m2, 32, 64);
  __syncthreads();
  if (lane < 16) red[wid * 16 + lane] = m2;
  __syncthreads();
  t = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += red[w * 16 + c];
  istd = rsqrtf(t / cnt + a.p.eps2);
}

// pool-2 window (y, x) of channel c: first max in row-major order of LeakyReLU(GN2(h2)); returns
// the pixel, its conv value h and its GN output av
__device__ __forceinline__ float block2_window(const F2Args& a, const float* h2, int c, int y, int x, float mu,
                                               float istd, float gm, float bt, int& bp, float& bh, float& ba) {
  bp = (y * a.p.ph) * a.Wo2 + x * a.p.pw;
  bh = h2[bp * H2S + c];
  ba = fmaf((bh - mu) * istd, gm, bt);
  float best = lrelu(ba, a.p.slope);
  for (int dy = 0; dy < a.p.ph; ++dy)
    for (int dx = 0; dx < a.p.pw; ++dx) {
      if (dy == 0 && dx == 0) continue;
      const int p = (y * a.p.ph + dy) * a.Wo2 + x * a.p.pw + dx;
      const float h = h2[p * H2S + c];
      const float av = fmaf((h - mu) * istd, gm, bt);
      const float yv = lrelu(av, a.p.slope);
      if (yv > best || (isnan(yv) && !isnan(best))) { best = yv; bp = p; bh = h; ba = av; }
    }
  return best;
}

__global__ void __launch_bounds__(FT) dfront2_fwd_kernel(F2Args a) {
  __shared__ float im[MAXPIX];
  __shared__ __attribute__((aligned(16))) float p1[MAXP1 * P1S];
  __shared__ float h2[MAXH2 * H2S];
  __shared__ float red[NW * 24];
  __shared__ float st[4 * FG];                // GN1 mean, invstd, GN2 mean, invstd
  const int n = blockIdx.x, g = threadIdx.x & 7, u = threadIdx.x >> 3;
  if (n >= live_rows(a.p.rows, gridDim.x)) return;   // a padding image (dynamic rows)
  const int NP1 = a.Hp * a.Wp, NO2 = a.Ho2 * a.Wo2;
  float* sv = a.save ? a.save + (int64_t)n * a.sv : nullptr;
  Quad q;
  load_quad_p(a.p.w1, a.p.sigma1, a.p.b1, a.p.g1, a.p.be1, g, q);
  stage_image_p(a.img, a.is, a.H, a.W, n, im);
  __syncthreads();
  float mu1, is1;
  PROBE(a, 10);
  block1_stats(a, im, q, u, red, mu1, is1);
  if (threadIdx.x < 8) { st[g] = mu1; st[FG + g] = is1; }
  PROBE(a, 11);
  block1_out(a, im, q, g, u, mu1, is1, p1, sv, sv ? sv + NP1 * FK : nullptr);
  __syncthreads();
  PROBE(a, 12);
  block2_conv(a, p1, h2);
  __syncthreads();
  PROBE(a, 13);
  if (sv) {
    float* sh2 = sv + 2 * NP1 * FK;
    for (int i = threadIdx.x; i < NO2 * K2; i += FT) sh2[i] = h2[(i >> 4) * H2S + (i & 15)];
  }
  float mu2, is2;
  block2_stats(a, h2, red, mu2, is2);
  if (threadIdx.x < 16 && (threadIdx.x & 1) == 0) {
    st[2 * FG + (threadIdx.x >> 1)] = mu2;
    st[3 * FG + (threadIdx.x >> 1)] = is2;
  }
  __syncthreads();
  if (threadIdx.x < 4 * FG) a.stats[(int64_t)n * 4 * FG + threadIdx.x] = st[threadIdx.x];
  // pool 2 -> features, f = c * Hq * Wq + y * Wq + x (NCHW flatten)
  const int HWq = a.Hq * a.Wq, F = K2 * HWq;
  float* out = a.feat + (int64_t)n * a.fs;
  for (int f = threadIdx.x; f < F; f += FT) {
    const int c = f / HWq, r = f - c * HWq, y = r / a.Wq, x = r - y * a.Wq;
    const int gg = c >> 1;
    int bp; float bh, ba;
    out[f] = block2_window(a, h2, c, y, x, st[2 * FG + gg], st[3 * FG + gg], a.p.g2 ? a.p.g2[c] : 1.f,
                           a.p.be2 ? a.p.be2[c] : 0.f, bp, bh, ba);
  }
  PROBE(a, 14);
}

// ---------------------------------------------------------------------------- backward pieces
// dW2[k][c][tap] = sum_p dh2[p][k] * p1[(oy + tr, ox + ts)][c]: column tiles t = wave + 8j of
// (tap = t >> 1, channels (t & 1) * 16 ..), K over the conv-2 pixels (rows >= NO2 of dh2 are 0)
template <int J>
__device__ __forceinline__ void wgrad2_tiles(const F2Args& a, const float* p1, const float* dh2, float* part) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r16 = lane & 15, kq = lane >> 4;
  const int NO2 = a.Ho2 * a.Wo2, nks = (NO2 + 3) >> 2;
  int coff[J];
  f32x4 acc[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = wid + j * NW, tap = t >> 1;
    coff[j] = ((tap / 3) * a.Wp + tap % 3) * P1S + (t & 1) * 16 + r16;
    acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  int p = kq, oy = kq / a.Wo2, ox = kq - oy * a.Wo2;
  for (int ks = 0; ks < nks; ++ks) {
    const float av = dh2[p * H2S + r16];                   // A[k = r16][pixel p]
    const int pb = p < NO2 ? (oy * a.Wp + ox) * P1S : 0;    // (padding rows: av = 0, any valid address)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, p1[pb + coff[j]], acc[j], 0, 0, 0);
    p += 4;
    ox += 4;
    while (ox >= a.Wo2) { ox -= a.Wo2; ++oy; }
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = wid + j * NW, tap = t >> 1, ch = (t & 1) * 16 + r16;
#pragma unroll
    for (int i = 0; i < 4; ++i) part[((kq * 4 + i) * FK + ch) * TAPS + tap] = acc[j][i];
  }
}

// dp1[q][c] = sum_{tap, k} dh2[(iy - tr, ix - ts)][k] * W2[k][c][tap] / sigma2 (0 outside the
// conv-2 map).  Row tiles of pooled block-1 pixels, two at a time, both 16-channel column tiles;
// per tap one 16-byte read of the lane's 4 channels (k = 4 kq + t) feeds 8 MFMAs.
__device__ __forceinline__ void dgrad2(const F2Args& a, const float* dh2, float* dp1) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r16 = lane & 15, kq = lane >> 4;
  const float inv = a.p.sigma2 ? 1.f / a.p.sigma2[0] : 1.f;
  float bd[TAPS][4][2];
#pragma unroll
  for (int tap = 0; tap < TAPS; ++tap)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) bd[tap][t][j] = a.p.w2[((kq * 4 + t) * FK + j * 16 + r16) * TAPS + tap] * inv;
  const int NP1 = a.Hp * a.Wp, NT1 = (NP1 + 15) >> 4;
  for (int rt0 = wid; rt0 < NT1; rt0 += 2 * NW) {   // tiles rt0 and rt0 + 8 (if any)
    const bool two = rt0 + NW < NT1;                 // wave-uniform
    int iy[2], ix[2];
    f32x4 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int qq = min((rt0 + m * NW) * 16 + r16, NP1 - 1);
      iy[m] = qq / a.Wp;
      ix[m] = qq - iy[m] * a.Wp;
      acc[m][0] = acc[m][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      const int tr = tap / 3, ts = tap % 3;
      float4 av[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int oy = iy[m] - tr, ox = ix[m] - ts;
        const bool ok = (unsigned)oy < (unsigned)a.Ho2 && (unsigned)ox < (unsigned)a.Wo2;
        const float4 v = *(const float4*)(dh2 + (ok ? oy * a.Wo2 + ox : 0) * H2S + kq * 4);
        av[m] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const float e0[4] = {av[0].x, av[0].y, av[0].z, av[0].w};
      const float e1[4] = {av[1].x, av[1].y, av[1].z, av[1].w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(e0[t], bd[tap][t][0], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(e0[t], bd[tap][t][1], acc[0][1], 0, 0, 0);
        if (two) {
          acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(e1[t], bd[tap][t][0], acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(e1[t], bd[tap][t][1], acc[1][1], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (m == 1 && !two) break;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qq = (rt0 + m * NW) * 16 + kq * 4 + i;
        if (qq < NP1) {
          dp1[qq * P1S + r16] = acc[m][0][i];
          dp1[qq * P1S + 16 + r16] = acc[m][1][i];
        }
      }
    }
  }
}

template <bool WDX, bool WW>
__global__ void __launch_bounds__(FT) dfront2_bwd_kernel(F2Args a) {
  __shared__ float im[MAXPIX];
  __shared__ __attribute__((aligned(16))) float p1[MAXP1 * P1S];   // block-1 output, then its gradient
  __shared__ __attribute__((aligned(16))) float R[RFL];            // h2 (then dh2) | dn; later e_rs / scratch
  __shared__ float red[NW * 24];
  __shared__ float kk[2 * G2];                // GN2 backward: mean(dn), mean(dn * xhat) per group
  float* h2 = R;
  float* dn = R + MAXH2 * H2S;
  const int n = blockIdx.x, g = threadIdx.x & 7, u = threadIdx.x >> 3;
  if (n >= live_rows(a.p.rows, gridDim.x)) return;   // a padding image (dynamic rows; no partial)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* part = WW ? a.part + (int64_t)n * NPART2 : nullptr;
  Quad q;
  load_quad_p(a.p.w1, a.p.sigma1, a.p.b1, a.p.g1, a.p.be1, g, q);
  stage_image_p(a.img, a.is, a.H, a.W, n, im);
  const float* st = a.stats + (int64_t)n * 4 * FG;
  const float mu1 = st[g], is1 = st[FG + g];
  for (int i = threadIdx.x; i < MAXH2 * H2S; i += FT) dn[i] = 0.f;
  // the forward's save: pooled block-1 map -> p1, block-2 conv map -> h2
  const int NP1 = a.Hp * a.Wp, NO2 = a.Ho2 * a.Wo2;
  const float* sv = a.save + (int64_t)n * a.sv;
  const float* shv = sv + NP1 * FK;
  PROBE(a, 0);
  for (int i = threadIdx.x; i < NP1 * (FK / 4); i += FT)
    *(float4*)(p1 + (i >> 3) * P1S + (i & 7) * 4) = ((const float4*)sv)[i];
  for (int i = threadIdx.x; i < NO2 * (K2 / 4); i += FT)
    *(float4*)(h2 + (i >> 2) * H2S + (i & 3) * 4) = ((const float4*)(sv + 2 * NP1 * FK))[i];
  __syncthreads();
  PROBE(a, 1);
  PROBE(a, 2);
  const float cnt2 = 2.f * NO2;

  // (1) pool-2 routing and the GN2 backward sums.  Thread t: channel c = t >> 5 (wave w holds the
  // channels 2w, 2w + 1 = group w), pooled outputs t & 31, +32, ...
  {
    const int c = threadIdx.x >> 5, l32 = threadIdx.x & 31, gg = c >> 1;
    const float m2 = st[2 * FG + gg], i2 = st[3 * FG + gg];
    const float gm = a.p.g2 ? a.p.g2[c] : 1.f, bt = a.p.be2 ? a.p.be2[c] : 0.f;
    const int HWq = a.Hq * a.Wq;
    const float* dfe = a.dfeat + (int64_t)n * a.dfs + c * HWq;
    float sdn = 0.f, sdx = 0.f, sg = 0.f, sb = 0.f;
    for (int r = l32; r < HWq; r += 32) {
      const int y = r / a.Wq, x = r - y * a.Wq;
      int bp; float bh, ba;
      block2_window(a, h2, c, y, x, m2, i2, gm, bt, bp, bh, ba);
      const float dout = dfe[r];
      const float dact = ba > 0.f ? dout : dout * a.p.slope;
      const float xh = (bh - m2) * i2;
      const float dnv = dact * gm;
      dn[bp * H2S + c] = dnv;
      sdn += dnv;
      sdx = fmaf(dnv, xh, sdx);
      sg = fmaf(dact, xh, sg);
      sb += dact;
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      sdn += __shfl_xor(sdn, o, 64);
      sdx += __shfl_xor(sdx, o, 64);
      sg += __shfl_xor(sg, o, 64);
      sb += __shfl_xor(sb, o, 64);
    }
    if (WW && l32 == 0) { part[O_DG2 + c] = sg; part[O_DBE2 + c] = sb; }
    sdn += __shfl_xor(sdn, 32, 64);
    sdx += __shfl_xor(sdx, 32, 64);
    if (lane == 0) { kk[gg] = sdn / cnt2; kk[G2 + gg] = sdx / cnt2; }
  }
  __syncthreads();
  // (2) dense GN2 backward: dh2 = istd (dn - mean(dn) - xhat mean(dn xhat)) over h2's slots; rows
  // NO2.. zeroed (the wgrad's K padding); conv-2 bias gradient = sum of dh2
  {
    const int c = threadIdx.x & 15, s = threadIdx.x >> 4, gg = c >> 1;
    const float m2 = st[2 * FG + gg], i2 = st[3 * FG + gg], k1 = kk[gg], k2 = kk[G2 + gg];
    float sb = 0.f;
    for (int p = s; p < NO2; p += 32) {
      const float xh = (h2[p * H2S + c] - m2) * i2;
      const float d = i2 * (dn[p * H2S + c] - k1 - xh * k2);
      h2[p * H2S + c] = d;
      sb += d;
    }
    for (int p = NO2 + s; p < MAXH2; p += 32) h2[p * H2S + c] = 0.f;
    if (WW) {
      sb += __shfl_xor(sb, 16, 64);
      sb += __shfl_xor(sb, 32, 64);
      if (lane < 16) red[wid * 16 + lane] = sb;
    }
  }
  __syncthreads();
  if (WW && threadIdx.x < K2) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w * 16 + threadIdx.x];
    part[O_DB2 + threadIdx.x] = t;
  }
  PROBE(a, 3);
  // (3) block-2 weight gradient (18 column tiles over 8 waves)
  if (WW) {
    const int nj = (18 - wid + NW - 1) / NW;
    if (nj == 3) wgrad2_tiles<3>(a, p1, h2, part);
    else wgrad2_tiles<2>(a, p1, h2, part);
  }
  __syncthreads();                            // p1 read by the wgrad before the dgrad overwrites it
  PROBE(a, 4);
  // (4) block-2 input gradient into p1's slots
  dgrad2(a, h2, p1);
  __syncthreads();
  PROBE(a, 5);

  // (5) block-1 backward (dfront_bwd_kernel's passes, dpooled from LDS, argmax recomputed)
  const int NP = a.Hp * a.Wp;
  const float cnt1 = (float)(CPG * a.Ho * a.Wo);
  float r[2 + 2 * CPG];
#pragma unroll
  for (int i = 0; i < 2 + 2 * CPG; ++i) r[i] = 0.f;
  for (int pp = u; pp < NP; pp += FT / 8) {
    const float4 h4 = *(const float4*)(shv + pp * FK + g * CPG);   // conv values at the argmaxes
    const float hvs[CPG] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      const float xh = (hvs[c] - mu1) * is1;
      const float av = fmaf(xh, q.gm[c], q.bt[c]);
      const float dvc = p1[pp * P1S + g * CPG + c];
      const float da = av > 0.f ? dvc : dvc * a.p.slope;
      const float dnv = da * q.gm[c];
      r[0] += dnv;
      r[1] = fmaf(dnv, xh, r[1]);
      r[2 + c] = fmaf(da, xh, r[2 + c]);
      r[2 + CPG + c] += da;
    }
  }
  quad_sum(r, R);
  if (WW && u == 0) {
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      part[O_DG1 + g * CPG + c] = r[2 + c];
      part[O_DBE1 + g * CPG + c] = r[2 + CPG + c];
    }
  }
  const float k1 = r[0] / cnt1, k2 = r[1] / cnt1;
  __syncthreads();                            // R's reduction scratch read by every thread
  PROBE(a, 6);
  float acc[CPG * TAPS + CPG];
#pragma unroll
  for (int i = 0; i < CPG * TAPS + CPG; ++i) acc[i] = 0.f;
  for (int pp = u; pp < NP; pp += FT / 8) {
    const int pi = pp / a.Wp, pj = pp - pi * a.Wp;
    float x[4][4], v[4][CPG];
    window(im, a.W, pi, pj, q, x, v);
    int bi[CPG];
#pragma unroll
    for (int c = 0; c < CPG; ++c) {
      float best;
      bi[c] = block1_argmax(v, c, q, mu1, is1, a.p.slope, best);
    }
    float e[4][TAPS];
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
#pragma unroll
      for (int t = 0; t < TAPS; ++t) e[pos][t] = 0.f;
#pragma unroll
      for (int c = 0; c < CPG; ++c) {
        const float xh = (v[pos][c] - mu1) * is1;
        float dnv = 0.f;
        if (bi[c] == pos) {
          const float av = fmaf(xh, q.gm[c], q.bt[c]);
          const float dvc = p1[pp * P1S + g * CPG + c];
          dnv = (av > 0.f ? dvc : dvc * a.p.slope) * q.gm[c];
        }
        const float dh = is1 * (dnv - k1 - xh * k2);
        acc[CPG * TAPS + c] += dh;
#pragma unroll
        for (int t = 0; t < TAPS; ++t) {
          acc[c * TAPS + t] = fmaf(dh, x[(pos >> 1) + t / 3][(pos & 1) + t % 3], acc[c * TAPS + t]);
          if constexpr (WDX) e[pos][t] = fmaf(dh, q.w[c][t], e[pos][t]);
        }
      }
    }
    if constexpr (WDX) {
      // sum the 36 values over the window's 8 lanes as a reduce-scatter (halving rounds over lane
      // bits 2, 1, 0: 20 + 10 + 5 shuffles instead of 3 x 36); lane g ends with values g*5 .. g*5+4
      // of the 40 (36 padded)
      float e40[40];
#pragma unroll
      for (int i = 0; i < 40; ++i) e40[i] = i < 4 * TAPS ? e[i / TAPS][i % TAPS] : 0.f;
      const bool b2 = g & 4, b1 = g & 2, b0 = g & 1;
      float h20[20], h10[10], h5[5];
#pragma unroll
      for (int i = 0; i < 20; ++i) {
        const float send = b2 ? e40[i] : e40[i + 20], keep = b2 ? e40[i + 20] : e40[i];
        h20[i] = keep + __shfl_xor(send, 4, 64);
      }
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const float send = b1 ? h20[i] : h20[i + 10], keep = b1 ? h20[i + 10] : h20[i];
        h10[i] = keep + __shfl_xor(send, 2, 64);
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const float send = b0 ? h10[i] : h10[i + 5], keep = b0 ? h10[i + 5] : h10[i];
        h5[i] = keep + __shfl_xor(send, 1, 64);
      }
      // lane g holds the sums of entries 20*b2 + 10*b1 + 5*b0 + i
      const int i0 = (b2 ? 20 : 0) + (b1 ? 10 : 0) + (b0 ? 5 : 0);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int idx = i0 + i;
        if (idx < 4 * TAPS) {
          const int pos = idx / TAPS, t = idx - pos * TAPS;
          const int o = (2 * pi + (pos >> 1)) * a.Wo + 2 * pj + (pos & 1);
          R[t * MAXOUT + o] = h5[i];
        }
      }
    }
  }
  PROBE(a, 7);
  if constexpr (WDX) {
    __syncthreads();
    float* dx = a.dx + n * a.dxs[0];
    for (int p = threadIdx.x; p < a.H * a.W; p += FT) {
      const int i = p / a.W, j = p - i * a.W;
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const int oh = i - t / 3, ow = j - t % 3;
        if (oh >= 0 && oh < a.Ho && ow >= 0 && ow < a.Wo) s += R[t * MAXOUT + oh * a.Wo + ow];
      }
      dx[i * a.dxs[2] + j * a.dxs[3]] = s;
    }
  }
  if constexpr (WW) {
    quad_sum(acc, R);                         // (its leading barrier orders the e_rs reads)
    if (u == 0) {
#pragma unroll
      for (int c = 0; c < CPG; ++c) {
#pragma unroll
        for (int t = 0; t < TAPS; ++t) part[O_W1 + (g * CPG + c) * TAPS + t] = acc[c * TAPS + t];
        part[O_DB1 + g * CPG + c] = acc[CPG * TAPS + c];
      }
    }
  }
  PROBE(a, 8);
}

// Sum the per-image partials over the images: dw1 / dw2 WRITTEN, the rest ACCUMULATED (+=); any
// output may be NULL
struct F2Out {
  float *dw1, *db1, *dg1, *dbe1, *dw2, *db2, *dg2, *dbe2;
};
__global__ void __launch_bounds__(1024) dfront2_part_reduce(const float* __restrict__ part, int N, F2Out o,
                                                            const int32_t* rows) {
  __shared__ float red[16][64];
  N = live_rows(rows, N);   // the live images' partials
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6, col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < NPART2)
    for (int n = sl; n < N; n += 16) s += part[(int64_t)n * NPART2 + col];
  red[sl][lane] = s;
  __syncthreads();
  if (sl != 0 || col >= NPART2) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k][lane];
  float* dst;
  bool acc = true;
  int i;
  if (col < O_DB2) { dst = o.dw2; i = col; acc = false; }
  else if (col < O_DG2) { dst = o.db2; i = col - O_DB2; }
  else if (col < O_DBE2) { dst = o.dg2; i = col - O_DG2; }
  else if (col < O_W1) { dst = o.dbe2; i = col - O_DBE2; }
  else if (col < O_DB1) { dst = o.dw1; i = col - O_W1; acc = false; }
  else if (col < O_DG1) { dst = o.db1; i = col - O_DB1; }
  else if (col < O_DBE1) { dst = o.dg1; i = col - O_DG1; }
  else { dst = o.dbe1; i = col - O_DBE1; }
  if (dst) dst[i] = acc ? dst[i] + t : t;
}

int f2_args(F2Args& a, const float* img, const int64_t is[4], int N, int H, int W, const es_dfront2_params_t* p) {
  ES_CHECK_ARG(img && is && p && p->w1 && p->w2 && N > 0, "es_dfront2: null argument");
  ES_CHECK_ARG(es_dfront2_ok(H, W, p->ph, p->pw), "es_dfront2: image %dx%d with pool %dx%d unsupported", H, W,
               p->ph, p->pw);
  a = F2Args{};
  a.img = img;
  for (int i = 0; i < 4; ++i) a.is[i] = is[i];
  a.H = H; a.W = W; a.Ho = H - 2; a.Wo = W - 2; a.Hp = a.Ho / 2; a.Wp = a.Wo / 2;
  a.Ho2 = a.Hp - 2; a.Wo2 = a.Wp - 2;
  a.Hq = (a.Ho2 - p->ph) / p->ph + 1; a.Wq = (a.Wo2 - p->pw) / p->pw + 1;
  a.p = *p;
  a.sv = es_dfront2_save_floats(H, W, p->ph, p->pw);
  a.probe = g_probe;
  return ES_OK;
}

}  // namespace

// debug hook (ES_DF2_PROBE builds only record): device buffer of >= 16 int64 phase timestamps
extern "C" void es_dfront2_set_probe(long long* p) { g_probe = p; }

extern "C" int es_dfront2_ok(int H, int W, int ph, int pw) {
  if (ph < 1 || pw < 1 || H < 8 || W < 8) return 0;
  const int Ho = H - 2, Wo = W - 2;
  if ((Ho & 1) || (Wo & 1) || H * W > MAXPIX || Ho * Wo > MAXOUT) return 0;
  const int Hp = Ho / 2, Wp = Wo / 2;
  if (Hp * Wp > MAXP1) return 0;
  const int Ho2 = Hp - 2, Wo2 = Wp - 2;
  return Ho2 >= ph && Wo2 >= pw && Ho2 * Wo2 <= MAXH2;
}

extern "C" int64_t es_dfront2_part_floats(int N) { return (int64_t)N * NPART2; }

extern "C" int64_t es_dfront2_save_floats(int H, int W, int ph, int pw) {
  if (!es_dfront2_ok(H, W, ph, pw)) return 0;
  const int Hp = (H - 2) / 2, Wp = (W - 2) / 2;
  return (int64_t)2 * Hp * Wp * FK + (int64_t)(Hp - 2) * (Wp - 2) * K2;
}

extern "C" int es_dfront2_fwd(const float* img, const int64_t is[4], int N, int H, int W, const es_dfront2_params_t* p,
                              float* stats, float* feat, int64_t feat_stride, float* save, es_stream_t stream) {
  F2Args a;
  if (int rc = f2_args(a, img, is, N, H, W, p)) return rc;
  ES_CHECK_ARG(stats && feat && feat_stride >= (int64_t)K2 * a.Hq * a.Wq, "es_dfront2_fwd: outputs");
  a.stats = stats; a.feat = feat; a.fs = feat_stride; a.save = save;
  hipLaunchKernelGGL(dfront2_fwd_kernel, dim3(N), dim3(FT), 0, (hipStream_t)stream, a);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_dfront2_bwd(const float* img, const int64_t is[4], int N, int H, int W, const es_dfront2_params_t* p,
                              const float* stats, const float* save, const float* dfeat, int64_t dfeat_stride, float* dx,
                              const int64_t dxs[4], float* part, float* dw1, float* db1, float* dg1, float* dbe1,
                              float* dw2, float* db2, float* dg2, float* dbe2, es_stream_t stream) {
  F2Args a;
  if (int rc = f2_args(a, img, is, N, H, W, p)) return rc;
  ES_CHECK_ARG(stats && save && dfeat && dfeat_stride >= (int64_t)K2 * a.Hq * a.Wq, "es_dfront2_bwd: inputs");
  a.save = (float*)save;
  ES_CHECK_ARG(!dx || dxs, "es_dfront2_bwd: dx without strides");
  ES_CHECK_ARG(dx || part, "es_dfront2_bwd: nothing to compute (no dx, no part)");
  a.stats = (float*)stats; a.dfeat = dfeat; a.dfs = dfeat_stride; a.dx = dx; a.part = part;
  if (dx)
    for (int i = 0; i < 4; ++i) a.dxs[i] = dxs[i];
  hipStream_t st = (hipStream_t)stream;
  if (dx && part) hipLaunchKernelGGL((dfront2_bwd_kernel<true, true>), dim3(N), dim3(FT), 0, st, a);
  else if (dx) hipLaunchKernelGGL((dfront2_bwd_kernel<true, false>), dim3(N), dim3(FT), 0, st, a);
  else hipLaunchKernelGGL((dfront2_bwd_kernel<false, true>), dim3(N), dim3(FT), 0, st, a);
  ES_CHECK_LAUNCH();
  if (part) {
    const F2Out o{dw1, db1, dg1, dbe1, dw2, db2, dg2, dbe2};
    hipLaunchKernelGGL(dfront2_part_reduce, dim3((NPART2 + 63) / 64), dim3(1024), 0, st, part, N, o, p->rows);
    ES_CHECK_LAUNCH();
  }
  return ES_OK;
}
