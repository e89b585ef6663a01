// Fused fc tail of the spectral-norm discriminator (neutron/discriminator.py:26-48,
// proton/discriminator.py:136-158):
//
//   SNLinear F -> 128 -> LayerNorm(128) -> LeakyReLU -> SNLinear 128 -> 64 -> LayerNorm(64)
//   -> LeakyReLU (= latent) -> SNLinear 64 -> 1
//
// Unfused these were ~12 launches per forward and ~22 per backward (GEMMs of 1 / 64 / 128 output
// columns, LayerNorm statistics / apply / backward passes, weight packing, bias reductions), each
// a few microseconds of launch-bound work: ~100 us per forward and ~230 us per weight-gradient
// backward at B = 1024.  Here one workgroup owns 16 samples (one MFMA row tile) and runs the whole
// chain with its intermediates in LDS; the GEMMs are v_mfma_f32_16x16x4_f32 (exact fp32 products,
// weights scaled by 1/sigma on load as es_pack_conv_weight does).
//
//   forward  reads the fc1 input rows; writes the fc1 / fc2 outputs (pre-LayerNorm), the LayerNorm
//            statistics, the latent and the logit (the backward reads them).
//   backward reads those and the logit / latent gradients; writes the fc1 input gradient
//            (optional) and per-workgroup weight-gradient partials (optional), summed over the
//            workgroups by a second launch (deterministic, no atomics): the W/sigma gradients are
//            written, biases and LayerNorm affines accumulated.
#include "common.h"

namespace {

constexpr int MT = 512, MNW = MT / 64;     // threads, waves
constexpr int RB = 16;                     // samples per workgroup
constexpr int H1 = 128, H2 = 64;           // fc1 / fc2 widths
constexpr int P1 = H1 + 4, P2 = H2 + 4;    // LDS row pitches
constexpr int MAXF = 2320;                 // fc1 input width limit (neutron 1305, proton 2313), x16
constexpr int SMEM = RB * (MAXF + 4);      // floats: the staged fc1-input tile (aliased by the rest)

// the staged fc1-input tile row pitch: 16-byte rows, conflict-free 16-byte reads of 16 rows
__host__ __device__ inline int x_pitch(int F) { return ((F + 15) / 16) * 16 + 4; }

// per-workgroup partials (F = fc1 input width): dW1 [128][F] | dW2 [64][128] | dW3 [64] | db1 | db2 |
// db3 (padded to 4) | dg1 | dbe1 | dg2 | dbe2
struct PartLayout {
  int64_t w1, w2, w3, b1, b2, b3, g1, be1, g2, be2, n;
};
__host__ __device__ inline PartLayout part_layout(int F) {
  PartLayout L;
  L.w1 = 0;
  L.w2 = (int64_t)H1 * F;
  L.w3 = L.w2 + H2 * H1;
  L.b1 = L.w3 + H2;
  L.b2 = L.b1 + H1;
  L.b3 = L.b2 + H2;
  L.g1 = L.b3 + 4;
  L.be1 = L.g1 + H1;
  L.g2 = L.be1 + H1;
  L.be2 = L.g2 + H2;
  L.n = L.be2 + H2;
  return L;
}

struct MlpArgs {
  const float* X; int64_t xs;              // fc1 input rows (row stride xs)
  int B, F;
  es_dmlp_params_t p;
  float* h3; float* s3;                    // [B][128] fc1 output, [B][2] LN1 mean / invstd
  float* h4; float* s4;                    // [B][64], [B][2]
  float* lat;                              // [B][64]
  float* out;                              // [B]
  const float* dout; const float* dlat;    // logit / latent gradients (either may be NULL)
  float* dX; int64_t dxs;                  // fc1 input gradient (or NULL)
  float* part;                             // [workgroups][PartLayout.n] (or NULL)
};

// 16 x 16 tile D[r][c] = sum_{k < K} A(r, k) B(k, c) on v_mfma_f32_16x16x4_f32: lane (r16, kq) feeds
// A(r16, k + kq) and B(k + kq, r16); two accumulator chains, k beyond K read as 0 by the callers'
// accessors' bounds (the accessors take only k: the lane's row / column is bound in them).
template <typename FA, typename FB>
__device__ __forceinline__ f32x4 mm16(int K, FA A, FB Bv) {
  const int kq = (threadIdx.x & 63) >> 4;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 8 <= K; k += 8) {
    const float a0 = A(k + kq), b0 = Bv(k + kq), a1 = A(k + 4 + kq), b1 = Bv(k + 4 + kq);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, c1, 0, 0, 0);
  }
  for (; k < K; k += 4) {
    const int kk = k + kq;
    const float a0 = kk < K ? A(kk) : 0.f, b0 = kk < K ? Bv(kk) : 0.f;
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, c0, 0, 0, 0);
  }
  return c0 + c1;
}

// 16 x 16 tile with A from LDS (16 rows, pitch PA floats, 16-byte aligned, zero beyond K up to the
// next multiple of 16) and B = the lane's k-contiguous global row (scaled): per 16 k one 16-byte LDS
// read and one 16-byte global load feed four MFMAs (MFMA t takes k = 16 c + 4 kq + t in A and B
// alike), four blocks per iteration so their loads are in flight together
__device__ __forceinline__ f32x4 mm16_rowb(const float* A, int PA, const float* Brow, int K, float scale) {
  const int lane = threadIdx.x & 63, r16 = lane & 15, kq = lane >> 4;
  const float* ar = A + r16 * PA + kq * 4;
  const float* br = Brow + kq * 4;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
  const int nfull = K / 16;
  int c = 0;
  float4 bn[4];                               // the next iteration's B blocks, loaded one ahead
  if (nfull >= 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_memcpy(&bn[u], br + u * 16, 16);
  for (; c + 4 <= nfull; c += 4) {
    float4 av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      av[u] = *(const float4*)(ar + (c + u) * 16);
      bv[u] = bn[u];
    }
    if (c + 8 <= nfull)
#pragma unroll
      for (int u = 0; u < 4; ++u) __builtin_memcpy(&bn[u], br + (c + 4 + u) * 16, 16);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4& cc = (u & 1) ? c1 : c0;
      cc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].x, bv[u].x * scale, cc, 0, 0, 0);
      cc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].y, bv[u].y * scale, cc, 0, 0, 0);
      cc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].z, bv[u].z * scale, cc, 0, 0, 0);
      cc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u].w, bv[u].w * scale, cc, 0, 0, 0);
    }
  }
  for (; c * 16 < K; ++c) {                 // remaining blocks (the last one partial)
    const float4 a4 = *(const float4*)(ar + c * 16);
    const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = c * 16 + kq * 4 + t;
      const float b = k < K ? br[c * 16 + t] * scale : 0.f;
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], b, c0, 0, 0, 0);
    }
  }
  return c0 + c1;
}

// stage rows r0 .. r0 + nrow - 1 of X (rows past the batch and columns past F: zeros) as a
// [RB][x_pitch(F)] tile in LDS, coalesced along the rows
// (8 loads in flight per thread before their LDS stores: the tile is ~40 loads per thread, and one
// load-store pair per trip left every trip waiting on a global round trip)
__device__ __forceinline__ void stage_x(const float* X, int64_t xs, int r0, int nrow, int F, float* t) {
  constexpr int U = 8;
  const int PX = x_pitch(F), W = PX - 4, n = RB * W;
  for (int i0 = threadIdx.x; i0 < n; i0 += U * MT) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * MT, r = i / W, k = i - r * W;
      v[u] = (i < n && r < nrow && k < F) ? X[(int64_t)(r0 + r) * xs + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * MT, r = i / W, k = i - r * W;
      if (i < n) t[r * PX + k] = v[u];
    }
  }
}

// LayerNorm of the tile rows held in LDS (t[row][0..W)), thread (row = t >> 5, 32 lanes per row):
// returns the per-row mean / invstd (biased variance, two passes) to every lane of the row
template <int W, int P>
__device__ __forceinline__ void row_stats(const float (*t)[P], int row, int l, float eps, float& mu, float& is) {
  constexpr int PER = W / 32;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) s += t[row][l + 32 * j];
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) s += __shfl_xor(s, o, 64);
  mu = s / W;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const float d = t[row][l + 32 * j] - mu;
    q = fmaf(d, d, q);
  }
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o, 64);
  is = rsqrtf(q / W + eps);
}

__global__ void __launch_bounds__(MT) dmlp_fwd_kernel(MlpArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float (*t3)[P1] = (float (*)[P1])smem;        // (aliases the staged input after fc1)
  float (*t4)[P2] = (float (*)[P2])(smem + RB * P1);
  a.B = live_rows(a.p.rows, a.B);               // dynamic rows: the live samples
  const int r0 = blockIdx.x * RB, nrow = min(RB, a.B - r0);
  if (nrow <= 0) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r16 = lane & 15, kq = lane >> 4;
  const es_dmlp_params_t& p = a.p;
  stage_x(a.X, a.xs, r0, nrow, a.F, smem);
  __syncthreads();
  // fc1: wave w -> output columns 16 w ..
  {
    const float inv = p.sigma1 ? 1.f / p.sigma1[0] : 1.f;
    const int col = wid * 16 + r16;
    const f32x4 acc = mm16_rowb(smem, x_pitch(a.F), p.w1 + (int64_t)col * a.F, a.F, inv);
    const float bv = p.b1 ? p.b1[col] : 0.f;
    __syncthreads();                              // every wave is done with the staged input
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = kq * 4 + i;
      const float h = acc[i] + bv;
      t3[row][col] = h;
      if (row < nrow) a.h3[(int64_t)(r0 + row) * H1 + col] = h;
    }
  }
  __syncthreads();
  {
    const int row = threadIdx.x >> 5, l = threadIdx.x & 31;
    float mu, is;
    row_stats<H1, P1>(t3, row, l, p.eps1, mu, is);
#pragma unroll
    for (int j = 0; j < H1 / 32; ++j) {
      const int f = l + 32 * j;
      t3[row][f] = lrelu(fmaf((t3[row][f] - mu) * is, p.g1 ? p.g1[f] : 1.f, p.be1 ? p.be1[f] : 0.f), p.slope);
    }
    if (l == 0 && row < nrow) { a.s3[(int64_t)(r0 + row) * 2] = mu; a.s3[(int64_t)(r0 + row) * 2 + 1] = is; }
  }
  __syncthreads();
  if (wid < H2 / 16) {   // fc2: waves 0..3 -> columns 16 w ..
    const float inv = p.sigma2 ? 1.f / p.sigma2[0] : 1.f;
    const int col = wid * 16 + r16;
    const f32x4 acc = mm16_rowb(&t3[0][0], P1, p.w2 + col * H1, H1, inv);
    const float bv = p.b2 ? p.b2[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = kq * 4 + i;
      const float h = acc[i] + bv;
      t4[row][col] = h;
      if (row < nrow) a.h4[(int64_t)(r0 + row) * H2 + col] = h;
    }
  }
  __syncthreads();
  {
    const int row = threadIdx.x >> 5, l = threadIdx.x & 31;
    float mu, is;
    row_stats<H2, P2>(t4, row, l, p.eps2, mu, is);
    const float inv3 = p.sigma3 ? 1.f / p.sigma3[0] : 1.f;
    float o = 0.f;
#pragma unroll
    for (int j = 0; j < H2 / 32; ++j) {
      const int f = l + 32 * j;
      const float y = lrelu(fmaf((t4[row][f] - mu) * is, p.g2 ? p.g2[f] : 1.f, p.be2 ? p.be2[f] : 0.f), p.slope);
      if (row < nrow) a.lat[(int64_t)(r0 + row) * H2 + f] = y;
      o = fmaf(y, p.w3[f] * inv3, o);
    }
#pragma unroll
    for (int s = 1; s < 32; s <<= 1) o += __shfl_xor(o, s, 64);
    if (l == 0 && row < nrow) {
      a.s4[(int64_t)(r0 + row) * 2] = mu;
      a.s4[(int64_t)(r0 + row) * 2 + 1] = is;
      a.out[r0 + row] = o + (p.b3 ? p.b3[0] : 0.f);
    }
  }
}

template <bool WDX, bool WW>
__global__ void __launch_bounds__(MT) dmlp_bwd_kernel(MlpArgs a) {
  // one LDS object: [0, SMEM) holds y3 / g4 / cs, later the staged fc1-input tile (dW1's B operand);
  // g3 lives past it
  __shared__ __attribute__((aligned(16))) float smem[SMEM + RB * P1];
  float (*y3)[P1] = (float (*)[P1])smem;                          // LN1 output (fc2 input)
  float (*g4)[P2] = (float (*)[P2])(smem + RB * P1);              // fc2 output gradient (dh4)
  float (*cs)[RB][P1] = (float (*)[RB][P1])(smem + RB * P1 + RB * P2);   // dgamma / dbeta terms
  float (*g3)[P1] = (float (*)[P1])(smem + SMEM);                 // dy3, then dh3
  a.B = live_rows(a.p.rows, a.B);               // dynamic rows: the live samples
  const int r0 = blockIdx.x * RB, nrow = min(RB, a.B - r0);
  if (nrow <= 0) return;                          // (dmlp_part_reduce skips its partial)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r16 = lane & 15, kq = lane >> 4;
  const es_dmlp_params_t& p = a.p;
  const PartLayout L = part_layout(a.F);
  float* part = WW ? a.part + (int64_t)blockIdx.x * L.n : nullptr;
  const int row = threadIdx.x >> 5, l = threadIdx.x & 31;
  const bool live = row < nrow;
  const int gr = r0 + (live ? row : 0);
  // y3 = LReLU(LN1(h3)) from the saved fc1 output and statistics
  {
    const float mu = a.s3[(int64_t)gr * 2], is = a.s3[(int64_t)gr * 2 + 1];
#pragma unroll
    for (int j = 0; j < H1 / 32; ++j) {
      const int f = l + 32 * j;
      const float h = a.h3[(int64_t)gr * H1 + f];
      y3[row][f] = live ? lrelu(fmaf((h - mu) * is, p.g1 ? p.g1[f] : 1.f, p.be1 ? p.be1[f] : 0.f), p.slope) : 0.f;
    }
  }
  // latent gradient -> LN2 backward -> dh4
  {
    const float inv3 = p.sigma3 ? 1.f / p.sigma3[0] : 1.f;
    const float mu = a.s4[(int64_t)gr * 2], is = a.s4[(int64_t)gr * 2 + 1];
    const float dov = (a.dout && live) ? a.dout[gr] : 0.f;
    float xh[H2 / 32], dn[H2 / 32], sdn = 0.f, sdx = 0.f;
#pragma unroll
    for (int j = 0; j < H2 / 32; ++j) {
      const int f = l + 32 * j;
      float dl = dov * p.w3[f] * inv3;
      if (a.dlat && live) dl += a.dlat[(int64_t)gr * H2 + f];
      xh[j] = (a.h4[(int64_t)gr * H2 + f] - mu) * is;
      const float gm = p.g2 ? p.g2[f] : 1.f;
      const float av = fmaf(xh[j], gm, p.be2 ? p.be2[f] : 0.f);
      const float da = live ? (av > 0.f ? dl : dl * p.slope) : 0.f;
      dn[j] = da * gm;
      sdn += dn[j];
      sdx = fmaf(dn[j], xh[j], sdx);
      if (WW) {
        cs[0][row][f] = da * xh[j];
        cs[1][row][f] = da;
        // dW3 / db3 terms: dout * latent (the latent of this row and feature)
        g4[row][f] = dov * a.lat[(int64_t)gr * H2 + f];
      }
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      sdn += __shfl_xor(sdn, o, 64);
      sdx += __shfl_xor(sdx, o, 64);
    }
    if (WW) {
      __syncthreads();
      if (threadIdx.x < H2) {                 // column sums over the rows: dgamma2, dbeta2, dW3
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
        for (int r = 0; r < RB; ++r) {
          s0 += cs[0][r][threadIdx.x];
          s1 += cs[1][r][threadIdx.x];
          s2 += g4[r][threadIdx.x];
        }
        part[L.g2 + threadIdx.x] = s0;
        part[L.be2 + threadIdx.x] = s1;
        part[L.w3 + threadIdx.x] = s2;
      }
      if (threadIdx.x == 64) {
        float s = 0.f;
        for (int r = 0; r < nrow; ++r) s += a.dout ? a.dout[r0 + r] : 0.f;
        part[L.b3] = s;
        part[L.b3 + 1] = part[L.b3 + 2] = part[L.b3 + 3] = 0.f;
      }
      __syncthreads();                         // g4 / cs reused below
    }
    const float k1 = sdn / H2, k2 = sdx / H2;
#pragma unroll
    for (int j = 0; j < H2 / 32; ++j) g4[row][l + 32 * j] = live ? is * (dn[j] - k1 - xh[j] * k2) : 0.f;
  }
  __syncthreads();
  if (WW) {
    // dW2[i][j] = sum_r dh4[r][i] y3[r][j] (8192 outputs, 16 per thread), db2[i] = sum_r dh4[r][i]
    for (int o = threadIdx.x; o < H2 * H1; o += MT) {
      const int i = o / H1, j = o - i * H1;
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < RB; ++r) s = fmaf(g4[r][i], y3[r][j], s);
      part[L.w2 + o] = s;
    }
    if (threadIdx.x < H2) {
      float s = 0.f;
      for (int r = 0; r < RB; ++r) s += g4[r][threadIdx.x];
      part[L.b2 + threadIdx.x] = s;
    }
  }
  // dy3 = dh4 W2 / sigma2: wave w -> columns 16 w .. (K = 64)
  {
    const float inv = p.sigma2 ? 1.f / p.sigma2[0] : 1.f;
    const int col = wid * 16 + r16;
    const f32x4 acc = mm16(H2, [&](int k) { return g4[r16][k]; }, [&](int k) { return p.w2[k * H1 + col] * inv; });
#pragma unroll
    for (int i = 0; i < 4; ++i) g3[kq * 4 + i][col] = acc[i];
  }
  __syncthreads();
  // LN1 backward -> dh3 (in g3)
  {
    const float mu = a.s3[(int64_t)gr * 2], is = a.s3[(int64_t)gr * 2 + 1];
    float xh[H1 / 32], dn[H1 / 32], sdn = 0.f, sdx = 0.f;
#pragma unroll
    for (int j = 0; j < H1 / 32; ++j) {
      const int f = l + 32 * j;
      xh[j] = (a.h3[(int64_t)gr * H1 + f] - mu) * is;
      const float gm = p.g1 ? p.g1[f] : 1.f;
      const float av = fmaf(xh[j], gm, p.be1 ? p.be1[f] : 0.f);
      const float dy = g3[row][f];
      const float da = live ? (av > 0.f ? dy : dy * p.slope) : 0.f;
      dn[j] = da * gm;
      sdn += dn[j];
      sdx = fmaf(dn[j], xh[j], sdx);
      if (WW) { cs[0][row][f] = da * xh[j]; cs[1][row][f] = da; }
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      sdn += __shfl_xor(sdn, o, 64);
      sdx += __shfl_xor(sdx, o, 64);
    }
    const float k1 = sdn / H1, k2 = sdx / H1;
    __syncthreads();                           // every g3 (dy3) read before dh3 overwrites it
#pragma unroll
    for (int j = 0; j < H1 / 32; ++j) g3[row][l + 32 * j] = live ? is * (dn[j] - k1 - xh[j] * k2) : 0.f;
  }
  __syncthreads();
  if (WW) {
    if (threadIdx.x < H1) {                    // dgamma1, dbeta1, db1
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
      for (int r = 0; r < RB; ++r) {
        s0 += cs[0][r][threadIdx.x];
        s1 += cs[1][r][threadIdx.x];
        s2 += g3[r][threadIdx.x];
      }
      part[L.g1 + threadIdx.x] = s0;
      part[L.be1 + threadIdx.x] = s1;
      part[L.b1 + threadIdx.x] = s2;
    }
    // dW1[i][k] = sum_r dh3[r][i] X[r][k]: wave w -> rows i in 16 w .., column tiles of k; K = 16
    // samples.  A(i, r) = dh3[r][i], B(r, k) = X[r][k] from the staged tile (rows past the batch: 0)
    __syncthreads();                             // y3 / g4 / cs are dead: stage X over them
    stage_x(a.X, a.xs, r0, nrow, a.F, smem);
    __syncthreads();
    const int i0 = wid * 16, PX = x_pitch(a.F);
    float av[4];
#pragma unroll
    for (int rs = 0; rs < 4; ++rs) av[rs] = g3[rs * 4 + kq][i0 + r16];
    for (int k0 = 0; k0 < a.F; k0 += 32) {         // two column tiles per iteration
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int rs = 0; rs < 4; ++rs) {
        const float* xr = smem + (rs * 4 + kq) * PX + k0 + r16;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[rs], xr[0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[rs], k0 + 16 < PX - 4 ? xr[16] : 0.f, acc1, 0, 0, 0);
      }
      const int k = k0 + r16;
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        float* pw = part + L.w1 + (int64_t)(i0 + kq * 4 + ii) * a.F;
        if (k < a.F) pw[k] = acc0[ii];
        if (k + 16 < a.F) pw[k + 16] = acc1[ii];
      }
    }
  }
  if (WDX) {
    // dX = dh3 W1 / sigma1: column tiles of k over the waves, K = 128
    // (a lane's 32 W1 values of the next column tile (rows i = 4 j + kq) are loaded before the current
    // tile's MFMAs: one global round trip per tile, overlapped, instead of one per 8 k; the two
    // accumulator chains and their order are mm16's)
    const float inv = p.sigma1 ? 1.f / p.sigma1[0] : 1.f;
    constexpr int NJ = H1 / 4;
    float bw[NJ];
    auto load_w = [&](int k0) {
      const int k = k0 + r16;
      const int kc = k < a.F ? k : 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) bw[j] = p.w1[(int64_t)(4 * j + kq) * a.F + kc];
    };
    if (wid * 16 < a.F) load_w(wid * 16);
    for (int k0 = wid * 16; k0 < a.F; k0 += MNW * 16) {
      const int k = k0 + r16;
      const bool kin = k < a.F;
      float bc[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bc[j] = bw[j];
      if (k0 + MNW * 16 < a.F) load_w(k0 + MNW * 16);
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NJ; j += 2) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(g3[r16][4 * j + kq], bc[j] * inv, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(g3[r16][4 * j + 4 + kq], bc[j + 1] * inv, c1, 0, 0, 0);
      }
      const f32x4 acc = c0 + c1;
      if (kin)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = kq * 4 + i;
          if (rr < nrow) a.dX[(int64_t)(r0 + rr) * a.dxs + k] = acc[i];
        }
    }
  }
}

// sum the per-workgroup partials: W/sigma gradients written, biases / LN affines accumulated
struct MlpOut {
  float *dw1, *db1, *dg1, *dbe1, *dw2, *db2, *dg2, *dbe2, *dw3, *db3;
};
__global__ void __launch_bounds__(1024) dmlp_part_reduce(const float* __restrict__ part, int nwg, int F,
                                                         MlpOut o, const int32_t* rows, int B) {
  __shared__ float red[16][64];
  if (rows) nwg = min(nwg, (live_rows(rows, B) + RB - 1) / RB);   // the live samples' workgroups
  const PartLayout L = part_layout(F);
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < L.n)
    for (int n = sl; n < nwg; n += 16) s += part[(int64_t)n * L.n + col];
  red[sl][lane] = s;
  __syncthreads();
  if (sl != 0 || col >= L.n) return;
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k][lane];
  float* dst;
  int64_t i;
  bool acc = true;
  if (col < L.w2) { dst = o.dw1; i = col; acc = false; }
  else if (col < L.w3) { dst = o.dw2; i = col - L.w2; acc = false; }
  else if (col < L.b1) { dst = o.dw3; i = col - L.w3; acc = false; }
  else if (col < L.b2) { dst = o.db1; i = col - L.b1; }
  else if (col < L.b3) { dst = o.db2; i = col - L.b2; }
  else if (col < L.g1) { dst = col == L.b3 ? o.db3 : nullptr; i = 0; }
  else if (col < L.be1) { dst = o.dg1; i = col - L.g1; }
  else if (col < L.g2) { dst = o.dbe1; i = col - L.be1; }
  else if (col < L.be2) { dst = o.dg2; i = col - L.g2; }
  else { dst = o.dbe2; i = col - L.be2; }
  if (dst) dst[i] = acc ? dst[i] + t : t;
}

int mlp_args(MlpArgs& a, const float* X, int64_t xs, int B, int F, const es_dmlp_params_t* p) {
  ES_CHECK_ARG(X && p && p->w1 && p->w2 && p->w3 && B > 0 && F > 0 && xs >= F, "es_dmlp: bad arguments");
  ES_CHECK_ARG(F <= MAXF, "es_dmlp: fc1 input width %d > %d", F, MAXF);
  a = MlpArgs{};
  a.X = X; a.xs = xs; a.B = B; a.F = F; a.p = *p;
  return ES_OK;
}

}  // namespace

extern "C" int64_t es_dmlp_part_floats(int B, int F) {
  return (int64_t)((B + RB - 1) / RB) * part_layout(F).n;
}

extern "C" int es_dmlp_fwd(const float* X, int64_t xs, int B, int F, const es_dmlp_params_t* p, float* h3, float* s3,
                           float* h4, float* s4, float* lat, float* out, es_stream_t stream) {
  MlpArgs a;
  if (int rc = mlp_args(a, X, xs, B, F, p)) return rc;
  ES_CHECK_ARG(h3 && s3 && h4 && s4 && lat && out, "es_dmlp_fwd: null output");
  a.h3 = h3; a.s3 = s3; a.h4 = h4; a.s4 = s4; a.lat = lat; a.out = out;
  hipLaunchKernelGGL(dmlp_fwd_kernel, dim3((B + RB - 1) / RB), dim3(MT), 0, (hipStream_t)stream, a);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_dmlp_bwd(const float* X, int64_t xs, int B, int F, const es_dmlp_params_t* p, const float* h3,
                           const float* s3, const float* h4, const float* s4, const float* lat, const float* dout,
                           const float* dlat, float* dX, int64_t dxs, float* part, float* dw1, float* db1,
                           float* dg1, float* dbe1, float* dw2, float* db2, float* dg2, float* dbe2, float* dw3,
                           float* db3, es_stream_t stream) {
  MlpArgs a;
  if (int rc = mlp_args(a, X, xs, B, F, p)) return rc;
  ES_CHECK_ARG(h3 && s3 && h4 && s4 && lat, "es_dmlp_bwd: saved forward values");
  ES_CHECK_ARG(dX || part, "es_dmlp_bwd: nothing to compute (no dX, no part)");
  ES_CHECK_ARG(!dX || dxs >= F, "es_dmlp_bwd: dX row stride");
  a.h3 = (float*)h3; a.s3 = (float*)s3; a.h4 = (float*)h4; a.s4 = (float*)s4; a.lat = (float*)lat;
  a.dout = dout; a.dlat = dlat; a.dX = dX; a.dxs = dxs; a.part = part;
  hipStream_t st = (hipStream_t)stream;
  const int nwg = (B + RB - 1) / RB;
  if (dX && part) hipLaunchKernelGGL((dmlp_bwd_kernel<true, true>), dim3(nwg), dim3(MT), 0, st, a);
  else if (dX) hipLaunchKernelGGL((dmlp_bwd_kernel<true, false>), dim3(nwg), dim3(MT), 0, st, a);
  else hipLaunchKernelGGL((dmlp_bwd_kernel<false, true>), dim3(nwg), dim3(MT), 0, st, a);
  ES_CHECK_LAUNCH();
  if (part) {
    const MlpOut o{dw1, db1, dg1, dbe1, dw2, db2, dg2, dbe2, dw3, db3};
    const int64_t n = part_layout(F).n;
    hipLaunchKernelGGL(dmlp_part_reduce, dim3((unsigned)((n + 63) / 64)), dim3(1024), 0, st, part, nwg, F, o, p->rows, B);
    ES_CHECK_LAUNCH();
  }
  return ES_OK;
}
