// Loss kernels of the expertsim train step and their gradients (single-pass, no host syncs).
//   hinge D          moe.py:518-523
//   gen hinge        moe.py:544
//   SDI diversity    moe.py:573-588 (closed form of the [B,1]/[B] broadcast: see es_gen_losses)
//   intensity L1     moe.py:590-642
//   log-cosh aux     proton/aux_reg.py:42-45 == neutron/aux_reg.py:70-74, x strength (moe.py:559)
//   gumbel softmax   routers/router.py:23 (torch F.gumbel_softmax, hard=False)
//   ALB router loss  train/utils.py:623-642, weighted as moe.py:407,418-434
#include "common.h"

namespace {
struct View {
  int n, c, h, w;
  int64_t s[4];
  const int32_t* rows;   // live images (es_view_t.rows)
  __device__ __forceinline__ int64_t off(int in, int ic, int ih, int iw) const {
    return in * s[0] + ic * s[1] + ih * s[2] + iw * s[3];
  }
};
View mkview(const es_view_t* v) {
  View r;
  r.n = v->n; r.c = v->c; r.h = v->h; r.w = v->w;
  for (int i = 0; i < 4; ++i) r.s[i] = v->s[i];
  r.rows = v->rows;
  return r;
}
__device__ __forceinline__ float ldf(const void* p, int bf, int64_t i) {
  return bf ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ float signf_(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ void __launch_bounds__(256) hinge_d_kernel(const float* ro, const float* fo, int n, const int32_t* rows,
                                                      const float* wp, float* out, float* dro, float* dfo) {
  __shared__ float sh[8];
  n = live_rows(rows, n);
  if (n == 0) {   // an expert without samples this step: loss 0 (moe.py:126-129)
    if (threadIdx.x == 0) out[0] = 0.f;
    return;
  }
  const float w = wp[0];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float tr = 1.f - ro[i], tf = 1.f + fo[i];
    a += fmaxf(tr, 0.f);
    b += fmaxf(tf, 0.f);
    if (dro) dro[i] = tr > 0.f ? -w / (float)n : 0.f;
    if (dfo) dfo[i] = tf > 0.f ? w / (float)n : 0.f;
  }
  a = block_sum(a, sh);
  b = block_sum(b, sh);
  if (threadIdx.x == 0) out[0] = (a / (float)n + b / (float)n) * w;
}

// one block per sample: s[b] = sum_{c,h,w} exp(x) - 1
__global__ void __launch_bounds__(256) expsum_kernel(View x, const void* xp, int bf, float* s) {
  __shared__ float sh[8];
  const int n = blockIdx.x;
  if (n >= live_rows(x.rows, x.n)) return;
  const int per = x.c * x.h * x.w;
  float a = 0.f;
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    const int w = i % x.w, t = i / x.w, h = t % x.h, c = t / x.h;
    a += expf(ldf(xp, bf, x.off(n, c, h, w))) - 1.f;
  }
  a = block_sum(a, sh);
  if (threadIdx.x == 0) s[n] = a;
}

__global__ void expsum_bwd_kernel(View x, const void* xp, int bf, const float* coef, View dx, float* dxp,
                                  float beta) {
  const int64_t total = (int64_t)live_rows(x.rows ? x.rows : dx.rows, x.n) * x.c * x.h * x.w;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int w = e % x.w; int64_t t = e / x.w; const int h = t % x.h; t /= x.h; const int c = t % x.c;
    const int n = t / x.c;
    float g = coef[n] * expf(ldf(xp, bf, x.off(n, c, h, w)));
    const int64_t o = dx.off(n, c, h, w);
    if (beta != 0.f) g += beta * dxp[o];
    dxp[o] = g;
  }
}

// Generator losses in three passes (no host sync):
//   A  one wave per sample: adl = mean|l1-l2| over the latent, adn = mean|n1-n2| over the noise,
//      div_b = adl / (adn + 1e-5)   -> coef[b] = div_b, dfo[b] = adn (scratch, rewritten by B)
//   B  one block: every batch sum, the metrics, and per-sample gradients (dfo, coef, dcoord) plus
//      the SDI gradient factor g_b -> dl2[b * latent] (scratch, rewritten by C)
//   C  one wave per sample: dl1 = g_b * sign(l1 - l2), dl2 = -dl1
__global__ void __launch_bounds__(256) gen_losses_a(es_gen_loss_t p, const float* l1, const float* l2,
                                                    const float* n1, const float* n2, float* div_out,
                                                    float* adn_out) {
  const int lane = threadIdx.x & 63, b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= live_rows(p.rows, p.n)) return;
  float adl = 0.f, adn = 0.f;
  for (int k = lane; k < p.latent; k += 64) adl += fabsf(l1[b * p.latent + k] - l2[b * p.latent + k]);
  for (int k = lane; k < p.noise; k += 64) adn += fabsf(n1[b * p.noise + k] - n2[b * p.noise + k]);
  adl = wave_sum(adl) / (float)p.latent;
  adn = wave_sum(adn) / (float)p.noise;
  if (lane == 0) { div_out[b] = adl / (adn + 1e-5f); adn_out[b] = adn; }
}

__global__ void __launch_bounds__(256) gen_losses_b(es_gen_loss_t p, const float* fo, const float* sd,
                                                    const float* s, const float* inten, const float* coord,
                                                    const float* pos, const float* wp, float* out, float* dfo,
                                                    float* coef, float* dcoord, float* dl2) {
  __shared__ float sh[8];
  __shared__ float sdiv[4096], sadn[4096];  // n <= 4096 checked on host
  const int n = live_rows(p.rows, p.n);
  if (n == 0) {   // an expert without samples this step: every metric 0 (moe.py:126-130)
    if (threadIdx.x < 8) out[threadIdx.x] = 0.f;
    return;
  }
  const float w = wp[0];
  const float fn = (float)n;
  for (int b = threadIdx.x; b < n; b += blockDim.x) { sdiv[b] = coef[b]; sadn[b] = dfo[b]; }
  __syncthreads();
  float sfo = 0.f, sstd = 0.f, ss = 0.f, sl1 = 0.f, saux = 0.f, sr = 0.f;
  for (int b = threadIdx.x; b < n; b += blockDim.x) {
    sfo += fo[b];
    sstd += sd[b];
    ss += s[b];
    sl1 += fabsf(s[b] - inten[b]);
    sr += 1.f / (sdiv[b] + 1e-5f);
    for (int k = 0; k < 2; ++k) {
      const float d = coord[b * 2 + k] - pos[b * 2 + k];
      const float z = -2.f * d;
      const float sp = z > 20.f ? z : log1pf(expf(z));
      saux += d + sp - 0.69314718055994531f;
    }
  }
  sfo = block_sum(sfo, sh);
  sstd = block_sum(sstd, sh);
  ss = block_sum(ss, sh);
  sl1 = block_sum(sl1, sh);
  saux = block_sum(saux, sh);
  sr = block_sum(sr, sh);
  const float ms = p.std_mean ? p.std_mean[0] : sstd / fn;   // data parallel: the expert's global mean
  const float smean = ss / fn;
  float sq = 0.f;
  for (int b = threadIdx.x; b < n; b += blockDim.x) { const float d = s[b] - smean; sq += d * d; }
  sq = block_sum(sq, sh);
  const float gen = -sfo / fn;
  const float div = ms * ((p.std_mean ? ms * fn : sstd) * sr / (fn * fn)) * p.di_strength;
  const float inl = sl1 / fn * p.in_strength;
  const float aux = saux / (2.f * fn) * p.aux_strength;
  // gradients (all scaled by w)
  const float kdiv = -p.di_strength * ms * ms / fn * w;   // d/d div_j = kdiv / (div_j+eps)^2
  for (int b = threadIdx.x; b < n; b += blockDim.x) {
    dfo[b] = -w / fn;
    coef[b] = w * p.in_strength / fn * signf_(s[b] - inten[b]);
    const float e = sdiv[b] + 1e-5f;
    dl2[b * p.latent] = kdiv / (e * e) / (sadn[b] + 1e-5f) / (float)p.latent;
    for (int k = 0; k < 2; ++k) {
      const float d = coord[b * 2 + k] - pos[b * 2 + k];
      const float z = -2.f * d;
      const float spg = z > 20.f ? 1.f : 1.f / (1.f + expf(-z));   // softplus'(z) = sigmoid(z)
      dcoord[b * 2 + k] = w * p.aux_strength / (2.f * fn) * (1.f - 2.f * spg);
    }
  }
  if (threadIdx.x == 0) {
    out[0] = (gen + div + inl + aux) * w;
    out[1] = gen;
    out[2] = div;
    out[3] = inl;
    out[4] = aux;
    out[5] = n > 1 ? sqrtf(sq / (fn - 1.f)) : NAN;
    out[6] = smean;
    out[7] = w;
  }
}

__global__ void __launch_bounds__(256) gen_losses_c(es_gen_loss_t p, const float* l1, const float* l2, float* dl1,
                                                    float* dl2) {
  const int lane = threadIdx.x & 63, b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= live_rows(p.rows, p.n)) return;
  const float g = dl2[b * p.latent];   // every lane's load precedes the wave's stores (data dependency)
  for (int k = lane; k < p.latent; k += 64) {
    const float sg = signf_(l1[b * p.latent + k] - l2[b * p.latent + k]);
    dl1[b * p.latent + k] = g * sg;
    dl2[b * p.latent + k] = -g * sg;
  }
}

__global__ void router_gumbel_kernel(const float* logits, const float* expo, int B, int E, float tau, float* gates,
                                     int32_t* idx, int32_t* counts) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    const float z = (logits[b * E + e] + (-logf(expo[b * E + e]))) / tau;
    mx = fmaxf(mx, z);
  }
  float sum = 0.f;
  for (int e = 0; e < E; ++e) {
    const float z = (logits[b * E + e] + (-logf(expo[b * E + e]))) / tau;
    sum += expf(z - mx);
  }
  int best = 0;
  float bv = -INFINITY;
  for (int e = 0; e < E; ++e) {
    const float z = (logits[b * E + e] + (-logf(expo[b * E + e]))) / tau;
    const float gte = expf(z - mx) / sum;
    gates[b * E + e] = gte;
    if (gte > bv) { bv = gte; best = e; }
  }
  idx[b] = best;
  if (counts) atomicAdd(&counts[best], 1);
}

__global__ void __launch_bounds__(256) router_alb_kernel(const float* gates, int B, int E, float tau, float coef,
                                                         float* out, float* dlogits) {
  __shared__ float sh[8];
  __shared__ float gS[64];
  float L = 0.f;
  for (int e = 0; e < E; ++e) {
    float s = 0.f;
    for (int b = threadIdx.x; b < B; b += blockDim.x) s += gates[b * E + e];
    s = block_sum(s, sh);
    const float inv = 1.f / (s + 1e-6f);
    const float ex = expf(inv);
    L += ex;
    if (threadIdx.x == 0) gS[e] = coef / (float)E * ex * (-inv * inv);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[0] = coef * (L / (float)E);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    float dot = 0.f;
    for (int e = 0; e < E; ++e) dot += gates[b * E + e] * gS[e];
    for (int e = 0; e < E; ++e) dlogits[b * E + e] = gates[b * E + e] * (gS[e] - dot) / tau;
  }
}
// Expert-distribution (ED) pair sums, train/utils.py:372-395 with gating = the straight-through
// one-hot gates (moe.py:103,264): T[a,e] = sum_{b: idx_b = e} |f_a - f_b| (cdist p=2 of the [B,1]
// per-sample photon sums).  One thread per (a, e); f / idx staged through LDS in 1024-row tiles.
// a: the B local rows; b: the Ball rows of the (all-gathered) global batch.
__global__ void __launch_bounds__(256) router_ed_pairs_kernel(const float* feat, int B, const float* feat_all,
                                                              const int32_t* idx_all, int Ball, int E, float* T) {
  __shared__ float fs[1024];
  __shared__ int32_t is[1024];
  const int a = blockIdx.x * blockDim.x + threadIdx.x, e = blockIdx.y;
  const float fa = a < B ? feat[a] : 0.f;
  float acc = 0.f;
  for (int b0 = 0; b0 < Ball; b0 += 1024) {
    const int nb = min(1024, Ball - b0);
    __syncthreads();
    for (int j = threadIdx.x; j < nb; j += blockDim.x) {
      fs[j] = feat_all[b0 + j];
      is[j] = idx_all[b0 + j];
    }
    __syncthreads();
    for (int j = 0; j < nb; ++j) acc += is[j] == e ? fabsf(fa - fs[j]) : 0.f;
  }
  if (a < B) T[a * E + e] = acc;
}

// S_e = sum_b gates[b, e] (a rank's share of the router's global gate sums)
__global__ void __launch_bounds__(256) router_colsum_kernel(const float* gates, int B, int E, float* out) {
  __shared__ float sh[8];
  for (int e = 0; e < E; ++e) {
    float s = 0.f;
    for (int b = threadIdx.x; b < B; b += blockDim.x) s += gates[b * E + e];
    s = block_sum(s, sh);
    if (threadIdx.x == 0) out[e] = s;
  }
}

// Router loss terms with gradient into the router (moe.py:258-268,407-434; train/utils.py:372-419,
// 623-642) and d loss / d logits through the Gumbel softmax (gates = softmax(z / tau)):
//   ALB  = alb_coef * mean_e exp(1 / (S_e + 1e-6)),      S_e = sum_b gates[b,e]
//   ENT  = util * sum_e avg_e log(avg_e + 1e-9),          avg_e = S_e / B  (= -entropy * util)
//   ED   = 0.1 * ed / B * sum_a T[a, idx_a]               (T from router_ed_pairs_kernel, or none)
// d/dgates[b,e] = alb_coef/E exp(inv_e)(-inv_e^2) + util/B (log(avg_e+1e-9) + avg_e/(avg_e+1e-9))
//               + 0.2 * ed / B * T[b,e];   dlogits = gates * (dG - <gates, dG>) / tau.
// out[0] = ALB, out[1] = ENT, out[2] = ED.  T aliases dlogits (each row is read before written).
__global__ void __launch_bounds__(1024) router_loss_kernel(const float* gates, const int32_t* idx, int B, int E,
                                                           float tau, float alb_coef, float util, float ed,
                                                           const float* colsum, float Btot, float* out,
                                                           float* dlogits) {
  __shared__ float sh[16];
  __shared__ float gS[64];
  float L = 0.f, ent = 0.f;
  for (int e = 0; e < E; ++e) {
    float s = 0.f;
    if (colsum) {
      s = colsum[e];                       // data parallel: the all-reduced global sums
    } else {
      for (int b = threadIdx.x; b < B; b += blockDim.x) s += gates[b * E + e];
      s = block_sum(s, sh);
    }
    const float inv = 1.f / (s + 1e-6f);
    const float ex = expf(inv);
    L += ex;
    const float avg = s / Btot;
    const float lg = logf(avg + 1e-9f);
    ent += avg * lg;
    if (threadIdx.x == 0)
      gS[e] = alb_coef / (float)E * ex * (-inv * inv) + util / Btot * (lg + avg / (avg + 1e-9f));
  }
  float edsum = 0.f;
  if (ed != 0.f) {
    for (int b = threadIdx.x; b < B; b += blockDim.x) edsum += dlogits[b * E + idx[b]];
    edsum = block_sum(edsum, sh);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = alb_coef * (L / (float)E);
    out[1] = util * ent;
    out[2] = 0.1f * (edsum / Btot) * ed;
  }
  const float ked = 0.2f * ed / Btot;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    float dg[64];
    float dot = 0.f;
    for (int e = 0; e < E; ++e) {
      dg[e] = gS[e] + (ed != 0.f ? ked * dlogits[b * E + e] : 0.f);
      dot += gates[b * E + e] * dg[e];
    }
    for (int e = 0; e < E; ++e) dlogits[b * E + e] = gates[b * E + e] * (dg[e] - dot) / tau;
  }
}

// Data-parallel metric merge: rows [world][E][10] = the ranks' per-expert metric rows (total, gen,
// div, int, aux, std_int, mean_int, w, disc) + the local sample count (0 when the rank did not run
// the expert).  Totals / w / disc (local-count-weighted losses) average over ranks; per-sample means
// (gen, div, int, aux, mean_int) are count-weighted; std_int merges (n, mean, M2) (Chan).
__global__ void dp_metrics_merge_kernel(const float* rows, int world, int E, float* out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  double N = 0.0, tot = 0.0, wsum = 0.0, disc = 0.0, c[4] = {0.0, 0.0, 0.0, 0.0}, mean = 0.0, M2 = 0.0;
  for (int r = 0; r < world; ++r) {
    const float* q = rows + ((int64_t)r * E + e) * 10;
    tot += q[0]; wsum += q[7]; disc += q[8];
    const double n = q[9];
    if (n <= 0.0) continue;
    for (int k = 0; k < 4; ++k) c[k] += n * q[1 + k];
    const double nt = N + n, dl = (double)q[6] - mean;
    M2 += (n - 1.0) * (double)q[5] * (double)q[5] + dl * dl * N * n / nt;
    mean += dl * n / nt;
    N = nt;
  }
  float* o = out + (int64_t)e * 9;
  o[0] = (float)(tot / world); o[7] = (float)(wsum / world); o[8] = (float)(disc / world);
  for (int k = 0; k < 4; ++k) o[1 + k] = N > 0.0 ? (float)(c[k] / N) : 0.f;
  o[6] = N > 0.0 ? (float)mean : 0.f;
  o[5] = N > 1.0 ? (float)sqrt(M2 / (N - 1.0)) : 0.f;
}

// Expert dispatch as a stable counting sort (moe.py:121-123: per expert, the rows with idx == e in
// batch order): perm = [rows of expert 0 | rows of expert 1 | ...], offs[e] = first position of
// expert e, offs[E] = B.  One block; per expert a block-wide exclusive scan over 1024-row tiles.
__global__ void __launch_bounds__(1024) router_dispatch_kernel(const int32_t* idx, int B, int E, int32_t* perm,
                                                               int32_t* offs) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int e = 0; e < E; ++e) {
    if (threadIdx.x == 0) offs[e] = base;
    for (int t0 = 0; t0 < B; t0 += 1024) {
      const int b = t0 + threadIdx.x;
      const int f = (b < B && idx[b] == e) ? 1 : 0;
      // inclusive scan within the wave
      int v = f;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
      }
      if (lane == 63) wsum[wid] = v;
      __syncthreads();
      int before = 0;
      for (int w = 0; w < wid; ++w) before += wsum[w];
      const int pos = base + before + v - f;
      if (f) perm[pos] = b;
      __syncthreads();
      if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < 16; ++w) tot += wsum[w];
        base += tot;
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) offs[E] = base;
}

// The step's metric dict (moe.py:480-502) from the per-expert rows and the router terms, in one
// launch.  out = [gen, disc, div, intensity, aux, router, ED, differentiation, entropy, ALB, gan,
// then per expert: gen_i, disc_i, div_i, int_i, aux_i, std_int_i, mean_int_i, n_i].
__global__ void step_metrics_kernel(const float* mbuf, int E, const float* rl, const int32_t* counts,
                                    const float* countsf, float gan_strength, float diff_strength, float dec_w,
                                    int flags, float* out) {
  if (threadIdx.x != 0) return;
  const bool router = flags & 1, trained = flags & 2, alb_on = flags & 4, util_on = flags & 8, ed_on = flags & 16;
  float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  const int col[5] = {0, 8, 2, 3, 4};
  for (int e = 0; e < E; ++e)
    for (int k = 0; k < 5; ++k) s[k] += mbuf[e * 9 + col[k]];
  for (int k = 0; k < 5; ++k) out[k] = s[k] / (float)E;
  float gan = 0.f, diff = 0.f, ent = 0.f, alb = 0.f, ed = 0.f, rloss = 0.f;
  if (router) {
    gan = out[0] * gan_strength;                                  // moe.py:255
    if (diff_strength != 0.f) {                                   // moe.py:395-405
      float dli = 0.f;
      for (int a = 0; a < E; ++a)
        for (int b = a + 1; b < E; ++b) dli += fabsf(mbuf[a * 9 + 6] - mbuf[b * 9 + 6]);
      diff = -(dli * diff_strength) * diff_strength;
    }
    alb = alb_on ? rl[0] / dec_w : 0.f;
    ent = util_on ? rl[1] : 0.f;
    ed = ed_on ? rl[2] : 0.f;
    rloss = trained ? ed + gan + diff + ent + dec_w * alb : 0.f;   // moe.py:424-442
  }
  out[5] = rloss; out[6] = ed; out[7] = diff; out[8] = ent; out[9] = alb; out[10] = gan;
  for (int e = 0; e < E; ++e) {
    float* o = out + 11 + 8 * e;
    const float* m = mbuf + e * 9;
    o[0] = m[0]; o[1] = m[8]; o[2] = m[2]; o[3] = m[3]; o[4] = m[4]; o[5] = m[5]; o[6] = m[6];
    o[7] = countsf ? countsf[e] : (float)counts[e];
  }
}

// mean_intensities_in_batch_expert[mask] = s (moe.py:196-198): dst[rows[i]] = src[i]
__global__ void scatter_rows_kernel(const float* src, const int32_t* rows, const int32_t* start, int n, float* dst,
                                    const int32_t* live) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (start) rows += start[0];
  if (i < live_rows(live, n)) dst[rows ? rows[i] : i] = src[i];
}
}  // namespace

extern "C" int es_hinge_d(const float* ro, const float* fo, int n, const int32_t* rows, const float* w_ptr, float* out,
                          float* dro, float* dfo, es_stream_t stream) {
  ES_CHECK_ARG(n > 0, "hinge_d: n must be > 0");
  hipLaunchKernelGGL(hinge_d_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, ro, fo, n, rows, w_ptr, out, dro,
                     dfo);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_image_expsum(const es_view_t* x, es_dtype_t dt, const void* xp, float* s, es_stream_t stream) {
  hipLaunchKernelGGL(expsum_kernel, dim3(x->n), dim3(256), 0, (hipStream_t)stream, mkview(x), xp, dt == ES_BF16, s);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_image_expsum_bwd(const es_view_t* x, es_dtype_t dt, const void* xp, const float* coef,
                                   const es_view_t* dx, void* dxp, float beta, es_stream_t stream) {
  const int64_t total = (int64_t)x->n * x->c * x->h * x->w;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(expsum_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, mkview(x), xp,
                     dt == ES_BF16, coef, mkview(dx), (float*)dxp, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_gen_losses(const es_gen_loss_t* p, const float* fo, const float* l1, const float* l2,
                             const float* n1, const float* n2, const float* std_, const float* s,
                             const float* intensity, const float* coord, const float* pos, const float* w_ptr,
                             float* out, float* dfo, float* dl1, float* dl2, float* dcoord, float* coef,
                             es_stream_t stream) {
  ES_CHECK_ARG(p->n > 0 && p->n <= 4096, "gen_losses: n=%d out of range (1..4096)", p->n);
  ES_CHECK_ARG(p->latent >= 1, "gen_losses: latent must be >= 1");
  hipStream_t st = (hipStream_t)stream;
  const dim3 waves((p->n + 3) / 4);
  hipLaunchKernelGGL(gen_losses_a, waves, dim3(256), 0, st, *p, l1, l2, n1, n2, coef, dfo);
  hipLaunchKernelGGL(gen_losses_b, dim3(1), dim3(256), 0, st, *p, fo, std_, s, intensity, coord, pos, w_ptr, out,
                     dfo, coef, dcoord, dl2);
  hipLaunchKernelGGL(gen_losses_c, waves, dim3(256), 0, st, *p, l1, l2, dl1, dl2);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_router_gumbel(const float* logits, const float* expo, int B, int E, float tau, float* gates,
                                int32_t* idx, int32_t* counts, es_stream_t stream) {
  hipLaunchKernelGGL(router_gumbel_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, logits, expo,
                     B, E, tau, gates, idx, counts);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_router_alb(const float* gates, int B, int E, float tau, float coef, float* out, float* dlogits,
                             es_stream_t stream) {
  ES_CHECK_ARG(E <= 64, "router_alb: E <= 64");
  hipLaunchKernelGGL(router_alb_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, gates, B, E, tau, coef, out,
                     dlogits);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_router_loss(const float* gates, const int32_t* idx, const float* feat, int B, int E, float tau,
                              float alb_coef, float util_strength, float ed_strength, const float* colsum,
                              int B_total, const float* feat_all, const int32_t* idx_all, int B_all, float* out,
                              float* dlogits, es_stream_t stream) {
  ES_CHECK_ARG(B > 0 && E >= 1 && E <= 64, "router_loss: B=%d E=%d (E <= 64)", B, E);
  ES_CHECK_ARG(ed_strength == 0.f || (feat && idx), "router_loss: ED needs feat and idx");
  hipStream_t st = (hipStream_t)stream;
  if (B_total <= 0) B_total = B;
  if (!feat_all) { feat_all = feat; idx_all = idx; B_all = B; }
  if (ed_strength != 0.f)
    hipLaunchKernelGGL(router_ed_pairs_kernel, dim3((B + 255) / 256, E), dim3(256), 0, st, feat, B, feat_all,
                       idx_all, B_all, E, dlogits);
  hipLaunchKernelGGL(router_loss_kernel, dim3(1), dim3(1024), 0, st, gates, idx, B, E, tau, alb_coef, util_strength,
                     ed_strength, colsum, (float)B_total, out, dlogits);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_router_colsum(const float* gates, int B, int E, float* out, es_stream_t stream) {
  ES_CHECK_ARG(B > 0 && E >= 1, "router_colsum: B=%d E=%d", B, E);
  hipLaunchKernelGGL(router_colsum_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, gates, B, E, out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_dp_metrics_merge(const float* rows, int world, int E, float* out, es_stream_t stream) {
  ES_CHECK_ARG(world >= 1 && E >= 1, "dp_metrics_merge: world=%d E=%d", world, E);
  hipLaunchKernelGGL(dp_metrics_merge_kernel, dim3((E + 63) / 64), dim3(64), 0, (hipStream_t)stream, rows, world, E,
                     out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_scatter_rows(const float* src, const int32_t* rows, int n, float* dst, es_stream_t stream) {
  if (n <= 0) return ES_OK;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, src, rows,
                     (const int32_t*)nullptr, n, dst, (const int32_t*)nullptr);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_router_dispatch(const int32_t* idx, int B, int E, int32_t* perm, int32_t* offs,
                                  es_stream_t stream) {
  ES_CHECK_ARG(B > 0 && E >= 1, "router_dispatch: B=%d E=%d", B, E);
  hipLaunchKernelGGL(router_dispatch_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, idx, B, E, perm, offs);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_step_metrics(const float* mbuf, int E, const float* rl, const int32_t* counts, const float* countsf,
                               float gan_strength, float diff_strength, float dec_w, int flags, float* out,
                               es_stream_t stream) {
  ES_CHECK_ARG(E >= 1 && (counts || countsf), "step_metrics: E=%d, counts", E);
  ES_CHECK_ARG(!(flags & 1) || rl, "step_metrics: router terms need rl");
  hipLaunchKernelGGL(step_metrics_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, mbuf, E, rl, counts, countsf,
                     gan_strength, diff_strength, dec_w, flags, out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_scatter_rows_at(const float* src, const int32_t* perm, const int32_t* start, int n,
                                  const int32_t* live, float* dst, es_stream_t stream) {
  if (n <= 0) return ES_OK;
  ES_CHECK_ARG(perm && start, "scatter_rows_at: perm / start");
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, src, perm, start,
                     n, dst, live);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
