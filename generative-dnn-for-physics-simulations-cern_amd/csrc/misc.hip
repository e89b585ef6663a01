// Pooling, resampling, layout, spectral norm, Adam, RNG and the error/ABI plumbing.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

// ------------------------------------------------------------------------------------- errors
static thread_local char g_err[512] = "";
void es_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
extern "C" const char* es_last_error(void) { return g_err; }
extern "C" int es_version(void) { return 1; }
extern "C" int es_device_sync(void) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) { es_set_error("hipDeviceSynchronize: %s", hipGetErrorString(e)); return ES_ERR_HIP; }
  return ES_OK;
}

namespace {
struct View {
  int n, c, h, w;
  int64_t s[4];
  const int32_t* rows;   // live images (es_view_t.rows; NULL: n)
  __device__ __forceinline__ int64_t off(int in, int ic, int ih, int iw) const {
    return in * s[0] + ic * s[1] + ih * s[2] + iw * s[3];
  }
  __device__ __forceinline__ int live() const { return live_rows(rows, n); }
  // elements of the live images
  __device__ __forceinline__ int64_t live_total() const { return (int64_t)live() * c * h * w; }
};
View mkview(const es_view_t* v) {
  View r;
  r.n = v->n; r.c = v->c; r.h = v->h; r.w = v->w;
  for (int i = 0; i < 4; ++i) r.s[i] = v->s[i];
  r.rows = v->rows;
  return r;
}
// the live-count pointer of a pair of views of one batch (either may carry it)
const int32_t* rows_of(const es_view_t* a, const es_view_t* b) { return a->rows ? a->rows : (b ? b->rows : nullptr); }
__device__ __forceinline__ float ldf(const void* p, int bf, int64_t i) {
  return bf ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ void stf(void* p, int bf, int64_t i, float v) {
  if (bf) ((bf16*)p)[i] = (bf16)v;
  else ((float*)p)[i] = v;
}
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
int grid_for(int64_t total) { return (int)std::min<int64_t>((total + 255) / 256, 8192); }
#define GRID_STRIDE(e, total) \
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (total); e += (int64_t)gridDim.x * blockDim.x)

// ------------------------------------------------------------------------------------ max pool
__global__ void maxpool_fwd_kernel(View x, const void* xp, int bf, int kh, int kw, int sh, int sw, View y,
                                   void* yp, uint8_t* idx) {
  const int64_t total = y.live_total();
  const bool cl = y.s[1] == 1 && y.c > 1;
  GRID_STRIDE(e, total) {
    int n, c, h, w;
    decompose(y, cl, e, n, c, h, w);
    float best = -INFINITY;
    int bi = 0;
    for (int i = 0; i < kh; ++i)
      for (int j = 0; j < kw; ++j) {
        const float v = ldf(xp, bf, x.off(n, c, h * sh + i, w * sw + j));
        if (v > best || (isnan(v) && !isnan(best))) { best = v; bi = i * kw + j; }
      }
    stf(yp, bf, y.off(n, c, h, w), best);
    if (idx) idx[e] = (uint8_t)bi;
  }
}

// gather form: every input position sums the output windows whose argmax it is
__global__ void maxpool_bwd_kernel(View dy, const void* dyp, int bf, const uint8_t* idx, int kh, int kw, int sh,
                                   int sw, View dx, void* dxp, float beta) {
  const int64_t total = dx.live_total();
  const bool cl = dx.s[1] == 1 && dx.c > 1;
  const bool ycl = dy.s[1] == 1 && dy.c > 1;
  GRID_STRIDE(e, total) {
    int n, c, h, w;
    decompose(dx, cl, e, n, c, h, w);
    float g = 0.f;
    // output rows oh with oh*sh <= h < oh*sh + kh
    const int oh0 = h >= kh ? (h - kh) / sh + 1 : 0, oh1 = min(dy.h - 1, h / sh);
    const int ow0 = w >= kw ? (w - kw) / sw + 1 : 0, ow1 = min(dy.w - 1, w / sw);
    for (int oh = oh0; oh <= oh1; ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int i = h - oh * sh, j = w - ow * sw;
        if (i < 0 || i >= kh || j < 0 || j >= kw) continue;
        // idx is stored in the dy view's element order (ycl)
        const int64_t ye = ycl ? ((((int64_t)n * dy.h + oh) * dy.w + ow) * dy.c + c)
                               : ((((int64_t)n * dy.c + c) * dy.h + oh) * dy.w + ow);
        if (idx[ye] == i * kw + j) g += ldf(dyp, bf, dy.off(n, c, oh, ow));
      }
    const int64_t o = dx.off(n, c, h, w);
    if (beta != 0.f) g += beta * ldf(dxp, bf, o);
    stf(dxp, bf, o, g);
  }
}

// Non-overlapping windows (kernel == stride) on dense NHWC views: every input position has at most
// one window, so a thread owns VN channels of one input pixel, reads the window's gradient and
// argmax bytes as vectors and writes the VN gradients with one 16-byte store.
template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_nhwc(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                       int N, int C, int H, int W, int P, int Q, int kh, int kw,
                                                       T* __restrict__ dx, float beta, const int32_t* rows) {
  constexpr int VN = 16 / sizeof(T);
  const int cv = C / VN;
  const uint32_t total = (uint32_t)live_rows(rows, N) * H * W * cv;
  for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < total; e += gridDim.x * 256u) {
    const uint32_t pix = e / cv;
    const int c0 = (int)(e - pix * cv) * VN;
    const uint32_t nh = pix / W;
    const int w = (int)(pix - nh * W);
    const int n = (int)(nh / H), h = (int)(nh - (uint32_t)n * H);
    const int oh = h / kh, ow = w / kw;
    float g[VN];
#pragma unroll
    for (int v = 0; v < VN; ++v) g[v] = 0.f;
    if (oh < P && ow < Q) {
      const int64_t ye = (((int64_t)n * P + oh) * Q + ow) * C + c0;
      const int want = (h - oh * kh) * kw + (w - ow * kw);
      T gv[VN];
      uint8_t iv[VN];
      *(uint4*)gv = *(const uint4*)(dy + ye);
      if constexpr (VN == 8) *(uint2*)iv = *(const uint2*)(idx + ye);
      else *(uint32_t*)iv = *(const uint32_t*)(idx + ye);
#pragma unroll
      for (int v = 0; v < VN; ++v) g[v] = iv[v] == want ? to_f(gv[v]) : 0.f;
    }
    T* o = dx + (int64_t)pix * C + c0;
    T ov[VN];
    if (beta != 0.f) *(uint4*)ov = *(const uint4*)o;
#pragma unroll
    for (int v = 0; v < VN; ++v) ov[v] = from_f<T>(beta != 0.f ? g[v] + beta * to_f(ov[v]) : g[v]);
    *(uint4*)o = *(const uint4*)ov;
  }
}

// Forward on dense NHWC views: a thread owns VN channels of one output pixel, reads the window's
// rows as 16-byte vectors and writes the VN maxima (one 16-byte store) and their argmax bytes
// (first max in row-major window order, NaN wins, as torch).  The generic kernel above decodes
// every element's coordinates and moves 2 / 4 bytes per access (~3.5x slower on the aux
// regressor's pools).
template <typename T>
__global__ void __launch_bounds__(256) maxpool_fwd_nhwc(const T* __restrict__ x, int N, int C, int H, int W, int P,
                                                       int Q, int kh, int kw, int sh, int sw, T* __restrict__ y,
                                                       uint8_t* __restrict__ idx, const int32_t* rows) {
  constexpr int VN = 16 / sizeof(T);
  const int cv = C / VN;
  const uint32_t total = (uint32_t)live_rows(rows, N) * P * Q * cv;
  for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < total; e += gridDim.x * 256u) {
    const uint32_t pix = e / cv;
    const int c0 = (int)(e - pix * cv) * VN;
    const uint32_t np = pix / Q;
    const int q = (int)(pix - np * Q);
    const int n = (int)(np / P), p = (int)(np - (uint32_t)n * P);
    float best[VN];
    uint8_t bi[VN];
#pragma unroll
    for (int v = 0; v < VN; ++v) { best[v] = -INFINITY; bi[v] = 0; }
    const T* xb = x + ((int64_t)n * H + p * sh) * W * C + (int64_t)(q * sw) * C + c0;
    for (int i = 0; i < kh; ++i)
      for (int j = 0; j < kw; ++j) {
        T xv[VN];
        *(uint4*)xv = *(const uint4*)(xb + ((int64_t)i * W + j) * C);
#pragma unroll
        for (int v = 0; v < VN; ++v) {
          const float f = to_f(xv[v]);
          if (f > best[v] || (isnan(f) && !isnan(best[v]))) { best[v] = f; bi[v] = (uint8_t)(i * kw + j); }
        }
      }
    T ov[VN];
#pragma unroll
    for (int v = 0; v < VN; ++v) ov[v] = from_f<T>(best[v]);
    *(uint4*)(y + (int64_t)pix * C + c0) = *(const uint4*)ov;
    if (idx) {
      if constexpr (VN == 8) *(uint2*)(idx + (int64_t)pix * C + c0) = *(const uint2*)bi;
      else *(uint32_t*)(idx + (int64_t)pix * C + c0) = *(const uint32_t*)bi;
    }
  }
}

bool dense_nhwc(const es_view_t* v) {
  const int64_t C = v->c;
  return v->s[1] == 1 && v->s[3] == C && v->s[2] == (int64_t)v->w * C && v->s[0] == (int64_t)v->h * v->w * C;
}

// ----------------------------------------------------------------------------- upsample bwd
__global__ void upsample_bwd_kernel(View du, const void* dup, int ubf, const int32_t* hs, const int32_t* hc,
                                    const int32_t* ws, const int32_t* wc, View dx, void* dxp, int xbf, float beta) {
  const int64_t total = dx.live_total();
  const bool cl = dx.s[1] == 1 && dx.c > 1;
  GRID_STRIDE(e, total) {
    int n, c, h, w;
    decompose(dx, cl, e, n, c, h, w);
    float g = 0.f;
    const int h0 = hs[h], w0 = ws[w];
    for (int i = 0; i < hc[h]; ++i)
      for (int j = 0; j < wc[w]; ++j) g += ldf(dup, ubf, du.off(n, c, h0 + i, w0 + j));
    const int64_t o = dx.off(n, c, h, w);
    if (beta != 0.f) g += beta * ldf(dxp, xbf, o);
    stf(dxp, xbf, o, g);
  }
}

// Dense NHWC forms (16-byte channel chunks per thread; the generic element-wise kernel above decodes
// every element and ran at ~1 TB/s): forward gather y[n,hu,wu,:] = x[n, hmap[hu], wmap[wu], :] (the
// proton generator's 35x19 -> 56x30 resize, materialised once per conv pass so that the conv runs on
// the ring kernels), and the backward sum over each source pixel's preimage rows / columns.
template <typename T>
__global__ void __launch_bounds__(256) upsample_fwd_nhwc(const T* __restrict__ x, int H, int W, int C,
                                                         const int32_t* __restrict__ hmap,
                                                         const int32_t* __restrict__ wmap, T* __restrict__ y,
                                                         int64_t rows, int Hu, int Wu, int N, const int32_t* nrows) {
  constexpr int V = 16 / sizeof(T);
  const int cv = C / V;
  if (nrows) rows = (int64_t)live_rows(nrows, N) * Hu * Wu;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * cv; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cv;
    const int c = (int)(i - r * cv) * V;
    const int64_t n = r / ((int64_t)Hu * Wu);
    const int hw = (int)(r - n * Hu * Wu), hu = hw / Wu, wu = hw - hu * Wu;
    *(uint4*)(y + r * C + c) = *(const uint4*)(x + ((n * H + hmap[hu]) * W + wmap[wu]) * C + c);
  }
}

template <typename T, typename TO>
__global__ void __launch_bounds__(256) upsample_bwd_nhwc(const T* __restrict__ du, int Hu, int Wu, int C,
                                                         const int32_t* __restrict__ hs, const int32_t* __restrict__ hc,
                                                         const int32_t* __restrict__ ws, const int32_t* __restrict__ wc,
                                                         TO* __restrict__ dx, int64_t rows, int H, int W, float beta,
                                                         int N, const int32_t* nrows) {
  const int cv = C / 4;
  if (nrows) rows = (int64_t)live_rows(nrows, N) * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * cv; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cv;
    const int c = (int)(i - r * cv) * 4;
    const int64_t n = r / ((int64_t)H * W);
    const int hw = (int)(r - n * H * W), h = hw / W, w = hw - h * W;
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    const int h0 = hs[h], w0 = ws[w], nh = hc[h], nw = wc[w];
    for (int a = 0; a < nh; ++a)
      for (int b = 0; b < nw; ++b) {
        const T* p = du + ((n * Hu + h0 + a) * Wu + w0 + b) * C + c;
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] += (float)p[e];
      }
    TO* o = dx + r * C + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (TO)(beta != 0.f ? g[e] + beta * (float)o[e] : g[e]);
  }
}

// ------------------------------------------------------------------------------------- copy
__global__ void copy_kernel(View x, const void* xp, int xbf, View y, void* yp, int ybf, float alpha, float beta) {
  const int64_t total = (int64_t)live_rows(x.rows ? x.rows : y.rows, x.n) * x.c * x.h * x.w;
  const bool cl = y.s[1] == 1 && y.c > 1;
  GRID_STRIDE(e, total) {
    int n, c, h, w;
    decompose(y, cl, e, n, c, h, w);
    float v = alpha * ldf(xp, xbf, x.off(n, c, h, w));
    const int64_t o = y.off(n, c, h, w);
    if (beta != 0.f) v += beta * ldf(yp, ybf, o);
    stf(yp, ybf, o, v);
  }
}

// Dense NCHW <-> NHWC re-layout (the neutron generator's fc2 rows [B][128*13*13] <-> the NHWC conv
// input, neutron/generator.py:18-20): per sample a [R][S] -> [S][R] transpose through a 64 x 64
// LDS tile, both sides read / written along contiguous rows (the generic element-wise copy above
// divides per element and ran at ~1 TB/s).
template <typename T>
__global__ void __launch_bounds__(256) transpose_kernel(const T* __restrict__ x, T* __restrict__ y, int R, int S,
                                                       const int32_t* rows) {
  __shared__ T tile[64][65];
  const int n = blockIdx.z, r0 = blockIdx.y * 64, s0 = blockIdx.x * 64;
  if (n >= live_rows(rows, gridDim.z)) return;
  const T* xs = x + (int64_t)n * R * S;
  T* ys = y + (int64_t)n * R * S;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 64; i += 4) {
    const int r = r0 + ty + i, c = s0 + tx;
    if (r < R && c < S) tile[ty + i][tx] = xs[(int64_t)r * S + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 64; i += 4) {
    const int c = s0 + ty + i, r = r0 + tx;
    if (r < R && c < S) ys[(int64_t)c * R + r] = tile[tx][ty + i];
  }
}

// x / y dense NCHW and dense NHWC of one shape (either direction): launch the transpose and
// return true
bool try_transpose(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_view_t* y, es_dtype_t ydt, void* yp,
                   hipStream_t st) {
  if (xdt != ydt || x->c <= 1) return false;
  const int64_t C = x->c, HW = (int64_t)x->h * x->w;
  auto nchw = [&](const es_view_t* v) {
    return v->s[3] == 1 && v->s[2] == v->w && v->s[1] == HW && v->s[0] == C * HW;
  };
  auto nhwc = [&](const es_view_t* v) {
    return v->s[1] == 1 && v->s[3] == C && v->s[2] == (int64_t)v->w * C && v->s[0] == C * HW;
  };
  int64_t R, S;
  if (nchw(x) && nhwc(y)) { R = C; S = HW; }
  else if (nhwc(x) && nchw(y)) { R = HW; S = C; }
  else return false;
  if (R * S * x->n * 4 >= (1ll << 31) || x->n > 65535) return false;
  const dim3 grid((unsigned)((S + 63) / 64), (unsigned)((R + 63) / 64), (unsigned)x->n);
  if (xdt == ES_BF16)
    hipLaunchKernelGGL(transpose_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)xp, (bf16*)yp, (int)R, (int)S,
                       rows_of(x, y));
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, st, (const float*)xp, (float*)yp, (int)R, (int)S,
                       rows_of(x, y));
  return true;
}

// ------------------------------------------------------------------------------- avg pool
__global__ void avgpool_fwd_kernel(View x, const void* xp, int bf, View y, void* yp) {
  // one wave per (n, c)
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (wave >= x.live() * x.c) return;
  const int n = wave / x.c, c = wave % x.c;
  const int hw = x.h * x.w;
  float s = 0.f;
  for (int i = lane; i < hw; i += 64) s += ldf(xp, bf, x.off(n, c, i / x.w, i % x.w));
  s = wave_sum(s);
  if (lane == 0) ((float*)yp)[y.off(n, c, 0, 0)] = s / (float)hw;
}
__global__ void avgpool_bwd_kernel(View dy, const float* dyp, View dx, void* dxp, int bf, float beta) {
  const int64_t total = (int64_t)live_rows(dx.rows ? dx.rows : dy.rows, dx.n) * dx.c * dx.h * dx.w;
  const bool cl = dx.s[1] == 1 && dx.c > 1;
  const float inv = 1.f / (float)(dx.h * dx.w);
  GRID_STRIDE(e, total) {
    int n, c, h, w;
    decompose(dx, cl, e, n, c, h, w);
    float g = dyp[dy.off(n, c, 0, 0)] * inv;
    const int64_t o = dx.off(n, c, h, w);
    if (beta != 0.f) g += beta * ldf(dxp, bf, o);
    stf(dxp, bf, o, g);
  }
}

__global__ void gather_rows_kernel(const float* src, int64_t sld, const int32_t* idx, const int32_t* start,
                                   int rows, int cols, float* dst, int64_t dld, const int32_t* live) {
  const int64_t total = (int64_t)rows * cols;
  if (start) idx += start[0];   // the expert's first position in the dispatch permutation (device)
  const int nl = live_rows(live, rows);   // rows past the live count (capacity padding): zeros
  GRID_STRIDE(e, total) {
    const int r = e / cols, c = e % cols;
    float v = 0.f;
    if (r < nl) {
      const int sr = idx ? idx[r] : r;
      v = src[sr * sld + c];
    }
    dst[r * dld + c] = v;
  }
}

// --------------------------------------------------------------------------- spectral norm
// One block.  v = normalize(W^T u); u = normalize(W v); sigma = u . (W v)
// (torch.nn.utils.spectral_norm.SpectralNorm.compute_weight, eps = 1e-12)
__device__ __forceinline__ void sn_power_body(const float* w, int h, int wd, float* u, float* v, float* sigma,
                                              int update, float* scratch, float* sh);

__global__ void __launch_bounds__(1024) sn_power_kernel(const float* w, int h, int wd, float* u, float* v,
                                                        float* sigma, int update, float* scratch, const int32_t* active) {
  __shared__ float sh[16];
  sn_power_body(w, h, wd, u, v, sigma, update && (active == nullptr || active[0] != 0), scratch, sh);
}

// several small layers' power iterations in one launch (one block per layer): the discriminator's
// conv_layers.0 / .4, fc2 and fc3 (neutron/discriminator.py:12-24) issue one launch instead of four
struct SnJobs {
  const float* w[ES_SN_BATCH_MAX];
  float* u[ES_SN_BATCH_MAX];
  float* v[ES_SN_BATCH_MAX];
  float* buf[ES_SN_BATCH_MAX];
  int h[ES_SN_BATCH_MAX], wd[ES_SN_BATCH_MAX];
};
__global__ void __launch_bounds__(1024) sn_power_batch_kernel(SnJobs j, int update, const int32_t* active) {
  __shared__ float sh[16];
  const int b = blockIdx.x;
  sn_power_body(j.w[b], j.h[b], j.wd[b], j.u[b], j.v[b], j.buf[b], update && (active == nullptr || active[0] != 0),
                j.buf[b] + 1, sh);
}

__device__ __forceinline__ void sn_power_body(const float* w, int h, int wd, float* u, float* v, float* sigma,
                                              int update, float* scratch, float* sh) {
  float* wv = scratch;       // [h]
  float* vt = scratch + h;   // [wd]
  if (update) {
    // t = W^T u: groups of 8 column chunks of 64 (lane = column), the block's waves split the
    // rows, per thread 8 independent column accumulators (loads of a row in flight together),
    // partials merged in LDS.  (A thread per column looping over every row was one dependent
    // load chain: ~30 us for the 64 x 128 fc2.)
    __shared__ float part[16][512];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    float ss = 0.f;
    for (int j0 = 0; j0 < wd; j0 += 512) {
      float t[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) t[c] = 0.f;
      for (int i = wid; i < h; i += nw) {
        const float ui = u[i];
        const float* wr = w + (int64_t)i * wd + j0 + lane;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (j0 + c * 64 + lane < wd) t[c] += wr[c * 64] * ui;
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) part[wid][c * 64 + lane] = t[c];
      __syncthreads();
      for (int jj = threadIdx.x; jj < 512 && j0 + jj < wd; jj += blockDim.x) {
        float sj = 0.f;
        for (int k = 0; k < nw; ++k) sj += part[k][jj];
        vt[j0 + jj] = sj;
        ss += sj * sj;
      }
      __syncthreads();
    }
    const float nv = fmaxf(sqrtf(block_sum(ss, sh)), 1e-12f);
    for (int j = threadIdx.x; j < wd; j += blockDim.x) v[j] = vt[j] / nv;
    __syncthreads();
  }
  // s = W v (a wave per row, lanes along the row, two independent accumulators)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int i = wid; i < h; i += nw) {
    float t0 = 0.f, t1 = 0.f;
    int j = lane;
    for (; j + 64 < wd; j += 128) {
      t0 += w[(int64_t)i * wd + j] * v[j];
      t1 += w[(int64_t)i * wd + j + 64] * v[j + 64];
    }
    if (j < wd) t0 += w[(int64_t)i * wd + j] * v[j];
    const float t = wave_sum(t0 + t1);
    if (lane == 0) wv[i] = t;
  }
  __syncthreads();
  if (update) {
    float ss = 0.f;
    for (int i = threadIdx.x; i < h; i += blockDim.x) ss += wv[i] * wv[i];
    const float nu = fmaxf(sqrtf(block_sum(ss, sh)), 1e-12f);
    for (int i = threadIdx.x; i < h; i += blockDim.x) u[i] = wv[i] / nu;
    __syncthreads();
  }
  float d = 0.f;
  for (int i = threadIdx.x; i < h; i += blockDim.x) d += u[i] * wv[i];
  d = block_sum(d, sh);
  if (threadIdx.x == 0) sigma[0] = d;
  // snapshot of the u, v this call used (for the backward; the next call updates them in place)
  float* snap = scratch + h + wd;
  for (int i = threadIdx.x; i < h; i += blockDim.x) snap[i] = u[i];
  for (int j = threadIdx.x; j < wd; j += blockDim.x) snap[h + j] = v[j];
}

// ---- multi-block power iteration for the large reshaped weights (discriminator fc1: 128 x 1305)
// t = W^T u : block = 64 columns x 4 row groups, LDS reduction over the row groups
__global__ void __launch_bounds__(256) sn_wtu_kernel(const float* __restrict__ w, int h, int wd,
                                                     const float* __restrict__ u, float* __restrict__ vt) {
  // (an inactive update still computes vt; sn_wv_kernel then reads the stored v instead)
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  float t = 0.f;
  if (j < wd)
    for (int i = rg; i < h; i += 4) t += w[(int64_t)i * wd + j] * u[i];
  __shared__ float sh[4][64];
  sh[rg][cl] = t;
  __syncthreads();
  if (rg == 0 && j < wd) vt[j] = sh[0][cl] + sh[1][cl] + sh[2][cl] + sh[3][cl];
}
// wv = W (x * scale), one wave per row; scale = 1/||x|| when `normalize` (x = the new v, written
// back normalised by block 0), else 1 (x = the stored v)
__global__ void __launch_bounds__(256) sn_wv_kernel(const float* __restrict__ w, int h, int wd, const float* x,
                                                    int normalize, float* v_out, float* __restrict__ wv,
                                                    const float* v_stored, const int32_t* active) {
  __shared__ float sh[8];
  if (normalize && active && active[0] == 0) {   // inactive: sigma from the stored v, no update
    normalize = 0;
    x = v_stored;
  }
  float sc = 1.f;
  if (normalize) {
    float ss = 0.f;
    for (int j = threadIdx.x; j < wd; j += 256) ss += x[j] * x[j];
    sc = 1.f / fmaxf(sqrtf(block_sum(ss, sh)), 1e-12f);
    if (blockIdx.x == 0)
      for (int j = threadIdx.x; j < wd; j += 256) v_out[j] = x[j] * sc;
  }
  const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= h) return;
  float t = 0.f;
  for (int j = lane; j < wd; j += 64) t += w[(int64_t)i * wd + j] * (x[j] * sc);
  t = wave_sum(t);
  if (lane == 0) wv[i] = t;
}
// u = wv / ||wv|| (update), sigma = u . wv
__global__ void __launch_bounds__(256) sn_final_kernel(int h, int wd, const float* wv, float* u, const float* v,
                                                       int update, float* sigma, float* snap, const int32_t* active) {
  __shared__ float sh[8];
  if (update && (active == nullptr || active[0] != 0)) {
    float ss = 0.f;
    for (int i = threadIdx.x; i < h; i += 256) ss += wv[i] * wv[i];
    const float nu = fmaxf(sqrtf(block_sum(ss, sh)), 1e-12f);
    for (int i = threadIdx.x; i < h; i += 256) u[i] = wv[i] / nu;
    __syncthreads();
  }
  float d = 0.f;
  for (int i = threadIdx.x; i < h; i += 256) d += u[i] * wv[i];
  d = block_sum(d, sh);
  if (threadIdx.x == 0) sigma[0] = d;
  for (int i = threadIdx.x; i < h; i += 256) snap[i] = u[i];
  for (int j = threadIdx.x; j < wd; j += 256) snap[h + j] = v[j];
}

// ---- multi-block backward: block partials of <G, W> (pass 1), then the elementwise update with
// every block re-reducing the (<= 256) partials (pass 2)
__global__ void __launch_bounds__(256) sn_dot_kernel(const float* __restrict__ g, const float* __restrict__ w,
                                                     int n, float* part) {
  __shared__ float sh[8];
  float d = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) d += g[i] * w[i];
  d = block_sum(d, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = d;
}
__global__ void __launch_bounds__(256) sn_bwd_apply_kernel(const float* __restrict__ g, int h, int wd,
                                                           const float* u, const float* v, const float* sigma,
                                                           const float* part, int nparts, float* dw, float beta) {
  __shared__ float sh[8];
  float d = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) d += part[i];
  d = block_sum(d, sh);
  const float s = sigma[0];
  const float c = d / (s * s);
  const int n = h * wd;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int r = i / wd, col = i - r * wd;
    const float val = g[i] / s - c * u[r] * v[col];
    dw[i] = (beta != 0.f ? beta * dw[i] : 0.f) + val;
  }
}

// dW_orig = beta*dW + G/s - (<G,W>/s^2) u v^T
__device__ __forceinline__ void sn_bwd_body(const float* w, const float* g, int h, int wd, const float* u,
                                            const float* v, const float* sigma, float* dw, float beta, float* sh);
__global__ void __launch_bounds__(1024) sn_bwd_kernel(const float* w, const float* g, int h, int wd,
                                                      const float* u, const float* v, const float* sigma,
                                                      float* dw, float beta) {
  __shared__ float sh[16];
  sn_bwd_body(w, g, h, wd, u, v, sigma, dw, beta, sh);
}
// several small layers' weight_orig gradients in one launch (one block per layer)
struct SnBwdJobs {
  const float* w[ES_SN_BATCH_MAX];
  const float* g[ES_SN_BATCH_MAX];
  const float* u[ES_SN_BATCH_MAX];
  const float* v[ES_SN_BATCH_MAX];
  const float* sigma[ES_SN_BATCH_MAX];
  float* dw[ES_SN_BATCH_MAX];
  int h[ES_SN_BATCH_MAX], wd[ES_SN_BATCH_MAX];
};
__global__ void __launch_bounds__(1024) sn_bwd_batch_kernel(SnBwdJobs j, float beta) {
  __shared__ float sh[16];
  const int b = blockIdx.x;
  sn_bwd_body(j.w[b], j.g[b], j.h[b], j.wd[b], j.u[b], j.v[b], j.sigma[b], j.dw[b], beta, sh);
}
__device__ __forceinline__ void sn_bwd_body(const float* w, const float* g, int h, int wd, const float* u,
                                            const float* v, const float* sigma, float* dw, float beta, float* sh) {
  const int n = h * wd;                     // < 2^20 (host check)
  const int bd = blockDim.x;
  float d0 = 0.f, d1 = 0.f;
  int i = threadIdx.x;
  for (; i + bd < n; i += 2 * bd) {         // two independent chains
    d0 += g[i] * w[i];
    d1 += g[i + bd] * w[i + bd];
  }
  if (i < n) d0 += g[i] * w[i];
  const float d = block_sum(d0 + d1, sh);
  const float s = sigma[0];
  const float c = d / (s * s);
  const float is = 1.f / s;
  for (int k = threadIdx.x; k < n; k += bd) {
    const int r = k / wd, col = k - r * wd;  // 32-bit division (a 64-bit one per element cost ~100 instructions)
    const float val = g[k] * is - c * u[r] * v[col];
    dw[k] = (beta != 0.f ? beta * dw[k] : 0.f) + val;
  }
}

// ----------------------------------------------------------------------------------- Adam
// torch.optim.Adam (single tensor): m.lerp_(g, 1-b1); v = b2*v + (1-b2)*g*g;
// p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                            float step_size, float bc2_sqrt, float gscale) {
  GRID_STRIDE(i, n) {
    const float gi = g[i] * gscale;
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = p[i] - step_size * (mi / (sqrtf(vi) / bc2_sqrt + eps));
  }
}

// step read on the device; bias corrections as torch computes them (double), per thread
__global__ void adam_dev_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                                const int32_t* __restrict__ step_ptr, float gscale, const int32_t* active) {
  if (active && active[0] == 0) return;   // an expert skipped this step (moe.py:126-135): no update
  const int step = step_ptr[0];
  const double bc1 = 1.0 - pow((double)b1, (double)step);
  const double bc2 = 1.0 - pow((double)b2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  GRID_STRIDE(i, n) {
    const float gi = g[i] * gscale;
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = p[i] - step_size * (mi / (sqrtf(vi) / bc2_sqrt + eps));
  }
}
__global__ void counter_add_kernel(int32_t* c, int32_t v, const int32_t* flag) {
  if (flag == nullptr || flag[0] != 0) c[0] += v;
}
__global__ void counter_add_i64_kernel(int64_t* c, int64_t v, const int32_t* flag) {
  if (flag == nullptr || flag[0] != 0) c[0] += v;
}

// Multi-expert step plan (moe.py:97-135 on the device): from the local expert counts and, data
// parallel, the all-gathered [world][E] counts, per expert e:
//   rows[e]   live local rows of the expert's capacity buffers: local count when the expert trains
//             (global count > 1, moe.py:126) and this rank runs it (>= min_local samples), else 0;
//   active[e] 1 when the expert trains this step (its optimizers, BatchNorm running statistics and
//             spectral-norm vectors update), else 0;
//   n0[e]     this rank's first sample in the expert's global batch (randomness at global indices);
//   w[e]      class_counts_adjusted = float(local count) / float(B) (moe.py:99-100, 522, 562);
//   gcnt[e]   the global count (float; SyncBN / SDI normalisers);
//   lcnt[e]   rows[e] as float (the data-parallel metric merge's per-rank weights).
__global__ void expert_plan_kernel(const int32_t* counts, const int32_t* counts_all, int world, int rank, int E, int B,
                                   int min_local, int32_t* rows, int32_t* active, int32_t* n0, float* w, float* gcnt,
                                   float* lcnt) {
  const int e = threadIdx.x;
  if (e >= E) return;
  int g = counts[e], before = 0;
  if (counts_all) {
    g = 0;
    for (int r = 0; r < world; ++r) {
      const int c = counts_all[r * E + e];
      g += c;
      if (r < rank) before += c;
    }
  }
  const int loc = counts[e];
  const int act = g > 1 ? 1 : 0;
  const int nr = act && loc >= min_local ? loc : 0;
  rows[e] = nr;
  active[e] = act;
  n0[e] = before;
  w[e] = (float)loc / (float)B;
  gcnt[e] = (float)g;
  lcnt[e] = (float)nr;
}
__global__ void div_by_kernel(float* x, int n, const float* d) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] / fmaxf(d[0], 1.f);
}

// EMA of a flat parameter buffer (EMAHelper.update, loop.py:392-400): s = decay*s + (1-decay)*p with
// the reference's two roundings and one add (contraction off: no FMA), float4 when aligned.
__global__ void ema_kernel(float* __restrict__ s, const float* __restrict__ p, int64_t n, float d, float omd) {
#pragma clang fp contract(off)
  const int64_t n4 = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(p)) & 15) ? 0 : n / 4;
  GRID_STRIDE(i, n4) {
    float4 a = reinterpret_cast<const float4*>(s)[i];
    const float4 b = reinterpret_cast<const float4*>(p)[i];
    a.x = d * a.x + omd * b.x;
    a.y = d * a.y + omd * b.y;
    a.z = d * a.z + omd * b.z;
    a.w = d * a.w + omd * b.w;
    reinterpret_cast<float4*>(s)[i] = a;
  }
  GRID_STRIDE(j, n - 4 * n4) {
    const int64_t i = 4 * n4 + j;
    s[i] = d * s[i] + omd * p[i];
  }
}

// ------------------------------------------------------------------------------------ RNG
__global__ void randn_kernel(float* out, int64_t n, uint64_t seed, uint32_t sid, const int32_t* step_ptr,
                             int32_t step_mul, int64_t pair0, const int32_t* off_ptr, int64_t off_pairs) {
  if (step_ptr) sid += (uint32_t)(step_ptr[0] * step_mul);
  if (off_ptr) pair0 += (int64_t)off_ptr[0] * off_pairs;
  // Box-Muller on pairs: counter = global pair index (pair0 = offset / 2)
  const int64_t pairs = (n + 1) / 2;
  GRID_STRIDE(i, pairs) {
    const int64_t q = i + pair0;
    u32x4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), sid, 0x5EED0001u, (uint32_t)seed,
                            (uint32_t)(seed >> 32));
    const float u1 = ((r.x >> 8) + 1) * (1.f / 16777217.f);   // (0, 1]
    const float u2 = (r.y >> 8) * (1.f / 16777216.f);
    const float rad = sqrtf(-2.f * logf(u1));
    float s, c;
    sincosf(6.2831853071795864f * u2, &s, &c);
    out[2 * i] = rad * c;
    if (2 * i + 1 < n) out[2 * i + 1] = rad * s;
  }
}
__global__ void rand_exp_kernel(float* out, int64_t n, uint64_t seed, uint32_t sid, const int32_t* step_ptr,
                                int32_t step_mul, int64_t off) {
  if (step_ptr) sid += (uint32_t)(step_ptr[0] * step_mul);
  GRID_STRIDE(i, n) {
    const int64_t q = i + off;
    u32x4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), sid, 0x5EED0002u, (uint32_t)seed,
                            (uint32_t)(seed >> 32));
    const float u = ((r.x >> 8) + 1) * (1.f / 16777217.f);
    out[i] = -logf(u);
  }
}
__global__ void dropout_mask_kernel(uint8_t* out, int64_t n, es_dropout_t d) {
  resolve_stream(d);
  GRID_STRIDE(i, n) out[i] = dropout_keep(d, (uint64_t)i) ? 1 : 0;
}
}  // namespace

// ============================================================================= C ABI
extern "C" int es_maxpool_fwd(const es_view_t* x, es_dtype_t dt, const void* xp, int kh, int kw, int sh,
                              int sw, const es_view_t* y, void* yp, uint8_t* idx, es_stream_t stream) {
  ES_CHECK_ARG(y->h == (x->h - kh) / sh + 1 && y->w == (x->w - kw) / sw + 1, "maxpool: output shape");
  const int64_t total = (int64_t)y->n * y->c * y->h * y->w;
  const int vn = dt == ES_BF16 ? 8 : 4;
  if (dense_nhwc(x) && dense_nhwc(y) && x->c % vn == 0 && x->c > 1 && total < (1ll << 31)) {
    const int64_t items = total / vn;
    const unsigned grid = (unsigned)std::min<int64_t>((items + 255) / 256, 16384);
    if (dt == ES_BF16)
      hipLaunchKernelGGL(maxpool_fwd_nhwc<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16*)xp,
                         x->n, x->c, x->h, x->w, y->h, y->w, kh, kw, sh, sw, (bf16*)yp, idx, rows_of(x, y));
    else
      hipLaunchKernelGGL(maxpool_fwd_nhwc<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)xp,
                         x->n, x->c, x->h, x->w, y->h, y->w, kh, kw, sh, sw, (float*)yp, idx, rows_of(x, y));
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  View yv = mkview(y);
  yv.rows = rows_of(x, y);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     mkview(x), xp, dt == ES_BF16, kh, kw, sh, sw, yv, yp, idx);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_maxpool_bwd(const es_view_t* dy, es_dtype_t dt, const void* dyp, const uint8_t* idx, int kh,
                              int kw, int sh, int sw, const es_view_t* dx, void* dxp, float beta,
                              es_stream_t stream) {
  const int64_t total = (int64_t)dx->n * dx->c * dx->h * dx->w;
  const int vn = dt == ES_BF16 ? 8 : 4;
  if (kh == sh && kw == sw && dense_nhwc(dy) && dense_nhwc(dx) && dx->c % vn == 0 && dx->c > 1 &&
      total < (1ll << 31)) {
    const int64_t items = total / vn;
    const unsigned grid = (unsigned)std::min<int64_t>((items + 255) / 256, 16384);
    if (dt == ES_BF16)
      hipLaunchKernelGGL(maxpool_bwd_nhwc<bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16*)dyp, idx,
                         dx->n, dx->c, dx->h, dx->w, dy->h, dy->w, kh, kw, (bf16*)dxp, beta, rows_of(dy, dx));
    else
      hipLaunchKernelGGL(maxpool_bwd_nhwc<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)dyp,
                         idx, dx->n, dx->c, dx->h, dx->w, dy->h, dy->w, kh, kw, (float*)dxp, beta, rows_of(dy, dx));
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  View dxv = mkview(dx);
  dxv.rows = rows_of(dy, dx);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     mkview(dy), dyp, dt == ES_BF16, idx, kh, kw, sh, sw, dxv, dxp, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_upsample_fwd(const es_view_t* x, es_dtype_t dt, const void* xp, const int32_t* hmap,
                               const int32_t* wmap, const es_view_t* y, void* yp, es_stream_t stream) {
  ES_CHECK_ARG(x->n == y->n && x->c == y->c && dense_nhwc(x) && dense_nhwc(y) && x->c % (dt == ES_BF16 ? 8 : 4) == 0,
               "upsample fwd: dense NHWC views with 16-byte channel chunks required");
  const int64_t rows = (int64_t)y->n * y->h * y->w;
  const int64_t n = rows * (x->c / (dt == ES_BF16 ? 8 : 4));
  if (n == 0) return ES_OK;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 16384);
  if (dt == ES_BF16)
    hipLaunchKernelGGL(upsample_fwd_nhwc<bf16>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16*)xp,
                       x->h, x->w, x->c, hmap, wmap, (bf16*)yp, rows, y->h, y->w, y->n, rows_of(x, y));
  else
    hipLaunchKernelGGL(upsample_fwd_nhwc<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float*)xp,
                       x->h, x->w, x->c, hmap, wmap, (float*)yp, rows, y->h, y->w, y->n, rows_of(x, y));
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_upsample_bwd(const es_view_t* dxu, es_dtype_t dt, const void* dxup, const int32_t* hstart,
                               const int32_t* hcount, const int32_t* wstart, const int32_t* wcount,
                               const es_view_t* dx, es_dtype_t dxdt, void* dxp, float beta, es_stream_t stream) {
  const int64_t total = (int64_t)dx->n * dx->c * dx->h * dx->w;
  if (dense_nhwc(dxu) && dense_nhwc(dx) && dxu->c == dx->c && dx->c % 4 == 0 && total > 0) {
    const int64_t rows = (int64_t)dx->n * dx->h * dx->w;
    const int blocks = (int)std::min<int64_t>((rows * (dx->c / 4) + 255) / 256, 16384);
    hipStream_t st = (hipStream_t)stream;
#define ES_UB(T, TO) hipLaunchKernelGGL((upsample_bwd_nhwc<T, TO>), dim3(blocks), dim3(256), 0, st, (const T*)dxup, \
                                        dxu->h, dxu->w, dx->c, hstart, hcount, wstart, wcount, (TO*)dxp, rows, dx->h, dx->w, beta, \
                                        dx->n, rows_of(dxu, dx))
    if (dt == ES_BF16 && dxdt == ES_BF16) ES_UB(bf16, bf16);
    else if (dt == ES_BF16) ES_UB(bf16, float);
    else if (dxdt == ES_BF16) ES_UB(float, bf16);
    else ES_UB(float, float);
#undef ES_UB
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  View dxv = mkview(dx);
  dxv.rows = rows_of(dxu, dx);
  hipLaunchKernelGGL(upsample_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     mkview(dxu), dxup, dt == ES_BF16, hstart, hcount, wstart, wcount, dxv, dxp,
                     dxdt == ES_BF16, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_copy(const es_view_t* x, es_dtype_t xdt, const void* xp, const es_view_t* y, es_dtype_t ydt,
                       void* yp, float alpha, float beta, es_stream_t stream) {
  ES_CHECK_ARG(x->n == y->n && x->c == y->c && x->h == y->h && x->w == y->w, "copy: shape mismatch");
  const int64_t total = (int64_t)x->n * x->c * x->h * x->w;
  if (total == 0) return ES_OK;
  if (alpha == 1.f && beta == 0.f && try_transpose(x, xdt, xp, y, ydt, yp, (hipStream_t)stream)) {
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  hipLaunchKernelGGL(copy_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, mkview(x), xp,
                     xdt == ES_BF16, mkview(y), yp, ydt == ES_BF16, alpha, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_avgpool_fwd(const es_view_t* x, es_dtype_t dt, const void* xp, const es_view_t* y, void* yp,
                              es_stream_t stream) {
  const int waves = x->n * x->c;
  View xv = mkview(x);
  xv.rows = rows_of(x, y);
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((waves + 3) / 4), dim3(256), 0, (hipStream_t)stream, xv, xp,
                     dt == ES_BF16, mkview(y), yp);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_avgpool_bwd(const es_view_t* dy, const void* dyp, const es_view_t* dx, es_dtype_t dxdt,
                              void* dxp, float beta, es_stream_t stream) {
  const int64_t total = (int64_t)dx->n * dx->c * dx->h * dx->w;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, mkview(dy),
                     (const float*)dyp, mkview(dx), dxp, dxdt == ES_BF16, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_gather_rows(const float* src, int64_t src_ld, const int32_t* idx, int rows, int cols, float* dst,
                              int64_t dst_ld, es_stream_t stream) {
  const int64_t total = (int64_t)rows * cols;
  if (total == 0) return ES_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, src, src_ld,
                     idx, (const int32_t*)nullptr, rows, cols, dst, dst_ld, (const int32_t*)nullptr);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_gather_rows_at(const float* src, int64_t src_ld, const int32_t* perm, const int32_t* start,
                                 int rows, int cols, float* dst, int64_t dst_ld, const int32_t* live,
                                 es_stream_t stream) {
  const int64_t total = (int64_t)rows * cols;
  if (total == 0) return ES_OK;
  ES_CHECK_ARG(perm && start, "gather_rows_at: perm / start");
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, src, src_ld,
                     perm, start, rows, cols, dst, dst_ld, live);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_sn_power_iter(const float* w, int h, int wd, float* u, float* v, float* sigma, int update,
                                const int32_t* active, es_stream_t stream) {
  // the caller's buffer: sigma[0], scratch [h + wd], then the snapshot of the u, v used [h + wd]
  // (1 + 2 (h + wd) floats)
  hipStream_t st = (hipStream_t)stream;
  if ((int64_t)h * wd >= 16384) {   // large weights (discriminator fc1): the two mat-vecs over the chip
    float* wv = sigma + 1;
    float* vt = sigma + 1 + h;
    if (update) hipLaunchKernelGGL(sn_wtu_kernel, dim3((wd + 63) / 64), dim3(256), 0, st, w, h, wd, u, vt);
    hipLaunchKernelGGL(sn_wv_kernel, dim3((h + 3) / 4), dim3(256), 0, st, w, h, wd, update ? (const float*)vt : v,
                       update, v, wv, (const float*)v, active);
    hipLaunchKernelGGL(sn_final_kernel, dim3(1), dim3(256), 0, st, h, wd, (const float*)wv, u, (const float*)v, update,
                       sigma, sigma + 1 + h + wd, active);
  } else {
    hipLaunchKernelGGL(sn_power_kernel, dim3(1), dim3(1024), 0, st, w, h, wd, u, v, sigma, update, sigma + 1, active);
  }
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_sn_power_iter_batch(int n, const float* const* w, const int* h, const int* wd, float* const* u,
                                      float* const* v, float* const* buf, int update, const int32_t* active,
                                      es_stream_t stream) {
  ES_CHECK_ARG(n >= 1 && n <= ES_SN_BATCH_MAX, "sn_power_iter_batch: 1 <= n <= ES_SN_BATCH_MAX");
  SnJobs j{};
  for (int i = 0; i < n; ++i) {
    ES_CHECK_ARG((int64_t)h[i] * wd[i] < 16384, "sn_power_iter_batch: layer too large for one block");
    j.w[i] = w[i]; j.u[i] = u[i]; j.v[i] = v[i]; j.buf[i] = buf[i]; j.h[i] = h[i]; j.wd[i] = wd[i];
  }
  hipLaunchKernelGGL(sn_power_batch_kernel, dim3(n), dim3(1024), 0, (hipStream_t)stream, j, update, active);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_sn_bwd_batch(int n, const float* const* w, const float* const* g, const int* h, const int* wd,
                               const float* const* u, const float* const* v, const float* const* sigma,
                               float* const* dw, float beta, es_stream_t stream) {
  ES_CHECK_ARG(n >= 1 && n <= ES_SN_BATCH_MAX, "sn_bwd_batch: 1 <= n <= ES_SN_BATCH_MAX");
  SnBwdJobs j{};
  for (int i = 0; i < n; ++i) {
    const int64_t e = (int64_t)h[i] * wd[i];
    ES_CHECK_ARG(!(e >= 16384 && h[i] + wd[i] >= 256), "sn_bwd_batch: layer too large for one block");
    j.w[i] = w[i]; j.g[i] = g[i]; j.u[i] = u[i]; j.v[i] = v[i]; j.sigma[i] = sigma[i]; j.dw[i] = dw[i];
    j.h[i] = h[i]; j.wd[i] = wd[i];
  }
  hipLaunchKernelGGL(sn_bwd_batch_kernel, dim3(n), dim3(1024), 0, (hipStream_t)stream, j, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_sn_bwd(const float* w, const float* g, int h, int wd, const float* u, const float* v,
                         const float* sigma, float* dw_orig, float beta, es_stream_t stream) {
  const int64_t n = (int64_t)h * wd;
  if (n >= 16384 && h + wd >= 256) {
    // partials go to the power iteration's scratch (sigma[1 .. h+wd]), free outside es_sn_power_iter
    float* part = const_cast<float*>(sigma) + 1;
    const int nb = (int)std::min<int64_t>(256, (n + 1023) / 1024);
    hipLaunchKernelGGL(sn_dot_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, g, w, (int)n, part);
    hipLaunchKernelGGL(sn_bwd_apply_kernel, dim3((unsigned)std::min<int64_t>(1024, (n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, g, h, wd, u, v, sigma, (const float*)part, nb, dw_orig, beta);
  } else {
    hipLaunchKernelGGL(sn_bwd_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, w, g, h, wd, u, v, sigma,
                       dw_orig, beta);
  }
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                       float beta2, float eps, int step, float grad_scale, es_stream_t stream) {
  ES_CHECK_ARG(step >= 1, "adam: step must be >= 1");
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  if (n == 0) return ES_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                     beta2, eps, step_size, bc2_sqrt, grad_scale);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                           float beta2, float eps, const int32_t* step_ptr, float grad_scale, const int32_t* active,
                           es_stream_t stream) {
  ES_CHECK_ARG(step_ptr != nullptr, "adam_dev: step_ptr is NULL");
  if (n == 0) return ES_OK;
  hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                     beta2, eps, step_ptr, grad_scale, active);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_ema_update(float* shadow, const float* p, int64_t n, float decay, float one_minus_decay,
                             es_stream_t stream) {
  ES_CHECK_ARG(n >= 0, "ema_update: n < 0");
  if (n == 0) return ES_OK;
  hipLaunchKernelGGL(ema_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, shadow, p, n, decay,
                     one_minus_decay);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_randn_dev(float* out, int64_t n, uint64_t seed, uint32_t stream_id, const int32_t* step_ptr,
                            int32_t step_mul, int64_t offset, es_stream_t stream) {
  if (n == 0) return ES_OK;
  ES_CHECK_ARG(offset >= 0 && offset % 2 == 0, "randn: offset %lld must be even and >= 0", (long long)offset);
  hipLaunchKernelGGL(randn_kernel, dim3(grid_for((n + 1) / 2)), dim3(256), 0, (hipStream_t)stream, out, n, seed,
                     stream_id, step_ptr, step_mul, offset / 2, (const int32_t*)nullptr, (int64_t)0);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
extern "C" int es_randn_dev_at(float* out, int64_t n, uint64_t seed, uint32_t stream_id, const int32_t* step_ptr,
                               int32_t step_mul, int64_t offset, const int32_t* off_ptr, int64_t off_mul,
                               es_stream_t stream) {
  if (n == 0) return ES_OK;
  ES_CHECK_ARG(offset >= 0 && offset % 2 == 0 && off_mul % 2 == 0, "randn_dev_at: even offsets required");
  hipLaunchKernelGGL(randn_kernel, dim3(grid_for((n + 1) / 2)), dim3(256), 0, (hipStream_t)stream, out, n, seed,
                     stream_id, step_ptr, step_mul, offset / 2, off_ptr, off_mul / 2);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
extern "C" int es_randn(float* out, int64_t n, uint64_t seed, uint32_t stream_id, es_stream_t stream) {
  return es_randn_dev(out, n, seed, stream_id, nullptr, 0, 0, stream);
}

extern "C" int es_rand_exponential_dev(float* out, int64_t n, uint64_t seed, uint32_t stream_id,
                                       const int32_t* step_ptr, int32_t step_mul, int64_t offset,
                                       es_stream_t stream) {
  if (n == 0) return ES_OK;
  ES_CHECK_ARG(offset >= 0, "rand_exponential: offset must be >= 0");
  hipLaunchKernelGGL(rand_exp_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, out, n, seed,
                     stream_id, step_ptr, step_mul, offset);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
extern "C" int es_rand_exponential(float* out, int64_t n, uint64_t seed, uint32_t stream_id, es_stream_t stream) {
  return es_rand_exponential_dev(out, n, seed, stream_id, nullptr, 0, 0, stream);
}

extern "C" int es_counter_add(int32_t* counter, int32_t v, es_stream_t stream) {
  return es_counter_add_if(counter, v, nullptr, stream);
}
extern "C" int es_counter_add_if(int32_t* counter, int32_t v, const int32_t* flag, es_stream_t stream) {
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counter, v, flag);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
namespace {
constexpr int NBT_MAX = 64;
struct CounterJobs {
  int64_t* c[NBT_MAX];
  int64_t v[NBT_MAX];
};
__global__ void counters_add_i64_kernel(CounterJobs j, int n, const int32_t* flag) {
  if (flag && flag[0] == 0) return;
  const int i = threadIdx.x;
  if (i < n) j.c[i][0] += j.v[i];
}
}  // namespace
extern "C" int es_counters_add_i64_if(int64_t* const* counters, const int64_t* v, int n, const int32_t* flag,
                                      es_stream_t stream) {
  ES_CHECK_ARG(n >= 0 && (n == 0 || (counters && v)), "counters_add: bad arguments");
  for (int b = 0; b < n; b += NBT_MAX) {
    CounterJobs j{};
    const int m = n - b < NBT_MAX ? n - b : NBT_MAX;
    for (int i = 0; i < m; ++i) {
      ES_CHECK_ARG(counters[b + i] != nullptr, "counters_add: null counter %d", b + i);
      j.c[i] = counters[b + i];
      j.v[i] = v[b + i];
    }
    hipLaunchKernelGGL(counters_add_i64_kernel, dim3(1), dim3(NBT_MAX), 0, (hipStream_t)stream, j, m, flag);
    ES_CHECK_LAUNCH();
  }
  return ES_OK;
}
extern "C" int es_counter_add_i64_if(int64_t* counter, int64_t v, const int32_t* flag, es_stream_t stream) {
  hipLaunchKernelGGL(counter_add_i64_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counter, v, flag);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
extern "C" int es_expert_plan(const int32_t* counts, const int32_t* counts_all, int world, int rank, int E, int B,
                              int min_local, int32_t* rows, int32_t* active, int32_t* n0, float* w, float* gcnt,
                              float* lcnt, es_stream_t stream) {
  ES_CHECK_ARG(counts && rows && active && n0 && w && gcnt && lcnt && E >= 1 && E <= 1024 && B >= 1,
               "expert_plan: bad arguments");
  ES_CHECK_ARG(counts_all == nullptr || (world >= 1 && rank >= 0 && rank < world), "expert_plan: world / rank");
  hipLaunchKernelGGL(expert_plan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, counts, counts_all, world, rank,
                     E, B, min_local, rows, active, n0, w, gcnt, lcnt);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
extern "C" int es_div_by(float* x, int n, const float* d, es_stream_t stream) {
  ES_CHECK_ARG(x && d && n >= 0, "div_by: bad arguments");
  if (n == 0) return ES_OK;
  hipLaunchKernelGGL(div_by_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, n, d);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_dropout_mask(uint8_t* out, int64_t n, const es_dropout_t* d, es_stream_t stream) {
  if (n == 0) return ES_OK;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, out, n, *d);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

// ABI check: sizeof of the structs the bindings mirror (0 view, 1 dropout, 2 conv desc, 3 norm,
// 4 chain, 5 gen loss, 6 dfront2 params, 7 dmlp params); -1 for an unknown index
extern "C" int64_t es_struct_size(int which) {
  switch (which) {
    case 0: return sizeof(es_view_t);
    case 1: return sizeof(es_dropout_t);
    case 2: return sizeof(es_conv_desc_t);
    case 3: return sizeof(es_norm_t);
    case 4: return sizeof(es_chain_t);
    case 5: return sizeof(es_gen_loss_t);
    case 6: return sizeof(es_dfront2_params_t);
    case 7: return sizeof(es_dmlp_params_t);
    case 8: return sizeof(es_pack_job_t);
    default: return -1;
  }
}
