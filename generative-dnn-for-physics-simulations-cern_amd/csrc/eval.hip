// Evaluation kernels: the 5-channel photon sums behind the Wasserstein
// metrics of MoEWrapper.evaluate (moe.py:644-692).
//   get_channel_masks       train/utils.py:18-59   checkerboard (i%2, j%2) = (0,1)/(1,0) split
//                                                  into 4 quadrants + the complementary squares
//   sum_channels_parallel   train/utils.py:62-78   masked sums per image
//   np.expm1 of the log1p-domain images            moe.py:646, train/utils.py:198 (fused here)
//
// One wave per image, four images per 256-thread block; every lane walks the image with a
// 64-pixel stride (coalesced row-major loads), classifies each pixel into one of the five
// disjoint masks and accumulates in fp64 (the reference sums the generated side in float64).
// HBM-bound: H*W*sizeof(dtype) bytes read and 40 bytes written per image.
#include "common.h"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) channel_sums_kernel(const T* __restrict__ x, int n, int h, int w,
                                                           int64_t sn, int64_t sh, int64_t sw, int log_domain,
                                                           double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int img = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (img >= n) return;                       // whole wave exits together (no block barrier below)
  const T* p = x + (int64_t)img * sn;
  const int mid_r = h >> 1, mid_c = w >> 1;
  const int hw = h * w;
  // pixel index i = lane + 64k, tracked as (row, col) without a division per pixel
  int r = lane / w, c = lane - (lane / w) * w;
  const int dr = 64 / w, dc = 64 - (64 / w) * w;
  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = lane; i < hw; i += 64) {
    float v = to_f(p[r * sh + c * sw]);
    if (log_domain) v = expm1f(v);            // float32 expm1, as numpy on the float32 array
    int ch;
    if (((r + c) & 1) == 0) ch = 4;           // mask5 = 1 - checkerboard
    else ch = (r < mid_r ? 2 : 0) + (c < mid_c ? 0 : 1);   // 1:BL 2:BR 3:TL 4:TR (0-based 0..3)
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] += (ch == k) ? (double)v : 0.0;
    r += dr;
    c += dc;
    if (c >= w) { c -= w; ++r; }
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) acc[k] = wave_sum_d(acc[k]);
  if (lane < 5) {
    double v = acc[0];
#pragma unroll
    for (int k = 1; k < 5; ++k) v = (lane == k) ? acc[k] : v;
    out[(int64_t)img * 5 + lane] = v;
  }
}

}  // namespace

extern "C" int es_channel_sums(const es_view_t* x, es_dtype_t dt, const void* xp, int log_domain, double* out,
                               es_stream_t stream) {
  ES_CHECK_ARG(x && xp && out, "channel_sums: null argument");
  ES_CHECK_ARG(x->c == 1, "channel_sums: images must have one channel (got %d)", x->c);
  ES_CHECK_ARG(x->h > 0 && x->w > 0, "channel_sums: empty image %dx%d", x->h, x->w);
  ES_CHECK_ARG(x->n >= 0, "channel_sums: negative count");
  if (x->n == 0) return ES_OK;
  const dim3 grid((x->n + 3) / 4), block(256);
  if (dt == ES_BF16)
    hipLaunchKernelGGL(channel_sums_kernel<bf16>, grid, block, 0, (hipStream_t)stream, (const bf16*)xp, x->n,
                       x->h, x->w, x->s[0], x->s[2], x->s[3], log_domain, out);
  else
    hipLaunchKernelGGL(channel_sums_kernel<float>, grid, block, 0, (hipStream_t)stream, (const float*)xp, x->n,
                       x->h, x->w, x->s[0], x->s[2], x->s[3], log_domain, out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
