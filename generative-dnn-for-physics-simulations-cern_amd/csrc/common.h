// Shared device helpers for the expertsim gfx950 kernels (CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/expertsim_hip.h"

typedef __bf16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

#define ES_WAVE 64

// ---------------------------------------------------------------- error reporting (host side)
void es_set_error(const char* fmt, ...);
#define ES_CHECK_ARG(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      es_set_error(__VA_ARGS__);           \
      return ES_ERR_ARG;                   \
    }                                      \
  } while (0)
#define ES_CHECK_LAUNCH()                                                     \
  do {                                                                        \
    hipError_t _e = hipGetLastError();                                        \
    if (_e != hipSuccess) {                                                   \
      es_set_error("%s: %s", __func__, hipGetErrorString(_e));                \
      return ES_ERR_HIP;                                                      \
    }                                                                         \
  } while (0)

// deterministic mode (es_set_deterministic; the fp32 parity mode turns it on): every float
// reduction in a fixed order, no float atomics (split-K partials + ordered reduces)
extern bool g_es_det;

// ---------------------------------------------------------------- scalar conversions
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float lrelu(float x, float slope) { return x > 0.f ? x : x * slope; }

// ---------------------------------------------------------------- wave / block reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the block; every thread gets the result.  `sh` needs blockDim/64 floats.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}

// ---------------------------------------------------------------- Philox4x32-10
// Same generator as expertsim/utils/philox.py (host restatement); bit-exact integer output.
struct u32x4 { uint32_t x, y, z, w; };
__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return {c0, c1, c2, c3};
}

// Random word for logical element `i` of dropout stream `stream` (see philox.py).
__device__ __forceinline__ uint32_t philox_word(uint64_t seed, uint32_t stream, uint64_t i) {
  const uint64_t q = i >> 2;
  u32x4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), stream, 0u, (uint32_t)seed,
                          (uint32_t)(seed >> 32));
  const uint32_t s = (uint32_t)(i & 3);
  return s == 0 ? r.x : (s == 1 ? r.y : (s == 2 ? r.z : r.w));
}
// stream + step * step_mul when the step lives on the device (captured train steps), and the
// index offset of a data-parallel rank's first sample when that lives on the device too
__device__ __forceinline__ void resolve_stream(es_dropout_t& d) {
  if (d.enabled && d.step_ptr) d.stream += (uint32_t)(d.step_ptr[0] * d.step_mul);
  if (d.enabled && d.index_ptr) d.index_offset += (uint64_t)d.index_ptr[0] * (uint64_t)d.index_mul;
}

// ---------------------------------------------------------------- dynamic batch (es_view_t.rows)
// live images of an n-capacity batch whose count lives on the device (NULL: all n); wave-uniform
__device__ __forceinline__ int live_rows(const int32_t* rows, int n) {
  if (rows == nullptr) return n;
  const int v = __builtin_amdgcn_readfirstlane(rows[0]);
  return v < 0 ? 0 : (v < n ? v : n);
}
__device__ __forceinline__ bool dropout_keep(const es_dropout_t& d, uint64_t i) {
  return (philox_word(d.seed, d.stream, i + d.index_offset) >> 8) < d.threshold;
}

// ---------------------------------------------------------------- logical 4-D index helpers
__device__ __forceinline__ int64_t off4(const int64_t* s, int64_t n, int64_t c, int64_t h, int64_t w) {
  return n * s[0] + c * s[1] + h * s[2] + w * s[3];
}
