// Split-fp32 arithmetic on the bf16 MFMA (shared by the ring conv kernels, conv_mfma.hip, and the
// fused discriminator front, d_front2.hip).
#pragma once
#include "common.h"

// ---------------------------------------------------------------------------------------------
// Split-fp32 arithmetic (the fp32 mode's fast MFMA path, SPL kernels).  An fp32 value is the exact
// sum of three bf16 values: x0 = rne(x), x1 = rne(x - x0), x2 = x - x0 - x1 (x - x0 has <= 16
// significant bits and x - x0 - x1 <= 8, so every difference is exact and x2 is representable).
// A product a*b is then sum_{p+q<=2} a_p b_q (6 bf16 products, each exact in the fp32 MFMA
// accumulator); the dropped terms a1 b2 + a2 b1 + a2 b2 are below 2^-23 |a b| (|x1| <= 2^-8 |x|,
// |x2| <= 2^-16 |x|), i.e. the size of one fp32 rounding, and the sums run in fp32 as in the exact
// fp32 MFMA.  v_mfma_f32_16x16x32_bf16 does 8192 MACs in 16 cycles against 1024 in 32 for
// v_mfma_f32_16x16x4_f32: the six products cost 6/16 of the fp32 MFMA time.
// ---------------------------------------------------------------------------------------------
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float x, float y) {   // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){x, y}, bf16x2_t));
}
__device__ __forceinline__ float bf_lo(uint32_t p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float bf_hi(uint32_t p) { return __builtin_bit_cast(float, p & 0xffff0000u); }
// two values -> their three bf16 planes, packed per plane (first value in the low half)
// (plain v_sub_f32: hipcc otherwise pairs the subtractions into v_pk_add_f32, which costs more issue
// cycles than two scalar ops beside MFMAs, MI355X_MICROARCH.md constants table)
__device__ __forceinline__ float fsub(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void split_pair(float x, float y, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = cvt_pk_bf16(x, y);
  const float rx = fsub(x, bf_lo(h)), ry = fsub(y, bf_hi(h));
  m = cvt_pk_bf16(rx, ry);
  l = cvt_pk_bf16(fsub(rx, bf_lo(m)), fsub(ry, bf_hi(m)));
}
// 8 fp32 values (a lane's k-slice of a 16x16x32 fragment, two 16-byte LDS chunks) -> planes p[0..2]
__device__ __forceinline__ void split8(const f32x4& x, const f32x4& y, bf16x8 p[3]) {
  uint32_t h0, h1, h2, h3, m0, m1, m2, m3, l0, l1, l2, l3;
  split_pair(x[0], x[1], h0, m0, l0);
  split_pair(x[2], x[3], h1, m1, l1);
  split_pair(y[0], y[1], h2, m2, l2);
  split_pair(y[2], y[3], h3, m3, l3);
  p[0] = __builtin_bit_cast(bf16x8, (u32x4_t){h0, h1, h2, h3});
  p[1] = __builtin_bit_cast(bf16x8, (u32x4_t){m0, m1, m2, m3});
  p[2] = __builtin_bit_cast(bf16x8, (u32x4_t){l0, l1, l2, l3});
}
// acc + the K-step's sum of the six plane products, small terms first.  The bf16 MFMA's fp32
// accumulation rounds with a negative bias (measured, tools/split_bias.py: summed outputs drift by
// -5e-8 .. -1.2e-6 of sum|y| when every product accumulates into the running sum), so the step's
// products go into a fresh accumulator (its rounding is on the scale of one K-step's partial sum)
// and the running sum takes them with one round-to-nearest add per element.  (A plain C++ add: the
// compiler's MFMA-result hazard wait states do not cover inline asm that reads the MFMA's output.)
__device__ __forceinline__ f32x4 mfma_split6(const bf16x8 a[3], const bf16x8 b[3], f32x4 acc) {
  f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
  return acc + c;
}
