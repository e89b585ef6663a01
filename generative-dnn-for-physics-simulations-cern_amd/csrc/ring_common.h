// Device helpers shared by the LDS-DMA ring kernels (conv_mfma.hip) and the wave-specialised
// split-fp32 weight gradient (conv_wgrad_ws.hip): buffer resources / LDS-DMA, the raw barrier and
// counted waits, the XCD-aware workgroup remap.
#pragma once
#include "common.h"

namespace {

constexpr uint32_t OOB = 0x80000000u;   // buffer offset past every num_records (< 2^31 bytes)

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mkres(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
// 64 lanes x 16 bytes -> LDS at lds_wave_base + 16 * lane (M0-based, lane-linear)
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_wave_base, 16, (int)voff, 0, 0, 0);
}

// s_barrier without __syncthreads()'s workgroup fence: that fence makes the compiler drain every
// in-flight LDS-DMA (vmcnt(0)), which would serialise the ring.  The ring's own vmcnt wait before
// the barrier is what publishes a wave's pieces; the asm memory clobber keeps the compiler from
// moving LDS accesses across it.
__device__ __forceinline__ void ring_barrier() { asm volatile("s_barrier" ::: "memory"); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// bijective remap: consecutive ids land on one XCD (round-robin dispatch over 8 XCDs)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

}  // namespace
