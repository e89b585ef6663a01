// 8-wave LDS-DMA ring kernels for the bf16 implicit-GEMM convolutions (the generator convs of
// neutron/generator.py:24,29,33 and proton/generator.py:27,33,38 and the aux-regressor convs:
// everything whose K-step is one filter tap over 64 contiguous channels).
//
// Same products as conv_igemm.hip (FWD: y = conv(x, W); DGRAD: dx with the integer upsample
// folded; WGRAD: dW), re-tiled for gfx950:
//   * 512 threads = 8 waves, one workgroup per CU (the 3-slot ring takes up to 144 KiB of the
//     160 KiB LDS), two waves per SIMD, each wave a 64x64 (64x32 / 32x64) tile of
//     v_mfma_f32_16x16x32_bf16;
//   * block tiles 256x128 (FWD/DGRAD) and 128x256 / 256x128 (WGRAD): 48 KiB of operands per
//     64-deep K-step for 4.2 MFLOP;
//   * operands go global -> LDS by DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave instruction,
//     no register round trip) into a 3-slot ring: at step t a wave waits only for ITS pieces of
//     slot t (s_waitcnt vmcnt(pieces per slot): slot t+1 stays in flight), one s_barrier, then it
//     issues slot t+2 into the slot everyone finished reading at t-1 and runs the MFMAs of t;
//   * IMAGE-MINOR ROW ORDER.  GEMM rows (FWD/DGRAD) and GEMM K (WGRAD) enumerate pixels as
//     (image group g of 64 images, pixel, image within the group): m = (g*PQ + pix)*64 + nl.
//     Each 8-row DMA piece (and each 64-deep WGRAD K-step) is then 8 (64) images at ONE pixel,
//     so the im2col gather address of a piece is a per-lane constant (image nl) plus a
//     WAVE-UNIFORM pixel/tap offset computed on the scalar unit: one VALU add per piece per
//     K-step instead of a per-lane coordinate decode (which made the first version VALU-issue
//     bound at ~4x the MFMA time).  Padding / out-of-image taps are uniform per piece and use an
//     out-of-range buffer offset, which the buffer unit returns as zeros; images beyond N fall
//     outside the buffer's num_records the same way;
//   * workgroup ids are remapped so that consecutive tiles (same 64 images, neighbouring pixels)
//     run on one XCD and share its L2.
//
// LDS images (per slot):
//   FWD/DGRAD  [rows][128 B] per operand, 16-byte chunk c of row r stored at chunk
//              c ^ ((r >> 1) & 7): the 16-row ds_read_b128 fragment reads are conflict-free.
//   WGRAD      [64 images][rows] per operand (rows contiguous in global memory: channels), read
//              with ds_read_b64_tr_b16; chunk c of k-row k stored at c ^ (2(k&3) | 8((k>>3)&1)).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "conv_common.h"
#include "ring_common.h"
#include "split_fp32.h"


namespace {

constexpr int RT = 512;   // threads per workgroup (8 waves)
constexpr int NSLOT = 3;  // ring depth
// split-fp32 SPB loop (8-wave FWD / DGRAD): column tiles of B planes read ahead of their MFMAs
constexpr int SPB_PFD = 2;
// SPB loop: column tile at which waves 4-7 issue their step's DMA (capped at RN - 1; waves 0-3 issue
// after column tile 0).  The two waves of a SIMD (w, w + 4) otherwise stall on their 7 LDS-DMA issues
// at the same point, leaving the SIMD's matrix pipe idle.  Measured (alternating A/B, B = 1024,
// ms/step): base 44.8-45.3; tile 2 45.34, 4 44.54, 5 44.60, 6 44.19 / 44.12, 7 44.05 / 44.50
// (conv_layers.5 FWD / DGRAD 3.15 / 3.05 -> 2.95 / 2.85 ms at 6).  Other placements (waves 0-3 later,
// the A(t+1) split of waves 4-7 moved, one fresh accumulator per two K-steps, the 4-wave SPB4 / SPA
// kernels, pre-split activation planes) measured slower or drifted and were removed in round 5
// (DESIGN.md §4 keeps the numbers).
constexpr int SPB_DMA_HI = 6;

// es_conv_set_ring(0) routes these shapes to the 4-wave kernels of conv_igemm.hip (tests)
bool g_ring_off = false;
// split-fp32 WGRAD with 128-row tiles: the wave-specialised kernel (1) or wgrad_coop_kernel (0);
// bitwise the same partials (es_conv_set_wgrad_ws, tests / A-B)
int g_wgrad_ws = 1;

// first argument type of a lambda's call operator (the fragment set of a ring's load lambda)
template <typename F>
struct lambda_arg : lambda_arg<decltype(&F::operator())> {};
template <typename C, typename R, typename A0, typename... As>
struct lambda_arg<R (C::*)(A0, As...) const> {
  typedef A0 type;
};


// Per-class sub-pixel values in registers: 4 x int16 packed in one 64-bit scalar, read with a
// shift.  Indexing the kernel-argument arrays with a runtime class makes hipcc reload them
// (s_load + lgkmcnt(0), which also drains the ds_reads) after every ring barrier, and a select
// chain over 4 copies becomes branches inside the loop.
struct ClsReg {
  uint64_t v;
  __device__ __forceinline__ void init(const int* src) {
    uint32_t lo = ((uint32_t)(uint16_t)src[0]) | ((uint32_t)(uint16_t)src[1] << 16);
    uint32_t hi = ((uint32_t)(uint16_t)src[2]) | ((uint32_t)(uint16_t)src[3] << 16);
    v = ((uint64_t)(uint32_t)uni((int)hi) << 32) | (uint32_t)uni((int)lo);
  }
  __device__ __forceinline__ int operator()(int c) const { return (int)(short)(uint16_t)(v >> (16 * c)); }
};

// byte offset of 16-byte chunk `chunk` of row `row` in a [rows][BK] bf16 slot image:
//   BK = 64 (128-byte rows): chunk ^ ((row >> 1) & 7)
//   BK = 32 (64-byte rows):  chunk ^ f(row / 4 mod 4), f = {0, 2, 3, 1}
// so that each of ds_read_b128's four 16-lane bank groups ({0-3, 12-15, 20-27}, {4-11, 16-19,
// 28-31}, and the same + 32; MI355X_MICROARCH.md §LDS) hits 16 distinct 16-byte bank slots when
// lane l reads row r0 + (l & 15), chunk l >> 4 (a plain ((row >> 2) & 3) leaves 2-way conflicts)
template <int BK = 64>
__device__ __forceinline__ int swz_x(int row) {
  return BK == 64 ? ((row >> 1) & 7) : ((0x78 >> (2 * ((row >> 2) & 3))) & 3);
}
template <int BK = 64>
__device__ __forceinline__ int swz(int row, int chunk) { return row * (BK * 2) + ((chunk ^ swz_x<BK>(row)) << 4); }

typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));

// 16-byte chunk swizzle of k-row k in a [64][BROWS] image: the 8 k-rows one half-wave reads with
// ds_read_b64_tr_b16 (k0 + {0..3, 8..11}) must hit 8 distinct 32-byte bank groups.
//   BROWS >= 128 (k-rows of >= 256 B, every k-row starts at bank 0): XOR 2(k&3) | 8((k>>3)&1)
//   BROWS == 64  (128-B k-rows, odd rows start at bank 32): XOR 2((k>>1)&1) | 4((k>>3)&1)
template <int BROWS>
__device__ __forceinline__ int swz_tr(int k) {
  if constexpr (BROWS >= 128) return ((k & 3) << 1) | (((k >> 3) & 1) << 3);
  else return (((k >> 1) & 1) << 1) | (((k >> 3) & 1) << 2);
}

// byte offset of (k-row k, row) in a [64][BROWS] bf16 image
template <int BROWS>
__device__ __forceinline__ int tr_off(int k, int row) {
  return k * (BROWS * 2) + ((((row >> 3) ^ swz_tr<BROWS>(k)) << 4) | ((row & 7) << 1));
}

// A/B fragment of v_mfma_f32_16x16x32_bf16 from a [k][rows] image: lane l gets row r0 + (l & 15),
// k = k0 + 8 (l >> 4) + 0..7, as two ds_read_b64_tr_b16.
template <int BROWS>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int k0, int r0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ka = k0 + 8 * g + q;
  const char* p0 = img + tr_off<BROWS>(ka, r0 + 4 * p);
  const char* p1 = img + tr_off<BROWS>(ka + 4, r0 + 4 * p);
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)p0);
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)p1);
  short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// The same fragment read as inline asm.  hipcc cannot tell which LDS-DMA a
// __builtin_amdgcn_ds_read_tr16_b64 may alias, so it drains every DMA in flight (vmcnt(0)) before
// the first one of each K-step, which serialises the ring; as asm the reads are invisible to its
// wait insertion and ring_loop orders them itself (lgkmcnt + an operand fence before the MFMAs).
typedef int int2v __attribute__((ext_vector_type(2)));
typedef int int4v __attribute__((ext_vector_type(4)));
typedef unsigned int v4u32_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ int2v ds_tr16(uint32_t addr) {
  int2v r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <int BROWS>
__device__ __forceinline__ bf16x8 tr_frag_asm(uint32_t img, int k0, int r0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ka = k0 + 8 * g + q;
  const int2v lo = ds_tr16(img + tr_off<BROWS>(ka, r0 + 4 * p));
  const int2v hi = ds_tr16(img + tr_off<BROWS>(ka + 4, r0 + 4 * p));
  const int4v v = {lo[0], lo[1], hi[0], hi[1]};
  return __builtin_bit_cast(bf16x8, v);
}
// make x depend on the preceding (volatile) wait: MFMAs reading x cannot move above it
__device__ __forceinline__ void fence_frag(bf16x8& x) {
  int4v v = __builtin_bit_cast(int4v, x);
  asm volatile("" : "+v"(v));
  x = __builtin_bit_cast(bf16x8, v);
}
template <int N>
__device__ __forceinline__ void wait_lgkmcnt() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// The ring main loop shared by the kernels.  Slot of K-step t = t % 3; two register fragment
// sets: the kk = 1 half of step t is read from LDS while the MFMAs of the kk = 0 half run, and the
// kk = 0 half of step t+1 while the kk = 1 MFMAs of step t run, so LDS latency hides behind MFMA
// work.  Per step, one barrier (after this wave's reads of slot t have completed and its DMA
// pieces of slot t+1 have landed): behind it every wave has finished slot t, which then takes the
// DMA of step t+3, and slot t+1 is complete.
//
// NLDS > 0: load() issues its LDS reads as inline asm (NLDS per call), invisible to hipcc's wait
// insertion; then before each mma the loop waits lgkmcnt(reads issued since) and fences the
// fragment (fence(f)) so the MFMAs cannot be scheduled above the wait.
// NS slots (3 or 4): NS - 1 steps in flight behind the one being computed.
template <int PW, int NLDS, int NS = 3, typename Issue, typename Load, typename Mma, typename Fence>
__device__ __forceinline__ void ring_loop(int nk, char* smem, int slot_bytes, Issue& issue, Load& load, Mma& mma,
                                          Fence& fence) {
  using Frag = typename std::remove_reference<typename lambda_arg<Load>::type>::type;
  constexpr int LATER = NLDS > 15 ? 15 : NLDS;   // lgkmcnt is a 4-bit count
  // issue() is called for steps 0, 1, 2, ... unconditionally; steps >= nk are all-OOB (zero-fill,
  // no memory traffic), so every iteration keeps exactly NS - 1 steps in flight and the loop body
  // is one basic block (the compiler's LDS waits stay counted instead of draining at branch joins)
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) issue(smem + i * slot_bytes);
  wait_vmcnt<(NS - 2) * PW>();
  ring_barrier();
  issue(smem + (NS - 1) * slot_bytes);
  Frag f0, f1;
  load(f0, smem, 0);
  int cur = 0;
  for (int t = 0; t < nk - 1; ++t) {
    load(f1, smem + cur * slot_bytes, 1);
    if constexpr (NLDS > 0) {                            // f0's reads done, f1's may be in flight
      wait_lgkmcnt<LATER>();
      fence(f0);
    }
    mma(f0);
    const int nxt = cur == NS - 1 ? 0 : cur + 1;
    wait_vmcnt<(NS - 2) * PW>();                         // step t+1 landed (this wave's pieces)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of slot t are done
    if constexpr (NLDS > 0) fence(f1);
    ring_barrier();
    load(f0, smem + nxt * slot_bytes, 0);
    issue(smem + cur * slot_bytes);                      // step t + NS
    mma(f1);
    cur = nxt;
  }
  load(f1, smem + cur * slot_bytes, 1);
  if constexpr (NLDS > 0) {
    wait_lgkmcnt<LATER>();
    fence(f0);
  }
  mma(f0);
  if constexpr (NLDS > 0) {
    wait_lgkmcnt<0>();
    fence(f1);
  }
  mma(f1);
  wait_vmcnt<0>();   // drain the zero-fill steps before the workgroup may exit
}

// Single fragment set variant (register-lean, for the 256 x 256 tiles): per step one barrier,
// then both fragment halves are read and multiplied in turn; the LDS latency is covered by the
// other wave of the SIMD.  Same slot / vmcnt discipline as ring_loop.
// HALVES = 1: one load + mma per step (the split-fp32 kernels: one fragment set covers the step).
template <int PW, int NS, int HALVES = 2, typename Issue, typename Load, typename Mma>
__device__ __forceinline__ void ring_loop_lean(int nk, char* smem, int slot_bytes, Issue& issue, Load& load,
                                               Mma& mma) {
  using Frag = typename std::remove_reference<typename lambda_arg<Load>::type>::type;
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) issue(smem + i * slot_bytes);
  int cur = 0, prv = NS - 1;
  for (int t = 0; t < nk; ++t) {
    wait_vmcnt<(NS - 2) * PW>();                         // step t landed (this wave's pieces)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of step t-1 are done
    ring_barrier();
    issue(smem + prv * slot_bytes);                      // step t + NS - 1 into step t-1's slot
    Frag f;
    load(f, smem + cur * slot_bytes, 0);
    mma(f);
    if constexpr (HALVES == 2) {
      load(f, smem + cur * slot_bytes, 1);
      mma(f);
    }
    prv = cur;
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  wait_vmcnt<0>();   // drain the zero-fill steps before the workgroup may exit
}

// split-fp32 helpers (split_pair / split8 / mfma_split6): split_fp32.h

// ---------------------------------------------------------------------------------------------
// FWD / DGRAD.  Rows m = (g*PQ + pix)*64 + nl (image n = 64 g + nl, pixel pix on the row grid),
// columns = channels of the packed weight, K-step = one tap x 64 channels.
//
// SP (sub-pixel decomposition of a conv over a x2 nearest-upsampled input, SubPixel in
// conv_common.h): FWD row tiles belong to one parity class of output pixels and run the class's
// dh x dw conv on the SOURCE grid with combined weights (packed by es_pack_conv_weight mode 2);
// DGRAD rows are source pixels and the K-steps run over (class, d, e, channels) against the
// mode-3 packing.  3x3 taps on the upsampled grid become 4 taps on the source grid: 2.25x fewer
// MACs and gathered bytes for the same result (up to the rounding of the combined weights).
// ---------------------------------------------------------------------------------------------
//
// BK = 64: K-steps of 64 channels (128-byte slot rows), 3 slots, 4 x 2 waves.
// BK = 32 (256 x 256 tiles): K-steps of 32 channels (64-byte rows), 4 slots (three steps in flight),
// 2 x 4 waves of 128 x 64; per step 32 KiB of operands for 4.2 MFLOP (the 256 x 128 BK = 64 tile
// moves 48 KiB for the same work), and an A row tile is gathered once for 256 output channels.
//
// SPL (T = float, BK = 64: 32 fp32 channels per K-step): split-fp32 arithmetic.  A lane reads the
// 16-byte chunks g16 and g16 + 4 of its fragment row (channels 4 g16 .. +3 and 16 + 4 g16 .. +3, the
// same k permutation for A and B), splits the 8 values into bf16 planes and issues the 6 plane
// products as v_mfma_f32_16x16x32_bf16; one fragment set per step (ring_loop_lean, HALVES = 1).
//
// SPL == 2 (SPB): the B operand (packed weights) arrives pre-split: es_pack_weight_planes stores each
// 32-element K block of the fp32 packing as three 64-byte bf16 planes (192 bytes, k in the same
// permutation as the A fragments), so only A is split in the kernel.  The slot holds B plane-major,
// [3][BN rows][64 B] (swizzled as the BK = 32 images), and the 8 waves are stacked along M (wave
// tile BM/8 x BN): every A element is split by one wave only.
//
template <int MODE, int BM, int BN, bool SP, int BK = 64, typename T = bf16, int SPL = 0>
__global__ void __launch_bounds__(RT) conv_ring_kernel(ConvArgs a) {
  static_assert(!SPL || (sizeof(T) == 4 && BK == 64), "split-fp32: fp32 operands, 128-byte slot rows");
  // (SPL 256 x 256: 2 x 4 waves of 128 x 64 and two 64 KiB slots; one step in flight covers a step
  // of 192 MFMAs per wave)
  constexpr bool SPB = SPL == 2;
  constexpr int NW = 8, NT = 64 * NW;                    // waves / threads per workgroup
  constexpr bool SPW = SPL == 1 && BN == 256;
  constexpr int WGM = SPB ? NW : ((BK == 32 || SPW) ? 2 : 4), WGN = NW / WGM;   // waves along M / N
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int RM = WM / 16, RN = WN / 16;
  constexpr int ROWB = BK * 2, PROWS = 1024 / ROWB;      // slot row bytes, rows per 1 KiB piece
  constexpr int EB = sizeof(T), BKC = ROWB / EB;         // operand bytes, channels per K-step (fp32: BK / 2)
  constexpr int EA = EB;                                 // bytes per value of the gathered (A) image
  constexpr int CPR = ROWB / 16;                         // 16-byte chunks per row
  constexpr int EBB = SPB ? 6 : EB;                      // bytes per B element in global memory
  constexpr int BPL = BN / 16;                           // SPB: 1 KiB pieces per B plane
  constexpr int BPIECES = SPB ? 3 * BPL : BN / PROWS;    // (SPB, BN = 64: 12 pieces + 4 zero-fill dummies)
  constexpr int APW = BM / PROWS / NW, BPW = (BPIECES + NW - 1) / NW;   // pieces per wave per slot
  constexpr int PW = APW + BPW;
  constexpr int ABYTES = BM * ROWB, BBYTES = SPB ? 3 * BN * 64 : BN * ROWB;
  constexpr int SLOT = ABYTES + BBYTES;
  // SPB ring depths: three full slots when they fit (NS = 3); else A gets three slots and B (the
  // weights, L2-resident) two: A stays two steps ahead, B one (SPLITD)
  constexpr bool SPLITD = SPB && 3 * SLOT > 144 * 1024;
  // (SPB 128 x 64: two slots, so that two workgroups share a CU and one's fill / epilogue overlaps
  // the other's MFMAs, as the short-K bf16 tiles do)
  constexpr int NS = SPW ? 2 : (SPB ? (BM == 128 && BN == 64 ? 2 : 3) : (BK == 32 ? 4 : NSLOT));
  constexpr int KH = BK == 64 ? 2 : 1;                   // MFMA K-halves per step
  constexpr int RMF = RM / (3 - KH);                     // A tiles per fragment set
  constexpr int SROWS = WM < 64 ? WM : 64;               // epilogue staging rows per pass
  constexpr int STAGE0 = NW * SROWS * (WN * 4 + 16);
  constexpr int TPITCH = BN * 2 + 16;                    // BK = 32 bf16 epilogue: whole-tile image
  constexpr int STAGE = BK == 32 && BM * TPITCH > STAGE0 ? BM * TPITCH : STAGE0;
  constexpr int RINGB = SPLITD ? 3 * ABYTES + 2 * BBYTES : NS * SLOT;
  constexpr int RING = RINGB > STAGE ? RINGB : STAGE;
  constexpr int JUNK = BPW * NW > BPIECES ? 1024 : 0;    // landing area of the dummy pieces
  // ONE __shared__ object (a second one beside the DMA ring makes hipcc wait vmcnt(0) before
  // every ds_read of the loop): the ring slots (also the epilogue staging), then the fused-stats
  // scratch [3][WGM][BN] floats, which no DMA targets
  __shared__ __attribute__((aligned(16))) char smem[RING + 3 * WGM * BN * 4 + JUNK];
  const es_conv_desc_t& d = a.d;
  const int NL = conv_live(a);   // live images (dynamic rows)
  const SubPixel& sp = a.sp;

  // Row order: image groups g of NG = a.ng images (8..64); inside a group, per class (SP FWD: 4
  // parity classes, else one) the class's pixels in tiles of NB = BM/NG pixels (each class
  // segment padded to whole tiles); a tile is NG images x NB pixels, a DMA piece (8 rows) is 8
  // images at one pixel.  Consecutive tiles (one XCD) stay on the same images, so their sources
  // share the L2; the host picks NG per operand (small groups keep a forward gather's source
  // footprint inside one XCD's L2).
  const int NG = a.ng, PPG = NG / PROWS;                 // pieces per pixel
  const int NB = BM / NG;
  int TT;                                                // row tiles per image group
  if constexpr (MODE == MODE_FWD && SP) TT = a.sp_merge ? sp.tile0[1] : (a.sp_tpc > 0 ? 4 * a.sp_tpc : sp.tile0[4]);
  else if constexpr (MODE == MODE_FWD) TT = (d.P * d.Q + NB - 1) / NB;
  else TT = ((a.fold ? d.H * d.W : d.Hu * d.Wu) + NB - 1) / NB;
  // tile order: the column tiles of one row tile are consecutive (they share the gathered rows).
  // Dynamic rows: the tiles of the live image groups (a prefix) are the ones remapped over the
  // XCDs, so that they spread over the whole chip; the others exit below.
  const int nt = gridDim.y, ntot = gridDim.x * nt, lin = blockIdx.x + blockIdx.y * gridDim.x;
  const int nlive = NL == d.N ? ntot : min(ntot, (NL + NG - 1) / NG * TT * nt);
  const int wg = lin < nlive ? xcd_remap(lin, nlive) : lin;
  const int tl = wg / nt, n0 = (wg % nt) * BN;
  int cls = 0, gh, gw, jt;
  if constexpr (MODE == MODE_FWD && SP) {
    if (a.sp_merge) {
      // merged classes: the rows are the (shared) source pixels of class 0's geometry, the
      // columns (class, channel); the class is resolved per wave in the epilogue
      jt = tl % TT;
    } else if (a.sp_tpc > 0) {
      // class-interleaved: tile r = 4 jt + class, so the 4 class tiles of the same source
      // pixels run back to back (one XCD, shared L2); classes with fewer tiles skip the tail
      const int r = tl % TT;
      cls = r & 3;
      jt = r >> 2;
      if (jt >= sp.tile0[cls + 1] - sp.tile0[cls]) {
        if (a.stats_part) {   // empty partial (count 0) for this tile
          float* pp = a.stats_part + (int64_t)tl * 3 * a.Ng;
          for (int c = threadIdx.x; c < BN; c += NT)
            if (n0 + c < a.Ng) pp[n0 + c] = 0.f;
        }
        return;
      }
    } else {
      const int r = tl % TT;
      cls = (r >= sp.tile0[1]) + (r >= sp.tile0[2]) + (r >= sp.tile0[3]);
      jt = r - sp.tile0[cls];
    }
    gh = sp.ph[cls];
    gw = sp.pw[cls];
  } else {
    if constexpr (MODE == MODE_FWD) {
      gh = d.P;
      gw = d.Q;
    } else {
      gh = a.fold ? d.H : d.Hu;
      gw = a.fold ? d.W : d.Wu;
    }
    jt = tl % TT;
  }
  const int PQ = gh * gw;
  const int gi = tl / TT;                                // image group: images NG gi ..
  const int pix0 = jt * NB;                              // first pixel of the tile
  if (gi * NG >= NL) {   // past the live images (dynamic rows): an empty partial, no work
    if (MODE == MODE_FWD && a.stats_part) {
      for (int c = threadIdx.x; c < BN; c += NT) {
        const int gc = n0 + c, cc = a.sp_merge ? gc / a.Ng : 0, ch = gc - cc * a.Ng;
        if (cc < 4 && ch < a.Ng) {
          float* pp = a.stats_part + (int64_t)(a.sp_merge ? tl * 4 + cc : tl) * 3 * a.Ng;
          pp[ch] = 0.f;
          pp[a.Ng + ch] = 0.f;
          pp[2 * a.Ng + ch] = 0.f;
        }
      }
    }
    return;
  }

  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int lrow = lane / CPR, pc = lane % CPR;

  const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * EA));
  // packed weights: row stride ldb (elements) and the class's block offset
  int ldb, bbase = 0, bbytes;
  if constexpr (SP && MODE == MODE_FWD) {
    ldb = sp.dh[cls] * sp.dw[cls] * d.C;
    bbase = sp.tap0[cls] * a.Ng * d.C;
    bbytes = sp.tap0[4] * a.Ng * d.C * EBB;
  } else if constexpr (SP) {
    ldb = sp.tap0[4] * d.K;
    bbytes = a.Ng * ldb * EBB;
  } else {
    ldb = (MODE == MODE_DGRAD && a.fold) ? d.R * d.S * d.K : a.Kd;
    bbytes = a.Ng * ldb * EBB;
  }
  const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)bbytes);
  const int as2b = (int)a.as[2] * EA, as3b = (int)a.as[3] * EA;

  // A pieces: per-lane constant (image, 16-byte chunk) + per-piece uniform pixel coordinates.
  constexpr int APC = APW, ALN = APW;
  uint32_t alane[ALN];
  int pc0[APC], pc1[APC];
  bool pval[APC];
#pragma unroll
  for (int j = 0; j < ALN; ++j) {
    const int pi = wid * APW + j;                 // piece of the tile: pixel pix0 + pi / PPG
    const int rr = pi * PROWS + lrow;             // row within the tile (swizzle)
    const int lc = pc ^ swz_x<BK>(rr);
    const int ppix = pi / PPG;
    const int pix = pix0 + ppix;
    pval[j] = pix < PQ;
    const int pp = pval[j] ? pix : 0;
    const int y = pp / gw, x = pp - y * gw;
    const int img = gi * NG + (pi - ppix * PPG) * PROWS + lrow;
    alane[j] = (uint32_t)(img * (int)a.as[0] * EB + lc * 16);   // images >= N: past num_records
    if constexpr (MODE == MODE_FWD && SP) {       // source row = u + oh + d
      pc0[j] = y + sp.oh[cls];
      pc1[j] = x + sp.ow[cls];
    } else if constexpr (MODE == MODE_FWD) {
      pc0[j] = y * d.stride - d.pad;
      pc1[j] = x * d.stride - d.pad;
    } else if constexpr (SP) {                    // source pixel (i, j)
      pc0[j] = y;
      pc1[j] = x;
    } else if (a.fold) {
      pc0[j] = y * d.up_h + d.pad;
      pc1[j] = x * d.up_w + d.pad;
    } else {
      pc0[j] = y + d.pad;
      pc1[j] = x + d.pad;
    }
  }
  constexpr int BLN = BPW;
  uint32_t blane[BLN];
#pragma unroll
  for (int j = 0; j < BLN; ++j) {
    if constexpr (SPB) {   // piece q: plane q / BPL, rows 16 (q % BPL) + lane / 4, 16-byte chunk lane % 4
      const int q = wid * BPW + j;
      const int rr = (q % BPL) * 16 + (lane >> 2);
      blane[j] = q < BPIECES ? (uint32_t)((bbase + (n0 + rr) * ldb) * EBB + (q / BPL) * 64 +
                                          (((lane & 3) ^ swz_x<32>(rr)) * 16))
                             : OOB;
    } else {
      const int rr = (wid * BPW + j) * PROWS + lrow;
      // rows past Ng read garbage columns that the epilogue drops (or zeros past num_records)
      blane[j] = (uint32_t)((bbase + (n0 + rr) * ldb) * EB + ((pc ^ swz_x<BK>(rr)) * 16));
    }
  }

  // K-step cursor (uniform, advanced once per issued slot).
  //   FWD      kk = ((r*S + s)*C + ch)                      (SP: taps d < dh, e < dw of the class)
  //   DGRAD    kk = (((ua*up_w + ub)*R + r)*S + s)*K + ch  with weight column kb = kk mod R*S*K
  //   DGRAD SP kk = ((class, d, e), ch)                    with column (tap0[class] + d*dw + e)*K + ch
  int cr = 0, cs = 0, cch = 0, cua = 0, cub = 0, ckb = 0, ccls = 0, cstep = 0;
  const int nch = MODE == MODE_FWD ? d.C : d.K;
  const int upw = d.up_w > 0 ? d.up_w : 1;
  int nk;
  if constexpr (SP && MODE == MODE_FWD) nk = ldb / BKC;
  else if constexpr (SP) nk = ldb / BKC;
  else nk = a.Kd / BKC;
  ClsReg Roh, Row, Rph, Rpw, Rp0, Rq0, Rtap0, Rdh, Rdw;
  if constexpr (SP && MODE == MODE_DGRAD) {
    Roh.init(sp.oh); Row.init(sp.ow); Rph.init(sp.ph); Rpw.init(sp.pw); Rp0.init(sp.p0); Rq0.init(sp.q0);
    Rtap0.init(sp.tap0); Rdh.init(sp.dh); Rdw.init(sp.dw);
  }
  int kh = SP ? uni(sp.dh[cls]) : d.R, kw = SP ? uni(sp.dw[cls]) : d.S;   // taps of the cursor's class
  // Per-tap cache: the pieces' offsets only change when the cursor enters a new tap (every
  // nch / BK steps); inside a tap a step adds BK channels.  Recomputing them every step cost
  // ~100 scalar instructions per K-step, which made the loop issue-bound (the CU's scalar unit
  // is shared by its 8 waves).
  uint32_t ua_t[APC], ub_t = 0;
#pragma unroll
  for (int j = 0; j < APC; ++j) ua_t[j] = OOB;
  auto issue = [&](char* slot) {
    if (cch == 0) {   // first step of a tap (wave-uniform branch, scalar work only)
      const bool live = cstep < nk;
#pragma unroll
      for (int j = 0; j < APC; ++j) {
        uint32_t u;
        if constexpr (MODE == MODE_FWD && SP) {
          const int hs = pc0[j] + cr, ws = pc1[j] + cs;
          const bool ok = live && pval[j] && (unsigned)hs < (unsigned)d.H && (unsigned)ws < (unsigned)d.W;
          u = ok ? (uint32_t)(hs * as2b + ws * as3b) : OOB;
        } else if constexpr (MODE == MODE_FWD) {
          const int hu = pc0[j] + cr, wu = pc1[j] + cs;
          const bool ok = live && pval[j] && (unsigned)hu < (unsigned)d.Hu && (unsigned)wu < (unsigned)d.Wu;
          // integer nearest upsample folded into the gather (factor 1 without upsample)
          const int sh = fdiv(hu, a.fUh), sw = fdiv(wu, a.fUw);
          u = ok ? (uint32_t)(sh * as2b + sw * as3b) : OOB;
        } else if constexpr (SP) {
          // output pixel (p0 + 2u, q0 + 2v) of class ccls feeds source pixel u + oh + d
          const int uu = pc0[j] - cr - Roh(ccls), vv = pc1[j] - cs - Row(ccls);
          const bool ok = live && pval[j] && (unsigned)uu < (unsigned)Rph(ccls) &&
                          (unsigned)vv < (unsigned)Rpw(ccls);
          u = ok ? (uint32_t)((Rp0(ccls) + 2 * uu) * as2b + (Rq0(ccls) + 2 * vv) * as3b) : OOB;
        } else {
          const int ph = pc0[j] + cua - cr, pw = pc1[j] + cub - cs;
          const int sh = d.stride == 2 ? 1 : 0;
          const bool ok = live && pval[j] && ph >= 0 && pw >= 0 && !(((ph | pw) & sh)) &&
                          (ph >> sh) < d.P && (pw >> sh) < d.Q;
          u = ok ? (uint32_t)((ph >> sh) * as2b + (pw >> sh) * as3b) : OOB;
        }
        ua_t[j] = u;
      }
      int kb;
      if constexpr (MODE == MODE_FWD) kb = (cr * kw + cs) * d.C;
      else if constexpr (SP) kb = (Rtap0(ccls) + cr * kw + cs) * d.K;
      else kb = ckb;
      ub_t = live ? (uint32_t)(kb * EBB) : OOB;
    }
    // (OOB + a channel offset stays past every num_records: offsets are < 1 GiB)
    const uint32_t co = (uint32_t)(cch * EA), cob = (uint32_t)(cch * EBB);
#pragma unroll
    for (int j = 0; j < APW; ++j) bdma16(ares, alane[j] + (ua_t[j] + co), slot + (wid * APW + j) * 1024);
    if constexpr (!SPB) {   // (SPB: B has its own ring and issue_b)
#pragma unroll
      for (int j = 0; j < BPW; ++j) {
        const int q = wid * BPW + j;
        char* dst = (!JUNK || q < BPIECES) ? slot + ABYTES + q * 1024 : smem + RING + 3 * WGM * BN * 4;
        bdma16(bres, blane[j] + (ub_t + cob), dst);
      }
    }
    ++cstep;
    cch += BKC;
    if (cch == nch) {   // tap done: advance the tap cursor (wave-uniform branch)
      cch = 0;
      ckb += nch;
      ++cs;
      const bool w2 = cs == kw;
      cs = w2 ? 0 : cs;
      cr += w2;
      const bool w3 = cr == kh;
      cr = w3 ? 0 : cr;
      ckb = w3 ? 0 : ckb;
      cub += w3;
      const bool w4 = cub == upw;
      cub = w4 ? 0 : cub;
      cua += w4;
      if constexpr (SP && MODE == MODE_DGRAD) {
        ccls += w3;
        const int cn = ccls < 4 ? ccls : 3;
        kh = Rdh(cn);
        kw = Rdw(cn);
      }
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment set kk: BK = 64 -> K half kk (all RM x RN tiles); BK = 32 -> the step's 32 channels
  // for A tiles kk*RM/2 .. (the wave's row half kk) and all RN B tiles
  const int r16 = lane & 15, g16 = lane >> 4;
  // (fp32: a lane's 16-byte chunk is 4 channels, fed to 4 v_mfma_f32_16x16x4_f32 with k = 4 g16 + t:
  // A and B use the same permutation of k, so each MFMA stays an exact fp32 FMA chain)
  typedef typename std::conditional<EB == 2, bf16x8, f32x4>::type FragT;
  struct Frag {
    FragT a[RMF], b[RN];
    int h;
  };
  auto load = [&](Frag& f, const char* slot, int kk) {
    const int seg = KH == 2 ? kk * 4 + g16 : g16;
    const int i0 = KH == 2 ? 0 : kk * RMF;
    f.h = kk;
#pragma unroll
    for (int i = 0; i < RMF; ++i) f.a[i] = *(const FragT*)(slot + swz<BK>(wm0 + (i0 + i) * 16 + r16, seg));
#pragma unroll
    for (int j = 0; j < RN; ++j) f.b[j] = *(const FragT*)(slot + ABYTES + swz<BK>(wn0 + j * 16 + r16, seg));
  };
  auto mma = [&](const Frag& f) {
    const int i0 = KH == 2 ? 0 : f.h * RMF;
#pragma unroll
    for (int i = 0; i < RMF; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        if constexpr (EB == 2) {
          acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[j], acc[i0 + i][j], 0, 0, 0);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[i][t], f.b[j][t], acc[i0 + i][j], 0, 0, 0);
        }
      }
  };
  if constexpr (SPB) {
    // Software-pipelined split-fp32 loop.  A (activations, fp32) and B (pre-split weight planes) have
    // their own rings: A in NSA slots, B in NSB.  Step t's MFMAs use A planes split during step t-1
    // (registers) and B(t) read from LDS per column tile; under them the wave reads A(t+1) and splits
    // it, and issues the DMA of B(t+NSB-1) / A(t+NSA).  Slot reuse: A(s) is read during step s-1 and
    // B(s) during step s, so behind the barrier of step t the slots of A(t) and B(t-1) are free.
    // Issue order A(0), B(0), A(1), [B(1), A(2)] ..., then per step B(t+NSB-1), A(t+NSA): at the top
    // of step t everything but the last (NSA-2) A and (NSB-2) B groups has landed, i.e. B(t), A(t+1).
    constexpr int NSA = SPLITD ? 3 : NS, NSB = SPLITD ? 2 : NS;
    constexpr int PROWAIT = (NSA - 1) * APW + (NSB - 1) * BPW, LOOPWAIT = (NSA - 2) * APW + (NSB - 2) * BPW;
    char* const aring = smem;
    char* const bring = smem + NSA * ABYTES;
    // B step s: the packed weight columns are K-linear, so its offset is (s mod period) * BKC elements
    // (DGRAD with a folded upsample repeats the R*S*K columns per upsample phase)
    const int bper = (MODE == MODE_DGRAD && !SP) ? (d.R * d.S * d.K) / BKC : nk;
    int bs = 0, bsm = 0;
    auto issue_b = [&](char* bslot) {
      const uint32_t ub = bs < nk ? (uint32_t)(bsm * BKC * EBB) : OOB;
#pragma unroll
      for (int j = 0; j < BPW; ++j) {
        const int q = wid * BPW + j;
        char* dst = (!JUNK || q < BPIECES) ? bslot + q * 1024 : smem + RING + 3 * WGM * BN * 4;
        bdma16(bres, blane[j] + ub, dst);
      }
      ++bs;
      bsm = bsm + 1 == bper ? 0 : bsm + 1;
    };
    auto rd_a = [&](f32x4 (&r)[RM][2], const char* aslot) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) r[i][h] = *(const f32x4*)(aslot + swz<BK>(wm0 + i * 16 + r16, g16 + 4 * h));
    };
    auto rd_b = [&](bf16x8 (&bp)[3], const char* bimg, int j) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        bp[pl] = *(const bf16x8*)(bimg + pl * (BN * 64) + swz<32>(wn0 + j * 16 + r16, g16));
    };
    if (a.prio && wid >= 4) __builtin_amdgcn_s_setprio(1);
    issue(aring);
#pragma unroll
    for (int st = 0; st < NSB - 1; ++st) {
      issue_b(bring + st * BBYTES);
      issue(aring + (st + 1) * ABYTES);
    }
#pragma unroll
    for (int st = NSB - 1; st < NSA - 1; ++st) issue(aring + (st + 1) * ABYTES);
    wait_vmcnt<PROWAIT>();
    ring_barrier();
    bf16x8 apc[RM][3];
    {
      f32x4 r[RM][2];
      rd_a(r, aring);
#pragma unroll
      for (int i = 0; i < RM; ++i) split8(r[i][0], r[i][1], apc[i]);
    }
    int sa1 = 1 % NSA, sb = 0, ia = 0, ib = NSB - 1;   // slots: A(t+1), B(t), A(t+NSA), B(t+NSB-1)
    constexpr int JS = RN > 2 ? RN / 2 : RN - 1;       // column tile after which A(t+1) is split
    constexpr int JDMA = SPB_DMA_HI < RN ? SPB_DMA_HI : RN - 1;
    for (int t = 0; t < nk; ++t) {
      wait_vmcnt<LOOPWAIT>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of the last step are done
      ring_barrier();
      const char* bimg = bring + sb * BBYTES;
      // B planes PFD column tiles ahead (LDS latency under load exceeds one tile's 12 MFMAs)
      constexpr int PFD = SPB_PFD;
      bf16x8 bq[PFD + 1][3];
#pragma unroll
      for (int j = 0; j < PFD && j < RN; ++j) rd_b(bq[j], bimg, j);
      f32x4 ra[RM][2];
      rd_a(ra, aring + sa1 * ABYTES);
      bf16x8 apn[RM][3];
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        if (j + PFD < RN) rd_b(bq[(j + PFD) % (PFD + 1)], bimg, j + PFD);
#pragma unroll
        for (int i = 0; i < RM; ++i) acc[i][j] = mfma_split6(apc[i], bq[j % (PFD + 1)], acc[i][j]);
        // the step's DMA, once its first MFMAs are queued (STAGGER: the two waves of a SIMD, w and
        // w + 4, at different column tiles, so one issues MFMAs while the other stalls on the issue)
        if (j == (wid >= 4 ? JDMA : 0)) {
          issue_b(bring + ib * BBYTES);
          issue(aring + ia * ABYTES);
        }
        if (j == JS) {
#pragma unroll
          for (int i = 0; i < RM; ++i) split8(ra[i][0], ra[i][1], apn[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) apc[i][pl] = apn[i][pl];
      sa1 = sa1 + 1 == NSA ? 0 : sa1 + 1;
      ia = ia + 1 == NSA ? 0 : ia + 1;
      sb = sb + 1 == NSB ? 0 : sb + 1;
      ib = ib + 1 == NSB ? 0 : ib + 1;
    }
    wait_vmcnt<0>();   // drain the zero-fill steps before the workgroup may exit
  } else if constexpr (SPL) {
    // The step's B tiles are read up front; the A row tiles are read inside the MFMA sequence, one
    // tile ahead (registers: the 256 x 256 tile holds 128 accumulators).  B tile j is split just
    // before its first MFMAs (row tile 0), so the step opens with one A and one B split.
    struct FragS {
      const char* slot;
    };
    auto rd_a = [&](f32x4 (&r)[2], const char* slot, int i) {
#pragma unroll
      for (int h = 0; h < 2; ++h) r[h] = *(const f32x4*)(slot + swz<BK>(wm0 + i * 16 + r16, g16 + 4 * h));
    };
    auto rd_b = [&](f32x4 (&r)[2], const char* slot, int j) {
#pragma unroll
      for (int h = 0; h < 2; ++h) r[h] = *(const f32x4*)(slot + ABYTES + swz<BK>(wn0 + j * 16 + r16, g16 + 4 * h));
    };
    auto load_s = [&](FragS& f, const char* slot, int) { f.slot = slot; };
    auto mma_s = [&](const FragS& f) {
      bf16x8 bp[RN][3], ap[3];
      f32x4 ra[2][2], rb[2][2];
      rd_a(ra[0], f.slot, 0);
      rd_b(rb[0], f.slot, 0);
      if constexpr (RN > 1) rd_b(rb[1], f.slot, 1);
      if constexpr (RM > 1) rd_a(ra[1], f.slot, 1);
      split8(ra[0][0], ra[0][1], ap);
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        split8(rb[j & 1][0], rb[j & 1][1], bp[j]);
        if (j + 2 < RN) rd_b(rb[j & 1], f.slot, j + 2);
        acc[0][j] = mfma_split6(ap, bp[j], acc[0][j]);
      }
#pragma unroll
      for (int i = 1; i < RM; ++i) {
        split8(ra[i & 1][0], ra[i & 1][1], ap);
        if (i + 1 < RM) rd_a(ra[(i + 1) & 1], f.slot, i + 1);
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = mfma_split6(ap, bp[j], acc[i][j]);
      }
    };
    if (a.prio && wid >= 4) __builtin_amdgcn_s_setprio(1);   // (wid is wave-uniform: readfirstlane)
    ring_loop_lean<PW, NS, 1>(nk, smem, SLOT, issue, load_s, mma_s);
  } else {
    auto nofence = [](Frag&) {};
    ring_loop<PW, 0, NS>(nk, smem, SLOT, issue, load, mma, nofence);
  }

  // epilogue.  Wave row r (0..WM-1) = tile row t = wm0 + r: pixel pix0 + t / NG, image
  // NG gi + t % NG.
  const int col16 = lane & 15, rq = (lane >> 4) * 4;
  // (no integer divisions per row: NG is a power of two and gw is divided by magic numbers; the
  // generic divides cost ~100 VALU per stored row, a third of the whole epilogue)
  const int lgNG = uni(31 - __builtin_clz(NG));
  FastDiv fgw;
  {
    uint32_t l = 0;
    while ((1u << l) < (uint32_t)gw) ++l;
    fgw.l = uni((int)l);
    fgw.m = (uint32_t)uni((int)(uint32_t)(((1ull << 32) * ((1ull << l) - (uint32_t)gw)) / (uint32_t)gw + 1));
  }
  auto row_pix = [&](int r) { return pix0 + ((wm0 + r) >> lgNG); };
  auto row_img = [&](int r) { return gi * NG + ((wm0 + r) & (NG - 1)); };
  // the wave's output columns: class ecls (merged sub-pixel FWD: column block / Ng), first
  // output channel kc0 (a wave's WN columns never straddle a class: Ng % 64 == 0)
  int ecls = cls, kc0 = n0 + wn0;
  if constexpr (SP && MODE == MODE_FWD) {
    if (a.sp_merge) {
      ecls = kc0 / a.Ng;
      kc0 -= ecls * a.Ng;
    }
  }
  auto row_off = [&](int r) -> int64_t {   // element offset of the wave row's output pixel
    const int pix = row_pix(r);
    int y = fdiv(pix, fgw), x = pix - y * gw;
    if constexpr (SP && MODE == MODE_FWD) {
      y = sp.p0[ecls] + 2 * y;
      x = sp.q0[ecls] + 2 * x;
    }
    return (int64_t)row_img(r) * a.os[0] + (int64_t)y * a.os[2] + (int64_t)x * a.os[3];
  };
  const int NLP = conv_live_px(a);   // pixel rows (rows_px > 0): image i pixel p live when i*PQ + p < NLP
  auto row_ok = [&](int r) { return row_pix(r) < PQ && row_img(r) < NL && row_img(r) * PQ + row_pix(r) < NLP; };
  // final values (bias added, rounded to the output dtype) back into acc
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int ng = kc0 + j * 16 + col16;
    float bv = 0.f;
    if constexpr (MODE == MODE_FWD) bv = (a.bias && ng < a.Ng) ? a.bias[ng] : 0.f;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float v = acc[i][j][jj] + bv;
        acc[i][j][jj] = a.out_bf16 ? (float)(bf16)v : v;
      }
  }
  if (BK == 32 || a.vec_out) {   // (the host runs BK = 32 only with vec_out)
    // BatchNorm statistics of the stored values (conv -> BatchNorm fusion): per column, count /
    // mean / M2 over the wave's valid rows (lanes own 16 rows, Chan-merged across the 4 row
    // groups by shuffles), then across the 4 row waves in LDS -> one [3][Ng] partial per row tile
    float* part = MODE == MODE_FWD ? a.stats_part : nullptr;   // (FWD only: compiled out of DGRAD)
    float (*st_n)[BN] = (float (*)[BN])(smem + RING);
    float (*st_m)[BN] = st_n + WGM;
    float (*st_q)[BN] = st_n + 2 * WGM;
    if (part) {
      const int wmi = wid / WGN;
      bool okr[RM][4];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) okr[i][jj] = row_ok(i * 16 + rq + jj);
      bool allok = true;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) allok = allok && okr[i][jj];
      const bool full = __all(allok);   // wave-uniform: no row of the wave is padding
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        float n_, m_, q;
        if (BK == 32 && full) {
          // 256 x 256 tiles: per column sum and sum of squares of the lane's 32 values (2 VALU per
          // value; the two-pass Chan form cost ~85 us of conv_layers.5's B = 1024 FWD epilogue),
          // summed over the 4 row groups, then (count, mean, M2) of the wave's 128 rows
          float s = 0.f, s2 = 0.f;
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const float v = acc[i][j][jj];
              s += v;
              s2 = fmaf(v, v, s2);
            }
#pragma unroll
          for (int o = 16; o <= 32; o <<= 1) {
            s += __shfl_xor(s, o, 64);
            s2 += __shfl_xor(s2, o, 64);
          }
          n_ = (float)(RM * 16);
          m_ = s * (1.f / (RM * 16));
          q = fmaxf(s2 - s * m_, 0.f);
        } else {
        float cnt = 0.f, s = 0.f;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            if (okr[i][jj]) { cnt += 1.f; s += acc[i][j][jj]; }
        const float mu = cnt > 0.f ? s / cnt : 0.f;
        q = 0.f;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            if (okr[i][jj]) { const float e = acc[i][j][jj] - mu; q += e * e; }
        n_ = cnt; m_ = mu;
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
          const float nb = __shfl_xor(n_, o, 64), mb = __shfl_xor(m_, o, 64), qb = __shfl_xor(q, o, 64);
          const float nt = n_ + nb;
          if (nt > 0.f) {
            const float dl = mb - m_, f = nb / nt;
            m_ += dl * f;
            q += qb + dl * dl * n_ * f;
          }
          n_ = nt;
        }
        }
        if (lane < 16) {
          st_n[wmi][wn0 + j * 16 + col16] = n_;
          st_m[wmi][wn0 + j * 16 + col16] = m_;
          st_q[wmi][wn0 + j * 16 + col16] = q;
        }
      }
    }
    if (BK == 32 && BN == 256 && a.out_bf16) {
      // The whole 256 x 256 tile is staged in LDS ([row][256 columns], pitch TPITCH), then every
      // store instruction writes two full 512-byte rows: tile rows t0 = (2 pp) NG + n and
      // t0 + NG, i.e. one image at two consecutive pixels.  Consecutive tile rows are different
      // images (image-minor order), so the per-wave staging below wrote 128-byte pieces of 8
      // images per instruction; with 1-KiB runs (merged sub-pixel FWD: pixels 2u..2u+3 of one
      // output row) the conv_layers.0 / .5 FWD epilogues drop from ~170 / ~245 us (B = 1024).
      __syncthreads();   // every wave is done with the ring slots
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            *(bf16*)(smem + (wm0 + i * 16 + rq + jj) * TPITCH + (wn0 + j * 16 + col16) * 2) = (bf16)acc[i][j][jj];
      __syncthreads();
      const int half = lane >> 5, kq = lane & 31;
      int scls = cls, sch = n0 + kq * 8;          // class / output channel of this lane's chunk
      if constexpr (SP && MODE == MODE_FWD) {
        if (a.sp_merge) {
          scls = sch / a.Ng;
          sch -= scls * a.Ng;
        }
      }
      const bool colok = sch < a.Ng && scls < 4;
      int py0 = 0, px0 = 0;
      if constexpr (SP && MODE == MODE_FWD) {
        py0 = (scls >> 1) ? sp.p0[2] : sp.p0[0];
        px0 = (scls & 1) ? sp.q0[1] : sp.q0[0];
      }
      for (int q = wid; q < BM / 2; q += 8) {
        const int t = ((2 * (q >> lgNG) + half) << lgNG) + (q & (NG - 1));
        const int pix = pix0 + (t >> lgNG), img = gi * NG + (t & (NG - 1));
        if (colok && pix < PQ && img < NL) {
          int y = fdiv(pix, fgw), x = pix - y * gw;
          if constexpr (SP && MODE == MODE_FWD) {
            y = py0 + 2 * y;
            x = px0 + 2 * x;
          }
          const int64_t o = (int64_t)img * a.os[0] + (int64_t)y * a.os[2] + (int64_t)x * a.os[3] + sch;
          *(uint4*)((bf16*)a.out + o) = *(const uint4*)(smem + t * TPITCH + kq * 16);
        }
      }
    } else {
    // stage the wave's tile in LDS (rows of WN values; passes of SROWS rows), then 16-byte
    // row-contiguous stores
    constexpr int PITCH = WN * 4 + 16;
    const int esz = a.out_bf16 ? 2 : 4;
    const int pitch = WN * esz + 16;
    char* stg = smem + wid * (SROWS * PITCH);
    const int cpr = WN * esz / 16;          // 16-byte chunks per row
    const int rpi = 64 / cpr;               // rows per wave instruction
    const int lr = lane / cpr, lch = lane % cpr;
#pragma unroll
    for (int ps = 0; ps < WM / SROWS; ++ps) {
      __syncthreads();   // every wave is done with the ring slots / the previous pass
#pragma unroll
      for (int i = 0; i < SROWS / 16; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            char* p = stg + (i * 16 + rq + jj) * pitch + (j * 16 + col16) * esz;
            const float v = acc[ps * (SROWS / 16) + i][j][jj];
            if (a.out_bf16) *(bf16*)p = (bf16)v;
            else *(float*)p = v;
          }
      __syncthreads();
      if (kc0 + lch * 16 / esz < a.Ng) {
        char* obase = (char*)a.out + (int64_t)kc0 * esz + lch * 16;
        for (int r = lr; r < SROWS; r += rpi)
          if (row_ok(ps * SROWS + r)) {
            const int64_t ro = row_off(ps * SROWS + r);
            const f32x4 vv = *(const f32x4*)(stg + r * pitch + lch * 16);
            *(uint4*)(obase + ro * esz) = __builtin_bit_cast(uint4, vv);
          }
      }
    }
    }
    if (part && wid < WGN) {   // the waves of row block 0 merge the WGM row waves of their columns
      for (int c = lane; c < WN; c += 64) {
        const int col = wn0 + c;
        float n_ = st_n[0][col], m_ = st_m[0][col], q = st_q[0][col];
        for (int w = 1; w < WGM; ++w) {
          const float nb = st_n[w][col];
          if (nb > 0.f) {
            const float mb = st_m[w][col], nt = n_ + nb, dl = mb - m_, f = nb / nt;
            m_ += dl * f;
            q += st_q[w][col] + dl * dl * n_ * f;
            n_ = nt;
          }
        }
        const int kc = kc0 + c;
        if (kc < a.Ng) {
          // one partial per row tile (merged sub-pixel FWD: per row tile and class)
          float* pp = part + (int64_t)(a.sp_merge ? tl * 4 + ecls : tl) * 3 * a.Ng;
          pp[kc] = n_;
          pp[a.Ng + kc] = m_;
          pp[2 * a.Ng + kc] = q;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < RM; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int r = i * 16 + rq + jj;
      if (!row_ok(r)) continue;
      const int64_t rowoff = row_off(r);
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int ng = n0 + wn0 + j * 16 + col16;
        if (ng >= a.Ng) continue;
        float v = acc[i][j][jj];
        const int64_t o = rowoff + (int64_t)ng * a.os[1];
        if (a.out_bf16) {
          bf16* yp = (bf16*)a.out + o;
          if (a.beta != 0.f) v += a.beta * (float)(*yp);
          *yp = (bf16)v;
        } else {
          float* yp = (float*)a.out + o;
          if (a.beta != 0.f) v += a.beta * (*yp);
          *yp = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// PERSISTENT short-K FWD / DGRAD: the generator's conv_layers.9 (neutron/generator.py:33, 2x2 taps
// x 128 channels -> 64: FWD 8 K-steps of 64 channels, 64 output columns) and its DGRAD (4 K-steps,
// 128 output columns); stride 1, no upsample, no sub-pixel packing.  With so few K-steps the ring
// kernel's per-tile pipeline fill and epilogue dominate: one 128 x 64 tile's 8 steps took ~11 us
// for ~1 us of MFMA work (0.30 of the HBM roofline at B = 1024).  Here
//   * one workgroup per CU loops over its tiles; the whole packed weight panel (nk K-steps x BN
//     rows x 128 B <= 64 KiB) is DMA'd into LDS once;
//   * the A ring runs over the workgroup's (tile, K-step) sequence without draining between tiles:
//     the next tile's first steps are in flight while the current tile's epilogue stores;
//   * the epilogue stages each wave's sub-tile in a private LDS region through inline-asm LDS
//     accesses (invisible to hipcc's wait insertion, ordered by explicit lgkmcnt waits) and stores
//     16-byte rows with buffer stores (invalid rows: out-of-range offsets, dropped), so every wave
//     issues a FIXED number of vector-memory ops per tile and the counted vmcnt waits stay exact
//     (vmcnt retires in issue order across loads, stores and LDS-DMA);
//   * FWD BatchNorm partials are Chan-merged per lane over the workgroup's tiles and written once
//     per workgroup at the end (chunks = workgroups instead of row tiles).
// Tile rows in the ring kernel's image-minor order (NG images x NB = BM / NG pixels per tile).  The
// tiles are split into 8 contiguous ranges, one per XCD, so the concurrently running tiles of one
// XCD are neighbouring pixels of the same images (shared input rows in its L2).
__device__ __forceinline__ void ds_write_u16(uint32_t addr, uint32_t v) {
  asm volatile("ds_write_b16 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ float ds_read_f32_asm(uint32_t addr) {
  float r;
  asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}
__device__ __forceinline__ void ds_write_f32_asm(uint32_t addr, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ int4v ds_read_b128_asm(uint32_t addr) {
  int4v r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}
__device__ __forceinline__ uint32_t ds_read_u8_asm(uint32_t addr) {
  uint32_t r;
  asm volatile("ds_read_u8 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}

// BNR (DGRAD only): the epilogue also runs the reduction pass of the BatchNorm backward that reads
// this dgrad's output dy (norm_fast.hip bn_reduce_fast, MODE 1): per channel sum of dnorm and
// dnorm * xhat, dnorm = d(chain)/dz * dy at z = gamma * xhat + beta, xhat = (h - mean) * invstd,
// with the stored bf16 dy values and the forward's dropout keep bits.  Each tile's epilogue issues
// LDS-DMA of the h rows (and keep bytes) its lanes just stored dy for into the wave's staging
// region; the NEXT tile's epilogue consumes them (by then the DMA has long landed, so the ring never
// drains for it) before it stages its own accumulators there.  The dgrad output is unchanged.
template <int MODE, int BN, bool BNR = false>
__global__ void __launch_bounds__(RT) conv_persist_kernel(ConvArgs a, int ntiles) {
  constexpr int BM = 128, BK = 64, WGM = 4, WGN = 2;
  constexpr int WM = BM / WGM, WN = BN / WGN;              // 32 x 32 (BN 64) / 32 x 64 (BN 128)
  constexpr int RM = WM / 16, RN = WN / 16;
  constexpr int ROWB = 2 * BK, PROWS = 1024 / ROWB, CPR = ROWB / 16;
  constexpr int APW = BM / PROWS / 8;                      // A pieces per wave per K-step
  constexpr int ABYTES = BM * ROWB;
  constexpr int NS = BN <= 64 ? 4 : 3;                     // ring slots (NS - 1 steps in flight)
  constexpr int PANEL = 65536;
  constexpr int SPITCH = WN * 2 + 16, STAGE = WM * SPITCH; // per-wave bf16 staging
  constexpr int OCPR = WN * 2 / 16, ORPI = 64 / OCPR, NST = WM / ORPI;   // 16-byte stores per tile
  constexpr int STB = 3 * WGM * BN * 4;
  // BNR: per wave NST x 1 KiB of h rows (lane-linear: piece p, lane l = the row / chunk the lane
  // stored in pass p) + 256 B of keep bytes ([32 rows][WN / 8]) in the staging region
  constexpr int KOFF = NST * 1024, KB = WN / 8, DPR = KB / 4;
  constexpr int NH = BNR ? NST + 1 : 0;                    // epilogue DMA ops (h pieces + keep)
  static_assert(!BNR || (MODE == MODE_DGRAD && KOFF + 256 <= STAGE && KB % 4 == 0), "BNR staging");
  __shared__ __attribute__((aligned(16))) char smem[PANEL + NS * ABYTES + 8 * STAGE + STB];
  char* const panel = smem;
  char* const ring = smem + PANEL;
  const es_conv_desc_t& d = a.d;
  const int NL = conv_live(a);   // live images (dynamic rows)
  const int nch = MODE == MODE_FWD ? d.C : d.K;
  const int cpt = nch / BK, nk = a.Kd / BK;
  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int lrow = lane / CPR, pc = lane % CPR;
  const uint32_t stg = lds_u32(ring + NS * ABYTES + wid * STAGE);
  float* const stb = (float*)(ring + NS * ABYTES + 8 * STAGE);
  const int NG = a.ng, PPG = NG / PROWS, NB = BM / NG;
  const int gh = MODE == MODE_FWD ? d.P : d.H, gw = MODE == MODE_FWD ? d.Q : d.W;
  const int PQ = gh * gw, TT = (PQ + NB - 1) / NB;
  ntiles = min(ntiles, (NL + NG - 1) / NG * TT);          // the live image groups' tiles
  const int lgNG = uni(31 - __builtin_clz(NG));
  FastDiv fgw;
  {
    uint32_t l2 = 0;
    while ((1u << l2) < (uint32_t)gw) ++l2;
    fgw.l = uni((int)l2);
    fgw.m = (uint32_t)uni((int)(uint32_t)(((1ull << 32) * ((1ull << l2) - (uint32_t)gw)) / (uint32_t)gw + 1));
  }
  // this workgroup's tiles: XCD x = blockIdx % 8 owns tiles [x * T / 8, (x + 1) * T / 8); its
  // workgroups (blockIdx / 8 = l of L) take every L-th tile of that range
  const int xcd = blockIdx.x & 7, L = (gridDim.x - xcd + 7) >> 3, lw = blockIdx.x >> 3;
  const int t_lo = (int)(((int64_t)ntiles * xcd) >> 3), t_hi = (int)(((int64_t)ntiles * (xcd + 1)) >> 3);
  const int my = t_hi - t_lo > lw ? (t_hi - t_lo - lw + L - 1) / L : 0;
  const int nsteps = my * nk;

  const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * 2));
  const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)(a.Ng * a.Kd * 2));
  const __amdgpu_buffer_rsrc_t ores = mkres(a.out, (uint32_t)(NL * a.os[0] * 2));
  // the weight panel: K-step k occupies [BN rows][128 B] at panel + k * BN * 128 (ring B layout)
  for (int pi = wid; pi < nk * (BN / PROWS); pi += 8) {
    const int k = pi / (BN / PROWS), rb = pi - k * (BN / PROWS);
    const int rr = rb * PROWS + lrow;
    bdma16(bres, (uint32_t)((rr * a.Kd + k * BK) * 2 + ((pc ^ swz_x<BK>(rr)) * 16)), panel + k * BN * ROWB + rb * 1024);
  }
  wait_vmcnt<0>();

  // issue cursor (tile iteration ii, K-step ik) and the issued tile's A pieces
  const int as0b = (int)a.as[0] * 2, as2b = (int)a.as[2] * 2, as3b = (int)a.as[3] * 2;
  uint32_t alane[APW];
  int pc0[APW], pc1[APW];
  bool pval[APW];
  int ii = 0, ik = 0;
  int icb = 0, ics = 0, icr = 0;   // issue K-step as (channel block, tap column, tap row): no divisions
  auto issue = [&](char* slot) {
    const bool live = ii < my;
    if (ik == 0 && live) {
      const int t = t_lo + lw + ii * L;
      const int gi = t / TT, pix0 = (t - gi * TT) * NB;
#pragma unroll
      for (int j = 0; j < APW; ++j) {
        const int pi = wid * APW + j, rr = pi * PROWS + lrow;
        const int ppix = pi / PPG, pix = pix0 + ppix;
        pval[j] = pix < PQ;
        const int pp = pval[j] ? pix : 0;
        const int y = fdiv(pp, fgw), x = pp - y * gw;
        const int img = gi * NG + (pi - ppix * PPG) * PROWS + lrow;
        alane[j] = (uint32_t)(img * as0b + ((pc ^ swz_x<BK>(rr)) * 16));   // images >= N: past num_records
        pc0[j] = MODE == MODE_FWD ? y - d.pad : y + d.pad;
        pc1[j] = MODE == MODE_FWD ? x - d.pad : x + d.pad;
      }
    }
    const int cb = icb, cr = icr, cs = ics;
#pragma unroll
    for (int j = 0; j < APW; ++j) {
      int hh, ww;
      bool ok;
      if constexpr (MODE == MODE_FWD) {
        hh = pc0[j] + cr; ww = pc1[j] + cs;
        ok = (unsigned)hh < (unsigned)d.H && (unsigned)ww < (unsigned)d.W;
      } else {
        hh = pc0[j] - cr; ww = pc1[j] - cs;
        ok = (unsigned)hh < (unsigned)d.P && (unsigned)ww < (unsigned)d.Q;
      }
      ok = ok && live && pval[j];
      const uint32_t u = ok ? (uint32_t)(hh * as2b + ww * as3b + cb * ROWB) : OOB;
      bdma16(ares, alane[j] + u, slot + (wid * APW + j) * 1024);
    }
    if (++icb == cpt) {
      icb = 0;
      if (++ics == d.S) {
        ics = 0;
        ++icr;
      }
    }
    if (++ik == nk) { ik = 0; ++ii; icb = ics = icr = 0; }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rn[RN], rmu[RN], rq2[RN];                 // running BatchNorm partial of the lane's columns
#pragma unroll
  for (int j = 0; j < RN; ++j) rn[j] = rmu[j] = rq2[j] = 0.f;
  // bias of the lane's columns, loaded before the ring starts (a VGPR load inside the loop makes
  // hipcc drain every DMA in flight with vmcnt(0) at its first use)
  float bcol[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) bcol[j] = (MODE == MODE_FWD && a.bias) ? a.bias[wn0 + j * 16 + (lane & 15)] : 0.f;
  const bool want_stats = MODE == MODE_FWD && a.stats_part != nullptr;
  const int r16 = lane & 15, g16 = lane >> 4, col16 = lane & 15, rq = (lane >> 4) * 4;
  const int elr = lane / OCPR, elch = lane % OCPR;        // epilogue: row pass / 8-channel chunk
  // BNR: the lane's 8 channels are fixed (wn0 + 8 elch ..), so are their statistics (loaded before
  // the ring starts, like bcol)
  float bmu[8], bis[8], bsc[8], bsh[8], bs1[8], bs2[8];
  int4v pdy[NST];                                         // the previous tile's stored dy
  const __amdgpu_buffer_rsrc_t hres = mkres(a.bnr_x, BNR ? (uint32_t)(NL * a.os[0] * 2) : 0u);
  const __amdgpu_buffer_rsrc_t kres = mkres(a.bnr_keep, BNR ? (uint32_t)((int64_t)NL * PQ * (a.Ng / 8)) : 0u);
  if constexpr (BNR) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = wn0 + elch * 8 + k;
      bmu[k] = a.bnr_mean[c];
      bis[k] = a.bnr_invstd[c];
      const float s = (a.bnr_gamma ? a.bnr_gamma[c] : 1.f) * bis[k];
      bsc[k] = s;
      bsh[k] = (a.bnr_beta ? a.bnr_beta[c] : 0.f) - bmu[k] * s;
      bs1[k] = bs2[k] = 0.f;
    }
#pragma unroll
    for (int p = 0; p < NST; ++p) pdy[p] = int4v{0, 0, 0, 0};
  }
  char* const stgp = ring + NS * ABYTES + wid * STAGE;
  // BNR: fold the previous tile's dy (pdy) with its h / keep bytes (landed in this wave's staging
  // region) into the per-lane sums; same expressions as bn_reduce_fast (norm_fast.hip)
  auto bnr_consume = [&]() {
    int4v hv[NST];
    uint32_t kb[NST];
#pragma unroll
    for (int p = 0; p < NST; ++p) {
      const int r = p * ORPI + elr;
      hv[p] = ds_read_b128_asm(stg + r * (WN * 2) + elch * 16);
      kb[p] = ds_read_u8_asm(stg + KOFF + r * KB + elch);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NST; ++p) {
      asm volatile("" : "+v"(hv[p]), "+v"(kb[p]));
      const bf16x8 h8 = __builtin_bit_cast(bf16x8, hv[p]), d8 = __builtin_bit_cast(bf16x8, pdy[p]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float v = (float)h8[k], dy = (float)d8[k];
        const bool keep = !a.bnr_drop || ((kb[p] >> k) & 1u);
        const float z = v * bsc[k] + bsh[k];
        const float zs = a.bnr_drop && a.bnr_dfirst ? z * a.bnr_scale : z;
        const float dsc = a.bnr_drop ? a.bnr_scale : 1.f;
        const float dn = keep ? dy * (zs > 0.f ? 1.f : a.bnr_slope) * dsc : 0.f;
        const float xh = (v - bmu[k]) * bis[k];
        bs1[k] += dn;
        bs2[k] += dn * xh;
      }
    }
  };
  struct Frag {
    bf16x8 a[RM], b[RN];
  };
  auto load = [&](Frag& f, const char* slot, const char* bk, int kk) {
    const int seg = kk * 4 + g16;
#pragma unroll
    for (int i = 0; i < RM; ++i) f.a[i] = *(const bf16x8*)(slot + swz<BK>(wm0 + i * 16 + r16, seg));
#pragma unroll
    for (int j = 0; j < RN; ++j) f.b[j] = *(const bf16x8*)(bk + swz<BK>(wn0 + j * 16 + r16, seg));
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
  };

  // epilogue of tile iteration ci: bias, rounding, fused statistics, staged 16-byte stores
  auto epilogue = [&](int ci) {
    const int t = t_lo + lw + ci * L;
    const int gi = t / TT, pix0 = (t - gi * TT) * NB;
    auto row_pix = [&](int r) { return pix0 + ((wm0 + r) >> lgNG); };
    auto row_img = [&](int r) { return gi * NG + ((wm0 + r) & (NG - 1)); };
    auto row_ok = [&](int r) { return row_pix(r) < PQ && row_img(r) < NL; };
    if constexpr (BNR) {
      if (ci > 0) {
        // the previous tile's h / keep DMA: older than the NS - 1 steps issued since (nk >= NS - 1)
        wait_vmcnt<(NS - 1) * APW>();
        bnr_consume();
      }
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][j][jj] = (float)(bf16)(acc[i][j][jj] + bcol[j]);
    }
    if (want_stats) {
      // the lane's (up to RM*4) valid values of each column, merged into its running partial:
      // no cross-lane traffic per tile (the lane groups and row waves are merged once, at the end)
      bool okr[RM][4];
      float nb = 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          okr[i][jj] = row_ok(i * 16 + rq + jj);
          nb += okr[i][jj] ? 1.f : 0.f;
        }
      if (nb > 0.f) {
        const float rb = __builtin_amdgcn_rcpf(nb);
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          float sm = 0.f;
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) sm += okr[i][jj] ? acc[i][j][jj] : 0.f;
          const float mb = sm * rb;
          float qb = 0.f;
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const float e = okr[i][jj] ? acc[i][j][jj] - mb : 0.f;
              qb = fmaf(e, e, qb);
            }
          const float nt = rn[j] + nb, f = nb * __builtin_amdgcn_rcpf(nt), dl = mb - rmu[j];
          rmu[j] = fmaf(dl, f, rmu[j]);
          rq2[j] += qb + dl * dl * rn[j] * f;
          rn[j] = nt;
        }
      }
    }
    // stage the wave's 32 x WN bf16 sub-tile (row pitch SPITCH), then 16-byte row stores
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const bf16 v = (bf16)acc[i][j][jj];
          ds_write_u16(stg + (i * 16 + rq + jj) * SPITCH + (j * 16 + col16) * 2, (uint32_t)__builtin_bit_cast(uint16_t, v));
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int lr = elr, lch = elch;
    int4v vals[NST];
#pragma unroll
    for (int p = 0; p < NST; ++p) vals[p] = ds_read_b128_asm(stg + (p * ORPI + lr) * SPITCH + lch * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < NST; ++p) asm volatile("" : "+v"(vals[p]));   // no use above the wait
    uint32_t voffs[NST];
#pragma unroll
    for (int p = 0; p < NST; ++p) {
      const int r = p * ORPI + lr;
      uint32_t voff = OOB;
      if (row_ok(r)) {
        const int pix = row_pix(r);
        const int y = fdiv(pix, fgw), x = pix - y * gw;
        const int64_t off = (int64_t)row_img(r) * a.os[0] + (int64_t)y * a.os[2] + (int64_t)x * a.os[3] + wn0 + lch * 8;
        voff = (uint32_t)(off * 2);
      }
      voffs[p] = voff;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, vals[p]), ores, voff, 0, 0);
    }
    if constexpr (BNR) {
      // this tile's h rows (the stored dy's positions: h has the output's layout) and keep bytes
      // -> the wave's staging region, consumed by the next epilogue (or after the loop)
#pragma unroll
      for (int p = 0; p < NST; ++p) {
        pdy[p] = vals[p];
        bdma16(hres, voffs[p], stgp + p * 1024);
      }
      const int kr = lane / DPR;
      uint32_t koff = OOB;
      if (kr < WM && row_ok(kr))
        koff = (uint32_t)(((int64_t)row_img(kr) * PQ + row_pix(kr)) * (a.Ng / 8) + (wn0 / 8) + (lane % DPR) * 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(kres, (lds_void*)(stgp + KOFF), 4, (int)koff, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

#pragma unroll
  for (int i = 0; i < NS - 1; ++i) issue(ring + i * ABYTES);
  int cur = 0, prv = NS - 1, ck = 0, ci = 0, last_epi = -1000;
  for (int s = 0; s < nsteps; ++s) {
    // step s landed: younger than its DMA are the NS - 2 later steps' pieces and, when an epilogue
    // ran within the last NS - 1 iterations (after step s was issued), its NST stores (+ BNR: its
    // NH h / keep DMA ops)
    if (s - last_epi <= NS - 1) wait_vmcnt<(NS - 2) * APW + NST + NH>();
    else wait_vmcnt<(NS - 2) * APW>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of step s - 1 are done
    ring_barrier();
    issue(ring + prv * ABYTES);                          // step s + NS - 1 into step s - 1's slot
    const char* slot = ring + cur * ABYTES;
    const char* bk = panel + ck * BN * ROWB;
    Frag f;
    load(f, slot, bk, 0);
    mma(f);
    load(f, slot, bk, 1);
    mma(f);
    if (++ck == nk) {
      epilogue(ci);
      ck = 0;
      ++ci;
      last_epi = s;
    }
    prv = cur;
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  wait_vmcnt<0>();
  if constexpr (BNR) {
    if (my > 0) bnr_consume();   // the last tile's rows
    // the workgroup's sums: the 64 / OCPR lanes of one channel chunk, then the WGM row waves
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int o = OCPR; o < 64; o <<= 1) {
        bs1[k] += __shfl_xor(bs1[k], o, 64);
        bs2[k] += __shfl_xor(bs2[k], o, 64);
      }
    float (*s1w)[BN] = (float (*)[BN])stb;
    float (*s2w)[BN] = s1w + WGM;
    const int wmi = wid / WGN;
    __syncthreads();
    if (lane < OCPR) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s1w[wmi][wn0 + lane * 8 + k] = bs1[k];
        s2w[wmi][wn0 + lane * 8 + k] = bs2[k];
      }
    }
    __syncthreads();
    if (wid < WGN) {
      for (int c = lane; c < WN; c += 64) {
        const int col = wn0 + c;
        float t1 = 0.f, t2 = 0.f;
        for (int w = 0; w < WGM; ++w) {
          t1 += s1w[w][col];
          t2 += s2w[w][col];
        }
        float* pp = a.bnr_part + (int64_t)blockIdx.x * 3 * a.Ng;
        pp[col] = 0.f;
        pp[a.Ng + col] = t1;
        pp[2 * a.Ng + col] = t2;
      }
    }
  }
  if (want_stats) {   // the workgroup's partial: merge the WGM row waves of each column
    float (*st_n)[BN] = (float (*)[BN])stb;
    float (*st_m)[BN] = st_n + WGM;
    float (*st_q)[BN] = st_n + 2 * WGM;
    const int wmi = wid / WGN;
#pragma unroll
    for (int j = 0; j < RN; ++j)           // the 4 lane groups of a column (rows rq..rq+3)
#pragma unroll
      for (int o = 16; o <= 32; o <<= 1) {
        const float nb = __shfl_xor(rn[j], o, 64), mb = __shfl_xor(rmu[j], o, 64), qb = __shfl_xor(rq2[j], o, 64);
        const float nt = rn[j] + nb;
        if (nt > 0.f) {
          const float dl = mb - rmu[j], f = nb / nt;
          rmu[j] += dl * f;
          rq2[j] += qb + dl * dl * rn[j] * f;
        }
        rn[j] = nt;
      }
    __syncthreads();
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        st_n[wmi][wn0 + j * 16 + col16] = rn[j];
        st_m[wmi][wn0 + j * 16 + col16] = rmu[j];
        st_q[wmi][wn0 + j * 16 + col16] = rq2[j];
      }
    }
    __syncthreads();
    if (wid < WGN) {
      for (int c = lane; c < WN; c += 64) {
        const int col = wn0 + c;
        float n_ = st_n[0][col], m_ = st_m[0][col], q = st_q[0][col];
        for (int w = 1; w < WGM; ++w) {
          const float nb = st_n[w][col];
          if (nb > 0.f) {
            const float mb = st_m[w][col], nt = n_ + nb, dl = mb - m_, f = nb / nt;
            m_ += dl * f;
            q += st_q[w][col] + dl * dl * n_ * f;
            n_ = nt;
          }
        }
        float* pp = a.stats_part + (int64_t)blockIdx.x * 3 * a.Ng;
        pp[col] = n_;
        pp[a.Ng + col] = m_;
        pp[2 * a.Ng + col] = q;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// PERSISTENT 256 x 256 merged sub-pixel FWD: the generator's conv_layers.0 / conv_layers.5
// (neutron/generator.py:25,30; 3x3 over the x2 upsample, run as one GEMM over (class, channel)
// columns, see conv_ring_kernel).  Measured on the ring kernel at B = 1024 (tools/ring_exp.py with
// the ES_RING_EXP builds): conv_layers.5 FWD 766 us with its epilogue, 521 us without; the
// epilogue (bias, statistics, 128 KiB of stores per tile) ran with the CU's MFMAs idle, since a
// 128 KiB ring leaves one workgroup per CU.  Here
//   * 256 workgroups (one per CU) loop over row tiles with a FIXED column tile each: the NT column
//     tiles of a row tile run side by side on one XCD (workgroups lw = NT l + ct), and each XCD
//     walks a contiguous range of row tiles (neighbouring pixels of the same images share its L2);
//   * the 4-slot ring (A and B pieces, 32-deep K-steps) continues across tiles: the next tile's
//     first steps are in flight while the epilogue runs, and its stores drain under the next
//     tile's MFMAs (fixed-count buffer stores, invalid rows at out-of-range offsets, so the
//     counted vmcnt waits stay exact: vmcnt retires in issue order across loads, stores, DMA);
//   * the epilogue stages 16-row passes of each wave's 128 x 64 sub-tile in a private 2.3 KiB LDS
//     region (inline-asm LDS accesses with explicit lgkmcnt waits) for 16-byte row stores;
//   * BatchNorm partials: per lane running sums / sums of squares of its 4 columns over all its
//     tiles (fixed columns), merged across lanes and row waves once at the end: one [3][Ng]
//     partial per (workgroup, class), chunks = 4 x 256.
template <int NT>
__global__ void __launch_bounds__(RT) conv_p256_kernel(ConvArgs a, int R) {
  constexpr int BM = 256, BN = 256, BK = 32, WGN = 4;
  constexpr int WM = 128, WN = 64, RM = WM / 16, RN = WN / 16, RMF = RM / 2;
  constexpr int ROWB = 2 * BK, PROWS = 1024 / ROWB, CPR = ROWB / 16;
  constexpr int APW = BM / PROWS / 8, BPW = BN / PROWS / 8, PW = APW + BPW;
  constexpr int NS = 4, ABYTES = BM * ROWB, SLOT = (BM + BN) * ROWB;
  constexpr int SPITCH = WN * 2 + 16, STAGE = 16 * SPITCH;   // per-wave staging: 16 rows
  constexpr int NST = WM / 8;                                 // 16-byte stores per tile per wave
  constexpr int LR = 32 / NT;                                 // workgroups per column tile per XCD
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT + 8 * STAGE + BN * 4 + 2 * 3 * BN * 4];
  const es_conv_desc_t& d = a.d;
  const int NL = conv_live(a);   // live images (dynamic rows)
  const SubPixel& sp = a.sp;
  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const uint32_t sbias = lds_u32(smem + NS * SLOT + 8 * STAGE);   // [BN] floats
  const uint32_t sst = sbias + BN * 4;                              // [2][3][BN] floats
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int lrow = lane / CPR, pc = lane % CPR;
  const int r16 = lane & 15, g16 = lane >> 4;
  const uint32_t stg = lds_u32(smem + NS * SLOT + wid * STAGE);

  // work of this workgroup: XCD x (blockIdx % 8) owns row tiles [R x / 8, R (x + 1) / 8); its
  // workgroup lw = NT l + ct takes column tile ct and every LR-th row tile from l
  const int xcd = blockIdx.x & 7, lw = blockIdx.x >> 3;
  const int ct = lw % NT, lr = lw / NT;
  const int n0 = ct * BN;
  const int NG = a.ng, PPG = NG / PROWS, NB = BM / NG;
  const int lgNG = uni(31 - __builtin_clz(NG));
  const int TT = sp.tile0[1], gh = sp.ph[0], gw = sp.pw[0], PQ = gh * gw;
  R = min(R, (NL + NG - 1) / NG * TT);                   // the live image groups' row tiles
  const int r_lo = (int)(((int64_t)R * xcd) >> 3), r_hi = (int)(((int64_t)R * (xcd + 1)) >> 3);
  const int my = r_hi - r_lo > lr ? (r_hi - r_lo - lr + LR - 1) / LR : 0;
  const int oh0 = sp.oh[0], ow0 = sp.ow[0], kw = sp.dw[0];
  const int ldb = sp.dh[0] * sp.dw[0] * d.C, nk = ldb / BK;
  FastDiv fgw;
  {
    uint32_t l = 0;
    while ((1u << l) < (uint32_t)gw) ++l;
    fgw.l = uni((int)l);
    fgw.m = (uint32_t)uni((int)(uint32_t)(((1ull << 32) * ((1ull << l) - (uint32_t)gw)) / (uint32_t)gw + 1));
  }
  // the wave's output class and first channel (a wave's 64 columns never straddle a class)
  const int ecls = (n0 + wn0) / a.Ng, kc0 = n0 + wn0 - ecls * a.Ng;
  const int py0 = sp.p0[0] + ((ecls >> 1) ? sp.p0[2] - sp.p0[0] : 0);
  const int px0 = sp.q0[0] + ((ecls & 1) ? sp.q0[1] - sp.q0[0] : 0);

  const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * 2));
  const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)(sp.tap0[4] * a.Ng * d.C * 2));
  const __amdgpu_buffer_rsrc_t ores = mkres(a.out, (uint32_t)(NL * a.os[0] * 2));
  const int as0b = (int)a.as[0] * 2, as2b = (int)a.as[2] * 2, as3b = (int)a.as[3] * 2;
  const int os0 = (int)a.os[0], os2 = (int)a.os[2], os3 = (int)a.os[3];   // (N * os0 * 2 < 2^31: host)
  uint32_t blane[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int rr = (wid * BPW + j) * PROWS + lrow;
    blane[j] = (uint32_t)((n0 + rr) * ldb * 2 + ((pc ^ swz_x<BK>(rr)) * 16));
  }

  // issue cursor: tile iteration ii, K-step ik = (tap cr, cs; channel cch); per-tap offset cache
  uint32_t alane[APW], ua_t[APW], ub_t = OOB;
  int pc0[APW], pc1[APW];
  bool pval[APW];
#pragma unroll
  for (int j = 0; j < APW; ++j) { alane[j] = 0; ua_t[j] = OOB; pc0[j] = pc1[j] = 0; pval[j] = false; }
  int ii = 0, ik = 0, cr = 0, cs = 0, cch = 0;
  auto issue = [&](char* slot) {
    const bool live = ii < my;
    if (ik == 0 && live) {   // a new tile: its A pieces (wave-uniform branch)
      const int tl = r_lo + lr + ii * LR;
      const int gi = tl / TT, pix0 = (tl - gi * TT) * NB;
#pragma unroll
      for (int j = 0; j < APW; ++j) {
        const int pi = wid * APW + j;
        const int rr = pi * PROWS + lrow;
        const int ppix = pi / PPG, pix = pix0 + ppix;
        pval[j] = pix < PQ;
        const int pp = pval[j] ? pix : 0;
        const int y = fdiv(pp, fgw), x = pp - y * gw;
        const int img = gi * NG + (pi - ppix * PPG) * PROWS + lrow;
        alane[j] = (uint32_t)(img * as0b + ((pc ^ swz_x<BK>(rr)) * 16));   // images >= N: past num_records
        pc0[j] = y + oh0;
        pc1[j] = x + ow0;
      }
    }
    if (cch == 0) {   // first step of a tap
#pragma unroll
      for (int j = 0; j < APW; ++j) {
        const int hs = pc0[j] + cr, ws = pc1[j] + cs;
        const bool ok = live && pval[j] && (unsigned)hs < (unsigned)d.H && (unsigned)ws < (unsigned)d.W;
        ua_t[j] = ok ? (uint32_t)(hs * as2b + ws * as3b) : OOB;
      }
      ub_t = live ? (uint32_t)((cr * kw + cs) * d.C * 2) : OOB;
    }
    const uint32_t co = (uint32_t)(cch * 2);
#pragma unroll
    for (int j = 0; j < APW; ++j) bdma16(ares, alane[j] + (ua_t[j] + co), slot + (wid * APW + j) * 1024);
#pragma unroll
    for (int j = 0; j < BPW; ++j) bdma16(bres, blane[j] + (ub_t + co), slot + ABYTES + (wid * BPW + j) * 1024);
    cch += BK;
    if (cch == d.C) {
      cch = 0;
      if (++cs == kw) { cs = 0; ++cr; }
    }
    if (++ik == nk) { ik = 0; ++ii; cr = cs = cch = 0; }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias of the lane's columns and the running statistics (sum, sum of squares, count)
  // the column tile's bias and the workgroup's statistics accumulators [2 row waves][3][BN] in LDS
  // (nothing of the epilogue stays in registers across the main loop), written through inline asm
  // like every epilogue LDS access (invisible to hipcc's DMA wait insertion)
  if (threadIdx.x < BN) {
    const int gcol = n0 + threadIdx.x;
    ds_write_f32_asm(sbias + threadIdx.x * 4, a.bias ? a.bias[gcol - (gcol / a.Ng) * a.Ng] : 0.f);
  }
  for (int i = threadIdx.x; i < 2 * 3 * BN; i += RT) ds_write_f32_asm(sst + i * 4, 0.f);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const bool want_stats = a.stats_part != nullptr;

  struct Frag {
    bf16x8 a[RMF], b[RN];
  };
  auto load = [&](Frag& f, const char* slot, int kk) {
#pragma unroll
    for (int i = 0; i < RMF; ++i) f.a[i] = *(const bf16x8*)(slot + swz<BK>(wm0 + (kk * RMF + i) * 16 + r16, g16));
#pragma unroll
    for (int j = 0; j < RN; ++j) f.b[j] = *(const bf16x8*)(slot + ABYTES + swz<BK>(wn0 + j * 16 + r16, g16));
  };
  auto mma = [&](const Frag& f, int kk) {
#pragma unroll
    for (int i = 0; i < RMF; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[kk * RMF + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[j], acc[kk * RMF + i][j], 0, 0, 0);
  };

  auto epilogue = [&](int ci) {
    const int tl = r_lo + lr + ci * LR;
    const int gi = tl / TT, pix0 = (tl - gi * TT) * NB;
    // per-lane values laundered through an empty asm: otherwise hipcc hoists the epilogue's
    // lane-constant addresses out of the main loop and spills them across it
    int le = lane;
    uint32_t stg_e = stg;
    asm volatile("" : "+v"(le), "+v"(stg_e));
    const int col16 = le & 15, rq = (le >> 4) * 4;
    float bcol[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) bcol[j] = ds_read_f32_asm(sbias + (wn0 + j * 16 + col16) * 4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // (every value an asm LDS read returned is passed through an empty asm after the wait, so no
    // use of it can be scheduled above the wait)
#pragma unroll
    for (int j = 0; j < RN; ++j) asm volatile("" : "+v"(bcol[j]));
    // store lanes: row lr8 (+ 8) of a pass, 16-byte chunk lch of the wave's 64 columns
    const int lr8 = le & 7, lch = le >> 3;
    float ts[8], ts2[8], npad = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) ts[k] = ts2[k] = 0.f;
    // 8 passes of 16 rows: bias + rounding, stage (row pitch SPITCH), then two 16-byte stores of
    // 8 rows each; the statistics accumulate from the stored rows (channels lch*8 .. of the lane)
#pragma unroll
    for (int i = 0; i < RM; ++i) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const bf16 vb = (bf16)(acc[i][j][jj] + bcol[j]);
          ds_write_u16(stg_e + (rq + jj) * SPITCH + (j * 16 + col16) * 2, (uint32_t)__builtin_bit_cast(uint16_t, vb));
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      int4v v0 = ds_read_b128_asm(stg_e + lr8 * SPITCH + lch * 16);
      int4v v1 = ds_read_b128_asm(stg_e + (lr8 + 8) * SPITCH + lch * 16);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("" : "+v"(v0), "+v"(v1));
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        // branch-free: the address is computed for every row, padding rows store out of range
        const int t = wm0 + i * 16 + p * 8 + lr8;
        const int pix = pix0 + (t >> lgNG), img = gi * NG + (t & (NG - 1));
        const bool ok = pix < PQ && img < NL;
        const int yy = fdiv(pix, fgw), xx = pix - yy * gw;
        const uint32_t voff = ok ? (uint32_t)(img * os0 + (py0 + 2 * yy) * os2 + (px0 + 2 * xx) * os3 + kc0 + lch * 8) * 2u : OOB;
        const int4v vv = p ? v1 : v0;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, vv), ores, voff, 0, 0);
        // a padding row gathered only zeros (out-of-range DMA), so its value is exactly
        // bf16(bias): summed with the rest, counted, and subtracted at the end of the tile
        npad += ok ? 0.f : 1.f;
        if (want_stats) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float lo = __uint_as_float((uint32_t)vv[k] << 16), hi = __uint_as_float((uint32_t)vv[k] & 0xFFFF0000u);
            ts[2 * k] += lo;
            ts2[2 * k] = fmaf(lo, lo, ts2[2 * k]);
            ts[2 * k + 1] += hi;
            ts2[2 * k + 1] = fmaf(hi, hi, ts2[2 * k + 1]);
          }
        }
      }
    }
    if (want_stats) {
      // the 8 row lanes of a chunk (lane bits 0..2), then lane lr8 == 0 adds the wave's totals of
      // its 8 channels into the row wave's LDS accumulators (one owner per address: deterministic)
#pragma unroll
      for (int o = 1; o <= 4; o <<= 1) {
        npad += __shfl_xor(npad, o, 64);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ts[k] += __shfl_xor(ts[k], o, 64);
          ts2[k] += __shfl_xor(ts2[k], o, 64);
        }
      }
      if (lr8 == 0) {
        const int wmi = wid / WGN;
        const uint32_t base = sst + (wmi * 3 * BN + wn0 + lch * 8) * 4;
        float o0[8], o1[8], o2[8], bb[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          o0[k] = ds_read_f32_asm(base + k * 4);
          o1[k] = ds_read_f32_asm(base + (BN + k) * 4);
          o2[k] = ds_read_f32_asm(base + (2 * BN + k) * 4);
          bb[k] = ds_read_f32_asm(sbias + (wn0 + lch * 8 + k) * 4);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(o0[k]), "+v"(o1[k]), "+v"(o2[k]), "+v"(bb[k]));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float vb = (float)(bf16)bb[k];
          ds_write_f32_asm(base + k * 4, o0[k] + ((float)WM - npad));
          ds_write_f32_asm(base + (BN + k) * 4, o1[k] + (ts[k] - npad * vb));
          ds_write_f32_asm(base + (2 * BN + k) * 4, o2[k] + (ts2[k] - npad * vb * vb));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // the ring (ring_loop_lean's single fragment set: register room for the epilogue), continued
  // across the workgroup's tiles
  const int nsteps = my * nk;
#pragma unroll
  for (int i = 0; i < NS - 1; ++i) issue(smem + i * SLOT);
  int cur = 0, prv = NS - 1, ck = 0, ci = 0, last_epi = -1000;
  for (int s = 0; s < nsteps; ++s) {
    // step s landed: younger than its DMA are the NS - 2 later steps' pieces and, when an
    // epilogue ran within the last NS - 1 iterations (after step s was issued), its NST stores
    if (s - last_epi <= NS - 1) wait_vmcnt<(NS - 2) * PW + NST>();
    else wait_vmcnt<(NS - 2) * PW>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of step s - 1 are done
    ring_barrier();
    issue(smem + prv * SLOT);                            // step s + NS - 1 into step s - 1's slot
    Frag f;
    load(f, smem + cur * SLOT, 0);
    mma(f, 0);
    load(f, smem + cur * SLOT, 1);
    mma(f, 1);
    if (++ck == nk) {
      epilogue(ci);
      ck = 0;
      ++ci;
      last_epi = s;
    }
    prv = cur;
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  wait_vmcnt<0>();   // every DMA (zero-fill steps included) and store retired
  if (want_stats) {
    // merge the 2 row waves' accumulators -> (count, mean, M2) per (workgroup, class)
    __syncthreads();
    for (int col = threadIdx.x; col < BN; col += RT) {
      float v[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) v[q] = ds_read_f32_asm(sst + (q * BN + col) * 4);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int q = 0; q < 6; ++q) asm volatile("" : "+v"(v[q]));
      const float n_ = v[0] + v[3], s_ = v[1] + v[4], q_ = v[2] + v[5];
      const float mu = n_ > 0.f ? s_ / n_ : 0.f;
      const int gcol = n0 + col, cc = gcol / a.Ng, ch = gcol - cc * a.Ng;
      float* pp = a.stats_part + ((int64_t)blockIdx.x * 4 + cc) * 3 * a.Ng;
      pp[ch] = n_;
      pp[a.Ng + ch] = mu;
      pp[2 * a.Ng + ch] = fmaxf(q_ - s_ * mu, 0.f);
    }
    // the classes outside this column tile: empty partials
    const int c_lo = n0 / a.Ng, c_hi = (n0 + BN - 1) / a.Ng;
    for (int idx = threadIdx.x; idx < 4 * a.Ng; idx += RT) {
      const int cc = idx / a.Ng, ch = idx - cc * a.Ng;
      if (cc < c_lo || cc > c_hi) {
        float* pp = a.stats_part + ((int64_t)blockIdx.x * 4 + cc) * 3 * a.Ng;
        pp[ch] = 0.f;
        pp[a.Ng + ch] = 0.f;
        pp[2 * a.Ng + ch] = 0.f;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// WGRAD: dW[m = k][ng = (r, s, c)] = sum over pixels of dy[pix][k] * xu[pix + (r, s)][c].
// Block tile BM out-channels x BN in-channels of ONE tap (C % BN == 0).  K-step t = (output
// pixel t / G, image group t % G): 64 images at one pixel.  Split over blockIdx.z with fp32
// atomics into the zeroed dw.
// SP: the tile's tap is a (class, d, e) tap of the sub-pixel decomposition; its K runs over the
// class's output pixels, and the epilogue adds the tile into every original tap (r, s) the
// combined tap covers (r in {2d - a, 2d - a + 1} within [0, R), likewise s).
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, bool SP>
__global__ void __launch_bounds__(RT) wgrad_ring_kernel(ConvArgs a) {
  constexpr int WGM = BM >= 64 ? BM / 64 : 1, WGN = 8 / WGM;   // waves along M / N
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int RM = WM / 16, RN = WN / 16;
  constexpr int AIMG = 64 * BM * 2, SLOT = 64 * (BM + BN) * 2;
  constexpr int APW = BM / 64, BPW = BN / 64;   // 1 KiB pieces per wave per slot
  constexpr int PW = APW + BPW;
  constexpr int ALPR = BM / 8, BLPR = BN / 8;   // lanes (16-byte chunks) per k-row
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];
  const es_conv_desc_t& d = a.d;
  const int NL = conv_live(a);   // live images (dynamic rows)
  const SubPixel& sp = a.sp;
  const int G = (NL + 63) >> 6;

  // blocks of one K split (same pixels) are consecutive on one XCD
  const int mt = gridDim.x, ntl = gridDim.y, tiles = mt * ntl;
  const int orig = blockIdx.x + (blockIdx.y + blockIdx.z * ntl) * mt;
  const int wg = xcd_remap(orig, tiles * gridDim.z);
  const int tile = wg % tiles, split = wg / tiles;
  const int m0 = (tile % mt) * BM, n0 = (tile / mt) * BN;
  const int rs = n0 / d.C, cb = n0 - rs * d.C;   // tap of the tile, channel base
  // the tile's tap and the pixel grid its K runs over
  int cls = 0, tr, ts, gq, npix;
  if constexpr (SP) {
    cls = (rs >= sp.tap0[1]) + (rs >= sp.tap0[2]) + (rs >= sp.tap0[3]);
    const int de = rs - sp.tap0[cls];
    tr = de / sp.dw[cls];
    ts = de - tr * sp.dw[cls];
    gq = sp.pw[cls];
    npix = sp.ph[cls] * gq;
  } else {
    tr = rs / d.S;
    ts = rs - tr * d.S;
    gq = d.Q;
    npix = d.P * d.Q;
  }
  const int kps = NL == a.d.N ? a.k_per_split : (npix * G + gridDim.z - 1) / gridDim.z;   // live K-steps
  const int tbeg = split * kps;                  // in K-steps
  const int tend = min(npix * G, tbeg + kps);
  if (tbeg >= tend) return;

  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * 2));
  const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)(NL * a.bs[0] * 2));
  const int as0b = (int)a.as[0] * 2, as2b = (int)a.as[2] * 2, as3b = (int)a.as[3] * 2;
  const int bs0b = (int)a.bs[0] * 2, bs2b = (int)a.bs[2] * 2, bs3b = (int)a.bs[3] * 2;

  uint32_t alane[APW], blane[BPW];
#pragma unroll
  for (int j = 0; j < APW; ++j) {
    const int kr = (wid * APW + j) * (64 / ALPR) + lane / ALPR;   // image of the K-step
    alane[j] = (uint32_t)(kr * as0b + (m0 + ((lane % ALPR) ^ swz_tr<BM>(kr)) * 8) * 2);
  }
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int kr = (wid * BPW + j) * (64 / BLPR) + lane / BLPR;
    const int chg = (lane % BLPR) ^ swz_tr<BN>(kr);
    blane[j] = (uint32_t)(kr * bs0b + (cb + chg * 8) * 2);
  }

  // K-step cursor (uniform): pixel (p, q) of the grid and image group gi of step t = (p*gq + q)*G + gi
  int cp, cq, cg, cstep = tbeg;
  {
    const int pix = tbeg / G;
    cg = tbeg - pix * G;
    cp = pix / gq;
    cq = pix - cp * gq;
  }
  // the tile's class values as register copies (no kernel-argument reloads inside the loop)
  const int cp0 = SP ? uni(sp.p0[cls]) : 0, cq0 = SP ? uni(sp.q0[cls]) : 0;
  const int coh = SP ? uni(sp.oh[cls]) : 0, cow = SP ? uni(sp.ow[cls]) : 0;
  auto issue = [&](char* slot) {
    const bool live = cstep < tend;
    uint32_t ua, ub;
    if constexpr (SP) {   // dy at output pixel (p0 + 2p, q0 + 2q), x at source (p + oh + d, q + ow + e)
      ua = live ? (uint32_t)(cg * 64 * as0b + (cp0 + 2 * cp) * as2b + (cq0 + 2 * cq) * as3b) : OOB;
      const int hs = cp + coh + tr, ws = cq + cow + ts;
      const bool ok = live && (unsigned)hs < (unsigned)d.H && (unsigned)ws < (unsigned)d.W;
      ub = ok ? (uint32_t)(cg * 64 * bs0b + hs * bs2b + ws * bs3b) : OOB;
    } else {
      ua = live ? (uint32_t)(cg * 64 * as0b + cp * as2b + cq * as3b) : OOB;
      const int hu = cp * d.stride - d.pad + tr, wu = cq * d.stride - d.pad + ts;
      const bool ok = live && (unsigned)hu < (unsigned)d.Hu && (unsigned)wu < (unsigned)d.Wu;
      ub = ok ? (uint32_t)(cg * 64 * bs0b + fdiv(hu, a.fUh) * bs2b + fdiv(wu, a.fUw) * bs3b) : OOB;
    }
#pragma unroll
    for (int j = 0; j < APW; ++j) bdma16(ares, alane[j] + ua, slot + (wid * APW + j) * 1024);
#pragma unroll
    for (int j = 0; j < BPW; ++j) bdma16(bres, blane[j] + ub, slot + AIMG + (wid * BPW + j) * 1024);
    ++cstep;
    ++cg;
    const bool w1 = cg == G;
    cg = w1 ? 0 : cg;
    cq += w1;
    const bool w2 = cq == gq;
    cq = w2 ? 0 : cq;
    cp += w2;
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  struct Frag {
    bf16x8 a[RM], b[RN];
  };
  auto load = [&](Frag& f, const char* slot, int kk) {
    const uint32_t base = lds_u32(slot);
#pragma unroll
    for (int i = 0; i < RM; ++i) f.a[i] = tr_frag_asm<BM>(base, kk * 32, wm0 + i * 16);
#pragma unroll
    for (int j = 0; j < RN; ++j) f.b[j] = tr_frag_asm<BN>(base + AIMG, kk * 32, wn0 + j * 16);
  };
  auto fence = [&](Frag& f) {
#pragma unroll
    for (int i = 0; i < RM; ++i) fence_frag(f.a[i]);
#pragma unroll
    for (int j = 0; j < RN; ++j) fence_frag(f.b[j]);
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
  };
  ring_loop<PW, 2 * (RM + RN)>(tend - tbeg, smem, SLOT, issue, load, mma, fence);

  const int col16 = lane & 15, rq = (lane >> 4) * 4;
  float* out = (float*)a.out;
  // original taps this tile's tap feeds: one (no SP) or up to 2 x 2 (SP)
  int r0 = tr, r1 = tr, s0 = ts, s1 = ts;
  if constexpr (SP) {
    const int ca = cls >> 1, cbb = cls & 1;
    r0 = max(0, 2 * tr - ca);
    r1 = min(d.R - 1, 2 * tr - ca + 1);
    s0 = max(0, 2 * ts - cbb);
    s1 = min(d.S - 1, 2 * ts - cbb + 1);
  }
  const int ldo = d.R * d.S * d.C;
  for (int r = r0; r <= r1; ++r)
    for (int s_ = s0; s_ <= s1; ++s_) {
      float* o = out + (r * d.S + s_) * d.C + cb + wn0 + col16;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int m = m0 + wm0 + i * 16 + rq + jj;
#pragma unroll
          for (int j = 0; j < RN; ++j) atomicAdd(o + (int64_t)m * ldo + j * 16, acc[i][j][jj]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// fp32 WGRAD (parity mode, v_mfma_f32_16x16x4_f32): the same product and image-minor K order as
// wgrad_ring_kernel, with K-steps of KI = 32 images at one pixel (so a slot has the bf16 kernel's
// byte geometry: 1 KiB DMA pieces, 3-slot ring).  An fp32 operand needs no transposing read: lane l
// of a 16x16x4 MFMA takes A[m = l & 15][k = l >> 4], one float of k-row k, so the LDS image is the
// DMA's natural [image][channel] layout read with ds_read_b32.  Odd k-rows have their 64-byte
// halves swapped (16-byte chunk c stored at c ^ 4): the two k-rows one 32-lane group reads then
// hit disjoint banks.
// DETERMINISTIC: every (tile, K split) stores its raw fp32 tile into its own slot of the partial
// buffer ws[split][M][taps * C] (no atomics); wgrad_reduce_kernel sums the splits (and, for SP, the
// four classes' combined taps over each original tap) in a fixed order.  The reference's same-seed
// reruns are bit-identical; with this, so are the parity mode's.
// ---------------------------------------------------------------------------------------------
// SPL: split-fp32 arithmetic (see split8).  A lane's 8 k-values of a 16x16x32 fragment are the
// images 4 j + (lane >> 4), j = 0..7, of the step (MFMA k = 8 (lane >> 4) + j; the same permutation
// for A and B), so each of the 8 ds_read_b32 instructions reads four consecutive k-rows, the access
// pattern the k-row swizzle was laid out for.
template <int BM, int BN, bool SP, bool SPL = false>
__global__ void __launch_bounds__(RT) wgrad_f32_kernel(ConvArgs a, float* __restrict__ ws, int ngt) {
  constexpr int KI = 32;                                       // images per K-step
  // waves along M / N: every wave tile at least 16 x 16 (64 x 64 tiles: 2 x 4 waves of 32 x 16)
  constexpr int WGM = BM >= 128 ? BM / 64 : (BN >= 128 ? 1 : 2), WGN = 8 / WGM;
  static_assert(BM / WGM >= 16 && BN / WGN >= 16, "wave tile below one 16 x 16 MFMA block");
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int RM = WM / 16, RN = WN / 16;
  constexpr int AIMG = KI * BM * 4, SLOT = KI * (BM + BN) * 4;
  constexpr int NSW = 3 * SLOT > 150 * 1024 ? 2 : NSLOT;        // (64 x 512 split tiles: 72 KiB slots)
  constexpr bool MT = BN == 512 && !SP;                         // a tile spans several taps (C < 512)
  constexpr int APW = BM / 64, BPW = BN / 64;                  // 1 KiB pieces per wave per slot
  constexpr int PW = APW + BPW;
  constexpr int ALPR = BM / 4, BLPR = BN / 4;                  // lanes (16-byte chunks) per k-row
  static_assert(ALPR >= 8 && BLPR >= 8, "the k-row swizzle flips 64-byte halves");
  __shared__ __attribute__((aligned(16))) char smem[NSW * SLOT];
  const es_conv_desc_t& d = a.d;
  const int NL = conv_live(a);   // live images (dynamic rows)
  const SubPixel& sp = a.sp;
  const int G = (NL + KI - 1) / KI;

  const int mt = gridDim.x, ntl = gridDim.y, tiles = mt * ntl;
  const int orig = blockIdx.x + (blockIdx.y + blockIdx.z * ntl) * mt;
  const int wg = xcd_remap(orig, tiles * gridDim.z);
  const int tile = wg % tiles, split = wg / tiles;
  const int m0 = (tile % mt) * BM, n0 = (tile / mt) * BN;
  const int rs = n0 / d.C, cb = n0 - rs * d.C;
  int cls = 0, tr, ts, gq, npix;
  if constexpr (SP) {
    cls = (rs >= sp.tap0[1]) + (rs >= sp.tap0[2]) + (rs >= sp.tap0[3]);
    const int de = rs - sp.tap0[cls];
    tr = de / sp.dw[cls];
    ts = de - tr * sp.dw[cls];
    gq = sp.pw[cls];
    npix = sp.ph[cls] * gq;
  } else {
    tr = rs / d.S;
    ts = rs - tr * d.S;
    gq = d.Q;
    npix = d.P * d.Q;
  }
  const int kps = NL == a.d.N ? a.k_per_split : (npix * G + gridDim.z - 1) / gridDim.z;   // live K-steps
  const int tbeg = min(split * kps, npix * G);
  const int tend = min(npix * G, tbeg + kps);

  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int col16 = lane & 15, rq = (lane >> 4) * 4;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (tbeg < tend) {
    const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * 4));
    const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)(NL * a.bs[0] * 4));
    const int as0b = (int)a.as[0] * 4, as2b = (int)a.as[2] * 4, as3b = (int)a.as[3] * 4;
    const int bs0b = (int)a.bs[0] * 4, bs2b = (int)a.bs[2] * 4, bs3b = (int)a.bs[3] * 4;
    uint32_t alane[APW], blane[BPW];
    int btr[MT ? BPW : 1], bts[MT ? BPW : 1];
#pragma unroll
    for (int j = 0; j < APW; ++j) {
      const int kr = (wid * APW + j) * (64 / ALPR) + lane / ALPR;   // image of the K-step
      alane[j] = (uint32_t)(kr * as0b + (m0 + ((lane % ALPR) ^ ((kr & 1) << 2)) * 4) * 4);
    }
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      // (a k-row of a 512-column tile spans two pieces)
      const int pc = wid * BPW + j;
      const int kr = BLPR > 64 ? pc / (BLPR / 64) : pc * (64 / BLPR) + lane / BLPR;
      const int ch = BLPR > 64 ? (pc % (BLPR / 64)) * 64 + lane : lane % BLPR;
      if constexpr (MT) {   // the lane's own tap and channel (the swizzle stays inside a tap: C % 32 == 0)
        const int ng = n0 + (ch ^ ((kr & 1) << 2)) * 4, rl = ng / d.C;
        btr[j] = rl / d.S;
        bts[j] = rl - btr[j] * d.S;
        blane[j] = (uint32_t)(kr * bs0b + (ng - rl * d.C) * 4);
      } else {
        blane[j] = (uint32_t)(kr * bs0b + (cb + (ch ^ ((kr & 1) << 2)) * 4) * 4);
      }
    }
    int cp, cq, cg, cstep = tbeg;
    if constexpr (MT) {   // pixel-minor K order: a step's right-hand taps are the next step's left ones (L2)
      cg = tbeg / npix;
      const int pix = tbeg - cg * npix;
      cp = pix / gq;
      cq = pix - cp * gq;
    } else {
      const int pix = tbeg / G;
      cg = tbeg - pix * G;
      cp = pix / gq;
      cq = pix - cp * gq;
    }
    const int cp0 = SP ? uni(sp.p0[cls]) : 0, cq0 = SP ? uni(sp.q0[cls]) : 0;
    const int coh = SP ? uni(sp.oh[cls]) : 0, cow = SP ? uni(sp.ow[cls]) : 0;
    auto issue = [&](char* slot) {
      const bool live = cstep < tend;
      uint32_t ua, ub;
      if constexpr (SP) {   // dy at output pixel (p0 + 2p, q0 + 2q), x at source (p + oh + d, q + ow + e)
        ua = live ? (uint32_t)(cg * KI * as0b + (cp0 + 2 * cp) * as2b + (cq0 + 2 * cq) * as3b) : OOB;
        const int hs = cp + coh + tr, wsx = cq + cow + ts;
        const bool ok = live && (unsigned)hs < (unsigned)d.H && (unsigned)wsx < (unsigned)d.W;
        ub = ok ? (uint32_t)(cg * KI * bs0b + hs * bs2b + wsx * bs3b) : OOB;
      } else if constexpr (MT) {   // one pixel per lane group: the B pieces' own taps
        ua = live ? (uint32_t)(cg * KI * as0b + cp * as2b + cq * as3b) : OOB;
        const int hb = cp * d.stride - d.pad, wb = cq * d.stride - d.pad;
#pragma unroll
        for (int j = 0; j < BPW; ++j) {
          const int hu = hb + btr[j], wu = wb + bts[j];
          const bool ok = live && (unsigned)hu < (unsigned)d.Hu && (unsigned)wu < (unsigned)d.Wu;
          const uint32_t u = ok ? (uint32_t)(cg * KI * bs0b + fdiv(hu, a.fUh) * bs2b + fdiv(wu, a.fUw) * bs3b) : OOB;
          bdma16(bres, blane[j] + u, slot + AIMG + (wid * BPW + j) * 1024);
        }
        ub = 0;
      } else {
        ua = live ? (uint32_t)(cg * KI * as0b + cp * as2b + cq * as3b) : OOB;
        const int hu = cp * d.stride - d.pad + tr, wu = cq * d.stride - d.pad + ts;
        const bool ok = live && (unsigned)hu < (unsigned)d.Hu && (unsigned)wu < (unsigned)d.Wu;
        ub = ok ? (uint32_t)(cg * KI * bs0b + fdiv(hu, a.fUh) * bs2b + fdiv(wu, a.fUw) * bs3b) : OOB;
      }
#pragma unroll
      for (int j = 0; j < APW; ++j) bdma16(ares, alane[j] + ua, slot + (wid * APW + j) * 1024);
      if constexpr (!MT) {
#pragma unroll
        for (int j = 0; j < BPW; ++j) bdma16(bres, blane[j] + ub, slot + AIMG + (wid * BPW + j) * 1024);
      }
      ++cstep;
      if constexpr (MT) {
        ++cq;
        const bool w1 = cq == gq;
        cq = w1 ? 0 : cq;
        cp += w1;
        const bool w2 = cp == d.P;
        cp = w2 ? 0 : cp;
        cg += w2;
      } else {
        ++cg;
        const bool w1 = cg == G;
        cg = w1 ? 0 : cg;
        cq += w1;
        const bool w2 = cq == gq;
        cq = w2 ? 0 : cq;
        cp += w2;
      }
    };
    // fragment set kk: images 16 kk .. 16 kk + 15 of the step, as 4 MFMA k-groups of 4 images
    struct Frag {
      float a[4][RM], b[4][RN];
    };
    const int kl = lane >> 4;
    auto rd = [&](const char* img, int rowb, int k, int row) {   // float (k-row k, row) of an image
      return *(const float*)(img + k * rowb + ((((row >> 2) ^ ((k & 1) << 2)) << 4) | ((row & 3) << 2)));
    };
    auto load = [&](Frag& f, const char* slot, int kk) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k = kk * 16 + 4 * t + kl;
#pragma unroll
        for (int i = 0; i < RM; ++i) f.a[t][i] = rd(slot, BM * 4, k, wm0 + i * 16 + col16);
#pragma unroll
        for (int j = 0; j < RN; ++j) f.b[t][j] = rd(slot + AIMG, BN * 4, k, wn0 + j * 16 + col16);
      }
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[t][i], f.b[t][j], acc[i][j], 0, 0, 0);
    };
    if constexpr (SPL) {
      struct FragS {
        float a[8][RM], b[8][RN];
      };
      // the lane's byte offsets of float (k-row 4 j + kl, row base + 16 i + col16) for i even / odd
      // (the odd-k-row swizzle flips bit 0 of base / 16 + i); the rest is an immediate 4 j rowb + 64 i
      const int sw = (kl & 1) * 64;
      const int sa0 = (wm0 >> 4) & 1 ? -sw : sw, sb0 = (wn0 >> 4) & 1 ? -sw : sw;
      const int oa0 = kl * BM * 4 + (wm0 + col16) * 4 + sa0, oa1 = oa0 - 2 * sa0;
      const int ob0 = AIMG + kl * BN * 4 + (wn0 + col16) * 4 + sb0, ob1 = ob0 - 2 * sb0;
      auto load_s = [&](FragS& f, const char* slot, int) {
        const char* pa[2] = {slot + oa0, slot + oa1};
        const char* pb[2] = {slot + ob0, slot + ob1};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int i = 0; i < RM; ++i) f.a[j][i] = *(const float*)(pa[i & 1] + j * 4 * BM * 4 + 64 * i);
#pragma unroll
          for (int jn = 0; jn < RN; ++jn) f.b[j][jn] = *(const float*)(pb[jn & 1] + j * 4 * BN * 4 + 64 * jn);
        }
      };
      auto mma_s = [&](const FragS& f) {
        bf16x8 bp[RN][3], ap[3];
        auto sa = [&](int i) {
          split8(f32x4{f.a[0][i], f.a[1][i], f.a[2][i], f.a[3][i]}, f32x4{f.a[4][i], f.a[5][i], f.a[6][i], f.a[7][i]},
                 ap);
        };
        sa(0);
#pragma unroll
        for (int jn = 0; jn < RN; ++jn) {   // B tiles split just before their first MFMAs
          split8(f32x4{f.b[0][jn], f.b[1][jn], f.b[2][jn], f.b[3][jn]},
                 f32x4{f.b[4][jn], f.b[5][jn], f.b[6][jn], f.b[7][jn]}, bp[jn]);
          acc[0][jn] = mfma_split6(ap, bp[jn], acc[0][jn]);
        }
#pragma unroll
        for (int i = 1; i < RM; ++i) {
          sa(i);
#pragma unroll
          for (int jn = 0; jn < RN; ++jn) acc[i][jn] = mfma_split6(ap, bp[jn], acc[i][jn]);
        }
      };
      if (a.prio && wid >= 4) __builtin_amdgcn_s_setprio(1);
      ring_loop_lean<PW, NSW, 1>(tend - tbeg, smem, SLOT, issue, load_s, mma_s);
    } else {
      auto nofence = [](Frag&) {};
      ring_loop<PW, 0>(tend - tbeg, smem, SLOT, issue, load, mma, nofence);
    }
  }
  // the raw tile of this split (zeros for an empty split): plain stores into its own slot
  float* o = ws + ((int64_t)split * a.M + m0 + wm0) * ngt + n0 + wn0 + col16;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int j = 0; j < RN; ++j) o[(int64_t)(i * 16 + rq + jj) * ngt + j * 16] = acc[i][j][jj];
}

// Ring loop that keeps the previous step's slot: compute of step t reads slots t and t-1, so the DMA
// issued at step t (step t + NS - 2) goes into step t-2's slot; NS - 2 steps in flight.
template <int PW, int NS, typename Issue, typename Load, typename Mma>
__device__ __forceinline__ void ring_loop_keep(int nk, char* smem, int slot_bytes, Issue& issue, Load& load,
                                               Mma& mma) {
  using Frag = typename std::remove_reference<typename lambda_arg<Load>::type>::type;
  static_assert(NS >= 3, "two live slots plus one in flight");
#pragma unroll
  for (int i = 0; i < NS - 2; ++i) issue(smem + i * slot_bytes);
  int cur = 0, prv = NS - 1, nxt = NS - 2;
  for (int t = 0; t < nk; ++t) {
    wait_vmcnt<(NS - 3) * PW>();                         // step t landed (this wave's pieces)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of step t-1 are done
    ring_barrier();
    issue(smem + nxt * slot_bytes);                      // step t + NS - 2 into step t-2's slot
    Frag f;
    load(f, smem + cur * slot_bytes, smem + prv * slot_bytes);
    mma(f);
    prv = cur;
    cur = cur == NS - 1 ? 0 : cur + 1;
    nxt = nxt == NS - 1 ? 0 : nxt + 1;
  }
  wait_vmcnt<0>();   // drain the zero-fill steps before the workgroup may exit
}

// Split-fp32 WGRAD of a 2 x 2, stride-1 convolution with 128 input and 64 output channels (neutron
// G conv_layers.9: 128 -> 64 on 46 x 46): one 64 x 512 tile (the four taps x 128 channels) whose
// K-steps walk the output columns of one row: column-step j of (image group g, row p) DMAs the input
// column x[g][p - pad + {0, 1}][j - pad][:] (2 rows x 128 channels) and dy[g][p][j - 1][:] (64
// channels), and multiplies dy(p, j - 1) with its four taps: the right-hand taps from this step's
// slot, the left-hand ones from the previous step's, so every input pixel is DMA'd into LDS once per
// row instead of once per tap (40 KiB per step instead of 72 KiB: the multi-tap tiles of
// wgrad_f32_kernel<64, 512> are LDS-fill bound).  A row is Q + 1 column-steps (the first loads only);
// a split starting inside a row first reloads the column before it (no MFMAs on such steps).
// Same deterministic partial slots and ordered reduce as wgrad_f32_kernel.
// (wgrad_f32_col2_kernel; a first version that split dy in every wave was slower.)  dy is split once per workgroup: the 8 waves share the tile's 64 dy rows,
// so instead of every wave splitting all of them (32 of a lane's 64 split values per step), dy is
// buffer-loaded into registers one step ahead (4 values per lane), split by the loading lane and
// written to LDS as bf16 planes in the fragment layout (as wgrad_coop_kernel), double-buffered; the
// x columns keep the DMA ring (32 KiB slots, two steps ahead, the previous slot kept).
__global__ void __launch_bounds__(RT) wgrad_f32_col2_kernel(ConvArgs a, float* __restrict__ ws, int ngt) {
  constexpr int KI = 32, CC = 128;
  constexpr int RM = 4, RN = 4;
  constexpr int SLOT = KI * 2 * CC * 4;                        // x: 32 images x 2 rows x 128 channels
  constexpr int NS = 4, BPW = 4;
  constexpr int APL = 4 * 1024, ABUF = 3 * APL;                // dy planes [plane][block][lane][8 k]
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT + 2 * ABUF];
  char* const abase = smem + NS * SLOT;
  const es_conv_desc_t& d = a.d;
  const int NL = conv_live(a);   // live images (dynamic rows)
  const int G = (NL + KI - 1) / KI, Q1 = d.Q + 1;
  const int split = xcd_remap(blockIdx.z, gridDim.z);
  const int nst = G * d.P * Q1;
  const int kps = NL == a.d.N ? a.k_per_split : (nst + gridDim.z - 1) / gridDim.z;   // live K-steps
  const int tbeg = min(split * kps, nst), tend = min(nst, tbeg + kps);

  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const int tap = wid >> 1, wtr = tap >> 1, wts = tap & 1, wc0 = (wid & 1) * 64;
  const int col16 = lane & 15, rq = (lane >> 4) * 4, kl = lane >> 4;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (tbeg < tend) {
    const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * 4));
    const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)(NL * a.bs[0] * 4));
    const int as0b = (int)a.as[0] * 4, as2b = (int)a.as[2] * 4, as3b = (int)a.as[3] * 4;
    const int bs0b = (int)a.bs[0] * 4, bs2b = (int)a.bs[2] * 4, bs3b = (int)a.bs[3] * 4;
    // dy half-block of this wave: rows 16 (wid >> 1) + col16, images 4 (4 (wid & 1) + jj) + kl
    const uint32_t alo = (uint32_t)((16 * (wid & 1) + kl) * as0b + (16 * (wid >> 1) + col16) * 4);
    const int awo = (wid >> 1) * 1024 + lane * 16 + (wid & 1) * 8;
    uint32_t blane[BPW];
    const int ltr = lane >> 5;
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int kr = wid * BPW + j;
      blane[j] = (uint32_t)(kr * bs0b + (((lane ^ ((kr & 1) << 2)) & 31) * 4) * 4);
    }
    int cg, cp, cj;
    {
      cg = tbeg / (d.P * Q1);
      const int r = tbeg - cg * d.P * Q1;
      cp = r / Q1;
      cj = r - cp * Q1;
    }
    const int s0 = tbeg - (cj > 0);
    cj -= cj > 0;
    int bstep = s0, bg = cg, bpr = cp, bj = cj;                 // DMA side (two steps ahead)
    int astep = s0, ag = cg, apr = cp, aj = cj;                 // dy side (one step ahead)
    {
      float4* z = (float4*)(smem + (NS - 1) * SLOT);
      for (int i = threadIdx.x; i < SLOT / 16; i += RT) z[i] = float4{0.f, 0.f, 0.f, 0.f};
    }
    auto adv = [&](int& st, int& g, int& pr, int& j) {
      ++st;
      ++j;
      const bool w1 = j == Q1;
      j = w1 ? 0 : j;
      pr += w1;
      const bool w2 = pr == d.P;
      pr = w2 ? 0 : pr;
      g += w2;
    };
    auto issue_b = [&](char* slot) {
      const int hu = bpr - d.pad + ltr, wu = bj - d.pad;
      const bool ok = bstep < tend && (unsigned)hu < (unsigned)d.H && (unsigned)wu < (unsigned)d.W;
      const uint32_t ub = ok ? (uint32_t)(bg * KI * bs0b + hu * bs2b + wu * bs3b) : OOB;
#pragma unroll
      for (int j = 0; j < BPW; ++j) bdma16(bres, blane[j] + ub, slot + (wid * BPW + j) * 1024);
      adv(bstep, bg, bpr, bj);
    };
    auto load_a = [&](float (&v)[4]) {   // zero on a row's first column and on a reloaded column
      const uint32_t ua = astep < tend && aj > 0 && astep >= tbeg
                              ? (uint32_t)(ag * KI * as0b + apr * as2b + (aj - 1) * as3b) : OOB;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        v[jj] = __builtin_bit_cast(float,
                                   __builtin_amdgcn_raw_buffer_load_b32(ares, (int)(ua + alo + jj * 4 * as0b), 0, 0));
      adv(astep, ag, apr, aj);
    };
    auto store_a = [&](const float (&v)[4], char* pb) {
      uint32_t h0, m0_, l0, h1, m1, l1;
      split_pair(v[0], v[1], h0, m0_, l0);
      split_pair(v[2], v[3], h1, m1, l1);
      *(uint2*)(pb + awo) = uint2{h0, h1};
      *(uint2*)(pb + APL + awo) = uint2{m0_, m1};
      *(uint2*)(pb + 2 * APL + awo) = uint2{l0, l1};
    };
    const int sw = (kl & 1) * 64;
    const int ob0 = kl * 2 * CC * 4 + (wtr * CC + wc0 + col16) * 4 + sw, ob1 = ob0 - 2 * sw;
    auto compute = [&](const char* slot, const char* prev, const char* pa) {
      const char* bimg = wts ? slot : prev;
      const char* pb[2] = {bimg + ob0, bimg + ob1};
      float fb[8][RN];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int jn = 0; jn < RN; ++jn) fb[j][jn] = *(const float*)(pb[jn & 1] + j * 4 * 2 * CC * 4 + 64 * jn);
      bf16x8 bp[RN][3], ap[3];
      const char* q = pa + lane * 16;
#pragma unroll
      for (int p = 0; p < 3; ++p) ap[p] = *(const bf16x8*)(q + p * APL);
#pragma unroll
      for (int jn = 0; jn < RN; ++jn) {
        split8(f32x4{fb[0][jn], fb[1][jn], fb[2][jn], fb[3][jn]}, f32x4{fb[4][jn], fb[5][jn], fb[6][jn], fb[7][jn]},
               bp[jn]);
        acc[0][jn] = mfma_split6(ap, bp[jn], acc[0][jn]);
      }
#pragma unroll
      for (int i = 1; i < RM; ++i) {
#pragma unroll
        for (int p = 0; p < 3; ++p) ap[p] = *(const bf16x8*)(q + p * APL + i * 1024);
#pragma unroll
        for (int jn = 0; jn < RN; ++jn) acc[i][jn] = mfma_split6(ap, bp[jn], acc[i][jn]);
      }
    };
    float av[4];
    load_a(av);                       // dy of the first step
    asm volatile("" ::: "memory");
    issue_b(smem);                    // x of the first two steps
    issue_b(smem + SLOT);
    store_a(av, abase);
    int cur = 0, prv = NS - 1, nxt = 2;
    const int nk = tend - s0;
    // (the x DMA of step t + 2 is issued after the dy planes are written: hipcc makes an LDS store
    // wait for every LDS-DMA in flight, vmcnt(0), which would otherwise drain it one step early)
    for (int t = 0; t < nk; ++t) {
      wait_vmcnt<BPW>();                                   // x of step t landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // dy planes of step t written, step t-1 read
      ring_barrier();
      load_a(av);                                          // dy of step t + 1
      asm volatile("" ::: "memory");
      compute(smem + cur * SLOT, smem + prv * SLOT, abase + (t & 1) * ABUF);
      store_a(av, abase + ((t & 1) ^ 1) * ABUF);           // (last read in step t - 1)
      asm volatile("" ::: "memory");
      issue_b(smem + nxt * SLOT);                          // x of step t + 2 (step t-2's slot)
      prv = cur;
      cur = cur == NS - 1 ? 0 : cur + 1;
      nxt = nxt == NS - 1 ? 0 : nxt + 1;
    }
    wait_vmcnt<0>();
  }
  float* o = ws + (int64_t)split * a.M * ngt + tap * CC + wc0 + col16;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int j = 0; j < RN; ++j) o[(int64_t)(i * 16 + rq + jj) * ngt + j * 16] = acc[i][j][jj];
}

// Split-fp32 WGRAD with a cooperative split (BM = 128: 2 x 4 waves of 64 x BN / 4).  In the
// DMA-ring kernels every wave splits its own A rows and B columns, so each value is split by the
// BN / WN (A) or BM / WM (B) waves that share it: 64 values per lane per K-step of 128 x 256,
// ~5.5 VALU instructions each, more vector issue than the step's 96 MFMAs leave free.  Here each
// value is split once: a K-step's A and B values are loaded straight into registers (one step
// ahead, plain buffer loads, zero outside the tensor), split by the lane that loaded them and
// written to LDS as three bf16 planes in the MFMA fragment layout ([plane][16-row block][lane]
// [8 k-values]: a wave's fragment is one conflict-free ds_read_b128), double-buffered behind one
// barrier per step.  (BM + BN) / 64 half-blocks of 4 values per lane: 24 values per lane per
// step of 128 x 256.  Same K order, arithmetic and partial slots as wgrad_f32_kernel<SPL>.
template <int BM, int BN, bool SP>
__global__ void __launch_bounds__(RT) wgrad_coop_kernel(ConvArgs a, float* __restrict__ ws, int ngt) {
  constexpr int KI = 32;
  constexpr int WGM = BM / 64, WGN = 8 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN, RM = WM / 16, RN = WN / 16;
  static_assert(BM == 128 && WN >= 16, "128-row tiles, wave tiles of >= 16 columns");
  constexpr int NBA = BM / 16, NB = (BM + BN) / 16;            // 16-row blocks: A's, A's and B's
  constexpr int NH = NB * 2 / 8, NHA = NBA * 2 / 8;             // half-blocks per wave (A's first)
  static_assert(NB * 2 % 8 == 0 && NBA * 2 % 8 == 0, "half-blocks split evenly over 8 waves");
  constexpr int PLANE = NB * 1024, PBUF = 3 * PLANE;
  __shared__ __attribute__((aligned(16))) char smem[2 * PBUF];
  const es_conv_desc_t& d = a.d;
  const int NL = conv_live(a);   // live images (dynamic rows)
  const SubPixel& sp = a.sp;
  const int G = (NL + KI - 1) / KI;

  const int mt = gridDim.x, ntl = gridDim.y, tiles = mt * ntl;
  const int orig = blockIdx.x + (blockIdx.y + blockIdx.z * ntl) * mt;
  const int wg = xcd_remap(orig, tiles * gridDim.z);
  const int tile = wg % tiles, split = wg / tiles;
  const int m0 = (tile % mt) * BM, n0 = (tile / mt) * BN;
  const int rs = n0 / d.C, cb = n0 - rs * d.C;
  int cls = 0, tr, ts, gq, npix;
  if constexpr (SP) {
    cls = (rs >= sp.tap0[1]) + (rs >= sp.tap0[2]) + (rs >= sp.tap0[3]);
    const int de = rs - sp.tap0[cls];
    tr = de / sp.dw[cls];
    ts = de - tr * sp.dw[cls];
    gq = sp.pw[cls];
    npix = sp.ph[cls] * gq;
  } else {
    tr = rs / d.S;
    ts = rs - tr * d.S;
    gq = d.Q;
    npix = d.P * d.Q;
  }
  const int kps = NL == a.d.N ? a.k_per_split : (npix * G + gridDim.z - 1) / gridDim.z;   // live K-steps
  const int tbeg = min(split * kps, npix * G);
  const int tend = min(npix * G, tbeg + kps);

  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int col16 = lane & 15, rq = (lane >> 4) * 4, kl = lane >> 4;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (tbeg < tend) {
    const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * 4));
    const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)(NL * a.bs[0] * 4));
    const int as0b = (int)a.as[0] * 4, as2b = (int)a.as[2] * 4, as3b = (int)a.as[3] * 4;
    const int bs0b = (int)a.bs[0] * 4, bs2b = (int)a.bs[2] * 4, bs3b = (int)a.bs[3] * 4;
    // half-block h of this wave: block b = (8 h + wid) / 2, k-half hh = wid & 1 (images
    // 4 (4 hh + jj) + kl, jj = 0..3, of the step), row / column 16 b + col16 of the tile
    uint32_t lofs[NH];
    int wofs[NH];   // LDS byte offset of the lane's 8 bytes in plane 0
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int hb = 8 * h + wid, b = hb >> 1, hh = hb & 1;
      if (h < NHA) lofs[h] = (uint32_t)((16 * hh + kl) * as0b + (m0 + 16 * b + col16) * 4);
      else lofs[h] = (uint32_t)((16 * hh + kl) * bs0b + (cb + 16 * (b - NBA) + col16) * 4);
      wofs[h] = b * 1024 + lane * 16 + hh * 8;
    }
    int cp, cq, cg;
    {
      const int pix = tbeg / G;
      cg = tbeg - pix * G;
      cp = pix / gq;
      cq = pix - cp * gq;
    }
    int cstep = tbeg;
    const int cp0 = SP ? uni(sp.p0[cls]) : 0, cq0 = SP ? uni(sp.q0[cls]) : 0;
    const int coh = SP ? uni(sp.oh[cls]) : 0, cow = SP ? uni(sp.ow[cls]) : 0;
    typedef float Stage[NH][4];
    auto load = [&](Stage& v) {   // the next K-step's values (zero past tend or outside the tensor)
      const bool live = cstep < tend;
      uint32_t ua, ub;
      if constexpr (SP) {
        ua = live ? (uint32_t)(cg * KI * as0b + (cp0 + 2 * cp) * as2b + (cq0 + 2 * cq) * as3b) : OOB;
        const int hs = cp + coh + tr, wsx = cq + cow + ts;
        const bool ok = live && (unsigned)hs < (unsigned)d.H && (unsigned)wsx < (unsigned)d.W;
        ub = ok ? (uint32_t)(cg * KI * bs0b + hs * bs2b + wsx * bs3b) : OOB;
      } else {
        ua = live ? (uint32_t)(cg * KI * as0b + cp * as2b + cq * as3b) : OOB;
        const int hu = cp * d.stride - d.pad + tr, wu = cq * d.stride - d.pad + ts;
        const bool ok = live && (unsigned)hu < (unsigned)d.Hu && (unsigned)wu < (unsigned)d.Wu;
        ub = ok ? (uint32_t)(cg * KI * bs0b + fdiv(hu, a.fUh) * bs2b + fdiv(wu, a.fUw) * bs3b) : OOB;
      }
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const uint32_t o = h < NHA ? ua + lofs[h] + jj * 4 * as0b : ub + lofs[h] + jj * 4 * bs0b;
          v[h][jj] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(h < NHA ? ares : bres,
                                                                                   (int)o, 0, 0));
        }
      ++cstep;
      ++cg;
      const bool w1 = cg == G;
      cg = w1 ? 0 : cg;
      cq += w1;
      const bool w2 = cq == gq;
      cq = w2 ? 0 : cq;
      cp += w2;
    };
    auto store = [&](const Stage& v, char* pb) {   // split and write the three planes
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        uint32_t h0, m0_, l0, h1, m1, l1;
        split_pair(v[h][0], v[h][1], h0, m0_, l0);
        split_pair(v[h][2], v[h][3], h1, m1, l1);
        *(uint2*)(pb + wofs[h]) = uint2{h0, h1};
        *(uint2*)(pb + PLANE + wofs[h]) = uint2{m0_, m1};
        *(uint2*)(pb + 2 * PLANE + wofs[h]) = uint2{l0, l1};
      }
    };
    auto load_b = [&](const char* pb, bf16x8 (&bp)[RN][3]) {
      const char* q = pb + lane * 16;
#pragma unroll
      for (int jn = 0; jn < RN; ++jn)
#pragma unroll
        for (int p = 0; p < 3; ++p) bp[jn][p] = *(const bf16x8*)(q + p * PLANE + (NBA + wn0 / 16 + jn) * 1024);
    };
    auto rows = [&](const char* pb, const bf16x8 (&bp)[RN][3]) {
      const char* q = pb + lane * 16;
      bf16x8 ap[3];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
#pragma unroll
        for (int p = 0; p < 3; ++p) ap[p] = *(const bf16x8*)(q + p * PLANE + (wm0 / 16 + i) * 1024);
#pragma unroll
        for (int jn = 0; jn < RN; ++jn) acc[i][jn] = mfma_split6(ap, bp[jn], acc[i][jn]);
      }
    };
    auto compute = [&](const char* pb) {
      bf16x8 bp[RN][3];
      load_b(pb, bp);
      rows(pb, bp);
    };
    auto sync = [] {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ring_barrier();
    };
    Stage s0;
    const int nk = tend - tbeg;
    load(s0);
    store(s0, smem);
    sync();
    // one stage of registers: step t + 1's loads are issued before step t's MFMAs and split after
    // them (two stages, 24 more registers, spill at 128 x 256; measured slower, round 4)
    for (int t = 0; t < nk; ++t) {
      char* cur = smem + (t & 1) * PBUF;
      char* nxt = smem + ((t & 1) ^ 1) * PBUF;
      load(s0);                 // step t + 1
      asm volatile("" ::: "memory");
      compute(cur);             // step t
      store(s0, nxt);           // step t + 1 (its buffer was last read in step t - 1)
      sync();
    }
    wait_vmcnt<0>();
    wait_vmcnt<0>();
  }
  float* o = ws + ((int64_t)split * a.M + m0 + wm0) * ngt + n0 + wn0 + col16;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int j = 0; j < RN; ++j) o[(int64_t)(i * 16 + rq + jj) * ngt + j * 16] = acc[i][j][jj];
}

// dW (torch layout [K][C][R][S], fp32) = beta * dW + sum over the splits of the partials
// ws[split][K][taps * C]; SP: original tap (r, s) sums the four classes' combined taps
// (d, e) = ((r + a) >> 1, (s + b) >> 1) of class (a, b).  A workgroup takes 32 consecutive outputs
// (c fastest: coalesced partial reads) x 8 split lanes; lane q sums splits q, q + 8, ... (classes
// innermost) and lane 0 adds the 8 lane sums in order: a fixed summation order, so reruns are bitwise
// equal.  (One thread per output looping over all splits was latency bound: 166 us for
// conv_layers.9's 512 splits.)
constexpr int WR_LANES = 8;
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int K, int C,
                                                           int R, int S, int ngt, SubPixel sp, float* __restrict__ dw,
                                                           float beta) {
  __shared__ float part[WR_LANES][32];
  const int64_t n = (int64_t)K * R * S * C;
  const int64_t zst = (int64_t)K * ngt;
  const int o = threadIdx.x & 31, q = threadIdx.x >> 5;
  for (int64_t i0 = blockIdx.x * (int64_t)32; i0 < n; i0 += (int64_t)gridDim.x * 32) {
    const int64_t i = i0 + o;
    float v = 0.f;
    int k = 0, r = 0, s = 0, c = 0;
    if (i < n) {
      c = (int)(i % C);
      int64_t t = i / C;
      s = (int)(t % S);
      t /= S;
      r = (int)(t % R);
      k = (int)(t / R);
      const float* p = ws + (int64_t)k * ngt + c + q * zst;
      if (sp.on) {
        int off[4];
#pragma unroll
        for (int cl = 0; cl < 4; ++cl)
          off[cl] = (sp.tap0[cl] + ((r + (cl >> 1)) >> 1) * sp.dw[cl] + ((s + (cl & 1)) >> 1)) * C;
        for (int z = q; z < splits; z += WR_LANES, p += WR_LANES * zst) {
#pragma unroll
          for (int cl = 0; cl < 4; ++cl) v += p[off[cl]];
        }
      } else {
        const int off = (r * S + s) * C;
#pragma unroll 4
        for (int z = q; z < splits; z += WR_LANES, p += WR_LANES * zst) v += p[off];
      }
    }
    part[q][o] = v;
    __syncthreads();
    if (q == 0 && i < n) {
      float u = part[0][o];
#pragma unroll
      for (int l = 1; l < WR_LANES; ++l) u += part[l][o];
      float* g = dw + (((int64_t)k * C + c) * R + r) * S + s;
      *g = (beta != 0.f ? beta * *g : 0.f) + u;
    }
    __syncthreads();
  }
}

// The same reduce with 4 consecutive channels per thread (C % 4 == 0): 16-byte partial loads, 128
// outputs per workgroup row; per output the summation order is the one above, so the results are
// bitwise those of wgrad_reduce_kernel (measured: that kernel moved its partials at ~1.4 TB/s, 23 us
// for conv_layers.5's 33.5 MB).
__global__ void __launch_bounds__(256) wgrad_reduce4_kernel(const float* __restrict__ ws, int splits, int K, int C,
                                                            int R, int S, int ngt, SubPixel sp, float* __restrict__ dw,
                                                            float beta) {
  __shared__ float4 part[WR_LANES][32];
  const int64_t n4 = (int64_t)K * R * S * (C >> 2);
  const int64_t zst = (int64_t)K * ngt;
  const int o = threadIdx.x & 31, q = threadIdx.x >> 5, C4 = C >> 2;
  for (int64_t i0 = blockIdx.x * (int64_t)32; i0 < n4; i0 += (int64_t)gridDim.x * 32) {
    const int64_t i = i0 + o;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = 0, r = 0, s = 0, c = 0;
    if (i < n4) {
      c = (int)(i % C4) * 4;
      int64_t t = i / C4;
      s = (int)(t % S);
      t /= S;
      r = (int)(t % R);
      k = (int)(t / R);
      const float* p = ws + (int64_t)k * ngt + c + q * zst;
      if (sp.on) {
        int off[4];
#pragma unroll
        for (int cl = 0; cl < 4; ++cl)
          off[cl] = (sp.tap0[cl] + ((r + (cl >> 1)) >> 1) * sp.dw[cl] + ((s + (cl & 1)) >> 1)) * C;
#pragma unroll 2
        for (int z = q; z < splits; z += WR_LANES, p += WR_LANES * zst) {
#pragma unroll
          for (int cl = 0; cl < 4; ++cl) {
            const float4 w = *(const float4*)(p + off[cl]);
            v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
          }
        }
      } else {
        const int off = (r * S + s) * C;
#pragma unroll 4
        for (int z = q; z < splits; z += WR_LANES, p += WR_LANES * zst) {
          const float4 w = *(const float4*)(p + off);
          v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
        }
      }
    }
    part[q][o] = v;
    __syncthreads();
    if (q == 0 && i < n4) {
      float4 u = part[0][o];
#pragma unroll
      for (int l = 1; l < WR_LANES; ++l) {
        const float4 w = part[l][o];
        u.x += w.x; u.y += w.y; u.z += w.z; u.w += w.w;
      }
      const float uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float* g = dw + (((int64_t)k * C + c + j) * R + r) * S + s;
        *g = (beta != 0.f ? beta * *g : 0.f) + uu[j];
      }
    }
    __syncthreads();
  }
}

// one deterministic reduce launch (the vector kernel when the channels allow it)
static void launch_wgrad_reduce(const float* ws, int splits, int K, int C, int R, int S, int ngt, const SubPixel& sp,
                                float* dw, float beta, hipStream_t st) {
  if (C % 4 == 0 && ngt % 4 == 0) {
    const int64_t n4 = (int64_t)K * C / 4 * R * S;
    const int blocks = (int)std::min<int64_t>((n4 + 31) / 32, 16384);
    hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3(blocks), dim3(256), 0, st, ws, splits, K, C, R, S, ngt, sp, dw, beta);
    return;
  }
  const int64_t n = (int64_t)K * C * R * S;
  const int blocks = (int)std::min<int64_t>((n + 31) / 32, 16384);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, splits, K, C, R, S, ngt, sp, dw, beta);
}
// host-side count of the MFMA conv kernels issued
// host-side count of the MFMA conv kernels issued (ring / persistent / p256 / fp32 wgrad), read by
// bench.py's probe to state how many launches one probed op is (fp32 image chunks)
int64_t g_conv_launches = 0;
extern "C" int64_t es_conv_launch_count() { return g_conv_launches; }

template <int MODE, int BM, int BN, bool SP, int BK = 64, typename T = bf16, int SPL = 0>
void launch_ring(const ConvArgs& a, int row_tiles, hipStream_t st) {
  dim3 grid(row_tiles, (a.Ng + BN - 1) / BN, 1);
  ++g_conv_launches;
  hipLaunchKernelGGL((conv_ring_kernel<MODE, BM, BN, SP, BK, T, SPL>), grid, dim3(RT), 0, st, a);
}

// minimum K-steps per WGRAD K-split (each split flushes its whole fp32 tile with atomics; 8 / 32 / 64
// / 128 measured within noise at B = 1024 and E = 4 B = 512, 128 slower)
constexpr int WGRAD_MINK = 8;
template <int BM, int BN, bool SP>
void launch_wgrad_ring(ConvArgs& a, hipStream_t st) {
  const int taps = SP ? a.sp.tap0[4] : a.d.R * a.d.S;
  const int tiles = (a.M / BM) * (taps * a.d.C / BN);
  int npix = a.d.P * a.d.Q;
  if (SP)
    for (int c = 0; c < 4; ++c) npix = c == 0 ? a.sp.ph[0] * a.sp.pw[0] : max(npix, a.sp.ph[c] * a.sp.pw[c]);
  const int ks = npix * ((a.d.N + 63) / 64);   // K-steps (the largest class)
  // one workgroup per CU: aim at two full rounds of the 256 CUs, >= g_wgrad_mink K-steps per split
  const int want = max(1, min(ks / WGRAD_MINK, 512 / tiles));
  const int per = (ks + want - 1) / want;
  a.k_per_split = per;
  dim3 grid(a.M / BM, taps * a.d.C / BN, (ks + per - 1) / per);
  ++g_conv_launches;
  hipLaunchKernelGGL((wgrad_ring_kernel<BM, BN, SP>), grid, dim3(RT), 0, st, a);
}

// a dense NHWC image stack (n outermost, rows of c contiguous values) below 1 GiB in bytes
template <int EB>
bool dense_small_t(const int64_t s[4], int n, int c, int h, int w) {
  return s[1] == 1 && s[3] == c && s[2] == (int64_t)w * c && s[0] == (int64_t)h * w * c &&
         (int64_t)n * s[0] * EB < (1ll << 30);
}
bool dense_small(const int64_t s[4], int n, int c, int h, int w) { return dense_small_t<2>(s, n, c, h, w); }

// Tuning constants, each chosen by alternating A/B on whole train steps:
//   * short-K FWD (<= 8 K-steps, e.g. conv_layers.9): 128 x 64 tiles, two workgroups per CU (201 -> 177 us);
//   * image-group size 64 of the row order (64 > 16 > 8 on the whole step; 8 for an isolated FWD),
//     16 under dynamic rows;
//   * sub-pixel FWD: class-interleaved tile order (14.45 -> 14.33 ms per step), one 256 x 256 GEMM over
//     (class, channel) columns when the 4 classes share their geometry;
//   * 256 x 256 tiles with 32-deep K-steps for FWD / DGRAD with >= 256 output columns;
//   * persistent short-K DGRAD (conv_persist_kernel: conv_layers.9 387 -> 259 us; as FWD it was slower
//     with fused statistics, 376 vs 364 us) and the persistent 256 x 256 merged sub-pixel FWD.
// The switches below are test hooks (es_conv_set_*: the kernel tests compare the paths bitwise).
constexpr int RING_NG = 64;
// Dynamic rows (multi-expert steps: capacity-B launches, a device count of live images): groups of
// 16 images, so the last, partly live group of an expert's rows carries at most 15 dead images
// through the MFMAs instead of up to 63 (E = 4, B = 512: 28.1 -> 26.8 ms/step fp32, 13.07 -> 12.69
// bf16, alternating against 64 and 32 on one box; profiles/r05_ngdyn_ab.log).  16 is also the
// smallest group the 32-deep K-step kernels' 16-row DMA pieces allow.
constexpr int RING_NG_DYN = 16;
bool g_subpixel_off = false;
bool g_ring256 = true;
bool g_persist = true;
bool g_p256 = true;

}  // namespace

thread_local StatsRequest g_stats_req;
thread_local BnRedRequest g_bnr_req;

// Class geometry of the sub-pixel decomposition (see SubPixel): output row p belongs to class
// a = (p - pad) mod 2, p = p0 + 2u, source row of combined tap d = u + oh + d, dh = taps.
// tile0: prefix over the classes of ceil(class pixels / row_tile) (row_tile = pixels per FWD tile).
void es_make_subpixel(const es_conv_desc_t& d, int row_tile, SubPixel& sp) {
  int dhv[2], dwv[2], p0v[2], q0v[2], phv[2], pwv[2], ohv[2], owv[2];
  for (int a = 0; a < 2; ++a) {
    dhv[a] = ((a + d.R - 1) >> 1) + 1;
    dwv[a] = ((a + d.S - 1) >> 1) + 1;
    p0v[a] = (a + d.pad) & 1;
    q0v[a] = (a + d.pad) & 1;
    phv[a] = d.P > p0v[a] ? (d.P - p0v[a] + 1) / 2 : 0;
    pwv[a] = d.Q > q0v[a] ? (d.Q - q0v[a] + 1) / 2 : 0;
    ohv[a] = (p0v[a] - d.pad - a) / 2;
    owv[a] = (q0v[a] - d.pad - a) / 2;
  }
  sp.on = 1;
  sp.tap0[0] = 0;
  sp.tile0[0] = 0;
  for (int c = 0; c < 4; ++c) {
    const int a = c >> 1, b = c & 1;
    sp.ph[c] = phv[a];
    sp.pw[c] = pwv[b];
    sp.p0[c] = p0v[a];
    sp.q0[c] = q0v[b];
    sp.oh[c] = ohv[a];
    sp.ow[c] = owv[b];
    sp.dh[c] = dhv[a];
    sp.dw[c] = dwv[b];
    sp.tap0[c + 1] = sp.tap0[c] + dhv[a] * dwv[b];
    const int pix = phv[a] * pwv[b];
    sp.tile0[c + 1] = sp.tile0[c] + (row_tile > 0 ? (pix + row_tile - 1) / row_tile : 0);
  }
}

extern "C" int es_conv_set_ring(int on) {
  const int old = !g_ring_off;
  g_ring_off = !on;
  return old;
}

extern "C" int es_conv_set_persist(int on) {
  // bit 0: the persistent kernel on / off; bit 1: also for FWD
  const int old = g_persist ? 1 : 0;
  g_persist = (on & 1) != 0;
  return old;
}

extern "C" int es_conv_set_p256(int on) {
  const int old = g_p256;
  g_p256 = on != 0;
  return old;
}

extern "C" int es_conv_set_ring256(int on) {
  const int old = g_ring256;
  g_ring256 = on != 0;
  return old;
}

extern "C" int es_conv_set_subpixel(int on) {
  const int old = !g_subpixel_off;
  g_subpixel_off = !on;
  return old;
}

extern "C" int es_subpixel_taps(int R, int S) {
  return (((R - 1) >> 1) + 1 + (R >> 1) + 1) * (((S - 1) >> 1) + 1 + (S >> 1) + 1);
}

// Whether es_conv2d_fwd / es_conv2d_dgrad take the sub-pixel path for this conv (then the weights
// must be packed with es_pack_conv_weight mode 2 / 3 and d->subpixel set): bf16, x2 integer
// upsample, stride 1, channels % 64 == 0, below the ring's size limits.  The activations must be
// dense NHWC at call time.
extern "C" int es_conv_subpixel_ok(const es_conv_desc_t* d, es_dtype_t dt) {
  if (g_ring_off || g_subpixel_off || !d || (dt != ES_BF16 && dt != ES_F32)) return 0;
  if (d->up_h != 2 || d->up_w != 2 || d->hmap || d->stride != 1) return 0;
  if (d->C % 64 || d->K % 64) return 0;
  const int eb = dt == ES_F32 ? 4 : 2;
  const int64_t xbytes = (int64_t)d->N * d->H * d->W * d->C * eb, ybytes = (int64_t)d->N * d->P * d->Q * d->K * eb;
  const int64_t wbytes = (int64_t)d->K * d->C * es_subpixel_taps(d->R, d->S) * eb;
  // fp32: the ring launches over image chunks below 1 GiB (es_conv_ring_launch_f32)
  if (dt == ES_F32) return wbytes < (1ll << 30) && (int64_t)d->H * d->W * d->C * eb < (1ll << 24) &&
                           (int64_t)d->P * d->Q * d->K * eb < (1ll << 24);
  // (bf16 too: operands of >= 1 GiB run as image chunks, es_conv_ring_launch; the merged 256 x 256
  // kernel's 32-bit output offsets are checked where it is chosen)
  (void)xbytes; (void)ybytes;
  return wbytes < (1ll << 30) && (int64_t)d->H * d->W * d->C * eb < (1ll << 24) &&
         (int64_t)d->P * d->Q * d->K * eb < (1ll << 24);
}

template <typename T, int SPL = 0>
int ring_fd(ConvArgs& a, int mode, hipStream_t st);
namespace {
int chunk_images(int64_t img_bytes, int N);
int ring_launch_chunks(ConvArgs& a, int mode, int nc, hipStream_t st);
}  // namespace

int es_conv_ring_launch(ConvArgs& a, int mode, hipStream_t st) {
  const es_conv_desc_t& d = a.d;
  const bool sp_weights = d.subpixel != 0;   // FWD / DGRAD operands packed for the sub-pixel path
  if (g_ring_off && !sp_weights) return 0;
  if (d.hmap != nullptr || d.stride > 2 || a.splitk) return sp_weights ? -1 : 0;
  // gathered operands of >= 1 GiB (a capacity-2048 expert's conv_layers.5 output gradient is 1.1 GB
  // in bf16): launches over image chunks below the limit, as the fp32 ring does
  {
    const int64_t img = (mode == MODE_WGRAD ? std::max<int64_t>(a.as[0], a.bs[0]) : a.as[0]) * 2;
    const int nc = chunk_images(img, d.N);
    if (nc < d.N) return ring_launch_chunks(a, mode, nc, st);
  }
  if (mode == MODE_WGRAD) {
    if (!dense_small(a.as, d.N, d.K, d.P, d.Q) || !dense_small(a.bs, d.N, d.C, d.H, d.W)) return 0;
    const bool sp = !g_subpixel_off && d.up_h == 2 && d.up_w == 2 && d.stride == 1;
    if (sp) es_make_subpixel(d, 0, a.sp);
#define ES_WG(BM, BN) (sp ? launch_wgrad_ring<BM, BN, true>(a, st) : launch_wgrad_ring<BM, BN, false>(a, st))
    if (d.K % 256 == 0 && d.C % 128 == 0) ES_WG(256, 128);
    else if (d.K % 128 == 0 && d.C % 256 == 0) ES_WG(128, 256);
    else if (d.K % 128 == 0 && d.C % 128 == 0) ES_WG(128, 128);
    else if (d.K == 64 && d.C % 128 == 0) ES_WG(64, 128);   // neutron G conv_layers.9 (128 -> 64)
    else return 0;
#undef ES_WG
    g_ring_hit = 1 | (sp ? 4 : 0);
    return 1;
  }
  const int rc = ring_fd<bf16>(a, mode, st);
  if (rc > 0) g_ring_hit = 1 | (sp_weights ? 4 : 0);
  return rc;
}

// FWD / DGRAD ring launch for bf16 or fp32 operands (fp32: the parity mode's exact fp32 MFMA, or with
// SPL the split-fp32 bf16-plane MFMA on 32-channel K-steps; the persistent kernels are bf16-only)
template <typename T, int SPL>
int ring_fd(ConvArgs& a, int mode, hipStream_t st) {
  const es_conv_desc_t& d = a.d;
  const bool sp_weights = d.subpixel != 0;
  if constexpr (SPL == 2) {   // the pre-split B planes follow the fp32 packing (es_pack_weight_planes)
    const int64_t nel = (int64_t)d.K * d.C * (sp_weights ? es_subpixel_taps(d.R, d.S) : d.R * d.S);
    a.b_src = (const char*)a.b_src + es_weight_planes_offset(nel);
  }
  constexpr int EB = sizeof(T);
  // caller checked: channels % (128 / EB) == 0, K % (128 / EB) == 0 per step
  int PQ;
  if (mode == MODE_FWD) {
    if (!dense_small_t<EB>(a.as, d.N, d.C, d.H, d.W)) return sp_weights ? -1 : 0;
    PQ = d.P * d.Q;
  } else {
    if (!dense_small_t<EB>(a.as, d.N, d.K, d.P, d.Q)) return sp_weights ? -1 : 0;
    PQ = a.fold ? d.H * d.W : d.Hu * d.Wu;
  }
  if ((int64_t)a.Ng * a.Kd * EB * (sp_weights ? 2 : 1) >= (1ll << 30)) return sp_weights ? -1 : 0;
  // image group size of the row order (see conv_ring_kernel).  Measured on the whole train step
  // (tools/gpu_ab.sh, one box): 64 > 16 > 8 for both FWD and DGRAD, although an isolated FWD
  // prefers 8 (less MALL traffic).  Dynamic rows take 16 (RING_NG_DYN).
  a.ng = d.rows ? RING_NG_DYN : RING_NG;
  while (a.ng > 8 && a.ng / 2 >= d.N) a.ng /= 2;   // small batches (per-expert shards): no empty rows
  const int NGI = (d.N + a.ng - 1) / a.ng;
  const int nt128 = (a.Ng + 127) / 128;
  // short-K FWD (<= 8 K-steps, e.g. conv_layers.9: 2x2 taps x 128 channels): 128 x 64 tiles (72 KiB
  // of LDS, two workgroups per CU) so one tile's fill and epilogue overlap another's MFMAs
  // (measured 201 -> 177 us; the same rule on the DGRAD of that conv was slower)
  // (bf16 only: the fp32 kernels' K-steps are 32 channels, so the same conv has 16 of them and takes
  // the 256-row tiles: conv_layers.9 FWD 1109 -> 1064 us per op at B = 1024, round 5)
  const bool shortk = mode == MODE_FWD && !sp_weights && a.Kd / 64 <= 8 && EB == 2;
  // persistent short-K kernel (conv_persist_kernel): FWD / DGRAD, stride 1, no upsample / sub-pixel,
  // <= 8 K-steps, the whole weight panel (nk x Ng x 128 B) within 64 KiB, dense 16-byte output rows
  {
    const int nkk = a.Kd / 64;
    const int nchk = mode == MODE_FWD ? d.C : d.K;
    const bool rows16 = a.os[1] == 1 && a.beta == 0.f && a.out_bf16 && a.os[0] % 8 == 0 && a.os[2] % 8 == 0 &&
                        a.os[3] % 8 == 0 && ((uintptr_t)a.out & 15) == 0 &&
                        (int64_t)d.N * a.os[0] * 2 < (1ll << 31);
    const bool geo = d.stride == 1 && !sp_weights && !a.fold && d.hmap == nullptr && d.up_h <= 0 &&
                     d.Hu == d.H && d.Wu == d.W && nchk % 64 == 0 && a.Kd % 64 == 0;
    const int NS = a.Ng <= 64 ? 4 : 3;
    if (EB == 2 && g_persist && mode == MODE_DGRAD && geo && rows16 && (a.Ng == 64 || a.Ng == 128) &&
        nkk >= NS - 1 && nkk <= 8 &&
        nkk * a.Ng <= 512 && a.ng >= 16) {
      const int NB = 128 / a.ng, TT = (PQ + NB - 1) / NB;
      const int ntiles = NGI * TT;
      const int nwg = std::min(ntiles, 256);
      a.stats_part = nullptr;
      if (mode == MODE_FWD && g_stats_req.part && (int64_t)nwg * 3 * a.Ng <= g_stats_req.floats) {
        a.stats_part = g_stats_req.part;
        g_stats_req.chunks = nwg;
      }
      // fused BatchNorm-backward reduction over the stored dy (es_conv2d_dgrad_bnred)
      const BnRedRequest& q = g_bnr_req;
      bool bnr = false;
      if (mode == MODE_DGRAD && q.part && (int64_t)nwg * 3 * a.Ng <= q.floats && q.nm && q.ch && q.x &&
          ((uintptr_t)q.x & 15) == 0 && (q.ch->act == ES_ACT_LRELU || q.ch->act == ES_ACT_RELU) &&
          (!q.ch->drop.enabled || q.ch->keep) && a.os[3] == a.Ng && a.os[2] == (int64_t)d.W * a.Ng &&
          a.os[0] == (int64_t)d.H * d.W * a.Ng) {
        a.bnr_x = q.x;
        a.bnr_keep = q.ch->keep;
        a.bnr_mean = q.nm->mean; a.bnr_invstd = q.nm->invstd; a.bnr_gamma = q.nm->gamma; a.bnr_beta = q.nm->beta;
        a.bnr_drop = q.ch->drop.enabled != 0;
        a.bnr_scale = a.bnr_drop ? q.ch->drop.scale : 1.f;
        a.bnr_dfirst = q.ch->dropout_first;
        a.bnr_slope = q.ch->act == ES_ACT_LRELU ? q.ch->slope : 0.f;
        a.bnr_part = q.part;
        g_bnr_req.chunks = nwg;
        bnr = true;
      }
      ++g_conv_launches;
      if (mode == MODE_FWD) {
        if (a.Ng == 64) hipLaunchKernelGGL((conv_persist_kernel<MODE_FWD, 64>), dim3(nwg), dim3(RT), 0, st, a, ntiles);
        else hipLaunchKernelGGL((conv_persist_kernel<MODE_FWD, 128>), dim3(nwg), dim3(RT), 0, st, a, ntiles);
      } else if (bnr) {
        if (a.Ng == 64) hipLaunchKernelGGL((conv_persist_kernel<MODE_DGRAD, 64, true>), dim3(nwg), dim3(RT), 0, st, a, ntiles);
        else hipLaunchKernelGGL((conv_persist_kernel<MODE_DGRAD, 128, true>), dim3(nwg), dim3(RT), 0, st, a, ntiles);
      } else {
        if (a.Ng == 64) hipLaunchKernelGGL((conv_persist_kernel<MODE_DGRAD, 64>), dim3(nwg), dim3(RT), 0, st, a, ntiles);
        else hipLaunchKernelGGL((conv_persist_kernel<MODE_DGRAD, 128>), dim3(nwg), dim3(RT), 0, st, a, ntiles);
      }
      return 1;
    }
  }
  // >= 3 rounds of 256-row tiles
  const bool big = !shortk && (int64_t)NGI * a.ng * PQ / 256 * nt128 >= 768;
  const int BM = big ? 256 : 128, NB = BM / a.ng;
  int row_tiles = NGI * ((PQ + NB - 1) / NB);
  if (sp_weights) {
    es_make_subpixel(d, NB, a.sp);   // FWD: tile0 = per-class tile prefix of one image group
    if (mode == MODE_FWD) row_tiles = NGI * a.sp.tile0[4];
  }
  // staged 16-byte row stores: channel-contiguous rows, 16-byte aligned, no beta
  const int vel = a.out_bf16 ? 8 : 4;
  a.vec_out = a.os[1] == 1 && a.beta == 0.f && a.os[0] % vel == 0 && a.os[2] % vel == 0 && a.os[3] % vel == 0 &&
              a.Ng % vel == 0 && ((uintptr_t)a.out & 15) == 0;
  a.sp_tpc = 0;
  a.sp_merge = 0;
  if (sp_weights && mode == MODE_FWD && g_ring256 && big && a.vec_out && a.ng >= 16 &&
      a.Ng % 64 == 0) {
    bool same = true;
    for (int c = 1; c < 4; ++c)
      same = same && a.sp.dh[c] == a.sp.dh[0] && a.sp.dw[c] == a.sp.dw[0] && a.sp.ph[c] == a.sp.ph[0] &&
             a.sp.pw[c] == a.sp.pw[0] && a.sp.oh[c] == a.sp.oh[0] && a.sp.ow[c] == a.sp.ow[0];
    if (same) {
      a.sp_merge = 1;
      row_tiles = NGI * a.sp.tile0[1];
    }
  }
  if (sp_weights && mode == MODE_FWD && !a.sp_merge) {
    for (int c = 0; c < 4; ++c) a.sp_tpc = std::max(a.sp_tpc, a.sp.tile0[c + 1] - a.sp.tile0[c]);
    row_tiles = NGI * 4 * a.sp_tpc;
  }
  // fused BatchNorm statistics (es_conv2d_fwd_stats): one [3][Ng] partial per row tile
  a.stats_part = nullptr;
  const int chunks = a.sp_merge ? 4 * row_tiles : row_tiles;
  if (mode == MODE_FWD && g_stats_req.part && a.vec_out && (int64_t)chunks * 3 * a.Ng <= g_stats_req.floats) {
    a.stats_part = g_stats_req.part;
    g_stats_req.chunks = chunks;
  }
  if (a.sp_merge) {   // (vec_out: the merged epilogue is the staged one)
    const int NT = 4 * a.Ng / 256;
    if (EB == 2 && g_p256 && (4 * a.Ng) % 256 == 0 && (NT == 1 || NT == 2 || NT == 4) && row_tiles >= 64 && a.out_bf16 &&
        (int64_t)d.N * a.os[0] * 2 < (1ll << 31)) {
      a.stats_part = nullptr;
      if (g_stats_req.part && (int64_t)256 * 4 * 3 * a.Ng <= g_stats_req.floats) {
        a.stats_part = g_stats_req.part;
        g_stats_req.chunks = 256 * 4;
      }
      ++g_conv_launches;
      if (NT == 1) hipLaunchKernelGGL((conv_p256_kernel<1>), dim3(256), dim3(RT), 0, st, a, row_tiles);
      else if (NT == 2) hipLaunchKernelGGL((conv_p256_kernel<2>), dim3(256), dim3(RT), 0, st, a, row_tiles);
      else hipLaunchKernelGGL((conv_p256_kernel<4>), dim3(256), dim3(RT), 0, st, a, row_tiles);
      return 1;
    }
    ++g_conv_launches;
    if constexpr (SPL == 2) {   // 256 x 128 tiles (a wave's 128 columns within one class) or 256 x 64
      if (a.Ng % 128 == 0) {
        dim3 grid(row_tiles, 4 * a.Ng / 128, 1);
        hipLaunchKernelGGL((conv_ring_kernel<MODE_FWD, 256, 128, true, 64, T, 2>), grid, dim3(RT), 0, st, a);
      } else {
        dim3 grid(row_tiles, 4 * a.Ng / 64, 1);
        hipLaunchKernelGGL((conv_ring_kernel<MODE_FWD, 256, 64, true, 64, T, 2>), grid, dim3(RT), 0, st, a);
      }
    } else if constexpr (SPL) {   // 256 x 256 tiles of 32-channel steps
      dim3 grid(row_tiles, (4 * a.Ng + 255) / 256, 1);
      hipLaunchKernelGGL((conv_ring_kernel<MODE_FWD, 256, 256, true, 64, T, 1>), grid, dim3(RT), 0, st, a);
    } else {
      dim3 grid(row_tiles, (4 * a.Ng + 255) / 256, 1);
      hipLaunchKernelGGL((conv_ring_kernel<MODE_FWD, 256, 256, true, 32, T>), grid, dim3(RT), 0, st, a);
    }
    return 1;
  }
#define ES_RING(MD, BMV, BNV)                                                                  \
  (sp_weights ? launch_ring<MD, BMV, BNV, true, 64, T, SPL>(a, row_tiles, st)                         \
              : launch_ring<MD, BMV, BNV, false, 64, T, SPL>(a, row_tiles, st))
  const bool wide = g_ring256 && big && !shortk && a.Ng >= 256 && a.ng >= 16 && a.vec_out &&
                    (sp_weights || mode == MODE_DGRAD);   // (plain FWD: register spills at 256 x 256)
  if constexpr (SPL == 1) if (wide) {   // split-fp32: 256 x 256 tiles of 32-channel steps
    if (mode == MODE_FWD) {   // (wide FWD is sub-pixel only)
      launch_ring<MODE_FWD, 256, 256, true, 64, T, 1>(a, row_tiles, st);
    } else {
      if (sp_weights) launch_ring<MODE_DGRAD, 256, 256, true, 64, T, 1>(a, row_tiles, st);
      else launch_ring<MODE_DGRAD, 256, 256, false, 64, T, 1>(a, row_tiles, st);
    }
    return 1;
  }
  if constexpr (SPL == 2) if (wide) {   // pre-split B: 256 x 128 tiles (256 x 256 does not fit the LDS)
    if (mode == MODE_FWD) launch_ring<MODE_FWD, 256, 128, true, 64, T, 2>(a, row_tiles, st);
    else if (sp_weights) launch_ring<MODE_DGRAD, 256, 128, true, 64, T, 2>(a, row_tiles, st);
    else launch_ring<MODE_DGRAD, 256, 128, false, 64, T, 2>(a, row_tiles, st);
    return 1;
  }
  if constexpr (!SPL) if (wide) {
    if (mode == MODE_FWD) {
      if (sp_weights) launch_ring<MODE_FWD, 256, 256, true, 32, T>(a, row_tiles, st);
      else launch_ring<MODE_FWD, 256, 256, false, 32, T>(a, row_tiles, st);
    } else {
      if (sp_weights) launch_ring<MODE_DGRAD, 256, 256, true, 32, T>(a, row_tiles, st);
      else launch_ring<MODE_DGRAD, 256, 256, false, 32, T>(a, row_tiles, st);
    }
    return 1;
  }
  if (mode == MODE_FWD) {
    if (a.Ng <= 64 || shortk) big ? ES_RING(MODE_FWD, 256, 64) : ES_RING(MODE_FWD, 128, 64);
    else big ? ES_RING(MODE_FWD, 256, 128) : ES_RING(MODE_FWD, 128, 128);
  } else {
    if (a.Ng <= 64 || shortk) big ? ES_RING(MODE_DGRAD, 256, 64) : ES_RING(MODE_DGRAD, 128, 64);
    else big ? ES_RING(MODE_DGRAD, 256, 128) : ES_RING(MODE_DGRAD, 128, 128);
  }
#undef ES_RING
  return 1;
}

// ---------------------------------------------------------------------------------------------
// fp32 (parity-mode) ring convolutions.  The ring's buffer offsets are 32-bit with an out-of-range
// marker at 2^31, so every gathered operand must stay below 1 GiB; larger fp32 batches
// (conv_layers.5's output gradient at B = 1024 is 1.1 GB) run as launches over image chunks on
// offset base pointers (chunks of whole 64-image groups).
// ---------------------------------------------------------------------------------------------
namespace {
int g_f32_chunk = 0;   // test knob (es_conv_set_f32_chunk): at most this many images per fp32 launch
// fp32 MFMA arithmetic of the ring kernels: 0 = exact fp32 (v_mfma_f32_16x16x4_f32), 1 = split-fp32
// (three bf16 planes, 6 products on v_mfma_f32_16x16x32_bf16); es_conv_set_f32_split / ES_F32_SPLIT
// (Plain functions, not lambdas: hipcc numbers the namespace-scope lambdas of a second anonymous
// namespace block from #1 again, and the duplicate symbols resolved to the first block's lambdas, so
// these globals were initialised by other variables' initialisers.)
int g_f32_split = 0;
// split-fp32 kernels: static s_setprio 1 for waves 4-7 (measured against 0: equal within noise, kept)
constexpr int SPL_PRIO = 1;
// images per launch: equal chunks (whole 64-image groups where the limit allows) below the limit
int chunk_images(int64_t img_bytes, int N) {
  int64_t lim = ((1ll << 30) - 1) / std::max<int64_t>(img_bytes, 1);
  if (g_f32_chunk > 0) lim = std::min<int64_t>(lim, g_f32_chunk);
  if (lim >= N) return N;
  lim = std::max<int64_t>(lim, 1);
  const int64_t nchunks = (N + lim - 1) / lim;
  int64_t nc = (N + nchunks - 1) / nchunks;
  if (nc % 64 && (nc + 63) / 64 * 64 <= lim) nc = (nc + 63) / 64 * 64;
  return (int)nc;
}
}  // namespace

namespace {
// bf16 ring launches over image chunks (es_conv_ring_launch): each chunk on offset base pointers
// with its first image as the dynamic-rows base; FWD statistics partials appended chunk after
// chunk; the fused BatchNorm-backward reduction of the persistent DGRAD is not offered to chunked
// launches (the caller runs the reduction pass).  WGRAD: the chunks' atomic accumulations into dW.
int ring_launch_chunks(ConvArgs& a, int mode, int nc, hipStream_t st) {
  const es_conv_desc_t& d = a.d;
  const int N = d.N;
  const int esz = a.out_bf16 ? 2 : 4;
  const StatsRequest req = g_stats_req;
  const BnRedRequest bnr = g_bnr_req;
  g_bnr_req.part = nullptr;
  int used = 0, rc = 1;
  bool stats_ok = req.part != nullptr;
  for (int n0 = 0; n0 < N; n0 += nc) {
    ConvArgs c = a;
    c.d.N = std::min(nc, N - n0);
    c.nbase = a.nbase + n0;
    c.a_src = (const char*)a.a_src + (int64_t)n0 * a.as[0] * 2;
    if (mode == MODE_WGRAD) {
      c.b_src = (const char*)a.b_src + (int64_t)n0 * a.bs[0] * 2;
      c.Kd = c.d.N * d.P * d.Q;
    } else {
      c.out = (char*)a.out + (int64_t)n0 * a.os[0] * esz;
      c.M = mode == MODE_FWD ? c.d.N * d.P * d.Q : (a.fold ? c.d.N * d.H * d.W : c.d.N * d.Hu * d.Wu);
    }
    if (req.part) g_stats_req = StatsRequest{req.part + (int64_t)used * 3 * a.Ng, req.floats - (int64_t)used * 3 * a.Ng, 0};
    rc = es_conv_ring_launch(c, mode, st);
    if (rc <= 0) {
      if (n0 > 0) {
        es_set_error("conv bf16 ring: image chunk at %d not eligible", n0);
        rc = -1;
      }
      break;
    }
    if (req.part) {
      stats_ok = stats_ok && g_stats_req.chunks > 0;
      used += g_stats_req.chunks;
    }
  }
  g_stats_req = StatsRequest{req.part, req.floats, rc > 0 && stats_ok ? used : 0};
  g_bnr_req = bnr;
  g_bnr_req.chunks = 0;
  return rc;
}
}  // namespace

// FWD / DGRAD: 1 launched, 0 not eligible (nothing launched), < 0 error
int es_conv_ring_launch_f32(ConvArgs& a, int mode, hipStream_t st) {
  const es_conv_desc_t& d = a.d;
  if (mode == MODE_WGRAD || d.hmap != nullptr || d.stride > 2 || a.splitk) return d.subpixel ? -1 : 0;
  const int N = d.N;
  const int ea = 4;   // bytes per value of the gathered operand
  const int nc = chunk_images(a.as[0] * ea, N);
  const int esz = a.out_bf16 ? 2 : 4;
  const StatsRequest req = g_stats_req;
  int used = 0;
  bool stats_ok = req.part != nullptr;
  for (int n0 = 0; n0 < N; n0 += nc) {
    ConvArgs c = a;
    c.d.N = std::min(nc, N - n0);
    c.nbase = a.nbase + n0;
    c.a_src = (const char*)a.a_src + (int64_t)n0 * a.as[0] * ea;
    c.out = (char*)a.out + (int64_t)n0 * a.os[0] * esz;
    c.M = mode == MODE_FWD ? c.d.N * d.P * d.Q : (a.fold ? c.d.N * d.H * d.W : c.d.N * d.Hu * d.Wu);
    if (req.part) g_stats_req = StatsRequest{req.part + (int64_t)used * 3 * a.Ng, req.floats - (int64_t)used * 3 * a.Ng, 0};
    c.prio = SPL_PRIO;
    const int rc = g_f32_split == 2 ? ring_fd<float, 2>(c, mode, st)
                   : g_f32_split ? ring_fd<float, 1>(c, mode, st) : ring_fd<float>(c, mode, st);
    if (rc <= 0) {
      g_stats_req = req;
      if (n0 == 0) return rc;
      es_set_error("conv f32 ring: chunk %d not eligible", n0);
      return -1;
    }
    if (req.part) {
      stats_ok = stats_ok && g_stats_req.chunks > 0;
      used += g_stats_req.chunks;
    }
  }
  g_stats_req = StatsRequest{req.part, req.floats, stats_ok ? used : 0};
  g_ring_hit = 1 | (g_f32_split ? 2 : 0) | (d.subpixel ? 4 : 0);
  return 1;
}

// WGRAD plan of the deterministic fp32 ring kernel: tile, image chunks, K splits per chunk
struct WgF32Plan {
  int bm, bn, sp, col, nc, nchunks, sc, ngt;
  SubPixel spg;
};
static bool wgrad_f32_plan(const es_conv_desc_t& d, const int64_t ys[4], const int64_t xs[4], WgF32Plan& p) {
  if (g_ring_off || d.hmap != nullptr || d.stride > 2) return false;
  auto dense = [](const int64_t s[4], int c, int h, int w) {
    return s[1] == 1 && s[3] == c && s[2] == (int64_t)w * c && s[0] == (int64_t)h * w * c;
  };
  if (!dense(ys, d.K, d.P, d.Q) || !dense(xs, d.C, d.H, d.W)) return false;
  if (d.K % 64 || d.C % 64) return false;
  p.bm = d.K % 128 == 0 ? 128 : 64;
  p.bn = d.C % 256 == 0 && p.bm == 128 ? 256 : (d.C % 128 == 0 ? 128 : 64);
  // split-fp32 with 64 output channels: 64 x 512 tiles (8 waves of 64 x 64, the per-wave shape of the
  // 128 x 256 tiles; 64 x 128 tiles make the in-kernel split VALU-bound)
  p.sp = !g_subpixel_off && d.up_h == 2 && d.up_w == 2 && d.stride == 1;
  if (g_f32_split && p.bm == 64 && !p.sp && (d.R * d.S * d.C) % 512 == 0) p.bn = 512;
  p.col = g_f32_split && !p.sp && d.R == 2 && d.S == 2 && d.stride == 1 && d.Hu == d.H &&
          d.Wu == d.W && d.C == 128 && d.K == 64;
  p.spg = SubPixel{};
  int npix = d.P * d.Q, taps = d.R * d.S;
  if (p.sp) {
    es_make_subpixel(d, 0, p.spg);
    taps = p.spg.tap0[4];
    npix = 0;
    for (int c = 0; c < 4; ++c) npix = std::max(npix, p.spg.ph[c] * p.spg.pw[c]);
  }
  p.ngt = taps * d.C;
  p.nc = chunk_images(std::max(ys[0], xs[0]) * 4, d.N);
  p.nchunks = (d.N + p.nc - 1) / p.nc;
  const int tiles = (d.K / p.bm) * (p.ngt / p.bn);
  const int ks = npix * ((p.nc + 31) / 32);   // K-steps of a full chunk (the largest class)
  // one round of 256 one-workgroup-per-CU tiles, >= 16 K-steps per split
  p.sc = std::max(1, std::min(256 / std::max(tiles, 1), ks / 16));
  return true;
}

int64_t es_wgrad_f32_ring_floats(const es_conv_desc_t& d, const int64_t ys[4], const int64_t xs[4]) {
  WgF32Plan p;
  if (!wgrad_f32_plan(d, ys, xs, p)) return -1;
  return (int64_t)p.nchunks * p.sc * d.K * p.ngt;
}

// launches the partial kernels and the reduce into dw (torch layout); 1 done, 0 not eligible
int es_wgrad_f32_ring(const es_conv_desc_t& d, const void* dy, const int64_t ys[4], const void* x,
                      const int64_t xs[4], float* dw, float beta, float* ws, int64_t ws_floats, hipStream_t st) {
  WgF32Plan p;
  if (!wgrad_f32_plan(d, ys, xs, p)) return 0;
  const int64_t need = (int64_t)p.nchunks * p.sc * d.K * p.ngt;
  if (ws == nullptr || ws_floats < need) {
    es_set_error("conv wgrad det: workspace of %lld floats, %lld needed", (long long)ws_floats, (long long)need);
    return -1;
  }
  for (int ch = 0; ch < p.nchunks; ++ch) {
    const int n0 = ch * p.nc;
    ConvArgs a{};
    a.d = d;
    a.prio = SPL_PRIO;
    a.d.N = std::min(p.nc, d.N - n0);
    a.nbase = n0;
    a.a_src = (const char*)dy + (int64_t)n0 * ys[0] * 4;
    a.b_src = (const char*)x + (int64_t)n0 * xs[0] * 4;
    for (int i = 0; i < 4; ++i) { a.as[i] = ys[i]; a.bs[i] = xs[i]; }
    a.fUh = mkdiv(d.up_h > 0 ? d.up_h : 1); a.fUw = mkdiv(d.up_w > 0 ? d.up_w : 1);
    a.M = d.K;
    a.sp = p.spg;
    int npix = d.P * d.Q;
    if (p.sp) { npix = 0; for (int c = 0; c < 4; ++c) npix = std::max(npix, p.spg.ph[c] * p.spg.pw[c]); }
    const int ks = p.col ? d.P * (d.Q + 1) * ((a.d.N + 31) / 32) : npix * ((a.d.N + 31) / 32);
    a.k_per_split = (ks + p.sc - 1) / p.sc;
    float* wsc = ws + (int64_t)ch * p.sc * d.K * p.ngt;
    dim3 grid(d.K / p.bm, p.ngt / p.bn, p.sc);
    if (p.col) {
      ++g_conv_launches;
      hipLaunchKernelGGL(wgrad_f32_col2_kernel, grid, dim3(RT), 0, st, a, wsc, p.ngt);
      continue;
    }
    if (g_f32_split && p.bm == 128) {
      ++g_conv_launches;
#define ES_WC(BN)                                                                                          \
  do {                                                                                                     \
    if (g_wgrad_ws && es_wgrad_ws_launch(BN, p.sp, grid, a, wsc, p.ngt, st) == 1) {                       \
    } else if (p.sp) hipLaunchKernelGGL((wgrad_coop_kernel<128, BN, true>), grid, dim3(RT), 0, st, a, wsc, p.ngt); \
    else hipLaunchKernelGGL((wgrad_coop_kernel<128, BN, false>), grid, dim3(RT), 0, st, a, wsc, p.ngt);     \
  } while (0)
      if (p.bn == 256) ES_WC(256);
      else if (p.bn == 128) ES_WC(128);
      else ES_WC(64);
#undef ES_WC
      continue;
    }
#define ES_WF(BM, BN)                                                                                 \
  do {                                                                                                \
    ++g_conv_launches;                                                                                \
    if (g_f32_split && (BM == 128 || BN == 512)) {  /* (64 x 128 tiles: VALU-bound split,      */    \
                                      /*  1.59 ms vs 1.41 exact for conv_layers.9 at B = 1024)   */    \
      if (p.sp) hipLaunchKernelGGL((wgrad_f32_kernel<BM, BN, true, true>), grid, dim3(RT), 0, st, a, wsc, p.ngt); \
      else hipLaunchKernelGGL((wgrad_f32_kernel<BM, BN, false, true>), grid, dim3(RT), 0, st, a, wsc, p.ngt);    \
    } else if (p.sp) hipLaunchKernelGGL((wgrad_f32_kernel<BM, BN, true>), grid, dim3(RT), 0, st, a, wsc, p.ngt); \
    else hipLaunchKernelGGL((wgrad_f32_kernel<BM, BN, false>), grid, dim3(RT), 0, st, a, wsc, p.ngt);       \
  } while (0)
    if (p.bm == 128 && p.bn == 256) ES_WF(128, 256);
    else if (p.bm == 128 && p.bn == 128) ES_WF(128, 128);
    else if (p.bm == 128) ES_WF(128, 64);
    else if (p.bn == 512) {   // (planned for split-fp32 without sub-pixel classes only)
      ++g_conv_launches;
      hipLaunchKernelGGL((wgrad_f32_kernel<64, 512, false, true>), grid, dim3(RT), 0, st, a, wsc, p.ngt);
    }
    else if (p.bn == 128) ES_WF(64, 128);
    else ES_WF(64, 64);
#undef ES_WF
  }
  launch_wgrad_reduce(ws, p.nchunks * p.sc, d.K, d.C, d.R, d.S, p.ngt, p.spg, dw, beta, st);
  g_ring_hit = 1 | (g_f32_split ? 2 : 0) | (p.sp ? 4 : 0);
  return 1;
}

// reduce of generic per-split partials ws[split][K][R*S*C] (conv_igemm / thin WGRAD, deterministic
// mode) into dW (torch layout)
void es_wgrad_reduce_plain(const float* ws, int splits, int K, int C, int R, int S, float* dw, float beta,
                           hipStream_t st) {
  SubPixel none{};
  launch_wgrad_reduce(ws, splits, K, C, R, S, R * S * C, none, dw, beta, st);
}

extern "C" int es_conv_set_f32_chunk(int images) {
  const int old = g_f32_chunk;
  g_f32_chunk = images > 0 ? images : 0;
  return old;
}

extern "C" int es_conv_set_wgrad_ws(int on) {
  const int old = g_wgrad_ws;
  g_wgrad_ws = on ? 1 : 0;
  return old;
}

extern "C" int es_conv_set_f32_split(int on) {
  const int old = g_f32_split;
  g_f32_split = on < 0 ? 0 : (on > 2 ? 2 : on);
  return old;
}
