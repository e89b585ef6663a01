// The wave-specialised split-fp32 weight gradient (conv_layers.0 / .5 of the neutron generator,
// neutron/generator.py:24,29, and the other 128-row split-fp32 WGRAD tiles).
#include "conv_common.h"
#include "ring_common.h"
#include "split_fp32.h"

namespace {

constexpr int RT = 512;

// Split-fp32 WGRAD, WAVE-SPECIALISED (BM = 128).  In wgrad_coop_kernel every wave loads, splits and
// multiplies, and the one barrier per K-step keeps the two waves of a SIMD in the same phase: both
// issue their loads, both want the matrix pipe, both split -- the pipe idles through the VALU phase
// (PMC: bf16-pipe busy 0.51).  Here the roles are separate: waves 0-3 (one per SIMD) only read
// fragments and issue MFMAs (wave tile 64 x BN/2, accumulators in registers), waves 4-7 (the
// other wave of each SIMD) only load, split and write the planes, two K-steps ahead in registers.
// A SIMD's matrix pipe is fed by one wave while its partner's vector work runs beside it; the
// barrier per step only hands the planes over.  Same LDS plane layout ([plane][16-row block][lane]
// [8 k-values]), K order, products and partial slots as wgrad_coop_kernel: bitwise the same result.
// A producer lane loads the 8 k-values of its own 16-byte fragment slot, so each plane of a block
// is one ds_write_b128 (no bank conflicts; the coop kernel's 8-byte stores conflicted 2-way).
// Measured (B = 1024, conv_layers.5, tools/mb_ab.py / gpu_pmc_ab.sh): 1584 -> 1395 us per launch,
// bf16-pipe busy 0.51 -> 0.62; conv_layers.0 1.23 -> 1.16 ms per op.  What bounds it now (removal
// builds): the consumers alone (producers loading nothing) 2.66 ms per op, the producers alone
// (consumers issuing no MFMA) 2.71 -- an MFMA holds its SIMD's vector issue for 8 of its 16 cycles
// (MI355X_MICROARCH.md), and the split (~5.5 VALU per value) plus the running-sum adds fill the rest.
// Tried, not kept: 8 consumer waves + 4 producers (12-wave workgroups): equal (0.63); scalar
// instead of packed running-sum adds: equal.
template <int BN, bool SP>
__global__ void __launch_bounds__(RT) wgrad_ws_kernel(ConvArgs a, float* __restrict__ ws, int ngt) {
  constexpr int BM = 128, KI = 32;
  // 4 consumer waves (waves 0-3, 2 x 2) and 4 producer waves: a workgroup's waves w and w + 4 share
  // a SIMD, so each SIMD runs one of each
  constexpr int NCW = 4, WGN = NCW / 2;
  constexpr int WM = 64, WN = BN / WGN, RM = WM / 16, RN = WN / 16;   // consumer wave tile
  static_assert(RN >= 1, "consumer wave tiles of >= 16 columns");
  constexpr int NBA = BM / 16, NB = (BM + BN) / 16;                 // 16-row blocks: A's, A's and B's
  constexpr int NBP = NB / 4, NBPA = NBA / 4;                       // blocks per producer wave (A first)
  static_assert(NB % 4 == 0 && NBA % 4 == 0, "blocks split evenly over 4 producer waves");
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
  const int nk = tend - tbeg;

  const int lane = threadIdx.x & 63, wid = uni(threadIdx.x >> 6);
  const int col16 = lane & 15, rq = (lane >> 4) * 4, kl = lane >> 4;
  const auto sync = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ring_barrier();
  };

  if (wid >= NCW) {
    // ---------------- producers: global -> registers (two steps ahead) -> split -> LDS planes
    if (nk <= 0) return;
    const int pw = wid - NCW;
    const __amdgpu_buffer_rsrc_t ares = mkres(a.a_src, (uint32_t)(NL * a.as[0] * 4));
    const __amdgpu_buffer_rsrc_t bres = mkres(a.b_src, (uint32_t)(NL * a.bs[0] * 4));
    const int as0b = (int)a.as[0] * 4, as2b = (int)a.as[2] * 4, as3b = (int)a.as[3] * 4;
    const int bs0b = (int)a.bs[0] * 4, bs2b = (int)a.bs[2] * 4, bs3b = (int)a.bs[3] * 4;
    // block h of this wave: b = 4 h + pw; the lane loads row / column 16 b + col16 at the step's
    // images 4 m + kl, m = 0..7 -- exactly the 8 k-values of its own 16-byte fragment slot, so each
    // plane is ONE ds_write_b128 per block (one wave per SIMD reaches the LDS rate with 16-byte
    // stores; 8-byte stores need ~4 waves per SIMD, MI355X_MICROARCH.md LDS table)
    uint32_t lofs[NBP];
#pragma unroll
    for (int h = 0; h < NBP; ++h) {
      const int blk = 4 * h + pw;
      if (h < NBPA) lofs[h] = (uint32_t)(kl * as0b + (m0 + 16 * blk + col16) * 4);
      else lofs[h] = (uint32_t)(kl * bs0b + (cb + 16 * (blk - NBA) + col16) * 4);
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
    typedef float Stage[NBP][8];
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
      for (int h = 0; h < NBP; ++h)
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const uint32_t o = h < NBPA ? ua + lofs[h] + m * 4 * as0b : ub + lofs[h] + m * 4 * bs0b;
          v[h][m] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(h < NBPA ? ares : bres,
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
      for (int h = 0; h < NBP; ++h) {
        uint32_t hi[4], mi[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split_pair(v[h][2 * q], v[h][2 * q + 1], hi[q], mi[q], lo[q]);
        char* dst = pb + (4 * h + pw) * 1024 + lane * 16;
        *(u32x4_t*)dst = u32x4_t{hi[0], hi[1], hi[2], hi[3]};
        *(u32x4_t*)(dst + PLANE) = u32x4_t{mi[0], mi[1], mi[2], mi[3]};
        *(u32x4_t*)(dst + 2 * PLANE) = u32x4_t{lo[0], lo[1], lo[2], lo[3]};
      }
    };
    Stage s0, s1;
    load(s0);                               // step 0
    load(s1);                               // step 1
    wait_vmcnt<NBP * 8>();
    store(s0, smem);
    sync();                                 // planes of step 0 published
    for (int t = 0; t < nk; t += 2) {
      // even t: step t + 1 sits in s1, step t + 2 goes into s0; odd: the roles swap (unrolled by two
      // so that the stages stay in fixed registers)
      load(s0);                             // step t + 2 (s0 held step t, stored one step ago)
      wait_vmcnt<NBP * 8>();                // step t + 1 landed
      store(s1, smem + PBUF);               // buffer 1, last read by the consumers in step t - 1
      sync();
      if (t + 1 >= nk) break;
      load(s1);                             // step t + 3
      wait_vmcnt<NBP * 8>();                // step t + 2 landed
      store(s0, smem);
      sync();
    }
    wait_vmcnt<0>();
    return;
  }

  // ---------------- consumers: fragments from LDS -> MFMA (one wave per SIMD)
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0) {
    const char* q0 = smem + lane * 16;
    auto rd = [&](bf16x8 (&f)[3], const char* pb, int blk) {
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *(const bf16x8*)(pb + p * PLANE + blk * 1024);
    };
    // six plane products of fragment pair (i, j) into a fresh accumulator (mfma_split6's order)
    auto chain = [&](const bf16x8 (&x)[3], const bf16x8 (&y)[3]) {
      f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[2], y[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], y[1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[2], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], y[0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[1], c, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[0], c, 0, 0, 0);
    };
    auto compute = [&](const char* pb) {
      bf16x8 ap[RM][3], bp[2][3];
      // the first pair's fragments first: its MFMAs wait for 6 reads, not for the whole A panel
      rd(ap[0], pb, wm0 / 16);
      rd(bp[0], pb, NBA + wn0 / 16);
#pragma unroll
      for (int i = 1; i < RM; ++i) rd(ap[i], pb, wm0 / 16 + i);
      // each pair's fresh sum is added to the running sum one pair later, under the next pair's
      // MFMAs (added right after its own chain, the wave waits out the last MFMA's latency with the
      // matrix pipe idle); same adds, same values
      f32x4 cprev;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        if (j + 1 < RN) rd(bp[(j + 1) & 1], pb, NBA + wn0 / 16 + j + 1);
#pragma unroll
        for (int i = 0; i < RM; ++i) {
          const f32x4 c = chain(ap[i], bp[j & 1]);
          if (i + j > 0) {
            const int pi = i == 0 ? RM - 1 : i - 1, pj = i == 0 ? j - 1 : j;
            acc[pi][pj] = acc[pi][pj] + cprev;
          }
          cprev = c;
        }
      }
      acc[RM - 1][RN - 1] = acc[RM - 1][RN - 1] + cprev;
    };
    sync();                                 // planes of step 0
    for (int t = 0; t < nk; ++t) {
      compute(q0 + (t & 1) * PBUF);
      sync();                               // done reading; planes of step t + 1 published
    }
  }
  float* o = ws + ((int64_t)split * a.M + m0 + wm0) * ngt + n0 + wn0 + col16;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int j = 0; j < RN; ++j) o[(int64_t)(i * 16 + rq + jj) * ngt + j * 16] = acc[i][j][jj];
}

}  // namespace

// 1 launched, 0 not eligible
int es_wgrad_ws_launch(int bn, bool sp, dim3 grid, const ConvArgs& a, float* wsc, int ngt, hipStream_t st) {
#define ES_WS(BN)                                                                                    \
  do {                                                                                               \
    if (sp) hipLaunchKernelGGL((wgrad_ws_kernel<BN, true>), grid, dim3(RT), 0, st, a, wsc, ngt);      \
    else hipLaunchKernelGGL((wgrad_ws_kernel<BN, false>), grid, dim3(RT), 0, st, a, wsc, ngt);        \
  } while (0)
  if (bn == 256) ES_WS(256);
  else if (bn == 128) ES_WS(128);
  else if (bn == 64) ES_WS(64);
  else return 0;
#undef ES_WS
  return 1;
}
