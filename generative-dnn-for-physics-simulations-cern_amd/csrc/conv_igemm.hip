// Implicit-GEMM convolution (and linear) forward / dgrad / wgrad on gfx950 MFMA.
//
// Replaces aten::convolution, aten::convolution_backward and aten::addmm/mm for every nn.Conv2d
// and nn.Linear on the expertsim hot path (see include/expertsim_hip.h for the call sites).
//
// GEMM views (one kernel template, three operand gathers):
//   FWD   : M = N*P*Q (output pixels), Ng = K (out channels), Kd = R*S*C  (c fastest)
//           A[m][kk] = xu[n, c, p*st-pad+r, q*st-pad+s]    B[ng][kk] = Wk[k][r][s][c]
//   DGRAD : M = N*Hu*Wu (upsampled input pixels), Ng = C, Kd = R*S*K (k fastest)
//           A[m][kk] = dy[n, k, (hu+pad-r)/st, (wu+pad-s)/st] (0 unless divisible / in range)
//           B[ng][kk] = Wd[c][r][s][k]
//   WGRAD : M = K, Ng = R*S*C, Kd = N*P*Q (split over blockIdx.z, fp32 atomics)
//           A[m][kk] = dy[pix][k]                        B[ng][kk] = xu[pix shifted by (r,s)][c]
// The nearest upsample of the generators (neutron/generator.py:23,29; proton/generator.py:26,32)
// is folded into the x gather through hmap/wmap (up row -> source row).
//
// Tiling: 256 threads = 4 waves in a 2x2 grid, block tile BM x BN, K-step = 128 bytes of operand
// per row (bf16: 64, fp32: 32).  LDS holds both operands K-contiguous ([row][k], 144-byte padded
// rows -> conflict-free 16-byte fragment reads), double buffered; global->register->LDS staging
// with the next tile's loads issued before the current tile's MFMAs.
//   bf16 : v_mfma_f32_16x16x32_bf16, lane l reads A[l&15][8*(l>>4)+0..7] as one 16-byte read
//   fp32 : v_mfma_f32_16x16x4_f32 x4, lane l reads A[l&15][4*(l>>4)+0..3] once and feeds the
//          four MFMAs with k = 4*(l>>4)+t (A and B use the same permutation of k, so the sum over
//          k is unchanged; each MFMA is an exact fp32 FMA chain).
#include <algorithm>
#include <cstdlib>

#include "conv_common.h"

// direct kernels for one-input-channel / one-output-channel convolutions (conv_thin.hip)
int es_thin_conv_fwd(const es_conv_desc_t* d, es_dtype_t dt, const void* x, const int64_t xs[4], const void* wk,
                     const float* bias, void* y, es_dtype_t ydt, const int64_t ys[4], hipStream_t st);
int es_thin_conv_dgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                       const void* wd, void* dx, es_dtype_t dxdt, const int64_t dxs[4], float beta,
                       hipStream_t st);
int es_thin_conv_wgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4], const void* x,
                       const int64_t xs[4], float* dw, hipStream_t st);

namespace {


// es_conv_set_glds(0) forces the register-staged kernels (tests compare the paths)
bool g_no_glds = false;

constexpr int KSTEP_BYTES = 128;               // operand bytes per row per K-step
constexpr int ROW_BYTES = KSTEP_BYTES + 16;    // padded LDS row
constexpr int NTHREADS = 256;

// LDS image of one operand for one K-step.
//  default : [rows][k] K-contiguous, 144-byte rows (fragments read with 16-byte ds_read)
//  TR      : bf16 WGRAD operands, whose global data is contiguous along the GEMM row (m / n):
//            [k][rows] row-contiguous image written with 16-byte stores (no transpose in
//            registers) and read with ds_read_b64_tr_b16 (gfx950 transposing LDS read).
//            Row stride = rows*2 + 32 bytes, and k-rows with bit 3 set XOR their byte column by
//            rows bytes, so the two 16-lane groups of a half-wave (k rows 8 apart) hit disjoint
//            banks.
template <typename T, int MODE, int BROWS>
struct LdsImg {
  static constexpr bool TR = (MODE == 2) && sizeof(T) == 2;
  static constexpr int BK = KSTEP_BYTES / sizeof(T);
  static constexpr int ROWB = TR ? BROWS * 2 + 32 : ROW_BYTES;
  static constexpr int BYTES = TR ? BK * ROWB : BROWS * ROW_BYTES;
  __device__ static __forceinline__ int tr_off(int k, int row) {   // byte offset of (k, row)
    return k * ROWB + ((row * 2) ^ (((k >> 3) & 1) * BROWS));
  }
};

__device__ __forceinline__ int src_row(const int32_t* map, int u) { return map ? map[u] : u; }
// nearest-upsample source index of upsampled row / column u
__device__ __forceinline__ int src_h(const ConvArgs& a, int u) {
  return a.d.up_h > 0 ? fdiv(u, a.fUh) : src_row(a.d.hmap, u);
}
__device__ __forceinline__ int src_w(const ConvArgs& a, int u) {
  return a.d.up_w > 0 ? fdiv(u, a.fUw) : src_row(a.d.wmap, u);
}

template <typename T> struct Vec16;
template <> struct Vec16<float> { typedef float4 type; static constexpr int N = 4; };
template <> struct Vec16<bf16> { typedef uint4 type; static constexpr int N = 8; };



// ---------------------------------------------------------------------------------------------
// Element gathers (scalar); used by the generic path and by the vector path for the base address
// ---------------------------------------------------------------------------------------------
// a Linear as a 1x1 conv of 1x1 images: rows m = sample, kk = feature (the generic decomposition
// below costs 8 integer divisions per element, ~30 us per launch for the small linears)
__device__ __forceinline__ bool is_linear(const ConvArgs& a) {
  const es_conv_desc_t& d = a.d;
  return d.R == 1 && d.S == 1 && d.P == 1 && d.Q == 1 && d.Hu == 1 && d.Wu == 1 && d.stride == 1 && d.pad == 0 &&
         !a.fold && d.hmap == nullptr;
}

template <typename T, int MODE>
__device__ __forceinline__ float gather_a(const ConvArgs& a, int m, int kk) {
  const es_conv_desc_t& d = a.d;
  const T* src = (const T*)a.a_src;
  if (is_linear(a)) {   // branch-free: clamped index + select (the loads of a chunk issue together)
    const bool ok = m < a.M && kk < a.Kd;
    int64_t i;
    if constexpr (MODE == MODE_WGRAD) i = (int64_t)kk * a.as[0] + (int64_t)m * a.as[1];
    else i = (int64_t)m * a.as[0] + (int64_t)kk * a.as[1];
    const float v = to_f(src[ok ? i : 0]);
    return ok ? v : 0.f;
  }
  if (m >= a.M || kk >= a.Kd) return 0.f;
  if constexpr (MODE == MODE_FWD) {
    const int c = kk % d.C; const int rs = kk / d.C; const int s = rs % d.S; const int r = rs / d.S;
    const int q = m % d.Q; const int np = m / d.Q; const int p = np % d.P; const int n = np / d.P;
    const int hu = p * d.stride - d.pad + r, wu = q * d.stride - d.pad + s;
    if (hu < 0 || hu >= d.Hu || wu < 0 || wu >= d.Wu) return 0.f;
    return to_f(src[off4(a.as, n, c, src_h(a, hu), src_w(a, wu))]);
  } else if constexpr (MODE == MODE_DGRAD) {
    int kr = kk, hu, wu, n;
    if (a.fold) {   // rows on the source grid, kk = (a, b, r, s, k)
      const int ab = kk / (d.R * d.S * d.K);
      kr = kk - ab * (d.R * d.S * d.K);
      const int ua = ab / d.up_w, ub = ab - ua * d.up_w;
      const int j = m % d.W; const int nh = m / d.W; const int i = nh % d.H; n = nh / d.H;
      hu = i * d.up_h + ua; wu = j * d.up_w + ub;
    } else {
      wu = m % d.Wu; const int nh = m / d.Wu; hu = nh % d.Hu; n = nh / d.Hu;
    }
    const int k = kr % d.K; const int rs = kr / d.K; const int s = rs % d.S; const int r = rs / d.S;
    const int ph = hu + d.pad - r, pw = wu + d.pad - s;
    if (ph < 0 || pw < 0 || ph % d.stride || pw % d.stride) return 0.f;
    const int p = ph / d.stride, q = pw / d.stride;
    if (p >= d.P || q >= d.Q) return 0.f;
    return to_f(src[off4(a.as, n, k, p, q)]);
  } else {  // WGRAD: A[m=k][kk=pix]
    const int q = kk % d.Q; const int np = kk / d.Q; const int p = np % d.P; const int n = np / d.P;
    return to_f(src[off4(a.as, n, m, p, q)]);
  }
}

template <typename T, int MODE>
__device__ __forceinline__ float gather_b(const ConvArgs& a, int ng, int kk) {
  const es_conv_desc_t& d = a.d;
  const T* src = (const T*)a.b_src;
  if (is_linear(a)) {
    const bool ok = ng < a.Ng && kk < a.Kd;
    int64_t i;
    if constexpr (MODE == MODE_WGRAD) i = (int64_t)kk * a.bs[0] + (int64_t)ng * a.bs[1];
    else i = (int64_t)ng * a.Kd + kk;   // packed weights (no upsample fold for a linear)
    const float v = to_f(src[ok ? i : 0]);
    return ok ? v : 0.f;
  }
  if (ng >= a.Ng || kk >= a.Kd) return 0.f;
  if constexpr (MODE == MODE_FWD) {
    return to_f(src[(int64_t)ng * a.Kd + kk]);
  } else if constexpr (MODE == MODE_DGRAD) {
    const int rsk = d.R * d.S * d.K;
    return to_f(src[(int64_t)ng * rsk + (a.fold ? kk % rsk : kk)]);
  } else {  // WGRAD: B[ng=(r,s,c)][kk=pix] = xu
    const int c = ng % d.C; const int rs = ng / d.C; const int s = rs % d.S; const int r = rs / d.S;
    const int q = kk % d.Q; const int np = kk / d.Q; const int p = np % d.P; const int n = np / d.P;
    const int hu = p * d.stride - d.pad + r, wu = q * d.stride - d.pad + s;
    if (hu < 0 || hu >= d.Hu || wu < 0 || wu >= d.Wu) return 0.f;
    return to_f(src[off4(a.bs, n, c, src_h(a, hu), src_w(a, wu))]);
  }
}

// ---------------------------------------------------------------------------------------------
// Tile staging.  A "chunk" is 16 bytes of one LDS row (VEC elements along k).
//   K-contiguous operands (FWD/DGRAD A, FWD/DGRAD B): a chunk = VEC consecutive kk of one row.
//   WGRAD operands: global data is contiguous along m / ng, so a chunk holds VEC consecutive rows
//   of one kk and is scattered into LDS element by element (transposing store).
// ---------------------------------------------------------------------------------------------
template <typename T, int MODE, int BROWS, bool IS_A, bool VEC>
struct Stager {
  typedef typename Vec16<T>::type V;
  static constexpr int VN = Vec16<T>::N;
  static constexpr int BK = KSTEP_BYTES / sizeof(T);
  static constexpr int CPR = KSTEP_BYTES / 16;          // chunks per LDS row (K-contiguous image)
  static constexpr int CHUNKS = BROWS * CPR;
  static constexpr int PER_THREAD = CHUNKS / NTHREADS;
  static constexpr bool TRANS = (MODE == MODE_WGRAD);
  V reg[PER_THREAD];
  // per-chunk state precomputed once per block (vector path): a base offset and two coordinates
  int64_t boff[PER_THREAD];
  int c0_[PER_THREAD], c1_[PER_THREAD];

  // --------------------------------------------------------------- precomputation (vector path)
  __device__ __forceinline__ void init(const ConvArgs& a, int row0) {
    if constexpr (!VEC) return;
    const es_conv_desc_t& d = a.d;
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int idx = threadIdx.x + i * NTHREADS;
      if constexpr (!TRANS) {
        const int row = row0 + idx / CPR;
        if constexpr (IS_A) {
          const int rr = row < a.M ? row : 0;
          if constexpr (MODE == MODE_FWD) {       // row = (n, p, q)
            const int np = fdiv(rr, a.fQ), q = rr - np * d.Q;
            const int n = fdiv(np, a.fP), p = np - n * d.P;
            boff[i] = row < a.M ? (int64_t)n * a.as[0] : -1;
            c0_[i] = p * d.stride - d.pad;
            c1_[i] = q * d.stride - d.pad;
          } else if (a.fold) {                      // DGRAD, folded upsample: row = (n, i, j) source grid
            const int nh = fdiv(rr, a.fW), j = rr - nh * d.W;
            const int n = fdiv(nh, a.fH), ii = nh - n * d.H;
            boff[i] = row < a.M ? (int64_t)n * a.as[0] : -1;
            c0_[i] = ii * d.up_h + d.pad;
            c1_[i] = j * d.up_w + d.pad;
          } else {                                  // DGRAD: row = (n, hu, wu)
            const int nh = fdiv(rr, a.fWu), wu = rr - nh * d.Wu;
            const int n = fdiv(nh, a.fHu), hu = nh - n * d.Hu;
            boff[i] = row < a.M ? (int64_t)n * a.as[0] : -1;
            c0_[i] = hu + d.pad;
            c1_[i] = wu + d.pad;
          }
        } else {
          const int ldb = (MODE == MODE_DGRAD && a.fold) ? d.R * d.S * d.K : a.Kd;
          boff[i] = row < a.Ng ? (int64_t)row * ldb : -1;
          c0_[i] = c1_[i] = 0;
        }
      } else {
        const int row = row0 + (idx % (BROWS / VN)) * VN;
        if constexpr (IS_A) {                       // WGRAD A: m = out channel
          boff[i] = row < a.M ? (int64_t)row * a.as[1] : -1;
          c0_[i] = c1_[i] = 0;
        } else {                                    // WGRAD B: ng = (r, s, c)
          const int rr = row < a.Ng ? row : 0;
          const int rs = fdiv(rr, a.fC), c = rr - rs * d.C;
          const int r = fdiv(rs, a.fS), s_ = rs - r * d.S;
          boff[i] = row < a.Ng ? (int64_t)c * a.bs[1] : -1;
          c0_[i] = r - d.pad;
          c1_[i] = s_ - d.pad;
        }
      }
    }
  }

  __device__ __forceinline__ void load(const ConvArgs& a, int row0, int k0) {
    if constexpr (VEC) {
      load_vec(a, k0);
    } else {
#pragma unroll
      for (int i = 0; i < PER_THREAD; ++i) {
        const int idx = threadIdx.x + i * NTHREADS;
        int row, kk;
        if constexpr (!TRANS) {
          row = row0 + idx / CPR;
          kk = k0 + (idx % CPR) * VN;
        } else {
          row = row0 + (idx % (BROWS / VN)) * VN;
          kk = k0 + idx / (BROWS / VN);
        }
        reg[i] = fetch_scalar(a, row, kk);
      }
    }
  }

  __device__ __forceinline__ V fetch_scalar(const ConvArgs& a, int row, int kk) {
    T e[VN];
#pragma unroll
    for (int j = 0; j < VN; ++j) {
      float f;
      if constexpr (!TRANS) f = IS_A ? gather_a<T, MODE>(a, row, kk + j) : gather_b<T, MODE>(a, row, kk + j);
      else f = IS_A ? gather_a<T, MODE>(a, row + j, kk) : gather_b<T, MODE>(a, row + j, kk);
      e[j] = from_f<T>(f);
    }
    V v; memcpy(&v, e, sizeof(v)); return v;
  }

  // vector path: the vector dimension is contiguous and VN-divisible (checked on the host)
  __device__ __forceinline__ void load_vec(const ConvArgs& a, int k0) {
    const es_conv_desc_t& d = a.d;
    const T* src = IS_A ? (const T*)a.a_src : (const T*)a.b_src;
    if constexpr (!TRANS) {
      const int kk = k0 + (int)(threadIdx.x % CPR) * VN;   // same column for all chunks
      const bool kin = kk < a.Kd;
      if constexpr (IS_A) {
        // kk -> (r, s, ch): ch = input channel (FWD) / output channel (DGRAD), fastest
        const FastDiv fch = MODE == MODE_FWD ? a.fC : a.fK;
        const int nch = MODE == MODE_FWD ? d.C : d.K;
        int kr = kk, ua = 0, ub = 0;
        if (MODE == MODE_DGRAD && a.fold) {        // kk = (phase a, phase b, r, s, k)
          const int ab = fdiv(kk, a.fRSK);
          kr = kk - ab * (d.R * d.S * d.K);
          ua = fdiv(ab, a.fUw); ub = ab - ua * d.up_w;
        }
        const int rs = fdiv(kr, fch), ch = kr - rs * nch;
        const int r = fdiv(rs, a.fS), s_ = rs - r * d.S;
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i) {
          const T* p = nullptr;
          if (kin && boff[i] >= 0) {
            if constexpr (MODE == MODE_FWD) {
              const int hu = c0_[i] + r, wu = c1_[i] + s_;
              if (hu >= 0 && hu < d.Hu && wu >= 0 && wu < d.Wu)
                p = src + boff[i] + (int64_t)ch * a.as[1] + (int64_t)src_h(a, hu) * a.as[2] +
                    (int64_t)src_w(a, wu) * a.as[3];
            } else {
              int ph = c0_[i] + ua - r, pw = c1_[i] + ub - s_;
              bool ok = ph >= 0 && pw >= 0;
              if (d.stride == 2) { ok = ok && !(ph & 1) && !(pw & 1); ph >>= 1; pw >>= 1; }
              if (ok && ph < d.P && pw < d.Q)
                p = src + boff[i] + (int64_t)ch * a.as[1] + (int64_t)ph * a.as[2] + (int64_t)pw * a.as[3];
            }
          }
          reg[i] = p ? *(const V*)p : V{};
        }
      } else {
        int kb = kk;
        if (MODE == MODE_DGRAD && a.fold) kb = kk - fdiv(kk, a.fRSK) * (d.R * d.S * d.K);
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i)
          reg[i] = (kin && boff[i] >= 0) ? *(const V*)(src + boff[i] + kb) : V{};
      }
    } else {
#pragma unroll
      for (int i = 0; i < PER_THREAD; ++i) {
        const int idx = threadIdx.x + i * NTHREADS;
        const int kk = k0 + idx / (BROWS / VN);                 // pixel (n, p, q)
        const T* p = nullptr;
        if (kk < a.Kd && boff[i] >= 0) {
          const int np = fdiv(kk, a.fQ), q = kk - np * d.Q;
          const int n = fdiv(np, a.fP), pp = np - n * d.P;
          if constexpr (IS_A) {
            p = src + boff[i] + (int64_t)n * a.as[0] + (int64_t)pp * a.as[2] + (int64_t)q * a.as[3];
          } else {
            const int hu = pp * d.stride + c0_[i], wu = q * d.stride + c1_[i];
            if (hu >= 0 && hu < d.Hu && wu >= 0 && wu < d.Wu)
              p = src + boff[i] + (int64_t)n * a.bs[0] + (int64_t)src_h(a, hu) * a.bs[2] +
                  (int64_t)src_w(a, wu) * a.bs[3];
          }
        }
        reg[i] = p ? *(const V*)p : V{};
      }
    }
  }

  __device__ __forceinline__ void store(char* lds) {
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int idx = threadIdx.x + i * NTHREADS;
      if constexpr (!TRANS) {
        const int row = idx / (KSTEP_BYTES / 16), ch = idx % (KSTEP_BYTES / 16);
        *(V*)(lds + row * ROW_BYTES + ch * 16) = reg[i];
      } else if constexpr (LdsImg<T, MODE, BROWS>::TR) {
        const int row = (idx % (BROWS / VN)) * VN, kk = idx / (BROWS / VN);
        *(V*)(lds + LdsImg<T, MODE, BROWS>::tr_off(kk, row)) = reg[i];
      } else {
        const int row = (idx % (BROWS / VN)) * VN, kk = idx / (BROWS / VN);
        T e[VN];
        memcpy(e, &reg[i], sizeof(e));
#pragma unroll
        for (int j = 0; j < VN; ++j) *(T*)(lds + (row + j) * ROW_BYTES + kk * sizeof(T)) = e[j];
      }
    }
  }
};

// ---------------------------------------------------------------------------------------------
// MFMA micro-kernel on one K-step held in LDS
// ---------------------------------------------------------------------------------------------
template <typename T, int RM, int RN>
__device__ __forceinline__ void mma_kstep(const char* As, const char* Bs, int wm0, int wn0,
                                          f32x4 (&acc)[RM][RN]) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int seg = kk * 4 + g;
    if constexpr (sizeof(T) == 2) {
      bf16x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(As + (wm0 + i * 16 + r16) * ROW_BYTES + seg * 16);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = *(const bf16x8*)(Bs + (wn0 + j * 16 + r16) * ROW_BYTES + seg * 16);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
      float4 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const float4*)(As + (wm0 + i * 16 + r16) * ROW_BYTES + seg * 16);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = *(const float4*)(Bs + (wn0 + j * 16 + r16) * ROW_BYTES + seg * 16);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].x, bfr[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].y, bfr[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].z, bfr[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].w, bfr[j].w, acc[i][j], 0, 0, 0);
        }
    }
  }
}

typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));

template <int BROWS>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int k0, int r0) {
  // A/B fragment of v_mfma_f32_16x16x32_bf16 from a [k][rows] image: lane l gets rows r0+(l&15),
  // k = k0 + 8*(l>>4) + 0..7, as two ds_read_b64_tr_b16 (4 k each).
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef LdsImg<bf16, 2, BROWS> L;
  const int ka = k0 + 8 * g + q;
  const char* p0 = img + L::tr_off(ka, r0 + 4 * p);
  const char* p1 = img + L::tr_off(ka + 4, r0 + 4 * p);
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)p0);
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)p1);
  short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int RM, int RN, int BM, int BN>
__device__ __forceinline__ void mma_kstep_tr(const char* As, const char* Bs, int wm0, int wn0,
                                             f32x4 (&acc)[RM][RN]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = tr_frag<BM>(As, kk * 32, wm0 + i * 16);
#pragma unroll
    for (int j = 0; j < RN; ++j) bfr[j] = tr_frag<BN>(Bs, kk * 32, wn0 + j * 16);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
}

// Epilogue shared by the GEMM kernels: row -> output offset, bias (FWD, split 0), beta, dtype,
// fp32 atomics for WGRAD and split-K.
template <typename T, int MODE, int BM, int BN>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const f32x4 (&acc)[BM / 32][BN / 32], int m0,
                                              int n0, int wm0, int wn0) {
  constexpr int RM = BM / 32, RN = BN / 32;
  const int lane = threadIdx.x & 63;
  const int col16 = lane & 15, rq = (lane >> 4) * 4;
  const es_conv_desc_t& d = a.d;
#pragma unroll
  for (int i = 0; i < RM; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int m = m0 + wm0 + i * 16 + rq + jj;
      if (m >= a.M) continue;
      int64_t rowoff = 0;
      if constexpr (MODE == MODE_FWD) {
        const int np = fdiv(m, a.fQ), q = m - np * d.Q;
        const int n = fdiv(np, a.fP), p = np - n * d.P;
        rowoff = n * a.os[0] + p * a.os[2] + q * a.os[3];
      } else if constexpr (MODE == MODE_DGRAD) {
        if (a.fold) {
          const int nh = fdiv(m, a.fW), j = m - nh * d.W;
          const int n = fdiv(nh, a.fH), ii = nh - n * d.H;
          rowoff = n * a.os[0] + ii * a.os[2] + j * a.os[3];
        } else {
          const int nh = fdiv(m, a.fWu), wu = m - nh * d.Wu;
          const int n = fdiv(nh, a.fHu), hu = nh - n * d.Hu;
          rowoff = n * a.os[0] + hu * a.os[2] + wu * a.os[3];
        }
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int ng = n0 + wn0 + j * 16 + col16;
        if (ng >= a.Ng) continue;
        float v = acc[i][j][jj];
        if constexpr (MODE == MODE_WGRAD) {
          if (a.det) ((float*)a.out)[((int64_t)blockIdx.z * a.mslot + m) * a.Ng + ng] = v;   // own partial slot
          else atomicAdd((float*)a.out + (int64_t)m * a.Ng + ng, v);
        } else {
          if constexpr (MODE == MODE_FWD) {
            if (a.bias && blockIdx.z == 0) v += a.bias[ng];
          }
          const int64_t o = rowoff + (int64_t)ng * a.os[1];
          if (a.splitk) {
            if (a.det) ((float*)a.det_ws)[(int64_t)blockIdx.z * a.mslot * a.Ng + o] = v;   // own partial slot
            else atomicAdd((float*)a.out + o, v);
          } else if (a.out_bf16) {
            bf16* y = (bf16*)a.out + o;
            if (a.beta != 0.f) v += a.beta * (float)(*y);
            *y = (bf16)v;
          } else {
            float* y = (float*)a.out + o;
            if (a.beta != 0.f) v += a.beta * (*y);
            *y = v;
          }
        }
      }
    }
  }
}

template <typename T, int MODE, int BM, int BN, bool AVEC, bool BVEC>
__global__ void __launch_bounds__(NTHREADS) conv_igemm_kernel(ConvArgs a) {
  constexpr int BK = KSTEP_BYTES / sizeof(T);
  constexpr int RM = BM / 32, RN = BN / 32;   // 16x16 tiles per wave (2x2 wave grid)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef LdsImg<T, MODE, BM> LA;
  typedef LdsImg<T, MODE, BN> LB;
  constexpr int BUF = LA::BYTES + LB::BYTES;   // one stage: A image then B image

  conv_live_gemm(a, MODE);
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * a.k_per_split;
  const int kend = min(a.Kd, kbeg + a.k_per_split);
  if ((kbeg >= kend || m0 >= a.M) && !a.det) return;   // (a partial slot is written even when empty)
  const int wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * (BM / 2), wn0 = (wid & 1) * (BN / 2);

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stager<T, MODE, BM, true, AVEC> sa;
  Stager<T, MODE, BN, false, BVEC> sb;
  sa.init(a, m0);
  sb.init(a, n0);
  sa.load(a, m0, kbeg);
  sb.load(a, n0, kbeg);
  sa.store(smem);
  sb.store(smem + LA::BYTES);
  __syncthreads();
  int cur = 0;
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) {
      sa.load(a, m0, k0 + BK);
      sb.load(a, n0, k0 + BK);
    }
    if constexpr (LA::TR)
      mma_kstep_tr<RM, RN, BM, BN>(smem + cur * BUF, smem + cur * BUF + LA::BYTES, wm0, wn0, acc);
    else
      mma_kstep<T, RM, RN>(smem + cur * BUF, smem + cur * BUF + LA::BYTES, wm0, wn0, acc);
    if (more) {
      sa.store(smem + (cur ^ 1) * BUF);
      sb.store(smem + (cur ^ 1) * BUF + LA::BYTES);
    }
    __syncthreads();
    cur ^= 1;
  }
  (void)BK;

  conv_epilogue<T, MODE, BM, BN>(a, acc, m0, n0, wm0, wn0);
}

// ---------------------------------------------------------------------------------------------
// bf16 FWD / DGRAD with LDS-DMA staging (global_load_lds_dwordx4).
//
// Used when every K-step (64 bf16) is ONE filter tap over 64 contiguous channels (C % 64 == 0 for
// FWD, K % 64 == 0 for DGRAD), so each GEMM row of a K-step is one contiguous 128-byte segment of
// an NHWC activation row (or all zero: padding / outside the image / stride-2 holes).
//   * A wave instruction moves 8 rows x 128 B straight into LDS (no register round trip); lanes
//     of padded rows read a 16-byte-aligned zero block instead.
//   * LDS image per operand: [rows][128 B] unpadded; logical 16-byte chunk lc of row r sits at
//     physical chunk lc ^ ((r >> 1) & 7) (the swizzle is applied on the global source address,
//     since the DMA destination is lane-linear), which makes the 16-row ds_read_b128 fragment
//     reads conflict-free.
//   * Two stages; one barrier per K-step: wait(stage t) + barrier, issue stage t+1, MFMAs on t.
//   * Block ids are remapped so that consecutive M tiles run on the same XCD (shared halo rows
//     stay in that XCD's L2).
// ---------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) char g_zero_row[128];   // zero-initialised at load

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <int RM, int RN>
__device__ __forceinline__ void mma_kstep_swz(const char* As, const char* Bs, int wm0, int wn0,
                                              f32x4 (&acc)[RM][RN]) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int seg = kk * 4 + g;
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(As + swz(wm0 + i * 16 + r16, seg));
#pragma unroll
    for (int j = 0; j < RN; ++j) bfr[j] = *(const bf16x8*)(Bs + swz(wn0 + j * 16 + r16, seg));
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
}

template <int MODE, int BM, int BN>
__global__ void __launch_bounds__(NTHREADS) conv_glds_kernel(ConvArgs a) {
  constexpr int RM = BM / 32, RN = BN / 32;
  constexpr int AI = BM / 32, BI = BN / 32;            // 8-row DMA pieces per wave (4 waves)
  constexpr int ABYTES = BM * 128, STAGE = (BM + BN) * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const es_conv_desc_t& d = a.d;
  conv_live_gemm(a, MODE);

  // XCD-aware tile order: consecutive tile ids on one XCD (bijective remap).  Dynamic rows: over the
  // live row tiles only (the rest exit), so that they spread over every XCD
  const int mt = (a.M + BM - 1) / BM;
  const int nwg = mt * gridDim.y;
  const int orig = blockIdx.x + blockIdx.y * gridDim.x;
  if (orig >= nwg) return;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int m0 = (wgid % mt) * BM, n0 = (wgid / mt) * BN;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * (BM / 2), wn0 = (wid & 1) * (BN / 2);
  const int lrow = lane >> 3, pc = lane & 7;          // row within an 8-row piece, physical chunk

  // per-lane rows of the A pieces: base offset (or -1) and two coordinates
  int64_t aoff[AI];
  int ac0[AI], ac1[AI], alc[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int rr = (wid * AI + j) * 8 + lrow;
    const int row = m0 + rr;
    alc[j] = pc ^ ((rr >> 1) & 7);
    const int rw = row < a.M ? row : 0;
    if constexpr (MODE == MODE_FWD) {
      const int np = fdiv(rw, a.fQ), q = rw - np * d.Q;
      const int n = fdiv(np, a.fP), p = np - n * d.P;
      aoff[j] = row < a.M ? (int64_t)n * a.as[0] + alc[j] * 8 : -1;
      ac0[j] = p * d.stride - d.pad;
      ac1[j] = q * d.stride - d.pad;
    } else if (a.fold) {
      const int nh = fdiv(rw, a.fW), jj = rw - nh * d.W;
      const int n = fdiv(nh, a.fH), ii = nh - n * d.H;
      aoff[j] = row < a.M ? (int64_t)n * a.as[0] + alc[j] * 8 : -1;
      ac0[j] = ii * d.up_h + d.pad;
      ac1[j] = jj * d.up_w + d.pad;
    } else {
      const int nh = fdiv(rw, a.fWu), wu = rw - nh * d.Wu;
      const int n = fdiv(nh, a.fHu), hu = nh - n * d.Hu;
      aoff[j] = row < a.M ? (int64_t)n * a.as[0] + alc[j] * 8 : -1;
      ac0[j] = hu + d.pad;
      ac1[j] = wu + d.pad;
    }
  }
  const int ldb = (MODE == MODE_DGRAD && a.fold) ? d.R * d.S * d.K : a.Kd;
  int64_t boff[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int rr = (wid * BI + j) * 8 + lrow;
    const int row = n0 + rr;
    boff[j] = row < a.Ng ? (int64_t)row * ldb + ((pc ^ ((rr >> 1) & 7)) * 8) : -1;
  }
  const bf16* asrc = (const bf16*)a.a_src;
  const bf16* bsrc = (const bf16*)a.b_src;
  const char* zero = g_zero_row;

  auto issue = [&](int kk, char* stage) {
    // K-step decode (uniform): tap (r, s), channel offset, upsample phase (folded DGRAD)
    int r, s_, ch0, ua = 0, ub = 0, kb = kk;
    if constexpr (MODE == MODE_FWD) {
      const int rs = fdiv(kk, a.fC);
      ch0 = kk - rs * d.C;
      r = fdiv(rs, a.fS); s_ = rs - r * d.S;
    } else {
      int kr = kk;
      if (a.fold) {
        const int ab = fdiv(kk, a.fRSK);
        kr = kk - ab * (d.R * d.S * d.K);
        kb = kr;
        ua = fdiv(ab, a.fUw); ub = ab - ua * d.up_w;
      }
      const int rs = fdiv(kr, a.fK);
      ch0 = kr - rs * d.K;
      r = fdiv(rs, a.fS); s_ = rs - r * d.S;
    }
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const void* src = zero;
      if (aoff[j] >= 0) {
        if constexpr (MODE == MODE_FWD) {
          const int hu = ac0[j] + r, wu = ac1[j] + s_;
          if (hu >= 0 && hu < d.Hu && wu >= 0 && wu < d.Wu)
            // integer upsample only on this path (no map loads: an ordinary load here would make
            // the compiler drain the in-flight DMA with vmcnt(0))
            src = asrc + aoff[j] + ch0 + (int64_t)(d.up_h > 0 ? fdiv(hu, a.fUh) : hu) * a.as[2] +
                  (int64_t)(d.up_w > 0 ? fdiv(wu, a.fUw) : wu) * a.as[3];
        } else {
          int ph = ac0[j] + ua - r, pw = ac1[j] + ub - s_;
          bool ok = ph >= 0 && pw >= 0;
          if (d.stride == 2) { ok = ok && !(ph & 1) && !(pw & 1); ph >>= 1; pw >>= 1; }
          if (ok && ph < d.P && pw < d.Q)
            src = asrc + aoff[j] + ch0 + (int64_t)ph * a.as[2] + (int64_t)pw * a.as[3];
        }
      }
      glds16(src, stage + (wid * AI + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const void* src = boff[j] >= 0 ? (const void*)(bsrc + boff[j] + kb) : (const void*)zero;
      glds16(src, stage + ABYTES + (wid * BI + j) * 1024);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kd / 64;
  issue(0, smem);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                   // stage t landed; stage t-1 fully read
    char* cur = smem + (t & 1) * STAGE;
    if (t + 1 < nk) issue((t + 1) * 64, smem + ((t + 1) & 1) * STAGE);
    mma_kstep_swz<RM, RN>(cur, cur + ABYTES, wm0, wn0, acc);
  }
  conv_epilogue<bf16, MODE, BM, BN>(a, acc, m0, n0, wm0, wn0);
}

template <typename T, int MODE, int BM, int BN>
int launch_tile(const ConvArgs& a, bool avec, bool bvec, hipStream_t st, int splits) {
  dim3 grid((a.M + BM - 1) / BM, (a.Ng + BN - 1) / BN, splits);
  const size_t lds = 2 * (LdsImg<T, MODE, BM>::BYTES + LdsImg<T, MODE, BN>::BYTES);
#define ES_LAUNCH(AV, BV)                                                                     \
  hipLaunchKernelGGL((conv_igemm_kernel<T, MODE, BM, BN, AV, BV>), grid, dim3(NTHREADS), lds, \
                     st, a)
  if (avec && bvec) ES_LAUNCH(true, true);
  else if (avec) ES_LAUNCH(true, false);
  else if (bvec) ES_LAUNCH(false, true);
  else ES_LAUNCH(false, false);
#undef ES_LAUNCH
  ES_CHECK_LAUNCH();
  return ES_OK;
}

// ---------------------------------------------------------------------------------------------
// bf16 WGRAD with LDS-DMA staging.  GEMM: dW[m = k][ng = (r,s,c)] = sum over pixels of
// dy[pix][k] * x[pix + (r,s)][c]; a K-step is 64 pixels.  Both operands are contiguous along the
// GEMM row (k / c), so each pixel contributes one 256-byte segment per operand per tile
// (K % 128 == 0 and C % 128 == 0: the 128 columns of a tile are one tap).
//   * LDS image [pixel][row] (256-byte k-rows, lane-linear DMA, 4 pixels per wave instruction),
//     read with ds_read_b64_tr_b16.  The 16-byte chunk index of k-row kr is XORed with
//     2*(kr & 3) | 8*((kr >> 3) & 1): the 8 k-rows one 32-lane half reads land on 8 disjoint
//     32-byte bank groups (conflict-free without padding, which a DMA image cannot have).
//   * Split-K over blockIdx.z with fp32 atomics (as the register-staged WGRAD).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int swz_tr(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }
// byte offset of element (k-row k, row) in a [64][128] bf16 image with 256-byte k-rows
__device__ __forceinline__ int trs_off(int k, int row) {
  return k * 256 + ((((row >> 3) ^ swz_tr(k)) << 4) | ((row & 7) << 1));
}

__device__ __forceinline__ bf16x8 trs_frag(const char* img, int k0, int r0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ka = k0 + 8 * g + q;
  const char* p0 = img + trs_off(ka, r0 + 4 * p);
  const char* p1 = img + trs_off(ka + 4, r0 + 4 * p);
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)p0);
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)p1);
  short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__global__ void __launch_bounds__(NTHREADS) conv_wgrad_glds_kernel(ConvArgs a) {
  constexpr int BM = 128, BN = 128, RM = 4, RN = 4;
  constexpr int IMG = 64 * 256, STAGE = 2 * IMG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const es_conv_desc_t& d = a.d;
  conv_live_gemm(a, MODE_WGRAD);

  // XCD-aware order: blocks of one K split (same pixels) are consecutive on one XCD
  const int mt = gridDim.x, ntl = gridDim.y, tiles = mt * ntl;
  const int nwg = tiles * gridDim.z;
  const int orig = blockIdx.x + (blockIdx.y + blockIdx.z * ntl) * mt;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tile = wgid % tiles, split = wgid / tiles;
  const int m0 = (tile % mt) * BM, n0 = (tile / mt) * BN;
  const int kbeg = split * a.k_per_split;
  const int kend = min(a.Kd, kbeg + a.k_per_split);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * (BM / 2), wn0 = (wid & 1) * (BN / 2);
  const int lrow = lane >> 4, pc = lane & 15;          // pixel row within a piece, physical chunk
  // the tile's tap and channel offset (C % 128 == 0: one tap per tile)
  const int rs = fdiv(n0, a.fC), cb = n0 - rs * d.C;
  const int tr = fdiv(rs, a.fS), ts = rs - tr * d.S;
  const bf16* dy = (const bf16*)a.a_src;
  const bf16* x = (const bf16*)a.b_src;
  const char* zero = g_zero_row;

  auto issue = [&](int k0, char* stage) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kr = (wid * 4 + j) * 4 + lrow;          // pixel row of the K-step, 0..63
      const int lc = pc ^ swz_tr(kr);
      const int pix = k0 + kr;
      const void* sa = zero;
      const void* sb = zero;
      if (pix < kend) {
        const int np = fdiv(pix, a.fQ), qq = pix - np * d.Q;
        const int n = fdiv(np, a.fP), pp = np - n * d.P;
        sa = dy + (int64_t)n * a.as[0] + (int64_t)pp * a.as[2] + (int64_t)qq * a.as[3] + m0 + lc * 8;
        const int hu = pp * d.stride - d.pad + tr, wu = qq * d.stride - d.pad + ts;
        if (hu >= 0 && hu < d.Hu && wu >= 0 && wu < d.Wu)
          sb = x + (int64_t)n * a.bs[0] + (int64_t)(d.up_h > 0 ? fdiv(hu, a.fUh) : hu) * a.bs[2] +
               (int64_t)(d.up_w > 0 ? fdiv(wu, a.fUw) : wu) * a.bs[3] + cb + lc * 8;
      }
      glds16(sa, stage + (wid * 4 + j) * 1024);
      glds16(sb, stage + IMG + (wid * 4 + j) * 1024);
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kbeg < kend) {
    const int nk = (kend - kbeg + 63) / 64;
    issue(kbeg, smem);
    for (int t = 0; t < nk; ++t) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const char* cur = smem + (t & 1) * STAGE;
      if (t + 1 < nk) issue(kbeg + (t + 1) * 64, smem + ((t + 1) & 1) * STAGE);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = trs_frag(cur, kk * 32, wm0 + i * 16);
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[j] = trs_frag(cur + IMG, kk * 32, wn0 + j * 16);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  conv_epilogue<bf16, MODE_WGRAD, BM, BN>(a, acc, m0, n0, wm0, wn0);
}

template <int MODE, int BM, int BN>
int launch_glds(ConvArgs& a, hipStream_t st) {
  const int mt = (a.M + BM - 1) / BM;
  dim3 grid(mt, (a.Ng + BN - 1) / BN, 1);
  a.k_per_split = a.Kd;
  a.splitk = 0;
  hipLaunchKernelGGL((conv_glds_kernel<MODE, BM, BN>), grid, dim3(NTHREADS), 2 * (BM + BN) * 128, st, a);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

template <typename T, int MODE>
int launch(ConvArgs& a, bool avec, bool bvec, hipStream_t st) {
  constexpr int BK = KSTEP_BYTES / sizeof(T);
  if constexpr (sizeof(T) == 2 && MODE != MODE_WGRAD) {
    // LDS-DMA path: one tap x 64 channels per K-step, big enough to fill the chip without split-K
    const int nch = MODE == MODE_FWD ? a.d.C : a.d.K;
    const int tiles = ((a.M + 127) / 128) * ((a.Ng + 127) / 128);
    const bool splitk_better = a.dense_f32_out && tiles < 256 && a.Kd / 64 >= 16;   // see below
    if (avec && bvec && nch % 64 == 0 && a.d.stride <= 2 && a.d.hmap == nullptr && a.M >= 128 && !splitk_better &&
        !g_no_glds) {
      a.k_per_split = a.Kd;
      a.splitk = 0;
      if (a.Kd % 64 == 0) {
        const int rc = es_conv_ring_launch(a, MODE, st);
        if (rc) {
          ES_CHECK_LAUNCH();
          return ES_OK;
        }
      }
      if (a.Ng > 64) return launch_glds<MODE, 128, 128>(a, st);
      return launch_glds<MODE, 128, 64>(a, st);
    }
  }
  if constexpr (sizeof(T) == 4 && MODE != MODE_WGRAD) {
    // fp32 parity mode: the 8-wave LDS-DMA ring kernels on v_mfma_f32_16x16x4_f32 (conv_mfma.hip)
    // for real convolutions whose K-steps are one tap x 32 channels
    const int nch = MODE == MODE_FWD ? a.d.C : a.d.K;
    // (the gathered grid's pixels per image: >= 8 keeps the row tiles' padding small; the aux
    // regressor's conv4 has a 1 x 15 output and a 3 x 17 input; linears take the pixel view)
    const int gpix = MODE == MODE_FWD ? a.d.P * a.d.Q : a.d.Hu * a.d.Wu;
    if (avec && bvec && nch % 32 == 0 && a.Kd % 32 == 0 && a.d.stride <= 2 && a.d.hmap == nullptr &&
        gpix >= 8 && a.M >= 128 && !g_no_glds) {
      a.k_per_split = a.Kd;
      a.splitk = 0;
      const int rc = es_conv_ring_launch_f32(a, MODE, st);
      if (rc < 0) return ES_ERR_ARG;
      if (rc > 0) {
        ES_CHECK_LAUNCH();
        return ES_OK;
      }
    }
  }
  // tile choice: 128x128 for big GEMMs, 64x64 when either side is small, or when the output is
  // split over K anyway (few tiles, long K: more, smaller workgroups)
  const int tiles128 = ((a.M + 127) / 128) * ((a.Ng + 127) / 128);
  // (deterministic mode: only with a partial workspace, es_conv2d_fwd_det / es_conv2d_dgrad_det)
  const bool splitk_case = MODE != MODE_WGRAD && a.dense_f32_out && tiles128 < 256 && (a.Kd + BK - 1) / BK >= 16 &&
                           !(sizeof(T) == 4 && g_es_det && g_det_req.ws == nullptr);
  // 128 x 128 only with enough tiles to fill the chip: a small GEMM (the discriminator / router /
  // aux linears at batch 512) is latency-bound per K-step, so more, smaller workgroups finish sooner
  const bool big = a.M >= 128 && a.Ng >= 96 && !splitk_case && tiles128 >= 128;
  // narrow fp32 GEMMs (the discriminator's 32->16 conv: FWD / DGRAD with N <= 32, WGRAD with
  // M = 16 output channels): a 64 x 64 tile wastes half or 3/4 of every MFMA; 128 x 32 and
  // 32 x 128 tiles keep the 2 x 2 wave grid with one 16-row (column) fragment per wave
  const bool narrow_n = sizeof(T) == 4 && MODE != MODE_WGRAD && a.Ng <= 32 && !splitk_case;
  const bool narrow_m = sizeof(T) == 4 && MODE == MODE_WGRAD && a.M <= 32 && !big;
  const int BM = big ? 128 : (narrow_n ? 128 : (narrow_m ? 32 : 64));
  const int BN = big ? 128 : (narrow_n ? 32 : (narrow_m ? 128 : 64));
  if constexpr (sizeof(T) == 2 && MODE == MODE_WGRAD) {
    if (!a.det && avec && bvec && !g_no_glds && es_conv_ring_launch(a, MODE, st)) {
      ES_CHECK_LAUNCH();
      return ES_OK;
    }
    if (!a.det && avec && bvec && a.d.K % 128 == 0 && a.d.C % 128 == 0 && a.d.stride <= 2 && a.d.hmap == nullptr &&
        !g_no_glds) {
      const int t128 = (a.M / 128) * (a.Ng / 128);
      const int ks = (a.Kd + 63) / 64;
      int want = (2048 + t128 - 1) / t128;
      want = max(1, min(want, ks / 4 > 0 ? ks / 4 : 1));
      const int per = ((ks + want - 1) / want) * 64;
      a.k_per_split = per;
      a.splitk = 0;
      dim3 grid(a.M / 128, a.Ng / 128, (a.Kd + per - 1) / per);
      hipLaunchKernelGGL(conv_wgrad_glds_kernel, grid, dim3(NTHREADS), 2 * 2 * 64 * 256, st, a);
      ES_CHECK_LAUNCH();
      return ES_OK;
    }
  }
  int splits = 1;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.Ng + BN - 1) / BN);
  const int ksteps = (a.Kd + BK - 1) / BK;
  a.k_per_split = a.Kd;
  a.splitk = 0;
  if (MODE == MODE_WGRAD) {
    int want = (2048 + tiles - 1) / tiles;            // ~2048 workgroups
    want = max(1, min(want, ksteps / 4 > 0 ? ksteps / 4 : 1));  // >= 4 K-steps per split
    if (a.det) {   // deterministic: one partial slot per split, within the caller's workspace
      const int64_t slot = (int64_t)a.M * a.Ng;
      want = (int)std::max<int64_t>(1, std::min<int64_t>(want, g_det_req.floats / slot));
    }
    const int per = ((ksteps + want - 1) / want) * BK;
    a.k_per_split = per;
    splits = (a.Kd + per - 1) / per;
    if (a.det) g_det_req.splits = splits;
  } else if (splitk_case) {
    // few output tiles and a long K (the linears at batch 512): split K over ~1024 workgroups,
    // at least 4 K-steps each
    int want = min((1024 + tiles - 1) / tiles, ksteps / 4);
    const bool det = g_det_req.ws != nullptr;
    if (det) want = (int)std::min<int64_t>(want, g_det_req.floats / ((int64_t)a.M * a.Ng));
    if (want > 1) {
      const int per = ((ksteps + want - 1) / want) * BK;
      a.k_per_split = per;
      splits = (a.Kd + per - 1) / per;
      a.splitk = splits > 1;
      if (det && a.splitk) {   // ordered: split z stores into its own slot, es_splitk_reduce sums
        a.det = 1;
        a.det_ws = g_det_req.ws;
        g_det_req.splits = splits;
      } else if (a.splitk && hipMemsetAsync(a.out, 0, (size_t)a.M * a.Ng * sizeof(float), st) != hipSuccess) {
        es_set_error("conv: split-K memset failed");
        return ES_ERR_HIP;
      }
    }
  }
  if (big) return launch_tile<T, MODE, 128, 128>(a, avec, bvec, st, splits);
  if constexpr (sizeof(T) == 4) {
    if constexpr (MODE != MODE_WGRAD) {
      if (narrow_n) return launch_tile<T, MODE, 128, 32>(a, avec, bvec, st, splits);
    } else {
      if (narrow_m) return launch_tile<T, MODE, 32, 128>(a, avec, bvec, st, splits);
    }
  }
  return launch_tile<T, MODE, 64, 64>(a, avec, bvec, st, splits);
}

template <int MODE>
int dispatch(ConvArgs& a, es_dtype_t dt, bool avec, bool bvec, hipStream_t st) {
  a.fC = mkdiv(a.d.C); a.fS = mkdiv(a.d.S); a.fK = mkdiv(a.d.K); a.fQ = mkdiv(a.d.Q);
  a.fP = mkdiv(a.d.P); a.fWu = mkdiv(a.d.Wu); a.fHu = mkdiv(a.d.Hu);
  a.fUh = mkdiv(a.d.up_h > 0 ? a.d.up_h : 1); a.fUw = mkdiv(a.d.up_w > 0 ? a.d.up_w : 1);
  a.fRSK = mkdiv(a.d.R * a.d.S * a.d.K); a.fW = mkdiv(a.d.W); a.fH = mkdiv(a.d.H);
  if (a.d.stride > 2) avec = bvec = false;   // vector DGRAD gather handles strides 1 and 2
  if (dt == ES_F32) return launch<float, MODE>(a, avec, bvec, st);
  if (dt == ES_BF16) return launch<bf16, MODE>(a, avec, bvec, st);
  es_set_error("conv: unsupported dtype %d", (int)dt);
  return ES_ERR_ARG;
}

// strides (n, c, h, w) describe a dense [n][h][w][c] tensor (rows of c contiguous values)
bool dense_rows(const int64_t s[4], int c, int h, int w) {
  return s[1] == 1 && (w == 1 || s[3] == c) && (h == 1 || s[2] == (int64_t)w * c) && s[0] == (int64_t)h * w * c;
}

int check_desc(const es_conv_desc_t* d) {
  ES_CHECK_ARG(d && d->N > 0 && d->C > 0 && d->K > 0 && d->R > 0 && d->S > 0 && d->stride > 0,
               "conv: bad descriptor");
  ES_CHECK_ARG(d->P == (d->Hu + 2 * d->pad - d->R) / d->stride + 1 &&
                   d->Q == (d->Wu + 2 * d->pad - d->S) / d->stride + 1,
               "conv: output size %dx%d inconsistent with input %dx%d k%dx%d s%d p%d", d->P, d->Q,
               d->Hu, d->Wu, d->R, d->S, d->stride, d->pad);
  ES_CHECK_ARG((d->hmap == nullptr) == (d->wmap == nullptr), "conv: hmap/wmap must both be set");
  ES_CHECK_ARG((d->up_h > 0) == (d->up_w > 0), "conv: up_h/up_w must both be set");
  ES_CHECK_ARG(d->up_h <= 0 || (d->Hu == d->H * d->up_h && d->Wu == d->W * d->up_w),
               "conv: Hu/Wu must equal H*up_h / W*up_w");
  ES_CHECK_ARG(d->hmap || d->up_h > 0 || (d->Hu == d->H && d->Wu == d->W), "conv: Hu/Wu != H/W without maps");
  const int64_t M1 = (int64_t)d->N * d->P * d->Q, M2 = (int64_t)d->N * d->Hu * d->Wu;
  ES_CHECK_ARG(M1 < (1ll << 31) && M2 < (1ll << 31), "conv: problem too large for int32 rows");
  return ES_OK;
}

// sub-pixel FWD / DGRAD: only the ring kernels read mode 2 / 3 packed weights
int ring_direct(ConvArgs& a, int mode, hipStream_t st, es_dtype_t dt) {
  a.fC = mkdiv(a.d.C); a.fS = mkdiv(a.d.S); a.fK = mkdiv(a.d.K); a.fQ = mkdiv(a.d.Q);
  a.fP = mkdiv(a.d.P); a.fWu = mkdiv(a.d.Wu); a.fHu = mkdiv(a.d.Hu);
  a.fUh = mkdiv(2); a.fUw = mkdiv(2);
  a.fRSK = mkdiv(a.d.R * a.d.S * a.d.K); a.fW = mkdiv(a.d.W); a.fH = mkdiv(a.d.H);
  a.k_per_split = a.Kd;
  a.splitk = 0;
  const int rc = dt == ES_F32 ? es_conv_ring_launch_f32(a, mode, st) : es_conv_ring_launch(a, mode, st);
  ES_CHECK_ARG(rc > 0, "conv: sub-pixel operands not dense NHWC (ring kernels required)");
  ES_CHECK_LAUNCH();
  return ES_OK;
}

}  // namespace

// ---------------------------------------------------------------- executed-work tally (es_conv_exec_flops)
thread_local int g_ring_hit = 0;
namespace {
// per host thread (the probe reads the thread that issued the convs)
thread_local double g_exec_flops[3] = {0.0, 0.0, 0.0};
// RAII around one conv entry: classifies the path the call took and adds its executed FLOPs, only
// when the entry returns ES_OK (ok() marks it: failed calls issue no work)
struct ExecTally {
  const es_conv_desc_t* d;
  es_dtype_t dt;
  bool thin = false;
  bool done = false;
  ExecTally(const es_conv_desc_t* d_, es_dtype_t dt_) : d(d_), dt(dt_) { g_ring_hit = 0; }
  int ok(int rc) {
    done = rc == ES_OK;
    return rc;
  }
  ~ExecTally() {
    if (!d || !done) return;
    double f = 2.0 * d->N * d->P * d->Q * (double)d->K * d->C * d->R * d->S;
    if (g_ring_hit & 4) f *= (double)es_subpixel_taps(d->R, d->S) / (4.0 * d->R * d->S);
    if (thin) g_exec_flops[2] += f;
    else if (dt == ES_BF16) g_exec_flops[0] += f;
    else if (g_ring_hit & 2) g_exec_flops[0] += 6.0 * f;
    else g_exec_flops[1] += f;
  }
};
}  // namespace

extern "C" int es_conv_exec_flops(double out[3], int reset) {
  ES_CHECK_ARG(out != nullptr, "conv exec flops: NULL out");
  for (int i = 0; i < 3; ++i) {
    out[i] = g_exec_flops[i];
    if (reset) g_exec_flops[i] = 0.0;
  }
  return ES_OK;
}

extern "C" int es_set_deterministic(int on) {
  const int old = g_es_det;
  g_es_det = on != 0;
  return old;
}

extern "C" int es_conv_set_glds(int on) {
  const int old = !g_no_glds;
  g_no_glds = !on;
  return old;
}

extern "C" int es_conv2d_fwd(const es_conv_desc_t* d, es_dtype_t dt, const void* x,
                             const int64_t xs[4], const void* wk, const float* bias, void* y,
                             es_dtype_t ydt, const int64_t ys[4], es_stream_t stream) {
  if (int e = check_desc(d)) return e;
  ExecTally tally(d, dt);
  if (d->subpixel) ES_CHECK_ARG(es_conv_subpixel_ok(d, dt), "conv fwd: sub-pixel weights for a conv the sub-pixel path cannot run");
  if (es_thin_conv_fwd(d, dt, x, xs, wk, bias, y, ydt, ys, (hipStream_t)stream)) {
    tally.thin = true;
    ES_CHECK_LAUNCH();
    return tally.ok(ES_OK);
  }
  ConvArgs a{};
  a.d = *d; a.a_src = x; a.b_src = wk; a.out = y; a.bias = bias; a.beta = 0.f;
  a.out_bf16 = ydt == ES_BF16;
  for (int i = 0; i < 4; ++i) { a.as[i] = xs[i]; a.os[i] = ys[i]; }
  a.M = d->N * d->P * d->Q; a.Ng = d->K; a.Kd = d->R * d->S * d->C;
  a.dense_f32_out = ydt == ES_F32 && dense_rows(ys, d->K, d->P, d->Q);
  const int vn = dt == ES_BF16 ? 8 : 4;
  const bool avec = xs[1] == 1 && d->C % vn == 0;
  const bool bvec = a.Kd % vn == 0;
  if (d->subpixel) return tally.ok(ring_direct(a, MODE_FWD, (hipStream_t)stream, dt));
  return tally.ok(dispatch<MODE_FWD>(a, dt, avec, bvec, (hipStream_t)stream));
}

extern "C" int es_conv2d_fwd_stats(const es_conv_desc_t* d, es_dtype_t dt, const void* x, const int64_t xs[4],
                                   const void* wk, const float* bias, void* y, es_dtype_t ydt, const int64_t ys[4],
                                   float* part, int64_t part_floats, int* chunks, es_stream_t stream) {
  ES_CHECK_ARG(part && chunks, "conv fwd stats: part / chunks NULL");
  g_stats_req = StatsRequest{part, part_floats, 0};
  const int rc = es_conv2d_fwd(d, dt, x, xs, wk, bias, y, ydt, ys, stream);
  *chunks = g_stats_req.chunks;
  g_stats_req = StatsRequest{nullptr, 0, 0};
  return rc;
}

extern "C" int es_conv2d_dgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy,
                               const int64_t ys[4], const void* wd, void* dxu, es_dtype_t dxdt,
                               const int64_t dxs[4], float beta, es_stream_t stream) {
  if (int e = check_desc(d)) return e;
  ExecTally tally(d, dt);
  if (d->subpixel) ES_CHECK_ARG(es_conv_subpixel_ok(d, dt), "conv dgrad: sub-pixel weights for a conv the sub-pixel path cannot run");
  if (es_thin_conv_dgrad(d, dt, dy, ys, wd, dxu, dxdt, dxs, beta, (hipStream_t)stream)) {
    tally.thin = true;
    ES_CHECK_LAUNCH();
    return tally.ok(ES_OK);
  }
  ConvArgs a{};
  a.d = *d; a.a_src = dy; a.b_src = wd; a.out = dxu; a.bias = nullptr; a.beta = beta;
  a.out_bf16 = dxdt == ES_BF16;
  for (int i = 0; i < 4; ++i) { a.as[i] = ys[i]; a.os[i] = dxs[i]; }
  a.fold = d->up_h > 0;
  if (a.fold) { a.M = d->N * d->H * d->W; a.Kd = d->up_h * d->up_w * d->R * d->S * d->K; }
  else { a.M = d->N * d->Hu * d->Wu; a.Kd = d->R * d->S * d->K; }
  a.Ng = d->C;
  {
    const int64_t oh = a.fold ? d->H : d->Hu, ow = a.fold ? d->W : d->Wu;
    a.dense_f32_out = dxdt == ES_F32 && beta == 0.f && dense_rows(dxs, d->C, (int)oh, (int)ow);
  }
  const int vn = dt == ES_BF16 ? 8 : 4;
  const bool avec = ys[1] == 1 && d->K % vn == 0;
  const bool bvec = a.Kd % vn == 0;
  if (d->subpixel) return tally.ok(ring_direct(a, MODE_DGRAD, (hipStream_t)stream, dt));
  return tally.ok(dispatch<MODE_DGRAD>(a, dt, avec, bvec, (hipStream_t)stream));
}

extern "C" int es_conv2d_dgrad_bnred(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                                     const void* wd, void* dx, es_dtype_t dxdt, const int64_t dxs[4],
                                     const void* x, const es_norm_t* nm, const es_chain_t* ch, float* part,
                                     int64_t part_floats, int* chunks, es_stream_t stream) {
  ES_CHECK_ARG(part && chunks && x && nm && ch, "conv dgrad bnred: NULL argument");
  g_bnr_req = BnRedRequest{x, nm, ch, part, part_floats, 0};
  const int rc = es_conv2d_dgrad(d, dt, dy, ys, wd, dx, dxdt, dxs, 0.f, stream);
  *chunks = g_bnr_req.chunks;
  g_bnr_req = BnRedRequest{nullptr, nullptr, nullptr, nullptr, 0, 0};
  return rc;
}

extern "C" int es_conv2d_wgrad(const es_conv_desc_t* d, es_dtype_t dt, const void* dy,
                               const int64_t ys[4], const void* x, const int64_t xs[4], float* dw,
                               es_stream_t stream) {
  if (int e = check_desc(d)) return e;
  ExecTally tally(d, dt);
  if (es_thin_conv_wgrad(d, dt, dy, ys, x, xs, dw, (hipStream_t)stream)) {
    tally.thin = true;
    ES_CHECK_LAUNCH();
    return tally.ok(ES_OK);
  }
  ConvArgs a{};
  a.d = *d; a.a_src = dy; a.b_src = x; a.out = dw;
  for (int i = 0; i < 4; ++i) { a.as[i] = ys[i]; a.bs[i] = xs[i]; }
  a.M = d->K; a.Ng = d->R * d->S * d->C; a.Kd = d->N * d->P * d->Q;
  const int vn = dt == ES_BF16 ? 8 : 4;
  const bool avec = ys[1] == 1 && d->K % vn == 0;
  const bool bvec = xs[1] == 1 && d->C % vn == 0;
  return tally.ok(dispatch<MODE_WGRAD>(a, dt, avec, bvec, (hipStream_t)stream));
}

// ------------------------------------------------------------------------- deterministic WGRAD
// (parity mode) dW = beta * dW + conv weight gradient, written in the torch layout [K][C][R][S] with
// a fixed summation order: the K splits store raw partials into the caller's workspace (no float
// atomics) and one ordered reduce sums them.  fp32 shapes the ring takes run wgrad_f32_kernel
// (conv_mfma.hip); the rest run the register-staged / thin kernels with per-split partials.
thread_local DetRequest g_det_req;
bool g_es_det = false;

namespace {
// generic path: partial slots offered = clamp(2^26 floats / slot, 8, 2048) (small thin-conv slots
// keep their ~1024 blocks; the big linear slots stay within ~256 MB)
int64_t generic_det_floats(const es_conv_desc_t* d) {
  const int64_t per = (int64_t)d->K * d->R * d->S * d->C;
  return per * std::max<int64_t>(8, std::min<int64_t>(2048, (1ll << 26) / per));
}
}  // namespace

extern "C" int64_t es_conv2d_wgrad_det_ws_bytes(const es_conv_desc_t* d, es_dtype_t dt, const int64_t ys[4],
                                                const int64_t xs[4]) {
  if (!d || check_desc(d)) return -1;
  int64_t f = -1;
  if (dt == ES_F32) f = es_wgrad_f32_ring_floats(*d, ys, xs);
  if (f < 0) f = generic_det_floats(d);
  return f * (int64_t)sizeof(float);
}

extern "C" int es_conv2d_wgrad_det(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                                   const void* x, const int64_t xs[4], float* dw, float beta, void* ws,
                                   int64_t ws_bytes, es_stream_t stream) {
  if (int e = check_desc(d)) return e;
  ES_CHECK_ARG(dw && ws, "conv wgrad det: NULL dw / workspace");
  ExecTally tally(d, dt);
  const hipStream_t st = (hipStream_t)stream;
  const int64_t floats = ws_bytes / (int64_t)sizeof(float);
  if (dt == ES_F32) {
    const int rc = es_wgrad_f32_ring(*d, dy, ys, x, xs, dw, beta, (float*)ws, floats, st);
    if (rc < 0) return ES_ERR_ARG;
    if (rc > 0) {
      ES_CHECK_LAUNCH();
      return tally.ok(ES_OK);
    }
  }
  const int64_t per = (int64_t)d->K * d->R * d->S * d->C;
  ES_CHECK_ARG(floats >= per, "conv wgrad det: workspace below one partial");
  g_det_req = DetRequest{(float*)ws, floats, 0};
  int rc = es_thin_conv_wgrad(d, dt, dy, ys, x, xs, (float*)ws, st) ? ES_OK : -1;
  tally.thin = rc == ES_OK;
  if (rc != ES_OK) {
    ConvArgs a{};
    a.d = *d; a.a_src = dy; a.b_src = x; a.out = ws;
    for (int i = 0; i < 4; ++i) { a.as[i] = ys[i]; a.bs[i] = xs[i]; }
    a.M = d->K; a.Ng = d->R * d->S * d->C; a.Kd = d->N * d->P * d->Q;
    const int vn = dt == ES_BF16 ? 8 : 4;
    const bool avec = ys[1] == 1 && d->K % vn == 0;
    const bool bvec = xs[1] == 1 && d->C % vn == 0;
    a.det = 1;
    rc = dispatch<MODE_WGRAD>(a, dt, avec, bvec, st);
  }
  const int splits = g_det_req.splits;
  g_det_req = DetRequest{nullptr, 0, 0};
  if (rc != ES_OK) return rc;
  ES_CHECK_ARG(splits > 0, "conv wgrad det: no partials written");
  es_wgrad_reduce_plain((const float*)ws, splits, d->K, d->C, d->R, d->S, dw, beta, st);
  ES_CHECK_LAUNCH();
  return tally.ok(ES_OK);
}

// deterministic split-K FWD / DGRAD (the fp32 linears with few output tiles and a long K: the
// generator's fc2 dgrad, K = 21632 / 92160): the splits store partials into ws, one ordered sum
namespace {
constexpr int kDetSplitK = 16;
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int64_t n, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += ws[z * n + i];
    out[i] = v;
  }
}
int splitk_det_finish(int rc, float* out, int64_t n, hipStream_t st) {
  const int splits = g_det_req.splits;
  const float* ws = g_det_req.ws;
  g_det_req = DetRequest{nullptr, 0, 0};
  if (rc != ES_OK || splits == 0) return rc;   // no split: the kernel wrote out itself
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, splits, n, out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
}  // namespace

extern "C" int64_t es_conv2d_splitk_ws_bytes(const es_conv_desc_t* d, int mode) {
  if (!d || check_desc(d) || (mode != MODE_FWD && mode != MODE_DGRAD)) return -1;
  const int64_t M = mode == MODE_FWD ? (int64_t)d->N * d->P * d->Q
                                     : (d->up_h > 0 ? (int64_t)d->N * d->H * d->W : (int64_t)d->N * d->Hu * d->Wu);
  const int64_t Ng = mode == MODE_FWD ? d->K : d->C;
  return M * Ng * kDetSplitK * (int64_t)sizeof(float);
}

extern "C" int es_conv2d_fwd_det(const es_conv_desc_t* d, es_dtype_t dt, const void* x, const int64_t xs[4],
                                 const void* wk, const float* bias, void* y, es_dtype_t ydt, const int64_t ys[4],
                                 void* ws, int64_t ws_bytes, es_stream_t stream) {
  ES_CHECK_ARG(ws, "conv fwd det: NULL workspace");
  g_det_req = DetRequest{(float*)ws, ws_bytes / (int64_t)sizeof(float), 0};
  const int rc = es_conv2d_fwd(d, dt, x, xs, wk, bias, y, ydt, ys, stream);
  return splitk_det_finish(rc, (float*)y, (int64_t)d->N * d->P * d->Q * d->K, (hipStream_t)stream);
}

extern "C" int es_conv2d_dgrad_det(const es_conv_desc_t* d, es_dtype_t dt, const void* dy, const int64_t ys[4],
                                   const void* wd, void* dxu, es_dtype_t dxdt, const int64_t dxs[4], void* ws,
                                   int64_t ws_bytes, es_stream_t stream) {
  ES_CHECK_ARG(ws, "conv dgrad det: NULL workspace");
  g_det_req = DetRequest{(float*)ws, ws_bytes / (int64_t)sizeof(float), 0};
  const int rc = es_conv2d_dgrad(d, dt, dy, ys, wd, dxu, dxdt, dxs, 0.f, stream);
  const int64_t M = d->up_h > 0 ? (int64_t)d->N * d->H * d->W : (int64_t)d->N * d->Hu * d->Wu;
  return splitk_det_finish(rc, (float*)dxu, M * d->C, (hipStream_t)stream);
}

// ------------------------------------------------------------------------- weight (un)packing
namespace {
// sub-pixel combined weight W'_t[d][e] (t = 2a + b) at (k, c): sum over the covered taps
__device__ __forceinline__ float subpixel_weight(const float* __restrict__ w, int k, int c, int C, int R, int S,
                                                 int t, int dd, int ee) {
  const int a = t >> 1, b = t & 1;
  const int r0 = max(0, 2 * dd - a), r1 = min(R - 1, 2 * dd - a + 1);
  const int s0 = max(0, 2 * ee - b), s1 = min(S - 1, 2 * ee - b + 1);
  float v = 0.f;
  for (int r = r0; r <= r1; ++r)
    for (int s = s0; s <= s1; ++s) v += w[(((int64_t)k * C + c) * R + r) * S + s];
  return v;
}

// taps of class t: dh = ((a + R - 1) >> 1) + 1, dw likewise
__host__ __device__ __forceinline__ int64_t es_weight_planes_offset_d(int64_t n) { return (n * 4 + 255) / 256 * 256; }
__device__ __forceinline__ int sp_dh(int t, int R) { return (((t >> 1) + R - 1) >> 1) + 1; }
__device__ __forceinline__ int sp_dw(int t, int S) { return (((t & 1) + S - 1) >> 1) + 1; }

template <typename T>
__global__ void pack_subpixel_kernel(const float* __restrict__ w, int K, int C, int R, int S, int mode,
                                     const float* inv_scale, T* out) {
  int tap0[5];
  tap0[0] = 0;
  for (int t = 0; t < 4; ++t) tap0[t + 1] = tap0[t] + sp_dh(t, R) * sp_dw(t, S);
  const int taps = tap0[4];
  const int64_t n = (int64_t)K * C * taps;
  const float sc = inv_scale ? 1.f / inv_scale[0] : 1.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int k, c, tap;
    if (mode == 2) {   // class blocks [K][d][e][C]
      const int64_t kc = (int64_t)K * C;
      tap = 0;
      int t = (i >= tap0[1] * kc) + (i >= tap0[2] * kc) + (i >= tap0[3] * kc);
      const int64_t rem = i - tap0[t] * kc;
      const int nde = sp_dh(t, R) * sp_dw(t, S);
      k = (int)(rem / ((int64_t)nde * C));
      const int r2 = (int)(rem - (int64_t)k * nde * C);
      const int de = r2 / C;
      c = r2 - de * C;
      tap = tap0[t] + de;
    } else {           // [C][tap][K]
      c = (int)(i / ((int64_t)taps * K));
      const int r2 = (int)(i - (int64_t)c * taps * K);
      tap = r2 / K;
      k = r2 - tap * K;
    }
    const int t = (tap >= tap0[1]) + (tap >= tap0[2]) + (tap >= tap0[3]);
    const int de = tap - tap0[t], dw = sp_dw(t, S);
    const int dd = de / dw, ee = de - dd * dw;
    out[i] = from_f<T>(subpixel_weight(w, k, c, C, R, S, t, dd, ee) * sc);
  }
}

template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int K, int C, int R, int S, int mode,
                                   const float* inv_scale, const int32_t* col_perm, T* out) {
  const int64_t n = (int64_t)K * C * R * S;
  const float sc = inv_scale ? 1.f / inv_scale[0] : 1.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    // i indexes the OUTPUT layout
    int k, c, r, s;
    const uint32_t i32 = (uint32_t)i;   // n < 2^31 (host-checked): 32-bit index math
    if (mode == 0) {  // [K][R][S][C]
      uint32_t t = i32 / C; c = i32 - t * C; s = t % S; t /= S; r = t % R; k = t / R;
    } else {          // [C][R][S][K]
      uint32_t t = i32 / K; k = i32 - t * K; s = t % S; t /= S; r = t % R; c = t / R;
    }
    const int cs = col_perm ? col_perm[c] : c;
    out[i] = from_f<T>(w[(((int64_t)k * C + cs) * R + r) * S + s] * sc);
  }
}

// mode 1 without a column permutation is a transpose of the fp32 master viewed as [K][C*R*S]
// into [C*R*S][K]: through a 64 x 64 LDS tile both sides stay row-contiguous (the element-wise
// kernel above read the master with a stride of C*R*S floats: 74 us for the 21632 x 256 linear)
template <typename T>
__global__ void __launch_bounds__(256) pack_t_kernel(const float* __restrict__ w, int rows, int cols,
                                                     const float* inv_scale, T* __restrict__ out) {
  __shared__ float tile[64][65];
  const float sc = inv_scale ? 1.f / inv_scale[0] : 1.f;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 64; i += 4) {
    const int r = r0 + ty + i, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + i][tx] = w[(int64_t)r * cols + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 64; i += 4) {
    const int c = c0 + ty + i, r = r0 + tx;
    if (r < rows && c < cols) out[(int64_t)c * rows + r] = from_f<T>(tile[tx][ty + i] * sc);
  }
}

__global__ void unpack_grad_kernel(const float* __restrict__ dw, int K, int C, int R, int S,
                                   const int32_t* col_perm, float* grad, float beta) {
  const int64_t n = (int64_t)K * C * R * S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    // i indexes dw layout [K][R][S][C]
    uint32_t t = (uint32_t)i / C;
    const int c = (int)((uint32_t)i - t * C);
    const int s = t % S; t /= S; const int r = t % R; const int k = t / R;
    const int cs = col_perm ? col_perm[c] : c;
    float* g = grad + (((int64_t)k * C + cs) * R + r) * S + s;
    *g = (beta != 0.f ? beta * *g : 0.f) + dw[i];
  }
}
// same, and the packed accumulator is left zeroed for the next weight gradient (each element is
// read and cleared by the one thread that owns it): no zero-fill launch per weight gradient
__global__ void unpack_grad_clear_kernel(float* __restrict__ dw, int K, int C, int R, int S, float* grad,
                                         float beta) {
  const int64_t n = (int64_t)K * C * R * S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t t = (uint32_t)i / C;
    const int c = (int)((uint32_t)i - t * C);
    const int s = t % S; t /= S; const int r = t % R; const int k = t / R;
    float* g = grad + (((int64_t)k * C + c) * R + r) * S + s;
    const float v = dw[i];
    dw[i] = 0.f;
    *g = (beta != 0.f ? beta * *g : 0.f) + v;
  }
}
}  // namespace

extern "C" int es_pack_conv_weight(const float* w, int K, int C, int R, int S, int mode,
                                   const float* inv_scale, const int32_t* col_perm, void* out,
                                   es_dtype_t dt, es_stream_t stream) {
  ES_CHECK_ARG(mode >= 0 && mode <= 3, "pack: bad mode");
  if (mode >= 2) {
    ES_CHECK_ARG(col_perm == nullptr, "pack: sub-pixel modes take no column permutation");
    const int64_t n = (int64_t)K * C * es_subpixel_taps(R, S);
    ES_CHECK_ARG(n < (1ll << 31), "pack: weight too large");
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    if (dt == ES_F32)
      hipLaunchKernelGGL(pack_subpixel_kernel<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                         w, K, C, R, S, mode, inv_scale, (float*)out);
    else
      hipLaunchKernelGGL(pack_subpixel_kernel<bf16>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                         w, K, C, R, S, mode, inv_scale, (bf16*)out);
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  const int64_t n = (int64_t)K * C * R * S;
  ES_CHECK_ARG(n < (1ll << 31), "pack: weight too large");
  if (mode == 1 && col_perm == nullptr && (int64_t)C * R * S < 65535 * 64) {
    const int cols = C * R * S;
    const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((K + 63) / 64));
    if (dt == ES_F32)
      hipLaunchKernelGGL(pack_t_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, w, K, cols, inv_scale,
                         (float*)out);
    else
      hipLaunchKernelGGL(pack_t_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, w, K, cols, inv_scale,
                         (bf16*)out);
    ES_CHECK_LAUNCH();
    return ES_OK;
  }
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  if (dt == ES_F32)
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       w, K, C, R, S, mode, inv_scale, col_perm, (float*)out);
  else
    hipLaunchKernelGGL(pack_weight_kernel<bf16>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       w, K, C, R, S, mode, inv_scale, col_perm, (bf16*)out);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

// Split-fp32 planes of a packed fp32 weight (es_conv_set_f32_split(2)): every 32-element block g
// of the packing becomes 192 bytes at planes + 192 g: three planes of 32 bf16, x0 = rne(x),
// x1 = rne(x - x0), x2 = x - x0 - x1 (exact), position 8 u + j of a plane holding element
// 4 u + j (j < 4) or 16 + 4 u + j - 4 of the block: the k order of the ring kernels' A fragments.
__global__ void pack_planes_kernel(const float* __restrict__ w, int64_t nblk, bf16* __restrict__ planes) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nblk * 32; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = i >> 5;
    const int q = (int)(i & 31), u = q >> 3, j = q & 7;
    const float x = w[g * 32 + (j < 4 ? 4 * u + j : 16 + 4 * u + j - 4)];
    const bf16 h = (bf16)x;
    const float r = x - (float)h;
    const bf16 m = (bf16)r;
    const bf16 l = (bf16)(r - (float)m);
    bf16* o = planes + g * 96 + q;
    o[0] = h;
    o[32] = m;
    o[64] = l;
  }
}

extern "C" int64_t es_weight_planes_offset(int64_t n) { return (n * 4 + 255) / 256 * 256; }

namespace {
// Batched packing (es_pack_conv_weights): blockIdx.y = job; each thread computes packed element i
// with the element-wise kernels' index math and writes it in the job's dtype, and for split-fp32
// jobs also its three bf16 plane values (the inverse of pack_planes_kernel's k permutation: block
// position p -> plane slot 8 (p / 4) + p % 4 for p < 16, 8 ((p - 16) / 4) + 4 + p % 4 otherwise).
constexpr int PACK_MAXJ = 32;
struct PackJobs {
  es_pack_job_t j[PACK_MAXJ];
};
__global__ void __launch_bounds__(256) pack_batch_kernel(PackJobs jobs) {
  const es_pack_job_t& jb = jobs.j[blockIdx.y];
  const int K = jb.K, C = jb.C, R = jb.R, S = jb.S, mode = jb.mode;
  int tap0[5] = {0, 0, 0, 0, 0};
  int64_t n;
  if (mode >= 2) {
    for (int t = 0; t < 4; ++t) tap0[t + 1] = tap0[t] + sp_dh(t, R) * sp_dw(t, S);
    n = (int64_t)K * C * tap0[4];
  } else {
    n = (int64_t)K * C * R * S;
  }
  const int64_t nplan = jb.planes ? (n / 32) * 32 : 0;
  bf16* planes = (bf16*)((char*)jb.out + es_weight_planes_offset_d(n));
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v;
    if (mode >= 2) {
      int k, c, tap;
      if (mode == 2) {
        const int64_t kc = (int64_t)K * C;
        const int t = (i >= tap0[1] * kc) + (i >= tap0[2] * kc) + (i >= tap0[3] * kc);
        const int64_t rem = i - tap0[t] * kc;
        const int nde = sp_dh(t, R) * sp_dw(t, S);
        k = (int)(rem / ((int64_t)nde * C));
        const int r2 = (int)(rem - (int64_t)k * nde * C);
        const int de = r2 / C;
        c = r2 - de * C;
        tap = tap0[t] + de;
      } else {
        const int taps = tap0[4];
        c = (int)(i / ((int64_t)taps * K));
        const int r2 = (int)(i - (int64_t)c * taps * K);
        tap = r2 / K;
        k = r2 - tap * K;
      }
      const int t = (tap >= tap0[1]) + (tap >= tap0[2]) + (tap >= tap0[3]);
      const int de = tap - tap0[t], dw = sp_dw(t, S);
      const int dd = de / dw, ee = de - dd * dw;
      v = subpixel_weight(jb.w, k, c, C, R, S, t, dd, ee);
    } else {
      int k, c, r, s_;
      const uint32_t i32 = (uint32_t)i;
      if (mode == 0) {
        uint32_t t = i32 / C; c = i32 - t * C; s_ = t % S; t /= S; r = t % R; k = t / R;
      } else {
        uint32_t t = i32 / K; k = i32 - t * K; s_ = t % S; t /= S; r = t % R; c = t / R;
      }
      v = jb.w[(((int64_t)k * C + c) * R + r) * S + s_];
    }
    if (jb.dt == ES_BF16) {
      ((bf16*)jb.out)[i] = (bf16)v;
    } else {
      ((float*)jb.out)[i] = v;
      if (i < nplan) {
        const int p = (int)(i & 31);
        const int q = p < 16 ? 8 * (p >> 2) + (p & 3) : 8 * ((p - 16) >> 2) + 4 + (p & 3);
        const bf16 h = (bf16)v;
        const float rr = v - (float)h;
        const bf16 m = (bf16)rr;
        const bf16 l = (bf16)(rr - (float)m);
        bf16* o = planes + (i >> 5) * 96 + q;
        o[0] = h;
        o[32] = m;
        o[64] = l;
      }
    }
  }
}
}  // namespace

extern "C" int es_pack_conv_weights(const es_pack_job_t* jobs, int n, es_stream_t stream) {
  ES_CHECK_ARG(n >= 0 && (n == 0 || jobs != nullptr), "pack batch: bad job list");
  hipStream_t st = (hipStream_t)stream;
  PackJobs batch{};
  int nb = 0;
  int64_t maxn = 0;
  auto flush = [&]() -> int {
    if (nb == 0) return ES_OK;
    const int blocks = (int)std::min<int64_t>((maxn + 255) / 256, 512);
    hipLaunchKernelGGL(pack_batch_kernel, dim3(blocks, nb), dim3(256), 0, st, batch);
    ES_CHECK_LAUNCH();
    nb = 0;
    maxn = 0;
    return ES_OK;
  };
  for (int q = 0; q < n; ++q) {
    const es_pack_job_t& jb = jobs[q];
    ES_CHECK_ARG(jb.w && jb.out && jb.mode >= 0 && jb.mode <= 3 && jb.K > 0 && jb.C > 0 && jb.R > 0 && jb.S > 0,
                 "pack batch: bad job %d", q);
    ES_CHECK_ARG(jb.dt == ES_F32 || jb.dt == ES_BF16, "pack batch: job %d dtype", q);
    ES_CHECK_ARG(!jb.planes || jb.dt == ES_F32, "pack batch: planes need an fp32 packing (job %d)", q);
    const int64_t ne = (int64_t)jb.K * jb.C * (jb.mode >= 2 ? es_subpixel_taps(jb.R, jb.S) : jb.R * jb.S);
    ES_CHECK_ARG(ne < (1ll << 31), "pack batch: weight too large (job %d)", q);
    if (jb.mode == 1 && (int64_t)jb.C * jb.R * jb.S >= 4096) {
      // a large transpose (the wide linears): the LDS-tiled kernel, then its planes
      if (int rc = es_pack_conv_weight(jb.w, jb.K, jb.C, jb.R, jb.S, 1, nullptr, nullptr, jb.out, (es_dtype_t)jb.dt,
                                       stream))
        return rc;
      if (jb.planes)
        if (int rc = es_pack_weight_planes((const float*)jb.out, ne, jb.out, stream)) return rc;
      continue;
    }
    batch.j[nb++] = jb;
    maxn = std::max(maxn, ne);
    if (nb == PACK_MAXJ)
      if (int rc = flush()) return rc;
  }
  return flush();
}

extern "C" int es_pack_weight_planes(const float* packed, int64_t n, void* base, es_stream_t stream) {
  const int64_t nblk = n / 32;
  if (nblk == 0) return ES_OK;
  const int blocks = (int)std::min<int64_t>((nblk * 32 + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_planes_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, packed, nblk,
                     (bf16*)((char*)base + es_weight_planes_offset(n)));
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_unpack_conv_grad_clear(float* dw, int K, int C, int R, int S, float* grad, float beta,
                                         es_stream_t stream) {
  const int64_t n = (int64_t)K * C * R * S;
  ES_CHECK_ARG(n < (1ll << 31), "unpack: weight too large");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(unpack_grad_clear_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dw, K, C, R, S,
                     grad, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}

extern "C" int es_unpack_conv_grad(const float* dw, int K, int C, int R, int S,
                                   const int32_t* col_perm, float* grad, float beta,
                                   es_stream_t stream) {
  const int64_t n = (int64_t)K * C * R * S;
  ES_CHECK_ARG(n < (1ll << 31), "unpack: weight too large");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(unpack_grad_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, dw, K, C,
                     R, S, col_perm, grad, beta);
  ES_CHECK_LAUNCH();
  return ES_OK;
}
