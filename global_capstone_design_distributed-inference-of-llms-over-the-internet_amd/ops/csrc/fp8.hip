// FP8 (OCP e4m3fn) W8A8 decode GEMM for gfx950 - the "fp8 MFMA path" of the Llama-3-70B
// configuration (BASELINE.json config 5).
//
// The reference has no quantized path (bitsandbytes NF4/INT8 exists only in the vendored,
// unreachable Petals server: petals/server/block_utils.py, convert_block).  On MI355X the
// natural 8-bit format is OCP fp8 with the native MFMA v_mfma_f32_16x16x32_fp8_fp8:
//
//   y[m, n] = a_m * s_n * sum_k  q8(x)[m, k] * q8(W)[n, k]
//
//   * weights: per-output-channel scale s_n = max|W[n, :]| / 448, packed once (ops.pack_weight_fp8)
//       Wq[N/16][K/64][lane][16 B]:  lane = 16 q + c holds W[16 nt + c][64 kc + 32 s + 8 q + j]
//       at byte 8 s + j  -> one 16-B load per lane feeds TWO 16x16x32 fp8 MFMAs (s = 0, 1);
//   * activations: per-row scale a_m = max|x[m, :]| / 448, quantized from the packed bf16
//     decode activation (quant_absmax + quant_apply) into the same [K/64][MT][lane][16 B] order;
//   * half the weight bytes of the bf16 path: decode stays HBM-bound, so the fp8 GEMM streams
//     a 70B stage in half the time.  Loop structure = the bf16 one-group-per-workgroup kernel
//     (gemm.hip): 8 waves interleave k-groups, ping-pong weight registers, LDS combine,
//     fused epilogues (scales, SwiGLU on 16-row-interleaved gate/up, residual).
#include "common.h"
#include <type_traits>
#include <stdlib.h>

namespace mp {

typedef __attribute__((ext_vector_type(2))) long i64x2;

__device__ __forceinline__ f32x4 mfma_fp8x2(const u16x8& a, const u16x8& b, f32x4 c) {
  const i64x2 av = __builtin_bit_cast(i64x2, a), bv = __builtin_bit_cast(i64x2, b);
  c = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av[0], bv[0], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av[1], bv[1], c, 0, 0, 0);
}

// 4 floats -> 4 OCP e4m3 bytes (round to nearest even; inputs already within +-448)
__device__ __forceinline__ int pack4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

// Packed bf16 decode activation Ap[K/32][MT][64][8] (M rows) -> fp8 A8[K/64][MT][64][16 B]
// plus per-row scales (MT*16 floats; rows >= M get a scale too and are never stored).
// Two short launches over a (16-row tile, K slice) grid so the whole chip works on it:
//   phase 1: per-slice row absmax -> part[MT*16][NS]   (no atomics, nothing to re-zero)
//   phase 2: row scale = max over slices / 448, quantize this slice (slice 0 stores the scale).
constexpr int Q_NS = 32;  // K slices per 16-row tile

__global__ __launch_bounds__(256) void quant_absmax_kernel(const bf16_t* __restrict__ ap, float* __restrict__ part,
                                                           int K, int MT) {
  __shared__ float red[4][16];
  const int mt = blockIdx.x, sl = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nks = K >> 5, per = (nks + Q_NS - 1) / Q_NS;
  const int k0 = sl * per, k1 = min(k0 + per, nks);
  float m = 0.f;
  for (int ks = k0 + wid; ks < k1; ks += 4) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(ap + (((int64_t)ks * MT + mt) * 64 + lane) * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(bf2f(v[j])));
  }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  if (lane < 16) red[wid][lane] = m;
  __syncthreads();
  if (tid < 16) part[(mt * 16 + tid) * Q_NS + sl] = fmaxf(fmaxf(red[0][tid], red[1][tid]), fmaxf(red[2][tid], red[3][tid]));
}

__global__ __launch_bounds__(256) void quant_apply_kernel(const bf16_t* __restrict__ ap, const float* __restrict__ part,
                                                          uint8_t* __restrict__ a8, float* __restrict__ scale, int K,
                                                          int MT) {
  const int mt = blockIdx.x, sl = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 15;
  const float* pr = part + (mt * 16 + r) * Q_NS;
  float mx = 0.f;
#pragma unroll 8
  for (int i = 0; i < Q_NS; ++i) mx = fmaxf(mx, pr[i]);
  const float s = mx > 0.f ? mx * (1.f / 448.f) : 1.f;
  const float inv = 1.f / s;
  if (sl == 0 && wid == 0 && lane < 16) scale[mt * 16 + lane] = s;
  const int nch = K >> 6, per = (nch + Q_NS - 1) / Q_NS;
  const int c0 = sl * per, c1 = min(c0 + per, nch);
  for (int c = c0 + wid; c < c1; c += 4) {
    const u16x8 v0 = *reinterpret_cast<const u16x8*>(ap + (((int64_t)(2 * c) * MT + mt) * 64 + lane) * 8);
    const u16x8 v1 = *reinterpret_cast<const u16x8*>(ap + (((int64_t)(2 * c + 1) * MT + mt) * 64 + lane) * 8);
    float f[16];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = fminf(fmaxf(bf2f(v0[j]) * inv, -448.f), 448.f);
      f[8 + j] = fminf(fmaxf(bf2f(v1[j]) * inv, -448.f), 448.f);
    }
    int4 o;
    o.x = pack4_fp8(f[0], f[1], f[2], f[3]);
    o.y = pack4_fp8(f[4], f[5], f[6], f[7]);
    o.z = pack4_fp8(f[8], f[9], f[10], f[11]);
    o.w = pack4_fp8(f[12], f[13], f[14], f[15]);
    *reinterpret_cast<int4*>(a8 + (((int64_t)c * MT + mt) * 64 + lane) * 16) = o;
  }
}

// One launch instead of the two above: a 1024-thread workgroup per row loads the whole row
// (16-B pieces of the packed layout, all in flight at once), reduces its absmax in the block and
// writes the row's e4m3 bytes + scale.  Same scale and rounding as the pair above, bit for bit.
// The decode rows are few (M <= 64), so the two-phase grid's extra launch and its second read of
// the activation cost more than the 64-CU width of this one (r2 70B profile: 4.8 + 5.3 us per
// site for the pair).
template <int MAXC>
__global__ __launch_bounds__(1024) void quant_row_kernel(const bf16_t* __restrict__ ap, uint8_t* __restrict__ a8,
                                                        float* __restrict__ scale, int K, int MT) {
  __shared__ float red[16];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int nc = K >> 3;  // 8-element pieces of the row
  const int mt = row >> 4, r16 = row & 15;
  u16x8 v[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int i = min(tid + 1024 * j, nc - 1);  // piece i = k-slice i / 4, quarter i % 4
    v[j] = *reinterpret_cast<const u16x8*>(ap + apk_off(row, i * 8, MT));
  }
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(bf2f(v[j][e])));
  m = block_max(m, red);
  const float sc = m > 0.f ? m * (1.f / 448.f) : 1.f;
  const float inv = 1.f / sc;
  if (tid == 0) scale[row] = sc;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int i = tid + 1024 * j;
    if (i < nc) {
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fminf(fmaxf(bf2f(v[j][e]) * inv, -448.f), 448.f);
      int2 o;
      o.x = pack4_fp8(f[0], f[1], f[2], f[3]);
      o.y = pack4_fp8(f[4], f[5], f[6], f[7]);
      const int sl = i >> 2, q = i & 3;
      *reinterpret_cast<int2*>(a8 + (((int64_t)(sl >> 1) * MT + mt) * 64 + q * 16 + r16) * 16 + (sl & 1) * 8) = o;
    }
  }
}

// Row-major bf16 x[M, K] (stride xs) -> fp8 A8 + row scales, one 1024-thread workgroup per row.
// The fp8 decode path has its producers (attention, the gate/up SwiGLU epilogue) write row-major
// activations for this kernel: a row is one contiguous run (coalesced 16-B loads; the packed
// layout scatters a row over 16-B pieces 256 B apart, and the packed-input kernel above spends
// ~10 us per 28672-wide row set on that), and each thread writes one whole 16-B A8 lane slot
// (k 64c + 8q .. +7 and 64c + 32 + 8q .. +7 of its row).
template <int MAXC>
__global__ __launch_bounds__(1024) void quant_rows_kernel(const bf16_t* __restrict__ x, int64_t xs,
                                                         uint8_t* __restrict__ a8, float* __restrict__ scale, int K,
                                                         int MT) {
  __shared__ float red[16];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int np = K >> 4;  // (64-k chunk, quarter) pieces: 2 x 8 elements each
  const bf16_t* xr = x + (int64_t)row * xs;
  u16x8 v0[MAXC], v1[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int p = min(tid + 1024 * j, np - 1), c = p >> 2, q = p & 3;
    v0[j] = *reinterpret_cast<const u16x8*>(xr + c * 64 + q * 8);
    v1[j] = *reinterpret_cast<const u16x8*>(xr + c * 64 + 32 + q * 8);
  }
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fmaxf(fabsf(bf2f(v0[j][e])), fabsf(bf2f(v1[j][e]))));
  m = block_max(m, red);
  const float sc = m > 0.f ? m * (1.f / 448.f) : 1.f;
  const float inv = 1.f / sc;
  if (tid == 0) scale[row] = sc;
  const int mt = row >> 4, r16 = row & 15;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int p = tid + 1024 * j;
    if (p < np) {
      float f[16];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        f[e] = fminf(fmaxf(bf2f(v0[j][e]) * inv, -448.f), 448.f);
        f[8 + e] = fminf(fmaxf(bf2f(v1[j][e]) * inv, -448.f), 448.f);
      }
      int4 o;
      o.x = pack4_fp8(f[0], f[1], f[2], f[3]);
      o.y = pack4_fp8(f[4], f[5], f[6], f[7]);
      o.z = pack4_fp8(f[8], f[9], f[10], f[11]);
      o.w = pack4_fp8(f[12], f[13], f[14], f[15]);
      const int c = p >> 2, q = p & 3;
      *reinterpret_cast<int4*>(a8 + (((int64_t)c * MT + mt) * 64 + q * 16 + r16) * 16) = o;
    }
  }
}

constexpr int F8_GU_MAX = 4;  // 64-k chunks per wave group

template <int MT, int NT, int EPI, bool OPK>
__global__ __launch_bounds__(512) void gemm_fp8_kernel(const uint8_t* __restrict__ a8, const float* __restrict__ ascale,
                                                       const uint8_t* __restrict__ wq, const float* __restrict__ wscale,
                                                       bf16_t* __restrict__ y, int64_t ys,
                                                       const bf16_t* __restrict__ res, int64_t rs, int M, int N,
                                                       int K) {
  constexpr int GU = (MT * NT >= 8) ? 2 : 4;  // 64-k chunks per group (2 at the widest tile: VGPR cap)
  __shared__ __attribute__((aligned(16))) float red[8][MT * NT * 4][64];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int nch = K >> 6;
  const int ngroups = nch / GU;
  const int nt0 = blockIdx.x * NT;

  const uint8_t* wbase[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wbase[t] = wq + ((int64_t)(nt0 + t) * nch) * 1024 + lane * 16;
  const uint8_t* abase = a8 + lane * 16;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);

  u16x8 b0[NT][GU], b1[NT][GU], a[MT][GU];
#define F8_LOAD_B(dst, grp)                                                                                  \
  _Pragma("unroll") for (int t = 0; t < NT; ++t) _Pragma("unroll") for (int u = 0; u < GU; ++u) dst[t][u] =   \
      __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wbase[t] + (int64_t)((grp) * GU + u) * 1024));
#define F8_LOAD_A(grp)                                                                                       \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) _Pragma("unroll") for (int u = 0; u < GU; ++u) a[mt][u] = \
      *reinterpret_cast<const u16x8*>(abase + ((int64_t)((grp) * GU + u) * MT + mt) * 1024);
#define F8_MMA(bb)                                                                                           \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) _Pragma("unroll") for (int u = 0; u < GU; ++u)           \
      _Pragma("unroll") for (int t = 0; t < NT; ++t) acc[mt][t] = mfma_fp8x2(a[mt][u], bb[t][u], acc[mt][t]);
  int g = wid;
  if (g < ngroups) {
    F8_LOAD_B(b0, g)
  }
  while (g < ngroups) {
    F8_LOAD_A(g)
    if (g + 8 < ngroups) {
      F8_LOAD_B(b1, g + 8)
      F8_MMA(b0)
    } else {
      F8_MMA(b0)
      break;
    }
    g += 8;
    F8_LOAD_A(g)
    if (g + 8 < ngroups) {
      F8_LOAD_B(b0, g + 8)
      F8_MMA(b1)
    } else {
      F8_MMA(b1)
      break;
    }
    g += 8;
  }
#undef F8_LOAD_B
#undef F8_LOAD_A
#undef F8_MMA

#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid][(mt * NT + t) * 4 + r][lane] = acc[mt][t][r];
  __syncthreads();
  for (int i = wid; i < MT * NT * 4; i += 8) {
    const int mt = i / (NT * 4), t = (i / 4) % NT, r = i & 3;
    const int row = mt * 16 + q * 4 + r;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += red[w][i][lane];
    if (row >= M) continue;
    const float as = ascale[row];
    if constexpr (EPI == 1) {
      if (t & 1) continue;  // up tile consumed with its gate tile
      float up = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) up += red[w][i + 4][lane];
      const int gcol = (nt0 + t) * 16 + c;
      const float gg = round_bf(s * as * wscale[gcol]);
      const float uu = round_bf(up * as * wscale[gcol + 16]);
      const float act = round_bf(gg / (1.f + __expf(-gg)));
      const int ncol = ((nt0 + t) >> 1) * 16 + c;
      const int64_t yo = OPK ? apk_off(row, ncol, MT) : (int64_t)row * ys + ncol;
      y[yo] = f2bf(act * uu);
    } else {
      const int col = (nt0 + t) * 16 + c;
      float v = s * as * wscale[col];
      if constexpr (EPI == 2) v = round_bf(v) + bf2f(res[(int64_t)row * rs + col]);
      y[(int64_t)row * ys + col] = f2bf(v);
    }
  }
}

template <int MT>
static int launch_gemm_fp8(const void* a8, const float* as, const void* wq, const float* ws, void* y, int64_t ys,
                           const void* res, int64_t rs, int M, int N, int K, int epi, int opk, hipStream_t stream) {
  const int ntiles = N / 16;
  const bool two = epi == 1 || (ntiles % 2 == 0 && ntiles / 2 >= 256);
#define F8_LAUNCH(NT_, EPI_, OPK_)                                                                              \
  hipLaunchKernelGGL((gemm_fp8_kernel<MT, NT_, EPI_, OPK_>), dim3(ntiles / NT_), dim3(512), 0, stream,           \
                     (const uint8_t*)a8, as, (const uint8_t*)wq, ws, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K)
  if (epi == 1) {
    if (ntiles % 2) return -2;
    if (opk) { F8_LAUNCH(2, 1, true); } else { F8_LAUNCH(2, 1, false); }
  } else if (opk) {
    return -3;
  } else if (epi == 2) {
    if (two) { F8_LAUNCH(2, 2, false); } else { F8_LAUNCH(1, 2, false); }
  } else {
    if (two) { F8_LAUNCH(2, 0, false); } else { F8_LAUNCH(1, 0, false); }
  }
#undef F8_LAUNCH
  return 0;
}

// ---------------------------------------------------------------------------------------
// Balanced ring form (the fp8 twin of gemm.hip's "rw" kernel): one 4-wave workgroup per CU owns
// a contiguous run of ceil / floor (tiles / CUs) column tiles (SwiGLU: gate/up tile PAIRS) and
// all of K; the waves take interleaved 64-k chunks through a 2-deep register ring holding both
// operands, then the 4 partial tiles are summed through LDS (in passes of at most 32 quads:
// the Llama-3-70B gate/up workgroup owns 14 tiles = 56 quads) and the scale / SwiGLU /
// residual epilogue runs.  The one-group kernel above gives the 70B gate/up (3584 tiles) 1792
// two-tile workgroups in 7 rounds over the CUs; here each CU streams its 7 pairs in one go.
constexpr int F8RW_WAVES = 4;
// A-fragment load; scripts/fp8_lab.hip overrides it to ablate the activation stream
#ifndef MP_F8_LOAD_A
#define MP_F8_LOAD_A(p) (*reinterpret_cast<const u16x8*>(p))
#endif
constexpr int F8RW_QC = 32;  // quads per combine pass (LDS: 4 waves x 32 x 1 KiB)

// ring depth: the largest of 8 / 4 / 2 slots (powers of two divide the per-wave chunk counts
// of the 70B shapes, 32 and 112) whose operands fit ~200 VGPRs (accumulators sit in AGPRs)
template <int MT, int NT>
constexpr int f8rw_depth() {
  return 4 * (MT + NT) * 8 <= 200 ? 8 : (4 * (MT + NT) * 4 <= 200 ? 4 : 2);
}

template <int MT, int NT, int EPI, bool OPK>
__device__ __forceinline__ void f8rw_body(const uint8_t* __restrict__ a8, const float* __restrict__ ascale,
                                          const uint8_t* __restrict__ wq, const float* __restrict__ wscale,
                                          bf16_t* __restrict__ y, int64_t ys, const bf16_t* __restrict__ res,
                                          int64_t rs, int M, int K, int tile0, f32x4* red) {
  constexpr int R = f8rw_depth<MT, NT>();
  constexpr int Q = MT * NT;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int nch = K >> 6;
  const int cnt = (nch + F8RW_WAVES - 1) / F8RW_WAVES;
  const uint8_t* wb = wq + ((int64_t)tile0 * nch) * 1024 + lane * 16;
  const uint8_t* ab = a8 + lane * 16;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);
  u16x8 ra[R][MT], rb[R][NT];
#define F8RW_LOAD(s, i)                                                                                      \
  {                                                                                                          \
    const int k_ = min(wid + F8RW_WAVES * (i), nch - 1);                                                     \
    _Pragma("unroll") for (int t = 0; t < NT; ++t) rb[s][t] =                                                \
        __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wb + ((int64_t)t * nch + k_) * 1024));    \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) ra[s][mt] =                                            \
        MP_F8_LOAD_A(ab + ((int64_t)k_ * MT + mt) * 1024);                                                   \
  }
#pragma unroll
  for (int s = 0; s < R; ++s) F8RW_LOAD(s, s)
  for (int i0 = 0; i0 < cnt; i0 += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if (wid + F8RW_WAVES * (i0 + s) < nch) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[mt][t] = mfma_fp8x2(ra[s][mt], rb[s][t], acc[mt][t]);
      }
      F8RW_LOAD(s, i0 + s + R)
    }
  }
#undef F8RW_LOAD
  // combine + epilogue in passes of QC quads (EPI 1: gate/up quads pair up inside a pass)
  constexpr int QC = Q < F8RW_QC ? Q : F8RW_QC;
#pragma unroll
  for (int p0 = 0; p0 < Q; p0 += QC) {
    if (p0 > 0) __syncthreads();  // the previous pass finished reading red
#pragma unroll
    for (int qd = p0; qd < p0 + QC && qd < Q; ++qd) red[(wid * QC + qd - p0) * 64 + lane] = acc[qd / NT][qd % NT];
    __syncthreads();
    for (int qd = p0 + wid; qd < p0 + QC && qd < Q; qd += F8RW_WAVES) {
      const int mt = qd / NT, t = qd % NT, tile = tile0 + t;
      if (EPI == 1 && (t & 1)) continue;  // up tile: consumed with its gate tile
      f32x4 v = red[(qd - p0) * 64 + lane], up = (f32x4)(0.f);
#pragma unroll
      for (int w = 1; w < F8RW_WAVES; ++w) v += red[(w * QC + qd - p0) * 64 + lane];
      if constexpr (EPI == 1) {
#pragma unroll
        for (int w = 0; w < F8RW_WAVES; ++w) up += red[(w * QC + qd + 1 - p0) * 64 + lane];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + q * 4 + r;
        if (row >= M) continue;
        const float as = ascale[row];
        if constexpr (EPI == 1) {
          const int gcol = tile * 16 + c;
          const float gg = round_bf(v[r] * as * wscale[gcol]);
          const float uu = round_bf(up[r] * as * wscale[gcol + 16]);
          const float act = round_bf(gg / (1.f + __expf(-gg)));
          const int ncol = (tile >> 1) * 16 + c;
          const int64_t yo = OPK ? apk_off(row, ncol, MT) : (int64_t)row * ys + ncol;
          y[yo] = f2bf(act * uu);
        } else {
          const int col = tile * 16 + c;
          float o = v[r] * as * wscale[col];
          if constexpr (EPI == 2) o = round_bf(o) + bf2f(res[(int64_t)row * rs + col]);
          y[(int64_t)row * ys + col] = f2bf(o);
        }
      }
    }
  }
}

template <int MT, int NTB, int NTS, int EPI, bool OPK>
__global__ __launch_bounds__(256) void gemm_fp8_rw_kernel(const uint8_t* __restrict__ a8,
                                                          const float* __restrict__ ascale,
                                                          const uint8_t* __restrict__ wq,
                                                          const float* __restrict__ wscale, bf16_t* __restrict__ y,
                                                          int64_t ys, const bf16_t* __restrict__ res, int64_t rs,
                                                          int M, int K, int n_big) {
  constexpr int QB = MT * NTB < F8RW_QC ? MT * NTB : F8RW_QC;
  __shared__ __attribute__((aligned(16))) f32x4 red[F8RW_WAVES * QB * 64];
  const int b = blockIdx.x;
  if (b < n_big) {
    f8rw_body<MT, NTB, EPI, OPK>(a8, ascale, wq, wscale, y, ys, res, rs, M, K, b * NTB, red);
  } else {
    f8rw_body<MT, NTS, EPI, OPK>(a8, ascale, wq, wscale, y, ys, res, rs, M, K, n_big * NTB + (b - n_big) * NTS, red);
  }
}

static int f8_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    n = v;
  }
  return n;
}

template <int MT, int NTB, int NTS>
static int launch_gemm_fp8_rw_cfg(const void* a8, const float* as, const void* wq, const float* ws, void* y, int64_t ys,
                                  const void* res, int64_t rs, int M, int K, int epi, bool opk, int G, int n_big,
                                  hipStream_t stream) {
#define F8RW(EPI_, OPK_)                                                                                          \
  hipLaunchKernelGGL((gemm_fp8_rw_kernel<MT, NTB, NTS, EPI_, OPK_>), dim3(G), dim3(256), 0, stream,               \
                     (const uint8_t*)a8, as, (const uint8_t*)wq, ws, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, \
                     n_big)
  if (epi == 1) {
    if constexpr (NTB % 2 == 0 && NTS % 2 == 0) {
      if (opk) { F8RW(1, true); } else { F8RW(1, false); }
    } else {
      return 1;
    }
  } else if (opk) {
    return -3;
  } else if (epi == 2) {
    F8RW(2, false);
  } else {
    F8RW(0, false);
  }
#undef F8RW
  return 0;
}

// Widths built: SwiGLU 2..14 tiles in pairs (7 pairs = the 70B gate/up on 256 CUs), plain 1..4.
template <int MT>
static int launch_gemm_fp8_rw(const void* a8, const float* as, const void* wq, const float* ws, void* y, int64_t ys,
                              const void* res, int64_t rs, int M, int N, int K, int epi, int opk, hipStream_t stream) {
  const int step = epi == 1 ? 2 : 1;
  const int units = (N / 16) / step;
  if ((N / 16) % step || units == 0) return 1;
  const int G = units < f8_num_cus() ? units : f8_num_cus();
  const int base = units / G, rem = units % G;
  const int ntb = (base + (rem ? 1 : 0)) * step;
  const int n_big = rem ? rem : G;
#define F8RWC(B_, S_) \
  return launch_gemm_fp8_rw_cfg<MT, B_, S_>(a8, as, wq, ws, y, ys, res, rs, M, K, epi, opk, G, n_big, stream)
  if (epi == 1) {
    switch (ntb) {
      case 2: if (rem) return 1; F8RWC(2, 2);
      case 4: F8RWC(4, 2);
      case 6: F8RWC(6, 4);
      case 8: F8RWC(8, 6);
      case 14: if (rem) return 1; F8RWC(14, 14);
      default: return 1;
    }
  }
  switch (ntb) {
    case 1: F8RWC(1, 1);
    case 2: F8RWC(2, 1);
    case 3: F8RWC(3, 2);
    case 4: F8RWC(4, 3);
    default: return 1;
  }
#undef F8RWC
}

// ---------------------------------------------------------------------------------------
// Split-K ring form (kind 2; the fp8 twin of gemm.hip's "rwk"): for the narrow 70B projections
// (o, down: N = 8192 -> 512 tiles, two per CU with all of K) every CU streams the whole fp8
// activation block (down: 64 x 28672 B) for 32 weight columns.  A workgroup here owns NT tiles
// and 1/S of K (C x S = #CUs) and writes an unscaled fp32 partial slab; a second launch sums the
// S slabs in order and applies a_scale[row] * w_scale[col] (+ residual).
template <int MT, int NT>
__global__ __launch_bounds__(256) void gemm_fp8_rwk_kernel(const uint8_t* __restrict__ a8,
                                                           const uint8_t* __restrict__ wq, float* __restrict__ part,
                                                           int M, int N, int K, int S) {
  constexpr int R = f8rw_depth<MT, NT>();
  constexpr int Q = MT * NT;
  constexpr int QC = Q < F8RW_QC ? Q : F8RW_QC;
  __shared__ __attribute__((aligned(16))) f32x4 red[F8RW_WAVES * QC * 64];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = blockIdx.x / S, sp = blockIdx.x - cg * S;
  const int tile0 = cg * NT;
  const int nch = K >> 6;
  const int k0 = (int)((int64_t)sp * nch / S), k1 = (int)((int64_t)(sp + 1) * nch / S);
  const int cnt = (k1 - k0 + F8RW_WAVES - 1) / F8RW_WAVES;
  const uint8_t* wb = wq + ((int64_t)tile0 * nch) * 1024 + lane * 16;
  const uint8_t* ab = a8 + lane * 16;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);
  u16x8 ra[R][MT], rb[R][NT];
#define F8K_LOAD(s, i)                                                                                       \
  {                                                                                                          \
    const int k_ = min(k0 + wid + F8RW_WAVES * (i), k1 - 1);                                                 \
    _Pragma("unroll") for (int t = 0; t < NT; ++t) rb[s][t] =                                                \
        __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wb + ((int64_t)t * nch + k_) * 1024));    \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) ra[s][mt] =                                            \
        MP_F8_LOAD_A(ab + ((int64_t)k_ * MT + mt) * 1024);                                                   \
  }
#pragma unroll
  for (int s = 0; s < R; ++s) F8K_LOAD(s, s)
  for (int i0 = 0; i0 < cnt; i0 += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if (k0 + wid + F8RW_WAVES * (i0 + s) < k1) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[mt][t] = mfma_fp8x2(ra[s][mt], rb[s][t], acc[mt][t]);
      }
      F8K_LOAD(s, i0 + s + R)
    }
  }
#undef F8K_LOAD
  float* slab = part + (int64_t)sp * M * N;
  const int cl = lane & 15, q = lane >> 4;
#pragma unroll
  for (int p0 = 0; p0 < Q; p0 += QC) {
    if (p0 > 0) __syncthreads();
#pragma unroll
    for (int qd = p0; qd < p0 + QC && qd < Q; ++qd) red[(wid * QC + qd - p0) * 64 + lane] = acc[qd / NT][qd % NT];
    __syncthreads();
    for (int qd = p0 + wid; qd < p0 + QC && qd < Q; qd += F8RW_WAVES) {
      f32x4 v = red[(qd - p0) * 64 + lane];
#pragma unroll
      for (int w = 1; w < F8RW_WAVES; ++w) v += red[(w * QC + qd - p0) * 64 + lane];
      const int mt = qd / NT, col = (tile0 + qd % NT) * 16 + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + q * 4 + r;
        if (row < M) slab[(int64_t)row * N + col] = v[r];
      }
    }
  }
}

template <int EPI, int S>
__global__ __launch_bounds__(256) void fp8_splitk_reduce_kernel(const float* __restrict__ part, int M, int N,
                                                                const float* __restrict__ ascale,
                                                                const float* __restrict__ wscale,
                                                                bf16_t* __restrict__ y, int64_t ys,
                                                                const bf16_t* __restrict__ res, int64_t rs) {
  const int row = blockIdx.y;
  const int col = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (col >= N) return;
  // all slab / scale / residual loads in flight before the first add (S <= 8 by the launcher)
  const float as = ascale[row];
  const f32x4 w0 = *reinterpret_cast<const f32x4*>(wscale + col), w1 = *reinterpret_cast<const f32x4*>(wscale + col + 4);
  u16x8 rv = (u16x8)(0);
  if constexpr (EPI == 2) rv = *reinterpret_cast<const u16x8*>(res + (int64_t)row * rs + col);
  f32x4 p0[S], p1[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const float* pp = part + ((int64_t)s * M + row) * N + col;
    p0[s] = *reinterpret_cast<const f32x4*>(pp);
    p1[s] = *reinterpret_cast<const f32x4*>(pp + 4);
  }
  f32x4 a0 = (f32x4)(0.f), a1 = (f32x4)(0.f);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    a0 += p0[s];
    a1 += p1[s];
  }
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = (j < 4 ? a0[j] : a1[j - 4]) * as * (j < 4 ? w0[j] : w1[j - 4]);
    if constexpr (EPI == 2) v = round_bf(v) + bf2f(rv[j]);
    o[j] = f2bf(v);
  }
  *reinterpret_cast<u16x8*>(y + (int64_t)row * ys + col) = o;
}

template <int MT>
static int launch_gemm_fp8_rwk(const void* a8, const float* as, const void* wq, const float* ws, void* y, int64_t ys,
                               const void* res, int64_t rs, int M, int N, int K, int epi, int opk, float* part,
                               int64_t part_bytes, hipStream_t stream) {
  if (epi == 1 || opk || part == nullptr || N % 2048) return 1;
  const int tiles = N / 16, C0 = f8_num_cus(), nch = K / 64;
  int nt = 0, S = 0;
  for (int cand : {8, 4, 2}) {
    if (tiles % cand || (cand == 8 && 4 * MT * 8 > 128)) continue;
    const int C = tiles / cand, sp = C0 / C;
    if (sp >= 2 && sp <= 8 && nch >= 4 * sp) { nt = cand; S = sp; break; }
  }
  if (nt == 0 || (int64_t)S * M * N * 4 > part_bytes) return 1;
  const dim3 g1((tiles / nt) * S);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, g1, dim3(256), 0, stream, (const uint8_t*)a8, (const uint8_t*)wq, part, M, N, K, S);
  };
  if (nt == 8) {
    if constexpr (4 * MT * 8 <= 128) go(gemm_fp8_rwk_kernel<MT, 8>);
  } else if (nt == 4) {
    go(gemm_fp8_rwk_kernel<MT, 4>);
  } else {
    go(gemm_fp8_rwk_kernel<MT, 2>);
  }
  const dim3 g2(N / 2048, M);
  auto reduce = [&](auto epi_c) {
    constexpr int E = decltype(epi_c)::value;
#define MP_F8R(S_)                                                                                              \
  hipLaunchKernelGGL((fp8_splitk_reduce_kernel<E, S_>), g2, dim3(256), 0, stream, part, M, N, as, ws, (bf16_t*)y, \
                     ys, (const bf16_t*)res, rs)
    switch (S) {
      case 2: MP_F8R(2); break;
      case 3: MP_F8R(3); break;
      case 4: MP_F8R(4); break;
      case 5: MP_F8R(5); break;
      case 6: MP_F8R(6); break;
      case 7: MP_F8R(7); break;
      default: MP_F8R(8); break;
    }
#undef MP_F8R
  };
  if (epi == 2) reduce(std::integral_constant<int, 2>{});
  else reduce(std::integral_constant<int, 0>{});
  return 0;
}

// 0 = one-group kernel, 1 = balanced ring kernel where it applies (M > 16; default); the autotuner
// (ops.autotune_fp8) sets it through mp_fp8_set_kernel
static int g_fp8_kernel = 1;

}  // namespace mp

extern "C" void mp_fp8_set_kernel(int kind) { mp::g_fp8_kernel = kind; }

// part: >= ceil(M/16) * 16 * Q_NS floats of scratch
extern "C" int mp_quant_act_fp8(const void* ap, void* a8, float* scale, float* part, int M, int K,
                                hipStream_t stream) {
  using namespace mp;
  if (M <= 0) return 0;
  if (K % 64) return -1;
  const int MT = (M + 15) / 16;
  const int per = (K / 8 + 1023) / 1024;
  if (per <= 4) {
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(M), dim3(1024), 0, stream, (const bf16_t*)ap, (uint8_t*)a8, scale, K, MT);
    };
    if (per <= 1) launch(quant_row_kernel<1>);
    else if (per <= 2) launch(quant_row_kernel<2>);
    else launch(quant_row_kernel<4>);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(quant_absmax_kernel, dim3(MT, Q_NS), dim3(256), 0, stream, (const bf16_t*)ap, part, K, MT);
  hipLaunchKernelGGL(quant_apply_kernel, dim3(MT, Q_NS), dim3(256), 0, stream, (const bf16_t*)ap, part, (uint8_t*)a8,
                     scale, K, MT);
  return (int)hipGetLastError();
}

extern "C" int mp_quant_rows_fp8(const void* x, int64_t xs, void* a8, float* scale, int M, int K,
                                 hipStream_t stream) {
  using namespace mp;
  if (M <= 0) return 0;
  if (K % 64 || xs % 8) return -1;
  const int MT = (M + 15) / 16;
  const int per = (K / 16 + 1023) / 1024;
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(M), dim3(1024), 0, stream, (const bf16_t*)x, xs, (uint8_t*)a8, scale, K, MT);
  };
  if (per <= 1) launch(quant_rows_kernel<1>);
  else if (per <= 2) launch(quant_rows_kernel<2>);
  else if (per <= 4) launch(quant_rows_kernel<4>);
  else return -2;
  return (int)hipGetLastError();
}

// a8/as: quant_act_fp8 output for M rows; wq/ws: pack_weight_fp8 output for W[N, K].
// kind: 0 = one-group kernel, 1 = balanced ring kernel (M > 16), 2 = split-K ring kernel + reduce
// launch (M > 16, epilogue 0 / 2, needs part: fp32 scratch of part_bytes), -1 = the start-up default
extern "C" int mp_gemm_fp8(const void* a8, const float* as, const void* wq, const float* ws, void* y, int64_t ys,
                           const void* res, int64_t rs, int M, int N, int K, int epilogue, int out_packed, int kind,
                           float* part, int64_t part_bytes, hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  if (M == 0) return 0;
  if (M > 64 || K % (64 * F8_GU_MAX) || N % 16) return -1;
  int rc;
  if (kind == 2 && M > 16) {
    if (M <= 32) rc = launch_gemm_fp8_rwk<2>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, part, part_bytes, stream);
    else if (M <= 48) rc = launch_gemm_fp8_rwk<3>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, part, part_bytes, stream);
    else rc = launch_gemm_fp8_rwk<4>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, part, part_bytes, stream);
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
    kind = 1;  // not covered: the balanced ring kernel
  }
  if ((kind < 0 ? g_fp8_kernel : kind) == 1 && M > 16) {
    if (M <= 32) rc = launch_gemm_fp8_rw<2>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, stream);
    else if (M <= 48) rc = launch_gemm_fp8_rw<3>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, stream);
    else rc = launch_gemm_fp8_rw<4>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, stream);
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if (M <= 16) rc = launch_gemm_fp8<1>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, stream);
  else if (M <= 32) rc = launch_gemm_fp8<2>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, stream);
  else if (M <= 48) rc = launch_gemm_fp8<3>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, stream);
  else rc = launch_gemm_fp8<4>(a8, as, wq, ws, y, ys, res, rs, M, N, K, epilogue, out_packed, stream);
  if (rc) return rc;
  return (int)hipGetLastError();
}
