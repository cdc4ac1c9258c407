// Row-split decode GEMM ("mw") for 65..256 rows on gfx950 - the wide-batch form.
//
// The ring kernels (gemm_kernels.h) give one workgroup ALL rows of a column group and split K over
// its 4 waves: at 256 rows every workgroup then takes in the whole 256 x K activation block (2 MB
// at K = 4096) for 192-384 KB of weights, and 256 accumulator AGPRs cap the group at 4 column
// tiles - measured slower than hipBLASLt (profiles/r4d: gate/up 116 vs 60 us).  Here the 4 waves
// split the ROWS instead (wave w owns row tiles [MTW w, MTW (w + 1))) and each walks all of the
// split's k-slices through its own register ring (A: its MTW fragments, B: the group's NT weight
// fragments, R slots in flight); the four waves read the same weight fragments together, so
// three of the four come from L2.  (A first version staged the weights once per workgroup
// through LDS with one barrier per 2 k-slices: latency-bound at 3-5x hipBLASLt, profiles/r4f.)
//
//   * K may be split over S workgroups of the same column group (ks0..ks1): S == 1 runs the
//     decode epilogues in the kernel (row-scaled consumer, packed SwiGLU, residual-stream
//     producer - tile_epilogue, every quad owned by exactly one wave, no cross-wave reduction);
//     S > 1 writes fp32 partial slabs [S][M][N] that a reduce launch sums in split order and
//     finishes with the same epilogue (splitk_reduce_kernel, splitk_swiglu_kernel below);
//   * the last column group may be partial (tiles past N clamp their loads and are not stored).
#pragma once
#include <string.h>

#include "gemm_kernels.h"

namespace mp {

constexpr int MW_KC = 2;  // (geometry granularity: a split keeps at least 2 x MW_KC k-slices)

// Register ring depth: 4 slots of one k-slice (A: MTW fragments, B: NT) while they fit ~160 VGPRs.
template <int MTW, int NT>
constexpr int mw_depth() { return 16 * (MTW + NT) <= 160 ? 4 : 2; }

template <int MTW, int NT, int EPI, bool OPK>
__global__ __launch_bounds__(256) void gemm_mw_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                      bf16_t* __restrict__ y, int64_t ys,
                                                      const bf16_t* __restrict__ res, int64_t rs,
                                                      float* __restrict__ part, int M, int N, int K, int S,
                                                      int tiles, const EpiArgs ep) {
  // EPI -1: partial slabs only (S > 1); else the epilogue runs here (S == 1)
  constexpr int R = mw_depth<MTW, NT>();
  __shared__ u64 rs_part[SS_PG][SS_ROWS];
  __shared__ float rs_lds[SS_ROWS];
  clear_other(ep);
  RowScale<(EPI >= 0 && EPI < 2), 4> rsc;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x / S, sp = blockIdx.x - c * S;
  const int tile0 = c * NT;
  const int nks = K >> 5;
  const int ks0 = (int)((int64_t)sp * nks / S), ks1 = (int)((int64_t)(sp + 1) * nks / S);
  const int cnt = ks1 - ks0;  // every wave walks every k-slice of the split, over its own rows
  const int mta = ep.mt_out;  // row tiles of the packed activation (a runtime stride)
  const int mt0 = wid * MTW;
  const bf16_t* xl = x + lane * 8;
  const bf16_t* wl = wp + lane * 8;
  int trow[NT];  // clamped column tiles (a partial last group re-reads its last tile, never stores it)
#pragma unroll
  for (int t = 0; t < NT; ++t) trow[t] = min(tile0 + t, tiles - 1);

  f32x4 acc[MTW][NT];
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);
  u16x8 ra[R][MTW], rb[R][NT];
  // the 4 waves read the same weight fragments at about the same time: default cache policy, so
  // the other three get them from L2 (a non-temporal load would not leave them there)
#define MW_LOAD(s_, i_)                                                                                   \
  {                                                                                                       \
    const int k_ = ks0 + min((i_), cnt - 1);                                                              \
    _Pragma("unroll") for (int t = 0; t < NT; ++t) rb[s_][t] =                                            \
        *reinterpret_cast<const u16x8*>(wl + (((int64_t)trow[t] * nks + k_) << 9));                       \
    _Pragma("unroll") for (int mt = 0; mt < MTW; ++mt) ra[s_][mt] =                                       \
        load_a_rows(xl + (((int64_t)k_ * mta + min(mt0 + mt, mta - 1)) << 9), lane, (mt0 + mt) * 16 + (lane & 15) < M); \
  }
#pragma unroll
  for (int s = 0; s < R; ++s) MW_LOAD(s, s)
  rsc.load(ep, wp);
  for (int i0 = 0; i0 < cnt; i0 += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if (i0 + s < cnt) {
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16(ra[s][mt], rb[s][t], acc[mt][t]);
      }
      MW_LOAD(s, i0 + s + R)
    }
  }
#undef MW_LOAD
  if constexpr (EPI < 0) {
    // fp32 partial slab of split sp: rows < M of this wave's tiles, columns of the group's tiles
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (tile0 + t >= tiles) continue;
        const int col = (tile0 + t) * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = (mt0 + mt) * 16 + (lane >> 4) * 4 + r;
          if (row < M) part[((int64_t)sp * M + row) * N + col] = acc[mt][t][r];
        }
      }
  } else {
    rsc.finish(ep, rs_part, rs_lds);
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (tile0 + t >= tiles) continue;
        if (EPI == 1 && (t & 1)) continue;  // up tile: consumed with its gate tile
        tile_epilogue<MTW, EPI, OPK>(mt0 + mt, tile0 + t, acc[mt][t], EPI == 1 ? acc[mt][(t + 1) % NT] : acc[mt][t],
                                     y, ys, res, rs, M, lane, ep, rs_lds, nullptr);
      }
  }
}

// Split-K reduce with the SwiGLU epilogue (gate / up tiles interleaved in 16-column blocks, as the
// ring kernels' EPI 1): output column oc of row r = silu(gate) * up with gate at column
// 32 (oc / 16) + oc % 16 of the slabs and up 16 columns further, both row-scaled (fused-norm
// consumer) and rounded as tile_epilogue does; row-major or packed (opk) output of N / 2 columns.
template <int S>
__global__ __launch_bounds__(256) void splitk_swiglu_kernel(const float* __restrict__ part, int M, int N,
                                                            bf16_t* __restrict__ y, int64_t ys, int opk,
                                                            const EpiArgs ep) {
  constexpr int CPT = 4;
  __shared__ float s_rs;
  const int row = blockIdx.y;
  const int oc = (blockIdx.x * 256 + threadIdx.x) * CPT;
  float sc = 1.f;
  if (ep.ss_in != nullptr) {
    if (threadIdx.x < 64) {
      u64 t = threadIdx.x < SS_NSH ? ep.ss_in[threadIdx.x * SS_ROWS + row] : 0ull;
#pragma unroll
      for (int o2 = 32; o2 > 0; o2 >>= 1) t += __shfl_xor(t, o2, 64);
      if (threadIdx.x == 0) s_rs = rsqrtf((float)t * (1.f / SS_FX) * ep.inv_k + ep.eps);
    }
    __syncthreads();
    sc = s_rs;
  }
  if (oc >= N / 2) return;
  const int gc = (oc >> 4) * 32 + (oc & 15);
  f32x4 pg[S], pu[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const float* pp = part + ((int64_t)s * M + row) * N + gc;
    pg[s] = *reinterpret_cast<const f32x4*>(pp);
    pu[s] = *reinterpret_cast<const f32x4*>(pp + 16);
  }
  f32x4 g = (f32x4)(0.f), u = (f32x4)(0.f);
#pragma unroll
  for (int s = 0; s < S; ++s) {  // fixed slab order: deterministic
    g += pg[s];
    u += pu[s];
  }
  u16x4 o;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const float gg = round_bf(g[j] * sc);
    const float a = round_bf(gg / (1.f + __expf(-gg)));
    o[j] = f2bf(a * round_bf(u[j] * sc));
  }
  if (opk)
    *reinterpret_cast<u16x4*>(y + apk_off(row, oc, ep.mt_out)) = o;
  else
    *reinterpret_cast<u16x4*>(y + (int64_t)row * ys + oc) = o;
}

// Geometry of the mw form for a shape: the column-group width NT and split count S with the
// lowest modelled time - per wave of workgroups the larger of the intake per CU (activation
// slice + the 4 waves' weight reads, the L2 -> CU path at ~64 B / clk) and the MFMA issue of one
// wave (MTW x NT quads x k-slices, 16 clk each), plus the slab round trip of a split (S x M x N
// fp32 written and read, ~3 KB / clk for the chip).  MPAMD_MW="NTxS" pins it (ablation).  nt = 0: no form fits.
static inline void mw_choose(int tiles, int nks, int M, int N, int MTW, int C0, int nt_max_s1, int& nt, int& S) {
  static const int pin_nt = [] { const char* v = getenv("MPAMD_MW"); return v ? atoi(v) : 0; }();
  static const int pin_s = [] {
    const char* v = getenv("MPAMD_MW");
    const char* xp = v ? strchr(v, 'x') : nullptr;
    return xp ? atoi(xp + 1) : 0;
  }();
  static constexpr int kNT[3] = {8, 6, 4};  // wider groups spill the register ring (12 / 16: scratch)
  nt = S = 0;
  double best = 1e30;
  for (int cand : kNT) {
    if (4 * MTW * cand > 256) continue;  // accumulators within 256 AGPRs
    if (pin_nt && cand != pin_nt) continue;
    const int C = (tiles + cand - 1) / cand;
    for (int s = 1; s <= 8; ++s) {
      if (pin_s && s != pin_s) continue;
      if (nks / s < 2 * MW_KC) break;
      if (s > 1 && (int64_t)s * M * N * 4 > RWK_SLAB_BYTES) break;
      if (s > 1 && C * s > C0) break;  // split only to fill the chip
      if (s == 1 && cand > nt_max_s1) continue;
      const double ks = (double)nks / s;
      // bytes into the CU per k-slice / (64 B / clk): the M-row activation slice + 4 waves x NT KiB
      const double intake = ks * ((double)M + 64.0 * cand);
      const double mfma = (double)MTW * cand * ks * 16.0;
      const double waves = (double)((C * s + C0 - 1) / C0);
      double t = waves * (intake > mfma ? intake : mfma);
      if (s > 1) t += 2.0 * s * M * (double)N * 4.0 / 3200.0;
      if (t < best) { best = t; nt = cand; S = s; }
    }
  }
}

// 1 if the mw form covers the shape / epilogue (no launch).
static inline int mw_ok(int N, int K, int epi, bool opk) {
  if (N % 32 || K % (32 * 2 * MW_KC) || epi == 2) return 0;
  return epi == 1 ? ((N / 16) % 2 == 0) : !opk;
}

template <int MTW>
static int launch_gemm_mw(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                          int N, int K, int epi, bool opk, const EpiArgs& ep, void* ws, hipStream_t stream) {
  if (!mw_ok(N, K, epi, opk)) return 1;
  const int tiles = N / 16, nks = K / 32, C0 = sk_num_cus();
  int nt = 0, S = 0;
  mw_choose(tiles, nks, M, N, MTW, C0, 8, nt, S);
  if (nt == 0 || (S > 1 && ws == nullptr)) return 1;
  float* part = S > 1 ? (float*)((char*)ws + (int64_t)SK_MAX_GROUPS * sizeof(int) + SK_ZERO_BYTES +
                                 (int64_t)SK_MAX_BLOCKS * 2 * SK_MAX_S * 64 * sizeof(float))
                      : nullptr;
  const dim3 g1(((tiles + nt - 1) / nt) * S);
#define MW_GO(NT_, EPI_, OPK_)                                                                              \
  hipLaunchKernelGGL((gemm_mw_kernel<MTW, NT_, EPI_, OPK_>), g1, dim3(256), 0, stream, (const bf16_t*)x,  \
                     (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, part, M, N, K, S, tiles, ep)
#define MW_NT(NT_)                                        \
  if (S > 1) {                                            \
    MW_GO(NT_, -1, false);                                \
  } else if (epi == 1) {                                  \
    if (opk) { MW_GO(NT_, 1, true); } else { MW_GO(NT_, 1, false); } \
  } else if (epi == 3) {                                  \
    MW_GO(NT_, 3, false);                                 \
  } else {                                                \
    MW_GO(NT_, 0, false);                                 \
  }
  switch (nt) {
    case 8: MW_NT(8) break;
    case 6: MW_NT(6) break;
    default: MW_NT(4) break;
  }
#undef MW_NT
#undef MW_GO
  if (S > 1) {
    if (epi == 1) {
      const dim3 g2((N / 2 + 1023) / 1024, M);
#define MW_SW(S_) \
  hipLaunchKernelGGL((splitk_swiglu_kernel<S_>), g2, dim3(256), 0, stream, part, M, N, (bf16_t*)y, ys, (int)opk, ep)
      switch (S) {
        case 2: MW_SW(2); break;
        case 3: MW_SW(3); break;
        case 4: MW_SW(4); break;
        case 5: MW_SW(5); break;
        case 6: MW_SW(6); break;
        case 7: MW_SW(7); break;
        default: MW_SW(8); break;
      }
#undef MW_SW
    } else {
      const dim3 g2((N + 256 * SKR_CPT - 1) / (256 * SKR_CPT), M);
      launch_splitk_reduce(S, epi, g2, stream, part, M, N, y, ys, res, rs, ep);
    }
  }
  return 0;
}

}  // namespace mp
