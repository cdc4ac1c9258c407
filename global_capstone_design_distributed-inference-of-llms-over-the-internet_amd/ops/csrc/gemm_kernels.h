// Weight-streaming skinny GEMM for decode on gfx950 (survey K3/K8/K10/K12) - the kernel
// templates and their launchers, shared by gemm.hip (M <= 64 bf16 entry point), gemm_wide.hip
// (65..128 rows) and gemm_w8.hip (fp8 weights): three translation units compile in parallel.
//
//   y[M, N'] = epilogue( x[M, K] . W[N, K]^T )        M <= 64 (decode micro-batches)
//
// The reference runs q/k/v/o/gate/up/down/lm_head as separate cuBLAS GEMV/GEMMs
// (reference petals/llama/block.py:88-90, :151, :237; src/llama_partition.py:470) and does
// the SwiGLU product and residual adds as further elementwise kernels.  At decode sizes the
// projections are bound by streaming W from HBM once, so this kernel is organised around
// that stream:
//
//   * W is stored PRE-PACKED in MFMA fragment order (ops.pack_weight):
//       Wp[n/16][k/32][lane][8],  lane = 16*q + c  holds  W[16*nt + c][32*ks + 8*q + j]
//     so the B operand of every v_mfma_f32_16x16x32_bf16 is ONE contiguous 1 KiB read
//     (64 lanes x 16 B), and a wave walking K streams a contiguous region: perfectly
//     coalesced, non-temporal (read once), straight to VGPRs (guide: "GEMV / M <= 16" row).
//   * x (A operand) is either row-major (lane (r, q) reads 16 B of row r at k offset 8q:
//     16 rows x 64 B per wave-instruction, TA-heavy) or - on the decode path - PACKED in the
//     same fragment order by its producer kernel (RMSNorm, attention, the SwiGLU epilogue):
//       Ap[k/32][m/16][lane][8]  -> every A fragment is one contiguous 1 KiB read too.
//   * one workgroup = 8 waves over NT column tiles (16 cols each) x all of K; the waves take
//     interleaved groups of U k-slices and their partial tiles are combined through LDS
//     (no atomics, no second pass); B is double-buffered in registers across groups.
//   * fused epilogues: 0 = store bf16; 1 = SwiGLU for a gate/up weight whose rows are
//     interleaved in 16-row blocks [g16 u16 g16 u16 ...] (tile 2t = gate, 2t+1 = up;
//     output N/2 columns); 2 = y = bf16(bf16(acc) + residual); 3 = the residual-stream
//     producer of the fused-norm decode path: r = bf16(bf16(acc) + residual) stored in place
//     (row-major) AND packed (the next GEMM's A operand), and sum(r^2) per row accumulated
//     into an fp32 vector with atomics (16 lanes reduce a row first).
//   * RMSNorm folded away (EpiArgs::ss_in): the consumer GEMMs (qkv, gate/up) read the RAW
//     residual stream with the norm weight folded into their packed weight columns
//     (W' = W diag(g)), and scale accumulator row r by rsqrt(ss[r] / H + eps) in the
//     epilogue - RMSNorm(x) W^T = rs * (x (gW)^T).  No normalisation kernel runs on the
//     decode path (2 launches per layer fewer).
#pragma once
#include "common.h"
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>

// Store form of the split-K slabs of the reduce-launch path (dirty lines left in the XCD L2s are
// written back at the kernel's end, before the next launch starts: MI355X_MICROARCH boundary row,
// + dirty bytes / 6 TB/s).  0 plain; 1 write-through (sc1; vs plain: 64 sessions 4.286 -> 4.264 ms,
// batch 1 2.682 -> 2.671, 70B fp8 16.89 -> 16.84, profiles/r6sc1); 2 nontemporal (default; vs sc1:
// 64 sessions 4.250 -> 4.199, 70B fp8 16.92 -> 16.84, 4 of 4 interleaved pairs each, profiles/r6nt)
#ifndef MP_SLAB_ST
#define MP_SLAB_ST 2
#endif

namespace mp {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// A-fragment load (16 B per lane); scripts/gemm_lab.hip overrides it to ablate the A stream.
#ifndef MP_LOAD_A_FRAG
#define MP_LOAD_A_FRAG(p) (*reinterpret_cast<const u16x8*>(p))
#endif

// A fragment of a packed-activation lane whose row (lane & 15 of its m-tile) may lie past the M
// real rows: such a lane loads its tile's row-0 chunk instead (the address lane 16 q of the same
// wave-instruction reads), so at batch 1 a fragment load touches 4 x 16 B instead of 1 KiB of
// L2 lines (the 16-row tile otherwise streams as many activation bytes as the N = 4096
// projections stream weights).  Rows >= M of the accumulators then hold row-0 products, which
// no epilogue stores (every epilogue, slab and row statistic is limited to rows < M).  No
// branch, no select on the loaded value: the ring's vmcnt accounting is unchanged.
__device__ __forceinline__ u16x8 load_a_rows(const bf16_t* p, int lane, bool row_ok) {
  return MP_LOAD_A_FRAG(row_ok ? p : p - (lane & 15) * 8);
}

// Epilogue side inputs/outputs of the fused-norm decode path (see the header).
//
// Row statistics travel as FIXED-POINT sums of squares: every element contributes
// round(x^2 * 2^20) as a 64-bit integer, so the sum is exact and independent of the order in
// which the 16-lane groups / workgroups / atomics add up (bitwise reproducible, and equal to
// what the stage-entry kernel computes for the same rows: a model split over stages gives
// the same bits as one stage).  Producers add into NSH shards [NSH][SS_ROWS] (shard = block % NSH:
// same-address atomics serialise at the memory side, 256 adders on one row cost ~20 us);
// consumers sum the shards of every row once per workgroup into LDS.
constexpr int SS_NSH = 32;
constexpr int SS_ROWS = 256;        // rows per shard: decode steps of up to 256 sessions
constexpr int SS_PG = 512 / SS_ROWS;  // shard groups a RowScale reduction uses at most (512 threads)
constexpr float SS_FX = 1048576.f;  // 2^20
typedef unsigned long long u64;
static_assert(SS_NSH == QP_SS_NSH && SS_ROWS == QP_SS_ROWS && SS_FX == QP_SS_FX,
              "row statistics layout shared with the attention kernels' qkv_part_load8");

struct EpiArgs {
  bf16_t* ap;          // EPI 3: packed copy of the output rows (mt_out row tiles)
  u64* ss_out;         // EPI 3: [SS_NSH][SS_ROWS] fixed-point sums of squares (atomics)
  u64* ss_zero;        // cleared by block 0 at kernel start: the other norm buffer
  const u64* ss_in;    // non-null: scale accumulator row r by rsqrt(sum_r / K + eps)
  float inv_k;
  float eps;
  int mt_out;
  const float* wsc;    // fp8 weights (W8A16 kernels): per-output-column dequantization scales
  int rot = 0;         // rotate each workgroup's k walk (rw_krot; flags bit 10, chosen per shape)
  const uint8_t* xsc = nullptr;  // MX activations (gemm_mx.hip): e8m0 block scales [K/128][MT][64]
};

// fp8 (OCP e4m3) weight fragment -> bf16 MFMA B operand (exact: every e4m3 value is a bf16
// value): the W8A16 form of the ring kernels streams 1 byte per weight and keeps bf16
// activations (no activation quantization launches between the layer's GEMMs).  8 bytes per lane
// per k-slice: byte j = W[col][32 ks + 8 q + j], the bf16 fragment's element order.  Four
// v_cvt_scalef32_pk_bf16_fp8 (unit scale) per fragment; the per-column dequantization scale
// multiplies the accumulators once, after the K loop.
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ u16x8 f8w_to_bf16(const u32x2& raw) {
  u16x8 r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const u16x2 lo = __builtin_bit_cast(u16x2, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(raw[h], 1.0f, false));
    const u16x2 hi = __builtin_bit_cast(u16x2, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(raw[h], 1.0f, true));
    r[4 * h + 0] = lo[0];
    r[4 * h + 1] = lo[1];
    r[4 * h + 2] = hi[0];
    r[4 * h + 3] = hi[1];
  }
  return r;
}

// MX decode GEMM (gemm_mx.hip): one 16x16x128 block-scaled e4m3 MFMA.  ``a`` / ``b``: the lane's 32
// bytes (four consecutive 32-k slices of the W8A16 fragment order, 8 bytes each); ``sa``: the e8m0
// scale this lane supplies in byte 0 (gfx950 takes the scale of 32-block b of a row from lane
// 16 b + r, mx_quant_kernel writes it there); the weight's e8m0 is 127 (= 1): its per-column scale is applied
// to the accumulators after the loop.
typedef __attribute__((ext_vector_type(8))) unsigned u32x8;
typedef __attribute__((ext_vector_type(8))) int i32x8_t;
__device__ __forceinline__ f32x4 mfma_mx(const u32x8& a, const u32x8& b, unsigned sa, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(__builtin_bit_cast(i32x8_t, a), __builtin_bit_cast(i32x8_t, b),
                                                          c, 0, 0, 0, (int)sa, 0, 127);
}

__device__ __forceinline__ u64 fx_sq(float f) { return (u64)__float2ull_rn(f * f * SS_FX); }

__device__ __forceinline__ void clear_other(const EpiArgs& ep) {
  if (ep.ss_zero != nullptr && blockIdx.x == 0) {
    for (int i = threadIdx.x; i < SS_NSH * SS_ROWS; i += blockDim.x) ep.ss_zero[i] = 0ull;
  }
}

// Consumer side (EPI 0 / 1 only; compiled out of the producer epilogues), in two halves around
// the main loop: thread t owns row t % R and shard group t / R (R: the step's row window, G =
// threads / R groups), loads its SS_NSH / G shard words right AFTER the kernel's first weight loads
// and folds them into one 64-bit partial (in-order vmcnt: waiting for them costs nothing beyond
// the first weight chunk the loop waits for anyway, and only 2 VGPRs stay live through the
// loop); the G partials of a row are reduced through LDS in the epilogue, after the main loop's
// last barrier.  Rows past the step's M read zeroed shards: their scale is never used.
template <bool ON, int NW = 8>
struct RowScale {
  // The step's rows use a power-of-two window R >= 16 x row tiles (at most SS_ROWS) and the
  // workgroup's threads form G = threads / R shard groups, so a small step spreads its 32 shard
  // words over more threads (batch 1: 16 rows x 16 groups, 2 loads a thread) while 256 rows
  // still fit (1 group of 256 at 4 waves).
  static constexpr int NT = NW * 64;
  static_assert(NT <= SS_PG * SS_ROWS, "shard partials fit the shared scratch");
  u64 v = 0;
  int R = SS_ROWS;
  __device__ __forceinline__ static int window(int mt_out) {
    int r = 16;
    while (r < 16 * mt_out && r < SS_ROWS) r <<= 1;
    return r;
  }
  __device__ __forceinline__ int groups() const { return NT / R < SS_NSH ? NT / R : SS_NSH; }
  __device__ __forceinline__ void load(const EpiArgs& ep, const void* any_valid) {
    if constexpr (ON) {
      R = window(ep.mt_out);
      const u64* src = ep.ss_in != nullptr ? ep.ss_in : reinterpret_cast<const u64*>(any_valid);
      const int tid = threadIdx.x, G = groups();
      const int row = tid % R, grp = tid / R;
      u64 t = 0;
      if (grp < G && row < 16 * ep.mt_out) {  // rows past the step's row tiles: never scaled, not loaded
        for (int j = 0; j < SS_NSH / G; ++j) t += src[ep.ss_in != nullptr ? (grp + G * j) * SS_ROWS + row : 0];
      }
      v = t;
    }
  }
  // every thread of the workgroup calls this (two barriers inside when ss_in is set)
  __device__ __forceinline__ void finish(const EpiArgs& ep, u64 (*part2)[SS_ROWS], float* rs) {
    if constexpr (ON) {
      if (ep.ss_in == nullptr) return;
      u64* part = &part2[0][0];
      const int tid = threadIdx.x, G = groups();
      if (tid / R < G) part[tid] = v;  // [grp][row] = grp * R + row = tid
      __syncthreads();
      if (tid < R) {
        u64 s = 0;
        for (int w = 0; w < G; ++w) s += part[w * R + tid];
        rs[tid] = rsqrtf((float)s * (1.f / SS_FX) * ep.inv_k + ep.eps);
      }
      __syncthreads();
    }
  }
};

template <int EPI>
__device__ __forceinline__ float row_scale(const EpiArgs& ep, const float* rs, int row) {
  if constexpr (EPI >= 2) return 1.f;
  return ep.ss_in != nullptr ? rs[row] : 1.f;
}

// sum over the 16 lanes that share lane >> 4 (one accumulator row of a 16x16 MFMA tile)
__device__ __forceinline__ u64 sum16(u64 v) { return sum16_u64(v); }

// EPI 3 store of one element (called by all 16 lanes of a row group together: sum16 inside).
// ``rv`` is the old residual value, PREFETCHED by the caller before its main loop: loaded here
// it would add one exposed memory round trip (~1.5 us) to every producer GEMM's tail.
__device__ __forceinline__ void epi3_store(const EpiArgs& ep, bf16_t* __restrict__ y, int64_t ys, int row, int col,
                                           float v, int c, bf16_t rv) {
  const bf16_t o = f2bf(round_bf(v) + bf2f(rv));
  y[(int64_t)row * ys + col] = o;
  ep.ap[apk_off(row, col, ep.mt_out)] = o;
  if (ep.ss_out == nullptr) return;  // (benchmark ablation only: the executor always passes ss_out)
  const u64 t = sum16(fx_sq(bf2f(o)));
  if (c == 0) atomicAdd(ep.ss_out + (blockIdx.x % SS_NSH) * SS_ROWS + row, t);
}

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                  0, 0, 0);
}

// Start offset of the k walk per workgroup (MP_RW_ROT, default on): every decode GEMM workgroup reads
// the SAME activation block, in lock-step from k-slice 0 up; rotating each workgroup's walk by a
// per-workgroup offset spreads the 256 concurrent A streams over the whole block (L2 channels)
// instead of one moving 16 KB window.  A bijection on the slices: every slice is still summed
// exactly once (the accumulation order per column group changes, deterministically).
// Per launch (EpiArgs::rot, flags bit 10) and chosen per shape by the start-up autotuners: it
// helped the Llama-2-7B and 70B fp8 shapes (profiles/r3_r, r3_s: 64 sessions 4.36 -> 4.32 ms, 70B
// 17.8 -> 17.3-17.4) and cost 2.4 % on Llama-3-8B's (r3_t), whose lock-step readers share L2 lines
// that a spread-out walk lets the weight stream evict.  -DMP_RW_ROT=0 compiles it out.
#ifndef MP_RW_ROT
#define MP_RW_ROT 1
#endif
__device__ __forceinline__ int rw_rot(int k, int rot, int n) {
  if constexpr (MP_RW_ROT == 0) return k;
  const int r = k + rot;
  return r >= n ? r - n : r;
}
__device__ __forceinline__ int rw_krot(int n, int on) {
  return (MP_RW_ROT && on) ? (int)((blockIdx.x * 37u) % (unsigned)n) : 0;
}

constexpr int GU_MAX = 4;  // k-slices (of 32) per wave group (x 16 B per lane per column tile)

template <int MT, int NT, int EPI, bool APK, bool OPK>
__global__ __launch_bounds__(512) void gemm_packed_kernel(const bf16_t* __restrict__ x, int64_t x_stride,
                                                          const bf16_t* __restrict__ wp, bf16_t* __restrict__ y,
                                                          int64_t y_stride, const bf16_t* __restrict__ res,
                                                          int64_t res_stride, int M, int N, int K,
                                                          const int* __restrict__ gate, const EpiArgs ep) {
  clear_other(ep);
  __shared__ u64 rs_part[SS_PG][SS_ROWS];
  __shared__ float rs_lds[SS_ROWS];
  RowScale<EPI < 2> rsc;
  // MoE expert gate (ops/moe.py): a device-side count of tokens routed to this expert; 0 ->
  // the whole grid exits before streaming any weight (output left as is, combine weight 0).
  // One uniform scalar load per workgroup keeps hipGraph-captured decode steps shape-static.
  if (gate != nullptr && *gate == 0) return;
  // fewer k-slices per group for the widest tiles keeps A + 2 x B + acc inside 256 VGPRs
  constexpr int GU = (MT * NT >= 6) ? 2 : 4;
  __shared__ __attribute__((aligned(16))) float red[8][MT * NT * 4][64];
  // wave id made provably uniform (readfirstlane): the group loop then compiles to scalar
  // branches instead of an exec-masked divergent loop around the MFMAs
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int nks = K >> 5;
  const int ngroups = nks / GU;
  const int nt0 = blockIdx.x * NT;

  const bf16_t* wbase[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wbase[t] = wp + ((int64_t)(nt0 + t) * nks) * 512 + lane * 8;

  // EPI 3: this wave's residual elements (slots i = wid + 8 j), in flight during the main loop
  constexpr int NSLOT = (MT * NT * 4 + 7) / 8;
  bf16_t rpre[NSLOT];
  if constexpr (EPI == 3) {
#pragma unroll
    for (int j = 0; j < NSLOT; ++j) {
      const int i = min(wid + 8 * j, MT * NT * 4 - 1);
      const int row = min((i / (NT * 4)) * 16 + q * 4 + (i & 3), M - 1);
      rpre[j] = res[(int64_t)row * res_stride + (nt0 + (i / 4) % NT) * 16 + c];
    }
  }

  // A rows >= M are clamped to a valid row (their accumulator rows are never stored): no
  // per-load branches, so hipcc can count vmcnt through the loop (guide §5 trap (c)).
  const bf16_t* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    if constexpr (APK) {
      xrow[mt] = x + ((int64_t)mt * 64 + lane) * 8;  // + slice * MT * 512
    } else {
      const int r = min(mt * 16 + c, M - 1);
      xrow[mt] = x + (int64_t)r * x_stride + 8 * q;
    }
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);

  // Ping-pong weight buffers (no register copies, which would force a vmcnt(0)), and the
  // A fragments of group g issued BEFORE the prefetch of group g+8: vmcnt retires loads in
  // issue order, so waiting for A leaves the weight prefetch in flight across the MFMAs.
  u16x8 b0[NT][GU], b1[NT][GU], a[MT][GU];
  const int grot = rw_krot(ngroups, ep.rot);
#define MP_LOAD_B(dst, grp)                                                                                   \
  _Pragma("unroll") for (int t = 0; t < NT; ++t) _Pragma("unroll") for (int u = 0; u < GU; ++u) dst[t][u] =    \
      __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wbase[t] + (int64_t)(rw_rot(grp, grot, ngroups) * GU + u) * 512));
#define MP_LOAD_A(grp)                                                                                        \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) _Pragma("unroll") for (int u = 0; u < GU; ++u) a[mt][u] =  \
      (APK ? load_a_rows(xrow[mt] + (int64_t)(rw_rot(grp, grot, ngroups) * GU + u) * MT * 512, lane, mt * 16 + (lane & 15) < M) \
           : MP_LOAD_A_FRAG(xrow[mt] + (int64_t)(rw_rot(grp, grot, ngroups) * GU * 32 + 32 * u)));
#define MP_MMA(bb)                                                                                            \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) _Pragma("unroll") for (int u = 0; u < GU; ++u)            \
      _Pragma("unroll") for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16(a[mt][u], bb[t][u], acc[mt][t]);
  int g = wid;
  if (g < ngroups) {
    MP_LOAD_B(b0, g)
  }
  rsc.load(ep, wp);
  while (g < ngroups) {
    MP_LOAD_A(g)
    if (g + 8 < ngroups) {
      MP_LOAD_B(b1, g + 8)
      MP_MMA(b0)
    } else {
      MP_MMA(b0)
      break;
    }
    g += 8;
    MP_LOAD_A(g)
    if (g + 8 < ngroups) {
      MP_LOAD_B(b0, g + 8)
      MP_MMA(b1)
    } else {
      MP_MMA(b1)
      break;
    }
    g += 8;
  }
#undef MP_LOAD_B
#undef MP_LOAD_A
#undef MP_MMA

  // ---- combine the 8 waves' partial tiles through LDS ----
  rsc.finish(ep, rs_part, rs_lds);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid][(mt * NT + t) * 4 + r][lane] = acc[mt][t][r];
  __syncthreads();
  // wave w finalises element slots i = w, w + 8, ... of the MT*NT*4 per-lane slots
#pragma unroll
  for (int j = 0; j < NSLOT; ++j) {
    const int i = wid + 8 * j;
    if (i >= MT * NT * 4) break;
    const int mt = i / (NT * 4), t = (i / 4) % NT, r = i & 3;
    const int row = mt * 16 + q * 4 + r;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += red[w][i][lane];
    if constexpr (EPI == 1) {
      if (t & 1) continue;  // the up tile is consumed by its gate tile
      float up = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) up += red[w][i + 4][lane];
      if (row < M) {
        const int ncol = ((nt0 + t) >> 1) * 16 + c;
        const float sc = row_scale<EPI>(ep, rs_lds, row);
        const float gg = round_bf(s * sc);
        const float a = round_bf(gg / (1.f + __expf(-gg)));
        const int64_t yo = OPK ? apk_off(row, ncol, MT) : (int64_t)row * y_stride + ncol;
        y[yo] = f2bf(a * round_bf(up * sc));
      }
    } else {
      if (row < M) {  // uniform over the 16 lanes of a row: sum16 in epi3_store is safe
        const int col = (nt0 + t) * 16 + c;
        float v = s * row_scale<EPI>(ep, rs_lds, row);
        if constexpr (EPI == 3) {
          epi3_store(ep, y, y_stride, row, col, v, c, rpre[j]);
        } else {
          if constexpr (EPI == 2) v = round_bf(v) + bf2f(res[(int64_t)row * res_stride + col]);
          y[(int64_t)row * y_stride + col] = f2bf(v);
        }
      }
    }
  }
}

template <int MT>
static int launch_gemm(const void* x, int64_t xs, const void* w, void* y, int64_t ys, const void* res, int64_t rs,
                       int M, int N, int K, int epi, int flags, const int* gate, const EpiArgs& ep,
                       hipStream_t stream) {
  const int ntiles = N / 16;
  // two column tiles per wave when there are enough workgroups to fill the 256 CUs
  const bool two = epi == 1 || (ntiles % 2 == 0 && ntiles / 2 >= 256);
  const bool apk = flags & 1, opk = flags & 2;
#define MP_LAUNCH(NT_, EPI_, APK_, OPK_)                                                                       \
  hipLaunchKernelGGL((gemm_packed_kernel<MT, NT_, EPI_, APK_, OPK_>), dim3(ntiles / NT_), dim3(512), 0, stream, \
                     (const bf16_t*)x, xs, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K, \
                     gate, ep)
  // Only the packed-activation form is instantiated: row-major callers pack x first
  // (mp_pack_act).  The row-major-A variant miscompiled at MT=1/NT=1 (ROCm 7.2, wrong
  // results with several k-groups per wave) and loses to the packed form anyway.
  if (!apk) return -4;
#define MP_APK(NT_, EPI_, OPK_) MP_LAUNCH(NT_, EPI_, true, OPK_);
  if (epi == 1) {
    if (ntiles % 2) return -2;
    if (opk) { MP_APK(2, 1, true) } else { MP_APK(2, 1, false) }
  } else if (opk) {
    return -3;  // packed output only for the SwiGLU epilogue (it feeds the down projection)
  } else if (epi == 2) {
    if (two) { MP_APK(2, 2, false) } else { MP_APK(1, 2, false) }
  } else if (epi == 3) {
    if (two) { MP_APK(2, 3, false) } else { MP_APK(1, 3, false) }
  } else {
    if (two) { MP_APK(2, 0, false) } else { MP_APK(1, 0, false) }
  }
#undef MP_APK
#undef MP_LAUNCH
  return 0;
}

// ---------------------------------------------------------------------------------------
// Stream-K form (M in 17..64, or any M when the caller gives a workspace).
//
// The one-group-per-workgroup kernel above leaves two things on the table at M = 32..64:
//   * tails: the grid is N/(16 NT) workgroups; 384 (qkv) or 688 (gate/up) workgroups on 256
//     CUs run 1.5 / 2.7 waves of workgroups, and at ~200 VGPRs only one fits per CU;
//   * activation re-reads: every workgroup reads all of x (M x K) for just NT column tiles,
//     so at M = 64 the L2->CU traffic of x is 2-4x the weight bytes.
// Here the grid is exactly one workgroup per CU and the work is the flat list of units
// (column group g of NT tiles, k-slice k), u = g * nks + k, cut into G equal contiguous
// ranges (stream-K): every CU streams the same number of weight bytes, a group may be split
// between consecutive workgroups, and with NT = 4 the activation traffic is 1/4 of the
// NT = 1 form.  Inside a workgroup the 8 waves take the units of a range round-robin in
// "chunks" of 8 consecutive k-slices (one per wave, chunks never straddle a group since
// nks % 8 == 0), through a D-deep register ring that holds BOTH operands of a k-slice:
// loads are issued D chunks ahead in consumption order, so in-order vmcnt never drains the
// ring (the A-before-B trick of the kernel above is not needed).
// Group boundaries: each wave parks its partial accumulators in LDS (one pending group at
// a time: nks >= 8 D), the next ring turn sums the 8 waves' partials and either runs the
// epilogue (group fully inside this range) or writes an fp32 slab; the last-arriving
// workgroup of a split group (agent-scope release/acquire + counter, guide §5 "In-launch
// split-K reduction") sums the slabs of all contributors in workgroup order
// (deterministic) and runs the epilogue.  The counter is re-zeroed by that reducer, so a
// zero-initialised workspace stays valid across launches and graph replays.
constexpr int SK_MAX_GROUPS = 1 << 15;
constexpr int SK_MAX_BLOCKS = 512;
constexpr int SK_MAX_S = 64;  // MT * NT * 4 accumulator slots per lane
constexpr int SK_ZERO_BYTES = 4 * 1024;  // zero A fragments (MT <= 4) for masked units

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// EPI 3 residual prefetch of one accumulator quad (4 rows x this lane's column)
template <int NT>
__device__ __forceinline__ u16x4 res_quad(const bf16_t* __restrict__ res, int64_t rs, int qd, int g, int M, int lane) {
  const int mt = qd / NT, t = qd % NT, c = lane & 15, q = lane >> 4;
  const int col = (g * NT + t) * 16 + c;
  u16x4 o;
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = res[(int64_t)min(mt * 16 + q * 4 + r, M - 1) * rs + col];
  return o;
}

// Epilogue of one accumulator quad (rows mt*16 + 4q .. +3 of column tile ``tile``, this lane's
// column); ``up`` is the matching up-projection quad for EPI 1.
template <int MT, int EPI, bool OPK>
__device__ __forceinline__ void tile_epilogue(int mt, int tile, const f32x4& v, const f32x4& up, bf16_t* __restrict__ y,
                                              int64_t ys, const bf16_t* __restrict__ res, int64_t rs, int M, int lane,
                                              const EpiArgs& ep, const float* rsl, const u16x4* rpv) {
  const int c = lane & 15, q = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = mt * 16 + q * 4 + r;
    if (row >= M) continue;  // uniform over the 16 lanes of a row (sum16 in epi3_store)
    const float sc = row_scale<EPI>(ep, rsl, row);
    if constexpr (EPI == 1) {
      const int ncol = (tile >> 1) * 16 + c;
      const float gg = round_bf(v[r] * sc);
      const float a = round_bf(gg / (1.f + __expf(-gg)));
      const int64_t yo = OPK ? apk_off(row, ncol, ep.mt_out) : (int64_t)row * ys + ncol;
      y[yo] = f2bf(a * round_bf(up[r] * sc));
    } else if constexpr (EPI == 3) {
      const bf16_t rv = rpv != nullptr ? (*rpv)[r] : res[(int64_t)row * rs + tile * 16 + c];
      epi3_store(ep, y, ys, row, tile * 16 + c, v[r] * sc, c, rv);
    } else {
      const int col = tile * 16 + c;
      float o = v[r] * sc;
      if constexpr (EPI == 2) o = round_bf(o) + bf2f(res[(int64_t)row * rs + col]);
      y[(int64_t)row * ys + col] = f2bf(o);
    }
  }
}

template <int MT, int NT, int EPI, bool OPK>
__device__ __forceinline__ void sk_epilogue(int qd, int g, const f32x4& v, const f32x4& up, bf16_t* __restrict__ y,
                                            int64_t ys, const bf16_t* __restrict__ res, int64_t rs, int M, int lane,
                                            const EpiArgs& ep, const float* rsl, const u16x4* rpv = nullptr) {
  tile_epilogue<MT, EPI, OPK>(qd / NT, g * NT + qd % NT, v, up, y, ys, res, rs, M, lane, ep, rsl, rpv);
}

// ---------------------------------------------------------------------------------------
// Shared-A form ("lds"): the 8 waves are KS = 8/CH k-splits x CH column groups. The CH waves
// of a k-split need the SAME activation fragments, so each stages 1/CH of a k-group's A block
// into LDS and all CH read it back with ds_read_b128. Global A traffic per weight byte drops by
// CH vs the one-group kernel, and the k reduction stays inside the workgroup (no split-group
// hand-off, which is what sank the all-column-split prototype in profiles/r1_gemm_lab.md).
// A is double-buffered in LDS (one barrier per k-group), B in registers, as in the kernels
// above; out-of-range k-groups of the last turn load a clamped group and skip the MFMAs so
// every wave runs the same barrier sequence.
template <int MT, int NT, int CH, int EPI, bool OPK>
__global__ __launch_bounds__(512) void gemm_lds_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                       bf16_t* __restrict__ y, int64_t ys,
                                                       const bf16_t* __restrict__ res, int64_t rs, int M, int N,
                                                       int K, const EpiArgs ep) {
  clear_other(ep);
  __shared__ u64 rs_part[SS_PG][SS_ROWS];
  __shared__ float rs_lds[SS_ROWS];
  RowScale<EPI < 2> rsc;
  constexpr int KS = 8 / CH;
  constexpr int NSL = (CH * MT * NT + 7) / 8;  // epilogue quads per wave
  u16x4 rpre[NSL];
  constexpr int GU = 2;               // k-slices (of 32) per group
  constexpr int F = GU * MT;          // A fragments (1 KiB) per group
  constexpr int FH = F / CH;          // fragments each wave of a k-split stages
  constexpr int Q = MT * NT;          // accumulator quads per lane
  constexpr int ABYTES = 2 * KS * F * 1024;
  constexpr int RBYTES = KS * CH * Q * 64 * 16;
  constexpr int LBYTES = ABYTES > RBYTES ? ABYTES : RBYTES;
  static_assert(F % CH == 0, "A group must split evenly over the column waves");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LBYTES];
  bf16_t* abuf = reinterpret_cast<bf16_t*>(smem);
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ksp = wid % KS, ch = wid / KS;
  const int nks = K >> 5, ngroups = nks / GU;
  const int niter = (ngroups + KS - 1) / KS;
  const int g0 = blockIdx.x * CH + ch;  // this wave's column group (NT tiles)

  const bf16_t* wbase[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wbase[t] = wp + ((int64_t)(g0 * NT + t) * nks) * 512 + lane * 8;
  const bf16_t* xl = x + lane * 8;
  if constexpr (EPI == 3) {
#pragma unroll
    for (int j = 0; j < NSL; ++j) {
      const int i = min(wid + 8 * j, CH * Q - 1);
      rpre[j] = res_quad<NT>(res, rs, i % Q, blockIdx.x * CH + i / Q, M, lane);
    }
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);

  u16x8 st[FH], b0[NT][GU], b1[NT][GU], a[MT][GU];
  const int grot = rw_krot(ngroups, ep.rot);
#define MP_GRP(it) rw_rot(min((it) * KS + ksp, ngroups - 1), grot, ngroups)
#define MP_LDA(it)                                                                                            \
  _Pragma("unroll") for (int f = 0; f < FH; ++f) st[f] =                                                     \
      *reinterpret_cast<const u16x8*>(xl + ((int64_t)MP_GRP(it) * F + ch * FH + f) * 512);
#define MP_LDB(dst, it)                                                                                       \
  _Pragma("unroll") for (int t = 0; t < NT; ++t) _Pragma("unroll") for (int u = 0; u < GU; ++u) dst[t][u] =    \
      __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wbase[t] + (int64_t)(MP_GRP(it) * GU + u) * 512));
#define MP_STA(buf)                                                                                           \
  _Pragma("unroll") for (int f = 0; f < FH; ++f) *reinterpret_cast<u16x8*>(                                 \
      abuf + (((buf) * KS + ksp) * F + ch * FH + f) * 512 + lane * 8) = st[f];
#define MP_RDA(buf)                                                                                           \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) _Pragma("unroll") for (int u = 0; u < GU; ++u) a[mt][u] =  \
      *reinterpret_cast<const u16x8*>(abuf + (((buf) * KS + ksp) * F + u * MT + mt) * 512 + lane * 8);
#define MP_MMA(bb, it)                                                                                        \
  if ((it) * KS + ksp < ngroups) {                                                                            \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) _Pragma("unroll") for (int u = 0; u < GU; ++u)          \
        _Pragma("unroll") for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16(a[mt][u], bb[t][u], acc[mt][t]);  \
  }
  MP_LDA(0)
  MP_LDB(b0, 0)
  rsc.load(ep, wp);
  for (int it = 0; it < niter; it += 2) {
    MP_STA(0)
    if (it + 1 < niter) {
      MP_LDA(it + 1)
      MP_LDB(b1, it + 1)
    }
    lds_barrier();
    MP_RDA(0)
    MP_MMA(b0, it)
    if (it + 1 >= niter) break;
    MP_STA(1)
    if (it + 2 < niter) {
      MP_LDA(it + 2)
      MP_LDB(b0, it + 2)
    }
    lds_barrier();
    MP_RDA(1)
    MP_MMA(b1, it + 1)
  }
#undef MP_GRP
#undef MP_LDA
#undef MP_LDB
#undef MP_STA
#undef MP_RDA
#undef MP_MMA
  lds_barrier();  // every wave is done reading A before the reduction buffer aliases it
  rsc.finish(ep, rs_part, rs_lds);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) red[((ksp * CH + ch) * Q + mt * NT + t) * 64 + lane] = acc[mt][t];
  lds_barrier();
#pragma unroll
  for (int j = 0; j < NSL; ++j) {
    const int i = wid + 8 * j;
    if (i >= CH * Q) break;
    const int chh = i / Q, qd = i % Q;
    if (EPI == 1 && (qd % NT) & 1) continue;  // up tile: consumed with its gate tile
    f32x4 v = (f32x4)(0.f), up = (f32x4)(0.f);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      v += red[((k * CH + chh) * Q + qd) * 64 + lane];
      if (EPI == 1) up += red[((k * CH + chh) * Q + qd + 1) * 64 + lane];
    }
    sk_epilogue<MT, NT, EPI, OPK>(qd, blockIdx.x * CH + chh, v, up, y, ys, res, rs, M, lane, ep, rs_lds,
                                  EPI == 3 ? &rpre[j] : nullptr);
  }
}

template <int MT, int NT, int CH>
static int launch_gemm_lds_cfg(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                               int N, int K, int epi, int flags, const EpiArgs& ep, hipStream_t stream) {
  if constexpr ((2 * MT) % CH != 0) {
    return 1;  // the A group does not split evenly over the column waves
  } else {
    const int ntiles = N / 16;
    const bool opk = flags & 2;
    if (ntiles % (CH * NT) || K % 64) return 1;
    if (opk && epi != 1) return -3;
    const dim3 grid(ntiles / (CH * NT));
#define MP_LL(EPI_, OPK_)                                                                                      \
  hipLaunchKernelGGL((gemm_lds_kernel<MT, NT, CH, EPI_, OPK_>), grid, dim3(512), 0, stream, (const bf16_t*)x,   \
                     (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K, ep)
    if (epi == 1) {
      if constexpr (NT % 2 == 0) {  // gate/up tile pairs must sit in one wave
        if (opk) { MP_LL(1, true); } else { MP_LL(1, false); }
      } else {
        return 1;
      }
    } else if (epi == 2) {
      MP_LL(2, false);
    } else if (epi == 3) {
      MP_LL(3, false);
    } else {
      MP_LL(0, false);
    }
#undef MP_LL
    return 0;
  }
}

// flags bits 5-6 pick (NT, CH): 0 = (2, 2), 1 = (2, 4), 2 = (1, 4), 3 = (4, 2)
template <int MT>
static int launch_gemm_lds(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                           int N, int K, int epi, int flags, const EpiArgs& ep, hipStream_t stream) {
  switch ((flags >> 5) & 3) {
    case 1: return launch_gemm_lds_cfg<MT, 2, 4>(x, w, y, ys, res, rs, M, N, K, epi, flags, ep, stream);
    case 2: return launch_gemm_lds_cfg<MT, 1, 4>(x, w, y, ys, res, rs, M, N, K, epi, flags, ep, stream);
    case 3: return launch_gemm_lds_cfg<MT, 4, 2>(x, w, y, ys, res, rs, M, N, K, epi, flags, ep, stream);
    default: return launch_gemm_lds_cfg<MT, 2, 2>(x, w, y, ys, res, rs, M, N, K, epi, flags, ep, stream);
  }
}

template <int MT, int NT, int D, int EPI, bool OPK>
__global__ __launch_bounds__(512) void gemm_sk_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                      bf16_t* __restrict__ y, int64_t ys, const bf16_t* __restrict__ res,
                                                      int64_t rs, int M, int N, int K, int* __restrict__ cnt,
                                                      f32x4* __restrict__ slab, int remap, const EpiArgs ep) {
  clear_other(ep);
  __shared__ u64 rs_part[SS_PG][SS_ROWS];
  __shared__ float rs_lds[SS_ROWS];
  RowScale<EPI < 2> rsc;
  constexpr int Q = MT * NT;  // accumulator quads (f32x4) per lane
  __shared__ __attribute__((aligned(16))) f32x4 red[8 * Q * 64 + 16];
  int* s_flag = reinterpret_cast<int*>(red + 8 * Q * 64);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int nks = K >> 5;
  const int U = ((N >> 4) / NT) * nks;
  // logical workgroup id: consecutive ranges (which share split groups) on the same XCD
  const int lb = ((G & 7) || !remap) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3);
  const int u0 = (int)((int64_t)lb * U / G), u1 = (int)((int64_t)(lb + 1) * U / G);
  const int c_first = u0 >> 3, nch = ((u1 - 1) >> 3) + 1 - c_first;
  auto start_of = [&](int b) { return (int)((int64_t)b * U / G); };
  auto block_of = [&](int u) { return (int)(((int64_t)(u + 1) * G - 1) / U); };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);
  u16x8 ra[D][MT], rb[D][NT];

  // Ring loads are unconditional (a conditional load makes hipcc fall back to vmcnt(0) before
  // every MFMA): units outside [u0, u1) - the ragged first/last chunk and the padding up to a
  // whole ring turn - load a clamped, valid weight address (an L2 hit) and a zero A fragment
  // from the workspace, so their MFMAs add exactly 0.
  const bf16_t* zero_a = reinterpret_cast<const bf16_t*>(cnt + SK_MAX_GROUPS);
#define SK_LOAD(s, cc)                                                                                      \
  {                                                                                                         \
    const int u_ = (cc) * 8 + wid;                                                                          \
    const bool act_ = u_ >= u0 && u_ < u1;                                                                  \
    const int uc_ = min(max(u_, u0), u1 - 1);                                                               \
    const int g_ = uc_ / nks, k_ = uc_ - g_ * nks;                                                          \
    _Pragma("unroll") for (int t = 0; t < NT; ++t) rb[s][t] = __builtin_nontemporal_load(                   \
        reinterpret_cast<const u16x8*>(wp + (((int64_t)(g_ * NT + t) * nks + k_) << 9) + lane * 8));        \
    const bf16_t* xa_ = act_ ? x + (((int64_t)k_ * MT) << 9) : zero_a;                                      \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) ra[s][mt] =                                            \
        load_a_rows(xa_ + (mt << 9) + lane * 8, lane, mt * 16 + (lane & 15) < M);                           \
  }

  // sum of the 8 waves' parked partials for quad qd (this lane)
  auto red_sum = [&](int qd) {
    f32x4 s = red[qd * 64 + lane];
#pragma unroll
    for (int w = 1; w < 8; ++w) s += red[(w * Q + qd) * 64 + lane];
    return s;
  };
  // EPI 3 (decode shapes; the launcher only picks this form when a range is at most one group
  // long, so every range spans <= 2 groups and any group finalised INSIDE the ring loop is a
  // split one): the in-loop reduce only writes slabs, keeping the epilogue's registers out of
  // the loop (it spilled otherwise), and the residual quads of the range's first / last group
  // - the only groups this workgroup can finalise - are loaded right after the loop, in flight
  // behind the ticket / slab hand-off.
  constexpr int NSQ = (Q + 7) / 8;
  u16x4 rp_first[NSQ], rp_last[NSQ];
  const int g_first = u0 / nks, g_last = (u1 - 1) / nks;
  auto load_rp = [&]() {
    if constexpr (EPI == 3) {
#pragma unroll
      for (int j = 0; j < NSQ; ++j) {
        rp_first[j] = res_quad<NT>(res, rs, min(wid + 8 * j, Q - 1), g_first, M, lane);
        rp_last[j] = res_quad<NT>(res, rs, min(wid + 8 * j, Q - 1), g_last, M, lane);
      }
    }
  };
  auto rp_of = [&](int g, int j) -> const u16x4* {
    if constexpr (EPI == 3) return g == g_first ? &rp_first[j] : (g == g_last ? &rp_last[j] : nullptr);
    return nullptr;
  };
  auto stage = [&]() {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        red[(wid * Q + mt * NT + t) * 64 + lane] = acc[mt][t];
        acc[mt][t] = (f32x4)(0.f);
      }
  };
  // Split groups: this workgroup's partial goes out as a write-through (sc1) fp32 slab right
  // away, but the hand-off (drain + arrival ticket) is deferred to the end of the range, so a
  // split head group never stalls the weight stream (one ticket episode per workgroup).
  // Guide §6 Guideline 16 R1: sc1 stores need no release fence; the reducer reads the slabs
  // with sc1 loads, which need no acquire.
  const __amdgpu_buffer_rsrc_t slab_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, (int)(SK_MAX_BLOCKS * 2 * Q * 64 * 16), 0x00020000);
  int split_g0 = -1, split_g1 = -1;  // split head / tail group of this range (uniform)
  bool rs_ready = false;             // row scales reduced (at the first group boundary; uniform)
  auto reduce = [&](int g, auto in_loop) {
    lds_barrier();
    if (!rs_ready) {
      rsc.finish(ep, rs_part, rs_lds);
      rs_ready = true;
    }
    constexpr bool no_epi = decltype(in_loop)::value && EPI == 3;
    const bool whole = g * nks >= u0 && (g + 1) * nks <= u1;
    bool done = false;
    if constexpr (!no_epi) {
      if (whole) {
#pragma unroll
        for (int j = 0; j < NSQ; ++j) {
          const int qd = wid + 8 * j;
          if (qd >= Q) break;
          if (EPI == 1 && (qd % NT) & 1) continue;  // up tile: consumed with its gate tile
          sk_epilogue<MT, NT, EPI, OPK>(qd, g, red_sum(qd), EPI == 1 ? red_sum(qd + 1) : (f32x4)(0.f), y, ys, res,
                                        rs, M, lane, ep, rs_lds, rp_of(g, j));
        }
        done = true;
      }
    }
    if (!done) {
      const int side = (u0 / nks == g) ? 0 : 1;
      if (side == 0) split_g0 = g; else split_g1 = g;
      for (int qd = wid; qd < Q; qd += 8)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, red_sum(qd)), slab_rsrc,
                                               (((lb * 2 + side) * Q + qd) * 64 + lane) * 16, 0, 16);
    }
    lds_barrier();  // red may be overwritten by the next stage()
  };
  auto finish_splits = [&]() {
    if (split_g0 < 0 && split_g1 < 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 slab stores landed
    lds_barrier();
    if (tid == 0) {
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int g = side ? split_g1 : split_g0;
        int last = 0;
        if (g >= 0) {
          const int bf = block_of(g * nks), bl = block_of((g + 1) * nks - 1);
          const int old = __hip_atomic_fetch_add(cnt + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last = old == bl - bf;
          if (last) __hip_atomic_store(cnt + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_flag[side] = last;
      }
    }
    lds_barrier();
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      if (!s_flag[side]) continue;
      const int g = side ? split_g1 : split_g0;
      const int bf = block_of(g * nks), bl = block_of((g + 1) * nks - 1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the slab loads below the ticket
#pragma unroll
      for (int j = 0; j < NSQ; ++j) {
        const int qd = wid + 8 * j;
        if (qd >= Q) break;
        if (EPI == 1 && (qd % NT) & 1) continue;
        f32x4 v = (f32x4)(0.f), up = (f32x4)(0.f);
        for (int b = bf; b <= bl; ++b) {  // fixed order: deterministic sums
          const int sd = (start_of(b) / nks == g) ? 0 : 1;
          const int base = ((b * 2 + sd) * Q) * 64;
          v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(slab_rsrc, ((base + qd * 64) + lane) * 16,
                                                                                0, 16));
          if (EPI == 1)
            up += __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(slab_rsrc, ((base + (qd + 1) * 64) + lane) * 16, 0, 16));
        }
        sk_epilogue<MT, NT, EPI, OPK>(qd, g, v, up, y, ys, res, rs, M, lane, ep, rs_lds, rp_of(g, j));
      }
    }
  };

  // prologue: fill the ring
  const int nch_pad = ((nch + D - 1) / D) * D;
#pragma unroll
  for (int s = 0; s < D; ++s) SK_LOAD(s, c_first + s)
  rsc.load(ep, wp);

  // group of a chunk (chunks never straddle groups; padding chunks clamp to the last one)
  auto chunk_group = [&](int cc) { return min(max(cc * 8, u0), u1 - 1) / nks; };
  int cur_g = chunk_group(c_first);
  bool pending = false;
  int pend_g = 0;
  for (int j0 = 0; j0 < nch_pad; j0 += D) {
    if (pending) {
      reduce(pend_g, std::true_type{});
      pending = false;
    }
#pragma unroll
    for (int s = 0; s < D; ++s) {
      const int cc = c_first + j0 + s;
      const int g = chunk_group(cc);
      if (g != cur_g) {  // at most one group boundary per ring turn (nks >= 8 D)
        stage();
        pending = true;
        pend_g = cur_g;
        cur_g = g;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16(ra[s][mt], rb[s][t], acc[mt][t]);
      SK_LOAD(s, cc + D)
    }
  }
#undef SK_LOAD
  load_rp();
  if (pending) reduce(pend_g, std::true_type{});
  stage();
  reduce(cur_g, std::false_type{});
  finish_splits();
}

static int sk_num_cus() {
  static int n[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n[dev] = v;
  }
  return n[dev];
}

template <int MT, int NT, int D>
static int launch_gemm_sk_cfg(const void* x, void* y, int64_t ys, const void* w, const void* res, int64_t rs, int M,
                              int N, int K, int epi, int flags, void* ws, int G, const EpiArgs& ep,
                              hipStream_t stream) {
  const int nks = K / 32;
  const int ngrp = (N / 16) / NT;
  if ((N / 16) % NT || nks % 8 || nks < 8 * D || ngrp > SK_MAX_GROUPS) return 1;  // caller falls back
  const int U = ngrp * nks;
  if (G > SK_MAX_BLOCKS) G = SK_MAX_BLOCKS;
  if (G > U) G = U;
  // EPI 3 keeps its epilogue out of the ring loop, which needs every range <= one group
  if (epi == 3 && (U + G - 1) / G > nks) return 1;
  int* cnt = (int*)ws;  // [SK_MAX_GROUPS] counters, [SK_ZERO_BYTES] zeros, slabs
  f32x4* slab = (f32x4*)((char*)ws + SK_MAX_GROUPS * sizeof(int) + SK_ZERO_BYTES);
  const bool opk = flags & 2;
#define MP_SK(EPI_, OPK_)                                                                                         \
  hipLaunchKernelGGL((gemm_sk_kernel<MT, NT, D, EPI_, OPK_>), dim3(G), dim3(512), 0, stream, (const bf16_t*)x,     \
                     (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K, cnt, slab, 1, ep)
  if (epi == 1) {
    if constexpr (NT % 2 == 0) {
      if (opk) { MP_SK(1, true); } else { MP_SK(1, false); }
    } else {
      return 1;
    }
  } else if (opk) {
    return -3;
  } else if (epi == 2) {
    MP_SK(2, false);
  } else if (epi == 3) {
    MP_SK(3, false);
  } else {
    MP_SK(0, false);
  }
#undef MP_SK
  return 0;
}

// Largest grid G in [0.9 C, C] that divides the group count (every workgroup then owns whole
// groups: no split-group hand-off at all), else 0.
static int sk_whole_grid(int ngrp, int C) {
  for (int G = C; G * 10 >= C * 9; --G)
    if (G > 0 && ngrp % G == 0) return G;
  return 0;
}

// Stream-K launch: prefer a column-group width NT (4, then 3 for non-SwiGLU, then 2) whose
// group count splits evenly over ~all CUs (no split groups); otherwise NT = 4 on every CU with
// split groups (deferred sc1 hand-off).
template <int MT>
static int launch_gemm_sk(const void* x, void* y, int64_t ys, const void* w, const void* res, int64_t rs, int M, int N,
                          int K, int epi, int flags, void* ws, const EpiArgs& ep, hipStream_t stream) {
  // ring depth 4 (3 when MT x NT >= 16: the 256-VGPR cap)
  constexpr int DW = (MT * 4 >= 16) ? 3 : 4, D3 = (MT * 3 >= 16) ? 3 : 4;
  const int C = sk_num_cus(), nt = N / 16;
  int G;
  if (nt % 4 == 0 && (G = sk_whole_grid(nt / 4, C)))
    return launch_gemm_sk_cfg<MT, 4, DW>(x, y, ys, w, res, rs, M, N, K, epi, flags, ws, G, ep, stream);
  if (epi != 1 && nt % 3 == 0 && (G = sk_whole_grid(nt / 3, C)))
    return launch_gemm_sk_cfg<MT, 3, D3>(x, y, ys, w, res, rs, M, N, K, epi, flags, ws, G, ep, stream);
  if (nt % 2 == 0 && (G = sk_whole_grid(nt / 2, C)))
    return launch_gemm_sk_cfg<MT, 2, 4>(x, y, ys, w, res, rs, M, N, K, epi, flags, ws, G, ep, stream);
  return launch_gemm_sk_cfg<MT, 4, DW>(x, y, ys, w, res, rs, M, N, K, epi, flags, ws, C, ep, stream);
}

// ---------------------------------------------------------------------------------------
// Balanced ring form ("rw"): every CU gets one workgroup of 4 waves (one per SIMD) that owns a
// CONTIGUOUS run of column tiles and all of K, with no split-K hand-off.  The tile count per
// workgroup is ceil or floor of tiles / CUs (SwiGLU: of gate/up tile PAIRS), so every CU streams
// about the same weight bytes.  This is what the layer shapes need: gate/up (1376 tiles =
// 32 x 43) gives the fixed-width kernels 172 workgroups of 8 tiles (84 CUs idle) or ragged
// waves of workgroups; here it is 176 x 6 + 80 x 4 tiles on 256 CUs.  The two widths are two
// template bodies behind one uniform branch.
// Inside a workgroup the waves take interleaved k-slices (k = wave + 4 i) through an R-deep
// register ring holding BOTH operands of a slice, loads issued R slices ahead in consumption
// order (in-order vmcnt never drains the ring; loads past the end are clamped to a valid slice
// and their MFMAs skipped), then the 4 partial tiles are summed through LDS and the shared
// epilogues run (row scale, SwiGLU, residual, the fused-norm producer).
#ifndef MP_RW_WAVES
#define MP_RW_WAVES 4
#endif
constexpr int RW_WAVES = MP_RW_WAVES;  // waves per ring workgroup (an ablation build sets 8)
// Ring tail: the loads a wave issues R steps ahead run past its last k-step; they are clamped to a
// valid step and their MFMAs skipped (in-order vmcnt needs every slot loaded).  Pointing those dead
// weight loads at the L2-resident activation helps the 128-deep MX steps (profiles/r6mx) but not
// these rings: 7B 64 / 1 sessions and 70B fp8 unchanged or 0.1-0.5 % slower (profiles/r6tail).
constexpr int RW_QC = 128 / RW_WAVES;  // quads per LDS combine pass (waves x RW_QC x 1 KiB = 128 KiB)

// Ring slots: a power of two (K / 32 / 4 waves is a multiple of it at K = 4096, 11008: no
// clamped tail turn); 4 (MT + NT) VGPRs each (one wave per SIMD: the accumulators go to AGPRs).
// Measured at M = 64 (lab, us): qkv depth 2 / 4 / 6 = 21.2 / 21.7 / 22.7, gate/up 35.1 / 35.3 /
// 35.4, o 14.3 / 13.7 / 14.1: two slots of 4 waves already cover the latency where tiles are wide.
// MP_RW_DEEP1 (default on): 8 slots for the narrowest forms (one row tile, one column tile: the
// batch-1 o projection, 256 workgroups of 128 KB of weights each), whose 4 waves x 4 slots keep
// only ~32 KB per CU in flight (batch 1: 2.809 -> 2.789 ms, profiles/r3_u).
#ifndef MP_RW_DEEP1
#define MP_RW_DEEP1 1
#endif
template <int MT, int NT>
constexpr int rw_depth() {
  if (MP_RW_DEEP1 && MT + NT <= 2) return 8;
  return 190 / (4 * (MT + NT)) >= 8 ? 4 : 2;
}
// fp8 weights: a slot is 4 MT + 2 NT VGPRs.  (4 slots for the 14-tile Llama-3-70B gate/up group
// measured 17.30-17.34 vs 17.23-17.25 ms with 2: profiles/r4ab2.)
template <int MT, int NT, bool F8>
constexpr int rw_depth2() {
  if constexpr (F8) {
    return 190 / (4 * MT + 2 * NT) >= 8 ? 4 : 2;
  } else {
    return rw_depth<MT, NT>();
  }
}

// MX ring step (128 k): 8 MT + 8 NT + 1 VGPRs per slot (rsa: the step's block-scale word)
template <int MT, int NT>
constexpr int mx_depth() {
  return 200 / (8 * MT + 8 * NT + 1) >= 4 ? 4 : 2;
}

// ``mt0`` / ``mta`` (row-split form, gemm_rwr_kernel): this workgroup computes the MT row tiles
// starting at tile mt0 of an activation packed with mta row tiles (default: all rows, mta = MT).
// NTW = false loads the weights with the default cache policy (a row-split pair re-reads them).
template <int MT, int NT, int EPI, bool OPK, bool F8 = false, bool NTW = true>
__device__ __forceinline__ void rw_body(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                        bf16_t* __restrict__ y, int64_t ys, const bf16_t* __restrict__ res, int64_t rs,
                                        int M, int K, int tile0, const EpiArgs& ep, f32x4* red, u64 (*rs_part)[SS_ROWS],
                                        float* rs_lds, int mt0 = 0, int mta = MT) {
  constexpr int R = rw_depth2<MT, NT, F8>();
  constexpr int Q = MT * NT;
  constexpr int NQ = (Q + RW_WAVES - 1) / RW_WAVES;  // epilogue quads per wave
  RowScale<EPI < 2, RW_WAVES> rsc;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nks = K >> 5;
  const int cnt = (nks + RW_WAVES - 1) / RW_WAVES;  // ring steps of the busiest wave
  const int krot = rw_krot(nks, ep.rot);
  // F8: the same fragment order at 1 byte per weight (offsets below count elements)
  using WT = std::conditional_t<F8, uint8_t, bf16_t>;
  using BT = std::conditional_t<F8, u32x2, u16x8>;
  const WT* wb = reinterpret_cast<const WT*>(wp) + ((int64_t)tile0 * nks) * 512 + lane * 8;
  const bf16_t* xl = x + lane * 8;
  float wsc[NT];
  if constexpr (F8) {
#pragma unroll
    for (int t = 0; t < NT; ++t) wsc[t] = ep.wsc[(tile0 + t) * 16 + (lane & 15)];
  }

  // EPI 3: the residual quads this wave finalises, in flight during the main loop
  u16x4 rpre[NQ];
  if constexpr (EPI == 3) {
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int qd = min(wid + RW_WAVES * j, Q - 1), mt = qd / NT, t = qd % NT;
      const int col = (tile0 + t) * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        rpre[j][r] = res[(int64_t)min((mt0 + mt) * 16 + (lane >> 4) * 4 + r, M - 1) * rs + col];
    }
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);
  u16x8 ra[R][MT];
  BT rb[R][NT];
#define RW_LOAD(s, i)                                                                                        \
  {                                                                                                          \
    const int k_ = rw_rot(min(wid + RW_WAVES * (i), nks - 1), krot, nks);                                  \
    _Pragma("unroll") for (int t = 0; t < NT; ++t) {                                                         \
      const BT* p_ = reinterpret_cast<const BT*>(wb + (((int64_t)t * nks + k_) << 9));                      \
      rb[s][t] = NTW ? __builtin_nontemporal_load(p_) : *p_;                                                 \
    }                                                                                                        \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) ra[s][mt] =                                            \
        load_a_rows(xl + (((int64_t)k_ * mta + min(mt0 + mt, mta - 1)) << 9), lane,                         \
                    (mt0 + mt) * 16 + (lane & 15) < M);                                                      \
  }
#pragma unroll
  for (int s = 0; s < R; ++s) RW_LOAD(s, s)
  rsc.load(ep, wp);
  for (int i0 = 0; i0 < cnt; i0 += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if (wid + RW_WAVES * (i0 + s) < nks) {
        if constexpr (F8) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const u16x8 b = f8w_to_bf16(rb[s][t]);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt][t] = mfma16(ra[s][mt], b, acc[mt][t]);
          }
        } else {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16(ra[s][mt], rb[s][t], acc[mt][t]);
        }
      }
      RW_LOAD(s, i0 + s + R)
    }
  }
#undef RW_LOAD
  if constexpr (F8) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[mt][t] *= wsc[t];
  }
  // ---- sum the 4 waves' partial tiles through LDS (passes of at most RW_QC quads: 128-row
  //      workgroups own up to 48), then the epilogue ----
  rsc.finish(ep, rs_part, rs_lds);
  constexpr int QC = Q < RW_QC ? Q : RW_QC;
#pragma unroll
  for (int p0 = 0; p0 < Q; p0 += QC) {
    if (p0 > 0) __syncthreads();  // the previous pass has finished reading red
#pragma unroll
    for (int qd = p0; qd < p0 + QC && qd < Q; ++qd) red[(wid * QC + qd - p0) * 64 + lane] = acc[qd / NT][qd % NT];
    __syncthreads();
    // quad qd = wid + 4 j lies in this pass exactly when j does (with several passes p0 and QC
    // are multiples of 4; a single pass has QC = Q)
#pragma unroll
    for (int j = p0 / RW_WAVES; j < (p0 + QC + RW_WAVES - 1) / RW_WAVES && j < NQ; ++j) {
      const int qd = wid + RW_WAVES * j;
      if (qd >= Q || qd >= p0 + QC) break;
      if (EPI == 1 && (qd % NT) & 1) continue;  // up tile: consumed with its gate tile
      f32x4 v = red[(qd - p0) * 64 + lane], up = (f32x4)(0.f);
#pragma unroll
      for (int w = 1; w < RW_WAVES; ++w) v += red[(w * QC + qd - p0) * 64 + lane];
      if constexpr (EPI == 1) {
#pragma unroll
        for (int w = 0; w < RW_WAVES; ++w) up += red[(w * QC + qd + 1 - p0) * 64 + lane];
      }
      tile_epilogue<MT, EPI, OPK>(mt0 + qd / NT, tile0 + qd % NT, v, up, y, ys, res, rs, M, lane, ep, rs_lds,
                                  EPI == 3 ? &rpre[j] : nullptr);
    }
  }
}

template <int MT, int NTB, int NTS, int EPI, bool OPK, bool F8 = false>
__global__ __launch_bounds__(RW_WAVES * 64) void gemm_rw_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                      bf16_t* __restrict__ y, int64_t ys,
                                                      const bf16_t* __restrict__ res, int64_t rs, int M, int K,
                                                      int n_big, const EpiArgs ep) {
  clear_other(ep);
  __shared__ u64 rs_part[SS_PG][SS_ROWS];
  __shared__ float rs_lds[SS_ROWS];
  __shared__ __attribute__((aligned(16))) f32x4 red[RW_WAVES * (MT * NTB < RW_QC ? MT * NTB : RW_QC) * 64];
  const int b = blockIdx.x;
  if (b < n_big) {
    rw_body<MT, NTB, EPI, OPK, F8>(x, wp, y, ys, res, rs, M, K, b * NTB, ep, red, rs_part, rs_lds, 0, ep.mt_out);
  } else {
    rw_body<MT, NTS, EPI, OPK, F8>(x, wp, y, ys, res, rs, M, K, n_big * NTB + (b - n_big) * NTS, ep, red, rs_part,
                                   rs_lds, 0, ep.mt_out);
  }
}

template <int MT, int NTB, int NTS, bool F8 = false>
static int launch_gemm_rw_cfg(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                              int K, int epi, bool opk, int G, int n_big, const EpiArgs& ep, hipStream_t stream,
                              bool dry) {
  if constexpr (F8) {
    // fp8-weight (W8A16) forms, M <= 64: the fused-norm decode epilogues (0 with row scale,
    // packed SwiGLU, residual-stream producer)
    if constexpr (MT > 4 || 4 * MT * NTB > 256) {
      return 1;
    } else {
      if (!(epi == 0 || epi == 3 || (epi == 1 && opk)) || (epi == 1 && (NTB % 2 || NTS % 2))) return 1;
      if (dry) return 0;
      if (epi == 1) {
        if constexpr (NTB % 2 == 0 && NTS % 2 == 0)
          hipLaunchKernelGGL((gemm_rw_kernel<MT, NTB, NTS, 1, true, true>), dim3(G), dim3(RW_WAVES * 64), 0, stream,
                             (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, n_big, ep);
      } else if (epi == 3) {
        hipLaunchKernelGGL((gemm_rw_kernel<MT, NTB, NTS, 3, false, true>), dim3(G), dim3(RW_WAVES * 64), 0, stream,
                           (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, n_big, ep);
      } else {
        hipLaunchKernelGGL((gemm_rw_kernel<MT, NTB, NTS, 0, false, true>), dim3(G), dim3(RW_WAVES * 64), 0, stream,
                           (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, n_big, ep);
      }
      return 0;
    }
  } else if constexpr (MT > 4) {
    // M = 65..256 (the packed decode path at 96..256 sessions): plain and packed-SwiGLU epilogues
    // only, accumulators within 192 AGPRs (MT <= 8) or all 256 (MT 9..16: 129..256 rows)
    if constexpr (4 * MT * NTB > (MT > 8 ? 256 : 192)) {
      return 1;
    } else {
      if (!(epi == 0 || (epi == 1 && opk)) || (epi == 1 && (NTB % 2 || NTS % 2))) return 1;
      if (dry) return 0;
      if (epi == 1) {
        if constexpr (NTB % 2 == 0 && NTS % 2 == 0)
          hipLaunchKernelGGL((gemm_rw_kernel<MT, NTB, NTS, 1, true>), dim3(G), dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x,
                             (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, n_big, ep);
      } else {
        hipLaunchKernelGGL((gemm_rw_kernel<MT, NTB, NTS, 0, false>), dim3(G), dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x,
                           (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, n_big, ep);
      }
      return 0;
    }
  } else {
  if (epi == 1 && (NTB % 2 || NTS % 2)) return 1;
  if (dry) return 0;
#define MP_RW(EPI_, OPK_)                                                                                          \
  hipLaunchKernelGGL((gemm_rw_kernel<MT, NTB, NTS, EPI_, OPK_>), dim3(G), dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x, \
                     (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, n_big, ep)
  if (epi == 1) {
    if constexpr (NTB % 2 == 0 && NTS % 2 == 0) {
      if (opk) { MP_RW(1, true); } else { MP_RW(1, false); }
    } else {
      return 1;
    }
  } else if (opk) {
    return -3;
  } else if (epi == 2) {
    MP_RW(2, false);
  } else if (epi == 3) {
    MP_RW(3, false);
  } else {
    MP_RW(0, false);
  }
#undef MP_RW
  return 0;
  }
}

// Split the column units (tiles, or gate/up tile pairs) over G = min(#CUs, units) workgroups:
// n_big of them take ceil, the rest floor.  Returns 1 (caller falls back) for widths not built.
template <int MT, bool F8 = false>
static int launch_gemm_rw(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                          int N, int K, int epi, int flags, const EpiArgs& ep, hipStream_t stream, bool dry = false) {
  const int step = epi == 1 ? 2 : 1;
  const int units = (N / 16) / step;
  if ((N / 16) % step || units == 0) return 1;
  int G = units < sk_num_cus() ? units : sk_num_cus();
  if constexpr (MT > 8) {
    // 129..256 rows: at most 64 / MT column tiles per workgroup (256 accumulator AGPRs), so wide
    // projections run more workgroups than CUs (gate/up at 256 rows: 344 groups of 4 tiles)
    const int per = ((64 / MT) / step) > 0 ? (64 / MT) / step : 1;
    if ((units + per - 1) / per > G) G = (units + per - 1) / per;
  }
  const int base = units / G, rem = units % G;
  const int ntb = (base + (rem ? 1 : 0)) * step;
  const int n_big = rem ? rem : G;
  const bool opk = flags & 2;
#define MP_RWC(B_, S_) \
  return launch_gemm_rw_cfg<MT, B_, S_, F8>(x, w, y, ys, res, rs, M, K, epi, opk, G, n_big, ep, stream, dry)
  if (epi == 1) {
    switch (ntb) {
      case 2: if (rem) return 1; MP_RWC(2, 2);
      case 4: MP_RWC(4, 2);
      case 6: MP_RWC(6, 4);
      case 8: MP_RWC(8, 6);
      case 14:  // Llama-3-70B gate/up (3584 tiles on 256 CUs), fp8 weights only
        if constexpr (F8) { if (rem) return 1; MP_RWC(14, 14); }
        return 1;
      default: return 1;
    }
  }
  switch (ntb) {
    case 1: MP_RWC(1, 1);
    case 2: MP_RWC(2, 1);
    case 3: MP_RWC(3, 2);
    case 4: MP_RWC(4, 3);
    case 6: if (rem) return 1; MP_RWC(6, 6);
    case 8: MP_RWC(8, 7);
    default: return 1;
  }
#undef MP_RWC
}

// ---------------------------------------------------------------------------------------
// Row-split ring form ("rwr") for the narrowest projection (o: N = K = 4096).  A ring workgroup
// that owns all M rows of NT column tiles takes in the whole M x K activation block for NT x 16
// weight columns: at M = 64, NT = 1 that is 4x the weight bytes through the CU's load path
// (profiles/r3_f).  Here a PAIR of workgroups shares NT = 2 column tiles and splits the rows
// (MTH = MT / 2 row tiles each): per CU the activation bytes halve and the weight bytes double,
// 512 KB instead of 643 KB of intake at M = 64, and no K split - so no partial slabs, no
// combine, and the fused epilogues (residual-stream producer) run straight from the ring.  The
// pair reads the same weight columns: blocks b and b + 8 (one XCD under round-robin dispatch,
// dispatched together) so the second read is an L2 / Infinity Cache hit; NTW picks the weight
// load policy (non-temporal or default).  Placement only - never correctness.
template <int MTH, int NT, int EPI, bool NTW>
__global__ __launch_bounds__(RW_WAVES * 64) void gemm_rwr_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                       bf16_t* __restrict__ y, int64_t ys,
                                                       const bf16_t* __restrict__ res, int64_t rs, int M, int K,
                                                       const EpiArgs ep) {
  clear_other(ep);
  __shared__ u64 rs_part[SS_PG][SS_ROWS];
  __shared__ float rs_lds[SS_ROWS];
  __shared__ __attribute__((aligned(16))) f32x4 red[RW_WAVES * (MTH * NT < RW_QC ? MTH * NT : RW_QC) * 64];
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int half = j & 1, g = (j >> 1) * 8 + xcd;
  rw_body<MTH, NT, EPI, false, false, NTW>(x, wp, y, ys, res, rs, M, K, g * NT, ep, red, rs_part, rs_lds, half * MTH,
                                           2 * MTH);
}

// Grid = 2 x (tiles / NT) = #CUs (a multiple of 16); epilogues 0 / 2 / 3, MT even.  Returns 1
// (caller falls back) when the shape does not split that way.
template <int MT>
static int launch_gemm_rwr(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                           int N, int K, int epi, int flags, const EpiArgs& ep, hipStream_t stream) {
  if constexpr (MT % 2 != 0) {
    return 1;
  } else {
    constexpr int MTH = MT / 2;
    const int tiles = N / 16, C0 = sk_num_cus();
    if (epi == 1 || (flags & 2) || C0 % 16 || (2 * tiles) % C0) return 1;
    const int nt = 2 * tiles / C0;
    const bool ntw = !(flags & 8192);
#define MP_RWR(NT_, EPI_)                                                                                          \
  {                                                                                                                \
    if (ntw)                                                                                                       \
      hipLaunchKernelGGL((gemm_rwr_kernel<MTH, NT_, EPI_, true>), dim3(C0), dim3(RW_WAVES * 64), 0, stream,       \
                         (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, ep);    \
    else                                                                                                           \
      hipLaunchKernelGGL((gemm_rwr_kernel<MTH, NT_, EPI_, false>), dim3(C0), dim3(RW_WAVES * 64), 0, stream,      \
                         (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, K, ep);    \
  }
#define MP_RWR_E(NT_) \
  { if (epi == 3) MP_RWR(NT_, 3) else if (epi == 2) MP_RWR(NT_, 2) else MP_RWR(NT_, 0) }
    switch (nt) {
      case 1: MP_RWR_E(1); break;
      case 2: MP_RWR_E(2); break;
      case 4: MP_RWR_E(4); break;
      default: return 1;
    }
#undef MP_RWR_E
#undef MP_RWR
    return 0;
  }
}

// ---------------------------------------------------------------------------------------
// Split-K ring form ("rwk") for the narrow projections (o, down: N = 4096 -> 256 column tiles,
// one per CU): with every CU owning all of K, each CU streams ALL of the activation block
// (M x K) for just 16 weight columns - at M = 64 that is 4x the weight bytes through the
// texture path (the lab: down 29 us, 16 us with the A loads removed).  Here a workgroup owns NT
// column tiles and 1/S of K (C x S = #CUs), so A per CU drops S-fold, and writes an fp32 partial
// slab; the sum over the S slabs and the epilogue (residual, packed copy, row sums of squares)
// run in a small second launch - a kernel boundary instead of an in-launch seam (the stream-K
// kernel's end-of-range hand-off costs ~7 us at these sizes).
constexpr int64_t RWK_SLAB_BYTES = (int64_t)32 << 20;  // S x M x N fp32 partials (workspace tail)

// INL >= 0: in-launch combine instead of the reduce launch - every split stores its summed
// tiles as write-through (sc1) fp32 slabs in fragment order, takes an arrival ticket on its
// column group, and the LAST of the S splits reads the S slabs back (sc1 loads, slab order:
// deterministic) and runs epilogue INL (0 with the optional row scale, 2, 3) itself - the
// stream-K kernel's hand-off protocol (guide: splitk-seam, publish-large).
//
// The last arriver of the S splits (arrival ticket) sums all S slabs in split order (0..S-1) from
// zero - the reduce launch's order, so both give the same bits - and runs the whole epilogue; no
// workgroup ever waits for another, so the result never depends on co-residency.  (A symmetric
// reduce-scatter combine, in which every split polled for its partners, was measured 2-3.5 us
// slower than the reduce launch and needed all S splits resident at once: removed, profiles/r4_seam.)
// Residual quads of EPI 3 are prefetched before the main loop.
// MX (with F8): the activation is MX fp8 (gemm_mx.hip: e4m3 bytes Ax[K/128][MT][64][32] in the
// W8A16 fragment order of four consecutive k-slices, e8m0 block scales in ep.xsc) and every ring
// step is one 128-deep k-step of v_mfma_scale_f32_16x16x128_f8f6f4: the fp8 weight fragments of
// the step's four k-slices go to the MFMA as they are (no conversion; weight scale byte 127 = 1,
// the column scales multiply the accumulators after the loop as in W8A16), the activation's
// block scales ride in the instruction.  Half the activation bytes of W8A16, a quarter of the
// MFMA instructions, no cvt.
template <int MT, int NT, bool F8 = false, int INL = -1, bool MX = false>
__global__ __launch_bounds__(RW_WAVES * 64) void gemm_rwk_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                       float* __restrict__ part, int M, int N, int K, int S,
                                                       const EpiArgs ep, bf16_t* __restrict__ y, int64_t ys,
                                                       const bf16_t* __restrict__ res, int64_t rs,
                                                       int* __restrict__ tick) {
  clear_other(ep);
  static_assert(!MX || (F8 && INL < 0), "MX: fp8 weights, reduce launch");
  constexpr int R = MX ? mx_depth<MT, NT>() : rw_depth2<MT, NT, F8>();
  using WT = std::conditional_t<F8, uint8_t, bf16_t>;
  using BT = std::conditional_t<MX, u32x8, std::conditional_t<F8, u32x2, u16x8>>;
  using AT = std::conditional_t<MX, u32x8, u16x8>;
  constexpr int KS = MX ? 4 : 1;  // k-slices (of 32) per ring step
  constexpr int Q = MT * NT;
  constexpr int QC = Q < RW_QC ? Q : RW_QC;
  constexpr int NQ = (Q + RW_WAVES - 1) / RW_WAVES;  // epilogue quads per wave (at most)
  __shared__ __attribute__((aligned(16))) f32x4 red[RW_WAVES * QC * 64];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int c, sp;
  if (INL >= 0 && (gridDim.x % (8 * S)) == 0) {
    // in-launch combine: the S splits of a column group share blockIdx % 8, i.e. one XCD under
    // round-robin dispatch, so the slab hand-off stays inside one L2 (MI355X_MICROARCH
    // handoff-payload: same-XCD 1.7x cross-XCD).  Placement only - never correctness.
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    c = x * (gridDim.x / (8 * S)) + j / S;
    sp = j % S;
  } else {
    c = blockIdx.x / S;
    sp = blockIdx.x - c * S;
  }
  const int tile0 = c * NT;
  const int nks = K >> 5;
  const int nst = nks / KS;  // ring steps over all of K
  const int ks0 = (int)((int64_t)sp * nst / S), ks1 = (int)((int64_t)(sp + 1) * nst / S);
  const int cnt = (ks1 - ks0 + RW_WAVES - 1) / RW_WAVES;
  const int krot = rw_krot(ks1 - ks0, ep.rot);
  const WT* wb = reinterpret_cast<const WT*>(wp) + ((int64_t)tile0 * nks) * 512 + lane * 8;
  const bf16_t* xl = x + lane * 8;
  const uint8_t* xm = reinterpret_cast<const uint8_t*>(x) + lane * 16;  // MX: this lane's 2 x 16 bytes
  const unsigned* xs = reinterpret_cast<const unsigned*>(ep.xsc) + lane;  // MX: its scale word per step
  float wsc[NT];
  if constexpr (F8) {
#pragma unroll
    for (int t = 0; t < NT; ++t) wsc[t] = ep.wsc[(tile0 + t) * 16 + (lane & 15)];
  }
  // EPI 3 in-launch: the residual quads this wave may finalise (qd = wid + 4 j of the whole
  // group), in flight during the loop
  u16x4 rpre[NQ];
  if constexpr (INL == 3) {
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int qd = wid + RW_WAVES * j;
      rpre[j] = res_quad<NT>(res, rs, min(qd, Q - 1), c, M, lane);
    }
  }
  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);
  AT ra[R][MT];
  BT rb[R][NT];
  unsigned rsa[MX ? R : 1];
#define RWK_LOAD(s, i)                                                                                     \
  {                                                                                                          \
    const int k_ = ks0 + rw_rot(min(wid + RW_WAVES * (i), ks1 - ks0 - 1), krot, ks1 - ks0);                \
    if constexpr (MX) {                                                                                      \
      /* steps past the split's end (the ring's tail) load the L2-resident activation instead of      */     \
      /* re-streaming a weight step from HBM (non-temporal loads do not stay in L2)                   */     \
      const bool live_ = wid + RW_WAVES * (i) < ks1 - ks0;                                                   \
      _Pragma("unroll") for (int t = 0; t < NT; ++t) {                                                       \
        const u32x2* p_ = reinterpret_cast<const u32x2*>(                                                    \
            live_ ? wb + (((int64_t)t * nks + 4 * k_) << 9) : reinterpret_cast<const WT*>(x) + lane * 8);   \
        const u32x2 w0 = __builtin_nontemporal_load(p_), w1 = __builtin_nontemporal_load(p_ + 64),           \
                    w2 = __builtin_nontemporal_load(p_ + 128), w3 = __builtin_nontemporal_load(p_ + 192);   \
        rb[s][t] = (u32x8){w0[0], w0[1], w1[0], w1[1], w2[0], w2[1], w3[0], w3[1]};                          \
      }                                                                                                      \
      _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                                    \
        const int64_t o_ = (int64_t)k_ * ep.mt_out + min(mt, ep.mt_out - 1);                                 \
        const u32x4 a0 = *reinterpret_cast<const u32x4*>(xm + (o_ << 11)),                                   \
                    a1 = *reinterpret_cast<const u32x4*>(xm + (o_ << 11) + 1024);                            \
        ra[s][mt] = (u32x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};                         \
      }                                                                                                      \
      rsa[s] = xs[(int64_t)k_ << 6];                                                                         \
    } else {                                                                                                 \
      _Pragma("unroll") for (int t = 0; t < NT; ++t) rb[s][t] =                                              \
          __builtin_nontemporal_load(reinterpret_cast<const BT*>(wb + (((int64_t)t * nks + k_) << 9)));     \
      _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) ra[s][mt] =                                          \
          load_a_rows(xl + (((int64_t)k_ * ep.mt_out + min(mt, ep.mt_out - 1)) << 9), lane,                \
                      mt * 16 + (lane & 15) < M);                                                            \
    }                                                                                                        \
  }
#pragma unroll
  for (int s = 0; s < R; ++s) RWK_LOAD(s, s)
  for (int i0 = 0; i0 < cnt; i0 += R) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if (ks0 + wid + RW_WAVES * (i0 + s) < ks1) {
        if constexpr (MX) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt][t] = mfma_mx(ra[s][mt], rb[s][t], rsa[s] >> (8 * mt), acc[mt][t]);
        } else if constexpr (F8) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const u16x8 b = f8w_to_bf16(rb[s][t]);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt][t] = mfma16(ra[s][mt], b, acc[mt][t]);
          }
        } else {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16(ra[s][mt], rb[s][t], acc[mt][t]);
        }
      }
      RWK_LOAD(s, i0 + s + R)
    }
  }
#undef RWK_LOAD
  if constexpr (F8) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[mt][t] *= wsc[t];
  }
  if constexpr (INL >= 0) {
    __shared__ u64 rs_part[SS_PG][SS_ROWS];
    __shared__ float rs_lds[SS_ROWS];
    __shared__ int s_last;
    RowScale<INL < 2, RW_WAVES> rsc;
    rsc.load(ep, wp);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(part, (short)0, (int)RWK_SLAB_BYTES, 0x00020000);
#pragma unroll
    for (int p0 = 0; p0 < Q; p0 += QC) {
      if (p0 > 0) __syncthreads();
#pragma unroll
      for (int qd = p0; qd < p0 + QC && qd < Q; ++qd) red[(wid * QC + qd - p0) * 64 + lane] = acc[qd / NT][qd % NT];
      __syncthreads();
      for (int qd = p0 + wid; qd < p0 + QC && qd < Q; qd += RW_WAVES) {
        f32x4 v = red[(qd - p0) * 64 + lane];
#pragma unroll
        for (int w = 1; w < RW_WAVES; ++w) v += red[(w * QC + qd - p0) * 64 + lane];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc,
                                                 (((c * S + sp) * Q + qd) * 64 + lane) * 16, 0, 16);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 slab stores landed
    __syncthreads();
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(tick + c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == S - 1;
      if (old == S - 1) __hip_atomic_store(tick + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the slab loads below the ticket
    rsc.finish(ep, rs_part, rs_lds);
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int qd = wid + RW_WAVES * j;
      if (qd >= Q) break;
      f32x4 v = (f32x4)(0.f);
      for (int s2 = 0; s2 < S; ++s2)
        v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rsrc, (((c * S + s2) * Q + qd) * 64 + lane) * 16, 0, 16));
      tile_epilogue<MT, INL, false>(qd / NT, tile0 + qd % NT, v, (f32x4)(0.f), y, ys, res, rs, M, lane, ep, rs_lds,
                                    INL == 3 ? &rpre[j] : nullptr);
    }
    return;
  }
  // sum the 4 waves' partial tiles through LDS and store this split's fp32 slab [M][N]
  float* slab = part + (int64_t)sp * M * N;
  const int cl = lane & 15, q = lane >> 4;
#pragma unroll
  for (int p0 = 0; p0 < Q; p0 += QC) {
    if (p0 > 0) __syncthreads();
#pragma unroll
    for (int qd = p0; qd < p0 + QC && qd < Q; ++qd) red[(wid * QC + qd - p0) * 64 + lane] = acc[qd / NT][qd % NT];
    __syncthreads();
    for (int qd = p0 + wid; qd < p0 + QC && qd < Q; qd += RW_WAVES) {
      f32x4 v = red[(qd - p0) * 64 + lane];
#pragma unroll
      for (int w = 1; w < RW_WAVES; ++w) v += red[(w * QC + qd - p0) * 64 + lane];
      const int mt = qd / NT, col = (tile0 + qd % NT) * 16 + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + q * 4 + r;
        if (row < M) {
#if MP_SLAB_ST == 1
          // write-through (sc1) store: the slab is not left dirty in this XCD's L2 for the
          // kernel-end writeback (MI355X_MICROARCH boundary row: + dirty bytes / 6 TB/s)
          __hip_atomic_store(slab + (int64_t)row * N + col, v[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#elif MP_SLAB_ST == 2
          __builtin_nontemporal_store(v[r], slab + (int64_t)row * N + col);
#else
          slab[(int64_t)row * N + col] = v[r];
#endif
        }
      }
    }
  }
}

// Sum the S fp32 slabs (fixed order: deterministic) + epilogue.  One thread per CPT consecutive
// columns of a row; a workgroup covers 256 CPT columns of one row (EPI 3: its row's sum of squares
// is reduced in the workgroup and added to one shard with a single atomic).  The kernel is one
// memory round trip deep (latency-bound at decode sizes), so CPT = 4 (default) puts twice as many
// workgroups - and loads in flight - on the chip as CPT = 8: 256 instead of 128 workgroups for a
// 64 x 4096 output (``-DMP_SKR_CPT=8``: the round-2 geometry).
#ifndef MP_SKR_CPT
#define MP_SKR_CPT 4
#endif
constexpr int SKR_CPT = MP_SKR_CPT;
// Store form of the row outputs (read by the next launch), measured per row width against plain
// stores: WT = write-through (sc1) for 4096-wide rows (Llama-2-7B o / down, 64 sessions: 4.225 ->
// 4.195 ms per step, profiles/r6osc; on 8192-wide rows it lost: 70B fp8 16.87 -> 17.05), else
// nontemporal stores (8192-wide, 70B fp8: 16.88 -> 16.75, profiles/r6nt).  launch_splitk_reduce_e:
// WT iff N <= MP_SKR_WT_MAXN (4096).
#ifndef MP_SKR_WT_MAXN
#define MP_SKR_WT_MAXN 4096
#endif
template <int EPI, int S, bool WT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int M, int N,
                                                            bf16_t* __restrict__ y, int64_t ys,
                                                            const bf16_t* __restrict__ res, int64_t rs,
                                                            const EpiArgs ep) {
  constexpr int CPT = SKR_CPT, NQ = CPT / 4;
  typedef __attribute__((ext_vector_type(CPT))) unsigned short uvec;
  __shared__ u64 red[4];
  __shared__ float s_rs;
  const int row = blockIdx.y;
  const int col = (blockIdx.x * 256 + threadIdx.x) * CPT;
  u64 sq = 0;
  float sc = 1.f;
  if constexpr (EPI == 0) {  // fused-norm consumer (qkv): row scale rsqrt(sum of squares / K + eps)
    if (ep.ss_in != nullptr) {
      if (threadIdx.x < 64) {
        u64 t = threadIdx.x < SS_NSH ? ep.ss_in[threadIdx.x * SS_ROWS + row] : 0ull;
        t = wave_sum_u64(t);
        if (threadIdx.x == 0) s_rs = rsqrtf((float)t * (1.f / SS_FX) * ep.inv_k + ep.eps);
      }
      __syncthreads();
      sc = s_rs;
    }
  }
  if (col < N) {
    // every slab load (and the residual) is issued before the first add: one memory round
    // trip instead of S dependent ones
    uvec rv = (uvec)(0);
    if constexpr (EPI != 0) rv = *reinterpret_cast<const uvec*>(res + (int64_t)row * rs + col);
    f32x4 pq[S][NQ];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const float* pp = part + ((int64_t)s * M + row) * N + col;
#pragma unroll
      for (int h = 0; h < NQ; ++h) pq[s][h] = *reinterpret_cast<const f32x4*>(pp + 4 * h);
    }
    f32x4 acc[NQ];
#pragma unroll
    for (int h = 0; h < NQ; ++h) acc[h] = (f32x4)(0.f);
#pragma unroll
    for (int s = 0; s < S; ++s)  // fixed slab order: deterministic
#pragma unroll
      for (int h = 0; h < NQ; ++h) acc[h] += pq[s][h];
    uvec o;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const float a = acc[j / 4][j & 3];
      if constexpr (EPI == 0) {
        o[j] = f2bf(a * sc);
      } else {
        o[j] = f2bf(round_bf(a) + bf2f(rv[j]));
        if constexpr (EPI == 3) sq += fx_sq(bf2f(o[j]));
      }
    }
    // (packed layout: 8 consecutive columns of a row are contiguous, so CPT in {4, 8} stays one store)
    if constexpr (WT && CPT == 4) {
      const u64 ob = __builtin_bit_cast(u64, o);
      __hip_atomic_store(reinterpret_cast<u64*>(y + (int64_t)row * ys + col), ob, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (EPI == 3)
        __hip_atomic_store(reinterpret_cast<u64*>(ep.ap + apk_off(row, col, ep.mt_out)), ob, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __builtin_nontemporal_store(o, reinterpret_cast<uvec*>(y + (int64_t)row * ys + col));
      if constexpr (EPI == 3)
        __builtin_nontemporal_store(o, reinterpret_cast<uvec*>(ep.ap + apk_off(row, col, ep.mt_out)));
    }
  }
  if constexpr (EPI == 3) {
    if (ep.ss_out == nullptr) return;
    sq = wave_sum_u64(sq);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0)
      atomicAdd(ep.ss_out + ((blockIdx.y * gridDim.x + blockIdx.x) % SS_NSH) * SS_ROWS + row,
                red[0] + red[1] + red[2] + red[3]);
  }
}

// The split count is a template parameter of the reduce (all S slab loads issued back to back).
template <int EPI>
static void launch_splitk_reduce_e(int S, dim3 g2, hipStream_t stream, const float* part, int M, int N, void* y,
                                   int64_t ys, const void* res, int64_t rs, const EpiArgs& ep) {
#define MP_SKR(S_)                                                                                          \
  if (N <= MP_SKR_WT_MAXN)                                                                                  \
    hipLaunchKernelGGL((splitk_reduce_kernel<EPI, S_, true>), g2, dim3(256), 0, stream, part, M, N, (bf16_t*)y, \
                       ys, (const bf16_t*)res, rs, ep);                                                     \
  else                                                                                                      \
    hipLaunchKernelGGL((splitk_reduce_kernel<EPI, S_, false>), g2, dim3(256), 0, stream, part, M, N,          \
                       (bf16_t*)y, ys, (const bf16_t*)res, rs, ep)
  switch (S) {
    case 2: MP_SKR(2); break;
    case 3: MP_SKR(3); break;
    case 4: MP_SKR(4); break;
    case 5: MP_SKR(5); break;
    case 6: MP_SKR(6); break;
    case 7: MP_SKR(7); break;
    default: MP_SKR(8); break;
  }
#undef MP_SKR
}

static inline void launch_splitk_reduce(int S, int epi, dim3 g2, hipStream_t stream, const float* part, int M, int N,
                                        void* y, int64_t ys, const void* res, int64_t rs, const EpiArgs& ep) {
  if (epi == 3) launch_splitk_reduce_e<3>(S, g2, stream, part, M, N, y, ys, res, rs, ep);
  else if (epi == 2) launch_splitk_reduce_e<2>(S, g2, stream, part, M, N, y, ys, res, rs, ep);
  else launch_splitk_reduce_e<0>(S, g2, stream, part, M, N, y, ys, res, rs, ep);
}

// Split-K ring geometry: column-group width NT and split count S (C x S <= #CUs, 2 <= S <= 8):
// the width whose grid C x S fills the most CUs, ties to the earlier candidate (qkv, 768 tiles:
// NT = 6, S = 2 fills 256 CUs where NT = 8, S = 2 leaves 64 idle).  fp8 weights: the bf16
// activation block costs 2M / (16 NT) x the weight bytes per CU - the widest group first.
// nt = 0 when no split applies.  (Widths 4 / 2 / 16 for the fp8 70B shapes were measured against 8:
// 8 is the optimum, profiles/r4ac, r4ad.)
static inline void rwk_choose(int tiles, int nks, int C0, bool f8, int& nt, int& S, int nt_max = 8) {
  static constexpr int kOrderBf16[5] = {4, 2, 8, 6, 1}, kOrderF8[5] = {8, 4, 2, 6, 1};
  nt = S = 0;
  int best_fill = 0;
  for (int cand : (f8 ? kOrderF8 : kOrderBf16)) {
    if (tiles % cand || cand > nt_max) continue;
    const int C = tiles / cand, s = C0 / C;
    if (s >= 2 && s <= 8 && nks >= 4 * s && C * s > best_fill) { nt = cand; S = s; best_fill = C * s; }
  }
  // lab override (geometry A/B runs): MPAMD_RWK_GEOM="tiles:nt:S[:f8[:nks]],..." replaces the choice
  // for that column-tile count (f8 field: 0 bf16 / 1 fp8 weights, -1 both; nks: only that K / 32)
  static const char* geo = getenv("MPAMD_RWK_GEOM");
  if (geo != nullptr) {
    const char* p = geo;
    while (*p) {
      int t = 0, n = 0, s = 0, w = -1, k = -1, used = 0;
      const int got = sscanf(p, "%d:%d:%d%n:%d%n:%d%n", &t, &n, &s, &used, &w, &used, &k, &used);
      if (got < 3) break;
      if (t == tiles && (w < 0 || w == (int)f8) && (k < 0 || k == nks) && n > 0 && n <= nt_max && tiles % n == 0 &&
          s >= 2 && s <= 8 && nks >= 4 * s) {
        nt = n;
        S = s;
      }
      p += used;
      while (*p == ',') ++p;
    }
  }
}

// MX ring steps are 128 deep: at S splits a wave runs K / (512 S) steps, too few to fill a 2-slot
// ring at the 70B / 7B widths (4 at the 70B o projection) - halve the split and the group width
// (every CU keeps a workgroup).  MPAMD_MX_NT=8 keeps the W8A16 geometry (A/B runs).
static inline void mx_geometry(int tiles, int& nt, int& S) {
  static const int mx_nt = getenv("MPAMD_MX_NT") ? atoi(getenv("MPAMD_MX_NT")) : 4;
  if (nt == 8 && mx_nt == 4 && S % 2 == 0 && tiles % 4 == 0) {
    nt = 4;
    S /= 2;
  }
}

// Widest split-K ring column group the instantiation for M rows holds in its accumulators: 192
// AGPRs up to 128 rows (MT 5..8), all 256 at 129..256 rows (built at MT 12 and 16).
constexpr int rwk_nt_max_mt(int MT) { return MT > 8 ? 64 / MT : (MT > 4 ? 192 / (4 * MT) : 8); }
static inline int rwk_nt_max(int M) {
  const int mt = (M + 15) / 16;
  return rwk_nt_max_mt(mt <= 8 ? mt : (mt <= 12 ? 12 : 16));
}

// ``comb``: 0 = reduce launch, 1 = in-launch combine by the last arriver (flags 256 = split-K ring,
// + 512 -> comb 1), -1 = partial slabs only (flags bit 14).
static inline int rwk_comb(int flags) {
  if (flags & 16384) return -1;  // bit 14: fp32 partial slabs only, no reduce launch
  return (flags & 512) ? 1 : 0;
}

template <int MT, bool F8 = false, bool MX = false>
static int launch_gemm_rwk(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                           int N, int K, int epi, const EpiArgs& ep, void* ws, hipStream_t stream,
                           int comb = 0) {
  const bool inl = comb > 0 && !MX;
  if (epi == 1 || ws == nullptr || N % 2048 != 0) return 1;
  const int tiles = N / 16, C0 = sk_num_cus(), nks = K / 32;
  int nt = 0, S = 0;
  // accumulators: 192 AGPRs up to 128 rows, all 256 beyond (MT 9..16 -> NT <= 64 / MT)
  constexpr int nt_max = rwk_nt_max_mt(MT);
  rwk_choose(tiles, MX ? nks / 4 : nks, C0, F8, nt, S, nt_max);
  if constexpr (MX) mx_geometry(tiles, nt, S);
  if (nt == 0) return 1;
  if ((int64_t)S * M * N * 4 > RWK_SLAB_BYTES) return 1;
  float* part = (float*)((char*)ws + (int64_t)SK_MAX_GROUPS * sizeof(int) + SK_ZERO_BYTES +
                         (int64_t)SK_MAX_BLOCKS * 2 * SK_MAX_S * 64 * sizeof(float));
  const dim3 g1((tiles / nt) * S);
  int* tick = (int*)ws + SK_MAX_GROUPS / 2;  // rwk arrival tickets (the stream-K kernel uses the low half)
  if (inl && MT <= 4 && nt >= 2 && tiles / nt <= SK_MAX_GROUPS / 8 - 1 &&
      (int64_t)tiles * MT * S * 1024 <= RWK_SLAB_BYTES) {
    if constexpr (MT <= 4) {
#define MP_RWKI(NT_, E_)                                                                                       \
  hipLaunchKernelGGL((gemm_rwk_kernel<MT, NT_, F8, E_>), g1, dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x,    \
                     (const bf16_t*)w, part, M, N, K, S, ep, (bf16_t*)y, ys, (const bf16_t*)res, rs, tick)
#define MP_RWKI_E(NT_) \
  { if (epi == 3) MP_RWKI(NT_, 3); else if (epi == 2) MP_RWKI(NT_, 2); else MP_RWKI(NT_, 0); }
      switch (nt) {
        case 2: MP_RWKI_E(2); break;
        case 4: MP_RWKI_E(4); break;
        case 6: MP_RWKI_E(6); break;
        default: MP_RWKI_E(8); break;
      }
#undef MP_RWKI_E
#undef MP_RWKI
      return 0;
    }
  }
  switch (nt) {
    case 1: hipLaunchKernelGGL((gemm_rwk_kernel<MT, 1, F8, -1, MX>), g1, dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x, (const bf16_t*)w, part, M, N, K, S, ep, nullptr, 0, nullptr, 0, nullptr); break;
    case 2: hipLaunchKernelGGL((gemm_rwk_kernel<MT, 2, F8, -1, MX>), g1, dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x, (const bf16_t*)w, part, M, N, K, S, ep, nullptr, 0, nullptr, 0, nullptr); break;
    case 4:
      if constexpr (4 <= nt_max)
        hipLaunchKernelGGL((gemm_rwk_kernel<MT, 4, F8, -1, MX>), g1, dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x, (const bf16_t*)w, part, M, N, K, S, ep, nullptr, 0, nullptr, 0, nullptr);
      break;
    case 6:
      if constexpr (6 <= nt_max)
        hipLaunchKernelGGL((gemm_rwk_kernel<MT, 6, F8, -1, MX>), g1, dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x, (const bf16_t*)w, part, M, N, K, S, ep, nullptr, 0, nullptr, 0, nullptr);
      break;
    default:
      if constexpr (8 <= nt_max)
        hipLaunchKernelGGL((gemm_rwk_kernel<MT, 8, F8, -1, MX>), g1, dim3(RW_WAVES * 64), 0, stream, (const bf16_t*)x, (const bf16_t*)w, part, M, N, K, S, ep, nullptr, 0, nullptr, 0, nullptr);
      break;
  }
  if (comb < 0) return 0;  // partials only: the consumer sums the S slabs itself (rwk_split)
  const dim3 g2(N / (256 * SKR_CPT), M);
  launch_splitk_reduce(S, epi, g2, stream, part, M, N, y, ys, res, rs, ep);
  return 0;
}

}  // namespace mp
