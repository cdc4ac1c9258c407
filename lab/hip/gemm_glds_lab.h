// LDS-DMA ring form ("rg") of the decode GEMMs: the operand stream goes HBM/L2 -> LDS by
// global_load_lds_dwordx4 (no VGPR destination) instead of HBM/L2 -> VGPRs.
//
//   y[M, N'] = epilogue( x[M, K] . W[N, K]^T ),  M <= 64, packed x and W (gemm_kernels.h header)
//
// Why: the register ring kernels (gemm_rw_kernel, gemm_rwk_kernel) keep at most two ring slots of
// both operands in VGPRs (the accumulators and the MFMA operands share the 256-VGPR budget), so a
// 4-wave workgroup has ~56-80 KiB in flight per CU and its loads retire into registers that the
// MFMAs are waiting on.  At 64 rows that streams the weights at 4.2-4.8 TB/s (profiles/r4q).  An
// LDS-DMA load only needs an address VGPR: each wave keeps D slots of its k-slice stream (D x
// (NT + MT) KiB: both operands of a k-slice) in flight in a private LDS ring of ~37 KiB, i.e.
// ~110-150 KiB per CU in flight, and reads a landed slot with ds_read_b128 (the packed layouts
// make every fragment a contiguous 1 KiB, so the LDS image is a plain copy: lane l reads bytes
// 16 l .. 16 l + 15 of each fragment, conflict-free).  MI355X_MICROARCH "ldsdma-fill": an LDS-DMA
// stream reaches 6.4-6.8 TB/s chip-wide; "nt-weights": non-temporal (aux 2) on the once-read
// weight stream, default policy on the activations that all 256 CUs re-read from L2.
//
// Each wave is its own pipeline (it consumes exactly the slots it issued), so the ring needs no
// barrier: a counted `s_waitcnt vmcnt((D - 1) x F)` retires the oldest slot (vmcnt counts this
// wave's loads in issue order), `s_waitcnt lgkmcnt(0)` after the slot's ds_reads frees it, and the
// refill is issued into it.  ONE __shared__ array holds the ring, the cross-wave combine buffer
// (aliased over the ring after the loop) and the row-statistics scratch (guide §5 trap (a): a
// second __shared__ object next to an LDS-DMA array can make hipcc wait vmcnt(0) per k-step).
//
// Work split: one workgroup per (column group, K split).  S = 1: the workgroup owns NT column
// tiles and all of K and runs the fused epilogues (row scale, SwiGLU + packed output, residual /
// fused-norm producer).  S > 1 (o / down at 64 rows: the activation block per CU drops S-fold):
// fp32 partial slabs [S][M][N] and the split-K reduce launch (splitk_reduce_kernel) - the same
// slab layout and reduce as gemm_rwk_kernel, so the results are bitwise those of the rwk form
// whenever the k walk is the same.
// Reference projection sites: /root/reference/petals/llama/block.py:88-90 (q/k/v), :151 (o),
// :237 (gate/up/down).
#pragma once
#include "gemm_kernels.h"  // (scripts/: built only by rg_lab.hip, -I ops/csrc)

namespace mp {

constexpr int RG_WAVES = 4;
constexpr int RG_RING_BYTES = 148 * 1024;  // staging ring of the 4 waves (and the combine buffer after the loop)
constexpr int RG_SS_BYTES = SS_PG * SS_ROWS * 8 + SS_ROWS * 4;  // RowScale scratch
constexpr int RG_LDS_BYTES = RG_RING_BYTES + RG_SS_BYTES;
static_assert(RG_RING_BYTES >= RG_WAVES * RW_QC * 64 * 16 || RW_WAVES != RG_WAVES,
              "the 4-wave combine buffer aliases the ring");

// Ring slots per wave: as many (NT + MT)-KiB slots as fit in the wave's share of the ring, at most 8
// (F8: the weight fragments are 512 B).
template <int MT, int NT, bool F8>
constexpr int rg_slot_bytes() {
  return (F8 ? NT * 512 : NT * 1024) + MT * 1024;
}
template <int MT, int NT, bool F8>
constexpr int rg_depth() {
  constexpr int d = RG_RING_BYTES / RG_WAVES / rg_slot_bytes<MT, NT, F8>();
  return d > 8 ? 8 : d;
}

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// one wave-instruction: 64 lanes x 16 B from per-lane global addresses into LDS at base + 16 lane
__device__ __forceinline__ void glds16_nt(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds, 16, 0, 2);
}
__device__ __forceinline__ void glds16(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// One workgroup's column group [tile0, tile0 + NT) over k-slices [ks0, ks1).  SPLIT: write this
// split's fp32 slab (part = slab base, [M][N]) instead of running the epilogue.
template <int MT, int NT, int EPI, bool OPK, bool SPLIT, bool F8>
__device__ __forceinline__ void rg_body(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                        bf16_t* __restrict__ y, int64_t ys, const bf16_t* __restrict__ res, int64_t rs,
                                        int M, int N, int K, int tile0, int ks0, int ks1, float* __restrict__ part,
                                        const EpiArgs& ep, unsigned char* smem) {
  constexpr int D = rg_depth<MT, NT, F8>();
  constexpr int WB = F8 ? 512 : 1024;             // weight fragment bytes
  constexpr int SB = rg_slot_bytes<MT, NT, F8>();  // slot bytes
  constexpr int LOADS = (F8 ? (NT + 1) / 2 : NT) + MT;  // glds instructions per slot
  constexpr int Q = MT * NT;
  constexpr int QC = Q < RW_QC ? Q : RW_QC;
  constexpr int NQ = (Q + RG_WAVES - 1) / RG_WAVES;
  static_assert(D >= 2, "ring needs two slots");
  static_assert((D - 1) * LOADS <= 63, "vmcnt is 6 bits");
  static_assert(!F8 || NT % 2 == 0, "fp8 weight fragments are fetched two tiles per 1 KiB load");
  constexpr bool ROWSCALE = EPI < 2 && !SPLIT;
  RowScale<ROWSCALE, RG_WAVES> rsc;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nks = K >> 5, nk = ks1 - ks0;
  const int cnt = (nk + RG_WAVES - 1) / RG_WAVES;  // ring steps of the busiest wave
  unsigned char* ring = smem + wid * (D * SB);
  auto* rs_part = reinterpret_cast<u64(*)[SS_ROWS]>(smem + RG_RING_BYTES);
  float* rs_lds = reinterpret_cast<float*>(smem + RG_RING_BYTES + SS_PG * SS_ROWS * 8);
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  using WT = std::conditional_t<F8, uint8_t, bf16_t>;
  const WT* wb = reinterpret_cast<const WT*>(wp) + (int64_t)tile0 * nks * 512;
  const int mta = ep.mt_out;  // row tiles of the packed activation (its stride)

  // loads whose results are used only after the loop go first: vmcnt retires in issue order, so
  // the ring's counted waits below never wait for them
  u16x4 rpre[NQ];
  if constexpr (EPI == 3 && !SPLIT) {
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int qd = min(wid + RG_WAVES * j, Q - 1), mt = qd / NT, t = qd % NT;
      const int col = (tile0 + t) * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) rpre[j][r] = res[(int64_t)min(mt * 16 + (lane >> 4) * 4 + r, M - 1) * rs + col];
    }
  }
  rsc.load(ep, wp);
  float wsc[F8 ? NT : 1];
  if constexpr (F8) {
#pragma unroll
    for (int t = 0; t < NT; ++t) wsc[t] = ep.wsc[(tile0 + t) * 16 + (lane & 15)];
  }

  // slot s <- k-slice ks0 + wid + 4 i (clamped: a turn past the end re-reads the last slice, an
  // L2 hit, and skips its MFMAs).  Weights: tile t's fragment (bf16: 1 KiB; fp8: two tiles' 512 B
  // fragments are NOT adjacent, so fp8 slots hold pairs of k-slices of one tile - see F8 below).
  auto issue = [&](int s, int i) {
    const int k = ks0 + min(wid + RG_WAVES * i, nk - 1);
    unsigned char* sl = ring + s * SB;
    if constexpr (F8) {
      // fp8 fragment of (tile t, slice k) is 512 B at wb + (t nks + k) 512 bytes; lanes 0-31 fetch
      // tile t, lanes 32-63 tile t + 1 (16 B each), so one instruction fills two 512 B fragments
#pragma unroll
      for (int t = 0; t < NT; t += 2) {
        const int tt = t + (lane >> 5);
        glds16_nt(wb + (((int64_t)tt * nks + k) << 9) + (lane & 31) * 16, sl + t * 512);
      }
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) glds16_nt(wb + (((int64_t)t * nks + k) << 9) + lane * 8, sl + t * 1024);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      glds16(x + ((((int64_t)k * mta + min(mt, mta - 1)) << 9) + lane * 8 -
                  ((mt * 16 + (lane & 15) < M) ? 0 : (lane & 15) * 8)),
             sl + NT * WB + mt * 1024);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = (f32x4)(0.f);

#pragma unroll
  for (int s = 0; s < D; ++s) issue(s, s);
  for (int i0 = 0; i0 < cnt; i0 += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      wait_vm<(D - 1) * LOADS>();  // slot s (issued D slots ago) has landed
      const unsigned char* sl = ring + s * SB;
      u16x8 a[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[mt] = *reinterpret_cast<const u16x8*>(sl + NT * WB + mt * 1024 + lane * 16);
      if constexpr (F8) {
        u32x2 bw[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) bw[t] = *reinterpret_cast<const u32x2*>(sl + t * 512 + lane * 8);
        if (wid + RG_WAVES * (i0 + s) < nk) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const u16x8 b = f8w_to_bf16(bw[t]);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[mt][t] = mfma16(a[mt], b, acc[mt][t]);
          }
        }
      } else {
        u16x8 b[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) b[t] = *reinterpret_cast<const u16x8*>(sl + t * 1024 + lane * 16);
        if (wid + RG_WAVES * (i0 + s) < nk) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16(a[mt], b[t], acc[mt][t]);
        }
      }
      wait_lgkm0();  // the slot's fragments are in registers: it may be refilled
      issue(s, i0 + s + D);
    }
  }
  wait_vm<0>();     // the clamped refills of the last turn
  __syncthreads();  // every wave is done with the ring: the combine buffer aliases it
  if constexpr (F8) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[mt][t] *= wsc[t];
  }
  rsc.finish(ep, rs_part, rs_lds);
  const int cl = lane & 15, q = lane >> 4;
#pragma unroll
  for (int p0 = 0; p0 < Q; p0 += QC) {
    if (p0 > 0) __syncthreads();
#pragma unroll
    for (int qd = p0; qd < p0 + QC && qd < Q; ++qd) red[(wid * QC + qd - p0) * 64 + lane] = acc[qd / NT][qd % NT];
    __syncthreads();
#pragma unroll
    for (int j = p0 / RG_WAVES; j < (p0 + QC + RG_WAVES - 1) / RG_WAVES && j < NQ; ++j) {
      const int qd = wid + RG_WAVES * j;
      if (qd >= Q || qd >= p0 + QC) break;
      if (EPI == 1 && !SPLIT && (qd % NT) & 1) continue;  // up tile: consumed with its gate tile
      f32x4 v = red[(qd - p0) * 64 + lane], up = (f32x4)(0.f);
#pragma unroll
      for (int w = 1; w < RG_WAVES; ++w) v += red[(w * QC + qd - p0) * 64 + lane];
      if constexpr (SPLIT) {
        const int mt = qd / NT, col = (tile0 + qd % NT) * 16 + cl;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mt * 16 + q * 4 + r;
          if (row < M) part[(int64_t)row * N + col] = v[r];
        }
      } else {
        if constexpr (EPI == 1) {
#pragma unroll
          for (int w = 0; w < RG_WAVES; ++w) up += red[(w * QC + qd + 1 - p0) * 64 + lane];
        }
        tile_epilogue<MT, EPI, OPK>(qd / NT, tile0 + qd % NT, v, up, y, ys, res, rs, M, lane, ep, rs_lds,
                                    EPI == 3 ? &rpre[j] : nullptr);
      }
    }
  }
}

// grid: groups x S workgroups (group-major: the S splits of a group are consecutive).  Groups
// [0, n_big) own NTB tiles, the rest NTS (S = 1 only).
template <int MT, int NTB, int NTS, int EPI, bool OPK, bool SPLIT, bool F8>
__global__ __launch_bounds__(RG_WAVES * 64) void gemm_rg_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                              bf16_t* __restrict__ y, int64_t ys,
                                                              const bf16_t* __restrict__ res, int64_t rs, int M, int N,
                                                              int K, int n_big, int S, float* __restrict__ part,
                                                              const EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[RG_LDS_BYTES];
  clear_other(ep);
  const int c = blockIdx.x / S, sp = blockIdx.x - c * S;
  const int nks = K >> 5;
  const int ks0 = (int)((int64_t)sp * nks / S), ks1 = (int)((int64_t)(sp + 1) * nks / S);
  float* slab = SPLIT ? part + (int64_t)sp * M * N : nullptr;
  if (c < n_big) {
    rg_body<MT, NTB, EPI, OPK, SPLIT, F8>(x, wp, y, ys, res, rs, M, N, K, c * NTB, ks0, ks1, slab, ep, smem);
  } else {
    rg_body<MT, NTS, EPI, OPK, SPLIT, F8>(x, wp, y, ys, res, rs, M, N, K, n_big * NTB + (c - n_big) * NTS, ks0, ks1,
                                          slab, ep, smem);
  }
}

// Geometry of the rg form for a shape: (NTB, NTS, n_big, S).  S = 1: the column units (tiles, or
// gate/up pairs) split over min(#CUs, units) workgroups as in launch_gemm_rw; S > 1 only for the
// split-K forms (epilogue 0 / 2 / 3): NT x S with (tiles / NT) x S = #CUs.
struct RgGeom {
  int ntb = 0, nts = 0, n_big = 0, S = 1, G = 0;
};

static inline RgGeom rg_geom(int N, int K, int epi, int S_req, int C0) {
  RgGeom g;
  const int tiles = N / 16, nks = K / 32;
  if (S_req > 1) {
    if (epi == 1 || C0 % S_req || tiles % (C0 / S_req) || nks < 4 * S_req) return g;
    const int nt = tiles / (C0 / S_req);
    g.ntb = g.nts = nt;
    g.n_big = C0 / S_req;
    g.S = S_req;
    g.G = C0;
    return g;
  }
  const int step = epi == 1 ? 2 : 1;
  const int units = tiles / step;
  if (tiles % step || units == 0) return g;
  const int G = units < C0 ? units : C0;
  const int base = units / G, rem = units % G;
  g.ntb = (base + (rem ? 1 : 0)) * step;
  g.nts = base * step;
  g.n_big = rem ? rem : G;
  if (!rem) g.nts = g.ntb;
  g.G = G;
  return g;
}

template <int MT, int NTB, int NTS, bool F8>
static int launch_rg_cfg(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M, int N,
                         int K, int epi, bool opk, const RgGeom& g, float* part, const EpiArgs& ep,
                         hipStream_t stream) {
  if constexpr (4 * MT * NTB > 192 || 4 * MT * NTS > 192 || (F8 && (NTB % 2 || NTS % 2))) {
    return 1;  // accumulators beyond 192 AGPRs / odd fp8 groups: not built
  } else {
#define MP_RG(EPI_, OPK_, SPLIT_)                                                                                 \
  hipLaunchKernelGGL((gemm_rg_kernel<MT, NTB, NTS, EPI_, OPK_, SPLIT_, F8>), dim3(g.G), dim3(RG_WAVES * 64), 0,  \
                     stream, (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K, \
                     g.n_big, g.S, part, ep)
    if (g.S > 1) {
      MP_RG(0, false, true);
      return 0;
    }
    if (epi == 1) {
      if constexpr (NTB % 2 == 0 && NTS % 2 == 0) {
        if (opk) { MP_RG(1, true, false); } else { MP_RG(1, false, false); }
        return 0;
      }
      return 1;
    }
    if (opk) return -3;
    if (epi == 2) { MP_RG(2, false, false); }
    else if (epi == 3) { MP_RG(3, false, false); }
    else { MP_RG(0, false, false); }
#undef MP_RG
    return 0;
  }
}

// flags bits 16-18: the K split (0 / 1 -> none, else S); the split forms need ws (slab region).
template <int MT, bool F8 = false>
static int launch_gemm_rg(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M, int N,
                          int K, int epi, int flags, const EpiArgs& ep, void* ws, hipStream_t stream) {
  const int S_req = (flags >> 16) & 7;
  const RgGeom g = rg_geom(N, K, epi, S_req, sk_num_cus());
  if (g.G == 0) return 1;
  float* part = nullptr;
  if (g.S > 1) {
    if (ws == nullptr || (int64_t)g.S * M * N * 4 > RWK_SLAB_BYTES) return 1;
    part = (float*)((char*)ws + (int64_t)SK_MAX_GROUPS * sizeof(int) + SK_ZERO_BYTES +
                    (int64_t)SK_MAX_BLOCKS * 2 * SK_MAX_S * 64 * sizeof(float));
  }
  const bool opk = flags & 2;
  int rc = 1;
#define MP_RGC(B_, S_) rc = launch_rg_cfg<MT, B_, S_, F8>(x, w, y, ys, res, rs, M, N, K, epi, opk, g, part, ep, stream)
  if (g.ntb == g.nts) {
    switch (g.ntb) {
      case 1: if constexpr (!F8) MP_RGC(1, 1); break;
      case 2: MP_RGC(2, 2); break;
      case 3: if constexpr (!F8) MP_RGC(3, 3); break;
      case 4: MP_RGC(4, 4); break;
      case 6: MP_RGC(6, 6); break;
      case 8: MP_RGC(8, 8); break;
      default: return 1;
    }
  } else {
    switch (g.ntb) {
      case 2: if constexpr (!F8) MP_RGC(2, 1); break;
      case 3: if constexpr (!F8) MP_RGC(3, 2); break;
      case 4: if constexpr (!F8) MP_RGC(4, 3); else MP_RGC(4, 2); break;
      case 6: MP_RGC(6, 4); break;
      case 8: MP_RGC(8, 6); break;
      default: return 1;
    }
  }
#undef MP_RGC
  if (rc != 0) return rc;
  if (g.S > 1) {
    const dim3 g2(N / (256 * SKR_CPT), M);
    launch_splitk_reduce(g.S, epi, g2, stream, part, M, N, y, ys, res, rs, ep);
  }
  return 0;
}

}  // namespace mp
