// Two-dimensionally tiled decode GEMM ("t2d") for 129..256 rows (survey K3 / K8 / K10 at 129-256
// sessions; the reference's projection sites: petals/llama/block.py:88-90, :151, :237).
//
// Why a different kernel above 128 rows.  Every other decode form here gives one workgroup ALL
// rows of its column group, so each CU takes in the whole M x K activation block (2 MB at
// M = 256, K = 4096) for a few hundred KB of weights, and the per-CU load path - not HBM - sets
// the time (profiles/r4d, r4g, r5a: time ~ W / HBM-share + A / L2-intake).  Here a workgroup owns
// a BLOCK of rows x columns (128 rows x 96 columns for qkv at 256 rows) and both operands are
// staged once per CU through LDS, where the 8 waves share them:
//
//   intake per CU = BM x K (activations) + BN x K (weights)      minimised at BM ~ BN
//   qkv at 256 rows: 1 MB + 0.77 MB = 1.8 MB instead of 2 MB + 0.39 MB = 2.4 MB
//
// and the two row blocks of a column group are blocks b and b + 8 (one XCD under round-robin
// dispatch, dispatched together), so the second weight read is an L2 hit.
//
// Pipeline: each k-stage (KU k-slices of 32) is FA = (BM/16) KU activation fragments + NB KU weight
// fragments of 1 KiB (both operands are stored in MFMA fragment order: ops.pack_weight /
// the packed activation layout, so a fragment is one contiguous 1 KiB wave load).  The 8 waves
// load the stage's fragments round-robin, in one of two forms:
//   * LDS-DMA ring (GL, the default for qkv / o / down and 8-tile waves): global_load_lds_dwordx4
//     straight into a P-slot LDS ring (3-6 stages, P - 1 in flight), a counted vmcnt and an
//     lgkmcnt-only barrier per stage - no staging registers, no ds_write;
//   * register ring (the SwiGLU gate/up form): D stages in registers, the oldest written into one
//     of two LDS buffers per stage.
// Wave (wm, wn) of the WM x WN grid computes MW x NW 16 x 16 tiles of the block from LDS reads
// (ds_read_b128).  Measurements: profiles/r5x (A/Bs of both forms, whole-step tables), r5pmc.
//
// Epilogues: the shared decode epilogues (tile_epilogue: 0 with the fused-norm row scale,
// 1 = SwiGLU with packed output, 3 = the residual-stream producer) straight from the accumulators,
// or (SPLIT) fp32 partial slabs [S][M][N] for the split-K reduce launch (splitk_reduce_kernel):
// the residual-stream producers (o, down) split K in two.
#pragma once
#include "gemm_kernels.h"

namespace mp {

// LDS budget of one workgroup: the staging buffers + the RowScale scratch, in ONE __shared__ array
// (guide §5 trap (a): a second __shared__ object beside an LDS-DMA staging array can make hipcc
// wait vmcnt(0) before every k-step's first ds_read).
constexpr int T2D_SS_BYTES = SS_PG * SS_ROWS * 8 + SS_ROWS * 4;
constexpr int T2D_LDS_BYTES = 160 * 1024;

// KU: k-slices (of 32) per stage.  GL: stages arrive by LDS-DMA (global_load_lds_dwordx4) into a
// P-slot LDS ring instead of through a D-deep register ring and ds_write.
template <int MW, int NW, int WM, int WN, int D, int KU, bool GL>
struct T2dGeom {
  static constexpr int BMT = WM * MW;                    // row tiles per block
  static constexpr int NBMAX = WN * NW;                  // column tiles per block (at most)
  static constexpr int FA = BMT * KU;                    // activation fragments per stage
  static constexpr int FMAX = FA + NBMAX * KU;           // fragments per stage (at most)
  static constexpr int J = (FMAX + 7) / 8;               // fragment loads per wave per stage
  static constexpr int STAGE_BYTES = FMAX * 1024;
  static constexpr int PMAX = (T2D_LDS_BYTES - T2D_SS_BYTES) / STAGE_BYTES;
  static constexpr int P = GL ? (PMAX > 6 ? 6 : PMAX) : 2;  // LDS stages
  static constexpr int LDS_BYTES = P * STAGE_BYTES + T2D_SS_BYTES;
  static_assert(WM * WN == 8, "8 waves per workgroup");
  static_assert(!GL || (P >= 3 && J * (P - 2) <= 63), "LDS-DMA ring: 3+ stages, vmcnt is 6 bits");
};

// blockIdx -> (column group, row block, k split): the MB x S blocks of one column group share
// blockIdx % 8 (one XCD) when the grid allows it.  Placement only - never correctness.
__device__ __forceinline__ void t2d_place(int MB, int S, int& cg, int& mb, int& sp) {
  const int b = blockIdx.x, G = gridDim.x, per = MB * S;
  int u;
  if (G % (8 * per) == 0) {
    const int j = b >> 3;
    u = j % per;
    cg = (j / per) * 8 + (b & 7);
  } else {
    u = b % per;
    cg = b / per;
  }
  mb = u / S;
  sp = u - mb * S;
}

template <int N>
__device__ __forceinline__ void t2d_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MW, int NW, int WM, int WN, int D, int KU, bool GL, int EPI, bool OPK, bool SPLIT>
__global__ __launch_bounds__(512) void gemm_t2d_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wp,
                                                       bf16_t* __restrict__ y, int64_t ys,
                                                       const bf16_t* __restrict__ res, int64_t rs,
                                                       float* __restrict__ part, int M, int N, int K, int MB, int S,
                                                       int nbig, int NBB, int NBS, const EpiArgs ep) {
  using G = T2dGeom<MW, NW, WM, WN, D, KU, GL>;
  constexpr int BMT = G::BMT, FA = G::FA, J = G::J, P = G::P, SB = G::STAGE_BYTES;
  clear_other(ep);
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS_BYTES];
  auto* rs_part = reinterpret_cast<u64(*)[SS_ROWS]>(smem + P * SB);
  float* rs_lds = reinterpret_cast<float*>(smem + P * SB + SS_PG * SS_ROWS * 8);
  RowScale<(EPI < 2) && !SPLIT> rsc;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid % WM, wn = wid / WM;
  int cg, mb, sp;
  t2d_place(MB, S, cg, mb, sp);
  const int tile0 = cg < nbig ? cg * NBB : nbig * NBB + (cg - nbig) * NBS;
  const int ntl = cg < nbig ? NBB : NBS;                  // column tiles of this block
  const int mto = ep.mt_out, mt0 = mb * BMT;              // packed row tiles; this block's first
  const int nks = K >> 5, nst = nks / KU;
  const int st0 = (int)((int64_t)sp * nst / S), st1 = (int)((int64_t)(sp + 1) * nst / S), n = st1 - st0;
  const int F = FA + ntl * KU;                            // fragments per stage of this block

  // this wave's J fragment streams: global base at stage st0, per-stage increment, LDS slot.
  // Typed global (address space 1): a stream whose base is picked between the activation and the
  // weight pointer at run time otherwise compiles to flat loads, which the per-stage barrier's
  // lgkmcnt(0) waits for - draining the whole register ring every stage.
  typedef __attribute__((address_space(1))) const bf16_t gbf16_t;
  const gbf16_t* gp[J];
  int64_t ginc[J];
  int slot[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int f = min(wid + 8 * j, F - 1);  // surplus loads repeat the last fragment (same bytes, same slot)
    slot[j] = f;
    if (f < FA) {
      const int u = f / BMT, mt = min(mt0 + f % BMT, mto - 1);
      gp[j] = (const gbf16_t*)x + (((int64_t)(st0 * KU + u) * mto + mt) << 9) + lane * 8;
      ginc[j] = (int64_t)KU * mto * 512;
    } else {
      const int g = f - FA, t = g / KU, u = g % KU;
      gp[j] = (const gbf16_t*)wp + (((int64_t)(tile0 + t) * nks + st0 * KU + u) << 9) + lane * 8;
      ginc[j] = KU * 512;
    }
  }
  // which of this wave's tiles are real (wave-uniform)
  const int ntw = min(NW, ntl - wn * NW);                  // column tiles of this wave (may be <= 0)
  const int mtw = min(MW, mto - (mt0 + wm * MW));          // row tiles of this wave

  // loads whose results are used only after the loop go first (vmcnt retires in issue order: the
  // ring's counted waits never wait for them).  EPI 3: this wave's residual quads.
  u16x4 rpre[MW][NW];
  if constexpr (EPI == 3 && !SPLIT) {
#pragma unroll
    for (int mt = 0; mt < MW; ++mt)
#pragma unroll
      for (int t = 0; t < NW; ++t) {
        const int col = (tile0 + min(wn * NW + t, ntl - 1)) * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          rpre[mt][t][r] = res[(int64_t)min((mt0 + wm * MW + mt) * 16 + (lane >> 4) * 4 + r, M - 1) * rs + col];
      }
  }
  rsc.load(ep, wp);

  f32x4 acc[MW][NW];
#pragma unroll
  for (int mt = 0; mt < MW; ++mt)
#pragma unroll
    for (int t = 0; t < NW; ++t) acc[mt][t] = (f32x4)(0.f);

  // compute one stage from LDS stage buffer at byte offset ``off`` (every tile of the wave: tiles
  // past the block's rows / columns compute on stale LDS and are never stored - no per-MFMA branches)
#define T2D_MMA(off)                                                                                     \
  {                                                                                                      \
    const unsigned char* sb_ = smem + (off) + lane * 16;                                                 \
    u16x8 a_[KU][MW], b_[KU][NW];                                                                        \
    _Pragma("unroll") for (int u = 0; u < KU; ++u) {                                                     \
      _Pragma("unroll") for (int mt = 0; mt < MW; ++mt) a_[u][mt] =                                      \
          *reinterpret_cast<const u16x8*>(sb_ + (u * BMT + wm * MW + mt) * 1024);                        \
      _Pragma("unroll") for (int t = 0; t < NW; ++t) b_[u][t] =                                          \
          *reinterpret_cast<const u16x8*>(sb_ + (FA + (wn * NW + t) * KU + u) * 1024);                   \
    }                                                                                                    \
    _Pragma("unroll") for (int u = 0; u < KU; ++u) _Pragma("unroll") for (int mt = 0; mt < MW; ++mt)      \
        _Pragma("unroll") for (int t = 0; t < NW; ++t) acc[mt][t] = mfma16(a_[u][mt], b_[u][t], acc[mt][t]); \
  }

  if constexpr (GL) {
    // LDS-DMA ring of P stages: stage s lives in slot s % P.  At step s: wait for this wave's part
    // of stage s (counted: the P - 2 younger stages stay in flight), barrier (everyone's part of
    // stage s landed, everyone finished step s - 1), refill the slot step s - 1 used with stage
    // s + P - 1, compute stage s.  The LDS image of a fragment is lane-linear (64 lanes x 16 B),
    // exactly what one global_load_lds_dwordx4 writes.
    typedef __attribute__((address_space(3))) void* lptr_t;
    auto issue = [&](int sl, int st) {
      const int64_t s_ = min(st, n - 1);
#pragma unroll
      for (int j = 0; j < J; ++j)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(gp[j] + s_ * ginc[j]),
                                         (lptr_t)(smem + sl * SB + slot[j] * 1024), 16, 0, 0);
    };
#pragma unroll
    for (int p = 0; p < P - 1; ++p) issue(p, p);
    int cur = 0;  // slot of stage s
    for (int s = 0; s < n; ++s) {
      t2d_wait_vm<J * (P - 2)>();
      lds_barrier();
      issue(cur == 0 ? P - 1 : cur - 1, s + P - 1);
      T2D_MMA(cur * SB)
      cur = cur + 1 == P ? 0 : cur + 1;
    }
    t2d_wait_vm<0>();  // the clamped refills of the last steps
  } else {
    u16x8 stg[D][J];
#define T2D_LOAD(d, st)                                                                                  \
  {                                                                                                      \
    const int64_t s_ = min(st, n - 1);                                                                   \
    _Pragma("unroll") for (int j = 0; j < J; ++j) stg[d][j] =                                            \
        *reinterpret_cast<__attribute__((address_space(1))) const u16x8*>(gp[j] + s_ * ginc[j]);          \
  }
#define T2D_STORE(d, buf)                                                                                \
  _Pragma("unroll") for (int j = 0; j < J; ++j) *reinterpret_cast<u16x8*>(                              \
      smem + (buf) * SB + slot[j] * 1024 + lane * 16) = stg[d][j];
#pragma unroll
    for (int d = 0; d < D; ++d) T2D_LOAD(d, d)
    T2D_STORE(0, 0)
    T2D_LOAD(0, D)
    lds_barrier();
    // invariant at the top of step s: LDS buffer s & 1 holds stage s; the ring holds stages
    // s + 1 .. s + D (slot (s + 1) % D is the oldest)
    for (int s0 = 0; s0 < n; s0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int s = s0 + d;
        if (s >= n) break;
        // D even: the LDS buffer of step s is d & 1
        T2D_MMA((d & 1) * SB)
        // (at s = n - 1 this stages a clamped copy nobody reads: no branch around the ring)
        T2D_STORE((d + 1) % D, (d + 1) & 1)
        T2D_LOAD((d + 1) % D, s + 1 + D)
        lds_barrier();
      }
    }
#undef T2D_STORE
#undef T2D_LOAD
  }
#undef T2D_MMA

  if constexpr (SPLIT) {
    float* slab = part + (int64_t)sp * M * N;
    const int cl = lane & 15, q = lane >> 4;
#pragma unroll
    for (int mt = 0; mt < MW; ++mt)
#pragma unroll
      for (int t = 0; t < NW; ++t) {
        if (mt >= mtw || t >= ntw) continue;
        const int col = (tile0 + wn * NW + t) * 16 + cl;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = (mt0 + wm * MW + mt) * 16 + q * 4 + r;
          if (row < M) slab[(int64_t)row * N + col] = acc[mt][t][r];
        }
      }
  } else {
    rsc.finish(ep, rs_part, rs_lds);  // (barriers inside: every wave calls it)
#pragma unroll
    for (int mt = 0; mt < MW; ++mt)
#pragma unroll
      for (int t = 0; t < NW; ++t) {
        if (mt >= mtw || t >= ntw) continue;
        if (EPI == 1 && (t & 1)) continue;  // up tile: consumed with its gate tile
        tile_epilogue<BMT, EPI, OPK>(mt0 + wm * MW + mt, tile0 + wn * NW + t, acc[mt][t],
                                     EPI == 1 ? acc[mt][(t + 1) % NW] : acc[mt][t], y, ys, res, rs, M, lane, ep,
                                     rs_lds, EPI == 3 ? &rpre[mt][t] : nullptr);
      }
  }
}

// Geometry chooser + launcher.  Returns 1 (caller falls back) when the shape is not covered.
// ``S_force`` > 0 forces the k split (lab); 0 picks (t2d_pick_split).
// ``dry``: only report coverage.
template <int MW, int NW, int WM, int WN, int D, int KU, bool GL>
static int launch_t2d_cfg(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, float* part,
                          int M, int N, int K, int epi, bool opk, int MB, int S, int G, int nbig, int NBB, int NBS,
                          const EpiArgs& ep, hipStream_t stream) {
#define T2D_L(EPI_, OPK_, SPLIT_)                                                                                  \
  hipLaunchKernelGGL((gemm_t2d_kernel<MW, NW, WM, WN, D, KU, GL, EPI_, OPK_, SPLIT_>), dim3(G), dim3(512), 0, stream, \
                     (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, part, M, N, K, MB, \
                     S, nbig, NBB, NBS, ep)
  if (S > 1) {
    T2D_L(0, false, true);
  } else if (epi == 1) {
    if constexpr (NW % 2 == 0) {
      if (opk) T2D_L(1, true, false); else T2D_L(1, false, false);
    } else {
      return 1;
    }
  } else if (epi == 3) {
    if constexpr (MW * NW <= 8) T2D_L(3, false, false); else return 1;  // (wider producers would spill)
  } else if (epi == 0) {
    T2D_L(0, false, false);
  } else {
    return 1;
  }
#undef T2D_L
  return 0;
}

// K split: two for the residual-stream producers (o, down: the reduce launch applies the epilogue)
// - the column groups double in width, so per CU the activation intake halves for 1.5x the weight
// intake: LDS-DMA form at 256 rows o 28.0 -> 23.5 us, down 60.7 -> 44.0 us (reduce included).  The
// row-scaled qkv consumer splits only in the register-ring form (49.9 -> 46.2 us; LDS-DMA form 44.0
// unsplit vs 45.7 split).  SwiGLU never (its epilogue needs the whole sum).
static inline int t2d_pick_split(int K, int epi, bool gl, int S_force) {
  if (S_force > 0) return S_force;
  if (epi == 3) return 2;
  return (epi == 0 && !gl) ? 2 : 1;
}

// WM = 4 x WN = 2 waves, MW = 2 (128-row blocks); NW by the column-group width.  flags bit 18:
// the LDS-DMA ring (2 k-slices per stage while a stage fits in 32 KB, else 1, so 4+ stages fit in
// LDS).  (64-row blocks - a quarter of the activation intake per block for twice the weight
// intake - measured slower on every shape, profiles/r5x, and were removed.)
static int launch_gemm_t2d(const void* x, const void* w, void* y, int64_t ys, const void* res, int64_t rs, int M,
                           int N, int K, int epi, int flags, const EpiArgs& ep, void* ws, hipStream_t stream,
                           int S_force = 0, bool dry = false) {
  constexpr int D = 4;
  const int mto = (M + 15) / 16;
  if (M <= 64 || M > 256 || N % 16 || K % 128 || (flags & 2 && epi != 1)) return 1;
  if (!(epi == 0 || epi == 1 || epi == 3)) return 1;
  // the SwiGLU consumer (gate/up: 6-tile waves) keeps the register ring: 4 stages of 40 KB in
  // registers against the LDS-DMA ring's 5 of 20 KB, 1-4 % faster at 192 / 256 rows (profiles/r5x)
  bool gl = (flags & 262144) && epi != 1;
  const int MB = (mto + 7) / 8;
  const int S = t2d_pick_split(K, epi, gl, S_force);
  if (S > 1 && (epi == 1 || ws == nullptr || (int64_t)S * M * N * 4 > RWK_SLAB_BYTES || N % (256 * SKR_CPT)))
    return 1;
  if (K / 64 < 2 * S) return 1;
  const int step = epi == 1 ? 2 : 1;
  const int units = (N / 16) / step;
  const int C0 = sk_num_cus();
  int NB = C0 / (MB * S);  // column groups for one block per CU
  if (NB < 1) NB = 1;
  if (NB > units) NB = units;
  const int base = units / NB, rem = units % NB;
  const int NBB = (base + (rem ? 1 : 0)) * step, NBS = base * step;
  const int nbig = rem ? rem : NB;
  const int G = NB * MB * S;
  float* part = S > 1 ? (float*)((char*)ws + (int64_t)SK_MAX_GROUPS * sizeof(int) + SK_ZERO_BYTES +
                                 (int64_t)SK_MAX_BLOCKS * 2 * SK_MAX_S * 64 * sizeof(float))
                      : nullptr;
  const bool opk = flags & 2;
  // the narrowest wave width that holds NBB tiles on 2 column waves (even for SwiGLU pairs)
  int nw = (NBB + 1) / 2;
  if (epi == 1 && nw % 2) ++nw;
  if (nw == 8) gl = true;  // 8-tile waves (Llama-3-8B gate/up): a register ring would spill
  int rc;
#define T2D_KU(MW_, NW_) ((4 * MW_ + 2 * NW_) * 2 <= 32 ? 2 : 1)
#define T2D_C(NW_)                                                                                                 \
  rc = dry ? 0                                                                                                     \
     : gl  ? launch_t2d_cfg<2, NW_, 4, 2, D, T2D_KU(2, NW_), true>(x, w, y, ys, res, rs, part, M, N, K, epi, opk,   \
                                                                  MB, S, G, nbig, NBB, NBS, ep, stream)             \
           : launch_t2d_cfg<2, NW_, 4, 2, D, 2, false>(x, w, y, ys, res, rs, part, M, N, K, epi, opk, MB, S, G, nbig, \
                                                      NBB, NBS, ep, stream)
  switch (nw) {
    case 1: if (epi == 1) return 1; T2D_C(1); break;
    case 2: T2D_C(2); break;
    case 3: if (epi == 1) return 1; T2D_C(3); break;
    case 4: T2D_C(4); break;
    case 6: T2D_C(6); break;
    case 8:
      rc = dry ? 0 : launch_t2d_cfg<2, 8, 4, 2, D, 1, true>(x, w, y, ys, res, rs, part, M, N, K, epi, opk, MB, S, G,
                                                           nbig, NBB, NBS, ep, stream);
      break;
    default: return 1;
  }
#undef T2D_C
#undef T2D_KU
  if (rc != 0 || dry) return rc;
  if (S > 1) {
    const dim3 g2(N / (256 * SKR_CPT), M);
    launch_splitk_reduce(S, epi, g2, stream, part, M, N, y, ys, res, rs, ep);
  }
  return 0;
}

}  // namespace mp
