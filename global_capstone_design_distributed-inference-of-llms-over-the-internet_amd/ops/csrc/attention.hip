// Paged flash-decoding attention for gfx950 (survey K6 + K7).
//
// The reference materialises repeat_kv'd K/V and a full [B, H, T, P+T] fp32
// score matrix with two matmuls (reference petals/llama/block.py:131-141).
// This kernel reads each cached K/V row once, straight from its page:
//
//   grid  = (num_parts, nkv, T)   one workgroup per (query row, kv head, context slice)
//   block = 256 threads (4 waves of 64)
//
// Each workgroup serves NREP (<= nh / nkv) query heads of one kv head (GQA without
// materialising repeat_kv): blockIdx.y * NREP is its first query head, so a GQA group of
// 8 heads runs as two workgroups of 4 (K/V re-read from L2, half the q/acc registers:
// the register count, not the math, limits how many K/V bytes a CU keeps in flight).  Lane mapping: LPT = D/8 lanes per token, each lane owns 8
// head dims (one 16-B load); a wave-instruction covers 64/LPT consecutive tokens, i.e.
// 1 KiB of contiguous cache.  Partial dot products are summed over the LPT lanes with
// DPP row permutes (no LDS traffic), scores live in LDS, softmax is done in the exp2
// domain, and P.V accumulates in fp32 registers.  With num_parts > 1 each slice
// writes (o, m, l) partials that `paged_attn_reduce` combines (split-K over context).
//
// Queries carry their own (sequence row, context length), so the same kernel runs
// decode (one query per sequence), chunked prefill (query i of a chunk sees
// ctx = start + i + 1 -> causal) and replay.  ctx == 0 rows (batch padding) output 0.
// packed_mt > 0 writes the output in the packed decode-GEMM activation layout (common.h).
//
// ROPE = true (decode only: one query per sequence, its own token is the last of the context):
// `q` is the UNROTATED fused qkv projection row and the kernel does rope_kv.hip's work itself,
// removing one launch + one qkv round trip per layer.  Every lane rotates its 8-dim chunk of
// the query heads and of the new token's k (rotate_half: the partner chunk sits D/2 away,
// fp32 cos/sin at pos[t], same expression order as rope_kv_kernel), keeps the rotated k and
// the v chunk in registers and substitutes them for the cache read of token ctx - 1; the
// first workgroup of the kv head whose context slice holds that token writes them to the
// page slot (slots[t] < 0: padded row, nothing written) for later steps.
#include "attn_common.h"
#include <stdlib.h>

// K/V page loads of the single-pass decode kernel: each cached row is read once per step, so
// by default they carry the non-temporal hint (MI355X_MICROARCH nt-weights: issued -> landed
// ~18 % shorter for once-read streams).  -DMP_ATTN_KV_NT=0 builds the default-policy ablation.
#ifndef MP_ATTN_KV_NT
#define MP_ATTN_KV_NT 1
#endif
#if MP_ATTN_KV_NT
#define MP_KV_LOAD(p) __builtin_nontemporal_load(p)
#else
#define MP_KV_LOAD(p) (*(p))
#endif

// minimum waves per SIMD the decode attention's register allocation must allow (4: 128 VGPRs; the
// dot2 form needs 122, the round-5 form 124) - an ablation knob for MPAMD_HIPCC_EXTRA lab builds
#ifndef MP_ATTN_MINW
#define MP_ATTN_MINW 4
#endif
// waves per workgroup of the flash-decoding kernel, picked per launch from the grid size (below);
// MP_ATTN_NW forces 4 or 8 (lab builds)
#ifndef MP_ATTN_NW
#define MP_ATTN_NW 0
#endif

namespace mp {

struct RopeFuse {
  const int64_t* pos;   // [T] rotary positions
  const float* cos_t;   // [max_pos, D/2]
  const float* sin_t;
  const int64_t* slots; // [T] cache slot of the new token (page * page_size + offset)
  bf16_t* kw;           // the k / v caches, written only at the new token's slot
  bf16_t* vw;
  QkvPart qp;           // qp.part != nullptr: q / k / v from the qkv GEMM's split-K partials
};

// The folded qkv projection (rf.qp: split-K partial slabs): the workgroup's NREP rotated query
// chunks, the rotated new key and the new value of token t, built once into LDS s[(NREP + 2) * D/8]
// (item-major, 8 columns per entry).  Bit-identical to RoPE over the reduce launch's bf16 row.
// Every thread of the workgroup must call it (ends in a barrier; qrs from qkv_part_scale).
template <int D, int NREP>
__device__ __forceinline__ void fold_qkv_lds(const RopeFuse& rf, int t, int hbase, int g, int nh, int nkv, float qrs,
                                             u16x8* s) {
  constexpr int LPT = D / 8, HALF = D / 2;
  const int64_t ps_ = rf.pos[t];
  for (int i = threadIdx.x; i < (NREP + 2) * LPT; i += blockDim.x) {
    const int item = i / LPT, sl = i % LPT;
    const int hc = item < NREP ? (hbase + item) * D : item == NREP ? (nh + g) * D : (nh + nkv + g) * D;
    const u16x8 me = qkv_part_load8(rf.qp, t, hc + sl * 8, qrs);
    if (item == NREP + 1) {
      s[i] = me;  // the value: no rotation
      continue;
    }
    const int c0 = (sl * 8) & (HALF - 1);
    const bool lo = sl * 8 < HALF;
    const u16x8 ot = qkv_part_load8(rf.qp, t, hc + sl * 8 + (lo ? HALF : -HALF), qrs);
    const f32x4 ca = *reinterpret_cast<const f32x4*>(rf.cos_t + ps_ * HALF + c0);
    const f32x4 cb = *reinterpret_cast<const f32x4*>(rf.cos_t + ps_ * HALF + c0 + 4);
    const f32x4 sa = *reinterpret_cast<const f32x4*>(rf.sin_t + ps_ * HALF + c0);
    const f32x4 sb = *reinterpret_cast<const f32x4*>(rf.sin_t + ps_ * HALF + c0 + 4);
    s[i] = rope8(me, ot, ca, cb, sa, sb, lo);
  }
  __syncthreads();
}

// In-launch split-K combine (NP > 1 with a counter buffer): every context-slice workgroup of a
// (query, head group) publishes its partials (plain stores, every wave drained, one agent-scope
// release by lane 0 before the arrival ticket), and the LAST arriver (ticket NP - 1) acquires,
// sums the NP slices in slice order (the same arithmetic as paged_attn_reduce_kernel, so the
// result is identical and deterministic) and writes the output; it re-zeroes the counter, so a
// zeroed buffer stays valid across launches and graph replays.  Saves the reduce launch (batch 1:
// ~4.8 us per layer, r2 profile).  Called by every thread of the workgroup.
template <int D, int NREP>
__device__ __forceinline__ void split_combine(int* cnt_slot, int NP, const float* part_o, const float* part_ml, int t,
                                              int hbase, int nh, bf16_t* out, int packed_mt, float* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(cnt_slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == NP - 1;
    if (last) {
      __hip_atomic_store(cnt_slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_flag[0] = last ? 1.f : 0.f;
  }
  __syncthreads();
  if (s_flag[0] == 0.f) return;
  for (int i = threadIdx.x; i < NREP * D; i += blockDim.x) {
    const int r = i / D, d = i - r * D;
    const int64_t h = (int64_t)t * nh + hbase + r;
    const float* ml = part_ml + h * NP * 2;
    float M = -INFINITY;
    for (int p = 0; p < NP; ++p)
      if (ml[2 * p + 1] > 0.f) M = fmaxf(M, ml[2 * p]);
    float num = 0.f, den = 0.f;
    for (int p = 0; p < NP; ++p) {
      const float l = ml[2 * p + 1];
      if (l > 0.f) {
        const float wgt = exp2f(ml[2 * p] - M);
        num += wgt * part_o[(h * NP + p) * D + d];
        den += wgt * l;
      }
    }
    const float v = den > 0.f ? num / den : 0.f;
    out[packed_mt > 0 ? apk_off(t, (hbase + r) * D + d, packed_mt) : h * D + d] = f2bf(v);
  }
}

// The decode kernel is single-pass.  (A two-pass form - K read, scores published to LDS, a
// barrier, then the V stream - kept ONE stream in flight per workgroup and idled the whole grid
// at the barrier; it was measured slower and removed.)  Each lane keeps an ONLINE softmax over the tokens it sees (running max m, sum l and the
// 8-dim P.V accumulator, exp2 domain), so the K and V loads of an iteration are issued together
// (8 x 16 B per lane in flight) and the page ids of the next iteration are fetched into registers
// while the current one computes (no dependent page-table round trip on the critical path).  The
// 4 token groups of a wave merge by xor shuffles, the 4 waves through LDS (rescaled by their
// maxima), and the output / split-K partials (o, m, l) have the two-pass kernel's format.
// NW = waves per workgroup (4 or 8 by grid size, launch_attn), PIPE = software-pipelined K / V
// stream (always on).
// (16-wave workgroups for small grids stopped paying once the 4-wave form was pipelined,
// profiles/r4o; the unpipelined form measured slower: both removed.)
template <int D, int NREP, bool ROPE, int NW, bool PIPE, int U = 4>
__global__ __launch_bounds__(NW * 64, MP_ATTN_MINW) void paged_attn1_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ kc,
    const bf16_t* __restrict__ vc, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ q_seq, const int32_t* __restrict__ q_ctx, bf16_t* __restrict__ out,
    float* __restrict__ part_o, float* __restrict__ part_ml, int nkv, int nh, int page_log2, int PS, int NP,
    float scale_log2, int packed_mt, RopeFuse rf, int* __restrict__ cnt) {
  constexpr int LPT = D / 8;
  constexpr int TPI = 64 / LPT;
  static_assert(U % 2 == 0, "P V pairs the tokens u, u + 1");
  // U: tokens per lane group per iteration (U = 8 measured 32 -> 43 us at 64 x 170, profiles/r4d)
  constexpr int TPW = TPI * U;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT_ = NW * 64;
  float* s_o = smem;                   // [NW][NREP][D] per-wave accumulators
  float* s_m = smem + NW * NREP * D;   // [NW][NREP] per-wave maxima
  float* s_l = s_m + NW * NREP;        // [NW][NREP] per-wave sums

  const int t = blockIdx.z, p = blockIdx.x;
  const int hbase = blockIdx.y * NREP;
  const int g = hbase / (nh / nkv);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int sl = lane % LPT, tg = lane / LPT;
  const int ctx = q_ctx[t];
  const int start = p * PS;
  const int end = min(start + PS, ctx);
  const int64_t obase = ((int64_t)t * nh + hbase) * D;
  if (start >= end) {
    if (NP == 1) {
      for (int i = tid; i < NREP * D; i += NT_)
        out[packed_mt > 0 ? apk_off(t, hbase * D + i, packed_mt) : obase + i] = 0;
    } else {
      if (tid < NREP) {
        float* ml = part_ml + (((int64_t)t * nh + hbase + tid) * NP + p) * 2;
        ml[0] = -INFINITY;
        ml[1] = 0.f;
      }
      if (cnt != nullptr)
        split_combine<D, NREP>(cnt + (int64_t)t * (nh / NREP) + blockIdx.y, NP, part_o, part_ml, t, hbase, nh, out,
                               packed_mt, smem);
    }
    return;
  }
  const int page_size = 1 << page_log2;
  const int32_t* bt = block_tables + (int64_t)q_seq[t] * bt_stride;
  const int64_t head_off = (int64_t)g * page_size * D + sl * 8;
  const int64_t page_stride = (int64_t)nkv * page_size * D;
  // page ids of this wave's first iteration (then prefetched one iteration ahead)
  int pgn[U];
  {
    const int b0 = start + w * TPW;
#pragma unroll
    for (int u = 0; u < U; ++u) pgn[u] = bt[min(b0 + u * TPI + tg, end - 1) >> page_log2];
  }

  auto issue = [&](int b, const int* pg, u16x8* kd, u16x8* vd) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tc = min(b + u * TPI + tg, end - 1);
      const int64_t off = (int64_t)pg[u] * page_stride + head_off + (int64_t)(tc & (page_size - 1)) * D;
      kd[u] = MP_KV_LOAD(reinterpret_cast<const u16x8*>(kc + off));
      vd[u] = MP_KV_LOAD(reinterpret_cast<const u16x8*>(vc + off));
    }
  };
  auto page_ids = [&](int b, int* pg) {
#pragma unroll
    for (int u = 0; u < U; ++u) pg[u] = bt[min(b + u * TPI + tg, end - 1) >> page_log2];
  };
  // first iteration's K / V (PIPE) issued here, ahead of the query / RoPE loads: the cache
  // stream's round trip overlaps the rotary-table round trip instead of following it
  u16x8 kv[U], vv[U];
  int pgm[U];
  if constexpr (PIPE) {
    page_ids(start + w * TPW + NW * TPW, pgm);
    issue(start + w * TPW, pgn, kv, vv);
  }

  // q as packed bf16 pairs, unscaled (the log2 softmax scale goes on the reduced score): the QK
  // dot products run on v_dot2c_f32_bf16 straight from the bf16 K lanes
  u32x4a qp[NREP];
  u16x8 kn = (u16x8)(0), vn = (u16x8)(0);
  int tnew = -1;
  if constexpr (ROPE) {
    constexpr int HALF = D / 2;
    const bf16_t* row = q + (int64_t)t * q_stride;
    const int c0 = (sl * 8) & (HALF - 1);
    const bool lo = sl * 8 < HALF;
    const int po = lo ? HALF : -HALF;
    if (rf.qp.part != nullptr) {
      // the qkv split-K partials: this workgroup's q / k / v chunks built once into LDS (every slab
      // element read once per workgroup, not once per token group of every wave)
      __shared__ u16x8 s_fold[(NREP + 2) * LPT];
      fold_qkv_lds<D, NREP>(rf, t, hbase, g, nh, nkv, qkv_part_scale(rf.qp, t), s_fold);
#pragma unroll
      for (int r = 0; r < NREP; ++r) qp[r] = __builtin_bit_cast(u32x4a, s_fold[r * LPT + sl]);
      kn = s_fold[NREP * LPT + sl];
      vn = s_fold[(NREP + 1) * LPT + sl];
    } else {
      const int64_t ps_ = rf.pos[t];
      const f32x4 ca = *reinterpret_cast<const f32x4*>(rf.cos_t + ps_ * HALF + c0);
      const f32x4 cb = *reinterpret_cast<const f32x4*>(rf.cos_t + ps_ * HALF + c0 + 4);
      const f32x4 sa = *reinterpret_cast<const f32x4*>(rf.sin_t + ps_ * HALF + c0);
      const f32x4 sb = *reinterpret_cast<const f32x4*>(rf.sin_t + ps_ * HALF + c0 + 4);
      auto rot = [&](int hc) {  // hc: first column of the head in the qkv row
        const u16x8 me = *reinterpret_cast<const u16x8*>(row + hc + sl * 8);
        const u16x8 ot = *reinterpret_cast<const u16x8*>(row + hc + sl * 8 + po);
        return rope8(me, ot, ca, cb, sa, sb, lo);
      };
#pragma unroll
      for (int r = 0; r < NREP; ++r) qp[r] = __builtin_bit_cast(u32x4a, rot((hbase + r) * D));
      kn = rot((nh + g) * D);
      vn = *reinterpret_cast<const u16x8*>(row + (nh + nkv + g) * D + sl * 8);
    }
    tnew = ctx - 1;
    const int64_t slot = rf.slots[t];
    if (tnew >= start && tnew < end && slot >= 0 && tid < LPT && hbase % (nh / nkv) == 0) {
      const int64_t pg = slot >> page_log2, off = slot & (page_size - 1);
      const int64_t dst = pg * page_stride + head_off + off * D;
      *reinterpret_cast<u16x8*>(rf.kw + dst) = kn;
      *reinterpret_cast<u16x8*>(rf.vw + dst) = vn;
    }
  } else {
#pragma unroll
    for (int r = 0; r < NREP; ++r)
      qp[r] = *reinterpret_cast<const u32x4a*>(q + (int64_t)t * q_stride + (hbase + r) * D + sl * 8);
  }

  float m[NREP], l[NREP], acc[NREP][8];
#pragma unroll
  for (int r = 0; r < NREP; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[r][j] = 0.f;
  }
  auto compute = [&](int base, u16x8 (&kv)[U], u16x8 (&vv)[U]) {
    if constexpr (ROPE) {
      // the new token's k / v from registers (its cache slot is written by this very launch):
      // only the wave iteration that holds it pays the selects (a wave-uniform branch)
      if (tnew >= base && tnew < base + TPW) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int tok = base + u * TPI + tg;
          kv[u] = tok == tnew ? kn : kv[u];
          vv[u] = tok == tnew ? vn : vv[u];
        }
      }
    }
#pragma unroll
      for (int r = 0; r < NREP; ++r) {
        float s[U];
        float mx = m[r];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const u32x4a kw = __builtin_bit_cast(u32x4a, kv[u]);
          float d0 = dot2bf(qp[r][0], kw[0], 0.f), d1 = dot2bf(qp[r][1], kw[1], 0.f);
          d0 = dot2bf(qp[r][2], kw[2], d0);
          d1 = dot2bf(qp[r][3], kw[3], d1);
          const float d = group_sum<LPT>(d0 + d1) * scale_log2;
          s[u] = base + u * TPI + tg < end ? d : -INFINITY;
          mx = fmaxf(mx, s[u]);
        }
        const float mref = mx == -INFINITY ? 0.f : mx;
        const float sc = __builtin_amdgcn_exp2f(m[r] - mref);
        l[r] *= sc;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[r][j] *= sc;
        // P V two tokens at a time: the probabilities of tokens u, u + 1 as one bf16 pair (the FA2
        // convention: P rounds to bf16 for the PV product; l sums the same rounded values), the
        // two tokens' V elements paired by v_perm_b32, one v_dot2c_f32_bf16 per output element
#pragma unroll
        for (int u = 0; u < U; u += 2) {
          // (v_exp_f32 directly: the arguments are <= 0, exp2(-inf) = 0; a result below the fp32
          // normal range is 0 for bf16 P anyway)
          const bf16_t b0 = f2bf(__builtin_amdgcn_exp2f(s[u] - mref)), b1 = f2bf(__builtin_amdgcn_exp2f(s[u + 1] - mref));
          l[r] += bf2f(b0) + bf2f(b1);
          const unsigned pp = (unsigned)b0 | ((unsigned)b1 << 16);
          const u32x4a v0 = __builtin_bit_cast(u32x4a, vv[u]), v1 = __builtin_bit_cast(u32x4a, vv[u + 1]);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            acc[r][2 * jj] = dot2bf(pp, __builtin_amdgcn_perm(v1[jj], v0[jj], 0x05040100u), acc[r][2 * jj]);
            acc[r][2 * jj + 1] = dot2bf(pp, __builtin_amdgcn_perm(v1[jj], v0[jj], 0x07060302u), acc[r][2 * jj + 1]);
          }
        }
        m[r] = mx;
      }

  };
  if constexpr (PIPE) {
    // software-pipelined: iteration i+1's K / V (and i+2's page ids) are in flight while
    // iteration i computes, so the stream never stops between iterations (the first
    // iteration's loads were issued ahead of the query / RoPE prologue)
    for (int base = start + w * TPW; base < end; base += NW * TPW) {
      const int nb = base + NW * TPW;
      u16x8 kx[U], vx[U];
      page_ids(nb + NW * TPW, pgn);
      if (nb < end) issue(nb, pgm, kx, vx);
      compute(base, kv, vv);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kv[u] = kx[u];
        vv[u] = vx[u];
        pgm[u] = pgn[u];
      }
    }
  } else {
    for (int base = start + w * TPW; base < end; base += NW * TPW) {
      issue(base, pgn, kv, vv);
      // next iteration's page ids, in flight behind the K / V loads
      page_ids(base + NW * TPW, pgn);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        asm volatile("" : "+v"(kv[u]));
        asm volatile("" : "+v"(vv[u]));
      }
      compute(base, kv, vv);
    }
  }
  // merge the token groups of the wave (lanes sl, sl + LPT, ...)
#pragma unroll
  for (int o = LPT; o < 64; o <<= 1) {
#pragma unroll
    for (int r = 0; r < NREP; ++r) {
      const float mo = __shfl_xor(m[r], o, 64);
      const float lo = __shfl_xor(l[r], o, 64);
      const float M = fmaxf(m[r], mo);
      const float mref = M == -INFINITY ? 0.f : M;
      const float a = exp2f(m[r] - mref), b = exp2f(mo - mref);
      l[r] = l[r] * a + lo * b;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[r][j] = acc[r][j] * a + __shfl_xor(acc[r][j], o, 64) * b;
      m[r] = M;
    }
  }
  if (tg == 0) {
#pragma unroll
    for (int r = 0; r < NREP; ++r) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s_o[(w * NREP + r) * D + sl * 8 + j] = acc[r][j];
      if (sl == 0) {
        s_m[w * NREP + r] = m[r];
        s_l[w * NREP + r] = l[r];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < NREP * D; i += NT_) {
    const int r = i / D, d = i - r * D;
    float M = s_m[r];
#pragma unroll
    for (int ww = 1; ww < NW; ++ww) M = fmaxf(M, s_m[ww * NREP + r]);
    const float mref = M == -INFINITY ? 0.f : M;
    float o = 0.f, L = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      const float a = exp2f(s_m[ww * NREP + r] - mref);
      o += a * s_o[(ww * NREP + r) * D + d];
      L += a * s_l[ww * NREP + r];
    }
    if (NP == 1) {
      out[packed_mt > 0 ? apk_off(t, hbase * D + i, packed_mt) : obase + i] = f2bf(o / L);
    } else {
      const int64_t hp = ((int64_t)t * nh + hbase + r) * NP + p;
      part_o[hp * D + d] = o;
      if (d == 0) {
        part_ml[hp * 2] = M;
        part_ml[hp * 2 + 1] = L;
      }
    }
  }
  if (NP > 1 && cnt != nullptr)
    split_combine<D, NREP>(cnt + (int64_t)t * (nh / NREP) + blockIdx.y, NP, part_o, part_ml, t, hbase, nh, out,
                           packed_mt, s_m);
}

// Combine split-K partials: one workgroup (D threads) per (query row, head).
__global__ void paged_attn_reduce_kernel(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                                         bf16_t* __restrict__ out, int NP, int D, int nh, int packed_mt) {
  const int64_t h = blockIdx.x;
  const float* ml = part_ml + h * NP * 2;
  float M = -INFINITY;
  for (int p = 0; p < NP; ++p)
    if (ml[2 * p + 1] > 0.f) M = fmaxf(M, ml[2 * p]);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float num = 0.f, den = 0.f;
    for (int p = 0; p < NP; ++p) {
      const float l = ml[2 * p + 1];
      if (l > 0.f) {
        const float wgt = exp2f(ml[2 * p] - M);
        num += wgt * part_o[(h * NP + p) * D + d];
        den += wgt * l;
      }
    }
    const float v = den > 0.f ? num / den : 0.f;
    if (packed_mt > 0)
      out[apk_off((int)(h / nh), (int)(h % nh) * D + d, packed_mt)] = f2bf(v);
    else
      out[h * D + d] = f2bf(v);
  }
}

template <int D, int NREP, int NW>
static void launch_attn_nw(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt,
                           int bt_stride, const int32_t* q_seq, const int32_t* q_ctx, void* out, float* ws_o,
                           float* ws_ml, int T, int nkv, int nh, int page_log2, int PS, int NP, float scale_log2,
                           int packed_mt, const RopeFuse& rf, int* cnt, hipStream_t stream) {
  const size_t lds = (size_t)(NW * NREP * D + 2 * NW * NREP + 4) * sizeof(float);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(NP, nh / NREP, T), dim3(64 * NW), lds, stream, (const bf16_t*)q, q_stride,
                       (const bf16_t*)kc, (const bf16_t*)vc, bt, bt_stride, q_seq, q_ctx, (bf16_t*)out, ws_o, ws_ml,
                       nkv, nh, page_log2, PS, NP, scale_log2, packed_mt, rf, cnt);
  };
  if (rf.pos) go(paged_attn1_kernel<D, NREP, true, NW, true>);
  else go(paged_attn1_kernel<D, NREP, false, NW, true>);
}

// Waves per workgroup from the grid: one (query, head group, context part) per workgroup, so a
// small grid (batch 1: 32 workgroups on 256 CUs) runs 8-wave workgroups - a short context is
// covered in one or two dependent iterations (cold 1 x 170 MHA: 10.4 -> 9.9 us) - and every other
// grid 4-wave ones.  (2-wave workgroups, the 64-session step's 2048 in one round of residency,
// measured 36.5 -> 38.1 us cold at 64 x 170: profiles/r6attn.)
template <int D, int NREP>
static void launch_attn(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt,
                        int bt_stride, const int32_t* q_seq, const int32_t* q_ctx, void* out, float* ws_o,
                        float* ws_ml, int T, int nkv, int nh, int page_log2, int PS, int NP, float scale_log2,
                        int packed_mt, const RopeFuse& rf, int* cnt, hipStream_t stream) {
  const int64_t wgs = (int64_t)NP * (nh / NREP) * T;
  const int nw = MP_ATTN_NW ? MP_ATTN_NW : (wgs <= 128 ? 8 : 4);
#define MP_ATTN_NW_CASE(W)                                                                                     \
  if (nw == W) {                                                                                               \
    launch_attn_nw<D, NREP, W>(q, q_stride, kc, vc, bt, bt_stride, q_seq, q_ctx, out, ws_o, ws_ml, T, nkv, nh,  \
                               page_log2, PS, NP, scale_log2, packed_mt, rf, cnt, stream);                     \
    return;                                                                                                    \
  }
  MP_ATTN_NW_CASE(8)
  MP_ATTN_NW_CASE(4)
#undef MP_ATTN_NW_CASE
}

}  // namespace mp

extern "C" int mp_paged_attention(const void* q, int64_t q_stride, const void* kc, const void* vc,
                                  const int32_t* bt, int bt_stride, const int32_t* q_seq, const int32_t* q_ctx,
                                  void* out, float* workspace, int T, int nh, int nkv, int D, int page_size,
                                  int PS, int NP, float scale, int packed_mt, const int64_t* rope_pos,
                                  const float* cos_t, const float* sin_t, const int64_t* slots, int* counters,
                                  int n_counters, const void* qkv_part_v, hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  RopeFuse rf{rope_pos, cos_t, sin_t, slots, (bf16_t*)const_cast<void*>(kc), (bf16_t*)const_cast<void*>(vc),
              QkvPart{nullptr, 0, 0, 0, nullptr, 0.f, 0.f}};
  const QkvPart* qkv_part = static_cast<const QkvPart*>(qkv_part_v);  // layout mirrored by bindings.cpp
  if (qkv_part != nullptr && qkv_part->part != nullptr) {
    if (rope_pos == nullptr || qkv_part->S < 1) return -4;  // partials only on the fused RoPE decode path
    rf.qp = *qkv_part;
  }
  if (T == 0) return 0;
  if (nh % nkv != 0 || PS % 64 != 0 || PS > 2048 || NP < 1) return -1;
  int page_log2 = 0;
  while ((1 << page_log2) < page_size) ++page_log2;
  if ((1 << page_log2) != page_size) return -2;
  const int nrep = nh / nkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  float* ws_o = workspace;
  float* ws_ml = workspace + (int64_t)T * nh * NP * D;
  // heads per workgroup: at most 4 of a GQA group (register budget), a divisor of nrep
  constexpr int hpb_max = 4;
  int hpb = 1;
  while (hpb * 2 <= hpb_max && nrep % (hpb * 2) == 0) hpb *= 2;
  // in-launch combine when the caller's zeroed counters cover every (query, head group)
  int* cnt = (NP > 1 && counters != nullptr && (int64_t)T * (nh / hpb) <= n_counters) ? counters : nullptr;
#define MP_ATTN_CASE(DD, RR)                                                                                  \
  if (D == DD && hpb == RR) {                                                                                 \
    launch_attn<DD, RR>(q, q_stride, kc, vc, bt, bt_stride, q_seq, q_ctx, out, ws_o, ws_ml, T, nkv, nh,       \
                        page_log2, PS, NP, scale_log2, packed_mt, rf, cnt, stream);                           \
    goto launched;                                                                                            \
  }
  MP_ATTN_CASE(128, 1)
  MP_ATTN_CASE(128, 2)
  MP_ATTN_CASE(128, 4)
  MP_ATTN_CASE(64, 1)
  MP_ATTN_CASE(64, 2)
  MP_ATTN_CASE(64, 4)
#undef MP_ATTN_CASE
  return -3;
launched:
  if (NP > 1 && cnt == nullptr) {
    hipLaunchKernelGGL(paged_attn_reduce_kernel, dim3(T * nh), dim3(D), 0, stream, ws_o, ws_ml, (bf16_t*)out, NP,
                       D, nh, packed_mt);
  }
  return (int)hipGetLastError();
}
