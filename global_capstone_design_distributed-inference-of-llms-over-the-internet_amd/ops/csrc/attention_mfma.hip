// MFMA flash attention over the paged KV cache for gfx950 (survey K7: "attn_prefill ...
// MFMA QK^T and PV, LDS tiles"; also GQA decode).
//
// A workgroup (4 waves) owns a block of 16 query ROWS of one kv head: row r is query token
// tok0 + r / HB of one sequence and query head hbase + r % HB (HB = heads of the GQA group
// in the block, TB = 16 / HB tokens).  So MHA prefill processes 16 consecutive tokens per
// block (K/V read once per 16 queries instead of once per query), and GQA decode puts the
// whole group (4 or 8 heads of one token) into the MFMA M dimension.
//
// Per wave and per 32-token step of the context (waves interleave steps):
//   S^T[tok][row] = K[tok, :] . Q[row, :]          2 x (D/32) v_mfma_f32_16x16x32_bf16
//       A = K rows straight from the cache page (lane (q, c): 16 B of token c at d = 8q),
//       B = Q^T fragments held in registers for the whole kernel;
//   online softmax per row in the exp2 domain (row = lane & 15; the 4 lanes of a row
//       combine with two xor shuffles), causal + context masking per row;
//   O[row][d] += P[row][tok] . V[tok][d]            D/16 MFMAs
//       A = P straight from the S^T accumulators: lane (q, c) holds row c at tokens
//       {4q..4q+3, 16+4q..16+4q+3}, used as the MFMA k order,
//       B = V^T read from a per-wave LDS tile [d][32 tok] (row pitch 36 bf16) that the
//       wave fills from the contiguous 8 KiB of V (the tile never straddles a 64-token page;
//       tokens past the context are zeroed so stale cache bytes never meet a p = 0)
//       -> two ds_read_b64 per fragment, in the same permuted k order.
// The 4 waves' (m, l, O) are merged through LDS; with num_parts > 1 the merged partials go
// to the split-K workspace reduced by paged_attn_reduce_kernel (attention.hip).
//
// ROPE = true (GQA decode: every block is ONE token of one sequence, the last of its context):
// `q` is the unrotated fused qkv row and the kernel also does rope_kv.hip's work.  The partner
// of a lane's q chunk kd (rotate_half, D/2 away) is its own chunk kd ^ KD/2, so q rotates in
// registers; the new token's k is rotated the same way, its score q.k_new is summed over the
// 4 lanes of the row with two xor shuffles and replaces the (stale) cache score of token
// ctx - 1, and its v chunk overwrites that token's column of the wave's LDS V tile.  The cache
// loads stay exactly as without ROPE.  Wave 0 of the first block of the kv head whose slice
// holds the token writes k / v to the page slot (slots[t] < 0: nothing written).
// (K/V loads keep the default cache policy here: non-temporal loads, a win for the MHA decode
// kernel in attention.hip, measured 12-14 % SLOWER on this kernel at 64 / 256 sessions, cold
// caches - profiles/r3_i/attn_nt.jsonl vs attn_def.jsonl.)
#include "common.h"
#include "mx_common.h"

namespace mp {

struct RopeFuseM {
  const int64_t* pos;
  const float* cos_t;
  const float* sin_t;
  const int64_t* slots;
  bf16_t* kw;
  bf16_t* vw;
  QkvPart qp;  // qp.part != nullptr: q / k / v from the qkv GEMM's split-K partials (ROPE path)
  uint8_t* mx_ax = nullptr;  // non-null (single-part launches): the output as the W8A8-MX GEMM's
  uint8_t* mx_as = nullptr;  //   activation (mx_common.h) instead of bf16 - the o projection's input
};

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_mf;

__device__ __forceinline__ f32x4 mfma_bf16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mf, a), __builtin_bit_cast(bf16x8_mf, b), c,
                                                 0, 0, 0);
}

constexpr int VT_PITCH = 36;  // bf16 per LDS row of the transposed V tile (32 tokens + pad; 8-B aligned rows)

// FOLD (ROPE only): q / k / v come from the qkv GEMM's split-K slabs through LDS (s_fold).  A
// compile-time choice: as a run-time one the LDS-or-global q / k / v loads compiled to flat
// loads, which count against vmcnt, so the RoPE prologue waited for the K / V stream issued
// before them.
template <int D, int HB, bool ROPE, bool FOLD = false>
__global__ __launch_bounds__(256, 2) void attn_mfma_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int bt_stride, const int32_t* __restrict__ q_seq,
    const int32_t* __restrict__ q_ctx, const int32_t* __restrict__ qb_tok0, const int32_t* __restrict__ qb_ntok,
    bf16_t* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_ml, int nkv, int nh,
    int page_log2, int PS, int NP, float scale_log2, int packed_mt, RopeFuseM rf) {
  constexpr int TB = 16 / HB;
  constexpr int KD = D / 32;  // k-chunks of the QK^T product
  constexpr int DT = D / 16;  // 16-column tiles of O
  __shared__ __attribute__((aligned(16))) bf16_t s_vt[4][D * VT_PITCH];
  __shared__ float s_m[4][16], s_l[4][16];
  __shared__ __attribute__((aligned(16))) float s_o[4][16][D + 1];

  const int b = blockIdx.x, p = blockIdx.z;
  const int hbase = blockIdx.y * HB;
  const int g = hbase / (nh / nkv);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, qd = lane >> 4;
  // ROPE (decode): block b is token b (``decode_qblocks``: one token per block, in order), so the
  // block-table walk starts from q_seq / q_ctx directly - one dependent global load fewer in the
  // chain (q_seq -> page id -> K / V) that sets the decode kernel's time
  const int tok0 = ROPE ? b : qb_tok0[b], ntok = ROPE ? 1 : qb_ntok[b];
  const int seq = q_seq[tok0];
  const int32_t* bt = block_tables + (int64_t)seq * bt_stride;
  const int page_size = 1 << page_log2;
  const int64_t page_stride = (int64_t)nkv * page_size * D;
  const int64_t head_off = (int64_t)g * page_size * D;

  // this lane's row (for Q^T fragments, masking and softmax state): row c
  const int my_t = c / HB, my_h = hbase + c % HB;
  const bool row_ok = my_t < ntok;
  const int my_ctx = row_ok ? q_ctx[tok0 + my_t] : 0;
  int blk_ctx = 0;  // context the block needs = the largest ctx of its tokens (causal: the last)
  for (int i = 0; i < ntok; ++i) blk_ctx = max(blk_ctx, q_ctx[tok0 + i]);
  const int start = p * PS, end = min(start + PS, blk_ctx);

  constexpr int NV = (32 * D * 2) / 1024;  // 16-B V chunks per lane per step
  auto load_k = [&](int bs, int64_t pg, u16x8 (&kr)[2][KD]) {
    const bf16_t* kpage = kc + pg * page_stride + head_off + (int64_t)(bs & (page_size - 1)) * D;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int kd = 0; kd < KD; ++kd)
        kr[sub][kd] = *reinterpret_cast<const u16x8*>(kpage + (int64_t)(sub * 16 + c) * D + kd * 32 + qd * 8);
  };
  auto load_v = [&](int bs, int64_t pg, u16x8 (&vr)[NV]) {
    const bf16_t* vpage = vc + pg * page_stride + head_off + (int64_t)(bs & (page_size - 1)) * D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int ci = i * 64 + lane;
      vr[i] = *reinterpret_cast<const u16x8*>(vpage + (int64_t)(ci % 32) * D + (ci / 32) * 8);
    }
  };
  // K in ping-pong register buffers one step ahead (no register copies: a copy of in-flight
  // loads would force a vmcnt(0) early); a step's V is issued at its top, ahead of the next
  // step's K and the page id two steps ahead, so waiting for it leaves those in flight
  u16x8 ka[2][KD], kb[2][KD], vr[NV];
  int64_t pg_cur = 0, pg_next = 0;
  const int b_first = start + w * 32;
  // The first step's page ids, then (below) the query / RoPE loads, then this step's K AND V:
  // the page-table round trip and the K / V stream overlap the query and rotary-table loads
  // instead of following the whole RoPE prologue (decode blocks have one or two steps per wave:
  // these dependent round trips, not the bytes, set the kernel time).
  if (b_first < end) pg_cur = bt[b_first >> page_log2];
  if (b_first + 128 < end) pg_next = bt[(b_first + 128) >> page_log2];

  // ROPE with qkv partials (decode blocks, one token): the block's HB query heads, its key and its
  // value summed from the split-K slabs, row-scaled and rounded (common.h qkv_part_finish8: the
  // reduce launch's bits) ONCE per block into LDS - every slab element read once, not once per
  // lane group of every wave; the RoPE below then reads them as it would the bf16 qkv row.
  // Issue order = need order (vmcnt retires in order): row-statistics shards and slab loads, the
  // rotary table, then the first step's K / V - so the fold's and the RoPE's waits leave the K / V
  // stream in flight, and its round trip overlaps theirs instead of following the fold's barrier.
  constexpr int CK = D / 8;  // 8-column chunks per head
  constexpr int NFOLD = (HB + 2) * CK;
  constexpr int NI = (NFOLD + 255) / 256;  // fold items per thread (256 threads)
  __shared__ u16x8 s_fold[NFOLD];
  constexpr bool from_part = ROPE && FOLD;
  int fcol[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int fi = min(tid + 256 * j, NFOLD - 1);  // (threads past the items fetch the last one again, unused)
    fcol[j] = (fi / CK < HB ? (hbase + fi / CK) * D : fi / CK == HB ? (nh + g) * D : (nh + nkv + g) * D) +
              (fi % CK) * 8;
  }
  unsigned long long ssv = 0;
  QkvPart8 ff[NI];
  if constexpr (from_part) {
    ssv = qkv_part_ss_load(rf.qp, tok0);
#pragma unroll
    for (int j = 0; j < NI; ++j) qkv_part_fetch8(rf.qp, tok0, fcol[j], ff[j]);
  }
  u16x8 qf[KD], kr[KD];
  u16x8 vn = (u16x8)(0);
  if constexpr (!from_part) {
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
      qf[kd] = row_ok ? *reinterpret_cast<const u16x8*>(q + (int64_t)(tok0 + my_t) * q_stride + (int64_t)my_h * D +
                                                        kd * 32 + qd * 8)
                      : (u16x8)(0);
    if constexpr (ROPE) {  // the new token's key and value from the bf16 qkv row
      const bf16_t* qrow = q + (int64_t)tok0 * q_stride;
#pragma unroll
      for (int kd = 0; kd < KD; ++kd) kr[kd] = *reinterpret_cast<const u16x8*>(qrow + (nh + g) * D + kd * 32 + qd * 8);
      vn = *reinterpret_cast<const u16x8*>(qrow + (nh + nkv + g) * D + ((lane * 8) % D));
    }
  }
  constexpr int HK = KD / 2, HALF = D / 2;
  f32x4 cs[ROPE ? HK : 1][2], sn[ROPE ? HK : 1][2];
  int64_t kv_slot = -1;
  if constexpr (ROPE) {
    kv_slot = rf.slots[tok0];
    const int64_t ps_ = rf.pos[tok0];
#pragma unroll
    for (int h = 0; h < HK; ++h) {
      const int64_t ci = ps_ * HALF + h * 32 + qd * 8;
      cs[h][0] = *reinterpret_cast<const f32x4*>(rf.cos_t + ci);
      cs[h][1] = *reinterpret_cast<const f32x4*>(rf.cos_t + ci + 4);
      sn[h][0] = *reinterpret_cast<const f32x4*>(rf.sin_t + ci);
      sn[h][1] = *reinterpret_cast<const f32x4*>(rf.sin_t + ci + 4);
    }
  }

  if (b_first < end) {
    load_k(b_first, pg_cur, ka);
    load_v(b_first, pg_cur, vr);
  }

  if constexpr (from_part) {
    const float qrs = qkv_part_ss_scale(rf.qp, ssv);
#pragma unroll
    for (int j = 0; j < NI; ++j)
      if (tid + 256 * j < NFOLD) s_fold[tid + 256 * j] = qkv_part_finish8(rf.qp, tok0, fcol[j], ff[j], qrs);
    lds_wait_barrier();  // (lgkmcnt only: the K / V loads stay in flight)
#pragma unroll
    for (int kd = 0; kd < KD; ++kd) qf[kd] = row_ok ? s_fold[(my_h - hbase) * CK + kd * 4 + qd] : (u16x8)(0);
  }

  int tnew = -1;
  float qk_new = 0.f;
  if constexpr (ROPE) {
    if constexpr (from_part) {
#pragma unroll
      for (int kd = 0; kd < KD; ++kd) kr[kd] = s_fold[HB * CK + kd * 4 + qd];
      vn = s_fold[(HB + 1) * CK + ((lane * 8) % D) / 8];
    }
    auto rot = [&](const u16x8 (&a)[KD], u16x8 (&r)[KD]) {
#pragma unroll
      for (int kd = 0; kd < KD; ++kd) {
        const int h = kd % HK;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float c_ = cs[h][j >> 2][j & 3], s_ = sn[h][j >> 2][j & 3];
          const float x = bf2f(a[kd][j]), y = bf2f(a[kd ^ HK][j]);
          r[kd][j] = kd < HK ? f2bf(x * c_ - y * s_) : f2bf(x * c_ + y * s_);
        }
      }
    };
    u16x8 qr[KD], kn[KD];
    rot(qf, qr);
    rot(kr, kn);
#pragma unroll
    for (int kd = 0; kd < KD; ++kd) qf[kd] = row_ok ? qr[kd] : (u16x8)(0);
    float part = 0.f;
#pragma unroll
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll
      for (int j = 0; j < 8; ++j) part += bf2f(qf[kd][j]) * bf2f(kn[kd][j]);
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    qk_new = part;
    tnew = blk_ctx - 1;
    const int64_t slot = kv_slot;
    if (w == 0 && tnew >= start && tnew < end && slot >= 0 && hbase % (nh / nkv) == 0) {
      const int64_t dst = (slot >> page_log2) * page_stride + head_off + (slot & (page_size - 1)) * D;
      if (c == 0) {
#pragma unroll
        for (int kd = 0; kd < KD; ++kd) *reinterpret_cast<u16x8*>(rf.kw + dst + kd * 32 + qd * 8) = kn[kd];
      }
      if (lane * 8 < D) *reinterpret_cast<u16x8*>(rf.vw + dst + lane * 8) = vn;
    }
  }

  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x4)(0.f);
  float m = -INFINITY, l = 0.f;
  bf16_t* vt = s_vt[w];

  // Software-pipelined walk over this wave's 32-token steps (b0 = start + 32 w + 128 i): the K
  // fragments of step i+1 (and the page id of step i+2) are loaded while step i computes, so a
  // step exposes one memory round trip (its V) instead of three dependent ones (page id -> K -> V).
  // At decode sizes every wave has one or two steps: the chain, not the bytes, set the time
  // (Llama-3-70B, 64 sessions: 16.9 us per layer for 37 MB of K/V).
  // one 32-token step over K / V fragments already in registers
  auto step = [&](int b0, const u16x8 (&kr)[2][KD], const u16x8 (&vr)[NV]) {
    // ---- S^T = K . Q^T for tokens b0 .. b0+31 (two 16-token subtiles) ----
    f32x4 st[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      st[sub] = (f32x4)(0.f);
#pragma unroll
      for (int kd = 0; kd < KD; ++kd) st[sub] = mfma_bf16(kr[sub][kd], qf[kd], st[sub]);
    }
    // ---- V tile -> LDS transposed [d][tok] (this wave only; in-order LDS needs no barrier) ----
    // tokens vary fastest across lanes: each half-wave's transposed stores are 32 consecutive
    // bf16 of one d row (token-major lanes would put 16 lanes on 4 banks, sub-dword)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int ci = i * 64 + lane;
      const int tk = ci % 32, d0 = (ci / 32) * 8;
      u16x8 vv = vr[i];
      if (b0 + tk >= end) vv = (u16x8)(0);
#pragma unroll
      for (int e = 0; e < 8; ++e) vt[(d0 + e) * VT_PITCH + tk] = vv[e];
    }
    if constexpr (ROPE) {  // the new token: its score and its V column come from registers
      const int rel = tnew - b0;
      if (rel >= 0 && rel < 32) {
        if (lane * 8 < D) {
#pragma unroll
          for (int e = 0; e < 8; ++e) vt[(lane * 8 + e) * VT_PITCH + rel] = vn[e];
        }
        if (qd == ((rel & 15) >> 2)) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (r == (rel & 3)) {
              if (rel < 16) st[0][r] = qk_new;
              else st[1][r] = qk_new;
            }
        }
      }
    }
    // ---- online softmax for row c over this lane's 8 tokens {4qd + r, 16 + 4qd + r} ----
    float s8[8];
    float lm = -INFINITY;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tk = b0 + sub * 16 + qd * 4 + r;
        const float v = (tk < my_ctx && tk < end) ? st[sub][r] * scale_log2 : -INFINITY;
        s8[sub * 4 + r] = v;
        lm = fmaxf(lm, v);
      }
    lm = fmaxf(lm, __shfl_xor(lm, 16, 64));
    lm = fmaxf(lm, __shfl_xor(lm, 32, 64));
    const float m_new = fmaxf(m, lm);
    const float alpha = (m_new == -INFINITY) ? 1.f : exp2f(m - m_new);
    u16x8 pa;
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float pv = (m_new == -INFINITY) ? 0.f : exp2f(s8[j] - m_new);
      const bf16_t pb = f2bf(pv);
      pa[j] = pb;
      ps += bf2f(pb);  // l accumulates the rounded p that the MFMA uses
    }
    l = l * alpha + ps;
    m = m_new;
    // O rows are 4qd + r: fetch those rows' alpha from lanes 4qd + r (row == lane & 15)
    float ar[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ar[r] = __shfl(alpha, qd * 4 + r, 64);
    // ---- O += P . V ----
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const bf16_t* vrow = vt + (dt * 16 + c) * VT_PITCH;
      const u16x4 lo = *reinterpret_cast<const u16x4*>(vrow + qd * 4);
      const u16x4 hi = *reinterpret_cast<const u16x4*>(vrow + 16 + qd * 4);
      const u16x8 vfrag = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= ar[r];
      o[dt] = mfma_bf16(pa, vfrag, o[dt]);
    }
  };
  for (int b0 = b_first; b0 < end; b0 += 256) {
    const bool more1 = b0 + 128 < end;
    if (b0 != b_first) load_v(b0, pg_cur, vr);
    int64_t pg2 = 0;
    if (more1) {
      load_k(b0 + 128, pg_next, kb);
      if (b0 + 256 < end) pg2 = bt[(b0 + 256) >> page_log2];
    }
    step(b0, ka, vr);
    if (!more1) break;
    const bool more2 = b0 + 256 < end;
    load_v(b0 + 128, pg_next, vr);
    int64_t pg3 = 0;
    if (more2) {
      load_k(b0 + 256, pg2, ka);
      if (b0 + 384 < end) pg3 = bt[(b0 + 384) >> page_log2];
    }
    step(b0 + 128, kb, vr);
    pg_cur = pg2;
    pg_next = pg3;
  }
  // row sums of l over the 4 lanes of each row
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (lane < 16) {
    s_m[w][lane] = m;
    s_l[w][lane] = l;
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_o[w][qd * 4 + r][dt * 16 + c] = o[dt][r];
  __syncthreads();
  // ---- merge the 4 waves; thread -> (row, d) ----
  for (int i = tid; i < 16 * D; i += 256) {
    const int row = i / D, d = i - row * D;
    const int t = row / HB, h = hbase + row % HB;
    if (t >= ntok) continue;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, s_m[ww][row]);
    float num = 0.f, den = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        const float f = exp2f(s_m[ww][row] - M);
        num += f * s_o[ww][row][d];
        den += f * s_l[ww][row];
      }
    }
    const int tok = tok0 + t;
    if (NP == 1) {
      const float v = den > 0.f ? num / den : 0.f;
      const int64_t col = (int64_t)h * D + d;
      if (rf.mx_ax != nullptr) {
        // MX block of (row, col): the 32 dims of this row with the same bit 4 and bits 6+ of col -
        // lanes l ^ {1, 2, 4, 8, 32} of this wave (a wave holds 64 consecutive dims of one row, so
        // the ``continue`` above is wave-uniform)
        const float vb = bf2f(f2bf(v));
        float a = fabsf(vb);
        a = fmaxf(a, __shfl_xor(a, 1, 64));
        a = fmaxf(a, __shfl_xor(a, 2, 64));
        a = fmaxf(a, __shfl_xor(a, 4, 64));
        a = fmaxf(a, __shfl_xor(a, 8, 64));
        a = fmaxf(a, __shfl_xor(a, 32, 64));
        const int e = mx_e8m0(a);
        const float qv = fminf(fmaxf(vb * mx_inv_scale(e), -448.f), 448.f);
        rf.mx_ax[mx_ax_off(tok, (int)col, packed_mt)] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(qv, 0.f, 0, false) & 255);
        if ((col & 0x2f) == 0) rf.mx_as[mx_as_off(tok, (int)col)] = (uint8_t)e;
        continue;
      }
      out[packed_mt > 0 ? apk_off(tok, (int)col, packed_mt) : (int64_t)tok * nh * D + col] = f2bf(v);
    } else {
      const int64_t hp = ((int64_t)tok * nh + h) * NP + p;
      part_o[hp * D + d] = num;
      if (d == 0) {
        part_ml[hp * 2] = M;
        part_ml[hp * 2 + 1] = den;
      }
    }
  }
}


// Grouped prefill form: a workgroup owns up to NWG (8) query blocks of ONE sequence (one per wave;
// superblock table sb_first / sb_n) and streams each 32-token context step ONCE into LDS for
// all of them - K as a [32][D] tile read back as MFMA A fragments, V transposed as above - so a
// long prompt reads its K/V 4x less often than with one block per workgroup (the one-block
// kernel re-streams the whole causal context for every 16 query rows: 2K-token MHA prefill was
// K/V-bandwidth-bound at ~94 TFLOP/s).  Every wave runs every step (barriers); a wave's rows
// only see tokens < their own ctx, and each wave finishes its own rows (no cross-wave merge).
template <int D, int HB, int NWG>
__global__ __launch_bounds__(NWG * 64) void attn_mfma_grp_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int bt_stride, const int32_t* __restrict__ q_seq,
    const int32_t* __restrict__ q_ctx, const int32_t* __restrict__ qb_tok0, const int32_t* __restrict__ qb_ntok,
    const int32_t* __restrict__ sb_first, const int32_t* __restrict__ sb_n, bf16_t* __restrict__ out,
    float* __restrict__ part_o, float* __restrict__ part_ml, int nkv, int nh, int page_log2, int PS, int NP,
    float scale_log2, int packed_mt) {
  constexpr int KD = D / 32;
  constexpr int DT = D / 16;
  constexpr int KP = D + 8;  // K tile row pitch (bf16): rows 272 B apart stagger the banks
  __shared__ __attribute__((aligned(16))) bf16_t s_k[32 * KP];
  __shared__ __attribute__((aligned(16))) bf16_t s_vt[D * VT_PITCH];

  const int p = blockIdx.z;
  const int hbase = blockIdx.y * HB;
  const int g = hbase / (nh / nkv);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, qd = lane >> 4;
  const int b_first = sb_first[blockIdx.x], nblk = sb_n[blockIdx.x];
  const bool wave_ok = w < nblk;
  const int b = b_first + (wave_ok ? w : 0);
  const int tok0 = qb_tok0[b], ntok = qb_ntok[b];
  const int32_t* bt = block_tables + (int64_t)q_seq[tok0] * bt_stride;
  const int page_size = 1 << page_log2;
  const int64_t page_stride = (int64_t)nkv * page_size * D;
  const int64_t head_off = (int64_t)g * page_size * D;

  const int my_t = c / HB, my_h = hbase + c % HB;
  const bool row_ok = wave_ok && my_t < ntok;
  const int my_ctx = row_ok ? q_ctx[tok0 + my_t] : 0;
  int grp_ctx = 0;  // the context the workgroup streams: the largest ctx of any of its tokens
  for (int bb = b_first; bb < b_first + nblk; ++bb)
    for (int i = 0; i < qb_ntok[bb]; ++i) grp_ctx = max(grp_ctx, q_ctx[qb_tok0[bb] + i]);
  const int start = p * PS, end = min(start + PS, grp_ctx);

  u16x8 qf[KD];
#pragma unroll
  for (int kd = 0; kd < KD; ++kd) {
    if (row_ok) qf[kd] = *reinterpret_cast<const u16x8*>(q + (int64_t)(tok0 + my_t) * q_stride + (int64_t)my_h * D +
                                                         kd * 32 + qd * 8);
    else qf[kd] = (u16x8)(0);
  }
  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x4)(0.f);
  float m = -INFINITY, l = 0.f;

  // the step's K and V (32 tokens, one page: b0 % 32 == 0 and pages hold 32k tokens) are
  // fetched into registers one step ahead, so the global loads of step i+1 are in flight while
  // step i computes out of LDS
  constexpr int NCH = 32 * D / 8;                           // 16-B chunks per tile
  constexpr int CPT = (NCH + NWG * 64 - 1) / (NWG * 64);  // per thread
  u16x8 kreg[CPT], vreg[CPT];
  auto fetch = [&](int s0) {
    const int64_t pg = bt[s0 >> page_log2];
    const bf16_t* kpage = kc + pg * page_stride + head_off + (int64_t)(s0 & (page_size - 1)) * D;
    const bf16_t* vpage = vc + pg * page_stride + head_off + (int64_t)(s0 & (page_size - 1)) * D;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int i = tid + NWG * 64 * j;
      if (NCH % (NWG * 64) != 0 && i >= NCH) break;
      const int tk = i / (D / 8), d0 = (i % (D / 8)) * 8;
      kreg[j] = *reinterpret_cast<const u16x8*>(kpage + (int64_t)tk * D + d0);
      // V: tokens vary fastest across lanes, so the transposed LDS writes below are 32
      // consecutive bf16 of one d row per half-wave (no bank conflicts; token-major lanes put
      // 16 lanes on 4 banks)
      const int tv = i % 32, dv = (i / 32) * 8;
      vreg[j] = *reinterpret_cast<const u16x8*>(vpage + (int64_t)tv * D + dv);
    }
  };
  if (start < end) fetch(start);
  for (int b0 = start; b0 < end; b0 += 32) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int i = tid + NWG * 64 * j;
      if (NCH % (NWG * 64) != 0 && i >= NCH) break;
      const int tk = i / (D / 8), d0 = (i % (D / 8)) * 8;
      const bool past = b0 + tk >= end;  // past the context: stale cache bytes never meet a p = 0
      *reinterpret_cast<u16x8*>(s_k + tk * KP + d0) = past ? (u16x8)(0) : kreg[j];
      const int tv = i % 32, dv = (i / 32) * 8;
      const bool vpast = b0 + tv >= end;
#pragma unroll
      for (int e = 0; e < 8; ++e) s_vt[(dv + e) * VT_PITCH + tv] = vpast ? (bf16_t)0 : vreg[j][e];
    }
    __syncthreads();
    if (b0 + 32 < end) fetch(b0 + 32);
    if (wave_ok) {
      f32x4 st[2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        st[sub] = (f32x4)(0.f);
#pragma unroll
        for (int kd = 0; kd < KD; ++kd) {
          const u16x8 kf = *reinterpret_cast<const u16x8*>(s_k + (sub * 16 + c) * KP + kd * 32 + qd * 8);
          st[sub] = mfma_bf16(kf, qf[kd], st[sub]);
        }
      }
      float s8[8];
      float lm = -INFINITY;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int tk = b0 + sub * 16 + qd * 4 + r;
          const float v = (tk < my_ctx && tk < end) ? st[sub][r] * scale_log2 : -INFINITY;
          s8[sub * 4 + r] = v;
          lm = fmaxf(lm, v);
        }
      lm = fmaxf(lm, __shfl_xor(lm, 16, 64));
      lm = fmaxf(lm, __shfl_xor(lm, 32, 64));
      const float m_new = fmaxf(m, lm);
      const float alpha = (m_new == -INFINITY) ? 1.f : exp2f(m - m_new);
      u16x8 pa;
      float ps = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pv = (m_new == -INFINITY) ? 0.f : exp2f(s8[j] - m_new);
        const bf16_t pb = f2bf(pv);
        pa[j] = pb;
        ps += bf2f(pb);
      }
      l = l * alpha + ps;
      m = m_new;
      float ar[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) ar[r] = __shfl(alpha, qd * 4 + r, 64);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const bf16_t* vrow = s_vt + (dt * 16 + c) * VT_PITCH;
        const u16x4 lo = *reinterpret_cast<const u16x4*>(vrow + qd * 4);
        const u16x4 hi = *reinterpret_cast<const u16x4*>(vrow + 16 + qd * 4);
        const u16x8 vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dt][r] *= ar[r];
        o[dt] = mfma_bf16(pa, vb, o[dt]);
      }
    }
    __syncthreads();  // the next step overwrites the tiles
  }
  if (!wave_ok) return;
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  // this lane holds O rows 4 qd + r (columns dt * 16 + c); row rr's m / l live in lane rr
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = qd * 4 + r;
    const float lr = __shfl(l, rr, 64), mr = __shfl(m, rr, 64);
    const int t = rr / HB, h = hbase + rr % HB;
    if (t >= ntok) continue;
    const int tok = tok0 + t;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d = dt * 16 + c;
      if (NP == 1) {
        const float v = lr > 0.f ? o[dt][r] / lr : 0.f;
        const int64_t col = (int64_t)h * D + d;
        out[packed_mt > 0 ? apk_off(tok, (int)col, packed_mt) : (int64_t)tok * nh * D + col] = f2bf(v);
      } else {
        const int64_t hp = ((int64_t)tok * nh + h) * NP + p;
        part_o[hp * D + d] = o[dt][r];
        if (d == 0) {
          part_ml[hp * 2] = mr;
          part_ml[hp * 2 + 1] = lr;
        }
      }
    }
  }
}

template <int D, int HB>
static void launch_attn_mfma(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt,
                             int bt_stride, const int32_t* q_seq, const int32_t* q_ctx, const int32_t* qb_tok0,
                             const int32_t* qb_ntok, int NB, void* out, float* ws_o, float* ws_ml, int nkv, int nh,
                             int page_log2, int PS, int NP, float scale_log2, int packed_mt, const RopeFuseM& rf,
                             const int32_t* sb_first, const int32_t* sb_n, int NSB, hipStream_t stream) {
  if (sb_first != nullptr && NSB > 0 && rf.pos == nullptr) {
    hipLaunchKernelGGL((attn_mfma_grp_kernel<D, HB, 8>), dim3(NSB, nh / HB, NP), dim3(512), 0, stream, (const bf16_t*)q,
                       q_stride, (const bf16_t*)kc, (const bf16_t*)vc, bt, bt_stride, q_seq, q_ctx, qb_tok0, qb_ntok,
                       sb_first, sb_n, (bf16_t*)out, ws_o, ws_ml, nkv, nh, page_log2, PS, NP, scale_log2, packed_mt);
    return;
  }
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(NB, nh / HB, NP), dim3(256), 0, stream, (const bf16_t*)q, q_stride,
                       (const bf16_t*)kc, (const bf16_t*)vc, bt, bt_stride, q_seq, q_ctx, qb_tok0, qb_ntok,
                       (bf16_t*)out, ws_o, ws_ml, nkv, nh, page_log2, PS, NP, scale_log2, packed_mt, rf);
  };
  if (rf.pos && rf.qp.part) go(attn_mfma_kernel<D, HB, true, true>);
  else if (rf.pos) go(attn_mfma_kernel<D, HB, true, false>);
  else go(attn_mfma_kernel<D, HB, false, false>);
}

__global__ void paged_attn_reduce_kernel(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                                         bf16_t* __restrict__ out, int NP, int D, int nh, int packed_mt);

}  // namespace mp

// Query blocks: qb_tok0[i] = first flat token of block i, qb_ntok[i] = its token count
// (<= 16 / heads_per_block, all from one sequence).  heads_per_block = min(nh / nkv, 16).
// Superblocks (optional, prefill): sb_first[j] / sb_n[j] = runs of <= 8 consecutive query blocks
// of one sequence, one workgroup each (attn_mfma_grp_kernel).
extern "C" int mp_attention_mfma(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt,
                                 int bt_stride, const int32_t* q_seq, const int32_t* q_ctx, const int32_t* qb_tok0,
                                 const int32_t* qb_ntok, int NB, void* out, float* workspace, int T, int nh, int nkv,
                                 int D, int page_size, int PS, int NP, float scale, int packed_mt,
                                 const int64_t* rope_pos, const float* cos_t, const float* sin_t,
                                 const int64_t* slots, const int32_t* sb_first, const int32_t* sb_n, int NSB,
                                 const void* qkv_part_v, void* mx_ax, void* mx_as, hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  RopeFuseM rf{rope_pos, cos_t, sin_t, slots, (bf16_t*)const_cast<void*>(kc), (bf16_t*)const_cast<void*>(vc),
               QkvPart{nullptr, 0, 0, 0, nullptr, 0.f, 0.f}};
  const QkvPart* qkv_part = static_cast<const QkvPart*>(qkv_part_v);  // layout mirrored by bindings.cpp
  if (qkv_part != nullptr && qkv_part->part != nullptr) {
    if (rope_pos == nullptr || qkv_part->S < 1) return -4;  // partials only on the fused RoPE decode path
    rf.qp = *qkv_part;
  }
  if (mx_ax != nullptr) {  // MX output: the fused RoPE decode path, one part, packed rows, 128-dim heads
    if (rope_pos == nullptr || NP != 1 || packed_mt <= 0 || D != 128 || mx_as == nullptr) return -7;
    rf.mx_ax = (uint8_t*)mx_ax;
    rf.mx_as = (uint8_t*)mx_as;
  }
  if (NB == 0 || T == 0) return 0;
  if (nh % nkv != 0 || PS % 128 != 0 || NP < 1 || page_size % 32 != 0) return -1;
  int page_log2 = 0;
  while ((1 << page_log2) < page_size) ++page_log2;
  if ((1 << page_log2) != page_size) return -2;
  const int nrep = nh / nkv;
  // the whole GQA group of a kv head in one workgroup's MFMA rows (spreading a group's heads over
  // several workgroups that re-read the same K / V measured 1.6-2.7x slower, profiles/r4k)
  const int hb = nrep >= 16 ? 16 : nrep;
  if (nrep % hb) return -3;
  const float scale_log2 = scale * 1.4426950408889634f;
  float* ws_o = workspace;
  float* ws_ml = workspace + (int64_t)T * nh * NP * D;
#define MP_AM_CASE(DD, HH)                                                                                      \
  if (D == DD && hb == HH) {                                                                                    \
    launch_attn_mfma<DD, HH>(q, q_stride, kc, vc, bt, bt_stride, q_seq, q_ctx, qb_tok0, qb_ntok, NB, out, ws_o,  \
                             ws_ml, nkv, nh, page_log2, PS, NP, scale_log2, packed_mt, rf, sb_first, sb_n, NSB, \
                             stream);                                                                           \
    goto launched;                                                                                              \
  }
  MP_AM_CASE(128, 1)
  MP_AM_CASE(128, 2)
  MP_AM_CASE(128, 4)
  MP_AM_CASE(128, 8)
  MP_AM_CASE(128, 16)
  MP_AM_CASE(64, 1)
  MP_AM_CASE(64, 2)
  MP_AM_CASE(64, 4)
  MP_AM_CASE(64, 8)
  MP_AM_CASE(64, 16)
#undef MP_AM_CASE
  return -4;
launched:
  if (NP > 1)
    hipLaunchKernelGGL(paged_attn_reduce_kernel, dim3(T * nh), dim3(D), 0, stream, ws_o, ws_ml, (bf16_t*)out, NP, D,
                       nh, packed_mt);
  return (int)hipGetLastError();
}
