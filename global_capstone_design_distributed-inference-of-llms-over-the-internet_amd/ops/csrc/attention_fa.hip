// Causal prefill attention over the paged KV cache on gfx950, FA2-style with 32x32x16 MFMA
// (survey K7 "attn_prefill: causal, MFMA 32x32x16 bf16 QK^T and PV, LDS tiling").
//
// The reference computes prefill attention as matmul -> fp32 softmax -> matmul over the whole
// [heads, T, P+T] score tensor, and without a causal mask (petals/llama/block.py:134-141,
// SURVEY §7.2).  Here one workgroup of NW waves owns 32 x NW query ROWS of one kv head and
// one sequence (row = token-major x the GQA group's HB heads: row r is token tok0 + r / HB,
// head hbase + r % HB), and streams the causal context in 64-token steps:
//
//   * K and V tiles [64 tok][128 d] are staged once per step for all NW waves through a
//     double-buffered LDS image (256-B rows, 16-B chunks XOR-swizzled by the row so both the
//     row reads of K and the transposed reads of V are bank-conflict-free); the next step's
//     tiles are fetched into registers while the current one computes (one barrier per step).
//   * S^T = K . Q^T per wave: 2 x (D/16) v_mfma_f32_32x32x16_bf16 (A = K rows from LDS with
//     ds_read_b128, B = Q^T fragments held in registers for the whole kernel).  The
//     accumulator's COLUMN is the query row, so each lane owns one row and 16 of its
//     scores per 32-token subtile: the online softmax (exp2 domain, causal + context mask)
//     is lane-local plus one xor-32 shuffle for the row maximum.
//   * O^T += V^T . P^T: the exponentiated scores are the B operand straight from the S^T
//     accumulators (no LDS round trip, permuted k order), and V^T comes from the row-major
//     V tile through ds_read_b64_tr_b16, the hardware transpose read: 16 MFMAs per step.
//     O^T's column is the query row too, so the softmax rescale is a per-lane scalar.
//   * causal skipping: a wave stops computing at its own rows' context (the diagonal steps
//     of the earlier waves), workgroups are launched longest-context first.
// Splits of the context (NP > 1) write (m, l, O) partials reduced by paged_attn_reduce_kernel.
#include "common.h"

namespace mp {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_fa;
typedef short s16x4_fa __attribute__((ext_vector_type(4)));
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_fa;

__device__ __forceinline__ f32x16 mfma32x16(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_fa, a), __builtin_bit_cast(bf16x8_fa, b), c,
                                                 0, 0, 0);
}

// LDS image of a [rows][128 bf16] tile (16-B chunks ch = 0..15): 8-row x 32-column subtiles of
// 512 B, the chunk's 4 low bits XOR-swizzled by the row (guide T10 image (a)).  Row reads of
// the 32x32x16 A operand (ds_read_b128) and transposed 4-row reads of V (ds_read_b64_tr_b16) are
// both bank-conflict-free on it, and within a lane every read of a step differs from one of two
// base addresses by an immediate offset (no per-read address arithmetic).
__device__ __forceinline__ int fa_off(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

__device__ __forceinline__ u16x4 tr16(const unsigned char* p) {
  const s16x4_fa v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_fa*)(const_cast<unsigned char*>(p)));
  return __builtin_bit_cast(u16x4, v);
}

// two fp32 -> packed bf16 pair (v_cvt_pk_bf16_f32)
typedef __attribute__((ext_vector_type(2))) float f32x2_fa;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_fa;
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const bf16x2_fa v = __builtin_convertvector((f32x2_fa){a, b}, bf16x2_fa);
  return __builtin_bit_cast(unsigned, v);
}

constexpr float FA_RESCALE_THR = 8.f;  // log2 units: P may reach 2^8 before O / l are rescaled (T13)

template <int HB, int NW>
__global__ __launch_bounds__(NW * 64) void attn_fa_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int bt_stride, const int32_t* __restrict__ q_seq,
    const int32_t* __restrict__ q_ctx, const int32_t* __restrict__ fb_tok0, const int32_t* __restrict__ fb_ntok,
    int NBF, bf16_t* __restrict__ out, int64_t out_stride, float* __restrict__ part_o, float* __restrict__ part_ml,
    int nkv, int nh, int page_log2, int PS, int NP, float scale_log2, int pair) {
  constexpr int D = 128;
  constexpr int STEP = 64;
  constexpr int TILE = STEP * D * 2;            // bytes of one K or V tile (16 KiB)
  constexpr int NT = NW * 64;
  constexpr int CPT = (STEP * D / 8) / NT;      // 16-B chunks per thread per tile
  static_assert((STEP * D / 8) % NT == 0, "tile chunks split evenly over the threads");
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 2 * TILE];  // [buf][K | V]

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: the query blocks of one head sit on one XCD (its K / V stay in that L2),
  // longest causal context first inside a head
  // pair (causal balance for small grids): workgroup j of a head runs query block NBF-1-j, then
  // block j - every workgroup streams the same total context (a long block + its short mirror),
  // instead of the longest blocks setting the kernel time on a grid of ~2 workgroups per CU
  const int G = gridDim.x, NHG = nh / HB;
  const int NBP = pair ? (NBF + 1) / 2 : NBF;  // workgroups per head
  int lin = blockIdx.x;
  if ((G & 7) == 0) lin = (lin & 7) * (G >> 3) + (lin >> 3);
  const int hg = lin / NBP;
  const int jb = lin - hg * NBP;
  const int p = blockIdx.y;
  const int hbase = hg * HB;
  const int g = hbase / (nh / nkv);
  const int npass = pair && (NBF - 1 - jb) != jb ? 2 : 1;
  (void)NHG;
  for (int pass = 0; pass < npass; ++pass) {
  const int bx = pair ? (pass == 0 ? NBF - 1 - jb : jb) : NBF - 1 - jb;
  const int tok0 = fb_tok0[bx], ntok = fb_ntok[bx];
  const int32_t* bt = block_tables + (int64_t)q_seq[tok0] * bt_stride;
  const int page_size = 1 << page_log2;
  const int64_t page_stride = (int64_t)nkv * page_size * D;
  const int64_t head_off = (int64_t)g * page_size * D;

  // contexts are non-decreasing along a sequence's tokens: the last token's is the largest
  const int grp_ctx = q_ctx[tok0 + ntok - 1];
  const int wt_first = (32 * w) / HB, wt_last = min((32 * w + 31) / HB, ntok - 1);
  const bool wave_rows = wt_first < ntok;
  const int wave_ctx = wave_rows ? q_ctx[tok0 + wt_last] : 0;
  const int start = p * PS, end = min(start + PS, grp_ctx);
  const int wave_lim0 = wave_rows ? min(q_ctx[tok0 + wt_first], end) : 0;  // smallest limit of its rows

  const int r = lane & 31, hh = lane >> 5;
  const int my_row = 32 * w + r;
  const int my_t = my_row / HB, my_h = hbase + my_row % HB;
  const bool row_ok = my_t < ntok;
  const int my_ctx = row_ok ? q_ctx[tok0 + my_t] : 0;
  const int lim = min(my_ctx, end);

  u16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    qf[s] = row_ok ? *reinterpret_cast<const u16x8*>(q + (int64_t)(tok0 + my_t) * q_stride + (int64_t)my_h * D +
                                                     16 * s + 8 * hh)
                   : (u16x8)(0);
  }
  f32x16 o[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) o[dt] = (f32x16)(0.f);
  float m = -INFINITY, l = 0.f;  // running max (log2 units, scale applied) and sum of row r

  u16x8 kreg[CPT], vreg[CPT];
  auto fetch = [&](int s0) {
    const int64_t pg = bt[s0 >> page_log2];
    const bf16_t* kp = kc + pg * page_stride + head_off + (int64_t)(s0 & (page_size - 1)) * D;
    const bf16_t* vp = vc + pg * page_stride + head_off + (int64_t)(s0 & (page_size - 1)) * D;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = tid + NT * j, row = c >> 4, ch = c & 15;
      kreg[j] = *reinterpret_cast<const u16x8*>(kp + row * D + ch * 8);
      vreg[j] = *reinterpret_cast<const u16x8*>(vp + row * D + ch * 8);
    }
  };
  auto stash = [&](int buf, int s0) {
    unsigned char* kb = smem + buf * 2 * TILE;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = tid + NT * j, row = c >> 4, ch = c & 15;
      const bool past = s0 + row >= end;  // past the context: stale cache bytes never meet a p = 0
      *reinterpret_cast<u16x8*>(kb + fa_off(row, ch)) = past ? (u16x8)(0) : kreg[j];
      *reinterpret_cast<u16x8*>(kb + TILE + fa_off(row, ch)) = past ? (u16x8)(0) : vreg[j];
    }
  };

  // per-lane LDS bases (every read of a step is one of them + an immediate):
  //   K row read (sub, s): row 32 sub + r, chunk 2 s + hh -> kbase[s & 1] + 8192 sub + 512 (s >> 1)
  //   V transposed read (sub, s2, dt, hi): this lane feeds row q of the 4-row block at
  //   32 sub + 16 s2 + 8 hi + 4 hh, chunk 4 dt + 2 (grp & 1) + (tp >> 1), + 8 (tp & 1) bytes
  //   -> vbase[hi] + 8192 sub + 4096 s2 + 512 dt
  const int grp = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int kbase0 = fa_off(r, hh), kbase1 = fa_off(r, 2 + hh);
  const int trc = 2 * (grp & 1) + (tp >> 1);
  const int vbase0 = TILE + fa_off(4 * hh + tq, trc) + 8 * (tp & 1);
  const int vbase1 = TILE + fa_off(8 + 4 * hh + tq, trc) + 8 * (tp & 1);

  if (start < end) {
    fetch(start);
    stash(0, start);
  }
  __syncthreads();
  int it = 0;
  for (int b0 = start; b0 < end; b0 += STEP, ++it) {
    const int cur = it & 1;
    const bool more = b0 + STEP < end;
    if (more) fetch(b0 + STEP);
    if (b0 < wave_ctx) {
      const unsigned char* tb = smem + cur * 2 * TILE;
      // ---- S^T = K . Q^T for the step's 64 tokens: 4 independent accumulation chains
      //      (two 32-token subtiles x two halves of d), summed afterwards ----
      f32x16 sa[2][2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          sa[sub][half] = (f32x16)(0.f);
#pragma unroll
          for (int s = 4 * half; s < 4 * half + 4; ++s) {
            const u16x8 a = *reinterpret_cast<const u16x8*>(tb + ((s & 1) ? kbase1 : kbase0) + 8192 * sub +
                                                            512 * (s >> 1));
            sa[sub][half] = mfma32x16(a, qf[s], sa[sub][half]);
          }
        }
      f32x16 st[2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) st[sub] = sa[sub][0] + sa[sub][1];
      // ---- online softmax of row r over this lane's 32 tokens (raw scores; the scale is
      //      folded into the exponent's FMA) ----
      if (b0 + STEP > wave_lim0) {  // diagonal / last step: causal and context mask
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int tk = b0 + 32 * sub + 4 * hh + (j & 3) + 8 * (j >> 2);
            st[sub][j] = tk < lim ? st[sub][j] : -INFINITY;
          }
      }
      float lm = -INFINITY;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int j = 0; j < 16; ++j) lm = fmaxf(lm, st[sub][j]);
      lm = fmaxf(lm, __shfl_xor(lm, 32, 64)) * scale_log2;
      // rescale O and l only when some row's maximum grew by more than the threshold
      if (!__all(lm <= m + FA_RESCALE_THR)) {
        const float m_new = fmaxf(m, lm);
        const float alpha = m_new == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m - m_new);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) o[dt] *= alpha;
        m = m_new;
      }
      const float mu = m == -INFINITY ? 0.f : m;  // fully masked row so far: every p is 0
      u16x8 pf[2][2];
      float ps = 0.f;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          unsigned pk[4];
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(st[sub][8 * s2 + j], scale_log2, -mu));
            const float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(st[sub][8 * s2 + j + 1], scale_log2, -mu));
            ps += p0 + p1;
            pk[j >> 1] = pk_bf16(p0, p1);
          }
          pf[sub][s2] = __builtin_bit_cast(u16x8, (u32x4_fa){pk[0], pk[1], pk[2], pk[3]});
        }
      l += ps;
      // ---- O^T += V^T . P^T: A = V^T by transposed LDS reads, B = P from registers ----
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int imm = 8192 * sub + 4096 * s2 + 512 * dt;
            const u16x4 lo = tr16(tb + vbase0 + imm);
            const u16x4 hi = tr16(tb + vbase1 + imm);
            const u16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[dt] = mfma32x16(a, pf[sub][s2], o[dt]);
          }
      }
    }
    if (more) stash(cur ^ 1, b0 + STEP);
    __syncthreads();
  }
  // ---- epilogue: lane owns row r; O^T accumulator register j of d-tile dt holds
  //      d = 32 dt + 8 (j >> 2) + 4 hh + (j & 3) ----
  l += __shfl_xor(l, 32, 64);
  if (!row_ok) continue;  // (every step above ended in a barrier: the LDS tiles are free)
  const int tok = tok0 + my_t;
  if (NP == 1) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* orow = out + (int64_t)tok * out_stride + (int64_t)my_h * D;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][4 * gq + e] * inv);
        *reinterpret_cast<u16x4*>(orow + 32 * dt + 8 * gq + 4 * hh) = v;
      }
  } else {
    const int64_t hp = ((int64_t)tok * nh + my_h) * NP + p;
    float* po = part_o + hp * D;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = o[dt][4 * gq + e];
        *reinterpret_cast<f32x4*>(po + 32 * dt + 8 * gq + 4 * hh) = v;
      }
    if (hh == 0) {
      part_ml[hp * 2] = m;
      part_ml[hp * 2 + 1] = l;
    }
  }
  }  // pass
}

__global__ void paged_attn_reduce_kernel(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                                         bf16_t* __restrict__ out, int NP, int D, int nh, int packed_mt);

}  // namespace mp

// Prefill blocks: fb_tok0[i] / fb_ntok[i] = first flat token / token count of block i (<= 32 x NW
// / heads_per_block consecutive tokens of ONE sequence, ops.fa_blocks).  D = 128, page_size a
// multiple of 64, heads_per_block = nh / nkv in {1, 2, 4, 8}; row-major output [T, nh * D].
extern "C" int mp_attention_fa(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt,
                               int bt_stride, const int32_t* q_seq, const int32_t* q_ctx, const int32_t* fb_tok0,
                               const int32_t* fb_ntok, int NBF, void* out, float* workspace, int T, int nh, int nkv,
                               int D, int page_size, int PS, int NP, float scale, int nw, int pair,
                               hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  if (NBF == 0 || T == 0) return 0;
  if (D != 128 || nh % nkv != 0 || PS % 64 != 0 || NP < 1 || page_size % 64 != 0) return -1;
  int page_log2 = 0;
  while ((1 << page_log2) < page_size) ++page_log2;
  if ((1 << page_log2) != page_size) return -2;
  const int hb = nh / nkv;
  pair = pair ? 1 : 0;
  const int nbp = pair ? (NBF + 1) / 2 : NBF;
  const float scale_log2 = scale * 1.4426950408889634f;
  float* ws_o = workspace;
  float* ws_ml = workspace + (int64_t)T * nh * NP * D;
#define MP_FA(HB_, NW_)                                                                                         \
  hipLaunchKernelGGL((attn_fa_kernel<HB_, NW_>), dim3(nbp * (nh / HB_), NP), dim3(NW_ * 64), 0, stream,           \
                     (const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, bt, bt_stride, q_seq, q_ctx, \
                     fb_tok0, fb_ntok, NBF, (bf16_t*)out, (int64_t)nh * D, ws_o, ws_ml, nkv, nh, page_log2, PS, NP,  \
                     scale_log2, pair)
#define MP_FA_NW(HB_) \
  if (nw == 8) MP_FA(HB_, 8); else MP_FA(HB_, 4);
  switch (hb) {
    case 1: MP_FA_NW(1); break;
    case 2: MP_FA_NW(2); break;
    case 4: MP_FA_NW(4); break;
    case 8: MP_FA_NW(8); break;
    default: return -3;
  }
#undef MP_FA_NW
#undef MP_FA
  if (NP > 1)
    hipLaunchKernelGGL(paged_attn_reduce_kernel, dim3(T * nh), dim3(D), 0, stream, ws_o, ws_ml, (bf16_t*)out, NP, D,
                       nh, 0);
  return (int)hipGetLastError();
}
