// Server-side token sampler for gfx950 (survey K13).
//
// Semantics follow the reference's `_sample_token` (reference
// src/rpc_handler.py:327-403), batched over rows with per-row parameters:
//   temperature <= 0           -> argmax of the raw logits
//   repetition penalty          -> every distinct id among the last <= 50 generated ids gets
//                                  logit /= rp**count (logit > 0) or *= rp**count (else);
//                                  if the last 3 ids are equal that id gets rp**3 more
//   softmax(logits / max(T, 1e-5)), top-k mask (0 < k < V), top-p "keep cum <= p, always
//   keep the first", renormalise, draw one id.
// Instead of a Python loop, torch.topk, a full sort and a cumsum, one 1024-thread block per
// row works on an fp32 copy of the row in LDS:
//   * top-k path (0 < k < V, the reference CLI default k = 50): penalty -> max -> softmax
//     normaliser Z -> a lower bound of the k-th largest logit from a histogram of the 1024
//     per-thread maxima -> the (few) candidates above it are collected, ranked by value
//     (index breaks ties, like a stable sort), and top-p / renormalise / the draw run on the
//     <= k sorted candidates only.  Four sweeps over the row, no sort of V, no V atomics.
//   * otherwise (no top-k, or a degenerate row with > 1024 candidates): radix-select on the
//     probabilities (4 x 8-bit passes) for top-k and on probability MASS for top-p, then an
//     inverse-CDF draw with a block scan.  Ties at a threshold value are kept together there.
// The per-row history of the last RECENT generated ids (repetition penalty input) is
// updated in place by the same kernel (``update`` flag), so the serving loop needs no extra
// device ops per token.
#include "common.h"
#include <stdlib.h>

namespace mp {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

typedef unsigned long long u64;
constexpr int SB = 1024;   // threads per block

// Phase timestamps of sample_kernel for the lab driver scripts/sampler_prof.hip (compiled out of
// the package build): thread 0 of block b stores clock64() at mark i into mp_sprof[b * 16 + i].
#ifdef MP_SAMPLE_PROF
__device__ unsigned long long mp_sprof[1024 * 16];
#define MP_PROF(i) \
  if (threadIdx.x == 0 && blockIdx.x < 1024) mp_sprof[blockIdx.x * 16 + (i)] = clock64()
#else
#define MP_PROF(i) ((void)0)
#endif
#ifdef MP_SAMPLE_PROF
#define MP_PROF_CNT(c) (mp_sprof[blockIdx.x * 16 + 15] = (unsigned long long)(c))
#else
#define MP_PROF_CNT(c) ((void)0)
#endif
constexpr int CAND = 1024;  // top-k candidate capacity of the fast path

// order-preserving unsigned key of a float (ascending key == ascending value)
__device__ __forceinline__ unsigned okey(float f) {
  const unsigned b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Append a generated id to a row's left-aligned history of the last `cap` ids.
__device__ __forceinline__ void push_history(int32_t* rec, int32_t* len, int cap, int tok) {
  int n = *len;
  if (n >= cap) {
    for (int j = 0; j + 1 < cap; ++j) rec[j] = rec[j + 1];
    n = cap - 1;
  }
  rec[n] = tok;
  *len = n + 1;
}

// The block appends `tok` to its row's left-aligned history of the last `cap` ids, in parallel:
// thread j < cap holds the old rec[j + 1] (`h_next`, loaded at kernel start), so a full history
// shifts by one store per thread instead of a serial load/store chain in one thread.  Every
// thread of the block calls it with the same tok / n_old.
__device__ __forceinline__ void push_history_block(int32_t* rec, int32_t* len, int cap, int n_old, int tok,
                                                   int h_next) {
  const int tid = threadIdx.x;
  if (n_old >= cap) {
    if (tid + 1 < cap) rec[tid] = h_next;
    else if (tid + 1 == cap) rec[tid] = tok;
  } else if (tid == n_old) {
    rec[tid] = tok;
  }
  if (tid == 0) *len = min(n_old + 1, cap);
}

// Wave reductions / scans: DPP lane moves (common.h), no ds_bpermute round trips.
__device__ __forceinline__ float wave_incl_scan_dpp(float v) {  // inclusive prefix sum over the lanes
  v += dppf<0x111>(v, 0.f);        // row_shr:1
  v += dppf<0x112>(v, 0.f);        // row_shr:2
  v += dppf<0x114>(v, 0.f);        // row_shr:4
  v += dppf<0x118>(v, 0.f);        // row_shr:8: inclusive within each row of 16
  v += dppf<0x142, 0xA>(v, 0.f);   // + the previous row's total (rows 1, 3)
  v += dppf<0x143, 0xC>(v, 0.f);   // + rows 0-1's total (rows 2, 3)
  return v;
}

template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ unsigned dppu(unsigned v) {  // identity 0 for unsigned max
  return dpp_u32<CTRL, ROW_MASK>(0u, v);
}
__device__ __forceinline__ unsigned wave_umax_dpp(unsigned v) {
  v = max(v, dppu<0xB1>(v));
  v = max(v, dppu<0x4E>(v));
  v = max(v, dppu<0x141>(v));
  v = max(v, dppu<0x140>(v));
  v = max(v, dppu<0x142, 0xA>(v));
  v = max(v, dppu<0x143, 0xC>(v));
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// Exact k-th largest (k >= 1) of the keys of the wave's lanes with `act`, by a ballot radix
// over the 32 key bits: uniform ballots and popcounts, no LDS.
__device__ __forceinline__ unsigned wave_kth_largest(unsigned key, bool act, int k) {
  unsigned prefix = 0u;
  for (int b = 31; b >= 0; --b) {
    const unsigned hi = (prefix >> b) | 1u;  // higher bits as decided, bit b = 1
    const int cnt = __popcll(__ballot(act && (key >> b) == hi));
    if (cnt >= k) prefix |= 1u << b;
    else k -= cnt;
  }
  return prefix;
}

// Rank of each active lane's (key desc, index asc) among the wave's active lanes: a ballot radix
// over the key bits, then the low IBITS bits of ~index (the index breaks ties like a stable sort).
template <int IBITS>
__device__ __forceinline__ int wave_rank_desc(unsigned key, unsigned idx, bool act) {
  unsigned long long eq = __ballot(act);  // lanes equal to this one on the bits so far
  int r = 0;
  for (int b = 31; b >= 0; --b) {
    const unsigned long long g = __ballot(act && ((key >> b) & 1u));
    if ((key >> b) & 1u) eq &= g;
    else {
      r += __popcll(eq & g);
      eq &= ~g;
    }
  }
  const unsigned ni = ~idx;
  for (int b = IBITS - 1; b >= 0; --b) {
    const unsigned long long g = __ballot(act && ((ni >> b) & 1u));
    if ((ni >> b) & 1u) eq &= g;
    else {
      r += __popcll(eq & g);
      eq &= ~g;
    }
  }
  return r;
}

// Block max / sum over SB threads: DPP wave reductions, then every lane reads the 16 wave totals
// with four 16-B LDS reads.
__device__ __forceinline__ float sb_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const f32x4* r4 = reinterpret_cast<const f32x4*>(red);
  const f32x4 a = r4[0], b = r4[1], c = r4[2], d = r4[3];
  float t = -INFINITY;
#pragma unroll
  for (int j = 0; j < 4; ++j) t = fmaxf(t, fmaxf(fmaxf(a[j], b[j]), fmaxf(c[j], d[j])));
  return t;
}
__device__ __forceinline__ float sb_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const f32x4* r4 = reinterpret_cast<const f32x4*>(red);
  const f32x4 a = r4[0], b = r4[1], c = r4[2], d = r4[3];
  float t = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) t += (a[j] + b[j]) + (c[j] + d[j]);
  return t;
}

// Exclusive block scan of one float per thread (blockDim == SB).
__device__ __forceinline__ float block_excl_scan(float v, float* red, float* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float inc = wave_incl_scan_dpp(v);
  __syncthreads();
  if (lane == 63) red[w] = inc;
  __syncthreads();
  if (w == 0) {  // wave 0 scans the SB / 64 wave totals (one row of 16 lanes: DPP row shifts)
    constexpr int NW = SB / 64;
    const float t = lane < NW ? red[lane] : 0.f;
    const float s = wave_incl_scan_dpp(t);
    if (lane < NW) red[lane] = s - t;
    if (lane == NW - 1) red[NW] = s;
  }
  __syncthreads();
  *total = red[SB / 64];
  return red[w] + inc - v;
}

// LDS = the working row lives in LDS (V <= 34K): a compile-time choice, so every access to it is
// a ds_* op (a run-time choice left `x` a generic pointer: flat loads / stores on every sweep)
template <bool LDS>
__global__ __launch_bounds__(SB) void sample_kernel(const bf16_t* __restrict__ logits, int64_t stride, int V,
                                                    const float* __restrict__ temps, const float* __restrict__ top_ps,
                                                    const int32_t* __restrict__ top_ks,
                                                    const float* __restrict__ rep_pens,
                                                    int32_t* __restrict__ recent, int recent_stride,
                                                    int32_t* __restrict__ recent_len,
                                                    const int64_t* __restrict__ seeds, float* __restrict__ ws,
                                                    int64_t* __restrict__ out, int use_lds, int update,
                                                    int only_unset) {
  __shared__ __attribute__((aligned(16))) float red[SB / 64 + 4];
  __shared__ unsigned hist[256];
  __shared__ float mass[256];
  __shared__ unsigned s_u[4];  // scratch: selected bin, fallback flag, remaining rank
  __shared__ int s_i[2];
  extern __shared__ __attribute__((aligned(16))) float s_row[];
  const int row = blockIdx.x, tid = threadIdx.x;
  if (only_unset && out[row] >= 0) return;  // the split sampler already drew this row
  MP_PROF(0);
  const bf16_t* lrow = logits + (int64_t)row * stride;
  // the working row lives in LDS when it fits (V <= 38K: every pass is an LDS sweep),
  // otherwise in the global workspace (L2-resident)
  (void)use_lds;
  float* x = LDS ? s_row : ws + (int64_t)row * V;
  const float temp = temps[row];
  // the row's history, loaded now so its round trip overlaps the row copy: rec[tid] (penalty)
  // and rec[tid + 1] (the shift of a full history on append)
  int32_t* hrow = recent + (int64_t)row * recent_stride;
  const int n_hist = recent_len[row];
  const int h_mine = tid < recent_stride ? hrow[tid] : 0;
  const int h_next = tid + 1 < recent_stride ? hrow[tid + 1] : 0;

  // ---- fp32 copy + max (max is needed by both the greedy and the sampling path) ----
  // 16-B loads, 4 in flight per thread before any use (one latency, not V/1024 of them)
  float mx = -INFINITY;
  int mi = 0x7fffffff;
  const bool vec = ((V & 7) == 0) && ((stride & 7) == 0);
  if (vec) {
    for (int base = tid * 8; base < V; base += SB * 8 * 4) {
      u16x8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i0 = base + u * SB * 8;
        v[u] = i0 < V ? *reinterpret_cast<const u16x8*>(lrow + i0) : (u16x8)(0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i0 = base + u * SB * 8;
        if (i0 < V) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float f = bf2f(v[u][j]);
            x[i0 + j] = f;
            if (f > mx) { mx = f; mi = i0 + j; }
          }
        }
      }
    }
  } else {
    for (int i = tid; i < V; i += SB) {
      const float f = bf2f(lrow[i]);
      x[i] = f;
      if (f > mx) { mx = f; mi = i; }
    }
  }
  if (temp <= 0.f) {  // greedy: first maximum of the raw logits
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(mx, o, 64);
      const int oi = __shfl_xor(mi, o, 64);
      if (ov > mx || (ov == mx && oi < mi)) { mx = ov; mi = oi; }
    }
    __shared__ float bv[SB / 64];
    __shared__ int bi[SB / 64];
    if ((tid & 63) == 0) { bv[tid >> 6] = mx; bi[tid >> 6] = mi; }
    __syncthreads();
    if (tid == 0) {
      float b = bv[0];
      int ix = bi[0];
      for (int k = 1; k < SB / 64; ++k)
        if (bv[k] > b || (bv[k] == b && bi[k] < ix)) { b = bv[k]; ix = bi[k]; }
      out[row] = ix == 0x7fffffff ? 0 : ix;
      s_i[1] = ix == 0x7fffffff ? 0 : ix;
    }
    if (update) {
      __syncthreads();
      push_history_block(hrow, recent_len + row, recent_stride, n_hist, s_i[1], h_next);
    }
    return;
  }
  // the history, staged in LDS (each thread scans all of it) under the copy's barrier
  const int nrec = min(n_hist, recent_stride);
  __shared__ int s_rec[SB];
  if (tid < nrec) s_rec[tid] = h_mine;
  __syncthreads();
  MP_PROF(1);

  // ---- repetition penalty (reference src/rpc_handler.py:345-374) ----
  const float rp = rep_pens[row];
  const int* rec = s_rec;
  if (rp != 1.f && nrec > 0) {
    if (tid < nrec) {
      const int tok = rec[tid];
      bool first = true;
      int count = 0;
      for (int j = 0; j < nrec; ++j) {
        if (rec[j] == tok) {
          ++count;
          if (j < tid) first = false;
        }
      }
      if (first && tok >= 0 && tok < V) {
        const float pen = powf(rp, (float)count);
        float v = x[tok];
        v = v > 0.f ? v / pen : v * pen;
        // the last three ids equal: that id gets rp**3 more, applied after the count penalty
        // by the same thread (no second barrier / serial pass)
        if (nrec >= 3 && tok == rec[nrec - 1] && rec[nrec - 2] == tok && rec[nrec - 3] == tok) {
          const float pen3 = rp * rp * rp;
          v = v > 0.f ? v / pen3 : v * pen3;
        }
        x[tok] = v;
      }
    }
    __syncthreads();
  }

  // ---- softmax(x / T): max and normaliser (x keeps the penalised logits) ----
  MP_PROF(2);
  const float inv_t = 1.f / fmaxf(temp, 1e-5f);
  // The sweeps below read the row in the copy's layout when it has one: thread tid owns the
  // 8-float chunks at tid * 8 + u * SB * 8 (two 16-B LDS reads each, unrolled, so a sweep is a
  // few LDS round trips per thread instead of V / SB dependent scalar reads).
  float lm = -INFINITY;
  if (vec) {
#pragma unroll 4
    for (int base = tid * 8; base < V; base += SB * 8) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(x + base), b = *reinterpret_cast<const f32x4*>(x + base + 4);
      lm = fmaxf(lm, fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])), fmaxf(fmaxf(b[0], b[1]), fmaxf(b[2], b[3]))));
    }
  } else {
    for (int i = tid; i < V; i += SB) lm = fmaxf(lm, x[i]);
  }
  // this thread's maximum as an order-preserving key (the top-k bound below; 0 = no element)
  const unsigned tmax = lm > -INFINITY ? okey(lm) : 0u;
  const float m = sb_max(lm, red);
  MP_PROF(3);
  float ls = 0.f;
  if (vec) {
#pragma unroll 4
    for (int base = tid * 8; base < V; base += SB * 8) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(x + base), b = *reinterpret_cast<const f32x4*>(x + base + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) ls += __expf((a[j] - m) * inv_t) + __expf((b[j] - m) * inv_t);
    }
  } else {
    for (int i = tid; i < V; i += SB) ls += __expf((x[i] - m) * inv_t);
  }
  const float inv_s = 1.f / sb_sum(ls, red);
  MP_PROF(4);
  const int k = top_ks[row];
  const float tp = top_ps[row];
  const uint64_t rnd = splitmix64((uint64_t)seeds[row] * 0x9E3779B97F4A7C15ull + (uint64_t)row);
  const float u01 = (float)((double)(rnd >> 11) * (1.0 / 9007199254740992.0));

  if (k > 0 && k < V) {
    // ---- fast top-k.  The k-th largest of the 1024 per-thread maxima, tau, is <= the k-th
    //      largest value (those k maxima are values of the row), so every top-k id has
    //      key >= tau, and few others do.  Selecting among 1024 maxima instead of V keys
    //      avoids the LDS-atomic pile-up on the few bins dense logits fall into. ----
    __shared__ __attribute__((aligned(16))) unsigned h2k[2 * CAND];  // radix bins, then (key, index) candidates
    uint2* c_ki = reinterpret_cast<uint2*>(h2k);
    __shared__ int c_idx[CAND];
    __shared__ float c_p[CAND];
    __shared__ int s_cnt;
    if (tid == 0) { s_cnt = 0; s_u[1] = 0u; }
    unsigned prefix = 0u, msk = 0u;
    int kk = k;
    constexpr int NW = SB / 64, QW = 64 / NW;  // 16 waves x their top 4 maxima = 64 keys
    const bool wave_bound = k <= 64;
    if (wave_bound) {
      // tau = the k-th largest of U, the union of every wave's QW largest thread maxima.  U is a
      // subset of the maxima, so tau <= their k-th largest <= the row's k-th largest value, and
      // it is close to it (the top k maxima rarely crowd into a few waves).  Wave shuffles and
      // two barriers instead of the radix select's ~18 (the exact ranking below makes the result
      // independent of how tight tau is; a loose one only costs candidates)
      const int lane = tid & 63;
      unsigned cur = tmax, mine = 0u;
#pragma unroll
      for (int j = 0; j < QW; ++j) {  // this wave's QW largest maxima, one DPP reduction each
        const unsigned mxk = wave_umax_dpp(cur);
        const unsigned long long hit = __ballot(cur == mxk);
        if (lane == __ffsll((long long)hit) - 1) cur = 0u;  // remove one holder of the maximum
        if (lane == j) mine = mxk;
      }
      if (lane < QW) h2k[(tid >> 6) * QW + lane] = mine;
      __syncthreads();
      if (tid < 64) {  // wave 0: the k-th largest of the 64 keys
        const unsigned t = wave_kth_largest(h2k[tid], true, k);
        if (tid == 0) s_u[0] = t;
      }
      __syncthreads();
      prefix = s_u[0];
      __syncthreads();  // h2k / s_u are reused below
    }
    // else: exact k-th largest of the per-thread maxima: radix select over 1024 keys (11 + 11 +
    // 10 bits), cheap however flat the row is (random-init logits are nearly uniform)
    for (int round = 0; round < (wave_bound ? 0 : 3); ++round) {
      const int shift = round == 0 ? 21 : (round == 1 ? 10 : 0);
      const unsigned nb = round < 2 ? 2048u : 1024u;
      for (int i = tid; i < 2048; i += SB) h2k[i] = 0;
      __syncthreads();
      if (tmax != 0u && (tmax & msk) == prefix) atomicAdd(&h2k[(tmax >> shift) & (nb - 1)], 1u);
      __syncthreads();
      const float own0 = (float)h2k[2 * tid], own1 = (float)h2k[2 * tid + 1];
      float tot;
      const float P = block_excl_scan(own0 + own1, red, &tot);  // keys in bins < 2 tid
      const float ge1 = tot - P - own0, ge0 = tot - P;          // keys in bins >= 2t+1 / >= 2t
      const float kf = (float)kk;
      if (ge1 >= kf && ge1 - own1 < kf) { s_u[0] = 2 * tid + 1; s_u[2] = (unsigned)(kk - (int)(ge1 - own1)); }
      if (ge0 >= kf && ge0 - own0 < kf) { s_u[0] = 2 * tid; s_u[2] = (unsigned)(kk - (int)(ge0 - own0)); }
      if (tid == 0 && tot < kf) s_u[1] = 1u;  // fewer maxima than k (tiny vocab): general path
      __syncthreads();
      if (s_u[1]) break;
      prefix |= s_u[0] << shift;
      msk |= (nb - 1) << shift;
      kk = (int)s_u[2];
      __syncthreads();
    }
    const unsigned tau = prefix;  // a value of the row <= the k-th largest value
    bool fast = s_u[1] == 0u;
    MP_PROF(5);
    if (fast) {
      if (vec) {
        // a thread whose maximum is below tau holds no candidate
#pragma unroll 4
        for (int base = tid * 8; base < (tmax >= tau ? V : 0); base += SB * 8) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(x + base), b = *reinterpret_cast<const f32x4*>(x + base + 4);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const unsigned key = okey(j < 4 ? a[j & 3] : b[j & 3]);
            if (key >= tau) {
              const int pos = atomicAdd(&s_cnt, 1);
              if (pos < CAND) c_ki[pos] = make_uint2(key, (unsigned)(base + j));
            }
          }
        }
      } else {
        for (int i = tid; i < V; i += SB) {
          const unsigned key = okey(x[i]);
          if (key >= tau) {
            const int pos = atomicAdd(&s_cnt, 1);
            if (pos < CAND) c_ki[pos] = make_uint2(key, (unsigned)i);
          }
        }
      }
      __syncthreads();
      fast = s_cnt <= CAND;
      MP_PROF(6);
      if (threadIdx.x == 0 && blockIdx.x < 1024) MP_PROF_CNT(s_cnt);
    }
    if (fast) {
      const int c = s_cnt;
      // rank by (value desc, index asc); rank < k survives top-k
      int rank = CAND, my_idx = 0;
      if (c <= 64 && V <= (1 << 20) && tid < 64) {  // wave 0 holds every candidate: ballot radix ranks
        const uint2 me = tid < c ? c_ki[tid] : make_uint2(0u, 0u);
        const int r = wave_rank_desc<20>(me.x, me.y, tid < c);
        if (tid < c) {
          rank = r;
          my_idx = (int)me.y;
        }
      } else if (tid < c) {
        const uint2 me = c_ki[tid];
        my_idx = (int)me.y;
        rank = 0;
        int j = 0;
        for (; j + 8 <= c; j += 8) {  // 8 broadcast 8-B LDS reads in flight per batch
          uint2 o[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) o[u] = c_ki[j + u];
#pragma unroll
          for (int u = 0; u < 8; ++u) rank += (o[u].x > me.x) || (o[u].x == me.x && o[u].y < me.y);
        }
        for (; j < c; ++j) {
          const uint2 o = c_ki[j];
          rank += (o.x > me.x) || (o.x == me.x && o.y < me.y);
        }
      }
      __syncthreads();
      MP_PROF(7);
      if (rank < k) {  // sorted (descending) survivors: index and FULL-softmax probability
        c_idx[rank] = my_idx;
        c_p[rank] = __expf((x[my_idx] - m) * inv_t) * inv_s;
      }
      __syncthreads();
      MP_PROF(8);
      const int kk = min(k, c);
      const float pv = tid < kk ? c_p[tid] : 0.f;
      float t1;
      const float ex1 = block_excl_scan(pv, red, &t1);
      // top-p (reference): keep sorted prefix with cumulative <= p, always keep the first
      const bool keep = tid < kk && (tid == 0 || !(tp > 0.f && tp < 1.f) || ex1 + pv <= tp);
      const float q = keep ? pv : 0.f;
      float t2;
      const float ex2 = block_excl_scan(q, red, &t2);
      const float uu = u01 * t2;
      if (tid == 0) s_i[1] = c_idx[0];  // rounding fallback: the most likely id
      __syncthreads();
      if (q > 0.f && uu >= ex2 && uu < ex2 + q) s_i[1] = c_idx[tid];
      __syncthreads();
      MP_PROF(9);
      if (tid == 0) out[row] = s_i[1];
      if (update) push_history_block(hrow, recent_len + row, recent_stride, n_hist, s_i[1], h_next);
      MP_PROF(10);
      return;
    }
    // degenerate row (too many candidates at the k-th value): general path below
  }
  // general path works on probabilities
  unsigned maxbits = 0;
  for (int i = tid; i < V; i += SB) {
    const float pv = __expf((x[i] - m) * inv_t) * inv_s;
    x[i] = pv;
    maxbits = max(maxbits, __float_as_uint(pv));
  }
  // block max of bits
  {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxbits = max(maxbits, (unsigned)__shfl_xor((int)maxbits, o, 64));
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = __uint_as_float(maxbits);
    __syncthreads();
    unsigned mb = 0;
    for (int k2 = 0; k2 < SB / 64; ++k2) mb = max(mb, __float_as_uint(red[k2]));
    maxbits = mb;
  }

  // ---- top-k: radix-select the k-th largest probability (bits are order-preserving, p >= 0) ----
  if (k > 0 && k < V) {
    unsigned prefix = 0, msk = 0;
    int kk = k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = tid; i < 256; i += SB) hist[i] = 0;
      __syncthreads();
      for (int i = tid; i < V; i += SB) {
        const unsigned b = __float_as_uint(x[i]);
        if ((b & msk) == prefix) atomicAdd(&hist[(b >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid < 64) {  // wave 0: parallel suffix count over bins 255..0, lane l owns bins 4l..4l+3
        const int l = tid;
        const unsigned h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2], h3 = hist[4 * l + 3];
        const int own = (int)(h0 + h1 + h2 + h3);
        int incl = own;  // inclusive suffix sum over lanes >= l
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int nb = __shfl_down(incl, o, 64);
          if (l + o < 64) incl += nb;
        }
        const unsigned long long hit = __ballot(incl >= kk);
        const int cl = hit ? 63 - __builtin_clzll(hit) : 0;  // highest lane whose suffix reaches kk
        if (l == cl) {
          int cum = incl - own;  // count strictly above this lane's bins
          int sel = 4 * l;
          const unsigned hb[4] = {h3, h2, h1, h0};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (cum + (int)hb[j] >= kk) { sel = 4 * l + 3 - j; break; }
            cum += hb[j];
          }
          s_u[0] = (unsigned)sel;
          s_i[0] = kk - cum;
        }
      }
      __syncthreads();
      prefix |= s_u[0] << shift;
      msk |= 255u << shift;
      kk = s_i[0];
      __syncthreads();
    }
    for (int i = tid; i < V; i += SB)
      if (__float_as_uint(x[i]) < prefix) x[i] = 0.f;
    __syncthreads();
  }

  // ---- top-p: smallest kept value = first value whose cumulative (descending) mass > p ----
  if (tp > 0.f && tp < 1.f) {
    unsigned prefix = 0, msk = 0;
    float above = 0.f;
    unsigned crit = 0;      // keep iff bits > crit
    bool crossed = false;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = tid; i < 256; i += SB) mass[i] = 0.f;
      __syncthreads();
      for (int i = tid; i < V; i += SB) {
        const float pv = x[i];
        const unsigned b = __float_as_uint(pv);
        if (pv > 0.f && (b & msk) == prefix) atomicAdd(&mass[(b >> shift) & 255u], pv);
      }
      __syncthreads();
      if (tid < 64) {  // wave 0: first bin (from the top) whose cumulative mass crosses tp
        const int l = tid;
        const float m0 = mass[4 * l], m1 = mass[4 * l + 1], m2 = mass[4 * l + 2], m3 = mass[4 * l + 3];
        const float own = (m0 + m1) + (m2 + m3);
        float incl = own;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const float nb = __shfl_down(incl, o, 64);
          if (l + o < 64) incl += nb;
        }
        const unsigned long long hit = __ballot(above + incl > tp);
        if (!hit) {
          if (l == 0) { s_i[0] = -1; red[0] = above + incl; }
        } else {
          const int cl = 63 - __builtin_clzll(hit);
          if (l == cl) {
            float a = above + (incl - own);
            int sel = -1;
            const float mb[4] = {m3, m2, m1, m0};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if (mb[j] == 0.f) continue;
              if (a + mb[j] <= tp) { a += mb[j]; continue; }
              sel = 4 * l + 3 - j;
              break;
            }
            if (sel < 0) sel = 4 * l;  // rounding: the crossing sits in this lane's lowest non-empty bin
            s_u[0] = (unsigned)sel;
            s_i[0] = sel;
            red[0] = a;
          }
        }
      }
      __syncthreads();
      const int sel = s_i[0];
      above = red[0];
      __syncthreads();
      if (sel < 0) {  // every candidate under this prefix is kept
        crit = prefix > 0 ? prefix - 1 : 0;
        crossed = true;
        break;
      }
      prefix |= (unsigned)sel << shift;
      msk |= 255u << shift;
    }
    if (!crossed) crit = prefix;  // the crossing value itself is dropped
    if (crit >= maxbits) crit = maxbits - 1;  // always keep the most likely id
    for (int i = tid; i < V; i += SB)
      if (__float_as_uint(x[i]) <= crit) x[i] = 0.f;
    __syncthreads();
  }

  // ---- one inverse-CDF draw over contiguous per-thread chunks ----
  const int C = (V + SB - 1) / SB;
  const int lo = tid * C, hi = min(lo + C, V);
  float loc = 0.f;
  for (int i = lo; i < hi; ++i) loc += x[i];
  float total;
  const float excl = block_excl_scan(loc, red, &total);
  const float u = u01 * total;
  if (tid == 0) s_i[1] = -1;
  __syncthreads();
  if (loc > 0.f && u >= excl && u < excl + loc) {
    float c = excl;
    int pick = -1;
    for (int i = lo; i < hi; ++i) {
      const float pv = x[i];
      if (pv > 0.f) {
        pick = i;
        c += pv;
        if (u < c) break;
      }
    }
    s_i[1] = pick;
  }
  __syncthreads();
  if (tid == 0) {
    int pick = s_i[1];
    if (pick < 0) {  // rounding pushed u past the last interval: take the most likely id
      for (int i = 0; i < V; ++i)
        if (__float_as_uint(x[i]) == maxbits) { pick = i; break; }
    }
    out[row] = pick < 0 ? 0 : pick;
    s_i[0] = pick < 0 ? 0 : pick;
  }
  if (update) {
    __syncthreads();
    push_history_block(hrow, recent_len + row, recent_stride, n_hist, s_i[0], h_next);
  }
}

// ---------------------------------------------------------------------------------------
// Split sampler: the rows' top-k path over CH-element chunks of the vocabulary, one 256-thread
// workgroup per (chunk, row) - a 128K vocabulary does not fit one workgroup's LDS, and a single
// 1024-thread workgroup per row left the 1K-64K-wide sweeps, ~40 barriers and one memory round
// trip per row on ~R CUs (Llama-3 vocab: 128 us per 64-row step).  Same semantics as the fast
// top-k path above: the union of the chunks' exact top-k sets holds the row's top-k set, the
// merge orders it by (value desc, index asc) - the single workgroup's tie order - and the
// probabilities are full-softmax ones from the chunk maxima / normalisers.  Rows the split
// cannot take (k <= 0, k > SPLIT_KMAX, more than SPLIT_CAND candidates at a chunk's k-th
// value) are left at -1 for sample_kernel(only_unset = 1).
constexpr int SPLIT_CH = 8192;     // chunk width (fp32 in LDS: 32 KiB)
constexpr int SPLIT_NT = 256;      // threads per chunk workgroup
constexpr int SPLIT_KMAX = 64;     // largest top-k the split path takes
constexpr int SPLIT_CAND = 512;    // candidates per chunk before the exact rank
constexpr int SPLIT_MAXC = 64;     // chunks per row (one merge lane each): V <= 512K
// per (row, chunk) record in the workspace: [0] max of the penalised logits, [1] sum exp((x - max)
// / T), [2] raw max (greedy), [3] raw argmax, [4] candidate count (-1: degenerate), then
// SPLIT_KMAX (key, index) pairs sorted by (value desc, index asc)
constexpr int SPLIT_REC = 8 + 2 * SPLIT_KMAX;

template <int CTRL>
__device__ __forceinline__ u64 dpp_u64(u64 v) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)v, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(v >> 32), CTRL, 0xF, 0xF, true);
  return ((u64)(unsigned)hi << 32) | (unsigned)lo;
}
__device__ __forceinline__ u64 max_u64(u64 a, u64 b) { return a > b ? a : b; }

__device__ __forceinline__ float okey_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ __launch_bounds__(SPLIT_NT) void sample_split_chunk_kernel(
    const bf16_t* __restrict__ logits, int64_t stride, int V, const float* __restrict__ temps,
    const int32_t* __restrict__ top_ks, const float* __restrict__ rep_pens, const int32_t* __restrict__ recent,
    int recent_stride, const int32_t* __restrict__ recent_len, float* __restrict__ ws) {
  __shared__ float x[SPLIT_CH];
  __shared__ float red[SPLIT_NT / 64 + 1];
  __shared__ unsigned hist[256];
  __shared__ unsigned c_key[SPLIT_CAND];
  __shared__ int c_idx[SPLIT_CAND];
  __shared__ int s_cnt, s_sel, s_kk;
  __shared__ float s_rmax[SPLIT_NT / 64];
  __shared__ int s_ridx[SPLIT_NT / 64];
  const int c = blockIdx.x, row = blockIdx.y, tid = threadIdx.x, C = gridDim.x;
  const int lo = c * SPLIT_CH, n = min(SPLIT_CH, V - lo);
  float* rec = ws + ((int64_t)row * C + c) * SPLIT_REC;
  const bf16_t* lrow = logits + (int64_t)row * stride + lo;
  // raw copy + raw max / first argmax (greedy rows take the argmax of the raw logits): 16-B loads,
  // all of a thread's (SPLIT_CH / SPLIT_NT / 8 = 4) issued before the first use
  float rmx = -INFINITY;
  int rmi = 0x7fffffff;
  if ((n & 7) == 0 && (stride & 7) == 0) {
    constexpr int NV = SPLIT_CH / SPLIT_NT / 8;
    u16x8 v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i0 = (u * SPLIT_NT + tid) * 8;
      v[u] = i0 < n ? *reinterpret_cast<const u16x8*>(lrow + i0) : (u16x8)(0);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i0 = (u * SPLIT_NT + tid) * 8;
      if (i0 < n) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(v[u][j]);
          x[i0 + j] = f;
          if (f > rmx) { rmx = f; rmi = lo + i0 + j; }
        }
      }
    }
  } else {
    for (int i = tid; i < n; i += SPLIT_NT) {
      const float f = bf2f(lrow[i]);
      x[i] = f;
      if (f > rmx) { rmx = f; rmi = lo + i; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(rmx, o, 64);
    const int oi = __shfl_xor(rmi, o, 64);
    if (ov > rmx || (ov == rmx && oi < rmi)) { rmx = ov; rmi = oi; }
  }
  if ((tid & 63) == 0) { s_rmax[tid >> 6] = rmx; s_ridx[tid >> 6] = rmi; }
  __syncthreads();
  const float temp = temps[row];
  const int k = top_ks[row];
  if (tid == 0) {
    float b = s_rmax[0];
    int ix = s_ridx[0];
    for (int w = 1; w < SPLIT_NT / 64; ++w)
      if (s_rmax[w] > b || (s_rmax[w] == b && s_ridx[w] < ix)) { b = s_rmax[w]; ix = s_ridx[w]; }
    rec[2] = b;
    rec[3] = __int_as_float(ix);
    if (temp <= 0.f || k <= 0 || k > SPLIT_KMAX || k >= V) rec[4] = __int_as_float(-1);
  }
  if (temp <= 0.f || k <= 0 || k > SPLIT_KMAX || k >= V) return;  // greedy / not a split row

  // repetition penalty (reference src/rpc_handler.py:345-374) on the ids of this chunk
  const float rp = rep_pens[row];
  const int nrec = min((int)recent_len[row], recent_stride);
  const int32_t* hrow = recent + (int64_t)row * recent_stride;
  if (rp != 1.f && nrec > 0) {
    if (tid < nrec) {
      const int tok = hrow[tid];
      bool first = true;
      int count = 0;
      for (int j = 0; j < nrec; ++j) {
        const int h = hrow[j];
        if (h == tok) {
          ++count;
          if (j < tid) first = false;
        }
      }
      if (first && tok >= lo && tok < lo + n) {
        const float pen = powf(rp, (float)count);
        const float v = x[tok - lo];
        x[tok - lo] = v > 0.f ? v / pen : v * pen;
      }
    }
    __syncthreads();
    if (tid == 0 && nrec >= 3) {
      const int a = hrow[nrec - 1];
      if (hrow[nrec - 2] == a && hrow[nrec - 3] == a && a >= lo && a < lo + n) {
        const float pen = rp * rp * rp;
        const float v = x[a - lo];
        x[a - lo] = v > 0.f ? v / pen : v * pen;
      }
    }
    __syncthreads();
  }
  // chunk max and normaliser; per-thread key maxima
  const float inv_t = 1.f / fmaxf(temp, 1e-5f);
  float lm = -INFINITY;
  unsigned tmax = 0u;
  for (int i = tid; i < n; i += SPLIT_NT) {
    lm = fmaxf(lm, x[i]);
    tmax = max(tmax, okey(x[i]));
  }
  const float m = block_max(lm, red);
  float ls = 0.f;
  for (int i = tid; i < n; i += SPLIT_NT) ls += __expf((x[i] - m) * inv_t);
  const float zs = block_sum(ls, red);
  // tau = the kk-th largest of the per-thread key maxima (<= the chunk's kk-th largest value),
  // by 8-bit radix rounds: wave 0 finds the bin holding it from the top
  const int kc = min(k, n);
  const int nmax = min(SPLIT_NT, n);  // threads that saw at least one element
  unsigned prefix = 0u, msk = 0u;
  int kk = min(kc, nmax);
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += SPLIT_NT) hist[i] = 0u;
    __syncthreads();
    if (tid < nmax && (tmax & msk) == prefix) atomicAdd(&hist[(tmax >> shift) & 255u], 1u);
    __syncthreads();
    if (tid < 64) {
      const int l = tid;
      const unsigned h0 = hist[4 * l], h1 = hist[4 * l + 1], h2 = hist[4 * l + 2], h3 = hist[4 * l + 3];
      const int own = (int)(h0 + h1 + h2 + h3);
      int incl = own;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int nb = __shfl_down(incl, o, 64);
        if (l + o < 64) incl += nb;
      }
      const unsigned long long hit = __ballot(incl >= kk);
      const int cl = hit ? 63 - __builtin_clzll(hit) : 0;
      if (l == cl) {
        int cum = incl - own;
        int sel = 4 * l;
        const unsigned hb[4] = {h3, h2, h1, h0};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (cum + (int)hb[j] >= kk) { sel = 4 * l + 3 - j; break; }
          cum += hb[j];
        }
        s_sel = sel;
        s_kk = kk - cum;
      }
    }
    __syncthreads();
    prefix |= (unsigned)s_sel << shift;
    msk |= 255u << shift;
    kk = s_kk;
    __syncthreads();
  }
  const unsigned tau = prefix;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  for (int i = tid; i < n; i += SPLIT_NT) {
    const unsigned key = okey(x[i]);
    if (key >= tau) {
      const int pos = atomicAdd(&s_cnt, 1);
      if (pos < SPLIT_CAND) {
        c_key[pos] = key;
        c_idx[pos] = lo + i;
      }
    }
  }
  __syncthreads();
  const int cnt = s_cnt;
  if (tid == 0) {
    rec[0] = m;
    rec[1] = zs;
    rec[4] = __int_as_float(cnt > SPLIT_CAND ? -1 : min(cnt, kc));
  }
  if (cnt > SPLIT_CAND) return;  // degenerate chunk: the row goes to the single-workgroup kernel
  for (int t = tid; t < cnt; t += SPLIT_NT) {  // exact rank by (value desc, index asc)
    const unsigned kt = c_key[t];
    const int it = c_idx[t];
    int rank = 0;
    for (int j = 0; j < cnt; ++j) {
      const unsigned kj = c_key[j];
      rank += (kj > kt) || (kj == kt && c_idx[j] < it);
    }
    if (rank < kc) {
      rec[8 + 2 * rank] = __uint_as_float(kt);
      rec[9 + 2 * rank] = __int_as_float(it);
    }
  }
}

// One 64-lane wave per row: lane l walks chunk l's sorted top-k list; k rounds of a wave-wide
// (key desc, index asc) argmax merge them into the row's sorted top-k; then the full-softmax
// probabilities, top-p (keep the sorted prefix with cumulative <= p, always the first), one
// inverse-CDF draw with the row's seeded uniform - the fast path's arithmetic.
__global__ __launch_bounds__(64) void sample_split_merge_kernel(
    int V, int C, const float* __restrict__ temps, const float* __restrict__ top_ps, const int32_t* __restrict__ top_ks,
    int32_t* __restrict__ recent, int recent_stride, int32_t* __restrict__ recent_len,
    const int64_t* __restrict__ seeds, const float* __restrict__ ws, int64_t* __restrict__ out, int update) {
  __shared__ unsigned s_key[SPLIT_KMAX];
  __shared__ int s_idx[SPLIT_KMAX];
  __shared__ unsigned l_key[SPLIT_MAXC][SPLIT_KMAX];  // the chunks' sorted lists, staged once
  __shared__ int l_idx[SPLIT_MAXC][SPLIT_KMAX];
  const int row = blockIdx.x, l = threadIdx.x;
  const float* base = ws + (int64_t)row * C * SPLIT_REC;
  const float temp = temps[row];
  const int k = top_ks[row];
  if (temp <= 0.f) {  // greedy: first maximum of the raw logits over the chunks
    if (l == 0) {
      float b = -INFINITY;
      int ix = 0x7fffffff;
      for (int c = 0; c < C; ++c) {
        const float v = base[c * SPLIT_REC + 2];
        const int i = __float_as_int(base[c * SPLIT_REC + 3]);
        if (v > b || (v == b && i < ix)) { b = v; ix = i; }
      }
      const int pick = ix == 0x7fffffff ? 0 : ix;
      out[row] = pick;
      if (update) push_history(recent + (int64_t)row * recent_stride, recent_len + row, recent_stride, pick);
    }
    return;
  }
  // any chunk unable to take the row (or k outside the split range): leave it to sample_kernel
  bool bad = k <= 0 || k > SPLIT_KMAX || k >= V;
  int mycnt = 0;
  float mc = -INFINITY, zc = 0.f;
  if (l < C) {
    const float* r = base + l * SPLIT_REC;
    mycnt = __float_as_int(r[4]);
    mc = r[0];
    zc = r[1];
    if (mycnt < 0) bad = true;
  }
  if (__ballot(bad)) {
    if (l == 0) out[row] = -1;
    return;
  }
  // global max and normaliser
  float M = mc;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
  const float inv_t = 1.f / fmaxf(temp, 1e-5f);
  float zp = l < C ? zc * __expf((mc - M) * inv_t) : 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) zp += __shfl_xor(zp, o, 64);
  const float inv_s = 1.f / zp;
  // stage every list in LDS (all loads in flight together: one memory round trip, not one per
  // merge step), then a k-way merge of the lists
  // (slots past a list's count hold stale words that the merge never reads)
  for (int c0 = 0; c0 < C; c0 += 8) {
    unsigned kv[8];
    int iv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (c0 + u < C) {
        kv[u] = __float_as_uint(base[(c0 + u) * SPLIT_REC + 8 + 2 * l]);
        iv[u] = __float_as_int(base[(c0 + u) * SPLIT_REC + 9 + 2 * l]);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (c0 + u < C) {
        l_key[c0 + u][l] = kv[u];
        l_idx[c0 + u][l] = iv[u];
      }
    }
  }
  __syncthreads();
  // each lane's head as one 64-bit composite, larger = earlier in (value desc, index asc) order:
  // (key << 32) | ~index (0: no head - every real key is > 0); the lists are merged by a
  // DPP max over the 16 lanes of a row (+ two shuffle rounds past 16 chunks)
  int pos = 0;
  int got = 0;
  auto head = [&]() -> u64 {
    return (l < C && pos < mycnt) ? (((u64)l_key[l][pos] << 32) | (u64)(~(unsigned)l_idx[l][pos])) : 0ull;
  };
  u64 h = head();
  for (int j = 0; j < k; ++j) {
    u64 b = h;
    b = max_u64(b, dpp_u64<0xB1>(b));   // quad_perm [1,0,3,2]
    b = max_u64(b, dpp_u64<0x4E>(b));   // quad_perm [2,3,0,1]
    b = max_u64(b, dpp_u64<0x141>(b));  // row_half_mirror
    b = max_u64(b, dpp_u64<0x140>(b));  // row_mirror: the 16-lane row's max in every lane
    if (C > 16) {
      b = max_u64(b, (u64)__shfl_xor((unsigned long long)b, 16, 64));
      b = max_u64(b, (u64)__shfl_xor((unsigned long long)b, 32, 64));
    }
    if (b == 0ull) break;  // every list exhausted (fewer than k ids in the row)
    if (l == 0) {
      s_key[j] = (unsigned)(b >> 32);
      s_idx[j] = (int)~(unsigned)b;
    }
    if (h == b) {  // this lane's head was taken
      ++pos;
      h = head();
    }
    ++got;
  }
  // rows 1..3 of the wave (no lists when C <= 16) left the loop at once: lane 0's count is the row's
  got = __shfl(got, 0, 64);
  __syncthreads();
  // probabilities of the sorted survivors (lane l holds ranks l and l + 64 - SPLIT_KMAX <= 64: one)
  const float pv = l < got ? __expf((okey_inv(s_key[l]) - M) * inv_t) * inv_s : 0.f;
  // exclusive prefix over the sorted order
  float inc = pv;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float nb = __shfl_up(inc, o, 64);
    if (l >= o) inc += nb;
  }
  const float ex1 = inc - pv;
  const float tp = top_ps[row];
  const bool keep = l < got && (l == 0 || !(tp > 0.f && tp < 1.f) || ex1 + pv <= tp);
  const float q = keep ? pv : 0.f;
  float inc2 = q;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float nb = __shfl_up(inc2, o, 64);
    if (l >= o) inc2 += nb;
  }
  const float t2 = __shfl(inc2, 63, 64);
  const float ex2 = inc2 - q;
  const uint64_t rnd = splitmix64((uint64_t)seeds[row] * 0x9E3779B97F4A7C15ull + (uint64_t)row);
  const float u01 = (float)((double)(rnd >> 11) * (1.0 / 9007199254740992.0));
  const float uu = u01 * t2;
  const unsigned long long hit = __ballot(q > 0.f && uu >= ex2 && uu < ex2 + q);
  if (l == 0) {
    const int pick = hit ? s_idx[__builtin_ctzll(hit)] : s_idx[0];  // rounding: the most likely id
    out[row] = pick;
    if (update) push_history(recent + (int64_t)row * recent_stride, recent_len + row, recent_stride, pick);
  }
}

}  // namespace mp

extern "C" int mp_sample(const void* logits, int64_t stride, int R, int V, const float* temps, const float* top_ps,
                         const int32_t* top_ks, const float* rep_pens, int32_t* recent, int recent_stride,
                         int32_t* recent_len, const int64_t* seeds, float* ws, int64_t* out, int update,
                         hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  if (R == 0) return 0;
  if (recent_stride > SB) return -1;
  const size_t lds = (size_t)V * sizeof(float);
  const int use_lds = lds <= 136 * 1024;  // + ~23 KB of histogram / candidate arrays
  // split path for wide vocabularies: the 128K Llama-3 vocabulary takes it, Llama-2's 32K does not
  // (splitting the 32K rows measured no gain, profiles/r4m)
  constexpr int split_min = 65536;
  const int C = (V + SPLIT_CH - 1) / SPLIT_CH;
  const bool split = V >= split_min && C <= SPLIT_MAXC && recent_stride <= SPLIT_NT &&
                     (int64_t)R * V >= (int64_t)R * C * SPLIT_REC;  // the records fit the workspace
  if (split) {
    hipLaunchKernelGGL(sample_split_chunk_kernel, dim3(C, R), dim3(SPLIT_NT), 0, stream, (const bf16_t*)logits,
                       stride, V, temps, top_ks, rep_pens, recent, recent_stride, recent_len, ws);
    hipLaunchKernelGGL(sample_split_merge_kernel, dim3(R), dim3(64), 0, stream, V, C, temps, top_ps, top_ks, recent,
                       recent_stride, recent_len, seeds, ws, out, update);
    // rows the split could not take (out = -1) run the single-workgroup kernel; the others exit
    // at once.  (Its global-workspace rows overlap the split records: only -1 rows use them.)
  }
  if (use_lds)
    hipLaunchKernelGGL(sample_kernel<true>, dim3(R), dim3(SB), lds, stream, (const bf16_t*)logits, stride, V, temps,
                       top_ps, top_ks, rep_pens, recent, recent_stride, recent_len, seeds, ws, out, 1, update,
                       split ? 1 : 0);
  else
    hipLaunchKernelGGL(sample_kernel<false>, dim3(R), dim3(SB), 0, stream, (const bf16_t*)logits, stride, V, temps,
                       top_ps, top_ks, rep_pens, recent, recent_stride, recent_len, seeds, ws, out, 0, update,
                       split ? 1 : 0);
  return (int)hipGetLastError();
}
