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

namespace mp {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

constexpr int SB = 1024;   // threads per block
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

// Exclusive block scan of one float per thread (blockDim == SB).
__device__ __forceinline__ float block_excl_scan(float v, float* red, float* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float n = __shfl_up(inc, o, 64);
    if (lane >= o) inc += n;
  }
  __syncthreads();
  if (lane == 63) red[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc = 0.f;
    for (int i = 0; i < SB / 64; ++i) {
      const float t = red[i];
      red[i] = acc;
      acc += t;
    }
    red[SB / 64] = acc;
  }
  __syncthreads();
  *total = red[SB / 64];
  return red[w] + inc - v;
}

__global__ __launch_bounds__(SB) void sample_kernel(const bf16_t* __restrict__ logits, int64_t stride, int V,
                                                    const float* __restrict__ temps, const float* __restrict__ top_ps,
                                                    const int32_t* __restrict__ top_ks,
                                                    const float* __restrict__ rep_pens,
                                                    int32_t* __restrict__ recent, int recent_stride,
                                                    int32_t* __restrict__ recent_len,
                                                    const int64_t* __restrict__ seeds, float* __restrict__ ws,
                                                    int64_t* __restrict__ out, int use_lds, int update) {
  __shared__ float red[SB / 64 + 1];
  __shared__ unsigned hist[256];
  __shared__ float mass[256];
  __shared__ unsigned s_u[4];  // scratch: selected bin, fallback flag, remaining rank
  __shared__ int s_i[2];
  extern __shared__ __attribute__((aligned(16))) float s_row[];
  const int row = blockIdx.x, tid = threadIdx.x;
  const bf16_t* lrow = logits + (int64_t)row * stride;
  // the working row lives in LDS when it fits (V <= 38K: every pass is an LDS sweep),
  // otherwise in the global workspace (L2-resident)
  float* x = (use_lds ? s_row : ws + (int64_t)row * V);
  const float temp = temps[row];

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
      if (update) push_history(recent + (int64_t)row * recent_stride, recent_len + row, recent_stride,
                               ix == 0x7fffffff ? 0 : ix);
    }
    return;
  }
  __syncthreads();

  // ---- repetition penalty (reference src/rpc_handler.py:345-374) ----
  const float rp = rep_pens[row];
  const int nrec = min((int)recent_len[row], recent_stride);
  __shared__ int s_rec[SB];
  if (tid < nrec) s_rec[tid] = recent[(int64_t)row * recent_stride + tid];
  __syncthreads();
  const int* rec = s_rec;  // the history, staged in LDS (each thread scans all of it)
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
        const float v = x[tok];
        x[tok] = v > 0.f ? v / pen : v * pen;
      }
    }
    __syncthreads();
    if (tid == 0 && nrec >= 3) {
      const int a = rec[nrec - 1];
      if (rec[nrec - 2] == a && rec[nrec - 3] == a && a >= 0 && a < V) {
        const float pen = rp * rp * rp;
        const float v = x[a];
        x[a] = v > 0.f ? v / pen : v * pen;
      }
    }
    __syncthreads();
  }

  // ---- softmax(x / T): max and normaliser (x keeps the penalised logits) ----
  const float inv_t = 1.f / fmaxf(temp, 1e-5f);
  float lm = -INFINITY;
  for (int i = tid; i < V; i += SB) lm = fmaxf(lm, x[i]);
  const float m = block_max(lm, red);
  float ls = 0.f;
  for (int i = tid; i < V; i += SB) ls += __expf((x[i] - m) * inv_t);
  const float inv_s = 1.f / block_sum(ls, red);
  const int k = top_ks[row];
  const float tp = top_ps[row];
  const uint64_t rnd = splitmix64((uint64_t)seeds[row] * 0x9E3779B97F4A7C15ull + (uint64_t)row);
  const float u01 = (float)((double)(rnd >> 11) * (1.0 / 9007199254740992.0));

  if (k > 0 && k < V) {
    // ---- fast top-k.  The k-th largest of the 1024 per-thread maxima, tau, is <= the k-th
    //      largest value (those k maxima are values of the row), so every top-k id has
    //      key >= tau, and few others do.  Selecting among 1024 maxima instead of V keys
    //      avoids the LDS-atomic pile-up on the few bins dense logits fall into. ----
    __shared__ unsigned h2k[2048];
    __shared__ unsigned c_key[CAND];
    __shared__ int c_idx[CAND];
    __shared__ float c_p[CAND];
    __shared__ int s_cnt;
    if (tid == 0) { s_cnt = 0; s_u[1] = 0u; }
    unsigned tmax = 0u;
    for (int i = tid; i < V; i += SB) tmax = max(tmax, okey(x[i]));
    // exact k-th largest of the per-thread maxima: radix select over 1024 keys (11 + 11 + 10
    // bits), cheap however flat the row is (random-init logits are nearly uniform)
    unsigned prefix = 0u, msk = 0u;
    int kk = k;
    for (int round = 0; round < 3; ++round) {
      const int shift = round == 0 ? 21 : (round == 1 ? 10 : 0);
      const unsigned nb = round < 2 ? 2048u : 1024u;
      for (int i = tid; i < 2048; i += SB) h2k[i] = 0;
      __syncthreads();
      if (tid < V && (tmax & msk) == prefix) atomicAdd(&h2k[(tmax >> shift) & (nb - 1)], 1u);
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
    if (fast) {
      for (int i = tid; i < V; i += SB) {
        const unsigned key = okey(x[i]);
        if (key >= tau) {
          const int pos = atomicAdd(&s_cnt, 1);
          if (pos < CAND) {
            c_key[pos] = key;
            c_idx[pos] = i;
          }
        }
      }
      __syncthreads();
      fast = s_cnt <= CAND;
    }
    if (fast) {
      const int c = s_cnt;
      // rank by (value desc, index asc); rank < k survives top-k
      int rank = CAND, my_idx = 0;
      if (tid < c) {
        const unsigned kt = c_key[tid];
        my_idx = c_idx[tid];
        rank = 0;
        for (int j = 0; j < c; ++j) {
          const unsigned kj = c_key[j];
          rank += (kj > kt) || (kj == kt && c_idx[j] < my_idx);
        }
      }
      __syncthreads();
      if (rank < k) {  // sorted (descending) survivors: index and FULL-softmax probability
        c_idx[rank] = my_idx;
        c_p[rank] = __expf((x[my_idx] - m) * inv_t) * inv_s;
      }
      __syncthreads();
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
      if (tid == 0) {
        out[row] = s_i[1];
        if (update) push_history(recent + (int64_t)row * recent_stride, recent_len + row, recent_stride, s_i[1]);
      }
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
    if (update) push_history(recent + (int64_t)row * recent_stride, recent_len + row, recent_stride,
                             pick < 0 ? 0 : pick);
  }
}

}  // namespace mp

extern "C" int mp_sample(const void* logits, int64_t stride, int R, int V, const float* temps, const float* top_ps,
                         const int32_t* top_ks, const float* rep_pens, int32_t* recent, int recent_stride,
                         int32_t* recent_len, const int64_t* seeds, float* ws, int64_t* out, int update,
                         hipStream_t stream) {
  using namespace mp;
  if (R == 0) return 0;
  if (recent_stride > SB) return -1;
  const size_t lds = (size_t)V * sizeof(float);
  const int use_lds = lds <= 136 * 1024;  // + ~23 KB of histogram / candidate arrays
  hipLaunchKernelGGL(sample_kernel, dim3(R), dim3(SB), use_lds ? lds : 0, stream, (const bf16_t*)logits, stride, V,
                     temps, top_ps, top_ks, rep_pens, recent, recent_stride, recent_len, seeds, ws, out, use_lds, update);
  return (int)hipGetLastError();
}
