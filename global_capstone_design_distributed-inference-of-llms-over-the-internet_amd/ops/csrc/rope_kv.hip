// RoPE + paged KV-cache write for gfx950 (fuses survey K4 + K5 + K6).
//
// The reference rotates q/k with HF `apply_rotary_pos_emb` (graph-captured at
// T == 1, reference petals/llama/block.py:44-49, :96-121) and then grows the KV
// cache with `torch.cat` every step (block.py:123-128, an O(P) copy per token).
// Here one kernel per layer reads the fused QKV projection output once:
//   * q heads are rotated in place (rotate_half convention, fp32 cos/sin table),
//   * k heads are rotated and written straight into their page slot,
//   * v heads are copied into their page slot,
// so the cache is written exactly once per token and never copied again.
//
// Layouts: qkv [T, (nh + 2*nkv) * D] (row stride given), cos/sin [max_pos, D/2] fp32,
// cache [num_pages, nkv, page_size, D] bf16, slots[t] = page * page_size + offset
// (negative slot = padded row: nothing is written).
#include "common.h"

namespace mp {

// Every load of a row is issued before the first store, unconditionally (indices clamped, so
// no exec-masked branches split the load phase): the old item loop stored into the same qkv
// row between loads, so each of its iterations paid a full memory round trip (5.5 us per call
// at 64 rows).  ROPE_MAXI items of 4 rotation pairs and ROPE_MAXV 16-B v chunks per thread.
constexpr int ROPE_THREADS = 512, ROPE_MAXI = 4, ROPE_MAXV = 2;

__global__ __launch_bounds__(ROPE_THREADS) void rope_kv_kernel(bf16_t* __restrict__ qkv, int64_t qkv_stride,
                                                               const int64_t* __restrict__ pos,
                                                               const float* __restrict__ cos_t,
                                                               const float* __restrict__ sin_t,
                                                               bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                                                               const int64_t* __restrict__ slots, int nh, int nkv,
                                                               int D, int page_size) {
  const int t = blockIdx.x;
  const int64_t slot = slots[t];
  const int64_t p = pos[t];
  bf16_t* row = qkv + (int64_t)t * qkv_stride;
  const int half = D >> 1;
  const int qpr = half >> 2;  // 4-pair groups per head
  const int nitems = (nh + nkv) * qpr;
  const int vch = D >> 3, nv = nkv * vch;
  const bf16_t* vsrc = row + (nh + nkv) * D;
  const float* ct = cos_t + p * half;
  const float* st = sin_t + p * half;

  u16x4 a[ROPE_MAXI], b[ROPE_MAXI];
  f32x4 cs[ROPE_MAXI], sn[ROPE_MAXI];
  u16x8 v[ROPE_MAXV];
#pragma unroll
  for (int k = 0; k < ROPE_MAXI; ++k) {
    const int it = min((int)threadIdx.x + k * ROPE_THREADS, nitems - 1);
    const int h = it / qpr, i = (it - h * qpr) * 4;
    a[k] = *reinterpret_cast<const u16x4*>(row + h * D + i);
    b[k] = *reinterpret_cast<const u16x4*>(row + h * D + half + i);
  }
#pragma unroll
  for (int k = 0; k < ROPE_MAXV; ++k) {
    const int it = min((int)threadIdx.x + k * ROPE_THREADS, nv - 1);
    const int h = it / vch, c = it - h * vch;
    v[k] = *reinterpret_cast<const u16x8*>(vsrc + h * D + c * 8);
  }
#pragma unroll
  for (int k = 0; k < ROPE_MAXI; ++k) {
    const int it = min((int)threadIdx.x + k * ROPE_THREADS, nitems - 1);
    const int i = (it % qpr) * 4;
    cs[k] = *reinterpret_cast<const f32x4*>(ct + i);
    sn[k] = *reinterpret_cast<const f32x4*>(st + i);
  }
  const int64_t page = slot >= 0 ? slot / page_size : 0;
  const int64_t off = slot >= 0 ? slot - page * page_size : 0;
  const int64_t page_base = page * (int64_t)nkv * page_size * D;
  // rotate and store: q in place, k and v into the page slot
#pragma unroll
  for (int k = 0; k < ROPE_MAXI; ++k) {
    const int it = threadIdx.x + k * ROPE_THREADS;
    if (it >= nitems) continue;
    const int h = it / qpr, i = (it - h * qpr) * 4;
    u16x4 oa, ob;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x1 = bf2f(a[k][j]), x2 = bf2f(b[k][j]);
      oa[j] = f2bf(x1 * cs[k][j] - x2 * sn[k][j]);
      ob[j] = f2bf(x2 * cs[k][j] + x1 * sn[k][j]);
    }
    if (h < nh) {
      *reinterpret_cast<u16x4*>(row + h * D + i) = oa;
      *reinterpret_cast<u16x4*>(row + h * D + half + i) = ob;
    } else if (slot >= 0) {
      bf16_t* dst = kc + page_base + ((int64_t)(h - nh) * page_size + off) * D;
      *reinterpret_cast<u16x4*>(dst + i) = oa;
      *reinterpret_cast<u16x4*>(dst + half + i) = ob;
    }
  }
  if (slot < 0) return;
#pragma unroll
  for (int k = 0; k < ROPE_MAXV; ++k) {
    const int it = threadIdx.x + k * ROPE_THREADS;
    if (it < nv) {
      const int h = it / vch, c = it - h * vch;
      *reinterpret_cast<u16x8*>(vc + page_base + ((int64_t)h * page_size + off) * D + c * 8) = v[k];
    }
  }
}

// Plain KV write without rotation (learned-position models such as GPT-2).
__global__ __launch_bounds__(256) void kv_write_kernel(const bf16_t* __restrict__ k, int64_t k_stride,
                                                       const bf16_t* __restrict__ v, int64_t v_stride,
                                                       bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                                                       const int64_t* __restrict__ slots, int nkv, int D,
                                                       int page_size) {
  const int t = blockIdx.x;
  const int64_t slot = slots[t];
  if (slot < 0) return;
  const int64_t page = slot / page_size, off = slot - page * page_size;
  const int64_t page_base = page * (int64_t)nkv * page_size * D;
  const int vch = D >> 3;
  for (int it = threadIdx.x; it < nkv * vch; it += blockDim.x) {
    const int h = it / vch, c = it - h * vch;
    const int64_t dst = page_base + ((int64_t)h * page_size + off) * D + c * 8;
    *reinterpret_cast<u16x8*>(kc + dst) = *reinterpret_cast<const u16x8*>(k + t * k_stride + h * D + c * 8);
    *reinterpret_cast<u16x8*>(vc + dst) = *reinterpret_cast<const u16x8*>(v + t * v_stride + h * D + c * 8);
  }
}

}  // namespace mp

extern "C" int mp_rope_kv_write(void* qkv, int64_t qkv_stride, const int64_t* pos, const float* cos_t,
                                const float* sin_t, void* kc, void* vc, const int64_t* slots, int T, int nh,
                                int nkv, int D, int page_size, hipStream_t stream) {
  using namespace mp;
  if (D % 8 != 0) return -1;
  if ((nh + nkv) * D / 8 > ROPE_THREADS * ROPE_MAXI || nkv * D / 8 > ROPE_THREADS * ROPE_MAXV) return -2;
  if (T == 0) return 0;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(T), dim3(ROPE_THREADS), 0, stream, (bf16_t*)qkv, qkv_stride, pos, cos_t, sin_t,
                     (bf16_t*)kc, (bf16_t*)vc, slots, nh, nkv, D, page_size);
  return (int)hipGetLastError();
}

extern "C" int mp_kv_write(const void* k, int64_t k_stride, const void* v, int64_t v_stride, void* kc, void* vc,
                           const int64_t* slots, int T, int nkv, int D, int page_size, hipStream_t stream) {
  using namespace mp;
  if (D % 8 != 0) return -1;
  if (T == 0) return 0;
  hipLaunchKernelGGL(kv_write_kernel, dim3(T), dim3(256), 0, stream, (const bf16_t*)k, k_stride,
                     (const bf16_t*)v, v_stride, (bf16_t*)kc, (bf16_t*)vc, slots, nkv, D, page_size);
  return (int)hipGetLastError();
}
