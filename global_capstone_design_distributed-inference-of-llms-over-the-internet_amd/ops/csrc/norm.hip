// RMSNorm family for gfx950.
//
// Replaces the reference's graph-captured HF LlamaRMSNorm callables
// (reference petals/llama/block.py:169-181, :210-213, :232-235) and the
// separate residual adds (block.py:227, :238) with ONE kernel per norm site:
//
//   mode 0:  y = rmsnorm(x) * w
//   mode 1:  residual = bf16(residual + x);  y = rmsnorm(residual) * w   (fused add)
//   mode 2:  residual = x;                   y = rmsnorm(x) * w          (stage entry)
//   mode 3:  residual = x;  y = x (raw);  ss[0][row] = sum(round(x^2 * 2^20)) as an exact u64,
//            ss[1..31][row] = 0   (stage entry of the fused-norm decode path: the GEMMs apply
//            the norm themselves and keep these fixed-point statistics, see gemm.hip EpiArgs)
// packed_mt > 0 writes y in the packed decode-GEMM activation layout (common.h apk_off).
// a8 != null (fp8 W8A8 decode path): y is instead quantized to OCP e4m3 with a per-row scale
// max|y| / 448 into the fp8 GEMM's A layout A8[K/64][MT][64][16 B] (fp8.hip) and a8_scale[row]:
// the norm owns whole rows, so the absmax needs no cross-workgroup pass (round 1 ran a
// separate two-launch quantization after every norm).
//
// `rows` (optional) gathers input rows (e.g. the last token of each prompt for
// the final norm before lm_head), so the output has one row per index.
// Rounding follows HF: the normalised value is rounded to bf16 before the
// weight multiply, math in fp32, vectorised 16-B loads, one block per row.
#include "common.h"
#include <stdlib.h>

namespace mp {

template <int MAXC, int NT = 256>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(
    const bf16_t* __restrict__ x, int64_t x_stride, bf16_t* __restrict__ res, int64_t res_stride,
    const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int64_t y_stride,
    const int32_t* __restrict__ rows, int H, float eps, int mode, int packed_mt,
    unsigned long long* __restrict__ ss_out, uint8_t* __restrict__ a8, float* __restrict__ a8_scale,
    const int64_t* __restrict__ gather, int64_t gather_n) {
  __shared__ float red[16];
  __shared__ float redm[16];
  __shared__ unsigned long long redq[16];
  const int orow = blockIdx.x;
  const int irow = rows ? rows[orow] : orow;
  const int nch = H >> 3;
  // gather (the stage entry of a first stage): input row = the token's embedding-table row, so the
  // embedding lookup and the stage-entry statistics are one launch; the residual row is the token's
  int64_t xrow = irow;
  if (gather != nullptr) {
    const int64_t id = gather[orow];
    xrow = (id < 0 || id >= gather_n) ? 0 : id;  // never read out of bounds; the host validates ids
  }
  const bf16_t* xr = x + xrow * x_stride;
  bf16_t* rr = res + (int64_t)(gather != nullptr ? orow : irow) * res_stride;
  // every global load (x, residual, weight) is issued before the first store and before the
  // block reduction, unconditionally (clamped chunk index: no exec-masked branches between the
  // loads): one memory round trip per call instead of three
  u16x8 v[MAXC], rv[MAXC], wv[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = min((int)threadIdx.x + k * NT, nch - 1);
    v[k] = *reinterpret_cast<const u16x8*>(xr + c * 8);
    rv[k] = *reinterpret_cast<const u16x8*>((mode == 1 ? rr : xr) + c * 8);
    wv[k] = *reinterpret_cast<const u16x8*>(w + c * 8);
  }
  float ss = 0.f;
  unsigned long long ssq = 0;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = threadIdx.x + k * NT;
    if (c < nch) {
      u16x8 a = v[k];
      if (mode == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = f2bf(bf2f(a[j]) + bf2f(rv[k][j]));
        *reinterpret_cast<u16x8*>(rr + c * 8) = a;
      } else if (mode >= 2) {
        *reinterpret_cast<u16x8*>(rr + c * 8) = a;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(a[j]);
        ss += f * f;
        if (mode == 3) ssq += (unsigned long long)__float2ull_rn(f * f * 1048576.f);
      }
      v[k] = a;
    }
  }
  // one wave per row: the shuffle reduction alone (no LDS round trip, no barrier)
  const float tot = NT == 64 ? wave_sum(ss) : block_sum(ss, red);
  const float r = rsqrtf(tot / (float)H + eps);
  if (mode == 3) {  // exact integer block sum (order-independent), then the 32 shards of this row
    ssq = wave_sum_u64(ssq);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (NT > 64) {
      if (lane == 0) redq[wid] = ssq;
      __syncthreads();
      ssq = 0;
      for (int i = 0; i < NT / 64; ++i) ssq += redq[i];
    }
    if (threadIdx.x < 32) ss_out[threadIdx.x * QP_SS_ROWS + orow] = threadIdx.x == 0 ? ssq : 0ull;  // [32][256] shards
  }
  bf16_t* yr = y + (int64_t)orow * y_stride;
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = threadIdx.x + k * NT;
    if (c < nch) {
      const u16x8 wv_ = wv[k];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = mode == 3 ? v[k][j] : f2bf(round_bf(bf2f(v[k][j]) * r) * bf2f(wv_[j]));
      if (a8 != nullptr) {
        v[k] = o;  // kept for the quantization pass below
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f(o[j])));
      } else if (packed_mt > 0) {
        *reinterpret_cast<u16x8*>(y + apk_off(orow, c * 8, packed_mt)) = o;
      } else {
        *reinterpret_cast<u16x8*>(yr + c * 8) = o;
      }
    }
  }
  if (a8 == nullptr) return;
  amax = NT == 64 ? wave_max(amax) : block_max(amax, redm);
  const float sc = amax > 0.f ? amax * (1.f / 448.f) : 1.f;
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) a8_scale[orow] = sc;
  const int mt = orow >> 4, r16 = orow & 15;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = threadIdx.x + k * NT;  // 8 columns 8c .. 8c+7
    if (c < nch) {
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(bf2f(v[k][j]) * inv, -448.f), 448.f);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
      const int col = c * 8, ch = col >> 6, half = (col >> 5) & 1, q = (col >> 3) & 3;
      int2 o2;
      o2.x = lo;
      o2.y = hi;
      *reinterpret_cast<int2*>(a8 + (((int64_t)ch * packed_mt + mt) * 64 + q * 16 + r16) * 16 + half * 8) = o2;
    }
  }
}

}  // namespace mp

extern "C" int mp_rmsnorm(const void* x, int64_t x_stride, void* res, int64_t res_stride, const void* w,
                          void* y, int64_t y_stride, const int32_t* rows, int nrows, int H, float eps,
                          int mode, int packed_mt, void* ss_out, void* a8, float* a8_scale,
                          const int64_t* gather, int64_t gather_n, hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  if (H % 8 != 0 || H > 8 * 256 * 8) return -1;
  if (mode == 3 && (ss_out == nullptr || nrows > QP_SS_ROWS)) return -2;
  if (a8 != nullptr && (packed_mt <= 0 || H % 64 || a8_scale == nullptr || mode == 3)) return -3;
  if (gather != nullptr && (mode < 2 || rows != nullptr || gather_n <= 0)) return -4;
  if (nrows == 0) return 0;
  const int nch = H / 8;
  // threads per row: 512 (one 16-B chunk per thread at H = 4096) measured best in the decode
  // step, 64 -> 512: 13433 / 13493 / 13615 / 13719 tok/s (Llama-2-7B, 64 sessions, one box,
  // profiles/r1_norm_threads/); the kernel itself only moves 5.06 -> 4.99 us, it is latency
  // bound at 64 rows.  1024 threads for wider rows (H = 8192: Llama-3-70B), so every thread still
  // owns one chunk
  const int nt = nch > 512 ? 1024 : 512;
  dim3 grid(nrows), block(nt);
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, block, 0, stream, (const bf16_t*)x, x_stride, (bf16_t*)res, res_stride,
                       (const bf16_t*)w, (bf16_t*)y, y_stride, rows, H, eps, mode, packed_mt,
                       (unsigned long long*)ss_out, (uint8_t*)a8, a8_scale, gather, gather_n);
  };
  // MAXC = chunks of 8 per thread; nch <= MAXC * nt
  const int per = (nch + nt - 1) / nt;
  if (nt == 1024) {
    if (per <= 1) args(rmsnorm_kernel<1, 1024>);
    else args(rmsnorm_kernel<2, 1024>);
  } else {
    if (per <= 1) args(rmsnorm_kernel<1, 512>);
    else if (per <= 2) args(rmsnorm_kernel<2, 512>);
    else args(rmsnorm_kernel<4, 512>);
  }
  return (int)hipGetLastError();
}
