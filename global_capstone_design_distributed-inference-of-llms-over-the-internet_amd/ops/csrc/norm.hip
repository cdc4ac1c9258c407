// RMSNorm family for gfx950.
//
// Replaces the reference's graph-captured HF LlamaRMSNorm callables
// (reference petals/llama/block.py:169-181, :210-213, :232-235) and the
// separate residual adds (block.py:227, :238) with ONE kernel per norm site:
//
//   mode 0:  y = rmsnorm(x) * w
//   mode 1:  residual = bf16(residual + x);  y = rmsnorm(residual) * w   (fused add)
//   mode 2:  residual = x;                   y = rmsnorm(x) * w          (stage entry)
// packed_mt > 0 writes y in the packed decode-GEMM activation layout (common.h apk_off).
//
// `rows` (optional) gathers input rows (e.g. the last token of each prompt for
// the final norm before lm_head), so the output has one row per index.
// Rounding follows HF: the normalised value is rounded to bf16 before the
// weight multiply, math in fp32, vectorised 16-B loads, one block per row.
#include "common.h"

namespace mp {

template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_kernel(
    const bf16_t* __restrict__ x, int64_t x_stride, bf16_t* __restrict__ res, int64_t res_stride,
    const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int64_t y_stride,
    const int32_t* __restrict__ rows, int H, float eps, int mode, int packed_mt) {
  __shared__ float red[16];
  const int orow = blockIdx.x;
  const int irow = rows ? rows[orow] : orow;
  const int nch = H >> 3;
  const bf16_t* xr = x + (int64_t)irow * x_stride;
  bf16_t* rr = res + (int64_t)irow * res_stride;
  // every global load (x, residual, weight) is issued before the first store and before the
  // block reduction, unconditionally (clamped chunk index: no exec-masked branches between the
  // loads): one memory round trip per call instead of three
  u16x8 v[MAXC], rv[MAXC], wv[MAXC];
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = min((int)threadIdx.x + k * 256, nch - 1);
    v[k] = *reinterpret_cast<const u16x8*>(xr + c * 8);
    rv[k] = *reinterpret_cast<const u16x8*>((mode == 1 ? rr : xr) + c * 8);
    wv[k] = *reinterpret_cast<const u16x8*>(w + c * 8);
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = threadIdx.x + k * 256;
    if (c < nch) {
      u16x8 a = v[k];
      if (mode == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = f2bf(bf2f(a[j]) + bf2f(rv[k][j]));
        *reinterpret_cast<u16x8*>(rr + c * 8) = a;
      } else if (mode == 2) {
        *reinterpret_cast<u16x8*>(rr + c * 8) = a;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f(a[j]);
        ss += f * f;
      }
      v[k] = a;
    }
  }
  const float tot = block_sum(ss, red);
  const float r = rsqrtf(tot / (float)H + eps);
  bf16_t* yr = y + (int64_t)orow * y_stride;
#pragma unroll
  for (int k = 0; k < MAXC; ++k) {
    const int c = threadIdx.x + k * 256;
    if (c < nch) {
      const u16x8 wv_ = wv[k];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(round_bf(bf2f(v[k][j]) * r) * bf2f(wv_[j]));
      if (packed_mt > 0)
        *reinterpret_cast<u16x8*>(y + apk_off(orow, c * 8, packed_mt)) = o;
      else
        *reinterpret_cast<u16x8*>(yr + c * 8) = o;
    }
  }
}

}  // namespace mp

extern "C" int mp_rmsnorm(const void* x, int64_t x_stride, void* res, int64_t res_stride, const void* w,
                          void* y, int64_t y_stride, const int32_t* rows, int nrows, int H, float eps,
                          int mode, int packed_mt, hipStream_t stream) {
  using namespace mp;
  if (H % 8 != 0 || H > 8 * 256 * 8) return -1;
  if (nrows == 0) return 0;
  const int nch = H / 8;
  dim3 grid(nrows), block(256);
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, block, 0, stream, (const bf16_t*)x, x_stride, (bf16_t*)res, res_stride,
                       (const bf16_t*)w, (bf16_t*)y, y_stride, rows, H, eps, mode, packed_mt);
  };
  if (nch <= 256) args(rmsnorm_kernel<1>);
  else if (nch <= 512) args(rmsnorm_kernel<2>);
  else if (nch <= 1024) args(rmsnorm_kernel<4>);
  else args(rmsnorm_kernel<8>);
  return (int)hipGetLastError();
}
