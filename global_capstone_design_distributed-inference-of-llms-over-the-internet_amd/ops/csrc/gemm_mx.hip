// W8A8-MX decode GEMM for gfx950: e4m3 weights (the W8A16 ring kernels' fp8 weights, unchanged) x
// e4m3 activations with e8m0 scales per 32-element block, on the CDNA4 block-scaled MFMA
// v_mfma_scale_f32_16x16x128_f8f6f4 - BASELINE config 5's "fp8 MFMA path" with the activation
// scale local to a block, so no row-wide absmax (the W8A8 path of fp8.hip needs one, i.e. two
// launches or a one-workgroup-per-row pass) and no per-element conversion in the GEMM.
// Reference: the upstream server's quantized default (NF4 on CUDA, petals/server/server.py:189-190)
// applies to the same projections (petals/llama/block.py:88-90 q / k / v, :151 o); here 8-bit
// weights and, in this mode, 8-bit activations go through the matrix cores directly.
//
// Fragment / scale map of the instruction (lab/hip/mx_probe*.hip, measured): lane l = 16 q + r of
// the A operand holds row r, byte j at k = 16 q + j (j < 16) and k = 64 + 16 q + j - 16 (j >= 16) of
// its 128-deep k-step; B likewise with column c = l & 15; the e8m0 scale of 32-block b = k / 32 of
// row r is taken from lane 16 b + r.  A and B may permute k identically without changing the
// product, so the GEMM feeds the weights in the W8A16 byte order (lane q, byte 8 s + j = k-slice
// 4 kb + s, column 8 q + j of that slice) and the activation in the same order; a hardware block b
// then covers lanes q = 2 (b & 1), 2 (b & 1) + 1 at bytes 16 (b >> 1) .. + 15, i.e. k-slices
// 4 kb + 2 (b >> 1) + {0, 1}, columns 16 (b & 1) .. + 15 of each - two runs of 16 consecutive k.
// mx_quant_kernel scales exactly those blocks and stores block b's scale where lane 16 b + r reads it.
//
//   Ax[K/128][MT][2][64][16]  e4m3  (bytes 16 h .. 16 h + 15 of lane l at [h][l]: each of the GEMM's two
//                                   16-B loads reads one contiguous KiB; rows >= M: zero bytes)
//   As[K/128][64][4]          e8m0  (byte mt of lane l's word: the scale lane l supplies for row
//                                   tile mt - one dword load per k-step; rows >= M: 127 = 1.0)
//
// The GEMM itself is the split-K ring kernel of gemm_kernels.h with MX = true (fp32 partial slabs,
// weight column scales after the loop) + the shared reduce launch and epilogues (row scale of the
// fused-norm consumer, residual-stream producer) - or partial slabs only for the qkv fold.
#include "gemm_kernels.h"
#include "mx_common.h"

namespace mp {

// One thread per (k-step kb, row tile mt, row r): reads the row's 128 values of the step (16 x 16 B
// of the packed bf16 activation), the four block maxima, writes the four lanes' 32 bytes and the
// four block scales.
__global__ __launch_bounds__(256) void mx_quant_kernel(const bf16_t* __restrict__ ap, uint8_t* __restrict__ ax,
                                                       uint8_t* __restrict__ as, int M, int MT, int nkb) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int r = idx & 15, pair = idx >> 4;
  if (pair >= nkb * MT) return;
  const int kb = pair / MT, mt = pair - kb * MT;
  const bool ok = mt * 16 + r < M;
  u16x8 v[4][4];  // [s][q]
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[s][q] = ok ? *reinterpret_cast<const u16x8*>(ap + ((((int64_t)(4 * kb + s) * MT + mt) * 64) + 16 * q + r) * 8)
                   : (u16x8)(0);
  float amax[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int b = 2 * (s >> 1) + (q >> 1);
        amax[b] = fmaxf(amax[b], fabsf(bf2f(v[s][q][j])));
      }
  float inv[4];
  int e[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    e[b] = mx_e8m0(amax[b]);
    inv[b] = __uint_as_float((unsigned)(254 - e[b]) << 23);  // 2^(127 - e)
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned w[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float sc = inv[2 * (s >> 1) + (q >> 1)];
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(bf2f(v[s][q][j]) * sc, -448.f), 448.f);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
      w[2 * s] = (unsigned)lo;
      w[2 * s + 1] = (unsigned)hi;
    }
    uint8_t* dst = ax + (int64_t)pair * 2048 + (16 * q + r) * 16;
    *reinterpret_cast<u32x4*>(dst) = (u32x4){w[0], w[1], w[2], w[3]};
    *reinterpret_cast<u32x4*>(dst + 1024) = (u32x4){w[4], w[5], w[6], w[7]};
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) as[((int64_t)kb * 64 + 16 * b + r) * 4 + mt] = (uint8_t)e[b];
}

}  // namespace mp

// Packed bf16 activation ap (M rows, K) -> MX e4m3 bytes ax [K/128][MT][2][64][16] + e8m0 scales
// as [K/128][64][4].
extern "C" int mp_quant_mx(const void* ap, void* ax, void* as, int M, int K, hipStream_t stream) {
  using namespace mp;
  if (M <= 0) return 0;
  if (K % 128) return -1;
  const int MT = (M + 15) / 16, nkb = K / 128;
  const int threads = nkb * MT * 16;
  hipLaunchKernelGGL(mx_quant_kernel, dim3((threads + 255) / 256), dim3(256), 0, stream, (const bf16_t*)ap,
                     (uint8_t*)ax, (uint8_t*)as, M, MT, nkb);
  return (int)hipGetLastError();
}

// MX activation (mp_quant_mx) x fp8 weight (W8A16 layout + column scales), M <= 64: the split-K
// ring kernel + reduce launch (epilogue 0 with the optional ss_in row scale, or 3), or partial
// slabs only (flags bit 14, the qkv fold).  Returns 1 when the shape has no split-K geometry.
extern "C" int mp_gemm_mx(const void* ax, const void* as, const void* wq, const float* wsc, void* y, int64_t y_stride,
                          const void* res, int64_t res_stride, int M, int N, int K, int epilogue, int flags, void* ws,
                          void* ap, void* ss_out, void* ss_zero, const void* ss_in, float inv_k, float eps,
                          hipStream_t stream) {
  (void)hipGetLastError();
  using namespace mp;
  if (M == 0) return 0;
  if (M > 64 || K % 128 || N % 16 || wsc == nullptr || as == nullptr || ws == nullptr) return -1;
  if (epilogue != 0 && epilogue != 3) return -2;
  if (epilogue == 3 && (ap == nullptr || res == nullptr)) return -5;
  EpiArgs ep{(bf16_t*)ap, (u64*)ss_out, (u64*)ss_zero, (const u64*)ss_in, inv_k, eps, (M + 15) / 16};
  ep.wsc = wsc;
  ep.rot = (flags >> 10) & 1;
  ep.xsc = (const uint8_t*)as;
  const int comb = (flags & 16384) ? -1 : 0;
  int rc;
  switch ((M + 15) / 16) {
    case 1: rc = launch_gemm_rwk<1, true, true>(ax, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, comb); break;
    case 2: rc = launch_gemm_rwk<2, true, true>(ax, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, comb); break;
    case 3: rc = launch_gemm_rwk<3, true, true>(ax, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, comb); break;
    default: rc = launch_gemm_rwk<4, true, true>(ax, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, comb); break;
  }
  if (rc != 0) return rc;
  return (int)hipGetLastError();
}
