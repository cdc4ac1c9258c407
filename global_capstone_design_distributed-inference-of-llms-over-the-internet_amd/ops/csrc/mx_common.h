// MX (e4m3 + e8m0 per 32-element block) helpers shared by the W8A8-MX GEMM's activation quantizer
// (gemm_mx.hip) and the producers that write its activation directly (attention_mfma.hip).
// Layout (gemm_mx.hip header): Ax[K/128][MT][2][64][16] e4m3 (row r = 16 mt + (l & 15) of lane l,
// byte 8 s + j of lane 16 q + r = k-slice s, column 8 q + j of the 128-deep step; byte b of 16 at
// half b >> 4), As[K/128][64][4] e8m0 (byte mt of lane 16 blk + r; blk = 2 (s >> 1) + (q >> 1)).
#pragma once
#include "common.h"

namespace mp {

// e8m0 exponent (biased 127) of the smallest power-of-two scale s with amax / s <= 448 (e4m3 max)
__device__ __forceinline__ int mx_e8m0(float amax) {
  if (!(amax > 0.f)) return 127;
  const unsigned b = __float_as_uint(amax * (1.f / 448.f));
  const int ex = (int)((b >> 23) & 255);
  int e = ex + ((b & 0x7fffff) != 0 ? 1 : 0);  // ceil(log2) + 127 (normal range)
  return e < 1 ? 1 : (e > 253 ? 253 : e);
}

__device__ __forceinline__ float mx_inv_scale(int e) { return __uint_as_float((unsigned)(254 - e) << 23); }

// byte offset of element (row, col) in Ax, and of its block's scale in As
__device__ __forceinline__ int64_t mx_ax_off(int row, int col, int MT) {
  const int kb = col >> 7, s = (col >> 5) & 3, q = (col >> 3) & 3, j = col & 7;
  return (((int64_t)kb * MT + (row >> 4)) * 2 + (s >> 1)) * 1024 + (16 * q + (row & 15)) * 16 + 8 * (s & 1) + j;
}
__device__ __forceinline__ int64_t mx_as_off(int row, int col) {
  const int kb = col >> 7, blk = 2 * ((col >> 6) & 1) + ((col >> 4) & 1);
  return ((int64_t)kb * 64 + 16 * blk + (row & 15)) * 4 + (row >> 4);
}

}  // namespace mp
