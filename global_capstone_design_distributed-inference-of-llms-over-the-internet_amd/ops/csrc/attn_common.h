// Device helpers of the decode attention kernels (attention.hip): DPP lane sums over a token's lane
// group, packed bf16 dot products, the fused RoPE of one 8-element chunk.
#pragma once
#include "common.h"

namespace mp {

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// Sum over groups of LPT consecutive lanes (LPT in {8, 16}); result valid in every lane.
template <int LPT>
__device__ __forceinline__ float group_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]  (xor 1)
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]  (xor 2)
  v += dpp_mov<0x141>(v);  // row_half_mirror      (8-lane total)
  if constexpr (LPT == 16) v += dpp_mov<0x140>(v);  // row_mirror (16-lane total)
  return v;
}

typedef __attribute__((ext_vector_type(4))) unsigned u32x4a;

// c + a.lo * b.lo + a.hi * b.hi over packed bf16 pairs (v_dot2c_f32_bf16: fp32 accumulate, no
// bf16 -> fp32 unpacking of either operand)
__device__ __forceinline__ float dot2bf(unsigned a, unsigned b, float c) {
  typedef __attribute__((ext_vector_type(2))) __bf16 v2bf;
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf, a), __builtin_bit_cast(v2bf, b), c, false);
}

// x * cos -/+ partner * sin for one 8-element chunk of a head (lo: the chunk is in the first
// half, its partner in the second), rounded to bf16 - the fused RoPE of the decode kernels.
__device__ __forceinline__ u16x8 rope8(u16x8 me, u16x8 ot, f32x4 ca, f32x4 cb, f32x4 sa, f32x4 sb, bool lo) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float c = j < 4 ? ca[j] : cb[j - 4], s = j < 4 ? sa[j] : sb[j - 4];
    const float x = bf2f(me[j]), y = bf2f(ot[j]);
    r[j] = lo ? f2bf(x * c - y * s) : f2bf(x * c + y * s);
  }
  return r;
}

}  // namespace mp
