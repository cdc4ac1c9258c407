// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this framework.
//
// Conventions used by every kernel in ops/csrc:
//   * bf16 tensors travel as raw 16-bit patterns (unsigned short); math is fp32.
//   * global loads/stores of bf16 are always vectorised (8 x bf16 = 16 B per lane),
//     the wave is 64 lanes wide, and blocks are multiples of 64 threads.
//   * every launcher takes the caller's hipStream_t so the ops are capturable
//     into hipGraphs (no allocation, no synchronisation inside a launcher).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mp {

typedef unsigned short bf16_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short s16x8;

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16_t u) {
  return __uint_as_float(((unsigned)u) << 16);
}

// Round-to-nearest-even fp32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32,
// which also keeps NaN a NaN).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// Wave-wide reductions on DPP lane moves (quad_perm, row mirrors, row_bcast15/31 - CDNA keeps
// the gfx9 row broadcasts): register-only steps.  __shfl_xor lowers to ds_bpermute, an LDS round
// trip per step, six dependent ones per 64-lane reduction.  `old` fills lanes a move leaves
// without a source (the reduction's identity).
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ unsigned dpp_u32(unsigned old, unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xF, false);
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dppf(float v, float old) {
  return __uint_as_float(dpp_u32<CTRL, ROW_MASK>(__float_as_uint(old), __float_as_uint(v)));
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ unsigned long long dpp_u64z(unsigned long long v) {  // 0 where no source
  const unsigned lo = dpp_u32<CTRL, ROW_MASK>(0u, (unsigned)v);
  const unsigned hi = dpp_u32<CTRL, ROW_MASK>(0u, (unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// every lane gets the sum / max of the wave (lane 63 collects it, then a readlane broadcast)
__device__ __forceinline__ float wave_sum(float v) {
  v += dppf<0xB1>(v, 0.f);        // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v, 0.f);        // quad_perm [2,3,0,1]
  v += dppf<0x141>(v, 0.f);       // row_half_mirror
  v += dppf<0x140>(v, 0.f);       // row_mirror: every lane of a row holds the row's sum
  v += dppf<0x142, 0xA>(v, 0.f);  // row_bcast15 into rows 1, 3
  v += dppf<0x143, 0xC>(v, 0.f);  // row_bcast31 into rows 2, 3: lane 63 holds the total
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dppf<0xB1>(v, -INFINITY));
  v = fmaxf(v, dppf<0x4E>(v, -INFINITY));
  v = fmaxf(v, dppf<0x141>(v, -INFINITY));
  v = fmaxf(v, dppf<0x140>(v, -INFINITY));
  v = fmaxf(v, dppf<0x142, 0xA>(v, -INFINITY));
  v = fmaxf(v, dppf<0x143, 0xC>(v, -INFINITY));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// workgroup barrier that waits for this wave's LDS operations only: global loads in flight (a
// register-staged stream) stay in flight across it, unlike __syncthreads()
__device__ __forceinline__ void lds_wait_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// exact integer sums (fixed-point row statistics): over the 16 lanes of each row of the wave
// (every lane gets its row's sum), and over the whole wave (every lane gets the total)
__device__ __forceinline__ unsigned long long sum16_u64(unsigned long long v) {
  v += dpp_u64z<0xB1>(v);
  v += dpp_u64z<0x4E>(v);
  v += dpp_u64z<0x141>(v);
  v += dpp_u64z<0x140>(v);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  v = sum16_u64(v);
  v += dpp_u64z<0x142, 0xA>(v);
  v += dpp_u64z<0x143, 0xC>(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), 63);
  return ((unsigned long long)hi << 32) | lo;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64). `red` needs >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Packed-activation ("fragment-native") layout shared by the decode kernels:
//   Ap[K/32][MT][64][8], MT = ceil(M/16);  lane = 16 * ((col >> 3) & 3) + (row & 15)
// i.e. exactly the A operand of v_mfma_f32_16x16x32_bf16 for k-slice col/32 and m-tile row/16,
// so the decode GEMM reads every A fragment as one contiguous 1 KiB.
__device__ __forceinline__ int64_t apk_off(int row, int col, int MT) {
  return ((((int64_t)(col >> 5) * MT + (row >> 4)) * 64 + ((col >> 3) & 3) * 16 + (row & 15)) << 3) + (col & 7);
}

// The qkv projection left as split-K partial slabs (decode GEMM flags bit 14, mp_gemm_rwk_split):
// part[s][row][col] fp32, s < S, plus the fused-norm row statistics (gemm_kernels.h EpiArgs::ss_in:
// QP_SS_NSH shards of QP_SS_ROWS rows, fixed-point sums of squares).  The decode attention kernels
// read q / k / v through qkv_part_load8, which is the split-K reduce launch's epilogue 0 inlined:
// the S slabs summed in split order from zero, times rsqrt(ss / K + eps), rounded to bf16 - the
// same bits the reduce launch would have stored, without its launch.
constexpr int QP_SS_NSH = 32, QP_SS_ROWS = 256;
constexpr float QP_SS_FX = 1048576.f;
struct QkvPart {
  const float* part;               // nullptr: read the bf16 qkv rows instead
  int S;                           // split count
  int64_t slab;                    // elements per slab (M x ldn)
  int ldn;                         // row pitch (the qkv width)
  const unsigned long long* ss;    // row statistics, or nullptr (no row scale)
  float inv_k, eps;
};

// The row scale in two halves, so a kernel can issue the shard loads early and reduce late:
// lane j < QP_SS_NSH loads shard j; every lane of the wave must call the reduction (the integer
// sum is exact in any order).
__device__ __forceinline__ unsigned long long qkv_part_ss_load(const QkvPart& qp, int row) {
  const int lane = threadIdx.x & 63;
  return (qp.ss != nullptr && lane < QP_SS_NSH) ? qp.ss[lane * QP_SS_ROWS + row] : 0ull;
}
__device__ __forceinline__ float qkv_part_ss_scale(const QkvPart& qp, unsigned long long v) {
  if (qp.ss == nullptr) return 1.f;
  return rsqrtf((float)wave_sum_u64(v) * (1.f / QP_SS_FX) * qp.inv_k + qp.eps);
}
__device__ __forceinline__ float qkv_part_scale(const QkvPart& qp, int row) {
  return qkv_part_ss_scale(qp, qkv_part_ss_load(qp, row));
}

// The S slabs' 8 columns (col .. col + 7 of ``row``), fetched and summed in two halves.  Up to
// QP_SMAX splits every slab load is issued at once (one memory round trip, not S dependent ones;
// slabs past S re-read the last one, an L2 hit, and are not added); qkv folds run S = 2 or 3.
constexpr int QP_SMAX = 4;
struct QkvPart8 {
  f32x4 a[QP_SMAX], b[QP_SMAX];
};
__device__ __forceinline__ void qkv_part_fetch8(const QkvPart& qp, int row, int col, QkvPart8& f) {
  const float* p0 = qp.part + (int64_t)row * qp.ldn + col;
#pragma unroll
  for (int s = 0; s < QP_SMAX; ++s) {
    const float* p = p0 + (int64_t)min(s, qp.S - 1) * qp.slab;
    f.a[s] = *reinterpret_cast<const f32x4*>(p);
    f.b[s] = *reinterpret_cast<const f32x4*>(p + 4);
  }
}
// bf16(sum * rs): the S slabs summed in split order from zero - the reduce launch's bits
__device__ __forceinline__ u16x8 qkv_part_finish8(const QkvPart& qp, int row, int col, const QkvPart8& f, float rs) {
  f32x4 a = (f32x4)(0.f), b = (f32x4)(0.f);
  if (qp.S <= QP_SMAX) {
#pragma unroll
    for (int s = 0; s < QP_SMAX; ++s) {
      if (s < qp.S) {  // (a select on registers: the loads are already issued)
        a += f.a[s];
        b += f.b[s];
      }
    }
  } else {
    for (int s = 0; s < qp.S; ++s) {  // more splits than the unrolled fetch holds: a plain loop
      const float* p = qp.part + s * qp.slab + (int64_t)row * qp.ldn + col;
      a += *reinterpret_cast<const f32x4*>(p);
      b += *reinterpret_cast<const f32x4*>(p + 4);
    }
  }
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = f2bf(a[j] * rs);
    r[j + 4] = f2bf(b[j] * rs);
  }
  return r;
}
__device__ __forceinline__ u16x8 qkv_part_load8(const QkvPart& qp, int row, int col, float rs) {
  QkvPart8 f;
  qkv_part_fetch8(qp, row, col, f);
  return qkv_part_finish8(qp, row, col, f, rs);
}

}  // namespace mp
