// Weight-streaming skinny GEMM for decode on gfx950 (survey K3/K8/K10/K12).
//
//   y[M, N'] = epilogue( x[M, K] . W[N, K]^T )        M <= 64 (decode micro-batches)
//
// The reference runs q/k/v/o/gate/up/down/lm_head as separate cuBLAS GEMV/GEMMs
// (reference petals/llama/block.py:88-90, :151, :237; src/llama_partition.py:470) and does
// the SwiGLU product and residual adds as further elementwise kernels.  At decode sizes the
// projections are bound by streaming W from HBM once, so this kernel is organised around
// that stream:
//
//   * MFMA v_mfma_f32_16x16x32_bf16, W as the B operand straight from HBM to VGPRs (no LDS
//     round trip: guide "GEMV / M <= 16" row), x as the A operand (L1/L2-resident).
//   * K-permuted fragments: within a 256-deep chunk, lane (c = l&15, q = l>>4) of MFMA i
//     holds k = 64q + 8i + j for both operands, so every lane reads 128 contiguous bytes
//     of one W row (eight 16-B loads in flight per lane) instead of 16-B pieces of 16 rows.
//   * one workgroup = 8 waves = NCT column tiles (16 cols each) x (8/NCT) K-slices; the
//     K-slices are combined through LDS inside the workgroup (no atomics, no second pass).
//   * fused epilogues: 0 = store bf16; 1 = SwiGLU for a gate/up weight stored as
//     16-row interleaved [g(16) u(16) g(16) u(16) ...] (output N/2 columns);
//     2 = y = bf16(bf16(acc) + residual).
// Grid: one workgroup per (16 * NCT)-column slab of W -> N/16 (or N/32) workgroups, i.e.
// 256-1376 workgroups x 8 waves for Llama-2-7B projections.
#include "common.h"

namespace mp {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                  0, 0, 0);
}

template <int MT, int NCT, int EPI>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(const bf16_t* __restrict__ x, int64_t x_stride,
                                                          const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                          int64_t y_stride, const bf16_t* __restrict__ res,
                                                          int64_t res_stride, int M, int N, int K) {
  constexpr int NKS = 8 / NCT;  // K-slices per workgroup
  __shared__ __attribute__((aligned(16))) float red[8][MT * 4][64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ct = wid % NCT, ks = wid / NCT;
  const int c = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * (16 * NCT) + ct * 16;
  const bf16_t* wrow = w + (int64_t)(n0 + c) * K + 64 * q;
  const int nchunks = K >> 8;

  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (f32x4)(0.f);

  // x rows this lane feeds (A operand row = lane & 15 within each 16-row tile)
  const bf16_t* xrow[MT];
  bool xok[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int r = mt * 16 + c;
    xok[mt] = r < M;
    xrow[mt] = x + (int64_t)(xok[mt] ? r : 0) * x_stride + 64 * q;
  }

  int ch = ks;
  u16x8 b[8];
  if (ch < nchunks) {
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wrow + (ch << 8) + 8 * i));
  }
  for (; ch < nchunks; ch += NKS) {
    const int nxt = ch + NKS;
    u16x8 bn[8];
    if (nxt < nchunks) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        bn[i] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wrow + (nxt << 8) + 8 * i));
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      u16x8 a[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        a[i] = xok[mt] ? *reinterpret_cast<const u16x8*>(xrow[mt] + (ch << 8) + 8 * i) : (u16x8)(0);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[mt] = mfma16(a[i], b[i], acc[mt]);
    }
    if (nxt < nchunks) {
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = bn[i];
    }
  }

  // ---- combine the K-slices through LDS ----
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][mt * 4 + r][lane] = acc[mt][r];
  __syncthreads();
  if (ks != 0) return;
  float sum[MT * 4];
#pragma unroll
  for (int i = 0; i < MT * 4; ++i) {
    float s = 0.f;
#pragma unroll
    for (int k2 = 0; k2 < NKS; ++k2) s += red[k2 * NCT + ct][i][lane];
    sum[i] = s;
  }
  if constexpr (EPI == 1) {
    // wave ct==0 holds the gate tile, ct==1 the matching up tile
    if (ct != 0) return;
    const int ncol = blockIdx.x * 16 + c;  // output column (N/2 wide)
#pragma unroll
    for (int i = 0; i < MT * 4; ++i) {
      float up = 0.f;
#pragma unroll
      for (int k2 = 0; k2 < NKS; ++k2) up += red[k2 * NCT + 1][i][lane];
      const int row = (i >> 2) * 16 + q * 4 + (i & 3);
      if (row < M) {
        const float g = round_bf(sum[i]);
        const float a = round_bf(g / (1.f + __expf(-g)));
        y[(int64_t)row * y_stride + ncol] = f2bf(a * round_bf(up));
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < MT * 4; ++i) {
      const int row = (i >> 2) * 16 + q * 4 + (i & 3);
      if (row < M) {
        float v = sum[i];
        if constexpr (EPI == 2) v = round_bf(v) + bf2f(res[(int64_t)row * res_stride + n0 + c]);
        y[(int64_t)row * y_stride + n0 + c] = f2bf(v);
      }
    }
  }
}

template <int MT>
static int launch_gemm(const void* x, int64_t xs, const void* w, void* y, int64_t ys, const void* res, int64_t rs,
                       int M, int N, int K, int epi, hipStream_t stream) {
  if (epi == 1) {
    if (N % 32) return -2;
    hipLaunchKernelGGL((gemm_skinny_kernel<MT, 2, 1>), dim3(N / 32), dim3(512), 0, stream, (const bf16_t*)x, xs,
                       (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K);
  } else if (epi == 2) {
    hipLaunchKernelGGL((gemm_skinny_kernel<MT, 1, 2>), dim3(N / 16), dim3(512), 0, stream, (const bf16_t*)x, xs,
                       (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K);
  } else {
    hipLaunchKernelGGL((gemm_skinny_kernel<MT, 1, 0>), dim3(N / 16), dim3(512), 0, stream, (const bf16_t*)x, xs,
                       (const bf16_t*)w, (bf16_t*)y, ys, (const bf16_t*)res, rs, M, N, K);
  }
  return 0;
}

}  // namespace mp

extern "C" int mp_gemm_bf16(const void* x, int64_t x_stride, const void* w, void* y, int64_t y_stride,
                            const void* res, int64_t res_stride, int M, int N, int K, int epilogue,
                            hipStream_t stream) {
  using namespace mp;
  if (M == 0) return 0;
  if (M > 64 || K % 256 || N % 16 || x_stride % 8) return -1;
  int rc;
  if (M <= 16) rc = launch_gemm<1>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, stream);
  else if (M <= 32) rc = launch_gemm<2>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, stream);
  else if (M <= 48) rc = launch_gemm<3>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, stream);
  else rc = launch_gemm<4>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, stream);
  if (rc) return rc;
  return (int)hipGetLastError();
}
