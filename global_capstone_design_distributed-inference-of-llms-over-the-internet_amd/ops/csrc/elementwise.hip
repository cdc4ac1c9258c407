// Small bandwidth-bound kernels for gfx950: embedding gather (survey K1), SwiGLU
// (K10's activation, HF LlamaMLP `act(gate(x)) * up(x)`, reference
// petals/llama/block.py:237), residual add at stage exits, and greedy argmax (the
// temperature <= 0 branch of reference src/rpc_handler.py:331-336).
// All bf16 traffic is 16 B per lane.
#include "common.h"

namespace mp {

// out[t, :] = table[ids[t], :]
__global__ __launch_bounds__(256) void embedding_kernel(const int64_t* __restrict__ ids,
                                                        const bf16_t* __restrict__ table,
                                                        bf16_t* __restrict__ out, int H, int64_t vocab) {
  const int t = blockIdx.x;
  int64_t id = ids[t];
  if (id < 0 || id >= vocab) id = 0;  // never read out of bounds; host validates ids
  const u16x8* src = reinterpret_cast<const u16x8*>(table + id * H);
  u16x8* dst = reinterpret_cast<u16x8*>(out + (int64_t)t * H);
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) dst[c] = src[c];
}

// gu = [T, 2F] with gate/up columns interleaved in blocks of 16 ([g16 u16 g16 u16 ...],
// the layout the fused gate_up weight is stored in), out = [T, F];
// HF rounding: a = bf16(silu(g)); y = bf16(a * u).
__global__ __launch_bounds__(256) void swiglu_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out,
                                                     int64_t T, int F) {
  const int64_t nch = T * (F / 8);
  const int fch = F / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nch; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / fch, c = i - t * fch;
    const int64_t gcol = ((c * 8) >> 4) * 32 + ((c * 8) & 15);
    const u16x8 g = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + gcol);
    const u16x8 u = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + gcol + 16);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = bf2f(g[j]);
      const float a = round_bf(x / (1.f + __expf(-x)));
      o[j] = f2bf(a * bf2f(u[j]));
    }
    *reinterpret_cast<u16x8*>(out + t * F + c * 8) = o;
  }
}

// y = bf16(a + b)
__global__ __launch_bounds__(256) void add_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                  bf16_t* __restrict__ y, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const u16x8 x = reinterpret_cast<const u16x8*>(a)[i];
    const u16x8 z = reinterpret_cast<const u16x8*>(b)[i];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(x[j]) + bf2f(z[j]));
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

// First maximum of each row (torch.argmax tie rule). logits bf16 [R, V], row stride given.
__global__ __launch_bounds__(256) void argmax_kernel(const bf16_t* __restrict__ logits, int64_t stride, int V,
                                                     int64_t* __restrict__ out) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const bf16_t* row = logits + (int64_t)blockIdx.x * stride;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  const int nv = V / 8;
  for (int c = threadIdx.x; c < nv; c += blockDim.x) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(row + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = bf2f(v[j]);
      if (f > best) { best = f; bi = c * 8 + j; }
    }
  }
  for (int i = nv * 8 + threadIdx.x; i < V; i += blockDim.x) {
    const float f = bf2f(row[i]);
    if (f > best || (f == best && i < bi)) { best = f; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sv[w] = best; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = sv[0];
    int ix = si[0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
      if (sv[k] > b || (sv[k] == b && si[k] < ix)) { b = sv[k]; ix = si[k]; }
    out[blockIdx.x] = ix == 0x7fffffff ? 0 : ix;
  }
}

static inline int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace mp

extern "C" int mp_embedding(const int64_t* ids, const void* table, void* out, int T, int H, int64_t vocab,
                            hipStream_t stream) {
  using namespace mp;
  if (H % 8) return -1;
  if (T == 0) return 0;
  hipLaunchKernelGGL(embedding_kernel, dim3(T), dim3(256), 0, stream, ids, (const bf16_t*)table, (bf16_t*)out, H,
                     vocab);
  return (int)hipGetLastError();
}

extern "C" int mp_swiglu(const void* gu, void* out, int64_t T, int F, hipStream_t stream) {
  using namespace mp;
  if (F % 16) return -1;
  if (T == 0) return 0;
  hipLaunchKernelGGL(swiglu_kernel, dim3(grid_for(T * (F / 8))), dim3(256), 0, stream, (const bf16_t*)gu,
                     (bf16_t*)out, T, F);
  return (int)hipGetLastError();
}

extern "C" int mp_add(const void* a, const void* b, void* y, int64_t n, hipStream_t stream) {
  using namespace mp;
  if (n % 8) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(n / 8)), dim3(256), 0, stream, (const bf16_t*)a, (const bf16_t*)b,
                     (bf16_t*)y, n / 8);
  return (int)hipGetLastError();
}

extern "C" int mp_argmax(const void* logits, int64_t stride, int R, int V, int64_t* out, hipStream_t stream) {
  using namespace mp;
  if (R == 0) return 0;
  if (stride % 8) return -1;
  hipLaunchKernelGGL(argmax_kernel, dim3(R), dim3(256), 0, stream, (const bf16_t*)logits, stride, V, out);
  return (int)hipGetLastError();
}
