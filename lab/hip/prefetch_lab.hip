// Prefetch lab: can the narrow decode projections (o: 4096 x 4096, down: 4096 x 11008, M = 64)
// run faster when their weights were read into the Infinity Cache while the attention kernel was
// still streaming the KV cache?  Per shape and form, four timings (us per projection):
//   cold     rotated weight copies (no cache reuse), the in-situ case today
//   warm     the same copy every call (weights resident in L2 / MALL): the ceiling of a prefetch
//   stream   a stand-in attention: one full-chip streaming read of `kv_mb` MB, then the projection
//            on cold weights (what a decode layer does today)
//   overlap  the same streaming read with a prefetch of the projection's weights on a second
//            stream (event fork / join), then the projection
// (overlap - stream) is what a prefetch buys per layer.
//
//   hipcc -O3 --offload-arch=gfx950 -I<ops/csrc> scripts/prefetch_lab.hip -o prefetch_lab && ./prefetch_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "gemm.hip"
#include "gemm_w8.hip"
#include "gemm_wide.hip"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void fill_bf16(unsigned short* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const float f = ((int)(h & 0xffff) - 32768) * (1.f / 32768.f) * scale;
    p[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}

// streaming read (stand-in attention when POL = 0, prefetch otherwise); the xor keeps the loads
// alive and is written only for an impossible value
template <int POL>
__global__ __launch_bounds__(256) void stream_read(const uint4* __restrict__ p, size_t n, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int M = 64;
  const size_t kv_mb = argc > 1 ? atoi(argv[1]) : 178;
  const int pf_groups = argc > 2 ? atoi(argv[2]) : 32;
  struct Shape {
    const char* name;
    int N, K, epi, flags;
  };
  const Shape shapes[] = {{"o rwr", 4096, 4096, 3, 4096},   {"o rwr+t", 4096, 4096, 3, 4096 | 8192},
                          {"o pk", 4096, 4096, 3, 8},       {"down rwk", 4096, 11008, 3, 256},
                          {"down rwk+r", 4096, 11008, 3, 256 | 1024}};
  const size_t pool_bytes = (size_t)1536 << 20;
  unsigned short *pool, *x, *res, *ap, *kv;
  unsigned* sink;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMalloc(&kv, kv_mb << 20));
  CK(hipMalloc(&sink, 4096));
  CK(hipMalloc(&x, (size_t)M * 11008 * 2));
  CK(hipMalloc(&res, (size_t)M * 4096 * 2));
  CK(hipMalloc(&ap, (size_t)M * 11008 * 2));
  const int ssn = mp_gemm_ss_elems();
  unsigned long long *ss, *ss2;
  CK(hipMalloc(&ss, ssn * 8));
  CK(hipMalloc(&ss2, ssn * 8));
  void* ws;
  const int64_t wsb = mp_gemm_workspace_bytes();
  CK(hipMalloc(&ws, wsb));
  CK(hipMemset(ws, 0, wsb));
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, pool, pool_bytes / 2, 1u, 0.05f);
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, kv, (kv_mb << 20) / 2, 3u, 0.05f);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, x, (size_t)M * 11008, 7u, 1.0f);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, res, (size_t)M * 4096, 9u, 1.0f);
  CK(hipMemset(ss, 0, ssn * 8));
  CK(hipDeviceSynchronize());
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1, fork, join;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  for (const Shape& s : shapes) {
    const size_t wbytes = (size_t)s.N * s.K * 2;
    const int copies = (int)(pool_bytes / wbytes);
    auto gemm = [&](int i) {
      const unsigned short* w = pool + (size_t)(i % copies) * (wbytes / 2);
      return mp_gemm_bf16(x, s.K, w, res, s.N, res, s.N, M, s.N, s.K, s.epi, 1 | s.flags, ws, nullptr, ap, ss, ss2,
                          nullptr, 1.f / s.K, 1e-5f, s0);
    };
    auto attn = [&]() {
      hipLaunchKernelGGL(stream_read<0>, dim3(2048), dim3(256), 0, s0, (const uint4*)kv, (kv_mb << 20) / 16, sink);
    };
    auto prefetch = [&](int i) {
      const unsigned short* w = pool + (size_t)(i % copies) * (wbytes / 2);
      hipLaunchKernelGGL(stream_read<1>, dim3(pf_groups), dim3(256), 0, s1, (const uint4*)w, wbytes / 16, sink);
    };
    if (gemm(0)) {
      printf("%-11s rc != 0 (form not built)\n", s.name);
      continue;
    }
    const int iters = 40;
    float t[5];
    for (int mode = 0; mode < 5; ++mode) {
      float best = 1e30f;
      for (int r = 0; r < 3; ++r) {
        CK(hipStreamSynchronize(s0));
        CK(hipEventRecord(e0, s0));
        for (int i = 1; i <= iters; ++i) {
          if (mode == 0) gemm(i);
          if (mode == 1) gemm(0);
          if (mode == 2) { attn(); gemm(i); }
          if (mode == 3) {
            CK(hipEventRecord(fork, s0));
            CK(hipStreamWaitEvent(s1, fork, 0));
            attn();
            prefetch(i);
            CK(hipEventRecord(join, s1));
            CK(hipStreamWaitEvent(s0, join, 0));
            gemm(i);
          }
          if (mode == 4) attn();
        }
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      t[mode] = best * 1000.f / iters;
    }
    printf("%-11s cold %6.2f  warm %6.2f  attn %6.2f  attn+gemm %6.2f  attn||prefetch+gemm %6.2f  gain %6.2f us  (kv %zu MB, prefetch groups %d)\n",
           s.name, t[0], t[1], t[4], t[2], t[3], t[2] - t[3], kv_mb, pf_groups);
    fflush(stdout);
  }
  CK(hipDeviceSynchronize());
  printf("PREFETCH_LAB OK\n");
  return 0;
}
