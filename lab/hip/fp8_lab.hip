// fp8 GEMM lab: times the fp8 decode GEMMs of ops/csrc/fp8.hip on the Llama-3-70B decode shapes
// (M = 64) as a standalone HIP program, weights rotated over a 2 GB pool (cold Infinity Cache).
//
//   hipcc -O3 --offload-arch=gfx950 -I<ops/csrc> scripts/fp8_lab.hip -o fp8_lab [-DLAB_NO_A]
//
// -DLAB_NO_A replaces the balanced-ring kernel's A-fragment loads by a register value (what the
// weight stream alone sustains in the same structure).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#if defined(LAB_NO_A)
#define MP_F8_LOAD_A(p) ((mp::u16x8)((unsigned short)(0x3838u + (threadIdx.x & 7))))
#endif
#include "fp8.hip"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void fill_u8(unsigned char* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13;
    p[i] = (unsigned char)((h & 0x77u) | ((h >> 8) & 0x80u));  // finite e4m3 codes
  }
}

struct Shape {
  const char* name;
  int N, K, epi;
};

int main() {
  const Shape shapes[] = {{"qkv", 10240, 8192, 0}, {"o", 8192, 8192, 0}, {"gate_up", 57344, 8192, 1},
                          {"down", 8192, 28672, 0}};
  const int M = 64;
  const size_t pool_bytes = (size_t)2048 << 20;
  unsigned char *pool, *a8;
  float *ws, *as;
  unsigned short* y;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMalloc(&a8, (size_t)64 * 28672));
  CK(hipMalloc(&ws, (size_t)57344 * 4));
  CK(hipMalloc(&as, 64 * 4));
  CK(hipMalloc(&y, (size_t)64 * 57344 * 2));
  float* part;
  CK(hipMalloc(&part, (size_t)16 << 20));
  hipLaunchKernelGGL(fill_u8, dim3(4096), dim3(256), 0, 0, pool, pool_bytes, 1u);
  hipLaunchKernelGGL(fill_u8, dim3(1024), dim3(256), 0, 0, a8, (size_t)64 * 28672, 7u);
  std::vector<float> one(57344, 1e-3f);
  CK(hipMemcpy(ws, one.data(), one.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(as, one.data(), 64 * 4, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : shapes) {
    const size_t wbytes = (size_t)s.N * s.K;
    const int copies = (int)(pool_bytes / wbytes);
    for (int kind = 0; kind < 3; ++kind) {
      auto run = [&](int i) {
        return mp_gemm_fp8(a8, as, pool + (size_t)(i % copies) * wbytes, ws, y, s.epi == 1 ? s.N / 2 : s.N, nullptr,
                           0, M, s.N, s.K, s.epi, 0, kind, part, (int64_t)16 << 20, 0);
      };
      if (int rc = run(0)) {
        printf("%-8s rc=%d\n", s.name, rc);
        continue;
      }
      for (int i = 1; i < 6; ++i) run(i);
      float best = 1e30f;
      const int iters = 30;
      for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) run(i);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
      }
      const double us = best * 1000.0 / iters;
      printf("%-8s M=%d N=%5d K=%5d %s %7.2f us %5.2f TB/s\n", s.name, M, s.N, s.K, kind == 2 ? "rwk" : kind ? "rw " : "pk ", us,
             wbytes / us / 1e6);
      fflush(stdout);
    }
  }
  return 0;
}
