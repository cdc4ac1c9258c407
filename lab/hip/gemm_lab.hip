// GEMM lab: times the decode GEMM kernels of ops/csrc/gemm.hip on the Llama-2-7B decode shapes
// as a standalone HIP program (no torch), rotating over enough weight copies that the 256 MB
// Infinity Cache cannot serve repeats (the real decode step streams 6.7 GB between two uses of
// one layer's weights).
//
//   hipcc -O3 --offload-arch=gfx950 -I<ops/csrc> scripts/gemm_lab.hip -o gemm_lab [-DLAB_NO_A]
//
// -DLAB_NO_A replaces every A-fragment load by a register value (ablation: what the weight stream
// alone sustains in the same kernel structure); -DLAB_A_L1 serves every A load from one 4 KiB
// L1-resident window; -DLAB_A_LDS from a 4 KiB LDS window; -DLAB_A_NT makes the A loads
// non-temporal; -DMP_RW_WAVES=8 builds the ring kernels with 8 waves per workgroup.  Results: profiles/r1_gemm_lab.md.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <vector>

#if defined(LAB_NO_A)
#define MP_LOAD_A_FRAG(p) ((mp::u16x8)((unsigned short)(0x3c00u + (threadIdx.x & 7))))
#elif defined(LAB_A_NT)  // non-temporal A loads
#define MP_LOAD_A_FRAG(p) __builtin_nontemporal_load(reinterpret_cast<const mp::u16x8*>(p))
#elif defined(LAB_A_LDS)  // every A load reads a 4 KiB LDS window (ablation: A at LDS cost)
typedef unsigned short lab_u16x8 __attribute__((ext_vector_type(8)));
__shared__ lab_u16x8 lab_lds[256];
#define MP_LOAD_A_FRAG(p) (lab_lds[((uintptr_t)(p) >> 4) & 255])
#elif defined(LAB_A_L1)  // every A load hits the same 4 KiB (L1-resident): prices the L2->CU path
#define MP_LOAD_A_FRAG(p) (*reinterpret_cast<const mp::u16x8*>((const char*)x + (((uintptr_t)(p) - (uintptr_t)x) & 4095)))
#endif
#include "gemm.hip"
#include "gemm_wide.hip"  // 65..128-row entry point (mp_gemm_bf16 calls it)
#include "gemm_w8.hip"

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__global__ void fill_bf16(unsigned short* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const float f = ((int)(h & 0xffff) - 32768) * (1.f / 32768.f) * 0.05f;
    p[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}

static float bf_host(unsigned short u) {
  const unsigned v = (unsigned)u << 16;
  float f;
  memcpy(&f, &v, 4);
  return f;
}

struct Shape {
  const char* name;
  int N, K, epi;
};

int main(int argc, char** argv) {
  const Shape shapes[] = {{"qkv", 12288, 4096, 0},
                          {"o", 4096, 4096, 0},
                          {"gate_up", 22016, 4096, 1},
                          {"down", 4096, 11008, 0},
                          {"lm_head", 32000, 4096, 0},
                          {"whole", 32768, 4096, 0}};  // cs1: exactly one whole group per CU
  std::vector<int> Ms = {16, 32, 64};
  if (argc > 1) {
    Ms.clear();
    for (char* t = strtok(argv[1], ","); t; t = strtok(nullptr, ",")) Ms.push_back(atoi(t));
  }
  for (int M : Ms)
    if (M < 1 || M > 128) {
      fprintf(stderr, "M must be in 1..128 (buffer sizes)\n");
      return 1;
    }
  const size_t pool_bytes = (size_t)1536 << 20;
  unsigned short *pool, *x, *y;
  CK(hipMalloc(&pool, pool_bytes));
  // sized for the largest M the kernels take (128 rows) and the widest shape
  CK(hipMalloc(&x, (size_t)128 * 11008 * 2));
  CK(hipMalloc(&y, (size_t)128 * 32768 * 2));
  void* ws;
  const int64_t wsb = mp_gemm_workspace_bytes();
  CK(hipMalloc(&ws, wsb));
  CK(hipMemset(ws, 0, wsb));
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, pool, pool_bytes / 2, 1u);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, x, (size_t)128 * 11008, 7u);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  unsigned short* yref;
  CK(hipMalloc(&yref, (size_t)128 * 32768 * 2));
  std::vector<unsigned short> h0(128 * 32768), h1(128 * 32768);
  const char* kname[8] = {"pk ", "sk ", "l22", "l24", "l14", "l42", "rw ", "rwk"};
  for (const Shape& s : shapes) {
    const size_t wbytes = (size_t)s.N * s.K * 2;
    const int copies = (int)(pool_bytes / wbytes);
    const int ncols = s.epi == 1 ? s.N / 2 : s.N;
    for (int M : Ms) {
      for (int kind = 0; kind < 8; ++kind) {
        const int flags = 1 | (kind == 0 ? 8 : kind == 1 ? 4 : kind == 6 ? 128 : kind == 7 ? 256 : 16 | ((kind - 2) << 5));
        auto run = [&](int i, unsigned short* out) {
          const unsigned short* w = pool + (size_t)(i % copies) * (wbytes / 2);
          return mp_gemm_bf16(x, s.K, w, out, ncols, nullptr, 0, M, s.N, s.K, s.epi, flags, ws, nullptr, nullptr,
                              nullptr, nullptr, nullptr, 0.f, 0.f, 0);
        };
        int rc = run(0, kind == 0 ? yref : y);
        if (rc) {
          printf("%-8s M=%2d %s rc=%d\n", s.name, M, kname[kind], rc);
          continue;
        }
        CK(hipDeviceSynchronize());
        float maxd = 0.f;
        if (kind > 0) {  // same weights (copy 0) as the pk reference
          CK(hipMemcpy(h0.data(), yref, (size_t)M * ncols * 2, hipMemcpyDeviceToHost));
          CK(hipMemcpy(h1.data(), y, (size_t)M * ncols * 2, hipMemcpyDeviceToHost));
          for (size_t i = 0; i < (size_t)M * ncols; ++i) {
            const float a = bf_host(h0[i]), b = bf_host(h1[i]);
            const float d = fabsf(a - b) / (fabsf(a) + 1e-2f);
            if (!(d <= maxd)) maxd = d;  // NaN-propagating max
          }
        }
        for (int i = 1; i < 8; ++i) run(i, y);
        float best = 1e30f;
        const int iters = 60;
        for (int r = 0; r < 3; ++r) {
          CK(hipEventRecord(e0, 0));
          for (int i = 0; i < iters; ++i) run(i, y);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        const double us = best * 1000.0 / iters;
        printf("%-8s M=%2d N=%5d K=%5d %s %7.2f us %5.2f TB/s  maxrel %.3g\n", s.name, M, s.N, s.K, kname[kind], us,
               wbytes / us / 1e6, maxd);
        fflush(stdout);
      }
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
