// rg lab: the LDS-DMA ring decode GEMM (ops/csrc/gemm_glds.h) against the kernels the decode step
// uses today at each Llama-2-7B projection shape, on rotated weight copies (no Infinity-Cache
// reuse between launches), with the fused epilogues the executor uses: qkv = epilogue 0 with the
// fused-norm row scale, gate/up = SwiGLU with packed output, o / down = the residual-stream
// producer (epilogue 3).  Each new form is checked against the current kernel (relative tolerance:
// the k summation order differs) and timed as 60 back-to-back launches (best of 3), so each time
// includes its kernel boundary - and for the split forms the reduce launch.
//
//   hipcc -O3 --offload-arch=gfx950 -I<ops/csrc> scripts/rg_lab.hip -o rg_lab && ./rg_lab [Ms]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "gemm.hip"
#include "gemm_glds_lab.h"
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

__global__ void fill_ss(unsigned long long* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (unsigned long long)(1048576.0 * 4096.0 * 0.33 / 32.0) + (unsigned long long)(i % 7) * 1000ull;
}

static float bf_host(unsigned short u) {
  const unsigned v = (unsigned)u << 16;
  float f;
  memcpy(&f, &v, 4);
  return f;
}

int main(int argc, char** argv) {
  struct Shape {
    const char* name;
    int N, K, epi, base_flags;  // base_flags: the decode step's kernel choice today (BENCH_r04)
  };
  const Shape shapes[] = {{"qkv", 12288, 4096, 0, 1 | 128},
                          {"gateup", 22016, 4096, 1, 1 | 2 | 128},
                          {"o", 4096, 4096, 3, 1 | 4096},
                          {"down", 4096, 11008, 3, 1 | 256 | 1024}};
  std::vector<int> Ms = {64};
  if (argc > 1) {
    Ms.clear();
    for (char* t = strtok(argv[1], ","); t; t = strtok(nullptr, ",")) Ms.push_back(atoi(t));
  }
  const size_t pool_bytes = (size_t)2048 << 20;
  unsigned short *pool, *x, *res, *res0, *ap, *yb, *yn;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMalloc(&x, (size_t)64 * 11008 * 2));
  CK(hipMalloc(&res, (size_t)64 * 22016 * 2));
  CK(hipMalloc(&res0, (size_t)64 * 22016 * 2));
  CK(hipMalloc(&yb, (size_t)64 * 22016 * 2));
  CK(hipMalloc(&yn, (size_t)64 * 22016 * 2));
  CK(hipMalloc(&ap, (size_t)64 * 22016 * 2));
  const int ssn = mp_gemm_ss_elems();
  unsigned long long *ss_in, *ss, *ss2;
  CK(hipMalloc(&ss_in, ssn * 8));
  CK(hipMalloc(&ss, ssn * 8));
  CK(hipMalloc(&ss2, ssn * 8));
  void* ws;
  const int64_t wsb = mp_gemm_workspace_bytes();
  CK(hipMalloc(&ws, wsb));
  CK(hipMemset(ws, 0, wsb));
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, pool, pool_bytes / 2, 1u, 0.05f);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, x, (size_t)64 * 11008, 7u, 1.0f);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, res0, (size_t)64 * 22016, 9u, 1.0f);
  hipLaunchKernelGGL(fill_ss, dim3((ssn + 255) / 256), dim3(256), 0, 0, ss_in, ssn);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned short> hb(64 * 22016), hn(64 * 22016);
  int bad = 0;
  for (const Shape& s : shapes) {
    const size_t wbytes = (size_t)s.N * s.K * 2;
    const int copies = (int)(pool_bytes / wbytes);
    const int Nout = s.epi == 1 ? s.N / 2 : s.N;
    for (int M : Ms) {
      const size_t ny = (size_t)M * Nout;
      const int MT = (M + 15) / 16;
      mp::EpiArgs ep{(mp::bf16_t*)ap, (mp::u64*)ss, (mp::u64*)ss2, s.epi < 2 ? (const mp::u64*)ss_in : nullptr,
                     1.f / s.K, 1e-5f, MT};
      // variant -1: today's kernel; v >= 0: rg with K split S = v (0 -> 1)
      const int splits[] = {-1, 1, 2, 4};
      for (int S : splits) {
        if (S > 1 && s.epi == 1) continue;
        unsigned short* y = s.epi == 3 ? res : (S < 0 ? yb : yn);
        auto run = [&](int i) -> int {
          const unsigned short* w = pool + (size_t)(i % copies) * (wbytes / 2);
          if (S < 0)
            return mp_gemm_bf16(x, s.K, w, y, Nout, s.epi == 3 ? res : nullptr, s.N, M, s.N, s.K, s.epi, s.base_flags,
                                ws, nullptr, ap, ss, ss2, s.epi < 2 ? ss_in : nullptr, 1.f / s.K, 1e-5f, 0);
          const int fl = (s.epi == 1 ? 2 : 0) | (S > 1 ? (S << 16) : 0);
          int rc;
          switch (MT) {
            case 1: rc = mp::launch_gemm_rg<1>(x, w, y, Nout, s.epi == 3 ? res : nullptr, s.N, M, s.N, s.K, s.epi, fl, ep, ws, 0); break;
            case 2: rc = mp::launch_gemm_rg<2>(x, w, y, Nout, s.epi == 3 ? res : nullptr, s.N, M, s.N, s.K, s.epi, fl, ep, ws, 0); break;
            case 3: rc = mp::launch_gemm_rg<3>(x, w, y, Nout, s.epi == 3 ? res : nullptr, s.N, M, s.N, s.K, s.epi, fl, ep, ws, 0); break;
            default: rc = mp::launch_gemm_rg<4>(x, w, y, Nout, s.epi == 3 ? res : nullptr, s.N, M, s.N, s.K, s.epi, fl, ep, ws, 0); break;
          }
          return rc;
        };
        CK(hipMemcpy(res, res0, (size_t)64 * 22016 * 2, hipMemcpyDeviceToDevice));
        CK(hipMemset(ss, 0, ssn * 8));
        CK(hipMemset(ap, 0, (size_t)64 * 22016 * 2));
        int rc = run(0);
        if (rc) {
          printf("%-6s M=%2d S=%2d rc=%d\n", s.name, M, S, rc);
          continue;
        }
        CK(hipDeviceSynchronize());
        float maxd = 0.f;
        if (S < 0) {
          CK(hipMemcpy(hb.data(), y, ny * 2, hipMemcpyDeviceToHost));
        } else {
          CK(hipMemcpy(hn.data(), y, ny * 2, hipMemcpyDeviceToHost));
          for (size_t i = 0; i < ny; ++i) {
            const float a = bf_host(hb[i]), b = bf_host(hn[i]);
            const float d = fabsf(a - b) / (fabsf(a) + 2e-2f);
            if (!(d <= maxd)) maxd = d;
          }
          if (!(maxd < 0.05f)) bad = 1;
        }
        for (int i = 1; i < 8; ++i) run(i);
        float best = 1e30f;
        const int iters = 60;
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
        printf("%-6s M=%2d N=%5d K=%5d %-8s S=%d %7.2f us %5.2f TB/s  maxrel_vs_today %.3g\n", s.name, M, s.N, s.K,
               S < 0 ? "today" : "rg", S < 0 ? 0 : S, us, wbytes / us / 1e6, maxd);
        fflush(stdout);
      }
    }
  }
  CK(hipDeviceSynchronize());
  printf(bad ? "RG_LAB FAIL\n" : "RG_LAB OK\n");
  return 0;
}
