// Seam lab: the narrow decode projections (o: 4096 x 4096, down: 4096 x 11008) with the fused-norm
// producer epilogue (EPI 3: residual add in place, packed copy, fixed-point row sums of squares)
// in every form that can carry it - one-group (pk), split-K ring + reduce launch (rwk), split-K
// ring with the last-arriver combine (rwki) or the symmetric combine (rwks), row-split ring (rwr,
// rwrt = default-policy weight loads) - timed over rotated weight copies (no Infinity Cache
// reuse), each checked against the reduce-launch form (bitwise for the in-launch combines, which
// sum in the same order) and pk (tolerance).
//
//   hipcc -O3 --offload-arch=gfx950 -I<ops/csrc> scripts/seam_lab.hip -o seam_lab && ./seam_lab [Ms]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

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

static float bf_host(unsigned short u) {
  const unsigned v = (unsigned)u << 16;
  float f;
  memcpy(&f, &v, 4);
  return f;
}

struct Kind {
  const char* name;
  int flags;
};

int main(int argc, char** argv) {
  struct Shape {
    const char* name;
    int N, K, epi;
  };
  const Shape shapes[] = {{"o", 4096, 4096, 3}, {"down", 4096, 11008, 3}, {"o_e0", 4096, 4096, 0},
                          {"qkv", 12288, 4096, 0}};
  std::vector<int> Ms = {32, 64};
  if (argc > 1) {
    Ms.clear();
    for (char* t = strtok(argv[1], ","); t; t = strtok(nullptr, ",")) Ms.push_back(atoi(t));
  }
  const Kind kinds[] = {{"pk", 8}, {"rw", 128}, {"rw+r", 128 | 1024}, {"rwkp", 256 | 16384},          {"pk+r", 8 | 1024},     {"rwk", 256},           {"rwk+r", 256 | 1024},
                        {"rwki", 256 | 512}, {"rwki+r", 256 | 512 | 1024}, {"rwks", 256 | 2048},
                        {"rwks+r", 256 | 2048 | 1024}, {"rwr", 4096}, {"rwr+r", 4096 | 1024},
                        {"rwrt", 4096 | 8192}, {"rwrt+r", 4096 | 8192 | 1024}};
  const int nkinds = sizeof(kinds) / sizeof(kinds[0]);
  const size_t pool_bytes = (size_t)1536 << 20;
  unsigned short *pool, *x, *res, *res0, *ap, *yref, *apref;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMalloc(&x, (size_t)64 * 11008 * 2));
  CK(hipMalloc(&res, (size_t)64 * 12288 * 2));
  CK(hipMalloc(&res0, (size_t)64 * 12288 * 2));
  CK(hipMalloc(&yref, (size_t)64 * 12288 * 2));
  CK(hipMalloc(&ap, (size_t)64 * 12288 * 2));
  CK(hipMalloc(&apref, (size_t)64 * 12288 * 2));
  const int ssn = mp_gemm_ss_elems();
  unsigned long long *ss, *ss2, *ssref;
  CK(hipMalloc(&ss, ssn * 8));
  CK(hipMalloc(&ss2, ssn * 8));
  CK(hipMalloc(&ssref, ssn * 8));
  void* ws;
  const int64_t wsb = mp_gemm_workspace_bytes();
  CK(hipMalloc(&ws, wsb));
  CK(hipMemset(ws, 0, wsb));
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, pool, pool_bytes / 2, 1u, 0.05f);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, x, (size_t)64 * 11008, 7u, 1.0f);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, res0, (size_t)64 * 4096, 9u, 1.0f);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned short> h0(64 * 12288), h1(64 * 12288);
  std::vector<unsigned long long> s0(ssn), s1(ssn);
  int bad = 0;
  for (const Shape& s : shapes) {
    const size_t wbytes = (size_t)s.N * s.K * 2;
    const int copies = (int)(pool_bytes / wbytes);
    for (int M : Ms) {
      const size_t ny = (size_t)M * s.N;
      for (int kk = 0; kk < nkinds; ++kk) {
        const Kind& kd = kinds[kk];
        auto run = [&](int i) {
          const unsigned short* w = pool + (size_t)(i % copies) * (wbytes / 2);
          unsigned short* y = s.epi == 3 ? res : yref + 0;  // EPI 3 updates the residual in place
          if (s.epi == 0) y = res;
          return mp_gemm_bf16(x, s.K, w, y, s.N, s.epi == 3 ? res : nullptr, s.N, M, s.N, s.K, s.epi, 1 | kd.flags,
                              ws, nullptr, ap, ss, ss2, nullptr, 1.f / s.K, 1e-5f, 0);
        };
        // correctness: one call from the saved residual with zeroed statistics
        CK(hipMemcpy(res, res0, (size_t)64 * 12288 * 2, hipMemcpyDeviceToDevice));
        CK(hipMemset(ss, 0, ssn * 8));
        CK(hipMemset(ap, 0, (size_t)64 * 12288 * 2));
        int rc = run(0);
        if (rc) {
          printf("%-6s M=%2d %-7s rc=%d\n", s.name, M, kd.name, rc);
          continue;
        }
        CK(hipDeviceSynchronize());
        int err = 0;
        CK(hipMemcpy(&err, (int*)ws + mp::SK_MAX_GROUPS - 1, 4, hipMemcpyDeviceToHost));
        if (kk == 0 || kk == 5) {  // pk: tolerance reference; rwk: bitwise reference of the split-K forms
          if (kk == 5) {
            CK(hipMemcpy(yref, res, ny * 2, hipMemcpyDeviceToDevice));
            CK(hipMemcpy(apref, ap, ny * 2, hipMemcpyDeviceToDevice));
            CK(hipMemcpy(ssref, ss, ssn * 8, hipMemcpyDeviceToDevice));
          }
          if (kk == 0) CK(hipMemcpy(h0.data(), res, ny * 2, hipMemcpyDeviceToHost));
        }
        CK(hipMemcpy(h1.data(), res, ny * 2, hipMemcpyDeviceToHost));
        float maxd = 0.f;
        for (size_t i = 0; i < ny; ++i) {
          const float a = bf_host(h0[i]), b = bf_host(h1[i]);
          const float d = fabsf(a - b) / (fabsf(a) + 1e-2f);
          if (!(d <= maxd)) maxd = d;
        }
        long long ndiff = -1;  // bitwise mismatches against rwk (split-K forms only)
        if ((kd.flags & 256) && !(kd.flags & 1024) && !(kd.flags & 16384) && kk >= 5) {  // rotated walks sum in another order
          std::vector<unsigned short> r0(ny), a0(ny), a1(ny);
          CK(hipMemcpy(r0.data(), yref, ny * 2, hipMemcpyDeviceToHost));
          CK(hipMemcpy(a0.data(), apref, ny * 2, hipMemcpyDeviceToHost));
          CK(hipMemcpy(a1.data(), ap, ny * 2, hipMemcpyDeviceToHost));
          CK(hipMemcpy(s0.data(), ssref, ssn * 8, hipMemcpyDeviceToHost));
          CK(hipMemcpy(s1.data(), ss, ssn * 8, hipMemcpyDeviceToHost));
          ndiff = 0;
          for (size_t i = 0; i < ny; ++i) ndiff += (r0[i] != h1[i]) + (s.epi == 3 && a0[i] != a1[i]);
          if (s.epi == 3) {  // row sums of squares: total per row over the shards
            for (int r = 0; r < M; ++r) {
              unsigned long long t0 = 0, t1 = 0;
              for (int sh = 0; sh < mp::SS_NSH; ++sh) t0 += s0[sh * mp::SS_ROWS + r], t1 += s1[sh * mp::SS_ROWS + r];
              ndiff += t0 != t1;
            }
          }
        }
        if (err || ndiff > 0 || !(maxd < 0.25f)) bad = 1;
        // timing: rotated weight copies
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
        printf("%-6s M=%2d N=%5d K=%5d %-7s %7.2f us %5.2f TB/s  maxrel_vs_pk %.3g  bitdiff_vs_rwk %lld  err %d\n",
               s.name, M, s.N, s.K, kd.name, us, wbytes / us / 1e6, maxd, ndiff, err);
        fflush(stdout);
      }
    }
  }
  CK(hipDeviceSynchronize());
  printf(bad ? "SEAM_LAB FAIL\n" : "SEAM_LAB OK\n");
  return 0;  // the verdict is the printed line (a mismatch is not a GPU fault)
}
