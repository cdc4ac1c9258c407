// Dual-stream lab: does splitting a decode step's 64 rows into two 32-row micro-batches on two
// HIP streams, running the SAME layer sequence a kernel apart, let the second stream's weight
// reads hit the Infinity Cache (256 MB; every projection of a Llama-2-7B layer is <= 180 MB)
// and overlap the two streams' kernel ramps / drains?  Times the GEMM chain of L layers
// (qkv, o, gate/up, down; weights rotated over distinct copies so nothing is reused across
// layers) as: one stream at M = 64, one stream at M = 32, and two streams at M = 32.
//
//   hipcc -O3 --offload-arch=gfx950 -I<ops/csrc> scripts/dual_lab.hip -o scripts/lab_dual
#include <hip/hip_runtime.h>
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

// a KV-streaming stand-in for attention: reads `bytes` once (non-temporal), writes a little
__global__ __launch_bounds__(256) void stream_read(const mp::u16x8* __restrict__ p, size_t n16, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const mp::u16x8 v = __builtin_nontemporal_load(p + i);
    acc += (float)v[0];
  }
  if (acc == 12345.f) out[0] = acc;
}

struct G {
  int N, K, epi, f64, f32;  // flags at M = 64 / M = 32 (the autotuner's round-3 picks)
};

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 24;  // layers per timed chain
  const bool attn = argc > 2 ? atoi(argv[2]) != 0 : true;
  const G g[4] = {{12288, 4096, 0, 128 | 1024, 4},          // qkv: rw+r / sk
                  {4096, 4096, 0, 8, 8},                    // o: pk / pk
                  {22016, 4096, 1, 2 | 128 | 1024, 2 | 16 | 32},  // gate/up: rw+r / lds24 (packed out)
                  {4096, 11008, 0, 256 | 1024, 256 | 1024}};     // down: rwk+r (+ reduce)
  size_t lw = 0;
  for (auto& s : g) lw += (size_t)s.N * s.K;
  unsigned short* wts;
  CK(hipMalloc(&wts, lw * 2 * L));
  hipLaunchKernelGGL(fill_bf16, dim3(8192), dim3(256), 0, 0, wts, lw * L, 3u, 0.02f);
  // KV stand-in: 64 sessions x ~150 tokens x 16 KiB per layer = 157 MB per layer (Llama-2-7B, MHA)
  const size_t kvb = attn ? (size_t)157 << 20 : 0;
  unsigned short* kv = nullptr;
  if (attn) CK(hipMalloc(&kv, kvb * L));
  float* sink;
  CK(hipMalloc(&sink, 64));
  unsigned short *x[2], *y[2], *ap[2];
  void* ws[2];
  const int64_t wsb = mp_gemm_workspace_bytes();
  for (int i = 0; i < 2; ++i) {
    CK(hipMalloc(&x[i], (size_t)64 * 11008 * 2));
    CK(hipMalloc(&y[i], (size_t)64 * 22016 * 2));
    CK(hipMalloc(&ap[i], (size_t)64 * 11008 * 2));
    CK(hipMalloc(&ws[i], wsb));
    CK(hipMemset(ws[i], 0, wsb));
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, x[i], (size_t)64 * 11008, 7u + i, 1.0f);
  }
  CK(hipDeviceSynchronize());
  hipStream_t st[2];
  CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
  auto kern = [&](int lane, int layer, int j, int M) {
    const G& s = g[j];
    size_t off = lw * (size_t)layer;
    for (int q = 0; q < j; ++q) off += (size_t)g[q].N * g[q].K;
    const int fl = 1 | (M > 32 ? s.f64 : s.f32);
    const int nc = s.epi == 1 ? s.N / 2 : s.N;
    const int rc = mp_gemm_bf16(x[lane], s.K, wts + off, s.epi == 1 ? ap[lane] : y[lane], nc, nullptr, 0, M, s.N,
                                s.K, s.epi, fl, ws[lane], nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f,
                                st[lane]);
    if (rc) {
      fprintf(stderr, "gemm rc=%d (N=%d K=%d M=%d)\n", rc, s.N, s.K, M);
      exit(1);
    }
  };
  auto attn_k = [&](int lane, int layer, size_t bytes, size_t off) {
    if (!attn) return;
    hipLaunchKernelGGL(stream_read, dim3(2048), dim3(256), 0, st[lane],
                       reinterpret_cast<const mp::u16x8*>((const char*)kv + kvb * layer + off), bytes / 16, sink);
  };
  // one stream, all M rows; the attention stand-in between qkv and o
  auto chain1 = [&](int M) {
    for (int l = 0; l < L; ++l) {
      kern(0, l, 0, M);
      attn_k(0, l, kvb * M / 64, 0);
      for (int j = 1; j < 4; ++j) kern(0, l, j, M);
    }
  };
  // two streams of 32 rows each, kernel by kernel (lane 1 one kernel behind lane 0)
  auto chain2 = [&]() {
    for (int l = 0; l < L; ++l) {
      for (int j = 0; j < 4; ++j) {
        kern(0, l, j, 32);
        if (j == 0) attn_k(0, l, kvb / 2, 0);
        kern(1, l, j, 32);
        if (j == 0) attn_k(1, l, kvb / 2, kvb / 2);
      }
    }
  };
  hipEvent_t e0, e1, f0, f1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&f0));
  CK(hipEventCreate(&f1));
  auto timeit = [&](const char* name, auto&& fn, bool two) {
    float best = 1e30f;
    for (int r = 0; r < 4; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, st[0]));
      if (two) CK(hipStreamWaitEvent(st[1], e0, 0));
      fn();
      if (two) {
        CK(hipEventRecord(f1, st[1]));
        CK(hipStreamWaitEvent(st[0], f1, 0));
      }
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) best = ms < best ? ms : best;  // round 0 warms up
    }
    printf("%-34s %8.2f us per layer (%d layers)\n", name, best * 1000.f / L, L);
    fflush(stdout);
  };
  timeit("one stream, M=64", [&] { chain1(64); }, false);
  timeit("one stream, M=32", [&] { chain1(32); }, false);
  timeit("two streams, M=32 each", [&] { chain2(); }, true);
  timeit("one stream, M=64 (again)", [&] { chain1(64); }, false);
  // per-kernel reuse check: the same weight twice in a row (second read from the Infinity Cache?)
  for (int j = 0; j < 4; ++j) {
    float t[2];
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, st[0]));
      kern(0, j, j, 32);
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t[rep], e0, e1));
    }
    printf("gemm %d M=32: cold %.2f us, repeat %.2f us\n", j, t[0] * 1000.f, t[1] * 1000.f);
  }
  CK(hipDeviceSynchronize());
  printf("DUAL_LAB OK\n");
  return 0;
}
