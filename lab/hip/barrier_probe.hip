// Persistent launch vs launch sequence for weight-streaming phases (VERDICT r5 #2 question): P phases,
// each streaming 32 MiB of cold memory (256 workgroups x 128 KiB, one per CU - a batch-1 decode
// projection's shape).  B: one launch per phase, captured in a hipGraph.  A0: ONE persistent launch
// with an XCD-hierarchical grid barrier between phases (per-XCD arrival counters, then a top counter
// that releases a generation word; monotonic counters, so nothing is re-zeroed).  A1: A0 with the
// next phase's loads issued BEFORE the barrier (weights do not depend on the previous phase; the
// prefetch a persistent engine can do and a kernel boundary cannot).
//
// Safety: the grid is one 256-thread workgroup per CU (always co-resident on a 256-CU part), every
// spin is bounded (2^24 polls, then the run reports an error instead of hanging), the barrier uses
// vector atomics and loads only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);      \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
constexpr int WG = 256;
constexpr int SLICE = 128 * 1024;            // bytes per workgroup per phase
constexpr int LOADS = SLICE / (WG * 16);     // 16-B loads per thread per phase (32)
constexpr int LINE = 16;                     // uints between counters (64 B)

__device__ __forceinline__ unsigned consume(const u32x4 (&r)[LOADS]) {
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < LOADS; ++i) s ^= r[i][0] + r[i][1] + r[i][2] + r[i][3];
  return s;
}

__device__ __forceinline__ void issue(u32x4 (&r)[LOADS], const unsigned char* base) {
#pragma unroll
  for (int i = 0; i < LOADS; ++i)
    r[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + ((size_t)i * WG + threadIdx.x) * 16));
}

__device__ __forceinline__ const unsigned char* slice(const unsigned char* buf, int phase, int nblk) {
  return buf + ((size_t)phase * nblk + blockIdx.x) * SLICE;
}

// generation ``gen`` (1, 2, ...): wait until every workgroup has arrived.  FENCE = false skips the
// release / acquire fences (nothing is published here: the floor of the synchronisation itself).
template <bool FENCE = true>
__device__ void grid_barrier(unsigned* bar, unsigned gen, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned per = gridDim.x / 8;
    const int x = blockIdx.x & 7;  // XCD under round-robin dispatch (placement only)
    if (FENCE) __threadfence();
    const unsigned old = atomicAdd(&bar[x * LINE], 1u);
    if (old == gen * per - 1) {
      const unsigned top = atomicAdd(&bar[8 * LINE], 1u);
      if (top == gen * 8 - 1) atomicExch(&bar[9 * LINE], gen);
    }
    int spins = 0;
    while (__hip_atomic_load(&bar[9 * LINE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      if (++spins > (1 << 24)) {
        atomicExch(err, 1);
        break;
      }
    }
    if (FENCE) __threadfence();
  }
  __syncthreads();
}

__global__ __launch_bounds__(WG) void phase_kernel(const unsigned char* buf, int phase, unsigned* sink) {
  u32x4 r[LOADS];
  issue(r, slice(buf, phase, gridDim.x));
  const unsigned s = consume(r);
  if (s == 0x12345678u) sink[blockIdx.x] = s;  // keeps the loads
}

template <bool PREFETCH, bool FENCE = true>
__global__ __launch_bounds__(WG) void persistent_kernel(const unsigned char* buf, int phases, unsigned* bar,
                                                        unsigned gen0, int* err, unsigned* sink) {
  u32x4 r[LOADS];
  unsigned s = 0;
  issue(r, slice(buf, 0, gridDim.x));
  for (int p = 0; p < phases; ++p) {
    s ^= consume(r);
    if (p + 1 < phases) {
      if (PREFETCH) issue(r, slice(buf, p + 1, gridDim.x));
      grid_barrier<FENCE>(bar, gen0 + p + 1, err);
      if (!PREFETCH) issue(r, slice(buf, p + 1, gridDim.x));
    }
  }
  if (s == 0x12345678u) sink[blockIdx.x] = s;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int nblk = cus;  // one workgroup per CU
  if (nblk % 8) {
    printf("CU count %d not a multiple of 8\n", nblk);
    return 1;
  }
  const int P = 32;
  const size_t bytes = (size_t)P * nblk * SLICE;  // 1 GiB at 256 CUs: every phase cold
  unsigned char* buf;
  unsigned *bar, *sink;
  int* err;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMemset(buf, 1, bytes));
  CHECK(hipMalloc(&bar, 16 * LINE * sizeof(unsigned)));
  CHECK(hipMemset(bar, 0, 16 * LINE * sizeof(unsigned)));
  CHECK(hipMalloc(&sink, nblk * sizeof(unsigned)));
  CHECK(hipMalloc(&err, sizeof(int)));
  CHECK(hipMemset(err, 0, sizeof(int)));
  unsigned char* flush;
  const size_t fbytes = (size_t)1 << 30;
  CHECK(hipMalloc(&flush, fbytes));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  // B: the launch sequence in a graph
  hipGraph_t graph;
  hipGraphExec_t exec;
  CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int p = 0; p < P; ++p) hipLaunchKernelGGL(phase_kernel, dim3(nblk), dim3(WG), 0, st, buf, p, sink);
  CHECK(hipStreamEndCapture(st, &graph));
  CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  unsigned gen = 0;
  const char* names[4] = {"launches (graph)", "persistent + barrier", "persistent + barrier + prefetch",
                          "persistent + fence-free barrier"};
  std::vector<float> best(4, 1e9f);
  for (int rep = 0; rep < 5; ++rep) {
    for (int v = 0; v < 4; ++v) {
      CHECK(hipMemsetAsync(flush, rep + v, fbytes, st));  // evict L2 / Infinity Cache
      CHECK(hipEventRecord(e0, st));
      if (v == 0) {
        CHECK(hipGraphLaunch(exec, st));
      } else if (v == 1) {
        hipLaunchKernelGGL(persistent_kernel<false>, dim3(nblk), dim3(WG), 0, st, buf, P, bar, gen, err, sink);
        gen += P - 1;
      } else if (v == 2) {
        hipLaunchKernelGGL(persistent_kernel<true>, dim3(nblk), dim3(WG), 0, st, buf, P, bar, gen, err, sink);
        gen += P - 1;
      } else {
        hipLaunchKernelGGL((persistent_kernel<false, false>), dim3(nblk), dim3(WG), 0, st, buf, P, bar, gen, err, sink);
        gen += P - 1;
      }
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best[v]) best[v] = ms;
    }
  }
  int h_err = 0;
  CHECK(hipMemcpy(&h_err, err, sizeof(int), hipMemcpyDeviceToHost));
  const double mb = (double)nblk * SLICE / 1e6;
  printf("%d phases x %.1f MB (%d workgroups x 128 KiB), cold; best of 5\n", P, mb, nblk);
  for (int v = 0; v < 4; ++v)
    printf("%-34s %8.1f us total  %6.2f us/phase  %5.2f TB/s\n", names[v], best[v] * 1e3, best[v] * 1e3 / P,
           P * mb / 1e6 / (best[v] / 1e3));
  printf(h_err ? "BARRIER TIMEOUT (results invalid)\n" : "barrier ok\n");
  return h_err ? 2 : 0;
}
