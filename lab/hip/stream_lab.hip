// Streaming-read ceiling on this part: how fast can a kernel read W MB of cold HBM (rotated windows
// of a 3 GB pool, so neither L2 nor the Infinity Cache holds the window) - the yardstick for the
// weight-streaming decode GEMMs (33.5 MB o, 90 MB down, 100 MB qkv, 180 MB gate/up at Llama-2-7B).
// Variants: grid = 256 / 512 / 1024 / 2048 workgroups of 256 threads, 16-B loads, U loads in flight
// per thread, default or non-temporal loads.  Prints us and TB/s per (size, grid, U, policy).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/stream_lab.hip -o scripts/streamlab.bin && ./scripts/streamlab.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void stream_read(const uint4* __restrict__ p, size_t n, unsigned* sink) {
  unsigned acc = 0;
  const size_t step = (size_t)gridDim.x * blockDim.x;
  // contiguous chunk per workgroup (weights are read as contiguous column-tile slabs)
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t b0 = blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  (void)step;
  for (size_t i = b0 + threadIdx.x; i < b1; i += 256 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t j = i + (size_t)u * 256;
      const u32x4v* q = reinterpret_cast<const u32x4v*>(p + j);
      u32x4v t = (u32x4v)(0u);
      if (j < b1) t = NT ? __builtin_nontemporal_load(q) : *q;
      v[u] = make_uint4(t.x, t.y, t.z, t.w);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

int main() {
  const size_t pool = (size_t)3 << 30;
  char* buf;
  unsigned* sink;
  CK(hipMalloc(&buf, pool));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 1, pool));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int sizes_mb[] = {34, 90, 100, 180};
  const int grids[] = {256, 512, 1024, 2048};
  for (int smb : sizes_mb) {
    const size_t bytes = (size_t)smb << 20;
    const int windows = (int)(pool / bytes);
    for (int g : grids) {
      for (int mode = 0; mode < 4; ++mode) {
        auto run = [&](int i) {
          const uint4* p = reinterpret_cast<const uint4*>(buf + (size_t)(i % windows) * bytes);
          const size_t n = bytes / 16;
          if (mode == 0) hipLaunchKernelGGL((stream_read<4, false>), dim3(g), dim3(256), 0, 0, p, n, sink);
          if (mode == 1) hipLaunchKernelGGL((stream_read<8, false>), dim3(g), dim3(256), 0, 0, p, n, sink);
          if (mode == 2) hipLaunchKernelGGL((stream_read<4, true>), dim3(g), dim3(256), 0, 0, p, n, sink);
          if (mode == 3) hipLaunchKernelGGL((stream_read<8, true>), dim3(g), dim3(256), 0, 0, p, n, sink);
        };
        for (int i = 0; i < windows; ++i) run(i);
        const int iters = 40;
        float best = 1e30f;
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
        printf("size %4d MB grid %5d U %d %s  %7.2f us  %5.2f TB/s\n", smb, g, (mode & 1) ? 8 : 4,
               mode >= 2 ? "nt " : "def", us, bytes / us / 1e6);
        fflush(stdout);
      }
    }
  }
  printf("STREAM_LAB OK\n");
  return 0;
}
