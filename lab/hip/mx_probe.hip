// Probe of gfx950's block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 A / B: which
// (row, k) each lane's 32 bytes hold, which block each lane's e8m0 scale applies to, and what the
// opsel byte select does.  First hypothesis (lane l = 16 q + r holds A[r][32 q + j], its own scale
// scales its own 32 bytes) FAILED; mx_probe2 / mx_probe3 found the map checked here (H):
//   lane l = 16 q + r, byte j:  k = 16 q + j (j < 16),  k = 64 + 16 q + (j - 16) (j >= 16);
//   B likewise with c = l & 15; C[4 (l >> 4) + i][l & 15] (the 16x16x32 map);
//   the e8m0 scale of 32-block b = k / 32 of row r (col c) is byte ``opsel`` of lane 16 b + r (+ c)
//   - so block b's 32 values sit in lanes q = 2 (b & 1), 2 (b & 1) + 1, bytes 16 (b >> 1) .. + 15.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int OPS>
__global__ void mx_kernel(const i32x8* a, const i32x8* b, const unsigned* sa, const unsigned* sb, f32x4* c) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, OPS, sa[l], OPS, sb[l]);
  c[l] = acc;
}

static float e4m3(unsigned char v) {  // OCP e4m3fn
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float x;
  if (e == 0) x = std::ldexp((float)m / 8.f, -6);
  else x = std::ldexp(1.f + (float)m / 8.f, e - 7);
  return s ? -x : x;
}

int main() {
  unsigned char A[64][32], B[64][32];
  unsigned sa[64], sb[64];
  srand(7);
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      unsigned char v;
      do { v = rand() & 255; } while ((v & 0x7f) == 0x7f || ((v >> 3) & 15) > 9);  // no NaN, |x| <= 2^3
      A[l][j] = v;
      do { v = rand() & 255; } while ((v & 0x7f) == 0x7f || ((v >> 3) & 15) > 9);
      B[l][j] = v;
    }
  unsigned char ea[64], eb[64];
  for (int l = 0; l < 64; ++l) { ea[l] = 124 + rand() % 7; eb[l] = 124 + rand() % 7; }  // 2^-3 .. 2^3
  i32x8 *dA, *dB;
  unsigned *dsa, *dsb;
  f32x4* dC;
  hipMalloc(&dA, sizeof(A)); hipMalloc(&dB, sizeof(B)); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
  hipMalloc(&dC, 64 * 16);
  hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
  hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
  int fails = 0;
  for (int ops = 0; ops < 4; ++ops) {
    for (int l = 0; l < 64; ++l) {  // the scale in byte ``ops``, junk (127 +- x) elsewhere
      sa[l] = sb[l] = 0;
      for (int by = 0; by < 4; ++by) {
        sa[l] |= (unsigned)(by == ops ? ea[l] : 120 + by) << (8 * by);
        sb[l] |= (unsigned)(by == ops ? eb[l] : 133 - by) << (8 * by);
      }
    }
    hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
    switch (ops) {
      case 0: mx_kernel<0><<<1, 64>>>(dA, dB, dsa, dsb, dC); break;
      case 1: mx_kernel<1><<<1, 64>>>(dA, dB, dsa, dsb, dC); break;
      case 2: mx_kernel<2><<<1, 64>>>(dA, dB, dsa, dsb, dC); break;
      default: mx_kernel<3><<<1, 64>>>(dA, dB, dsa, dsb, dC); break;
    }
    float C[64][4];
    hipMemcpy(C, dC, sizeof(C), hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 4; ++i) {
        const int row = 4 * (l >> 4) + i, col = l & 15;
        double ref = 0;
        for (int q = 0; q < 4; ++q)
          for (int j = 0; j < 32; ++j) {
            const int blk = j < 16 ? q / 2 : 2 + q / 2;
            ref += (double)e4m3(A[16 * q + row][j]) * e4m3(B[16 * q + col][j]) *
                   std::ldexp(1.0, (int)ea[16 * blk + row] - 127) * std::ldexp(1.0, (int)eb[16 * blk + col] - 127);
          }
        const double e = std::fabs(C[l][i] - ref) / (std::fabs(ref) + 1e-3);
        if (e > maxerr) maxerr = e;
      }
    printf("opsel %d: max rel err vs hypothesis H = %.3e -> %s\n", ops, maxerr, maxerr < 1e-5 ? "PASS" : "FAIL");
    fails += maxerr >= 1e-5;
  }
  printf(fails ? "MX PROBE FAIL\n" : "MX PROBE PASS\n");
  return fails ? 1 : 0;
}
