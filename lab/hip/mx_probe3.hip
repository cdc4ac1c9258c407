// Third probe of v_mfma_scale_f32_16x16x128_f8f6f4: which lane's e8m0 scale applies to which lane's
// 32-byte block (data only in lane group qd, scale 2^q' on lane group q'), and what opsel selects.
#include <hip/hip_runtime.h>
#include <cstdio>
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

static unsigned char A[64][32], B[64][32];
static unsigned SA[64], SB[64];
static float C[64][4];
static i32x8 *dA, *dB;
static unsigned *dsa, *dsb;
static f32x4* dC;

static void run(int ops) {
  (void)hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
  (void)hipMemcpy(dsa, SA, 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsb, SB, 256, hipMemcpyHostToDevice);
  if (ops == 0) mx_kernel<0><<<1, 64>>>(dA, dB, dsa, dsb, dC);
  if (ops == 1) mx_kernel<1><<<1, 64>>>(dA, dB, dsa, dsb, dC);
  if (ops == 2) mx_kernel<2><<<1, 64>>>(dA, dB, dsa, dsb, dC);
  if (ops == 3) mx_kernel<3><<<1, 64>>>(dA, dB, dsa, dsb, dC);
  (void)hipMemcpy(C, dC, sizeof(C), hipMemcpyDeviceToHost);
}

int main() {
  (void)hipMalloc(&dA, sizeof(A)); (void)hipMalloc(&dB, sizeof(B)); (void)hipMalloc(&dsa, 256); (void)hipMalloc(&dsb, 256);
  (void)hipMalloc(&dC, 64 * 16);
  memset(B, 0x38, sizeof(B));
  for (int l = 0; l < 64; ++l) SB[l] = 0x7f7f7f7fu;
  // scale_a of lane group q' = 2^q' (byte 0), data 1.0 only in lane group qd (and only the first
  // 16 or the last 16 bytes: is a lane's block split?)
  for (int half = 0; half < 3; ++half)
    for (int qd = 0; qd < 4; ++qd) {
      memset(A, 0, sizeof(A));
      for (int r = 0; r < 16; ++r)
        for (int j = 0; j < 32; ++j)
          if (half == 2 || (half == 0 ? j < 16 : j >= 16)) A[16 * qd + r][j] = 0x38;
      for (int l = 0; l < 64; ++l) SA[l] = 0x7f7f7f00u | (127u + (l >> 4));
      run(0);
      printf("data in group %d bytes %s: C[r0,c0] = %g (= count x 2^q of the applied scale)\n", qd,
             half == 0 ? "0-15 " : half == 1 ? "16-31" : "0-31 ", C[0][0]);
    }
  // opsel: scale word bytes [127, 128, 129, 130] on every lane
  memset(A, 0x38, sizeof(A));
  for (int ops = 0; ops < 4; ++ops) {
    for (int l = 0; l < 64; ++l) { SA[l] = 0x8281807fu; SB[l] = 0x7f7f7f7fu; }
    run(ops);
    printf("opsel %d, scale_a bytes [127,128,129,130]: C = %g (128 x 2^byte-127)\n", ops, C[0][0]);
    for (int l = 0; l < 64; ++l) { SA[l] = 0x7f7f7f7fu; SB[l] = 0x8281807fu; }
    run(ops);
    printf("opsel %d, scale_b bytes [127,128,129,130]: C = %g\n", ops, C[0][0]);
  }
  return 0;
}
