// Second probe of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 A / B): the lane / byte -> (row, k) maps
// and the scale block map, from one-hot operands (1.0 = 0x38) and unit scales (e8m0 127).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void mx_kernel(const i32x8* a, const i32x8* b, const unsigned* sa, const unsigned* sb, f32x4* c) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  c[l] = acc;
}

static unsigned char A[64][32], B[64][32];
static unsigned SA[64], SB[64];
static float C[64][4];
static i32x8 *dA, *dB;
static unsigned *dsa, *dsb;
static f32x4* dC;

static void run() {
  (void)hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
  (void)hipMemcpy(dsa, SA, 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsb, SB, 256, hipMemcpyHostToDevice);
  mx_kernel<<<1, 64>>>(dA, dB, dsa, dsb, dC);
  (void)hipMemcpy(C, dC, sizeof(C), hipMemcpyDeviceToHost);
}
// C[row][col] from (lane l, reg i) under the 16x16 C map: row 4 (l >> 4) + i, col l & 15
static void print_nonzero(const char* tag) {
  printf("%s:", tag);
  int n = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i)
      if (C[l][i] != 0.f && n++ < 40) printf(" (r%d,c%d)=%g", 4 * (l >> 4) + i, l & 15, C[l][i]);
  printf("  [%d nonzero]\n", n);
}

int main() {
  (void)hipMalloc(&dA, sizeof(A)); (void)hipMalloc(&dB, sizeof(B)); (void)hipMalloc(&dsa, 256); (void)hipMalloc(&dsb, 256);
  (void)hipMalloc(&dC, 64 * 16);
  for (int l = 0; l < 64; ++l) SA[l] = SB[l] = 0x7f7f7f7fu;
  // E2: A one-hot (lane la, byte j), B all ones -> the row of (la, j); E3 the mirror for B
  memset(B, 0x38, sizeof(B));
  const int probes[][2] = {{0, 0}, {0, 1}, {0, 8}, {0, 16}, {0, 31}, {1, 0}, {5, 7}, {16, 0}, {17, 3}, {32, 0}, {48, 31}};
  for (auto& p : probes) {
    memset(A, 0, sizeof(A));
    A[p[0]][p[1]] = 0x38;
    run();
    char t[64];
    snprintf(t, sizeof t, "A one-hot lane %2d byte %2d", p[0], p[1]);
    print_nonzero(t);
  }
  memset(A, 0x38, sizeof(A));
  for (auto& p : probes) {
    memset(B, 0, sizeof(B));
    B[p[0]][p[1]] = 0x38;
    run();
    char t[64];
    snprintf(t, sizeof t, "B one-hot lane %2d byte %2d", p[0], p[1]);
    print_nonzero(t);
  }
  // E4: k pairing: A one-hot (la, ja) and B one-hot (lb, jb) -> nonzero iff same k
  int pairs = 0;
  for (int qa = 0; qa < 4; ++qa)
    for (int ja = 0; ja < 32; ja += 5) {
      memset(A, 0, sizeof(A));
      A[16 * qa][ja] = 0x38;
      for (int qb = 0; qb < 4; ++qb)
        for (int jb = 0; jb < 32; ++jb) {
          memset(B, 0, sizeof(B));
          B[16 * qb][jb] = 0x38;
          run();
          if (C[0][0] != 0.f) { printf("k-pair: A(q%d,b%d) <-> B(q%d,b%d) = %g\n", qa, ja, qb, jb, C[0][0]); ++pairs; }
        }
    }
  printf("k pairs found: %d\n", pairs);
  // E5: scale block map: A, B all ones; raise ONE lane's scale byte 0 to 128 (x2)
  memset(A, 0x38, sizeof(A));
  memset(B, 0x38, sizeof(B));
  for (int ls : {0, 1, 16, 17, 33, 63}) {
    for (int l = 0; l < 64; ++l) SA[l] = SB[l] = 0x7f7f7f7fu;
    SA[ls] = 0x7f7f7f80u;
    run();
    printf("scale_a lane %2d byte0=128:", ls);
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 4; ++i)
        if (C[l][i] != 128.f) printf(" (r%d,c%d)=%g", 4 * (l >> 4) + i, l & 15, C[l][i]);
    printf("\n");
    for (int l = 0; l < 64; ++l) SA[l] = 0x7f7f7f7fu;
    SB[ls] = 0x7f7f7f80u;
    run();
    printf("scale_b lane %2d byte0=128:", ls);
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 4; ++i)
        if (C[l][i] != 128.f) printf(" (r%d,c%d)=%g", 4 * (l >> 4) + i, l & 15, C[l][i]);
    printf("\n");
  }
  return 0;
}
