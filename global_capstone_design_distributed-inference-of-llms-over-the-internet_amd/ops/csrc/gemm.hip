// Decode GEMM entry points, M <= 64 rows (bf16 weights), plus the weight / activation packers.
// The kernels live in gemm_kernels.h; 65..128 rows and fp8 weights are gemm_wide.hip and
// gemm_w8.hip (separate translation units: the build compiles them in parallel).
#include "gemm_kernels.h"

extern "C" int mp_gemm_bf16_wide(const void* x, const void* w, void* y, int64_t y_stride, const void* res,
                                 int64_t res_stride, int M, int N, int K, int epilogue, int flags, void* ws,
                                 const mp::EpiArgs& ep, hipStream_t stream);

namespace mp {

// Pack W[N, K] (row-major) into the fragment-native layout Wp[N/16][K/32][64][8].
__global__ __launch_bounds__(256) void pack_weight_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp,
                                                          int N, int K) {
  const int nks = K >> 5;
  const int64_t total = (int64_t)(N >> 4) * nks * 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const int64_t tile = i >> 6;
    const int ks = (int)(tile % nks);
    const int64_t nt = tile / nks;
    const int c = lane & 15, q = lane >> 4;
    const u16x8 v = *reinterpret_cast<const u16x8*>(w + (nt * 16 + c) * (int64_t)K + ks * 32 + q * 8);
    *reinterpret_cast<u16x8*>(wp + i * 8) = v;
  }
}

}  // namespace mp

extern "C" int mp_gemm_ss_elems() { return mp::SS_NSH * mp::SS_ROWS; }

// byte offset / size of the split-K partial-slab region inside the GEMM workspace (shared with
// the fp8 split-K kernel, fp8.hip)
extern "C" int64_t mp_gemm_slab_offset() {
  using namespace mp;
  return (int64_t)SK_MAX_GROUPS * sizeof(int) + SK_ZERO_BYTES + (int64_t)SK_MAX_BLOCKS * 2 * SK_MAX_S * 64 * sizeof(float);
}
extern "C" int64_t mp_gemm_slab_bytes() { return mp::RWK_SLAB_BYTES; }

// Split count S of the split-K ring form for this shape (0: not covered): with flags bit 14 the
// GEMM leaves S fp32 partial slabs [S][M][N] at mp_gemm_slab_offset() of the workspace for a
// consumer that sums them (fixed order s = 0..S-1 from zero: the reduce launch's bits).
extern "C" int mp_gemm_rwk_split(int M, int N, int K, int f8) {
  using namespace mp;
  if (M < 1 || M > 128 || N % 2048 || K % 128) return 0;
  int nt, S;
  // the same width bound launch_gemm_rwk<MT, F8> uses, so a consumer of the partial slabs sees the
  // split count the launch picks
  const int nt_max = rwk_nt_max(M);
  // f8 == 2: the MX form (gemm_mx.hip), whose ring steps are 128 deep
  rwk_choose(N / 16, f8 == 2 ? K / 128 : K / 32, sk_num_cus(), f8 != 0, nt, S, nt_max);
  if (f8 == 2 && nt) mx_geometry(N / 16, nt, S);
  if (nt == 0 || (int64_t)S * M * N * 4 > RWK_SLAB_BYTES) return 0;
  return S;
}

extern "C" int64_t mp_gemm_workspace_bytes() {
  using namespace mp;
  return (int64_t)SK_MAX_GROUPS * sizeof(int) + SK_ZERO_BYTES +
         (int64_t)SK_MAX_BLOCKS * 2 * SK_MAX_S * 64 * sizeof(float) + RWK_SLAB_BYTES;
}

// flags: bit 0 = x is packed (Ap[K/32][ceil(M/16)][64][8]); bit 1 = SwiGLU output packed;
//        bit 2 = use the stream-K kernel (needs ws: mp_gemm_workspace_bytes(), zero-initialised,
//        used by one stream at a time); bit 3 = force the one-group-per-workgroup kernel;
//        bit 4 = shared-A (LDS-staged activation) kernel when the shape allows it;
//        bit 7 = balanced ring kernel; bit 8 = split-K ring kernel + reduce launch (epilogue
//        0 / 2 / 3, needs ws); bits 8 + 9 = split-K ring kernel with the in-launch combine;
//        bit 10 = rotated k walk per workgroup (EpiArgs::rot); bits 8 + 11 = split-K ring with
//        the symmetric in-launch combine; bit 12 = row-split ring (epilogue 0 / 2 / 3, even row
//        tiles), + bit 13 = its weights loaded with the default cache policy.
//        epilogue 3 / ss_in: the fused-norm decode path (EpiArgs above; ap / ss_out / ss_zero /
//        ss_in may be null when unused).
extern "C" int mp_gemm_bf16(const void* x, int64_t x_stride, const void* w, void* y, int64_t y_stride,
                            const void* res, int64_t res_stride, int M, int N, int K, int epilogue, int flags,
                            void* ws, const int* gate, void* ap, void* ss_out, void* ss_zero, const void* ss_in,
                            float inv_k, float eps, hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  if (M == 0) return 0;
  if (epilogue == 3 && (ap == nullptr || res == nullptr)) return -5;
  EpiArgs ep{(bf16_t*)ap, (u64*)ss_out, (u64*)ss_zero, (const u64*)ss_in, inv_k, eps, (M + 15) / 16};
  ep.rot = (flags >> 10) & 1;
  if (M > 256 || K % (32 * GU_MAX) || N % 16 || ((flags & 1) == 0 && x_stride % 8)) return -1;
  int rc;
  if (M > 64) {  // 65..256 rows: gemm_wide.hip (split-K ring / balanced ring, packed A, no gate)
    if (!(flags & 1) || gate != nullptr) return -1;
    return mp_gemm_bf16_wide(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ws, ep, stream);
  }
  if ((flags & 1) && (flags & 4096) && !(flags & 2) && gate == nullptr) {  // row-split ring
    switch ((M + 15) / 16) {
      case 2: rc = launch_gemm_rwr<2>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream); break;
      case 4: rc = launch_gemm_rwr<4>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream); break;
      default: rc = 1; break;
    }
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if ((flags & 1) && (flags & 256) && !(flags & 2) && gate == nullptr && ws != nullptr) {  // split-K ring
#define MP_RWK(MT_) \
  rc = launch_gemm_rwk<MT_>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, rwk_comb(flags))
    switch ((M + 15) / 16) {  // the packed layout's row-tile count is part of its strides
      case 1: MP_RWK(1); break;
      case 2: MP_RWK(2); break;
      case 3: MP_RWK(3); break;
      default: MP_RWK(4); break;
    }
#undef MP_RWK
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if (flags & 16384) return -6;  // partials only: nothing else writes them
  if (gate != nullptr) flags &= ~(4 | 16 | 128);  // gated (MoE expert) GEMMs use the one-group kernel
  if ((flags & 1) && (flags & 128) && !(flags & 8)) {  // balanced ring kernel
    if (M <= 16) rc = launch_gemm_rw<1>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    else if (M <= 32) rc = launch_gemm_rw<2>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    else if (M <= 48) rc = launch_gemm_rw<3>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    else rc = launch_gemm_rw<4>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if ((flags & 1) && (flags & 16) && !(flags & 8)) {  // shared-A kernel
    if (M <= 16) rc = launch_gemm_lds<1>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    else if (M <= 32) rc = launch_gemm_lds<2>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    else if (M <= 48) rc = launch_gemm_lds<3>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    else rc = launch_gemm_lds<4>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if ((flags & 1) && (flags & 4) && !(flags & 8) && ws != nullptr) {
    if (M <= 16) rc = launch_gemm_sk<1>(x, y, y_stride, w, res, res_stride, M, N, K, epilogue, flags, ws, ep, stream);
    else if (M <= 32)
      rc = launch_gemm_sk<2>(x, y, y_stride, w, res, res_stride, M, N, K, epilogue, flags, ws, ep, stream);
    else if (M <= 48)
      rc = launch_gemm_sk<3>(x, y, y_stride, w, res, res_stride, M, N, K, epilogue, flags, ws, ep, stream);
    else rc = launch_gemm_sk<4>(x, y, y_stride, w, res, res_stride, M, N, K, epilogue, flags, ws, ep, stream);
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
    // rc == 1: shape not covered by the stream-K form -> one-group-per-workgroup kernel
  }
  if (M <= 16) rc = launch_gemm<1>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, gate, ep,
                                   stream);
  else if (M <= 32) rc = launch_gemm<2>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, gate,
                                        ep, stream);
  else if (M <= 48) rc = launch_gemm<3>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, gate,
                                        ep, stream);
  else rc = launch_gemm<4>(x, x_stride, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, gate, ep, stream);
  if (rc) return rc;
  return (int)hipGetLastError();
}

namespace mp {
// Pack row-major x[M, K] into Ap[K/32][ceil(M/16)][64][8] (rows >= M left untouched).
__global__ __launch_bounds__(256) void pack_act_kernel(const bf16_t* __restrict__ x, int64_t xs, bf16_t* __restrict__ ap,
                                                       int M, int K, int MT) {
  const int nch = K >> 3;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M * nch; i += gridDim.x * blockDim.x) {
    const int row = i / nch, col = (i - row * nch) * 8;
    *reinterpret_cast<u16x8*>(ap + apk_off(row, col, MT)) = *reinterpret_cast<const u16x8*>(x + row * xs + col);
  }
}
}  // namespace mp

extern "C" int mp_pack_act(const void* x, int64_t xs, void* ap, int M, int K, hipStream_t stream) {
  using namespace mp;
  if (K % 32 || xs % 8) return -1;
  if (M == 0) return 0;
  const int MT = (M + 15) / 16;
  const int n = M * (K / 8);
  hipLaunchKernelGGL(pack_act_kernel, dim3(min((n + 255) / 256, 4096)), dim3(256), 0, stream, (const bf16_t*)x, xs,
                     (bf16_t*)ap, M, K, MT);
  return (int)hipGetLastError();
}

extern "C" int mp_pack_weight(const void* w, void* wp, int N, int K, hipStream_t stream) {
  using namespace mp;
  if (N % 16 || K % 32) return -1;
  const int64_t total = (int64_t)(N / 16) * (K / 32) * 64;
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(pack_weight_kernel, dim3((int)g), dim3(256), 0, stream, (const bf16_t*)w, (bf16_t*)wp, N, K);
  return (int)hipGetLastError();
}
