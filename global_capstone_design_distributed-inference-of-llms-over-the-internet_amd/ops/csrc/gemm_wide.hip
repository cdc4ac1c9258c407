// Decode GEMM for 65..256 rows (the packed decode path at 96..256 sessions): split-K ring (o,
// down) and balanced ring kernels at MT = 5..8, 12 and 16 (kernels: gemm_kernels.h), and the
// two-dimensionally tiled kernel (gemm_t2d.h, flags bit 15), which ops picks from ops.T2D_MIN
// (129) rows up: there the ring forms measured slower than hipBLASLt (profiles/r4d) and the tiled
// form faster (profiles/r5x).
#include "gemm_t2d.h"

extern "C" int mp_gemm_bf16_wide(const void* x, const void* w, void* y, int64_t y_stride, const void* res,
                                 int64_t res_stride, int M, int N, int K, int epilogue, int flags, void* ws,
                                 const mp::EpiArgs& ep, hipStream_t stream) {
  using namespace mp;
  int rc = 1;
  if (flags & 32768) {  // two-dimensionally tiled form (gemm_t2d.h); bits 16-17: forced k split
    rc = launch_gemm_t2d(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, ws, stream,
                         (flags >> 16) & 3);
    if (rc == 1 && ((flags >> 16) & 3)) return -7;  // a forced split this shape does not take (lab)
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if ((flags & 256) && !(flags & 2) && ws != nullptr) {  // split-K ring
#define MP_RWK(MT_) \
  rc = launch_gemm_rwk<MT_>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, rwk_comb(flags))
    switch ((M + 15) / 16) {
      case 5: MP_RWK(5); break;
      case 6: MP_RWK(6); break;
      case 7: MP_RWK(7); break;
      case 8: MP_RWK(8); break;
      case 9: case 10: case 11: case 12: MP_RWK(12); break;
      default: MP_RWK(16); break;
    }
#undef MP_RWK
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if (M <= 80) rc = launch_gemm_rw<5>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
  else if (M <= 96) rc = launch_gemm_rw<6>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
  else if (M <= 112) rc = launch_gemm_rw<7>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
  else if (M <= 128) rc = launch_gemm_rw<8>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
  else if (M <= 192) rc = launch_gemm_rw<12>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
  else rc = launch_gemm_rw<16>(x, w, y, y_stride, res, res_stride, M, N, K, epilogue, flags, ep, stream);
  if (rc != 0) return rc < 0 ? rc : -1;
  return (int)hipGetLastError();
}

// 1 if the two-dimensionally tiled form covers this shape (flags as mp_gemm_bf16; no launch).
extern "C" int mp_gemm_t2d_ok(int M, int N, int K, int epilogue, int out_packed, int with_ws) {
  using namespace mp;
  EpiArgs ep{};
  ep.mt_out = (M + 15) / 16;
  char dummy = 0;
  return launch_gemm_t2d(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue, 1 | (out_packed ? 2 : 0), ep,
                         with_ws ? &dummy : nullptr, 0, 0, true) == 0 &&
         launch_gemm_t2d(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue,
                         1 | (out_packed ? 2 : 0) | 262144, ep, with_ws ? &dummy : nullptr, 0, 0, true) == 0;
}

// 1 if mp_gemm_bf16 covers a packed-activation decode GEMM of M = 65..256 rows (balanced ring
// kernel: the widths built, epilogue 0 or packed SwiGLU), else 0.  No launch.
extern "C" int mp_gemm_rw_ok(int M, int N, int K, int epilogue, int out_packed) {
  using namespace mp;
  if (M <= 64 || M > 256 || K % (32 * GU_MAX) || N % 16) return 0;
  // the fused-norm producer (residual + packed copy + row statistics) at 65..256 rows runs as
  // the split-K ring + its reduce launch (the reduce applies the epilogue): o / down widths
  if (epilogue == 3) return !out_packed && N % 2048 == 0;
  EpiArgs ep{};
  ep.mt_out = (M + 15) / 16;
  const int flags = 1 | (out_packed ? 2 : 0) | 128;
  int rc;
  if (M <= 80) rc = launch_gemm_rw<5>(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue, flags, ep, 0, true);
  else if (M <= 96) rc = launch_gemm_rw<6>(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue, flags, ep, 0, true);
  else if (M <= 112) rc = launch_gemm_rw<7>(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue, flags, ep, 0, true);
  else if (M <= 128) rc = launch_gemm_rw<8>(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue, flags, ep, 0, true);
  else if (M <= 192) rc = launch_gemm_rw<12>(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue, flags, ep, 0, true);
  else rc = launch_gemm_rw<16>(nullptr, nullptr, nullptr, 0, nullptr, 0, M, N, K, epilogue, flags, ep, 0, true);
  return rc == 0;
}

