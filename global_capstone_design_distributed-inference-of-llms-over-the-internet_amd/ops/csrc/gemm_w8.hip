// W8A16 decode GEMM entry point (fp8 weights dequantized into the bf16 MFMA; kernels:
// gemm_kernels.h, F8 = true instantiations).
#include "gemm_kernels.h"

// W8A16 decode GEMM: fp8 (e4m3) weights in the bf16 fragment order at 1 byte per element
// (Wq[N/16][K/32][64][8], per-output-column scales wsc[N]), packed bf16 activations, M <= 64.
// flags: bit 1 = packed SwiGLU output; bit 7 = balanced ring kernel; bit 8 = split-K ring +
// reduce launch (epilogue 0 / 3, needs ws).  Same epilogues / EpiArgs as mp_gemm_bf16.
// Returns 1 when neither form covers the shape (nothing launched).
extern "C" int mp_gemm_w8(const void* x, const void* wq, const float* wsc, void* y, int64_t y_stride,
                          const void* res, int64_t res_stride, int M, int N, int K, int epilogue, int flags, void* ws,
                          void* ap, void* ss_out, void* ss_zero, const void* ss_in, float inv_k, float eps,
                          hipStream_t stream) {
  (void)hipGetLastError();  // an earlier non-mpamd HIP call's stale error is not this launch's
  using namespace mp;
  if (M == 0) return 0;
  if (M > 64 || K % (32 * GU_MAX) || N % 16 || wsc == nullptr) return -1;
  if (epilogue == 3 && (ap == nullptr || res == nullptr)) return -5;
  EpiArgs ep{(bf16_t*)ap, (u64*)ss_out, (u64*)ss_zero, (const u64*)ss_in, inv_k, eps, (M + 15) / 16};
  ep.wsc = wsc;
  ep.rot = (flags >> 10) & 1;
  int rc = 1;
  if ((flags & 256) && !(flags & 2) && ws != nullptr) {
    switch ((M + 15) / 16) {
      case 1: rc = launch_gemm_rwk<1, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, rwk_comb(flags)); break;
      case 2: rc = launch_gemm_rwk<2, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, rwk_comb(flags)); break;
      case 3: rc = launch_gemm_rwk<3, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, rwk_comb(flags)); break;
      default: rc = launch_gemm_rwk<4, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, ep, ws, stream, rwk_comb(flags)); break;
    }
    if (rc < 0) return rc;
    if (rc == 0) return (int)hipGetLastError();
  }
  if (flags & 16384) return -6;  // partials only: nothing else writes them
  const int fl = flags | 1;
  if (M <= 16) rc = launch_gemm_rw<1, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, fl, ep, stream);
  else if (M <= 32) rc = launch_gemm_rw<2, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, fl, ep, stream);
  else if (M <= 48) rc = launch_gemm_rw<3, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, fl, ep, stream);
  else rc = launch_gemm_rw<4, true>(x, wq, y, y_stride, res, res_stride, M, N, K, epilogue, fl, ep, stream);
  if (rc != 0) return rc;
  return (int)hipGetLastError();
}

