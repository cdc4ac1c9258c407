// torch custom-op registrations (namespace `mpamd`) for the gfx950 kernels.
//
// Every op writes into caller-provided outputs and launches on the current HIP
// stream, so a whole stage step can be captured into one hipGraph.  Shape and
// dtype checks happen here, on the host, before any kernel sees a pointer.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>

#include <cmath>

extern "C" {
int mp_rmsnorm(const void* x, int64_t x_stride, void* res, int64_t res_stride, const void* w, void* y,
               int64_t y_stride, const int32_t* rows, int nrows, int H, float eps, int mode, int packed_mt,
               void* ss_out, void* a8, float* a8_scale, const int64_t* gather, int64_t gather_n,
               hipStream_t stream);
int mp_rope_kv_write(void* qkv, int64_t qkv_stride, const int64_t* pos, const float* cos_t, const float* sin_t,
                     void* kc, void* vc, const int64_t* slots, int T, int nh, int nkv, int D, int page_size,
                     hipStream_t stream);
int mp_kv_write(const void* k, int64_t k_stride, const void* v, int64_t v_stride, void* kc, void* vc,
                const int64_t* slots, int T, int nkv, int D, int page_size, hipStream_t stream);
int mp_paged_attention(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt,
                       int bt_stride, const int32_t* q_seq, const int32_t* q_ctx, void* out, float* workspace, int T,
                       int nh, int nkv, int D, int page_size, int PS, int NP, float scale, int packed_mt,
                       const int64_t* rope_pos, const float* cos_t, const float* sin_t, const int64_t* slots,
                       int* counters, int n_counters, const void* qkv_part, hipStream_t stream);
int mp_embedding(const int64_t* ids, const void* table, void* out, int T, int H, int64_t vocab, hipStream_t stream);
int mp_swiglu(const void* gu, void* out, int64_t T, int F, hipStream_t stream);
int mp_add(const void* a, const void* b, void* y, int64_t n, hipStream_t stream);
int mp_argmax(const void* logits, int64_t stride, int R, int V, int64_t* out, hipStream_t stream);
int mp_sample(const void* logits, int64_t stride, int R, int V, const float* temps, const float* top_ps,
              const int32_t* top_ks, const float* rep_pens, int32_t* recent, int recent_stride, int32_t* recent_len,
              const int64_t* seeds, float* ws, int64_t* out, int update, hipStream_t stream);
int64_t mp_gemm_workspace_bytes();
int64_t mp_gemm_slab_offset();
int mp_gemm_rwk_split(int M, int N, int K, int f8);
int mp_attention_mfma(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt, int bt_stride,
                      const int32_t* q_seq, const int32_t* q_ctx, const int32_t* qb_tok0, const int32_t* qb_ntok, int NB,
                      void* out, float* workspace, int T, int nh, int nkv, int D, int page_size, int PS, int NP,
                      float scale, int packed_mt, const int64_t* rope_pos, const float* cos_t, const float* sin_t,
                      const int64_t* slots, const int32_t* sb_first, const int32_t* sb_n, int NSB,
                      const void* qkv_part, void* mx_ax, void* mx_as, hipStream_t stream);
int mp_attention_fa(const void* q, int64_t q_stride, const void* kc, const void* vc, const int32_t* bt, int bt_stride,
                    const int32_t* q_seq, const int32_t* q_ctx, const int32_t* fb_tok0, const int32_t* fb_ntok, int NBF,
                    void* out, float* workspace, int T, int nh, int nkv, int D, int page_size, int PS, int NP,
                    float scale, int nw, int pair, hipStream_t stream);
int mp_quant_act_fp8(const void* ap, void* a8, float* scale, float* part, int M, int K, hipStream_t stream);
int mp_gemm_fp8(const void* a8, const float* as, const void* wq, const float* ws, void* y, int64_t ys, const void* res,
                int64_t rs, int M, int N, int K, int epilogue, int out_packed, int kind, float* part,
                int64_t part_bytes, hipStream_t stream);
int64_t mp_gemm_slab_offset();
int64_t mp_gemm_slab_bytes();
void mp_fp8_set_kernel(int kind);
int mp_gemm_rw_ok(int M, int N, int K, int epilogue, int out_packed);
int mp_gemm_t2d_ok(int M, int N, int K, int epilogue, int out_packed, int with_ws);
int mp_quant_rows_fp8(const void* x, int64_t xs, void* a8, float* scale, int M, int K, hipStream_t stream);
int mp_gemm_bf16(const void* x, int64_t x_stride, const void* w, void* y, int64_t y_stride, const void* res,
                 int64_t res_stride, int M, int N, int K, int epilogue, int flags, void* ws, const int* gate,
                 void* ap, void* ss_out, void* ss_zero, const void* ss_in, float inv_k, float eps,
                 hipStream_t stream);
int mp_gemm_ss_elems();
int mp_gemm_w8(const void* x, const void* wq, const float* wsc, void* y, int64_t y_stride, const void* res,
               int64_t res_stride, int M, int N, int K, int epilogue, int flags, void* ws, void* ap, void* ss_out,
               void* ss_zero, const void* ss_in, float inv_k, float eps, hipStream_t stream);
int mp_pack_act(const void* x, int64_t xs, void* ap, int M, int K, hipStream_t stream);
int mp_quant_mx(const void* ap, void* ax, void* as, int M, int K, hipStream_t stream);
int mp_gemm_mx(const void* ax, const void* as, const void* wq, const float* wsc, void* y, int64_t y_stride,
               const void* res, int64_t res_stride, int M, int N, int K, int epilogue, int flags, void* ws, void* ap,
               void* ss_out, void* ss_zero, const void* ss_in, float inv_k, float eps, hipStream_t stream);
int mp_pack_weight(const void* w, void* wp, int N, int K, hipStream_t stream);
}

namespace {

#define MP_CHECK(cond, msg) TORCH_CHECK(cond, "mpamd: ", msg)

inline void check_launch(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "mpamd: ", what, " launch failed with code ", rc);
}

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

inline void check_bf16_cuda(const at::Tensor& t, const char* name) {
  MP_CHECK(t.is_cuda(), std::string(name) + " must be on the GPU");
  MP_CHECK(t.scalar_type() == at::kBFloat16, std::string(name) + " must be bf16");
}

inline void check_rows(const at::Tensor& t, const char* name) {
  MP_CHECK(t.dim() == 2, std::string(name) + " must be 2-D [rows, cols]");
  MP_CHECK(t.stride(1) == 1, std::string(name) + " must have unit inner stride");
  MP_CHECK(t.stride(0) % 8 == 0, std::string(name) + " row stride must be a multiple of 8");
  MP_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, std::string(name) + " must be 16-B aligned");
}

inline int64_t packed_numel(int64_t M, int64_t K) { return ((M + 15) / 16) * 16 * K; }

// fused-norm row statistics: int64 [32 shards][256 rows] fixed-point sums (gemm.hip EpiArgs)
inline void* opt_ss(const c10::optional<at::Tensor>& t, const char* name) {
  if (!t.has_value()) return nullptr;
  MP_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous() && t->numel() >= mp_gemm_ss_elems(),
           std::string(name) + ": int64 cuda contiguous [32, 256] (ops.norm_stats_buffer)");
  return t->data_ptr();
}

void rmsnorm(const at::Tensor& x, at::Tensor& residual, const at::Tensor& w, at::Tensor& y, double eps, int64_t mode,
             const c10::optional<at::Tensor>& rows, int64_t packed, const c10::optional<at::Tensor>& ss,
             const c10::optional<at::Tensor>& a8, const c10::optional<at::Tensor>& a8_scale,
             const c10::optional<at::Tensor>& gather) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(y, "y");
  check_rows(x, "x");
  const int H = x.size(1);
  MP_CHECK(w.numel() == H && w.is_contiguous(), "weight shape");
  if (!packed) {
    check_rows(y, "y");
    MP_CHECK(y.size(1) == H, "y cols");
  }
  MP_CHECK(mode >= 0 && mode <= 3, "mode");
  void* ssp = opt_ss(ss, "ss");
  // gather: x is an embedding table and row t of the output / residual is x[gather[t]] (stage entry)
  const int64_t* gp = nullptr;
  int nrows = x.size(0);
  if (gather.has_value()) {
    MP_CHECK(gather->is_cuda() && gather->scalar_type() == at::kLong && gather->is_contiguous() && gather->dim() == 1,
             "gather: int64 cuda [T]");
    MP_CHECK(mode >= 2 && !rows.has_value(), "gather with mode 2 / 3, no rows");
    gp = gather->data_ptr<int64_t>();
    nrows = gather->numel();
  }
  MP_CHECK(mode != 3 || (ssp != nullptr && nrows <= 256), "mode 3 needs ss and <= 256 rows");
  if (mode != 0) {
    check_bf16_cuda(residual, "residual");
    check_rows(residual, "residual");
    MP_CHECK(residual.size(0) == nrows && residual.size(1) == H, "residual shape");
  }
  const int32_t* rp = nullptr;
  if (rows.has_value()) {
    MP_CHECK(rows->scalar_type() == at::kInt && rows->is_contiguous() && rows->is_cuda(), "rows: int32 cuda");
    MP_CHECK(mode == 0, "row gather only with mode 0");
    rp = rows->data_ptr<int32_t>();
    nrows = rows->numel();
  }
  int pmt = 0;
  if (packed) {
    MP_CHECK(H % 32 == 0 && y.is_contiguous() && y.numel() >= packed_numel(nrows, H), "packed y too small");
    pmt = (nrows + 15) / 16;
  } else {
    MP_CHECK(y.size(0) >= nrows, "y rows");
  }
  void* a8p = nullptr;
  float* a8s = nullptr;
  if (a8.has_value()) {  // fp8 output (W8A8 decode path): A8 [K/64][MT][64][16 B] + per-row scales
    MP_CHECK(packed && a8_scale.has_value(), "fp8 output needs packed=1 and a8_scale");
    MP_CHECK(a8->is_cuda() && a8->scalar_type() == at::kByte && a8->is_contiguous() &&
                 a8->numel() >= packed_numel(nrows, H) && H % 64 == 0, "a8: uint8 [packed_numel(rows, H)], H % 64");
    MP_CHECK(a8_scale->is_cuda() && a8_scale->scalar_type() == at::kFloat && a8_scale->numel() >= nrows,
             "a8_scale: fp32 [rows]");
    a8p = a8->data_ptr();
    a8s = a8_scale->data_ptr<float>();
  }
  check_launch(mp_rmsnorm(x.data_ptr(), x.stride(0), mode ? residual.data_ptr() : nullptr,
                          mode ? residual.stride(0) : 0, w.data_ptr(), y.data_ptr(), packed ? 0 : y.stride(0), rp,
                          nrows, H, (float)eps, (int)mode, pmt, ssp, a8p, a8s, gp, gp ? x.size(0) : 0,
                          cur_stream()),
               "rmsnorm");
}

void rope_kv_write(at::Tensor& qkv, const at::Tensor& positions, const at::Tensor& cos, const at::Tensor& sin,
                   at::Tensor& k_cache, at::Tensor& v_cache, const at::Tensor& slots, int64_t nh, int64_t nkv) {
  check_bf16_cuda(qkv, "qkv");
  check_rows(qkv, "qkv");
  check_bf16_cuda(k_cache, "k_cache");
  check_bf16_cuda(v_cache, "v_cache");
  MP_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous(), "cache [pages, nkv, page, D]");
  MP_CHECK(k_cache.sizes() == v_cache.sizes(), "k/v cache shapes differ");
  const int D = k_cache.size(3), page = k_cache.size(2);
  MP_CHECK(k_cache.size(1) == nkv, "cache kv heads");
  MP_CHECK(qkv.size(1) == (nh + 2 * nkv) * D, "qkv width");
  const int T = qkv.size(0);
  MP_CHECK(positions.scalar_type() == at::kLong && positions.numel() == T && positions.is_contiguous(), "positions");
  MP_CHECK(slots.scalar_type() == at::kLong && slots.numel() == T && slots.is_contiguous(), "slots");
  MP_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
               sin.is_contiguous() && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(),
           "cos/sin tables fp32 [max_pos, D/2]");
  check_launch(mp_rope_kv_write(qkv.data_ptr(), qkv.stride(0), positions.data_ptr<int64_t>(), cos.data_ptr<float>(),
                                sin.data_ptr<float>(), k_cache.data_ptr(), v_cache.data_ptr(),
                                slots.data_ptr<int64_t>(), T, nh, nkv, D, page, cur_stream()),
               "rope_kv_write");
}

void kv_write(const at::Tensor& k, const at::Tensor& v, at::Tensor& k_cache, at::Tensor& v_cache,
              const at::Tensor& slots) {
  check_bf16_cuda(k, "k");
  check_bf16_cuda(v, "v");
  check_rows(k, "k");
  check_rows(v, "v");
  MP_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous(), "cache layout");
  const int nkv = k_cache.size(1), page = k_cache.size(2), D = k_cache.size(3);
  MP_CHECK(k.size(1) == nkv * D && v.size(1) == nkv * D, "k/v width");
  MP_CHECK(slots.scalar_type() == at::kLong && slots.numel() == k.size(0), "slots");
  check_launch(mp_kv_write(k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0), k_cache.data_ptr(),
                           v_cache.data_ptr(), slots.data_ptr<int64_t>(), k.size(0), nkv, D, page, cur_stream()),
               "kv_write");
}

// Host mirror of mp::QkvPart (common.h): the qkv projection as split-K partial slabs
// [S][M][width] fp32 + the fused-norm row statistics, read by the decode attention kernels.
struct QkvPartArgs {
  const float* part;
  int S;
  int64_t slab;
  int ldn;
  const unsigned long long* ss;
  float inv_k, eps;
};

static bool qkv_part_args(const c10::optional<at::Tensor>& part, int64_t splits, const c10::optional<at::Tensor>& ss,
                          double inv_k, double eps, int64_t T, int64_t width, QkvPartArgs& a) {
  if (!part.has_value()) return false;
  MP_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() && part->dim() == 3 &&
               part->size(0) == splits && part->size(1) == T && part->size(2) == width,
           "qkv_part: fp32 [S, T, qkv width] split-K slabs (ops.linear_partials)");
  MP_CHECK(splits >= 1 && splits <= 8, "qkv_part splits");
  const unsigned long long* ssp = nullptr;
  if (ss.has_value()) {
    MP_CHECK(ss->is_cuda() && ss->scalar_type() == at::kLong && ss->is_contiguous() && ss->numel() >= mp_gemm_ss_elems(),
             "part_ss: row statistics [32, 256] int64");
    ssp = reinterpret_cast<const unsigned long long*>(ss->data_ptr<int64_t>());
  }
  a = QkvPartArgs{part->data_ptr<float>(), (int)splits, T * width, (int)width, ssp, (float)inv_k, (float)eps};
  return true;
}

static void paged_attention_impl(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                                 const at::Tensor& block_tables, const at::Tensor& q_seq, const at::Tensor& q_ctx,
                                 at::Tensor& out, at::Tensor& workspace, int64_t nh, int64_t nkv, double scale,
                                 int64_t part_size, int64_t num_parts, int64_t packed, const int64_t* rope_pos,
                                 const float* cos_t, const float* sin_t, const int64_t* slots,
                                 const c10::optional<at::Tensor>& counters, const QkvPartArgs* qp = nullptr) {
  check_bf16_cuda(q, "q");
  check_rows(q, "q");
  check_bf16_cuda(out, "out");
  MP_CHECK(out.is_contiguous(), "out contiguous");
  const int D = k_cache.size(3);
  const int T = q.size(0);
  MP_CHECK(q.size(1) >= nh * D, "q width");
  if (packed) {
    MP_CHECK(out.numel() >= packed_numel(T, nh * D) && (nh * D) % 32 == 0, "packed out numel");
  } else {
    MP_CHECK(out.numel() == (int64_t)T * nh * D, "out numel");
  }
  MP_CHECK(k_cache.size(1) == nkv && k_cache.is_contiguous() && v_cache.is_contiguous(), "cache");
  MP_CHECK(block_tables.scalar_type() == at::kInt && block_tables.dim() == 2 && block_tables.stride(1) == 1,
           "block_tables int32 [S, max_pages]");
  MP_CHECK(q_seq.scalar_type() == at::kInt && q_seq.numel() == T, "q_seq");
  MP_CHECK(q_ctx.scalar_type() == at::kInt && q_ctx.numel() == T, "q_ctx");
  MP_CHECK(workspace.scalar_type() == at::kFloat, "workspace fp32");
  if (num_parts > 1) MP_CHECK(workspace.numel() >= (int64_t)T * nh * num_parts * (D + 2), "workspace too small");
  int* cp = nullptr;
  int ncnt = 0;
  if (counters.has_value()) {
    MP_CHECK(counters->is_cuda() && counters->scalar_type() == at::kInt && counters->is_contiguous(),
             "counters: zero-initialised cuda int32");
    cp = counters->data_ptr<int32_t>();
    ncnt = (int)counters->numel();
  }
  check_launch(mp_paged_attention(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                  block_tables.data_ptr<int32_t>(), block_tables.stride(0), q_seq.data_ptr<int32_t>(),
                                  q_ctx.data_ptr<int32_t>(), out.data_ptr(), workspace.data_ptr<float>(), T, nh, nkv,
                                  D, k_cache.size(2), part_size, num_parts, (float)scale,
                                  packed ? (int)((T + 15) / 16) : 0, rope_pos, cos_t, sin_t, slots, cp, ncnt,
                                  qp, cur_stream()),
               "paged_attention");
}

void paged_attention(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                     const at::Tensor& block_tables, const at::Tensor& q_seq, const at::Tensor& q_ctx,
                     at::Tensor& out, at::Tensor& workspace, int64_t nh, int64_t nkv, double scale, int64_t part_size,
                     int64_t num_parts, int64_t packed, const c10::optional<at::Tensor>& counters) {
  paged_attention_impl(q, k_cache, v_cache, block_tables, q_seq, q_ctx, out, workspace, nh, nkv, scale, part_size,
                       num_parts, packed, nullptr, nullptr, nullptr, nullptr, counters);
}

// Decode attention with RoPE + KV write fused in (attention.hip ROPE path): q is the unrotated
// fused qkv row; k_cache / v_cache receive the new token at slots[t].
void paged_attention_rope(const at::Tensor& qkv, at::Tensor& k_cache, at::Tensor& v_cache,
                          const at::Tensor& block_tables, const at::Tensor& q_seq, const at::Tensor& q_ctx,
                          const at::Tensor& positions, const at::Tensor& cos, const at::Tensor& sin,
                          const at::Tensor& slots, at::Tensor& out, at::Tensor& workspace, int64_t nh, int64_t nkv,
                          double scale, int64_t part_size, int64_t num_parts, int64_t packed,
                          const c10::optional<at::Tensor>& counters, const c10::optional<at::Tensor>& qkv_part,
                          int64_t part_splits, const c10::optional<at::Tensor>& part_ss, double inv_k, double eps) {
  check_bf16_cuda(k_cache, "k_cache");
  check_bf16_cuda(v_cache, "v_cache");
  MP_CHECK(k_cache.dim() == 4 && k_cache.sizes() == v_cache.sizes(), "cache [pages, nkv, page, D]");
  const int D = k_cache.size(3), T = qkv.size(0);
  MP_CHECK(qkv.size(1) == (nh + 2 * nkv) * D, "qkv width");
  MP_CHECK(positions.scalar_type() == at::kLong && positions.numel() == T && positions.is_contiguous(), "positions");
  MP_CHECK(slots.scalar_type() == at::kLong && slots.numel() == T && slots.is_contiguous(), "slots");
  MP_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
               sin.is_contiguous() && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(),
           "cos/sin tables fp32 [max_pos, D/2]");
  MP_CHECK(D % 16 == 0, "head dim");
  QkvPartArgs qp;
  const bool has_qp = qkv_part_args(qkv_part, part_splits, part_ss, inv_k, eps, T, qkv.size(1), qp);
  paged_attention_impl(qkv, k_cache, v_cache, block_tables, q_seq, q_ctx, out, workspace, nh, nkv, scale, part_size,
                       num_parts, packed, positions.data_ptr<int64_t>(), cos.data_ptr<float>(), sin.data_ptr<float>(),
                       slots.data_ptr<int64_t>(), counters, has_qp ? &qp : nullptr);
}

static void attention_mfma_impl(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                                const at::Tensor& block_tables, const at::Tensor& q_seq, const at::Tensor& q_ctx,
                                const at::Tensor& qblocks, at::Tensor& out, at::Tensor& workspace, int64_t nh,
                                int64_t nkv, double scale, int64_t part_size, int64_t num_parts, int64_t packed,
                                const int64_t* rope_pos, const float* cos_t, const float* sin_t,
                                const int64_t* slots, const c10::optional<at::Tensor>& superblocks = c10::nullopt,
                                const QkvPartArgs* qp = nullptr, void* mx_ax = nullptr, void* mx_as = nullptr) {
  check_bf16_cuda(q, "q");
  check_rows(q, "q");
  check_bf16_cuda(out, "out");
  MP_CHECK(out.is_contiguous(), "out contiguous");
  const int D = k_cache.size(3);
  const int T = q.size(0);
  MP_CHECK(q.size(1) >= nh * D, "q width");
  if (packed) {
    MP_CHECK(out.numel() >= packed_numel(T, nh * D) && (nh * D) % 32 == 0, "packed out numel");
  } else {
    MP_CHECK(out.numel() == (int64_t)T * nh * D, "out numel");
  }
  MP_CHECK(k_cache.size(1) == nkv && k_cache.is_contiguous() && v_cache.is_contiguous(), "cache");
  MP_CHECK(block_tables.scalar_type() == at::kInt && block_tables.dim() == 2 && block_tables.stride(1) == 1,
           "block_tables int32 [S, max_pages]");
  MP_CHECK(q_seq.scalar_type() == at::kInt && q_seq.numel() == T, "q_seq");
  MP_CHECK(q_ctx.scalar_type() == at::kInt && q_ctx.numel() == T, "q_ctx");
  MP_CHECK(workspace.scalar_type() == at::kFloat, "workspace fp32");
  if (num_parts > 1) MP_CHECK(workspace.numel() >= (int64_t)T * nh * num_parts * (D + 2), "workspace too small");
  MP_CHECK(qblocks.scalar_type() == at::kInt && qblocks.dim() == 2 && qblocks.size(0) == 2 && qblocks.is_contiguous(),
           "qblocks int32 [2, NB] (first token, token count)");
  const int NB = qblocks.size(1);
  const int32_t* sbp = nullptr;
  int NSB = 0;
  if (superblocks.has_value()) {  // prefill superblocks: int32 [2, NSB] (first query block, count <= 4)
    MP_CHECK(superblocks->is_cuda() && superblocks->scalar_type() == at::kInt && superblocks->dim() == 2 &&
                 superblocks->size(0) == 2 && superblocks->is_contiguous() && superblocks->size(1) <= NB,
             "superblocks int32 [2, NSB] (ops.query_superblocks)");
    sbp = superblocks->data_ptr<int32_t>();
    NSB = superblocks->size(1);
  }
  check_launch(mp_attention_mfma(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                 block_tables.data_ptr<int32_t>(), block_tables.stride(0), q_seq.data_ptr<int32_t>(),
                                 q_ctx.data_ptr<int32_t>(), qblocks.data_ptr<int32_t>(),
                                 qblocks.data_ptr<int32_t>() + NB, NB, out.data_ptr(), workspace.data_ptr<float>(), T,
                                 nh, nkv, D, k_cache.size(2), part_size, num_parts, (float)scale,
                                 packed ? (int)((T + 15) / 16) : 0, rope_pos, cos_t, sin_t, slots, sbp,
                                 sbp != nullptr ? sbp + NSB : nullptr, NSB, qp, mx_ax, mx_as, cur_stream()),
               "attention_mfma");
}

void attention_mfma(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                    const at::Tensor& block_tables, const at::Tensor& q_seq, const at::Tensor& q_ctx,
                    const at::Tensor& qblocks, at::Tensor& out, at::Tensor& workspace, int64_t nh, int64_t nkv,
                    double scale, int64_t part_size, int64_t num_parts, int64_t packed,
                    const c10::optional<at::Tensor>& superblocks) {
  attention_mfma_impl(q, k_cache, v_cache, block_tables, q_seq, q_ctx, qblocks, out, workspace, nh, nkv, scale,
                      part_size, num_parts, packed, nullptr, nullptr, nullptr, nullptr, superblocks);
}

// Causal prefill attention, 32x32x16 MFMA FA2 form (attention_fa.hip): row-major output.
void attention_fa(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                  const at::Tensor& block_tables, const at::Tensor& q_seq, const at::Tensor& q_ctx,
                  const at::Tensor& fablocks, at::Tensor& out, at::Tensor& workspace, int64_t nh, int64_t nkv,
                  double scale, int64_t part_size, int64_t num_parts, int64_t waves, int64_t pair) {
  check_bf16_cuda(q, "q");
  check_rows(q, "q");
  check_bf16_cuda(out, "out");
  check_bf16_cuda(k_cache, "k_cache");
  check_bf16_cuda(v_cache, "v_cache");
  MP_CHECK(out.is_contiguous(), "out contiguous");
  MP_CHECK(k_cache.dim() == 4 && k_cache.sizes() == v_cache.sizes(), "cache [pages, nkv, page, D]");
  const int D = k_cache.size(3);
  const int T = q.size(0);
  MP_CHECK(D == 128, "attention_fa: head_dim 128");
  MP_CHECK(q.size(1) >= nh * D, "q width");
  MP_CHECK(out.numel() == (int64_t)T * nh * D, "out numel");
  MP_CHECK(k_cache.size(1) == nkv && k_cache.is_contiguous() && v_cache.is_contiguous(), "cache");
  MP_CHECK(block_tables.scalar_type() == at::kInt && block_tables.dim() == 2 && block_tables.stride(1) == 1,
           "block_tables int32 [S, max_pages]");
  MP_CHECK(q_seq.scalar_type() == at::kInt && q_seq.numel() == T, "q_seq");
  MP_CHECK(q_ctx.scalar_type() == at::kInt && q_ctx.numel() == T, "q_ctx");
  MP_CHECK(workspace.scalar_type() == at::kFloat, "workspace fp32");
  if (num_parts > 1) MP_CHECK(workspace.numel() >= (int64_t)T * nh * num_parts * (D + 2), "workspace too small");
  MP_CHECK(fablocks.is_cuda() && fablocks.scalar_type() == at::kInt && fablocks.dim() == 2 && fablocks.size(0) == 2 &&
               fablocks.is_contiguous(),
           "fablocks int32 [2, NB] (first token, token count), ops.fa_blocks");
  MP_CHECK(waves == 4 || waves == 8, "waves 4 or 8");
  const int NB = fablocks.size(1);
  check_launch(mp_attention_fa(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                               block_tables.data_ptr<int32_t>(), block_tables.stride(0), q_seq.data_ptr<int32_t>(),
                               q_ctx.data_ptr<int32_t>(), fablocks.data_ptr<int32_t>(),
                               fablocks.data_ptr<int32_t>() + NB, NB, out.data_ptr(), workspace.data_ptr<float>(), T,
                               nh, nkv, D, k_cache.size(2), part_size, num_parts, (float)scale, (int)waves,
                               (int)pair, cur_stream()),
               "attention_fa");
}

// GQA decode with RoPE + KV write fused (attention_mfma.hip ROPE path): one token per query block,
// block b = token b (the kernel reads no qblocks on this path; ``decode_qblocks`` builds exactly that).
void attention_mfma_rope(const at::Tensor& qkv, at::Tensor& k_cache, at::Tensor& v_cache,
                         const at::Tensor& block_tables, const at::Tensor& q_seq, const at::Tensor& q_ctx,
                         const at::Tensor& qblocks, const at::Tensor& positions, const at::Tensor& cos,
                         const at::Tensor& sin, const at::Tensor& slots, at::Tensor& out, at::Tensor& workspace,
                         int64_t nh, int64_t nkv, double scale, int64_t part_size, int64_t num_parts, int64_t packed,
                         const c10::optional<at::Tensor>& qkv_part, int64_t part_splits,
                         const c10::optional<at::Tensor>& part_ss, double inv_k, double eps,
                         const c10::optional<at::Tensor>& mx_ax, const c10::optional<at::Tensor>& mx_as) {
  check_bf16_cuda(k_cache, "k_cache");
  check_bf16_cuda(v_cache, "v_cache");
  MP_CHECK(k_cache.dim() == 4 && k_cache.sizes() == v_cache.sizes(), "cache [pages, nkv, page, D]");
  const int D = k_cache.size(3), T = qkv.size(0);
  MP_CHECK(qkv.size(1) == (nh + 2 * nkv) * D, "qkv width");
  MP_CHECK(positions.scalar_type() == at::kLong && positions.numel() == T && positions.is_contiguous(), "positions");
  MP_CHECK(slots.scalar_type() == at::kLong && slots.numel() == T && slots.is_contiguous(), "slots");
  MP_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
               sin.is_contiguous() && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(),
           "cos/sin tables fp32 [max_pos, D/2]");
  MP_CHECK(qblocks.size(1) == T, "fused RoPE needs one query token per block (decode)");
  QkvPartArgs qp;
  const bool has_qp = qkv_part_args(qkv_part, part_splits, part_ss, inv_k, eps, T, qkv.size(1), qp);
  void* axp = nullptr;
  void* asp = nullptr;
  if (mx_ax.has_value()) {  // the output as the W8A8-MX GEMM's activation (ops.quant_mx layout)
    MP_CHECK(mx_as.has_value() && packed && num_parts == 1 && D == 128, "mx output: packed, one part, D 128, as_");
    const int64_t K = nh * D, rows = ((T + 15) / 16) * 16;
    MP_CHECK(mx_ax->is_cuda() && mx_ax->scalar_type() == at::kByte && mx_ax->is_contiguous() && mx_ax->numel() >= rows * K,
             "mx_ax: uint8 [ceil(T/16)*16*K]");
    MP_CHECK(mx_as->is_cuda() && mx_as->scalar_type() == at::kByte && mx_as->is_contiguous() && mx_as->numel() >= 2 * K,
             "mx_as: uint8 [2K]");
    axp = mx_ax->data_ptr();
    asp = mx_as->data_ptr();
  }
  attention_mfma_impl(qkv, k_cache, v_cache, block_tables, q_seq, q_ctx, qblocks, out, workspace, nh, nkv, scale,
                      part_size, num_parts, packed, positions.data_ptr<int64_t>(), cos.data_ptr<float>(),
                      sin.data_ptr<float>(), slots.data_ptr<int64_t>(), c10::nullopt, has_qp ? &qp : nullptr, axp, asp);
}

void embedding(const at::Tensor& ids, const at::Tensor& table, at::Tensor& out) {
  check_bf16_cuda(table, "table");
  check_bf16_cuda(out, "out");
  MP_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "ids int64");
  MP_CHECK(table.is_contiguous() && out.is_contiguous(), "contiguous");
  MP_CHECK(out.numel() == ids.numel() * table.size(1), "out shape");
  check_launch(mp_embedding(ids.data_ptr<int64_t>(), table.data_ptr(), out.data_ptr(), ids.numel(), table.size(1),
                            table.size(0), cur_stream()),
               "embedding");
}

void swiglu(const at::Tensor& gu, at::Tensor& out) {
  check_bf16_cuda(gu, "gu");
  check_bf16_cuda(out, "out");
  MP_CHECK(gu.is_contiguous() && out.is_contiguous(), "contiguous");
  const int64_t T = gu.size(0);
  const int F = gu.size(1) / 2;
  MP_CHECK(out.numel() == T * F, "out shape");
  check_launch(mp_swiglu(gu.data_ptr(), out.data_ptr(), T, F, cur_stream()), "swiglu");
}

void add(const at::Tensor& a, const at::Tensor& b, at::Tensor& y) {
  check_bf16_cuda(a, "a");
  check_bf16_cuda(b, "b");
  check_bf16_cuda(y, "y");
  MP_CHECK(a.is_contiguous() && b.is_contiguous() && y.is_contiguous(), "contiguous");
  MP_CHECK(a.numel() == b.numel() && a.numel() == y.numel(), "numel");
  check_launch(mp_add(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), cur_stream()), "add");
}

void argmax(const at::Tensor& logits, at::Tensor& out) {
  check_bf16_cuda(logits, "logits");
  check_rows(logits, "logits");
  MP_CHECK(out.scalar_type() == at::kLong && out.numel() == logits.size(0), "out int64 [R]");
  check_launch(mp_argmax(logits.data_ptr(), logits.stride(0), logits.size(0), logits.size(1),
                         out.data_ptr<int64_t>(), cur_stream()),
               "argmax");
}

void sample(const at::Tensor& logits, const at::Tensor& temps, const at::Tensor& top_ps, const at::Tensor& top_ks,
            const at::Tensor& rep_pens, at::Tensor& recent, at::Tensor& recent_len, const at::Tensor& seeds,
            at::Tensor& workspace, at::Tensor& out, int64_t update) {
  check_bf16_cuda(logits, "logits");
  check_rows(logits, "logits");
  const int R = logits.size(0), V = logits.size(1);
  MP_CHECK(temps.scalar_type() == at::kFloat && temps.numel() == R, "temps");
  MP_CHECK(top_ps.scalar_type() == at::kFloat && top_ps.numel() == R, "top_ps");
  MP_CHECK(top_ks.scalar_type() == at::kInt && top_ks.numel() == R, "top_ks");
  MP_CHECK(rep_pens.scalar_type() == at::kFloat && rep_pens.numel() == R, "rep_pens");
  MP_CHECK(recent.scalar_type() == at::kInt && recent.dim() == 2 && recent.size(0) == R && recent.is_contiguous(),
           "recent int32 [R, n]");
  MP_CHECK(recent_len.scalar_type() == at::kInt && recent_len.numel() == R, "recent_len");
  MP_CHECK(seeds.scalar_type() == at::kLong && seeds.numel() == R, "seeds");
  MP_CHECK(workspace.scalar_type() == at::kFloat && workspace.numel() >= (int64_t)R * V, "workspace");
  MP_CHECK(out.scalar_type() == at::kLong && out.numel() == R, "out");
  check_launch(mp_sample(logits.data_ptr(), logits.stride(0), R, V, temps.data_ptr<float>(), top_ps.data_ptr<float>(),
                         top_ks.data_ptr<int32_t>(), rep_pens.data_ptr<float>(), recent.data_ptr<int32_t>(),
                         recent.size(1), recent_len.data_ptr<int32_t>(), seeds.data_ptr<int64_t>(),
                         workspace.data_ptr<float>(), out.data_ptr<int64_t>(), (int)update, cur_stream()),
               "sample");
}

// flags bit 0: x is packed (holds ceil(M/16)*16*K elements, M given); bit 1: packed SwiGLU output
void gemm(const at::Tensor& x, const at::Tensor& wp, at::Tensor& y, const c10::optional<at::Tensor>& residual,
          int64_t epilogue, int64_t M_, int64_t flags, const c10::optional<at::Tensor>& workspace,
          const c10::optional<at::Tensor>& gate, const c10::optional<at::Tensor>& ap,
          const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& ss_zero,
          const c10::optional<at::Tensor>& ss_in, double inv_k, double eps) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(wp, "wp");
  check_bf16_cuda(y, "y");
  MP_CHECK(wp.dim() == 4 && wp.size(2) == 64 && wp.size(3) == 8 && wp.is_contiguous(),
           "wp must be a packed weight [N/16, K/32, 64, 8] (ops.pack_weight)");
  const int N = 16 * wp.size(0), K = 32 * wp.size(1);
  const bool apk = flags & 1, opk = flags & 2;
  int M;
  if (apk) {
    M = (int)M_;
    MP_CHECK(x.is_contiguous() && x.numel() >= packed_numel(M, K), "packed x too small");
  } else {
    check_rows(x, "x");
    M = x.size(0);
    MP_CHECK(x.size(1) == K, "K mismatch between x and packed weight");
  }
  const int ncols = epilogue == 1 ? N / 2 : N;
  if (opk) {
    MP_CHECK(epilogue == 1 && y.is_contiguous() && y.numel() >= packed_numel(M, ncols), "packed y");
  } else {
    check_rows(y, "y");
    MP_CHECK(y.size(0) == M && y.size(1) == ncols, "y shape");
  }
  const void* rp = nullptr;
  int64_t rs = 0;
  if (residual.has_value()) {
    check_bf16_cuda(*residual, "residual");
    check_rows(*residual, "residual");
    MP_CHECK(residual->size(0) == M && residual->size(1) == N, "residual shape");
    rp = residual->data_ptr();
    rs = residual->stride(0);
  }
  MP_CHECK(epilogue < 2 || rp != nullptr, "residual epilogue needs residual");
  MP_CHECK(epilogue >= 0 && epilogue <= 3, "epilogue");
  void* app = nullptr;
  if (ap.has_value()) {
    check_bf16_cuda(*ap, "ap");
    MP_CHECK(ap->is_contiguous() && ap->numel() >= packed_numel(M, N), "ap: packed [ceil(M/16)*16*N]");
    app = ap->data_ptr();
  }
  void* sso = opt_ss(ss_out, "ss_out");
  void* ssz = opt_ss(ss_zero, "ss_zero");
  const void* ssi = opt_ss(ss_in, "ss_in");
  MP_CHECK(epilogue != 3 || (app != nullptr && !opk), "epilogue 3 needs ap (and ss_out outside ablations)");
  void* ws = nullptr;
  if (workspace.has_value()) {
    MP_CHECK(workspace->is_cuda() && workspace->is_contiguous() &&
                 workspace->numel() * workspace->element_size() >= mp_gemm_workspace_bytes(),
             "gemm workspace too small (ops.gemm_workspace)");
    ws = workspace->data_ptr();
  }
  const int* gp = nullptr;
  if (gate.has_value()) {  // MoE expert gate: one int32 on the device (0 -> the GEMM is skipped)
    MP_CHECK(gate->is_cuda() && gate->scalar_type() == at::kInt && gate->numel() == 1, "gate must be one cuda int32");
    gp = gate->data_ptr<int>();
  }
  check_launch(mp_gemm_bf16(x.data_ptr(), apk ? 0 : x.stride(0), wp.data_ptr(), y.data_ptr(), opk ? 0 : y.stride(0),
                            rp, rs, M, N, K, (int)epilogue, (int)flags, ws, gp, app, sso, ssz, ssi, (float)inv_k,
                            (float)eps, cur_stream()),
               "gemm");
}

void pack_act(const at::Tensor& x, at::Tensor& ap) {
  check_bf16_cuda(x, "x");
  check_rows(x, "x");
  MP_CHECK(ap.is_contiguous() && ap.numel() >= packed_numel(x.size(0), x.size(1)), "ap too small");
  check_launch(mp_pack_act(x.data_ptr(), x.stride(0), ap.data_ptr(), x.size(0), x.size(1), cur_stream()), "pack_act");
}

at::Tensor pack_weight(const at::Tensor& w) {
  check_bf16_cuda(w, "w");
  MP_CHECK(w.dim() == 2 && w.is_contiguous(), "w [N, K] contiguous");
  const int N = w.size(0), K = w.size(1);
  MP_CHECK(N % 16 == 0 && K % 32 == 0, "pack_weight needs N % 16 == 0 and K % 32 == 0");
  auto wp = at::empty({N / 16, K / 32, 64, 8}, w.options());
  check_launch(mp_pack_weight(w.data_ptr(), wp.data_ptr(), N, K, cur_stream()), "pack_weight");
  return wp;
}

// W8A16 decode GEMM (gemm.hip mp_gemm_w8): packed bf16 x (M rows), fp8 weight Wq uint8
// [N/16, K/32, 64, 8] + per-column fp32 scales; flags as mp_gemm_w8 (bit 1 packed SwiGLU out,
// bit 7 ring, bit 8 split-K ring)
void gemm_w8(const at::Tensor& x, const at::Tensor& wq, const at::Tensor& wsc, at::Tensor& y,
             const c10::optional<at::Tensor>& residual, int64_t epilogue, int64_t M_, int64_t flags,
             const c10::optional<at::Tensor>& workspace, const c10::optional<at::Tensor>& ap,
             const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& ss_zero,
             const c10::optional<at::Tensor>& ss_in, double inv_k, double eps) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(y, "y");
  MP_CHECK(wq.is_cuda() && wq.scalar_type() == at::kByte && wq.dim() == 4 && wq.size(2) == 64 && wq.size(3) == 8 &&
               wq.is_contiguous(),
           "wq must be an fp8 weight uint8 [N/16, K/32, 64, 8] (ops.pack_weight_w8)");
  const int N = 16 * wq.size(0), K = 32 * wq.size(1);
  MP_CHECK(wsc.is_cuda() && wsc.scalar_type() == at::kFloat && wsc.is_contiguous() && wsc.numel() == N,
           "wsc: fp32 [N] column scales");
  const int M = (int)M_;
  const bool opk = flags & 2;
  MP_CHECK(M >= 0 && M <= 64, "gemm_w8: 0 <= M <= 64");
  MP_CHECK(x.is_contiguous() && x.numel() >= packed_numel(M, K), "packed x too small");
  const int ncols = epilogue == 1 ? N / 2 : N;
  if (opk) {
    MP_CHECK(epilogue == 1 && y.is_contiguous() && y.numel() >= packed_numel(M, ncols), "packed y");
  } else {
    check_rows(y, "y");
    MP_CHECK(y.size(0) == M && y.size(1) == ncols, "y shape");
  }
  MP_CHECK(epilogue == 0 || epilogue == 3 || (epilogue == 1 && opk), "gemm_w8: epilogue 0, 3 or packed SwiGLU");
  const void* rp = nullptr;
  int64_t rs = 0;
  if (residual.has_value()) {
    check_bf16_cuda(*residual, "residual");
    check_rows(*residual, "residual");
    MP_CHECK(residual->size(0) == M && residual->size(1) == N, "residual shape");
    rp = residual->data_ptr();
    rs = residual->stride(0);
  }
  void* app = nullptr;
  if (ap.has_value()) {
    check_bf16_cuda(*ap, "ap");
    MP_CHECK(ap->is_contiguous() && ap->numel() >= packed_numel(M, N), "ap: packed [ceil(M/16)*16*N]");
    app = ap->data_ptr();
  }
  MP_CHECK(epilogue != 3 || (app != nullptr && rp != nullptr), "epilogue 3 needs residual and ap");
  void* ws = nullptr;
  if (workspace.has_value()) {
    MP_CHECK(workspace->is_cuda() && workspace->is_contiguous() &&
                 workspace->numel() * workspace->element_size() >= mp_gemm_workspace_bytes(),
             "gemm workspace too small (ops.gemm_workspace)");
    ws = workspace->data_ptr();
  }
  const int rc = mp_gemm_w8(x.data_ptr(), wq.data_ptr(), wsc.data_ptr<float>(), y.data_ptr(), opk ? 0 : y.stride(0),
                            rp, rs, M, N, K, (int)epilogue, (int)flags, ws, app, opt_ss(ss_out, "ss_out"),
                            opt_ss(ss_zero, "ss_zero"), opt_ss(ss_in, "ss_in"), (float)inv_k, (float)eps, cur_stream());
  TORCH_CHECK(rc != 1, "mpamd: gemm_w8: no fp8-weight kernel covers M=", M, " N=", N, " K=", K, " epilogue=",
              epilogue);
  check_launch(rc, "gemm_w8");
}

int64_t gemm_workspace_bytes() { return mp_gemm_workspace_bytes(); }
int64_t gemm_slab_offset() { return mp_gemm_slab_offset(); }
int64_t gemm_rwk_split(int64_t M, int64_t N, int64_t K, int64_t f8) {
  return mp_gemm_rwk_split((int)M, (int)N, (int)K, (int)f8);
}
void fp8_gemm_kernel(int64_t kind) { mp_fp8_set_kernel((int)kind); }
bool gemm_t2d_ok(int64_t M, int64_t N, int64_t K, int64_t epilogue, int64_t out_packed) {
  return mp_gemm_t2d_ok((int)M, (int)N, (int)K, (int)epilogue, (int)out_packed, 1) != 0;
}

bool gemm_rw_ok(int64_t M, int64_t N, int64_t K, int64_t epilogue, int64_t out_packed) {
  return mp_gemm_rw_ok((int)M, (int)N, (int)K, (int)epilogue, (int)out_packed) != 0;
}

// packed bf16 decode activation (M rows) -> fp8 A8 [K/64][MT][64][16] (uint8) + row scales (fp32, >= MT*16)
void quant_act_fp8(const at::Tensor& ap, at::Tensor& a8, at::Tensor& scale, int64_t M, int64_t K) {
  check_bf16_cuda(ap, "ap");
  MP_CHECK(ap.is_contiguous() && ap.numel() >= packed_numel(M, K), "packed activation too small");
  MP_CHECK(a8.is_cuda() && a8.scalar_type() == at::kByte && a8.is_contiguous() && a8.numel() >= packed_numel(M, K),
           "a8: uint8 [packed_numel(M, K)]");
  const int64_t rows = ((M + 15) / 16) * 16;
  MP_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() >= rows * 33,
           "scale: fp32 [ceil(M/16)*16 * 33] (row scales + per-slice absmax scratch)");
  MP_CHECK(K % 64 == 0, "K % 64");
  check_launch(mp_quant_act_fp8(ap.data_ptr(), a8.data_ptr(), scale.data_ptr<float>(), scale.data_ptr<float>() + rows,
                                (int)M, (int)K, cur_stream()),
               "quant_act_fp8");
}

// packed bf16 activation (M rows, K) -> MX e4m3 bytes ax [K/128 * MT * 2 * 64 * 16] + e8m0 block
// scales as [K/128 * 64 * 4] (gemm_mx.hip)
void quant_mx(const at::Tensor& ap, at::Tensor& ax, at::Tensor& as, int64_t M, int64_t K) {
  check_bf16_cuda(ap, "ap");
  MP_CHECK(M >= 1 && M <= 64 && K % 128 == 0, "quant_mx: 1 <= M <= 64, K % 128 == 0");
  MP_CHECK(ap.is_contiguous() && ap.numel() >= packed_numel(M, K), "packed activation too small");
  const int64_t rows = ((M + 15) / 16) * 16;
  MP_CHECK(ax.is_cuda() && ax.scalar_type() == at::kByte && ax.is_contiguous() && ax.numel() >= rows * K,
           "ax: uint8 [ceil(M/16)*16*K]");
  MP_CHECK(as.is_cuda() && as.scalar_type() == at::kByte && as.is_contiguous() && as.numel() >= 2 * K,
           "as: uint8 [K/128 * 64 * 4]");
  check_launch(mp_quant_mx(ap.data_ptr(), ax.data_ptr(), as.data_ptr(), (int)M, (int)K, cur_stream()), "quant_mx");
}

// W8A8-MX decode GEMM (gemm_mx.hip): ax / as from quant_mx, fp8 weight in the W8A16 layout + column
// scales; epilogue 0 (optional ss_in row scale) or 3; flags bit 10 rotated k walk, bit 14 partial
// slabs only (y unused, the slabs stay in the workspace)
void gemm_mx(const at::Tensor& ax, const at::Tensor& as, const at::Tensor& wq, const at::Tensor& wsc, at::Tensor& y,
             const c10::optional<at::Tensor>& residual, int64_t epilogue, int64_t M_, int64_t flags,
             const at::Tensor& workspace, const c10::optional<at::Tensor>& ap,
             const c10::optional<at::Tensor>& ss_out, const c10::optional<at::Tensor>& ss_zero,
             const c10::optional<at::Tensor>& ss_in, double inv_k, double eps) {
  MP_CHECK(wq.is_cuda() && wq.scalar_type() == at::kByte && wq.dim() == 4 && wq.size(2) == 64 && wq.size(3) == 8 &&
               wq.is_contiguous(),
           "wq must be an fp8 weight uint8 [N/16, K/32, 64, 8] (ops.pack_weight_w8)");
  const int N = 16 * wq.size(0), K = 32 * wq.size(1);
  const int M = (int)M_;
  MP_CHECK(M >= 1 && M <= 64 && K % 128 == 0, "gemm_mx: 1 <= M <= 64, K % 128 == 0");
  const int64_t rows = ((M + 15) / 16) * 16;
  MP_CHECK(ax.is_cuda() && ax.scalar_type() == at::kByte && ax.is_contiguous() && ax.numel() >= rows * K, "ax size");
  MP_CHECK(as.is_cuda() && as.scalar_type() == at::kByte && as.is_contiguous() && as.numel() >= 2 * K, "as size");
  MP_CHECK(wsc.is_cuda() && wsc.scalar_type() == at::kFloat && wsc.is_contiguous() && wsc.numel() == N,
           "wsc: fp32 [N] column scales");
  MP_CHECK(epilogue == 0 || epilogue == 3, "gemm_mx: epilogue 0 or 3");
  const bool partial = flags & 16384;
  if (!partial) {
    check_bf16_cuda(y, "y");
    check_rows(y, "y");
    MP_CHECK(y.size(0) == M && y.size(1) == N, "y shape");
  }
  const void* rp = nullptr;
  int64_t rs = 0;
  if (residual.has_value()) {
    check_bf16_cuda(*residual, "residual");
    check_rows(*residual, "residual");
    MP_CHECK(residual->size(0) == M && residual->size(1) == N, "residual shape");
    rp = residual->data_ptr();
    rs = residual->stride(0);
  }
  void* app = nullptr;
  if (ap.has_value()) {
    check_bf16_cuda(*ap, "ap");
    MP_CHECK(ap->is_contiguous() && ap->numel() >= packed_numel(M, N), "ap: packed [ceil(M/16)*16*N]");
    app = ap->data_ptr();
  }
  MP_CHECK(epilogue != 3 || (app != nullptr && rp != nullptr), "epilogue 3 needs residual and ap");
  MP_CHECK(workspace.is_cuda() && workspace.is_contiguous() &&
               workspace.numel() * workspace.element_size() >= mp_gemm_workspace_bytes(),
           "gemm workspace too small (ops.gemm_workspace)");
  const int rc = mp_gemm_mx(ax.data_ptr(), as.data_ptr(), wq.data_ptr(), wsc.data_ptr<float>(),
                            partial ? nullptr : y.data_ptr(), partial ? 0 : y.stride(0), rp, rs, M, N, K,
                            (int)epilogue, (int)flags, workspace.data_ptr(), app, opt_ss(ss_out, "ss_out"),
                            opt_ss(ss_zero, "ss_zero"), opt_ss(ss_in, "ss_in"), (float)inv_k, (float)eps, cur_stream());
  TORCH_CHECK(rc != 1, "mpamd: gemm_mx: no split-K geometry for M=", M, " N=", N, " K=", K);
  check_launch(rc, "gemm_mx");
}

// row-major bf16 x[M, K] -> fp8 A8 (the fp8 GEMM's A layout) + per-row scales
void quant_rows_fp8(const at::Tensor& x, at::Tensor& a8, at::Tensor& scale) {
  check_bf16_cuda(x, "x");
  MP_CHECK(x.dim() == 2 && x.stride(1) == 1, "x: [M, K] with unit column stride");
  const int64_t M = x.size(0), K = x.size(1);
  MP_CHECK(a8.is_cuda() && a8.scalar_type() == at::kByte && a8.is_contiguous() && a8.numel() >= packed_numel(M, K),
           "a8: uint8 [packed_numel(M, K)]");
  MP_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() >= M, "scale: fp32 [>= M]");
  MP_CHECK(K % 64 == 0 && K <= 65536, "K % 64 == 0 and K <= 65536");
  check_launch(mp_quant_rows_fp8(x.data_ptr(), x.stride(0), a8.data_ptr(), scale.data_ptr<float>(), (int)M, (int)K,
                                 cur_stream()),
               "quant_rows_fp8");
}

// y = epilogue((a8 * as) . (wq * ws)^T); wq: [N/16, K/64, 64, 16] uint8 (ops.pack_weight_fp8)
void gemm_fp8(const at::Tensor& a8, const at::Tensor& as, const at::Tensor& wq, const at::Tensor& ws, at::Tensor& y,
              const c10::optional<at::Tensor>& residual, int64_t epilogue, int64_t M, int64_t out_packed,
              int64_t kind, const c10::optional<at::Tensor>& workspace) {
  MP_CHECK(wq.is_cuda() && wq.scalar_type() == at::kByte && wq.dim() == 4 && wq.size(2) == 64 && wq.size(3) == 16 &&
               wq.is_contiguous(),
           "wq must be a packed fp8 weight [N/16, K/64, 64, 16]");
  const int N = 16 * wq.size(0), K = 64 * wq.size(1);
  MP_CHECK(a8.is_cuda() && a8.scalar_type() == at::kByte && a8.numel() >= packed_numel(M, K), "a8");
  MP_CHECK(as.is_cuda() && as.scalar_type() == at::kFloat && as.numel() >= M, "as");
  MP_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.numel() == N, "ws: fp32 [N]");
  check_bf16_cuda(y, "y");
  const int ncols = epilogue == 1 ? N / 2 : N;
  if (out_packed) {
    MP_CHECK(epilogue == 1 && y.is_contiguous() && y.numel() >= packed_numel(M, ncols), "packed y");
  } else {
    check_rows(y, "y");
    MP_CHECK(y.size(0) == M && y.size(1) == ncols, "y shape");
  }
  const void* rp = nullptr;
  int64_t rs = 0;
  if (residual.has_value()) {
    check_bf16_cuda(*residual, "residual");
    check_rows(*residual, "residual");
    rp = residual->data_ptr();
    rs = residual->stride(0);
  }
  MP_CHECK(epilogue != 2 || rp != nullptr, "residual epilogue needs residual");
  float* part = nullptr;
  int64_t part_bytes = 0;
  if (workspace.has_value()) {  // the GEMM workspace (ops.gemm_workspace): its split-K slab region
    MP_CHECK(workspace->is_cuda() && workspace->is_contiguous() &&
                 workspace->numel() * workspace->element_size() >= mp_gemm_workspace_bytes(),
             "workspace: ops.gemm_workspace");
    part = (float*)((char*)workspace->data_ptr() + mp_gemm_slab_offset());
    part_bytes = mp_gemm_slab_bytes();
  }
  check_launch(mp_gemm_fp8(a8.data_ptr(), as.data_ptr<float>(), wq.data_ptr(), ws.data_ptr<float>(), y.data_ptr(),
                           out_packed ? 0 : y.stride(0), rp, rs, (int)M, N, K, (int)epilogue, (int)out_packed,
                           (int)kind, part, part_bytes, cur_stream()),
               "gemm_fp8");
}

}  // namespace

TORCH_LIBRARY(mpamd, m) {
  m.def("gemm_workspace_bytes() -> int", &gemm_workspace_bytes);
  m.def("gemm_slab_offset() -> int", &gemm_slab_offset);
  m.def("gemm_rwk_split(int M, int N, int K, int f8) -> int", &gemm_rwk_split);
  m.def("fp8_gemm_kernel(int kind) -> ()", &fp8_gemm_kernel);
  m.def("gemm_rw_ok(int M, int N, int K, int epilogue, int out_packed) -> bool", &gemm_rw_ok);
  m.def("gemm_t2d_ok(int M, int N, int K, int epilogue, int out_packed) -> bool", &gemm_t2d_ok);
  m.def(
      "rmsnorm(Tensor x, Tensor(a!) residual, Tensor w, Tensor(b!) y, float eps, int mode, Tensor? rows, "
      "int packed, Tensor(c!)? ss=None, Tensor(d!)? a8=None, Tensor(e!)? a8_scale=None, Tensor? gather=None) -> ()");
  m.def(
      "rope_kv_write(Tensor(a!) qkv, Tensor positions, Tensor cos, Tensor sin, Tensor(b!) k_cache, "
      "Tensor(c!) v_cache, Tensor slots, int nh, int nkv) -> ()");
  m.def("kv_write(Tensor k, Tensor v, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slots) -> ()");
  m.def(
      "paged_attention(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor q_seq, Tensor q_ctx, "
      "Tensor(a!) out, Tensor(b!) workspace, int nh, int nkv, float scale, int part_size, int num_parts, "
      "int packed, Tensor(c!)? counters=None) -> ()");
  m.def(
      "paged_attention_rope(Tensor qkv, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor block_tables, Tensor q_seq, "
      "Tensor q_ctx, Tensor positions, Tensor cos, Tensor sin, Tensor slots, Tensor(c!) out, Tensor(d!) workspace, "
      "int nh, int nkv, float scale, int part_size, int num_parts, int packed, Tensor(e!)? counters=None, "
      "Tensor? qkv_part=None, int part_splits=0, Tensor? part_ss=None, float inv_k=0., float eps=0.) -> ()");
  m.def(
      "attention_mfma(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor q_seq, Tensor q_ctx, "
      "Tensor qblocks, Tensor(a!) out, Tensor(b!) workspace, int nh, int nkv, float scale, int part_size, "
      "int num_parts, int packed, Tensor? superblocks=None) -> ()");
  m.def(
      "attention_fa(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor q_seq, Tensor q_ctx, "
      "Tensor fablocks, Tensor(a!) out, Tensor(b!) workspace, int nh, int nkv, float scale, int part_size, "
      "int num_parts, int waves, int pair=0) -> ()");
  m.def(
      "attention_mfma_rope(Tensor qkv, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor block_tables, Tensor q_seq, "
      "Tensor q_ctx, Tensor qblocks, Tensor positions, Tensor cos, Tensor sin, Tensor slots, Tensor(c!) out, "
      "Tensor(d!) workspace, int nh, int nkv, float scale, int part_size, int num_parts, int packed, "
      "Tensor? qkv_part=None, int part_splits=0, Tensor? part_ss=None, float inv_k=0., float eps=0., "
      "Tensor(e!)? mx_ax=None, Tensor(f!)? mx_as=None) -> ()");
  m.def("embedding(Tensor ids, Tensor table, Tensor(a!) out) -> ()");
  m.def("swiglu(Tensor gu, Tensor(a!) out) -> ()");
  m.def("add(Tensor a, Tensor b, Tensor(a!) y) -> ()");
  m.def("argmax(Tensor logits, Tensor(a!) out) -> ()");
  m.def(
      "sample(Tensor logits, Tensor temps, Tensor top_ps, Tensor top_ks, Tensor rep_pens, Tensor(c!) recent, "
      "Tensor(d!) recent_len, Tensor seeds, Tensor(a!) workspace, Tensor(b!) out, int update=0) -> ()");
  m.def(
      "gemm(Tensor x, Tensor wp, Tensor(a!) y, Tensor? residual, int epilogue, int M, int flags, "
      "Tensor(b!)? workspace=None, Tensor? gate=None, Tensor(c!)? ap=None, Tensor(d!)? ss_out=None, "
      "Tensor(e!)? ss_zero=None, Tensor? ss_in=None, float inv_k=0., float eps=0.) -> ()");
  m.def(
      "gemm_w8(Tensor x, Tensor wq, Tensor wsc, Tensor(a!) y, Tensor? residual, int epilogue, int M, int flags, "
      "Tensor(b!)? workspace=None, Tensor(c!)? ap=None, Tensor(d!)? ss_out=None, Tensor(e!)? ss_zero=None, "
      "Tensor? ss_in=None, float inv_k=0., float eps=0.) -> ()");
  m.def("pack_act(Tensor x, Tensor(a!) ap) -> ()");
  m.def("pack_weight(Tensor w) -> Tensor");
  m.def("quant_act_fp8(Tensor ap, Tensor(a!) a8, Tensor(b!) scale, int M, int K) -> ()");
  m.def("quant_rows_fp8(Tensor x, Tensor(a!) a8, Tensor(b!) scale) -> ()");
  m.def("quant_mx(Tensor ap, Tensor(a!) ax, Tensor(b!) as_, int M, int K) -> ()");
  m.def(
      "gemm_mx(Tensor ax, Tensor as_, Tensor wq, Tensor wsc, Tensor(a!) y, Tensor? residual, int epilogue, int M, "
      "int flags, Tensor(b!) workspace, Tensor(c!)? ap=None, Tensor(d!)? ss_out=None, Tensor(e!)? ss_zero=None, "
      "Tensor? ss_in=None, float inv_k=0., float eps=0.) -> ()");
  m.def(
      "gemm_fp8(Tensor a8, Tensor a_scale, Tensor wq, Tensor w_scale, Tensor(a!) y, Tensor? residual, int epilogue, "
      "int M, int out_packed, int kind=-1, Tensor(b!)? workspace=None) -> ()");
}

TORCH_LIBRARY_IMPL(mpamd, CUDA, m) {
  m.impl("rmsnorm", &rmsnorm);
  m.impl("rope_kv_write", &rope_kv_write);
  m.impl("kv_write", &kv_write);
  m.impl("paged_attention", &paged_attention);
  m.impl("paged_attention_rope", &paged_attention_rope);
  m.impl("attention_mfma", &attention_mfma);
  m.impl("attention_fa", &attention_fa);
  m.impl("attention_mfma_rope", &attention_mfma_rope);
  m.impl("embedding", &embedding);
  m.impl("swiglu", &swiglu);
  m.impl("add", &add);
  m.impl("argmax", &argmax);
  m.impl("sample", &sample);
  m.impl("gemm", &gemm);
  m.impl("gemm_w8", &gemm_w8);
  m.impl("pack_weight", &pack_weight);
  m.impl("pack_act", &pack_act);
  m.impl("quant_act_fp8", &quant_act_fp8);
  m.impl("quant_rows_fp8", &quant_rows_fp8);
  m.impl("quant_mx", &quant_mx);
  m.impl("gemm_mx", &gemm_mx);
  m.impl("gemm_fp8", &gemm_fp8);
}
