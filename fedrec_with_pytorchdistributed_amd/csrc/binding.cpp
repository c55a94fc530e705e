// torch.ops.fedrec.* registrations for the gfx950 kernels (TORCH_LIBRARY; no pybind).
//
// Each op validates shapes/dtypes on the host (a kernel never sees a shape it was not
// written for), allocates outputs with the caching allocator, and launches on the current
// HIP stream.  The kernels live in *.hip files compiled without torch headers; they export
// plain C launchers (fr_*) that return a non-zero code for an unsupported shape.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <algorithm>
#include <tuple>
#include <vector>

extern "C" {
void fr_gemm_set_variant(int v);
void fr_title_attn_set_waves(int w);
void fr_title_attn_bwd_set_variant(int v);
void fr_score_set_variant(int v);
void fr_ln_set_wide(int v);
int fr_gemm_nt_bf16(const void* A, const void* W, const float* bias, const void* R, void* C, int M, int N, int K, int act,
                    int c_rows, hipStream_t s);
int fr_layer_norm_bwd_bf16(const void* x, const float* w, const void* dy, void* dx, float* dw, float* db, int rows, int D,
                           float eps, hipStream_t s, float* dxs, void* dxz, float pdrop, unsigned long long seed,
                           unsigned long long offset);
int fr_gelu_bf16(const void* z, const void* dh, void* out, long n, int bwd, hipStream_t s);
int fr_title_attention_bwd_bf16(const void* qkv, const void* dout, const int* mask, void* dqkv, int n_titles, int T, int H,
                                int D, hipStream_t s);
int fr_layer_norm_bf16(const void* x, const float* w, const float* b, void* y, int rows, int D, float eps,
                       const void* res, hipStream_t s);
int fr_embed_ln_bf16(const int* tokens, const void* word, const void* pos, const float* w, const float* b, void* y,
                     int rows, int D, int T, float eps, hipStream_t s);
int fr_title_attention_bf16(const void* qkv, const int* mask, void* out, int n_titles, int T, int H, int D,
                            hipStream_t s);
int fr_additive_pool_fwd(const void* x, const void* e, const float* w2, const float* b2, float* out, float* alpha,
                         int n, int T, int D, int Q, int is_bf16, const int* keep, hipStream_t s);
int fr_additive_pool_rows(int T, int D, int Q, int is_bf16);
int fr_additive_pool_bwd(const void* x, const void* e, const float* alpha, const float* w2, const float* g, float* dx,
                         void* dpre, float* dw2, float* db2, float* dsum, int n, int T, int D, int Q, int R,
                         int is_bf16, hipStream_t s);
int fr_head_supported(int D, int Q, int T);
int fr_head_score(const void* table, const int* ids, int U, int T, int D, int Q, const void* W1, const float* b1,
                  const float* w2, const float* b2, void* e_out, float* a_out, const int* nreal, hipStream_t s);
int fr_head_score_slices(int Q);
int fr_head_pool(const void* table, const int* ids, const float* a, int slices, const int* tokens, int U, int T, int D,
                 float* pooled, float* alpha, const int* nreal, hipStream_t s,
                 void* pooled_b);
int fr_head_pool_bwd(const void* table, const int* ids, const float* alpha, const float* g, int U, int T, int D,
                     float* da, float* db2p, const int* nreal, hipStream_t s);
long fr_head_wgrad(const void* e, const void* table, const int* ids, const float* da, const float* db2p,
                   const float* w2, int U, int T, int D, int Q, float* dW1, float* db1, float* dw2, float* db2,
                   float* scratch, const int* nreal, hipStream_t s);
int fr_head_g_supported(int D, int Q, int T);
int fr_head_pool_bwd_g(const void* table, const int* ids, const float* alpha, const float* g, int U, int T, int D,
                       int Q, float* da, float* db2p, void* e, float* cs, const int* nreal, hipStream_t s);
long fr_head_wgrad_g(const void* G, const void* table, const int* ids, const float* cs, const float* db2p,
                     const float* w2, int U, int T, int D, int Q, float* dW1, float* db1, float* dw2, float* db2,
                     float* scratch, const int* nreal, hipStream_t s, const void* pend, int pend_cblocks,
                     int pend_total);
void fr_head_wgrad_g_set_kt(int kt);
int fr_ipc_create(long cap, void* handle_out);
int fr_ipc_open(int id, const void* handles, int me, int W, const long long* local_ptrs);
long long fr_ipc_region(int id);
int* fr_ipc_status(int id);
int fr_ipc_allreduce(int id, void* x, long n, int is_int, long long epoch, int mode, int blocks, double timeout_s,
                     hipStream_t s);
int fr_ipc_destroy(int id);
int fr_ipc_allreduce_local(const int* ids, void* const* xs, int W, long n, int is_int, long long epoch, int mode,
                           int blocks, double timeout_s, hipStream_t s);
int fr_user_attn_fwd(const float* qkv, float* ctx, float* stats, int B, int H, int NH, int dk, const int* keep,
                     hipStream_t s, void* ctx_b);
int fr_user_qkv_attn_fwd(const void* xd, const void* W, const float* bias, int Din, float* qkv, float* ctx,
                         float* stats, int B, int H, int NH, int dk, const int* keep, hipStream_t s, void* ctx_b);
int fr_user_attn_bwd_dctx(const float* qkv, const float* stats, const float* dctx, void* dqkv, const void* dpre,
                          const void* w1t, int Qd, int B, int H, int NH, int dk, const int* keep, hipStream_t s);
int fr_user_attn_bwd(const float* qkv, const float* stats, const float* dctx, void* dqkv, int B, int H, int NH,
                     int dk, const int* keep, hipStream_t s, int out_bf16);
int fr_score_ce(const float* cand, const float* user, float* loss, float* scores, float* dcand, float* duser, int B,
                int C, int D, int sigm, const int* ci, float* loss_total, hipStream_t s);
int fr_segment_sum_rows(const float* rows, const int* perm, const int* seg_ptr, const int* inv, float* out, int U, int D,
                        int R, float* scratch, hipStream_t s, int zero_empty);
int fr_segsum_chunks(int R);
void fr_segsum_set_variant(int v);
void fr_segsum_set_ldp_block(int v);
void fr_small_gemm_set_rd(int v);
int fr_user_pool_score(const float* x, const float* e, const float* w2, const float* b2, const int* keep,
                       const float* cand, const int* ci, int B, int T, int D, int Q, int C, int sigm, float* lossb,
                       float* scores, float* dcand, float* loss_total, float* dctx, float* dpre, void* dpre_b,
                       float* da8, hipStream_t s);
void fr_head_score_set_rows(int r);
void fr_head_score_set_ilv(int v);
int fr_segment_sum_rows_ldp(const float* rows, const int* perm, const int* seg_ptr, const int* inv, float* out, int U,
                            int D, int R, float* scratch, float clip, float noise_std, unsigned long long seed,
                            unsigned long long offset, const unsigned long long* dev_off, hipStream_t s);
int fr_ldp_rows(const float* rows, float* out, int R, int D, float clip, float noise_std, unsigned long long seed,
                unsigned long long offset, hipStream_t s, const unsigned long long* dev_off);
int fr_adam_dev(float* p, float* g, float* m, float* v, void* plow, long n, float lr, float b1, float b2, float eps,
                float grad_scale, const long long* step, const float* loss, float* ring, int ring_n, hipStream_t s,
                int nseg, const float* const* gsrc, const long* goff, const long* gn, const int* skip);
int fr_adam_flat(float* p, const float* g, float* m, float* v, void* plow, long n, float lr, float b1, float b2,
                 float eps, float bc1, float bc2, float grad_scale, hipStream_t s);
int fr_sample_batch(const int* rows, const int* pos, const long long* neg_ptr, const int* negs, const long long* his_ptr,
                    const int* his, int* cand, int* hout, int B, int npr, int H, int truncate, unsigned long long seed,
                    unsigned long long offset, int valid, hipStream_t s);
int fr_dedup(const int* ids, int R, int num_news, int* uniq, int* inv, int* perm, int* seg_ptr, int* u_count,
             hipStream_t s);
int fr_secagg_mask(const float* x, int* out, long n, float scale, float clipv, const unsigned long long* seeds,
                   const int* signs, int npeers, unsigned long long round, hipStream_t s);
int fr_secagg_unmask(const int* x, float* out, long n, float inv_scale, hipStream_t s);
int fr_title_plan(const int* mask, int n, int T, int* rowmap, int* src, int* kv_start, int* kv_len, int* qstart,
                  int* n_kv, hipStream_t s);
int fr_title_attention_packed_bf16(const void* qkv, const int* rowmap, const int* kv_start, const int* kv_len,
                                   const int* qstart, void* out, int n_titles, int T, int H, int D, hipStream_t s);
int fr_gemm_nt_bf16_split(const void* A, const void* W, const float* bias, void* C, int M, int N, int K, int c_rows,
                          const int* full_rows, int n_partial, hipStream_t s);
int fr_embed_ln_rows_bf16(const int* tokens, const int* src, const void* word, const void* pos, const float* w,
                          const float* b, void* y, int rows, int D, int T, float eps, hipStream_t s);
int fr_layer_norm_scatter_bf16(const void* x, const float* w, const float* b, void* y, int rows, int D, float eps,
                               const void* res, const int* dst, hipStream_t s);
int fr_colsum_bf16(const void* x, int M, int N, float* partial, float* out, hipStream_t s, int ld);
int fr_gelu_bwd_colsum_bf16(const void* df, const void* z, void* dz, int M, int N, float* partial, float* out,
                            hipStream_t s);
int fr_gemm_gelu_bwd_colpart(const void* A, const void* W, const void* Z, void* C, float* colpart, int M, int N, int K,
                             int c_rows, hipStream_t s);
int fr_colsum_chunks();
int fr_gemm_nt_bf16_dual(const void* A, const void* W, const float* bias, void* C, void* Z, int M, int N, int K,
                         int c_rows, hipStream_t s);
int fr_embed_grad_bf16(const void* dx, const int* sorted, const int* perm, int R, int D, float* dword, int* scratch,
                       hipStream_t s);
int fr_secagg_hist(const float* x, long n, unsigned* scratch, int* out, const unsigned long long* seeds,
                   const int* signs, int npeers, unsigned long long round, hipStream_t s);
int fr_secagg_mask_exact(const float* x, int* out, long n, const int* H, int W, const unsigned long long* seeds,
                         const int* signs, int npeers, unsigned long long round, hipStream_t s);
int fr_secagg_unmask_exact(const int* x, float* out, long n, const int* H, int W, hipStream_t s);
long fr_small_gemm(const void* const* ptrs, const int* ints, const float* floats, const unsigned long long* seeds,
                   const unsigned long long* dev_off, int n, float* scratch, int tile, hipStream_t s);
void fr_small_gemm_set_defer(int on);
int fr_small_gemm_has_pending();
int fr_small_gemm_batch_bytes();
int fr_small_gemm_take_pending(void* dst, int dst_bytes, int* c_blocks, int* total);
int fr_small_gemm_flush_pending(hipStream_t s);
int fr_multi_cast(const float* const* src, void* const* dst, const long* n, const int* to_bf16, int nseg,
                  long long* bump, hipStream_t s, long long* bump2, const long* nsrc, const int* fill, int ntseg,
                  const float* const* tsrc, void* const* tdst, const int* tR, const int* tC, const int* tld);
int fr_multi_cast_t(const float* const* src, void* const* dst, const int* R, const int* C, const int* ld, int nseg,
                    hipStream_t s);
int fr_multi_copy(const int* const* src, int* const* dst, const long* nsrc, const long* ndst, const int* fill, int n,
                  hipStream_t s);
long fr_colsum_f32(const float* const* xs, float* const* outs, const int* ints, int n, float* part, hipStream_t s);
int fr_upool_bwd_da(const float* x, const float* e, const float* alpha, const float* w2, const float* g, float* dx,
                    float* dpre, float* da8, int n, int T, int D, int Q, hipStream_t s, void* dpre_b);
int fr_dropout_add_bf16(const void* h, const void* res, void* out, long n, float p, unsigned long long seed,
                        unsigned long long offset, hipStream_t s);
int fr_title_attention_drop_bf16(const void* qkv, const int* mask, void* out, int n_titles, int T, int H, int D,
                                 float pdrop, unsigned long long seed, unsigned long long offset, hipStream_t s);
int fr_title_attention_bwd_drop_bf16(const void* qkv, const void* dout, const int* mask, void* dqkv, int n_titles,
                                     int T, int H, int D, float pdrop, unsigned long long seed,
                                     unsigned long long offset, hipStream_t s);
int fr_gather_dropout(const float* v, const int* idx, void* out, int out_bf16, int M, int K, float p,
                      unsigned long long seed, unsigned long long offset, const unsigned long long* dev_off,
                      hipStream_t s);
long fr_wgrad_bf16(const void* dY, const void* X, float* C, float* scratch, int M, int N, int K, int accumulate,
                   hipStream_t s);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "fedrec: ", name, " must be a device tensor");
  TORCH_CHECK(t.is_contiguous(), "fedrec: ", name, " must be contiguous");
}

void check_rc(int rc, const char* op) { TORCH_CHECK(rc == 0, "fedrec::", op, ": unsupported shape (code ", rc, ")"); }

at::Tensor linear(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b, int64_t act,
                  const c10::optional<at::Tensor>& residual) {
  check_dev(x, "x");
  check_dev(w, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "fedrec::linear: bf16 x/w");
  const c10::DeviceGuard g(x.device());
  const int64_t K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "fedrec::linear: K mismatch");
  const int64_t M = x.numel() / K;
  auto out_shape = x.sizes().vec();
  out_shape.back() = N;
  // rows padded to the 256-row tile: the GEMM epilogue then stores without a row predicate
  const int64_t c_rows = (M + 255) / 256 * 256;
  auto out = at::empty({c_rows * N}, x.options()).narrow(0, 0, M * N).view(out_shape);
  const float* bp = nullptr;
  at::Tensor bf;
  if (b.has_value() && b->defined()) {
    bf = b->to(at::kFloat).contiguous();
    TORCH_CHECK(bf.numel() == N, "fedrec::linear: bias size");
    bp = bf.data_ptr<float>();
  }
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    check_dev(*residual, "residual");
    TORCH_CHECK(residual->scalar_type() == at::kBFloat16 && residual->numel() == M * N, "fedrec::linear: residual");
    rp = residual->data_ptr();
  }
  if (M == 0) return out;
  check_rc(fr_gemm_nt_bf16(x.data_ptr(), w.data_ptr(), bp, rp, out.data_ptr(), (int)M, (int)N, (int)K, (int)act,
                           (int)c_rows, cur_stream()),
           "linear");
  return out;
}

at::Tensor layer_norm(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, double eps,
                      const c10::optional<at::Tensor>& residual) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "fedrec::layer_norm: bf16");
  const c10::DeviceGuard g(x.device());
  const int64_t D = x.size(-1);
  auto wf = w.to(at::kFloat).contiguous(), bf = b.to(at::kFloat).contiguous();
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    check_dev(*residual, "residual");
    TORCH_CHECK(residual->scalar_type() == at::kBFloat16 && residual->numel() == x.numel(),
                "fedrec::layer_norm: residual must match x (bf16)");
    rp = residual->data_ptr();
  }
  auto y = at::empty_like(x);
  check_rc(fr_layer_norm_bf16(x.data_ptr(), wf.data_ptr<float>(), bf.data_ptr<float>(), y.data_ptr(),
                              (int)(x.numel() / D), (int)D, (float)eps, rp, cur_stream()),
           "layer_norm");
  return y;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> layer_norm_bwd_impl(const at::Tensor& x, const at::Tensor& w,
                                                                             const at::Tensor& dy, double eps,
                                                                             bool want_dxsum) {
  check_dev(x, "x");
  check_dev(dy, "dy");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16, "fedrec::layer_norm_bwd: bf16");
  const c10::DeviceGuard g(x.device());
  const int64_t D = x.size(-1);
  auto wf = w.to(at::kFloat).contiguous();
  auto dx = at::empty_like(x);
  // the kernel accumulates dw / db (/ dx column sums) across row blocks: one zeroed buffer,
  // one fill launch (three at::zeros were 75 fill launches per config-5 step)
  auto acc = at::zeros({want_dxsum ? 3 : 2, D}, x.options().dtype(at::kFloat));
  auto dw = acc[0];
  auto db = acc[1];
  at::Tensor dxs = want_dxsum ? acc[2] : at::Tensor();
  check_rc(fr_layer_norm_bwd_bf16(x.data_ptr(), wf.data_ptr<float>(), dy.data_ptr(), dx.data_ptr(), dw.data_ptr<float>(),
                                  db.data_ptr<float>(), (int)(x.numel() / D), (int)D, (float)eps, cur_stream(),
                                  want_dxsum ? dxs.data_ptr<float>() : nullptr, nullptr, 0.f, 0ull, 0ull),
           "layer_norm_bwd");
  return {dx, dw, db, dxs};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> layer_norm_bwd(const at::Tensor& x, const at::Tensor& w,
                                                               const at::Tensor& dy, double eps) {
  auto r = layer_norm_bwd_impl(x, w, dy, eps, false);
  return {std::get<0>(r), std::get<1>(r), std::get<2>(r)};
}

// + the column sums of dx (bias gradient of the layer feeding the LayerNorm)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> layer_norm_bwd_colsum(const at::Tensor& x,
                                                                                 const at::Tensor& w,
                                                                                 const at::Tensor& dy, double eps) {
  return layer_norm_bwd_impl(x, w, dy, eps, true);
}

// + the dropout backward of the layer feeding the LayerNorm: (dx, dx o Z, dw, db, colsum(dx o Z))
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> layer_norm_bwd_drop(
    const at::Tensor& x, const at::Tensor& w, const at::Tensor& dy, double eps, double p, int64_t seed, int64_t offset) {
  check_dev(x, "x");
  check_dev(dy, "dy");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16, "fedrec::layer_norm_bwd_drop: bf16");
  TORCH_CHECK(x.is_contiguous() && dy.is_contiguous() && dy.numel() == x.numel(), "fedrec::layer_norm_bwd_drop: shapes");
  const c10::DeviceGuard g(x.device());
  const int64_t D = x.size(-1);
  auto wf = w.to(at::kFloat).contiguous();
  auto dx = at::empty_like(x);
  auto dxz = at::empty_like(x);
  auto acc = at::zeros({3, D}, x.options().dtype(at::kFloat));
  check_rc(fr_layer_norm_bwd_bf16(x.data_ptr(), wf.data_ptr<float>(), dy.data_ptr(), dx.data_ptr(),
                                  acc[0].data_ptr<float>(), acc[1].data_ptr<float>(), (int)(x.numel() / D), (int)D,
                                  (float)eps, cur_stream(), acc[2].data_ptr<float>(), dxz.data_ptr(), (float)p,
                                  (unsigned long long)seed, (unsigned long long)offset),
           "layer_norm_bwd_drop");
  return {dx, dxz, acc[0], acc[1], acc[2]};
}

at::Tensor gelu(const at::Tensor& z, const c10::optional<at::Tensor>& dh) {
  check_dev(z, "z");
  TORCH_CHECK(z.scalar_type() == at::kBFloat16, "fedrec::gelu: bf16");
  const c10::DeviceGuard g(z.device());
  auto out = at::empty_like(z);
  const void* dp = nullptr;
  if (dh.has_value() && dh->defined()) {
    check_dev(*dh, "dh");
    TORCH_CHECK(dh->scalar_type() == at::kBFloat16 && dh->numel() == z.numel(), "fedrec::gelu: dh");
    dp = dh->data_ptr();
  }
  check_rc(fr_gelu_bf16(z.data_ptr(), dp, out.data_ptr(), (long)z.numel(), dp ? 1 : 0, cur_stream()), "gelu");
  return out;
}

at::Tensor title_attention_bwd(const at::Tensor& qkv, const at::Tensor& dout, const at::Tensor& mask, int64_t n_heads) {
  check_dev(qkv, "qkv");
  check_dev(dout, "dout");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && dout.scalar_type() == at::kBFloat16, "fedrec::title_attention_bwd");
  const c10::DeviceGuard g(qkv.device());
  auto mk = mask.to(at::kInt).contiguous();
  const int64_t n = mk.size(0), T = mk.size(1), D = qkv.size(-1) / 3;
  auto dqkv = at::empty_like(qkv);
  check_rc(fr_title_attention_bwd_bf16(qkv.data_ptr(), dout.data_ptr(), mk.data_ptr<int>(), dqkv.data_ptr(), (int)n,
                                       (int)T, (int)n_heads, (int)D, cur_stream()),
           "title_attention_bwd");
  return dqkv;
}

// ---- dropout (backbone train mode; dropout.hip, title_attn*.hip) ------------------------------
at::Tensor dropout_add(const at::Tensor& h, const c10::optional<at::Tensor>& res, double p, int64_t seed,
                       int64_t offset) {
  check_dev(h, "h");
  TORCH_CHECK(h.scalar_type() == at::kBFloat16, "fedrec::dropout_add: bf16");
  const c10::DeviceGuard g(h.device());
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_dev(*res, "res");
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->numel() == h.numel(), "fedrec::dropout_add: res");
    rp = res->data_ptr();
  }
  auto out = at::empty_like(h);
  check_rc(fr_dropout_add_bf16(h.data_ptr(), rp, out.data_ptr(), (long)h.numel(), (float)p, (unsigned long long)seed,
                               (unsigned long long)offset, cur_stream()),
           "dropout_add");
  return out;
}

at::Tensor title_attention_drop(const at::Tensor& qkv, const at::Tensor& mask, int64_t n_heads, double p, int64_t seed,
                                int64_t offset) {
  check_dev(qkv, "qkv");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16, "fedrec::title_attention_drop: bf16");
  const c10::DeviceGuard g(qkv.device());
  auto mk = mask.to(at::kInt).contiguous();
  const int64_t n = mk.size(0), T = mk.size(1), D = qkv.size(-1) / 3;
  TORCH_CHECK(qkv.numel() == n * T * 3 * D, "fedrec::title_attention_drop: qkv shape");
  auto out = at::empty({n * T, D}, qkv.options());
  check_rc(fr_title_attention_drop_bf16(qkv.data_ptr(), mk.data_ptr<int>(), out.data_ptr(), (int)n, (int)T,
                                        (int)n_heads, (int)D, (float)p, (unsigned long long)seed,
                                        (unsigned long long)offset, cur_stream()),
           "title_attention_drop");
  return out;
}

at::Tensor title_attention_bwd_drop(const at::Tensor& qkv, const at::Tensor& dout, const at::Tensor& mask,
                                    int64_t n_heads, double p, int64_t seed, int64_t offset) {
  check_dev(qkv, "qkv");
  check_dev(dout, "dout");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && dout.scalar_type() == at::kBFloat16,
              "fedrec::title_attention_bwd_drop");
  const c10::DeviceGuard g(qkv.device());
  auto mk = mask.to(at::kInt).contiguous();
  const int64_t n = mk.size(0), T = mk.size(1), D = qkv.size(-1) / 3;
  TORCH_CHECK(qkv.numel() == n * T * 3 * D && dout.numel() == n * T * D, "fedrec::title_attention_bwd_drop: shapes");
  auto dqkv = at::empty_like(qkv);
  check_rc(fr_title_attention_bwd_drop_bf16(qkv.data_ptr(), dout.data_ptr(), mk.data_ptr<int>(), dqkv.data_ptr(),
                                            (int)n, (int)T, (int)n_heads, (int)D, (float)p, (unsigned long long)seed,
                                            (unsigned long long)offset, cur_stream()),
           "title_attention_bwd_drop");
  return dqkv;
}

at::Tensor embed_ln(const at::Tensor& tokens, const at::Tensor& word, const at::Tensor& pos, const at::Tensor& w,
                    const at::Tensor& b, double eps) {
  check_dev(word, "word");
  check_dev(pos, "pos");
  TORCH_CHECK(word.scalar_type() == at::kBFloat16 && pos.scalar_type() == at::kBFloat16, "fedrec::embed_ln: bf16");
  const c10::DeviceGuard g(word.device());
  auto tok = tokens.to(at::kInt).contiguous();
  TORCH_CHECK(tok.dim() == 2, "fedrec::embed_ln: tokens [n, T]");
  const int64_t n = tok.size(0), T = tok.size(1), D = word.size(1);
  TORCH_CHECK(T <= pos.size(0), "fedrec::embed_ln: T > max positions");
  auto wf = w.to(at::kFloat).contiguous(), bf = b.to(at::kFloat).contiguous();
  auto y = at::empty({n * T, D}, word.options());
  check_rc(fr_embed_ln_bf16(tok.data_ptr<int>(), word.data_ptr(), pos.data_ptr(), wf.data_ptr<float>(),
                            bf.data_ptr<float>(), y.data_ptr(), (int)(n * T), (int)D, (int)T, (float)eps, cur_stream()),
           "embed_ln");
  return y;
}

at::Tensor title_attention(const at::Tensor& qkv, const at::Tensor& mask, int64_t n_heads) {
  check_dev(qkv, "qkv");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16, "fedrec::title_attention: bf16");
  const c10::DeviceGuard g(qkv.device());
  auto mk = mask.to(at::kInt).contiguous();
  const int64_t n = mk.size(0), T = mk.size(1), D = qkv.size(-1) / 3;
  TORCH_CHECK(qkv.numel() == n * T * 3 * D, "fedrec::title_attention: qkv shape");
  auto out = at::empty({n * T, D}, qkv.options());
  check_rc(fr_title_attention_bf16(qkv.data_ptr(), mk.data_ptr<int>(), out.data_ptr(), (int)n, (int)T, (int)n_heads,
                                   (int)D, cur_stream()),
           "title_attention");
  return out;
}

// keep: optional [B, H] int32 mask (nonzero = attend / pool), the mask_padding option
const int* key_mask_ptr(const c10::optional<at::Tensor>& keep, int64_t B, int64_t H, const char* what) {
  if (!keep.has_value() || !keep->defined()) return nullptr;
  check_dev(*keep, "keep");
  TORCH_CHECK(keep->scalar_type() == at::kInt && keep->is_contiguous() && keep->numel() == B * H, "fedrec::", what,
              ": keep int32 [B, H]");
  return keep->data_ptr<int>();
}

std::tuple<at::Tensor, at::Tensor> additive_pool_fwd(const at::Tensor& x, const at::Tensor& e, const at::Tensor& w2,
                                                     const at::Tensor& b2, const c10::optional<at::Tensor>& keep) {
  check_dev(x, "x");
  check_dev(e, "e");
  TORCH_CHECK(x.dim() == 3 && e.dim() == 3 && x.scalar_type() == e.scalar_type(), "fedrec::additive_pool_fwd");
  const c10::DeviceGuard g(x.device());
  const int64_t n = x.size(0), T = x.size(1), D = x.size(2), Q = e.size(2);
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || x.scalar_type() == at::kFloat, "fedrec::additive_pool_fwd: dtype");
  auto out = at::empty({n, D}, x.options().dtype(at::kFloat));
  auto alpha = at::empty({n, T}, x.options().dtype(at::kFloat));
  check_rc(fr_additive_pool_fwd(x.data_ptr(), e.data_ptr(), w2.data_ptr<float>(), b2.data_ptr<float>(),
                                out.data_ptr<float>(), alpha.data_ptr<float>(), (int)n, (int)T, (int)D, (int)Q, bf,
                                key_mask_ptr(keep, n, T, "additive_pool_fwd"), cur_stream()),
           "additive_pool_fwd");
  return {out, alpha};
}

// ---- fused text head over gathered hidden states (text_head.hip) ----------------------------
// table [rows, D] bf16 (the HBM hidden-state cache viewed as rows, or a batch's hidden states);
// ids [U] int32 title indices (None: titles 0..U-1 of the table); T tokens per title.
namespace {
int64_t head_titles(const at::Tensor& table, const c10::optional<at::Tensor>& ids, int64_t T) {
  check_dev(table, "table");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous() && table.scalar_type() == at::kBFloat16,
              "fedrec::head: table [rows, D] contiguous bf16");
  TORCH_CHECK(T >= 1 && table.size(0) % T == 0, "fedrec::head: table rows not a multiple of T");
  if (ids.has_value()) {
    check_dev(*ids, "ids");
    TORCH_CHECK(ids->dim() == 1 && ids->is_contiguous() && ids->scalar_type() == at::kInt, "fedrec::head: ids int32 [U]");
    return ids->size(0);
  }
  return table.size(0) / T;
}
const int* opt_int_ptr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr<int>() : nullptr; }

// the text-head ops' optional device count of REAL titles (a padded step graph: titles past it
// are skipped, their outputs zero): int32 [1] on the table's device
const int* opt_nreal(const c10::optional<at::Tensor>& t, const at::Tensor& table) {
  if (!t.has_value()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kInt && t->numel() == 1 && t->device() == table.device(),
              "fedrec::head_*: nreal int32 [1] on the table's device");
  return t->data_ptr<int>();
}
}  // namespace

// ---- peer-to-peer all-reduce over IPC-mapped buffers (ipc_allreduce.hip) --------------------
std::tuple<int64_t, at::Tensor> ipc_create(int64_t cap) {
  auto h = at::empty({64}, at::TensorOptions().dtype(at::kByte));
  const int id = fr_ipc_create((long)cap, h.data_ptr());
  TORCH_CHECK(id >= 0, "fedrec::ipc_create failed (code ", id, ")");
  return {id, h};
}

void ipc_open(int64_t id, const at::Tensor& handles, int64_t me, int64_t W, const c10::optional<at::Tensor>& local) {
  TORCH_CHECK(!handles.is_cuda() && handles.scalar_type() == at::kByte && handles.numel() == 64 * W &&
                  handles.is_contiguous(),
              "fedrec::ipc_open: handles uint8 [W*64] on the host");
  const long long* lp = nullptr;
  at::Tensor lc;
  if (local.has_value()) {
    lc = local->to(at::kLong).contiguous();
    TORCH_CHECK(!lc.is_cuda() && lc.numel() == W, "fedrec::ipc_open: local_ptrs int64 [W] on the host");
    lp = (const long long*)lc.data_ptr<int64_t>();
  }
  const int rc = fr_ipc_open((int)id, handles.data_ptr(), (int)me, (int)W, lp);
  TORCH_CHECK(rc == 0, "fedrec::ipc_open failed (code ", rc, ")");
}

int64_t ipc_region(int64_t id) { return (int64_t)fr_ipc_region((int)id); }

// the context's status word as a device tensor view (no ownership; valid until ipc_destroy):
// the in-graph Adam reads it to skip the update of a step whose all-reduce timed out
at::Tensor ipc_status_word(int64_t id) {
  int* st = fr_ipc_status((int)id);
  TORCH_CHECK(st != nullptr, "fedrec::ipc_status_word: bad id");
  int dev = 0;
  TORCH_CHECK(hipPointerGetAttribute(&dev, HIP_POINTER_ATTRIBUTE_DEVICE_ORDINAL, (hipDeviceptr_t)st) == hipSuccess,
              "fedrec::ipc_status_word: pointer attribute");
  return at::from_blob(st, {1}, at::TensorOptions().dtype(at::kInt).device(at::Device(at::kCUDA, dev)));
}

int64_t ipc_status(int64_t id) {  // device -> host read (tests / diagnostics only)
  int* st = fr_ipc_status((int)id);
  TORCH_CHECK(st != nullptr, "fedrec::ipc_status: bad id");
  int v = 0;
  TORCH_CHECK(hipMemcpy(&v, st, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess, "fedrec::ipc_status: copy");
  return v;
}

void ipc_allreduce_(int64_t id, at::Tensor x, int64_t epoch, int64_t mode, int64_t blocks, double timeout_s) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kInt) && x.numel() % 4 == 0,
              "fedrec::ipc_allreduce_: contiguous fp32 / int32, numel % 4 == 0");
  const c10::DeviceGuard g(x.device());
  check_rc(fr_ipc_allreduce((int)id, x.data_ptr(), (long)x.numel(), x.scalar_type() == at::kInt ? 1 : 0,
                            (long long)epoch, (int)mode, (int)blocks, timeout_s, cur_stream()),
           "ipc_allreduce_");
}

void ipc_destroy(int64_t id) { (void)fr_ipc_destroy((int)id); }

// single-process rehearsal: every rank's context + tensor, one launch playing all ranks
void ipc_allreduce_local_(at::IntArrayRef ids, at::TensorList xs, int64_t epoch, int64_t mode, int64_t blocks,
                          double timeout_s) {
  TORCH_CHECK(ids.size() == xs.size() && !xs.empty() && xs.size() <= 16, "fedrec::ipc_allreduce_local_: W tensors");
  std::vector<int> iv(ids.begin(), ids.end());
  std::vector<void*> pv;
  for (const auto& x : xs) {
    check_dev(x, "x");
    TORCH_CHECK(x.is_contiguous() && x.scalar_type() == xs[0].scalar_type() && x.numel() == xs[0].numel() &&
                    (x.scalar_type() == at::kFloat || x.scalar_type() == at::kInt) && x.numel() % 4 == 0,
                "fedrec::ipc_allreduce_local_: contiguous fp32 / int32 tensors of one size, numel % 4 == 0");
    pv.push_back(x.data_ptr());
  }
  const c10::DeviceGuard g(xs[0].device());
  check_rc(fr_ipc_allreduce_local(iv.data(), pv.data(), (int)xs.size(), (long)xs[0].numel(),
                                  xs[0].scalar_type() == at::kInt ? 1 : 0, (long long)epoch, (int)mode, (int)blocks,
                                  timeout_s, cur_stream()),
           "ipc_allreduce_local_");
}

bool head_supported(int64_t D, int64_t Q, int64_t T) { return fr_head_supported((int)D, (int)Q, (int)T) != 0; }

std::tuple<at::Tensor, at::Tensor> head_score(const at::Tensor& table, const c10::optional<at::Tensor>& ids, int64_t T,
                                              const at::Tensor& w1, const at::Tensor& b1, const at::Tensor& w2,
                                              const at::Tensor& b2, bool store_e,
                                              const c10::optional<at::Tensor>& nreal) {
  const int64_t U = head_titles(table, ids, T), D = table.size(1), Q = w1.size(0);
  check_dev(w1, "w1");
  TORCH_CHECK(w1.scalar_type() == at::kBFloat16 && w1.is_contiguous() && w1.size(1) == D, "fedrec::head_score: w1 bf16 [Q, D]");
  TORCH_CHECK(b1.scalar_type() == at::kFloat && w2.scalar_type() == at::kFloat && b2.scalar_type() == at::kFloat &&
                  b1.numel() == Q && w2.numel() == Q && b2.numel() == 1 && b1.is_contiguous() && w2.is_contiguous() &&
                  b1.is_cuda() && w2.is_cuda() && b2.is_cuda(),
              "fedrec::head_score: b1 / w2 [Q], b2 [1] fp32 device");
  TORCH_CHECK(fr_head_supported((int)D, (int)Q, (int)T), "fedrec::head_score: unsupported shape D=", D, " Q=", Q, " T=", T);
  // (ids are not range-checked here: that needs a device->host read every step; the engine's
  // ids come from the dedup over [0, N) by construction)
  const c10::DeviceGuard g(table.device());
  auto e = store_e ? at::empty({U * T, Q}, table.options()) : at::empty({0}, table.options());
  // [slices, U*T]: partial scores per Q slice of the tiling (summed by head_pool); 1 slice -> [U*T]
  const int slices = fr_head_score_slices((int)Q);
  auto a = slices > 1 ? at::empty({slices, U * T}, table.options().dtype(at::kFloat))
                      : at::empty({U * T}, table.options().dtype(at::kFloat));
  check_rc(fr_head_score(table.data_ptr(), opt_int_ptr(ids), (int)U, (int)T, (int)D, (int)Q, w1.data_ptr(),
                         b1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(),
                         store_e ? e.data_ptr() : nullptr, a.data_ptr<float>(), opt_nreal(nreal, table), cur_stream()),
           "head_score");
  return {e, a};
}

// want_bf16: also the pooled rows rounded to bf16 (the fc GEMM's operand; empty otherwise)
std::tuple<at::Tensor, at::Tensor, at::Tensor> head_pool(const at::Tensor& table, const c10::optional<at::Tensor>& ids,
                                                         int64_t T, const at::Tensor& a,
                                                         const c10::optional<at::Tensor>& tokens,
                                                         const c10::optional<at::Tensor>& nreal, bool want_bf16) {
  const int64_t U = head_titles(table, ids, T), D = table.size(1);
  check_dev(a, "a");
  TORCH_CHECK(a.scalar_type() == at::kFloat && (a.numel() == U * T || (a.dim() == 2 && a.size(0) == 2 && a.size(1) == U * T)) &&
                  a.is_contiguous(),
              "fedrec::head_pool: a [U*T] (or [2, U*T] score partials) fp32");
  if (tokens.has_value()) {
    check_dev(*tokens, "tokens");
    TORCH_CHECK(tokens->scalar_type() == at::kInt && tokens->dim() == 3 && tokens->size(1) == 2 &&
                    tokens->size(2) == T && tokens->is_contiguous() && tokens->size(0) * T >= table.size(0),
                "fedrec::head_pool: tokens int32 [N, 2, T] covering the table");
  }
  const c10::DeviceGuard g(table.device());
  auto pooled = at::empty({U, D}, a.options());
  auto alpha = at::empty({U, T}, a.options());
  auto pooled_b = at::empty({want_bf16 ? U : 0, D}, a.options().dtype(at::kBFloat16));
  check_rc(fr_head_pool(table.data_ptr(), opt_int_ptr(ids), a.data_ptr<float>(), a.dim() == 2 ? (int)a.size(0) : 1,
                        opt_int_ptr(tokens), (int)U, (int)T,
                        (int)D, pooled.data_ptr<float>(), alpha.data_ptr<float>(), opt_nreal(nreal, table), cur_stream(),
                        want_bf16 ? pooled_b.data_ptr() : nullptr),
           "head_pool");
  return {pooled, alpha, pooled_b};
}

std::tuple<at::Tensor, at::Tensor> head_pool_bwd(const at::Tensor& table, const c10::optional<at::Tensor>& ids,
                                                 int64_t T, const at::Tensor& alpha, const at::Tensor& g,
                                                 const c10::optional<at::Tensor>& nreal) {
  const int64_t U = head_titles(table, ids, T), D = table.size(1);
  check_dev(alpha, "alpha");
  check_dev(g, "g");
  TORCH_CHECK(alpha.scalar_type() == at::kFloat && alpha.numel() == U * T && alpha.is_contiguous() &&
                  g.scalar_type() == at::kFloat && g.numel() == U * D && g.is_contiguous(),
              "fedrec::head_pool_bwd: alpha [U, T], g [U, D] fp32");
  const c10::DeviceGuard dg(table.device());
  auto da = at::empty({U * T}, alpha.options());
  auto db2p = at::empty({std::max<int64_t>(U, 1)}, alpha.options());
  check_rc(fr_head_pool_bwd(table.data_ptr(), opt_int_ptr(ids), alpha.data_ptr<float>(), g.data_ptr<float>(), (int)U,
                            (int)T, (int)D, da.data_ptr<float>(), db2p.data_ptr<float>(), opt_nreal(nreal, table),
                            cur_stream()),
           "head_pool_bwd");
  return {da, db2p};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> head_wgrad(const at::Tensor& table,
                                                                      const c10::optional<at::Tensor>& ids, int64_t T,
                                                                      const at::Tensor& e, const at::Tensor& da,
                                                                      const at::Tensor& w2, const at::Tensor& db2p,
                                                                      const c10::optional<at::Tensor>& nreal) {
  const int64_t U = head_titles(table, ids, T), D = table.size(1), Q = w2.numel();
  check_dev(e, "e");
  check_dev(da, "da");
  check_dev(w2, "w2");
  check_dev(db2p, "db2p");
  TORCH_CHECK(e.scalar_type() == at::kBFloat16 && e.is_contiguous() && e.numel() == U * T * Q,
              "fedrec::head_wgrad: e bf16 [U*T, Q]");
  TORCH_CHECK(da.scalar_type() == at::kFloat && da.numel() == U * T && w2.scalar_type() == at::kFloat &&
                  w2.is_contiguous() && db2p.scalar_type() == at::kFloat && db2p.numel() >= U,
              "fedrec::head_wgrad: da / w2 / db2p");
  TORCH_CHECK(fr_head_supported((int)D, (int)Q, (int)T), "fedrec::head_wgrad: unsupported shape");
  const c10::DeviceGuard g(table.device());
  auto fopt = da.options();
  auto dW1 = at::empty({Q, D}, fopt);
  auto small = at::empty({2 * Q + 1}, fopt);
  float* db1 = small.data_ptr<float>();
  float* dw2 = db1 + Q;
  float* db2 = dw2 + Q;
  const long need = fr_head_wgrad(e.data_ptr(), table.data_ptr(), opt_int_ptr(ids), da.data_ptr<float>(),
                                  db2p.data_ptr<float>(), w2.data_ptr<float>(), (int)U, (int)T, (int)D, (int)Q,
                                  dW1.data_ptr<float>(), db1, dw2, db2, nullptr, nullptr, cur_stream());
  TORCH_CHECK(need > 0, "fedrec::head_wgrad: unsupported shape");
  auto scratch = at::empty({need}, fopt);
  check_rc((int)fr_head_wgrad(e.data_ptr(), table.data_ptr(), opt_int_ptr(ids), da.data_ptr<float>(),
                              db2p.data_ptr<float>(), w2.data_ptr<float>(), (int)U, (int)T, (int)D, (int)Q,
                              dW1.data_ptr<float>(), db1, dw2, db2, scratch.data_ptr<float>(), opt_nreal(nreal, table),
                              cur_stream()),
           "head_wgrad");
  return {dW1, small.narrow(0, 0, Q), small.narrow(0, Q, Q), small.narrow(0, 2 * Q, 1)};
}

// the G path: the pool backward also rewrites e (bf16 [U*T, Q], in place) into g = da (1 - e^2)
// and writes the per-title column partials cs [2, U, Q]; the weight gradient is then a plain
// TN GEMM over g (head_wgrad_g).  Q = 384 only (head_g_supported).
bool head_g_supported(int64_t D, int64_t Q, int64_t T) { return fr_head_g_supported((int)D, (int)Q, (int)T) != 0; }

std::tuple<at::Tensor, at::Tensor, at::Tensor> head_pool_bwd_g(const at::Tensor& table,
                                                               const c10::optional<at::Tensor>& ids, int64_t T,
                                                               const at::Tensor& alpha, const at::Tensor& g,
                                                               at::Tensor e, const c10::optional<at::Tensor>& nreal) {
  const int64_t U = head_titles(table, ids, T), D = table.size(1);
  check_dev(alpha, "alpha");
  check_dev(g, "g");
  check_dev(e, "e");
  TORCH_CHECK(alpha.scalar_type() == at::kFloat && alpha.numel() == U * T && alpha.is_contiguous() &&
                  g.scalar_type() == at::kFloat && g.numel() == U * D && g.is_contiguous(),
              "fedrec::head_pool_bwd_g: alpha [U, T], g [U, D] fp32");
  TORCH_CHECK(e.scalar_type() == at::kBFloat16 && e.is_contiguous() && U > 0 && e.numel() % (U * T) == 0,
              "fedrec::head_pool_bwd_g: e bf16 [U*T, Q]");
  const int64_t Q = U > 0 ? e.numel() / (U * T) : 0;
  TORCH_CHECK(fr_head_g_supported((int)D, (int)Q, (int)T), "fedrec::head_pool_bwd_g: unsupported shape");
  const c10::DeviceGuard dg(table.device());
  auto da = at::empty({U * T}, alpha.options());
  auto db2p = at::empty({std::max<int64_t>(U, 1)}, alpha.options());
  auto cs = at::empty({2, U, Q}, alpha.options());
  check_rc(fr_head_pool_bwd_g(table.data_ptr(), opt_int_ptr(ids), alpha.data_ptr<float>(), g.data_ptr<float>(),
                              (int)U, (int)T, (int)D, (int)Q, da.data_ptr<float>(), db2p.data_ptr<float>(),
                              e.data_ptr(), cs.data_ptr<float>(), opt_nreal(nreal, table), cur_stream()),
           "head_pool_bwd_g");
  return {da, db2p, cs};
}


// the partials of a deferred small-GEMM split-K reduction, held until the launch that reduces them
static at::Tensor g_sg_pending_scratch;

void head_wgrad_g_set_kt(int64_t kt) { fr_head_wgrad_g_set_kt((int)kt); }

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> head_wgrad_g(const at::Tensor& table,
                                                                        const c10::optional<at::Tensor>& ids, int64_t T,
                                                                        const at::Tensor& G, const at::Tensor& cs,
                                                                        const at::Tensor& w2, const at::Tensor& db2p,
                                                                        const c10::optional<at::Tensor>& nreal,
                                                                        const c10::optional<std::vector<at::Tensor>>& out) {
  const int64_t U = head_titles(table, ids, T), D = table.size(1), Q = w2.numel();
  check_dev(G, "G");
  check_dev(cs, "cs");
  check_dev(w2, "w2");
  check_dev(db2p, "db2p");
  TORCH_CHECK(G.scalar_type() == at::kBFloat16 && G.is_contiguous() && G.numel() == U * T * Q,
              "fedrec::head_wgrad_g: G bf16 [U*T, Q]");
  TORCH_CHECK(cs.scalar_type() == at::kFloat && cs.is_contiguous() && cs.numel() == 2 * U * Q &&
                  w2.scalar_type() == at::kFloat && w2.is_contiguous() && db2p.scalar_type() == at::kFloat &&
                  db2p.numel() >= U,
              "fedrec::head_wgrad_g: cs [2, U, Q] / w2 / db2p");
  TORCH_CHECK(fr_head_g_supported((int)D, (int)Q, (int)T), "fedrec::head_wgrad_g: unsupported shape");
  const c10::DeviceGuard g(table.device());
  auto fopt = cs.options();
  at::Tensor dW1, small, o_db1, o_dw2, o_db2;
  float *db1, *dw2, *db2;
  if (out.has_value()) {  // the destinations given (the flat gradient buffer's slots): dW1, db1, dw2, db2
    TORCH_CHECK(out->size() == 4, "fedrec::head_wgrad_g: out = [dW1, db1, dw2, db2]");
    const int64_t sizes[4] = {Q * D, Q, Q, 1};
    for (int i = 0; i < 4; ++i) {
      const auto& t = (*out)[i];
      check_dev(t, "head_wgrad_g out");
      TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == sizes[i] &&
                      t.device() == table.device() && (i > 0 || ((uintptr_t)t.data_ptr() & 15) == 0),
                  "fedrec::head_wgrad_g: out tensors fp32 contiguous [Q, D] / [Q] / [Q] / [1]");
    }
    dW1 = (*out)[0];
    o_db1 = (*out)[1];
    o_dw2 = (*out)[2];
    o_db2 = (*out)[3];
    db1 = o_db1.data_ptr<float>();
    dw2 = o_dw2.data_ptr<float>();
    db2 = o_db2.data_ptr<float>();
  } else {
    dW1 = at::empty({Q, D}, fopt);
    small = at::empty({2 * Q + 1}, fopt);
    db1 = small.data_ptr<float>();
    dw2 = db1 + Q;
    db2 = dw2 + Q;
    o_db1 = small.narrow(0, 0, Q);
    o_dw2 = small.narrow(0, Q, Q);
    o_db2 = small.narrow(0, 2 * Q, 1);
  }
  const long need = fr_head_wgrad_g(G.data_ptr(), table.data_ptr(), opt_int_ptr(ids), cs.data_ptr<float>(),
                                    db2p.data_ptr<float>(), w2.data_ptr<float>(), (int)U, (int)T, (int)D, (int)Q,
                                    dW1.data_ptr<float>(), db1, dw2, db2, nullptr, nullptr, cur_stream(), nullptr,
                                    0, 0);
  TORCH_CHECK(need > 0, "fedrec::head_wgrad_g: unsupported shape");
  auto scratch = at::empty({need}, fopt);
  // a deferred small-GEMM split-K reduction (the text FC backward's weight gradients) rides in
  // the reduce launch; its partials stay alive until that launch is enqueued
  std::vector<unsigned char> pend((size_t)fr_small_gemm_batch_bytes());
  int pc = 0, pt = 0;
  const bool has_pend = fr_small_gemm_take_pending(pend.data(), (int)pend.size(), &pc, &pt) != 0;
  check_rc((int)fr_head_wgrad_g(G.data_ptr(), table.data_ptr(), opt_int_ptr(ids), cs.data_ptr<float>(),
                                db2p.data_ptr<float>(), w2.data_ptr<float>(), (int)U, (int)T, (int)D, (int)Q,
                                dW1.data_ptr<float>(), db1, dw2, db2, scratch.data_ptr<float>(),
                                opt_nreal(nreal, table), cur_stream(), has_pend ? pend.data() : nullptr, pc, pt),
           "head_wgrad_g");
  if (has_pend) g_sg_pending_scratch = at::Tensor();
  return {dW1, o_db1, o_dw2, o_db2};
}

// user pool backward with da out (column 0 of [n T, 8]) instead of dw2 / db2 (fr_upool_bwd_da)
// bf16_out: dpre rounded to bf16 as a fourth output (the bf16 dctx GEMM's operand); otherwise
// the fourth output is empty
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> upool_bwd_da(const at::Tensor& x, const at::Tensor& e,
                                                                        const at::Tensor& alpha, const at::Tensor& w2,
                                                                        const at::Tensor& g, bool bf16_out) {
  for (auto* t : {&x, &e, &alpha, &w2, &g}) {
    check_dev(*t, "upool_bwd_da input");
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "fedrec::upool_bwd_da: contiguous fp32");
  }
  const c10::DeviceGuard dg(x.device());
  const int64_t n = x.size(0), T = x.size(1), D = x.size(2), Q = e.size(2);
  TORCH_CHECK(e.size(0) == n && e.size(1) == T && alpha.numel() == n * T && w2.numel() == Q && g.numel() == n * D,
              "fedrec::upool_bwd_da: shapes");
  auto dx = at::empty({n, T, D}, x.options());
  auto dpre = at::empty({n, T, Q}, x.options());
  auto da8 = at::empty({n * T, 8}, x.options());
  auto dpre_b = at::empty({bf16_out ? n : 0, T, Q}, x.options().dtype(at::kBFloat16));
  check_rc(fr_upool_bwd_da(x.data_ptr<float>(), e.data_ptr<float>(), alpha.data_ptr<float>(), w2.data_ptr<float>(),
                           g.data_ptr<float>(), dx.data_ptr<float>(), dpre.data_ptr<float>(), da8.data_ptr<float>(),
                           (int)n, (int)T, (int)D, (int)Q, cur_stream(), bf16_out ? dpre_b.data_ptr() : nullptr),
           "upool_bwd_da");
  return {dx, dpre, da8, dpre_b};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> additive_pool_bwd(
    const at::Tensor& x, const at::Tensor& e, const at::Tensor& alpha, const at::Tensor& w2, const at::Tensor& g,
    bool want_dx) {
  check_dev(x, "x");
  check_dev(e, "e");
  check_dev(alpha, "alpha");
  check_dev(g, "g");
  const c10::DeviceGuard dg(x.device());
  const int64_t n = x.size(0), T = x.size(1), D = x.size(2), Q = e.size(2);
  const bool bf = x.scalar_type() == at::kBFloat16;
  auto fopt = x.options().dtype(at::kFloat);
  at::Tensor dx = want_dx ? at::empty({n, T, D}, fopt) : at::empty({0}, fopt);
  auto dpre = at::empty({n, T, Q}, e.options());
  // partial rows, one per block (no float atomics)
  const int64_t R = std::max<int64_t>(1, n * fr_additive_pool_rows((int)T, (int)D, (int)Q, bf ? 1 : 0));
  auto red = at::empty({2 * R * Q + R}, fopt);  // [dw2 rows | dpre col-sum rows | db2 rows]
  float* dw2p = red.data_ptr<float>();
  float* dsump = dw2p + R * Q;
  float* db2p = dsump + R * Q;
  const int rc = fr_additive_pool_bwd(x.data_ptr(), e.data_ptr(), alpha.data_ptr<float>(), w2.data_ptr<float>(),
                                      g.data_ptr<float>(), want_dx ? dx.data_ptr<float>() : nullptr, dpre.data_ptr(),
                                      dw2p, db2p, dsump, (int)n, (int)T, (int)D, (int)Q, (int)R, bf, cur_stream());
  TORCH_CHECK(rc <= 0, "fedrec::additive_pool_bwd: kernel launch rejected the arguments (code ", rc, ")");
  // the partial rows -> sums, one deterministic colsum launch (dw2, db2 and, from the text
  // kernel, the dpre column sums)
  auto sums = at::empty({2 * Q + 1}, fopt);
  const float* xs[3] = {dw2p, db2p, dsump};
  float* os[3] = {sums.data_ptr<float>(), sums.data_ptr<float>() + Q, sums.data_ptr<float>() + Q + 1};
  const int ints[12] = {(int)R, (int)Q, (int)Q, 0, (int)R, 1, 1, 0, (int)R, (int)Q, (int)Q, 0};
  const int ncs = rc == 0 ? 3 : 2;
  const long need = fr_colsum_f32(xs, os, ints, ncs, nullptr, cur_stream());
  auto part = at::empty({std::max<long>(need, 1)}, fopt);
  TORCH_CHECK(need >= 0 && fr_colsum_f32(xs, os, ints, ncs, part.data_ptr<float>(), cur_stream()) == 0,
              "fedrec::additive_pool_bwd: colsum failed");
  auto dw2 = sums.narrow(0, 0, Q);
  auto db2 = sums.narrow(0, Q, 1);
  auto dsum = rc == 0 ? sums.narrow(0, Q + 1, Q) : at::empty({0}, fopt);
  return {dx, dpre, dw2, db2, dsum};
}

// ctx_b (optional, bf16 [B, H, heads * head_dim], written): ctx rounded to bf16 as well
std::tuple<at::Tensor, at::Tensor> user_attention_fwd(const at::Tensor& qkv, int64_t heads, int64_t head_dim,
                                                      const c10::optional<at::Tensor>& keep,
                                                      const c10::optional<at::Tensor>& ctx_b) {
  check_dev(qkv, "qkv");
  TORCH_CHECK(qkv.scalar_type() == at::kFloat && qkv.dim() == 3, "fedrec::user_attention_fwd: fp32 [B,H,3D]");
  const c10::DeviceGuard g(qkv.device());
  const int64_t B = qkv.size(0), H = qkv.size(1);
  TORCH_CHECK(qkv.size(2) == 3 * heads * head_dim, "fedrec::user_attention_fwd: width");
  auto ctx = at::empty({B, H, heads * head_dim}, qkv.options());
  auto stats = at::empty({B, heads, H, 2}, qkv.options());
  void* cb = nullptr;
  if (ctx_b.has_value()) {
    check_dev(*ctx_b, "ctx_b");
    TORCH_CHECK(ctx_b->scalar_type() == at::kBFloat16 && ctx_b->numel() == ctx.numel(),
                "fedrec::user_attention_fwd: ctx_b bf16 like ctx");
    cb = H <= 64 ? ctx_b->data_ptr() : nullptr;  // long histories: converted below
  }
  check_rc(fr_user_attn_fwd(qkv.data_ptr<float>(), ctx.data_ptr<float>(), stats.data_ptr<float>(), (int)B, (int)H,
                            (int)heads, (int)head_dim, key_mask_ptr(keep, B, H, "user_attention_fwd"), cur_stream(), cb),
           "user_attention_fwd");
  if (ctx_b.has_value() && cb == nullptr) ctx_b->copy_(ctx.view_as(*ctx_b));
  return {ctx, stats};
}

// The Q|K|V projection fused into the attention forward (user_attn.hip user_qkv_attn_fwd_kernel):
// xd bf16 [B*H, Din] (the gathered, dropped-out history rows), W bf16 [3*heads*head_dim, Din],
// bias fp32 [3*heads*head_dim] -> (ctx [B, H, D], stats, qkv [B, H, 3D] fp32 -- the backward's
// input).  H <= 64; ctx_b (optional): ctx rounded to bf16 as well.
std::tuple<at::Tensor, at::Tensor, at::Tensor> user_qkv_attention_fwd(const at::Tensor& xd, const at::Tensor& W,
                                                                      const at::Tensor& bias, int64_t B, int64_t heads,
                                                                      int64_t head_dim,
                                                                      const c10::optional<at::Tensor>& keep,
                                                                      const c10::optional<at::Tensor>& ctx_b) {
  check_dev(xd, "xd");
  check_dev(W, "W");
  check_dev(bias, "bias");
  const c10::DeviceGuard g(xd.device());
  TORCH_CHECK(xd.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16 && bias.scalar_type() == at::kFloat &&
                  xd.dim() == 2 && W.dim() == 2 && xd.is_contiguous() && W.is_contiguous() && bias.is_contiguous(),
              "fedrec::user_qkv_attention_fwd: contiguous bf16 xd [B*H, Din], bf16 W [3D, Din], fp32 bias [3D]");
  const int64_t D = heads * head_dim, Din = xd.size(1);
  TORCH_CHECK(B > 0 && xd.size(0) % B == 0, "fedrec::user_qkv_attention_fwd: xd rows = B*H");
  const int64_t H = xd.size(0) / B;
  TORCH_CHECK(W.size(0) == 3 * D && W.size(1) == Din && bias.numel() == 3 * D && H >= 1 && H <= 64,
              "fedrec::user_qkv_attention_fwd: W [3D, Din], bias [3D], H <= 64");
  auto opt = xd.options().dtype(at::kFloat);
  auto qkv = at::empty({B, H, 3 * D}, opt);
  auto ctx = at::empty({B, H, D}, opt);
  auto stats = at::empty({B, heads, H, 2}, opt);
  void* cb = nullptr;
  if (ctx_b.has_value()) {
    check_dev(*ctx_b, "ctx_b");
    TORCH_CHECK(ctx_b->scalar_type() == at::kBFloat16 && ctx_b->numel() == ctx.numel() && ctx_b->is_contiguous(),
                "fedrec::user_qkv_attention_fwd: ctx_b bf16 like ctx");
    cb = ctx_b->data_ptr();
  }
  check_rc(fr_user_qkv_attn_fwd(xd.data_ptr(), W.data_ptr(), bias.data_ptr<float>(), (int)Din, qkv.data_ptr<float>(),
                                ctx.data_ptr<float>(), stats.data_ptr<float>(), (int)B, (int)H, (int)heads,
                                (int)head_dim, key_mask_ptr(keep, B, H, "user_qkv_attention_fwd"), cur_stream(), cb),
           "user_qkv_attention_fwd");
  return {ctx, stats, qkv};
}

// The attention backward with the additive pool's input-gradient GEMM fused in (user_attn.hip,
// FD form): dctx = dctx_direct (read, not written) + dpre W1 per head slice; dpre bf16 [B*H, Qd],
// w1t bf16 [D, Qd] (W1^T, the step's cast).  -> dqkv bf16 [B, H, 3D].  H <= 64.
at::Tensor user_attention_bwd_dctx(const at::Tensor& qkv, const at::Tensor& stats, const at::Tensor& dctx,
                                   const at::Tensor& dpre, const at::Tensor& w1t, int64_t heads, int64_t head_dim,
                                   const c10::optional<at::Tensor>& keep) {
  check_dev(qkv, "qkv");
  check_dev(stats, "stats");
  check_dev(dctx, "dctx");
  check_dev(dpre, "dpre");
  check_dev(w1t, "w1t");
  const c10::DeviceGuard g(qkv.device());
  TORCH_CHECK(qkv.scalar_type() == at::kFloat && qkv.dim() == 3 && qkv.is_contiguous(),
              "fedrec::user_attention_bwd_dctx: fp32 contiguous qkv [B,H,3D]");
  const int64_t B = qkv.size(0), H = qkv.size(1), D = heads * head_dim;
  TORCH_CHECK(qkv.size(2) == 3 * D && H <= 64, "fedrec::user_attention_bwd_dctx: qkv width 3D, H <= 64");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() == B * heads * H * 2,
              "fedrec::user_attention_bwd_dctx: stats");
  TORCH_CHECK(dctx.scalar_type() == at::kFloat && dctx.is_contiguous() && dctx.numel() == B * H * D,
              "fedrec::user_attention_bwd_dctx: fp32 contiguous dctx [B,H,D]");
  TORCH_CHECK(dpre.scalar_type() == at::kBFloat16 && w1t.scalar_type() == at::kBFloat16 && dpre.is_contiguous() &&
                  w1t.is_contiguous() && dpre.dim() == 2 && w1t.dim() == 2 && dpre.size(0) == B * H &&
                  w1t.size(0) == D && w1t.size(1) == dpre.size(1),
              "fedrec::user_attention_bwd_dctx: bf16 dpre [B*H, Qd], bf16 w1t [D, Qd]");
  auto out = at::empty({B, H, 3 * D}, qkv.options().dtype(at::kBFloat16));
  check_rc(fr_user_attn_bwd_dctx(qkv.data_ptr<float>(), stats.data_ptr<float>(), dctx.data_ptr<float>(), out.data_ptr(),
                                 dpre.data_ptr(), w1t.data_ptr(), (int)dpre.size(1), (int)B, (int)H, (int)heads,
                                 (int)head_dim, key_mask_ptr(keep, B, H, "user_attention_bwd_dctx"), cur_stream()),
           "user_attention_bwd_dctx");
  return out;
}

// bf16_out: dqkv in bf16 (the input / weight gradient GEMMs' operand)
at::Tensor user_attention_bwd(const at::Tensor& qkv, const at::Tensor& stats, const at::Tensor& dctx, int64_t heads,
                              int64_t head_dim, const c10::optional<at::Tensor>& keep, bool bf16_out) {
  check_dev(qkv, "qkv");
  check_dev(stats, "stats");
  check_dev(dctx, "dctx");
  const c10::DeviceGuard g(qkv.device());
  const int64_t B = qkv.size(0), H = qkv.size(1);
  auto d = dctx.to(at::kFloat).contiguous();
  const bool bf = bf16_out && H <= 64;  // long histories: converted below
  auto dqkv = at::empty_like(qkv, bf ? qkv.options().dtype(at::kBFloat16) : qkv.options());
  check_rc(fr_user_attn_bwd(qkv.data_ptr<float>(), stats.data_ptr<float>(), d.data_ptr<float>(), dqkv.data_ptr(),
                            (int)B, (int)H, (int)heads, (int)head_dim, key_mask_ptr(keep, B, H, "user_attention_bwd"),
                            cur_stream(), bf ? 1 : 0),
           "user_attention_bwd");
  return bf16_out && !bf ? dqkv.to(at::kBFloat16) : dqkv;
}

// The user side's tail in one launch (csrc/score_ce.hip user_pool_score_kernel): the additive
// pool of ctx [B, T, D] with scores from e [B, T, Q], the candidate scores + CE against rows
// ci of the table, their gradients into dcand_out [B C, D], and (want_bwd) the pool's backward
// for du.  -> (loss, scores, dctx, dpre, dpre_b, da8); an empty loss when the shape is outside
// the kernel's domain (the caller takes the separate kernels).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> user_pool_score(
    const at::Tensor& x, const at::Tensor& e, const at::Tensor& w2, const at::Tensor& b2,
    const c10::optional<at::Tensor>& keep, const at::Tensor& table, const at::Tensor& ci, int64_t act,
    at::Tensor dcand_out, bool want_bwd) {
  for (const at::Tensor* t : {&x, &e, &w2, &b2, &table, &ci}) check_dev(*t, "user_pool_score input");
  check_dev(dcand_out, "dcand_out");
  TORCH_CHECK(x.scalar_type() == at::kFloat && e.scalar_type() == at::kFloat && w2.scalar_type() == at::kFloat &&
                  b2.scalar_type() == at::kFloat && table.scalar_type() == at::kFloat &&
                  ci.scalar_type() == at::kInt && dcand_out.scalar_type() == at::kFloat && x.dim() == 3 &&
                  e.dim() == 3 && table.dim() == 2,
              "fedrec::user_pool_score: fp32 x [B,T,D], e [B,T,Q], table [U,D]; int32 ci");
  const c10::DeviceGuard g(x.device());
  const int64_t B = x.size(0), T = x.size(1), D = x.size(2), Q = e.size(2);
  TORCH_CHECK(e.size(0) == B && e.size(1) == T && w2.numel() == Q && table.size(1) == D && B > 0 &&
                  ci.numel() % B == 0 && dcand_out.numel() == ci.numel() * D,
              "fedrec::user_pool_score: shapes");
  const int64_t C = ci.numel() / B;
  auto fo = x.options();
  auto lossb = at::empty({B + 1}, fo);
  auto loss = lossb.narrow(0, B, 1).squeeze(0);
  auto scores = at::empty({B, C}, fo);
  const int64_t nb = want_bwd ? B : 0;
  auto dctx = at::empty({nb, T, D}, fo);
  auto dpre = at::empty({nb, T, Q}, fo);
  auto dpre_b = at::empty({nb, T, Q}, fo.dtype(at::kBFloat16));
  auto da8 = at::empty({nb * T, 8}, fo);
  const int* kp = nullptr;
  at::Tensor k32;
  if (keep.has_value() && keep->defined()) {
    k32 = keep->to(at::kInt).contiguous();
    TORCH_CHECK(k32.numel() == B * T, "fedrec::user_pool_score: keep [B, T]");
    kp = k32.data_ptr<int>();
  }
  const int rc = fr_user_pool_score(x.contiguous().data_ptr<float>(), e.contiguous().data_ptr<float>(),
                                    w2.contiguous().data_ptr<float>(), b2.data_ptr<float>(), kp, table.data_ptr<float>(),
                                    ci.data_ptr<int>(), (int)B, (int)T, (int)D, (int)Q, (int)C, (int)act,
                                    lossb.data_ptr<float>(), scores.data_ptr<float>(), dcand_out.data_ptr<float>(),
                                    loss.data_ptr<float>(), want_bwd ? dctx.data_ptr<float>() : nullptr,
                                    want_bwd ? dpre.data_ptr<float>() : nullptr,
                                    want_bwd ? dpre_b.data_ptr() : nullptr, want_bwd ? da8.data_ptr<float>() : nullptr,
                                    cur_stream());
  if (rc != 0) return {at::empty({0}, fo), scores, dctx, dpre, dpre_b, da8};
  return {loss, scores, dctx, dpre, dpre_b, da8};
}

// ci (optional): candidates as rows of a table -- cand is then [U, D], candidate (b, c) its row
// ci[b C + c]; dcand_out (optional): a [B C, D] fp32 buffer the candidate gradient is written to
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> score_ce(const at::Tensor& cand, const at::Tensor& user,
                                                                    int64_t act, const c10::optional<at::Tensor>& ci,
                                                                    const c10::optional<at::Tensor>& dcand_out) {
  check_dev(cand, "cand");
  check_dev(user, "user");
  TORCH_CHECK(cand.scalar_type() == at::kFloat && user.scalar_type() == at::kFloat && cand.is_contiguous() &&
                  user.is_contiguous(),
              "fedrec::score_ce: contiguous fp32");
  const c10::DeviceGuard g(cand.device());
  const bool gathered = ci.has_value() && ci->defined();
  const int64_t B = user.size(0), D = user.size(1);
  int64_t C;
  if (gathered) {
    check_dev(*ci, "ci");
    TORCH_CHECK(cand.dim() == 2 && cand.size(1) == D && ci->scalar_type() == at::kInt && ci->is_contiguous() &&
                    B > 0 && ci->numel() % B == 0,
                "fedrec::score_ce: table [U, D] + int32 ci [B C]");
    C = ci->numel() / B;  // ci values index the table: produced by dedup (in range by construction)
  } else {
    TORCH_CHECK(cand.dim() == 3 && cand.size(0) == B && cand.size(2) == D, "fedrec::score_ce: cand [B, C, D]");
    C = cand.size(1);
  }
  // per-impression losses, then the deterministic colsum (no float atomics: bit-reproducible loss)
  auto lossb = at::empty({std::max<int64_t>(B, 1) + 1}, cand.options());
  auto loss = lossb.narrow(0, B > 0 ? B : 0, 1).squeeze(0);  // 0-d view (view({}) would pick view(ScalarType))
  auto scores = at::empty({B, C}, cand.options());
  at::Tensor dcand;
  if (dcand_out.has_value() && dcand_out->defined()) {
    check_dev(*dcand_out, "dcand_out");
    TORCH_CHECK(dcand_out->scalar_type() == at::kFloat && dcand_out->is_contiguous() && dcand_out->numel() == B * C * D,
                "fedrec::score_ce: dcand_out fp32 [B C, D]");
    dcand = *dcand_out;
  } else {
    dcand = at::empty({B, C, D}, cand.options());
  }
  auto duser = at::empty_like(user);
  // the batch loss is summed inside the launch by its last block (impression order); the
  // wave-per-impression form leaves it to a deterministic colsum
  const int rc = fr_score_ce(cand.data_ptr<float>(), user.data_ptr<float>(), lossb.data_ptr<float>(),
                             scores.data_ptr<float>(), dcand.data_ptr<float>(), duser.data_ptr<float>(), (int)B, (int)C,
                             (int)D, (int)act, gathered ? ci->data_ptr<int>() : nullptr, loss.data_ptr<float>(),
                             cur_stream());
  if (rc == 2) {
    check_rc(fr_score_ce(cand.data_ptr<float>(), user.data_ptr<float>(), lossb.data_ptr<float>(),
                         scores.data_ptr<float>(), dcand.data_ptr<float>(), duser.data_ptr<float>(), (int)B, (int)C,
                         (int)D, (int)act, gathered ? ci->data_ptr<int>() : nullptr, nullptr, cur_stream()),
             "score_ce");
    const float* xs[1] = {lossb.data_ptr<float>()};
    float* os[1] = {loss.data_ptr<float>()};
    const int ints[4] = {(int)B, 1, 1, 0};
    const long need = fr_colsum_f32(xs, os, ints, 1, nullptr, cur_stream());
    auto part = at::empty({std::max<long>(need, 1)}, cand.options());
    TORCH_CHECK(need >= 0 && fr_colsum_f32(xs, os, ints, 1, part.data_ptr<float>(), cur_stream()) == 0,
                "fedrec::score_ce: loss sum");
  } else {
    check_rc(rc, "score_ce");
  }
  // with dcand_out the gradient lives in the caller's buffer (no output aliasing an input)
  if (dcand_out.has_value() && dcand_out->defined()) return {loss, scores, at::empty({0}, cand.options()), duser};
  return {loss, scores, dcand, duser};
}

at::Tensor segment_sum_rows(const at::Tensor& rows, const at::Tensor& perm, const at::Tensor& seg_ptr, int64_t num_out,
                            double clip, double noise_std, int64_t seed, int64_t offset,
                            const c10::optional<at::Tensor>& inv, bool zero_empty,
                            const c10::optional<at::Tensor>& dev_off) {
  check_dev(rows, "rows");
  check_dev(perm, "perm");
  check_dev(seg_ptr, "seg_ptr");
  TORCH_CHECK(rows.scalar_type() == at::kFloat && perm.scalar_type() == at::kInt && seg_ptr.scalar_type() == at::kInt,
              "fedrec::segment_sum_rows: dtypes");
  TORCH_CHECK(seg_ptr.numel() == num_out + 1, "fedrec::segment_sum_rows: seg_ptr size");
  const c10::DeviceGuard g(rows.device());
  const int64_t D = rows.size(-1);
  // empty segments (padded unique lists of the step graphs) come out as zero rows: the chunked
  // kernel writes them itself (no separate fill launch), the block-per-row form clears first
  auto out = at::empty({num_out, D}, rows.options());
  at::Tensor src = rows;
  const int64_t R = perm.numel();
  auto scratch = at::empty({(int64_t)fr_segsum_chunks((int)R) * 2 * D}, rows.options());
  const int* invp = nullptr;
  if (inv.has_value() && inv->defined()) {
    check_dev(*inv, "inv");
    TORCH_CHECK(inv->scalar_type() == at::kInt && inv->numel() == R, "fedrec::segment_sum_rows: inv int32[R]");
    invp = inv->data_ptr<int>();
  }
  if (clip > 0.0 || noise_std > 0.0) {  // LDP: clip + noise every occurrence
    const unsigned long long* dop = nullptr;
    if (dev_off.has_value() && dev_off->defined()) {  // device step counter (graph replays: fresh noise)
      check_dev(*dev_off, "dev_off");
      TORCH_CHECK(dev_off->scalar_type() == at::kLong && dev_off->numel() == 1, "fedrec::segment_sum_rows: dev_off int64[1]");
      dop = (const unsigned long long*)dev_off->data_ptr();
    }
    TORCH_CHECK(rows.numel() / D == R, "fedrec::segment_sum_rows: rows / perm sizes");
    // fused into the chunk pass when the layout allows (K16 + K17 in one launch)
    if (fr_segment_sum_rows_ldp(rows.data_ptr<float>(), perm.data_ptr<int>(), seg_ptr.data_ptr<int>(), invp,
                                out.data_ptr<float>(), (int)num_out, (int)D, (int)R, scratch.data_ptr<float>(),
                                (float)clip, (float)noise_std, (unsigned long long)seed, (unsigned long long)offset, dop,
                                cur_stream()) == 0)
      return out;
    src = at::empty_like(rows);  // the parallel clip + noise pass first, then the plain sum
    check_rc(fr_ldp_rows(rows.data_ptr<float>(), src.data_ptr<float>(), (int)(rows.numel() / D), (int)D, (float)clip,
                         (float)noise_std, (unsigned long long)seed, (unsigned long long)offset, cur_stream(), dop),
             "ldp_rows");
  }
  check_rc(fr_segment_sum_rows(src.data_ptr<float>(), perm.data_ptr<int>(), seg_ptr.data_ptr<int>(), invp,
                               out.data_ptr<float>(), (int)num_out, (int)D, (int)R, scratch.data_ptr<float>(),
                               cur_stream(), zero_empty ? 1 : 0),
           "segment_sum_rows");
  return out;
}

// Adam with the step count (and the per-step loss ring) on the device: capturable in a graph.
// step: int64 [1], already advanced for this step (the step's cast launch, multi_cast bump2)
// gsrc / goff (optional): the step's per-parameter gradient tensors and their flat offsets --
// Adam gathers the gradient from them and writes it into g (no separate copy launch)
void adam_dev(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, const at::Tensor& step,
              const at::Tensor& loss, at::Tensor ring, double lr, double b1, double b2, double eps, double grad_scale,
              const c10::optional<std::vector<c10::optional<at::Tensor>>>& gsrc,
              const c10::optional<std::vector<int64_t>>& goff, const c10::optional<at::Tensor>& skip) {
  for (auto* t : {&p, &m, &v}) check_dev(*t, "adam_dev buffer");
  const int* skp = nullptr;
  if (skip.has_value() && skip->defined()) {  // the gradient all-reduce's status word (int32 [1])
    check_dev(*skip, "skip");
    TORCH_CHECK(skip->scalar_type() == at::kInt && skip->numel() == 1 && skip->device() == p.device(),
                "fedrec::adam_dev: skip int32 [1] on p's device");
    skp = skip->data_ptr<int>();
  }
  check_dev(g, "g");
  check_dev(step, "step");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat &&
                  v.scalar_type() == at::kFloat && p.numel() == g.numel() && p.numel() == m.numel() &&
                  p.numel() == v.numel() && p.is_contiguous() && g.is_contiguous() && m.is_contiguous() &&
                  v.is_contiguous(),
              "fedrec::adam_dev: fp32 flat buffers of one size");
  TORCH_CHECK(step.scalar_type() == at::kLong && step.numel() == 1, "fedrec::adam_dev: int64 step [1]");
  const bool has_ring = ring.numel() > 0;
  if (has_ring) {
    check_dev(loss, "loss");
    check_dev(ring, "ring");
    TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.numel() == 1 && ring.scalar_type() == at::kFloat &&
                    ring.is_contiguous(),
                "fedrec::adam_dev: fp32 loss [1] and ring");
  }
  const c10::DeviceGuard dg(p.device());
  std::vector<const float*> sp;
  std::vector<long> so, sn;
  if (gsrc.has_value()) {
    TORCH_CHECK(goff.has_value() && goff->size() == gsrc->size(), "fedrec::adam_dev: gsrc / goff sizes");
    for (size_t j = 0; j < gsrc->size(); ++j) {
      const auto& t = (*gsrc)[j];
      if (t.has_value()) {
        check_dev(*t, "adam_dev gradient segment");
        TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "fedrec::adam_dev: fp32 contiguous grads");
      }
      sp.push_back(t.has_value() ? t->data_ptr<float>() : nullptr);
      so.push_back((long)(*goff)[j]);
      sn.push_back(t.has_value() ? (long)t->numel() : 0L);
    }
  }
  check_rc(fr_adam_dev(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), nullptr,
                       (long)p.numel(), (float)lr, (float)b1, (float)b2, (float)eps, (float)grad_scale,
                       (const long long*)step.data_ptr<int64_t>(), has_ring ? loss.data_ptr<float>() : nullptr,
                       has_ring ? ring.data_ptr<float>() : nullptr, (int)ring.numel(), cur_stream(), (int)sp.size(),
                       sp.data(), so.data(), sn.data(), skp),
           "adam_dev");
}

void adam_flat(at::Tensor p, const at::Tensor& g, at::Tensor m, at::Tensor v, const c10::optional<at::Tensor>& plow,
               double lr, double b1, double b2, double eps, double bc1, double bc2, double grad_scale) {
  check_dev(p, "p");
  check_dev(g, "g");
  check_dev(m, "m");
  check_dev(v, "v");
  TORCH_CHECK(p.scalar_type() == at::kFloat && p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(),
              "fedrec::adam_flat: fp32 flat buffers of one size");
  void* lp = nullptr;
  if (plow.has_value() && plow->defined()) {
    check_dev(*plow, "p_lowp");
    TORCH_CHECK(plow->scalar_type() == at::kBFloat16 && plow->numel() == p.numel(), "fedrec::adam_flat: p_lowp");
    lp = plow->data_ptr();
  }
  const c10::DeviceGuard dg(p.device());
  check_rc(fr_adam_flat(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), lp,
                        (long)p.numel(), (float)lr, (float)b1, (float)b2, (float)eps, (float)bc1, (float)bc2,
                        (float)grad_scale, cur_stream()),
           "adam_flat");
}

// the dedup's one-kernel-chain path covers up to this many ids; past it the sort path queues
// work after its unique-count read (the engine then waits on an event: dedup_sync_max())
constexpr int64_t kDedupKernelMax = 8192;
int64_t dedup_sync_max() { return kDedupKernelMax; }

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> dedup(const at::Tensor& ids, int64_t num_news) {
  check_dev(ids, "ids");
  TORCH_CHECK(ids.scalar_type() == at::kInt && ids.dim() == 1, "fedrec::dedup: int32 [R]");
  const c10::DeviceGuard g(ids.device());
  const int64_t R = ids.numel();
  auto opt = ids.options();
  if (R == 0 || R > kDedupKernelMax) {  // large batches: sort-based path (still on the device)
    auto sorted = at::sort(ids.to(at::kLong), /*stable=*/true, 0, false);
    auto sid = std::get<0>(sorted);
    auto perm = std::get<1>(sorted).to(at::kInt);
    auto uq = std::get<0>(at::_unique2(sid, true, true, true));
    (void)num_news;
    auto flags = at::ones({R}, opt);
    if (R > 1) flags.slice(0, 1).copy_(sid.slice(0, 1).ne(sid.slice(0, 0, R - 1)).to(at::kInt));
    auto rank = at::cumsum(flags, 0).to(at::kInt) - 1;
    auto inv = at::empty({R}, opt);
    inv.index_put_({perm.to(at::kLong)}, rank);
    const int64_t U = uq.numel();
    auto counts = at::bincount(rank.to(at::kLong), {}, U);
    auto seg = at::zeros({U + 1}, opt);
    seg.slice(0, 1).copy_(at::cumsum(counts, 0).to(at::kInt));
    return {uq.to(at::kInt), inv, perm, seg};
  }
  auto uniq = at::empty({R}, opt);
  auto inv = at::empty({R}, opt);
  auto perm = at::empty({R}, opt);
  auto seg = at::empty({R + 1}, opt);
  auto ucount = at::empty({1}, opt);
  // num_news bounds the ids (the engine passes its table size): <= 2^19 selects 32-bit sort keys
  check_rc(fr_dedup(ids.data_ptr<int>(), (int)R, (int)std::min<int64_t>(num_news, 1 << 30), uniq.data_ptr<int>(),
                    inv.data_ptr<int>(), perm.data_ptr<int>(), seg.data_ptr<int>(), ucount.data_ptr<int>(),
                    cur_stream()),
           "dedup");
  const int64_t U = ucount.item<int>();  // the backbone grid depends on U: one small D2H per step
  return {uniq.slice(0, 0, U), inv, perm, seg.slice(0, 0, U + 1)};
}

std::tuple<at::Tensor, at::Tensor> sample_batch(const at::Tensor& rows, const at::Tensor& pos, const at::Tensor& neg_ptr,
                                                const at::Tensor& negs, const at::Tensor& his_ptr, const at::Tensor& his,
                                                int64_t npratio, int64_t H, bool truncate, int64_t seed,
                                                int64_t offset, bool valid) {
  for (auto* t : {&rows, &pos, &negs, &his}) {
    check_dev(*t, "sample_batch input");
    TORCH_CHECK(t->scalar_type() == at::kInt, "fedrec::sample_batch: int32 ids");
  }
  check_dev(neg_ptr, "neg_ptr");
  check_dev(his_ptr, "his_ptr");
  TORCH_CHECK(neg_ptr.scalar_type() == at::kLong && his_ptr.scalar_type() == at::kLong, "fedrec::sample_batch: int64 ptr");
  TORCH_CHECK(neg_ptr.numel() == pos.numel() + 1 && his_ptr.numel() == pos.numel() + 1, "fedrec::sample_batch: CSR");
  const c10::DeviceGuard g(rows.device());
  const int64_t B = rows.numel();
  // cand and his side by side in one buffer: the dedup reads [cand | his] as one id list without
  // a concatenating copy (LocalEngine.prepare)
  auto both = at::empty({B * (npratio + 1) + B * H}, rows.options());
  auto cand = both.narrow(0, 0, B * (npratio + 1)).view({B, npratio + 1});
  auto hout = both.narrow(0, B * (npratio + 1), B * H).view({B, H});
  check_rc(fr_sample_batch(rows.data_ptr<int>(), pos.data_ptr<int>(), (const long long*)neg_ptr.data_ptr<int64_t>(),
                           negs.data_ptr<int>(), (const long long*)his_ptr.data_ptr<int64_t>(), his.data_ptr<int>(),
                           cand.data_ptr<int>(), hout.data_ptr<int>(), (int)B, (int)npratio, (int)H, truncate ? 1 : 0,
                           (unsigned long long)seed, (unsigned long long)offset, valid ? 1 : 0, cur_stream()),
           "sample_batch");
  return {cand, hout};
}

std::tuple<at::Tensor> secagg_mask(const at::Tensor& x, const at::Tensor& seeds, const at::Tensor& signs, double scale,
                                   double clipv, int64_t round) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat, "fedrec::secagg_mask: fp32");
  const c10::DeviceGuard g(x.device());
  auto sd = seeds.to(x.device(), at::kLong).contiguous();
  auto sg = signs.to(x.device(), at::kInt).contiguous();
  auto out = at::empty(x.sizes(), x.options().dtype(at::kInt));
  check_rc(fr_secagg_mask(x.data_ptr<float>(), out.data_ptr<int>(), (long)x.numel(), (float)scale, (float)clipv,
                          (const unsigned long long*)sd.data_ptr<int64_t>(), sg.data_ptr<int>(), (int)sd.numel(),
                          (unsigned long long)round, cur_stream()),
           "secagg_mask");
  return {out};
}

at::Tensor secagg_unmask(const at::Tensor& x, double inv_scale) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kInt, "fedrec::secagg_unmask: int32");
  const c10::DeviceGuard g(x.device());
  auto out = at::empty(x.sizes(), x.options().dtype(at::kFloat));
  check_rc(fr_secagg_unmask(x.data_ptr<int>(), out.data_ptr<float>(), (long)x.numel(), (float)inv_scale, cur_stream()),
           "secagg_unmask");
  return out;
}

// ---- small GEMMs on MFMA (small_gemm.hip): up to 6 independent GEMMs per launch ------------
// ints: 14 per GEMM (M, N, K, lda, ldb, ldc, a_mode, b_mode, act, accumulate, drop_ld, drop_on, gather_on, kseg);
// A / B fp32 or bf16 (the kernel takes the dtype flags from the tensors), C fp32;
// tile: 0 = the launcher's choice, 1..4 = 64x64 / 128x64 / 64x128 / 128x128 (benchmarks);
// Bseg: per GEMM 0 or 2 extra [kseg, N] row blocks of a K-segmented B (kseg > 0)
// floats: (alpha, pdrop) per GEMM; seeds: (seed, offset) per GEMM.  C tensors are written.
// elements addressable from t.data_ptr() to the end of its storage (strided operand views)
int64_t avail(const at::Tensor& t) {
  return (int64_t)(t.storage().nbytes() / t.element_size()) - t.storage_offset();
}

void small_gemm(const std::vector<at::Tensor>& A, const c10::List<c10::optional<at::Tensor>>& gidx,
                const std::vector<at::Tensor>& B, const c10::List<c10::optional<at::Tensor>>& bias,
                const std::vector<at::Tensor>& C, at::IntArrayRef ints, at::ArrayRef<double> floats,
                at::IntArrayRef seeds, const c10::optional<at::Tensor>& dev_off, const std::vector<at::Tensor>& Bseg,
                int64_t tile, const c10::List<c10::optional<at::Tensor>>& asum) {
  const size_t n = A.size();
  TORCH_CHECK(n >= 1 && n <= 6 && B.size() == n && C.size() == n && gidx.size() == n && bias.size() == n &&
                  asum.size() == n &&
                  ints.size() == 14 * n && floats.size() == 2 * n && seeds.size() == 2 * n,
              "fedrec::small_gemm: descriptor sizes");
  const c10::DeviceGuard g(A[0].device());
  std::vector<const void*> ptrs(8 * n);
  std::vector<int> iv(16 * n);
  size_t seg_used = 0;
  std::vector<float> fv(2 * n);
  std::vector<unsigned long long> sv(2 * n);
  for (size_t i = 0; i < n; ++i) {
    const int64_t* q = ints.data() + 14 * i;
    const int64_t M = q[0], N = q[1], K = q[2], lda = q[3], ldb = q[4], ldc = q[5], am = q[6], bm = q[7];
    for (const at::Tensor* t : {&A[i], &B[i], &C[i]}) {  // row-major views with any leading dimension
      TORCH_CHECK(t->is_cuda() && (t->scalar_type() == at::kFloat || (t != &C[i] && t->scalar_type() == at::kBFloat16)) &&
                      (t->dim() == 0 || t->stride(-1) == 1),
                  "fedrec::small_gemm: fp32 / bf16 device operands (fp32 C) with unit inner stride");
    }
    // bounds of the strided accesses the kernel makes (a kernel never sees a shape it was not written for)
    const auto gv = gidx.get(i);
    const bool gathered = gv.has_value() && gv->defined();
    const int64_t gather_on = q[12];
    // a gathered operand's rows are gidx values (checked in range by the producer: dedup)
    if (!(gathered && gather_on == 1))
      TORCH_CHECK(avail(A[i]) >= (am == 0 ? (M - 1) * lda + K : (K - 1) * lda + M) || M == 0 || K == 0,
                  "fedrec::small_gemm: A too small");
    const int64_t kseg = q[13];
    const int64_t b_rows = kseg > 0 ? std::min<int64_t>(K, kseg) : K;
    if (!(gathered && gather_on == 2))
      TORCH_CHECK(avail(B[i]) >= (bm == 0 ? (N - 1) * ldb + K : (b_rows - 1) * ldb + N) || N == 0 || K == 0,
                  "fedrec::small_gemm: B too small");
    TORCH_CHECK(gathered == (gather_on != 0), "fedrec::small_gemm: gidx given iff gather_on");
    TORCH_CHECK(avail(C[i]) >= (M - 1) * ldc + N || M == 0 || N == 0, "fedrec::small_gemm: C too small");
    ptrs[8 * i + 0] = A[i].data_ptr();
    ptrs[8 * i + 1] = nullptr;
    ptrs[8 * i + 5] = ptrs[8 * i + 6] = nullptr;
    if (kseg > 0) {  // the extra row blocks of a K-segmented B come from Bseg in order
      TORCH_CHECK(bm == 1 && seg_used + 2 <= Bseg.size(), "fedrec::small_gemm: K-segmented B needs b_mode 1 + 2 Bseg");
      for (int j = 0; j < 2; ++j) {
        const at::Tensor& t = Bseg[seg_used + j];
        TORCH_CHECK(t.is_cuda() && t.scalar_type() == B[i].scalar_type() && t.stride(-1) == 1 &&
                        avail(t) >= (kseg - 1) * ldb + N,
                    "fedrec::small_gemm: Bseg block");
        ptrs[8 * i + 5 + j] = t.data_ptr();
      }
      seg_used += 2;
    }
    if (gathered) {
      TORCH_CHECK(gv->is_cuda() && gv->scalar_type() == at::kInt && gv->numel() >= (gather_on == 1 ? M : K),
                  "fedrec::small_gemm: gidx int32[M] (A rows) or int32[K] (B rows)");
      ptrs[8 * i + 1] = gv->data_ptr();
    }
    ptrs[8 * i + 2] = B[i].data_ptr();
    const auto bv = bias.get(i);
    ptrs[8 * i + 3] = nullptr;
    if (bv.has_value() && bv->defined()) {
      TORCH_CHECK(bv->is_cuda() && bv->scalar_type() == at::kFloat && bv->numel() >= N, "fedrec::small_gemm: bias");
      ptrs[8 * i + 3] = bv->data_ptr();
    }
    ptrs[8 * i + 4] = C[i].data_ptr();
    ptrs[8 * i + 7] = nullptr;
    const auto av = asum.get(i);
    if (av.has_value() && av->defined()) {  // column sums of A (a_mode 1): fp32 [M], contiguous
      TORCH_CHECK(av->is_cuda() && av->scalar_type() == at::kFloat && av->is_contiguous() && av->numel() >= M &&
                      am == 1,
                  "fedrec::small_gemm: asum fp32 [M] (a_mode 1)");
      ptrs[8 * i + 7] = av->data_ptr();
    }
    for (int j = 0; j < 14; ++j) iv[16 * i + j] = (int)q[j];
    iv[16 * i + 14] = A[i].scalar_type() == at::kBFloat16;
    iv[16 * i + 15] = B[i].scalar_type() == at::kBFloat16;
    fv[2 * i] = (float)floats[2 * i];
    fv[2 * i + 1] = (float)floats[2 * i + 1];
    sv[2 * i] = (unsigned long long)seeds[2 * i];
    sv[2 * i + 1] = (unsigned long long)seeds[2 * i + 1];
  }
  const unsigned long long* dop = nullptr;
  if (dev_off.has_value() && dev_off->defined()) {  // int64 device counter added to every dropout offset
    TORCH_CHECK(dev_off->is_cuda() && dev_off->scalar_type() == at::kLong && dev_off->numel() >= 1,
                "fedrec::small_gemm: dev_off int64[1]");
    dop = (const unsigned long long*)dev_off->data_ptr<int64_t>();
  }
  // first call: validate + ask for split-K partial space; second call: launch
  long need = fr_small_gemm(ptrs.data(), iv.data(), fv.data(), sv.data(), dop, (int)n, nullptr, (int)tile, cur_stream());
  TORCH_CHECK(need >= 0, "fedrec::small_gemm: descriptor rejected (code ", need, ")");
  at::Tensor scratch;
  if (need > 0) {
    scratch = at::empty({need}, A[0].options().dtype(at::kFloat));
    const long rc = fr_small_gemm(ptrs.data(), iv.data(), fv.data(), sv.data(), dop, (int)n,
                                  scratch.data_ptr<float>(), (int)tile, cur_stream());
    TORCH_CHECK(rc == 0, "fedrec::small_gemm: launch failed (code ", rc, ")");
    if (fr_small_gemm_has_pending() && !g_sg_pending_scratch.defined()) g_sg_pending_scratch = scratch;
  }
}

// deferred split-K reductions (ops.functional.deferred_reduces): the next small-GEMM launch whose
// split descs are all weight gradients leaves its reduction to the text head's reduce launch
void small_gemm_set_defer(bool on) { fr_small_gemm_set_defer(on ? 1 : 0); }
bool small_gemm_flush_pending() {
  const bool had = fr_small_gemm_flush_pending(cur_stream()) != 0;
  g_sg_pending_scratch = at::Tensor();
  return had;
}

// column sums of fp32 matrices [M, N] (row stride ld) into out[N] (accumulate: out += sums)
void colsum_f32(const std::vector<at::Tensor>& X, const std::vector<at::Tensor>& out, at::IntArrayRef ints) {
  const size_t n = X.size();
  TORCH_CHECK(n >= 1 && n <= 6 && out.size() == n && ints.size() == 4 * n, "fedrec::colsum_f32: sizes");
  const c10::DeviceGuard g(X[0].device());
  std::vector<const float*> xs(n);
  std::vector<float*> os(n);
  std::vector<int> iv(4 * n);
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(X[i].is_cuda() && X[i].scalar_type() == at::kFloat && out[i].is_cuda() &&
                    out[i].scalar_type() == at::kFloat && (X[i].dim() == 0 || X[i].stride(-1) == 1) &&
                    (out[i].dim() == 0 || out[i].stride(-1) == 1),
                "fedrec::colsum_f32: fp32 device");
    const int64_t M = ints[4 * i], N = ints[4 * i + 1], ld = ints[4 * i + 2];
    TORCH_CHECK(avail(out[i]) >= N && (M == 0 || avail(X[i]) >= (M - 1) * ld + N), "fedrec::colsum_f32: shapes");
    xs[i] = X[i].data_ptr<float>();
    os[i] = out[i].data_ptr<float>();
    for (int j = 0; j < 4; ++j) iv[4 * i + j] = (int)ints[4 * i + j];
  }
  const long need = fr_colsum_f32(xs.data(), os.data(), iv.data(), (int)n, nullptr, cur_stream());
  TORCH_CHECK(need >= 0, "fedrec::colsum_f32: descriptor rejected");
  auto part = at::empty({std::max<long>(need, 1)}, X[0].options());
  TORCH_CHECK(fr_colsum_f32(xs.data(), os.data(), iv.data(), (int)n, part.data_ptr<float>(), cur_stream()) == 0,
              "fedrec::colsum_f32: launch failed");
}

// A cast destination given as a transposed view of a bf16 matrix (dst = T[:, a:b].t(): sizes
// [R, C], strides (1, ld >= R)) of a contiguous fp32 [R, C] source: the cast writes the
// transposed copy (multi_cast's T segments; the register-direct GEMMs' k-contiguous weights)
struct TSegs {
  std::vector<const float*> src;
  std::vector<void*> dst;
  std::vector<int> R, C, ld;
};
static bool is_tdst(const at::Tensor& src, const at::Tensor& dst) {
  return dst.dim() == 2 && src.dim() == 2 && dst.scalar_type() == at::kBFloat16 && src.scalar_type() == at::kFloat &&
         src.is_contiguous() && src.sizes() == dst.sizes() && dst.stride(0) == 1 && dst.size(0) > 1 &&
         dst.stride(1) >= dst.size(0) && src.is_cuda() && dst.is_cuda();
}
static void add_tseg(TSegs& t, const at::Tensor& src, const at::Tensor& dst) {
  TORCH_CHECK(t.src.size() < 8, "fedrec: at most 8 transposed cast segments per launch");
  t.src.push_back(src.data_ptr<float>());
  t.dst.push_back(dst.data_ptr());
  t.R.push_back((int)src.size(0));
  t.C.push_back((int)src.size(1));
  t.ld.push_back((int)dst.stride(1));
}

// fp32 tensors -> bf16 / fp32 destinations (contiguous slices allowed) in one launch per 96
// (adam.hip), any size / alignment; false = not launched (an empty segment).  bump (optional
// int64 [1] on the same device): advanced by one by the first launch
bool multi_cast(const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst,
                const c10::optional<at::Tensor>& bump, const c10::optional<at::Tensor>& bump2) {
  const size_t n = src.size();
  TORCH_CHECK(n >= 1 && dst.size() == n, "fedrec::multi_cast: sizes");
  const c10::DeviceGuard g(dst[0].device());
  long long* bp = nullptr;
  if (bump.has_value() && bump->defined()) {
    TORCH_CHECK(bump->device() == dst[0].device() && bump->scalar_type() == at::kLong && bump->numel() == 1 &&
                    bump->is_contiguous(),
                "fedrec::multi_cast: bump must be an int64 [1] tensor on the destinations' device");
    bp = (long long*)bump->data_ptr<int64_t>();
  }
  long long* bp2 = nullptr;
  if (bump2.has_value() && bump2->defined()) {
    TORCH_CHECK(bump2->device() == dst[0].device() && bump2->scalar_type() == at::kLong && bump2->numel() == 1 &&
                    bump2->is_contiguous(),
                "fedrec::multi_cast: bump2 must be an int64 [1] tensor on the destinations' device");
    bp2 = (long long*)bump2->data_ptr<int64_t>();
  }
  std::vector<const float*> sp;
  std::vector<void*> dp;
  std::vector<long> ne;
  std::vector<int> bf;
  TSegs ts;
  for (size_t i = 0; i < n; ++i) {
    if (is_tdst(src[i], dst[i])) {
      add_tseg(ts, src[i], dst[i]);
      continue;
    }
    TORCH_CHECK(src[i].is_cuda() && dst[i].is_cuda() && src[i].is_contiguous() && dst[i].is_contiguous() &&
                    src[i].scalar_type() == at::kFloat &&
                    (dst[i].scalar_type() == at::kBFloat16 || dst[i].scalar_type() == at::kFloat) &&
                    src[i].numel() == dst[i].numel(),
                "fedrec::multi_cast: contiguous fp32 sources, bf16/fp32 destinations of the same size "
                "(or transposed bf16 views)");
    sp.push_back(src[i].data_ptr<float>());
    dp.push_back(dst[i].data_ptr());
    ne.push_back((long)src[i].numel());
    bf.push_back(dst[i].scalar_type() == at::kBFloat16 ? 1 : 0);
  }
  const size_t nn = sp.size();
  for (size_t i = 0; i < nn; ++i)
    if (ne[i] <= 0) return false;
  TORCH_CHECK(nn >= 1, "fedrec::multi_cast: at least one plain segment");
  for (size_t i0 = 0; i0 < nn; i0 += 96) {  // 96 segments per launch (kernel-argument size)
    const int k = (int)std::min<size_t>(96, nn - i0);
    const bool first = i0 == 0;
    TORCH_CHECK(fr_multi_cast(sp.data() + i0, dp.data() + i0, ne.data() + i0, bf.data() + i0, k, first ? bp : nullptr,
                              cur_stream(), first ? bp2 : nullptr, nullptr, nullptr, first ? (int)ts.src.size() : 0,
                              ts.src.data(), ts.dst.data(), ts.R.data(), ts.C.data(), ts.ld.data()) == 0,
                "fedrec::multi_cast: launch rejected");
  }
  return true;
}

// A step graph's per-replay launch: the batch into the graph's static inputs (copies of 4-byte
// words; a destination longer than its source gets the fill word past it) and the step's weight
// casts + counter bumps (multi_cast), ONE launch instead of a copy launch and an in-graph cast
// launch.  false = nothing launched (an empty cast segment).
bool copy_cast(const std::vector<at::Tensor>& csrc, const std::vector<at::Tensor>& cdst, at::IntArrayRef fill,
               const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst,
               const c10::optional<at::Tensor>& bump, const c10::optional<at::Tensor>& bump2) {
  const size_t nc = csrc.size(), n = src.size();
  TORCH_CHECK(cdst.size() == nc && fill.size() == nc && dst.size() == n && nc + n >= 1 && nc + n <= 96,
              "fedrec::copy_cast: sizes");
  const at::Tensor& ref = nc ? cdst[0] : dst[0];
  const c10::DeviceGuard g(ref.device());
  auto bptr = [&](const c10::optional<at::Tensor>& b) -> long long* {
    if (!b.has_value() || !b->defined()) return nullptr;
    TORCH_CHECK(b->device() == ref.device() && b->scalar_type() == at::kLong && b->numel() == 1 && b->is_contiguous(),
                "fedrec::copy_cast: bumps must be int64 [1] tensors on the destinations' device");
    return (long long*)b->data_ptr<int64_t>();
  };
  long long* bp = bptr(bump);
  long long* bp2 = bptr(bump2);
  std::vector<const float*> sp;
  std::vector<void*> dp;
  std::vector<long> ne, ns;
  std::vector<int> bf, fv;
  for (size_t i = 0; i < nc; ++i) {
    TORCH_CHECK(csrc[i].is_cuda() && cdst[i].is_cuda() && csrc[i].is_contiguous() && cdst[i].is_contiguous() &&
                    csrc[i].element_size() == 4 && cdst[i].scalar_type() == csrc[i].scalar_type() &&
                    csrc[i].numel() <= cdst[i].numel(),
                "fedrec::copy_cast: copies are contiguous device tensors of one 4-byte dtype, source <= destination");
    if (cdst[i].numel() == 0) continue;
    sp.push_back((const float*)csrc[i].data_ptr());
    dp.push_back(cdst[i].data_ptr());
    ne.push_back((long)cdst[i].numel());
    ns.push_back((long)csrc[i].numel());
    bf.push_back(0);
    fv.push_back((int)fill[i]);
  }
  TSegs ts;
  for (size_t i = 0; i < n; ++i) {
    if (is_tdst(src[i], dst[i])) {
      add_tseg(ts, src[i], dst[i]);
      continue;
    }
    TORCH_CHECK(src[i].is_cuda() && dst[i].is_cuda() && src[i].is_contiguous() && dst[i].is_contiguous() &&
                    src[i].scalar_type() == at::kFloat &&
                    (dst[i].scalar_type() == at::kBFloat16 || dst[i].scalar_type() == at::kFloat) &&
                    src[i].numel() == dst[i].numel(),
                "fedrec::copy_cast: contiguous fp32 cast sources, bf16/fp32 destinations of the same size "
                "(or transposed bf16 views)");
    if (src[i].numel() == 0) return false;
    sp.push_back(src[i].data_ptr<float>());
    dp.push_back(dst[i].data_ptr());
    ne.push_back((long)src[i].numel());
    ns.push_back((long)src[i].numel());
    bf.push_back(dst[i].scalar_type() == at::kBFloat16 ? 1 : 0);
    fv.push_back(0);
  }
  if (sp.empty()) return false;
  TORCH_CHECK(fr_multi_cast(sp.data(), dp.data(), ne.data(), bf.data(), (int)sp.size(), bp, cur_stream(), bp2,
                            ns.data(), fv.data(), (int)ts.src.size(), ts.src.data(), ts.dst.data(), ts.R.data(),
                            ts.C.data(), ts.ld.data()) == 0,
              "fedrec::copy_cast: launch rejected (more than 8 padded copies?)");
  return true;
}

// fp32 [R, C] masters -> transposed bf16 copies (dst: [C, ld] views, ld = row stride >= R) in one
// launch per 96 (adam.hip); false = not launched (shape / alignment), the caller transposes itself
bool multi_cast_t(const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst) {
  const size_t n = src.size();
  TORCH_CHECK(n >= 1 && dst.size() == n, "fedrec::multi_cast_t: sizes");
  const c10::DeviceGuard g(dst[0].device());
  std::vector<const float*> sp(n);
  std::vector<void*> dp(n);
  std::vector<int> R(n), C(n), ld(n);
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(src[i].is_cuda() && dst[i].is_cuda() && src[i].is_contiguous() && src[i].dim() == 2 &&
                    dst[i].dim() == 2 && src[i].scalar_type() == at::kFloat && dst[i].scalar_type() == at::kBFloat16 &&
                    dst[i].size(0) == src[i].size(1) && dst[i].size(1) == src[i].size(0) && dst[i].stride(1) == 1,
                "fedrec::multi_cast_t: fp32 [R, C] sources, bf16 [C, R] row-major destinations");
    sp[i] = src[i].data_ptr<float>();
    dp[i] = dst[i].data_ptr();
    R[i] = (int)src[i].size(0);
    C[i] = (int)src[i].size(1);
    ld[i] = (int)dst[i].stride(0);
    if (R[i] % 64 || C[i] % 64 || ld[i] % 8 || ((uintptr_t)sp[i] & 15) || ((uintptr_t)dp[i] & 15)) return false;
  }
  for (size_t i0 = 0; i0 < n; i0 += 96) {
    const int k = (int)std::min<size_t>(96, n - i0);
    TORCH_CHECK(fr_multi_cast_t(sp.data() + i0, dp.data() + i0, R.data() + i0, C.data() + i0, ld.data() + i0, k,
                                cur_stream()) == 0,
                "fedrec::multi_cast_t: launch rejected");
  }
  return true;
}

// several small copies (+ fills of the tails) in one launch, in 4-byte words
void multi_copy(const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst, at::IntArrayRef fill) {
  const size_t n = src.size();
  TORCH_CHECK(n >= 1 && n <= 8 && dst.size() == n && fill.size() == n, "fedrec::multi_copy: sizes");
  const c10::DeviceGuard g(dst[0].device());
  std::vector<const int*> sp(n);
  std::vector<int*> dp(n);
  std::vector<long> ns(n), nd(n);
  std::vector<int> fv(n);
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(src[i].is_cuda() && dst[i].is_cuda() && src[i].is_contiguous() && dst[i].is_contiguous() &&
                    src[i].element_size() % 4 == 0 && dst[i].element_size() == src[i].element_size(),
                "fedrec::multi_copy: contiguous device tensors of one 4/8-byte dtype");
    sp[i] = (const int*)src[i].data_ptr();
    dp[i] = (int*)dst[i].data_ptr();
    ns[i] = (long)(src[i].numel() * src[i].element_size() / 4);
    nd[i] = (long)(dst[i].numel() * dst[i].element_size() / 4);
    TORCH_CHECK(ns[i] <= nd[i], "fedrec::multi_copy: source larger than destination");
    fv[i] = (int)fill[i];
  }
  check_rc(fr_multi_copy(sp.data(), dp.data(), ns.data(), nd.data(), fv.data(), (int)n, cur_stream()), "multi_copy");
}

// exact secure aggregation (parallel/secagg.py ExactMasker): a masked exponent histogram agrees on
// the fixed-point bound (one tiny all-reduce), then the masked payload -- no host read, no sync
at::Tensor secagg_hist(const at::Tensor& x, const at::Tensor& seeds, const at::Tensor& signs, int64_t round) {
  check_dev(x, "x");
  check_dev(seeds, "seeds");
  check_dev(signs, "signs");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && seeds.scalar_type() == at::kLong &&
                  signs.scalar_type() == at::kInt && seeds.numel() == signs.numel(),
              "fedrec::secagg_hist: dtypes");
  const c10::DeviceGuard g(x.device());
  auto scratch = at::zeros({2}, x.options().dtype(at::kInt));
  auto out = at::empty({256}, x.options().dtype(at::kInt));
  check_rc(fr_secagg_hist(x.data_ptr<float>(), (long)x.numel(), (unsigned*)scratch.data_ptr<int>(), out.data_ptr<int>(),
                          (const unsigned long long*)seeds.data_ptr<int64_t>(), signs.data_ptr<int>(),
                          (int)seeds.numel(), (unsigned long long)round, cur_stream()),
           "secagg_hist");
  return out;
}

at::Tensor secagg_mask_exact(const at::Tensor& x, const at::Tensor& seeds, const at::Tensor& signs,
                             const at::Tensor& hist, int64_t W, int64_t round) {
  check_dev(x, "x");
  check_dev(seeds, "seeds");
  check_dev(signs, "signs");
  check_dev(hist, "hist");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && hist.scalar_type() == at::kInt &&
                  hist.numel() == 256 && seeds.scalar_type() == at::kLong && signs.scalar_type() == at::kInt &&
                  seeds.numel() == signs.numel(),
              "fedrec::secagg_mask_exact: dtypes");
  const c10::DeviceGuard g(x.device());
  auto out = at::empty(x.sizes(), x.options().dtype(at::kInt));
  check_rc(fr_secagg_mask_exact(x.data_ptr<float>(), out.data_ptr<int>(), (long)x.numel(), hist.data_ptr<int>(),
                                (int)W, (const unsigned long long*)seeds.data_ptr<int64_t>(), signs.data_ptr<int>(),
                                (int)seeds.numel(), (unsigned long long)round, cur_stream()),
           "secagg_mask_exact");
  return out;
}

void secagg_unmask_exact_(const at::Tensor& q, const at::Tensor& hist, int64_t W, at::Tensor out) {
  check_dev(q, "q");
  check_dev(hist, "hist");
  check_dev(out, "out");
  TORCH_CHECK(q.scalar_type() == at::kInt && out.scalar_type() == at::kFloat && q.numel() == out.numel() &&
                  hist.scalar_type() == at::kInt && hist.numel() == 256 && out.is_contiguous(),
              "fedrec::secagg_unmask_exact_");
  const c10::DeviceGuard g(q.device());
  check_rc(fr_secagg_unmask_exact(q.data_ptr<int>(), out.data_ptr<float>(), (long)q.numel(), hist.data_ptr<int>(),
                                  (int)W, cur_stream()),
           "secagg_unmask_exact_");
}

// ---- packed title rows (frozen backbone forward; title_attn.hip) ----------------------------
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> title_plan(const at::Tensor& mask) {
  check_dev(mask, "mask");
  const c10::DeviceGuard g(mask.device());
  auto mk = mask.to(at::kInt).contiguous();
  TORCH_CHECK(mk.dim() == 2, "fedrec::title_plan: mask [n, T]");
  const int64_t n = mk.size(0), T = mk.size(1);
  TORCH_CHECK(T >= 1 && T <= 64, "fedrec::title_plan: T in [1, 64]");
  auto io = mk.options();
  auto rowmap = at::empty({n, T}, io), src = at::empty({n * T}, io);
  auto kv_start = at::empty({n}, io), kv_len = at::empty({n}, io), qstart = at::empty({n}, io);
  auto n_kv = at::zeros({1}, io);
  check_rc(fr_title_plan(mk.data_ptr<int>(), (int)n, (int)T, rowmap.data_ptr<int>(), src.data_ptr<int>(),
                         kv_start.data_ptr<int>(), kv_len.data_ptr<int>(), qstart.data_ptr<int>(), n_kv.data_ptr<int>(),
                         cur_stream()),
           "title_plan");
  return {rowmap, src, kv_start, kv_len, qstart, n_kv};
}

at::Tensor embed_ln_rows(const at::Tensor& tokens, const at::Tensor& src, const at::Tensor& word, const at::Tensor& pos,
                         const at::Tensor& w, const at::Tensor& b, double eps) {
  check_dev(word, "word");
  check_dev(pos, "pos");
  check_dev(src, "src");
  TORCH_CHECK(word.scalar_type() == at::kBFloat16 && pos.scalar_type() == at::kBFloat16, "fedrec::embed_ln_rows: bf16");
  const c10::DeviceGuard g(word.device());
  auto tok = tokens.to(at::kInt).contiguous();
  TORCH_CHECK(tok.dim() == 2 && src.scalar_type() == at::kInt && src.numel() == tok.numel(),
              "fedrec::embed_ln_rows: tokens [n, T], src [n*T] int32");
  const int64_t n = tok.size(0), T = tok.size(1), D = word.size(1);
  TORCH_CHECK(T <= pos.size(0) && D % 256 == 0, "fedrec::embed_ln_rows: T <= max positions, D % 256 == 0");
  auto wf = w.to(at::kFloat).contiguous(), bf = b.to(at::kFloat).contiguous();
  auto y = at::empty({n * T, D}, word.options());
  check_rc(fr_embed_ln_rows_bf16(tok.data_ptr<int>(), src.data_ptr<int>(), word.data_ptr(), pos.data_ptr(),
                                 wf.data_ptr<float>(), bf.data_ptr<float>(), y.data_ptr(), (int)(n * T), (int)D, (int)T,
                                 (float)eps, cur_stream()),
           "embed_ln_rows");
  return y;
}

at::Tensor linear_split(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                        const at::Tensor& full_rows, int64_t n_partial) {
  check_dev(x, "x");
  check_dev(w, "w");
  check_dev(full_rows, "full_rows");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "fedrec::linear_split: bf16 x/w");
  TORCH_CHECK(full_rows.scalar_type() == at::kInt && full_rows.numel() == 1, "fedrec::linear_split: full_rows int32[1]");
  const c10::DeviceGuard g(x.device());
  const int64_t K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && n_partial > 0 && n_partial <= N, "fedrec::linear_split: shapes");
  const int64_t M = x.numel() / K;
  const int64_t c_rows = (M + 255) / 256 * 256;
  auto out = at::empty({c_rows * N}, x.options()).narrow(0, 0, M * N).view({M, N});
  const float* bp = nullptr;
  at::Tensor bf;
  if (b.has_value() && b->defined()) {
    bf = b->to(at::kFloat).contiguous();
    TORCH_CHECK(bf.numel() == N, "fedrec::linear_split: bias size");
    bp = bf.data_ptr<float>();
  }
  if (M == 0) return out;
  check_rc(fr_gemm_nt_bf16_split(x.data_ptr(), w.data_ptr(), bp, out.data_ptr(), (int)M, (int)N, (int)K, (int)c_rows,
                                 full_rows.data_ptr<int>(), (int)n_partial, cur_stream()),
           "linear_split");
  return out;
}

at::Tensor title_attention_packed(const at::Tensor& qkv, const at::Tensor& rowmap, const at::Tensor& kv_start,
                                  const at::Tensor& kv_len, const at::Tensor& qstart, int64_t n_heads) {
  check_dev(qkv, "qkv");
  check_dev(rowmap, "rowmap");
  check_dev(kv_start, "kv_start");
  check_dev(kv_len, "kv_len");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16, "fedrec::title_attention_packed: bf16");
  TORCH_CHECK(rowmap.dim() == 2 && rowmap.scalar_type() == at::kInt, "fedrec::title_attention_packed: rowmap [n, T]");
  const c10::DeviceGuard g(qkv.device());
  const int64_t n = rowmap.size(0), T = rowmap.size(1), D = qkv.size(-1) / 3;
  check_dev(qstart, "qstart");
  TORCH_CHECK(qkv.numel() == n * T * 3 * D && kv_start.numel() == n && kv_len.numel() == n && qstart.numel() == n,
              "fedrec::title_attention_packed: shapes");
  auto out = at::empty({n * T, D}, qkv.options());
  check_rc(fr_title_attention_packed_bf16(qkv.data_ptr(), rowmap.data_ptr<int>(), kv_start.data_ptr<int>(),
                                          kv_len.data_ptr<int>(), qstart.data_ptr<int>(), out.data_ptr(), (int)n, (int)T,
                                          (int)n_heads, (int)D,
                                          cur_stream()),
           "title_attention_packed");
  return out;
}

at::Tensor layer_norm_scatter(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b, double eps,
                              const c10::optional<at::Tensor>& residual, const at::Tensor& dst,
                              const c10::optional<at::Tensor>& out) {
  check_dev(x, "x");
  check_dev(dst, "dst");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "fedrec::layer_norm_scatter: bf16");
  const c10::DeviceGuard g(x.device());
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(dst.scalar_type() == at::kInt && dst.numel() == rows && D % 256 == 0,
              "fedrec::layer_norm_scatter: dst int32[rows], D % 256 == 0");
  auto wf = w.to(at::kFloat).contiguous(), bf = b.to(at::kFloat).contiguous();
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    check_dev(*residual, "residual");
    TORCH_CHECK(residual->scalar_type() == at::kBFloat16 && residual->numel() == x.numel(),
                "fedrec::layer_norm_scatter: residual must match x (bf16)");
    rp = residual->data_ptr();
  }
  // out (optional): the destination rows in place (the hidden-state cache's chunk) -- no copy
  at::Tensor y;
  if (out.has_value() && out->defined()) {
    check_dev(*out, "out");
    TORCH_CHECK(out->scalar_type() == at::kBFloat16 && out->is_contiguous() && out->numel() == x.numel(),
                "fedrec::layer_norm_scatter: out bf16 contiguous, x's size");
    y = *out;
  } else {
    y = at::empty_like(x);
  }
  check_rc(fr_layer_norm_scatter_bf16(x.data_ptr(), wf.data_ptr<float>(), bf.data_ptr<float>(), y.data_ptr(), (int)rows,
                                      (int)D, (float)eps, rp, dst.data_ptr<int>(), cur_stream()),
           "layer_norm_scatter");
  return y;
}

// ---- training FFN1: h = GELU(z), z = x w^T + b from one GEMM pass ------------------------------
std::tuple<at::Tensor, at::Tensor> linear_gelu_dual(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b) {
  check_dev(x, "x");
  check_dev(w, "w");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "fedrec::linear_gelu_dual: bf16");
  const c10::DeviceGuard g(x.device());
  const int64_t K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "fedrec::linear_gelu_dual: K mismatch");
  const int64_t M = x.numel() / K;
  const int64_t c_rows = (M + 255) / 256 * 256;
  auto h = at::empty({c_rows * N}, x.options()).narrow(0, 0, M * N).view({M, N});
  auto z = at::empty({c_rows * N}, x.options()).narrow(0, 0, M * N).view({M, N});
  auto bf = b.to(at::kFloat).contiguous();
  TORCH_CHECK(bf.numel() == N, "fedrec::linear_gelu_dual: bias size");
  if (M == 0) return {h, z};
  const int rc = fr_gemm_nt_bf16_dual(x.data_ptr(), w.data_ptr(), bf.data_ptr<float>(), h.data_ptr(), z.data_ptr(),
                                      (int)M, (int)N, (int)K, (int)c_rows, cur_stream());
  if (rc == 3) {  // outside the fused kernel's domain: GEMM, then the GELU pass
    check_rc(fr_gemm_nt_bf16(x.data_ptr(), w.data_ptr(), bf.data_ptr<float>(), nullptr, z.data_ptr(), (int)M, (int)N,
                             (int)K, 0, (int)c_rows, cur_stream()),
             "linear_gelu_dual");
    check_rc(fr_gelu_bf16(z.data_ptr(), nullptr, h.data_ptr(), (long)(M * N), 0, cur_stream()), "linear_gelu_dual");
  } else {
    check_rc(rc, "linear_gelu_dual");
  }
  return {h, z};
}

// ---- training-path reductions (train_grad.hip) ----------------------------------------------
// dz = (dh W^T) * GELU'(z) and its column sums (FFN1 bias gradient) from one GEMM pass;
// returns (dz, colsum) -- colsum is undefined when the shape is outside the fused kernel's
// domain (the caller then sums dz itself)
std::tuple<at::Tensor, at::Tensor> linear_gelu_bwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& z) {
  check_dev(x, "x");
  check_dev(w, "w");
  check_dev(z, "z");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && z.scalar_type() == at::kBFloat16,
              "fedrec::linear_gelu_bwd: bf16");
  const c10::DeviceGuard g(x.device());
  const int64_t K = x.size(-1), N = w.size(0), M = x.numel() / K;
  TORCH_CHECK(w.size(1) == K && z.numel() == M * N, "fedrec::linear_gelu_bwd: shapes");
  const int64_t c_rows = (M + 255) / 256 * 256;
  auto out = at::empty({c_rows * N}, x.options()).narrow(0, 0, M * N).view({M, N});
  auto part = at::empty({c_rows / 256 * 2, N}, x.options().dtype(at::kFloat));
  const int rc = fr_gemm_gelu_bwd_colpart(x.data_ptr(), w.data_ptr(), z.data_ptr(), out.data_ptr(),
                                          part.data_ptr<float>(), (int)M, (int)N, (int)K, (int)c_rows, cur_stream());
  if (rc == 0) return {out, part.sum(0)};
  check_rc(fr_gemm_nt_bf16(x.data_ptr(), w.data_ptr(), nullptr, z.data_ptr(), out.data_ptr(), (int)M, (int)N, (int)K, 3,
                           (int)c_rows, cur_stream()),
           "linear_gelu_bwd");
  return {out, at::Tensor()};
}

// streaming GELU backward + its column sums: (dz, colsum)
std::tuple<at::Tensor, at::Tensor> gelu_bwd_colsum(const at::Tensor& df, const at::Tensor& z) {
  check_dev(df, "df");
  check_dev(z, "z");
  TORCH_CHECK(df.scalar_type() == at::kBFloat16 && z.scalar_type() == at::kBFloat16 && df.numel() == z.numel(),
              "fedrec::gelu_bwd_colsum: bf16, same shape");
  const c10::DeviceGuard g(df.device());
  const int64_t N = df.size(-1), M = df.numel() / N;
  auto dz = at::empty_like(df);
  auto out = at::zeros({N}, df.options().dtype(at::kFloat));
  if (M == 0) return {dz, out};
  auto partial = at::empty({(int64_t)fr_colsum_chunks() * N}, df.options().dtype(at::kFloat));
  check_rc(fr_gelu_bwd_colsum_bf16(df.data_ptr(), z.data_ptr(), dz.data_ptr(), (int)M, (int)N,
                                   partial.data_ptr<float>(), out.data_ptr<float>(), cur_stream()),
           "gelu_bwd_colsum");
  return {dz, out};
}

at::Tensor colsum(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda(), "fedrec::colsum: x must be a device tensor");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "fedrec::colsum: bf16");
  const c10::DeviceGuard g(x.device());
  // contiguous [.., N], or a 2-D column slice with unit column stride (row stride = ld)
  const bool strided = x.dim() == 2 && x.stride(1) == 1 && x.stride(0) != x.size(1);
  TORCH_CHECK(strided || x.is_contiguous(), "fedrec::colsum: contiguous rows or a 2-D column slice");
  const int64_t N = x.size(-1), M = x.numel() / N;
  const int64_t ld = strided ? x.stride(0) : N;
  TORCH_CHECK(((uintptr_t)x.data_ptr()) % 16 == 0, "fedrec::colsum: 16-byte aligned rows");
  auto out = at::empty({N}, x.options().dtype(at::kFloat));
  if (M == 0) return out.zero_();
  auto partial = at::empty({(int64_t)fr_colsum_chunks() * N}, x.options().dtype(at::kFloat));
  check_rc(fr_colsum_bf16(x.data_ptr(), (int)M, (int)N, partial.data_ptr<float>(), out.data_ptr<float>(), cur_stream(),
                          (int)ld),
           "colsum");
  return out;
}

at::Tensor embed_grad(const at::Tensor& dx, const at::Tensor& sorted, const at::Tensor& perm, int64_t num_rows) {
  check_dev(dx, "dx");
  check_dev(sorted, "sorted");
  check_dev(perm, "perm");
  TORCH_CHECK(dx.scalar_type() == at::kBFloat16 && dx.dim() == 2, "fedrec::embed_grad: dx bf16 [R, D]");
  TORCH_CHECK(sorted.scalar_type() == at::kInt && perm.scalar_type() == at::kInt && sorted.numel() == dx.size(0) &&
                  perm.numel() == dx.size(0),
              "fedrec::embed_grad: sorted/perm int32 [R]");
  const c10::DeviceGuard g(dx.device());
  auto dword = at::zeros({num_rows, dx.size(1)}, dx.options().dtype(at::kFloat));
  auto scratch = at::zeros({dx.size(0) + 1}, sorted.options());
  check_rc(fr_embed_grad_bf16(dx.data_ptr(), sorted.data_ptr<int>(), perm.data_ptr<int>(), (int)dx.size(0),
                              (int)dx.size(1), dword.data_ptr<float>(), scratch.data_ptr<int>(), cur_stream()),
           "embed_grad");
  return dword;
}

// out[m] = v[idx[m]] * Philox dropout mask (small_gemm.hip), fp32 or bf16 (bf16_out)
at::Tensor gather_dropout(const at::Tensor& v, const at::Tensor& idx, double p, int64_t seed, int64_t offset,
                          const c10::optional<at::Tensor>& dev_off, bool bf16_out) {
  check_dev(v, "v");
  check_dev(idx, "idx");
  TORCH_CHECK(v.scalar_type() == at::kFloat && v.dim() == 2 && idx.scalar_type() == at::kInt && idx.dim() == 1,
              "fedrec::gather_dropout: fp32 v [U, K], int32 idx [M]");
  TORCH_CHECK(v.size(1) % 4 == 0, "fedrec::gather_dropout: K % 4");
  const c10::DeviceGuard g(v.device());
  const unsigned long long* dp = nullptr;
  if (dev_off.has_value() && dev_off->defined()) {
    check_dev(*dev_off, "dev_off");
    TORCH_CHECK(dev_off->scalar_type() == at::kLong && dev_off->numel() >= 1, "fedrec::gather_dropout: dev_off");
    dp = (const unsigned long long*)dev_off->data_ptr<int64_t>();
  }
  auto out = at::empty({idx.size(0), v.size(1)}, v.options().dtype(bf16_out ? at::kBFloat16 : at::kFloat));
  check_rc(fr_gather_dropout(v.data_ptr<float>(), idx.data_ptr<int>(), out.data_ptr(), bf16_out ? 1 : 0,
                             (int)idx.size(0), (int)v.size(1), (float)p, (unsigned long long)seed,
                             (unsigned long long)offset, dp, cur_stream()),
           "gather_dropout");
  return out;
}

// dW[N, K] = dy[M, N]^T x[M, K] in fp32 (gemm_wgrad.hip)
at::Tensor wgrad(const at::Tensor& dy, const at::Tensor& x) {
  check_dev(dy, "dy");
  check_dev(x, "x");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "fedrec::wgrad: bf16 dy/x");
  const c10::DeviceGuard g(dy.device());
  const int64_t N = dy.size(-1), K = x.size(-1), M = dy.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(x.numel() == M * K, "fedrec::wgrad: row count mismatch");
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0, "fedrec::wgrad: N, K must be multiples of 8");
  TORCH_CHECK(M < (1ll << 31), "fedrec::wgrad: too many rows");
  auto C = at::empty({N, K}, dy.options().dtype(at::kFloat));
  if (M == 0) return C.zero_();
  const long need = fr_wgrad_bf16(dy.data_ptr(), x.data_ptr(), C.data_ptr<float>(), nullptr, (int)M, (int)N, (int)K, 0,
                                  cur_stream());
  TORCH_CHECK(need >= 0, "fedrec::wgrad: unsupported shape");
  if (need > 0) {
    auto scratch = at::empty({need}, C.options());
    TORCH_CHECK(fr_wgrad_bf16(dy.data_ptr(), x.data_ptr(), C.data_ptr<float>(), scratch.data_ptr<float>(), (int)M,
                              (int)N, (int)K, 0, cur_stream()) == 0,
                "fedrec::wgrad: launch");
  }
  return C;
}

void gemm_set_variant(int64_t v) { fr_gemm_set_variant((int)v); }
void title_attn_set_waves(int64_t w) { fr_title_attn_set_waves((int)w); }
void title_attn_bwd_set_variant(int64_t v) { fr_title_attn_bwd_set_variant((int)v); }
void score_set_variant(int64_t v) { fr_score_set_variant((int)v); }
void segsum_set_variant(int64_t v) { fr_segsum_set_variant((int)v); }
void segsum_set_ldp_block(int64_t v) { fr_segsum_set_ldp_block((int)v); }
void small_gemm_set_rd(int64_t v) { fr_small_gemm_set_rd((int)v); }
void head_score_set_rows(int64_t r) { fr_head_score_set_rows((int)r); }
void head_score_set_ilv(int64_t v) { fr_head_score_set_ilv((int)v); }
void ln_set_wide(int64_t v) { fr_ln_set_wide((int)v); }

}  // namespace

TORCH_LIBRARY(fedrec, m) {
  m.def("gemm_set_variant(int v) -> ()", &gemm_set_variant);
  m.def("title_attn_set_waves(int w) -> ()", &title_attn_set_waves);
  m.def("title_attn_bwd_set_variant(int v) -> ()", &title_attn_bwd_set_variant);
  m.def("score_set_variant(int v) -> ()", &score_set_variant);
  m.def("segsum_set_variant(int v) -> ()", &segsum_set_variant);
  m.def("segsum_set_ldp_block(int v) -> ()", &segsum_set_ldp_block);
  m.def("small_gemm_set_rd(int v) -> ()", &small_gemm_set_rd);
  m.def("user_pool_score(Tensor x, Tensor e, Tensor w2, Tensor b2, Tensor? keep, Tensor table, Tensor ci, int act, Tensor(a!) dcand_out, bool want_bwd) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("head_score_set_rows(int r) -> ()", &head_score_set_rows);
  m.def("head_score_set_ilv(int v) -> ()", &head_score_set_ilv);
  m.def("ln_set_wide(int v) -> ()", &ln_set_wide);
  m.def("linear(Tensor x, Tensor w, Tensor? b, int act, Tensor? residual) -> Tensor");
  m.def("linear_gelu_bwd(Tensor x, Tensor w, Tensor z) -> (Tensor, Tensor)");
  m.def("gelu_bwd_colsum(Tensor df, Tensor z) -> (Tensor, Tensor)");
  m.def("layer_norm(Tensor x, Tensor w, Tensor b, float eps, Tensor? residual=None) -> Tensor");
  m.def("layer_norm_bwd(Tensor x, Tensor w, Tensor dy, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("layer_norm_bwd_colsum(Tensor x, Tensor w, Tensor dy, float eps) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("layer_norm_bwd_drop(Tensor x, Tensor w, Tensor dy, float eps, float p, int seed, int offset) -> "
        "(Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("gelu(Tensor z, Tensor? dh) -> Tensor");
  m.def("title_attention_bwd(Tensor qkv, Tensor dout, Tensor mask, int n_heads) -> Tensor");
  m.def("embed_ln(Tensor tokens, Tensor word, Tensor pos, Tensor w, Tensor b, float eps) -> Tensor");
  m.def("title_attention(Tensor qkv, Tensor mask, int n_heads) -> Tensor");
  m.def("head_supported(int D, int Q, int T) -> bool", &head_supported);
  m.def("dedup_sync_max() -> int", &dedup_sync_max);
  m.def("head_g_supported(int D, int Q, int T) -> bool", &head_g_supported);
  m.def("head_wgrad_g_set_kt(int kt) -> ()", &head_wgrad_g_set_kt);
  m.def("small_gemm_set_defer(bool on) -> ()", &small_gemm_set_defer);
  m.def("small_gemm_flush_pending() -> bool", &small_gemm_flush_pending);
  m.def("head_pool_bwd_g(Tensor table, Tensor? ids, int T, Tensor alpha, Tensor g, Tensor(a!) e, Tensor? nreal=None) -> (Tensor, Tensor, Tensor)");
  m.def("head_wgrad_g(Tensor table, Tensor? ids, int T, Tensor G, Tensor cs, Tensor w2, Tensor db2p, Tensor? nreal=None, Tensor(a!)[]? out=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("ipc_create(int cap) -> (int, Tensor)", &ipc_create);
  m.def("ipc_open(int id, Tensor handles, int me, int W, Tensor? local_ptrs) -> ()", &ipc_open);
  m.def("ipc_region(int id) -> int", &ipc_region);
  m.def("ipc_status(int id) -> int", &ipc_status);
  m.def("ipc_status_word(int id) -> Tensor", &ipc_status_word);
  m.def("ipc_destroy(int id) -> ()", &ipc_destroy);
  m.def("ipc_allreduce_(int id, Tensor(a!) x, int epoch, int mode, int blocks, float timeout_s=60.) -> ()");
  m.def("ipc_allreduce_local_(int[] ids, Tensor(a!)[] xs, int epoch, int mode, int blocks, float timeout_s=60.) -> ()");
  m.def("head_score(Tensor table, Tensor? ids, int T, Tensor w1, Tensor b1, Tensor w2, Tensor b2, bool store_e, Tensor? nreal=None) -> (Tensor, Tensor)");
  m.def("head_pool(Tensor table, Tensor? ids, int T, Tensor a, Tensor? tokens, Tensor? nreal=None, bool want_bf16=False) -> (Tensor, Tensor, Tensor)");
  m.def("head_pool_bwd(Tensor table, Tensor? ids, int T, Tensor alpha, Tensor g, Tensor? nreal=None) -> (Tensor, Tensor)");
  m.def("head_wgrad(Tensor table, Tensor? ids, int T, Tensor e, Tensor da, Tensor w2, Tensor db2p, Tensor? nreal=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("additive_pool_fwd(Tensor x, Tensor e, Tensor w2, Tensor b2, Tensor? keep=None) -> (Tensor, Tensor)");
  m.def("upool_bwd_da(Tensor x, Tensor e, Tensor alpha, Tensor w2, Tensor g, bool bf16_out=False) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("additive_pool_bwd(Tensor x, Tensor e, Tensor alpha, Tensor w2, Tensor g, bool want_dx) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("user_attention_fwd(Tensor qkv, int heads, int head_dim, Tensor? keep=None, Tensor(a!)? ctx_b=None) -> (Tensor, Tensor)");
  m.def("user_attention_bwd_dctx(Tensor qkv, Tensor stats, Tensor dctx, Tensor dpre, Tensor w1t, int heads, "
        "int head_dim, Tensor? keep=None) -> Tensor");
  m.def("user_qkv_attention_fwd(Tensor xd, Tensor W, Tensor bias, int B, int heads, int head_dim, Tensor? keep=None, "
        "Tensor(a!)? ctx_b=None) -> (Tensor, Tensor, Tensor)");
  m.def("user_attention_bwd(Tensor qkv, Tensor stats, Tensor dctx, int heads, int head_dim, Tensor? keep=None, bool bf16_out=False) -> Tensor");
  m.def("score_ce(Tensor cand, Tensor user, int act, Tensor? ci=None, Tensor(a!)? dcand_out=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("segment_sum_rows(Tensor rows, Tensor perm, Tensor seg_ptr, int num_out, float clip, float noise_std, int seed, int offset, Tensor? inv=None, bool zero_empty=False, Tensor? dev_off=None) -> Tensor");
  m.def("adam_dev(Tensor(a!) p, Tensor(d!) g, Tensor(b!) m, Tensor(c!) v, Tensor step, Tensor loss, Tensor(f!) ring, float lr, float b1, float b2, float eps, float grad_scale, Tensor?[]? gsrc=None, int[]? goff=None, Tensor? skip=None) -> ()");
  m.def("adam_flat(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? p_lowp, float lr, float b1, float b2, float eps, float bc1, float bc2, float grad_scale) -> ()");
  m.def("dedup(Tensor ids, int num_news) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("sample_batch(Tensor rows, Tensor pos, Tensor neg_ptr, Tensor negs, Tensor his_ptr, Tensor his, int npratio, int H, bool truncate, int seed, int offset, bool valid=False) -> (Tensor, Tensor)");
  m.def("secagg_mask(Tensor x, Tensor seeds, Tensor signs, float scale, float clipv, int round) -> (Tensor)");
  m.def("secagg_unmask(Tensor x, float inv_scale) -> Tensor");
  m.def("title_plan(Tensor mask) -> (Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("embed_ln_rows(Tensor tokens, Tensor src, Tensor word, Tensor pos, Tensor w, Tensor b, float eps) -> Tensor");
  m.def("linear_split(Tensor x, Tensor w, Tensor? b, Tensor full_rows, int n_partial) -> Tensor");
  m.def("title_attention_packed(Tensor qkv, Tensor rowmap, Tensor kv_start, Tensor kv_len, Tensor qstart, int n_heads) -> Tensor");
  m.def("layer_norm_scatter(Tensor x, Tensor w, Tensor b, float eps, Tensor? residual, Tensor dst, Tensor(a!)? out=None) -> Tensor");
  m.def("colsum(Tensor x) -> Tensor");
  m.def("linear_gelu_dual(Tensor x, Tensor w, Tensor b) -> (Tensor, Tensor)");
  m.def("embed_grad(Tensor dx, Tensor sorted, Tensor perm, int num_rows) -> Tensor");
  m.def("small_gemm(Tensor[] A, Tensor?[] gidx, Tensor[] B, Tensor?[] bias, Tensor(a!)[] C, int[] ints, float[] floats, int[] seeds, Tensor? dev_off, Tensor[] Bseg, int tile, Tensor?[] asum) -> ()");
  m.def("multi_copy(Tensor[] src, Tensor(a!)[] dst, int[] fill) -> ()");
  m.def("multi_cast(Tensor[] src, Tensor(a!)[] dst, Tensor(b!)? bump=None, Tensor(c!)? bump2=None) -> bool");
  m.def("multi_cast_t(Tensor[] src, Tensor(a!)[] dst) -> bool");
  m.def("copy_cast(Tensor[] csrc, Tensor(a!)[] cdst, int[] fill, Tensor[] src, Tensor(b!)[] dst, Tensor(c!)? bump=None, "
        "Tensor(d!)? bump2=None) -> bool");
  m.def("colsum_f32(Tensor[] X, Tensor(a!)[] out, int[] ints) -> ()");
  m.def("secagg_hist(Tensor x, Tensor seeds, Tensor signs, int round) -> Tensor");
  m.def("secagg_mask_exact(Tensor x, Tensor seeds, Tensor signs, Tensor hist, int W, int round) -> Tensor");
  m.def("secagg_unmask_exact_(Tensor q, Tensor hist, int W, Tensor(a!) out) -> ()");
  m.def("dropout_add(Tensor h, Tensor? res, float p, int seed, int offset) -> Tensor");
  m.def("title_attention_drop(Tensor qkv, Tensor mask, int n_heads, float p, int seed, int offset) -> Tensor");
  m.def("title_attention_bwd_drop(Tensor qkv, Tensor dout, Tensor mask, int n_heads, float p, int seed, int offset) -> Tensor");
  m.def("wgrad(Tensor dy, Tensor x) -> Tensor");
  m.def("gather_dropout(Tensor v, Tensor idx, float p, int seed, int offset, Tensor? dev_off, bool bf16_out=False) -> Tensor");
}

TORCH_LIBRARY_IMPL(fedrec, CUDA, m) {
  m.impl("linear", &linear);
  m.impl("linear_gelu_bwd", &linear_gelu_bwd);
  m.impl("gelu_bwd_colsum", &gelu_bwd_colsum);
  m.impl("layer_norm", &layer_norm);
  m.impl("layer_norm_bwd", &layer_norm_bwd);
  m.impl("layer_norm_bwd_colsum", &layer_norm_bwd_colsum);
  m.impl("layer_norm_bwd_drop", &layer_norm_bwd_drop);
  m.impl("gelu", &gelu);
  m.impl("title_attention_bwd", &title_attention_bwd);
  m.impl("embed_ln", &embed_ln);
  m.impl("title_attention", &title_attention);
  m.impl("ipc_allreduce_", &ipc_allreduce_);
  m.impl("ipc_allreduce_local_", &ipc_allreduce_local_);
  m.impl("head_score", &head_score);
  m.impl("head_pool", &head_pool);
  m.impl("head_pool_bwd", &head_pool_bwd);
  m.impl("head_wgrad", &head_wgrad);
  m.impl("head_pool_bwd_g", &head_pool_bwd_g);
  m.impl("head_wgrad_g", &head_wgrad_g);
  m.impl("additive_pool_fwd", &additive_pool_fwd);
  m.impl("additive_pool_bwd", &additive_pool_bwd);
  m.impl("upool_bwd_da", &upool_bwd_da);
  m.impl("user_attention_fwd", &user_attention_fwd);
  m.impl("user_qkv_attention_fwd", &user_qkv_attention_fwd);
  m.impl("user_attention_bwd_dctx", &user_attention_bwd_dctx);
  m.impl("user_attention_bwd", &user_attention_bwd);
  m.impl("score_ce", &score_ce);
  m.impl("user_pool_score", &user_pool_score);
  m.impl("segment_sum_rows", &segment_sum_rows);
  m.impl("adam_flat", &adam_flat);
  m.impl("adam_dev", &adam_dev);
  m.impl("dedup", &dedup);
  m.impl("sample_batch", &sample_batch);
  m.impl("secagg_mask", &secagg_mask);
  m.impl("secagg_unmask", &secagg_unmask);
  m.impl("title_plan", &title_plan);
  m.impl("embed_ln_rows", &embed_ln_rows);
  m.impl("linear_split", &linear_split);
  m.impl("title_attention_packed", &title_attention_packed);
  m.impl("layer_norm_scatter", &layer_norm_scatter);
  m.impl("colsum", &colsum);
  m.impl("linear_gelu_dual", &linear_gelu_dual);
  m.impl("embed_grad", &embed_grad);
  m.impl("dropout_add", &dropout_add);
  m.impl("secagg_hist", &secagg_hist);
  m.impl("secagg_mask_exact", &secagg_mask_exact);
  m.impl("small_gemm", &small_gemm);
  m.impl("colsum_f32", &colsum_f32);
  m.impl("multi_copy", &multi_copy);
  m.impl("multi_cast", &multi_cast);
  m.impl("multi_cast_t", &multi_cast_t);
  m.impl("copy_cast", &copy_cast);
  m.impl("secagg_unmask_exact_", &secagg_unmask_exact_);
  m.impl("title_attention_drop", &title_attention_drop);
  m.impl("title_attention_bwd_drop", &title_attention_bwd_drop);
  m.impl("wgrad", &wgrad);
  m.impl("gather_dropout", &gather_dropout);
}
