// Python bindings for the edgellm HIP kernels.
// The kernels live in .hip translation units with plain C launchers (raw pointers + stream) so
// they compile without torch headers; this file validates tensors, allocates outputs through
// torch's caching allocator (graph-capture safe) and launches on torch's current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <optional>
#include <vector>

#include "b1_engine.h"
#include <tuple>

extern "C" {
int edge_norm(const void* x, const void* res, const void* w, const void* b, void* y, void* yq, float* ys,
              void* res_out, int rows, int H, float eps, int rms, int quant, const float* xpart, int S, int h16,
              hipStream_t st);
int edge_w8a8_gemv_norm(const float* part, int S, const void* res, const void* gamma, float eps, void* res_out,
                        const void* Wp, const float* sw, const void* bias, void* out, float* os, int M, int N, int K,
                        int epi, hipStream_t st);
void edge_w8a8_gemv_norm_cfg(int on);
int edge_w8a8_gemv_ln(const void* x, const void* res, const void* gamma, const void* beta, float eps, void* res_out,
                      const void* Wp, const float* sw, const void* bias, void* out, float* os, int M, int N, int K,
                      int epi, hipStream_t st);
int edge_gemv_bf16_norm(const float* part, int S, const void* res, const void* gamma, float eps, void* res_out,
                        const void* W, const void* bias, void* out, int M, int N, int K, int epi, hipStream_t st,
                        int h16);
int edge_gemv_bf16_ln(const void* x, const void* res, const void* gamma, const void* beta, float eps, void* res_out,
                      const void* W, const void* bias, void* out, int M, int N, int K, int epi, hipStream_t st,
                      int h16, void* y_out);
int edge_w8a8_gemv_norm_on();
int edge_w8a8_gemm_splitk(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias,
                          float* part, int M, int N, int K, int KT, int a_mode, int Mpad, int S, hipStream_t st);
int edge_act(const void* x, void* y, void* yq, float* ys, int rows, int F, int mode, int quant, int h16,
             hipStream_t st);
int edge_quant(const void* x, void* q, float* s, int rows, int H, hipStream_t st);
int edge_group_quant(const void* x, void* q, float* s, int M, int K, int Mpad, hipStream_t st);
int edge_embedding(const int64_t* ids, const void* table, void* out, int rows, int H, int V, int out_f32, int h16,
                   hipStream_t st);
int edge_max_prob(const void* logits, float* out, int rows, int V, int dt, hipStream_t st);
int edge_rope_kv_write(const void* qkv, const int* start_pos, const float* cs, void* q_out, void* k_cache,
                       void* v_cache, int B, int T, int Hq, int Hkv, int D, int rot, int64_t c_sb, int64_t c_sh,
                       int S, void* k2, void* v2, int64_t c2_sb, int64_t c2_sh, int S2, int split_h,
                       const int* cpos2, int h16, hipStream_t st);
int edge_decode_attn_plan(int B, int Hkv, int max_len, int D, int* ch_out, int* nsplit_out);
int edge_decode_attn(const void* q, int64_t q_sb, void* k_cache, void* v_cache, int64_t c_sb, int64_t c_sh,
                     const int* seq_lens, int B, int Hq, int Hkv, int D, float scale, int ch, int nsplit, void* out,
                     int64_t o_sb, float* part_acc, float* part_ml, const int* pos, const float* cs, int rot,
                     void* out_q, float* out_s, int Mpad, int h16, hipStream_t st);
int edge_prefill_attn(const void* q, const void* k_cache, const void* v_cache, int64_t c_sb, int64_t c_sh,
                      const int* start_pos, void* out, int B, int T, int Hq, int Hkv, int D, float scale,
                      int causal, int h16, hipStream_t st);
int edge_w8a8_gemm(const void* A, const float* sa, const void* Wp, const float* sw, const void* bias, void* out,
                   float* os, int M, int N, int K, int KT, int a_mode, int Mpad, int epi, hipStream_t st);
int edge_sample(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                float inv_temperature, float penalty, int top_k, float top_p, int do_sample, const int* rng,
                int64_t* out_tok, void* workspace, hipStream_t st);
size_t edge_sample_workspace(int B, int V);
int edge_sample_shard_mode(int do_sample, float temperature, int top_k, float top_p, int V);
int edge_sample_shard_chunks(int Vs, int V);
int edge_sample_shard(const void* logits, int is_bf16, const uint8_t* seen, int B, int Vs, int v0, int V,
                      float temperature, float inv_temperature, float penalty, int top_k, float top_p, int do_sample,
                      const int* rng, uint64_t* pc, uint32_t* pthr, hipStream_t st);
int edge_sample_merge(const uint64_t* pc, const uint32_t* pthr, int B, int C, int V, float temperature, int top_k,
                      float top_p, int do_sample, const int* rng, int64_t* out_tok, hipStream_t st);
int edge_sample_advance(const void* logits, int is_bf16, uint8_t* seen, int B, int V, float temperature,
                        float inv_temperature, float penalty, int top_k, float top_p, int do_sample, int* rng,
                        int64_t* out_tok, void* workspace, int64_t* tok, int64_t* out, int64_t out_sb, int ncols,
                        int64_t* step, int* pos, int* lens, int* ctr, hipStream_t st);
int edge_decode_advance(const int64_t* nxt, int64_t* tok, int64_t* out, int64_t out_sb, int ncols, int64_t* step,
                        int* pos, int* lens, int* rng, const int* inc, int B, hipStream_t st);
void edge_sample_rowwide_min(int v);
void edge_sample_vec(int v);
void edge_prefill_fa(int v, int stag);
void edge_prefill_fa_order(int v);
void edge_prefill_fa_sm(int prio, int thr);
int edge_sample_timestamps(int enable, unsigned long long* host_out16);
int edge_copy_head_block(void* dst, int64_t dst_sb, int64_t dst_sh, const void* src, int64_t src_sb, int64_t src_sh,
                         int B, int heads, int64_t row_bytes, int elem_bytes, hipStream_t st, int mode, int* used);
void edge_w8a8_gemv_config(int nw, int unroll);
int edge_w8a8_rows128_ok(int K, int S);
int edge_w8a8_rows256_ok(int K);
int edge_w8a8_rows256_splits(int K);
void edge_w8a8_prefill_x32(int v);
int edge_gemv_bf16(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int epi,
                   hipStream_t st, const void* add, int h16);
int edge_gemv_bf16_splitk(const void* A, const void* W, const void* bias, float* part, int M, int N, int K, int S,
                          hipStream_t st, int h16);
int edge_llmint8_prep(const void* x, int M, int K, float thr, int cmax, void* q, float* sa, int* cols, float* xo,
                      int* count, hipStream_t st);
int edge_llmint8_outlier(void* out, const float* xo, const int* cols, const int* count, const void* wt,
                         const float* scb, int M, int N, int cmax, hipStream_t st);
int edge_llmint8_gemv(const void* x, float thr, const void* Wp, const float* sw, const void* bias, const void* wt,
                      const float* scb, void* out, int N, int K, hipStream_t st, int act);
int edge_llmint8_gemv_norm(const void* x, const void* res, const void* gamma, const void* beta, float eps, int ln,
                           void* res_out, void* y_out, float thr, const void* Wp, const float* sw, const void* bias,
                           const void* wt, const float* scb, void* out, int N, int K, hipStream_t st, int glu,
                           int act);
int edge_llmint8_prep_rows(const void* x, int M, int K, float thr, void* q, float* sa, int* cols, int* count,
                           uint32_t* flags, uint32_t* take, hipStream_t st);
int edge_llmint8_outlier_rows(void* out, const void* x, const int* cols, const int* count, const void* wt,
                              const float* scb, int M, int N, int K, hipStream_t st);
void edge_w8a8_gemv_ntw(int ntw);
void edge_w8a8_gemv_ring(int on);
void edge_w8a8_prefill_apack(int v);
int edge_w8a8_apack_ok(int M, int N, int K, int KT);
int edge_w8a8_prefill_glu(const void* A, void* Ap, const float* sa, const void* Wp, const float* sw, const void* bias,
                          void* out, int M, int N, int K, int KT, hipStream_t st);
int edge_w8a8_gemm_apk(const void* A, void* Ap, const float* sa, const void* Wp, const float* sw, const void* bias,
                       void* out, int M, int N, int K, int KT, hipStream_t st);
void edge_decode_attn_config(int target_wg);
int edge_decode_attn_i8(const void* qkv, int64_t qkv_sb, void* kc, void* vc, float* ks, float* vs, int64_t c_sb,
                        int64_t c_sh, int64_t s_sb, int64_t s_sh, const int* seq_lens, int B, int Hq, int Hkv, int D,
                        float scale, int ch, int nsplit, void* out, int64_t o_sb, float* part_acc, float* part_ml,
                        const int* pos, const float* cs, int rot, void* out_q, float* out_s, int Mpad, int S,
                        hipStream_t st);
int edge_decode_attn_i8_plan(int B, int Hkv, int max_len, int D, int* ch_out, int* nsplit_out, int G);
void edge_decode_attn_i8_wave_max(int v);
int edge_kv_quant_append(const void* src, int64_t x_sb, int64_t x_sh, const int* start_pos, void* dst, int64_t c_sb,
                         int64_t c_sh, float* sc, int64_t s_sb, int64_t s_sh, int B, int Hkv, int T, int D, int S,
                         hipStream_t st);
void edge_decode_attn_occ(int occ);
int edge_kv_dequant(const void* src, int64_t c_sb, int64_t c_sh, const float* sc, int64_t s_sb, int64_t s_sh, void* dst,
                    int64_t d_sb, int64_t d_sh, int B, int Hkv, int T, int D, hipStream_t st);
int edge_gemm_bf16_ring(const void* A, const void* W, const void* bias, void* out, int M, int N, int K, int epi, int S,
                        hipStream_t st);
int edge_bf16_ring_splits(int N, int K);
int edge_bf16_ring_min_rows();
void edge_decode_attn_gsplit(int v);
void edge_decode_attn_small(int v);
void edge_decode_attn_early(int v);
void edge_decode_attn_unroll(int v);
void edge_w8a8_wreg_cfg(int v);
int edge_w8a8_r256_ok(int M, int N, int K, int epi);
int edge_w8a8_r256(const void* Ap, const float* sa, const void* Wp, const float* sw, const void* bias, void* out,
                   int M, int N, int K, int epi, hipStream_t st);
void edge_w8a8_r256_cfg(int on);
int edge_b1_lds_bytes(int D, int xqb, int sxn, int scb);
int edge_b1_decode(const B1Params* p, int G, int D, int HD, int lds, hipStream_t st);
}

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
// Every entry point runs on the device of its first tensor argument: the kernels launch on the
// current device's current stream, so a caller whose current device differs (a layer of another
// pipeline stage, parallel/split.py) still gets its kernels on the owning GPU and stream.
#define DEVICE_GUARD(t) const c10::hip::OptionalHIPGuardMasqueradingAsCUDA device_guard_((t).is_cuda() ? std::optional<c10::Device>((t).device()) : std::nullopt)

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "edgellm HIP kernel '", what, "' failed with code ", rc,
              rc > 0 ? std::string(" (") + hipGetErrorString((hipError_t)rc) + ")" : std::string(""));
}

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

int64_t rows_of(const at::Tensor& x) { return x.numel() / x.size(-1); }

// A 16-bit float activation / weight: bf16 (the default) or fp16 (the fp16 agents).  Returns 1 for
// fp16, 0 for bf16.
int need16(const at::Tensor& t, const char* name, bool contiguous = true) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, name, " has dtype ",
              t.scalar_type(), ", expected bfloat16 or float16");
  TORCH_CHECK(!contiguous || t.is_contiguous(), name, " must be contiguous");
  return t.scalar_type() == at::kHalf ? 1 : 0;
}
void need_same(const at::Tensor& t, const at::Tensor& like, const char* name) {
  TORCH_CHECK(t.scalar_type() == like.scalar_type(), name, " has dtype ", t.scalar_type(), ", expected ",
              like.scalar_type());
}

// ---------------------------------------------------------------------------------- norms
std::tuple<at::Tensor, std::optional<at::Tensor>, at::Tensor> norm(const at::Tensor& x,
                                                                    const std::optional<at::Tensor>& residual,
                                                                    const at::Tensor& w,
                                                                    const std::optional<at::Tensor>& b, double eps,
                                                                    bool rms, int64_t quant) {
  DEVICE_GUARD(x);
  const int h16 = need16(x, "x");
  TORCH_CHECK(!(h16 && quant), "int8 output from fp16 rows is not supported");
  need16(w, "weight");
  need_same(w, x, "weight");
  const int64_t H = x.size(-1), R = rows_of(x);
  TORCH_CHECK(w.numel() == H, "norm weight size mismatch");
  if (b) { need16(*b, "bias"); need_same(*b, x, "bias"); TORCH_CHECK(b->numel() == H); }
  at::Tensor res_out = x;
  if (residual) {
    need16(*residual, "residual");
    need_same(*residual, x, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes(), "residual shape mismatch");
    res_out = at::empty_like(x);
  }
  at::Tensor y, s;
  if (quant == 2) {
    // fragment-packed for the 256-row decode GEMM: a [256, H] buffer, its first R "rows" returned
    TORCH_CHECK(R <= 256 && H % 64 == 0 && x.dim() == 2, "packed int8 output: <= 256 rows, H % 64 == 0");
    y = at::empty({256, H}, x.options().dtype(at::kChar)).narrow(0, 0, R);
    s = at::empty({R}, x.options().dtype(at::kFloat));
  } else if (quant) {
    y = at::empty(x.sizes(), x.options().dtype(at::kChar));
    auto ss = x.sizes().vec();
    ss.pop_back();
    s = at::empty(ss, x.options().dtype(at::kFloat));
  } else {
    y = at::empty_like(x);
  }
  check(edge_norm(x.data_ptr(), residual ? residual->data_ptr() : nullptr, w.data_ptr(),
                  b ? b->data_ptr() : nullptr, quant ? nullptr : y.data_ptr(), quant ? y.data_ptr() : nullptr,
                  quant ? s.data_ptr<float>() : nullptr, residual ? res_out.data_ptr() : nullptr, (int)R, (int)H,
                  (float)eps, rms, quant, nullptr, 0, h16, stream()),
        "norm");
  return {y, quant ? std::optional<at::Tensor>(s) : std::nullopt, res_out};
}

// RMSNorm whose input is S fp32 split-K partial slices [S, M, H] of a decode projection (summed in
// slice order, rounded to the weight's 16-bit type): returns (y or q, scale, h) with h = rnd(sum)
// (+ residual).  fp16 weights: no int8 output.
std::tuple<at::Tensor, std::optional<at::Tensor>, at::Tensor> rms_norm_parts(const at::Tensor& parts,
                                                                              const std::optional<at::Tensor>& residual,
                                                                              const at::Tensor& w, double eps, int64_t quant) {
  DEVICE_GUARD(parts);
  need(parts, at::kFloat, "parts");
  const int h16 = need16(w, "weight");
  TORCH_CHECK(!(h16 && quant), "int8 output from fp16 rows is not supported");
  TORCH_CHECK(parts.dim() == 3, "parts must be [S, M, H]");
  const int64_t S = parts.size(0), R = parts.size(1), H = parts.size(2);
  TORCH_CHECK(w.numel() == H, "norm weight size mismatch");
  auto opts = w.options();
  at::Tensor res_out = at::empty({R, H}, opts);
  if (residual) {
    need16(*residual, "residual");
    need_same(*residual, w, "residual");
    TORCH_CHECK(residual->numel() == R * H, "residual shape mismatch");
  }
  at::Tensor y, s;
  if (quant == 2) {                                   // fragment-packed (see norm)
    TORCH_CHECK(R <= 256 && H % 64 == 0, "packed int8 output: <= 256 rows, H % 64 == 0");
    y = at::empty({256, H}, opts.dtype(at::kChar)).narrow(0, 0, R);
    s = at::empty({R}, opts.dtype(at::kFloat));
  } else if (quant) {
    y = at::empty({R, H}, opts.dtype(at::kChar));
    s = at::empty({R}, opts.dtype(at::kFloat));
  } else {
    y = at::empty({R, H}, opts);
  }
  check(edge_norm(nullptr, residual ? residual->data_ptr() : nullptr, w.data_ptr(), nullptr,
                  quant ? nullptr : y.data_ptr(), quant ? y.data_ptr() : nullptr, quant ? s.data_ptr<float>() : nullptr,
                  res_out.data_ptr(), (int)R, (int)H, (float)eps, 1, quant, parts.data_ptr<float>(), (int)S, h16,
                  stream()),
        "rms_norm_parts");
  return {y, quant ? std::optional<at::Tensor>(s) : std::nullopt, res_out};
}


// ---------------------------------------------------------------------------------- activations
std::tuple<at::Tensor, std::optional<at::Tensor>> act(const at::Tensor& x, int64_t mode, bool quant) {
  DEVICE_GUARD(x);
  const int h16 = need16(x, "x");
  TORCH_CHECK(!(h16 && quant), "int8 output from fp16 rows is not supported");
  const int64_t W = x.size(-1), R = rows_of(x);
  const int64_t F = (mode == 0 || mode == 3) ? W / 2 : W;
  TORCH_CHECK(mode != 3 || F % 16 == 0, "blocked GLU needs F % 16 == 0");
  auto os = x.sizes().vec();
  os.back() = F;
  at::Tensor y, s;
  if (quant) {
    y = at::empty(os, x.options().dtype(at::kChar));
    auto ss = os;
    ss.pop_back();
    s = at::empty(ss, x.options().dtype(at::kFloat));
  } else {
    y = at::empty(os, x.options());
  }
  check(edge_act(x.data_ptr(), quant ? nullptr : y.data_ptr(), quant ? y.data_ptr() : nullptr,
                 quant ? s.data_ptr<float>() : nullptr, (int)R, (int)F, (int)mode, quant, h16, stream()),
        "act");
  return {y, quant ? std::optional<at::Tensor>(s) : std::nullopt};
}

std::tuple<at::Tensor, at::Tensor> quant(const at::Tensor& x) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  const int64_t H = x.size(-1), R = rows_of(x);
  auto q = at::empty(x.sizes(), x.options().dtype(at::kChar));
  auto ss = x.sizes().vec();
  ss.pop_back();
  auto s = at::empty(ss, x.options().dtype(at::kFloat));
  check(edge_quant(x.data_ptr(), q.data_ptr(), s.data_ptr<float>(), (int)R, (int)H, stream()), "quant");
  return {q, s};
}

// out_f32: fp32 rows (the bf16 values, exact) — the one split-K "slice" a deferred first norm sums
at::Tensor embedding(const at::Tensor& ids, const at::Tensor& table, bool out_f32) {
  DEVICE_GUARD(ids);
  need(ids, at::kLong, "ids");
  const int h16 = need16(table, "table");
  auto os = ids.sizes().vec();
  os.push_back(table.size(1));
  auto out = at::empty(os, out_f32 ? table.options().dtype(at::kFloat) : table.options());
  check(edge_embedding(ids.data_ptr<int64_t>(), table.data_ptr(), out.data_ptr(), (int)ids.numel(),
                       (int)table.size(1), (int)table.size(0), out_f32 ? 1 : 0, h16, stream()),
        "embedding");
  return out;
}

at::Tensor max_prob(const at::Tensor& logits) {
  DEVICE_GUARD(logits);
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous());
  const int bf = logits.scalar_type() == at::kBFloat16 ? 1 : logits.scalar_type() == at::kHalf ? 2 : 0;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat, "logits must be bf16, fp16 or f32");
  const int64_t V = logits.size(-1), R = rows_of(logits);
  auto os = logits.sizes().vec();
  os.pop_back();
  auto out = at::empty(os, logits.options().dtype(at::kFloat));
  check(edge_max_prob(logits.data_ptr(), out.data_ptr<float>(), (int)R, (int)V, bf, stream()), "max_prob");
  return out;
}

// ---------------------------------------------------------------------------------- rope + kv
// 16-bit KV cache rows: bf16, or fp16 for fp16 activations (dt)
void check_cache(const at::Tensor& c, const char* name, int64_t D, at::ScalarType dt = at::kBFloat16) {
  TORCH_CHECK(c.is_cuda() && c.scalar_type() == dt, name, " must be a ", dt == at::kHalf ? "fp16" : "bf16",
              " GPU tensor (the activations' dtype)");
  TORCH_CHECK(c.dim() == 4 && c.size(3) == D && c.stride(3) == 1 && c.stride(2) == D,
              name, " must be [B, Hkv, S, D] with contiguous rows");
}

at::Tensor rope_kv_write(const at::Tensor& qkv, const at::Tensor& start_pos, const std::optional<at::Tensor>& rope,
                         at::Tensor& k_cache, at::Tensor& v_cache, int64_t Hq, int64_t Hkv, int64_t D, int64_t rot,
                         const std::optional<at::Tensor>& k2, const std::optional<at::Tensor>& v2, int64_t split,
                         const std::optional<at::Tensor>& cpos2) {
  DEVICE_GUARD(qkv);
  const int h16 = need16(qkv, "qkv");
  const auto dt = qkv.scalar_type();
  need(start_pos, at::kInt, "start_pos");
  check_cache(k_cache, "k_cache", D, dt);
  check_cache(v_cache, "v_cache", D, dt);
  TORCH_CHECK(k_cache.strides() == v_cache.strides() && k_cache.sizes() == v_cache.sizes());
  const int64_t B = k_cache.size(0);
  TORCH_CHECK(start_pos.numel() == B, "start_pos must have one entry per cache row");
  const int64_t split_h = split < 0 ? Hkv : split;
  TORCH_CHECK(qkv.size(-1) == (Hq + 2 * Hkv) * D && k_cache.size(1) == split_h, "qkv / cache head mismatch");
  if (split_h < Hkv) {
    TORCH_CHECK(k2.has_value() && v2.has_value(), "split cache needs k2/v2");
    check_cache(*k2, "k2", D, dt);
    check_cache(*v2, "v2", D, dt);
    TORCH_CHECK(k2->strides() == v2->strides() && k2->size(0) == B && k2->size(1) == Hkv - split_h);
    if (cpos2) { need(*cpos2, at::kInt, "cpos2"); TORCH_CHECK(cpos2->numel() == B); }
  }
  const int64_t ntok = rows_of(qkv);
  TORCH_CHECK(ntok % B == 0, "qkv rows must be B*T");
  const int64_t T = ntok / B;
  if (rot > 0) {
    TORCH_CHECK(rope.has_value(), "rope table required when rot > 0");
    need(*rope, at::kFloat, "rope");
    TORCH_CHECK(rope->size(1) == rot / 2);
  }
  auto q = at::empty({B, T, Hq, D}, qkv.options());
  const bool sp2 = split_h < Hkv;
  check(edge_rope_kv_write(qkv.data_ptr(), start_pos.data_ptr<int>(), rot > 0 ? rope->data_ptr<float>() : nullptr,
                           q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), (int)B, (int)T, (int)Hq, (int)Hkv,
                           (int)D, (int)rot, k_cache.stride(0), k_cache.stride(1), (int)k_cache.size(2),
                           sp2 ? k2->data_ptr() : nullptr, sp2 ? v2->data_ptr() : nullptr, sp2 ? k2->stride(0) : 0,
                           sp2 ? k2->stride(1) : 0, sp2 ? (int)k2->size(2) : 0, (int)split_h,
                           (sp2 && cpos2) ? cpos2->data_ptr<int>() : nullptr, h16, stream()),
        "rope_kv_write");
  return q;
}

// ---------------------------------------------------------------------------------- attention
at::Tensor decode_attn(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                       const at::Tensor& seq_lens, double scale, int64_t max_len_hint) {
  DEVICE_GUARD(q);
  const int h16 = need16(q, "q", false);
  TORCH_CHECK(q.dim() == 3, "q must be [B, Hq, D]");
  TORCH_CHECK(q.stride(2) == 1 && q.stride(1) == q.size(2), "q heads must be contiguous");
  const int64_t B = q.size(0), Hq = q.size(1), D = q.size(2);
  check_cache(k_cache, "k_cache", D, q.scalar_type());
  check_cache(v_cache, "v_cache", D, q.scalar_type());
  TORCH_CHECK(k_cache.strides() == v_cache.strides());
  need(seq_lens, at::kInt, "seq_lens");
  TORCH_CHECK(seq_lens.numel() == B && k_cache.size(0) == B);
  const int64_t Hkv = k_cache.size(1);
  TORCH_CHECK(max_len_hint > 0 && max_len_hint <= k_cache.size(2), "max_len_hint out of range");
  int ch = 0, nsplit = 0;
  edge_decode_attn_plan((int)B, (int)Hkv, (int)max_len_hint, (int)D, &ch, &nsplit);
  auto out = at::empty({B, Hq, D}, q.options());
  at::Tensor pacc, pml;
  if (nsplit > 1) {
    pacc = at::empty({B, Hq, nsplit, D}, q.options().dtype(at::kFloat));
    pml = at::empty({B, Hq, nsplit, 2}, q.options().dtype(at::kFloat));
  }
  check(edge_decode_attn(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(), k_cache.stride(0),
                         k_cache.stride(1), seq_lens.data_ptr<int>(), (int)B, (int)Hq, (int)Hkv, (int)D, (float)scale,
                         ch, nsplit, out.data_ptr(), out.stride(0), nsplit > 1 ? pacc.data_ptr<float>() : nullptr,
                         nsplit > 1 ? pml.data_ptr<float>() : nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0,
                         h16, stream()),
        "decode_attn");
  return out;
}

// Decode step straight from the QKV projection: rotates q, appends the new k/v at start_pos[b]
// and attends over [0, seq_lens[b]).  quant_out: returns (int8 [B, Hq*D], scales [Hq*D/64, Mpad])
// for a W8A8 consumer; else (bf16 [B, Hq, D], None).
std::tuple<at::Tensor, std::optional<at::Tensor>> decode_attn_fused(
    const at::Tensor& qkv, const at::Tensor& start_pos, const std::optional<at::Tensor>& rope, at::Tensor& k_cache,
    at::Tensor& v_cache, const at::Tensor& seq_lens, int64_t Hq, double scale, int64_t max_len_hint, int64_t rot,
    bool quant_out) {
  DEVICE_GUARD(qkv);
  const int h16 = need16(qkv, "qkv");
  TORCH_CHECK(!(h16 && quant_out), "int8 attention output from fp16 rows is not supported");
  TORCH_CHECK(qkv.dim() == 2, "qkv must be [B, (Hq + 2 Hkv) * D]");
  const int64_t B = qkv.size(0), D = k_cache.size(3), Hkv = k_cache.size(1);
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv width does not match the cache geometry");
  check_cache(k_cache, "k_cache", D, qkv.scalar_type());
  check_cache(v_cache, "v_cache", D, qkv.scalar_type());
  TORCH_CHECK(k_cache.strides() == v_cache.strides() && k_cache.size(0) == B);
  need(start_pos, at::kInt, "start_pos");
  need(seq_lens, at::kInt, "seq_lens");
  TORCH_CHECK(start_pos.numel() == B && seq_lens.numel() == B);
  TORCH_CHECK(max_len_hint > 0 && max_len_hint <= k_cache.size(2), "max_len_hint out of range");
  const float* cs = nullptr;
  if (rot > 0) {
    TORCH_CHECK(rope.has_value(), "rope table required for rot > 0");
    need(*rope, at::kFloat, "rope");
    TORCH_CHECK(rope->size(-2) * 2 == rot, "rope table width must be rot/2");
    cs = rope->data_ptr<float>();
  }
  int ch = 0, nsplit = 0;
  edge_decode_attn_plan((int)B, (int)Hkv, (int)max_len_hint, (int)D, &ch, &nsplit);
  at::Tensor pacc, pml, out, oq;
  std::optional<at::Tensor> os;
  if (nsplit > 1) {
    pacc = at::empty({B, Hq, nsplit, D}, qkv.options().dtype(at::kFloat));
    pml = at::empty({B, Hq, nsplit, 2}, qkv.options().dtype(at::kFloat));
  }
  const int64_t Mpad = (B + 15) / 16 * 16;
  if (quant_out) {
    TORCH_CHECK(D % 64 == 0, "quantised attention output needs head_dim % 64 == 0");
    oq = at::empty({B, Hq * D}, qkv.options().dtype(at::kChar));
    os = at::empty({Hq * D / 64, Mpad}, qkv.options().dtype(at::kFloat));
  } else {
    out = at::empty({B, Hq, D}, qkv.options());
  }
  check(edge_decode_attn(qkv.data_ptr(), qkv.stride(0), k_cache.data_ptr(), v_cache.data_ptr(), k_cache.stride(0),
                         k_cache.stride(1), seq_lens.data_ptr<int>(), (int)B, (int)Hq, (int)Hkv, (int)D, (float)scale,
                         ch, nsplit, quant_out ? nullptr : out.data_ptr(), quant_out ? 0 : out.stride(0),
                         nsplit > 1 ? pacc.data_ptr<float>() : nullptr, nsplit > 1 ? pml.data_ptr<float>() : nullptr,
                         start_pos.data_ptr<int>(), cs, (int)rot, quant_out ? oq.data_ptr() : nullptr,
                         quant_out ? os->data_ptr<float>() : nullptr, (int)Mpad, h16, stream()),
        "decode_attn_fused");
  if (quant_out) return {oq, os};
  return {out, std::nullopt};
}

// ---------------------------------------------------------------------------- int8 KV cache
void check_cache8(const at::Tensor& c, const at::Tensor& s, const char* name, int64_t D) {
  TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kChar, name, " must be an int8 GPU tensor");
  TORCH_CHECK(c.dim() == 4 && c.size(3) == D && c.stride(3) == 1 && c.stride(2) == D,
              name, " must be [B, Hkv, S, D] with contiguous rows");
  TORCH_CHECK(s.is_cuda() && s.scalar_type() == at::kFloat && s.dim() == 3 && s.stride(2) == 1 &&
                  s.size(0) == c.size(0) && s.size(1) == c.size(1) && s.size(2) == c.size(2),
              name, " scales must be fp32 [B, Hkv, S]");
}

std::tuple<at::Tensor, std::optional<at::Tensor>> decode_attn_i8(
    const at::Tensor& qkv, const at::Tensor& start_pos, const std::optional<at::Tensor>& rope, at::Tensor& k_cache,
    at::Tensor& v_cache, at::Tensor& k_scale, at::Tensor& v_scale, const at::Tensor& seq_lens, int64_t Hq,
    double scale, int64_t max_len_hint, int64_t rot, bool quant_out) {
  DEVICE_GUARD(qkv);
  need(qkv, at::kBFloat16, "qkv");
  TORCH_CHECK(qkv.dim() == 2, "qkv must be [B, (Hq + 2 Hkv) * D]");
  const int64_t B = qkv.size(0), D = k_cache.size(3), Hkv = k_cache.size(1);
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv width does not match the cache geometry");
  TORCH_CHECK(D == 64 || D == 128 || D == 256, "int8 KV cache needs head_dim 64 / 128 / 256");
  check_cache8(k_cache, k_scale, "k_cache", D);
  check_cache8(v_cache, v_scale, "v_cache", D);
  TORCH_CHECK(k_cache.strides() == v_cache.strides() && k_scale.strides() == v_scale.strides() && k_cache.size(0) == B);
  need(start_pos, at::kInt, "start_pos");
  need(seq_lens, at::kInt, "seq_lens");
  TORCH_CHECK(start_pos.numel() == B && seq_lens.numel() == B);
  TORCH_CHECK(max_len_hint > 0 && max_len_hint <= k_cache.size(2), "max_len_hint out of range");
  const float* cs = nullptr;
  if (rot > 0) {
    TORCH_CHECK(rope.has_value(), "rope table required for rot > 0");
    need(*rope, at::kFloat, "rope");
    TORCH_CHECK(rope->size(-2) * 2 == rot, "rope table width must be rot/2");
    cs = rope->data_ptr<float>();
  }
  int ch = 0, nsplit = 0;
  edge_decode_attn_i8_plan((int)B, (int)Hkv, (int)max_len_hint, (int)D, &ch, &nsplit, (int)(Hq / Hkv));
  at::Tensor pacc, pml, out, oq;
  std::optional<at::Tensor> os;
  if (nsplit > 1) {
    pacc = at::empty({B, Hq, nsplit, D}, qkv.options().dtype(at::kFloat));
    pml = at::empty({B, Hq, nsplit, 2}, qkv.options().dtype(at::kFloat));
  }
  const int64_t Mpad = (B + 15) / 16 * 16;
  if (quant_out) {
    oq = at::empty({B, Hq * D}, qkv.options().dtype(at::kChar));
    os = at::empty({Hq * D / 64, Mpad}, qkv.options().dtype(at::kFloat));
  } else {
    out = at::empty({B, Hq, D}, qkv.options());
  }
  check(edge_decode_attn_i8(qkv.data_ptr(), qkv.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                            k_scale.data_ptr<float>(), v_scale.data_ptr<float>(), k_cache.stride(0), k_cache.stride(1),
                            k_scale.stride(0), k_scale.stride(1), seq_lens.data_ptr<int>(), (int)B, (int)Hq, (int)Hkv,
                            (int)D, (float)scale, ch, nsplit, quant_out ? nullptr : out.data_ptr(),
                            quant_out ? 0 : out.stride(0), nsplit > 1 ? pacc.data_ptr<float>() : nullptr,
                            nsplit > 1 ? pml.data_ptr<float>() : nullptr, start_pos.data_ptr<int>(), cs, (int)rot,
                            quant_out ? oq.data_ptr() : nullptr, quant_out ? os->data_ptr<float>() : nullptr,
                            (int)Mpad, (int)k_cache.size(2), stream()),
        "decode_attn_i8");
  if (quant_out) return {oq, os};
  return {out, std::nullopt};
}

// src: bf16 [B, Hkv, >= start + T, D] rows (rotated k or v); writes rows [start_pos[b], +T) quantised
void kv_quant_append(const at::Tensor& src, const at::Tensor& start_pos, int64_t T, at::Tensor& cache,
                     at::Tensor& scales) {
  DEVICE_GUARD(src);
  const int64_t D = cache.size(3), B = cache.size(0), Hkv = cache.size(1);
  check_cache(src, "src", D);
  check_cache8(cache, scales, "cache", D);
  TORCH_CHECK(src.size(0) == B && src.size(1) == Hkv, "src geometry");
  need(start_pos, at::kInt, "start_pos");
  TORCH_CHECK(start_pos.numel() == B);
  check(edge_kv_quant_append(src.data_ptr(), src.stride(0), src.stride(1), start_pos.data_ptr<int>(), cache.data_ptr(),
                             cache.stride(0), cache.stride(1), scales.data_ptr<float>(), scales.stride(0),
                             scales.stride(1), (int)B, (int)Hkv, (int)T, (int)D, (int)cache.size(2), stream()),
        "kv_quant_append");
}

// dst bf16 [B, Hkv, >= T, D] <- the first T int8 rows of cache (+ scales) of every (b, h)
void kv_dequant(const at::Tensor& cache, const at::Tensor& scales, at::Tensor& dst, int64_t T) {
  DEVICE_GUARD(cache);
  const int64_t D = cache.size(3), B = cache.size(0), Hkv = cache.size(1);
  check_cache8(cache, scales, "cache", D);
  check_cache(dst, "dst", D);
  TORCH_CHECK(dst.size(0) == B && dst.size(1) == Hkv && dst.size(2) >= T && cache.size(2) >= T, "dst geometry");
  check(edge_kv_dequant(cache.data_ptr(), cache.stride(0), cache.stride(1), scales.data_ptr<float>(), scales.stride(0),
                        scales.stride(1), dst.data_ptr(), dst.stride(0), dst.stride(1), (int)B, (int)Hkv, (int)T, (int)D,
                        stream()),
        "kv_dequant");
}

at::Tensor prefill_attn(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                        const at::Tensor& start_pos, double scale, bool causal) {
  DEVICE_GUARD(q);
  const int h16 = need16(q, "q");
  TORCH_CHECK(q.dim() == 4, "q must be [B, T, Hq, D]");
  const int64_t B = q.size(0), T = q.size(1), Hq = q.size(2), D = q.size(3);
  check_cache(k_cache, "k_cache", D, q.scalar_type());
  check_cache(v_cache, "v_cache", D, q.scalar_type());
  TORCH_CHECK(k_cache.strides() == v_cache.strides() && k_cache.size(0) == B);
  need(start_pos, at::kInt, "start_pos");
  TORCH_CHECK(start_pos.numel() == B);
  auto out = at::empty_like(q);
  check(edge_prefill_attn(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), k_cache.stride(0), k_cache.stride(1),
                          start_pos.data_ptr<int>(), out.data_ptr(), (int)B, (int)T, (int)Hq, (int)k_cache.size(1),
                          (int)D, (float)scale, causal, h16, stream()),
        "prefill_attn");
  return out;
}

// ---------------------------------------------------------------------------------- int8 gemm
// Activation scales: per token (sa [M]) or per (token, 64-column group) (sa [KT, Mpad], M <= 256).
int64_t a_scale_mpad(const at::Tensor& sa, int64_t M, int64_t KT) {
  need(sa, at::kFloat, "a_scale");
  if (sa.dim() == 2) {
    TORCH_CHECK(sa.size(0) == KT && sa.size(1) >= (M + 15) / 16 * 16 && sa.size(1) % 16 == 0,
                "grouped a_scale must be [K/64, Mpad]");
    TORCH_CHECK(M <= 256, "grouped activation scales are a decode (M <= 256) feature");
    return sa.size(1);
  }
  TORCH_CHECK(sa.numel() == M, "a_scale must have one entry per row");
  return 0;
}

void check_w8a8_operands(const at::Tensor& wp, const at::Tensor& sw, const std::optional<at::Tensor>& bias,
                         int64_t N, int64_t K) {
  need(wp, at::kChar, "w_packed");
  need(sw, at::kFloat, "w_scale");
  TORCH_CHECK(sw.numel() == N);
  TORCH_CHECK(wp.numel() == (N + 15) / 16 * ((K + 63) / 64) * 1024, "packed weight has wrong size");
  if (bias) { need(*bias, at::kBFloat16, "bias"); TORCH_CHECK(bias->numel() == N); }
}

// Prefill gate_up of a 16-blocked SwiGLU layer with the SwiGLU in the GEMM epilogue: bf16 h [M, N / 2],
// or None when the x32 kernel does not take the shape (the caller runs w8a8_gemm + act instead).
std::optional<at::Tensor> w8a8_prefill_glu(const at::Tensor& a, const at::Tensor& sa, const at::Tensor& wp,
                                           const at::Tensor& sw, const std::optional<at::Tensor>& bias, int64_t N,
                                           int64_t K) {
  DEVICE_GUARD(a);
  need(a, at::kChar, "a");
  TORCH_CHECK(a.size(-1) == K && a.is_contiguous(), "activation: contiguous [.., K]");
  check_w8a8_operands(wp, sw, bias, N, K);
  need(sa, at::kFloat, "a_scale");
  const int64_t M = rows_of(a), KT = (K + 63) / 64;
  TORCH_CHECK(sa.numel() == M, "per-token activation scales");
  if (M <= 64 || N % 256 != 0 || K % 64 != 0) return std::nullopt;
  auto os = a.sizes().vec();
  os.back() = N / 2;
  auto out = at::empty(os, a.options().dtype(at::kBFloat16));
  const bool apk = edge_w8a8_apack_ok((int)M, (int)N, (int)K, (int)KT);
  auto ap = apk ? at::empty({(M + 15) / 16 * 16 * K}, a.options()) : at::Tensor();
  const int rc = edge_w8a8_prefill_glu(a.data_ptr(), apk ? ap.data_ptr() : nullptr, sa.data_ptr<float>(), wp.data_ptr(),
                                       sw.data_ptr<float>(), bias ? bias->data_ptr() : nullptr, out.data_ptr(), (int)M,
                                       (int)N, (int)K, (int)KT, stream());
  if (rc == -2) return std::nullopt;
  check(rc, "w8a8_prefill_glu");
  return out;
}

// addend (optional, bf16 [.., N]): out = bf16(bf16(y) + addend) — the other branch of a parallel-
// residual block, added in the GEMV epilogue at <= 64 rows (a separate add above)
at::Tensor w8a8_gemm(const at::Tensor& a, const at::Tensor& sa, const at::Tensor& wp, const at::Tensor& sw,
                     const std::optional<at::Tensor>& bias, int64_t N, int64_t K,
                     const std::optional<at::Tensor>& addend) {
  DEVICE_GUARD(a);
  need(a, at::kChar, "a");
  TORCH_CHECK(a.size(-1) == K, "activation K mismatch");
  check_w8a8_operands(wp, sw, bias, N, K);
  const int64_t M = rows_of(a), KT = (K + 63) / 64;
  const int64_t mpad = a_scale_mpad(sa, M, KT);
  auto os = a.sizes().vec();
  os.back() = N;
  auto out = at::empty(os, a.options().dtype(at::kBFloat16));
  if (addend) {
    need(*addend, at::kBFloat16, "addend");
    TORCH_CHECK(addend->numel() == M * N, "addend must hold M * N elements");
    if (M <= 64) {
      check(edge_w8a8_gemm(a.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                           bias ? bias->data_ptr() : nullptr, out.data_ptr(), (float*)addend->data_ptr(), (int)M,
                           (int)N, (int)K, (int)KT, mpad > 0 ? 1 : 0, (int)mpad, 0, stream()),
            "w8a8_gemm");
      return out;
    }
  }
  if (mpad == 0 && a.is_contiguous() && edge_w8a8_apack_ok((int)M, (int)N, (int)K, (int)KT)) {
    // prefill: A fragment-packed into a stream-ordered scratch, then the ring GEMM on contiguous pieces
    auto ap = at::empty({(M + 15) / 16 * 16 * K}, a.options());
    check(edge_w8a8_gemm_apk(a.data_ptr(), ap.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                             bias ? bias->data_ptr() : nullptr, out.data_ptr(), (int)M, (int)N, (int)K, (int)KT,
                             stream()),
          "w8a8_gemm_apk");
    return out;
  }
  check(edge_w8a8_gemm(a.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                       bias ? bias->data_ptr() : nullptr, out.data_ptr(), nullptr, (int)M, (int)N, (int)K, (int)KT,
                       mpad > 0 ? 1 : 0, (int)mpad, 0, stream()),
        "w8a8_gemm");
  if (addend) out.add_(addend->view(out.sizes()));
  return out;
}

// Split-K W8A8 GEMV (decode, M <= 64, <= 128 where rows128_ok(K, S), <= 256 where rows256_ok(K)): fp32 partial slices
// [S, M, N] (w-scale and bias applied; bias in slice 0) for a consumer that sums them (rms_norm_parts).  S = 0 picks the split count.
// 129-256 decode rows on a fragment-packed activation (norm(..., quant=2)): ap is the [M, K] view of
// a [256, K] packed buffer; sa per-token [M].  Returns bf16 [M, N], or an empty tensor when the packed
// kernel does not take the shape.
at::Tensor w8a8_r256(const at::Tensor& ap, const at::Tensor& sa, const at::Tensor& wp, const at::Tensor& sw,
                     const std::optional<at::Tensor>& bias, int64_t N, int64_t K) {
  DEVICE_GUARD(ap);
  need(ap, at::kChar, "a");
  need(sa, at::kFloat, "a_scale");
  const int64_t M = ap.size(0);
  TORCH_CHECK(ap.dim() == 2 && ap.size(1) == K && ap.stride(0) == K, "a must be the [M, K] view of a packed buffer");
  check_w8a8_operands(wp, sw, bias, N, K);
  if (!edge_w8a8_r256_ok((int)M, (int)N, (int)K, 0)) return at::Tensor();
  at::Tensor out = at::empty({M, N}, sw.options().dtype(at::kBFloat16));
  check(edge_w8a8_r256(ap.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                       bias ? bias->data_ptr() : nullptr, out.data_ptr(), (int)M, (int)N, (int)K, 0, stream()),
        "w8a8_r256");
  return out;
}

at::Tensor w8a8_gemm_splitk(const at::Tensor& a, const at::Tensor& sa, const at::Tensor& wp, const at::Tensor& sw,
                            const std::optional<at::Tensor>& bias, int64_t N, int64_t K, int64_t S) {
  DEVICE_GUARD(a);
  need(a, at::kChar, "a");
  TORCH_CHECK(a.size(-1) == K && K % 64 == 0, "split-K GEMV needs K % 64 == 0");
  check_w8a8_operands(wp, sw, bias, N, K);
  const int64_t M = rows_of(a), KT = K / 64;
  TORCH_CHECK(M <= 256, "split-K GEMV is a decode (M <= 256) kernel");
  const int64_t mpad = a_scale_mpad(sa, M, KT);
  if (M > 128) S = edge_w8a8_rows256_splits((int)K);     // 129-256 rows: fixed per K (gemm_i8.hip rows256)
  TORCH_CHECK(M <= 128 || S > 1, "no 129-256-row split-K kernel for this K");
  if (S <= 0 && M > 64) S = 4;                           // 65-128 rows: 4 slices (gemm_i8.hip rows128)
  if (S <= 0) {
    const int64_t ntw = M <= 16 ? 2 : 4;                 // tiles per workgroup (gemm_i8.hip launcher)
    const int64_t groups = ((N + 15) / 16 + ntw - 1) / ntw;
    S = std::max<int64_t>(1, std::min<int64_t>(8, (256 + groups / 2) / groups));
  }
  S = std::min<int64_t>(S, KT);
  auto part = at::empty({S, M, N}, a.options().dtype(at::kFloat));
  check(edge_w8a8_gemm_splitk(a.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                              bias ? bias->data_ptr() : nullptr, part.data_ptr<float>(), (int)M, (int)N, (int)K,
                              (int)KT, mpad > 0 ? 1 : 0, (int)mpad, (int)S, stream()),
        "w8a8_gemm_splitk");
  return part;
}

// bf16 decode GEMV (M <= 64, K % 64 == 0, N % 16 == 0): x [.., K] . W[N, K]^T (+ bias) -> bf16, with
// W fragment-packed (ops.pack_bf16_weight).  epi: 0 plain, 1 SwiGLU over [gate | up] (result
// [.., N/2]), 2 gelu-tanh, 3 gelu (erf).
at::Tensor gemv_bf16(const at::Tensor& x, const at::Tensor& wp, const std::optional<at::Tensor>& bias, int64_t N,
                     int64_t epi, const std::optional<at::Tensor>& addend) {
  DEVICE_GUARD(x);
  const int h16 = need16(x, "x");
  need_same(wp, x, "weight (packed)");
  const int64_t K = x.size(-1), M = rows_of(x);
  TORCH_CHECK(wp.numel() == N * K, "packed weight must hold N * K elements");
  if (bias) { need_same(*bias, x, "bias"); TORCH_CHECK(bias->numel() == N); }
  auto os = x.sizes().vec();
  os.back() = epi == 1 ? N / 2 : N;
  auto out = at::empty(os, x.options());
  if (addend) {
    need_same(*addend, x, "addend");
    TORCH_CHECK(epi == 0 && addend->numel() == M * N, "addend: plain output only, M * N elements");
  }
  check(edge_gemv_bf16(x.data_ptr(), wp.data_ptr(), bias ? bias->data_ptr() : nullptr, out.data_ptr(), (int)M, (int)N,
                       (int)K, (int)epi, stream(), addend ? addend->data_ptr() : nullptr, h16),
        "gemv_bf16");
  return out;
}

// Split-K bf16 decode GEMV: fp32 partial slices [S, M, N] (bias in slice 0) for rms_norm_parts.
at::Tensor gemv_bf16_splitk(const at::Tensor& x, const at::Tensor& wp, const std::optional<at::Tensor>& bias,
                            int64_t N, int64_t S) {
  DEVICE_GUARD(x);
  const int h16 = need16(x, "x");
  need_same(wp, x, "weight (packed)");
  const int64_t K = x.size(-1), M = rows_of(x);
  TORCH_CHECK(wp.numel() == N * K, "packed weight must hold N * K elements");
  if (bias) { need_same(*bias, x, "bias"); TORCH_CHECK(bias->numel() == N); }
  auto part = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  check(edge_gemv_bf16_splitk(x.data_ptr(), wp.data_ptr(), bias ? bias->data_ptr() : nullptr, part.data_ptr<float>(),
                              (int)M, (int)N, (int)K, (int)S, stream(), h16),
        "gemv_bf16_splitk");
  return part;
}

// bf16 decode projection at 17-256 rows on the ring2 kernel (gemm_i8.hip, bf16 operand mode) over
// the same fragment-packed weight as gemv_bf16.  epi 0: bf16 [.., N]; 1: SwiGLU over [gate | up]
// -> bf16 [.., N / 2]; 3: split-K fp32 partial slices [S, M, N] (S = 0: the launcher's choice).
at::Tensor gemm_bf16_ring(const at::Tensor& x, const at::Tensor& wp, const std::optional<at::Tensor>& bias, int64_t N,
                          int64_t epi, int64_t S) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  need(wp, at::kBFloat16, "weight (packed)");
  const int64_t K = x.size(-1), M = rows_of(x);
  TORCH_CHECK(wp.numel() == N * K, "packed weight must hold N * K elements");
  TORCH_CHECK(M >= 1 && M <= 256, "bf16 ring GEMM takes 1-256 rows");
  if (bias) { need(*bias, at::kBFloat16, "bias"); TORCH_CHECK(bias->numel() == N); }
  at::Tensor out;
  if (epi == 3) {
    if (S <= 0) S = edge_bf16_ring_splits((int)N, (int)K);
    TORCH_CHECK(S > 1, "split-K bf16 ring needs >= 2 slices at this shape");
    out = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  } else {
    auto os = x.sizes().vec();
    os.back() = epi == 1 ? N / 2 : N;
    out = at::empty(os, x.options());
    S = 1;
  }
  check(edge_gemm_bf16_ring(x.data_ptr(), wp.data_ptr(), bias ? bias->data_ptr() : nullptr, out.data_ptr(), (int)M,
                            (int)N, (int)K, (int)epi, (int)S, stream()),
        "gemm_bf16_ring");
  return out;
}

// LLM.int8 decode preparation (M <= 16): (q int8 [M, K] with the outlier columns zeroed, per-token
// scales [M], outlier columns [cmax] (first `count`), outlier values [M, cmax], count [1]).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> llmint8_prep(const at::Tensor& x, double thr,
                                                                                    int64_t cmax) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 2, "x must be [M, K]");
  const int64_t M = x.size(0), K = x.size(1);
  auto q = at::empty({M, K}, x.options().dtype(at::kChar));
  auto sa = at::empty({M}, x.options().dtype(at::kFloat));
  auto cols = at::zeros({cmax}, x.options().dtype(at::kInt));
  auto xo = at::zeros({M, cmax}, x.options().dtype(at::kFloat));
  auto count = at::empty({1}, x.options().dtype(at::kInt));
  check(edge_llmint8_prep(x.data_ptr(), (int)M, (int)K, (float)thr, (int)cmax, q.data_ptr(), sa.data_ptr<float>(),
                          cols.data_ptr<int>(), xo.data_ptr<float>(), count.data_ptr<int>(), stream()),
        "llmint8_prep");
  return {q, sa, cols, xo, count};
}

// out bf16 [M, N] += xo[:, :count] . W^T[cols[:count]] * SCB / 127 (wt = int8 W^T [K, N]), in place.
void llmint8_outlier(at::Tensor& out, const at::Tensor& xo, const at::Tensor& cols, const at::Tensor& count,
                     const at::Tensor& wt, const at::Tensor& scb) {
  DEVICE_GUARD(out);
  need(out, at::kBFloat16, "out");
  need(xo, at::kFloat, "xo");
  need(cols, at::kInt, "cols");
  need(count, at::kInt, "count");
  need(wt, at::kChar, "weight_t");
  need(scb, at::kFloat, "SCB");
  const int64_t M = out.size(0), N = out.size(1);
  TORCH_CHECK(out.dim() == 2 && wt.dim() == 2 && wt.size(1) == N && xo.size(0) == M && xo.size(1) == cols.numel());
  check(edge_llmint8_outlier(out.data_ptr(), xo.data_ptr<float>(), cols.data_ptr<int>(), count.data_ptr<int>(),
                             wt.data_ptr(), scb.data_ptr<float>(), (int)M, (int)N, (int)cols.numel(), stream()),
        "llmint8_outlier");
}

// LLM.int8 projection of one bf16 row [1, K] in one launch (gemm_i8.hip l8_prologue: outlier
// columns, int8 quant, GEMV, outlier part): bf16 [1, N], or None when the shape is not taken.
std::optional<at::Tensor> llmint8_gemv(const at::Tensor& x, double thr, const at::Tensor& wp, const at::Tensor& sw,
                                       const std::optional<at::Tensor>& bias, const at::Tensor& wt,
                                       const at::Tensor& scb, int64_t N, int64_t act) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  need(wt, at::kChar, "weight_t");
  need(scb, at::kFloat, "SCB");
  TORCH_CHECK(x.dim() == 2 && x.size(0) == 1 && x.is_contiguous(), "x must be contiguous [1, K]");
  const int64_t K = x.size(1);
  check_w8a8_operands(wp, sw, bias, N, K);
  TORCH_CHECK(wt.dim() == 2 && wt.size(0) == K && wt.size(1) == N && wt.is_contiguous() && scb.numel() == N,
              "weight_t [K, N], SCB [N]");
  auto out = at::empty({1, N}, x.options());
  const int r = edge_llmint8_gemv(x.data_ptr(), (float)thr, wp.data_ptr(), sw.data_ptr<float>(),
                                  bias ? bias->data_ptr() : nullptr, wt.data_ptr(), scb.data_ptr<float>(),
                                  out.data_ptr(), (int)N, (int)K, stream(), (int)act);
  if (r == -2) return std::nullopt;
  check(r, "llmint8_gemv");
  return out;
}

// The same over RMSNorm (ln false) / LayerNorm (ln true) of x + residual computed first; res_out gets
// x + residual, y_out (optional) the normalised row.
std::optional<at::Tensor> llmint8_gemv_norm(const at::Tensor& x, const std::optional<at::Tensor>& residual,
                                            const at::Tensor& gamma, const std::optional<at::Tensor>& beta,
                                            double eps, bool ln, const at::Tensor& res_out,
                                            const std::optional<at::Tensor>& y_out, double thr, const at::Tensor& wp,
                                            const at::Tensor& sw, const std::optional<at::Tensor>& bias,
                                            const at::Tensor& wt, const at::Tensor& scb, int64_t N, bool glu,
                                            int64_t act) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  need(gamma, at::kBFloat16, "gamma");
  need(res_out, at::kBFloat16, "res_out");
  need(wt, at::kChar, "weight_t");
  need(scb, at::kFloat, "SCB");
  TORCH_CHECK(x.dim() == 2 && x.size(0) == 1 && x.is_contiguous(), "x must be contiguous [1, K]");
  const int64_t K = x.size(1);
  check_w8a8_operands(wp, sw, bias, N, K);
  TORCH_CHECK(wt.dim() == 2 && wt.size(0) == K && wt.size(1) == N && wt.is_contiguous() && scb.numel() == N,
              "weight_t [K, N], SCB [N]");
  TORCH_CHECK(gamma.numel() == K && res_out.numel() == K, "gamma [K], res_out [1, K]");
  if (beta) { need(*beta, at::kBFloat16, "beta"); TORCH_CHECK(beta->numel() == K, "beta [K]"); }
  if (residual) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == K && residual->data_ptr() != res_out.data_ptr(), "residual [1, K]");
  }
  if (y_out) { need(*y_out, at::kBFloat16, "y_out"); TORCH_CHECK(y_out->numel() == K, "y_out [1, K]"); }
  auto out = at::empty({1, glu ? N / 2 : N}, x.options());
  const int r = edge_llmint8_gemv_norm(x.data_ptr(), residual ? residual->data_ptr() : nullptr, gamma.data_ptr(),
                                       beta ? beta->data_ptr() : nullptr, (float)eps, ln ? 1 : 0, res_out.data_ptr(),
                                       y_out ? y_out->data_ptr() : nullptr, (float)thr, wp.data_ptr(),
                                       sw.data_ptr<float>(), bias ? bias->data_ptr() : nullptr, wt.data_ptr(),
                                       scb.data_ptr<float>(), out.data_ptr(), (int)N, (int)K, stream(), glu ? 1 : 0,
                                       (int)act);
  if (r == -2) return std::nullopt;
  check(r, "llmint8_gemv_norm");
  return out;
}

// LLM.int8 preparation for any number of rows, uncapped (every outlier column to the 16-bit part):
// (q int8 [M, K] with the outlier columns zeroed, per-token scales [M], outlier columns [K] (first
// `count`), count [1]).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> llmint8_prep_rows(const at::Tensor& x, double thr) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "x must be contiguous [M, K]");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 32 == 0 && M > 0, "llmint8_prep_rows: K % 32 == 0");
  auto q = at::empty({M, K}, x.options().dtype(at::kChar));
  auto sa = at::empty({M}, x.options().dtype(at::kFloat));
  auto cols = at::empty({K}, x.options().dtype(at::kInt));
  auto count = at::empty({1}, x.options().dtype(at::kInt));
  auto bits = at::empty({2 * (K / 32)}, x.options().dtype(at::kInt));
  uint32_t* flags = reinterpret_cast<uint32_t*>(bits.data_ptr<int>());
  check(edge_llmint8_prep_rows(x.data_ptr(), (int)M, (int)K, (float)thr, q.data_ptr(), sa.data_ptr<float>(),
                               cols.data_ptr<int>(), count.data_ptr<int>(), flags, flags + K / 32, stream()),
        "llmint8_prep_rows");
  return {q, sa, cols, count};
}

// out bf16 [M, N] += x[:, cols[:count]] . W^T[cols[:count]] * SCB / 127 (wt = int8 W^T [K, N]), in place.
void llmint8_outlier_rows(at::Tensor& out, const at::Tensor& x, const at::Tensor& cols, const at::Tensor& count,
                          const at::Tensor& wt, const at::Tensor& scb) {
  DEVICE_GUARD(out);
  need(out, at::kBFloat16, "out");
  need(x, at::kBFloat16, "x");
  need(cols, at::kInt, "cols");
  need(count, at::kInt, "count");
  need(wt, at::kChar, "weight_t");
  need(scb, at::kFloat, "SCB");
  const int64_t M = out.size(0), N = out.size(1), K = x.size(1);
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && x.dim() == 2 && x.is_contiguous() && x.size(0) == M &&
                  wt.dim() == 2 && wt.is_contiguous() && wt.size(0) == K && wt.size(1) == N && cols.numel() == K &&
                  scb.numel() == N,
              "llmint8_outlier_rows: shapes");
  check(edge_llmint8_outlier_rows(out.data_ptr(), x.data_ptr(), cols.data_ptr<int>(), count.data_ptr<int>(),
                                  wt.data_ptr(), scb.data_ptr<float>(), (int)M, (int)N, (int)K, stream()),
        "llmint8_outlier_rows");
}

// Per-(token, 64 columns) int8 quantisation: (q [M, K], scales [K/64, Mpad]).
std::tuple<at::Tensor, at::Tensor> group_quant(const at::Tensor& x) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 64 == 0, "group_quant needs [M, K] with K % 64 == 0");
  const int64_t M = x.size(0), K = x.size(1), Mpad = (M + 15) / 16 * 16;
  auto q = at::empty({M, K}, x.options().dtype(at::kChar));
  auto s = at::empty({K / 64, Mpad}, x.options().dtype(at::kFloat));
  check(edge_group_quant(x.data_ptr(), q.data_ptr(), s.data_ptr<float>(), (int)M, (int)K, (int)Mpad, stream()),
        "group_quant");
  return {q, s};
}

// Decode W8A8 GEMV (M <= 4 rows) over RMSNorm(sum of split-K slices parts [S, M, K] + residual),
// the norm and its per-token int8 quantisation computed in the GEMV's prologue (gemm_i8.hip
// NormIn).  epi 0: (bf16 y [M, N], None); epi 2 (16-blocked gate_up, quantising SwiGLU): (int8 h
// [M, N/2], scales [N/128, 16]); the new residual rows (sum + residual, bf16) are written to
// res_out ([M, K], not aliasing residual).  Returns None when no kernel takes it.
std::optional<std::tuple<at::Tensor, std::optional<at::Tensor>>> w8a8_gemv_norm(
    const at::Tensor& parts, const std::optional<at::Tensor>& residual, const at::Tensor& gamma, double eps,
    const at::Tensor& res_out,
    const at::Tensor& wp, const at::Tensor& sw, const std::optional<at::Tensor>& bias, int64_t N, int64_t K,
    int64_t epi) {
  DEVICE_GUARD(parts);
  need(parts, at::kFloat, "parts");
  need(gamma, at::kBFloat16, "gamma");
  check_w8a8_operands(wp, sw, bias, N, K);
  TORCH_CHECK(parts.dim() == 3 && parts.size(2) == K, "parts must be [S, M, K]");
  const int64_t M = parts.size(1);
  TORCH_CHECK(gamma.numel() == K, "gamma [K]");
  need(res_out, at::kBFloat16, "res_out");
  TORCH_CHECK(res_out.numel() == M * K, "res_out: [M, K]");
  if (residual) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == M * K && res_out.data_ptr() != residual->data_ptr(),
                "residual [M, K], not aliasing res_out");
  }
  TORCH_CHECK(epi == 0 || epi == 2, "epi 0 (out) or 2 (quantising GLU)");
  const int64_t S = parts.size(0);
  if (!edge_w8a8_gemv_norm_on() || M < 1 || M > 4 || S < 1 || S > 4 || (K != 2048 && K != 4096) || N % (epi == 2 ? 128 : 16) != 0)
    return std::nullopt;
  at::Tensor y;
  std::optional<at::Tensor> s;
  if (epi == 0) {
    y = at::empty({M, N}, res_out.options());
  } else {
    y = at::empty({M, N / 2}, res_out.options().dtype(at::kChar));
    s = at::empty({N / 128, 16}, res_out.options().dtype(at::kFloat));
  }
  check(edge_w8a8_gemv_norm(parts.data_ptr<float>(), (int)S, residual ? residual->data_ptr() : nullptr,
                            gamma.data_ptr(), (float)eps,
                            res_out.data_ptr(), wp.data_ptr(), sw.data_ptr<float>(), bias ? bias->data_ptr() : nullptr,
                            y.data_ptr(), s ? s->data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, (int)epi,
                            stream()),
        "w8a8_gemv_norm");
  return std::make_tuple(y, s);
}

// 16-bit decode GEMV (M <= 4) over RMSNorm(sum(parts) + residual) computed in its prologue
// (gemv_bf16.hip norm16_prologue): epi 0 -> y [M, N], 1 -> SwiGLU of [gate | up], y [M, N / 2];
// the new residual rows go to res_out.  None when no kernel takes the shape.
std::optional<at::Tensor> gemv_bf16_norm(const at::Tensor& parts, const std::optional<at::Tensor>& residual,
                                         const at::Tensor& gamma, double eps, const at::Tensor& res_out,
                                         const at::Tensor& wp, const std::optional<at::Tensor>& bias, int64_t N,
                                         int64_t epi) {
  DEVICE_GUARD(parts);
  need(parts, at::kFloat, "parts");
  const bool h16 = gamma.scalar_type() == at::kHalf;
  const auto dt = h16 ? at::kHalf : at::kBFloat16;
  need(gamma, dt, "gamma");
  need(res_out, dt, "res_out");
  need(wp, dt, "weight");
  TORCH_CHECK(parts.dim() == 3, "parts must be [S, M, K]");
  const int64_t S = parts.size(0), M = parts.size(1), K = parts.size(2);
  TORCH_CHECK(gamma.numel() == K && res_out.numel() == M * K, "gamma [K], res_out [M, K]");
  TORCH_CHECK(wp.numel() == N * K, "packed weight [N, K]");
  if (residual) {
    need(*residual, dt, "residual");
    TORCH_CHECK(residual->numel() == M * K && res_out.data_ptr() != residual->data_ptr(),
                "residual [M, K], not aliasing res_out");
  }
  if (bias) { need(*bias, dt, "bias"); TORCH_CHECK(bias->numel() == N, "bias [N]"); }
  TORCH_CHECK(epi == 0 || epi == 1, "epi 0 (out) or 1 (SwiGLU)");
  if (M < 1 || M > 4 || S < 1 || S > 4 || (K != 2048 && K != 4096) || N % (epi == 1 ? 32 : 16) != 0)
    return std::nullopt;
  auto y = at::empty({M, epi == 1 ? N / 2 : N}, res_out.options());
  const int r = edge_gemv_bf16_norm(parts.data_ptr<float>(), (int)S, residual ? residual->data_ptr() : nullptr,
                                    gamma.data_ptr(), (float)eps, res_out.data_ptr(), wp.data_ptr(),
                                    bias ? bias->data_ptr() : nullptr, y.data_ptr(), (int)M, (int)N, (int)K, (int)epi,
                                    stream(), h16 ? 1 : 0);
  if (r == -2) return std::nullopt;
  check(r, "gemv_bf16_norm");
  return y;
}

// 16-bit decode GEMV (M <= 4) over LayerNorm(x + residual) computed in its prologue (the
// parallel-residual decoders): epi 0 -> y [M, N], 2 / 3 -> gelu (tanh / erf); x + residual goes to
// res_out.  None when no kernel takes the shape.
std::optional<at::Tensor> gemv_bf16_ln(const at::Tensor& x, const std::optional<at::Tensor>& residual,
                                       const at::Tensor& gamma, const std::optional<at::Tensor>& beta, double eps,
                                       const at::Tensor& res_out, const at::Tensor& wp,
                                       const std::optional<at::Tensor>& bias, int64_t N, int64_t epi,
                                       const std::optional<at::Tensor>& y_out) {
  DEVICE_GUARD(x);
  const bool h16 = gamma.scalar_type() == at::kHalf;
  const auto dt = h16 ? at::kHalf : at::kBFloat16;
  need(x, dt, "x");
  need(gamma, dt, "gamma");
  need(res_out, dt, "res_out");
  need(wp, dt, "weight");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "x must be contiguous [M, K]");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(gamma.numel() == K && res_out.numel() == M * K && wp.numel() == N * K, "gamma [K], res_out [M, K], W [N, K]");
  if (beta) { need(*beta, dt, "beta"); TORCH_CHECK(beta->numel() == K, "beta [K]"); }
  if (residual) {
    need(*residual, dt, "residual");
    TORCH_CHECK(residual->numel() == M * K && res_out.data_ptr() != residual->data_ptr(),
                "residual [M, K], not aliasing res_out");
  }
  if (bias) { need(*bias, dt, "bias"); TORCH_CHECK(bias->numel() == N, "bias [N]"); }
  if (y_out) {
    need(*y_out, dt, "y_out");
    TORCH_CHECK(y_out->numel() == M * K && y_out->data_ptr() != res_out.data_ptr(), "y_out [M, K]");
  }
  TORCH_CHECK(epi == 0 || epi == 2 || epi == 3, "epi 0 (out), 2 (gelu tanh), 3 (gelu erf)");
  if (M < 1 || M > 4 || K > 4096 || K % 64 != 0 || N % 16 != 0) return std::nullopt;
  auto y = at::empty({M, N}, res_out.options());
  const int r = edge_gemv_bf16_ln(x.data_ptr(), residual ? residual->data_ptr() : nullptr, gamma.data_ptr(),
                                  beta ? beta->data_ptr() : nullptr, (float)eps, res_out.data_ptr(), wp.data_ptr(),
                                  bias ? bias->data_ptr() : nullptr, y.data_ptr(), (int)M, (int)N, (int)K, (int)epi,
                                  stream(), h16 ? 1 : 0, y_out ? y_out->data_ptr() : nullptr);
  if (r == -2) return std::nullopt;
  check(r, "gemv_bf16_ln");
  return y;
}

// W8A8 decode GEMV (M <= 4) over LayerNorm(x + residual) of bf16 rows, int8 per token, computed
// in its prologue: epi 0 -> (y bf16 [M, N], None); 4 / 5 -> gelu (tanh / erf) of the output, int8
// per (token, 64 columns): (q [M, N], scales [N/64, 16]).  None when no kernel takes the shape.
std::optional<std::tuple<at::Tensor, std::optional<at::Tensor>>> w8a8_gemv_ln(
    const at::Tensor& x, const std::optional<at::Tensor>& residual, const at::Tensor& gamma,
    const std::optional<at::Tensor>& beta, double eps, const at::Tensor& res_out, const at::Tensor& wp,
    const at::Tensor& sw, const std::optional<at::Tensor>& bias, int64_t N, int64_t K, int64_t epi) {
  DEVICE_GUARD(x);
  need(x, at::kBFloat16, "x");
  need(gamma, at::kBFloat16, "gamma");
  need(res_out, at::kBFloat16, "res_out");
  check_w8a8_operands(wp, sw, bias, N, K);
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) == K, "x must be contiguous [M, K]");
  const int64_t M = x.size(0);
  TORCH_CHECK(gamma.numel() == K && res_out.numel() == M * K, "gamma [K], res_out [M, K]");
  if (beta) { need(*beta, at::kBFloat16, "beta"); TORCH_CHECK(beta->numel() == K, "beta [K]"); }
  if (residual) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == M * K && res_out.data_ptr() != residual->data_ptr(),
                "residual [M, K], not aliasing res_out");
  }
  TORCH_CHECK(epi == 0 || epi == 4 || epi == 5, "epi 0 (out), 4 / 5 (gelu tanh / erf + grouped int8)");
  if (!edge_w8a8_gemv_norm_on() || M < 1 || M > 4 || K > 4096 || K % 64 != 0 || N % (epi ? 64 : 16) != 0)
    return std::nullopt;
  at::Tensor y;
  std::optional<at::Tensor> s;
  if (epi == 0) {
    y = at::empty({M, N}, res_out.options());
  } else {
    y = at::empty({M, N}, res_out.options().dtype(at::kChar));
    s = at::zeros({N / 64, 16}, res_out.options().dtype(at::kFloat));
  }
  const int r = edge_w8a8_gemv_ln(x.data_ptr(), residual ? residual->data_ptr() : nullptr, gamma.data_ptr(),
                                  beta ? beta->data_ptr() : nullptr, (float)eps, res_out.data_ptr(), wp.data_ptr(),
                                  sw.data_ptr<float>(), bias ? bias->data_ptr() : nullptr, y.data_ptr(),
                                  s ? s->data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, (int)epi, stream());
  if (r == -2) return std::nullopt;
  check(r, "w8a8_gemv_ln");
  return std::make_tuple(y, s);
}

// gate_up projection (16-blocked rows) fused with silu(g) * u: returns bf16 h [M, N/2].
at::Tensor w8a8_gemm_glu(const at::Tensor& a, const at::Tensor& sa, const at::Tensor& wp, const at::Tensor& sw,
                         const std::optional<at::Tensor>& bias, int64_t N, int64_t K) {
  DEVICE_GUARD(a);
  need(a, at::kChar, "a");
  TORCH_CHECK(a.size(-1) == K, "activation K mismatch");
  check_w8a8_operands(wp, sw, bias, N, K);
  const int64_t M = rows_of(a), KT = (K + 63) / 64;
  TORCH_CHECK(M <= 64 && N % 32 == 0, "fused GLU needs M <= 64 and N % 32 == 0");
  TORCH_CHECK(a_scale_mpad(sa, M, KT) == 0, "fused GLU takes per-token activation scales");
  auto h = at::empty({M, N / 2}, a.options().dtype(at::kBFloat16));
  check(edge_w8a8_gemm(a.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                       bias ? bias->data_ptr() : nullptr, h.data_ptr(), nullptr, (int)M, (int)N, (int)K, (int)KT, 0,
                       0, 1, stream()),
        "w8a8_gemm_glu");
  return h;
}

// As w8a8_gemm_glu, then int8 per-(token, 64 features) quantisation in the same kernel:
// returns (q int8 [M, N/2], scales [N/128, Mpad]).
std::tuple<at::Tensor, at::Tensor> w8a8_gemm_gluq(const at::Tensor& a, const at::Tensor& sa, const at::Tensor& wp,
                                                  const at::Tensor& sw, const std::optional<at::Tensor>& bias,
                                                  int64_t N, int64_t K) {
  DEVICE_GUARD(a);
  need(a, at::kChar, "a");
  TORCH_CHECK(a.size(-1) == K, "activation K mismatch");
  check_w8a8_operands(wp, sw, bias, N, K);
  const int64_t M = rows_of(a), KT = (K + 63) / 64, Mpad = (M + 15) / 16 * 16;
  TORCH_CHECK((M <= 64 || (M <= 128 && edge_w8a8_rows128_ok((int)K, 1)) || (M <= 256 && edge_w8a8_rows256_ok((int)K)))
                  && N % 128 == 0,
              "quantising GLU needs M <= 64 (128 where rows128_ok(K), 256 where rows256_ok(K)) and N % 128 == 0");
  TORCH_CHECK(a_scale_mpad(sa, M, KT) == 0, "fused GLU takes per-token activation scales");
  auto q = at::empty({M, N / 2}, a.options());
  auto s = at::empty({N / 128, Mpad}, a.options().dtype(at::kFloat));
  check(edge_w8a8_gemm(a.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                       bias ? bias->data_ptr() : nullptr, q.data_ptr(), s.data_ptr<float>(), (int)M, (int)N, (int)K,
                       (int)KT, 0, (int)Mpad, 2, stream()),
        "w8a8_gemm_gluq");
  return {q, s};
}

// W8A8 up projection + GELU (tanh or erf) + per-(token, 64 columns) int8 quantisation in one launch
// (M <= 64, N % 64 == 0): (q [M, N] int8, scales [N / 64, Mpad]) for the down projection's grouped-
// scale GEMV — the GELU MLPs' (Phi-2, Pythia) replacement for GEMV -> act_kernel + quant.
std::tuple<at::Tensor, at::Tensor> w8a8_gemm_geluq(const at::Tensor& a, const at::Tensor& sa, const at::Tensor& wp,
                                                   const at::Tensor& sw, const std::optional<at::Tensor>& bias,
                                                   int64_t N, int64_t K, bool tanh_approx) {
  DEVICE_GUARD(a);
  need(a, at::kChar, "a");
  TORCH_CHECK(a.size(-1) == K, "activation K mismatch");
  check_w8a8_operands(wp, sw, bias, N, K);
  const int64_t M = rows_of(a), KT = (K + 63) / 64, Mpad = (M + 15) / 16 * 16;
  TORCH_CHECK(M <= 64 && N % 64 == 0, "quantising GELU needs M <= 64 and N % 64 == 0");
  TORCH_CHECK(a_scale_mpad(sa, M, KT) == 0, "fused GELU takes per-token activation scales");
  auto q = at::empty({M, N}, a.options());
  auto s = at::empty({N / 64, Mpad}, a.options().dtype(at::kFloat));
  check(edge_w8a8_gemm(a.data_ptr(), sa.data_ptr<float>(), wp.data_ptr(), sw.data_ptr<float>(),
                       bias ? bias->data_ptr() : nullptr, q.data_ptr(), s.data_ptr<float>(), (int)M, (int)N, (int)K,
                       (int)KT, 0, (int)Mpad, tanh_approx ? 4 : 5, stream()),
        "w8a8_gemm_geluq");
  return {q, s};
}

// ---------------------------------------------------------------------------------- sampler
// Returns an empty tensor when the configuration needs the host fallback.
at::Tensor sample(const at::Tensor& logits, const std::optional<at::Tensor>& seen, double temperature,
                  int64_t top_k, double top_p, double penalty, bool do_sample, const at::Tensor& rng) {
  DEVICE_GUARD(logits);
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2);
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat);
  need(rng, at::kInt, "rng");
  const int64_t B = logits.size(0), V = logits.size(1);
  if (seen) { need(*seen, at::kByte, "seen"); TORCH_CHECK(seen->sizes() == logits.sizes()); }
  auto out = at::empty({B}, logits.options().dtype(at::kLong));
  auto ws = at::empty({(int64_t)edge_sample_workspace((int)B, (int)V)}, logits.options().dtype(at::kByte));
  const double inv_t = temperature > 0 ? 1.0 / temperature : 1.0;
  const int rc = edge_sample(logits.data_ptr(), bf, seen ? seen->data_ptr<uint8_t>() : nullptr, (int)B, (int)V,
                             (float)temperature, (float)inv_t, (float)penalty, (int)top_k, (float)top_p, do_sample,
                             rng.data_ptr<int>(), out.data_ptr<int64_t>(), ws.data_ptr(), stream());
  if (rc == -5) return at::Tensor();
  check(rc, "sample");
  return out;
}

// Vocab-sharded sampler (parallel/vocab_head.py).  sample_shard: phase 1 over logits [B, Vs] =
// columns [v0, v0 + Vs) of a V-wide row -> (pc int64 [B, C * 128] composites + pthr int32 [B, C])
// for top-k, or (pc [B, C], empty) for greedy / full-vocab sampling; None when the configuration
// does not shard (top-k > 128, top-p without top-k).
std::optional<std::tuple<at::Tensor, at::Tensor>> sample_shard(const at::Tensor& logits,
                                                               const std::optional<at::Tensor>& seen, double temperature,
                                                               int64_t top_k, double top_p, double penalty,
                                                               bool do_sample, const at::Tensor& rng, int64_t v0,
                                                               int64_t V) {
  DEVICE_GUARD(logits);
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2);
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat, "sample_shard: bf16 or fp32 logits");
  need(rng, at::kInt, "rng");
  const int64_t B = logits.size(0), Vs = logits.size(1);
  TORCH_CHECK(v0 >= 0 && v0 + Vs <= V, "shard outside the vocabulary");
  if (seen) { need(*seen, at::kByte, "seen"); TORCH_CHECK(seen->sizes() == logits.sizes()); }
  const int mode = edge_sample_shard_mode(do_sample, (float)temperature, (int)top_k, (float)top_p, (int)V);
  if (mode < 0) return std::nullopt;
  const int64_t C = edge_sample_shard_chunks((int)Vs, (int)V);
  auto pc = at::empty({B, mode == 2 ? C * 128 : C}, logits.options().dtype(at::kLong));
  auto pthr = at::empty({B, mode == 2 ? C : 0}, logits.options().dtype(at::kInt));
  const double inv_t = temperature > 0 ? 1.0 / temperature : 1.0;
  check(edge_sample_shard(logits.data_ptr(), bf, seen ? seen->data_ptr<uint8_t>() : nullptr, (int)B, (int)Vs, (int)v0,
                          (int)V, (float)temperature, (float)inv_t, (float)penalty, (int)top_k, (float)top_p, do_sample,
                          rng.data_ptr<int>(), reinterpret_cast<uint64_t*>(pc.data_ptr<int64_t>()),
                          mode == 2 ? reinterpret_cast<uint32_t*>(pthr.data_ptr<int>()) : nullptr, stream()),
        "sample_shard");
  return std::make_tuple(pc, pthr);
}

// Phase 2 over the shards' lists concatenated per row (pc [B, C_total * 128] + pthr [B, C_total],
// or pc [B, C_total]) -> tokens int64 [B].
at::Tensor sample_merge(const at::Tensor& pc, const at::Tensor& pthr, int64_t V, double temperature, int64_t top_k,
                        double top_p, bool do_sample, const at::Tensor& rng) {
  DEVICE_GUARD(pc);
  need(pc, at::kLong, "pc");
  need(rng, at::kInt, "rng");
  const int mode = edge_sample_shard_mode(do_sample, (float)temperature, (int)top_k, (float)top_p, (int)V);
  TORCH_CHECK(mode >= 0, "sample_merge: configuration is not shardable");
  const int64_t B = pc.size(0);
  int64_t C = pc.size(1);
  if (mode == 2) {
    need(pthr, at::kInt, "pthr");
    TORCH_CHECK(pthr.size(0) == B && pc.size(1) == pthr.size(1) * 128, "pc / pthr shapes");
    C = pthr.size(1);
  }
  auto out = at::empty({B}, pc.options());
  check(edge_sample_merge(reinterpret_cast<const uint64_t*>(pc.data_ptr<int64_t>()),
                          mode == 2 ? reinterpret_cast<const uint32_t*>(pthr.data_ptr<int>()) : nullptr, (int)B, (int)C,
                          (int)V, (float)temperature, (int)top_k, (float)top_p, do_sample, rng.data_ptr<int>(),
                          out.data_ptr<int64_t>(), stream()),
        "sample_merge");
  return out;
}

int64_t sample_shard_chunks(int64_t Vs, int64_t V) { return edge_sample_shard_chunks((int)Vs, (int)V); }
int64_t sample_shard_mode(bool do_sample, double temperature, int64_t top_k, double top_p, int64_t V) {
  return edge_sample_shard_mode(do_sample, (float)temperature, (int)top_k, (float)top_p, (int)V);
}

// After the sampler: tok = nxt, out[:, step] = nxt, pos += inc, seq_lens += inc (inc: int32 [B] or
// None = 1), rng[1] += 1, step += 1 (one launch; the decode state's buffers, all on the sampler's device).
void decode_advance(const at::Tensor& nxt, at::Tensor& tok, at::Tensor& out, at::Tensor& step, at::Tensor& pos,
                    at::Tensor& seq_lens, at::Tensor& rng, const std::optional<at::Tensor>& inc) {
  DEVICE_GUARD(nxt);
  need(nxt, at::kLong, "nxt");
  need(tok, at::kLong, "tok");
  need(out, at::kLong, "out");
  need(step, at::kLong, "step");
  need(pos, at::kInt, "pos");
  need(seq_lens, at::kInt, "seq_lens");
  need(rng, at::kInt, "rng");
  const int64_t B = nxt.numel();
  TORCH_CHECK(tok.numel() == B && pos.numel() == B && seq_lens.numel() == B && step.numel() == 1 && rng.numel() == 2,
              "decode_advance: B-row state, one step counter, [seed, step] rng");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == B && out.stride(1) == 1, "out: [B, max_new] with contiguous rows");
  TORCH_CHECK(nxt.is_contiguous() && tok.is_contiguous() && pos.is_contiguous() && seq_lens.is_contiguous() &&
              rng.is_contiguous(), "decode_advance: contiguous state");
  if (inc) {
    need(*inc, at::kInt, "inc");
    TORCH_CHECK(inc->numel() == B && inc->is_contiguous(), "inc: int32 [B]");
  }
  check(edge_decode_advance(nxt.data_ptr<int64_t>(), tok.data_ptr<int64_t>(), out.data_ptr<int64_t>(), out.stride(0),
                            (int)out.size(1), step.data_ptr<int64_t>(), pos.data_ptr<int>(), seq_lens.data_ptr<int>(),
                            rng.data_ptr<int>(), inc ? inc->data_ptr<int>() : nullptr, (int)B, stream()),
        "decode_advance");
}

// sample + decode_advance (inc = 1) with the bookkeeping in the sampler's last launch.  ctr: int32 [1],
// zero before the first call (each call leaves it zero).  Returns an empty tensor when the
// configuration needs the host fallback (nothing was launched then).
at::Tensor sample_advance(const at::Tensor& logits, const std::optional<at::Tensor>& seen, double temperature,
                          int64_t top_k, double top_p, double penalty, bool do_sample, at::Tensor& rng, at::Tensor& tok,
                          at::Tensor& out, at::Tensor& step, at::Tensor& pos, at::Tensor& seq_lens, at::Tensor& ctr) {
  DEVICE_GUARD(logits);
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2);
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat);
  need(rng, at::kInt, "rng");
  need(tok, at::kLong, "tok");
  need(out, at::kLong, "out");
  need(step, at::kLong, "step");
  need(pos, at::kInt, "pos");
  need(seq_lens, at::kInt, "seq_lens");
  need(ctr, at::kInt, "ctr");
  const int64_t B = logits.size(0), V = logits.size(1);
  if (seen) { need(*seen, at::kByte, "seen"); TORCH_CHECK(seen->sizes() == logits.sizes()); }
  TORCH_CHECK(tok.numel() == B && pos.numel() == B && seq_lens.numel() == B && step.numel() == 1 && rng.numel() == 2 &&
              ctr.numel() >= 1, "sample_advance: B-row state, one step counter, [seed, step] rng, a counter");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == B && out.stride(1) == 1, "out: [B, max_new] with contiguous rows");
  TORCH_CHECK(tok.is_contiguous() && pos.is_contiguous() && seq_lens.is_contiguous() && rng.is_contiguous(),
              "sample_advance: contiguous state");
  auto nxt = at::empty({B}, logits.options().dtype(at::kLong));
  auto ws = at::empty({(int64_t)edge_sample_workspace((int)B, (int)V)}, logits.options().dtype(at::kByte));
  const double inv_t = temperature > 0 ? 1.0 / temperature : 1.0;
  const int rc = edge_sample_advance(logits.data_ptr(), bf, seen ? seen->data_ptr<uint8_t>() : nullptr, (int)B, (int)V,
                                     (float)temperature, (float)inv_t, (float)penalty, (int)top_k, (float)top_p,
                                     do_sample, rng.data_ptr<int>(), nxt.data_ptr<int64_t>(), ws.data_ptr(),
                                     tok.data_ptr<int64_t>(), out.data_ptr<int64_t>(), out.stride(0), (int)out.size(1),
                                     step.data_ptr<int64_t>(), pos.data_ptr<int>(), seq_lens.data_ptr<int>(),
                                     ctr.data_ptr<int>(), stream());
  if (rc == -5) return at::Tensor();
  check(rc, "sample_advance");
  return nxt;
}

std::vector<int64_t> sample_timestamps(bool enable) {
  std::vector<unsigned long long> ts(16, 0);
  check(edge_sample_timestamps(enable ? 1 : 0, ts.data()), "sample_timestamps");
  return std::vector<int64_t>(ts.begin(), ts.end());
}

// ---------------------------------------------------------------------------------- offload
// dst/src: [B, c, L, D] views of head-major caches (last two dims contiguous), any mix of pinned
// host and device memory; async on the current stream.
int64_t copy_head_block(at::Tensor& dst, const at::Tensor& src, int64_t mode) {
  DEVICE_GUARD((dst.is_cuda() ? dst : src));
  TORCH_CHECK(dst.dim() == 4 && src.dim() == 4 && dst.sizes() == src.sizes(), "head blocks must match [B,c,L,D]");
  TORCH_CHECK(dst.scalar_type() == src.scalar_type());
  const int64_t D = dst.size(3), L = dst.size(2);
  TORCH_CHECK(dst.stride(3) == 1 && src.stride(3) == 1 && dst.stride(2) == D && src.stride(2) == D,
              "positions x head_dim must be contiguous");
  TORCH_CHECK(dst.is_cuda() || dst.is_pinned(), "host side must be pinned");
  TORCH_CHECK(src.is_cuda() || src.is_pinned(), "host side must be pinned");
  const int es = (int)dst.element_size();
  int used = 0;
  check(edge_copy_head_block(dst.data_ptr(), dst.stride(0), dst.stride(1), src.data_ptr(), src.stride(0),
                             src.stride(1), (int)dst.size(0), (int)dst.size(1), L * D * es, es, stream(), (int)mode,
                             &used),
        "copy_head_block");
  return used;          // 1: copy kernel over mapped memory, 2: copy engines (hipMemcpy2DAsync)
}

// stream a device tensor's bytes through the cache hierarchy (MALL warm-up ahead of a reader)


// Batch-1 persistent decode (b1_engine.hip; the layout and buffers come from engine/b1_engine.py).
// t: ws, sw_q, sw_o, sw_gu, sw_d, gam1, gam2, rope, x0, xout, kc, vc, pos, gx, gq, ga, gr, gh, ctl [, stamps]
// iv: fmax, kv_l, kv_h, L, H, Hq, Hkv, F, NQ, gpc_x, gpc_q, gpc_h, xqb, sxn, scb, G, D, HD, lds
void b1_decode(const std::vector<torch::Tensor>& t, const std::vector<int64_t>& iv, double eps, double scale) {
  TORCH_CHECK((t.size() == 19 || t.size() == 20) && iv.size() == 19, "b1_decode: argument count");
  for (const auto& x : t) TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "b1_decode: contiguous GPU tensors");
  const at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(t[0].device());
  B1Params p{};
  p.ws = (const int8_t*)t[0].data_ptr();
  p.fmax = iv[0];
  p.sw_q = t[1].data_ptr<float>();
  p.sw_o = t[2].data_ptr<float>();
  p.sw_gu = t[3].data_ptr<float>();
  p.sw_d = t[4].data_ptr<float>();
  p.gam1 = (const b1_bf16_t*)t[5].data_ptr();
  p.gam2 = (const b1_bf16_t*)t[6].data_ptr();
  p.rope = t[7].data_ptr<float>();
  p.x0 = (const b1_bf16_t*)t[8].data_ptr();
  p.xout = (b1_bf16_t*)t[9].data_ptr();
  p.kc = (b1_bf16_t*)t[10].data_ptr();
  p.vc = (b1_bf16_t*)t[11].data_ptr();
  p.kv_l = iv[1];
  p.kv_h = iv[2];
  p.pos = t[12].data_ptr<int>();
  p.gx = (uint64_t*)t[13].data_ptr();
  p.gq = (uint64_t*)t[14].data_ptr();
  p.ga = (uint64_t*)t[15].data_ptr();
  p.gr = (uint64_t*)t[16].data_ptr();
  p.gh = (uint64_t*)t[17].data_ptr();
  p.ctl = t[18].data_ptr<int>();
  p.stamps = t.size() == 20 ? (long long*)t[19].data_ptr() : nullptr;
  p.L = (int)iv[3]; p.H = (int)iv[4]; p.Hq = (int)iv[5]; p.Hkv = (int)iv[6]; p.F = (int)iv[7]; p.NQ = (int)iv[8];
  p.eps = (float)eps;
  p.scale = (float)scale;
  p.gpc_x = (int)iv[9]; p.gpc_q = (int)iv[10]; p.gpc_h = (int)iv[11];
  p.xqb = (int)iv[12]; p.sxn = (int)iv[13]; p.scb = (int)iv[14];
  check(edge_b1_decode(&p, (int)iv[15], (int)iv[16], (int)iv[17], (int)iv[18], stream()), "b1_decode");
}

int b1_lds_bytes(int D, int xqb, int sxn, int scb) { return edge_b1_lds_bytes(D, xqb, sxn, scb); }

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("copy_head_block", &copy_head_block, py::arg("dst"), py::arg("src"), py::arg("mode") = 0);
  m.doc() = "edgellm CDNA4 (gfx950) HIP kernels";
  m.def("b1_decode", &b1_decode);
  m.def("b1_lds_bytes", &b1_lds_bytes);
  m.def("norm", &norm);
  m.def("act", &act);
  m.def("quant", &quant);
  m.def("embedding", &embedding, py::arg("ids"), py::arg("table"), py::arg("out_f32") = false);
  m.def("max_prob", &max_prob);
  m.def("rope_kv_write", &rope_kv_write, py::arg("qkv"), py::arg("start_pos"), py::arg("rope"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"), py::arg("rot"), py::arg("k2") = py::none(),
        py::arg("v2") = py::none(), py::arg("split") = -1, py::arg("cpos2") = py::none());
  m.def("decode_attn", &decode_attn);
  m.def("prefill_attn", &prefill_attn);
  m.def("w8a8_gemm", &w8a8_gemm, py::arg("a"), py::arg("sa"), py::arg("wp"), py::arg("sw"), py::arg("bias"),
        py::arg("N"), py::arg("K"), py::arg("addend") = py::none());
  m.def("llmint8_prep", &llmint8_prep, "LLM.int8 decode preparation (outlier columns on the device)");
  m.def("llmint8_outlier", &llmint8_outlier, "LLM.int8 decode outlier part, added in place");
  m.def("gemv_bf16_norm", &gemv_bf16_norm, "16-bit decode GEMV with the RMSNorm in its prologue (M <= 4)");
  m.def("gemv_bf16_ln", &gemv_bf16_ln, "16-bit decode GEMV with the LayerNorm in its prologue (M <= 4)");
  m.def("w8a8_gemv_ln", &w8a8_gemv_ln, "W8A8 decode GEMV with the LayerNorm + int8 quant in its prologue (M <= 4)");
  m.def("llmint8_gemv", &llmint8_gemv, "LLM.int8 projection of one row in one launch (prep in the GEMV prologue)");
  m.def("llmint8_gemv_norm", &llmint8_gemv_norm, "LLM.int8 projection of RMSNorm / LayerNorm(x + residual), one launch");
  m.def("llmint8_prep_rows", &llmint8_prep_rows, "LLM.int8 preparation for any rows (uncapped, on the device)");
  m.def("llmint8_outlier_rows", &llmint8_outlier_rows, "LLM.int8 outlier part for any rows, added in place");
  m.def("gemv_bf16_splitk", &gemv_bf16_splitk, "bf16 decode GEMV, split-K fp32 partial slices");
  m.def("gemm_bf16_ring", &gemm_bf16_ring, "bf16 decode GEMM, 17-256 rows (ring2 kernel, bf16 MFMA)");
  m.def("bf16_ring_splits", [](int64_t N, int64_t K) { return (int64_t)edge_bf16_ring_splits((int)N, (int)K); });
  m.def("bf16_ring_min_rows", []() { return (int64_t)edge_bf16_ring_min_rows(); });
  m.def("gemv_bf16", &gemv_bf16, "bf16 decode GEMV (M <= 16), optional fused SwiGLU over [gate | up]", py::arg("x"),
        py::arg("wp"), py::arg("bias"), py::arg("N"), py::arg("epi"), py::arg("addend") = py::none());
  m.def("decode_attn_fused", &decode_attn_fused);
  m.def("decode_attn_i8", &decode_attn_i8, "decode attention over an int8 KV cache, fused RoPE + quantising append");
  m.def("kv_dequant", &kv_dequant, "dequantise the first T rows of an int8 KV cache into a bf16 scratch");
  m.def("kv_quant_append", &kv_quant_append, "quantise bf16 K/V rows into an int8 KV cache (prefill append)");
  m.def("w8a8_gemm_glu", &w8a8_gemm_glu);
  m.def("w8a8_gemm_splitk", &w8a8_gemm_splitk);
  m.def("w8a8_r256", &w8a8_r256, "129-256-row W8A8 GEMM on a fragment-packed activation (empty: shape not taken)");
  m.def("r256_ok", [](int64_t M, int64_t N, int64_t K) { return edge_w8a8_r256_ok((int)M, (int)N, (int)K, 0) != 0; },
        "whether the packed-activation 256-row kernel takes this shape");
  m.def("rms_norm_parts", &rms_norm_parts);
  m.def("w8a8_gemm_gluq", &w8a8_gemm_gluq);
  m.def("w8a8_gemv_norm", &w8a8_gemv_norm, "batch-1 W8A8 GEMV with the RMSNorm of split-K slices in its prologue");
  m.def("gemv_norm_on", []() { return edge_w8a8_gemv_norm_on() != 0; });
  m.def("w8a8_gemm_geluq", &w8a8_gemm_geluq, "W8A8 GEMV + GELU + per-(token, 64) int8 quantisation (M <= 64)");
  m.def("group_quant", &group_quant);
  m.def("w8a8_prefill_glu", &w8a8_prefill_glu, "prefill gate_up (16-blocked SwiGLU) with silu(g) * u in the epilogue: bf16 h or None");
  m.def("sample", &sample);
  m.def("sample_shard", &sample_shard, "sampler phase 1 over a vocab shard (global ids)");
  m.def("sample_merge", &sample_merge, "sampler phase 2 over the shards' concatenated candidate lists");
  m.def("sample_shard_chunks", &sample_shard_chunks);
  m.def("sample_shard_mode", &sample_shard_mode);
  m.def("sample_advance", &sample_advance, "sampler + decode-step bookkeeping in the sampler's last launch");
  m.def("decode_advance", &decode_advance, "decode-step bookkeeping after the sampler (one launch)");
  m.def("sample_timestamps", &sample_timestamps);
  m.def("rows128_ok", [](int64_t K, int64_t S) { return edge_w8a8_rows128_ok((int)K, (int)S) != 0; },
        "whether the 65-128 row decode GEMV has a kernel for K (in S split-K slices)");
  m.def("rows256_ok", [](int64_t K) { return edge_w8a8_rows256_ok((int)K) != 0; },
        "whether the 129-256 row decode GEMMs (row-split ring2) take this K");
  m.def("tune", [](const std::string& what, int64_t a, int64_t b) {
    if (what == "gemv") edge_w8a8_gemv_config((int)a, (int)b);
    else if (what == "gemv_ntw") edge_w8a8_gemv_ntw((int)a);
    else if (what == "gemv_ring") edge_w8a8_gemv_ring((int)a);
    else if (what == "prefill_x32") edge_w8a8_prefill_x32((int)a);
    else if (what == "prefill_apack") edge_w8a8_prefill_apack((int)a);
    else if (what == "decode_attn") edge_decode_attn_config((int)a);
    else if (what == "decode_attn_occ") edge_decode_attn_occ((int)a);
    else if (what == "decode_attn_small") edge_decode_attn_small((int)a);
    else if (what == "decode_attn_gsplit") edge_decode_attn_gsplit((int)a);
    else if (what == "decode_attn_early") edge_decode_attn_early((int)a);
    else if (what == "decode_attn_unroll") edge_decode_attn_unroll((int)a);
    else if (what == "attn8_wave_max") edge_decode_attn_i8_wave_max((int)a);
    else if (what == "sample_rowwide") edge_sample_rowwide_min((int)a);
    else if (what == "sample_vec") edge_sample_vec((int)a);
    else if (what == "prefill_fa") edge_prefill_fa((int)a, b == 0 ? 1 : (int)b - 1);   // b: 0 default, 1 lockstep, 2 stagger
    else if (what == "prefill_fa_order") edge_prefill_fa_order((int)a);
    else if (what == "prefill_fa_sm") edge_prefill_fa_sm((int)a, (int)b);
    else if (what == "gemv_norm") edge_w8a8_gemv_norm_cfg((int)a);
    else if (what == "r256_packed") edge_w8a8_r256_cfg((int)a);
    else if (what == "r256_wreg") edge_w8a8_wreg_cfg((int)a);
    else TORCH_CHECK(false, "unknown tunable ", what);
  });
}
