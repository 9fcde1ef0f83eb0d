// PyTorch custom-op layer over the C ABI (include/mmfd.h): registers the hot-path entry points as
// torch.ops.mmfd.* (schemas with declared mutations; CUDA(=HIP) dispatch key; fake kernels are
// registered from Python, mmfd/ops.py). Every op only unpacks tensors into the C-ABI argument
// structs and calls libmmfd_hip.so on torch's current HIP stream; PyTorch owns every buffer (the
// out-variant ops write into caller-allocated tensors, as the C ABI requires), the only
// allocation here is the split-K / reduction workspace, taken from torch's caching allocator.
//
// Host code only (no device code): built with hipcc against the torch headers, linked to
// libmmfd_hip.so (csrc/Makefile, target ../libmmfd_torch.so).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../../include/mmfd.h"

namespace {

mmfd_stream_t stream_of(const at::Tensor& t) {
  return (mmfd_stream_t)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return MMFD_F32;
    case at::kBFloat16: return MMFD_BF16;
    case at::kHalf: return MMFD_F16;
    default: TORCH_CHECK(false, "mmfd: unsupported dtype ", t.scalar_type());
  }
}

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed (code ", rc, "): ", mmfd_last_error_string());
}

int64_t ld2(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, "mmfd: ", name, " must be a 2-D row-major view, got ",
              t.sizes(), " strides ", t.strides());
  return t.stride(0);
}

template <typename T>
T* ptr_or_null(const std::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

const uint64_t* seed_ptr(const std::optional<at::Tensor>& seed) {
  return ptr_or_null<const uint64_t>(seed);
}

// ---- GEMM (mmfd_gemm): out = epilogue(alpha * op(A) op(B)) (+ beta * out) ------------------------
void gemm(const at::Tensor& A, const at::Tensor& B, bool trans_a, bool trans_b, at::Tensor& out, double alpha,
          double beta, const std::optional<at::Tensor>& bias, const std::optional<at::Tensor>& residual,
          bool residual_first, int64_t act, const std::optional<at::Tensor>& aux, double dropout_p,
          const std::optional<at::Tensor>& seed, int64_t salt, int64_t splits, const std::optional<at::Tensor>& a_rowsum,
          double a_rowsum_beta, const std::optional<at::Tensor>& a_planes = std::nullopt,
          const std::optional<at::Tensor>& b_planes = std::nullopt,
          const std::optional<at::Tensor>& out_planes = std::nullopt, bool write_out = true,
          bool a_planes_only = false, bool b_planes_only = false) {
  TORCH_CHECK(A.scalar_type() == B.scalar_type(), "mmfd::gemm operands must share a dtype");
  mmfd_gemm_args a{};
  a.struct_size = sizeof(mmfd_gemm_args);
  a.dtype = dtype_code(A);
  a.trans_a = trans_a;
  a.trans_b = trans_b;
  a.M = trans_a ? A.size(1) : A.size(0);
  a.K = trans_a ? A.size(0) : A.size(1);
  a.N = trans_b ? B.size(1) : B.size(0);
  TORCH_CHECK((trans_b ? B.size(0) : B.size(1)) == a.K, "mmfd::gemm inner dims differ");
  TORCH_CHECK(out.size(0) == a.M && out.size(1) == a.N, "mmfd::gemm out shape ", out.sizes());
  a.A = A.data_ptr(); a.lda = ld2(A, "A");
  a.B = B.data_ptr(); a.ldb = ld2(B, "B");
  a.C = out.data_ptr(); a.ldc = ld2(out, "out"); a.c_dtype = dtype_code(out);
  a.alpha = (float)alpha; a.beta = (float)beta;
  a.ep.bias = ptr_or_null<const float>(bias);
  if (residual.has_value() && residual->defined()) {
    a.ep.residual = residual->data_ptr(); a.ep.ldr = ld2(*residual, "residual");
    a.ep.residual_first = residual_first ? 1 : 0;
  }
  if (aux.has_value() && aux->defined()) { a.ep.aux = aux->data_ptr(); a.ep.ldaux = ld2(*aux, "aux"); }
  a.ep.act = (int)act;
  a.ep.dropout_p = (float)dropout_p;
  a.ep.seed = seed_ptr(seed);
  a.ep.salt = (uint64_t)salt;
  a.splits = (int)splits;
  a.a_rowsum = ptr_or_null<float>(a_rowsum);
  a.a_rowsum_beta = (float)a_rowsum_beta;
  auto planes = [&](const std::optional<at::Tensor>& p, const at::Tensor& src, const char* name) -> const void* {
    if (!p.has_value() || !p->defined()) return nullptr;
    TORCH_CHECK(p->scalar_type() == at::kBFloat16 && p->is_contiguous() && p->dim() == 3 && p->size(0) == 3 &&
                    p->size(1) == src.size(0) && p->size(2) == src.size(1),
                "mmfd::gemm: ", name, " must be contiguous bf16 [3, ", src.size(0), ", ", src.size(1), "]");
    return p->data_ptr();
  };
  a.a_planes = planes(a_planes, A, "a_planes");
  a.b_planes = planes(b_planes, B, "b_planes");
  a.a_planes_only = (a_planes_only && a.a_planes) ? 1 : 0;
  a.b_planes_only = (b_planes_only && a.b_planes) ? 1 : 0;
  if (out_planes.has_value() && out_planes->defined()) {
    TORCH_CHECK(out.scalar_type() == at::kFloat, "mmfd::gemm: out_planes need an fp32 output");
    a.ep.out_planes = const_cast<void*>(planes(out_planes, out, "out_planes"));
  }
  if (!write_out) {
    TORCH_CHECK(a.ep.out_planes != nullptr && beta == 0.0, "mmfd::gemm: write_out=False needs out_planes and beta = 0");
    a.C = nullptr; a.ldc = a.N;
  }
  const int64_t need = mmfd_gemm_workspace_bytes(&a);
  at::Tensor ws;
  if (need > 0) {
    ws = at::empty({need / 4 + 1}, A.options().dtype(at::kFloat));
    a.workspace = ws.data_ptr(); a.workspace_bytes = need;
  }
  check(mmfd_gemm(&a, stream_of(A)), "mmfd::gemm");
}

// fp32 [rows, cols] (row-major view) -> bf16 planes [3, rows, cols] (mmfd_split3)
void split3(const at::Tensor& x, at::Tensor& planes) {
  TORCH_CHECK(x.scalar_type() == at::kFloat, "mmfd::split3: x must be fp32");
  TORCH_CHECK(planes.scalar_type() == at::kBFloat16 && planes.is_contiguous() && planes.dim() == 3 &&
                  planes.size(0) == 3 && planes.size(1) == x.size(0) && planes.size(2) == x.size(1),
              "mmfd::split3: planes must be contiguous bf16 [3, rows, cols]");
  check(mmfd_split3(x.size(0), x.size(1), x.data_ptr<float>(), ld2(x, "x"), planes.data_ptr(), stream_of(x)),
        "mmfd::split3");
}

// functional nn.Linear forward (x [..., K] @ w[N, K]^T + b, optional fused GELU / ReLU / tanh /
// sigmoid): the op the standalone layers dispatch through
at::Tensor linear(const at::Tensor& x, const at::Tensor& w, const std::optional<at::Tensor>& bias, int64_t act) {
  auto x2 = x.reshape({-1, x.size(-1)});
  if (x2.stride(1) != 1) x2 = x2.contiguous();
  auto sizes = x.sizes().vec();
  sizes.back() = w.size(0);
  at::Tensor out = at::empty({x2.size(0), w.size(0)}, x.options());
  gemm(x2, w, false, false, out, 1.0, 0.0, bias, std::nullopt, false, act, std::nullopt, 0.0, std::nullopt, 0, 0,
       std::nullopt, 0.0);
  return out.view(sizes);
}

// ---- attention ------------------------------------------------------------------------------------
void head_view(const at::Tensor& t, const char* name, const void** p, int64_t* sb, int64_t* st) {
  TORCH_CHECK(t.dim() == 3 && t.stride(2) == 1, "mmfd: ", name, " must be a [B, L, H*D] view with a contiguous last dim");
  *p = t.data_ptr(); *sb = t.stride(0); *st = t.stride(1);
}

mmfd_attn_args attn_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t heads, double scale,
                         const std::optional<at::Tensor>& key_bias, const std::optional<at::Tensor>& rel_bias,
                         int64_t rel_bias_sb, int64_t rel_bias_mod, double dropout_p,
                         const std::optional<at::Tensor>& seed, int64_t salt) {
  mmfd_attn_args a{};
  a.struct_size = sizeof(mmfd_attn_args);
  a.dtype = dtype_code(q);
  a.B = q.size(0); a.H = heads; a.Lq = q.size(1); a.Lk = k.size(1); a.D = q.size(2) / heads;
  a.scale = (float)scale;
  const void* p;
  head_view(q, "q", &p, &a.q_sb, &a.q_st); a.q = p;
  head_view(k, "k", &p, &a.k_sb, &a.k_st); a.k = p;
  head_view(v, "v", &p, &a.v_sb, &a.v_st); a.v = p;
  a.key_bias = ptr_or_null<const float>(key_bias);
  a.rel_bias = ptr_or_null<const float>(rel_bias);
  a.rel_bias_sb = rel_bias_sb; a.rel_bias_mod = rel_bias_mod;
  a.dropout_p = (float)dropout_p; a.seed = seed_ptr(seed); a.salt = (uint64_t)salt;
  return a;
}

// the dropout keep-bitmask buffer: int32 (uint32 words) [B*H*Lq*ceil(Lk/32)], contiguous, on the device
uint32_t* drop_mask_ptr(const std::optional<at::Tensor>& m, const mmfd_attn_args& a) {
  if (!m.has_value() || !m->defined()) return nullptr;
  TORCH_CHECK(m->scalar_type() == at::kInt && m->is_contiguous() && m->is_cuda() &&
                  m->numel() == a.B * a.H * a.Lq * ((a.Lk + 31) / 32),
              "mmfd attention: drop_mask must be a contiguous int32 device tensor of B*H*Lq*ceil(Lk/32) words");
  return reinterpret_cast<uint32_t*>(m->data_ptr());
}

void attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& out, at::Tensor& lse,
              int64_t heads, double scale, const std::optional<at::Tensor>& key_bias,
              const std::optional<at::Tensor>& rel_bias, int64_t rel_bias_sb, int64_t rel_bias_mod, double dropout_p,
              const std::optional<at::Tensor>& seed, int64_t salt, const std::optional<at::Tensor>& cos_logit_scale,
              double cos_max_log, const std::optional<at::Tensor>& o_planes = std::nullopt,
              const std::optional<at::Tensor>& drop_mask = std::nullopt) {
  mmfd_attn_args a = attn_args(q, k, v, heads, scale, key_bias, rel_bias, rel_bias_sb, rel_bias_mod, dropout_p, seed, salt);
  const void* p;
  head_view(out, "out", &p, &a.o_sb, &a.o_st); a.o = const_cast<void*>(p);
  a.lse = lse.data_ptr<float>();
  a.cos_logit_scale = ptr_or_null<const float>(cos_logit_scale);
  a.cos_max_log = (float)cos_max_log;
  if (o_planes.has_value() && o_planes->defined()) {
    TORCH_CHECK(o_planes->scalar_type() == at::kBFloat16 && o_planes->is_contiguous() && o_planes->numel() == 3 * out.numel(),
                "mmfd::attn_fwd: o_planes must be contiguous bf16 [3, B*L, H*D]");
    a.o_planes = o_planes->data_ptr();
  }
  a.drop_mask = drop_mask_ptr(drop_mask, a);
  check(mmfd_attn_fwd(&a, stream_of(q)), "mmfd::attn_fwd");
}

void attn_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
              const at::Tensor& dout, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv, int64_t heads, double scale,
              const std::optional<at::Tensor>& key_bias, const std::optional<at::Tensor>& rel_bias, int64_t rel_bias_sb,
              int64_t rel_bias_mod, double dropout_p, const std::optional<at::Tensor>& seed, int64_t salt,
              bool accumulate_dq, bool accumulate_dkv, const std::optional<at::Tensor>& dqkv_planes = std::nullopt,
              bool planes_only = false, const std::optional<at::Tensor>& drop_mask = std::nullopt) {
  mmfd_attn_args a = attn_args(q, k, v, heads, scale, key_bias, rel_bias, rel_bias_sb, rel_bias_mod, dropout_p, seed, salt);
  const void* p;
  head_view(o, "o", &p, &a.o_sb, &a.o_st); a.o = const_cast<void*>(p);
  a.lse = const_cast<float*>(lse.data_ptr<float>());
  head_view(dout, "dout", &p, &a.do_sb, &a.do_st); a.dout = p;
  head_view(dq, "dq", &p, &a.dq_sb, &a.dq_st); a.dq = const_cast<void*>(p);
  head_view(dk, "dk", &p, &a.dk_sb, &a.dk_st); a.dk = const_cast<void*>(p);
  head_view(dv, "dv", &p, &a.dv_sb, &a.dv_st); a.dv = const_cast<void*>(p);
  at::Tensor delta = at::empty({a.B, a.H, a.Lq}, q.options().dtype(at::kFloat));
  a.delta = delta.data_ptr<float>();
  a.accumulate_dq = accumulate_dq; a.accumulate_dkv = accumulate_dkv;
  if (dqkv_planes.has_value() && dqkv_planes->defined()) {
    TORCH_CHECK(dqkv_planes->scalar_type() == at::kBFloat16 && dqkv_planes->is_contiguous() &&
                    dqkv_planes->numel() == 3 * a.B * a.Lq * 3 * a.H * a.D,
                "mmfd::attn_bwd: dqkv_planes must be contiguous bf16 [3, B*L, 3*H*D]");
    a.dqkv_planes = dqkv_planes->data_ptr();
    a.planes_only = planes_only ? 1 : 0;
  }
  a.drop_mask = drop_mask_ptr(drop_mask, a);
  check(mmfd_attn_bwd(&a, stream_of(q)), "mmfd::attn_bwd");
}

// ---- LayerNorm ------------------------------------------------------------------------------------
void layernorm_fwd(const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& beta, double eps, at::Tensor& y,
                   at::Tensor& mean, at::Tensor& rstd, const std::optional<at::Tensor>& planes = std::nullopt) {
  if (planes.has_value() && planes->defined()) {
    TORCH_CHECK(x.scalar_type() == at::kFloat && planes->scalar_type() == at::kBFloat16 && planes->is_contiguous() &&
                    planes->numel() == 3 * x.size(0) * x.size(1),
                "mmfd::layernorm_fwd: planes must be contiguous bf16 [3, rows, width] of an fp32 LayerNorm");
    check(mmfd_layernorm_fwd_split(x.size(0), x.size(1), x.data_ptr<float>(), ld2(x, "x"), gamma.data_ptr<float>(),
                                   beta.data_ptr<float>(), (float)eps, y.data_ptr<float>(), ld2(y, "y"),
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(), planes->data_ptr(), stream_of(x)),
          "mmfd::layernorm_fwd");
    return;
  }
  check(mmfd_layernorm_fwd(dtype_code(x), x.size(0), x.size(1), x.data_ptr(), ld2(x, "x"), gamma.data_ptr<float>(),
                           beta.data_ptr<float>(), (float)eps, y.data_ptr(), ld2(y, "y"), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), stream_of(x)), "mmfd::layernorm_fwd");
}

void layernorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& mean,
                   const at::Tensor& rstd, at::Tensor& dx, const std::optional<at::Tensor>& dx_add,
                   const std::optional<at::Tensor>& dgamma, const std::optional<at::Tensor>& dbeta, double beta_acc,
                   const std::optional<at::Tensor>& dx_drop, double dropout_p, const std::optional<at::Tensor>& seed,
                   int64_t salt, const std::optional<at::Tensor>& planes = std::nullopt) {
  const int64_t R = dy.size(0), W = dy.size(1);
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((R + 3) / 4, 2048));
  at::Tensor ws = at::empty({nb * 2 * W}, dy.options().dtype(at::kFloat));
  const bool has_add = dx_add.has_value() && dx_add->defined();
  if (planes.has_value() && planes->defined()) {
    TORCH_CHECK(dy.scalar_type() == at::kFloat && planes->scalar_type() == at::kBFloat16 && planes->is_contiguous() &&
                    planes->numel() == 3 * R * W,
                "mmfd::layernorm_bwd: planes must be contiguous bf16 [3, rows, width] of an fp32 LayerNorm");
    check(mmfd_layernorm_bwd_split(R, W, dy.data_ptr<float>(), ld2(dy, "dy"), x.data_ptr<float>(), ld2(x, "x"),
                                   gamma.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                                   dx.data_ptr<float>(), ld2(dx, "dx"), has_add ? dx_add->data_ptr<float>() : nullptr,
                                   has_add ? ld2(*dx_add, "dx_add") : 0, ptr_or_null<float>(dgamma),
                                   ptr_or_null<float>(dbeta), (float)beta_acc, ptr_or_null<float>(dx_drop),
                                   (float)dropout_p, seed_ptr(seed), (uint64_t)salt, ws.data_ptr(), ws.numel() * 4,
                                   planes->data_ptr(), stream_of(dy)),
          "mmfd::layernorm_bwd");
    return;
  }
  check(mmfd_layernorm_bwd(dtype_code(dy), R, W, dy.data_ptr(), ld2(dy, "dy"), x.data_ptr(), ld2(x, "x"),
                           gamma.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(),
                           ld2(dx, "dx"), has_add ? dx_add->data_ptr() : nullptr, has_add ? ld2(*dx_add, "dx_add") : 0,
                           ptr_or_null<float>(dgamma), ptr_or_null<float>(dbeta), (float)beta_acc,
                           ptr_or_null<void>(dx_drop), (float)dropout_p, seed_ptr(seed), (uint64_t)salt, ws.data_ptr(),
                           ws.numel() * 4, stream_of(dy)), "mmfd::layernorm_bwd");
}

// ---- summed per-path cross entropy ------------------------------------------------------------------
void xent(at::TensorList logits, at::IntArrayRef cols, const at::Tensor& labels, at::Tensor& loss,
          at::TensorList dlogits, const std::optional<at::Tensor>& dloss_scale) {
  const int n = (int)logits.size();
  TORCH_CHECK(n >= 1 && n <= 4 && (int64_t)cols.size() == n, "mmfd::xent: 1..4 paths, one label column each");
  TORCH_CHECK(dlogits.empty() || (int)dlogits.size() == n, "mmfd::xent: one dlogits tensor per path");
  std::vector<const float*> lp(n);
  std::vector<float*> dp(n);
  std::vector<int> cp(n);
  for (int i = 0; i < n; ++i) {
    TORCH_CHECK(logits[i].scalar_type() == at::kFloat && logits[i].is_contiguous(), "mmfd::xent: contiguous fp32 logits");
    lp[i] = logits[i].data_ptr<float>();
    cp[i] = (int)cols[i];
    if (!dlogits.empty()) dp[i] = dlogits[i].data_ptr<float>();
  }
  const int64_t ld = labels.dim() > 1 ? labels.stride(0) : 1;
  check(mmfd_xent_fwd_bwd(n, logits[0].size(0), logits[0].size(1), lp.data(), cp.data(), labels.data_ptr<int64_t>(),
                          ld, loss.data_ptr<float>(), (int)loss.numel(), dlogits.empty() ? nullptr : dp.data(),
                          ptr_or_null<const float>(dloss_scale), stream_of(loss)), "mmfd::xent");
}

// ---- AdamW over a device pointer table (mmfd_adamw_tensor[n], see mmfd.optim) ------------------------
void adamw(const at::Tensor& table, int64_t n, int64_t max_numel, double lr, double beta1, double beta2, double eps,
           double weight_decay) {
  check(mmfd_adamw((int)n, reinterpret_cast<const mmfd_adamw_tensor*>(table.data_ptr()), max_numel, (float)lr,
                   (float)beta1, (float)beta2, (float)eps, (float)weight_decay, stream_of(table)), "mmfd::adamw");
}

// ---- small elementwise / reduction ops --------------------------------------------------------------
void seq_mean_fwd(const at::Tensor& x, at::Tensor& out) {
  TORCH_CHECK(x.is_contiguous() && x.dim() == 3, "mmfd::seq_mean_fwd: contiguous [B, L, D]");
  check(mmfd_seq_mean_fwd(dtype_code(x), x.size(0), x.size(1), x.size(2), x.data_ptr(), out.data_ptr(),
                          ld2(out, "out"), stream_of(x)), "mmfd::seq_mean_fwd");
}

void seq_mean_bwd(const at::Tensor& dout, at::Tensor& dx) {
  check(mmfd_seq_mean_bwd(dtype_code(dout), dx.size(0), dx.size(1), dx.size(2), dout.data_ptr(), ld2(dout, "dout"),
                          dx.data_ptr(), stream_of(dout)), "mmfd::seq_mean_bwd");
}

void cast(const at::Tensor& x, at::Tensor& out) {
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() == out.numel(), "mmfd::cast: contiguous, same size");
  if (x.numel() == 0) return;
  check(mmfd_cast(dtype_code(x), dtype_code(out), x.numel(), x.data_ptr(), out.data_ptr(), stream_of(x)), "mmfd::cast");
}

void cosine_scores(const at::Tensor& queries, const at::Tensor& corpus, int64_t mode, double eps, at::Tensor& out) {
  check(mmfd_cosine_scores(dtype_code(corpus), queries.size(0), corpus.size(0), queries.size(1),
                           queries.data_ptr<float>(), ld2(queries, "queries"), corpus.data_ptr(), ld2(corpus, "corpus"),
                           (int)mode, (float)eps, out.data_ptr<float>(), ld2(out, "out"), stream_of(corpus)),
        "mmfd::cosine_scores");
}

void topk(const at::Tensor& scores, int64_t k, at::Tensor& values, at::Tensor& indices) {
  const int64_t Q = scores.size(0), N = scores.size(1);
  const int64_t nbytes = mmfd_topk_workspace_bytes(Q, N, k);
  at::Tensor ws = at::empty({std::max<int64_t>(nbytes, 8)}, scores.options().dtype(at::kByte));
  check(mmfd_topk(Q, N, scores.data_ptr<float>(), ld2(scores, "scores"), k, values.data_ptr<float>(),
                  indices.data_ptr<int64_t>(), ws.data_ptr(), nbytes, stream_of(scores)), "mmfd::topk");
}

}  // namespace

TORCH_LIBRARY(mmfd, m) {
  m.def("gemm(Tensor A, Tensor B, bool trans_a, bool trans_b, Tensor(a!) out, float alpha, float beta, Tensor? bias, "
        "Tensor? residual, bool residual_first, int act, Tensor(b!)? aux, float dropout_p, Tensor? seed, int salt, "
        "int splits, Tensor(c!)? a_rowsum, float a_rowsum_beta, Tensor? a_planes=None, Tensor? b_planes=None, "
        "Tensor(d!)? out_planes=None, bool write_out=True, bool a_planes_only=False, bool b_planes_only=False) -> ()");
  m.def("split3(Tensor x, Tensor(a!) planes) -> ()");
  m.def("linear(Tensor x, Tensor w, Tensor? bias, int act=0) -> Tensor");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, Tensor(a!) out, Tensor(b!) lse, int heads, float scale, "
        "Tensor? key_bias, Tensor? rel_bias, int rel_bias_sb, int rel_bias_mod, float dropout_p, Tensor? seed, int salt, "
        "Tensor? cos_logit_scale, float cos_max_log, Tensor(c!)? o_planes=None, Tensor(d!)? drop_mask=None) -> ()");
  m.def("attn_bwd(Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor dout, Tensor(a!) dq, Tensor(b!) dk, "
        "Tensor(c!) dv, int heads, float scale, Tensor? key_bias, Tensor? rel_bias, int rel_bias_sb, int rel_bias_mod, "
        "float dropout_p, Tensor? seed, int salt, bool accumulate_dq, bool accumulate_dkv, "
        "Tensor(d!)? dqkv_planes=None, bool planes_only=False, Tensor? drop_mask=None)-> ()");
  m.def("layernorm_fwd(Tensor x, Tensor gamma, Tensor beta, float eps, Tensor(a!) y, Tensor(b!) mean, "
        "Tensor(c!) rstd, Tensor(d!)? planes=None) -> ()");
  m.def("layernorm_bwd(Tensor dy, Tensor x, Tensor gamma, Tensor mean, Tensor rstd, Tensor(a!) dx, Tensor? dx_add, "
        "Tensor(b!)? dgamma, Tensor(c!)? dbeta, float beta_acc, Tensor(d!)? dx_drop, float dropout_p, Tensor? seed, "
        "int salt, Tensor(e!)? planes=None) -> ()");
  m.def("xent(Tensor[] logits, int[] cols, Tensor labels, Tensor(a!) loss, Tensor(b!)[] dlogits, "
        "Tensor? dloss_scale) -> ()");
  m.def("adamw(Tensor table, int n, int max_numel, float lr, float beta1, float beta2, float eps, "
        "float weight_decay) -> ()");
  m.def("seq_mean_fwd(Tensor x, Tensor(a!) out) -> ()");
  m.def("seq_mean_bwd(Tensor dout, Tensor(a!) dx) -> ()");
  m.def("cast(Tensor x, Tensor(a!) out) -> ()");
  m.def("cosine_scores(Tensor queries, Tensor corpus, int mode, float eps, Tensor(a!) out) -> ()");
  m.def("topk(Tensor scores, int k, Tensor(a!) values, Tensor(b!) indices) -> ()");
}

TORCH_LIBRARY_IMPL(mmfd, CUDA, m) {
  m.impl("gemm", &gemm);
  m.impl("split3", &split3);
  m.impl("linear", &linear);
  m.impl("attn_fwd", &attn_fwd);
  m.impl("attn_bwd", &attn_bwd);
  m.impl("layernorm_fwd", &layernorm_fwd);
  m.impl("layernorm_bwd", &layernorm_bwd);
  m.impl("xent", &xent);
  m.impl("adamw", &adamw);
  m.impl("seq_mean_fwd", &seq_mean_fwd);
  m.impl("seq_mean_bwd", &seq_mean_bwd);
  m.impl("cast", &cast);
  m.impl("cosine_scores", &cosine_scores);
  m.impl("topk", &topk);
}
