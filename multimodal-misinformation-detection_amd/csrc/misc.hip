// Memory-bound kernels on the training path: sequence mean pooling, summed cross entropy,
// BERT embeddings (+LayerNorm), ViT patchify / token assembly, multi-tensor AdamW.
#include "common.h"
#include <algorithm>
#include <math.h>

namespace {
inline unsigned gridn(int64_t n, int per) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, 16384));
}

// ---------------------------------------------------------------------------------------------
// mean over the sequence dim: x [B][L][D] -> out [B][ldo]  (model.py:332 `S.mean(dim=1)`)
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void seq_mean_fwd_kernel(int64_t B, int64_t L, int64_t D, const T* __restrict__ x, T* __restrict__ out,
                                    int64_t ldo) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B * D; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / D, d = i % D;
    const T* p = x + b * L * D + d;
    float s = 0.f;
    for (int64_t l = 0; l < L; ++l) s += to_f32(p[l * D]);
    out[b * ldo + d] = from_f32<T>(s / (float)L);
  }
}
__device__ __forceinline__ void load8(const bf16* p, float (&v)[8]) {
  const uint4 w = *reinterpret_cast<const uint4*>(p);
  const uint32_t a[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(a[i] << 16); v[2 * i + 1] = __uint_as_float(a[i] & 0xffff0000u); }
}
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
// vector form (D % 8 == 0, 16-B aligned rows): block = 32 column chunks of 8 x 32 row groups;
// each thread sums every 32nd row of its chunk with 16-B loads (all independent, so a short batch
// with long sequences is not a serial chain of L dependent loads), then the 32 row-group partials
// are combined in LDS in a fixed order.
template <typename T>
__global__ void __launch_bounds__(1024) seq_mean_fwd_vec_kernel(int64_t L, int64_t D, const T* __restrict__ x,
                                                                T* __restrict__ out, int64_t ldo) {
  __shared__ float part[32][32 * 8 + 4];
  const int cc = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int64_t b = blockIdx.y, c8 = ((int64_t)blockIdx.x * 32 + cc) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c8 < D) {
    const T* p = x + b * L * D + c8;
    for (int64_t l = rg; l < L; l += 32) {
      float v[8];
      load8(p + l * D, v);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += v[u];
    }
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) part[rg][cc * 8 + u] = acc[u];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int col = threadIdx.x;  // 32 chunks x 8 columns
    const int64_t d = (int64_t)blockIdx.x * 256 + col;
    float t = 0.f;
    for (int r = 0; r < 32; ++r) t += part[r][col];
    if (d < D) out[b * ldo + d] = from_f32<T>(t / (float)L);
  }
}

template <typename T>
__global__ void seq_mean_bwd_kernel(int64_t B, int64_t L, int64_t D, const T* __restrict__ dout, int64_t ldo,
                                    T* __restrict__ dx) {
  const float inv = 1.0f / (float)L;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B * L * D; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = i % D, b = i / (L * D);
    dx[i] = from_f32<T>(to_f32(dout[b * ldo + d]) * inv);
  }
}

// ---------------------------------------------------------------------------------------------
// summed cross entropy over paths; one block, rows = n_paths * B
// ---------------------------------------------------------------------------------------------
struct XentPtrs {
  const float* logits[4];
  float* dlogits[4];
  int col[4];  // label column (= the reference's path index, train.py:165) of each present path
  int has_grad;
};

__global__ void xent_kernel(int n_paths, int64_t B, int64_t C, XentPtrs ptrs, const int64_t* __restrict__ labels,
                            int64_t label_ld, float* __restrict__ loss, int n_slots, const float* __restrict__ dscale) {
  __shared__ float red[4][256];
  const float sc = dscale ? *dscale : 1.0f;
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t rr = threadIdx.x; rr < (int64_t)n_paths * B; rr += blockDim.x) {
    const int path = (int)(rr / B);
    const int64_t b = rr % B;
    const float* z = ptrs.logits[path] + b * C;
    float mx = -INFINITY;
    for (int64_t c = 0; c < C; ++c) mx = fmaxf(mx, z[c]);
    float se = 0.f;
    for (int64_t c = 0; c < C; ++c) se += expf(z[c] - mx);
    const float lse = mx + logf(se);
    const int64_t y = labels[b * label_ld + ptrs.col[path]];
    part[path] += lse - z[y];
    if (ptrs.has_grad) {
      float* dz = ptrs.dlogits[path] + b * C;
      for (int64_t c = 0; c < C; ++c) dz[c] = (expf(z[c] - lse) - (c == y ? 1.f : 0.f)) * sc / (float)B;
    }
  }
  for (int p = 0; p < 4; ++p) red[p][threadIdx.x] = part[p];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int p = 0; p < 4; ++p) red[p][threadIdx.x] += red[p][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    for (int s = 1; s < n_slots; ++s) loss[s] = 0.f;
    float tot = 0.f;
    for (int p = 0; p < n_paths; ++p) {
      const float lp = red[p][0] / (float)B;
      loss[1 + ptrs.col[p]] = lp;
      tot += lp;
    }
    loss[0] = tot;
  }
}

// ---------------------------------------------------------------------------------------------
// BERT embeddings: sum = word[id] + pos[t] + type[tt]; y = dropout(LN(sum))   (wave per token)
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) embed_ln_fwd_kernel(int64_t B, int64_t L, int64_t D, const int64_t* __restrict__ ids,
                                                           const int64_t* __restrict__ pos_ids,
                                                           const int64_t* __restrict__ tts, const float* __restrict__ word,
                                                           const float* __restrict__ pos, const float* __restrict__ type,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           float eps, T* __restrict__ sum_out, T* __restrict__ y,
                                                           float* __restrict__ mean, float* __restrict__ rstd, float p,
                                                           uint32_t thr, const uint64_t* __restrict__ seedp, uint64_t salt) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B * L) return;
  const int64_t t = pos_ids ? pos_ids[row] : row % L;
  const int64_t id = ids[row];
  const int64_t tt = tts ? tts[row] : 0;
  constexpr int MAXV = 16;  // D <= 1024
  float v[MAXV];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int64_t d = lane + 64 * j;
    v[j] = 0.f;
    if (d < D) {
      float e = word[id * D + d] + pos[t * D + d];
      if (type) e += type[tt * D + d];
      if (sum_out) {
        e = to_f32(from_f32<T>(e));  // the stored sum is what the backward LayerNorm re-reads
        sum_out[row * D + d] = from_f32<T>(e);
      }
      v[j] = e;
      s += e;
    }
  }
  const float mu = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int64_t d = lane + 64 * j;
    if (d < D) q += (v[j] - mu) * (v[j] - mu);
  }
  const float rs = rsqrtf(wave_sum(q) / (float)D + eps);
  const uint64_t seed = p > 0.f ? *seedp : 0ull;
  const float keep = 1.0f / (1.0f - p);
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int64_t d = lane + 64 * j;
    if (d < D) {
      float o = (v[j] - mu) * rs * gamma[d] + beta[d];
      if (p > 0.f) {
        const uint32_t h = mmfd_hash(seed, salt, (uint64_t)(row * D + d));
        o = (h < thr) ? 0.f : o * keep;
      }
      y[row * D + d] = from_f32<T>(o);
    }
  }
  if (lane == 0 && mean) { mean[row] = mu; rstd[row] = rs; }
}

// MPNet/RoBERTa position ids: padding_idx + cumsum(id != padding_idx) on non-pad tokens, else
// padding_idx (HF create_position_ids_from_input_ids). One thread per sequence.
__global__ void position_ids_kernel(int64_t B, int64_t L, const int64_t* __restrict__ ids, int64_t padding_idx,
                                    int64_t* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int64_t c = 0;
  for (int64_t t = 0; t < L; ++t) {
    const bool tok = ids[b * L + t] != padding_idx;
    c += tok ? 1 : 0;
    out[b * L + t] = (tok ? c : 0) + padding_idx;
  }
}

// relative position bias out[h][q][k] = table[bucket[q][k]][h]
__global__ void rel_bias_kernel(int64_t H, int64_t Lq, int64_t Lk, const int32_t* __restrict__ bucket,
                                const float* __restrict__ table, float* __restrict__ out) {
  const int64_t n = H * Lq * Lk;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = i / (Lq * Lk), qk = i % (Lq * Lk);
    out[i] = table[(int64_t)bucket[qk] * H + h];
  }
}

// ---------------------------------------------------------------------------------------------
// ViT
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void patchify_kernel(int64_t B, int64_t C, int64_t Hh, int64_t Ww, int64_t P, const float* __restrict__ px,
                                T* __restrict__ out) {
  const int64_t nph = Hh / P, npw = Ww / P, np = nph * npw;
  const int64_t total = B * np * C * P;  // one thread per (row, c, kh): P consecutive kw
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t kh = i % P, c = (i / P) % C, rp = i / (P * C);
    const int64_t b = rp / np, pidx = rp % np, ph = pidx / npw, pw = pidx % npw;
    const float* src = px + ((b * C + c) * Hh + ph * P + kh) * Ww + pw * P;
    T* dst = out + rp * (C * P * P) + (c * P + kh) * P;
    for (int64_t kw = 0; kw < P; ++kw) dst[kw] = from_f32<T>(src[kw]);
  }
}
// vector form (P % 4 == 0, Ww % 4 == 0, 16-B aligned pixels): one thread per 4 consecutive
// source pixels of an image row (coalesced float4 loads), stored as 4 consecutive patch-row
// elements (8-B bf16 / 16-B fp32 stores)
template <typename T>
__global__ void patchify_vec_kernel(int64_t B, int64_t C, int64_t Hh, int64_t Ww, int64_t P,
                                    const float* __restrict__ px, T* __restrict__ out) {
  const int64_t nph = Hh / P, npw = Ww / P, np = nph * npw, w4n = Ww / 4;
  const int64_t total = B * C * nph * P * w4n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w4 = i % w4n, h = (i / w4n) % (nph * P), c = (i / (w4n * nph * P)) % C, b = i / (w4n * nph * P * C);
    const int64_t w = w4 * 4, ph = h / P, kh = h % P, pw = w / P, kw = w % P;
    const float4 v = *reinterpret_cast<const float4*>(px + ((b * C + c) * Hh + h) * Ww + w);
    T* dst = out + (b * np + ph * npw + pw) * (C * P * P) + (c * P + kh) * P + kw;
    if constexpr (sizeof(T) == 2) {
      const uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, from_f32<T>(v.x)) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, from_f32<T>(v.y)) << 16);
      const uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, from_f32<T>(v.z)) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, from_f32<T>(v.w)) << 16);
      *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
    } else {
      *reinterpret_cast<float4*>(dst) = v;
    }
  }
}
template <typename T>
__global__ void vit_tokens_fwd_kernel(int64_t B, int64_t NP, int64_t D, const T* __restrict__ patch,
                                      const float* __restrict__ cls, const float* __restrict__ pos, T* __restrict__ out) {
  const int64_t total = B * (NP + 1) * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = i % D, t = (i / D) % (NP + 1), b = i / ((NP + 1) * D);
    const float base = t == 0 ? cls[d] : to_f32(patch[(b * NP + t - 1) * D + d]);
    out[i] = from_f32<T>(base + pos[t * D + d]);
  }
}
template <typename T>
__global__ void vit_tokens_dpatch_kernel(int64_t B, int64_t NP, int64_t D, const T* __restrict__ dout, T* __restrict__ dpatch) {
  const int64_t total = B * NP * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = i % D, pr = i / D, b = pr / NP, t = pr % NP + 1;
    dpatch[i] = dout[(b * (NP + 1) + t) * D + d];
  }
}
template <typename T>
__global__ void vit_tokens_dpos_kernel(int64_t B, int64_t NP, int64_t D, const T* __restrict__ dout, float* __restrict__ dcls,
                                       float* __restrict__ dpos) {
  const int64_t n = (NP + 1) * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int64_t b = 0; b < B; ++b) s += to_f32(dout[b * n + i]);
    dpos[i] = s;
    if (i < D) dcls[i] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// AdamW (torch.optim.AdamW, decoupled weight decay), multi-tensor: grid.y = tensor index
// ---------------------------------------------------------------------------------------------
__global__ void step_inc_kernel(const mmfd_adamw_tensor* __restrict__ tab, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) tab[i].step[0] += 1.0f;
}

__global__ void adamw_kernel(const mmfd_adamw_tensor* __restrict__ tab, float lr, float b1, float b2, float eps, float wd) {
  const mmfd_adamw_tensor t = tab[blockIdx.y];
  const double step = (double)t.step[0];
  const float bc1 = (float)(1.0 - pow((double)b1, step));
  const float bc2s = (float)sqrt(1.0 - pow((double)b2, step));
  const float step_size = lr / bc1;
  const float decay = 1.0f - lr * wd;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.numel; i += (int64_t)gridDim.x * blockDim.x) {
    const float g = t.grad[i];
    float p = t.param[i] * decay;
    float m = t.exp_avg[i];
    m = m + (1.0f - b1) * (g - m);
    float v = t.exp_avg_sq[i] * b2 + (1.0f - b2) * g * g;
    const float denom = sqrtf(v) / bc2s + eps;
    p = p - step_size * (m / denom);
    t.param[i] = p;
    t.exp_avg[i] = m;
    t.exp_avg_sq[i] = v;
    if (t.param_bf16) reinterpret_cast<bf16*>(t.param_bf16)[i] = (bf16)p;
  }
}

__global__ void mask_bias_kernel(int64_t n, const int64_t* __restrict__ mask, float* __restrict__ out, float neg) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = mask[i] ? 0.f : neg;
}
}  // namespace

extern "C" int mmfd_seq_mean_fwd(int dtype, int64_t B, int64_t L, int64_t D, const void* x, void* out, int64_t ldo,
                                 mmfd_stream_t stream) {
  MMFD_CHECK_ARG(L > 0, "seq_mean: L must be > 0");
  hipStream_t s = (hipStream_t)stream;
  const int esz = dtype == MMFD_BF16 ? 2 : 4;
  if (D % 8 == 0 && ((uintptr_t)x % 16) == 0 && (D * esz) % 16 == 0) {
    const dim3 grid((unsigned)((D + 255) / 256), (unsigned)B);
    if (dtype == MMFD_BF16)
      hipLaunchKernelGGL((seq_mean_fwd_vec_kernel<bf16>), grid, dim3(1024), 0, s, L, D, (const bf16*)x, (bf16*)out, ldo);
    else
      hipLaunchKernelGGL((seq_mean_fwd_vec_kernel<float>), grid, dim3(1024), 0, s, L, D, (const float*)x, (float*)out, ldo);
    MMFD_CHECK_LAUNCH("seq_mean_fwd");
    return 0;
  }
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((seq_mean_fwd_kernel<bf16>), dim3(gridn(B * D, 256)), dim3(256), 0, s, B, L, D, (const bf16*)x, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL((seq_mean_fwd_kernel<float>), dim3(gridn(B * D, 256)), dim3(256), 0, s, B, L, D, (const float*)x, (float*)out, ldo);
  MMFD_CHECK_LAUNCH("seq_mean_fwd");
  return 0;
}

extern "C" int mmfd_seq_mean_bwd(int dtype, int64_t B, int64_t L, int64_t D, const void* dout, int64_t ldo, void* dx,
                                 mmfd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((seq_mean_bwd_kernel<bf16>), dim3(gridn(B * L * D, 256)), dim3(256), 0, s, B, L, D, (const bf16*)dout, ldo, (bf16*)dx);
  else
    hipLaunchKernelGGL((seq_mean_bwd_kernel<float>), dim3(gridn(B * L * D, 256)), dim3(256), 0, s, B, L, D, (const float*)dout, ldo, (float*)dx);
  MMFD_CHECK_LAUNCH("seq_mean_bwd");
  return 0;
}

extern "C" int mmfd_xent_fwd_bwd(int n_paths, int64_t B, int64_t C, const float* const* logits, const int* path_cols,
                                 const int64_t* labels, int64_t label_ld, float* loss, int n_slots,
                                 float* const* dlogits, const float* dloss_scale, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(n_paths >= 1 && n_paths <= 4, "xent: 1..4 paths");
  MMFD_CHECK_ARG(B > 0 && C > 0 && logits, "xent: bad shape");
  XentPtrs ptrs = {};
  for (int i = 0; i < n_paths; ++i) {
    ptrs.logits[i] = logits[i];
    ptrs.dlogits[i] = dlogits ? dlogits[i] : nullptr;
    ptrs.col[i] = path_cols ? path_cols[i] : i;
    MMFD_CHECK_ARG(ptrs.col[i] >= 0 && ptrs.col[i] < label_ld && 1 + ptrs.col[i] < n_slots,
                   "xent: label column outside labels / loss slots");
  }
  ptrs.has_grad = dlogits != nullptr;
  hipLaunchKernelGGL(xent_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n_paths, B, C, ptrs, labels, label_ld, loss,
                     n_slots, dloss_scale);
  MMFD_CHECK_LAUNCH("xent");
  return 0;
}

extern "C" int mmfd_embed_ln_fwd_ex(int dtype, int64_t B, int64_t L, int64_t D, const int64_t* input_ids,
                                    const int64_t* position_ids, const int64_t* token_type_ids, const float* word,
                                    const float* pos, const float* type, const float* gamma, const float* beta, float eps,
                                    void* sum_out, void* y, float* mean, float* rstd, float dropout_p,
                                    const uint64_t* seed, uint64_t salt, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(D <= 1024, "embed: D <= 1024");
  MMFD_CHECK_ARG(dropout_p <= 0.f || seed, "embed: dropout needs seed");
  MMFD_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "embed: mean and rstd go together");
  const int64_t rows = B * L;
  if (rows == 0) return 0;
  const float p = dropout_p > 0.f ? dropout_p : 0.f;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((embed_ln_fwd_kernel<bf16>), grid, dim3(256), 0, s, B, L, D, input_ids, position_ids, token_type_ids,
                       word, pos, type, gamma, beta, eps, (bf16*)sum_out, (bf16*)y, mean, rstd, p, mmfd_drop_threshold(p),
                       seed, salt);
  else
    hipLaunchKernelGGL((embed_ln_fwd_kernel<float>), grid, dim3(256), 0, s, B, L, D, input_ids, position_ids, token_type_ids,
                       word, pos, type, gamma, beta, eps, (float*)sum_out, (float*)y, mean, rstd, p, mmfd_drop_threshold(p),
                       seed, salt);
  MMFD_CHECK_LAUNCH("embed_ln_fwd");
  return 0;
}

extern "C" int mmfd_embed_ln_fwd(int dtype, int64_t B, int64_t L, int64_t D, const int64_t* input_ids,
                                 const int64_t* token_type_ids, const float* word, const float* pos, const float* type,
                                 const float* gamma, const float* beta, float eps, void* sum_out, void* y, float* mean,
                                 float* rstd, float dropout_p, const uint64_t* seed, uint64_t salt, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(sum_out && mean && rstd && type, "embed_ln_fwd: sum_out/mean/rstd/type required (see _ex)");
  return mmfd_embed_ln_fwd_ex(dtype, B, L, D, input_ids, nullptr, token_type_ids, word, pos, type, gamma, beta, eps,
                              sum_out, y, mean, rstd, dropout_p, seed, salt, stream);
}

extern "C" int mmfd_position_ids(int64_t B, int64_t L, const int64_t* input_ids, int64_t padding_idx, int64_t* out,
                                 mmfd_stream_t stream) {
  if (B * L == 0) return 0;
  hipLaunchKernelGGL(position_ids_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, B, L,
                     input_ids, padding_idx, out);
  MMFD_CHECK_LAUNCH("position_ids");
  return 0;
}

extern "C" int mmfd_rel_bias(int64_t H, int64_t Lq, int64_t Lk, const int32_t* bucket, const float* table, float* out,
                             mmfd_stream_t stream) {
  const int64_t n = H * Lq * Lk;
  if (n == 0) return 0;
  hipLaunchKernelGGL(rel_bias_kernel, dim3(gridn(n, 256)), dim3(256), 0, (hipStream_t)stream, H, Lq, Lk, bucket, table, out);
  MMFD_CHECK_LAUNCH("rel_bias");
  return 0;
}

extern "C" int mmfd_patchify(int dtype, int64_t B, int64_t C, int64_t Hh, int64_t Ww, int64_t P, const float* pixels,
                             void* out, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(P > 0 && Hh % P == 0 && Ww % P == 0, "patchify: image not divisible by patch");
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = B * (Hh / P) * (Ww / P) * C * P;
  if (total == 0) return 0;
  if (P % 4 == 0 && Ww % 4 == 0 && ((uintptr_t)pixels % 16) == 0 && ((uintptr_t)out % 16) == 0) {
    const int64_t vt = total * P / 4;
    if (dtype == MMFD_BF16)
      hipLaunchKernelGGL((patchify_vec_kernel<bf16>), dim3(gridn(vt, 256)), dim3(256), 0, s, B, C, Hh, Ww, P, pixels, (bf16*)out);
    else
      hipLaunchKernelGGL((patchify_vec_kernel<float>), dim3(gridn(vt, 256)), dim3(256), 0, s, B, C, Hh, Ww, P, pixels, (float*)out);
    MMFD_CHECK_LAUNCH("patchify");
    return 0;
  }
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((patchify_kernel<bf16>), dim3(gridn(total, 256)), dim3(256), 0, s, B, C, Hh, Ww, P, pixels, (bf16*)out);
  else
    hipLaunchKernelGGL((patchify_kernel<float>), dim3(gridn(total, 256)), dim3(256), 0, s, B, C, Hh, Ww, P, pixels, (float*)out);
  MMFD_CHECK_LAUNCH("patchify");
  return 0;
}

extern "C" int mmfd_vit_tokens_fwd(int dtype, int64_t B, int64_t NP, int64_t D, const void* patch, const float* cls,
                                   const float* pos, void* out, mmfd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = B * (NP + 1) * D;
  if (total == 0) return 0;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((vit_tokens_fwd_kernel<bf16>), dim3(gridn(total, 256)), dim3(256), 0, s, B, NP, D, (const bf16*)patch, cls, pos, (bf16*)out);
  else
    hipLaunchKernelGGL((vit_tokens_fwd_kernel<float>), dim3(gridn(total, 256)), dim3(256), 0, s, B, NP, D, (const float*)patch, cls, pos, (float*)out);
  MMFD_CHECK_LAUNCH("vit_tokens_fwd");
  return 0;
}

extern "C" int mmfd_vit_tokens_bwd(int dtype, int64_t B, int64_t NP, int64_t D, const void* dout, void* dpatch, float* dcls,
                                   float* dpos, void* workspace, int64_t workspace_bytes, mmfd_stream_t stream) {
  (void)workspace; (void)workspace_bytes;
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = B * NP * D;
  if (dtype == MMFD_BF16) {
    if (dpatch) hipLaunchKernelGGL((vit_tokens_dpatch_kernel<bf16>), dim3(gridn(total, 256)), dim3(256), 0, s, B, NP, D, (const bf16*)dout, (bf16*)dpatch);
    hipLaunchKernelGGL((vit_tokens_dpos_kernel<bf16>), dim3(gridn((NP + 1) * D, 256)), dim3(256), 0, s, B, NP, D, (const bf16*)dout, dcls, dpos);
  } else {
    if (dpatch) hipLaunchKernelGGL((vit_tokens_dpatch_kernel<float>), dim3(gridn(total, 256)), dim3(256), 0, s, B, NP, D, (const float*)dout, (float*)dpatch);
    hipLaunchKernelGGL((vit_tokens_dpos_kernel<float>), dim3(gridn((NP + 1) * D, 256)), dim3(256), 0, s, B, NP, D, (const float*)dout, dcls, dpos);
  }
  MMFD_CHECK_LAUNCH("vit_tokens_bwd");
  return 0;
}

extern "C" int mmfd_adamw(int n_tensors, const mmfd_adamw_tensor* table, int64_t max_numel, float lr, float beta1,
                          float beta2, float eps, float weight_decay, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(n_tensors >= 0 && table, "adamw: bad args");
  if (n_tensors == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(step_inc_kernel, dim3((unsigned)((n_tensors + 255) / 256)), dim3(256), 0, s, table, n_tensors);
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((max_numel + 1023) / 1024, 1024));
  hipLaunchKernelGGL(adamw_kernel, dim3(gx, (unsigned)n_tensors), dim3(256), 0, s, table, lr, beta1, beta2, eps, weight_decay);
  MMFD_CHECK_LAUNCH("adamw");
  return 0;
}

extern "C" int mmfd_mask_to_bias(int64_t n, const int64_t* mask, float* out, float neg, mmfd_stream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(mask_bias_kernel, dim3(gridn(n, 256)), dim3(256), 0, (hipStream_t)stream, n, mask, out, neg);
  MMFD_CHECK_LAUNCH("mask_to_bias");
  return 0;
}

// ---------------------------------------------------------------------------------------------
// DeBERTa-v3 helpers (transformers modeling_deberta_v2.py; the reference's default text encoder)
// ---------------------------------------------------------------------------------------------
namespace {
// tile of 32 query rows x 64 keys of one (b, h). The p2c gather reads, for a fixed key j, the
// scores p2c[j][idx(i, j)] of 32 consecutive rows i: idx is monotone in i, so those are one short
// contiguous run (lanes over i, coalesced) and go through an LDS transpose; the c2p gather
// (row i, lanes over j) and the fp32 output row are coalesced directly.
constexpr int RB_TI = 32, RB_TJ = 64;
template <typename T>
__global__ void __launch_bounds__(256) deberta_rel_bias_kernel(int64_t B, int64_t H, int64_t L, const T* __restrict__ c2p,
                                                               const T* __restrict__ p2c, int64_t ld,
                                                               const int32_t* __restrict__ c2p_idx,
                                                               const int32_t* __restrict__ p2c_idx, float inv_scale,
                                                               float* __restrict__ out) {
  __shared__ float tp[RB_TI][RB_TJ + 1];
  const int64_t j0 = (int64_t)blockIdx.x * RB_TJ, i0 = (int64_t)blockIdx.y * RB_TI;
  const int64_t bh = blockIdx.z, b = bh / H, h = bh % H;
  const int64_t hb = h * B * L + b * L;
  const int t = threadIdx.x;
  {
    const int il = t % RB_TI;
    const int64_t i = i0 + il;
    for (int jl = t / RB_TI; jl < RB_TJ; jl += 256 / RB_TI) {
      const int64_t j = j0 + jl;
      float v = 0.f;
      if (i < L && j < L) v = to_f32(p2c[(hb + j) * ld + p2c_idx[j * L + i]]);
      tp[il][jl] = v;
    }
  }
  __syncthreads();
  const int jl = t % RB_TJ;
  const int64_t j = j0 + jl;
  if (j >= L) return;
  for (int il = t / RB_TJ; il < RB_TI; il += 256 / RB_TJ) {
    const int64_t i = i0 + il;
    if (i >= L) break;
    const float c = to_f32(c2p[(hb + i) * ld + c2p_idx[i * L + j]]);
    out[(bh * L + i) * L + j] = c * inv_scale + tp[il][jl] * inv_scale;  // score += c2p / s; += p2c / s (:329, :345)
  }
}

template <typename T>
__global__ void mask_rows_kernel(int64_t rows, int64_t D, T* __restrict__ x, int64_t ldx,
                                 const int64_t* __restrict__ mask) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < rows * D; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / D, d = e % D;
    if (mask[r] == 0) x[r * ldx + d] = from_f32<T>(0.f);
  }
}

// one block per (b, h): blocks of a batch row without padding return at once; otherwise Dh threads
// (x up to 4 row groups) average v over all L keys in fp32 and write the masked query rows
template <typename T>
__global__ void __launch_bounds__(256) attn_fill_masked_rows_kernel(int64_t H, int64_t L, int64_t Dh,
                                                                    const T* __restrict__ v, int64_t v_sb, int64_t v_st,
                                                                    T* __restrict__ o, int64_t o_sb, int64_t o_st,
                                                                    const int64_t* __restrict__ mask) {
  const int64_t b = blockIdx.x / H, h = blockIdx.x % H;
  __shared__ int any;
  __shared__ float part[4][64];
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < L; i += blockDim.x)
    if (mask[b * L + i] == 0) any = 1;
  __syncthreads();
  if (!any) return;
  const int d = threadIdx.x & 63, rg = threadIdx.x >> 6;
  float s = 0.f;
  if (d < Dh)
    for (int64_t t = rg; t < L; t += 4) s += to_f32(v[b * v_sb + t * v_st + h * Dh + d]);
  part[rg][d] = s;
  __syncthreads();
  if (d < Dh) {  // every row group writes a quarter of the masked rows
    const T mean = from_f32<T>((part[0][d] + part[1][d] + part[2][d] + part[3][d]) / (float)L);
    for (int64_t i = rg; i < L; i += 4)
      if (mask[b * L + i] == 0) o[b * o_sb + i * o_st + h * Dh + d] = mean;
  }
}
}  // namespace

extern "C" int mmfd_deberta_rel_bias(int dtype, int64_t B, int64_t H, int64_t L, const void* c2p, const void* p2c,
                                     int64_t ld, const int32_t* c2p_idx, const int32_t* p2c_idx, float inv_scale,
                                     float* out, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(B >= 0 && H > 0 && L >= 0 && ld > 0, "deberta_rel_bias: bad shape");
  MMFD_CHECK_ARG(dtype == MMFD_F32 || dtype == MMFD_BF16, "deberta_rel_bias: bad dtype");
  const int64_t total = B * H * L * L;
  if (total == 0) return 0;
  MMFD_CHECK_ARG(c2p && p2c && c2p_idx && p2c_idx && out, "deberta_rel_bias: null pointer");
  hipStream_t s = (hipStream_t)stream;
  MMFD_CHECK_ARG(B * H < 65536 && L < (1 << 20), "deberta_rel_bias: grid too large");
  const dim3 grid((unsigned)((L + RB_TJ - 1) / RB_TJ), (unsigned)((L + RB_TI - 1) / RB_TI), (unsigned)(B * H));
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((deberta_rel_bias_kernel<bf16>), grid, dim3(256), 0, s, B, H, L,
                       (const bf16*)c2p, (const bf16*)p2c, ld, c2p_idx, p2c_idx, inv_scale, out);
  else
    hipLaunchKernelGGL((deberta_rel_bias_kernel<float>), grid, dim3(256), 0, s, B, H, L,
                       (const float*)c2p, (const float*)p2c, ld, c2p_idx, p2c_idx, inv_scale, out);
  MMFD_CHECK_LAUNCH("deberta_rel_bias");
  return 0;
}

extern "C" int mmfd_mask_rows(int dtype, int64_t rows, int64_t D, void* x, int64_t ldx, const int64_t* mask,
                              mmfd_stream_t stream) {
  MMFD_CHECK_ARG(rows >= 0 && D >= 0 && ldx >= D, "mask_rows: bad shape");
  if (rows * D == 0) return 0;
  MMFD_CHECK_ARG(x && mask, "mask_rows: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((mask_rows_kernel<bf16>), dim3(gridn(rows * D, 256)), dim3(256), 0, s, rows, D, (bf16*)x, ldx, mask);
  else
    hipLaunchKernelGGL((mask_rows_kernel<float>), dim3(gridn(rows * D, 256)), dim3(256), 0, s, rows, D, (float*)x, ldx, mask);
  MMFD_CHECK_LAUNCH("mask_rows");
  return 0;
}

extern "C" int mmfd_attn_fill_masked_rows(int dtype, int64_t B, int64_t H, int64_t L, int64_t Dh, const void* v,
                                          int64_t v_sb, int64_t v_st, void* o, int64_t o_sb, int64_t o_st,
                                          const int64_t* mask, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(B >= 0 && H > 0 && L >= 0 && Dh > 0 && Dh <= 64, "attn_fill_masked_rows: bad shape (Dh <= 64)");
  if (B * L == 0) return 0;
  MMFD_CHECK_ARG(v && o && mask, "attn_fill_masked_rows: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((attn_fill_masked_rows_kernel<bf16>), dim3((unsigned)(B * H)), dim3(256), 0, s, H, L, Dh,
                       (const bf16*)v, v_sb, v_st, (bf16*)o, o_sb, o_st, mask);
  else
    hipLaunchKernelGGL((attn_fill_masked_rows_kernel<float>), dim3((unsigned)(B * H)), dim3(256), 0, s, H, L, Dh,
                       (const float*)v, v_sb, v_st, (float*)o, o_sb, o_st, mask);
  MMFD_CHECK_LAUNCH("attn_fill_masked_rows");
  return 0;
}
