// Swinv2 image encoder pieces (the reference's default image encoder,
// Swinv2Model.from_pretrained("microsoft/swinv2-base-patch4-window8-256"), train.py:332, called at
// train.py:142-143 and preprocess_embeddings.py:91-92; arithmetic of transformers modeling_swinv2.py,
// restated in oracle/swinv2.py).
//
// The encoder's GEMMs, LayerNorms and windowed attention run on the shared kernels (gemm.hip,
// layernorm.hip, attention.hip with a per-window-position rel_bias). What is Swin-specific is
// data movement and three tiny bias/normalisation passes:
//   row_gather   : one HBM pass that moves token rows between the natural raster order, the
//                  (shifted) window order of the next block, and the 2x2 patch-merging concat
//                  (G source rows per output row). Index tables come from the host, one image's
//                  worth, so every permutation of a stage (roll + window_partition, its inverse,
//                  and their composition) is one launch.
//   swin_cpb     : continuous position-bias MLP  relu(coords W1^T + b1) W2^T  -> [T][H]
//   swin_bias    : 16 * sigmoid(table[rpi[i][j]][h]) (+ 2 * shift mask[w][i][j])  -> [nW][H][L][L]
//                  (HF adds the window mask twice, modeling_swinv2.py Swinv2SelfAttention.forward)
//   swin_qk_norm : cosine attention: q_h <- q_h / max(|q_h|, 1e-12) * exp(min(logit_scale_h, ln 100)),
//                  k_h <- k_h / max(|k_h|, 1e-12), in place on the packed QKV rows
#include "common.h"

namespace {

// one thread per 16-byte chunk of an output row; consecutive threads -> consecutive chunks
__global__ void __launch_bounds__(256) row_gather_kernel(int64_t B, int64_t rows_out, int64_t G, int64_t chunks,
                                                         int64_t src_rows, const uint4* __restrict__ src,
                                                         const int32_t* __restrict__ idx, uint4* __restrict__ dst) {
  const int64_t per_img = rows_out * G * chunks;
  const int64_t total = B * per_img;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / per_img;
    const int64_t rem = t - b * per_img;
    const int64_t rg = rem / chunks;       // (output row, group) pair
    const int64_t c = rem - rg * chunks;
    const int64_t sr = idx[rg];
    dst[t] = src[(b * src_rows + sr) * chunks + c];
  }
}

// one block per table entry; 512 hidden units = 512 threads (8 waves)
__global__ void __launch_bounds__(512) swin_cpb_kernel(int H, const float* __restrict__ coords,
                                                       const float* __restrict__ w1, const float* __restrict__ b1,
                                                       const float* __restrict__ w2, float* __restrict__ out) {
  __shared__ float part[32][8];
  const int t = blockIdx.x, k = threadIdx.x, lane = k & 63, wave = k >> 6;
  const float c0 = coords[2 * t], c1 = coords[2 * t + 1];
  const float hk = fmaxf(fmaf(w1[2 * k], c0, fmaf(w1[2 * k + 1], c1, b1[k])), 0.f);
  for (int h = 0; h < H; ++h) {
    const float v = wave_sum(w2[h * 512 + k] * hk);
    if (lane == 0) part[h][wave] = v;
  }
  __syncthreads();
  if (k < H) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += part[k][w];
    out[t * H + k] = s;
  }
}

__global__ void __launch_bounds__(256) swin_bias_kernel(int64_t nW, int64_t H, int64_t L, const float* __restrict__ table,
                                                        const int32_t* __restrict__ rpi, const float* __restrict__ mask,
                                                        float* __restrict__ out) {
  const int64_t LL = L * L, total = nW * H * LL;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ij = t % LL;
    const int64_t wh = t / LL;
    const int64_t h = wh % H, w = wh / H;
    const float x = table[(int64_t)rpi[ij] * H + h];
    float v = 16.f / (1.f + expf(-x));
    if (mask) {
      const float m = mask[w * LL + ij];
      v = (v + m) + m;
    }
    out[t] = v;
  }
}

// one thread per (row, head, q|k); d <= 64 elements, d * esz a multiple of 16 B
template <typename T, int d>
__global__ void __launch_bounds__(256) swin_qk_norm_kernel(int64_t rows, int H, T* __restrict__ qkv, int64_t ld,
                                                           const float* __restrict__ logit_scale, float max_log) {
  constexpr int N = 16 / sizeof(T);
  const int64_t total = rows * H * 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int which = (int)(t % 2);          // 0 = q, 1 = k
  const int h = (int)((t / 2) % H);
  const int64_t row = t / (2 * H);
  T* p = qkv + row * ld + (int64_t)which * H * d + (int64_t)h * d;
  constexpr int nch = d / N;
  float v[d];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < nch; ++c) {
    const uint4 raw = reinterpret_cast<const uint4*>(p)[c];
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int j = 0; j < N; ++j) { v[c * N + j] = to_f32(e[j]); ss = fmaf(v[c * N + j], v[c * N + j], ss); }
  }
  float s = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  const float mult = which == 0 ? expf(fminf(logit_scale[h], max_log)) : 1.f;
#pragma unroll
  for (int c = 0; c < nch; ++c) {
    uint4 raw;
    T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
    for (int j = 0; j < N; ++j) e[j] = from_f32<T>((v[c * N + j] * s) * mult);
    reinterpret_cast<uint4*>(p)[c] = raw;
  }
}

unsigned blocks_for(int64_t n, int per) {
  int64_t b = (n + per - 1) / per;
  if (b > 65536) b = 65536;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" int mmfd_row_gather(int64_t B, int64_t rows_out, int64_t G, int64_t row_bytes, int64_t src_rows,
                               const void* src, const int32_t* idx, void* dst, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(row_bytes > 0 && row_bytes % 16 == 0, "row_gather: row bytes must be a positive multiple of 16");
  MMFD_CHECK_ARG(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "row_gather: 16-B aligned buffers");
  MMFD_CHECK_ARG(B >= 0 && rows_out >= 0 && G > 0 && src_rows > 0, "row_gather: bad shape");
  const int64_t total = B * rows_out * G * (row_bytes / 16);
  if (total == 0) return 0;
  hipLaunchKernelGGL(row_gather_kernel, dim3(blocks_for(total, 256)), dim3(256), 0, (hipStream_t)stream, B, rows_out,
                     G, row_bytes / 16, src_rows, (const uint4*)src, idx, (uint4*)dst);
  MMFD_CHECK_LAUNCH("row_gather");
  return 0;
}

extern "C" int mmfd_swin_cpb(int64_t T, int64_t H, const float* coords, const float* w1, const float* b1,
                             const float* w2, float* out, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(H > 0 && H <= 32 && T > 0, "swin_cpb: 1 <= H <= 32 heads");
  hipLaunchKernelGGL(swin_cpb_kernel, dim3((unsigned)T), dim3(512), 0, (hipStream_t)stream, (int)H, coords, w1, b1, w2,
                     out);
  MMFD_CHECK_LAUNCH("swin_cpb");
  return 0;
}

extern "C" int mmfd_swin_bias(int64_t nW, int64_t H, int64_t L, const float* table, const int32_t* rpi,
                              const float* mask, float* out, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(nW > 0 && H > 0 && L > 0, "swin_bias: bad shape");
  const int64_t total = nW * H * L * L;
  hipLaunchKernelGGL(swin_bias_kernel, dim3(blocks_for(total, 256)), dim3(256), 0, (hipStream_t)stream, nW, H, L, table,
                     rpi, mask, out);
  MMFD_CHECK_LAUNCH("swin_bias");
  return 0;
}

extern "C" int mmfd_swin_qk_norm(int dtype, int64_t rows, int64_t H, int64_t d, void* qkv, int64_t ld,
                                 const float* logit_scale, float max_log, mmfd_stream_t stream) {
  const int esz = dtype == MMFD_BF16 ? 2 : 4;
  MMFD_CHECK_ARG(d > 0 && d <= 64 && (d * esz) % 16 == 0, "swin_qk_norm: head dim %lld unsupported", (long long)d);
  MMFD_CHECK_ARG(((uintptr_t)qkv & 15) == 0 && (ld * esz) % 16 == 0, "swin_qk_norm: 16-B aligned rows");
  const int64_t total = rows * H * 2;
  if (total == 0) return 0;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
#define QKN(T, D) hipLaunchKernelGGL((swin_qk_norm_kernel<T, D>), grid, dim3(256), 0, s, rows, (int)H, (T*)qkv, ld, logit_scale, max_log)
  if (dtype == MMFD_BF16) {
    if (d == 16) QKN(bf16, 16); else if (d == 32) QKN(bf16, 32); else if (d == 64) QKN(bf16, 64);
    else MMFD_CHECK_ARG(false, "swin_qk_norm: head dim %lld unsupported", (long long)d);
  } else {
    if (d == 16) QKN(float, 16); else if (d == 32) QKN(float, 32); else if (d == 64) QKN(float, 64);
    else MMFD_CHECK_ARG(false, "swin_qk_norm: head dim %lld unsupported", (long long)d);
  }
#undef QKN
  MMFD_CHECK_LAUNCH("swin_qk_norm");
  return 0;
}
