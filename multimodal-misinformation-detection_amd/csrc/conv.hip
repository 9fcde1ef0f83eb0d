// Convolution support for the ResNet50 evidence-image extractor (im2im_retrieval.py:14-36): NHWC
// activations, every convolution lowered to the MFMA GEMM (1x1 stride-1 convs read the activation
// directly; 3x3 / strided / stem convs go through an im2col gather), eval-mode BatchNorm folded
// into the GEMM weights and bias, ReLU and the bottleneck's residual add in the GEMM epilogue.
#include "common.h"
#include <algorithm>

namespace {

inline unsigned grid_for(int64_t n, int per) { return (unsigned)std::min<int64_t>((n + per - 1) / per, 65535 * 8); }

// out_w[co][(kh*KW + kw)*Cin + ci] = w[co][ci][kh][kw] * s[co], zero for k >= KH*KW*Cin;
// out_b[co] = beta[co] - mean[co] * s[co], s = gamma / sqrt(var + eps) (s = 1, b = 0 without BN)
template <typename T>
__global__ void weight_prep_kernel(int64_t Cout, int64_t Cin, int64_t KH, int64_t KW, int64_t Kpad,
                                   const float* __restrict__ w, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, const float* __restrict__ mean,
                                   const float* __restrict__ var, float eps, T* __restrict__ out_w,
                                   float* __restrict__ out_b) {
  const int64_t n = Cout * Kpad;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t co = i / Kpad, k = i % Kpad;
    const float sc = gamma ? gamma[co] / sqrtf(var[co] + eps) : 1.f;
    float v = 0.f;
    if (k < KH * KW * Cin) {
      const int64_t ci = k % Cin, kk = k / Cin, kw = kk % KW, kh = kk / KW;
      v = w[((co * Cin + ci) * KH + kh) * KW + kw] * sc;
    }
    out_w[i] = from_f32<T>(v);
    if (k == 0 && out_b) out_b[co] = gamma ? beta[co] - mean[co] * sc : 0.f;
  }
}

// im2col of an NHWC activation: out[(n*Ho + ho)*Wo + wo][(kh*KW + kw)*C + c], 16-B chunks of C
template <typename T>
__global__ void im2col_nhwc_kernel(int64_t N, int64_t H, int64_t W, int64_t C, int KH, int KW, int stride, int pad,
                                   int64_t Ho, int64_t Wo, int64_t Kpad, const T* __restrict__ x, T* __restrict__ out) {
  constexpr int EPC = 16 / sizeof(T);
  const int64_t cch = C / EPC;
  const int64_t per_row = (int64_t)KH * KW * cch;
  const int64_t n_total = N * Ho * Wo * per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / per_row, r = i % per_row;
    const int64_t c = (r % cch) * EPC, kk = r / cch;
    const int kw = (int)(kk % KW), kh = (int)(kk / KW);
    const int64_t wo = row % Wo, t = row / Wo, ho = t % Ho, nimg = t / Ho;
    const int64_t hi = ho * stride - pad + kh, wi = wo * stride - pad + kw;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (hi >= 0 && hi < H && wi >= 0 && wi < W) v = *reinterpret_cast<const uint4*>(x + ((nimg * H + hi) * W + wi) * C + c);
    *reinterpret_cast<uint4*>(out + row * Kpad + kk * C + c) = v;
  }
  // zero the K padding columns
  const int64_t kreal = (int64_t)KH * KW * C;
  if (Kpad > kreal) {
    const int64_t padw = Kpad - kreal, np = N * Ho * Wo * padw;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x)
      out[(i / padw) * Kpad + kreal + i % padw] = from_f32<T>(0.f);
  }
}

// stem im2col straight from the fp32 NCHW pixel tensor (C = 3): out[row][(kh*KW + kw)*C + c].
// Consecutive threads write consecutive output elements (coalesced: the output is the big side,
// 1.95 GB at bs = 256 fp32); each block walks 16 rows at a time; the k -> (c, kh, kw) decomposition
// comes from per-block LDS tables (pixel offset of the tap, kh, kw; kh = -1 for the K padding
// columns), so an element costs three 32-bit divisions (row, pixel) and one gathered load (the
// pixels are L2 hits: each is read by ~KH*KW/stride^2 windows). Round 1's form — one thread per
// element with 64-bit divisions for every index — ran at ~0.9 TB/s (2.1 ms at bs = 256), a
// thread-per-(row, kh) form with 21 scalar stores per thread 3x slower still.
constexpr int kStemKmax = 512;
template <typename T>
__global__ void __launch_bounds__(256) im2col_nchw_kernel(uint32_t N, uint32_t C, uint32_t H, uint32_t W, uint32_t KH,
                                                          uint32_t KW, uint32_t stride, uint32_t pad, uint32_t Ho,
                                                          uint32_t Wo, uint32_t Kpad, const float* __restrict__ x,
                                                          T* __restrict__ out) {
  __shared__ int tap_off[kStemKmax];
  __shared__ short tap_kh[kStemKmax], tap_kw[kStemKmax];
  const uint32_t tid = threadIdx.x;
  for (uint32_t k = tid; k < Kpad; k += 256) {
    if (k < KH * KW * C) {
      const uint32_t c = k % C, kk = k / C, kw = kk % KW, kh = kk / KW;
      tap_off[k] = (int)(c * H * W + kh * W + kw);
      tap_kh[k] = (short)kh;
      tap_kw[k] = (short)kw;
    } else {
      tap_off[k] = 0; tap_kh[k] = -1; tap_kw[k] = 0;
    }
  }
  __syncthreads();
  constexpr uint32_t RB = 16;
  const uint32_t rows = N * Ho * Wo;
  for (uint32_t r0 = blockIdx.x * RB; r0 < rows; r0 += gridDim.x * RB) {
    const uint32_t nel = min(RB, rows - r0) * Kpad;
    for (uint32_t idx = tid; idx < nel; idx += 256) {
      const uint32_t rl = idx / Kpad, k = idx - rl * Kpad, row = r0 + rl;
      const uint32_t wo = row % Wo, t = row / Wo, ho = t % Ho, n = t / Ho;
      const int kh = tap_kh[k];
      const int hi = (int)(ho * stride) - (int)pad + kh, wi = (int)(wo * stride) - (int)pad + tap_kw[k];
      float v = 0.f;
      if (kh >= 0 && hi >= 0 && hi < (int)H && wi >= 0 && wi < (int)W)
        v = x[(size_t)n * C * H * W + (size_t)(tap_off[k] + (int)(ho * stride - pad) * (int)W + (int)(wo * stride) - (int)pad)];
      out[(size_t)row * Kpad + k] = from_f32<T>(v);
    }
  }
}

// max pooling on NHWC (padding never wins: -inf), 8 channels per thread for bf16 / 4 for fp32
template <typename T>
__global__ void maxpool_nhwc_kernel(int64_t N, int64_t H, int64_t W, int64_t C, int k, int stride, int pad, int64_t Ho,
                                    int64_t Wo, const T* __restrict__ x, T* __restrict__ out) {
  constexpr int EPC = 16 / sizeof(T);
  const int64_t cch = C / EPC;
  const int64_t n_total = N * Ho * Wo * cch;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = (i % cch) * EPC, row = i / cch;
    const int64_t wo = row % Wo, t = row / Wo, ho = t % Ho, nimg = t / Ho;
    float m[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) m[e] = -INFINITY;
    for (int kh = 0; kh < k; ++kh) {
      const int64_t hi = ho * stride - pad + kh;
      if (hi < 0 || hi >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int64_t wi = wo * stride - pad + kw;
        if (wi < 0 || wi >= W) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(x + ((nimg * H + hi) * W + wi) * C + c);
        const T* tv = reinterpret_cast<const T*>(&v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) m[e] = fmaxf(m[e], to_f32(tv[e]));
      }
    }
    T o[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) o[e] = from_f32<T>(m[e]);
    *reinterpret_cast<uint4*>(out + row * C + c) = *reinterpret_cast<const uint4*>(o);
  }
}

// global average pool NHWC [N][HW][C] -> fp32 [N][C]; block = (image, 256-channel slab), 4 waves
// split the spatial positions, fixed-order LDS combine
template <typename T>
__global__ void __launch_bounds__(256) avgpool_kernel(int64_t HW, int64_t C, const T* __restrict__ x,
                                                      float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t n = blockIdx.y;
  for (int64_t c0 = (int64_t)blockIdx.x * 64; c0 < C; c0 += (int64_t)gridDim.x * 64) {
    const int64_t c = c0 + lane;
    float s = 0.f;
    if (c < C)
      for (int64_t p = wave; p < HW; p += 4) s += to_f32(x[(n * HW + p) * C + c]);
    red[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && c < C) out[n * C + c] = ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) / (float)HW;
    __syncthreads();
  }
}

}  // namespace

extern "C" int mmfd_conv_weight_prep(int dtype, int64_t Cout, int64_t Cin, int64_t KH, int64_t KW, int64_t Kpad,
                                     const float* w, const float* gamma, const float* beta, const float* mean,
                                     const float* var, float eps, void* out_w, float* out_b, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(Kpad >= KH * KW * Cin, "conv_weight_prep: Kpad < KH*KW*Cin");
  MMFD_CHECK_ARG(!gamma || (beta && mean && var), "conv_weight_prep: BN needs gamma, beta, mean, var");
  const int64_t n = Cout * Kpad;
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((weight_prep_kernel<bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, Cout, Cin, KH, KW, Kpad, w, gamma,
                       beta, mean, var, eps, (bf16*)out_w, out_b);
  else
    hipLaunchKernelGGL((weight_prep_kernel<float>), dim3(grid_for(n, 256)), dim3(256), 0, s, Cout, Cin, KH, KW, Kpad, w,
                       gamma, beta, mean, var, eps, (float*)out_w, out_b);
  MMFD_CHECK_LAUNCH("conv_weight_prep");
  return 0;
}

extern "C" int mmfd_im2col_nhwc(int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int KH, int KW, int stride,
                                int pad, int64_t Ho, int64_t Wo, int64_t Kpad, const void* x, void* out,
                                mmfd_stream_t stream) {
  const int epc = dtype == MMFD_BF16 ? 8 : 4;
  MMFD_CHECK_ARG(C % epc == 0, "im2col_nhwc: C must be a multiple of %d", epc);
  MMFD_CHECK_ARG(Kpad >= (int64_t)KH * KW * C, "im2col_nhwc: Kpad too small");
  MMFD_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 && Kpad % epc == 0, "im2col_nhwc: alignment");
  const int64_t n = N * Ho * Wo * KH * KW * (C / epc);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((im2col_nhwc_kernel<bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, N, H, W, C, KH, KW, stride, pad,
                       Ho, Wo, Kpad, (const bf16*)x, (bf16*)out);
  else
    hipLaunchKernelGGL((im2col_nhwc_kernel<float>), dim3(grid_for(n, 256)), dim3(256), 0, s, N, H, W, C, KH, KW, stride,
                       pad, Ho, Wo, Kpad, (const float*)x, (float*)out);
  MMFD_CHECK_LAUNCH("im2col_nhwc");
  return 0;
}

extern "C" int mmfd_im2col_nchw(int dtype, int64_t N, int64_t C, int64_t H, int64_t W, int KH, int KW, int stride,
                                int pad, int64_t Ho, int64_t Wo, int64_t Kpad, const float* x, void* out,
                                mmfd_stream_t stream) {
  MMFD_CHECK_ARG(Kpad >= (int64_t)KH * KW * C, "im2col_nchw: Kpad too small");
  MMFD_CHECK_ARG(C * H * W < (1ll << 31) && N * Ho * Wo < (1ll << 31) && Kpad <= kStemKmax && KH > 0 && KW > 0 &&
                 stride > 0, "im2col_nchw: sizes past the kernel's index range (Kpad <= %d)", kStemKmax);
  const int64_t n = (N * Ho * Wo + 15) / 16 * 256;  // 16 rows per block-iteration
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((im2col_nchw_kernel<bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, (uint32_t)N, (uint32_t)C,
                       (uint32_t)H, (uint32_t)W, (uint32_t)KH, (uint32_t)KW, (uint32_t)stride, (uint32_t)pad, (uint32_t)Ho,
                       (uint32_t)Wo, (uint32_t)Kpad, x, (bf16*)out);
  else
    hipLaunchKernelGGL((im2col_nchw_kernel<float>), dim3(grid_for(n, 256)), dim3(256), 0, s, (uint32_t)N, (uint32_t)C,
                       (uint32_t)H, (uint32_t)W, (uint32_t)KH, (uint32_t)KW, (uint32_t)stride, (uint32_t)pad, (uint32_t)Ho,
                       (uint32_t)Wo, (uint32_t)Kpad, x, (float*)out);
  MMFD_CHECK_LAUNCH("im2col_nchw");
  return 0;
}

extern "C" int mmfd_maxpool_nhwc(int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int k, int stride, int pad,
                                 int64_t Ho, int64_t Wo, const void* x, void* out, mmfd_stream_t stream) {
  const int epc = dtype == MMFD_BF16 ? 8 : 4;
  MMFD_CHECK_ARG(C % epc == 0, "maxpool_nhwc: C must be a multiple of %d", epc);
  const int64_t n = N * Ho * Wo * (C / epc);
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((maxpool_nhwc_kernel<bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, N, H, W, C, k, stride, pad, Ho,
                       Wo, (const bf16*)x, (bf16*)out);
  else
    hipLaunchKernelGGL((maxpool_nhwc_kernel<float>), dim3(grid_for(n, 256)), dim3(256), 0, s, N, H, W, C, k, stride, pad, Ho,
                       Wo, (const float*)x, (float*)out);
  MMFD_CHECK_LAUNCH("maxpool_nhwc");
  return 0;
}

extern "C" int mmfd_global_avgpool(int dtype, int64_t N, int64_t HW, int64_t C, const void* x, float* out,
                                   mmfd_stream_t stream) {
  if (N * C == 0) return 0;
  MMFD_CHECK_ARG(HW > 0, "global_avgpool: HW must be > 0");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)std::min<int64_t>((C + 63) / 64, 64), (unsigned)N);
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((avgpool_kernel<bf16>), grid, dim3(256), 0, s, HW, C, (const bf16*)x, out);
  else
    hipLaunchKernelGGL((avgpool_kernel<float>), grid, dim3(256), 0, s, HW, C, (const float*)x, out);
  MMFD_CHECK_LAUNCH("global_avgpool");
  return 0;
}
