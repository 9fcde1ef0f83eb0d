// LayerNorm forward / backward (one or two rows per wave, width <= 1024, width % 4 == 0).
// Replaces nn.LayerNorm in the fusion head (model.py:39-46, 155-162; eps 1e-5) and the BERT/ViT
// LayerNorms (eps 1e-12). Statistics in fp32; gamma/beta gradients via a deterministic two-pass
// column reduction (per-lane column ownership -> per-block partials -> final sum).
#include "common.h"
#include <algorithm>

namespace {
constexpr int MAXC = 4;  // 4-element chunks per lane -> width <= 1024

template <typename T> struct V4;
template <> struct V4<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[4]) {
    const float4 x = *reinterpret_cast<const float4*>(p); v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct V4<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[4]) {
    const uint2 x = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
  }
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[4]) {
    typedef __attribute__((ext_vector_type(4))) __bf16 b4;
    b4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    *reinterpret_cast<uint2*>(p) = __builtin_bit_cast(uint2, o);
  }
};

template <typename T>
__global__ void __launch_bounds__(256) ln_fwd_kernel(int64_t rows, int width, const T* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, T* __restrict__ y, int64_t ldy, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nch = width >> 2;
  float v[MAXC][4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < nch) {
      V4<T>::load(x + row * ldx + 4 * c, v[j]);
      s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
    }
  }
  const float mu = wave_sum(s) / (float)width;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < nch)
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[j][e] - mu; q += d * d; }
  }
  const float rs = rsqrtf(wave_sum(q) / (float)width + eps);
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    const int c = lane + 64 * j;
    if (c < nch) {
      const float4 gg = *reinterpret_cast<const float4*>(gamma + 4 * c);
      const float4 bb = *reinterpret_cast<const float4*>(beta + 4 * c);
      float o[4];
      o[0] = (v[j][0] - mu) * rs * gg.x + bb.x;
      o[1] = (v[j][1] - mu) * rs * gg.y + bb.y;
      o[2] = (v[j][2] - mu) * rs * gg.z + bb.z;
      o[3] = (v[j][3] - mu) * rs * gg.w + bb.w;
      V4<T>::store(y + row * ldy + 4 * c, o);
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

template <typename T>
__global__ void __launch_bounds__(256) ln_bwd_kernel(int64_t rows, int width, const T* __restrict__ dy, int64_t lddy,
                                                     const T* __restrict__ x, int64_t ldx, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     T* __restrict__ dx, int64_t lddx, const T* __restrict__ dx_add,
                                                     int64_t ldadd, T* __restrict__ dx_drop, float p, uint32_t thr,
                                                     const uint64_t* __restrict__ seedp, uint64_t salt,
                                                     float* __restrict__ part) {
  __shared__ float red[4][2][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = width >> 2;
  const uint64_t seed = (dx_drop && p > 0.f) ? *seedp : 0ull;
  const float keep = 1.0f / (1.0f - p);
  float pg[MAXC][4], pb[MAXC][4];
#pragma unroll
  for (int j = 0; j < MAXC; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) { pg[j][e] = 0.f; pb[j][e] = 0.f; }

  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < rows; row += (int64_t)gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXC][4], g[MAXC][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
        float d[4], xv[4];
        V4<T>::load(dy + row * lddy + 4 * c, d);
        V4<T>::load(x + row * ldx + 4 * c, xv);
        const float4 gg = *reinterpret_cast<const float4*>(gamma + 4 * c);
        const float gv[4] = {gg.x, gg.y, gg.z, gg.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[j][e] = (xv[e] - mu) * rs;
          g[j][e] = d[e] * gv[e];
          s1 += g[j][e];
          s2 += g[j][e] * xh[j][e];
          pg[j][e] += d[e] * xh[j][e];
          pb[j][e] += d[e];
        }
      }
    }
    const float c1 = wave_sum(s1) / (float)width;
    const float c2 = wave_sum(s2) / (float)width;
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
        float o[4], add[4] = {0.f, 0.f, 0.f, 0.f};
        if (dx_add) V4<T>::load(dx_add + row * ldadd + 4 * c, add);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs * (g[j][e] - c1 - xh[j][e] * c2) + add[e];
        V4<T>::store(dx + row * lddx + 4 * c, o);
        if (dx_drop) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t h = mmfd_hash(seed, salt, (uint64_t)row * (uint64_t)width + 4 * c + e);
            o[e] = (p > 0.f && h < thr) ? 0.f : o[e] * (p > 0.f ? keep : 1.f);
          }
          V4<T>::store(dx_drop + row * lddx + 4 * c, o);
        }
      }
    }
  }
  // block reduction of the per-lane column partials: chunk c = lane + 64 j, handled 256 cols at a time
#pragma unroll
  for (int j = 0; j < MAXC; ++j) {
    if (64 * j >= nch) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[wave][0][lane * 4 + e] = pg[j][e];
      red[wave][1][lane * 4 + e] = pb[j][e];
    }
    __syncthreads();
    const int col_local = threadIdx.x;  // 0..255 within this 256-column slab
    const int col = 256 * j + col_local;
    if (col < width) {
      const float sg = red[0][0][col_local] + red[1][0][col_local] + red[2][0][col_local] + red[3][0][col_local];
      const float sb = red[0][1][col_local] + red[1][1][col_local] + red[2][1][col_local] + red[3][1][col_local];
      part[((int64_t)blockIdx.x * 2 + 0) * width + col] = sg;
      part[((int64_t)blockIdx.x * 2 + 1) * width + col] = sb;
    }
    __syncthreads();
  }
}


// ---- 16-byte vector variants (width a multiple of 8 bf16 / 4 fp32): one wave per row, lane owns
// 16-B chunks c = lane + 64 j
template <typename T> struct VN;
template <> struct VN<float> {
  static constexpr int N = 4, MAXV = 4;
  __device__ __forceinline__ static void load(const float* p, float (&v)[N]) {
    const float4 x = *reinterpret_cast<const float4*>(p); v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[N]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct VN<bf16> {
  static constexpr int N = 8, MAXV = 2;
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[N]) {
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
  }
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[N]) {
    bf16x8 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
    *reinterpret_cast<uint4*>(p) = __builtin_bit_cast(uint4, o);
  }
};

template <typename T>
__device__ __forceinline__ void load_f32xN(const float* p, float (&v)[VN<T>::N]) {
#pragma unroll
  for (int i = 0; i < VN<T>::N; i += 4) {
    const float4 a = *reinterpret_cast<const float4*>(p + i);
    v[i] = a.x; v[i + 1] = a.y; v[i + 2] = a.z; v[i + 3] = a.w;
  }
}

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LPR lanes per row (64 / LPR rows per wave), CH 16-B chunks per lane (lane l owns chunks l + LPR j):
// <T, 64, VN<T>::MAXV> is the row-per-wave form for any width <= 1024; bf16 rows of 33-128 chunks
// (width 264-1024: BERT / ViT-B's 768 = 96 chunks) run <bf16, 32, 3 | 4>, two rows per wave and no
// idle lanes (the row-per-wave form left half the lanes of its second chunk idle at 96 chunks and
// moved 1.5 KB per wave)
template <typename T, int LPR, int CH>
__global__ void __launch_bounds__(256) ln_fwd16_kernel(int64_t rows, int width, const T* __restrict__ x, int64_t ldx,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, T* __restrict__ y, int64_t ldy,
                                                       float* __restrict__ mean, float* __restrict__ rstd,
                                                       const T* __restrict__ res = nullptr, int64_t ldr = 0,
                                                       bf16* __restrict__ pl = nullptr, int64_t pl_stride = 0) {
  constexpr int N = VN<T>::N, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, l = lane % LPR;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  if (row >= rows) return;  // whole LPR groups leave together: the group shuffles stay inside live lanes
  const int nch = width / N;
  float v[CH][N];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = l + LPR * j;
    if (c < nch) {
      VN<T>::load(x + row * ldx + N * c, v[j]);
#pragma unroll
      for (int e = 0; e < N; ++e) s += v[j][e];
    }
  }
  const float mu = group_sum<LPR>(s) / (float)width;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = l + LPR * j;
    if (c < nch)
#pragma unroll
      for (int e = 0; e < N; ++e) { const float d = v[j][e] - mu; q += d * d; }
  }
  const float rs = rsqrtf(group_sum<LPR>(q) / (float)width + eps);
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = l + LPR * j;
    if (c < nch) {
      float gg[N], bb[N], o[N];
      load_f32xN<T>(gamma + N * c, gg);
      load_f32xN<T>(beta + N * c, bb);
#pragma unroll
      for (int e = 0; e < N; ++e) o[e] = (v[j][e] - mu) * rs * gg[e] + bb[e];
      if (res) {  // y = res + LN(x) (Swinv2 res-post-norm)
        float r[N];
        VN<T>::load(res + row * ldr + N * c, r);
#pragma unroll
        for (int e = 0; e < N; ++e) o[e] += r[e];
      }
      VN<T>::store(y + row * ldy + N * c, o);
      if constexpr (sizeof(T) == 4) {
        if (pl) {  // fp32: the output's split planes (hi, mid, lo) for split-operand GEMMs
          bf16 h[N], m[N], lo[N];
#pragma unroll
          for (int e = 0; e < N; ++e) {
            h[e] = (bf16)o[e];
            const float r1 = o[e] - (float)h[e];
            m[e] = (bf16)r1;
            lo[e] = (bf16)(r1 - (float)m[e]);
          }
          bf16* d = pl + row * width + N * c;
          *reinterpret_cast<uint2*>(d) = __builtin_bit_cast(uint2, h);
          *reinterpret_cast<uint2*>(d + pl_stride) = __builtin_bit_cast(uint2, m);
          *reinterpret_cast<uint2*>(d + 2 * pl_stride) = __builtin_bit_cast(uint2, lo);
        }
      }
    }
  }
  if (l == 0 && mean) { mean[row] = mu; rstd[row] = rs; }
}

// the row-per-wave or two-rows-per-wave form for a 16-B-vectorisable row of `width` elements
// (> 32 chunks; narrower rows take ln_fwd16_narrow_kernel)
template <typename T, typename... A>
void launch_ln_fwd16(hipStream_t s, int64_t rows, int width, A... args) {
  const int nch = width / VN<T>::N;
  if (nch > 32 && nch <= 128 / (int)(sizeof(T) / 2)) {  // bf16 33-128 chunks, fp32 33-64
    const dim3 grid((unsigned)((rows + 7) / 8));
    if constexpr (sizeof(T) == 4) hipLaunchKernelGGL((ln_fwd16_kernel<T, 32, 2>), grid, dim3(256), 0, s, rows, width, args...);
    else if (nch <= 96) hipLaunchKernelGGL((ln_fwd16_kernel<T, 32, 3>), grid, dim3(256), 0, s, rows, width, args...);
    else hipLaunchKernelGGL((ln_fwd16_kernel<T, 32, 4>), grid, dim3(256), 0, s, rows, width, args...);
    return;
  }
  hipLaunchKernelGGL((ln_fwd16_kernel<T, 64, VN<T>::MAXV>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, rows,
                     width, args...);
}

// narrow rows (width / elements-per-16B <= LPR): 64 / LPR rows per wave, LPR lanes per row, one
// 16-B chunk per lane, group reductions over the LPR lanes (the one-row-per-wave kernel leaves 3/4
// of the lanes idle at width 128 bf16: Swinv2 stage 1, and half of them at the fusion head's 256)
template <typename T, int LPR>
__global__ void __launch_bounds__(256) ln_fwd16_narrow_kernel(int64_t rows, int width, const T* __restrict__ x,
                                                              int64_t ldx, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float eps,
                                                              T* __restrict__ y, int64_t ldy, float* __restrict__ mean,
                                                              float* __restrict__ rstd, const T* __restrict__ res,
                                                              int64_t ldr) {
  constexpr int N = VN<T>::N, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, l = lane % LPR;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  if (row >= rows) return;  // whole LPR groups leave together: the group shuffles stay inside live lanes
  const int nch = width / N;
  const bool on = l < nch;
  float v[N];
  float s = 0.f;
  if (on) {
    VN<T>::load(x + row * ldx + N * l, v);
#pragma unroll
    for (int e = 0; e < N; ++e) s += v[e];
  }
  const float mu = group_sum<LPR>(s) / (float)width;
  float q = 0.f;
  if (on) {
#pragma unroll
    for (int e = 0; e < N; ++e) { const float d = v[e] - mu; q += d * d; }
  }
  const float rs = rsqrtf(group_sum<LPR>(q) / (float)width + eps);
  if (on) {
    float gg[N], bb[N], o[N];
    load_f32xN<T>(gamma + N * l, gg);
    load_f32xN<T>(beta + N * l, bb);
#pragma unroll
    for (int e = 0; e < N; ++e) o[e] = (v[e] - mu) * rs * gg[e] + bb[e];
    if (res) {
      float r[N];
      VN<T>::load(res + row * ldr + N * l, r);
#pragma unroll
      for (int e = 0; e < N; ++e) o[e] += r[e];
    }
    VN<T>::store(y + row * ldy + N * l, o);
  }
  if (l == 0 && mean) { mean[row] = mu; rstd[row] = rs; }
}

// launches the narrow kernel when a row fits 16 / 32 lanes; false -> caller uses the row-per-wave one
template <typename T>
bool launch_ln_narrow(hipStream_t s, int64_t rows, int width, const T* x, int64_t ldx, const float* gamma,
                      const float* beta, float eps, T* y, int64_t ldy, float* mean, float* rstd, const T* res,
                      int64_t ldr) {
  const int nch = width / VN<T>::N;
  if (nch <= 16) {
    hipLaunchKernelGGL((ln_fwd16_narrow_kernel<T, 16>), dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, s, rows,
                       width, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, res, ldr);
    return true;
  }
  if (nch <= 32) {
    hipLaunchKernelGGL((ln_fwd16_narrow_kernel<T, 32>), dim3((unsigned)((rows + 7) / 8)), dim3(256), 0, s, rows,
                       width, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, res, ldr);
    return true;
  }
  return false;
}

// one 16-B chunk as loaded (converted to fp32 after the next row's loads are issued)
template <typename T> struct VR;
template <> struct VR<float> {
  float4 v;
  __device__ __forceinline__ void load(const float* p) { v = *reinterpret_cast<const float4*>(p); }
  __device__ __forceinline__ void get(float (&f)[4]) const { f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w; }
};
template <> struct VR<bf16> {
  uint4 v;
  __device__ __forceinline__ void load(const bf16* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void get(float (&f)[8]) const {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(w[i] << 16); f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
  }
};

// backward, LPR lanes per row and CH chunks per lane as ln_fwd16_kernel; each wave walks rows with
// a grid stride; with PF the next row's dy / x / dx_add chunks and statistics are loaded before this
// row's reductions (one row's HBM latency per wave hidden behind the previous row's math: bf16
// 768-wide rows 1.2-1.3x; the fp32 row-per-wave form, at 3 KB per row already, measured 1-3 %
// slower with it — its doubled registers halve the waves per SIMD — and runs without)
template <typename T, int LPR, int CH, bool PF = true>
__global__ void __launch_bounds__(256) ln_bwd16_kernel(int64_t rows, int width, const T* __restrict__ dy, int64_t lddy,
                                                       const T* __restrict__ x, int64_t ldx, const float* __restrict__ gamma,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       T* __restrict__ dx, int64_t lddx, const T* __restrict__ dx_add,
                                                       int64_t ldadd, T* __restrict__ dx_drop, float p, uint32_t thr,
                                                       const uint64_t* __restrict__ seedp, uint64_t salt,
                                                       float* __restrict__ part, bf16* __restrict__ pl = nullptr,
                                                       int64_t pl_stride = 0) {
  constexpr int N = VN<T>::N, RPW = 64 / LPR;
  __shared__ float red[4][2][64 * N];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l = lane % LPR;
  const int nch = width / N;
  const uint64_t seed = (dx_drop && p > 0.f) ? *seedp : 0ull;
  const float keep = 1.0f / (1.0f - p);
  float pg[CH][N], pb[CH][N], gv[CH][N];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = l + LPR * j;
#pragma unroll
    for (int e = 0; e < N; ++e) { pg[j][e] = 0.f; pb[j][e] = 0.f; gv[j][e] = 0.f; }
    if (PF && c < nch) load_f32xN<T>(gamma + N * c, gv[j]);  // (held across rows with PF only)
  }
  const int64_t rstep = (int64_t)gridDim.x * 4 * RPW;
  int64_t row = ((int64_t)blockIdx.x * 4 + wave) * RPW + lane / LPR;
  VR<T> rd[CH], rx[CH], ra[CH];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t r) {
    if (r < rows) {
      nmu = mean[r];
      nrs = rstd[r];
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int c = l + LPR * j;
        if (c < nch) {
          rd[j].load(dy + r * lddy + N * c);
          rx[j].load(x + r * ldx + N * c);
          if (dx_add) ra[j].load(dx_add + r * ldadd + N * c);
        }
      }
    }
  };
  if constexpr (PF) fetch(row);
  for (; row < rows; row += rstep) {
    if constexpr (!PF) fetch(row);
    const float mu = nmu, rs = nrs;
    float xh[CH][N], g[CH][N], add[CH][N];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = l + LPR * j;
      if (c < nch) {
        float d[N], gq[N];
        rd[j].get(d);
        rx[j].get(xh[j]);
        if (dx_add) ra[j].get(add[j]);
        if constexpr (PF) {
#pragma unroll
          for (int e = 0; e < N; ++e) gq[e] = gv[j][e];
        } else {
          load_f32xN<T>(gamma + N * c, gq);
        }
#pragma unroll
        for (int e = 0; e < N; ++e) {
          xh[j][e] = (xh[j][e] - mu) * rs;
          g[j][e] = d[e] * gq[e];
          s1 += g[j][e];
          s2 += g[j][e] * xh[j][e];
          pg[j][e] += d[e] * xh[j][e];
          pb[j][e] += d[e];
        }
      }
    }
    if constexpr (PF) fetch(row + rstep);
    const float c1 = group_sum<LPR>(s1) / (float)width;
    const float c2 = group_sum<LPR>(s2) / (float)width;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = l + LPR * j;
      if (c < nch) {
        float o[N];
#pragma unroll
        for (int e = 0; e < N; ++e) o[e] = rs * (g[j][e] - c1 - xh[j][e] * c2) + (dx_add ? add[j][e] : 0.f);
        VN<T>::store(dx + row * lddx + N * c, o);
        if (dx_drop) {
#pragma unroll
          for (int e = 0; e < N; ++e) {
            const uint32_t h = mmfd_hash(seed, salt, (uint64_t)row * (uint64_t)width + N * c + e);
            o[e] = (p > 0.f && h < thr) ? 0.f : o[e] * (p > 0.f ? keep : 1.f);
          }
          VN<T>::store(dx_drop + row * lddx + N * c, o);
        }
        if constexpr (sizeof(T) == 4) {
          if (pl) {  // fp32: split planes of the GEMM operand (dx_drop when present, else dx)
            bf16 h[N], m[N], lo[N];
#pragma unroll
            for (int e = 0; e < N; ++e) {
              h[e] = (bf16)o[e];
              const float r1 = o[e] - (float)h[e];
              m[e] = (bf16)r1;
              lo[e] = (bf16)(r1 - (float)m[e]);
            }
            bf16* dpl = pl + row * width + N * c;
            *reinterpret_cast<uint2*>(dpl) = __builtin_bit_cast(uint2, h);
            *reinterpret_cast<uint2*>(dpl + pl_stride) = __builtin_bit_cast(uint2, m);
            *reinterpret_cast<uint2*>(dpl + 2 * pl_stride) = __builtin_bit_cast(uint2, lo);
          }
        }
      }
    }
  }
  // block reduction of the per-lane column partials: slab j holds chunks [LPR j, LPR (j + 1)), the
  // RPW row groups of a wave hold the same columns
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    if (LPR * j >= nch) break;
#pragma unroll
    for (int e = 0; e < N; ++e) {
      red[wave][0][lane * N + e] = pg[j][e];
      red[wave][1][lane * N + e] = pb[j][e];
    }
    __syncthreads();
    for (int cl = threadIdx.x; cl < LPR * N; cl += 256) {
      const int col = LPR * N * j + cl;
      if (col < width) {
        float sg = 0.f, sb = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
          for (int r = 0; r < RPW; ++r) {
            sg += red[w][0][r * LPR * N + cl];
            sb += red[w][1][r * LPR * N + cl];
          }
        part[((int64_t)blockIdx.x * 2 + 0) * width + col] = sg;
        part[((int64_t)blockIdx.x * 2 + 1) * width + col] = sb;
      }
    }
    __syncthreads();
  }
}

// narrow rows (width / elements-per-16B <= LPR): 64 / LPR rows per wave, one 16-B chunk per lane;
// gamma/beta partials of a column chunk are summed over the waves AND the row groups of the block
template <typename T, int LPR>
__global__ void __launch_bounds__(256) ln_bwd16_narrow_kernel(int64_t rows, int width, const T* __restrict__ dy,
                                                              int64_t lddy, const T* __restrict__ x, int64_t ldx,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd, T* __restrict__ dx,
                                                              int64_t lddx, const T* __restrict__ dx_add, int64_t ldadd,
                                                              T* __restrict__ dx_drop, float p, uint32_t thr,
                                                              const uint64_t* __restrict__ seedp, uint64_t salt,
                                                              float* __restrict__ part) {
  constexpr int N = VN<T>::N, RPW = 64 / LPR;
  __shared__ float red[4][2][64 * N];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l = lane % LPR, sub = lane / LPR;
  const int nch = width / N;
  const bool on = l < nch;
  const uint64_t seed = (dx_drop && p > 0.f) ? *seedp : 0ull;
  const float keep = 1.0f / (1.0f - p);
  float pg[N], pb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) { pg[e] = 0.f; pb[e] = 0.f; }
  for (int64_t row = ((int64_t)blockIdx.x * 4 + wave) * RPW + sub; row < rows; row += (int64_t)gridDim.x * 4 * RPW) {
    const float mu = mean[row], rs = rstd[row];
    float xh[N], g[N], add[N];
    float s1 = 0.f, s2 = 0.f;
    if (on) {
      float d[N], gv[N];
      VN<T>::load(dy + row * lddy + N * l, d);
      VN<T>::load(x + row * ldx + N * l, xh);
      if (dx_add) VN<T>::load(dx_add + row * ldadd + N * l, add);
      load_f32xN<T>(gamma + N * l, gv);
#pragma unroll
      for (int e = 0; e < N; ++e) {
        xh[e] = (xh[e] - mu) * rs;
        g[e] = d[e] * gv[e];
        s1 += g[e];
        s2 += g[e] * xh[e];
        pg[e] += d[e] * xh[e];
        pb[e] += d[e];
      }
    }
    const float c1 = group_sum<LPR>(s1) / (float)width;
    const float c2 = group_sum<LPR>(s2) / (float)width;
    if (on) {
      float o[N];
#pragma unroll
      for (int e = 0; e < N; ++e) o[e] = rs * (g[e] - c1 - xh[e] * c2) + (dx_add ? add[e] : 0.f);
      VN<T>::store(dx + row * lddx + N * l, o);
      if (dx_drop) {
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const uint32_t h = mmfd_hash(seed, salt, (uint64_t)row * (uint64_t)width + N * l + e);
          o[e] = (p > 0.f && h < thr) ? 0.f : o[e] * (p > 0.f ? keep : 1.f);
        }
        VN<T>::store(dx_drop + row * lddx + N * l, o);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < N; ++e) {
    red[wave][0][lane * N + e] = pg[e];
    red[wave][1][lane * N + e] = pb[e];
  }
  __syncthreads();
  for (int col = threadIdx.x; col < width; col += 256) {  // col = chunk * N + e, chunk < LPR
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        sg += red[w][0][r * LPR * N + col];
        sb += red[w][1][r * LPR * N + col];
      }
    part[((int64_t)blockIdx.x * 2 + 0) * width + col] = sg;
    part[((int64_t)blockIdx.x * 2 + 1) * width + col] = sb;
  }
}

}  // namespace

extern "C" int mmfd_layernorm_fwd(int dtype, int64_t rows, int64_t width, const void* x, int64_t ldx,
                                  const float* gamma, const float* beta, float eps, void* y, int64_t ldy,
                                  float* mean, float* rstd, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(width > 0 && width <= 1024 && width % 4 == 0, "layernorm: width %lld unsupported", (long long)width);
  MMFD_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0, "layernorm: leading dims must be multiples of 4");
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  const int epc = dtype == MMFD_BF16 ? 8 : 4;
  const bool v16 = width % epc == 0 && ldx % epc == 0 && ldy % epc == 0 && ((uintptr_t)x & 15) == 0 &&
                   ((uintptr_t)y & 15) == 0 && ((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0;
  if (v16) {
    if (dtype == MMFD_BF16 ? launch_ln_narrow<bf16>(s, rows, (int)width, (const bf16*)x, ldx, gamma, beta, eps, (bf16*)y,
                                                    ldy, mean, rstd, nullptr, 0)
                           : launch_ln_narrow<float>(s, rows, (int)width, (const float*)x, ldx, gamma, beta, eps,
                                                     (float*)y, ldy, mean, rstd, nullptr, 0)) {
    } else if (dtype == MMFD_BF16)
      launch_ln_fwd16<bf16>(s, rows, (int)width, (const bf16*)x, ldx, gamma, beta, eps, (bf16*)y, ldy, mean, rstd);
    else
      launch_ln_fwd16<float>(s, rows, (int)width, (const float*)x, ldx, gamma, beta, eps, (float*)y, ldy, mean, rstd);
  } else if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((ln_fwd_kernel<bf16>), grid, dim3(256), 0, s, rows, (int)width, (const bf16*)x, ldx, gamma, beta, eps, (bf16*)y, ldy, mean, rstd);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<float>), grid, dim3(256), 0, s, rows, (int)width, (const float*)x, ldx, gamma, beta, eps, (float*)y, ldy, mean, rstd);
  MMFD_CHECK_LAUNCH("layernorm_fwd");
  return 0;
}

extern "C" int mmfd_layernorm_fwd_split(int64_t rows, int64_t width, const float* x, int64_t ldx, const float* gamma,
                                        const float* beta, float eps, float* y, int64_t ldy, float* mean, float* rstd,
                                        void* planes, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(width > 0 && width <= 1024 && width % 8 == 0, "layernorm_fwd_split: width %lld unsupported",
                 (long long)width);
  MMFD_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
                     ((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0 && ((uintptr_t)planes & 15) == 0,
                 "layernorm_fwd_split: 16-B aligned rows required");
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  launch_ln_fwd16<float>(s, rows, (int)width, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, (const float*)nullptr,
                         (int64_t)0, (bf16*)planes, rows * width);
  MMFD_CHECK_LAUNCH("layernorm_fwd_split");
  return 0;
}

extern "C" int mmfd_layernorm_fwd_res(int dtype, int64_t rows, int64_t width, const void* x, int64_t ldx,
                                      const float* gamma, const float* beta, float eps, const void* res,
                                      int64_t ldr, void* y, int64_t ldy, float* mean, float* rstd,
                                      mmfd_stream_t stream) {
  const int epc = dtype == MMFD_BF16 ? 8 : 4;
  MMFD_CHECK_ARG(width > 0 && width <= 1024 && width % epc == 0, "layernorm_res: width %lld unsupported", (long long)width);
  MMFD_CHECK_ARG(ldx % epc == 0 && ldy % epc == 0 && ldr % epc == 0 && ((uintptr_t)x & 15) == 0 &&
                     ((uintptr_t)y & 15) == 0 && ((uintptr_t)res & 15) == 0 && ((uintptr_t)gamma & 15) == 0 &&
                     ((uintptr_t)beta & 15) == 0,
                 "layernorm_res: 16-B aligned rows required");
  MMFD_CHECK_ARG((mean == nullptr) == (rstd == nullptr), "layernorm_res: mean and rstd both or neither");
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == MMFD_BF16 ? launch_ln_narrow<bf16>(s, rows, (int)width, (const bf16*)x, ldx, gamma, beta, eps, (bf16*)y,
                                                  ldy, mean, rstd, (const bf16*)res, ldr)
                         : launch_ln_narrow<float>(s, rows, (int)width, (const float*)x, ldx, gamma, beta, eps,
                                                   (float*)y, ldy, mean, rstd, (const float*)res, ldr)) {
  } else if (dtype == MMFD_BF16)
    launch_ln_fwd16<bf16>(s, rows, (int)width, (const bf16*)x, ldx, gamma, beta, eps, (bf16*)y, ldy, mean, rstd,
                          (const bf16*)res, ldr);
  else
    launch_ln_fwd16<float>(s, rows, (int)width, (const float*)x, ldx, gamma, beta, eps, (float*)y, ldy, mean, rstd,
                           (const float*)res, ldr);
  MMFD_CHECK_LAUNCH("layernorm_fwd_res");
  return 0;
}

namespace {
int layernorm_bwd_impl(int dtype, int64_t rows, int64_t width, const void* dy, int64_t lddy,
                       const void* x, int64_t ldx, const float* gamma, const float* mean,
                       const float* rstd, void* dx, int64_t lddx, const void* dx_add, int64_t ldadd,
                       float* dgamma, float* dbeta, float beta_acc, void* dx_drop,
                       float dropout_p, const uint64_t* seed, uint64_t salt,
                       void* workspace, int64_t workspace_bytes, mmfd_stream_t stream, bf16* planes);
}  // namespace

extern "C" int mmfd_layernorm_bwd(int dtype, int64_t rows, int64_t width, const void* dy, int64_t lddy,
                                  const void* x, int64_t ldx, const float* gamma, const float* mean,
                                  const float* rstd, void* dx, int64_t lddx, const void* dx_add, int64_t ldadd,
                                  float* dgamma, float* dbeta, float beta_acc, void* dx_drop,
                                  float dropout_p, const uint64_t* seed, uint64_t salt,
                                  void* workspace, int64_t workspace_bytes, mmfd_stream_t stream) {
  return layernorm_bwd_impl(dtype, rows, width, dy, lddy, x, ldx, gamma, mean, rstd, dx, lddx, dx_add, ldadd, dgamma,
                            dbeta, beta_acc, dx_drop, dropout_p, seed, salt, workspace, workspace_bytes, stream,
                            nullptr);
}

extern "C" int mmfd_layernorm_bwd_split(int64_t rows, int64_t width, const float* dy, int64_t lddy, const float* x,
                                        int64_t ldx, const float* gamma, const float* mean, const float* rstd,
                                        float* dx, int64_t lddx, const float* dx_add, int64_t ldadd, float* dgamma,
                                        float* dbeta, float beta_acc, float* dx_drop, float dropout_p,
                                        const uint64_t* seed, uint64_t salt, void* workspace,
                                        int64_t workspace_bytes, void* planes, mmfd_stream_t stream) {
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  MMFD_CHECK_ARG(width % 8 == 0 && width / 4 > 32 && width <= 1024 && lddy % 4 == 0 && ldx % 4 == 0 &&
                     lddx % 4 == 0 && (!dx_add || (ldadd % 4 == 0 && al(dx_add))) && al(dy) && al(x) && al(dx) &&
                     al(gamma) && (!dx_drop || al(dx_drop)) && al(planes),
                 "layernorm_bwd_split: fp32 rows of 132..1024 (multiple of 8) elements, 16-B aligned");
  return layernorm_bwd_impl(MMFD_F32, rows, width, dy, lddy, x, ldx, gamma, mean, rstd, dx, lddx, dx_add, ldadd,
                            dgamma, dbeta, beta_acc, dx_drop, dropout_p, seed, salt, workspace, workspace_bytes, stream,
                            (bf16*)planes);
}

namespace {
// LayerNorm gamma / beta gradients from the backward kernels' per-block partials ([nparts][2][width],
// gamma at +0, beta at +width): one launch for both; a block owns 16 of the 2*width columns and its
// 64 part groups of 16 lanes stride over the partials (8 independent loads in flight per lane), the
// groups combined through LDS in a fixed order (deterministic). Against two launches of 64-column
// blocks (12 + 12 workgroups at width 768, each lane walking 128 partials): all CUs, 4x shorter chains.
__global__ void __launch_bounds__(1024) ln_gb_reduce_kernel(const float* __restrict__ part, int nparts, int64_t width,
                                                            float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                            float beta) {
  __shared__ float red[64][17];
  const int c = threadIdx.x & 15, pg = threadIdx.x >> 4;
  const int64_t col = (int64_t)blockIdx.x * 16 + c;  // in [0, 2 * width)
  const int64_t stride = 2 * width;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < stride) {
    int p = pg;
    for (; p + 7 * 64 < nparts; p += 8 * 64) {
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += part[(int64_t)(p + u * 64) * stride + col];
    }
    for (; p < nparts; p += 64) s[0] += part[(int64_t)p * stride + col];
  }
  red[pg][c] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (pg == 0 && col < stride) {
    float tot = 0.f;
#pragma unroll 8
    for (int w = 0; w < 64; ++w) tot += red[w][c];
    float* out = col < width ? (dgamma ? dgamma + col : nullptr) : (dbeta ? dbeta + (col - width) : nullptr);
    if (out) *out = (beta != 0.f ? beta * *out : 0.f) + tot;
  }
}
}  // namespace


namespace {
// backward blocks (A/B: env MMFD_LN_BWD_BLOCKS, read once at load)
const int g_ln_bwd_blocks = [] {
  const char* v = getenv("MMFD_LN_BWD_BLOCKS");
  const int n = v ? atoi(v) : 0;
  return n > 0 ? n : 512;
}();

int layernorm_bwd_impl(int dtype, int64_t rows, int64_t width, const void* dy, int64_t lddy,
                       const void* x, int64_t ldx, const float* gamma, const float* mean,
                       const float* rstd, void* dx, int64_t lddx, const void* dx_add, int64_t ldadd,
                       float* dgamma, float* dbeta, float beta_acc, void* dx_drop,
                       float dropout_p, const uint64_t* seed, uint64_t salt,
                       void* workspace, int64_t workspace_bytes, mmfd_stream_t stream, bf16* planes) {
  MMFD_CHECK_ARG(width > 0 && width <= 1024 && width % 4 == 0, "layernorm_bwd: width %lld unsupported", (long long)width);
  MMFD_CHECK_ARG(!(dx_drop && dropout_p > 0.f) || seed, "layernorm_bwd: dropout needs seed");
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  // backward grid: the kernels walk rows with a grid stride, so every resident block is busy with
  // g_ln_bwd_blocks of them (2 per CU at their register counts); each block leaves one gamma / beta
  // partial row, which ln_gb_reduce_kernel then sums — more blocks only add partials
  int nblocks = (int)std::min<int64_t>((rows + 3) / 4, g_ln_bwd_blocks);
  const int64_t per = 2 * width * 4;
  if (workspace_bytes < nblocks * per) nblocks = (int)(workspace_bytes / per);
  MMFD_CHECK_ARG(nblocks >= 1 && workspace, "layernorm_bwd: workspace too small");
  const float p = dropout_p > 0.f ? dropout_p : 0.f;
  const uint32_t thr = mmfd_drop_threshold(p);
  const int epc = dtype == MMFD_BF16 ? 8 : 4;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  const bool v16 = width % epc == 0 && lddy % epc == 0 && ldx % epc == 0 && lddx % epc == 0 &&
                   (!dx_add || (ldadd % epc == 0 && al(dx_add))) && al(dy) && al(x) && al(dx) && al(gamma) &&
                   (!dx_drop || al(dx_drop));
  const int nch16 = (int)(width / epc);
  if (v16 && nch16 <= 32) {
    // narrow rows: RPW rows per wave, so a block covers 4 * RPW rows
    const int rpb = nch16 <= 16 ? 16 : 8;
    nblocks = (int)std::min<int64_t>((rows + rpb - 1) / rpb, g_ln_bwd_blocks);
    if (workspace_bytes < nblocks * per) nblocks = (int)(workspace_bytes / per);
#define LNB(T, LPR) hipLaunchKernelGGL((ln_bwd16_narrow_kernel<T, LPR>), dim3(nblocks), dim3(256), 0, s, rows, (int)width, \
                                       (const T*)dy, lddy, (const T*)x, ldx, gamma, mean, rstd, (T*)dx, lddx,             \
                                       (const T*)dx_add, ldadd, (T*)dx_drop, p, thr, seed, salt, (float*)workspace)
    if (dtype == MMFD_BF16) {
      if (nch16 <= 16) LNB(bf16, 16); else LNB(bf16, 32);
    } else {
      if (nch16 <= 16) LNB(float, 16); else LNB(float, 32);
    }
#undef LNB
  } else if (v16 && nch16 <= (dtype == MMFD_BF16 ? 128 : 64)) {
    // two rows per wave (ln_fwd16_kernel's comment)
    nblocks = (int)std::min<int64_t>((rows + 7) / 8, g_ln_bwd_blocks);
    if (workspace_bytes < nblocks * per) nblocks = (int)(workspace_bytes / per);
#define LNB2(T, CH) hipLaunchKernelGGL((ln_bwd16_kernel<T, 32, CH>), dim3(nblocks), dim3(256), 0, s, rows, (int)width, \
                                       (const T*)dy, lddy, (const T*)x, ldx, gamma, mean, rstd, (T*)dx, lddx,          \
                                       (const T*)dx_add, ldadd, (T*)dx_drop, p, thr, seed, salt, (float*)workspace,    \
                                       planes, rows * width)
    if (dtype == MMFD_F32) LNB2(float, 2);
    else if (nch16 <= 96) LNB2(bf16, 3);
    else LNB2(bf16, 4);
#undef LNB2
  } else if (v16) {
    if (dtype == MMFD_BF16)
      hipLaunchKernelGGL((ln_bwd16_kernel<bf16, 64, 2>), dim3(nblocks), dim3(256), 0, s, rows, (int)width,
                         (const bf16*)dy, lddy, (const bf16*)x, ldx, gamma, mean, rstd, (bf16*)dx, lddx,
                         (const bf16*)dx_add, ldadd, (bf16*)dx_drop, p, thr, seed, salt, (float*)workspace);
    else
      hipLaunchKernelGGL((ln_bwd16_kernel<float, 64, 4, false>), dim3(nblocks), dim3(256), 0, s, rows, (int)width,
                         (const float*)dy, lddy, (const float*)x, ldx, gamma, mean, rstd, (float*)dx, lddx,
                         (const float*)dx_add, ldadd, (float*)dx_drop, p, thr, seed, salt, (float*)workspace, planes,
                         rows * width);
  } else if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((ln_bwd_kernel<bf16>), dim3(nblocks), dim3(256), 0, s, rows, (int)width, (const bf16*)dy, lddy,
                       (const bf16*)x, ldx, gamma, mean, rstd, (bf16*)dx, lddx, (const bf16*)dx_add, ldadd, (bf16*)dx_drop,
                       p, thr, seed, salt, (float*)workspace);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<float>), dim3(nblocks), dim3(256), 0, s, rows, (int)width, (const float*)dy, lddy,
                       (const float*)x, ldx, gamma, mean, rstd, (float*)dx, lddx, (const float*)dx_add, ldadd,
                       (float*)dx_drop, p, thr, seed, salt, (float*)workspace);
  // part layout [block][2][width]: gamma partials at offset 0, beta partials at +width, stride 2*width;
  // both reduced by one launch of 16-column blocks (2*width / 16 of them)
  if (dgamma || dbeta)
    hipLaunchKernelGGL(ln_gb_reduce_kernel, dim3((unsigned)((2 * width + 15) / 16)), dim3(1024), 0, s,
                       (const float*)workspace, nblocks, width, dgamma, dbeta, beta_acc);
  MMFD_CHECK_LAUNCH("layernorm_bwd");
  return 0;
}
}  // namespace
