// Library plumbing (error strings, version, dropout hash) and small elementwise kernels.
#include "common.h"
#include <stdarg.h>
#include <stdio.h>
#include <algorithm>

static thread_local char g_err[512] = "no error";

int mmfd_set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code == 0 ? MMFD_ERR_INVALID : code;
}

extern "C" const char* mmfd_last_error_string(void) { return g_err; }
extern "C" int mmfd_version(void) { return MMFD_ABI_VERSION; }
extern "C" uint32_t mmfd_dropout_hash(uint64_t seed, uint64_t salt, uint64_t index) {
  return mmfd_hash(seed, salt, index);
}

namespace {

inline int grid_for(int64_t n, int per_block) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + per_block - 1) / per_block, 8192));
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = from_f32<TO>(to_f32(in[i]));
}

// vectorised fp32 -> bf16 (8 elements per thread-iteration)
__global__ void cast_f32_bf16_vec(const float4* __restrict__ in, uint4* __restrict__ out, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 a = in[2 * i], b = in[2 * i + 1];
    bf16x8 v = {(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w, (bf16)b.x, (bf16)b.y, (bf16)b.z, (bf16)b.w};
    out[i] = __builtin_bit_cast(uint4, v);
  }
}

__global__ void zero_kernel(uint4* __restrict__ v, int64_t n16, unsigned char* __restrict__ tail, int64_t ntail) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) v[i] = make_uint4(0, 0, 0, 0);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ntail; i += stride) tail[i] = 0;
}

template <typename T>
__global__ void axpby_kernel(int64_t n, float a, const T* __restrict__ x, float b, const T* __restrict__ y,
                             T* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = a * to_f32(x[i]);
    if (y) v += b * to_f32(y[i]);
    out[i] = from_f32<T>(v);
  }
}

template <typename T>
__global__ void dropout_kernel(int64_t n, const T* __restrict__ x, T* __restrict__ out, float p, uint32_t thr,
                               const uint64_t* __restrict__ seedp, uint64_t salt) {
  const uint64_t seed = *seedp;
  const float sc = 1.0f / (1.0f - p);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h = mmfd_hash(seed, salt, (uint64_t)i);
    out[i] = from_f32<T>(h < thr ? 0.0f : to_f32(x[i]) * sc);
  }
}

__global__ void seed_advance_kernel(uint64_t* seed) { seed[0] += 1; }

template <typename T>
__global__ void act_bwd_kernel(int64_t n, int64_t width, const T* __restrict__ dy, const T* __restrict__ aux, int act,
                               float p, uint32_t thr, const uint64_t* __restrict__ seedp, uint64_t salt, T* __restrict__ out) {
  const uint64_t seed = p > 0.f ? *seedp : 0ull;
  const float sc = 1.0f / (1.0f - p);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float z = to_f32(dy[i]);
    if (p > 0.f) z = (mmfd_hash(seed, salt, (uint64_t)i) < thr) ? 0.f : z * sc;
    const float a = to_f32(aux[i]);
    if (act == MMFD_ACT_GELU) z *= gelu_grad_f(a);
    else if (act == MMFD_ACT_RELU) z = a > 0.f ? z : 0.f;
    out[i] = from_f32<T>(z);
  }
}

}  // namespace

// out[c][r] = in[r][c] for 2- or 4-byte elements: 64x64 tiles through LDS (one padding column:
// conflict-free column reads), 256 threads, every global access a coalesced row segment
template <typename T>
__global__ void __launch_bounds__(256) transpose_kernel(int64_t rows, int64_t cols, const T* __restrict__ in,
                                                        int64_t ldi, T* __restrict__ out, int64_t ldo) {
  __shared__ T tile[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t r = r0 + ty + 4 * k, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + 4 * k][tx] = in[r * ldi + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t c = c0 + ty + 4 * k, r = r0 + tx;
    if (c < cols && r < rows) out[c * ldo + r] = tile[tx][ty + 4 * k];
  }
}

extern "C" int mmfd_transpose(int dtype, int64_t rows, int64_t cols, const void* in, int64_t ldi, void* out, int64_t ldo,
                              mmfd_stream_t stream) {
  MMFD_CHECK_ARG(dtype == MMFD_F32 || dtype == MMFD_BF16, "mmfd_transpose: dtype %d", dtype);
  MMFD_CHECK_ARG(rows >= 0 && cols >= 0 && ldi >= cols && ldo >= rows, "mmfd_transpose: bad shape / leading dims");
  if (rows == 0 || cols == 0) return 0;
  MMFD_CHECK_ARG(in && out && in != out, "mmfd_transpose: null or aliased pointers");
  MMFD_CHECK_ARG((rows + 63) / 64 < 65536, "mmfd_transpose: too many rows");
  const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL(transpose_kernel<bf16>, grid, dim3(256), 0, s, rows, cols, (const bf16*)in, ldi, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, s, rows, cols, (const float*)in, ldi, (float*)out, ldo);
  MMFD_CHECK_LAUNCH("transpose");
  return 0;
}

extern "C" int mmfd_cast(int dtype_in, int dtype_out, int64_t n, const void* in, void* out, mmfd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  MMFD_CHECK_ARG(in && out, "mmfd_cast: null pointer");
  if (dtype_in == MMFD_F32 && dtype_out == MMFD_BF16 && (n % 8) == 0 && ((uintptr_t)in & 15) == 0 &&
      ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(cast_f32_bf16_vec, dim3(grid_for(n / 8, 256)), dim3(256), 0, s, (const float4*)in, (uint4*)out, n / 8);
  } else if (dtype_in == MMFD_F32 && dtype_out == MMFD_BF16) {
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, (const float*)in, (bf16*)out, n);
  } else if (dtype_in == MMFD_BF16 && dtype_out == MMFD_F32) {
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(grid_for(n, 256)), dim3(256), 0, s, (const bf16*)in, (float*)out, n);
  } else if (dtype_in == MMFD_F32 && dtype_out == MMFD_F32) {
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(grid_for(n, 256)), dim3(256), 0, s, (const float*)in, (float*)out, n);
  } else if (dtype_in == MMFD_BF16 && dtype_out == MMFD_BF16) {
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, (const bf16*)in, (bf16*)out, n);
  } else {
    return mmfd_set_error(MMFD_ERR_INVALID, "mmfd_cast: bad dtypes %d->%d", dtype_in, dtype_out);
  }
  MMFD_CHECK_LAUNCH("cast");
  return 0;
}

extern "C" int mmfd_zero(void* dst, int64_t bytes, mmfd_stream_t stream) {
  if (bytes == 0) return 0;
  MMFD_CHECK_ARG(dst != nullptr && bytes > 0, "mmfd_zero: bad buffer");
  // a kernel, not hipMemsetAsync: identical inside captured HIP graphs and eager streams
  const int64_t n16 = ((uintptr_t)dst & 15) == 0 ? bytes / 16 : 0;
  hipLaunchKernelGGL(zero_kernel, dim3(grid_for(std::max<int64_t>(n16, 1), 256)), dim3(256), 0, (hipStream_t)stream,
                     (uint4*)dst, n16, (unsigned char*)dst + n16 * 16, bytes - n16 * 16);
  MMFD_CHECK_LAUNCH("zero");
  return 0;
}

extern "C" int mmfd_axpby(int dtype, int64_t n, float a, const void* x, float b, const void* y, void* out,
                          mmfd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((axpby_kernel<bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, n, a, (const bf16*)x, b, (const bf16*)y, (bf16*)out);
  else if (dtype == MMFD_F32)
    hipLaunchKernelGGL((axpby_kernel<float>), dim3(grid_for(n, 256)), dim3(256), 0, s, n, a, (const float*)x, b, (const float*)y, (float*)out);
  else return mmfd_set_error(MMFD_ERR_INVALID, "mmfd_axpby: bad dtype");
  MMFD_CHECK_LAUNCH("axpby");
  return 0;
}

extern "C" int mmfd_dropout(int dtype, int64_t n, const void* x, void* out, float p, const uint64_t* seed,
                            uint64_t salt, mmfd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  MMFD_CHECK_ARG(p >= 0.f && p < 1.f && seed, "mmfd_dropout: bad p/seed");
  if (n == 0) return 0;
  const uint32_t thr = mmfd_drop_threshold(p);
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((dropout_kernel<bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, n, (const bf16*)x, (bf16*)out, p, thr, seed, salt);
  else
    hipLaunchKernelGGL((dropout_kernel<float>), dim3(grid_for(n, 256)), dim3(256), 0, s, n, (const float*)x, (float*)out, p, thr, seed, salt);
  MMFD_CHECK_LAUNCH("dropout");
  return 0;
}

extern "C" int mmfd_act_bwd(int dtype, int64_t n, const void* dy, const void* aux, int act, float dropout_p,
                            const uint64_t* seed, uint64_t salt, void* out, mmfd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  MMFD_CHECK_ARG(act == MMFD_ACT_GELU || act == MMFD_ACT_RELU || act == MMFD_ACT_NONE, "act_bwd: bad act");
  MMFD_CHECK_ARG(dropout_p <= 0.f || seed, "act_bwd: dropout needs seed");
  if (n == 0) return 0;
  const float p = dropout_p > 0.f ? dropout_p : 0.f;
  const uint32_t thr = mmfd_drop_threshold(p);
  if (dtype == MMFD_BF16)
    hipLaunchKernelGGL((act_bwd_kernel<bf16>), dim3(grid_for(n, 256)), dim3(256), 0, s, n, (int64_t)0, (const bf16*)dy,
                       (const bf16*)aux, act, p, thr, seed, salt, (bf16*)out);
  else
    hipLaunchKernelGGL((act_bwd_kernel<float>), dim3(grid_for(n, 256)), dim3(256), 0, s, n, (int64_t)0, (const float*)dy,
                       (const float*)aux, act, p, thr, seed, salt, (float*)out);
  MMFD_CHECK_LAUNCH("act_bwd");
  return 0;
}

extern "C" int mmfd_seed_advance(uint64_t* seed, mmfd_stream_t stream) {
  hipLaunchKernelGGL(seed_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, seed);
  MMFD_CHECK_LAUNCH("seed_advance");
  return 0;
}
