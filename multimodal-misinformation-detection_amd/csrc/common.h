// Shared device helpers for the mmfd HIP kernels (gfx950 / CDNA4 only).
//
// Storage types: fp32 (`float`) and bf16 (`__bf16`). All arithmetic accumulates in fp32.
// MFMA fragments are always moved as 16-byte chunks: one chunk = 8 bf16 or 4 fp32 elements,
// which is exactly one lane's operand for v_mfma_f32_16x16x32_bf16, or four consecutive k-steps
// of v_mfma_f32_16x16x4_f32 (see mma16 below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/mmfd.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(2))) short i16x2;

#define MMFD_LDS __attribute__((address_space(3)))

// ---------------------------------------------------------------------------------------------
// error reporting (host side, implemented in runtime.hip)
// ---------------------------------------------------------------------------------------------
int mmfd_set_error(int code, const char* fmt, ...);
#define MMFD_CHECK_ARG(cond, ...)                                              \
  do {                                                                         \
    if (!(cond)) return mmfd_set_error(MMFD_ERR_INVALID, __VA_ARGS__);        \
  } while (0)
// ABI guard of the argument structs (include/mmfd.h struct_size): a caller compiled against another
// layout passes another size and is refused before any field is read
#define MMFD_CHECK_STRUCT(p, type, what)                                                              \
  do {                                                                                               \
    if ((p) == nullptr) return mmfd_set_error(MMFD_ERR_INVALID, "%s: NULL arguments", what);        \
    if ((p)->struct_size != (int64_t)sizeof(type))                                                   \
      return mmfd_set_error(MMFD_ERR_INVALID,                                                        \
                            "%s: " #type ".struct_size = %lld, this library expects %lld (ABI version " \
                            "%d): rebuild the caller against this include/mmfd.h",                    \
                            what, (long long)(p)->struct_size, (long long)sizeof(type), MMFD_ABI_VERSION); \
  } while (0)
#define MMFD_CHECK_LAUNCH(name)                                                \
  do {                                                                         \
    hipError_t e__ = hipGetLastError();                                        \
    if (e__ != hipSuccess)                                                     \
      return mmfd_set_error((int)e__, "%s: launch failed: %s", name,          \
                            hipGetErrorString(e__));                           \
  } while (0)

// ---------------------------------------------------------------------------------------------
// scalar conversions
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

template <typename T> struct elem_traits;
template <> struct elem_traits<float> { static constexpr int per16 = 4; static constexpr int code = MMFD_F32; };
template <> struct elem_traits<bf16>  { static constexpr int per16 = 8; static constexpr int code = MMFD_BF16; };

// ---------------------------------------------------------------------------------------------
// activations (exact erf GELU as nn.GELU() / HF "gelu")
// ---------------------------------------------------------------------------------------------
// erf(z) by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7), branch-free: one v_rcp_f32, one
// v_exp_f32 and five FMAs (the libm erff is ~35 instructions with a divergent branch; the
// correctly rounded __frcp_rn / denormal-safe exp2f sequences cost ~10 more each). The hardware
// rcp (1 ulp) and exp2 (flushes results below 2^-126, where the erf tail is exactly 1 in fp32)
// stay inside the A&S bound. e = exp(-z*z) is returned too: GELU's derivative needs
// exp(-x*x/2) = exp(-z*z) for z = x/sqrt(2).
__device__ __forceinline__ float erf_fast(float z, float& e) {
  const float a = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  e = __builtin_amdgcn_exp2f(-a * a * 1.4426950408889634f);
  return copysignf(fmaf(-poly, e, 1.0f), z);
}
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f, e));
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float e;
  const float cdf = 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f, e));
  return fmaf(x * 0.39894228040143268f, e, cdf);
}

// GELU and its derivative from one erf evaluation (MMFD_ACT_GELU_D): the operations of gelu_f and
// gelu_grad_f, so both values are bit-identical to theirs — the backward's x gelu'(pre) becomes a
// multiply by the saved derivative (MMFD_ACT_MUL_AUX) with the same fp32 result
__device__ __forceinline__ float gelu_and_grad_f(float x, float& d) {
  float e;
  const float r = erf_fast(x * 0.70710678118654752f, e);
  d = fmaf(x * 0.39894228040143268f, e, 0.5f * (1.0f + r));
  return 0.5f * x * (1.0f + r);
}

// forward-only epilogue activations past ReLU (MMFD_ACT_TANH / MMFD_ACT_SIGMOID)
__device__ __forceinline__ float act_tail_f(int act, float z) {
  return act == MMFD_ACT_TANH ? tanhf(z) : 1.0f / (1.0f + expf(-z));
}

// ---------------------------------------------------------------------------------------------
// counter-based dropout RNG: keep(element) is a pure function of (seed, salt, index), so the
// backward pass regenerates the forward mask and the CPU oracle can reproduce it bit-for-bit.
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t mmfd_mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
// per-call key from (seed, salt): loop invariant, hoisted out of every element loop
__host__ __device__ __forceinline__ uint32_t mmfd_hash_key(uint64_t seed, uint64_t salt) {
  const uint32_t k0 = mmfd_mix32((uint32_t)seed ^ mmfd_mix32((uint32_t)(seed >> 32) ^ 0x85ebca6bu));
  return mmfd_mix32(k0 ^ (uint32_t)salt ^ mmfd_mix32((uint32_t)(salt >> 32) ^ 0xc2b2ae35u));
}
// one mix round per element: the index enters through odd multipliers (a bijection of the low
// word for a fixed high word)
__host__ __device__ __forceinline__ uint32_t mmfd_hash_k(uint32_t key, uint64_t idx) {
  return mmfd_mix32(key ^ ((uint32_t)idx * 0x9e3779b1u) ^ ((uint32_t)(idx >> 32) * 0x85ebca77u));
}
__host__ __device__ __forceinline__ uint32_t mmfd_hash(uint64_t seed, uint64_t salt, uint64_t idx) {
  return mmfd_hash_k(mmfd_hash_key(seed, salt), idx);
}
// 16-bit threshold of the attention kernels' pair hashes (attention.hip pair_keep): keep <=> the
// element's 16-bit half >= thr16 = round(p * 65536); 65536 drops everything
__host__ __device__ __forceinline__ uint32_t mmfd_drop_threshold16(float p) {
  const double t = (double)p * 65536.0 + 0.5;
  return t >= 65536.0 ? 65536u : (uint32_t)t;
}
// threshold so that keep <=> hash >= thr, i.e. P(drop) = p
__host__ __device__ __forceinline__ uint32_t mmfd_drop_threshold(float p) {
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) return 0xffffffffu;
  return (uint32_t)t;
}

// ---------------------------------------------------------------------------------------------
// wave reductions (wave64)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------------------------
// 16x16 MFMA over one 16-byte-per-lane chunk of K.
//   bf16: one v_mfma_f32_16x16x32_bf16; lane l holds k = 8*(l>>4) .. +7 of the 32-wide chunk.
//   fp32: four v_mfma_f32_16x16x4_f32; lane l holds k = 4*(l>>4) .. +3 of a 16-wide chunk, and
//         step s consumes element s (a consistent permutation of k on both operands).
// Accumulator layout (both): col = l & 15, row = 4*(l>>4) + r, r = 0..3.
// ---------------------------------------------------------------------------------------------
template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int KC = 32;  // k per chunk
  __device__ __forceinline__ static void run(f32x4& acc, const uint4& a, const uint4& b) {
    bf16x8 av = __builtin_bit_cast(bf16x8, a);
    bf16x8 bv = __builtin_bit_cast(bf16x8, b);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
  // N independent accumulators, one chunk each
  template <int N>
  __device__ __forceinline__ static void runN(f32x4* acc, const uint4* a, const uint4* b) {
#pragma unroll
    for (int i = 0; i < N; ++i) run(acc[i], a[i], b[i]);
  }
};
template <> struct Mma<float> {
  static constexpr int KC = 16;
  __device__ __forceinline__ static void run(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
  // N independent accumulators with their k-steps interleaved: back to back, one chain's 16x16x4
  // MFMAs would wait out the 40-cycle dependent latency instead of the 32-cycle issue
  template <int N>
  __device__ __forceinline__ static void runN(f32x4* acc, const uint4* a, const uint4* b) {
#pragma unroll
    for (int i = 0; i < N; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].x), __uint_as_float(b[i].x), acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < N; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].y), __uint_as_float(b[i].y), acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < N; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].z), __uint_as_float(b[i].z), acc[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < N; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i].w), __uint_as_float(b[i].w), acc[i], 0, 0, 0);
  }
};

__device__ __forceinline__ uint4 lds_read16(const char* base, int byte_off) {
  return *reinterpret_cast<const uint4*>(base + byte_off);
}

// transposed 4x16 read (gfx950 ds_read_b64_tr_b16): lane 4q+p of each 16-lane group gives the
// address of row q, columns 4p..4p+3; lane i receives column i of the 4 rows.
__device__ __forceinline__ uint2 lds_read_tr16(const char* addr) {
  i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((MMFD_LDS i16x4*)(addr));
  return __builtin_bit_cast(uint2, v);
}

// shared deterministic reduction of per-block column partials (gemm.hip)
__global__ void mmfd_reduce_partials_kernel(const float* __restrict__ part, int nparts, int64_t stride, int64_t N,
                                            float* __restrict__ out, float beta);

__device__ __forceinline__ int xcd_remap(int id, int total) {
  // blocks are dealt round-robin over the 8 XCDs; give each XCD a contiguous run of tiles
  // (bijective for any total, speed only).
  const int xcd = id & 7, local = id >> 3;
  const int q = total >> 3, r = total & 7;
  const int start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + local;
}
