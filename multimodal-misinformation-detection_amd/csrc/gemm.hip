// MFMA GEMM with fused epilogue for gfx950.
//
// Tile 128x128, 256 threads = 4 waves (2x2), each wave owns 64x64 = 4x4 tiles of the 16x16 MFMA.
// K is staged 128 bytes per tile row (64 bf16 / 32 fp32) through a double-buffered LDS image
// (register staging: global loads for tile t+1 are issued before the MFMAs of tile t and written
// to the other buffer after them, one barrier per K tile).
//
// Operand layouts (template TA / TB):
//   0 = "K-contiguous" (A[m][k], or B[n][k] = nn.Linear weight): LDS image [128 rows][128 B],
//       16-B chunk c of row r stored at chunk c ^ (r & 7) (conflict-free ds_read_b128);
//   1 = "MN-contiguous" (A[k][m] or B[k][n]): LDS image [BK rows][128 elements]; bf16 fragments
//       come from ds_read_b64_tr_b16 (hardware transpose), fp32 fragments from 4 ds_read_b32.
// The three nn.Linear products are (TA,TB) = (0,0) forward, (0,1) grad-input, (1,1) grad-weight.
#include "common.h"
#include <algorithm>
#include <type_traits>
#include <stdlib.h>
#include <string.h>

#include "gemm_tiles.h"
#include "gemm256.h"

namespace mmfd_gemmx {
// the four-wave kernel's epilogue mode for this product, -1 when it does not take it (gemm_g4.hip)
int g4_epi(const mmfd_gemm_args& a, const EpiArgs& e, int splits);
}  // namespace mmfd_gemmx

namespace {

// CONV: implicit-GEMM convolution (ConvGeom): A is the NHWC activation and its fill gathers the
// im2col rows per K-tile (ConvFill); TA = 0 only. The body is shared by gemm_mfma_kernel and
// conv_mfma_kernel (two kernel names, so the plain GEMM's name in traces stays what it was).
// BNT: the tile's N width — 128, or 64 for N <= 64 (the ResNet stem / layer1 convolutions: a 128-wide
// tile spent half its MFMAs on zero columns); BNT = 64 takes K-contiguous B only (TB = 0)
template <typename T, int TA, int TB, typename TC, bool CONV, int BNT = BN>
__device__ __forceinline__ void
gemm_mfma_body(const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
               TC* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N,
               int64_t K, float alpha, int tiles_per_split, const EpiArgs& e, const ConvGeom& cg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(BNT == BN || (BNT == 64 && TB == 0), "the 64-wide tile takes K-contiguous B only");
  constexpr int BBYTES = BNT * ROWB, SBYTES = A_BYTES + BBYTES;  // B image, one stage
  constexpr int WNS = BNT / 32;                     // 16-column subtiles per wave (2 wave columns)
  constexpr int APIECES = A_BYTES / 1024 / NWAVES;  // 4 pieces per wave
  constexpr int BPIECES = BBYTES / 1024 / NWAVES;   // 2 (1 for BNT = 64) pieces per wave
  constexpr int PIECES = APIECES + BPIECES;         // DMA instructions per wave per tile

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int gx = gridDim.x, gy = gridDim.y;
  const int lin = blockIdx.y * gx + blockIdx.x;
  const int tile = xcd_remap(lin, gx * gy);
  const int tm = tile / gx, tn = tile % gx;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BNT;

  const int nkt_total = (int)((K + GT<T>::BK - 1) / GT<T>::BK);
  const int kt0 = blockIdx.z * tiles_per_split;
  const int nk = min(nkt_total, kt0 + tiles_per_split) - kt0;

  f32x4 acc[4][WNS];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < WNS; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t a_bytes = CONV ? cg.H * cg.W * cg.C * (M / (cg.Ho * cg.Wo)) * (int64_t)sizeof(T)
                               : (TA == 0 ? M : K) * lda * (int64_t)sizeof(T);
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A, a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(B, (TB == 0 ? N : K) * ldb * (int64_t)sizeof(T));
  std::conditional_t<CONV, ConvFill<T, APIECES>, Fill<T, TA, BM, APIECES>> fa;
  Fill<T, TB, BNT, BPIECES> fb;
  if constexpr (CONV) fa.init(cg, m0, M, wave, lane);
  else fa.init(lda, m0, M, wave, lane);
  fb.init(ldb, n0, N, wave, lane);

  auto issue = [&](int t) {
    const int64_t k0 = (int64_t)(kt0 + t) * GT<T>::BK;
    const bool tail = k0 + GT<T>::BK > K;
    char* st = smem + (t % NSTAGE) * SBYTES;
    if constexpr (CONV) fa.issue(rsa, st, cg, k0, K, wave);
    else fa.issue(rsa, st, (uint32_t)(k0 * (TA == 0 ? 1 : lda) * (int64_t)sizeof(T)), tail, k0, K, wave, lane);
    fb.issue(rsb, st + A_BYTES, (uint32_t)(k0 * (TB == 0 ? 1 : ldb) * (int64_t)sizeof(T)), tail, k0, K, wave, lane);
  };

  if (nk > 0) issue(0);
  if (nk > 1) issue(1);
  for (int t = 0; t < nk; ++t) {
    // tile t landed (keep tile t+1 in flight); the barrier also retires every wave's reads of the
    // stage about to be refilled (tile t-1)
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < nk) issue(t + 2);
    const char* la = smem + (t % NSTAGE) * SBYTES;
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int kc = 0; kc < GT<T>::KCH; ++kc) {
      uint4 xa[4], xb[WNS];
#pragma unroll
      for (int i = 0; i < 4; ++i) xa[i] = load_frag<T, TA, BM>(la, wm * 4 + i, kc, lane);
#pragma unroll
      for (int j = 0; j < WNS; ++j) xb[j] = load_frag<T, TB, BNT>(lb, wn * WNS + j, kc, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < WNS; ++j) Mma<T>::run(acc[i][j], xa[i], xb[j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: stage the 256x128 fp32 tile through LDS in four 64-row quarters (one wave row
  // each), then every thread handles 4 consecutive columns of a row (coalesced stores).
  constexpr int LDC = BNT + 4;
  float* ct = reinterpret_cast<float*>(smem);
  const int g = lane >> 4, ci = lane & 15;
  const uint32_t seed = (!ws && e.p > 0.0f) ? mmfd_hash_key(*e.seed, e.salt) : 0u;  // dropout hash key
  float* slab = ws ? ws + (int64_t)blockIdx.z * M * N : nullptr;
#pragma unroll
  for (int qtr = 0; qtr < 4; ++qtr) {
    if (wm == qtr) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < WNS; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ct[(i * 16 + 4 * g + r) * LDC + wn * (BNT / 2) + j * 16 + ci] = acc[i][j][r];
    }
    __syncthreads();
    // 64 rows x BNT/8 groups of 8 columns
    for (int idx = tid; idx < 64 * (BNT / 8); idx += NT) {
      const int lr = idx / (BNT / 8), c8 = (idx % (BNT / 8)) * 8;
      const int64_t row = m0 + qtr * 64 + lr;
      const int64_t col = n0 + c8;
      if (row >= M || col >= N) continue;
      const float* src = ct + lr * LDC + c8;
      const float4 a4 = *reinterpret_cast<const float4*>(src), b4 = *reinterpret_cast<const float4*>(src + 4);
      float vv[8] = {alpha * a4.x, alpha * a4.y, alpha * a4.z, alpha * a4.w,
                     alpha * b4.x, alpha * b4.y, alpha * b4.z, alpha * b4.w};
      const bool full = col + 8 <= N;
      if (slab) {
        if (full && (N % 4) == 0) {
          *reinterpret_cast<float4*>(slab + row * N + col) = make_float4(vv[0], vv[1], vv[2], vv[3]);
          *reinterpret_cast<float4*>(slab + row * N + col + 4) = make_float4(vv[4], vv[5], vv[6], vv[7]);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (col + q < N) slab[row * N + col + q] = vv[q];
        }
      } else if (full && e.vec) {
        epilogue_store8<TC>(e, C, ldc, N, row, col, vv, seed);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (col + q < N) epilogue_store<TC>(e, C, ldc, N, row, col + q, vv[q], seed);
      }
    }
    __syncthreads();
  }
}


template <typename T, int TA, int TB, typename TC>
__global__ void __launch_bounds__(NT, 1)
gemm_mfma_kernel(const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
                 TC* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N,
                 int64_t K, float alpha, int tiles_per_split, EpiArgs e) {
  gemm_mfma_body<T, TA, TB, TC, false>(A, lda, B, ldb, C, ldc, ws, M, N, K, alpha, tiles_per_split, e, ConvGeom{});
}
// the 256x64 tile for N <= 64 with K-contiguous B
template <typename T, int TA, typename TC>
__global__ void __launch_bounds__(NT, 1)
gemm_mfma_n64_kernel(const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
                     TC* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N,
                     int64_t K, float alpha, int tiles_per_split, EpiArgs e) {
  gemm_mfma_body<T, TA, 0, TC, false, 64>(A, lda, B, ldb, C, ldc, ws, M, N, K, alpha, tiles_per_split, e, ConvGeom{});
}
// implicit-GEMM convolution on the 256x128 kernel (mmfd_gemm_args.conv): A = the NHWC activation
template <typename T, typename TC, int BNT>
__global__ void __launch_bounds__(NT, 1)
conv_mfma_kernel(const T* __restrict__ X, const T* __restrict__ B, int64_t ldb, TC* __restrict__ C, int64_t ldc,
                 float* __restrict__ ws, int64_t M, int64_t N, int64_t K, float alpha, int tiles_per_split, EpiArgs e,
                 ConvGeom cg) {
  gemm_mfma_body<T, 0, 0, TC, true, BNT>(X, cg.C, B, ldb, C, ldc, ws, M, N, K, alpha, tiles_per_split, e, cg);
}

// The epilogue activations MMFD_ACT_GELU_D (GELU, aux <- gelu'(z)) and MMFD_ACT_MUL_AUX (z *= aux)
// run in the four-wave kernel's register epilogue (gemm_g4.hip, the bf16 training FFN), and
// everywhere else in the split-K reduce / simple kernels only: a product with one of them that the
// four-wave kernel does not take writes its raw fp32 sums to a workspace slab (one split at least)
// and the reduce applies the whole epilogue. The tile kernels' shared epilogues (gemm_tiles.h) keep
// their round-5 code — the two extra activations inlined there made every GEMM's epilogue slower
// (config-5 extract −4 %, profiles/r06t_extract_regression.log).
// The forward-only tanh / sigmoid (the cross-encoder's pooler and score) go the same way: the tile
// kernels' epilogues carry only NONE / GELU / ReLU and their backward forms.
__device__ __host__ __forceinline__ bool act_ext(int act) {
  return act == MMFD_ACT_GELU_D || act == MMFD_ACT_MUL_AUX || act == MMFD_ACT_TANH || act == MMFD_ACT_SIGMOID;
}

// epilogue_store (gemm_tiles.h) with the two extra activations: bias, [residual first], the
// activation, then the unchanged tail (dropout, residual, beta, store / planes)
template <typename TC>
__device__ __forceinline__ void epilogue_store_x(const EpiArgs& e, TC* C, int64_t ldc, int64_t N, int64_t row,
                                                 int64_t col, float z, uint32_t hkey) {
  if (!act_ext(e.act)) return epilogue_store<TC>(e, C, ldc, N, row, col, z, hkey);
  if (e.bias) z += e.bias[col];
  if (e.res_first && e.residual) z += to_f32(reinterpret_cast<const TC*>(e.residual)[row * e.ldr + col]);
  TC* ax = reinterpret_cast<TC*>(e.aux) + row * e.ldaux + col;
  if (e.act == MMFD_ACT_GELU_D) {
    float d;
    z = gelu_and_grad_f(z, d);
    if (e.aux) *ax = from_f32<TC>(d);
  } else if (e.act == MMFD_ACT_MUL_AUX) {
    z *= to_f32(*ax);
  } else {
    z = act_tail_f(e.act, z);
  }
  EpiArgs t = e;
  t.act = MMFD_ACT_NONE; t.bias = nullptr;
  if (e.res_first) t.residual = nullptr;
  epilogue_store<TC>(t, C, ldc, N, row, col, z, hkey);
}

template <typename TC>
__device__ __forceinline__ void epilogue_store8_x(const EpiArgs& e, TC* C, int64_t ldc, int64_t N, int64_t row,
                                                  int64_t col, float (&z)[8], uint32_t hkey) {
  if (!act_ext(e.act)) return epilogue_store8<TC>(e, C, ldc, N, row, col, z, hkey);
  if (e.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(e.bias + col), b1 = *reinterpret_cast<const float4*>(e.bias + col + 4);
    z[0] += b0.x; z[1] += b0.y; z[2] += b0.z; z[3] += b0.w; z[4] += b1.x; z[5] += b1.y; z[6] += b1.z; z[7] += b1.w;
  }
  if (e.res_first && e.residual) {
    float r[8];
    V8<TC>::load(reinterpret_cast<const TC*>(e.residual) + row * e.ldr + col, r);
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] += r[q];
  }
  TC* ax = reinterpret_cast<TC*>(e.aux) + row * e.ldaux + col;
  if (e.act == MMFD_ACT_GELU_D) {
    float d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] = gelu_and_grad_f(z[q], d[q]);
    if (e.aux) V8<TC>::store(ax, d);
  } else if (e.act == MMFD_ACT_MUL_AUX) {
    float a[8];
    V8<TC>::load(ax, a);
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] *= a[q];
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] = act_tail_f(e.act, z[q]);
  }
  EpiArgs t = e;
  t.act = MMFD_ACT_NONE; t.bias = nullptr;
  if (e.res_first) t.residual = nullptr;
  epilogue_store8<TC>(t, C, ldc, N, row, col, z, hkey);
}

// split-K reduce, one output per thread (outputs that are not 16-B vectorisable; else splitk_reduce8_kernel)
template <typename TC>
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, TC* __restrict__ C,
                                     int64_t ldc, int64_t M, int64_t N, EpiArgs e, const float* __restrict__ rs_part,
                                     int rs_nparts,
                                     float* __restrict__ rs_out, float rs_beta) {
  const uint32_t seed = (e.p > 0.0f) ? mmfd_hash_key(*e.seed, e.salt) : 0u;  // dropout hash key
  const int64_t total = M * N;
  if (rs_part) {  // the fused row sums' per-split partials (G8 split-K), summed in split order
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
      float t = 0.f;
      for (int s = 0; s < rs_nparts; ++s) t += rs_part[(int64_t)s * M + m];
      rs_out[m] = (rs_beta != 0.f ? rs_beta * rs_out[m] : 0.f) + t;
    }
  }
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float z = 0.f;
    for (int s = 0; s < splits; ++s) z += ws[(int64_t)s * total + idx];
    epilogue_store_x<TC>(e, C, ldc, N, idx / N, idx % N, z, seed);
  }
}

// split-K reduce for 16-B-aligned outputs with N % 8 == 0: 8 consecutive outputs per thread group,
// the splits cut into P contiguous ranges summed by P threads (each in split order) and combined
// through LDS in range order — deterministic, and P x the threads of one-thread-per-8-outputs: a
// weight gradient's 768 x 768 output is 73,728 groups, 288 busy blocks on 256 CUs at P = 1 (the
// slab reads ran at ~1 TB/s), 2,304 at P = 8
template <typename TC, int P>
__global__ void __launch_bounds__(256) splitk_reduce8_kernel(const float* __restrict__ ws, int splits,
                                                             TC* __restrict__ C, int64_t ldc, int64_t M, int64_t N,
                                                             EpiArgs e, const float* __restrict__ rs_part,
                                                             int rs_nparts, float* __restrict__ rs_out, float rs_beta) {
  constexpr int G = 256 / P;  // output groups per block pass
  __shared__ float red[P > 1 ? P - 1 : 1][G][9];
  const uint32_t seed = (e.p > 0.0f) ? mmfd_hash_key(*e.seed, e.salt) : 0u;  // dropout hash key
  const int64_t total = M * N, groups = total / 8;
  if (rs_part) {  // the fused row sums' per-split partials (G8 split-K), summed in split order
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
      float t = 0.f;
      for (int s = 0; s < rs_nparts; ++s) t += rs_part[(int64_t)s * M + m];
      rs_out[m] = (rs_beta != 0.f ? rs_beta * rs_out[m] : 0.f) + t;
    }
  }
  const int gi = threadIdx.x % G, pi = threadIdx.x / G;
  const int per = (splits + P - 1) / P;
  const int s0 = pi * per, s1 = min(splits, s0 + per);
  for (int64_t gb = (int64_t)blockIdx.x * G; gb < groups; gb += (int64_t)gridDim.x * G) {
    const int64_t g = gb + gi;
    float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (g < groups) {
      const float* base = ws + g * 8;
      int s = s0;
      for (; s + 4 <= s1; s += 4) {  // four slabs' loads in flight before their adds (split order)
        float4 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float* q = base + (int64_t)(s + u) * total;
          a[u] = *reinterpret_cast<const float4*>(q);
          b[u] = *reinterpret_cast<const float4*>(q + 4);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          z[0] += a[u].x; z[1] += a[u].y; z[2] += a[u].z; z[3] += a[u].w;
          z[4] += b[u].x; z[5] += b[u].y; z[6] += b[u].z; z[7] += b[u].w;
        }
      }
      for (; s < s1; ++s) {
        const float* q = base + (int64_t)s * total;
        const float4 a = *reinterpret_cast<const float4*>(q), b = *reinterpret_cast<const float4*>(q + 4);
        z[0] += a.x; z[1] += a.y; z[2] += a.z; z[3] += a.w; z[4] += b.x; z[5] += b.y; z[6] += b.z; z[7] += b.w;
      }
    }
    if constexpr (P > 1) {
      if (pi > 0) {
#pragma unroll
        for (int u = 0; u < 8; ++u) red[pi - 1][gi][u] = z[u];
      }
      __syncthreads();
      if (pi == 0) {
#pragma unroll
        for (int q = 0; q < P - 1; ++q)
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] += red[q][gi][u];
      }
      __syncthreads();
    }
    if (pi == 0 && g < groups) epilogue_store8_x<TC>(e, C, ldc, N, (g * 8) / N, (g * 8) % N, z, seed);
  }
}

// Plain FMA GEMM for shapes the MFMA path cannot take (tiny / unaligned: classifier heads).
template <typename T, typename TC>
__global__ void gemm_simple_kernel(const T* __restrict__ A, int64_t lda, int ta, const T* __restrict__ B,
                                   int64_t ldb, int tb, TC* __restrict__ C, int64_t ldc, int64_t M,
                                   int64_t N, int64_t K, float alpha, EpiArgs e) {
  const uint32_t seed = (e.p > 0.0f) ? mmfd_hash_key(*e.seed, e.salt) : 0u;  // dropout hash key
  const int64_t total = M * N;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = idx / N, n = idx % N;
    float s = 0.f;
    for (int64_t k = 0; k < K; ++k) {
      const float a = to_f32(ta ? A[k * lda + m] : A[m * lda + k]);
      const float b = to_f32(tb ? B[k * ldb + n] : B[n * ldb + k]);
      s = fmaf(a, b, s);
    }
    epilogue_store_x<TC>(e, C, ldc, N, m, n, alpha * s, seed);
  }
}

template <typename T, int TA, int TB, typename TC>
void launch_mfma(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps,
                 hipStream_t s) {
  if constexpr (TB == 0) {
    if (a.N <= 64) {  // the 256x64 tile (no zero half-tile of B)
      dim3 grid(1u, (unsigned)((a.M + BM - 1) / BM), (unsigned)splits);
      constexpr int lds = NSTAGE * (A_BYTES + 64 * ROWB);
      static bool attr64 = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_mfma_n64_kernel<T, TA, TC>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
      }();
      (void)attr64;
      hipLaunchKernelGGL((gemm_mfma_n64_kernel<T, TA, TC>), grid, dim3(NT), lds, s, (const T*)a.A, a.lda,
                         (const T*)a.B, a.ldb, (TC*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, tps, e);
      return;
    }
  }
  dim3 grid((unsigned)((a.N + BN - 1) / BN), (unsigned)((a.M + BM - 1) / BM), (unsigned)splits);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_mfma_kernel<T, TA, TB, TC>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_mfma_kernel<T, TA, TB, TC>), grid, dim3(NT), LDS_BYTES, s,
                     (const T*)a.A, a.lda, (const T*)a.B, a.ldb, (TC*)a.C, a.ldc, ws, a.M, a.N, a.K,
                     a.alpha, tps, e);
}
template <typename T, typename TC, int BNT>
void launch_conv_mfma_t(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps, hipStream_t s,
                        const ConvGeom& cg) {
  dim3 grid((unsigned)((a.N + BNT - 1) / BNT), (unsigned)((a.M + BM - 1) / BM), (unsigned)splits);
  constexpr int lds = NSTAGE * (A_BYTES + BNT * ROWB);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_mfma_kernel<T, TC, BNT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((conv_mfma_kernel<T, TC, BNT>), grid, dim3(NT), lds, s, (const T*)a.A, (const T*)a.B, a.ldb,
                     (TC*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, tps, e, cg);
}
template <typename T, typename TC>
void launch_conv_mfma(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps, hipStream_t s,
                      const ConvGeom& cg) {
  if (a.N <= 64) launch_conv_mfma_t<T, TC, 64>(a, e, ws, splits, tps, s, cg);
  else launch_conv_mfma_t<T, TC, BN>(a, e, ws, splits, tps, s, cg);
}


template <typename T, int TA, int TB, typename TC>
void launch_g8(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps, float* rs_out,
               int rs_mode, hipStream_t s, const X6Args* x6, const void* xa, const void* xb) {
  const X6Args none{1, 0, 0};
  if constexpr (std::is_same<TC, float>::value) {
    // fp32-output instantiations live in gemm_f32out.hip (built without SLP vectorisation)
    if constexpr (std::is_same<T, bf16>::value) {
      if (x6) {  // split-operand fp32 GEMM: A / B are the bf16 planes, leading dim = stored columns
        const int64_t lda = TA == 0 ? a.K : a.M, ldb = TB == 0 ? a.K : a.N;
        return mmfd_gemmx::launch_g8_f32out<T, TA, TB, true>(a, e, ws, splits, tps, rs_out, rs_mode, s, xa, lda, xb,
                                                             ldb, *x6);
      }
    }
    return mmfd_gemmx::launch_g8_f32out<T, TA, TB, false>(a, e, ws, splits, tps, rs_out, rs_mode, s, a.A, a.lda, a.B,
                                                          a.ldb, none);
  } else {
    const bool bwd_act = e.act == MMFD_ACT_GELU_BWD || e.act == MMFD_ACT_RELU_BWD || e.act == MMFD_ACT_MUL_AUX;
    const int streams = (e.residual ? 1 : 0) + (bwd_act ? 1 : 0) + (e.beta != 0.f ? 1 : 0);
    if (streams == 1 && !ws && e.vec)
      return launch_g8_v<T, TA, TB, TC, true, false>(a, e, ws, splits, tps, rs_out, rs_mode, s, a.A, a.lda, a.B, a.ldb, none);
    launch_g8_v<T, TA, TB, TC, false, false>(a, e, ws, splits, tps, rs_out, rs_mode, s, a.A, a.lda, a.B, a.ldb, none);
  }
}

template <typename T, typename TC>
void dispatch_g8(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps, float* rs_out,
                 int rs_mode, hipStream_t s, const X6Args* x6 = nullptr, const void* xa = nullptr,
                 const void* xb = nullptr) {
  if (!a.trans_a && !a.trans_b) launch_g8<T, 0, 0, TC>(a, e, ws, splits, tps, rs_out, rs_mode, s, x6, xa, xb);
  else if (!a.trans_a && a.trans_b) launch_g8<T, 0, 1, TC>(a, e, ws, splits, tps, rs_out, rs_mode, s, x6, xa, xb);
  else if (a.trans_a && !a.trans_b) launch_g8<T, 1, 0, TC>(a, e, ws, splits, tps, rs_out, rs_mode, s, x6, xa, xb);
  else launch_g8<T, 1, 1, TC>(a, e, ws, splits, tps, rs_out, rs_mode, s, x6, xa, xb);
}

// split-operand kernel: fused planes (gemm256_x6f_kernel, the default) or the segmented K loop
// (gemm256_kernel<X6>, env MMFD_X6_SEGMENTED=1, kept for A/B measurements)
bool x6_fused() {
  static const bool seg = getenv("MMFD_X6_SEGMENTED") != nullptr;
  return !seg;
}

// fp32 operand -> three bf16 planes (hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid),
// each difference exact in fp32): stored rows x cols (ld) -> planes [3][rows][cols]; 8 columns per
// thread (two 16-B loads, one 16-B store per plane), cols % 8 == 0
__global__ void __launch_bounds__(256) split3_kernel(const float* __restrict__ X, int64_t ldx, int64_t rows,
                                                     int64_t cols, bf16* __restrict__ P, int64_t plane) {
  // one 8-column chunk of one row per thread, grid-stride over all chunks (narrow rows — 768
  // columns = 96 chunks — keep every lane busy)
  const uint32_t c8 = (uint32_t)(cols / 8);
  const uint32_t total = (uint32_t)(rows * c8);
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t r = i / c8;
    const int64_t c = (int64_t)(i - r * c8) * 8;
    const float* src = X + (int64_t)r * ldx + c;
    const float4 x0 = *reinterpret_cast<const float4*>(src);
    const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
    const float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    bf16x8 h, m, l;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bf16 hu = (bf16)x[u];
      const float r1 = x[u] - (float)hu;
      const bf16 mu = (bf16)r1;
      h[u] = hu;
      m[u] = mu;
      l[u] = (bf16)(r1 - (float)mu);
    }
    bf16* d = P + (int64_t)r * cols + c;
    *reinterpret_cast<uint4*>(d) = __builtin_bit_cast(uint4, h);
    *reinterpret_cast<uint4*>(d + plane) = __builtin_bit_cast(uint4, m);
    *reinterpret_cast<uint4*>(d + 2 * plane) = __builtin_bit_cast(uint4, l);
  }
}

void launch_split3(const float* X, int64_t ldx, int64_t rows, int64_t cols, bf16* P, hipStream_t s) {
  const int64_t chunks = rows * (cols / 8);
  const unsigned blocks = (unsigned)std::min<int64_t>((chunks + 255) / 256, 8192);
  hipLaunchKernelGGL(split3_kernel, dim3(blocks), dim3(256), 0, s, X, ldx, rows, cols, P, rows * cols);
}

// fp32 x fp32 -> fp32 GEMM mode: 1 = split operands (six bf16 MFMA products per fp32 product, see
// gemm256_kernel's X6 note; about 1.6x the fp32 MFMA rate at the encoder shapes), 0 = fp32 MFMA
int g_fp32_mode = [] {
  const char* v = getenv("MMFD_FP32_GEMM");
  return (v && (!strcmp(v, "native") || !strcmp(v, "0"))) ? 0 : 1;
}();

bool use_g8(const mmfd_gemm_args& a) {
  static const bool off = getenv("MMFD_GEMM_V1") != nullptr;
  static const bool off_f32 = getenv("MMFD_GEMM_F32_V1") != nullptr;
  static const bool narrow_g8 = getenv("MMFD_GEMM_NARROW_G8") != nullptr;
  // tall GEMMs with N <= 128 or K < 64 (Swinv2 stage-1 out-projection / FFN2 at N = 128, its 4x4
  // patch embedding at K = 48): the 256x256 tile is half padding / all prologue, and the 256x128
  // kernel measured 20-35 % faster per launch (45 vs 66 us, 85 vs 107 us, 36 vs 55 us)
  if (!narrow_g8 && a.M >= 4096 && (a.N <= 128 || a.K < 64)) return false;
  if (off) return false;
  if (a.dtype == MMFD_BF16) return true;
  // fp32 operands (the parity / headline mode): the 256x256 tile halves the B-panel traffic per
  // MFMA of the 256x128 kernel; fp32 C only (a bf16 C from fp32 operands stays on the 256x128 kernel)
  return a.dtype == MMFD_F32 && a.c_dtype == MMFD_F32 && !off_f32;
}

template <typename T, typename TC>
void dispatch_layout(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps,
                     hipStream_t s) {
  if (!a.trans_a && !a.trans_b) launch_mfma<T, 0, 0, TC>(a, e, ws, splits, tps, s);
  else if (!a.trans_a && a.trans_b) launch_mfma<T, 0, 1, TC>(a, e, ws, splits, tps, s);
  else if (a.trans_a && !a.trans_b) launch_mfma<T, 1, 0, TC>(a, e, ws, splits, tps, s);
  else launch_mfma<T, 1, 1, TC>(a, e, ws, splits, tps, s);
}

bool mfma_ok(const mmfd_gemm_args& a) {
  const int epc = (a.dtype == MMFD_BF16) ? 8 : 4;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (a.conv) {  // implicit convolution: checked by conv_geom(); B as below
    const int64_t esz = a.dtype == MMFD_BF16 ? 2 : 4;
    const int64_t bbytes = (a.trans_b ? a.K : a.N) * a.ldb * esz;
    return al16(a.B) && a.ldb % epc == 0 && (a.trans_b ? a.N : a.K) % epc == 0 && a.N >= 16 &&
           bbytes < (1ll << 31) - 4096;
  }
  if (!al16(a.A) || !al16(a.B)) return false;
  if (a.lda % epc || a.ldb % epc) return false;
  const int64_t a_ext = a.trans_a ? a.M : a.K;  // contiguous extent
  const int64_t b_ext = a.trans_b ? a.N : a.K;
  if (a_ext % epc || b_ext % epc) return false;
  if (a.M < 16 || a.N < 16 || a.K < 16) return false;
  const int64_t esz = a.dtype == MMFD_BF16 ? 2 : 4;
  const int64_t abytes = (a.trans_a ? a.K : a.M) * a.lda * esz, bbytes = (a.trans_b ? a.K : a.N) * a.ldb * esz;
  if (abytes >= (1ll << 31) - 4096 || bbytes >= (1ll << 31) - 4096) return false;  // 32-bit buffer offsets
  return true;
}

int choose_splits(const mmfd_gemm_args& a, int64_t* ws_bytes_needed, bool x6 = false) {
  const int T = (a.dtype == MMFD_BF16 || x6) ? 64 : 32;
  const bool xf = x6 && x6_fused();  // fused planes: one unit = one 32-deep step of all six products
  const int64_t nkt = xf ? (a.K + 31) / 32 : x6 ? 6 * ((a.K + 63) / 64) : (a.K + T - 1) / T;
  int splits = 1;
  if (use_g8(a)) {
    // one 256x256 block per CU: pick the split count that minimises rounds-of-256 per unit of work
    const int64_t tiles = ((a.M + G8_BM - 1) / G8_BM) * ((a.N + G8_BN - 1) / G8_BN);
    if (a.splits > 0) splits = a.splits;
    else if (nkt >= 16 && tiles < 256) {
      // modelled time (us): rounds of 256 blocks x (K-tiles per block x ~1.8 us + ~3 us block
      // overhead) + the fp32 slab round trip (written by the blocks, read by the reduce) at ~5 TB/s
      double best = 1e30;
      // (up to one round of blocks: the fusion head's 256x256 weight gradients over 32k-50k rows are
      // a single tile, and 32 splits left 224 CUs idle for ~180 us per launch)
      const int smax = (int)std::min<int64_t>(std::max<int64_t>(32, 256 / tiles), nkt / 8);
      // one 256x256 K-tile (bf16 / fp32 MFMA rate; a fused split-operand step = 3 bf16 K-tiles of MFMA)
      const double kt_us = xf ? 3.6 : (a.dtype == MMFD_BF16 || x6) ? 1.8 : 7.0;
      for (int sp = 1; sp <= smax; ++sp) {
        const double rounds = (double)((tiles * sp + 255) / 256);
        const double kts = (double)((nkt + sp - 1) / sp);
        double cost = rounds * (kts * kt_us + 3.0);
        if (sp > 1) cost += (double)sp * a.M * a.N * 8.0 / 5.0e6 + 4.0;
        if (cost < best) { best = cost; splits = sp; }
      }
    }
  } else if (a.splits > 0) splits = a.splits;
  else if (((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) < 200 && nkt >= 16) {
    const int64_t tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    splits = (int)((384 + tiles - 1) / tiles);
    splits = (int)std::min<int64_t>(splits, nkt / 8);
    splits = std::min(splits, 16);
    if (splits < 1) splits = 1;
  }
  if (splits > nkt) splits = (int)nkt;
  if (splits < 1) splits = 1;
  *ws_bytes_needed = (splits > 1) ? (int64_t)splits * a.M * a.N * 4 : 0;
  return splits;
}


// split-operand eligibility: fp32 in / fp32 out on the 256x256 path, stored column counts a
// multiple of 8 (16-B plane rows), three planes of each operand < 2 GB (32-bit buffer offsets), and
// K a whole number of 64-row tiles when an operand is MN-contiguous (its K rows are plane rows:
// a partial tile would read into the next plane)
struct X6Plan { bool on; int64_t rows_a, cols_a, rows_b, cols_b, pa, pb; };
X6Plan x6_plan(const mmfd_gemm_args& a) {
  X6Plan p{};
  if (g_fp32_mode != 1 || a.dtype != MMFD_F32 || a.c_dtype != MMFD_F32 || !use_g8(a)) return p;
  p.rows_a = a.trans_a ? a.K : a.M; p.cols_a = a.trans_a ? a.M : a.K;
  if (a.conv) {  // the planes of the NHWC activation, not of the (never written) im2col matrix
    p.rows_a = a.conv->N * a.conv->H * a.conv->W; p.cols_a = a.conv->C;
  }
  p.rows_b = a.trans_b ? a.K : a.N; p.cols_b = a.trans_b ? a.N : a.K;
  if (p.cols_a % 8 || p.cols_b % 8) return p;
  if ((a.trans_a || a.trans_b) && a.K % (x6_fused() ? 32 : 64)) return p;
  p.pa = p.rows_a * p.cols_a * 2; p.pb = p.rows_b * p.cols_b * 2;
  if (3 * p.pa >= (1ll << 31) - 4096 || 3 * p.pb >= (1ll << 31) - 4096) return p;
  p.on = true;
  return p;
}
int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// extra workspace for the fused row sums: per-split partials (G8) or the colsum partials (others)
int64_t rowsum_ws_bytes(const mmfd_gemm_args& a, int splits, bool g8) {
  if (!a.a_rowsum) return 0;
  if (g8) {  // per-(split, column tile) partials (gemm256_kernel rs_mode 3)
    const int64_t parts = (int64_t)splits * ((a.N + G8_BN - 1) / G8_BN);
    return parts > 1 ? parts * a.M * 4 : 0;
  }
  const int64_t nparts = std::min<int64_t>(256, std::max<int64_t>(1, a.K / 64));
  return nparts * a.M * 4;
}

// row sums of op(A) for the non-G8 paths: with trans_a, op(A) rows are the columns of the stored
// [K][M] matrix, i.e. mmfd_colsum
int rowsum_fallback(const mmfd_gemm_args& a, void* ws, int64_t ws_bytes, hipStream_t s) {
  if (!a.a_rowsum) return 0;
  if (!a.trans_a)
    return mmfd_set_error(MMFD_ERR_UNSUPPORTED, "mmfd_gemm: a_rowsum without trans_a needs the bf16 MFMA path");
  return mmfd_colsum(a.dtype, a.K, a.M, a.A, a.lda, a.a_rowsum, a.a_rowsum_beta, ws, ws_bytes, s);
}

// the implicit-convolution geometry of `a` (on = 0 without one), or an error string
const char* conv_geom(const mmfd_gemm_args& a, ConvGeom& g) {
  g = ConvGeom{};
  if (!a.conv) return nullptr;
  const mmfd_conv_geom& c = *a.conv;
  const int64_t kstep = a.dtype == MMFD_BF16 ? 64 : 32;  // K per K-tile / split-operand K-step
  if (a.trans_a) return "conv needs trans_a = 0";
  if (c.N <= 0 || c.H <= 0 || c.W <= 0 || c.C <= 0 || c.KH <= 0 || c.KW <= 0 || c.stride <= 0 || c.pad < 0)
    return "conv: bad geometry";
  if (c.Ho != (c.H + 2 * c.pad - c.KH) / c.stride + 1 || c.Wo != (c.W + 2 * c.pad - c.KW) / c.stride + 1)
    return "conv: Ho / Wo do not match H, W, KH, KW, stride, pad";
  if (a.M != c.N * c.Ho * c.Wo || a.K != (int64_t)c.KH * c.KW * c.C) return "conv: M != N*Ho*Wo or K != KH*KW*C";
  if (c.C % kstep) return "conv: C must be a multiple of 32 (fp32) / 64 (bf16)";
  if (((uintptr_t)a.A & 15) != 0) return "conv: x must be 16-B aligned";
  if (a.a_rowsum || a.a_planes_only) return "conv: no a_rowsum / a_planes_only";
  const int64_t esz = a.dtype == MMFD_BF16 ? 2 : 4;
  if (c.N * c.H * c.W * c.C * esz >= (1ll << 31) - 4096) return "conv: activation >= 2 GB";
  g.on = 1; g.KW = c.KW; g.stride = c.stride; g.pad = c.pad;
  g.H = c.H; g.W = c.W; g.C = c.C; g.Ho = c.Ho; g.Wo = c.Wo;
  return nullptr;
}

}  // namespace

#ifdef MMFD_G8_STAMPS
extern "C" int mmfd_debug_g8_stamps(void* host_dst, int64_t bytes) {
  return (int)hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g8_stamps), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
#endif

namespace {
EpiArgs make_epi(const mmfd_gemm_args& a) {
  EpiArgs e;
  e.bias = a.ep.bias; e.residual = a.ep.residual; e.ldr = a.ep.ldr; e.aux = a.ep.aux;
  e.ldaux = a.ep.ldaux; e.act = a.ep.act; e.p = a.ep.dropout_p > 0.f ? a.ep.dropout_p : 0.f;
  e.thr = mmfd_drop_threshold(e.p); e.keep_scale = 1.0f / (1.0f - e.p);
  e.seed = a.ep.seed; e.salt = a.ep.salt; e.beta = a.beta; e.res_first = a.ep.residual_first ? 1 : 0;
  e.pl = a.c_dtype == MMFD_F32 ? (bf16*)a.ep.out_planes : nullptr;
  e.pl_stride = a.M * a.N;
  e.c_out = (a.C != nullptr) ? 1 : 0;
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  bool v = (a.C == nullptr || al(a.C)) && (a.ldc % 8) == 0;
  if (a.ep.residual) v = v && al(a.ep.residual) && (a.ep.ldr % 8) == 0;
  if (a.ep.aux) v = v && al(a.ep.aux) && (a.ep.ldaux % 8) == 0;
  if (a.ep.bias) v = v && al(a.ep.bias);
  e.vec = v ? 1 : 0;
  return e;
}

// a GELU_D / MUL_AUX product on the MFMA paths that the four-wave kernel does not take: the tile
// kernels write raw sums to a slab (at least one split) and the reduce runs the epilogue
bool ext_slab(const mmfd_gemm_args& a, int splits, bool x6_on) {
  const int act = a.ep.act;
  if (!act_ext(act)) return false;
  if (splits == 1 && use_g8(a) && a.dtype == MMFD_BF16 && a.c_dtype == MMFD_BF16 && !a.conv &&
      mmfd_gemmx::g4_epi(a, make_epi(a), splits) >= 0)
    return false;
  // the split-operand kernel's ext instantiation: GELU_D / MUL_AUX without dropout, one split, and
  // every tile on the epilogue's fast path (full 256x256 tiles, 16-B aligned operands: its per-element
  // path for partial tiles is the shared one, which does not carry the two)
  if (splits == 1 && (act == MMFD_ACT_GELU_D || act == MMFD_ACT_MUL_AUX) && a.ep.dropout_p <= 0.f && !a.conv &&
      x6_on && x6_fused() && a.M % 256 == 0 && a.N % 256 == 0 && make_epi(a).vec)
    return false;
  return true;
}
}  // namespace

// The queries return -1 (error string set) for arguments of another ABI layout (struct_size).
static bool gemm_struct_ok(const mmfd_gemm_args* a, const char* what) {
  if (a && a->struct_size == (int64_t)sizeof(mmfd_gemm_args)) return true;
  mmfd_set_error(MMFD_ERR_INVALID, "%s: mmfd_gemm_args.struct_size = %lld, this library expects %lld (ABI version %d)",
                 what, a ? (long long)a->struct_size : 0ll, (long long)sizeof(mmfd_gemm_args), MMFD_ABI_VERSION);
  return false;
}

extern "C" int64_t mmfd_gemm_workspace_bytes(const mmfd_gemm_args* a) {
  if (!gemm_struct_ok(a, "mmfd_gemm_workspace_bytes")) return -1;
  if (!mfma_ok(*a)) return rowsum_ws_bytes(*a, 1, false);
  const X6Plan xp = x6_plan(*a);
  int64_t need = 0;
  const int splits = choose_splits(*a, &need, xp.on);
  if (ext_slab(*a, splits, xp.on) && need < a->M * a->N * 4) need = a->M * a->N * 4;
  need += rowsum_ws_bytes(*a, splits, use_g8(*a));
  if (xp.on)  // + the bf16 planes of the operands not handed over already split
    need = align256(need) + (a->a_planes ? 0 : align256(3 * xp.pa)) + (a->b_planes ? 0 : 3 * xp.pb);
  return need;
}

extern "C" int mmfd_gemm_splits(const mmfd_gemm_args* a) {
  if (!gemm_struct_ok(a, "mmfd_gemm_splits")) return -1;
  if (!mfma_ok(*a)) return 1;
  int64_t need = 0;
  return choose_splits(*a, &need, x6_plan(*a).on);
}

extern "C" int mmfd_gemm_runs_split(const mmfd_gemm_args* a) {
  if (!gemm_struct_ok(a, "mmfd_gemm_runs_split")) return -1;
  if (!mfma_ok(*a)) return 0;
  const X6Plan xp = x6_plan(*a);
  return xp.on ? (x6_fused() ? 2 : 1) : 0;
}

extern "C" int mmfd_set_fp32_gemm_mode(int mode) {
  MMFD_CHECK_ARG(mode == 0 || mode == 1, "mmfd_set_fp32_gemm_mode: mode %d (0 = fp32 MFMA, 1 = split operands)", mode);
  const int old = g_fp32_mode;
  g_fp32_mode = mode;
  return old;
}

extern "C" int mmfd_gemm(const mmfd_gemm_args* ap, mmfd_stream_t stream) {
  MMFD_CHECK_STRUCT(ap, mmfd_gemm_args, "mmfd_gemm");
  const mmfd_gemm_args& a = *ap;
  hipStream_t s = (hipStream_t)stream;
  MMFD_CHECK_ARG(a.dtype == MMFD_F32 || a.dtype == MMFD_BF16, "mmfd_gemm: bad dtype %d", a.dtype);
  MMFD_CHECK_ARG(a.c_dtype == MMFD_F32 || a.c_dtype == MMFD_BF16, "mmfd_gemm: bad c_dtype %d", a.c_dtype);
  MMFD_CHECK_ARG(a.M >= 0 && a.N >= 0 && a.K >= 0, "mmfd_gemm: negative shape");
  MMFD_CHECK_ARG(a.C != nullptr || (a.ep.out_planes != nullptr && a.c_dtype == MMFD_F32 && a.beta == 0.f),
                 "mmfd_gemm: null C (allowed only with fp32 out_planes and beta = 0)");
  MMFD_CHECK_ARG(a.ep.out_planes == nullptr || (a.N % 8 == 0 && ((uintptr_t)a.ep.out_planes & 15) == 0),
                 "mmfd_gemm: out_planes need N %% 8 == 0 and 16-B alignment");
  MMFD_CHECK_ARG(a.ldc >= a.N, "mmfd_gemm: ldc %lld < N %lld", (long long)a.ldc, (long long)a.N);
  const int act = a.ep.act;
  MMFD_CHECK_ARG(act >= 0 && act <= MMFD_ACT_MUL_AUX, "mmfd_gemm: bad act %d", act);
  MMFD_CHECK_ARG(!(act == MMFD_ACT_GELU_BWD || act == MMFD_ACT_RELU_BWD || act == MMFD_ACT_MUL_AUX) ||
                     a.ep.aux != nullptr,
                 "mmfd_gemm: backward act needs aux");
  MMFD_CHECK_ARG(a.ep.dropout_p <= 0.f || a.ep.seed != nullptr, "mmfd_gemm: dropout needs seed");
  MMFD_CHECK_ARG(a.ep.dropout_p < 1.f, "mmfd_gemm: dropout p must be < 1");
  if (a.M == 0 || a.N == 0) return 0;
  MMFD_CHECK_ARG(a.K == 0 || (a.A && a.B), "mmfd_gemm: null operand");

  const EpiArgs e = make_epi(a);

  const bool bf = a.dtype == MMFD_BF16, cbf = a.c_dtype == MMFD_BF16;
  ConvGeom cg;
  if (const char* why = conv_geom(a, cg)) return mmfd_set_error(MMFD_ERR_INVALID, "mmfd_gemm: %s", why);
  if (cg.on && !mfma_ok(a))
    return mmfd_set_error(MMFD_ERR_UNSUPPORTED, "mmfd_gemm: conv with an unaligned / oversized B operand");
  // an operand whose fp32 copy was never written can only be read through its planes: refuse every
  // path that would read the fp32 copy (the simple kernel below included)
  if ((a.a_planes_only || a.b_planes_only) && (!mfma_ok(a) || !x6_plan(a).on))
    return mmfd_set_error(MMFD_ERR_UNSUPPORTED, "mmfd_gemm: an operand exists only as split planes, but this "
                          "product (M %lld N %lld K %lld) does not run on split operands", (long long)a.M,
                          (long long)a.N, (long long)a.K);
  if (!mfma_ok(a)) {
    const int64_t total = a.M * a.N;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
#define SIMPLE(T, TC)                                                                          \
  hipLaunchKernelGGL((gemm_simple_kernel<T, TC>), dim3(blocks), dim3(256), 0, s, (const T*)a.A, \
                     a.lda, a.trans_a, (const T*)a.B, a.ldb, a.trans_b, (TC*)a.C, a.ldc, a.M, a.N, \
                     a.K, a.alpha, e)
    if (bf) { if (cbf) SIMPLE(bf16, bf16); else SIMPLE(bf16, float); }
    else { if (cbf) SIMPLE(float, bf16); else SIMPLE(float, float); }
#undef SIMPLE
    MMFD_CHECK_LAUNCH("gemm_simple");
    return rowsum_fallback(a, a.workspace, a.workspace_bytes, s);
  }

  // split-operand fp32 GEMM only with the full workspace it asked for (else the fp32 MFMA path)
  X6Plan xp = x6_plan(a);
  if (xp.on) {  // (no workspace at all when both operands come split and there is no split-K)
    const int64_t wneed = mmfd_gemm_workspace_bytes(&a);
    if (wneed > 0 && (a.workspace == nullptr || a.workspace_bytes < wneed)) xp.on = false;
  }
  if (!xp.on && (a.a_planes_only || a.b_planes_only))
    return mmfd_set_error(MMFD_ERR_UNSUPPORTED, "mmfd_gemm: an operand exists only as split planes, but this "
                          "product (M %lld N %lld K %lld) does not run on split operands", (long long)a.M,
                          (long long)a.N, (long long)a.K);
  int64_t need = 0;
  int splits = choose_splits(a, &need, xp.on);
  if (!xp.on && splits > 1 && (a.workspace == nullptr || a.workspace_bytes < need + rowsum_ws_bytes(a, splits, use_g8(a)))) {
    // shrink to what the workspace allows
    const int64_t per = a.M * a.N * 4 + (a.a_rowsum ? a.M * 4 : 0);
    int fit = (a.workspace && per > 0) ? (int)std::min<int64_t>(a.workspace_bytes / per, 32) : 1;
    splits = fit > 1 ? std::min(splits, fit) : 1;
  }
  const int T = (bf || xp.on) ? 64 : 32;
  const bool xf = xp.on && x6_fused();
  const int nkt = (int)(xf ? (a.K + 31) / 32 : xp.on ? 6 * ((a.K + 63) / 64) : (a.K + T - 1) / T);
  const int tps = (nkt + splits - 1) / std::max(splits, 1);
  splits = tps > 0 ? (nkt + tps - 1) / tps : 1;
  if (splits < 1) splits = 1;
  // GELU_D / MUL_AUX off the four-wave kernel: raw sums to a slab, the reduce runs the epilogue
  const bool xs = ext_slab(a, splits, xp.on);  // (xp.on as decided above: the workspace held the planes)
  if (xs) {
    MMFD_CHECK_ARG(!a.a_rowsum, "mmfd_gemm: act %d with a_rowsum is not supported", act);
    MMFD_CHECK_ARG(a.workspace && a.workspace_bytes >= (int64_t)splits * a.M * a.N * 4,
                   "mmfd_gemm: act %d on this product needs a workspace of %lld bytes (mmfd_gemm_workspace_bytes)",
                   act, (long long)((int64_t)splits * a.M * a.N * 4));
  }
  float* ws = (splits > 1 || xs) ? (float*)a.workspace : nullptr;
  const bool g8 = use_g8(a);
  // fused row sums: G8 writes them directly (one split) or as per-split partials after the slabs
  // row-sum partials after the split-K slabs: [splits][column tiles][M] when the workspace holds
  // them (rs_mode 3), else the first column tile sums alone (per-split partials / direct)
  const int64_t gxt = (a.N + G8_BN - 1) / G8_BN;
  const int64_t slab_bytes = ws ? (int64_t)splits * a.M * a.N * 4 : 0;
  const int rs_parts3 = (int)(splits * gxt);
  const bool rs3 = a.a_rowsum && g8 && rs_parts3 > 1 && a.workspace &&
                   a.workspace_bytes >= slab_bytes + (int64_t)rs_parts3 * a.M * 4;
  float* rs_part = (a.a_rowsum && g8 && (rs3 || splits > 1)) ? (float*)((char*)a.workspace + slab_bytes) : nullptr;
  const int rs_mode = (!a.a_rowsum || !g8) ? 0 : (rs3 ? 3 : (splits > 1 ? 2 : 1));
  const int rs_nparts = rs_mode == 3 ? rs_parts3 : splits;
  float* rs_out = rs_mode >= 2 ? rs_part : a.a_rowsum;

  if (xp.on) {
    char* planes = (char*)a.workspace + align256((int64_t)(ws ? splits : 0) * a.M * a.N * 4 +
                                                 rowsum_ws_bytes(a, splits, true));
    const bf16* pa = (const bf16*)a.a_planes;
    const bf16* pb = (const bf16*)a.b_planes;
    if (!pa) {
      launch_split3((const float*)a.A, cg.on ? cg.C : a.lda, xp.rows_a, xp.cols_a, (bf16*)planes, s);
      pa = (const bf16*)planes;
      planes += align256(3 * xp.pa);
    }
    if (!pb) {
      launch_split3((const float*)a.B, a.ldb, xp.rows_b, xp.cols_b, (bf16*)planes, s);
      pb = (const bf16*)planes;
    }
    MMFD_CHECK_LAUNCH("split3");
    if (xf) {
      dispatch_x6f(a, e, ws, splits, tps, rs_out, rs_mode, s, pa, pb, X6Args{nkt, (uint32_t)xp.pa, (uint32_t)xp.pb}, cg);
    } else if (cg.on) {
      return mmfd_set_error(MMFD_ERR_UNSUPPORTED, "mmfd_gemm: conv on the segmented split-operand kernel");
    } else {
      const X6Args x6{(int)((a.K + 63) / 64), (uint32_t)xp.pa, (uint32_t)xp.pb};
      dispatch_g8<bf16, float>(a, e, ws, splits, tps, rs_out, rs_mode, s, &x6, pa, pb);
    }
  } else if (cg.on) {  // implicit convolution: the 256x128 kernel with the window-gathering A fill
    if (bf) { if (cbf) launch_conv_mfma<bf16, bf16>(a, e, ws, splits, tps, s, cg); else launch_conv_mfma<bf16, float>(a, e, ws, splits, tps, s, cg); }
    else { if (cbf) launch_conv_mfma<float, bf16>(a, e, ws, splits, tps, s, cg); else launch_conv_mfma<float, float>(a, e, ws, splits, tps, s, cg); }
  } else if (g8 && bf && cbf && !ws && mmfd_gemmx::launch_g4(a, e, splits, s)) {
  } else if (g8 && bf) { if (cbf) dispatch_g8<bf16, bf16>(a, e, ws, splits, tps, rs_out, rs_mode, s); else dispatch_g8<bf16, float>(a, e, ws, splits, tps, rs_out, rs_mode, s); }
  else if (g8) dispatch_g8<float, float>(a, e, ws, splits, tps, rs_out, rs_mode, s);
  else if (bf) { if (cbf) dispatch_layout<bf16, bf16>(a, e, ws, splits, tps, s); else dispatch_layout<bf16, float>(a, e, ws, splits, tps, s); }
  else { if (cbf) dispatch_layout<float, bf16>(a, e, ws, splits, tps, s); else dispatch_layout<float, float>(a, e, ws, splits, tps, s); }
  MMFD_CHECK_LAUNCH("gemm_mfma");
  if (ws) {
    const int64_t total = a.M * a.N;
    // the row sums' partials (rs_mode 2 / 3) are reduced by the same launch
    const float* rsp = rs_mode >= 2 ? rs_part : nullptr;
    if (e.vec && a.N % 8 == 0) {
      // split ranges per group: up to 8, while the threads stay under ~2^19 (2,048 per CU)
      const int64_t groups = total / 8;
      int P = 1;
      while (P < 8 && 2 * P <= splits && groups * P < ((int64_t)1 << 19)) P *= 2;
      const int G = 256 / P;
      const int blocks = (int)std::min<int64_t>(std::max<int64_t>((groups + G - 1) / G, (a.M + 255) / 256), 16384);
#define SKR(TC, PP) hipLaunchKernelGGL((splitk_reduce8_kernel<TC, PP>), dim3(blocks), dim3(256), 0, s, ws, splits, \
                                       (TC*)a.C, a.ldc, a.M, a.N, e, rsp, rs_nparts, a.a_rowsum, a.a_rowsum_beta)
      if (cbf) { if (P == 8) SKR(bf16, 8); else if (P == 4) SKR(bf16, 4); else if (P == 2) SKR(bf16, 2); else SKR(bf16, 1); }
      else { if (P == 8) SKR(float, 8); else if (P == 4) SKR(float, 4); else if (P == 2) SKR(float, 2); else SKR(float, 1); }
#undef SKR
      MMFD_CHECK_LAUNCH("splitk_reduce");
    } else {
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
    if (cbf) hipLaunchKernelGGL((splitk_reduce_kernel<bf16>), dim3(blocks), dim3(256), 0, s, ws, splits, (bf16*)a.C, a.ldc,
                                a.M, a.N, e, rsp, rs_nparts, a.a_rowsum, a.a_rowsum_beta);
    else hipLaunchKernelGGL((splitk_reduce_kernel<float>), dim3(blocks), dim3(256), 0, s, ws, splits, (float*)a.C, a.ldc,
                            a.M, a.N, e, rsp, rs_nparts, a.a_rowsum, a.a_rowsum_beta);
    MMFD_CHECK_LAUNCH("splitk_reduce");
    }
  } else if (rs_mode == 3) {  // no split-K: only the column tiles' row-sum partials to reduce
    hipLaunchKernelGGL(mmfd_reduce_partials_kernel, dim3((unsigned)((a.M + 63) / 64)), dim3(1024), 0, s,
                       (const float*)rs_part, rs_nparts, a.M, a.M, a.a_rowsum, a.a_rowsum_beta);
    MMFD_CHECK_LAUNCH("rowsum_reduce");
  }
  if (a.a_rowsum && !g8) {
    char* base = (char*)a.workspace + (ws ? (int64_t)splits * a.M * a.N * 4 : 0);
    const int64_t left = a.workspace_bytes - (ws ? (int64_t)splits * a.M * a.N * 4 : 0);
    return rowsum_fallback(a, base, left, s);
  }
  return 0;
}

extern "C" int mmfd_split3(int64_t rows, int64_t cols, const float* x, int64_t ld, void* planes, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(rows >= 0 && cols >= 0 && ld >= cols, "mmfd_split3: bad shape");
  MMFD_CHECK_ARG(cols % 8 == 0 && ld % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)planes & 15) == 0,
                 "mmfd_split3: cols must be a multiple of 8 and rows 16-B aligned");
  MMFD_CHECK_ARG(rows * (cols / 8) < (1ll << 32) && rows * ld < (1ll << 31), "mmfd_split3: matrix too large");
  if (rows == 0 || cols == 0) return 0;
  launch_split3(x, ld, rows, cols, (bf16*)planes, (hipStream_t)stream);
  MMFD_CHECK_LAUNCH("split3");
  return 0;
}

// ------------------------------------------------------------------------------------------------
// column sums (bias gradients), deterministic two-pass
// ------------------------------------------------------------------------------------------------
namespace {
// pass 1 (vector path): block = 4 waves x 64 lanes; a lane owns one 16-B chunk of columns, the 4
// waves stride over the block's row slab; the waves' partials are combined in LDS.
template <typename T>
__global__ void __launch_bounds__(256) colsum_partial_vec_kernel(const T* __restrict__ X, int64_t ldx, int64_t M,
                                                                 int64_t N, int64_t rows_per_block,
                                                                 float* __restrict__ part) {
  constexpr int EPC = 16 / sizeof(T);
  __shared__ float red[4][64 * EPC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = ((int64_t)blockIdx.x * 64 + lane) * EPC;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float acc[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) acc[e] = 0.f;
  if (col < N) {
    for (int64_t r = r0 + wave; r < r1; r += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(X + r * ldx + col);
      const T* t = reinterpret_cast<const T*>(&v);
#pragma unroll
      for (int e = 0; e < EPC; ++e) acc[e] += to_f32(t[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < EPC; ++e) red[wave][lane * EPC + e] = acc[e];
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * EPC; i += 256) {
    const int64_t c = (int64_t)blockIdx.x * 64 * EPC + i;
    if (c < N) part[(int64_t)blockIdx.y * N + c] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}
template <typename T>
__global__ void colsum_partial_kernel(const T* __restrict__ X, int64_t ldx, int64_t M, int64_t N,
                                      int64_t rows_per_block, float* __restrict__ part) {
  const int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += to_f32(X[r * ldx + col]);
  part[(int64_t)blockIdx.y * N + col] = s;
}
}  // namespace

// pass 2, shared with the LayerNorm backward: out[c] = beta*out[c] + sum_p part[p*stride + c];
// block = 64 columns x 16 waves splitting the partials (4 independent loads in flight per lane),
// combined through LDS in a fixed order (deterministic).
__global__ void __launch_bounds__(1024) mmfd_reduce_partials_kernel(const float* __restrict__ part, int nparts,
                                                                    int64_t stride, int64_t N, float* __restrict__ out,
                                                                    float beta) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    int p = wave;
    for (; p + 48 < nparts; p += 64) {
      s0 += part[(int64_t)p * stride + col];
      s1 += part[(int64_t)(p + 16) * stride + col];
      s2 += part[(int64_t)(p + 32) * stride + col];
      s3 += part[(int64_t)(p + 48) * stride + col];
    }
    for (; p < nparts; p += 16) s0 += part[(int64_t)p * stride + col];
  }
  red[wave][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (wave == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    out[col] = (beta != 0.f ? beta * out[col] : 0.f) + t;
  }
}

extern "C" int mmfd_colsum(int dtype, int64_t M, int64_t N, const void* X, int64_t ldx, float* out,
                           float beta, void* workspace, int64_t workspace_bytes, mmfd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  MMFD_CHECK_ARG(dtype == MMFD_F32 || dtype == MMFD_BF16, "mmfd_colsum: bad dtype");
  if (N == 0) return 0;
  int nparts = (int)std::min<int64_t>(256, std::max<int64_t>(1, M / 64));
  if (workspace_bytes < (int64_t)nparts * N * 4) nparts = (int)(workspace_bytes / (N * 4));
  MMFD_CHECK_ARG(nparts >= 1 && workspace, "mmfd_colsum: workspace too small");
  const int64_t rpb = (M + nparts - 1) / nparts;
  const int epc = dtype == MMFD_BF16 ? 8 : 4;
  const bool vec = (N % epc) == 0 && (ldx % epc) == 0 && ((uintptr_t)X & 15) == 0;
  if (vec) {
    dim3 g1((unsigned)((N / epc + 63) / 64), (unsigned)nparts);
    if (dtype == MMFD_BF16)
      hipLaunchKernelGGL((colsum_partial_vec_kernel<bf16>), g1, dim3(256), 0, s, (const bf16*)X, ldx, M, N, rpb, (float*)workspace);
    else
      hipLaunchKernelGGL((colsum_partial_vec_kernel<float>), g1, dim3(256), 0, s, (const float*)X, ldx, M, N, rpb, (float*)workspace);
  } else {
    dim3 g1((unsigned)((N + 255) / 256), (unsigned)nparts);
    if (dtype == MMFD_BF16)
      hipLaunchKernelGGL((colsum_partial_kernel<bf16>), g1, dim3(256), 0, s, (const bf16*)X, ldx, M, N, rpb, (float*)workspace);
    else
      hipLaunchKernelGGL((colsum_partial_kernel<float>), g1, dim3(256), 0, s, (const float*)X, ldx, M, N, rpb, (float*)workspace);
  }
  hipLaunchKernelGGL(mmfd_reduce_partials_kernel, dim3((unsigned)((N + 63) / 64)), dim3(1024), 0, s,
                     (const float*)workspace, nparts, N, N, out, beta);
  MMFD_CHECK_LAUNCH("colsum");
  return 0;
}
