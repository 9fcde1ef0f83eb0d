// Split-operand fp32 GEMM, four waves per 256x256 tile with the accumulators in AGPRs
// (gemm256_x6w_kernel) and its launcher.
//
// The same product as gemm256_x6f_kernel (gemm_x6f.hip): A and B arrive as bf16 planes
// x = hi + mid + lo, and every 32-deep K-step adds the six plane products mid*mid, hi*lo, lo*hi,
// hi*mid, mid*hi, hi*hi (A plane * B plane, small first) straight into the fp32 accumulators — the
// same operations in the same order per accumulator element, so the two kernels return identical
// bits. What differs is the schedule:
//
//   x6f: 8 waves (two per SIMD) as 2 x 4, 64x32 quadrants, the two wave rows handing the MFMA pipe
//        to each other at a workgroup barrier every 48 MFMAs (8 hand-offs per K-step): a K-step
//        measured ~8,100 cycles against 6,144 of MFMA issue.
//   x6w: 4 waves (one per SIMD) as 2 x 2, each owning a 128 x 128 block = 8 x 8 accumulator tiles
//        (256 fp32 per lane) held in the AGPR half of the 512-entry register file (this file is
//        built without -amdgpu-mfma-vgpr-form, so the MFMAs take the AGPR form), the fragments in
//        VGPRs. A wave issues its 384 MFMAs of a K-step back to back (dependent MFMAs on one
//        accumulator issue at the full rate: srcC forwarding, tools/mb/mfma_rate.hip) with the LDS
//        reads of the next A subtile interleaved; two workgroup barriers per K-step.
//
// LDS (144 KB): A double-buffered (2 buffers x 2 halves x 3 planes x 8 KB), B single-buffered
// (2 halves x 3 planes x 8 KB); the slot images are the x6f ones (XfImg). Per K-step t:
//   barrier 1  A(t), B(t) landed (own vmcnt(0) + barrier); every wave is past step t-1, so the other
//              A buffer is free: issue A(t+1) into it
//   B reads    the wave's whole B half (8 fragments x 3 planes) and A subtile 0, in the order the
//              first subtile's products consume them
//   subtile i  A subtile i+1 read, then 48 MFMAs (8 B fragments x 6 plane products)
//   barrier 2  (after subtile 1: every wave holds B(t) in registers) issue B(t+1) into the B slots
// =================================================================================================
#include "common.h"
#include <algorithm>
#include <type_traits>

#include "gemm_tiles.h"

namespace {

// Diagnostic builds only (tools/w4_stamps.py): -DMMFD_W4_STAMPS writes s_memtime stamps of one
// mid-loop K-step and of the tile phases to a buffer no computation reads; -DW4_DIAG=n removes one
// piece of the schedule (results wrong by design): 1 = the B-refill barrier, 2 = the loop's DMA,
// 3 = the epilogue's stores (accumulators staged, nothing written)
#ifndef W4_DIAG
#define W4_DIAG 0
#endif
#ifdef MMFD_W4_STAMPS
__device__ uint64_t w4_stamps[4096 * 4 * 24];
#define W4_TSTAMP(k)                                                                                  \
  do {                                                                                                \
    const uint64_t t__ = __builtin_amdgcn_s_memtime();                                               \
    const int64_t b__ = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;                                \
    if (lane == 0 && b__ < 4096) w4_stamps[(b__ * 4 + wave) * 24 + (k)] = t__;                       \
  } while (0)
#define W4_STAMP(k)                                                                                   \
  do {                                                                                                \
    if (t == w4_t) W4_TSTAMP(k);                                                                      \
  } while (0)
#else
#define W4_STAMP(k) do { } while (0)
#define W4_TSTAMP(k) do { } while (0)
#endif

constexpr int W4_NT = 256;
constexpr int W4_LDS = 18 * XF_SLOT;  // 147456: A 12 slots + B 6 slots; epilogue staging 128 x 260 fp32 fits
static_assert(128 * (G8_BN + 4) * 4 <= W4_LDS, "epilogue staging");

__device__ __forceinline__ void w4_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// one K-step's six plane products of A subtile a (planes a[0..2] = hi, mid, lo) against the wave's
// eight B fragments, jj-major (each accumulator's six products back to back)
__device__ __forceinline__ void w4_mma(f32x4 (&acc)[8], const uint4 (&a)[3], const uint4 (&b)[8][3]) {
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    Mma<bf16>::run(acc[jj], b[jj][1], a[1]);  // mid * mid
    Mma<bf16>::run(acc[jj], b[jj][2], a[0]);  // A hi * B lo
    Mma<bf16>::run(acc[jj], b[jj][0], a[2]);  // A lo * B hi
    Mma<bf16>::run(acc[jj], b[jj][1], a[0]);  // A hi * B mid
    Mma<bf16>::run(acc[jj], b[jj][0], a[1]);  // A mid * B hi
    Mma<bf16>::run(acc[jj], b[jj][0], a[0]);  // hi * hi
  }
}

// Epilogue: two passes of 128 rows; in pass mq the two waves of wave row mq stage their 128 x 128
// blocks (fp32, [128][260]) and all 256 threads apply the epilogue to 8-column chunks (16 rows per
// thread) with 16-B accesses — g8_epilogue's non-PRE paths for 4 waves and fp32 C.
__device__ __forceinline__ void w4_epilogue(f32x4 (&acc)[8][8], char* smem, const EpiArgs& e, float* __restrict__ C,
                                            int64_t ldc, float* __restrict__ ws, int split, int64_t M, int64_t N,
                                            float alpha, int64_t m0, int64_t n0, int tid, int lane, int wr, int wc) {
  constexpr int LDC = G8_BN + 4;
  float* ct = reinterpret_cast<float*>(smem);
  const int g = lane >> 4, ci = lane & 15;
  const uint32_t seed = (!ws && e.p > 0.0f) ? mmfd_hash_key(*e.seed, e.salt) : 0u;
  float* slab = ws ? ws + (int64_t)split * M * N : nullptr;
  auto stage = [&](int mq) {
    if (wr == mq) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          *reinterpret_cast<f32x4*>(ct + (i * 16 + ci) * LDC + wc * 128 + (jj >> 1) * 32 + 8 * g + 4 * (jj & 1)) =
              acc[i][jj];
    }
    __syncthreads();
  };
  if (!slab && e.vec && m0 + G8_BM <= M && n0 + G8_BN <= N) {
    const int c8 = (tid % (G8_BN / 8)) * 8;
    const int64_t col = n0 + c8;
    float bia[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) bia[u] = e.bias ? e.bias[col + u] : 0.f;
    const bool bwd_act = e.act == MMFD_ACT_GELU_BWD || e.act == MMFD_ACT_RELU_BWD;
    const bool fwd_act = e.act == MMFD_ACT_GELU || e.act == MMFD_ACT_RELU;
    constexpr int IT = 128 * (G8_BN / 8) / W4_NT;  // 16 rows per thread
    const int lr0 = tid / (G8_BN / 8);
    const int64_t rstep = W4_NT / (G8_BN / 8);     // 8 rows between a thread's rows
#pragma unroll
    for (int mq = 0; mq < 2; ++mq) {
      stage(mq);
      const int64_t rbase = m0 + mq * 128;
      const int oc = lr0 * (int)ldc + c8, orr = lr0 * (int)e.ldr + c8, oa = lr0 * (int)e.ldaux + c8;
      float* cp = C ? C + rbase * ldc + n0 + oc : nullptr;
      const float* rp = e.residual ? reinterpret_cast<const float*>(e.residual) + rbase * e.ldr + n0 + orr : nullptr;
      const float* xp = bwd_act ? reinterpret_cast<const float*>(e.aux) + rbase * e.ldaux + n0 + oa : nullptr;
      float* ap = (fwd_act && e.aux) ? reinterpret_cast<float*>(e.aux) + rbase * e.ldaux + n0 + oa : nullptr;
      const uint64_t hidx = (uint64_t)(rbase + lr0) * (uint64_t)N + (uint64_t)col;
      const int64_t cs = rstep * ldc, rs = rstep * e.ldr, xs = rstep * e.ldaux;
      const float* src = ct + lr0 * LDC + c8;
      constexpr int GI = 2;
#pragma unroll
      for (int k0 = 0; k0 < IT; k0 += GI) {
        Raw8<float> rres[GI], raux[GI], rc[GI];
#pragma unroll
        for (int k = 0; k < GI; ++k) {
          const int kk = k0 + k;
          if (rp) rres[k].load(rp + kk * rs);
          if (xp) raux[k].load(xp + kk * xs);
          if (e.beta != 0.f) rc[k].load(cp + kk * cs);
        }
#pragma unroll
        for (int k = 0; k < GI; ++k) {
          const int kk = k0 + k;
          const float4 a4 = *reinterpret_cast<const float4*>(src + kk * rstep * LDC);
          const float4 b4 = *reinterpret_cast<const float4*>(src + kk * rstep * LDC + 4);
          float z[8] = {a4.x, a4.y, a4.z, a4.w, b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] = fmaf(alpha, z[u], bia[u]);
          float t[8];
          if (rp && e.res_first) {
            rres[k].get(t);
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] += t[u];
          }
          if (fwd_act) {
            if (ap) V8<float>::store(ap + kk * xs, z);
            if (e.act == MMFD_ACT_GELU) {
#pragma unroll
              for (int u = 0; u < 8; ++u) z[u] = gelu_f(z[u]);
            } else {
#pragma unroll
              for (int u = 0; u < 8; ++u) z[u] = fmaxf(z[u], 0.f);
            }
          } else if (xp) {
            raux[k].get(t);
            if (e.act == MMFD_ACT_GELU_BWD) {
#pragma unroll
              for (int u = 0; u < 8; ++u) z[u] *= gelu_grad_f(t[u]);
            } else {
#pragma unroll
              for (int u = 0; u < 8; ++u) z[u] = t[u] > 0.f ? z[u] : 0.f;
            }
          } else if (e.act >= MMFD_ACT_TANH) {
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] = act_tail_f(e.act, z[u]);
          }
          if (e.p > 0.f) {
            const uint64_t base = hidx + (uint64_t)(kk * rstep) * (uint64_t)N;
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] = (mmfd_hash_k(seed, base + u) < e.thr) ? 0.f : z[u] * e.keep_scale;
          }
          if (rp && !e.res_first) {
            rres[k].get(t);
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] += t[u];
          }
          if (e.beta != 0.f) {
            rc[k].get(t);
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] = fmaf(e.beta, t[u], z[u]);
          }
          if (e.pl) {
            planes_store8(e, N, rbase + lr0 + kk * rstep, col, z);
            if (!e.c_out) continue;
          }
          V8<float>::store(cp + kk * cs, z);
        }
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int mq = 0; mq < 2; ++mq) {
    stage(mq);
    const int64_t rbase = m0 + mq * 128;
    for (int idx = tid; idx < 128 * (G8_BN / 8); idx += W4_NT) {
      const int lr = idx / (G8_BN / 8), c8 = (idx % (G8_BN / 8)) * 8;
      const int64_t row = rbase + lr, col = n0 + c8;
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
          for (int u = 0; u < 8; ++u)
            if (col + u < N) slab[row * N + col + u] = vv[u];
        }
      } else if (full && e.vec) {
        epilogue_store8<float>(e, C, ldc, N, row, col, vv, seed);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (col + u < N) epilogue_store<float>(e, C, ldc, N, row, col + u, vv[u], seed);
      }
    }
    __syncthreads();
  }
}

// Epilogue straight from the accumulators (full tiles): accumulator pair (i, 2q), (i, 2q + 1) gives
// lane (g, ci) row i * 16 + ci, the 8 consecutive columns q * 32 + 8 g .. + 7 of the wave's block —
// a wave's store covers 16 rows x 128 B (whole cache lines), so no LDS staging and no workgroup
// barrier: the four waves run their epilogues independently. Per accumulator row the operand
// stream loads (residual / saved pre-activation / C) of its four column groups are issued before
// any math. Same operations and order per element as epilogue_store8 / g8_epilogue.
struct W4Epi {
  const EpiArgs& e;
  float* C;
  int64_t ldc, N;
  float alpha;
  int64_t row0, colg;
  uint32_t seed;
  bool bwd_act, fwd_act;
  // one accumulator row i (compile time: a run-time index would put the accumulators in scratch)
  template <int I>
  __device__ __forceinline__ void row(f32x4 (&acc)[8][8]) const {
    if constexpr (I < 8) {
      const int64_t r = row0 + I * 16;
      const float* rp = reinterpret_cast<const float*>(e.residual);
      const float* xp = bwd_act ? reinterpret_cast<const float*>(e.aux) : nullptr;
      float* ap = (fwd_act && e.aux) ? reinterpret_cast<float*>(e.aux) : nullptr;
      Raw8<float> rres[4], raux[4], rc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t col = colg + q * 32;
        if (rp) rres[q].load(rp + r * e.ldr + col);
        if (xp) raux[q].load(xp + r * e.ldaux + col);
        if (e.beta != 0.f) rc[q].load(C + r * ldc + col);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t col = colg + q * 32;
        const f32x4 a4 = acc[I][2 * q], b4 = acc[I][2 * q + 1];
        float z[8] = {a4[0], a4[1], a4[2], a4[3], b4[0], b4[1], b4[2], b4[3]};
        if (e.bias) {
          const float4 b0 = *reinterpret_cast<const float4*>(e.bias + col);
          const float4 b1 = *reinterpret_cast<const float4*>(e.bias + col + 4);
          const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] = fmaf(alpha, z[u], bb[u]);
        } else {
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] = fmaf(alpha, z[u], 0.f);
        }
        float t[8];
        if (rp && e.res_first) {
          rres[q].get(t);
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] += t[u];
        }
        if (fwd_act) {
          if (ap) V8<float>::store(ap + r * e.ldaux + col, z);
          if (e.act == MMFD_ACT_GELU) {
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] = gelu_f(z[u]);
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] = fmaxf(z[u], 0.f);
          }
        } else if (xp) {
          raux[q].get(t);
          if (e.act == MMFD_ACT_GELU_BWD) {
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] *= gelu_grad_f(t[u]);
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] = t[u] > 0.f ? z[u] : 0.f;
          }
        } else if (e.act >= MMFD_ACT_TANH) {
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] = act_tail_f(e.act, z[u]);
        }
        if (e.p > 0.f) {
          const uint64_t base = (uint64_t)r * (uint64_t)N + (uint64_t)col;
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] = (mmfd_hash_k(seed, base + u) < e.thr) ? 0.f : z[u] * e.keep_scale;
        }
        if (rp && !e.res_first) {
          rres[q].get(t);
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] += t[u];
        }
        if (e.beta != 0.f) {
          rc[q].get(t);
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] = fmaf(e.beta, t[u], z[u]);
        }
        if (e.pl) {
          planes_store8(e, N, r, col, z);
          if (!e.c_out) continue;
        }
        V8<float>::store(C + r * ldc + col, z);
      }
      row<I + 1>(acc);
    }
  }
};

__device__ __forceinline__ void w4_epilogue_direct(f32x4 (&acc)[8][8], const EpiArgs& e, float* __restrict__ C,
                                                   int64_t ldc, float* __restrict__ slab, int64_t N, float alpha,
                                                   int64_t r0, int64_t c0, int lane) {
  const int g = lane >> 4, ci = lane & 15;
  const int64_t row0 = r0 + ci, colg = c0 + 8 * g;
  if (slab) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float* d = slab + (row0 + i * 16) * N + colg + q * 32;
        const f32x4 a = acc[i][2 * q], b = acc[i][2 * q + 1];
        *reinterpret_cast<float4*>(d) = make_float4(alpha * a[0], alpha * a[1], alpha * a[2], alpha * a[3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(alpha * b[0], alpha * b[1], alpha * b[2], alpha * b[3]);
      }
    return;
  }
  const W4Epi ep{e, C, ldc, N, alpha, row0, colg, e.p > 0.0f ? mmfd_hash_key(*e.seed, e.salt) : 0u,
                 e.act == MMFD_ACT_GELU_BWD || e.act == MMFD_ACT_RELU_BWD, e.act == MMFD_ACT_GELU || e.act == MMFD_ACT_RELU};
  ep.row<0>(acc);
}

template <int TA, int TB>
__global__ void __launch_bounds__(W4_NT, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm256_x6w_kernel(const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb,
                   float* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K,
                   float alpha, int steps_per_split, EpiArgs e, float* __restrict__ rs_out, float rs_beta,
                   int rs_mode, X6Args x6) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int gx = gridDim.x, gy = gridDim.y;
  // XCD-aware order over the whole grid, split-K index included (see gemm256_kernel)
  const int lt = xcd_remap((blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x, gx * gy * gridDim.z);
  const int split = lt / (gx * gy);
  const int tile = lt - split * (gx * gy);
  const int trow = tile / gx, tcol = tile - trow * gx;
  const int64_t m0 = (int64_t)trow * G8_BM, n0 = (int64_t)tcol * G8_BN;
  const int nst = x6.nkt;  // 32-deep K-steps in all
  const int st0 = split * steps_per_split;
  const int nk = min(nst, st0 + steps_per_split) - st0;
  W4_TSTAMP(16);
#ifdef MMFD_W4_STAMPS
  const int w4_t = min(4, nk - 1);
#endif

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A, 3 * (int64_t)x6.pa);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(B, 3 * (int64_t)x6.pb);
  // each wave fills two of the eight 1-KB pieces of every slot: pieces 2w and 2w + 1
  XfFill<TA> fa[2][2];
  XfFill<TB> fb[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fa[h][j].init(lda, m0 + h * 128, M, 2 * wave + j, lane);
      fb[h][j].init(ldb, n0 + h * 128, N, 2 * wave + j, lane);
    }
  auto aslot = [&](int buf, int h, int p) -> char* { return smem + ((buf * 2 + h) * 3 + p) * XF_SLOT; };
  auto bslot = [&](int h, int p) -> char* { return smem + (12 + h * 3 + p) * XF_SLOT; };
  auto issue_a = [&](int t) {
    const int64_t k0 = (int64_t)(st0 + t) * XF_BK;
    const uint32_t so = (uint32_t)(k0 * (TA == 0 ? 1 : lda) * 2);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fa[h][j].issue(rsa, aslot(t & 1, h, p), so + (uint32_t)p * x6.pa, k0, K, 2 * wave + j);
  };
  auto issue_b = [&](int t) {
    const int64_t k0 = (int64_t)(st0 + t) * XF_BK;
    const uint32_t so = (uint32_t)(k0 * (TB == 0 ? 1 : ldb) * 2);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[h][j].issue(rsb, bslot(h, p), so + (uint32_t)p * x6.pb, k0, K, 2 * wave + j);
  };

  // fused row sums of op(A) (bias gradient), per K-step as gemm256_kernel: wave wc sums the A
  // subtiles i with (i & 1) == wc of its half from the fragments in registers
  const int rs_cols = rs_mode == 3 ? gx : 1;
  const bool do_rs = rs_mode != 0 && tcol < rs_cols;
  float rsum[4] = {0.f, 0.f, 0.f, 0.f};
  int rs_ph = (st0 % rs_cols);

  if (nk > 0) {
    issue_a(0);
    issue_b(0);
  }
  // DMA piece k (0..11) of one operand's K-step: half k / 6, plane (k / 2) % 3, wave piece k % 2
  auto dma_a = [&](int t, int k) {
    const int h = k / 6, p = (k >> 1) % 3, j = k & 1;
    const int64_t k0 = (int64_t)(st0 + t) * XF_BK;
    const uint32_t so = (uint32_t)(k0 * (TA == 0 ? 1 : lda) * 2) + (uint32_t)p * x6.pa;
    fa[h][j].issue(rsa, aslot(t & 1, h, p), so, k0, K, 2 * wave + j);
  };
  auto dma_b = [&](int t, int k) {
    const int h = k / 6, p = (k >> 1) % 3, j = k & 1;
    const int64_t k0 = (int64_t)(st0 + t) * XF_BK;
    const uint32_t so = (uint32_t)(k0 * (TB == 0 ? 1 : ldb) * 2) + (uint32_t)p * x6.pb;
    fb[h][j].issue(rsb, bslot(h, p), so, k0, K, 2 * wave + j);
  };
  uint4 fbr[8][3], far[2][3];
  for (int t = 0; t < nk; ++t) {
    bool rs_t = false;
    if (do_rs) {
      rs_t = rs_ph == tcol;
      rs_ph = rs_ph + 1 == rs_cols ? 0 : rs_ph + 1;
    }
    W4_STAMP(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own pieces of A(t), B(t)
    W4_STAMP(1);
    w4_barrier();
    W4_STAMP(2);
    const bool more = t + 1 < nk;
    const char* abase = aslot(t & 1, wr, 0);
    // The step as 64 groups (A subtile i, B fragment jj) of six products, in this order, with the
    // LDS reads one group ahead of their first use and the 24 LDS-DMA pieces of step t+1 spread one
    // per group (A(t+1) over subtiles 0-1; B(t+1) over subtiles 2-3, after barrier 2): a wave issues
    // its MFMAs back to back, and a DMA instruction never stalls more than one group's products.
    {
      int ln = lane;
      asm volatile("" : "+v"(ln));  // fragment addresses computed here, not kept live across the loop
#pragma unroll
      for (int p = 0; p < 3; ++p) far[0][p] = xf_frag_a<TA>(abase + p * XF_SLOT, 0, ln);
#pragma unroll
      for (int p = 0; p < 3; ++p) fbr[0][p] = xf_frag_b<TB>(bslot(wc, p), 0, 0, ln);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        {
          int ln = lane;
          asm volatile("" : "+v"(ln));
          if (i == 0 && jj + 1 < 8) {
#pragma unroll
            for (int p = 0; p < 3; ++p) fbr[jj + 1][p] = xf_frag_b<TB>(bslot(wc, p), (jj + 1) >> 1, (jj + 1) & 1, ln);
          }
          if (i + 1 < 8 && jj == (i == 0 ? 4 : 0)) {
#pragma unroll
            for (int p = 0; p < 3; ++p) far[(i + 1) & 1][p] = xf_frag_a<TA>(abase + p * XF_SLOT, i + 1, ln);
          }
        }
        if (jj == 0 && rs_t && (i & 1) == wc) {
          const uint4* fr = far[i & 1];
          rsum[i >> 1] += (g8_sum16b<bf16>(fr[0]) + g8_sum16b<bf16>(fr[1])) + g8_sum16b<bf16>(fr[2]);
        }
        const uint4* a = far[i & 1];
        const uint4* b = fbr[jj];
        Mma<bf16>::run(acc[i][jj], b[1], a[1]);  // mid * mid
        Mma<bf16>::run(acc[i][jj], b[2], a[0]);  // A hi * B lo
        Mma<bf16>::run(acc[i][jj], b[0], a[2]);  // A lo * B hi
        Mma<bf16>::run(acc[i][jj], b[1], a[0]);  // A hi * B mid
        Mma<bf16>::run(acc[i][jj], b[0], a[1]);  // A mid * B hi
        Mma<bf16>::run(acc[i][jj], b[0], a[0]);  // hi * hi
        if (W4_DIAG != 2 && more) {
          const int gidx = i * 8 + jj;
          if (gidx < 12) dma_a(t + 1, gidx);                    // the other A buffer (free since barrier 1)
          else if (gidx >= 16 && gidx < 28) dma_b(t + 1, gidx - 16);  // the B slots (free since barrier 2)
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (i == 0) W4_STAMP(3);
      if (i == 1) {
        // every wave holds B(t) in registers: the B slots may be refilled
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        W4_STAMP(4);
        if (W4_DIAG != 1) w4_barrier();
        W4_STAMP(5);
      }
    }
    W4_STAMP(6);
  }
  W4_TSTAMP(17);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (do_rs) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      rsum[m] += __shfl_xor(rsum[m], 16, 64);
      rsum[m] += __shfl_xor(rsum[m], 32, 64);
    }
    if (lane < 16) {
      float* dst = rs_mode == 1 ? rs_out : rs_out + (int64_t)(split * rs_cols + tcol) * M;
      const float bt = rs_mode == 1 ? rs_beta : 0.f;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t r = m0 + wr * 128 + (2 * m + wc) * 16 + lane;
        if (r < M) dst[r] = (bt != 0.f ? bt * dst[r] : 0.f) + rsum[m];
      }
    }
  }
  W4_TSTAMP(18);
  float* slab = ws ? ws + (int64_t)split * M * N : nullptr;
  const bool full = m0 + G8_BM <= M && n0 + G8_BN <= N;
  if (W4_DIAG != 3 && full && (slab ? (N % 4) == 0 : e.vec != 0)) {
    w4_epilogue_direct(acc, e, C, ldc, slab, N, alpha, m0 + wr * 128, n0 + wc * 128, lane);
  } else if (W4_DIAG == 3) {
    float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) *reinterpret_cast<f32x4*>(ct + ((wave * 64 + i * 8 + jj) * 64 + lane) * 4 % 30000) = acc[i][jj];
  } else {
    w4_epilogue(acc, smem, e, C, ldc, ws, split, M, N, alpha, m0, n0, tid, lane, wr, wc);
  }
#ifdef MMFD_W4_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  W4_TSTAMP(19);
#endif
}

}  // namespace

#ifdef MMFD_W4_STAMPS
extern "C" int mmfd_debug_w4_stamps(void* host_dst, int64_t bytes) {
  return (int)hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(w4_stamps), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
#endif

namespace mmfd_gemmx {
template <int TA, int TB>
void launch_x6w(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int sps, float* rs_out,
                int rs_mode, hipStream_t s, const void* pa, const void* pb, X6Args x6) {
  dim3 grid((unsigned)((a.N + G8_BN - 1) / G8_BN), (unsigned)((a.M + G8_BM - 1) / G8_BM), (unsigned)splits);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_x6w_kernel<TA, TB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, W4_LDS) == hipSuccess;
  }();
  (void)attr;
  const int64_t lda = TA == 0 ? a.K : a.M, ldb = TB == 0 ? a.K : a.N;  // the planes' stored column count
  hipLaunchKernelGGL((gemm256_x6w_kernel<TA, TB>), grid, dim3(W4_NT), W4_LDS, s, (const bf16*)pa, lda, (const bf16*)pb,
                     ldb, (float*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, sps, e, rs_out, a.a_rowsum_beta, rs_mode, x6);
}
void dispatch_x6w(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int sps, float* rs_out,
                  int rs_mode, hipStream_t s, const void* pa, const void* pb, X6Args x6) {
  if (!a.trans_a && !a.trans_b) launch_x6w<0, 0>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
  else if (!a.trans_a && a.trans_b) launch_x6w<0, 1>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
  else if (a.trans_a && !a.trans_b) launch_x6w<1, 0>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
  else launch_x6w<1, 1>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
}
}  // namespace mmfd_gemmx
