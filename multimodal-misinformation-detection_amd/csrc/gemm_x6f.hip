// Split-operand fp32 GEMM, fused planes (gemm256_x6f_kernel) and its launcher; the shared 256x256
// pieces (LDS-DMA fills, B fragment gather, epilogue) are in gemm_tiles.h.
#include "common.h"
#include <algorithm>
#include <type_traits>

#include "gemm_tiles.h"

namespace {

// =================================================================================================
// Split-operand fp32 GEMM with the three planes of each operand staged together ("fused planes").
// A and B arrive as bf16 planes x = hi + mid + lo (split3_kernel). For every 32-deep K-step the
// stage holds all three planes of both operands, so each 16x16x32 fragment read from LDS feeds
// several of the six products: per (subtile, K-step) the wave runs the chain
//   t = mid*mid; t += hi*lo; t += lo*hi; t += hi*mid; t += mid*hi; t += hi*hi   (A plane * B plane)
// from t = 0 and adds t to the fp32 accumulator with one v_add per element. Against the segmented
// kernel (gemm256_kernel<X6>: the K loop six times, one plane pair per pass) this halves the
// L2->LDS bytes (each plane loaded once per tile instead of 2x on average) and the LDS fragment
// reads per MFMA; the accumulator takes K/32 round-to-nearest fp32 adds at full scale (the chain's
// own MFMA-internal rounding happens at the scale of one K-step's partial sum), so the result is at
// least as close to the exact product as the segmented kernel's.
//
// Geometry: the 256x256 tile, 8 waves as 2 (M) x 4 (N) with four 64x32 quadrants per wave, the
// swapped-operand accumulator layout and epilogue of gemm256_kernel (g8_epilogue). LDS: one
// 8-KB slot per (half-tile, plane) of a K-step — layout 0 (K-contiguous) as [128 rows][64 B],
// 16-B chunk c of row r at c ^ ((r >> 2) & 2) (conflict-free for the A and the interleaved B
// fragment reads, tools/lds_banks.py model), layout 1 (MN-contiguous) as [32 K rows][128 elements]
// (the gemm256 bf16 layout-1 image). Slots: A-h0, B-h1, A-h1 single-buffered, B-h0 double-buffered
// (15 slots, 120 KB). One step = four phases, each reading one half-tile's three planes:
//   phase 0: quadrant (0,0) reads A-h0 + B-h0(t)    refills B-h0(t+1) (other buffer)
//   phase 1: quadrant (0,1) reads B-h1 (A-h0 kept)  refills A-h0(t+1)
//   phase 2: quadrant (1,1) reads A-h1 (B-h1 kept)  refills B-h1(t+1)
//   phase 3: quadrant (1,0) reads B-h0(t) (A-h1 kept) refills A-h1(t+1)
// Every refill writes a slot whose last reader (both wave rows) finished before the phase, one
// LDS-DMA piece per wave per plane (3 per phase), and lands 2 phases before it is read (counted
// vmcnt(6) at the end of each read phase). The two wave rows run one barrier apart (ping-pong) as
// in gemm256_kernel: per phase one row issues its reads / DMA while the other runs 48 MFMAs.
// =================================================================================================
// Diagnostic build only (-DMMFD_XF_STAMPS, tools/xf_stamps.py): s_memtime at the phase boundaries of
// one mid-loop K-step, per wave, into a buffer no computation reads.
#ifdef MMFD_XF_STAMPS
__device__ uint64_t xf_stamps[4096 * 8 * 20];
#define XF_TSTAMP(k)                                                                                  \
  do {                                                                                                \
    const uint64_t t__ = __builtin_amdgcn_s_memtime();                                               \
    const int64_t b__ = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;                                \
    if (lane == 0 && b__ < 4096) xf_stamps[(b__ * 8 + wave) * 20 + (k)] = t__;                       \
  } while (0)
#define XF_STAMP(k)                                                                                   \
  do {                                                                                                \
    if (t == xf_t) {                                                                                  \
      const uint64_t t__ = __builtin_amdgcn_s_memtime();                                             \
      const int64_t b__ = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;                              \
      if (lane == 0 && b__ < 4096) xf_stamps[(b__ * 8 + wave) * 20 + (k)] = t__;                     \
    }                                                                                                 \
  } while (0)
#else
#define XF_STAMP(k) do { } while (0)
#define XF_TSTAMP(k) do { } while (0)
#endif

// the six plane products of one K-step for one quadrant: per (i, j) a chain from zero, then one
// fp32 add into the accumulator (a[i][p] / b[j][p]: plane p = hi, mid, lo). The two chains of an A
// subtile run interleaved, and their adds are placed after the next subtile's first products (the
// chains' last MFMAs have retired by then: no wait states); scalar v_add_f32 (packed adds beside
// MFMAs cost more issue cycles), pinned in place by an empty asm so the compiler does not defer
// them past the phase's barrier
// XF_DIAG (tools/xf_stamps.py variants only, results wrong by design): 1 = no accumulator adds,
// 2 = no LDS-DMA refills in the loop, 3 = no fragment reads in the loop
#ifndef XF_DIAG
#define XF_DIAG 0
#endif
__device__ __forceinline__ void xf_add(f32x4& acc, const f32x4& t) {
  if (XF_DIAG == 1) {
    asm volatile("" ::"v"(t));
    return;
  }
  acc[0] += t[0]; acc[1] += t[1]; acc[2] += t[2]; acc[3] += t[3];
}
#ifndef XF_PRIO_STATIC
#define XF_PRIO_STATIC 1
#endif
#ifndef XF_CHAINS
#define XF_CHAINS 0
#endif
// one (i, j) chain of the six products from zero: mid*mid, hi*lo, lo*hi, hi*mid, mid*hi, hi*hi
#define XF_P(t, j, i, pb, pa) Mma<bf16>::run(t, b[j][pb], a[i][pa])
__device__ __forceinline__ void xf_mma(f32x4 (&acc)[4][2], const uint4 (&a)[4][3], const uint4 (&b)[2][3]) {
  if (!XF_PRIO_STATIC) __builtin_amdgcn_s_setprio(1);
#if XF_CHAINS == 0
  // the six products straight into the fp32 accumulators, small first per K-step, the two B
  // subtiles' chains interleaved. tools/mb/mfma_rate.hip (one wave per SIMD, this phase's 48
  // MFMAs): 16.4 cycles per MFMA, against 19.6 for the partial-sum chains from zero plus one
  // accumulator add each (the adds wait on their chain's last MFMA). Rounding: six adds at the
  // accumulator's scale per 32-deep K-step, where the fp32 MFMA takes eight (16x16x4 steps)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    XF_P(acc[i][0], 0, i, 1, 1); XF_P(acc[i][1], 1, i, 1, 1);  // mid * mid
    XF_P(acc[i][0], 0, i, 2, 0); XF_P(acc[i][1], 1, i, 2, 0);  // A hi * B lo
    XF_P(acc[i][0], 0, i, 0, 2); XF_P(acc[i][1], 1, i, 0, 2);  // A lo * B hi
    XF_P(acc[i][0], 0, i, 1, 0); XF_P(acc[i][1], 1, i, 1, 0);  // A hi * B mid
    XF_P(acc[i][0], 0, i, 0, 1); XF_P(acc[i][1], 1, i, 0, 1);  // A mid * B hi
    XF_P(acc[i][0], 0, i, 0, 0); XF_P(acc[i][1], 1, i, 0, 0);  // hi * hi
  }
#elif XF_CHAINS == 4
  // two A subtiles per group: four independent chains interleaved (an MFMA depends on the one
  // four slots earlier)
  f32x4 p[4];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    f32x4 t[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) t[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) XF_P(t[c], c & 1, 2 * g + (c >> 1), 1, 1);
#pragma unroll
    for (int c = 0; c < 4; ++c) XF_P(t[c], c & 1, 2 * g + (c >> 1), 2, 0);
    if (g > 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) xf_add(acc[c >> 1][c & 1], p[c]);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) XF_P(t[c], c & 1, 2 * g + (c >> 1), 0, 2);
#pragma unroll
    for (int c = 0; c < 4; ++c) XF_P(t[c], c & 1, 2 * g + (c >> 1), 1, 0);
#pragma unroll
    for (int c = 0; c < 4; ++c) XF_P(t[c], c & 1, 2 * g + (c >> 1), 0, 1);
#pragma unroll
    for (int c = 0; c < 4; ++c) XF_P(t[c], c & 1, 2 * g + (c >> 1), 0, 0);
#pragma unroll
    for (int c = 0; c < 4; ++c) p[c] = t[c];
    if (g > 0) {
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) xf_add(acc[2 + (c >> 1)][c & 1], p[c]);
#else
  f32x4 p0, p1;  // the previous subtile's sums
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 t0 = f32x4{0.f, 0.f, 0.f, 0.f}, t1 = f32x4{0.f, 0.f, 0.f, 0.f};
#if XF_CHAINS == 1
    // one chain after the other: each MFMA depends on the one just before it
    XF_P(t0, 0, i, 1, 1); XF_P(t0, 0, i, 2, 0);
    if (i > 0) xf_add(acc[i - 1][0], p0);
    XF_P(t0, 0, i, 0, 2); XF_P(t0, 0, i, 1, 0); XF_P(t0, 0, i, 0, 1); XF_P(t0, 0, i, 0, 0);
    XF_P(t1, 1, i, 1, 1); XF_P(t1, 1, i, 2, 0);
    if (i > 0) xf_add(acc[i - 1][1], p1);
    XF_P(t1, 1, i, 0, 2); XF_P(t1, 1, i, 1, 0); XF_P(t1, 1, i, 0, 1); XF_P(t1, 1, i, 0, 0);
    p0 = t0;
    p1 = t1;
    if (i > 0) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    }
#else
    Mma<bf16>::run(t0, b[0][1], a[i][1]);  // mid * mid
    Mma<bf16>::run(t1, b[1][1], a[i][1]);
    Mma<bf16>::run(t0, b[0][2], a[i][0]);  // A hi * B lo
    Mma<bf16>::run(t1, b[1][2], a[i][0]);
    if (i > 0) {
      xf_add(acc[i - 1][0], p0);
      xf_add(acc[i - 1][1], p1);
    }
    Mma<bf16>::run(t0, b[0][0], a[i][2]);  // A lo * B hi
    Mma<bf16>::run(t1, b[1][0], a[i][2]);
    Mma<bf16>::run(t0, b[0][1], a[i][0]);  // A hi * B mid
    Mma<bf16>::run(t1, b[1][1], a[i][0]);
    Mma<bf16>::run(t0, b[0][0], a[i][1]);  // A mid * B hi
    Mma<bf16>::run(t1, b[1][0], a[i][1]);
    Mma<bf16>::run(t0, b[0][0], a[i][0]);  // hi * hi
    Mma<bf16>::run(t1, b[1][0], a[i][0]);
    p0 = t0;
    p1 = t1;
    if (i > 0) {
      // the previous subtile's 8 adds one per MFMA gap after this subtile's first four products
      // (by then the chains they read have retired: no wait states; at most one 4-cycle VALU op
      // beside each 16-cycle MFMA)
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    }
#endif
    __builtin_amdgcn_sched_barrier(0);
  }
  xf_add(acc[3][0], p0);
  xf_add(acc[3][1], p1);
#endif
  // keep every add inside the phase (an input-only use: the compiler may not sink them past the
  // barrier into the next iteration, where the sums would stay live and spill fragments)
  asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][1]), "v"(acc[1][0]), "v"(acc[1][1]), "v"(acc[2][0]), "v"(acc[2][1]),
               "v"(acc[3][0]), "v"(acc[3][1]));
  if (!XF_PRIO_STATIC) __builtin_amdgcn_s_setprio(0);
}
#undef XF_P

// sum of the 3 x 8 bf16 values of one A fragment's planes (hi + mid + lo = the fp32 elements)
__device__ __forceinline__ float xf_sum3(uint4 h, uint4 m, uint4 l) {
  return (g8_sum16b<bf16>(h) + g8_sum16b<bf16>(m)) + g8_sum16b<bf16>(l);
}

// CONV: implicit-GEMM convolution (ConvGeom): A is the planes [3][N*H*W][C] of the NHWC activation,
// its fill gathers the im2col rows per K-step (XfConvFill); TA = 0 only. The body is shared by
// gemm256_x6f_kernel and conv_x6f_kernel (the plain GEMM keeps its kernel name in traces)
template <int TA, int TB, bool CONV, bool LEAN = false, bool EXT = false>
__device__ __forceinline__ void
x6f_body(const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb,
         float* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K,
         float alpha, int steps_per_split, const EpiArgs& e, float* __restrict__ rs_out, float rs_beta,
         int rs_mode, const X6Args& x6, const ConvGeom& cg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  XF_TSTAMP(16);
  const int gx = gridDim.x, gy = gridDim.y;
  // XCD-aware order over the whole grid, split-K index included (see gemm256_kernel)
  const int lt = xcd_remap((blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x, gx * gy * gridDim.z);
  const int split = lt / (gx * gy);
  const int tile = lt - split * (gx * gy);
  const int trow = tile / gx, tcol = tile - trow * gx;
  const int64_t m0 = (int64_t)trow * G8_BM, n0 = (int64_t)tcol * G8_BN;
  const int nst = x6.nkt;  // K-steps in all (host: ceil(K / 32))
  const int st0 = split * steps_per_split;
  const int nk = min(nst, st0 + steps_per_split) - st0;
#ifdef MMFD_XF_STAMPS
  const int xf_t = min(4, nk - 1);
#endif

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A, 3 * (int64_t)x6.pa);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(B, 3 * (int64_t)x6.pb);
  std::conditional_t<CONV, XfConvFill, XfFill<TA>> fa0, fa1;
  XfFill<TB> fb0, fb1;
  if constexpr (CONV) {
    fa0.init(cg, m0, M, wave, lane);
    fa1.init(cg, m0 + 128, M, wave, lane);
  } else {
    fa0.init(lda, m0, M, wave, lane);
    fa1.init(lda, m0 + 128, M, wave, lane);
  }
  fb0.init(ldb, n0, N, wave, lane);
  fb1.init(ldb, n0 + 128, N, wave, lane);

  // slot bases: A-h0 0, B-h1 24 KB, A-h1 48 KB, B-h0 72 KB + (t & 1) * 24 KB; plane p at + p * 8 KB
  auto slot = [&](int h, int t) -> char* {
    const int base = h == 0 ? 0 : h == 3 ? 3 : h == 1 ? 6 : 9 + 3 * (t & 1);  // h: 0 A-h0, 1 A-h1, 2 B-h0, 3 B-h1
    return smem + base * XF_SLOT;
  };
  // half-tile h of K-step t (local step index): three planes, one DMA piece per wave each
  auto issue = [&](int h, int t) {
    const int64_t k0 = (int64_t)(st0 + t) * XF_BK;
    char* s = slot(h, t);
    if (h < 2 && CONV) {
      if constexpr (CONV) {  // the window gather: one offset per lane for the three planes
        const uint32_t o = (h == 0 ? fa0 : fa1).off(cg, k0, K);
#pragma unroll
        for (int p = 0; p < 3; ++p) dma16(rsa, s + p * XF_SLOT + wave * 1024, o, (uint32_t)p * x6.pa);
      }
    } else if (h < 2) {
      if constexpr (!CONV) {
        const uint32_t so = (uint32_t)(k0 * (TA == 0 ? 1 : lda) * 2);
        const XfFill<TA>& f = h == 0 ? fa0 : fa1;
#pragma unroll
        for (int p = 0; p < 3; ++p) f.issue(rsa, s + p * XF_SLOT, so + (uint32_t)p * x6.pa, k0, K, wave);
      }
    } else {
      const uint32_t so = (uint32_t)(k0 * (TB == 0 ? 1 : ldb) * 2);
      const XfFill<TB>& f = h == 2 ? fb0 : fb1;
#pragma unroll
      for (int p = 0; p < 3; ++p) f.issue(rsb, s + p * XF_SLOT, so + (uint32_t)p * x6.pb, k0, K, wave);
    }
  };

  if (nk > 0) {
    issue(2, 0); issue(0, 0); issue(3, 0); issue(1, 0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // A-h0, B-h0 of step 0 landed
  }
  g8_barrier();
  if (wr == 1) g8_barrier();  // stagger the second wave row by one barrier
  // static priority for the second-dispatched half (waves 4-7), set once: without it that half
  // loses every issue arbitration to its SIMD partner (MI355X_MICROARCH.md, two waves per SIMD, 4)
  if (XF_PRIO_STATIC && wr == 1) __builtin_amdgcn_s_setprio(1);

  // fused row sums of op(A) (bias gradient): as gemm256_kernel, per K-step; wave wc sums A
  // subtile wc of each A half-tile (all three planes: hi + mid + lo = the fp32 value)
  const int rs_cols = rs_mode == 3 ? gx : 1;
  const bool do_rs = rs_mode != 0 && tcol < rs_cols;
  float rs0 = 0.f, rs1 = 0.f;
  int rs_ph = (st0 % rs_cols);
  // (from the A fragments in registers: subtile i == wc, a wave-uniform branch per compile-time
  // index; a lambda over the fragment array or a runtime index would put the array in scratch)
#define XF_ROWSUM(dst)                                                   \
  do {                                                                   \
    if (wc == 0) dst += xf_sum3(fa[0][0], fa[0][1], fa[0][2]);           \
    else if (wc == 1) dst += xf_sum3(fa[1][0], fa[1][1], fa[1][2]);      \
    else if (wc == 2) dst += xf_sum3(fa[2][0], fa[2][1], fa[2][2]);      \
    else dst += xf_sum3(fa[3][0], fa[3][1], fa[3][2]);                   \
  } while (0)
  auto wait_next = [&](int t, bool deep) {  // the next phase's half-tile landed (own pieces)
    if (t + 1 < nk) {
      if (deep) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  uint4 fa[4][3], fb[2][3];
  for (int t = 0; t < nk; ++t) {
    bool rs_t = false;
    if (do_rs) {
      rs_t = rs_ph == tcol;
      rs_ph = rs_ph + 1 == rs_cols ? 0 : rs_ph + 1;
    }
    // phase 0: quadrant (0,0) from A-h0, B-h0(t)
    {
      int ln = lane;
      asm volatile("" : "+v"(ln));  // recompute the fragment addresses here (no hoisted copies)
      XF_STAMP(0);
      const char* ia = slot(0, t);
      const char* ib = slot(2, t);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int i = 0; i < 4; ++i) if (XF_DIAG != 3 || t == 0) fa[i][p] = xf_frag_a<TA>(ia + p * XF_SLOT, wr * 4 + i, ln);
#pragma unroll
        for (int j = 0; j < 2; ++j) if (XF_DIAG != 3 || t == 0) fb[j][p] = xf_frag_b<TB>(ib + p * XF_SLOT, wc, j, ln);
      }
      if (rs_t) XF_ROWSUM(rs0);
      if (XF_DIAG != 2 && t + 1 < nk) issue(2, t + 1);
      wait_next(t, false);
      XF_STAMP(1);
      g8_pre_barrier();
      XF_STAMP(2);
      xf_mma(acc[0][0], fa, fb);
      XF_STAMP(3);
      g8_barrier();
    }
    // phase 1: quadrant (0,1) from B-h1 (A-h0 kept)
    {
      int ln = lane;
      asm volatile("" : "+v"(ln));  // recompute the fragment addresses here (no hoisted copies)
      XF_STAMP(4);
      const char* ib = slot(3, t);
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j) if (XF_DIAG != 3 || t == 0) fb[j][p] = xf_frag_b<TB>(ib + p * XF_SLOT, wc, j, ln);
      if (XF_DIAG != 2 && t + 1 < nk) issue(0, t + 1);
      wait_next(t, false);
      XF_STAMP(5);
      g8_pre_barrier();
      XF_STAMP(6);
      xf_mma(acc[0][1], fa, fb);
      XF_STAMP(7);
      g8_barrier();
    }
    // phase 2: quadrant (1,1) from A-h1 (B-h1 kept)
    {
      int ln = lane;
      asm volatile("" : "+v"(ln));  // recompute the fragment addresses here (no hoisted copies)
      XF_STAMP(8);
      const char* ia = slot(1, t);
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i) if (XF_DIAG != 3 || t == 0) fa[i][p] = xf_frag_a<TA>(ia + p * XF_SLOT, wr * 4 + i, ln);
      if (rs_t) XF_ROWSUM(rs1);
      if (XF_DIAG != 2 && t + 1 < nk) issue(3, t + 1);
      wait_next(t, true);
      XF_STAMP(9);
      g8_pre_barrier();
      XF_STAMP(10);
      xf_mma(acc[1][1], fa, fb);
      XF_STAMP(11);
      g8_barrier();
    }
    // phase 3: quadrant (1,0) from B-h0(t) (A-h1 kept)
    {
      int ln = lane;
      asm volatile("" : "+v"(ln));  // recompute the fragment addresses here (no hoisted copies)
      XF_STAMP(12);
      const char* ib = slot(2, t);
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j) if (XF_DIAG != 3 || t == 0) fb[j][p] = xf_frag_b<TB>(ib + p * XF_SLOT, wc, j, ln);
      if (XF_DIAG != 2 && t + 1 < nk) issue(1, t + 1);
      wait_next(t, false);
      XF_STAMP(13);
      g8_pre_barrier();
      XF_STAMP(14);
      xf_mma(acc[1][0], fa, fb);
      XF_STAMP(15);
      g8_barrier();
    }
  }

  if (XF_PRIO_STATIC && wr == 1) __builtin_amdgcn_s_setprio(0);
  if (wr == 0) g8_barrier();  // re-align the wave rows
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  XF_TSTAMP(17);
  if (do_rs) {
    rs0 += __shfl_xor(rs0, 16, 64);
    rs0 += __shfl_xor(rs0, 32, 64);
    rs1 += __shfl_xor(rs1, 16, 64);
    rs1 += __shfl_xor(rs1, 32, 64);
    if (lane < 16) {
      float* dst = rs_mode == 1 ? rs_out : rs_out + (int64_t)(split * rs_cols + tcol) * M;
      const float bt = rs_mode == 1 ? rs_beta : 0.f;
      const int64_t r0 = m0 + wr * 64 + wc * 16 + lane, r1 = r0 + 128;
      if (r0 < M) dst[r0] = (bt != 0.f ? bt * dst[r0] : 0.f) + rs0;
      if (r1 < M) dst[r1] = (bt != 0.f ? bt * dst[r1] : 0.f) + rs1;
    }
  }
  g8_epilogue<float, false, LEAN, EXT>(acc, smem, e, C, ldc, ws, split, M, N, alpha, m0, n0, tid, lane, wave, wr, wc);
#ifdef MMFD_XF_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  XF_TSTAMP(18);
#endif
#undef XF_ROWSUM
}

// two instantiations per layout: gemm256_x6f_kernel for the products without an activation or
// dropout (weight and most data gradients, QKV: their epilogue compiles without that code, 1-2 %
// faster per launch, profiles/r06y_x6f_lean_epilogue.log), gemm256_x6f_act_kernel for the rest
template <int TA, int TB>
__global__ void __launch_bounds__(NT, 1)
gemm256_x6f_kernel(const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb,
                   float* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K,
                   float alpha, int steps_per_split, EpiArgs e, float* __restrict__ rs_out, float rs_beta,
                   int rs_mode, X6Args x6) {
  x6f_body<TA, TB, false, true>(A, lda, B, ldb, C, ldc, ws, M, N, K, alpha, steps_per_split, e, rs_out, rs_beta,
                                rs_mode, x6, ConvGeom{});
}
template <int TA, int TB>
__global__ void __launch_bounds__(NT, 1)
gemm256_x6f_act_kernel(const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb,
                       float* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K,
                       float alpha, int steps_per_split, EpiArgs e, float* __restrict__ rs_out, float rs_beta,
                       int rs_mode, X6Args x6) {
  x6f_body<TA, TB, false, false>(A, lda, B, ldb, C, ldc, ws, M, N, K, alpha, steps_per_split, e, rs_out, rs_beta,
                                 rs_mode, x6, ConvGeom{});
}
// MMFD_ACT_GELU_D / MMFD_ACT_MUL_AUX without dropout (the fp32 training FFN's GELU with its derivative
// saved, and the data gradient through it)
template <int TA, int TB>
__global__ void __launch_bounds__(NT, 1)
gemm256_x6f_ext_kernel(const bf16* __restrict__ A, int64_t lda, const bf16* __restrict__ B, int64_t ldb,
                       float* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K,
                       float alpha, int steps_per_split, EpiArgs e, float* __restrict__ rs_out, float rs_beta,
                       int rs_mode, X6Args x6) {
  x6f_body<TA, TB, false, false, true>(A, lda, B, ldb, C, ldc, ws, M, N, K, alpha, steps_per_split, e, rs_out, rs_beta,
                                       rs_mode, x6, ConvGeom{});
}
// implicit-GEMM convolution on split operands (mmfd_gemm_args.conv): X = the activation's planes
__global__ void __launch_bounds__(NT, 1)
conv_x6f_kernel(const bf16* __restrict__ X, const bf16* __restrict__ B, int64_t ldb, float* __restrict__ C,
                int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K, float alpha, int steps_per_split,
                EpiArgs e, X6Args x6, ConvGeom cg) {
  x6f_body<0, 0, true>(X, cg.C, B, ldb, C, ldc, ws, M, N, K, alpha, steps_per_split, e, nullptr, 0.f, 0, x6, cg);
}



}  // namespace

#ifdef MMFD_XF_STAMPS
extern "C" int mmfd_debug_xf_stamps(void* host_dst, int64_t bytes) {
  return (int)hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(xf_stamps), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
#endif

namespace mmfd_gemmx {
template <int TA, int TB>
void launch_x6f(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int sps, float* rs_out,
                int rs_mode, hipStream_t s, const void* pa, const void* pb, X6Args x6) {
  dim3 grid((unsigned)((a.N + G8_BN - 1) / G8_BN), (unsigned)((a.M + G8_BM - 1) / G8_BM), (unsigned)splits);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_x6f_kernel<TA, TB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, G8_LDS) == hipSuccess &&
           hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_x6f_act_kernel<TA, TB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, G8_LDS) == hipSuccess &&
           hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_x6f_ext_kernel<TA, TB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, G8_LDS) == hipSuccess;
  }();
  (void)attr;
  // the planes' leading dim = the stored column count
  const int64_t lda = TA == 0 ? a.K : a.M, ldb = TB == 0 ? a.K : a.N;
  // (with split-K slabs the tile kernel runs no epilogue at all: the reduce does)
  const bool lean = ws != nullptr || (e.act == MMFD_ACT_NONE && e.p <= 0.f);
  const bool ext = !lean && (e.act == MMFD_ACT_GELU_D || e.act == MMFD_ACT_MUL_AUX);  // (no dropout: gemm.hip ext_slab)
  if (ext)
    hipLaunchKernelGGL((gemm256_x6f_ext_kernel<TA, TB>), grid, dim3(NT), G8_LDS, s, (const bf16*)pa, lda,
                       (const bf16*)pb, ldb, (float*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, sps, e, rs_out,
                       a.a_rowsum_beta, rs_mode, x6);
  else if (lean)
    hipLaunchKernelGGL((gemm256_x6f_kernel<TA, TB>), grid, dim3(NT), G8_LDS, s, (const bf16*)pa, lda, (const bf16*)pb,
                       ldb, (float*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, sps, e, rs_out, a.a_rowsum_beta, rs_mode, x6);
  else
    hipLaunchKernelGGL((gemm256_x6f_act_kernel<TA, TB>), grid, dim3(NT), G8_LDS, s, (const bf16*)pa, lda,
                       (const bf16*)pb, ldb, (float*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, sps, e, rs_out,
                       a.a_rowsum_beta, rs_mode, x6);
}
void launch_conv_x6f(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int sps, hipStream_t s,
                     const void* pa, const void* pb, X6Args x6, const ConvGeom& cg) {
  dim3 grid((unsigned)((a.N + G8_BN - 1) / G8_BN), (unsigned)((a.M + G8_BM - 1) / G8_BM), (unsigned)splits);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_x6f_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, G8_LDS) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(conv_x6f_kernel, grid, dim3(NT), G8_LDS, s, (const bf16*)pa, (const bf16*)pb, a.K, (float*)a.C,
                     a.ldc, ws, a.M, a.N, a.K, a.alpha, sps, e, x6, cg);
}
void dispatch_x6f(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int sps, float* rs_out,
                  int rs_mode, hipStream_t s, const void* pa, const void* pb, X6Args x6, const ConvGeom& cg) {
  if (cg.on) launch_conv_x6f(a, e, ws, splits, sps, s, pa, pb, x6, cg);
  else if (!a.trans_a && !a.trans_b) launch_x6f<0, 0>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
  else if (!a.trans_a && a.trans_b) launch_x6f<0, 1>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
  else if (a.trans_a && !a.trans_b) launch_x6f<1, 0>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
  else launch_x6f<1, 1>(a, e, ws, splits, sps, rs_out, rs_mode, s, pa, pb, x6);
}

}  // namespace mmfd_gemmx
