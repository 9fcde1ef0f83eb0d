// The 256x256 G8 GEMM kernel (gemm256_kernel) and its launcher, shared by gemm.hip (bf16-output
// instantiations) and gemm_f32out.hip (fp32-output ones). Two translation units so that each
// instantiation family gets the compiler flags under which it is spill-free (Makefile: the
// fp32-output ones without SLP vectorisation; the SLP-packed code spilled 8-40 dwords there).
#pragma once
#include "gemm_tiles.h"

namespace {

// G8_PF: the bf16 loop's kc = 0 fragment reads one phase ahead, interleaved into the previous
// phase's MFMA block (see the main loop; +3.9 % over the encoder GEMM shapes, same-box A/B;
// profiles/r05_g8_*_ab.txt for the variants measured); 0 = the round-4 schedule
#ifndef G8_PF
#define G8_PF 1
#endif

// PRE: the epilogue has exactly one bf16 operand stream (residual, saved pre-activation or C),
// prefetched for all of a thread's rows before the accumulators are staged (see the epilogue)

// LEAN: no activation and no dropout in the epilogue (or split-K slabs): the epilogue's fast path
// compiles without that code (g8_epilogue); gemm256_kernel is the lean instantiation, gemm256_act_kernel
// the full one (as gemm256_x6f_kernel / gemm256_x6f_act_kernel)
template <typename T, int TA, int TB, typename TC, bool PRE, bool X6, bool LEAN>
__device__ __forceinline__ void
gemm256_body(const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
             TC* __restrict__ C, int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K,
             float alpha, int tiles_per_split, const EpiArgs& e, float* __restrict__ rs_out, float rs_beta,
             int rs_mode, int group_m, const X6Args& x6) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  G8_STAMP(0);
  const int gx = gridDim.x, gy = gridDim.y;
  // XCD-aware order over the whole grid, split-K index included: the hardware deals workgroups
  // round-robin over the 8 XCDs in linear (x, y, z) order, and each XCD gets a contiguous run of
  // (split, row, column) tiles — the blocks of one K range sharing A / B panels sit in one L2
  // (remapping (x, y) alone put split z's tiles on XCD (id + 36 z) mod 8: the split-K weight-
  // gradient GEMMs re-fetched their operands 4-5x)
  const int lt = xcd_remap((blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x, gx * gy * gridDim.z);
  const int split = lt / (gx * gy);
  const int tile = lt - split * (gx * gy);
  // grouped raster: an XCD's consecutive tiles sweep group_m row panels x the column tiles, so the
  // ~32 tiles it runs at once share group_m A panels and 32/group_m B panels in its L2
  int trow, tcol;
  {
    const int gsz = group_m * gx, g = tile / gsz, first = g * group_m, gm = min(gy - first, group_m);
    const int r = tile - g * gsz;
    trow = first + r % gm;
    tcol = r / gm;
  }
  const int64_t m0 = (int64_t)trow * G8_BM, n0 = (int64_t)tcol * G8_BN;
  constexpr int G8_BK = G8T<T>::BK;
  constexpr int64_t ESZ = sizeof(T);
  const int nkt_total = X6 ? 6 * x6.nkt : (int)((K + G8_BK - 1) / G8_BK);
  const int kt0 = split * tiles_per_split;
  const int nk = min(nkt_total, kt0 + tiles_per_split) - kt0;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A, X6 ? 3 * (int64_t)x6.pa : (TA == 0 ? M : K) * lda * ESZ);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(B, X6 ? 3 * (int64_t)x6.pb : (TB == 0 ? N : K) * ldb * ESZ);
  Fill<T, TA, 128, 2> fa0, fa1;
  Fill<T, TB, 128, 2, 1> fb0, fb1;
  fa0.init(lda, m0, M, wave, lane);
  fa1.init(lda, m0 + 128, M, wave, lane);
  fb0.init(ldb, n0, N, wave, lane);
  fb1.init(ldb, n0 + 128, N, wave, lane);

  // half-tile h of K-tile t: 0 = A-h0, 1 = A-h1, 2 = B-h0, 3 = B-h1; buffer t & 1
  auto img = [&](int t, int h) -> char* { return smem + ((t & 1) * 4 + h) * G8_HALF; };
  auto issue = [&](int h, int t) {
    int64_t k0 = (int64_t)(kt0 + t) * G8_BK;
    uint32_t pofs = 0;  // X6: byte offset of the segment's plane
    if constexpr (X6) {
      const int v = kt0 + t, sg = v / x6.nkt;
      k0 = (int64_t)(v - sg * x6.nkt) * G8_BK;
      pofs = h < 2 ? ((X6_CA >> (2 * sg)) & 3u) * x6.pa : ((X6_CB >> (2 * sg)) & 3u) * x6.pb;
    }
    const bool tail = k0 + G8_BK > K;
    if (h < 2) {
      const uint32_t so = (uint32_t)(k0 * (TA == 0 ? 1 : lda) * ESZ) + pofs;
      if (h == 0) fa0.issue(rsa, img(t, 0), so, tail, k0, K, wave, lane);
      else fa1.issue(rsa, img(t, 1), so, tail, k0, K, wave, lane);
    } else {
      const uint32_t so = (uint32_t)(k0 * (TB == 0 ? 1 : ldb) * ESZ) + pofs;
      if (h == 2) fb0.issue(rsb, img(t, 2), so, tail, k0, K, wave, lane);
      else fb1.issue(rsb, img(t, 3), so, tail, k0, K, wave, lane);
    }
  };

  constexpr bool PH2 = sizeof(T) == 2;  // bf16: two-phase schedule (see the main loop)
  if (PH2 && nk > 0) {
    // two-phase schedule: A-h0, B-h0, B-h1 of K-tile t are read in phase X(t), A-h1 in phase Y(t)
    issue(0, 0); issue(2, 0); issue(3, 0); issue(1, 0);
    if (nk > 1) {
      issue(0, 1); issue(2, 1); issue(3, 1);
      // (G8_PF: all of K-tile 0, A-h1 included — the leading row reads it in X(0)'s MFMA block)
      if (G8_PF) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else if (nk > 0) {
    issue(0, 0); issue(3, 0); issue(1, 0); issue(2, 0);
    if (nk > 1) {
      issue(0, 1); issue(3, 1); issue(1, 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  g8_barrier();
  if (wr == 1) g8_barrier();  // stagger the second wave row by one barrier

  // fused row sums of op(A) (bias gradient); wave wc sums A subtile i == wc of each A fragment set
  // it loads, lane (g, i) covering k-chunk g of row i. rs_mode 1 / 2: the first column tile sums
  // every K-tile (direct / per-split partials); rs_mode 3: the gx column tiles share the K-tiles
  // round robin (K-tile v goes to column tile v mod gx) into per-(split, column tile) partials —
  // one column of blocks doing all of it made the whole launch wait on them (+25 % on the
  // weight-gradient GEMMs)
  const int rs_cols = rs_mode == 3 ? gx : 1;
  const bool do_rs = rs_mode != 0 && tcol < rs_cols;
  float rs0 = 0.f, rs1 = 0.f;
  int rs_ph = (kt0 % rs_cols);  // column tile owning the current K-tile's row sums
  // X6: only the segments that carry each A plane once contribute to the row sums
  auto rs_on = [&](int t) { return !X6 || ((X6_RS >> ((kt0 + t) / x6.nkt)) & 1u); };

  uint4 fa[4][2], fb[2][2];
  if constexpr (PH2 && G8_PF) {
    // The two-phase schedule below with each phase's kc = 0 fragments read one phase AHEAD, inside
    // the previous phase's MFMA block right after the kc = 0 products that free their registers:
    // X(t)'s MFMAs read A-h1(t) kc 0, Y(t)'s read A-h0 / B-h0 / B-h1 of t+1 kc 0, so each read section
    // keeps only the kc = 1 half (X 8 reads instead of 16, Y 4 instead of 8). Landing: the lagging
    // wave row must have landed the next phase's pieces before the barrier that opens the leading
    // row's MFMA block, hence one counted wait before each closing barrier — vmcnt(2) after X (only
    // X's own A-h1 refill may fly), vmcnt(6) after Y — on pieces issued a whole phase earlier.
    uint4 fbh[2][2];
    if (nk > 0) {
      g8_frag_a_kc<T, TA>(fa, img(0, 0), wr, lane, 0);
      g8_frag_b_kc<T, TB>(fb, img(0, 2), wc, lane, 0);
      g8_frag_b_kc<T, TB>(fbh, img(0, 3), wc, lane, 0);
    }
    for (int t = 0; t < nk; ++t) {
      bool rs_t = false;
      if (do_rs) {
        rs_t = rs_ph == tcol && rs_on(t);
        rs_ph = rs_ph + 1 == rs_cols ? 0 : rs_ph + 1;
      }
      // phase X(t)
      g8_frag_a_kc<T, TA>(fa, img(t, 0), wr, lane, 1);
      g8_frag_b_kc<T, TB>(fb, img(t, 2), wc, lane, 1);
      g8_frag_b_kc<T, TB>(fbh, img(t, 3), wc, lane, 1);
      if (rs_t) rs0 += g8_rowsum<T, TA>(img(t, 0), wr, wc, lane);
      if (t + 1 < nk) {
        issue(1, t + 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      g8_pre_barrier();
      __builtin_amdgcn_s_setprio(1);
      g8_mma2_kc<T>(acc[0][0], acc[0][1], fa, fb, fbh, 0);
      g8_frag_a_kc<T, TA>(fa, img(t, 1), wr, lane, 0);  // Y(t)'s A-h1, kc 0
      g8_mma2_kc<T>(acc[0][0], acc[0][1], fa, fb, fbh, 1);
      // the 4 reads one per 4 of the kc = 1 products (as one burst after the kc = 0 products: -2.7 %)
      __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      g8_barrier();
      // phase Y(t)
      g8_frag_a_kc<T, TA>(fa, img(t, 1), wr, lane, 1);
      if (rs_t) rs1 += g8_rowsum<T, TA>(img(t, 1), wr, wc, lane);
      if (t + 2 < nk) {
        issue(0, t + 2); issue(2, t + 2); issue(3, t + 2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      g8_pre_barrier();
      __builtin_amdgcn_s_setprio(1);
      g8_mma2_kc<T>(acc[1][0], acc[1][1], fa, fb, fbh, 0);
      {  // X(t+1)'s kc 0, straight-line: past the last K-tile the reads fetch an unused image (in bounds)
        const int tn = t + 1 < nk ? t + 1 : t;
        g8_frag_a_kc<T, TA>(fa, img(tn, 0), wr, lane, 0);
        g8_frag_b_kc<T, TB>(fb, img(tn, 2), wc, lane, 0);
        g8_frag_b_kc<T, TB>(fbh, img(tn, 3), wc, lane, 0);
      }
      g8_mma2_kc<T>(acc[1][0], acc[1][1], fa, fb, fbh, 1);
      // the 8 reads one per 2 of the kc = 1 products
      __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      g8_barrier();
    }
  } else if constexpr (PH2) {
    // Two phases per K-tile, 32 MFMAs each (one quadrant per phase, as fp32 below, measured 3.5 %
    // slower over the encoder shapes: twice the barrier hand-offs): X(t) = quadrants (0,0), (0,1)
    // from A-h0 and both B halves; Y(t) = quadrants (1,0), (1,1) from A-h1 with the B fragments
    // kept in registers. Refills: X(t) issues A-h1 of
    // t+1 (last read in Y(t-1)), Y(t) issues A-h0 / B-h0 / B-h1 of t+2 (last read in X(t)); each
    // phase then waits until at most the 8 pieces issued after the next phase's operands remain.
    // Segment stamps of one mid-loop K-tile (G8_PSTAMP, tools/g8_stamps.py): each phase's read
    // side (fragment reads ~30 cycles per ds_read_b128 issue, LDS-DMA pieces ~130 cycles each,
    // the vmcnt wait < 100) outlasts the partner row's 32 MFMAs, so a K-tile takes ~3,600 cycles
    // against 2,048 of MFMA. Moving two of Y's six pieces into X (four per phase) measured
    // neutral (+0.5 % over the encoder shapes, profiles/r04_bf16_g8_stamps.log): a piece costs
    // more beside X's 16 reads than beside Y's 8.
    uint4 fbh[2][2];
    for (int t = 0; t < nk; ++t) {
      bool rs_t = false;
      if (do_rs) {  // (uniform; kept off the path of GEMMs without row sums)
        rs_t = rs_ph == tcol && rs_on(t);
        rs_ph = rs_ph + 1 == rs_cols ? 0 : rs_ph + 1;
      }
      // phase X(t)
      G8_PSTAMP(8);
      g8_frag_a<T, TA>(fa, img(t, 0), wr, lane);
      g8_frag_b<T, TB>(fb, img(t, 2), wc, lane);
      g8_frag_b<T, TB>(fbh, img(t, 3), wc, lane);
      if (rs_t) rs0 += g8_rowsum<T, TA>(img(t, 0), wr, wc, lane);
      G8_PSTAMP(17);
      if (t + 1 < nk) {
        issue(1, t + 1);
        G8_PSTAMP(18);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      G8_PSTAMP(9);
      g8_pre_barrier();
      G8_PSTAMP(10);
      g8_mma2<T>(acc[0][0], acc[0][1], fa, fb, fbh);
      G8_PSTAMP(11);
      g8_barrier();
      // phase Y(t)
      G8_PSTAMP(12);
      g8_frag_a<T, TA>(fa, img(t, 1), wr, lane);
      if (rs_t) rs1 += g8_rowsum<T, TA>(img(t, 1), wr, wc, lane);
      G8_PSTAMP(19);
      if (t + 2 < nk) {
        issue(0, t + 2); issue(2, t + 2); issue(3, t + 2);
        G8_PSTAMP(20);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      G8_PSTAMP(13);
      g8_pre_barrier();
      G8_PSTAMP(14);
      g8_mma2<T>(acc[1][0], acc[1][1], fa, fb, fbh);
      G8_PSTAMP(15);
      g8_barrier();
      G8_PSTAMP(16);
    }
  } else {
    // fp32: four phases of one quadrant each (the two-phase schedule pushes the fp32 layout-1
    // fragment addressing past 256 VGPRs into scratch and measured no faster)
    for (int t = 0; t < nk; ++t) {
      bool rs_t = false;
      if (do_rs) {
        rs_t = rs_ph == tcol;
        rs_ph = rs_ph + 1 == rs_cols ? 0 : rs_ph + 1;
      }
      // phase 0: quadrant (0,0)
      g8_frag_a<T, TA>(fa, img(t, 0), wr, lane);
      g8_frag_b<T, TB>(fb, img(t, 2), wc, lane);
      if (rs_t) rs0 += g8_rowsum<T, TA>(img(t, 0), wr, wc, lane);
      if (t + 1 < nk) issue(2, t + 1);
      g8_pre_barrier();
      g8_mma<T>(acc[0][0], fa, fb);
      g8_barrier();
      // phase 1: quadrant (0,1)
      g8_frag_b<T, TB>(fb, img(t, 3), wc, lane);
      if (t + 2 < nk) issue(0, t + 2);
      g8_pre_barrier();
      g8_mma<T>(acc[0][1], fa, fb);
      g8_barrier();
      // phase 2: quadrant (1,1)
      g8_frag_a<T, TA>(fa, img(t, 1), wr, lane);
      if (rs_t) rs1 += g8_rowsum<T, TA>(img(t, 1), wr, wc, lane);
      if (t + 2 < nk) issue(3, t + 2);
      g8_pre_barrier();
      g8_mma<T>(acc[1][1], fa, fb);
      g8_barrier();
      // phase 3: quadrant (1,0); K-tile t+1 must have landed before the next phase reads it
      g8_frag_b<T, TB>(fb, img(t, 2), wc, lane);
      if (t + 2 < nk) {
        issue(1, t + 2);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      g8_pre_barrier();
      g8_mma<T>(acc[1][0], fa, fb);
      g8_barrier();
    }
  }

  G8_STAMP(1);
  if (wr == 0) g8_barrier();  // re-align the wave rows
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  G8_STAMP(2);
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

  g8_epilogue<TC, PRE, LEAN>(acc, smem, e, C, ldc, ws, split, M, N, alpha, m0, n0, tid, lane, wave, wr, wc);
}

#define G8_KERNEL(NAME, LEAN)                                                                           \
  template <typename T, int TA, int TB, typename TC, bool PRE, bool X6>                               \
  __global__ void __launch_bounds__(NT, 1)                                                            \
  NAME(const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb, TC* __restrict__ C, \
       int64_t ldc, float* __restrict__ ws, int64_t M, int64_t N, int64_t K, float alpha, int tiles_per_split, \
       EpiArgs e, float* __restrict__ rs_out, float rs_beta, int rs_mode, int group_m, X6Args x6) {      \
    gemm256_body<T, TA, TB, TC, PRE, X6, LEAN>(A, lda, B, ldb, C, ldc, ws, M, N, K, alpha, tiles_per_split, e, \
                                              rs_out, rs_beta, rs_mode, group_m, x6);                  \
  }
G8_KERNEL(gemm256_kernel, true)
G8_KERNEL(gemm256_act_kernel, false)
#undef G8_KERNEL

int g8_group_m() {
  static const int gm = getenv("MMFD_G8_GROUP_M") ? std::max(1, atoi(getenv("MMFD_G8_GROUP_M"))) : 1;
  return gm;
}

template <typename T, int TA, int TB, typename TC, bool PRE, bool X6>
void launch_g8_v(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps, float* rs_out,
                 int rs_mode, hipStream_t s, const void* A, int64_t lda, const void* B, int64_t ldb, X6Args x6) {
  dim3 grid((unsigned)((a.N + G8_BN - 1) / G8_BN), (unsigned)((a.M + G8_BM - 1) / G8_BM), (unsigned)splits);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_kernel<T, TA, TB, TC, PRE, X6>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, G8_LDS) == hipSuccess &&
           hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_act_kernel<T, TA, TB, TC, PRE, X6>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, G8_LDS) == hipSuccess;
  }();
  (void)attr;
  if (ws != nullptr || (e.act == MMFD_ACT_NONE && e.p <= 0.f))
    hipLaunchKernelGGL((gemm256_kernel<T, TA, TB, TC, PRE, X6>), grid, dim3(NT), G8_LDS, s, (const T*)A, lda,
                       (const T*)B, ldb, (TC*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, tps, e, rs_out,
                       a.a_rowsum_beta, rs_mode, g8_group_m(), x6);
  else
    hipLaunchKernelGGL((gemm256_act_kernel<T, TA, TB, TC, PRE, X6>), grid, dim3(NT), G8_LDS, s, (const T*)A, lda,
                       (const T*)B, ldb, (TC*)a.C, a.ldc, ws, a.M, a.N, a.K, a.alpha, tps, e, rs_out,
                       a.a_rowsum_beta, rs_mode, g8_group_m(), x6);
}

}  // namespace
