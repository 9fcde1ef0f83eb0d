"""Generates multimodal-misinformation-detection_amd/csrc/gemm_g4.hip: the four-wave bf16 forward GEMM
(C[M][N] = A[M][K] . B[N][K]^T + bias, bf16 out) whose main loop is one inline-assembly block — the
instruction schedule measured in tools/mb/gen_g4loop.py (V2 / V4: 2,476-3,436 cycles per 64-deep
K-tile against the compiler-scheduled G8's ~3,600, profiles/r05_g4loop_mb_*.log) with the operand
rows of a real tile behind the LDS-DMA pieces:

  * 4 waves (one per SIMD) as 2 (M) x 2 (N), 128 x 128 each, the 256 fp32 accumulators in AGPRs;
  * per 64-deep K-tile two parts of 64 MFMAs (K halves kc0 / kc1); each part reads the other
    half's 16 fragments (ds_read_b128, one per 4 MFMAs) and issues 8 LDS-DMA pieces (one per 8
    MFMAs) refilling the half it no longer needs, two tiles ahead, in two 64-KB LDS stages;
  * LDS region of one K half = 16 fragments of 1 KB; fragment f of A = rows 16 f + r (r < 16),
    four 16-B K chunks per row, stored row-major with the chunk slot XOR (r / 2) % 4, so the DMA
    fetches each row's 64 contiguous bytes with four consecutive lanes and the MFMA-order reads
    (lane l: row l % 16, chunk l / 16) are conflict-free; fragment j of the wave's B = columns
    wn*128 + 8 r + j, so a lane's 8 accumulators of an output row are 8 CONSECUTIVE columns;
  * register epilogue: v_accvgpr_read, + bias, v_cvt_pk_bf16_f32 (round to nearest even, as the
    G8 epilogue's conversion), one nontemporal 16-B store per (row group, register): 16 lanes write
    256 contiguous bytes of a row — no LDS staging, no barrier.

Full tiles only (M, N multiples of 256, K of 64), alpha 1, no other epilogue: gemm.hip routes the
rest to gemm256_kernel. Run: python3 tools/gen_gemm_g4.py (the Makefile compiles the output).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "mb"))
import gen_g4loop as G  # noqa: E402  (mfma / reads / part: the measured schedule)

OUT = os.environ.get("G4_OUT") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "multimodal-misinformation-detection_amd", "csrc", "gemm_g4.hip")


def dmas(part):
    """8 pieces of K half `part`: 4 A fragments (rows 16 f + lane%16, f = 4 wave + p: source step
    %[psa] = 16 rows) and 4 B fragments (f = 4 wave + p -> wn = wave / 2, j = 4 (wave % 2) + p:
    rows 8 c + j, source step %[psb] = 1 row); s40 = 128 B x the K-tile being fetched"""
    out = []
    for p in range(8):
        if p < 4:
            reg, vo, rs, stp = "s42", "%[voffa]", "%[srda]", "%[psa]"
        else:
            reg, vo, rs, stp = "s43", "%[voffb]", "%[srdb]", "%[psb]"
        step = [f"s_add_u32 s41, s40, {part * 64}"] if p % 4 == 0 else [f"s_add_u32 s41, s41, {stp}"]
        out.append([f"s_mov_b32 m0, {reg}"] + step +
                   [f"buffer_load_dwordx4 {vo}, {rs}, s41 offen lds", f"s_add_u32 {reg}, {reg}, 1024"])
    return out


def prologue():
    """DMA of a tile's K-tiles 0 and 1 into stages 0 and 1, after a barrier (every wave is done
    reading the previous tile's stages: the main loop drained its own reads and DMA)"""
    # m0 is reserved to the compiler: saved here and restored at the end (the DMA pieces walk it)
    L = ["s_barrier", "s_mov_b32 s47, m0", "s_mov_b32 s40, 0"]
    for st in (0, 1):
        for half in (0, 1):
            L += [f"s_add_u32 s42, %[mA], {st * 65536 + half * 16384}", f"s_add_u32 s43, %[mB], {st * 65536 + half * 16384}"]
            for d in dmas(half):
                L += d
        L += ["s_add_u32 s40, s40, 128"]
    L += ["s_mov_b32 m0, s47"]
    return L


def body():
    """the main loop of a tile whose prologue was issued: accumulators zeroed, wait for K-tile 0's
    first half (vmcnt(24) right after the prologue; %[vw] when the previous tile's epilogue issued
    its loads / stores after it: they are younger, and each counts), K-tiles 2.. fetched two ahead"""
    L = ["s_mov_b32 s47, m0"] + [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    L += ["s_mov_b32 s44, %[nit]", "s_mov_b32 s40, 256", "s_mov_b32 s45, 0"]
    L += ["s_cmp_eq_u32 %[first], 0", "s_cbranch_scc0 L_w24_%=", "s_waitcnt vmcnt(%[vw])", "s_branch L_wd_%=",
          "L_w24_%=:", "s_waitcnt vmcnt(24)", "L_wd_%=:", "s_barrier"]
    L += G.reads(0, "%[rA0]", "%[rB0]", 0)
    L += ["L_top_%=:", "s_waitcnt vmcnt(16) lgkmcnt(0)", "s_barrier", "s_cmp_eq_u32 s45, 0",
          "s_cselect_b32 s42, %[mA], %[mA1]", "s_cselect_b32 s43, %[mB], %[mB1]"]
    parts = {}
    for st in (0, 1):
        rA, rB = ("%[rA0]", "%[rB0]") if st == 0 else ("%[rA1]", "%[rB1]")
        nA, nB = ("%[rA1]", "%[rB1]") if st == 0 else ("%[rA0]", "%[rB0]")
        pa = G.part(0, 2, G.reads(1, rA, rB, 1), dmas(0))
        mid = ["s_waitcnt vmcnt(16) lgkmcnt(0)", "s_barrier",
               f"s_add_u32 s42, %[mA{'' if st == 0 else '1'}], 16384", f"s_add_u32 s43, %[mB{'' if st == 0 else '1'}], 16384"]
        pb = G.part(1, 2, G.reads(0, nA, nB, 0), dmas(1))
        parts[st] = pa + mid + pb
    L += ["s_cbranch_scc0 L_odd_%="] + parts[0] + ["s_branch L_next_%=", "L_odd_%=:"] + parts[1] + ["L_next_%=:"]
    L += ["s_xor_b32 s45, s45, 1", "s_add_u32 s40, s40, 128", "s_sub_u32 s44, s44, 1", "s_cmp_eq_u32 s44, 0",
          "s_cbranch_scc0 L_top_%="]
    # the pieces fetched past the last K-tile land in stages nobody reads; drain them before the
    # workgroup's LDS is refilled (the next tile's prologue) or released
    L += ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_mov_b32 m0, s47"]
    return L


def acc_reads():
    """one asm statement per A fragment i: its 32 accumulators (8 B fragments x 4 registers) into
    VGPRs, z[e][j] = a[4 (8 i + j) + e] (rows 16 i + 4 (lane / 16) + e, columns 8 (lane % 16) + j)"""
    out = []
    for i in range(8):
        outs = ", ".join(f'"=v"(z[{e}][{j}])' for e in range(4) for j in range(8))
        ins = "\\n\\t".join(f"v_accvgpr_read_b32 %{8 * e + j}, a{4 * (8 * i + j) + e}"
                             for e in range(4) for j in range(8))
        out.append(f"""  if (i == {i}) asm volatile("{ins}" : {outs});""")
    return "\n".join(out)


SRC = r'''// GENERATED by tools/gen_gemm_g4.py — do not edit; see the generator's docstring.
// Four-wave bf16 forward GEMM (gfx950): C = A . B^T + bias, full 256x256 tiles, main loop and
// register epilogue as one inline-assembly block (hand-placed fragment reads / LDS-DMA between the
// MFMAs; AGPR accumulators). Routed from gemm.hip (mmfd_gemmx::launch_g4) for eligible products.
#include "gemm_tiles.h"

namespace {

struct G4Args {
  uint32_t voffa, voffb;
  __amdgpu_buffer_rsrc_t srda, srdb;
  uint32_t nit, psa, psb;
  uint32_t mA, mB, mA1, mB1, rA0, rB0, rA1, rB1;
};

__device__ __forceinline__ void g4_prologue(const G4Args& x) {
  asm volatile("@PRO@"
      :
      : [voffa] "v"(x.voffa), [voffb] "v"(x.voffb), [srda] "s"(x.srda), [srdb] "s"(x.srdb),
        [psa] "s"(x.psa), [psb] "s"(x.psb), [mA] "s"(x.mA), [mB] "s"(x.mB)
      : "s40", "s41", "s42", "s43", "s47", "scc", "memory");
}

// VW: the vmcnt that leaves K-tile 0's first 8 pieces landed when the previous tile's epilogue
// (at least VW - 24 vector-memory operations per wave) was issued after this tile's prologue
template <int VW>
__device__ __forceinline__ void g4_body(const G4Args& x, int first) {
  asm volatile("@ASM@"
      :
      : [voffa] "v"(x.voffa), [voffb] "v"(x.voffb), [srda] "s"(x.srda), [srdb] "s"(x.srdb), [nit] "s"(x.nit),
        [psa] "s"(x.psa), [psb] "s"(x.psb), [mA] "s"(x.mA), [mB] "s"(x.mB), [mA1] "s"(x.mA1), [mB1] "s"(x.mB1),
        [rA0] "v"(x.rA0), [rB0] "v"(x.rB0), [rA1] "v"(x.rA1), [rB1] "v"(x.rB1), [first] "s"(first), [vw] "i"(VW)
      : @CLOB@);
}

// the 32 accumulators of A fragment i (the main loop's asm left them in a[0:255]; nothing between
// that asm and these reads allocates AGPRs: the kernel's own code stays far below 256 VGPRs)
template <int i>
__device__ __forceinline__ void g4_acc(float (&z)[4][8]) {
@ACCREADS@
}

// Persistent: workgroup b walks tiles b, b + G, b + 2G ... (G = gridDim.x: one per CU, or one per
// tile — MMFD_G4_PERSIST=0 — which is the one-tile-per-workgroup form). The next tile's prologue
// (its K-tiles 0 and 1) is issued right after this tile's main loop, so its DMA latency hides under
// this tile's register epilogue (both LDS stages are free then). Tiles in XCD-contiguous runs
// (workgroup b runs on XCD b % 8; with G and the tile count multiples of 8 each XCD walks
// consecutive row-major tiles, which share A panels).
template <int EPI>
__global__ void __launch_bounds__(256) gemm_g4_kernel(const bf16* __restrict__ A, int64_t lda,
                                                      const bf16* __restrict__ B, int64_t ldb, bf16* __restrict__ C,
                                                      int64_t ldc, EpiArgs ep, int M, int N, int K) {
  const int ntn = N / 256;
  __shared__ __attribute__((aligned(1024))) char smem[131072];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const uint32_t base = (uint32_t)(size_t)smem;
  const uint32_t nb = gridDim.x, b0 = blockIdx.x;
  const uint32_t tiles = (uint32_t)(M / 256) * (uint32_t)ntn;
  const bool xcd = (nb % 8u) == 0 && (tiles % 8u) == 0;
  auto tile_of = [&](uint32_t tt) { return xcd ? (tt % 8u) * (tiles / 8u) + tt / 8u : tt; };
  const uint32_t rowa = (uint32_t)lda * 2u, rowb = (uint32_t)ldb * 2u;
  G4Args x;
  // LDS-DMA: lane q of a piece lands at 16 q = fragment row q / 4, chunk slot q % 4, and fetches
  // that row's 16-B K chunk (q % 4) ^ sw(row): four consecutive lanes read one row's 64 contiguous
  // bytes (coalesced), and the XOR sw(r) = (r / 2) % 4 makes the MFMA-order reads below conflict-free
  const int qr = lane >> 2, qc = (lane & 3) ^ ((qr >> 1) & 3);
  x.voffa = (uint32_t)(wave * 64 + qr) * rowa + (uint32_t)qc * 16u;
  x.voffb = (uint32_t)((wave >> 1) * 128 + 8 * qr + 4 * (wave & 1)) * rowb + (uint32_t)qc * 16u;
  x.psa = 16u * rowa;
  x.psb = rowb;
  auto set_tile = [&](uint32_t bid) {
    const uint32_t tm = bid / (uint32_t)ntn, tn = bid % (uint32_t)ntn;
    x.srda = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(A) + (int64_t)tm * 256 * lda, 0, (int)(256u * rowa), 0x00020000);
    x.srdb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(B) + (int64_t)tn * 256 * ldb, 0, (int)(256u * rowb), 0x00020000);
  };
  x.nit = (uint32_t)(K / 64);
  // stage s (64 KB at s * 64 KB): A-kc0 +0, A-kc1 +16K, B-kc0 +32K, B-kc1 +48K; wave w fills
  // fragments 4w .. 4w+3 of each region; wave (wm, wn) reads A fragments 8 wm + i, B 8 wn + j
  x.mA = base + wave * 4096; x.mB = base + 32768 + wave * 4096;
  x.mA1 = x.mA + 65536; x.mB1 = x.mB + 65536;
  // fragment read, MFMA operand order: lane l takes row l % 16, K chunk l / 16 -> slot 4 r + (c ^ sw(r))
  const int fr = lane & 15, fc = lane >> 4;
  const uint32_t slot = (uint32_t)(4 * fr + (fc ^ ((fr >> 1) & 3))) * 16u;
  x.rA0 = base + wm * 8192 + slot;
  x.rB0 = base + 32768 + wn * 8192 + slot;
  x.rA1 = x.rA0 + 65536; x.rB1 = x.rB0 + 65536;
  constexpr bool RES = EPI == 1 || EPI == 2, DROP = EPI == 2, GELU = EPI == 3 || EPI == 5, BWD = EPI == 4 || EPI == 6;
  constexpr bool GD = EPI == 5, MUL = EPI == 6;  // GELU_D: aux <- GELU'(z); MUL_AUX: x aux
  constexpr bool STREAM = RES || BWD;  // one bf16 operand stream read per output: residual or aux
  // vector-memory operations per wave issued after the next tile's prologue: at least the 32
  // output stores (+ 32 aux stores when a GELU mode keeps aux, + 28 + 4 residual / aux loads in
  // the STREAM modes); waiting for vmcnt(24 + 32) leaves K-tile 0's first 8 pieces landed in every
  // mode (the extra operations are older than nothing the loop needs: it only waits longer)
  constexpr int VW = 24 + 32;
  const uint32_t seed = DROP ? mmfd_hash_key(*ep.seed, ep.salt) : 0u;
  const int64_t ls = RES ? ep.ldr : ep.ldaux;
  uint32_t tt = b0;
  set_tile(tile_of(tt));
  g4_prologue(x);
  for (int first = 1;; first = 0) {
    const uint32_t bid = tile_of(tt);
    const uint32_t tm = bid / (uint32_t)ntn, tn = bid % (uint32_t)ntn;
    // epilogue operands before the main loop, so their latency hides under it: the bias of the
    // lane's 8 columns, the first row group's residual
    const int64_t row0 = (int64_t)tm * 256 + wm * 128 + 4 * (lane >> 4);
    const int64_t col = (int64_t)tn * 256 + wn * 128 + 8 * (lane & 15);
    float bia[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) bia[u] = 0.f;
    if (ep.bias) {
      const float4 b0v = *reinterpret_cast<const float4*>(ep.bias + col), b1v = *reinterpret_cast<const float4*>(ep.bias + col + 4);
      bia[0] = b0v.x; bia[1] = b0v.y; bia[2] = b0v.z; bia[3] = b0v.w; bia[4] = b1v.x; bia[5] = b1v.y; bia[6] = b1v.z; bia[7] = b1v.w;
    }
    const bf16* rp = RES ? reinterpret_cast<const bf16*>(ep.residual) + row0 * ep.ldr + col
                   : BWD ? reinterpret_cast<const bf16*>(ep.aux) + row0 * ep.ldaux + col : nullptr;
    bf16* ap = GELU && ep.aux ? reinterpret_cast<bf16*>(ep.aux) + row0 * ep.ldaux + col : nullptr;
    bf16* cp = C + row0 * ldc + col;
    Raw8<bf16> cur[4], nxt[4];
    if constexpr (STREAM) {
#pragma unroll
      for (int e = 0; e < 4; ++e) cur[e].load(rp + e * ls);
    }
    g4_body<VW>(x, first);
    const uint32_t tn2 = tt + nb;
    if (tn2 < tiles) {  // the next tile's K-tiles 0 and 1, in flight during this epilogue
      set_tile(tile_of(tn2));
      g4_prologue(x);
    }
    // the G8 fast path's operation order (gemm_tiles.h g8_epilogue) for the modes EPI: 0 = + bias,
    // 1 = + bias + residual, 2 = + bias, dropout, + residual, 3 = + bias, GELU (pre-activation to
    // aux), 4 = (+ bias) x GELU'(aux) (the data gradient through the FFN's GELU, read from the saved
    // pre-activation), 5 = + bias, GELU (its derivative to aux), 6 = (+ bias) x aux (the saved
    // derivative); rounded to bf16 once. Lane (r4 = lane / 16, c = lane % 16) owns rows wm*128 + 16 i +
    // 4 r4 + e and the 8 consecutive columns wn*128 + 8 c ..: 16 lanes load / store 256 contiguous
    // bytes of a row. A loop over the 8 row groups (the accumulator reads are per-group code, the
    // math one body: the unrolled form did not fit the instruction cache), the next group's
    // residual loaded before this group's stores.
    float z[4][8];
    for (int I = 0; I < 8; ++I) {
      if constexpr (STREAM) {
        if (I < 7) {
#pragma unroll
          for (int e = 0; e < 4; ++e) nxt[e].load(rp + (int64_t)(16 * (I + 1) + e) * ls);
        }
      }
      switch (I) {
        case 0: g4_acc<0>(z); break;
        case 1: g4_acc<1>(z); break;
        case 2: g4_acc<2>(z); break;
        case 3: g4_acc<3>(z); break;
        case 4: g4_acc<4>(z); break;
        case 5: g4_acc<5>(z); break;
        case 6: g4_acc<6>(z); break;
        default: g4_acc<7>(z); break;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t ro = 16 * I + e;
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = z[e][u] + bia[u];
        if constexpr (GD) {
          float d[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = gelu_and_grad_f(v[u], d[u]);
          if (ap) V8<bf16>::store(ap + ro * ep.ldaux, d);
        } else if constexpr (GELU) {
          if (ap) V8<bf16>::store(ap + ro * ep.ldaux, v);
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = gelu_f(v[u]);
        }
        if constexpr (BWD) {
          float t[8];
          cur[e].get(t);
          if constexpr (MUL) {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] *= t[u];
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] *= gelu_grad_f(t[u]);
          }
        }
        if constexpr (DROP) {
          const uint64_t hb = (uint64_t)(row0 + ro) * (uint64_t)N + (uint64_t)col;
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = (mmfd_hash_k(seed, hb + u) < ep.thr) ? 0.f : v[u] * ep.keep_scale;
        }
        if constexpr (RES) {
          float t[8];
          cur[e].get(t);
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] += t[u];
        }
        V8<bf16>::store(cp + ro * ldc, v);
      }
      if constexpr (STREAM) {
#pragma unroll
        for (int e = 0; e < 4; ++e) cur[e] = nxt[e];
      }
    }
  if (tn2 >= tiles) break;
    tt = tn2;
  }
}

}  // namespace

namespace mmfd_gemmx {
// the products the four-wave kernel takes: bf16 x bf16 -> bf16, both operands K-contiguous (the
// nn.Linear forward), full tiles, alpha 1 and at most a bias in the epilogue; env MMFD_G4=0 sends
// them to gemm256_kernel (A/B measurements, tests). The switches are read from the environment once,
// when the library loads (MMFD_G4=0: off; MMFD_G4_GELU=0: not the FFN1 GELU modes; MMFD_G4_KMAX), and
// changed at run time only through mmfd_set_g4_mode / mmfd_set_g4_kmax — never a getenv per launch
int g_g4_mode = [] {
  const char* v = getenv("MMFD_G4");
  const char* g = getenv("MMFD_G4_GELU");
  return (v && v[0] == '0') ? 0 : (g && g[0] == '0') ? 1 : 2;
}();
int g_g4_persist = [] {  // MMFD_G4_PERSIST=0: one workgroup per tile (A/B)
  const char* v = getenv("MMFD_G4_PERSIST");
  return (v && v[0] == '0') ? 0 : 1;
}();
// compute units of the current device (the persistent grid), cached per device
int64_t g4_cus() {
  static int64_t cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}
int64_t g_g4_kmax = [] {
  const char* k = getenv("MMFD_G4_KMAX");
  return k ? (int64_t)atoll(k) : (int64_t)1024;
}();
int g4_epi(const mmfd_gemm_args& a, const EpiArgs& e, int splits) {
  const int mode = g_g4_mode;
  if (mode == 0) return -1;
  if (a.dtype != MMFD_BF16 || a.c_dtype != MMFD_BF16 || a.trans_a || a.trans_b || splits > 1) return -1;
  if (a.M % 256 || a.N % 256 || a.K % 64 || a.K < 64 || a.alpha != 1.0f || a.beta != 0.0f || a.a_rowsum) return -1;
  // K <= 1024: the short-K products (QKV, attention output, FFN1 at K = 768) gain from the register
  // epilogue; at K = 3072 (FFN2) the power-limited main loop is no faster than gemm256_kernel's and
  // ViT's FFN2 measured 10 % slower (profiles/r05_g4_vs_g8_vs_hipblaslt.log)
  if (a.K > g_g4_kmax) return -1;
  if (!e.vec || e.pl || e.beta != 0.0f) return -1;
  // the epilogue modes of the encoder forward Linears (anything else runs on gemm256_kernel)
  int epi = -1;
  if (e.act == MMFD_ACT_NONE && !e.residual && e.p <= 0.0f) epi = 0;                    // QKV
  else if (e.act == MMFD_ACT_NONE && e.residual && !e.res_first) epi = e.p > 0.0f ? 2 : 1;  // out / FFN2
  // FFN1 (bias + GELU [+ its derivative or the pre-activation to aux]): mode 2, the default since
  // the derivative-saving form (EPI 5, the training FFN1): bf16 step +0.8 % on two boxes
  // (profiles/r06n_g4_gelu_ab.log; the pre-activation form measured 0.89-1.03x of gemm256_kernel per
  // GEMM across boxes in round 5, profiles/r05_g4_schedule_ab.log)
  else if (e.act == MMFD_ACT_GELU && !e.residual && e.p <= 0.0f && mode == 2) epi = 3;
  else if (e.act == MMFD_ACT_GELU_D && !e.residual && e.p <= 0.0f && mode == 2) epi = 5;
  // the FFN's data gradient through GELU (x GELU'(pre-activation)): the product of dY with the
  // K-contiguous (transposed) weight copy, blocks.linear_dx
  else if (e.act == MMFD_ACT_GELU_BWD && e.aux && !e.residual && e.p <= 0.0f) epi = 4;
  else if (e.act == MMFD_ACT_MUL_AUX && e.aux && !e.residual && e.p <= 0.0f) epi = 6;  // (its GELU_D form)
  if (epi < 0) return -1;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al16(a.A) || !al16(a.B) || !al16(a.C)) return -1;
  if (a.lda % 8 || a.ldb % 8 || a.ldc % 8 || a.lda < a.K || a.ldb < a.K || a.ldc < a.N) return -1;
  if (256 * a.lda * 2 >= (int64_t)1 << 31 || 256 * a.ldb * 2 >= (int64_t)1 << 31 || 256 * a.ldc * 2 >= (int64_t)1 << 31)
    return -1;
  const int64_t tiles = (a.M / 256) * (a.N / 256);
  if (tiles >= ((int64_t)1 << 31)) return -1;
  return epi;
}

bool launch_g4(const mmfd_gemm_args& a, const EpiArgs& e, int splits, hipStream_t s) {
  const int epi = g4_epi(a, e, splits);
  if (epi < 0) return false;
  const int64_t tiles = (a.M / 256) * (a.N / 256);
  // persistent grid: one workgroup per CU (128 KB of LDS: one fits), each walking its tiles
  const int64_t grid = g_g4_persist ? std::min<int64_t>(tiles, g4_cus()) : tiles;
#define G4_LAUNCH(E)                                                                                 \
  hipLaunchKernelGGL(gemm_g4_kernel<E>, dim3((unsigned)grid), dim3(256), 0, s, (const bf16*)a.A, a.lda, \
                     (const bf16*)a.B, a.ldb, (bf16*)a.C, a.ldc, e, (int)a.M, (int)a.N, (int)a.K)
  if (epi == 0) G4_LAUNCH(0);
  else if (epi == 1) G4_LAUNCH(1);
  else if (epi == 2) G4_LAUNCH(2);
  else if (epi == 3) G4_LAUNCH(3);
  else if (epi == 4) G4_LAUNCH(4);
  else if (epi == 5) G4_LAUNCH(5);
  else G4_LAUNCH(6);
#undef G4_LAUNCH
  return true;
}
}  // namespace mmfd_gemmx

extern "C" int mmfd_set_g4_mode(int mode) {
  MMFD_CHECK_ARG(mode >= -1 && mode <= 2, "mmfd_set_g4_mode: mode %d (-1 query, 0 off, 1 on, 2 on + GELU)", mode);
  const int old = mmfd_gemmx::g_g4_mode;
  if (mode >= 0) mmfd_gemmx::g_g4_mode = mode;
  return old;
}

extern "C" int mmfd_set_g4_persist(int on) {
  MMFD_CHECK_ARG(on >= -1 && on <= 1, "mmfd_set_g4_persist: %d (-1 query, 0 one tile per workgroup, 1 persistent)", on);
  const int old = mmfd_gemmx::g_g4_persist;
  if (on >= 0) mmfd_gemmx::g_g4_persist = on;
  return old;
}

extern "C" int64_t mmfd_set_g4_kmax(int64_t kmax) {
  const int64_t old = mmfd_gemmx::g_g4_kmax;
  if (kmax > 0) mmfd_gemmx::g_g4_kmax = kmax;
  return old;
}
'''


def main():
    clob = [f'"v{r}"' for r in range(4, 132)] + [f'"a{r}"' for r in range(256)] + \
           [f'"s{r}"' for r in range(40, 48)] + ['"scc"', '"memory"']
    src = SRC.replace("@ASM@", "\\n\\t".join(body())).replace("@PRO@", "\\n\\t".join(prologue()))
    src = src.replace("@CLOB@", ", ".join(clob)).replace("@ACCREADS@", acc_reads())
    with open(OUT, "w") as f:
        f.write(src)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
