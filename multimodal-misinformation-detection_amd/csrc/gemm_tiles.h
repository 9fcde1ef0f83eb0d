// Shared pieces of the MFMA GEMM kernels (gemm.hip): epilogue arguments and stores,
// LDS operand images and their swizzles, LDS-DMA stage fills, MFMA fragment loads.
#pragma once
#include "common.h"
#include <type_traits>

// types shared by the GEMM translation units (gemm.hip)
namespace mmfd_gemmx {
struct EpiArgs {
  const float* bias;
  const void* residual; int64_t ldr;
  void* aux; int64_t ldaux;
  int act;
  float p; uint32_t thr; float keep_scale;
  const uint64_t* seed; uint64_t salt;
  float beta;
  int vec;  // host-checked: C / residual / aux 16-B aligned with leading dims multiple of 8
  int res_first;  // residual added before the forward activation
  // fp32 C only: the output's bf16 split planes [3][M][N] (hi, mid, lo; see split3_kernel) written
  // beside C or instead of it (c_out = 0) — the operand form of the next split-operand GEMM
  bf16* pl; int64_t pl_stride; int c_out;
};

// X6 (fp32 GEMMs from bf16 split operands, see mmfd_gemm): A and B are three bf16 planes each
// (x = hi + mid + lo), x6.pa / x6.pb bytes apart; the K loop runs over six segments of x6.nkt
// K-tiles, segment s multiplying A plane X6_CA[s] with B plane X6_CB[s]. The segments go from the
// smallest products to hi*hi, so the fp32 accumulator collects the 2^-16 / 2^-8 correction terms
// first and then takes the K hi*hi products (exact in fp32) exactly as a plain fp32 sum would: the
// rounding of the result is that of the fp32 dot product.
struct X6Args { int nkt; uint32_t pa, pb; };
constexpr uint32_t X6_CA = 0x121;  // A planes per segment (2 bits each): m h l h m h
constexpr uint32_t X6_CB = 0x049;  // B planes per segment:                m l h m h h
constexpr uint32_t X6_RS = 0x25;   // segments whose A plane appears once (m, l, h): row sums of op(A)
// split-operand fp32 GEMM with fused planes (gemm_x6f.hip): launches gemm256_x6f_kernel for the
// operand layout of `a` (A / B = the bf16 planes pa / pb, x6.nkt = 32-deep K-steps in all)
void dispatch_x6f(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int sps, float* rs_out,
                  int rs_mode, hipStream_t s, const void* pa, const void* pb, X6Args x6);
// fp32-output 256x256 GEMMs (gemm_f32out.hip): gemm256_kernel<T, TA, TB, float, false, X6>
template <typename T, int TA, int TB, bool X6>
void launch_g8_f32out(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps, float* rs_out,
                      int rs_mode, hipStream_t s, const void* A, int64_t lda, const void* B, int64_t ldb, X6Args x6);
}  // namespace mmfd_gemmx

namespace {
using mmfd_gemmx::EpiArgs;
using mmfd_gemmx::X6Args;
using mmfd_gemmx::X6_CA;
using mmfd_gemmx::X6_CB;
using mmfd_gemmx::X6_RS;
using mmfd_gemmx::dispatch_x6f;


// Tile geometry: 256 (M) x 128 (N) x 128 B of K (64 bf16 / 32 fp32), 8 waves as 4 (M) x 2 (N), each
// wave a 64 x 64 block of 4 x 4 16x16 MFMA tiles. Three LDS stages of 48 KB (A 32 KB + B 16 KB).
constexpr int BM = 256, BN = 128, ROWB = 128, NT = 512, NWAVES = 8;
constexpr int A_BYTES = 32768, B_BYTES = 16384, STAGE_BYTES = A_BYTES + B_BYTES, NSTAGE = 3;
constexpr int LDS_BYTES = NSTAGE * STAGE_BYTES;  // 147456

template <typename T> struct GT {
  static constexpr int ESZ = sizeof(T);
  static constexpr int BK = ROWB / ESZ;        // K per tile
  static constexpr int EPC = 16 / ESZ;         // elements per 16-B chunk
  static constexpr int KCH = BK / Mma<T>::KC;  // MFMA chunks per tile (2)
};



typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

__device__ __forceinline__ void split1(float x, bf16& h, bf16& m, bf16& l) {
  h = (bf16)x;
  const float r = x - (float)h;
  m = (bf16)r;
  l = (bf16)(r - (float)m);
}
// 8 consecutive outputs of row `row` into the planes (16-B stores)
__device__ __forceinline__ void planes_store8(const EpiArgs& e, int64_t N, int64_t row, int64_t col, const float (&z)[8]) {
  bf16x8 h, m, l;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    bf16 a, b, c;
    split1(z[u], a, b, c);
    h[u] = a; m[u] = b; l[u] = c;
  }
  bf16* d = e.pl + row * N + col;
  *reinterpret_cast<uint4*>(d) = __builtin_bit_cast(uint4, h);
  *reinterpret_cast<uint4*>(d + e.pl_stride) = __builtin_bit_cast(uint4, m);
  *reinterpret_cast<uint4*>(d + 2 * e.pl_stride) = __builtin_bit_cast(uint4, l);
}

template <typename TC>
__device__ __forceinline__ void epilogue_store(const EpiArgs& e, TC* C, int64_t ldc, int64_t N,
                                               int64_t row, int64_t col, float z, uint32_t hkey) {
  if (e.bias) z += e.bias[col];
  if (e.res_first && e.residual) z += to_f32(reinterpret_cast<const TC*>(e.residual)[row * e.ldr + col]);
  if (e.act == MMFD_ACT_GELU || e.act == MMFD_ACT_RELU) {
    if (e.aux) reinterpret_cast<TC*>(e.aux)[row * e.ldaux + col] = from_f32<TC>(z);
    z = (e.act == MMFD_ACT_GELU) ? gelu_f(z) : fmaxf(z, 0.0f);
  } else if (e.act == MMFD_ACT_GELU_BWD) {
    z *= gelu_grad_f(to_f32(reinterpret_cast<const TC*>(e.aux)[row * e.ldaux + col]));
  } else if (e.act == MMFD_ACT_RELU_BWD) {
    z = (to_f32(reinterpret_cast<const TC*>(e.aux)[row * e.ldaux + col]) > 0.0f) ? z : 0.0f;
  } else if (e.act >= MMFD_ACT_TANH) {
    z = act_tail_f(e.act, z);
  }
  if (e.p > 0.0f) {
    const uint32_t h = mmfd_hash_k(hkey, (uint64_t)row * (uint64_t)N + (uint64_t)col);
    z = (h < e.thr) ? 0.0f : z * e.keep_scale;
  }
  if (e.residual && !e.res_first) z += to_f32(reinterpret_cast<const TC*>(e.residual)[row * e.ldr + col]);
  TC* cp = C + row * ldc + col;
  if (e.beta != 0.0f) z += e.beta * to_f32(*cp);
  if (std::is_same<TC, float>::value && e.pl) {
    bf16 h, m, l;
    split1(z, h, m, l);
    bf16* d = e.pl + row * N + col;
    d[0] = h; d[e.pl_stride] = m; d[2 * e.pl_stride] = l;
    if (!e.c_out) return;
  }
  *cp = from_f32<TC>(z);
}

template <typename TC> struct V8;
template <> struct V8<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[8]) {
    const uint4 x = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
  }
  // streaming (nontemporal) stores: the epilogue's outputs are written once and read by a later
  // launch; +1.3 % over the bf16 encoder GEMM shapes, +0.6 % on the bf16 step (same-box A/B,
  // tools/lib_ab.sh, profiles/r04_epi_nt_ab.log)
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[8]) {
    bf16x8 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4_t, o), reinterpret_cast<u32x4_t*>(p));
  }
};
template <> struct V8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
    // (nontemporal here and in planes_store8 measured neutral on the fp32 GEMMs and −0.3 % on the
    // fp32 step: profiles/r04_epi_nt_ab.log)
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// raw 16-B (bf16) / 32-B (fp32) holders for 8 consecutive elements, converted after all loads of a
// pass are in flight
template <typename TC> struct Raw8;
template <> struct Raw8<bf16> {
  uint4 v;
  __device__ __forceinline__ void load(const bf16* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void get(float (&f)[8]) const {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(w[i] << 16); f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
  }
};
template <> struct Raw8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p); b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void get(float (&f)[8]) const {
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
};

// 8 consecutive columns [col, col+8) of one row; same operation order as epilogue_store
template <typename TC>
__device__ __forceinline__ void epilogue_store8(const EpiArgs& e, TC* C, int64_t ldc, int64_t N, int64_t row,
                                                int64_t col, float (&z)[8], uint32_t hkey) {
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
  if (e.act == MMFD_ACT_GELU || e.act == MMFD_ACT_RELU) {
    if (e.aux) V8<TC>::store(reinterpret_cast<TC*>(e.aux) + row * e.ldaux + col, z);
    if (e.act == MMFD_ACT_GELU) {
#pragma unroll
      for (int q = 0; q < 8; ++q) z[q] = gelu_f(z[q]);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) z[q] = fmaxf(z[q], 0.0f);
    }
  } else if (e.act == MMFD_ACT_GELU_BWD || e.act == MMFD_ACT_RELU_BWD) {
    float a[8];
    V8<TC>::load(reinterpret_cast<const TC*>(e.aux) + row * e.ldaux + col, a);
    if (e.act == MMFD_ACT_GELU_BWD) {
#pragma unroll
      for (int q = 0; q < 8; ++q) z[q] *= gelu_grad_f(a[q]);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) z[q] = a[q] > 0.0f ? z[q] : 0.0f;
    }
  } else if (e.act >= MMFD_ACT_TANH) {
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] = act_tail_f(e.act, z[q]);
  }
  if (e.p > 0.0f) {
    const uint64_t base = (uint64_t)row * (uint64_t)N + (uint64_t)col;
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] = (mmfd_hash_k(hkey, base + q) < e.thr) ? 0.0f : z[q] * e.keep_scale;
  }
  if (e.residual && !e.res_first) {
    float r[8];
    V8<TC>::load(reinterpret_cast<const TC*>(e.residual) + row * e.ldr + col, r);
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] += r[q];
  }
  TC* cp = C + row * ldc + col;
  if (e.beta != 0.0f) {
    float c[8];
    V8<TC>::load(cp, c);
#pragma unroll
    for (int q = 0; q < 8; ++q) z[q] += e.beta * c[q];
  }
  if (std::is_same<TC, float>::value && e.pl) {
    planes_store8(e, N, row, col, z);
    if (!e.c_out) return;
  }
  V8<TC>::store(cp, z);
}

// -------------------------------------------------------------------------------------------------
// LDS images. Operand layout 0 ("K-contiguous": A[m][k] / nn.Linear W[n][k]): [rows][128 B], 16-B
// chunk c of row r at chunk c ^ (r & 7) (conflict-free ds_read_b128 fragments). Layout 1
// ("MN-contiguous": A[k][m] / B[k][n]): [BK rows][MNW elements]; bf16 fragments come from
// ds_read_b64_tr_b16 with 8-B unit u of row r at u ^ 4*((r&3) | ((r>>3)&1)<<2) (conflict-free tr
// reads), fp32 fragments from 4 ds_read_b32 with chunk c at c ^ 4*((r>>2)&3) (see swz).
// -------------------------------------------------------------------------------------------------
// SW = 1 (layout 0 only): the B image of the 256x256 kernel, whose fragments gather rows
// 8p + 4j + (0..3) (see g8_load_b); chunk c of row r at c ^ (2*((r>>1)&1) | 4*((r>>3)&1)) keeps
// those ds_read_b128 reads conflict-free.
template <typename T, int LAYOUT, int MNW, int SW = 0>
struct Img {
  static constexpr int RBY = LAYOUT == 0 ? ROWB : MNW * (int)sizeof(T);  // bytes per image row
  static constexpr int CPR = RBY / 16;                                    // 16-B chunks per row
  static constexpr int RPI = 1024 / RBY;                                  // rows per 1-KB DMA piece
  __device__ __forceinline__ static int swz(int r, int c) {  // physical chunk <-> logical chunk
    if (LAYOUT == 0 && SW == 1) return c ^ ((((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2));
    if (LAYOUT == 0) return c ^ (r & 7);
    if (sizeof(T) == 2) return c ^ (2 * ((r & 3) | (((r >> 3) & 1) << 2)));
    // fp32, MN-contiguous: a fragment is 4 ds_read_b32 whose 16-lane groups g read rows 4g + s (the
    // rows of a group are 4 * 128 or 256 dwords apart = the same banks). A-type fragments read 4
    // consecutive chunks per group: XOR by 4 * g puts the groups on disjoint banks. The G8 B image
    // (SW = 1) is read as chunks {b, b+2, b+4, b+6}: XOR by {0, 1, 8, 9} separates those.
    if (SW == 1) return c ^ (((r >> 2) & 1) | (((r >> 3) & 1) << 3));
    return c ^ (4 * ((r >> 2) & 3));
  }
};

constexpr uint32_t OOB = 0x80000000u;  // operands are < 2 GB (checked on the host)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// One 1-KB LDS-DMA piece: lane l's 16 bytes land at lds_dst + 16 l. Written as inline asm so that
// hipcc does not treat later ds_reads as dependent on it (it would drain vmcnt(0) before every
// k-step); completion is tracked by hand with counted s_waitcnt vmcnt + s_barrier.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_dst, uint32_t voff, uint32_t soff) {
  const uint32_t lds = (uint32_t)(size_t)(MMFD_LDS char*)lds_dst;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "v"(voff), "s"(rs), "s"(soff)
      : "memory");
}

// One operand's share of a stage fill: NP 1-KB LDS-DMA pieces per wave (buffer_load ... lds). The
// per-lane source offsets are loop invariant (the K tile advances through soffset) and chunks
// outside the matrix point past num_records, so the DMA writes zeros there.
template <typename T, int LAYOUT, int MNW, int NP, int SW = 0>
struct Fill {
  uint32_t off[NP];
  __device__ __forceinline__ void init(int64_t ld, int64_t mn0, int64_t mn_ext, int wave, int lane) {
    using I = Img<T, LAYOUT, MNW, SW>;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int q = wave * NP + j;                     // piece index within the image
      const int row = q * I::RPI + lane / I::CPR;      // image row this lane writes
      const int c = I::swz(row, lane % I::CPR);        // source chunk for that position
      int64_t el;
      bool ok;
      if (LAYOUT == 0) { el = (mn0 + row) * ld + (int64_t)c * GT<T>::EPC; ok = mn0 + row < mn_ext; }
      else { el = (int64_t)row * ld + mn0 + (int64_t)c * GT<T>::EPC; ok = mn0 + (int64_t)c * GT<T>::EPC < mn_ext; }
      off[j] = ok ? (uint32_t)(el * (int64_t)sizeof(T)) : OOB;
    }
  }
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* img, uint32_t soff, bool tail, int64_t k0,
                                        int64_t K, int wave, int lane) {
    using I = Img<T, LAYOUT, MNW, SW>;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      uint32_t o = off[j];
      if (LAYOUT == 0 && tail) {  // partial last K tile: zero the chunks past K
        const int row = (wave * NP + j) * I::RPI + lane / I::CPR;
        const int c = I::swz(row, lane % I::CPR);
        if (k0 + (int64_t)c * GT<T>::EPC >= K) o = OOB;
      }
      dma16(rs, img + (wave * NP + j) * 1024, o, soff);
    }
  }
};

// 16-row (layout 0) / 16-column (layout 1) MFMA fragment for K chunk kc
template <typename T, int LAYOUT, int MNW>
__device__ __forceinline__ uint4 load_frag(const char* img, int sub, int kc, int lane) {
  using I = Img<T, LAYOUT, MNW>;
  const int g = lane >> 4, i = lane & 15;
  if (LAYOUT == 0) {
    const int row = sub * 16 + i;
    return lds_read16(img, row * ROWB + (I::swz(row, kc * 4 + g) << 4));
  } else if (sizeof(T) == 2) {
    const int q = i >> 2, p = i & 3;
    const int r1 = kc * 32 + 8 * g + q, r2 = r1 + 4;
    const int u = sub * 4 + p;  // 8-B unit (4 bf16)
    const uint2 a = lds_read_tr16(img + r1 * I::RBY + (I::swz(r1, u >> 1) << 4) + ((u & 1) << 3));
    const uint2 b = lds_read_tr16(img + r2 * I::RBY + (I::swz(r2, u >> 1) << 4) + ((u & 1) << 3));
    return make_uint4(a.x, a.y, b.x, b.y);
  } else {
    const int col = sub * 16 + i;
    uint32_t v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int row = kc * 16 + 4 * g + s;
      v[s] = *reinterpret_cast<const uint32_t*>(img + row * I::RBY + (I::swz(row, col >> 2) << 4) + (col & 3) * 4);
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
}


// =================================================================================================
// 256x256 kernel ("G8", bf16 and fp32 operands): 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns four
// 64x32 quadrants (mq, nq): rows mq*128 + wr*64 + [0,64), cols nq*128 + wc*32 + [0,32). Each K-tile
// (128 B of K per row: 64 bf16 / 32 fp32) is
// staged as four 16-KB half-tiles (A rows [0,128) / [128,256), B cols [0,128) / [128,256)) into
// one of two LDS buffers by LDS-DMA, and consumed in four phases, one quadrant (16 MFMAs) each:
//   phase 0: (0,0) reads A-h0, B-h0   phase 1: (0,1) reads B-h1
//   phase 2: (1,1) reads A-h1         phase 3: (1,0) reads B-h0
// Every phase refills the half-tile whose last read was the previous phase (one half-tile = two
// DMA pieces per wave), so three half-tiles stay in flight across the barriers; the only wait is
// a counted vmcnt(6) in phase 3. The two wave rows run one barrier apart (ping-pong): while one
// row issues its LDS reads and DMA the other row's MFMAs run.
// =================================================================================================
constexpr int G8_HALF = 16384;
constexpr int G8_LDS = 128 * (256 + 4) * 4;  // >= 2 buffers x 4 half-tiles (128 KB); 128-row epilogue staging
constexpr int G8_BM = 256, G8_BN = 256;
template <typename T> struct G8T { static constexpr int BK = ROWB / (int)sizeof(T); };  // K per K-tile

__device__ __forceinline__ void g8_pre_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own LDS reads retired (WAR vs the next refill)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void g8_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename T, int LAYOUT>
__device__ __forceinline__ void g8_frag_a(uint4 (&a)[4][2], const char* img, int wr, int lane) {
#pragma unroll
  for (int kc = 0; kc < 2; ++kc)
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i][kc] = load_frag<T, LAYOUT, 128>(img, wr * 4 + i, kc, lane);
}
// B fragment j (j = 0, 1) of the wave's 32 columns gathers the 4-column units 2p + j (p = 0..3),
// and the MFMA runs with swapped operands (acc = B-fragment x A-fragment = the C^T block): lane
// (g, ci) of accumulator (i, j) then holds row i*16 + ci, columns 8g + 4j .. +3, i.e. every lane
// owns 8 CONSECUTIVE columns of a row (fragment 0 the low four) — one 16-byte bf16 chunk for the
// register epilogue. The K-contiguous B image uses the SW = 1 swizzle under which these
// ds_read_b128 are conflict-free; the MN-contiguous (transposed ds_read_b64_tr_b16) B reads are
// 2-way (each 16-B chunk is read in one half only), well inside the LDS budget of a K-tile.
// fp32 operands: the same column interleave, the 16x16x4 fragment being 4 consecutive k of the
// row (layout 0: one ds_read_b128; layout 1: 4 ds_read_b32 down the K rows of the column)
template <typename T, int LAYOUT>
__device__ __forceinline__ uint4 g8_load_b(const char* img, int wc, int j, int kc, int lane) {
  using I = Img<T, LAYOUT, 128, 1>;
  const int g = lane >> 4, i = lane & 15;
  if (LAYOUT == 0) {
    const int row = wc * 32 + 4 * (2 * (i >> 2) + j) + (i & 3);
    return lds_read16(img, row * ROWB + (I::swz(row, kc * 4 + g) << 4));
  } else if (sizeof(T) == 2) {
    const int q = i >> 2, p = i & 3;
    const int r1 = kc * 32 + 8 * g + q, r2 = r1 + 4;
    const int u = wc * 8 + 2 * p + j;  // 8-B unit (4 bf16)
    const uint2 a = lds_read_tr16(img + r1 * I::RBY + (I::swz(r1, u >> 1) << 4) + ((u & 1) << 3));
    const uint2 b = lds_read_tr16(img + r2 * I::RBY + (I::swz(r2, u >> 1) << 4) + ((u & 1) << 3));
    return make_uint4(a.x, a.y, b.x, b.y);
  } else {
    const int col = wc * 32 + 4 * (2 * (i >> 2) + j) + (i & 3);
    uint32_t v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int row = kc * 16 + 4 * g + s;
      v[s] = *reinterpret_cast<const uint32_t*>(img + row * I::RBY + (I::swz(row, col >> 2) << 4) + (col & 3) * 4);
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
}
template <typename T, int LAYOUT>
__device__ __forceinline__ void g8_frag_b(uint4 (&b)[2][2], const char* img, int wc, int lane) {
#pragma unroll
  for (int kc = 0; kc < 2; ++kc)
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j][kc] = g8_load_b<T, LAYOUT>(img, wc, j, kc, lane);
}
template <typename T>
__device__ __forceinline__ void g8_mma(f32x4 (&acc)[4][2], const uint4 (&a)[4][2], const uint4 (&b)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kc = 0; kc < 2; ++kc)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) Mma<T>::run(acc[i][j], b[j][kc], a[i][kc]);
  __builtin_amdgcn_s_setprio(0);
}

// two quadrants sharing the A fragments (one phase of the two-phase schedule)
template <typename T>
__device__ __forceinline__ void g8_mma2(f32x4 (&acc0)[4][2], f32x4 (&acc1)[4][2], const uint4 (&a)[4][2],
                                        const uint4 (&b0)[2][2], const uint4 (&b1)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kc = 0; kc < 2; ++kc)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        Mma<T>::run(acc0[i][j], b0[j][kc], a[i][kc]);
        Mma<T>::run(acc1[i][j], b1[j][kc], a[i][kc]);
      }
  __builtin_amdgcn_s_setprio(0);
}

// one k-chunk (kc) of the fragment sets / of a two-quadrant phase: the bf16 loop's kc = 0 halves are
// read one phase ahead (G8_PF, see gemm256_kernel)
template <typename T, int LAYOUT>
__device__ __forceinline__ void g8_frag_a_kc(uint4 (&a)[4][2], const char* img, int wr, int lane, int kc) {
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i][kc] = load_frag<T, LAYOUT, 128>(img, wr * 4 + i, kc, lane);
}
template <typename T, int LAYOUT>
__device__ __forceinline__ void g8_frag_b_kc(uint4 (&b)[2][2], const char* img, int wc, int lane, int kc) {
#pragma unroll
  for (int j = 0; j < 2; ++j) b[j][kc] = g8_load_b<T, LAYOUT>(img, wc, j, kc, lane);
}
template <typename T>
__device__ __forceinline__ void g8_mma2_kc(f32x4 (&acc0)[4][2], f32x4 (&acc1)[4][2], const uint4 (&a)[4][2],
                                           const uint4 (&b0)[2][2], const uint4 (&b1)[2][2], int kc) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      Mma<T>::run(acc0[i][j], b0[j][kc], a[i][kc]);
      Mma<T>::run(acc1[i][j], b1[j][kc], a[i][kc]);
    }
}

template <typename T>
__device__ __forceinline__ float g8_sum16b(uint4 x) {  // the elements of one 16-B chunk
  if (sizeof(T) == 4)
    return (__uint_as_float(x.x) + __uint_as_float(x.y)) + (__uint_as_float(x.z) + __uint_as_float(x.w));
  return ((__uint_as_float(x.x << 16) + __uint_as_float(x.x & 0xffff0000u)) +
          (__uint_as_float(x.y << 16) + __uint_as_float(x.y & 0xffff0000u))) +
         ((__uint_as_float(x.z << 16) + __uint_as_float(x.z & 0xffff0000u)) +
          (__uint_as_float(x.w << 16) + __uint_as_float(x.w & 0xffff0000u)));
}
// wave wc sums A subtile wc of the half-tile (its own two LDS reads: a runtime subtile index into
// the fragment registers would push them to scratch)
template <typename T, int LAYOUT>
__device__ __forceinline__ float g8_rowsum(const char* img, int wr, int wc, int lane) {
  return g8_sum16b<T>(load_frag<T, LAYOUT, 128>(img, wr * 4 + wc, 0, lane)) +
         g8_sum16b<T>(load_frag<T, LAYOUT, 128>(img, wr * 4 + wc, 1, lane));
}

// Diagnostic build only (-DMMFD_G8_STAMPS, tools/g8_stamps.py): per-wave s_memtime stamps at
// the phase boundaries of the 256x256 kernel, to a buffer no computation reads.
#ifdef MMFD_G8_STAMPS
constexpr int G8_NSTAMP = 24;  // 0-7 kernel phases, 8-16 the bf16 main-loop segments of K-tile 4
__device__ uint64_t g8_stamps[16384 * 8 * G8_NSTAMP];
#define G8_STAMP(k)                                                                                    \
  do {                                                                                                 \
    const uint64_t t__ = __builtin_amdgcn_s_memtime();                                                \
    const int64_t b__ = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;                                 \
    if (lane == 0 && b__ < 16384) g8_stamps[(b__ * 8 + wave) * G8_NSTAMP + (k)] = t__;                \
  } while (0)
#define G8_PSTAMP(k)                                                                                   \
  do {                                                                                                 \
    if (t == 4) G8_STAMP(k);                                                                           \
  } while (0)
#else
#define G8_STAMP(k) do { } while (0)
#define G8_PSTAMP(k) do { } while (0)
#endif

// Split-operand LDS slots (gemm_x6f.hip): one plane of one 128-row / 128-column half-tile of a
// 32-deep K-step, 8 KB
constexpr int XF_SLOT = 8192;
constexpr int XF_BK = 32;  // K per step

template <int LAYOUT> struct XfImg;  // LDS slot image of one plane of one half-tile
template <> struct XfImg<0> {        // [128 rows][64 B]
  static constexpr int CPR = 4, RPI = 16;  // 64-B rows
  __device__ __forceinline__ static int swz(int r, int c) { return c ^ ((r >> 2) & 2); }
};
template <> struct XfImg<1> {  // [32 K rows][128 bf16]
  static constexpr int CPR = 16, RPI = 4;  // 256-B rows
  __device__ __forceinline__ static int swz(int r, int c) { return Img<bf16, 1, 128>::swz(r, c); }
};

// one 1-KB piece of one plane slot per wave (8 waves fill the 8-KB slot)
template <int LAYOUT>
struct XfFill {
  uint32_t off;
  int cbase;  // layout 0: the element column (k) of this lane's chunk within the K-step
  __device__ __forceinline__ void init(int64_t ld, int64_t mn0, int64_t mn_ext, int wave, int lane) {
    using I = XfImg<LAYOUT>;
    const int row = wave * I::RPI + lane / I::CPR;
    const int c = I::swz(row, lane % I::CPR);
    int64_t el;
    bool ok;
    if (LAYOUT == 0) { el = (mn0 + row) * ld + (int64_t)c * 8; ok = mn0 + row < mn_ext; cbase = c * 8; }
    else { el = (int64_t)row * ld + mn0 + (int64_t)c * 8; ok = mn0 + (int64_t)c * 8 < mn_ext; cbase = 0; }
    off = ok ? (uint32_t)(el * 2) : OOB;
  }
  // soff: byte offset of (plane, K-step) in the operand's planes
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* slot, uint32_t soff, int64_t k0, int64_t K,
                                        int wave) const {
    uint32_t o = off;
    if (LAYOUT == 0 && k0 + XF_BK > K && k0 + (int64_t)cbase >= K) o = OOB;  // partial last K-step
    dma16(rs, slot + wave * 1024, o, soff);
  }
};

// fragment of 16 rows (A) of a layout-0 slot: lane (g, i) = row sub*16 + i, k-chunk g
__device__ __forceinline__ uint4 xf_frag_a0(const char* img, int sub, int lane) {
  const int g = lane >> 4, i = lane & 15, row = sub * 16 + i;
  return lds_read16(img, row * 64 + (XfImg<0>::swz(row, g) << 4));
}
template <int LAYOUT>
__device__ __forceinline__ uint4 xf_frag_a(const char* img, int sub, int lane) {
  if constexpr (LAYOUT == 0) return xf_frag_a0(img, sub, lane);
  else return load_frag<bf16, 1, 128>(img, sub, 0, lane);
}
// B fragment j of the wave's 32 columns (column units 2p + j, see g8_load_b)
template <int LAYOUT>
__device__ __forceinline__ uint4 xf_frag_b(const char* img, int wc, int j, int lane) {
  if constexpr (LAYOUT == 0) {
    const int g = lane >> 4, i = lane & 15;
    const int row = wc * 32 + 4 * (2 * (i >> 2) + j) + (i & 3);
    return lds_read16(img, row * 64 + (XfImg<0>::swz(row, g) << 4));
  } else {
    return g8_load_b<bf16, 1>(img, wc, j, 0, lane);
  }
}


// Epilogue of the 256x256 kernels (gemm256_kernel, gemm256_x6f_kernel): two passes of 128 rows
// (quadrant row mq = pass); every wave stages its fp32 accumulators, then all threads apply the
// epilogue to 8-column chunks with 16-B accesses
template <typename TC, bool PRE>
__device__ __forceinline__ void g8_epilogue(f32x4 (&acc)[2][2][4][2], char* smem, const EpiArgs& e, TC* __restrict__ C,
                                            int64_t ldc, float* __restrict__ ws, int split, int64_t M, int64_t N,
                                            float alpha, int64_t m0, int64_t n0, int tid, int lane, int wave,
                                            int wr, int wc) {
  constexpr int LDC = G8_BN + 4;
  float* ct = reinterpret_cast<float*>(smem);
  const int g = lane >> 4, ci = lane & 15;
  const uint32_t seed = (!ws && e.p > 0.0f) ? mmfd_hash_key(*e.seed, e.salt) : 0u;  // dropout hash key
  float* slab = ws ? ws + (int64_t)split * M * N : nullptr;
  // fast path (full tile, 16-B aligned operands, no split-K slab): every thread owns the same 8
  // columns in all its rows, so the bias is loaded once; per pass all residual / aux / C loads of
  // the thread's 8 rows are issued before any math or store (one wait per pass, not per row)
  if (!slab && e.vec && m0 + G8_BM <= M && n0 + G8_BN <= N) {
    const int c8 = (tid % (G8_BN / 8)) * 8;
    const int64_t col = n0 + c8;
    float bia[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) bia[u] = e.bias ? e.bias[col + u] : 0.f;
    const bool bwd_act = e.act == MMFD_ACT_GELU_BWD || e.act == MMFD_ACT_RELU_BWD;
    const bool fwd_act = e.act == MMFD_ACT_GELU || e.act == MMFD_ACT_RELU;
    // one pass per 128-row half; a lambda per pass (not an unrolled loop, whose body is too big to
    // unroll) keeps every accumulator index a compile-time constant
    auto pass = [&](auto mqc) {
      constexpr int mq = decltype(mqc)::value;
      if constexpr (PRE) {
        // exactly one operand stream (residual OR aux OR C; chosen on the host): all IT rows of it
        // are loaded before the accumulators are staged, so their HBM latency overlaps the
        // staging and its barrier instead of being paid once per row group
        constexpr int IT = 128 * (G8_BN / 8) / NT;
        const int lr0 = tid / (G8_BN / 8);
        const int64_t rstep = NT / (G8_BN / 8);
        const int64_t rbase = m0 + mq * 128;
        const int oc = lr0 * (int)ldc + c8, orr = lr0 * (int)e.ldr + c8, oa = lr0 * (int)e.ldaux + c8;
        TC* cp = C + rbase * ldc + n0 + oc;
        const int64_t cs = rstep * ldc, rs = rstep * e.ldr, xs = rstep * e.ldaux;
        const bool res = e.residual != nullptr;
        const TC* lp = res ? reinterpret_cast<const TC*>(e.residual) + rbase * e.ldr + n0 + orr
                           : bwd_act ? reinterpret_cast<const TC*>(e.aux) + rbase * e.ldaux + n0 + oa : cp;
        const int64_t ls = res ? rs : (bwd_act ? xs : cs);
        Raw8<TC> pre[IT];
#pragma unroll
        for (int k = 0; k < IT; ++k) pre[k].load(lp + k * ls);
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              *reinterpret_cast<f32x4*>(ct + (wr * 64 + i * 16 + ci) * LDC + nq * 128 + wc * 32 + 8 * g + 4 * j) =
                  acc[mq][nq][i][j];
        __syncthreads();
        TC* ap = (fwd_act && e.aux) ? reinterpret_cast<TC*>(e.aux) + rbase * e.ldaux + n0 + oa : nullptr;
        const uint64_t hidx = (uint64_t)(rbase + lr0) * (uint64_t)N + (uint64_t)col;
        const float* src = ct + lr0 * LDC + c8;
#pragma unroll
        for (int kk = 0; kk < IT; ++kk) {
          const float4 a4 = *reinterpret_cast<const float4*>(src + kk * rstep * LDC);
          const float4 b4 = *reinterpret_cast<const float4*>(src + kk * rstep * LDC + 4);
          float z[8] = {a4.x, a4.y, a4.z, a4.w, b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int u = 0; u < 8; ++u) z[u] = fmaf(alpha, z[u], bia[u]);
          float t[8];
          pre[kk].get(t);
          if (res && e.res_first) {
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] += t[u];
          }
          if (fwd_act) {
            if (ap) V8<TC>::store(ap + kk * xs, z);
            if (e.act == MMFD_ACT_GELU) {
#pragma unroll
              for (int u = 0; u < 8; ++u) z[u] = gelu_f(z[u]);
            } else {
#pragma unroll
              for (int u = 0; u < 8; ++u) z[u] = fmaxf(z[u], 0.f);
            }
          } else if (bwd_act) {
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
          if (res && !e.res_first) {
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] += t[u];
          }
          if (!res && !bwd_act) {  // the stream is C: beta * C
#pragma unroll
            for (int u = 0; u < 8; ++u) z[u] = fmaf(e.beta, t[u], z[u]);
          }
          V8<TC>::store(cp + kk * cs, z);
        }
        __syncthreads();
      } else {
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            *reinterpret_cast<f32x4*>(ct + (wr * 64 + i * 16 + ci) * LDC + nq * 128 + wc * 32 + 8 * g + 4 * j) =
                acc[mq][nq][i][j];
      if (mq == 0) G8_STAMP(3);
      __syncthreads();
      if (mq == 0) G8_STAMP(4);
      constexpr int IT = 128 * (G8_BN / 8) / NT;  // 8 rows per thread, in two groups of 4
      // every thread owns 8 columns of rows lr0 + 16 k (k < IT): the operand / output row pointers
      // advance by a scalar stride (no per-row 64-bit address math), every epilogue branch is
      // uniform, and the residual / aux / C loads of GI rows are in flight before their math
      const int lr0 = tid / (G8_BN / 8);
      const int64_t rstep = NT / (G8_BN / 8);  // 16 rows between a thread's rows
      const int64_t rbase = m0 + mq * 128;     // uniform part of the row
      // uniform (scalar) tile bases + 32-bit per-lane offsets (host-checked: operands < 2^31 elements)
      const int oc = lr0 * (int)ldc + c8, orr = lr0 * (int)e.ldr + c8, oa = lr0 * (int)e.ldaux + c8;
      TC* cp = C + rbase * ldc + n0 + oc;
      const TC* rp = e.residual ? reinterpret_cast<const TC*>(e.residual) + rbase * e.ldr + n0 + orr : nullptr;
      const TC* xp = bwd_act ? reinterpret_cast<const TC*>(e.aux) + rbase * e.ldaux + n0 + oa : nullptr;
      TC* ap = (fwd_act && e.aux) ? reinterpret_cast<TC*>(e.aux) + rbase * e.ldaux + n0 + oa : nullptr;
      const uint64_t hidx = (uint64_t)(rbase + lr0) * (uint64_t)N + (uint64_t)col;
      const int64_t cs = rstep * ldc, rs = rstep * e.ldr, xs = rstep * e.ldaux;
      const float* src = ct + lr0 * LDC + c8;
      constexpr int GI = 2;
#pragma unroll
      for (int k0 = 0; k0 < IT; k0 += GI) {
        Raw8<TC> rres[GI], raux[GI], rc[GI];
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
            if (ap) V8<TC>::store(ap + kk * xs, z);
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
          if (std::is_same<TC, float>::value && e.pl) {
            planes_store8(e, N, rbase + lr0 + kk * rstep, col, z);
            if (!e.c_out) continue;
          }
          V8<TC>::store(cp + kk * cs, z);
        }
      }
      __syncthreads();
      if (mq == 0) G8_STAMP(5);
      }
    };
    pass(std::integral_constant<int, 0>{});
    pass(std::integral_constant<int, 1>{});
    G8_STAMP(6);
#ifdef MMFD_G8_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    G8_STAMP(7);
#endif
    return;
  }
#pragma unroll
  for (int mq = 0; mq < 2; ++mq) {
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<f32x4*>(ct + (wr * 64 + i * 16 + ci) * LDC + nq * 128 + wc * 32 + 8 * g + 4 * j) =
              acc[mq][nq][i][j];
    __syncthreads();
    const int64_t rbase = m0 + mq * 128;
    for (int idx = tid; idx < 128 * (G8_BN / 8); idx += NT) {
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
        epilogue_store8<TC>(e, C, ldc, N, row, col, vv, seed);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (col + u < N) epilogue_store<TC>(e, C, ldc, N, row, col + u, vv[u], seed);
      }
    }
    __syncthreads();
  }
}

}  // namespace
