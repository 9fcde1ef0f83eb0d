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
}  // namespace mmfd_gemmx

namespace {
using mmfd_gemmx::EpiArgs;
using mmfd_gemmx::X6Args;
using mmfd_gemmx::X6_CA;
using mmfd_gemmx::X6_CB;
using mmfd_gemmx::X6_RS;


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
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[8]) {
    bf16x8 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
    *reinterpret_cast<uint4*>(p) = __builtin_bit_cast(uint4, o);
  }
};
template <> struct V8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
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


}  // namespace
