// Flash-style multi-head attention for gfx950 (head_dim 32 or 64, L <= a few hundred).
//
// Replaces: src/model/layers.py:36-58 (MultiHeadAttention, eager and SDPA branches; no mask) and the
// self-attention of the HF BERT / ViT / MPNet encoders called at train.py:137-143 (key padding mask
// as an additive per-key bias, MPNet relative-position bias as an additive [H][Lq][Lk] bias).
//
// Every product runs on 16x16 MFMAs (bf16: 16x16x32, fp32: 16x16x4). Work split:
//   forward  : workgroup = (b, h, 64 queries), wave = 16 queries; loops over 64-key blocks staged
//              in LDS. S^T = K Q^T puts the query on the lane, so the online-softmax statistics are
//              lane-local (reduced over 4 lanes) and P^T's accumulator is directly the A operand of
//              O = P V (keys in the "split" order {4g..4g+3, 16+4g..16+4g+3}); V is read with the
//              hardware-transposing ds_read_b64_tr_b16.
//   backward : two kernels, no atomics (deterministic): dK/dV per 64-key block looping over query
//              blocks (S = Q K^T puts the key on the lane: P and dS are directly the A operands of
//              dV = P^T dO and dK = dS^T Q), and dQ per 64-query block looping over key blocks
//              (S^T again). delta = rowsum(dO * O) comes from a small kernel first.
// Dropout on P (layers.py:53 / SDPA dropout_p) is counter based: index ((b*H+h)*Lq+q)*Lk+k.
#include "common.h"
#include <algorithm>
#include <type_traits>
#include <math.h>
#include <stdlib.h>
#include <string.h>

namespace {

struct AttnP {
  int64_t B, H, Lq, Lk;
  int D;  // real head dim (<= the template's padded D; padding columns are zero)
  float scale;
  const void* q; int64_t q_sb, q_st;
  const void* k; int64_t k_sb, k_st;
  const void* v; int64_t v_sb, v_st;
  void* o; int64_t o_sb, o_st;
  float* lse;
  const float* key_bias;
  const float* rel_bias; int64_t rb_sb, rb_mod;
  const float* cos_ls; float cos_max_log;  // Swinv2 cosine attention (REL forward only)
  float p; uint32_t thr16; float keep_scale;
  int64_t kp;  // key pairs per query row, ceil(Lk / 2): attention dropout hashes one index per pair
  const uint64_t* seed; uint64_t salt;
  const void* dout; int64_t do_sb, do_st;
  void* dq; int64_t dq_sb, dq_st;
  void* dk; int64_t dk_sb, dk_st;
  void* dv; int64_t dv_sb, dv_st;
  float* delta;
  int acc_dq, acc_dkv;
  // fp32 backward: split planes of the packed [dq | dk | dv] buffer (base = dq), see mmfd_attn_args
  bf16* pl; int64_t pl_stride; const float* pl_base; int pl_only;
  int idx32;  // every dropout index fits 32 bits (hash_c1)
  int vst;    // x6 backward stores as 4-column groups (16-B fp32, 8-B planes): outputs and planes aligned
  int dbg;  // x6 phase experiments (MMFD_X6A_DBG): 1 = stage zeros, 2 = skip the products
  // dropout keep-bitmask (mmfd_attn_args::drop_mask): forward kernels that hash the mask write it,
  // backward kernels read it instead of re-hashing; dmw = words per query row, dm_lds = the dK/dV
  // kernel stages the head's rows in LDS (room left by its images)
  uint32_t* dm; int dmw; int dm_lds;
};

// word ((b*H + h)*Lq + q)*dmw + k/32 of the keep-bitmask, bit k % 32 = 1 when element (q, k) is kept
__device__ __forceinline__ uint32_t* dm_row(const AttnP& p, int64_t bh, int64_t q) { return p.dm + (bh * p.Lq + q) * p.dmw; }
// forward, S^T layout (lane (g, li): query q0 + li, keys k0 + ks*16 + 4g + r): `kb` holds the lane's
// keep bits of one 64-key chunk at bit ks*4 + r; the four lane groups' bits are merged by shuffles
// into the words k0/32 and k0/32 + 1 of the query's row (all 64 lanes must be active)
__device__ __forceinline__ void dm_write64(const AttnP& p, int64_t bh, int64_t myq, int k0, int g, uint32_t kb) {
  uint32_t w0 = ((kb & 0xFu) << (4 * g)) | (((kb >> 4) & 0xFu) << (16 + 4 * g));
  uint32_t w1 = (((kb >> 8) & 0xFu) << (4 * g)) | (((kb >> 12) & 0xFu) << (16 + 4 * g));
  w0 |= __shfl_xor(w0, 16, 64);
  w0 |= __shfl_xor(w0, 32, 64);
  w1 |= __shfl_xor(w1, 16, 64);
  w1 |= __shfl_xor(w1, 32, 64);
  if (myq < p.Lq) {
    const int w = k0 >> 5;
    uint32_t* row = dm_row(p, bh, myq);
    if (g == 0 && w < p.dmw) row[w] = w0;
    if (g == 1 && w + 1 < p.dmw) row[w + 1] = w1;
  }
}

// one fp32 gradient element into the planes at its offset in the packed buffer
__device__ __forceinline__ void plane_put(const AttnP& p, const float* dst, float v) {
  const int64_t off = dst - p.pl_base;
  const bf16 h = (bf16)v;
  const float r = v - (float)h;
  const bf16 m = (bf16)r;
  p.pl[off] = h;
  p.pl[off + p.pl_stride] = m;
  p.pl[off + 2 * p.pl_stride] = (bf16)(r - (float)m);
}

// Dropout with 32-bit indices (B*H*Lq*Lk <= 2^32: AttnP::idx32, required by the x6 kernels): mmfd_hash_k(key, idx) = mix32(key ^ lo(idx) * C1 ^
// hi(idx) * C2) with hi(idx) = 0, and lo(idx) * C1 (mod 2^32) advances by additions — C1 per key,
// Lk * C1 per query — so an element costs one v_add in place of the 64-bit index arithmetic and
// its two extra 32-bit multiplies (bit-identical masks).
constexpr uint32_t HASH_C1 = 0x9e3779b1u;

// 4x4 transpose across each lane quad (lanes 4j + t): afterwards lane t, register c holds what lane
// c held in register t. A 16x16 MFMA accumulator (lane (g, i): rows 4g + r, column i) becomes
// rows 4g + (i & 3) with 4 consecutive columns 4 (i >> 2) + c per lane — one 16-B fp32 store and
// 8-B plane stores per 4 outputs instead of one 4-B and three 2-B stores per output
__device__ __forceinline__ void quad_tr(float (&x)[4], int t) {
  const bool o1 = t & 1, o2 = t & 2;
#pragma unroll
  for (int j = 0; j < 4; j += 2) {
    const float r = __shfl_xor(o1 ? x[j] : x[j + 1], 1, 64);
    if (o1) x[j] = r; else x[j + 1] = r;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float r = __shfl_xor(o2 ? x[j] : x[j + 2], 2, 64);
    if (o2) x[j] = r; else x[j + 2] = r;
  }
}

typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

// four consecutive fp32 outputs at dst (16-B aligned; AttnP::vst), accumulated onto dst when acc,
// and their split planes when p.pl (the same split3 rule as plane_put)
__device__ __forceinline__ void x6_put4(const AttnP& p, float* dst, const float (&x)[4], bool acc) {
  float4 v = make_float4(x[0], x[1], x[2], x[3]);
  if (acc) {
    const float4 o = *reinterpret_cast<const float4*>(dst);
    v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
  }
  if (p.pl) {
    const float e[4] = {v.x, v.y, v.z, v.w};
    bf16x4 h, m, l;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bf16 hu = (bf16)e[u];
      const float r = e[u] - (float)hu;
      const bf16 mu = (bf16)r;
      h[u] = hu;
      m[u] = mu;
      l[u] = (bf16)(r - (float)mu);
    }
    bf16* pp = p.pl + (dst - p.pl_base);
    *reinterpret_cast<uint2*>(pp) = __builtin_bit_cast(uint2, h);
    *reinterpret_cast<uint2*>(pp + p.pl_stride) = __builtin_bit_cast(uint2, m);
    *reinterpret_cast<uint2*>(pp + 2 * p.pl_stride) = __builtin_bit_cast(uint2, l);
    if (p.pl_only) return;
  }
  *reinterpret_cast<float4*>(dst) = v;
}
__device__ __forceinline__ uint32_t hash_c1(uint32_t key, uint32_t idx_c1) { return mmfd_mix32(key ^ idx_c1); }

// Attention dropout draws ONE 32-bit hash per key pair: element (row, k) of the [B*H*Lq][Lk] score
// matrix (row = (b*H + h)*Lq + q) uses h = mmfd_hash_k(key, row * kp + k / 2), kp = ceil(Lk / 2),
// and is kept when its 16-bit half (low for even k, high for odd k) is >= thr16 = round(p * 65536)
// (p = 0.1: thr16 = 6554, a keep probability within 6e-6 of 0.9). oracle/dropout_hash.py
// attn_keep_mask restates it. A lane holding 4 consecutive keys (forward, dQ) hashes twice where it
// hashed four times; a lane holding one key of 4 queries (dK/dV) hashes 2 of the 4 pairs and takes
// the other 2 from its neighbour lane (the pair partner key).
__device__ __forceinline__ bool pair_keep(uint32_t h, int odd, uint32_t thr16) {
  return (odd ? (h >> 16) : (h & 0xffffu)) >= thr16;
}
__device__ __forceinline__ uint32_t attn_hash64(uint32_t hkey, const AttnP& p, int64_t row, int64_t key) {
  return mmfd_hash_k(hkey, (uint64_t)row * (uint64_t)p.kp + (uint64_t)(key >> 1));
}
// keep factors (keep_scale or 0) of 4 consecutive keys starting at an even key, from the pair hashes
// h0 (keys 0, 1) and h1 (keys 2, 3)
__device__ __forceinline__ void keep4_pairs(uint32_t h0, uint32_t h1, const AttnP& p, float (&z)[4]) {
  z[0] = pair_keep(h0, 0, p.thr16) ? p.keep_scale : 0.f;
  z[1] = pair_keep(h0, 1, p.thr16) ? p.keep_scale : 0.f;
  z[2] = pair_keep(h1, 0, p.thr16) ? p.keep_scale : 0.f;
  z[3] = pair_keep(h1, 1, p.thr16) ? p.keep_scale : 0.f;
}
// one key per lane, 4 query rows r: this lane hashed rows (odd ? 2 : 0) -> ha and (odd ? 3 : 1) -> hb
// of its key pair; the partner lane (lane ^ 1, the pair's other key) hashed the other two rows. All
// 64 lanes must be active.
__device__ __forceinline__ void keep4_col(uint32_t ha, uint32_t hb, int odd, const AttnP& p, float (&z)[4]) {
  const uint32_t xa = __shfl_xor(ha, 1, 64), xb = __shfl_xor(hb, 1, 64);
  const uint32_t h[4] = {odd ? xa : ha, odd ? xb : hb, odd ? ha : xa, odd ? hb : xb};
#pragma unroll
  for (int r = 0; r < 4; ++r) z[r] = pair_keep(h[r], odd, p.thr16) ? p.keep_scale : 0.f;
}

template <typename T, int D>
struct AT {
  static constexpr int ESZ = sizeof(T);
  static constexpr int RB = D * ESZ;          // bytes per row
  static constexpr int NCH = RB / 16;         // 16-B chunks per row
  static constexpr int EPC = 16 / ESZ;
  static constexpr int KCH = D / Mma<T>::KC;  // MFMA chunks along D
  static constexpr int TILE = 64 * RB;        // one 64-row image
  static constexpr int DT = D / 16;           // 16-wide output subtiles along D
  static constexpr int PCH = 64 / Mma<T>::KC; // MFMA chunks along a 64-row block
};

// ROW image: 16-B chunk c of row r
template <typename T, int D>
__device__ __forceinline__ int row_off(int r, int c) {
  constexpr int NCH = AT<T, D>::NCH;
  return r * AT<T, D>::RB + ((c ^ (r & (NCH - 1))) << 4);
}
// TR image: 16-B chunk c of row r (layout chosen for the transposed operand reads)
template <typename T, int D>
__device__ __forceinline__ int tr_chunk(int r, int c) {
  if (sizeof(T) == 2) {
    // D = 64 (128-B rows): the ROW swizzle c ^ (r & 7) is also conflict-free for the transposed
    // 8-row reads, so one image serves both kinds of read (DUAL below)
    if (D == 64) return c ^ (r & 7);
    return c ^ (2 * ((r >> 2) & 1));
  }
  // fp32: the ROW swizzle c ^ (r & (NCH-1)) again; the 4-byte transposed reads of rows r+4g
  // (g = 0..3) then land in distinct 4-chunk groups at D = 64 (16 chunks per row)
  return c ^ (r & (AT<T, D>::NCH - 1));
}

// stage 64 rows [row0, row0+64) of a (token-strided) head slice into an image
template <typename T, int D, bool TR>
__device__ __forceinline__ void stage_rows(char* lds, const T* __restrict__ base, int64_t st, int64_t row0,
                                           int64_t nrows, int tid, int dreal) {
  constexpr int NCH = AT<T, D>::NCH, EPC = AT<T, D>::EPC;
  for (int c = tid; c < 64 * NCH; c += 256) {
    const int r = c / NCH, ch = c % NCH;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row0 + r < nrows && ch * EPC < dreal) v = *reinterpret_cast<const uint4*>(base + (row0 + r) * st + ch * EPC);
    const int off = TR ? (r * AT<T, D>::RB + (tr_chunk<T, D>(r, ch) << 4)) : row_off<T, D>(r, ch);
    *reinterpret_cast<uint4*>(lds + off) = v;
  }
}

// A-operand fragment (16 rows starting at sub*16) from a ROW image, MFMA chunk kc along D
template <typename T, int D>
__device__ __forceinline__ uint4 row_frag(const char* lds, int sub, int kc, int lane) {
  const int row = sub * 16 + (lane & 15);
  return lds_read16(lds, row_off<T, D>(row, kc * 4 + (lane >> 4)));
}

// B-operand fragment from a TR image: k = rows of the 64-row block (split order for bf16),
// n = 16 columns starting at dsub*16. chunk c covers rows [c*KC, c*KC+KC).
template <typename T, int D>
__device__ __forceinline__ uint4 tr_frag(const char* lds, int c, int dsub, int lane) {
  const int g = lane >> 4, i = lane & 15;
  constexpr int RB = AT<T, D>::RB;
  if (sizeof(T) == 2) {
    const int q = i >> 2, p = i & 3;
    const int u = dsub * 4 + p;  // 8-B unit (4 bf16)
    uint2 x[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = c * 32 + 16 * h + 4 * g + q;
      const int ch = tr_chunk<T, D>(r, u >> 1);
      x[h] = lds_read_tr16(lds + r * RB + (ch << 4) + ((u & 1) << 3));
    }
    return make_uint4(x[0].x, x[0].y, x[1].x, x[1].y);
  } else {
    const int col = dsub * 16 + i;
    uint32_t v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r = c * 16 + 4 * g + s;
      const int ch = tr_chunk<T, D>(r, col >> 2);
      v[s] = *reinterpret_cast<const uint32_t*>(lds + r * RB + (ch << 4) + (col & 3) * 4);
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
}

// pack 16x16 accumulators (rows in split order) into the A fragment of MFMA chunk c
template <typename T>
__device__ __forceinline__ uint4 pack_acc(const f32x4* s, int c) {
  if (sizeof(T) == 2) {
    const f32x4 a = s[2 * c], b = s[2 * c + 1];
    bf16x8 v = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
    return __builtin_bit_cast(uint4, v);
  } else {
    const f32x4 a = s[c];
    return make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3]));
  }
}

// dot product of two 16-B chunks of T elements (fp32 sum)
template <typename T>
__device__ __forceinline__ float row_chunk_dot(const uint4& a, const uint4& b) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 x = __builtin_bit_cast(bf16x8, a), y = __builtin_bit_cast(bf16x8, b);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s = fmaf((float)x[e], (float)y[e], s);
    return s;
  } else {
    return fmaf(__uint_as_float(a.x), __uint_as_float(b.x),
                fmaf(__uint_as_float(a.y), __uint_as_float(b.y),
                     fmaf(__uint_as_float(a.z), __uint_as_float(b.z), __uint_as_float(a.w) * __uint_as_float(b.w))));
  }
}

// per-lane 16-B operand chunks of one row (query or key) held in registers
template <typename T, int D>
__device__ __forceinline__ void load_row_regs(uint4* f, const T* __restrict__ base, int64_t st,
                                              int64_t row, int64_t nrows, int lane, int dreal) {
  const int g = lane >> 4;
#pragma unroll
  for (int kc = 0; kc < AT<T, D>::KCH; ++kc) {
    f[kc] = make_uint4(0, 0, 0, 0);
    const int col = (kc * 4 + g) * AT<T, D>::EPC;
    if (row < nrows && col < dreal) f[kc] = *reinterpret_cast<const uint4*>(base + row * st + col);
  }
}

// batch offset of rel_bias: b * sb, or (b % mod) * sb when the bias repeats every `mod` batch rows
// (Swinv2 shifted-window masks: one [H][L][L] bias per window position, windows batch-major)
__device__ __forceinline__ int64_t rb_off(const AttnP& p, int64_t b) {
  return (p.rb_mod > 0 ? b % p.rb_mod : b) * p.rb_sb;
}

__device__ __forceinline__ float bias_at(const AttnP& p, int64_t b, int64_t h, int64_t q, int64_t key) {
  float v = 0.f;
  if (p.key_bias) v += p.key_bias[b * p.Lk + key];
  if (p.rel_bias) v += p.rel_bias[rb_off(p, b) + (h * p.Lq + q) * p.Lk + key];
  return v;
}

// --------------------------------------------------------------------------------------------
// forward
// --------------------------------------------------------------------------------------------
template <typename T, int D>
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnP p) {
  using C = AT<T, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* k_img = smem;
  char* v_img = smem + C::TILE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int64_t bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t q0 = (int64_t)blockIdx.x * 64 + wave * 16;
  const T* qb = reinterpret_cast<const T*>(p.q) + b * p.q_sb + h * p.D;
  const T* kb = reinterpret_cast<const T*>(p.k) + b * p.k_sb + h * p.D;
  const T* vb = reinterpret_cast<const T*>(p.v) + b * p.v_sb + h * p.D;
  const int64_t myq = q0 + li;

  uint4 qf[C::KCH];
  load_row_regs<T, D>(qf, qb, p.q_st, myq, p.Lq, lane, p.D);
  const uint64_t seed = p.p > 0.f ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);

  float m = -INFINITY, lsum = 0.f;
  f32x4 o[C::DT];
#pragma unroll
  for (int d = 0; d < C::DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int64_t k0 = 0; k0 < p.Lk; k0 += 64) {
    __syncthreads();
    stage_rows<T, D, false>(k_img, kb, p.k_st, k0, p.Lk, tid, p.D);
    stage_rows<T, D, true>(v_img, vb, p.v_st, k0, p.Lk, tid, p.D);
    __syncthreads();

    f32x4 s[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      s[ks] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) Mma<T>::run(s[ks], row_frag<T, D>(k_img, ks, kc, lane), qf[kc]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t key = k0 + ks * 16 + 4 * g + r;
        float v = s[ks][r] * p.scale;
        if (key >= p.Lk) v = -INFINITY;
        else if (p.key_bias || p.rel_bias) v += bias_at(p, b, h, myq < p.Lq ? myq : 0, key);
        s[ks][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx);
    const float alpha = __expf(m - mnew);
    float rs = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __expf(s[ks][r] - mnew);
        rs += e;
        float pe = e;
        if (p.p > 0.f) {
          const int64_t key = k0 + ks * 16 + 4 * g + r;
          const uint32_t hsh = attn_hash64(hkey, p, bh * p.Lq + myq, key);
          pe = pair_keep(hsh, (int)(key & 1), p.thr16) ? e * p.keep_scale : 0.f;
        }
        s[ks][r] = pe;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    lsum = lsum * alpha + rs;
    m = mnew;
    // rescale O rows (row = local query 4g+r, whose alpha sits in lane 4g+r)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) o[d][r] *= ar;
    }
#pragma unroll
    for (int c = 0; c < C::PCH; ++c) {
      const uint4 a = pack_acc<T>(s, c);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) Mma<T>::run(o[d], a, tr_frag<T, D>(v_img, c, d, lane));
    }
  }

  T* ob = reinterpret_cast<T*>(p.o) + b * p.o_sb + h * p.D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float lr = __shfl(lsum, 4 * g + r, 64);
    const int64_t q = q0 + 4 * g + r;
    const float inv = 1.0f / lr;
    if (q < p.Lq) {
#pragma unroll
      for (int d = 0; d < C::DT; ++d)
        if (d * 16 + li < p.D) ob[q * p.o_st + d * 16 + li] = from_f32<T>(o[d][r] * inv);
    }
  }
  if (g == 0 && myq < p.Lq) p.lse[bh * p.Lq + myq] = m + __logf(lsum);
}

// --------------------------------------------------------------------------------------------
// backward: delta = rowsum(dO * O)
// --------------------------------------------------------------------------------------------
template <typename T, int D>
__global__ void attn_delta_kernel(AttnP p) {
  // 8 lanes per (b,h,q) row for D=64 (4 for D=32): each lane a 16-B chunk
  constexpr int LPR = AT<T, D>::NCH;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = gid / LPR;
  const int ch = gid % LPR;
  const int64_t total = p.B * p.H * p.Lq;
  float s = 0.f;
  if (row < total) {
    const int64_t q = row % p.Lq, bh = row / p.Lq, b = bh / p.H, h = bh % p.H;
    if (ch * AT<T, D>::EPC < p.D) {
      const T* o = reinterpret_cast<const T*>(p.o) + b * p.o_sb + q * p.o_st + h * p.D + ch * AT<T, D>::EPC;
      const T* d = reinterpret_cast<const T*>(p.dout) + b * p.do_sb + q * p.do_st + h * p.D + ch * AT<T, D>::EPC;
#pragma unroll
      for (int j = 0; j < AT<T, D>::EPC; ++j) s += to_f32(o[j]) * to_f32(d[j]);
    }
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (row < total && ch == 0) p.delta[row] = s;
}

// --------------------------------------------------------------------------------------------
// backward: dK, dV (workgroup = 64 keys, wave = 16 keys)
// --------------------------------------------------------------------------------------------
template <typename T, int D>
__global__ void __launch_bounds__(256) attn_bwd_dkdv_kernel(AttnP p) {
  using C = AT<T, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* q_row = smem;
  char* q_tr = smem + C::TILE;
  char* do_row = smem + 2 * C::TILE;
  char* do_tr = smem + 3 * C::TILE;
  float* s_lse = reinterpret_cast<float*>(smem + 4 * C::TILE);
  float* s_delta = s_lse + 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int64_t bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t k0 = (int64_t)blockIdx.x * 64 + wave * 16;
  const int64_t mykey = k0 + li;
  const T* qb = reinterpret_cast<const T*>(p.q) + b * p.q_sb + h * p.D;
  const T* kb = reinterpret_cast<const T*>(p.k) + b * p.k_sb + h * p.D;
  const T* vb = reinterpret_cast<const T*>(p.v) + b * p.v_sb + h * p.D;
  const T* dob = reinterpret_cast<const T*>(p.dout) + b * p.do_sb + h * p.D;
  const uint64_t seed = p.p > 0.f ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);

  uint4 kf[C::KCH], vf[C::KCH];
  load_row_regs<T, D>(kf, kb, p.k_st, mykey, p.Lk, lane, p.D);
  load_row_regs<T, D>(vf, vb, p.v_st, mykey, p.Lk, lane, p.D);

  f32x4 dk[C::DT], dv[C::DT];
#pragma unroll
  for (int d = 0; d < C::DT; ++d) { dk[d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[d] = dk[d]; }

  for (int64_t qs0 = 0; qs0 < p.Lq; qs0 += 64) {
    __syncthreads();
    stage_rows<T, D, false>(q_row, qb, p.q_st, qs0, p.Lq, tid, p.D);
    stage_rows<T, D, true>(q_tr, qb, p.q_st, qs0, p.Lq, tid, p.D);
    stage_rows<T, D, false>(do_row, dob, p.do_st, qs0, p.Lq, tid, p.D);
    stage_rows<T, D, true>(do_tr, dob, p.do_st, qs0, p.Lq, tid, p.D);
    if (tid < 64) {
      const int64_t q = qs0 + tid;
      s_lse[tid] = q < p.Lq ? p.lse[bh * p.Lq + q] : INFINITY;
      s_delta[tid] = q < p.Lq ? p.delta[bh * p.Lq + q] : 0.f;
    }
    __syncthreads();

    f32x4 pd[4], ds[4];
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sv;
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) {
        Mma<T>::run(sv, row_frag<T, D>(q_row, qs, kc, lane), kf[kc]);
        Mma<T>::run(dp, row_frag<T, D>(do_row, qs, kc, lane), vf[kc]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lq = qs * 16 + 4 * g + r;
        const int64_t q = qs0 + lq;
        float pr = 0.f;
        if (mykey < p.Lk) {
          float sc = sv[r] * p.scale;
          if ((p.key_bias || p.rel_bias) && q < p.Lq) sc += bias_at(p, b, h, q, mykey);
          pr = __expf(sc - s_lse[lq]);
        }
        float z = 1.f;
        if (p.p > 0.f) {
          const uint32_t hsh = attn_hash64(hkey, p, bh * p.Lq + q, mykey);
          z = pair_keep(hsh, (int)(mykey & 1), p.thr16) ? p.keep_scale : 0.f;
        }
        pd[qs][r] = pr * z;
        ds[qs][r] = pr * (dp[r] * z - s_delta[lq]);
      }
    }
#pragma unroll
    for (int c = 0; c < C::PCH; ++c) {
      const uint4 ap = pack_acc<T>(pd, c);
      const uint4 as = pack_acc<T>(ds, c);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        Mma<T>::run(dv[d], ap, tr_frag<T, D>(do_tr, c, d, lane));
        Mma<T>::run(dk[d], as, tr_frag<T, D>(q_tr, c, d, lane));
      }
    }
  }

  T* dkb = reinterpret_cast<T*>(p.dk) + b * p.dk_sb + h * p.D;
  T* dvb = reinterpret_cast<T*>(p.dv) + b * p.dv_sb + h * p.D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t key = k0 + 4 * g + r;
    if (key < p.Lk) {
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        if (d * 16 + li >= p.D) continue;
        T* pk = dkb + key * p.dk_st + d * 16 + li;
        T* pv = dvb + key * p.dv_st + d * 16 + li;
        float vk = dk[d][r] * p.scale, vv = dv[d][r];
        if (p.acc_dkv) { vk += to_f32(*pk); vv += to_f32(*pv); }
        *pk = from_f32<T>(vk);
        *pv = from_f32<T>(vv);
      }
    }
  }
}

// --------------------------------------------------------------------------------------------
// backward: dQ (workgroup = 64 queries, wave = 16 queries)
// --------------------------------------------------------------------------------------------
template <typename T, int D>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(AttnP p) {
  using C = AT<T, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* k_row = smem;
  char* k_tr = smem + C::TILE;
  char* v_row = smem + 2 * C::TILE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int64_t bh = blockIdx.y, b = bh / p.H, h = bh % p.H;
  const int64_t q0 = (int64_t)blockIdx.x * 64 + wave * 16;
  const int64_t myq = q0 + li;
  const T* qb = reinterpret_cast<const T*>(p.q) + b * p.q_sb + h * p.D;
  const T* kb = reinterpret_cast<const T*>(p.k) + b * p.k_sb + h * p.D;
  const T* vb = reinterpret_cast<const T*>(p.v) + b * p.v_sb + h * p.D;
  const T* dob = reinterpret_cast<const T*>(p.dout) + b * p.do_sb + h * p.D;
  const uint64_t seed = p.p > 0.f ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);

  uint4 qf[C::KCH], dof[C::KCH];
  load_row_regs<T, D>(qf, qb, p.q_st, myq, p.Lq, lane, p.D);
  load_row_regs<T, D>(dof, dob, p.do_st, myq, p.Lq, lane, p.D);
  const float lse = myq < p.Lq ? p.lse[bh * p.Lq + myq] : INFINITY;
  const float dlt = myq < p.Lq ? p.delta[bh * p.Lq + myq] : 0.f;

  f32x4 dq[C::DT];
#pragma unroll
  for (int d = 0; d < C::DT; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int64_t k0 = 0; k0 < p.Lk; k0 += 64) {
    __syncthreads();
    stage_rows<T, D, false>(k_row, kb, p.k_st, k0, p.Lk, tid, p.D);
    stage_rows<T, D, true>(k_tr, kb, p.k_st, k0, p.Lk, tid, p.D);
    stage_rows<T, D, false>(v_row, vb, p.v_st, k0, p.Lk, tid, p.D);
    __syncthreads();

    f32x4 ds[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sv;
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) {
        Mma<T>::run(sv, row_frag<T, D>(k_row, ks, kc, lane), qf[kc]);
        Mma<T>::run(dp, row_frag<T, D>(v_row, ks, kc, lane), dof[kc]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t key = k0 + ks * 16 + 4 * g + r;
        float pr = 0.f;
        if (key < p.Lk) {
          float sc = sv[r] * p.scale;
          if ((p.key_bias || p.rel_bias) && myq < p.Lq) sc += bias_at(p, b, h, myq, key);
          pr = __expf(sc - lse);
        }
        float z = 1.f;
        if (p.p > 0.f) {
          const uint32_t hsh = attn_hash64(hkey, p, bh * p.Lq + myq, key);
          z = pair_keep(hsh, (int)(key & 1), p.thr16) ? p.keep_scale : 0.f;
        }
        ds[ks][r] = pr * (dp[r] * z - dlt);
      }
    }
#pragma unroll
    for (int c = 0; c < C::PCH; ++c) {
      const uint4 as = pack_acc<T>(ds, c);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) Mma<T>::run(dq[d], as, tr_frag<T, D>(k_tr, c, d, lane));
    }
  }

  T* dqb = reinterpret_cast<T*>(p.dq) + b * p.dq_sb + h * p.D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t q = q0 + 4 * g + r;
    if (q < p.Lq) {
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        if (d * 16 + li >= p.D) continue;
        T* pq = dqb + q * p.dq_st + d * 16 + li;
        float vq = dq[d][r] * p.scale;
        if (p.acc_dq) vq += to_f32(*pq);
        *pq = from_f32<T>(vq);
      }
    }
  }
}

// =================================================================================================
// v2 kernels (Lq and Lk <= 256; bf16 forward up to 512 keys): one workgroup of 8 waves per (b, h).
// The whole K/V (forward, dQ) or Q/dO (dK/dV) of the head is staged in LDS ONCE and every wave
// sweeps 16-row blocks against it: no per-block restaging and no repeated K/V reads from L2. Rows
// are padded only to one MFMA k-chunk (bf16: 32, fp32: 16), so L = 197 computes on 224 / 208 rows
// instead of the streaming kernels' 256.
// =================================================================================================
constexpr int V2_LMAX = 256;      // backward kernels (Q/dO or K/V images of the head); fp32 forward
constexpr int V2_LMAX_FWD = 512;  // bf16 forward: K/V images of 512 keys (128 KB at D = 64) fit the 160-KB LDS
constexpr int V2_THREADS = 512;   // forward / dQ: 8 waves sharing one K/V image
// dK/dV: bf16 images are small enough for two workgroups per CU; an fp32 head image (up to 128 KB)
// allows one, so it gets 8 waves
template <typename T> struct V2T { static constexpr int DKDV_THREADS = sizeof(T) == 4 ? 512 : 256; };
// row image == transposed image (no second copy): bf16 at D = 64 and every fp32 layout
template <typename T, int D> struct V2 { static constexpr bool DUAL = sizeof(T) == 4 || D == 64; };
// rows per MFMA k-chunk, and 16-row subtiles per chunk
template <typename T> __host__ __device__ constexpr int v2_kc() { return sizeof(T) == 2 ? 32 : 16; }
__host__ __device__ inline int v2_pad(int64_t n, int kc) { return (int)((n + kc - 1) / kc * kc); }

// Head staging: STAGE_BATCH 16-B chunks per thread and source are loaded before the first LDS
// write, so a workgroup waits out one global-load latency per batch instead of one per chunk (the
// one-chunk loop waited vmcnt(0) before every ds_write: 14 serial round trips for a ViT dK/dV head)
constexpr int STAGE_BATCH = 4;

template <typename T, int D, bool TR>
__device__ __forceinline__ int stage_off(int r, int ch) {
  return TR ? (r * AT<T, D>::RB + (tr_chunk<T, D>(r, ch) << 4)) : row_off<T, D>(r, ch);
}

template <typename T, int D, bool TR, int NTH = V2_THREADS>
__device__ __forceinline__ void stage_all(char* lds, const T* __restrict__ base, int64_t st, int64_t nrows,
                                          int nrows_pad, int tid, int dreal) {
  constexpr int NCH = AT<T, D>::NCH, EPC = AT<T, D>::EPC;
  const int total = nrows_pad * NCH;
  for (int c0 = tid; c0 < total; c0 += NTH * STAGE_BATCH) {
    uint4 v[STAGE_BATCH];
#pragma unroll
    for (int j = 0; j < STAGE_BATCH; ++j) {
      const int c = c0 + j * NTH, r = c / NCH, ch = c % NCH;
      v[j] = make_uint4(0, 0, 0, 0);
      if (c < total && r < nrows && ch * EPC < dreal) v[j] = *reinterpret_cast<const uint4*>(base + (int64_t)r * st + ch * EPC);
    }
#pragma unroll
    for (int j = 0; j < STAGE_BATCH; ++j) {
      const int c = c0 + j * NTH;
      if (c < total) *reinterpret_cast<uint4*>(lds + stage_off<T, D, TR>(c / NCH, c % NCH)) = v[j];
    }
  }
}

// two head slices of the same row count (K and V, Q and dO, or one tensor into both layouts),
// every load of a batch of both issued before its writes
template <typename T, int D, bool TRA, bool TRB, int NTH = V2_THREADS>
__device__ __forceinline__ void stage_two(char* lds_a, const T* __restrict__ base_a, int64_t st_a, char* lds_b,
                                          const T* __restrict__ base_b, int64_t st_b, int64_t nrows, int nrows_pad,
                                          int tid, int dreal) {
  constexpr int NCH = AT<T, D>::NCH, EPC = AT<T, D>::EPC;
  const int total = nrows_pad * NCH;
  for (int c0 = tid; c0 < total; c0 += NTH * STAGE_BATCH) {
    uint4 va[STAGE_BATCH], vb[STAGE_BATCH];
#pragma unroll
    for (int j = 0; j < STAGE_BATCH; ++j) {
      const int c = c0 + j * NTH, r = c / NCH, ch = c % NCH;
      va[j] = vb[j] = make_uint4(0, 0, 0, 0);
      if (c < total && r < nrows && ch * EPC < dreal) {
        va[j] = *reinterpret_cast<const uint4*>(base_a + (int64_t)r * st_a + ch * EPC);
        vb[j] = *reinterpret_cast<const uint4*>(base_b + (int64_t)r * st_b + ch * EPC);
      }
    }
#pragma unroll
    for (int j = 0; j < STAGE_BATCH; ++j) {
      const int c = c0 + j * NTH, r = c / NCH, ch = c % NCH;
      if (c < total) {
        *reinterpret_cast<uint4*>(lds_a + stage_off<T, D, TRA>(r, ch)) = va[j];
        *reinterpret_cast<uint4*>(lds_b + stage_off<T, D, TRB>(r, ch)) = vb[j];
      }
    }
  }
}

// K rows staged as k / max(|k|, 1e-12) (Swinv2 cosine attention): the NCH chunks of a row belong to
// NCH consecutive lanes, so the row's sum of squares is a butterfly over those lanes
template <int D, int NTH>
__device__ __forceinline__ void stage_rows_cos(char* lds, const bf16* __restrict__ base, int64_t st, int64_t nrows,
                                               int nrows_pad, int tid, int dreal) {
  constexpr int NCH = AT<bf16, D>::NCH, EPC = AT<bf16, D>::EPC;
  for (int c = tid; c < nrows_pad * NCH; c += NTH) {
    const int r = c / NCH, ch = c % NCH;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nrows && ch * EPC < dreal) v = *reinterpret_cast<const uint4*>(base + (int64_t)r * st + ch * EPC);
    const bf16x8 x = __builtin_bit_cast(bf16x8, v);
    float f[EPC], ss = 0.f;
#pragma unroll
    for (int e = 0; e < EPC; ++e) { f[e] = (float)x[e]; ss = fmaf(f[e], f[e], ss); }
#pragma unroll
    for (int o = 1; o < NCH; o <<= 1) ss += __shfl_xor(ss, o, 64);
    const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
    bf16x8 y;
#pragma unroll
    for (int e = 0; e < EPC; ++e) y[e] = (bf16)(f[e] * inv);
    *reinterpret_cast<uint4*>(lds + row_off<bf16, D>(r, ch)) = __builtin_bit_cast(uint4, y);
  }
}

// q fragments (load_row_regs layout: a row's chunks sit in lanes li, li+16, li+32, li+48) scaled to
// q / max(|q|, 1e-12) * mult, rounded as the separate normalisation pass would
template <int D>
__device__ __forceinline__ void cos_norm_q(uint4* f, float mult) {
  constexpr int KCH = AT<bf16, D>::KCH;
  float ss = 0.f;
  float v[KCH][8];
#pragma unroll
  for (int kc = 0; kc < KCH; ++kc) {
    const bf16x8 x = __builtin_bit_cast(bf16x8, f[kc]);
#pragma unroll
    for (int e = 0; e < 8; ++e) { v[kc][e] = (float)x[e]; ss = fmaf(v[kc][e], v[kc][e], ss); }
  }
  ss += __shfl_xor(ss, 16, 64);
  ss += __shfl_xor(ss, 32, 64);
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
  for (int kc = 0; kc < KCH; ++kc) {
    bf16x8 y;
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = (bf16)((v[kc][e] * inv) * mult);
    f[kc] = __builtin_bit_cast(uint4, y);
  }
}

constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;

// max / sum over the four lanes li, li+16, li+32, li+48 (the lane groups of one S^T column) by two
// VALU half-swaps (v_permlane16/32_swap) instead of LDS permutes: the same pairs as __shfl_xor 16
// then 32, so a sum rounds identically
__device__ __forceinline__ float rows4_max(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rows4_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// v2 kernel modes, chosen on the host: 0 = any (dropout, key bias, keep-bitmask, tested at run
// time), 1 = plain (no dropout, no key bias: ViT, the fusion head at eval), 2 = hashed dropout with
// a key bias and no bitmask (BERT training). The fixed modes take the per-subtile branches out of
// the softmax loops, and mode 1 folds the scale into the exponent (exp2(s * c2 - m) as one fma).
// bf16 forward only: the running max is raised only when some lane's chunk max passes it by more
// than 8 (log2 units), so P = exp2(t - m) stays <= 256 and the O / l rescale (and its lane
// broadcasts) is skipped for most chunks; O and l are scaled by the same stale max, so O / l is
// unchanged up to rounding
constexpr float V2_RESCALE_TH = 8.f;

// per-key additive bias in log2 units for the head's batch row: log2e * key_bias (clamped so a
// fully masked row stays finite, as HF's finfo.min mask does) for k < Lk, -inf for padded keys
template <int NTH>
__device__ __forceinline__ void stage_kbias(float* dst, const AttnP& p, int64_t b, int npad, int tid) {
  for (int i = tid; i < npad; i += NTH)
    dst[i] = i < p.Lk ? (p.key_bias ? fmaxf(p.key_bias[b * p.Lk + i] * LOG2E, -1e30f) : 0.f) : -INFINITY;
}

// bf16 without the relative bias: at most 128 VGPRs (4 waves per SIMD) so that two 8-wave
// workgroups share a CU — the bf16 K/V images allow it, and one VGPR over halves the occupancy
// (ViT fwd +45 %); the REL instantiation needs ~148 and would spill under that bound
template <typename T, int D, int HPB, bool REL, int MODE>
__global__ void __launch_bounds__(V2_THREADS, sizeof(T) == 2 && !REL ? 4 : 1) attn_fwd_v2_kernel(AttnP p) {
  static_assert(MODE == 0 || (HPB == 1 && !REL), "fixed modes: one head per workgroup, no relative bias");
  constexpr bool LAZY = sizeof(T) == 2;
  // K/V of the head resident in LDS; each wave sweeps 16-query blocks with an online softmax (exp2
  // domain) over 64-key chunks (the last one holds only the padded key count's subtiles); key
  // mask/padding come from a per-key bias vector in LDS.
  // HPB > 1 (short windows: Lq <= 64 / 32, Lk <= 64, e.g. Swinv2's 8x8 windows): the 8 waves split
  // into HPB groups, each owning one (b, h) with its own LDS images, so no wave idles on a head
  // that has fewer 16-query blocks than the workgroup has waves.
  using C = AT<T, D>;
  constexpr int KC = v2_kc<T>(), SUBS = KC / 16;
  constexpr int WPH = (V2_THREADS / 64) / HPB;  // waves per head
  constexpr int TPH = V2_THREADS / HPB;         // threads per head
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = wave_all / WPH, wave = wave_all % WPH, htid = tid % TPH;
  const int64_t nbh = p.B * p.H, bh_raw = (int64_t)blockIdx.x * HPB + sub;
  const bool active = bh_raw < nbh;
  const int64_t bh = active ? bh_raw : nbh - 1, b = bh / p.H, h = bh % p.H;
  const int lk_pad = v2_pad(p.Lk, KC);
  char* hbase = smem + sub * (2 * lk_pad * C::RB + lk_pad * 4);
  char* k_img = hbase;
  char* v_img = hbase + lk_pad * C::RB;
  float* kbias = reinterpret_cast<float*>(hbase + 2 * lk_pad * C::RB);
  const T* qb = reinterpret_cast<const T*>(p.q) + b * p.q_sb + h * p.D;
  const T* kb_g = reinterpret_cast<const T*>(p.k) + b * p.k_sb + h * p.D;
  const int nqb = (int)((p.Lq + 15) / 16);
  uint4 qn[C::KCH];  // next query block's fragments, prefetched one block ahead (the first under the staging)
  load_row_regs<T, D>(qn, qb, p.q_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
  bool cosine = false;
  if constexpr (sizeof(T) == 2) {
    cosine = REL && p.cos_ls != nullptr;
    if (cosine) stage_rows_cos<D, TPH>(k_img, kb_g, p.k_st, p.Lk, lk_pad, htid, p.D);
  }
  const T* vb_g = reinterpret_cast<const T*>(p.v) + b * p.v_sb + h * p.D;
  if (!cosine)
    stage_two<T, D, false, true, TPH>(k_img, kb_g, p.k_st, v_img, vb_g, p.v_st, p.Lk, lk_pad, htid, p.D);
  else
    stage_all<T, D, true, TPH>(v_img, vb_g, p.v_st, p.Lk, lk_pad, htid, p.D);
  stage_kbias<TPH>(kbias, p, b, lk_pad, htid);
  __syncthreads();
  if (!active) return;
  const uint64_t seed = p.p > 0.f ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);
  const bool drop = MODE == 0 ? p.p > 0.f : MODE == 2;
  const float c2 = p.scale * LOG2E;
  const float qmult = cosine ? expf(fminf(p.cos_ls[h], p.cos_max_log)) : 1.f;
  const bool rel4 = p.rel_bias && (p.Lk & 3) == 0 && (reinterpret_cast<uintptr_t>(p.rel_bias) & 15) == 0 &&
                    (p.rb_sb & 3) == 0;
  T* ob = reinterpret_cast<T*>(p.o) + b * p.o_sb + h * p.D;
  for (int qbk = wave; qbk < nqb; qbk += WPH) {
    const int64_t q0 = (int64_t)qbk * 16, myq = q0 + li;
    uint4 qf[C::KCH];
#pragma unroll
    for (int kc = 0; kc < C::KCH; ++kc) qf[kc] = qn[kc];
    load_row_regs<T, D>(qn, qb, p.q_st, q0 + WPH * 16 + li, p.Lq, lane, p.D);
    if constexpr (sizeof(T) == 2) {
      if (cosine) cos_norm_q<D>(qf, qmult);
    }
    const uint64_t hrow = (uint64_t)(bh * p.Lq + myq) * (uint64_t)p.kp;  // pair-index base of this query row
    const uint32_t rowc1 = ((uint32_t)hrow + (uint32_t)(2 * g)) * HASH_C1;
    const float* relrow = REL ? p.rel_bias + rb_off(p, b) + (h * p.Lq + (myq < p.Lq ? myq : 0)) * p.Lk : nullptr;
    float m = -INFINITY, lsum = 0.f;
    f32x4 o[C::DT];
#pragma unroll
    for (int d = 0; d < C::DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one 64-key chunk with NS 16-key subtiles present (NS < 4 only for the last, padded chunk;
    // NS = 0: that count at run time, `ns_rt`); a compile-time NS keeps every per-subtile branch
    // out of the full chunks. FOLD (mode 1, a full chunk of real keys): the chunk max is taken on
    // the raw scores and the scale goes into the exponent's fma
    auto chunk = [&](int k0, auto nsc, int ns_rt, auto foldc) {
      constexpr int NS = decltype(nsc)::value;
      constexpr bool FOLD = decltype(foldc)::value;
      const int nsub = NS ? NS : ns_rt;
      const char* kc_img = k_img + k0 * C::RB;
      const char* vc_img = v_img + k0 * C::RB;
      f32x4 s[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) s[ks] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (sizeof(T) == 4 && nsub == 4) {  // fp32: four interleaved S^T chains, K read one k-chunk ahead
        uint4 fa[4], fb[4], fn[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) { fa[ks] = row_frag<T, D>(kc_img, ks, 0, lane); fb[ks] = qf[0]; }
#pragma unroll
        for (int kc = 0; kc < C::KCH; ++kc) {
          if (kc + 1 < C::KCH) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) fn[ks] = row_frag<T, D>(kc_img, ks, kc + 1, lane);
          }
          Mma<T>::template runN<4>(s, fa, fb);
          if (kc + 1 < C::KCH) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) { fa[ks] = fn[ks]; fb[ks] = qf[kc + 1]; }
          }
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < (NS ? NS : 4); ++ks) {
          if (ks < nsub) {
#pragma unroll
            for (int kc = 0; kc < C::KCH; ++kc) Mma<T>::run(s[ks], row_frag<T, D>(kc_img, ks, kc, lane), qf[kc]);
          }
        }
      }
      float mx = -INFINITY;
      if constexpr (FOLD) {  // c2 > 0: max(s) * c2 == max(s * c2) (rounding is monotone)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[ks][r]);
        mx *= c2;
      } else {
#pragma unroll
      for (int ks = 0; ks < (NS ? NS : 4); ++ks) {
        if (ks >= nsub) continue;
        const float4 kb4 = *reinterpret_cast<const float4*>(kbias + k0 + ks * 16 + 4 * g);
        const float kb[4] = {kb4.x, kb4.y, kb4.z, kb4.w};
        float rb[4] = {0.f, 0.f, 0.f, 0.f};
        const int kk = k0 + ks * 16 + 4 * g;
        if (REL) {  // the 4 keys of a lane are contiguous: one 16-B load per subtile when aligned
          if (rel4) {
            if (kk < p.Lk) {
              const float4 v = *reinterpret_cast<const float4*>(relrow + kk);
              rb[0] = v.x; rb[1] = v.y; rb[2] = v.z; rb[3] = v.w;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) rb[r] = kk + r < p.Lk ? relrow[kk + r] : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t = fmaf(s[ks][r], c2, kb[r]);
          if (REL && kk + r < p.Lk) t = fmaf(rb[r], LOG2E, t);
          s[ks][r] = t;
          mx = fmaxf(mx, t);
        }
      }
      }
      mx = rows4_max(mx);
      // (LAZY: a wave-uniform decision; otherwise every chunk rescales)
      const bool grow = !LAZY || __ballot(mx > m + V2_RESCALE_TH) != 0ull;
      float mnew = m, alpha = 1.f;
      if (grow) {
        mnew = fmaxf(m, mx);
        alpha = __builtin_amdgcn_exp2f(m - mnew);
      }
      float rs = 0.f;
#pragma unroll
      for (int ks = 0; ks < (NS ? NS : 4); ++ks) {
        if (ks >= nsub) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = FOLD ? __builtin_amdgcn_exp2f(fmaf(s[ks][r], c2, -mnew))
                               : __builtin_amdgcn_exp2f(s[ks][r] - mnew);
          rs += e;
          s[ks][r] = e;
        }
        if (drop) {  // one uniform branch per subtile (none in the fixed modes)
          float z[4];
          if (p.idx32) {
            const uint32_t c = rowc1 + (uint32_t)((k0 + ks * 16) >> 1) * HASH_C1;
            keep4_pairs(hash_c1(hkey, c), hash_c1(hkey, c + HASH_C1), p, z);
          } else {
            const uint64_t pi = hrow + (uint64_t)((k0 + ks * 16 + 4 * g) >> 1);
            keep4_pairs(mmfd_hash_k(hkey, pi), mmfd_hash_k(hkey, pi + 1), p, z);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) s[ks][r] *= z[r];
        }
      }
      if (MODE == 0 && p.p > 0.f && p.dm) {
        // the keep-bitmask for the backward, read back from P: a dropped element is 0, a kept one
        // e * keep_scale > 0 unless exp2 underflowed — and then the backward's P of it is 0 too,
        // so recording it as dropped changes no gradient (one register, no hash state kept live)
        uint32_t kbits = 0;
#pragma unroll
        for (int ks = 0; ks < (NS ? NS : 4); ++ks) {
          if (ks >= nsub) continue;
#pragma unroll
          for (int r = 0; r < 4; ++r) kbits |= (uint32_t)(s[ks][r] != 0.f) << (ks * 4 + r);
        }
        dm_write64(p, bh, myq, k0, g, kbits);
      }
      lsum = lsum * alpha + rs;  // per-lane partial over this lane's keys; reduced at the end
      m = mnew;
      if (grow) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
          for (int d = 0; d < C::DT; ++d) o[d][r] *= ar;
        }
      }
#pragma unroll
      for (int c = 0; c < (NS ? NS : 4) / SUBS; ++c) {
        if (c * SUBS >= nsub) continue;
        uint4 fa[C::DT], fb[C::DT];
        const uint4 a = pack_acc<T>(s, c);
#pragma unroll
        for (int d = 0; d < C::DT; ++d) { fa[d] = a; fb[d] = tr_frag<T, D>(vc_img, c, d, lane); }
        Mma<T>::template runN<C::DT>(o, fa, fb);
      }
    };
    if constexpr (SUBS == 1) {
      // fp32 (MFMA-bound): one instance with the subtile count at run time — two compile-time
      // instances (full chunk + tail) raised it from 154 to 255 VGPRs and cost 7 % at L = 128
      for (int k0 = 0; k0 < lk_pad; k0 += 64)
        chunk(k0, std::integral_constant<int, 0>{}, min(4, (lk_pad - k0) >> 4), std::false_type{});
    } else {
      // bf16 (VALU-bound): the full chunks free of per-subtile branches (128 VGPRs: two workgroups
      // per CU), the 32-key padded tail as its own instance; mode 1 folds the full chunks of real keys
      int k0 = 0;
      if constexpr (MODE == 1) {
        for (; k0 + 64 <= p.Lk; k0 += 64) chunk(k0, std::integral_constant<int, 4>{}, 4, std::true_type{});
      }
      for (; k0 + 64 <= lk_pad; k0 += 64) chunk(k0, std::integral_constant<int, 4>{}, 4, std::false_type{});
      if (k0 < lk_pad) chunk(k0, std::integral_constant<int, 2>{}, 2, std::false_type{});
    }
    lsum = rows4_sum(lsum);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float lr = __shfl(lsum, 4 * g + r, 64);
      const int64_t q = q0 + 4 * g + r;
      const float inv = 1.0f / lr;
      if (q < p.Lq) {
#pragma unroll
        for (int d = 0; d < C::DT; ++d)
          if (d * 16 + li < p.D) {
            const float val = o[d][r] * inv;
            ob[q * p.o_st + d * 16 + li] = from_f32<T>(val);
            if constexpr (std::is_same<T, float>::value) {
              if (p.pl) plane_put(p, reinterpret_cast<const float*>(ob) + q * p.o_st + d * 16 + li, val);
            }
          }
      }
    }
    if (g == 0 && myq < p.Lq) p.lse[bh * p.Lq + myq] = (m + log2f(lsum)) * LN2;
  }
}

template <typename T, int D, int NTH, bool REL, int MODE>
__global__ void __launch_bounds__(NTH) attn_dkdv_v2_kernel(AttnP p) {
  static_assert(MODE == 0 || !REL, "fixed modes: no relative bias");
  // Q/dO of the head resident in LDS (plus lse, delta in log2 units); each wave owns 16 keys.
  // REL: the additive [H][Lq][Lk] bias (MPNet / DeBERTa) — its loads and batch-modulus address
  // math stay out of the bias-free instantiation (BERT, ViT, fusion head)
  using C = AT<T, D>;
  constexpr int KC = v2_kc<T>(), SUBS = KC / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const int lq_pad = v2_pad(p.Lq, KC);
  const int img = lq_pad * C::RB;
  constexpr bool DUAL = V2<T, D>::DUAL;
  char* q_row = smem;
  char* do_row = smem + img;
  char* q_tr = DUAL ? q_row : smem + 2 * img;
  char* do_tr = DUAL ? do_row : smem + 3 * img;
  float* s_lse = reinterpret_cast<float*>(smem + (DUAL ? 2 : 4) * img);
  float* s_delta = s_lse + V2_LMAX;
  float* kbias = s_delta + V2_LMAX;
  uint32_t* s_dm = reinterpret_cast<uint32_t*>(kbias + V2_LMAX);  // dm_lds: the head's keep-bitmask rows
  if (MODE == 0 && p.dm_lds) {
    const uint32_t* src = dm_row(p, bh, 0);
    const int nw = (int)p.Lq * p.dmw;
    for (int i = tid; i < lq_pad * p.dmw; i += NTH) s_dm[i] = i < nw ? src[i] : 0u;
  }
  const T* qb = reinterpret_cast<const T*>(p.q) + b * p.q_sb + h * p.D;
  const T* dob = reinterpret_cast<const T*>(p.dout) + b * p.do_sb + h * p.D;
  const T* kb = reinterpret_cast<const T*>(p.k) + b * p.k_sb + h * p.D;
  const T* vb = reinterpret_cast<const T*>(p.v) + b * p.v_sb + h * p.D;
  // PF (bf16 fixed modes, where the registers allow it): the wave's next key block loaded one block
  // ahead, the first under the staging
  constexpr bool PF = sizeof(T) == 2 && !REL && MODE != 0;
  uint4 kn[C::KCH], vn[C::KCH];
  if constexpr (PF) {
    load_row_regs<T, D>(kn, kb, p.k_st, (int64_t)wave * 16 + li, p.Lk, lane, p.D);
    load_row_regs<T, D>(vn, vb, p.v_st, (int64_t)wave * 16 + li, p.Lk, lane, p.D);
  }
  stage_two<T, D, false, false, NTH>(q_row, qb, p.q_st, do_row, dob, p.do_st, p.Lq, lq_pad, tid, p.D);
  if (!DUAL) stage_two<T, D, true, true, NTH>(q_tr, qb, p.q_st, do_tr, dob, p.do_st, p.Lq, lq_pad, tid, p.D);
  for (int i = tid; i < lq_pad; i += NTH) {
    s_lse[i] = i < p.Lq ? p.lse[bh * p.Lq + i] * LOG2E : INFINITY;
    s_delta[i] = i < p.Lq ? p.delta[bh * p.Lq + i] : 0.f;
  }
  stage_kbias<NTH>(kbias, p, b, (int)((p.Lk + 15) & ~15), tid);
  __syncthreads();
  T* dkb = reinterpret_cast<T*>(p.dk) + b * p.dk_sb + h * p.D;
  T* dvb = reinterpret_cast<T*>(p.dv) + b * p.dv_sb + h * p.D;
  const uint64_t seed = p.p > 0.f ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);
  const bool drop = MODE == 0 ? p.p > 0.f : MODE == 2;
  const float c2 = p.scale * LOG2E;
  const int nkb = (int)((p.Lk + 15) / 16);
  const int nqc = lq_pad / KC;  // query chunks of one MFMA k-chunk
  for (int kbk = wave; kbk < nkb; kbk += NTH / 64) {
    const int64_t k0 = (int64_t)kbk * 16, mykey = k0 + li;
    uint4 kf[C::KCH], vf[C::KCH];
    if constexpr (PF) {
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) { kf[kc] = kn[kc]; vf[kc] = vn[kc]; }
      load_row_regs<T, D>(kn, kb, p.k_st, k0 + NTH / 64 * 16 + li, p.Lk, lane, p.D);
      load_row_regs<T, D>(vn, vb, p.v_st, k0 + NTH / 64 * 16 + li, p.Lk, lane, p.D);
    } else {
      load_row_regs<T, D>(kf, kb, p.k_st, mykey, p.Lk, lane, p.D);
      load_row_regs<T, D>(vf, vb, p.v_st, mykey, p.Lk, lane, p.D);
    }
    // -inf for padded keys -> P = 0 (mode 1: their dK / dV rows are computed but never stored)
    const float kb2 = MODE == 1 ? 0.f : kbias[mykey];
    const uint64_t hcol = (uint64_t)(bh * p.Lq) * (uint64_t)p.kp + (uint64_t)(mykey >> 1);  // pair index, query 0
    const int kodd = (int)(mykey & 1);
    const float* relcol = REL ? p.rel_bias + rb_off(p, b) + h * p.Lq * p.Lk + (mykey < p.Lk ? mykey : 0) : nullptr;
    f32x4 dkv[2 * C::DT];  // dV (even) and dK (odd) of each 16-wide D subtile
#pragma unroll
    for (int i = 0; i < 2 * C::DT; ++i) dkv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Q / dO row fragments of the first query chunk; each iteration prefetches the next chunk's
    uint4 qa[SUBS * C::KCH], da[SUBS * C::KCH];
#pragma unroll
    for (int i = 0; i < SUBS * C::KCH; ++i) {
      qa[i] = row_frag<T, D>(q_row, i / C::KCH, i % C::KCH, lane);
      da[i] = row_frag<T, D>(do_row, i / C::KCH, i % C::KCH, lane);
    }
    for (int qc = 0; qc < nqc; ++qc) {
      // transposed dO / Q fragments of this chunk (B operands of dV / dK), read ahead of the softmax
      uint4 tb[2 * C::DT];
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        tb[2 * d] = tr_frag<T, D>(do_tr, qc, d, lane);
        tb[2 * d + 1] = tr_frag<T, D>(q_tr, qc, d, lane);
      }
      f32x4 sd[2 * SUBS];  // S (even) and dP (odd) of each 16-query subtile, interleaved chains
#pragma unroll
      for (int i = 0; i < 2 * SUBS; ++i) sd[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) {
        uint4 fa[2 * SUBS], fb[2 * SUBS];
#pragma unroll
        for (int h2 = 0; h2 < SUBS; ++h2) {
          fa[2 * h2] = qa[h2 * C::KCH + kc]; fb[2 * h2] = kf[kc];
          fa[2 * h2 + 1] = da[h2 * C::KCH + kc]; fb[2 * h2 + 1] = vf[kc];
        }
        Mma<T>::template runN<2 * SUBS>(sd, fa, fb);
      }
      if (qc + 1 < nqc) {
#pragma unroll
        for (int i = 0; i < SUBS * C::KCH; ++i) {
          qa[i] = row_frag<T, D>(q_row, SUBS * (qc + 1) + i / C::KCH, i % C::KCH, lane);
          da[i] = row_frag<T, D>(do_row, SUBS * (qc + 1) + i / C::KCH, i % C::KCH, lane);
        }
      }
      f32x4 pd[SUBS], ds[SUBS];
#pragma unroll
      for (int h2 = 0; h2 < SUBS; ++h2) {
        const int qs = SUBS * qc + h2;
        const f32x4 sv = sd[2 * h2], dp = sd[2 * h2 + 1];
        const float4 l4 = *reinterpret_cast<const float4*>(s_lse + qs * 16 + 4 * g);
        const float4 d4 = *reinterpret_cast<const float4*>(s_delta + qs * 16 + 4 * g);
        const float lq2[4] = {l4.x, l4.y, l4.z, l4.w}, dl[4] = {d4.x, d4.y, d4.z, d4.w};
        float z[4] = {1.f, 1.f, 1.f, 1.f};
        if (drop) {  // one uniform branch per subtile; the element index advances by Lk per query
          if (MODE == 0 && p.dm_lds) {  // bit mykey of the query rows' words (LDS broadcast reads)
            const uint32_t* col = s_dm + (mykey >> 5);
            const int sh = (int)(mykey & 31);
#pragma unroll
            for (int r = 0; r < 4; ++r) z[r] = ((col[(qs * 16 + 4 * g + r) * p.dmw] >> sh) & 1u) ? p.keep_scale : 0.f;
          } else if (p.idx32) {
            const uint32_t kpc1 = (uint32_t)p.kp * HASH_C1;
            const uint32_t c = ((uint32_t)hcol + (uint32_t)(qs * 16 + 4 * g + 2 * kodd) * (uint32_t)p.kp) * HASH_C1;
            keep4_col(hash_c1(hkey, c), hash_c1(hkey, c + kpc1), kodd, p, z);
          } else {
            const uint64_t idx = hcol + (uint64_t)(qs * 16 + 4 * g + 2 * kodd) * (uint64_t)p.kp;
            keep4_col(mmfd_hash_k(hkey, idx), mmfd_hash_k(hkey, idx + (uint64_t)p.kp), kodd, p, z);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lq = qs * 16 + 4 * g + r;
          float pr;
          if constexpr (MODE == 1) {  // (lse = +inf on padded queries: P = 0)
            pr = __builtin_amdgcn_exp2f(fmaf(sv[r], c2, -lq2[r]));
          } else {
            float t = fmaf(sv[r], c2, kb2);
            if (REL && lq < p.Lq && mykey < p.Lk) t = fmaf(relcol[(int64_t)lq * p.Lk], LOG2E, t);
            pr = __builtin_amdgcn_exp2f(t - lq2[r]);
          }
          pd[h2][r] = pr * z[r];
          ds[h2][r] = pr * (dp[r] * z[r] - dl[r]);
        }
      }
      const uint4 ap = pack_acc<T>(pd, 0);
      const uint4 as = pack_acc<T>(ds, 0);
      uint4 fa[2 * C::DT];
#pragma unroll
      for (int d = 0; d < C::DT; ++d) { fa[2 * d] = ap; fa[2 * d + 1] = as; }
      Mma<T>::template runN<2 * C::DT>(dkv, fa, tb);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t key = k0 + 4 * g + r;
      if (key < p.Lk) {
#pragma unroll
        for (int d = 0; d < C::DT; ++d) {
          if (d * 16 + li >= p.D) continue;
          T* pk = dkb + key * p.dk_st + d * 16 + li;
          T* pv = dvb + key * p.dv_st + d * 16 + li;
          float vk = dkv[2 * d + 1][r] * p.scale, vv = dkv[2 * d][r];
          if (p.acc_dkv) { vk += to_f32(*pk); vv += to_f32(*pv); }
          if constexpr (std::is_same<T, float>::value) {
            if (p.pl) {
              plane_put(p, pk, vk);
              plane_put(p, pv, vv);
              if (p.pl_only) continue;
            }
          }
          *pk = from_f32<T>(vk);
          *pv = from_f32<T>(vv);
        }
      }
    }
  }
}

template <typename T, int D, bool REL, int MODE>
__global__ void __launch_bounds__(V2_THREADS, sizeof(T) == 2 ? 4 : 1) attn_dq_v2_kernel(AttnP p) {
  static_assert(MODE == 0 || !REL, "fixed modes: no relative bias");
  // K/V of the head resident in LDS; each wave owns 16 queries: dQ = dS K (REL as in dK/dV)
  using C = AT<T, D>;
  constexpr int KC = v2_kc<T>(), SUBS = KC / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const int lk_pad = v2_pad(p.Lk, KC);
  const int img = lk_pad * C::RB;
  constexpr bool DUAL = V2<T, D>::DUAL;
  char* k_row = smem;
  char* v_row = smem + img;
  char* k_tr = DUAL ? k_row : smem + 2 * img;
  float* kbias = reinterpret_cast<float*>(smem + (DUAL ? 2 : 3) * img);
  const T* kb = reinterpret_cast<const T*>(p.k) + b * p.k_sb + h * p.D;
  const T* qb = reinterpret_cast<const T*>(p.q) + b * p.q_sb + h * p.D;
  const T* dob = reinterpret_cast<const T*>(p.dout) + b * p.do_sb + h * p.D;
  const T* obq = reinterpret_cast<const T*>(p.o) + b * p.o_sb + h * p.D;
  // PF (bf16 fixed modes, where the registers allow it): the wave's next query block's Q / dO / O
  // rows loaded one block ahead, the first under the staging
  constexpr bool PF = sizeof(T) == 2 && !REL && MODE != 0;
  uint4 qn[C::KCH], dn[C::KCH], on[C::KCH];
  if constexpr (PF) {
    load_row_regs<T, D>(qn, qb, p.q_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
    load_row_regs<T, D>(dn, dob, p.do_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
    load_row_regs<T, D>(on, obq, p.o_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
  }
  stage_two<T, D, false, false>(k_row, kb, p.k_st, v_row, reinterpret_cast<const T*>(p.v) + b * p.v_sb + h * p.D,
                                p.v_st, p.Lk, lk_pad, tid, p.D);
  if (!DUAL) stage_all<T, D, true>(k_tr, kb, p.k_st, p.Lk, lk_pad, tid, p.D);
  stage_kbias<V2_THREADS>(kbias, p, b, lk_pad, tid);
  __syncthreads();
  T* dqb = reinterpret_cast<T*>(p.dq) + b * p.dq_sb + h * p.D;
  const uint64_t seed = p.p > 0.f ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);
  const bool drop = MODE == 0 ? p.p > 0.f : MODE == 2;
  const float c2 = p.scale * LOG2E;
  const int nqb = (int)((p.Lq + 15) / 16);
  const int nkc = lk_pad / KC;
  for (int qbk = wave; qbk < nqb; qbk += V2_THREADS / 64) {
    const int64_t q0 = (int64_t)qbk * 16, myq = q0 + li;
    uint4 qf[C::KCH], dof[C::KCH], of[C::KCH];
    if constexpr (PF) {
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) { qf[kc] = qn[kc]; dof[kc] = dn[kc]; of[kc] = on[kc]; }
      if (qbk + V2_THREADS / 64 < nqb) {
        const int64_t nq = myq + V2_THREADS / 64 * 16;
        load_row_regs<T, D>(qn, qb, p.q_st, nq, p.Lq, lane, p.D);
        load_row_regs<T, D>(dn, dob, p.do_st, nq, p.Lq, lane, p.D);
        load_row_regs<T, D>(on, obq, p.o_st, nq, p.Lq, lane, p.D);
      }
    } else {
      load_row_regs<T, D>(qf, qb, p.q_st, myq, p.Lq, lane, p.D);
      load_row_regs<T, D>(dof, dob, p.do_st, myq, p.Lq, lane, p.D);
      load_row_regs<T, D>(of, obq, p.o_st, myq, p.Lq, lane, p.D);
    }
    const float lse2 = myq < p.Lq ? p.lse[bh * p.Lq + myq] * LOG2E : INFINITY;
    // delta = rowsum(dO * O) from the dO fragments in registers and the O row (this kernel runs
    // before dK/dV and writes delta for it: no separate delta pass)
    float dlt;
    {
      float ds = 0.f;
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) ds += row_chunk_dot<T>(of[kc], dof[kc]);
      ds += __shfl_xor(ds, 16, 64);
      ds += __shfl_xor(ds, 32, 64);
      dlt = myq < p.Lq ? ds : 0.f;
      if (g == 0 && myq < p.Lq) p.delta[bh * p.Lq + myq] = ds;
    }
    const uint64_t hrow = (uint64_t)(bh * p.Lq + myq) * (uint64_t)p.kp;  // pair-index base of this query row
    const float* relrow = REL ? p.rel_bias + rb_off(p, b) + (h * p.Lq + (myq < p.Lq ? myq : 0)) * p.Lk : nullptr;
    const uint32_t* dmrow = MODE == 0 && p.dm ? dm_row(p, bh, myq < p.Lq ? myq : 0) : nullptr;
    f32x4 dq[C::DT];
#pragma unroll
    for (int d = 0; d < C::DT; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fp32 (MFMA-bound, two waves per SIMD whatever the registers): K / V row fragments of the
    // next key chunk and this chunk's transposed K are read ahead; bf16 reads them where they are
    // used, which keeps the kernel at <= 128 VGPRs and two workgroups per CU (the read-ahead form
    // measured 211 -> 298 us per ViT/BERT call in bf16)
    constexpr bool PF = sizeof(T) == 4;
    uint4 ka[SUBS * C::KCH], va[SUBS * C::KCH];
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < SUBS * C::KCH; ++i) {
        ka[i] = row_frag<T, D>(k_row, i / C::KCH, i % C::KCH, lane);
        va[i] = row_frag<T, D>(v_row, i / C::KCH, i % C::KCH, lane);
      }
    }
    for (int kc2 = 0; kc2 < nkc; ++kc2) {
      // the keep word of this chunk's keys (dropout bitmask), loaded ahead of the products
      const uint32_t kw = (MODE == 0 && p.p > 0.f && p.dm) ? dmrow[(SUBS * kc2) >> 1] : 0u;
      uint4 tk[C::DT];  // transposed K fragments (B operand of dQ)
      if constexpr (PF) {
#pragma unroll
        for (int d = 0; d < C::DT; ++d) tk[d] = tr_frag<T, D>(k_tr, kc2, d, lane);
      }
      f32x4 sd[2 * SUBS];
#pragma unroll
      for (int i = 0; i < 2 * SUBS; ++i) sd[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < C::KCH; ++kc) {
        uint4 fa[2 * SUBS], fb[2 * SUBS];
#pragma unroll
        for (int h2 = 0; h2 < SUBS; ++h2) {
          if constexpr (PF) {
            fa[2 * h2] = ka[h2 * C::KCH + kc];
            fa[2 * h2 + 1] = va[h2 * C::KCH + kc];
          } else {
            fa[2 * h2] = row_frag<T, D>(k_row, SUBS * kc2 + h2, kc, lane);
            fa[2 * h2 + 1] = row_frag<T, D>(v_row, SUBS * kc2 + h2, kc, lane);
          }
          fb[2 * h2] = qf[kc];
          fb[2 * h2 + 1] = dof[kc];
        }
        Mma<T>::template runN<2 * SUBS>(sd, fa, fb);
      }
      if (PF && kc2 + 1 < nkc) {
#pragma unroll
        for (int i = 0; i < SUBS * C::KCH; ++i) {
          ka[i] = row_frag<T, D>(k_row, SUBS * (kc2 + 1) + i / C::KCH, i % C::KCH, lane);
          va[i] = row_frag<T, D>(v_row, SUBS * (kc2 + 1) + i / C::KCH, i % C::KCH, lane);
        }
      }
      f32x4 ds[SUBS];
#pragma unroll
      for (int h2 = 0; h2 < SUBS; ++h2) {
        const int ks = SUBS * kc2 + h2;
        const f32x4 sv = sd[2 * h2], dp = sd[2 * h2 + 1];
        float z[4] = {1.f, 1.f, 1.f, 1.f};
        if (drop) {  // one uniform branch per subtile
          if (MODE == 0 && p.dm) {
#pragma unroll
            for (int r = 0; r < 4; ++r) z[r] = ((kw >> ((ks & 1) * 16 + 4 * g + r)) & 1u) ? p.keep_scale : 0.f;
          } else if (p.idx32) {
            const uint32_t c = ((uint32_t)hrow + (uint32_t)(ks * 8 + 2 * g)) * HASH_C1;
            keep4_pairs(hash_c1(hkey, c), hash_c1(hkey, c + HASH_C1), p, z);
          } else {
            const uint64_t pi = hrow + (uint64_t)(ks * 8 + 2 * g);
            keep4_pairs(mmfd_hash_k(hkey, pi), mmfd_hash_k(hkey, pi + 1), p, z);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = ks * 16 + 4 * g + r;
          float pr;
          if constexpr (MODE == 1) {
            // padded keys: their K rows are zero, so their dS adds nothing to dQ = dS K
            pr = __builtin_amdgcn_exp2f(fmaf(sv[r], c2, -lse2));
          } else {
            float t = fmaf(sv[r], c2, kbias[ks * 16 + 4 * g + r]);
            if (REL && key < p.Lk) t = fmaf(relrow[key], LOG2E, t);
            pr = __builtin_amdgcn_exp2f(t - lse2);
          }
          ds[h2][r] = pr * (dp[r] * z[r] - dlt);
        }
      }
      const uint4 as = pack_acc<T>(ds, 0);
      uint4 fa[C::DT];
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        fa[d] = as;
        if constexpr (!PF) tk[d] = tr_frag<T, D>(k_tr, kc2, d, lane);
      }
      Mma<T>::template runN<C::DT>(dq, fa, tk);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t q = q0 + 4 * g + r;
      if (q < p.Lq) {
#pragma unroll
        for (int d = 0; d < C::DT; ++d) {
          if (d * 16 + li >= p.D) continue;
          T* pq = dqb + q * p.dq_st + d * 16 + li;
          float vq = dq[d][r] * p.scale;
          if (p.acc_dq) vq += to_f32(*pq);
          if constexpr (std::is_same<T, float>::value) {
            if (p.pl) {
              plane_put(p, pq, vq);
              if (p.pl_only) continue;
            }
          }
          *pq = from_f32<T>(vq);
        }
      }
    }
  }
}

// --------------------------------------------------------------------------------------------
// fp32 attention on split bf16 operands (the fp32 step's attention; mmfd_set_fp32_attn_mode)
// --------------------------------------------------------------------------------------------
// gfx950 has no xf32 MFMA and its fp32 MFMA runs at 1/16 of the bf16 rate. As in gemm256_x6f,
// every fp32 operand is split into three bf16 planes x = hi + mid + lo (the split3 rule; 24
// significand bits, all of x) and each product accumulates the six plane products
//   mid*mid, hi*lo, lo*hi, hi*mid, mid*hi, hi*hi
// on v_mfma_f32_16x16x32_bf16 into fp32 (bf16 x bf16 products are exact; the dropped mid*lo,
// lo*mid, lo*lo are below 2^-24 relative): 6 x 16 cycles per 16x16x32 fp32 product against
// 8 x 32 for the fp32 MFMA. Operands resident in LDS (K/V, or Q/dO) are split while they are
// staged (one fp32 read from HBM, three bf16 plane images of 128-B rows, the bf16 D = 64 swizzle
// that serves both the row and the ds_read_b64_tr_b16 transposed reads); the per-wave register
// operands (the wave's own 16 queries or keys) are split once per block, and the softmax-side
// operands (P, dS) are split in registers right before their products.
//
// Geometry (D = 64 images; any D <= 64 with D % 8 == 0, the zero columns skipped by uniform
// branches): one 8-wave workgroup per (b, h) as the v2 kernels. Two tensors x three planes x
// L16 rows x 128 B must fit the 160-KB LDS: L16 = L padded to 16 rows <= 208 (BERT L = 128, ViT
// L = 197). Rows are padded to 16, not to the 32-row k-chunk: the last chunk of a 16-row remainder
// runs its h = 1 half on a repeat of its h = 0 rows (h1off = 0) against operands that are zero.
void set_lds_attr(const void* fn, int bytes) {
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// Diagnostic build only (-DMMFD_X6A_STAMPS, tools/x6a_stamps.py): s_memtime per wave at the phase
// boundaries of the split-operand forward into a buffer no computation reads.
#ifdef MMFD_X6A_STAMPS
__device__ uint64_t x6a_stamps[8192 * 8 * 16];
#define X6A_STAMP(k)                                                                               \
  do {                                                                                             \
    const uint64_t t__ = __builtin_amdgcn_s_memtime();                                             \
    if (lane == 0 && blockIdx.x < 8192) x6a_stamps[((int64_t)blockIdx.x * 8 + wave) * 16 + (k)] = t__; \
  } while (0)
#else
#define X6A_STAMP(k) do { } while (0)
#endif
constexpr int X6A_LMAX = 208;
constexpr int X6A_RB = 128;  // bytes per plane row (64 bf16)
constexpr int X6A_LDS = 6 * X6A_LMAX * X6A_RB + 3 * X6A_LMAX * 4;

// A/B switch: MMFD_ATTN_V2_GENERIC=1 (or mmfd_debug_set_attn_v2_generic) runs every v2 call on mode 0
int g_v2_generic = [] {
  const char* v = getenv("MMFD_ATTN_V2_GENERIC");
  return v && atoi(v) != 0 ? 1 : 0;
}();

// A/B switch: MMFD_ATTN_V1=1 sends every call to the streaming v1 kernels (read once, not per launch)
const bool g_attn_v1 = getenv("MMFD_ATTN_V1") != nullptr;

int g_fp32_attn_mode = [] {
  const char* v = getenv("MMFD_FP32_ATTN");
  const char* gm = getenv("MMFD_FP32_GEMM");
  const bool native = (v && (!strcmp(v, "native") || !strcmp(v, "0"))) ||
                      (!v && gm && (!strcmp(gm, "native") || !strcmp(gm, "0")));
  return native ? 0 : 1;
}();

__device__ __forceinline__ void split8(const float* x, uint4& hi, uint4& mid, uint4& lo) {
  bf16x8 h, m, l;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const bf16 hu = (bf16)x[u];
    const float r = x[u] - (float)hu;
    const bf16 mu = (bf16)r;
    h[u] = hu;
    m[u] = mu;
    l[u] = (bf16)(r - (float)mu);
  }
  hi = __builtin_bit_cast(uint4, h);
  mid = __builtin_bit_cast(uint4, m);
  lo = __builtin_bit_cast(uint4, l);
}

// acc += (a0 + a1 + a2) (b0 + b1 + b2) over one 32-deep chunk, planes 0/1/2 = hi/mid/lo, small first
__device__ __forceinline__ void mma6(f32x4& acc, const uint4& ah, const uint4& am, const uint4& al, const uint4& bh,
                                     const uint4& bm, const uint4& bl) {
  Mma<bf16>::run(acc, am, bm);
  Mma<bf16>::run(acc, ah, bl);
  Mma<bf16>::run(acc, al, bh);
  Mma<bf16>::run(acc, ah, bm);
  Mma<bf16>::run(acc, am, bh);
  Mma<bf16>::run(acc, ah, bh);
}

// the planes of 16x16 fp32 accumulators (rows in split order) as the A fragment of one 32-key chunk
__device__ __forceinline__ void split_acc(const f32x4& a, const f32x4& b, uint4& hi, uint4& mid, uint4& lo) {
  const float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  split8(x, hi, mid, lo);
}

// one fp32 row's MFMA fragments (lane: elements (kc*4 + g)*8 .. +7): loaded raw, split into planes
// f[plane][kc] later (the loads of the next block issue before the current block's products)
template <int KCH> struct X6Row { float4 v[KCH][2]; };
template <int KCH>
__device__ __forceinline__ void x6_row_load(X6Row<KCH>& x, const float* __restrict__ base, int64_t st, int64_t row,
                                            int64_t nrows, int lane, int dreal) {
  const int g = lane >> 4;
#pragma unroll
  for (int kc = 0; kc < KCH; ++kc) {
    const int col = (kc * 4 + g) * 8;
    x.v[kc][0] = x.v[kc][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < nrows && col < dreal) {
      const float* src = base + row * st + col;
      x.v[kc][0] = *reinterpret_cast<const float4*>(src);
      x.v[kc][1] = *reinterpret_cast<const float4*>(src + 4);
    }
  }
}
template <int KCH>
__device__ __forceinline__ void x6_row_split(uint4 (&f)[3][KCH], const X6Row<KCH>& x) {
#pragma unroll
  for (int kc = 0; kc < KCH; ++kc) {
    const float4 a = x.v[kc][0], b = x.v[kc][1];
    const float e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    split8(e, f[0][kc], f[1][kc], f[2][kc]);
  }
}

// stage two fp32 head slices (rows [0, nrows), zero rows up to nrows_pad) as three plane images
// each: every load of the thread is issued before the first split, so the HBM latency is paid once
// per workgroup rather than once per 16-B chunk (the one-chunk-at-a-time loop took ~16k cycles
// for a 197-row K|V pair, 26 % of the ViT forward workgroup)
template <int D, int NTH>
__device__ __forceinline__ void x6_stage2(char* img_a, const float* __restrict__ base_a, int64_t st_a, char* img_b,
                                          const float* __restrict__ base_b, int64_t st_b, int img, int64_t nrows,
                                          int nrows_pad, int tid, int dreal, int dbg) {
  constexpr int NC = D / 8;
  constexpr int MAXT = (X6A_LMAX * NC + NTH - 1) / NTH;
  const int total = nrows_pad * NC;
  float4 xa[MAXT][2], xb[MAXT][2];
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    const int c = tid + j * NTH;
    const int r = c / NC, ch = c % NC;
    xa[j][0] = xa[j][1] = xb[j][0] = xb[j][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < total && r < nrows && ch * 8 < dreal && !(dbg & 1)) {
      const float* sa = base_a + (int64_t)r * st_a + ch * 8;
      const float* sb = base_b + (int64_t)r * st_b + ch * 8;
      xa[j][0] = *reinterpret_cast<const float4*>(sa);
      xa[j][1] = *reinterpret_cast<const float4*>(sa + 4);
      xb[j][0] = *reinterpret_cast<const float4*>(sb);
      xb[j][1] = *reinterpret_cast<const float4*>(sb + 4);
    }
  }
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    const int c = tid + j * NTH;
    if (c < total) {
      const int r = c / NC, ch = c % NC;
      const int off = row_off<bf16, 64>(r, ch);
      uint4 h, m, l;
      {
        const float e[8] = {xa[j][0].x, xa[j][0].y, xa[j][0].z, xa[j][0].w, xa[j][1].x, xa[j][1].y, xa[j][1].z, xa[j][1].w};
        split8(e, h, m, l);
        *reinterpret_cast<uint4*>(img_a + off) = h;
        *reinterpret_cast<uint4*>(img_a + img + off) = m;
        *reinterpret_cast<uint4*>(img_a + 2 * img + off) = l;
      }
      {
        const float e[8] = {xb[j][0].x, xb[j][0].y, xb[j][0].z, xb[j][0].w, xb[j][1].x, xb[j][1].y, xb[j][1].z, xb[j][1].w};
        split8(e, h, m, l);
        *reinterpret_cast<uint4*>(img_b + off) = h;
        *reinterpret_cast<uint4*>(img_b + img + off) = m;
        *reinterpret_cast<uint4*>(img_b + 2 * img + off) = l;
      }
    }
  }
}

// transposed B fragment of one 32-row chunk c (rows in split order) from a plane image; h1off =
// byte distance of the chunk's second 16 rows (16 * 128, or 0 to repeat the first half)
__device__ __forceinline__ uint4 x6_tr_frag(const char* lds, int c, int dsub, int lane, int h1off) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2;
  const int u = dsub * 4 + (i & 3);
  const int r = c * 32 + 4 * g + q;
  const int off = r * X6A_RB + (((u >> 1) ^ (r & 7)) << 4) + ((u & 1) << 3);
  const uint2 x0 = lds_read_tr16(lds + off);
  const uint2 x1 = lds_read_tr16(lds + off + h1off);
  return make_uint4(x0.x, x0.y, x1.x, x1.y);
}

__device__ __forceinline__ void x6_row_frag3(uint4* f, const char* lds, int img, int sub, int kc, int lane) {
  f[0] = row_frag<bf16, 64>(lds, sub, kc, lane);
  f[1] = row_frag<bf16, 64>(lds + img, sub, kc, lane);
  f[2] = row_frag<bf16, 64>(lds + 2 * img, sub, kc, lane);
}
__device__ __forceinline__ void x6_tr_frag3(uint4* f, const char* lds, int img, int c, int d, int lane, int h1off) {
  f[0] = x6_tr_frag(lds, c, d, lane, h1off);
  f[1] = x6_tr_frag(lds + img, c, d, lane, h1off);
  f[2] = x6_tr_frag(lds + 2 * img, c, d, lane, h1off);
}

// Every product phase below is software pipelined by hand: the fragments of step i + 1 are read
// (into the other half of a two-deep register buffer) before step i's six MFMAs issue, and the
// first step of the phase after the softmax is read before the softmax's vector work, so LDS
// latency hides behind MFMAs instead of stalling each group of six (the compiler-scheduled form
// read and waited per group: ViT forward 732 us).

template <int D, bool DROP>
__global__ void __launch_bounds__(V2_THREADS, 1) attn_fwd_x6_kernel(AttnP p) {
  // K/V planes of the head resident; each wave sweeps 16-query blocks with the v2 online softmax
  constexpr int KCH = D / 32, DT = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  X6A_STAMP(0);
  const int lk16 = v2_pad(p.Lk, 16);
  const int img = lk16 * X6A_RB;
  char* k_img = smem;
  char* v_img = smem + 3 * img;
  float* kbias = reinterpret_cast<float*>(smem + 6 * img);
  const float* qb = reinterpret_cast<const float*>(p.q) + b * p.q_sb + h * p.D;
  X6Row<KCH> qn;  // the wave's next query block, raw (one block ahead)
  x6_row_load<KCH>(qn, qb, p.q_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
  x6_stage2<D, V2_THREADS>(k_img, reinterpret_cast<const float*>(p.k) + b * p.k_sb + h * p.D, p.k_st, v_img,
                           reinterpret_cast<const float*>(p.v) + b * p.v_sb + h * p.D, p.v_st, img, p.Lk, lk16, tid,
                           p.D, p.dbg);
  stage_kbias<V2_THREADS>(kbias, p, b, lk16, tid);
  __syncthreads();
  X6A_STAMP(1);
  const uint64_t seed = DROP ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);
  const float c2 = p.scale * LOG2E;
  float* ob = reinterpret_cast<float*>(p.o) + b * p.o_sb + h * p.D;
  const int nqb = (int)((p.Lq + 15) / 16);
  // one query block over the 64-key chunks [c0, c1) (online softmax state o, m, lsum)
  const int nfc = lk16 / 64;                       // full 64-key chunks
  const int nchk = nfc + ((lk16 & 63) ? 1 : 0);    // + the padded tail chunk
  auto qrun = [&](int qbk, const uint4 (&qf)[3][KCH], int c0, int c1, f32x4 (&o)[DT], float& m, float& lsum) {
    const int64_t q0 = (int64_t)qbk * 16, myq = q0 + li;
    const uint64_t hrow = (uint64_t)(bh * p.Lq + myq) * (uint64_t)p.kp;  // pair-index base of this query row
    const uint32_t rowc1 = ((uint32_t)hrow + (uint32_t)(2 * g)) * HASH_C1;
    auto chunk = [&](int k0, auto nsc) {
      constexpr int NS = decltype(nsc)::value;  // 16-key subtiles present (4 but in the last chunk)
      constexpr int NC = (NS + 1) / 2;           // 32-key chunks of P V
      const char* kc_img = k_img + k0 * X6A_RB;
      const char* vc_img = v_img + k0 * X6A_RB;
      f32x4 s[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) s[ks] = f32x4{0.f, 0.f, 0.f, 0.f};
      {  // S^T = K Q^T, steps (kc, ks)
        constexpr int N = KCH * NS;
        uint4 f[2][3];
        x6_row_frag3(f[0], kc_img, img, 0, 0, lane);
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (i + 1 < N) x6_row_frag3(f[(i + 1) & 1], kc_img, img, (i + 1) % NS, (i + 1) / NS, lane);
          const int kc = i / NS, ks = i % NS;
          mma6(s[ks], f[i & 1][0], f[i & 1][1], f[i & 1][2], qf[0][kc], qf[1][kc], qf[2][kc]);
        }
      }
      // P V steps (c, d); an odd last subtile pairs with zero P (s[NS] stays 0) over repeated V rows
      constexpr int NV = NC * DT;
      auto ld_v = [&](int i, uint4* f) {
        const int c = i / DT, d = i % DT;
        x6_tr_frag3(f, vc_img, img, c, d, lane, (2 * c + 1 < NS) ? 16 * X6A_RB : 0);
      };
      uint4 vf[2][3];
      ld_v(0, vf[0]);
      float mx = -INFINITY;
#pragma unroll
      for (int ks = 0; ks < NS; ++ks) {
        const float4 kb4 = *reinterpret_cast<const float4*>(kbias + k0 + ks * 16 + 4 * g);
        const float kb[4] = {kb4.x, kb4.y, kb4.z, kb4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t = fmaf(s[ks][r], c2, kb[r]);
          s[ks][r] = t;
          mx = fmaxf(mx, t);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      float rs = 0.f;
#pragma unroll
      for (int ks = 0; ks < NS; ++ks) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(s[ks][r] - mnew);
          rs += e;
          s[ks][r] = e;
        }
      }
      if constexpr (DROP) {
        const uint32_t cc = rowc1 + (uint32_t)(k0 >> 1) * HASH_C1;
        uint32_t kbits = 0;
#pragma unroll
        for (int ks = 0; ks < NS; ++ks) {
          const uint32_t h0 = hash_c1(hkey, cc + (uint32_t)(ks * 8) * HASH_C1);
          const uint32_t h1 = hash_c1(hkey, cc + (uint32_t)(ks * 8 + 1) * HASH_C1);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool kp = pair_keep(r < 2 ? h0 : h1, r & 1, p.thr16);
            s[ks][r] = kp ? s[ks][r] * p.keep_scale : 0.f;
            kbits |= (uint32_t)kp << (ks * 4 + r);
          }
        }
        if (p.dm) dm_write64(p, bh, myq, k0, g, kbits);  // the backward kernels read it
      }
      lsum = lsum * alpha + rs;
      m = mnew;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
        for (int d = 0; d < DT; ++d) o[d][r] *= ar;
      }
      uint4 pp[NC][3];
#pragma unroll
      for (int c = 0; c < NC; ++c) split_acc(s[2 * c], s[2 * c + 1], pp[c][0], pp[c][1], pp[c][2]);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        if (i + 1 < NV) ld_v(i + 1, vf[(i + 1) & 1]);
        const int c = i / DT, d = i % DT;
        mma6(o[d], pp[c][0], pp[c][1], pp[c][2], vf[i & 1][0], vf[i & 1][1], vf[i & 1][2]);
      }
    };
    const int ce = c1 < nfc ? c1 : nfc;
    for (int c = c0; c < ce; ++c) chunk(c * 64, std::integral_constant<int, 4>{});
    if (c1 > nfc) {
      const int k0 = nfc * 64;
      switch ((lk16 - k0) >> 4) {
        case 1: chunk(k0, std::integral_constant<int, 1>{}); break;
        case 2: chunk(k0, std::integral_constant<int, 2>{}); break;
        case 3: chunk(k0, std::integral_constant<int, 3>{}); break;
        default: break;
      }
    }
  };
  // normalise and store one query block (lsum already summed over the four lane groups)
  auto qfin = [&](int qbk, const f32x4 (&o)[DT], float m, float lsum) {
    const int64_t q0 = (int64_t)qbk * 16, myq = q0 + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float lr = __shfl(lsum, 4 * g + r, 64);
      const int64_t q = q0 + 4 * g + r;
      const float inv = 1.0f / lr;
      if (q < p.Lq) {
#pragma unroll
        for (int d = 0; d < DT; ++d)
          if (d * 16 + li < p.D) {
            const float val = o[d][r] * inv;
            ob[q * p.o_st + d * 16 + li] = val;
            if (p.pl) plane_put(p, ob + q * p.o_st + d * 16 + li, val);
          }
      }
    }
    if (g == 0 && myq < p.Lq) p.lse[bh * p.Lq + myq] = (m + log2f(lsum)) * LN2;
  };
  if (p.dbg & 2) return;
  // the last query block halved over the key chunks between two SIMD pairs when the blocks do not
  // spread evenly (ViT: 13 blocks), as in dK/dV; the halves' softmax states merge in LDS
  const int R = nqb - V2_THREADS / 64;
  const bool split = R >= 1 && R <= V2_THREADS / 64 && (R & 3) == 1 && nchk >= 2;
  const int nwhole = split ? nqb - 1 : nqb;
  for (int qbk = wave; qbk < nwhole; qbk += V2_THREADS / 64) {
    uint4 qf[3][KCH];
    x6_row_split<KCH>(qf, qn);
    if (qbk + V2_THREADS / 64 < nwhole)
      x6_row_load<KCH>(qn, qb, p.q_st, (int64_t)(qbk + V2_THREADS / 64) * 16 + li, p.Lq, lane, p.D);
    if (qbk == wave) X6A_STAMP(2);
    float m = -INFINITY, lsum = 0.f;
    f32x4 o[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    qrun(qbk, qf, 0, nchk, o, m, lsum);
    if (qbk == wave) X6A_STAMP(7);
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    qfin(qbk, o, m, lsum);
    if (qbk == wave) X6A_STAMP(8);
  }
  if (split) {
    const int sb = nqb - 1, hc = nchk / 2;
    const bool own = wave == R - 1, part = wave == R;
    float m = -INFINITY, lsum = 0.f;
    f32x4 o[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (own || part) {
      X6Row<KCH> qr;
      x6_row_load<KCH>(qr, qb, p.q_st, (int64_t)sb * 16 + li, p.Lq, lane, p.D);
      uint4 qf[3][KCH];
      x6_row_split<KCH>(qf, qr);
      qrun(sb, qf, own ? 0 : hc, own ? hc : nchk, o, m, lsum);
      lsum += __shfl_xor(lsum, 16, 64);
      lsum += __shfl_xor(lsum, 32, 64);
    }
    __syncthreads();  // every wave is done with the K / V images: reuse them for the exchange
    f32x4* xo = reinterpret_cast<f32x4*>(smem);
    float* xm = reinterpret_cast<float*>(smem + DT * 64 * 16);
    if (part) {
#pragma unroll
      for (int d = 0; d < DT; ++d) xo[d * 64 + lane] = o[d];
      xm[lane] = m;
      xm[64 + lane] = lsum;
    }
    __syncthreads();
    if (own) {  // merge: m = max, each half's sums rescaled by exp2(m_half - m)
      const float mb = xm[lane], lb = xm[64 + lane];
      const float mm = fmaxf(m, mb);
      const float aa = __builtin_amdgcn_exp2f(m - mm), ab = __builtin_amdgcn_exp2f(mb - mm);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ra = __shfl(aa, 4 * g + r, 64), rb = __shfl(ab, 4 * g + r, 64);
#pragma unroll
        for (int d = 0; d < DT; ++d) o[d][r] = o[d][r] * ra + xo[d * 64 + lane][r] * rb;
      }
      qfin(sb, o, mm, lsum * aa + lb * ab);
    }
  }
  X6A_STAMP(9);
}

// DROP (dK/dV, dQ): 0 = none, 1 = re-hash the forward's mask, 2 = read the forward's keep-bitmask
template <int D, int DROP>
__global__ void __launch_bounds__(V2_THREADS, 1) attn_dkdv_x6_kernel(AttnP p) {
  // Q/dO planes of the head resident (+ lse, delta, key bias); each wave owns 16 keys
  constexpr int KCH = D / 32, DT = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const int lq16 = v2_pad(p.Lq, 16), lk16 = v2_pad(p.Lk, 16);
  const int img = lq16 * X6A_RB;
  char* q_img = smem;
  char* do_img = smem + 3 * img;
  float* s_lse = reinterpret_cast<float*>(smem + 6 * img);
  float* s_delta = s_lse + lq16;
  float* kbias = s_delta + lq16;
  uint32_t* s_dm = reinterpret_cast<uint32_t*>(kbias + lk16);  // DROP == 2: the head's keep-bitmask rows
  const float* kb = reinterpret_cast<const float*>(p.k) + b * p.k_sb + h * p.D;
  const float* vb = reinterpret_cast<const float*>(p.v) + b * p.v_sb + h * p.D;
  if constexpr (DROP == 2) {
    const uint32_t* src = dm_row(p, bh, 0);
    const int nw = (int)p.Lq * p.dmw;
    for (int i = tid; i < lq16 * p.dmw; i += V2_THREADS) s_dm[i] = i < nw ? src[i] : 0u;
  }
  X6Row<KCH> kn, vn;  // the wave's first key block, raw (loaded with the staging)
  x6_row_load<KCH>(kn, kb, p.k_st, (int64_t)wave * 16 + li, p.Lk, lane, p.D);
  x6_row_load<KCH>(vn, vb, p.v_st, (int64_t)wave * 16 + li, p.Lk, lane, p.D);
  x6_stage2<D, V2_THREADS>(q_img, reinterpret_cast<const float*>(p.q) + b * p.q_sb + h * p.D, p.q_st, do_img,
                           reinterpret_cast<const float*>(p.dout) + b * p.do_sb + h * p.D, p.do_st, img, p.Lq, lq16,
                           tid, p.D, p.dbg);
  for (int i = tid; i < lq16; i += V2_THREADS) {
    s_lse[i] = i < p.Lq ? p.lse[bh * p.Lq + i] * LOG2E : INFINITY;
    s_delta[i] = i < p.Lq ? p.delta[bh * p.Lq + i] : 0.f;
  }
  stage_kbias<V2_THREADS>(kbias, p, b, lk16, tid);
  __syncthreads();
  float* dkb = reinterpret_cast<float*>(p.dk) + b * p.dk_sb + h * p.D;
  float* dvb = reinterpret_cast<float*>(p.dv) + b * p.dv_sb + h * p.D;
  const uint64_t seed = DROP ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);
  const float c2 = p.scale * LOG2E;
  const int nkb = lk16 / 16;
  // one key block; called for the first block on the rows loaded with the staging and then on
  // fresh loads (a loop over both would keep the prefetched rows live across the back edge)
  // dK / dV of one key block over the query chunks [qa, qb) into dkv (dV even, dK odd per 16-wide
  // D subtile)
  auto kblock = [&](int kbk, const X6Row<KCH>& kr, const X6Row<KCH>& vr, int qa, int qb, f32x4 (&dkv)[2 * DT]) {
    const int64_t k0 = (int64_t)kbk * 16, mykey = k0 + li;
    uint4 kf[3][KCH], vf[3][KCH];
    x6_row_split<KCH>(kf, kr);
    x6_row_split<KCH>(vf, vr);
    const float kb2 = kbias[mykey];  // -inf for padded keys -> P = 0
    const uint64_t hcol = (uint64_t)(bh * p.Lq) * (uint64_t)p.kp + (uint64_t)(mykey >> 1);  // pair index, query 0
    const int kodd = (int)(mykey & 1);
    const uint32_t kpc1 = (uint32_t)p.kp * HASH_C1;
    const uint32_t colc1 = (uint32_t)hcol * HASH_C1 + (uint32_t)(4 * g + 2 * kodd) * kpc1;
    auto chunk = [&](int qc, auto nsc) {
      constexpr int NS = decltype(nsc)::value;  // 16-query subtiles of this 32-query chunk
      f32x4 sd[4];  // S (even) and dP (odd) per subtile
#pragma unroll
      for (int i = 0; i < 4; ++i) sd[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      {  // S = Q K^T and dP = dO V^T, steps (kc, h2)
        constexpr int N = KCH * NS;
        uint4 f[2][6];
        auto ld = [&](int i, uint4* fr) {
          const int sub = 2 * qc + i % NS, kc = i / NS;
          x6_row_frag3(fr, q_img, img, sub, kc, lane);
          x6_row_frag3(fr + 3, do_img, img, sub, kc, lane);
        };
        ld(0, f[0]);
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (i + 1 < N) ld(i + 1, f[(i + 1) & 1]);
          const int kc = i / NS, h2 = i % NS;
          const uint4* fr = f[i & 1];
          mma6(sd[2 * h2], fr[0], fr[1], fr[2], kf[0][kc], kf[1][kc], kf[2][kc]);
          mma6(sd[2 * h2 + 1], fr[3], fr[4], fr[5], vf[0][kc], vf[1][kc], vf[2][kc]);
        }
      }
      constexpr int h1off = NS == 2 ? 16 * X6A_RB : 0;
      uint4 tb[2][6];  // transposed dO / Q planes of one D subtile (B operands of dV / dK)
      auto ldt = [&](int d, uint4* fr) {
        x6_tr_frag3(fr, do_img, img, qc, d, lane, h1off);
        x6_tr_frag3(fr + 3, q_img, img, qc, d, lane, h1off);
      };
      ldt(0, tb[0]);
      f32x4 pd[2], ds[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) { pd[h2] = f32x4{0.f, 0.f, 0.f, 0.f}; ds[h2] = pd[h2]; }
      float z[NS][4];
#pragma unroll
      for (int h2 = 0; h2 < NS; ++h2)
#pragma unroll
        for (int r = 0; r < 4; ++r) z[h2][r] = 1.f;
      if constexpr (DROP == 1) {  // the element index advances by Lk per query
#pragma unroll
        for (int h2 = 0; h2 < NS; ++h2) {
          const uint32_t e = colc1 + (uint32_t)((2 * qc + h2) * 16) * kpc1;
          keep4_col(hash_c1(hkey, e), hash_c1(hkey, e + kpc1), kodd, p, z[h2]);
        }
      } else if constexpr (DROP == 2) {  // bit mykey of the query rows' words (LDS broadcast reads)
        const uint32_t* col = s_dm + (mykey >> 5);
        const int sh = (int)(mykey & 31);
#pragma unroll
        for (int h2 = 0; h2 < NS; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            z[h2][r] = ((col[((2 * qc + h2) * 16 + 4 * g + r) * p.dmw] >> sh) & 1u) ? p.keep_scale : 0.f;
      }
#pragma unroll
      for (int h2 = 0; h2 < NS; ++h2) {
        const int qs = 2 * qc + h2;
        const f32x4 sv = sd[2 * h2], dp = sd[2 * h2 + 1];
        const float4 l4 = *reinterpret_cast<const float4*>(s_lse + qs * 16 + 4 * g);
        const float4 d4 = *reinterpret_cast<const float4*>(s_delta + qs * 16 + 4 * g);
        const float lq2[4] = {l4.x, l4.y, l4.z, l4.w}, dl[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pr = __builtin_amdgcn_exp2f(fmaf(sv[r], c2, kb2) - lq2[r]);
          pd[h2][r] = pr * z[h2][r];
          ds[h2][r] = pr * (dp[r] * z[h2][r] - dl[r]);
        }
      }
      uint4 ph, pm, pl, sh, sm, sl;
      split_acc(pd[0], pd[1], ph, pm, pl);
      split_acc(ds[0], ds[1], sh, sm, sl);
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        if (d + 1 < DT) ldt(d + 1, tb[(d + 1) & 1]);
        const uint4* fr = tb[d & 1];
        mma6(dkv[2 * d], ph, pm, pl, fr[0], fr[1], fr[2]);
        mma6(dkv[2 * d + 1], sh, sm, sl, fr[3], fr[4], fr[5]);
      }
    };
    const int nfull = lq16 / 32;
    const int qe = qb < nfull ? qb : nfull;
    for (int qc = qa; qc < qe; ++qc) chunk(qc, std::integral_constant<int, 2>{});
    if (qb > nfull) chunk(nfull, std::integral_constant<int, 1>{});
  };
  auto kstore = [&](int kbk, const f32x4 (&dkv)[2 * DT]) {
    const int64_t k0 = (int64_t)kbk * 16;
    if (p.vst) {  // (uniform) quad transposes, then 4-column stores
      const int t = li & 3, c4 = 4 * (li >> 2);
      const int64_t key = k0 + 4 * g + t;
      float* krow = dkb + key * p.dk_st + c4;
      float* vrow = dvb + key * p.dv_st + c4;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        float xk[4] = {dkv[2 * d + 1][0] * p.scale, dkv[2 * d + 1][1] * p.scale, dkv[2 * d + 1][2] * p.scale,
                       dkv[2 * d + 1][3] * p.scale};
        float xv[4] = {dkv[2 * d][0], dkv[2 * d][1], dkv[2 * d][2], dkv[2 * d][3]};
        quad_tr(xk, t);
        quad_tr(xv, t);
        if (key < p.Lk && d * 16 + c4 < p.D) {
          x6_put4(p, krow + d * 16, xk, p.acc_dkv);
          x6_put4(p, vrow + d * 16, xv, p.acc_dkv);
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t key = k0 + 4 * g + r;
      if (key < p.Lk) {
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          if (d * 16 + li >= p.D) continue;
          float* pk = dkb + key * p.dk_st + d * 16 + li;
          float* pv = dvb + key * p.dv_st + d * 16 + li;
          float vk = dkv[2 * d + 1][r] * p.scale, vv = dkv[2 * d][r];
          if (p.acc_dkv) { vk += *pk; vv += *pv; }
          if (p.pl) {
            plane_put(p, pk, vk);
            plane_put(p, pv, vv);
            if (p.pl_only) continue;
          }
          *pk = vk;
          *pv = vv;
        }
      }
    }
  };
  if (p.dbg & 2) return;
  // 8 waves share the key blocks round robin; waves w and w + 4 share a SIMD, so with R = nkb - 8
  // extra blocks and R % 4 == 1 (ViT: 13 blocks) one SIMD pair would carry one block more than the
  // others. The last block is then halved over the query chunks between waves R - 1 and R (two
  // SIMD pairs), whose partial sums meet in LDS once every wave is done with the Q / dO images.
  const int nch = lq16 / 32 + ((lq16 & 16) ? 1 : 0);
  const int R = nkb - V2_THREADS / 64;
  const bool split = R >= 1 && R <= V2_THREADS / 64 && (R & 3) == 1 && nch >= 2;
  const int nwhole = split ? nkb - 1 : nkb;
  if (wave < nwhole) {
    f32x4 dkv[2 * DT];
#pragma unroll
    for (int i = 0; i < 2 * DT; ++i) dkv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    kblock(wave, kn, vn, 0, nch, dkv);
    kstore(wave, dkv);
  }
  for (int kbk = wave + V2_THREADS / 64; kbk < nwhole; kbk += V2_THREADS / 64) {
    X6Row<KCH> kr, vr;
    x6_row_load<KCH>(kr, kb, p.k_st, (int64_t)kbk * 16 + li, p.Lk, lane, p.D);
    x6_row_load<KCH>(vr, vb, p.v_st, (int64_t)kbk * 16 + li, p.Lk, lane, p.D);
    f32x4 dkv[2 * DT];
#pragma unroll
    for (int i = 0; i < 2 * DT; ++i) dkv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    kblock(kbk, kr, vr, 0, nch, dkv);
    kstore(kbk, dkv);
  }
  if (split) {
    const int sb = nkb - 1, hc = nch / 2;
    const bool own = wave == R - 1, part = wave == R;
    f32x4 dkv[2 * DT];
#pragma unroll
    for (int i = 0; i < 2 * DT; ++i) dkv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (own || part) {
      X6Row<KCH> kr, vr;
      x6_row_load<KCH>(kr, kb, p.k_st, (int64_t)sb * 16 + li, p.Lk, lane, p.D);
      x6_row_load<KCH>(vr, vb, p.v_st, (int64_t)sb * 16 + li, p.Lk, lane, p.D);
      kblock(sb, kr, vr, own ? 0 : hc, own ? hc : nch, dkv);
    }
    __syncthreads();  // every wave is done with the Q / dO images: reuse them for the exchange
    f32x4* xch = reinterpret_cast<f32x4*>(smem);
    if (part) {
#pragma unroll
      for (int i = 0; i < 2 * DT; ++i) xch[i * 64 + lane] = dkv[i];
    }
    __syncthreads();
    if (own) {
#pragma unroll
      for (int i = 0; i < 2 * DT; ++i) dkv[i] += xch[i * 64 + lane];
      kstore(sb, dkv);
    }
  }
}

template <int D, int DROP>
__global__ void __launch_bounds__(V2_THREADS, 1) attn_dq_x6_kernel(AttnP p) {
  // K/V planes of the head resident; each wave owns 16 queries: dQ = dS K
  constexpr int KCH = D / 32, DT = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const int lk16 = v2_pad(p.Lk, 16);
  const int img = lk16 * X6A_RB;
  char* k_img = smem;
  char* v_img = smem + 3 * img;
  float* kbias = reinterpret_cast<float*>(smem + 6 * img);
  const float* qb = reinterpret_cast<const float*>(p.q) + b * p.q_sb + h * p.D;
  const float* dob = reinterpret_cast<const float*>(p.dout) + b * p.do_sb + h * p.D;
  const float* obp = reinterpret_cast<const float*>(p.o) + b * p.o_sb + h * p.D;
  X6Row<KCH> qn, don, on;  // the wave's first query block, raw (loaded with the staging)
  x6_row_load<KCH>(qn, qb, p.q_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
  x6_row_load<KCH>(don, dob, p.do_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
  x6_row_load<KCH>(on, obp, p.o_st, (int64_t)wave * 16 + li, p.Lq, lane, p.D);
  x6_stage2<D, V2_THREADS>(k_img, reinterpret_cast<const float*>(p.k) + b * p.k_sb + h * p.D, p.k_st, v_img,
                           reinterpret_cast<const float*>(p.v) + b * p.v_sb + h * p.D, p.v_st, img, p.Lk, lk16, tid,
                           p.D, p.dbg);
  stage_kbias<V2_THREADS>(kbias, p, b, lk16, tid);
  __syncthreads();
  float* dqb = reinterpret_cast<float*>(p.dq) + b * p.dq_sb + h * p.D;
  const uint64_t seed = DROP ? *p.seed : 0ull;
  const uint32_t hkey = mmfd_hash_key(seed, p.salt);
  const float c2 = p.scale * LOG2E;
  const int nqb = (int)((p.Lq + 15) / 16);
  // dQ of one query block over the key chunks [ka, kb2e) into dq (as kblock in dK/dV)
  // delta = rowsum(dO * O) of the block's queries is computed here from the rows the wave loads
  // anyway (no separate delta pass: the dQ kernel runs first and writes it for dK/dV)
  auto qblock = [&](int qbk, const X6Row<KCH>& qr, const X6Row<KCH>& dr, const X6Row<KCH>& orow, bool wdelta,
                    int ka, int kb2e, f32x4 (&dq)[DT]) {
    const int64_t q0 = (int64_t)qbk * 16, myq = q0 + li;
    uint4 qf[3][KCH], dof[3][KCH];
    x6_row_split<KCH>(qf, qr);
    x6_row_split<KCH>(dof, dr);
    const float lse2 = myq < p.Lq ? p.lse[bh * p.Lq + myq] * LOG2E : INFINITY;
    float dsum = 0.f;
#pragma unroll
    for (int kc = 0; kc < KCH; ++kc)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const float4 a = orow.v[kc][hh], c = dr.v[kc][hh];
        dsum = fmaf(a.x, c.x, fmaf(a.y, c.y, fmaf(a.z, c.z, fmaf(a.w, c.w, dsum))));
      }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    const float dlt = myq < p.Lq ? dsum : 0.f;
    if (wdelta && g == 0 && myq < p.Lq) p.delta[bh * p.Lq + myq] = dsum;
    const uint64_t hrow = (uint64_t)(bh * p.Lq + myq) * (uint64_t)p.kp;  // pair-index base of this query row
    const uint32_t rowc1 = ((uint32_t)hrow + (uint32_t)(2 * g)) * HASH_C1;
    const uint32_t* dmrow = DROP == 2 ? dm_row(p, bh, myq < p.Lq ? myq : 0) : nullptr;
    auto chunk = [&](int kc2, auto nsc) {
      constexpr int NS = decltype(nsc)::value;  // 16-key subtiles of this 32-key chunk
      uint32_t kw = 0;  // DROP == 2: the chunk's keep word (32 keys), loaded ahead of the products
      if constexpr (DROP == 2) kw = dmrow[kc2];
      f32x4 sd[4];  // S^T (even) and dP^T (odd) per subtile
#pragma unroll
      for (int i = 0; i < 4; ++i) sd[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      {  // S^T = K Q^T and dP^T = V dO^T, steps (kc, h2)
        constexpr int N = KCH * NS;
        uint4 f[2][6];
        auto ld = [&](int i, uint4* fr) {
          const int sub = 2 * kc2 + i % NS, kc = i / NS;
          x6_row_frag3(fr, k_img, img, sub, kc, lane);
          x6_row_frag3(fr + 3, v_img, img, sub, kc, lane);
        };
        ld(0, f[0]);
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (i + 1 < N) ld(i + 1, f[(i + 1) & 1]);
          const int kc = i / NS, h2 = i % NS;
          const uint4* fr = f[i & 1];
          mma6(sd[2 * h2], fr[0], fr[1], fr[2], qf[0][kc], qf[1][kc], qf[2][kc]);
          mma6(sd[2 * h2 + 1], fr[3], fr[4], fr[5], dof[0][kc], dof[1][kc], dof[2][kc]);
        }
      }
      constexpr int h1off = NS == 2 ? 16 * X6A_RB : 0;
      uint4 tk[2][3];  // transposed K planes of one D subtile (B operand of dQ)
      x6_tr_frag3(tk[0], k_img, img, kc2, 0, lane, h1off);
      f32x4 ds[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) ds[h2] = f32x4{0.f, 0.f, 0.f, 0.f};
      float z[NS][4];
#pragma unroll
      for (int h2 = 0; h2 < NS; ++h2)
#pragma unroll
        for (int r = 0; r < 4; ++r) z[h2][r] = 1.f;
      if constexpr (DROP == 1) {
#pragma unroll
        for (int h2 = 0; h2 < NS; ++h2) {
          const uint32_t e = rowc1 + (uint32_t)((2 * kc2 + h2) * 8) * HASH_C1;
          keep4_pairs(hash_c1(hkey, e), hash_c1(hkey, e + HASH_C1), p, z[h2]);
        }
      } else if constexpr (DROP == 2) {
#pragma unroll
        for (int h2 = 0; h2 < NS; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r) z[h2][r] = ((kw >> (h2 * 16 + 4 * g + r)) & 1u) ? p.keep_scale : 0.f;
      }
#pragma unroll
      for (int h2 = 0; h2 < NS; ++h2) {
        const int ks = 2 * kc2 + h2;
        const f32x4 sv = sd[2 * h2], dp = sd[2 * h2 + 1];
        const float4 kb4 = *reinterpret_cast<const float4*>(kbias + ks * 16 + 4 * g);
        const float kbr[4] = {kb4.x, kb4.y, kb4.z, kb4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pr = __builtin_amdgcn_exp2f(fmaf(sv[r], c2, kbr[r]) - lse2);
          ds[h2][r] = pr * (dp[r] * z[h2][r] - dlt);
        }
      }
      uint4 sh, sm, sl;
      split_acc(ds[0], ds[1], sh, sm, sl);
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        if (d + 1 < DT) x6_tr_frag3(tk[(d + 1) & 1], k_img, img, kc2, d + 1, lane, h1off);
        const uint4* fr = tk[d & 1];
        mma6(dq[d], sh, sm, sl, fr[0], fr[1], fr[2]);
      }
    };
    const int nfull = lk16 / 32;
    const int ke = kb2e < nfull ? kb2e : nfull;
    for (int kc2 = ka; kc2 < ke; ++kc2) chunk(kc2, std::integral_constant<int, 2>{});
    if (kb2e > nfull) chunk(nfull, std::integral_constant<int, 1>{});
  };
  auto qstore = [&](int qbk, const f32x4 (&dq)[DT]) {
    const int64_t q0 = (int64_t)qbk * 16;
    if (p.vst) {  // (uniform) quad transposes, then 4-column stores
      const int t = li & 3, c4 = 4 * (li >> 2);
      const int64_t q = q0 + 4 * g + t;
      float* qrow = dqb + q * p.dq_st + c4;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        float x[4] = {dq[d][0] * p.scale, dq[d][1] * p.scale, dq[d][2] * p.scale, dq[d][3] * p.scale};
        quad_tr(x, t);
        if (q < p.Lq && d * 16 + c4 < p.D) x6_put4(p, qrow + d * 16, x, p.acc_dq);
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t q = q0 + 4 * g + r;
      if (q < p.Lq) {
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          if (d * 16 + li >= p.D) continue;
          float* pq = dqb + q * p.dq_st + d * 16 + li;
          float vq = dq[d][r] * p.scale;
          if (p.acc_dq) vq += *pq;
          if (p.pl) {
            plane_put(p, pq, vq);
            if (p.pl_only) continue;
          }
          *pq = vq;
        }
      }
    }
  };
  if (p.dbg & 2) return;
  // the last query block halved over the key chunks between two SIMD pairs, as in dK/dV
  const int nch = lk16 / 32 + ((lk16 & 16) ? 1 : 0);
  const int R = nqb - V2_THREADS / 64;
  const bool split = R >= 1 && R <= V2_THREADS / 64 && (R & 3) == 1 && nch >= 2;
  const int nwhole = split ? nqb - 1 : nqb;
  if (wave < nwhole) {
    f32x4 dq[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    qblock(wave, qn, don, on, true, 0, nch, dq);
    qstore(wave, dq);
  }
  for (int qbk = wave + V2_THREADS / 64; qbk < nwhole; qbk += V2_THREADS / 64) {
    X6Row<KCH> qr, dr, orr;
    x6_row_load<KCH>(qr, qb, p.q_st, (int64_t)qbk * 16 + li, p.Lq, lane, p.D);
    x6_row_load<KCH>(dr, dob, p.do_st, (int64_t)qbk * 16 + li, p.Lq, lane, p.D);
    x6_row_load<KCH>(orr, obp, p.o_st, (int64_t)qbk * 16 + li, p.Lq, lane, p.D);
    f32x4 dq[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    qblock(qbk, qr, dr, orr, true, 0, nch, dq);
    qstore(qbk, dq);
  }
  if (split) {
    const int sb = nqb - 1, hc = nch / 2;
    const bool own = wave == R - 1, part = wave == R;
    f32x4 dq[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (own || part) {
      X6Row<KCH> qr, dr, orr;
      x6_row_load<KCH>(qr, qb, p.q_st, (int64_t)sb * 16 + li, p.Lq, lane, p.D);
      x6_row_load<KCH>(dr, dob, p.do_st, (int64_t)sb * 16 + li, p.Lq, lane, p.D);
      x6_row_load<KCH>(orr, obp, p.o_st, (int64_t)sb * 16 + li, p.Lq, lane, p.D);
      qblock(sb, qr, dr, orr, own, own ? 0 : hc, own ? hc : nch, dq);
    }
    __syncthreads();  // every wave is done with the K / V images: reuse them for the exchange
    f32x4* xch = reinterpret_cast<f32x4*>(smem);
    if (part) {
#pragma unroll
      for (int d = 0; d < DT; ++d) xch[d * 64 + lane] = dq[d];
    }
    __syncthreads();
    if (own) {
#pragma unroll
      for (int d = 0; d < DT; ++d) dq[d] += xch[d * 64 + lane];
      qstore(sb, dq);
    }
  }
}

// the split-operand kernels take this call: fp32, no relative bias, D <= 64 in 16-B-pair chunks,
// both resident lengths within X6A_LMAX (bwd) / the key length (fwd)
bool x6_attn_ok(const mmfd_attn_args& a, bool bwd) {
  if (g_fp32_attn_mode != 1 || a.dtype != MMFD_F32 || a.rel_bias || a.cos_logit_scale) return false;
  if (a.D % 8 || a.D > 64) return false;
  if (v2_pad(a.Lk, 16) > X6A_LMAX || (bwd && v2_pad(a.Lq, 16) > X6A_LMAX)) return false;
  // dropout indices advanced in 32 bits (hash_c1)
  if (a.dropout_p > 0.f && (uint64_t)a.B * (uint64_t)a.H * (uint64_t)a.Lq * (uint64_t)a.Lk > (1ull << 32)) return false;
  return !g_attn_v1;
}

template <int D, bool DROP>
void launch_fwd_x6_d(const AttnP& p, hipStream_t s) {
  static bool once = (set_lds_attr(reinterpret_cast<const void*>(&attn_fwd_x6_kernel<D, DROP>), X6A_LDS), true);
  (void)once;
  const int lk16 = v2_pad(p.Lk, 16);
  hipLaunchKernelGGL((attn_fwd_x6_kernel<D, DROP>), dim3((unsigned)(p.B * p.H)), dim3(V2_THREADS),
                     6 * lk16 * X6A_RB + lk16 * 4, s, p);
}

constexpr int X6A_LDS_MAX = 160 * 1024;
// the dK/dV kernel's LDS, with the head's keep-bitmask rows when `dm`
int x6_dkdv_lds(const AttnP& p, bool dm) {
  const int lq16 = v2_pad(p.Lq, 16), lk16 = v2_pad(p.Lk, 16);
  return 6 * lq16 * X6A_RB + (2 * lq16 + lk16) * 4 + (dm ? lq16 * p.dmw * 4 : 0);
}

template <int D, int DQD, int DKD>
void launch_bwd_x6_d(const AttnP& p, hipStream_t s) {
  static bool once = (set_lds_attr(reinterpret_cast<const void*>(&attn_dkdv_x6_kernel<D, DKD>), X6A_LDS_MAX),
                      set_lds_attr(reinterpret_cast<const void*>(&attn_dq_x6_kernel<D, DQD>), X6A_LDS), true);
  (void)once;
  // dQ first: it computes delta = rowsum(dO * O) for dK/dV (no separate delta pass)
  const int lk16 = v2_pad(p.Lk, 16);
  hipLaunchKernelGGL((attn_dq_x6_kernel<D, DQD>), dim3((unsigned)(p.B * p.H)), dim3(V2_THREADS),
                     6 * lk16 * X6A_RB + lk16 * 4, s, p);
  hipLaunchKernelGGL((attn_dkdv_x6_kernel<D, DKD>), dim3((unsigned)(p.B * p.H)), dim3(V2_THREADS),
                     x6_dkdv_lds(p, DKD == 2), s, p);
}

// dropout as a template argument: a run-time flag let the compiler if-convert the hash into every
// chunk (its multiplies issued for dropout-free calls too)
void launch_fwd_x6(const AttnP& p, hipStream_t s) {
  const bool dr = p.p > 0.f;
  if (p.D > 32) { if (dr) launch_fwd_x6_d<64, true>(p, s); else launch_fwd_x6_d<64, false>(p, s); }
  else { if (dr) launch_fwd_x6_d<32, true>(p, s); else launch_fwd_x6_d<32, false>(p, s); }
}
// dropout in the backward: the forward's keep-bitmask when the caller kept one (dQ reads its row
// words from memory; dK/dV stages the head's rows in LDS when they fit beside its images, else
// re-hashes), otherwise the hash again
template <int D>
void launch_bwd_x6_dd(const AttnP& p, hipStream_t s) {
  if (p.p <= 0.f) return launch_bwd_x6_d<D, 0, 0>(p, s);
  if (!p.dm) return launch_bwd_x6_d<D, 1, 1>(p, s);
  if (x6_dkdv_lds(p, true) <= X6A_LDS_MAX) return launch_bwd_x6_d<D, 2, 2>(p, s);
  launch_bwd_x6_d<D, 2, 1>(p, s);
}
void launch_bwd_x6(const AttnP& p, hipStream_t s) {
  if (p.D > 32) launch_bwd_x6_dd<64>(p, s);
  else launch_bwd_x6_dd<32>(p, s);
}

int fill(const mmfd_attn_args& a, AttnP& p, bool bwd) {
  MMFD_CHECK_ARG(a.dtype == MMFD_F32 || a.dtype == MMFD_BF16, "attn: bad dtype");
  MMFD_CHECK_ARG(a.D > 0 && a.D <= 64, "attn: head_dim %lld unsupported (<= 64)", (long long)a.D);
  MMFD_CHECK_ARG(a.B >= 0 && a.H > 0 && a.Lq >= 0 && a.Lk > 0, "attn: bad shape");
  MMFD_CHECK_ARG(a.q && a.k && a.v && a.o && a.lse, "attn: null pointer");
  const int epc = a.dtype == MMFD_BF16 ? 8 : 4;
  MMFD_CHECK_ARG(a.D % epc == 0, "attn: head_dim*element_size must be a multiple of 16 bytes");
  auto al = [&](const void* ptr, int64_t sb, int64_t st) {
    return ((uintptr_t)ptr & 15) == 0 && sb % epc == 0 && st % epc == 0;
  };
  MMFD_CHECK_ARG(al(a.q, a.q_sb, a.q_st) && al(a.k, a.k_sb, a.k_st) && al(a.v, a.v_sb, a.v_st),
                 "attn: q/k/v must be 16-B aligned with strides multiple of 16 B");
  MMFD_CHECK_ARG(a.dropout_p <= 0.f || a.seed, "attn: dropout needs seed");
  MMFD_CHECK_ARG(a.dropout_p < 1.f, "attn: dropout p must be < 1");
  if (bwd) {
    MMFD_CHECK_ARG(a.dout && a.dq && a.dk && a.dv && a.delta, "attn_bwd: null pointer");
    MMFD_CHECK_ARG(al(a.dout, a.do_sb, a.do_st), "attn_bwd: dout alignment");
    MMFD_CHECK_ARG(a.d_rel_bias == nullptr, "attn_bwd: relative-bias gradient not supported");
    MMFD_CHECK_ARG(a.cos_logit_scale == nullptr, "attn_bwd: cosine attention is inference-only");
  }
  p.B = a.B; p.H = a.H; p.Lq = a.Lq; p.Lk = a.Lk; p.scale = a.scale; p.D = (int)a.D;
  p.q = a.q; p.q_sb = a.q_sb; p.q_st = a.q_st;
  p.k = a.k; p.k_sb = a.k_sb; p.k_st = a.k_st;
  p.v = a.v; p.v_sb = a.v_sb; p.v_st = a.v_st;
  p.o = a.o; p.o_sb = a.o_sb; p.o_st = a.o_st;
  p.lse = a.lse; p.key_bias = a.key_bias; p.rel_bias = a.rel_bias; p.rb_sb = a.rel_bias ? a.rel_bias_sb : 0;
  p.rb_mod = a.rel_bias ? a.rel_bias_mod : 0;
  p.cos_ls = a.cos_logit_scale; p.cos_max_log = a.cos_max_log;
  p.p = a.dropout_p > 0.f ? a.dropout_p : 0.f; p.thr16 = mmfd_drop_threshold16(p.p); p.kp = (a.Lk + 1) / 2;
  p.keep_scale = 1.0f / (1.0f - p.p); p.seed = a.seed; p.salt = a.salt;
  p.dout = a.dout; p.do_sb = a.do_sb; p.do_st = a.do_st;
  p.dq = a.dq; p.dq_sb = a.dq_sb; p.dq_st = a.dq_st;
  p.dk = a.dk; p.dk_sb = a.dk_sb; p.dk_st = a.dk_st;
  p.dv = a.dv; p.dv_sb = a.dv_sb; p.dv_st = a.dv_st;
  p.delta = a.delta;
  p.acc_dq = a.accumulate_dq; p.acc_dkv = a.accumulate_dkv;
  p.idx32 = (uint64_t)a.B * (uint64_t)a.H * (uint64_t)a.Lq * (uint64_t)a.Lk <= (1ull << 32);
  auto al4 = [](const void* ptr, int64_t sb, int64_t st) {
    return ptr && ((uintptr_t)ptr & 15) == 0 && sb % 4 == 0 && st % 4 == 0;
  };
  // (the forward keeps its per-element stores: the 4-column form measured 2-8 % slower there)
  p.vst = a.dtype == MMFD_F32 && bwd && al4(a.dq, a.dq_sb, a.dq_st) && al4(a.dk, a.dk_sb, a.dk_st) &&
          al4(a.dv, a.dv_sb, a.dv_st);
  p.pl = nullptr; p.pl_only = 0;
  static const int dbg = getenv("MMFD_X6A_DBG") ? atoi(getenv("MMFD_X6A_DBG")) : 0;
  p.dbg = dbg;
  p.dm = p.p > 0.f ? a.drop_mask : nullptr;
  p.dmw = (int)((a.Lk + 31) / 32);
  p.dm_lds = 0;
  MMFD_CHECK_ARG(!p.dm || ((uintptr_t)p.dm & 3) == 0, "attn: drop_mask must be 4-B aligned");
  return 0;
}

// the keep-bitmask from the hash, for forward kernels that do not write it (the streaming v1 path)
__global__ void dm_fill_kernel(AttnP p) {
  const int64_t words = p.B * p.H * p.Lq * p.dmw;
  const uint32_t hkey = mmfd_hash_key(*p.seed, p.salt);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / p.dmw, w = i - row * p.dmw;  // row = bh * Lq + q
    uint32_t bits = 0;
    for (int j = 0; j < 32; j += 2) {  // one hash per key pair (k even, k + 1)
      const int64_t k = w * 32 + j;
      if (k >= p.Lk) break;
      const uint32_t hsh = attn_hash64(hkey, p, row, k);
      if (pair_keep(hsh, 0, p.thr16)) bits |= 1u << j;
      if (k + 1 < p.Lk && pair_keep(hsh, 1, p.thr16)) bits |= 1u << (j + 1);
    }
    p.dm[i] = bits;
  }
}

template <typename T, int D, int HPB, bool REL, int MODE>
void launch_fwd_v2_hpb(const AttnP& p, hipStream_t s) {
  constexpr int RB = AT<T, D>::RB;
  const int lk_pad = v2_pad(p.Lk, v2_kc<T>());
  const int lds = HPB * (2 * lk_pad * RB + lk_pad * 4);
  constexpr int lmax = HPB == 1 ? (sizeof(T) == 2 ? V2_LMAX_FWD : V2_LMAX) : 64;
  static bool once = (set_lds_attr(reinterpret_cast<const void*>(&attn_fwd_v2_kernel<T, D, HPB, REL, MODE>),
                                   HPB * (2 * lmax * RB + lmax * 4)), true);
  (void)once;
  const int64_t nbh = p.B * p.H;
  hipLaunchKernelGGL((attn_fwd_v2_kernel<T, D, HPB, REL, MODE>), dim3((unsigned)((nbh + HPB - 1) / HPB)),
                     dim3(V2_THREADS), lds, s, p);
}

// the fixed v2 mode for these arguments (see V2_RESCALE_TH): 1 plain, 2 hashed dropout with or
// without a key bias (the per-key bias vector is staged either way: 0 for real keys when there is
// none, -inf for the padding — round 6: the fusion head's dropout-only attention had run the
// generic mode at ~50 VALU instructions per MFMA), 0 anything else (relative bias, keep-bitmask,
// a key bias without dropout)
inline int v2_mode(const AttnP& p) {
  if (p.rel_bias || g_v2_generic) return 0;
  if (p.p == 0.f && !p.key_bias) return 1;
  if (p.p > 0.f && !p.dm) return 2;
  return 0;
}

// the relative-bias instantiation carries the extra loads / registers; plain attention (BERT, ViT,
// fusion head) keeps the bias-free one
template <typename T, int D, int HPB>
void launch_fwd_v2_hpb(const AttnP& p, hipStream_t s) {
  if (p.rel_bias) {
    launch_fwd_v2_hpb<T, D, HPB, true, 0>(p, s);
  } else if constexpr (HPB == 1) {
    const int mode = v2_mode(p);
    if (mode == 1) launch_fwd_v2_hpb<T, D, 1, false, 1>(p, s);
    else if (mode == 2) launch_fwd_v2_hpb<T, D, 1, false, 2>(p, s);
    else launch_fwd_v2_hpb<T, D, 1, false, 0>(p, s);
  } else {
    launch_fwd_v2_hpb<T, D, HPB, false, 0>(p, s);
  }
}

template <typename T, int D>
void launch_fwd_v2(const AttnP& p, hipStream_t s) {
  // short windows: several heads per workgroup so all 8 waves own a 16-query block
  if (p.Lk <= 64 && p.Lq <= 32)
    launch_fwd_v2_hpb<T, D, 4>(p, s);
  else if (p.Lk <= 64 && p.Lq <= 64)
    launch_fwd_v2_hpb<T, D, 2>(p, s);
  else
    launch_fwd_v2_hpb<T, D, 1>(p, s);
}

template <typename T, int D, bool REL, int MODE>
void launch_bwd_v2_rel(const AttnP& p, hipStream_t s) {
  constexpr int RB = AT<T, D>::RB, NTH = V2T<T>::DKDV_THREADS;
  const int lq_pad = v2_pad(p.Lq, v2_kc<T>()), lk_pad = v2_pad(p.Lk, v2_kc<T>());
  constexpr int NI1 = V2<T, D>::DUAL ? 2 : 4, NI2 = V2<T, D>::DUAL ? 2 : 3;  // LDS images per kernel
  const int lds1n = NI1 * lq_pad * RB + 3 * V2_LMAX * 4;
  const int lds2 = NI2 * lk_pad * RB + lk_pad * 4;
  constexpr int lds1_max = NI1 * V2_LMAX * RB + 3 * V2_LMAX * 4 + V2_LMAX * (V2_LMAX / 32) * 4;
  static_assert(lds1_max <= 160 * 1024, "dK/dV LDS");
  AttnP q = p;  // dK/dV stages the head's keep-bitmask rows in LDS when the caller kept them
  q.dm_lds = p.p > 0.f && p.dm && lds1n + lq_pad * p.dmw * 4 <= lds1_max;
  const int lds1 = lds1n + (q.dm_lds ? lq_pad * p.dmw * 4 : 0);
  static bool once = (set_lds_attr(reinterpret_cast<const void*>(&attn_dkdv_v2_kernel<T, D, NTH, REL, MODE>), lds1_max),
                      set_lds_attr(reinterpret_cast<const void*>(&attn_dq_v2_kernel<T, D, REL, MODE>),
                                   NI2 * V2_LMAX * RB + V2_LMAX * 4),
                      true);
  (void)once;
  // dQ first: it writes delta = rowsum(dO * O) for dK/dV (no separate delta pass)
  hipLaunchKernelGGL((attn_dq_v2_kernel<T, D, REL, MODE>), dim3((unsigned)(p.B * p.H)), dim3(V2_THREADS), lds2, s, q);
  hipLaunchKernelGGL((attn_dkdv_v2_kernel<T, D, NTH, REL, MODE>), dim3((unsigned)(p.B * p.H)), dim3(NTH), lds1, s, q);
}

template <typename T, int D>
void launch_bwd_v2(const AttnP& p, hipStream_t s) {
  const int mode = v2_mode(p);
  if (p.rel_bias) launch_bwd_v2_rel<T, D, true, 0>(p, s);
  else if (mode == 1) launch_bwd_v2_rel<T, D, false, 1>(p, s);
  else if (mode == 2) launch_bwd_v2_rel<T, D, false, 2>(p, s);
  else launch_bwd_v2_rel<T, D, false, 0>(p, s);
}

template <typename T, int D>
void launch_fwd(const AttnP& p, hipStream_t s) {
  dim3 grid((unsigned)((p.Lq + 63) / 64), (unsigned)(p.B * p.H));
  constexpr int lds = 2 * AT<T, D>::TILE;
  hipLaunchKernelGGL((attn_fwd_kernel<T, D>), grid, dim3(256), lds, s, p);
}
template <typename T, int D>
void launch_bwd(const AttnP& p, hipStream_t s) {
  const int64_t rows = p.B * p.H * p.Lq;
  constexpr int nch = AT<T, D>::NCH;
  constexpr int lds1 = 4 * AT<T, D>::TILE + 512;
  constexpr int lds2 = 3 * AT<T, D>::TILE;
  const int64_t threads = rows * nch;
  hipLaunchKernelGGL((attn_delta_kernel<T, D>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, p);
  dim3 g1((unsigned)((p.Lk + 63) / 64), (unsigned)(p.B * p.H));
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<T, D>), g1, dim3(256), lds1, s, p);
  dim3 g2((unsigned)((p.Lq + 63) / 64), (unsigned)(p.B * p.H));
  hipLaunchKernelGGL((attn_bwd_dq_kernel<T, D>), g2, dim3(256), lds2, s, p);
}

}  // namespace

extern "C" int mmfd_attn_fwd(const mmfd_attn_args* a, mmfd_stream_t stream) {
  MMFD_CHECK_STRUCT(a, mmfd_attn_args, "mmfd_attn_fwd");
  AttnP p;
  int rc = fill(*a, p, false);
  if (rc) return rc;
  if (p.B == 0 || p.Lq == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  // one workgroup per (b, h): past 256 keys only when there are enough heads to fill the chip (a
  // batch-1 pair at L = 512 runs faster on the 64-query-block streaming kernel)
  // (fp32 K/V images of 512 keys would not fit the LDS)
  const bool bf = a->dtype == MMFD_BF16;
  const bool x6 = x6_attn_ok(*a, false);
  const bool v2 = x6 || ((p.Lk <= V2_LMAX || (bf && p.Lk <= V2_LMAX_FWD && p.B * p.H >= 256)) && !g_attn_v1);
  MMFD_CHECK_ARG(!a->cos_logit_scale || (v2 && bf && a->rel_bias),
                 "attn_fwd: cosine attention needs bf16, the resident-K/V kernel (Lk <= 256) and a rel_bias");
  p.pl = nullptr; p.pl_only = 0;
  const int64_t W = a->H * a->D;
  if (a->o_planes) {
    MMFD_CHECK_ARG(!bf && a->o_st == W && a->o_sb == a->Lq * W && W % 8 == 0,
                   "attn_fwd: o_planes need an fp32 output in one contiguous [B, Lq, H*D] buffer");
    if (v2) { p.pl = (bf16*)a->o_planes; p.pl_stride = p.B * p.Lq * W; p.pl_base = (const float*)a->o; }
  }
  if (x6) launch_fwd_x6(p, s);
  else if (v2 && bf) { if (a->D > 32) launch_fwd_v2<bf16, 64>(p, s); else launch_fwd_v2<bf16, 32>(p, s); }
  else if (v2) { if (a->D > 32) launch_fwd_v2<float, 64>(p, s); else launch_fwd_v2<float, 32>(p, s); }
  else if (a->dtype == MMFD_BF16) { if (a->D > 32) launch_fwd<bf16, 64>(p, s); else launch_fwd<bf16, 32>(p, s); }
  else { if (a->D > 32) launch_fwd<float, 64>(p, s); else launch_fwd<float, 32>(p, s); }
  MMFD_CHECK_LAUNCH("attn_fwd");
  if (p.dm && !v2) {  // the streaming kernels hash without writing the mask: fill it for the backward
    const int64_t words = p.B * p.H * p.Lq * p.dmw;
    hipLaunchKernelGGL(dm_fill_kernel, dim3((unsigned)std::min<int64_t>((words + 255) / 256, 8192)), dim3(256), 0, s, p);
    MMFD_CHECK_LAUNCH("attn_fwd dm_fill");
  }
  if (a->o_planes && !v2)  // the streaming kernels write fp32 only: split afterwards
    return mmfd_split3(p.B * p.Lq, W, (const float*)a->o, W, a->o_planes, stream);
  return 0;
}

extern "C" int mmfd_attn_bwd(const mmfd_attn_args* a, mmfd_stream_t stream) {
  MMFD_CHECK_STRUCT(a, mmfd_attn_args, "mmfd_attn_bwd");
  AttnP p;
  int rc = fill(*a, p, true);
  if (rc) return rc;
  if (p.B == 0 || p.Lq == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool x6 = x6_attn_ok(*a, true);
  const bool v2 = x6 || (p.Lk <= V2_LMAX && p.Lq <= V2_LMAX && !g_attn_v1);
  p.pl = nullptr; p.pl_only = 0;
  const int64_t W = 3 * a->H * a->D;
  if (a->dqkv_planes) {
    MMFD_CHECK_ARG(a->dtype == MMFD_F32 && a->Lq == a->Lk && a->dk == (const float*)a->dq + a->H * a->D &&
                       a->dv == (const float*)a->dq + 2 * a->H * a->D && a->dq_st == W && a->dk_st == W &&
                       a->dv_st == W && a->dq_sb == a->Lq * W && a->dk_sb == a->dq_sb && a->dv_sb == a->dq_sb,
                   "attn_bwd: dqkv_planes need fp32 dq | dk | dv packed in one contiguous [B, L, 3*H*D] buffer");
    MMFD_CHECK_ARG(!a->planes_only || (!a->accumulate_dq && !a->accumulate_dkv),
                   "attn_bwd: planes_only excludes accumulate");
    if (v2) {  // the v2 kernels write the planes from their stores
      p.pl = (bf16*)a->dqkv_planes; p.pl_stride = p.B * p.Lq * W; p.pl_base = (const float*)a->dq;
      if ((uintptr_t)p.pl & 7) p.vst = 0;
      p.pl_only = a->planes_only;
    }
  }
  if (x6) launch_bwd_x6(p, s);
  else if (v2 && a->dtype == MMFD_BF16) { if (a->D > 32) launch_bwd_v2<bf16, 64>(p, s); else launch_bwd_v2<bf16, 32>(p, s); }
  else if (v2) { if (a->D > 32) launch_bwd_v2<float, 64>(p, s); else launch_bwd_v2<float, 32>(p, s); }
  else if (a->dtype == MMFD_BF16) { if (a->D > 32) launch_bwd<bf16, 64>(p, s); else launch_bwd<bf16, 32>(p, s); }
  else { if (a->D > 32) launch_bwd<float, 64>(p, s); else launch_bwd<float, 32>(p, s); }
  MMFD_CHECK_LAUNCH("attn_bwd");
  if (a->dqkv_planes && !v2)  // the v1 kernels write fp32 only: split afterwards
    return mmfd_split3(p.B * p.Lq, W, (const float*)a->dq, W, a->dqkv_planes, stream);
  return 0;
}

// A/B switch for the fixed v2 modes (not part of include/mmfd.h): returns the old value
extern "C" int mmfd_debug_set_attn_v2_generic(int on) {
  const int old = g_v2_generic;
  g_v2_generic = on ? 1 : 0;
  return old;
}

extern "C" int mmfd_set_fp32_attn_mode(int mode) {
  MMFD_CHECK_ARG(mode == 0 || mode == 1, "mmfd_set_fp32_attn_mode: mode %d (0 = fp32 MFMA, 1 = split operands)", mode);
  const int old = g_fp32_attn_mode;
  g_fp32_attn_mode = mode;
  return old;
}

#ifdef MMFD_X6A_STAMPS
extern "C" int mmfd_debug_x6a_stamps(void* host_dst, int64_t bytes) {
  return (int)hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(x6a_stamps), (size_t)bytes, 0, hipMemcpyDeviceToHost);
}
#endif
