// Evidence retrieval scoring for gfx950: cosine similarity of a batch of queries against a
// device-resident corpus, and an exact top-k (descending score, ties -> lower corpus index first,
// i.e. the order of Python's stable sort over the reference's insertion-ordered dict).
//
// Reference: ImageCorpus.retrieve_similar_images (src/evidence/im2im_retrieval.py:80-106: one
// nn.CosineSimilarity(dim=1, eps=1e-6) call per corpus image in a Python loop, then sorted(...,
// reverse=True)) and SemanticSimilarity.search (src/evidence/text2text_retrieval.py:49-66:
// sentence_transformers.util.semantic_search over fp16 embeddings, top_k*5 hits per corpus).
//
// Scores are HBM-bound: every corpus row is read once per pass of up to QT queries (row-blocked
// GEMV; the query tile sits in LDS, each lane streams 16-B chunks of R rows and reuses every LDS
// query chunk R times). The row's squared norm is accumulated in the same pass. Top-k is a radix
// select, one workgroup per query (see topk_radix_kernel).
#include "common.h"
#include <algorithm>

namespace {

typedef _Float16 f16;

constexpr int CS_THREADS = 256;  // 4 waves
constexpr int CS_R = 4;          // corpus rows per wave per step
constexpr int CS_QT = 8;         // queries per pass

template <typename T> struct Chunk;  // one 16-B chunk of a corpus row, as fp32
template <> struct Chunk<float> {
  static constexpr int E = 4;
  __device__ __forceinline__ static void load(const float* p, float (&x)[8]) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
};
template <> struct Chunk<bf16> {
  static constexpr int E = 8;
  __device__ __forceinline__ static void load(const bf16* p, float (&x)[8]) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { x[2 * i] = __uint_as_float(w[i] << 16); x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
  }
};
template <> struct Chunk<f16> {
  static constexpr int E = 8;
  __device__ __forceinline__ static void load(const f16* p, float (&x)[8]) {
    typedef __attribute__((ext_vector_type(8))) _Float16 h8;
    const h8 v = *reinterpret_cast<const h8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (float)v[i];
  }
};

__device__ __forceinline__ float cos_finish(float dot, float qq, float cc, int mode, float eps) {
  float s;
  if ((mode & 3) == MMFD_COS_PAIR) {
    s = dot / sqrtf(fmaxf(qq * cc, eps * eps));
  } else {
    s = dot / (fmaxf(sqrtf(qq), eps) * fmaxf(sqrtf(cc), eps));
  }
  if (mode & MMFD_COS_ROUND_F16) s = (float)(f16)s;
  return s;
}

// grid.x = row blocks; each of the 4 waves takes CS_R rows per step, CS_QT queries per launch
// (the host launches one pass per query tile). D % E == 0 and 16-B aligned rows (host-checked).
template <typename T>
__global__ void __launch_bounds__(CS_THREADS) cosine_scores_kernel(int64_t N, int64_t D, int nq,
                                                                   const float* __restrict__ q, int64_t ldq,
                                                                   const T* __restrict__ c, int64_t ldc, int mode,
                                                                   float eps, float* __restrict__ out, int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) float qs[];  // [nq][D] + [CS_QT] squared norms
  float* qn = qs + (int64_t)nq * D;
  for (int64_t i = threadIdx.x; i < (int64_t)nq * D; i += CS_THREADS) {
    const int j = (int)(i / D);
    qs[i] = q[(int64_t)j * ldq + (i - (int64_t)j * D)];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave == 0) {
    for (int j = 0; j < nq; ++j) {
      float s = 0.f;
      for (int64_t d = lane; d < D; d += 64) s = fmaf(qs[j * D + d], qs[j * D + d], s);
      s = wave_sum(s);
      if (lane == 0) qn[j] = s;
    }
  }
  __syncthreads();
  constexpr int E = Chunk<T>::E;
  const int64_t nchunk = D / E;
  const int64_t rows_per_block = 4 * CS_R;
  for (int64_t r0 = (int64_t)blockIdx.x * rows_per_block + wave * CS_R; r0 < N; r0 += (int64_t)gridDim.x * rows_per_block) {
    float acc[CS_R][CS_QT], sq[CS_R];
#pragma unroll
    for (int r = 0; r < CS_R; ++r) {
      sq[r] = 0.f;
#pragma unroll
      for (int j = 0; j < CS_QT; ++j) acc[r][j] = 0.f;
    }
#pragma unroll 2
    for (int64_t ch = lane; ch < nchunk; ch += 64) {
      float x[CS_R][8];
#pragma unroll
      for (int r = 0; r < CS_R; ++r) {
        const int64_t row = min(r0 + r, N - 1);  // clamped rows are computed and discarded
        Chunk<T>::load(c + row * ldc + ch * E, x[r]);
      }
#pragma unroll
      for (int r = 0; r < CS_R; ++r)
#pragma unroll
        for (int e = 0; e < E; ++e) sq[r] = fmaf(x[r][e], x[r][e], sq[r]);
#pragma unroll
      for (int j = 0; j < CS_QT; ++j) {
        if (j >= nq) break;
        float qv[8];
        const float4 a = *reinterpret_cast<const float4*>(qs + j * D + ch * E);
        qv[0] = a.x; qv[1] = a.y; qv[2] = a.z; qv[3] = a.w;
        if (E == 8) {
          const float4 b = *reinterpret_cast<const float4*>(qs + j * D + ch * E + 4);
          qv[4] = b.x; qv[5] = b.y; qv[6] = b.z; qv[7] = b.w;
        }
#pragma unroll
        for (int r = 0; r < CS_R; ++r)
#pragma unroll
          for (int e = 0; e < E; ++e) acc[r][j] = fmaf(x[r][e], qv[e], acc[r][j]);
      }
    }
#pragma unroll
    for (int r = 0; r < CS_R; ++r) {
      const float cc = wave_sum(sq[r]);
#pragma unroll
      for (int j = 0; j < CS_QT; ++j) {
        if (j >= nq) break;
        const float dot = wave_sum(acc[r][j]);
        if (lane == 0 && r0 + r < N) out[(int64_t)j * ldo + r0 + r] = cos_finish(dot, qn[j], cc, mode, eps);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// top-k: one 1024-thread workgroup per query (radix select, exact)
//   1. four 8-bit digit passes over the order-preserving score bits (LDS histograms, wave-scan of
//      the 256 bins from the top) find T = the bits of the k-th largest score and kr = how many
//      elements equal to T belong to the top k;
//   2. a collect pass keeps every element above T and the kr LOWEST-index elements equal to T
//      (an index-ordered block scan, only when T is tied beyond kr);
//   3. the k candidates are sorted in LDS by 64-bit key (score bits | ~index), descending.
// ---------------------------------------------------------------------------------------------
constexpr int TK_THREADS = 1024;
constexpr int TK_MAXK = 2048;

// order-preserving map of fp32 to uint32 (larger float -> larger integer)
__device__ __forceinline__ uint32_t ord_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_bits(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
// key: descending key order == descending score, then ascending index
__device__ __forceinline__ uint64_t make_key(uint32_t ord, uint32_t idx) {
  return ((uint64_t)ord << 32) | (uint64_t)(0xffffffffu - idx);
}

__global__ void __launch_bounds__(TK_THREADS) topk_radix_kernel(int64_t N, const float* __restrict__ scores,
                                                                int64_t lds, int k, float* __restrict__ out_val,
                                                                int64_t* __restrict__ out_idx) {
  // 16 replicas of the 256 bins (replica = lane & 15, bin-major: the replicas of a bin sit in 16
  // different banks), so that the lanes of a wave hitting the same bin do not serialise
  __shared__ uint32_t hist[256 * 16];
  __shared__ uint32_t wsum[TK_THREADS / 64];
  __shared__ uint32_t wmin[TK_THREADS / 64], wmax[TK_THREADS / 64];
  __shared__ uint32_t s_prefix, s_kr, s_eq, s_ngt, s_neq;
  __shared__ uint64_t cand[TK_MAXK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* __restrict__ s = scores + (int64_t)blockIdx.x * lds;
  const int kk = (int)min((int64_t)k, N);
  // bits shared by every element need no digit pass: start below the common prefix of min / max
  uint32_t lo = 0xffffffffu, hi = 0u;
  for (int64_t i = tid; i < N; i += TK_THREADS) {
    const uint32_t u = ord_bits(s[i]);
    lo = min(lo, u);
    hi = max(hi, u);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64));
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
  }
  if (lane == 0) { wmin[wave] = lo; wmax[wave] = hi; }
  __syncthreads();
  lo = wmin[0]; hi = wmax[0];
  for (int w = 1; w < TK_THREADS / 64; ++w) { lo = min(lo, wmin[w]); hi = max(hi, wmax[w]); }
  const int common = (lo == hi) ? 32 : __clz((int)(lo ^ hi));
  uint32_t mask = common == 0 ? 0u : (common == 32 ? 0xffffffffu : (0xffffffffu << (32 - common)));
  uint32_t prefix = lo & mask, kr = (uint32_t)kk, eq_total = (uint32_t)N;
  for (int r = 32 - common; r > 0;) {
    const int wdt = min(8, r), shift = r - wdt;
    const uint32_t dmask = (1u << wdt) - 1u;
    for (int i = tid; i < 256 * 16; i += TK_THREADS) hist[i] = 0;
    __syncthreads();
    // 8 independent loads in flight per thread before the LDS atomics
    for (int64_t i0 = 0; i0 < N; i0 += 8 * TK_THREADS) {
      uint32_t u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t i = i0 + j * TK_THREADS + tid;
        u[j] = i < N ? ord_bits(s[i]) : 0u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (i0 + j * TK_THREADS + tid < N && (u[j] & mask) == prefix)
          atomicAdd(&hist[((u[j] >> shift) & dmask) * 16 + (lane & 15)], 1u);
    }
    __syncthreads();
    if (wave == 0) {  // lane l owns bins 255-4l .. 252-4l (scanned from the top)
      uint32_t c[4], tot = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int bin = 255 - 4 * lane - j;
        uint32_t v = 0;
#pragma unroll
        for (int rep = 0; rep < 16; ++rep) v += hist[bin * 16 + ((rep + lane) & 15)];
        c[j] = v;
        tot += v;
      }
      uint32_t incl = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
      }
      const uint32_t excl = incl - tot;
      const uint64_t hit = __ballot(incl >= kr);
      const int first = __ffsll((long long)hit) - 1;  // lane holding the selected bin
      if (lane == first) {
        uint32_t cum = excl;
        int j = 0;
        while (cum + c[j] < kr) { cum += c[j]; ++j; }
        const uint32_t bin = 255u - 4u * lane - j;
        s_prefix = prefix | (bin << shift);
        s_kr = kr - cum;
        s_eq = c[j];
      }
    }
    __syncthreads();
    prefix = s_prefix;
    mask |= dmask << shift;
    kr = s_kr;
    eq_total = s_eq;
    r = shift;
  }
  // collect: all elements above T, and the kr lowest-index ones equal to T
  const uint32_t T = prefix;
  if (tid == 0) { s_ngt = 0; s_neq = 0; }
  __syncthreads();
  const uint32_t n_above = (uint32_t)kk - kr;
  const bool cut = eq_total > kr;  // ties at T beyond the k-th: index order decides
  uint32_t eq_base = 0;
  if (!cut) {  // every element at or above T is taken: no ordering needed while collecting
    for (int64_t i0 = 0; i0 < N; i0 += 8 * TK_THREADS) {
      uint32_t u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t i = i0 + j * TK_THREADS + tid;
        u[j] = i < N ? ord_bits(s[i]) : 0u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t i = i0 + j * TK_THREADS + tid;
        if (i < N && u[j] > T) cand[atomicAdd(&s_ngt, 1u)] = make_key(u[j], (uint32_t)i);
        else if (i < N && u[j] == T) cand[n_above + atomicAdd(&s_neq, 1u)] = make_key(u[j], (uint32_t)i);
      }
    }
  }
  for (int64_t c0 = 0; cut && c0 < N; c0 += TK_THREADS) {
    const int64_t i = c0 + tid;
    const uint32_t u = i < N ? ord_bits(s[i]) : 0u;
    const bool gt = i < N && u > T, eq = i < N && u == T;
    if (gt) cand[atomicAdd(&s_ngt, 1u)] = make_key(u, (uint32_t)i);
    {
      const uint64_t m = __ballot(eq);
      if (lane == 0) wsum[wave] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t before = 0, chunk = 0;
      for (int w = 0; w < TK_THREADS / 64; ++w) { if (w < wave) before += wsum[w]; chunk += wsum[w]; }
      const uint32_t rank = eq_base + before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      if (eq && rank < kr) cand[n_above + rank] = make_key(u, (uint32_t)i);
      eq_base += chunk;
      __syncthreads();
      if (eq_base >= kr && c0 + TK_THREADS < N) {
        // every remaining element above T still has to be gathered
        for (int64_t j = c0 + TK_THREADS + tid; j < N; j += TK_THREADS) {
          const uint32_t v = ord_bits(s[j]);
          if (v > T) cand[atomicAdd(&s_ngt, 1u)] = make_key(v, (uint32_t)j);
        }
        break;
      }
    }
  }
  __syncthreads();
  // bitonic sort of the kk candidates (padded with 0 keys) to the next power of two, descending
  int P = 1;
  while (P < kk) P <<= 1;
  for (int i = kk + tid; i < P; i += TK_THREADS) cand[i] = 0ull;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = tid; t < P / 2; t += TK_THREADS) {
        const int i = 2 * stride * (t / stride) + (t % stride), j = i + stride;
        const bool desc = ((i & size) == 0);
        const uint64_t x = cand[i], y = cand[j];
        if ((x < y) == desc) { cand[i] = y; cand[j] = x; }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < k; i += TK_THREADS) {
    const int64_t o = (int64_t)blockIdx.x * k + i;
    if (i < kk) {
      const uint64_t key = cand[i];
      out_val[o] = unord_bits((uint32_t)(key >> 32));
      out_idx[o] = (int64_t)(0xffffffffu - (uint32_t)key);
    } else {  // fewer than k elements
      out_val[o] = -INFINITY;
      out_idx[o] = -1;
    }
  }
}

}  // namespace

extern "C" int mmfd_cosine_scores(int corpus_dtype, int64_t Q, int64_t N, int64_t D, const float* queries,
                                  int64_t ldq, const void* corpus, int64_t ldc, int mode, float eps,
                                  float* scores, int64_t lds, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(corpus_dtype == MMFD_F32 || corpus_dtype == MMFD_BF16 || corpus_dtype == MMFD_F16,
                 "mmfd_cosine_scores: bad corpus dtype %d", corpus_dtype);
  MMFD_CHECK_ARG(Q >= 0 && N >= 0 && D > 0, "mmfd_cosine_scores: bad shape");
  MMFD_CHECK_ARG((mode & 3) == MMFD_COS_PAIR || (mode & 3) == MMFD_COS_NORMALIZED, "mmfd_cosine_scores: bad mode %d", mode);
  if (Q == 0 || N == 0) return 0;
  const int E = corpus_dtype == MMFD_F32 ? 4 : 8;
  const int64_t esz = corpus_dtype == MMFD_F32 ? 4 : 2;
  MMFD_CHECK_ARG(D % 8 == 0 && ldc % E == 0 && ldq >= D && ldc >= D && lds >= N,
                 "mmfd_cosine_scores: D and ldc must be multiples of 8 / 16 bytes");
  MMFD_CHECK_ARG(((uintptr_t)corpus & 15) == 0 && ((uintptr_t)queries & 3) == 0,
                 "mmfd_cosine_scores: corpus must be 16-byte aligned");
  MMFD_CHECK_ARG(((int64_t)CS_QT * D + CS_QT) * 4 <= 160 * 1024, "mmfd_cosine_scores: D=%lld too large", (long long)D);
  (void)esz;
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows_per_block = 4 * CS_R;
  // ~4 blocks per CU: each block stages its query tile once and then streams many rows
  const int blocks = (int)std::min<int64_t>((N + rows_per_block - 1) / rows_per_block, 1024);
  for (int64_t q0 = 0; q0 < Q; q0 += CS_QT) {
    const int nq = (int)std::min<int64_t>(CS_QT, Q - q0);
    const int64_t smem = ((int64_t)nq * D + CS_QT) * 4;
    const float* qp = queries + q0 * ldq;
    float* op = scores + q0 * lds;
#define LAUNCH(T)                                                                                     \
  do {                                                                                                \
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&cosine_scores_kernel<T>),   \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == \
                       hipSuccess;                                                                    \
    (void)attr;                                                                                       \
    hipLaunchKernelGGL((cosine_scores_kernel<T>), dim3(blocks), dim3(CS_THREADS), (size_t)smem, s, N, D, nq, qp, ldq, \
                       (const T*)corpus, ldc, mode, eps, op, lds);                                    \
  } while (0)
    if (corpus_dtype == MMFD_F32) LAUNCH(float);
    else if (corpus_dtype == MMFD_BF16) LAUNCH(bf16);
    else LAUNCH(f16);
#undef LAUNCH
    MMFD_CHECK_LAUNCH("cosine_scores");
  }
  return 0;
}

extern "C" int64_t mmfd_topk_workspace_bytes(int64_t Q, int64_t N, int64_t k) {
  (void)Q; (void)N; (void)k;
  return 0;  // the radix select keeps everything in LDS
}

extern "C" int mmfd_topk(int64_t Q, int64_t N, const float* scores, int64_t lds, int64_t k, float* out_val,
                         int64_t* out_idx, void* workspace, int64_t workspace_bytes, mmfd_stream_t stream) {
  (void)workspace; (void)workspace_bytes;
  MMFD_CHECK_ARG(Q >= 0 && N >= 0 && k >= 0 && lds >= N, "mmfd_topk: bad shape");
  MMFD_CHECK_ARG(k <= TK_MAXK, "mmfd_topk: k=%lld > %d", (long long)k, TK_MAXK);
  MMFD_CHECK_ARG(N < 0xffffffffll, "mmfd_topk: N too large");
  if (Q == 0 || k == 0) return 0;
  MMFD_CHECK_ARG(N > 0, "mmfd_topk: empty corpus");
  MMFD_CHECK_ARG(Q <= 0x7fffffffll, "mmfd_topk: Q too large");
  hipLaunchKernelGGL(topk_radix_kernel, dim3((unsigned)Q), dim3(TK_THREADS), 0, (hipStream_t)stream, N, scores, lds,
                     (int)k, out_val, out_idx);
  MMFD_CHECK_LAUNCH("topk_radix");
  return 0;
}
