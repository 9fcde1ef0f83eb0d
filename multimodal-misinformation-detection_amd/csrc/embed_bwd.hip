// BERT embedding backward: the gradient of the pre-LayerNorm sum (word + position + token type,
// modeling_bert.py BertEmbeddings.forward) scattered into the three tables — deterministically.
//
// The word table is a scatter-add over repeated token ids. Since round 5 it is no longer done with
// fp32 atomics (whose order, and so the last bits of the result, changed from run to run): the
// token rows are stably radix-sorted by id (rocPRIM, over the id bits of the vocabulary only:
// 15 for BERT's 30,522 rows, two 8-bit digit passes instead of four), each id's rows are summed in row order in
// pieces of at most kSegChunk sorted rows, and the pieces are added in order by a single writer
// per table row. The
// token-type table (two rows) sums fixed row slabs into workspace partials and reduces the slabs in
// slab order; the position table sums over the batch in batch order. Same inputs, same bits —
// which the graph-captured data-parallel step's self-check (mmfd.dp, tests/test_dp_gpu.py) relies on.
#include "common.h"
#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>

namespace {
constexpr int kTypeSlabs = 1024;

inline unsigned gridn(int64_t n, int per) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, 16384));
}
inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// keys = token ids (as u32: ids are table rows, < 2^32), values = row numbers
__global__ void embed_sort_prep_kernel(int64_t rows, const int64_t* __restrict__ ids, uint32_t* __restrict__ keys,
                                       int32_t* __restrict__ vals) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    keys[r] = (uint32_t)ids[r];
    vals[r] = (int32_t)r;
  }
}

// The sorted positions are cut into chunks of kSegChunk; one wavefront per chunk walks its runs of
// equal ids and sums each run's rows in row order (the sort is stable). A run wholly inside the chunk
// is added to its table row directly (its only writer); the pieces of a run that crosses chunk
// boundaries go to per-chunk partials — part_last[c] for the piece a run starts with at the end
// of chunk c, part_first[c] for the piece that continues a run from chunk c - 1 — and
// embed_word_join_kernel adds them in chunk order. A repeated id ([CLS], [SEP], "the") costs
// ceil(count / kSegChunk) parallel pieces and one short ordered join, not a serial walk.
constexpr int kSegChunk = 32;

// one 256-thread block per chunk (thread t owns columns t + 256 u): 32 rows' loads per thread in
// flight across the unrolled row loop, 4 waves per chunk
template <typename T>
__global__ void __launch_bounds__(256) embed_word_segsum_kernel(int64_t rows, int64_t D, const uint32_t* __restrict__ keys,
                                                                const int32_t* __restrict__ vals, const T* __restrict__ dsum,
                                                                float* __restrict__ dword, float* __restrict__ part_first,
                                                                float* __restrict__ part_last, int64_t padding_idx) {
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t i0 = c * kSegChunk;
  const int64_t i1 = i0 + kSegChunk < rows ? i0 + kSegChunk : rows;
  for (int64_t s = i0; s < i1;) {
    const uint32_t key = keys[s];
    int64_t e = s + 1;
    while (e < i1 && keys[e] == key) ++e;
    const bool before = s == i0 && i0 > 0 && keys[i0 - 1] == key;
    const bool after = e == i1 && i1 < rows && keys[i1] == key;
    const bool pad = (int64_t)key == padding_idx;
    if (!pad || before || after) {
      float* dst = before ? part_first + c * D : after ? part_last + c * D : dword + (int64_t)key * D;
      for (int64_t d0 = 0; d0 < D; d0 += 1024) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
        for (int64_t j = s; j < e; ++j) {
          const T* src = dsum + (int64_t)vals[j] * D + d0 + t;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (d0 + t + 256 * u < D) acc[u] += to_f32(src[256 * u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t d = d0 + t + 256 * u;
          if (d < D) {
            if (before || after) dst[d] = acc[u];
            else dst[d] += acc[u];
          }
        }
      }
    }
    s = e;
  }
}

// one block per chunk whose last run starts in it and crosses into the next chunk: the run's pieces
// (part_last of this chunk, part_first of the following ones) added in chunk order
__global__ void __launch_bounds__(256) embed_word_join_kernel(int64_t rows, int64_t D, const uint32_t* __restrict__ keys,
                                                              const float* __restrict__ part_first,
                                                              const float* __restrict__ part_last,
                                                              float* __restrict__ dword, int64_t padding_idx) {
  const int t = threadIdx.x, lane = t & 63;
  const int64_t c = blockIdx.x;
  const int64_t i0 = c * kSegChunk, i1 = i0 + kSegChunk;
  if (i1 >= rows) return;  // the last chunk has no successor
  const uint32_t key = keys[i1 - 1];
  if (keys[i1] != key) return;
  // the run must start inside this chunk (else an earlier chunk joins it)
  if (keys[i0] == key && i0 > 0 && keys[i0 - 1] == key) return;
  if ((int64_t)key == padding_idx) return;
  // the following chunks the run reaches are those that start with its id (the keys are sorted):
  // 64 chunks tested per ballot (every wave of the block computes the same count)
  const int64_t nch = (rows + kSegChunk - 1) / kSegChunk;
  int64_t n = 0;
  for (;;) {
    const int64_t cc = c + 1 + n + lane;
    const bool in = cc < nch && keys[cc * kSegChunk] == key;
    const uint64_t m = __ballot(in);
    const int run = m == ~0ull ? 64 : __builtin_ctzll(~m);  // leading chunks of the run (m has no gaps)
    n += run;
    if (run < 64) break;
  }
  for (int64_t d = t; d < D; d += 256) {
    float acc = part_last[c * D + d];
#pragma unroll 8
    for (int64_t cc = c + 1; cc <= c + n; ++cc) acc += part_first[cc * D + d];
    dword[(int64_t)key * D + d] += acc;
  }
}

// dpos[t][d] += sum_b dsum[b][t][d] (batch order)
template <typename T>
__global__ void embed_pos_bwd_kernel(int64_t B, int64_t L, int64_t D, const T* __restrict__ dsum, float* __restrict__ dpos) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < L * D; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
#pragma unroll 8
    for (int64_t b = 0; b < B; ++b) s += to_f32(dsum[b * L * D + i]);
    dpos[i] += s;
  }
}

// token types 0/1: block (x = 256 columns, y = row slab) writes its slab's two column sums to
// part[slab][type][d]; embed_type_reduce_kernel adds them in a fixed order (16 runs of slabs, each
// in slab order, then the runs in order)
template <typename T>
__global__ void embed_type_part_kernel(int64_t rows, int64_t D, const int64_t* __restrict__ tts, const T* __restrict__ dsum,
                                       float* __restrict__ part) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = (int64_t)blockIdx.y * per, r1 = std::min<int64_t>(rows, r0 + per);
  float s0 = 0.f, s1 = 0.f;
#pragma unroll 8
  for (int64_t r = r0; r < r1; ++r) {
    const float g = to_f32(dsum[r * D + d]);
    if (tts && tts[r] == 1) s1 += g; else s0 += g;
  }
  part[((int64_t)blockIdx.y * 2) * D + d] = s0;
  part[((int64_t)blockIdx.y * 2 + 1) * D + d] = s1;
}
// 64 outputs (of the 2 x D) per 1,024-thread block: wave w sums slabs [w S/16, (w+1) S/16) in order,
// wave 0 adds the 16 wave sums in wave order
__global__ void __launch_bounds__(1024) embed_type_reduce_kernel(int64_t D, int slabs, const float* __restrict__ part,
                                                                 float* __restrict__ dtype_emb) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;  // output index over 2 * D
  const bool ok = i < 2 * D;
  const int64_t t = ok ? i / D : 0, d = ok ? i % D : 0;
  const int per = (slabs + 15) / 16, k0 = w * per, k1 = min(slabs, k0 + per);
  float s = 0.f;
  if (ok) {
#pragma unroll 8
    for (int k = k0; k < k1; ++k) s += part[((int64_t)k * 2 + t) * D + d];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && ok) {
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) r += red[q][lane];
    dtype_emb[i] += r;
  }
}

struct EmbedWs {
  int64_t keys0, keys1, vals0, vals1, sort_tmp, sort_tmp_bytes, part, seg_first, seg_last, total;
};
hipError_t embed_ws_layout(int64_t rows, int64_t D, EmbedWs& w) {
  size_t tmp = 0;
  rocprim::double_buffer<uint32_t> k(nullptr, nullptr);
  rocprim::double_buffer<int32_t> v(nullptr, nullptr);
  // the temporary storage of the widest sort (all 32 key bits): an upper bound for every end_bit
  const hipError_t e = rocprim::radix_sort_pairs(nullptr, tmp, k, v, (size_t)rows, 0, 32, (hipStream_t)0);
  int64_t o = 0;
  w.keys0 = o; o += align256(rows * 4);
  w.keys1 = o; o += align256(rows * 4);
  w.vals0 = o; o += align256(rows * 4);
  w.vals1 = o; o += align256(rows * 4);
  w.sort_tmp = o; w.sort_tmp_bytes = (int64_t)tmp; o += align256((int64_t)tmp);
  w.part = o; o += align256((int64_t)kTypeSlabs * 2 * D * 4);
  const int64_t nch = (rows + kSegChunk - 1) / kSegChunk;
  w.seg_first = o; o += align256(nch * D * 4);
  w.seg_last = o; o += align256(nch * D * 4);
  w.total = o;
  return e;
}
// key bits that hold every id < vocab (all 32 when the vocabulary is not given)
unsigned id_bits(int64_t vocab) {
  if (vocab <= 0 || vocab > ((int64_t)1 << 32)) return 32;
  unsigned b = 1;
  while (b < 32 && ((int64_t)1 << b) < vocab) ++b;
  return b;
}
int type_slabs(int64_t rows) { return (int)std::min<int64_t>(kTypeSlabs, std::max<int64_t>(1, rows / 64)); }
}  // namespace

extern "C" int64_t mmfd_embed_bwd_workspace_bytes(int64_t B, int64_t L, int64_t D) {
  if (B <= 0 || L <= 0 || D <= 0 || B * L > INT32_MAX) return 0;
  EmbedWs w;
  if (embed_ws_layout(B * L, D, w) != hipSuccess) return -1;
  return w.total;
}

extern "C" int mmfd_embed_bwd(int dtype, int64_t B, int64_t L, int64_t D, int64_t vocab, const int64_t* input_ids,
                              const int64_t* token_type_ids, const void* dsum, float* dword, float* dpos, float* dtype_emb,
                              int64_t padding_idx, void* workspace, int64_t workspace_bytes, mmfd_stream_t stream) {
  const int64_t rows = B * L;
  if (rows == 0) return 0;
  MMFD_CHECK_ARG(B > 0 && L > 0 && D > 0 && rows <= INT32_MAX, "embed_bwd: bad shape B=%lld L=%lld D=%lld",
                 (long long)B, (long long)L, (long long)D);
  MMFD_CHECK_ARG(dtype == MMFD_BF16 || dtype == MMFD_F32, "embed_bwd: dtype %d", dtype);
  EmbedWs w;
  if (embed_ws_layout(rows, D, w) != hipSuccess) return mmfd_set_error(MMFD_ERR_INVALID, "embed_bwd: sort size query failed");
  MMFD_CHECK_ARG(workspace != nullptr && workspace_bytes >= w.total,
                 "embed_bwd: workspace %lld B, needs %lld (mmfd_embed_bwd_workspace_bytes)", (long long)workspace_bytes,
                 (long long)w.total);
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const bool bf = dtype == MMFD_BF16;
  if (dword) {
    rocprim::double_buffer<uint32_t> k((uint32_t*)(ws + w.keys0), (uint32_t*)(ws + w.keys1));
    rocprim::double_buffer<int32_t> v((int32_t*)(ws + w.vals0), (int32_t*)(ws + w.vals1));
    hipLaunchKernelGGL(embed_sort_prep_kernel, dim3(gridn(rows, 256)), dim3(256), 0, s, rows, input_ids, k.current(),
                       v.current());
    size_t tmp = (size_t)w.sort_tmp_bytes;
    const hipError_t e = rocprim::radix_sort_pairs(ws + w.sort_tmp, tmp, k, v, (size_t)rows, 0, id_bits(vocab), s);
    if (e != hipSuccess) return mmfd_set_error((int)e, "embed_bwd: radix sort: %s", hipGetErrorString(e));
    const dim3 g((unsigned)((rows + kSegChunk - 1) / kSegChunk));
    float* pf = (float*)(ws + w.seg_first);
    float* pl = (float*)(ws + w.seg_last);
    if (bf)
      hipLaunchKernelGGL((embed_word_segsum_kernel<bf16>), g, dim3(256), 0, s, rows, D, k.current(), v.current(),
                         (const bf16*)dsum, dword, pf, pl, padding_idx);
    else
      hipLaunchKernelGGL((embed_word_segsum_kernel<float>), g, dim3(256), 0, s, rows, D, k.current(), v.current(),
                         (const float*)dsum, dword, pf, pl, padding_idx);
    hipLaunchKernelGGL(embed_word_join_kernel, g, dim3(256), 0, s, rows, D, k.current(), pf, pl, dword, padding_idx);
  }
  if (dpos) {
    if (bf) hipLaunchKernelGGL((embed_pos_bwd_kernel<bf16>), dim3(gridn(L * D, 256)), dim3(256), 0, s, B, L, D, (const bf16*)dsum, dpos);
    else hipLaunchKernelGGL((embed_pos_bwd_kernel<float>), dim3(gridn(L * D, 256)), dim3(256), 0, s, B, L, D, (const float*)dsum, dpos);
  }
  if (dtype_emb) {
    const int slabs = type_slabs(rows);
    float* part = (float*)(ws + w.part);
    const dim3 gt((unsigned)((D + 255) / 256), (unsigned)slabs);
    if (bf) hipLaunchKernelGGL((embed_type_part_kernel<bf16>), gt, dim3(256), 0, s, rows, D, token_type_ids, (const bf16*)dsum, part);
    else hipLaunchKernelGGL((embed_type_part_kernel<float>), gt, dim3(256), 0, s, rows, D, token_type_ids, (const float*)dsum, part);
    hipLaunchKernelGGL(embed_type_reduce_kernel, dim3((unsigned)((2 * D + 63) / 64)), dim3(1024), 0, s, D, slabs, part, dtype_emb);
  }
  MMFD_CHECK_LAUNCH("embed_bwd");
  return 0;
}
