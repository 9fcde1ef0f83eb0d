// The fp32-output instantiations of the 256x256 GEMM (gemm256.h): the bf16 weight gradients whose
// fp32 result feeds the optimizer (C = fp32), the segmented split-operand product and the fp32-MFMA
// kernels. Built as its own translation unit without SLP vectorisation (Makefile): with the SLP
// vectorizer the max-ilp schedule of these instantiations spilled 8-40 dwords of scratch (the
// packed epilogue temporaries), without it they are spill-free and the bf16-output kernels of
// gemm.hip keep the vectorised code that measured 4-7 % faster on the forward shapes
// (gpurun_out/ab_ilpnoslp_gemm_bench_bf16, round 5). `make` refuses any GEMM with scratch.
#include "common.h"
#include <algorithm>
#include <type_traits>
#include <stdlib.h>

#include "gemm_tiles.h"
#include "gemm256.h"

namespace mmfd_gemmx {

template <typename T, int TA, int TB, bool X6>
void launch_g8_f32out(const mmfd_gemm_args& a, const EpiArgs& e, float* ws, int splits, int tps, float* rs_out,
                      int rs_mode, hipStream_t s, const void* A, int64_t lda, const void* B, int64_t ldb, X6Args x6) {
  launch_g8_v<T, TA, TB, float, false, X6>(a, e, ws, splits, tps, rs_out, rs_mode, s, A, lda, B, ldb, x6);
}

#define MMFD_F32OUT(T, X6)                                                                                  \
  template void launch_g8_f32out<T, 0, 0, X6>(const mmfd_gemm_args&, const EpiArgs&, float*, int, int, float*, \
                                              int, hipStream_t, const void*, int64_t, const void*, int64_t,   \
                                              X6Args);                                                        \
  template void launch_g8_f32out<T, 0, 1, X6>(const mmfd_gemm_args&, const EpiArgs&, float*, int, int, float*, \
                                              int, hipStream_t, const void*, int64_t, const void*, int64_t,   \
                                              X6Args);                                                        \
  template void launch_g8_f32out<T, 1, 0, X6>(const mmfd_gemm_args&, const EpiArgs&, float*, int, int, float*, \
                                              int, hipStream_t, const void*, int64_t, const void*, int64_t,   \
                                              X6Args);                                                        \
  template void launch_g8_f32out<T, 1, 1, X6>(const mmfd_gemm_args&, const EpiArgs&, float*, int, int, float*, \
                                              int, hipStream_t, const void*, int64_t, const void*, int64_t,   \
                                              X6Args);
MMFD_F32OUT(bf16, false)
MMFD_F32OUT(bf16, true)
MMFD_F32OUT(float, false)

}  // namespace mmfd_gemmx
