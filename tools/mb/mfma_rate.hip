// Microbenchmark: cycles per v_mfma_f32_16x16x32_bf16 in the x6f GEMM's phase shape (48 MFMAs: 4 A
// subtiles x 2 B subtiles x 6 plane products, two interleaved chains from zero, accumulator adds),
// one wave per SIMD, operands in registers; variants by the operand / chain pattern.
//   hipcc -O3 --offload-arch=gfx950 [-mllvm -amdgpu-mfma-vgpr-form] tools/mb/mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ void mma(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}

template <int V>
__global__ void __launch_bounds__(256) kern(const bf16x8* in, float* out, uint64_t* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4][3], b[2][3];
  for (int i = 0; i < 4; ++i) for (int p = 0; p < 3; ++p) a[i][p] = in[(i * 3 + p) * 64 + lane];
  for (int j = 0; j < 2; ++j) for (int p = 0; p < 3; ++p) b[j][p] = in[(12 + j * 3 + p) * 64 + lane];
  f32x4 acc[4][2];
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (V == 0) {  // x6f: per A subtile two chains from zero (t0, t1 interleaved), then acc += t
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x4 t0 = {0.f, 0.f, 0.f, 0.f}, t1 = {0.f, 0.f, 0.f, 0.f};
        mma(t0, b[0][1], a[i][1]); mma(t1, b[1][1], a[i][1]);
        mma(t0, b[0][2], a[i][0]); mma(t1, b[1][2], a[i][0]);
        mma(t0, b[0][0], a[i][2]); mma(t1, b[1][0], a[i][2]);
        mma(t0, b[0][1], a[i][0]); mma(t1, b[1][1], a[i][0]);
        mma(t0, b[0][0], a[i][1]); mma(t1, b[1][0], a[i][1]);
        mma(t0, b[0][0], a[i][0]); mma(t1, b[1][0], a[i][0]);
        acc[i][0] += t0; acc[i][1] += t1;
      }
    } else if (V == 1) {  // same products straight into the 8 accumulators (no partial sums, no adds)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        mma(acc[i][0], b[0][1], a[i][1]); mma(acc[i][1], b[1][1], a[i][1]);
        mma(acc[i][0], b[0][2], a[i][0]); mma(acc[i][1], b[1][2], a[i][0]);
        mma(acc[i][0], b[0][0], a[i][2]); mma(acc[i][1], b[1][0], a[i][2]);
        mma(acc[i][0], b[0][1], a[i][0]); mma(acc[i][1], b[1][1], a[i][0]);
        mma(acc[i][0], b[0][0], a[i][1]); mma(acc[i][1], b[1][0], a[i][1]);
        mma(acc[i][0], b[0][0], a[i][0]); mma(acc[i][1], b[1][0], a[i][0]);
      }
    } else if (V == 2) {  // 8 accumulators round robin (each MFMA depends on the one 8 earlier)
#pragma unroll
      for (int p = 0; p < 6; ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          mma(acc[i][0], b[0][p % 3], a[i][p / 2]);
          mma(acc[i][1], b[1][p % 3], a[i][p / 2]);
        }
    } else {  // one operand pair, one accumulator (the guide's back-to-back figure)
#pragma unroll
      for (int k = 0; k < 48; ++k) mma(acc[0][0], b[0][0], a[0][0]);
    }
  }
  asm volatile("s_nop 0" ::: "memory");
  float s = 0.f;
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 2; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  bf16x8* in; float* out; uint64_t* cyc;
  hipMalloc(&in, 18 * 64 * 16); hipMemset(in, 0, 18 * 64 * 16);
  hipMalloc(&out, 256 * 256 * 4); hipMalloc(&cyc, 256 * 4 * 8);
  const int iters = 200;
  uint64_t h[1024];
  const char* names[4] = {"x6f chains+adds", "direct 8 acc", "round robin 8 acc", "1 acc same operands"};
  for (int v = 0; v < 4; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      if (v == 0) hipLaunchKernelGGL(kern<0>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
      if (v == 1) hipLaunchKernelGGL(kern<1>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
      if (v == 2) hipLaunchKernelGGL(kern<2>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
      if (v == 3) hipLaunchKernelGGL(kern<3>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, 1024 * 8, hipMemcpyDeviceToHost);
    double m = 0; for (int i = 0; i < 1024; ++i) m += h[i];
    m /= 1024;
    printf("%-22s %.2f cycles per MFMA (one wave per SIMD)\n", names[v], m / (iters * 48.0));
  }
  return 0;
}
