// Store-rate probe for the GEMM epilogue question: does one CU write its 256 KB output tile at the
// same rate when it is the only CU storing as when all 256 are? One 512-thread workgroup per CU
// (160 KB of dynamic LDS), `active` of them store 256 KB each in the epilogue's pattern (each thread
// 8 consecutive floats of a row, 2 x 16 B per row, rows 16 apart), the rest exit. s_memtime per WG.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

__global__ void __launch_bounds__(512, 1) store_tile(float* out, int active, int nt, unsigned long long* t) {
  extern __shared__ char lds[];
  const int b = blockIdx.x;
  if (b >= active) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float* tile = out + (size_t)b * 65536;   // 256 x 256 floats
  const int tid = threadIdx.x, lr0 = tid / 32, c8 = (tid % 32) * 8;
  float z[8];
  for (int u = 0; u < 8; ++u) z[u] = (float)(tid + u);
  lds[tid] = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int k = 0; k < 8; ++k) {
      float* p = tile + (size_t)(pass * 128 + lr0 + 16 * k) * 256 + c8;
      if (nt) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(f4{z[0], z[1], z[2], z[3]}, reinterpret_cast<f4*>(p));
        __builtin_nontemporal_store(f4{z[4], z[5], z[6], z[7]}, reinterpret_cast<f4*>(p + 4));
      } else {
        *reinterpret_cast<float4*>(p) = make_float4(z[0], z[1], z[2], z[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(z[4], z[5], z[6], z[7]);
      }
    }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) { t[2 * b] = t0; t[2 * b + 1] = t1; }
}

int main() {
  float* out; unsigned long long* t;
  hipMalloc(&out, (size_t)256 * 65536 * 4);
  hipMalloc(&t, 512 * 8);
  hipFuncSetAttribute((const void*)store_tile, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int acts[] = {1, 8, 32, 128, 256};
  for (int nt = 0; nt < 2; ++nt)
    for (int a : acts) {
      std::vector<unsigned long long> h(512);
      double best = 1e30, med = 0;
      for (int it = 0; it < 5; ++it) {
        hipMemset(t, 0, 512 * 8);
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(store_tile, dim3(256), dim3(512), 160 * 1024, 0, out, a, nt, t);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h.data(), t, 512 * 8, hipMemcpyDeviceToHost);
        std::vector<double> d;
        for (int b = 0; b < a; ++b) d.push_back((double)(h[2 * b + 1] - h[2 * b]));
        std::sort(d.begin(), d.end());
        med = d[d.size() / 2];
        best = std::min(best, (double)ms);
      }
      printf("nt=%d active=%3d: median WG store time %8.0f memtime ticks (%.1f B/tick per CU), kernel %.1f us\n", nt, a,
             med, 262144.0 / med, best * 1e3);
    }
  return 0;
}
