// Raw-image preprocessing on gfx950: bilinear resize + crop + ToTensor +
// Normalize of a batch of decoded uint8 RGB images straight into the fp32 NCHW pixel tensor the
// encoders read.
//
// Reference: `preprocess` at src/model/dataset.py:14-19 (Resize(256) -> CenterCrop(256) ->
// ToTensor -> Normalize(mean 0.5, ImageNet std)) and the ImageSimilarity transform at
// src/evidence/im2im_retrieval.py:19-27 (Resize((224, 224)) -> ToTensor -> Normalize(ImageNet)).
// torchvision resizes PIL images with PIL's Image.resize(BILINEAR): a separable, antialiased
// (support scaled by the downsampling factor) filter in 22-bit fixed point, horizontal pass first,
// rounded to uint8 between the passes. The per-output-position taps are computed on the host in
// double precision exactly as PIL does and passed in as int32 tables ([xmin, n, k0 .. k_{K-1}] per
// output position); the kernels do PIL's integer arithmetic, so the uint8 image, and therefore
// the normalised fp32 output, is bit-identical to PIL + torchvision.
//
// Pass 1 (horizontal): one thread per (source row, output column), 3 channels; uint8 rows into a
//   workspace [h][out_w][3].
// Pass 2 (vertical + crop + normalise): one thread per output pixel of the crop window; writes
//   ((v / 255) - mean[c]) / std[c] in fp32 (ToTensor's division, Normalize's sub/div, IEEE ops).
#include "common.h"
#include <algorithm>

namespace {

constexpr int PB = 22;  // PIL's PRECISION_BITS for 8-bit images

__device__ __forceinline__ uint32_t clip8(int64_t ss) {
  const int64_t v = ss >> PB;
  return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__global__ void resize_h_kernel(const mmfd_image_desc* __restrict__ d, const int32_t* __restrict__ coef,
                                uint8_t* __restrict__ ws) {
  const mmfd_image_desc im = d[blockIdx.y];
  const int64_t total = im.h * (int64_t)im.out_w;
  const int K = im.kx_size;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t y = t / im.out_w;
    const int xx = (int)(t - y * im.out_w);
    const int32_t* k = coef + im.kx_off + (int64_t)xx * (K + 2);
    const int xmin = k[0], n = k[1];
    const uint8_t* row = im.src + y * im.stride + (int64_t)xmin * 3;
    int64_t s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < n; ++x) {
      const int64_t w = k[2 + x];
      s0 += (int64_t)row[3 * x + 0] * w;
      s1 += (int64_t)row[3 * x + 1] * w;
      s2 += (int64_t)row[3 * x + 2] * w;
    }
    uint8_t* o = ws + im.tmp_off + t * 3;
    o[0] = (uint8_t)clip8(s0);
    o[1] = (uint8_t)clip8(s1);
    o[2] = (uint8_t)clip8(s2);
  }
}

__global__ void resize_v_norm_kernel(const mmfd_image_desc* __restrict__ d, const int32_t* __restrict__ coef,
                                     const uint8_t* __restrict__ ws, int64_t Ho, int64_t Wo, float m0, float m1,
                                     float m2, float s0, float s1, float s2, float* __restrict__ out) {
  const mmfd_image_desc im = d[blockIdx.y];
  const int K = im.ky_size;
  const int64_t total = Ho * Wo;
  float* o = out + (int64_t)blockIdx.y * 3 * total;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t oy = t / Wo, ox = t - oy * Wo;
    const int64_t yy = im.crop_y + oy, xx = im.crop_x + ox;
    const int32_t* k = coef + im.ky_off + yy * (K + 2);
    const int ymin = k[0], n = k[1];
    const uint8_t* col = ws + im.tmp_off + ((int64_t)ymin * im.out_w + xx) * 3;
    int64_t a0 = 1 << (PB - 1), a1 = a0, a2 = a0;
    for (int y = 0; y < n; ++y) {
      const int64_t w = k[2 + y];
      const uint8_t* p = col + (int64_t)y * im.out_w * 3;
      a0 += (int64_t)p[0] * w;
      a1 += (int64_t)p[1] * w;
      a2 += (int64_t)p[2] * w;
    }
    o[t] = ((float)clip8(a0) / 255.0f - m0) / s0;
    o[total + t] = ((float)clip8(a1) / 255.0f - m1) / s1;
    o[2 * total + t] = ((float)clip8(a2) / 255.0f - m2) / s2;
  }
}

}  // namespace

extern "C" int mmfd_resize_normalize(int64_t n_images, const mmfd_image_desc* descs, int64_t max_h,
                                     int64_t max_out_w, const int32_t* coef, void* workspace, int64_t Ho, int64_t Wo,
                                     const float* mean3, const float* std3, float* out, mmfd_stream_t stream) {
  MMFD_CHECK_ARG(n_images >= 0 && Ho > 0 && Wo > 0, "mmfd_resize_normalize: bad shape");
  MMFD_CHECK_ARG(mean3 && std3, "mmfd_resize_normalize: mean/std are host arrays of 3 floats");
  if (n_images == 0) return 0;
  MMFD_CHECK_ARG(n_images <= 65535, "mmfd_resize_normalize: at most 65535 images per call");
  hipStream_t s = (hipStream_t)stream;
  const int64_t h_work = max_h * max_out_w;
  const unsigned gx1 = (unsigned)std::min<int64_t>((h_work + 255) / 256, 4096);
  hipLaunchKernelGGL(resize_h_kernel, dim3(gx1, (unsigned)n_images), dim3(256), 0, s, descs, coef, (uint8_t*)workspace);
  MMFD_CHECK_LAUNCH("resize_h");
  const unsigned gx2 = (unsigned)std::min<int64_t>((Ho * Wo + 255) / 256, 4096);
  hipLaunchKernelGGL(resize_v_norm_kernel, dim3(gx2, (unsigned)n_images), dim3(256), 0, s, descs, coef,
                     (const uint8_t*)workspace, Ho, Wo, mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2], out);
  MMFD_CHECK_LAUNCH("resize_v_norm");
  return 0;
}
