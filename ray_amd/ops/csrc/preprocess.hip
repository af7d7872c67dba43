// Ray Data GPU preprocessing kernels (map_batches on device tensors).
//
//   ra_image_normalize: uint8 NHWC -> bf16/f32 NCHW, y = (x/255 - mean[c]) / std[c]
//   ra_resize_bilinear: bf16/f32 NCHW bilinear resize (align_corners=False)
//   ra_cast_scale     : uint8 -> bf16 with scale (Atari frames: x/255)
//
// The NHWC -> NCHW transpose goes through an LDS tile so both the uint8 reads
// (contiguous W*C bytes per image row) and the planar writes are coalesced.
#include "common.h"

#define TW 64
// grid: (ceil(W/TW), H, N); block 256 threads.
template <bool BF16_OUT>
__global__ __launch_bounds__(256) void image_normalize_kernel(const uint8_t* __restrict__ x,
                                                              void* __restrict__ y, int H, int W,
                                                              int C, const float* __restrict__ mean,
                                                              const float* __restrict__ istd) {
  __shared__ float tile[TW * 4 + 4];  // up to C=4 channels
  const int n = blockIdx.z, h = blockIdx.y, w0 = blockIdx.x * TW;
  const int wn = min(TW, W - w0);
  const uint8_t* src = x + (((size_t)n * H + h) * W + w0) * C;
  for (int i = threadIdx.x; i < wn * C; i += blockDim.x) tile[i] = (float)src[i];
  __syncthreads();
  for (int i = threadIdx.x; i < wn * C; i += blockDim.x) {
    const int c = i / wn, w = i % wn;
    const float v = (tile[w * C + c] * (1.f / 255.f) - mean[c]) * istd[c];
    const size_t o = (((size_t)n * C + c) * H + h) * W + w0 + w;
    if (BF16_OUT) reinterpret_cast<bf16_t*>(y)[o] = f2bf(v);
    else reinterpret_cast<float*>(y)[o] = v;
  }
}

template <bool BF16>
__global__ __launch_bounds__(256) void resize_bilinear_kernel(const void* __restrict__ x,
                                                              void* __restrict__ y, int NC, int H,
                                                              int W, int OH, int OW) {
  const long total = (long)NC * OH * OW;
  const float sh = (float)H / OH, sw = (float)W / OW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ow = i % OW, oh = (i / OW) % OH;
    const long nc = i / ((long)OW * OH);
    float fy = fmaxf((oh + 0.5f) * sh - 0.5f, 0.f), fx = fmaxf((ow + 0.5f) * sw - 0.5f, 0.f);
    int y0 = min((int)fy, H - 1), x0 = min((int)fx, W - 1);
    int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const float ly = fy - y0, lx = fx - x0;
    auto ld = [&](int yy, int xx) -> float {
      const long o = (nc * H + yy) * W + xx;
      return BF16 ? bf2f(reinterpret_cast<const bf16_t*>(x)[o]) : reinterpret_cast<const float*>(x)[o];
    };
    const float v = (1 - ly) * ((1 - lx) * ld(y0, x0) + lx * ld(y0, x1)) +
                    ly * ((1 - lx) * ld(y1, x0) + lx * ld(y1, x1));
    if (BF16) reinterpret_cast<bf16_t*>(y)[i] = f2bf(v);
    else reinterpret_cast<float*>(y)[i] = v;
  }
}

__global__ __launch_bounds__(256) void cast_scale_kernel(const uint8_t* __restrict__ x,
                                                         bf16_t* __restrict__ y, long n8,
                                                         float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    const uint2 u = reinterpret_cast<const uint2*>(x)[i];
    float f[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = (float)((u.x >> (8 * j)) & 0xff) * scale;
      f[4 + j] = (float)((u.y >> (8 * j)) & 0xff) * scale;
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

RA_EXPORT int ra_image_normalize(const void* x, void* y, int N, int H, int W, int C,
                                 const float* mean, const float* istd, int bf16_out,
                                 hipStream_t st) {
  if (C > 4) return hipErrorInvalidValue;
  dim3 g((W + TW - 1) / TW, H, N);
  if (bf16_out)
    hipLaunchKernelGGL(image_normalize_kernel<true>, g, dim3(256), 0, st, (const uint8_t*)x, y, H,
                       W, C, mean, istd);
  else
    hipLaunchKernelGGL(image_normalize_kernel<false>, g, dim3(256), 0, st, (const uint8_t*)x, y,
                       H, W, C, mean, istd);
  return hipGetLastError();
}

RA_EXPORT int ra_resize_bilinear(const void* x, void* y, int NC, int H, int W, int OH, int OW,
                                 int bf16, hipStream_t st) {
  const long total = (long)NC * OH * OW;
  if (bf16)
    hipLaunchKernelGGL(resize_bilinear_kernel<true>, dim3(ra_grid(total, 256)), dim3(256), 0, st,
                       x, y, NC, H, W, OH, OW);
  else
    hipLaunchKernelGGL(resize_bilinear_kernel<false>, dim3(ra_grid(total, 256)), dim3(256), 0, st,
                       x, y, NC, H, W, OH, OW);
  return hipGetLastError();
}

RA_EXPORT int ra_cast_scale_u8(const void* x, void* y, long n, float scale, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_scale_kernel, dim3(ra_grid(n / 8, 256)), dim3(256), 0, st,
                     (const uint8_t*)x, (bf16_t*)y, n / 8, scale);
  return hipGetLastError();
}
