// Ray Data GPU preprocessing kernels (map_batches on device tensors).
//
//   ra_image_normalize: uint8 NHWC -> bf16/f32 NCHW, y = (x/255 - mean[c]) / std[c]
//   ra_resize_bilinear: bf16/f32 NCHW bilinear resize (align_corners=False)
//   ra_cast_scale     : uint8 -> bf16 with scale (Atari frames: x/255)
//   ra_gather_cast_u8 : y[i] = x[idx[i]] * scale, uint8 rows -> bf16 (PPO minibatch frames)
//
// image_normalize treats each image as a flat run of H*W pixels (NHWC -> NCHW never
// needs a row structure): 16 pixels per thread, 16-byte loads and stores.
#include "common.h"

// y[c] = x * scale[c] + bias[c]  with scale = 1/(255 std), bias = -mean/std (one FMA)
struct NormParams {
  float scale[4];
  float bias[4];
};

// Vector path (H*W % 16 == 0): one thread = 16 consecutive pixels of one image.
// Loads 16*C bytes as C x 16-byte loads (adjacent lanes read adjacent 16*C-byte chunks,
// fully coalesced), converts bytes with v_cvt_f32_ubyteN + one FMA, and writes each of
// the C output planes as 32 contiguous bytes (bf16: 2 x 16-byte stores; fp32: 4).
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <int C, bool BF16_OUT, bool NT>
__global__ __launch_bounds__(256) void image_normalize_vec_kernel(const uint8_t* __restrict__ x,
                                                                  void* __restrict__ y,
                                                                  long groups, long hw16,
                                                                  NormParams p) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= groups) return;
  const long n = g / hw16;
  const long hw = (g - n * hw16) * 16;
  const long HW = hw16 * 16;
  uint32_t w[4 * C];
  const u32x4_t* src = reinterpret_cast<const u32x4_t*>(x) + g * C;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const u32x4_t v = NT ? __builtin_nontemporal_load(src + k) : src[k];
    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int b = j * C + c;  // compile-time byte index
      f[j] = (float)((w[b >> 2] >> ((b & 3) * 8)) & 0xffu) * p.scale[c] + p.bias[c];
    }
    const long o = (n * C + c) * HW + hw;
    u32x4_t v[BF16_OUT ? 2 : 4];
    if (BF16_OUT) {
      float a[8], b2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] = f[j]; b2[j] = f[8 + j]; }
      const uint4 p0 = pack8(a), p1 = pack8(b2);
      v[0] = u32x4_t{p0.x, p0.y, p0.z, p0.w};
      v[1] = u32x4_t{p1.x, p1.y, p1.z, p1.w};
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[q] = u32x4_t{__float_as_uint(f[4 * q]), __float_as_uint(f[4 * q + 1]),
                       __float_as_uint(f[4 * q + 2]), __float_as_uint(f[4 * q + 3])};
    }
    u32x4_t* dst = reinterpret_cast<u32x4_t*>(reinterpret_cast<char*>(y) +
                                              o * (BF16_OUT ? 2 : 4));
#pragma unroll
    for (int q = 0; q < (BF16_OUT ? 2 : 4); ++q) {
      if (NT) __builtin_nontemporal_store(v[q], dst + q);
      else dst[q] = v[q];
    }
  }
}

// Generic path: one thread per pixel.
template <bool BF16_OUT>
__global__ __launch_bounds__(256) void image_normalize_px_kernel(const uint8_t* __restrict__ x,
                                                                 void* __restrict__ y, long npx,
                                                                 long HW, int C, NormParams p) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= npx) return;
  const long n = i / HW, hw = i - n * HW;
  for (int c = 0; c < C; ++c) {
    const float v = (float)x[i * C + c] * p.scale[c] + p.bias[c];
    const long o = (n * C + c) * HW + hw;
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

// Minibatch gather + cast in one pass: y[i, :] = x[idx[i], :] * scale (uint8 rows of
// `row` bytes, row % 16 == 0) — the PPO learner's minibatch frames straight from the
// resident train batch, 16 pixels per thread (16-B load, 2 x 16-B stores).
__global__ __launch_bounds__(256) void gather_cast_kernel(const uint8_t* __restrict__ x,
                                                          const long* __restrict__ idx,
                                                          bf16_t* __restrict__ y, int row16,
                                                          long n16, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / row16, c = i - r * row16;
    const uint4 u = reinterpret_cast<const uint4*>(x)[idx[r] * row16 + c];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    float f[8], h[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = (float)((w[0] >> (8 * j)) & 0xff) * scale;
      f[4 + j] = (float)((w[1] >> (8 * j)) & 0xff) * scale;
      h[j] = (float)((w[2] >> (8 * j)) & 0xff) * scale;
      h[4 + j] = (float)((w[3] >> (8 * j)) & 0xff) * scale;
    }
    uint4* yo = reinterpret_cast<uint4*>(y) + 2 * i;
    yo[0] = pack8(f);
    yo[1] = pack8(h);
  }
}

// mean / std are HOST pointers (C floats): folded into kernel arguments, no H2D copy.
RA_EXPORT int ra_image_normalize(const void* x, void* y, int N, int H, int W, int C,
                                 const float* mean, const float* std_, int bf16_out,
                                 hipStream_t st) {
  if (C < 1 || C > 4) return hipErrorInvalidValue;
  NormParams p;
  for (int c = 0; c < 4; ++c) {
    const float sd = c < C ? std_[c] : 1.f, m = c < C ? mean[c] : 0.f;
    p.scale[c] = 1.f / (255.f * sd);
    p.bias[c] = -m / sd;
  }
  const long HW = (long)H * W;
  const bool vec = (HW % 16) == 0 && (((uintptr_t)x) % 16) == 0 && (((uintptr_t)y) % 16) == 0;
  if (vec) {
    const long groups = (long)N * HW / 16;
    const dim3 g((unsigned)((groups + 255) / 256));
    // plain loads/stores: nontemporal ones measured slower on MI355X (4.4 vs 5.5 TB/s)
#define RA_IMN2(CC, NTV)                                                                        \
  if (bf16_out)                                                                                 \
    hipLaunchKernelGGL((image_normalize_vec_kernel<CC, true, NTV>), g, dim3(256), 0, st,        \
                       (const uint8_t*)x, y, groups, HW / 16, p);                              \
  else                                                                                          \
    hipLaunchKernelGGL((image_normalize_vec_kernel<CC, false, NTV>), g, dim3(256), 0, st,       \
                       (const uint8_t*)x, y, groups, HW / 16, p);
#define RA_IMN(CC)                                                                              \
  if (C == CC) {                                                                                \
    RA_IMN2(CC, false)                                                                          \
  }
    RA_IMN(1) RA_IMN(2) RA_IMN(3) RA_IMN(4)
#undef RA_IMN
#undef RA_IMN2
  } else {
    const long npx = (long)N * HW;
    const dim3 g((unsigned)((npx + 255) / 256));
    if (bf16_out)
      hipLaunchKernelGGL(image_normalize_px_kernel<true>, g, dim3(256), 0, st, (const uint8_t*)x,
                         y, npx, HW, C, p);
    else
      hipLaunchKernelGGL(image_normalize_px_kernel<false>, g, dim3(256), 0, st, (const uint8_t*)x,
                         y, npx, HW, C, p);
  }
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

// idx values must lie in [0, rows of x): the caller passes a permutation of the batch.
RA_EXPORT int ra_gather_cast_u8(const void* x, const long* idx, void* y, long nrows, long row,
                                float scale, hipStream_t st) {
  if (row % 16 || row / 16 > (1L << 30)) return hipErrorInvalidValue;
  const long n16 = nrows * (row / 16);
  hipLaunchKernelGGL(gather_cast_kernel, dim3(ra_grid(n16, 256)), dim3(256), 0, st,
                     (const uint8_t*)x, idx, (bf16_t*)y, (int)(row / 16), n16, scale);
  return hipGetLastError();
}

RA_EXPORT int ra_cast_scale_u8(const void* x, void* y, long n, float scale, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_scale_kernel, dim3(ra_grid(n / 8, 256)), dim3(256), 0, st,
                     (const uint8_t*)x, (bf16_t*)y, n / 8, scale);
  return hipGetLastError();
}
