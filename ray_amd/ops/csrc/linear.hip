// Split-K weight-gradient epilogue for the GPT-2 projections.
//
// The wgrad GEMM dW[N,K] = dY^T[N,M] · X[M,K] of a transformer linear has a small output
// (N,K <= 3072) and a long reduction (M = batch*seq tokens): a plain GEMM gets only
// (N/128)*(K/128) = 36..144 output tiles, far below the 256 CUs (measured 210-530 TFLOPS
// on MI355X vs ~1 PFLOPS for the forward). The linear op therefore runs it as S batched
// GEMMs over token slices with fp32 outputs (hipBLASLt) and this kernel finishes:
//
//   grad[i] = bf16( grad[i] + sum_s part[s][i] )          (grad = flat gradient buffer view)
//
// one HBM pass that also replaces autograd's separate AccumulateGrad add, and sums the
// split partials in fp32 (relative error 1.5e-6 vs 1.7e-3 for a bf16-output GEMM). With
// the default fp32 flat gradient buffer the sum is never rounded to bf16 at all.
#include "common.h"

template <bool OUT_F32>
__global__ __launch_bounds__(256) void splitk_accum_kernel(const float* __restrict__ part, int S,
                                                           long n4, void* __restrict__ grad,
                                                           int accumulate) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = reinterpret_cast<const float4*>(part)[i];
    for (int s = 1; s < S; ++s) {
      const float4 b = reinterpret_cast<const float4*>(part)[(long)s * n4 + i];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    if (OUT_F32) {
      // fp32 flat gradient (default): the split partials land in full precision
      float4* g = reinterpret_cast<float4*>(grad) + i;
      if (accumulate) {
        const float4 o = *g;
        a.x += o.x;
        a.y += o.y;
        a.z += o.z;
        a.w += o.w;
      }
      *g = a;
    } else {
      uint2* g = reinterpret_cast<uint2*>(grad) + i;
      float v[4] = {a.x, a.y, a.z, a.w};
      if (accumulate) {
        float o[4];
        unpack4(*g, o);
        v[0] += o[0];
        v[1] += o[1];
        v[2] += o[2];
        v[3] += o[3];
      }
      *g = pack4(v);
    }
  }
}

// Fixed-S variant: all S partial loads of an element are issued before the first add
// (the runtime-S loop above load-waits-adds one partial at a time: a memory round trip
// per partial per wave, ~1.5 TB/s in the step), and the element's grad read joins them.
template <bool OUT_F32, int S>
__global__ __launch_bounds__(256) void splitk_accum_s_kernel(const float* __restrict__ part,
                                                             long n4, void* __restrict__ grad,
                                                             int accumulate) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 b[S];
#pragma unroll
    for (int s = 0; s < S; ++s) b[s] = reinterpret_cast<const float4*>(part)[(long)s * n4 + i];
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (accumulate) {
      if (OUT_F32) {
        const float4 o = reinterpret_cast<const float4*>(grad)[i];
        v[0] = o.x, v[1] = o.y, v[2] = o.z, v[3] = o.w;
      } else {
        unpack4(reinterpret_cast<const uint2*>(grad)[i], v);
      }
    }
    // partials summed first (same order as the runtime-S kernel), then the old gradient
    float4 a = b[0];
#pragma unroll
    for (int s = 1; s < S; ++s) {
      a.x += b[s].x;
      a.y += b[s].y;
      a.z += b[s].z;
      a.w += b[s].w;
    }
    v[0] += a.x, v[1] += a.y, v[2] += a.z, v[3] += a.w;
    if (OUT_F32)
      reinterpret_cast<float4*>(grad)[i] = make_float4(v[0], v[1], v[2], v[3]);
    else
      reinterpret_cast<uint2*>(grad)[i] = pack4(v);
  }
}

// part: [S, n] fp32; grad: n bf16 or fp32 (n % 4 == 0, 16-byte aligned).
// flags: bit0 accumulate into grad, bit1 grad is fp32.
RA_EXPORT int ra_splitk_accum(const float* part, int S, long n, void* grad, int flags,
                              hipStream_t st) {
  if (n % 4 || S < 1) return hipErrorInvalidValue;
  const long n4 = n / 4;
  const dim3 grid(ra_grid(n4, 256));
#define SK(F32, SS)                                                                            \
  hipLaunchKernelGGL((splitk_accum_s_kernel<F32, SS>), grid, dim3(256), 0, st, part, n4, grad, \
                     flags & 1)
#define SKS(F32)                   \
  switch (S) {                     \
    case 2: SK(F32, 2); break;     \
    case 4: SK(F32, 4); break;     \
    case 8: SK(F32, 8); break;     \
    case 16: SK(F32, 16); break;   \
    default: goto runtime_s;       \
  }                                \
  return hipGetLastError();
  if (flags & 2) {
    SKS(true)
  } else {
    SKS(false)
  }
#undef SKS
#undef SK
runtime_s:
  if (flags & 2)
    hipLaunchKernelGGL(splitk_accum_kernel<true>, dim3(ra_grid(n4, 256)), dim3(256), 0, st, part,
                       S, n4, grad, flags & 1);
  else
    hipLaunchKernelGGL(splitk_accum_kernel<false>, dim3(ra_grid(n4, 256)), dim3(256), 0, st, part,
                       S, n4, grad, flags & 1);
  return hipGetLastError();
}

// sink[i] += (*g) * src[i]   (src fp32; sink fp32 or bf16 by `sink_f32`; g device scalar or
// null = 1). Used by fused ops that precompute a parameter gradient before the upstream
// gradient is known (the LM-head cross-entropy computes it inside forward).
template <bool SINK_F32>
__global__ __launch_bounds__(256) void scaled_accum_kernel(const float* __restrict__ src,
                                                           void* __restrict__ sink, long n4,
                                                           const float* __restrict__ g) {
  const float sc = g ? *g : 1.f;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(src)[i];
    if (SINK_F32) {
      float4* o = reinterpret_cast<float4*>(sink) + i;
      float4 v = *o;
      v.x += sc * a.x;
      v.y += sc * a.y;
      v.z += sc * a.z;
      v.w += sc * a.w;
      *o = v;
    } else {
      uint2* o = reinterpret_cast<uint2*>(sink) + i;
      float v[4];
      unpack4(*o, v);
      v[0] += sc * a.x;
      v[1] += sc * a.y;
      v[2] += sc * a.z;
      v[3] += sc * a.w;
      *o = pack4(v);
    }
  }
}

RA_EXPORT int ra_scaled_accum(const float* src, void* sink, long n, int sink_f32, const float* g,
                              hipStream_t st) {
  if (n % 4) return hipErrorInvalidValue;
  const long n4 = n / 4;
  if (sink_f32)
    hipLaunchKernelGGL(scaled_accum_kernel<true>, dim3(ra_grid(n4, 256)), dim3(256), 0, st, src,
                       sink, n4, g);
  else
    hipLaunchKernelGGL(scaled_accum_kernel<false>, dim3(ra_grid(n4, 256)), dim3(256), 0, st, src,
                       sink, n4, g);
  return hipGetLastError();
}

// x[i] *= (*g), bf16 in place (n % 8 == 0)
__global__ __launch_bounds__(256) void scale_bf16_kernel(bf16_t* __restrict__ x, long n8,
                                                         const float* __restrict__ g) {
  const float sc = *g;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float v[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= sc;
    reinterpret_cast<uint4*>(x)[i] = pack8(v);
  }
}

RA_EXPORT int ra_scale_bf16(void* x, long n, const float* g, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scale_bf16_kernel, dim3(ra_grid(n / 8, 256)), dim3(256), 0, st, (bf16_t*)x,
                     n / 8, g);
  return hipGetLastError();
}

// ------------------------------------------------------------------ bf16 transpose
// dst[c][r] = src[r][c] for a row-major [rows][cols] bf16 matrix (the transposed weight
// copy of the input-gradient GEMM). One 64x64 tile per workgroup through LDS: a wave
// reads 64 consecutive columns of one source row per instruction (128 B, coalesced) and
// writes 64 consecutive columns of one destination row; the +2 element row pad keeps the
// column-order LDS reads free of bank conflicts. (torch's strided copy reads the source
// column-wise: 93 us per GPT-2 weight beside the backward's GEMMs, r4h kernels.md.)
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const unsigned short* __restrict__ src,
                                                             unsigned short* __restrict__ dst,
                                                             int rows, int cols) {
  __shared__ unsigned short tile[64][66];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4 threads
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + ty + 4 * i, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + 4 * i][tx] = src[(long)r * cols + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = c0 + ty + 4 * i, r = r0 + tx;  // destination row c, column r
    if (c < cols && r < rows) dst[(long)c * rows + r] = tile[tx][ty + 4 * i];
  }
}

RA_EXPORT int ra_transpose_bf16(const void* src, void* dst, int rows, int cols, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256),
                     0, st, (const unsigned short*)src, (unsigned short*)dst, rows, cols);
  return hipGetLastError();
}
