// Fused GEMM epilogues for the GPT-2 MLP / projections, bf16 in and out.
//
//   ra_bias_gelu_fwd   y  = gelu_tanh(h + bias)
//   ra_bias_gelu_bwd   dh = dy * gelu_tanh'(h + bias);  dbias = sum_rows(dh)
//   ra_bias_residual   y  = res + h + bias
//   ra_colsum_bf16     out = sum_rows(x)     (bias gradient of a projection)
//
// The GEMM itself stays on hipBLASLt (plain library GEMM); these kernels fuse
// everything around it into one HBM pass. Each thread moves 8 bf16 (16 bytes);
// column reductions keep 8 fp32 partials per thread in registers over a row
// chunk and finish with `colsum` over P partial rows.
#include "common.h"

__device__ __forceinline__ float gelu_tanh(float u, float* dgelu) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float z = k0 * (u + k1 * u * u * u);
  // tanh(z) = 1 - 2 / (exp(2z) + 1): v_exp_f32 + v_rcp_f32 (no IEEE division sequence)
  const float e = __builtin_amdgcn_exp2f(2.885390081777927f * z);  // exp(2z)
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  if (dgelu) {
    const float dz = k0 * (1.f + 3.f * k1 * u * u);
    *dgelu = 0.5f * (1.f + t) + 0.5f * u * (1.f - t * t) * dz;
  }
  return 0.5f * u * (1.f + t);
}

// grid-stride over 16-B vectors; 32-bit index math (n8 < 2^31 is checked on the host)
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const bf16_t* __restrict__ h,
                                                            const bf16_t* __restrict__ bias,
                                                            bf16_t* __restrict__ y, int n8,
                                                            int F8) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const int c8 = (int)((unsigned)i % (unsigned)F8);
    float hv[8], bv[8], o[8];
    unpack8(reinterpret_cast<const uint4*>(h)[i], hv);
    unpack8(reinterpret_cast<const uint4*>(bias)[c8], bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gelu_tanh(hv[j] + bv[j], nullptr);
    reinterpret_cast<uint4*>(y)[i] = pack8(o);
  }
}

// grid: (ceil(F8/256), P). Thread owns 8 columns, walks the rows of chunk blockIdx.y.
template <bool GELU>
__global__ __launch_bounds__(64) void bwd_colpart_kernel(const bf16_t* __restrict__ dy,
                                                          const bf16_t* __restrict__ h,
                                                          const bf16_t* __restrict__ bias,
                                                          bf16_t* __restrict__ dh,
                                                          float* __restrict__ part, int N,
                                                          int F8, int rows_per_part) {
  const int c8 = blockIdx.x * blockDim.x + threadIdx.x;
  if (c8 >= F8) return;
  const int r0 = blockIdx.y * rows_per_part;
  const int r1 = min(N, r0 + rows_per_part);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  float bv[8];
  if (GELU) unpack8(reinterpret_cast<const uint4*>(bias)[c8], bv);
  // RB rows per batch: all loads of a batch are issued before any use, so each wave
  // keeps RB (x2 with GELU) 16-B loads in flight — the grid is only ~6 waves per CU
  constexpr int RB = 4;
  const uint4* dy4 = reinterpret_cast<const uint4*>(dy);
  const uint4* h4 = reinterpret_cast<const uint4*>(h);
  for (int rb = r0; rb < r1; rb += RB) {
    uint4 dv[RB], hv4[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int r = rb + k < r1 ? rb + k : r1 - 1;
      const long idx = (long)r * F8 + c8;
      dv[k] = dy4[idx];
      if (GELU) hv4[k] = h4[idx];
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      if (rb + k >= r1) break;
      const long idx = (long)(rb + k) * F8 + c8;
      float d[8];
      unpack8(dv[k], d);
      if (GELU) {
        float hv[8], o[8];
        unpack8(hv4[k], hv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float dg;
          gelu_tanh(hv[j] + bv[j], &dg);
          o[j] = d[j] * dg;
          acc[j] += o[j];
        }
        reinterpret_cast<uint4*>(dh)[idx] = pack8(o);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += d[j];
      }
    }
  }
  float* pr = part + (size_t)blockIdx.y * F8 * 8 + (size_t)c8 * 8;
  *reinterpret_cast<float4*>(pr) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(pr + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

__global__ __launch_bounds__(256) void bias_residual_kernel(const bf16_t* __restrict__ h,
                                                            const bf16_t* __restrict__ bias,
                                                            const bf16_t* __restrict__ res,
                                                            bf16_t* __restrict__ y, long n8,
                                                            int F8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8;
       i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % F8);
    float hv[8], bv[8], rv[8], o[8];
    unpack8(reinterpret_cast<const uint4*>(h)[i], hv);
    unpack8(reinterpret_cast<const uint4*>(res)[i], rv);
    if (bias) unpack8(reinterpret_cast<const uint4*>(bias)[c8], bv);
    else for (int j = 0; j < 8; ++j) bv[j] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = rv[j] + hv[j] + bv[j];
    reinterpret_cast<uint4*>(y)[i] = pack8(o);
  }
}

// Row partitions of a column reduction: enough (64-thread) blocks to put ~ra_knobs[1]
// waves on the chip (8192 = 32 per CU) whatever F is (F = 768 gives only 2 column
// blocks), >= 32 rows per partial.
static inline int parts_for(int N, int F) {
  const int bx = (F / 8 + 63) / 64;
  const int waves = ra_knobs[1] > 0 ? ra_knobs[1] : 8192;
  int p = (waves + bx - 1) / bx;
  if (p < 256) p = 256;
  const int pmax = (N + 31) / 32;
  return p < pmax ? p : (pmax > 0 ? pmax : 1);
}

RA_EXPORT int ra_colsum_parts(int N, int F) { return parts_for(N, F); }

// fp32 workspace (floats) for ra_bias_gelu_bwd / ra_colsum_bf16.
RA_EXPORT long ra_colsum_work(int N, int F) {
  return (long)parts_for(N, F) * F + (long)kColsumSplits * F;
}

RA_EXPORT int ra_bias_gelu_fwd(const void* h, const void* bias, void* y, long N, int F,
                               hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const long n8 = N * (long)F / 8;
  if (n8 >= (1L << 31) - 65536L * 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3(ra_grid(n8, 256)), dim3(256), 0, st,
                     (const bf16_t*)h, (const bf16_t*)bias, (bf16_t*)y, (int)n8, F / 8);
  return hipGetLastError();
}

// Sink flags shared by the bias-gradient entry points below:
//   bit0: accumulate into `out` (direct write into a flat gradient buffer view)
//   bit1: `out` is fp32 (the default fp32 gradient buffer) instead of bf16
static inline int sink_flags(int flags) {
  return ((flags & 1) ? kColsumAcc : 0) | ((flags & 2) ? 0 : kColsumBF16);
}

// work: ra_colsum_work(N, F) floats
RA_EXPORT int ra_bias_gelu_bwd(const void* dy, const void* h, const void* bias, void* dh,
                               void* dbias, float* work, int N, int F, int flags,
                               hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const int P = parts_for(N, F), F8 = F / 8;
  const int rpp = (N + P - 1) / P;
  hipLaunchKernelGGL(bwd_colpart_kernel<true>, dim3((F8 + 63) / 64, P), dim3(64), 0, st,
                     (const bf16_t*)dy, (const bf16_t*)h, (const bf16_t*)bias, (bf16_t*)dh, work,
                     N, F8, rpp);
  colsum_launch(work, work + (size_t)P * F, dbias, P, F, sink_flags(flags), st);
  return hipGetLastError();
}

RA_EXPORT int ra_colsum_bf16(const void* x, void* out, float* work, int N, int F, int flags,
                             hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const int P = parts_for(N, F), F8 = F / 8;
  const int rpp = (N + P - 1) / P;
  hipLaunchKernelGGL(bwd_colpart_kernel<false>, dim3((F8 + 63) / 64, P), dim3(64), 0, st,
                     (const bf16_t*)x, nullptr, nullptr, nullptr, work, N, F8, rpp);
  colsum_launch(work, work + (size_t)P * F, out, P, F, sink_flags(flags), st);
  return hipGetLastError();
}

RA_EXPORT int ra_bias_residual(const void* h, const void* bias, const void* res, void* y, long N,
                               int F, hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const long n8 = N * (long)F / 8;
  hipLaunchKernelGGL(bias_residual_kernel, dim3(ra_grid(n8, 256)), dim3(256), 0, st,
                     (const bf16_t*)h, (const bf16_t*)bias, (const bf16_t*)res, (bf16_t*)y, n8,
                     F / 8);
  return hipGetLastError();
}
