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
// split partials in fp32 (relative error 1.5e-6 vs 1.7e-3 for a bf16-output GEMM).
#include "common.h"

__global__ __launch_bounds__(256) void splitk_accum_kernel(const float* __restrict__ part, int S,
                                                           long n4, bf16_t* __restrict__ grad,
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

// part: [S, n] fp32; grad: n bf16 (n % 4 == 0, 8-byte aligned)
RA_EXPORT int ra_splitk_accum(const float* part, int S, long n, void* grad, int accumulate,
                              hipStream_t st) {
  if (n % 4 || S < 1) return hipErrorInvalidValue;
  const long n4 = n / 4;
  hipLaunchKernelGGL(splitk_accum_kernel, dim3(ra_grid(n4, 256)), dim3(256), 0, st, part, S, n4,
                     (bf16_t*)grad, accumulate);
  return hipGetLastError();
}
