// Fused softmax cross-entropy over a (padded) vocabulary, bf16 logits.
//
// forward : one 256-thread block per row; a single pass keeps an online
//           (max, sum-exp) pair per lane over 16-byte bf16x8 loads, combines
//           them across the block, and writes loss[row] and lse[row].
// backward: dlogits = (softmax - onehot) * grad_out[0] * inv_count, read from
//           the device scalar so no host sync is needed; columns >= V (vocab
//           padding) and rows whose target == ignore_index get zero gradient.
//
// Versus torch's log_softmax + nll_loss this never materialises fp32
// probabilities: 1 read in forward, 1 read + 1 write in backward.
#include "common.h"

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

__global__ __launch_bounds__(256) void xent_fwd_kernel(const bf16_t* __restrict__ logits,
                                                       const long* __restrict__ targets,
                                                       float* __restrict__ loss,
                                                       float* __restrict__ lse, int V, int Vp,
                                                       long ignore_index) {
  const int row = blockIdx.x;
  const bf16_t* lr = logits + (size_t)row * Vp;
  float m = -INFINITY, s = 0.f;
  const int V8 = V / 8;
  for (int c8 = threadIdx.x; c8 < V8; c8 += 256) {
    float v[8];
    unpack8(reinterpret_cast<const uint4*>(lr)[c8], v);
    float bm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) bm = fmaxf(bm, v[j]);
    const float mn = fmaxf(m, bm);
    float acc = s * __expf(m - mn);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(v[j] - mn);
    s = acc;
    m = mn;
  }
  for (int c = V8 * 8 + threadIdx.x; c < V; c += 256) {
    const float v = bf2f(lr[c]);
    const float mn = fmaxf(m, v);
    s = s * __expf(m - mn) + __expf(v - mn);
    m = mn;
  }
  // wave-level combine
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
  __shared__ float sm[4], ss[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < 4; ++i) online_merge(M, S, sm[i], ss[i]);
    const float l = logf(S) + M;
    lse[row] = l;
    const long t = targets[row];
    loss[row] = (t == ignore_index || t < 0 || t >= V) ? 0.f : (l - bf2f(lr[t]));
  }
}

__global__ __launch_bounds__(256) void xent_bwd_kernel(const bf16_t* __restrict__ logits,
                                                       const long* __restrict__ targets,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ grad_out,
                                                       float inv_count, bf16_t* __restrict__ dl,
                                                       int V, int Vp, long ignore_index) {
  const int row = blockIdx.x;
  const long t = targets[row];
  const bool ign = (t == ignore_index || t < 0 || t >= V);
  const float scale = ign ? 0.f : grad_out[0] * inv_count;
  const float l = lse[row];
  const bf16_t* lr = logits + (size_t)row * Vp;
  bf16_t* dr = dl + (size_t)row * Vp;
  const int Vp8 = Vp / 8;
  for (int c8 = threadIdx.x; c8 < Vp8; c8 += 256) {
    float v[8], o[8];
    unpack8(reinterpret_cast<const uint4*>(lr)[c8], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c8 * 8 + j;
      float p = (c < V) ? __expf(v[j] - l) : 0.f;
      if (c == t) p -= 1.f;
      o[j] = p * scale;
    }
    reinterpret_cast<uint4*>(dr)[c8] = pack8(o);
  }
}

RA_EXPORT int ra_xent_fwd(const void* logits, const long* targets, float* loss, float* lse,
                          int N, int V, int Vp, long ignore_index, hipStream_t st) {
  if (Vp % 8 || V > Vp) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(N), dim3(256), 0, st, (const bf16_t*)logits, targets,
                     loss, lse, V, Vp, ignore_index);
  return hipGetLastError();
}

RA_EXPORT int ra_xent_bwd(const void* logits, const long* targets, const float* lse,
                          const float* grad_out, float inv_count, void* dlogits, int N, int V,
                          int Vp, long ignore_index, hipStream_t st) {
  if (Vp % 8 || V > Vp) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(N), dim3(256), 0, st, (const bf16_t*)logits, targets,
                     lse, grad_out, inv_count, (bf16_t*)dlogits, V, Vp, ignore_index);
  return hipGetLastError();
}
