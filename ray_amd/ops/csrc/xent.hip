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

// ---------------------------------------------------------------------------------------
// Fused LM-head cross-entropy chunk (forward AND backward in one pass, in place).
//
// The LM head runs token-chunk by token-chunk (ops.functional.lm_head_cross_entropy):
//   logits_c = h_c @ W^T (hipBLASLt) -> THIS KERNEL -> dh_c = dlogits_c @ W,
//   dW += dlogits_c^T @ h_c (hipBLASLt, fp32 accumulate)
// so the [tokens, vocab] logits tensor (6.6 GB at 64x1024 tokens x 50304) never exists
// whole. Each 512-thread block owns one row and keeps it in REGISTERS (NV 16-byte
// vectors per lane: 8 waves x 64 lanes x NV x 8 = up to 65536 columns), so the row is
// read from HBM/MALL once and overwritten once with
//   dlogits = (softmax(row) - onehot(target)) * inv_count     (0 on padding columns)
// and loss[row] = lse - row[target]. inv_count is a device scalar (no host sync).
//
// VALU diet (the kernel is VALU- as much as HBM-bound at 50304 columns): the max pass
// is unpack+max; the sum pass computes e = exp2(v*log2e - m*log2e) ONCE and keeps it,
// re-packed to bf16, in the same registers; the output pass is one multiply per element.
// Column bounds are checked per 8-wide vector, not per element, and the target column
// is patched by its owning lane from the fp32 target logit (p_t - 1 must not lose the
// cancellation to a bf16-rounded e).
template <int NV>
__global__ __launch_bounds__(512) void xent_fused_kernel(bf16_t* __restrict__ logits,
                                                         const long* __restrict__ targets,
                                                         const float* __restrict__ inv_count,
                                                         float* __restrict__ loss, int V, int Vp,
                                                         long ignore_index) {
  __shared__ float red[8];
  __shared__ float tlogit;
  const int row = blockIdx.x;
  bf16_t* lr = logits + (size_t)row * Vp;
  const long t = targets[row];
  const bool ign = (t == ignore_index || t < 0 || t >= V);
  if (threadIdx.x == 0) tlogit = ign ? 0.f : bf2f(lr[t]);  // read before any overwrite
  const int Vp8 = Vp >> 3;
  const int Vfull = V >> 3;  // vectors [0, Vfull) hold only real columns
  uint4 raw[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c8 = k * 512 + threadIdx.x;
    if (c8 < Vp8) raw[k] = reinterpret_cast<const uint4*>(lr)[c8];
  }
  // vector-level masks: partial vector (the one holding column V-1 when V % 8) and
  // all-padding vectors get per-element / zero treatment
  auto masked = [&](int c8, float (&v)[8]) __attribute__((always_inline)) {
    if (c8 >= Vfull) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c8 * 8 + j >= V) v[j] = -INFINITY;
    }
  };
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c8 = k * 512 + threadIdx.x;
    if (c8 < Vp8) {
      float v[8];
      unpack8(raw[k], v);
      masked(c8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, v[j]);
    }
  }
  m = block_max<8>(m, red);
  const float L2E = 1.4426950408889634f;
  const float mb = m * L2E;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c8 = k * 512 + threadIdx.x;
    if (c8 < Vp8) {
      float v[8];
      unpack8(raw[k], v);
      masked(c8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = __builtin_amdgcn_exp2f(fmaf(v[j], L2E, -mb));  // exp(-inf) = 0 on padding
        s += v[j];
      }
      raw[k] = pack8(v);
    }
  }
  s = block_sum<8>(s, red);
  const float lse = m + __logf(s);
  const float scale = ign ? 0.f : *inv_count;
  const float c = scale / s;
  const int tv = ign ? -1 : (int)(t >> 3);
  const float pt_grad = (__expf(tlogit - lse) - 1.f) * scale;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c8 = k * 512 + threadIdx.x;
    if (c8 < Vp8) {
      float o[8];
      unpack8(raw[k], o);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] *= c;
      if (c8 == tv) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j == (int)(t & 7)) o[j] = pt_grad;
      }
      reinterpret_cast<uint4*>(lr)[c8] = pack8(o);
    }
  }
  if (threadIdx.x == 0) loss[row] = ign ? 0.f : lse - tlogit;
}

// logits: [N, Vp] bf16, overwritten with dlogits. loss: [N] fp32 (per-row, unscaled).
RA_EXPORT int ra_xent_fused(void* logits, const long* targets, const float* inv_count,
                            float* loss, int N, int V, int Vp, long ignore_index,
                            hipStream_t st) {
  if (Vp % 8 || V > Vp || N <= 0) return hipErrorInvalidValue;
  const int per = (Vp / 8 + 511) / 512;
#define X(NV)                                                                                 \
  hipLaunchKernelGGL((xent_fused_kernel<NV>), dim3(N), dim3(512), 0, st, (bf16_t*)logits,     \
                     targets, inv_count, loss, V, Vp, ignore_index)
  if (per <= 2) X(2);
  else if (per <= 4) X(4);
  else if (per <= 8) X(8);
  else if (per <= 13) X(13);
  else if (per <= 16) X(16);
  else return hipErrorInvalidValue;
#undef X
  return hipGetLastError();
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
