// Fused GEMM epilogues for the GPT-2 MLP / projections, bf16 in and out.
//
//   ra_bias_gelu_fwd   y  = gelu_tanh(h + bias)
//   ra_bias_gelu_bwd   dh = dy * gelu_tanh'(h + bias);  dbias = sum_rows(dh)
//   ra_bias_residual   y  = res + h + bias
//   ra_colsum_bf16     out = sum_rows(x)     (bias gradient of a projection)
//   ra_bias_relu_fwd   y  = relu(h + bias)   (conv / linear epilogue, rows = NHWC pixels)
//   ra_relu_bwd_bias   dh = dy * (y > 0);  dbias = sum_rows(dh)   (two launches)
//
// The GEMM itself stays on hipBLASLt (plain library GEMM); these kernels fuse
// everything around it into one HBM pass. Each thread moves 8 bf16 (16 bytes);
// column reductions keep 8 fp32 partials per thread in registers over a row
// chunk and finish with `colsum` over P partial rows.
#include "common.h"

typedef unsigned v4u32_t __attribute__((ext_vector_type(4)));

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
template <bool RELU>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const bf16_t* __restrict__ h,
                                                           const bf16_t* __restrict__ bias,
                                                           bf16_t* __restrict__ y, int n8,
                                                           int F8) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const int c8 = (int)((unsigned)i % (unsigned)F8);
    float hv[8], bv[8], o[8];
    unpack8(reinterpret_cast<const uint4*>(h)[i], hv);
    unpack8(reinterpret_cast<const uint4*>(bias)[c8], bv);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = RELU ? fmaxf(hv[j] + bv[j], 0.f) : gelu_tanh(hv[j] + bv[j], nullptr);
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

// v2 of the above, used whenever the chunk fits 32-bit offsets: the chunk [r0, r1) is addressed
// through buffer resources that END at r1, so rows past the chunk load zeros and their
// stores are dropped -- the loop has no guards and no break. v1's guarded batch made the
// compiler sink every load to its use: one full memory round trip per row per wave.
// Rows alternate between two register sets, so the next row's loads are in flight while
// one is reduced (K row pairs per loop iteration).
template <bool GELU, int K>
__global__ __launch_bounds__(64) void bwd_colpart2_kernel(const bf16_t* __restrict__ dy,
                                                          const bf16_t* __restrict__ h,
                                                          const bf16_t* __restrict__ bias,
                                                          bf16_t* __restrict__ dh,
                                                          float* __restrict__ part, int N,
                                                          int F8, int rows_per_part) {
  const int c8 = blockIdx.x * blockDim.x + threadIdx.x;
  if (c8 >= F8) return;
  const int r0 = blockIdx.y * rows_per_part;
  const int r1 = min(N, r0 + rows_per_part);
  const int nrows = r1 > r0 ? r1 - r0 : 0;
  const size_t base = (size_t)r0 * F8 * 16;  // bytes
  const int bytes = nrows * F8 * 16;
  const auto rDY = __builtin_amdgcn_make_buffer_rsrc((char*)dy + base, 0, bytes, 0x00020000);
  const auto rH = __builtin_amdgcn_make_buffer_rsrc((char*)h + (GELU ? base : 0), 0,
                                                    GELU ? bytes : 0, 0x00020000);
  const auto rDH = __builtin_amdgcn_make_buffer_rsrc((char*)dh + (GELU ? base : 0), 0,
                                                     GELU ? bytes : 0, 0x00020000);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  float bv[8];
  if (GELU) unpack8(reinterpret_cast<const uint4*>(bias)[c8], bv);
  struct Row {
    uint4 d, h;
  };
  auto load = [&](Row& b, int rr) __attribute__((always_inline)) {
    const int off = (rr * F8 + c8) * 16;
    b.d = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rDY, off, 0, 0));
    if (GELU) b.h = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rH, off, 0, 0));
  };
  auto compute = [&](const Row& b, int rr) __attribute__((always_inline)) {
    float d[8];
    unpack8(b.d, d);
    if (GELU) {
      float hv[8], o[8];
      unpack8(b.h, hv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float dg;
        gelu_tanh(hv[j] + bv[j], &dg);
        o[j] = d[j] * dg;
        acc[j] += o[j];
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, pack8(o)), rDH,
                                             (rr * F8 + c8) * 16, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += d[j];
    }
  };
  // K row pairs per iteration through two register sets (A: even rows, B: odd rows)
  const int iters = (nrows + 2 * K - 1) / (2 * K);
  Row A, B;
  if (iters > 0) load(A, 0);
  int rr = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < K; ++k, rr += 2) {
      load(B, rr + 1);  // past the chunk: zeros, stores dropped
      __builtin_amdgcn_sched_barrier(0);
      compute(A, rr);
      __builtin_amdgcn_sched_barrier(0);
      load(A, rr + 2);
      __builtin_amdgcn_sched_barrier(0);
      compute(B, rr + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float* pr = part + (size_t)blockIdx.y * F8 * 8 + (size_t)c8 * 8;
  *reinterpret_cast<float4*>(pr) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(pr + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// ReLU backward + bias-gradient partials for NARROW rows (F8 divides 256: conv channel
// counts 32/64/..., F <= 2048). A 256-thread block covers 256/F8 rows per step, so every
// lane is busy even at F = 32 (the wide-row kernel above would run 4 of 64 lanes).
// part[blockIdx.x][F] = column sums of dh over this block's rows.
__global__ __launch_bounds__(256) void relu_bwd_rows_kernel(const bf16_t* __restrict__ dy,
                                                            const bf16_t* __restrict__ y,
                                                            bf16_t* __restrict__ dh,
                                                            float* __restrict__ part, int N,
                                                            int F8, int rows_per_block) {
  __shared__ float red[256 * 8];
  const int t = threadIdx.x, c8 = t % F8, rs = t / F8, RPI = 256 / F8;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(N, r0 + rows_per_block);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const uint4* dy4 = reinterpret_cast<const uint4*>(dy);
  const uint4* y4 = reinterpret_cast<const uint4*>(y);
  constexpr int RB = 4;
  for (int rb = r0 + rs; rb < r1; rb += RB * RPI) {
    uint4 dv[RB], yv[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int r = rb + k * RPI < r1 ? rb + k * RPI : rb;
      const long ix = (long)r * F8 + c8;
      dv[k] = dy4[ix];
      yv[k] = y4[ix];
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int r = rb + k * RPI;
      if (r >= r1) break;
      float d[8], o[8];
      unpack8(dv[k], d);
      const uint32_t w[4] = {yv[k].x, yv[k].y, yv[k].z, yv[k].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // bf16 > 0 <=> sign bit clear and not +0 (ReLU outputs are never negative or NaN)
        const uint32_t b = (j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xffffu);
        o[j] = b != 0 && b < 0x8000u ? d[j] : 0.f;
        acc[j] += o[j];
      }
      reinterpret_cast<uint4*>(dh)[(long)r * F8 + c8] = pack8(o);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t * 8 + j] = acc[j];
  __syncthreads();
  const int F = F8 * 8;
  for (int c = t; c < F; c += 256) {
    float s = 0.f;
    for (int q = 0; q < RPI; ++q) s += red[(q * F8 + (c >> 3)) * 8 + (c & 7)];
    part[(size_t)blockIdx.x * F + c] = s;
  }
}

// out[c] (+)= sum_p part[p][c]: grid ceil(F/64) blocks of 64 columns x 16 row lanes
// (a single block serves F <= 64, so the row walk must be short and wide).
template <bool OUT_BF16, bool ACC>
__global__ __launch_bounds__(1024) void colsum_final_kernel(const float* __restrict__ part,
                                                            void* out, int P, int F) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s0 = 0.f, s1 = 0.f;
  if (c < F) {
    int p = ty;
    for (; p + 16 < P; p += 32) {
      s0 += part[(size_t)p * F + c];
      s1 += part[(size_t)(p + 16) * F + c];
    }
    if (p < P) s0 += part[(size_t)p * F + c];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty != 0 || c >= F) return;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += red[q][tx];
  if (OUT_BF16) {
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + c;
    *o = f2bf(ACC ? s + bf2f(*o) : s);
  } else {
    float* o = reinterpret_cast<float*>(out) + c;
    *o = ACC ? *o + s : s;
  }
}

static inline int relu_rows_per_block(int N, int F8) {
  const int RPI = 256 / F8;
  int rpb = (N + 511) / 512;                   // <= 512 partial rows
  rpb = (rpb + RPI - 1) / RPI * RPI;           // whole block steps
  return rpb < RPI ? RPI : rpb;
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

// Row partitions of a column reduction: enough (64-thread) blocks to put ~8192
// waves on the chip (8192 = 32 per CU) whatever F is (F = 768 gives only 2 column
// blocks), >= 32 rows per partial.
static inline int parts_for(int N, int F) {
  const int bx = (F / 8 + 63) / 64;
  int p = (8192 + bx - 1) / bx;
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
  hipLaunchKernelGGL(bias_act_fwd_kernel<false>, dim3(ra_grid(n8, 256)), dim3(256), 0, st,
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
  if ((long)rpp * F8 * 16 < (1L << 31))
    hipLaunchKernelGGL((bwd_colpart2_kernel<true, 1>), dim3((F8 + 63) / 64, P), dim3(64), 0, st,
                       (const bf16_t*)dy, (const bf16_t*)h, (const bf16_t*)bias, (bf16_t*)dh,
                       work, N, F8, rpp);
  else
    hipLaunchKernelGGL(bwd_colpart_kernel<true>, dim3((F8 + 63) / 64, P), dim3(64), 0, st,
                       (const bf16_t*)dy, (const bf16_t*)h, (const bf16_t*)bias, (bf16_t*)dh,
                       work, N, F8, rpp);
  colsum_launch(work, work + (size_t)P * F, dbias, P, F, sink_flags(flags), st);
  return hipGetLastError();
}

RA_EXPORT int ra_colsum_bf16(const void* x, void* out, float* work, int N, int F, int flags,
                             hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const int P = parts_for(N, F), F8 = F / 8;
  const int rpp = (N + P - 1) / P;
  if ((long)rpp * F8 * 16 < (1L << 31))
    hipLaunchKernelGGL((bwd_colpart2_kernel<false, 1>), dim3((F8 + 63) / 64, P), dim3(64), 0,
                       st, (const bf16_t*)x, nullptr, nullptr, nullptr, work, N, F8, rpp);
  else
    hipLaunchKernelGGL(bwd_colpart_kernel<false>, dim3((F8 + 63) / 64, P), dim3(64), 0, st,
                       (const bf16_t*)x, nullptr, nullptr, nullptr, work, N, F8, rpp);
  colsum_launch(work, work + (size_t)P * F, out, P, F, sink_flags(flags), st);
  return hipGetLastError();
}

RA_EXPORT int ra_bias_relu_fwd(const void* h, const void* bias, void* y, long N, int F,
                               hipStream_t st) {
  if (F % 8) return hipErrorInvalidValue;
  const long n8 = N * (long)F / 8;
  if (n8 >= (1L << 31) - 65536L * 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bias_act_fwd_kernel<true>, dim3(ra_grid(n8, 256)), dim3(256), 0, st,
                     (const bf16_t*)h, (const bf16_t*)bias, (bf16_t*)y, (int)n8, F / 8);
  return hipGetLastError();
}

// fp32 workspace (floats) for ra_relu_bwd_bias
RA_EXPORT long ra_relu_bwd_work(int N, int F) {
  const int F8 = F / 8;
  if (F % 8 || 256 % F8) return -1;
  const int rpb = relu_rows_per_block(N, F8);
  return (long)((N + rpb - 1) / rpb) * F;
}

// dh = dy * (y > 0), dbias (+)= sum_rows(dh); flags as sink_flags (bit0 accumulate,
// bit1 fp32 destination). Narrow rows only (F8 | 256); work: ra_relu_bwd_work floats.
RA_EXPORT int ra_relu_bwd_bias(const void* dy, const void* y, void* dh, void* dbias,
                               float* work, int N, int F, int flags, hipStream_t st) {
  const int F8 = F / 8;
  if (F % 8 || 256 % F8 || N <= 0) return hipErrorInvalidValue;
  const int rpb = relu_rows_per_block(N, F8);
  const int P = (N + rpb - 1) / rpb;
  hipLaunchKernelGGL(relu_bwd_rows_kernel, dim3(P), dim3(256), 0, st, (const bf16_t*)dy,
                     (const bf16_t*)y, (bf16_t*)dh, work, N, F8, rpb);
  const dim3 g((F + 63) / 64), b(1024);
  switch (((flags & 1) ? 2 : 0) | ((flags & 2) ? 0 : 1)) {
    case 0: hipLaunchKernelGGL((colsum_final_kernel<false, false>), g, b, 0, st, work, dbias, P, F); break;
    case 1: hipLaunchKernelGGL((colsum_final_kernel<true, false>), g, b, 0, st, work, dbias, P, F); break;
    case 2: hipLaunchKernelGGL((colsum_final_kernel<false, true>), g, b, 0, st, work, dbias, P, F); break;
    default: hipLaunchKernelGGL((colsum_final_kernel<true, true>), g, b, 0, st, work, dbias, P, F);
  }
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
