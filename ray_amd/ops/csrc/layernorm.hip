// Fused LayerNorm forward/backward for bf16 activations (fp32 statistics).
//
// Forward: one wave64 per row, 4 rows per 256-thread block; each lane holds
// VPL x 4 elements in registers (8-byte bf16x4 loads), so the row is read from
// HBM exactly once and mean/var are two in-register passes + wave shuffles.
// Backward: each wave walks rows grid-stride, accumulating dgamma/dbeta per lane
// in registers; waves combine through LDS atomics and write one fp32 partial row
// per block; `colsum_partials` finishes the column reduction.
//
// Replaces torch.nn.functional.layer_norm (used by GPT-2 blocks, reference
// workload: release/train_tests + train/examples GPT-2 DDP).
#include "common.h"

template <int VPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ g,
                                                     const bf16_t* __restrict__ b,
                                                     bf16_t* __restrict__ y,
                                                     float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int N, int D,
                                                     float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const bf16_t* xr = x + (size_t)row * D;
  float v[VPL][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
      unpack4(*reinterpret_cast<const uint2*>(xr + col), v[i]);
    } else {
      v[i][0] = v[i][1] = v[i][2] = v[i][3] = 0.f;
    }
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float invD = 1.f / (float)D;
  const float mu = wave_sum(s) * invD;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mu;
        q += d * d;
      }
    }
  }
  const float rs = rsqrtf(wave_sum(q) * invD + eps);
  bf16_t* yr = y + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
      float gg[4], bb[4], o[4];
      unpack4(*reinterpret_cast<const uint2*>(g + col), gg);
      unpack4(*reinterpret_cast<const uint2*>(b + col), bb);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mu) * rs * gg[j] + bb[j];
      *reinterpret_cast<uint2*>(yr + col) = pack4(o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

template <int VPL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ dg_part,
    float* __restrict__ db_part, int N, int D) {
  // dres (optional): gradient arriving at x through the residual branch, added into dx here
  // so the two gradients of the residual stream are summed in this pass (no separate add)
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2][D]
  float* sdg = lds;
  float* sdb = lds + D;
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float gg[VPL][4], adg[VPL][4], adb[VPL][4];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) unpack4(*reinterpret_cast<const uint2*>(g + col), gg[i]);
    else gg[i][0] = gg[i][1] = gg[i][2] = gg[i][3] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) adg[i][j] = adb[i][j] = 0.f;
  }
  const float invD = 1.f / (float)D;
  for (int row = blockIdx.x * 4 + w; row < N; row += gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    float xh[VPL][4], wd[VPL][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int col = (i * 64 + lane) * 4;
      float xv[4], dv[4];
      if (col < D) {
        unpack4(*reinterpret_cast<const uint2*>(x + (size_t)row * D + col), xv);
        unpack4(*reinterpret_cast<const uint2*>(dy + (size_t)row * D + col), dv);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[j] = dv[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[i][j] = (xv[j] - mu) * rs;
        wd[i][j] = dv[j] * gg[i][j];
        s1 += wd[i][j];
        s2 += wd[i][j] * xh[i][j];
        adg[i][j] += dv[j] * xh[i][j];
        adb[i][j] += dv[j];
      }
    }
    const float c1 = wave_sum(s1) * invD;
    const float c2 = wave_sum(s2) * invD;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int col = (i * 64 + lane) * 4;
      if (col < D) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (wd[i][j] - c1 - xh[i][j] * c2) * rs;
        if (dres) {
          float r[4];
          unpack4(*reinterpret_cast<const uint2*>(dres + (size_t)row * D + col), r);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] += r[j];
        }
        *reinterpret_cast<uint2*>(dx + (size_t)row * D + col) = pack4(o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        atomicAdd(&sdg[col + j], adg[i][j]);
        atomicAdd(&sdb[col + j], adb[i][j]);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    dg_part[(size_t)blockIdx.x * D + i] = sdg[i];
    db_part[(size_t)blockIdx.x * D + i] = sdb[i];
  }
}

#define LN_DISPATCH(MACRO)                       \
  switch ((D + 255) / 256) {                     \
    case 1: MACRO(1); break;                     \
    case 2: MACRO(2); break;                     \
    case 3: MACRO(3); break;                     \
    case 4: MACRO(4); break;                     \
    case 5: MACRO(5); break;                     \
    case 6: MACRO(6); break;                     \
    case 7: MACRO(7); break;                     \
    case 8: MACRO(8); break;                     \
    case 12: MACRO(12); break;                   \
    case 16: MACRO(16); break;                   \
    default: return hipErrorInvalidValue;        \
  }

RA_EXPORT int ra_layernorm_fwd(const void* x, const void* g, const void* b, void* y, float* mean,
                               float* rstd, int N, int D, float eps, hipStream_t st) {
  if (D % 4 != 0) return hipErrorInvalidValue;
  dim3 grid((N + 3) / 4);
#define L(V)                                                                                  \
  hipLaunchKernelGGL(ln_fwd_kernel<V>, grid, dim3(256), 0, st, (const bf16_t*)x,              \
                     (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, mean, rstd, N, D, eps)
  LN_DISPATCH(L)
#undef L
  return hipGetLastError();
}

// Partial-row count for the backward (1024 blocks x 4 waves fill 256 CUs 4-deep).
RA_EXPORT int ra_layernorm_bwd_parts(int N) {
  int p = (N + 3) / 4;
  return p < 1024 ? p : 1024;
}

// fp32 workspace (in floats) required by ra_layernorm_bwd.
RA_EXPORT long ra_layernorm_bwd_work(int N, int D) {
  return 2L * ra_layernorm_bwd_parts(N) * D + 2L * kColsumSplits * D;
}

RA_EXPORT int ra_layernorm_bwd(const void* dy, const void* x, const void* g, const float* mean,
                               const float* rstd, const void* dres, void* dx, void* dg, void* db,
                               float* work,
                               int N, int D, int flags, hipStream_t st) {
  // flags: bit0 bf16 dg/db, bit1 accumulate dg/db into the (flat) gradient buffers
  if (D % 4 != 0) return hipErrorInvalidValue;
  const int P = ra_layernorm_bwd_parts(N);
  float* dgp = work;
  float* dbp = work + (size_t)P * D;
  float* scr = work + 2 * (size_t)P * D;
  const size_t lds = 2 * (size_t)D * sizeof(float);
#define L(V)                                                                                  \
  hipLaunchKernelGGL(ln_bwd_kernel<V>, dim3(P), dim3(256), lds, st, (const bf16_t*)dy,        \
                     (const bf16_t*)x, (const bf16_t*)g, mean, rstd, (const bf16_t*)dres,      \
                     (bf16_t*)dx, dgp, dbp, N, D)
  LN_DISPATCH(L)
#undef L
  colsum_launch(dgp, scr, dg, P, D, flags, st);
  colsum_launch(dbp, scr + (size_t)kColsumSplits * D, db, P, D, flags, st);
  return hipGetLastError();
}

// out[c] = sum_p part[p][c]; scratch: kColsumSplits * D floats.
RA_EXPORT int ra_colsum(const float* part, float* scratch, void* out, int P, int D, int flags,
                        hipStream_t st) {
  colsum_launch(part, scratch, out, P, D, flags, st);
  return hipGetLastError();
}
