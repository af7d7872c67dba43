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

// RES: the row is x = h + bias + skip (pre-LN residual add of the previous sub-block,
// fused: x is computed once, written once (the next residual input) and normalised)
template <int VPL, bool RES>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ rbias,
                                                     const bf16_t* __restrict__ skip,
                                                     bf16_t* __restrict__ xout,
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
      if (RES) {
        float sk[4], bb[4] = {0.f, 0.f, 0.f, 0.f};
        unpack4(*reinterpret_cast<const uint2*>(skip + (size_t)row * D + col), sk);
        if (rbias) unpack4(*reinterpret_cast<const uint2*>(rbias + col), bb);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] += bb[j] + sk[j];
        const uint2 packed = pack4(v[i]);
        *reinterpret_cast<uint2*>(xout + (size_t)row * D + col) = packed;
        unpack4(packed, v[i]);  // normalise exactly the bf16 values the next layer sees
      }
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

// Backward. dres (optional): gradient reaching x through the skip connection, added into
// dx here (the residual stream's two gradients summed in this pass). NP = 3 also emits
// the column sums of dx itself: the bias gradient of the residual add that produced x.
// Each wave handles two rows per iteration (twice the loads in flight per wave).
template <int VPL, int NP>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ part, int N,
    int D) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [NP][D]
  for (int i = threadIdx.x; i < NP * D; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float gg[VPL][4], acc[NP][VPL][4];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) unpack4(*reinterpret_cast<const uint2*>(g + col), gg[i]);
    else gg[i][0] = gg[i][1] = gg[i][2] = gg[i][3] = 0.f;
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[k][i][j] = 0.f;
  }
  const float invD = 1.f / (float)D;
  const int stride = gridDim.x * 4;
  const int step = 2 * stride;
  // software pipeline: the next row pair's raw (packed bf16) loads are issued before the
  // current pair is reduced, so each wave keeps two pairs of rows in flight
  uint2 rx[2][VPL], rd[2][VPL], rr[2][VPL];
  float rmu[2], rrs[2];  // the row statistics travel with the prefetched rows
  auto load_pair = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = r0 + u * stride;
      if (row < N) {
        rmu[u] = mean[row];
        rrs[u] = rstd[row];
      }
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int col = (i * 64 + lane) * 4;
        if (row < N && col < D) {
          const size_t o = (size_t)row * D + col;
          rx[u][i] = *reinterpret_cast<const uint2*>(x + o);
          rd[u][i] = *reinterpret_cast<const uint2*>(dy + o);
          if (dres) rr[u][i] = *reinterpret_cast<const uint2*>(dres + o);
        }
      }
    }
  };
  constexpr bool PF = VPL <= 8;  // wider rows: the doubled register set would spill
  int r0 = blockIdx.x * 4 + w;
  if (PF && r0 < N) load_pair(r0);
  for (; r0 < N; r0 += step) {
    if (!PF) load_pair(r0);
    const int rows[2] = {r0, r0 + stride};
    float xv[2][VPL][4], dv[2][VPL][4], rv[2][VPL][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool ok = rows[u] < N;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int col = (i * 64 + lane) * 4;
        if (ok && col < D) {
          unpack4(rx[u][i], xv[u][i]);
          unpack4(rd[u][i], dv[u][i]);
          if (dres) unpack4(rr[u][i], rv[u][i]);
          else rv[u][i][0] = rv[u][i][1] = rv[u][i][2] = rv[u][i][3] = 0.f;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) xv[u][i][j] = dv[u][i][j] = rv[u][i][j] = 0.f;
        }
      }
    }
    const float cmu[2] = {rmu[0], rmu[1]}, crs[2] = {rrs[0], rrs[1]};
    if (PF && r0 + step < N) load_pair(r0 + step);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (rows[u] >= N) break;
      const float mu = cmu[u], rs = crs[u];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < VPL; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = (xv[u][i][j] - mu) * rs;
          const float wd = dv[u][i][j] * gg[i][j];
          xv[u][i][j] = xh;
          s1 += wd;
          s2 += wd * xh;
          acc[0][i][j] += dv[u][i][j] * xh;
          acc[1][i][j] += dv[u][i][j];
        }
      const float c1 = wave_sum(s1) * invD;
      const float c2 = wave_sum(s2) * invD;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int col = (i * 64 + lane) * 4;
        if (col < D) {
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            o[j] = (dv[u][i][j] * gg[i][j] - c1 - xv[u][i][j] * c2) * rs + rv[u][i][j];
            if (NP == 3) acc[NP - 1][i][j] += o[j];
          }
          *reinterpret_cast<uint2*>(dx + (size_t)rows[u] * D + col) = pack4(o);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
#pragma unroll
      for (int k = 0; k < NP; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(&lds[k * D + col + j], acc[k][i][j]);
    }
  }
  __syncthreads();
  const size_t P = gridDim.x;
  for (int i = threadIdx.x; i < NP * D; i += blockDim.x) {
    const int k = i / D, c = i - k * D;
    part[((size_t)k * P + blockIdx.x) * D + c] = lds[i];
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
  hipLaunchKernelGGL((ln_fwd_kernel<V, false>), grid, dim3(256), 0, st, (const bf16_t*)x,     \
                     nullptr, nullptr, nullptr, (const bf16_t*)g, (const bf16_t*)b,           \
                     (bf16_t*)y, mean, rstd, N, D, eps)
  LN_DISPATCH(L)
#undef L
  return hipGetLastError();
}

// xout = h + rbias + skip (rbias may be null); y = LayerNorm(xout)
RA_EXPORT int ra_residual_layernorm_fwd(const void* h, const void* rbias, const void* skip,
                                        void* xout, const void* g, const void* b, void* y,
                                        float* mean, float* rstd, int N, int D, float eps,
                                        hipStream_t st) {
  if (D % 4 != 0) return hipErrorInvalidValue;
  dim3 grid((N + 3) / 4);
#define L(V)                                                                                  \
  hipLaunchKernelGGL((ln_fwd_kernel<V, true>), grid, dim3(256), 0, st, (const bf16_t*)h,      \
                     (const bf16_t*)rbias, (const bf16_t*)skip, (bf16_t*)xout,                \
                     (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, mean, rstd, N, D, eps)
  LN_DISPATCH(L)
#undef L
  return hipGetLastError();
}

int ra_knobs[8] = {512, 8192, 1, 0, 0, 0, 0, 0};

RA_EXPORT int ra_set_knob(int k, int v) {
  if (k < 0 || k >= 8) return hipErrorInvalidValue;
  ra_knobs[k] = v;
  return hipSuccess;
}

// Partial-row count for the backward: up to ra_knobs[0] blocks, each wave >= 2 rows.
// Measured at 65536 x 768 (profiles/r2_perf_bench.log, "norm"): 512 blocks beat 1024 /
// 2048 / 4096 — more blocks only add partial-slab traffic and LDS-atomic tails.
RA_EXPORT int ra_layernorm_bwd_parts(int N) {
  int p = (N + 7) / 8;
  const int cap = ra_knobs[0] > 0 ? ra_knobs[0] : 2048;
  return p < cap ? p : cap;
}

// fp32 workspace (in floats) required by ra_layernorm_bwd (3 partial slabs + scratch).
RA_EXPORT long ra_layernorm_bwd_work(int N, int D) {
  return 3L * ra_layernorm_bwd_parts(N) * D + 3L * kColsumSplits * D;
}

// dbias (optional): column sums of dx (bias grad of the residual add that produced x).
// flags: bit0 bf16 dg/db/dbias, bit1 accumulate them into (flat) gradient buffers.
RA_EXPORT int ra_layernorm_bwd(const void* dy, const void* x, const void* g, const float* mean,
                               const float* rstd, const void* dres, void* dx, void* dg, void* db,
                               void* dbias, float* work, int N, int D, int flags,
                               hipStream_t st) {
  if (D % 4 != 0) return hipErrorInvalidValue;
  const int P = ra_layernorm_bwd_parts(N);
  const int NP = dbias ? 3 : 2;
  float* scr = work + (size_t)NP * P * D;
  const size_t lds = (size_t)NP * D * sizeof(float);
#define L(V)                                                                                  \
  if (NP == 3)                                                                                \
    hipLaunchKernelGGL((ln_bwd_kernel<V, 3>), dim3(P), dim3(256), lds, st, (const bf16_t*)dy, \
                       (const bf16_t*)x, (const bf16_t*)g, mean, rstd, (const bf16_t*)dres,   \
                       (bf16_t*)dx, work, N, D);                                              \
  else                                                                                        \
    hipLaunchKernelGGL((ln_bwd_kernel<V, 2>), dim3(P), dim3(256), lds, st, (const bf16_t*)dy, \
                       (const bf16_t*)x, (const bf16_t*)g, mean, rstd, (const bf16_t*)dres,   \
                       (bf16_t*)dx, work, N, D);
  LN_DISPATCH(L)
#undef L
  void* outs[3] = {dg, db, dbias};
  for (int k = 0; k < NP; ++k)
    colsum_launch(work + (size_t)k * P * D, scr + (size_t)k * kColsumSplits * D, outs[k], P, D,
                  flags, st);
  return hipGetLastError();
}

// out[c] = sum_p part[p][c]; scratch: kColsumSplits * D floats.
RA_EXPORT int ra_colsum(const float* part, float* scratch, void* out, int P, int D, int flags,
                        hipStream_t st) {
  colsum_launch(part, scratch, out, P, D, flags, st);
  return hipGetLastError();
}
