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

typedef unsigned v2u32_t __attribute__((ext_vector_type(2)));

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

// Wave-wide sum without LDS: DPP within each 16-lane row (xor 1, xor 2, half-row mirror,
// row mirror), then the gfx950 permlane16/32 swaps across rows (v1's __shfl_xor is six
// ds_bpermute round trips through LDS per reduction).
#define RA_DPP(v, ctrl) \
  __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, false))
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += RA_DPP(v, 0xB1);   // quad_perm [1,0,3,2]
  v += RA_DPP(v, 0x4E);   // quad_perm [2,3,0,1]
  v += RA_DPP(v, 0x141);  // row_half_mirror
  v += RA_DPP(v, 0x140);  // row_mirror
  const int lane = threadIdx.x & 63;
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto s16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v += __builtin_bit_cast(float, (lane & 16) ? s16[0] : s16[1]);
  const unsigned u2 = __builtin_bit_cast(unsigned, v);
  const auto s32 = __builtin_amdgcn_permlane32_swap(u2, u2, false, false);
  v += __builtin_bit_cast(float, (lane & 32) ? s32[0] : s32[1]);
  return v;
}

// Backward v2, for D == VPL * 256 (each lane owns VPL x 4 columns, no column guards) and
// tensors under 2 GiB: rows are read and written through buffer resources, so a row past
// N loads zeros and its store is dropped and the main loop has no branches. v1's guarded
// loads/stores made the compiler wait for every outstanding access (vmcnt(0)) at each
// branch join -- including the previous row pair's stores -- which serialised every
// iteration on a full memory round trip (2.9 TB/s standalone at 65536 x 768).
// Here the next row pair is always prefetched before the current one is reduced, the
// only waits are counted ones, and row statistics also come in through buffer loads.
template <int VPL, int NP, bool RES, int K>
__global__ __launch_bounds__(256) void ln_bwd2_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ part, int N,
    int D, float* __restrict__ o0, float* __restrict__ o1, float* __restrict__ o2) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [NP][D]
  for (int i = threadIdx.x; i < NP * D; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int bytes = N * D * 2;
  const auto rX = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, bytes, 0x00020000);
  const auto rDY = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, bytes, 0x00020000);
  const auto rR = __builtin_amdgcn_make_buffer_rsrc((void*)dres, 0, RES ? bytes : 0, 0x00020000);
  const auto rDX = __builtin_amdgcn_make_buffer_rsrc((void*)dx, 0, bytes, 0x00020000);
  const auto rM = __builtin_amdgcn_make_buffer_rsrc((void*)mean, 0, N * 4, 0x00020000);
  const auto rS = __builtin_amdgcn_make_buffer_rsrc((void*)rstd, 0, N * 4, 0x00020000);
  float gg[VPL][4], acc[NP][VPL][4];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    unpack4(*reinterpret_cast<const uint2*>(g + (i * 64 + lane) * 4), gg[i]);
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[k][i][j] = 0.f;
  }
  const float invD = 1.f / (float)D;
  const int stride = gridDim.x * 4;
  const int r_first = blockIdx.x * 4 + w;
  // rows r_first + k * stride, through a ring of K row register sets: while one row is
  // reduced, the next K - 1 are in flight
  const int iters = r_first < N ? (N - r_first + K * stride - 1) / (K * stride) : 0;
  struct Row {
    uint2 x[VPL], d[VPL], r[VPL];
    float mu, rs;
  };
  auto load = [&](Row& b, int row) __attribute__((always_inline)) {
    b.mu = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rM, row * 4, 0, 0));
    b.rs = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rS, row * 4, 0, 0));
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int off = (row * D + (i * 64 + lane) * 4) * 2;
      b.x[i] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rX, off, 0, 0));
      b.d[i] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rDY, off, 0, 0));
      if (RES)
        b.r[i] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rR, off, 0, 0));
    }
  };
  auto compute = [&](const Row& b, int row) __attribute__((always_inline)) {
    float xh[VPL][4], dv[VPL][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float xv[4];
      unpack4(b.x[i], xv);
      unpack4(b.d[i], dv[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[i][j] = (xv[j] - b.mu) * b.rs;
        const float wd = dv[i][j] * gg[i][j];
        s1 += wd;
        s2 += wd * xh[i][j];
        acc[0][i][j] += dv[i][j] * xh[i][j];
        acc[1][i][j] += dv[i][j];
      }
    }
    const float c1 = wave_sum_dpp(s1) * invD;
    const float c2 = wave_sum_dpp(s2) * invD;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float rv[4] = {0.f, 0.f, 0.f, 0.f}, o[4];
      if (RES) unpack4(b.r[i], rv);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = (dv[i][j] * gg[i][j] - c1 - xh[i][j] * c2) * b.rs + rv[j];
        if (NP == 3) acc[NP - 1][i][j] += o[j];
      }
      const int off = (row * D + (i * 64 + lane) * 4) * 2;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, pack4(o)), rDX, off, 0,
                                            0);
    }
  };
  Row ring[K];
  int r = r_first;
  if (iters > 0) {
#pragma unroll
    for (int k = 0; k < K - 1; ++k) load(ring[k], r + k * stride);
  }
  // sched_barrier: keep each set's loads where they are written (the machine scheduler
  // otherwise hoists every set's loads to the loop top, behind a full vmcnt(0) wait)
  for (int it = 0; it < iters; ++it, r += K * stride) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      load(ring[(k + K - 1) % K], r + (k + K - 1) * stride);  // past N: zeros, no stores
      __builtin_amdgcn_sched_barrier(0);
      compute(ring[k], r + k * stride);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int col = (i * 64 + lane) * 4;
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(&lds[k * D + col + j], acc[k][i][j]);
  }
  __syncthreads();
  if (o0) {
    // fp32 sinks accumulated in place (the flat gradient): the block's column sums go
    // straight in with lane-linear float atomics (P adds per address, 256 contiguous bytes
    // per wave instruction), instead of a partial slab and one colsum launch per sink
    for (int i = threadIdx.x; i < NP * D; i += blockDim.x) {
      const int k = i / D, c = i - k * D;
      unsafeAtomicAdd((k == 0 ? o0 : k == 1 ? o1 : o2) + c, lds[i]);
    }
    return;
  }
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

// Partial-row count for the v1 backward: up to 512 blocks, each wave >= 2 rows.
// Measured at 65536 x 768 (profiles/r2_perf_bench.log, "norm"): 512 blocks beat 1024 /
// 2048 / 4096 — more blocks only add partial-slab traffic and LDS-atomic tails.
RA_EXPORT int ra_layernorm_bwd_parts(int N) {
  int p = (N + 7) / 8;
  return p < 512 ? p : 512;
}

// v2 applies to D in {256, 512, 768, 1024} with N*D*2 < 2^31.
static bool ln_bwd_v2(int N, int D) {
  return D % 256 == 0 && D <= 1024 && (long)N * D * 2 < (1L << 31);
}

// v2 grid: 512 blocks, each wave >= 2 rows. Measured at 65536 x 768
// (scripts/ln_bwd_bench.py, kernel only): 256 / 512 blocks 84 / 87 us (4.8 / 4.7 TB/s),
// 768-1024 blocks 92-95 us, v1 105 us; a 3-deep row ring is no faster.
static int ln_bwd_blocks(int N, int D) {
  if (!ln_bwd_v2(N, D)) return ra_layernorm_bwd_parts(N);
  int p = (N + 7) / 8;
  return p < 512 ? p : 512;
}

// fp32 workspace (in floats) required by ra_layernorm_bwd (3 partial slabs + scratch).
RA_EXPORT long ra_layernorm_bwd_work(int N, int D) {
  const int P = ln_bwd_blocks(N, D);
  return 3L * P * D + 3L * kColsumSplits * D;
}

// dbias (optional): column sums of dx (bias grad of the residual add that produced x).
// flags: bit0 bf16 dg/db/dbias, bit1 accumulate them into (flat) gradient buffers.
RA_EXPORT int ra_layernorm_bwd(const void* dy, const void* x, const void* g, const float* mean,
                               const float* rstd, const void* dres, void* dx, void* dg, void* db,
                               void* dbias, float* work, int N, int D, int flags,
                               hipStream_t st) {
  if (D % 4 != 0) return hipErrorInvalidValue;
  const int P = ln_bwd_blocks(N, D);
  const int NP = dbias ? 3 : 2;
  float* scr = work + (size_t)NP * P * D;
  const size_t lds = (size_t)NP * D * sizeof(float);
  if (ln_bwd_v2(N, D)) {
    // fp32 sinks accumulated in place: column sums by atomics inside the kernel
    const bool direct = !(flags & kColsumBF16) && (flags & kColsumAcc);
    float* o0 = direct ? (float*)dg : nullptr;
    float* o1 = direct ? (float*)db : nullptr;
    float* o2 = direct ? (float*)dbias : nullptr;
#define L2K(V, NPV, R, KK)                                                                     \
  hipLaunchKernelGGL((ln_bwd2_kernel<V, NPV, R, KK>), dim3(P), dim3(256), lds, st,              \
                     (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)g, mean, rstd,         \
                     (const bf16_t*)dres, (bf16_t*)dx, work, N, D, o0, o1, o2)
#define L2(V, NPV, R) L2K(V, NPV, R, 2)
#define L2V(V)                                       \
  if (NP == 3) {                                     \
    if (dres) L2(V, 3, true); else L2(V, 3, false);  \
  } else {                                           \
    if (dres) L2(V, 2, true); else L2(V, 2, false);  \
  }
    switch (D / 256) {
      case 1: L2V(1); break;
      case 2: L2V(2); break;
      case 3: L2V(3); break;
      default: L2V(4); break;
    }
#undef L2V
#undef L2
#undef L2K
    if (direct) return hipGetLastError();
    void* outs[3] = {dg, db, dbias};
    for (int k = 0; k < NP; ++k)
      colsum_launch(work + (size_t)k * P * D, scr + (size_t)k * kColsumSplits * D, outs[k], P,
                    D, flags, st);
    return hipGetLastError();
  }
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
