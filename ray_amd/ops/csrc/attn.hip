// Causal flash attention for head_dim 64 on CDNA4 MFMA (v_mfma_f32_32x32x16_bf16).
//
// Reads Q/K/V straight from the packed QKV GEMM output [B, T, 3, H, 64] and writes
// O as [B, T, H, 64] (= the proj GEMM's input) and dQKV packed like QKV, so the
// model needs no permute / contiguous / cat copies around attention.
//
// Orientation (see cdna_hip_programming.md §3 "An accumulator tile as the next
// MFMA's operand"): the forward computes S^T = K·Q^T so each lane owns ONE query
// (column) and 16 keys (registers) — row-max / row-sum / rescale are lane-local
// plus one xor-32 exchange — and P^T's accumulator registers feed O^T = V^T·P^T
// directly as the B operand (no LDS round trip for P). V is staged transposed in
// LDS so its A fragments are two 8-byte reads.
//
// Backward = two kernels (no float atomics; dQ would otherwise cost ~400 MB of
// atomic adds per step at GPT-2 shape, far above the 1.3 TB/s atomic rate):
//   attn_bwd_dkdv : one workgroup per 128 keys, each wave owns 32 keys; loops over
//                   the causal q tiles: S = Q·K^T, dP = dO·V^T (keys on lanes), then
//                   dV += P^T·dO and dK += dS^T·Q with P / dS as A operands.
//   attn_bwd_dq   : one workgroup per 128 queries (forward orientation):
//                   dQ^T += K^T·dS^T.
// Softmax statistics are kept in the log2 domain (exp2 with scale·log2e folded).
#include "common.h"

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define HD 64
#define TSTR 72  // LDS row stride (elements) for 64-wide tiles: 144 B, conflict-free b128 rows

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

// two 4-element (8-byte) LDS reads → one 8-element fragment
__device__ __forceinline__ bf16x8_t ld4x2(const bf16_t* p0, const bf16_t* p1) {
  bf16x4_t a = *reinterpret_cast<const bf16x4_t*>(p0);
  bf16x4_t b = *reinterpret_cast<const bf16x4_t*>(p1);
  return bf16x8_t{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// registers 8s..8s+7 of an accumulator → bf16 fragment (k-step s of a following MFMA)
__device__ __forceinline__ bf16x8_t acc_frag(const f32x16& x, int s) {
  bf16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[8 * s + j];
  return r;
}

// row index (within a 32x32 C tile) of accumulator register i for lane half hh
__device__ __forceinline__ int crow(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

// ----------------------------------------------------------------------------
// Stage a [64 rows][64] bf16 tile from global (row stride `gstride` elements) into
// LDS, natural layout (dst[row*TSTR + c]) and/or transposed (dstT[c*TSTR + row]).
// 256 threads, 2 x 16-byte chunks each.
struct TileRegs {
  uint4 v[2];
};

__device__ __forceinline__ void tile_load(TileRegs& r, const bf16_t* g, long gstride, int rows_valid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = threadIdx.x + 256 * u;
    const int row = c >> 3, col = (c & 7) * 8;
    if (row < rows_valid) r.v[u] = *reinterpret_cast<const uint4*>(g + row * gstride + col);
    else r.v[u] = make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void tile_store(const TileRegs& r, bf16_t* dst, bf16_t* dstT) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = threadIdx.x + 256 * u;
    const int row = c >> 3, col = (c & 7) * 8;
    if (dst) *reinterpret_cast<uint4*>(dst + row * TSTR + col) = r.v[u];
    if (dstT) {
      const bf16_t* e = reinterpret_cast<const bf16_t*>(&r.v[u]);
#pragma unroll
      for (int j = 0; j < 8; ++j) dstT[(col + j) * TSTR + row] = e[j];
    }
  }
}

// ============================================================================ forward
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                       bf16_t* __restrict__ out,
                                                       float* __restrict__ lse, int T, int H,
                                                       float sc_log2) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 64 * TSTR];
  bf16_t* Ks = lds;
  bf16_t* Vt = lds + 64 * TSTR;
  const int nqb = T / 128;
  const int qb = nqb - 1 - (int)(blockIdx.x % nqb);  // heaviest causal blocks first
  const int bh = blockIdx.x / nqb;
  const int b = bh / H, h = bh % H;
  const int C = H * HD;
  const long tok = 3L * C;
  const bf16_t* base = qkv + (long)b * T * tok + h * HD;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = qb * 128;
  const int qrow = q0 + 32 * w + r;
  bf16x8_t qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) qf[kk] = ld8(base + (long)qrow * tok + 16 * kk + 8 * hh);
  f32x16 o[2] = {};
  float m_run = -INFINITY, l_run = 0.f;
  const int ntiles = (q0 + 128) / 64;
  TileRegs kr, vr;
  tile_load(kr, base + C, tok, 64);
  tile_load(vr, base + 2 * C, tok, 64);
  const int wave_qmax = q0 + 32 * w + 31;
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    tile_store(kr, Ks, nullptr);
    tile_store(vr, nullptr, Vt);
    __syncthreads();
    if (t + 1 < ntiles) {
      const long off = (long)(t + 1) * 64 * tok;
      tile_load(kr, base + C + off, tok, 64);
      tile_load(vr, base + 2 * C + off, tok, 64);
    }
    const int kv0 = t * 64;
    if (kv0 > wave_qmax) continue;  // fully masked for this wave (still joined the barriers)
    f32x16 st[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      st[kt] = f32x16{};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        st[kt] = mfma32(ld8(Ks + (32 * kt + r) * TSTR + 16 * kk + 8 * hh), qf[kk], st[kt]);
    }
    const bool diag = kv0 + 63 > q0 + 32 * w;
    float mt = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float s = st[kt][i] * sc_log2;
        if (diag && kv0 + 32 * kt + crow(i, hh) > qrow) s = -INFINITY;
        st[kt][i] = s;
        mt = fmaxf(mt, s);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = exp2f(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = exp2f(st[kt][i] - m_new);
        st[kt][i] = p;
        ls += p;
      }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t pf = acc_frag(st[kt], s);
        const int key = 32 * kt + 16 * s + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16_t* vrow = Vt + (32 * dt + r) * TSTR + key;
          o[dt] = mfma32(ld4x2(vrow, vrow + 8), pf, o[dt]);
        }
      }
  }
  const float inv = 1.f / l_run;
  bf16_t* orow = out + ((long)b * T + qrow) * C + h * HD;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v[4] = {o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv,
                    o[dt][4 * g + 3] * inv};
      *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * g + 4 * hh) = pack4(v);
    }
  if (hh == 0) lse[(long)bh * T + qrow] = m_run + log2f(l_run);
}

// ============================================================================ backward
// delta[bh][t] = sum_d dO[b,t,h,d] * O[b,t,h,d]   (one wave per (b, t), 4 heads' rows per block)
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           float* __restrict__ delta, int BT,
                                                           int T, int H) {
  // each thread handles one (token, head) row of 64 elements with 8 x 16B loads
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)BT * H) return;
  const long tokn = idx / H;
  const int h = (int)(idx % H);
  const bf16_t* po = o + idx * HD;
  const bf16_t* pd = dout + idx * HD;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float a[8], d[8];
    unpack8(*reinterpret_cast<const uint4*>(po + 8 * c), a);
    unpack8(*reinterpret_cast<const uint4*>(pd + 8 * c), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] * d[j];
  }
  const long b = tokn / T, t = tokn % T;
  delta[(b * H + h) * T + t] = s;
}

// dK, dV: workgroup = 128 keys of one (b, h); wave owns 32 keys.
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    int T, int H, float sc_log2, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[4 * 64 * TSTR];
  __shared__ float s_lse[64], s_del[64];
  bf16_t* Qs = lds;                 // [q][d]
  bf16_t* Qt = lds + 64 * TSTR;     // [d][q]
  bf16_t* Ds = lds + 128 * TSTR;    // dO [q][d]
  bf16_t* Dt = lds + 192 * TSTR;    // dO^T [d][q]
  const int nkb = T / 128;
  const int kb = (int)(blockIdx.x % nkb);
  const int bh = blockIdx.x / nkb;
  const int b = bh / H, h = bh % H;
  const int C = H * HD;
  const long tok = 3L * C;
  const bf16_t* base = qkv + (long)b * T * tok + h * HD;
  const bf16_t* dobase = dout + (long)b * T * C + h * HD;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int kv0 = kb * 128;
  const int key = kv0 + 32 * w + r;  // this lane's key (C-tile column)
  bf16x8_t kf[4], vf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    kf[kk] = ld8(base + C + (long)key * tok + 16 * kk + 8 * hh);
    vf[kk] = ld8(base + 2 * C + (long)key * tok + 16 * kk + 8 * hh);
  }
  f32x16 dv[2] = {}, dk[2] = {};
  const int t0 = kv0 / 64;
  const int ntiles = T / 64;
  const int wave_kmin = kv0 + 32 * w;
  TileRegs qr, dr;
  tile_load(qr, base + (long)t0 * 64 * tok, tok, 64);
  tile_load(dr, dobase + (long)t0 * 64 * C, C, 64);
  for (int t = t0; t < ntiles; ++t) {
    const int q0 = t * 64;
    __syncthreads();
    tile_store(qr, Qs, Qt);
    tile_store(dr, Ds, Dt);
    if (threadIdx.x < 64) {
      s_lse[threadIdx.x] = lse[(long)bh * T + q0 + threadIdx.x];
      s_del[threadIdx.x] = delta[(long)bh * T + q0 + threadIdx.x];
    }
    __syncthreads();
    if (t + 1 < ntiles) {
      tile_load(qr, base + (long)(t + 1) * 64 * tok, tok, 64);
      tile_load(dr, dobase + (long)(t + 1) * 64 * C, C, 64);
    }
    if (q0 + 63 < wave_kmin) continue;
    const bool diag = q0 < wave_kmin + 31;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      // S = Q K^T (rows q, cols = this wave's keys), dP = dO V^T
      f32x16 s = {}, dp = {};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        s = mfma32(ld8(Qs + (32 * qt + r) * TSTR + 16 * kk + 8 * hh), kf[kk], s);
        dp = mfma32(ld8(Ds + (32 * qt + r) * TSTR + 16 * kk + 8 * hh), vf[kk], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = 32 * qt + crow(i, hh);
        float p = exp2f(s[i] * sc_log2 - s_lse[ql]);
        if (diag && key > q0 + ql) p = 0.f;
        s[i] = p;                        // P
        dp[i] = p * (dp[i] - s_del[ql]);  // dS (wrt scaled scores)
      }
      // dV += P^T dO ; dK += dS^T Q   (P / dS registers as A operands, k = q)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t pa = acc_frag(s, ks);
        const bf16x8_t da = acc_frag(dp, ks);
        const int qk = 32 * qt + 16 * ks + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16_t* drow = Dt + (32 * dt + r) * TSTR + qk;
          const bf16_t* qrow = Qt + (32 * dt + r) * TSTR + qk;
          dv[dt] = mfma32(pa, ld4x2(drow, drow + 8), dv[dt]);
          dk[dt] = mfma32(da, ld4x2(qrow, qrow + 8), dk[dt]);
        }
      }
    }
  }
  // dV / dK tiles: rows = keys (registers), cols = d (lane)
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kr = kv0 + 32 * w + crow(i, hh);
      bf16_t* g = dqkv + ((long)b * T + kr) * tok + h * HD + 32 * dt + r;
      g[C] = f2bf(dk[dt][i] * scale);
      g[2 * C] = f2bf(dv[dt][i]);
    }
}

// dQ: workgroup = 128 queries; forward orientation (S^T, lanes = queries).
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    int T, int H, float sc_log2, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[3 * 64 * TSTR];
  bf16_t* Ks = lds;                // [key][d]
  bf16_t* Kt = lds + 64 * TSTR;    // [d][key]
  bf16_t* Vs = lds + 128 * TSTR;   // [key][d]
  const int nqb = T / 128;
  const int qb = nqb - 1 - (int)(blockIdx.x % nqb);
  const int bh = blockIdx.x / nqb;
  const int b = bh / H, h = bh % H;
  const int C = H * HD;
  const long tok = 3L * C;
  const bf16_t* base = qkv + (long)b * T * tok + h * HD;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int q0 = qb * 128;
  const int qrow = q0 + 32 * w + r;
  bf16x8_t qf[4], df[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    qf[kk] = ld8(base + (long)qrow * tok + 16 * kk + 8 * hh);
    df[kk] = ld8(dout + ((long)b * T + qrow) * C + h * HD + 16 * kk + 8 * hh);
  }
  const float lq = lse[(long)bh * T + qrow];
  const float dq_del = delta[(long)bh * T + qrow];
  f32x16 dq[2] = {};
  const int ntiles = (q0 + 128) / 64;
  const int wave_qmax = q0 + 32 * w + 31;
  TileRegs kr, vr;
  tile_load(kr, base + C, tok, 64);
  tile_load(vr, base + 2 * C, tok, 64);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();
    tile_store(kr, Ks, Kt);
    tile_store(vr, Vs, nullptr);
    __syncthreads();
    if (t + 1 < ntiles) {
      const long off = (long)(t + 1) * 64 * tok;
      tile_load(kr, base + C + off, tok, 64);
      tile_load(vr, base + 2 * C + off, tok, 64);
    }
    const int kv0 = t * 64;
    if (kv0 > wave_qmax) continue;
    const bool diag = kv0 + 63 > q0 + 32 * w;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      f32x16 st = {}, dpt = {};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        st = mfma32(ld8(Ks + (32 * kt + r) * TSTR + 16 * kk + 8 * hh), qf[kk], st);
        dpt = mfma32(ld8(Vs + (32 * kt + r) * TSTR + 16 * kk + 8 * hh), df[kk], dpt);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = exp2f(st[i] * sc_log2 - lq);
        if (diag && kv0 + 32 * kt + crow(i, hh) > qrow) p = 0.f;
        dpt[i] = p * (dpt[i] - dq_del);  // dS^T
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t bfrag = acc_frag(dpt, s);
        const int kk2 = 32 * kt + 16 * s + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16_t* krow = Kt + (32 * dt + r) * TSTR + kk2;
          dq[dt] = mfma32(ld4x2(krow, krow + 8), bfrag, dq[dt]);
        }
      }
    }
  }
  bf16_t* g = dqkv + ((long)b * T + qrow) * tok + h * HD;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      float v[4] = {dq[dt][4 * gi] * scale, dq[dt][4 * gi + 1] * scale,
                    dq[dt][4 * gi + 2] * scale, dq[dt][4 * gi + 3] * scale};
      *reinterpret_cast<uint2*>(g + 32 * dt + 8 * gi + 4 * hh) = pack4(v);
    }
}

static inline bool attn_shape_ok(int T, int D) { return D == HD && T % 128 == 0 && T >= 128; }

RA_EXPORT int ra_attn_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, int D,
                          float scale, hipStream_t st) {
  if (!attn_shape_ok(T, D)) return hipErrorInvalidValue;
  const float sc_log2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (bf16_t*)out, lse, T, H, sc_log2);
  return hipGetLastError();
}

// delta: B*H*T floats workspace
RA_EXPORT int ra_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                          float* delta, void* dqkv, int B, int T, int H, int D, float scale,
                          hipStream_t st) {
  if (!attn_shape_ok(T, D)) return hipErrorInvalidValue;
  const float sc_log2 = scale * 1.4426950408889634f;
  const long rows = (long)B * T * H;
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((rows + 255) / 256), dim3(256), 0, st,
                     (const bf16_t*)out, (const bf16_t*)dout, delta, B * T, T, H);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, T, H,
                     sc_log2, scale);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, T, H,
                     sc_log2, scale);
  return hipGetLastError();
}
