// Causal flash attention for head_dim 64 on CDNA4 MFMA (v_mfma_f32_32x32x16_bf16).
//
// Reads Q/K/V straight from the packed QKV GEMM output [B, T, 3, H, 64] and writes
// O as [B, T, H, 64] (= the proj GEMM's input) and dQKV packed like QKV, so the
// model needs no permute / contiguous / cat copies around attention.
//
// Orientation (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's
// operand"): the forward computes S^T = K·Q^T so each lane owns ONE query (column)
// and 16 keys (registers) — row-max / row-sum / rescale are lane-local plus one
// permlane32 swap — and P^T's accumulator registers feed O^T = V^T·P^T directly as
// the B operand (no LDS round trip for P).
//
// LDS images: every K/V/Q/dO tile is staged ONCE, row-major ([row][64] bf16, 128-B
// rows, no padding) with 16-byte writes, under an XOR swizzle of the 16-B chunk
// index (`swz`). The same image serves row reads (ds_read_b128, MFMA operand with k
// along the row) and column reads (ds_read_b64_tr_b16 hardware transpose, operand
// with k down the column) — both conflict-free:
//   * b128 row reads: a 16-lane group reads 16 rows at one chunk; rows alternate
//     between the two 64-B bank halves (row&1) and swz(row) takes all 8 values over
//     each group's 8 same-parity rows.
//   * tr reads: a 32-lane half reads rows R..R+3 (R%4==0) × 32 columns; swz(R) and
//     swz(R+2) differ in bit 2, so rows R and R+2 use complementary chunk sets.
// Tiles are double buffered: one barrier per tile; the next tile's global loads are
// in flight during the current tile's MFMAs.
//
// Backward = two kernels, no float atomics (a fused one-pass form with fp32 dQ atomics
// measured 730 us against 384 + 337 us at B64 T1024 H12, profiles/r2/
// attn_bwd_fused_vs_split.md: 0.9 GB of fp32 dQ partials per call cost more than recomputing
// S and dP at head_dim 64):
//   attn_bwd_dkdv : one workgroup per 128 keys, each wave owns 32 keys; loops over
//                   the causal q tiles: S = Q·K^T, dP = dO·V^T (keys on lanes), then
//                   dV += P^T·dO and dK += dS^T·Q with P / dS as A operands. The
//                   accumulators of S and dP start at -LSE/c and -delta (row constants
//                   as the initial accumulator), so P = exp2(c·S'), dS = P·dP'.
//   attn_bwd_dq   : one workgroup per 128 queries (forward orientation):
//                   dQ^T += K^T·dS^T.
// Softmax statistics are kept in the log2 domain (exp2 with scale·log2e folded).
#include "common.h"

#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define HD 64
#define TILE_ELEMS (64 * 64)

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t ld8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

__device__ __forceinline__ bf16x4_t tr4(const bf16_t* p) {
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)const_cast<bf16_t*>(p));
  return __builtin_bit_cast(bf16x4_t, v);
}

__device__ __forceinline__ bf16x8_t cat44(bf16x4_t a, bf16x4_t b) {
  return bf16x8_t{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// registers 8s..8s+7 of an accumulator → bf16 fragment (k-step s of a following MFMA)
__device__ __forceinline__ bf16x8_t acc_frag(const f32x16& x, int s) {
  bf16x8_t r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[8 * s + j];
  return r;
}

// value of x in the other 32-lane half (lane ^ 32)
__device__ __forceinline__ float half_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// row index (within a 32x32 C tile) of accumulator register i for lane half hh
__device__ __forceinline__ int crow(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

// ---------------------------------------------------------------- swizzled LDS image
__device__ __forceinline__ int swz(int row) {
  const int u = (row >> 1) & 7;
  return ((u & 1) << 2) | (u & 2) | (u >> 2);  // bit0 <-> bit2 of (row>>1)&7
}
// element offset of 16-B chunk `ch` (0..7) of row `row`
__device__ __forceinline__ int img_off(int row, int ch) { return row * 64 + ((ch ^ swz(row)) << 3); }

// Lane-constant offsets. Row read of a 32-row operand block starting at row 32x:
// lane (r, hh) reads row 32x + r, chunk 2kk + hh → offset 2048x + rowoff[kk].
// Transposed read (k rows kb + 4hh + 8e + q, columns 32dt + 16(g&1) + 4p) for a
// k-block starting at kb (multiple of 16): offset 64*kb + troff[e][dt].
struct LaneOffs {
  int row[4];
  int tr[2][2];
  __device__ __forceinline__ LaneOffs(int lane) {
    const int r = lane & 31, hh = lane >> 5, g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) row[kk] = img_off(r, 2 * kk + hh);
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int col = 32 * dt + 16 * (g & 1) + 4 * p;
        tr[e][dt] = img_off(4 * hh + 8 * e + q, col >> 3) + (col & 7);
      }
  }
};

// operand fragment with k down the image's rows: k = kb + {4hh+0..3, 8+4hh+0..3}
// (the acc_frag k order), column 32dt + (lane&31)
__device__ __forceinline__ bf16x8_t tr_frag(const bf16_t* img, const LaneOffs& lo, int kb, int dt) {
  return cat44(tr4(img + 64 * kb + lo.tr[0][dt]), tr4(img + 64 * kb + lo.tr[1][dt]));
}

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2): map
// physical block id → logical id so that consecutive logical blocks (the q- or key-blocks
// of one (b, h), which all stream the same K/V or Q/dO) share an XCD and its L2.
__device__ __forceinline__ int xcd_block(int bid, int n) {
  return (n & 7) ? bid : (bid & 7) * (n >> 3) + (bid >> 3);
}

// ---------------------------------------------------------------- tile staging
// [64 rows][64] bf16 tile, global row stride `gstride` elements; 256 threads x 2 chunks
// native vector type: HIP's uint4 is a struct, whose copies lower to memcpy through a
// stack slot (scratch) that SROA cannot promote
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct TileRegs {
  u32x4 v0, v1;
};
struct KV {
  TileRegs k, v;
};
struct QD {
  TileRegs q, d;
  float rc;  // -lse/c (threads 0..63) or -delta (64..127) of the tile's rows
};

__device__ __forceinline__ void tile_load(TileRegs& r, const bf16_t* g, long gstride) {
  const int c = threadIdx.x;
  r.v0 = *reinterpret_cast<const u32x4*>(g + (c >> 3) * gstride + (c & 7) * 8);
  r.v1 = *reinterpret_cast<const u32x4*>(g + ((c + 256) >> 3) * gstride + (c & 7) * 8);
}

// The same [64 rows][64] tile through a buffer resource: the per-thread offsets are fixed
// (voff0/voff1, bytes) and the tile's position is a scalar byte offset, so a tile costs no
// 64-bit VALU address arithmetic (2 loads instead of ~8 VALU + 2 loads)
struct TileAddr {
  int voff0, voff1;
  __device__ __forceinline__ TileAddr(long gstride) {
    const int c = threadIdx.x;
    voff0 = (int)(((c >> 3) * gstride + (c & 7) * 8) * 2);
    voff1 = (int)((((c + 256) >> 3) * gstride + (c & 7) * 8) * 2);
  }
};
__device__ __forceinline__ void tile_load_buf(TileRegs& r, __amdgpu_buffer_rsrc_t rs,
                                              const TileAddr& a, int soff) {
  r.v0 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, a.voff0, soff, 0));
  r.v1 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, a.voff1, soff, 0));
}

__device__ __forceinline__ void tile_store(const TileRegs& r, bf16_t* img) {
  const int c = threadIdx.x;
  *reinterpret_cast<u32x4*>(img + img_off(c >> 3, c & 7)) = r.v0;
  *reinterpret_cast<u32x4*>(img + img_off((c + 256) >> 3, c & 7)) = r.v1;
}

// ============================================================================ forward
// One workgroup covers 128 queries: each wave owns 32 (QB = 1 block of 32), two waves per SIMD.
// (Measured and removed: two 32-query blocks per wave at one wave per SIMD, and a 3-waves-
// per-SIMD register budget — profiles/r5/r5ao, r5at.)
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                       bf16_t* __restrict__ out,
                                                       float* __restrict__ lse, int T, int H,
                                                       float sc_log2) {
  constexpr int QB = 1;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * TILE_ELEMS];  // [buf][K,V]
  constexpr int QW = 32 * QB;    // queries per wave
  constexpr int QBLK = 4 * QW;   // queries per workgroup
  const int nqb = T / QBLK;
  const int L = xcd_block(blockIdx.x, gridDim.x);
  const int qb = nqb - 1 - L % nqb;  // heaviest causal blocks first
  const int bh = L / nqb;
  const int b = bh / H, h = bh % H;
  const int C = H * HD;
  const long tok = 3L * C;
  const bf16_t* base = qkv + (long)b * T * tok + h * HD;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const LaneOffs lo(lane);
  const int q0 = qb * QBLK;
  const int wave_qmin = q0 + QW * w;
  const int wave_qmax = wave_qmin + QW - 1;
  int qrow[QB];
  bf16x8_t qf[QB][4];
  f32x16 o[QB][2];
  float m_run[QB], l_run[QB];
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    qrow[j] = wave_qmin + 32 * j + r;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) qf[j][kk] = ld8(base + (long)qrow[j] * tok + 16 * kk + 8 * hh);
    o[j][0] = f32x16{};
    o[j][1] = f32x16{};
    m_run[j] = -INFINITY;
    l_run[j] = 0.f;
  }
  const int ntiles = (q0 + QBLK) / 64;
  KV A, B;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (T - 1) * (int)tok * 2 + 3 * C * 2,
                                        0x00020000);
  const TileAddr ta(tok);
  auto load_kv = [&](KV& x, int t) __attribute__((always_inline)) {
    const int off = t * 64 * (int)tok * 2;
    tile_load_buf(x.k, rs, ta, off + C * 2);
    tile_load_buf(x.v, rs, ta, off + 2 * C * 2);
  };
  auto store_kv = [&](const KV& x, int t) __attribute__((always_inline)) {
    bf16_t* d = lds + (t & 1) * 2 * TILE_ELEMS;
    tile_store(x.k, d);
    tile_store(x.v, d + TILE_ELEMS);
  };
  auto body = [&](int t, auto diag_c) __attribute__((always_inline)) {
    constexpr bool diag = decltype(diag_c)::value;
    const bf16_t* Ks = lds + (t & 1) * 2 * TILE_ELEMS;
    const bf16_t* Vs = Ks + TILE_ELEMS;
    const int kv0 = t * 64;
    f32x16 st[QB][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int j = 0; j < QB; ++j) st[j][kt] = f32x16{};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8_t kfrag = ld8(Ks + 2048 * kt + lo.row[kk]);
#pragma unroll
        for (int j = 0; j < QB; ++j) st[j][kt] = mfma32(kfrag, qf[j][kk], st[j][kt]);
      }
    }
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      if (diag) {  // diagonal tile: mask keys > query
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (kv0 + 32 * kt + crow(i, hh) > qrow[j]) st[j][kt][i] = -INFINITY;
      }
      float mt = st[j][0][0];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) mt = fmaxf(mt, st[j][kt][i]);
      mt = half_max(mt) * sc_log2;
      // Lazy rescaling: the running max moves (and O / l are rescaled) only when some
      // query's tile max exceeds it by more than 8 (log2 units). Otherwise the stale max
      // stays, p <= 2^8 — exact in fp32, and the final O / l is unchanged: the common tile
      // skips the 32 multiplies of the O rescale and the exp of alpha. A wave-uniform
      // branch (the first tile always takes it: m_run = -inf). A tile entirely above the
      // diagonal for this block (QB 2, first block) has mt = -inf and changes nothing.
      if (__builtin_amdgcn_ballot_w64(mt > m_run[j] + 8.f)) {
        const float m_new = fmaxf(m_run[j], mt);
        const float alpha = fast_exp2(m_run[j] - m_new);
        l_run[j] *= alpha;
        m_run[j] = m_new;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[j][dt][i] *= alpha;
      }
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fast_exp2(fmaf(st[j][kt][i], sc_log2, -m_run[j]));
          st[j][kt][i] = p;
          ls += p;
        }
      l_run[j] += half_sum(ls);
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16x8_t vfrag = tr_frag(Vs, lo, 32 * kt + 16 * s, dt);
#pragma unroll
          for (int j = 0; j < QB; ++j) o[j][dt] = mfma32(vfrag, acc_frag(st[j][kt], s), o[j][dt]);
        }
      }
  };
  auto compute = [&](int t) __attribute__((always_inline)) {
    const int kv0 = t * 64;
    if (kv0 <= wave_qmax) {
      if (kv0 + 63 > wave_qmin) body(t, std::true_type{});
      else body(t, std::false_type{});
    }
  };
  // 2-deep register prefetch: tile t+2's loads are in flight during tiles t and t+1
  auto step = [&](int t, KV& held, KV& next) __attribute__((always_inline)) {
    if (t + 2 < ntiles) load_kv(next, t + 2);
    compute(t);
    if (t + 1 < ntiles) store_kv(held, t + 1);
    __syncthreads();
  };
  load_kv(A, 0);
  store_kv(A, 0);
  load_kv(A, 1);  // ntiles >= 2
  __syncthreads();
  for (int t = 0; t < ntiles; t += 2) {
    step(t, A, B);
    if (t + 1 < ntiles) step(t + 1, B, A);
  }
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const float inv = 1.f / l_run[j];
    bf16_t* orow = out + ((long)b * T + qrow[j]) * C + h * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v[4] = {o[j][dt][4 * g] * inv, o[j][dt][4 * g + 1] * inv,
                      o[j][dt][4 * g + 2] * inv, o[j][dt][4 * g + 3] * inv};
        *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * g + 4 * hh) = pack4(v);
      }
    if (hh == 0) lse[(long)bh * T + qrow[j]] = m_run[j] + log2f(l_run[j]);
  }
}

// ============================================================================ backward
// dK, dV: workgroup = 128 keys of one (b, h); wave owns 32 keys; loops over the causal
// 64-query tiles with one Q/dO register set (tile t+1 loaded at the top of tile t and written
// to LDS after its compute). Both 32-query halves of a tile are in flight at once: the S / dP
// chains of both halves issue first, then each half's softmax VALU runs while the other
// half's MFMAs execute. (Measured and removed: a two-register-set prefetch, a fused pass that
// also produced dQ through fp32 atomics, row constants read from global memory instead of
// LDS — profiles/r2/attn_bwd_fused_vs_split.md, profiles/r5/r5aj, r5au.)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    int T, int H, float sc_log2, float scale) {
  // [buf][Q, dO] images, then per buf 64 x (-lse/c) and 64 x (-delta)
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * TILE_ELEMS + 2 * 2 * 64 * 2];
  float* rowc = reinterpret_cast<float*>(lds + 4 * TILE_ELEMS);  // [buf][2][64]
  const int nkb = T / 128;
  const int L = xcd_block(blockIdx.x, gridDim.x);
  const int kb = L % nkb;  // kb 0 = most q tiles: heaviest first
  const int bh = L / nkb;
  const int b = bh / H, h = bh % H;
  const int C = H * HD;
  const long tok = 3L * C;
  const bf16_t* base = qkv + (long)b * T * tok + h * HD;
  const bf16_t* dobase = dout + (long)b * T * C + h * HD;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const LaneOffs lo(lane);
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
  const float inv_c = -1.f / sc_log2;
  const float* lse_bh = lse + (long)bh * T;
  const float* del_bh = delta + (long)bh * T;
  QD A;
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
      (void*)base, 0, (T - 1) * (int)tok * 2 + 3 * C * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dobase, 0, T * C * 2, 0x00020000);
  const TileAddr taq(tok), tad(C);
  const __amdgpu_buffer_rsrc_t rl =
      __builtin_amdgcn_make_buffer_rsrc((void*)lse_bh, 0, T * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rdl =
      __builtin_amdgcn_make_buffer_rsrc((void*)del_bh, 0, T * 4, 0x00020000);
  auto load_qd = [&](QD& x, int t) __attribute__((always_inline)) {
    tile_load_buf(x.q, rq, taq, t * 64 * (int)tok * 2);
    tile_load_buf(x.d, rd, tad, t * 64 * C * 2);
    if (threadIdx.x < 128) {  // waves 0 / 1: -lse/c / -delta of the tile's 64 rows
      // (the b32 builtin returns the raw 32 bits as an integer)
      const float v = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(threadIdx.x < 64 ? rl : rdl,
                                                      (t * 64 + (threadIdx.x & 63)) * 4, 0, 0));
      x.rc = threadIdx.x < 64 ? v * inv_c : -v;
    }
  };
  auto store_qd = [&](const QD& x, int t) __attribute__((always_inline)) {
    const int buf = (t - t0) & 1;
    bf16_t* d = lds + buf * 2 * TILE_ELEMS;
    tile_store(x.q, d);
    tile_store(x.d, d + TILE_ELEMS);
    if (threadIdx.x < 128) rowc[buf * 128 + threadIdx.x] = x.rc;
  };
  // DIAG is a template-like constant: the causal mask costs 3 VALU per score element
  // (compare, select, index add), so only the diagonal tiles instantiate it — the
  // compiler does not split a runtime-predicated mask out of the unrolled loop itself.
  auto body = [&](int t, auto diag_c) __attribute__((always_inline)) {
    constexpr bool diag = decltype(diag_c)::value;
    const int cur = (t - t0) & 1;
    const int q0 = t * 64;
    const bf16_t* Qs = lds + cur * 2 * TILE_ELEMS;
    const bf16_t* Ds = Qs + TILE_ELEMS;
    const float* nl = rowc + cur * 128;
    const float* nd = nl + 64;
    // S' = Q K^T - LSE/c ; dP' = dO V^T - delta   (rows q, cols = this wave's keys): the
    // row constants are the accumulators' initial values
    f32x16 s[2], dp[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 a = *reinterpret_cast<const float4*>(nl + 32 * qt + 8 * g + 4 * hh);
        const float4 d = *reinterpret_cast<const float4*>(nd + 32 * qt + 8 * g + 4 * hh);
        s[qt][4 * g] = a.x; s[qt][4 * g + 1] = a.y; s[qt][4 * g + 2] = a.z;
        s[qt][4 * g + 3] = a.w;
        dp[qt][4 * g] = d.x; dp[qt][4 * g + 1] = d.y; dp[qt][4 * g + 2] = d.z;
        dp[qt][4 * g + 3] = d.w;
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        s[qt] = mfma32(ld8(Qs + 2048 * qt + lo.row[kk]), kf[kk], s[qt]);
        dp[qt] = mfma32(ld8(Ds + 2048 * qt + lo.row[kk]), vf[kk], dp[qt]);
      }
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = fast_exp2(s[qt][i] * sc_log2);
        if (diag && key > q0 + 32 * qt + crow(i, hh)) p = 0.f;
        s[qt][i] = p;                    // P
        dp[qt][i] = p * dp[qt][i];       // dS (wrt scaled scores)
      }
      // dV += P^T dO ; dK += dS^T Q   (P / dS registers as A operands, k = q)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t pa = acc_frag(s[qt], ks);
        const bf16x8_t da = acc_frag(dp[qt], ks);
        const int kbq = 32 * qt + 16 * ks;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = mfma32(pa, tr_frag(Ds, lo, kbq, dt), dv[dt]);
          dk[dt] = mfma32(da, tr_frag(Qs, lo, kbq, dt), dk[dt]);
        }
      }
    }
  };
  auto compute = [&](int t) __attribute__((always_inline)) {
    const int q0 = t * 64;
    if (q0 + 63 >= wave_kmin) {
      if (q0 < wave_kmin + 31) body(t, std::true_type{});
      else body(t, std::false_type{});
    }
  };
  load_qd(A, t0);
  store_qd(A, t0);
  __syncthreads();
  for (int t = t0; t < ntiles; ++t) {
    if (t + 1 < ntiles) load_qd(A, t + 1);  // lands during compute(t)
    compute(t);
    if (t + 1 < ntiles) store_qd(A, t + 1);  // the other buffer: last read by tile t - 1
    __syncthreads();
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

// dQ: workgroup = 128 queries; forward orientation (S^T, lanes = queries); two K/V register
// sets (tile t+2 in flight). The kernel also computes delta = rowsum(dO * O) of its own
// queries (each lane already holds half of its query's dO row; O is read the same way and
// the halves meet by one permlane32 swap) and writes it for the dK/dV kernel that runs after
// it — no separate pre-pass over O and dO (50 us per layer at B64 T1024 H12).
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    int T, int H, float sc_log2, float scale, const bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * TILE_ELEMS];  // [buf][K, V]
  const int nqb = T / 128;
  const int L = xcd_block(blockIdx.x, gridDim.x);
  const int qb = nqb - 1 - L % nqb;
  const int bh = L / nqb;
  const int b = bh / H, h = bh % H;
  const int C = H * HD;
  const long tok = 3L * C;
  const bf16_t* base = qkv + (long)b * T * tok + h * HD;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const LaneOffs lo(lane);
  const int q0 = qb * 128;
  const int qrow = q0 + 32 * w + r;
  bf16x8_t qf[4], df[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    qf[kk] = ld8(base + (long)qrow * tok + 16 * kk + 8 * hh);
    df[kk] = ld8(dout + ((long)b * T + qrow) * C + h * HD + 16 * kk + 8 * hh);
  }
  const float nlq = -lse[(long)bh * T + qrow] / sc_log2;
  float part = 0.f;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const bf16x8_t of = ld8(out + ((long)b * T + qrow) * C + h * HD + 16 * kk + 8 * hh);
#pragma unroll
    for (int j = 0; j < 8; ++j) part += (float)of[j] * (float)df[kk][j];
  }
  const float dl = half_sum(part);
  if (hh == 0) delta[(long)bh * T + qrow] = dl;
  const float ndel = -dl;
  f32x16 dq[2] = {};
  const int ntiles = (q0 + 128) / 64;
  const int wave_qmax = q0 + 32 * w + 31;
  KV A, B;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)base, 0, (T - 1) * (int)tok * 2 + 3 * C * 2, 0x00020000);
  const TileAddr ta(tok);
  auto load_kv = [&](KV& x, int t) __attribute__((always_inline)) {
    const int off = t * 64 * (int)tok * 2;
    tile_load_buf(x.k, rs, ta, off + C * 2);
    tile_load_buf(x.v, rs, ta, off + 2 * C * 2);
  };
  auto store_kv = [&](const KV& x, int t) __attribute__((always_inline)) {
    bf16_t* d = lds + (t & 1) * 2 * TILE_ELEMS;
    tile_store(x.k, d);
    tile_store(x.v, d + TILE_ELEMS);
  };
  auto body = [&](int t, auto diag_c) __attribute__((always_inline)) {
    constexpr bool diag = decltype(diag_c)::value;
    const int kv0 = t * 64;
    const bf16_t* Ks = lds + (t & 1) * 2 * TILE_ELEMS;
    const bf16_t* Vs = Ks + TILE_ELEMS;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      f32x16 st, dpt;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[i] = nlq;
        dpt[i] = ndel;
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        st = mfma32(ld8(Ks + 2048 * kt + lo.row[kk]), qf[kk], st);
        dpt = mfma32(ld8(Vs + 2048 * kt + lo.row[kk]), df[kk], dpt);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = fast_exp2(st[i] * sc_log2);
        if (diag && kv0 + 32 * kt + crow(i, hh) > qrow) p = 0.f;
        dpt[i] = p * dpt[i];  // dS^T
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8_t bfrag = acc_frag(dpt, s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          dq[dt] = mfma32(tr_frag(Ks, lo, 32 * kt + 16 * s, dt), bfrag, dq[dt]);
      }
    }
  };
  auto compute = [&](int t) __attribute__((always_inline)) {
    const int kv0 = t * 64;
    if (kv0 <= wave_qmax) {
      if (kv0 + 63 > q0 + 32 * w) body(t, std::true_type{});
      else body(t, std::false_type{});
    }
  };
  auto step = [&](int t, KV& held, KV& next) __attribute__((always_inline)) {
    if (t + 2 < ntiles) load_kv(next, t + 2);
    compute(t);
    if (t + 1 < ntiles) store_kv(held, t + 1);
    __syncthreads();
  };
  load_kv(A, 0);
  store_kv(A, 0);
  load_kv(A, 1);  // ntiles >= 2
  __syncthreads();
  for (int t = 0; t < ntiles; t += 2) {
    step(t, A, B);
    if (t + 1 < ntiles) step(t + 1, B, A);
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

// Backward: dQ first (it computes delta on the way), then dK/dV. delta: B*H*T floats.
RA_EXPORT int ra_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                          float* delta, void* dqkv, int B, int T, int H, int D, float scale,
                          hipStream_t st) {
  if (!attn_shape_ok(T, D)) return hipErrorInvalidValue;
  const float sc_log2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, T, H,
                     sc_log2, scale, (const bf16_t*)out);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, T, H,
                     sc_log2, scale);
  return hipGetLastError();
}
