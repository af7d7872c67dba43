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
// Backward, split form (ra_attn_bwd, default: no float atomics) = two kernels below; fused
// form (ra_attn_bwd_fused) = attn_bwd_dkdv_kernel<true>: dQ from the same pass through
// LDS-staged dS and fp32 atomics. Measured at B64 T1024 H12 (rocprofv3): split 384 + 337 us,
// fused 730 us (436 without the dQ product, 606 with plain stores instead of atomics): the
// 16 KB of fp32 dQ per workgroup x q-tile (0.9 GB per call) costs more than recomputing S
// and dP at head_dim 64, so the fused form stays opt-in (RAY_AMD_ATTN_BWD=fused):
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
// QB = 32-query blocks per wave (1: a workgroup covers 128 queries; 2: 256 queries, every K
// row fragment and V transposed fragment read from LDS feeds two MFMAs, and each wave has
// two independent S / softmax / PV chains in flight; ra_knobs[9] = 1 selects QB 2).
// WPE > 0: the register budget of WPE waves per SIMD (QB 1 at WPE 3: 162 registers, no spill,
// vs 208 = 2 waves unconstrained; ra_knobs[9] = 2 selects it).
template <int QB, int WPE = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1, WPE > 0 ? WPE : 8))) void attn_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                       bf16_t* __restrict__ out,
                                                       float* __restrict__ lse, int T, int H,
                                                       float sc_log2) {
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
// delta[bh][t] = sum_d dO[b,t,h,d] * O[b,t,h,d]   (one thread per (token, head) row)
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           float* __restrict__ delta, int BT,
                                                           int T, int H) {
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
// FUSED: the same pass also produces dQ. Each tile's dS (bf16) is staged once in LDS as a
// [128 keys][64 q] image beside a [128 keys][64 d] image of the workgroup's K, and after a
// barrier wave w computes the 32 x 32 block (q half w>>1, d half w&1) of dQ_tile = dS K
// over all 128 keys (8 MFMAs) and adds it to an fp32 dQ workspace with no-return float
// atomics (two 128-B row segments per instruction: the full-rate shape). This replaces the
// separate dq kernel, which recomputed S and dP (2 of its 3 MFMA products) from scratch.
// PF: Q/dO register prefetch depth (2: two register sets, tile t+2 in flight; 1: one set,
// tile t+1 loaded at the top of tile t and written to LDS after its compute — 17 fewer
// VGPRs for the compiler's LDS-fragment prefetch). ra_knobs[11] = 1 selects PF 1.
// ILP (non-FUSED, with PF 1): both 32-query halves of a tile are in flight at once — the
// S / dP chains of both halves issue first, then each half's softmax VALU runs while the
// other half's MFMAs execute (the 17 VGPRs PF 1 frees hold the second half's S / dP).
// RCG (PF 1, not FUSED, ra_knobs[11] = 3; with ILP it spills): the row constants come straight from global
// memory into registers (16 broadcast buffer loads per tile, issued at the top of the tile and
// consumed after the S / dP chains, which start from zero accumulators: p = exp2(c S - lse),
// dS = p (dP - delta)) instead of through LDS. The kernel then needs exactly 32 KB of LDS,
// which fits beside a 128 KB weight-gradient workgroup of the side stream on one CU (160 KB);
// with the 1 KB LDS row-constant buffer it did not (profiles/r5/README.md).
template <bool FUSED, int PF = 2, bool ILP = false, bool RCG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ dqkv,
    float* __restrict__ dq_ws, int T, int H, float sc_log2, float scale, int dbg) {
  static_assert(!RCG || (PF == 1 && !FUSED), "RCG: PF 1 split form only");
  // [buf][Q, dO] images, then per buf 64 x (-lse/c) and 64 x (-delta); FUSED: + K image
  // [128][64] and dS^T image [128][64]
  __shared__ __attribute__((aligned(16)))
  bf16_t lds[2 * 2 * TILE_ELEMS + (RCG ? 0 : 2 * 2 * 64 * 2) + (FUSED ? 4 * TILE_ELEMS : 0)];
  float* rowc = reinterpret_cast<float*>(lds + 4 * TILE_ELEMS);  // [buf][2][64]
  bf16_t* Kimg = lds + 4 * TILE_ELEMS + 512;
  bf16_t* dsT = Kimg + 2 * TILE_ELEMS;
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
  // FUSED: this wave's K operand is read from the K image (frees 16 VGPRs: the fused
  // pass is at the 256-register cap and spill reloads would drain the dQ atomics)
  bf16x8_t kf[FUSED ? 1 : 4], vf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    if (!FUSED) kf[kk] = ld8(base + C + (long)key * tok + 16 * kk + 8 * hh);
    vf[kk] = ld8(base + 2 * C + (long)key * tok + 16 * kk + 8 * hh);
  }
  if (FUSED) {  // K rows kv0..kv0+127 -> swizzled image (visible after the first barrier)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = threadIdx.x + 256 * j, row = c >> 3, ch = c & 7;
      *reinterpret_cast<u32x4*>(Kimg + img_off(row, ch)) =
          *reinterpret_cast<const u32x4*>(base + C + (long)(kv0 + row) * tok + ch * 8);
    }
  }
  f32x16 dv[2] = {}, dk[2] = {};
  const int t0 = kv0 / 64;
  const int ntiles = T / 64;
  const int wave_kmin = kv0 + 32 * w;
  const float inv_c = -1.f / sc_log2;
  const float* lse_bh = lse + (long)bh * T;
  const float* del_bh = delta + (long)bh * T;
  QD A;
  [[maybe_unused]] QD B;
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
    if (!RCG && threadIdx.x < 128) {  // waves 0 / 1: -lse/c / -delta of the tile's 64 rows
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
    if (!RCG && threadIdx.x < 128) rowc[buf * 128 + threadIdx.x] = x.rc;
  };
  // DIAG is a template-like constant: the causal mask costs 3 VALU per score element
  // (compare, select, index add), so only the diagonal tiles instantiate it — the
  // compiler does not split a runtime-predicated mask out of the unrolled loop itself.
  auto body = [&](int t, auto diag_c) __attribute__((always_inline)) {
    constexpr bool diag = decltype(diag_c)::value;
    const int cur = (t - t0) & 1;
    const int q0 = t * 64;
    if constexpr (ILP && !FUSED) {
      const bf16_t* Qs = lds + cur * 2 * TILE_ELEMS;
      const bf16_t* Ds = Qs + TILE_ELEMS;
      const float* nl = rowc + cur * 128;
      const float* nd = nl + 64;
      f32x16 s[2], dp[2];
      [[maybe_unused]] f32x16 rl_[2], rd_[2];  // RCG: lse / delta of the accumulator rows
      if constexpr (RCG) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int off = (q0 + 32 * qt + 8 * g + 4 * hh) * 4;
            const u32x4 a = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, off, 0, 0));
            const u32x4 d = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rdl, off, 0, 0));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              rl_[qt][4 * g + j] = __uint_as_float(a[j]);
              rd_[qt][4 * g + j] = __uint_as_float(d[j]);
            }
          }
      }
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        if constexpr (RCG) {
          s[qt] = f32x16{};
          dp[qt] = f32x16{};
        } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 a = *reinterpret_cast<const float4*>(nl + 32 * qt + 8 * g + 4 * hh);
          const float4 d = *reinterpret_cast<const float4*>(nd + 32 * qt + 8 * g + 4 * hh);
          s[qt][4 * g] = a.x; s[qt][4 * g + 1] = a.y; s[qt][4 * g + 2] = a.z;
          s[qt][4 * g + 3] = a.w;
          dp[qt][4 * g] = d.x; dp[qt][4 * g + 1] = d.y; dp[qt][4 * g + 2] = d.z;
          dp[qt][4 * g + 3] = d.w;
        }
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
          float p = RCG ? fast_exp2(fmaf(s[qt][i], sc_log2, -rl_[qt][i]))
                        : fast_exp2(s[qt][i] * sc_log2);
          if (diag && key > q0 + 32 * qt + crow(i, hh)) p = 0.f;
          s[qt][i] = p;
          dp[qt][i] = RCG ? p * (dp[qt][i] - rd_[qt][i]) : p * dp[qt][i];
        }
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
    } else {
      const bf16_t* Qs = lds + cur * 2 * TILE_ELEMS;
      const bf16_t* Ds = Qs + TILE_ELEMS;
      const float* nl = rowc + cur * 128;
      const float* nd = nl + 64;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        // S' = Q K^T - LSE/c ; dP' = dO V^T - delta   (rows q, cols = this wave's keys)
        f32x16 s, dp;
        [[maybe_unused]] f32x16 rl_, rd_;
        if constexpr (RCG) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int off = (q0 + 32 * qt + 8 * g + 4 * hh) * 4;
            const u32x4 a = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, off, 0, 0));
            const u32x4 d = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rdl, off, 0, 0));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              rl_[4 * g + j] = __uint_as_float(a[j]);
              rd_[4 * g + j] = __uint_as_float(d[j]);
            }
          }
          s = f32x16{};
          dp = f32x16{};
        } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 a = *reinterpret_cast<const float4*>(nl + 32 * qt + 8 * g + 4 * hh);
          const float4 d = *reinterpret_cast<const float4*>(nd + 32 * qt + 8 * g + 4 * hh);
          s[4 * g] = a.x; s[4 * g + 1] = a.y; s[4 * g + 2] = a.z; s[4 * g + 3] = a.w;
          dp[4 * g] = d.x; dp[4 * g + 1] = d.y; dp[4 * g + 2] = d.z; dp[4 * g + 3] = d.w;
        }
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          s = mfma32(ld8(Qs + 2048 * qt + lo.row[kk]),
                     FUSED ? ld8(Kimg + 2048 * w + lo.row[kk]) : kf[FUSED ? 0 : kk], s);
          dp = mfma32(ld8(Ds + 2048 * qt + lo.row[kk]), vf[kk], dp);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float p = RCG ? fast_exp2(fmaf(s[i], sc_log2, -rl_[i])) : fast_exp2(s[i] * sc_log2);
          if (diag && key > q0 + 32 * qt + crow(i, hh)) p = 0.f;
          s[i] = p;                                   // P
          dp[i] = RCG ? p * (dp[i] - rd_[i]) : p * dp[i];  // dS (wrt scaled scores)
        }
        if (FUSED) {  // dS^T rows = this lane's key, 4 consecutive q per 8-byte write
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float v4[4] = {dp[4 * g], dp[4 * g + 1], dp[4 * g + 2], dp[4 * g + 3]};
            *reinterpret_cast<uint2*>(dsT + img_off(32 * w + r, 4 * qt + g) + 4 * hh) =
                pack4(v4);
          }
        }
        // dV += P^T dO ; dK += dS^T Q   (P / dS registers as A operands, k = q)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8_t pa = acc_frag(s, ks);
          const bf16x8_t da = acc_frag(dp, ks);
          const int kbq = 32 * qt + 16 * ks;
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            dv[dt] = mfma32(pa, tr_frag(Ds, lo, kbq, dt), dv[dt]);
            dk[dt] = mfma32(da, tr_frag(Qs, lo, kbq, dt), dk[dt]);
          }
        }
      }
    }
  };
  auto compute = [&](int t) __attribute__((always_inline)) {
    const int q0 = t * 64;
    if (q0 + 63 >= wave_kmin) {
      if (q0 < wave_kmin + 31) body(t, std::true_type{});
      else body(t, std::false_type{});
    } else if (FUSED) {  // every key of this wave is after every query of the tile: dS = 0
#pragma unroll
      for (int c = 0; c < 8; ++c)
        *reinterpret_cast<uint2*>(dsT + img_off(32 * w + r, c) + 4 * hh) = make_uint2(0, 0);
    }
  };
  const int qh = w >> 1, dh = w & 1;  // FUSED: this wave's dQ block
  float* dq_bh = FUSED ? dq_ws + (long)bh * T * HD : nullptr;
  auto dq_tile = [&](int t) __attribute__((always_inline)) {
    f32x16 acc = {};
#pragma unroll 2  // bounded fragment prefetch: keeps the pass under the register cap
    for (int ks = 0; ks < 8; ++ks)
      acc = mfma32(tr_frag(dsT, lo, 16 * ks, qh), tr_frag(Kimg, lo, 16 * ks, dh), acc);
    float* g = dq_bh + (long)(t * 64 + 32 * qh) * HD + 32 * dh + r;
    if (dbg & 1) {  // diagnostic (ra_knobs[6]): plain stores instead of atomics
#pragma unroll
      for (int i = 0; i < 16; ++i) g[crow(i, hh) * HD] = acc[i];
      return;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) unsafeAtomicAdd(g + crow(i, hh) * HD, acc[i]);
  };
  if constexpr (PF == 2) {
    auto step = [&](int t, QD& held, QD& next) __attribute__((always_inline)) {
      if (t + 2 < ntiles) load_qd(next, t + 2);
      compute(t);
      if (FUSED) {
        __syncthreads();  // dS^T image complete
        if (!(dbg & 2)) dq_tile(t);
      }
      if (t + 1 < ntiles) store_qd(held, t + 1);
      __syncthreads();
    };
    load_qd(A, t0);
    store_qd(A, t0);
    load_qd(A, t0 + 1);  // t0 + 2 <= ntiles
    __syncthreads();
    for (int t = t0; t < ntiles; t += 2) {
      step(t, A, B);
      if (t + 1 < ntiles) step(t + 1, B, A);
    }
  } else {
    load_qd(A, t0);
    store_qd(A, t0);
    __syncthreads();
    for (int t = t0; t < ntiles; ++t) {
      if (t + 1 < ntiles) load_qd(A, t + 1);  // lands during compute(t)
      compute(t);
      if (FUSED) {
        __syncthreads();
        if (!(dbg & 2)) dq_tile(t);
      }
      if (t + 1 < ntiles) store_qd(A, t + 1);  // the other buffer: last read by tile t - 1
      __syncthreads();
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
// PF as in attn_bwd_dkdv_kernel (K/V tiles); ra_knobs[12] = 1 selects PF 1.
// ILP: both 32-key halves of a tile in flight (as attn_bwd_dkdv_kernel's ILP).
// DELTA: the kernel computes delta = rowsum(dO * O) of its own queries (each lane already
// holds half of its query's dO row; O is read the same way and the halves meet by one
// permlane32 swap) and writes it for the dK/dV kernel that runs after it: this replaces the
// attn_bwd_pre_kernel pass (a separate read of O and dO, 50 us per layer at B64 T1024 H12).
template <int PF = 2, bool ILP = false, bool DELTA = false>
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
  float ndel;
  if constexpr (DELTA) {
    float part = 0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bf16x8_t of = ld8(out + ((long)b * T + qrow) * C + h * HD + 16 * kk + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)of[j] * (float)df[kk][j];
    }
    const float dl = half_sum(part);
    if (hh == 0) delta[(long)bh * T + qrow] = dl;
    ndel = -dl;
  } else {
    ndel = -delta[(long)bh * T + qrow];
  }
  f32x16 dq[2] = {};
  const int ntiles = (q0 + 128) / 64;
  const int wave_qmax = q0 + 32 * w + 31;
  KV A;
  [[maybe_unused]] KV B;
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
    if constexpr (ILP) {
      const bf16_t* Ks = lds + (t & 1) * 2 * TILE_ELEMS;
      const bf16_t* Vs = Ks + TILE_ELEMS;
      f32x16 st[2], dpt[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          st[kt][i] = nlq;
          dpt[kt][i] = ndel;
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          st[kt] = mfma32(ld8(Ks + 2048 * kt + lo.row[kk]), qf[kk], st[kt]);
          dpt[kt] = mfma32(ld8(Vs + 2048 * kt + lo.row[kk]), df[kk], dpt[kt]);
        }
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float p = fast_exp2(st[kt][i] * sc_log2);
          if (diag && kv0 + 32 * kt + crow(i, hh) > qrow) p = 0.f;
          dpt[kt][i] = p * dpt[kt][i];
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8_t bfrag = acc_frag(dpt[kt], s2);
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
            dq[dt] = mfma32(tr_frag(Ks, lo, 32 * kt + 16 * s2, dt), bfrag, dq[dt]);
        }
      }
    } else {
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
    }
  };
  auto compute = [&](int t) __attribute__((always_inline)) {
    const int kv0 = t * 64;
    if (kv0 <= wave_qmax) {
      if (kv0 + 63 > q0 + 32 * w) body(t, std::true_type{});
      else body(t, std::false_type{});
    }
  };
  if constexpr (PF == 2) {
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
  } else {
    load_kv(A, 0);
    store_kv(A, 0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
      if (t + 1 < ntiles) load_kv(A, t + 1);
      compute(t);
      if (t + 1 < ntiles) store_kv(A, t + 1);
      __syncthreads();
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

// dqkv[b, t, 0, h, :] = bf16(scale * dq_ws[b, h, t, :]); one thread per 8 head dims,
// threads ordered by the OUTPUT (contiguous 16-B stores, 32-B contiguous reads)
__global__ __launch_bounds__(256) void attn_dq_convert_kernel(const float* __restrict__ ws,
                                                              bf16_t* __restrict__ dqkv, long n8,
                                                              int T, int H, float scale) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const int c8 = (int)(i & 7);
  const long row = i >> 3;  // (b*T + t)*H + h
  const int h = (int)(row % H);
  const long bt = row / H;
  const long b = bt / T, t = bt - b * T;
  const float* src = ws + ((b * H + h) * T + t) * HD + 8 * c8;
  const float4 x0 = *reinterpret_cast<const float4*>(src);
  const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
  float v[8] = {x0.x * scale, x0.y * scale, x0.z * scale, x0.w * scale,
                x1.x * scale, x1.y * scale, x1.z * scale, x1.w * scale};
  *reinterpret_cast<uint4*>(dqkv + bt * 3L * H * HD + (long)h * HD + 8 * c8) = pack8(v);
}

static inline bool attn_shape_ok(int T, int D) { return D == HD && T % 128 == 0 && T >= 128; }

RA_EXPORT int ra_attn_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, int D,
                          float scale, hipStream_t st) {
  if (!attn_shape_ok(T, D)) return hipErrorInvalidValue;
  const float sc_log2 = scale * 1.4426950408889634f;
  if (ra_knobs[9] == 1 && T % 256 == 0)
    hipLaunchKernelGGL(attn_fwd_kernel<2>, dim3(B * H * (T / 256)), dim3(256), 0, st,
                       (const bf16_t*)qkv, (bf16_t*)out, lse, T, H, sc_log2);
  else if (ra_knobs[9] == 2)
    hipLaunchKernelGGL((attn_fwd_kernel<1, 3>), dim3(B * H * (T / 128)), dim3(256), 0, st,
                       (const bf16_t*)qkv, (bf16_t*)out, lse, T, H, sc_log2);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<1>, dim3(B * H * (T / 128)), dim3(256), 0, st,
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
  auto kkv = attn_bwd_dkdv_kernel<false, 2>;
  if (ra_knobs[11] == 1) kkv = attn_bwd_dkdv_kernel<false, 1>;
  else if (ra_knobs[11] == 2) kkv = attn_bwd_dkdv_kernel<false, 1, true>;
  else if (ra_knobs[11] == 3) kkv = attn_bwd_dkdv_kernel<false, 1, false, true>;
  // ra_knobs[13] = 1: the separate delta pre-pass and the dQ kernel after dK/dV (round 4's
  // order); default: dQ first, computing delta on the way (attn_bwd_dq_kernel DELTA)
  if (ra_knobs[13] == 1) {
    hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((rows + 255) / 256), dim3(256), 0, st,
                       (const bf16_t*)out, (const bf16_t*)dout, delta, B * T, T, H);
    hipLaunchKernelGGL(kkv, dim3(B * H * (T / 128)), dim3(256), 0, st,
                       (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv,
                       (float*)nullptr, T, H, sc_log2, scale, 0);
    auto kq = attn_bwd_dq_kernel<2>;
    if (ra_knobs[12] == 1) kq = attn_bwd_dq_kernel<1>;
    else if (ra_knobs[12] == 2) kq = attn_bwd_dq_kernel<1, true>;
    else if (ra_knobs[12] == 3) kq = attn_bwd_dq_kernel<2, true>;
    hipLaunchKernelGGL(kq, dim3(B * H * (T / 128)), dim3(256), 0, st,
                       (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, T, H,
                       sc_log2, scale, (const bf16_t*)nullptr);
    return hipGetLastError();
  }
  auto kq = attn_bwd_dq_kernel<2, false, true>;
  if (ra_knobs[12] == 1) kq = attn_bwd_dq_kernel<1, false, true>;
  else if (ra_knobs[12] == 2) kq = attn_bwd_dq_kernel<1, true, true>;
  else if (ra_knobs[12] == 3) kq = attn_bwd_dq_kernel<2, true, true>;
  hipLaunchKernelGGL(kq, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, T, H,
                     sc_log2, scale, (const bf16_t*)out);
  hipLaunchKernelGGL(kkv, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv,
                     (float*)nullptr, T, H, sc_log2, scale, 0);
  return hipGetLastError();
}

// Fused backward: dK, dV and dQ in one pass over the key blocks (see attn_bwd_dkdv_kernel).
// dq_ws: B*H*T*64 floats of workspace (zeroed here).
RA_EXPORT int ra_attn_bwd_fused(const void* qkv, const void* out, const void* dout,
                                const float* lse, float* delta, float* dq_ws, void* dqkv, int B,
                                int T, int H, int D, float scale, hipStream_t st) {
  if (!attn_shape_ok(T, D)) return hipErrorInvalidValue;
  const float sc_log2 = scale * 1.4426950408889634f;
  const long rows = (long)B * T * H;
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((rows + 255) / 256), dim3(256), 0, st,
                     (const bf16_t*)out, (const bf16_t*)dout, delta, B * T, T, H);
  (void)hipMemsetAsync(dq_ws, 0, (size_t)rows * HD * sizeof(float), st);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel<true>, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, dq_ws,
                     T, H, sc_log2, scale, ra_knobs[6]);
  const long n8 = rows * 8;
  hipLaunchKernelGGL(attn_dq_convert_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0,
                     st, (const float*)dq_ws, (bf16_t*)dqkv, n8, T, H, scale);
  return hipGetLastError();
}

// Split backward as two launches for two streams: ra_attn_bwd_kv (delta pre-pass + dK/dV)
// and ra_attn_bwd_q (dQ, after delta). The caller orders q after kv's pre-pass with an
// event; the two main kernels then run concurrently (each one's causal tail is filled by
// the other's blocks).
RA_EXPORT int ra_attn_bwd_pre(const void* out, const void* dout, float* delta, int B, int T,
                              int H, hipStream_t st) {
  const long rows = (long)B * T * H;
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((rows + 255) / 256), dim3(256), 0, st,
                     (const bf16_t*)out, (const bf16_t*)dout, delta, B * T, T, H);
  return hipGetLastError();
}

RA_EXPORT int ra_attn_bwd_kv(const void* qkv, const void* dout, const float* lse,
                             const float* delta, void* dqkv, int B, int T, int H, int D,
                             float scale, hipStream_t st) {
  if (!attn_shape_ok(T, D)) return hipErrorInvalidValue;
  const float sc_log2 = scale * 1.4426950408889634f;
  auto kkv = attn_bwd_dkdv_kernel<false, 2>;
  if (ra_knobs[11] == 1) kkv = attn_bwd_dkdv_kernel<false, 1>;
  else if (ra_knobs[11] == 2) kkv = attn_bwd_dkdv_kernel<false, 1, true>;
  else if (ra_knobs[11] == 3) kkv = attn_bwd_dkdv_kernel<false, 1, false, true>;
  hipLaunchKernelGGL(kkv, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv,
                     (float*)nullptr, T, H, sc_log2, scale, 0);
  return hipGetLastError();
}

RA_EXPORT int ra_attn_bwd_q(const void* qkv, const void* dout, const float* lse,
                            const float* delta, void* dqkv, int B, int T, int H, int D,
                            float scale, hipStream_t st) {
  if (!attn_shape_ok(T, D)) return hipErrorInvalidValue;
  const float sc_log2 = scale * 1.4426950408889634f;
  auto kq = attn_bwd_dq_kernel<2>;
  if (ra_knobs[12] == 1) kq = attn_bwd_dq_kernel<1>;
  else if (ra_knobs[12] == 2) kq = attn_bwd_dq_kernel<1, true>;
  else if (ra_knobs[12] == 3) kq = attn_bwd_dq_kernel<2, true>;
  hipLaunchKernelGGL(kq, dim3(B * H * (T / 128)), dim3(256), 0, st,
                     (const bf16_t*)qkv, (const bf16_t*)dout, lse, (float*)delta,
                     (bf16_t*)dqkv, T, H, sc_log2, scale, (const bf16_t*)nullptr);
  return hipGetLastError();
}
