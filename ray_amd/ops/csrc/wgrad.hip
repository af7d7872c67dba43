// Weight-gradient GEMM for nn.Linear on CDNA4 (gfx950), fp32 accumulation into the flat
// gradient buffer:
//
//   dW[N, K] (+)= sum_t dY[t, n] * X[t, k]        t = 0 .. M-1 (tokens), bf16 operands
//   db[N]    (+)= sum_t dY[t, n]                  (optional: the bias gradient, fused)
//
// Both operands are stored token-major ([M, N] and [M, K] row-major, the activations as
// autograd saved them), so the reduction index t is the ROW index of both. A 64-token
// K-step of each operand is staged row-major in LDS (global_load_lds, 16 B per lane, two
// 512-byte rows per wave instruction) and both MFMA operands are read with
// ds_read_b64_tr_b16: the hardware transpose read hands each lane 4 consecutive tokens of
// one column, two of them make the 8-token operand fragment of v_mfma_f32_16x16x32_bf16
// (cdna_hip_programming.md §5.5 T10). No transposed copy of dY or X is ever written.
//
// Geometry: 256 (n) x 256 (k) output tile per workgroup, 8 waves as 2 (n) x 4 (k), each
// wave 128 n x 64 k = 8 x 4 accumulators of 16 x 16 (128 VGPRs). MFMA orientation
// D[k][n] = X_frag . dY_frag: a lane's 4 accumulator registers are 4 consecutive k of
// one n, i.e. one 16-byte fp32 store into the row-major [N, K] gradient.
//
// Split-K over tokens fills the chip: grid = tiles x S, S chosen by the host so that
// tiles x S <= #CUs (one wave of workgroups, 1 per CU at 128 KB LDS). Workgroups of one
// split (one token range) are packed onto one XCD (bijective XCD remap, T1), so every dY /
// X panel of that token range is fetched from HBM once and re-read from that XCD's L2 by
// the 3-12 tiles that share it. S == 1: the workgroup read-modify-writes its tile of the
// sink directly (single writer). S > 1: each split writes an fp32 slab [S][N][K], summed
// into the sink by ra_splitk_accum (one HBM pass, far fewer bytes than hipBLASLt's 16-way
// batched partials).
//
// LDS image of one operand tile: [64 tokens][256 cols] bf16, 512-byte rows. Bank swizzle
// for the transposed reads: 16-byte chunk c of row r is stored at chunk c ^ 2 f(r),
// f(r) = (r & 3) | ((r >> 1) & 4). One 32-lane half of a tr read touches rows
// {r0..r0+3, r0+8..r0+11} x one 32-byte column pair; f gives those 8 rows 8 distinct pair
// slots of the 256-byte bank row -> conflict-free. The DMA destination is lane-linear, so
// the permutation is applied to the per-lane global SOURCE address and the same XOR on the
// read address (rule 21).
//
// Schedule: the staggered two-group loop of gemm.hip (variant 0): per K-step
// R0 | M0 | R1 | M1 with a barrier between slots, waves 4-7 one barrier behind waves 0-3,
// so in every slot one wave of each SIMD issues MFMAs while its partner reads LDS.
//
// Reference: torch autograd's linear backward (dW = grad_output^T @ input), the op the
// reference's Ray Train GPT-2 benchmark runs through DDP
// (release/air_tests/air_benchmarks/workloads/torch_benchmark.py:81).
#include "common.h"

namespace {

typedef __bf16 bf16x8w_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4w_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2w_t __attribute__((ext_vector_type(2)));
typedef short s16x4w_t __attribute__((ext_vector_type(4)));
typedef float f32x4w_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_w;
typedef __attribute__((address_space(1))) void glb_void_w;

constexpr int kT = 64;            // tokens per K-step
constexpr int kTile = 256;        // output tile edge (n and k)
constexpr int kImg = kT * kTile;  // bf16 elements of one operand image
constexpr int kStage = 2 * kImg;  // X image then dY image
constexpr int kThreads = 512;

__device__ __forceinline__ int fsw(int r) { return (r & 3) | ((r >> 1) & 4); }

__device__ __forceinline__ bf16x4w_t tr4(const bf16_t* p) {
  typedef __attribute__((address_space(3))) s16x4w_t lds_s16x4;
  s16x4w_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)const_cast<bf16_t*>(p));
  return __builtin_bit_cast(bf16x4w_t, v);
}

__device__ __forceinline__ int xcd_remap_w(int b, int G) {
  const int q = G / 8, rr = G % 8, x = b % 8;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + b / 8;
}

// 16-byte global -> LDS DMA as inline asm (LDS address = M0 + lane * 16). Through the
// builtin, hipcc cannot tell the DMA's LDS write from the fragment reads of the other
// stage buffer and drains the prefetch with s_waitcnt vmcnt(0) in front of them; as asm it
// is ordered only by the loop's explicit vmcnt + barrier protocol. M0 saved and restored.
__device__ __forceinline__ void glds16_w(const bf16_t* gsrc, bf16_t* ldst) {
  const unsigned la = __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long)(__attribute__((address_space(3))) void*)ldst);
  unsigned saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(gsrc), "s"(la)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm_w() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct WgradArgs {
  const bf16_t* dy;  // [M][ldy]
  const bf16_t* x;   // [M][ldx]
  long ldy, ldx;
  void* out;         // S == 1: the sink [N][K] (fp32 or bf16); S > 1: fp32 slabs [S][N][K]
  float* bias_out;   // S == 1: the bias sink (fp32 / bf16 by flags); S > 1: fp32 [S][N]
  int N, K, nks;     // nks = M / 64 token steps
  int S, tk_cnt, ntiles;
  int flags;         // bit0: sink bf16, bit1: accumulate into the sink, bit2: bias grad
};

// One operand tile (64 token rows x 256 columns from col0) -> swizzled lane-linear image.
// Wave w stages rows 8w .. 8w+7 (4 DMA instructions of 2 rows each).
__device__ __forceinline__ void stage_t(bf16_t* img, const bf16_t* __restrict__ g, long ld,
                                        int col0, int cols, long t0, int w, int lane) {
  const int rsub = lane >> 5, cp = lane & 31;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 8 * w + 2 * j + rsub;
    const int c = cp ^ (2 * fsw(r));
    int col = col0 + 8 * c;
    col = col < cols ? col : cols - 8;  // ragged edge: clamp (outputs masked at the store)
    const bf16_t* src = g + (t0 + r) * ld + col;
    glds16_w(src, img + (8 * w + 2 * j) * kTile);
  }
}

// One workgroup's share of one output tile: acc (+ bias column sums) over `total` token
// steps from `s_beg`. Shared by the single-problem and the grouped kernel.
struct TileJob {
  const bf16_t* dy;
  const bf16_t* x;
  long ldy, ldx;
  int N, K, n0, k0, s_beg, total;
  bool do_bias;
};

__device__ __forceinline__ void wgrad_mainloop(bf16_t* lds, const TileJob& j,
                                               f32x4w_t (&acc)[4][8], float (&bsum)[2],
                                               int w, int lane) {
  const int wm = w >> 2, wn = w & 3;  // wave tile: n rows 128 wm.., k cols 64 wn..
  const bool g1 = wm == 1;             // wave-uniform: the late group
  const bool do_bias = j.do_bias;
  const int total = j.total;

  // per-lane tr-read addresses (elements, relative to an image base; + ks*32 rows and the
  // +4-row second read are lane-independent immediates)
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int fl = q | ((gq & 1) << 2);
  const int row_off = (8 * gq + q) * kTile + 4 * (p & 1);
  int xoff[4], yoff[8];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const int m = wn * 4 + kb;  // 16-col block within the tile
    xoff[kb] = row_off + 8 * ((2 * m + (p >> 1)) ^ (2 * fl));
  }
#pragma unroll
  for (int nb = 0; nb < 8; ++nb) {
    const int m = wm * 8 + nb;
    yoff[nb] = row_off + 8 * ((2 * m + (p >> 1)) ^ (2 * fl));
  }

  auto stage = [&](int buf, int ks) __attribute__((always_inline)) {
    bf16_t* img = lds + buf * kStage;
    const long t0 = (long)ks * kT;
    stage_t(img, j.x, j.ldx, j.k0, j.K, t0, w, lane);
    stage_t(img + kImg, j.dy, j.ldy, j.n0, j.N, t0, w, lane);
  };
  auto barrier = []() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) acc[i][jj] = f32x4w_t{0.f, 0.f, 0.f, 0.f};
  bsum[0] = bsum[1] = 0.f;
  bf16x8w_t xf[4], yf[8];

  auto read_frags = [&](int buf, int h) __attribute__((always_inline)) {
    const bf16_t* sx = lds + buf * kStage + h * 32 * kTile;
    const bf16_t* sy = sx + kImg;
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const bf16x4w_t lo = tr4(sy + yoff[nb]);
      const bf16x4w_t hi = tr4(sy + yoff[nb] + 4 * kTile);
      yf[nb] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const bf16x4w_t lo = tr4(sx + xoff[kb]);
      const bf16x4w_t hi = tr4(sx + xoff[kb] + 4 * kTile);
      xf[kb] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto mfma_cluster = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int nb = 0; nb < 8; ++nb)
        acc[kb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[kb], yf[nb], acc[kb][nb], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (do_bias) {
      // bias gradient: this wave sums n-blocks 2wn, 2wn+1 of its dY fragments (the four
      // k-waves of a wave row split the eight blocks), 4 dot2 per fragment beside the MFMAs
      // (wn is wave-uniform but not a constant: one scalar branch per value keeps the
      // fragment indices static — a runtime index would put yf in scratch, rule 20)
      auto dot8 = [&](const bf16x8w_t& v, float& acc_) __attribute__((always_inline)) {
        const bf16x2w_t one = {(__bf16)1.f, (__bf16)1.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16x2w_t pr = {v[2 * e], v[2 * e + 1]};
          acc_ = __builtin_amdgcn_fdot2_f32_bf16(pr, one, acc_, false);
        }
      };
      if (wn == 0) {
        dot8(yf[0], bsum[0]);
        dot8(yf[1], bsum[1]);
      } else if (wn == 1) {
        dot8(yf[2], bsum[0]);
        dot8(yf[3], bsum[1]);
      } else if (wn == 2) {
        dot8(yf[4], bsum[0]);
        dot8(yf[5], bsum[1]);
      } else {
        dot8(yf[6], bsum[0]);
        dot8(yf[7], bsum[1]);
      }
    }
  };

  if (total > 0) {
    stage(0, j.s_beg);
    wait_vm_w<0>();
  }
  barrier();
  if (g1) barrier();
  for (int s = 0; s < total; ++s) {
    const int buf = s & 1;
    if (s + 1 < total) stage(buf ^ 1, j.s_beg + s + 1);  // buffer of step s-1: reads retired
    read_frags(buf, 0);
    barrier();
    mfma_cluster();
    barrier();
    read_frags(buf, 1);
    if (g1) wait_vm_w<0>();
    barrier();
    mfma_cluster();
    if (!g1) wait_vm_w<0>();
    barrier();
  }
  if (!g1) barrier();  // group 1 ran one extra barrier at the start
  if (do_bias) {
    // lanes l, l+16, l+32, l+48 hold different tokens of the same column
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bsum[i] += __shfl_xor(bsum[i], 16, 64);
      bsum[i] += __shfl_xor(bsum[i], 32, 64);
    }
  }
}

template <int MODE>  // 0: fp32 slab store, 1: fp32 sink RMW, 2: bf16 sink RMW
__global__ __launch_bounds__(kThreads) void wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * kStage];
  const int G = gridDim.x;
  const int L = xcd_remap_w(blockIdx.x, G);
  const int split = L / a.ntiles, tile = L - split * a.ntiles;
  const int tn = tile / a.tk_cnt, tk = tile - tn * a.tk_cnt;
  const int n0 = tn * kTile, k0 = tk * kTile;
  const int s_beg = (int)((long)split * a.nks / a.S);
  const int s_end = (int)((long)(split + 1) * a.nks / a.S);

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wm = w >> 2, wn = w & 3;
  const bool do_bias = (a.flags & 4) && tk == 0;
  f32x4w_t acc[4][8];
  float bsum[2];
  const TileJob job{a.dy, a.x, a.ldy, a.ldx, a.N, a.K, n0, k0, s_beg, s_end - s_beg, do_bias};
  wgrad_mainloop(lds, job, acc, bsum, w, lane);

  // ---- epilogue: lane holds D[k = kc + 4(lane>>4) + r][n = nc + (lane & 15)]
  const int nrow = n0 + wm * 128 + (lane & 15);
  const int kcol = k0 + wn * 64 + 4 * (lane >> 4);
  const long NK = (long)a.N * a.K;
  if (MODE == 0) {
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const int n = nrow + nb * 16;
      if (n >= a.N) continue;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int k = kcol + kb * 16;
        if (k >= a.K) continue;  // K % 4 == 0: a lane's 4 columns are all valid or none
        const f32x4w_t v = acc[kb][nb];
        float* dst = reinterpret_cast<float*>(a.out) + (long)split * NK + (long)n * a.K + k;
        *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  } else {
    // read-modify-write of the sink, 8 loads in flight per batch: addresses are clamped to
    // a valid element (never a branch around a load, which would serialise the batch) and
    // only the stores are masked
    const bool acc_old = a.flags & 2;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int k = kcol + kb * 16;
      const int kc = k < a.K ? k : a.K - 4;
      float old[8][4];
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        const int n = nrow + nb * 16;
        const long o = (long)(n < a.N ? n : a.N - 1) * a.K + kc;
        if (MODE == 1) {
          const float4 t = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.out) + o);
          old[nb][0] = t.x, old[nb][1] = t.y, old[nb][2] = t.z, old[nb][3] = t.w;
        } else {
          unpack4(*reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(a.out) + o),
                  old[nb]);
        }
      }
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        const int n = nrow + nb * 16;
        if (n >= a.N || k >= a.K) continue;
        const f32x4w_t v = acc[kb][nb];
        float f[4] = {v[0], v[1], v[2], v[3]};
        if (acc_old) {
#pragma unroll
          for (int i = 0; i < 4; ++i) f[i] += old[nb][i];
        }
        const long o = (long)n * a.K + k;
        if (MODE == 1)
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.out) + o) =
              make_float4(f[0], f[1], f[2], f[3]);
        else
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(a.out) + o) = pack4(f);
      }
    }
  }
  if (do_bias) {
    if (lane < 16) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int n = n0 + wm * 128 + (2 * wn + i) * 16 + lane;
        if (n >= a.N) continue;
        if (MODE == 0) {
          a.bias_out[(long)split * a.N + n] = bsum[i];
        } else if (MODE == 1) {
          float* d = a.bias_out + n;
          *d = (a.flags & 2) ? *d + bsum[i] : bsum[i];
        } else {
          bf16_t* d = reinterpret_cast<bf16_t*>(a.bias_out) + n;
          *d = f2bf((a.flags & 2) ? bf2f(*d) + bsum[i] : bsum[i]);
        }
      }
    }
  }
}

int g_cus_w = 0;

}  // namespace

// dW[N][K] (+)= dY[:M]^T X[:M] (+ bias gradient) over the first M - M % 64 tokens.
//   S = 1: RMW into `sink` (flags bit0: bf16 sink, bit1: accumulate) and `bias_sink`.
//   S > 1: fp32 slabs ws[S][N][K] (+ bias slabs bws[S][N]); the caller sums them.
// Requirements (checked): N % 8 == 0, K % 8 == 0, ldy / ldx % 8 == 0, 16-byte aligned
// pointers. S (>= 1, clamped to the 64-token slices) is chosen by ra_wgrad_splits.
RA_EXPORT int ra_wgrad(const void* dy, long ldy, const void* x, long ldx, int M, int N, int K,
                       int S, void* out, void* bias_out, int flags, hipStream_t st) {
  if (M < 64 || N <= 0 || K <= 0 || N % 8 || K % 8 || ldy % 8 || ldx % 8 || S < 1)
    return hipErrorInvalidValue;
  if ((flags & 4) && bias_out == nullptr) return hipErrorInvalidValue;
  WgradArgs a;
  a.dy = (const bf16_t*)dy;
  a.x = (const bf16_t*)x;
  a.ldy = ldy;
  a.ldx = ldx;
  a.out = out;
  a.bias_out = (float*)bias_out;
  a.N = N;
  a.K = K;
  a.nks = M / kT;
  a.tk_cnt = (K + kTile - 1) / kTile;
  a.ntiles = ((N + kTile - 1) / kTile) * a.tk_cnt;
  if (S > a.nks) S = a.nks;
  a.S = S;
  a.flags = flags;
  const int G = a.ntiles * S;
  void (*k)(WgradArgs);
  if (S == 1)
    k = (flags & 1) ? wgrad_kernel<2> : wgrad_kernel<1>;
  else
    k = wgrad_kernel<0>;
  hipLaunchKernelGGL(k, dim3(G), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

// Splits that fill the chip with one wave of workgroups: tiles * S <= #CUs (fewer tiles
// than CUs), or the fewest partly-filled waves (more tiles than CUs).
RA_EXPORT int ra_wgrad_splits(int M, int N, int K) {
  if (g_cus_w == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_cus_w, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        g_cus_w <= 0)
      g_cus_w = 256;
  }
  // (measured: two waves of shorter workgroups or a partial fill of the CUs were no
  // faster in the step, profiles/r5/r5ah; fixed split counts on several side streams
  // slower, profiles/r6/r6b)
  const int tiles = ((N + kTile - 1) / kTile) * ((K + kTile - 1) / kTile);
  int S = g_cus_w / tiles;
  const int nks = M / kT;
  if (S < 1) {
    // more tiles than CUs (the LM head's dW: 197 x 3 = 591 tiles): the split count that
    // minimises the partly-filled last wave, ceil(tiles * S / CUs) / S in full-K tile
    // times (591 tiles: S = 3, 7 waves of 1/3-K workgroups = 2.33 vs 3 at S = 1)
    S = 1;
    double best = (double)((tiles + g_cus_w - 1) / g_cus_w);
    for (int s = 2; s <= 4 && s <= nks; ++s) {
      const double t = (double)((tiles * s + g_cus_w - 1) / g_cus_w) / s;
      if (t < best - 1e-9) best = t, S = s;
    }
  }
  if (S > nks) S = nks;
  if (S < 1) S = 1;
  return S;
}
