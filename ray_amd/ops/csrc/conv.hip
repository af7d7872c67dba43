// NHWC implicit-GEMM convolutions on CDNA4 MFMA for the RLlib Nature-CNN encoder
// (rllib/models/torch/visionnet.py / core/models/torch/encoder.py conv stack:
// 8x8/4 -> 4x4/2 -> 3x3/1, 32/64/64 filters, ReLU).
//
//   ra_conv_fwd    y = relu(conv(x, w) + b)   (bias + ReLU in the epilogue)
//   ra_conv_wgrad  dW = sum_m dY[m]^T . im2col(x)[m]   (split-M partials, then one
//                  reduction that writes the flat gradient buffer directly)
//
// Layouts: activations NHWC (= channels-last NCHW), weights OHWI (= channels-last
// [O, I, KH, KW]), so the GEMM K index k = (kh, kw, ci) is contiguous in both, and
// each receptive-field row kh is one contiguous run of KW*C input elements.
// The first layer reads the uint8 frame batch directly — gathered by a row index
// (the learner's minibatch permutation) and scaled by 1/255 while loading — so no
// gathered/converted bf16 copy of the frames is ever written.
//
// Forward orientation (mfma_f32_32x32x16_bf16, C^T = W . im2col^T): A = weights
// (rows = output channels) from an LDS copy of a 32-filter slice, B = im2col^T
// (columns = 32 output pixels per wave) loaded straight from global memory: lane
// (r, h) needs pixel r's 8 contiguous k values 8h..8h+7 of a 16-wide k step — one
// 16-byte load (8 bytes for uint8). Accumulator register i holds channel
// (i&3) + 8(i>>2) + 4h of pixel r, so the epilogue writes 4 channels (8 bytes) per store.
//
// Weight gradient: the reduction runs over output pixels m, which is the ROW index
// of both dY [M, NOUT] and im2col [M, K]; 64-pixel chunks of both are staged
// row-major in LDS (double buffered, one barrier per chunk) and both MFMA operands
// are read with ds_read_b64_tr_b16 (hardware transpose: k = pixel runs down the
// image's rows). Each workgroup owns one (pixel range, 64- or 128-wide k block) and
// writes a fp32 [NOUT, K] partial; `conv_wgrad_reduce` sums the partials.
#include "common.h"

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4_t tr4(const bf16_t* p) {
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)const_cast<bf16_t*>(p));
  return __builtin_bit_cast(bf16x4_t, v);
}

// 8 uint8 (one uint2) -> 8 bf16 * scale
__device__ __forceinline__ bf16x8_t u8x8_to_bf16(uint2 u, float scale) {
  bf16x8_t r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (__bf16)((float)((u.x >> (8 * j)) & 0xff) * scale);
    r[4 + j] = (__bf16)((float)((u.y >> (8 * j)) & 0xff) * scale);
  }
  return r;
}

struct ConvArgs {
  const void* x;        // NHWC input: bf16, or uint8 frames when U8
  const long* idx;      // U8 only: image b of the batch is frame idx[b] (null = b)
  const bf16_t* w;      // OHWI [NOUT][K]
  const bf16_t* bias;   // [NOUT] (fwd, may be null)
  const bf16_t* dy;     // [M][NOUT] (wgrad)
  void* out;            // fwd: y [M][NOUT] bf16; wgrad: fp32 partials [P][NOUT][K]
  int B, H, W, OH, OW;  // batch, input and output spatial dims
  int rows_per_wg;      // wgrad: output pixels per workgroup (multiple of 64)
  int relu;
  float scale;          // U8 dequantisation scale (1/255)
};

// ------------------------------------------------------------------ forward
// grid (ceil(M/128), NOUT/32): workgroup = 4 waves x 32 pixels, one 32-channel slice of
// the filter bank in LDS (<= 37 KB static: no > 64 KB dynamic-LDS opt-in, which graph
// replays do not honour).
template <int KH, int KW, int C, int S, int NOUT, bool U8>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvArgs a) {
  constexpr int K = KH * KW * C, KWC = KW * C, LDW = K + 8, KS = KWC / 16;
  static_assert(KWC % 16 == 0 && NOUT % 32 == 0, "conv tile shape");
  __shared__ __attribute__((aligned(16))) bf16_t Ws[32 * LDW];
  const int nb = blockIdx.y * 32;
  for (int i = threadIdx.x; i < 32 * (K / 8); i += 256) {
    const int n = i / (K / 8), k8 = i - n * (K / 8);
    *reinterpret_cast<uint4*>(Ws + n * LDW + k8 * 8) =
        reinterpret_cast<const uint4*>(a.w + (long)(nb + n) * K)[k8];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int ohw = a.OH * a.OW, M = a.B * ohw;
  const int m0 = (blockIdx.x * 4 + wv) * 32;
  if (m0 >= M) return;  // no barrier follows
  const int m = min(m0 + r, M - 1);  // tail lanes compute a duplicate and skip the store
  const int b = m / ohw, rem = m - b * ohw, oh = rem / a.OW, ow = rem - oh * a.OW;
  const long img = (U8 && a.idx) ? a.idx[b] : (long)b;
  const long base = img * (long)a.H * a.W * C + ((long)oh * S * a.W + (long)ow * S) * C + 8 * h;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int kh = 0; kh < KH; ++kh) {
    const long rb = base + (long)kh * a.W * C;
    bf16x8_t bf[KS];
#pragma unroll
    for (int kc = 0; kc < KS; ++kc) {
      if constexpr (U8)
        bf[kc] = u8x8_to_bf16(*reinterpret_cast<const uint2*>(
                                  reinterpret_cast<const uint8_t*>(a.x) + rb + kc * 16),
                              a.scale);
      else
        bf[kc] = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const bf16_t*>(a.x) + rb +
                                                    kc * 16);
    }
#pragma unroll
    for (int kc = 0; kc < KS; ++kc) {
      const int k0 = kh * KWC + kc * 16 + 8 * h;
      acc = mfma32(*reinterpret_cast<const bf16x8_t*>(Ws + r * LDW + k0), bf[kc], acc);
    }
  }
  if (m0 + r >= M) return;
  bf16_t* y = reinterpret_cast<bf16_t*>(a.out) + (long)(m0 + r) * NOUT + nb;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n = 8 * q + 4 * h;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = acc[4 * q + j] + (a.bias ? bf2f(a.bias[nb + n + j]) : 0.f);
      if (a.relu) v[j] = fmaxf(v[j], 0.f);
    }
    *reinterpret_cast<uint2*>(y + n) = pack4(v);
  }
}

// ------------------------------------------------------------------ weight gradient
// LDS row strides (elements) chosen so the 4 rows of a transposed read land on
// disjoint 16-bank groups: 64-B rows (32 cols), 192-B rows (64 cols + pad),
// 320-B rows (128 cols + pad).
constexpr int kMaxWgRows = 512;  // wgrad pixels per workgroup (LDS origin table)
template <int COLS> struct Pitch { static constexpr int v = COLS == 32 ? 32 : COLS == 64 ? 96 : 160; };

template <int KH, int KW, int C, int S, int NOUT, bool U8, int KB>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvArgs a) {
  constexpr int K = KH * KW * C, KWC = KW * C;
  constexpr int DS = Pitch<NOUT>::v, XS = Pitch<KB>::v;
  constexpr int DP = 64 * NOUT / 8 / 256, XP = 64 * KB / 8 / 256;  // 16-B pieces per thread
  static_assert(NOUT * KB == 4096, "4 waves x one 32x32 tile");
  static_assert(K % KB == 0 && DP >= 1 && XP >= 1, "wgrad tile shape");
  __shared__ __attribute__((aligned(16))) bf16_t dys[2][64 * DS];
  __shared__ __attribute__((aligned(16))) bf16_t xs[2][64 * XS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5;
  const int ohw = a.OH * a.OW, M = a.B * ohw;
  const int kbase = blockIdx.y * KB;
  const int mbeg = blockIdx.x * a.rows_per_wg, mend = min(M, mbeg + a.rows_per_wg);
  const int nchunks = (mend - mbeg + 63) / 64;

  // Receptive-field origin of every pixel of this workgroup's range, computed once
  // (divisions and the frame-index lookup stay out of the chunk loop, whose loads are
  // then single independent trips)
  __shared__ int sbase[kMaxWgRows];
  for (int j = tid; j < mend - mbeg; j += 256) {
    const int m = mbeg + j, b = m / ohw, rem = m - b * ohw, oh = rem / a.OW, ow = rem - oh * a.OW;
    const long img = (U8 && a.idx) ? a.idx[b] : (long)b;
    sbase[j] = (int)(img * a.H * a.W * C + ((long)oh * S * a.W + (long)ow * S) * C);
  }
  // im2col pieces: PE contiguous k values (16 uint8 = one 16-B load, or 8 bf16); every
  // piece of a thread has the same k (so one k offset), rows rowb + i*rstep of a chunk
  constexpr int PE = U8 ? 16 : 8, XPR = KB / PE, XQ = 64 * XPR / 256;  // XQ pieces/thread
  static_assert(KWC % PE == 0 && 256 % XPR == 0 && XQ >= 1, "im2col pieces");
  const int xk = tid % XPR, xrow = tid / XPR;
  const int kx = kbase + xk * PE, kxh = kx / KWC;
  const int koff = kxh * a.W * C + (kx - kxh * KWC);
  // Raw global data of one chunk in registers (uint8 pieces stay packed until the LDS
  // store, so the loads of a chunk can stay in flight for two chunk steps)
  struct Regs {
    uint4 d[DP], x[XQ];
  };
  auto load = [&](int c, Regs& R) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < DP; ++i) {
      const int pc = tid + 256 * i, row = pc / (NOUT / 8), c8 = pc - row * (NOUT / 8);
      const int m = mbeg + c * 64 + row;
      R.d[i] = m < mend ? *reinterpret_cast<const uint4*>(a.dy + (long)m * NOUT + c8 * 8)
                        : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int local = c * 64 + xrow + i * (256 / XPR);
      if (mbeg + local >= mend) {
        R.x[i] = make_uint4(0, 0, 0, 0);
        continue;
      }
      const long off = (long)sbase[local] + koff;
      if constexpr (U8)
        R.x[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(a.x) + off);
      else
        R.x[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.x) + off);
    }
  };
  auto store = [&](int buf, const Regs& R) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < DP; ++i) {
      const int pc = tid + 256 * i, row = pc / (NOUT / 8), c8 = pc - row * (NOUT / 8);
      *reinterpret_cast<uint4*>(&dys[buf][row * DS + c8 * 8]) = R.d[i];
    }
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int row = xrow + i * (256 / XPR);
      bf16_t* dst = &xs[buf][row * XS + xk * PE];
      if constexpr (U8) {
        const uint4 u = R.x[i];
        *reinterpret_cast<uint4*>(dst) =
            __builtin_bit_cast(uint4, u8x8_to_bf16(make_uint2(u.x, u.y), a.scale));
        *reinterpret_cast<uint4*>(dst + 8) =
            __builtin_bit_cast(uint4, u8x8_to_bf16(make_uint2(u.z, u.w), a.scale));
      } else {
        *reinterpret_cast<uint4*>(dst) = R.x[i];
      }
    }
  };
  __syncthreads();  // sbase

  // wave tile: rows (output channels) nt*32.., columns (k) kt*32..
  constexpr int KTW = KB / 32;
  const int nt = wv / KTW, kt = wv - nt * KTW;
  // transposed-read lane addressing: lane 4q+p of 16-lane group g reads row 4(g>>1)+q,
  // columns 16(g&1) + 4p .. +3 of a 16-row k block; a second read 8 rows further down
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int trow = 4 * (g >> 1) + q, tcol = 16 * (g & 1) + 4 * p;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const bf16_t* D = dys[buf];
    const bf16_t* X = xs[buf];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int r0 = 16 * ks + trow;
      const bf16x4_t a0 = tr4(D + r0 * DS + nt * 32 + tcol);
      const bf16x4_t a1 = tr4(D + (r0 + 8) * DS + nt * 32 + tcol);
      const bf16x4_t b0 = tr4(X + r0 * XS + kt * 32 + tcol);
      const bf16x4_t b1 = tr4(X + (r0 + 8) * XS + kt * 32 + tcol);
      const bf16x8_t af = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const bf16x8_t bfr = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      acc = mfma32(af, bfr, acc);
    }
  };

  // two register sets: chunk c+2 is loading while chunk c is computed from LDS and
  // chunk c+1 is written to the other LDS buffer (one barrier per chunk)
  Regs RA, RB;
  if (nchunks > 0) load(0, RA);
  if (nchunks > 1) load(1, RB);
  if (nchunks > 0) store(0, RA);
  __syncthreads();
  for (int c = 0; c < nchunks; c += 2) {
    if (c + 2 < nchunks) load(c + 2, RA);
    compute(0);
    if (c + 1 < nchunks) store(1, RB);
    __syncthreads();
    if (c + 1 >= nchunks) break;
    if (c + 3 < nchunks) load(c + 3, RB);
    compute(1);
    if (c + 2 < nchunks) store(0, RA);
    __syncthreads();
  }
  // partial tile -> part[blockIdx.x][n][k]
  float* part = reinterpret_cast<float*>(a.out) + (size_t)blockIdx.x * NOUT * K;
  const int col = kbase + kt * 32 + (lane & 31);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int n = nt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
    part[(size_t)n * K + col] = acc[i];
  }
}

// out[j] (+)= sum_p part[p][j], j < NK: 64 columns x 16 partial lanes per block.
template <bool OUT_BF16, bool ACC>
__global__ __launch_bounds__(1024) void conv_wgrad_reduce(const float* __restrict__ part,
                                                          void* out, int P, int NK) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + tx;
  float s0 = 0.f, s1 = 0.f;
  if (j < NK) {
    int pp = ty;
    for (; pp + 16 < P; pp += 32) {
      s0 += part[(size_t)pp * NK + j];
      s1 += part[(size_t)(pp + 16) * NK + j];
    }
    if (pp < P) s0 += part[(size_t)pp * NK + j];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty != 0 || j >= NK) return;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += red[i][tx];
  if (OUT_BF16) {
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + j;
    *o = f2bf(ACC ? s + bf2f(*o) : s);
  } else {
    float* o = reinterpret_cast<float*>(out) + j;
    *o = ACC ? *o + s : s;
  }
}

// ------------------------------------------------------------------ input gradient
// dX[b, ih, iw, ci] = sum over taps (kh, kw) with ih = S*oh + kh, iw = S*ow + kw of
// dY[b, oh, ow, :] . W[:, kh, kw, ci]. Input pixels are split into S*S parity classes
// (ph, pw) = (ih % S, iw % S): inside a class the taps are kh = ph + S*j, kw = pw + S*jw
// and oh = ih/S - j, so each class is a stride-1 implicit GEMM over TAPS*NOUT
// reduction values with the SAME filter taps for every pixel (MFMA operand shared by the
// wave). Orientation as the forward: A = W^T slice [32 ci][tap, co] transposed into LDS
// once per workgroup, B = gathered dY rows (16-B loads, zero outside the output), C =
// 32 input channels x 32 pixels.
struct DgradArgs {
  const bf16_t* dy;   // [B, OH, OW, NOUT]
  const bf16_t* w;    // [NOUT, KH, KW, CI]
  bf16_t* dx;         // [B, H, W, CI]
  int B, H, W, OH, OW;
  int wg_start[10];   // prefix sums of workgroups per parity class (S*S <= 9)
};

template <int KH, int KW, int CI, int S, int NOUT>
__global__ __launch_bounds__(256) void conv_dgrad_kernel(DgradArgs a) {
  constexpr int TH = KH / S, TW = KW / S, TAPS = TH * TW, KP = TAPS * NOUT, LDW = KP + 8;
  static_assert(KH % S == 0 && KW % S == 0 && NOUT % 16 == 0 && CI % 32 == 0, "dgrad shape");
  __shared__ __attribute__((aligned(16))) bf16_t Wt[32 * LDW];
  int cls = 0;
  while (cls + 1 < S * S && (int)blockIdx.x >= a.wg_start[cls + 1]) ++cls;
  const int ph = cls / S, pw = cls % S;
  const int H2 = (a.H - ph + S - 1) / S, W2 = (a.W - pw + S - 1) / S;
  const int cib = blockIdx.y * 32;
  // W[co][kh][kw][ci] -> Wt[ci - cib][t * NOUT + co], t = j * TW + jw (this class's taps)
  for (int i = threadIdx.x; i < TAPS * NOUT * 4; i += 256) {
    const int c8 = i & 3, rest = i >> 2, co = rest % NOUT, t = rest / NOUT;
    const int kh = ph + S * (t / TW), kw = pw + S * (t % TW);
    const uint4 u = *reinterpret_cast<const uint4*>(
        a.w + (((long)co * KH + kh) * KW + kw) * CI + cib + c8 * 8);
    const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 8; ++e)
      Wt[(c8 * 8 + e) * LDW + t * NOUT + co] =
          (bf16_t)((e & 1) ? (wd[e >> 1] >> 16) : (wd[e >> 1] & 0xffffu));
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int npx = a.B * H2 * W2;
  const int m0 = ((blockIdx.x - a.wg_start[cls]) * 4 + wv) * 32;
  if (m0 >= npx) return;
  const int m = min(m0 + r, npx - 1);
  const int b = m / (H2 * W2), rem = m - b * (H2 * W2), ih2 = rem / W2, iw2 = rem - ih2 * W2;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int t = 0; t < TAPS; ++t) {
    const int oh = ih2 - t / TW, ow = iw2 - t % TW;
    const bool ok = oh >= 0 && oh < a.OH && ow >= 0 && ow < a.OW;
    const bf16_t* src = a.dy + (((long)b * a.OH + (ok ? oh : 0)) * a.OW + (ok ? ow : 0)) * NOUT +
                        8 * h;
    bf16x8_t bv[NOUT / 16];
#pragma unroll
    for (int kc = 0; kc < NOUT / 16; ++kc) {
      const uint4 u = ok ? *reinterpret_cast<const uint4*>(src + kc * 16) : make_uint4(0, 0, 0, 0);
      bv[kc] = __builtin_bit_cast(bf16x8_t, u);
    }
#pragma unroll
    for (int kc = 0; kc < NOUT / 16; ++kc)
      acc = mfma32(*reinterpret_cast<const bf16x8_t*>(Wt + r * LDW + t * NOUT + kc * 16 + 8 * h),
                   bv[kc], acc);
  }
  if (m0 + r >= npx) return;
  const int ih = S * ih2 + ph, iw = S * iw2 + pw;
  bf16_t* o = a.dx + (((long)b * a.H + ih) * a.W + iw) * CI + cib;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = acc[4 * q + j];
    *reinterpret_cast<uint2*>(o + 8 * q + 4 * h) = pack4(v);
  }
}

// ------------------------------------------------------------------ dispatch
// Supported layer shapes (KH, KW, C, S, NOUT, U8): the Nature-CNN stack; anything else
// returns hipErrorNotSupported and the caller uses MIOpen.
enum { kUnsupported = -1 };

static int config_id(int KH, int KW, int C, int S, int NOUT, int u8) {
  if (KH == 8 && KW == 8 && C == 4 && S == 4 && NOUT == 32) return u8 ? 0 : 1;
  if (KH == 4 && KW == 4 && C == 32 && S == 2 && NOUT == 64 && !u8) return 2;
  if (KH == 3 && KW == 3 && C == 64 && S == 1 && NOUT == 64 && !u8) return 3;
  return kUnsupported;
}

template <int KH, int KW, int C, int S, int NOUT, bool U8>
static int launch_fwd(const ConvArgs& a, hipStream_t st) {
  const int M = a.B * a.OH * a.OW;
  hipLaunchKernelGGL((conv_fwd_kernel<KH, KW, C, S, NOUT, U8>), dim3((M + 127) / 128, NOUT / 32),
                     dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int KH, int KW, int C, int S, int NOUT, bool U8>
static int launch_wgrad(const ConvArgs& a, int P, hipStream_t st) {
  constexpr int K = KH * KW * C, KB = NOUT == 32 ? 128 : 64;
  hipLaunchKernelGGL((conv_wgrad_kernel<KH, KW, C, S, NOUT, U8, KB>), dim3(P, K / KB), dim3(256),
                     0, st, a);
  return hipGetLastError();
}

// output pixels per wgrad workgroup: ~512 (8 chunks), at least 64
static int wgrad_rows(int M, int K, int NOUT) {
  (void)K;
  (void)NOUT;
  int want = 512;
  if (want > kMaxWgRows) want = kMaxWgRows;
  int r = (want + 63) / 64 * 64;
  return M < r ? (M + 63) / 64 * 64 : r;
}

}  // namespace

// Input-gradient kernels exist for the activation layers (conv2, conv3 shapes).
static int dgrad_id(int KH, int KW, int C, int S, int NOUT) {
  if (KH == 4 && KW == 4 && C == 32 && S == 2 && NOUT == 64) return 0;
  if (KH == 3 && KW == 3 && C == 64 && S == 1 && NOUT == 64) return 1;
  return kUnsupported;
}

RA_EXPORT int ra_conv_dgrad_supported(int KH, int KW, int C, int S, int NOUT) {
  return dgrad_id(KH, KW, C, S, NOUT) != kUnsupported;
}

// dx [B, H, W, C] bf16 (every element written) from dy [B, OH, OW, NOUT] and w OHWI.
RA_EXPORT int ra_conv_dgrad(const void* dy, const void* w, void* dx, int B, int H, int W, int C,
                            int KH, int KW, int S, int NOUT, hipStream_t st) {
  const int id = dgrad_id(KH, KW, C, S, NOUT);
  if (id == kUnsupported || H < KH || W < KW || S * S > 9) return hipErrorNotSupported;
  DgradArgs a{};
  a.dy = (const bf16_t*)dy; a.w = (const bf16_t*)w; a.dx = (bf16_t*)dx;
  a.B = B; a.H = H; a.W = W; a.OH = (H - KH) / S + 1; a.OW = (W - KW) / S + 1;
  int total = 0;
  for (int c = 0; c < S * S; ++c) {
    const int ph = c / S, pw = c % S;
    const int np = B * ((H - ph + S - 1) / S) * ((W - pw + S - 1) / S);
    a.wg_start[c] = total;
    total += (np + 127) / 128;
  }
  for (int c = S * S; c < 10; ++c) a.wg_start[c] = total;
  const dim3 g(total, C / 32), b(256);
  if (id == 0) hipLaunchKernelGGL((conv_dgrad_kernel<4, 4, 32, 2, 64>), g, b, 0, st, a);
  else hipLaunchKernelGGL((conv_dgrad_kernel<3, 3, 64, 1, 64>), g, b, 0, st, a);
  return hipGetLastError();
}

RA_EXPORT int ra_conv_supported(int KH, int KW, int C, int S, int NOUT, int u8) {
  return config_id(KH, KW, C, S, NOUT, u8) != kUnsupported;
}

// y [B*OH*OW][NOUT] bf16 = act(conv(x, w) + bias); x NHWC [*, H, W, C] (uint8 rows
// selected by idx when u8). relu: 0/1. scale: uint8 dequantisation.
RA_EXPORT int ra_conv_fwd(const void* x, const long* idx, int u8, const void* w, const void* bias,
                          void* y, int B, int H, int W, int C, int KH, int KW, int S, int NOUT,
                          float scale, int relu, hipStream_t st) {
  const int id = config_id(KH, KW, C, S, NOUT, u8);
  if (id == kUnsupported || H < KH || W < KW) return hipErrorNotSupported;
  ConvArgs a{};
  a.x = x; a.idx = idx; a.w = (const bf16_t*)w; a.bias = (const bf16_t*)bias; a.out = y;
  a.B = B; a.H = H; a.W = W; a.OH = (H - KH) / S + 1; a.OW = (W - KW) / S + 1;
  a.relu = relu; a.scale = scale;
  switch (id) {
    case 0: return launch_fwd<8, 8, 4, 4, 32, true>(a, st);
    case 1: return launch_fwd<8, 8, 4, 4, 32, false>(a, st);
    case 2: return launch_fwd<4, 4, 32, 2, 64, false>(a, st);
    default: return launch_fwd<3, 3, 64, 1, 64, false>(a, st);
  }
}

// fp32 workspace (floats) for ra_conv_wgrad
RA_EXPORT long ra_conv_wgrad_work(int B, int H, int W, int C, int KH, int KW, int S, int NOUT) {
  const int OH = (H - KH) / S + 1, OW = (W - KW) / S + 1, M = B * OH * OW, K = KH * KW * C;
  const int rows = wgrad_rows(M, K, NOUT);
  return (long)((M + rows - 1) / rows) * NOUT * K;
}

// dW [NOUT][K] (OHWI) (+)= sum over output pixels of dY^T . im2col(x).
// flags: bit0 accumulate into dw, bit1 dw is fp32 (else bf16).
// work_cap: floats available at `work` (checked: the partial slab size depends on knob 7).
RA_EXPORT int ra_conv_wgrad(const void* x, const long* idx, int u8, const void* dy, float* work,
                            long work_cap, void* dw, int flags, int B, int H, int W, int C, int KH,
                            int KW, int S, int NOUT, float scale, hipStream_t st) {
  const int id = config_id(KH, KW, C, S, NOUT, u8);
  if (id == kUnsupported || H < KH || W < KW) return hipErrorNotSupported;
  ConvArgs a{};
  a.x = x; a.idx = idx; a.dy = (const bf16_t*)dy; a.out = work;
  a.B = B; a.H = H; a.W = W; a.OH = (H - KH) / S + 1; a.OW = (W - KW) / S + 1;
  a.scale = scale;
  const int M = B * a.OH * a.OW, K = KH * KW * C;
  a.rows_per_wg = wgrad_rows(M, K, NOUT);
  const int P = (M + a.rows_per_wg - 1) / a.rows_per_wg;
  if ((long)P * NOUT * K > work_cap) return hipErrorInvalidValue;
  int e;
  switch (id) {
    case 0: e = launch_wgrad<8, 8, 4, 4, 32, true>(a, P, st); break;
    case 1: e = launch_wgrad<8, 8, 4, 4, 32, false>(a, P, st); break;
    case 2: e = launch_wgrad<4, 4, 32, 2, 64, false>(a, P, st); break;
    default: e = launch_wgrad<3, 3, 64, 1, 64, false>(a, P, st);
  }
  if (e != hipSuccess) return e;
  const int NK = NOUT * K;
  const dim3 g((NK + 63) / 64), b(1024);
  switch (((flags & 1) ? 2 : 0) | ((flags & 2) ? 0 : 1)) {
    case 0: hipLaunchKernelGGL((conv_wgrad_reduce<false, false>), g, b, 0, st, work, dw, P, NK); break;
    case 1: hipLaunchKernelGGL((conv_wgrad_reduce<true, false>), g, b, 0, st, work, dw, P, NK); break;
    case 2: hipLaunchKernelGGL((conv_wgrad_reduce<false, true>), g, b, 0, st, work, dw, P, NK); break;
    default: hipLaunchKernelGGL((conv_wgrad_reduce<true, true>), g, b, 0, st, work, dw, P, NK);
  }
  return hipGetLastError();
}
