// Persistent bf16 MFMA GEMM for the GPT-2 projections, with fused epilogues.
//
//   C[M, N] = epi( A[M, K] · B[N, K]^T )        bf16 in, fp32 accumulate, bf16 out
//
// "NT" form only: both operands K-contiguous (nn.Linear's forward x·W^T; the input
// gradient dY·W takes W^T as B, a cheap per-step transpose). Epilogues (template EPI):
//   EPI_NONE       C = acc
//   EPI_BIAS       C = acc + bias[n]
//   EPI_BIAS_GELU  aux = acc (pre-activation, saved for backward), C = gelu_tanh(acc + bias)
//   EPI_DGELU      C = acc * gelu_tanh'(aux + bias)  and per-128-row column partial sums of
//                  C into colpart[M/128][N] (the bias gradient, finished by colsum_launch)
// so the MLP's bias+GELU forward pass and its GELU-backward + bias-gradient pass (two full
// HBM round trips of the [tokens, 3072] activation each) disappear into the GEMMs.
//
// Design (cdna_hip_programming.md §5):
//  * 256x256 output tile, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns
//    128 x 64 of C = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (128 VGPRs).
//  * Operands staged global -> LDS with 16-byte global_load_lds (no VGPR round trip), two
//    64 KB stage buffers: tile k+1 streams in while tile k is consumed; one vmcnt(0) +
//    barrier per K-step.
//  * LDS images are lane-linear (the DMA writes base + lane*16); the bank swizzle is put on
//    the per-lane SOURCE address (chunk p of row r holds global chunk p ^ ((r>>1)&7)) and
//    the same XOR on the ds_read_b128 — each 16-lane read group then covers all 16 slots
//    of the 256-B bank row (rule 21 / T2).
//  * Persistent: one workgroup per CU walks tiles L, L+G, ...; the K-steps of consecutive
//    tiles form ONE pipeline, so the next tile's first stage is in flight during the
//    current tile's last K-step and its epilogue stores drain under the next MFMAs.
//  * XCD-aware: logical block = contiguous chunk per XCD (T1), tiles ordered so that the
//    blocks of one XCD share operand panels in its L2.
//  * MFMA orientation D = B_tile · A_tile^T: a lane's 4 accumulator registers are 4
//    consecutive output COLUMNS of one row, so every store / aux load is one 8-byte access.
#include "common.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBM = 256, kBN = 256, kThreads = 512;

enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_DGELU = 3 };

__device__ __forceinline__ float gelu_fwd(float u) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float z = k0 * (u + k1 * u * u * u);
  const float e = __builtin_amdgcn_exp2f(2.885390081777927f * z);
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  return 0.5f * u * (1.f + t);
}
__device__ __forceinline__ float gelu_grad(float u) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float z = k0 * (u + k1 * u * u * u);
  const float e = __builtin_amdgcn_exp2f(2.885390081777927f * z);
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  const float dz = k0 * (1.f + 3.f * k1 * u * u);
  return 0.5f * (1.f + t) + 0.5f * u * (1.f - t * t) * dz;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// 16-byte global -> LDS DMA as inline asm (LDS address = M0 + lane * 16), M0 saved and
// restored. Through __builtin_amdgcn_global_load_lds hipcc cannot tell the DMA's LDS write
// from the fragment reads of the other stage buffer and puts s_waitcnt vmcnt(0) in front of
// them, draining the prefetch every K-step (the same fix as ops/csrc/wgrad.hip glds16_w).
__device__ __forceinline__ void glds16(const bf16_t* gsrc, bf16_t* ldst) {
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


// LDS bank swizzle of a [rows][BK] bf16 image: 16-B chunk p of row r holds global chunk
// p ^ swz(r). BK = 64 (128-B rows, two rows per 256-B bank row): (r>>1)&7; BK = 32 (64-B
// rows, four per bank row): (r>>2)&3. Either way the 16 lanes of a ds_read_b128 group
// (16 consecutive rows, one logical chunk) hit 16 distinct 16-B slots.
template <int BK>
__device__ __forceinline__ int swz(int r) {
  return BK == 64 ? (r >> 1) & 7 : (r >> 2) & 3;
}

// One operand tile (256 rows x BK) -> lane-linear LDS image. A DMA instruction moves 1 KB
// (64 lanes x 16 B) = 1024 / (2 BK) rows; wave w stages rows 32w .. 32w+31.
template <int BK>
__device__ __forceinline__ void stage_operand(bf16_t* img, const bf16_t* __restrict__ g,
                                              long ld, int row0, int rows, int k0, int w,
                                              int lane) {
  constexpr int CPR = BK / 8;          // 16-B chunks per row
  constexpr int RPI = 64 / CPR;        // rows per DMA instruction
  constexpr int NI = 32 / RPI;         // instructions per wave
  const int rsub = lane / CPR, p = lane % CPR;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int r = 32 * w + RPI * j + rsub;  // row within the tile
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;  // clamp ragged edges (results masked at the store)
    const int ch = p ^ swz<BK>(r);
    const bf16_t* src = g + (long)gr * ld + k0 + 8 * ch;
    glds16(src, img + (32 * w + RPI * j) * BK);
  }
}

__device__ __forceinline__ int xcd_remap(int b, int G) {
  // bijective for any G (guide §5 'XCD swizzle must be bijective')
  const int q = G / 8, rr = G % 8, x = b % 8;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + b / 8;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Tile epilogue: wave (wm, wn)'s 128 x 64 block of C from its accumulators, then zero them.
template <int EPI>
__device__ __forceinline__ void epilogue_tile(f32x4_t (&acc)[4][8], int m0, int n0, int wm, int wn,
                                            int lane, int M, int N, bf16_t* __restrict__ C,
                                            long ldc, const bf16_t* __restrict__ bias,
                                            bf16_t* __restrict__ aux, long ldaux,
                                            float* __restrict__ colpart) {
  const int mrow = m0 + wm * 128 + (lane & 15);
  const int ncol = n0 + wn * 64 + 4 * (lane >> 4);
  float csum[4][4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int n = ncol + nb * 16;
    const bool nok = n < N;  // N % 4 == 0: a lane's 4 columns are all valid or all not
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (EPI != EPI_NONE && nok) unpack4(*reinterpret_cast<const uint2*>(bias + n), bv);
#pragma unroll
    for (int i = 0; i < 4; ++i) csum[nb][i] = 0.f;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      const int m = mrow + mb * 16;
      if (!nok || m >= M) continue;
      float v[4] = {acc[nb][mb][0], acc[nb][mb][1], acc[nb][mb][2], acc[nb][mb][3]};
      if (EPI == EPI_BIAS) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += bv[i];
      } else if (EPI == EPI_BIAS_GELU) {
        *reinterpret_cast<uint2*>(aux + (long)m * ldaux + n) = pack4(v);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = gelu_fwd(v[i] + bv[i]);
      } else if (EPI == EPI_DGELU) {
        float u[4];
        unpack4(*reinterpret_cast<const uint2*>(aux + (long)m * ldaux + n), u);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] *= gelu_grad(u[i] + bv[i]);
          csum[nb][i] += v[i];
        }
      }
      *reinterpret_cast<uint2*>(C + (long)m * ldc + n) = pack4(v);
    }
  }
  if (EPI == EPI_DGELU) {
    // sum the 16 rows held by lanes l&15 = 0..15 (same columns), then lanes 0,16,32,48
    // write the wave's 128-row partial of their 4 x 4 columns
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float s = csum[nb][i];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        csum[nb][i] = s;
      }
    if ((lane & 15) == 0 && m0 + wm * 128 < M) {  // colpart has ceil(M / 128) rows
      float* prow = colpart + (long)(m0 / 128 + wm) * N;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int n = ncol + nb * 16;
        if (n < N)
          *reinterpret_cast<float4*>(prow + n) =
              make_float4(csum[nb][0], csum[nb][1], csum[nb][2], csum[nb][3]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
}

// Staggered two-group schedule: BK = 64, two stage buffers (measured faster than the
// single-group, BK 32 x 4-stage and quadrant 8-phase forms it replaced: profiles/r5).
// Waves w and w+4 share a SIMD; waves 0-3 (group 0) and 4-7 (group 1) run the same
// slot sequence per K-step — R0 (stage next step, read ks0 fragments) | M0 (16x16x32
// MFMA cluster on ks0) | R1 | M1 — with barriers between slots, and group 1 starts one
// barrier late. In every slot one wave of each SIMD reads LDS while the other issues its
// 32 MFMAs, so the MFMA pipe never idles behind a ds_read latency (the guide's 8-phase
// idea in its smallest form). Every R slot retires its reads (lgkmcnt(0)) before the
// barrier so that the DMA restaging a buffer can never overtake them; a step's DMAs are
// waited by their issuing wave before the barrier preceding group 0's first read of it.
template <int EPI>
__global__ __launch_bounds__(kThreads) void gemm_nt_stagger_kernel(
    const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ B, long ldb,
    bf16_t* __restrict__ C, long ldc, int M, int N, int K, const bf16_t* __restrict__ bias,
    bf16_t* __restrict__ aux, long ldaux, float* __restrict__ colpart) {
  constexpr int BK = 64;
  constexpr int kStage = (kBM + kBN) * BK;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * kStage];
  const int G = gridDim.x;
  const int L = xcd_remap(blockIdx.x, G);
  const int tm_cnt = (M + kBM - 1) / kBM, tn_cnt = (N + kBN - 1) / kBN;
  const int ntiles = tm_cnt * tn_cnt;
  const bool n_major = tm_cnt <= tn_cnt;
  const int nk = K / BK;
  if (L >= ntiles) return;
  const int total = ((ntiles - 1 - L) / G + 1) * nk;  // K-steps this workgroup runs

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wm = w >> 2, wn = w & 3;
  const bool g1 = wm == 1;  // wave-uniform
  int roff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
    roff[ks] = (lane & 15) * BK + 8 * ((4 * ks + (lane >> 4)) ^ swz<BK>(lane & 15));

  auto tile_mn = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
    if (n_major) {
      n0 = (t / tm_cnt) * kBN;
      m0 = (t % tm_cnt) * kBM;
    } else {
      m0 = (t / tn_cnt) * kBM;
      n0 = (t % tn_cnt) * kBN;
    }
  };
  auto stage = [&](int buf, int t, int kt) __attribute__((always_inline)) {
    int m0, n0;
    tile_mn(t, m0, n0);
    bf16_t* img = lds + buf * kStage;
    stage_operand<BK>(img, A, lda, m0, M, kt * BK, w, lane);
    stage_operand<BK>(img + kBM * BK, B, ldb, n0, N, kt * BK, w, lane);
  };
  auto barrier = []() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x4_t acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t bf[4], af[8];
  auto read_frags = [&](int buf, int ks) __attribute__((always_inline)) {
    const bf16_t* sA = lds + buf * kStage + (wm * 128) * BK;
    const bf16_t* sB = lds + buf * kStage + kBM * BK + (wn * 64) * BK;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      bf[nb] = *reinterpret_cast<const bf16x8_t*>(sB + nb * 16 * BK + roff[ks]);
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
      af[mb] = *reinterpret_cast<const bf16x8_t*>(sA + mb * 16 * BK + roff[ks]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto mfma_cluster = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < 8; ++mb)
        acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[nb], af[mb], acc[nb][mb], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  int t = L, kt = 0;
  stage(0, t, 0);
  wait_vm<0>();
  barrier();
  if (g1) barrier();
  for (int s = 0; s < total; ++s) {
    const int buf = s & 1;
    int nt = t, nkt = kt + 1;
    if (nkt == nk) {
      nkt = 0;
      nt = t + G;
    }
    if (s + 1 < total) stage(buf ^ 1, nt, nkt);  // buffer of step s-1: every read retired
    read_frags(buf, 0);
    barrier();
    mfma_cluster();
    barrier();
    read_frags(buf, 1);
    if (g1) wait_vm<0>();
    barrier();
    mfma_cluster();
    if (!g1) wait_vm<0>();
    if (kt == nk - 1) {
      int m0, n0;
      tile_mn(t, m0, n0);
      epilogue_tile<EPI>(acc, m0, n0, wm, wn, lane, M, N, C, ldc, bias, aux, ldaux, colpart);
    }
    barrier();
    t = nt;
    kt = nkt;
  }
  if (!g1) barrier();  // group 1 ran one extra barrier at the start
}

template <int EPI>
static void launch_epi(int G, hipStream_t st, const bf16_t* a, long lda, const bf16_t* b,
                       long ldb, bf16_t* c, long ldc, int M, int N, int K, const bf16_t* bi,
                       bf16_t* ax, long ldaux, float* colpart) {
  hipLaunchKernelGGL((gemm_nt_stagger_kernel<EPI>), dim3(G), dim3(kThreads), 0, st, a, lda, b,
                     ldb, c, ldc, M, N, K, bi, ax, ldaux, colpart);
}

int g_num_cus = 0;

}  // namespace

// C = epi(A · B^T). Requirements (checked): K % 64 == 0, N % 4 == 0, 16-byte aligned rows
// (lda, ldb % 8 == 0), ldc / ldaux % 4 == 0. EPI_DGELU: colpart holds ceil(M/128) * N floats;
// with db != nullptr the bias gradient is finished here (colsum over the partial rows into
// db: flags bit0 = bf16 db, bit1 = accumulate), `scratch` = kColsumSplits * N floats.
RA_EXPORT int ra_gemm_nt(const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                         int M, int N, int K, int epi, const void* bias, void* aux, long ldaux,
                         float* colpart, void* db, float* scratch, int db_flags, int grid_cap,
                         hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 4 || lda % 8 || ldb % 8 || ldc % 4)
    return hipErrorInvalidValue;
  if (epi != EPI_NONE && bias == nullptr) return hipErrorInvalidValue;
  if ((epi == EPI_BIAS_GELU || epi == EPI_DGELU) && (aux == nullptr || ldaux % 4))
    return hipErrorInvalidValue;
  if (epi == EPI_DGELU && colpart == nullptr) return hipErrorInvalidValue;
  if (g_num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        g_num_cus <= 0)
      g_num_cus = 256;
  }
  const long ntiles = (long)((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
  int G = grid_cap > 0 ? grid_cap : g_num_cus;
  if (G > ntiles) G = (int)ntiles;
  const auto a = (const bf16_t*)A;
  const auto b = (const bf16_t*)B;
  const auto c = (bf16_t*)C;
  const auto bi = (const bf16_t*)bias;
  const auto ax = (bf16_t*)aux;
  switch (epi) {
    case EPI_NONE:
      launch_epi<EPI_NONE>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux, colpart);
      break;
    case EPI_BIAS:
      launch_epi<EPI_BIAS>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux, colpart);
      break;
    case EPI_BIAS_GELU:
      launch_epi<EPI_BIAS_GELU>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux,
                                colpart);
      break;
    case EPI_DGELU:
      launch_epi<EPI_DGELU>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux,
                            colpart);
      if (db != nullptr) {
        if (scratch == nullptr) return hipErrorInvalidValue;
        colsum_launch(colpart, scratch, db, (M + 127) / 128, N, db_flags, st);
      }
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// floats of workspace EPI_DGELU needs: colpart + colsum scratch
RA_EXPORT long ra_gemm_dgelu_work(int M, int N) {
  return (long)((M + 127) / 128) * N + (long)kColsumSplits * N;
}
