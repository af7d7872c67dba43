// Persistent bf16 MFMA GEMM, four waves per workgroup, 128 x 128 outputs per wave.
//
//   C[M, N] = epi( A[M, K] · B[N, K]^T )      bf16 in, fp32 accumulate, bf16 out
//
// Why this shape (measured against ops/csrc/gemm.hip, whose 8-wave 128 x 64-per-wave
// schedules reach 0.6-0.8x hipBLASLt however they are pipelined): at 1 wave per SIMD a
// wave can hold a 128 x 128 tile — 64 v_mfma_f32_16x16x32_bf16 accumulators = 256
// accumulation registers in the AGPR half of the 512-entry file — so every fragment read
// from LDS feeds 8 MFMAs (0.25 ds_read_b128 per MFMA instead of 0.375-0.44) and there is
// ONE barrier per 64 MFMAs per wave.
//
//  * tile 256 x 256, BK = 32, 4 LDS stages of 32 KB (A [256][32], B [256][32]) + a 32 KB
//    epilogue region = 160 KB, one workgroup per CU;
//  * staging: 16-byte global_load_lds, lane-linear images with the bank swizzle on the
//    SOURCE address (rule 21). 64-B rows: 16-B chunk c of row r sits at c ^ f(r>>2 & 3),
//    f = {0,3,2,1}, which makes every ds_read_b128 lane group ({0-3,12-15,20-27}, ...)
//    hit 16 distinct 16-B slots of the 256-B bank row;
//  * software pipeline: at the top of K-tile k every wave retires the DMAs of K-tile k+1
//    (counted vmcnt, never 0 in the steady state), barriers, restages the buffer of
//    K-tile k (its fragments are already in registers) with K-tile k+4, then issues the
//    16 fragment reads of K-tile k+1 under the 64 MFMAs of K-tile k — 3 K-tiles of DMA
//    latency in flight, the LDS read latency hidden behind the MFMA stream;
//  * persistent over tiles with one continuous K-tile pipeline; XCD-aware block order;
//  * epilogue through LDS (guide T21: widen the stores): each wave converts its
//    accumulators to bf16 into a private 8 KB region (8-byte granules XOR-swizzled by row:
//    conflict-free ds_write_b64), reads them back row-contiguous and stores full 256-B
//    row segments with global_store_dwordx4; the elementwise epilogues (bias, bias+GELU
//    with the pre-activation saved, GELU-backward with the bias-gradient column partials)
//    run on those row-contiguous values with coalesced 16-B bias / aux accesses.
//
// MFMA orientation D = B_frag · A_frag^T: lane l holds output row m = 16 mb + (l & 15) and
// columns n = 16 nb + 4 (l >> 4) + 0..3 of each 16 x 16 block.
#include "common.h"

#include <type_traits>

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

constexpr int kBM = 256, kBN = 256, kBK = 32, kNS = 4, kThreads = 256;
constexpr int kStageElems = (kBM + kBN) * kBK;                // 16384 bf16 = 32 KB
constexpr int kEpiElemsPerWave = 32 * 128;                    // 32 rows x 128 cols bf16
constexpr int kLdsElems = kNS * kStageElems + 4 * kEpiElemsPerWave;  // 160 KB

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

// physical 16-B chunk of logical chunk c (0..3) in 64-B row r
__device__ __forceinline__ int chunk_swz(int r, int c) {
  const int g = (r >> 2) & 3;
  return c ^ ((4 - g) & 3);
}

__device__ __forceinline__ int xcd_remap(int b, int G) {
  const int q = G / 8, rr = G % 8, x = b % 8;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + b / 8;
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in {0, 8, ..., 56}; the hardware
// counter holds up to 63
__device__ __forceinline__ void wait_vm_dyn(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 40: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 48: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
  }
}

// 16-byte global -> LDS DMA (global_load_lds_dwordx4; LDS address = M0 + lane * 16) as
// inline asm. Issued through the builtin, hipcc sees an LDS write it cannot disambiguate
// from the fragment reads of the OTHER stage buffers and drains every DMA in flight with
// s_waitcnt vmcnt(0) in front of them — the whole prefetch pipeline. Written as asm the
// DMA is ordered only by the explicit counted vmcnt + barrier protocol of the K loop
// (the hardware still counts it in vmcnt). M0 is saved and restored around it.
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

// epilogue LDS image of one wave: [32 rows][32 granules of 8 B]; granule g of row r is
// stored at g ^ (r & 15) (conflict-free ds_write_b64 from the accumulator layout)
__device__ __forceinline__ int epi_off(int r, int g) { return r * 128 + ((g ^ (r & 15)) << 2); }

template <int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm4w_nt_kernel(
    const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ B, long ldb,
    bf16_t* __restrict__ C, long ldc, int M, int N, int K, const bf16_t* __restrict__ bias,
    bf16_t* __restrict__ aux, long ldaux, float* __restrict__ colpart) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[kLdsElems];
  const int G = gridDim.x;
  const int L = xcd_remap(blockIdx.x, G);
  const int tm_cnt = (M + kBM - 1) / kBM, tn_cnt = (N + kBN - 1) / kBN;
  const int ntiles = tm_cnt * tn_cnt;
  const bool n_major = tm_cnt <= tn_cnt;
  const int nk = K / kBK;
  if (L >= ntiles) return;
  const int total = ((ntiles - 1 - L) / G + 1) * nk;  // K-tiles this workgroup runs

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wr = w >> 1, wc = w & 1;
  // fragment read offset inside a 16-row block: row lane & 15, logical chunk lane >> 4
  const int roff = (lane & 15) * kBK + 8 * chunk_swz(lane & 15, lane >> 4);

  auto tile_mn = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
    if (n_major) {
      n0 = (t / tm_cnt) * kBN;
      m0 = (t % tm_cnt) * kBM;
    } else {
      m0 = (t / tn_cnt) * kBM;
      n0 = (t % tn_cnt) * kBN;
    }
  };
  // K-tile g -> stage buffer g % 4: 8 DMA instructions per thread (A: 4, B: 4); wave w,
  // instruction j moves rows 64 w + 16 j .. +15 (1 KB)
  auto stage = [&](int g) __attribute__((always_inline)) {
    const int t = L + (g / nk) * G, kt = g % nk;
    int m0, n0;
    tile_mn(t, m0, n0);
    bf16_t* img = lds + (g % kNS) * kStageElems;
    const int rsub = lane >> 2, p = lane & 3;
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      const bf16_t* src = op ? B : A;
      const long ld = op ? ldb : lda;
      const int row0 = op ? n0 : m0;
      const int rows = op ? N : M;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r0 = 64 * w + 16 * j;
        const int r = r0 + rsub;
        int gr = row0 + r;
        gr = gr < rows ? gr : rows - 1;  // ragged edge: clamp (masked at the store)
        const bf16_t* s = src + (long)gr * ld + kt * kBK + 8 * chunk_swz(r, p);
        glds16(s, img + op * kBM * kBK + r0 * kBK);
      }
    }
  };

  f32x4_t acc[8][8];  // written by the first K-tile of every tile (C operand 0)
  // ONE fragment set (64 VGPRs). The 64 MFMAs of a K-tile run as four quadrants of
  // (4 A-blocks x 4 B-blocks); a fragment is re-read for the NEXT K-tile as soon as its
  // last quadrant has issued, and the quadrant order alternates between even and odd
  // K-tiles so that each K-tile starts on fragments that were read one or two quadrants
  // earlier:
  //   even: (A0,B0) (A0,B1) | A0' (A1,B1) | B1' (A1,B0) | A1' B0'
  //   odd:  (A0,B1) (A0,B0) | A0' (A1,B0) | B0' (A1,B1) | A1' B1'
  // (Ah = A-blocks 4h..4h+3, Bh likewise; X' = the next K-tile's fragments of X).
  bf16x8_t fa[8], fb[8];
  auto read_a = [&](int g, int h) __attribute__((always_inline)) {
    const bf16_t* sa = lds + (g % kNS) * kStageElems + (wr * 128) * kBK + roff;
#pragma unroll
    for (int i = 4 * h; i < 4 * h + 4; ++i)
      fa[i] = *reinterpret_cast<const bf16x8_t*>(sa + i * 16 * kBK);
  };
  auto read_b = [&](int g, int h) __attribute__((always_inline)) {
    const bf16_t* sb = lds + (g % kNS) * kStageElems + kBM * kBK + (wc * 128) * kBK + roff;
#pragma unroll
    for (int i = 4 * h; i < 4 * h + 4; ++i)
      fb[i] = *reinterpret_cast<const bf16x8_t*>(sb + i * 16 * kBK);
  };
  auto quad = [&](int ha, int hb, auto first_c) __attribute__((always_inline)) {
    constexpr bool first = decltype(first_c)::value;
#pragma unroll
    for (int nb = 4 * hb; nb < 4 * hb + 4; ++nb)
#pragma unroll
      for (int mb = 4 * ha; mb < 4 * ha + 4; ++mb)
        acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            fb[nb], fa[mb], first ? f32x4_t{0.f, 0.f, 0.f, 0.f} : acc[nb][mb], 0, 0, 0);
  };

  // ---- epilogue of the tile whose accumulators are complete (see header). Every global
  // access is a buffer instruction whose out-of-range lanes are dropped by the hardware
  // (offset past num_records), so each wave issues the same number of VMEM instructions
  // on every tile, ragged or not — the counted vmcnt targets above rely on it.
  bf16_t* epi = lds + kNS * kStageElems + w * kEpiElemsPerWave;
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    int m0, n0;
    tile_mn(t, m0, n0);
    const int mw = m0 + wr * 128, nw = n0 + wc * 128;
    const int rows_ok = mw < M ? (M - mw < 128 ? M - mw : 128) : 0;
    // row-contiguous view: lane handles column chunk cc = lane & 15 (8 columns) of rows
    // (lane >> 4) + 4 i of each 32-row round
    const int cc = lane & 15, rq = lane >> 4;
    const int ncol = nw + 8 * cc;
    const bool nok = ncol < N;  // N % 8 == 0: a lane's 8 columns are all valid or none
    const int kOOB = 0x7ffffff0;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(C + (long)(rows_ok ? mw : 0) * ldc), 0, rows_ok * (int)ldc * 2, 0x00020000);
    __amdgpu_buffer_rsrc_t rx = rc;
    if (EPI == EPI_BIAS_GELU || EPI == EPI_DGELU)
      rx = __builtin_amdgcn_make_buffer_rsrc((void*)(aux + (long)(rows_ok ? mw : 0) * ldaux), 0,
                                             rows_ok * (int)ldaux * 2, 0x00020000);
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (EPI != EPI_NONE) {
      const __amdgpu_buffer_rsrc_t rb =
          __builtin_amdgcn_make_buffer_rsrc((void*)bias, 0, N * 2, 0x00020000);
      const auto u = __builtin_amdgcn_raw_buffer_load_b128(rb, nok ? ncol * 2 : kOOB, 0, 0);
      unpack8(make_uint4(u[0], u[1], u[2], u[3]), bv);
    }
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rnd = 0; rnd < 4; ++rnd) {
      // accumulators of m-blocks 2 rnd, 2 rnd + 1 -> LDS (bf16, 4 columns per 8-B granule)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) {
          const f32x4_t v = acc[nb][2 * rnd + h];
          float f[4] = {v[0], v[1], v[2], v[3]};
          const int r = 16 * h + (lane & 15);
          const int gr = 4 * nb + (lane >> 4);
          *reinterpret_cast<uint2*>(epi + epi_off(r, gr)) = pack4(f);
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = rq + 4 * i;
        const uint2 lo = *reinterpret_cast<const uint2*>(epi + epi_off(r, 2 * cc));
        const uint2 hi = *reinterpret_cast<const uint2*>(epi + epi_off(r, 2 * cc + 1));
        const int mr = 32 * rnd + r;  // row within the wave's 128-row block
        const bool ok = nok && mr < rows_ok;
        uint4 u = make_uint4(lo.x, lo.y, hi.x, hi.y);
        if (EPI != EPI_NONE) {
          float v[8];
          unpack8(u, v);
          if (EPI == EPI_BIAS) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bv[e];
          } else if (EPI == EPI_BIAS_GELU) {  // save the pre-activation for backward
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, u), rx,
                ok ? (mr * (int)ldaux + ncol) * 2 : kOOB, 0, 0);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = gelu_fwd(v[e] + bv[e]);
          } else {  // EPI_DGELU
            const auto a = __builtin_amdgcn_raw_buffer_load_b128(
                rx, ok ? (mr * (int)ldaux + ncol) * 2 : kOOB, 0, 0);
            float pre[8];
            unpack8(make_uint4(a[0], a[1], a[2], a[3]), pre);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              v[e] *= gelu_grad(pre[e] + bv[e]);
              csum[e] += ok ? v[e] : 0.f;
            }
          }
          u = pack8(v);
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, u), rc,
            ok ? (mr * (int)ldc + ncol) * 2 : kOOB, 0, 0);
      }
      // the next round rewrites the region: this round's reads must have landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (EPI == EPI_DGELU) {
      // lanes cc, cc+16, cc+32, cc+48 hold the same 8 columns (different rows)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s = csum[e];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        csum[e] = s;
      }
      // colpart row mw / 128 (this wave's 128-row block); lanes 0-15 write
      const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(colpart + (long)(rows_ok ? mw / 128 : 0) * N), 0, rows_ok ? N * 4 : 0,
          0x00020000);
      const int off = (rq == 0 && nok) ? ncol * 4 : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                             make_float4(csum[0], csum[1], csum[2], csum[3])), rp, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                             make_float4(csum[4], csum[5], csum[6], csum[7])), rp,
          off == kOOB ? kOOB : off + 16, 0, 0);
    }
  };
  // VMEM instructions one epilogue issues per wave (uniform, see above)
  constexpr int kEpiOps = EPI == EPI_NONE ? 32 : EPI == EPI_BIAS ? 33 : EPI == EPI_BIAS_GELU ? 65 : 67;

  // ---- prologue: up to 4 K-tiles in flight, K-tile 0 landed, its fragments read
  const int npro = total < kNS ? total : kNS;
  for (int g = 0; g < npro; ++g) stage(g);
  wait_vm_dyn(8 * (npro - 1));
  __builtin_amdgcn_s_barrier();
  read_a(0, 0);
  read_a(0, 1);
  read_b(0, 0);
  read_b(0, 1);

  // Tile loop with a nested K loop (the accumulators stay in the same AGPRs: no copies at
  // a back edge); the DMA pipeline runs on the global K-tile index g across tiles. The
  // last epilogue's VMEM operations are counted in the vmcnt targets of the next K-tiles.
  bool epi_recent = false;  // an epilogue was issued within the last 3 K-tiles
  // K-tile g (odd = g & 1 picks the quadrant order); the next K-tile's reads go to
  // buffer (g+1) % 4, which the wait + barrier at the top made visible
  auto kbody = [&](int g, int odd, int kt, auto first_c) __attribute__((always_inline)) {
    // retire K-tile g+1's DMAs: everything issued after them may stay in flight
    if (g + 1 < total) {
      if (__builtin_expect(g + 3 < total && !(epi_recent && kt < 3), 1)) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else {
        int younger = 8 * ((g + 2 < total) + (g + 3 < total));
        if (epi_recent && kt < 3) younger += kEpiOps;
        // any count <= the true number of younger operations is correct (it only waits
        // longer); wait_vm_dyn takes multiples of 8 up to 56
        wait_vm_dyn(younger > 56 ? 56 : younger & ~7);
      }
    }
    // every wave's reads of K-tile g (buffer g % 4) have landed: restage it after the
    // barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (g + kNS < total) stage(g + kNS);
    const bool nxt = g + 1 < total;
    const int b0 = odd, b1 = odd ^ 1;  // B halves in this K-tile's order
    quad(0, b0, first_c);
    quad(0, b1, first_c);
    if (nxt) read_a(g + 1, 0);
    quad(1, b1, first_c);
    if (nxt) read_b(g + 1, b1);
    quad(1, b0, first_c);
    if (nxt) {
      read_a(g + 1, 1);
      read_b(g + 1, b0);
    }
  };
  const int ntl = total / nk;
  int g = 0;
  for (int tl = 0; tl < ntl; ++tl) {
    kbody(g, 0, 0, std::true_type{});
    kbody(g + 1, 1, 1, std::false_type{});
    g += 2;
    for (int kt = 2; kt < nk; kt += 2, g += 2) {
      kbody(g, 0, kt, std::false_type{});
      kbody(g + 1, 1, kt + 1, std::false_type{});
    }
    epilogue(L + tl * G);
    epi_recent = true;
  }
}

int g_num_cus = 0;

template <int EPI>
void launch(int G, hipStream_t st, const bf16_t* a, long lda, const bf16_t* b, long ldb,
            bf16_t* c, long ldc, int M, int N, int K, const bf16_t* bi, bf16_t* ax, long ldaux,
            float* colpart) {
  hipLaunchKernelGGL((gemm4w_nt_kernel<EPI>), dim3(G), dim3(kThreads), 0, st, a, lda, b, ldb, c,
                     ldc, M, N, K, bi, ax, ldaux, colpart);
}

}  // namespace

// C = epi(A · B^T) on the 4-wave kernel. Requirements (checked): K % 64 == 0, K >= 128,
// N % 8 == 0, lda / ldb / ldc / ldaux % 8 == 0 (16-byte rows). EPI_DGELU: colpart holds
// ceil(M / 128) * N floats; with db != nullptr the bias gradient is finished into db
// (flags bit0 = bf16 db, bit1 = accumulate), scratch = kColsumSplits * N floats.
RA_EXPORT int ra_gemm4w_nt(const void* A, long lda, const void* B, long ldb, void* C, long ldc,
                           int M, int N, int K, int epi, const void* bias, void* aux, long ldaux,
                           float* colpart, void* db, float* scratch, int db_flags, int grid_cap,
                           hipStream_t st) {
  if (M <= 0 || N <= 0 || K < 128 || K % (2 * kBK) || N % 8 || lda % 8 || ldb % 8 || ldc % 8)
    return hipErrorInvalidValue;
  if (epi != EPI_NONE && bias == nullptr) return hipErrorInvalidValue;
  if ((epi == EPI_BIAS_GELU || epi == EPI_DGELU) && (aux == nullptr || ldaux % 8))
    return hipErrorInvalidValue;
  if (epi == EPI_DGELU && colpart == nullptr) return hipErrorInvalidValue;
  if (g_num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess ||
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
    case EPI_NONE: launch<EPI_NONE>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux, colpart); break;
    case EPI_BIAS: launch<EPI_BIAS>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux, colpart); break;
    case EPI_BIAS_GELU:
      launch<EPI_BIAS_GELU>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux, colpart);
      break;
    case EPI_DGELU:
      launch<EPI_DGELU>(G, st, a, lda, b, ldb, c, ldc, M, N, K, bi, ax, ldaux, colpart);
      if (db != nullptr) {
        if (scratch == nullptr) return hipErrorInvalidValue;
        colsum_launch(colpart, scratch, db, (M + 127) / 128, N, db_flags, st);
      }
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
