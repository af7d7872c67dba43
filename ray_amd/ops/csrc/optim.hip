// Flat-buffer optimizer kernels (one launch for the whole model).
//
// The trainer keeps every parameter as a view into ONE bf16 buffer (compute
// copy) backed by ONE fp32 master buffer, and every gradient as a view into
// ONE grad buffer — fp32 by default (the reference's DDP precision), bf16 when
// gradient compression is requested — which is also what RCCL all-reduces,
// bucket by bucket, with no packing copy. So the optimizer step is a single
// streaming pass (fp32 grads, zeroed in the same pass):
//   read g p m v -> write p m v p16 g(=0) = 38 B/param.
// Decayed parameters occupy [0, n_decay), the rest is not decayed.
// Global-norm clipping stays on device: ra_sumsq_bf16 -> ra_clip_scale writes
// the scale factor that ra_adamw_flat reads through a pointer (no host sync).
#include "common.h"

__global__ __launch_bounds__(256) void sumsq_kernel(const bf16_t* __restrict__ g, long n4,
                                                    float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float v[4];
    unpack4(reinterpret_cast<const uint2*>(g)[i], v);
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void clip_scale_kernel(const float* __restrict__ part, int P, float max_norm,
                                  float pre_scale, float* __restrict__ scale_out,
                                  float* __restrict__ norm_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < P; i += blockDim.x) s += part[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s) * pre_scale;
    if (norm_out) *norm_out = norm;
    float sc = pre_scale;
    if (max_norm > 0.f && norm > max_norm) sc *= max_norm / (norm + 1e-6f);
    *scale_out = sc;
  }
}

// G = bf16_t (compressed gradient buffer) or float (default fp32 gradient buffer).
// ZERO: also clear the gradient after reading it — the optimizer is the last reader of
// the flat grad every step, so this replaces the separate zero_grad memset pass.
template <typename G, bool ZERO>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p32,
                                                    bf16_t* __restrict__ p16,
                                                    G* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    long n4, long nd4, float lr, float b1,
                                                    float b2, float eps, float wd, float rbc1,
                                                    float rbc2, const float* __restrict__ gscale,
                                                    const float* __restrict__ hyper) {
  const float sc = gscale ? *gscale : 1.f;
  if (hyper) {  // graph-replayed step: {lr, 1/(1-b1^t), 1/(1-b2^t)} from device memory
    lr = hyper[0];
    rbc1 = hyper[1];
    rbc2 = hyper[2];
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float gv[4];
    if constexpr (sizeof(G) == 2) {
      unpack4(reinterpret_cast<const uint2*>(g)[i], gv);
      if (ZERO) reinterpret_cast<uint2*>(g)[i] = make_uint2(0u, 0u);
    } else {
      const float4 g4 = reinterpret_cast<const float4*>(g)[i];
      gv[0] = g4.x; gv[1] = g4.y; gv[2] = g4.z; gv[3] = g4.w;
      if (ZERO) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 p = reinterpret_cast<float4*>(p32)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    const float decay = (i < nd4) ? (1.f - lr * wd) : 1.f;
    float pa[4] = {p.x, p.y, p.z, p.w};
    float ma[4] = {mm.x, mm.y, mm.z, mm.w};
    float va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gr = gv[j] * sc;
      ma[j] = b1 * ma[j] + (1.f - b1) * gr;
      va[j] = b2 * va[j] + (1.f - b2) * gr * gr;
      const float upd = (ma[j] * rbc1) / (sqrtf(va[j] * rbc2) + eps);
      pa[j] = pa[j] * decay - lr * upd;
    }
    reinterpret_cast<float4*>(p32)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    reinterpret_cast<float4*>(m)[i] = make_float4(ma[0], ma[1], ma[2], ma[3]);
    reinterpret_cast<float4*>(v)[i] = make_float4(va[0], va[1], va[2], va[3]);
    if (p16) reinterpret_cast<uint2*>(p16)[i] = pack4(pa);
  }
}

// Plain SGD/momentum on the same flat layout (used by RL learners).
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p32, bf16_t* __restrict__ p16,
                                                  const bf16_t* __restrict__ g,
                                                  float* __restrict__ buf, long n4, float lr,
                                                  float mom, float wd,
                                                  const float* __restrict__ gscale) {
  const float sc = gscale ? *gscale : 1.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float gv[4];
    unpack4(reinterpret_cast<const uint2*>(g)[i], gv);
    float4 p = reinterpret_cast<float4*>(p32)[i];
    float4 b = reinterpret_cast<float4*>(buf)[i];
    float pa[4] = {p.x, p.y, p.z, p.w}, ba[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gr = gv[j] * sc + wd * pa[j];
      ba[j] = mom * ba[j] + gr;
      pa[j] -= lr * ba[j];
    }
    reinterpret_cast<float4*>(p32)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    reinterpret_cast<float4*>(buf)[i] = make_float4(ba[0], ba[1], ba[2], ba[3]);
    if (p16) reinterpret_cast<uint2*>(p16)[i] = pack4(pa);
  }
}

// fp32-grad variant of AdamW (for fp32 learners, e.g. RLlib policies).
__global__ __launch_bounds__(256) void adamw_f32_kernel(float* __restrict__ p,
                                                        const float* __restrict__ g,
                                                        float* __restrict__ m,
                                                        float* __restrict__ v, long n, long nd,
                                                        float lr, float b1, float b2, float eps,
                                                        float wd, float rbc1, float rbc2,
                                                        const float* __restrict__ gscale) {
  const float sc = gscale ? *gscale : 1.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float gr = g[i] * sc;
    const float mm = b1 * m[i] + (1.f - b1) * gr;
    const float vv = b2 * v[i] + (1.f - b2) * gr * gr;
    m[i] = mm;
    v[i] = vv;
    const float decay = (i < nd) ? (1.f - lr * wd) : 1.f;
    p[i] = p[i] * decay - lr * (mm * rbc1) / (sqrtf(vv * rbc2) + eps);
  }
}

__global__ __launch_bounds__(256) void sumsq_f32_kernel(const float* __restrict__ g, long n,
                                                        float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride)
    s += g[i] * g[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

static const int kNormParts = 1024;

RA_EXPORT int ra_norm_parts() { return kNormParts; }

// work: kNormParts floats. scale_out/norm_out: device floats.
RA_EXPORT int ra_grad_clip(const void* g, long n, int is_bf16, float max_norm, float pre_scale,
                           float* work, float* scale_out, float* norm_out, hipStream_t st) {
  if (is_bf16) {
    if (n % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sumsq_kernel, dim3(kNormParts), dim3(256), 0, st, (const bf16_t*)g, n / 4,
                       work);
  } else {
    hipLaunchKernelGGL(sumsq_f32_kernel, dim3(kNormParts), dim3(256), 0, st, (const float*)g, n,
                       work);
  }
  hipLaunchKernelGGL(clip_scale_kernel, dim3(1), dim3(256), 0, st, work, kNormParts, max_norm,
                     pre_scale, scale_out, norm_out);
  return hipGetLastError();
}

// flags: bit0 g is fp32 (else bf16), bit1 zero g after use. p16 may be null.
// hyper (nullable): device {lr, 1/(1-b1^t), 1/(1-b2^t)} read by the kernel instead of the
// lr / step arguments — a captured (HIP-graph) optimizer step whose schedule advances
// between replays without re-capture
RA_EXPORT int ra_adamw_flat_dev(float* p32, void* p16, void* g, float* m, float* v, long n,
                                long n_decay, float lr, float b1, float b2, float eps, float wd,
                                int step, const float* gscale, int flags, const float* hyper,
                                hipStream_t st);

RA_EXPORT int ra_adamw_flat(float* p32, void* p16, void* g, float* m, float* v, long n,
                            long n_decay, float lr, float b1, float b2, float eps, float wd,
                            int step, const float* gscale, int flags, hipStream_t st) {
  return ra_adamw_flat_dev(p32, p16, g, m, v, n, n_decay, lr, b1, b2, eps, wd, step, gscale,
                           flags, nullptr, st);
}

RA_EXPORT int ra_adamw_flat_dev(float* p32, void* p16, void* g, float* m, float* v, long n,
                                long n_decay, float lr, float b1, float b2, float eps, float wd,
                                int step, const float* gscale, int flags, const float* hyper,
                                hipStream_t st) {
  if (n % 4 || n_decay % 4) return hipErrorInvalidValue;
  const float rbc1 = 1.f / (1.f - powf(b1, (float)step));
  const float rbc2 = 1.f / (1.f - powf(b2, (float)step));
  const dim3 grid(ra_grid(n / 4, 256)), blk(256);
#define A(G, Z)                                                                              \
  hipLaunchKernelGGL((adamw_kernel<G, Z>), grid, blk, 0, st, p32, (bf16_t*)p16, (G*)g, m, v, \
                     n / 4, n_decay / 4, lr, b1, b2, eps, wd, rbc1, rbc2, gscale, hyper)
  switch (flags & 3) {
    case 0: A(bf16_t, false); break;
    case 1: A(float, false); break;
    case 2: A(bf16_t, true); break;
    default: A(float, true);
  }
#undef A
  return hipGetLastError();
}

RA_EXPORT int ra_adamw_f32(float* p, const float* g, float* m, float* v, long n, long n_decay,
                           float lr, float b1, float b2, float eps, float wd, int step,
                           const float* gscale, hipStream_t st) {
  const float rbc1 = 1.f / (1.f - powf(b1, (float)step));
  const float rbc2 = 1.f / (1.f - powf(b2, (float)step));
  hipLaunchKernelGGL(adamw_f32_kernel, dim3(ra_grid(n, 256)), dim3(256), 0, st, p, g, m, v, n,
                     n_decay, lr, b1, b2, eps, wd, rbc1, rbc2, gscale);
  return hipGetLastError();
}

RA_EXPORT int ra_sgd_flat(float* p32, void* p16, const void* g, float* buf, long n, float lr,
                          float mom, float wd, const float* gscale, hipStream_t st) {
  if (n % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sgd_kernel, dim3(ra_grid(n / 4, 256)), dim3(256), 0, st, p32, (bf16_t*)p16,
                     (const bf16_t*)g, buf, n / 4, lr, mom, wd, gscale);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// AdamW that also refreshes the transposed bf16 copy W^T of every nn.Linear weight
// (the dX = dY . W input-gradient GEMM reads W^T so that it runs in the forward GEMMs'
// operand layout: ops/functional.py _transposed_weight). The flat layout puts those
// weights first, [0, n_wt) (FlatParams(transpose=...)); each is processed as 64 x 64
// tiles: the tile's p/m/v/g are read and written row-major (coalesced, as the 1-D pass),
// its bf16 values go through an LDS tile and are stored transposed — also coalesced — into
// pt16, which mirrors [0, n_wt) with W^T [C][R] at the weight's own offset. The rest of
// the buffer, [n_wt, n), is the ordinary 1-D grid-stride pass. One launch, one HBM pass:
// the per-weight transpose kernels that used to run beside the forward GEMMs are gone.
struct WtSeg {
  long off;   // flat offset (elements) of W [R][C] (= offset of W^T in pt16)
  int R, C;   // C % 4 == 0
  int tile0;  // first tile index of this segment
  int tc;     // tiles along C
};
constexpr int kWtMaxSeg = 256;
struct WtTable {
  int nseg;
  WtSeg seg[kWtMaxSeg];
};

__device__ __forceinline__ void adam_elem4(float (&pa)[4], float (&ma)[4], float (&va)[4],
                                           const float (&gv)[4], float sc, float b1, float b2,
                                           float eps, float lr, float rbc1, float rbc2,
                                           float decay) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float gr = gv[j] * sc;
    ma[j] = b1 * ma[j] + (1.f - b1) * gr;
    va[j] = b2 * va[j] + (1.f - b2) * gr * gr;
    const float upd = (ma[j] * rbc1) / (sqrtf(va[j] * rbc2) + eps);
    pa[j] = pa[j] * decay - lr * upd;
  }
}

template <typename G, bool ZERO>
__global__ __launch_bounds__(256) void adamw_wt_kernel(
    float* __restrict__ p32, bf16_t* __restrict__ p16, bf16_t* __restrict__ pt16,
    G* __restrict__ g, float* __restrict__ m, float* __restrict__ v, long n4, long nd,
    long nwt4, int ntiles, float lr, float b1, float b2, float eps, float wd, float rbc1,
    float rbc2, const float* __restrict__ gscale, const float* __restrict__ hyper,
    const WtTable* __restrict__ tab) {
  const float sc = gscale ? *gscale : 1.f;
  if (hyper) {
    lr = hyper[0];
    rbc1 = hyper[1];
    rbc2 = hyper[2];
  }
  auto load_g = [&](long i, float (&gv)[4]) __attribute__((always_inline)) {
    if constexpr (sizeof(G) == 2) {
      unpack4(reinterpret_cast<const uint2*>(g)[i], gv);
      if (ZERO) reinterpret_cast<uint2*>(g)[i] = make_uint2(0u, 0u);
    } else {
      const float4 g4 = reinterpret_cast<const float4*>(g)[i];
      gv[0] = g4.x, gv[1] = g4.y, gv[2] = g4.z, gv[3] = g4.w;
      if (ZERO) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto update4 = [&](long i, float (&pa)[4]) __attribute__((always_inline)) {
    float gv[4];
    load_g(i, gv);
    const float4 p = reinterpret_cast<float4*>(p32)[i];
    const float4 mm = reinterpret_cast<float4*>(m)[i];
    const float4 vv = reinterpret_cast<float4*>(v)[i];
    pa[0] = p.x, pa[1] = p.y, pa[2] = p.z, pa[3] = p.w;
    float ma[4] = {mm.x, mm.y, mm.z, mm.w}, va[4] = {vv.x, vv.y, vv.z, vv.w};
    adam_elem4(pa, ma, va, gv, sc, b1, b2, eps, lr, rbc1, rbc2,
               (4 * i < nd) ? (1.f - lr * wd) : 1.f);
    reinterpret_cast<float4*>(p32)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    reinterpret_cast<float4*>(m)[i] = make_float4(ma[0], ma[1], ma[2], ma[3]);
    reinterpret_cast<float4*>(v)[i] = make_float4(va[0], va[1], va[2], va[3]);
    reinterpret_cast<uint2*>(p16)[i] = pack4(pa);
  };

  if ((int)blockIdx.x < ntiles) {
    // ---- one 64 x 64 tile of a transposed weight
    __shared__ __attribute__((aligned(16))) bf16_t tl[64 * 72];  // [col][row], 144-B rows
    const int b = blockIdx.x;
    int s = 0;
    while (s + 1 < tab->nseg && tab->seg[s + 1].tile0 <= b) ++s;
    const WtSeg sg = tab->seg[s];
    const int t = b - sg.tile0;
    const int r0 = (t / sg.tc) * 64, c0 = (t % sg.tc) * 64;
    const int lr_ = threadIdx.x >> 4, lc = (threadIdx.x & 15) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + lr_ + 16 * i, c = c0 + lc;
      float pa[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < sg.R && c < sg.C) update4((sg.off + (long)r * sg.C + c) >> 2, pa);
#pragma unroll
      for (int j = 0; j < 4; ++j) tl[(lc + j) * 72 + lr_ + 16 * i] = f2bf(pa[j]);
    }
    __syncthreads();
    // W^T rows c0 + cc, 16 rows of W (32 B) per thread
    const int cc = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 16;
    const int c = c0 + cc;
    if (c < sg.C) {
      const uint4 a0 = *reinterpret_cast<const uint4*>(tl + cc * 72 + rr);
      const uint4 a1 = *reinterpret_cast<const uint4*>(tl + cc * 72 + rr + 8);
      bf16_t* dst = pt16 + sg.off + (long)c * sg.R + r0 + rr;
      if (r0 + rr + 16 <= sg.R && (sg.R % 8) == 0) {
        reinterpret_cast<uint4*>(dst)[0] = a0;
        reinterpret_cast<uint4*>(dst)[1] = a1;
      } else {
        const bf16_t* src = tl + cc * 72 + rr;
        for (int k = 0; k < 16 && r0 + rr + k < sg.R; ++k) dst[k] = src[k];
      }
    }
    return;
  }
  // ---- 1-D grid-stride over [n_wt, n)
  const long stride = (long)(gridDim.x - ntiles) * blockDim.x;
  for (long i = nwt4 + (long)(blockIdx.x - ntiles) * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    float pa[4];
    update4(i, pa);
  }
}

// AdamW over the flat buffer + W^T refresh of the table's weights (device table built by
// FlatParams: WtTable bytes). n_wt: elements at the start of the buffer covered by the
// table (every segment lies inside [0, n_wt), which must lie inside the decay group or
// straddle nothing: decay is decided per element against n_decay). flags as
// ra_adamw_flat_dev.
RA_EXPORT int ra_adamw_flat_wt(float* p32, void* p16, void* pt16, void* g, float* m, float* v,
                               long n, long n_decay, long n_wt, const void* table, int ntiles,
                               float lr, float b1, float b2, float eps, float wd, int step,
                               const float* gscale, int flags, const float* hyper,
                               hipStream_t st) {
  if (n % 4 || n_decay % 4 || n_wt % 4 || !p16 || !pt16 || !table || ntiles < 0)
    return hipErrorInvalidValue;
  const float rbc1 = 1.f / (1.f - powf(b1, (float)step));
  const float rbc2 = 1.f / (1.f - powf(b2, (float)step));
  const int g1 = ra_grid((n - n_wt) / 4, 256);
  const dim3 grid(ntiles + g1), blk(256);
#define A(G, Z)                                                                             \
  hipLaunchKernelGGL((adamw_wt_kernel<G, Z>), grid, blk, 0, st, p32, (bf16_t*)p16,          \
                     (bf16_t*)pt16, (G*)g, m, v, n / 4, n_decay, n_wt / 4, ntiles, lr, b1,  \
                     b2, eps, wd, rbc1, rbc2, gscale, hyper, (const WtTable*)table)
  switch (flags & 3) {
    case 0: A(bf16_t, false); break;
    case 1: A(float, false); break;
    case 2: A(bf16_t, true); break;
    default: A(float, true);
  }
#undef A
  return hipGetLastError();
}

RA_EXPORT int ra_wt_table_bytes() { return (int)sizeof(WtTable); }
RA_EXPORT int ra_wt_max_segments() { return kWtMaxSeg; }
