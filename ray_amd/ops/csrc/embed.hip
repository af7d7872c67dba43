// Token + position embedding backward straight into the flat fp32 gradient sinks.
//
//   wte_grad[idx[n], :] += dx[n, :]          n = 0 .. B*T-1   (scatter-add, fp32 atomics)
//   wpe_grad[t, :]      += sum_b dx[b, t, :]                   (column reduction, no atomics)
//
// Replaces torch's `index_add_(0, idx, dx.to(fp32))` (a bf16 -> fp32 copy of dx, then an
// atomic index kernel) and `add_(dx.float().sum(0))` (another fp32 copy and a reduce):
// dx is read twice as bf16 and nothing else is materialised. Both passes run in one launch
// on disjoint workgroup ranges: the first N/4 workgroups scatter one row per wave (lane-
// linear fp32 atomic adds, 256 contiguous bytes per instruction), the rest reduce one
// (position, 8-column) cell per lane over the batch. Reference: the embedding gradient of
// torch.nn.functional.embedding that the reference's GPT-2 benchmark runs through DDP
// (release/air_tests/air_benchmarks/workloads/torch_benchmark.py).
#include "common.h"

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void embed_bwd_kernel(
    const bf16_t* __restrict__ dx, const long* __restrict__ idx, float* __restrict__ wte_g,
    float* __restrict__ wpe_g, int B, int T, int C, int V, int scatter_blocks) {
  const int C8 = C >> 3;
  if ((int)blockIdx.x < scatter_blocks) {
    // one row per wave; lane l adds columns l, l + 64, ...: every atomic instruction of
    // the wave covers 256 contiguous bytes of the sink row (4-byte words, lane-linear),
    // the coalesced shape for L2 atomics (per-lane 8-column runs would scatter each
    // instruction over 2 KB)
    const long n = (long)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (n >= (long)B * T) return;
    const long tok = idx[n];
    if (tok < 0 || tok >= V) return;
    const int lane = threadIdx.x & 63;
    const bf16_t* src = dx + n * C;
    float* g = wte_g + tok * C;
    for (int c = lane; c < C; c += 64) unsafeAtomicAdd(g + c, bf2f(src[c]));
    return;
  }
  const long item = (long)(blockIdx.x - scatter_blocks) * kThreads + threadIdx.x;
  const long t = item / C8;
  if (t >= T) return;
  const int c8 = (int)(item - t * C8);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) {
    float v[8];
    unpack8(reinterpret_cast<const uint4*>(dx + ((long)b * T + t) * C)[c8], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  float4* g = reinterpret_cast<float4*>(wpe_g + t * C + c8 * 8);
  float4 a = g[0], b2 = g[1];
  a.x += acc[0], a.y += acc[1], a.z += acc[2], a.w += acc[3];
  b2.x += acc[4], b2.y += acc[5], b2.z += acc[6], b2.w += acc[7];
  g[0] = a;
  g[1] = b2;
}

}  // namespace

// dx: [B*T, C] bf16 contiguous (C % 8 == 0); idx: [B*T] int64 token ids; wte_g: fp32
// [V, C] sink (accumulated); wpe_g: fp32 [>= T, C] sink (rows 0..T-1 accumulated).
RA_EXPORT int ra_embed_bwd(const void* dx, const long* idx, float* wte_g, float* wpe_g, int B,
                           int T, int C, int V, hipStream_t st) {
  if (B <= 0 || T <= 0 || C <= 0 || C % 8 || V <= 0) return hipErrorInvalidValue;
  const long rows = (long)B * T;
  const long reduce_items = (long)T * (C / 8);
  const int sb = (int)((rows + kThreads / 64 - 1) / (kThreads / 64));
  const int rb = (int)((reduce_items + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(sb + rb), dim3(kThreads), 0, st,
                     (const bf16_t*)dx, idx, wte_g, wpe_g, B, T, C, V, sb);
  return hipGetLastError();
}
