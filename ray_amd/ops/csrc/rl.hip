// RLlib learner hot-loop kernels: GAE, V-trace, fused PPO loss (fwd+bwd),
// running observation normalisation.
//
// Reference semantics:
//   GAE      rllib/evaluation/postprocessing.py:compute_advantages (discount_cumsum of
//            delta_t = r_t + gamma*V_{t+1}*(1-d_t) - V_t with factor gamma*lambda)
//   V-trace  rllib/algorithms/impala/vtrace_torch.py:from_importance_weights
//   PPO loss rllib/algorithms/ppo/torch/ppo_torch_learner.py:compute_loss_for_module
//   obs norm rllib/utils/filter.py:MeanStdFilter (Welford / Chan merge)
//
// Layout: rollouts are [T, B] (time-major, env-minor) as produced by vectorised
// env runners. Both GAE and V-trace are reverse affine recurrences
//     x_t = b_t + a_t * x_{t+1}
// which we solve with a wave64 chunked scan: lane l owns T/64 consecutive steps,
// composes its affine map, the 64 maps are combined with 6 __shfl_down steps,
// and each lane replays its chunk from the correct carry-in. One wave per env
// column; when B is large a serial thread-per-column kernel is used instead
// (already coalesced, no scan needed).
#include "common.h"

enum { MODE_GAE = 0, MODE_VTRACE = 1 };

struct ScanArgs {
  const float* rewards;    // [T,B]
  const float* values;     // [T,B]
  const float* dones;      // [T,B]  (GAE: terminal flag; VTRACE: unused)
  const float* discounts;  // [T,B]  (VTRACE: gamma*(1-done); GAE: unused)
  const float* log_rhos;   // [T,B]  (VTRACE)
  const float* bootstrap;  // [B]
  float* out0;             // GAE: advantages      VTRACE: vs
  float* out1;             // GAE: value targets   VTRACE: pg advantages
  int T, B;
  float gamma, lam;                 // GAE
  float rho_bar, c_bar, pg_rho_bar;  // VTRACE (lam reused as c scale)
};

template <int MODE>
__device__ __forceinline__ void coeffs(const ScanArgs& a, int t, int b, float vnext, float& av,
                                       float& bv) {
  const long i = (long)t * a.B + b;
  if (MODE == MODE_GAE) {
    const float nt = 1.f - a.dones[i];
    bv = a.rewards[i] + a.gamma * vnext * nt - a.values[i];
    av = a.gamma * a.lam * nt;
  } else {
    const float rho = __expf(a.log_rhos[i]);
    const float disc = a.discounts[i];
    bv = fminf(a.rho_bar, rho) * (a.rewards[i] + disc * vnext - a.values[i]);
    av = disc * a.lam * fminf(a.c_bar, rho);
  }
}

template <int MODE>
__device__ __forceinline__ void emit(const ScanArgs& a, int t, int b, float x, float xnext,
                                     float vnext_boot) {
  const long i = (long)t * a.B + b;
  const float v = a.values[i];
  if (MODE == MODE_GAE) {
    a.out0[i] = x;
    a.out1[i] = x + v;
  } else {
    a.out0[i] = v + x;
    // vs_{t+1}: for t = T-1 it is the bootstrap value, else V_{t+1} + x_{t+1}
    const float vs_next = (t == a.T - 1) ? vnext_boot : (a.values[i + a.B] + xnext);
    const float rho = __expf(a.log_rhos[i]);
    a.out1[i] = fminf(a.pg_rho_bar, rho) * (a.rewards[i] + a.discounts[i] * vs_next - v);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void scan_serial_kernel(ScanArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const float boot = a.bootstrap[b];
  float x = 0.f, vnext = boot;
  for (int t = a.T - 1; t >= 0; --t) {
    float av, bv;
    coeffs<MODE>(a, t, b, vnext, av, bv);
    const float xn = x;
    x = bv + av * x;
    emit<MODE>(a, t, b, x, xn, boot);
    vnext = a.values[(long)t * a.B + b];
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void scan_wave_kernel(ScanArgs a) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.B) return;
  const int C = (a.T + 63) / 64;
  const int t0 = lane * C;
  const int t1 = min(a.T, t0 + C);
  const float boot = a.bootstrap[b];
  // 1) compose this lane's chunk: x_{t0} = Bc + Ac * x_{t1}
  float Ac = 1.f, Bc = 0.f;
  for (int t = t1 - 1; t >= t0; --t) {
    const float vnext = (t == a.T - 1) ? boot : a.values[(long)(t + 1) * a.B + b];
    float av, bv;
    coeffs<MODE>(a, t, b, vnext, av, bv);
    Bc = bv + av * Bc;
    Ac = av * Ac;
  }
  // 2) suffix-compose across lanes: F_l = f_l o f_{l+1} o ... o f_63
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float Ao = __shfl_down(Ac, off, 64);
    const float Bo = __shfl_down(Bc, off, 64);
    if (lane + off < 64) {
      Bc = Bc + Ac * Bo;
      Ac = Ac * Ao;
    }
  }
  // x at start of lane l's chunk = F_l(0); carry-in of lane l = start of lane l+1
  float carry = __shfl_down(Bc, 1, 64);
  if (lane == 63) carry = 0.f;
  // 3) replay the chunk from the carry-in
  float x = carry;
  for (int t = t1 - 1; t >= t0; --t) {
    const float vnext = (t == a.T - 1) ? boot : a.values[(long)(t + 1) * a.B + b];
    float av, bv;
    coeffs<MODE>(a, t, b, vnext, av, bv);
    const float xn = x;
    x = bv + av * x;
    emit<MODE>(a, t, b, x, xn, boot);
  }
}

template <int MODE>
static int launch_scan(const ScanArgs& a, hipStream_t st) {
  if (a.B >= 1024 || a.T <= 64) {
    hipLaunchKernelGGL(scan_serial_kernel<MODE>, dim3((a.B + 255) / 256), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(scan_wave_kernel<MODE>, dim3((a.B + 3) / 4), dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

RA_EXPORT int ra_gae(const float* rewards, const float* values, const float* dones,
                     const float* bootstrap, float* adv, float* vtarg, int T, int B, float gamma,
                     float lam, hipStream_t st) {
  ScanArgs a{};
  a.rewards = rewards; a.values = values; a.dones = dones; a.bootstrap = bootstrap;
  a.out0 = adv; a.out1 = vtarg; a.T = T; a.B = B; a.gamma = gamma; a.lam = lam;
  return launch_scan<MODE_GAE>(a, st);
}

RA_EXPORT int ra_vtrace(const float* log_rhos, const float* discounts, const float* rewards,
                        const float* values, const float* bootstrap, float* vs, float* pg_adv,
                        int T, int B, float rho_bar, float c_bar, float pg_rho_bar, float lam,
                        hipStream_t st) {
  ScanArgs a{};
  a.log_rhos = log_rhos; a.discounts = discounts; a.rewards = rewards; a.values = values;
  a.bootstrap = bootstrap; a.out0 = vs; a.out1 = pg_adv; a.T = T; a.B = B;
  a.rho_bar = rho_bar; a.c_bar = c_bar; a.pg_rho_bar = pg_rho_bar; a.lam = lam;
  return launch_scan<MODE_VTRACE>(a, st);
}

// ---------------------------------------------------------------------------
// Fused PPO loss, categorical policy. One thread per sample, logits in registers.
// stats[0..5] += {total, policy_loss, vf_loss, entropy, kl, clip_frac} (means)
//
// The policy outputs (logits, vpred) are the minibatch rows in order, fp32 or bf16
// (the learner's bf16 heads are read directly: no cast kernels). The behaviour-side
// fields (old_logits, action, old_logp, adv, vtarg) are read through row pointers +
// row strides, optionally GATHERED by `idx` from the full train batch: the learner
// packs them into one fp32 table [N_full, A+4], so a minibatch needs no gather
// kernels at all.
struct PPOArgs {
  const void* logits;       // [N,A] current policy (bf16 when in_bf16)
  const void* vpred;        // [N] (may be null: no value loss)
  const float* old_logits;  // row r at old_logits + r*ld_old; may be null
  const void* actions;      // long (act_f32 == 0) or float, row r at actions + r*ld_act
  const float* old_logp;    // row r at + r*ld_aux (same stride for old_logp/adv/vtarg)
  const float* adv;
  const float* vtarg;
  const long* idx;          // [N] rows of the behaviour table; null = identity
  float* dlogits;           // [N,A] fp32 d(mean loss)/dlogits
  float* dvpred;            // [N]
  float* stats;             // [6] accumulated (the caller zeroes it when it wants)
  const float* kl_dev;      // device-resident KL coefficient (overrides kl_coeff; may be null)
  int N, A, in_bf16, act_f32, ld_old, ld_act, ld_aux;
  float clip, vf_clip, vf_coeff, ent_coeff, kl_coeff, inv_n;
};

__device__ __forceinline__ float ld_in(const void* p, long k, int bf) {
  return bf ? bf2f(reinterpret_cast<const bf16_t*>(p)[k]) : reinterpret_cast<const float*>(p)[k];
}

template <int AMAX>
__global__ __launch_bounds__(256) void ppo_loss_kernel(PPOArgs p) {
  __shared__ float red[4];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float s_total = 0.f, s_pol = 0.f, s_vf = 0.f, s_ent = 0.f, s_kl = 0.f, s_clip = 0.f;
  if (i < p.N) {
    const long r = p.idx ? p.idx[i] : (long)i;
    float z[AMAX], lp[AMAX];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < AMAX; ++j) {
      z[j] = (j < p.A) ? ld_in(p.logits, (long)i * p.A + j, p.in_bf16) : -INFINITY;
      mx = fmaxf(mx, z[j]);
    }
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < AMAX; ++j) se += (j < p.A) ? __expf(z[j] - mx) : 0.f;
    const float lse = mx + __logf(se);
    float ent = 0.f;
#pragma unroll
    for (int j = 0; j < AMAX; ++j) {
      lp[j] = (j < p.A) ? z[j] - lse : 0.f;
      if (j < p.A) ent -= __expf(lp[j]) * lp[j];
    }
    // KL(old || new)
    float kl = 0.f, olp[AMAX];
    if (p.old_logits) {
      const float* orow = p.old_logits + r * p.ld_old;
      float omx = -INFINITY;
#pragma unroll
      for (int j = 0; j < AMAX; ++j) {
        olp[j] = (j < p.A) ? orow[j] : -INFINITY;
        omx = fmaxf(omx, olp[j]);
      }
      float ose = 0.f;
#pragma unroll
      for (int j = 0; j < AMAX; ++j) ose += (j < p.A) ? __expf(olp[j] - omx) : 0.f;
      const float olse = omx + __logf(ose);
#pragma unroll
      for (int j = 0; j < AMAX; ++j) {
        olp[j] = (j < p.A) ? olp[j] - olse : 0.f;
        if (j < p.A) kl += __expf(olp[j]) * (olp[j] - lp[j]);
      }
    }
    const long act = p.act_f32 ? (long)reinterpret_cast<const float*>(p.actions)[r * p.ld_act]
                               : reinterpret_cast<const long*>(p.actions)[r * p.ld_act];
    float logp = 0.f;
#pragma unroll
    for (int j = 0; j < AMAX; ++j) if (j == act) logp = lp[j];
    const long ra = r * p.ld_aux;
    const float ratio = __expf(logp - p.old_logp[ra]);
    const float A_ = p.adv[ra];
    const float rc = fminf(fmaxf(ratio, 1.f - p.clip), 1.f + p.clip);
    const float s1 = A_ * ratio, s2 = A_ * rc;
    const float surr = fminf(s1, s2);
    // d surr / d logp
    float dsurr;
    if (s1 <= s2) dsurr = A_ * ratio;
    else dsurr = (ratio > 1.f - p.clip && ratio < 1.f + p.clip) ? A_ * ratio : 0.f;
    const bool clipped = (ratio < 1.f - p.clip) || (ratio > 1.f + p.clip);
    float vf = 0.f, dv = 0.f;
    if (p.vpred) {
      const float e = ld_in(p.vpred, i, p.in_bf16) - p.vtarg[ra];
      const float e2 = e * e;
      vf = fminf(e2, p.vf_clip);
      dv = (e2 < p.vf_clip) ? 2.f * e : 0.f;
      p.dvpred[i] = p.vf_coeff * dv * p.inv_n;
    }
    const float kl_c = p.kl_dev ? p.kl_dev[0] : p.kl_coeff;
    const float total = -surr + p.vf_coeff * vf - p.ent_coeff * ent + kl_c * kl;
    // gradient wrt logits
#pragma unroll
    for (int j = 0; j < AMAX; ++j) {
      if (j < p.A) {
        const float pj = __expf(lp[j]);
        float g = -dsurr * ((j == act ? 1.f : 0.f) - pj);   // policy term
        g += p.ent_coeff * pj * (lp[j] + ent);               // -c * dH/dz, dH/dz = -p(logp+H)
        if (p.old_logits) g += kl_c * (pj - __expf(olp[j]));
        p.dlogits[(long)i * p.A + j] = g * p.inv_n;
      }
    }
    s_total = total; s_pol = -surr; s_vf = vf; s_ent = ent; s_kl = kl; s_clip = clipped ? 1.f : 0.f;
  }
  float vals[6] = {s_total, s_pol, s_vf, s_ent, s_kl, s_clip};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const float t = block_sum<4>(vals[k], red);
    if (threadIdx.x == 0) atomicAdd(&p.stats[k], t * p.inv_n);
  }
}

static int ppo_launch(const PPOArgs& p, hipStream_t st) {
  const dim3 g((p.N + 255) / 256);
  if (p.A <= 4) hipLaunchKernelGGL(ppo_loss_kernel<4>, g, dim3(256), 0, st, p);
  else if (p.A <= 8) hipLaunchKernelGGL(ppo_loss_kernel<8>, g, dim3(256), 0, st, p);
  else if (p.A <= 18) hipLaunchKernelGGL(ppo_loss_kernel<18>, g, dim3(256), 0, st, p);
  else if (p.A <= 32) hipLaunchKernelGGL(ppo_loss_kernel<32>, g, dim3(256), 0, st, p);
  else if (p.A <= 64) hipLaunchKernelGGL(ppo_loss_kernel<64>, g, dim3(256), 0, st, p);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Contiguous per-minibatch inputs (fp32 or bf16 logits/vpred); stats are zeroed here.
RA_EXPORT int ra_ppo_loss(const void* logits, const float* old_logits, const long* actions,
                          const float* old_logp, const float* adv, const void* vpred,
                          const float* vtarg, float* dlogits, float* dvpred, float* stats, int N,
                          int A, float clip, float vf_clip, float vf_coeff, float ent_coeff,
                          float kl_coeff, int in_bf16, hipStream_t st) {
  PPOArgs p{logits, vpred, old_logits, actions, old_logp, adv, vtarg, nullptr, dlogits, dvpred,
            stats, nullptr, N, A, in_bf16, 0, A, 1, 1, clip, vf_clip, vf_coeff, ent_coeff,
            kl_coeff, 1.f / (float)N};
  hipMemsetAsync(stats, 0, 6 * sizeof(float), st);
  return ppo_launch(p, st);
}

// Behaviour fields packed in one fp32 table aux[N_full, ld] = [old_logits(A) | action |
// old_logp | adv | vtarg] and gathered by idx[N] inside the kernel; stats ACCUMULATE
// (the learner sums them over every minibatch of an update without extra kernels).
// kl_dev (optional) is a device scalar read at run time, so a captured graph survives
// the adaptive KL coefficient changing between updates.
RA_EXPORT int ra_ppo_loss_packed(const void* logits, const void* vpred, const float* aux, int ld,
                                 int has_old, const long* idx, float* dlogits, float* dvpred,
                                 float* stats, int N, int A, float clip, float vf_clip,
                                 float vf_coeff, float ent_coeff, float kl_coeff,
                                 const float* kl_dev, int in_bf16, float inv_n, hipStream_t st) {
  if (ld < A + 4) return hipErrorInvalidValue;
  PPOArgs p{logits, vpred, has_old ? aux : nullptr, aux + A, aux + A + 1, aux + A + 2,
            aux + A + 3, idx, dlogits, dvpred, stats, kl_dev, N, A, in_bf16, 1, ld, ld, ld, clip,
            vf_clip, vf_coeff, ent_coeff, kl_coeff, inv_n};
  return ppo_launch(p, st);
}

// out_bf16[k] = g[0] * src[k] for the concatenated fp32 loss gradients (one launch for
// dlogits and dvpred; g is the upstream scalar gradient, read on device).
__global__ __launch_bounds__(256) void scale_to_bf16_kernel(const float* __restrict__ src, long n,
                                                             const float* __restrict__ g,
                                                             bf16_t* __restrict__ out) {
  const float s = g ? g[0] : 1.f;
  for (long k = blockIdx.x * (long)blockDim.x + threadIdx.x; k < n;
       k += (long)gridDim.x * blockDim.x)
    out[k] = f2bf(src[k] * s);
}

RA_EXPORT int ra_scale_to_bf16(const float* src, long n, const float* g, void* out,
                               hipStream_t st) {
  hipLaunchKernelGGL(scale_to_bf16_kernel, dim3(ra_grid(n, 256)), dim3(256), 0, st, src, n, g,
                     (bf16_t*)out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Running mean/std (Chan et al. parallel merge). stats layout (f32):
//   mean[D], m2[D]; count kept on the host (exact integer).
__global__ __launch_bounds__(256) void colmoments_kernel(const float* __restrict__ x, int N, int D,
                                                         int rows_per_part,
                                                         float* __restrict__ pmean,
                                                         float* __restrict__ pm2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  const int r0 = blockIdx.y * rows_per_part, r1 = min(N, r0 + rows_per_part);
  float mean = 0.f, m2 = 0.f;
  int n = 0;
  for (int r = r0; r < r1; ++r) {
    const float v = x[(long)r * D + c];
    ++n;
    const float d = v - mean;
    mean += d / n;
    m2 += d * (v - mean);
  }
  pmean[(long)blockIdx.y * D + c] = mean;
  pm2[(long)blockIdx.y * D + c] = m2;
}

__global__ __launch_bounds__(256) void merge_moments_kernel(const float* __restrict__ pmean,
                                                            const float* __restrict__ pm2, int P,
                                                            int rows_per_part, int N, int D,
                                                            double count, float* __restrict__ mean,
                                                            float* __restrict__ m2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  double na = count, ma = mean[c], sa = m2[c];
  for (int p = 0; p < P; ++p) {
    const int nb_i = min(N, (p + 1) * rows_per_part) - p * rows_per_part;
    if (nb_i <= 0) break;
    const double nb = nb_i, mb = pmean[(long)p * D + c], sb = pm2[(long)p * D + c];
    const double n = na + nb;
    const double d = mb - ma;
    ma = ma + d * nb / n;
    sa = sa + sb + d * d * na * nb / n;
    na = n;
  }
  mean[c] = (float)ma;
  m2[c] = (float)sa;
}

__global__ __launch_bounds__(256) void obsnorm_apply_kernel(const float* __restrict__ x,
                                                            float* __restrict__ y,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ m2,
                                                            long n, int D, float inv_cnt,
                                                            float clip, float eps) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    const float sd = sqrtf(fmaxf(m2[c] * inv_cnt, 0.f));
    float v = (x[i] - mean[c]) / (sd + eps);
    y[i] = fminf(fmaxf(v, -clip), clip);
  }
}

// work: 2 * P * D floats, P = ra_obsnorm_parts(N)
RA_EXPORT int ra_obsnorm_parts(int N) {
  int p = (N + 63) / 64;
  return p < 128 ? p : 128;
}

RA_EXPORT int ra_obsnorm_update(const float* x, int N, int D, double count, float* mean,
                                float* m2, float* work, hipStream_t st) {
  const int P = ra_obsnorm_parts(N);
  const int rpp = (N + P - 1) / P;
  float* pmean = work;
  float* pm2 = work + (size_t)P * D;
  hipLaunchKernelGGL(colmoments_kernel, dim3((D + 255) / 256, P), dim3(256), 0, st, x, N, D, rpp,
                     pmean, pm2);
  hipLaunchKernelGGL(merge_moments_kernel, dim3((D + 255) / 256), dim3(256), 0, st, pmean, pm2, P,
                     rpp, N, D, count, mean, m2);
  return hipGetLastError();
}

RA_EXPORT int ra_obsnorm_apply(const float* x, float* y, const float* mean, const float* m2,
                               long N, int D, double count, float clip, float eps,
                               hipStream_t st) {
  const long n = N * (long)D;
  const float inv = count > 1 ? (float)(1.0 / (count - 1)) : 1.f;
  hipLaunchKernelGGL(obsnorm_apply_kernel, dim3(ra_grid(n, 256)), dim3(256), 0, st, x, y, mean,
                     m2, n, D, inv, clip, eps);
  return hipGetLastError();
}
