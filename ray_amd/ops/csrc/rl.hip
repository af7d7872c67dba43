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

// Per-sample PPO loss and its gradient: z = logits (registers), v = value prediction,
// r = row of the behaviour table. Writes dz = d(total)/dz and *dv (NOT yet scaled by
// 1/N) and the six statistics of the sample.
template <int AMAX>
__device__ __forceinline__ void ppo_row(const PPOArgs& p, long r, const float (&z)[AMAX], float v,
                                        bool has_v, float (&dz)[AMAX], float* dv, float (&s6)[6]) {
  float lp[AMAX];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < AMAX; ++j) mx = fmaxf(mx, j < p.A ? z[j] : -INFINITY);
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
  float vf = 0.f;
  *dv = 0.f;
  if (has_v) {
    const float e = v - p.vtarg[ra];
    const float e2 = e * e;
    vf = fminf(e2, p.vf_clip);
    *dv = p.vf_coeff * ((e2 < p.vf_clip) ? 2.f * e : 0.f);
  }
  const float kl_c = p.kl_dev ? p.kl_dev[0] : p.kl_coeff;
  const float total = -surr + p.vf_coeff * vf - p.ent_coeff * ent + kl_c * kl;
#pragma unroll
  for (int j = 0; j < AMAX; ++j) {
    dz[j] = 0.f;
    if (j < p.A) {
      const float pj = __expf(lp[j]);
      float g = -dsurr * ((j == act ? 1.f : 0.f) - pj);   // policy term
      g += p.ent_coeff * pj * (lp[j] + ent);               // -c * dH/dz, dH/dz = -p(logp+H)
      if (p.old_logits) g += kl_c * (pj - __expf(olp[j]));
      dz[j] = g;
    }
  }
  s6[0] = total; s6[1] = -surr; s6[2] = vf; s6[3] = ent; s6[4] = kl; s6[5] = clipped ? 1.f : 0.f;
}

template <int AMAX>
__global__ __launch_bounds__(256) void ppo_loss_kernel(PPOArgs p) {
  __shared__ float red[4];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float s6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < p.N) {
    const long r = p.idx ? p.idx[i] : (long)i;
    float z[AMAX], dz[AMAX], dv;
#pragma unroll
    for (int j = 0; j < AMAX; ++j)
      z[j] = (j < p.A) ? ld_in(p.logits, (long)i * p.A + j, p.in_bf16) : 0.f;
    const float v = p.vpred ? ld_in(p.vpred, i, p.in_bf16) : 0.f;
    ppo_row<AMAX>(p, r, z, v, p.vpred != nullptr, dz, &dv, s6);
    if (p.vpred) p.dvpred[i] = dv * p.inv_n;
#pragma unroll
    for (int j = 0; j < AMAX; ++j)
      if (j < p.A) p.dlogits[(long)i * p.A + j] = dz[j] * p.inv_n;
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const float t = block_sum<4>(s6[k], red);
    if (threadIdx.x == 0) atomicAdd(&p.stats[k], t * p.inv_n);
  }
}

// ---------------------------------------------------------------------------
// Fused policy/value heads + PPO loss (shared encoder): per minibatch row, one wave
//   forward : logits = h Wpi^T + bpi, v = h wvf + bvf (wave dot products over F),
//             the PPO row math, d7[row] = [dlogits | dv] / N       (ra_ppo_heads_fwd)
//   backward: dh = g * (d7[:, :A] Wpi + d7[:, A] wvf), per-wave partials of
//             dW = d7^T h and db = sum d7, then one reduction writing the four
//             parameter gradients (flat-buffer sinks)                (ra_ppo_heads_bwd)
// replacing two head GEMMs, two bias adds, the loss, two casts, four backward GEMMs,
// the dX add and two bias reductions of the unfused graph.
struct HeadsArgs {
  const bf16_t* h;      // [N, F]
  const bf16_t* wpi;    // [A, F]
  const bf16_t* bpi;    // [A]
  const bf16_t* wvf;    // [F]
  const bf16_t* bvf;    // [1]
  float* d7;            // [N, A+1]
  const float* g;       // upstream scalar gradient (bwd; may be null = 1)
  bf16_t* dh;           // [N, F]
  float* part;          // [P4][(A+1)*(F+1)] per-wave partials
  int F;
};

template <int AMAX>
__global__ __launch_bounds__(256) void ppo_heads_fwd_kernel(PPOArgs p, HeadsArgs q) {
  __shared__ float red[4][6];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int A = p.A, F = q.F;
  float sacc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = blockIdx.x * 4 + wv; i < p.N; i += gridDim.x * 4) {
    float z[AMAX], v = 0.f;
#pragma unroll
    for (int j = 0; j < AMAX; ++j) z[j] = 0.f;
    for (int c = lane * 8; c < F; c += 512) {
      float hv[8], wv8[8];
      unpack8(*reinterpret_cast<const uint4*>(q.h + (long)i * F + c), hv);
#pragma unroll
      for (int j = 0; j < AMAX; ++j) {
        if (j >= A) break;
        unpack8(*reinterpret_cast<const uint4*>(q.wpi + (long)j * F + c), wv8);
#pragma unroll
        for (int e = 0; e < 8; ++e) z[j] += hv[e] * wv8[e];
      }
      unpack8(*reinterpret_cast<const uint4*>(q.wvf + c), wv8);
#pragma unroll
      for (int e = 0; e < 8; ++e) v += hv[e] * wv8[e];
    }
#pragma unroll
    for (int j = 0; j < AMAX; ++j) z[j] = j < A ? wave_sum(z[j]) + bf2f(q.bpi[j]) : 0.f;
    v = wave_sum(v) + bf2f(q.bvf[0]);
    // heads outputs are bf16 in the unfused model: round the same way
#pragma unroll
    for (int j = 0; j < AMAX; ++j) z[j] = bf2f(f2bf(z[j]));
    v = bf2f(f2bf(v));
    const long r = p.idx ? p.idx[i] : (long)i;
    float dz[AMAX], dv, s6[6];
    ppo_row<AMAX>(p, r, z, v, true, dz, &dv, s6);
    if (lane == 0) {
      float* o = q.d7 + (long)i * (A + 1);
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A) o[j] = dz[j] * p.inv_n;
      o[A] = dv * p.inv_n;
#pragma unroll
      for (int k = 0; k < 6; ++k) sacc[k] += s6[k];
    }
  }
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) red[wv][k] = sacc[k];
  __syncthreads();
  if (threadIdx.x < 6)
    atomicAdd(&p.stats[threadIdx.x], (red[0][threadIdx.x] + red[1][threadIdx.x] +
                                      red[2][threadIdx.x] + red[3][threadIdx.x]) * p.inv_n);
}

// grid P blocks x 4 waves; wave w of block b takes rows b*4+w, +4P, ...; each lane owns
// 8-column slices c = 8*lane + 512k of F and keeps (A+1) x 8 dW partials per slice.
template <int AMAX, int NSL>
__global__ __launch_bounds__(256) void ppo_heads_bwd_kernel(int N, int A, HeadsArgs q) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, F = q.F;
  const int wave = blockIdx.x * 4 + wv, nwaves = gridDim.x * 4;
  const float gs = q.g ? q.g[0] : 1.f;
  float acc[NSL][AMAX + 1][8];
  float dbacc[AMAX + 1];
#pragma unroll
  for (int s = 0; s < NSL; ++s)
#pragma unroll
    for (int j = 0; j <= AMAX; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[s][j][e] = 0.f;
#pragma unroll
  for (int j = 0; j <= AMAX; ++j) dbacc[j] = 0.f;
  for (int i = wave; i < N; i += nwaves) {
    float d[AMAX + 1];
#pragma unroll
    for (int j = 0; j <= AMAX; ++j) d[j] = 0.f;
    for (int j = 0; j <= A; ++j) d[j < A ? j : AMAX] = gs * q.d7[(long)i * (A + 1) + j];
#pragma unroll
    for (int j = 0; j <= AMAX; ++j) dbacc[j] += d[j];
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const int c = lane * 8 + 512 * s;
      if (c >= F) break;
      float hv[8], o[8], w8[8];
      unpack8(*reinterpret_cast<const uint4*>(q.h + (long)i * F + c), hv);
      unpack8(*reinterpret_cast<const uint4*>(q.wvf + c), w8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = d[AMAX] * w8[e];
        acc[s][AMAX][e] += d[AMAX] * hv[e];
      }
#pragma unroll
      for (int j = 0; j < AMAX; ++j) {
        if (j >= A) break;
        unpack8(*reinterpret_cast<const uint4*>(q.wpi + (long)j * F + c), w8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] += d[j] * w8[e];
          acc[s][j][e] += d[j] * hv[e];
        }
      }
      *reinterpret_cast<uint4*>(q.dh + (long)i * F + c) = pack8(o);
    }
  }
  // per-wave partial row: [W rows 0..A-1 = pi, row A = vf][F] then [b 0..A]
  const int L = (A + 1) * (F + 1);
  float* pr = q.part + (size_t)wave * L;
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    const int c = lane * 8 + 512 * s;
    if (c >= F) break;
#pragma unroll
    for (int j = 0; j <= AMAX; ++j) {
      if (j < AMAX && j >= A) continue;
      const int row = j < AMAX ? j : A;
      float* dst = pr + (size_t)row * F + c;
      *reinterpret_cast<float4*>(dst) = make_float4(acc[s][j][0], acc[s][j][1], acc[s][j][2], acc[s][j][3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[s][j][4], acc[s][j][5], acc[s][j][6], acc[s][j][7]);
    }
  }
  if (lane == 0)
#pragma unroll
    for (int j = 0; j <= AMAX; ++j) {
      if (j < AMAX && j >= A) continue;
      pr[(size_t)(A + 1) * F + (j < AMAX ? j : A)] = dbacc[j];
    }
}

// out[col] (+)= sum over the P4 wave partials; columns map to the four gradients.
struct HeadsGrads {
  void* wpi; void* bpi; void* wvf; void* bvf;
};

template <bool F32, bool ACC>
__global__ __launch_bounds__(1024) void ppo_heads_reduce(const float* __restrict__ part, int P4,
                                                         int A, int F, HeadsGrads o) {
  __shared__ float red[16][65];
  const int L = (A + 1) * (F + 1);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + tx;
  float s = 0.f;
  if (j < L)
    for (int p = ty; p < P4; p += 16) s += part[(size_t)p * L + j];
  red[ty][tx] = s;
  __syncthreads();
  if (ty != 0 || j >= L) return;
  s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += red[i][tx];
  void* dst;
  long k;
  if (j < A * F) { dst = o.wpi; k = j; }
  else if (j < (A + 1) * F) { dst = o.wvf; k = j - A * F; }
  else if (j < (A + 1) * F + A) { dst = o.bpi; k = j - (A + 1) * F; }
  else { dst = o.bvf; k = 0; }
  if (F32) {
    float* d = reinterpret_cast<float*>(dst) + k;
    *d = ACC ? *d + s : s;
  } else {
    bf16_t* d = reinterpret_cast<bf16_t*>(dst) + k;
    *d = f2bf(ACC ? s + bf2f(*d) : s);
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

static constexpr int kHeadsWaves = 64 * 4;  // bwd partial rows (64 blocks x 4 waves)

RA_EXPORT int ra_ppo_heads_fwd(const void* h, int F, const void* wpi, const void* bpi,
                               const void* wvf, const void* bvf, const float* aux, int ld,
                               int has_old, const long* idx, float* d7, float* stats, int N,
                               int A, float clip, float vf_clip, float vf_coeff, float ent_coeff,
                               float kl_coeff, const float* kl_dev, float inv_n, hipStream_t st) {
  if (ld < A + 4 || F % 8 || F > 1024 || A > 18 || N <= 0) return hipErrorInvalidValue;
  PPOArgs p{nullptr, nullptr, has_old ? aux : nullptr, aux + A, aux + A + 1, aux + A + 2,
            aux + A + 3, idx, nullptr, nullptr, stats, kl_dev, N, A, 0, 1, ld, ld, ld, clip,
            vf_clip, vf_coeff, ent_coeff, kl_coeff, inv_n};
  HeadsArgs q{(const bf16_t*)h, (const bf16_t*)wpi, (const bf16_t*)bpi, (const bf16_t*)wvf,
              (const bf16_t*)bvf, d7, nullptr, nullptr, nullptr, F};
  int blocks = (N + 3) / 4;
  if (blocks > 128) blocks = 128;
  if (A <= 8) hipLaunchKernelGGL(ppo_heads_fwd_kernel<8>, dim3(blocks), dim3(256), 0, st, p, q);
  else hipLaunchKernelGGL(ppo_heads_fwd_kernel<18>, dim3(blocks), dim3(256), 0, st, p, q);
  return hipGetLastError();
}

RA_EXPORT long ra_ppo_heads_work(int A, int F) { return (long)kHeadsWaves * (A + 1) * (F + 1); }

// flags: bit0 accumulate into the gradients, bit1 gradients are fp32 (else bf16)
RA_EXPORT int ra_ppo_heads_bwd(const void* h, int F, const void* wpi, const void* wvf,
                               const float* d7, const float* g, void* dh, float* work,
                               void* dwpi, void* dbpi, void* dwvf, void* dbvf, int flags, int N,
                               int A, hipStream_t st) {
  if (F % 8 || F > 1024 || A > 18 || N <= 0) return hipErrorInvalidValue;
  HeadsArgs q{(const bf16_t*)h, (const bf16_t*)wpi, nullptr, (const bf16_t*)wvf, nullptr,
              const_cast<float*>(d7), g, (bf16_t*)dh, work, F};
  const dim3 gb(kHeadsWaves / 4), b(256);
  if (A <= 8) {
    if (F <= 512) hipLaunchKernelGGL((ppo_heads_bwd_kernel<8, 1>), gb, b, 0, st, N, A, q);
    else hipLaunchKernelGGL((ppo_heads_bwd_kernel<8, 2>), gb, b, 0, st, N, A, q);
  } else {
    if (F <= 512) hipLaunchKernelGGL((ppo_heads_bwd_kernel<18, 1>), gb, b, 0, st, N, A, q);
    else hipLaunchKernelGGL((ppo_heads_bwd_kernel<18, 2>), gb, b, 0, st, N, A, q);
  }
  HeadsGrads o{dwpi, dbpi, dwvf, dbvf};
  const int L = (A + 1) * (F + 1);
  const dim3 rg((L + 63) / 64), rb(1024);
  switch (flags & 3) {
    case 0: hipLaunchKernelGGL((ppo_heads_reduce<false, false>), rg, rb, 0, st, work, kHeadsWaves, A, F, o); break;
    case 1: hipLaunchKernelGGL((ppo_heads_reduce<false, true>), rg, rb, 0, st, work, kHeadsWaves, A, F, o); break;
    case 2: hipLaunchKernelGGL((ppo_heads_reduce<true, false>), rg, rb, 0, st, work, kHeadsWaves, A, F, o); break;
    default: hipLaunchKernelGGL((ppo_heads_reduce<true, true>), rg, rb, 0, st, work, kHeadsWaves, A, F, o);
  }
  return hipGetLastError();
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
