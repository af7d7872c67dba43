// bf16 x bf16 -> fp32 GEMMs through hipBLASLt with per-shape solution selection.
//
// Why: the weight-gradient GEMMs write (or accumulate into) the fp32 flat-gradient sink.
// PyTorch's TunableOp only tunes GEMMs whose output dtype equals the input dtype, so these
// ran on hipBLASLt's first heuristic choice (~0.9 PF/s at GPT-2 shapes, vs 1.1-1.5 for
// the tuned bf16 GEMMs), and the old path also round-tripped split-K fp32 partials
// through HBM. Here the sink is the GEMM's C/D operand (beta = 1: D = A*B + D, the
// accumulation is free), and each problem shape picks the fastest of up to 128 heuristic
// candidates, timed on the device (ra_lt_tune) and cached by the Python side.
//
// Column-major BLAS convention (hipBLASLt): D[m x n] = op(A)[m x k] * op(B)[k x n].
#include "common.h"

#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace {

typedef std::tuple<int, int, long, long, long, long, long, long, int, long, long, long> LtKey;

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  std::vector<hipblasLtMatmulHeuristicResult_t> cands;
  std::vector<signed char> streamk;  // per candidate: 1 = stream-K kernel
  bool sk_only = false;  // hipBLASLt offers nothing but stream-K for this shape
  int choice = 0;
};

hipblasLtHandle_t g_handle = nullptr;
const size_t kWs = 64ull << 20;
std::map<LtKey, LtPlan*> g_plans;
std::mutex g_mu;
// One workspace AND one hipBLASLt handle PER STREAM. Stream-K kernels keep partial tiles
// and arrival flags in the workspace, and hipBLASLt keeps further stream-K synchronisation
// state per handle: two stream-K GEMMs running concurrently on two streams through ONE
// handle hang even with separate workspaces (profiles/r4/README.md §2: the two-stream
// ops/lt repro hung with per-stream workspaces and a shared handle; torch's own GEMMs on
// two streams share torch's handle the same way). Heuristic queries and plans use g_handle;
// every launch uses its stream's handle.
std::map<hipStream_t, void*> g_ws_by_stream;
std::map<hipStream_t, hipblasLtHandle_t> g_handle_by_stream;
std::mutex g_ws_mu;  // not g_mu: the GEMM entry points call this with g_mu held

bool env_on(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '1';
}

// RAY_AMD_LT_SHARED_HANDLE=1: launch everything through g_handle (diagnostic only: the
// failure above, scripts/lmhead_hang_repro.py mode lt2h)
hipblasLtHandle_t handle_for(hipStream_t st) {
  static const bool shared = env_on("RAY_AMD_LT_SHARED_HANDLE");
  if (shared) return g_handle;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_handle_by_stream.find(st);
  if (it != g_handle_by_stream.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return g_handle;
  g_handle_by_stream[st] = h;
  return h;
}

void* workspace(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  // RAY_AMD_LT_SHARED_WS=1: one workspace for every stream (diagnostic only, mode lt2shared)
  static const bool shared = env_on("RAY_AMD_LT_SHARED_WS");
  if (shared) st = nullptr;
  auto it = g_ws_by_stream.find(st);
  if (it != g_ws_by_stream.end()) return it->second;
  void* w = nullptr;
  if (hipMalloc(&w, kWs) != hipSuccess) return nullptr;
  g_ws_by_stream[st] = w;
  return w;
}

// Stream-K policy. On gfx950 every hipBLASLt bf16 kernel is a Tensile StreamK=3 kernel
// (`..._SK3_SKXCCM8_...` in every name, tests/test_train_gpu.py): whether a launch splits
// K across workgroups (with a fixup in which the tile's owner spin-waits on the partial
// tiles of later workgroups of the SAME grid) is decided per launch from the problem size.
// ra_lt_allow_streamk(0) (RAY_AMD_LT_NO_STREAMK=1) restricts choices to kernels without a
// stream-K tag where any exist; a plan with nothing else keeps its candidates (sk_only).
bool g_allow_sk = true;

bool is_streamk_name(const std::string& n) {
  for (size_t i = n.find("_SK"); i != std::string::npos; i = n.find("_SK", i + 1))
    if (i + 3 < n.size() && n[i + 3] >= '0' && n[i + 3] <= '9') return true;
  return n.find("StreamK") != std::string::npos;
}

std::string cand_name(LtPlan* p, int i) {
  return hipblaslt_ext::getKernelNameFromAlgo(g_handle, p->cands[i].algo);
}

bool cand_sk(LtPlan* p, int i) {
  if (p->streamk.size() != p->cands.size()) {
    p->streamk.assign(p->cands.size(), 0);
    for (size_t j = 0; j < p->cands.size(); ++j)
      p->streamk[j] = is_streamk_name(cand_name(p, (int)j)) ? 1 : 0;
  }
  return p->streamk[i] != 0;
}

bool usable(LtPlan* p, int i) { return g_allow_sk || p->sk_only || !cand_sk(p, i); }

int first_usable(LtPlan* p) {
  for (int i = 0; i < (int)p->cands.size(); ++i)
    if (usable(p, i)) return i;
  return -1;
}

int init_handle() {
  if (g_handle) return 0;
  if (hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return -1;
  return 0;
}

LtPlan* get_plan(int ta, int tb, long m, long n, long k, long lda, long ldb, long ldc,
                 int batch = 1, long sa = 0, long sb = 0, long sc = 0) {
  const LtKey key(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second;
  if (init_handle() != 0) return nullptr;
  LtPlan* p = new LtPlan();
  hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
  hipblasLtMatrixLayoutCreate(&p->a, HIP_R_16BF, ta ? k : m, ta ? m : k, lda);
  hipblasLtMatrixLayoutCreate(&p->b, HIP_R_16BF, tb ? n : k, tb ? k : n, ldb);
  hipblasLtMatrixLayoutCreate(&p->c, HIP_R_32F, m, n, ldc);
  if (batch > 1) {
    const int32_t bc = batch;
    const int64_t st[3] = {sa, sb, sc};
    hipblasLtMatrixLayout_t ls[3] = {p->a, p->b, p->c};
    for (int i = 0; i < 3; ++i) {
      hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc,
                                        sizeof(bc));
      hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET,
                                        &st[i], sizeof(st[i]));
    }
  }
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wsz = kWs;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz,
                                        sizeof(wsz));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(128);
  int got = 0;
  hipblasLtMatmulAlgoGetHeuristic(g_handle, p->desc, p->a, p->b, p->c, p->c, pref, 128,
                                  res.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  for (int i = 0; i < got; ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= kWs)
      p->cands.push_back(res[i]);
  const int f = first_usable(p);
  // only stream-K solutions (small shapes on gfx950): keep them, flagged; the caller then
  // runs this GEMM on the main stream (ra_lt_choice_is_streamk), never beside another GEMM
  if (f < 0 && !p->cands.empty()) p->sk_only = true;
  else if (f >= 0) p->choice = f;
  g_plans[key] = p;
  return p;
}

int run(LtPlan* p, int idx, const void* A, const void* B, float* C, float alpha, float beta,
        hipStream_t st) {
  const hipblasStatus_t s =
      hipblasLtMatmul(handle_for(st), p->desc, &alpha, A, p->a, B, p->b, &beta, C, p->c, C,
                      p->c, &p->cands[idx].algo, workspace(st), kWs, st);
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : 1000 + (int)s;
}

}  // namespace

// Number of usable candidates for a shape (creates the plan); < 0 on failure.
RA_EXPORT int ra_lt_num_cands(int ta, int tb, long m, long n, long k, long lda, long ldb,
                              long ldc) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_plan(ta, tb, m, n, k, lda, ldb, ldc);
  return p ? (int)p->cands.size() : -1;
}

RA_EXPORT int ra_lt_set_choice(int ta, int tb, long m, long n, long k, long lda, long ldb,
                               long ldc, int choice) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_plan(ta, tb, m, n, k, lda, ldb, ldc);
  if (!p || choice < 0 || choice >= (int)p->cands.size()) return -1;
  if (!usable(p, choice)) return -2;  // recorded choice is stream-K: keep the default
  p->choice = choice;
  return 0;
}

// C (fp32) = alpha * op(A) * op(B) + beta * C
RA_EXPORT int ra_lt_gemm(int ta, int tb, long m, long n, long k, const void* A, long lda,
                         const void* B, long ldb, float* C, long ldc, float alpha, float beta,
                         hipStream_t st) {
  LtPlan* p;
  {
    std::lock_guard<std::mutex> g(g_mu);
    p = get_plan(ta, tb, m, n, k, lda, ldb, ldc);
  }
  if (!p || p->cands.empty()) return -1;
  return run(p, p->choice, A, B, C, alpha, beta, st);
}

// Strided-batched variant: batch GEMMs, operand i at base + i * stride (elements).
RA_EXPORT int ra_lt_gemm_batched(int ta, int tb, long m, long n, long k, const void* A, long lda,
                                 long sa, const void* B, long ldb, long sb, float* C, long ldc,
                                 long sc, int batch, float alpha, float beta, hipStream_t st) {
  LtPlan* p;
  {
    std::lock_guard<std::mutex> g(g_mu);
    p = get_plan(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc);
  }
  if (!p || p->cands.empty()) return -1;
  return run(p, p->choice, A, B, C, alpha, beta, st);
}

RA_EXPORT int ra_lt_num_cands_batched(int ta, int tb, long m, long n, long k, long lda, long ldb,
                                      long ldc, int batch, long sa, long sb, long sc) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_plan(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc);
  return p ? (int)p->cands.size() : -1;
}

RA_EXPORT int ra_lt_set_choice_batched(int ta, int tb, long m, long n, long k, long lda,
                                       long ldb, long ldc, int batch, long sa, long sb, long sc,
                                       int choice) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_plan(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc);
  if (!p || choice < 0 || choice >= (int)p->cands.size()) return -1;
  if (!usable(p, choice)) return -2;
  p->choice = choice;
  return 0;
}

// Kernel name of a plan's current choice into out[cap] (diagnostics / tests). Returns the
// choice index, or < 0.
RA_EXPORT int ra_lt_choice_name(int ta, int tb, long m, long n, long k, long lda, long ldb,
                                long ldc, int batch, long sa, long sb, long sc, char* out,
                                int cap) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_plan(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc);
  if (!p || p->cands.empty() || cap <= 0) return -1;
  const std::string n_ = cand_name(p, p->choice);
  std::strncpy(out, n_.c_str(), cap - 1);
  out[cap - 1] = 0;
  return p->choice;
}

// 1 if the shape's current choice is a stream-K kernel (the GEMM must not run concurrently
// with another stream's GEMMs), 0 if not, < 0 if there is no solution.
RA_EXPORT int ra_lt_choice_is_streamk(int ta, int tb, long m, long n, long k, long lda,
                                      long ldb, long ldc, int batch, long sa, long sb,
                                      long sc) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_plan(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc);
  if (!p || p->cands.empty()) return -1;
  return cand_sk(p, p->choice) ? 1 : 0;
}

// 1: allow stream-K candidates (only safe when no other stream runs GEMMs concurrently).
// Applies to plans created afterwards and to later tuning / set_choice calls.
RA_EXPORT void ra_lt_allow_streamk(int on) {
  std::lock_guard<std::mutex> g(g_mu);
  g_allow_sk = on != 0;
}

// Drop the handle and workspace cached for a stream that is about to be destroyed (the
// capture stream of a graph, a per-chunk stream, a data actor's stream): without it each
// short-lived stream that ran an lt GEMM keeps a handle and kWs bytes of HBM, and a later
// stream allocated at the same address would silently reuse the stale entry. Work queued on
// the stream is drained first (the workspace may still be read). Returns the entries freed.
RA_EXPORT int ra_lt_release_stream(void* stream) {
  hipStream_t st = (hipStream_t)stream;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  int freed = 0;
  auto w = g_ws_by_stream.find(st);
  auto h = g_handle_by_stream.find(st);
  if (w == g_ws_by_stream.end() && h == g_handle_by_stream.end()) return 0;
  hipStreamSynchronize(st);
  if (w != g_ws_by_stream.end()) {
    hipFree(w->second);
    g_ws_by_stream.erase(w);
    ++freed;
  }
  if (h != g_handle_by_stream.end()) {
    if (h->second != g_handle) hipblasLtDestroy(h->second);
    g_handle_by_stream.erase(h);
    ++freed;
  }
  return freed;
}

RA_EXPORT int ra_lt_num_streams() {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  return (int)(g_ws_by_stream.size() > g_handle_by_stream.size() ? g_ws_by_stream.size()
                                                                   : g_handle_by_stream.size());
}

// ----------------------------------------------------------------- epilogue GEMMs
// D (bf16) = epilogue(op(A) * op(B)) for the fused MLP: GELU_AUX_BIAS (forward: D = gelu(AB +
// bias), aux = AB + bias) and DGELU_BGRAD (backward: D = AB * gelu'(aux), bias = colsum(D)).
// Epilogue pointers are per-call descriptor attributes; plans are cached per shape + epilogue.
namespace {
typedef std::tuple<int, int, long, long, long, long, long, long, int, long> EpKey;
std::map<EpKey, LtPlan*> g_ep_plans;

LtPlan* get_ep_plan(int ta, int tb, long m, long n, long k, long lda, long ldb, long ldd, int ep,
                    long ldaux) {
  const EpKey key(ta, tb, m, n, k, lda, ldb, ldd, ep, ldaux);
  auto it = g_ep_plans.find(key);
  if (it != g_ep_plans.end()) return it->second;
  if (init_handle() != 0) return nullptr;
  LtPlan* p = new LtPlan();
  hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
  uint32_t e = (uint32_t)ep;
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  // bias: bf16 input for GELU_AUX_BIAS, fp32 output for DGELU_BGRAD
  int32_t bt = ep == HIPBLASLT_EPILOGUE_DGELU_BGRAD ? HIP_R_32F : HIP_R_16BF;
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  int64_t la = ldaux;
  hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &la, sizeof(la));
  hipblasLtMatrixLayoutCreate(&p->a, HIP_R_16BF, ta ? k : m, ta ? m : k, lda);
  hipblasLtMatrixLayoutCreate(&p->b, HIP_R_16BF, tb ? n : k, tb ? k : n, ldb);
  hipblasLtMatrixLayoutCreate(&p->c, HIP_R_16BF, m, n, ldd);
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wsz = kWs;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz,
                                        sizeof(wsz));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(64);
  int got = 0;
  hipblasLtMatmulAlgoGetHeuristic(g_handle, p->desc, p->a, p->b, p->c, p->c, pref, 64,
                                  res.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  for (int i = 0; i < got; ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= kWs)
      p->cands.push_back(res[i]);
  g_ep_plans[key] = p;
  return p;
}
}  // namespace

// Candidates for an epilogue GEMM (0 = unsupported on this hipBLASLt / arch).
RA_EXPORT int ra_lt_ep_num_cands(int ta, int tb, long m, long n, long k, long lda, long ldb,
                                 long ldd, int ep, long ldaux) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_ep_plan(ta, tb, m, n, k, lda, ldb, ldd, ep, ldaux);
  return p ? (int)p->cands.size() : -1;
}

RA_EXPORT int ra_lt_ep_set_choice(int ta, int tb, long m, long n, long k, long lda, long ldb,
                                  long ldd, int ep, long ldaux, int choice) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_ep_plan(ta, tb, m, n, k, lda, ldb, ldd, ep, ldaux);
  if (!p || choice < 0 || choice >= (int)p->cands.size()) return -1;
  p->choice = choice;
  return 0;
}

// choice < 0: the plan's current choice. D may alias nothing else; aux is read (DGELU) or
// written (GELU_AUX); bias is read (GELU_AUX_BIAS, bf16) or written (DGELU_BGRAD, fp32).
RA_EXPORT int ra_lt_gemm_ep(int ta, int tb, long m, long n, long k, const void* A, long lda,
                            const void* B, long ldb, void* D, long ldd, int ep, void* bias,
                            void* aux, long ldaux, int choice, hipStream_t st) {
  LtPlan* p;
  {
    std::lock_guard<std::mutex> g(g_mu);
    p = get_ep_plan(ta, tb, m, n, k, lda, ldb, ldd, ep, ldaux);
    if (!p || p->cands.empty()) return -1;
    hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                    sizeof(bias));
    hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux,
                                    sizeof(aux));
  }
  const int idx = choice >= 0 && choice < (int)p->cands.size() ? choice : p->choice;
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t s =
      hipblasLtMatmul(handle_for(st), p->desc, &alpha, A, p->a, B, p->b, &beta, D, p->c, D,
                      p->c, &p->cands[idx].algo, workspace(st), kWs, st);
  return s == HIPBLAS_STATUS_SUCCESS ? 0 : 1000 + (int)s;
}

// Time every candidate (beta = 0 into `scratch`: the C footprint), keep the
// fastest as the shape's choice. Returns its index; *best_ms gets its time.
RA_EXPORT int ra_lt_tune(int ta, int tb, long m, long n, long k, const void* A, long lda,
                         const void* B, long ldb, float* scratch, long ldc, int iters,
                         float* best_ms, int batch, long sa, long sb, long sc, hipStream_t st) {
  std::lock_guard<std::mutex> g(g_mu);
  LtPlan* p = get_plan(ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc);
  if (!p || p->cands.empty()) return -1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int best = -1;
  float bt = 1e30f;
  for (int i = 0; i < (int)p->cands.size(); ++i) {
    if (!usable(p, i)) continue;
    if (run(p, i, A, B, scratch, 1.f, 0.f, st) != 0) continue;  // warmup / validity
    hipEventRecord(e0, st);
    bool ok = true;
    for (int r = 0; r < iters && ok; ++r) ok = run(p, i, A, B, scratch, 1.f, 0.f, st) == 0;
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (ok && ms / iters < bt) {
      bt = ms / iters;
      best = i;
    }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (best >= 0) p->choice = best;
  if (best_ms) *best_ms = bt;
  return best;
}
