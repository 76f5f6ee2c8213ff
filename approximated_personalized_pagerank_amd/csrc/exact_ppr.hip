// exact_ppr.hip -- batched exact single-source PPR on the GPU: the quality
// oracle of the reference's benchmark harness, pprSingleSource (include/internal/
// pprSingleSource.h:28-75, called as pprSingleSource(graph, 100, .85, 1e-4, node) by
// benchmarkAlgorithm, include/benchmarkAlgorithm.h:91), for S sources at once.
//
// Per source s, iteration i (while i < iterations and diff_s >= tol, diff_s starting at tol):
//     next = {src_s: 1-d};  next[u] += score[v] * d/deg(v)  for every edge v -> u with v scored;
//     diff_s = norm1(score, next);  score = next
// Mass reaching a dangling node stays there (the reference does not redistribute it).
//
// Layout: scores are dense, node-major X[n][S] (the S values of a node contiguous), so the pull
// over the transposed graph -- y[u][s] = [u == src_s](1-d) + sum_{v -> u} x[v][s] * d/deg(v) --
// reads every predecessor's S values as one coalesced run: per iteration m * S * 8 bytes, an
// SpMM with a skinny dense operand, HBM bound. The reference sums a node's contributions in its
// unordered_map order; here they are summed in predecessor (CSR-of-transpose) order with fma, so
// scores agree to rounding (<= 1e-12, tests/test_gpu_exact.py), not bit for bit. Absent keys of
// the reference's maps are the zero entries here (a key reached with exactly 0 is lost only
// when d = 0).
//
// diff_s is reduced deterministically (per-wave partials, then a fixed-order sum), so the stop
// iteration of every source is reproducible run to run. A converged source's column is copied
// through unchanged. keepTop(K) of each column uses the engine's top-L tie rule (ppr_device.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/ppr_hip.h"
#include "plan.h"
#include "wg_merge.h"

namespace pprk {

constexpr int EX_WAVES = 4096;  // waves of the pull grid (grid-stride over targets)

struct ppr_exact_impl {
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t n = 0, m = 0;
  int S = 0;
  double damping = 0.85;
  int64_t* d_rpt = nullptr;     // transposed CSR: predecessors of every node
  int32_t* d_colt = nullptr;
  double* d_f = nullptr;        // d / deg(v) (0 for a dangling v, which has no out-edges)
  int32_t* d_src = nullptr;     // [S]
  double* d_x = nullptr;        // [n][S] current scores
  double* d_y = nullptr;        // [n][S] next scores
  double* d_part = nullptr;     // [EX_WAVES][S] per-wave norm1 partials
  double* d_diff = nullptr;     // [S]
  int32_t* d_act = nullptr;     // [S] 1 while the source iterates
  int32_t* d_iters = nullptr;   // [S] iterations run
  int32_t* d_nact = nullptr;    // sources still iterating
};

__global__ void __launch_bounds__(256) k_exact_init(double* x, int64_t n, int S, const int32_t* src, int32_t* act,
                                                    int32_t* iters, double* diff, double tol) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * S) x[i] = 0.0;
  if (i < S) { act[i] = 1; iters[i] = 0; diff[i] = tol; }
}

__global__ void __launch_bounds__(256) k_exact_seed(double* x, int S, const int32_t* src) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < S) x[(int64_t)src[s] * S + s] = 1.0;  // scores = {src: 1.0}
}

// one wave per target node per step (grid-stride), lanes over sources
__global__ void __launch_bounds__(256) k_exact_pull(const int64_t* rpt, const int32_t* colt, const double* f,
                                                    const int32_t* src, const int32_t* act, const double* x,
                                                    double* y, double* part, int64_t n, int S, double damping) {
  const int wv = threadIdx.x >> 6, l = lane_id();
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int s0 = 0; s0 < S; s0 += WAVE) {
    const int s = s0 + l;
    const bool on = s < S && act[s];
    const int mysrc = s < S ? src[s] : -1;
    double dpart = 0.0;
    for (int64_t u = gw; u < n; u += nw) {
      if (s >= S) continue;
      const double old = x[u * S + s];
      if (!on) { y[u * S + s] = old; continue; }  // converged: carried through
      double acc = (u == mysrc) ? 1.0 - damping : 0.0;
      const int64_t b = rpt[u], e = rpt[u + 1];
      for (int64_t k = b; k < e; k++) {
        const int v = colt[k];
        acc = fma(x[(int64_t)v * S + s], f[v], acc);
      }
      y[u * S + s] = acc;
      dpart += fabs(acc - old);
    }
    if (s < S) part[gw * S + s] = dpart;
  }
}

// diff_s = sum of the per-wave partials in wave order; a source stops once diff < tol
// (include/internal/pprSingleSource.h:47, 68-71)
__global__ void __launch_bounds__(256) k_exact_reduce(const double* part, int nwaves, int S, double tol,
                                                      double* diff, int32_t* act, int32_t* iters, int32_t* nact) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S || !act[s]) return;
  double t = 0.0;
  for (int w = 0; w < nwaves; w++) t += part[(int64_t)w * S + s];
  diff[s] = t;
  iters[s]++;
  if (t >= tol) atomicAdd(nact, 1);
  else act[s] = 0;
}

// keepTop(K) of source s's column (nonzero entries), by the top-L tie rule; out rows by (score
// desc, id asc)
__global__ void __launch_bounds__(WG_THREADS) k_exact_topk(const double* x, int64_t n, int S, const int32_t* src, int K,
                                                           int Kp, int32_t* out_ids, double* out_sc, int32_t* out_len) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int s = blockIdx.x;
  const WgLds L = wg_carve(smem, 0, Kp, 0);
  const uint32_t ts = tie_salt(src[s]);
  auto val = [&](int64_t i) { return x[i * S + s]; };
  auto occ = [&](int i) { return val(i) != 0.0; };
  if (threadIdx.x == 0) L.misc[M_PLEN] = 0;
  __syncthreads();
  int cnt = 0;
  for (int64_t i = threadIdx.x; i < n; i += WG_THREADS) cnt += occ((int)i);
  cnt = wave_sum(cnt);
  if (lane_id() == 0) atomicAdd(&L.misc[M_PLEN], cnt);
  __syncthreads();
  const int nz = L.misc[M_PLEN];
  __syncthreads();
  if (threadIdx.x == 0) L.misc[M_PLEN] = 0;
  __syncthreads();
  if (nz <= K) {
    for (int64_t i = threadIdx.x; i < n; i += WG_THREADS)
      if (occ((int)i)) { const int p = atomicAdd(&L.misc[M_PLEN], 1); L.rv[p] = dbits(val(i)); L.rk[p] = (int)i; }
  } else {
    const SelCrit c = wg_select_top(L, (int)n, K, [&](int i) { return i; }, [&](int i) { return val(i); }, occ, ts);
    for (int64_t i = threadIdx.x; i < n; i += WG_THREADS) {
      if (!occ((int)i)) continue;
      const double v = val(i);
      if (sel_test(c, dbits(v), tie_w((int)i, ts))) {
        const int p = atomicAdd(&L.misc[M_PLEN], 1);
        L.rv[p] = dbits(v);
        L.rk[p] = (int)i;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < WAVE) {
    const int c = L.misc[M_PLEN];
    row_sort(L.rv, L.rk, c, Kp);
    for (int i = lane_id(); i < K; i += WAVE) {
      out_ids[(int64_t)s * K + i] = i < c ? L.rk[i] : -1;
      out_sc[(int64_t)s * K + i] = i < c ? bitsd(L.rv[i]) : 0.0;
    }
    if (lane_id() == 0) out_len[s] = c;
  }
}

__global__ void __launch_bounds__(256) k_exact_gather(const double* x, int64_t n, int S, int Q, const int32_t* keys,
                                                      double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)S * Q) return;
  const int s = (int)(i / Q);
  const int k = keys[i];
  out[i] = (k >= 0 && k < n) ? x[(int64_t)k * S + s] : 0.0;
}

}  // namespace pprk

using namespace pprk;

struct ppr_exact : ppr_exact_impl {};

static void exact_free(ppr_exact* h) {
  if (!h) return;
  hipFree(h->d_rpt); hipFree(h->d_colt); hipFree(h->d_f); hipFree(h->d_src); hipFree(h->d_x); hipFree(h->d_y);
  hipFree(h->d_part); hipFree(h->d_diff); hipFree(h->d_act); hipFree(h->d_iters); hipFree(h->d_nact);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
}

#define EX_TRY(x) do { if ((x) != hipSuccess) { exact_free(h); return PPR_ERR_HIP; } } while (0)
#define EX_ALLOC(p, cnt) do { if (hipMalloc((void**)&(p), sizeof(*(p)) * std::max<size_t>(1, (size_t)(cnt))) != hipSuccess) { exact_free(h); return PPR_ERR_OOM; } } while (0)

extern "C" int ppr_exact_create(const ppr_csr* g, const int32_t* sources, int32_t S, double damping,
                                const ppr_opts* o, ppr_exact** out) {
  if (!g || !out || !sources || S <= 0 || g->n <= 0 || !g->row_ptr) return PPR_ERR_ARG;
  if (damping < 0 || damping > 1) return PPR_ERR_DAMPING;
  const int64_t n = g->n, m = g->row_ptr[n];
  if (m > 0 && !g->col) return PPR_ERR_ARG;
  for (int32_t s = 0; s < S; s++)
    if (sources[s] < 0 || sources[s] >= n) return PPR_ERR_SOURCE;
  for (int64_t e = 0; e < m; e++)
    if (g->col[e] < 0 || g->col[e] >= n) return PPR_ERR_GRAPH;
  ppr_exact* h = new (std::nothrow) ppr_exact();
  if (!h) return PPR_ERR_OOM;
  h->n = n; h->m = m; h->S = S; h->damping = damping;
  h->device = (o && o->device >= 0) ? o->device : 0;
  EX_TRY(hipSetDevice(h->device));
  EX_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  // transposed CSR on the host: predecessors of u in increasing source order
  std::vector<int64_t> rpt(n + 1, 0);
  std::vector<int32_t> colt(m > 0 ? m : 1);
  std::vector<double> f(n);
  for (int64_t e = 0; e < m; e++) rpt[g->col[e] + 1]++;
  for (int64_t u = 0; u < n; u++) rpt[u + 1] += rpt[u];
  {
    std::vector<int64_t> fill(rpt.begin(), rpt.end() - 1);
    for (int64_t v = 0; v < n; v++)
      for (int64_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; e++) colt[fill[g->col[e]]++] = (int32_t)v;
  }
  for (int64_t v = 0; v < n; v++) {
    const int64_t deg = g->row_ptr[v + 1] - g->row_ptr[v];
    f[v] = deg ? damping / (double)deg : 0.0;
  }
  EX_ALLOC(h->d_rpt, n + 1);
  EX_ALLOC(h->d_colt, m);
  EX_ALLOC(h->d_f, n);
  EX_ALLOC(h->d_src, S);
  EX_ALLOC(h->d_x, (size_t)n * S);
  EX_ALLOC(h->d_y, (size_t)n * S);
  EX_ALLOC(h->d_part, (size_t)EX_WAVES * S);
  EX_ALLOC(h->d_diff, S);
  EX_ALLOC(h->d_act, S);
  EX_ALLOC(h->d_iters, S);
  EX_ALLOC(h->d_nact, 1);
  EX_TRY(hipMemcpy(h->d_rpt, rpt.data(), 8 * (n + 1), hipMemcpyHostToDevice));
  if (m) EX_TRY(hipMemcpy(h->d_colt, colt.data(), 4 * m, hipMemcpyHostToDevice));
  EX_TRY(hipMemcpy(h->d_f, f.data(), 8 * n, hipMemcpyHostToDevice));
  EX_TRY(hipMemcpy(h->d_src, sources, 4 * (size_t)S, hipMemcpyHostToDevice));
  *out = h;
  return PPR_OK;
}

extern "C" void ppr_exact_destroy(ppr_exact* h) { exact_free(h); }

extern "C" int ppr_exact_run(ppr_exact* h, uint32_t iterations, double tolerance, int32_t* iters_run) {
  if (!h) return PPR_ERR_ARG;
  if (iterations == 0) return PPR_ERR_ITERS;  // "iterations must be positive"
  HIP_OK(hipSetDevice(h->device));
  hipStream_t st = h->stream;
  const int64_t ns = h->n * h->S;
  hipLaunchKernelGGL(k_exact_init, dim3((unsigned)((std::max<int64_t>(ns, h->S) + 255) / 256)), dim3(256), 0, st,
                     h->d_x, h->n, h->S, h->d_src, h->d_act, h->d_iters, h->d_diff, tolerance);
  hipLaunchKernelGGL(k_exact_seed, dim3((unsigned)((h->S + 255) / 256)), dim3(256), 0, st, h->d_x, h->S, h->d_src);
  HIP_OK(hipGetLastError());
  for (uint32_t i = 0; i < iterations; i++) {
    HIP_OK(hipMemsetAsync(h->d_nact, 0, 4, st));
    hipLaunchKernelGGL(k_exact_pull, dim3(EX_WAVES / 4), dim3(256), 0, st, h->d_rpt, h->d_colt, h->d_f, h->d_src,
                       h->d_act, h->d_x, h->d_y, h->d_part, h->n, h->S, h->damping);
    hipLaunchKernelGGL(k_exact_reduce, dim3((unsigned)((h->S + 255) / 256)), dim3(256), 0, st, h->d_part, EX_WAVES,
                       h->S, tolerance, h->d_diff, h->d_act, h->d_iters, h->d_nact);
    HIP_OK(hipGetLastError());
    std::swap(h->d_x, h->d_y);  // score.swap(nextScores)
    int32_t nact = 0;
    HIP_OK(hipMemcpyAsync(&nact, h->d_nact, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (nact == 0) break;
  }
  if (iters_run) {
    HIP_OK(hipMemcpyAsync(iters_run, h->d_iters, 4 * (size_t)h->S, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  return PPR_OK;
}

extern "C" int ppr_exact_topk(ppr_exact* h, uint32_t K, int32_t* out_ids, double* out_scores, int32_t* out_len) {
  if (!h || K == 0 || K > (uint32_t)MAX_L || !out_ids || !out_scores || !out_len) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(h->device));
  hipStream_t st = h->stream;
  const int Kp = pow2_at_least(K);
  int32_t* d_ids = nullptr; double* d_sc = nullptr; int32_t* d_len = nullptr;
  if (hipMalloc(&d_ids, 4 * (size_t)h->S * K) != hipSuccess || hipMalloc(&d_sc, 8 * (size_t)h->S * K) != hipSuccess ||
      hipMalloc(&d_len, 4 * (size_t)h->S) != hipSuccess) {
    hipFree(d_ids); hipFree(d_sc); hipFree(d_len);
    return PPR_ERR_OOM;
  }
  const size_t lds = wg_lds_bytes(0, Kp, 0);
  hipFuncSetAttribute((const void*)k_exact_topk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(k_exact_topk, dim3((unsigned)h->S), dim3(WG_THREADS), lds, st, h->d_x, h->n, h->S, h->d_src, (int)K,
                     Kp, d_ids, d_sc, d_len);
  int rc = hipGetLastError() == hipSuccess ? PPR_OK : PPR_ERR_HIP;
  if (!rc && (hipMemcpyAsync(out_ids, d_ids, 4 * (size_t)h->S * K, hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipMemcpyAsync(out_scores, d_sc, 8 * (size_t)h->S * K, hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipMemcpyAsync(out_len, d_len, 4 * (size_t)h->S, hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipStreamSynchronize(st) != hipSuccess))
    rc = PPR_ERR_HIP;
  hipFree(d_ids); hipFree(d_sc); hipFree(d_len);
  return rc;
}

extern "C" int ppr_exact_gather(ppr_exact* h, int32_t Q, const int32_t* keys, double* out) {
  if (!h || Q <= 0 || !keys || !out) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(h->device));
  hipStream_t st = h->stream;
  const size_t cnt = (size_t)h->S * Q;
  int32_t* d_k = nullptr; double* d_o = nullptr;
  if (hipMalloc(&d_k, 4 * cnt) != hipSuccess || hipMalloc(&d_o, 8 * cnt) != hipSuccess) {
    hipFree(d_k); hipFree(d_o);
    return PPR_ERR_OOM;
  }
  int rc = PPR_OK;
  if (hipMemcpyAsync(d_k, keys, 4 * cnt, hipMemcpyHostToDevice, st) != hipSuccess) rc = PPR_ERR_HIP;
  if (!rc) {
    hipLaunchKernelGGL(k_exact_gather, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, h->d_x, h->n, h->S, Q, d_k,
                       d_o);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(out, d_o, 8 * cnt, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      rc = PPR_ERR_HIP;
  }
  hipFree(d_k); hipFree(d_o);
  return rc;
}
