// mccp2.hip -- MCCompletePathV2 (include/mccompletepathv2.h:182-258) on the MI355X.
//
// The reference walks nodes in executionOrder (:209) and builds each node's basket
//     S[v] = topL( {v: 1/f} + sum_{s in succ(v), in order} X[s] ) * f,     f = d / deg(v)
// where X[s] is s's final basket when s came earlier in the order and otherwise the basket of
// R random walks from s, computed once, the first time it is needed (:228-241). Dangling nodes
// get {v: 1.0} (f = 1). Which X a predecessor reads is fixed by the order alone:
//     edge v -> s reads the final basket  iff  pos(s) < pos(v),
// so the whole computation is restated without sequential state:
//   1. host: executionOrder (ppr_execution_order_csr), per-edge read-slot bit, the walk set
//      W = { s : some edge v -> s with pos(s) >= pos(v) }, and combine levels
//      level(v) = 1 + max level over v's final-basket successors (dangling nodes: none);
//   2. k_mc_walk over W (one wave per node, Philox walks, merge_mc.h) -> slab slot 1;
//   3. dangling finals {v: 1.0} -> slot 0; then level by level the GRank merge tiers in MC mode
//      (seed 1/f, plain `+=` order, keepTop(L) then * f) -> slot 0;
//   4. final keepTop(K) = the first K entries of each sorted row (k_topk).
// Levels run in order and a level only reads slot-0 rows of lower levels and slot-1 rows, so the
// result equals the reference's sequential sweep given the same walk baskets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "plan.h"
#include "merge_mc.h"

namespace {
int mc_table_slots(uint32_t L) {
  return pow2_at_least(((int64_t)L + 64) * 3 / 2);
}
}  // namespace

extern "C" int ppr_mccp2_plan_create(const ppr_csr* g, uint32_t K, uint32_t L, double damping,
                                     const ppr_opts* o, ppr_plan** out) {
  if (!g || !out || g->n < 0 || (g->n > 0 && !g->row_ptr)) return PPR_ERR_ARG;
  if (g->n > 0 && g->row_ptr[g->n] > 0 && !g->col) return PPR_ERR_ARG;
  int rc = check_params(K, L, 1, damping);
  if (rc != PPR_OK) return rc;
  if (L > (uint32_t)MAX_L) return PPR_ERR_RANGE;
  if (g->n >= (1LL << 31) - 1) return PPR_ERR_RANGE;
  const int64_t n = g->n;
  const int64_t m = n ? g->row_ptr[n] : 0;
  const int64_t* rp = g->row_ptr;
  for (int64_t e = 0; e < m; e++)
    if (g->col[e] < 0 || g->col[e] >= n) return PPR_ERR_GRAPH;
  std::vector<int32_t> order(n > 0 ? n : 1);
  if (n) { rc = ppr_execution_order_csr(g, order.data()); if (rc) return rc; }
  std::vector<int32_t> pos(n > 0 ? n : 1);
  for (int64_t i = 0; i < n; i++) pos[order[i]] = (int32_t)i;

  std::vector<int32_t> colx(m > 0 ? m : 1);
  std::vector<uint8_t> inW(n > 0 ? n : 1, 0);
  for (int64_t v = 0; v < n; v++)
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) {
      const int32_t s = g->col[e];
      const bool walk = pos[s] >= pos[v];
      colx[e] = s | (walk ? (int32_t)0x80000000 : 0);
      if (walk) inW[s] = 1;
    }
  // combine levels in execution order (final-basket successors come earlier)
  std::vector<int32_t> level(n > 0 ? n : 1, -1);
  int32_t maxlev = -1;
  for (int64_t i = 0; i < n; i++) {
    const int32_t v = order[i];
    if (rp[v + 1] == rp[v]) continue;  // dangling: no combine
    int32_t lv = 0;
    for (int64_t e = rp[v]; e < rp[v + 1]; e++)
      if (colx[e] >= 0) lv = std::max(lv, level[colx[e]] + 1);
    level[v] = lv;
    maxlev = std::max(maxlev, lv);
  }
  ppr_plan* p = nullptr;
  rc = plan_alloc(n, rp, colx.data(), K, L, damping, o, &p, true);
  if (rc) return rc;
  p->mc = true;
  std::vector<int64_t> off(maxlev + 2, 0);
  std::vector<int32_t> walk, dang;
  for (int64_t v = 0; v < n; v++) {
    if (level[v] >= 0) off[level[v] + 1]++;
    else dang.push_back((int32_t)v);
    if (inW[v]) walk.push_back((int32_t)v);
  }
  for (int32_t l = 0; l <= maxlev; l++) off[l + 1] += off[l];
  std::vector<int32_t> byl(off[maxlev + 1] > 0 ? off[maxlev + 1] : 1);
  {
    std::vector<int64_t> fill(off.begin(), off.end() - 1);
    for (int64_t i = 0; i < n; i++) {  // execution order inside a level
      const int32_t v = order[i];
      if (level[v] >= 0) byl[fill[level[v]]++] = v;
    }
  }
  p->mc_level_off = off;
  p->mc_nwalk = (int64_t)walk.size();
  p->mc_ndangling = (int64_t)dang.size();
  p->mc_T = mc_table_slots(L);
  TRY(dalloc(&p->d_mc_walk, walk.size()));
  TRY(dalloc(&p->d_mc_levels, byl.size()));
  TRY(dalloc(&p->d_mc_dangling, dang.size()));
  hipStream_t st = p->stream;
  if ((!walk.empty() && hipMemcpyAsync(p->d_mc_walk, walk.data(), 4 * walk.size(), hipMemcpyHostToDevice, st) != hipSuccess) ||
      (off[maxlev + 1] > 0 && hipMemcpyAsync(p->d_mc_levels, byl.data(), 4 * (size_t)off[maxlev + 1], hipMemcpyHostToDevice, st) != hipSuccess) ||
      (!dang.empty() && hipMemcpyAsync(p->d_mc_dangling, dang.data(), 4 * dang.size(), hipMemcpyHostToDevice, st) != hipSuccess) ||
      hipStreamSynchronize(st) != hipSuccess) {
    plan_free(p);
    return PPR_ERR_HIP;
  }
  const size_t lds = mc_wave_lds(p->mc_T);
  if (lds > 160 * 1024) { plan_free(p); return PPR_ERR_RANGE; }
  if (lds > 64 * 1024)
    hipFuncSetAttribute((const void*)k_mc_walk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  *out = p;
  return PPR_OK;
}

extern "C" int ppr_mccp2_plan_info(ppr_plan* p, int64_t* walk_nodes, int64_t* levels, int64_t* dangling) {
  if (!p || !p->mc) return PPR_ERR_ARG;
  if (walk_nodes) *walk_nodes = p->mc_nwalk;
  if (levels) *levels = (int64_t)p->mc_level_off.size() - 1;
  if (dangling) *dangling = p->mc_ndangling;
  return PPR_OK;
}

extern "C" int ppr_mccp2_plan_walk(ppr_plan* p, uint32_t walks, uint64_t seed, int64_t begin, int64_t end) {
  if (!p || !p->mc) return PPR_ERR_ARG;
  if (walks == 0) return PPR_ERR_ITERS;
  begin = std::max<int64_t>(0, begin);
  end = std::min<int64_t>(p->mc_nwalk, end);
  if (end <= begin) return PPR_OK;
  HIP_OK(hipSetDevice(p->device));
  McArgs m;
  m.R = walks;
  // walks = static_cast<size_t>(static_cast<double>(walks) * damping) (:132)
  m.nw = (uint64_t)((double)walks * p->damping);
  m.damping = p->damping;
  m.seed = seed;
  m.T = p->mc_T;
  m.slot = 1;
  DevGraph g{p->d_rp, p->d_colx, p->n};
  const DevSlab s = dev_slab(p);
  HIP_OK(hipEventRecord(p->ev_m0, p->stream));
  hipLaunchKernelGGL(k_mc_walk, dim3((unsigned)(end - begin)), dim3(64), mc_wave_lds(p->mc_T), p->stream, g, s, m,
                     p->d_mc_walk + begin, end - begin);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(p->ev_m1, p->stream));
  HIP_OK(hipEventSynchronize(p->ev_m1));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, p->ev_m0, p->ev_m1));
  p->mc_walk_ms += ms;
  p->mc_walks += (int64_t)m.nw * (end - begin);
  return PPR_OK;
}

extern "C" int ppr_mccp2_plan_combine(ppr_plan* p) {
  if (!p || !p->mc) return PPR_ERR_ARG;
  if (p->n == 0) return PPR_OK;
  HIP_OK(hipSetDevice(p->device));
  const DevSlab s = dev_slab(p);
  if (p->mc_ndangling) {
    hipLaunchKernelGGL(k_mc_selfrow, dim3((unsigned)((p->mc_ndangling + 3) / 4)), dim3(256), 0, p->stream, s,
                       p->d_mc_dangling, p->mc_ndangling, 0);
    HIP_OK(hipGetLastError());
  }
  IterArgs a;
  a.sA = 0;       // colx bit 0: final basket (slot 0)
  a.sB = 1;       // colx bit 1: random-walk basket (slot 1)
  a.active = 0;
  a.damping = p->damping;
  a.unit = 0u;
  a.stats = (p->flags & PPR_FLAG_STATS) ? 1u : 0u;
  a.mc = 1u;
  // the reference's order (include/mccompletepathv2.h:228-240) by default; PPR_MC_SUM=exact: the
  // order-free exact sum with 72 fraction bits (merge_xs.h XS_F_MC)
  a.xs = p->xsum ? 1u : 0u;
  a.xsf = XS_F_MC;
  a.rp = p->d_rp;
  a.diag = p->d_diag;
  a.lds_rank = p->lds_rank;
  a.nt = (uint32_t)p->nt_loads;
  a.whatif = ((uint32_t)p->whatif & 0xffffu) | (p->rank_permute ? WI_RANK_PERMUTE : 0u);
  a.iter = -1;
  a.spec = 0.0;
  const int64_t nl = (int64_t)p->mc_level_off.size() - 1;
  HIP_OK(hipEventRecord(p->ev_m0, p->stream));
  p->ovl_pending = nullptr;
  const bool lvlog = getenv("PPR_MC_LEVEL_LOG") != nullptr;  // diagnostics: one line per level
  for (int64_t l = 0; l < nl; l++) {
    const int64_t b = p->mc_level_off[l], e = p->mc_level_off[l + 1];
    if (lvlog) { HIP_OK(hipEventRecord(p->ev_a, p->stream)); p->last_nbig = p->last_maxneed = 0; }
    int rc = run_merge(p, a, p->d_mc_levels + b, e - b, p->d_maxdiff + PPR_MAX_ITER_STATS);
    if (rc) return rc;
    if (lvlog) {
      HIP_OK(hipEventRecord(p->ev_b, p->stream));
      HIP_OK(hipEventSynchronize(p->ev_b));
      float ms = 0.f;
      hipEventElapsedTime(&ms, p->ev_a, p->ev_b);
      fprintf(stderr, "mc_level %lld %lld %lld %lld %.4f\n", (long long)l, (long long)(e - b),
              (long long)p->last_nbig, (long long)p->last_maxneed, ms);
    }
  }
  {  // a level's hub overflow list is read with the next level's classification; the last one here
    int rc = run_merge_flush(p, a, p->d_maxdiff + PPR_MAX_ITER_STATS);
    if (rc) return rc;
  }
  HIP_OK(hipEventRecord(p->ev_m1, p->stream));
  HIP_OK(hipEventSynchronize(p->ev_m1));
  {
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, p->ev_m0, p->ev_m1));
    p->merge_ms += ms;
  }
  // final keepTop(K) (:252-256): prefix of every row in slot 0
  {
    const int rc = launch_topk(p, 0, 0);
    if (rc) return rc;
  }
  // bounded probes: the combine's merge kernels (grank.hip's word) and the walks (this module's)
  {
    const int rc = probe_take();
    if (rc) return rc;
  }
  unsigned int v = 0u;
  HIP_OK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_probe_err), sizeof(v), 0, hipMemcpyDeviceToHost));
  if (v) {
    const unsigned int z = 0u;
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe_err), &z, sizeof(z), 0, hipMemcpyHostToDevice));
    return PPR_ERR_PROBE;
  }
  return PPR_OK;
}

extern "C" int ppr_mccp2_plan_run(ppr_plan* p, uint32_t walks, uint64_t seed, ppr_mc_stats* st) {
  if (!p || !p->mc) return PPR_ERR_ARG;
  if (walks == 0) return PPR_ERR_ITERS;
  HIP_OK(hipSetDevice(p->device));
  hipStream_t s = p->stream;
  HIP_OK(hipMemsetAsync(p->d_stats, 0, 8 * PPR_NSTATS, s));
  p->merge_launches = 0;
  p->merge_ms = 0.0;
  p->mc_walk_ms = 0.0;
  p->mc_walks = 0;
  HIP_OK(hipEventRecord(p->ev_a, s));
  int rc = ppr_mccp2_plan_walk(p, walks, seed, 0, p->mc_nwalk);
  if (rc) return rc;
  rc = ppr_mccp2_plan_combine(p);
  if (rc) return rc;
  HIP_OK(hipEventRecord(p->ev_b, s));
  HIP_OK(hipEventSynchronize(p->ev_b));
  if (st) {
    std::memset(st, 0, sizeof(*st));
    float ms = 0;
    hipEventElapsedTime(&ms, p->ev_a, p->ev_b);
    st->device_ms = ms;
    st->walk_ms = p->mc_walk_ms;
    st->combine_ms = p->merge_ms;
    st->walk_nodes = p->mc_nwalk;
    st->walks = p->mc_walks;
    st->levels = (int64_t)p->mc_level_off.size() - 1;
    st->merge_launches = p->merge_launches;
    unsigned long long sv[2];
    HIP_OK(hipMemcpyAsync(sv, p->d_stats, 16, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    st->candidates = (int64_t)sv[0];
    st->algo_bytes = (int64_t)sv[1];
  }
  return PPR_OK;
}

extern "C" int ppr_plan_fetch_slot(ppr_plan* p, int32_t slot, int32_t* ids, double* scores, int32_t* len) {
  // raw slab slot (rows of width L; only the first len[v] entries of a row are meaningful)
  if (!p || slot < 0 || slot > 1) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  hipStream_t st = p->stream;
  HIP_OK(hipStreamSynchronize(st));
  const size_t nl = (size_t)p->n * p->L;
  if (ids && nl) HIP_OK(hipMemcpyAsync(ids, p->d_ids + (size_t)slot * nl, 4 * nl, hipMemcpyDeviceToHost, st));
  if (scores && nl) HIP_OK(hipMemcpyAsync(scores, p->d_sc + (size_t)slot * nl, 8 * nl, hipMemcpyDeviceToHost, st));
  if (len && p->n) HIP_OK(hipMemcpyAsync(len, p->d_len + (size_t)slot * p->n, 4 * (size_t)p->n, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  return PPR_OK;
}

extern "C" int ppr_mccp2_csr(const ppr_csr* g, uint32_t K, uint32_t L, uint32_t walks, double damping,
                             uint64_t seed, const ppr_opts* o, int32_t* out_ids, double* out_scores,
                             int32_t* out_len, ppr_mc_stats* st) {
  int rc = check_params(K, L, walks, damping);
  if (rc) return rc;
  if (!g) return PPR_ERR_ARG;
  if (g->n == 0) { if (st) std::memset(st, 0, sizeof(*st)); return PPR_OK; }
  ppr_plan* p = nullptr;
  rc = ppr_mccp2_plan_create(g, K, L, damping, o, &p);
  if (rc) return rc;
  rc = ppr_mccp2_plan_run(p, walks, seed, st);
  if (!rc) rc = ppr_grank_plan_fetch(p, out_ids, out_scores, out_len);
  ppr_grank_plan_destroy(p);
  return rc;
}
