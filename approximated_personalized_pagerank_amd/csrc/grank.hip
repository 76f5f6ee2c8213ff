// grank.hip -- MI355X (gfx950) GRank engine: basket-merge kernels + the C ABI of include/ppr_hip.h.
//
// Hot path: for every active source v of the iteration's partition
//     B'[v] = topL( {v: 1-d} (+) sum_{u in succ(v), in order} (d/deg v) * B[u] )
// (reference include/grank.h:96-126, header-only/grankMulti.h:230-268), followed by
// maxDiff = max_v norm1(B'[v], B[v]) (include/grank.h:123).
//
// HBM layout (DESIGN.md "data layout"):
//   rp   int64 [n+1]        CSR row pointers (dense ids = graph iteration order)
//   colx int32 [m]          successor id | partition-of-successor << 31
//   ids  int32 [2][n][L]    basket slab, two slots per node (ping-pong per partition)
//   sc   f64   [2][n][L]
//   len  int32 [2][n]
// A node of partition p has been updated upd(p,it) = p ? it/2 : (it+1)/2 times before
// iteration `it`; its current basket lives in slot upd & 1, an active node writes slot upd^1.
// Nothing is copied for the inactive partition (include/grank.h:133-134 becomes a slot choice).
//
// Kernels per iteration:
//   k_classify    one wave per active source: C_v = sum len[u] -> tier lists (LDS table size)
//   k_merge_lds   one wave per source, LDS hash table sized by tier, owner-round accumulation in
//                 successor order, radix top-L select, bitonic row sort, norm1, write row
//   k_merge_glb   sources whose candidates exceed the largest LDS tier: same algorithm with the
//                 table in HBM scratch, one successor basket per step (keys unique per basket)
// Init (include/grank.h:64-83) runs the same kernels in UNIT mode: every successor contributes
// the basket {u: 1.0}, and fma(1.0, f, acc) == acc + f reproduces `scores[v][s] += factor`.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/ppr_hip.h"
#include "merge_wave.h"
#include "wg_merge.h"
#include "merge_hub.h"
#include "merge_glb.h"
#include "merge_hot.h"
#include "merge_xs.h"
#include "merge_sv.h"
#include "merge_xm.h"
#include "merge_xg.h"

using namespace pprk;

#include "plan.h"
#include "host_par.h"

namespace pprk {
// Probe of the LDS atomic order chunk_accumulate's `ordered` mode relies on: every lane of a wave
// adds 1 to a counter chosen with heavy collisions; the returned old value must equal the number
// of lower lanes on the same counter, for every collision pattern tried. It runs at the bucket
// waves' own launch shape: the same grid (every CU filled to its LDS limit), the same waves per
// block, the same per-wave LDS footprint and the counters at the same offset inside it (the
// T-slot table, ChunkLds::cnt at 12 T). ok[0] (the 32-bit add ranks: the scatter and the chunked
// bucket accumulation) and ok[1] (the 64-bit CAS / add of the one-shot buckets, below) are probed
// separately: each stays 1 only if no lane of any wave ever disagrees.
__global__ void __launch_bounds__(256) k_probe_lds_rank(int* ok, int trials, int T, int wave_bytes) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6, l = lane_id();
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + (size_t)wv * wave_bytes + (size_t)T * 12);
  int bad = 0;
  for (int t = 0; t < trials; t++) {
    const uint32_t r = hash32(t * 104729u + blockIdx.x * 7919u + wv * 31u + 7u);
    const uint32_t S = 1u << (r % 10);
    for (int i = l; i < T; i += WAVE) cnt[i] = 0;
    wave_fence();
    const uint32_t hl = hash32(r ^ (uint32_t)(l * 2654435761u));
    const uint32_t slot = (hl & (S - 1)) % (uint32_t)T;
    // odd trials: increments 1..4 and a few inactive lanes (the scatter's run heads)
    const uint32_t inc = (t & 1) ? 1u + ((hl >> 12) & 3u) : 1u;
    const bool act = !(t & 1) || ((hl >> 16) & 7u) != 0;
    uint32_t got = 0;
    if (act) got = atomicAdd(&cnt[slot], inc);
    uint32_t want = 0;
    for (int j = 0; j < WAVE; j++) {
      const uint32_t sj = (uint32_t)__shfl((int)slot, j);
      const uint32_t ij = (uint32_t)__shfl((int)inc, j);
      const int aj = __shfl((int)act, j);
      if (j < l && aj && sj == slot) want += ij;
    }
    bad |= act && got != want;
    wave_fence();
  }
  if (bad) atomicAnd(&ok[0], 0);
  bad = 0;
  // (informational since round 5: the round-2 one-shot bucket path relied on the same order for
  // the 64-bit add and the 64-bit CAS on its slot words; the current one needs only the 32-bit add
  // order above. ok[1] is reported by PPR_TIMING as lds_rank64.)
  unsigned long long* w64 = reinterpret_cast<unsigned long long*>(smem + (size_t)wv * wave_bytes);
  for (int t = 0; t < trials; t++) {
    const uint32_t r = hash32(t * 7727u + blockIdx.x * 104723u + wv * 37u + 3u);
    const uint32_t S = 1u << (r % 10);
    for (int i = l; i < T; i += WAVE) w64[i] = 0xffffffffull;
    wave_fence();
    const uint32_t slot = (hash32(r ^ (uint32_t)(l * 2246822519u)) & (S - 1)) % (uint32_t)T;
    const unsigned long long prev = atomicCAS(&w64[slot], 0xffffffffull, (1ull << 32) | (uint32_t)l);
    unsigned long long got = 0;
    if (prev != 0xffffffffull) got = atomicAdd(&w64[slot], 1ull << 32) >> 32;
    uint32_t below = 0;
    for (int j = 0; j < l; j++) below += (uint32_t)__shfl((int)slot, j) == slot;
    if (below == 0) bad |= prev != 0xffffffffull;
    else bad |= (uint32_t)prev == 0xffffffffu || got != below;
    wave_fence();
  }
  if (bad) atomicAnd(&ok[1], 0);
}

}  // namespace pprk

int plan_alloc(int64_t n, const int64_t* row_ptr, const int32_t* colx, uint32_t K, uint32_t L,
               double damping, const ppr_opts* o, ppr_plan** out, bool mc) {
  const int64_t m = n ? row_ptr[n] : 0;
  // per-source candidate counts (<= deg * L + 1) and the hub staging offsets derived from them
  // are 32-bit on the device: reject a graph whose widest source could exceed that
  for (int64_t v = 0; v < n; v++)
    if ((row_ptr[v + 1] - row_ptr[v]) * (int64_t)L + 1 > (int64_t)INT32_MAX) return PPR_ERR_RANGE;
  ppr_plan* p = new (std::nothrow) ppr_plan();
  if (!p) return PPR_ERR_OOM;
  p->n = n; p->m = m; p->K = K; p->L = L; p->damping = damping;
  p->Lp = pow2_at_least(L);
  p->flags = o ? o->flags : 0;
  p->device = (o && o->device >= 0) ? o->device : -1;
  if (p->device >= 0) { if (hipSetDevice(p->device) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; } }
  else { if (hipGetDevice(&p->device) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; } }
  if (o && o->stream) p->stream = (hipStream_t)o->stream;
  else {
    if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
    p->own_stream = true;
  }
  if (hipEventCreate(&p->ev_a) != hipSuccess || hipEventCreate(&p->ev_b) != hipSuccess ||
      hipEventCreate(&p->ev_m0) != hipSuccess || hipEventCreate(&p->ev_m1) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }

  // tiers: T = 256 << t; capacity 3/4 T; a block of 4 waves must fit the 160 KB LDS
  // PPR_TIER_MASK (diagnostics / tests): bit t enables wave tier t, bit NT the workgroup tier;
  // disabled tiers fall through to the next enabled one, ultimately the HBM-table path
  {
    const char* env = getenv("PPR_TIER_MASK");
    const int mask = env ? (int)strtol(env, nullptr, 0) : 0xef;  // workgroup tier off by default
    int T0 = 256;
    for (int t = 0; t < NT; t++) {
      const int T = T0 << t;
      if (!((mask >> t) & 1) || lds_wave_bytes(T, p->Lp) * WAVES_PER_BLOCK > 160 * 1024) { p->tierT[t] = 0; p->tierCap[t] = 0; continue; }
      p->tierT[t] = T;
      p->tierCap[t] = T / 4 * 3;
    }
    // workgroup tier: up to WG_TIER_PASSES key-bucket passes over the slab stream; beyond that
    // the hub pipeline's one partition pass is cheaper than re-reading the stream
    p->tierCap[NT] = 0;
    p->wg_lds = wg_lds_bytes(WG_T, p->Lp, wg_pl(p->Lp));
    const int pmax = WG_TIER_PASSES;
    p->hub_enabled = ((mask >> (NT + 1)) & 1) && pmax >= 1 && p->wg_lds <= 160 * 1024;
    if (((mask >> NT) & 1) && pmax >= 1 && p->wg_lds <= 160 * 1024)
      p->tierCap[NT] = pmax * WG_PASS_CAP;
    // a disabled tier has cap 0 (k_classify skips it); enabled caps must be non-decreasing
    int run = 0;
    for (int t = 0; t <= NT; t++) {
      if (!p->tierCap[t]) continue;
      if (p->tierCap[t] < run) p->tierCap[t] = 0;
      else run = p->tierCap[t];
    }
  }
  // init list: nodes with successors (merged), then the dangling ones (k_init_dangling)
  std::vector<int32_t> all(n > 0 ? n : 1);
  {
    int64_t k = 0;
    for (int64_t v = 0; v < n; v++)
      if (row_ptr[v + 1] > row_ptr[v]) all[k++] = (int32_t)v;
    p->n_nd = k;
    for (int64_t v = 0; v < n; v++)
      if (row_ptr[v + 1] == row_ptr[v]) all[k++] = (int32_t)v;
  }
  p->h_rp.assign(row_ptr, row_ptr + n + 1);
  for (int64_t v = 0; v < n; v++) p->max_deg = std::max<int64_t>(p->max_deg, row_ptr[v + 1] - row_ptr[v]);

  const size_t slab = (size_t)2 * n * L;
  TRY(dalloc(&p->d_rp, n + 1));
  TRY(dalloc(&p->d_colx, m));
  TRY(dalloc(&p->d_part, n));
  TRY(dalloc(&p->d_ids, slab));
  TRY(dalloc(&p->d_sc, slab));
  TRY(dalloc(&p->d_len, 2 * n));
  TRY(dalloc(&p->d_rix, (size_t)2 * n * NRANGE));
  TRY(dalloc(&p->d_rmin, 2 * n));
  TRY(dalloc(&p->d_all, n));
  TRY(dalloc(&p->d_cand, n));
  TRY(dalloc(&p->d_tier_lists, (size_t)NLISTS * (n > 0 ? n : 1)));
  TRY(dalloc(&p->d_tier_cnt, NLISTS + 2));
  TRY(dalloc(&p->d_big, n));
  TRY(dalloc(&p->d_tier_cap, NT + 1));
  TRY(dalloc(&p->d_ovf, n));
  TRY(dalloc(&p->d_maxdiff, PPR_MAX_ITER_STATS + 1));
  TRY(dalloc(&p->d_stats, PPR_NSTATS));
  TRY(dalloc(&p->d_out_ids, (size_t)n * K));
  TRY(dalloc(&p->d_out_sc, (size_t)n * K));
  TRY(dalloc(&p->d_out_len, n));
  if (getenv("PPR_DIAG")) {
    TRY(dalloc(&p->d_diag, PPR_DIAG_SLOTS));
    if (hipMemset(p->d_diag, 0, PPR_DIAG_SLOTS * 8) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
  }
  hipStream_t st = p->stream;
  if (n) {
    if (hipMemcpyAsync(p->d_rp, row_ptr, 8 * (n + 1), hipMemcpyHostToDevice, st) != hipSuccess ||
        (m && hipMemcpyAsync(p->d_colx, colx, 4 * m, hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipMemsetAsync(p->d_part, 0, n, st) != hipSuccess ||
        hipMemsetAsync(p->d_len, 0, 8 * n, st) != hipSuccess ||
        hipMemsetAsync(p->d_rix, 0, sizeof(uint16_t) * 2 * n * NRANGE, st) != hipSuccess ||
        hipMemsetAsync(p->d_rmin, 0, 16 * n, st) != hipSuccess ||
        hipMemcpyAsync(p->d_all, all.data(), 4 * n, hipMemcpyHostToDevice, st) != hipSuccess) {
      plan_free(p); return PPR_ERR_HIP;
    }
  }
  int32_t caps[NT + 1];
  for (int t = 0; t <= NT; t++) caps[t] = p->tierCap[t];
  if (hipMemcpyAsync(p->d_tier_cap, caps, sizeof(caps), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
  for (int t = 0; t < NT; t++)
    if (p->tierT[t]) {
      const size_t bytes = lds_wave_bytes(p->tierT[t], p->Lp) * WAVES_PER_BLOCK;
      if (bytes > 64 * 1024) {
        hipFuncSetAttribute((const void*)k_merge_lds<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_merge_lds<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_merge_lds<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_merge_lds<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      }
    }
  if (p->tierCap[NT])
    hipFuncSetAttribute((const void*)k_merge_wg, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  p->hub_lds_wg = wg_lds_bytes(WG_T, p->Lp, wg_pl(p->Lp));
  p->hub_lds_final = wg_lds_bytes(0, p->Lp, 0);
  {
    const char* e1 = getenv("PPR_HUB_BUCKET");
    const char* e2 = getenv("PPR_HUB_WAVE_T");
    p->hub_bucket = e1 ? std::max(64, atoi(e1)) : (mc ? HUB_BUCKET_MC : HUB_BUCKET);
    p->hub_wave_t = e2 ? (std::max(256, atoi(e2)) + 63) / 64 * 64 : (mc ? HUB_WAVE_T_MC : HUB_WAVE_T);  // a multiple of 64
    p->hub_wave_t = std::min(p->hub_wave_t, 8192);
    // table fill before a bucket spills (a group may bring 64 new keys): PPR_BW_FILL percent
    const char* e17 = getenv("PPR_BW_FILL");
    const int fill = e17 ? std::max(50, std::min(100, atoi(e17))) : 85;  // 448 x 85 %: 380 keys
    p->hub_bw_budget = std::max(WAVE, std::min(p->hub_wave_t, p->hub_wave_t * fill / 100));
  }
  {
    const char* e4 = getenv("PPR_BW_NG");
    const char* e5 = getenv("PPR_BW_WAVES");
    // segmented hub buckets (k_hub_seg): PPR_HUB_SEG=0 disables, PPR_SEG_BUCKET target candidates
    // per bucket, PPR_SEG_T wave table slots, PPR_SEG_WPB waves per block
    const char* s1 = getenv("PPR_HUB_SEG");
    const char* s2 = getenv("PPR_SEG_BUCKET");
    const char* s3 = getenv("PPR_SEG_T");
    const char* s4 = getenv("PPR_SEG_WPB");
    p->seg_enabled = s1 ? atoi(s1) != 0 : false;  // measured no faster than the staged partition

    p->seg_bucket = s2 ? std::max(32, atoi(s2)) : 256;
    p->seg_t = s3 ? pow2_at_least(std::max(256, atoi(s3))) : 512;
    p->seg_t = std::min(p->seg_t, 4096);
    p->seg_wpb = s4 ? std::max(1, std::min(4, atoi(s4))) : 1;
    // two groups per chunk: the smaller chunk staging (vals / touched) buys a wave slot per CU,
    // measured 3 % faster than four groups on RMAT-22
    p->hub_bw_ng = e4 ? (atoi(e4) == 8 ? 8 : atoi(e4) == 4 ? 4 : atoi(e4) == 1 ? 1 : 2) : 2;
    p->hub_bw_waves = e5 ? std::max(1, std::min(4, atoi(e5))) : 1;
    const char* e19 = getenv("PPR_HUB_RANGE");
    if (e19) p->hub_range = std::max(0, std::min(32, atoi(e19)));
    const char* e6 = getenv("PPR_HUB_SLICE");
    p->hub_slice = std::max<int>(std::max<int>(64, (int)L), e6 ? atoi(e6) : HUB_SLICE);
    // k_hub_reduce stages its slice in LDS when it fits beside the select's arrays (PPR_RED_LDS=0: off)
    const char* e21 = getenv("PPR_RED_LDS");
    const size_t red_lds = wg_lds_bytes(0, p->Lp, p->hub_slice);
    p->red_pl = (!(e21 && atoi(e21) == 0) && red_lds <= 160 * 1024) ? p->hub_slice : 0;
    p->hub_lds_red = p->red_pl ? red_lds : p->hub_lds_final;
    if (p->red_pl)
      hipFuncSetAttribute((const void*)k_hub_reduce, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const char* e7 = getenv("PPR_HUB_STREAMS");
    p->hub_streams = (e7 && atoi(e7) == 1) ? 1 : 2;
    const char* e14 = getenv("PPR_WAVE_WPB");
    p->wave_wpb = e14 ? (atoi(e14) >= 4 ? 4 : atoi(e14) >= 2 ? 2 : 1) : 1;
    const char* e15 = getenv("PPR_TILE_WPB_P");
    p->tile_wpb_p = e15 ? std::max(1, atoi(e15)) : 4096;
    const char* e18 = getenv("PPR_HUB_REGIONS");
    p->hub_regions = e18 ? std::max(2, std::min(ppr_plan::MAX_REGIONS, atoi(e18))) : 3;
    const char* e10 = getenv("PPR_HUB_MIX");
    p->hub_mix = e10 ? std::max(0, std::min(HUB_MAX_LOGP, atoi(e10))) : 6;
    const char* e9 = getenv("PPR_HUB_TILE_PB");
    p->hub_tile_pb = e9 ? std::max(0, std::min(64, atoi(e9))) : HUB_TILE_PER_BUCKET;
    const char* e9b = getenv("PPR_HUB_TILE_CAND");
    if (e9b) p->hub_tile_cand = std::max(256, std::min(1 << 20, atoi(e9b)));
    const char* ets = getenv("PPR_TILE_SPLIT_LOGP");  // 12 (HUB_MAX_LOGP): one tile list
    if (ets) p->tile_split_logp = std::max(0, std::min(HUB_MAX_LOGP, atoi(ets)));
    const char* esp = getenv("PPR_SPEC");
    if (esp) p->spec_ratio = std::max(0.0, std::min(1.0, atof(esp)));
    const char* esf = getenv("PPR_SPEC_FROM");
    if (esf) p->spec_from = std::max(0, atoi(esf));
    const char* ent = getenv("PPR_NT");
    if (ent) p->nt_loads = (int)strtol(ent, nullptr, 0) & 3;
    const char* ewi = getenv("PPR_WHATIF");
    if (ewi) p->whatif = (int)strtol(ewi, nullptr, 0);
    const char* ebd = getenv("PPR_WAVE_BY_D");  // exact sum: wave tiers sized by the last distinct-key count
    if (ebd) p->wave_by_d = atoi(ebd) != 0;
    const char* etd = getenv("PPR_WAVE_TDIV");  // tests: wave-tier tables T >> this (bounded probes run out)
    if (etd) p->wave_tdiv = std::max(0, std::min(6, atoi(etd)));
    const char* exr = getenv("PPR_XROUTE");
    if (exr && atoi(exr) == 0) p->xroute = false;
    const char* exb = getenv("PPR_XTEST_BADSIZE");
    if (exb) p->xtest_badsize = atoi(exb);
    const char* erp = getenv("PPR_TEST_RANK_PERMUTE");
    p->rank_permute = erp && atoi(erp) != 0;
    const char* exf = getenv("PPR_XTEST_FAIL");
    if (exf && sscanf(exf, "%d,%d", &p->xtest_fail_rank, &p->xtest_fail_it) != 2) p->xtest_fail_rank = -1;
    const char* ext = getenv("PPR_XTIMEOUT");
    if (ext) p->x_timeout_s = std::max(1.0, atof(ext));
    const char* e9e = getenv("PPR_WG_PASSES");  // tests: force workgroup-tier overflows
    if (e9e) p->wg_max_passes = std::max(1, std::min(WG_MAX_PASSES, atoi(e9e)));
    const char* e9d = getenv("PPR_FUSED_MAX");
    if (e9d) p->fused_max = std::max(0LL, atoll(e9d));
    const char* e9c = getenv("PPR_HUB_LONG_MIN");
    if (e9c) p->hub_long_min = std::max(0LL, atoll(e9c));
    const char* e8 = getenv("PPR_HUB_BUDGET");
    if (e8) p->hub_budget = std::max<int64_t>(1024, std::min<int64_t>(1LL << 28, atoll(e8)));
    // hot pass (merge_hot.h): PPR_HOT_N members (0 = off), built at iteration PPR_HOT_AT from
    // every PPR_HOT_STRIDE-th row
    const char* h1 = getenv("PPR_HOT_N");
    const char* h2 = getenv("PPR_HOT_AT");
    const char* h3 = getenv("PPR_HOT_STRIDE");
    if (h1) p->hot_cap = std::max(0, std::min(16384, atoi(h1)));
    if (h2) p->hot_at = std::max(0, atoi(h2));
    if (h3) p->hot_stride = std::max(1, atoi(h3));
    if (hot_wave_lds(p->hot_cap) > 160 * 1024) p->hot_cap = 0;
    const char* h4 = getenv("PPR_HOT_MAX");
    if (h4) p->hot_max_need = std::max(0, atoi(h4));
  }
  {
    // PPR_BW2=0: no one-shot bucket path (merge_hub.h bucket_oneshot); its table shares the wave's LDS
    const char* e = getenv("PPR_BW2");
    p->hub_bw2 = !(e && atoi(e) == 0);
  }
  p->hub_wave_stride = (int)std::max(hub_wave_lds(p->hub_wave_t, p->hub_bw_ng), p->hub_bw2 ? bw2_lds(p->hub_wave_t) : 0);
  p->hub_lds_wave = (size_t)p->hub_wave_stride * p->hub_bw_waves;
  if (p->hub_streams == 2) {
    // PPR_SV_PRIO=1: stream4 (the sieve's large and small classes) at the highest stream priority
    // (experiment: the large class needs whole CUs and starves beside the wave tier)
    const char* epr = getenv("PPR_SV_PRIO");
    int prio_lo = 0, prio_hi = 0;
    hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    const int prio4 = (epr && atoi(epr) == 1) ? prio_hi : (epr && atoi(epr) == 2) ? prio_lo : 0;
    if (hipStreamCreateWithFlags(&p->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&p->stream4, hipStreamNonBlocking, prio4) != hipSuccess ||
        hipStreamCreateWithFlags(&p->stream3, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&p->ev_wave, hipEventDisableTiming) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
    if (hipStreamCreateWithFlags(&p->stream5, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&p->ev_hot0, hipEventDisableTiming) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
    for (int i = 0; i < ppr_plan::MAX_REGIONS; i++)
      if (hipEventCreateWithFlags(&p->ev_part[i], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&p->ev_buck[i], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&p->ev_fin[i], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&p->ev_hot[i], hipEventDisableTiming) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
  }
  p->stream_wave = p->stream3;
  {
    hipDeviceProp_t prop;
    p->num_cus = hipGetDeviceProperties(&prop, p->device) == hipSuccess ? prop.multiProcessorCount : 256;
    // persistent bucket waves: as many blocks as fit on every CU at once (LDS-bound)
    const int per_cu = std::max<int>(1, std::min<int>(32 / p->hub_bw_waves, (int)((160 * 1024) / p->hub_lds_wave)));
    p->hub_bw_blocks = p->num_cus * per_cu;
  }
  {
    // chunk_accumulate's occurrence ranks from returning LDS atomics need same-address lanes served
    // in lane order: probe it once on this device, fall back to ballot ranks otherwise
    const char* e = getenv("PPR_LDS_RANK");
    int* d_ok = nullptr;
    int ok[2] = {0, 0};
    if ((!e || atoi(e) != 0) && hipMalloc(&d_ok, sizeof(ok)) == hipSuccess) {
      ok[0] = ok[1] = 1;
      if (hipMemcpy(d_ok, ok, sizeof(ok), hipMemcpyHostToDevice) == hipSuccess) {
        hipFuncSetAttribute((const void*)k_probe_lds_rank, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipLaunchKernelGGL(k_probe_lds_rank, dim3((unsigned)p->hub_bw_blocks), dim3(64 * p->hub_bw_waves),
                           p->hub_lds_wave, p->stream, d_ok, 64, p->hub_wave_t,
                           p->hub_wave_stride);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(p->stream) != hipSuccess ||
            hipMemcpy(ok, d_ok, sizeof(ok), hipMemcpyDeviceToHost) != hipSuccess)
          ok[0] = ok[1] = 0;
      } else {
        ok[0] = ok[1] = 0;
      }
      hipFree(d_ok);
    }
    p->lds_rank = ok[0] ? 1u : 0u;
    p->lds_rank64 = ok[1] ? 1u : 0u;
  }
  // exact-sum GRank (merge_xs.h): the default outside the MC combine; PPR_FLAG_CHAIN_SUM or
  // PPR_SUM=chain keep the reference's in-order fma chains (and the hub pipeline of merge_hub.h)
  {
    p->xsum = !mc && !(p->flags & PPR_FLAG_CHAIN_SUM);
    const char* es = getenv("PPR_SUM");
    if (es && !strcmp(es, "chain")) p->xsum = false;
    if (es && !strcmp(es, "exact") && !mc) p->xsum = true;
    // MCCompletePathV2's combine: PPR_MC_SUM=exact sums with the same order-free engines (72 fraction
    // bits, merge_xs.h XS_F_MC; restated by oracle/mc_oracle.c's exact mode)
    const char* em = getenv("PPR_MC_SUM");
    if (mc) p->xsum = em && !strcmp(em, "exact");
    if (mc && p->xsum) {
      // the 96-bit accumulators hold totals below 2^(95 - 72) = 2^23: a combine total is at most
      // the seed 1/f = deg/d plus deg baskets' entries (MC entries stay near 1), so refuse a graph
      // whose widest node could pass it instead of wrapping silently
      // (PPR_MC_XS_LOG2 lowers the limit: tests)
      const char* el = getenv("PPR_MC_XS_LOG2");
      const double lim = std::ldexp(1.0, el ? std::max(1, std::min(23, atoi(el))) : 95 - XS_F_MC);
      int64_t maxdeg = 0;
      for (int64_t v = 0; v < n; v++) maxdeg = std::max<int64_t>(maxdeg, row_ptr[v + 1] - row_ptr[v]);
      const double seed = damping > 0.0 ? (double)std::max<int64_t>(1, maxdeg) / damping : 1.0;
      if ((double)maxdeg + seed >= lim) { plan_free(p); return PPR_ERR_RANGE; }
    }
    const char* ee = getenv("PPR_XSHARD_ENDS");  // (any summation mode)
    p->xshard_ends = !(ee && atoi(ee) == 0);
    {  // split wave tiers, any summation mode
      const char* ews = getenv("PPR_WAVE_SPLIT");
      if (ews) p->wave_split_T = std::max(0, atoi(ews));
      const char* ewsc = getenv("PPR_WAVE_SPLIT_CHAIN");
      if (ewsc) p->wave_split_chain = std::max(0, atoi(ewsc));
      const char* ewsm = getenv("PPR_WAVE_SPLIT_MC");
      if (ewsm) p->wave_split_mc = std::max(0, atoi(ewsm));
      const char* ewm = getenv("PPR_WL_MAX_MB");  // (tests: a small bound forces the chunked lists)
      if (ewm) p->wl_max = std::max<size_t>(1, (size_t)atoll(ewm)) << 20;
      const char* ewc = getenv("PPR_WAVE_CAP");
      if (ewc) p->wave_cap = std::max(0, atoi(ewc));
    }
    if (p->xsum) {
      // the order-bound alternatives of the chain path do not apply: no hot pass, no speculative
      // bound, no workgroup tier (its overflow would fall to the chain-order HBM table)
      p->hot_cap = 0;
      p->spec_ratio = 0.0;
      p->tierCap[NT] = 0;
      p->seg_enabled = false;
      p->hub_range = 0;
      const char* e1 = getenv("PPR_XR_T");
      const char* e3 = getenv("PPR_XR_RMAX");
      const char* e4 = getenv("PPR_XR_FILL");
      if (e1) p->xr_T = std::max(1024, std::min(8192, pow2_at_least(atoi(e1))));
      p->xr_W = p->xr_T / (8 * WAVE);  // every thread settles 8 table slots (merge_xs.h XR_SLOTS)
      if (e3) p->xr_rmax = std::max(1, std::min(64, atoi(e3)));
      if (e4) p->xr_fill = std::max(20, std::min(85, atoi(e4)));
      const char* e5 = getenv("PPR_XR_DSCALE");
      if (e5) p->xr_dscale = std::max(1, std::min(1000, atoi(e5)));
      const char* e6 = getenv("PPR_HUB_MAX_LOGP");
      if (e6) p->hub_max_logp = std::max(1, std::min(HUB_MAX_LOGP, atoi(e6)));
      const char* e7 = getenv("PPR_XG_CAP");
      p->xg_cap = std::max<int>((int)L, std::min(XG_CAP, e7 ? atoi(e7) : XG_CAP));
      while (xr_lds_bytes(p->xr_T, p->xr_T / (8 * WAVE), p->Lp) > 160 * 1024 && p->xr_T > 1024) p->xr_T /= 2;
      p->xr_W = p->xr_T / (8 * WAVE);
      if (xr_lds_bytes(p->xr_T, p->xr_W, p->Lp) > 160 * 1024 || xf_lds_bytes(p->Lp, 64) > 160 * 1024) {
        plan_free(p);
        return PPR_ERR_RANGE;
      }
      p->xf_stage = (int)std::min<size_t>(XF_STAGE, (160 * 1024 - xf_lds_bytes(p->Lp, 0)) / 12) & ~15;
      for (int t = 0; t < NT; t++)
        if (p->tierT[t] && lds_wave_bytes_x(p->tierT[t], p->Lp) * p->wave_wpb > 160 * 1024) {
          p->tierT[t] = 0;
          p->tierCap[t] = 0;
        }
      TRY(dalloc(&p->d_dlast, n));
      TRY(dalloc(&p->d_wovl, n + 1));
      p->xr_cap = 2 * p->Lp;
      const char* exc = getenv("PPR_XR_LISTCAP");  // (0: k_xr selects every one-range source itself)
      if (exc) p->xr_cap = atoi(exc) <= 0 ? 0 : std::max<int>((int)L, atoi(exc));
      const char* e9 = getenv("PPR_XR_BUDGET");
      p->xr_budget_over = e9 && strcmp(e9, "over") == 0;
      if (hipMemset(p->d_dlast, 0, 4 * (size_t)(n > 0 ? n : 1)) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
      int32_t caps[NT + 1];
      for (int t = 0; t <= NT; t++) caps[t] = p->tierCap[t];
      if (hipMemcpy(p->d_tier_cap, caps, sizeof(caps), hipMemcpyHostToDevice) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
      // the sieve (merge_sv.h) for the wide sources: its prev table takes 2 Lp <= one slot per thread
      const char* s0 = getenv("PPR_SV");
      // (rows of at most two 64-entry groups: L <= 128; wider baskets take the range / partition
      // engines, exact either way)
      p->sv_enabled = !(s0 && atoi(s0) == 0) && p->Lp <= 2 * WAVE &&
                      sv_lds_bytes(p->Lp, SV_LARGE) <= 160 * 1024 && svf_lds_bytes(p->Lp) <= 160 * 1024;
      const char* s1 = getenv("PPR_SV_SLICE");
      const char* s2 = getenv("PPR_SV_MIN");
      if (s1) p->sv_slice = std::max<int64_t>(64, atoll(s1));
      if (s2) p->sv_min = std::max<int64_t>(0, atoll(s2));
      const char* s5 = getenv("PPR_SV_SMALL");
      const char* s6 = getenv("PPR_SV_MID");
      if (s5) p->sv_small = std::max<int64_t>(0, atoll(s5));
      if (s6) p->sv_mid = std::max<int64_t>(0, atoll(s6));
      const char* exm = getenv("PPR_XM");  // one-range sources of the smallest class: k_xm (1) or k_xr (0, default:
      p->xm = exm && atoi(exm) == 1;       // k_xm measured 2.8 % slower per job)
      const char* ex = getenv("PPR_XR_ORDER");
      p->xr_big_first = ex && atoi(ex) == 1;
      const char* eh = getenv("PPR_XH_FIRST");
      p->xh_first = !(eh && atoi(eh) == 0);
      const char* s7 = getenv("PPR_SV_REDO");
      p->sv_redo_mid = !(s7 && atoi(s7) == 0);
      const char* s9 = getenv("PPR_SV_P2SKIP");
      p->sv_p2skip = !(s9 && atoi(s9) == 0);
      const char* s8 = getenv("PPR_SV_REDO_LARGE");
      p->sv_redo_large = s8 && atoi(s8) != 0;
      const char* s3 = getenv("PPR_SV_BUDGET");
      if (s3) p->sv_budget = std::max(0, std::min(SV_XT_BUDGET, atoi(s3)));
      // Streams of the exact sum: a process has 4 hardware queues (HIP's default), and streams
      // beyond them share queues -- a kernel then waits behind another stream's kernel. The hot
      // pass's stream5 is unused here (no hot pass), so it goes, and each of the 4 remaining streams
      // gets its own queue: the plan stream (classification, then the sieve's mid class), stream2
      // (the wave tier, then the multi-slice chain: the wave tier is heavy in the partition with
      // many small sources, the multi-slice sources live in the other), stream4 (the sieve's large
      // and small classes) and stream3 (the range engines for the sources the sieve does not take
      // or hands back)
      if (p->stream5) { hipStreamDestroy(p->stream5); p->stream5 = nullptr; }
      if (p->sv_enabled && p->stream2) p->stream_wave = p->stream2;
      p->stream_sv = p->stream2 ? p->stream2 : p->stream;
      p->stream_sv2 = p->stream4 ? p->stream4 : p->stream;
      p->stream_sv3 = p->stream;
      if (p->sv_enabled && hipEventCreateWithFlags(&p->ev_sv, hipEventDisableTiming) != hipSuccess) {
        plan_free(p);
        return PPR_ERR_HIP;
      }
    }
  }
  // every kernel that may take more than the default 64 KB of dynamic LDS; a refusal (e.g. a
  // kernel that also declares static LDS) fails the plan instead of surfacing later as a launch error
  {
    const std::pair<const void*, const char*> big_lds[] = {
        {(const void*)k_hub_bucket_w<1>, "k_hub_bucket_w<1>"},
        {(const void*)k_hub_bucket_w<2>, "k_hub_bucket_w<2>"},
        {(const void*)k_hub_bucket_w<4>, "k_hub_bucket_w<4>"},
        {(const void*)k_hub_bucket_w<8>, "k_hub_bucket_w<8>"},
        {(const void*)k_hub_range<1>, "k_hub_range<1>"},
        {(const void*)k_hub_range<2>, "k_hub_range<2>"},
        {(const void*)k_hub_range<4>, "k_hub_range<4>"},
        {(const void*)k_hub_range<8>, "k_hub_range<8>"},
        {(const void*)k_hub_seg<4>, "k_hub_seg<4>"},
        {(const void*)k_hub_bucket, "k_hub_bucket"},
        {(const void*)k_hub_final, "k_hub_final"},
        {(const void*)k_topk, "k_topk"},
        {(const void*)k_hub_count<false>, "k_hub_count<false>"},
        {(const void*)k_hub_scatter<false>, "k_hub_scatter<false>"},
        {(const void*)k_hub_count<true>, "k_hub_count<true>"},
        {(const void*)k_hub_scatter<true>, "k_hub_scatter<true>"},
        {(const void*)k_hub_hot, "k_hub_hot"},
        {(const void*)k_hub_join, "k_hub_join"},
        {(const void*)k_merge_lds_x<false>, "k_merge_lds_x"},
        {(const void*)k_merge_lds_x<true>, "k_merge_lds_x<split>"},
        {(const void*)k_wfin, "k_wfin"},
        {(const void*)k_xr, "k_xr"},
        {(const void*)k_xm<4>, "k_xm<4>"},
        {(const void*)k_xb, "k_xb"},
        {(const void*)k_xfinal<XDesc>, "k_xfinal<XDesc>"},
        {(const void*)k_xfinal<HubDesc>, "k_xfinal<HubDesc>"},
        {(const void*)k_sv1, "k_sv1"},
        {(const void*)k_sv1_redo, "k_sv1_redo"},
        {(const void*)k_sv1_list, "k_sv1_list"},
        {(const void*)k_svA, "k_svA"},
        {(const void*)k_svB, "k_svB"},
        {(const void*)k_svF, "k_svF"},
        {(const void*)k_svfin, "k_svfin"},
        {(const void*)k_xfin1, "k_xfin1"},
        {(const void*)k_xg_fin, "k_xg_fin"},
    };
    for (const auto& k : big_lds)
      if (hipFuncSetAttribute(k.first, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) {
        fprintf(stderr, "ppr_hip: 160 KB dynamic LDS refused for %s\n", k.second);
        hipGetLastError();
        plan_free(p);
        return PPR_ERR_HIP;
      }
  }
  *out = p;
  return PPR_OK;
}

static IterArgs iter_args(const ppr_plan* p, int it, bool unit);

// Hot key set of this run (merge_hot.h), from the rows iteration `it` reads: weights over every
// hot_stride-th row, a 4096-bin histogram to find the weight bin at which the top hot_cap end,
// the keys above it plus the heaviest of that bin (weight desc, id asc) on the host.
static int hot_build(ppr_plan* p, int it) {
  hipStream_t st = p->stream;
  const int64_t n = p->n;
  const IterArgs a = iter_args(p, it, false);
  HIP_OK(hipMemsetAsync(p->d_hot_w, 0, 4 * (size_t)n, st));
  HIP_OK(hipMemsetAsync(p->d_hot_hist, 0, 4 * (HOT_BINS + 2), st));
  const int64_t ns = (n + p->hot_stride - 1) / p->hot_stride;
  hipLaunchKernelGGL(k_hot_weight, dim3((unsigned)((ns + 3) / 4)), dim3(256), 0, st, dev_slab(p), a, p->d_part,
                     p->d_indeg, p->hot_stride, p->d_hot_w);
  HIP_OK(hipGetLastError());
  const unsigned hb = (unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 255) / 256));
  hipLaunchKernelGGL(k_hot_hist, dim3(hb), dim3(256), 0, st, p->d_hot_w, n, p->d_hot_hist);
  HIP_OK(hipGetLastError());
  std::vector<uint32_t> hist(HOT_BINS);
  HIP_OK(hipMemcpyAsync(hist.data(), p->d_hot_hist, 4 * HOT_BINS, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  int64_t above = 0;
  int bound = 0;  // no bin overflows the cap: every key with a weight is taken
  for (int b = HOT_BINS - 1; b > 0; b--) {
    if (above + hist[b] > p->hot_cap) { bound = b; break; }
    above += hist[b];
  }
  const int64_t room_max = (p->hot_list_cap - p->hot_cap) / 2;
  hipLaunchKernelGGL(k_hot_collect, dim3(hb), dim3(256), 0, st, p->d_hot_w, n, (uint32_t)bound, p->d_hot_list,
                     p->hot_list_cap, room_max, p->d_hot_hist + HOT_BINS);
  HIP_OK(hipGetLastError());
  uint32_t cnt[2];
  HIP_OK(hipMemcpyAsync(cnt, p->d_hot_hist + HOT_BINS, 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  std::vector<int32_t> keys(cnt[0]);
  const int64_t nb = std::min<int64_t>(cnt[1], room_max);
  std::vector<int32_t> tail(2 * nb);
  if (cnt[0]) HIP_OK(hipMemcpyAsync(keys.data(), p->d_hot_list, 4 * (size_t)cnt[0], hipMemcpyDeviceToHost, st));
  if (nb) HIP_OK(hipMemcpyAsync(tail.data(), p->d_hot_list + p->hot_list_cap - 2 * nb, 8 * (size_t)nb,
                                hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (bound > 0 && nb) {
    // the boundary bin's pairs, heaviest first (ties: smaller id), fill the remaining room
    std::vector<std::pair<uint32_t, int32_t>> bb(nb);
    for (int64_t j = 0; j < nb; j++) bb[j] = {(uint32_t)tail[2 * j + 1], tail[2 * j]};
    std::sort(bb.begin(), bb.end(), [](const std::pair<uint32_t, int32_t>& x, const std::pair<uint32_t, int32_t>& y) {
      return x.first > y.first || (x.first == y.first && x.second < y.second);
    });
    const int64_t take = std::min<int64_t>(nb, p->hot_cap - (int64_t)keys.size());
    for (int64_t j = 0; j < take; j++) keys.push_back(bb[j].second);
  }
  std::sort(keys.begin(), keys.end());  // dense indices in id order (run-to-run identical layout)
  p->hot_n = (int)keys.size();
  HIP_OK(hipMemsetAsync(p->d_hot_bits, 0, 4 * (size_t)((n + 31) / 32), st));
  if (p->hot_n) {
    HIP_OK(hipMemcpyAsync(p->d_hot_keys, keys.data(), 4 * keys.size(), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_hot_set, dim3((unsigned)((p->hot_n + 255) / 256)), dim3(256), 0, st, p->d_hot_keys,
                       p->hot_n, p->d_hot_bits, p->d_hot_idx);
    HIP_OK(hipGetLastError());
    // stored ids switch to the hot encoding: every row written so far is re-encoded
    hipLaunchKernelGGL(k_hot_encode, dim3((unsigned)((2 * n + 3) / 4)), dim3(256), 0, st, dev_slab(p));
    HIP_OK(hipGetLastError());
  }
  p->h_hot_keys = keys;
  HIP_OK(hipStreamSynchronize(st));  // `keys` leaves scope
  return PPR_OK;
}

extern "C" int ppr_grank_plan_create(const ppr_csr* g, const uint8_t* part_in, uint32_t K,
                                     uint32_t L, double damping, const ppr_opts* o,
                                     ppr_plan** out) {
  if (!g || !out || g->n < 0 || (g->n > 0 && !g->row_ptr)) return PPR_ERR_ARG;
  if (g->n > 0 && g->row_ptr[g->n] > 0 && !g->col) return PPR_ERR_ARG;
  int rc = check_params(K, L, 1, damping);
  if (rc != PPR_OK) return rc;
  if (L > (uint32_t)MAX_L) return PPR_ERR_RANGE;
  if (g->n >= (1LL << 31) - 1) return PPR_ERR_RANGE;
  const int64_t n = g->n;
  const int64_t m = n ? g->row_ptr[n] : 0;
  const bool timing = getenv("PPR_TIMING") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  const auto t0 = now();
  const int nth = pprh::host_threads();
  std::vector<uint8_t> part(n > 0 ? n : 1, 0);
  {
    std::atomic<bool> bad(false);
    pprh::parallel_for(m, nth, [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; i++)
        if (g->col[i] < 0 || g->col[i] >= n) { bad = true; return; }
    });
    if (bad) return PPR_ERR_GRAPH;
  }
  // no partitions given: the BFS 2-colouring on the device, on the plan's own copy of the graph
  // (raw successor ids uploaded once; the pass ORs the partition bits in) with the not yet used
  // basket slab as its scratch -- tens of ms at RMAT-22 instead of the host BFS's 0.3-0.5 s. The
  // host BFS for graphs the device pass declines (long paths: PPR_ERR_RANGE) or when PPR_HOST_BFS=1.
  const bool dev_part = !part_in && n && !(getenv("PPR_HOST_BFS") && atoi(getenv("PPR_HOST_BFS")) == 1);
  if (part_in) std::memcpy(part.data(), part_in, n);
  else if (n && !dev_part && (rc = ppr_find_partitions_csr(g, part.data()))) return rc;
  const auto t1 = now();
  // host-side CSR with partition bit of the successor (the device pass sets it itself)
  std::vector<int32_t> colx;
  auto build_colx = [&] {
    colx.resize(m > 0 ? m : 1);
    pprh::parallel_for(m, nth, [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; i++) colx[i] = g->col[i] | (part[g->col[i]] ? (int32_t)0x80000000 : 0);
    });
  };
  if (!dev_part) build_colx();
  const auto t2 = now();
  ppr_plan* p = nullptr;
  rc = plan_alloc(n, g->row_ptr, dev_part ? g->col : colx.data(), K, L, damping, o, &p);
  if (rc) return rc;
  const auto t3 = now();
  double part_dev_s = 0.0;
  if (dev_part) {
    const size_t slab = (size_t)2 * n * L;  // int32 entries of d_ids
    int32_t* scr = nullptr;
    bool own = false;
    if ((size_t)m + 2 * (size_t)n + 2 <= slab) scr = p->d_ids;
    else if (hipMalloc(&scr, 4 * ((size_t)m + 2 * (size_t)n + 2)) == hipSuccess) own = true;
    else { plan_free(p); return PPR_ERR_OOM; }
    rc = pprpart::partitions_core(p->d_rp, p->d_colx, n, m, p->d_part, part.data(), true, scr, scr + m,
                                  scr + m + n, scr + m + 2 * n, p->stream);
    if (own) hipFree(scr);
    if (rc == PPR_ERR_RANGE) {  // (d_colx still raw)
      rc = ppr_find_partitions_csr(g, part.data());
      if (!rc) {
        build_colx();
        if (m && hipMemcpy(p->d_colx, colx.data(), 4 * (size_t)m, hipMemcpyHostToDevice) != hipSuccess) rc = PPR_ERR_HIP;
      }
    }
    if (rc) { plan_free(p); return rc; }
    part_dev_s = sec(t3, now());
  }
  const auto t4 = now();
  std::vector<int32_t> act[2];
  for (int64_t v = 0; v < n; v++)
    if (g->row_ptr[v + 1] > g->row_ptr[v]) act[part[v]].push_back((int32_t)v);
  // merge work estimate per active source (balanced source shards): sum over successors of the
  // initial basket bound min(L, deg(u) + 1)
  for (int q = 0; q < 2; q++) {
    p->work[q].resize(act[q].size());
    pprh::parallel_for((int64_t)act[q].size(), nth, [&](int64_t b, int64_t e2, int) {
      for (int64_t i = b; i < e2; i++) {
        const int v = act[q][i];
        double w = 1.0;
        for (int64_t e = g->row_ptr[v]; e < g->row_ptr[v + 1]; e++) {
          const int u = g->col[e];
          w += (double)std::min<int64_t>(L, g->row_ptr[u + 1] - g->row_ptr[u] + 1);
        }
        p->work[q][i] = w;
      }
    });
  }
  if (timing)
    fprintf(stderr, "ppr_timing plan_create partitions_s %.3f colx_s %.3f alloc_upload_s %.3f work_s %.3f\n",
            sec(t0, t1) + part_dev_s, sec(t1, t2), sec(t2, t3), sec(t4, now()));
  p->nact[0] = (int64_t)act[0].size();
  p->nact[1] = (int64_t)act[1].size();
  if (p->hot_cap > 0 && n > 0) {
    std::vector<int32_t> indeg(n, 0);
    for (int64_t e = 0; e < m; e++) indeg[g->col[e]]++;
    p->hot_list_cap = p->hot_cap + 2 * std::min<int64_t>(n, 1 << 20);
    TRY(dalloc(&p->d_hot_bits, (n + 31) / 32));
    TRY(dalloc(&p->d_hot_idx, n));
    TRY(dalloc(&p->d_hot_keys, p->hot_cap));
    TRY(dalloc(&p->d_hot_w, n));
    TRY(dalloc(&p->d_hot_hist, HOT_BINS + 2));
    TRY(dalloc(&p->d_hot_list, p->hot_list_cap));
    TRY(dalloc(&p->d_indeg, n));
    if (hipMemcpy(p->d_indeg, indeg.data(), 4 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) {
      plan_free(p); return PPR_ERR_HIP;
    }
  } else {
    p->hot_cap = 0;
  }
  TRY(dalloc(&p->d_act[0], p->nact[0]));
  TRY(dalloc(&p->d_act[1], p->nact[1]));
  hipStream_t st = p->stream;
  if (n) {
    if (hipMemcpyAsync(p->d_part, part.data(), n, hipMemcpyHostToDevice, st) != hipSuccess ||
        (p->nact[0] && hipMemcpyAsync(p->d_act[0], act[0].data(), 4 * p->nact[0], hipMemcpyHostToDevice, st) != hipSuccess) ||
        (p->nact[1] && hipMemcpyAsync(p->d_act[1], act[1].data(), 4 * p->nact[1], hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess) {
      plan_free(p); return PPR_ERR_HIP;
    }
  }
  *out = p;
  return PPR_OK;
}

extern "C" void ppr_grank_plan_destroy(ppr_plan* p) { plan_free(p); }
extern "C" void* ppr_grank_plan_stream(ppr_plan* p) { return p ? (void*)p->stream : nullptr; }

static IterArgs iter_args(const ppr_plan* p, int it, bool unit) {
  IterArgs a;
  a.damping = p->damping;
  a.mc = 0u;
  a.rp = p->d_rp;
  a.diag = p->d_diag;
  a.unit = unit ? 1u : 0u;
  a.stats = (p->flags & PPR_FLAG_STATS) ? 1u : 0u;
  a.lds_rank = p->lds_rank;
  a.nt = (uint32_t)p->nt_loads;
  a.whatif = ((uint32_t)p->whatif & 0xffffu) | (p->sv_p2skip ? 0u : WI_SV_NO_P2SKIP) |
             (p->rank_permute ? WI_RANK_PERMUTE : 0u);
  a.iter = unit ? -1 : it;
  a.spec = (unit || p->hot_cap > 0 || it < p->spec_from) ? 0.0 : p->spec_ratio;
  a.xs = p->xsum ? 1u : 0u;
  a.xsf = XS_F;
  if (unit) { a.sA = 0; a.sB = 0; a.active = -1; return a; }
  a.sA = ((it + 1) / 2) & 1;
  a.sB = (it / 2) & 1;
  a.active = it & 1;
  return a;
}

static int run_merge_impl(ppr_plan* p, const IterArgs& a, const int32_t* list, int64_t count,
                          unsigned long long* maxdiff);

static int ensure_scratch(ppr_plan* p, size_t need) {
  if (need <= p->scratch_bytes) return PPR_OK;
  HIP_OK(hipStreamSynchronize(p->stream));
  hipFree(p->d_scratch);
  p->d_scratch = nullptr;
  p->scratch_bytes = 0;
  if (hipMalloc(&p->d_scratch, need) != hipSuccess) return PPR_ERR_OOM;
  p->scratch_bytes = need;
  return PPR_OK;
}

static int ensure_dev(unsigned char** ptr, size_t* cap, size_t need);

static int ceil_log2(int64_t x) { return x <= 1 ? 0 : 64 - __builtin_clzll((unsigned long long)(x - 1)); }

// Hub pipeline over `big` (sources beyond the workgroup tier), in batches bounded by the staging
// budget. Everything is planned on the host up front from the candidate counts (O(#hubs)); the
// per-batch task lists are expanded on the device and no step of a batch waits for the host, so
// the batches run back to back. Sources with a bucket that overflows every LDS table are appended
// to `fallback` (HBM-table path) after the last batch (the only host sync here).
static int run_hubs(ppr_plan* p, const IterArgs& a, const int32_t* big,
                    const int32_t* cand /* parallel to big, then the out-degrees */, size_t nbig, unsigned long long* maxdiff,
                    std::vector<int32_t>& fallback, const int32_t* dest = nullptr) {
  hipStream_t st = p->stream;
  DevGraph g{p->d_rp, p->d_colx, p->n};
  const DevSlab s = dev_slab(p);
  const int64_t L = p->L;
  const int64_t budget = p->hub_budget;  // staged candidates per batch (default 4 GiB of 16-B records)
  const auto t_plan0 = std::chrono::steady_clock::now();
  p->last_nbig = (int64_t)nbig;  // PPR_MC_LEVEL_LOG
  p->last_maxneed = 0;
  for (size_t i = 0; i < nbig; i++) p->last_maxneed = std::max<int64_t>(p->last_maxneed, cand[i]);
  const int slice = p->hub_slice;
  using Batch = HubBatch;
  std::vector<Batch>& batches = p->hub_batches;
  batches.clear();
  {
    int rc0 = ensure_pinned(&p->h_desc_pin, &p->h_desc_bytes, sizeof(HubDesc) * (nbig + 1));
    if (rc0) return rc0;
  }
  HubDesc* desc = (HubDesc*)p->h_desc_pin;
  size_t nd_all = 0;
  // hot pass for every staged source of this merge (not in init, not in the MC combine); rows
  // are stored with the hot encoding exactly when hot_n > 0
  const bool hot = p->hot_n > 0 && !a.unit && !a.mc;
  const HotSet H{p->d_hot_bits, p->d_hot_idx, p->d_hot_keys, hot ? p->hot_n : 0};
  // need < 2^31 (plan-create range check): 32-bit divisions; the planning loop below runs once per
  // hub source per iteration (hundreds of thousands), on the critical path before the first batch
  const uint32_t hb = (uint32_t)p->hub_bucket, sgb = (uint32_t)p->seg_bucket;
  auto cdiv32 = [](uint32_t x, uint32_t d) { return x / d + (x % d != 0); };
  auto logp_of = [&](int64_t need) {
    return std::max(1, std::min(HUB_MAX_LOGP, ceil_log2((int64_t)cdiv32((uint32_t)need, hb))));
  };
  std::vector<uint8_t> lpv(nbig);
  if (a.xs) {
    // exact sum: buckets sized by the expected distinct keys (dest), one workgroup table each
    const int64_t capb = (int64_t)p->xr_T * p->xr_fill / 100;
    for (size_t i = 0; i < nbig; i++)
      lpv[i] = (uint8_t)std::max(1, std::min(p->hub_max_logp, ceil_log2((dest[i] + capb - 1) / capb)));
  } else {
    for (size_t i = 0; i < nbig; i++) lpv[i] = (uint8_t)logp_of(cand[i]);
  }
  // batches mix large and small sources: that hides the long hot-key buckets of the large ones
  // (grouping them by size measured 10 % slower), and it balances the two pipeline stages, whose
  // costs differ by source size (large partitions: count + scatter bound; many small sources:
  // bucket bound). PPR_HUB_MIX > 0 interleaves sources with P >= 2^PPR_HUB_MIX evenly among the
  // others; 0 keeps the classification's list order.
  std::vector<uint32_t> order(nbig);
  if (p->hub_mix > 0) {
    std::vector<uint32_t> lg, sm;
    lg.reserve(nbig);
    sm.reserve(nbig);
    for (size_t i = 0; i < nbig; i++) (lpv[i] >= p->hub_mix ? lg : sm).push_back((uint32_t)i);
    size_t a0 = 0, b0 = 0, k = 0;
    while (a0 < lg.size() || b0 < sm.size()) {
      // take from the list that is behind its share (a0 / |lg| vs b0 / |sm|)
      const bool take_lg = b0 >= sm.size() || (a0 < lg.size() && a0 * sm.size() <= b0 * lg.size());
      order[k++] = take_lg ? lg[a0++] : sm[b0++];
    }
  } else {
    for (size_t i = 0; i < nbig; i++) order[i] = (uint32_t)i;
  }
  // Long tiles (tile_pb candidates per bucket) cut the scatter's partial-line stores but leave
  // fewer tiles per source: they pay only when the call has hub work enough to fill the chip
  // anyway (a GRank iteration: billions of candidates), not for the few lone hubs of an MC level.
  const auto t_plan1 = std::chrono::steady_clock::now();
  int64_t need_all = 0;
  for (size_t i = 0; i < nbig; i++) need_all += cand[i];
  const int tile_pb = need_all >= p->hub_long_min ? p->hub_tile_pb : 1;
  // per partition size 2^lp: successors per tile, list-region entries, reduce slices
  int tw_of[HUB_MAX_LOGP + 1], nsl_of[HUB_MAX_LOGP + 1];
  int64_t ptc_of[HUB_MAX_LOGP + 1];
  for (int lp = 0; lp <= HUB_MAX_LOGP; lp++) {
    // tile = tw successors (windows of 64 on one wave); large partitions get long tiles
    const int64_t tcand = std::max<int64_t>(p->hub_tile_cand, (int64_t)tile_pb << lp);
    const int64_t tw0 = std::max<int64_t>(1, tcand / L);
    tw_of[lp] = (int)(tw0 > WAVE ? (tw0 + WAVE - 1) / WAVE * WAVE : tw0);
    ptc_of[lp] = (int64_t)(1 << lp) * L;
    nsl_of[lp] = ptc_of[lp] > 2 * slice ? (int)((ptc_of[lp] + slice - 1) / slice) : 0;
  }
  {
    size_t oi = 0;
    while (oi < nbig) {
      Batch b{nd_all, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
      while (oi < nbig) {
        const size_t i = order[oi];
        const int v = big[i];
        const int64_t need = cand[i];
        const int64_t deg = cand[nbig + i];
        // segmented path (no partition pass): iterations only (the init has no successor rows),
        // and at most 2^RANGE_BITS buckets of about seg_bucket candidates
        const int lseg = p->seg_enabled ? std::max(0, ceil_log2((int64_t)cdiv32((uint32_t)need, sgb))) : RANGE_BITS + 1;
        const bool seg = p->seg_enabled && !a.unit && !hot && lseg <= RANGE_BITS;
        const int logP = seg ? lseg : (int)lpv[i];
        const int64_t ptc = ptc_of[logP];
        if (nd_all > b.d0 &&
            (b.stg + (seg ? 0 : need) > budget || b.pt + ptc > budget || (seg && b.nseg + (1 << lseg) > (1 << 24))))
          break;
        const int P = 1 << logP;
        const int tw = tw_of[logP];
        const int T = seg ? 0 : (int)cdiv32((uint32_t)deg, (uint32_t)tw);  // tiles cover every successor
        const int nsl = nsl_of[logP];
        // staging offsets are cumulative candidate counts in descriptor order, the same order the
        // device scan walks the concatenated count matrices in: scanned cm = absolute offsets
        // tiles of small-partition sources (logP <= split) and of large ones go to two lists,
        // small first: count / scatter run them as separate launches, the small ones with LDS for
        // their own few bucket counters (maxP_s) instead of the batch's largest P -- one 2^12-bucket
        // source in a batch otherwise held every tile of the batch to 16 KB of LDS (9 waves per CU)
        const bool small = logP <= p->tile_split_logp;
        desc[nd_all++] = HubDesc{v, logP, T, (int32_t)need, tw, nsl, -1, (int32_t)b.nrange, b.cm, b.stg, b.pt, b.red,
                                 small ? b.ntiles_s : b.ntiles - b.ntiles_s, b.nbuck, b.nrt, seg ? b.nseg : -1};
        if (!seg && p->hub_range > 0) b.nrange += (P + p->hub_range - 1) / p->hub_range;
        b.cm += (int64_t)P * T;
        b.stg += seg ? 0 : need - 1;
        b.pt += ptc;
        b.red += (int64_t)nsl * L;
        b.ntiles += T;
        if (small) { b.ntiles_s += T; if (T) b.maxP_s = std::max(b.maxP_s, P); }
        if (seg) b.nseg += P; else b.nbuck += P;
        b.nrt += nsl;
        b.maxP = std::max(b.maxP, P);
        oi++;
      }
      b.d1 = nd_all;
      // large sources' tiles follow the small ones
      for (size_t j = b.d0; j < b.d1; j++)
        if (desc[j].logP > p->tile_split_logp) desc[j].tile_off += b.ntiles_s;
      batches.push_back(b);
    }
  }
  const auto t_plan2 = std::chrono::steady_clock::now();
  p->host_plan_part[0] += std::chrono::duration<double>(t_plan1 - t_plan0).count();
  p->host_plan_part[1] += std::chrono::duration<double>(t_plan2 - t_plan1).count();
  p->host_plan_hubs += (int64_t)nbig;
  // hot tasks: every source, in descending candidate count (one launch; the longest fma chains
  // start first); hot list / cold list j belong to the j-th task
  std::vector<HotTask> htask;
  if (hot) {
    std::vector<uint32_t> ord;
    for (size_t j = 0; j < nd_all; j++)
      if (desc[j].need <= p->hot_max_need) ord.push_back((uint32_t)j);
    std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
      return desc[x].need > desc[y].need || (desc[x].need == desc[y].need && x < y);
    });
    htask.resize(ord.size());
    for (size_t j = 0; j < ord.size(); j++) {
      desc[ord[j]].hot = (int32_t)j;
      htask[j] = HotTask{desc[ord[j]].v, (int32_t)j};
    }
  }
  if (p->d_diag && !a.unit)
    for (size_t j = 0; j < nd_all; j++) {
      p->diag_hub_cand += (double)(desc[j].need - 1);
      if ((int64_t)desc[j].need > ((int64_t)hb << HUB_MAX_LOGP)) { p->diag_cap_src += 1; p->diag_cap_cand += desc[j].need - 1; }
    }
  const size_t nht = htask.size();
  const bool hot_any = nht > 0;
  // one scratch layout for every batch (maxima), so no batch reallocates under a running one
  Batch mx{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1};
  size_t maxnd = 0;
  for (const Batch& b : batches) {
    mx.cm = std::max(mx.cm, b.cm); mx.stg = std::max(mx.stg, b.stg); mx.pt = std::max(mx.pt, b.pt);
    mx.ntiles = std::max(mx.ntiles, b.ntiles); mx.nbuck = std::max(mx.nbuck, b.nbuck);
    mx.nrt = std::max(mx.nrt, b.nrt); mx.red = std::max(mx.red, b.red); mx.nseg = std::max(mx.nseg, b.nseg);
    mx.nrange = std::max(mx.nrange, b.nrange);
    maxnd = std::max(maxnd, b.d1 - b.d0);
  }
  size_t scan_tmp = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (const int32_t*)nullptr, (int32_t*)nullptr, (int)mx.cm, st);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  // shared: descriptors + overflow list; then one (or two) per-batch regions
  size_t off = 0;
  const size_t o_desc = off; off = al(off + sizeof(HubDesc) * nd_all);
  const size_t o_ovl = off;  off = al(off + 4 * (nd_all + 1));
  const size_t o_rsp = off;  off = al(off + 4 * (nd_all + 1));
  const size_t o_ht = off;   off = al(off + sizeof(HotTask) * (nht + 1));
  const size_t o_hk = off;   off = al(off + 4 * (size_t)L * nht);
  const size_t o_hs = off;   off = al(off + 8 * (size_t)L * nht);
  const size_t o_hc = off;   off = al(off + 4 * (nht + 1));
  const size_t o_hth = off;  off = al(off + 8 * (nht + 1));
  const size_t o_ck = off;   off = al(off + 4 * (size_t)L * nht);
  const size_t o_cs = off;   off = al(off + 8 * (size_t)L * nht);
  const size_t o_cc = off;   off = al(off + 4 * (nht + 1));
  const size_t shared = off;
  off = 0;
  const size_t o_tile = off; off = al(off + sizeof(HubTask) * mx.ntiles);
  const size_t o_buck = off; off = al(off + sizeof(HubTask) * mx.nbuck);
  const size_t o_rt = off;   off = al(off + sizeof(HubTask) * (mx.nrt + 1));
  const size_t o_sg = off;   off = al(off + sizeof(HubTask) * (mx.nseg + 1));
  const size_t o_cm = off;   off = al(off + 4 * (size_t)mx.cm);
  const size_t o_cmx = off;  off = al(off + 4 * (size_t)mx.cm);
  const size_t o_tmp = off;  off = al(off + scan_tmp);
  const size_t o_st = off;   off = al(off + sizeof(HubRec) * (size_t)mx.stg);
  const size_t o_pk = off;   off = al(off + 4 * (size_t)mx.pt);
  const size_t o_ps = off;   off = al(off + 8 * (size_t)mx.pt);
  const size_t o_rk = off;   off = al(off + 4 * (size_t)(mx.red + 1));
  const size_t o_rs = off;   off = al(off + 8 * (size_t)(mx.red + 1));
  const size_t o_pc = off;   off = al(off + 4 * maxnd);
  const size_t o_tau = off;  off = al(off + 8 * maxnd);
  const size_t o_of = off;   off = al(off + 4 * maxnd);
  const size_t o_gl = off;   off = al(off + sizeof(HubTask) * (mx.nbuck + 1));
  const size_t o_cnt = off;  off = al(off + 16);
  const size_t o_sd = off;   off = al(off + 4 * maxnd);
  const size_t o_rg = off;   off = al(off + sizeof(HubTask) * (mx.nrange + 1));
  const size_t o_bw = off;   off = al(off + sizeof(BucketWork) * (a.xs ? 1 : mx.nbuck));
  const size_t o_xt = off;   off = al(off + 8 * maxnd);   // exact sum: sources' list bounds
  const size_t o_ds = off;   off = al(off + 4 * maxnd);   // exact sum: distinct keys per source
  const size_t region = off;
  // two streams only pay when there is a next batch to overlap with
  const bool ms = p->hub_streams == 2 && batches.size() > 1;
  const int nreg = ms ? (int)std::min<size_t>(p->hub_regions, batches.size()) : 1;
  int rc = ensure_scratch(p, shared + region * nreg);
  if (rc) return rc;
  char* base = (char*)p->d_scratch;
  HubDesc* d_desc_all = (HubDesc*)(base + o_desc);
  int32_t* d_ovl = (int32_t*)(base + o_ovl);     // [0] count, [1..] sources for the HBM-table path
  int32_t* d_rsp = (int32_t*)(base + o_rsp);     // [0] count, [1..] descriptors whose speculative bound failed
  p->host_plan_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t_plan0).count();
  p->host_plan_calls++;
  HIP_OK(hipMemcpyAsync(d_desc_all, desc, sizeof(HubDesc) * nd_all, hipMemcpyHostToDevice, st));
  // (d_ovl[0] is cleared by the first batch's k_hub_expand)
  HotTask* d_htask = (HotTask*)(base + o_ht);
  int32_t* d_hkey = (int32_t*)(base + o_hk);
  double* d_hsc = (double*)(base + o_hs);
  uint32_t* d_hcnt = (uint32_t*)(base + o_hc);
  unsigned long long* d_tau_hot = (unsigned long long*)(base + o_hth);
  int32_t* d_ckey = (int32_t*)(base + o_ck);
  double* d_csc = (double*)(base + o_cs);
  uint32_t* d_ccnt = (uint32_t*)(base + o_cc);
  if (hot_any) {
    // the host vector is read by the copy before the plan's stream syncs at the end of run_hubs
    HIP_OK(hipMemcpyAsync(d_htask, htask.data(), sizeof(HotTask) * nht, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(d_hcnt, 0, 4 * (nht + 1), st));
    HIP_OK(hipMemsetAsync(d_tau_hot, 0, 8 * (nht + 1), st));
  }
  // partition stage (expand, count, scan, scatter, prep) of batch i on `st`, its bucket stage
  // (bucket waves, spills, segments, reduce, final) on `sb`; batch i+2 reuses batch i's region
  // once batch i's bucket stage has finished
  hipStream_t sb = ms ? p->stream2 : st;   // bucket waves, spills, segments
  hipStream_t sf = ms ? p->stream4 : st;   // reduce + final
  hipStream_t sh = ms ? p->stream5 : st;   // hot pass
  if (hot_any) {
    if (ms) {
      HIP_OK(hipEventRecord(p->ev_hot0, st));  // tasks uploaded, hot lists cleared
      HIP_OK(hipStreamWaitEvent(sh, p->ev_hot0, 0));
    }
    // hot lists live outside the regions: the whole hot pass runs beside the batches
    hipLaunchKernelGGL(k_hub_hot, dim3((unsigned)nht), dim3(64), hot_wave_lds(p->hot_n), sh, g, s, a, d_htask,
                       (int64_t)nht, d_hkey, d_hsc, d_hcnt, d_tau_hot);
    HIP_OK(hipGetLastError());
    p->merge_launches++;
    if (ms) HIP_OK(hipEventRecord(p->ev_hot[0], sh));
  }
  for (size_t bi = 0; bi < batches.size(); bi++) {
    const Batch& b = batches[bi];
    const int r = (int)(bi % nreg);
    char* rb = base + shared + region * r;
    HubTask* d_tile = (HubTask*)(rb + o_tile);
    HubTask* d_buck = (HubTask*)(rb + o_buck);
    HubTask* d_rt = (HubTask*)(rb + o_rt);
    HubTask* d_sg = (HubTask*)(rb + o_sg);
    int32_t* d_cm = (int32_t*)(rb + o_cm);
    int32_t* d_cmx = (int32_t*)(rb + o_cmx);
    void* d_tmp = (void*)(rb + o_tmp);
    HubRec* d_st = (HubRec*)(rb + o_st);
    int32_t* d_pk = (int32_t*)(rb + o_pk);
    double* d_ps = (double*)(rb + o_ps);
    int32_t* d_rk = (int32_t*)(rb + o_rk);
    double* d_rs = (double*)(rb + o_rs);
    uint32_t* d_pc = (uint32_t*)(rb + o_pc);
    unsigned long long* d_tau = (unsigned long long*)(rb + o_tau);
    int32_t* d_oflag = (int32_t*)(rb + o_of);
    HubTask* d_gl = (HubTask*)(rb + o_gl);
    uint32_t* d_lc = (uint32_t*)(rb + o_cnt);    // [1] spill list length
    BucketWork* d_bw = (BucketWork*)(rb + o_bw);
    uint32_t* d_sd = (uint32_t*)(rb + o_sd);
    HubTask* d_rg = (HubTask*)(rb + o_rg);
    unsigned long long* d_xt = (unsigned long long*)(rb + o_xt);
    uint32_t* d_ds = (uint32_t*)(rb + o_ds);
    const size_t nd = b.d1 - b.d0;
    HubDesc* d_desc = d_desc_all + b.d0;
    const int maxP = b.maxP;
    if (ms && bi >= (size_t)nreg) HIP_OK(hipStreamWaitEvent(st, p->ev_fin[r], 0));  // region free again
    // (k_hub_expand also clears d_sd, d_pc, d_tau, d_oflag, d_lc and, in the first batch, d_ovl[0])
    hipLaunchKernelGGL(k_hub_expand, dim3((unsigned)nd), dim3(256), 0, st, d_desc, d_tile, d_buck, d_rt, d_sg, d_rg,
                       p->hub_range, d_sd, d_pc, d_tau, d_oflag, d_lc, bi == 0 ? d_ovl : nullptr,
                       bi == 0 ? d_rsp : nullptr);
    HIP_OK(hipGetLastError());
    if (a.xs) {  // list bounds and distinct counts (adjacent: one fill)
      HIP_OK(hipMemsetAsync(d_xt, 0, (size_t)(o_ds - o_xt) + 4 * nd, st));
    }
    const int64_t ntiles = b.ntiles;
    const int64_t nbuck = b.nbuck;
    if (ntiles) {
      // two tile lists (small-partition sources first): per-wave bucket counters (maxP ints) sized
      // for each list's own largest P; with large partitions one wave per block leaves no LDS
      // stranded by the block granularity
      struct TileList { const HubTask* t; int64_t n; int maxP; };
      const TileList tl[2] = {{d_tile, b.ntiles_s, b.maxP_s}, {d_tile + b.ntiles_s, ntiles - b.ntiles_s, maxP}};
      auto launch_tiles = [&](bool scatter, const IterArgs& a) -> int {
        for (const TileList& x : tl) {
          if (!x.n) continue;
          const int twpb = x.maxP >= p->tile_wpb_p ? 1 : WAVES_PER_BLOCK;
          const size_t lds_tile = (size_t)twpb * (x.maxP * 4 + HUB_WALK_FLAGS);
          const unsigned tb = (unsigned)((x.n + twpb - 1) / twpb);
          // (kernels for hot-encoded rows only when the rows are: see DevSlab::keyd)
          if (scatter)
            hipLaunchKernelGGL(p->hot_n > 0 ? k_hub_scatter<true> : k_hub_scatter<false>, dim3(tb), dim3(64 * twpb),
                               lds_tile, st, g, s, a, d_desc, x.t, x.n, x.maxP, d_cmx, d_st);
          else
            hipLaunchKernelGGL(p->hot_n > 0 ? k_hub_count<true> : k_hub_count<false>, dim3(tb), dim3(64 * twpb),
                               lds_tile, st, g, s, a, d_desc, x.t, x.n, x.maxP, d_cm, d_tau, d_sd);
          HIP_OK(hipGetLastError());
        }
        return PPR_OK;
      };
      for (int rep = 0; rep < ((p->whatif & 4) ? 2 : 1); rep++) {
        if (rep) HIP_OK(hipMemsetAsync(d_sd, 0, 4 * nd, st));  // (the staged counts are summed)
        int rc1 = launch_tiles(false, a);
        if (rc1) return rc1;
      }
      HIP_OK(hipcub::DeviceScan::ExclusiveSum(d_tmp, scan_tmp, d_cm, d_cmx, (int)b.cm, st));
      for (int rep = 0; rep < ((p->whatif & 8) ? 2 : 1); rep++) {
        // (PPR_WHATIF 256: the first of the two scatters stores lane-contiguously, the second,
        // the real one, rewrites every staged record)
        IterArgs ar = a;
        if (rep == 0 && (p->whatif & 256)) ar.whatif |= WI_SCAT_COALESCED;
        if (rep == 0 && (p->whatif & 4096)) ar.whatif |= WI_SCAT_NOSTORE;
        if (rep == 0 && (p->whatif & 8192)) ar.whatif |= WI_SCAT_NOSCORE;
        if (rep == 0 && (p->whatif & 16384)) ar.whatif |= WI_SCAT_COUNT;
        if (rep == 0 && (p->whatif & 32768)) ar.whatif |= WI_SCAT_WALK;
        int rc1 = launch_tiles(true, ar);
        if (rc1) return rc1;
      }
    }
    // a batch of sources without successors (init of dangling nodes) has no tiles but still has
    // buckets: the one holding the source's own seed entry
    if (nbuck && p->hub_range == 0 && !a.xs) {
      hipLaunchKernelGGL(k_hub_prep, dim3((unsigned)((nbuck + 255) / 256)), dim3(256), 0, st, g, s, a, H, d_desc, d_buck,
                         nbuck, d_cmx, d_sd, d_tau, d_tau_hot, d_bw);
      HIP_OK(hipGetLastError());
    }
    if (ms) {
      HIP_OK(hipEventRecord(p->ev_part[r], st));
      HIP_OK(hipStreamWaitEvent(sb, p->ev_part[r], 0));
    }
    if (b.nseg) {
      hipLaunchKernelGGL(k_hub_seg<4>, dim3((unsigned)((b.nseg + p->seg_wpb - 1) / p->seg_wpb)), dim3(64 * p->seg_wpb),
                         hub_wave_lds(p->seg_t, 4) * p->seg_wpb, sb, g, s, a, d_desc, d_sg, b.nseg, d_pk, d_ps, d_pc,
                         d_oflag, d_ovl, p->seg_t);
      HIP_OK(hipGetLastError());
      p->merge_launches++;
    }
    if (a.xs) {
      // exact sum: one workgroup per bucket, then one per source over the buckets' lists
      const int budget = p->xr_budget_over ? 2 * p->xr_T : std::min(p->xr_T * 85 / 100, p->xr_T - p->xr_W * WAVE - WAVE);
      if (nbuck) {
        hipLaunchKernelGGL(k_xb, dim3((unsigned)nbuck), dim3(64 * p->xr_W), xr_lds_bytes(p->xr_T, p->xr_W, p->Lp), sb, s,
                           a, d_desc, d_buck, d_cmx, d_sd, d_st, d_tau, p->xr_T, budget, p->Lp, d_xt, d_pk, d_ps, d_pc,
                           d_ds, d_oflag, d_ovl, p->d_rp);
        HIP_OK(hipGetLastError());
        p->merge_launches++;
      }
      if (ms) {
        HIP_OK(hipEventRecord(p->ev_buck[r], sb));
        HIP_OK(hipStreamWaitEvent(sf, p->ev_buck[r], 0));
      }
      hipLaunchKernelGGL(k_xfinal<HubDesc>, dim3((unsigned)nd), dim3(256), xf_lds_bytes(p->Lp, p->xf_stage), sf, s, a,
                         d_desc, d_xt, d_pk, d_ps, d_pc, d_ds, d_oflag, p->d_dlast, p->Lp, p->xf_stage, maxdiff,
                         p->d_stats);
      HIP_OK(hipGetLastError());
      p->merge_launches++;
      if (ms) HIP_OK(hipEventRecord(p->ev_fin[r], sf));
      continue;
    }
    if (nbuck) {
      // every bucket goes to a single wave first: a bucket made long by one hot key (a core node
      // present in most successor baskets) still has few distinct keys, and its sequential fma
      // chain must not hold a whole workgroup. Only table overflows move to the workgroup kernel.
      const int wpb = p->hub_bw_waves;
      const int cap2 = (p->hub_bw2 && p->lds_rank) ? BW2_CAP : 0;
      const int64_t blocks = (nbuck + wpb - 1) / wpb;
      const dim3 grid((unsigned)blocks), blk(64 * wpb);
      if (p->hub_range > 0) {
        const dim3 rgrid((unsigned)((b.nrange + wpb - 1) / wpb));
        if (p->hub_bw_ng == 1)
          hipLaunchKernelGGL(k_hub_range<1>, rgrid, blk, p->hub_lds_wave, sb, g, s, a, H, d_desc, d_rg, b.nrange,
                             p->hub_range, d_cmx, d_sd, d_tau, d_tau_hot, d_st, d_pk, d_ps, d_pc, d_gl, d_lc + 1,
                             p->hub_wave_t, p->hub_bw_budget);
        else if (p->hub_bw_ng == 8)
          hipLaunchKernelGGL(k_hub_range<8>, rgrid, blk, p->hub_lds_wave, sb, g, s, a, H, d_desc, d_rg, b.nrange,
                             p->hub_range, d_cmx, d_sd, d_tau, d_tau_hot, d_st, d_pk, d_ps, d_pc, d_gl, d_lc + 1,
                             p->hub_wave_t, p->hub_bw_budget);
        else if (p->hub_bw_ng == 4)
          hipLaunchKernelGGL(k_hub_range<4>, rgrid, blk, p->hub_lds_wave, sb, g, s, a, H, d_desc, d_rg, b.nrange,
                             p->hub_range, d_cmx, d_sd, d_tau, d_tau_hot, d_st, d_pk, d_ps, d_pc, d_gl, d_lc + 1,
                             p->hub_wave_t, p->hub_bw_budget);
        else
          hipLaunchKernelGGL(k_hub_range<2>, rgrid, blk, p->hub_lds_wave, sb, g, s, a, H, d_desc, d_rg, b.nrange,
                             p->hub_range, d_cmx, d_sd, d_tau, d_tau_hot, d_st, d_pk, d_ps, d_pc, d_gl, d_lc + 1,
                             p->hub_wave_t, p->hub_bw_budget);
      } else if (p->hub_bw_ng == 1)
        hipLaunchKernelGGL(k_hub_bucket_w<1>, grid, blk, p->hub_lds_wave, sb, s, a, d_bw, nbuck, d_st, d_pk, d_ps, d_pc,
                           d_gl, d_lc + 1, p->hub_wave_t, p->hub_bw_budget, 0, p->hub_wave_stride, cap2);
      else if (p->hub_bw_ng == 2) {
        if (p->whatif & 16)  // timing experiment: a dry pass first (no emission, no spills)
          hipLaunchKernelGGL(k_hub_bucket_w<2>, grid, blk, p->hub_lds_wave, sb, s, a, d_bw, nbuck, d_st, d_pk, d_ps,
                             d_pc, d_gl, d_lc + 1, p->hub_wave_t, p->hub_bw_budget, 1, p->hub_wave_stride, cap2);
        hipLaunchKernelGGL(k_hub_bucket_w<2>, grid, blk, p->hub_lds_wave, sb, s, a, d_bw, nbuck, d_st, d_pk, d_ps, d_pc,
                           d_gl, d_lc + 1, p->hub_wave_t, p->hub_bw_budget, 0, p->hub_wave_stride, cap2);
      }
      else if (p->hub_bw_ng == 8)
        hipLaunchKernelGGL(k_hub_bucket_w<8>, grid, blk, p->hub_lds_wave, sb, s, a, d_bw, nbuck, d_st, d_pk, d_ps, d_pc,
                           d_gl, d_lc + 1, p->hub_wave_t, p->hub_bw_budget, 0, p->hub_wave_stride, cap2);
      else
        hipLaunchKernelGGL(k_hub_bucket_w<4>, grid, blk, p->hub_lds_wave, sb, s, a, d_bw, nbuck, d_st, d_pk, d_ps, d_pc,
                           d_gl, d_lc + 1, p->hub_wave_t, p->hub_bw_budget, 0, p->hub_wave_stride, cap2);
      HIP_OK(hipGetLastError());
      // spilled buckets (distinct keys beyond the wave table): persistent workgroups over the spill
      // list, whose length only the device knows
      if (!(p->whatif & 1)) {
        hipLaunchKernelGGL(k_hub_bucket, dim3((unsigned)p->num_cus), dim3(WG_THREADS), p->hub_lds_wg, sb, s, a, g, H,
                           d_desc, d_gl, d_lc + 1, d_cmx, d_sd, d_st, d_pk, d_ps, d_pc, d_tau, d_tau_hot, p->Lp, d_oflag,
                           d_ovl);
        HIP_OK(hipGetLastError());
      }
    }
    if (ms) {
      HIP_OK(hipEventRecord(p->ev_buck[r], sb));
      HIP_OK(hipStreamWaitEvent(sf, p->ev_buck[r], 0));
    }
    // long appended lists are cut (k_hub_reduce) so no k_hub_final workgroup selects from more
    // than a few slices' worth of entries; slices are reserved for the worst case, idle ones exit
    const int fslice = (p->whatif & 2) ? (1 << 28) : slice;  // timing experiment: no reduce (2 * fslice must fit an int)
    if (b.nrt && !(p->whatif & 2)) {
      // LDS-staged slices in the MC combine only: beside a GRank iteration's bucket waves (other
      // streams, same CUs) a 100-KB workgroup crowds them out (measured 3.34 -> 3.66 s per job)
      const bool rstage = a.mc && p->red_pl > 0;
      for (int rep = 0; rep < ((p->whatif & 64) ? 2 : 1); rep++) {
        hipLaunchKernelGGL(k_hub_reduce, dim3((unsigned)b.nrt), dim3(WG_THREADS),
                           rstage ? p->hub_lds_red : p->hub_lds_final, sf, s, d_desc, d_rt, d_pc, d_pk, d_ps, d_rk,
                           d_rs, p->Lp, slice, rstage ? p->red_pl : 0);
        HIP_OK(hipGetLastError());
      }
      p->merge_launches++;
    }
    for (int rep = 0; rep < ((p->whatif & 32) ? 2 : 1); rep++) {
      hipLaunchKernelGGL(k_hub_final, dim3((unsigned)nd), dim3(WG_THREADS), p->hub_lds_final, sf, s, a, d_desc,
                         d_oflag, d_pc, d_pk, d_ps, d_rk, d_rs, fslice, d_ccnt, d_ckey, d_csc, p->Lp, maxdiff, p->d_stats,
                         d_rsp, (int32_t)b.d0);
      HIP_OK(hipGetLastError());
    }
    p->merge_launches += 9;
    if (ms) HIP_OK(hipEventRecord(p->ev_fin[r], sf));
  }
  if (ms) HIP_OK(hipStreamWaitEvent(st, p->ev_fin[(batches.size() - 1) % nreg], 0));  // finals run in order
  if (hot_any) {
    // every hot-pass source's row = top-L of its hot and cold halves
    if (ms) HIP_OK(hipStreamWaitEvent(st, p->ev_hot[0], 0));
    hipLaunchKernelGGL(k_hub_join, dim3((unsigned)nht), dim3(WG_THREADS), p->hub_lds_final, st, s, a, d_htask, d_ccnt,
                       d_ckey, d_csc, d_hcnt, d_hkey, d_hsc, p->Lp, maxdiff, p->d_stats);
    HIP_OK(hipGetLastError());
    p->merge_launches++;
  }
  if (a.mc && !hot_any) {
    // MC combine: the overflow count is read with the next level's classification (one host
    // sync per level; run_merge_impl redoes that level's classification when it is non-zero)
    p->ovl_pending = d_ovl;
    return PPR_OK;
  }
  int32_t novf = 0, nrsp = 0;
  HIP_OK(hipMemcpyAsync(&novf, d_ovl, 4, hipMemcpyDeviceToHost, st));
  if (a.spec > 0.0) HIP_OK(hipMemcpyAsync(&nrsp, d_rsp, 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (novf) {
    std::vector<int32_t> ov(novf);
    HIP_OK(hipMemcpyAsync(ov.data(), d_ovl + 1, 4 * (size_t)novf, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    fallback.insert(fallback.end(), ov.begin(), ov.end());
  }
  if (nrsp) {
    // sources whose speculative bound k_hub_final could not prove: merged again with the rigorous
    // bound (their rows were not written), one more hub pass over just them
    std::vector<int32_t> di(nrsp);
    HIP_OK(hipMemcpyAsync(di.data(), d_rsp + 1, 4 * (size_t)nrsp, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    std::vector<int32_t> rb(nrsp), rc(2 * (size_t)nrsp);  // sources | candidate counts, out-degrees
    for (int32_t k = 0; k < nrsp; k++) {
      const HubDesc& dk = desc[di[k]];
      rb[k] = dk.v;
      rc[k] = dk.need;
      rc[nrsp + k] = (int32_t)(p->h_rp[dk.v + 1] - p->h_rp[dk.v]);
    }
    p->spec_redo += nrsp;
    IterArgs a2 = a;
    a2.spec = 0.0;
    return run_hubs(p, a2, rb.data(), rc.data(), (size_t)nrsp, maxdiff, fallback);
  }
  return PPR_OK;
}

// Exact-sum merge in one HBM table (merge_xg.h) of sources the bucket partition can not split
// finely enough (more expected distinct keys than 2^hub_max_logp tables hold), one source at a time
// on the plan stream: walk, digit-by-digit search of the L-th largest selection key, compaction,
// finish. Its cost is a few passes over a table of 2 x candidates slots (20 B each).
static int run_xg(ppr_plan* p, const IterArgs& a, const std::vector<int32_t>& src, const std::vector<int32_t>& cand,
                  unsigned long long* maxdiff) {
  hipStream_t st = p->stream;
  DevGraph g{p->d_rp, p->d_colx, p->n};
  const DevSlab s = dev_slab(p);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  for (size_t i = 0; i < src.size(); i++) {
    const int v = src[i];
    int64_t T = 1024;
    while (T < 2 * (int64_t)cand[i] + 64) T <<= 1;
    size_t off = 0;
    const size_t o_k = off;  off = al(off + 4 * (size_t)T);
    const size_t o_a = off;  off = al(off + 8 * (size_t)T);
    const size_t o_b = off;  off = al(off + 8 * (size_t)T);
    const size_t o_st = off; off = al(off + sizeof(XgState));
    const size_t o_h = off;  off = al(off + 4 * (size_t)XG_BINS);
    const size_t o_e = off;  off = al(off + 4);
    const size_t zeroed = off;  // table, state, histogram, error flag
    const size_t o_dk = off; off = al(off + 4 * (size_t)XG_CAP);
    const size_t o_dv = off; off = al(off + 8 * (size_t)XG_CAP);
    { int rc = ensure_dev(&p->d_xg, &p->xg_bytes, off); if (rc) return rc; }
    unsigned char* b = p->d_xg;
    uint32_t* keys = (uint32_t*)(b + o_k);
    unsigned long long* A = (unsigned long long*)(b + o_a);
    unsigned long long* B = (unsigned long long*)(b + o_b);
    XgState* stp = (XgState*)(b + o_st);
    uint32_t* hist = (uint32_t*)(b + o_h);
    int32_t* err = (int32_t*)(b + o_e);
    int32_t* dk = (int32_t*)(b + o_dk);
    double* dv = (double*)(b + o_dv);
    HIP_OK(hipMemsetAsync(b, 0, zeroed, st));
    const int64_t deg = p->h_rp[v + 1] - p->h_rp[v];
    const int64_t blocks = std::max<int64_t>(1, (deg + 4 * WAVE - 1) / (4 * WAVE));
    hipLaunchKernelGGL(k_xg_walk, dim3((unsigned)blocks), dim3(256), 0, st, g, s, a, v, T, keys, A, B, stp);
    HIP_OK(hipGetLastError());
    const unsigned gb = (unsigned)std::min<int64_t>(2048, (T + 1023) / 1024);
    for (int lvl = 0; lvl < XG_LEVELS; lvl++) {
      hipLaunchKernelGGL(k_xg_hist, dim3(gb), dim3(1024), 0, st, v, T, keys, A, B, stp, lvl, hist, a.xsf);
      HIP_OK(hipGetLastError());
      hipLaunchKernelGGL(k_xg_pick, dim3(1), dim3(256), 0, st, stp, lvl, hist, (int)p->L, p->xg_cap);
      HIP_OK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_xg_compact, dim3((unsigned)std::min<int64_t>(8192, (T + 255) / 256)), dim3(256), 0, st, v, T,
                       keys, A, B, stp, dk, dv, a.xsf);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_xg_fin, dim3(1), dim3(64), xg_fin_lds_bytes(p->Lp), st, s, a, v, stp, dk, dv, p->Lp, maxdiff,
                       p->d_stats, err);
    HIP_OK(hipGetLastError());
    p->merge_launches += 4 + 2 * XG_LEVELS;
    int32_t herr = 0;
    HIP_OK(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (herr) return PPR_ERR_HIP;  // (a table of 2 x candidates slots can not fill)
    p->xg_sources++;
  }
  return PPR_OK;
}

// Exact-sum merge of the hub sources src[0..n) (candidate counts cand, out-degrees deg, expected
// distinct keys dest): a source whose keys fit xr_rmax workgroup tables is walked by that many
// range workgroups (k_xr; one range finishes the source itself, several append to a list that
// k_xfinal selects from) on the wave-tier stream, the others are partitioned into buckets of one
// table each (run_hubs: count, scan, scatter, k_xb, k_xfinal) beside them. A table that overflows
// sends its source back here with a larger estimate.
// per-kernel roofline bookkeeping (plan.h NKST groups): events around a group's launches on its
// stream; kst_fold reads the pair once the stream has been synchronised
static void kst_reset(ppr_plan* p) {
  for (int g = 0; g < ppr_plan::NKST; g++) {
    p->kst_ms[g] = 0.0; p->kst_bytes[g] = 0.0; p->kst_pend_bytes[g] = 0.0;
    p->kst_launches[g] = 0; p->kst_live[g] = false;
  }
}
static void kst_begin(ppr_plan* p, int g, hipStream_t s) {
  if (!p->ev_k[2 * g] && hipEventCreate(&p->ev_k[2 * g]) != hipSuccess) return;
  if (!p->ev_k[2 * g + 1] && hipEventCreate(&p->ev_k[2 * g + 1]) != hipSuccess) return;
  hipEventRecord(p->ev_k[2 * g], s);
}
static void kst_end(ppr_plan* p, int g, hipStream_t s, double bytes) {
  if (!p->ev_k[2 * g + 1]) return;
  hipEventRecord(p->ev_k[2 * g + 1], s);
  p->kst_live[g] = true;
  p->kst_pend_bytes[g] = bytes;
}
static void kst_fold(ppr_plan* p, int g) {
  if (!p->kst_live[g]) return;
  p->kst_live[g] = false;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, p->ev_k[2 * g], p->ev_k[2 * g + 1]) == hipSuccess) {
    p->kst_ms[g] += ms;
    p->kst_bytes[g] += p->kst_pend_bytes[g];
    p->kst_launches[g]++;
  }
}

// A range-engine call whose completion is collected later (xhubs_finish): the launches are queued
// on stream3 and the host goes on planning the sieve, so both run from the iteration's start.
struct XhDefer {
  bool want = false;   // the caller accepts a deferred completion
  bool live = false;   // launches queued, not yet collected
  int depth = 0;
  size_t o_ov = 0;
  // the caller's lists (run_xhubs keeps them alive and unchanged until xhubs_finish)
  const std::vector<int32_t>* src = nullptr;
  const std::vector<int32_t>* cand = nullptr;
  const std::vector<int32_t>* deg = nullptr;
  const std::vector<int64_t>* dest = nullptr;
  std::vector<int32_t> xv;
};
static int xhubs_finish(ppr_plan* p, const IterArgs& a, XhDefer& df, unsigned long long* maxdiff);

// (PPR_SV_LOG) host planning sub-phase laps: xh_sub[k] += seconds since t
static inline void sub_lap(ppr_plan* p, int k, std::chrono::steady_clock::time_point& t) {
  const auto t2 = std::chrono::steady_clock::now();
  p->xh_sub[k] += std::chrono::duration<double>(t2 - t).count();
  t = t2;
}

static int run_xhubs_list(ppr_plan* p, const IterArgs& a, const std::vector<int32_t>& src,
                          const std::vector<int32_t>& cand, const std::vector<int32_t>& deg,
                          const std::vector<int64_t>& dest, unsigned long long* maxdiff, int depth,
                          XhDefer* defer = nullptr) {
  const size_t n = src.size();
  if (!n) return PPR_OK;
  auto tsub = std::chrono::steady_clock::now();
  hipStream_t st = p->stream;
  hipStream_t sw = p->stream3 ? p->stream3 : st;
  DevGraph g{p->d_rp, p->d_colx, p->n};
  const DevSlab s = dev_slab(p);
  const int64_t L = p->L;
  // workgroup table classes (slots, waves): 16 waves per CU in each
  struct Cls { int T, W; };
  // (T / 512 waves: the epilogue settles XR_SLOTS = 8 slots per thread)
  const Cls cls[3] = {{std::min(2048, p->xr_T), std::min(2048, p->xr_T) / 512},
                      {std::min(4096, p->xr_T), std::min(4096, p->xr_T) / 512},
                      {p->xr_T, p->xr_T / 512}};
  auto cap_of = [&](int T) { return (int64_t)T * p->xr_fill / 100; };
  // (per-thread scratch kept across calls: no page faults on fresh vectors each iteration; a call's
  // lists are dead before the nested redo call of its tail or of xhubs_finish reuses them)
  static thread_local std::vector<int32_t> rng_tl;
  static thread_local std::vector<uint8_t> ci_tl;
  static thread_local std::vector<XDesc> xd_tl;
  static thread_local std::vector<XTask> tasks_tl[3];
  std::vector<int32_t>& rng = rng_tl;  // ranges per walked source (0: partitioned, -1: HBM table)
  std::vector<uint8_t>& ci = ci_tl;    // table class of a walked source
  rng.resize(n);
  ci.resize(n);
  std::vector<int32_t> bsrc, bcand;    // partitioned: sources | candidate counts, then degrees
  std::vector<int32_t> bdest;
  const int64_t capA = cap_of(p->xr_T);
  // the bucket partition's reach: 2^hub_max_logp tables; a source expected beyond it -- or still
  // overflowing after XG_REDO redos -- goes to the HBM table (rng -1), which can not overflow
  const int64_t reach = capA << p->hub_max_logp;
  constexpr int XG_REDO = 8;
  std::vector<int32_t> xgs, xgc;
  for (size_t i = 0; i < n; i++) {
    const int64_t R = std::max<int64_t>(1, (dest[i] + capA - 1) / capA);
    if (depth > XG_REDO || (p->hub_enabled && R > p->xr_rmax && dest[i] > reach)) {
      rng[i] = -1;
      xgs.push_back(src[i]);
      xgc.push_back(cand[i]);
    } else if (R <= p->xr_rmax || !p->hub_enabled) {
      rng[i] = (int32_t)R;
      int c = 2;
      if (R == 1) c = dest[i] <= cap_of(cls[0].T) ? 0 : dest[i] <= cap_of(cls[1].T) ? 1 : 2;
      ci[i] = (uint8_t)c;
    } else {
      rng[i] = 0;
      bsrc.push_back(src[i]);
      bdest.push_back((int32_t)std::min<int64_t>(dest[i], INT32_MAX));
    }
  }
  sub_lap(p, 0, tsub);  // range planning: classes
  // ranged sources: multi-range ones first (k_xfinal covers descriptors [0, nmulti))
  std::vector<XDesc>& xd = xd_tl;
  std::vector<XTask>* tasks = tasks_tl;
  xd.clear();
  for (int c = 0; c < 3; c++) tasks[c].clear();
  xd.reserve(n);
  tasks[0].reserve(n);
  int64_t pt = 0;
  for (int pass = 0; pass < 2; pass++)
    for (size_t i = 0; i < n; i++) {
      if (rng[i] <= 0 || (rng[i] > 1) != (pass == 0)) continue;
      const int32_t d = (int32_t)xd.size();
      XDesc x;
      x.v = src[i];
      x.R = rng[i];
      x.pt_off = pt;
      // (merge_factor / self_seed of ppr_common.h: GRank d/deg and 1 - d, the MC combine 1 and 1/f)
      x.factor = a.mc ? 1.0 : p->damping / (double)deg[i];
      x.selfval = a.mc ? 1.0 / (p->damping / (double)deg[i]) : 1.0 - p->damping;
      // every range of a multi-range source appends at most L entries; a one-range source its whole
      // top-L, or up to xr_cap unselected entries (k_xfin1 selects)
      pt += rng[i] == 1 ? (int64_t)std::max<int64_t>(L, p->xr_cap) : (int64_t)rng[i] * L;
      xd.push_back(x);
      for (int r = 0; r < rng[i]; r++) tasks[ci[i]].push_back(XTask{d, r});
    }
  sub_lap(p, 1, tsub);  // range planning: descriptors
  int64_t nmulti = 0;
  for (const XDesc& x : xd) nmulti += x.R > 1;
  const size_t nx = xd.size();
  // the 2048-slot class's one-range sources on k_xm (merge_xm.h): self-contained task records;
  // init (unit) merges and baskets wider than 128 keep k_xr
  const bool use_xm = p->xm && !a.unit && p->Lp <= 2 * WAVE && xm_lds_bytes(cls[0].T) <= 160 * 1024;
  std::vector<XmTask> xmt;
  if (use_xm) {
    xmt.reserve(tasks[0].size());
    for (const XTask& t : tasks[0]) {
      const XDesc& x = xd[(size_t)t.d];
      xmt.push_back(XmTask{x.pt_off, x.factor, x.selfval, t.d, x.v});
    }
    tasks[0].clear();
  }
  size_t ntask = 0;
  for (int c = 0; c < 3; c++) ntask += tasks[c].size();
  // device scratch: descriptors | tasks | list keys | list scores | pc | dsum | oflag | ovl | xtau
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  const size_t o_d = off;  off = al(off + sizeof(XDesc) * (nx + 1));
  const size_t o_t = off;  off = al(off + sizeof(XTask) * (ntask + 1));
  const size_t o_m = off;  off = al(off + sizeof(XmTask) * (xmt.size() + 1));
  const size_t o_k = off;  off = al(off + 4 * (size_t)(pt + 1));
  const size_t o_s = off;  off = al(off + 8 * (size_t)(pt + 1));
  const size_t o_z = off;  // zeroed together: pc | dsum | oflag | ovl | xtau
  const size_t o_pc = off; off = al(off + 4 * (nx + 1));
  const size_t o_ds = off; off = al(off + 4 * (nx + 1));
  const size_t o_of = off; off = al(off + 4 * (nx + 1));
  const size_t o_ov = off; off = al(off + 4 * (nx + 2));
  const size_t o_xt = off; off = al(off + 8 * (nx + 1));
  const size_t total = off;
  std::vector<int32_t> ovl_h;
  if (nx) {
    {
      int rc = ensure_dev(&p->d_xs, &p->xs_bytes, total);
      if (rc) return rc;
    }
    unsigned char* b = p->d_xs;
    XDesc* d_xd = (XDesc*)(b + o_d);
    XTask* d_tk = (XTask*)(b + o_t);
    int32_t* d_pk = (int32_t*)(b + o_k);
    double* d_ps = (double*)(b + o_s);
    uint32_t* d_pc = (uint32_t*)(b + o_pc);
    uint32_t* d_ds = (uint32_t*)(b + o_ds);
    int32_t* d_of = (int32_t*)(b + o_of);
    int32_t* d_ov = (int32_t*)(b + o_ov);
    unsigned long long* d_xt = (unsigned long long*)(b + o_xt);
    // descriptors and tasks through the pinned staging buffer (one upload)
    const size_t up = o_m + sizeof(XmTask) * xmt.size();
    {
      // (its own pinned buffer: run_hubs below restages h_desc_pin while this upload may be pending;
      // the previous upload from it completed at the last call's closing sync of sw)
      int rc = ensure_pinned(&p->h_xs_pin, &p->h_xs_bytes, up);
      if (rc) return rc;
    }
    unsigned char* hb = (unsigned char*)p->h_xs_pin;
    std::memcpy(hb + o_d, xd.data(), sizeof(XDesc) * nx);
    if (!xmt.empty()) std::memcpy(hb + o_m, xmt.data(), sizeof(XmTask) * xmt.size());
    size_t tofs[3];
    {
      size_t k = 0;
      for (int c = 0; c < 3; c++) {
        tofs[c] = k;
        if (!tasks[c].empty()) std::memcpy(hb + o_t + sizeof(XTask) * k, tasks[c].data(), sizeof(XTask) * tasks[c].size());
        k += tasks[c].size();
      }
    }
    sub_lap(p, 2, tsub);  // range planning: staging
    HIP_OK(hipMemcpyAsync(b, hb, up, hipMemcpyHostToDevice, sw));
    HIP_OK(hipMemsetAsync(b + o_z, 0, total - o_z, sw));
    // kernel-stat group 5: the range engines (k_xr, k_xfinal, k_xfin1) of this call on sw; SURVEY
    // s8d bytes with the rows at min(L, candidates + 1) entries (the host knows no row lengths)
    if (!a.unit && !a.mc) {
      double bytes = 0.0;
      for (size_t i = 0; i < n; i++)
        if (rng[i] > 0)
          bytes += 8.0 + 8.0 * deg[i] + 12.0 * ((double)cand[i] - 1.0) +
                   24.0 * (double)std::min<int64_t>(L, (int64_t)cand[i] + 1) + 4.0;
      kst_begin(p, 5, sw);
      p->kst_pend_bytes[5] = bytes;
    }
    const bool big_first = p->xr_big_first;  // (experiment)
    if (!xmt.empty()) {
      const int T = cls[0].T, W = cls[0].W;
      const int budget = p->xr_budget_over ? 2 * T : std::min(T * 85 / 100, T - W * WAVE - WAVE);
      // (4 waves: 8 waves at 3 workgroups per CU would need more than 80 VGPRs)
      hipLaunchKernelGGL(k_xm<4>, dim3((unsigned)xmt.size()), dim3(64 * 4), xm_lds_bytes(T), sw, g, s, a,
                         (const XmTask*)(b + o_m), T, budget, d_pk, d_ps, d_pc, d_ds, d_of, d_ov);
      HIP_OK(hipGetLastError());
      p->merge_launches++;
    }
    for (int c0 = 0; c0 < 3; c0++) {
      const int c = big_first ? 2 - c0 : c0;
      if (tasks[c].empty()) continue;
      const int T = cls[c].T, W = cls[c].W;
      // (PPR_XR_BUDGET=over, tests: no budget stop -- the tables fill and the bounded probes run
      // out, which must end in the overflow redo)
      const int budget = p->xr_budget_over ? 2 * T : std::min(T * 85 / 100, T - W * WAVE - WAVE);
      hipLaunchKernelGGL(k_xr, dim3((unsigned)tasks[c].size()), dim3(64 * W), xr_lds_bytes(T, W, p->Lp), sw, g, s, a,
                         d_xd, d_tk + tofs[c], T, budget, p->Lp, d_xt, d_pk, d_ps, d_pc, d_ds, d_of, d_ov, p->xr_cap);
      HIP_OK(hipGetLastError());
      p->merge_launches++;
    }
    if (nmulti) {
      hipLaunchKernelGGL(k_xfinal<XDesc>, dim3((unsigned)nmulti), dim3(256), xf_lds_bytes(p->Lp, p->xf_stage), sw, s, a,
                         d_xd, d_xt, d_pk, d_ps, d_pc, d_ds, d_of, p->d_dlast, p->Lp, p->xf_stage, maxdiff, p->d_stats);
      HIP_OK(hipGetLastError());
      p->merge_launches++;
    }
    if ((int64_t)nx > nmulti) {
      hipLaunchKernelGGL(k_xfin1, dim3((unsigned)((int64_t)nx - nmulti)), dim3(64), xf1_lds_bytes(p->Lp), sw, s, a, d_xd,
                         (int)nmulti, d_pk, d_ps, d_pc, d_ds, d_of, p->d_dlast, p->Lp, maxdiff, p->d_stats);
      HIP_OK(hipGetLastError());
      p->merge_launches++;
    }
    if (!a.unit && !a.mc) kst_end(p, 5, sw, p->kst_pend_bytes[5]);
  }
  sub_lap(p, 3, tsub);  // range planning: launches
  // deferred completion (no partitioned or HBM-table source in this call: those plan on the host
  // from device counts and would serialise behind the range engines here anyway)
  if (defer && defer->want && nx && bsrc.empty() && xgs.empty()) {
    defer->live = true;
    defer->depth = depth;
    defer->o_ov = o_ov;
    defer->src = &src; defer->cand = &cand; defer->deg = &deg; defer->dest = &dest;
    defer->xv.resize(nx);
    for (size_t i = 0; i < nx; i++) defer->xv[i] = xd[i].v;
    return PPR_OK;
  }
  // partitioned sources beside them
  std::vector<int32_t> fallback;
  if (!bsrc.empty()) {
    const size_t nb = bsrc.size();
    std::vector<int32_t> cd(2 * nb);
    {
      size_t k = 0;
      for (size_t i = 0; i < n; i++)
        if (rng[i] == 0) { cd[k] = cand[i]; cd[nb + k] = deg[i]; k++; }
    }
    int rc = run_hubs(p, a, bsrc.data(), cd.data(), nb, maxdiff, fallback, bdest.data());
    if (rc) return rc;
  }
  if (nx) {
    int32_t novf = 0;
    HIP_OK(hipMemcpyAsync(&novf, p->d_xs + o_ov, 4, hipMemcpyDeviceToHost, sw));
    HIP_OK(hipStreamSynchronize(sw));
    kst_fold(p, 5);
    if (novf) {
      std::vector<int32_t> od(novf);
      HIP_OK(hipMemcpyAsync(od.data(), p->d_xs + o_ov + 4, 4 * (size_t)novf, hipMemcpyDeviceToHost, sw));
      HIP_OK(hipStreamSynchronize(sw));
      for (int32_t d : od) fallback.push_back(xd[d].v);
    }
  }
  if (!xgs.empty()) { int rc = run_xg(p, a, xgs, xgc, maxdiff); if (rc) return rc; }
  if (fallback.empty()) return PPR_OK;
  // overflowed tables: those sources again, expecting 4x the distinct keys
  p->xr_redo += (int64_t)fallback.size();
  std::vector<int32_t> rsrc, rcand, rdeg;
  std::vector<int64_t> rdest;
  {
    // index of each overflowed source in this call's list
    std::vector<std::pair<int32_t, int32_t>> idx(n);
    for (size_t i = 0; i < n; i++) idx[i] = {src[i], (int32_t)i};
    std::sort(idx.begin(), idx.end());
    for (int32_t v : fallback) {
      auto it = std::lower_bound(idx.begin(), idx.end(), std::make_pair(v, (int32_t)-1));
      if (it == idx.end() || it->first != v) return PPR_ERR_HIP;
      const size_t i = (size_t)it->second;
      rsrc.push_back(src[i]);
      rcand.push_back(cand[i]);
      rdeg.push_back(deg[i]);
      // (an estimate already at the candidate count still grows: with the fill target near the
      // budget a range or bucket can overflow by hash variance alone, and only more of them help)
      const int64_t grown = 4 * dest[i] + 64;
      rdest.push_back(dest[i] >= (int64_t)cand[i] ? grown : std::min<int64_t>((int64_t)cand[i], grown));
    }
  }
  return run_xhubs_list(p, a, rsrc, rcand, rdeg, rdest, maxdiff, depth + 1);
}

// the completion of a deferred run_xhubs_list: wait for the range engines, redo the overflowed
// sources (synchronously, with 4x the estimate), exactly as the undeferred call does
static int xhubs_finish(ppr_plan* p, const IterArgs& a, XhDefer& df, unsigned long long* maxdiff) {
  if (!df.live) return PPR_OK;
  df.live = false;
  hipStream_t sw = p->stream3 ? p->stream3 : p->stream;
  int32_t novf = 0;
  HIP_OK(hipMemcpyAsync(&novf, p->d_xs + df.o_ov, 4, hipMemcpyDeviceToHost, sw));
  HIP_OK(hipStreamSynchronize(sw));
  kst_fold(p, 5);
  if (!novf) return PPR_OK;
  std::vector<int32_t> od(novf);
  HIP_OK(hipMemcpyAsync(od.data(), p->d_xs + df.o_ov + 4, 4 * (size_t)novf, hipMemcpyDeviceToHost, sw));
  HIP_OK(hipStreamSynchronize(sw));
  p->xr_redo += novf;
  const std::vector<int32_t>& dsrc = *df.src;
  const std::vector<int32_t>& dcand = *df.cand;
  const std::vector<int32_t>& ddeg = *df.deg;
  const std::vector<int64_t>& ddest = *df.dest;
  std::vector<std::pair<int32_t, int32_t>> idx(dsrc.size());
  for (size_t i = 0; i < dsrc.size(); i++) idx[i] = {dsrc[i], (int32_t)i};
  std::sort(idx.begin(), idx.end());
  std::vector<int32_t> rsrc, rcand, rdeg;
  std::vector<int64_t> rdest;
  for (int32_t d : od) {
    const int32_t v = df.xv[(size_t)d];
    auto it = std::lower_bound(idx.begin(), idx.end(), std::make_pair(v, (int32_t)-1));
    if (it == idx.end() || it->first != v) return PPR_ERR_HIP;
    const size_t i = (size_t)it->second;
    rsrc.push_back(dsrc[i]);
    rcand.push_back(dcand[i]);
    rdeg.push_back(ddeg[i]);
    const int64_t grown = 4 * ddest[i] + 64;
    rdest.push_back(ddest[i] >= (int64_t)dcand[i] ? grown : std::min<int64_t>((int64_t)dcand[i], grown));
  }
  return run_xhubs_list(p, a, rsrc, rcand, rdeg, rdest, maxdiff, df.depth + 1);
}

// ---------------------------------------------------------------------------------------------
// The sieve (merge_sv.h) for sources `src` (candidate counts `cand`): one-slice sources by k_sv1 on
// stream_sv2 (largest first), multi-slice sources by k_svA -> k_svB -> k_svF on stream_sv. The
// launches are asynchronous; sieve_collect waits and returns the sources handed back.
struct SvRun {
  std::vector<int32_t> pos;  // index into the caller's source list of each descriptor
  size_t o_ovl = 0;          // offset of the overflow list in d_sv
  size_t o_os = 0;           // ... and of the small class's first overflows (redone on the device)
  size_t o_om = 0;           // ... and of the mid class's (redone on the device, large geometry)
  bool live = false;
};

static int sieve_launch(ppr_plan* p, const IterArgs& a, const std::vector<int32_t>& src,
                        const std::vector<int32_t>& cand, const std::vector<int32_t>& deg, unsigned long long* maxdiff,
                        SvRun& run) {
  const size_t n = src.size();
  run.live = false;
  if (!n) return PPR_OK;
  auto tsub = std::chrono::steady_clock::now();
  DevGraph g{p->d_rp, p->d_colx, p->n};
  const DevSlab s = dev_slab(p);
  const int Lp = p->Lp;
  // descriptor order: multi-slice sources first (descriptors [0, nm)), then the one-slice ones by
  // size class (large, mid, small), each by candidates descending in eighth-octave steps (largest
  // first keeps the tail short). A counting sort: the host plans hundreds of thousands of sources
  // per iteration while the wave tier runs, and this planning is on the critical path.
  auto klass = [&](int64_t c) { return c > p->sv_slice ? 0 : c >= p->sv_mid ? 1 : c >= p->sv_small ? 2 : 3; };
  auto step = [](int64_t c) { return std::min(255, (int)(8.0 * std::log2((double)std::max<int64_t>(1, c)))); };
  constexpr int NKEY = 4 * 256;
  std::vector<uint32_t>& cnt = p->xhs.svcnt;
  cnt.assign(NKEY + 1, 0u);
  std::vector<uint16_t>& key = p->xhs.svkey;
  key.resize(n);
  for (size_t i = 0; i < n; i++) {
    key[i] = (uint16_t)(klass(cand[i]) * 256 + (255 - step(cand[i])));
    cnt[key[i] + 1]++;
  }
  for (int k = 0; k < NKEY; k++) cnt[k + 1] += cnt[k];
  const size_t nm = cnt[256], nx = n;
  size_t cls_end[3] = {cnt[512], cnt[768], cnt[NKEY]};  // one-slice class ends (descriptor indices)
  run.pos.resize(nx);
  for (size_t i = 0; i < n; i++) run.pos[cnt[key[i]]++] = (int32_t)i;
  // SURVEY s8d bytes of a sieved source: row pointer, its successors' ids and lengths, their rows,
  // its own old row (full: L) and the new one, the length
  auto sv_algo_bytes = [&](size_t i) {
    return 8.0 + 8.0 * deg[i] + 12.0 * ((double)cand[i] - 1.0) + 24.0 * (double)p->L + 4.0;
  };
  sub_lap(p, 4, tsub);  // sieve planning: order
  std::vector<SvDesc> desc(nm);
  std::vector<SvTask> tasks;
  int64_t tg_total = 0;
  for (size_t k = 0; k < nm; k++) {
    const size_t i = (size_t)run.pos[k];
    SvDesc& d = desc[k];
    d = SvDesc{};
    d.v = src[i];
    d.S = (int32_t)std::min<int64_t>(((int64_t)cand[i] + p->sv_slice - 1) / p->sv_slice, std::max<int32_t>(1, deg[i]));
    d.factor = p->damping / (double)deg[i];
    d.gsk = (int64_t)k * SV_R * (1 << SV_LARGE.wlog);
    d.gpt = (int64_t)k * 2 * Lp;
    // every slice flushes at most its table's keys: half-full global table at worst
    d.tg = pow2_at_least(std::min<int64_t>(2 * (int64_t)d.S * (SV_LARGE.budget + SV_LARGE.threads() + 1),
                                           2 * (int64_t)cand[i] + 64));
    d.gxt = tg_total;
    tg_total += d.tg;
    for (int s2 = 0; s2 < d.S; s2++) tasks.push_back(SvTask{(int32_t)k, s2});
  }
  const size_t nt = tasks.size();
  // d_sv: node ids [nx] | multi descriptors [nm] | tasks | one-slice selections (keys, values) |
  // zeroed: ovl[1 + nx] | selected counts[nx] | oflag[nm] | gpt | gsk | gkeys | ga | gb
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  const size_t o_v = off; off = al(off + 4 * nx);
  const size_t o_d = off; off = al(off + sizeof(SvDesc) * (nm + 1));
  const size_t o_t = off; off = al(off + sizeof(SvTask) * (nt + 1));
  const size_t up = off;
  const size_t o_sk = off; off = al(off + 4 * (size_t)sv_ostride(Lp) * nx);
  const size_t o_sv = off; off = al(off + 8 * (size_t)sv_ostride(Lp) * nx);
  const size_t o_z = off;
  const size_t o_ov = off; off = al(off + 4 * (1 + nx));
  const size_t o_os = off; off = al(off + 4 * (1 + nx));  // small class's first overflows (device redo)
  const size_t o_om = off; off = al(off + 4 * (1 + nx));  // mid class's first overflows (device redo)
  const size_t o_sn = off; off = al(off + 4 * nx);
  const size_t o_of = off; off = al(off + 4 * (nm + 1));
  const size_t o_pt = off; off = al(off + 8 * 2 * (size_t)Lp * nm);
  const size_t o_gs = off; off = al(off + 4 * (size_t)SV_R * ((size_t)1 << SV_LARGE.wlog) * nm);
  const size_t o_gk = off; off = al(off + 4 * (size_t)tg_total);
  const size_t o_ga = off; off = al(off + 8 * (size_t)tg_total);
  const size_t o_gb = off; off = al(off + 8 * (size_t)tg_total);
  const size_t total = off;
  { int r = ensure_dev(&p->d_sv, &p->sv_bytes, total); if (r) return r; }
  { int r = ensure_pinned(&p->h_sv_pin, &p->h_sv_bytes, up); if (r) return r; }
  unsigned char* hb = (unsigned char*)p->h_sv_pin;
  int32_t* hv = (int32_t*)(hb + o_v);
  for (size_t k = 0; k < nx; k++) hv[k] = src[(size_t)run.pos[k]];
  if (nm) std::memcpy(hb + o_d, desc.data(), sizeof(SvDesc) * nm);
  if (nt) std::memcpy(hb + o_t, tasks.data(), sizeof(SvTask) * nt);
  unsigned char* b = p->d_sv;
  hipStream_t s1 = p->stream_sv, s2 = p->stream_sv2, s3 = p->stream_sv3;
  // descriptors up and the zeroed region cleared on the mid class's stream (the plan stream: idle
  // once the classification is read), the other sieve streams wait for it
  sub_lap(p, 5, tsub);  // sieve planning: descriptors + staging
  HIP_OK(hipMemcpyAsync(b, hb, up, hipMemcpyHostToDevice, s3));
  HIP_OK(hipMemsetAsync(b + o_z, 0, total - o_z, s3));
  HIP_OK(hipEventRecord(p->ev_sv, s3));
  if (s1 != s3) HIP_OK(hipStreamWaitEvent(s1, p->ev_sv, 0));
  if (s2 != s3) HIP_OK(hipStreamWaitEvent(s2, p->ev_sv, 0));
  const int32_t* d_v = (const int32_t*)(b + o_v);
  const SvDesc* d_d = (const SvDesc*)(b + o_d);
  const SvTask* d_t = (const SvTask*)(b + o_t);
  int32_t* d_ov = (int32_t*)(b + o_ov);
  int32_t* d_os = (int32_t*)(b + o_os);
  int32_t* d_om = (int32_t*)(b + o_om);
  int32_t* d_of = (int32_t*)(b + o_of);
  unsigned long long* d_pt = (unsigned long long*)(b + o_pt);
  uint32_t* d_sk = (uint32_t*)(b + o_gs);
  int32_t* d_ok = (int32_t*)(b + o_sk);
  double* d_ovv = (double*)(b + o_sv);
  int32_t* d_on = (int32_t*)(b + o_sn);
  uint32_t* d_gk = (uint32_t*)(b + o_gk);
  unsigned long long* d_ga = (unsigned long long*)(b + o_ga);
  unsigned long long* d_gb = (unsigned long long*)(b + o_gb);
  const size_t lds = sv_lds_bytes(Lp, SV_LARGE);
  {
    // one-slice classes beside the multi-slice chain (stream_sv): large on stream_sv2, mid then
    // small on stream_sv3 (the mid class ends long before the large one; the small class's 40-KB
    // workgroups fill the LDS the 116-KB ones leave; behind the large class it ran alone at the end
    // of the iteration: round 6, -0.5 % per job)
    const SvGeom geo[3] = {SV_LARGE, SV_MID, SV_SMALL};
    hipStream_t cs[3] = {s2, s3, s3};
    size_t c0 = nm;
    for (int c = 0; c < 3; c++) {
      const size_t cnt_c = cls_end[c] - c0;
      const int d0 = (int)c0;
      double bytes = 0.0;
      for (size_t k = c0; k < cls_end[c]; k++) bytes += sv_algo_bytes((size_t)run.pos[k]);
      c0 = cls_end[c];
      if (!cnt_c) continue;
      const SvGeom G = geo[c];
      kst_begin(p, 1 + c, cs[c]);
      // the small class's overflows are redone at once with the mid geometry (it hands back ~7 % of
      // its sources, the mid class < 0.5 %); only a second overflow reaches the host
      const bool redo = c == 2 && p->sv_redo_mid;
      // the mid class's overflows (< 10 % of its sources; with the small class's second ones, most
      // of the host hand-backs) are redone at once with the large geometry
      const bool redo_l = c == 1 && p->sv_redo_large;
      hipLaunchKernelGGL(k_sv1, dim3((unsigned)cnt_c), dim3(G.threads()), sv_lds_bytes(Lp, G), cs[c], g, s, a, d_v, d0,
                         Lp, G, std::min(p->sv_budget, G.budget), redo ? d_os : redo_l ? d_om : d_ov, d_ok, d_ovv,
                         d_on);
      HIP_OK(hipGetLastError());
      if (redo_l) {
        // (grid: the class overflows ~7 % of its sources at RMAT-22; past the grid the host takes them)
        const unsigned gl = (unsigned)std::min<size_t>(cnt_c, cnt_c / 8 + 64);
        hipLaunchKernelGGL(k_sv1_list, dim3(gl), dim3(SV_LARGE.threads()), sv_lds_bytes(Lp, SV_LARGE), cs[c],
                           g, s, a, d_v, d_om, Lp, SV_LARGE, std::min(p->sv_budget, SV_LARGE.budget), d_ov, d_ok, d_ovv,
                           d_on);
        HIP_OK(hipGetLastError());
        p->merge_launches++;
      }
      if (redo) {
        hipLaunchKernelGGL(k_sv1_redo, dim3((unsigned)std::min<size_t>(cnt_c, 512)), dim3(SV_MID.threads()),
                           sv_lds_bytes(Lp, SV_MID), cs[c], g, s, a, d_v, d_os, Lp, SV_MID,
                           std::min(p->sv_budget, SV_MID.budget), d_ov, d_ok, d_ovv, d_on);
        HIP_OK(hipGetLastError());
        p->merge_launches++;
      }
      hipLaunchKernelGGL(k_svfin, dim3((unsigned)cnt_c), dim3(64), svfin_lds_bytes(Lp), cs[c], s, a, d_v, d0, d_ok,
                         d_ovv, d_on, Lp, maxdiff, p->d_stats);
      HIP_OK(hipGetLastError());
      kst_end(p, 1 + c, cs[c], bytes);
      p->merge_launches += 2;
    }
  }
  if (nm) {
    double bytes = 0.0;
    for (size_t k = 0; k < nm; k++) bytes += sv_algo_bytes((size_t)run.pos[k]);
    kst_begin(p, 4, s1);
    hipLaunchKernelGGL(k_svA, dim3((unsigned)nt), dim3(SV_THREADS), lds, s1, g, s, a, d_d, d_t, Lp, d_sk, d_pt);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_svB, dim3((unsigned)nt), dim3(SV_THREADS), lds, s1, g, s, a, d_d, d_t, Lp, p->sv_budget, d_sk,
                       d_pt, d_gk, d_ga, d_gb, d_of);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(k_svF, dim3((unsigned)nm), dim3(256), svf_lds_bytes(Lp), s1, s, a, d_d, Lp, d_pt, d_gk, d_ga,
                       d_gb, d_of, d_ov, maxdiff, p->d_stats);
    HIP_OK(hipGetLastError());
    kst_end(p, 4, s1, bytes);
    p->merge_launches += 3;
  }
  sub_lap(p, 6, tsub);  // sieve planning: launches
  p->sv_sources += (int64_t)nx;
  run.o_ovl = o_ov;
  run.o_os = o_os;
  run.o_om = o_om;
  run.live = true;
  return PPR_OK;
}

// wait for the sieve, append the sources it handed back (table overflows) to `back`, as indices
// into the list sieve_launch was given
static int sieve_collect(ppr_plan* p, SvRun& run, std::vector<int32_t>& back) {
  if (!run.live) return PPR_OK;
  run.live = false;
  if (p->stream_sv2 != p->stream_sv) {
    HIP_OK(hipEventRecord(p->ev_sv, p->stream_sv2));
    HIP_OK(hipStreamWaitEvent(p->stream_sv, p->ev_sv, 0));
  }
  if (p->stream_sv3 != p->stream_sv) {
    HIP_OK(hipEventRecord(p->ev_sv, p->stream_sv3));
    HIP_OK(hipStreamWaitEvent(p->stream_sv, p->ev_sv, 0));
  }
  int32_t novf = 0, nsm = 0, nmd = 0;
  HIP_OK(hipMemcpyAsync(&novf, p->d_sv + run.o_ovl, 4, hipMemcpyDeviceToHost, p->stream_sv));
  HIP_OK(hipMemcpyAsync(&nsm, p->d_sv + run.o_os, 4, hipMemcpyDeviceToHost, p->stream_sv));
  HIP_OK(hipMemcpyAsync(&nmd, p->d_sv + run.o_om, 4, hipMemcpyDeviceToHost, p->stream_sv));
  HIP_OK(hipStreamSynchronize(p->stream_sv));
  p->sv_redo_dev += nsm + nmd;
  for (int g = 1; g < ppr_plan::NKST; g++) kst_fold(p, g);
  if (!novf) return PPR_OK;
  std::vector<int32_t> od(novf);
  HIP_OK(hipMemcpyAsync(od.data(), p->d_sv + run.o_ovl + 4, 4 * (size_t)novf, hipMemcpyDeviceToHost, p->stream_sv));
  HIP_OK(hipStreamSynchronize(p->stream_sv));
  for (int32_t d : od) back.push_back(run.pos[(size_t)d]);
  p->sv_redo += novf;
  return PPR_OK;
}

// the exact-sum merge of the `count` sources of device list `d_list` (hub tier, or any tier the
// plan leaves without a wave kernel): candidate counts, degrees, last distinct counts and current
// row lengths gathered on the device; sources with a full current row go through the sieve
// (merge_sv.h), the others -- and any the sieve hands back -- through the range / partition
// engines with the distinct-key estimate planned on the host
static int run_xhubs(ppr_plan* p, const IterArgs& a, const int32_t* d_list, int64_t count, unsigned long long* maxdiff) {
  if (count <= 0) return PPR_OK;
  auto now = [] { return std::chrono::steady_clock::now(); };
  double lapv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto lap = [&](int k, std::chrono::steady_clock::time_point& t) {
    const auto t2 = now();
    const double d = std::chrono::duration<double>(t2 - t).count();
    p->xh_s[k] += d;
    lapv[k] += d;
    t = t2;
  };
  auto tl = now();
  const auto t_in = tl;
  struct LapLog {  // PPR_SV_LOG: this call's host phases (ms), printed when it returns
    ppr_plan* p; const IterArgs& a; double* v; std::chrono::steady_clock::time_point t0;
    ~LapLog() {
      if (!getenv("PPR_SV_LOG")) return;
      const double tot = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      fprintf(stderr, "ppr_xh_laps it %d total %.2f gather %.2f classify %.2f sieve_launch %.2f engines %.2f "
              "sieve_wait %.2f handback %.2f\n", a.iter, 1e3 * tot, 1e3 * v[0], 1e3 * v[1], 1e3 * v[2], 1e3 * v[3],
              1e3 * v[4], 1e3 * (v[5] + v[6]));
      const double* u = p->xh_sub;
      fprintf(stderr, "ppr_xh_sub it %d range classes %.2f descriptors %.2f staging %.2f launches %.2f sieve order %.2f "
              "descriptors+staging %.2f launches %.2f\n", a.iter, 1e3 * u[0], 1e3 * u[1], 1e3 * u[2], 1e3 * u[3],
              1e3 * u[4], 1e3 * u[5], 1e3 * u[6]);
      for (int k = 0; k < 8; k++) p->xh_sub[k] = 0.0;
    }
  } laplog{p, a, lapv, t_in};
  hipStream_t st = p->stream;
  const size_t nh = (size_t)count;
  {
    size_t capb = p->h_hub_cap * 12;
    void* ptr = p->h_hub_pin;
    int r = ensure_pinned(&ptr, &capb, 20 * nh);
    if (r) return r;
    p->h_hub_pin = (int32_t*)ptr;
    p->h_hub_cap = capb / 12;
  }
  if (4 * nh > (size_t)p->n) { int r = ensure_dev((unsigned char**)&p->d_gath, &p->gath_bytes, 16 * nh); if (r) return r; }
  int32_t* d_g = 4 * nh > (size_t)p->n ? p->d_gath : p->d_ovf;
  int32_t* h = p->h_hub_pin;
  HIP_OK(hipMemcpyAsync(h, d_list, 4 * nh, hipMemcpyDeviceToHost, st));
  hipLaunchKernelGGL(k_gather_sv, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, d_list, (int64_t)nh,
                     p->d_cand, p->d_rp, (const int32_t*)p->d_dlast, dev_slab(p), a, d_g);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(h + nh, d_g, 16 * nh, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  std::vector<int32_t>& hcopy = p->xhs.h;  // (the pinned buffer is restaged by later calls)
  hcopy.assign(h, h + 5 * nh);
  h = hcopy.data();
  lap(0, tl);  // gather + copy back
  const bool sieve = p->sv_enabled && a.xs && !a.unit && !a.mc && p->hot_n == 0;
  std::vector<int32_t>& src = p->xhs.src; std::vector<int32_t>& cand = p->xhs.cand;
  std::vector<int32_t>& deg = p->xhs.deg; std::vector<int32_t>& ssrc = p->xhs.ssrc;
  std::vector<int32_t>& scand = p->xhs.scand; std::vector<int32_t>& sdeg = p->xhs.sdeg;
  std::vector<int32_t>& sidx = p->xhs.sidx;
  std::vector<int64_t>& dest = p->xhs.dest;
  src.clear(); cand.clear(); deg.clear(); ssrc.clear(); scand.clear(); sdeg.clear(); sidx.clear(); dest.clear();
  // distinct keys expected: the last merge's count (rows change little between updates) plus a
  // margin, else (first merge) 60 % of the candidates; never more than the candidates + 1
  auto estimate = [&](size_t i) {
    const int64_t dl = h[3 * nh + i];
    const int64_t c = (int64_t)h[nh + i];
    int64_t x = std::min<int64_t>(c, dl > 0 ? dl + dl / 8 + 64 : c * 3 / 5 + 64);
    if (p->xr_dscale != 100) x = std::max<int64_t>(1, x * p->xr_dscale / 100);
    return x;
  };
  src.reserve(nh); cand.reserve(nh); deg.reserve(nh); dest.reserve(nh);
  if (sieve) { ssrc.reserve(nh); scand.reserve(nh); sdeg.reserve(nh); sidx.reserve(nh); }
  for (size_t i = 0; i < nh; i++) {
    const int32_t c = h[nh + i];
    if (sieve && h[4 * nh + i] == (int32_t)p->L && c >= p->sv_min && c < (1 << 30)) {
      ssrc.push_back(h[i]);
      scand.push_back(c);
      sdeg.push_back(h[2 * nh + i]);
      sidx.push_back((int32_t)i);
    } else {
      src.push_back(h[i]);
      cand.push_back(c);
      deg.push_back(h[2 * nh + i]);
      dest.push_back(estimate(i));
    }
  }
  lap(1, tl);  // classification
  SvRun run;
  // the larger of the two host plannings goes second: when the range engines take more sources
  // than the sieve (the big partition's iterations: ~258 K mid-sized sources at RMAT-22), they are
  // planned and queued first and collected after the sieve's launches (PPR_XH_FIRST=0: sieve first)
  XhDefer df;
  df.want = p->xh_first && src.size() > ssrc.size();
  if (df.want) { int r = run_xhubs_list(p, a, src, cand, deg, dest, maxdiff, 0, &df); if (r) return r; }
  if (!ssrc.empty()) { int r = sieve_launch(p, a, ssrc, scand, sdeg, maxdiff, run); if (r) return r; }
  lap(2, tl);  // sieve planning + launches
  if (df.want) {
    int r = xhubs_finish(p, a, df, maxdiff);
    if (r) return r;
  } else if (!src.empty()) {
    int r = run_xhubs_list(p, a, src, cand, deg, dest, maxdiff, 0);
    if (r) return r;
  }
  lap(3, tl);  // range / partition engines (their syncs included)
  std::vector<int32_t>& back = p->xhs.back;
  back.clear();
  const int64_t dev0 = p->sv_redo_dev;
  { int r = sieve_collect(p, run, back); if (r) return r; }
  lap(4, tl);  // waiting for the sieve
  if (getenv("PPR_SV_LOG"))
    fprintf(stderr, "ppr_sv_log it %d sieved %zu range %zu dev_redo %lld handed_back %zu\n", a.iter, ssrc.size(),
            src.size(), (long long)(p->sv_redo_dev - dev0), back.size());
  if (back.empty()) return PPR_OK;
  // handed back: the range / partition engines, with the usual estimate
  src.clear(); cand.clear(); deg.clear(); dest.clear();
  for (int32_t k : back) {
    const size_t i = (size_t)sidx[(size_t)k];
    src.push_back(h[i]);
    cand.push_back(h[nh + i]);
    deg.push_back(h[2 * nh + i]);
    dest.push_back(estimate(i));
  }
  lap(5, tl);  // hand-back planning
  const int r = run_xhubs_list(p, a, src, cand, deg, dest, maxdiff, 0);
  lap(6, tl);  // hand-backs merged
  return r;
}

// classify + launch all tiers for `count` sources of `list`; the span is timed with events on
// the plan's stream and added to merge_ms (iterations only, not init)
int run_merge(ppr_plan* p, const IterArgs& a, const int32_t* list, int64_t count,
              unsigned long long* maxdiff) {
  if (count <= 0) return PPR_OK;
  // MC combine levels are timed as a whole by the caller: no per-level event sync
  if (!a.mc) HIP_OK(hipEventRecord(p->ev_m0, p->stream));
  p->wave_x_launched = false;
  int rc = run_merge_impl(p, a, list, count, maxdiff);
  if (p->stream_wave && p->stream_wave != p->stream) {  // the wave tiers ran on their own stream
    HIP_OK(hipEventRecord(p->ev_wave, p->stream_wave));
    HIP_OK(hipStreamWaitEvent(p->stream, p->ev_wave, 0));
  }
  if (!rc && p->wave_x_launched) {
    // exact wave tier: sources whose table ran out (only with PPR_WAVE_TDIV: the tables hold 4/3 of
    // the tier's candidate cap) wrote no row; the workgroup engines merge them again
    int32_t nw = 0;
    HIP_OK(hipMemcpyAsync(&nw, p->d_wovl, 4, hipMemcpyDeviceToHost, p->stream));
    HIP_OK(hipStreamSynchronize(p->stream));
    if (nw) {
      p->wave_redo += nw;
      rc = run_xhubs(p, a, p->d_wovl + 1, nw, maxdiff);
    }
  }
  if (rc || a.mc) return rc;
  HIP_OK(hipEventRecord(p->ev_m1, p->stream));
  HIP_OK(hipEventSynchronize(p->ev_m1));
  kst_fold(p, 0);
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, p->ev_m0, p->ev_m1));
  if (!a.unit) p->merge_ms += ms;
  return PPR_OK;
}

// HBM-table path (k_merge_glb) for sources beyond every LDS tier and LDS-table overflows
static int run_glb(ppr_plan* p, const IterArgs& a, std::vector<int32_t>& big, unsigned long long* maxdiff) {
  hipStream_t st = p->stream;
  DevGraph g{p->d_rp, p->d_colx, p->n};
  const DevSlab s = dev_slab(p);
  if (big.empty()) return PPR_OK;
  std::vector<int32_t> cand(p->n);
  HIP_OK(hipMemcpyAsync(cand.data(), p->d_cand, 4 * (size_t)p->n, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  // batches bounded by a scratch budget: slots * (4+8) * 2 (table + compacted copy)
  const size_t budget_slots = (size_t)1 << 26;  // 64 Mi slots -> 1.5 GiB
  size_t i0 = 0;
  while (i0 < big.size()) {
    std::vector<GlbWork> work;
    int64_t off = 0;
    size_t i = i0;
    while (i < big.size()) {
      const int64_t T = pow2_at_least(std::max<int64_t>(2 * (int64_t)cand[big[i]], 64));
      if (!work.empty() && (size_t)(off + T) > budget_slots) break;
      work.push_back(GlbWork{big[i], 0, off, T});
      off += T;
      i++;
    }
    const size_t need = (size_t)off * 24;
    if (need > p->scratch_bytes) {
      hipFree(p->d_scratch);
      p->d_scratch = nullptr;
      if (hipMalloc(&p->d_scratch, need) != hipSuccess) return PPR_ERR_OOM;
      p->scratch_bytes = need;
    }
    if ((int64_t)work.size() > p->work_cap) {
      hipFree(p->d_work);
      if (hipMalloc((void**)&p->d_work, sizeof(GlbWork) * work.size()) != hipSuccess) return PPR_ERR_OOM;
      p->work_cap = (int64_t)work.size();
    }
    HIP_OK(hipMemcpyAsync(p->d_work, work.data(), sizeof(GlbWork) * work.size(), hipMemcpyHostToDevice, st));
    int32_t* gkeys = (int32_t*)p->d_scratch;
    double* gacc = (double*)((char*)p->d_scratch + (size_t)off * 4);
    int32_t* ckeys = (int32_t*)((char*)p->d_scratch + (size_t)off * 12);
    double* cacc = (double*)((char*)p->d_scratch + (size_t)off * 16);
    const size_t lds = (size_t)p->Lp * 12 + 1024 + (size_t)p->Lp * 4 * 5;
    hipLaunchKernelGGL(k_merge_glb, dim3((unsigned)work.size()), dim3(64), lds, st, g, s, a,
                       p->d_work, (int64_t)work.size(), gkeys, gacc, ckeys, cacc, p->Lp, maxdiff,
                       p->d_stats);
    HIP_OK(hipGetLastError());
    p->merge_launches++;
    HIP_OK(hipStreamSynchronize(st));  // work/scratch reused by the next batch
    i0 = i;
  }
  return PPR_OK;
}

// an MC level's deferred hub overflow list (run_hubs): read it (host sync) and redo those sources
static int flush_ovl(ppr_plan* p, const IterArgs& a, unsigned long long* maxdiff) {
  int32_t* ovl = p->ovl_pending;
  if (!ovl) return PPR_OK;
  p->ovl_pending = nullptr;
  hipStream_t st = p->stream;
  int32_t novf = 0;
  HIP_OK(hipMemcpyAsync(&novf, ovl, 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (!novf) return PPR_OK;
  if (p->d_diag) fprintf(stderr, "ppr_diag: deferred hub overflow redo %d\n", novf);
  std::vector<int32_t> big(novf);
  HIP_OK(hipMemcpyAsync(big.data(), ovl + 1, 4 * (size_t)novf, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  return run_glb(p, a, big, maxdiff);
}

int run_merge_flush(ppr_plan* p, const IterArgs& a, unsigned long long* maxdiff) {
  return flush_ovl(p, a, maxdiff);
}

static int run_merge_impl(ppr_plan* p, const IterArgs& a, const int32_t* list, int64_t count,
                          unsigned long long* maxdiff) {
  hipStream_t st = p->stream;
  DevGraph g{p->d_rp, p->d_colx, p->n};
  const DevSlab s = dev_slab(p);
  // small MC levels: classification, the hub sources' gather and the previous level's deferred
  // overflow count come back in one host sync (the combine's ~1800 levels are latency-bound)
  const bool fused = a.mc && count <= p->fused_max && GATHER_HDR + 3 * count <= p->n;
  if (!fused) {
    int r = flush_ovl(p, a, maxdiff);
    if (r) return r;
  } else {
    size_t capb = p->h_hub_cap * 12;
    void* ptr = p->h_hub_pin;
    int r = ensure_pinned(&ptr, &capb, 4 * (GATHER_HDR + 3 * (size_t)count));
    if (r) return r;
    p->h_hub_pin = (int32_t*)ptr;
    p->h_hub_cap = capb / 12;
  }
reclassify:
  HIP_OK(hipMemsetAsync(p->d_tier_cnt, 0, sizeof(uint32_t) * (NLISTS + 2), st));
  const int cls_pw = count <= CLS_SMALL ? 1 : CLS_PER_WAVE;
  const int64_t cls_pb = (int64_t)cls_pw * WAVES_PER_BLOCK;
  const int64_t nb = (count + cls_pb - 1) / cls_pb;
  hipLaunchKernelGGL(k_classify, dim3((unsigned)nb), dim3(256), 0, st, g, s, a, list, count,
                     p->d_tier_cap, p->d_tier_lists, p->d_tier_cnt, p->n, p->d_cand, p->d_stats, p->d_big, cls_pw,
                     (p->wave_by_d && a.xs && !a.unit && !a.mc) ? (const int32_t*)p->d_dlast : nullptr);
  HIP_OK(hipGetLastError());
  if (!a.unit && p->max_deg > CLS_BIG_DEG) {
    // grid-stride over the long-list sources, at most one block per listed source
    hipLaunchKernelGGL(k_classify_big, dim3((unsigned)std::min<int64_t>(256, count)), dim3(CLS_BIG_THREADS), 0, st, g,
                       s, a, p->d_tier_cap,
                       p->d_tier_lists, p->d_tier_cnt, p->n, p->d_cand, p->d_stats, p->d_big,
                       (p->wave_by_d && a.xs && !a.unit && !a.mc) ? (const int32_t*)p->d_dlast : nullptr);
  }
  HIP_OK(hipGetLastError());
  uint32_t cnt[NLISTS + 1];
  if (fused) {
    static_assert(NLISTS + 1 < GATHER_HDR, "tier counters and the pending count fit the header");
    hipLaunchKernelGGL(k_gather_cand_deg_dev, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st,
                       p->d_tier_lists + (int64_t)TIER_BIG * p->n, p->d_tier_cnt, NLISTS + 1, TIER_BIG,
                       p->ovl_pending, count, p->d_cand, p->d_rp, p->d_ovf);
    HIP_OK(hipGetLastError());
    // one copy: counters, pending overflow count, hub list, candidate counts, degrees
    HIP_OK(hipMemcpyAsync(p->h_hub_pin, p->d_ovf, 4 * (GATHER_HDR + 3 * (size_t)count), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    std::memcpy(cnt, p->h_hub_pin, sizeof(cnt));
    const int32_t pend = p->h_hub_pin[NLISTS + 1];
    if (p->ovl_pending) {
      if (pend) {  // the previous level left sources to redo: their rows feed this classification
        int r = flush_ovl(p, a, maxdiff);
        if (r) return r;
        goto reclassify;
      }
      p->ovl_pending = nullptr;
    }
  } else {
    HIP_OK(hipMemcpyAsync(cnt, p->d_tier_cnt, sizeof(cnt), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  // the classification is complete (host sync): the wave tiers need no event to start on their stream
  hipStream_t sw = p->stream_wave ? p->stream_wave : st;
  bool wave_ev = false;
  // split wave tiers (exact sum): every tier's lists in one region, reused tier after tier (walk,
  // then its rows); a tier whose lists would pass wl_max bytes goes in chunks. (Queueing every
  // tier's walk before the first row kernel, one region per tier, measured neutral: round 6.)
  WList wls[NT];
  const int wcap = p->wave_cap ? std::max<int>((int)p->L, p->wave_cap) : 2 * p->Lp;
  const size_t wrec = (size_t)wcap * 12 + 4;  // list bytes per source
  const int64_t wchunk = std::max<int64_t>(1, (int64_t)((p->wl_max - 512) / wrec));  // sources per chunk
  {
    int64_t most = 0;
    for (int t = 0; t < NT; t++) {
      wls[t] = WList{nullptr, nullptr, nullptr, 0};
      const int split_T = a.xs ? p->wave_split_T : a.mc ? p->wave_split_mc : p->wave_split_chain;
      if (!cnt[t] || !p->tierT[t] || a.unit || split_T <= 0 || std::max(64, p->tierT[t] >> p->wave_tdiv) < split_T)
        continue;
      wls[t].cap = wcap;
      most = std::max<int64_t>(most, std::min<int64_t>((int64_t)cnt[t], wchunk));
    }
    if (most) {
      int rc = ensure_dev(&p->d_wl, &p->wl_bytes, (size_t)most * wrec + 512);
      if (rc) return rc;
      const size_t nk = (size_t)most * (size_t)wcap;
      for (int t = 0; t < NT; t++)
        if (wls[t].cap) {
          wls[t].v = reinterpret_cast<double*>(p->d_wl);
          wls[t].k = reinterpret_cast<int32_t*>(p->d_wl + nk * 8);
          wls[t].n = reinterpret_cast<int32_t*>(p->d_wl + nk * 12);
        }
    }
  }
#ifndef PPR_WFIN_WPB
#define PPR_WFIN_WPB 1  // (round 6: one source per block, -0.2 to -0.4 % against 4 in 4 same-box pairs)
#endif
  auto launch_wfin = [&](const int32_t* tl, int64_t c, const WList& wl) {
    constexpr int wpb = PPR_WFIN_WPB;  // sources (waves) per block
    hipLaunchKernelGGL(k_wfin, dim3((unsigned)((c + wpb - 1) / wpb)), dim3(64 * wpb), wfin_lds_bytes(p->Lp) * wpb, sw, s,
                       a, tl, c, wl, p->Lp, maxdiff, p->d_stats);
    p->merge_launches++;
  };
  for (int t = 0; t < NT; t++) {
    if (!cnt[t] || !p->tierT[t]) continue;
    if (!wave_ev && !a.unit && !a.mc) { kst_begin(p, 0, sw); wave_ev = true; }
    // one wave per block by default: no LDS left unusable by a 4-wave block granularity
    const int wpb = p->wave_wpb;
    const int64_t blocks = ((int64_t)cnt[t] + wpb - 1) / wpb;
    if (a.xs) {
      if (!p->wave_x_launched) HIP_OK(hipMemsetAsync(p->d_wovl, 0, 4, sw));
      p->wave_x_launched = true;
      const int Tw = std::max(64, p->tierT[t] >> p->wave_tdiv);  // (PPR_WAVE_TDIV: tests of the overflow redo)
      // the tables end after their compaction: the row in k_wfin (merge_xs.h WList)
      const WList wl = wls[t];
      const bool split = wl.cap != 0;
      const int32_t* tl = p->d_tier_lists + (int64_t)t * p->n;
      const size_t wlds = split ? lds_wave_bytes_xs(Tw) : lds_wave_bytes_x(Tw, p->Lp);
      const int64_t step = split ? wchunk : (int64_t)cnt[t];
      for (int64_t c0 = 0; c0 < (int64_t)cnt[t]; c0 += step) {
        const int64_t c = std::min<int64_t>(step, (int64_t)cnt[t] - c0);
        hipLaunchKernelGGL(split ? k_merge_lds_x<true> : k_merge_lds_x<false>, dim3((unsigned)((c + wpb - 1) / wpb)),
                           dim3(64 * wpb), wlds * wpb, sw, g, s, a, tl + c0, c, Tw, p->Lp, maxdiff, p->d_stats,
                           p->d_dlast, p->d_wovl, wl);
        if (split) {
          HIP_OK(hipGetLastError());
          launch_wfin(tl + c0, c, wl);
        }
      }
    } else {
      const int Tw = std::max(64, p->tierT[t] >> p->wave_tdiv);  // (PPR_WAVE_TDIV: tests of the bounded probes)
      const WList wl = wls[t];
      const bool split = wl.cap != 0;
      const int32_t* tl = p->d_tier_lists + (int64_t)t * p->n;
      const size_t bytes = (split ? lds_wave_bytes_s(Tw) : lds_wave_bytes(Tw, p->Lp)) * wpb;
      const bool hk = p->hot_n > 0;
      const int64_t step = split ? wchunk : (int64_t)cnt[t];
      for (int64_t c0 = 0; c0 < (int64_t)cnt[t]; c0 += step) {
        const int64_t c = std::min<int64_t>(step, (int64_t)cnt[t] - c0);
        hipLaunchKernelGGL(split ? (hk ? k_merge_lds<true, true> : k_merge_lds<false, true>)
                                 : (hk ? k_merge_lds<true, false> : k_merge_lds<false, false>),
                           dim3((unsigned)((c + wpb - 1) / wpb)), dim3(64 * wpb), bytes, sw, g, s, a, tl + c0, c, Tw,
                           p->Lp, maxdiff, p->d_stats, wl);
        if (split) {
          HIP_OK(hipGetLastError());
          launch_wfin(tl + c0, c, wl);
        }
      }
    }
    HIP_OK(hipGetLastError());
    p->merge_launches++;
  }
  if (wave_ev) kst_end(p, 0, sw, 0.0);  // (bytes: the device counter, read at the end of the run)
  if (a.xs) {
    // exact sum: every source no wave tier took (the hub tier, tiers the plan left without a
    // wave kernel) goes through the range / bucket workgroups -- nothing falls to the chain-order
    // HBM table
    int r = PPR_OK;
    for (int t = 0; t < NT && !r; t++)
      if (cnt[t] && !p->tierT[t]) r = run_xhubs(p, a, p->d_tier_lists + (int64_t)t * p->n, cnt[t], maxdiff);
    if (!r && cnt[TIER_WG]) r = run_xhubs(p, a, p->d_tier_lists + (int64_t)TIER_WG * p->n, cnt[TIER_WG], maxdiff);
    if (!r && cnt[TIER_BIG]) r = run_xhubs(p, a, p->d_tier_lists + (int64_t)TIER_BIG * p->n, cnt[TIER_BIG], maxdiff);
    return r;
  }
  if (cnt[TIER_WG]) {
    hipLaunchKernelGGL(k_merge_wg, dim3(cnt[TIER_WG]), dim3(WG_THREADS), p->wg_lds, st, g, s, a,
                       p->d_tier_lists + (int64_t)TIER_WG * p->n, (int64_t)cnt[TIER_WG], p->d_cand,
                       p->Lp, maxdiff, p->d_stats, p->d_ovf, p->d_tier_cnt + NLISTS, p->wg_max_passes);
    HIP_OK(hipGetLastError());
    p->merge_launches++;
    HIP_OK(hipMemcpyAsync(&cnt[NLISTS], p->d_tier_cnt + NLISTS, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  // sources beyond the workgroup tier, plus workgroup-tier overflows
  std::vector<int32_t> big;
  auto pull = [&](const int32_t* dptr, uint32_t k) -> int {
    if (!k) return PPR_OK;
    std::vector<int32_t> tmp(k);
    HIP_OK(hipMemcpyAsync(tmp.data(), dptr, 4 * (size_t)k, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    big.insert(big.end(), tmp.begin(), tmp.end());
    return PPR_OK;
  };
  for (int t = 0; t < NT; t++)
    if (cnt[t] && !p->tierT[t]) { int r = pull(p->d_tier_lists + (int64_t)t * p->n, cnt[t]); if (r) return r; }
  { int r = pull(p->d_ovf, cnt[NLISTS]); if (r) return r; }
  if (cnt[TIER_BIG] && fused) {
    // hub list and gathered counts | degrees arrived with the classification
    const size_t nh = cnt[TIER_BIG];
    if (p->hub_enabled) {
      int r = run_hubs(p, a, p->h_hub_pin + GATHER_HDR, p->h_hub_pin + GATHER_HDR + count, nh, maxdiff, big);
      if (r) return r;
    } else {
      big.insert(big.end(), p->h_hub_pin + GATHER_HDR, p->h_hub_pin + GATHER_HDR + nh);
    }
  } else if (cnt[TIER_BIG]) {
    const size_t nh = cnt[TIER_BIG];
    {
      size_t capb = p->h_hub_cap * 12;
      void* ptr = p->h_hub_pin;
      int r = ensure_pinned(&ptr, &capb, 12 * nh);
      if (r) return r;
      p->h_hub_pin = (int32_t*)ptr;
      p->h_hub_cap = capb / 12;
    }
    int32_t* hubs = p->h_hub_pin;
    int32_t* hcand = p->h_hub_pin + nh;  // | out-degrees at hcand + nh
    HIP_OK(hipMemcpyAsync(hubs, p->d_tier_lists + (int64_t)TIER_BIG * p->n, 4 * nh, hipMemcpyDeviceToHost, st));
    // candidate counts and degrees of the hub sources only (gathered on the device, so the host
    // planning loop reads them sequentially)
    if (2 * nh > (size_t)p->n) { int r = ensure_dev((unsigned char**)&p->d_gath, &p->gath_bytes, 8 * nh); if (r) return r; }
    int32_t* d_g = 2 * nh > (size_t)p->n ? p->d_gath : p->d_ovf;
    hipLaunchKernelGGL(k_gather_cand_deg, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st,
                       p->d_tier_lists + (int64_t)TIER_BIG * p->n, (int64_t)nh, p->d_cand, p->d_rp, d_g);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(hcand, d_g, 8 * nh, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (p->hub_enabled) {
      int r = run_hubs(p, a, hubs, hcand, nh, maxdiff, big);
      if (r) return r;
    } else {
      big.insert(big.end(), hubs, hubs + nh);
    }
  }
  // An MC level's deferred hub overflow list lives in d_scratch, which run_glb overwrites (and may
  // reallocate): read it and redo its sources before the HBM-table pass of this level's other
  // leftovers (same level, disjoint sources, so the order of the two does not matter)
  if (!big.empty() && p->ovl_pending) {
    int r = flush_ovl(p, a, maxdiff);
    if (r) return r;
  }
  return run_glb(p, a, big, maxdiff);
}

// a single contribution p as the exact sum stores it (merge_xs.h xs_single): floor(p * 2^F) rounded
// back to the nearest double (the 128-bit integer's conversion is correctly rounded)
static double xs_single_host(double p, int F) {
  uint64_t b;
  std::memcpy(&b, &p, 8);
  int e = (int)((b >> 52) & 0x7ffu);
  uint64_t m = b & ((1ull << 52) - 1ull);
  if (e) m |= 1ull << 52; else e = 1;
  const int sh = e - 1075 + F;
  const unsigned __int128 X = sh >= 0 ? ((unsigned __int128)m << sh) : (sh > -64 ? (unsigned __int128)(m >> -sh) : 0);
  return std::ldexp((double)X, -F);
}

// the dangling nodes' init rows (merge_glb.h k_init_dangling), on the plan stream; the seed as the
// plan's summation stores it (the exact sum's fixed point, or the chain's 1 - d as is)
static int init_dangling(ppr_plan* p, const int32_t* list, int64_t cnt) {
  if (cnt <= 0) return PPR_OK;
  const int64_t th = cnt * NRANGE;
  const double seed = p->xsum ? xs_single_host(1.0 - p->damping, XS_F) : 1.0 - p->damping;
  hipLaunchKernelGGL(k_init_dangling, dim3((unsigned)std::min<int64_t>((th + 255) / 256, 1 << 20)), dim3(256), 0,
                     p->stream, dev_slab(p), list, cnt, seed);
  HIP_OK(hipGetLastError());
  return PPR_OK;
}

extern "C" int ppr_grank_plan_init(ppr_plan* p) {
  if (!p) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  p->md_shared_it = -1;  // a new run: iteration numbers start over
  p->hot_n = 0;          // the hot set is rebuilt from this run's rows at iteration hot_at
  p->hot_built_it = -1;
  // every job plans from its own merges only: the range engines' distinct-key estimates (d_dlast,
  // the last merge's count) start over, so a repeated run is a cold call
  if (p->d_dlast) HIP_OK(hipMemsetAsync(p->d_dlast, 0, 4 * (size_t)std::max<int64_t>(1, p->n), p->stream));
  IterArgs a = iter_args(p, 0, true);
  int rc = init_dangling(p, p->d_all + p->n_nd, p->n - p->n_nd);
  if (rc) return rc;
  return run_merge(p, a, p->d_all, p->n_nd, p->d_maxdiff + PPR_MAX_ITER_STATS);
}

extern "C" int ppr_grank_plan_active_count(ppr_plan* p, int32_t it, int64_t* count) {
  if (!p || !count || it < 0) return PPR_ERR_ARG;
  *count = p->nact[it & 1];
  return PPR_OK;
}

extern "C" int ppr_grank_plan_iterate(ppr_plan* p, int32_t it, int64_t begin, int64_t end) {
  if (!p || it < 0) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  const int part = it & 1;
  begin = std::max<int64_t>(0, begin);
  end = std::min<int64_t>(p->nact[part], end);
  // once per iteration on every rank, even one whose range is empty (a sharded run all-reduces
  // every rank's maxDiff slot, and decodes the other ranks' rows through this rank's hot set)
  if (p->hot_cap > 0 && it == p->hot_at && p->hot_built_it != it) {
    int rc0 = hot_build(p, it);
    if (rc0) return rc0;
    p->hot_built_it = it;
  }
  unsigned long long* md = p->d_maxdiff + (it < PPR_MAX_ITER_STATS ? it : PPR_MAX_ITER_STATS);
  if (it >= PPR_MAX_ITER_STATS && p->md_shared_it != it) {
    // the shared slot still holds an earlier iteration's maximum (the kernels only atomicMax it)
    HIP_OK(hipMemsetAsync(md, 0, 8, p->stream));
    p->md_shared_it = it;
  }
  if (end <= begin) return PPR_OK;
  IterArgs a = iter_args(p, it, false);
  int rc = run_merge(p, a, p->d_act[part] + begin, end - begin, md);
  if (rc) return rc;
  if (a.stats) {  // bytes of the rows this iteration wrote (outside the timed merge span)
    const DevSlab s = dev_slab(p);
    const int64_t cnt = end - begin;
    const unsigned blocks = (unsigned)std::min<int64_t>((cnt + 255) / 256, 1024);
    hipLaunchKernelGGL(k_stat_written, dim3(blocks), dim3(256), 0, p->stream, s, a,
                       p->d_act[part] + begin, cnt, p->d_stats);
    HIP_OK(hipGetLastError());
  }
  return PPR_OK;
}

extern "C" int ppr_grank_plan_read_maxdiff(ppr_plan* p, int32_t it, double* maxdiff) {
  if (!p || !maxdiff || it < 0) return PPR_ERR_ARG;
  unsigned long long b = 0;
  HIP_OK(hipMemcpyAsync(&b, p->d_maxdiff + (it < PPR_MAX_ITER_STATS ? it : PPR_MAX_ITER_STATS),
                        8, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  double d;
  std::memcpy(&d, &b, 8);
  *maxdiff = d;
  return PPR_OK;
}

// this module's bounded-probe error word (ppr_device.h probe_fail): PPR_ERR_PROBE once set (and
// cleared), read once per run (a device-wide sync)
int probe_take() {
  unsigned int v = 0u;
  HIP_OK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_probe_err), sizeof(v), 0, hipMemcpyDeviceToHost));
  if (!v) return PPR_OK;
  const unsigned int z = 0u;
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe_err), &z, sizeof(z), 0, hipMemcpyHostToDevice));
  return PPR_ERR_PROBE;
}

extern "C" int ppr_grank_plan_finish(ppr_plan* p, int32_t iterations_run) {
  if (!p || iterations_run < 0) return PPR_ERR_ARG;
  if (p->n == 0) return PPR_OK;
  HIP_OK(hipSetDevice(p->device));
  const int rc = launch_topk(p, ((iterations_run + 1) / 2) & 1, (iterations_run / 2) & 1, nullptr, 0);
  if (rc) return rc;
  return probe_take();
}

int launch_topk(ppr_plan* p, int sA, int sB, const int8_t* owner, int rank) {  // (defaults: plan.h)
  if (p->n == 0) return PPR_OK;
  const DevSlab s = dev_slab(p);
  const int wpb = p->Lp <= 1024 ? 4 : 1;  // one wave per row, Lp * 12 B of LDS each
  const int64_t blocks = (p->n + wpb - 1) / wpb;
  hipLaunchKernelGGL(k_topk, dim3((unsigned)blocks), dim3(64 * wpb), (size_t)wpb * p->Lp * 12, p->stream, s,
                     p->d_part, sA, sB, (int)p->K, p->Lp, p->d_out_ids, p->d_out_sc, p->d_out_len, owner, rank);
  HIP_OK(hipGetLastError());
  return PPR_OK;
}

// per-iteration maxDiff (iterations < PPR_MAX_ITER_STATS) into st->max_diff, one copy
static int read_maxdiff_history(ppr_plan* p, uint32_t its, ppr_stats* st) {
  const uint32_t k = std::min<uint32_t>(its, PPR_MAX_ITER_STATS);
  if (!k) return PPR_OK;
  std::vector<unsigned long long> b(k);
  HIP_OK(hipMemcpyAsync(b.data(), p->d_maxdiff, 8 * (size_t)k, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  for (uint32_t i = 0; i < k; i++) std::memcpy(&st->max_diff[i], &b[i], 8);
  return PPR_OK;
}

extern "C" int ppr_grank_plan_run(ppr_plan* p, uint32_t iterations, double tolerance,
                                  ppr_stats* st) {
  if (!p) return PPR_ERR_ARG;
  if (iterations == 0) return PPR_ERR_ITERS;
  HIP_OK(hipSetDevice(p->device));
  hipStream_t s = p->stream;
  HIP_OK(hipMemsetAsync(p->d_maxdiff, 0, 8 * (PPR_MAX_ITER_STATS + 1), s));
  HIP_OK(hipMemsetAsync(p->d_stats, 0, 8 * PPR_NSTATS, s));
  p->merge_launches = 0;
  p->merge_ms = 0.0;
  kst_reset(p);
  HIP_OK(hipEventRecord(p->ev_a, s));
  int rc = ppr_grank_plan_init(p);
  if (rc) return rc;
  // stopping rule of include/grank.h:90-94,140
  double md[2] = {tolerance, tolerance};
  uint32_t it = 0;
  for (; it < iterations && std::max(md[0], md[1]) >= tolerance; it++) {
    int64_t cnt = p->nact[it & 1];
    rc = ppr_grank_plan_iterate(p, (int32_t)it, 0, cnt);
    if (rc) return rc;
    // the stop rule needs maxDiff on the host only when it can stop the loop (tolerance > 0); the
    // history for the stats is read once at the end
    if (tolerance > 0) {
      double d = 0.0;
      rc = ppr_grank_plan_read_maxdiff(p, (int32_t)it, &d);
      if (rc) return rc;
      md[0] = d;
      std::swap(md[0], md[1]);
    }
  }
  rc = ppr_grank_plan_finish(p, (int32_t)it);
  if (rc) return rc;
  HIP_OK(hipEventRecord(p->ev_b, s));
  HIP_OK(hipEventSynchronize(p->ev_b));
  if (st) {
    rc = read_maxdiff_history(p, it, st);
    if (rc) return rc;
    float ms = 0;
    hipEventElapsedTime(&ms, p->ev_a, p->ev_b);
    st->iterations_run = (int32_t)it;
    st->device_ms = ms;
    st->merge_ms = p->merge_ms;
    unsigned long long sv[3];
    HIP_OK(hipMemcpyAsync(sv, p->d_stats, 24, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    st->candidates = (int64_t)sv[0];
    st->algo_bytes = (int64_t)sv[1];
    st->merge_launches = p->merge_launches;
    p->kst_bytes[0] = (double)sv[2];
  }
  return PPR_OK;
}

extern "C" int ppr_grank_plan_kernel_stats(ppr_plan* p, int32_t n, double* bytes, double* ms, int64_t* launches) {
  if (!p || n < 0) return PPR_ERR_ARG;
  for (int g = 0; g < n && g < ppr_plan::NKST; g++) {
    if (bytes) bytes[g] = p->kst_bytes[g];
    if (ms) ms[g] = p->kst_ms[g];
    if (launches) launches[g] = p->kst_launches[g];
  }
  return PPR_OK;
}

extern "C" int ppr_grank_plan_fetch(ppr_plan* p, int32_t* out_ids, double* out_scores,
                                    int32_t* out_len) {
  if (!p) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  const size_t nk = (size_t)p->n * p->K;
  if (out_ids) HIP_OK(hipMemcpyAsync(out_ids, p->d_out_ids, 4 * nk, hipMemcpyDeviceToHost, p->stream));
  if (out_scores) HIP_OK(hipMemcpyAsync(out_scores, p->d_out_sc, 8 * nk, hipMemcpyDeviceToHost, p->stream));
  if (out_len) HIP_OK(hipMemcpyAsync(out_len, p->d_out_len, 4 * (size_t)p->n, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  return PPR_OK;
}

extern "C" int ppr_grank_plan_fetch_rows(ppr_plan* p, int64_t begin, int64_t end, int32_t* out_ids,
                                         double* out_scores, int32_t* out_len) {
  if (!p || begin < 0 || end < begin || end > p->n) return PPR_ERR_ARG;
  if (end == begin) return PPR_OK;
  HIP_OK(hipSetDevice(p->device));
  const size_t K = p->K, r0 = (size_t)begin, c = (size_t)(end - begin);
  if (out_ids) HIP_OK(hipMemcpyAsync(out_ids, p->d_out_ids + r0 * K, 4 * c * K, hipMemcpyDeviceToHost, p->stream));
  if (out_scores)
    HIP_OK(hipMemcpyAsync(out_scores, p->d_out_sc + r0 * K, 8 * c * K, hipMemcpyDeviceToHost, p->stream));
  if (out_len) HIP_OK(hipMemcpyAsync(out_len, p->d_out_len + r0, 4 * c, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  return PPR_OK;
}

extern "C" int ppr_host_alloc(int64_t bytes, void** out) {
  if (!out || bytes < 0) return PPR_ERR_ARG;
  *out = nullptr;
  if (bytes == 0) return PPR_OK;
  return hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault) == hipSuccess ? PPR_OK : PPR_ERR_OOM;
}

extern "C" void ppr_host_free(void* ptr) {
  if (ptr) (void)hipHostFree(ptr);
}

extern "C" int ppr_grank_plan_fetch_slab(ppr_plan* p, int32_t iterations_run, int32_t* ids,
                                         double* scores, int32_t* len) {
  if (!p || iterations_run < 0) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  const int sA = ((iterations_run + 1) / 2) & 1, sB = (iterations_run / 2) & 1;
  hipStream_t st = p->stream;
  HIP_OK(hipStreamSynchronize(st));  // the plan's stream is non-blocking: drain it first
  std::vector<uint8_t> part(p->n);
  if (p->n) {
    HIP_OK(hipMemcpyAsync(part.data(), p->d_part, p->n, hipMemcpyDeviceToHost, st));
  }
  const size_t L = p->L;
  for (int sl = 0; sl < 2; sl++) {
    // copy the slot wholesale, then keep rows whose partition reads this slot
    std::vector<int32_t> ti(p->n * L), tl(p->n);
    std::vector<double> ts(p->n * L);
    if (p->n) {
      HIP_OK(hipMemcpyAsync(ti.data(), p->d_ids + (size_t)sl * p->n * L, 4 * p->n * L, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(ts.data(), p->d_sc + (size_t)sl * p->n * L, 8 * p->n * L, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(tl.data(), p->d_len + (size_t)sl * p->n, 4 * p->n, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
    }
    // rows are stored in hash order: hand them out sorted by (score desc, id asc)
    std::vector<std::pair<double, int32_t>> row(L);
    for (int64_t v = 0; v < p->n; v++) {
      const int want = part[v] ? sB : sA;
      if (want != sl) continue;
      const int ln = tl[v];
      if (len) len[v] = ln;
      for (int i = 0; i < ln; i++) {
        const int32_t id = ti[v * L + i];  // stored id: HOT_TAG | hot index for a hot key
        row[i] = {ts[v * L + i], id >= 0 ? id : p->h_hot_keys[(uint32_t)id & 0x7fffffffu]};
      }
      std::sort(row.begin(), row.begin() + ln, [](const std::pair<double, int32_t>& x, const std::pair<double, int32_t>& y) {
        return x.first > y.first || (x.first == y.first && x.second < y.second);
      });
      for (size_t i = 0; i < L; i++) {
        const bool in = (int)i < ln;
        if (ids) ids[v * L + i] = in ? row[i].second : -1;
        if (scores) scores[v * L + i] = in ? row[i].first : 0.0;
      }
    }
  }
  return PPR_OK;
}

extern "C" int ppr_grank_plan_row_bytes(ppr_plan* p, int64_t* bytes) {
  // bound of one row's share of a compact exchange block (merge_glb.h): offset + ids + scores
  if (!p || !bytes) return PPR_ERR_ARG;
  const int64_t Le = ((int64_t)p->L + 1) & ~1LL;
  *bytes = 8 + 4 * Le + 8 * (int64_t)p->L;
  return PPR_OK;
}

static int ensure_dev(unsigned char** ptr, size_t* cap, size_t need);

struct XRange {
  int64_t begin, cnt;
  int nxt;
  const int32_t* list;
};

static int xrange(ppr_plan* p, int32_t it, int64_t begin, int64_t end, XRange* x) {
  if (!p || it < 0) return PPR_ERR_ARG;
  const int part = it & 1;
  begin = std::max<int64_t>(0, begin);
  end = std::min<int64_t>(p->nact[part], end);
  x->begin = begin;
  x->cnt = std::max<int64_t>(0, end - begin);
  const IterArgs a = iter_args(p, it, false);
  x->nxt = ((a.active == 1) ? a.sB : a.sA) ^ 1;
  x->list = p->d_act[part] + begin;
  return PPR_OK;
}

// compact block of `cnt` rows (node ids `list`, slot `nxt`) into buf (capacity >= 8 + cnt * row
// bytes); the block's size is also written to the device int64 *d_total when given. Asynchronous
// on the plan's stream.
static int xpack_nodes(ppr_plan* p, int nxt, const int32_t* list, int64_t cnt, unsigned char* buf, int64_t* d_total) {
  hipStream_t st = p->stream;
  int64_t* off = reinterpret_cast<int64_t*>(buf);
  if (cnt == 0) {
    HIP_OK(hipMemsetAsync(buf, 0, 8, st));
    if (d_total) hipLaunchKernelGGL(k_xtotal, dim3(1), dim3(64), 0, st, (const int64_t*)off, (int64_t)0, d_total);
    HIP_OK(hipGetLastError());
    return PPR_OK;
  }
  const DevSlab s = dev_slab(p);
  // row sizes into the payload area (free until the pack), scanned into the offset header
  int64_t* sz = reinterpret_cast<int64_t*>(buf + 8 * (cnt + 1));
  hipLaunchKernelGGL(k_xsize, dim3((unsigned)((cnt + 256) / 256)), dim3(256), 0, st, s, nxt, list, cnt, sz);
  size_t tmp = 0;
  HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, sz, off, (int)(cnt + 1), st));
  int rc = ensure_dev(&p->d_xtmp, &p->xtmp_bytes, tmp);
  if (rc) return rc;
  HIP_OK(hipcub::DeviceScan::ExclusiveSum(p->d_xtmp, tmp, sz, off, (int)(cnt + 1), st));
  hipLaunchKernelGGL(k_xpack, dim3((unsigned)((cnt + 3) / 4)), dim3(256), 0, st, s, nxt, list, cnt, buf);
  if (d_total) hipLaunchKernelGGL(k_xtotal, dim3(1), dim3(64), 0, st, (const int64_t*)off, cnt, d_total);
  HIP_OK(hipGetLastError());
  return PPR_OK;
}

static int xunpack_nodes(ppr_plan* p, int nxt, const int32_t* list, int64_t cnt, const unsigned char* buf) {
  if (cnt == 0) return PPR_OK;
  hipLaunchKernelGGL(k_xunpack, dim3((unsigned)((cnt + 3) / 4)), dim3(256), 0, p->stream, dev_slab(p), nxt, list, cnt,
                     buf);
  HIP_OK(hipGetLastError());
  return PPR_OK;
}

// compact block of a range of iteration it's active list (the rows it wrote)
static int xpack(ppr_plan* p, int32_t it, int64_t begin, int64_t end, unsigned char* buf, int64_t cap,
                 int64_t* d_total) {
  XRange x;
  int rc = xrange(p, it, begin, end, &x);
  if (rc) return rc;
  int64_t rb = 0;
  ppr_grank_plan_row_bytes(p, &rb);
  if (!buf || cap < 8 + x.cnt * rb) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  return xpack_nodes(p, x.nxt, x.list, x.cnt, buf, d_total);
}

static int xunpack(ppr_plan* p, int32_t it, int64_t begin, int64_t end, const unsigned char* buf) {
  XRange x;
  int rc = xrange(p, it, begin, end, &x);
  if (rc) return rc;
  if (x.cnt == 0) return PPR_OK;
  if (!buf) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  return xunpack_nodes(p, x.nxt, x.list, x.cnt, buf);
}

extern "C" int ppr_grank_plan_pack(ppr_plan* p, int32_t it, int64_t begin, int64_t end, void* dev_buf,
                                   int64_t cap) {
  return xpack(p, it, begin, end, (unsigned char*)dev_buf, cap, nullptr);
}

extern "C" int ppr_grank_plan_unpack(ppr_plan* p, int32_t it, int64_t begin, int64_t end, const void* dev_buf) {
  return xunpack(p, it, begin, end, (const unsigned char*)dev_buf);
}

extern "C" int ppr_grank_plan_fold_maxdiff(ppr_plan* p, int32_t it, double maxdiff) {
  // all-reduced maxDiff of a sharded iteration written back (ppr_grank_plan_finish-side reads)
  if (!p || it < 0) return PPR_ERR_ARG;
  unsigned long long b;
  std::memcpy(&b, &maxdiff, 8);
  HIP_OK(hipMemcpyAsync(p->d_maxdiff + (it < PPR_MAX_ITER_STATS ? it : PPR_MAX_ITER_STATS), &b, 8,
                        hipMemcpyHostToDevice, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  return PPR_OK;
}

extern "C" int ppr_grank_plan_active_list(ppr_plan* p, int32_t it, int32_t* out) {
  // host copy of iteration `it`'s active sources in list order (the order ranges refer to)
  if (!p || !out || it < 0) return PPR_ERR_ARG;
  const int part = it & 1;
  if (p->nact[part])
    HIP_OK(hipMemcpy(out, p->d_act[part], 4 * (size_t)p->nact[part], hipMemcpyDeviceToHost));
  return PPR_OK;
}

#define NCCL_OK(expr)                                                                        \
  do {                                                                                       \
    ncclResult_t _r = (expr);                                                                \
    if (_r != ncclSuccess) {                                                                 \
      fprintf(stderr, "ppr_hip: %s failed: %s\n", #expr, ncclGetErrorString(_r));           \
      return PPR_ERR_HIP;                                                                    \
    }                                                                                        \
  } while (0)

extern "C" int ppr_device_count(int32_t* count) {
  if (!count) return PPR_ERR_ARG;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *count = c;
  return PPR_OK;
}

extern "C" int ppr_comm_unique_id(void* id_out) {
  if (!id_out) return PPR_ERR_ARG;
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return PPR_OK;
}

extern "C" int ppr_grank_plan_comm_init(ppr_plan* p, const void* id, int32_t nranks, int32_t rank) {
  if (!p || !id || nranks < 1 || rank < 0 || rank >= nranks) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  if (p->comm) { ncclCommDestroy(p->comm); p->comm = nullptr; }
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCL_OK(ncclCommInitRank(&p->comm, nranks, uid, rank));
  int rc = ensure_dev(&p->d_xsz, &p->xsz_bytes, 8 * (size_t)nranks);
  if (rc) return rc;
  p->nranks = nranks;
  p->rank = rank;
  return PPR_OK;
}

// contiguous ranges of the active list with balanced estimated work
static void shard_bounds(const std::vector<double>& w, int world, std::vector<int64_t>& b) {
  const int64_t n = (int64_t)w.size();
  b.assign(world + 1, 0);
  double tot = 0;
  for (double x : w) tot += x;
  double run = 0;
  int64_t i = 0;
  for (int r = 1; r < world; r++) {
    const double target = tot * r / world;
    while (i < n && run + w[i] <= target) run += w[i++];
    b[r] = i;
  }
  b[world] = n;
}

extern "C" int ppr_grank_plan_shard_bounds(ppr_plan* p, int32_t it, int32_t world, int64_t* bounds) {
  if (!p || !bounds || world < 1 || it < 0) return PPR_ERR_ARG;
  std::vector<int64_t> b;
  shard_bounds(p->work[it & 1], world, b);
  std::memcpy(bounds, b.data(), sizeof(int64_t) * (world + 1));
  return PPR_OK;
}

static int ensure_dev(unsigned char** ptr, size_t* cap, size_t need) {
  if (need <= *cap) return PPR_OK;
  hipFree(*ptr);
  *ptr = nullptr;
  *cap = 0;
  if (hipMalloc((void**)ptr, need) != hipSuccess) return PPR_ERR_OOM;
  *cap = need;
  return PPR_OK;
}

// ---- the sharded loop's two collectives: RCCL, or an in-process group of plans ----
// LocalGroup: N plans of one process, one thread each, running the same native loop; block
// blocks (device-to-device copies) and maxDiff go through host-side rendezvous. It tests
// everything of ppr_grank_plan_run_sharded but the RCCL calls on a one-GPU box (RCCL refuses two
// ranks on one device). A rank that fails marks the group, and the others leave their barriers.
struct LocalGroup {
  int n;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  int64_t gen = 0;
  bool failed = false;
  std::vector<unsigned char*> bufs;
  std::vector<unsigned long long> md;
  std::vector<int64_t> iv;                         // int64 all-gather (MC walk block sizes)
  std::vector<int> ok;                             // routed exchange: every rank's size check
  std::vector<std::vector<unsigned char*>> pbufs;  // routed blocks: [sender][receiver]
  std::vector<std::vector<int64_t>> psz;
  explicit LocalGroup(int n_)
      : n(n_), bufs(n_), md(n_), iv(n_), ok(n_, 1), pbufs(n_, std::vector<unsigned char*>(n_)),
        psz(n_, std::vector<int64_t>(n_)) {}
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (failed) return false;
    const int64_t g = gen;
    if (++arrived == n) { arrived = 0; gen++; cv.notify_all(); return true; }
    cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || failed; });
    if (gen != g) return true;  // (everyone arrived: a failure flagged since is the next barrier's)
    failed = true;
    cv.notify_all();
    return false;
  }
  void fail() { std::lock_guard<std::mutex> lk(mu); failed = true; cv.notify_all(); }
};

// Waits of the sharded loops. With an RCCL communicator a peer that failed never posts its side of
// a collective, and the RCCL kernels waiting for it would spin forever (a blocking sync with them):
// these waits poll instead and give up when RCCL reports an asynchronous error or after
// x_timeout_s seconds (PPR_XTIMEOUT) without the stream finishing. The loops' error path then
// aborts the communicator (x_abort), which also releases this rank's RCCL kernels; every peer
// leaves the same way, by its own error or its own time limit. Without a communicator (one rank,
// or the in-process LocalGroup, whose barriers carry the failure) a wait is a plain sync.
static int x_sync(ppr_plan* p, hipStream_t s) {
  if (!p->comm) { HIP_OK(hipStreamSynchronize(s)); return PPR_OK; }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return PPR_OK;
    if (e != hipErrorNotReady) return PPR_ERR_HIP;
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(p->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
      return PPR_ERR_HIP;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > p->x_timeout_s)
      return PPR_ERR_HIP;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}
static int x_sync_event(ppr_plan* p, hipEvent_t ev) {
  if (!p->comm) { HIP_OK(hipEventSynchronize(ev)); return PPR_OK; }
  HIP_OK(hipStreamWaitEvent(p->stream, ev, 0));
  return x_sync(p, p->stream);
}
// a failed sharded run on an RCCL communicator: abort it (its peers' waits end by their own error
// or time limit); the plan needs ppr_grank_plan_comm_init again before the next sharded run
static void x_abort(ppr_plan* p) {
  if (p->comm) {
    ncclCommAbort(p->comm);
    p->comm = nullptr;
  }
}

// every non-empty rank's block (its d_xsend, sz[r] bytes) into d_xrecv + xo[r] of every other rank
static int x_blocks(ppr_plan* p, const std::vector<int64_t>& b, const std::vector<int64_t>& sz,
                    const std::vector<size_t>& xo, hipStream_t s) {
  if (p->lgroup) {
    LocalGroup& G = *p->lgroup;
    HIP_OK(hipStreamSynchronize(s));  // this rank's block is complete
    G.bufs[p->rank] = p->d_xsend;
    if (!G.barrier()) return PPR_ERR_HIP;
    for (int r = 0; r < p->nranks; r++)
      if (r != p->rank && b[r + 1] > b[r])
        HIP_OK(hipMemcpyAsync(p->d_xrecv + xo[r], G.bufs[r], (size_t)sz[r], hipMemcpyDeviceToDevice, s));
    HIP_OK(hipStreamSynchronize(s));
    return G.barrier() ? PPR_OK : PPR_ERR_HIP;  // no rank reuses its send buffer before all copied
  }
  ncclResult_t nr = ncclGroupStart();
  for (int r = 0; r < p->nranks && nr == ncclSuccess; r++) {
    if (b[r + 1] == b[r]) continue;
    unsigned char* dst = r == p->rank ? p->d_xsend : p->d_xrecv + xo[r];
    nr = ncclBroadcast(p->d_xsend, dst, (size_t)sz[r], ncclUint8, r, p->comm, s);
  }
  const ncclResult_t ne = ncclGroupEnd();  // (always closed, whatever failed inside)
  return nr == ncclSuccess && ne == ncclSuccess ? PPR_OK : PPR_ERR_HIP;
}

// maxDiff >= 0: the IEEE bit patterns order like the values, so an integer MAX is exact
static int x_allreduce_max(ppr_plan* p, unsigned long long* mdp, hipStream_t s) {
  if (p->lgroup) {
    LocalGroup& G = *p->lgroup;
    unsigned long long v = 0;
    HIP_OK(hipMemcpyAsync(&v, mdp, 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    G.md[p->rank] = v;
    if (!G.barrier()) return PPR_ERR_HIP;
    for (unsigned long long x : G.md) v = x > v ? x : v;
    if (!G.barrier()) return PPR_ERR_HIP;
    HIP_OK(hipMemcpyAsync(mdp, &v, 8, hipMemcpyHostToDevice, s));
    HIP_OK(hipStreamSynchronize(s));
    return PPR_OK;
  }
  NCCL_OK(ncclAllReduce(mdp, mdp, 1, ncclUint64, ncclMax, p->comm, s));
  return PPR_OK;
}

// the broadcast exchange of iteration it: this rank's whole range to every rank (bounds b)
static int x_exchange_bulk(ppr_plan* p, uint32_t it, const std::vector<int64_t>& b) {
  hipStream_t s = p->stream;
  int64_t rb = 0;
  ppr_grank_plan_row_bytes(p, &rb);
  // all-gather of compact blocks (merge_glb.h): only the entries travel; every rank broadcasts its
  // block from its send buffer (grouped; the root broadcasts in place, so it copies nothing) and
  // unpacks the others'. Every block travels at its bound, 8 + rows * row_bytes (the offset header
  // inside says where each row ends): the bounds are known on every host, so no size exchange and
  // no host sync before the broadcasts.
  const int64_t mine = b[p->rank + 1] - b[p->rank];
  int rc = ensure_dev(&p->d_xsend, &p->xsend_bytes, (size_t)(8 + mine * rb));
  if (rc) return rc;
  rc = xpack(p, (int32_t)it, b[p->rank], b[p->rank + 1], p->d_xsend, (int64_t)p->xsend_bytes, nullptr);
  if (rc) return rc;
  std::vector<int64_t> sz(p->nranks);
  for (int r = 0; r < p->nranks; r++) sz[r] = 8 + (b[r + 1] - b[r]) * rb;
  std::vector<size_t> xo(p->nranks + 1, 0);
  for (int r = 0; r < p->nranks; r++) xo[r + 1] = xo[r] + (r == p->rank ? 0 : (size_t)sz[r]);
  rc = ensure_dev(&p->d_xrecv, &p->xrecv_bytes, std::max<size_t>(8, xo[p->nranks]));
  if (rc) return rc;
  p->x_bytes += (int64_t)xo[p->nranks];
  p->x_rows_sent += mine;
  rc = x_blocks(p, b, sz, xo, s);
  if (rc) return rc;
  for (int r = 0; r < p->nranks; r++) {
    if (r == p->rank || b[r + 1] == b[r]) continue;
    rc = xunpack(p, (int32_t)it, b[r], b[r + 1], p->d_xrecv + xo[r]);
    if (rc) return rc;
  }
  return PPR_OK;
}

// Consumer routing: per partition q, the rows of this rank's range that each peer d reads (send
// lists) and the rows of each peer r's range that this rank reads (receive lists), node ids in
// list order. Both sides derive a list from the same mask and bounds, so they agree on it without
// exchanging it.
struct XRoute {
  std::vector<int64_t> scnt[2], rcnt[2];   // [world] rows
  std::vector<size_t> soff[2], roff[2];    // [world] int offsets into d_xlists
};

static int xroute_build(ppr_plan* p, const std::vector<int64_t> (&bd)[2], XRoute& xr) {
  const int W = p->nranks, me = p->rank;
  const int64_t n = p->n;
  hipStream_t s = p->stream;
  int rc = PPR_OK;
  if (!p->d_xowner) { rc = dalloc(&p->d_xowner, n); if (rc) return rc; }
  if (!p->d_xcmask) { rc = dalloc(&p->d_xcmask, n); if (rc) return rc; }
  HIP_OK(hipMemsetAsync(p->d_xowner, 0xff, (size_t)n, s));
  HIP_OK(hipMemsetAsync(p->d_xcmask, 0, 4 * (size_t)n, s));
  for (int q = 0; q < 2; q++) {
    if (!p->nact[q]) continue;
    XBounds xb{};
    xb.world = W;
    for (int r = 0; r <= W; r++) xb.b[r] = bd[q][r];
    hipLaunchKernelGGL(k_xowner, dim3((unsigned)((p->nact[q] + 255) / 256)), dim3(256), 0, s, p->d_act[q], p->nact[q],
                       xb, p->d_xowner);
  }
  hipLaunchKernelGGL(k_xcmask, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, p->d_rp, p->d_colx, n, p->d_xowner,
                     p->d_xcmask);
  HIP_OK(hipGetLastError());
  size_t total = 0;
  for (int q = 0; q < 2; q++) {
    xr.scnt[q].assign(W, 0); xr.rcnt[q].assign(W, 0);
    xr.soff[q].assign(W, 0); xr.roff[q].assign(W, 0);
    const int64_t mine = bd[q][me + 1] - bd[q][me];
    for (int d = 0; d < W; d++) {
      if (d == me) continue;
      xr.soff[q][d] = total; total += (size_t)mine;
      xr.roff[q][d] = total; total += (size_t)(bd[q][d + 1] - bd[q][d]);
    }
  }
  rc = ensure_dev((unsigned char**)&p->d_xlists, &p->xlists_cap, 4 * std::max<size_t>(1, total) + 8 * 4 * (size_t)W);
  if (rc) return rc;
  int32_t* nsel = reinterpret_cast<int32_t*>(p->d_xlists + std::max<size_t>(1, total));  // [2][2][W] counts
  HIP_OK(hipMemsetAsync(nsel, 0, 4 * 4 * (size_t)W, s));
  size_t tmp = 0, need = 0;
  for (int q = 0; q < 2; q++)
    for (int r = 0; r < W; r++) {
      const int64_t cnt = bd[q][r + 1] - bd[q][r];
      if (!cnt) continue;
      HIP_OK(hipcub::DeviceSelect::If(nullptr, tmp, p->d_act[q], p->d_xlists, nsel, (int)cnt,
                                      XConsumedBy{p->d_xcmask, 1u}, s));
      need = std::max(need, tmp);
    }
  rc = ensure_dev(&p->d_xtmp, &p->xtmp_bytes, std::max<size_t>(need, 1));
  if (rc) return rc;
  for (int q = 0; q < 2; q++)
    for (int d = 0; d < W; d++) {
      if (d == me) continue;
      const int64_t ms = bd[q][me + 1] - bd[q][me], rs = bd[q][d + 1] - bd[q][d];
      tmp = p->xtmp_bytes;
      if (ms) HIP_OK(hipcub::DeviceSelect::If(p->d_xtmp, tmp, p->d_act[q] + bd[q][me], p->d_xlists + xr.soff[q][d],
                                              nsel + (q * 2 + 0) * W + d, (int)ms, XConsumedBy{p->d_xcmask, 1u << d}, s));
      tmp = p->xtmp_bytes;
      if (rs) HIP_OK(hipcub::DeviceSelect::If(p->d_xtmp, tmp, p->d_act[q] + bd[q][d], p->d_xlists + xr.roff[q][d],
                                              nsel + (q * 2 + 1) * W + d, (int)rs, XConsumedBy{p->d_xcmask, 1u << me},
                                              s));
    }
  std::vector<int32_t> h(4 * (size_t)W);
  HIP_OK(hipMemcpyAsync(h.data(), nsel, 4 * h.size(), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  for (int q = 0; q < 2; q++)
    for (int d = 0; d < W; d++) {
      xr.scnt[q][d] = h[(q * 2 + 0) * W + d];
      xr.rcnt[q][d] = h[(q * 2 + 1) * W + d];
    }
  return PPR_OK;
}

// the routed exchange of iteration it: per peer, the rows it reads; exact block sizes (one 8-byte
// send / receive per peer first), then the blocks, then the unpacks
static int x_exchange_routed(ppr_plan* p, uint32_t it, const XRoute& xr, int slot = -1) {
  const int W = p->nranks, me = p->rank, q = (int)(it & 1);
  hipStream_t s = p->stream;
  int64_t rb = 0;
  ppr_grank_plan_row_bytes(p, &rb);
  // (slot >= 0: the rows of partition it & 1 in that slot -- the sharded init's, slot 0)
  const int nxt = slot >= 0 ? slot
                            : ((iter_args(p, (int)it, false).active == 1) ? iter_args(p, (int)it, false).sB
                                                                           : iter_args(p, (int)it, false).sA) ^ 1;
  std::vector<size_t> so(W + 1, 0), ro(W + 1, 0);
  for (int d = 0; d < W; d++) {
    so[d + 1] = so[d] + (xr.scnt[q][d] ? (size_t)(8 + xr.scnt[q][d] * rb) : 0);
    ro[d + 1] = ro[d] + (xr.rcnt[q][d] ? (size_t)(8 + xr.rcnt[q][d] * rb) : 0);
  }
  int rc = ensure_dev(&p->d_xsend, &p->xsend_bytes, std::max<size_t>(8, so[W]));
  if (rc) return rc;
  rc = ensure_dev(&p->d_xrecv, &p->xrecv_bytes, std::max<size_t>(8, ro[W]));
  if (rc) return rc;
  rc = ensure_dev(&p->d_xsz, &p->xsz_bytes, 16 * (size_t)W + 8);
  if (rc) return rc;
  int64_t* tx = reinterpret_cast<int64_t*>(p->d_xsz);
  int64_t* rx = tx + W;
  for (int d = 0; d < W; d++) {
    if (!xr.scnt[q][d]) continue;
    rc = xpack_nodes(p, nxt, p->d_xlists + xr.soff[q][d], xr.scnt[q][d], p->d_xsend + so[d], tx + d);
    if (rc) return rc;
    p->x_rows_sent += xr.scnt[q][d];
  }
  std::vector<int64_t> hsz(2 * (size_t)W, 0);
  // Every rank checks the block sizes it is about to receive and the ranks agree on the outcome
  // BEFORE any block moves: a rank that bailed out alone would leave its peers blocked in their
  // sends / receives (a grouped RCCL call cannot be abandoned half-posted).
  auto size_ok = [&](int r, int64_t z) { return z >= 8 && (size_t)z <= ro[r + 1] - ro[r]; };
  if (p->lgroup) {
    LocalGroup& G = *p->lgroup;
    G.ok[me] = 1;  // (this call's verdict only: written again below, before the second barrier)
    HIP_OK(hipMemcpyAsync(hsz.data(), tx, 8 * (size_t)W, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));  // this rank's blocks are complete
    for (int d = 0; d < W; d++) {
      G.pbufs[me][d] = p->d_xsend + so[d];
      G.psz[me][d] = xr.scnt[q][d] ? hsz[d] + (me == p->xtest_badsize ? ((int64_t)1 << 40) : 0) : 0;
    }
    if (!G.barrier()) return PPR_ERR_HIP;
    int mine_ok = 1;
    for (int r = 0; r < W; r++)
      if (r != me && xr.rcnt[q][r] && !size_ok(r, G.psz[r][me])) mine_ok = 0;
    G.ok[me] = mine_ok;
    if (!G.barrier()) return PPR_ERR_HIP;
    for (int r = 0; r < W; r++)
      if (!G.ok[r]) return PPR_ERR_RANGE;  // (every rank returns here, none is left waiting)
    for (int r = 0; r < W; r++) {
      if (r == me || !xr.rcnt[q][r]) continue;
      const int64_t z = G.psz[r][me];
      hsz[W + r] = z;
      HIP_OK(hipMemcpyAsync(p->d_xrecv + ro[r], G.pbufs[r][me], (size_t)z, hipMemcpyDeviceToDevice, s));
    }
    HIP_OK(hipStreamSynchronize(s));
    if (!G.barrier()) return PPR_ERR_HIP;  // no rank reuses its send buffer before all copied
  } else {
    if (me == p->xtest_badsize) {
      HIP_OK(hipMemcpyAsync(hsz.data(), tx, 8 * (size_t)W, hipMemcpyDeviceToHost, s));
      HIP_OK(hipStreamSynchronize(s));
      for (int d = 0; d < W; d++) hsz[d] += (int64_t)1 << 40;
      HIP_OK(hipMemcpyAsync(tx, hsz.data(), 8 * (size_t)W, hipMemcpyHostToDevice, s));
    }
    ncclResult_t nr = ncclGroupStart();
    for (int d = 0; d < W && nr == ncclSuccess; d++) {
      if (d == me) continue;
      if (xr.scnt[q][d]) nr = ncclSend(tx + d, 1, ncclInt64, d, p->comm, s);
      if (nr == ncclSuccess && xr.rcnt[q][d]) nr = ncclRecv(rx + d, 1, ncclInt64, d, p->comm, s);
    }
    const ncclResult_t ne = ncclGroupEnd();  // (always closed, whatever failed inside)
    if (nr != ncclSuccess || ne != ncclSuccess) return PPR_ERR_HIP;
    HIP_OK(hipMemcpyAsync(hsz.data(), tx, 16 * (size_t)W, hipMemcpyDeviceToHost, s));
    rc = x_sync(p, s);
    if (rc) return rc;
    int32_t* okd = reinterpret_cast<int32_t*>(rx + W);  // (d_xsz holds 2 W + 1 words)
    int32_t mine_ok = 1;
    for (int d = 0; d < W; d++)
      if (d != me && xr.rcnt[q][d] && !size_ok(d, hsz[W + d])) mine_ok = 0;
    HIP_OK(hipMemcpyAsync(okd, &mine_ok, 4, hipMemcpyHostToDevice, s));
    NCCL_OK(ncclAllReduce(okd, okd, 1, ncclInt32, ncclMin, p->comm, s));
    HIP_OK(hipMemcpyAsync(&mine_ok, okd, 4, hipMemcpyDeviceToHost, s));
    rc = x_sync(p, s);
    if (rc) return rc;
    if (!mine_ok) return PPR_ERR_RANGE;  // every rank saw the same minimum: none posts a block
    nr = ncclGroupStart();
    for (int d = 0; d < W && nr == ncclSuccess; d++) {
      if (d == me) continue;
      if (xr.scnt[q][d]) nr = ncclSend(p->d_xsend + so[d], (size_t)hsz[d], ncclUint8, d, p->comm, s);
      if (nr == ncclSuccess && xr.rcnt[q][d]) nr = ncclRecv(p->d_xrecv + ro[d], (size_t)hsz[W + d], ncclUint8, d, p->comm, s);
    }
    const ncclResult_t ne2 = ncclGroupEnd();
    if (nr != ncclSuccess || ne2 != ncclSuccess) return PPR_ERR_HIP;
  }
  for (int r = 0; r < W; r++) {
    if (r == me || !xr.rcnt[q][r]) continue;
    p->x_bytes += hsz[W + r];
    rc = xunpack_nodes(p, nxt, p->d_xlists + xr.roff[q][r], xr.rcnt[q][r], p->d_xrecv + ro[r]);
    if (rc) return rc;
  }
  return PPR_OK;
}

// Sharded init (routed runs): every rank merges the init baskets of its own sources of both
// partitions and of the dangling nodes (their {v: 1-d} rows are the same on every rank), then sends
// each peer the init rows it reads -- the same consumer lists as an iteration's exchange, slot 0.
static int init_sharded(ppr_plan* p, const std::vector<int64_t> (&bd)[2], const XRoute& xr) {
  hipStream_t s = p->stream;
  if (p->own_world != p->nranks || p->own_rank != p->rank || !p->d_own) {
    const int64_t m0 = bd[0][p->rank + 1] - bd[0][p->rank], m1 = bd[1][p->rank + 1] - bd[1][p->rank];
    if (!p->d_own) { int rc = dalloc(&p->d_own, std::max<int64_t>(1, p->n)); if (rc) return rc; }
    if (m0) HIP_OK(hipMemcpyAsync(p->d_own, p->d_act[0] + bd[0][p->rank], 4 * (size_t)m0, hipMemcpyDeviceToDevice, s));
    if (m1) HIP_OK(hipMemcpyAsync(p->d_own + m0, p->d_act[1] + bd[1][p->rank], 4 * (size_t)m1, hipMemcpyDeviceToDevice, s));
    p->own_cnt = m0 + m1;
    p->own_world = p->nranks;
    p->own_rank = p->rank;
  }
  p->md_shared_it = -1;
  p->hot_n = 0;
  p->hot_built_it = -1;
  if (p->d_dlast) HIP_OK(hipMemsetAsync(p->d_dlast, 0, 4 * (size_t)std::max<int64_t>(1, p->n), s));
  IterArgs a = iter_args(p, 0, true);
  int rc = init_dangling(p, p->d_all + p->n_nd, p->n - p->n_nd);
  if (rc) return rc;
  rc = run_merge(p, a, p->d_own, p->own_cnt, p->d_maxdiff + PPR_MAX_ITER_STATS);
  if (rc) return rc;
  for (uint32_t q = 0; q < 2; q++) {
    rc = x_exchange_routed(p, q, xr, 0);
    if (rc) return rc;
  }
  return PPR_OK;
}

// Sharded final top-K (routed runs): every rank selects the top-K of its own rows (and of the
// dangling nodes') and the K-wide rows are all-gathered, one block per rank and partition -- instead
// of an L-wide broadcast of every row and a top-K of all n rows on every rank
static int x_gather_topk(ppr_plan* p, int q, const std::vector<int64_t>& b) {
  const int W = p->nranks, me = p->rank;
  hipStream_t s = p->stream;
  const int64_t K = p->K;
  const int64_t ob = 12 * K + 4;  // bytes of a K-entry row at most
  std::vector<int64_t> sz(W);
  std::vector<size_t> xo(W + 1, 0);
  for (int r = 0; r < W; r++) {
    const int64_t c = b[r + 1] - b[r];
    sz[r] = 8 * (c + 1) + c * ob;
    xo[r + 1] = xo[r] + (r == me ? 0 : (size_t)sz[r]);
  }
  int rc = ensure_dev(&p->d_xsend, &p->xsend_bytes, (size_t)sz[me]);
  if (rc) return rc;
  rc = ensure_dev(&p->d_xrecv, &p->xrecv_bytes, std::max<size_t>(8, xo[W]));
  if (rc) return rc;
  const int64_t mine = b[me + 1] - b[me];
  const int32_t* ml = p->d_act[q] + b[me];
  unsigned char* buf = p->d_xsend;
  int64_t* off = reinterpret_cast<int64_t*>(buf);
  if (mine == 0) {
    HIP_OK(hipMemsetAsync(buf, 0, 8, s));
  } else {
    int64_t* rsz = reinterpret_cast<int64_t*>(buf + 8 * (mine + 1));  // (the payload area, free until the pack)
    hipLaunchKernelGGL(k_osize, dim3((unsigned)((mine + 256) / 256)), dim3(256), 0, s, p->d_out_len, ml, mine, rsz);
    size_t tmp = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, rsz, off, (int)(mine + 1), s));
    rc = ensure_dev(&p->d_xtmp, &p->xtmp_bytes, tmp);
    if (rc) return rc;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(p->d_xtmp, tmp, rsz, off, (int)(mine + 1), s));
    hipLaunchKernelGGL(k_opack, dim3((unsigned)((mine + 3) / 4)), dim3(256), 0, s, p->d_out_ids, p->d_out_sc,
                       p->d_out_len, (int)K, ml, mine, buf);
    HIP_OK(hipGetLastError());
  }
  p->x_bytes += (int64_t)xo[W];
  rc = x_blocks(p, b, sz, xo, s);
  if (rc) return rc;
  for (int r = 0; r < W; r++) {
    const int64_t c = b[r + 1] - b[r];
    if (r == me || !c) continue;
    hipLaunchKernelGGL(k_ounpack, dim3((unsigned)((c + 3) / 4)), dim3(256), 0, s, p->d_out_ids, p->d_out_sc,
                       p->d_out_len, (int)K, p->d_act[q] + b[r], c, p->d_xrecv + xo[r]);
    HIP_OK(hipGetLastError());
  }
  return PPR_OK;
}

// Measurement (tools/shard_floor.py): on this one plan, the device time rank `rank` of a `world`-rank
// routed run spends in one of its sharded ends (the exchanges around them are not included):
// what 0 = the top-K of its own rows and the dangling ones (of the plan's current rows: time it
// after a job), what 1 = the init of its own sources and the dangling nodes (rewrites those rows).
extern "C" int ppr_grank_plan_ends_time(ppr_plan* p, int32_t world, int32_t rank, int32_t iterations_run,
                                        int32_t what, double* ms_out) {
  if (!p || world < 1 || rank < 0 || rank >= world || world > 127 || iterations_run < 0 || what < 0 || what > 1)
    return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  hipStream_t s = p->stream;
  std::vector<int64_t> bd[2];
  shard_bounds(p->work[0], world, bd[0]);
  shard_bounds(p->work[1], world, bd[1]);
  float ms = 0.f;
  if (what == 0) {
    if (!p->d_xowner) { int rc = dalloc(&p->d_xowner, p->n); if (rc) return rc; }
    HIP_OK(hipMemsetAsync(p->d_xowner, 0xff, (size_t)p->n, s));
    for (int q = 0; q < 2; q++) {
      if (!p->nact[q]) continue;
      XBounds xb{};
      xb.world = world;
      for (int r = 0; r <= world; r++) xb.b[r] = bd[q][r];
      hipLaunchKernelGGL(k_xowner, dim3((unsigned)((p->nact[q] + 255) / 256)), dim3(256), 0, s, p->d_act[q],
                         p->nact[q], xb, p->d_xowner);
    }
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(p->ev_a, s));
    int rc = launch_topk(p, ((iterations_run + 1) / 2) & 1, (iterations_run / 2) & 1, p->d_xowner, rank);
    if (rc) return rc;
  } else {
    const int64_t m0 = bd[0][rank + 1] - bd[0][rank], m1 = bd[1][rank + 1] - bd[1][rank];
    if (!p->d_own) { int rc = dalloc(&p->d_own, std::max<int64_t>(1, p->n)); if (rc) return rc; }
    p->own_world = 0;  // (init_sharded rebuilds its own list)
    if (m0) HIP_OK(hipMemcpyAsync(p->d_own, p->d_act[0] + bd[0][rank], 4 * (size_t)m0, hipMemcpyDeviceToDevice, s));
    if (m1) HIP_OK(hipMemcpyAsync(p->d_own + m0, p->d_act[1] + bd[1][rank], 4 * (size_t)m1, hipMemcpyDeviceToDevice, s));
    HIP_OK(hipEventRecord(p->ev_a, s));
    IterArgs a = iter_args(p, 0, true);
    int rc = init_dangling(p, p->d_all + p->n_nd, p->n - p->n_nd);
    if (rc) return rc;
    rc = run_merge(p, a, p->d_own, m0 + m1, p->d_maxdiff + PPR_MAX_ITER_STATS);
    if (rc) return rc;
  }
  HIP_OK(hipEventRecord(p->ev_b, s));
  HIP_OK(hipEventSynchronize(p->ev_b));
  hipEventElapsedTime(&ms, p->ev_a, p->ev_b);
  if (ms_out) *ms_out = ms;
  return probe_take();
}

static int run_sharded_impl(ppr_plan* p, uint32_t iterations, double tolerance, ppr_stats* st) {
  if (iterations == 0) return PPR_ERR_ITERS;
  if (p->nranks > 1 && !p->comm && !p->lgroup) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  hipStream_t s = p->stream;
  HIP_OK(hipMemsetAsync(p->d_maxdiff, 0, 8 * (PPR_MAX_ITER_STATS + 1), s));
  HIP_OK(hipMemsetAsync(p->d_stats, 0, 8 * PPR_NSTATS, s));
  p->merge_launches = 0;
  p->merge_ms = 0.0;
  p->x_bytes = 0;
  p->x_rows_sent = 0;
  HIP_OK(hipEventRecord(p->ev_a, s));
  std::vector<int64_t> bd[2];
  shard_bounds(p->work[0], p->nranks, bd[0]);
  shard_bounds(p->work[1], p->nranks, bd[1]);
  // consumer routing: during the run a row goes only to the ranks that read it. The ends are
  // sharded too (PPR_XSHARD_ENDS=0: not): each rank inits its own sources and the dangling nodes
  // and sends the init rows its peers read; at the end each rank selects the top-K of its own rows
  // and the K-wide rows are all-gathered. Without them every rank inits every source, and the
  // result rows of both partitions are broadcast L-wide so that every rank's top-K reads every row.
  const bool route = p->nranks > 1 && p->nranks <= 32 && p->xroute;
  const bool shard_ends = route && p->xshard_ends;
  XRoute xr;
  int rc = PPR_OK;
  if (route) { rc = xroute_build(p, bd, xr); if (rc) return rc; }
  rc = shard_ends ? init_sharded(p, bd, xr) : ppr_grank_plan_init(p);
  if (rc) return rc;
  double md[2] = {tolerance, tolerance};
  uint32_t it = 0;
  for (; it < iterations && std::max(md[0], md[1]) >= tolerance; it++) {
    const std::vector<int64_t>& b = bd[it & 1];
    rc = ppr_grank_plan_iterate(p, (int32_t)it, b[p->rank], b[p->rank + 1]);
    if (rc) return rc;
    if (p->rank == p->xtest_fail_rank && (int)it == p->xtest_fail_it) return PPR_ERR_HIP;  // (tests)
    unsigned long long* mdp = p->d_maxdiff + (it < PPR_MAX_ITER_STATS ? it : PPR_MAX_ITER_STATS);
    if (p->nranks > 1) {
      rc = route ? x_exchange_routed(p, it, xr) : x_exchange_bulk(p, it, bd[it & 1]);
      if (rc) return rc;
      rc = x_allreduce_max(p, mdp, s);
      if (rc) return rc;
      rc = x_sync(p, s);  // (a stuck collective is found here, before any blocking wait of the next merge)
      if (rc) return rc;
    }
    if (tolerance > 0) {  // (the all-reduced value: every rank takes the same stop decision)
      double d = 0.0;
      rc = ppr_grank_plan_read_maxdiff(p, (int32_t)it, &d);
      if (rc) return rc;
      md[0] = d;
      std::swap(md[0], md[1]);
    }
  }
  if (shard_ends) {
    rc = x_sync(p, s);  // (init / last exchange)
    if (rc) return rc;
    rc = launch_topk(p, ((it + 1) / 2) & 1, (it / 2) & 1, p->d_xowner, p->rank);
    if (rc) return rc;
    for (int q = 0; q < 2; q++) {
      rc = x_gather_topk(p, q, bd[q]);
      if (rc) return rc;
    }
    rc = probe_take();
    if (rc) return rc;
  } else {
    if (route)
      for (int q = 0; q < 2; q++) {  // each partition's rows as its last iteration wrote them
        const int64_t last = (int64_t)it - 1 - (((int64_t)it - 1 - q) & 1);
        if (last < 0 || (last & 1) != q) continue;
        rc = x_exchange_bulk(p, (uint32_t)last, bd[q]);
        if (rc) return rc;
      }
    rc = x_sync(p, s);
    if (rc) return rc;
    rc = ppr_grank_plan_finish(p, (int32_t)it);
    if (rc) return rc;
  }
  HIP_OK(hipEventRecord(p->ev_b, s));
  rc = x_sync_event(p, p->ev_b);
  if (rc) return rc;
  if (st) {
    rc = read_maxdiff_history(p, it, st);
    if (rc) return rc;
    float ms = 0;
    hipEventElapsedTime(&ms, p->ev_a, p->ev_b);
    st->iterations_run = (int32_t)it;
    st->device_ms = ms;
    st->merge_ms = p->merge_ms;
    unsigned long long sv[2];
    HIP_OK(hipMemcpyAsync(sv, p->d_stats, 16, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    st->candidates = (int64_t)sv[0];
    st->algo_bytes = (int64_t)sv[1];
    st->merge_launches = p->merge_launches;
  }
  return PPR_OK;
}

// A failing rank aborts its RCCL communicator (x_abort): its peers' waits end by their own errors or
// time limits (x_sync) instead of waiting forever for a rank that left
extern "C" int ppr_grank_plan_run_sharded(ppr_plan* p, uint32_t iterations, double tolerance,
                                          ppr_stats* st) {
  if (!p) return PPR_ERR_ARG;
  const int rc = run_sharded_impl(p, iterations, tolerance, st);
  if (rc) x_abort(p);
  return rc;
}

extern "C" int ppr_grank_plan_exchange_bytes(ppr_plan* p, int64_t* recv_bytes, int64_t* rows_sent) {
  if (!p) return PPR_ERR_ARG;
  if (recv_bytes) *recv_bytes = p->x_bytes;
  if (rows_sent) *rows_sent = p->x_rows_sent;
  return PPR_OK;
}

// Test entry: the native sharded loop with n plans of this process as the ranks (LocalGroup),
// one thread each; every plan must be built on the same graph and parameters. st: n stats or null.
extern "C" int ppr_grank_plan_run_local_group(ppr_plan** plans, int32_t n, uint32_t iterations, double tolerance,
                                              ppr_stats* st) {
  if (!plans || n < 1) return PPR_ERR_ARG;
  for (int i = 0; i < n; i++)
    if (!plans[i] || plans[i]->comm || plans[i]->n != plans[0]->n) return PPR_ERR_ARG;
  for (int i = 0; i < n; i++) {
    int rc = ensure_dev(&plans[i]->d_xsz, &plans[i]->xsz_bytes, 8 * (size_t)n);
    if (rc) return rc;
  }
  LocalGroup G(n);
  std::vector<int> rcs(n, PPR_OK);
  for (int i = 0; i < n; i++) {
    plans[i]->lgroup = &G;
    plans[i]->nranks = n;
    plans[i]->rank = i;
  }
  std::vector<std::thread> th;
  for (int i = 0; i < n; i++)
    th.emplace_back([&, i] {
      rcs[i] = ppr_grank_plan_run_sharded(plans[i], iterations, tolerance, st ? st + i : nullptr);
      if (rcs[i]) G.fail();
    });
  for (auto& t : th) t.join();
  // the group lives on this stack frame: no plan keeps it
  for (int i = 0; i < n; i++) { plans[i]->lgroup = nullptr; plans[i]->nranks = 1; plans[i]->rank = 0; }
  for (int i = 0; i < n; i++)
    if (rcs[i]) return rcs[i];
  return PPR_OK;
}

// one int64 per rank (device word d_val) gathered on every host: out[r] = rank r's value
static int x_allgather_i64(ppr_plan* p, const int64_t* d_val, std::vector<int64_t>& out, hipStream_t s) {
  const int W = p->nranks;
  out.assign(W, 0);
  if (p->lgroup) {
    LocalGroup& G = *p->lgroup;
    int64_t v = 0;
    HIP_OK(hipMemcpyAsync(&v, d_val, 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    G.iv[p->rank] = v;
    if (!G.barrier()) return PPR_ERR_HIP;
    out = G.iv;
    return G.barrier() ? PPR_OK : PPR_ERR_HIP;
  }
  int rc = ensure_dev(&p->d_xsz, &p->xsz_bytes, 16 * (size_t)W + 8);
  if (rc) return rc;
  int64_t* all = reinterpret_cast<int64_t*>(p->d_xsz);
  NCCL_OK(ncclAllGather(d_val, all, 1, ncclInt64, p->comm, s));
  HIP_OK(hipMemcpyAsync(out.data(), all, 8 * (size_t)W, hipMemcpyDeviceToHost, s));
  rc = x_sync(p, s);
  if (rc) return rc;
  return PPR_OK;
}

// ---- MCCompletePathV2 on several ranks (include/mccompletepathv2.h:211-250, the whole job) ----
// The walk set is split into W contiguous ranges of equal size (a walk's expected length is
// 1 / (1 - d) whatever the node, so nodes cost about the same); each rank walks its range. A walk
// basket does not depend on which rank computes it (the Philox streams are keyed by seed, step,
// walk and source), so the job equals the one-GPU run bit for bit. The walk baskets then travel as
// one compact block per rank (merge_glb.h format, slab slot 1): the exact block sizes are
// all-gathered first (one int64 per rank), every rank checks them (all ranks see the same sizes,
// so all take the same decision before any block moves), then the blocks are broadcast
// (x_blocks). Every rank runs the combine and the top-K itself: the combine is level-sequential
// (1,804 levels at RMAT-22), each level's time set by a lone hub's dependent chain, so splitting a
// level's sources over ranks would not shorten it and would add two collectives per level.
static int mc_run_sharded(ppr_plan* p, uint32_t walks, uint64_t seed, ppr_mc_stats* st) {
  if (!p || !p->mc) return PPR_ERR_ARG;
  if (walks == 0) return PPR_ERR_ITERS;
  if (p->nranks > 1 && !p->comm && !p->lgroup) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  hipStream_t s = p->stream;
  const int W = p->nranks, me = p->rank;
  HIP_OK(hipMemsetAsync(p->d_stats, 0, 8 * PPR_NSTATS, s));
  p->merge_launches = 0;
  p->merge_ms = 0.0;
  p->mc_walk_ms = 0.0;
  p->mc_walks = 0;
  p->x_bytes = 0;
  p->x_rows_sent = 0;
  HIP_OK(hipEventRecord(p->ev_a, s));
  std::vector<int64_t> b(W + 1);
  for (int r = 0; r <= W; r++) b[r] = p->mc_nwalk * r / W;
  int rc = ppr_mccp2_plan_walk(p, walks, seed, b[me], b[me + 1]);
  if (rc) return rc;
  if (me == p->xtest_fail_rank && p->xtest_fail_it == 0) return PPR_ERR_HIP;  // (tests)
  if (W > 1) {
    int64_t rb = 0;
    ppr_grank_plan_row_bytes(p, &rb);
    const int64_t mine = b[me + 1] - b[me];
    rc = ensure_dev(&p->d_xsend, &p->xsend_bytes, (size_t)(8 + mine * rb));
    if (rc) return rc;
    rc = ensure_dev(&p->d_xsz, &p->xsz_bytes, 16 * (size_t)W + 8);
    if (rc) return rc;
    int64_t* d_tot = reinterpret_cast<int64_t*>(p->d_xsz) + W;
    rc = xpack_nodes(p, 1, p->d_mc_walk + b[me], mine, p->d_xsend, d_tot);
    if (rc) return rc;
    std::vector<int64_t> sz;
    rc = x_allgather_i64(p, d_tot, sz, s);
    if (rc) return rc;
    for (int r = 0; r < W; r++)  // (every rank sees the same sizes: the same verdict everywhere)
      if (b[r + 1] > b[r] && (sz[r] < 8 || sz[r] > 8 + (b[r + 1] - b[r]) * rb)) return PPR_ERR_RANGE;
    std::vector<size_t> xo(W + 1, 0);
    for (int r = 0; r < W; r++) xo[r + 1] = xo[r] + (r == me || b[r + 1] == b[r] ? 0 : (size_t)sz[r]);
    rc = ensure_dev(&p->d_xrecv, &p->xrecv_bytes, std::max<size_t>(8, xo[W]));
    if (rc) return rc;
    p->x_bytes += (int64_t)xo[W];
    p->x_rows_sent += mine;
    rc = x_blocks(p, b, sz, xo, s);
    if (rc) return rc;
    rc = x_sync(p, s);
    if (rc) return rc;
    for (int r = 0; r < W; r++) {
      if (r == me || b[r + 1] == b[r]) continue;
      rc = xunpack_nodes(p, 1, p->d_mc_walk + b[r], b[r + 1] - b[r], p->d_xrecv + xo[r]);
      if (rc) return rc;
    }
  }
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

extern "C" int ppr_mccp2_plan_run_sharded(ppr_plan* p, uint32_t walks, uint64_t seed, ppr_mc_stats* st) {
  const int rc = mc_run_sharded(p, walks, seed, st);
  if (rc && p) x_abort(p);
  return rc;
}

// Test entry: the sharded MC job with n MC plans of this process as the ranks (LocalGroup)
extern "C" int ppr_mccp2_plan_run_local_group(ppr_plan** plans, int32_t n, uint32_t walks, uint64_t seed,
                                              ppr_mc_stats* st) {
  if (!plans || n < 1) return PPR_ERR_ARG;
  for (int i = 0; i < n; i++)
    if (!plans[i] || !plans[i]->mc || plans[i]->comm || plans[i]->n != plans[0]->n ||
        plans[i]->mc_nwalk != plans[0]->mc_nwalk)
      return PPR_ERR_ARG;
  LocalGroup G(n);
  std::vector<int> rcs(n, PPR_OK);
  for (int i = 0; i < n; i++) {
    plans[i]->lgroup = &G;
    plans[i]->nranks = n;
    plans[i]->rank = i;
  }
  std::vector<std::thread> th;
  for (int i = 0; i < n; i++)
    th.emplace_back([&, i] {
      rcs[i] = mc_run_sharded(plans[i], walks, seed, st ? st + i : nullptr);
      if (rcs[i]) G.fail();
    });
  for (auto& t : th) t.join();
  for (int i = 0; i < n; i++) { plans[i]->lgroup = nullptr; plans[i]->nranks = 1; plans[i]->rank = 0; }
  for (int i = 0; i < n; i++)
    if (rcs[i]) return rcs[i];
  return PPR_OK;
}

// host-staged row exchange (gloo rehearsal on a single GPU; the RCCL path never uses these):
// the same compact blocks, copied through host memory. Synchronous.
extern "C" int ppr_grank_plan_pack_host(ppr_plan* p, int32_t it, int64_t begin, int64_t end, void* host,
                                        int64_t cap, int64_t* bytes) {
  if (!p || it < 0 || !host || !bytes) return PPR_ERR_ARG;
  XRange x;
  int rc = xrange(p, it, begin, end, &x);
  if (rc) return rc;
  rc = ensure_dev(&p->d_xsz, &p->xsz_bytes, 8);
  if (rc) return rc;
  int64_t rb = 0;
  ppr_grank_plan_row_bytes(p, &rb);
  rc = ensure_dev(&p->d_xsend, &p->xsend_bytes, (size_t)(8 + x.cnt * rb));
  if (rc) return rc;
  int64_t* d_tot = reinterpret_cast<int64_t*>(p->d_xsz);
  rc = xpack(p, it, begin, end, p->d_xsend, (int64_t)p->xsend_bytes, d_tot);
  if (rc) return rc;
  int64_t tot = 0;
  HIP_OK(hipMemcpyAsync(&tot, d_tot, 8, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  if (tot > cap) return PPR_ERR_ARG;
  HIP_OK(hipMemcpyAsync(host, p->d_xsend, (size_t)tot, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  *bytes = tot;
  return PPR_OK;
}

extern "C" int ppr_grank_plan_unpack_host(ppr_plan* p, int32_t it, int64_t begin, int64_t end, const void* host,
                                          int64_t bytes) {
  if (!p || it < 0) return PPR_ERR_ARG;
  XRange x;
  int rc = xrange(p, it, begin, end, &x);
  if (rc) return rc;
  if (x.cnt == 0) return PPR_OK;
  if (!host || bytes < 8 * (x.cnt + 1)) return PPR_ERR_ARG;
  rc = ensure_dev(&p->d_xrecv, &p->xrecv_bytes, (size_t)bytes);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(p->d_xrecv, host, (size_t)bytes, hipMemcpyHostToDevice, p->stream));
  rc = xunpack(p, it, begin, end, p->d_xrecv);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(p->stream));
  return PPR_OK;
}

extern "C" int ppr_grank_csr(const ppr_csr* g, const uint8_t* part, uint32_t K, uint32_t L,
                             uint32_t iterations, double damping, double tolerance,
                             const ppr_opts* o, int32_t* out_ids, double* out_scores,
                             int32_t* out_len, ppr_stats* st) {
  int rc = check_params(K, L, iterations, damping);
  if (rc) return rc;
  if (!g) return PPR_ERR_ARG;
  if (g->n == 0) { if (st) { std::memset(st, 0, sizeof(*st)); } return PPR_OK; }
  ppr_plan* p = nullptr;
  rc = ppr_grank_plan_create(g, part, K, L, damping, o, &p);
  if (rc) return rc;
  rc = ppr_grank_plan_run(p, iterations, tolerance, st);
  if (!rc) rc = ppr_grank_plan_fetch(p, out_ids, out_scores, out_len);
  ppr_grank_plan_destroy(p);
  return rc;
}

#ifndef PPR_SRC_SHA256
#define PPR_SRC_SHA256 "unknown"
#endif
#ifndef PPR_OFFLOAD_ARCH
#define PPR_OFFLOAD_ARCH "unknown"
#endif
extern "C" const char* ppr_build_info(void) {
  return "ppr_src_sha256=" PPR_SRC_SHA256 " arch=" PPR_OFFLOAD_ARCH " hipcc=" __clang_version__;
}

extern "C" const char* ppr_strerror(int code) {
  switch (code) {
    case PPR_OK: return "ok";
    case PPR_ERR_ARG: return "invalid argument";
    case PPR_ERR_K: return "K must be positive";
    case PPR_ERR_L: return "L must be positive";
    case PPR_ERR_KL: return "K must be <= L";
    case PPR_ERR_ITERS: return "iterations must be positive";
    case PPR_ERR_DAMPING: return "damping must be [0,1]";
    case PPR_ERR_THREADS: return "nThreads must be positive";
    case PPR_ERR_GRAPH: return "successor is not a node of the graph";
    case PPR_ERR_HIP: return "HIP runtime error";
    case PPR_ERR_OOM: return "device out of memory";
    case PPR_ERR_RANGE: return "parameter outside the supported range";
    case PPR_ERR_SOURCE: return "source node not part of the graph";
    case PPR_ERR_PROBE: return "a hash table ran out of slots (table sizing error)";
    default: return "unknown error";
  }
}
