// merge_hub.h -- sources beyond the workgroup tier ("hubs"): stable key-bucket partition.
#pragma once
#include "wg_merge.h"
#include "merge_wave.h"

namespace pprk {

// ---------------------------------------------------------------------------------------------
// Hub pipeline (sources beyond the workgroup tier). A source's candidate stream (successor order)
// is split by key into P = 2^logP buckets with a STABLE partition, so each key's contributions
// keep their successor order inside its bucket; every bucket is then accumulated on its own (one
// key set per bucket, disjoint across buckets) and the bucket results that can still be in the
// top-L are appended to one list per source, merged by one workgroup per source.
//   k_hub_count    wave per tile (64 successors): per-bucket counts -> cm[b][t], and the pruning
//                  bound tau (below)
//   (device scan)  exclusive scan of every source's cm in (b, t) order, sources concatenated ->
//                  absolute staging offsets (hipcub, host side)
//   k_hub_scatter  wave per tile: ballot ranks inside a group + running per-bucket counters
//   k_hub_bucket_w wave per bucket, private LDS table, no barriers: a hot key's long fma chain
//                  occupies one wave while the CU's other waves keep working
//   k_hub_bucket   workgroup per bucket whose distinct keys overflow the wave table
//   k_hub_final    workgroup per source: top-L of the appended bucket results, row, norm1
// Pruning bound: every contribution is >= 0, so a key's final value is at least any single
// contribution, fma(s, f, acc) >= round(s * f) (monotone rounding). A successor u with a full
// row (len = L) thus puts L distinct keys at >= round(rmin[u] * f), and
//     tau = round(f * max_{u: len[u] = L} min(row u))
// is a lower bound of the L-th largest final value: a bucket never needs to emit a key below tau
// (ties at tau are kept, the (score desc, id asc) order decides them in k_hub_final).
constexpr int HUB_TILE_CAND = 4096;   // target candidates per tile: tw = max(1, target / L) successors
constexpr int HUB_TILE_PER_BUCKET = 16;  // ... and target >= 16 P (capped by tw <= 64): runs of ~16
                                         // records per bucket per tile keep the scatter's stores near
                                         // whole 128-B lines, and the count matrix <= 1/16 int per candidate
constexpr int HUB_BUCKET = 448;       // default target candidates per bucket (PPR_HUB_BUCKET)
constexpr int HUB_MAX_LOGP = 12;      // per-wave LDS counters of the partition: 16 KB
constexpr int HUB_WAVE_T = 512;       // default wave bucket table slots (PPR_HUB_WAVE_T, a multiple of 64):
                                      // 9.7 KB of LDS per wave with 2 groups per chunk, 16 waves per CU
// the MC combine's defaults: larger buckets (fewer per-bucket fixed costs on a level's critical
// path, where a few lone hubs leave most of the chip idle anyway): 640 / 768 measured 5-6 % faster
// per job than 448 / 512 (896 / 1024: 3 %, 1280 / 1536: ±0, 1792 / 2048: +11 %)
constexpr int HUB_BUCKET_MC = 640;
constexpr int HUB_WAVE_T_MC = 768;
constexpr int HUB_BW_BATCH = 8;       // staged groups a bucket wave keeps in flight
constexpr int HUB_SLICE = 8192;       // k_hub_reduce: appended entries per reducing workgroup (PPR_HUB_SLICE)


// wave bucket LDS: acc f64[T] | keys i32[T] | cnt u16[T] | vals f64[CHUNK] | touched u16[CHUNK] |
// tof u16[CHUNK + 2] | ord u32[CHUNK]; the radix histogram of the final select (1 KB) aliases vals
__host__ __device__ constexpr size_t hub_wave_lds(int T, int ng) {  // 16-B multiple: acc stays aligned
  return ((size_t)T * 16 + ((size_t)(ng * WAVE) * 16 > 1024 ? (size_t)(ng * WAVE) * 16 : 1024) + 4 + 15) & ~(size_t)15;
}

struct HubDesc {
  int32_t v;
  int32_t logP;
  int32_t T;       // tiles
  int32_t need;    // candidates + 1
  int32_t tw;      // successors per tile (<= 64; about 4096 candidates per tile)
  int32_t nsl;     // k_hub_reduce slices reserved (upper bound from P * L appended entries)
  int32_t hot;     // >= 0: the hot pass (k_hub_hot) accumulates the source's hot keys into hot list
                   // `hot`, and the partition carries only its cold keys; -1: no hot pass
  int32_t rg_off;  // first bucket-range task of this source in its batch (k_hub_range)
  int64_t cm_off;  // count matrix (P*T ints; after the scan: absolute staging offsets)
  int64_t st_off;  // staging (need-1 keys / scores)
  int64_t pt_off;  // appended bucket results (<= P*L entries, pt_cnt[desc] of them used)
  int64_t red;     // offset of the sliced reduction (k_hub_reduce), used iff pt_cnt > 2 * slice
  int64_t tile_off, buck_off, rt_off;  // first tile / bucket / reduce task of this source in its batch
  int64_t sg_off;  // >= 0: segmented source (k_hub_seg), first segment task; -1: staged partition
};

// the batch's task lists, expanded on the device from the descriptors (one block per source):
// tiles (d, t) for k_hub_count / k_hub_scatter, buckets (d, b) for k_hub_prep, reduce slices (d, x)
struct HubTask;

// staging range of bucket x of source d (cm holds the scanned, absolute offsets; the source's
// staged records start at cm[cm_off] and number `staged`, its candidates minus its hot ones)
__device__ __forceinline__ void hub_bucket_range(const HubDesc& d, const int32_t* cm, uint32_t staged, int x,
                                                 int64_t& start, int64_t& nb) {
  const int P = 1 << d.logP;
  if (d.T == 0) { start = d.st_off; nb = 0; return; }  // no successors (init of a dangling node)
  start = cm[d.cm_off + (int64_t)x * d.T];
  const int64_t end = (x + 1 < P) ? (int64_t)cm[d.cm_off + (int64_t)(x + 1) * d.T]
                                  : (int64_t)cm[d.cm_off] + (int64_t)staged;
  nb = end - start;
}
struct HubTask { int32_t d; int32_t x; };   // (descriptor, tile or bucket)

// It also clears the batch's per-source counters (staged count, appended-list length, pruning
// bound, overflow flag), the spill list length and, for a merge call's first batch, the overflow
// list count: one launch instead of a fill per array (an MC level is latency-bound)
__global__ void __launch_bounds__(256) k_hub_expand(const HubDesc* desc, HubTask* tiles, HubTask* buckets,
                                                    HubTask* rts, HubTask* segs, HubTask* ranges, int krange,
                                                    uint32_t* staged, uint32_t* pt_cnt, unsigned long long* tau,
                                                    int32_t* oflag, uint32_t* lc, int32_t* ovl, int32_t* rsp) {
  const int d = blockIdx.x;
  const HubDesc D = desc[d];
  if (threadIdx.x == 0) {
    staged[d] = 0u;
    pt_cnt[d] = 0u;
    tau[d] = 0ull;
    oflag[d] = 0;
    if (d == 0) {
      lc[0] = 0u;
      lc[1] = 0u;
      if (ovl) ovl[0] = 0;
      if (rsp) rsp[0] = 0;
    }
  }
  const int P = 1 << D.logP;
  for (int t = threadIdx.x; t < D.T; t += blockDim.x) tiles[D.tile_off + t] = HubTask{d, t};
  if (D.sg_off >= 0) {
    for (int b = threadIdx.x; b < P; b += blockDim.x) segs[D.sg_off + b] = HubTask{d, b};
  } else if (krange > 0) {
    for (int r = threadIdx.x; r * krange < P; r += blockDim.x) ranges[D.rg_off + r] = HubTask{d, r * krange};
  } else {
    for (int b = threadIdx.x; b < P; b += blockDim.x) buckets[D.buck_off + b] = HubTask{d, b};
  }
  for (int x = threadIdx.x; x < D.nsl; x += blockDim.x) rts[D.rt_off + x] = HubTask{d, x};
}

// one staged candidate: score and key packed in 12 bytes (dword aligned, one dwordx3 store /
// load), so a scattered store touches one partial line instead of two (separate key / score
// arrays); measured as fast as a padded 16-B record, with 3/4 of its staging memory. The score
// comes first: a dwordx3 load lands in an even-aligned register triple, so the score is an
// aligned 64-bit pair as loaded (key first, the compiler re-aligned it with moves that waited for
// the load)
struct HubRec {
  uint32_t w[3];
};
__device__ __forceinline__ HubRec hub_rec(int key, double sc) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(sc);
  HubRec r{};
  r.w[0] = (uint32_t)b; r.w[1] = (uint32_t)(b >> 32); r.w[2] = (uint32_t)key;
  return r;
}
__device__ __forceinline__ int rec_key(const HubRec& r) { return (int)r.w[2]; }
__device__ __forceinline__ double rec_sc(const HubRec& r) {
  return __longlong_as_double((long long)(((unsigned long long)r.w[1] << 32) | r.w[0]));
}

__device__ __forceinline__ uint32_t hub_digit(int key, int logP) {
  return logP == 0 ? 0u : (hash_b((uint32_t)key) >> (32 - logP));
}

// walk the candidates of tile t (successors [t * tw, (t + 1) * tw) of source v) in successor
// order: windows of 64 successors, 64 candidates per step
template <class F, class S = WalkNoSucc>
__device__ __forceinline__ void hub_tile_walk(const DevGraph& g, const DevSlab& s, const IterArgs& a,
                                              int v, int t, int tw, uint8_t* fl, F f, S succ = S{}) {
  const int64_t b = g.rp[v] + (int64_t)t * tw;
  const int64_t e = min(g.rp[v + 1], b + (int64_t)tw);
  for (int64_t w0 = b; w0 < e; w0 += WAVE) hub_window_walk(g, s, a, w0, min(e, w0 + WAVE), fl, f, succ);
}

template <bool HK>
__global__ void __launch_bounds__(256) k_hub_count(DevGraph g, DevSlab s, IterArgs a,
                                                   const HubDesc* desc, const HubTask* tasks,
                                                   int64_t ntasks, int maxP, int32_t* cm,
                                                   unsigned long long* tau, uint32_t* staged) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  // neighbouring tiles write neighbouring columns of the count matrix: on one XCD their partial
  // lines merge in its L2
  const int64_t w = xcd_block(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + wv;
  if (w >= ntasks) return;
  const HubTask tk = tasks[w];
  const HubDesc d = desc[tk.d];
  const int P = 1 << d.logP;
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem) + (size_t)wv * maxP;
  uint8_t* fl = smem + (size_t)(blockDim.x >> 6) * maxP * 4 + (size_t)wv * HUB_WALK_FLAGS;
  for (int i = lane_id(); i < P; i += WAVE) hist[i] = 0;
  wave_fence();
  // the walk also hands over every successor's row length and minimum: tau = max over this tile's
  // full-row successors of their row minimum (unscaled)
  unsigned long long mb = 0;
  // hot keys (stored with HOT_TAG, merge_hot.h) go to k_hub_hot, not to the partition
  int nst = 0;
  // (a source without a hot pass stages every key, decoded)
  const bool hotp = d.hot >= 0;
  hub_tile_walk(g, s, a, d.v, tk.x, d.tw, fl, [&](bool valid, int id, double, bool) {
    if (valid && (id >= 0 || !hotp)) { atomicAdd(&hist[hub_digit(s.keyd<HK>(id), d.logP)], 1u); nst++; }
  }, WalkRowMin{&mb, (int)s.L});
  nst = wave_sum(nst);
  if (lane_id() == 0 && nst) {
    atomicAdd(&staged[tk.d], (uint32_t)nst);
    if (a.diag) diag_add(a.diag, 140, (unsigned long long)nst);
  }
  if (!a.unit) {
#pragma unroll
    for (int o = 32; o; o >>= 1) { const unsigned long long y = __shfl_xor(mb, o); mb = y > mb ? y : mb; }
    if (lane_id() == 0 && mb) atomicMax(&tau[tk.d], mb);
  }
  wave_fence();
  for (int i = lane_id(); i < P; i += WAVE) cm[d.cm_off + (int64_t)i * d.T + tk.x] = (int32_t)hist[i];
}

template <bool HK>
__global__ void __launch_bounds__(256, 5) k_hub_scatter(DevGraph g, DevSlab s, IterArgs a,
                                                     const HubDesc* desc, const HubTask* tasks,
                                                     int64_t ntasks, int maxP, const int32_t* cm,
                                                     HubRec* st) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  // consecutive tiles of a source append to the same bucket runs: keep them on one XCD so the
  // partial staging lines merge in its L2 instead of being written back piecemeal
  const int64_t w = xcd_block(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + wv;
  if (w >= ntasks) return;
  const HubTask tk = tasks[w];
  const HubDesc d = desc[tk.d];
  const int P = 1 << d.logP;
  // running staging position of every bucket for this tile, seeded from the scanned count
  // matrix once (one strided gather), so the per-group scatter never waits on global memory
  // (offsets are relative to the source's staging start: they fit 32 bits)
  uint32_t* run = reinterpret_cast<uint32_t*>(smem) + (size_t)wv * maxP;
  // 16 strided loads per lane in flight at once (a 4096-bucket column is 64 loads per lane)
  const int64_t base0 = cm[d.cm_off];  // the source's first staged record (scanned counts)
  {
    const int32_t* col = cm + d.cm_off + tk.x;
    constexpr int GB = 16;
    for (int i0 = 0; i0 < P; i0 += WAVE * GB) {
      int32_t v[GB];
#pragma unroll
      for (int k = 0; k < GB; k++) {
        const int i = i0 + k * WAVE + lane_id();
        v[k] = i < P ? col[(int64_t)i * d.T] : 0;
      }
#pragma unroll
      for (int k = 0; k < GB; k++) {
        const int i = i0 + k * WAVE + lane_id();
        if (i < P) run[i] = (uint32_t)(v[k] - base0);
      }
    }
  }
  wave_fence();
  const uint64_t lt = lanemask_lt();
  HubRec* stv = st + base0;
  uint8_t* fl = smem + (size_t)(blockDim.x >> 6) * maxP * 4 + (size_t)wv * HUB_WALK_FLAGS;
  const bool hotp = d.hot >= 0;
#ifndef PPR_SCATTER_ORDERED
#define PPR_SCATTER_ORDERED 1
#endif
#ifndef PPR_SCATTER_ANYROW
#define PPR_SCATTER_ANYROW 0  // (A/B timing only: one add for every group, as before round 6)
#endif
#ifndef PPR_SCATTER_ROWS
#define PPR_SCATTER_ROWS 4
#endif
  constexpr int SCAT_ROWS = PPR_SCATTER_ROWS;  // most baskets a group may span and still take the adds
  const bool ordered = PPR_SCATTER_ORDERED && a.lds_rank != 0;
  hub_tile_walk(g, s, a, d.v, tk.x, d.tw, fl, [&](bool valid0, int id, double sv, bool one_row, int rr, int nr) {
    const bool valid = valid0 && (id >= 0 || !hotp);  // with a hot pass: cold keys only
    const int key = valid ? s.keyd<HK>(id) : 0;
    const uint32_t dg = valid ? hub_digit(key, d.logP) : 0u;
    if (a.whatif & (WI_SCAT_COUNT | WI_SCAT_WALK)) {  // (timing only: non-returning rank atomics / walk only)
      if (valid && (a.whatif & WI_SCAT_COUNT)) atomicAdd(&run[dg], 1u);
      if (valid && key == -5 && sv == -1.0) stv[0] = hub_rec(key, sv);
      return;
    }
    // The atomic ranks need no particular service order among lanes whose keys are distinct: a
    // stable partition only has to keep each KEY's contributions in stream order, and across
    // instructions program order does. The candidates of one successor basket have distinct keys,
    // so a group spanning up to SCAT_ROWS baskets takes one returning add per basket (exec-masked,
    // in basket order); wider groups take the ballot ranks. No result depends on the order in
    // which the LDS serves same-address atomics (round 6; before, on the per-plan probe alone).
    if (ordered && (nr <= SCAT_ROWS || PPR_SCATTER_ANYROW)) {
      uint32_t pos = 0u;
      const int nrr = PPR_SCATTER_ANYROW ? 1 : nr;
      for (int r = 0; r < nrr; r++) {
        const bool mine = valid && (PPR_SCATTER_ANYROW || rr == r);
        if (!(a.whatif & WI_RANK_PERMUTE)) {
          if (mine) pos = atomicAdd(&run[dg], 1u);
        } else {  // (tests: odd lanes first)
          if (mine && (lane_id() & 1)) pos = atomicAdd(&run[dg], 1u);
          wave_fence();
          if (mine && !(lane_id() & 1)) pos = atomicAdd(&run[dg], 1u);
        }
        wave_fence();
      }
      if (a.whatif & WI_SCAT_COALESCED) {  // (timing only: the same records stored lane-contiguously)
        const uint64_t vm = __ballot(valid);
        if (!vm) return;
        const uint32_t p0 = (uint32_t)__shfl((int)pos, __ffsll((long long)vm) - 1);
        pos = min(p0 + (uint32_t)lane_id(), (uint32_t)(d.need - 2));
      }
      // (timing only: keeps the loads and ranks, stores nothing)
      if (valid && (!(a.whatif & WI_SCAT_NOSTORE) || (sv == -1.0 && key == -5))) stv[pos] = hub_rec(key, sv);
      return;
    }
    // lanes holding the same digit: AND of per-bit ballots (stable rank = lower lanes first)
    uint64_t match = __ballot(valid);
    for (int bit = 0; bit < d.logP; bit++) {
      const uint64_t bb = __ballot(valid && ((dg >> bit) & 1u));
      match &= ((dg >> bit) & 1u) ? bb : ~bb;
    }
    const int rank = __popcll(match & lt);
    const uint32_t base = valid ? run[dg] : 0u;
    wave_fence();
    if (valid) {
      if (rank == 0) run[dg] = base + (uint32_t)__popcll(match);
      stv[base + rank] = hub_rec(key, sv);
    }
    wave_fence();
  });
}

// one bucket of the wave kernel, resolved once by k_hub_prep (thread per bucket) so the
// persistent bucket waves start each bucket with a single 64-B load
struct BucketWork {
  int64_t start;    // staging index of the bucket's first record
  int64_t pt_off;   // the source's appended-results list
  int32_t nb;       // records
  int32_t d;        // descriptor
  int32_t x;        // bucket (digit)
  int32_t seed;     // the source id when this bucket holds the source's own key, else -1
  double factor, tau, selfval;
  uint32_t ts;      // tie salt of the source (top-L ties, ppr_device.h)
  int32_t pad;
};

// pruning bound of a source's buckets: the larger of tau (full successor rows) and, once the hot
// pass of the source has published it, the L-th largest hot value (both are lower bounds of the
// L-th largest final value; a bound read as 0 before it is published only prunes less)
__device__ __forceinline__ double hub_tau(const HubDesc& d, const unsigned long long* tau_b, int di,
                                          const unsigned long long* tau_hot, double factor) {
  double t = tau_b[di] ? bitsd(tau_b[di]) * factor : 0.0;  // no bound: keep all (deg 0: factor inf)
  if (d.hot >= 0) {
    const unsigned long long th = __hip_atomic_load(&tau_hot[d.hot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (th && bitsd(th) > t) t = bitsd(th);
  }
  return t;
}

__global__ void __launch_bounds__(256) k_hub_prep(DevGraph g, DevSlab s, IterArgs a, HotSet H, const HubDesc* desc,
                                                  const HubTask* tasks, int64_t ntasks, const int32_t* cm,
                                                  const uint32_t* staged, const unsigned long long* tau_b,
                                                  const unsigned long long* tau_hot, BucketWork* bw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ntasks) return;
  const HubTask tk = tasks[i];
  const HubDesc d = desc[tk.d];
  BucketWork w;
  int64_t nb;
  hub_bucket_range(d, cm, staged[tk.d], tk.x, w.start, nb);
  w.nb = (int32_t)nb;
  w.pt_off = d.pt_off;
  w.d = tk.d;
  w.x = tk.x;
  // the source's own seed entry goes to its bucket, unless the hot pass owns the key
  w.seed = ((int)hub_digit(d.v, d.logP) == tk.x && !(d.hot >= 0 && H.has(d.v))) ? d.v : -1;
  const int64_t deg = g.rp[d.v + 1] - g.rp[d.v];
  w.factor = merge_factor(a, deg);
  w.tau = fmax(hub_tau(d, tau_b, tk.d, tau_hot, w.factor), spec_tau(s, a, d.v));
  w.selfval = self_seed(a, deg);
  w.ts = tie_salt(d.v);
  w.pad = 0;
  bw[i] = w;
}

// Bucket waves: one wave per bucket, its work record resolved by k_hub_prep. Per bucket: private LDS table (T slots, 3/4 usable; a bucket with more distinct
// keys spills to k_hub_bucket), chunks of NG groups loaded at once and accumulated with
// chunk_accumulate, then the keys >= tau, at most L of them, appended to the source's list.
// ---------------------------------------------------------------------------------------------
// One bucket on one wave: private LDS table (T slots, 3/4 usable), chunks of NG groups of 64
// ordered candidates accumulated with chunk_accumulate, then the keys >= tau, at most L of them,
// appended to the source's result list. Shared by the staged buckets (k_hub_bucket_w) and the
// segmented buckets (k_hub_seg).
struct BucketWave {
  LdsTable t;
  ChunkLds ck;
  uint32_t* hist;
  int T, budget, fill;
  bool overflow;
  bool ordered;  // lane-ordered LDS atomics (IterArgs::lds_rank), verified where used (chunk_accumulate)
  bool permute;  // (tests) WI_RANK_PERMUTE

  // T: any multiple of 64 (slots by multiply-shift of the key hash, linear probing with wrap)
  __device__ __forceinline__ void setup(unsigned char* base, int T_, int NG, bool ordered_, int budget_ = -1,
                                        bool permute_ = false) {
    T = T_;
    ordered = ordered_;
    permute = permute_;
    t.acc = reinterpret_cast<double*>(base);
    t.keys = reinterpret_cast<int*>(base + (size_t)T * 8);
    t.mask = (uint32_t)T - 1;
    t.nbits = 32 - __clz(T - 1);
    ck.cnt = reinterpret_cast<uint32_t*>(base + (size_t)T * 12);
    ck.vals = reinterpret_cast<double*>(base + (size_t)T * 16);
    ck.touched = reinterpret_cast<uint16_t*>(base + (size_t)T * 16 + (size_t)(NG * WAVE) * 8);
    ck.tof = ck.touched + NG * WAVE;
    ck.ord = ck.tof + NG * WAVE + 2;  // (tof holds NG * 64 + 1)
    hist = reinterpret_cast<uint32_t*>(ck.vals);  // final select only (after accumulation)
    budget = budget_ > 0 ? budget_ : T / 4 * 3;
    fill = 0;
    overflow = false;
    for (int i = lane_id(); i < T; i += WAVE) { t.keys[i] = EMPTY; ck.cnt[i] = 0; }
    wave_fence();
  }

  // an empty table again (the chunk counters are all-zero after every chunk)
  __device__ __forceinline__ void reset(int T_) {
    for (int i = lane_id(); i < T_; i += WAVE) t.keys[i] = EMPTY;
    fill = 0;
    overflow = false;
    wave_fence();
  }

  __device__ __forceinline__ uint32_t slot_of(int key) const {
    return (uint32_t)(((unsigned long long)hash32((uint32_t)key) * (uint32_t)T) >> 32);
  }

  __device__ __forceinline__ void seed(int key, double val) {
    if (lane_id() == 0) { const uint32_t sl = slot_of(key); t.keys[sl] = key; t.acc[sl] = val; }  // empty table
    fill = 1;
    wave_fence();
  }

  // find-or-insert the NG groups' keys, then accumulate them in stream order; sets overflow
  // (uniform) instead when the table could run out of slots
  template <int NG>
  __device__ __forceinline__ void chunk(const bool (&cv)[NG], const int (&kk)[NG], const double (&cs)[NG],
                                        double factor, unsigned long long* ph = nullptr) {
    uint32_t sl[NG];
    // the first probe of every group is read up front (NG LDS reads in flight instead of one
    // round trip per group): a slot only ever goes EMPTY -> key, so a stale EMPTY is caught by
    // the CAS below and a key read early is final
    uint32_t h0[NG];
    int c0[NG];
#pragma unroll
    for (int k = 0; k < NG; k++) {
      h0[k] = slot_of(kk[k]);
      c0[k] = cv[k] ? t.keys[h0[k]] : EMPTY;
    }
#pragma unroll
    for (int k = 0; k < NG; k++) {
      // uniform: at most the lanes whose early probe did not already show their key can bring a
      // new key (a stale EMPTY counts as new), so a bucket spills only when the table could
      // really pass its budget -- not whenever it holds more than budget - 64 keys
      const int maybe_new = __popcll(__ballot(cv[k] && c0[k] != kk[k]));
      if (fill + maybe_new > budget) overflow = true;
      bool ins = false, lost = false;
      uint32_t h = 0;
      if (cv[k] && !overflow) {
        h = h0[k];
        int c = c0[k];
        for (;;) {
          if (c == kk[k]) break;
          if (c == EMPTY) {
            const int prev = atomicCAS(&t.keys[h], EMPTY, kk[k]);
            if (prev == EMPTY) { t.acc[h] = 0.0; ins = true; break; }
            if (prev == kk[k]) break;
          }
          h = (h + 1 == (uint32_t)T) ? 0u : h + 1;
          if (h == h0[k]) { lost = true; break; }  // (bounded: back at the start, the table is full --
          c = t.keys[h];                            // the bucket spills like one past its budget)
        }
      }
      if (__ballot(lost)) overflow = true;
      sl[k] = h;
      fill += __popcll(__ballot(ins));
      wave_fence();
    }
    if (overflow) return;
    long long t1 = 0;
    if (ph) {  // PPR_DIAG phase split: find-or-insert (with the probes) | ordered accumulation
      t1 = (long long)clock64();
      ph[2] += (unsigned long long)(t1 - (long long)ph[8]);
    }
    chunk_accumulate<NG>(t.acc, ck, t.nbits, cv, sl, cs, factor, ordered, ph, permute);
    if (ph) {
      const int z = t.keys[0];  // wait for the chains' LDS traffic before reading the clock
      if (z == 0x7ffffffe) wave_fence();
      const long long t2 = (long long)clock64();
      ph[3] += (unsigned long long)(t2 - t1);
      ph[8] = (unsigned long long)t2;
    }
  }

  // keys >= tau (at most L by (score desc, tie_w desc)) appended to the source's list
  __device__ __forceinline__ void emit(double tau, int Lw, uint32_t* pt_cnt_d, int32_t* pt_key, double* pt_sc,
                                       const IterArgs& a, uint32_t ts, unsigned long long* ph = nullptr) {
    const int l = lane_id();
    // compact the occupied slots that can still reach the top-L (value >= tau) to the front, in
    // one pass (writes land at or below the slots already read)
    int U = 0, Uall = 0;
    for (int i0 = 0; i0 < T; i0 += WAVE) {
      const int i = i0 + l;
      const int k = t.keys[i];
      const double x = t.acc[i];
      const bool occ = k != EMPTY;
      const bool keep = occ && x >= tau;
      const uint64_t m = __ballot(keep);
      if (a.diag) Uall += __popcll(__ballot(occ));
      wave_fence();
      if (keep) { const int pos = U + __popcll(m & lanemask_lt()); t.keys[pos] = k; t.acc[pos] = x; }
      U += __popcll(m);
      wave_fence();
    }
    if (a.diag && l == 0) {  // distinct keys / kept keys per bucket
      diag_add(a.diag, 64 + (31 - __clz(Uall | 1)), 1ull);
      diag_add(a.diag, 96 + (31 - __clz(U | 1)), 1ull);
    }
    const int cnt = U <= Lw ? U : Lw;
    if (cnt == 0) return;
    SelCrit c;
    const int* keys = t.keys;
    const double* acc = t.acc;
    if (U > Lw) c = select_top(U, Lw, [&](int i) { return keys[i]; }, [&](int i) { return acc[i]; }, hist, ts);
    long long t1 = 0;
    if (ph) {
      t1 = (long long)clock64();
      ph[4] += (unsigned long long)(t1 - (long long)ph[8]);
      if (l == 0) { ph[9] += U > Lw ? 1ull : 0ull; ph[10] += (unsigned long long)cnt; }
    }
    int at = 0;
    if (l == 0) at = (int)atomicAdd(pt_cnt_d, (uint32_t)cnt);
    at = __builtin_amdgcn_readlane(at, 0);
    int32_t* ok = pt_key + at;
    double* os = pt_sc + at;
    if (ph) ph[5] += (unsigned long long)((long long)clock64() - t1);
    if (U <= Lw) {
      for (int i = l; i < U; i += WAVE) { ok[i] = t.keys[i]; os[i] = t.acc[i]; }
      return;
    }
    int pos0 = 0;
    for (int i0 = 0; i0 < U; i0 += WAVE) {
      const int i = i0 + l;
      bool sel = false;
      if (i < U) sel = sel_test(c, dbits(acc[i]), tie_w(keys[i], ts));
      const uint64_t m = __ballot(sel);
      if (sel) { const int pos = pos0 + __popcll(m & lanemask_lt()); ok[pos] = keys[i]; os[pos] = acc[i]; }
      pos0 += __popcll(m);
    }
  }
};

// ---------------------------------------------------------------------------------------------
// One-shot bucket (default for buckets of at most BW2_CAP records, with lane-ordered LDS atomics):
// the whole bucket is loaded into registers at once and accumulated in one pass instead of chunk
// by chunk. Per table slot a 32-bit key and a 32-bit counter:
//   P1  per group, in stream order: find-or-insert every key (32-bit CAS; which lane of a group
//       wins an empty slot does not matter), then one returning 32-bit add on the key's counter
//       for every lane at once -- same-address lanes of one instruction are served in lane order
//       (probed per plan, k_probe_lds_rank ok[0]) and the groups go in order, so the returned
//       value is the record's occurrence index in stream order; new slots listed;
//   P2  exclusive scan of the listed slots' counts -> each slot's run base (over its counter);
//   P3  every record's value to vals[base + occurrence]: the bucket's values grouped by key, in
//       stream order inside a key;
//   P4  one lane per listed slot: the key's fma chain over its run, seeded with the source's own
//       value for the seed key (include/grank.h:103-116 order); the total overwrites the run's
//       last value;
//   P5  totals >= tau (at most L by (score desc, tie_w desc)) appended to the source's list.
// (Round 5: the round-2 form kept key, count and base in one 64-bit word and needed the 64-bit
// CAS and add in lane order too; on the round-5 MI355X boxes only the 32-bit order held, which
// had switched this path and the ordered ranks of the scatter and the chunks off.)
// The chunked path needs ~10 dependent LDS round trips per 128 records plus a 512-slot compaction
// per bucket; this one ~20 per bucket. Buckets it cannot take (more records) use the chunked path.
constexpr int BW2_GROUPS = 8;
constexpr int BW2_CAP = BW2_GROUPS * WAVE;  // records
__host__ __device__ constexpr size_t bw2_lds(int T) {  // keys | counters | vals | listed slots | select histogram
  return ((size_t)T * 8 + (size_t)BW2_CAP * 8 + (size_t)BW2_CAP * 2 + 1024 + 15) & ~(size_t)15;
}

__device__ __forceinline__ uint32_t bw2_slot(int key, int T) {
  return (uint32_t)(((unsigned long long)hash32((uint32_t)key) * (uint32_t)T) >> 32);
}

// returns false when the bucket's distinct keys could exceed `budget` (the caller spills it)
__device__ __forceinline__ bool bucket_oneshot(unsigned char* base, int T, int budget, const BucketWork& W, int nb,
                                               const HubRec* st, const IterArgs& a, int Lw, uint32_t* pt_cnt_d,
                                               int32_t* pt_key, double* pt_sc) {
  const int l = lane_id();
  // (-DPPR_PHASE_TIMING builds, PPR_DIAG: lane-0 cycles per phase into slots 288.., buckets in 296)
#if defined(PPR_PHASE_TIMING)
  long long tq = a.diag ? (long long)clock64() : 0;
  auto lap = [&](int k) {
    if (!a.diag) return;
    const long long t2 = (long long)clock64();
    if (l == 0) diag_add(a.diag, 288 + k, (unsigned long long)(t2 - tq));
    tq = t2;
  };
#else
  auto lap = [](int) {};
#endif
  uint32_t* keys = reinterpret_cast<uint32_t*>(base);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(base + (size_t)T * 4);
  double* vals = reinterpret_cast<double*>(base + (size_t)T * 8);
  uint16_t* listed = reinterpret_cast<uint16_t*>(base + (size_t)T * 8 + (size_t)BW2_CAP * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + (size_t)T * 8 + (size_t)BW2_CAP * 10);
  // stream positions of the values (P3, P4: verifies the occurrence order; the select's histogram,
  // used only after P4, occupies the same 1 KB)
  uint16_t* ord = reinterpret_cast<uint16_t*>(hist);
  static_assert(BW2_CAP * 2 <= 1024, "one-shot positions alias the select histogram");
  constexpr uint32_t EMPTYK = 0xffffffffu;  // (keys are >= 0)
  const int ng = (nb + WAVE - 1) / WAVE;  // (uniform) groups holding records
  int kk[BW2_GROUPS];
  double cs[BW2_GROUPS];
#pragma unroll
  for (int k = 0; k < BW2_GROUPS; k++) {  // every load in flight at once
    const int q = k * WAVE + l;
    HubRec r{};
    if (q < nb) r = st[W.start + q];
    kk[k] = rec_key(r);
    cs[k] = rec_sc(r);
  }
  for (int i = l; i < T; i += WAVE) { keys[i] = EMPTYK; cnt[i] = 0u; }
  wave_fence();
  int nt = 0;
  if (W.seed >= 0) {  // the source's own key: listed, no occurrence yet (its chain starts at selfval)
    if (l == 0) {
      const uint32_t h = bw2_slot(W.seed, T);
      keys[h] = (uint32_t)W.seed;
      listed[0] = (uint16_t)h;
    }
    nt = 1;
    wave_fence();
  }
  {  // (timing: wait for the record loads)
    int z = 0;
#pragma unroll
    for (int k = 0; k < BW2_GROUPS; k++) z += kk[k];
    if (z == 0x7ffffff1) wave_fence();
  }
  lap(0);  // loads + table clear
  const uint64_t lt = lanemask_lt();
  uint32_t sl[BW2_GROUPS], occ[BW2_GROUPS], c0[BW2_GROUPS];
#pragma unroll
  for (int k = 0; k < BW2_GROUPS; k++) {  // first probes up front (a stale EMPTY is caught by the CAS)
    sl[k] = bw2_slot(kk[k], T);
    c0[k] = (k < ng && k * WAVE + l < nb) ? keys[sl[k]] : EMPTYK;
  }
  // P1
#pragma unroll
  for (int k = 0; k < BW2_GROUPS; k++) {
    if (k >= ng) break;  // uniform
    const bool v = k * WAVE + l < nb;
    // at most the lanes whose early probe did not show their key bring a new key
    const int maybe_new = __popcll(__ballot(v && c0[k] != (uint32_t)kk[k]));
    if (nt + maybe_new > budget) return false;
    uint32_t h = sl[k];
    bool fresh = false;
    bool lost = false;
    if (v) {
      uint32_t w = c0[k];
      lost = true;  // (bounded probe: a full table fails the pass, the caller spills the bucket)
      for (int n = 0; n < 2 * T; n++) {
        if (w == (uint32_t)kk[k]) { lost = false; break; }
        if (w == EMPTYK) {
          const uint32_t prev = atomicCAS(&keys[h], EMPTYK, (uint32_t)kk[k]);
          if (prev == EMPTYK) { fresh = true; lost = false; break; }
          w = prev;  // taken meanwhile (another lane or an earlier group): test the same slot again
          continue;
        }
        h = (h + 1 == (uint32_t)T) ? 0u : h + 1;
        w = keys[h];
      }
    }
    if (__ballot(lost)) return false;
    wave_fence();
    // occurrence indices: one returning add for the whole group, same-slot lanes in the hardware's
    // order (lane order where probed; P4 verifies it)
    occ[k] = 0u;
    if (!(a.whatif & WI_RANK_PERMUTE)) {
      if (v) occ[k] = atomicAdd(&cnt[h], 1u);
    } else {  // (tests: odd lanes first)
      if (v && (l & 1)) occ[k] = atomicAdd(&cnt[h], 1u);
      wave_fence();
      if (v && !(l & 1)) occ[k] = atomicAdd(&cnt[h], 1u);
    }
    sl[k] = h;
    const uint64_t fm = __ballot(fresh);
    if (fresh) listed[nt + __popcll(fm & lt)] = (uint16_t)h;
    nt += __popcll(fm);
    wave_fence();
  }
  lap(1);  // P1
  // P2: run bases (listed order) over the counters; the total after the last run
  int run = 0;
  for (int i0 = 0; i0 < nt; i0 += WAVE) {
    const int i = i0 + l;
    int c = 0;
    if (i < nt) c = (int)cnt[listed[i]];
    const int incl = wave_incl_scan(c);
    if (i < nt) cnt[listed[i]] = (uint32_t)(run + incl - c);
    run += __builtin_amdgcn_readlane(incl, WAVE - 1);
  }
  const int total = run;
  wave_fence();
  lap(2);
  // P3: values grouped by key, each with its stream position; then the order check (ppr_device.h
  // chunk_accumulate: a record with occurrence index > 0 must come after its left neighbour)
  uint32_t qq[BW2_GROUPS];
#pragma unroll
  for (int k = 0; k < BW2_GROUPS; k++) {
    qq[k] = 0u;
    if (k >= ng) break;
    if (k * WAVE + l < nb) {
      qq[k] = cnt[sl[k]] + occ[k];
      vals[qq[k]] = cs[k];
      ord[qq[k]] = (uint16_t)(k * WAVE + l);
    }
  }
  wave_fence();
  bool bad = false;
#pragma unroll
  for (int k = 0; k < BW2_GROUPS; k++) {
    if (k >= ng) break;
    if (k * WAVE + l < nb && occ[k] > 0u) bad = bad || (int)ord[qq[k] - 1] > k * WAVE + l;
  }
  const bool sorted_path = __ballot(bad) != 0ull;
  lap(3);
  // run of listed slot i: [cnt[listed[i]], next run's base or the total)
  auto run_end = [&](int i) { return i + 1 < nt ? (int)cnt[listed[i + 1]] : total; };
  // P4: one chain per listed slot
  const double f = W.factor;
  for (int i0 = 0; i0 < nt; i0 += WAVE) {
    const int i = i0 + l;
    if (i < nt) {
      const int b = (int)cnt[listed[i]], e = run_end(i);
      const double x0 = ((int)keys[listed[i]] == W.seed) ? W.selfval : 0.0;
      const double x = __builtin_expect(sorted_path, 0)
                           ? fma_chain_sorted(vals, [&](int j) { return (int)ord[j]; }, b, e, f, x0)
                           : fma_chain_lds(vals, b, e, f, x0);
      if (e > b) vals[e - 1] = x;
    }
  }
  wave_fence();
  lap(4);
  // P5: keys reaching tau, at most L of them, appended
  auto total_of = [&](int i) {
    const int b = (int)cnt[listed[i]], e = run_end(i);
    return e > b ? vals[e - 1] : W.selfval;  // (a slot without occurrences is the seed key)
  };
  auto key_of = [&](int i) { return (int)keys[listed[i]]; };
  int kept = 0;
  for (int i0 = 0; i0 < nt; i0 += WAVE) {
    const int i = i0 + l;
    kept += __popcll(__ballot(i < nt && total_of(i) >= W.tau));
  }
  if (a.diag && l == 0) {  // distinct keys / kept keys per bucket
    diag_add(a.diag, 64 + (31 - __clz(nt | 1)), 1ull);
    diag_add(a.diag, 96 + (31 - __clz(kept | 1)), 1ull);
  }
  if (kept == 0) { lap(5); return true; }
  const int cntk = kept <= Lw ? kept : Lw;
  SelCrit c;
  const uint32_t ts = W.ts;
  const double tau = W.tau;
  if (kept > Lw)  // keys below tau rank as 0 (every kept total is >= tau > 0 here)
    c = select_top(nt, Lw, key_of, [&](int i) { const double x = total_of(i); return x >= tau ? x : 0.0; }, hist, ts);
  lap(5);  // kept count + select
  int at = 0;
  if (l == 0) at = (int)atomicAdd(pt_cnt_d, (uint32_t)cntk);
  at = __builtin_amdgcn_readlane(at, 0);
  lap(6);  // appending atomic
  int pos0 = 0;
  for (int i0 = 0; i0 < nt; i0 += WAVE) {
    const int i = i0 + l;
    bool sel = false;
    double x = 0.0;
    int key = 0;
    if (i < nt) {
      x = total_of(i);
      key = key_of(i);
      sel = x >= tau && (kept <= Lw || sel_test(c, dbits(x), tie_w(key, ts)));
    }
    const uint64_t m = __ballot(sel);
    if (sel) { const int pos = at + pos0 + __popcll(m & lt); pt_key[pos] = key; pt_sc[pos] = x; }
    pos0 += __popcll(m);
  }
  lap(7);  // emission
#if defined(PPR_PHASE_TIMING)
  if (a.diag && l == 0) diag_add(a.diag, 296, 1ull);
#endif
  return true;
}

// Bucket waves over the staged partition: one wave per bucket, its work record resolved by
// k_hub_prep; a bucket with more distinct keys than the table holds spills to k_hub_bucket.
template <int NG>
__global__ void __launch_bounds__(256) k_hub_bucket_w(DevSlab s, IterArgs a, const BucketWork* bw,
                                                      int64_t nbuck, const HubRec* st,
                                                      int32_t* pt_key, double* pt_sc, uint32_t* pt_cnt,
                                                      HubTask* spill, uint32_t* spill_cnt, int T, int budget, int dry,
                                                      int wbytes, int cap2) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int l = lane_id();
  // one bucket per wave (persistent waves with a static stride or a shared work counter measured
  // slower: the hardware refills CUs better than a fixed grid balances hot buckets)
  const int64_t cur = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (cur >= nbuck) return;
  const long long t_start = a.diag ? (long long)clock64() : 0;
  const BucketWork W = bw[cur];
  // PPR_DIAG: per-phase cycles of this wave (lane-uniform registers; [8] = last stamp):
  // 0 work record + table setup, 1 record loads, 2 find-or-insert, 3 ordered accumulation,
  // 4 compaction + select, 5 appending atomic; 9 buckets that select (U > L), 10 entries appended
  // (compiled in only with -DPPR_PHASE_TIMING, tools/build_variant.py: the counters live in private
  // memory -- 128 B of scratch per lane, 3 TB of scratch writes per RMAT-22 job if always present)
#if defined(PPR_PHASE_TIMING)
  unsigned long long phv[15] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // (11-14: chunk phases A-D)
  unsigned long long* ph = (a.diag && (cur & 7) == 0) ? phv : nullptr;  // one wave in 8 (the clock reads cost)
#else
  unsigned long long* ph = nullptr;
#endif
  // (PPR_WHATIF 128, timing only: long buckets cut to 2048 records -- what the hot-key chains cost)
  const int nb = ((a.whatif & 128u) && W.nb > 2048) ? 2048 : W.nb;
  if (nb <= cap2 && !dry && !ph) {  // (cap2 = 0: one-shot path off, or LDS atomics not lane-ordered)
    if (!bucket_oneshot(smem + (size_t)wv * wbytes, T, budget, W, nb, st, a, s.L, &pt_cnt[W.d], pt_key + W.pt_off,
                        pt_sc + W.pt_off)) {
      if (l == 0) { const uint32_t pos = atomicAdd(spill_cnt, 1u); spill[pos] = HubTask{W.d, W.x}; }
      if (a.diag && l == 0) {
        diag_add(a.diag, 152, 1ull);
        diag_add(a.diag, 153, (unsigned long long)nb);
      }
    } else if (a.diag && l == 0) {
      const int bin = 31 - __clz(nb | 1);
      diag_add(a.diag, bin, 1ull);
      diag_add(a.diag, 32 + bin, (unsigned long long)((long long)clock64() - t_start));
    }
    return;
  }
  BucketWave B;
  B.setup(smem + (size_t)wv * wbytes, T, NG, a.lds_rank != 0, budget, (a.whatif & WI_RANK_PERMUTE) != 0);
  if (W.seed >= 0) B.seed(W.seed, W.selfval);
  if (ph) { ph[8] = (unsigned long long)clock64(); ph[0] = ph[8] - (unsigned long long)t_start; }
  // the next chunk's records are loaded while the current chunk is accumulated (MC combine
  // 1028-1030 -> 1017-1018 ms same-box)
  HubRec nxt[NG];
  auto load_chunk = [&](int g0, HubRec (&r)[NG]) {
#pragma unroll
    for (int k = 0; k < NG; k++) {
      const int q = g0 + k * WAVE + l;
      r[k] = HubRec{};
      if (q < nb) {
        if (a.nt & 2u) {
          const uint32_t* w = st[W.start + q].w;
          r[k].w[0] = __builtin_nontemporal_load(w);
          r[k].w[1] = __builtin_nontemporal_load(w + 1);
          r[k].w[2] = __builtin_nontemporal_load(w + 2);
        } else {
          r[k] = st[W.start + q];
        }
      }
    }
  };
  load_chunk(0, nxt);
  for (int g0 = 0; g0 < nb; g0 += NG * WAVE) {
    bool cv[NG];
    double cs[NG];
    int kk[NG];
#pragma unroll
    for (int k = 0; k < NG; k++) {
      cv[k] = g0 + k * WAVE + l < nb;
      kk[k] = rec_key(nxt[k]);
      cs[k] = rec_sc(nxt[k]);
    }
    if (g0 + NG * WAVE < nb) load_chunk(g0 + NG * WAVE, nxt);
    if (ph) {  // wait for the loads before timing them
      int z = 0;
#pragma unroll
      for (int k = 0; k < NG; k++) z += kk[k] + (int)(cs[k] > 2.0);
      if (z == 0x7fffffff) wave_fence();
      const long long t2 = (long long)clock64();
      ph[1] += (unsigned long long)(t2 - (long long)ph[8]);
      ph[8] = (unsigned long long)t2;
    }
    B.chunk<NG>(cv, kk, cs, W.factor, ph);
    if (B.overflow) break;
  }
  if (dry) {  // PPR_WHATIF timing pass: accumulate only (keep the table live)
    if (l == 0 && B.t.keys[0] == 0x7ffffffe) pt_cnt[W.d] = 0;
    return;
  }
  if (B.overflow) {
    if (l == 0) { const uint32_t pos = atomicAdd(spill_cnt, 1u); spill[pos] = HubTask{W.d, W.x}; }
    if (a.diag && l == 0) {  // spilled buckets and their records
      diag_add(a.diag, 152, 1ull);
      diag_add(a.diag, 153, (unsigned long long)nb);
    }
    return;
  }
  if (a.diag && l == 0) {  // bucket length histogram: count and cycles per log2(length) bin
    const int bin = 31 - __clz(nb | 1);
    diag_add(a.diag, bin, 1ull);
    diag_add(a.diag, 32 + bin, (unsigned long long)((long long)clock64() - t_start));
  }
  B.emit(W.tau, s.L, &pt_cnt[W.d], pt_key + W.pt_off, pt_sc + W.pt_off, a, W.ts, ph);
  if (ph && l == 0) {
    for (int k = 0; k < 6; k++) diag_add(a.diag, 160 + k, ph[k]);
    diag_add(a.diag, 166, 1ull);
    diag_add(a.diag, 167, (unsigned long long)nb);
    diag_add(a.diag, 168, ph[9]);
    diag_add(a.diag, 169, ph[10]);
    for (int k = 11; k < 15; k++) diag_add(a.diag, 172 + k - 11, ph[k]);
  }
}

// Bucket ranges: one wave per range of krange consecutive buckets of one source (HubTask (d, x0)),
// its LDS table reused bucket after bucket. A bucket wave pays a few dependent global round
// trips that its ~100-300 records cannot hide (its work record, then its records, then the
// returning atomic of its emission); a range pays the first two once: the bucket bounds of the
// whole range come from one load of the scanned count matrix, and the records stream through
// the range with the next chunk -- the next bucket's first chunk included -- in flight while the
// current one is accumulated or emitted. Per bucket the semantics are k_hub_bucket_w's: seed,
// ordered accumulation, spill to k_hub_bucket on overflow, keys >= tau (at most L) appended.
template <int NG>
__global__ void __launch_bounds__(256) k_hub_range(DevGraph g, DevSlab s, IterArgs a, HotSet H, const HubDesc* desc,
                                                   const HubTask* tasks, int64_t ntasks, int krange, const int32_t* cm,
                                                   const uint32_t* staged, const unsigned long long* tau_b,
                                                   const unsigned long long* tau_hot, const HubRec* st,
                                                   int32_t* pt_key, double* pt_sc, uint32_t* pt_cnt,
                                                   HubTask* spill, uint32_t* spill_cnt, int T, int budget) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int l = lane_id();
  const int64_t cur = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (cur >= ntasks) return;
  const HubTask tk = tasks[cur];
  const HubDesc d = desc[tk.d];
  const int P = 1 << d.logP;
  const int x0 = tk.x, x1 = min(P, x0 + krange);
  // lane i: staging start of bucket x0 + i (lane x1 - x0: the end of the last one)
  int64_t bs = d.st_off;
  if (d.T > 0 && l <= x1 - x0) {
    const int x = x0 + l;
    bs = x < P ? (int64_t)cm[d.cm_off + (int64_t)x * d.T] : (int64_t)cm[d.cm_off] + (int64_t)staged[tk.d];
  }
  const int v = d.v;
  const int64_t deg = g.rp[v + 1] - g.rp[v];
  const double factor = merge_factor(a, deg);
  const double tau = hub_tau(d, tau_b, tk.d, tau_hot, factor);
  const int seed_x = (d.hot >= 0 && H.has(v)) ? -1 : (int)hub_digit(v, d.logP);
  BucketWave B;
  unsigned char* base = smem + (size_t)wv * hub_wave_lds(T, NG);
  B.setup(base, T, NG, a.lds_rank != 0, budget, (a.whatif & WI_RANK_PERMUTE) != 0);
  auto bstart = [&](int x) { return (int64_t)__shfl((long long)bs, x - x0); };
  bool cv[NG], nv[NG];
  int kk[NG], nk[NG];
  double cs[NG], ns[NG];
  auto load = [&](int x, int g0, bool (&vv)[NG], int (&kv)[NG], double (&sv)[NG]) {
    const int64_t b0 = bstart(x), nb = bstart(x + 1) - b0;
#pragma unroll
    for (int k = 0; k < NG; k++) {
      const int q = g0 + k * WAVE + l;
      vv[k] = q < nb;
      const HubRec r = vv[k] ? st[b0 + q] : HubRec{};
      kv[k] = rec_key(r);
      sv[k] = rec_sc(r);
    }
  };
  int x = x0, g0 = 0;
  load(x, 0, nv, nk, ns);
  while (x < x1) {
#pragma unroll
    for (int k = 0; k < NG; k++) { cv[k] = nv[k]; kk[k] = nk[k]; cs[k] = ns[k]; }
    const int nb = (int)(bstart(x + 1) - bstart(x));
    int nx = x, ng0 = g0 + NG * WAVE;
    if (ng0 >= nb) { nx = x + 1; ng0 = 0; }
    if (nx < x1) load(nx, ng0, nv, nk, ns);  // in flight while this chunk is used
    if (g0 == 0 && x == seed_x) B.seed(v, self_seed(a, deg));
    if (!B.overflow) B.chunk<NG>(cv, kk, cs, factor);
    if (nx != x) {  // bucket x complete
      if (B.overflow) {
        if (l == 0) { const uint32_t pos = atomicAdd(spill_cnt, 1u); spill[pos] = HubTask{tk.d, x}; }
      } else {
        B.emit(tau, s.L, &pt_cnt[tk.d], pt_key + d.pt_off, pt_sc + d.pt_off, a, tie_salt(v));
      }
      if (nx < x1) B.reset(T);
    }
    x = nx;
    g0 = ng0;
  }
}

// Segmented buckets (no partition pass): basket rows are stored in hash_b order with a range
// index (DevSlab::rix), so bucket x of a source with logP <= RANGE_BITS buckets -- the keys whose
// top logP hash bits equal x -- is ONE contiguous segment of every successor row. One wave per
// (source, bucket) walks the successors in order, 64 at a time: per successor the segment bounds
// (two u16 of one 128-B index line) and, for the pruning bound, the row minimum of full rows;
// then the window's segments are gathered as one ordered candidate stream, NG groups per chunk.
// Stream order is successor order, so every key's fma chain keeps the reference order.
template <int NG>
__global__ void __launch_bounds__(256) k_hub_seg(DevGraph g, DevSlab s, IterArgs a, const HubDesc* desc,
                                                 const HubTask* tasks, int64_t ntasks, int32_t* pt_key,
                                                 double* pt_sc, uint32_t* pt_cnt, int32_t* ovf_flag,
                                                 int32_t* ovf_list, int T) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int l = lane_id();
  const int64_t cur = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (cur >= ntasks) return;
  const HubTask tk = tasks[cur];
  const HubDesc d = desc[tk.d];
  const int v = d.v;
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = merge_factor(a, e - b);
  const int sh = RANGE_BITS - d.logP;                // ranges per bucket: 1 << sh
  const int r0 = tk.x << sh, r1 = (tk.x + 1) << sh;  // ranges [r0, r1)
  // PPR_DIAG: cycles per phase (setup, successor window, gather, accumulate, emit), waves, candidates
  const bool dg = a.diag != nullptr;
  long long tc = dg ? (long long)clock64() : 0;
  unsigned long long ph[5] = {0, 0, 0, 0, 0}, ncand = 0;
  auto lap = [&](int k) {
    if (dg) { const long long t2 = (long long)clock64(); ph[k] += (unsigned long long)(t2 - tc); tc = t2; }
  };
  BucketWave B;
  B.setup(smem + (size_t)wv * hub_wave_lds(T, NG), T, NG, a.lds_rank != 0, -1, (a.whatif & WI_RANK_PERMUTE) != 0);
  {
    const int rg = (int)row_range(v);
    if (rg >= r0 && rg < r1) B.seed(v, self_seed(a, e - b));
  }
  lap(0);
  unsigned long long mb = 0;  // max row minimum over full successor rows (unscaled)
  for (int64_t e0 = b; e0 < e; e0 += WAVE) {
    const int64_t i = e0 + l;
    int u = 0, sl = 0, lo = 0, ln = 0;
    if (i < e) {
      const int32_t cx = g.colx[i];
      u = cx & 0x7fffffff;
      sl = read_slot(a, cx);
      const uint16_t* ix = s.rix + s.xrow(sl, u);
      lo = r0 ? (int)ix[r0 - 1] : 0;
      ln = (int)ix[r1 - 1] - lo;
      if ((int)ix[NRANGE - 1] == s.L) {
        const unsigned long long m = dbits(s.rmin[s.lrow(sl, u)]);
        mb = m > mb ? m : mb;
      }
    }
    const int incl = wave_incl_scan(ln);
    const int total = __builtin_amdgcn_readlane(incl, WAVE - 1);
    ncand += (unsigned long long)total;
    lap(1);
    for (int g0 = 0; g0 < total; g0 += NG * WAVE) {
      bool cv[NG];
      double cs[NG];
      int kk[NG];
#pragma unroll
      for (int k = 0; k < NG; k++) {
        const int c = g0 + k * WAVE + l;
        int j = 0;
#pragma unroll
        for (int step = 32; step; step >>= 1) {
          const int pv = __shfl(incl, j + step - 1);
          if (pv <= c) j += step;
        }
        const int jj = j < WAVE ? j : WAVE - 1;
        const int exv = __shfl(incl, jj > 0 ? jj - 1 : 0);
        const int ex = jj > 0 ? exv : 0;
        const int uj = __shfl(u, jj);
        const int sj = __shfl(sl, jj);
        const int lj = __shfl(lo, jj);
        cv[k] = c < total;
        kk[k] = 0;
        cs[k] = 0.0;
        if (cv[k]) {
          const int64_t r = s.row(sj, uj) + lj + (c - ex);
          kk[k] = s.key(s.ids[r]);
          cs[k] = s.sc[r];
        }
      }
      if (dg) {  // wait for the gathers before timing them
        int z = 0;
#pragma unroll
        for (int k = 0; k < NG; k++) z += kk[k] + (int)(cs[k] > 2.0);
        if (z == 0x7fffffff) wave_fence();
        lap(2);
      }
      B.chunk<NG>(cv, kk, cs, factor);
      lap(3);
      if (B.overflow) break;
    }
    if (B.overflow) break;
  }
  if (B.overflow) {
    // more distinct keys than the wave table: the whole source takes the HBM-table path
    if (l == 0 && atomicExch(&ovf_flag[tk.d], 1) == 0) {
      const int pos = atomicAdd(&ovf_list[0], 1);
      ovf_list[1 + pos] = v;
    }
    return;
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) { const unsigned long long y = __shfl_xor(mb, o); mb = y > mb ? y : mb; }
  const double tau = mb ? bitsd(mb) * factor : 0.0;
  B.emit(tau, s.L, &pt_cnt[tk.d], pt_key + d.pt_off, pt_sc + d.pt_off, a, tie_salt(v));
  if (dg) {
    lap(4);
    if (l == 0) {
      for (int k = 0; k < 5; k++) diag_add(a.diag, 128 + k, ph[k]);
      diag_add(a.diag, 133, 1ull);
      diag_add(a.diag, 134, ncand);
    }
  }
}

__device__ __forceinline__ void hub_bucket_one(const DevSlab& s, const IterArgs& a, const DevGraph& g, const HotSet& H,
                                               const HubDesc* desc, const HubTask tk, const int32_t* cm,
                                               const uint32_t* staged, const HubRec* st, int32_t* pt_key, double* pt_sc,
                                               uint32_t* pt_cnt, const unsigned long long* tau_b,
                                               const unsigned long long* tau_hot, int Lp,
                                               int32_t* ovf_flag, int32_t* ovf_list) {
  extern __shared__ __align__(16) unsigned char smem[];
  const HubDesc d = desc[tk.d];

  const WgLds L = wg_carve(smem, WG_T, Lp, wg_pl(Lp));
  const int wv = threadIdx.x >> 6;
  const int l = lane_id();
  const int v = d.v;
  int64_t sb, nb;
  hub_bucket_range(d, cm, staged[tk.d], tk.x, sb, nb);
  const bool seed = (int)hub_digit(v, d.logP) == tk.x && !(d.hot >= 0 && H.has(v));
  const int64_t deg = g.rp[v + 1] - g.rp[v];
  const double factor = merge_factor(a, deg);
  const int Lw = s.L;
  // the bucket stream: staged (key, score) in successor order, next chunk loaded ahead
  auto each = [&](auto&& fn) {
    auto ld = [&](int64_t q, bool& vv, int& kk, double& ss) {
      vv = q < nb;
      const HubRec r = vv ? st[sb + q] : HubRec{};
      kk = rec_key(r);
      ss = rec_sc(r);
    };
    bool nv0, nv1;
    int nk0, nk1;
    double ns0, ns1;
    ld(wv * 128 + l, nv0, nk0, ns0);
    ld(wv * 128 + 64 + l, nv1, nk1, ns1);
    for (int64_t c0 = 0; c0 < nb; c0 += WG_CHUNK) {
      const bool cv0 = nv0, cv1 = nv1;
      const int ck0 = nk0, ck1 = nk1;
      const double cs0 = ns0, cs1 = ns1;
      if (c0 + WG_CHUNK < nb) {
        ld(c0 + WG_CHUNK + wv * 128 + l, nv0, nk0, ns0);
        ld(c0 + WG_CHUNK + wv * 128 + 64 + l, nv1, nk1, ns1);
      }
      fn(cv0, ck0, cs0, cv1, ck1, cs1);
    }
  };
  // optimistic single pass: a bucket dominated by a few hot keys holds few distinct keys
  int Pp = 1;
  for (;;) {
    if (wg_accumulate(L, Pp, 0x51ed270bu, seed, v, self_seed(a, deg), factor, Lw, each)) break;
    Pp *= 2;
    if (Pp > WG_MAX_PASSES) {
      if (threadIdx.x == 0 && atomicExch(&ovf_flag[tk.d], 1) == 0) {
        const int pos = atomicAdd(&ovf_list[0], 1);
        ovf_list[1 + pos] = d.v;
      }
      return;
    }
  }
  if (wv == 0) {  // append the bucket's top-L entries >= tau
    const double tau = hub_tau(d, tau_b, tk.d, tau_hot, factor);
    const int n = L.misc[M_PLEN];
    int cnt = 0;
    for (int i = l; i < n; i += WAVE) cnt += L.pv[i] >= tau;
    cnt = wave_sum(cnt);
    if (cnt == 0) return;
    int at = 0;
    if (l == 0) at = (int)atomicAdd(&pt_cnt[tk.d], (uint32_t)cnt);
    at = __builtin_amdgcn_readlane(at, 0);
    int pos0 = 0;
    for (int i0 = 0; i0 < n; i0 += WAVE) {
      const int i = i0 + l;
      const bool keep = i < n && L.pv[i] >= tau;
      const uint64_t m = __ballot(keep);
      if (keep) {
        const int64_t q = d.pt_off + at + pos0 + __popcll(m & lanemask_lt());
        pt_key[q] = L.pk[i];
        pt_sc[q] = L.pv[i];
      }
      pos0 += __popcll(m);
    }
  }
}

// persistent grid over the spill list of k_hub_bucket_w (its length is read on the device, so
// the host never waits for it); a bucket that overflows here too flags its source for the
// HBM-table path (ovf_flag[d], source id appended to ovf_list[1..], count in ovf_list[0])
__global__ void __launch_bounds__(WG_THREADS) k_hub_bucket(DevSlab s, IterArgs a,
                                                           const DevGraph g, HotSet H, const HubDesc* desc,
                                                           const HubTask* tasks, const uint32_t* ntasks_p,
                                                           const int32_t* cm, const uint32_t* staged,
                                                           const HubRec* st,
                                                           int32_t* pt_key, double* pt_sc, uint32_t* pt_cnt,
                                                           const unsigned long long* tau_b,
                                                           const unsigned long long* tau_hot, int Lp,
                                                           int32_t* ovf_flag, int32_t* ovf_list) {
  const uint32_t ntasks = *ntasks_p;
  for (uint32_t task = blockIdx.x; task < ntasks; task += gridDim.x) {
    __syncthreads();  // LDS of the previous task fully consumed
    hub_bucket_one(s, a, g, H, desc, tasks[task], cm, staged, st, pt_key, pt_sc, pt_cnt, tau_b, tau_hot, Lp,
                   ovf_flag, ovf_list);
  }
}
// Long appended lists (a hub with thousands of buckets) are cut before k_hub_final: one
// workgroup per HUB_SLICE entries keeps the slice's top-L (the top-L of a union lies in the union
// of its parts' top-Ls); every full slice then contributes exactly L entries at red + slice * L.
__global__ void __launch_bounds__(WG_THREADS) k_hub_reduce(DevSlab s, const HubDesc* desc, const HubTask* tasks,
                                                           const uint32_t* pt_cnt, const int32_t* pt_key,
                                                           const double* pt_sc, int32_t* red_key, double* red_sc,
                                                           int Lp, int slice, int pl) {
  extern __shared__ __align__(16) unsigned char smem[];
  const HubTask tk = tasks[blockIdx.x];
  const HubDesc d = desc[tk.d];
  // pl > 0: the slice is staged in LDS once (pk / pv of pl entries), so the radix passes of the
  // select and the output pass read LDS instead of re-reading the list from L2 / HBM
  const WgLds L = wg_carve(smem, 0, Lp, pl);
  const int Lw = s.L;
  const int n_all = (int)pt_cnt[tk.d];
  if (n_all <= 2 * slice) return;  // short list: k_hub_final selects from it directly
  const int b = tk.x * slice;
  if (b >= n_all) return;          // slices are reserved for the worst case P * L
  const int n = min(slice, n_all - b);
  const int32_t* pk = pt_key + d.pt_off + b;
  const double* pv = pt_sc + d.pt_off + b;
  int32_t* ok = red_key + d.red + (int64_t)tk.x * Lw;
  double* os = red_sc + d.red + (int64_t)tk.x * Lw;
  if (n <= Lw) {
    for (int i = threadIdx.x; i < n; i += WG_THREADS) { ok[i] = pk[i]; os[i] = pv[i]; }
    return;
  }
  if (threadIdx.x == 0) L.misc[M_PLEN] = 0;
  const bool staged = n <= pl;
  if (staged)
    for (int i = threadIdx.x; i < n; i += WG_THREADS) { L.pk[i] = pk[i]; L.pv[i] = pv[i]; }
  __syncthreads();
  const int32_t* ck = staged ? L.pk : pk;
  const double* cv = staged ? L.pv : pv;
  const uint32_t ts = tie_salt(d.v);
  const SelCrit c = wg_select_top(L, n, Lw, [&](int i) { return ck[i]; }, [&](int i) { return cv[i]; },
                                  [&](int) { return true; }, ts);
  for (int i = threadIdx.x; i < n; i += WG_THREADS) {
    if (sel_test(c, dbits(cv[i]), tie_w(ck[i], ts))) {
      const int pos = atomicAdd(&L.misc[M_PLEN], 1);
      ok[pos] = ck[i];
      os[pos] = cv[i];
    }
  }
}

// top-L by (score desc, tie_w desc) of `total` entries (keyat / valat) into L.rv / L.rk, in no
// particular order; returns their count (every thread of the workgroup)
template <class KeyAt, class ValAt>
__device__ __forceinline__ int hub_select_lds(const WgLds& L, int total, int Lw, KeyAt keyat, ValAt valat,
                                              uint32_t ts) {
  auto occ = [&](int) { return true; };
  if (threadIdx.x == 0) L.misc[M_PLEN] = 0;
  __syncthreads();
  if (total <= Lw) {
    for (int i = threadIdx.x; i < total; i += WG_THREADS) {
      const int pos = atomicAdd(&L.misc[M_PLEN], 1);
      L.rv[pos] = dbits(valat(i));
      L.rk[pos] = keyat(i);
    }
  } else {
    const SelCrit c = wg_select_top(L, total, Lw, keyat, valat, occ, ts);
    for (int i = threadIdx.x; i < total; i += WG_THREADS) {
      const double x = valat(i);
      const int k = keyat(i);
      if (sel_test(c, dbits(x), tie_w(k, ts))) {
        const int pos = atomicAdd(&L.misc[M_PLEN], 1);
        L.rv[pos] = dbits(x);
        L.rk[pos] = k;
      }
    }
  }
  __syncthreads();
  return L.misc[M_PLEN];
}

// One workgroup per source of the batch: top-L of the appended bucket results. Without a hot
// pass that is the source's new row (written, norm1 folded into maxDiff). With one (d.hot >= 0)
// it is only the cold half: it goes to cold list d.hot (count ~0u when a bucket overflowed and
// the HBM-table path redoes the source), and k_hub_join unites it with the hot list.
__global__ void __launch_bounds__(WG_THREADS) k_hub_final(DevSlab s, IterArgs a, const HubDesc* desc,
                                                          const int32_t* ovf_flag, const uint32_t* pt_cnt,
                                                          const int32_t* pt_key, const double* pt_sc,
                                                          const int32_t* red_key, const double* red_sc, int slice,
                                                          uint32_t* cold_cnt, int32_t* cold_key, double* cold_sc,
                                                          int Lp, unsigned long long* maxdiff,
                                                          unsigned long long* stats, int32_t* rsp, int32_t d0) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int di = (int)blockIdx.x;
  const HubDesc d = desc[di];
  if (ovf_flag[di]) {  // a bucket overflowed every LDS table: the HBM-table path redoes the source
    if (d.hot >= 0 && threadIdx.x == 0) cold_cnt[d.hot] = ~0u;
    return;
  }
  const WgLds L = wg_carve(smem, 0, Lp, 0);
  const int Lw = s.L;
  int n = (int)pt_cnt[di];  // appended bucket results, any order
  if (a.diag && threadIdx.x == 0) {  // appended entries per source (vs L)
    diag_add(a.diag, 170, 1ull);
    diag_add(a.diag, 171, (unsigned long long)n);
    diag_add(a.diag, 192 + (31 - __clz(n | 1)), 1ull);
  }
  const int32_t* pk = pt_key + d.pt_off;
  const double* pv = pt_sc + d.pt_off;
  if (n > 2 * slice) {  // the list was cut to the top-L of every HUB_SLICE entries by k_hub_reduce
    const int ns = (n + slice - 1) / slice, last = n - (ns - 1) * slice;
    n = (ns - 1) * Lw + (last < Lw ? last : Lw);
    pk = red_key + d.red;
    pv = red_sc + d.red;
  }
  const int cnt = hub_select_lds(L, n, Lw, [&](int i) { return pk[i]; }, [&](int i) { return pv[i]; },
                                 tie_salt(d.v));
  const double ts = spec_tau(s, a, d.v);
  if (ts > 0.0) {
    // speculation verified: L selected entries, every one at or above the speculative bound (then
    // no key left unemitted can reach the top-L); otherwise the row is not written here
    // (an LDS flag, not __syncthreads_or: that one declares static LDS, and this kernel's launch
    // attribute already claims all 160 KB as dynamic LDS)
    if (threadIdx.x == 0) L.misc[M_SPEC] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < cnt; i += WG_THREADS)
      if (bitsd(L.rv[i]) < ts) L.misc[M_SPEC] = 1;
    __syncthreads();
    const bool fail = L.misc[M_SPEC] != 0 || cnt < Lw;
    if (a.diag && threadIdx.x == 0) {
      diag_add(a.diag, 180, 1ull);
      if (fail) {
        diag_add(a.diag, 181, 1ull);
        if (a.iter >= 0 && a.iter < 32) diag_add(a.diag, 224 + a.iter, 1ull);
      }
    }
    if (fail) {  // not proven: the source is redone with the rigorous bound (run_hubs, its descriptor index)
      if (threadIdx.x == 0) rsp[1 + atomicAdd(&rsp[0], 1)] = d0 + di;
      return;
    }
  }
  if (d.hot >= 0) {
    int32_t* ok = cold_key + (int64_t)d.hot * Lw;
    double* os = cold_sc + (int64_t)d.hot * Lw;
    for (int i = threadIdx.x; i < cnt; i += WG_THREADS) { ok[i] = L.rk[i]; os[i] = bitsd(L.rv[i]); }
    if (threadIdx.x == 0) cold_cnt[d.hot] = (uint32_t)cnt;
    return;
  }
  if ((threadIdx.x >> 6) == 0) {
    const uint64_t* rv = L.rv;
    const int* rk = L.rk;
    // rows already hold the final set: finish_source with U <= L only sorts/writes/norm1
    finish_source(d.v, cnt, [&](int i) { return rk[i]; }, [&](int i) { return bitsd(rv[i]); }, s, a,
                  L.hist, L.rv, L.rk, Lp, L.hk, L.hv, L.mf, maxdiff, stats);
  }
}

}  // namespace pprk
