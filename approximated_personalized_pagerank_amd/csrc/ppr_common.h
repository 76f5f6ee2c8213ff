// ppr_common.h -- device-side types shared by every merge kernel, and the per-source epilogue.
//
// HBM layout (DESIGN.md "data layout"):
//   rp   int64 [n+1]        CSR row pointers (dense ids = graph iteration order)
//   colx int32 [m]          successor id | partition-of-successor << 31
//   ids  int32 [2][n][L]    basket slab, two slots per node (ping-pong per partition)
//   sc   f64   [2][n][L]
//   len  int32 [2][n]
// A node of partition p has been updated upd(p,it) = p ? it/2 : (it+1)/2 times before
// iteration `it`; its current basket lives in slot upd & 1 and an active node writes slot upd^1,
// so the inactive partition's carry-over (include/grank.h:133-134) costs nothing.
#pragma once
#include <hip/hip_runtime.h>

#include "ppr_device.h"

namespace pprk {
using namespace pprd;

constexpr int NT = 4;                 // single-wave LDS table tiers (256 << t slots)
constexpr int TIER_WG = NT;           // workgroup tier (k_merge_wg)
constexpr int TIER_BIG = NT + 1;      // hub pipeline
constexpr int NLISTS = NT + 2;
constexpr int MAX_L = 4096;           // widest basket the kernels accept
constexpr int WAVES_PER_BLOCK = 4;
constexpr int PPR_NSTATS = 8;         // device counters: candidates, algorithmic bytes, wave-tier bytes
// PPR_DIAG counters (u64, printed at plan destruction, plan.h): PPR_DIAG_BASE counters, plus as
// many per shard -- per-wave counters go to a shard picked by block and wave, so hundreds of
// millions of waves do not serialise on a few addresses (that contention distorted the timings)
constexpr int PPR_DIAG_BASE = 304;  // (256..279: the sieve's size classes, merge_sv.h; 288..296: one-shot bucket phases)
constexpr int PPR_DIAG_SHARDS = 256;
constexpr int PPR_DIAG_SLOTS = PPR_DIAG_BASE * (1 + PPR_DIAG_SHARDS);
__device__ __forceinline__ void diag_add(unsigned long long* d, int idx, unsigned long long v) {
  const uint32_t sh = (blockIdx.x * 7u + (threadIdx.x >> 6)) & (uint32_t)(PPR_DIAG_SHARDS - 1);
  atomicAdd(&d[(size_t)PPR_DIAG_BASE * (1 + sh) + idx], v);
}

// one source of the HBM-table path (k_merge_glb)
struct GlbWork {
  int32_t v;
  int32_t pad;
  int64_t off;   // slot offset into the scratch arrays
  int64_t T;     // table slots (power of two)
};

// XCD-aware block remap (cdna_hip_programming.md T1): blocks with the same blockIdx % 8 share
// an XCD (and its L2); give each such group a contiguous range of logical blocks, so neighbouring
// work (adjacent tiles, adjacent output lines) lands in one L2. Bijective for any grid size.
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// one batch of the hub pipeline (host planning): descriptor range and the batch's totals
// (ntiles_s / maxP_s: the tiles of the batch's small-partition sources, listed first, which count
// and scatter launch separately with LDS for maxP_s counters -- see run_hubs)
struct HubBatch {
  size_t d0, d1; int64_t cm, stg, pt, ntiles, nbuck, nrt, red, nseg; int maxP; int64_t nrange = 0;
  int64_t ntiles_s = 0; int maxP_s = 1;
};

struct DevGraph {
  const int64_t* rp;
  const int32_t* colx;
  int64_t n;
};

// Basket rows are stored in ascending hash_b(key) order, with a 64-entry range index per row:
// rix[r] = number of entries whose key lies in hash range <= r (range = top 6 bits of hash_b),
// so the entries of any hash-prefix bucket form one contiguous segment of every row (the
// segmented hub merge reads them without a partition pass), and rmin = the row's smallest score
// (the hubs' top-L pruning bound).
constexpr int NRANGE = 64;
constexpr int RANGE_BITS = 6;
__device__ __forceinline__ uint32_t row_range(int key) { return hash_b((uint32_t)key) >> (32 - RANGE_BITS); }

// Stored ids: once a run has built its hot set (merge_hot.h), a hot key is stored as
// HOT_TAG | its dense hot index and every other key as itself (ids are < 2^31), so a reader of a
// row tells hot from cold -- and gets a hot key's accumulator index -- without a lookup.
// Every reader that needs the key itself decodes through DevSlab::key.
constexpr uint32_t HOT_TAG = 0x80000000u;

struct DevSlab {
  int32_t* ids;
  double* sc;
  int32_t* len;
  int64_t n;
  int32_t L;
  uint16_t* rix;   // [2][n][NRANGE]
  double* rmin;    // [2][n]
  // hot-key encoding of stored ids (hn = 0: ids are stored as is)
  const uint32_t* hbits;  // [ceil(n / 32)] membership
  const uint16_t* hidx;   // [n] dense hot index
  const int32_t* hkeys;   // [hn] key of each hot index
  int hn;
  __device__ __forceinline__ int64_t row(int slot, int64_t u) const { return ((int64_t)slot * n + u) * L; }
  __device__ __forceinline__ int64_t lrow(int slot, int64_t u) const { return (int64_t)slot * n + u; }
  __device__ __forceinline__ int64_t xrow(int slot, int64_t u) const { return ((int64_t)slot * n + u) * NRANGE; }
  // stored id -> key
  __device__ __forceinline__ int key(int32_t id) const { return id >= 0 ? id : hkeys[(uint32_t)id & 0x7fffffffu]; }
  // decode for a kernel compiled for one encoding (HK = the rows may hold hot ids, plan hot_n > 0).
  // Without hot ids no load is emitted: the decode's conditional load (never taken) otherwise costs
  // an s_waitcnt vmcnt(0) per candidate group after it, which drains the walk's prefetched batch
  template <bool HK>
  __device__ __forceinline__ int keyd(int32_t id) const { return HK ? key(id) : id; }
  // key -> stored id
  __device__ __forceinline__ int32_t enc(int key) const {
    if (hn && ((hbits[(uint32_t)key >> 5] >> ((uint32_t)key & 31u)) & 1u)) return (int32_t)(HOT_TAG | hidx[key]);
    return key;
  }
};

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int o = 32; o; o >>= 1) { const uint64_t y = (uint64_t)__shfl_xor((unsigned long long)x, o); x = y < x ? y : x; }
  return x;
}

// Store a finished row of cnt entries held in LDS (rv = score bits, rk = ids) into slot `slot` of
// node v: sorted in place by hash_b(key), scores multiplied by `scale` when `scaled` (MC), plus
// the range index and the row minimum. One wave.
__device__ __forceinline__ void write_row(const DevSlab& s, int slot, int v, uint64_t* rv, int* rk, int cnt,
                                          int Lp, bool scaled, double scale) {
  row_sort_hash(rv, rk, cnt, Lp);
  const int64_t r = s.row(slot, v);
  uint64_t mn = ~0ull;
  for (int i = lane_id(); i < cnt; i += WAVE) {
    double x = bitsd(rv[i]);
    if (scaled) x *= scale;
    s.ids[r + i] = s.enc(rk[i]);
    s.sc[r + i] = x;
    const uint64_t b = dbits(x);
    mn = b < mn ? b : mn;
  }
  mn = wave_min_u64(mn);
  // lane q: entries with range <= q (ranges ascend along the sorted row)
  const uint32_t q = (uint32_t)lane_id();
  int pos = 0;
  for (int b = Lp; b; b >>= 1)
    if (pos + b <= cnt && row_range(rk[pos + b - 1]) <= q) pos += b;
  s.rix[s.xrow(slot, v) + q] = (uint16_t)pos;
  if (lane_id() == 0) {
    s.len[s.lrow(slot, v)] = cnt;
    s.rmin[s.lrow(slot, v)] = cnt ? bitsd(mn) : 0.0;
  }
  wave_fence();
}

constexpr int XS_F = 93;     // fraction bits of the exact sums (merge_xs.h; oracle/grank_oracle.c XS_F)
constexpr int XS_F_MC = 72;  // ... in the MC combine (IterArgs::xsf): its totals reach deg / d (the seed
                             // 1/f and up to deg successor baskets of scores <= 1), < 2^22 at RMAT-22,
                             // so 72 fraction bits keep every total below 2^94 (oracle/mc_oracle.c)

struct IterArgs {
  int sA, sB;        // read slot of successors whose colx bit 31 is 0 / 1
  int active;        // partition updated in this iteration (-1 = init)
  double damping;
  uint32_t unit;     // init mode: every successor contributes {u: 1.0}
  uint32_t stats;
  uint32_t mc;       // MCCompletePathV2 combine (include/mccompletepathv2.h:211-249)
  const int64_t* rp; // row pointers (out-degree of the source in the epilogue)
  unsigned long long* diag;  // PPR_DIAG: per-kernel histograms (nullptr = off)
  uint32_t lds_rank;         // LDS atomics return same-address lanes in lane order (probed per plan)
  uint32_t nt;               // PPR_NT: 1 = basket-row gathers of the candidate walks, 2 = staged-record
                             // reads of the bucket waves, as non-temporal loads (streamed once: they
                             // should not evict the scatter's partially written staging lines from L2)
  uint32_t whatif;           // PPR_WHATIF bits that act inside kernels (timing experiments, plan.h;
                             // bits 0-15 as set by the user, WI_* below set per launch by the host)
  uint32_t xs;               // exact-sum merge (merge_xs.h): GRank by default, the MC combine with PPR_MC_SUM=exact
  int xsf;                   // its fixed-point fraction bits (merge_xs.h XS_F, XS_F_MC)
  int iter;                  // GRank iteration (diagnostics)
  double spec;               // speculative pruning ratio (PPR_SPEC; 0 = off): spec_tau below
};

// per-launch timing variants of one repeated scatter pass (PPR_WHATIF 256/4096/8192/16384/32768
// with 8, plan.h): never set from the environment, so the real pass can not inherit them
constexpr uint32_t WI_SCAT_COALESCED = 1u << 20, WI_SCAT_NOSTORE = 1u << 21, WI_SCAT_NOSCORE = 1u << 22,
                   WI_SCAT_COUNT = 1u << 23, WI_SCAT_WALK = 1u << 24;
// the sieve's exact pass-2 skip turned off (PPR_SV_P2SKIP=0, tests: the skip must not change a bit)
constexpr uint32_t WI_SV_NO_P2SKIP = 1u << 25;
// (tests, PPR_TEST_RANK_PERMUTE=1) the ordered paths take their same-address LDS atomics odd lanes
// first, then even lanes: the occurrence order a device without lane-ordered atomics could return.
// The results must not change (ppr_device.h chunk_accumulate, merge_hub.h bucket_oneshot verify the
// order they got and fall back to stream order).
constexpr uint32_t WI_RANK_PERMUTE = 1u << 26;

// Speculative top-L pruning bound of a hub source (GRank iterations): spec x the smallest score of
// the source's previous row when that row was full. Bucket waves then emit only keys whose exact
// total reaches it; k_hub_final verifies the speculation (L emitted keys at or above it make it a
// true lower bound of the L-th largest total, so the top-L is among them) and flags the source
// for a redo with the rigorous bound otherwise.

template <class T>
__device__ __forceinline__ T ld_nt(const T* p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }

__device__ __forceinline__ int read_slot(const IterArgs& a, int32_t cx) { return (cx < 0) ? a.sB : a.sA; }

__device__ __forceinline__ double spec_tau(const DevSlab& s, const IterArgs& a, int v) {
  if (a.spec <= 0.0 || a.unit || a.mc) return 0.0;
  const int64_t r = s.lrow((a.active == 1) ? a.sB : a.sA, v);
  return s.len[r] == s.L ? a.spec * s.rmin[r] : 0.0;
}

// The hot key set (merge_hot.h): up to a few thousand keys that sit in most successor baskets of
// the hub sources. A hub's hot keys are accumulated densely by k_hub_hot, its other ("cold") keys
// go through the staged partition. Membership changes only which engine sums a key, never the
// result: both keep every key's contributions in successor order.
struct HotSet {
  const uint32_t* bits;   // [ceil(n / 32)] membership bitmap (512 KB at RMAT-22: L2-resident)
  const uint16_t* idx;    // [n] dense index of a member (undefined for other keys)
  const int32_t* keys;    // [members] key of each index
  int n;                  // members; 0 = no hot pass
  __device__ __forceinline__ bool has(int key) const {
    return n != 0 && ((bits[(uint32_t)key >> 5] >> ((uint32_t)key & 31u)) & 1u);
  }
};

// Per-source constants of the two combines (deg > 0 for every merged source):
//   GRank  acc = {v: 1-d};      acc[k] = fma(s, d/deg, acc[k]);      row = topL(acc)
//          (include/grank.h:103-116)
//   MC     acc = {v: 1/(d/deg)}; acc[k] = acc[k] + s (== fma(s, 1, acc[k]));
//          row = topL(acc) * (d/deg)   (include/mccompletepathv2.h:214-247)
__device__ __forceinline__ double merge_factor(const IterArgs& a, int64_t deg) {
  return a.mc ? 1.0 : a.damping / (double)deg;
}
__device__ __forceinline__ double self_seed(const IterArgs& a, int64_t deg) {
  return a.mc ? 1.0 / (a.damping / (double)deg) : 1.0 - a.damping;
}
// slot an active source writes: GRank ping-pongs per partition, MC writes its final basket to
// slot 0 (slot 1 holds the random-walk baskets)
__device__ __forceinline__ int write_slot(const IterArgs& a) {
  return a.mc ? 0 : (((a.active == 1) ? a.sB : a.sA) ^ 1);
}

// Epilogue of one source, run by ONE wave: select the top-L of U candidates (keys/vals in LDS
// or HBM), sort the row, write it to the next slot, norm1 against the old row, fold maxDiff.
// (PPR_DIAG, dg >= 0: lane 0 adds its cycles of select / row write / norm1 to slots dg .. dg + 2)
__device__ __forceinline__ void fs_lap(const IterArgs& a, int dg, int k, long long& t) {
  if (dg < 0 || !a.diag || lane_id() != 0) return;
  const long long now = (long long)clock64();
  diag_add(a.diag, dg + k, (unsigned long long)(now - t));
  t = now;
}
// Register epilogue of a GRank row of cnt <= 128 entries (Lp <= 128): lane l holds the new
// entries l and l + 64 (k0/v0, k1/v1, candidate order) and the old row's entries l and l + 64
// (o0/os0, o1/os1, stored order, loaded before the select). hash_b is a bijection, so an entry's
// place in the stored order is its rank -- the number of entries with a smaller hash -- counted
// against every other entry's hash read with v_readlane (no sort network, no LDS round trips); the
// range index is a 64-bin count and a wave scan. The row is stored straight from the ranks. norm1 keeps
// oracle/grank_oracle.c:norm1_rows' lane pattern exactly: lane l adds |new - old| of the stored
// positions l then l + 64 (the d values are permuted into stored order through LDS), then the
// unmatched old entries l then l + 64, then the xor butterfly. LDS: hk/hv (2 Lp), mf (Lp), rv
// (old scores by position, Lp), hist (d by position: <= 128 doubles = its 1 KB).
__device__ __forceinline__ double finish_row_reg(const DevSlab& s, int nxt, int v, int cnt, int k0, uint64_t v0,
                                                 int k1, uint64_t v1, int o0, double os0, int o1, double os1,
                                                 int olen, uint64_t* rv, uint32_t* hist, int* hk, int* hv, int* mf,
                                                 int Lp, const IterArgs& a, int dg, long long& tl) {
  const int l = lane_id();
  const bool e0 = l < cnt, e1 = l + WAVE < cnt;
  const uint32_t h0 = hash_b((uint32_t)k0), h1 = hash_b((uint32_t)k1);
  // range index: entries per hash range (LDS counts), inclusive scan over the 64 lanes
  hist[l] = 0u;
  wave_fence();
  if (e0) atomicAdd(&hist[h0 >> (32 - RANGE_BITS)], 1u);
  if (e1) atomicAdd(&hist[h1 >> (32 - RANGE_BITS)], 1u);
  wave_fence();
  const int rx = wave_incl_scan((int)hist[l]);
  int r0 = 0, r1 = 0;
  // (cnt is wave-uniform: scalar loops; entries past cnt hash EMPTY's value and are counted out
  // by the trip counts, 4 lanes per trip so the compares interleave)
  const int n0 = cnt < WAVE ? cnt : WAVE;
  auto cmp4 = [&](uint32_t hv, int i) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t sh = (uint32_t)__builtin_amdgcn_readlane((int)hv, i + u);
      r0 += sh < h0;
      r1 += sh < h1;
    }
  };
  auto cmp1 = [&](uint32_t hv, int i) {
    const uint32_t sh = (uint32_t)__builtin_amdgcn_readlane((int)hv, i);
    r0 += sh < h0;
    r1 += sh < h1;
  };
  int i = 0;
  for (; i + 4 <= n0; i += 4) cmp4(h0, i);
  for (; i < n0; i++) cmp1(h0, i);
  const int n1 = cnt - WAVE;
  for (i = 0; i + 4 <= n1; i += 4) cmp4(h1, i);
  for (; i < n1; i++) cmp1(h1, i);
  const int64_t r = s.row(nxt, v);
  uint64_t mn = ~0ull;
  if (e0) { s.ids[r + r0] = s.enc(k0); s.sc[r + r0] = bitsd(v0); mn = v0; }
  if (e1) { s.ids[r + r1] = s.enc(k1); s.sc[r + r1] = bitsd(v1); mn = v1 < mn ? v1 : mn; }
  mn = wave_min_u64(mn);
  s.rix[s.xrow(nxt, v) + l] = (uint16_t)rx;
  if (l == 0) {
    s.len[s.lrow(nxt, v)] = cnt;
    s.rmin[s.lrow(nxt, v)] = cnt ? bitsd(mn) : 0.0;
  }
  fs_lap(a, dg, 1, tl);
  // norm1: LDS hash of the old keys (positions j, scores rv[j]), probed by the new keys
  const int hsize = 2 * Lp;
  const uint32_t hmask = (uint32_t)hsize - 1;
  for (int i = l; i < hsize; i += WAVE) hk[i] = EMPTY;
  const bool f0 = l < olen, f1 = l + WAVE < olen;
  if (f0) { mf[l] = 0; rv[l] = dbits(os0); }
  if (f1) { mf[l + WAVE] = 0; rv[l + WAVE] = dbits(os1); }
  wave_fence();
#pragma unroll
  for (int q = 0; q < 2; q++) {
    if (!(q ? f1 : f0)) continue;
    const int key = q ? o1 : o0;
    uint32_t h = hash32((uint32_t)key) & hmask;
    for (int c = 0; c < hsize; c++) {  // 2 Lp slots hold at most L keys: never full
      const int prev = atomicCAS(&hk[h], EMPTY, key);
      if (prev == EMPTY) { hv[h] = l + q * WAVE; break; }
      h = (h + 1) & hmask;
    }
  }
  wave_fence();
  double* dd = reinterpret_cast<double*>(hist);
#pragma unroll
  for (int q = 0; q < 2; q++) {
    if (!(q ? e1 : e0)) continue;
    const int key = q ? k1 : k0;
    uint32_t h = hash32((uint32_t)key) & hmask;
    double o = 0.0;
    for (int c = 0; c < hsize; c++) {
      const int cur = hk[h];
      if (cur == key) { const int j = hv[h]; o = bitsd(rv[j]); mf[j] = 1; break; }
      if (cur == EMPTY) break;
      h = (h + 1) & hmask;
    }
    dd[q ? r1 : r0] = fabs(bitsd(q ? v1 : v0) - o);
  }
  wave_fence();
  double p = 0.0;
  if (e0) p += dd[l];
  if (e1) p += dd[l + WAVE];
  if (f0 && !mf[l]) p += os0;
  if (f1 && !mf[l + WAVE]) p += os1;
#pragma unroll
  for (int o = 32; o; o >>= 1) p = p + __shfl_xor(p, o);
  wave_fence();
  return p;
}

template <class KeyAt, class ValAt>
__device__ __forceinline__ void finish_source(int v, int U, KeyAt keyat, ValAt valat,
                                              const DevSlab& s, const IterArgs& a, uint32_t* hist,
                                              uint64_t* rv, int* rk, int Lp, int* hk, int* hv,
                                              int* mf, unsigned long long* maxdiff,
                                              unsigned long long* stats, int dg = -1) {
  const int L = s.L;
  U = __builtin_amdgcn_readfirstlane(U);  // (wave-uniform: scalar loop bounds below)
  long long tl = (dg >= 0 && a.diag) ? (long long)clock64() : 0;
  // GRank rows of <= 128 entries take the register epilogue: the old row is loaded here, ahead of
  // the select, whose work hides its latency (all L entries of the row, masked by its length later)
  const bool reg = Lp <= 2 * WAVE && !a.unit && !a.mc;
  const int cur = (a.active == 1) ? a.sB : a.sA;
  int o0 = EMPTY, o1 = EMPTY, olen = 0;
  double os0 = 0.0, os1 = 0.0;
  if (reg) {
    const int64_t ro = s.row(cur, v);
    const int l = lane_id();
    olen = __builtin_amdgcn_readfirstlane(s.len[s.lrow(cur, v)]);
    if (l < L) { o0 = s.ids[ro + l]; os0 = s.sc[ro + l]; }
    if (l + WAVE < L) { o1 = s.ids[ro + l + WAVE]; os1 = s.sc[ro + l + WAVE]; }
  }
  int cnt;
  if (U <= L) {
    for (int i = lane_id(); i < U; i += WAVE) { rv[i] = dbits(valat(i)); rk[i] = keyat(i); }
    cnt = U;
  } else {
    const uint32_t ts = tie_salt(v);
    const SelCrit c = select_top(U, L, keyat, valat, hist, ts);
    int base = 0;
    for (int i0 = 0; i0 < U; i0 += WAVE) {
      const int i = i0 + lane_id();
      bool sel = false;
      uint64_t vb = 0;
      int key = 0;
      if (i < U) { key = keyat(i); vb = dbits(valat(i)); sel = sel_test(c, vb, tie_w(key, ts)); }
      const uint64_t m = __ballot(sel);
      if (sel) { const int pos = base + __popcll(m & lanemask_lt()); rv[pos] = vb; rk[pos] = key; }
      base += __popcll(m);
    }
    cnt = L;
  }
  wave_fence();
  if (a.unit) {
    // init writes both slots: a dangling source never updates, so its basket must be valid in
    // whichever slot its partition reads
    write_row(s, 0, v, rv, rk, cnt, Lp, false, 1.0);
    write_row(s, 1, v, rv, rk, cnt, Lp, false, 1.0);
    return;
  }
  if (a.mc) {
    // keepTop(L) first, then `*= factor` (include/mccompletepathv2.h:243-247)
    const double f = a.damping / (double)(a.rp[v + 1] - a.rp[v]);
    write_row(s, 0, v, rv, rk, cnt, Lp, true, f);
    return;
  }
  const int nxt = cur ^ 1;
  fs_lap(a, dg, 0, tl);
  double d1;
  if (reg) {
    const int l = lane_id();
    const int k0 = l < cnt ? rk[l] : EMPTY, k1 = l + WAVE < cnt ? rk[l + WAVE] : EMPTY;
    const uint64_t v0 = l < cnt ? rv[l] : 0ull, v1 = l + WAVE < cnt ? rv[l + WAVE] : 0ull;
    wave_fence();
    d1 = finish_row_reg(s, nxt, v, cnt, k0, v0, k1, v1, l < olen ? s.key(o0) : EMPTY, os0,
                        l + WAVE < olen ? s.key(o1) : EMPTY, os1, olen, rv, hist, hk, hv, mf, Lp, a, dg, tl);
  } else {
    // rv/rk are left in the stored (hash) order: norm1 walks the new row in that order
    write_row(s, nxt, v, rv, rk, cnt, Lp, false, 1.0);
    fs_lap(a, dg, 1, tl);
    const int64_t ro = s.row(cur, v);
    const int olen2 = s.len[s.lrow(cur, v)];
    d1 = row_norm1(rv, rk, cnt, s.ids + ro, s.sc + ro, olen2, hk, hv, mf, 2 * Lp,
                   [&](int32_t id) { return s.key(id); });
  }
  fs_lap(a, dg, 2, tl);
  if (lane_id() == 0) {
    // maxDiff only grows: skip the contended atomic when a larger value is already published
    const unsigned long long b = (unsigned long long)dbits(d1);
    if (b > __hip_atomic_load(maxdiff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(maxdiff, b);
    if (a.diag) {  // PPR_DIAG: merged rows, and rows left bit-identical (norm1 = 0)
      atomicAdd(&a.diag[150], 1ull);
      if (d1 == 0.0) atomicAdd(&a.diag[151], 1ull);
    }
  }
  (void)stats;  // written-row bytes are summed by k_stat_written (no per-source atomics)
}

}  // namespace pprk
