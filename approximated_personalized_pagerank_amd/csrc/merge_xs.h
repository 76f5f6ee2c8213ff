// merge_xs.h -- the exact-sum basket merge (the plan default for GRank).
//
// Every contribution p = fl(s * d/deg) of a successor basket (and the seed 1-d) is added EXACTLY
// into a fixed-point accumulator of its key, X[k] += floor(p * 2^93) (96 bits: a 64-bit low word
// and a 32-bit high word), and the basket value is X[k] * 2^-93 rounded to nearest once. Integer
// addition is associative, so the order of the adds is free: any lane, wave or workgroup adds
// with LDS atomics, no stable partition, no ordered chains. The result is the exact sum of the
// rounded products rounded once -- at least as accurate as the reference's in-order fma chain
// (include/grank.h:107-116), which it matches to a few ulps -- and the same on every run and every
// GPU count. Restated bit for bit by oracle/grank_oracle.c ("exact" mode). Every basket sums to
// <= 1, so a key's total stays < 4 (X < 2^95: the high word never reaches the key tag above it).
//
//   k_merge_lds_x  one wave per small source (candidates + 1 <= 1536), 16-B LDS slots
//   k_xr           one workgroup per (hub source, key range): walks the source's successor rows,
//                  accumulates the keys of its hash range in a shared LDS table (up to 8192
//                  slots), then either finishes the source (one range) or appends its top-L
//   k_xb           one workgroup per staged bucket of a partitioned hub source (the partition
//                  of merge_hub.h: count, scan, scatter), same table and epilogue as k_xr
//   k_xfinal       one workgroup per listed source: top-L of its ranges' / buckets' lists
#pragma once
#include "merge_hub.h"

namespace pprk {

// (XS_F / XS_F_MC, the fixed-point fraction bits: ppr_common.h)
constexpr double XR_SPEC = 0.9;  // speculative bound of a whole-source table: this x its previous L-th score

// floor(p * 2^F) of p in [0, 2^(95 - F)): lo = low 64 bits, hi = bits 64..94 (F = 93: p < 4)
__device__ __forceinline__ void xs_conv(double p, unsigned long long& lo, uint32_t& hi, int F = XS_F) {
  const unsigned long long b = dbits(p);
  int e = (int)((b >> 52) & 0x7ffu);
  unsigned long long m = b & ((1ull << 52) - 1ull);
  if (e) m |= 1ull << 52; else e = 1;
  const int sh = e - 1075 + F;
  if (sh >= 0) {
    lo = m << sh;
    hi = sh > 11 ? (uint32_t)(m >> (64 - sh)) : 0u;
  } else {
    lo = -sh < 64 ? (m >> -sh) : 0ull;
    hi = 0u;
  }
}

// X * 2^-93 rounded to nearest even: the top 64 bits of X with a sticky bit, one correctly rounded
// u64 -> f64 conversion, an exact power-of-two scale (oracle_xs_to_double)
__device__ __forceinline__ double xs_to_double(uint32_t hi, unsigned long long lo, int F = XS_F) {
  if (hi == 0u) return ldexp((double)lo, -F);
  const int n = 32 - __clz(hi);
  const unsigned long long top = ((unsigned long long)hi << (64 - n)) | (lo >> n);
  const unsigned long long sticky = (lo & ((1ull << n) - 1ull)) != 0ull ? 1ull : 0ull;
  return ldexp((double)(top | sticky), n - F);
}

// value of a single contribution p as the exact path stores it: a lower bound of the total of any
// key that receives p (totals of nonnegative terms only grow, rounding is monotone)
__device__ __forceinline__ double xs_single(double p, int F = XS_F) {
  unsigned long long lo;
  uint32_t hi;
  xs_conv(p, lo, hi, F);
  return xs_to_double(hi, lo, F);
}

// LDS table of 16-B slots in three arrays: keys u32 (key + 1, 0 = empty), lo u64 (low word of the
// sum), hi u32 (high word). Slots are probed in aligned groups of four keys, one ds_read_b128 per
// step: the longest probe among a group's 64 lanes (the wave waits for it) stays short at fills
// where single-slot linear probing ran long chains.
struct XTable {
  uint32_t* keys;
  unsigned long long* lo;
  uint32_t* hi;
  uint32_t mask;
};

// find-or-insert `key`, then add X: the low word's returning add yields its carry, which goes
// with the high word into hi. Returns 1 when this lane inserted the key, 0 when it was there, -1
// when the probe ran out (T/4 groups visited or T/4 insert races lost: the table is full) -- no
// add then, and the caller takes its overflow path. Every caller sizes or budgets its table so
// that this cannot happen; the bound turns a sizing bug into a redone source instead of a hang
// (tests: PPR_WAVE_TDIV, PPR_XR_BUDGET=over force it).
__device__ __forceinline__ int xt_add(const XTable& t, int key, unsigned long long xlo, uint32_t xhi) {
  const uint32_t tag = (uint32_t)key + 1u;
  uint32_t g = hash32((uint32_t)key) & t.mask & ~3u;
  int ins = 0;
  uint32_t h = 0;
  const uint32_t groups = (t.mask + 1u) >> 2;
  uint32_t moves = 0, races = 0;
  for (;;) {
    if (moves >= groups || races > groups) return -1;
    const uint4 q = *reinterpret_cast<const uint4*>(t.keys + g);
    if (q.x == tag) { h = g; break; }
    if (q.y == tag) { h = g + 1; break; }
    if (q.z == tag) { h = g + 2; break; }
    if (q.w == tag) { h = g + 3; break; }
    const int e = q.x == 0u ? 0 : q.y == 0u ? 1 : q.z == 0u ? 2 : q.w == 0u ? 3 : -1;
    if (e >= 0) {
      const uint32_t prev = atomicCAS(&t.keys[g + e], 0u, tag);
      if (prev == 0u) { h = g + e; ins = 1; break; }
      if (prev == tag) { h = g + e; break; }
      races++;
      continue;  // another key took it: read the group again
    }
    g = (g + 4u) & t.mask;
    moves++;
  }
  const unsigned long long old = atomicAdd(&t.lo[h], xlo);
  const uint32_t up = xhi + ((old + xlo < old) ? 1u : 0u);
  if (up) atomicAdd(&t.hi[h], up);
  return ins;
}

// the slot of `key` within a loaded group of four (or -1)
__device__ __forceinline__ int xt_match(const uint4& q, uint32_t g, uint32_t tag) {
  return q.x == tag ? (int)g : q.y == tag ? (int)g + 1 : q.z == tag ? (int)g + 2 : q.w == tag ? (int)g + 3 : -1;
}
// find-or-insert only (xt_add's bounded probe); returns the slot, `ins` when this lane inserted,
// -1 when the table is full
__device__ __forceinline__ int xt_slot(const XTable& t, int key, bool& ins) {
  const uint32_t tag = (uint32_t)key + 1u;
  uint32_t g = hash32((uint32_t)key) & t.mask & ~3u;
  ins = false;
  const uint32_t groups = (t.mask + 1u) >> 2;
  uint32_t moves = 0, races = 0;
  while (moves < groups && races <= groups) {
    const uint4 q = *reinterpret_cast<const uint4*>(t.keys + g);
    const int m = xt_match(q, g, tag);
    if (m >= 0) return m;
    const int e = q.x == 0u ? 0 : q.y == 0u ? 1 : q.z == 0u ? 2 : q.w == 0u ? 3 : -1;
    if (e >= 0) {
      const uint32_t prev = atomicCAS(&t.keys[g + e], 0u, tag);
      if (prev == 0u) { ins = true; return (int)(g + e); }
      if (prev == tag) return (int)(g + e);
      races++;
      continue;
    }
    g = (g + 4u) & t.mask;
    moves++;
  }
  return -1;
}

__host__ __device__ constexpr size_t xt_bytes(int T) { return (size_t)T * 16; }
// carve a T-slot table at p (16-B aligned)
__device__ __forceinline__ XTable xt_carve(unsigned char* p, int T) {
  XTable t;
  t.keys = reinterpret_cast<uint32_t*>(p);
  t.lo = reinterpret_cast<unsigned long long*>(p + (size_t)T * 4);
  t.hi = reinterpret_cast<uint32_t*>(p + (size_t)T * 12);
  t.mask = (uint32_t)T - 1u;
  return t;
}

// ---------------------------------------------------------------------------------------------
// wave tier: layout table (16 T) | hist u32[256] | rv u64[Lp] | rk i32[Lp] | hk i32[2Lp] |
// hv i32[2Lp] | mf i32[Lp]; a split wave (WList) has no row epilogue: table and hist only
__host__ __device__ constexpr size_t lds_wave_bytes_x(int T, int Lp) {
  return (size_t)T * 16 + (size_t)Lp * 12 + 1024 + (size_t)Lp * 20;
}
__host__ __device__ constexpr size_t lds_wave_bytes_xs(int T) { return (size_t)T * 16 + 1024; }

// Split epilogue (round 6, the tiers with the largest tables): the wave stops after the compaction
// and writes its kept entries (at most `cap`, the common case by far: ~150 of them) to a list in
// HBM; k_wfin (below) then selects, writes the row and its norm1 with one 5-KB wave per source. A
// 2048-slot table costs 38 KB of LDS per wave: holding it through the select, the row write and
// norm1 (more than half of the wave's time, PPR_DIAG) kept the tier at 4 waves per CU.
// (WList, wave_emit_list: merge_wave.h)

// (a table that runs out -- never, at T >= 4/3 of the tier's candidate cap, unless PPR_WAVE_TDIV
// shrinks it for the tests -- writes no row: the source goes to `wovl` ([0] count, then sources)
// and the host merges it again with the workgroup engines)
#ifndef PPR_WX_WAVES
#define PPR_WX_WAVES 1  // (A/B: waves per SIMD the compiler sizes the split k_merge_lds_x's registers for)
#endif
template <bool kSplit>
__global__ void __launch_bounds__(256, kSplit ? PPR_WX_WAVES : 1) k_merge_lds_x(DevGraph g, DevSlab s, IterArgs a, const int32_t* list,
                                                     int64_t count, int T, int Lp, unsigned long long* maxdiff,
                                                     unsigned long long* stats, int32_t* dlast, int32_t* wovl,
                                                     WList wl) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w >= count) return;
  unsigned char* base = smem + (size_t)wv * (kSplit ? lds_wave_bytes_xs(T) : lds_wave_bytes_x(T, Lp));
  const XTable t = xt_carve(base, T);
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + (size_t)T * 16);
  uint64_t* rv = reinterpret_cast<uint64_t*>(base + (size_t)T * 16 + 1024);
  int* rk = reinterpret_cast<int*>(base + (size_t)T * 16 + 1024 + (size_t)Lp * 8);
  int* hk = reinterpret_cast<int*>(base + (size_t)T * 16 + 1024 + (size_t)Lp * 12);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;

  const int v = list[w];
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = merge_factor(a, e - b);
  long long tl = a.diag ? (long long)clock64() : 0;  // PPR_DIAG: wave-tier phases, slots 280..287
  for (int i = lane_id(); i < T; i += WAVE) { t.keys[i] = 0u; t.lo[i] = 0ull; t.hi[i] = 0u; }
  wave_fence();
  bool bad = false;
  if (lane_id() == 0) {
    unsigned long long lo;
    uint32_t hi;
    xs_conv(self_seed(a, e - b), lo, hi, a.xsf);
    bad = xt_add(t, v, lo, hi) < 0;
  }
  wave_fence();
  unsigned long long mb = 0;
  if (a.unit) {
    unsigned long long flo;
    uint32_t fhi;
    xs_conv(factor, flo, fhi, a.xsf);  // init: every successor contributes 1.0 * d/deg
    for (int64_t e0 = b; e0 < e; e0 += WAVE) {
      const int64_t i = e0 + lane_id();
      if (i < e && xt_add(t, g.colx[i] & 0x7fffffff, flo, fhi) < 0) bad = true;
    }
  } else {
    for (int64_t e0 = b; e0 < e; e0 += WAVE)
      hub_window_walk(g, s, a, e0, min(e, e0 + WAVE), reinterpret_cast<uint8_t*>(hist),
                      [&](bool valid, int id, double sv, bool) {
                        if (valid) {
                          unsigned long long lo;
                          uint32_t hi;
                          xs_conv(sv * factor, lo, hi, a.xsf);
                          if (xt_add(t, id, lo, hi) < 0) bad = true;
                        }
                      },
                      WalkRowMin{&mb, (int)s.L});
  }
  wave_fence();
  if (__ballot(bad)) {  // table ran out: no row, the host redoes the source
    if (lane_id() == 0) {
      wovl[1 + atomicAdd(&wovl[0], 1)] = v;
      if (kSplit) wl.n[w] = -1;
    }
    return;
  }
  fs_lap(a, 280, 1, tl);  // (slot 281: setup + walk)
#pragma unroll
  for (int o = 32; o; o >>= 1) { const unsigned long long y = __shfl_xor(mb, o); mb = y > mb ? y : mb; }
  // keys below the pruning bound cannot reach the top-L (a full successor row puts L distinct keys
  // at >= the single-contribution value of its minimum)
  const double tau = (!a.unit && mb) ? xs_single(bitsd(mb) * factor, a.xsf) : 0.0;
  // settle + compact in place: (double value, key) pairs over the front of the table
  double* vals = reinterpret_cast<double*>(t.lo);
  int* keys = reinterpret_cast<int*>(t.keys);
  // speculative bound: 0.9 x the source's previous L-th score (a full current row's minimum), kept
  // only when at least L keys reach it -- the top-L then lies among them (exact either way)
  double tspec = 0.0;
  if (!a.unit && !a.mc) {
    const int64_t cr = s.lrow((a.active == 1) ? a.sB : a.sA, v);
    if (s.len[cr] == s.L) tspec = fmax(tau, XR_SPEC * s.rmin[cr]);
  }
  int U = 0, D = 0, Uhi = 0;
  for (int base0 = 0; base0 < T; base0 += WAVE) {
    const int i = base0 + lane_id();
    const uint32_t kt = t.keys[i];
    const unsigned long long lo = t.lo[i];
    const bool occ = kt != 0u;
    const double x = occ ? xs_to_double(t.hi[i], lo, a.xsf) : 0.0;
    const bool keep = occ && x >= tau;
    const uint64_t m = __ballot(keep);
    D += __popcll(__ballot(occ));
    Uhi += __popcll(__ballot(keep && x >= tspec));
    wave_fence();
    if (keep) {
      const int pos = U + __popcll(m & lanemask_lt());
      vals[pos] = x;
      keys[pos] = (int)kt - 1;
    }
    wave_fence();
    U += __popcll(m);
  }
  if (tspec > tau && Uhi >= (int)s.L && Uhi < U) {
    // keep only the entries at or above the speculative bound (in place, order kept)
    int U2 = 0;
    for (int i0 = 0; i0 < U; i0 += WAVE) {
      const int i = i0 + lane_id();
      const double x = i < U ? vals[i] : 0.0;
      const int k = i < U ? keys[i] : 0;
      const bool keep = i < U && x >= tspec;
      const uint64_t m = __ballot(keep);
      wave_fence();
      if (keep) { const int pos = U2 + __popcll(m & lanemask_lt()); vals[pos] = x; keys[pos] = k; }
      wave_fence();
      U2 += __popcll(m);
    }
    U = U2;
  }
  if (dlast && !a.unit && lane_id() == 0) dlast[v] = D;  // (init counts predict nothing)
  fs_lap(a, 280, 2, tl);  // (slot 282: settle + compact)
  if (a.diag && !a.unit && lane_id() == 0) { diag_add(a.diag, 280, 1ull); diag_add(a.diag, 287, (unsigned long long)U); }
  if (kSplit) {  // the list for k_wfin: every kept entry, or the top-L of more than cap (cap >= L)
    wave_emit_list(wl, w, U, keys, vals, v, (int)s.L, hist);
  } else {
    finish_source(v, U, [&](int i) { return keys[i]; }, [&](int i) { return vals[i]; }, s, a, hist, rv, rk, Lp, hk, hv,
                  mf, maxdiff, stats, a.unit ? -1 : 283);  // (283 select, 284 row write, 285 norm1)
  }
}

// the row of a split wave-tier source from its list (one wave per source, 4 per block)
__host__ __device__ constexpr size_t wfin_lds_bytes(int Lp) { return (size_t)Lp * 12 + 1024 + (size_t)Lp * 20; }
__global__ void __launch_bounds__(256) k_wfin(DevSlab s, IterArgs a, const int32_t* list, int64_t count, WList wl,
                                              int Lp, unsigned long long* maxdiff, unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w >= count) return;
  const int n = wl.n[w];
  if (n < 0) return;  // finished by the wave itself, or overflowed
  unsigned char* base = smem + (size_t)wv * wfin_lds_bytes(Lp);
  uint64_t* rv = reinterpret_cast<uint64_t*>(base);
  int* rk = reinterpret_cast<int*>(base + (size_t)Lp * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + (size_t)Lp * 12);
  int* hk = reinterpret_cast<int*>(base + (size_t)Lp * 12 + 1024);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;
  const int64_t o = w * (int64_t)wl.cap;
  const int32_t* lk = wl.k + o;
  const double* lv = wl.v + o;
  finish_source(list[w], n, [&](int i) { return lk[i]; }, [&](int i) { return lv[i]; }, s, a, hist, rv, rk, Lp, hk,
                hv, mf, maxdiff, stats, 283);
}

// ---------------------------------------------------------------------------------------------
// Range / bucket workgroups. LDS: table (16 T) | flags u8[W][HUB_WALK_FLAGS] | hist u32[256] |
// misc i32[64] | rv u64[Lp] | rk i32[Lp] | hk i32[2Lp] | hv i32[2Lp] | mf i32[Lp]
__host__ __device__ constexpr size_t xr_lds_bytes(int T, int W, int Lp) {
  return (size_t)T * 16 + (size_t)W * HUB_WALK_FLAGS + 1024 + 256 + (size_t)Lp * 32;
}

// one hub source merged by workgroups (k_xr / k_xb): the source, its constants and outputs
struct XDesc {
  int32_t v;
  int32_t R;        // key ranges (k_xr; 1 = one workgroup finishes the source), 0 for a k_xb source
  int64_t pt_off;   // appended-entry list (R * L, or P * L entries)
  double factor, selfval;
};

// misc slots (ints; M_BIN..M_HB = 4..6 belong to wg_radix_kth, 8..9 hold k_xr's row-minimum bound)
enum { XM_FILL = 0, XM_OVF = 1, XM_CNT = 2, XM_U = 3, XM_MIN = 10 /* u64: 10..11 */ };

struct XrLds {
  XTable t;
  uint8_t* fl;
  WgLds w;  // hist / misc and the row buffers (the select and finish_source scratch)
};

__device__ __forceinline__ XrLds xr_carve(unsigned char* smem, int T, int W, int Lp) {
  XrLds x;
  unsigned char* p = smem;
  x.t = xt_carve(p, T); p += xt_bytes(T);
  x.fl = p; p += (size_t)W * HUB_WALK_FLAGS;
  x.w = WgLds{};
  x.w.hist = reinterpret_cast<uint32_t*>(p); p += 1024;
  x.w.misc = reinterpret_cast<int*>(p); p += 256;
  x.w.rv = reinterpret_cast<uint64_t*>(p); p += (size_t)Lp * 8;
  x.w.rk = reinterpret_cast<int*>(p); p += (size_t)Lp * 4;
  x.w.hk = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  x.w.hv = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  x.w.mf = reinterpret_cast<int*>(p);
  return x;
}

// PPR_DIAG: cycles since the last lap into counter `slot` (thread 0 only)
__device__ __forceinline__ void xr_lap(const IterArgs& a, int slot, long long& t) {
  if (!a.diag || threadIdx.x != 0) return;
  const long long now = (long long)clock64();
  diag_add(a.diag, slot, (unsigned long long)(now - t));
  t = now;
}

__device__ __forceinline__ void xr_clear(const XrLds& x, int T) {
  for (int i = threadIdx.x; i < T; i += blockDim.x) { x.t.keys[i] = 0u; x.t.lo[i] = 0ull; x.t.hi[i] = 0u; }
  if (threadIdx.x < 64) x.w.misc[threadIdx.x] = 0;
}

// one accumulated contribution of the calling lane (valid lanes only); a group's new keys are
// counted by its wave's lowest lane (the workgroup's distinct-key budget, xr_stop)
// a probe that ran out of slots: the fill count jumps past any budget, so the workgroup stops and
// the source takes the overflow redo
constexpr int XR_FULL = 1 << 24;
__device__ __forceinline__ void xr_apply(const XrLds& x, bool valid, int key, double p, int budget, int F) {
  int r = 0;
  if (valid) {
    unsigned long long lo;
    uint32_t hi;
    xs_conv(p, lo, hi, F);
    r = xt_add(x.t, key, lo, hi);
  }
  const int n = __popcll(__ballot(r > 0)) + (__ballot(r < 0) ? XR_FULL : 0);
  if (n && lane_id() == 0) atomicAdd(&x.w.misc[XM_FILL], n);  // (no return: xr_stop reads the count)
}
// every wave checks the shared count before each group: once it passes the budget no wave starts
// another group, so the table holds at most budget + W * 64 keys (a budget <= T - W * 64 - 1 never
// lets a probe run out of empty slots)
__device__ __forceinline__ bool xr_stop(const XrLds& x, int budget) {
  return __hip_atomic_load(&x.w.misc[XM_FILL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > budget;
}

// Epilogue of one range / bucket workgroup after its last add (every thread):
//   settle  each thread turns its (at most XR_SLOTS) occupied slots into (key, double) pairs and
//           keeps those at or above the pruning bound tau0 (no other key can reach the top-L);
//   compact the kept pairs to a dense array over the front of the table (after a barrier, so no
//           slot is overwritten before it was read);
//   select  top-L of the dense array when it holds more than L (radix select over U entries, not T);
//   emit    the selected pairs -> the source's list; with `publish` (several ranges / buckets per
//           source) the range's L-th value first raises the source's bound xtau[d] and only pairs at
//           or above the current bound are appended.
// The row itself is written by k_xfin1 / k_xfinal from the list.
constexpr int XR_SLOTS = 8;  // table slots per thread (T <= 8 * blockDim: T / W = 512 in every class)
__device__ __forceinline__ void xr_finish(const XrLds& x, int T, const DevSlab& s, const IterArgs& a,
                                          const XDesc& xd, int d, bool publish, double tau0, double tau_spec,
                                          unsigned long long* xtau, int32_t* pk, double* ps, uint32_t* pc,
                                          uint32_t* dsum, long long* tph = nullptr, int slot = 0, int cap = 0) {
  const int L = s.L;
  const int v = xd.v;
  // a list range may already filter by the bound the source's other ranges published
  if (publish) tau0 = fmax(tau0, bitsd(__hip_atomic_load(&xtau[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
  // speculative bound (one-range sources): kept only when at least L keys reach it -- then the
  // top-L lies among them, so the result never depends on it
  const double ts_hi = fmax(tau0, tau_spec);
  int kk[XR_SLOTS];
  double kv[XR_SLOTS];
  int c = 0, c_hi = 0;
  // (all slot reads issued unconditionally and back to back -- a read under `if (key)` waited on
  // its own; an index past T re-reads slot T - 1 and is dropped)
  uint32_t kt[XR_SLOTS], kh[XR_SLOTS];
  unsigned long long kl[XR_SLOTS];
#pragma unroll
  for (int j = 0; j < XR_SLOTS; j++) {
    const int i = min(T - 1, (int)threadIdx.x + j * (int)blockDim.x);
    kt[j] = x.t.keys[i];
    kl[j] = x.t.lo[i];
    kh[j] = x.t.hi[i];
  }
#pragma unroll
  for (int j = 0; j < XR_SLOTS; j++) {
    const bool in = (int)threadIdx.x + j * (int)blockDim.x < T;
    kv[j] = xs_to_double(kh[j], kl[j], a.xsf);
    kk[j] = (in && kt[j] && kv[j] >= tau0) ? (int)kt[j] - 1 : -1;
    c += kk[j] >= 0 ? 1 : 0;
    c_hi += (kk[j] >= 0 && kv[j] >= ts_hi) ? 1 : 0;
  }
  if (tau_spec > tau0) {
    const int w_hi = wave_sum(c_hi);
    if (lane_id() == 0 && w_hi) atomicAdd(&x.w.misc[XM_CNT], w_hi);
    __syncthreads();
    if (x.w.misc[XM_CNT] >= L) {  // (uniform)
      tau0 = ts_hi;
      c = c_hi;
#pragma unroll
      for (int j = 0; j < XR_SLOTS; j++)
        if (kk[j] >= 0 && kv[j] < ts_hi) kk[j] = -1;
    }
  }
  // wave-aggregated positions in the dense array
  const int incl = wave_incl_scan(c);
  int base = 0;
  if (lane_id() == WAVE - 1 && incl) base = atomicAdd(&x.w.misc[XM_U], incl);
  base = __builtin_amdgcn_readlane(base, WAVE - 1) + incl - c;
  __syncthreads();  // every slot read
  int* dk = reinterpret_cast<int*>(x.t.keys);
  double* dv = reinterpret_cast<double*>(x.t.lo);
#pragma unroll
  for (int j = 0; j < XR_SLOTS; j++)
    if (kk[j] >= 0) { dk[base] = kk[j]; dv[base] = kv[j]; base++; }
  __syncthreads();
  const int D = x.w.misc[XM_FILL];
  const int U = x.w.misc[XM_U];
  if (threadIdx.x == 0 && D) atomicAdd(&dsum[d], (uint32_t)D);
  const uint32_t ts = tie_salt(v);
  auto keyat = [&](int i) { return dk[i]; };
  auto valat = [&](int i) { return dv[i]; };
  SelCrit sc;
  sc.tie = false; sc.pa = 0; sc.ma = 0; sc.pb = 0; sc.mb = 0;
  // (a one-range source with at most `cap` kept entries emits them all: k_xfin1 selects, with a
  // 5-KB wave instead of this workgroup's table -- round 6, as the wave tier's k_wfin)
  const bool cut = U > L && !(cap && !publish && U <= cap);
  if (tph) xr_lap(a, slot, *tph);  // settle + compact
  if (cut) sc = wg_select_top(x.w, U, L, keyat, valat, [](int) { return true; }, ts);
  // (wg_select_top ends on a barrier)
  if (tph) xr_lap(a, slot + 1, *tph);  // select
  double tb = tau0;
  if (publish) {
    if (cut) {
      // the L-th value of this range: the smallest selected value (u64 bits order like the values),
      // reduced over the whole workgroup before it may raise the source's bound
      unsigned long long* wmin = reinterpret_cast<unsigned long long*>(&x.w.misc[XM_MIN]);
      if (threadIdx.x == 0) *wmin = ~0ull;
      __syncthreads();
      unsigned long long mn = ~0ull;
      for (int i = threadIdx.x; i < U; i += blockDim.x) {
        const unsigned long long vb = dbits(dv[i]);
        if (sel_test(sc, vb, tie_w(dk[i], ts))) mn = vb < mn ? vb : mn;
      }
      mn = wave_min_u64(mn);
      if (lane_id() == 0 && mn != ~0ull) atomicMin(wmin, mn);
      __syncthreads();
      if (threadIdx.x == 0 && *wmin != ~0ull) atomicMax(&xtau[d], *wmin);
      __syncthreads();
    }
    tb = fmax(tb, bitsd(__hip_atomic_load(&xtau[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
  }
  for (int i0 = 0; i0 < U; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    bool k = false;
    if (i < U) {
      const uint64_t vb = dbits(dv[i]);
      k = dv[i] >= tb && (!cut || sel_test(sc, vb, tie_w(dk[i], ts)));
    }
    const uint64_t m = __ballot(k);
    uint32_t b0 = 0;
    if (m && lane_id() == 0) b0 = atomicAdd(&pc[d], (uint32_t)__popcll(m));
    b0 = (uint32_t)__shfl((int)b0, 0);
    if (k) {
      const int64_t o = xd.pt_off + b0 + __popcll(m & lanemask_lt());
      pk[o] = dk[i];
      ps[o] = dv[i];
    }
  }
  if (tph) xr_lap(a, slot + 2, *tph);  // emission
}

// The row of a one-range source (k_xr emitted at most L entries, its whole top-L): one wave per
// source copies the list and runs finish_source (row in hash order, range index, norm1, maxDiff)
// -- the big-table workgroup is gone by then, so the row work runs at full occupancy.
__host__ __device__ constexpr size_t xf1_lds_bytes(int Lp) { return (size_t)Lp * 12 + 1024 + (size_t)Lp * 20; }
__global__ void __launch_bounds__(64) k_xfin1(DevSlab s, IterArgs a, const XDesc* xdesc, int d0, const int32_t* pk,
                                              const double* ps, const uint32_t* pc, const uint32_t* dsum,
                                              const int32_t* skip, int32_t* dlast, int Lp,
                                              unsigned long long* maxdiff, unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int d = d0 + (int)blockIdx.x;
  if (skip[d]) return;  // overflowed: redone by the host
  const XDesc xd = xdesc[d];
  uint64_t* rv = reinterpret_cast<uint64_t*>(smem);
  int* rk = reinterpret_cast<int*>(smem + (size_t)Lp * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + (size_t)Lp * 12);
  int* hk = reinterpret_cast<int*>(smem + (size_t)Lp * 12 + 1024);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;
  const int n = (int)pc[d];  // (<= L, or <= the k_xr list cap: finish_source selects then)
  if (dlast && !a.unit && lane_id() == 0) dlast[xd.v] = (int32_t)dsum[d];
  const int32_t* lk = pk + xd.pt_off;
  const double* lv = ps + xd.pt_off;
  finish_source(xd.v, n, [&](int i) { return lk[i]; }, [&](int i) { return lv[i]; }, s, a, hist, rv, rk, Lp, hk, hv, mf,
                maxdiff, stats);
}

// range r of R of a hub source: key k belongs to range ((hash_b(k) * R) >> 32) -- hash_b orders the
// stored rows, the table slot hash is hash32, so the two are independent
__device__ __forceinline__ bool xr_in(int key, int r, int R) {
  return R == 1 || (int)(((uint64_t)hash_b((uint32_t)key) * (uint32_t)R) >> 32) == r;
}

struct XTask { int32_t d; int32_t r; };

// One workgroup per (source, range): every wave walks its windows of the source's successor rows
// (a short successor list: all waves share each window, each taking every W-th batch of groups).
__global__ void __launch_bounds__(1024) k_xr(DevGraph g, DevSlab s, IterArgs a, const XDesc* xdesc,
                                             const XTask* tasks, int T, int budget, int Lp, unsigned long long* xtau,
                                             int32_t* pk, double* ps, uint32_t* pc, uint32_t* dsum,
                                             int32_t* oflag, int32_t* ovl, int xcap) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const XrLds x = xr_carve(smem, T, W, Lp);
  const XTask tk = tasks[blockIdx.x];
  const XDesc xd = xdesc[tk.d];
  const int v = xd.v, R = xd.R, r = tk.r;
  long long tph = a.diag ? (long long)clock64() : 0;  // PPR_DIAG phase cycles (thread 0, between barriers)
  xr_clear(x, T);
  __syncthreads();
  if (threadIdx.x == 0 && xr_in(v, r, R)) {
    unsigned long long lo;
    uint32_t hi;
    xs_conv(xd.selfval, lo, hi, a.xsf);
    xt_add(x.t, v, lo, hi);
    x.w.misc[XM_FILL] = 1;
  }
  __syncthreads();
  xr_lap(a, 183, tph);
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = xd.factor;
  unsigned long long mb = 0;
  uint8_t* fl = x.fl + (size_t)wv * HUB_WALK_FLAGS;
  auto fn = [&](bool valid, int id, double sv, bool) {
#if defined(PPR_XR_WALK_ONLY)  // (timing-only build: the walk alone, no table work)
    if (valid && id == -9 && sv == -1.0) x.w.misc[XM_FILL] = 1;
    return;
#endif
    if (xr_stop(x, budget)) return;  // (uniform per wave: one LDS read per group)
    xr_apply(x, valid && xr_in(id, r, R), id, sv * factor, budget, a.xsf);
  };
  if (a.unit) {
    for (int64_t e0 = b + (int64_t)wv * WAVE; e0 < e; e0 += (int64_t)W * WAVE) {
      const int64_t i = e0 + lane_id();
      const int key = i < e ? (g.colx[i] & 0x7fffffff) : 0;
      if (xr_stop(x, budget)) break;
      xr_apply(x, i < e && xr_in(key, r, R), key, factor, budget, a.xsf);
    }
  } else {
    // each wave walks its own contiguous share of the successor list (one window setup per 64
    // successors, every wave busy at once); sharing each window among the waves cost every wave
    // the window's dependent setup loads once per window, one window after another
    const int64_t chunk = (e - b + W - 1) / W;
    const int64_t c0 = b + (int64_t)wv * chunk, c1 = min(e, c0 + chunk);
    for (int64_t w0 = c0; w0 < c1; w0 += WAVE)
      hub_window_walk(g, s, a, w0, min(c1, w0 + WAVE), fl, fn, WalkRowMin{&mb, (int)s.L});
  }
  __syncthreads();
  xr_lap(a, 184, tph);
  if (a.diag && threadIdx.x == 0) {
    diag_add(a.diag, 182, 1ull);
    diag_add(a.diag, 188, (unsigned long long)(xd.R > 0 ? (e - b) : 0));
    diag_add(a.diag, 189, (unsigned long long)x.w.misc[XM_FILL]);
  }
  if (x.w.misc[XM_FILL] > budget) {
    if (threadIdx.x == 0 && atomicExch(&oflag[tk.d], 1) == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = tk.d;
    return;
  }
  // pruning bound from the full successor rows (every wave saw every row's minimum)
#pragma unroll
  for (int o = 32; o; o >>= 1) { const unsigned long long y = __shfl_xor(mb, o); mb = y > mb ? y : mb; }
  if (lane_id() == 0 && mb) atomicMax(reinterpret_cast<unsigned long long*>(&x.w.misc[8]), mb);
  __syncthreads();
  const unsigned long long mbb = *reinterpret_cast<unsigned long long*>(&x.w.misc[8]);
  const double tau_rows = (!a.unit && mbb) ? xs_single(bitsd(mbb) * factor, a.xsf) : 0.0;
  // one-range source: its previous L-th score (row minimum of a full current row) x XR_SPEC as a
  // speculative bound (scores move little between updates; the check in xr_finish keeps it exact)
  double tau_spec = 0.0;
  if (R == 1 && !a.unit && !a.mc) {
    const int64_t cr = s.lrow((a.active == 1) ? a.sB : a.sA, v);
    if (s.len[cr] == s.L) tau_spec = XR_SPEC * s.rmin[cr];
  }
  xr_finish(x, T, s, a, xd, tk.d, R > 1, tau_rows, tau_spec, xtau, pk, ps, pc, dsum, a.diag ? &tph : nullptr, 185, xcap);
}

// One workgroup per staged bucket of a partitioned hub source: the bucket's records are
// contiguous (merge_hub.h k_hub_scatter), W waves take every W-th group of 64.
constexpr int XB_BATCH = 4;  // groups a wave loads before applying them
__global__ void __launch_bounds__(1024) k_xb(DevSlab s, IterArgs a, const HubDesc* desc, const HubTask* tasks,
                                             const int32_t* cm, const uint32_t* staged, const HubRec* st,
                                             const unsigned long long* tau_b, int T, int budget, int Lp,
                                             unsigned long long* xtau, int32_t* pk, double* ps, uint32_t* pc,
                                             uint32_t* dsum, int32_t* oflag, int32_t* ovl, const int64_t* rp) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const XrLds x = xr_carve(smem, T, W, Lp);
  const HubTask tk = tasks[blockIdx.x];
  const HubDesc d = desc[tk.d];
  int64_t start, nb;
  hub_bucket_range(d, cm, staged[tk.d], tk.x, start, nb);
  const int v = d.v;
  const int64_t deg = rp[v + 1] - rp[v];
  const double factor = merge_factor(a, deg);
  long long tph = a.diag ? (long long)clock64() : 0;
  xr_clear(x, T);
  __syncthreads();
  if (threadIdx.x == 0 && (int)hub_digit(v, d.logP) == tk.x) {
    unsigned long long lo;
    uint32_t hi;
    xs_conv(self_seed(a, deg), lo, hi, a.xsf);
    xt_add(x.t, v, lo, hi);
    x.w.misc[XM_FILL] = 1;
  }
  __syncthreads();
  const HubRec* rec = st + start;
  const int64_t ng = (nb + WAVE - 1) / WAVE;
  // a batch of XB_BATCH groups per wave (groups wv, wv + W, ...), the next batch's loads issued
  // before the current one is applied (clamped, unconditional loads: a load under a branch ends
  // in its own vmcnt(0) wait)
  struct Batch { HubRec r[XB_BATCH]; };
  auto load = [&](int64_t g0, Batch& hr) {
#pragma unroll
    for (int k = 0; k < XB_BATCH; k++) {
      const int64_t q = (g0 + (int64_t)k * W) * WAVE + lane_id();
      hr.r[k] = rec[q < nb ? q : nb - 1];
    }
  };
  // (no early exits inside a batch: a break there made the compiler shuffle the prefetched
  // registers, which waits for the prefetch)
  // Hot key of the wave: a bucket holding one of the source's core keys has that key in a third
  // or more of its records (one per successor row), and same-address LDS atomics serialise lane by
  // lane. Each wave picks the most frequent of 8 sampled keys of its first group (when it fills
  // >= 1/8 of the group) and sums that key's contributions in a per-lane register accumulator --
  // exact 96-bit adds, order-free like the table -- added to the table once per lane at the end.
  int hk = -1;
  unsigned long long hlo = 0ull;
  uint32_t hhi = 0u;
  // A batch's XB_BATCH groups are applied together: their group-of-four probe reads issued back
  // to back, then the rare misses (new keys, longer probes) resolved one group after another,
  // then all returning low-word adds, then the high-word adds -- a few dependent LDS round trips
  // per batch instead of per group (the waves sat 59 % of their cycles waiting).
  // Budget: before a group inserts new keys its wave checks the shared count (an LDS read) and
  // adds the group's inserts to it right after, before its next check, so at most one group per
  // wave (64 keys) is ever uncounted and the table holds at most budget + W * 64 keys. (A batch
  // that checked once for its four groups let the other waves' checks miss up to 4 * 64 keys of
  // each batch in flight: a table could fill up and a probe run forever.) Past the budget a
  // wave drops its new keys: the source overflows and is merged again.
  auto apply = [&](int64_t g0, const Batch& hr) {
    bool v[XB_BATCH];
    int key[XB_BATCH];
    unsigned long long lo[XB_BATCH];
    uint32_t hi[XB_BATCH], g[XB_BATCH];
    uint4 q[XB_BATCH];
#pragma unroll
    for (int k = 0; k < XB_BATCH; k++) {
      const int64_t gk = g0 + (int64_t)k * W;
      key[k] = rec_key(hr.r[k]);
      v[k] = gk < ng && gk * WAVE + lane_id() < nb;
      xs_conv(rec_sc(hr.r[k]) * factor, lo[k], hi[k], a.xsf);
      if (v[k] && key[k] == hk) {
        const unsigned long long nl = hlo + lo[k];
        hhi += hi[k] + (nl < hlo ? 1u : 0u);
        hlo = nl;
        v[k] = false;
      }
      g[k] = hash32((uint32_t)key[k]) & x.t.mask & ~3u;
    }
#pragma unroll
    for (int k = 0; k < XB_BATCH; k++) q[k] = *reinterpret_cast<const uint4*>(x.t.keys + g[k]);
    int h[XB_BATCH];
#pragma unroll
    for (int k = 0; k < XB_BATCH; k++) {
      h[k] = xt_match(q[k], g[k], (uint32_t)key[k] + 1u);
      if (__ballot(v[k] && h[k] < 0)) {
        if (xr_stop(x, budget)) {
          if (h[k] < 0) v[k] = false;
        } else {
          bool ins = false;
          if (v[k] && h[k] < 0) h[k] = xt_slot(x.t, key[k], ins);
          const bool full = v[k] && h[k] < 0;  // (the probe ran out: overflow redo)
          if (full) v[k] = false;
          const int nins = __popcll(__ballot(ins)) + (__ballot(full) ? XR_FULL : 0);
          if (nins && lane_id() == 0) atomicAdd(&x.w.misc[XM_FILL], nins);
        }
      }
    }
    // (unconditional atomics -- an idle lane adds 0 to slot 0 -- so the four returning adds are in
    // flight together: under a per-lane branch each one ended in its own wait)
    unsigned long long old[XB_BATCH];
#pragma unroll
    for (int k = 0; k < XB_BATCH; k++) {
      if (!v[k]) { h[k] = 0; lo[k] = 0ull; hi[k] = 0u; }
      old[k] = atomicAdd(&x.t.lo[h[k]], lo[k]);
    }
#pragma unroll
    for (int k = 0; k < XB_BATCH; k++) atomicAdd(&x.t.hi[h[k]], hi[k] + ((old[k] + lo[k] < old[k]) ? 1u : 0u));
  };
  Batch ba, bb;
  const int64_t step = (int64_t)W * XB_BATCH;
  if (wv < ng) {
    load(wv, ba);
    // (the first group only: its lanes are valid up to nb)
    const bool v0 = (int64_t)wv * WAVE + lane_id() < nb;
    const int k0 = rec_key(ba.r[0]);
    int best = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const int cand = __builtin_amdgcn_readlane(k0, c * 8);
      const int n = __popcll(__ballot(v0 && k0 == cand));
      if (n > best && __builtin_amdgcn_readlane((int)v0, c * 8)) { best = n; hk = cand; }
    }
    if (best < 8) hk = -1;
  }
  // (sched_barrier: the scheduler otherwise pulls the next batch's first uses up into the current
  // batch, waiting for the prefetch right after issuing it)
  for (int64_t g0 = wv; g0 < ng; g0 += 2 * step) {
    load(g0 + step < ng ? g0 + step : g0, bb);  // (unconditional: past the end it reloads a batch)
    __builtin_amdgcn_sched_barrier(0);
    apply(g0, ba);
    __builtin_amdgcn_sched_barrier(0);
    if (g0 + step >= ng) break;
    load(g0 + 2 * step < ng ? g0 + 2 * step : g0, ba);
    __builtin_amdgcn_sched_barrier(0);
    apply(g0 + step, bb);
    __builtin_amdgcn_sched_barrier(0);
  }
  // the hot key's register sums (a lane's sum stays below the key's total < 2^95): once per lane
  if (hk >= 0 && (hlo | hhi)) {
    const int r = xt_add(x.t, hk, hlo, hhi);
    if (r) atomicAdd(&x.w.misc[XM_FILL], r > 0 ? 1 : XR_FULL);
  }
  __syncthreads();
  xr_lap(a, 155, tph);
  if (a.diag && threadIdx.x == 0) {
    diag_add(a.diag, 154, 1ull);
    diag_add(a.diag, 159, (unsigned long long)nb);
  }
  if (x.w.misc[XM_FILL] > budget) {
    if (threadIdx.x == 0 && atomicExch(&oflag[tk.d], 1) == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = v;
    return;
  }
  const double tau_rows = (!a.unit && tau_b[tk.d]) ? xs_single(bitsd(tau_b[tk.d]) * factor, a.xsf) : 0.0;
  XDesc xd;
  xd.v = v; xd.R = 0; xd.pt_off = d.pt_off; xd.factor = factor; xd.selfval = 0.0;
  xr_finish(x, T, s, a, xd, tk.d, true, tau_rows, 0.0, xtau, pk, ps, pc, dsum, a.diag ? &tph : nullptr, 156);
}

// One workgroup per listed source: top-L of the entries its ranges / buckets appended (keys are
// disjoint across them) at or above the final bound, then the row, norm1, maxDiff.
// (Desc: XDesc of a ranged source or HubDesc of a partitioned one: v and pt_off)
constexpr int XF_STAGE = 4096;  // entries staged in LDS (beyond: the select reads the list in HBM)
__host__ __device__ constexpr size_t xf_lds_bytes(int Lp, int stage) { return (size_t)stage * 12 + 1024 + 256 + (size_t)Lp * 32; }

template <class Desc>
__global__ void __launch_bounds__(256) k_xfinal(DevSlab s, IterArgs a, const Desc* desc,
                                                const unsigned long long* xtau, const int32_t* pk, const double* ps,
                                                const uint32_t* pc, const uint32_t* dsum, const int32_t* skip,
                                                int32_t* dlast, int Lp, int stage, unsigned long long* maxdiff,
                                                unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int d = blockIdx.x;
  if (skip && skip[d]) return;  // overflowed: redone by the host (uniform: one load per thread, set before this launch)
  const int v = desc[d].v;
  const int L = s.L;
  unsigned char* p = smem;
  double* sv = reinterpret_cast<double*>(p); p += (size_t)stage * 8;
  int* sk = reinterpret_cast<int*>(p); p += (size_t)stage * 4;
  WgLds w = WgLds{};
  w.hist = reinterpret_cast<uint32_t*>(p); p += 1024;
  w.misc = reinterpret_cast<int*>(p); p += 256;
  w.rv = reinterpret_cast<uint64_t*>(p); p += (size_t)Lp * 8;
  w.rk = reinterpret_cast<int*>(p); p += (size_t)Lp * 4;
  w.hk = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  w.hv = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  w.mf = reinterpret_cast<int*>(p);
  const int64_t off = desc[d].pt_off;
  const int n = (int)pc[d];
  const double tb = bitsd(xtau[d]);
  if (threadIdx.x < 64) w.misc[threadIdx.x] = 0;
  __syncthreads();
  // stage the entries >= the final bound (the top-L all are: one range alone holds L keys >= it)
  for (int i0 = 0; i0 < n; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    const bool keep = i < n && ps[off + i] >= tb;
    const uint64_t m = __ballot(keep);
    int base = 0;
    if (m && lane_id() == 0) base = atomicAdd(&w.misc[XM_CNT], __popcll(m));
    base = __shfl(base, 0);
    const int pos = base + __popcll(m & lanemask_lt());
    if (keep && pos < stage) { sv[pos] = ps[off + i]; sk[pos] = pk[off + i]; }
  }
  __syncthreads();
  const int U = w.misc[XM_CNT];
  const uint32_t ts = tie_salt(v);
  const bool staged = U <= stage;
  auto keyat = [&](int i) { return staged ? sk[i] : pk[off + i]; };
  auto valat = [&](int i) { return staged ? sv[i] : ps[off + i]; };
  const int N = staged ? U : n;
  auto elig = [&](int i) { return staged || ps[off + i] >= tb; };
  const bool cut = U > L;
  SelCrit sc;
  sc.tie = false; sc.pa = 0; sc.ma = 0; sc.pb = 0; sc.mb = 0;
  if (cut) sc = wg_select_top(w, N, L, keyat, valat, elig, ts);
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    if (!elig(i)) continue;
    const uint64_t vb = dbits(valat(i));
    const int key = keyat(i);
    if (cut && !sel_test(sc, vb, tie_w(key, ts))) continue;
    const int pos = atomicAdd(&w.misc[XM_U], 1);
    w.rv[pos] = vb;
    w.rk[pos] = key;
  }
  __syncthreads();
  if (threadIdx.x < WAVE) {
    const int cnt = w.misc[XM_U];
    const uint64_t* rv = w.rv;
    const int* rk = w.rk;
    if (dlast && !a.unit && lane_id() == 0) dlast[v] = (int32_t)dsum[d];
    finish_source(v, cnt, [&](int i) { return rk[i]; }, [&](int i) { return bitsd(rv[i]); }, s, a, w.hist, w.rv,
                  w.rk, Lp, w.hk, w.hv, w.mf, maxdiff, stats);
  }
}

}  // namespace pprk
