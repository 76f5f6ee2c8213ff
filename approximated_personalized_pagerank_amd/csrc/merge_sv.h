// merge_sv.h -- the sieve merge of the wide GRank sources (exact sum).
//
// A wide source (more candidates than a wave table holds) has up to millions of distinct keys, yet
// only its top-L survive the merge, and between two updates they barely change (RMAT-22 at
// iteration 20: all 128 previous top-L keys are again the top-L of >99 % of the wide sources,
// profiles/r04_sieve_workload_rmat22.json). The sieve uses that without trusting it:
//
//   pass 1  every candidate (k, s) of the source: p = s * d/deg. If k is one of the L keys of the
//           source's current row (the "prev" table PT, LDS), p is added EXACTLY to k's fixed-point
//           accumulator; otherwise ceil(p * 2^31) is added to SV_R counters of a count-min sketch
//           (one per row, hashed). Sketch counters only over-estimate a key's total.
//   bound   theta = the smallest exact total of the L prev keys: L distinct keys reach it, so the
//           L-th largest total is >= theta (rigorous, whatever the rows did).
//   pass 2  the candidates again: a key outside PT whose SV_R counters all reach theta ("passes")
//           is accumulated exactly in a second LDS table XT; every other key's total is < theta
//           and cannot be in the top-L (nor tied at its cut).
//   select  top-L of PT u XT by (value desc, tie hash desc) -- the same set and the same order as
//           the exact sum over all keys (merge_xs.h), so the row, norm1 and maxDiff are bit-identical.
// A source whose passing keys overflow XT is handed back to the range / partition engines of
// merge_xs.h (correct either way, slower). Sources whose current row is not full (no L keys to
// bound with) never enter the sieve.
//
// Exact accumulators: X = sum floor(p * 2^93) (oracle/grank_oracle.c "exact") held as two u64
// words that are only ever added to -- A = sum of the low 32 bits of each X_i, B = sum of X_i >> 32
// -- so X = B * 2^32 + A needs no returning atomic (no carry chase) and any lane, wave or
// workgroup may add in any order.
//
//   k_sv1   one 16-wave workgroup per source of one slice: pass 1, bound, pass 2, select, row
//   k_svA   pass 1 of one slice of a multi-slice source: the sketch and PT partial sums are added
//           to the source's global copies
//   k_svB   pass 2 of one slice: bound and sieve from the global copies, XT flushed into the
//           source's global table
//   k_svF   one workgroup per multi-slice source: top-L of PT u global table, row
#pragma once
#include "merge_xs.h"

namespace pprk {

constexpr int SV_R = 3;                       // sketch rows
constexpr int SV_UNIT_LOG = 31;               // a counter unit is 2^-31 (GRank totals are <= 1)
constexpr int SV_XS = 4;                      // pass-2 table slots per thread in every size class
// Size classes of the one-slice workgroups (host: sieve_launch): the widest sources take 16 waves
// and a 3 x 8192 sketch (one workgroup per CU), narrower ones 8 waves / 3 x 4096 (two per CU) or
// 4 waves / 3 x 2048 (four per CU) -- a narrow source's few batches per wave cannot hide their HBM
// latencies unless several sources share the CU. Multi-slice sources use the widest class.
struct SvGeom {
  int wlog;     // counters per sketch row = 2^wlog
  int waves;
  int xt;       // pass-2 table slots (= SV_XS * threads)
  int budget;   // distinct passing keys before the table overflows
  __host__ __device__ constexpr int threads() const { return waves * WAVE; }
  __host__ __device__ constexpr int bm_words() const { return SV_R * (1 << wlog) / 64; }
  __host__ __device__ constexpr size_t sketch_bytes() const { return (size_t)SV_R * ((size_t)1 << wlog) * 4; }
  __host__ __device__ constexpr size_t region() const {
    return sketch_bytes() > (size_t)xt * 20 ? sketch_bytes() : (size_t)xt * 20;
  }
};
__host__ __device__ constexpr SvGeom sv_geom(int wlog, int waves) {
  return SvGeom{wlog, waves, SV_XS * waves * WAVE, SV_XS * waves * WAVE * 85 / 100 - waves * WAVE};
}
constexpr SvGeom SV_LARGE = sv_geom(13, 16), SV_MID = sv_geom(12, 8), SV_SMALL = sv_geom(11, 4);
constexpr int SV_THREADS = 16 * WAVE;         // the widest class (multi-slice kernels)
constexpr int SV_XT_BUDGET = SV_LARGE.budget;
constexpr int SVF_CAP = 4096;                 // k_svF: dense entries at or above the bound
constexpr uint32_t WI_SV_P1WALK = 1u << 11;   // PPR_WHATIF 2048: sieve pass 1 through hub_window_walk (A/B)

// ---------------------------------------------------------------------------------------------
// split exact accumulators (keys u32 | A u64 | B u64: 20 B a slot)
struct X2Table {
  uint32_t* keys;
  unsigned long long* a;
  unsigned long long* b;
  uint32_t mask;
};
__host__ __device__ constexpr size_t x2_bytes(int T) { return (size_t)T * 20; }
__device__ __forceinline__ X2Table x2_carve(unsigned char* p, int T) {
  X2Table t;
  t.keys = reinterpret_cast<uint32_t*>(p);
  t.a = reinterpret_cast<unsigned long long*>(p + (size_t)T * 4);
  t.b = reinterpret_cast<unsigned long long*>(p + (size_t)T * 12);
  t.mask = (uint32_t)T - 1u;
  return t;
}
__device__ __forceinline__ void x2_add(const X2Table& t, int h, unsigned long long lo, uint32_t hi) {
  atomicAdd(&t.a[h], lo & 0xffffffffull);
  atomicAdd(&t.b[h], (lo >> 32) | ((unsigned long long)hi << 32));
}
// X = B * 2^32 + A (< 2^95) rounded to a double like xs_to_double
__device__ __forceinline__ double x2_value(unsigned long long A, unsigned long long B) {
  const unsigned long long lo = ((B & 0xffffffffull) << 32) + A;
  const uint32_t hi = (uint32_t)(B >> 32) + (lo < A ? 1u : 0u);
  return xs_to_double(hi, lo);
}
// membership probe of a table that no longer changes: the slot of `key` or -1. (Insert-only
// group probing: a key sits in the first group of its sequence that had an empty slot when it was
// inserted, so a group with an empty slot ends the search.)
__device__ __forceinline__ int x2_find(const X2Table& t, int key) {
  const uint32_t tag = (uint32_t)key + 1u;
  uint32_t g = hash32((uint32_t)key) & t.mask & ~3u;
  for (uint32_t n = 0; n <= t.mask; n += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(t.keys + g);
    const int m = xt_match(q, g, tag);
    if (m >= 0) return m;
    if (q.x == 0u || q.y == 0u || q.z == 0u || q.w == 0u) return -1;
    g = (g + 4u) & t.mask;
  }
  return -1;
}
// find-or-insert with a bounded probe: at most T/4 groups visited and T/4 lost insert races
// (each lost race fills a slot), -1 when both run out -- the caller takes the overflow path
// instead of spinning
__device__ __forceinline__ int x2_slot(const X2Table& t, int key, bool& ins) {
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
      continue;  // another key took it: read the group again
    }
    g = (g + 4u) & t.mask;
    moves++;
  }
  return -1;
}

// ---------------------------------------------------------------------------------------------
// count-min sketch: SV_R counters per key from one 64-bit mix (independent of hash32 / hash_b)
__device__ __forceinline__ uint64_t sv_mix(uint32_t k) {
  uint64_t x = (uint64_t)k * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 32;
  return x;
}
__device__ __forceinline__ uint32_t sv_cell(uint64_t x, int j, int wlog) {
  return ((uint32_t)j << wlog) + ((uint32_t)(x >> (wlog * j)) & ((1u << wlog) - 1u));
}
// ceil(p * 2^31): an upper bound of the contribution in counter units
__device__ __forceinline__ uint32_t sv_units(double p) {
  const double x = ceil(ldexp(p, SV_UNIT_LOG));
  return x >= 4294967295.0 ? 0xffffffffu : (uint32_t)x;
}
// counter threshold of the bound theta: a key whose total reaches theta has every counter >=
// 2^31 * theta * (1 - 2^-52) (its stored value rounds up by at most half an ulp); the margin
// below makes the test conservative (a counter at the threshold passes)
__device__ __forceinline__ uint32_t sv_thr(double theta) {
  const double x = floor(ldexp(theta, SV_UNIT_LOG) * (1.0 - 0x1p-40));
  return x <= 0.0 ? 0u : x >= 4294967295.0 ? 0xffffffffu : (uint32_t)x;
}
__device__ __forceinline__ void sv_sketch_add(uint32_t* sk, int key, uint32_t u, int wlog) {
  const uint64_t x = sv_mix((uint32_t)key);
#pragma unroll
  for (int j = 0; j < SV_R; j++) atomicAdd(&sk[sv_cell(x, j, wlog)], u);
}
// every counter of `key` at or above the threshold (bitmap of the counters that are)
__device__ __forceinline__ bool sv_passes(const uint64_t* bm, int key, int wlog) {
  const uint64_t x = sv_mix((uint32_t)key);
  uint64_t w[SV_R];
  uint32_t c[SV_R];
#pragma unroll
  for (int j = 0; j < SV_R; j++) { c[j] = sv_cell(x, j, wlog); w[j] = bm[c[j] >> 6]; }
  bool ok = true;
#pragma unroll
  for (int j = 0; j < SV_R; j++) ok = ok && ((w[j] >> (c[j] & 63u)) & 1ull);
  return ok;
}

// ---------------------------------------------------------------------------------------------
// one sieve source: descriptor, and one slice of a multi-slice source
struct SvDesc {
  int32_t v;
  int32_t S;          // slices (1: k_sv1)
  double factor;      // d / deg
  int64_t gsk;        // multi: u32 offset of its global sketch (SV_LARGE: SV_R * 8192)
  int64_t gpt;        // multi: offset of its PT sums (Lp pairs of u64: A, B by prev-row position)
  int64_t gxt;        // multi: slot offset of its global table
  int32_t tg;         // multi: global table slots (power of two)
  int32_t pad;
};
struct SvTask { int32_t d; int32_t k; };

// LDS of the slice / single-source workgroups:
//   region (sketch in pass 1; XT in pass 2; dense (value, key) list in the select)
//   PT (2 Lp slots) | pti i32[2 Lp] (prev-row position of a PT slot) | bitmap u64[bm_words] |
//   walk flags u8[waves][HUB_WALK_FLAGS] | misc i32[64] | hist u32[256] (block select)
enum { SVM_FILL = 0, SVM_OVF = 1, SVM_U = 2, SVM_PT = 3, SVM_THETA = 8 /* u64: 8..9 */ };
__host__ __device__ constexpr size_t sv_lds_bytes(int Lp, SvGeom G) {
  return G.region() + x2_bytes(2 * Lp) + (size_t)8 * Lp + (size_t)G.bm_words() * 8 +
         (size_t)G.waves * HUB_WALK_FLAGS + 256 + 1024;
}
struct SvLds {
  unsigned char* region;
  X2Table pt;
  int* pti;
  uint64_t* bm;
  uint8_t* fl;
  int* misc;
  uint32_t* hist;
  int wlog;
  int bm_words;
};
__device__ __forceinline__ SvLds sv_carve(unsigned char* smem, int Lp, SvGeom G) {
  SvLds x;
  unsigned char* p = smem;
  x.region = p; p += G.region();
  x.pt = x2_carve(p, 2 * Lp); p += x2_bytes(2 * Lp);
  x.pti = reinterpret_cast<int*>(p); p += (size_t)8 * Lp;
  x.bm = reinterpret_cast<uint64_t*>(p); p += (size_t)G.bm_words() * 8;
  x.fl = p; p += (size_t)G.waves * HUB_WALK_FLAGS;
  x.misc = reinterpret_cast<int*>(p); p += 256;
  x.hist = reinterpret_cast<uint32_t*>(p);
  x.wlog = G.wlog;
  x.bm_words = G.bm_words();
  return x;
}

__device__ __forceinline__ void sv_lap(const IterArgs& a, int slot, long long& t) {
  if (!a.diag || threadIdx.x != 0) return;
  const long long now = (long long)clock64();
  diag_add(a.diag, slot, (unsigned long long)(now - t));
  t = now;
}

// the current row of v (L distinct keys) into PT, zeroed sums; misc cleared; pti = row position
__device__ __forceinline__ void sv_build_pt(const SvLds& x, const DevSlab& s, const IterArgs& a, int v, int Lp) {
  const int T = 2 * Lp;
  for (int i = threadIdx.x; i < T; i += blockDim.x) { x.pt.keys[i] = 0u; x.pt.a[i] = 0ull; x.pt.b[i] = 0ull; }
  if (threadIdx.x < 64) x.misc[threadIdx.x] = 0;
  __syncthreads();
  const int cur = (a.active == 1) ? a.sB : a.sA;
  const int64_t r = s.row(cur, v);
  const int len = s.len[s.lrow(cur, v)];
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    bool ins;
    const int h = x2_slot(x.pt, s.key(s.ids[r + i]), ins);
    if (h >= 0) x.pti[h] = i;
  }
}

// successors [b0, b1) of a slice, one contiguous chunk per wave, windows of 64 successors
template <class F>
__device__ __forceinline__ void sv_walk(const DevGraph& g, const DevSlab& s, const IterArgs& a, const SvLds& x,
                                        int64_t b0, int64_t b1, F f) {
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const int64_t chunk = (b1 - b0 + W - 1) / W;
  const int64_t c0 = b0 + (int64_t)wv * chunk, c1 = min(b1, c0 + chunk);
  uint8_t* fl = x.fl + (size_t)wv * HUB_WALK_FLAGS;
  for (int64_t w0 = c0; w0 < c1; w0 += WAVE) hub_window_walk(g, s, a, w0, min(c1, w0 + WAVE), fl, f);
}

// pass 1 over successors [b0, b1): prev keys exactly into PT, every other key into the sketch
__device__ __forceinline__ void sv_pass1(const DevGraph& g, const DevSlab& s, const IterArgs& a, const SvLds& x,
                                         int64_t b0, int64_t b1, double factor, uint32_t* sk) {
  sv_walk(g, s, a, x, b0, b1, [&](bool valid, int id, double sv, bool) {
    if (!valid) return;
    const double p = sv * factor;
    const int h = x2_find(x.pt, id);
    if (h >= 0) {
      unsigned long long lo;
      uint32_t hi;
      xs_conv(p, lo, hi);
      x2_add(x.pt, h, lo, hi);
    } else {
      sv_sketch_add(sk, id, sv_units(p), x.wlog);
    }
  });
}

// The candidates of successors [i0, e) (<= 64) like hub_window_walk, a batch of HUB_TW_BATCH
// groups at a time (the next batch's loads in flight): fb(valid[], key[], ridx[], score[]) with each
// candidate's slab index; scores are loaded only with kScores (pass 2 loads a score only for a
// candidate that passes).
template <bool kScores, class FB>
__device__ __forceinline__ void sv_window(const DevGraph& g, const DevSlab& s, const IterArgs& a, int64_t i0,
                                          int64_t e, uint8_t* fl, FB fb) {
  constexpr int NB = HUB_TW_BATCH;
  const int64_t i = i0 + lane_id();
  int u = 0, sl = 0, ln = 0;
  if (i < e) {
    const int32_t cx = g.colx[i];
    u = cx & 0x7fffffff;
    sl = read_slot(a, cx);
    ln = s.len[s.lrow(sl, u)];
  }
  const int incl = wave_incl_scan(ln);
  const int total = __builtin_amdgcn_readlane(incl, WAVE - 1);
  const bool flags = !__ballot(i < e && ln == 0);
  auto load = [&](int g0, int (&key)[NB], int64_t (&ri)[NB], double (&sv)[NB]) {
    if (flags) {
#pragma unroll
      for (int q = 0; q < NB / 4; q++) reinterpret_cast<uint32_t*>(fl)[q * WAVE + lane_id()] = 0u;
      wave_fence();
      if (incl > g0 && incl < g0 + WAVE * NB) fl[incl - g0] = 1;
      wave_fence();
    }
#pragma unroll
    for (int k = 0; k < NB; k++) {
      const int c = g0 + k * WAVE + lane_id();
      int j = 0;
      if (flags) {
        const int G = g0 + k * WAVE;
        const uint64_t ends = __ballot(fl[k * WAVE + lane_id()] != 0) & ~1ull;
        j = __popcll(__ballot(incl <= G)) + __popcll(ends & (lanemask_lt() | (1ull << lane_id())));
      } else {
#pragma unroll
        for (int step = 32; step; step >>= 1) {
          const int pv = __shfl(incl, j + step - 1);
          if (pv <= c) j += step;
        }
      }
      const int jj = j < WAVE ? j : WAVE - 1;
      const int exv = __shfl(incl, jj > 0 ? jj - 1 : 0);
      const int ex = jj > 0 ? exv : 0;
      const int uj = __shfl(u, jj);
      const int sj = __shfl(sl, jj);
      key[k] = 0;
      ri[k] = 0;
      sv[k] = 0.0;
      if (c < total) {
        ri[k] = s.row(sj, uj) + (c - ex);
        key[k] = ld_nt(&s.ids[ri[k]], a.nt & 1u);
        if (kScores) sv[k] = ld_nt(&s.sc[ri[k]], a.nt & 1u);
      }
    }
  };
  int key[NB], nkey[NB];
  int64_t ri[NB], nri[NB];
  double sv[NB], nsv[NB];
  if (total > 0) load(0, nkey, nri, nsv);
  for (int g0 = 0; g0 < total; g0 += WAVE * NB) {
    bool valid[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
      key[k] = nkey[k];
      ri[k] = nri[k];
      sv[k] = nsv[k];
      valid[k] = g0 + k * WAVE + lane_id() < total;
    }
    if (g0 + WAVE * NB < total) load(g0 + WAVE * NB, nkey, nri, nsv);
    fb(valid, key, ri, sv);
  }
}

// pass 1, one batch at a time: the first PT group of every candidate read at once, the rare
// longer probes after, then the exact PT adds or the sketch adds
__device__ __forceinline__ void sv_pass1b(const DevGraph& g, const DevSlab& s, const IterArgs& a, const SvLds& x,
                                          int64_t b0, int64_t b1, double factor, uint32_t* sk) {
  constexpr int NB = HUB_TW_BATCH;
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const int64_t chunk = (b1 - b0 + W - 1) / W;
  const int64_t c0 = b0 + (int64_t)wv * chunk, c1 = min(b1, c0 + chunk);
  uint8_t* fl = x.fl + (size_t)wv * HUB_WALK_FLAGS;
  for (int64_t w0 = c0; w0 < c1; w0 += WAVE)
    sv_window<true>(g, s, a, w0, min(c1, w0 + WAVE), fl, [&](const bool (&valid)[NB], const int (&key)[NB],
                                                            const int64_t (&)[NB], const double (&sv)[NB]) {
      uint4 q[NB];
      uint32_t g0[NB];
#pragma unroll
      for (int k = 0; k < NB; k++) {
        g0[k] = hash32((uint32_t)key[k]) & x.pt.mask & ~3u;
        q[k] = *reinterpret_cast<const uint4*>(x.pt.keys + g0[k]);
      }
#pragma unroll
      for (int k = 0; k < NB; k++) {
        if (!valid[k]) continue;
        int h = xt_match(q[k], g0[k], (uint32_t)key[k] + 1u);
        if (h < 0 && q[k].x && q[k].y && q[k].z && q[k].w) h = x2_find(x.pt, key[k]);  // (a full group: probe on)
        const double p = sv[k] * factor;
        if (h >= 0) {
          unsigned long long lo;
          uint32_t hi;
          xs_conv(p, lo, hi);
          x2_add(x.pt, h, lo, hi);
        } else {
          sv_sketch_add(sk, key[k], sv_units(p), x.wlog);
        }
      }
    });
}

// pass 2 over successors [b0, b1): keys outside PT that pass the sieve, exactly into XT (budget
// checked before every group that inserts; past it the workgroup only flags the overflow). Per
// batch: the sieve tests of all its groups, then the passing candidates' scores (loads in flight
// together), then the inserts.
__device__ __forceinline__ void sv_pass2(const DevGraph& g, const DevSlab& s, const IterArgs& a, const SvLds& x,
                                         const X2Table& xt, int64_t b0, int64_t b1, double factor, int budget) {
  constexpr int NB = HUB_TW_BATCH;
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const int64_t chunk = (b1 - b0 + W - 1) / W;
  const int64_t c0 = b0 + (int64_t)wv * chunk, c1 = min(b1, c0 + chunk);
  uint8_t* fl = x.fl + (size_t)wv * HUB_WALK_FLAGS;
  for (int64_t w0 = c0; w0 < c1; w0 += WAVE)
    sv_window<false>(g, s, a, w0, min(c1, w0 + WAVE), fl, [&](const bool (&valid)[NB], const int (&key)[NB],
                                                             const int64_t (&ri)[NB], const double (&)[NB]) {
      bool want[NB];
      bool any = false;
#pragma unroll
      for (int k = 0; k < NB; k++) {
        want[k] = valid[k] && sv_passes(x.bm, key[k], x.wlog);
        if (want[k]) want[k] = x2_find(x.pt, key[k]) < 0;
        any = any || want[k];
      }
      if (!__ballot(any)) return;
      double sv[NB];
#pragma unroll
      for (int k = 0; k < NB; k++) sv[k] = want[k] ? ld_nt(&s.sc[ri[k]], a.nt & 1u) : 0.0;
#pragma unroll
      for (int k = 0; k < NB; k++) {
        if (!__ballot(want[k])) continue;
        if (__hip_atomic_load(&x.misc[SVM_FILL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > budget) {
          if (lane_id() == 0) x.misc[SVM_OVF] = 1;
          return;
        }
        bool ins = false;
        int h = -1;
        if (want[k]) h = x2_slot(xt, key[k], ins);
        const int nins = __popcll(__ballot(ins));
        if (nins && lane_id() == 0) atomicAdd(&x.misc[SVM_FILL], nins);
        if (__ballot(want[k] && h < 0) && lane_id() == 0) x.misc[SVM_OVF] = 1;
        if (h >= 0) {
          unsigned long long lo;
          uint32_t hi;
          xs_conv(sv[k] * factor, lo, hi);
          x2_add(xt, h, lo, hi);
        }
        if (a.diag && lane_id() == 0) diag_add(a.diag, 138, (unsigned long long)__popcll(__ballot(want[k])));
      }
    });
}

// the self seed (1 - d) of v: into PT when v is a prev key, else into the sketch (pass 1)
__device__ __forceinline__ void sv_seed1(const SvLds& x, int v, double seed, uint32_t* sk) {
  const int h = x2_find(x.pt, v);
  if (h >= 0) {
    unsigned long long lo;
    uint32_t hi;
    xs_conv(seed, lo, hi);
    x2_add(x.pt, h, lo, hi);
  } else {
    sv_sketch_add(sk, v, sv_units(seed), x.wlog);
  }
}
// ... and into XT in pass 2 when v is not a prev key and passes
__device__ __forceinline__ void sv_seed2(const SvLds& x, const X2Table& xt, int v, double seed) {
  if (x2_find(x.pt, v) >= 0 || !sv_passes(x.bm, v, x.wlog)) return;
  bool ins;
  const int h = x2_slot(xt, v, ins);
  if (h < 0) { x.misc[SVM_OVF] = 1; return; }
  if (ins) atomicAdd(&x.misc[SVM_FILL], 1);
  unsigned long long lo;
  uint32_t hi;
  xs_conv(seed, lo, hi);
  x2_add(xt, h, lo, hi);
}

// sieve bitmap: bit c = counter c >= thr (one ballot per 64 counters)
template <class Get>
__device__ __forceinline__ void sv_bitmap(const SvLds& x, uint32_t thr, Get get) {
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  for (int w = wv; w < x.bm_words; w += W) {
    const uint64_t m = __ballot(get(w * 64 + lane_id()) >= thr);
    if (lane_id() == 0) x.bm[w] = m;
  }
}

// theta = the smallest of the L prev totals (value bits; every value >= 0), published in misc
template <class Val>
__device__ __forceinline__ double sv_theta(const SvLds& x, int n, Val val) {
  unsigned long long mn = ~0ull;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const unsigned long long b = dbits(val(i));
    mn = b < mn ? b : mn;
  }
  mn = wave_min_u64(mn);
  unsigned long long* th = reinterpret_cast<unsigned long long*>(&x.misc[SVM_THETA]);
  if (lane_id() == 0 && mn != ~0ull) atomicMin(th, mn);
  __syncthreads();
  return bitsd(*th);
}

__device__ __forceinline__ void sv_clear_region(const SvLds& x, size_t bytes) {
  uint4* r = reinterpret_cast<uint4*>(x.region);
  for (size_t i = threadIdx.x; i < bytes / 16; i += blockDim.x) r[i] = make_uint4(0u, 0u, 0u, 0u);
}

// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(SV_THREADS) k_sv1(DevGraph g, DevSlab s, IterArgs a, const SvDesc* desc, int d0,
                                                    int Lp, SvGeom G, int budget, int32_t* ovl, int32_t* out_k,
                                                    double* out_v, int32_t* out_n) {
  extern __shared__ __align__(16) unsigned char smem[];
  const SvLds x = sv_carve(smem, Lp, G);
  const int d = d0 + (int)blockIdx.x;
  const SvDesc sd = desc[d];
  const int v = sd.v;
  const int L = s.L;
  // (the host sends only sources with a full current row: L keys to bound with)
  if (s.len[s.lrow((a.active == 1) ? a.sB : a.sA, v)] != L) {
    if (threadIdx.x == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = d;
    return;
  }
  long long tph = a.diag ? (long long)clock64() : 0;
  uint32_t* sk = reinterpret_cast<uint32_t*>(x.region);
  sv_clear_region(x, G.sketch_bytes());
  sv_build_pt(x, s, a, v, Lp);
  __syncthreads();
  if (threadIdx.x == 0) {
    *reinterpret_cast<unsigned long long*>(&x.misc[SVM_THETA]) = ~0ull;
    sv_seed1(x, v, 1.0 - a.damping, sk);
  }
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  if (a.whatif & WI_SV_P1WALK) sv_pass1(g, s, a, x, b, e, sd.factor, sk);
  else sv_pass1b(g, s, a, x, b, e, sd.factor, sk);
  __syncthreads();
  sv_lap(a, 145, tph);
  // bound: the smallest exact total of the L prev keys
  const int Tpt = 2 * Lp;
  const double theta = sv_theta(x, Tpt, [&](int i) {
    return x.pt.keys[i] ? x2_value(x.pt.a[i], x.pt.b[i]) : bitsd(~0ull >> 1);  // (empty: above every value)
  });
  const uint32_t thr = sv_thr(theta);
  sv_bitmap(x, thr, [&](int c) { return sk[c]; });
  __syncthreads();
  const X2Table xt = x2_carve(x.region, G.xt);
  sv_clear_region(x, x2_bytes(G.xt));
  __syncthreads();
  sv_lap(a, 146, tph);
  if (threadIdx.x == 0) sv_seed2(x, xt, v, 1.0 - a.damping);
  sv_pass2(g, s, a, x, xt, b, e, sd.factor, budget);
  __syncthreads();
  sv_lap(a, 147, tph);
  if (x.misc[SVM_OVF] || x.misc[SVM_FILL] > budget + G.waves * WAVE) {
    if (threadIdx.x == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = d;
    if (a.diag && threadIdx.x == 0) diag_add(a.diag, 137, 1ull);
    return;
  }
  // dense (value, key) list of PT u {XT keys >= theta}: the table's slot values into registers
  // (SV_XS per thread), then written over the front of the region after every slot was read; the
  // PT entries (outside the region) after them
  double xv[SV_XS];
  int xk[SV_XS];
  int c = 0;
#pragma unroll
  for (int j = 0; j < SV_XS; j++) {
    const int i = (int)threadIdx.x + j * (int)blockDim.x;
    const uint32_t kt = xt.keys[i];
    const double val = kt ? x2_value(xt.a[i], xt.b[i]) : 0.0;
    xk[j] = (kt && val >= theta) ? (int)kt - 1 : -1;
    xv[j] = val;
    c += xk[j] >= 0;
  }
  const int incl = wave_incl_scan(c);
  int base = 0;
  if (lane_id() == WAVE - 1 && incl) base = atomicAdd(&x.misc[SVM_U], incl);
  base = __builtin_amdgcn_readlane(base, WAVE - 1) + incl - c;
  __syncthreads();  // every slot read
  const int cap = G.xt + Lp;
  double* dv = reinterpret_cast<double*>(x.region);
  int* dk = reinterpret_cast<int*>(x.region + (size_t)cap * 8);
#pragma unroll
  for (int j = 0; j < SV_XS; j++)
    if (xk[j] >= 0) { dv[base] = xv[j]; dk[base] = xk[j]; base++; }
  for (int i0 = 0; i0 < Tpt; i0 += blockDim.x) {
    const int i = i0 + (int)threadIdx.x;
    const bool has = i < Tpt && x.pt.keys[i] != 0u;
    const uint64_t m = __ballot(has);
    int b0 = 0;
    if (m && lane_id() == 0) b0 = atomicAdd(&x.misc[SVM_U], __popcll(m));
    b0 = __shfl(b0, 0) + __popcll(m & lanemask_lt());
    if (has) { dv[b0] = x2_value(x.pt.a[i], x.pt.b[i]); dk[b0] = (int)x.pt.keys[i] - 1; }
  }
  __syncthreads();
  const int U = x.misc[SVM_U];
  if (a.diag && threadIdx.x == 0) {
    diag_add(a.diag, 135, 1ull);
    diag_add(a.diag, 136, (unsigned long long)x.misc[SVM_FILL]);
    diag_add(a.diag, 139, (unsigned long long)(U - L));
  }
  // top-L of the dense list (every thread: a block radix select when U > L), emitted for k_svfin,
  // which writes the row at full occupancy once this LDS-heavy workgroup is gone
  const uint32_t ts = tie_salt(v);
  SelCrit sc;
  sc.tie = false; sc.pa = 0; sc.ma = 0; sc.pb = 0; sc.mb = 0;
  const bool cut = U > L;
  if (cut) {
    WgLds w = WgLds{};
    w.hist = x.hist;
    w.misc = x.misc;
    sc = wg_select_top(w, U, L, [&](int i) { return dk[i]; }, [&](int i) { return dv[i]; }, [](int) { return true; }, ts);
  }
  if (threadIdx.x == 0) x.misc[SVM_PT] = 0;
  __syncthreads();
  int32_t* ok = out_k + (int64_t)d * Lp;
  double* ov = out_v + (int64_t)d * Lp;
  for (int i0 = 0; i0 < U; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    const bool sel = i < U && (!cut || sel_test(sc, dbits(dv[i]), tie_w(dk[i], ts)));
    const uint64_t m = __ballot(sel);
    int b0 = 0;
    if (m && lane_id() == 0) b0 = atomicAdd(&x.misc[SVM_PT], __popcll(m));
    b0 = __shfl(b0, 0);
    if (sel) {
      const int pos = b0 + __popcll(m & lanemask_lt());
      ok[pos] = dk[i];
      ov[pos] = dv[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out_n[d] = x.misc[SVM_PT];
  if (threadIdx.x == 0) sv_lap(a, 148, tph);
}

// the row of a one-slice source from its selected entries (k_sv1): one wave per source -- sort in
// hash order, write, range index, norm1 against the old row, maxDiff (finish_source)
__host__ __device__ constexpr size_t svfin_lds_bytes(int Lp) { return (size_t)Lp * 12 + 1024 + (size_t)Lp * 20; }
__global__ void __launch_bounds__(64) k_svfin(DevSlab s, IterArgs a, const SvDesc* desc, int d0, const int32_t* in_k,
                                              const double* in_v, const int32_t* in_n, int Lp,
                                              unsigned long long* maxdiff, unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int d = d0 + (int)blockIdx.x;
  const int n = in_n[d];
  if (n <= 0) return;  // handed back (a written source has L >= 1 entries)
  const int v = desc[d].v;
  uint64_t* rv = reinterpret_cast<uint64_t*>(smem);
  int* rk = reinterpret_cast<int*>(smem + (size_t)Lp * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + (size_t)Lp * 12);
  int* hk = reinterpret_cast<int*>(smem + (size_t)Lp * 12 + 1024);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;
  const int32_t* ik = in_k + (int64_t)d * Lp;
  const double* iv = in_v + (int64_t)d * Lp;
  for (int i = lane_id(); i < n; i += WAVE) { rk[i] = ik[i]; rv[i] = dbits(iv[i]); }
  wave_fence();
  finish_source(v, n, [&](int i) { return rk[i]; }, [&](int i) { return bitsd(rv[i]); }, s, a, hist, rv, rk, Lp, hk, hv,
                mf, maxdiff, stats);
}

// slice k of S of the successor list [b, e)
__device__ __forceinline__ void sv_slice(int64_t b, int64_t e, int k, int S, int64_t& b0, int64_t& b1) {
  const int64_t n = e - b;
  b0 = b + n * k / S;
  b1 = b + n * (k + 1) / S;
}

__global__ void __launch_bounds__(SV_THREADS) k_svA(DevGraph g, DevSlab s, IterArgs a, const SvDesc* desc,
                                                    const SvTask* tasks, int Lp, uint32_t* gsk,
                                                    unsigned long long* gpt) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr SvGeom G = SV_LARGE;
  const SvLds x = sv_carve(smem, Lp, G);
  const SvTask tk = tasks[blockIdx.x];
  const SvDesc sd = desc[tk.d];
  const int v = sd.v;
  uint32_t* sk = reinterpret_cast<uint32_t*>(x.region);
  sv_clear_region(x, G.sketch_bytes());
  sv_build_pt(x, s, a, v, Lp);
  __syncthreads();
  if (tk.k == 0 && threadIdx.x == 0) sv_seed1(x, v, 1.0 - a.damping, sk);
  int64_t b0, b1;
  sv_slice(g.rp[v], g.rp[v + 1], tk.k, sd.S, b0, b1);
  if (a.whatif & WI_SV_P1WALK) sv_pass1(g, s, a, x, b0, b1, sd.factor, sk);
  else sv_pass1b(g, s, a, x, b0, b1, sd.factor, sk);
  __syncthreads();
  uint32_t* gs = gsk + sd.gsk;
  for (int c = threadIdx.x; c < SV_R * (1 << G.wlog); c += blockDim.x) {
    const uint32_t u = sk[c];
    if (u) atomicAdd(&gs[c], u);
  }
  unsigned long long* gp = gpt + sd.gpt;
  for (int i = threadIdx.x; i < 2 * Lp; i += blockDim.x) {
    if (!x.pt.keys[i]) continue;
    const unsigned long long A = x.pt.a[i], B = x.pt.b[i];
    const int r = x.pti[i];
    if (A) atomicAdd(&gp[2 * r], A);
    if (B) atomicAdd(&gp[2 * r + 1], B);
  }
}

// a global table slot of `key` (find-or-insert, linear probing, bounded by the table), -1 if full
__device__ __forceinline__ int64_t sv_gslot(uint32_t* keys, int64_t T, int key) {
  const uint32_t tag = (uint32_t)key + 1u;
  int64_t h = (int64_t)(hash32((uint32_t)key) & (uint32_t)(T - 1));
  for (int64_t n = 0; n < T; n++) {
    const uint32_t k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == tag) return h;
    if (k == 0u) {
      const uint32_t prev = atomicCAS(&keys[h], 0u, tag);
      if (prev == 0u || prev == tag) return h;
    }
    h = (h + 1) & (T - 1);
  }
  return -1;
}

__global__ void __launch_bounds__(SV_THREADS) k_svB(DevGraph g, DevSlab s, IterArgs a, const SvDesc* desc,
                                                    const SvTask* tasks, int Lp, int budget, const uint32_t* gsk,
                                                    const unsigned long long* gpt, uint32_t* gkeys,
                                                    unsigned long long* ga, unsigned long long* gb, int32_t* oflag) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr SvGeom G = SV_LARGE;
  const SvLds x = sv_carve(smem, Lp, G);
  const SvTask tk = tasks[blockIdx.x];
  const SvDesc sd = desc[tk.d];
  const int v = sd.v;
  const int L = s.L;
  sv_build_pt(x, s, a, v, Lp);
  __syncthreads();
  if (threadIdx.x == 0) *reinterpret_cast<unsigned long long*>(&x.misc[SVM_THETA]) = ~0ull;
  __syncthreads();
  const unsigned long long* gp = gpt + sd.gpt;
  const double theta = sv_theta(x, L, [&](int i) { return x2_value(gp[2 * i], gp[2 * i + 1]); });
  const uint32_t thr = sv_thr(theta);
  const uint32_t* gs = gsk + sd.gsk;
  sv_bitmap(x, thr, [&](int c) { return gs[c]; });
  const X2Table xt = x2_carve(x.region, G.xt);
  sv_clear_region(x, x2_bytes(G.xt));
  __syncthreads();
  if (tk.k == 0 && threadIdx.x == 0) sv_seed2(x, xt, v, 1.0 - a.damping);
  int64_t b0, b1;
  sv_slice(g.rp[v], g.rp[v + 1], tk.k, sd.S, b0, b1);
  sv_pass2(g, s, a, x, xt, b0, b1, sd.factor, budget);
  __syncthreads();
  if (x.misc[SVM_OVF] || x.misc[SVM_FILL] > budget + G.waves * WAVE) {
    if (threadIdx.x == 0) oflag[tk.d] = 1;
    return;
  }
  if (a.diag && threadIdx.x == 0) diag_add(a.diag, 136, (unsigned long long)x.misc[SVM_FILL]);
  uint32_t* gk = gkeys + sd.gxt;
  unsigned long long* gA = ga + sd.gxt;
  unsigned long long* gB = gb + sd.gxt;
  bool full = false;
  for (int i = threadIdx.x; i < G.xt; i += blockDim.x) {
    const uint32_t kt = xt.keys[i];
    if (!kt) continue;
    const int64_t h = sv_gslot(gk, sd.tg, (int)kt - 1);
    if (h < 0) { full = true; continue; }
    const unsigned long long A = xt.a[i], B = xt.b[i];
    if (A) atomicAdd(&gA[h], A);
    if (B) atomicAdd(&gB[h], B);
  }
  if (full) oflag[tk.d] = 1;
}

// k_svF LDS: dense values f64[SVF_CAP + Lp] | keys i32[SVF_CAP + Lp] | misc | finish_source scratch
__host__ __device__ constexpr size_t svf_lds_bytes(int Lp) {
  return (size_t)(SVF_CAP + Lp) * 12 + 256 + 1024 + (size_t)Lp * 32;
}
__global__ void __launch_bounds__(256) k_svF(DevSlab s, IterArgs a, const SvDesc* desc, int Lp,
                                             const unsigned long long* gpt, const uint32_t* gkeys,
                                             const unsigned long long* ga, const unsigned long long* gb,
                                             const int32_t* oflag, int32_t* ovl, unsigned long long* maxdiff,
                                             unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int d = blockIdx.x;
  const SvDesc sd = desc[d];
  const int v = sd.v;
  const int L = s.L;
  const int cap = SVF_CAP + Lp;
  unsigned char* p = smem;
  double* dv = reinterpret_cast<double*>(p); p += (size_t)cap * 8;
  int* dk = reinterpret_cast<int*>(p); p += (size_t)cap * 4;
  int* misc = reinterpret_cast<int*>(p); p += 256;
  uint32_t* hist = reinterpret_cast<uint32_t*>(p); p += 1024;
  uint64_t* rv = reinterpret_cast<uint64_t*>(p); p += (size_t)Lp * 8;
  int* rk = reinterpret_cast<int*>(p); p += (size_t)Lp * 4;
  int* hk = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  int* hv = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  int* mf = reinterpret_cast<int*>(p);
  if (oflag[d] || s.len[s.lrow((a.active == 1) ? a.sB : a.sA, v)] != L) {
    if (threadIdx.x == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = d;
    return;
  }
  if (threadIdx.x < 64) misc[threadIdx.x] = 0;
  if (threadIdx.x == 0) *reinterpret_cast<unsigned long long*>(&misc[SVM_THETA]) = ~0ull;
  __syncthreads();
  const unsigned long long* gp = gpt + sd.gpt;
  const int cur = (a.active == 1) ? a.sB : a.sA;
  const int64_t r = s.row(cur, v);
  // the L prev keys with their exact totals (all >= theta), then the table's keys >= theta
  unsigned long long mn = ~0ull;
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const double val = x2_value(gp[2 * i], gp[2 * i + 1]);
    dv[i] = val;
    dk[i] = s.key(s.ids[r + i]);
    const unsigned long long bb = dbits(val);
    mn = bb < mn ? bb : mn;
  }
  mn = wave_min_u64(mn);
  if (lane_id() == 0 && mn != ~0ull) atomicMin(reinterpret_cast<unsigned long long*>(&misc[SVM_THETA]), mn);
  if (threadIdx.x == 0) misc[SVM_U] = L;
  __syncthreads();
  const double theta = bitsd(*reinterpret_cast<unsigned long long*>(&misc[SVM_THETA]));
  const uint32_t* gk = gkeys + sd.gxt;
  const unsigned long long* gA = ga + sd.gxt;
  const unsigned long long* gB = gb + sd.gxt;
  for (int64_t i0 = 0; i0 < sd.tg; i0 += blockDim.x) {
    const int64_t i = i0 + threadIdx.x;
    bool keep = false;
    double val = 0.0;
    uint32_t kt = 0u;
    if (i < sd.tg) {
      kt = gk[i];
      if (kt) { val = x2_value(gA[i], gB[i]); keep = val >= theta; }
    }
    const uint64_t m = __ballot(keep);
    int base = 0;
    if (m && lane_id() == 0) base = atomicAdd(&misc[SVM_U], __popcll(m));
    base = __shfl(base, 0);
    const int pos = base + __popcll(m & lanemask_lt());
    if (keep && pos < cap) { dv[pos] = val; dk[pos] = (int)kt - 1; }
  }
  __syncthreads();
  const int U = misc[SVM_U];
  if (U > cap) {
    if (threadIdx.x == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = d;
    return;
  }
  if (a.diag && threadIdx.x == 0) {
    diag_add(a.diag, 149, 1ull);
    diag_add(a.diag, 139, (unsigned long long)(U - L));
  }
  if (threadIdx.x < WAVE)
    finish_source(v, U, [&](int i) { return dk[i]; }, [&](int i) { return dv[i]; }, s, a, hist, rv, rk, Lp, hk, hv,
                  mf, maxdiff, stats);
}

// gather for the sieve planning: candidates, degree, last distinct count, current row length
__global__ void __launch_bounds__(256) k_gather_sv(const int32_t* list, int64_t count, const int32_t* cand,
                                                   const int64_t* rp, const int32_t* dlast, DevSlab s, IterArgs a,
                                                   int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int v = list[i];
  out[i] = cand[v];
  out[count + i] = (int32_t)(rp[v + 1] - rp[v]);
  out[2 * count + i] = dlast[v];
  out[3 * count + i] = s.len[s.lrow((a.active == 1) ? a.sB : a.sA, v)];
}

}  // namespace pprk
