// merge_sv.h -- the sieve merge of the wide GRank sources (exact sum).
//
// A wide source (more candidates than a wave table holds) has up to millions of distinct keys, yet
// only its top-L survive the merge, and between two updates they barely change (RMAT-22, sampled
// wide sources: at iterations 20 / 21 all 128 previous top-L keys are again in the new top-L of
// 90 / 94 %, 127.9 of 128 on average; tools/sieve_stats.py, profiles/r04_sieve_workload_rmat22.json).
// The sieve uses that without trusting it:
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
constexpr size_t SV_LIST_BYTES = (size_t)WAVE * 12;  // pass-2 staging list of one wave: t f64[64] | key i32[64]
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
  // pass 2 holds XT (20 B a slot) and one 64-entry staging list per wave (sv_pass2) in the region
  __host__ __device__ constexpr size_t p2_bytes() const { return (size_t)xt * 20 + (size_t)waves * SV_LIST_BYTES; }
  __host__ __device__ constexpr size_t region() const {
    return sketch_bytes() > p2_bytes() ? sketch_bytes() : p2_bytes();
  }
};
__host__ __device__ constexpr SvGeom sv_geom(int wlog, int waves) {
  return SvGeom{wlog, waves, SV_XS * waves * WAVE, SV_XS * waves * WAVE * 85 / 100 - waves * WAVE};
}
constexpr SvGeom SV_LARGE = sv_geom(13, 16), SV_MID = sv_geom(12, 8), SV_SMALL = sv_geom(11, 4);
// (the staging lists fit beside XT in the sketch's bytes: no class grows)
static_assert(SV_LARGE.region() == SV_LARGE.sketch_bytes() && SV_MID.region() == SV_MID.sketch_bytes() &&
              SV_SMALL.region() == SV_SMALL.sketch_bytes(), "sieve LDS per class");
constexpr int SV_THREADS = 16 * WAVE;         // the widest class (multi-slice kernels)
constexpr int SV_XT_BUDGET = SV_LARGE.budget;
constexpr int SVF_CAP = 4096;                 // k_svF: dense entries at or above the bound

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
__device__ __forceinline__ double x2_value(unsigned long long A, unsigned long long B, int F = XS_F) {
  const unsigned long long lo = ((B & 0xffffffffull) << 32) + A;
  const uint32_t hi = (uint32_t)(B >> 32) + (lo < A ? 1u : 0u);
  return xs_to_double(hi, lo, F);
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
// Three multiplicative hashes of a key (Knuth: the top bits of key * an odd constant mix every key
// bit; v_mul_lo_u32 issues at the VALU's full rate on gfx950, tools/valu_rates.hip). h0's top bits
// place the key in PT (a multiply-high by the group count); the top wlog bits of h0, h1 and h2 are its
// three sketch cells -- one shift each, no bit-field mixing (round 6: the old 24-bit mixer and its
// three bit fields took 16 VALU instructions of a pass-1 group, these take 6). Independent of hash_b,
// which orders the stored rows; the hashes' quality only moves the false-positive rate, never the
// result.
struct SvHash {
  uint32_t h0, h1, h2;
};
__device__ __forceinline__ SvHash sv_hash(int key) {
  const uint32_t k = (uint32_t)key;
  return SvHash{k * 0x9E3779B1u, k * 0x85EBCA77u, k * 0xC2B2AE3Du};
}
// an upper bound of p * 2^31 in counter units, from fl(p * 2^31) = fl(s * (f * 2^31)) (a
// power-of-two scale commutes with the rounding; below the normal range both round to < 1 unit):
// floor + 1 > p * 2^31. GRank contributions are <= 1: no saturation.
__device__ __forceinline__ uint32_t sv_units31(double p31) { return (uint32_t)p31 + 1u; }
__device__ __forceinline__ uint32_t sv_units(double p) { return sv_units31(p * 0x1p31); }
// counter threshold of the bound theta: a key whose total reaches theta has every counter >=
// 2^31 * theta * (1 - 2^-52) (its stored value rounds up by at most half an ulp); the margin
// below makes the test conservative (a counter at the threshold passes)
__device__ __forceinline__ uint32_t sv_thr(double theta) {
  const double x = floor(ldexp(theta, SV_UNIT_LOG) * (1.0 - 0x1p-40));
  return x <= 0.0 ? 0u : x >= 4294967295.0 ? 0xffffffffu : (uint32_t)x;
}
// the key's three counters (row j: counters (j << wlog) + top wlog bits of h_j)
__device__ __forceinline__ void sv_sketch_add(uint32_t* sk, const SvHash& hs, uint32_t u, int wlog) {
  const int sh = 32 - wlog;
  atomicAdd(&sk[hs.h0 >> sh], u);
  atomicAdd(&sk[(1u << wlog) + (hs.h1 >> sh)], u);
  atomicAdd(&sk[(2u << wlog) + (hs.h2 >> sh)], u);
}
// every counter of the key at or above the threshold (bitmap of the counters that are; the three
// words are read together). Counter c = h >> sh is bit c & 31 of word c >> 5 = h >> (sh + 5); the
// 32-bit shift by c takes its low five bits by itself.
__device__ __forceinline__ bool sv_passes(const uint32_t* bm, const SvHash& hs, int wlog) {
  const int sh = 32 - wlog;
  const int rw = (1 << wlog) >> 5;  // bitmap words per row
  const uint32_t w0 = bm[hs.h0 >> (sh + 5)];
  const uint32_t w1 = bm[rw + (hs.h1 >> (sh + 5))];
  const uint32_t w2 = bm[2 * rw + (hs.h2 >> (sh + 5))];
  return ((w0 >> ((hs.h0 >> sh) & 31u)) & (w1 >> ((hs.h1 >> sh) & 31u)) & (w2 >> ((hs.h2 >> sh) & 31u)) & 1u) != 0u;
}
// The split accumulator's two addends of one contribution p = fl(s * f), from t = p * 2^61:
// X = floor(p * 2^93) (merge_xs.h xs_conv), A = X mod 2^32, B = X >> 32 = floor(t). t is exact
// (a power-of-two scale), and so is t = fl(s * (f * 2^61)) -- rounding commutes with the scale
// (for p below 2^-93, where the two could differ in the subnormal range, X = 0 either way). No
// integer shifts and no branches: B's words are two truncating conversions, and t - B < 2^32 and
// its fraction are exact (they are multiples of ulp(t)), so A = trunc(frac(t) * 2^32).
__device__ __forceinline__ void sv_split_t(double t, unsigned long long& A, unsigned long long& B) {
  const uint32_t bh = (uint32_t)(t * 0x1p-32);                    // t <= 2^61 (p <= 1)
  const uint32_t bl = (uint32_t)fma(-(double)bh, 0x1p32, t);      // t - bh 2^32 in [0, 2^32), exact
  A = (unsigned long long)(uint32_t)(__builtin_amdgcn_fract(t) * 0x1p32);  // frac(t) 2^32 < 2^32
  B = ((unsigned long long)bh << 32) | bl;
}
// accumulators of slot i at ab[2 i] (A) and ab[2 i + 1] (B): one address, the second add at +8
__device__ __forceinline__ void sv_split_add_t(unsigned long long* ab, int i, double t) {
  unsigned long long A, B;
  sv_split_t(t, A, B);
  atomicAdd(&ab[2 * i], A);
  atomicAdd(&ab[2 * i + 1], B);
}
__device__ __forceinline__ void sv_split_add(unsigned long long* ab, int i, double p) {
  sv_split_add_t(ab, i, p * 0x1p61);
}
// (XT: separate A and B arrays)
__device__ __forceinline__ void sv_split_add_t(unsigned long long* a, unsigned long long* b, int i, double t) {
  unsigned long long A, B;
  sv_split_t(t, A, B);
  atomicAdd(&a[i], A);
  atomicAdd(&b[i], B);
}
__device__ __forceinline__ void sv_split_add(unsigned long long* a, unsigned long long* b, int i, double p) {
  sv_split_add_t(a, b, i, p * 0x1p61);
}

// ---------------------------------------------------------------------------------------------
// PT: the L keys of the source's current row, in T = 4 Lp slots probed as aligned groups of four
// (one ds_read_b128 from the key's home group: load 1/4, so a home group rarely fills). A key that
// found its home group full sits in the next group with room, and bit 31 of the home group's first
// tag word says so -- a lookup continues past its home group only then (< 1 % of the groups; keys
// and their tags (key + 1) stay below 2^31). Accumulators are indexed by slot (slots T .. T + 63: the
// per-lane dummies of the round-4 branch-free pass 1, kept in the layout, no longer written).
struct SvPt {
  uint32_t* keys;            // [T] key + 1 (0 = empty); bit 31 of word 4 g: home group g overflowed
  unsigned long long* ab;    // [2 (T + 64)] split accumulators of slot i: A at 2 i (low 32 bits of each
                             // X_i), B at 2 i + 1 (X_i >> 32)
  int* pos;                  // [T] row position of the slot's key
  int T;
  uint32_t gmask;            // T / 4 - 1
};
__host__ __device__ constexpr size_t svpt_bytes(int Lp) { return (size_t)4 * Lp * 24 + 64 * 16; }
__device__ __forceinline__ SvPt svpt_carve(unsigned char* p, int Lp) {
  SvPt t;
  t.T = 4 * Lp;
  t.ab = reinterpret_cast<unsigned long long*>(p); p += (size_t)(t.T + 64) * 16;
  t.keys = reinterpret_cast<uint32_t*>(p); p += (size_t)t.T * 4;
  t.pos = reinterpret_cast<int*>(p);
  t.gmask = (uint32_t)(t.T / 4) - 1u;
  return t;
}
constexpr uint32_t SV_OVF_BIT = 0x80000000u;
// first slot of the home group of a key with hash h0: its top bits times the slot count, rounded
// down to the group (a multiply-high and a mask)
__device__ __forceinline__ uint32_t svpt_home(const SvPt& t, uint32_t h0) { return __umulhi(h0, (uint32_t)t.T) & ~3u; }
// the slot of tag past its home group g4 (the group overflowed): groups in order until the tag or
// an empty slot (the key would have taken it)
__device__ __forceinline__ int svpt_find_from(const SvPt& t, uint32_t tag, uint32_t g4) {
  for (int n = 0; n < (int)t.gmask + 1; n++) {
    g4 = (g4 + 4u) & (uint32_t)(t.T - 1);
    const uint4 q = *reinterpret_cast<const uint4*>(t.keys + g4);
    const uint32_t x = q.x & ~SV_OVF_BIT;
    if (x == tag) return (int)g4;
    if (q.y == tag) return (int)g4 + 1;
    if (q.z == tag) return (int)g4 + 2;
    if (q.w == tag) return (int)g4 + 3;
    if (x == 0u || q.y == 0u || q.z == 0u || q.w == 0u) return -1;
  }
  return -1;
}
// the PT slot of `key` (hash h) or -1; `active` lanes only take the rare continuation. Wave-wide:
// every lane of the wave must call it (one ballot).
__device__ __forceinline__ int svpt_slot(const SvPt& t, int key, uint32_t h, bool active) {
  const uint32_t tag = (uint32_t)key + 1u;
  const uint32_t g4 = svpt_home(t, h);
  const uint4 q = *reinterpret_cast<const uint4*>(t.keys + g4);
  int m = q.w == tag ? 3 : -1;
  m = q.z == tag ? 2 : m;
  m = q.y == tag ? 1 : m;
  m = (q.x & ~SV_OVF_BIT) == tag ? 0 : m;
  int slot = m >= 0 ? (int)g4 + m : -1;
  const bool more = active && m < 0 && (q.x & SV_OVF_BIT);
  if (__builtin_expect(__ballot(more) != 0ull, 0)) {
    if (more) slot = svpt_find_from(t, tag, g4);
  }
  return slot;
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
//   region (sketch in pass 1; XT in pass 2; dense (value, key) list in the select) | PT (svpt_bytes)
//   | bitmap u64[bm_words] | misc i32[64] | hist u32[256] (block select)
enum { SVM_FILL = 0, SVM_OVF = 1, SVM_U = 2, SVM_PT = 3, SVM_ROWS = 4, SVM_THETA = 8 /* u64: 8..9 */ };
__host__ __device__ constexpr size_t sv_lds_bytes(int Lp, SvGeom G) {
  return G.region() + svpt_bytes(Lp) + (size_t)G.bm_words() * 8 + 256 + 1024;
}
struct SvLds {
  unsigned char* region;
  SvPt pt;
  uint64_t* bm;
  int* misc;
  uint32_t* hist;
  int wlog;
  int bm_words;
};
__device__ __forceinline__ SvLds sv_carve(unsigned char* smem, int Lp, SvGeom G) {
  SvLds x;
  unsigned char* p = smem;
  x.region = p; p += G.region();
  x.pt = svpt_carve(p, Lp); p += svpt_bytes(Lp);
  x.bm = reinterpret_cast<uint64_t*>(p); p += (size_t)G.bm_words() * 8;
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

// the current row of v (L distinct keys) into PT with zeroed sums (dummies included); misc cleared
__device__ __forceinline__ void sv_build_pt(const SvLds& x, const DevSlab& s, const IterArgs& a, int v, int Lp) {
  const SvPt& t = x.pt;
  for (int i = threadIdx.x; i < t.T; i += blockDim.x) t.keys[i] = 0u;
  for (int i = threadIdx.x; i < 2 * (t.T + 64); i += blockDim.x) t.ab[i] = 0ull;
  if (threadIdx.x < 64) x.misc[threadIdx.x] = 0;
  __syncthreads();
  const int cur = (a.active == 1) ? a.sB : a.sA;
  const int64_t r = s.row(cur, v);
  const int len = s.len[s.lrow(cur, v)];
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    const int key = s.key(s.ids[r + i]);
    const uint32_t tag = (uint32_t)key + 1u;
    const uint32_t home = svpt_home(t, sv_hash(key).h0);
    uint32_t g4 = home;
    for (int n = 0; n <= (int)t.gmask; n++) {  // (T = 4 L slots: a free slot always exists)
      int got = -1;
#pragma unroll
      for (int j = 0; j < 4 && got < 0; j++)
        if (atomicCAS(&t.keys[g4 + j], 0u, tag) == 0u) got = (int)g4 + j;
      if (got >= 0) { t.pos[got] = i; break; }
      if (g4 == home) atomicOr(&t.keys[home], SV_OVF_BIT);  // (its first word is taken: never reads 0)
      g4 = (g4 + 4u) & (uint32_t)(t.T - 1);
    }
  }
}

// The wave's share of a slice: contiguous successors [c0, c1) taken row by row. Row metadata comes
// per window of 64 successors, one successor per lane (colx two windows ahead, lengths one window
// ahead); a row's base and length are read off its lane into scalar registers. A lane takes
// entries lane and 64 + lane of each row (rows of up to 128 entries: the sieve takes L <= 128,
// grank.hip sv_enabled), loads issued unconditionally inside the row (a row slot always
// holds L entries: lanes past the row's length read stale entries and are masked, no exec branch).
// NS rows a batch, the next batch's loads in flight while fb(key, score, valid) takes the current
// batch's groups; scores are loaded only with kScores. Every branch here is wave-uniform.
template <int NS>
struct SvBatch {
  int key[2 * NS];
  double sv[2 * NS];
  int rl[NS];        // row length (0: no row)
  int64_t base[NS];
};
// every group of a batch that holds entries: g(k, key, score, valid, slab index)
template <int NS, class G>
__device__ __forceinline__ void sv_groups(const SvBatch<NS>& bt, G g) {
  const int lane = lane_id();
#pragma unroll
  for (int k = 0; k < 2 * NS; k++) {
    const int rl = bt.rl[k >> 1];
    if ((k & 1) && rl <= WAVE) continue;  // (wave-uniform; a missing row, rl = 0, has no valid lane)
    g(k, bt.key[k], bt.sv[k], (k & 1) * WAVE + lane < rl, bt.base[k >> 1] + (k & 1) * WAVE + lane);
  }
}
__device__ __forceinline__ int64_t sv_readlane64(int64_t x, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// `succ(ln, rmin_bits)` (optional, merge_wave.h WalkRowMin) sees every successor's basket length and
// row minimum once (the minimum loaded beside the length, one window ahead)
template <bool kScores, int NS, class FB, class RM = WalkNoSucc>
__device__ __forceinline__ void sv_rows(const DevGraph& g, const DevSlab& s, const IterArgs& a, int64_t c0, int64_t c1,
                                        FB fb, RM succ = RM{}) {
  const int lane = lane_id();
  const int lcl = lane < s.L ? lane : 0;  // (rows narrower than a wave: stay inside the row slot)
  // second-half lane, clamped inside the row slot (L < 128: lanes past L would read the next row,
  // past the slab's end for its last row)
  const int lhi = WAVE + lane < s.L ? WAVE + lane : lcl;
  auto colx_at = [&](int64_t w0) { return w0 + lane < c1 ? g.colx[w0 + lane] : (int32_t)-1; };
  auto len_of = [&](int32_t cx) { return cx == -1 ? 0 : s.len[s.lrow(read_slot(a, cx), cx & 0x7fffffff)]; };
  auto base_of = [&](int32_t cx) { return cx == -1 ? (int64_t)0 : s.row(read_slot(a, cx), cx & 0x7fffffff); };
  auto rmin_of = [&](int32_t cx) {
    return cx == -1 ? 0ull : dbits(s.rmin[s.lrow(read_slot(a, cx), cx & 0x7fffffff)]);
  };
  int32_t ncx = colx_at(c0);
  int32_t nncx = c0 + WAVE < c1 ? colx_at(c0 + WAVE) : -1;
  int nln = len_of(ncx);
  unsigned long long nrm = RM::kWant ? rmin_of(ncx) : 0ull;
  for (int64_t w0 = c0; w0 < c1; w0 += WAVE) {
    const int32_t cx = ncx;
    const int ln = nln;
    if (RM::kWant) succ(ln, nrm);
    const int64_t base = base_of(cx);
    ncx = nncx;
    if (w0 + 2 * WAVE < c1) nncx = colx_at(w0 + 2 * WAVE);
    nln = len_of(ncx);
    if (RM::kWant) nrm = rmin_of(ncx);
    const int nrows = (int)min((int64_t)WAVE, c1 - w0);
    auto load = [&](int q0, SvBatch<NS>& bt) {
#pragma unroll
      for (int q = 0; q < NS; q++) {
        const bool has = q0 + q < nrows;
        const int qq = has ? q0 + q : 0;
        bt.rl[q] = has ? __builtin_amdgcn_readlane(ln, qq) : 0;
        bt.base[q] = has ? sv_readlane64(base, qq) : (int64_t)0;  // (row 0: a valid address)
        bt.key[2 * q] = s.ids[bt.base[q] + lcl];
        if (kScores) bt.sv[2 * q] = s.sc[bt.base[q] + lcl];
        // the second half is loaded unconditionally (a row of <= 64 entries re-reads its first
        // half's lines, and sv_groups skips it): with a load count that does not depend on the
        // row lengths the compiler's vmcnt waits can count the next batch's loads exactly (a
        // branch around the load made it merge both paths and wait for half of the prefetch)
        const int i2 = bt.rl[q] > WAVE ? lhi : lcl;
        bt.key[2 * q + 1] = s.ids[bt.base[q] + i2];
        if (kScores) bt.sv[2 * q + 1] = s.sc[bt.base[q] + i2];
      }
    };
    auto run = [&](const SvBatch<NS>& bt) { fb(bt); };
    // two batch buffers in turn (no per-batch copy of one into the other); sched_barrier keeps the
    // next batch's loads ahead of this batch's work without pulling its first uses up
    // The loads are issued unconditionally (a batch past the window's rows loads row 0 of the slab
    // and has no valid lane): every path through the loop issues the same loads in the same order,
    // so the compiler's vmcnt waits count the batch in flight exactly instead of merging in a path
    // without it (which made it wait for the whole prefetch before the last groups of a batch).
    SvBatch<NS> ba, bb;
    load(0, ba);
    for (int q0 = 0; q0 < nrows; q0 += 2 * NS) {
      load(q0 + NS, bb);
      __builtin_amdgcn_sched_barrier(0);
      run(ba);
      __builtin_amdgcn_sched_barrier(0);
      if (q0 + NS >= nrows) break;
      load(q0 + 2 * NS, ba);
      __builtin_amdgcn_sched_barrier(0);
      run(bb);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// the wave's contiguous successor chunk of [b0, b1), as wave-uniform (scalar) bounds
__device__ __forceinline__ int64_t sv_uniform(int64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void sv_chunk(int64_t b0, int64_t b1, int64_t& c0, int64_t& c1) {
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const int64_t chunk = (b1 - b0 + W - 1) / W;
  c0 = sv_uniform(b0 + (int64_t)wv * chunk);
  c1 = sv_uniform(min(b1, c0 + chunk));
}

// pass 1 over successors [b0, b1): prev keys exactly into PT, every other key into the sketch.
// Per group: the PT probe for every lane, then the split add for the PT lanes and the sketch adds
// for the others, each under its lane mask.
#ifndef PPR_SV_NS1
#define PPR_SV_NS1 4
#endif
#ifndef PPR_SV_NS2
#define PPR_SV_NS2 4
#endif
#ifndef PPR_SV_P2_SCORES
#define PPR_SV_P2_SCORES 0
#endif
// pass 2 loads keys only (4 B per candidate): the staging list keeps a passing candidate's slab
// index and its score is gathered when the list is flushed, one memory latency per 64 passing
// candidates (round 5: 1344-1355 -> 1337-1338 ms per job against loading every score with its key,
// which paid before the list, when each inserting group waited for its own score)
constexpr bool SV_P2_SCORES = PPR_SV_P2_SCORES != 0;
// timing-only build switches (tools/build_variant.py; round 6: build-time instead of PPR_WHATIF bits,
// whose per-group test cost pass 2 a branch in every group)
#ifndef PPR_SV_WALK_ONLY
#define PPR_SV_WALK_ONLY 0
#endif
#ifndef PPR_SV_NO_INSERT
#define PPR_SV_NO_INSERT 0
#endif
// rows per batch in pass 1 (keys and scores) and pass 2 (keys only: a lighter group, so more rows
// in flight to cover the gather latency); build-time knobs for A/B variants (tools/build_variant.py)
constexpr int SV_NS1 = PPR_SV_NS1, SV_NS2 = PPR_SV_NS2;
__device__ __forceinline__ void sv_pass1(const DevGraph& g, const DevSlab& s, const IterArgs& a, const SvLds& x,
                                         int64_t b0, int64_t b1, double factor, uint32_t* sk) {
  int64_t c0, c1;
  sv_chunk(b0, b1, c0, c1);
  const double f61 = factor * 0x1p61, f31 = factor * 0x1p31;
  sv_rows<true, SV_NS1>(g, s, a, c0, c1, [&](const SvBatch<SV_NS1>& bt) {
    sv_groups(bt, [&](int, int key, double sc, bool valid, int64_t) {
      const SvHash hs = sv_hash(key);
      const int slot = svpt_slot(x.pt, key, hs.h0, valid);
      const bool inpt = valid && slot >= 0;
      // exec-masked adds (round 5: 1335-1341 -> 1320-1324 ms per job against the branch-free form
      // that sent non-PT lanes to per-lane dummy slots and PT lanes' zero units to the sketch)
      if (inpt) sv_split_add_t(x.pt.ab, slot, sc * f61);  // (t = p * 2^61, exact: sv_split_t)
      if (valid && !inpt) sv_sketch_add(sk, hs, sv_units31(sc * f31), x.wlog);
    });
  });
}

// pass 2 over successors [b0, b1): keys outside PT that pass the sieve, exactly into XT (budget
// checked before every insert step; past it the workgroup only flags the overflow). Per group the
// sieve test (three bitmap words) for every lane without a branch. A passing lane is rare -- but
// about half of the groups hold one (RMAT-22: 8.2e8 of 1.66e9 groups per job), and inserting
// group by group ran the PT check, the find-or-insert and the adds with one or two live lanes of
// 64. So the passing candidates (key, p * 2^61) are appended to the wave's 64-entry staging list
// in LDS (one ballot and a store per group) and inserted 64 at a time, every lane busy
// (sv_list_flush). A batch with more passing lanes than the list holds inserts group by group
// (PPR_SV_LIST=0: always).
#ifndef PPR_SV_LIST
#define PPR_SV_LIST 1
#endif
// insert `n` (<= 64) candidates (key, t = p * 2^61) of the wave into XT: PT keys skipped
__device__ __forceinline__ void sv_insert(const SvLds& x, const X2Table& xt, const IterArgs& a, bool live, int key,
                                          double t, int budget) {
  const int lane = lane_id();
  const bool w = live && svpt_slot(x.pt, key, sv_hash(key).h0, live) < 0;
  if (!__ballot(w)) return;
  if (a.diag && lane == 0) diag_add(a.diag, 148, 1ull);
  if (__hip_atomic_load(&x.misc[SVM_FILL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > budget) {
    if (lane == 0) x.misc[SVM_OVF] = 1;
    return;
  }
  bool ins = false;
  int hs = -1;
  if (w) hs = x2_slot(xt, key, ins);
  const int nins = __popcll(__ballot(ins));
  if (nins && lane == 0) atomicAdd(&x.misc[SVM_FILL], nins);
  if (__ballot(w && hs < 0) && lane == 0) x.misc[SVM_OVF] = 1;
  if (hs >= 0) sv_split_add_t(xt.a, xt.b, hs, t);
  if (a.diag && lane == 0) diag_add(a.diag, 138, (unsigned long long)__popcll(__ballot(w)));
}
__device__ __forceinline__ void sv_pass2(const DevGraph& g, const DevSlab& s, const IterArgs& a, const SvLds& x,
                                         const X2Table& xt, int64_t b0, int64_t b1, double factor, int budget) {
  int64_t c0, c1;
  sv_chunk(b0, b1, c0, c1);
  const uint32_t* bm32 = reinterpret_cast<const uint32_t*>(x.bm);
  const double f61 = factor * 0x1p61;
  const int lane = lane_id();
  const uint64_t lt = lanemask_lt();
  // the wave's staging list, past XT in the region (SvGeom::p2_bytes)
  double* lst = reinterpret_cast<double*>(x.region + (size_t)(xt.mask + 1u) * 20 + (size_t)(threadIdx.x >> 6) * SV_LIST_BYTES);
  int* lsk = reinterpret_cast<int*>(lst + WAVE);
  int nl = 0;  // (wave-uniform) entries in the list
  // A full list is flushed in two steps. `issue` moves it into registers (key, and the score gather
  // from its slab index, in flight) and frees the list; `complete` inserts those entries at the top
  // of the next batch, after that batch's successor loads were issued. The gather is then never the
  // youngest load when its result is used, so its wait leaves the walk's prefetch in flight (used
  // at once, it was: in-order vmcnt made every flush drain the pipeline).
  int pn = 0;        // (wave-uniform) entries pending
  int pk = 0;        // this lane's pending key
  double pt = 0.0;   // its score (or t, with the pass's score loads)
  auto issue = [&]() {
    wave_fence();
    const bool live = lane < nl;
    pk = live ? lsk[lane] : 0;
    if (SV_P2_SCORES) pt = lst[lane];
    else pt = s.sc[live ? __double_as_longlong(lst[lane]) : 0ll];  // (dead lanes: slab entry 0)
    pn = nl;
    nl = 0;
    wave_fence();
  };
  auto complete = [&]() {
    if (pn) {
      sv_insert(x, xt, a, lane < pn, pk, SV_P2_SCORES ? pt : pt * f61, budget);
      pn = 0;
    }
  };
  sv_rows<SV_P2_SCORES, SV_NS2>(g, s, a, c0, c1, [&](const SvBatch<SV_NS2>& bt) {
    constexpr int NG = 2 * SV_NS2;
    complete();
    bool want[NG];
    int tot = 0;
#pragma unroll
    for (int k = 0; k < NG; k++) want[k] = false;
    sv_groups(bt, [&](int k, int key, double, bool valid, int64_t) {
      // (PPR_SV_WALK_ONLY build, timing only: the walk alone, every key fails the test)
      want[k] = valid && (PPR_SV_WALK_ONLY ? key == -7 : sv_passes(bm32, sv_hash(key), x.wlog));
      tot += __popcll(__ballot(want[k]));
    });
    if (a.diag && lane == 0) {  // (PPR_DIAG: groups walked)
      int ng = 0;
#pragma unroll
      for (int k = 0; k < NG; k++) { ng += ((k & 1) ? bt.rl[k >> 1] > WAVE : bt.rl[k >> 1] > 0) ? 1 : 0; }
      diag_add(a.diag, 190, (unsigned long long)ng);
    }
    if (__builtin_expect(tot == 0, 1)) return;
    if (PPR_SV_NO_INSERT) return;  // (timing-only build: no insert path)
    if (a.diag && lane == 0) {
      int np = 0;
#pragma unroll
      for (int k = 0; k < NG; k++) np += __ballot(want[k]) ? 1 : 0;
      diag_add(a.diag, 147, (unsigned long long)np);
    }
    if (PPR_SV_LIST && tot <= WAVE) {
      if (nl + tot > WAVE) issue();  // (nothing pending: complete() ran at the top of this batch)
#pragma unroll
      for (int k = 0; k < NG; k++) {
        const uint64_t m = __ballot(want[k]);
        if (!m) continue;
        if (want[k]) {
          const int pos = nl + __popcll(m & lt);
          lsk[pos] = bt.key[k];
          lst[pos] = SV_P2_SCORES ? bt.sv[k] * f61
                                  : __longlong_as_double((long long)(bt.base[k >> 1] + (k & 1) * WAVE + lane));
        }
        nl += __popcll(m);
      }
      return;
    }
    // a batch with more passing lanes than the list holds: group by group
#pragma unroll
    for (int k = 0; k < NG; k++) {
      if (!__ballot(want[k])) continue;
      const double sc = SV_P2_SCORES ? bt.sv[k] : (want[k] ? s.sc[bt.base[k >> 1] + (k & 1) * WAVE + lane] : 0.0);
      sv_insert(x, xt, a, want[k], bt.key[k], sc * f61, budget);
    }
  });
  complete();
  if (nl) {
    issue();
    complete();
  }
}

// the self seed (1 - d) of v: into PT when v is a prev key, else into the sketch (pass 1; one thread)
__device__ __forceinline__ int svpt_slot1(const SvPt& t, int key) {
  const uint32_t tag = (uint32_t)key + 1u;
  const uint32_t g4 = svpt_home(t, sv_hash(key).h0);
  const uint4 q = *reinterpret_cast<const uint4*>(t.keys + g4);
  if ((q.x & ~SV_OVF_BIT) == tag) return (int)g4;
  if (q.y == tag) return (int)g4 + 1;
  if (q.z == tag) return (int)g4 + 2;
  if (q.w == tag) return (int)g4 + 3;
  return (q.x & SV_OVF_BIT) ? svpt_find_from(t, tag, g4) : -1;
}
__device__ __forceinline__ void sv_seed1(const SvLds& x, int v, double seed, uint32_t* sk) {
  const int h = svpt_slot1(x.pt, v);
  if (h >= 0) sv_split_add(x.pt.ab, h, seed);
  else sv_sketch_add(sk, sv_hash(v), sv_units(seed), x.wlog);
}
// ... and into XT in pass 2 when v is not a prev key and passes
__device__ __forceinline__ void sv_seed2(const SvLds& x, const X2Table& xt, int v, double seed) {
  if (svpt_slot1(x.pt, v) >= 0 || !sv_passes(reinterpret_cast<const uint32_t*>(x.bm), sv_hash(v), x.wlog)) return;
  bool ins;
  const int h = x2_slot(xt, v, ins);
  if (h < 0) { x.misc[SVM_OVF] = 1; return; }
  if (ins) atomicAdd(&x.misc[SVM_FILL], 1);
  sv_split_add(xt.a, xt.b, h, seed);
}

// sieve bitmap: bit c = counter c >= thr (one ballot per 64 counters); misc[SVM_ROWS] bit j = row j
// has a set bit (a row without one proves that no key outside PT passes: pass 2 is skipped)
template <class Get>
__device__ __forceinline__ void sv_bitmap(const SvLds& x, uint32_t thr, Get get) {
  const int W = blockDim.x >> 6, wv = threadIdx.x >> 6;
  const int per_row = x.bm_words / SV_R;
  int rows = 0;
  for (int w = wv; w < x.bm_words; w += W) {
    const uint64_t m = __ballot(get(w * 64 + lane_id()) >= thr);
    if (lane_id() == 0) x.bm[w] = m;
    if (m) rows |= 1 << (w / per_row);
  }
  if (lane_id() == 0 && rows) atomicOr(&x.misc[SVM_ROWS], rows);
}
__device__ __forceinline__ bool sv_rows_all(const SvLds& x) { return x.misc[SVM_ROWS] == (1 << SV_R) - 1; }

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

// entries per one-slice source in the k_sv1 -> k_svfin lists: a source with at most this many
// kept entries emits them unselected and k_svfin (one 5-KB wave) selects its top-L, so the
// workgroup's table is released before the select (round 6, as the wave tier's k_wfin)
#ifndef PPR_SV_OSTRIDE_X
#define PPR_SV_OSTRIDE_X 2
#endif
__host__ __device__ constexpr int sv_ostride(int Lp) { return PPR_SV_OSTRIDE_X * Lp; }

// ---------------------------------------------------------------------------------------------
// one source (descriptor d) of a one-slice class, the whole workgroup; a source that overflows
// (or has no full row) goes to `ovl` and writes nothing
__device__ __forceinline__ void sv1_source(unsigned char* smem, DevGraph g, DevSlab s, IterArgs a, const int32_t* vid,
                                           int d, int Lp, SvGeom G, int budget, int32_t* ovl, int32_t* out_k,
                                           double* out_v, int32_t* out_n) {
  const SvLds x = sv_carve(smem, Lp, G);
  const int v = vid[d];
  const int L = s.L;
  // (the host sends only sources with a full current row: L keys to bound with)
  if (s.len[s.lrow((a.active == 1) ? a.sB : a.sA, v)] != L) {
    if (threadIdx.x == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = d;
    return;
  }
  long long tph = a.diag ? (long long)clock64() : 0;
  // PPR_DIAG per size class: 256 + 8 class + {setup, pass 1, bound, pass 2, select, sources, rows, handed back}
  const int dg = 256 + 8 * (G.wlog == 13 ? 0 : G.wlog == 12 ? 1 : 2);
  uint32_t* sk = reinterpret_cast<uint32_t*>(x.region);
  sv_clear_region(x, G.sketch_bytes());
  sv_build_pt(x, s, a, v, Lp);
  __syncthreads();
  if (threadIdx.x == 0) {
    *reinterpret_cast<unsigned long long*>(&x.misc[SVM_THETA]) = ~0ull;
    sv_seed1(x, v, 1.0 - a.damping, sk);
  }
  sv_lap(a, dg + 0, tph);
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = merge_factor(a, e - b);
  sv_pass1(g, s, a, x, b, e, factor, sk);
  __syncthreads();
  sv_lap(a, dg + 1, tph);
  // bound: the smallest exact total of the L prev keys
  const int Tpt = x.pt.T;
  const double theta = sv_theta(x, Tpt, [&](int i) {
    return (x.pt.keys[i] & ~SV_OVF_BIT) ? x2_value(x.pt.ab[2 * i], x.pt.ab[2 * i + 1]) : bitsd(~0ull >> 1);  // (empty: above every value)
  });
  const uint32_t thr = sv_thr(theta);
  sv_bitmap(x, thr, [&](int c) { return sk[c]; });
  __syncthreads();
  const X2Table xt = x2_carve(x.region, G.xt);
  sv_clear_region(x, x2_bytes(G.xt));
  __syncthreads();
  sv_lap(a, dg + 2, tph);
  // a sketch row with no counter at or above thr: no key outside PT can pass, pass 2 would insert
  // nothing (exact skip)
  if (sv_rows_all(x) || (a.whatif & WI_SV_NO_P2SKIP)) {
    if (threadIdx.x == 0) sv_seed2(x, xt, v, 1.0 - a.damping);
    sv_pass2(g, s, a, x, xt, b, e, factor, budget);
    __syncthreads();
  } else if (a.diag && threadIdx.x == 0) {
    diag_add(a.diag, 145, 1ull);
  }
  sv_lap(a, dg + 3, tph);
  if (a.diag && threadIdx.x == 0) { diag_add(a.diag, dg + 5, 1ull); diag_add(a.diag, dg + 6, (unsigned long long)(e - b)); }
  if (x.misc[SVM_OVF] || x.misc[SVM_FILL] > budget + G.waves * WAVE) {
    if (threadIdx.x == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = d;
    if (a.diag && threadIdx.x == 0) { diag_add(a.diag, 137, 1ull); diag_add(a.diag, dg + 7, 1ull); }
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
    const uint32_t kt = i < Tpt ? (x.pt.keys[i] & ~SV_OVF_BIT) : 0u;
    const bool has = kt != 0u;
    const uint64_t m = __ballot(has);
    int b0 = 0;
    if (m && lane_id() == 0) b0 = atomicAdd(&x.misc[SVM_U], __popcll(m));
    b0 = __shfl(b0, 0) + __popcll(m & lanemask_lt());
    if (has) { dv[b0] = x2_value(x.pt.ab[2 * i], x.pt.ab[2 * i + 1]); dk[b0] = (int)kt - 1; }
  }
  __syncthreads();
  const int U = x.misc[SVM_U];
  if (a.diag && threadIdx.x == 0) {
    diag_add(a.diag, 135, 1ull);
    diag_add(a.diag, 136, (unsigned long long)x.misc[SVM_FILL]);
    diag_add(a.diag, 139, (unsigned long long)(U - L));
    if (U == L) diag_add(a.diag, 146, 1ull);
  }
  // top-L of the dense list (every thread: a block radix select when U > L), emitted for k_svfin,
  // which writes the row at full occupancy once this LDS-heavy workgroup is gone
  const uint32_t ts = tie_salt(v);
  SelCrit sc;
  sc.tie = false; sc.pa = 0; sc.ma = 0; sc.pb = 0; sc.mb = 0;
  const bool cut = U > sv_ostride(Lp);  // (else k_svfin selects: every kept entry goes to the list)
  if (cut) {
    WgLds w = WgLds{};
    w.hist = x.hist;
    w.misc = x.misc;
    sc = wg_select_top(w, U, L, [&](int i) { return dk[i]; }, [&](int i) { return dv[i]; }, [](int) { return true; }, ts);
  }
  if (threadIdx.x == 0) x.misc[SVM_PT] = 0;
  __syncthreads();
  int32_t* ok = out_k + (int64_t)d * sv_ostride(Lp);
  double* ov = out_v + (int64_t)d * sv_ostride(Lp);
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
  if (threadIdx.x == 0) sv_lap(a, dg + 4, tph);
}

__global__ void __launch_bounds__(SV_THREADS) k_sv1(DevGraph g, DevSlab s, IterArgs a, const int32_t* vid, int d0,
                                                    int Lp, SvGeom G, int budget, int32_t* ovl, int32_t* out_k,
                                                    double* out_v, int32_t* out_n) {
  extern __shared__ __align__(16) unsigned char smem[];
  sv1_source(smem, g, s, a, vid, d0 + (int)blockIdx.x, Lp, G, budget, ovl, out_k, out_v, out_n);
}

// the sources a smaller class handed back (`list`: [0] count, [1..] descriptors), again with a
// larger geometry G, grid-stride; a second overflow goes to `ovl` (the host's hand-back list). It
// runs on the handing class's stream right after it: no host round trip for the first overflow.
// (8 waves: the mid geometry; the grid-stride loop needs more than the 128 VGPRs of 16 waves)
static_assert(SV_MID.waves == 8, "k_sv1_redo launch bounds: the mid geometry");
__global__ void __launch_bounds__(8 * WAVE) k_sv1_redo(DevGraph g, DevSlab s, IterArgs a, const int32_t* vid,
                                                         const int32_t* list, int Lp, SvGeom G, int budget,
                                                         int32_t* ovl, int32_t* out_k, double* out_v,
                                                         int32_t* out_n) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = list[0];
  for (int k = (int)blockIdx.x; k < n; k += (int)gridDim.x) {
    __syncthreads();  // the previous source's LDS reads are done
    sv1_source(smem, g, s, a, vid, list[1 + k], Lp, G, budget, ovl, out_k, out_v, out_n);
  }
}

// the sources a class handed back (`list`: [0] count, [1..] descriptors) again with a larger
// geometry G, one workgroup each, over a grid sized for the expected overflows (a workgroup of
// the large geometry holds 113 KB of LDS, so even a block that leaves at once occupies a CU; a
// grid-stride loop spills at the 16-wave VGPR cap). Overflows beyond the grid, and second
// overflows, go to `ovl` (the host's hand-back list). It runs on the class's
// stream right after it: the mid class's overflows take the large geometry (twice the pass-2
// table, a 3 x 8192 sketch) without a host round trip.
__global__ void __launch_bounds__(SV_THREADS) k_sv1_list(DevGraph g, DevSlab s, IterArgs a, const int32_t* vid,
                                                         const int32_t* list, int Lp, SvGeom G, int budget,
                                                         int32_t* ovl, int32_t* out_k, double* out_v,
                                                         int32_t* out_n) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = list[0];
  if (blockIdx.x == 0)  // more overflows than blocks: the rest go to the host hand-back at once
    for (int k = (int)gridDim.x + (int)threadIdx.x; k < n; k += (int)blockDim.x) ovl[1 + atomicAdd(&ovl[0], 1)] = list[1 + k];
  if ((int)blockIdx.x >= n) return;
  sv1_source(smem, g, s, a, vid, list[1 + blockIdx.x], Lp, G, budget, ovl, out_k, out_v, out_n);
}

// the row of a one-slice source from its entries (k_sv1; more than L: the top-L first): one wave
// per source -- sort in hash order, write, range index, norm1 against the old row, maxDiff
// (finish_source)
__host__ __device__ constexpr size_t svfin_lds_bytes(int Lp) { return (size_t)Lp * 12 + 1024 + (size_t)Lp * 20; }
__global__ void __launch_bounds__(64) k_svfin(DevSlab s, IterArgs a, const int32_t* vid, int d0, const int32_t* in_k,
                                              const double* in_v, const int32_t* in_n, int Lp,
                                              unsigned long long* maxdiff, unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int d = d0 + (int)blockIdx.x;
  const int n = in_n[d];
  if (n <= 0) return;  // handed back (a written source has L >= 1 entries)
  const int v = vid[d];
  uint64_t* rv = reinterpret_cast<uint64_t*>(smem);
  int* rk = reinterpret_cast<int*>(smem + (size_t)Lp * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + (size_t)Lp * 12);
  int* hk = reinterpret_cast<int*>(smem + (size_t)Lp * 12 + 1024);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;
  const int32_t* ik = in_k + (int64_t)d * sv_ostride(Lp);
  const double* iv = in_v + (int64_t)d * sv_ostride(Lp);
  finish_source(v, n, [&](int i) { return ik[i]; }, [&](int i) { return iv[i]; }, s, a, hist, rv, rk, Lp, hk, hv, mf,
                maxdiff, stats);
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
  sv_pass1(g, s, a, x, b0, b1, sd.factor, sk);
  __syncthreads();
  uint32_t* gs = gsk + sd.gsk;
  for (int c = threadIdx.x; c < SV_R * (1 << G.wlog); c += blockDim.x) {
    const uint32_t u = sk[c];
    if (u) atomicAdd(&gs[c], u);
  }
  unsigned long long* gp = gpt + sd.gpt;
  for (int i = threadIdx.x; i < x.pt.T; i += blockDim.x) {
    if (!(x.pt.keys[i] & ~SV_OVF_BIT)) continue;
    const unsigned long long A = x.pt.ab[2 * i], B = x.pt.ab[2 * i + 1];
    const int r = x.pt.pos[i];
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
