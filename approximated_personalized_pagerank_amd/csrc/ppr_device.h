// ppr_device.h -- wave-level device primitives of the basket-merge kernels (gfx950, wave64).
//
// Everything here is executed by ONE 64-lane wavefront and relies on the in-order execution of
// a wave's LDS instructions; `wave_fence()` only stops the compiler from moving memory
// operations across phase boundaries (it emits no instruction).
//
// Semantics implemented (reference file:line):
//  * accumulation   include/grank.h:107-116  acc[k] = fma(s, d/deg, acc[k]) in successor order;
//                   a key appears at most once per successor basket, so within a 64-candidate
//                   group the only conflicts are the same key from different successors; lanes
//                   sharing a slot are found with ballots over the slot bits and chained lowest
//                   lane (= earliest successor) first in registers (apply_group).
//  * top-L          include/internal/pprInternal.h:109-137 with the deterministic order
//                   (score desc, dense id asc): radix select on the fp64 bit pattern (scores are
//                   >= 0, so IEEE bits order like the values), ties resolved on ~id.
//  * norm1          include/internal/pprInternal.h:147-165, summed in the fixed 64-lane pattern
//                   restated in oracle/grank_oracle.c:norm1_rows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pprd {

constexpr int WAVE = 64;
constexpr int EMPTY = -1;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ void wave_fence() { __asm__ __volatile__("" ::: "memory"); }
__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}
__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double bitsd(uint64_t x) { return __longlong_as_double((long long)x); }

// A hash probe that ran out of slots (every table is sized or budgeted so that this cannot happen;
// a bounded probe turns a sizing bug into an error instead of a hang): each module's kernels set
// its word, the host reads it once per run and fails the run with PPR_ERR_PROBE. Engines with an
// overflow path (the exact-sum tables, the workgroup / bucket tables) take that path instead.
static __device__ unsigned int g_probe_err = 0u;
__device__ __forceinline__ void probe_fail() { atomicOr(&g_probe_err, 1u); }

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// the basket-row order and the hub key-bucket digit: rows are stored by ascending hash_b(key)
// (a bijection of the 32-bit id space, so distinct keys never tie)
__device__ __forceinline__ uint32_t hash_b(uint32_t x) { return hash32(x ^ 0x9e3779b9u); }

// Ties at a top-L cut. The reference leaves them to its unordered_map order + nth_element
// (include/internal/pprInternal.h:115-119): an accident of each map's insertion history, so
// different rows resolve ties differently. A single global order (say by id) instead makes every
// row drop the same keys, and the loss compounds through later iterations (RMAT-12 K16/L32: top-K
// Jaccard vs exact PPR 0.864, the reference 0.90). Here a tie goes to the smaller
// hash32(key ^ tie_salt(source)): deterministic, a bijection of the key for a fixed source, and
// independent across sources (RMAT-12: 0.911; Jaccard vs the reference 0.952, the reference vs
// itself relabelled 0.958). Restated in oracle/grank_oracle.c (tie_key).
__device__ __forceinline__ uint32_t tie_salt(int v) { return hash32((uint32_t)v * 0x9e3779b9u + 1u); }
// larger = preferred (selection keeps the largest (score, tie_w) pairs)
__device__ __forceinline__ uint32_t tie_w(int key, uint32_t ts) { return ~hash32((uint32_t)key ^ ts); }

// Inclusive wave64 scan with DPP (no LDS round trip, unlike __shfl_up's ds_bpermute): Hillis-
// Steele within each 16-lane row (row_shr 1, 2, 4, 8), then row 15's total into rows 1 and 3
// (row_bcast:15) and lane 31's into rows 2 and 3 (row_bcast:31). A lane whose DPP source does not
// exist keeps `old` = 0. Every lane of the wave must be active.
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}
__device__ __forceinline__ uint64_t wave_or(uint64_t x) {
#pragma unroll
  for (int o = 32; o; o >>= 1) x |= (uint64_t)__shfl_xor((unsigned long long)x, o);
  return x;
}
__device__ __forceinline__ uint64_t wave_and(uint64_t x) {
#pragma unroll
  for (int o = 32; o; o >>= 1) x &= (uint64_t)__shfl_xor((unsigned long long)x, o);
  return x;
}
__device__ __forceinline__ int wave_sum(int x) {  // every lane of the wave active
  return __builtin_amdgcn_readlane(wave_incl_scan(x), WAVE - 1);
}

// ---------------------------------------------------------------------------------------------
// LDS accumulation table: open addressing, linear probing, keys unique.
struct LdsTable {
  int* keys;
  double* acc;
  uint32_t mask;  // capacity - 1 (power of two)
  int nbits;      // log2(capacity)
};

__device__ __forceinline__ void table_clear(const LdsTable& t) {
  for (uint32_t i = lane_id(); i <= t.mask; i += WAVE) t.keys[i] = EMPTY;
  wave_fence();
}

// find-or-insert; an inserting lane zeroes the accumulator (reference: operator[] value-inits)
__device__ __forceinline__ uint32_t table_slot(const LdsTable& t, int key) {
  uint32_t h = hash32((uint32_t)key) & t.mask;
  for (uint32_t n = 0; n <= t.mask; n++) {
    const int cur = t.keys[h];
    if (cur == key) return h;
    if (cur == EMPTY) {
      const int prev = atomicCAS(&t.keys[h], EMPTY, key);
      if (prev == EMPTY) { t.acc[h] = 0.0; return h; }
      if (prev == key) return h;
    }
    h = (h + 1) & t.mask;
  }
  probe_fail();  // (T >= 4/3 of the tier's candidate cap: cannot happen; PPR_WAVE_TDIV forces it)
  return 0u;
}

__device__ __forceinline__ double readlane_d(double x, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
  return __hiloint2double(hi, lo);
}

// Apply one group of <= 64 ordered candidates (lane order == successor order) whose table slots
// are resolved. Keys are distinct within one successor basket, so equal slots in a group come
// from different successors: they are chained lowest lane first, in registers, and the slot is
// read and written once. `nbits` bits of the slot index distinguish slots.
__device__ __forceinline__ void apply_group(double* acc, bool valid, uint32_t slot, double s,
                                            double factor, int nbits) {
  const uint64_t vmask = __ballot(valid);
  uint64_t m = vmask;
  for (int b = 0; b < nbits; b++) {
    const bool bit = (slot >> b) & 1u;
    const uint64_t bb = __ballot(valid && bit);
    m &= bit ? bb : ~bb;
  }
  if (!valid) m = 0;
  const uint64_t me = 1ull << lane_id();
  if (!__ballot((m & ~me) != 0)) {  // all keys of the group distinct
    if (valid) acc[slot] = fma(s, factor, acc[slot]);
    wave_fence();
    return;
  }
  const bool leader = valid && (m & lanemask_lt()) == 0;
  const int first = __ffsll((long long)vmask) - 1;
  if (__shfl((unsigned long long)m, first) == vmask) {  // one key for the whole group
    double a = acc[slot];  // same address in every valid lane
    for (uint64_t r = vmask; r; r &= r - 1) a = fma(readlane_d(s, __ffsll((long long)r) - 1), factor, a);
    if (leader) acc[slot] = a;
    wave_fence();
    return;
  }
  double a = 0.0;
  if (leader) a = fma(s, factor, acc[slot]);
  uint64_t rest = leader ? (m & ~me) : 0ull;
  while (__ballot(rest != 0)) {
    const int idx = rest ? (__ffsll((long long)rest) - 1) : lane_id();
    const double sv = __shfl(s, idx);
    if (rest) { a = fma(sv, factor, a); rest &= rest - 1; }
  }
  if (leader) acc[slot] = a;
  wave_fence();
}

__device__ __forceinline__ void table_apply(const LdsTable& t, bool valid, int key, double s,
                                            double factor) {
  const uint32_t slot = valid ? table_slot(t, key) : 0u;
  wave_fence();
  apply_group(t.acc, valid, slot, s, factor, t.nbits);
}

// table_apply with a cheap duplicate test first: every valid lane stores its lane id into own[slot]
// (one byte per slot); when every lane reads its own id back, the group's slots are distinct (two
// lanes sharing a slot cannot both win the store) and each lane applies its fma directly -- the
// usual case in the wave tier, where a group mostly holds one successor's basket (distinct keys).
// Groups with a repeated slot take apply_group's ordered chains.
__device__ __forceinline__ void table_apply_own(const LdsTable& t, uint8_t* own, bool valid, int key, double s,
                                                double factor) {
  const uint32_t slot = valid ? table_slot(t, key) : 0u;
  const uint8_t l = (uint8_t)lane_id();
  if (valid) own[slot] = l;
  wave_fence();
  const bool dup = valid && own[slot] != l;
  wave_fence();
  if (!__ballot(dup)) {
    if (valid) t.acc[slot] = fma(s, factor, t.acc[slot]);
    wave_fence();
    return;
  }
  apply_group(t.acc, valid, slot, s, factor, t.nbits);
}

// Grouped accumulation of one chunk of up to NG * 64 ordered records (record q = lane q % 64 of
// group q / 64), an alternative to apply_group for streams with many repeated keys:
//   A  per group, in order: find-or-insert every key (`slotfn`), rank the lanes sharing a slot
//      (ballots over the slot bits), and give each record its occurrence index within the
//      chunk for its slot; slots first seen in the chunk go to a `touched` list;
//   B  exclusive scan of the per-slot counts over the touched list -> per-slot offsets;
//   C  every record's value goes to vals[offset(slot) + occurrence];
//   D  one lane per touched slot runs that slot's fma chain over vals in stream order.
// A key's contributions therefore still meet acc in stream order (bit-exact with apply_group),
// but a hot key costs one dependent fma per occurrence instead of a cross-lane round per
// occurrence. cnt must be all-zero on entry and is left all-zero.
struct ChunkLds {
  uint32_t* cnt;      // [T] per-slot occurrences in the chunk, then offsets
  double* vals;       // [NG * 64]
  uint16_t* touched;  // [NG * 64]
  uint16_t* tof;      // [NG * 64 + 1]
  uint16_t* ord;      // [NG * 64] (ordered mode) stream position of vals[j]: the order is verified
};

// With `ordered` (lane-ordered LDS atomics, verified on the device at plan creation: see
// k_probe_lds_rank), phase A takes each record's occurrence index straight from a returning LDS
// atomic add on its slot's counter -- same-address lanes of one instruction receive the old
// values in lane order, i.e. stream order -- instead of from ballots over the slot bits.
// (ph: PPR_DIAG cycle counters of phases A..D at ph[11..14], each phase's LDS traffic waited for
// before the clock is read; nullptr = no timing)
__device__ __forceinline__ void diag_lap(unsigned long long* ph, int k, long long& t, const volatile uint32_t* lds) {
  if (!ph) return;
  if (*lds == 0xfffffffeu) wave_fence();  // an LDS read in order behind the phase's own
  const long long t2 = (long long)clock64();
  ph[k] += (unsigned long long)(t2 - t);
  t = t2;
}

// The ordered mode's occurrence indices come from the hardware's order of same-address LDS atomics.
// Nothing documents that order, so it is verified where it is used: every value's stream position
// goes beside it (ord), every value with an occurrence index > 0 is compared with its left neighbour
// (the same key's previous occurrence: its position must be smaller -- sorted runs are exactly those
// whose adjacent pairs are), and if any pair is out of order the wave's chains are recomputed in
// stream order (fma_chain_sorted). The result does not depend on the
// hardware order. (Round 6; PPR_TEST_RANK_PERMUTE forces a permuted order in the tests.)
template <class Ord>
__device__ __forceinline__ double fma_chain_sorted(const double* vals, Ord ord, int b, int e, double f, double x) {
  int last = -1;
  for (int n = b; n < e; n++) {  // the next position: the smallest one past the last (O(n^2), rare)
    int best = b, bo = 0x10000;
    for (int j = b; j < e; j++) {
      const int o = ord(j);
      if (o > last && o < bo) { bo = o; best = j; }
    }
    x = fma(vals[best], f, x);
    last = bo;
  }
  return x;
}
// x = fma(vals[j], f, x) for j = b .. e-1, in that order (one key's ordered chain). The next 8
// values are loaded while the current 8 are folded in, so the dependent fma chain -- not the LDS
// read latency after every few loads -- sets the pace (tools/fma_chain.hip: ~12.5 cycles per fma
// fed this way against ~35-50 for load-4-then-fold-4)
__device__ __forceinline__ double fma_chain_lds(const double* vals, int b, int e, double f, double x) {
  int j = b;
  if (e - j >= 16) {
    double v0 = vals[j], v1 = vals[j + 1], v2 = vals[j + 2], v3 = vals[j + 3];
    double v4 = vals[j + 4], v5 = vals[j + 5], v6 = vals[j + 6], v7 = vals[j + 7];
    for (j += 8; j + 8 <= e; j += 8) {
      const double w0 = vals[j], w1 = vals[j + 1], w2 = vals[j + 2], w3 = vals[j + 3];
      const double w4 = vals[j + 4], w5 = vals[j + 5], w6 = vals[j + 6], w7 = vals[j + 7];
      x = fma(v0, f, x); x = fma(v1, f, x); x = fma(v2, f, x); x = fma(v3, f, x);
      x = fma(v4, f, x); x = fma(v5, f, x); x = fma(v6, f, x); x = fma(v7, f, x);
      v0 = w0; v1 = w1; v2 = w2; v3 = w3; v4 = w4; v5 = w5; v6 = w6; v7 = w7;
    }
    x = fma(v0, f, x); x = fma(v1, f, x); x = fma(v2, f, x); x = fma(v3, f, x);
    x = fma(v4, f, x); x = fma(v5, f, x); x = fma(v6, f, x); x = fma(v7, f, x);
  }
  for (; j + 4 <= e; j += 4) {
    const double v0 = vals[j], v1 = vals[j + 1], v2 = vals[j + 2], v3 = vals[j + 3];
    x = fma(v0, f, x); x = fma(v1, f, x); x = fma(v2, f, x); x = fma(v3, f, x);
  }
  for (; j < e; j++) x = fma(vals[j], f, x);
  return x;
}

template <int NG>
__device__ __forceinline__ void chunk_accumulate(double* acc, const ChunkLds& c, int nbits,
                                                 const bool (&valid)[NG], const uint32_t (&slot)[NG],
                                                 const double (&val)[NG], double factor, bool ordered,
                                                 unsigned long long* ph = nullptr, bool permute = false) {
  const uint64_t lt = lanemask_lt();
  uint32_t occ[NG];
  int nt = 0;
  long long tph = ph ? (long long)clock64() : 0;
  if (ordered) {
#pragma unroll
    for (int k = 0; k < NG; k++) {
      uint32_t o = 1u;
      if (!permute) {
        if (valid[k]) o = atomicAdd(&c.cnt[slot[k]], 1u);
      } else {  // (tests: odd lanes first -- the order a device without lane-ordered atomics may return)
        if (valid[k] && (lane_id() & 1)) o = atomicAdd(&c.cnt[slot[k]], 1u);
        wave_fence();
        if (valid[k] && !(lane_id() & 1)) o = atomicAdd(&c.cnt[slot[k]], 1u);
      }
      const bool fresh = valid[k] && o == 0;
      const uint64_t fm = __ballot(fresh);
      if (fresh) c.touched[nt + __popcll(fm & lt)] = (uint16_t)slot[k];
      nt += __popcll(fm);
      occ[k] = o;
    }
    wave_fence();
  } else
#pragma unroll
  for (int k = 0; k < NG; k++) {
    uint64_t mm = __ballot(valid[k]);
    for (int b = 0; b < nbits; b++) {
      const bool bit = (slot[k] >> b) & 1u;
      const uint64_t bb = __ballot(valid[k] && bit);
      mm &= bit ? bb : ~bb;
    }
    if (!valid[k]) mm = 0;
    const bool leader = valid[k] && (mm & lt) == 0;
    uint32_t base = 0;
    if (leader) {
      base = c.cnt[slot[k]];
      c.cnt[slot[k]] = base + (uint32_t)__popcll(mm);
    }
    const bool fresh = leader && base == 0;
    const uint64_t fm = __ballot(fresh);
    if (fresh) c.touched[nt + __popcll(fm & lt)] = (uint16_t)slot[k];
    nt += __popcll(fm);
    const int lead = mm ? (__ffsll((long long)mm) - 1) : lane_id();
    base = (uint32_t)__shfl((int)base, lead);
    occ[k] = base + (uint32_t)__popcll(mm & lt);
    wave_fence();
  }
  diag_lap(ph, 11, tph, c.cnt);
  // B: offsets of the touched slots (touched order), written over their counts
  int run = 0;
  for (int i0 = 0; i0 < nt; i0 += WAVE) {
    const int i = i0 + lane_id();
    const int n = i < nt ? c.cnt[c.touched[i]] : 0;
    const int incl = wave_incl_scan(n);
    if (i < nt) { c.tof[i] = (uint16_t)(run + incl - n); c.cnt[c.touched[i]] = (uint32_t)(run + incl - n); }
    run += __builtin_amdgcn_readlane(incl, WAVE - 1);
  }
  if (lane_id() == 0) c.tof[nt] = (uint16_t)run;
  wave_fence();
  diag_lap(ph, 12, tph, c.cnt);
  // C: values grouped by slot, stream order inside a slot (ordered mode: with the stream position)
  uint32_t qq[NG];
#pragma unroll
  for (int k = 0; k < NG; k++) {
    qq[k] = valid[k] ? c.cnt[slot[k]] + occ[k] : 0u;
    if (valid[k]) {
      c.vals[qq[k]] = val[k];
      if (ordered) c.ord[qq[k]] = (uint16_t)(k * WAVE + lane_id());
    }
  }
  wave_fence();
  // (ordered) the order check, every record at once, off the chains' path: a record with an
  // occurrence index > 0 has its slot's previous occurrence just before it, which must come earlier
  // in the stream (across groups program order guarantees it; only same-instruction lanes can fail)
  bool sorted_path = false;
  if (ordered) {
    bool bad = false;
#pragma unroll
    for (int k = 0; k < NG; k++)
      if (valid[k] && occ[k] > 0u) bad = bad || (int)c.ord[qq[k] - 1] > k * WAVE + lane_id();
    sorted_path = __ballot(bad) != 0ull;
  }
  diag_lap(ph, 13, tph, c.cnt);
  // D: one lane per touched slot
  for (int i = lane_id(); i < nt; i += WAVE) {
    const uint32_t sl = c.touched[i];
    const int b = c.tof[i], e = c.tof[i + 1];
    if (__builtin_expect(sorted_path, 0))
      acc[sl] = fma_chain_sorted(c.vals, [&](int j) { return (int)c.ord[j]; }, b, e, factor, acc[sl]);
    else
      acc[sl] = fma_chain_lds(c.vals, b, e, factor, acc[sl]);
    c.cnt[sl] = 0;
  }
  wave_fence();
  diag_lap(ph, 14, tph, c.cnt);
}

// In-place compaction of occupied slots to the front (keys[0..U), acc[0..U)); returns U.
__device__ __forceinline__ int table_compact(const LdsTable& t) {
  int U = 0;
  for (uint32_t base = 0; base <= t.mask; base += WAVE) {
    const uint32_t i = base + lane_id();
    const int k = t.keys[i];
    const double a = t.acc[i];
    const bool occ = k != EMPTY;
    const uint64_t m = __ballot(occ);
    wave_fence();
    if (occ) {
      const int pos = U + __popcll(m & lanemask_lt());
      t.keys[pos] = k;
      t.acc[pos] = a;
    }
    wave_fence();
    U += __popcll(m);
  }
  return U;
}

// In-place compaction of the occupied slots whose value is >= lo (the top-L pruning bound).
__device__ __forceinline__ int table_compact_min(const LdsTable& t, double lo) {
  int U = 0;
  for (uint32_t base = 0; base <= t.mask; base += WAVE) {
    const uint32_t i = base + lane_id();
    const int k = t.keys[i];
    const double a = t.acc[i];
    const bool keep = k != EMPTY && a >= lo;
    const uint64_t m = __ballot(keep);
    wave_fence();
    if (keep) {
      const int pos = U + __popcll(m & lanemask_lt());
      t.keys[pos] = k;
      t.acc[pos] = a;
    }
    wave_fence();
    U += __popcll(m);
  }
  return U;
}

// ---------------------------------------------------------------------------------------------
// Top-`need` selection by (score desc, tie_w desc) over n entries (keys[i], vals[i]) held in LDS
// or global memory. Result: entry i is selected iff
//     (v & ma) > pa  ||  ((v & ma) == pa && (!tie || (w & mb) >= pb))
// v = bits(score), w = tie_w(key, ts)
struct SelCrit {
  uint64_t pa, ma;
  uint64_t pb, mb;
  bool tie;
};

// radix select of the k-th largest 64-bit value among filtered entries (8-bit digits from the
// highest bit that varies). On return: prefix/mask fix the boundary bucket; k = how many of the
// boundary bucket are selected; resolved = boundary holds exactly-equal values with more than k
// members (a tie that the caller must break on another field).
template <class GetV, class Filt>
__device__ __forceinline__ void radix_kth_desc(int n, int& k, GetV getv, Filt filt,
                                               uint32_t* hist, uint64_t& prefix, uint64_t& mask,
                                               bool& tie_left) {
  uint64_t lor = 0, land = ~0ull;
  int cnt = 0;
  for (int i = lane_id(); i < n; i += WAVE)
    if (filt(i)) { const uint64_t v = getv(i); lor |= v; land &= v; cnt++; }
  lor = wave_or(lor);
  land = wave_and(land);
  cnt = wave_sum(cnt);
  const uint64_t diff = lor ^ land;
  if (diff == 0) {  // every filtered value equal
    prefix = land; mask = ~0ull; tie_left = cnt > k;
    return;
  }
  const int top = 63 - __clzll((long long)diff);
  mask = top == 63 ? 0ull : ~((2ull << top) - 1ull);
  prefix = land & mask;
  int shift = top >= 7 ? top - 7 : 0;
  for (;;) {
    for (int b = lane_id(); b < 256; b += WAVE) hist[b] = 0;
    wave_fence();
    for (int i = lane_id(); i < n; i += WAVE) {
      if (!filt(i)) continue;
      const uint64_t v = getv(i);
      if ((v & mask) == prefix) atomicAdd(&hist[(uint32_t)(v >> shift) & 255u], 1u);
    }
    wave_fence();
    // lane l owns bins 255-4l .. 252-4l (descending), scan finds the boundary bin
    const int l = lane_id();
    uint32_t c[4];
#pragma unroll
    for (int j = 0; j < 4; j++) c[j] = hist[255 - 4 * l - j];
    const int s = (int)(c[0] + c[1] + c[2] + c[3]);
    const int incl = wave_incl_scan(s);
    int run = incl - s;
    int bin = -1, above = 0, hb = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (bin < 0 && run < k && run + (int)c[j] >= k) { bin = 255 - 4 * l - j; above = run; hb = (int)c[j]; }
      run += (int)c[j];
    }
    const uint64_t who = __ballot(bin >= 0);
    const int src = __ffsll((long long)who) - 1;
    bin = __shfl(bin, src);
    above = __shfl(above, src);
    hb = __shfl(hb, src);
    k -= above;
    prefix |= (uint64_t)bin << shift;
    mask |= 255ull << shift;
    wave_fence();
    if (hb == k) { tie_left = false; return; }
    if (shift == 0) { tie_left = true; return; }
    shift = shift >= 8 ? shift - 8 : 0;
  }
}

// Top-`need` of at most 4 * 64 entries with the values in registers (round 6): the need-th largest
// value is found bit by bit from the highest varying bit, each step one compare and one ballot per
// register and scalar popcounts -- no LDS histogram, no fence -- and the search stops as soon as the
// entries at or above the current bound are exactly `need`. Exact ties at the cut are broken by the
// largest tie_w the same way. The selected set is radix_kth_desc's: {v > v*} plus, at v = v*, all
// of them or those with tie_w >= w* (w* the k-th largest tie_w there).
struct SelAll {
  __device__ bool operator()(int) const { return true; }
};
#ifndef PPR_SEL_REG
#define PPR_SEL_REG 1  // (A/B only: 0 = the histogram passes for every size)
#endif
template <class KeyAt, class ValAt, class Occ = SelAll>
__device__ __forceinline__ SelCrit select_top_reg(int n, int need, KeyAt keyat, ValAt valat, uint32_t ts,
                                                  Occ occ = Occ{}) {
  constexpr int R = 4;
  uint64_t v[R];
  bool ok[R];
  uint64_t lor = 0, land = ~0ull;
#pragma unroll
  for (int j = 0; j < R; j++) {
    const int i = j * WAVE + lane_id();
    ok[j] = i < n && occ(i);
    v[j] = ok[j] ? dbits(valat(i)) : 0ull;
    if (ok[j]) { lor |= v[j]; land &= v[j]; }
  }
  lor = wave_or(lor);
  land = wave_and(land);
  auto count_ge = [&](uint64_t x) {
    int c = 0;
#pragma unroll
    for (int j = 0; j < R; j++) c += __popcll(__ballot(ok[j] && v[j] >= x));
    return c;
  };
  SelCrit c;
  c.tie = false; c.pb = 0; c.mb = 0; c.ma = ~0ull;
  const uint64_t diff = lor ^ land;
  uint64_t x = land;  // every value equal: the bound is that value
  int cx = 0;         // entries >= x
#pragma unroll
  for (int j = 0; j < R; j++) cx += __popcll(__ballot(ok[j]));
  if (diff) {
    const int top = 63 - __clzll((long long)diff);
    x = land & (top == 63 ? 0ull : ~((2ull << top) - 1ull));  // the shared high bits, zeros below
    for (int b = top; b >= 0 && cx != need; b--) {
      const uint64_t cand = x | (1ull << b);
      const int cnt = count_ge(cand);
      if (cnt >= need) { x = cand; cx = cnt; }
    }
  }
  c.pa = x;  // v >= x selects cx entries; cx == need unless values equal to x straddle the cut
  if (cx > need) {
    // exact ties at x: the (need - #{v > x}) largest tie_w among them
    int gt = 0;
#pragma unroll
    for (int j = 0; j < R; j++) gt += __popcll(__ballot(ok[j] && v[j] > x));
    const int k2 = need - gt;
    uint32_t w[R];
    bool eq[R];
    uint32_t wor = 0, wand = ~0u;
#pragma unroll
    for (int j = 0; j < R; j++) {
      eq[j] = ok[j] && v[j] == x;
      w[j] = eq[j] ? tie_w(keyat(j * WAVE + lane_id()), ts) : 0u;
      if (eq[j]) { wor |= w[j]; wand &= w[j]; }
    }
    wor = (uint32_t)wave_or(wor);
    wand = (uint32_t)wave_and(wand);
    const uint32_t wd = wor ^ wand;
    uint32_t y = wand;
    int cy = 0;
#pragma unroll
    for (int j = 0; j < R; j++) cy += __popcll(__ballot(eq[j]));
    if (wd) {
      const int top = 31 - __clz(wd);
      y = wand & (top == 31 ? 0u : ~((2u << top) - 1u));
      for (int b = top; b >= 0 && cy != k2; b--) {
        const uint32_t cand = y | (1u << b);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < R; j++) cnt += __popcll(__ballot(eq[j] && w[j] >= cand));
        if (cnt >= k2) { y = cand; cy = cnt; }
      }
    }
    c.tie = true;
    c.pb = y;
    c.mb = 0xffffffffull;
  }
  return c;
}

template <class KeyAt, class ValAt>
__device__ __forceinline__ SelCrit select_top(int n, int need, KeyAt keyat, ValAt valat,
                                              uint32_t* hist, uint32_t ts) {
  if (PPR_SEL_REG && n <= 4 * WAVE) return select_top_reg(n, need, keyat, valat, ts);
  SelCrit c;
  c.tie = false; c.pb = 0; c.mb = 0;
  int k = need;
  bool tie = false;
  radix_kth_desc(n, k, [&](int i) { return dbits(valat(i)); }, [&](int) { return true; },
                 hist, c.pa, c.ma, tie);
  if (tie) {
    // all boundary entries carry exactly the same score: keep the k with the largest tie_w
    const uint64_t pa = c.pa;
    bool tie2 = false;
    radix_kth_desc(n, k, [&](int i) { return (uint64_t)tie_w(keyat(i), ts); },
                   [&](int i) { return dbits(valat(i)) == pa; }, hist, c.pb, c.mb, tie2);
    c.tie = true;
  }
  return c;
}

__device__ __forceinline__ bool sel_test(const SelCrit& c, uint64_t v, uint32_t w) {
  const uint64_t va = v & c.ma;
  if (va != c.pa) return va > c.pa;
  return !c.tie || ((uint64_t)w & c.mb) >= c.pb;
}

// ---------------------------------------------------------------------------------------------
// Row buffer (LDS): rv = score bits, rk = id; bitonic sort, (score desc, id asc) -- the output
// order -- or, with `by_tie`, (score desc, tie_w desc) -- the selection order.
__device__ __forceinline__ bool row_less(uint64_t av, int ak, uint64_t bv, int bk) {
  // "a ranks below b"
  return av < bv || (av == bv && (uint32_t)~ak < (uint32_t)~bk);
}

__device__ __forceinline__ void row_sort(uint64_t* rv, int* rk, int cnt, int Lp, bool by_tie = false,
                                         uint32_t ts = 0) {
  // the network spans the smallest power of two >= cnt (<= Lp, the buffer's size): a short row
  // (52 % of the RMAT-22 rows are dangling nodes' {v: 1-d}) sorts in a few stages, not log^2 Lp
  int N = 1;
  while (N < cnt) N <<= 1;
  Lp = N < Lp ? N : Lp;
  for (int i = cnt + lane_id(); i < Lp; i += WAVE) { rv[i] = 0; rk[i] = -1; }  // sentinels last
  wave_fence();
  for (int k = 2; k <= Lp; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = lane_id(); t < (Lp >> 1); t += WAVE) {
        const int i = ((t / j) * 2 * j) + (t % j);
        const int p = i + j;
        const uint64_t av = rv[i], bv = rv[p];
        const int ak = rk[i], bk = rk[p];
        // descending overall: blocks with (i & k) == 0 descend
        const bool desc = (i & k) == 0;
        // selection order: sentinels (id -1, score 0) rank below every entry of equal score
        const uint64_t ra = ak < 0 ? 0ull : 1ull + tie_w(ak, ts), rb = bk < 0 ? 0ull : 1ull + tie_w(bk, ts);
        const bool lt_ab = by_tie ? (av < bv || (av == bv && ra < rb)) : row_less(av, ak, bv, bk);
        const bool lt_ba = by_tie ? (bv < av || (bv == av && rb < ra)) : row_less(bv, bk, av, ak);
        const bool swap = desc ? lt_ab : lt_ba;
        if (swap) { rv[i] = bv; rv[p] = av; rk[i] = bk; rk[p] = ak; }
      }
      wave_fence();
    }
  }
}

// Row buffer sorted by ascending hash_b(key) (the stored basket order); EMPTY keys sort last.
__device__ __forceinline__ uint64_t hash_order(int key) {
  return key == EMPTY ? ~0ull : (uint64_t)hash_b((uint32_t)key);
}
__device__ __forceinline__ void row_sort_hash(uint64_t* rv, int* rk, int cnt, int Lp) {
  for (int i = cnt + lane_id(); i < Lp; i += WAVE) { rv[i] = 0; rk[i] = EMPTY; }  // sentinels last
  wave_fence();
  for (int k = 2; k <= Lp; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = lane_id(); t < (Lp >> 1); t += WAVE) {
        const int i = ((t / j) * 2 * j) + (t % j);
        const int p = i + j;
        const uint64_t av = rv[i], bv = rv[p];
        const int ak = rk[i], bk = rk[p];
        const uint64_t ha = hash_order(ak), hb = hash_order(bk);
        const bool asc = (i & k) == 0;
        const bool swap = asc ? (ha > hb) : (ha < hb);
        if (swap) { rv[i] = bv; rv[p] = av; rk[i] = bk; rk[p] = ak; }
      }
      wave_fence();
    }
  }
}

// norm1 between the new row (LDS rv/rk, cnt) and the old row (global ids/scores, olen), with
// the fixed lane pattern of oracle/grank_oracle.c:norm1_rows. hk/hv: LDS hash of 2*Lp slots,
// mf: LDS flags (Lp); dec maps a stored id of the old row to its key.
template <class Dec>
__device__ __forceinline__ double row_norm1(const uint64_t* rv, const int* rk, int cnt,
                                            const int* oid, const double* osc, int olen,
                                            int* hk, int* hv, int* mf, int hsize, Dec dec) {
  const uint32_t hmask = (uint32_t)hsize - 1;
  for (int i = lane_id(); i < hsize; i += WAVE) hk[i] = EMPTY;
  for (int j = lane_id(); j < olen; j += WAVE) mf[j] = 0;
  wave_fence();
  for (int j = lane_id(); j < olen; j += WAVE) {
    const int key = dec(oid[j]);  // the old row's stored id -> key
    uint32_t h = hash32((uint32_t)key) & hmask;
    bool done = false;
    for (uint32_t n = 0; n <= hmask && !done; n++) {  // (2 Lp slots for <= L keys: never full)
      const int prev = atomicCAS(&hk[h], EMPTY, key);
      if (prev == EMPTY) { hv[h] = j; done = true; }
      h = (h + 1) & hmask;
    }
    if (!done) probe_fail();
  }
  wave_fence();
  double p = 0.0;
  for (int i = lane_id(); i < cnt; i += WAVE) {
    const int key = rk[i];
    uint32_t h = hash32((uint32_t)key) & hmask;
    double o = 0.0;
    for (uint32_t n = 0; n <= hmask; n++) {
      const int cur = hk[h];
      if (cur == key) { const int j = hv[h]; o = osc[j]; mf[j] = 1; break; }
      if (cur == EMPTY) break;
      h = (h + 1) & hmask;
    }
    p += fabs(bitsd(rv[i]) - o);
  }
  wave_fence();
  for (int j = lane_id(); j < olen; j += WAVE)
    if (!mf[j]) p += osc[j];
#pragma unroll
  for (int o = 32; o; o >>= 1) p = p + __shfl_xor(p, o);
  return p;
}

}  // namespace pprd
