// merge_mc.h -- MCCompletePathV2 random walks.
//
// walkNode (include/mccompletepathv2.h:115-165) for every node u of the walk set W (nodes some
// predecessor reads before u has its final basket):
//   * deg(u) == 0: basket {u: 1.0}                                                       (:162-163)
//   * else res = {u: R}; floor(R * d) walks from u (:124-132); each walk moves along an edge,
//     counts the node it reaches if that key is already in res or res holds < L keys (:152-153),
//     and continues while U(0,1) <= d (:155), stopping at a dangling node (:144-145);
//     finally every count is divided by R (:159-160).
// RNG (a13): the reference draws from one process-global mt19937 seeded by std::random_device
// and walks a process-global round-robin successor index per node (:149), so it is neither
// reproducible nor parallel. Here, per source: a node held in res keeps its own round-robin
// index (start offset hashed from (seed, source, node)) -- the systematic successor choice that
// keeps the estimator's variance at the reference's level -- and any other node takes a Philox
// pick; Philox4x32-10 is keyed by the 64-bit seed with counter (step, walk lo, walk hi, source),
// and a walk continues while the 53-bit uniform from its other two words is <= d. Walks are cut
// at MC_MAX_STEPS (the reference never ends a walk when d == 1 and no dangling node is
// reachable). oracle/mc_oracle.c restates the same definition (walk_node) sequentially.
//
// Schedule (one wave per source, res in an LDS hash table with u64 counts and u32 round-robin
// indices): 64 walk slots advance in lockstep rounds; a lane whose walk ended takes the next
// walk index (lane order); the step phase moves every live lane one edge, lanes standing on the
// same held node taking consecutive round-robin indices in lane order; the apply phase counts
// the reached nodes in lane order, new keys admitted in lane order while res holds < L keys.
#pragma once
#include "ppr_common.h"

namespace pprk {

constexpr int MC_MAX_STEPS = 1 << 14;           // hard cap on one walk's length
constexpr unsigned long long MC_REJ = ~0ull;    // slot holds a key that lost admission

struct McArgs {
  uint64_t R;        // walks per node ("iterations" of mccompletepathv2)
  uint64_t nw;       // walks actually run: floor(R * d) (include/mccompletepathv2.h:132)
  double damping;
  uint64_t seed;     // Philox key
  int T;             // LDS table slots (power of two, >= 1.5 (L + 64))
  int slot;          // slab slot receiving the walk baskets
};

// per-wave LDS: counts u64[T] | keys i32[T] | round-robin indices u32[T]
__host__ __device__ constexpr size_t mc_wave_lds(int T) { return (size_t)T * 16; }

__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

struct McTable {
  unsigned long long* cnt;
  int* keys;
  uint32_t* rr;
  uint32_t mask;
  int nbits;
};

__device__ __forceinline__ uint32_t mc_find(const McTable& t, int key, bool& present) {
  uint32_t h = hash32((uint32_t)key) & t.mask;
  for (uint32_t n = 0; n <= t.mask; n++) {
    const int k = t.keys[h];
    if (k == key) { present = true; return h; }
    if (k == EMPTY) { present = false; return h; }
    h = (h + 1) & t.mask;
  }
  probe_fail();  // (the walk table holds at most L + 64 keys of its 2^k >= 2 (L + 64) slots)
  present = true;
  return 0u;
}

// lanes of `valid` holding the same slot (ballots over the slot bits)
__device__ __forceinline__ uint64_t mc_match(bool valid, uint32_t slot, int nbits) {
  uint64_t mm = __ballot(valid);
  for (int b = 0; b < nbits; b++) {
    const bool bit = (slot >> b) & 1u;
    const uint64_t bb = __ballot(valid && bit);
    mm &= bit ? bb : ~bb;
  }
  return valid ? mm : 0ull;
}

// apply <= 64 visits in lane order; returns the key's slot, `held` = key is in res
__device__ __forceinline__ uint32_t mc_apply(const McTable& t, bool valid, int key, int L, int& size,
                                             bool& frozen, bool& held) {
  bool present = false;
  uint32_t h = valid ? mc_find(t, key, present) : 0u;
  wave_fence();
  const bool absent = valid && !present;
  if (!frozen && __ballot(absent)) {
    if (absent) {
      bool done = false;
      for (uint32_t n = 0; n <= t.mask && !done; n++) {
        const int prev = atomicCAS(&t.keys[h], EMPTY, key);
        if (prev == EMPTY) { t.cnt[h] = 0ull; t.rr[h] = 0u; done = true; }
        else if (prev == key) done = true;
        else h = (h + 1) & t.mask;
      }
      if (!done) { probe_fail(); h = 0u; }
    }
    wave_fence();
    // lanes holding the same new key share a slot: the lowest lane is its first occurrence
    const uint64_t mm = mc_match(absent, h, t.nbits);
    const bool first = absent && (mm & lanemask_lt()) == 0;
    const uint64_t fm = __ballot(first);
    const int room = L - size;
    if (first && __popcll(fm & lanemask_lt()) >= room) t.cnt[h] = MC_REJ;
    size += min(__popcll(fm), room);
    frozen = size >= L;
    wave_fence();
  }
  held = valid && t.keys[h] == key && t.cnt[h] != MC_REJ;
  if (held) atomicAdd(&t.cnt[h], 1ull);
  wave_fence();
  return h;
}

__global__ void __launch_bounds__(64) k_mc_walk(DevGraph g, DevSlab s, McArgs m, const int32_t* list,
                                                int64_t count) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t w = blockIdx.x;
  if (w >= count) return;
  McTable t;
  t.cnt = reinterpret_cast<unsigned long long*>(smem);
  t.keys = reinterpret_cast<int*>(smem + (size_t)m.T * 8);
  t.rr = reinterpret_cast<uint32_t*>(smem + (size_t)m.T * 12);
  t.mask = (uint32_t)m.T - 1;
  t.nbits = 31 - __clz(m.T);
  const int l = lane_id();
  const int src = list[w];
  const int L = s.L;
  const int64_t rs = s.row(m.slot, src);
  if (g.rp[src + 1] == g.rp[src]) {
    s.rix[s.xrow(m.slot, src) + l] = row_range(src) <= (uint32_t)l ? 1 : 0;
    if (l == 0) { s.ids[rs] = src; s.sc[rs] = 1.0; s.len[s.lrow(m.slot, src)] = 1; s.rmin[s.lrow(m.slot, src)] = 1.0; }
    return;
  }
  for (int i = l; i < m.T; i += WAVE) t.keys[i] = EMPTY;
  wave_fence();
  bool pr;
  const uint32_t hsrc = mc_find(t, src, pr);
  if (l == 0) {
    t.keys[hsrc] = src;
    t.cnt[hsrc] = m.R;  // every walk starts at the source (include/mccompletepathv2.h:124)
    t.rr[hsrc] = 0u;
  }
  wave_fence();
  int size = 1;
  bool frozen = size >= L;
  const uint32_t k0 = (uint32_t)m.seed, k1 = (uint32_t)(m.seed >> 32);
  const uint64_t skey = m.seed ^ ((uint64_t)(uint32_t)src << 32);

  uint64_t next = 0, wi = 0;
  bool alive = false, held = false;
  int cur = src, j = 0;
  uint32_t cslot = 0;
  for (;;) {
    const uint64_t need = __ballot(!alive);
    if (!alive) {
      const uint64_t r = next + (uint64_t)__popcll(need & lanemask_lt());
      if (r < m.nw) { wi = r; alive = true; cur = src; j = 0; cslot = hsrc; held = true; }
    }
    next += (uint64_t)__popcll(need);
    if (!__ballot(alive)) break;
    // step phase
    int64_t b = 0, deg = 0;
    if (alive) {
      b = g.rp[cur];
      deg = g.rp[cur + 1] - b;
      if (deg == 0) alive = false;  // (:144-145)
    }
    const bool stepping = alive;
    const bool rrl = stepping && held;
    const uint64_t mm = mc_match(rrl, cslot, t.nbits);
    uint32_t base = 0;
    if (rrl && (mm & lanemask_lt()) == 0) base = atomicAdd(&t.rr[cslot], (uint32_t)__popcll(mm));
    const int lead = mm ? (__ffsll((long long)mm) - 1) : l;
    base = (uint32_t)__shfl((int)base, lead);
    int key = 0;
    if (stepping) {
      uint32_t c[4] = {(uint32_t)j, (uint32_t)wi, (uint32_t)(wi >> 32), (uint32_t)src};
      philox4x32_10(c, k0, k1);
      uint64_t pick;
      if (rrl) {
        const uint32_t k = base + (uint32_t)__popcll(mm & lanemask_lt());
        const uint32_t h = (uint32_t)(mix64(skey ^ (uint64_t)(uint32_t)cur) >> 32);
        const uint64_t off = ((uint64_t)h * (uint64_t)deg) >> 32;
        pick = off + (uint64_t)(k % (uint32_t)deg);
        if (pick >= (uint64_t)deg) pick -= (uint64_t)deg;
      } else {
        pick = ((uint64_t)c[0] * (uint64_t)deg) >> 32;
      }
      key = g.colx[b + (int64_t)pick] & 0x7fffffff;
      cur = key;
      j++;
      const double u = (double)((((uint64_t)c[2] << 32) | c[3]) >> 11) * 0x1.0p-53;
      if (!(u <= m.damping) || j >= MC_MAX_STEPS) alive = false;  // (:155)
    }
    // apply phase
    cslot = mc_apply(t, stepping, key, L, size, frozen, held);
  }

  // basket: held keys, count / R (include/mccompletepathv2.h:159-160), compacted in place to the
  // front of the table and stored like every other basket row (hash order, range index, minimum)
  const double R = (double)m.R;
  uint64_t* rv = reinterpret_cast<uint64_t*>(t.cnt);
  int U = 0;
  for (int base = 0; base < m.T; base += WAVE) {
    const int i = base + l;
    const int k = t.keys[i];
    const unsigned long long c = t.cnt[i];
    const bool occ = k != EMPTY && c != MC_REJ;
    const uint64_t mb = __ballot(occ);
    wave_fence();
    if (occ) {
      const int pos = U + __popcll(mb & lanemask_lt());
      t.keys[pos] = k;
      rv[pos] = dbits((double)c / R);
    }
    U += __popcll(mb);
    wave_fence();
  }
  const int Lp = L <= 1 ? 1 : (1 << (32 - __clz(L - 1)));
  (void)rs;
  write_row(s, m.slot, src, rv, t.keys, U, Lp, false, 1.0);
}

// final basket of a dangling node: {v: 1.0} (include/mccompletepathv2.h:214, factor 1.0);
// one wave per node (lane q writes range-index entry q)
__global__ void __launch_bounds__(256) k_mc_selfrow(DevSlab s, const int32_t* list, int64_t count, int slot) {
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x >> 6);
  if (i >= count) return;
  const int v = list[i];
  const uint32_t q = (uint32_t)lane_id();
  s.rix[s.xrow(slot, v) + q] = row_range(v) <= q ? 1 : 0;
  if (q == 0) {
    const int64_t r = s.row(slot, v);
    s.ids[r] = v;
    s.sc[r] = 1.0;
    s.len[s.lrow(slot, v)] = 1;
    s.rmin[s.lrow(slot, v)] = 1.0;
  }
}

}  // namespace pprk
