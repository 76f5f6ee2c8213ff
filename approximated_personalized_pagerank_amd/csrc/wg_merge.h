// wg_merge.h -- workgroup-cooperative basket merge (8 waves, one source per workgroup).
//
// For sources whose candidate count exceeds a single wave's LDS table. The 8 waves share ONE
// LDS hash table; every key has an owner wave (bits of its hash) and only the owner touches
// it, so each key's fma chain is applied by one wave in stream order (include/grank.h:107-116
// order is preserved). Each chunk of 1024 candidates (in successor order) is routed to the
// owner waves through a stable LDS partition: per (wave, half) group counts by ballot, an
// exclusive scan over groups, then ranks inside a group by ballot popcount.
//
// Sources with more distinct keys than one table holds are processed in P key-bucket passes
// (bucket = second hash of the key mod P; each pass accumulates only its bucket's keys, so a
// key's chain is still complete within one pass) and the per-pass top-L lists are merged at the
// end: the top-L of the union of disjoint key sets is inside the union of their top-Ls.
#pragma once
#include "ppr_device.h"

namespace pprd {

constexpr int WG_WAVES = 8;
constexpr int WG_THREADS = WG_WAVES * WAVE;      // 512
constexpr int WG_CHUNK = 2 * WG_THREADS;         // candidates per routing step
constexpr int WG_WIN = WG_THREADS;               // successors per window

__device__ __forceinline__ uint32_t hash_b(uint32_t x) { return hash32(x ^ 0x9e3779b9u); }

// shared-table variant of table_slot with an occupancy budget (returns 0xffffffff when full)
__device__ __forceinline__ uint32_t wg_slot(int* keys, double* acc, uint32_t T, uint32_t h0,
                                            int key, uint32_t* fill, uint32_t budget) {
  uint32_t h = h0;
  for (;;) {
    const int cur = keys[h];
    if (cur == key) return h;
    if (cur == EMPTY) {
      if (*fill >= budget) return 0xffffffffu;
      const int prev = atomicCAS(&keys[h], EMPTY, key);
      if (prev == EMPTY) { acc[h] = 0.0; atomicAdd(fill, 1u); return h; }
      if (prev == key) return h;
    }
    h = (h + 1 == T) ? 0 : h + 1;
  }
}

struct WgLds {
  // table
  double* acc;      // [T]
  int* keys;        // [T]
  uint32_t* owner;  // [T]
  // routing queue
  int* qk;          // [WG_CHUNK]
  double* qs;       // [WG_CHUNK]
  int* cnt;         // [16 groups][8 owners]
  int* pre;         // [16][8] exclusive prefix per owner over groups
  int* seg;         // [8 + 1] owner segment offsets
  // window of successors
  int* wpre;        // [WG_WIN] inclusive prefix of lens
  int* wu;          // [WG_WIN]
  int* wsl;         // [WG_WIN]
  // partial top-L lists of all passes
  int* pk;          // [PL]
  double* pv;       // [PL]
  // selection / row
  uint32_t* hist;   // [256]
  int* misc;        // [64] scalars shared by the block
  uint64_t* rv;     // [Lp]
  int* rk;          // [Lp]
  int* hk;          // [2Lp]
  int* hv;          // [2Lp]
  int* mf;          // [Lp]
};

__host__ __device__ constexpr size_t wg_lds_bytes(int T, int Lp, int PL) {
  return (size_t)T * 16 + (size_t)WG_CHUNK * 12 + 128 * 4 * 2 + 16 * 4 + (size_t)WG_WIN * 12 +
         (size_t)PL * 12 + 1024 + 256 + (size_t)Lp * 12 + (size_t)Lp * 20 + 64;
}

__device__ __forceinline__ WgLds wg_carve(unsigned char* base, int T, int Lp, int PL) {
  WgLds w;
  unsigned char* p = base;
  w.acc = reinterpret_cast<double*>(p); p += (size_t)T * 8;
  w.qs = reinterpret_cast<double*>(p); p += (size_t)WG_CHUNK * 8;
  w.pv = reinterpret_cast<double*>(p); p += (size_t)PL * 8;
  w.rv = reinterpret_cast<uint64_t*>(p); p += (size_t)Lp * 8;
  w.keys = reinterpret_cast<int*>(p); p += (size_t)T * 4;
  w.owner = reinterpret_cast<uint32_t*>(p); p += (size_t)T * 4;
  w.qk = reinterpret_cast<int*>(p); p += (size_t)WG_CHUNK * 4;
  w.cnt = reinterpret_cast<int*>(p); p += 128 * 4;
  w.pre = reinterpret_cast<int*>(p); p += 128 * 4;
  w.seg = reinterpret_cast<int*>(p); p += 16 * 4;
  w.wpre = reinterpret_cast<int*>(p); p += (size_t)WG_WIN * 4;
  w.wu = reinterpret_cast<int*>(p); p += (size_t)WG_WIN * 4;
  w.wsl = reinterpret_cast<int*>(p); p += (size_t)WG_WIN * 4;
  w.pk = reinterpret_cast<int*>(p); p += (size_t)PL * 4;
  w.hist = reinterpret_cast<uint32_t*>(p); p += 1024;
  w.misc = reinterpret_cast<int*>(p); p += 256;
  w.rk = reinterpret_cast<int*>(p); p += (size_t)Lp * 4;
  w.hk = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  w.hv = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  w.mf = reinterpret_cast<int*>(p); p += (size_t)Lp * 4;
  return w;
}

// misc slots
enum { M_FILL = 0, M_OVF = 1, M_PLEN = 2, M_U = 3, M_BIN = 4, M_ABOVE = 5, M_HB = 6, M_TOT = 7,
       M_LOR0 = 8, M_LOR1 = 9, M_LAND0 = 10, M_LAND1 = 11, M_CNT = 12 };

// Route one chunk (each lane holds 2 candidates, valid flag) to owner waves, then every wave
// applies its owner segment in order. Returns false on table overflow.
__device__ __forceinline__ void wg_route_apply(const WgLds& w, uint32_t T, uint32_t budget,
                                               bool v0, int k0, double s0, bool v1, int k1,
                                               double s1, double factor) {
  const int wv = threadIdx.x >> 6;
  const int l = lane_id();
  const uint32_t h0 = hash32((uint32_t)k0), h1 = hash32((uint32_t)k1);
  const int o0 = (int)((h0 >> 5) & 7u), o1 = (int)((h1 >> 5) & 7u);
  // counts per (group, owner): group = wave*2 + half
  int r0 = 0, r1 = 0;
#pragma unroll
  for (int o = 0; o < WG_WAVES; o++) {
    const uint64_t b0 = __ballot(v0 && o0 == o);
    const uint64_t b1 = __ballot(v1 && o1 == o);
    if (o0 == o) r0 = __popcll(b0 & lanemask_lt());
    if (o1 == o) r1 = __popcll(b1 & lanemask_lt());
    if (l == o) { w.cnt[(wv * 2) * 8 + o] = __popcll(b0); w.cnt[(wv * 2 + 1) * 8 + o] = __popcll(b1); }
  }
  __syncthreads();
  if (threadIdx.x < WG_WAVES) {
    const int o = threadIdx.x;
    int run = 0;
    for (int gi = 0; gi < 2 * WG_WAVES; gi++) { w.pre[gi * 8 + o] = run; run += w.cnt[gi * 8 + o]; }
    w.misc[16 + o] = run;  // totals
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int o = 0; o < WG_WAVES; o++) { w.seg[o] = run; run += w.misc[16 + o]; }
    w.seg[WG_WAVES] = run;
  }
  __syncthreads();
  if (v0) { const int pos = w.seg[o0] + w.pre[(wv * 2) * 8 + o0] + r0; w.qk[pos] = k0; w.qs[pos] = s0; }
  if (v1) { const int pos = w.seg[o1] + w.pre[(wv * 2 + 1) * 8 + o1] + r1; w.qk[pos] = k1; w.qs[pos] = s1; }
  __syncthreads();
  // owner wave wv applies its segment in order
  const int b = w.seg[wv], e = w.seg[wv + 1];
  const uint32_t me = (uint32_t)l;
  for (int g0 = b; g0 < e; g0 += WAVE) {
    const int i = g0 + l;
    const bool valid = i < e;
    const int key = valid ? w.qk[i] : 0;
    const double s = valid ? w.qs[i] : 0.0;
    uint32_t slot = 0;
    bool ok = true;
    if (valid) {
      slot = wg_slot(w.keys, w.acc, T, (uint32_t)(((uint64_t)hash32((uint32_t)key) * T) >> 32), key,
                     reinterpret_cast<uint32_t*>(&w.misc[M_FILL]), budget);
      ok = slot != 0xffffffffu;
      if (!ok) w.misc[M_OVF] = 1;
    }
    wave_fence();
    bool pending = valid && ok;
    while (__ballot(pending)) {
      if (pending) atomicMin(&w.owner[slot], me);
      wave_fence();
      if (pending && w.owner[slot] == me) {
        w.acc[slot] = fma(s, factor, w.acc[slot]);
        w.owner[slot] = NO_OWNER;
        pending = false;
      }
      wave_fence();
    }
  }
  __syncthreads();
}

// block-wide radix select of the top-`need` (score desc, id asc) among n entries in LDS.
// Same criterion as select_top (wave version); one wave scans the histogram.
template <class GetV, class Filt>
__device__ __forceinline__ void wg_radix_kth(const WgLds& w, int n, int& k, GetV getv, Filt filt,
                                             uint64_t& prefix, uint64_t& mask, bool& tie_left) {
  const int l = lane_id();
  uint64_t lor = 0, land = ~0ull;
  int c = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    if (filt(i)) { const uint64_t v = getv(i); lor |= v; land &= v; c++; }
  lor = wave_or(lor); land = wave_and(land); c = wave_sum(c);
  uint64_t* red = reinterpret_cast<uint64_t*>(w.hist);  // 8 waves x 2 u64 + counts (fits 1 KB)
  int* redc = reinterpret_cast<int*>(w.hist) + 64;
  if (l == 0) { red[(threadIdx.x >> 6) * 2] = lor; red[(threadIdx.x >> 6) * 2 + 1] = land; redc[threadIdx.x >> 6] = c; }
  __syncthreads();
  lor = 0; land = ~0ull; c = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) { lor |= red[2 * i]; land &= red[2 * i + 1]; c += redc[i]; }
  __syncthreads();
  const uint64_t diff = lor ^ land;
  if (diff == 0) { prefix = land; mask = ~0ull; tie_left = c > k; return; }
  const int top = 63 - __clzll((long long)diff);
  mask = top == 63 ? 0ull : ~((2ull << top) - 1ull);
  prefix = land & mask;
  int shift = top >= 7 ? top - 7 : 0;
  for (;;) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) w.hist[b] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      if (!filt(i)) continue;
      const uint64_t v = getv(i);
      if ((v & mask) == prefix) atomicAdd(&w.hist[(uint32_t)(v >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < WAVE) {
      uint32_t cc[4];
#pragma unroll
      for (int j = 0; j < 4; j++) cc[j] = w.hist[255 - 4 * l - j];
      const int s = (int)(cc[0] + cc[1] + cc[2] + cc[3]);
      const int incl = wave_incl_scan(s);
      int run = incl - s, bin = -1, above = 0, hb = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if (bin < 0 && run < k && run + (int)cc[j] >= k) { bin = 255 - 4 * l - j; above = run; hb = (int)cc[j]; }
        run += (int)cc[j];
      }
      if (bin >= 0) { w.misc[M_BIN] = bin; w.misc[M_ABOVE] = above; w.misc[M_HB] = hb; }
    }
    __syncthreads();
    const int bin = w.misc[M_BIN], above = w.misc[M_ABOVE], hb = w.misc[M_HB];
    __syncthreads();
    k -= above;
    prefix |= (uint64_t)bin << shift;
    mask |= 255ull << shift;
    if (hb == k) { tie_left = false; return; }
    if (shift == 0) { tie_left = true; return; }
    shift = shift >= 8 ? shift - 8 : 0;
  }
}

template <class KeyAt, class ValAt, class Occ>
__device__ __forceinline__ SelCrit wg_select_top(const WgLds& w, int n, int need, KeyAt keyat,
                                                 ValAt valat, Occ occ) {
  SelCrit c;
  c.tie = false; c.pb = 0; c.mb = 0;
  int k = need;
  bool tie = false;
  wg_radix_kth(w, n, k, [&](int i) { return dbits(valat(i)); }, occ, c.pa, c.ma, tie);
  if (tie) {
    const uint64_t pa = c.pa;
    bool tie2 = false;
    wg_radix_kth(w, n, k, [&](int i) { return (uint64_t)(uint32_t)~keyat(i); },
                 [&](int i) { return occ(i) && dbits(valat(i)) == pa; }, c.pb, c.mb, tie2);
    c.tie = true;
  }
  return c;
}

// block inclusive scan of one int per thread (512 threads); scratch: 8 ints
__device__ __forceinline__ int wg_incl_scan(int x, int* scratch) {
  const int incl = wave_incl_scan(x);
  if (lane_id() == WAVE - 1) scratch[threadIdx.x >> 6] = incl;
  __syncthreads();
  int add = 0;
  for (int i = 0; i < (int)(threadIdx.x >> 6); i++) add += scratch[i];
  __syncthreads();
  return incl + add;
}

}  // namespace pprd
