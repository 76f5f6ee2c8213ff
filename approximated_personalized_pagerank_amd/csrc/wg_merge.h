// wg_merge.h -- workgroup-cooperative basket merge (8 waves, one source per workgroup).
//
// For sources whose candidate count exceeds a single wave's LDS table. The 8 waves share ONE
// LDS hash table; every key has an owner wave (bits of its hash) and only the owner touches
// it, so each key's fma chain is applied by one wave in stream order (include/grank.h:107-116
// order is preserved). Each chunk of 1024 candidates (in successor order) is routed to the
// owner waves through a stable LDS partition: per (wave, half) group counts by ballot, an
// exclusive scan over groups, then ranks inside a group by ballot popcount.
//
// Streams with more distinct keys than one table holds are processed in P key-bucket passes
// (bucket = salted hash of the key mod P; each pass accumulates only its bucket's keys, so a
// key's chain is still complete within one pass). The top-L of each pass is folded into a
// running top-L: the top-L of a union of disjoint key sets lies inside the union of their
// top-Ls. A pass that overflows the table restarts the stream with twice as many passes.
#pragma once
#include "ppr_common.h"

namespace pprk {

constexpr int WG_WAVES = 8;
constexpr int WG_THREADS = WG_WAVES * WAVE;      // 512
constexpr int WG_CHUNK = 2 * WG_THREADS;         // candidates per routing step
constexpr int WG_WIN = WG_THREADS;               // successors per window


// shared-table variant of table_slot with an occupancy budget (returns 0xffffffff when full)
__device__ __forceinline__ uint32_t wg_slot(int* keys, double* acc, uint32_t T, uint32_t h0,
                                            int key, uint32_t* fill, uint32_t budget) {
  uint32_t h = h0;
  for (uint32_t n = 0; n < T; n++) {
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
  return 0xffffffffu;  // (full: the caller's overflow pass)
}

struct WgLds {
  // table
  double* acc;      // [T]
  int* keys;        // [T]
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

// partial (running top-L) list capacity: the running L plus one pass's L
__host__ __device__ constexpr int wg_pl(int Lp) { return 2 * Lp; }

__host__ __device__ constexpr size_t wg_lds_bytes(int T, int Lp, int PL) {
  return (size_t)T * 12 + (size_t)WG_CHUNK * 12 + 128 * 4 * 2 + 16 * 4 + (size_t)WG_WIN * 12 +
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
       M_LOR0 = 8, M_LOR1 = 9, M_LAND0 = 10, M_LAND1 = 11, M_CNT = 12, M_SPEC = 13 };

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
  for (int g0 = b; g0 < e; g0 += WAVE) {
    const int i = g0 + l;
    const bool valid = i < e;
    const int key = valid ? w.qk[i] : 0;
    const double s = valid ? w.qs[i] : 0.0;
    uint32_t slot = 0;
    bool ok = valid;
    if (valid) {
      slot = wg_slot(w.keys, w.acc, T, (uint32_t)(((uint64_t)hash32((uint32_t)key) * T) >> 32), key,
                     reinterpret_cast<uint32_t*>(&w.misc[M_FILL]), budget);
      ok = slot != 0xffffffffu;
      if (!ok) { w.misc[M_OVF] = 1; slot = 0; }
    }
    wave_fence();
    apply_group(w.acc, ok, slot, s, factor, 32 - __clz((int)T - 1));
  }
  __syncthreads();
}

// block-wide radix select of the top-`need` (score desc, tie_w desc) among n entries in LDS.
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
                                                 ValAt valat, Occ occ, uint32_t ts) {
  SelCrit c;
  if (PPR_SEL_REG && n <= 4 * WAVE) {
    // (round 6) few entries: one wave selects with the values in registers (ppr_device.h
    // select_top_reg, no histogram passes) and publishes the criterion
    uint64_t* pub = reinterpret_cast<uint64_t*>(w.hist);
    if (threadIdx.x < WAVE) {
      c = select_top_reg(n, need, keyat, valat, ts, occ);
      if (threadIdx.x == 0) { pub[0] = c.pa; pub[1] = c.ma; pub[2] = c.pb; pub[3] = c.mb; pub[4] = c.tie ? 1ull : 0ull; }
    }
    __syncthreads();
    c.pa = pub[0]; c.ma = pub[1]; c.pb = pub[2]; c.mb = pub[3]; c.tie = pub[4] != 0ull;
    __syncthreads();  // (ends on a barrier like the radix path: the histogram region is free again)
    return c;
  }
  c.tie = false; c.pb = 0; c.mb = 0;
  int k = need;
  bool tie = false;
  wg_radix_kth(w, n, k, [&](int i) { return dbits(valat(i)); }, occ, c.pa, c.ma, tie);
  if (tie) {
    const uint64_t pa = c.pa;
    bool tie2 = false;
    wg_radix_kth(w, n, k, [&](int i) { return (uint64_t)tie_w(keyat(i), ts); },
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


constexpr int WG_T = 10240;           // workgroup table slots (12 B each)
constexpr int WG_PASS_CAP = 6144;     // expected distinct keys per pass when sizing P
constexpr int WG_MAX_PASSES = 64;

// Accumulate one ordered candidate stream (`each` calls its callback once per chunk with two
// candidates per lane, in stream order) in P key-bucket passes. On success pk/pv[0..M_PLEN)
// hold the stream's top-L by (score desc, tie_w desc) (all entries when there are fewer).
template <class EachChunk>
__device__ __forceinline__ bool wg_accumulate(const WgLds& L, int P, uint32_t salt, bool seed_here,
                                              int v, double selfval, double factor, int Lw,
                                              EachChunk each) {
  const uint32_t T = WG_T, budget = WG_T - 1024;
  const uint32_t ts = tie_salt(v);
  if (threadIdx.x == 0) { L.misc[M_PLEN] = 0; L.misc[M_OVF] = 0; }
  for (int pass = 0; pass < P; pass++) {
    for (int i = threadIdx.x; i < (int)T; i += blockDim.x) L.keys[i] = EMPTY;
    if (threadIdx.x == 0) L.misc[M_FILL] = 0;
    __syncthreads();
    auto inpass = [&](int key) { return P == 1 || (int)(hash32((uint32_t)key ^ salt) % (uint32_t)P) == pass; };
    if (threadIdx.x == 0 && seed_here && inpass(v)) {
      const uint32_t sl = wg_slot(L.keys, L.acc, T, (uint32_t)(((uint64_t)hash32((uint32_t)v) * T) >> 32), v,
                                  reinterpret_cast<uint32_t*>(&L.misc[M_FILL]), budget);
      L.acc[sl] = selfval;
    }
    __syncthreads();
    each([&](bool v0, int k0, double s0, bool v1, int k1, double s1) {
      wg_route_apply(L, T, budget, v0 && inpass(k0), k0, s0, v1 && inpass(k1), k1, s1, factor);
    });
    if (L.misc[M_OVF]) return false;  // uniform: written before the last barrier
    const int U = L.misc[M_FILL];
    auto occ = [&](int i) { return L.keys[i] != EMPTY; };
    if (U <= Lw) {
      for (int i = threadIdx.x; i < (int)T; i += blockDim.x)
        if (occ(i)) { const int pos = atomicAdd(&L.misc[M_PLEN], 1); L.pk[pos] = L.keys[i]; L.pv[pos] = L.acc[i]; }
    } else {
      const SelCrit c = wg_select_top(L, (int)T, Lw, [&](int i) { return L.keys[i]; },
                                      [&](int i) { return L.acc[i]; }, occ, ts);
      for (int i = threadIdx.x; i < (int)T; i += blockDim.x) {
        if (!occ(i)) continue;
        const int key = L.keys[i];
        if (sel_test(c, dbits(L.acc[i]), tie_w(key, ts))) {
          const int pos = atomicAdd(&L.misc[M_PLEN], 1);
          L.pk[pos] = key;
          L.pv[pos] = L.acc[i];
        }
      }
    }
    __syncthreads();
    if (L.misc[M_PLEN] > Lw && threadIdx.x < WAVE) {  // fold the running list back to L
      const int n = L.misc[M_PLEN];
      const int* pk = L.pk;
      const double* pv = L.pv;
      const SelCrit c = select_top(n, Lw, [&](int i) { return pk[i]; }, [&](int i) { return pv[i]; }, L.hist, ts);
      int base = 0;
      for (int i0 = 0; i0 < n; i0 += WAVE) {
        const int i = i0 + lane_id();
        bool sel = false;
        if (i < n) sel = sel_test(c, dbits(pv[i]), tie_w(pk[i], ts));
        const uint64_t m = __ballot(sel);
        if (sel) { const int pos = base + __popcll(m & lanemask_lt()); L.rv[pos] = dbits(pv[i]); L.rk[pos] = pk[i]; }
        base += __popcll(m);
      }
      wave_fence();
      for (int i = lane_id(); i < Lw; i += WAVE) { L.pk[i] = L.rk[i]; L.pv[i] = bitsd(L.rv[i]); }
      if (lane_id() == 0) L.misc[M_PLEN] = Lw;
    }
    __syncthreads();
  }
  return true;
}

// the ordered candidate stream of source v read from the basket slab: windows of 512
// successors (block prefix scan of their basket lengths), chunks of 1024 candidates, the next
// chunk's gathers issued before the current chunk is routed
template <class F>
__device__ __forceinline__ void wg_slab_stream(const WgLds& L, const DevGraph& g, const DevSlab& s,
                                               const IterArgs& a, int v, F fn) {
  const int wv = threadIdx.x >> 6;
  const int l = lane_id();
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  if (a.unit) {
    const int64_t deg = e - b;
    for (int64_t c0 = 0; c0 < deg; c0 += WG_CHUNK) {
      const int64_t q0 = c0 + wv * 128 + l, q1 = q0 + 64;
      const bool v0 = q0 < deg, v1 = q1 < deg;
      fn(v0, v0 ? (g.colx[b + q0] & 0x7fffffff) : 0, 1.0, v1, v1 ? (g.colx[b + q1] & 0x7fffffff) : 0, 1.0);
    }
    return;
  }
  for (int64_t wb = b; wb < e; wb += WG_WIN) {
    const int64_t i = wb + threadIdx.x;
    int u = 0, sl = 0, ln = 0;
    if (i < e) {
      const int32_t cx = g.colx[i];
      u = cx & 0x7fffffff;
      sl = read_slot(a, cx);
      ln = s.len[s.lrow(sl, u)];
    }
    const int incl = wg_incl_scan(ln, L.cnt);
    L.wpre[threadIdx.x] = incl;
    L.wu[threadIdx.x] = u;
    L.wsl[threadIdx.x] = sl;
    __syncthreads();
    const int W = L.wpre[WG_WIN - 1];
    auto fetch = [&](int q, bool& vv, int& kk, double& ss) {
      vv = q < W;
      kk = 0;
      ss = 0.0;
      if (vv) {
        int j = 0;
#pragma unroll
        for (int step = WG_WIN / 2; step; step >>= 1)
          if (L.wpre[j + step - 1] <= q) j += step;
        const int ex = j > 0 ? L.wpre[j - 1] : 0;
        const int64_t r = s.row(L.wsl[j], L.wu[j]) + (q - ex);
        kk = s.key(s.ids[r]);
        ss = s.sc[r];
      }
    };
    bool nv0, nv1;
    int nk0, nk1;
    double ns0, ns1;
    fetch(wv * 128 + l, nv0, nk0, ns0);
    fetch(wv * 128 + 64 + l, nv1, nk1, ns1);
    for (int c0 = 0; c0 < W; c0 += WG_CHUNK) {
      const bool cv0 = nv0, cv1 = nv1;
      const int ck0 = nk0, ck1 = nk1;
      const double cs0 = ns0, cs1 = ns1;
      if (c0 + WG_CHUNK < W) {
        fetch(c0 + WG_CHUNK + wv * 128 + l, nv0, nk0, ns0);
        fetch(c0 + WG_CHUNK + wv * 128 + 64 + l, nv1, nk1, ns1);
      }
      fn(cv0, ck0, cs0, cv1, ck1, cs1);
    }
    __syncthreads();  // window arrays are rewritten next
  }
}

// one workgroup (8 waves) per source read from the slab
static __global__ void __launch_bounds__(WG_THREADS) k_merge_wg(DevGraph g, DevSlab s, IterArgs a,
                                                         const int32_t* list, int64_t count,
                                                         const int32_t* cand, int Lp,
                                                         unsigned long long* maxdiff,
                                                         unsigned long long* stats,
                                                         int32_t* ovf_list, uint32_t* ovf_cnt, int max_passes) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t w = blockIdx.x;
  if (w >= count) return;
  const WgLds L = wg_carve(smem, WG_T, Lp, wg_pl(Lp));
  const int v = list[w];
  const int64_t deg = g.rp[v + 1] - g.rp[v];
  const double factor = merge_factor(a, deg);
  int P = (cand[v] + WG_PASS_CAP - 1) / WG_PASS_CAP;
  if (P > max_passes) {  // (PPR_WG_PASSES below the pass count a source needs: tests of the overflow path)
    if (threadIdx.x == 0) { const uint32_t pos = atomicAdd(ovf_cnt, 1u); ovf_list[pos] = v; }
    return;
  }
  for (;;) {
    const bool ok = wg_accumulate(L, P, 0x9e3779b9u, true, v, self_seed(a, deg), factor, s.L,
                                  [&](auto&& fn) { wg_slab_stream(L, g, s, a, v, fn); });
    if (ok) break;
    P *= 2;
    if (P > max_passes) {
      if (threadIdx.x == 0) { const uint32_t pos = atomicAdd(ovf_cnt, 1u); ovf_list[pos] = v; }
      return;
    }
  }
  if (threadIdx.x < WAVE) {
    const int n = L.misc[M_PLEN];
    const int* pk = L.pk;
    const double* pv = L.pv;
    finish_source(v, n, [&](int i) { return pk[i]; }, [&](int i) { return pv[i]; }, s, a, L.hist,
                  L.rv, L.rk, Lp, L.hk, L.hv, L.mf, maxdiff, stats);
  }
}

}  // namespace pprk
