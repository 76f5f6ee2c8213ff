// merge_xg.h -- exact-sum merge of a source of any size in one HBM table (the fallback of the
// exact-sum hub engines). The bucket partition (run_hubs) splits a source into at most
// 2^hub_max_logp buckets of one workgroup table each, so a source with more distinct keys than
// 2^hub_max_logp x (table budget) -- about 28 M keys at xr_T = 8192, 3.4 M at L = 4096 -- can not be
// partitioned; it comes here instead of failing. Same sum as every other exact engine
// (merge_xs.h: X = sum of floor(p * 2^93) per key, split into A = sum of the low 32 bits and
// B = sum of X >> 32), so the row is bit-identical to theirs and to oracle/grank_oracle.c.
//
//   k_xg_walk     every wave walks 64 successors of the source (hub_window_walk) and adds each
//                 candidate to the HBM table (find-or-insert, linear probing; the table has
//                 >= 2 x candidates slots, so it never fills)
//   k_xg_hist     histogram of one 12-bit digit of the 96-bit selection key
//                 (score bits << 32 | tie_w(key, tie_salt(v))) over the table's keys that share
//                 the digits fixed so far
//   k_xg_pick     fixes the digit that holds the L-th largest key; once the keys at or above the
//                 fixed prefix number at most `cap` (<= XG_CAP, >= L) the search stops (at the
//                 latest after the 8th digit: the 96-bit key is unique, so fewer than L keys lie
//                 above the prefix and one in it)
//   k_xg_compact  the keys at or above that prefix into a dense list (<= XG_CAP)
//   k_xg_fin      finish_source on the dense list (select top-L, row, norm1, maxDiff)
// The planner (grank.hip run_xg) runs them for one source at a time on the plan stream.
#pragma once
#include "merge_xs.h"

namespace pprk {

constexpr int XG_DIGIT = 12;
constexpr int XG_BINS = 1 << XG_DIGIT;
constexpr int XG_LEVELS = 8;            // 96-bit key / 12-bit digits
constexpr int XG_CAP = 1 << 16;         // dense list entries (PPR_XG_CAP, tests: fewer, >= L)

struct XgState {
  unsigned long long pv;  // fixed prefix: score bits
  uint32_t pt;            //               tie_w bits
  int32_t done;           // prefix found (keys >= it: at most XG_CAP)
  long long need;         // keys still to take below the fixed prefix
  long long above;        // keys above the prefix's digits (already in)
  int32_t cnt;            // dense entries (k_xg_compact)
  int32_t err;            // table full (cannot happen: >= 2 x candidates slots)
};

__device__ __forceinline__ unsigned __int128 xg_key(double val, int key, uint32_t ts) {
  return ((unsigned __int128)dbits(val) << 32) | (unsigned __int128)tie_w(key, ts);
}
__device__ __forceinline__ unsigned __int128 xg_prefix(const XgState& st) {
  return ((unsigned __int128)st.pv << 32) | (unsigned __int128)st.pt;
}

// global find-or-insert (linear probing over T slots, -1 when full)
__device__ __forceinline__ int64_t xg_slot(uint32_t* keys, int64_t T, int key) {
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
__device__ __forceinline__ void xg_add(uint32_t* keys, unsigned long long* A, unsigned long long* B, int64_t T,
                                       int key, double p, XgState* st, int F) {
  unsigned long long lo;
  uint32_t hi;
  xs_conv(p, lo, hi, F);
  const int64_t h = xg_slot(keys, T, key);
  if (h < 0) { st->err = 1; return; }
  atomicAdd(&A[h], lo & 0xffffffffull);
  atomicAdd(&B[h], (lo >> 32) | ((unsigned long long)hi << 32));
}

// 4 waves a block, one window of 64 successors each
__global__ void __launch_bounds__(256) k_xg_walk(DevGraph g, DevSlab s, IterArgs a, int v, int64_t T, uint32_t* keys,
                                                 unsigned long long* A, unsigned long long* B, XgState* st) {
  __shared__ __align__(16) uint8_t fl[4 * HUB_WALK_FLAGS];
  const int wv = threadIdx.x >> 6;
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = merge_factor(a, e - b);
  const int64_t w0 = b + ((int64_t)blockIdx.x * 4 + wv) * WAVE;
  if (blockIdx.x == 0 && threadIdx.x == 0) xg_add(keys, A, B, T, v, self_seed(a, e - b), st, a.xsf);
  if (w0 >= e) return;
  hub_window_walk(g, s, a, w0, min(e, w0 + WAVE), fl + wv * HUB_WALK_FLAGS, [&](bool valid, int id, double sv, bool) {
    if (valid) xg_add(keys, A, B, T, a.unit ? id : s.key(id), sv * factor, st, a.xsf);
  });
}

__global__ void __launch_bounds__(1024) k_xg_hist(int v, int64_t T, const uint32_t* keys, const unsigned long long* A,
                                                  const unsigned long long* B, const XgState* st, int level,
                                                  uint32_t* ghist, int F) {
  __shared__ uint32_t h[XG_BINS];
  if (st->done) return;
  for (int i = threadIdx.x; i < XG_BINS; i += blockDim.x) h[i] = 0u;
  __syncthreads();
  const uint32_t ts = tie_salt(v);
  const unsigned __int128 P = xg_prefix(*st);
  const int top = 96 - XG_DIGIT * level;  // bits above `top` are fixed
  const int sh = top - XG_DIGIT;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t kt = keys[i];
    if (!kt) continue;
    const unsigned __int128 k = xg_key(x2_value(A[i], B[i], F), (int)kt - 1, ts);
    if (level > 0 && (k >> top) != (P >> top)) continue;
    atomicAdd(&h[(uint32_t)(k >> sh) & (XG_BINS - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < XG_BINS; i += blockDim.x)
    if (h[i]) atomicAdd(&ghist[i], h[i]);
}

// one block: fix this level's digit, clear the histogram for the next level
__global__ void __launch_bounds__(256) k_xg_pick(XgState* st, int level, uint32_t* ghist, int L, int cap) {
  __shared__ int go;
  if (threadIdx.x == 0) {
    go = 0;
    if (level == 0) { st->need = L; st->above = 0; st->pv = 0ull; st->pt = 0u; st->done = 0; st->cnt = 0; }
    if (!st->done) {
      go = 1;
      long long total = 0;
      for (int i = 0; i < XG_BINS; i++) total += ghist[i];
      if (st->above + total <= cap) {
        st->done = 1;  // every key of the region fits: take them all, the select does the rest
      } else {
        long long cum = 0;
        int bsel = 0;
        for (int i = XG_BINS - 1; i >= 0; i--) {
          if (cum + (long long)ghist[i] >= st->need) { bsel = i; break; }
          cum += ghist[i];
        }
        st->above += cum;
        st->need -= cum;
        const int sh = 96 - XG_DIGIT * (level + 1);
        unsigned __int128 P = xg_prefix(*st) | ((unsigned __int128)(uint32_t)bsel << sh);
        st->pv = (unsigned long long)(P >> 32);
        st->pt = (uint32_t)P;
        if (st->above + (long long)ghist[bsel] <= cap || level == XG_LEVELS - 1) st->done = 1;
      }
    }
  }
  __syncthreads();
  if (go)
    for (int i = threadIdx.x; i < XG_BINS; i += blockDim.x) ghist[i] = 0u;
}

__global__ void __launch_bounds__(256) k_xg_compact(int v, int64_t T, const uint32_t* keys, const unsigned long long* A,
                                                    const unsigned long long* B, XgState* st, int32_t* dk,
                                                    double* dv, int F) {
  const uint32_t ts = tie_salt(v);
  const unsigned __int128 P = xg_prefix(*st);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t kt = keys[i];
    bool keep = false;
    double val = 0.0;
    if (kt) {
      val = x2_value(A[i], B[i], F);
      keep = xg_key(val, (int)kt - 1, ts) >= P;
    }
    if (keep) {
      const int pos = atomicAdd(&st->cnt, 1);
      if (pos < XG_CAP) { dk[pos] = (int)kt - 1; dv[pos] = val; }
    }
  }
}

// one wave: finish_source over the dense list (global), scratch in LDS
__host__ __device__ constexpr size_t xg_fin_lds_bytes(int Lp) { return 1024 + (size_t)Lp * 32; }
__global__ void __launch_bounds__(64) k_xg_fin(DevSlab s, IterArgs a, int v, const XgState* st, const int32_t* dk,
                                               const double* dv, int Lp, unsigned long long* maxdiff,
                                               unsigned long long* stats, int32_t* err) {
  extern __shared__ __align__(16) unsigned char smem[];
  unsigned char* p = smem;
  uint32_t* hist = reinterpret_cast<uint32_t*>(p); p += 1024;
  uint64_t* rv = reinterpret_cast<uint64_t*>(p); p += (size_t)Lp * 8;
  int* rk = reinterpret_cast<int*>(p); p += (size_t)Lp * 4;
  int* hk = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  int* hv = reinterpret_cast<int*>(p); p += (size_t)Lp * 8;
  int* mf = reinterpret_cast<int*>(p);
  if (st->err || st->cnt > XG_CAP || !st->done) {
    if (lane_id() == 0) *err = 1;
    return;
  }
  finish_source(v, st->cnt, [&](int i) { return dk[i]; }, [&](int i) { return dv[i]; }, s, a, hist, rv, rk, Lp, hk, hv,
                mf, maxdiff, stats);
}

}  // namespace pprk
