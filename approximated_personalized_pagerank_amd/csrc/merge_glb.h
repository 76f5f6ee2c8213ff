// merge_glb.h -- last-resort path: one wave per source with its hash table in HBM scratch
// (one successor basket per step; the keys of one basket are distinct, so lanes never collide
// within a step and the per-key order is the successor order). Used only for sources whose
// key-bucket passes still overflow the workgroup table, and for tier tests.
#pragma once
#include "ppr_common.h"

namespace pprk {

// ---------------------------------------------------------------------------------------------
// big sources: one wave per source, table in HBM scratch (per-source region of T slots)

// out[i] = src[list[i]]
__global__ void __launch_bounds__(256) k_gather_i32(const int32_t* list, int64_t count, const int32_t* src,
                                                    int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = src[list[i]];
}

// hub planning inputs, gathered so the host walks them sequentially: candidate counts and
// out-degrees of the listed sources (out[0..count) | out[count..2 count))
__global__ void __launch_bounds__(256) k_gather_cand_deg(const int32_t* list, int64_t count, const int32_t* cand,
                                                         const int64_t* rp, int32_t* out,
                                                         const int32_t* dlast = nullptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int v = list[i];
  out[i] = cand[v];
  out[count + i] = (int32_t)(rp[v + 1] - rp[v]);
  if (dlast) out[2 * count + i] = dlast[v];  // exact-sum planning: distinct keys of the last merge
}

// the same gather with the hub count read on the device (at most cap), for the fused small-level
// path: everything the host needs after a classification lands in ONE buffer, so it comes back in
// one copy: out[0, ncnt) = the tier counters, out[ncnt] = the previous level's deferred overflow
// count (*pend_p, 0 without one), then from out + GATHER_HDR: the hub list (cap slots), its
// candidate counts (nh) and its out-degrees (nh)
constexpr int GATHER_HDR = 16;
__global__ void __launch_bounds__(256) k_gather_cand_deg_dev(const int32_t* list, const uint32_t* tier_cnt, int ncnt,
                                                             int tier_big, const int32_t* pend_p, int64_t cap,
                                                             const int32_t* cand, const int64_t* rp, int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < GATHER_HDR)
    out[threadIdx.x] = (int)threadIdx.x < ncnt ? (int32_t)tier_cnt[threadIdx.x]
                       : ((int)threadIdx.x == ncnt && pend_p ? *pend_p : 0);
  const int64_t nh = min((int64_t)tier_cnt[tier_big], cap);
  if (i >= nh) return;
  const int v = list[i];
  int32_t* o = out + GATHER_HDR;
  o[i] = v;
  o[cap + i] = cand[v];
  o[cap + nh + i] = (int32_t)(rp[v + 1] - rp[v]);
}

__global__ void __launch_bounds__(64) k_merge_glb(DevGraph g, DevSlab s, IterArgs a,
                                                  const GlbWork* work, int64_t count,
                                                  int32_t* gkeys, double* gacc, int32_t* ckeys,
                                                  double* cacc, int Lp,
                                                  unsigned long long* maxdiff,
                                                  unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t w = blockIdx.x;
  if (w >= count) return;
  const GlbWork wk = work[w];
  const int v = wk.v;
  int32_t* keys = gkeys + wk.off;
  double* acc = gacc + wk.off;
  const uint64_t mask = (uint64_t)wk.T - 1;
  uint64_t* rv = reinterpret_cast<uint64_t*>(smem);
  int* rk = reinterpret_cast<int*>(smem + (size_t)Lp * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + (size_t)Lp * 12);
  int* hk = reinterpret_cast<int*>(smem + (size_t)Lp * 12 + 1024);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;

  for (int64_t i = lane_id(); i < wk.T; i += WAVE) keys[i] = EMPTY;
  __threadfence_block();
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = merge_factor(a, e - b);

  auto slot_of = [&](int key) -> uint64_t {
    uint64_t h = hash32((uint32_t)key) & mask;
    for (uint64_t n = 0; n <= mask; n++) {
      const int prev = atomicCAS(&keys[h], EMPTY, key);
      if (prev == EMPTY) {
        __hip_atomic_store(&acc[h], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return h;
      }
      if (prev == key) return h;
      h = (h + 1) & mask;
    }
    probe_fail();  // (>= 2 x candidates slots: cannot happen)
    return (uint64_t)0;
  };
  if (lane_id() == 0) {
    const uint64_t h = slot_of(v);
    __hip_atomic_store(&acc[h], self_seed(a, e - b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __threadfence_block();
  // one successor basket per step: its keys are distinct, so lanes never collide within a step
  for (int64_t i = b; i < e; i++) {
    const int32_t cx = g.colx[i];
    const int u = cx & 0x7fffffff;
    int ln;
    int64_t r = 0;
    if (a.unit) ln = 1;
    else { const int sl = read_slot(a, cx); ln = s.len[s.lrow(sl, u)]; r = s.row(sl, u); }
    for (int j = lane_id(); j < ln; j += WAVE) {
      const int key = a.unit ? u : s.key(s.ids[r + j]);
      const double sv = a.unit ? 1.0 : s.sc[r + j];
      const uint64_t h = slot_of(key);
      const double cur = __hip_atomic_load(&acc[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&acc[h], fma(sv, factor, cur), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __threadfence_block();
  }
  // compact into ckeys/cacc
  int32_t* ck = ckeys + wk.off;
  double* ca = cacc + wk.off;
  int U = 0;
  for (int64_t base = 0; base < wk.T; base += WAVE) {
    const int64_t i = base + lane_id();
    const int k = __hip_atomic_load(&keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool occ = k != EMPTY;
    const uint64_t m = __ballot(occ);
    if (occ) {
      const int pos = U + __popcll(m & lanemask_lt());
      ck[pos] = k;
      ca[pos] = __hip_atomic_load(&acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    U += __popcll(m);
  }
  __threadfence_block();
  finish_source(v, U, [&](int i) { return ck[i]; }, [&](int i) { return ca[i]; }, s, a, hist, rv,
                rk, Lp, hk, hv, mf, maxdiff, stats);
}

// ---------------------------------------------------------------------------------------------
// final top-K (include/grank.h:143-147): the stored row is in hash order, so each wave loads it
// into LDS, keeps its top-K by the top-L rule (score desc, tie_w desc) and writes them by (score
// desc, id asc)
__global__ void __launch_bounds__(256) k_topk(DevSlab s, const uint8_t* part, int sA, int sB, int K, int Lp,
                                              int32_t* oid, double* osc, int32_t* olen, const int8_t* owner,
                                              int rank) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int64_t v = (int64_t)blockIdx.x * (blockDim.x / WAVE) + wv;
  if (v >= s.n) return;
  // sharded run: this rank's own rows and the dangling nodes' (identical everywhere) only -- the
  // others' rows are stale here, their top-K arrive from their owners (grank.hip x_gather_topk)
  if (owner && owner[v] >= 0 && owner[v] != rank) return;
  uint64_t* rv = reinterpret_cast<uint64_t*>(smem) + (size_t)wv * Lp;
  int* rk = reinterpret_cast<int*>(smem + (size_t)(blockDim.x / WAVE) * Lp * 8) + (size_t)wv * Lp;
  const int sl = part[v] ? sB : sA;
  const int len = s.len[s.lrow(sl, v)];
  const int k = len < K ? len : K;
  const int64_t r = s.row(sl, v);
  for (int i = lane_id(); i < len; i += WAVE) { rv[i] = dbits(s.sc[r + i]); rk[i] = s.key(s.ids[r + i]); }
  wave_fence();
  if (len > K) {
    // the K kept by the top-L tie rule (keepTop(K), include/grank.h:143-147), then output order
    row_sort(rv, rk, len, Lp, true, tie_salt((int)v));
    row_sort(rv, rk, K, Lp);
  } else {
    row_sort(rv, rk, len, Lp);
  }
  for (int i = lane_id(); i < K; i += WAVE) {
    oid[v * K + i] = i < k ? rk[i] : -1;
    osc[v * K + i] = i < k ? bitsd(rv[i]) : 0.0;
  }
  if (lane_id() == 0) olen[v] = k;
}

// Init of the dangling nodes (no successors): their basket is {v: 1-d} for good (include/grank.h
// :64-83 -- the reference never merges them again), in both slots like every init row
// (finish_source, unit mode), with its row minimum and 64-range index. One thread per (node,
// range): no table, no select -- the merge engines spent as long on these 52 % of RMAT-22's nodes
// as on all the others' init.
__device__ __forceinline__ void init_dangling_one(DevSlab s, const int32_t* list, int64_t t, double seed) {
  const int64_t v = list[t / NRANGE];
  const int q = (int)(t % NRANGE);
  const uint16_t x = row_range((int)v) <= (uint32_t)q ? 1 : 0;
#pragma unroll
  for (int sl = 0; sl < 2; sl++) {
    s.rix[s.xrow(sl, v) + q] = x;
    if (q == 0) {
      const int64_t r = s.row(sl, v);
      s.ids[r] = (int32_t)v;  // (init precedes any hot set: ids are stored as themselves)
      s.sc[r] = seed;
      s.len[s.lrow(sl, v)] = 1;
      s.rmin[s.lrow(sl, v)] = seed;
    }
  }
}
// (grid-stride: cnt * NRANGE work items pass 2^32 at 2^26 nodes)
__global__ void k_init_dangling(DevSlab s, const int32_t* list, int64_t cnt, double seed) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cnt * NRANGE;
       t += (int64_t)gridDim.x * blockDim.x)
    init_dangling_one(s, list, t, seed);
}

// Row exchange for source sharding: one compact block per active-list range of `count` rows (the
// next-slot rows the iteration wrote, in stored order):
//   int64 off[count + 1]                payload offset of row r (off[0] = 0, off[count] = payload bytes)
//   payload: per row int32 ids[Le] f64 scores[len]   (Le = len rounded up to even: 8-B aligned)
// A row of len entries takes 12 len (+4 when len is odd) bytes, so len = (off[r+1] - off[r]) / 12.
// Only the entries travel: the receiver rebuilds the row minimum and the 64-range index from them
// exactly as write_row does (ppr_common.h), so a block is 8 + 12 len bytes per row instead of the
// slab's fixed 4 Le + 8 L + 8 + 128.
__device__ __forceinline__ int64_t xrow_bytes(int len) { return 12 * (int64_t)len + 4 * (len & 1); }

__global__ void k_xsize(DevSlab s, int nxt, const int32_t* list, int64_t count, int64_t* sz) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < count) sz[r] = xrow_bytes(s.len[s.lrow(nxt, list[r])]);
  else if (r == count) sz[r] = 0;
}

// block bytes of a packed range -> *total (the size the ranks exchange before the payload)
__global__ void k_xtotal(const int64_t* off, int64_t count, int64_t* total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *total = 8 * (count + 1) + off[count];
}

// The final top-K rows of a sharded run travel in the same block layout (int64 off[count + 1], then
// per row int32 ids[Le] and f64 scores[len]) from the output arrays: K entries at most a row.
__global__ void k_osize(const int32_t* olen, const int32_t* list, int64_t count, int64_t* sz) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < count) sz[r] = xrow_bytes(olen[list[r]]);
  else if (r == count) sz[r] = 0;
}
__global__ void k_opack(const int32_t* oid, const double* osc, const int32_t* olen, int K, const int32_t* list,
                        int64_t count, unsigned char* buf) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x >> 6);
  if (r >= count) return;
  const int64_t* off = reinterpret_cast<const int64_t*>(buf);
  const int64_t v = list[r];
  const int len = olen[v];
  unsigned char* row = buf + 8 * (count + 1) + off[r];
  int32_t* rid = reinterpret_cast<int32_t*>(row);
  double* rsc = reinterpret_cast<double*>(row + 4 * (int64_t)((len + 1) & ~1));
  for (int i = lane_id(); i < len; i += WAVE) { rid[i] = oid[v * K + i]; rsc[i] = osc[v * K + i]; }
}
__global__ void k_ounpack(int32_t* oid, double* osc, int32_t* olen, int K, const int32_t* list, int64_t count,
                          const unsigned char* buf) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x >> 6);
  if (r >= count) return;
  const int64_t* off = reinterpret_cast<const int64_t*>(buf);
  const int64_t v = list[r];
  const int len = (int)((off[r + 1] - off[r]) / 12);
  const unsigned char* row = buf + 8 * (count + 1) + off[r];
  const int32_t* rid = reinterpret_cast<const int32_t*>(row);
  const double* rsc = reinterpret_cast<const double*>(row + 4 * (int64_t)((len + 1) & ~1));
  for (int i = lane_id(); i < K; i += WAVE) {
    oid[v * K + i] = i < len ? rid[i] : -1;
    osc[v * K + i] = i < len ? rsc[i] : 0.0;
  }
  if (lane_id() == 0) olen[v] = len;
}

__global__ void k_xpack(DevSlab s, int nxt, const int32_t* list, int64_t count, unsigned char* buf) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x >> 6);
  if (r >= count) return;
  const int64_t* off = reinterpret_cast<const int64_t*>(buf);
  const int v = list[r];
  const int len = s.len[s.lrow(nxt, v)];
  unsigned char* row = buf + 8 * (count + 1) + off[r];
  int32_t* rid = reinterpret_cast<int32_t*>(row);
  double* rsc = reinterpret_cast<double*>(row + 4 * (int64_t)((len + 1) & ~1));
  const int64_t src = s.row(nxt, v);
  // blocks carry plain keys: a hot index (HOT_TAG | index) is this rank's own encoding, and each
  // rank builds its hot set on its own (k_xunpack re-encodes with the receiver's set)
  for (int i = lane_id(); i < len; i += WAVE) { rid[i] = s.key(s.ids[src + i]); rsc[i] = s.sc[src + i]; }
}

__global__ void k_xunpack(DevSlab s, int nxt, const int32_t* list, int64_t count, const unsigned char* buf) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x >> 6);
  if (r >= count) return;
  const int64_t* off = reinterpret_cast<const int64_t*>(buf);
  const int v = list[r];
  const int len = (int)((off[r + 1] - off[r]) / 12);
  const unsigned char* row = buf + 8 * (count + 1) + off[r];
  const int32_t* rid = reinterpret_cast<const int32_t*>(row);
  const double* rsc = reinterpret_cast<const double*>(row + 4 * (int64_t)((len + 1) & ~1));
  const int64_t dst = s.row(nxt, v);
  uint64_t mn = ~0ull;
  for (int i = lane_id(); i < len; i += WAVE) {
    const double x = rsc[i];
    s.ids[dst + i] = s.enc(rid[i]);  // plain key -> this rank's stored id
    s.sc[dst + i] = x;
    const uint64_t b = dbits(x);
    mn = b < mn ? b : mn;
  }
  mn = wave_min_u64(mn);
  // lane q: entries whose key's hash range is <= q (the row ascends in hash_b order)
  const uint32_t q = (uint32_t)lane_id();
  int lp = 1;
  while (lp < len) lp <<= 1;
  int pos = 0;
  for (int b = lp; b; b >>= 1)
    if (pos + b <= len && row_range(rid[pos + b - 1]) <= q) pos += b;
  s.rix[s.xrow(nxt, v) + q] = (uint16_t)pos;
  if (lane_id() == 0) {
    s.len[s.lrow(nxt, v)] = len;
    s.rmin[s.lrow(nxt, v)] = len ? bitsd(mn) : 0.0;
  }
}

// ---- consumer routing of the sharded loop's rows (grank.hip xroute_build) ----
// work-balanced range bounds of one partition's active list (at most 32 ranks: a u32 mask per node)
struct XBounds {
  int64_t b[33];
  int32_t world;
};
// owner rank of every active node of one partition's list
__global__ void k_xowner(const int32_t* act, int64_t cnt, XBounds xb, int8_t* owner) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cnt) return;
  int r = 0;
  while (r + 1 < xb.world && xb.b[r + 1] <= i) r++;
  owner[act[i]] = (int8_t)r;
}
// bit r of cmask[u]: some source merged by rank r (in either partition) reads u's row. One wave per
// source; a bit already set is not or-ed again (a popular row would otherwise serialise millions
// of atomics on one address).
__global__ void k_xcmask(const int64_t* rp, const int32_t* colx, int64_t n, const int8_t* owner, uint32_t* cmask) {
  const int64_t v = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x >> 6);
  if (v >= n) return;
  const int r = owner[v];
  if (r < 0) return;
  const uint32_t bit = 1u << r;
  for (int64_t e = rp[v] + lane_id(); e < rp[v + 1]; e += WAVE) {
    const int u = colx[e] & 0x7fffffff;
    if (!(__hip_atomic_load(&cmask[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(&cmask[u], bit);
  }
}
// hipcub::DeviceSelect::If predicate: the node's row is read by rank `bit`
struct XConsumedBy {
  const uint32_t* m;
  uint32_t bit;
  __host__ __device__ bool operator()(const int32_t& v) const { return (m[v] & bit) != 0u; }
};

__global__ void k_zero_u64(unsigned long long* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0ull;
}


}  // namespace pprk
