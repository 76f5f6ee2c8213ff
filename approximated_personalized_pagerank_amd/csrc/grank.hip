// grank.hip -- MI355X (gfx950) GRank engine: basket-merge kernels + the C ABI of include/ppr_hip.h.
//
// Hot path: for every active source v of the iteration's partition
//     B'[v] = topL( {v: 1-d} (+) sum_{u in succ(v), in order} (d/deg v) * B[u] )
// (reference include/grank.h:96-126, header-only/grankMulti.h:230-268), followed by
// maxDiff = max_v norm1(B'[v], B[v]) (include/grank.h:123).
//
// HBM layout (DESIGN.md "data layout"):
//   rp   int64 [n+1]        CSR row pointers (dense ids = graph iteration order)
//   colx int32 [m]          successor id | partition-of-successor << 31
//   ids  int32 [2][n][L]    basket slab, two slots per node (ping-pong per partition)
//   sc   f64   [2][n][L]
//   len  int32 [2][n]
// A node of partition p has been updated upd(p,it) = p ? it/2 : (it+1)/2 times before
// iteration `it`; its current basket lives in slot upd & 1, an active node writes slot upd^1.
// Nothing is copied for the inactive partition (include/grank.h:133-134 becomes a slot choice).
//
// Kernels per iteration:
//   k_classify    one wave per active source: C_v = sum len[u] -> tier lists (LDS table size)
//   k_merge_lds   one wave per source, LDS hash table sized by tier, owner-round accumulation in
//                 successor order, radix top-L select, bitonic row sort, norm1, write row
//   k_merge_glb   sources whose candidates exceed the largest LDS tier: same algorithm with the
//                 table in HBM scratch, one successor basket per step (keys unique per basket)
// Init (include/grank.h:64-83) runs the same kernels in UNIT mode: every successor contributes
// the basket {u: 1.0}, and fma(1.0, f, acc) == acc + f reproduces `scores[v][s] += factor`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/ppr_hip.h"
#include "ppr_device.h"
#include "wg_merge.h"

using namespace pprd;

#define HIP_OK(expr)                                  \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) {                           \
      fprintf(stderr, "ppr_hip: %s failed: %s (%s:%d)\n", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
      return PPR_ERR_HIP;                             \
    }                                                 \
  } while (0)

namespace {

constexpr int NT = 4;                 // single-wave LDS table tiers
constexpr int TIER_WG = NT;           // workgroup tier (k_merge_wg)
constexpr int TIER_BIG = NT + 1;      // beyond the workgroup tier
constexpr int NLISTS = NT + 2;
constexpr int WG_T = 7168;            // workgroup table slots
constexpr int WG_PASS_CAP = 4096;     // expected distinct keys per key-bucket pass
constexpr int WG_PL = 1024;           // partial-list entries (P * L)
constexpr int MAX_L = 4096;           // widest basket the kernels accept
constexpr int WAVES_PER_BLOCK = 4;

struct DevGraph {
  const int64_t* rp;
  const int32_t* colx;
  int64_t n;
};

struct DevSlab {
  int32_t* ids;
  double* sc;
  int32_t* len;
  int64_t n;
  int32_t L;
  __device__ __forceinline__ int64_t row(int slot, int64_t u) const { return ((int64_t)slot * n + u) * L; }
  __device__ __forceinline__ int64_t lrow(int slot, int64_t u) const { return (int64_t)slot * n + u; }
};

struct IterArgs {
  int sA, sB;        // read slot of partition 0 / 1 nodes
  int active;        // partition updated in this iteration (-1 = init)
  double damping;
  uint32_t unit;     // init mode
  uint32_t stats;
};

__device__ __forceinline__ int read_slot(const IterArgs& a, int32_t cx) { return (cx < 0) ? a.sB : a.sA; }

// ---------------------------------------------------------------------------------------------
// classification: C_v = number of candidates of source v (+1 for its own key)
__global__ void __launch_bounds__(256) k_classify(DevGraph g, DevSlab s, IterArgs a,
                                                  const int32_t* list, int64_t count,
                                                  const int32_t* tier_cap, int32_t* tier_lists,
                                                  uint32_t* tier_cnt, int64_t list_cap,
                                                  int32_t* cand, unsigned long long* stats) {
  __shared__ unsigned long long red[2][WAVES_PER_BLOCK];
  const int wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wv;
  unsigned long long my_c = 0, my_b = 0;
  if (w < count) {
    const int v = list[w];
    const int64_t b = g.rp[v], e = g.rp[v + 1];
    int64_t c = 0;
    if (a.unit) {
      c = e - b;
    } else {
      for (int64_t i = b + lane_id(); i < e; i += WAVE) {
        const int32_t cx = g.colx[i];
        c += s.len[s.lrow(read_slot(a, cx), cx & 0x7fffffff)];
      }
#pragma unroll
      for (int o = 32; o; o >>= 1) c += __shfl_xor((long long)c, o);
    }
    if (lane_id() == 0) {
      const int64_t need = c + 1;
      cand[v] = (int32_t)(need > 0x7fffffff ? 0x7fffffff : need);
      int t = 0;
      while (t < NT + 1 && need > tier_cap[t]) t++;
      const uint32_t pos = atomicAdd(&tier_cnt[t], 1u);
      tier_lists[(int64_t)t * list_cap + pos] = v;
      const int ownlen = a.unit ? 0 : s.len[s.lrow(a.active == 0 ? a.sA : a.sB, v)];
      my_c = (unsigned long long)c;
      my_b = (unsigned long long)(8 + 8 * (e - b) + 12 * c + 12 * ownlen);
    }
  }
  if (a.stats) {
    if (lane_id() == 0) { red[0][wv] = my_c; red[1][wv] = my_b; }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long sc = 0, sb = 0;
      for (int i = 0; i < WAVES_PER_BLOCK; i++) { sc += red[0][i]; sb += red[1][i]; }
      if (sc) atomicAdd(&stats[0], sc);
      if (sb) atomicAdd(&stats[1], sb);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// finish one source from a compacted candidate set (keys/vals, U entries, LDS or global):
// select top-L, sort, write the next-slot row, norm1 against the old row, maxDiff.
template <class KeyAt, class ValAt>
__device__ __forceinline__ void finish_source(int v, int U, KeyAt keyat, ValAt valat,
                                              const DevSlab& s, const IterArgs& a, uint32_t* hist,
                                              uint64_t* rv, int* rk, int Lp, int* hk, int* hv,
                                              int* mf, unsigned long long* maxdiff,
                                              unsigned long long* stats) {
  const int L = s.L;
  int cnt;
  if (U <= L) {
    for (int i = lane_id(); i < U; i += WAVE) { rv[i] = dbits(valat(i)); rk[i] = keyat(i); }
    cnt = U;
  } else {
    const SelCrit c = select_top(U, L, keyat, valat, hist);
    int base = 0;
    for (int i0 = 0; i0 < U; i0 += WAVE) {
      const int i = i0 + lane_id();
      bool sel = false;
      uint64_t vb = 0;
      int key = 0;
      if (i < U) { key = keyat(i); vb = dbits(valat(i)); sel = sel_test(c, vb, (uint32_t)~key); }
      const uint64_t m = __ballot(sel);
      if (sel) { const int pos = base + __popcll(m & lanemask_lt()); rv[pos] = vb; rk[pos] = key; }
      base += __popcll(m);
    }
    cnt = L;
  }
  wave_fence();
  row_sort(rv, rk, cnt, Lp);
  const int cur = (a.active == 1) ? a.sB : a.sA;
  if (a.unit) {
    // init: slot 0; dangling sources never update, so their basket is valid in both slots
    const int nslots = 2;
    for (int sl = 0; sl < nslots; sl++) {
      const int64_t r = s.row(sl, v);
      for (int i = lane_id(); i < cnt; i += WAVE) { s.ids[r + i] = rk[i]; s.sc[r + i] = bitsd(rv[i]); }
      if (lane_id() == 0) s.len[s.lrow(sl, v)] = cnt;
    }
    return;
  }
  const int nxt = cur ^ 1;
  const int64_t r = s.row(nxt, v);
  for (int i = lane_id(); i < cnt; i += WAVE) { s.ids[r + i] = rk[i]; s.sc[r + i] = bitsd(rv[i]); }
  if (lane_id() == 0) s.len[s.lrow(nxt, v)] = cnt;
  const int64_t ro = s.row(cur, v);
  const int olen = s.len[s.lrow(cur, v)];
  const double d1 = row_norm1(rv, rk, cnt, s.ids + ro, s.sc + ro, olen, hk, hv, mf, 2 * Lp);
  if (lane_id() == 0) {
    atomicMax(maxdiff, (unsigned long long)dbits(d1));
    if (a.stats) atomicAdd(&stats[1], (unsigned long long)(12 * cnt + 4));
  }
}

// per-wave LDS bytes for table size T and padded width Lp
// layout: acc f64[T] | keys i32[T] | owner u32[T] | rv u64[Lp] | rk i32[Lp] | hist u32[256] |
//         hk i32[2Lp] | hv i32[2Lp] | mf i32[Lp]
__host__ __device__ constexpr size_t lds_wave_bytes(int T, int Lp) {
  return (size_t)T * 16 + (size_t)Lp * 12 + 1024 + (size_t)Lp * 20;
}

// ---------------------------------------------------------------------------------------------
// one wave per source, LDS table of T slots (dynamic LDS: WAVES_PER_BLOCK regions)
__global__ void __launch_bounds__(256) k_merge_lds(DevGraph g, DevSlab s, IterArgs a,
                                                   const int32_t* list, int64_t count, int T,
                                                   int Lp, unsigned long long* maxdiff,
                                                   unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wv;
  if (w >= count) return;
  unsigned char* base = smem + (size_t)wv * lds_wave_bytes(T, Lp);
  LdsTable t;
  t.acc = reinterpret_cast<double*>(base);
  t.keys = reinterpret_cast<int*>(base + (size_t)T * 8);
  t.owner = reinterpret_cast<uint32_t*>(base + (size_t)T * 12);
  t.mask = (uint32_t)T - 1;
  uint64_t* rv = reinterpret_cast<uint64_t*>(base + (size_t)T * 16);
  int* rk = reinterpret_cast<int*>(base + (size_t)T * 16 + (size_t)Lp * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + (size_t)T * 16 + (size_t)Lp * 12);

  const int v = list[w];
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = a.damping / (double)(e - b);

  table_clear(t);
  if (lane_id() == 0) { const uint32_t sl = table_slot(t, v); t.acc[sl] = 1.0 - a.damping; }
  wave_fence();

  if (a.unit) {
    for (int64_t e0 = b; e0 < e; e0 += WAVE) {
      const int64_t i = e0 + lane_id();
      const bool valid = i < e;
      const int key = valid ? (g.colx[i] & 0x7fffffff) : 0;
      table_apply(t, valid, key, 1.0, factor);
    }
  } else {
    for (int64_t e0 = b; e0 < e; e0 += WAVE) {
      const int64_t i = e0 + lane_id();
      int u = 0, sl = 0, ln = 0;
      if (i < e) {
        const int32_t cx = g.colx[i];
        u = cx & 0x7fffffff;
        sl = read_slot(a, cx);
        ln = s.len[s.lrow(sl, u)];
      }
      const int incl = wave_incl_scan(ln);
      const int total = __shfl(incl, WAVE - 1);
      for (int g0 = 0; g0 < total; g0 += WAVE) {
        const int c = g0 + lane_id();
        const bool valid = c < total;
        // successor j = number of window entries whose inclusive prefix is <= c
        int j = 0;
#pragma unroll
        for (int step = 32; step; step >>= 1) {
          const int pv = __shfl(incl, j + step - 1);
          if (pv <= c) j += step;
        }
        const int jj = j < WAVE ? j : WAVE - 1;
        // every lane must execute the bpermute (an inactive source lane reads back 0)
        const int exv = __shfl(incl, jj > 0 ? jj - 1 : 0);
        const int ex = jj > 0 ? exv : 0;
        const int uj = __shfl(u, jj);
        const int sj = __shfl(sl, jj);
        int key = 0;
        double sv = 0.0;
        if (valid) {
          const int64_t r = s.row(sj, uj) + (c - ex);
          key = s.ids[r];
          sv = s.sc[r];
        }
        table_apply(t, valid, key, sv, factor);
      }
    }
  }
  wave_fence();
  const int U = table_compact(t);
  int* hk = reinterpret_cast<int*>(base + (size_t)T * 16 + (size_t)Lp * 12 + 1024);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;
  const int* keys = t.keys;
  const double* acc = t.acc;
  finish_source(v, U, [&](int i) { return keys[i]; }, [&](int i) { return acc[i]; }, s, a, hist,
                rv, rk, Lp, hk, hv, mf, maxdiff, stats);
}

// ---------------------------------------------------------------------------------------------
// one workgroup (8 waves) per source, shared LDS table, P key-bucket passes (wg_merge.h)
__global__ void __launch_bounds__(WG_THREADS) k_merge_wg(DevGraph g, DevSlab s, IterArgs a,
                                                         const int32_t* list, int64_t count,
                                                         const int32_t* cand, int Lp,
                                                         unsigned long long* maxdiff,
                                                         unsigned long long* stats,
                                                         int32_t* ovf_list, uint32_t* ovf_cnt) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t w = blockIdx.x;
  if (w >= count) return;
  const WgLds L = wg_carve(smem, WG_T, Lp, WG_PL);
  const int wv = threadIdx.x >> 6;
  const int l = lane_id();
  const int v = list[w];
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = a.damping / (double)(e - b);
  const int need = cand[v];
  const int P = (need + WG_PASS_CAP - 1) / WG_PASS_CAP;
  const uint32_t T = WG_T, budget = WG_T - 512;
  const int Lw = s.L;
  if (threadIdx.x == 0) { L.misc[M_PLEN] = 0; L.misc[M_OVF] = 0; }

  for (int pass = 0; pass < P; pass++) {
    for (int i = threadIdx.x; i < (int)T; i += WG_THREADS) { L.keys[i] = EMPTY; L.owner[i] = NO_OWNER; }
    if (threadIdx.x == 0) L.misc[M_FILL] = 0;
    __syncthreads();
    if (threadIdx.x == 0 && (P == 1 || (int)(hash_b((uint32_t)v) % (uint32_t)P) == pass)) {
      const uint32_t sl = wg_slot(L.keys, L.acc, T, (uint32_t)(((uint64_t)hash32((uint32_t)v) * T) >> 32), v,
                                  reinterpret_cast<uint32_t*>(&L.misc[M_FILL]), budget);
      L.acc[sl] = 1.0 - a.damping;
    }
    __syncthreads();
    auto inpass = [&](int key) { return P == 1 || (int)(hash_b((uint32_t)key) % (uint32_t)P) == pass; };
    if (a.unit) {
      const int64_t deg = e - b;
      for (int64_t c0 = 0; c0 < deg; c0 += WG_CHUNK) {
        const int64_t q0 = c0 + wv * 128 + l, q1 = q0 + 64;
        const bool v0 = q0 < deg, v1 = q1 < deg;
        const int k0 = v0 ? (g.colx[b + q0] & 0x7fffffff) : 0;
        const int k1 = v1 ? (g.colx[b + q1] & 0x7fffffff) : 0;
        wg_route_apply(L, T, budget, v0 && inpass(k0), k0, 1.0, v1 && inpass(k1), k1, 1.0, factor);
      }
    } else {
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
        for (int c0 = 0; c0 < W; c0 += WG_CHUNK) {
          int kk[2] = {0, 0};
          double ss[2] = {0.0, 0.0};
          bool vv[2] = {false, false};
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int q = c0 + wv * 128 + h * 64 + l;
            if (q < W) {
              int j = 0;
#pragma unroll
              for (int step = WG_WIN / 2; step; step >>= 1)
                if (L.wpre[j + step - 1] <= q) j += step;
              const int ex = j > 0 ? L.wpre[j - 1] : 0;
              const int64_t r = s.row(L.wsl[j], L.wu[j]) + (q - ex);
              kk[h] = s.ids[r];
              ss[h] = s.sc[r];
              vv[h] = inpass(kk[h]);
            }
          }
          wg_route_apply(L, T, budget, vv[0], kk[0], ss[0], vv[1], kk[1], ss[1], factor);
        }
        __syncthreads();  // window arrays are rewritten next
      }
    }
    if (L.misc[M_OVF]) break;  // uniform: read after the last barrier of wg_route_apply
    // this pass's top-L (by the global rule) goes to the partial list
    const int U = L.misc[M_FILL];
    auto occ = [&](int i) { return L.keys[i] != EMPTY; };
    if (U <= Lw) {
      for (int i = threadIdx.x; i < (int)T; i += WG_THREADS)
        if (occ(i)) { const int pos = atomicAdd(&L.misc[M_PLEN], 1); L.pk[pos] = L.keys[i]; L.pv[pos] = L.acc[i]; }
    } else {
      const SelCrit c = wg_select_top(L, (int)T, Lw, [&](int i) { return L.keys[i]; },
                                      [&](int i) { return L.acc[i]; }, occ);
      for (int i = threadIdx.x; i < (int)T; i += WG_THREADS) {
        if (!occ(i)) continue;
        const int key = L.keys[i];
        if (sel_test(c, dbits(L.acc[i]), (uint32_t)~key)) {
          const int pos = atomicAdd(&L.misc[M_PLEN], 1);
          L.pk[pos] = key;
          L.pv[pos] = L.acc[i];
        }
      }
    }
    __syncthreads();
  }
  if (L.misc[M_OVF]) {
    if (threadIdx.x == 0) { const uint32_t pos = atomicAdd(ovf_cnt, 1u); ovf_list[pos] = v; }
    return;
  }
  if (wv == 0) {
    const int n = L.misc[M_PLEN];
    const int* pk = L.pk;
    const double* pv = L.pv;
    finish_source(v, n, [&](int i) { return pk[i]; }, [&](int i) { return pv[i]; }, s, a, L.hist,
                  L.rv, L.rk, Lp, L.hk, L.hv, L.mf, maxdiff, stats);
  }
}

// ---------------------------------------------------------------------------------------------
// big sources: one wave per source, table in HBM scratch (per-source region of T slots)
struct GlbWork {
  int32_t v;
  int32_t pad;
  int64_t off;   // slot offset into the scratch arrays
  int64_t T;     // table slots (power of two)
};

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
  const double factor = a.damping / (double)(e - b);

  auto slot_of = [&](int key) -> uint64_t {
    uint64_t h = hash32((uint32_t)key) & mask;
    for (;;) {
      const int prev = atomicCAS(&keys[h], EMPTY, key);
      if (prev == EMPTY) {
        __hip_atomic_store(&acc[h], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return h;
      }
      if (prev == key) return h;
      h = (h + 1) & mask;
    }
  };
  if (lane_id() == 0) {
    const uint64_t h = slot_of(v);
    __hip_atomic_store(&acc[h], 1.0 - a.damping, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
      const int key = a.unit ? u : s.ids[r + j];
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
// final top-K (include/grank.h:143-147): rows are sorted, so top-K is the first min(K, len)
__global__ void k_topk(DevSlab s, const uint8_t* part, int sA, int sB, int K, int32_t* oid,
                       double* osc, int32_t* olen) {
  const int64_t v = (int64_t)blockIdx.x * (blockDim.x / WAVE) + (threadIdx.x >> 6);
  if (v >= s.n) return;
  const int sl = part[v] ? sB : sA;
  const int len = s.len[s.lrow(sl, v)];
  const int k = len < K ? len : K;
  const int64_t r = s.row(sl, v);
  for (int i = lane_id(); i < K; i += WAVE) {
    oid[v * K + i] = i < k ? s.ids[r + i] : -1;
    osc[v * K + i] = i < k ? s.sc[r + i] : 0.0;
  }
  if (lane_id() == 0) olen[v] = k;
}

__global__ void k_zero_u64(unsigned long long* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0ull;
}

int pow2_at_least(int64_t x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

// ================================================================================================
// plan
struct ppr_plan {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int64_t n = 0, m = 0;
  uint32_t K = 0, L = 0;
  int Lp = 1;
  double damping = 0.85;
  int64_t* d_rp = nullptr;
  int32_t* d_colx = nullptr;
  uint8_t* d_part = nullptr;
  int32_t* d_ids = nullptr;
  double* d_sc = nullptr;
  int32_t* d_len = nullptr;
  int32_t* d_all = nullptr;       // 0..n-1 (init list)
  int32_t* d_act[2] = {nullptr, nullptr};
  int64_t nact[2] = {0, 0};
  int32_t* d_cand = nullptr;
  int32_t* d_tier_lists = nullptr;   // NLISTS * n
  uint32_t* d_tier_cnt = nullptr;    // NLISTS (+1: workgroup overflow count)
  int32_t* d_tier_cap = nullptr;     // NT + 1
  int32_t* d_ovf = nullptr;          // sources the workgroup tier could not hold
  int tierT[NT] = {0, 0, 0, 0};
  int tierCap[NT + 1] = {0, 0, 0, 0, 0};
  size_t wg_lds = 0;
  unsigned long long* d_maxdiff = nullptr;  // PPR_MAX_ITER_STATS + 1
  unsigned long long* d_stats = nullptr;    // 2
  GlbWork* d_work = nullptr;
  int64_t work_cap = 0;
  void* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  int32_t* d_out_ids = nullptr;
  double* d_out_sc = nullptr;
  int32_t* d_out_len = nullptr;
  int flags = 0;
  int64_t merge_launches = 0;
  double merge_ms = 0.0;           // sum of merge-phase spans (classify .. last merge kernel)
  hipEvent_t ev_a = nullptr, ev_b = nullptr, ev_m0 = nullptr, ev_m1 = nullptr;
};

static void plan_free(ppr_plan* p) {
  if (!p) return;
  hipFree(p->d_rp); hipFree(p->d_colx); hipFree(p->d_part); hipFree(p->d_ids); hipFree(p->d_sc);
  hipFree(p->d_len); hipFree(p->d_all); hipFree(p->d_act[0]); hipFree(p->d_act[1]);
  hipFree(p->d_cand); hipFree(p->d_tier_lists); hipFree(p->d_tier_cnt); hipFree(p->d_tier_cap);
  hipFree(p->d_ovf);
  hipFree(p->d_maxdiff); hipFree(p->d_stats); hipFree(p->d_work); hipFree(p->d_scratch);
  hipFree(p->d_out_ids); hipFree(p->d_out_sc); hipFree(p->d_out_len);
  if (p->ev_a) hipEventDestroy(p->ev_a);
  if (p->ev_b) hipEventDestroy(p->ev_b);
  if (p->ev_m0) hipEventDestroy(p->ev_m0);
  if (p->ev_m1) hipEventDestroy(p->ev_m1);
  if (p->own_stream && p->stream) hipStreamDestroy(p->stream);
  delete p;
}

static int check_params(uint32_t K, uint32_t L, uint32_t iterations, double damping) {
  if (K == 0) return PPR_ERR_K;
  if (L == 0) return PPR_ERR_L;
  if (K > L) return PPR_ERR_KL;
  if (iterations == 0) return PPR_ERR_ITERS;
  if (damping < 0 || damping > 1) return PPR_ERR_DAMPING;
  return PPR_OK;
}

template <class T>
static int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, sizeof(T) * count) != hipSuccess) return PPR_ERR_OOM;
  return PPR_OK;
}

#define TRY(x) do { int _r = (x); if (_r != PPR_OK) { plan_free(p); return _r; } } while (0)

extern "C" int ppr_grank_plan_create(const ppr_csr* g, const uint8_t* part_in, uint32_t K,
                                     uint32_t L, double damping, const ppr_opts* o,
                                     ppr_plan** out) {
  if (!g || !out || g->n < 0 || (g->n > 0 && !g->row_ptr)) return PPR_ERR_ARG;
  if (g->n > 0 && g->row_ptr[g->n] > 0 && !g->col) return PPR_ERR_ARG;
  int rc = check_params(K, L, 1, damping);
  if (rc != PPR_OK) return rc;
  if (L > (uint32_t)MAX_L) return PPR_ERR_RANGE;
  if (g->n >= (1LL << 31) - 1) return PPR_ERR_RANGE;
  const int64_t n = g->n;
  const int64_t m = n ? g->row_ptr[n] : 0;
  for (int64_t e = 0; e < m; e++)
    if (g->col[e] < 0 || g->col[e] >= n) return PPR_ERR_GRAPH;
  std::vector<uint8_t> part(n > 0 ? n : 1, 0);
  if (part_in) std::memcpy(part.data(), part_in, n);
  else if (n) { rc = ppr_find_partitions_csr(g, part.data()); if (rc) return rc; }

  ppr_plan* p = new (std::nothrow) ppr_plan();
  if (!p) return PPR_ERR_OOM;
  p->n = n; p->m = m; p->K = K; p->L = L; p->damping = damping;
  p->Lp = pow2_at_least(L);
  p->flags = o ? o->flags : 0;
  p->device = (o && o->device >= 0) ? o->device : -1;
  if (p->device >= 0) { if (hipSetDevice(p->device) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; } }
  else { if (hipGetDevice(&p->device) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; } }
  if (o && o->stream) p->stream = (hipStream_t)o->stream;
  else {
    if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
    p->own_stream = true;
  }
  if (hipEventCreate(&p->ev_a) != hipSuccess || hipEventCreate(&p->ev_b) != hipSuccess ||
      hipEventCreate(&p->ev_m0) != hipSuccess || hipEventCreate(&p->ev_m1) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }

  // tiers: T = 256 << t; capacity 3/4 T; a block of 4 waves must fit the 160 KB LDS
  // PPR_TIER_MASK (diagnostics / tests): bit t enables wave tier t, bit NT the workgroup tier;
  // disabled tiers fall through to the next enabled one, ultimately the HBM-table path
  {
    const char* env = getenv("PPR_TIER_MASK");
    const int mask = env ? (int)strtol(env, nullptr, 0) : 0xff;
    int T0 = 256;
    for (int t = 0; t < NT; t++) {
      const int T = T0 << t;
      if (!((mask >> t) & 1) || lds_wave_bytes(T, p->Lp) * WAVES_PER_BLOCK > 160 * 1024) { p->tierT[t] = 0; p->tierCap[t] = 0; continue; }
      p->tierT[t] = T;
      p->tierCap[t] = T / 4 * 3;
    }
    // workgroup tier: P = ceil(need / WG_PASS_CAP) key-bucket passes with P * L <= WG_PL
    p->tierCap[NT] = 0;
    p->wg_lds = wg_lds_bytes(WG_T, p->Lp, WG_PL);
    const int pmax = WG_PL / (int)L;
    if (((mask >> NT) & 1) && pmax >= 1 && p->wg_lds <= 160 * 1024)
      p->tierCap[NT] = std::min(pmax, 8) * WG_PASS_CAP;
    // a disabled tier has cap 0 (k_classify skips it); enabled caps must be non-decreasing
    int run = 0;
    for (int t = 0; t <= NT; t++) {
      if (!p->tierCap[t]) continue;
      if (p->tierCap[t] < run) p->tierCap[t] = 0;
      else run = p->tierCap[t];
    }
  }

  // host-side CSR with partition bit of the successor
  std::vector<int32_t> colx(m > 0 ? m : 1);
  for (int64_t e = 0; e < m; e++) colx[e] = g->col[e] | (part[g->col[e]] ? (int32_t)0x80000000 : 0);
  std::vector<int32_t> all(n > 0 ? n : 1), act[2];
  for (int64_t v = 0; v < n; v++) {
    all[v] = (int32_t)v;
    if (g->row_ptr[v + 1] > g->row_ptr[v]) act[part[v]].push_back((int32_t)v);
  }
  p->nact[0] = (int64_t)act[0].size();
  p->nact[1] = (int64_t)act[1].size();

  const size_t slab = (size_t)2 * n * L;
  TRY(dalloc(&p->d_rp, n + 1));
  TRY(dalloc(&p->d_colx, m));
  TRY(dalloc(&p->d_part, n));
  TRY(dalloc(&p->d_ids, slab));
  TRY(dalloc(&p->d_sc, slab));
  TRY(dalloc(&p->d_len, 2 * n));
  TRY(dalloc(&p->d_all, n));
  TRY(dalloc(&p->d_act[0], p->nact[0]));
  TRY(dalloc(&p->d_act[1], p->nact[1]));
  TRY(dalloc(&p->d_cand, n));
  TRY(dalloc(&p->d_tier_lists, (size_t)NLISTS * (n > 0 ? n : 1)));
  TRY(dalloc(&p->d_tier_cnt, NLISTS + 1));
  TRY(dalloc(&p->d_tier_cap, NT + 1));
  TRY(dalloc(&p->d_ovf, n));
  TRY(dalloc(&p->d_maxdiff, PPR_MAX_ITER_STATS + 1));
  TRY(dalloc(&p->d_stats, 2));
  TRY(dalloc(&p->d_out_ids, (size_t)n * K));
  TRY(dalloc(&p->d_out_sc, (size_t)n * K));
  TRY(dalloc(&p->d_out_len, n));
  hipStream_t st = p->stream;
  if (n) {
    if (hipMemcpyAsync(p->d_rp, g->row_ptr, 8 * (n + 1), hipMemcpyHostToDevice, st) != hipSuccess ||
        (m && hipMemcpyAsync(p->d_colx, colx.data(), 4 * m, hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipMemcpyAsync(p->d_part, part.data(), n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(p->d_all, all.data(), 4 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        (p->nact[0] && hipMemcpyAsync(p->d_act[0], act[0].data(), 4 * p->nact[0], hipMemcpyHostToDevice, st) != hipSuccess) ||
        (p->nact[1] && hipMemcpyAsync(p->d_act[1], act[1].data(), 4 * p->nact[1], hipMemcpyHostToDevice, st) != hipSuccess)) {
      plan_free(p); return PPR_ERR_HIP;
    }
  }
  int32_t caps[NT + 1];
  for (int t = 0; t <= NT; t++) caps[t] = p->tierCap[t];
  if (hipMemcpyAsync(p->d_tier_cap, caps, sizeof(caps), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) { plan_free(p); return PPR_ERR_HIP; }
  for (int t = 0; t < NT; t++)
    if (p->tierT[t]) {
      const size_t bytes = lds_wave_bytes(p->tierT[t], p->Lp) * WAVES_PER_BLOCK;
      if (bytes > 64 * 1024)
        hipFuncSetAttribute((const void*)k_merge_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    }
  if (p->tierCap[NT])
    hipFuncSetAttribute((const void*)k_merge_wg, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  *out = p;
  return PPR_OK;
}

extern "C" void ppr_grank_plan_destroy(ppr_plan* p) { plan_free(p); }
extern "C" void* ppr_grank_plan_stream(ppr_plan* p) { return p ? (void*)p->stream : nullptr; }

static IterArgs iter_args(const ppr_plan* p, int it, bool unit) {
  IterArgs a;
  a.damping = p->damping;
  a.unit = unit ? 1u : 0u;
  a.stats = (p->flags & PPR_FLAG_STATS) ? 1u : 0u;
  if (unit) { a.sA = 0; a.sB = 0; a.active = -1; return a; }
  a.sA = ((it + 1) / 2) & 1;
  a.sB = (it / 2) & 1;
  a.active = it & 1;
  return a;
}

static int run_merge_impl(ppr_plan* p, const IterArgs& a, const int32_t* list, int64_t count,
                          unsigned long long* maxdiff);

// classify + launch all tiers for `count` sources of `list`; the span is timed with events on
// the plan's stream and added to merge_ms (iterations only, not init)
static int run_merge(ppr_plan* p, const IterArgs& a, const int32_t* list, int64_t count,
                     unsigned long long* maxdiff) {
  if (count <= 0) return PPR_OK;
  HIP_OK(hipEventRecord(p->ev_m0, p->stream));
  int rc = run_merge_impl(p, a, list, count, maxdiff);
  if (rc) return rc;
  HIP_OK(hipEventRecord(p->ev_m1, p->stream));
  HIP_OK(hipEventSynchronize(p->ev_m1));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, p->ev_m0, p->ev_m1));
  if (!a.unit) p->merge_ms += ms;
  return PPR_OK;
}

static int run_merge_impl(ppr_plan* p, const IterArgs& a, const int32_t* list, int64_t count,
                          unsigned long long* maxdiff) {
  hipStream_t st = p->stream;
  DevGraph g{p->d_rp, p->d_colx, p->n};
  DevSlab s{p->d_ids, p->d_sc, p->d_len, p->n, (int32_t)p->L};
  HIP_OK(hipMemsetAsync(p->d_tier_cnt, 0, sizeof(uint32_t) * (NLISTS + 1), st));
  const int64_t nb = (count + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  hipLaunchKernelGGL(k_classify, dim3((unsigned)nb), dim3(256), 0, st, g, s, a, list, count,
                     p->d_tier_cap, p->d_tier_lists, p->d_tier_cnt, p->n, p->d_cand, p->d_stats);
  HIP_OK(hipGetLastError());
  uint32_t cnt[NLISTS + 1];
  HIP_OK(hipMemcpyAsync(cnt, p->d_tier_cnt, sizeof(cnt), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  for (int t = 0; t < NT; t++) {
    if (!cnt[t] || !p->tierT[t]) continue;
    const size_t bytes = lds_wave_bytes(p->tierT[t], p->Lp) * WAVES_PER_BLOCK;
    const int64_t blocks = ((int64_t)cnt[t] + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
    hipLaunchKernelGGL(k_merge_lds, dim3((unsigned)blocks), dim3(256), bytes, st, g, s, a,
                       p->d_tier_lists + (int64_t)t * p->n, (int64_t)cnt[t], p->tierT[t], p->Lp,
                       maxdiff, p->d_stats);
    HIP_OK(hipGetLastError());
    p->merge_launches++;
  }
  if (cnt[TIER_WG]) {
    hipLaunchKernelGGL(k_merge_wg, dim3(cnt[TIER_WG]), dim3(WG_THREADS), p->wg_lds, st, g, s, a,
                       p->d_tier_lists + (int64_t)TIER_WG * p->n, (int64_t)cnt[TIER_WG], p->d_cand,
                       p->Lp, maxdiff, p->d_stats, p->d_ovf, p->d_tier_cnt + NLISTS);
    HIP_OK(hipGetLastError());
    p->merge_launches++;
    HIP_OK(hipMemcpyAsync(&cnt[NLISTS], p->d_tier_cnt + NLISTS, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  // sources beyond the workgroup tier, plus workgroup-tier overflows
  std::vector<int32_t> big;
  auto pull = [&](const int32_t* dptr, uint32_t k) -> int {
    if (!k) return PPR_OK;
    std::vector<int32_t> tmp(k);
    HIP_OK(hipMemcpyAsync(tmp.data(), dptr, 4 * (size_t)k, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    big.insert(big.end(), tmp.begin(), tmp.end());
    return PPR_OK;
  };
  for (int t = 0; t < NT; t++)
    if (cnt[t] && !p->tierT[t]) { int r = pull(p->d_tier_lists + (int64_t)t * p->n, cnt[t]); if (r) return r; }
  { int r = pull(p->d_tier_lists + (int64_t)TIER_BIG * p->n, cnt[TIER_BIG]); if (r) return r; }
  { int r = pull(p->d_ovf, cnt[NLISTS]); if (r) return r; }
  if (big.empty()) return PPR_OK;
  std::vector<int32_t> cand(p->n);
  HIP_OK(hipMemcpyAsync(cand.data(), p->d_cand, 4 * (size_t)p->n, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  // batches bounded by a scratch budget: slots * (4+8) * 2 (table + compacted copy)
  const size_t budget_slots = (size_t)1 << 26;  // 64 Mi slots -> 1.5 GiB
  size_t i0 = 0;
  while (i0 < big.size()) {
    std::vector<GlbWork> work;
    int64_t off = 0;
    size_t i = i0;
    while (i < big.size()) {
      const int64_t T = pow2_at_least(std::max<int64_t>(2 * (int64_t)cand[big[i]], 64));
      if (!work.empty() && (size_t)(off + T) > budget_slots) break;
      work.push_back(GlbWork{big[i], 0, off, T});
      off += T;
      i++;
    }
    const size_t need = (size_t)off * 24;
    if (need > p->scratch_bytes) {
      hipFree(p->d_scratch);
      p->d_scratch = nullptr;
      if (hipMalloc(&p->d_scratch, need) != hipSuccess) return PPR_ERR_OOM;
      p->scratch_bytes = need;
    }
    if ((int64_t)work.size() > p->work_cap) {
      hipFree(p->d_work);
      if (hipMalloc((void**)&p->d_work, sizeof(GlbWork) * work.size()) != hipSuccess) return PPR_ERR_OOM;
      p->work_cap = (int64_t)work.size();
    }
    HIP_OK(hipMemcpyAsync(p->d_work, work.data(), sizeof(GlbWork) * work.size(), hipMemcpyHostToDevice, st));
    int32_t* gkeys = (int32_t*)p->d_scratch;
    double* gacc = (double*)((char*)p->d_scratch + (size_t)off * 4);
    int32_t* ckeys = (int32_t*)((char*)p->d_scratch + (size_t)off * 12);
    double* cacc = (double*)((char*)p->d_scratch + (size_t)off * 16);
    const size_t lds = (size_t)p->Lp * 12 + 1024 + (size_t)p->Lp * 4 * 5;
    hipLaunchKernelGGL(k_merge_glb, dim3((unsigned)work.size()), dim3(64), lds, st, g, s, a,
                       p->d_work, (int64_t)work.size(), gkeys, gacc, ckeys, cacc, p->Lp, maxdiff,
                       p->d_stats);
    HIP_OK(hipGetLastError());
    p->merge_launches++;
    HIP_OK(hipStreamSynchronize(st));  // work/scratch reused by the next batch
    i0 = i;
  }
  return PPR_OK;
}

extern "C" int ppr_grank_plan_init(ppr_plan* p) {
  if (!p) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  IterArgs a = iter_args(p, 0, true);
  return run_merge(p, a, p->d_all, p->n, p->d_maxdiff + PPR_MAX_ITER_STATS);
}

extern "C" int ppr_grank_plan_active_count(ppr_plan* p, int32_t it, int64_t* count) {
  if (!p || !count || it < 0) return PPR_ERR_ARG;
  *count = p->nact[it & 1];
  return PPR_OK;
}

extern "C" int ppr_grank_plan_iterate(ppr_plan* p, int32_t it, int64_t begin, int64_t end) {
  if (!p || it < 0) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  const int part = it & 1;
  begin = std::max<int64_t>(0, begin);
  end = std::min<int64_t>(p->nact[part], end);
  if (end <= begin) return PPR_OK;
  IterArgs a = iter_args(p, it, false);
  unsigned long long* md = p->d_maxdiff + (it < PPR_MAX_ITER_STATS ? it : PPR_MAX_ITER_STATS);
  return run_merge(p, a, p->d_act[part] + begin, end - begin, md);
}

extern "C" int ppr_grank_plan_read_maxdiff(ppr_plan* p, int32_t it, double* maxdiff) {
  if (!p || !maxdiff || it < 0) return PPR_ERR_ARG;
  unsigned long long b = 0;
  HIP_OK(hipMemcpyAsync(&b, p->d_maxdiff + (it < PPR_MAX_ITER_STATS ? it : PPR_MAX_ITER_STATS),
                        8, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  double d;
  std::memcpy(&d, &b, 8);
  *maxdiff = d;
  return PPR_OK;
}

extern "C" int ppr_grank_plan_finish(ppr_plan* p, int32_t iterations_run) {
  if (!p || iterations_run < 0) return PPR_ERR_ARG;
  if (p->n == 0) return PPR_OK;
  HIP_OK(hipSetDevice(p->device));
  const int sA = ((iterations_run + 1) / 2) & 1, sB = (iterations_run / 2) & 1;
  DevSlab s{p->d_ids, p->d_sc, p->d_len, p->n, (int32_t)p->L};
  const int64_t blocks = (p->n + 3) / 4;
  hipLaunchKernelGGL(k_topk, dim3((unsigned)blocks), dim3(256), 0, p->stream, s, p->d_part, sA, sB,
                     (int)p->K, p->d_out_ids, p->d_out_sc, p->d_out_len);
  HIP_OK(hipGetLastError());
  return PPR_OK;
}

extern "C" int ppr_grank_plan_run(ppr_plan* p, uint32_t iterations, double tolerance,
                                  ppr_stats* st) {
  if (!p) return PPR_ERR_ARG;
  if (iterations == 0) return PPR_ERR_ITERS;
  HIP_OK(hipSetDevice(p->device));
  hipStream_t s = p->stream;
  HIP_OK(hipMemsetAsync(p->d_maxdiff, 0, 8 * (PPR_MAX_ITER_STATS + 1), s));
  HIP_OK(hipMemsetAsync(p->d_stats, 0, 16, s));
  p->merge_launches = 0;
  p->merge_ms = 0.0;
  HIP_OK(hipEventRecord(p->ev_a, s));
  int rc = ppr_grank_plan_init(p);
  if (rc) return rc;
  // stopping rule of include/grank.h:90-94,140
  double md[2] = {tolerance, tolerance};
  uint32_t it = 0;
  for (; it < iterations && std::max(md[0], md[1]) >= tolerance; it++) {
    int64_t cnt = p->nact[it & 1];
    rc = ppr_grank_plan_iterate(p, (int32_t)it, 0, cnt);
    if (rc) return rc;
    double d = 0.0;
    if (tolerance > 0 || st) {
      rc = ppr_grank_plan_read_maxdiff(p, (int32_t)it, &d);
      if (rc) return rc;
    }
    md[0] = d;
    std::swap(md[0], md[1]);
    if (st && it < PPR_MAX_ITER_STATS) st->max_diff[it] = d;
  }
  rc = ppr_grank_plan_finish(p, (int32_t)it);
  if (rc) return rc;
  HIP_OK(hipEventRecord(p->ev_b, s));
  HIP_OK(hipEventSynchronize(p->ev_b));
  if (st) {
    float ms = 0;
    hipEventElapsedTime(&ms, p->ev_a, p->ev_b);
    st->iterations_run = (int32_t)it;
    st->device_ms = ms;
    st->merge_ms = p->merge_ms;
    unsigned long long sv[2];
    HIP_OK(hipMemcpyAsync(sv, p->d_stats, 16, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    st->candidates = (int64_t)sv[0];
    st->algo_bytes = (int64_t)sv[1];
    st->merge_launches = p->merge_launches;
  }
  return PPR_OK;
}

extern "C" int ppr_grank_plan_fetch(ppr_plan* p, int32_t* out_ids, double* out_scores,
                                    int32_t* out_len) {
  if (!p) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  const size_t nk = (size_t)p->n * p->K;
  if (out_ids) HIP_OK(hipMemcpyAsync(out_ids, p->d_out_ids, 4 * nk, hipMemcpyDeviceToHost, p->stream));
  if (out_scores) HIP_OK(hipMemcpyAsync(out_scores, p->d_out_sc, 8 * nk, hipMemcpyDeviceToHost, p->stream));
  if (out_len) HIP_OK(hipMemcpyAsync(out_len, p->d_out_len, 4 * (size_t)p->n, hipMemcpyDeviceToHost, p->stream));
  HIP_OK(hipStreamSynchronize(p->stream));
  return PPR_OK;
}

extern "C" int ppr_grank_plan_fetch_slab(ppr_plan* p, int32_t iterations_run, int32_t* ids,
                                         double* scores, int32_t* len) {
  if (!p || iterations_run < 0) return PPR_ERR_ARG;
  HIP_OK(hipSetDevice(p->device));
  const int sA = ((iterations_run + 1) / 2) & 1, sB = (iterations_run / 2) & 1;
  hipStream_t st = p->stream;
  HIP_OK(hipStreamSynchronize(st));  // the plan's stream is non-blocking: drain it first
  std::vector<uint8_t> part(p->n);
  if (p->n) {
    HIP_OK(hipMemcpyAsync(part.data(), p->d_part, p->n, hipMemcpyDeviceToHost, st));
  }
  const size_t L = p->L;
  for (int sl = 0; sl < 2; sl++) {
    // copy the slot wholesale, then keep rows whose partition reads this slot
    std::vector<int32_t> ti(p->n * L), tl(p->n);
    std::vector<double> ts(p->n * L);
    if (p->n) {
      HIP_OK(hipMemcpyAsync(ti.data(), p->d_ids + (size_t)sl * p->n * L, 4 * p->n * L, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(ts.data(), p->d_sc + (size_t)sl * p->n * L, 8 * p->n * L, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(tl.data(), p->d_len + (size_t)sl * p->n, 4 * p->n, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
    }
    for (int64_t v = 0; v < p->n; v++) {
      const int want = part[v] ? sB : sA;
      if (want != sl) continue;
      if (len) len[v] = tl[v];
      for (size_t i = 0; i < L; i++) {
        const bool in = (int)i < tl[v];
        if (ids) ids[v * L + i] = in ? ti[v * L + i] : -1;
        if (scores) scores[v * L + i] = in ? ts[v * L + i] : 0.0;
      }
    }
  }
  return PPR_OK;
}

extern "C" int ppr_grank_plan_row_bytes(ppr_plan* p, int64_t* bytes) {
  if (!p || !bytes) return PPR_ERR_ARG;
  *bytes = (int64_t)p->L * 12 + 8;
  return PPR_OK;
}

extern "C" int ppr_grank_plan_pack(ppr_plan*, int32_t, int64_t, int64_t, void*) { return PPR_ERR_RANGE; }
extern "C" int ppr_grank_plan_unpack(ppr_plan*, int32_t, int64_t, int64_t, const void*) { return PPR_ERR_RANGE; }

extern "C" int ppr_grank_csr(const ppr_csr* g, const uint8_t* part, uint32_t K, uint32_t L,
                             uint32_t iterations, double damping, double tolerance,
                             const ppr_opts* o, int32_t* out_ids, double* out_scores,
                             int32_t* out_len, ppr_stats* st) {
  int rc = check_params(K, L, iterations, damping);
  if (rc) return rc;
  if (!g) return PPR_ERR_ARG;
  if (g->n == 0) { if (st) { std::memset(st, 0, sizeof(*st)); } return PPR_OK; }
  ppr_plan* p = nullptr;
  rc = ppr_grank_plan_create(g, part, K, L, damping, o, &p);
  if (rc) return rc;
  rc = ppr_grank_plan_run(p, iterations, tolerance, st);
  if (!rc) rc = ppr_grank_plan_fetch(p, out_ids, out_scores, out_len);
  ppr_grank_plan_destroy(p);
  return rc;
}

extern "C" const char* ppr_strerror(int code) {
  switch (code) {
    case PPR_OK: return "ok";
    case PPR_ERR_ARG: return "invalid argument";
    case PPR_ERR_K: return "K must be positive";
    case PPR_ERR_L: return "L must be positive";
    case PPR_ERR_KL: return "K must be <= L";
    case PPR_ERR_ITERS: return "iterations must be positive";
    case PPR_ERR_DAMPING: return "damping must be [0,1]";
    case PPR_ERR_THREADS: return "nThreads must be positive";
    case PPR_ERR_GRAPH: return "successor is not a node of the graph";
    case PPR_ERR_HIP: return "HIP runtime error";
    case PPR_ERR_OOM: return "device out of memory";
    case PPR_ERR_RANGE: return "parameter outside the supported range";
    default: return "unknown error";
  }
}
