// merge_wave.h -- per-iteration classification and the single-wave merge tier.
//
//   k_classify     C_v = sum_{u in succ(v)} len[u] (the candidates of source v),
//                  then route v to the smallest tier whose table holds C_v + 1 keys. Tier
//                  counters are bumped once per block (64 sources), not once per source.
//   k_merge_lds    one wave per source, LDS hash table of T = 256 << t slots: candidates are
//                  streamed in successor order (64 successors per window, prefix scan of their
//                  basket lengths, binary search per lane), one group ahead of the accumulation
//                  so the next group's HBM gathers overlap the current group's LDS work.
//   k_stat_written SURVEY s8d bytes of the rows an iteration wrote (12 * len + 4 per source).
#pragma once
#include "ppr_common.h"

namespace pprk {

constexpr int CLS_PER_WAVE = 16;
constexpr int CLS_PER_BLOCK = CLS_PER_WAVE * WAVES_PER_BLOCK;
constexpr int CLS_BIG_DEG = 512;      // sources with more successors are summed by k_classify_big
constexpr int CLS_BIG_THREADS = 1024;

__global__ void __launch_bounds__(256) k_classify(DevGraph g, DevSlab s, IterArgs a,
                                                  const int32_t* list, int64_t count,
                                                  const int32_t* tier_cap, int32_t* tier_lists,
                                                  uint32_t* tier_cnt, int64_t list_cap,
                                                  int32_t* cand, unsigned long long* stats,
                                                  int32_t* big_list) {
  __shared__ int s_tier[CLS_PER_BLOCK];
  __shared__ int s_src[CLS_PER_BLOCK];
  __shared__ uint32_t s_base[NLISTS];
  __shared__ unsigned long long s_red[2][WAVES_PER_BLOCK];
  const int wv = threadIdx.x >> 6;
  unsigned long long my_c = 0, my_b = 0;
  for (int k = 0; k < CLS_PER_WAVE; k++) {
    const int slot = wv * CLS_PER_WAVE + k;
    const int64_t idx = (int64_t)blockIdx.x * CLS_PER_BLOCK + slot;
    if (idx >= count) { if (lane_id() == 0) s_tier[slot] = -1; continue; }
    const int v = list[idx];
    const int64_t b = g.rp[v], e = g.rp[v + 1];
    if (!a.unit && e - b > CLS_BIG_DEG) {
      // a long successor list would serialise this wave's 16 sources: hand it to k_classify_big
      if (lane_id() == 0) {
        s_tier[slot] = -1;
        big_list[atomicAdd(&tier_cnt[NLISTS + 1], 1u)] = v;
      }
      continue;
    }
    long long c = 0;
    if (a.unit) {
      c = e - b;
    } else {
      for (int64_t i = b + lane_id(); i < e; i += WAVE) {
        const int32_t cx = g.colx[i];
        c += s.len[s.lrow(read_slot(a, cx), cx & 0x7fffffff)];
      }
#pragma unroll
      for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o);
    }
    if (lane_id() == 0) {
      const int64_t need = c + 1;
      cand[v] = (int32_t)(need > 0x7fffffff ? 0x7fffffff : need);
      int t = 0;
      while (t < NT + 1 && need > tier_cap[t]) t++;
      s_tier[slot] = t;
      s_src[slot] = v;
      const int ownlen = (a.unit || a.mc) ? 0 : s.len[s.lrow(a.active == 0 ? a.sA : a.sB, v)];
      my_c += (unsigned long long)c;
      my_b += (unsigned long long)(8 + 8 * (e - b) + 12 * c + 12 * ownlen);
    }
  }
  __syncthreads();
  if (threadIdx.x < NLISTS) {
    uint32_t n = 0;
    for (int i = 0; i < CLS_PER_BLOCK; i++) n += s_tier[i] == (int)threadIdx.x;
    s_base[threadIdx.x] = n ? atomicAdd(&tier_cnt[threadIdx.x], n) : 0u;
  }
  if (a.stats && lane_id() == 0) { s_red[0][wv] = my_c; s_red[1][wv] = my_b; }
  __syncthreads();
  if (threadIdx.x < CLS_PER_BLOCK) {
    const int t = s_tier[threadIdx.x];
    if (t >= 0) {
      uint32_t r = 0;
      for (int i = 0; i < (int)threadIdx.x; i++) r += s_tier[i] == t;
      tier_lists[(int64_t)t * list_cap + s_base[t] + r] = s_src[threadIdx.x];
    }
  }
  if (a.stats && threadIdx.x == 0) {
    unsigned long long sc = 0, sb = 0;
    for (int i = 0; i < WAVES_PER_BLOCK; i++) { sc += s_red[0][i]; sb += s_red[1][i]; }
    if (sc) atomicAdd(&stats[0], sc);
    if (sb) atomicAdd(&stats[1], sb);
  }
}

// k_classify's long-list sources: one block per source (grid-stride over the list), the
// successor sum split over the block; same tier rule and statistics as k_classify
__global__ void __launch_bounds__(CLS_BIG_THREADS) k_classify_big(DevGraph g, DevSlab s, IterArgs a,
                                                                  const int32_t* tier_cap, int32_t* tier_lists,
                                                                  uint32_t* tier_cnt, int64_t list_cap,
                                                                  int32_t* cand, unsigned long long* stats,
                                                                  const int32_t* big_list) {
  __shared__ long long red[CLS_BIG_THREADS / WAVE];
  const uint32_t nbig = __hip_atomic_load(&tier_cnt[NLISTS + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) {
    const int v = big_list[i];
    const int64_t b = g.rp[v], e = g.rp[v + 1];
    long long c = 0;
    for (int64_t k = b + threadIdx.x; k < e; k += CLS_BIG_THREADS) {
      const int32_t cx = g.colx[k];
      c += s.len[s.lrow(read_slot(a, cx), cx & 0x7fffffff)];
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o);
    if (lane_id() == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      c = 0;
      for (int k = 0; k < CLS_BIG_THREADS / WAVE; k++) c += red[k];
      const int64_t need = c + 1;
      cand[v] = (int32_t)(need > 0x7fffffff ? 0x7fffffff : need);
      int t = 0;
      while (t < NT + 1 && need > tier_cap[t]) t++;
      tier_lists[(int64_t)t * list_cap + atomicAdd(&tier_cnt[t], 1u)] = v;
      if (a.stats) {
        const int ownlen = a.mc ? 0 : s.len[s.lrow(a.active == 0 ? a.sA : a.sB, v)];
        atomicAdd(&stats[0], (unsigned long long)c);
        atomicAdd(&stats[1], (unsigned long long)(8 + 8 * (e - b) + 12 * c + 12 * ownlen));
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_stat_written(DevSlab s, IterArgs a, const int32_t* list,
                                                      int64_t count, unsigned long long* stats) {
  __shared__ unsigned long long red[WAVES_PER_BLOCK];
  const int nxt = write_slot(a);
  unsigned long long b = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x)
    b += 12ull * (unsigned long long)s.len[s.lrow(nxt, list[i])] + 4ull;
#pragma unroll
  for (int o = 32; o; o >>= 1) b += __shfl_xor(b, o);
  if (lane_id() == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int i = 0; i < WAVES_PER_BLOCK; i++) t += red[i];
    atomicAdd(&stats[1], t);
  }
}

// per-wave LDS bytes for table size T and padded width Lp
// layout: acc f64[T] | keys i32[T] | rv u64[Lp] | rk i32[Lp] | hist u32[256] | hk i32[2Lp] |
//         hv i32[2Lp] | mf i32[Lp] | own u8[T]
__host__ __device__ constexpr size_t lds_wave_bytes(int T, int Lp) {
  return (size_t)T * 13 + (size_t)Lp * 12 + 1024 + (size_t)Lp * 20;
}

// the candidate of stream position c inside the current successor window (all lanes execute:
// the binary search and the operand fetches are cross-lane bpermutes)
// With `fl` (64 bytes of LDS; every basket of the window non-empty, so basket ends are distinct)
// the successor index comes from end flags and two ballots instead of the binary search.
__device__ __forceinline__ void window_fetch(const DevSlab& s, int incl, int u, int sl, int total,
                                             int c, bool& valid, int& key, double& sv, uint8_t* fl) {
  valid = c < total;
  int j = 0;
  if (fl) {
    const int G = c - lane_id();  // the group's first stream position
    reinterpret_cast<uint32_t*>(fl)[lane_id() & 15] = 0u;
    wave_fence();
    if (incl > G && incl < G + WAVE) fl[incl - G] = 1;
    wave_fence();
    const uint64_t ends = __ballot(fl[lane_id()] != 0) & ~1ull;
    wave_fence();
    j = __popcll(__ballot(incl <= G)) + __popcll(ends & (lanemask_lt() | (1ull << lane_id())));
  } else {
#pragma unroll
    for (int step = 32; step; step >>= 1) {
      const int pv = __shfl(incl, j + step - 1);
      if (pv <= c) j += step;
    }
  }
  const int jj = j < WAVE ? j : WAVE - 1;
  const int exv = __shfl(incl, jj > 0 ? jj - 1 : 0);  // every lane executes the bpermute
  const int ex = jj > 0 ? exv : 0;
  const int uj = __shfl(u, jj);
  const int sj = __shfl(sl, jj);
  key = 0;
  sv = 0.0;
  if (valid) {
    const int64_t r = s.row(sj, uj) + (c - ex);
    key = s.ids[r];
    sv = s.sc[r];
  }
}

__global__ void __launch_bounds__(256) k_merge_lds(DevGraph g, DevSlab s, IterArgs a,
                                                   const int32_t* list, int64_t count, int T,
                                                   int Lp, unsigned long long* maxdiff,
                                                   unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w >= count) return;
  unsigned char* base = smem + (size_t)wv * lds_wave_bytes(T, Lp);
  LdsTable t;
  t.acc = reinterpret_cast<double*>(base);
  t.keys = reinterpret_cast<int*>(base + (size_t)T * 8);
  t.mask = (uint32_t)T - 1;
  t.nbits = 31 - __clz(T);
  uint64_t* rv = reinterpret_cast<uint64_t*>(base + (size_t)T * 12);
  int* rk = reinterpret_cast<int*>(base + (size_t)T * 12 + (size_t)Lp * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + (size_t)T * 12 + (size_t)Lp * 12);
  int* hk = reinterpret_cast<int*>(base + (size_t)T * 12 + (size_t)Lp * 12 + 1024);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;
  uint8_t* own = reinterpret_cast<uint8_t*>(mf + Lp);

  const int v = list[w];
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = merge_factor(a, e - b);

  table_clear(t);
  unsigned long long mb = 0;  // top-L pruning bound: max row minimum over full successor rows
  if (lane_id() == 0) { const uint32_t sl = table_slot(t, v); t.acc[sl] = self_seed(a, e - b); }
  wave_fence();

  if (a.unit) {
    for (int64_t e0 = b; e0 < e; e0 += WAVE) {
      const int64_t i = e0 + lane_id();
      const bool valid = i < e;
      const int key = valid ? (g.colx[i] & 0x7fffffff) : 0;
      table_apply_own(t, own, valid, key, 1.0, factor);
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
        const unsigned long long rm = dbits(s.rmin[s.lrow(sl, u)]);  // loaded beside len
        if (ln == s.L && rm > mb) mb = rm;
      }
      const int incl = wave_incl_scan(ln);
      const int total = __shfl(incl, WAVE - 1);
      // end flags live in the select histogram's LDS, unused until the epilogue
      uint8_t* fl = __ballot(i < e && ln == 0) ? nullptr : reinterpret_cast<uint8_t*>(hist);
      bool nv;
      int nk;
      double ns;
      window_fetch(s, incl, u, sl, total, lane_id(), nv, nk, ns, fl);
      for (int g0 = 0; g0 < total; g0 += WAVE) {
        const bool cv = nv;
        const int ck = nk;
        const double cs = ns;
        if (g0 + WAVE < total) window_fetch(s, incl, u, sl, total, g0 + WAVE + lane_id(), nv, nk, ns, fl);
        table_apply_own(t, own, cv, ck, cs, factor);
      }
    }
  }
  wave_fence();
  // keys below the bound cannot reach the top-L (a full successor row puts L distinct keys at
  // >= round(rmin * factor), the hub pipeline's tau): dropped before the select
#pragma unroll
  for (int o = 32; o; o >>= 1) { const unsigned long long y = __shfl_xor(mb, o); mb = y > mb ? y : mb; }
  const double tau = (!a.unit && mb) ? bitsd(mb) * factor : 0.0;
  const int U = table_compact_min(t, tau);
  const int* keys = t.keys;
  const double* acc = t.acc;
  finish_source(v, U, [&](int i) { return keys[i]; }, [&](int i) { return acc[i]; }, s, a, hist,
                rv, rk, Lp, hk, hv, mf, maxdiff, stats);
}

}  // namespace pprk
