// merge_wave.h -- per-iteration classification and the single-wave merge tier.
//
//   k_classify     C_v = sum_{u in succ(v)} len[u] (the candidates of source v),
//                  then route v to the smallest tier whose table holds C_v + 1 keys. Tier
//                  counters are bumped once per block (64 sources), not once per source.
//   k_merge_lds    one wave per source, LDS hash table of T = 256 << t slots: candidates are
//                  streamed in successor order by hub_window_walk (64 successors per window,
//                  prefix scan of their basket lengths, successor of each candidate from LDS end
//                  flags), HUB_TW_BATCH groups gathered at once and one batch ahead of the
//                  accumulation, so the next batch's HBM gathers overlap the current LDS work.
//   k_stat_written SURVEY s8d bytes of the rows an iteration wrote (12 * len + 4 per source).
#pragma once
#include <type_traits>

#include "ppr_common.h"

namespace pprk {

constexpr int CLS_PER_WAVE = 16;     // sources per wave of a large list (throughput: an iteration)
constexpr int CLS_PER_BLOCK = CLS_PER_WAVE * WAVES_PER_BLOCK;
constexpr int64_t CLS_SMALL = 65536;  // lists up to this size take one source per wave: a wave's
                                      // sources are summed one after another (three dependent
                                      // loads each), which bounds a small MC level's latency
constexpr int CLS_BIG_DEG = 512;      // sources with more successors are summed by k_classify_big
constexpr int CLS_BIG_THREADS = 1024;

// sum of the current basket lengths of successors [b, e) taken from i0 in steps of `stride`:
// four successor ids loaded before their four lengths, so a long list costs a quarter of the
// dependent round trips (a short MC level waits on exactly these)
__device__ __forceinline__ long long succ_len_sum(const DevGraph& g, const DevSlab& s, const IterArgs& a,
                                                  int64_t i0, int64_t e, int stride) {
  long long c = 0;
  int64_t i = i0;
  for (; i + 3 * (int64_t)stride < e; i += 4 * (int64_t)stride) {
    int32_t cx[4];
#pragma unroll
    for (int k = 0; k < 4; k++) cx[k] = g.colx[i + k * (int64_t)stride];
#pragma unroll
    for (int k = 0; k < 4; k++) c += s.len[s.lrow(read_slot(a, cx[k]), cx[k] & 0x7fffffff)];
  }
  for (; i < e; i += stride) {
    const int32_t cx = g.colx[i];
    c += s.len[s.lrow(read_slot(a, cx), cx & 0x7fffffff)];
  }
  return c;
}

// Tier rule: the candidates + 1 bound a source's distinct keys, so a table of 4/3 of them never
// fills. With `dlast` (exact sum, PPR_WAVE_BY_D) a source is sized by its last merge's distinct keys
// + 1/8 + 64 instead, when that is smaller: a table that still runs out sends the source to the
// overflow redo (k_merge_lds_x's bounded probes).
__device__ __forceinline__ int64_t tier_need(int64_t need, const int32_t* dlast, int v) {
  if (!dlast) return need;
  const int64_t d = dlast[v];
  if (d <= 0) return need;
  const int64_t e = d + d / 8 + 64;
  return e < need ? e : need;
}

__global__ void __launch_bounds__(256) k_classify(DevGraph g, DevSlab s, IterArgs a,
                                                  const int32_t* list, int64_t count,
                                                  const int32_t* tier_cap, int32_t* tier_lists,
                                                  uint32_t* tier_cnt, int64_t list_cap,
                                                  int32_t* cand, unsigned long long* stats,
                                                  int32_t* big_list, int per_wave, const int32_t* dlast) {
  // per_wave sources per wave (CLS_PER_WAVE, or 1 for a short list), per_block per block
  const int per_block = per_wave * WAVES_PER_BLOCK;
  __shared__ int s_tier[CLS_PER_BLOCK];
  __shared__ int s_src[CLS_PER_BLOCK];
  __shared__ uint32_t s_base[NLISTS];
  __shared__ unsigned long long s_red[3][WAVES_PER_BLOCK];
  const int wv = threadIdx.x >> 6;
  unsigned long long my_c = 0, my_b = 0, my_w = 0;
  for (int k = 0; k < per_wave; k++) {
    const int slot = wv * per_wave + k;
    const int64_t idx = (int64_t)blockIdx.x * per_block + slot;
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
      c = succ_len_sum(g, s, a, b + lane_id(), e, WAVE);
#pragma unroll
      for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o);
    }
    if (lane_id() == 0) {
      const int64_t need = c + 1;
      cand[v] = (int32_t)(need > 0x7fffffff ? 0x7fffffff : need);
      int t = 0;
      const int64_t tneed = tier_need(need, dlast, v);
      while (t < NT + 1 && tneed > tier_cap[t]) t++;
      s_tier[slot] = t;
      s_src[slot] = v;
      const int ownlen = (a.unit || a.mc) ? 0 : s.len[s.lrow(a.active == 0 ? a.sA : a.sB, v)];
      my_c += (unsigned long long)c;
      my_b += (unsigned long long)(8 + 8 * (e - b) + 12 * c + 12 * ownlen);
      if (t < NT) my_w += (unsigned long long)(8 + 8 * (e - b) + 12 * c + 12 * ownlen);  // (wave-tier share)
    }
  }
  __syncthreads();
  if (threadIdx.x < NLISTS) {
    uint32_t n = 0;
    for (int i = 0; i < per_block; i++) n += s_tier[i] == (int)threadIdx.x;
    s_base[threadIdx.x] = n ? atomicAdd(&tier_cnt[threadIdx.x], n) : 0u;
  }
  if (a.stats && lane_id() == 0) { s_red[0][wv] = my_c; s_red[1][wv] = my_b; s_red[2][wv] = my_w; }
  __syncthreads();
  if ((int)threadIdx.x < per_block) {
    const int t = s_tier[threadIdx.x];
    if (t >= 0) {
      uint32_t r = 0;
      for (int i = 0; i < (int)threadIdx.x; i++) r += s_tier[i] == t;
      tier_lists[(int64_t)t * list_cap + s_base[t] + r] = s_src[threadIdx.x];
    }
  }
  if (a.stats && threadIdx.x == 0) {
    unsigned long long sc = 0, sb = 0, sw = 0;
    for (int i = 0; i < WAVES_PER_BLOCK; i++) { sc += s_red[0][i]; sb += s_red[1][i]; sw += s_red[2][i]; }
    if (sc) atomicAdd(&stats[0], sc);
    if (sb) atomicAdd(&stats[1], sb);
    if (sw) atomicAdd(&stats[2], sw);
  }
}

// k_classify's long-list sources: one block per source (grid-stride over the list), the
// successor sum split over the block; same tier rule and statistics as k_classify
__global__ void __launch_bounds__(CLS_BIG_THREADS) k_classify_big(DevGraph g, DevSlab s, IterArgs a,
                                                                  const int32_t* tier_cap, int32_t* tier_lists,
                                                                  uint32_t* tier_cnt, int64_t list_cap,
                                                                  int32_t* cand, unsigned long long* stats,
                                                                  const int32_t* big_list, const int32_t* dlast) {
  __shared__ long long red[CLS_BIG_THREADS / WAVE];
  const uint32_t nbig = __hip_atomic_load(&tier_cnt[NLISTS + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t i = blockIdx.x; i < nbig; i += gridDim.x) {
    const int v = big_list[i];
    const int64_t b = g.rp[v], e = g.rp[v + 1];
    long long c = succ_len_sum(g, s, a, b + threadIdx.x, e, CLS_BIG_THREADS);
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
      const int64_t tneed = tier_need(need, dlast, v);
      while (t < NT + 1 && tneed > tier_cap[t]) t++;
      tier_lists[(int64_t)t * list_cap + atomicAdd(&tier_cnt[t], 1u)] = v;
      if (a.stats) {
        const int ownlen = a.mc ? 0 : s.len[s.lrow(a.active == 0 ? a.sA : a.sB, v)];
        atomicAdd(&stats[0], (unsigned long long)c);
        atomicAdd(&stats[1], (unsigned long long)(8 + 8 * (e - b) + 12 * c + 12 * ownlen));
        if (t < NT) atomicAdd(&stats[2], (unsigned long long)(8 + 8 * (e - b) + 12 * c + 12 * ownlen));
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

// per-wave LDS bytes for table size T and padded width Lp (layout: k_merge_lds below)
__host__ __device__ constexpr size_t lds_wave_bytes(int T, int Lp) {
  return (size_t)T * 13 + (size_t)Lp * 12 + 1024 + (size_t)Lp * 20;
}

#ifndef PPR_TW_BATCH
#define PPR_TW_BATCH 8
#endif
constexpr int HUB_TW_BATCH = PPR_TW_BATCH;  // candidate groups a walking wave gathers before using them

// walk the candidates of successors [i0, e) (at most one per lane) in successor order, 64 per step:
// f(valid, id, score, one_row) per group: id = the stored id (HOT_TAG-ed for hot keys, DevSlab::key
// decodes it; in init mode the successor itself), one_row = every candidate of the group comes
// from the same successor basket (so its keys are distinct; always false in init mode).
// `succ(ln, rmin_bits)` (optional) sees every lane's successor basket length and row minimum once
// per window (non-unit mode; invalid lanes report length 0).
// hub_window_walk_part: the same walk restricted to every nparts-th batch of groups starting at
// batch `part` (the waves of a workgroup sharing one short successor window, merge_xs.h k_xr);
// f still sees this wave's candidates in stream order
template <class F, class S>
__device__ __forceinline__ void hub_window_walk_part(const DevGraph& g, const DevSlab& s, const IterArgs& a,
                                                     int64_t i0, int64_t e, uint8_t* fl, F f, S succ, int part,
                                                     int nparts) {
  const int64_t i = i0 + lane_id();
  if (a.unit) {  // init: every successor contributes {u: 1.0}
    const bool valid = i < e;
    if constexpr (std::is_invocable_v<F, bool, int, double, bool, int, int>)
      f(valid, valid ? (g.colx[i] & 0x7fffffff) : 0, 1.0, false, lane_id(), WAVE);  // (one successor a lane)
    else
      f(valid, valid ? (g.colx[i] & 0x7fffffff) : 0, 1.0, false);
    return;
  }
  int u = 0, sl = 0, ln = 0;
  unsigned long long rm = 0;
  if (i < e) {
    const int32_t cx = g.colx[i];
    u = cx & 0x7fffffff;
    sl = read_slot(a, cx);
    ln = s.len[s.lrow(sl, u)];
    if (S::kWant) rm = dbits(s.rmin[s.lrow(sl, u)]);  // loaded beside len
  }
  succ(ln, rm);
  const int incl = wave_incl_scan(ln);
  const int total = __builtin_amdgcn_readlane(incl, WAVE - 1);
  // successor of candidate c: j = #{successors whose basket ends at or before c}. With every
  // basket non-empty the ends are distinct, so a batch marks them as byte flags in LDS and a
  // group reads j off one ballot of its 64 flags (instead of a 6-step cross-lane binary search)
  const bool flags = fl != nullptr && !__ballot(i < e && ln == 0);
  // HUB_TW_BATCH groups of 64 candidates are gathered together (one memory latency per batch),
  // and the next batch is in flight while f consumes the current one; f still sees the
  // candidates in stream order
  // (f may also take the lane's row within the group and the group's row count: rr, nr)
  constexpr bool kRows = std::is_invocable_v<F, bool, int, double, bool, int, int>;
  // (rr: 8 bits per group, 4 groups per word; nr: wave-uniform)
  constexpr int RW = (HUB_TW_BATCH + 3) / 4;
  auto load = [&](int g0, int (&key)[HUB_TW_BATCH], double (&sv)[HUB_TW_BATCH], bool (&one)[HUB_TW_BATCH],
                  uint32_t (&rr)[RW], int (&nr)[HUB_TW_BATCH]) {
    if (kRows)
#pragma unroll
      for (int q = 0; q < RW; q++) rr[q] = 0u;
    if (flags) {
#pragma unroll
      for (int q = 0; q < HUB_TW_BATCH / 4; q++)  // WAVE * HUB_TW_BATCH flag bytes
        reinterpret_cast<uint32_t*>(fl)[q * WAVE + lane_id()] = 0u;
      wave_fence();
      if (incl > g0 && incl < g0 + WAVE * HUB_TW_BATCH) fl[incl - g0] = 1;
      wave_fence();
    }
#pragma unroll
    for (int k = 0; k < HUB_TW_BATCH; k++) {
      const int c = g0 + k * WAVE + lane_id();
      const bool valid = c < total;
      int j = 0;
      if (flags) {
        const int G = g0 + k * WAVE;
        const uint64_t ends = __ballot(fl[k * WAVE + lane_id()] != 0) & ~1ull;  // ends in (G, G + 64)
        j = __popcll(__ballot(incl <= G)) + __popcll(ends & (lanemask_lt() | (1ull << lane_id())));
      } else {
#pragma unroll
        for (int step = 32; step; step >>= 1) {
          const int pv = __shfl(incl, j + step - 1);
          if (pv <= c) j += step;
        }
      }
      const int jj = j < WAVE ? j : WAVE - 1;
      // every candidate of the group from one successor basket: its keys are distinct
      one[k] = !__ballot(valid && jj != __builtin_amdgcn_readlane(jj, 0));
      if (kRows) {
        const uint64_t vm = __ballot(valid);
        const int j0 = __builtin_amdgcn_readlane(jj, 0);
        rr[k / 4] |= (uint32_t)min(jj - j0, 255) << (8 * (k % 4));
        nr[k] = __builtin_amdgcn_readfirstlane(vm ? __shfl(jj, 63 - __clzll((long long)vm)) - j0 + 1 : 1);
      }
      const int exv = __shfl(incl, jj > 0 ? jj - 1 : 0);
      const int ex = jj > 0 ? exv : 0;
      const int uj = __shfl(u, jj);
      const int sj = __shfl(sl, jj);
      key[k] = 0;
      sv[k] = 0.0;
      if (valid) {
        const int64_t r = s.row(sj, uj) + (c - ex);
        key[k] = ld_nt(&s.ids[r], a.nt & 1u);
        sv[k] = (a.whatif & WI_SCAT_NOSCORE) ? 0.5 : ld_nt(&s.sc[r], a.nt & 1u);  // (timing only)
      }
    }
  };
  int key[HUB_TW_BATCH], nkey[HUB_TW_BATCH];
  double sv[HUB_TW_BATCH], nsv[HUB_TW_BATCH];
  bool one[HUB_TW_BATCH], none[HUB_TW_BATCH];
  uint32_t rr[RW], nrr[RW];
  int nr[HUB_TW_BATCH], nnr[HUB_TW_BATCH];
  const int step = WAVE * HUB_TW_BATCH * nparts;
  const int gs = WAVE * HUB_TW_BATCH * part;
  if (gs < total) load(gs, nkey, nsv, none, nrr, nnr);
  for (int g0 = gs; g0 < total; g0 += step) {
#pragma unroll
    for (int k = 0; k < HUB_TW_BATCH; k++) {
      key[k] = nkey[k]; sv[k] = nsv[k]; one[k] = none[k];
      if (kRows) nr[k] = nnr[k];
    }
    if (kRows)
#pragma unroll
      for (int q = 0; q < RW; q++) rr[q] = nrr[q];
    if (g0 + step < total) load(g0 + step, nkey, nsv, none, nrr, nnr);
#pragma unroll
    for (int k = 0; k < HUB_TW_BATCH; k++) {
      if (g0 + k * WAVE >= total) break;  // uniform
      if constexpr (kRows)
        f(g0 + k * WAVE + lane_id() < total, key[k], sv[k], one[k], (int)((rr[k / 4] >> (8 * (k % 4))) & 255u), nr[k]);
      else
        f(g0 + k * WAVE + lane_id() < total, key[k], sv[k], one[k]);
    }
  }
}

template <class F, class S>
__device__ __forceinline__ void hub_window_walk(const DevGraph& g, const DevSlab& s, const IterArgs& a,
                                                int64_t i0, int64_t e, uint8_t* fl, F f, S succ) {
  hub_window_walk_part(g, s, a, i0, e, fl, f, succ, 0, 1);
}

struct WalkNoSucc {
  static constexpr bool kWant = false;
  __device__ void operator()(int, unsigned long long) const {}
};
// top-L pruning bound of the wave tier: max row minimum over full successor rows (unscaled bits)
struct WalkRowMin {
  static constexpr bool kWant = true;
  unsigned long long* mb;
  int L;
  __device__ void operator()(int ln, unsigned long long rm) const { if (ln == L && rm > *mb) *mb = rm; }
};
template <class F>
__device__ __forceinline__ void hub_window_walk(const DevGraph& g, const DevSlab& s, const IterArgs& a,
                                                int64_t i0, int64_t e, uint8_t* fl, F f) {
  hub_window_walk(g, s, a, i0, e, fl, f, WalkNoSucc{});
}
// flag bytes per wave of hub_window_walk
constexpr int HUB_WALK_FLAGS = WAVE * HUB_TW_BATCH;

// Split epilogue of the wave tiers (round 6): the wave stops after its compaction
// and writes its kept entries to a list in HBM; k_wfin (merge_xs.h) selects, writes the row and its
// norm1 with a 5-KB wave, so the table's LDS is held for the walk only.
struct WList {
  int32_t* k;  // [count * cap] keys
  double* v;   // [count * cap] values
  int32_t* n;  // [count] entries (-1: the table ran out, the host redoes the source)
  int cap;     // 0: no split; else >= L
};
// source w's list: every one of its U kept entries, or the top-L of more than cap (cap >= L)
template <class K, class V>
__device__ __forceinline__ void wave_emit_list(const WList& wl, int64_t w, int U, const K* keys, const V* vals, int v,
                                               int L, uint32_t* hist) {
  U = __builtin_amdgcn_readfirstlane(U);
  const int64_t o = w * (int64_t)wl.cap;
  if (U <= wl.cap) {
    for (int i = lane_id(); i < U; i += WAVE) { wl.k[o + i] = (int32_t)keys[i]; wl.v[o + i] = (double)vals[i]; }
    if (lane_id() == 0) wl.n[w] = U;
    return;
  }
  const uint32_t ts = tie_salt(v);
  const SelCrit c = select_top(U, L, [&](int i) { return (int)keys[i]; }, [&](int i) { return (double)vals[i]; }, hist, ts);
  int nb = 0;
  for (int i0 = 0; i0 < U; i0 += WAVE) {
    const int i = i0 + lane_id();
    const bool sel = i < U && sel_test(c, dbits((double)vals[i]), tie_w((int)keys[i], ts));
    const uint64_t m = __ballot(sel);
    if (sel) {
      const int64_t q = o + nb + __popcll(m & lanemask_lt());
      wl.k[q] = (int32_t)keys[i];
      wl.v[q] = (double)vals[i];
    }
    nb += __popcll(m);
  }
  if (lane_id() == 0) wl.n[w] = nb;
}

// chain-order wave tier. LDS: acc f64[T] | keys i32[T] | own u8[T] | hist u32[256] | rv u64[Lp] |
// rk i32[Lp] | hk i32[2Lp] | hv i32[2Lp] | mf i32[Lp]; split (kSplit): up to hist
__host__ __device__ constexpr size_t lds_wave_bytes_s(int T) { return (size_t)T * 13 + 1024; }
template <bool HK, bool kSplit = false>
__global__ void __launch_bounds__(256) k_merge_lds(DevGraph g, DevSlab s, IterArgs a,
                                                   const int32_t* list, int64_t count, int T,
                                                   int Lp, unsigned long long* maxdiff,
                                                   unsigned long long* stats, WList wl = WList{}) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w >= count) return;
  unsigned char* base = smem + (size_t)wv * (kSplit ? lds_wave_bytes_s(T) : lds_wave_bytes(T, Lp));
  LdsTable t;
  t.acc = reinterpret_cast<double*>(base);
  t.keys = reinterpret_cast<int*>(base + (size_t)T * 8);
  t.mask = (uint32_t)T - 1;
  t.nbits = 31 - __clz(T);
  uint8_t* own = base + (size_t)T * 12;
  uint32_t* hist = reinterpret_cast<uint32_t*>(base + (size_t)T * 13);  // (T: a multiple of 64)
  uint64_t* rv = reinterpret_cast<uint64_t*>(base + (size_t)T * 13 + 1024);
  int* rk = reinterpret_cast<int*>(base + (size_t)T * 13 + 1024 + (size_t)Lp * 8);
  int* hk = reinterpret_cast<int*>(base + (size_t)T * 13 + 1024 + (size_t)Lp * 12);
  int* hv = hk + 2 * Lp;
  int* mf = hv + 2 * Lp;

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
    // the select histogram's LDS is idle until the epilogue: it holds the walk's end flags
    for (int64_t e0 = b; e0 < e; e0 += WAVE)
      hub_window_walk(g, s, a, e0, min(e, e0 + WAVE), reinterpret_cast<uint8_t*>(hist),
                      [&](bool valid, int id, double sv, bool) { table_apply_own(t, own, valid, s.keyd<HK>(id), sv, factor); },
                      WalkRowMin{&mb, (int)s.L});
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
  if (kSplit)
    wave_emit_list(wl, w, U, keys, acc, v, (int)s.L, hist);
  else
    finish_source(v, U, [&](int i) { return keys[i]; }, [&](int i) { return acc[i]; }, s, a, hist,
                  rv, rk, Lp, hk, hv, mf, maxdiff, stats);
}

}  // namespace pprk
