// merge_hot.h -- the hub sources' hot keys: chosen once per run, accumulated densely.
//
// On RMAT the hubs' candidate streams are dominated by a small global core: the ~2048 keys that
// sit in most successor baskets carry 75-85 % of all hub candidates (RMAT-16/18, L = 128), and
// they are also what makes the staged partition slow -- a core key has one contribution per
// successor, i.e. a fma chain as long as the source's out-degree, run by one lane of a bucket
// wave while the other 63 idle. So the hub path splits every source's keys in two:
//   hot   (member of the hot set H)  k_hub_hot: one wave per source walks its successors in
//         order and keeps one accumulator per hot key in LDS, indexed by the key's dense hot
//         index, which the stored id itself carries (HOT_TAG, ppr_common.h); a group of 64
//         candidates from one successor basket has distinct keys, so each lane updates its
//         accumulator directly (groups straddling two baskets take apply_group's ordered
//         chains). No staging, no partition, no table probes. k_hub_join unites the hot and the
//         cold top-L of the source.
//   cold  (everything else)             the staged partition of merge_hub.h, now ~1/5 the volume
//         and without the core keys' long chains.
// Both engines keep every key's contributions in successor order (acc = fma(s, d/deg, acc),
// include/grank.h:107-116), so the split changes no bit of the result, whatever H is.
//
// H is chosen from the state of the run (k_hot_weight / k_hot_hist / k_hot_collect, host picks
// the top `cap` keys by weight, k_hot_set builds the membership bitmap and dense index): key k's
// weight is sum over sampled rows u containing k of indeg(u), i.e. how often k is a candidate
// of some source.
#pragma once
#include "merge_hub.h"

namespace pprk {

struct HotTask {
  int32_t v;  // hub source
  int32_t h;  // its hot list (HubDesc::hot)
};

// k_hub_hot LDS per wave: acc f64[cap] | ck u16[cap] (16-B aligned) | select histogram u32[256] |
// walk flags
__host__ __device__ constexpr size_t hot_wave_lds(int cap) {
  return (((size_t)cap * 10 + 15) & ~(size_t)15) + 1024 + HUB_WALK_FLAGS;
}

constexpr uint64_t HOT_ABSENT = 0x8000000000000000ull;  // -0.0: no contribution yet

// One wave per hub source (tasks in descending candidate count: the longest chains start
// first). Accumulators start at -0.0: fma(s, f, -0.0) == round(s * f) == fma(s, f, +0.0) for
// s, f >= 0 (the reference's operator[] value-init), and a key that received any contribution
// ends >= +0.0, so -0.0 marks the hot keys absent from this source. The self seed {v: 1-d}
// (include/grank.h:100-101) is set first when v is hot. Hot candidates are told apart by their
// HOT_TAG-ed stored id, which also carries the accumulator index: no lookup per candidate.
// Output: the top-L present hot keys >= tau (by (score desc, id asc)) in hot list tk.h, their
// count, and -- when L of them exist -- the L-th largest value as a pruning bound for the
// source's cold buckets (k_hub_prep / hub_tau).
__global__ void __launch_bounds__(64) k_hub_hot(DevGraph g, DevSlab s, IterArgs a, const HotTask* tasks,
                                                int64_t ntasks, int32_t* hot_key, double* hot_sc,
                                                uint32_t* hot_cnt, unsigned long long* tau_hot) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int64_t w = blockIdx.x;
  if (w >= ntasks) return;
  const HotTask tk = tasks[w];
  const int nh = s.hn;
  const int l = lane_id();
  const unsigned long long t_start = a.diag ? wall_clock64() : 0;
  double* acc = reinterpret_cast<double*>(smem);
  uint16_t* ck = reinterpret_cast<uint16_t*>(smem + (size_t)nh * 8);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + (((size_t)nh * 10 + 15) & ~(size_t)15));
  uint8_t* fl = reinterpret_cast<uint8_t*>(hist + 256);
  for (int i = l; i < nh; i += WAVE) acc[i] = bitsd(HOT_ABSENT);
  const int v = tk.v;
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double factor = merge_factor(a, e - b);
  wave_fence();
  if (l == 0) {
    const int32_t sv = s.enc(v);
    if (sv < 0) acc[(uint32_t)sv & 0x7fffffffu] = self_seed(a, e - b);
  }
  wave_fence();
  const int nbits = nh > 1 ? 32 - __clz(nh - 1) : 0;
  unsigned long long mb = 0;  // tau: max row minimum over full successor rows (unscaled bits)
  for (int64_t w0 = b; w0 < e; w0 += WAVE)
    hub_window_walk(g, s, a, w0, min(e, w0 + WAVE), fl, [&](bool valid, int id, double sv, bool one) {
      const bool hot = valid && id < 0;
      if (!__ballot(hot)) return;
      const uint32_t hi = hot ? ((uint32_t)id & 0x7fffffffu) : 0u;
      if (one) {  // one successor basket: distinct keys, distinct accumulators
        if (hot) acc[hi] = fma(sv, factor, acc[hi]);
        wave_fence();
      } else {
        apply_group(acc, hot, hi, sv, factor, nbits);
      }
    }, WalkRowMin{&mb, (int)s.L});
  wave_fence();
#pragma unroll
  for (int o = 32; o; o >>= 1) { const unsigned long long y = __shfl_xor(mb, o); mb = y > mb ? y : mb; }
  const double tau = mb ? bitsd(mb) * factor : 0.0;
  // compact the present hot keys >= tau to the front (hot index -> ck, value -> acc, in place)
  int U = 0;
  for (int i0 = 0; i0 < nh; i0 += WAVE) {
    const int i = i0 + l;
    const double x = i < nh ? acc[i] : 0.0;
    const bool keep = i < nh && dbits(x) != HOT_ABSENT && x >= tau;
    const uint64_t m = __ballot(keep);
    wave_fence();
    if (keep) {
      const int pos = U + __popcll(m & lanemask_lt());
      ck[pos] = (uint16_t)i;
      acc[pos] = x;
    }
    wave_fence();
    U += __popcll(m);
  }
  const int Lw = s.L;
  int32_t* ok = hot_key + (int64_t)tk.h * Lw;
  double* os = hot_sc + (int64_t)tk.h * Lw;
  uint64_t vmin = ~0ull;
  int cnt;
  if (U <= Lw) {
    for (int i = l; i < U; i += WAVE) {
      ok[i] = s.hkeys[ck[i]];
      os[i] = acc[i];
      vmin = dbits(acc[i]) < vmin ? dbits(acc[i]) : vmin;
    }
    cnt = U;
  } else {
    const uint32_t ts = tie_salt(tk.v);
    const SelCrit c = select_top(U, Lw, [&](int i) { return s.hkeys[ck[i]]; }, [&](int i) { return acc[i]; }, hist, ts);
    int pos0 = 0;
    for (int i0 = 0; i0 < U; i0 += WAVE) {
      const int i = i0 + l;
      bool sel = false;
      int k = 0;
      double x = 0.0;
      if (i < U) { k = s.hkeys[ck[i]]; x = acc[i]; sel = sel_test(c, dbits(x), tie_w(k, ts)); }
      const uint64_t m = __ballot(sel);
      if (sel) {
        const int pos = pos0 + __popcll(m & lanemask_lt());
        ok[pos] = k;
        os[pos] = x;
        vmin = dbits(x) < vmin ? dbits(x) : vmin;
      }
      pos0 += __popcll(m);
    }
    cnt = Lw;
  }
  vmin = wave_min_u64(vmin);
  if (l == 0 && a.diag) {  // PPR_DIAG: hot-pass wall time (100 MHz ticks): longest task, sum, task 0
    const unsigned long long dt = wall_clock64() - t_start;
    atomicMax(&a.diag[141], dt);
    atomicAdd(&a.diag[142], dt);
    if (w == 0) atomicAdd(&a.diag[143], dt);
    atomicAdd(&a.diag[144], 1ull);
  }
  if (l == 0) {
    hot_cnt[tk.h] = (uint32_t)cnt;
    // L hot keys with exact final values: the L-th largest final value is at least their minimum
    if (cnt == Lw && vmin != 0ull)
      __hip_atomic_store(&tau_hot[tk.h], (unsigned long long)vmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One workgroup per hub source with a hot pass: its row = top-L of (cold top-L from k_hub_final
// cold-list mode) u (hot top-L from k_hub_hot) -- disjoint key sets, so the top-L of the union
// is the top-L of all its keys -- written with norm1 folded into maxDiff (finish_source).
__global__ void __launch_bounds__(WG_THREADS) k_hub_join(DevSlab s, IterArgs a, const HotTask* tasks,
                                                         const uint32_t* cold_cnt, const int32_t* cold_key,
                                                         const double* cold_sc, const uint32_t* hot_cnt,
                                                         const int32_t* hot_key, const double* hot_sc, int Lp,
                                                         unsigned long long* maxdiff, unsigned long long* stats) {
  extern __shared__ __align__(16) unsigned char smem[];
  const HotTask tk = tasks[blockIdx.x];
  const uint32_t nc = cold_cnt[tk.h];
  if (nc == ~0u) return;  // the HBM-table path redoes this source
  const WgLds L = wg_carve(smem, 0, Lp, 0);
  const int Lw = s.L;
  const int n = (int)nc, nh = (int)hot_cnt[tk.h];
  const int32_t* ck = cold_key + (int64_t)tk.h * Lw;
  const double* cs = cold_sc + (int64_t)tk.h * Lw;
  const int32_t* hk = hot_key + (int64_t)tk.h * Lw;
  const double* hs = hot_sc + (int64_t)tk.h * Lw;
  const int cnt = hub_select_lds(L, n + nh, Lw, [&](int i) { return i < n ? ck[i] : hk[i - n]; },
                                 [&](int i) { return i < n ? cs[i] : hs[i - n]; }, tie_salt(tk.v));
  if ((threadIdx.x >> 6) == 0) {
    const uint64_t* rv = L.rv;
    const int* rk = L.rk;
    finish_source(tk.v, cnt, [&](int i) { return rk[i]; }, [&](int i) { return bitsd(rv[i]); }, s, a, L.hist,
                  L.rv, L.rk, Lp, L.hk, L.hv, L.mf, maxdiff, stats);
  }
}

// every stored row (both slots) re-encoded for a freshly built hot set (rows before it store
// plain keys); one wave per (slot, node)
__global__ void __launch_bounds__(256) k_hot_encode(DevSlab s) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= 2 * s.n) return;
  const int sl = (int)(r / s.n);
  const int64_t u = r - (int64_t)sl * s.n;
  const int len = s.len[s.lrow(sl, u)];
  const int64_t o = s.row(sl, u);
  for (int i = lane_id(); i < len; i += WAVE) {
    const int32_t id = s.ids[o + i];
    if (id >= 0) s.ids[o + i] = s.enc(id);
  }
}

// ---- choosing H ----------------------------------------------------------------------------
// weight of key k: sum over sampled rows u (u % stride == 0) holding k of indeg(u), one wave per
// sampled row; rows are the current baskets of iteration `a` (slot by the node's partition)
__global__ void __launch_bounds__(256) k_hot_weight(DevSlab s, IterArgs a, const uint8_t* part,
                                                    const int32_t* indeg, int stride, uint32_t* W) {
  const int64_t u = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * stride;
  if (u >= s.n) return;
  const uint32_t w = (uint32_t)indeg[u];
  if (!w) return;
  const int sl = part[u] ? a.sB : a.sA;
  const int len = s.len[s.lrow(sl, u)];
  const int64_t r = s.row(sl, u);
  for (int i = lane_id(); i < len; i += WAVE) atomicAdd(&W[s.ids[r + i]], w);
}

// 4096-bin histogram of the weights by the top 12 bits of their float value (sign, exponent and
// 3 mantissa bits: monotone in the weight)
constexpr int HOT_BINS = 4096;
__device__ __forceinline__ uint32_t hot_bin(uint32_t w) { return __float_as_uint((float)w) >> 20; }

__global__ void __launch_bounds__(256) k_hot_hist(const uint32_t* W, int64_t n, uint32_t* hist) {
  __shared__ uint32_t h[HOT_BINS];
  for (int i = threadIdx.x; i < HOT_BINS; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    if (W[k]) atomicAdd(&h[hot_bin(W[k])], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < HOT_BINS; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// keys above the boundary bin -> list[0..) (count in cnt[0]); keys in the boundary bin ->
// (key, weight) pairs from the back of `list` (count in cnt[1], at most `room`)
__global__ void __launch_bounds__(256) k_hot_collect(const uint32_t* W, int64_t n, uint32_t bound,
                                                     int32_t* list, int64_t cap_list, int64_t room,
                                                     uint32_t* cnt) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = W[k];
    if (!w) continue;
    const uint32_t b = hot_bin(w);
    if (b > bound) {
      list[atomicAdd(&cnt[0], 1u)] = (int32_t)k;
    } else if (b == bound) {
      const uint32_t j = atomicAdd(&cnt[1], 1u);
      if (j < (uint32_t)room) { list[cap_list - 2 - 2 * (int64_t)j] = (int32_t)k; list[cap_list - 1 - 2 * (int64_t)j] = (int32_t)w; }
    }
  }
}

// membership bitmap and dense index of the chosen keys (bits cleared beforehand)
__global__ void __launch_bounds__(256) k_hot_set(const int32_t* keys, int nh, uint32_t* bits, uint16_t* idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nh) return;
  const int k = keys[i];
  idx[k] = (uint16_t)i;
  atomicOr(&bits[(uint32_t)k >> 5], 1u << ((uint32_t)k & 31u));
}

}  // namespace pprk
