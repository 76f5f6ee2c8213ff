// merge_xm.h -- the one-range exact-sum merge (round 6): k_xm replaces k_xr for the sources one
// workgroup table holds (XDesc R == 1; merge_xs.h), with the sieve's per-candidate machinery.
//
// k_xr walks a source's successors with hub_window_walk (a flattened stream: a prefix scan, flag
// bytes and ballots per group) and adds each contribution with xt_add: a branchy 96-bit fixed-point
// conversion and a RETURNING 64-bit LDS add whose carry goes to the high word. PPR_DIAG of the
// round-6 build: 1.67 K workgroup cycles per successor row walked, 70 % of it in those adds (a
// walk-only build: 0.49 K). At RMAT-22 these are ~258 K sources of 1.5 K-4 K candidates in every
// other iteration, on that iteration's critical path (33 ms of 42).
//
// k_xm: the same source, the same table budget and the same outputs (the source's list at pt_off,
// its count pc[d], its distinct keys dsum[d], oflag / ovl on overflow: k_xfin1 writes the row and
// the host redoes an overflow exactly as for k_xr), but
//   walk   the sieve's row-wise walk (merge_sv.h sv_rows: each lane holds entries lane and
//          64 + lane of one successor row, the next batch of rows in flight, column ids two windows
//          ahead), successor row minima loaded beside the lengths (the pruning bound tau);
//   table  split accumulators (merge_sv.h X2Table: key, A = sum of the low 32 bits of each X_i,
//          B = sum of X_i >> 32), find-or-insert by x2_slot and two non-returning adds per
//          contribution; the addends come from t = p * 2^(F - 32) by two conversions and a v_fract
//          (sv_split_t) -- the same X = floor(p * 2^F) as xs_conv, so the same exact sum, bit for bit;
//   epilogue as xr_finish (one range: no published bound): settle, keep >= tau (and the verified
//          0.9 x previous L-th bound), compact, radix select, emit.
// A 20-B slot costs 25 % more LDS than k_xr's 16 B: at T = 2048 both run 3 workgroups per CU (k_xr's
// walk flag bytes are gone). Sources with more expected keys keep k_xr's larger classes.
#pragma once
#include "merge_sv.h"

namespace pprk {

// one source of k_xm: its descriptor's fields in the task itself (task -> row pointers -> colx ->
// lengths -> rows: k_xr's task -> descriptor -> ... is one round trip longer). (The row pointers
// come from the device: looking them up on the host for ~258 K sources per iteration cost the
// planning ~25 ms of random reads.)
struct XmTask {
  int64_t pt_off;    // the source's list (XDesc::pt_off)
  double factor, selfval;
  int32_t d, v;      // descriptor index (pc / dsum / oflag / ovl), source
};

// LDS: table (20 T) | misc i32[64] | hist u32[256]
__host__ __device__ constexpr size_t xm_lds_bytes(int T) { return (size_t)T * 20 + 256 + 1024; }

// (W waves; `waves per SIMD` asks the compiler for the registers of 3 workgroups per CU)
template <int W>
__global__ void __launch_bounds__(W * WAVE, 3 * W / 4) k_xm(DevGraph g, DevSlab s, IterArgs a, const XmTask* tasks,
                                                 int T, int budget, int32_t* pk, double* ps, uint32_t* pc,
                                                 uint32_t* dsum, int32_t* oflag, int32_t* ovl) {
  extern __shared__ __align__(16) unsigned char smem[];
  const X2Table xt = x2_carve(smem, T);
  int* misc = reinterpret_cast<int*>(smem + (size_t)T * 20);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + (size_t)T * 20 + 256);
  const XmTask xd = tasks[blockIdx.x];
  const int d = xd.d;
  const int v = xd.v;
  const int L = s.L;
  const int F = a.xsf;
  const double tsc = ldexp(1.0, F - 32);  // t = p * 2^(F - 32): B = floor(t), A = frac(t) 2^32
  long long tph = a.diag ? (long long)clock64() : 0;  // (PPR_DIAG: k_xr's phase slots 183..187)
  {
    uint4* r = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < T * 20 / 16; i += blockDim.x) r[i] = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x < 64) misc[threadIdx.x] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bool ins;
    const int h = x2_slot(xt, v, ins);  // (an empty table: always a slot)
    sv_split_add_t(xt.a, xt.b, h, xd.selfval * tsc);
    misc[XM_FILL] = 1;
  }
  __syncthreads();
  xr_lap(a, 183, tph);
  const int64_t b = g.rp[v], e = g.rp[v + 1];
  const double ft = xd.factor * tsc;
  unsigned long long mb = 0;
  int64_t c0, c1;
  sv_chunk(b, e, c0, c1);
  sv_rows<true, SV_NS1>(g, s, a, c0, c1, [&](const SvBatch<SV_NS1>& bt) {
    sv_groups(bt, [&](int, int key, double sc, bool valid, int64_t) {
      // (every wave checks the shared count before each group: at most budget + W * 64 keys)
      if (__hip_atomic_load(&misc[XM_FILL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > budget) return;
      bool ins = false;
      int h = -1;
      if (valid) h = x2_slot(xt, key, ins);
      const int n = __popcll(__ballot(ins)) + (__ballot(valid && h < 0) ? XR_FULL : 0);
      if (n && lane_id() == 0) atomicAdd(&misc[XM_FILL], n);
      if (h >= 0) sv_split_add_t(xt.a, xt.b, h, sc * ft);
    });
  }, WalkRowMin{&mb, L});
  __syncthreads();
  xr_lap(a, 184, tph);
  const int D = misc[XM_FILL];
  if (a.diag && threadIdx.x == 0) {
    diag_add(a.diag, 182, 1ull);
    diag_add(a.diag, 188, (unsigned long long)(e - b));
    diag_add(a.diag, 189, (unsigned long long)D);
  }
  if (D > budget) {
    if (threadIdx.x == 0 && atomicExch(&oflag[d], 1) == 0) ovl[1 + atomicAdd(&ovl[0], 1)] = d;
    return;
  }
  // pruning bound from the full successor rows (every wave saw its rows' minima)
#pragma unroll
  for (int o = 32; o; o >>= 1) { const unsigned long long y = __shfl_xor(mb, o); mb = y > mb ? y : mb; }
  unsigned long long* wmb = reinterpret_cast<unsigned long long*>(&misc[8]);
  if (lane_id() == 0 && mb) atomicMax(wmb, mb);
  __syncthreads();
  const unsigned long long mbb = *wmb;
  const double tau0 = mbb ? xs_single(bitsd(mbb) * xd.factor, F) : 0.0;
  // speculative bound: 0.9 x the source's previous L-th score (a full current row's minimum), kept
  // only when at least L keys reach it -- the top-L then lies among them (exact either way)
  double ts_hi = tau0;
  if (!a.mc) {
    const int64_t cr = s.lrow((a.active == 1) ? a.sB : a.sA, v);
    if (s.len[cr] == L) ts_hi = fmax(tau0, XR_SPEC * s.rmin[cr]);
  }
  // settle: each thread's slots (T / threads of them, reads issued back to back)
  constexpr int MAXS = 8;  // (T <= 8 * threads: the host's classes)
  const int per = T / (int)blockDim.x;
  int kk[MAXS];
  double kv[MAXS];
  int c = 0, c_hi = 0;
#pragma unroll
  for (int j = 0; j < MAXS; j++) {
    kk[j] = -1;
    kv[j] = 0.0;
    if (j < per) {
      const int i = (int)threadIdx.x + j * (int)blockDim.x;
      const uint32_t kt = xt.keys[i];
      kv[j] = kt ? x2_value(xt.a[i], xt.b[i], F) : 0.0;
      kk[j] = (kt && kv[j] >= tau0) ? (int)kt - 1 : -1;
      c += kk[j] >= 0 ? 1 : 0;
      c_hi += (kk[j] >= 0 && kv[j] >= ts_hi) ? 1 : 0;
    }
  }
  if (ts_hi > tau0) {
    const int w_hi = wave_sum(c_hi);
    if (lane_id() == 0 && w_hi) atomicAdd(&misc[XM_CNT], w_hi);
    __syncthreads();
    if (misc[XM_CNT] >= L) {  // (uniform)
      c = c_hi;
#pragma unroll
      for (int j = 0; j < MAXS; j++)
        if (kk[j] >= 0 && kv[j] < ts_hi) kk[j] = -1;
    }
  }
  const int incl = wave_incl_scan(c);
  int base = 0;
  if (lane_id() == WAVE - 1 && incl) base = atomicAdd(&misc[XM_U], incl);
  base = __builtin_amdgcn_readlane(base, WAVE - 1) + incl - c;
  __syncthreads();  // every slot read: the dense list goes over the front of the table
  double* dv = reinterpret_cast<double*>(smem);
  int* dk = reinterpret_cast<int*>(smem + (size_t)T * 8);
#pragma unroll
  for (int j = 0; j < MAXS; j++)
    if (kk[j] >= 0) { dv[base] = kv[j]; dk[base] = kk[j]; base++; }
  __syncthreads();
  const int U = misc[XM_U];
  if (threadIdx.x == 0 && D) atomicAdd(&dsum[d], (uint32_t)D);
  xr_lap(a, 185, tph);  // settle + compact
  const uint32_t tsalt = tie_salt(v);
  SelCrit sc;
  sc.tie = false; sc.pa = 0; sc.ma = 0; sc.pb = 0; sc.mb = 0;
  const bool cut = U > L;
  if (cut) {
    WgLds w = WgLds{};
    w.hist = hist;
    w.misc = misc;
    sc = wg_select_top(w, U, L, [&](int i) { return dk[i]; }, [&](int i) { return dv[i]; }, [](int) { return true; },
                       tsalt);
  }
  xr_lap(a, 186, tph);  // select
  for (int i0 = 0; i0 < U; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    const bool k = i < U && (!cut || sel_test(sc, dbits(dv[i]), tie_w(dk[i], tsalt)));
    const uint64_t m = __ballot(k);
    uint32_t b0 = 0;
    if (m && lane_id() == 0) b0 = atomicAdd(&pc[d], (uint32_t)__popcll(m));
    b0 = (uint32_t)__shfl((int)b0, 0);
    if (k) {
      const int64_t o = xd.pt_off + b0 + __popcll(m & lanemask_lt());
      pk[o] = dk[i];
      ps[o] = dv[i];
    }
  }
  xr_lap(a, 187, tph);  // emission
}

}  // namespace pprk
