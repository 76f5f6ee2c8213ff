// plan.h -- the device-resident state of one engine instance (ppr_plan, include/ppr_hip.h) and
// the host-side helpers shared by the GRank (grank.hip) and MCCompletePathV2 (mccp2.hip) drivers.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/ppr_hip.h"
#include "ppr_common.h"

using namespace pprk;

#define HIP_OK(expr)                                  \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) {                           \
      fprintf(stderr, "ppr_hip: %s failed: %s (%s:%d)\n", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
      return PPR_ERR_HIP;                             \
    }                                                 \
  } while (0)

constexpr int WG_TIER_PASSES = 3;

inline int pow2_at_least(int64_t x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}


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
  uint16_t* d_rix = nullptr;      // [2][n][NRANGE] row range index
  double* d_rmin = nullptr;       // [2][n] row minimum
  int32_t* d_all = nullptr;       // init list: the n_nd nodes with successors, then the dangling ones
  int64_t n_nd = 0;
  int32_t* d_act[2] = {nullptr, nullptr};
  int64_t nact[2] = {0, 0};
  int32_t* d_cand = nullptr;
  int32_t* d_tier_lists = nullptr;   // NLISTS * n
  uint32_t* d_tier_cnt = nullptr;    // NLISTS, +1 workgroup overflow count, +1 k_classify_big list length
  int32_t* d_big = nullptr;          // sources k_classify hands to k_classify_big
  int64_t max_deg = 0;
  int32_t* d_tier_cap = nullptr;     // NT + 1
  int32_t* d_ovf = nullptr;          // sources the workgroup tier could not hold
  int tierT[NT] = {0, 0, 0, 0};
  int tierCap[NT + 1] = {0, 0, 0, 0, 0};
  size_t wg_lds = 0;
  // PPR_WHATIF (timing experiments only; tools/whatif.py): 1 no spill grid, 2 no reduce (k_hub_final
  // selects from the whole list), 4 count twice, 8 scatter twice, 16 an extra dry bucket-wave pass
  // (no emission), 32 final twice, 64 reduce twice, 128 bucket waves stop after 2048 records,
  // 256 (with 8) the first of the two scatters stores lane-contiguously (its scattered stores' cost),
  // 4096 (with 8) ... stores nothing, 8192 (with 8) ... loads no scores, 16384 (with 8) ... only
  // counts (non-returning rank atomics), 32768 (with 8) ... only walks
  int whatif = 0;
  int nt_loads = 0;         // PPR_NT (IterArgs::nt): non-temporal candidate gathers (1) / staged-record reads (2)
  double spec_ratio = 0.0;  // PPR_SPEC: speculative hub pruning bound (ppr_common.h spec_tau), 0 = off
  int spec_from = 6;        // PPR_SPEC_FROM: first iteration that speculates (rows settle after a few)
  int64_t spec_redo = 0;    // hub sources redone after a failed speculation (PPR_TIMING at destroy)
  int wg_max_passes = 64;  // (WG_MAX_PASSES) PPR_WG_PASSES (tests): workgroup-tier key-bucket passes before overflow
  bool hub_enabled = true;
  unsigned long long* d_maxdiff = nullptr;  // PPR_MAX_ITER_STATS + 1
  // iterations >= PPR_MAX_ITER_STATS share the last maxDiff slot: it is zeroed at the first
  // ppr_grank_plan_iterate call of each such iteration (a sharded iteration may call it per range)
  int32_t md_shared_it = -1;
  unsigned long long* d_stats = nullptr;    // PPR_NSTATS: candidates, algorithmic bytes, wave-tier bytes
  // per-kernel roofline (ppr_grank_plan_kernel_stats): HIP events around each kernel group on the
  // stream it runs on, algorithmic bytes of the sources it merged (SURVEY s8d per source)
  static constexpr int NKST = 6;      // wave tier | sieve large | sieve mid | sieve small | sieve multi-slice | range
  hipEvent_t ev_k[2 * NKST] = {};
  bool kst_live[NKST] = {};
  double kst_ms[NKST] = {}, kst_bytes[NKST] = {}, kst_pend_bytes[NKST] = {};
  int64_t kst_launches[NKST] = {};
  GlbWork* d_work = nullptr;
  int64_t work_cap = 0;
  void* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  int32_t* d_out_ids = nullptr;
  double* d_out_sc = nullptr;
  int32_t* d_out_len = nullptr;
  int flags = 0;
  std::vector<int64_t> h_rp;       // host row pointers (hub planning)
  size_t hub_lds_count = 0, hub_lds_wg = 0, hub_lds_final = 0, hub_lds_wave = 0;
  size_t hub_lds_red = 0;  // k_hub_reduce: hub_lds_final + the LDS-staged slice (red_pl entries, 0 = unstaged)
  int red_pl = 0;
  int hub_bucket = 448, hub_wave_t = 512;  // PPR_HUB_BUCKET, PPR_HUB_WAVE_T (merge_hub.h defaults)
  // pinned host staging of the hub planning (hub list + candidate counts down, descriptors up):
  // pageable copies of these (tens of MB per iteration) stalled the stream for milliseconds
  int32_t* h_hub_pin = nullptr;    // [2 * cap]: hub ids | candidate counts
  size_t h_hub_cap = 0;
  void* h_desc_pin = nullptr;
  size_t h_desc_bytes = 0;
  std::vector<HubBatch> hub_batches;
  int32_t* d_gath = nullptr;       // hub planning gather when 2 * hubs > n (d_ovf is n ints)
  size_t gath_bytes = 0;
  int num_cus = 256;
  int hub_bw_blocks = 0;           // persistent k_hub_bucket_w grid
  bool rank_permute = false;       // PPR_TEST_RANK_PERMUTE (tests): IterArgs WI_RANK_PERMUTE
  uint32_t lds_rank = 0;           // k_probe_lds_rank: 32-bit add ranks in lane order (PPR_LDS_RANK=0 forces the ballot path)
  uint32_t lds_rank64 = 0;         // ... and the 64-bit add order (reported by PPR_TIMING only; round 6:
                                   // the ordered paths check every chain's order themselves, so no
                                   // result depends on either probe)
  bool seg_enabled = false;        // segmented hub buckets (k_hub_seg, PPR_HUB_SEG=1)
  int seg_bucket = 256, seg_t = 512, seg_wpb = 1;
  int hub_bw_ng = 2;               // PPR_BW_NG: groups per chunk (1, 2, 4 or 8)
  bool hub_bw2 = true;             // PPR_BW2: one-shot path for buckets of <= BW2_CAP records
  int hub_wave_stride = 0;         // LDS bytes per bucket wave (chunked table or one-shot table)
  int hub_bw_waves = 1;            // PPR_BW_WAVES: waves per block of k_hub_bucket_w
  int hub_range = 0;               // PPR_HUB_RANGE: buckets per k_hub_range wave (0 = k_hub_bucket_w, one each;
                                   // ranges measured no faster: the bucket stage is LDS-latency bound)
  int hub_slice = 8192;            // PPR_HUB_SLICE: k_hub_reduce slice (>= L)
  // source sharding (ppr_grank_plan_comm_init / ppr_grank_plan_run_sharded)
  ncclComm_t comm = nullptr;
  double x_timeout_s = 600.0;        // PPR_XTIMEOUT: seconds an RCCL wait may go without progress (x_sync)
  int xtest_fail_rank = -1, xtest_fail_it = -1;  // PPR_XTEST_FAIL="rank,it" (tests): that rank fails there
  struct LocalGroup* lgroup = nullptr;  // tests: the ranks are plans of this process (grank.hip)
  int nranks = 1, rank = 0;
  std::vector<double> work[2];        // per active source: merge work estimate (list order)
  unsigned char* d_xsend = nullptr;   // compact block of this rank's rows (merge_glb.h)
  unsigned char* d_xrecv = nullptr;   // the other ranks' blocks
  unsigned char* d_xsz = nullptr;     // int64 block size per rank (all-gathered)
  unsigned char* d_xtmp = nullptr;    // scan temporary of the block offsets
  size_t xsend_bytes = 0, xrecv_bytes = 0, xsz_bytes = 0, xtmp_bytes = 0;
  int64_t fused_max = 65536;          // PPR_FUSED_MAX: MC levels up to this many sources take one host sync (round 5: 16384 -> 65536, combine 926 -> 909 ms)
  int64_t last_nbig = 0, last_maxneed = 0;
  double host_plan_s = 0.0;                  // host time planning hub batches (PPR_TIMING, at destroy)
  int64_t host_plan_calls = 0, host_plan_hubs = 0;
  double host_plan_part[2] = {0.0, 0.0};     // ordering, batch/descriptor loop  // the last hub pass: sources, largest candidate count
  int32_t* ovl_pending = nullptr;     // MC combine: a level's hub overflow list not yet read (run_hubs)
  int64_t x_bytes = 0;                // block bytes received by this rank in the last sharded run
  // consumer routing (grank.hip xroute_build): a row goes only to the ranks whose sources read it;
  // PPR_XROUTE=0 sends every row to every rank (the broadcast exchange)
  bool xroute = true;
  int xtest_badsize = -1;             // tests (PPR_XTEST_BADSIZE=r): rank r advertises wrong block sizes
  int8_t* d_xowner = nullptr;         // [n] rank merging each active node (-1: dangling)
  int32_t* d_own = nullptr;           // sharded init: this rank's active nodes (both partitions), then
  int64_t own_cnt = 0;                // every dangling node (identical on every rank)
  int own_world = 0, own_rank = -1;   // the shard the list was built for
  uint32_t* d_xcmask = nullptr;       // [n] ranks reading each node's row
  int32_t* d_xlists = nullptr;        // per partition: send lists to each peer, receive lists from each peer
  size_t xlists_cap = 0;
  int64_t x_rows_sent = 0;            // rows this rank sent in the last sharded run
  int64_t merge_launches = 0;
  double merge_ms = 0.0;           // sum of merge-phase spans (classify .. last merge kernel)
  hipEvent_t ev_a = nullptr, ev_b = nullptr, ev_m0 = nullptr, ev_m1 = nullptr;
  // PPR_HUB_STREAMS=2 (default): the hub pipeline's bucket stage of batch i runs on stream2 while
  // the partition stage of batch i+1 runs on the plan's stream (two scratch regions), and the wave
  // tiers run on stream3 beside the whole hub pipeline (disjoint sources)
  int hub_streams = 2;
  hipStream_t stream_wave = nullptr;  // the wave tiers' stream (stream3; stream2 in the exact sum with the sieve)
  int wave_wpb = 1;                // PPR_WAVE_WPB: waves per block of k_merge_lds (1, 2 or 4)
  int tile_wpb_p = 4096;           // PPR_TILE_WPB_P: count / scatter run one wave per block from this maxP on
  int tile_split_logp = 10;        // PPR_TILE_SPLIT_LOGP: count / scatter tiles of sources with P <= 2^this
                                   // in a launch of their own (LDS for their P counters only)
  int hub_bw_budget = 380;         // distinct keys a bucket wave's table takes before it spills
  int hub_mix = 6;                 // PPR_HUB_MIX: interleave sources with P >= 2^hub_mix among the others
  int hub_tile_cand = 4096;         // PPR_HUB_TILE_CAND: minimum tile candidates (HUB_TILE_CAND)
  int64_t hub_long_min = 1LL << 26; // PPR_HUB_LONG_MIN: hub candidates of a call from which tile_pb applies
  int hub_tile_pb = 16;             // PPR_HUB_TILE_PB: tile candidates >= this many per bucket (0: 4096 / L)
  int64_t hub_budget = 1LL << 28;  // PPR_HUB_BUDGET: staged candidates per hub batch (16-B records)
  // with PPR_HUB_REGIONS (default 3) scratch regions the partition stage runs up to two batches
  // ahead, and the reduce + final of batch i (stream4) overlap the bucket waves of batch i+1
  static constexpr int MAX_REGIONS = 4;
  int hub_regions = 3;
  hipStream_t stream2 = nullptr, stream3 = nullptr, stream4 = nullptr;
  hipEvent_t ev_part[MAX_REGIONS] = {}, ev_buck[MAX_REGIONS] = {}, ev_fin[MAX_REGIONS] = {}, ev_wave = nullptr;
  unsigned long long* d_diag = nullptr;  // PPR_DIAG=1: kernel histograms, printed at destroy
  // hot key set of the hub path (merge_hot.h): chosen at iteration hot_at of every run from rows
  // sampled every hot_stride nodes; hot_cap = PPR_HOT_N (0 disables the hot pass)
  int hot_cap = 0, hot_at = 2, hot_stride = 16;  // measured: no net gain at RMAT-22
  int hot_n = 0;                      // members of the current set (0 until it is built)
  int32_t hot_built_it = -1;          // iteration of this run that built it (sharded runs iterate per range)
  std::vector<int32_t> h_hot_keys;    // host copy (fetch_slab decodes stored ids)
  int hot_max_need = 0x7fffffff;      // PPR_HOT_MAX: sources with more candidates skip the hot pass
  double diag_cap_cand = 0.0, diag_cap_src = 0.0;  // PPR_DIAG: hub sources past 2^HUB_MAX_LOGP full buckets
  double diag_hub_cand = 0.0;         // PPR_DIAG: candidates of the hub sources planned (iterations)
  uint32_t* d_hot_bits = nullptr;     // [ceil(n / 32)]
  uint16_t* d_hot_idx = nullptr;      // [n]
  int32_t* d_hot_keys = nullptr;      // [hot_cap]
  uint32_t* d_hot_w = nullptr;        // [n] weights
  uint32_t* d_hot_hist = nullptr;     // [HOT_BINS + 2]: histogram, then the collect counters
  int32_t* d_hot_list = nullptr;      // [hot_list_cap]: collected keys
  int64_t hot_list_cap = 0;
  int32_t* d_indeg = nullptr;         // [n] in-degree (how many sources read the node's row)
  hipStream_t stream5 = nullptr;      // k_hub_hot beside the partition / bucket stages
  hipEvent_t ev_hot0 = nullptr, ev_hot[MAX_REGIONS] = {};
  // exact-sum GRank (merge_xs.h; PPR_FLAG_CHAIN_SUM / PPR_SUM=chain turn it off)
  bool xsum = false;
  int32_t* d_dlast = nullptr;         // [n] distinct keys of each source's last merge (hub planning)
  int xr_T = 8192, xr_W = 16;         // PPR_XR_T: range / bucket workgroup table slots (waves = T / 512)
  int xr_rmax = 3;                    // PPR_XR_RMAX: most key ranges a source is walked in (beyond: partition)
  int xr_fill = 85;                   // PPR_XR_FILL: planned distinct keys per table, % of its slots (round-5 sweep: 80 -> 85, -0.3-0.6 %)
  int xf_stage = 4096;                // k_xfinal entries staged in LDS
  int xr_dscale = 100;                // PPR_XR_DSCALE (tests): distinct-key estimates scaled, % (forces overflows)
  unsigned char* d_xs = nullptr;      // range-workgroup scratch (descriptors, tasks, lists)
  size_t xs_bytes = 0;
  void* h_xs_pin = nullptr;           // pinned staging of its descriptors and tasks
  size_t h_xs_bytes = 0;
  int64_t xr_redo = 0;                // sources redone after a table overflow (PPR_TIMING at destroy)
  // exact-sum HBM-table fallback (merge_xg.h): sources past the bucket partition's reach
  int hub_max_logp = 12;              // PPR_HUB_MAX_LOGP (tests): most bucket bits of an exact-sum partition
                                      // (<= merge_hub.h HUB_MAX_LOGP)
  unsigned char* d_xg = nullptr;      // table | dense list | state | histogram
  size_t xg_bytes = 0;
  int64_t xg_sources = 0;             // sources merged there (PPR_TIMING at destroy)
  // bounded probes (tests force them to run out): exact wave-tier overflow list and knobs
  int32_t* d_wovl = nullptr;          // [1 + n]: count, sources whose wave-tier table ran out
  int wave_split_T = 256;             // PPR_WAVE_SPLIT: wave tiers with T >= this end in k_wfin (0: none)
  int wave_split_chain = 256;         // PPR_WAVE_SPLIT_CHAIN: the same for GRank's chain-order wave tiers
                                      // (round 6: -1.3 % per chain job)
  int wave_split_mc = 0;              // PPR_WAVE_SPLIT_MC: ... and the MC combine's (+1.6-2 %: off)
  // run_xhubs's per-call host lists, kept across iterations (capacity only): fresh vectors of a
  // few hundred thousand entries each cost the planning their page faults every iteration
  struct XhScratch {
    std::vector<int32_t> h, src, cand, deg, ssrc, scand, sdeg, sidx, back;
    std::vector<int64_t> dest;
    std::vector<uint16_t> svkey;
    std::vector<uint32_t> svcnt;
  } xhs;
  double xh_sub[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // (PPR_SV_LOG) host planning sub-phases, seconds
  int xr_cap = 0;                     // PPR_XR_LISTCAP: one-range k_xr sources emit up to this many unselected
                                      // entries for k_xfin1 (set to 2 Lp at plan creation; 0: k_xr selects)
  int wave_cap = 0;                   // (tests) PPR_WAVE_CAP: list entries per split source (>= L; 0: 2 Lp)
  unsigned char* d_wl = nullptr;      // their lists (merge_xs.h WList)
  size_t wl_max = (size_t)4 << 30;    // PPR_WL_MAX_MB: most list bytes of one split-tier launch (else chunks)
  size_t wl_bytes = 0;
  bool wave_x_launched = false;
  int wave_tdiv = 0;                  // PPR_WAVE_TDIV (tests): wave-tier tables T >> this
  bool wave_by_d = false;             // PPR_WAVE_BY_D: exact-sum wave tiers by last distinct keys
  bool xr_budget_over = false;        // PPR_XR_BUDGET=over (tests): range / bucket tables fill up
  int64_t wave_redo = 0;              // wave-tier sources redone (PPR_TIMING at destroy)
  int xg_cap = 1 << 16;               // dense list of the selection (PPR_XG_CAP, tests: L <= cap <= XG_CAP)
  // sieve merge of the wide exact-sum sources (merge_sv.h): PPR_SV=0 turns it off
  bool sv_enabled = false;
  int64_t sv_slice = 1LL << 19;       // PPR_SV_SLICE: candidates per slice workgroup (round-5 sweep: 2^18 -> 2^19, -1.6 %)
  // read per plan in plan_alloc (a process may switch them between plans; tests cover both ways)
  bool xm = false;                    // PPR_XM=1: k_xm for the one-range sources of the 2048-slot class
  bool xr_big_first = false;          // PPR_XR_ORDER=1: range tasks largest source first (experiment)
  bool xh_first = true;               // PPR_XH_FIRST: range engines planned and queued before the sieve
  bool xshard_ends = true;            // PPR_XSHARD_ENDS: sharded init and K-wide top-K (routed exchange)
  int64_t sv_min = 4096;              // PPR_SV_MIN: sources with fewer candidates keep the range engines
                                      // (measured: 4096 beats 0 by 2-3 % -- the smallest sources overflow the
                                      // 4-wave class's sketch and were handed back -- and 16384 by 5 %)
  bool sv_redo_mid = true;            // PPR_SV_REDO=0: small-class overflows go straight to the host hand-back
  bool sv_p2skip = true;             // PPR_SV_P2SKIP=0: pass 2 runs even when a sketch row proves it inserts nothing
  bool sv_redo_large = false;         // PPR_SV_REDO_LARGE=1: mid-class overflows redone on the device (k_sv1_list;
                                      // off by default: at RMAT-22 the mid class now overflows ~1 source per job,
                                      // and the redo grid's 113-KB workgroups still pass through the CUs)
  int sv_budget = 2457;               // PPR_SV_BUDGET (tests): passing keys a table takes (<= SV_XT_BUDGET)
  int64_t sv_small = 32768, sv_mid = 65536;  // PPR_SV_SMALL / PPR_SV_MID: one-slice size classes by candidates
                                      // (same-box sweep of SV_SMALL 16 K / 32 K / 48 K / 64 K: 1632 / 1589-1594 /
                                      // 1593 / 1664 ms per job; SV_MID 32 K / 131 K: +-0)
  hipStream_t stream_sv = nullptr, stream_sv2 = nullptr, stream_sv3 = nullptr;  // large + multi-slice | mid | small
                                      // (borrowed: stream2 / stream4 / stream5, not owned)
  hipEvent_t ev_sv = nullptr;
  unsigned char* d_sv = nullptr;      // descriptors, tasks, overflow list, global sketches / tables
  size_t sv_bytes = 0;
  void* h_sv_pin = nullptr;           // pinned staging of descriptors and tasks, overflow count
  size_t h_sv_bytes = 0;
  int64_t sv_sources = 0, sv_redo = 0;  // sieved sources, handed back after an overflow (PPR_TIMING)
  int64_t sv_redo_dev = 0;            // small / mid-class overflows redone on the device (mid / large geometry)
  double xh_s[8] = {};                // run_xhubs host sections, s (PPR_TIMING at destroy)
  // MCCompletePathV2 (mccp2.hip)
  bool mc = false;
  int32_t* d_mc_walk = nullptr;       // walk set W (nodes read before their final basket exists)
  int64_t mc_nwalk = 0;
  int32_t* d_mc_levels = nullptr;     // non-dangling nodes grouped by combine level
  std::vector<int64_t> mc_level_off;  // level l = d_mc_levels[off[l] .. off[l+1])
  int32_t* d_mc_dangling = nullptr;
  int64_t mc_ndangling = 0;
  int mc_T = 0;
  double mc_walk_ms = 0.0;
  int64_t mc_walks = 0;
};

inline void plan_free(ppr_plan* p) {
  if (!p) return;
  hipFree(p->d_rp); hipFree(p->d_colx); hipFree(p->d_part); hipFree(p->d_ids); hipFree(p->d_sc); hipFree(p->d_rix); hipFree(p->d_rmin);
  hipFree(p->d_len); hipFree(p->d_all); hipFree(p->d_act[0]); hipFree(p->d_act[1]);
  hipFree(p->d_cand); hipFree(p->d_tier_lists); hipFree(p->d_tier_cnt); hipFree(p->d_tier_cap); hipFree(p->d_big);
  hipFree(p->d_ovf); hipFree(p->d_gath); hipFree(p->d_dlast); hipFree(p->d_xs);
  hipFree(p->d_maxdiff); hipFree(p->d_stats); hipFree(p->d_work); hipFree(p->d_scratch);
  hipFree(p->d_out_ids); hipFree(p->d_out_sc); hipFree(p->d_out_len);
  if (p->ev_a) hipEventDestroy(p->ev_a);
  if (p->ev_b) hipEventDestroy(p->ev_b);
  if (p->ev_m0) hipEventDestroy(p->ev_m0);
  if (p->ev_m1) hipEventDestroy(p->ev_m1);
  for (int i = 0; i < ppr_plan::MAX_REGIONS; i++) {
    if (p->ev_part[i]) hipEventDestroy(p->ev_part[i]);
    if (p->ev_buck[i]) hipEventDestroy(p->ev_buck[i]);
    if (p->ev_fin[i]) hipEventDestroy(p->ev_fin[i]);
  }
  if (p->ev_wave) hipEventDestroy(p->ev_wave);
  for (int i = 0; i < 2 * ppr_plan::NKST; i++)
    if (p->ev_k[i]) hipEventDestroy(p->ev_k[i]);
  if (p->ev_hot0) hipEventDestroy(p->ev_hot0);
  for (int i = 0; i < ppr_plan::MAX_REGIONS; i++)
    if (p->ev_hot[i]) hipEventDestroy(p->ev_hot[i]);
  if (p->stream5) hipStreamDestroy(p->stream5);
  hipFree(p->d_hot_bits); hipFree(p->d_hot_idx); hipFree(p->d_hot_keys); hipFree(p->d_hot_w);
  hipFree(p->d_hot_hist); hipFree(p->d_hot_list); hipFree(p->d_indeg);
  if (p->stream2) hipStreamDestroy(p->stream2);
  if (p->stream3) hipStreamDestroy(p->stream3);
  if (p->stream4) hipStreamDestroy(p->stream4);
  if (p->comm) ncclCommDestroy(p->comm);
  hipFree(p->d_xsend); hipFree(p->d_xrecv); hipFree(p->d_xsz); hipFree(p->d_xtmp);
  hipFree(p->d_xowner); hipFree(p->d_xcmask); hipFree(p->d_xlists); hipFree(p->d_own);
  if (p->h_hub_pin) hipHostFree(p->h_hub_pin);
  if (p->h_desc_pin) hipHostFree(p->h_desc_pin);
  if (p->h_xs_pin) hipHostFree(p->h_xs_pin);
  hipFree(p->d_sv);
  hipFree(p->d_xg);
  hipFree(p->d_wovl);
  hipFree(p->d_wl);
  if (p->h_sv_pin) hipHostFree(p->h_sv_pin);
  if (p->ev_sv) hipEventDestroy(p->ev_sv);
  if (getenv("PPR_TIMING") && p->sv_sources)
    fprintf(stderr, "ppr_timing sieve_sources %lld sieve_redo %lld sieve_redo_dev %lld\n", (long long)p->sv_sources,
            (long long)p->sv_redo, (long long)p->sv_redo_dev);
  if (getenv("PPR_TIMING") && p->sv_sources)
    fprintf(stderr, "ppr_timing xhubs_host_s gather %.4f classify %.4f sieve_launch %.4f engines %.4f sieve_wait %.4f "
            "handback_plan %.4f handback_run %.4f\n", p->xh_s[0], p->xh_s[1], p->xh_s[2], p->xh_s[3], p->xh_s[4],
            p->xh_s[5], p->xh_s[6]);
  if (getenv("PPR_TIMING") && p->xr_redo)
    fprintf(stderr, "ppr_timing xr_redo_sources %lld\n", (long long)p->xr_redo);
  if (getenv("PPR_TIMING") && p->wave_redo)
    fprintf(stderr, "ppr_timing wave_redo_sources %lld\n", (long long)p->wave_redo);
  if (getenv("PPR_TIMING") && p->xg_sources)
    fprintf(stderr, "ppr_timing hbm_table_sources %lld\n", (long long)p->xg_sources);
  if (getenv("PPR_TIMING") && p->spec_redo)
    fprintf(stderr, "ppr_timing spec_redo_sources %lld\n", (long long)p->spec_redo);
  if (getenv("PPR_TIMING") && p->host_plan_calls)
    fprintf(stderr, "ppr_timing hub_paths lds_rank %u lds_rank64 %u one_shot %d\n", p->lds_rank, p->lds_rank64,
            (int)p->hub_bw2);
  if (getenv("PPR_TIMING") && p->host_plan_calls)
    fprintf(stderr, "ppr_timing hub_planning host_s %.4f calls %lld hubs %lld order_s %.4f batches_s %.4f\n",
            p->host_plan_s, (long long)p->host_plan_calls, (long long)p->host_plan_hubs, p->host_plan_part[0],
            p->host_plan_part[1]);
  if (p->d_diag) {
    std::vector<unsigned long long> hv(PPR_DIAG_SLOTS);
    if (hipMemcpy(hv.data(), p->d_diag, 8 * hv.size(), hipMemcpyDeviceToHost) == hipSuccess) {
      unsigned long long h[PPR_DIAG_BASE];
      for (int i = 0; i < PPR_DIAG_BASE; i++) {  // shards summed (max-type counters are unsharded)
        h[i] = hv[i];
        for (int sh = 1; sh <= PPR_DIAG_SHARDS; sh++) h[i] += hv[(size_t)sh * PPR_DIAG_BASE + i];
      }
      fprintf(stderr, "ppr_diag bucket_w: log2(x) | buckets by len, Mcycles | by distinct keys | by kept keys\n");
      for (int b = 0; b < 32; b++)
        if (h[b] || h[64 + b] || h[96 + b])
          fprintf(stderr, "ppr_diag %2d %12llu %12.1f | %12llu | %12llu\n", b, h[b], h[32 + b] / 1e6,
                  h[64 + b], h[96 + b]);
      if (h[144])
        fprintf(stderr, "ppr_diag hot pass: %d keys, %llu tasks, hub candidates %.3e staged (cold) %.3e (%.1f %%), "
                "task ms: longest %.2f, first %.2f, sum %.1f\n", p->hot_n, h[144], p->diag_hub_cand, (double)h[140],
                100.0 * (double)h[140] / (p->diag_hub_cand > 0 ? p->diag_hub_cand : 1.0), h[141] / 1e5, h[143] / 1e5,
                h[142] / 1e5);
      if (p->diag_cap_src > 0)
        fprintf(stderr, "ppr_diag sources beyond the bucket cap %.0f, candidates %.3e of %.3e\n", p->diag_cap_src,
                p->diag_cap_cand, p->diag_hub_cand);
      if (h[296]) {  // (-DPPR_PHASE_TIMING builds) one-shot bucket phases, lane 0
        const double tot = (double)(h[288] + h[289] + h[290] + h[291] + h[292] + h[293] + h[294] + h[295]);
        fprintf(stderr, "ppr_diag one-shot buckets %llu, %.1f K cycles each: loads+clear %.1f %% P1 %.1f %% P2 %.1f %% "
                "P3 %.1f %% P4 %.1f %% count+select %.1f %% append atomic %.1f %% emit %.1f %%\n", h[296],
                tot / 1e3 / (double)h[296], 100.0 * h[288] / tot, 100.0 * h[289] / tot, 100.0 * h[290] / tot,
                100.0 * h[291] / tot, 100.0 * h[292] / tot, 100.0 * h[293] / tot, 100.0 * h[294] / tot,
                100.0 * h[295] / tot);
      }
      if (h[152])
        fprintf(stderr, "ppr_diag spilled buckets %llu, records %llu (%.1f per bucket)\n", h[152], h[153],
                (double)h[153] / (double)h[152]);
      if (h[150])
        fprintf(stderr, "ppr_diag rows merged %llu, unchanged (norm1 = 0) %llu (%.2f %%)\n", h[150], h[151],
                100.0 * (double)h[151] / (double)h[150]);
      if (h[180]) {
        fprintf(stderr, "ppr_diag speculative bound: %llu hub sources, %llu failed (%.3f %%); failures by iteration:",
                h[180], h[181], 100.0 * (double)h[181] / (double)h[180]);
        for (int it = 0; it < 32; it++)
          if (h[224 + it]) fprintf(stderr, " %d:%llu", it, h[224 + it]);
        fprintf(stderr, "\n");
      }
      if (h[166]) {
        const double tot = (double)(h[160] + h[161] + h[162] + h[163] + h[164] + h[165]);
        fprintf(stderr, "ppr_diag bucket_w phases, 1 wave in 8 (%llu waves, %.3e records, %.1f Gcycles): work+setup %.1f %% loads %.1f %% "
                "insert %.1f %% accumulate %.1f %% compact+select %.1f %% append %.1f %%; buckets selecting (U > L) %llu, "
                "entries appended %.3e\n", h[166], (double)h[167], tot / 1e9, 100.0 * h[160] / tot, 100.0 * h[161] / tot,
                100.0 * h[162] / tot, 100.0 * h[163] / tot, 100.0 * h[164] / tot, 100.0 * h[165] / tot, h[168],
                (double)h[169]);
        const double acc = (double)(h[172] + h[173] + h[174] + h[175]);
        if (acc > 0)
          fprintf(stderr, "ppr_diag bucket_w accumulate phases: A occurrence ranks %.1f %% B slot offsets %.1f %% "
                  "C value placement %.1f %% D per-slot chains %.1f %%\n", 100.0 * h[172] / acc, 100.0 * h[173] / acc,
                  100.0 * h[174] / acc, 100.0 * h[175] / acc);
      }
      if (h[182])
        fprintf(stderr, "ppr_diag k_xr: %llu workgroups, %.3e successor edges walked, %.3e distinct keys; Gcycles "
                "(thread 0) setup %.2f accumulate %.2f settle %.2f select %.2f finish %.2f\n", h[182], (double)h[188],
                (double)h[189], h[183] / 1e9, h[184] / 1e9, h[185] / 1e9, h[186] / 1e9, h[187] / 1e9);
      if (h[135] || h[149])
        fprintf(stderr, "ppr_diag sieve: %llu one-slice sources (%llu handed back), %llu multi-slice; passing keys %.3e "
                "(candidates %.3e), entries beside the prev keys at the select %.3e; pass 2 skipped (a sketch "
                "row below the bound) %llu, sources with no new key (U = L) %llu\n", h[135], h[137], h[149],
                (double)h[136], (double)h[138], (double)h[139], h[145], h[146]);
      if (h[190])
        fprintf(stderr, "ppr_diag sieve pass 2: %.3e groups walked, %.3e with a lane past the bitmap test; %.3e insert "
                "steps (staging-list flushes or groups) inserting %.3e non-prev candidates\n", (double)h[190],
                (double)h[147], (double)h[148], (double)h[138]);
      if (h[280])
        fprintf(stderr, "ppr_diag wave tier: %llu sources, %.1f kept entries each; kcycles per source (lane 0): "
                "setup+walk %.2f settle %.2f select %.2f row write %.2f norm1 %.2f\n", h[280],
                (double)h[287] / (double)h[280], h[281] / 1e3 / (double)h[280], h[282] / 1e3 / (double)h[280],
                h[283] / 1e3 / (double)h[280], h[284] / 1e3 / (double)h[280], h[285] / 1e3 / (double)h[280]);
      for (int c = 0; c < 3; c++) {
        const unsigned long long* q = h + 256 + 8 * c;
        if (q[5])
          fprintf(stderr, "ppr_diag sieve class %s: %llu sources, %.1f successor rows each, %llu handed back; Mcycles "
                  "per source (thread 0): setup %.3f pass1 %.3f bound %.3f pass2 %.3f select %.3f\n",
                  c == 0 ? "large" : c == 1 ? "mid" : "small", q[5], (double)q[6] / (double)q[5], q[7],
                  q[0] / 1e6 / (double)q[5], q[1] / 1e6 / (double)q[5], q[2] / 1e6 / (double)q[5],
                  q[3] / 1e6 / (double)q[5], q[4] / 1e6 / (double)q[5]);
      }
      if (h[154])
        fprintf(stderr, "ppr_diag k_xb: %llu workgroups, %.3e records (%.0f per bucket); Gcycles (thread 0) setup+accumulate "
                "%.2f settle %.2f select %.2f emit %.2f\n", h[154], (double)h[159], (double)h[159] / (double)h[154],
                h[155] / 1e9, h[156] / 1e9, h[157] / 1e9, h[158] / 1e9);
      if (h[170]) {
        fprintf(stderr, "ppr_diag hub final: %llu sources, appended entries %.3e (%.1f per source, %.1f x L); by log2(entries):",
                h[170], (double)h[171], (double)h[171] / (double)h[170], (double)h[171] / (double)h[170] / (double)p->L);
        for (int b = 0; b < 32; b++)
          if (h[192 + b]) fprintf(stderr, " %d:%llu", b, h[192 + b]);
        fprintf(stderr, "\n");
      }
      if (h[133])
        fprintf(stderr, "ppr_diag k_hub_seg: %llu waves, %.1f candidates/wave, Mcycles setup %.1f window %.1f "
                "gather %.1f accumulate %.1f emit %.1f\n", h[133], (double)h[134] / (double)h[133], h[128] / 1e6,
                h[129] / 1e6, h[130] / 1e6, h[131] / 1e6, h[132] / 1e6);
    }
    hipFree(p->d_diag);
  }
  hipFree(p->d_mc_walk); hipFree(p->d_mc_levels); hipFree(p->d_mc_dangling);
  if (p->own_stream && p->stream) hipStreamDestroy(p->stream);
  delete p;
}

inline int check_params(uint32_t K, uint32_t L, uint32_t iterations, double damping) {
  if (K == 0) return PPR_ERR_K;
  if (L == 0) return PPR_ERR_L;
  if (K > L) return PPR_ERR_KL;
  if (iterations == 0) return PPR_ERR_ITERS;
  if (damping < 0 || damping > 1) return PPR_ERR_DAMPING;
  return PPR_OK;
}

inline DevSlab dev_slab(const ppr_plan* p) {
  return DevSlab{p->d_ids, p->d_sc, p->d_len, p->n, (int32_t)p->L, p->d_rix, p->d_rmin,
                 p->d_hot_bits, p->d_hot_idx, p->d_hot_keys, p->hot_n};
}

// grow-only pinned host buffer
inline int ensure_pinned(void** ptr, size_t* cap, size_t need) {
  if (need <= *cap) return PPR_OK;
  if (*ptr) hipHostFree(*ptr);
  *ptr = nullptr;
  *cap = 0;
  need = need + need / 4 + 4096;
  if (hipHostMalloc(ptr, need, hipHostMallocDefault) != hipSuccess) return PPR_ERR_OOM;
  *cap = need;
  return PPR_OK;
}

template <class T>
inline int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, sizeof(T) * count) != hipSuccess) return PPR_ERR_OOM;
  return PPR_OK;
}

#define TRY(x) do { int _r = (x); if (_r != PPR_OK) { plan_free(p); return _r; } } while (0)

// plan buffers + merge tiers for a CSR whose colx (successor | read-slot bit << 31) is given;
// no partitions, no active lists (grank.hip / mccp2.hip add their own)
// (mc: the MCCompletePathV2 combine's bucket defaults, HUB_BUCKET_MC / HUB_WAVE_T_MC)
int plan_alloc(int64_t n, const int64_t* row_ptr, const int32_t* colx, uint32_t K, uint32_t L,
               double damping, const ppr_opts* o, ppr_plan** out, bool mc = false);
namespace pprpart {  // partition.hip: the BFS 2-colouring on graph arrays already in HBM
int partitions_core(const int64_t* d_rp, int32_t* d_col, int64_t n, int64_t m, uint8_t* d_part, uint8_t* h_part,
                    bool mark, int32_t* d_src, int32_t* d_lab, int32_t* d_depth, int32_t* d_flag, hipStream_t st);
}
// final top-K: prefix K of the row in slot sA (partition 0 nodes) / sB (partition 1 nodes)
int launch_topk(ppr_plan* p, int sA, int sB, const int8_t* owner = nullptr, int rank = 0);
// classify + every merge tier for `count` sources of the device list `list`
// MC combine: read and redo the last level's deferred hub overflow list (host sync)
int run_merge_flush(ppr_plan* p, const IterArgs& a, unsigned long long* maxdiff);
int probe_take();  // grank.hip: PPR_ERR_PROBE when one of its kernels' bounded probes ran out
int run_merge(ppr_plan* p, const IterArgs& a, const int32_t* list, int64_t count,
              unsigned long long* maxdiff);
