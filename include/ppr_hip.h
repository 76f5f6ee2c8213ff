/*
 * ppr_hip.h -- C ABI of the MI355X-native all-sources approximate PPR engine (libppr_hip.so).
 *
 * The reference (fruttasecca/approximated_personalized_pagerank) has no FFI: its surface is the
 * C++ templates ppr::grank / ppr::grankMulti / ppr::mccompletepathv2. This ABI is what those
 * templates bind to in the drop-in headers include/ppr/grank.h, include/ppr/grankMulti.h and
 * include/ppr/mccompletepathv2.h (same signatures as the reference), and what the Python mirror
 * binds with ctypes. Plain pointers and sizes only; no torch / HIP types in signatures
 * (streams are passed as void*).
 *
 * Dense ids: node i is the i-th key of the graph in its iteration order; col[] keeps each
 * node's successor order (the reference sums contributions in that order,
 * include/grank.h:107-116, and its partitions depend on the iteration order,
 * include/internal/pprInternal.h:57-63).
 *
 * All entry points are synchronous unless stated, thread-safe per call, and keep no globals.
 * Return value: PPR_OK (0) or a PPR_ERR_* code; ppr_strerror() names it.
 */
#ifndef PPR_HIP_H
#define PPR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  PPR_OK = 0,
  PPR_ERR_ARG = 1,       /* bad pointer / size */
  PPR_ERR_K = 2,         /* "K must be positive"          include/grank.h:51 */
  PPR_ERR_L = 3,         /* "L must be positive"          include/grank.h:52 */
  PPR_ERR_KL = 4,        /* "K must be <= L"              include/grank.h:53 */
  PPR_ERR_ITERS = 5,     /* "iterations must be positive" include/grank.h:54 */
  PPR_ERR_DAMPING = 6,   /* "damping must be [0,1]"       include/grank.h:55 */
  PPR_ERR_THREADS = 7,   /* "nThreads must be positive"   header-only/grankMulti.h:304 */
  PPR_ERR_GRAPH = 8,     /* successor id out of range (UB in the reference, README.md:69-73) */
  PPR_ERR_HIP = 9,       /* HIP runtime failure (no device, launch failure, ...) */
  PPR_ERR_OOM = 10,      /* device allocation failed */
  PPR_ERR_RANGE = 11,    /* L / K / node count beyond what the kernels support */
  PPR_ERR_SOURCE = 12,   /* "source node not part of the graph" include/internal/pprSingleSource.h:39 */
  PPR_ERR_PROBE = 13     /* a bounded hash probe ran out of slots: a table sizing error (never on a
                            correct build; the exact-sum engines redo such a source instead) */
};

/* graph in dense CSR form (borrowed; host memory unless a *_dev entry point says otherwise) */
typedef struct ppr_csr {
  int64_t n;               /* nodes */
  const int64_t* row_ptr;  /* [n+1], row_ptr[0] = 0, edges m = row_ptr[n] */
  const int32_t* col;      /* [m] dense successor ids, successor order preserved */
} ppr_csr;

typedef struct ppr_opts {
  int32_t device;          /* HIP device ordinal; -1 = current device */
  int32_t flags;           /* PPR_FLAG_* */
  void* stream;            /* hipStream_t to run on; NULL = library-owned stream */
} ppr_opts;

enum {
  PPR_FLAG_STATS = 1,      /* collect candidate counts / algorithmic bytes per iteration */
  PPR_FLAG_CHAIN_SUM = 2   /* GRank: sum each key's contributions with the reference's in-order fma
                              chain (include/grank.h:107-116; bit-identical to it where no top-L tie
                              is cut). Default: the exact sum -- every contribution fl(s * d/deg)
                              added exactly, rounded once (order-free). The
                              environment variable PPR_SUM=chain|exact overrides the default. */
};

#define PPR_MAX_ITER_STATS 256

typedef struct ppr_stats {
  int32_t iterations_run;          /* iterations actually executed (tolerance may stop early) */
  int32_t reserved;
  double max_diff[PPR_MAX_ITER_STATS];   /* maxDiff of the partition updated in iteration i */
  double device_ms;                /* init + iterations + final top-K, device events */
  double merge_ms;                 /* basket-merge kernels only (sum over iterations) */
  int64_t candidates;              /* sum over iterations of candidates (PPR_FLAG_STATS) */
  int64_t algo_bytes;              /* SURVEY s8d algorithmic bytes over iterations (STATS) */
  int64_t merge_launches;          /* number of merge-kernel launches */
} ppr_stats;

const char* ppr_strerror(int code);

/* Build record of this library: "ppr_src_sha256=<hex> arch=<gfx target> hipcc=<clang version>".
 * The digest covers every source and header the library was compiled from (build.py); the Python
 * loader refuses a library whose digest differs from the sources beside it. No reference
 * counterpart (provenance of the drop-in binary). */
const char* ppr_build_info(void);

/* ---- host-side graph preparation (no GPU) ---- */

/* BFS 2-colouring of include/internal/pprInternal.h:29-99; part[i] = 0 for partitions.first */
int ppr_find_partitions_csr(const ppr_csr* g, uint8_t* part);
/* The same partitions computed on the device (`device` < 0: the current one): min-label components
 * and a level-synchronous BFS from each component's first node (csrc/partition.hip). Returns
 * PPR_ERR_RANGE for graphs that need more rounds than it allows (long paths): use the host BFS.
 * ppr_grank_plan_create / ppr_grank_csr take it when the caller passes no partitions, falling back
 * to the host BFS (PPR_HOST_BFS=1: the host BFS only). */
int ppr_find_partitions_csr_device(const ppr_csr* g, uint8_t* part, int32_t device);

/* MCCompletePathV2 node order, include/mccompletepathv2.h:36-113 (the same library sort on the
 * same records, so ties come out in the reference's order) */
int ppr_execution_order_csr(const ppr_csr* g, int32_t* order);

/* Edge-list importer of the reference CLI (src/main.cc:78-112): "a,b" per line, targets inserted
 * first, repeated edges kept once; dense ids follow the resulting unordered_map's iteration order
 * (the reference's). Call with keys/row_ptr/col NULL for n and m, then with buffers. */
int ppr_import_edge_csv(const char* path, int64_t* n, int64_t* m, int32_t* keys, int64_t* row_ptr,
                        int32_t* col);

/* Synthetic RMAT graph (Graph500 recursion, scrambled labels, deduped, successors ascending).
 * Call with col = NULL to get m (row_ptr[n+1] is filled either way); returns m or -error. */
int64_t ppr_rmat_generate(int32_t scale, int32_t edge_factor, double a, double b, double c,
                          uint64_t seed, int64_t* row_ptr, int32_t* col, int64_t col_cap);

/* ---- GRank (ppr::grank / ppr::grankMulti, include/grank.h:42-150) ----
 * One call: upload, init, iterate, final top-K, download. out_ids / out_scores are n*K
 * (row v = the K best (id, score) of source v, score desc, id asc; unused slots id -1),
 * out_len is n. part: partition bits from ppr_find_partitions_csr (or NULL to compute). */
int ppr_grank_csr(const ppr_csr* g, const uint8_t* part, uint32_t K, uint32_t L,
                  uint32_t iterations, double damping, double tolerance, const ppr_opts* o,
                  int32_t* out_ids, double* out_scores, int32_t* out_len, ppr_stats* st);

/* ---- device-resident plan (benchmarks, multi-GPU source sharding) ---- */
typedef struct ppr_plan ppr_plan;

/* Uploads the CSR and partition lists to HBM and allocates the two L-wide basket slabs. */
int ppr_grank_plan_create(const ppr_csr* g, const uint8_t* part, uint32_t K, uint32_t L,
                          double damping, const ppr_opts* o, ppr_plan** out);
void ppr_grank_plan_destroy(ppr_plan* p);

/* Whole device phase: init baskets, run up to `iterations` with the reference's stopping rule,
 * final top-K into the plan's device output. Inputs are already resident. */
int ppr_grank_plan_run(ppr_plan* p, uint32_t iterations, double tolerance, ppr_stats* st);

/* Step-level entry points (multi-GPU sharding; each is asynchronous on the plan's stream):
 *   init:    initial baskets of every node
 *   iterate: merge the active sources with index [begin, end) of iteration `it`'s active list
 *            (the partition's non-dangling nodes in dense-id order, see ppr_grank_plan_active_list), writing
 *            their new rows into the next-slot slab and folding norm1 into a device max
 *   finish:  final top-K of every node into the device output */
int ppr_grank_plan_init(ppr_plan* p);
int ppr_grank_plan_active_count(ppr_plan* p, int32_t it, int64_t* count);
int ppr_grank_plan_iterate(ppr_plan* p, int32_t it, int64_t begin, int64_t end);
int ppr_grank_plan_read_maxdiff(ppr_plan* p, int32_t it, double* maxdiff); /* syncs */
int ppr_grank_plan_finish(ppr_plan* p, int32_t iterations_run);

/* Row exchange for source sharding: pack/unpack of an active-list range of the rows iteration `it`
 * wrote, as one compact block: int64 off[cnt + 1] (payload offset per row, off[cnt] = payload
 * bytes), then per row int32 ids[Le] and f64 scores[len] (Le = len rounded up to even; a row
 * takes 12 len (+4 if len is odd) bytes, so len = (off[r+1] - off[r]) / 12). Only the entries
 * travel; the receiver rebuilds each row's minimum and hash-range index. Block size =
 * 8 (cnt + 1) + off[cnt] <= 8 + cnt * ppr_grank_plan_row_bytes; `cap` is the buffer's capacity.
 * Asynchronous on the plan's stream. */
int ppr_grank_plan_row_bytes(ppr_plan* p, int64_t* bytes);
int ppr_grank_plan_pack(ppr_plan* p, int32_t it, int64_t begin, int64_t end, void* dev_buf, int64_t cap);
int ppr_grank_plan_unpack(ppr_plan* p, int32_t it, int64_t begin, int64_t end, const void* dev_buf);
/* Active sources of iteration `it` in list order (host copy, nact entries), and the write-back of
 * an all-reduced maxDiff for a sharded iteration. */
int ppr_grank_plan_active_list(ppr_plan* p, int32_t it, int32_t* out);
int ppr_grank_plan_fold_maxdiff(ppr_plan* p, int32_t it, double maxdiff);

/* ---- source sharding over RCCL (one process per GPU) ----
 * Replaces the reference's per-iteration thread fan-out (header-only/grankMulti.h:376-396).
 * Rank 0 creates a 128-byte RCCL unique id, the caller broadcasts it (any channel), and every rank
 * calls ppr_grank_plan_comm_init. ppr_grank_plan_run_sharded then runs the whole job like
 * ppr_grank_plan_run, but each rank merges only its work-balanced range of every iteration's
 * active list (ppr_grank_plan_shard_bounds) and the rows it wrote travel as compact blocks on the
 * plan's stream:
 *   routed (default, up to 32 ranks): a row goes only to the ranks whose sources read it (its
 *     consumers, computed once per run from the CSR and the fixed bounds); per iteration one
 *     grouped ncclSend/ncclRecv of the exact 8-byte block sizes, then one of the blocks; after
 *     the last iteration each partition's final rows are broadcast once, so every rank ends with
 *     the whole slab;
 *   PPR_XROUTE=0: every rank's block to every rank (grouped ncclBroadcast at the block's bound,
 *     8 + rows * ppr_grank_plan_row_bytes, no size exchange).
 * maxDiff is combined with ncclAllReduce(MAX) on its IEEE bits, so every rank applies the
 * reference's stopping rule to the same value. Results equal the 1-GPU run bit for bit.
 * ppr_grank_plan_exchange_bytes: block bytes this rank received and rows it sent in its last
 * sharded run (no reference counterpart: measurement). */
int ppr_device_count(int32_t* count);
int ppr_comm_unique_id(void* id128);
int ppr_grank_plan_comm_init(ppr_plan* p, const void* id128, int32_t nranks, int32_t rank);
int ppr_grank_plan_shard_bounds(ppr_plan* p, int32_t it, int32_t nranks, int64_t* bounds);
int ppr_grank_plan_run_sharded(ppr_plan* p, uint32_t iterations, double tolerance, ppr_stats* st);
int ppr_grank_plan_exchange_bytes(ppr_plan* p, int64_t* recv_bytes, int64_t* rows_sent);
/* Measurement (no reference counterpart; tools/shard_floor.py): device milliseconds that rank
 * `rank` of a `world`-rank routed run spends in one of its sharded ends, timed on this one plan:
 * what 0 = its final top-K (own rows and the dangling ones; time it after a job), what 1 = its init
 * (own sources and the dangling nodes; rewrites those rows). */
int ppr_grank_plan_ends_time(ppr_plan* p, int32_t world, int32_t rank, int32_t iterations_run, int32_t what,
                             double* ms);
/* Per-kernel roofline of the last ppr_grank_plan_run (no reference counterpart: measurement).
 * Kernel groups, in this order: 0 wave tier (k_merge_lds_x), 1 sieve large (k_sv1 + k_svfin, 16
 * waves), 2 sieve mid (8 waves), 3 sieve small (4 waves), 4 sieve multi-slice (k_svA + k_svB +
 * k_svF), 5 range engines (k_xr + k_xfinal + k_xfin1: sources the sieve does not take or hands
 * back). bytes: SURVEY s8d algorithmic bytes of the sources the group merged (the wave tier's
 * without the written rows; the range group's with rows of min(L, candidates + 1) entries); ms:
 * HIP event time of the group's launches on its stream; launches:
 * event pairs summed. Up to n groups are written. */
int ppr_grank_plan_kernel_stats(ppr_plan* p, int32_t n, double* bytes, double* ms, int64_t* launches);
/* Tests: the same native loop with n plans of this process as the ranks (one thread each, block
 * exchange by device copies instead of RCCL: RCCL refuses two ranks on one GPU). st: n stats or
 * null. Every plan must be built on the same graph and parameters. */
int ppr_grank_plan_run_local_group(ppr_plan** plans, int32_t n, uint32_t iterations, double tolerance,
                                   ppr_stats* st);
/* host-staged variants of pack/unpack (rehearsal without RCCL; synchronous): pack_host writes the
 * block (at most cap bytes) and its size to *bytes; unpack_host takes a block of `bytes` bytes */
int ppr_grank_plan_pack_host(ppr_plan* p, int32_t it, int64_t begin, int64_t end, void* host_buf, int64_t cap,
                             int64_t* bytes);
int ppr_grank_plan_unpack_host(ppr_plan* p, int32_t it, int64_t begin, int64_t end, const void* host_buf,
                               int64_t bytes);

/* Downloads: final top-K (n*K) and the current L-slab (n*L, len per node; each row returned
 * sorted by (score desc, id asc) -- the device keeps rows in key-hash order). */
int ppr_grank_plan_fetch(ppr_plan* p, int32_t* out_ids, double* out_scores, int32_t* out_len);
int ppr_grank_plan_fetch_slab(ppr_plan* p, int32_t iterations_run, int32_t* ids, double* scores,
                              int32_t* len);
/* Rows [begin, end) of the final top-K (ids/scores (end - begin) * K, len end - begin; any may be
 * null), synchronous. With buffers from ppr_host_alloc (page-locked host memory: DMA at link rate
 * instead of a staged copy) the drop-in template downloads chunk by chunk while its threads
 * materialise the chunks already down (include/ppr/grank.h; no reference counterpart). */
int ppr_grank_plan_fetch_rows(ppr_plan* p, int64_t begin, int64_t end, int32_t* ids, double* scores,
                              int32_t* len);
int ppr_host_alloc(int64_t bytes, void** out);
void ppr_host_free(void* ptr);
/* Device stream the plan runs on (hipStream_t as void*), for event timing by the caller. Work the
 * plan puts on its internal side streams (hub bucket stage, wave tiers) is joined back into this
 * stream before each merge returns. */
void* ppr_grank_plan_stream(ppr_plan* p);
/* Raw basket slab slot (n*L ids / scores, n lengths; only the first len[v] entries of a row are
 * meaningful). MC plans: slot 0 = final baskets, slot 1 = random-walk baskets of the walk set. */
int ppr_plan_fetch_slot(ppr_plan* p, int32_t slot, int32_t* ids, double* scores, int32_t* len);

/* ---- MCCompletePathV2 (ppr::mccompletepathv2, include/mccompletepathv2.h:182-258) ----
 * `walks` is the reference's `iterations` (R): floor(R*d) walks per walk-set node. The walks use
 * counter-based Philox4x32-10 keyed by `seed` (the reference seeds a global mt19937 from
 * std::random_device, so runs are only statistically comparable); the combine is deterministic.
 * Results: out_ids / out_scores n*K (rows score desc, id asc, unused id -1), out_len n. */
typedef struct ppr_mc_stats {
  double device_ms;        /* walks + combine + top-K, device events */
  double walk_ms;          /* k_mc_walk */
  double combine_ms;       /* level-synchronous merge kernels */
  int64_t walk_nodes;      /* |W|: nodes whose random-walk basket some predecessor reads */
  int64_t walks;           /* walks run (|W| * floor(R*d)) */
  int64_t levels;          /* combine levels */
  int64_t merge_launches;
  int64_t candidates;      /* combine candidates (PPR_FLAG_STATS) */
  int64_t algo_bytes;      /* combine algorithmic bytes (PPR_FLAG_STATS) */
} ppr_mc_stats;

int ppr_mccp2_csr(const ppr_csr* g, uint32_t K, uint32_t L, uint32_t walks, double damping,
                  uint64_t seed, const ppr_opts* o, int32_t* out_ids, double* out_scores,
                  int32_t* out_len, ppr_mc_stats* st);
/* Plan form: executionOrder, walk set and combine levels are computed once and the graph stays
 * resident. ppr_mccp2_plan_walk runs the walks of walk-set entries [begin, end) (walk-count
 * sharding across GPUs needs no exchange); combine merges level by level and writes the top-K,
 * fetched with ppr_grank_plan_fetch; destroy with ppr_grank_plan_destroy. */
int ppr_mccp2_plan_create(const ppr_csr* g, uint32_t K, uint32_t L, double damping,
                          const ppr_opts* o, ppr_plan** out);
int ppr_mccp2_plan_info(ppr_plan* p, int64_t* walk_nodes, int64_t* levels, int64_t* dangling);
int ppr_mccp2_plan_walk(ppr_plan* p, uint32_t walks, uint64_t seed, int64_t begin, int64_t end);
int ppr_mccp2_plan_combine(ppr_plan* p);
int ppr_mccp2_plan_run(ppr_plan* p, uint32_t walks, uint64_t seed, ppr_mc_stats* st);
/* The whole MC job on several ranks (one process per GPU, after ppr_grank_plan_comm_init on the MC
 * plan): each rank walks an equal contiguous range of the walk set, the walk baskets are
 * all-gathered as compact blocks (exact sizes all-gathered and checked first, then one grouped
 * ncclBroadcast per rank), and every rank runs the level-sequential combine and the top-K. The
 * result equals ppr_mccp2_plan_run with the same seed bit for bit on every rank. st: walk_ms and
 * walks are this rank's share; ppr_grank_plan_exchange_bytes gives the walk-basket bytes it
 * received. (Replaces the single-process sweep of include/mccompletepathv2.h:211-250.) */
int ppr_mccp2_plan_run_sharded(ppr_plan* p, uint32_t walks, uint64_t seed, ppr_mc_stats* st);
/* Tests: the same with n MC plans of this process as the ranks (device copies instead of RCCL). */
int ppr_mccp2_plan_run_local_group(ppr_plan** plans, int32_t n, uint32_t walks, uint64_t seed,
                                   ppr_mc_stats* st);

/* ---- Exact single-source PPR, batched (the reference's quality oracle) -------------------------
 * Replaces ppr::pprInternal::pprSingleSource(graph, iterations, damping, tolerance, source)
 * (include/internal/pprSingleSource.h:28-75) for S sources at once, and the keepTop(K) +
 * score lookups benchmarkAlgorithm does on its result (include/benchmarkAlgorithm.h:91-121).
 * Scores agree with the reference to rounding (the per-node summation order differs). */
typedef struct ppr_exact ppr_exact;
int ppr_exact_create(const ppr_csr* g, const int32_t* sources, int32_t S, double damping,
                     const ppr_opts* o, ppr_exact** out);
/* power iteration of every source until its norm1 step < tolerance or `iterations`;
 * iters_run[S] (optional): iterations each source ran */
int ppr_exact_run(ppr_exact* h, uint32_t iterations, double tolerance, int32_t* iters_run);
/* keepTop(K) of every source's vector (nonzero entries), rows [S][K] by (score desc, id asc) */
int ppr_exact_topk(ppr_exact* h, uint32_t K, int32_t* out_ids, double* out_scores, int32_t* out_len);
/* out[s][q] = score of node keys[s][q] for source s (0 for a node it never reached) */
int ppr_exact_gather(ppr_exact* h, int32_t Q, const int32_t* keys, double* out);
void ppr_exact_destroy(ppr_exact* h);

#ifdef __cplusplus
}
#endif
#endif /* PPR_HIP_H */
