/*
 * oracle/mc_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, single-threaded restatement of the reference's MCCompletePathV2 path, used as the
 * parity checker for the HIP path (tests/, __graft_entry__.smoke() only); never linked into the
 * product library.
 *
 * Semantics restated (reference include/mccompletepathv2.h):
 *   executionOrder :36-113  records (node, indegree, outdegree) in graph order, sorted by
 *                           (indegree desc, outdegree asc) with libstdc++'s std::sort (an
 *                           introsort: median-of-3 pivot, unguarded partition, heapsort past
 *                           2*floor(log2 n) levels, insertion sort below 16 elements), restated
 *                           below step for step so ties land where the reference puts them;
 *                           then the predecessor-release BFS.
 *   mccompletepathv2 :182-258  nodes in that order; map = {v: 1/f} (f = d/deg, 1 for dangling);
 *                           for s in succ(v): map += (final basket of s if s came earlier, else
 *                           the walk basket of s, computed once); keepTop(L); map *= f; finally
 *                           keepTop(K) of the scaled map. keepTop ties: (score desc, dense id
 *                           asc) (the reference leaves ties to unordered_map order).
 *   walkNode :115-165       {u: R}; floor(R*d) walks; a walk moves while the current node has
 *                           successors, counts the reached node if present or fewer than L keys
 *                           are held, continues while U <= d; counts / R. Dangling: {u: 1.0}.
 *   RNG :32-34, :149        NOT restatable (std::random_device seed; a process-global
 *                           round-robin successor index per node, shared by all walks of all
 *                           sources in sequence). Replaced by the engine's definition: per
 *                           source, nodes held in res keep their own round-robin index (start
 *                           offset from a hash of (seed, source, node)), other nodes take
 *                           floor(x0 * deg / 2^32) from Philox4x32-10 keyed by the seed with
 *                           counter (step, walk lo, walk hi, source); a walk continues while
 *                           ((x2:x3) >> 11) * 2^-53 <= d, at most 2^14 steps. The round-robin
 *                           part is what keeps the estimator's variance at the reference's
 *                           level (top-K Jaccard vs exact PPR: iid picks lose ~3 points).
 *                           "First come" follows the kernel's schedule (walk_node below).
 * Parity of the walks against the reference is therefore statistical (tests/test_mc_*.py);
 * executionOrder and the combine are exact.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MC_MAX_STEPS (1 << 14)

/* ---------------------------------------------------------------------------------------------
 * executionOrder */
typedef struct { int32_t node; int64_t in, out; } rec_t;

static int rless(const rec_t* a, const rec_t* b) {  /* the reference's comparator (:57-62) */
  return a->in > b->in ? 1 : (a->in == b->in ? a->out < b->out : 0);
}
static void rswap(rec_t* a, rec_t* b) { rec_t t = *a; *a = *b; *b = t; }

static void push_heap_(rec_t* f, int64_t hole, int64_t top, rec_t val) {
  int64_t parent = (hole - 1) / 2;
  while (hole > top && rless(&f[parent], &val)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = val;
}
static void adjust_heap_(rec_t* f, int64_t hole, int64_t len, rec_t val) {
  const int64_t top = hole;
  int64_t child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (rless(&f[child], &f[child - 1])) child--;
    f[hole] = f[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    f[hole] = f[child - 1];
    hole = child - 1;
  }
  push_heap_(f, hole, top, val);
}
static void heap_sort_(rec_t* f, int64_t len) {
  if (len >= 2) {  /* make_heap */
    for (int64_t parent = (len - 2) / 2;; parent--) {
      adjust_heap_(f, parent, len, f[parent]);
      if (parent == 0) break;
    }
  }
  for (int64_t last = len - 1; last > 0; last--) {  /* sort_heap: pop_heap(first, last, last) */
    rec_t v = f[last];
    f[last] = f[0];
    adjust_heap_(f, 0, last, v);
  }
}
static void median_to_first_(rec_t* r, rec_t* a, rec_t* b, rec_t* c) {
  if (rless(a, b)) {
    if (rless(b, c)) rswap(r, b);
    else if (rless(a, c)) rswap(r, c);
    else rswap(r, a);
  } else if (rless(a, c)) rswap(r, a);
  else if (rless(b, c)) rswap(r, c);
  else rswap(r, b);
}
static rec_t* unguarded_partition_(rec_t* first, rec_t* last, rec_t* pivot) {
  for (;;) {
    while (rless(first, pivot)) first++;
    last--;
    while (rless(pivot, last)) last--;
    if (!(first < last)) return first;
    rswap(first, last);
    first++;
  }
}
static void introsort_loop_(rec_t* first, rec_t* last, int64_t depth) {
  while (last - first > 16) {
    if (depth == 0) { heap_sort_(first, last - first); return; }
    depth--;
    rec_t* mid = first + (last - first) / 2;
    median_to_first_(first, first + 1, mid, last - 1);
    rec_t* cut = unguarded_partition_(first + 1, last, first);
    introsort_loop_(cut, last, depth);
    last = cut;
  }
}
static void linear_insert_(rec_t* last) {
  rec_t val = *last;
  rec_t* next = last - 1;
  while (rless(&val, next)) { *last = *next; last = next; next--; }
  *last = val;
}
static void insertion_sort_(rec_t* first, rec_t* last) {
  if (first == last) return;
  for (rec_t* i = first + 1; i != last; i++) {
    if (rless(i, first)) {
      rec_t val = *i;
      memmove(first + 1, first, (size_t)(i - first) * sizeof(rec_t));
      *first = val;
    } else {
      linear_insert_(i);
    }
  }
}
static void std_sort_(rec_t* first, rec_t* last) {
  const int64_t n = last - first;
  if (n == 0) return;
  int lg = 63 - __builtin_clzll((unsigned long long)n);
  introsort_loop_(first, last, 2 * (int64_t)lg);
  if (n > 16) {
    insertion_sort_(first, first + 16);
    for (rec_t* i = first + 16; i != last; i++) linear_insert_(i);
  } else {
    insertion_sort_(first, last);
  }
}

int oracle_execution_order(int64_t n, const int64_t* rp, const int32_t* col, int32_t* order) {
  if (n == 0) return 0;
  const int64_t m = rp[n];
  int64_t* prp = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
  int32_t* pcol = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  rec_t* recs = (rec_t*)malloc(sizeof(rec_t) * (size_t)n);
  int64_t* wait = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  uint8_t* vis = (uint8_t*)calloc((size_t)n, 1);
  int32_t* q = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  /* predecessors in graph order, one entry per edge (:40-50) */
  for (int64_t e = 0; e < m; e++) prp[col[e] + 1]++;
  for (int64_t i = 0; i < n; i++) prp[i + 1] += prp[i];
  for (int64_t i = 0; i < n; i++) fill[i] = prp[i];
  for (int64_t v = 0; v < n; v++)
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) pcol[fill[col[e]]++] = (int32_t)v;
  for (int64_t i = 0; i < n; i++) {
    recs[i].node = (int32_t)i;
    recs[i].in = prp[i + 1] - prp[i];
    recs[i].out = rp[i + 1] - rp[i];
    wait[i] = rp[i + 1] - rp[i];
  }
  std_sort_(recs, recs + n);
  int64_t out = 0;
  for (int64_t i = 0; i < n; i++) {  /* predecessor-release BFS (:81-111) */
    const int32_t node = recs[i].node;
    if (vis[node]) continue;
    int64_t qh = 0, qt = 0;
    q[qt++] = node;
    while (qh < qt) {
      const int32_t x = q[qh++];
      order[out++] = x;
      vis[x] = 1;
      for (int64_t e = prp[x]; e < prp[x + 1]; e++) {
        const int32_t p = pcol[e];
        if (wait[p]-- > 0 && wait[p] == 0 && !vis[p]) q[qt++] = p;
      }
    }
  }
  free(prp); free(pcol); free(fill); free(recs); free(wait); free(vis); free(q);
  return out == n ? 0 : -1;
}

/* ---------------------------------------------------------------------------------------------
 * walks */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* round-robin start of node x in the walks of src: a fixed pseudo-random offset in [0, deg) */
static uint32_t rr_offset(uint64_t seed, int32_t src, int32_t x, int64_t deg) {
  const uint32_t h = (uint32_t)(mix64(seed ^ ((uint64_t)(uint32_t)src << 32) ^ (uint64_t)(uint32_t)x) >> 32);
  return (uint32_t)(((uint64_t)h * (uint64_t)deg) >> 32);
}

#define MC_LANES 64

/* walkNode of `src` into (ids, sc) (admission order); returns the basket size.
 * Restates the HIP kernel's schedule (merge_mc.h:k_mc_walk): 64 walk slots advance in lockstep
 * rounds; a free slot takes the next walk index (slot order) at the start of a round; in the
 * step phase every live slot moves one edge (slot order): from a node held in res it takes the
 * node's next round-robin successor (offset rr_offset, the reference's per-node index :149),
 * elsewhere a Philox pick; in the apply phase the reached nodes are counted in slot order, a new
 * key entering while res holds < L keys (:152-153).
 * cnt/adm/rr are n-sized scratch, zero on entry and left zero. */
static int walk_node(int64_t n, const int64_t* rp, const int32_t* col, int32_t src, int32_t L,
                     uint32_t R, double d, uint64_t seed, double* cnt, uint8_t* adm, uint32_t* rr,
                     int32_t* ids, double* sc) {
  (void)n;
  if (rp[src + 1] == rp[src]) { ids[0] = src; sc[0] = 1.0; return 1; }
  int size = 0;
  ids[size++] = src;
  adm[src] = 1;
  rr[src] = 0;
  cnt[src] = (double)R;                               /* res[node] = walks (:124) */
  const uint64_t nw = (uint64_t)((double)R * d);      /* (:132) */
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  int alive[MC_LANES] = {0}, jj[MC_LANES] = {0};
  int32_t cur[MC_LANES] = {0}, vis[MC_LANES];
  uint64_t wi[MC_LANES] = {0};
  uint64_t next = 0;
  for (;;) {
    int any = 0;
    for (int l = 0; l < MC_LANES; l++) {
      if (!alive[l] && next < nw) { alive[l] = 1; wi[l] = next++; cur[l] = src; jj[l] = 0; }
      any |= alive[l];
    }
    if (!any) break;
    for (int l = 0; l < MC_LANES; l++) {              /* step phase */
      vis[l] = -1;
      if (!alive[l]) continue;
      const int32_t x = cur[l];
      const int64_t deg = rp[x + 1] - rp[x];
      if (deg == 0) { alive[l] = 0; continue; }      /* (:144-145) */
      uint32_t c[4] = {(uint32_t)jj[l], (uint32_t)wi[l], (uint32_t)(wi[l] >> 32), (uint32_t)src};
      philox4x32_10(c, k0, k1);
      uint64_t pick;
      if (adm[x]) {
        const uint32_t k = rr[x]++;
        pick = ((uint64_t)rr_offset(seed, src, x, deg) + (uint64_t)k % (uint64_t)deg) % (uint64_t)deg;
      } else {
        pick = ((uint64_t)c[0] * (uint64_t)deg) >> 32;
      }
      cur[l] = col[rp[x] + (int64_t)pick];
      vis[l] = cur[l];
      jj[l]++;
      const double u = (double)((((uint64_t)c[2] << 32) | c[3]) >> 11) * 0x1.0p-53;
      if (!(u <= d) || jj[l] >= MC_MAX_STEPS) alive[l] = 0;  /* (:155) */
    }
    for (int l = 0; l < MC_LANES; l++) {              /* apply phase */
      const int32_t y = vis[l];
      if (y < 0) continue;
      if (adm[y]) cnt[y] += 1.0;
      else if (size < L) { adm[y] = 1; rr[y] = 0; cnt[y] = 1.0; ids[size++] = y; }
    }
  }
  for (int t = 0; t < size; t++) {
    sc[t] = cnt[ids[t]] / (double)R;                  /* (:159-160) */
    cnt[ids[t]] = 0.0;
    adm[ids[t]] = 0;
    rr[ids[t]] = 0;
  }
  return size;
}

/* ---- summation mode of the combine (oracle_set_mc_sum; the HIP plan's PPR_MC_SUM): chain = the
 * reference's in-order `map[k] += x` (include/mccompletepathv2.h:240-241); exact = every term (and
 * the seed 1/f) converted exactly to floor(x * 2^72) and summed in 128-bit integers, the total
 * rounded once (grank_oracle.c's exact sum with 72 fraction bits: MC totals reach deg / d) */
typedef unsigned __int128 xs_t;
xs_t oracle_xs_conv_f(double p, int F);
double oracle_xs_to_double_f(uint64_t hi, uint64_t lo, int F);
#define XS_F_MC 72 /* approximated_personalized_pagerank_amd/csrc/merge_xs.h XS_F_MC */
static int g_mc_exact = 0;
void oracle_set_mc_sum(int exact) { g_mc_exact = exact ? 1 : 0; }
int oracle_get_mc_sum(void) { return g_mc_exact; }
static double mc_value(xs_t x) { return oracle_xs_to_double_f((uint64_t)(x >> 64), (uint64_t)x, XS_F_MC); }

typedef struct { int32_t key; double sc; uint32_t tie; } ment_t;
/* output order: (score desc, key asc) */
static int cmp_ment(const void* a, const void* b) {
  const ment_t* x = (const ment_t*)a;
  const ment_t* y = (const ment_t*)b;
  if (x->sc > y->sc) return -1;
  if (x->sc < y->sc) return 1;
  return (x->key < y->key) ? -1 : (x->key > y->key);
}
/* keepTop selection order: (score desc, per-source tie key asc), as in GRank (grank_oracle.c) */
uint32_t oracle_tie_key(int32_t source, int32_t key);
static int cmp_msel(const void* a, const void* b) {
  const ment_t* x = (const ment_t*)a;
  const ment_t* y = (const ment_t*)b;
  if (x->sc > y->sc) return -1;
  if (x->sc < y->sc) return 1;
  return (x->tie < y->tie) ? -1 : (x->tie > y->tie);
}
/* keep the top `keep` of ent[0..U) of source v by the selection order, then order them for output */
static void mkeep(ment_t* ent, int64_t U, int64_t keep, int32_t v) {
  if (U > keep) {
    for (int64_t t = 0; t < U; t++) ent[t].tie = oracle_tie_key(v, ent[t].key);
    qsort(ent, (size_t)U, sizeof(ment_t), cmp_msel);
  }
  qsort(ent, (size_t)keep, sizeof(ment_t), cmp_ment);
}

/* Whole MCCompletePathV2. out_* n*K / n; walk_* (optional) n*L / n: walk basket of every node
 * of the walk set (len 0 elsewhere), rows in admission order. */
int oracle_mccp2(int64_t n, const int64_t* rp, const int32_t* col, int32_t K, int32_t L, uint32_t R,
                 double d, uint64_t seed, int32_t* out_ids, double* out_sc, int32_t* out_len,
                 int32_t* walk_ids, double* walk_sc, int32_t* walk_len) {
  if (n == 0) return 0;
  int32_t* order = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  if (oracle_execution_order(n, rp, col, order)) { free(order); return -1; }
  int32_t* pos = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  for (int64_t i = 0; i < n; i++) pos[order[i]] = (int32_t)i;
  int32_t* fid = (int32_t*)malloc(sizeof(int32_t) * (size_t)n * L);
  double* fsc = (double*)malloc(sizeof(double) * (size_t)n * L);
  int32_t* flen = (int32_t*)calloc((size_t)n, sizeof(int32_t));
  int32_t* wid = (int32_t*)malloc(sizeof(int32_t) * (size_t)n * L);
  double* wsc = (double*)malloc(sizeof(double) * (size_t)n * L);
  int32_t* wlen = (int32_t*)calloc((size_t)n, sizeof(int32_t));
  uint8_t* haswalk = (uint8_t*)calloc((size_t)n, 1);
  double* cnt = (double*)calloc((size_t)n, sizeof(double));
  uint8_t* adm = (uint8_t*)calloc((size_t)n, 1);
  uint32_t* rrc = (uint32_t*)calloc((size_t)n, sizeof(uint32_t));
  double* acc = (double*)calloc((size_t)n, sizeof(double));
  xs_t* xacc = g_mc_exact ? (xs_t*)calloc((size_t)n, sizeof(xs_t)) : NULL;
  uint8_t* touched = (uint8_t*)calloc((size_t)n, 1);
  ment_t* ent = (ment_t*)malloc(sizeof(ment_t) * (size_t)n);
  for (int64_t i = 0; i < n; i++) {
    const int32_t v = order[i];
    const int64_t deg = rp[v + 1] - rp[v];
    if (deg == 0) { fid[(int64_t)v * L] = v; fsc[(int64_t)v * L] = 1.0; flen[v] = 1; continue; }
    const double f = d / (double)deg;
    int64_t U = 0;
    ent[U++].key = v;
    touched[v] = 1;
    acc[v] = 1.0 / f;                                  /* (:226) */
    if (xacc) xacc[v] = oracle_xs_conv_f(1.0 / f, XS_F_MC);
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) {
      const int32_t s = col[e];
      const int32_t* rk;
      const double* rs;
      int32_t rl;
      if (pos[s] < pos[v]) {
        rk = fid + (int64_t)s * L; rs = fsc + (int64_t)s * L; rl = flen[s];
      } else {
        if (!haswalk[s]) {                            /* (:235-239) */
          wlen[s] = walk_node(n, rp, col, s, L, R, d, seed, cnt, adm, rrc, wid + (int64_t)s * L,
                              wsc + (int64_t)s * L);
          haswalk[s] = 1;
        }
        rk = wid + (int64_t)s * L; rs = wsc + (int64_t)s * L; rl = wlen[s];
      }
      for (int32_t t = 0; t < rl; t++) {              /* map[k] += x (:240-241) */
        const int32_t k = rk[t];
        if (!touched[k]) { touched[k] = 1; acc[k] = 0.0; if (xacc) xacc[k] = 0; ent[U++].key = k; }
        if (xacc) xacc[k] += oracle_xs_conv_f(rs[t], XS_F_MC);
        else acc[k] = acc[k] + rs[t];
      }
    }
    for (int64_t t = 0; t < U; t++) {
      ent[t].sc = xacc ? mc_value(xacc[ent[t].key]) : acc[ent[t].key];
      touched[ent[t].key] = 0;
    }
    const int64_t keep = U < L ? U : L;
    mkeep(ent, U, keep, v);                            /* keepTop(L) (:243) */
    for (int64_t t = 0; t < keep; t++) {              /* *= factor (:246-247) */
      fid[(int64_t)v * L + t] = ent[t].key;
      fsc[(int64_t)v * L + t] = ent[t].sc * f;
    }
    flen[v] = (int32_t)keep;
  }
  for (int64_t v = 0; v < n; v++) {                   /* keepTop(K) (:252-256) on the scaled map */
    const int32_t k = flen[v] < K ? flen[v] : K;
    for (int32_t t = 0; t < flen[v]; t++) { ent[t].key = fid[v * L + t]; ent[t].sc = fsc[v * L + t]; }
    mkeep(ent, flen[v], k, (int32_t)v);                /* scaling can tie two scores */
    for (int32_t t = 0; t < K; t++) {
      out_ids[v * K + t] = t < k ? ent[t].key : -1;
      out_sc[v * K + t] = t < k ? ent[t].sc : 0.0;
    }
    out_len[v] = k;
  }
  if (walk_len) {
    for (int64_t v = 0; v < n; v++) {
      walk_len[v] = haswalk[v] ? wlen[v] : 0;
      for (int32_t t = 0; t < L; t++) {
        const int ok = haswalk[v] && t < wlen[v];
        walk_ids[v * L + t] = ok ? wid[v * L + t] : -1;
        walk_sc[v * L + t] = ok ? wsc[v * L + t] : 0.0;
      }
    }
  }
  free(order); free(pos); free(fid); free(fsc); free(flen); free(wid); free(wsc); free(wlen);
  free(haswalk); free(cnt); free(adm); free(rrc); free(acc); free(touched); free(ent);
  free(xacc);
  return 0;
}

/* ---- one combine step of MCCompletePathV2 for listed sources (the sampled RMAT-22 GPU test):
 * for v, succ s contributes its final basket (f_*) when pos[s] < pos[v], else its walk basket
 * (w_*), exactly as oracle_mccp2's sweep does (include/mccompletepathv2.h:211-249):
 * map = {v: 1/f}; map[k] += x over successors in CSR order; keepTop(L); *= f. Output rows
 * (stride L) by (scaled score desc, key asc). */
int oracle_mc_combine(int64_t n, const int64_t* rp, const int32_t* col, const int32_t* pos, int32_t L, double d,
                      const int32_t* f_ids, const double* f_sc, const int32_t* f_len,
                      const int32_t* w_ids, const double* w_sc, const int32_t* w_len,
                      const int32_t* list, int64_t count, int32_t* out_ids, double* out_sc, int32_t* out_len) {
  double* acc = (double*)calloc((size_t)n, sizeof(double));
  xs_t* xacc = g_mc_exact ? (xs_t*)calloc((size_t)n, sizeof(xs_t)) : NULL;
  uint8_t* touched = (uint8_t*)calloc((size_t)n, 1);
  int64_t cap = 16;
  ment_t* ent = (ment_t*)malloc(sizeof(ment_t) * (size_t)cap);
  if (!acc || !touched || !ent) return -1;
  for (int64_t q = 0; q < count; q++) {
    const int32_t v = list[q];
    const int64_t deg = rp[v + 1] - rp[v];
    if (deg == 0) { out_ids[q * L] = v; out_sc[q * L] = 1.0; out_len[q] = 1; continue; }
    const double f = d / (double)deg;
    int64_t need = 1;
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) need += pos[col[e]] < pos[v] ? f_len[col[e]] : w_len[col[e]];
    if (need > cap) { free(ent); cap = need; ent = (ment_t*)malloc(sizeof(ment_t) * (size_t)cap); if (!ent) return -1; }
    int64_t U = 0;
    ent[U++].key = v;
    touched[v] = 1;
    acc[v] = 1.0 / f;
    if (xacc) xacc[v] = oracle_xs_conv_f(1.0 / f, XS_F_MC);
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) {
      const int32_t s = col[e];
      const int fin = pos[s] < pos[v];
      const int32_t* rk = (fin ? f_ids : w_ids) + (int64_t)s * L;
      const double* rs = (fin ? f_sc : w_sc) + (int64_t)s * L;
      const int32_t rl = fin ? f_len[s] : w_len[s];
      for (int32_t t = 0; t < rl; t++) {
        const int32_t k = rk[t];
        if (!touched[k]) { touched[k] = 1; acc[k] = 0.0; if (xacc) xacc[k] = 0; ent[U++].key = k; }
        if (xacc) xacc[k] += oracle_xs_conv_f(rs[t], XS_F_MC);
        else acc[k] = acc[k] + rs[t];
      }
    }
    for (int64_t t = 0; t < U; t++) {
      ent[t].sc = xacc ? mc_value(xacc[ent[t].key]) : acc[ent[t].key];
      touched[ent[t].key] = 0;
    }
    const int64_t keep = U < L ? U : L;
    mkeep(ent, U, keep, v);
    for (int64_t t = 0; t < keep; t++) { ent[t].sc = ent[t].sc * f; }
    qsort(ent, (size_t)keep, sizeof(ment_t), cmp_ment);  /* scaling can tie two scores */
    for (int32_t t = 0; t < L; t++) {
      out_ids[q * L + t] = t < keep ? ent[t].key : -1;
      out_sc[q * L + t] = t < keep ? ent[t].sc : 0.0;
    }
    out_len[q] = (int32_t)keep;
  }
  free(acc); free(touched); free(ent); free(xacc);
  return 0;
}
