/*
 * oracle/grank_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference's GRank hot path, used as the parity
 * checker for the MI355X HIP path (tests/, __graft_entry__.smoke(), bench.py cpu_baseline only).
 * It is never linked into, called by, or shipped with the product library.
 *
 * Pinned against the compiled reference (oracle/_ref/ref_driver, built from /root/reference by
 * oracle/Makefile) through the golden vectors in tests/golden/ (tests/test_oracle_golden.py):
 * bit-exact where the reference has no top-L truncation (ring G1, RMAT-10 L>=|V| G2, the
 * known-answer graphs), tie-aware statistics elsewhere.
 *
 * Semantics restated (reference file:line):
 *   init         include/grank.h:64-83       B[v] = {v: 1-d}; B[v][s] += d/deg for s in succ(v);
 *                                             keepTop(L)
 *   partitions   include/internal/pprInternal.h:29-99   BFS 2-colouring, roots in graph order,
 *                                             successors then predecessors get the opposite colour
 *   iteration    include/grank.h:90-141      Jacobi sweep over the active partition, then swap
 *   merge        include/grank.h:96-126      acc = {v: 1-d}; for u in succ(v) (CSR order), for
 *                                             (k,s) in B[u]: acc[k] = fma(s, d/deg, acc[k])
 *                                             (-O3 -march=native contracts this into an FMA)
 *   keepTop      include/internal/pprInternal.h:109-137  keep L largest; the reference breaks
 *                                             ties by unordered_map order + nth_element, which
 *                                             differs from row to row; this restatement (and the
 *                                             HIP path) breaks them by a per-source hash of the key
 *                                             (oracle_tie_key) and stores rows by (score desc, id
 *                                             asc)
 *   norm1        include/internal/pprInternal.h:147-165  sum |new-old| over the key union; the
 *                                             summation order here is the HIP kernel's fixed
 *                                             64-lane pattern over rows in their stored (hash)
 *                                             order (norm1_rows, norm1_stored) so maxDiff is
 *                                             bit-identical too
 *   stop rule    include/grank.h:90-94,140   maxDiff[2] = {tol, tol}; loop while
 *                                             i < iterations && max(maxDiff) >= tol
 *   final top-K  include/grank.h:143-147      keepTop(K) of each row by the same rule (row_topk)
 *
 * Summation mode (oracle_set_sum; the HIP plan's PPR_FLAG_CHAIN_SUM):
 *   chain  the reference's own order: acc[k] = fma(s, d/deg, acc[k]) per key in successor order
 *          (include/grank.h:107-116 under -O3 -march=native)
 *   exact  (default) every contribution p = fl(s * d/deg) is added EXACTLY into a 128-bit fixed-point
 *          accumulator X[k] += floor(p * 2^93) (the seed 1-d likewise), and the basket value is
 *          X[k] * 2^-93 rounded to nearest once: order-free (the GPU sums in any order) and at least
 *          as accurate as the chain (each key's sum is correctly rounded from the rounded products;
 *          the 2^-93 truncation is ~1e-28 absolute per term)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int32_t key; double sc; uint32_t tie; } ent_t;

/* output / storage order: (score desc, key asc) */
static int cmp_ent(const void* a, const void* b) {
  const ent_t* x = (const ent_t*)a;
  const ent_t* y = (const ent_t*)b;
  if (x->sc > y->sc) return -1;
  if (x->sc < y->sc) return 1;
  return (x->key < y->key) ? -1 : (x->key > y->key);
}

/* selection order of keepTop (pprInternal.h:109-137), whose ties the reference leaves to each
 * unordered_map's history (so they fall differently in every row): (score desc, tie asc) with
 * tie = mix32(key ^ mix32(source * 0x9e3779b9 + 1)), a per-source bijection of the key -- the HIP
 * path's tie_salt / tie_w (ppr_device.h) */
static uint32_t mix32(uint32_t x);
uint32_t oracle_tie_key(int32_t source, int32_t key) {
  return mix32((uint32_t)key ^ mix32((uint32_t)source * 0x9e3779b9u + 1u));
}
static int cmp_sel(const void* a, const void* b) {
  const ent_t* x = (const ent_t*)a;
  const ent_t* y = (const ent_t*)b;
  if (x->sc > y->sc) return -1;
  if (x->sc < y->sc) return 1;
  return (x->tie < y->tie) ? -1 : (x->tie > y->tie);
}

/* ---- summation mode ---- */
static int g_sum_exact = 1;
void oracle_set_sum(int exact) { g_sum_exact = exact ? 1 : 0; }
int oracle_get_sum(void) { return g_sum_exact; }

#define XS_F 93 /* fixed-point fraction bits (approximated_personalized_pagerank_amd/csrc/merge_xs.h) */
typedef unsigned __int128 xs_t;

/* floor(p * 2^F) of a double p >= 0 (GRank: F = 93, p < 4, every basket sums to <= 1; the MC
 * combine's exact mode: F = 72, mc_oracle.c) */
xs_t oracle_xs_conv_f(double p, int F) {
  uint64_t b;
  memcpy(&b, &p, 8);
  int e = (int)((b >> 52) & 0x7ff);
  uint64_t m = b & ((1ull << 52) - 1);
  if (e) m |= 1ull << 52; else e = 1;
  const int sh = e - 1075 + F;
  if (sh >= 0) return (xs_t)m << sh;
  if (-sh >= 64) return 0;
  return (xs_t)(m >> -sh);
}
static xs_t xs_conv(double p) { return oracle_xs_conv_f(p, XS_F); }

/* X * 2^-F rounded to nearest even (X < 2^95): the top 64 bits with a sticky bit, one correctly
 * rounded u64 -> double conversion, an exact power-of-two scale */
double oracle_xs_to_double_f(uint64_t hi, uint64_t lo, int F) {
  if (hi == 0) return ldexp((double)lo, -F);
  const int n = 64 - __builtin_clzll(hi);
  const uint64_t top = (hi << (64 - n)) | (lo >> n);
  const uint64_t sticky = (lo & ((1ull << n) - 1)) != 0;
  return ldexp((double)(top | sticky), n - F);
}
double oracle_xs_to_double(uint64_t hi, uint64_t lo) { return oracle_xs_to_double_f(hi, lo, XS_F); }
static double xs_to_double(xs_t x) { return oracle_xs_to_double((uint64_t)(x >> 64), (uint64_t)x); }
void oracle_xs_conv(double p, uint64_t* hi, uint64_t* lo) {
  const xs_t x = xs_conv(p);
  *hi = (uint64_t)(x >> 64);
  *lo = (uint64_t)x;
}

/* ---- open-addressing accumulator (keys unique, insertion-order independent) ---- */
typedef struct {
  int64_t cap;
  int32_t* keys;
  double* acc;
  xs_t* x;        /* exact mode: fixed-point sums */
  int64_t used;
  int64_t* slots; /* occupied slot list, for cheap reset */
} acc_t;

static uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

static void acc_init(acc_t* a, int64_t need) {
  int64_t cap = 16;
  while (cap < 2 * need + 2) cap <<= 1;
  if (cap > a->cap) {
    free(a->keys); free(a->acc); free(a->x); free(a->slots);
    a->cap = cap;
    a->keys = (int32_t*)malloc(sizeof(int32_t) * cap);
    a->acc = (double*)malloc(sizeof(double) * cap);
    a->x = (xs_t*)malloc(sizeof(xs_t) * cap);
    a->slots = (int64_t*)malloc(sizeof(int64_t) * cap);
    for (int64_t i = 0; i < cap; i++) a->keys[i] = -1;
    a->used = 0;
  }
}

static void acc_reset(acc_t* a) {
  for (int64_t i = 0; i < a->used; i++) a->keys[a->slots[i]] = -1;
  a->used = 0;
}

static int64_t acc_slot(acc_t* a, int32_t key) {
  uint64_t mask = (uint64_t)a->cap - 1;
  uint64_t h = mix32((uint32_t)key) & mask;
  for (;;) {
    if (a->keys[h] == key) return (int64_t)h;
    if (a->keys[h] == -1) {
      a->keys[h] = key;
      a->acc[h] = 0.0;
      a->x[h] = 0;
      a->slots[a->used++] = (int64_t)h;
      return (int64_t)h;
    }
    h = (h + 1) & mask;
  }
}

/* the source's seed entry {v: val} (include/grank.h:103-104) */
static void acc_seed(acc_t* a, int32_t key, double val) {
  const int64_t h = acc_slot(a, key);
  if (g_sum_exact) a->x[h] = xs_conv(val); else a->acc[h] = val;
}
/* one contribution s of a successor basket to key: acc = fma(s, f, acc) (include/grank.h:114-115),
 * or exactly X += floor(fl(s * f) * 2^93) */
static void acc_add(acc_t* a, int32_t key, double s, double f) {
  const int64_t h = acc_slot(a, key);
  if (g_sum_exact) a->x[h] += xs_conv(s * f); else a->acc[h] = fma(s, f, a->acc[h]);
}
/* init (include/grank.h:73-75): B[v][s] += d/deg, i.e. a contribution 1.0 * f */
static void acc_add_unit(acc_t* a, int32_t key, double f) {
  const int64_t h = acc_slot(a, key);
  if (g_sum_exact) a->x[h] += xs_conv(f); else a->acc[h] = a->acc[h] + f;
}
/* exact mode: the basket values from the fixed-point sums (once per merge, before keepTop) */
static void acc_settle(acc_t* a) {
  if (!g_sum_exact) return;
  for (int64_t i = 0; i < a->used; i++) a->acc[a->slots[i]] = xs_to_double(a->x[a->slots[i]]);
}

static void acc_free(acc_t* a) { free(a->keys); free(a->acc); free(a->x); free(a->slots); memset(a, 0, sizeof(*a)); }

/* keepTop(L) of source v's accumulator: the first L by the selection order, stored by the output
 * order; returns len */
static int32_t acc_top(acc_t* a, int32_t v, int32_t L, ent_t** buf, int64_t* bufcap, int32_t* ids, double* sc) {
  acc_settle(a);
  if (a->used > *bufcap) { free(*buf); *bufcap = a->used; *buf = (ent_t*)malloc(sizeof(ent_t) * (*bufcap)); }
  ent_t* e = *buf;
  for (int64_t i = 0; i < a->used; i++) {
    int64_t s = a->slots[i];
    e[i].key = a->keys[s]; e[i].sc = a->acc[s]; e[i].tie = oracle_tie_key(v, e[i].key);
  }
  int32_t len = a->used < L ? (int32_t)a->used : L;
  if (a->used > L) qsort(e, (size_t)a->used, sizeof(ent_t), cmp_sel);
  qsort(e, (size_t)len, sizeof(ent_t), cmp_ent);
  for (int32_t i = 0; i < len; i++) { ids[i] = e[i].key; sc[i] = e[i].sc; }
  return len;
}

/* final keepTop(K) of a stored row of source v (include/grank.h:143-147): out = the K kept by the
 * selection order, by the output order; returns their count */
static int32_t row_topk(int32_t v, const int32_t* ids, const double* sc, int32_t len, int32_t K,
                        int32_t* out_ids, double* out_sc) {
  ent_t* e = (ent_t*)malloc(sizeof(ent_t) * (size_t)(len + 1));
  for (int32_t i = 0; i < len; i++) { e[i].key = ids[i]; e[i].sc = sc[i]; e[i].tie = oracle_tie_key(v, ids[i]); }
  const int32_t k = len < K ? len : K;
  if (len > K) qsort(e, (size_t)len, sizeof(ent_t), cmp_sel);
  qsort(e, (size_t)k, sizeof(ent_t), cmp_ent);
  for (int32_t j = 0; j < K; j++) { out_ids[j] = j < k ? e[j].key : -1; out_sc[j] = j < k ? e[j].sc : 0.0; }
  free(e);
  return k;
}

/* norm1 with the HIP kernel's fixed summation pattern: 64 lane partials, entry i of the new row
 * goes to lane i%64 (in increasing i), then old entries j absent from the new row go to lane
 * j%64 (in increasing j), then an xor butterfly 32,16,8,4,2,1. */
static double norm1_rows(const int32_t* nid, const double* nsc, int32_t nlen,
                         const int32_t* oid, const double* osc, int32_t olen) {
  double p[64];
  for (int l = 0; l < 64; l++) p[l] = 0.0;
  for (int32_t i = 0; i < nlen; i++) {
    double o = 0.0;
    for (int32_t j = 0; j < olen; j++) if (oid[j] == nid[i]) { o = osc[j]; break; }
    p[i & 63] += fabs(nsc[i] - o);
  }
  for (int32_t j = 0; j < olen; j++) {
    int found = 0;
    for (int32_t i = 0; i < nlen; i++) if (nid[i] == oid[j]) { found = 1; break; }
    if (!found) p[j & 63] += osc[j];
  }
  for (int off = 32; off >= 1; off >>= 1) {
    double q[64];
    for (int l = 0; l < 64; l++) q[l] = p[l] + p[l ^ off];
    memcpy(p, q, sizeof(p));
  }
  return p[0];
}

/* The HIP path stores every basket row in ascending hash_b(key) order (the hub merge reads
 * hash-range segments of rows), and norm1 walks the rows in that stored order: restate it by
 * sorting copies of both rows by hash_b before the fixed lane pattern above. */
static uint32_t hash_b(uint32_t x) { return mix32(x ^ 0x9e3779b9u); }

static int cmp_hash(const void* a, const void* b) {
  const uint32_t x = hash_b((uint32_t)((const ent_t*)a)->key), y = hash_b((uint32_t)((const ent_t*)b)->key);
  return (x > y) - (x < y);
}

static double norm1_stored(const int32_t* nid, const double* nsc, int32_t nlen,
                           const int32_t* oid, const double* osc, int32_t olen) {
  ent_t* e = (ent_t*)malloc(sizeof(ent_t) * (size_t)(nlen + olen + 1));
  int32_t* ni = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nlen + olen + 1));
  double* ns = (double*)malloc(sizeof(double) * (size_t)(nlen + olen + 1));
  for (int32_t i = 0; i < nlen; i++) { e[i].key = nid[i]; e[i].sc = nsc[i]; }
  for (int32_t j = 0; j < olen; j++) { e[nlen + j].key = oid[j]; e[nlen + j].sc = osc[j]; }
  qsort(e, (size_t)nlen, sizeof(ent_t), cmp_hash);
  qsort(e + nlen, (size_t)olen, sizeof(ent_t), cmp_hash);
  for (int32_t i = 0; i < nlen + olen; i++) { ni[i] = e[i].key; ns[i] = e[i].sc; }
  const double d = norm1_rows(ni, ns, nlen, ni + nlen, ns + nlen, olen);
  free(e); free(ni); free(ns);
  return d;
}

/* ---- partitions: include/internal/pprInternal.h:29-99 in dense (graph-iteration) order ---- */
int oracle_find_partitions(int64_t n, const int64_t* rp, const int32_t* col, uint8_t* part) {
  int64_t m = n ? rp[n] : 0;
  int64_t* prp = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
  int32_t* pcol = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m ? m : 1));
  char* vis = (char*)calloc((size_t)(n ? n : 1), 1);
  int32_t* q = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  if (!prp || !pcol || !vis || !q) return -1;
  /* predecessors[s] in the order nodes are iterated (pprInternal.h:38-47) */
  for (int64_t e = 0; e < m; e++) prp[col[e] + 1]++;
  for (int64_t i = 0; i < n; i++) prp[i + 1] += prp[i];
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
  for (int64_t i = 0; i < n; i++) fill[i] = prp[i];
  for (int64_t v = 0; v < n; v++)
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) pcol[fill[col[e]]++] = (int32_t)v;
  free(fill);
  for (int64_t r = 0; r < n; r++) {
    int64_t qh = 0, qt = 0;
    if (!vis[r]) { vis[r] = 1; q[qt++] = (int32_t)r; part[r] = 0; }
    while (qh < qt) {
      int32_t nx = q[qh++];
      uint8_t c = part[nx] == 0 ? 1 : 0; /* pprInternal.h:79-80 */
      for (int64_t e = rp[nx]; e < rp[nx + 1]; e++) {
        int32_t s = col[e];
        if (!vis[s]) { vis[s] = 1; part[s] = c; q[qt++] = s; }
      }
      for (int64_t e = prp[nx]; e < prp[nx + 1]; e++) {
        int32_t s = pcol[e];
        if (!vis[s]) { vis[s] = 1; part[s] = c; q[qt++] = s; }
      }
    }
  }
  free(prp); free(pcol); free(vis); free(q);
  return 0;
}

/* ---- GRank on a fixed-width |V| x L slab ----
 * Inputs: CSR in dense order (successor order preserved), partition bits (0 = first).
 * Outputs (all optional except out_*): final top-K rows, the final L-slab, maxDiff history.
 * Returns 0 on success. */
int oracle_grank(int64_t n, const int64_t* rp, const int32_t* col, const uint8_t* part,
                 int32_t K, int32_t L, int32_t iterations, double damping, double tolerance,
                 int32_t* out_ids, double* out_sc, int32_t* out_len,
                 int32_t* slab_ids, double* slab_sc, int32_t* slab_len,
                 double* maxdiff_hist, int32_t* iters_run) {
  if (K <= 0 || L <= 0 || K > L || iterations < 0 || damping < 0 || damping > 1) return -2;  /* 0 = init only (diagnostics) */
  int32_t* ci = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n * L + 1));
  double* cs = (double*)malloc(sizeof(double) * (size_t)(n * L + 1));
  int32_t* cl = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
  int32_t* ni = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n * L + 1));
  double* ns = (double*)malloc(sizeof(double) * (size_t)(n * L + 1));
  int32_t* nl = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
  if (!ci || !cs || !cl || !ni || !ns || !nl) return -1;
  acc_t a; memset(&a, 0, sizeof(a));
  ent_t* buf = NULL; int64_t bufcap = 0;
  const double self = 1.0 - damping;

  /* init: include/grank.h:64-83 */
  for (int64_t v = 0; v < n; v++) {
    int64_t deg = rp[v + 1] - rp[v];
    double factor = damping / (double)deg;
    acc_init(&a, deg + 1);
    acc_seed(&a, (int32_t)v, self);
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) acc_add_unit(&a, col[e], factor);
    cl[v] = acc_top(&a, (int32_t)v, L, &buf, &bufcap, ci + v * L, cs + v * L);
    acc_reset(&a);
  }

  double md[2] = {tolerance, tolerance};
  int32_t it;
  for (it = 0; it < iterations && (md[0] > md[1] ? md[0] : md[1]) >= tolerance; it++) {
    uint8_t active = (uint8_t)(it & 1); /* partitions.first at even iterations */
    md[0] = 0.0;
    for (int64_t v = 0; v < n; v++) {
      if (part[v] != active) continue;
      int64_t deg = rp[v + 1] - rp[v];
      double factor = damping / (double)deg;
      int64_t cand = 1;
      for (int64_t e = rp[v]; e < rp[v + 1]; e++) cand += cl[col[e]];
      acc_init(&a, cand);
      acc_seed(&a, (int32_t)v, self);
      for (int64_t e = rp[v]; e < rp[v + 1]; e++) {
        int32_t u = col[e];
        const int32_t* ui = ci + (int64_t)u * L;
        const double* us = cs + (int64_t)u * L;
        for (int32_t j = 0; j < cl[u]; j++) acc_add(&a, ui[j], us[j], factor);
      }
      nl[v] = acc_top(&a, (int32_t)v, L, &buf, &bufcap, ni + v * L, ns + v * L);
      acc_reset(&a);
      double d1 = norm1_stored(ni + v * L, ns + v * L, nl[v], ci + v * L, cs + v * L, cl[v]);
      if (d1 > md[0]) md[0] = d1;
    }
    for (int64_t v = 0; v < n; v++) {
      if (part[v] != active) continue;
      memcpy(ci + v * L, ni + v * L, sizeof(int32_t) * (size_t)nl[v]);
      memcpy(cs + v * L, ns + v * L, sizeof(double) * (size_t)nl[v]);
      cl[v] = nl[v];
    }
    if (maxdiff_hist) maxdiff_hist[it] = md[0];
    double t = md[0]; md[0] = md[1]; md[1] = t;
  }
  if (iters_run) *iters_run = it;

  for (int64_t v = 0; v < n; v++)
    out_len[v] = row_topk((int32_t)v, ci + v * L, cs + v * L, cl[v], K, out_ids + v * K, out_sc + v * K);
  if (slab_ids) memcpy(slab_ids, ci, sizeof(int32_t) * (size_t)(n * L));
  if (slab_sc) memcpy(slab_sc, cs, sizeof(double) * (size_t)(n * L));
  if (slab_len) memcpy(slab_len, cl, sizeof(int32_t) * (size_t)n);
  free(ci); free(cs); free(cl); free(ni); free(ns); free(nl); free(buf);
  acc_free(&a);
  return 0;
}

/* ---- stepping interface (tests of the source-sharded driver): the same maths as oracle_grank,
 * split into init + one Jacobi step over an explicit list of sources ---- */
int oracle_init_state(int64_t n, const int64_t* rp, const int32_t* col, int32_t L, double damping,
                      int32_t* ids, double* sc, int32_t* len) {
  acc_t a; memset(&a, 0, sizeof(a));
  ent_t* buf = NULL; int64_t bufcap = 0;
  for (int64_t v = 0; v < n; v++) {
    int64_t deg = rp[v + 1] - rp[v];
    double factor = damping / (double)deg;
    acc_init(&a, deg + 1);
    acc_seed(&a, (int32_t)v, 1.0 - damping);
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) acc_add_unit(&a, col[e], factor);
    len[v] = acc_top(&a, (int32_t)v, L, &buf, &bufcap, ids + v * L, sc + v * L);
    acc_reset(&a);
  }
  free(buf); acc_free(&a);
  return 0;
}

int oracle_step(int64_t n, const int64_t* rp, const int32_t* col, int32_t L, double damping,
                const int32_t* ids, const double* sc, const int32_t* len, const int32_t* list,
                int64_t count, int32_t* nids, double* nsc, int32_t* nlen, double* maxdiff) {
  acc_t a; memset(&a, 0, sizeof(a));
  ent_t* buf = NULL; int64_t bufcap = 0;
  double md = 0.0;
  (void)n;
  for (int64_t q = 0; q < count; q++) {
    int32_t v = list[q];
    int64_t deg = rp[v + 1] - rp[v];
    double factor = damping / (double)deg;
    int64_t cand = 1;
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) cand += len[col[e]];
    acc_init(&a, cand);
    acc_seed(&a, v, 1.0 - damping);
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) {
      int32_t u = col[e];
      for (int32_t j = 0; j < len[u]; j++) acc_add(&a, ids[(int64_t)u * L + j], sc[(int64_t)u * L + j], factor);
    }
    nlen[v] = acc_top(&a, v, L, &buf, &bufcap, nids + (int64_t)v * L, nsc + (int64_t)v * L);
    acc_reset(&a);
    double d1 = norm1_stored(nids + (int64_t)v * L, nsc + (int64_t)v * L, nlen[v], ids + (int64_t)v * L,
                           sc + (int64_t)v * L, len[v]);
    if (d1 > md) md = d1;
  }
  free(buf); acc_free(&a);
  *maxdiff = md;
  return 0;
}

/* oracle_step without the per-source norm1 (the whole-iteration maxDiff comes from
 * oracle_norm1_max): the full-size digests (tools/make_c3_digest.py) run it on chunks of one
 * iteration's sources in parallel host threads -- it keeps no state between calls. */
int oracle_step_rows(const int64_t* rp, const int32_t* col, int32_t L, double damping, const int32_t* ids,
                     const double* sc, const int32_t* len, const int32_t* list, int64_t count, int32_t* nids,
                     double* nsc, int32_t* nlen) {
  acc_t a; memset(&a, 0, sizeof(a));
  ent_t* buf = NULL; int64_t bufcap = 0;
  for (int64_t q = 0; q < count; q++) {
    int32_t v = list[q];
    int64_t deg = rp[v + 1] - rp[v];
    double factor = damping / (double)deg;
    int64_t cand = 1;
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) cand += len[col[e]];
    acc_init(&a, cand);
    acc_seed(&a, v, 1.0 - damping);
    for (int64_t e = rp[v]; e < rp[v + 1]; e++) {
      int32_t u = col[e];
      for (int32_t j = 0; j < len[u]; j++) acc_add(&a, ids[(int64_t)u * L + j], sc[(int64_t)u * L + j], factor);
    }
    nlen[v] = acc_top(&a, v, L, &buf, &bufcap, nids + (int64_t)v * L, nsc + (int64_t)v * L);
    acc_reset(&a);
  }
  free(buf); acc_free(&a);
  return 0;
}

/* final keepTop(K) (include/grank.h:143-147) of the listed rows of a slab, into [n][K] outputs */
int oracle_topk_rows(int32_t L, int32_t K, const int32_t* ids, const double* sc, const int32_t* len,
                     const int32_t* list, int64_t count, int32_t* out_ids, double* out_sc, int32_t* out_len) {
  for (int64_t q = 0; q < count; q++) {
    const int64_t v = list[q];
    out_len[v] = row_topk((int32_t)v, ids + v * L, sc + v * L, len[v], K, out_ids + v * K, out_sc + v * K);
  }
  return 0;
}

/* ---- maxDiff of a whole iteration (the sampled-scale GPU tests): the norm1_stored pattern of
 * every listed source, old row -> new row, in O(L log L) per row: both rows sorted by hash_b (the
 * stored order; hash_b is a bijection, so equal hashes are equal keys) and matched by a merge,
 * then the same 64 lane partials as norm1_rows (new entries by position, then the old entries
 * the new row lacks by position) and the same butterfly. Rows: stride L, first len entries. */
static int cmp_hash_ent(const void* a, const void* b) { return cmp_hash(a, b); }

int oracle_norm1_max(int32_t L, const int32_t* list, int64_t count, const int32_t* o_ids, const double* o_sc,
                     const int32_t* o_len, const int32_t* n_ids, const double* n_sc, const int32_t* n_len,
                     double* out_max) {
  ent_t* ne = (ent_t*)malloc(sizeof(ent_t) * (size_t)(L + 1));
  ent_t* oe = (ent_t*)malloc(sizeof(ent_t) * (size_t)(L + 1));
  uint8_t* hit = (uint8_t*)malloc((size_t)(L + 1));
  if (!ne || !oe || !hit) return -1;
  double md = 0.0;
  for (int64_t q = 0; q < count; q++) {
    const int64_t v = list[q];
    const int32_t nl = n_len[v], ol = o_len[v];
    for (int32_t i = 0; i < nl; i++) { ne[i].key = n_ids[v * L + i]; ne[i].sc = n_sc[v * L + i]; }
    for (int32_t j = 0; j < ol; j++) { oe[j].key = o_ids[v * L + j]; oe[j].sc = o_sc[v * L + j]; hit[j] = 0; }
    qsort(ne, (size_t)nl, sizeof(ent_t), cmp_hash_ent);
    qsort(oe, (size_t)ol, sizeof(ent_t), cmp_hash_ent);
    double p[64];
    for (int l = 0; l < 64; l++) p[l] = 0.0;
    int32_t j = 0;
    for (int32_t i = 0; i < nl; i++) {
      const uint32_t hn = hash_b((uint32_t)ne[i].key);
      while (j < ol && hash_b((uint32_t)oe[j].key) < hn) j++;
      double o = 0.0;
      if (j < ol && oe[j].key == ne[i].key) { o = oe[j].sc; hit[j] = 1; }
      p[i & 63] += fabs(ne[i].sc - o);
    }
    for (int32_t k = 0; k < ol; k++)
      if (!hit[k]) p[k & 63] += oe[k].sc;
    for (int off = 32; off >= 1; off >>= 1) {
      double t[64];
      for (int l = 0; l < 64; l++) t[l] = p[l] + p[l ^ off];
      memcpy(p, t, sizeof(p));
    }
    if (p[0] > md) md = p[0];
  }
  free(ne); free(oe); free(hit);
  *out_max = md;
  return 0;
}
