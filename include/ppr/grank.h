// ppr/grank.h -- drop-in replacement for the reference's ppr::grank (include/grank.h:42-48,
// header-only/grank.h:214-220), running on an MI355X through libppr_hip.so (include/ppr_hip.h).
//
// Same template, same signature, same parameter checks with the same messages and
// exit(EXIT_FAILURE) (include/grank.h:51-55), same result shape. Link with -lppr_hip.
//
// What happens per call (DESIGN.md "boundary"):
//   1. dense ids = the graph's iteration order, CSR keeps every successor vector's order
//      (the reference's partitions and summation order depend on both);
//   2. ppr_grank_plan_create/run (ppr_grank_csr's steps): BFS partitions
//      (include/internal/pprInternal.h:29-99), upload, init, iterations, final top-K on the device;
//   3. the top-K rows come down in chunks while the host threads materialise them back into
//      unordered_map<Key, unordered_map<Key,double>> (download_materialize).
// Results vs the reference (INTEGRATION.md "Numerical contract"):
//   default (exact sum)  every score within 1e-12 relative of the reference's: each basket value is
//                        the exact sum of the rounded products, rounded once (the reference rounds
//                        after every add of its fma chain, include/grank.h:114-115)
//   PPR_SUM=chain        the reference's in-order fma chain: bit-identical scores wherever the
//                        reference never cuts a basket at a tie
// Which keys survive among those tied at a top-L/top-K cut: a per-source hash of the key (the
// reference leaves it to its hash-map history).
// Limits (INTEGRATION.md "Limits"): L <= 4096 and deg(v) * L + 1 < 2^31 for every node; beyond
// them the call prints "parameter outside the supported range" and exits (PPR_ERR_RANGE).
#ifndef PPR_HIP_DROPIN_GRANK_H
#define PPR_HIP_DROPIN_GRANK_H

#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <iostream>
#include <memory>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../ppr_hip.h"

#if defined(__GLIBC__)
#include <malloc.h>
#endif

namespace ppr {
namespace hipdetail {

// While the result maps are built (~130 M node allocations at RMAT-22, from every host thread),
// glibc grows each thread's malloc heap M_TOP_PAD bytes at a time (default 128 KB). Every growth
// step is an mprotect that takes the process's mmap lock exclusively against the other threads'
// page faults; with the default step the fill ran 3-5x slower (8 threads: 6-10 s vs 1.8-2.5 s at
// 64 MB). mallopt is process-wide, so this is OPT-IN: PPR_HEAP_PAD=<MB> sets M_TOP_PAD for the
// duration of the calls that are materialising results; the last of several concurrent calls to
// finish sets it back to MALLOC_TOP_PAD_ (else glibc's 128 KB) -- glibc has no getter for a value
// the application may have set itself, so an application that sets M_TOP_PAD should leave
// PPR_HEAP_PAD unset (INTEGRATION.md "Process-wide side effects").
struct HeapGrowth {
#if defined(__GLIBC__)
  static std::atomic<int>& active() {
    static std::atomic<int> n(0);
    return n;
  }
  bool on = false;
  HeapGrowth() {
    const char* e = getenv("PPR_HEAP_PAD");
    const int mb = e && *e ? atoi(e) : 0;
    if (mb <= 0) return;
    on = true;
    active().fetch_add(1);
    mallopt(M_TOP_PAD, (mb > 1024 ? 1024 : mb) << 20);
  }
  ~HeapGrowth() {
    if (!on || active().fetch_sub(1) != 1) return;
    const char* e = getenv("MALLOC_TOP_PAD_");
    mallopt(M_TOP_PAD, e && *e ? atoi(e) : 128 * 1024);
  }
#endif
};

// host threads of one call: the caller's count (ppr::grankMulti's nThreads), else PPR_HOST_THREADS,
// else OMP_NUM_THREADS (set to the CPU share on shared hosts, where hardware_concurrency() reports
// every CPU of the machine), else hardware_concurrency()
inline size_t host_threads(size_t requested = 0) {
  if (requested > 0) return requested;
  const char* e = getenv("PPR_HOST_THREADS");
  if (!e || !*e) e = getenv("OMP_NUM_THREADS");
  if (e && *e && atoi(e) > 0) return (size_t)atoi(e);
  return std::max<size_t>(1, std::thread::hardware_concurrency());
}

// run f(begin, end) over [0, n) on up to nt host threads (the map <-> CSR conversions dominate
// end-to-end time once the device phase takes seconds)
template <class F>
inline void parallel_ranges(size_t n, size_t nt, F f) {
  nt = std::min<size_t>(std::max<size_t>(1, nt), std::max<size_t>(1, n / 4096));
  if (nt <= 1) { f((size_t)0, n); return; }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (size_t t = 0; t < nt; t++) th.emplace_back(f, n * t / nt, n * (t + 1) / nt);
  for (auto& x : th) x.join();
}

template <typename Key>
struct Flat {
  std::vector<const Key*> keys;  // dense id -> key (points into the caller's graph)
  std::vector<int64_t> rp;
  std::vector<int32_t> col;
};

// key -> dense id: open addressing over a mix of std::hash<Key>, filled by all host threads at
// once (slots claimed by CAS; the graph's keys are unique) -- a serial unordered_map of 4 M keys
// took most of flatten's time. Small trivially copyable keys (integers) are compared against a
// dense copy instead of through the pointer into the caller's map node (a cache miss per lookup).
template <typename Key, bool Copy = std::is_trivially_copyable<Key>::value && (sizeof(Key) <= 8)>
struct KeyStore {  // (generic keys: through the pointer)
  const std::vector<const Key*>* keys = nullptr;
  void build(const std::vector<const Key*>& k, size_t) { keys = &k; }
  const Key& at(size_t i) const { return *(*keys)[i]; }
};
template <typename Key>
struct KeyStore<Key, true> {
  std::vector<Key> copy;
  void build(const std::vector<const Key*>& k, size_t nt) {
    copy.resize(k.size());
    parallel_ranges(k.size(), nt, [&](size_t b, size_t e) {
      for (size_t i = b; i < e; i++) copy[i] = *k[i];
    });
  }
  const Key& at(size_t i) const { return copy[i]; }
};

template <typename Key>
struct KeyIndex {
  std::unique_ptr<std::atomic<int32_t>[]> slot;
  uint64_t mask = 0;
  KeyStore<Key> ks;
  // integer keys of <= 32 bits in a dense range (span <= 4 n + 1024: ids, as in the reference's
  // examples and RMAT graphs): a direct key -> id array instead of the hash, one memory access per
  // lookup (the flatten's successor lookups were two cache misses each: slot, then the key copy)
  std::vector<int32_t> direct;
  int64_t lo = 0;
  template <typename K = Key>
  typename std::enable_if<std::is_integral<K>::value && sizeof(K) <= 4, bool>::type build_direct(
      const std::vector<const Key*>& k, size_t nt) {
    if (k.empty()) return false;
    nt = std::max<size_t>(1, std::min(nt, k.size() / 4096));  // (no thread per 10 keys on tiny graphs)
    std::vector<int64_t> mn(nt, INT64_MAX), mx(nt, INT64_MIN);
    std::vector<size_t> part(nt + 1);
    for (size_t t = 0; t <= nt; t++) part[t] = k.size() * t / nt;
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; t++)
      th.emplace_back([&, t] {
        for (size_t i = part[t]; i < part[t + 1]; i++) {
          const int64_t x = (int64_t)*k[i];
          mn[t] = std::min(mn[t], x);
          mx[t] = std::max(mx[t], x);
        }
      });
    for (auto& x : th) x.join();
    const int64_t a = *std::min_element(mn.begin(), mn.end()), b = *std::max_element(mx.begin(), mx.end());
    if (b - a > 4 * (int64_t)k.size() + 1024) return false;
    lo = a;
    direct.resize((size_t)(b - a + 1));
    parallel_ranges(direct.size(), nt, [&](size_t x0, size_t x1) {
      for (size_t i = x0; i < x1; i++) direct[i] = -1;
    });
    parallel_ranges(k.size(), nt, [&](size_t x0, size_t x1) {
      for (size_t v = x0; v < x1; v++) direct[(size_t)((int64_t)*k[v] - lo)] = (int32_t)v;
    });
    return true;
  }
  template <typename K = Key>
  typename std::enable_if<!(std::is_integral<K>::value && sizeof(K) <= 4), bool>::type build_direct(
      const std::vector<const Key*>&, size_t) {
    return false;
  }
  static uint64_t mix(uint64_t x) {  // splitmix64 finaliser: std::hash of integers is the identity
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL; x ^= x >> 27; x *= 0x94d049bb133111ebULL; x ^= x >> 31;
    return x;
  }
  void build(const std::vector<const Key*>& k, size_t nt) {
    if (build_direct(k, nt)) return;
    ks.build(k, nt);
    uint64_t cap = 16;
    while (cap < 2 * (uint64_t)k.size()) cap <<= 1;
    mask = cap - 1;
    slot.reset(new std::atomic<int32_t>[cap]);
    parallel_ranges((size_t)cap, nt, [&](size_t b, size_t e) {
      for (size_t i = b; i < e; i++) slot[i].store(-1, std::memory_order_relaxed);
    });
    parallel_ranges(k.size(), nt, [&](size_t b, size_t e) {
      for (size_t v = b; v < e; v++) {
        uint64_t h = mix((uint64_t)std::hash<Key>()(ks.at(v))) & mask;
        for (;;) {
          int32_t expect = -1;
          if (slot[h].compare_exchange_strong(expect, (int32_t)v, std::memory_order_relaxed)) break;
          h = (h + 1) & mask;
        }
      }
    });
  }
  int32_t find(const Key& key) const {  // -1: not a key of the graph
    if (!direct.empty()) return find_direct(key);
    uint64_t h = mix((uint64_t)std::hash<Key>()(key)) & mask;
    for (;;) {
      const int32_t s = slot[h].load(std::memory_order_relaxed);
      if (s < 0 || ks.at((size_t)s) == key) return s;
      h = (h + 1) & mask;
    }
  }
  template <typename K = Key>
  typename std::enable_if<std::is_integral<K>::value && sizeof(K) <= 4, int32_t>::type find_direct(const K& key) const {
    const int64_t i = (int64_t)key - lo;
    return (i < 0 || i >= (int64_t)direct.size()) ? -1 : direct[(size_t)i];
  }
  template <typename K = Key>
  typename std::enable_if<!(std::is_integral<K>::value && sizeof(K) <= 4), int32_t>::type find_direct(const K&) const {
    return -1;
  }
};

// The graph's nodes in iteration order (dense id = position), on nt threads. Node-based hash maps
// (libstdc++, libc++) keep each bucket's nodes contiguous in their one iteration list, so the list
// is the buckets' node runs in some bucket order: per bucket (threads) its node count and where
// the list continues after its last node (++ of find(last key)); the bucket chain from begin()
// gives every run's dense offset (one serial pass over non-empty buckets, not over nodes); the
// nodes are then written run by run (threads). Any inconsistency (a library that does not keep
// runs contiguous) falls back to one serial walk of the list.
template <typename Key>
inline void iteration_order(const std::unordered_map<Key, std::vector<Key>>& graph, size_t nt,
                            std::vector<const Key*>& keys, std::vector<const std::vector<Key>*>& succ) {
  const size_t n = graph.size();
  keys.resize(n);
  succ.resize(n);
  auto serial = [&] {
    size_t v = 0;
    for (const auto& kv : graph) {
      keys[v] = &kv.first;
      succ[v] = &kv.second;
      v++;
    }
  };
  const size_t B = graph.bucket_count();
  if (nt <= 1 || n < (1u << 16) || B == 0) { serial(); return; }
  std::vector<int64_t> cnt(B), nxt(B), start(B, -1);
  parallel_ranges(B, nt, [&](size_t b0, size_t b1) {
    for (size_t b = b0; b < b1; b++) {
      int64_t c = 0;
      const Key* last = nullptr;
      for (auto it = graph.begin(b); it != graph.end(b); ++it) { c++; last = &it->first; }
      cnt[b] = c;
      nxt[b] = -1;
      if (c) {
        auto it = graph.find(*last);
        ++it;
        nxt[b] = it == graph.end() ? -2 : (int64_t)graph.bucket(it->first);
      }
    }
  });
  size_t off = 0, runs = 0;
  for (int64_t b = (int64_t)graph.bucket(graph.begin()->first); b >= 0 && runs < B; b = nxt[(size_t)b], runs++) {
    if (start[(size_t)b] >= 0 || !cnt[(size_t)b]) { off = n + 1; break; }  // (a bucket twice: not runs)
    start[(size_t)b] = (int64_t)off;
    off += (size_t)cnt[(size_t)b];
  }
  if (off != n) { serial(); return; }
  parallel_ranges(B, nt, [&](size_t b0, size_t b1) {
    for (size_t b = b0; b < b1; b++) {
      if (!cnt[b]) continue;
      size_t v = (size_t)start[b];
      for (auto it = graph.begin(b); it != graph.end(b); ++it, v++) {
        keys[v] = &it->first;
        succ[v] = &it->second;
      }
    }
  });
}

template <typename Key>
inline Flat<Key> flatten(const std::unordered_map<Key, std::vector<Key>>& graph, size_t nt) {
  Flat<Key> f;
  const size_t n = graph.size();
  std::vector<const std::vector<Key>*> succ;
  iteration_order(graph, nt, f.keys, succ);
  KeyIndex<Key> idx;
  idx.build(f.keys, nt);  // (threads joined: every slot is published to the readers below)
  f.rp.assign(n + 1, 0);
  parallel_ranges(n, nt, [&](size_t b, size_t e) {
    for (size_t v = b; v < e; v++) f.rp[v + 1] = (int64_t)succ[v]->size();
  });
  for (size_t v = 0; v < n; v++) f.rp[v + 1] += f.rp[v];
  f.col.resize((size_t)f.rp[n]);
  std::atomic<bool> bad(false);
  parallel_ranges(n, nt, [&](size_t b, size_t e) {
    for (size_t v = b; v < e; v++) {
      int64_t o = f.rp[v];
      for (const Key& s : *succ[v]) {
        const int32_t id = idx.find(s);
        // every successor must be a key (README.md:69-73); the reference's behaviour is undefined
        if (id < 0) { bad = true; return; }
        f.col[(size_t)o++] = id;
      }
    }
  });
  if (bad) { std::cerr << ppr_strerror(PPR_ERR_GRAPH) << std::endl; exit(EXIT_FAILURE); }
  return f;
}

// include/grank.h:51-55 / header-only/grankMulti.h:299-304, same order and text
inline void check_params(size_t K, size_t L, size_t iterations, double damping) {
  if (K == 0) { std::cerr << "K must be positive" << std::endl; exit(EXIT_FAILURE); }
  if (L == 0) { std::cerr << "L must be positive" << std::endl; exit(EXIT_FAILURE); }
  if (K > L) { std::cerr << "K must be <= L" << std::endl; exit(EXIT_FAILURE); }
  if (iterations == 0) { std::cerr << "iterations must be positive" << std::endl; exit(EXIT_FAILURE); }
  if (damping < 0 || damping > 1) { std::cerr << "damping must be [0,1]" << std::endl; exit(EXIT_FAILURE); }
}

inline void fail(int rc) {
  std::cerr << ppr_strerror(rc) << std::endl;
  exit(EXIT_FAILURE);
}

// The result's outer map: one (empty) inner map per source, in dense order. It needs only the
// keys, so it is built on a host thread of its own WHILE the device computes (the outer inserts
// are one thread's work: ~1 s at 4 M sources, hidden behind the device call).
template <typename Key>
struct Outer {
  std::unordered_map<Key, std::unordered_map<Key, double>> out;
  std::vector<std::unordered_map<Key, double>*> row;  // dense id -> its inner map (stable: node-based)
  void build(const Flat<Key>& f) {
    const size_t n = f.keys.size();
    out.reserve(n);
    row.resize(n);
    for (size_t v = 0; v < n; v++) row[v] = &out[*f.keys[v]];
  }
};

// inner maps from one chunk of the device's top-K rows [v0, v0 + cnt) (independent per source)
template <typename Key>
inline void materialize_rows(const Flat<Key>& f, Outer<Key>& o, size_t K, size_t v0, size_t cnt,
                             const int32_t* ids, const double* sc, const int32_t* len) {
  for (size_t r = 0; r < cnt; r++) {
    std::unordered_map<Key, double>& m = *o.row[v0 + r];
    m.reserve((size_t)len[r]);
    for (int32_t i = 0; i < len[r]; i++) m.emplace(*f.keys[ids[r * K + i]], sc[r * K + i]);
  }
}

// all rows from whole host copies (n*K ids/scores, n lengths), on nt threads
template <typename Key>
inline void materialize_rows(const Flat<Key>& f, Outer<Key>& o, size_t K, const std::vector<int32_t>& ids,
                             const std::vector<double>& sc, const std::vector<int32_t>& len, size_t nt) {
  parallel_ranges(f.keys.size(), nt, [&](size_t b, size_t e) {
    materialize_rows(f, o, K, b, e - b, ids.data() + b * K, sc.data() + b * K, len.data() + b);
  });
}

// The top-K rows come down chunk by chunk into a ring of page-locked slots (DMA at link rate: the
// whole 3.2 GB of an RMAT-22 result into fresh pageable vectors cost a zero fill, the page faults
// and a staged copy) while nt threads materialise the chunks already down, so the download hides
// behind the inner-map fills. The calling thread fetches, then frees the plan's device memory
// while the fills finish; the workers take chunks in order.
template <typename Key>
inline int download_materialize(ppr_plan* p, const Flat<Key>& f, Outer<Key>& o, size_t K, size_t nt) {
  const size_t n = f.keys.size(), C = 8192, nc = (n + C - 1) / C;
  nt = std::max<size_t>(1, std::min(nt, nc));
  const size_t S = std::min(nc, nt + 2), ids_b = C * K * 4, slot_b = C * K * 12 + C * 4;
  void* ring = nullptr;
  int rc = ppr_host_alloc((int64_t)(S * slot_b), &ring);
  if (rc) { ppr_grank_plan_destroy(p); return rc; }
  std::unique_ptr<std::atomic<uint8_t>[]> done(new std::atomic<uint8_t>[nc]);
  for (size_t c = 0; c < nc; c++) done[c].store(0, std::memory_order_relaxed);
  std::atomic<size_t> fetched(0), next(0);
  std::atomic<int> err(0);
  auto slot = [&](size_t c) { return (char*)ring + (c % S) * slot_b; };
  std::vector<std::thread> th;
  th.reserve(nt);
  for (size_t t = 0; t < nt; t++)
    th.emplace_back([&] {
      for (;;) {
        const size_t c = next.fetch_add(1);
        if (c >= nc) return;
        while (fetched.load(std::memory_order_acquire) <= c) {
          if (err.load(std::memory_order_relaxed)) return;
          std::this_thread::yield();
        }
        char* b = slot(c);
        const size_t v0 = c * C;
        materialize_rows(f, o, K, v0, std::min(C, n - v0), (const int32_t*)b, (const double*)(b + ids_b),
                         (const int32_t*)(b + C * K * 12));
        done[c].store(1, std::memory_order_release);
      }
    });
  for (size_t c = 0; c < nc && !rc; c++) {
    if (c >= S)
      while (!done[c - S].load(std::memory_order_acquire)) std::this_thread::yield();
    char* b = slot(c);
    const size_t v0 = c * C;
    rc = ppr_grank_plan_fetch_rows(p, (int64_t)v0, (int64_t)std::min(n, v0 + C), (int32_t*)b,
                                   (double*)(b + ids_b), (int32_t*)(b + C * K * 12));
    if (rc) err.store(rc);
    else fetched.store(c + 1, std::memory_order_release);
  }
  ppr_grank_plan_destroy(p);  // (beside the last fills)
  for (auto& x : th) x.join();
  ppr_host_free(ring);
  return rc;
}

template <typename Key>
inline std::unordered_map<Key, std::unordered_map<Key, double>> grank_device(
    const std::unordered_map<Key, std::vector<Key>>& graph, size_t K, size_t L, size_t iterations,
    double damping, double tolerance, size_t nthreads = 0) {
  if (graph.empty()) return {};
  if (K > 0xffffffffu || L > 0xffffffffu || iterations > 0xffffffffu) fail(PPR_ERR_RANGE);
  const size_t nt = host_threads(nthreads);
  const auto t0 = std::chrono::steady_clock::now();
  Flat<Key> f = flatten(graph, nt);
  const size_t n = f.keys.size();
  ppr_csr g{(int64_t)n, f.rp.data(), f.col.empty() ? nullptr : f.col.data()};
  ppr_stats st;
  const auto t1 = std::chrono::steady_clock::now();
  HeapGrowth heap;  // (outer map and inner maps)
  Outer<Key> o;
  double outer_s = 0.0;
  std::thread outer([&] {  // beside the device call
    const auto a = std::chrono::steady_clock::now();
    o.build(f);
    outer_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
  });
  // plan (partitions, upload), device job; ppr_grank_csr's steps with the download left to the fills
  ppr_plan* p = nullptr;
  int rc = ppr_grank_plan_create(&g, nullptr, (uint32_t)K, (uint32_t)L, damping, nullptr, &p);
  if (!rc) {
    rc = ppr_grank_plan_run(p, (uint32_t)iterations, tolerance, &st);
    if (rc) ppr_grank_plan_destroy(p);
  }
  const auto t2 = std::chrono::steady_clock::now();
  outer.join();
  if (rc != PPR_OK) fail(rc);
  const auto t2b = std::chrono::steady_clock::now();
  rc = download_materialize(p, f, o, K, nt);
  if (rc != PPR_OK) fail(rc);
  if (getenv("PPR_TIMING")) {  // phase breakdown of one call (stderr)
    const auto t3 = std::chrono::steady_clock::now();
    auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double>(b - a).count();
    };
    std::cerr << "ppr_timing flatten_s " << sec(t0, t1) << " csr_call_s " << sec(t1, t2) << " device_s "
              << st.device_ms / 1e3 << " materialize_s " << sec(t2, t3) << " outer_build_s " << outer_s
              << " outer_wait_s " << sec(t2, t2b) << " inner_fill_s " << sec(t2b, t3) << std::endl;
  }
  return std::move(o.out);
}

}  // namespace hipdetail

/**
 * Approximated Personalized Pagerank for all nodes in the graph (the reference's ppr::grank).
 * @param graph      node -> successors; nodes without edges map to an empty vector
 * @param K          entries kept per source in the result (K <= L)
 * @param L          entries kept per source during the computation
 * @param iterations max number of iterations (the tolerance may stop earlier)
 * @param damping    damping factor, in [0, 1]
 * @param tolerance  stop when the norm-1 change of both partitions is below it; negative = never
 * @return source -> its top-K {node: score}
 */
template <typename Key>
std::unordered_map<Key, std::unordered_map<Key, double>> grank(
    const std::unordered_map<Key, std::vector<Key>>& graph, size_t K, size_t L, size_t iterations,
    double damping, double tolerance) {
  hipdetail::check_params(K, L, iterations, damping);
  return hipdetail::grank_device(graph, K, L, iterations, damping, tolerance);
}

}  // namespace ppr

#endif  // PPR_HIP_DROPIN_GRANK_H
