// host_graph.cpp -- host-side graph preparation behind the C ABI (include/ppr_hip.h).
//
//  * ppr_find_partitions_csr: the BFS 2-colouring GRank alternates over
//    (reference include/internal/pprInternal.h:29-99), on the dense CSR whose ids follow the
//    graph's iteration order, so it reproduces the reference's partitions exactly.
//  * ppr_execution_order_csr: MCCompletePathV2's node order (include/mccompletepathv2.h:36-113).
//  * ppr_rmat_generate: the synthetic RMAT graphs the benchmarks run on (Graph500 a/b/c/d
//    quadrant recursion, counter-based RNG, vertex labels scrambled by a bijection, duplicate
//    edges removed, self-loops kept, successors ascending).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <chrono>
#include <vector>

#include "../../include/ppr_hip.h"
#include "../../include/ppr/importGraph.h"
#include "host_par.h"

namespace {

inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// bijection on `bits`-bit integers: odd multiplies and xor-shifts modulo 2^bits
inline uint64_t scramble(uint64_t x, int bits, uint64_t seed) {
  if (bits == 0) return 0;
  const uint64_t mask = bits >= 64 ? ~0ULL : ((1ULL << bits) - 1);
  uint64_t s = seed ^ 0xD1B54A32D192ED03ULL;
  for (int r = 0; r < 3; r++) {
    uint64_t mul = splitmix64(s) | 1ULL;
    uint64_t add = splitmix64(s);
    x = (x * mul + add) & mask;
    x ^= x >> ((bits + 1) / 2);
  }
  return x & mask;
}

using pprh::parallel_for;
using pprh::host_threads;
using pprh::hw_threads;

}  // namespace

extern "C" {

int ppr_find_partitions_csr(const ppr_csr* g, uint8_t* part) {
  // The reference's BFS (pprInternal.h:29-99) takes roots in graph order, puts a root in
  // partitions.first and every newly reached successor / predecessor in the partition opposite
  // to the node that reached it. In a FIFO BFS all nodes that can reach a node first sit at the
  // same depth, so partition(v) = parity of the undirected BFS distance from the root of v's weakly
  // connected component, and that root is the component's first node in graph order (earlier
  // components are exhausted before the next root is taken). Both are order-free, so they are
  // computed in parallel: union-find for the roots, a level-synchronous multi-source BFS for the
  // depths -- same partitions as the sequential sweep, on all host threads.
  if (!g || !part || g->n < 0) return PPR_ERR_ARG;
  const int64_t n = g->n;
  if (n == 0) return PPR_OK;
  const int64_t* rp = g->row_ptr;
  const int32_t* col = g->col;
  const int64_t m = rp[n];
  const int nth = host_threads();
  std::atomic<bool> bad(false);
  const bool tm = getenv("PPR_TIMING") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!tm) return;
    const auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "ppr_timing partitions %s %.4f\n", what, std::chrono::duration<double>(t1 - t0).count());
    t0 = t1;
  };
  // (successor ids checked here; no predecessor lists are built: the union-find needs none, and the
  // BFS below finds a node's predecessors in the frontier from its own successor list)
  parallel_for(n, nth, [&](int64_t b, int64_t e, int) {
    for (int64_t k = rp[b]; k < rp[e]; k++)
      if (col[k] < 0 || col[k] >= n) { bad = true; return; }
  });
  if (bad) return PPR_ERR_GRAPH;
  lap("check");
  // weakly connected components, representative = smallest id (lock-free union by index)
  std::vector<int32_t> parent(n);
  for (int64_t v = 0; v < n; v++) parent[v] = (int32_t)v;
  auto find = [&](int32_t x) {
    for (;;) {
      const int32_t p = __atomic_load_n(&parent[x], __ATOMIC_RELAXED);
      if (p == x) return x;
      const int32_t gp = __atomic_load_n(&parent[p], __ATOMIC_RELAXED);
      if (gp != p) __atomic_compare_exchange_n(&parent[x], const_cast<int32_t*>(&p), gp, false, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED);
      x = p;
    }
  };
  parallel_for(n, nth, [&](int64_t b, int64_t e, int) {
    for (int64_t v = b; v < e; v++)
      for (int64_t k = rp[v]; k < rp[v + 1]; k++) {
        int32_t x = (int32_t)v, y = col[k];
        for (;;) {
          x = find(x);
          y = find(y);
          if (x == y) break;
          if (x > y) std::swap(x, y);
          int32_t expect = y;  // hang the larger root under the smaller one
          if (__atomic_compare_exchange_n(&parent[y], &expect, x, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) break;
        }
      }
  });
  lap("union_find");
  // multi-source BFS from every component's smallest node over the undirected graph, with out-edges
  // only: a level joins (a) the unvisited successors of the frontier (top-down, CAS) and then (b)
  // every unvisited node with a successor in the frontier (a predecessor of it: bottom-up over the
  // shrinking list of unvisited nodes, stopping at the first hit). Depths are the shortest
  // undirected distances either way; no predecessor lists (a transpose cost more than this).
  std::vector<int32_t> depth(n, -1);
  std::vector<int32_t> front, rest;
  for (int64_t v = 0; v < n; v++)
    if (find((int32_t)v) == (int32_t)v) { depth[v] = 0; front.push_back((int32_t)v); }
  {
    std::vector<std::vector<int32_t>> part_rest(nth);
    parallel_for(n, nth, [&](int64_t b, int64_t e, int t) {
      for (int64_t v = b; v < e; v++)
        if (depth[v] == -1) part_rest[t].push_back((int32_t)v);
    });
    for (auto& x : part_rest) rest.insert(rest.end(), x.begin(), x.end());
  }
  std::vector<std::vector<int32_t>> next(nth), keep(nth);
  // The bottom-up scan costs O(|rest|) per level, O(depth x n) in all: fine on small-diameter graphs
  // (RMAT-22: ~20 levels), minutes on a long path or a road network. Once the scans have cost
  // more than the graph itself, the predecessor lists are built once and the remaining levels go
  // top-down over both edge directions (O(n + m) from there on).
  double scanned = 0.0;
  const double scan_cap = 2.0 * (double)(n + m) + 1e6;
  std::vector<int64_t> prp;
  std::vector<int32_t> pcol;
  int32_t d = 0;
  for (; !front.empty(); d++) {
    if (scanned > scan_cap || getenv("PPR_BFS_TRANSPOSE")) break;
    scanned += (double)rest.size();
    for (auto& x : next) x.clear();
    parallel_for((int64_t)front.size(), nth, [&](int64_t b, int64_t e, int t) {
      std::vector<int32_t>& out = next[t];
      for (int64_t i = b; i < e; i++) {
        const int32_t x = front[i];
        for (int64_t k = rp[x]; k < rp[x + 1]; k++) {
          const int32_t s = col[k];
          int32_t expect = -1;
          if (__atomic_load_n(&depth[s], __ATOMIC_RELAXED) == -1 &&
              __atomic_compare_exchange_n(&depth[s], &expect, d + 1, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED))
            out.push_back(s);
        }
      }
    });
    // bottom-up: the still unvisited nodes with a successor at depth d (their writes go to their
    // own entry only, after which they are at d + 1, never d)
    for (auto& x : keep) x.clear();
    parallel_for((int64_t)rest.size(), nth, [&](int64_t b, int64_t e, int t) {
      std::vector<int32_t>& out = next[t];
      std::vector<int32_t>& kp = keep[t];
      for (int64_t i = b; i < e; i++) {
        const int32_t v = rest[i];
        if (__atomic_load_n(&depth[v], __ATOMIC_RELAXED) != -1) continue;  // (joined top-down)
        bool hit = false;
        for (int64_t k = rp[v]; k < rp[v + 1] && !hit; k++) hit = __atomic_load_n(&depth[col[k]], __ATOMIC_RELAXED) == d;
        if (hit) {
          __atomic_store_n(&depth[v], d + 1, __ATOMIC_RELAXED);
          out.push_back(v);
        } else {
          kp.push_back(v);
        }
      }
    });
    rest.clear();
    for (auto& x : keep) rest.insert(rest.end(), x.begin(), x.end());
    front.clear();
    for (auto& x : next) front.insert(front.end(), x.begin(), x.end());
  }
  if (!front.empty()) {
    // transposed mode: predecessor lists (counting sort by target), then plain top-down levels
    // over successors and predecessors
    prp.assign(n + 1, 0);
    for (int64_t k = 0; k < m; k++) prp[col[k] + 1]++;
    for (int64_t i = 0; i < n; i++) prp[i + 1] += prp[i];
    pcol.resize(m > 0 ? m : 1);
    {
      std::vector<int64_t> fill(prp.begin(), prp.end() - 1);
      for (int64_t v = 0; v < n; v++)
        for (int64_t k = rp[v]; k < rp[v + 1]; k++) pcol[fill[col[k]]++] = (int32_t)v;
    }
    if (tm) fprintf(stderr, "ppr_timing partitions transposed_at_level %d\n", (int)d);
    for (; !front.empty(); d++) {
      for (auto& x : next) x.clear();
      parallel_for((int64_t)front.size(), nth, [&](int64_t b, int64_t e, int t) {
        std::vector<int32_t>& out = next[t];
        auto visit = [&](int32_t s) {
          int32_t expect = -1;
          if (__atomic_load_n(&depth[s], __ATOMIC_RELAXED) == -1 &&
              __atomic_compare_exchange_n(&depth[s], &expect, d + 1, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED))
            out.push_back(s);
        };
        for (int64_t i = b; i < e; i++) {
          const int32_t x = front[i];
          for (int64_t k = rp[x]; k < rp[x + 1]; k++) visit(col[k]);
          for (int64_t k = prp[x]; k < prp[x + 1]; k++) visit(pcol[k]);
        }
      });
      front.clear();
      for (auto& x : next) front.insert(front.end(), x.begin(), x.end());
    }
  }
  parallel_for(n, nth, [&](int64_t b, int64_t e, int) {
    for (int64_t v = b; v < e; v++) part[v] = (uint8_t)(depth[v] & 1);
  });
  lap("bfs");
  return PPR_OK;
}

int ppr_execution_order_csr(const ppr_csr* g, int32_t* order) {
  if (!g || !order || g->n < 0) return PPR_ERR_ARG;
  const int64_t n = g->n;
  if (n == 0) return PPR_OK;
  const int64_t* rp = g->row_ptr;
  const int32_t* col = g->col;
  const int64_t m = rp[n];
  std::vector<int64_t> prp(n + 1, 0);
  for (int64_t e = 0; e < m; e++) prp[col[e] + 1]++;
  for (int64_t i = 0; i < n; i++) prp[i + 1] += prp[i];
  std::vector<int32_t> pcol(m > 0 ? m : 1);
  {
    std::vector<int64_t> fill(prp.begin(), prp.end() - 1);
    for (int64_t v = 0; v < n; v++)
      for (int64_t e = rp[v]; e < rp[v + 1]; e++) pcol[fill[col[e]]++] = (int32_t)v;
  }
  // sort by (indegree desc, outdegree asc) (include/mccompletepathv2.h:52-62). The reference uses
  // the unstable std::sort on records in graph order; the order it leaves equal (in, out) pairs
  // in is a function of the key sequence and the comparator only, so running the same library
  // sort on (node, in, out) records in the same order reproduces it exactly.
  struct Rec { int32_t node; int64_t in, out; };
  std::vector<Rec> recs(n);
  for (int64_t i = 0; i < n; i++) recs[i] = Rec{(int32_t)i, prp[i + 1] - prp[i], rp[i + 1] - rp[i]};
  std::sort(recs.begin(), recs.end(), [](const Rec& a, const Rec& b) {
    return a.in > b.in ? true : (a.in == b.in ? a.out < b.out : false);
  });
  std::vector<int32_t> sorted(n);
  for (int64_t i = 0; i < n; i++) sorted[i] = recs[i].node;
  // predecessor-release BFS (:64-111)
  std::vector<int64_t> wait(n);
  for (int64_t v = 0; v < n; v++) wait[v] = rp[v + 1] - rp[v];
  std::vector<uint8_t> vis(n, 0);
  std::vector<int32_t> q(n);
  int64_t out = 0;
  for (int64_t i = 0; i < n; i++) {
    const int32_t node = sorted[i];
    if (vis[node]) continue;
    int64_t qh = 0, qt = 0;
    q[qt++] = node;
    while (qh < qt) {
      const int32_t x = q[qh++];
      if (out >= n) return PPR_ERR_GRAPH;
      order[out++] = x;
      vis[x] = 1;
      for (int64_t e = prp[x]; e < prp[x + 1]; e++) {
        const int32_t p = pcol[e];
        if (wait[p]-- > 0) {
          if (wait[p] == 0 && !vis[p]) q[qt++] = p;
        }
      }
    }
  }
  // every node is emitted exactly once: released at most once (wait hits 0 once) and taken as
  // a root only when unvisited with an empty queue
  return (int)(out == n ? PPR_OK : PPR_ERR_GRAPH);
}

int64_t ppr_rmat_generate(int32_t scale, int32_t edge_factor, double a, double b, double c,
                          uint64_t seed, int64_t* row_ptr, int32_t* col, int64_t col_cap) {
  if (scale < 0 || scale > 30 || edge_factor < 0 || !row_ptr) return -PPR_ERR_ARG;
  const int64_t n = 1LL << scale;
  const int64_t m0 = (int64_t)edge_factor * n;
  const int nth = hw_threads();
  const double ab = a + b, abc = a + b + c;
  std::vector<uint64_t> edges(m0);
  parallel_for(m0, nth, [&](int64_t b0, int64_t e0, int) {
    for (int64_t e = b0; e < e0; e++) {
      uint64_t s = seed * 0x100000001B3ULL ^ (uint64_t)e * 0x9E3779B97F4A7C15ULL;
      splitmix64(s);
      uint64_t src = 0, dst = 0;
      for (int l = 0; l < scale; l++) {
        const double u = (double)(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0);
        const uint64_t bs = u >= ab, bd = (u >= a && u < ab) || u >= abc;
        src = (src << 1) | bs;
        dst = (dst << 1) | bd;
      }
      src = scramble(src, scale, seed);
      dst = scramble(dst, scale, seed);
      edges[e] = (src << 32) | dst;
    }
  });
  // bucket by source (counting sort), then sort + unique each row
  std::vector<int64_t> cnt(n + 1, 0);
  for (int64_t e = 0; e < m0; e++) cnt[(edges[e] >> 32) + 1]++;
  for (int64_t i = 0; i < n; i++) cnt[i + 1] += cnt[i];
  std::vector<uint32_t> tmp(m0);
  {
    std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
    for (int64_t e = 0; e < m0; e++) tmp[fill[edges[e] >> 32]++] = (uint32_t)(edges[e] & 0xffffffffu);
  }
  std::vector<uint64_t>().swap(edges);
  std::vector<int64_t> deg(n, 0);
  parallel_for(n, nth, [&](int64_t b0, int64_t e0, int) {
    for (int64_t v = b0; v < e0; v++) {
      uint32_t* p = tmp.data() + cnt[v];
      int64_t k = cnt[v + 1] - cnt[v];
      std::sort(p, p + k);
      deg[v] = std::unique(p, p + k) - p;
    }
  });
  row_ptr[0] = 0;
  for (int64_t v = 0; v < n; v++) row_ptr[v + 1] = row_ptr[v] + deg[v];
  const int64_t m = row_ptr[n];
  if (!col) return m;          // size query
  if (col_cap < m) return -PPR_ERR_ARG;
  parallel_for(n, nth, [&](int64_t b0, int64_t e0, int) {
    for (int64_t v = b0; v < e0; v++)
      std::memcpy(col + row_ptr[v], tmp.data() + cnt[v], sizeof(int32_t) * deg[v]);
  });
  return m;
}

}  // extern "C"

extern "C" int ppr_import_edge_csv(const char* path, int64_t* n_out, int64_t* m_out, int32_t* keys,
                                   int64_t* row_ptr, int32_t* col) {
  // src/main.cc:78-112 through ppr::importGraph; dense ids = the map's iteration order. Call
  // with keys/row_ptr/col NULL for the sizes, then again with buffers of n, n+1 and m entries.
  if (!path || !n_out || !m_out) return PPR_ERR_ARG;
  std::ifstream probe(path);
  if (!probe) return PPR_ERR_ARG;
  probe.close();
  std::unordered_map<int, std::vector<int>> g;
  try {
    g = ppr::importGraph(path, false);
  } catch (...) {
    return PPR_ERR_ARG;  // a line std::stoi rejects (the reference throws)
  }
  const int64_t n = (int64_t)g.size();
  int64_t m = 0;
  for (const auto& kv : g) m += (int64_t)kv.second.size();
  *n_out = n;
  *m_out = m;
  if (!keys && !row_ptr && !col) return PPR_OK;
  if (!keys || !row_ptr || (m > 0 && !col)) return PPR_ERR_ARG;
  std::unordered_map<int, int32_t> idx;
  idx.reserve(g.size());
  int32_t i = 0;
  for (const auto& kv : g) { keys[i] = kv.first; idx[kv.first] = i; i++; }
  row_ptr[0] = 0;
  int64_t o = 0;
  i = 0;
  for (const auto& kv : g) {
    for (int s : kv.second) col[o++] = idx.at(s);
    row_ptr[++i] = o;
  }
  return PPR_OK;
}
