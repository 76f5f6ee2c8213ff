// ppr/grank.h -- drop-in replacement for the reference's ppr::grank (include/grank.h:42-48,
// header-only/grank.h:214-220), running on an MI355X through libppr_hip.so (include/ppr_hip.h).
//
// Same template, same signature, same parameter checks with the same messages and
// exit(EXIT_FAILURE) (include/grank.h:51-55), same result shape. Link with -lppr_hip.
//
// What happens per call (DESIGN.md "boundary"):
//   1. dense ids = the graph's iteration order, CSR keeps every successor vector's order
//      (the reference's partitions and summation order depend on both);
//   2. ppr_grank_csr(): BFS partitions (include/internal/pprInternal.h:29-99), upload, init,
//      iterations, final top-K on the device, download;
//   3. the top-K rows are materialised back into unordered_map<Key, unordered_map<Key,double>>.
// Ties at a top-L/top-K cut are broken by (score desc, dense id asc); the reference leaves them to
// its hash-map order.
#ifndef PPR_HIP_DROPIN_GRANK_H
#define PPR_HIP_DROPIN_GRANK_H

#include <stdint.h>
#include <stdlib.h>

#include <iostream>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../ppr_hip.h"

namespace ppr {
namespace hipdetail {

template <typename Key>
struct Flat {
  std::vector<const Key*> keys;  // dense id -> key (points into the caller's graph)
  std::vector<int64_t> rp;
  std::vector<int32_t> col;
};

template <typename Key>
inline Flat<Key> flatten(const std::unordered_map<Key, std::vector<Key>>& graph) {
  Flat<Key> f;
  std::unordered_map<Key, int32_t> idx;
  idx.reserve(graph.size());
  f.keys.reserve(graph.size());
  for (const auto& kv : graph) {
    idx.emplace(kv.first, (int32_t)f.keys.size());
    f.keys.push_back(&kv.first);
  }
  f.rp.reserve(graph.size() + 1);
  f.rp.push_back(0);
  for (const Key* k : f.keys) {
    for (const Key& s : graph.find(*k)->second) {
      auto it = idx.find(s);
      // every successor must be a key (README.md:69-73); the reference's behaviour is undefined
      if (it == idx.end()) { std::cerr << ppr_strerror(PPR_ERR_GRAPH) << std::endl; exit(EXIT_FAILURE); }
      f.col.push_back(it->second);
    }
    f.rp.push_back((int64_t)f.col.size());
  }
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

template <typename Key>
inline std::unordered_map<Key, std::unordered_map<Key, double>> materialize(
    const Flat<Key>& f, size_t K, const std::vector<int32_t>& ids, const std::vector<double>& sc,
    const std::vector<int32_t>& len) {
  std::unordered_map<Key, std::unordered_map<Key, double>> out;
  out.reserve(f.keys.size());
  for (size_t v = 0; v < f.keys.size(); v++) {
    std::unordered_map<Key, double>& m = out[*f.keys[v]];
    m.reserve((size_t)len[v]);
    for (int32_t i = 0; i < len[v]; i++) m.emplace(*f.keys[ids[v * K + i]], sc[v * K + i]);
  }
  return out;
}

template <typename Key>
inline std::unordered_map<Key, std::unordered_map<Key, double>> grank_device(
    const std::unordered_map<Key, std::vector<Key>>& graph, size_t K, size_t L, size_t iterations,
    double damping, double tolerance) {
  if (graph.empty()) return {};
  if (K > 0xffffffffu || L > 0xffffffffu || iterations > 0xffffffffu) fail(PPR_ERR_RANGE);
  Flat<Key> f = flatten(graph);
  const size_t n = f.keys.size();
  ppr_csr g{(int64_t)n, f.rp.data(), f.col.empty() ? nullptr : f.col.data()};
  std::vector<int32_t> ids(n * K), len(n);
  std::vector<double> sc(n * K);
  const int rc = ppr_grank_csr(&g, nullptr, (uint32_t)K, (uint32_t)L, (uint32_t)iterations, damping,
                               tolerance, nullptr, ids.data(), sc.data(), len.data(), nullptr);
  if (rc != PPR_OK) fail(rc);
  return materialize(f, K, ids, sc, len);
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
