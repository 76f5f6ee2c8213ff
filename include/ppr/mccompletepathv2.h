// ppr/mccompletepathv2.h -- drop-in replacement for the reference's ppr::mccompletepathv2
// (include/mccompletepathv2.h:182-187, header-only/mccompletepathv2.h:42-47), running on an
// MI355X through libppr_hip.so (ppr_mccp2_csr, include/ppr_hip.h).
//
// Same template, same signature, same parameter checks with the same messages and
// exit(EXIT_FAILURE) (include/mccompletepathv2.h:190-194), same result shape. `iterations` is the
// number of random walks per node (R). The reference seeds a process-global mt19937 from
// std::random_device, so its results vary run to run; here the walks use counter-based Philox
// keyed by a seed drawn the same way (std::random_device) unless PPR_MC_SEED is set in the
// environment, which makes a run reproducible. executionOrder and the combine are exact.
#ifndef PPR_HIP_DROPIN_MCCOMPLETEPATHV2_H
#define PPR_HIP_DROPIN_MCCOMPLETEPATHV2_H

#include <random>

#include "grank.h"

namespace ppr {
namespace hipdetail {

inline uint64_t mc_seed() {
  const char* e = getenv("PPR_MC_SEED");
  if (e && *e) return strtoull(e, nullptr, 0);
  std::random_device rd;
  return ((uint64_t)rd() << 32) ^ (uint64_t)rd();
}

}  // namespace hipdetail

/**
 * Approximated Personalized Pagerank for all nodes in the graph, Monte Carlo complete path
 * (the reference's ppr::mccompletepathv2).
 * @param graph      node -> successors; nodes without edges map to an empty vector
 * @param K          entries kept per source in the result (K <= L)
 * @param L          entries kept per source during the computation
 * @param iterations random walks per node in the worst case
 * @param damping    damping factor, in [0, 1]
 * @return source -> its top-K {node: score}
 */
template <typename Key>
std::unordered_map<Key, std::unordered_map<Key, double>> mccompletepathv2(
    const std::unordered_map<Key, std::vector<Key>>& graph, size_t K, size_t L, size_t iterations,
    double damping) {
  hipdetail::check_params(K, L, iterations, damping);
  if (graph.empty()) return {};
  if (K > 0xffffffffu || L > 0xffffffffu || iterations > 0xffffffffu) hipdetail::fail(PPR_ERR_RANGE);
  const size_t nt = hipdetail::host_threads();
  hipdetail::Flat<Key> f = hipdetail::flatten(graph, nt);
  const size_t n = f.keys.size();
  ppr_csr g{(int64_t)n, f.rp.data(), f.col.empty() ? nullptr : f.col.data()};
  std::vector<int32_t> ids(n * K), len(n);
  std::vector<double> sc(n * K);
  hipdetail::HeapGrowth heap;  // (outer map and inner maps)
  hipdetail::Outer<Key> o;
  std::thread outer([&] { o.build(f); });  // the result's outer map, beside the device call
  const int rc = ppr_mccp2_csr(&g, (uint32_t)K, (uint32_t)L, (uint32_t)iterations, damping, hipdetail::mc_seed(),
                               nullptr, ids.data(), sc.data(), len.data(), nullptr);
  outer.join();
  if (rc != PPR_OK) hipdetail::fail(rc);
  hipdetail::materialize_rows(f, o, K, ids, sc, len, nt);
  return std::move(o.out);
}

}  // namespace ppr

#endif  // PPR_HIP_DROPIN_MCCOMPLETEPATHV2_H
