// ppr/grankMulti.h -- drop-in replacement for the reference's ppr::grankMulti
// (header-only/grankMulti.h:289-296). The reference splits the active partition over nThreads
// std::threads per iteration (header-only/grankMulti.h:325-333,378-396,417-433); here the merge
// runs on the GPU, so the result is the same as ppr::grank's (as the reference's own tests require,
// test/grankMultiThreadTest.cc:384-576) and nThreads is the number of host threads of the call's
// host-side work: flattening the map graph to CSR and materialising the result maps (SURVEY.md
// s8b). For several GPUs use the source-sharded entry points of include/ppr_hip.h
// (ppr_grank_plan_run_sharded).
#ifndef PPR_HIP_DROPIN_GRANKMULTI_H
#define PPR_HIP_DROPIN_GRANKMULTI_H

#include "grank.h"

namespace ppr {

template <typename Key>
std::unordered_map<Key, std::unordered_map<Key, double>> grankMulti(
    const std::unordered_map<Key, std::vector<Key>>& graph, size_t K, size_t L, size_t iterations,
    double damping, double tolerance, size_t nThreads) {
  hipdetail::check_params(K, L, iterations, damping);
  if (nThreads == 0) { std::cerr << "nThreads must be positive" << std::endl; exit(EXIT_FAILURE); }
  return hipdetail::grank_device(graph, K, L, iterations, damping, tolerance, nThreads);
}

}  // namespace ppr

#endif  // PPR_HIP_DROPIN_GRANKMULTI_H
