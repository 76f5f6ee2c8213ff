// host_par.h -- host threads for the graph preparation behind the C ABI (partitions, plan
// creation, executionOrder): static ranges over std::thread.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

namespace pprh {

template <class F>
inline void parallel_for(int64_t n, int nthreads, F f) {
  if (nthreads <= 1 || n < 4096) { f((int64_t)0, n, 0); return; }
  std::vector<std::thread> th;
  const int64_t chunk = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; t++) {
    const int64_t b = t * chunk, e = std::min<int64_t>(n, b + chunk);
    if (b >= e) break;
    th.emplace_back(f, b, e, t);
  }
  for (auto& t : th) t.join();
}

// one thread per task index 0..k-1 (for a few coarse tasks, which parallel_for would run serially)
template <class F>
inline void parallel_tasks(int k, F f) {
  std::vector<std::thread> th;
  for (int t = 1; t < k; t++) th.emplace_back(f, t);
  if (k > 0) f(0);
  for (auto& t : th) t.join();
}

inline int hw_threads() {
  unsigned h = std::thread::hardware_concurrency();
  if (h == 0) h = 1;
  return (int)std::min<unsigned>(h, 16);
}

// PPR_HOST_THREADS, else OMP_NUM_THREADS (the CPU share on shared hosts), else hw_threads()
inline int host_threads() {
  const char* e = getenv("PPR_HOST_THREADS");
  if (!e || !*e) e = getenv("OMP_NUM_THREADS");
  if (e && *e && atoi(e) > 0) return std::min(atoi(e), 64);
  return hw_threads();
}

}  // namespace pprh
