// Host-side sanitizer driver (SURVEY.md s5 "race detection / sanitizers"): the host code of the
// engine -- csrc/host_graph.cpp (partitions, executionOrder, RMAT generator, CSV importer) and the
// drop-in header's flatten (threaded iteration-order walk, the CAS-built KeyIndex) and result
// materialisation -- compiled with g++ -fsanitize=address,undefined (build.build_host_asan) and run
// on RMAT graphs, printing digests the test compares with the production library's results.
//   host_asan_test graph <scale> <seed>   digests of partitions / executionOrder / CSR
//   host_asan_test flatten <scale>        map graph -> CSR -> fake rows -> result maps (dense ids)
//   host_asan_test flatten_sparse <scale> the same with keys spread over the int range
//   host_asan_test csv <path>             ppr_import_edge_csv digests
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <unordered_map>
#include <vector>

#include "ppr/grank.h"

static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
  const unsigned char* b = (const unsigned char*)p;
  for (size_t i = 0; i < n; i++) { h ^= b[i]; h *= 1099511628211ull; }
  return h;
}

static int rmat(int scale, int seed, std::vector<int64_t>& rp, std::vector<int32_t>& col) {
  const int64_t n = 1LL << scale;
  rp.assign(n + 1, 0);
  const int64_t m = ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, (uint64_t)seed, rp.data(), nullptr, 0);
  col.assign(m, 0);
  ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, (uint64_t)seed, rp.data(), col.data(), m);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string mode = argv[1];
  if (mode == "graph") {
    std::vector<int64_t> rp;
    std::vector<int32_t> col;
    rmat(atoi(argv[2]), atoi(argv[3]), rp, col);
    const int64_t n = (int64_t)rp.size() - 1;
    ppr_csr g{n, rp.data(), col.data()};
    std::vector<uint8_t> part(n);
    std::vector<int32_t> order(n);
    if (ppr_find_partitions_csr(&g, part.data()) != PPR_OK) return 3;
    if (ppr_execution_order_csr(&g, order.data()) != PPR_OK) return 3;
    printf("{\"n\": %lld, \"m\": %lld, \"csr\": \"%016llx\", \"part\": \"%016llx\", \"order\": \"%016llx\"}\n",
           (long long)n, (long long)col.size(),
           (unsigned long long)fnv(col.data(), 4 * col.size(), fnv(rp.data(), 8 * rp.size())),
           (unsigned long long)fnv(part.data(), part.size()), (unsigned long long)fnv(order.data(), 4 * order.size()));
    return 0;
  }
  if (mode == "flatten" || mode == "flatten_sparse") {
    std::vector<int64_t> rp;
    std::vector<int32_t> col;
    rmat(atoi(argv[2]), 42, rp, col);
    const int64_t n = (int64_t)rp.size() - 1;
    // flatten_sparse: keys spread over the int range (the KeyIndex hash, not its dense-id array)
    const bool sparse = mode == "flatten_sparse";
    auto key = [&](int64_t v) { return sparse ? (int)((uint32_t)v * 2654435761u >> 1) : (int)v; };
    std::unordered_map<int, std::vector<int>> graph;
    for (int64_t v = n - 1; v >= 0; v--) {
      std::vector<int>& s = graph[key(v)];
      for (int64_t e = rp[v]; e < rp[v + 1]; e++) s.push_back(key(col[e]));
    }
    const size_t nt = 8;
    ppr::hipdetail::Flat<int> f = ppr::hipdetail::flatten(graph, nt);
    // CSR of the dense ids must describe the same graph
    int bad = 0;
    for (size_t v = 0; v < f.keys.size(); v++) {
      const std::vector<int>& s = graph.at(*f.keys[v]);
      if ((int64_t)s.size() != f.rp[v + 1] - f.rp[v]) { bad++; continue; }
      for (size_t j = 0; j < s.size(); j++)
        if (*f.keys[(size_t)f.col[(size_t)f.rp[v] + j]] != s[j]) bad++;
    }
    // materialise fake top-K rows (each source: its first K successors' ids, decreasing scores)
    const size_t K = 8;
    std::vector<int32_t> ids(f.keys.size() * K), len(f.keys.size());
    std::vector<double> sc(f.keys.size() * K);
    for (size_t v = 0; v < f.keys.size(); v++) {
      std::vector<int32_t> u;
      for (int64_t e = f.rp[v]; e < f.rp[v + 1] && u.size() < K; e++)
        if (std::find(u.begin(), u.end(), f.col[(size_t)e]) == u.end()) u.push_back(f.col[(size_t)e]);
      len[v] = (int32_t)u.size();
      for (size_t i = 0; i < u.size(); i++) { ids[v * K + i] = u[i]; sc[v * K + i] = 1.0 / (double)(i + 1); }
    }
    ppr::hipdetail::HeapGrowth heap;
    ppr::hipdetail::Outer<int> o;
    o.build(f);
    ppr::hipdetail::materialize_rows(f, o, K, ids, sc, len, nt);
    for (size_t v = 0; v < f.keys.size(); v++)
      if (o.out.at(*f.keys[v]).size() != (size_t)len[v]) bad++;
    printf("{\"n\": %zu, \"bad\": %d}\n", f.keys.size(), bad);
    return bad ? 1 : 0;
  }
  if (mode == "csv") {
    int64_t n = 0, m = 0;
    if (ppr_import_edge_csv(argv[2], &n, &m, nullptr, nullptr, nullptr) != PPR_OK) return 3;
    std::vector<int32_t> keys(n), col(m);
    std::vector<int64_t> rp(n + 1);
    if (ppr_import_edge_csv(argv[2], &n, &m, keys.data(), rp.data(), col.data()) != PPR_OK) return 3;
    printf("{\"n\": %lld, \"m\": %lld, \"keys\": \"%016llx\", \"csr\": \"%016llx\"}\n", (long long)n, (long long)m,
           (unsigned long long)fnv(keys.data(), 4 * keys.size()),
           (unsigned long long)fnv(col.data(), 4 * col.size(), fnv(rp.data(), 8 * rp.size())));
    return 0;
  }
  return 2;
}
