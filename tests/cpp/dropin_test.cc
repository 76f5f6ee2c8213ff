// Drop-in check: code written against the reference's API (the README examples and the shape of
// test/grankTest.cc) compiled unchanged against include/ppr/*.h and linked with libppr_hip.so.
//   dropin_test bad <case>   parameter errors: same message + exit(EXIT_FAILURE), no device use
//   dropin_test empty        empty graph -> empty result
//   dropin_test ring         README ring of 100, K50 L100 30 it 1e-3: prints "src key score" rows
//   dropin_test known        known answers of test/grankTest.cc (exit 0 when all hold)
//   dropin_test mcbad <case> / mcknown   the same for mccompletepathv2 (test/mccompletepathv2Test.cc)
//   dropin_test e2e <scale> [iters]  RMAT graph as unordered_map, ppr::grank(K64, L128, iters (10)) end
//                                    to end (PPR_TIMING=1: flatten / device / materialise split on stderr)
//   dropin_test e2echeck <scale> <iters> <stride>  the same call; every stride-th result row compared
//                                    with the device rows of ppr_grank_csr on the same CSR, bit for bit
//   dropin_test multieq <scale> <iters>  grankMulti(..., 1) == grankMulti(..., 8) == grank(...) maps
//   dropin_test order <n> <seed>     (host only) the threaded iteration-order walk of flatten equals the
//                                    map's own iteration order, for int and string keys, after inserts,
//                                    erasures and rehashes
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "ppr/grank.h"
#include "ppr/grankMulti.h"
#include "ppr/mccompletepathv2.h"

using namespace std;

static int check(bool c, const char* what) {
  if (!c) { fprintf(stderr, "FAILED: %s\n", what); return 1; }
  return 0;
}

// flatten's threaded iteration-order walk == the map's own order (1 = mismatch)
template <typename K>
static int same_order(const unordered_map<K, vector<K>>& g, const char* what) {
  vector<const K*> k1, k2;
  vector<const vector<K>*> s1, s2;
  ppr::hipdetail::iteration_order(g, 1, k1, s1);
  ppr::hipdetail::iteration_order(g, 8, k2, s2);
  int bad = check(k1.size() == g.size() && k1 == k2 && s1 == s2, what);
  size_t v = 0;
  for (typename unordered_map<K, vector<K>>::const_iterator it = g.begin(); it != g.end(); ++it, ++v)
    if (v >= k1.size() || k1[v] != &it->first) return bad + check(false, what);
  return bad;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  string mode = argv[1];
  unordered_map<int, vector<int>> graph;
  if (mode == "bad") {
    int c = atoi(argv[2]);
    switch (c) {  // test/grankTest.cc:20-29, test/grankMultiThreadTest.cc:22-32
      case 0: ppr::grank(graph, 0, 3, 42, 0.5, 0.0001); break;
      case 1: ppr::grank(graph, 2, 0, 32, 0.85, 0.0001); break;
      case 2: ppr::grank(graph, 2, 1, 10, 0.5, 0.0001); break;
      case 3: ppr::grank(graph, 2, 2, 0, 0.5, 0.0001); break;
      case 4: ppr::grank(graph, 2, 2, 10, 1.5, 0.0001); break;
      case 5: ppr::grank(graph, 2, 2, 10, -1.5, 0.0001); break;
      case 6: ppr::grankMulti(graph, 2, 2, 10, 0.5, 0.0001, 0); break;
    }
    return 0;
  }
  if (mode == "mcbad") {
    int c = atoi(argv[2]);
    switch (c) {  // test/mccompletepathv2Test.cc:20-29
      case 0: ppr::mccompletepathv2(graph, 0, 3, 42, 0.5); break;
      case 1: ppr::mccompletepathv2(graph, 2, 0, 32, 0.85); break;
      case 2: ppr::mccompletepathv2(graph, 2, 1, 10, 0.5); break;
      case 3: ppr::mccompletepathv2(graph, 2, 2, 0, 0.5); break;
      case 4: ppr::mccompletepathv2(graph, 2, 2, 10, 1.5); break;
      case 5: ppr::mccompletepathv2(graph, 2, 2, 10, -1.5); break;
    }
    return 0;
  }
  if (mode == "mcknown") {
    int bad = 0;
    bad += check(ppr::mccompletepathv2(graph, 10, 30, 100, 0.85).empty(), "mc empty");
    for (int i = 0; i < 10; i++) graph[i];
    auto r = ppr::mccompletepathv2(graph, 10, 30, 100, 0.85);  // :38-50
    for (int i = 0; i < 10; i++) bad += check(r[i].size() == 1 && fabs(r[i][i] - 1.0) < 1e-4, "mc no edges");
    unordered_map<int, vector<int>> star;
    for (int i = 0; i < 6; i++) star[i];
    for (int i = 1; i < 6; i++) star[i].push_back(0);
    r = ppr::mccompletepathv2(star, 10, 30, 100, 0.85);  // :154-172
    bad += check(r[0].size() == 1 && fabs(r[0][0] - 1.0) < 1e-4, "mc star centre");
    for (int i = 1; i < 6; i++) bad += check(r[i].size() == 2 && fabs(r[i][0] - 0.85) < 1e-4, "mc star leaf");
    unordered_map<int, vector<int>> rev;
    for (int i = 0; i < 6; i++) rev[i];
    for (int i = 1; i < 6; i++) rev[0].push_back(i);
    r = ppr::mccompletepathv2(rev, 10, 30, 100, 0.85);  // :184-205
    bad += check(r[0].size() == 6 && fabs(r[0][0] - 1.0) < 1e-4, "mc reversed star centre");
    for (int i = 1; i < 6; i++)
      bad += check(r[i].size() == 1 && fabs(r[0][i] - 0.85 / 5) < 1e-4, "mc reversed star leaf");
    unordered_map<int, vector<int>> ring;
    for (int i = 0; i < 100; i++) ring[i];
    for (int i = 0; i < 99; i++) ring[i].push_back(i + 1);
    ring[99].push_back(0);
    r = ppr::mccompletepathv2(ring, 10, 20, 100, 0.85);  // :221-255
    for (int i = 0; i < 100; i++) {
      bad += check(r[i].size() == 10, "mc ring size");
      for (int u = 0; u < 9; u++) bad += check(r[i][(i + u) % 100] >= r[i][(i + u + 1) % 100], "mc ring order");
    }
    return bad ? 1 : 0;
  }
  if (mode == "e2e") {
    const int scale = atoi(argv[2]);
    const int iters = argc > 3 ? atoi(argv[3]) : 10;
    const int64_t n = 1LL << scale;
    std::vector<int64_t> rp(n + 1);
    const int64_t m = ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, 42, rp.data(), nullptr, 0);
    std::vector<int32_t> col(m);
    ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, 42, rp.data(), col.data(), m);
    auto t0 = std::chrono::steady_clock::now();
    for (int64_t v = 0; v < n; v++) {
      std::vector<int>& s = graph[(int)v];
      s.assign(col.begin() + rp[v], col.begin() + rp[v + 1]);
    }
    auto t1 = std::chrono::steady_clock::now();
    auto res = ppr::grank(graph, 64, 128, iters, 0.85, -1.0);
    auto t2 = std::chrono::steady_clock::now();
    size_t entries = 0;
    for (auto& kv : res) entries += kv.second.size();
    printf("{\"nodes\": %lld, \"edges\": %lld, \"rows\": %zu, \"entries\": %zu, \"build_s\": %.3f, \"total_s\": %.3f}\n",
           (long long)n, (long long)m, res.size(), entries,
           std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
    return 0;
  }
  if (mode == "e2echeck") {  // e2echeck <scale> <iters> <stride>: the materialised maps == the device rows
    const int scale = atoi(argv[2]);
    const int iters = atoi(argv[3]);
    const int64_t stride = atoll(argv[4]);
    const int64_t n = 1LL << scale;
    std::vector<int64_t> rp(n + 1);
    const int64_t m = ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, 42, rp.data(), nullptr, 0);
    std::vector<int32_t> col(m);
    ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, 42, rp.data(), col.data(), m);
    for (int64_t v = 0; v < n; v++) graph[(int)v].assign(col.begin() + rp[v], col.begin() + rp[v + 1]);
    const size_t K = 64, L = 128;
    auto res = ppr::grank(graph, K, L, iters, 0.85, -1.0);
    // the same call through the C ABI on the same flattening (dense id = graph iteration order)
    ppr::hipdetail::Flat<int> f = ppr::hipdetail::flatten(graph, ppr::hipdetail::host_threads());
    ppr_csr g{(int64_t)f.keys.size(), f.rp.data(), f.col.data()};
    std::vector<int32_t> ids(f.keys.size() * K), len(f.keys.size());
    std::vector<double> sc(f.keys.size() * K);
    if (ppr_grank_csr(&g, nullptr, (uint32_t)K, (uint32_t)L, (uint32_t)iters, 0.85, -1.0, nullptr, ids.data(), sc.data(),
                      len.data(), nullptr) != PPR_OK)
      return 3;
    int bad = check(res.size() == f.keys.size(), "one result row per source");
    int64_t rows = 0, entries = 0;
    for (size_t v = 0; v < f.keys.size(); v += (size_t)stride) {
      const auto it = res.find(*f.keys[v]);
      if (it == res.end()) { bad += check(false, "row present"); continue; }
      bad += check(it->second.size() == (size_t)len[v], "row length");
      for (int32_t i = 0; i < len[v]; i++) {
        const auto e = it->second.find(*f.keys[(size_t)ids[v * K + i]]);
        bad += check(e != it->second.end() && e->second == sc[v * K + i], "entry key and score (bit for bit)");
      }
      rows++;
      entries += len[v];
    }
    printf("{\"rows_checked\": %lld, \"entries_checked\": %lld, \"bad\": %d}\n", (long long)rows, (long long)entries, bad);
    return bad ? 1 : 0;
  }
  if (mode == "multieq") {
    const int scale = atoi(argv[2]);
    const int iters = atoi(argv[3]);
    const int64_t n = 1LL << scale;
    std::vector<int64_t> rp(n + 1);
    const int64_t m = ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, 7, rp.data(), nullptr, 0);
    std::vector<int32_t> col(m);
    ppr_rmat_generate(scale, 16, 0.57, 0.19, 0.19, 7, rp.data(), col.data(), m);
    for (int64_t v = 0; v < n; v++) graph[(int)v].assign(col.begin() + rp[v], col.begin() + rp[v + 1]);
    auto a = ppr::grankMulti(graph, 32, 64, iters, 0.85, 1e-4, 1);
    auto b = ppr::grankMulti(graph, 32, 64, iters, 0.85, 1e-4, 8);
    auto c = ppr::grank(graph, 32, 64, iters, 0.85, 1e-4);
    int bad = check(a == b, "grankMulti 1 thread == 8 threads") + check(a == c, "grankMulti == grank");
    return bad ? 1 : 0;
  }
  if (mode == "order") {
    const size_t n = (size_t)atoll(argv[2]);
    uint64_t s = (uint64_t)atoll(argv[3]) * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    int bad = 0;
    auto same = [&](int r, const char*) { bad += r; };
    unordered_map<int, vector<int>> gi;
    for (size_t i = 0; i < n; i++) gi[(int)(rnd() % (4 * n))].push_back((int)i);
    same(same_order(gi, "int keys"), "");
    for (size_t i = 0; i < n / 3; i++) gi.erase((int)(rnd() % (4 * n)));
    same(same_order(gi, "int keys after erasures"), "");
    gi.rehash(gi.bucket_count() * 4);
    same(same_order(gi, "int keys after a rehash"), "");
    gi.max_load_factor(4.0f);
    gi.rehash(1);
    same(same_order(gi, "int keys, load factor 4"), "");
    unordered_map<string, vector<string>> gs;
    for (size_t i = 0; i < n / 2; i++) gs["k" + to_string(rnd() % (2 * n))].push_back("x");
    same(same_order(gs, "string keys"), "");
    return bad ? 1 : 0;
  }
  if (mode == "empty") {
    auto res = ppr::grank(graph, 10, 30, 100, 0.85, 0.0001);
    return res.empty() ? 0 : 1;
  }
  if (mode == "ring") {  // README.md "GRank" example
    for (int i = 0; i < 100; i++) graph[i].push_back((i + 1) % 100);
    auto res = ppr::grank(graph, 50, 100, 30, 0.85, 0.001);
    for (auto& kv : res)
      for (auto& e : kv.second) printf("%d %d %.17g\n", kv.first, e.first, e.second);
    return 0;
  }
  if (mode == "known") {
    int bad = 0;
    for (int i = 0; i < 10; i++) graph[i];
    auto r = ppr::grank(graph, 10, 30, 100, 0.85, 0.0001);  // no edges (grankTest.cc:38-50)
    for (int i = 0; i < 10; i++) bad += check(r[i].size() == 1 && fabs(r[i][i] - 0.15) < 1e-4, "no edges");
    unordered_map<int, vector<int>> one;
    one[0].push_back(0);
    r = ppr::grank(one, 10, 30, 100, 0.85, 0.0001);  // self loop (:70-84)
    bad += check(fabs(r[0][0] - 1.0) < 1e-4, "self loop");
    unordered_map<int, vector<int>> star;
    for (int i = 0; i < 6; i++) star[i];
    for (int i = 1; i < 6; i++) star[i].push_back(0);
    r = ppr::grankMulti(star, 10, 30, 100, 0.85, 0.0001, 4);  // star (:154-182)
    bad += check(r[0].size() == 1 && fabs(r[0][0] - 0.15) < 1e-4, "star centre");
    for (int i = 1; i < 6; i++) bad += check(r[i].size() == 2 && fabs(r[i][0] - 0.15 * 0.85) < 1e-4, "star leaf");
    unordered_map<int, vector<int>> ring;
    for (int i = 0; i < 100; i++) ring[i];
    for (int i = 0; i < 99; i++) ring[i].push_back(i + 1);
    ring[99].push_back(0);
    r = ppr::grank(ring, 10, 10, 100, 0.85, 0.0001);  // testNodesGreaterThanK (:184-240)
    for (int i = 0; i < 100; i++) {
      bad += check(r[i].size() == 10, "ring size");
      for (int u = 0; u < 9; u++) bad += check(r[i][(i + u) % 100] > r[i][(i + u + 1) % 100], "ring order");
    }
    return bad ? 1 : 0;
  }
  return 2;
}
