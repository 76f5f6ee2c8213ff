// oracle/ref_driver.cc -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
//
// A thin driver compiled against the UNMODIFIED reference headers where they lie
// (/root/reference/header-only, /root/reference/include) by oracle/Makefile. Output goes only
// to oracle/_ref/ (git-ignored). It is used to
//   (1) generate the golden vectors under tests/golden/ (tools/make_golden.py), and
//   (2) time the reference's own per-source merge (grankMultiInternal::combineMaps,
//       header-only/grankMulti.h:230-268) on a bounded, stratified sample of sources for
//       bench.py's cpu_baseline (mode bench_combine).
//
// No reference source is copied here: the algorithms are #included from the reference tree.
//
// Binary graph file (little endian), written by tools / bench:
//   int64 n, int64 m, int32 keys[n], int64 row_ptr[n+1], int32 succ[m]   (succ holds KEY values)
// The driver inserts keys[i] in order, then pushes successors in CSR order, so the
// unordered_map is built deterministically; its iteration order is then RECORDED in the output
// (it defines the dense-id order used by the MI355X path, see DESIGN.md "dense ids").
//
// Output file of the algorithm modes:
//   int64 n, int32 order[n]                  -- graph iteration order (keys)
//   int64 m, int64 row_ptr[n+1], int32 col[m] -- CSR in that order, col = dense successor index
//   uint8 part[n]                            -- 0 = partitions.first of findPartitions
//   int32 exec_order[n] (dense)               -- MCCompletePathV2 executionOrder (mc mode only, else -1s)
//   double elapsed_ms
//   per dense node: int32 cnt, cnt x {int32 dense_key, double score}
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>
#include <algorithm>

#include <grank.h>          // /root/reference/header-only/grank.h
#include <grankMulti.h>     // /root/reference/header-only/grankMulti.h
#include <mccompletepathv2.h>  // /root/reference/header-only/mccompletepathv2.h
#include <internal/pprSingleSource.h>  // /root/reference/include/internal/pprSingleSource.h

typedef std::unordered_map<int, std::vector<int>> Graph;
typedef std::unordered_map<int, std::unordered_map<int, double>> Result;

static void die(const char* m) { fprintf(stderr, "ref_driver: %s\n", m); exit(2); }

static Graph read_graph_bin(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) die("cannot open graph");
  int64_t n, m;
  if (fread(&n, 8, 1, f) != 1 || fread(&m, 8, 1, f) != 1) die("short read");
  std::vector<int32_t> keys(n);
  std::vector<int64_t> rp(n + 1);
  std::vector<int32_t> succ(m);
  if (n && fread(keys.data(), 4, n, f) != (size_t)n) die("short read keys");
  if (fread(rp.data(), 8, n + 1, f) != (size_t)(n + 1)) die("short read rp");
  if (m && fread(succ.data(), 4, m, f) != (size_t)m) die("short read succ");
  fclose(f);
  Graph g;
  for (int64_t i = 0; i < n; i++) g[keys[i]];
  for (int64_t i = 0; i < n; i++) {
    std::vector<int>& s = g[keys[i]];
    for (int64_t e = rp[i]; e < rp[i + 1]; e++) s.push_back(succ[e]);
  }
  return g;
}

// Edge-list CSV ingest with the same observable behaviour as src/main.cc:78-112
// (target inserted first, duplicate edges skipped, first-occurrence order kept).
static Graph read_graph_csv(const char* path) {
  std::ifstream in(path);
  if (!in) die("cannot open csv");
  Graph g;
  std::unordered_map<int, std::unordered_map<int, bool>> seen;
  std::string line;
  while (std::getline(in, line)) {
    line.erase(std::remove(line.begin(), line.end(), '\r'), line.end());
    size_t pos = line.find(',');
    if (pos == std::string::npos) continue;
    int a = std::stoi(line.substr(0, pos));
    int b = std::stoi(line.substr(pos + 1));
    g[b];
    if (!seen[a][b]) { seen[a][b] = true; g[a].push_back(b); }
  }
  return g;
}

struct Dense {
  std::vector<int32_t> order;
  std::unordered_map<int, int32_t> idx;
  std::vector<int64_t> rp;
  std::vector<int32_t> col;
};

static Dense densify(const Graph& g) {
  Dense d;
  for (const auto& kv : g) { d.idx[kv.first] = (int32_t)d.order.size(); d.order.push_back(kv.first); }
  d.rp.push_back(0);
  for (int32_t k : d.order) {
    for (int s : g.find(k)->second) d.col.push_back(d.idx.at(s));
    d.rp.push_back((int64_t)d.col.size());
  }
  return d;
}

static void write_out(const char* path, const Graph& g, const Dense& d, const Result& r,
                      const std::vector<int32_t>& exec_order, double ms) {
  FILE* f = fopen(path, "wb");
  if (!f) die("cannot open out");
  int64_t n = (int64_t)d.order.size(), m = (int64_t)d.col.size();
  fwrite(&n, 8, 1, f);
  fwrite(d.order.data(), 4, n, f);
  fwrite(&m, 8, 1, f);
  fwrite(d.rp.data(), 8, n + 1, f);
  fwrite(d.col.data(), 4, m, f);
  auto parts = ppr::grankMultiInternal::findPartitions<int>(g);
  std::vector<uint8_t> part(n, 1);
  for (int k : parts.first) part[d.idx.at(k)] = 0;
  fwrite(part.data(), 1, n, f);
  std::vector<int32_t> eo(n, -1);
  for (size_t i = 0; i < exec_order.size() && i < (size_t)n; i++) eo[i] = exec_order[i];
  fwrite(eo.data(), 4, n, f);
  fwrite(&ms, 8, 1, f);
  for (int32_t k : d.order) {
    auto it = r.find(k);
    int32_t cnt = it == r.end() ? 0 : (int32_t)it->second.size();
    fwrite(&cnt, 4, 1, f);
    if (!cnt) continue;
    for (const auto& kv : it->second) {
      int32_t dk = d.idx.at(kv.first);
      fwrite(&dk, 4, 1, f);
      fwrite(&kv.second, 8, 1, f);
    }
  }
  fclose(f);
}

// bench mode: time the reference's per-source merge, grankMultiInternal::combineMaps
// (header-only/grankMulti.h:230-268), over stratified samples of sources, with the reference's
// own containers, split over nThreads exactly as grankMulti does (:379-396).
// sample file (dense ids, written by bench.py):
//   int32 L, int64 s, int32 src[s], int64 rp[s+1], int32 succ[rp[s]],
//   int64 nb, nb x { int32 id, int32 len, int32 ids[len], double sc[len] }   (baskets of every
//   sampled source and of every successor), int64 nstrata, int64 off[nstrata+1]
// prints one JSON line per stratum: {"stratum": h, "sources": k, "ms": t}
template <class T> static void rd(FILE* f, T* p, size_t n) {
  if (n && fread(p, sizeof(T), n, f) != n) die("short sample file");
}
static int bench_combine(const char* sample_path, int nthreads, double damping) {
  FILE* f = fopen(sample_path, "rb");
  if (!f) die("cannot open sample");
  int32_t L; int64_t s;
  rd(f, &L, 1); rd(f, &s, 1);
  std::vector<int32_t> src(s);
  std::vector<int64_t> rp(s + 1);
  rd(f, src.data(), s); rd(f, rp.data(), s + 1);
  std::vector<int32_t> succ(rp[s]);
  rd(f, succ.data(), rp[s]);
  Graph g;
  for (int64_t i = 0; i < s; i++) g[src[i]] = std::vector<int>(succ.begin() + rp[i], succ.begin() + rp[i + 1]);
  int64_t nb; rd(f, &nb, 1);
  Result scores, next;
  scores.reserve(nb); next.reserve(s);
  std::vector<int32_t> ids; std::vector<double> sc;
  for (int64_t b = 0; b < nb; b++) {
    int32_t id, len; rd(f, &id, 1); rd(f, &len, 1);
    ids.resize(len); sc.resize(len);
    rd(f, ids.data(), len); rd(f, sc.data(), len);
    auto& mp = scores[id];
    mp.reserve(len);
    for (int32_t i = 0; i < len; i++) mp[ids[i]] = sc[i];
  }
  for (int64_t i = 0; i < s; i++) next[src[i]];
  int64_t ns; rd(f, &ns, 1);
  std::vector<int64_t> off(ns + 1);
  rd(f, off.data(), ns + 1);
  fclose(f);
  for (int64_t h = 0; h < ns; h++) {
    std::vector<double> maxDiffs(nthreads, 0);
    std::vector<std::thread> th;
    auto b0 = src.begin() + off[h], e0 = src.begin() + off[h + 1];
    size_t chunk = (size_t)(off[h + 1] - off[h]) / nthreads;
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < nthreads; t++) {
      auto b = b0 + chunk * t;
      auto e = (t == nthreads - 1) ? e0 : b0 + chunk * (t + 1);
      th.emplace_back(ppr::grankMultiInternal::combineMaps<int, std::vector<int32_t>::iterator>,
                      b, e, std::cref(g), std::cref(scores), std::ref(next), std::ref(maxDiffs[t]),
                      (size_t)L, damping);
    }
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    printf("{\"stratum\": %lld, \"sources\": %lld, \"ms\": %.3f, \"threads\": %d}\n", (long long)h,
           (long long)(off[h + 1] - off[h]), ms, nthreads);
    fflush(stdout);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) die("usage: ref_driver MODE ...");
  std::string mode = argv[1];
  if (mode == "bench_combine") {
    if (argc < 5) die("bench_combine sample nthreads damping");
    return bench_combine(argv[2], atoi(argv[3]), atof(argv[4]));
  }
  // algorithm modes: MODE in.{bin|csv} out.bin K L iters damping tol threads
  if (argc < 10) die("MODE in out K L iters damping tol threads");
  const char* in = argv[2];
  const char* out = argv[3];
  size_t K = strtoull(argv[4], 0, 10), L = strtoull(argv[5], 0, 10), it = strtoull(argv[6], 0, 10);
  double d = atof(argv[7]), tol = atof(argv[8]);
  size_t nth = strtoull(argv[9], 0, 10);
  std::string ip = in;
  Graph g = (ip.size() > 4 && ip.substr(ip.size() - 4) == ".csv") || (ip.size() > 4 && ip.substr(ip.size() - 4) == ".txt")
                ? read_graph_csv(in) : read_graph_bin(in);
  Dense dn = densify(g);
  Result r;
  std::vector<int32_t> eo;
  auto t0 = std::chrono::steady_clock::now();
  if (mode == "grank") r = ppr::grank(g, K, L, it, d, tol);
  else if (mode == "grankmulti") r = ppr::grankMulti(g, K, L, it, d, tol, nth);
  else if (mode == "mc") {
    r = ppr::mccompletepathv2(g, K, L, it, d);
  } else if (mode == "pprss_list") {
    // exact single-source PPR for the dense sources listed (int32) in file argv[10]
    if (argc < 11) die("pprss_list needs a list file");
    FILE* lf = fopen(argv[10], "rb");
    if (!lf) die("cannot open list");
    int32_t x;
    while (fread(&x, 4, 1, lf) == 1)
      r[dn.order[x]] = ppr::pprInternal::pprSingleSource(g, it, d, tol, dn.order[x]);
    fclose(lf);
  } else if (mode == "pprss") {
    // exact single-source PPR (include/internal/pprSingleSource.h:28-75) for the first K
    // dense sources listed in iteration order starting at dense index L (quality oracle);
    // iters / damping / tol are passed through.
    for (size_t i = L; i < L + K && i < dn.order.size(); i++)
      r[dn.order[i]] = ppr::pprInternal::pprSingleSource(g, it, d, tol, dn.order[i]);
  } else die("unknown mode");
  auto t1 = std::chrono::steady_clock::now();
  if (mode == "mc") {
    auto o = ppr::mccompletepathv2Internal::executionOrder(g);
    for (int k : o) eo.push_back(dn.idx.at(k));
  }
  double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  write_out(out, g, dn, r, eo, ms);
  fprintf(stderr, "ref_driver %s: n=%zu m=%zu %.1f ms\n", mode.c_str(), dn.order.size(), dn.col.size(), ms);
  return 0;
}
