// ppr/importGraph.h -- the reference CLI's edge-list importer (src/main.cc:78-112), as a header
// (SURVEY.md s8f f4). One "a,b" edge per line; '\r' / '\n' stripped; the target is inserted
// into the map first (a node without out-edges still appears); a repeated edge is kept once.
// Returns the same std::unordered_map<int, std::vector<int>> built by the same sequence of
// insertions as the reference, so it iterates in the reference's order (which fixes GRank's
// partitions and MCCompletePathV2's ties). Prints "nodes: N edges: M" like the reference.
// ppr_import_edge_csv (include/ppr_hip.h) is the same importer behind the C ABI.
#ifndef PPR_HIP_DROPIN_IMPORTGRAPH_H
#define PPR_HIP_DROPIN_IMPORTGRAPH_H

#include <algorithm>
#include <fstream>
#include <iostream>
#include <string>
#include <unordered_map>
#include <vector>

namespace ppr {

inline std::unordered_map<int, std::vector<int>> importGraph(const std::string& fname, bool verbose = true) {
  size_t edges_kept = 0;
  std::ifstream in(fname, std::ifstream::in);
  std::unordered_map<int, std::vector<int>> graph;
  std::unordered_map<int, std::unordered_map<int, bool>> seen;
  std::string line;
  while (std::getline(in, line)) {
    const size_t pos = line.find(',');
    line.erase(std::remove(line.begin(), line.end(), '\r'), line.end());
    line.erase(std::remove(line.begin(), line.end(), '\n'), line.end());
    const int a = std::stoi(line.substr(0, pos));
    const int b = std::stoi(line.substr(pos + 1));
    graph[b];
    if (!seen[a][b]) {
      seen[a][b] = true;
      graph[a].push_back(b);
      edges_kept++;
    }
  }
  if (verbose) std::cout << "nodes: " << graph.size() << " edges: " << edges_kept << std::endl;
  return graph;
}

}  // namespace ppr

#endif  // PPR_HIP_DROPIN_IMPORTGRAPH_H
