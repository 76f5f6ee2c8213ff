// partition.hip -- GRank's BFS 2-colouring (findPartitions, include/internal/pprInternal.h:29-99)
// on the device, for plan creation when the caller passes no partitions (the drop-in templates).
//
// The reference's sequential BFS gives every node the parity of its undirected BFS distance from
// the first node (in graph order = dense id order) of its weakly connected component
// (host_graph.cpp ppr_find_partitions_csr restates why). Both parts are order-free, so:
//   components  min-label propagation over the undirected edges with pointer jumping: labels only
//               decrease, and once no edge joins two labels every node holds the smallest id of
//               its component -- its BFS root
//   depths      level-synchronous BFS from every root at once over the undirected graph, with the
//               out-edges only: a level first claims the unvisited successors of its frontier
//               (top-down), then every unvisited node with a successor in the frontier (bottom-up:
//               a predecessor of it)
// Same result as the host BFS (tests: test_gpu_partitions_match_host). Graphs whose propagation or
// BFS needs many rounds (long paths: diameter in the thousands) return PPR_ERR_RANGE and the caller
// falls back to the host BFS, which switches to predecessor lists on such graphs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/ppr_hip.h"

namespace pprpart {

__global__ void k_cc_init(int32_t* lab, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) lab[v] = (int32_t)v;
}

// one thread per edge (u -> v): both ends take the smaller label
__global__ void k_cc_hook(const int64_t* rp, const int32_t* col, const int32_t* src, int64_t m, int32_t* lab,
                          int32_t* changed) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m) return;
  const int32_t u = src[e], v = col[e];
  const int32_t lu = lab[u], lv = lab[v];
  if (lu == lv) return;
  const int32_t lo = lu < lv ? lu : lv;
  if (lu != lo) atomicMin(&lab[u], lo);
  if (lv != lo) atomicMin(&lab[v], lo);
  // (the label nodes too: a root relabelled pulls its whole tree along at the next jump)
  atomicMin(&lab[lu > lv ? lu : lv], lo);
  *changed = 1;
}

// pointer jumping: lab[v] <- lab[lab[v]] until it stands still
__global__ void k_cc_jump(int32_t* lab, int64_t n) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  int32_t l = lab[v];
  for (int k = 0; k < 64; k++) {
    const int32_t l2 = lab[l];
    if (l2 == l) break;
    l = l2;
  }
  lab[v] = l;
}

// source node of every edge (for the one-thread-per-edge passes): one wave per node, grid-stride
// (a wave per node in one grid passed the 2^32 work-item limit at n >= 2^26)
__global__ void k_edge_src(const int64_t* rp, int64_t n, int32_t* src) {
  const int64_t W = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t v = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); v < n; v += W)
    for (int64_t e = rp[v] + (threadIdx.x & 63); e < rp[v + 1]; e += 64) src[e] = (int32_t)v;
}

__global__ void k_bfs_roots(const int32_t* lab, int64_t n, int32_t* depth) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n) depth[v] = lab[v] == (int32_t)v ? 0 : -1;
}

// top-down: one thread per edge whose source sits at depth d claims an unvisited target
__global__ void k_bfs_down(const int32_t* src, const int32_t* col, int64_t m, int32_t* depth, int d,
                           int32_t* grew) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m) return;
  if (depth[src[e]] != d) return;
  const int32_t v = col[e];
  if (depth[v] == -1 && atomicCAS(&depth[v], -1, d + 1) == -1) *grew = 1;
}

// bottom-up: an unvisited node with a successor at depth d joins level d + 1 (its own entry only)
__global__ void k_bfs_up(const int64_t* rp, const int32_t* col, int64_t n, int32_t* depth, int d, int32_t* grew) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  if (__hip_atomic_load(&depth[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != -1) return;
  for (int64_t e = rp[v]; e < rp[v + 1]; e++)
    if (__hip_atomic_load(&depth[col[e]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == d) {
      atomicCAS(&depth[v], -1, d + 1);
      *grew = 1;
      return;
    }
}

__global__ void k_bfs_parity(const int32_t* depth, int64_t n, uint8_t* part, int32_t* bad) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int32_t d = depth[v];
  if (d < 0) *bad = 1;
  part[v] = (uint8_t)(d & 1);
}

// successors' partition bits into the CSR column words (the plan's colx: bit 31 = part of col)
__global__ void k_col_mark(int32_t* col, int64_t m, const uint8_t* part) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < m) col[e] |= part[col[e]] ? (int32_t)0x80000000 : 0;
}

#define PP_OK(x)                                 \
  do {                                           \
    if ((x) != hipSuccess) return PPR_ERR_HIP;   \
  } while (0)

// The two passes on graph arrays already in HBM (d_col raw ids), on stream st: d_part[n] and the
// host copy h_part[n]; mark: then OR the partition bits into d_col. Scratch: d_src[m], d_lab[n],
// d_depth[n], d_flag[2]. PPR_ERR_RANGE leaves d_col untouched.
int partitions_core(const int64_t* d_rp, int32_t* d_col, int64_t n, int64_t m, uint8_t* d_part, uint8_t* h_part,
                    bool mark, int32_t* d_src, int32_t* d_lab, int32_t* d_depth, int32_t* d_flag, hipStream_t st) {
  constexpr int CC_ROUNDS = 64, BFS_LEVELS = 512;
  // one thread per node / edge in the passes below: past 2^32 work items the launches would fail,
  // so such graphs take the host BFS (PPR_ERR_RANGE, like a graph that needs too many rounds)
  if (n > (int64_t)UINT32_MAX - 256 || m > (int64_t)UINT32_MAX - 256) return PPR_ERR_RANGE;
  const unsigned bn = (unsigned)((n + 255) / 256), bm = (unsigned)((m + 255) / 256);
  int32_t h[2] = {0, 0};
  hipLaunchKernelGGL(k_edge_src, dim3((unsigned)std::min<int64_t>((n + 3) / 4, 1 << 16)), dim3(256), 0, st, d_rp, n,
                     d_src);
  hipLaunchKernelGGL(k_cc_init, dim3(bn), dim3(256), 0, st, d_lab, n);
  PP_OK(hipGetLastError());
  {
    int r = 0;
    for (; r < CC_ROUNDS; r++) {
      PP_OK(hipMemsetAsync(d_flag, 0, 4, st));
      if (m) hipLaunchKernelGGL(k_cc_hook, dim3(bm), dim3(256), 0, st, d_rp, d_col, d_src, m, d_lab, d_flag);
      hipLaunchKernelGGL(k_cc_jump, dim3(bn), dim3(256), 0, st, d_lab, n);
      PP_OK(hipGetLastError());
      PP_OK(hipMemcpyAsync(h, d_flag, 4, hipMemcpyDeviceToHost, st));
      PP_OK(hipStreamSynchronize(st));
      if (!h[0]) break;
    }
    if (r == CC_ROUNDS) return PPR_ERR_RANGE;
  }
  hipLaunchKernelGGL(k_bfs_roots, dim3(bn), dim3(256), 0, st, d_lab, n, d_depth);
  PP_OK(hipGetLastError());
  {
    int d = 0;
    for (; d < BFS_LEVELS; d++) {
      PP_OK(hipMemsetAsync(d_flag, 0, 4, st));
      if (m) hipLaunchKernelGGL(k_bfs_down, dim3(bm), dim3(256), 0, st, d_src, d_col, m, d_depth, d, d_flag);
      hipLaunchKernelGGL(k_bfs_up, dim3(bn), dim3(256), 0, st, d_rp, d_col, n, d_depth, d, d_flag);
      PP_OK(hipGetLastError());
      PP_OK(hipMemcpyAsync(h, d_flag, 4, hipMemcpyDeviceToHost, st));
      PP_OK(hipStreamSynchronize(st));
      if (!h[0]) break;
    }
    if (d == BFS_LEVELS) return PPR_ERR_RANGE;
  }
  PP_OK(hipMemsetAsync(d_flag, 0, 4, st));
  hipLaunchKernelGGL(k_bfs_parity, dim3(bn), dim3(256), 0, st, d_depth, n, d_part, d_flag);
  PP_OK(hipGetLastError());
  PP_OK(hipMemcpyAsync(h_part, d_part, (size_t)n, hipMemcpyDeviceToHost, st));
  PP_OK(hipMemcpyAsync(h, d_flag, 4, hipMemcpyDeviceToHost, st));
  PP_OK(hipStreamSynchronize(st));
  if (h[0]) return PPR_ERR_HIP;  // (a node no root reached: cannot happen)
  if (mark && m) {
    hipLaunchKernelGGL(k_col_mark, dim3(bm), dim3(256), 0, st, d_col, m, d_part);
    PP_OK(hipGetLastError());
    PP_OK(hipStreamSynchronize(st));
  }
  return PPR_OK;
}

}  // namespace pprpart

// part[n] of the CSR graph on device `device` (the current one when < 0). PPR_ERR_RANGE: the graph
// needs more rounds than partitions_core's caps (the caller takes the host BFS).
extern "C" int ppr_find_partitions_csr_device(const ppr_csr* g, uint8_t* part, int32_t device) {
  using namespace pprpart;
  if (!g || !part || g->n < 0) return PPR_ERR_ARG;
  const int64_t n = g->n;
  if (n == 0) return PPR_OK;
  if (n >= (1LL << 31) - 1) return PPR_ERR_RANGE;
  const int64_t m = g->row_ptr[n];
  int rc = PPR_ERR_HIP;
  int64_t* d_rp = nullptr;
  int32_t *d_col = nullptr, *d_src = nullptr, *d_lab = nullptr, *d_depth = nullptr, *d_flag = nullptr;
  uint8_t* d_part = nullptr;
  hipStream_t st = nullptr;
  if (device >= 0 && hipSetDevice(device) != hipSuccess) return PPR_ERR_HIP;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess && hipMalloc(&d_rp, 8 * (size_t)(n + 1)) == hipSuccess &&
      hipMalloc(&d_col, 4 * (size_t)(m > 0 ? m : 1)) == hipSuccess &&
      hipMalloc(&d_src, 4 * (size_t)(m > 0 ? m : 1)) == hipSuccess && hipMalloc(&d_lab, 4 * (size_t)n) == hipSuccess &&
      hipMalloc(&d_depth, 4 * (size_t)n) == hipSuccess && hipMalloc(&d_flag, 8) == hipSuccess &&
      hipMalloc(&d_part, (size_t)n) == hipSuccess &&
      hipMemcpyAsync(d_rp, g->row_ptr, 8 * (size_t)(n + 1), hipMemcpyHostToDevice, st) == hipSuccess &&
      (!m || hipMemcpyAsync(d_col, g->col, 4 * (size_t)m, hipMemcpyHostToDevice, st) == hipSuccess))
    rc = partitions_core(d_rp, d_col, n, m, d_part, part, false, d_src, d_lab, d_depth, d_flag, st);
  if (st) hipStreamSynchronize(st);
  hipFree(d_rp); hipFree(d_col); hipFree(d_src); hipFree(d_lab); hipFree(d_depth); hipFree(d_flag); hipFree(d_part);
  if (st) hipStreamDestroy(st);
  return rc;
}
