// tools/lds_atomic_bench.hip -- LDS throughput of the exact-sum table operations on gfx950
// (design input for merge_xs.h): 16-wave workgroups, one per CU x4, an 8192-slot table of two u64
// words per slot, random slots (optionally a fraction of lanes on one hot slot), per variant:
//   0 ds_read_b64            1 ds_add_u64 (no return)     2 ds_add_rtn_u64
//   3 ds_add_rtn_u64 + dependent ds_add_u64 (the current xt_add)   4 two ds_add_u64
//   5 ds_read_b64 + ds_add_rtn_u64 + ds_add_u64 (probe + add)       6 ds_add_u32 (no return)
// hipcc --offload-arch=gfx950 -O3 -o tools/lds_atomic_bench tools/lds_atomic_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int V>
__global__ void __launch_bounds__(1024) k_bench(int iters, int hot_pct, unsigned long long* out) {
  __shared__ unsigned long long t0[8192];
  __shared__ unsigned long long t1[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) { t0[i] = 0; t1[i] = 0; }
  __syncthreads();
  unsigned long long acc = 0;
  uint32_t st = mix(blockIdx.x * 1024u + threadIdx.x);
  for (int it = 0; it < iters; it++) {
    st = mix(st + 0x9e3779b9u);
    const bool hot = (st >> 25) % 100u < (uint32_t)hot_pct;
    const uint32_t h = hot ? 0u : (st & 8191u);
    const unsigned long long x = st | 1ull << 40;
    if (V == 0) acc += t0[h];
    if (V == 1) atomicAdd(&t0[h], x);
    if (V == 2) acc += atomicAdd(&t0[h], x);
    if (V == 3) { const unsigned long long o = atomicAdd(&t0[h], x); if (o + x < o) atomicAdd(&t1[h], 1ull); acc += o; }
    if (V == 4) { atomicAdd(&t0[h], x & 0xffffffffull); atomicAdd(&t1[h], x >> 32); }
    if (V == 5) {
      const unsigned long long k = t1[h];
      const uint32_t hh = (k >> 32) == 7u ? (h + 1u) & 8191u : h;
      const unsigned long long o = atomicAdd(&t0[hh], x);
      atomicAdd(&t1[hh], (o + x < o) ? 2ull : 1ull);
    }
    if (V == 6) atomicAdd(reinterpret_cast<uint32_t*>(t0) + h, (uint32_t)x);
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, acc + t0[5] + t1[7]);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  unsigned long long* d;
  hipMalloc(&d, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = 256 * 4;
  for (int hot : {0, 30}) {
    for (int v = 0; v <= 6; v++) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(a);
        switch (v) {
          case 0: hipLaunchKernelGGL(k_bench<0>, dim3(grid), dim3(1024), 0, 0, iters, hot, d); break;
          case 1: hipLaunchKernelGGL(k_bench<1>, dim3(grid), dim3(1024), 0, 0, iters, hot, d); break;
          case 2: hipLaunchKernelGGL(k_bench<2>, dim3(grid), dim3(1024), 0, 0, iters, hot, d); break;
          case 3: hipLaunchKernelGGL(k_bench<3>, dim3(grid), dim3(1024), 0, 0, iters, hot, d); break;
          case 4: hipLaunchKernelGGL(k_bench<4>, dim3(grid), dim3(1024), 0, 0, iters, hot, d); break;
          case 5: hipLaunchKernelGGL(k_bench<5>, dim3(grid), dim3(1024), 0, 0, iters, hot, d); break;
          default: hipLaunchKernelGGL(k_bench<6>, dim3(grid), dim3(1024), 0, 0, iters, hot, d); break;
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      const double ops = (double)grid * 1024 * iters;
      // per CU: lane-ops per cycle at 2.4 GHz
      printf("hot %2d%% variant %d: %.3f ms, %.1f G lane-ops/s, %.2f lane-ops per CU-cycle\n", hot, v, best,
             ops / best / 1e6, ops / (best * 1e-3) / 256 / 2.4e9);
    }
  }
  hipFree(d);
  return 0;
}
