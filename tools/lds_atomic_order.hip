// Probe: do same-address LDS atomic adds with return inside one wave64 instruction hand out
// their old values in lane order? (lane i gets the number of lower lanes on the same address)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

__global__ void probe(unsigned long long* bad, unsigned long long* total, int trials) {
  __shared__ uint32_t cnt[4][512];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  unsigned long long nbad = 0, ntot = 0;
  for (int t = 0; t < trials; t++) {
    const uint32_t r = mix(blockIdx.x * 7919u + t * 104729u + wv * 31u);
    const int S = 1 << (r % 10);  // 1 .. 512 distinct addresses
    for (int i = l; i < 512; i += 64) cnt[wv][i] = (uint32_t)(t & 3);
    __builtin_amdgcn_wave_barrier();
    const uint32_t slot = mix(r ^ (l * 2654435761u)) % S;
    const uint32_t got = atomicAdd(&cnt[wv][slot], 1u) - (uint32_t)(t & 3);
    // expected: lanes below with the same slot
    uint32_t want = 0;
    for (int j = 0; j < l; j++) want += (__shfl(slot, j) == slot);
    // every lane executes the shfl loop body for all j < 64 to keep the shuffles uniform
    uint32_t w2 = 0;
    for (int j = 0; j < 64; j++) { const uint32_t sj = __shfl(slot, j); if (j < l && sj == slot) w2++; }
    nbad += (got != w2);
    ntot++;
    (void)want;
    __builtin_amdgcn_wave_barrier();
  }
  atomicAdd(bad, nbad);
  atomicAdd(total, ntot);
}

int main() {
  unsigned long long *d, h[2];
  hipMalloc(&d, 16);
  hipMemset(d, 0, 16);
  hipLaunchKernelGGL(probe, dim3(2048), dim3(256), 0, 0, d, d + 1, 400);
  hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("lane-order violations: %llu of %llu lane results\n", h[0], h[1]);
  return h[0] != 0;
}
