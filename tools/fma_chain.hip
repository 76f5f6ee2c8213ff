// Latency probe: cycles per dependent fp64 fma in one wave (the MC combine's hot-key chain floor),
// also fed from LDS 4 at a time (phase D of chunk_accumulate) and through readlane (register fold).
//   hipcc --offload-arch=gfx950 -O3 -o tools/fma_chain tools/fma_chain.hip && tools/fma_chain
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_chain(double* out, long long* cyc, int n, double f) {
  __shared__ double vals[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) vals[i] = 1e-9 * (i + 1);
  __syncthreads();
  double x = out[0], y = out[1], z = out[2];
  const double v = vals[threadIdx.x];
  long long t0 = clock64();
  for (int i = 0; i < n; i++) x = fma(v, f, x);  // register chain
  long long t1 = clock64();
  for (int i = 0; i < n; i += 4) {                // LDS-fed chain, 4 loads then 4 fmas
    const int j = i & 4095;
    const double a = vals[j], b = vals[j + 1], c = vals[j + 2], d = vals[j + 3];
    y = fma(a, f, y); y = fma(b, f, y); y = fma(c, f, y); y = fma(d, f, y);
  }
  long long t2 = clock64();
  for (int i = 0; i < n; i++) {                   // readlane-fed chain
    const unsigned long long bb = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)bb, i & 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(bb >> 32), i & 63);
    z = fma(__longlong_as_double((long long)(((unsigned long long)hi << 32) | lo)), f, z);
  }
  long long t3 = clock64();
  if (threadIdx.x == 0) { out[0] = x; out[1] = y; out[2] = z; cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; }
}

int main() {
  double* d;
  long long* c;
  hipMalloc(&d, 3 * sizeof(double));
  hipMalloc(&c, 3 * sizeof(long long));
  hipMemset(d, 0, 3 * sizeof(double));
  const int n = 1 << 16;
  for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, d, c, n, 1.0);
  long long h[3];
  hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  printf("cycles per dependent fp64 fma: registers %.2f  LDS-fed (4 loads, 4 fmas) %.2f  readlane-fed %.2f\n",
         (double)h[0] / n, (double)h[1] / n, (double)h[2] / n);
  return 0;
}
