// tools/pmc_calib.hip -- calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns of the basket merge (MI355X_MICROARCH.md "HBM": only 16-B/lane streaming reads and
// stores are calibrated there; every other width must be calibrated on a known byte count).
// Every kernel moves a known number of bytes from / to buffers far beyond the 256 MiB
// Infinity Cache:
//   cal_rows_i32   one wave per random 128-entry row of int32 ids    (basket ids in the walks)
//   cal_rows_f64   one wave per random 128-entry row of f64 scores   (basket scores in the walks)
//   cal_rec12_rd   streaming 12-B records, one per lane              (k_hub_bucket_w staging reads)
//   cal_rec12_wr   streaming 12-B records, one per lane              (store width of the scatter)
//   cal_rec12_sc   12-B records through a stable partition: tiles of 16384 records, 4096 buckets,
//                  4 records per (bucket, tile) run                  (k_hub_scatter's pattern)
// Prints {"kernel": known bytes} as JSON; tools/pmc_calib.py turns the counter runs into factors.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Rec { uint32_t w[3]; };

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ void __launch_bounds__(256) cal_rows_i32(const int32_t* ids, int64_t nrows, int64_t rows, int32_t* sink) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int l = threadIdx.x & 63;
  if (w >= rows) return;
  const int64_t r = mix((uint32_t)w * 2654435761u + 1u) % nrows;
  const int32_t a = ids[r * 128 + l], b = ids[r * 128 + 64 + l];
  if ((a ^ b) == 0x7fffffff) sink[w & 1023] = a;
}

__global__ void __launch_bounds__(256) cal_rows_f64(const double* sc, int64_t nrows, int64_t rows, double* sink) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int l = threadIdx.x & 63;
  if (w >= rows) return;
  const int64_t r = mix((uint32_t)w * 2654435761u + 7u) % nrows;
  const double a = sc[r * 128 + l], b = sc[r * 128 + 64 + l];
  if (a + b == 12345.678) sink[w & 1023] = a;
}

__global__ void __launch_bounds__(256) cal_rec12_rd(const Rec* st, int64_t n, uint32_t* sink) {
  uint32_t x = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const Rec r = st[i];
    x ^= r.w[0] ^ r.w[1] ^ r.w[2];
  }
  if (x == 0x9e3779b9u) sink[threadIdx.x] = x;
}

__global__ void __launch_bounds__(256) cal_rec12_wr(Rec* st, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    st[i] = Rec{{(uint32_t)i, (uint32_t)(i >> 32), 7u}};
}

// record q of tile t goes to bucket b = q % 4096, slot (q / 4096) of the (b, t) run; bucket b's
// region holds its runs of every tile in tile order (the stable partition's layout)
__global__ void __launch_bounds__(256) cal_rec12_sc(Rec* st, int64_t tiles) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;  // one wave per tile
  const int l = threadIdx.x & 63;
  if (w >= tiles) return;
  for (int q = l; q < 16384; q += 64) {
    const int64_t b = q & 4095, k = q >> 12;
    st[(b * tiles + w) * 4 + k] = Rec{{(uint32_t)q, (uint32_t)w, 1u}};
  }
}

int main() {
  const int64_t nrows = 8ll << 20;   // 8 Mi rows: 4 GiB of ids, 8 GiB of scores
  const int64_t rows = 4ll << 20;    // rows gathered per kernel
  const int64_t nrec = 512ll << 20;  // 6 GiB of 12-B records
  int32_t* ids; double* sc; Rec* st; int32_t* s32; double* s64; uint32_t* su;
  CK(hipMalloc(&ids, nrows * 128 * 4));
  CK(hipMalloc(&sc, nrows * 128 * 8));
  CK(hipMalloc(&st, nrec * 12));
  CK(hipMalloc(&s32, 4096 * 4)); CK(hipMalloc(&s64, 4096 * 8)); CK(hipMalloc(&su, 4096 * 4));
  CK(hipMemset(ids, 1, nrows * 128 * 4));
  CK(hipMemset(sc, 0, nrows * 128 * 8));
  CK(hipMemset(st, 2, nrec * 12));
  CK(hipDeviceSynchronize());
  const unsigned wb = (unsigned)((rows * 64 + 255) / 256);
  hipLaunchKernelGGL(cal_rows_i32, dim3(wb), dim3(256), 0, 0, ids, nrows, rows, s32);
  hipLaunchKernelGGL(cal_rows_f64, dim3(wb), dim3(256), 0, 0, sc, nrows, rows, s64);
  hipLaunchKernelGGL(cal_rec12_rd, dim3(8192), dim3(256), 0, 0, st, nrec, su);
  hipLaunchKernelGGL(cal_rec12_wr, dim3(8192), dim3(256), 0, 0, st, nrec);
  const int64_t tiles = nrec / 16384;
  hipLaunchKernelGGL(cal_rec12_sc, dim3((unsigned)((tiles * 64 + 255) / 256)), dim3(256), 0, 0, st, tiles);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("{\"cal_rows_i32\": {\"fetch\": %lld}, \"cal_rows_f64\": {\"fetch\": %lld}, "
         "\"cal_rec12_rd\": {\"fetch\": %lld}, \"cal_rec12_wr\": {\"write\": %lld}, \"cal_rec12_sc\": {\"write\": %lld}}\n",
         (long long)(rows * 512), (long long)(rows * 1024), (long long)(nrec * 12), (long long)(nrec * 12),
         (long long)(tiles * 16384 * 12));
  hipFree(ids); hipFree(sc); hipFree(st); hipFree(s32); hipFree(s64); hipFree(su);
  return 0;
}
