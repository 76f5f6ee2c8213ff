// tools/valu_rates.hip -- issue cost of the VALU instructions the sieve's inner loops use (gfx950).
// One wave per SIMD, 8 independent instances per step so latency is hidden: cycles per instruction
// per wave (s_memtime = shader cycles). A full-rate wave64 op is 4 cycles.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o tools/valu_rates && tools/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N_IT 256
#define OPS(X)                                                                                           \
  X(0, "v_cvt_u32_f64", asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(u[j]) : "v"(d[j])))                   \
  X(1, "v_cvt_f64_u32", asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(e[j]) : "v"(u[j])))                   \
  X(2, "v_ldexp_f64", asm volatile("v_ldexp_f64 %0, %1, 32" : "=v"(e[j]) : "v"(d[j])))                    \
  X(3, "v_fma_f64", asm volatile("v_fma_f64 %0, %1, %1, %1" : "=v"(e[j]) : "v"(d[j])))                    \
  X(4, "v_mul_f64", asm volatile("v_mul_f64 %0, %1, %1" : "=v"(e[j]) : "v"(d[j])))                        \
  X(5, "v_add_f64", asm volatile("v_add_f64 %0, %1, %1" : "=v"(e[j]) : "v"(d[j])))                        \
  X(6, "v_cvt_f32_f64", asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[j]) : "v"(d[j])))                   \
  X(7, "v_cvt_u32_f32", asm volatile("v_cvt_u32_f32 %0, %1" : "=v"(u[j]) : "v"(f[j])))                   \
  X(8, "v_mul_u32_u24", asm volatile("v_mul_u32_u24 %0, %1, %1" : "=v"(w[j]) : "v"(u[j])))               \
  X(9, "v_mul_lo_u32", asm volatile("v_mul_lo_u32 %0, %1, %1" : "=v"(w[j]) : "v"(u[j])))                 \
  X(10, "v_mul_hi_u32", asm volatile("v_mul_hi_u32 %0, %1, %1" : "=v"(w[j]) : "v"(u[j])))                \
  X(11, "v_lshlrev_b64", asm volatile("v_lshlrev_b64 %0, %1, %2" : "=v"(q[j]) : "v"(u[j]), "v"(q[j])))   \
  X(12, "v_lshrrev_b64", asm volatile("v_lshrrev_b64 %0, %1, %2" : "=v"(q[j]) : "v"(u[j]), "v"(q[j])))   \
  X(13, "v_bfe_u32", asm volatile("v_bfe_u32 %0, %1, 13, 13" : "=v"(w[j]) : "v"(u[j])))                  \
  X(14, "v_mad_u64_u32", asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %2" : "=v"(q[j]) : "v"(u[j]), "v"(q[j]) : "vcc")) \
  X(15, "v_xor_b32", asm volatile("v_xor_b32 %0, %1, %1" : "=v"(w[j]) : "v"(u[j])))                      \
  X(16, "v_mul_hi_u32_u24", asm volatile("v_mul_hi_u32_u24 %0, %1, %1" : "=v"(w[j]) : "v"(u[j])))       \
  X(17, "v_lshl_add_u32", asm volatile("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(w[j]) : "v"(u[j])))         \
  X(18, "v_cvt_f64_i32", asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(e[j]) : "v"(u[j])))                  \
  X(19, "v_frexp_exp_i32_f64", asm volatile("v_frexp_exp_i32_f64 %0, %1" : "=v"(w[j]) : "v"(d[j])))      \
  X(20, "v_trunc_f64", asm volatile("v_trunc_f64 %0, %1" : "=v"(e[j]) : "v"(d[j])))                      \
  X(21, "v_fract_f64", asm volatile("v_fract_f64 %0, %1" : "=v"(e[j]) : "v"(d[j])))                      \
  X(22, "v_alignbit_b32", asm volatile("v_alignbit_b32 %0, %1, %1, 7" : "=v"(w[j]) : "v"(u[j])))         \
  X(23, "v_mul_u64_via_pk", asm volatile("v_pk_mul_f32 %0, %1, %1" : "=v"(q[j]) : "v"(q[j])))            \
  X(24, "v_cndmask_b32", asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(w[j]) : "v"(u[j]), "v"(w[j])))

template <int OP>
__global__ void __launch_bounds__(1024) k_rate(unsigned long long* cyc, uint32_t* sink) {
  double d[8], e[8];
  float f[8];
  uint32_t u[8], w[8];
  uint64_t q[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    d[j] = 1.5 + threadIdx.x + j;
    e[j] = 0.0;
    f[j] = 2.5f + j;
    u[j] = threadIdx.x * 7u + j;
    w[j] = 0u;
    q[j] = j;
  }
  asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < N_IT; it++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
      for (int j = 0; j < 8; j++) {
#define CASE(id, name, stmt) if (OP == id) { stmt; }
        OPS(CASE)
#undef CASE
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) acc += u[j] + w[j] + (uint32_t)q[j] + (uint32_t)e[j] + (uint32_t)f[j];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x * 4] = (unsigned long long)(t1 - t0);
}

template <int OP>
static void run(const char* name, unsigned long long* dc, uint32_t* ds, int blocks) {
  double per[2];
  for (int v = 0; v < 2; v++) {
    const int wps = v ? 4 : 1;  // waves per SIMD
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256 * wps), 0, 0, dc, ds);
    hipDeviceSynchronize();
    unsigned long long h[4];
    hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
    per[v] = (double)h[0] / (N_IT * 4 * 8) / wps;  // SIMD cycles per wave-instruction
  }
  printf("%-22s %6.2f cycles per wave-instruction at 1 wave per SIMD, %6.2f at 4 (SIMD throughput)\n", name, per[0], per[1]);
}

int main() {
  unsigned long long* dc;
  uint32_t* ds;
  hipMalloc(&dc, 4096 * 8);
  hipMalloc(&ds, 4096 * 256 * 4);
  const int blocks = 256;
#define RUN(id, name, stmt) run<id>(name, dc, ds, blocks);
  OPS(RUN)
#undef RUN
  return 0;
}
