// Microbenchmark: 12-limb modular add/sub carry chains on gfx950.
//   (a) clang __builtin_addc/subc (VOP2 chains through VCC; the compiler puts s_nop 1 between dependent links)
//   (b) inline asm chains through an SGPR pair (VOP3 e64 forms), 4 limbs per statement
// Both are checked against each other on every lane. Build: hipcc --offload-arch=gfx950 -O3 -o bench/microbench_add bench/microbench_add.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include "../drand_amd/csrc/fp.hpp"
using namespace dh;

#define ADD4(first, o, x, y, c)                                                                                   \
  asm volatile(first "\n\tv_addc_co_u32_e64 %1, %4, %6, %10, %4\n\tv_addc_co_u32_e64 %2, %4, %7, %11, %4\n\t"    \
               "v_addc_co_u32_e64 %3, %4, %8, %12, %4"                                                            \
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "+s"(c)                                      \
               : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]))
#define SUB4(first, o, x, y, c)                                                                                   \
  asm volatile(first "\n\tv_subb_co_u32_e64 %1, %4, %6, %10, %4\n\tv_subb_co_u32_e64 %2, %4, %7, %11, %4\n\t"    \
               "v_subb_co_u32_e64 %3, %4, %8, %12, %4"                                                            \
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "+s"(c)                                      \
               : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]))

__device__ __forceinline__ void add12(uint32_t* o, const uint32_t* x, const uint32_t* y, uint64_t& c) {
  ADD4("v_add_co_u32_e64 %0, %4, %5, %9", o, x, y, c);
  ADD4("v_addc_co_u32_e64 %0, %4, %5, %9, %4", (o + 4), (x + 4), (y + 4), c);
  ADD4("v_addc_co_u32_e64 %0, %4, %5, %9, %4", (o + 8), (x + 8), (y + 8), c);
}
__device__ __forceinline__ void sub12(uint32_t* o, const uint32_t* x, const uint32_t* y, uint64_t& c) {
  SUB4("v_sub_co_u32_e64 %0, %4, %5, %9", o, x, y, c);
  SUB4("v_subb_co_u32_e64 %0, %4, %5, %9, %4", (o + 4), (x + 4), (y + 4), c);
  SUB4("v_subb_co_u32_e64 %0, %4, %5, %9, %4", (o + 8), (x + 8), (y + 8), c);
}
__device__ __forceinline__ void sel12(uint32_t* o, const uint32_t* keep, const uint32_t* other, uint64_t c) {
  // o = c ? keep : other  (per lane)
#pragma unroll
  for (int i = 0; i < 12; i++) asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(o[i]) : "v"(other[i]), "v"(keep[i]), "s"(c));
}

__device__ __forceinline__ fp fp_add_asm(const fp& a, const fp& b) {
  const uint32_t P[12] = {DH_P0, DH_P1, DH_P2, DH_P3, DH_P4, DH_P5, DH_P6, DH_P7, DH_P8, DH_P9, DH_P10, DH_P11};
  fp s, t, r;
  uint64_t c;
  add12(s.v, a.v, b.v, c);
  sub12(t.v, s.v, P, c);
  sel12(r.v, s.v, t.v, c);  // borrow: s < p, keep s
  return r;
}
__device__ __forceinline__ fp fp_sub_asm(const fp& a, const fp& b) {
  const uint32_t P[12] = {DH_P0, DH_P1, DH_P2, DH_P3, DH_P4, DH_P5, DH_P6, DH_P7, DH_P8, DH_P9, DH_P10, DH_P11};
  fp s, t, r;
  uint64_t c;
  sub12(s.v, a.v, b.v, c);
  uint64_t c2;
  add12(t.v, s.v, P, c2);
  sel12(r.v, t.v, s.v, c);  // borrow: a < b, take s + p
  return r;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_bench(fp* x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  fp a = x[2 * i], b = x[2 * i + 1];
  for (int k = 0; k < iters; k++) {
    if (MODE == 0) {
      a = fp_add(a, b);
      b = fp_sub(b, a);
    } else {
      a = fp_add_asm(a, b);
      b = fp_sub_asm(b, a);
    }
  }
  x[2 * i] = a;
  x[2 * i + 1] = b;
}

int main() {
  const int nthr = 256 * 1024 * 2, iters = 2000;
  fp* h = (fp*)malloc(sizeof(fp) * 2 * nthr);
  uint64_t s = 1;
  for (int i = 0; i < 2 * nthr; i++) {
    for (int j = 0; j < 12; j++) {
      s = s * 6364136223846793005ULL + 1442695040888963407ULL;
      h[i].v[j] = (uint32_t)(s >> 32);
    }
    h[i].v[11] &= 0x0fffffffu;  // < p
  }
  fp *d0, *d1;
  hipMalloc(&d0, sizeof(fp) * 2 * nthr);
  hipMalloc(&d1, sizeof(fp) * 2 * nthr);
  float ms[2];
  for (int mode = 0; mode < 2; mode++) {
    fp* d = mode ? d1 : d0;
    hipMemcpy(d, h, sizeof(fp) * 2 * nthr, hipMemcpyHostToDevice);
    if (mode == 0) hipLaunchKernelGGL(k_bench<0>, dim3(nthr / 256), dim3(256), 0, 0, d, 1);
    else hipLaunchKernelGGL(k_bench<1>, dim3(nthr / 256), dim3(256), 0, 0, d, 1);
    hipMemcpy(d, h, sizeof(fp) * 2 * nthr, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    if (mode == 0) hipLaunchKernelGGL(k_bench<0>, dim3(nthr / 256), dim3(256), 0, 0, d, iters);
    else hipLaunchKernelGGL(k_bench<1>, dim3(nthr / 256), dim3(256), 0, 0, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[mode], e0, e1);
  }
  fp* r0 = (fp*)malloc(sizeof(fp) * 2 * nthr);
  fp* r1 = (fp*)malloc(sizeof(fp) * 2 * nthr);
  hipMemcpy(r0, d0, sizeof(fp) * 2 * nthr, hipMemcpyDeviceToHost);
  hipMemcpy(r1, d1, sizeof(fp) * 2 * nthr, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < 2 * nthr; i++) bad += memcmp(&r0[i], &r1[i], sizeof(fp)) != 0;
  const double ops = 2.0 * iters * nthr;
  printf("{\"op\": \"fp_add+fp_sub builtin chains\", \"Gops_per_s\": %.2f}\n", ops / ms[0] / 1e6);
  printf("{\"op\": \"fp_add+fp_sub asm SGPR chains\", \"Gops_per_s\": %.2f}\n", ops / ms[1] / 1e6);
  printf("{\"check\": \"asm vs builtin\", \"mismatching_lanes\": %ld}\n", bad);
  return 0;
}
