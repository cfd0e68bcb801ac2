// Microbenchmark: integer / fp64 multiply throughput on gfx950 and the Fp Montgomery product.
// Pins the "peak" used by bench.py's integer-VALU roofline (SURVEY.md §8d asks for a measured value).
// Build: hipcc --offload-arch=gfx950 -O3 -o bench/microbench_mul bench/microbench_mul.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../drand_amd/csrc/fp.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

// 8 independent v_mad_u64_u32 chains per lane, pure: acc_k = x_k * b + acc_k with the full 64-bit
// accumulator as the addend, so each step is ONE instruction (no v_mov staging an addend; the r01 form
// acc * b + (acc >> 32) compiled to 8 v_mad_u64_u32 + 8 v_mov per iteration, half the issue slots moves).
// The 8 MACs are one asm statement: the ISA is exactly this (checked with hipcc -S, bench/microbench_mul.isa.txt).
__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  uint64_t c;
  for (int it = 0; it < ITERS / 4; it++) {  // 32 MACs per statement: one hazard s_nop per 32 (between statements)
    asm volatile(
        "v_mad_u64_u32 %0, %8, %10, %9, %0\n\t"
        "v_mad_u64_u32 %1, %8, %11, %9, %1\n\t"
        "v_mad_u64_u32 %2, %8, %12, %9, %2\n\t"
        "v_mad_u64_u32 %3, %8, %13, %9, %3\n\t"
        "v_mad_u64_u32 %4, %8, %14, %9, %4\n\t"
        "v_mad_u64_u32 %5, %8, %15, %9, %5\n\t"
        "v_mad_u64_u32 %6, %8, %16, %9, %6\n\t"
        "v_mad_u64_u32 %7, %8, %17, %9, %7\n\t"
        "v_mad_u64_u32 %0, %8, %10, %9, %0\n\t"
        "v_mad_u64_u32 %1, %8, %11, %9, %1\n\t"
        "v_mad_u64_u32 %2, %8, %12, %9, %2\n\t"
        "v_mad_u64_u32 %3, %8, %13, %9, %3\n\t"
        "v_mad_u64_u32 %4, %8, %14, %9, %4\n\t"
        "v_mad_u64_u32 %5, %8, %15, %9, %5\n\t"
        "v_mad_u64_u32 %6, %8, %16, %9, %6\n\t"
        "v_mad_u64_u32 %7, %8, %17, %9, %7\n\t"
        "v_mad_u64_u32 %0, %8, %10, %9, %0\n\t"
        "v_mad_u64_u32 %1, %8, %11, %9, %1\n\t"
        "v_mad_u64_u32 %2, %8, %12, %9, %2\n\t"
        "v_mad_u64_u32 %3, %8, %13, %9, %3\n\t"
        "v_mad_u64_u32 %4, %8, %14, %9, %4\n\t"
        "v_mad_u64_u32 %5, %8, %15, %9, %5\n\t"
        "v_mad_u64_u32 %6, %8, %16, %9, %6\n\t"
        "v_mad_u64_u32 %7, %8, %17, %9, %7\n\t"
        "v_mad_u64_u32 %0, %8, %10, %9, %0\n\t"
        "v_mad_u64_u32 %1, %8, %11, %9, %1\n\t"
        "v_mad_u64_u32 %2, %8, %12, %9, %2\n\t"
        "v_mad_u64_u32 %3, %8, %13, %9, %3\n\t"
        "v_mad_u64_u32 %4, %8, %14, %9, %4\n\t"
        "v_mad_u64_u32 %5, %8, %15, %9, %5\n\t"
        "v_mad_u64_u32 %6, %8, %16, %9, %6\n\t"
        "v_mad_u64_u32 %7, %8, %17, %9, %7"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=&s"(c)
        : "v"(b), "v"(x), "v"(x + 1), "v"(x + 2), "v"(x + 3), "v"(x + 4), "v"(x + 5), "v"(x + 6), "v"(x + 7));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// the same 8 MACs each followed by its carry v_addc_co_u32 (the product-scanning column step of fp_mul_fips.hpp:
// 2 VALU per 32x32 product): the rate the Montgomery product itself can reach
__global__ void k_mac_carry(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  uint64_t c;
  for (int it = 0; it < ITERS; it++) {
    asm volatile(
        "v_mad_u64_u32 %0, %8, %10, %9, %0\n\tv_addc_co_u32_e64 %4, %8, 0, %4, %8\n\t"
        "v_mad_u64_u32 %1, %8, %11, %9, %1\n\tv_addc_co_u32_e64 %5, %8, 0, %5, %8\n\t"
        "v_mad_u64_u32 %2, %8, %12, %9, %2\n\tv_addc_co_u32_e64 %6, %8, 0, %6, %8\n\t"
        "v_mad_u64_u32 %3, %8, %13, %9, %3\n\tv_addc_co_u32_e64 %7, %8, 0, %7, %8\n\t"
        "v_mad_u64_u32 %0, %8, %10, %9, %0\n\tv_addc_co_u32_e64 %4, %8, 0, %4, %8\n\t"
        "v_mad_u64_u32 %1, %8, %11, %9, %1\n\tv_addc_co_u32_e64 %5, %8, 0, %5, %8\n\t"
        "v_mad_u64_u32 %2, %8, %12, %9, %2\n\tv_addc_co_u32_e64 %6, %8, 0, %6, %8\n\t"
        "v_mad_u64_u32 %3, %8, %13, %9, %3\n\tv_addc_co_u32_e64 %7, %8, 0, %7, %8"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "=&s"(c)
          : "v"(b), "v"(x), "v"(x + 1), "v"(x + 2), "v"(x + 3));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ h0 ^ h1 ^ h2 ^ h3;
}

// 8 independent v_mul_lo_u32 chains
__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t acc[8];
  uint32_t b = blockIdx.x * 7 + 13;
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + seed + k;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = acc[k] * (b + k) + 1;
  }
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 8 independent v_fma_f64 chains
__global__ void k_fma64(double* out, double seed) {
  double acc[8];
  double b = 1.0000001 + blockIdx.x * 1e-9;
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = threadIdx.x + seed + k;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = fma(acc[k], b, 0.5);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Fp Montgomery multiplication chain (2 independent chains per lane)
constexpr int FP_ITERS = 256;
__global__ void k_fpmul(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < FP_ITERS; it++) {
    x = dh::fp_mul(x, y);
    z = dh::fp_mul(z, y);
  }
  out[gid] = dh::fp_add(x, z);
}

template <typename K, typename... Args>
float time_kernel(K k, int blocks, int threads, Args... args) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, args...);  // warm
  hipDeviceSynchronize();
  hipEventRecord(s);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, args...);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms / 5;
}

int main() {
  int blocks = 256 * 32, threads = 256;
  size_t n = (size_t)blocks * threads;
  void* buf;
  CHECK(hipMalloc(&buf, n * sizeof(dh::fp)));
  dh::fp* in;
  CHECK(hipMalloc(&in, 1024 * sizeof(dh::fp)));
  dh::fp hin[1024];
  for (int i = 0; i < 1024; i++)
    for (int j = 0; j < 12; j++) hin[i].v[j] = (j == 11) ? (0x0fffffffu & (i * 2654435761u + j)) : (i * 2654435761u + j * 40503u);
  CHECK(hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice));

  float ms = time_kernel(k_mad64, blocks, threads, (uint64_t*)buf, 1u);
  double ops = (double)n * ITERS * 8;
  printf("{\"op\": \"v_mad_u64_u32\", \"Gops_per_s\": %.1f, \"ms\": %.4f}\n", ops / ms / 1e6, ms);
  ms = time_kernel(k_mac_carry, blocks, threads, (uint64_t*)buf, 1u);
  printf("{\"op\": \"v_mad_u64_u32+v_addc_co_u32\", \"Gmac_per_s\": %.1f, \"ms\": %.4f}\n", ops / ms / 1e6, ms);
  ms = time_kernel(k_mullo, blocks, threads, (uint32_t*)buf, 1u);
  printf("{\"op\": \"v_mul_lo_u32+add\", \"Gops_per_s\": %.1f}\n", ops / ms / 1e6);
  ms = time_kernel(k_fma64, blocks, threads, (double*)buf, 1.0);
  printf("{\"op\": \"v_fma_f64\", \"Gops_per_s\": %.1f}\n", ops / ms / 1e6);
  int fb = 256 * 16;
  ms = time_kernel(k_fpmul, fb, threads, (dh::fp*)buf, (const dh::fp*)in);
  double fops = (double)fb * threads * FP_ITERS * 2;
  printf("{\"op\": \"fp_mul_12x32\", \"Gops_per_s\": %.3f, \"mul32_equiv_T_per_s\": %.3f}\n", fops / ms / 1e6,
         fops * 288 / ms / 1e9);
  return 0;
}
