// Microbenchmark: integer / fp64 multiply throughput on gfx950 and the Fp Montgomery product.
// Pins the "peak" used by bench.py's integer-VALU roofline (SURVEY.md §8d asks for a measured value).
// Build: hipcc --offload-arch=gfx950 -O3 -o bench/microbench_mul bench/microbench_mul.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../drand_amd/csrc/fp.hpp"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

// 8 independent v_mad_u64_u32 chains per lane
__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x * 7 + 13;
  uint64_t acc[8];
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = a + k;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = (uint64_t)(uint32_t)acc[k] * (b + k) + (acc[k] >> 32);
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
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
  printf("{\"op\": \"v_mad_u64_u32\", \"Gops_per_s\": %.1f}\n", ops / ms / 1e6);
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
