// Microbenchmark: the product-scanning MAC step of the Fp product (fp_mul_fips.hpp) in several register forms, to
// find what bounds it on gfx950: v_mad_u64_u32 (64-bit column accumulator += a*b, carry-out to an SGPR pair) +
// v_addc_co_u32 (third column word += carry).
//   sgpr1   4 independent accumulator chains, ONE SGPR carry pair shared by every MAC (the k_mac_carry form)
//   sgpr4   4 chains, one SGPR carry pair per chain
//   vcc     4 chains, carry through VCC, the add in its VOP2 (_e32) encoding
//   chain1  ONE dependent MAC + carry chain (one column of the product)
//   chain2  two interleaved dependent chains (two columns accumulated at once)
//   mad1    one dependent v_mad_u64_u32 chain, no carry (the MAD's dependent latency)
// Each asm statement holds 32 MAC steps, so the inter-statement hazard s_nop is amortised.
// Build: hipcc --offload-arch=gfx950 -O3 -o bench/microbench_carry bench/microbench_carry.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                  \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

constexpr int ITERS = 1024;  // x 32 MAC steps per iteration

#define M4S1(A, H) "v_mad_u64_u32 %" #A ", %8, %10, %9, %" #A "\n\tv_addc_co_u32_e64 %" #H ", %8, 0, %" #H ", %8\n\t"
__global__ void k_sgpr1(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  uint64_t c;
  for (int it = 0; it < ITERS; it++) {
#define Q M4S1(0, 4) M4S1(1, 5) M4S1(2, 6) M4S1(3, 7)
    asm volatile(Q Q Q Q Q Q Q Q
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "=&s"(c)
                 : "v"(b), "v"(x));
#undef Q
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ h0 ^ h1 ^ h2 ^ h3;
}

#define M4S4(A, H, C) "v_mad_u64_u32 %" #A ", %" #C ", %13, %12, %" #A "\n\tv_addc_co_u32_e64 %" #H ", %" #C ", 0, %" #H ", %" #C "\n\t"
__global__ void k_sgpr4(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  uint64_t c0, c1, c2, c3;
  for (int it = 0; it < ITERS; it++) {
#define Q M4S4(0, 4, 8) M4S4(1, 5, 9) M4S4(2, 6, 10) M4S4(3, 7, 11)
    asm volatile(Q Q Q Q Q Q Q Q
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "=&s"(c0), "=&s"(c1),
                   "=&s"(c2), "=&s"(c3)
                 : "v"(b), "v"(x));
#undef Q
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ h0 ^ h1 ^ h2 ^ h3;
}

#define M4V(A, H) "v_mad_u64_u32 %" #A ", vcc, %9, %8, %" #A "\n\tv_addc_co_u32_e32 %" #H ", vcc, 0, %" #H ", vcc\n\t"
__global__ void k_vcc(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  for (int it = 0; it < ITERS; it++) {
#define Q M4V(0, 4) M4V(1, 5) M4V(2, 6) M4V(3, 7)
    asm volatile(Q Q Q Q Q Q Q Q
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3)
                 : "v"(b), "v"(x)
                 : "vcc");
#undef Q
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ h0 ^ h1 ^ h2 ^ h3;
}

#define M1(A, H) "v_mad_u64_u32 %" #A ", %2, %4, %3, %" #A "\n\tv_addc_co_u32_e64 %" #H ", %2, 0, %" #H ", %2\n\t"
__global__ void k_chain1(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed;
  uint32_t h0 = 0;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  uint64_t c;
  for (int it = 0; it < ITERS; it++) {
#define Q M1(0, 1) M1(0, 1) M1(0, 1) M1(0, 1)
    asm volatile(Q Q Q Q Q Q Q Q : "+v"(a0), "+v"(h0), "=&s"(c) : "v"(b), "v"(x));
#undef Q
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ h0;
}

#define M2(A, H, C) "v_mad_u64_u32 %" #A ", %" #C ", %7, %6, %" #A "\n\tv_addc_co_u32_e64 %" #H ", %" #C ", 0, %" #H ", %" #C "\n\t"
__global__ void k_chain2(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed, a1 = a0 + 5;
  uint32_t h0 = 0, h1 = 0;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  uint64_t c0, c1;
  for (int it = 0; it < ITERS; it++) {
#define Q M2(0, 2, 4) M2(1, 3, 5) M2(0, 2, 4) M2(1, 3, 5)
    asm volatile(Q Q Q Q Q Q Q Q : "+v"(a0), "+v"(a1), "+v"(h0), "+v"(h1), "=&s"(c0), "=&s"(c1) : "v"(b), "v"(x));
#undef Q
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ h0 ^ h1;
}

#define MD "v_mad_u64_u32 %0, %1, %3, %2, %0\n\t"
__global__ void k_mad1(uint64_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x + seed;
  const uint32_t b = blockIdx.x * 7 + 13, x = threadIdx.x * 3 + seed;
  uint64_t c;
  for (int it = 0; it < ITERS; it++) {
#define Q MD MD MD MD
    asm volatile(Q Q Q Q Q Q Q Q : "+v"(a0), "=&s"(c) : "v"(b), "v"(x));
#undef Q
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0;
}

template <typename K>
float time_kernel(K k, int blocks, int threads, uint64_t* buf) {
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 1u);  // warm
  hipDeviceSynchronize();
  hipEventRecord(s);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 1u);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms / 5;
}

int main() {
  const int threads = 256;
  uint64_t* buf;
  CHECK(hipMalloc(&buf, (size_t)256 * 64 * threads * sizeof(uint64_t)));
  // waves per SIMD: blocks / 256 CUs x 4 waves per block / 4 SIMDs
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256 * wps;
    const double steps = (double)blocks * threads * ITERS * 32;
    struct {
      const char* name;
      float ms;
    } r[] = {{"sgpr1", time_kernel(k_sgpr1, blocks, threads, buf)}, {"sgpr4", time_kernel(k_sgpr4, blocks, threads, buf)},
             {"vcc", time_kernel(k_vcc, blocks, threads, buf)},     {"chain1", time_kernel(k_chain1, blocks, threads, buf)},
             {"chain2", time_kernel(k_chain2, blocks, threads, buf)}, {"mad1", time_kernel(k_mad1, blocks, threads, buf)}};
    for (auto& x : r)
      printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"T_mac_per_s\": %.2f}\n", x.name, wps, steps / x.ms / 1e9);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
