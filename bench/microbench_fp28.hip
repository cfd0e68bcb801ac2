// Microbenchmark: a 14 x 28-bit-limb Montgomery product for Fp against the 12 x 32-bit product of fp.hpp.
// With 28-bit limbs a 28x28 product is < 2^56, so a 64-bit column accumulator absorbs every product of a column
// (<= 28 of them plus the carry-in) with ONE v_mad_u64_u32 each and no carry add; the 32-bit form needs a
// v_addc_co_u32 per product, which costs as much as the multiply (profiles/microbench_carry_r02.txt).
// The 12 x 32-bit interface is kept: x is sliced into 28-bit limbs, y into 28-bit limbs of y * 2^8, so the
// 28-bit Montgomery product (R = 2^392) returns x * y * 2^8 / 2^392 = x * y / 2^384, the same value as fp_mul.
// Checks every result against dh::fp_mul / dh::fp_sqr and reports mismatches.
// Build: hipcc --offload-arch=gfx950 -O3 -o bench/microbench_fp28 bench/microbench_fp28.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include "../drand_amd/csrc/fp.hpp"
#include "../drand_amd/csrc/fp_mul28.hpp"

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

using namespace dh;  // m28:: from fp_mul28.hpp

constexpr int IT = 256;

__global__ void k_mul28(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) {
    m28::mul(x.v, x.v, y.v);
    m28::mul(z.v, z.v, y.v);
  }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_mul32(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) {
    x = dh::fp_mul(x, y);
    z = dh::fp_mul(z, y);
  }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_sqr28(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) {
    m28::sqr(x.v, x.v);
    m28::sqr(z.v, z.v);
  }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_sqr32(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) {
    x = dh::fp_sqr(x);
    z = dh::fp_sqr(z);
  }
  out[gid] = dh::fp_add(x, z);
}

template <typename K>
float time_kernel(K k, int blocks, int threads, dh::fp* out, const dh::fp* in) {
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, in);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(s);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, in);
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms;
  (void)hipEventElapsedTime(&ms, s, e);
  return ms / 5;
}

int main() {
  const int threads = 256, blocks = 256 * 16;
  const size_t n = (size_t)blocks * threads;
  dh::fp *a, *b, *in;
  CHECK(hipMalloc(&a, n * sizeof(dh::fp)));
  CHECK(hipMalloc(&b, n * sizeof(dh::fp)));
  CHECK(hipMalloc(&in, 1024 * sizeof(dh::fp)));
  dh::fp hin[1024];
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (int i = 0; i < 1024; i++) {
    for (int j = 0; j < 12; j++) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      hin[i].v[j] = (uint32_t)s;
    }
    hin[i].v[11] &= 0x0fffffffu;  // < p
  }
  CHECK(hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice));
  const double ops = (double)n * IT * 2;
  struct { const char* name; float ms; } r[4];
  r[0] = {"mul32", time_kernel(k_mul32, blocks, threads, a, in)};
  r[1] = {"mul28", time_kernel(k_mul28, blocks, threads, b, in)};
  std::vector<dh::fp> ha(n), hb(n);
  CHECK(hipMemcpy(ha.data(), a, n * sizeof(dh::fp), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hb.data(), b, n * sizeof(dh::fp), hipMemcpyDeviceToHost));
  size_t bad_mul = 0;
  for (size_t i = 0; i < n; i++) bad_mul += memcmp(&ha[i], &hb[i], sizeof(dh::fp)) != 0;
  r[2] = {"sqr32", time_kernel(k_sqr32, blocks, threads, a, in)};
  r[3] = {"sqr28", time_kernel(k_sqr28, blocks, threads, b, in)};
  CHECK(hipMemcpy(ha.data(), a, n * sizeof(dh::fp), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hb.data(), b, n * sizeof(dh::fp), hipMemcpyDeviceToHost));
  size_t bad_sqr = 0;
  for (size_t i = 0; i < n; i++) bad_sqr += memcmp(&ha[i], &hb[i], sizeof(dh::fp)) != 0;
  for (auto& x : r) printf("{\"op\": \"%s\", \"G_per_s\": %.2f, \"ms\": %.3f}\n", x.name, ops / x.ms / 1e6, x.ms);
  printf("{\"mismatch_mul\": %zu, \"mismatch_sqr\": %zu, \"n\": %zu}\n", bad_mul, bad_sqr, n);
  return 0;
}
