// Microbenchmark + correctness check of the Fp Montgomery product variants on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -o bench/microbench_fp bench/microbench_fp.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "../drand_amd/csrc/fp.hpp"
#include "fp32/fp_mul_fips.hpp"

constexpr int IT = 256;
__global__ void k_cios(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { x = dh::fp_mul_cios(x, y); z = dh::fp_mul_cios(z, y); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_fips(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { dh::fips_mont_mul(x.v, x.v, y.v); dh::fips_mont_mul(z.v, z.v, y.v); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_fips1(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { dh::fips_mont_mul1(x.v, x.v, y.v); dh::fips_mont_mul1(z.v, z.v, y.v); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_fsqr1(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { dh::fips_mont_sqr1(x.v, x.v); dh::fips_mont_sqr1(z.v, z.v); }
  out[gid] = dh::fp_add(x, z);
}
// the production form: out-of-line vector-ABI calls (fp.hpp fp_mul / fp_sqr)
__global__ void k_call_mul(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { x = dh::fp_mul(x, y); z = dh::fp_mul(z, y); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_call_sqr(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { x = dh::fp_sqr(x); z = dh::fp_sqr(z); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_fipsc(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { dh::fips_mont_mul_c(x.v, x.v, y.v); dh::fips_mont_mul_c(z.v, z.v, y.v); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_fsqr(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { dh::fips_mont_sqr(x.v, x.v); dh::fips_mont_sqr(z.v, z.v); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_fsqr_col(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { dh::fips_mont_sqr_col(x.v, x.v); dh::fips_mont_sqr_col(z.v, z.v); }
  out[gid] = dh::fp_add(x, z);
}
__global__ void k_csqr(dh::fp* out, const dh::fp* in) {
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { x = dh::fp_mul_cios(x, x); z = dh::fp_mul_cios(z, z); }
  out[gid] = dh::fp_add(x, z);
}

typedef unsigned __int128 u128;
static const uint64_t P64[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                                0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static void host_mont(uint32_t* r32, const uint32_t* a32, const uint32_t* b32) {
  uint64_t a[6], b[6], t[8] = {0};
  memcpy(a, a32, 48); memcpy(b, b32, 48);
  for (int i = 0; i < 6; i++) {
    u128 c = 0;
    for (int j = 0; j < 6; j++) { c += (u128)a[j] * b[i] + t[j]; t[j] = (uint64_t)c; c >>= 64; }
    u128 s = (u128)t[6] + c; t[6] = (uint64_t)s; t[7] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * 0x89f3fffcfffcfffdULL;
    c = (u128)m * P64[0] + t[0]; c >>= 64;
    for (int j = 1; j < 6; j++) { c += (u128)m * P64[j] + t[j]; t[j - 1] = (uint64_t)c; c >>= 64; }
    s = (u128)t[6] + c; t[5] = (uint64_t)s; t[6] = t[7] + (uint64_t)(s >> 64);
  }
  // reduce
  int ge = 1;
  for (int i = 5; i >= 0; i--) { if (t[i] > P64[i]) { ge = 1; break; } if (t[i] < P64[i]) { ge = 0; break; } }
  if (ge) { u128 br = 0; for (int i = 0; i < 6; i++) { u128 d = (u128)t[i] - P64[i] - br; t[i] = (uint64_t)d; br = (d >> 64) & 1; } }
  memcpy(r32, t, 48);
}

// occupancy-limited variant: dynamic LDS caps resident 256-thread blocks per CU (1 block = 1 wave/SIMD)
extern "C" __global__ void k_call_mul_lds(dh::fp* out, const dh::fp* in) {
  extern __shared__ uint32_t pad[];
  int gid = blockIdx.x * blockDim.x + threadIdx.x;
  dh::fp x = in[gid & 1023], y = in[(gid + 1) & 1023], z = in[(gid + 2) & 1023];
  for (int it = 0; it < IT; it++) { x = dh::fp_mul(x, y); z = dh::fp_mul(z, y); }
  if (gid < 0) pad[threadIdx.x] = 0;
  out[gid] = dh::fp_add(x, z);
}

template <typename K>
float tk(K k, int blocks, dh::fp* o, const dh::fp* i, size_t lds = 0) {
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, o, i);
  hipDeviceSynchronize();
  hipEventRecord(s);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, o, i);
  hipEventRecord(e); hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 16;
  const size_t n = (size_t)blocks * 256;
  dh::fp *in, *o1, *o2;
  hipMalloc(&in, 1024 * sizeof(dh::fp)); hipMalloc(&o1, n * sizeof(dh::fp)); hipMalloc(&o2, n * sizeof(dh::fp));
  static dh::fp hin[1024];
  uint64_t s = 88172645463325252ULL;
  for (int i = 0; i < 1024; i++) {
    for (int j = 0; j < 12; j++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; hin[i].v[j] = (uint32_t)s; }
    hin[i].v[11] &= 0x0fffffffu;  // < p
  }
  hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  int bad = 0;
  // correctness on a small grid (IT iterations) vs host reference
  {
    hipLaunchKernelGGL(k_fips, dim3(4), dim3(256), 0, 0, o1, in);
    hipLaunchKernelGGL(k_cios, dim3(4), dim3(256), 0, 0, o2, in);
    hipLaunchKernelGGL(k_fsqr, dim3(4), dim3(256), 0, 0, o1 + 1024, in);
    static dh::fp r3[1024];
    hipLaunchKernelGGL(k_fipsc, dim3(4), dim3(256), 0, 0, o2 + 2048, in);
    hipMemcpy(r3, o2 + 2048, sizeof(r3), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_csqr, dim3(4), dim3(256), 0, 0, o2 + 1024, in);
    static dh::fp r1[2048], r2[2048];
    hipMemcpy(r1, o1, sizeof(r1), hipMemcpyDeviceToHost);
    hipMemcpy(r2, o2, sizeof(r2), hipMemcpyDeviceToHost);
    // host check of lane 0..63 of k_cios/k_fips
    for (int g = 0; g < 64; g++) {
      uint32_t x[12], y[12], z[12];
      memcpy(x, hin[g & 1023].v, 48); memcpy(y, hin[(g + 1) & 1023].v, 48); memcpy(z, hin[(g + 2) & 1023].v, 48);
      for (int it = 0; it < IT; it++) { host_mont(x, x, y); host_mont(z, z, y); }
      // x+z mod p
      u128 c = 0; uint64_t a[6], b[6], t[6]; memcpy(a, x, 48); memcpy(b, z, 48);
      for (int i = 0; i < 6; i++) { c += (u128)a[i] + b[i]; t[i] = (uint64_t)c; c >>= 64; }
      int ge = 1; for (int i = 5; i >= 0; i--) { if (t[i] > P64[i]) { ge = 1; break; } if (t[i] < P64[i]) { ge = 0; break; } }
      if (ge) { u128 br = 0; for (int i = 0; i < 6; i++) { u128 d = (u128)t[i] - P64[i] - br; t[i] = (uint64_t)d; br = (d >> 64) & 1; } }
      if (memcmp(t, r1[g].v, 48)) bad |= 1;
      if (memcmp(t, r2[g].v, 48)) bad |= 2;
      if (memcmp(t, r3[g].v, 48)) bad |= 8;
    }
    for (int g = 0; g < 1024; g++) if (memcmp(r1[1024 + g].v, r2[1024 + g].v, 48)) bad |= 4;
    // old single-MAC forms and the out-of-line call forms agree with the grouped ones
    static dh::fp q1[1024], q2[1024];
    hipLaunchKernelGGL(k_fips1, dim3(4), dim3(256), 0, 0, o2, in);
    hipMemcpy(q1, o2, sizeof(q1), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_call_mul, dim3(4), dim3(256), 0, 0, o2, in);
    hipMemcpy(q2, o2, sizeof(q2), hipMemcpyDeviceToHost);
    for (int g = 0; g < 1024; g++) if (memcmp(q1[g].v, r1[g].v, 48) || memcmp(q2[g].v, r1[g].v, 48)) bad |= 16;
    hipLaunchKernelGGL(k_fsqr1, dim3(4), dim3(256), 0, 0, o2, in);
    hipMemcpy(q1, o2, sizeof(q1), hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_call_sqr, dim3(4), dim3(256), 0, 0, o2, in);
    hipMemcpy(q2, o2, sizeof(q2), hipMemcpyDeviceToHost);
    for (int g = 0; g < 1024; g++) if (memcmp(q1[g].v, r1[1024 + g].v, 48) || memcmp(q2[g].v, r1[1024 + g].v, 48)) bad |= 32;
    hipLaunchKernelGGL(k_fsqr_col, dim3(4), dim3(256), 0, 0, o2, in);
    hipMemcpy(q1, o2, sizeof(q1), hipMemcpyDeviceToHost);
    for (int g = 0; g < 1024; g++) if (memcmp(q1[g].v, r1[1024 + g].v, 48)) bad |= 64;
  }
  printf("{\"check\": \"fp_mul fips/cios/sqr vs host\", \"bad_mask\": %d}\n", bad);
  double ops = (double)n * IT * 2;
  float ms = tk(k_cios, blocks, o1, in);
  printf("{\"op\": \"fp_mul_cios\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_fips, blocks, o1, in);
  printf("{\"op\": \"fp_mul_fips\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_fips1, blocks, o1, in);
  printf("{\"op\": \"fp_mul_fips_1mac_per_asm\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_fsqr_col, blocks, o1, in);
  printf("{\"op\": \"fp_sqr_fips_column_form\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_fsqr1, blocks, o1, in);
  printf("{\"op\": \"fp_sqr_fips_1mac_per_asm\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_call_mul, blocks, o1, in);
  printf("{\"op\": \"fp_mul_call (production)\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_call_sqr, blocks, o1, in);
  printf("{\"op\": \"fp_sqr_call (production)\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  hipFuncSetAttribute((const void*)k_call_mul_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int w : {1, 2, 3, 4}) {
    size_t lds = (160 * 1024) / w - 1024;
    ms = tk(k_call_mul_lds, blocks, o1, in, lds);
    printf("{\"op\": \"fp_mul_call, occupancy %d wave/SIMD\", \"Gops_per_s\": %.2f}\n", w, ops / ms / 1e6);
  }
  ms = tk(k_fipsc, blocks, o1, in);
  printf("{\"op\": \"fp_mul_fips_plain_c\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_csqr, blocks, o1, in);
  printf("{\"op\": \"fp_sqr_cios\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  ms = tk(k_fsqr, blocks, o1, in);
  printf("{\"op\": \"fp_sqr_fips\", \"Gops_per_s\": %.2f}\n", ops / ms / 1e6);
  return bad ? 1 : 0;
}
