// Microbenchmark: Fp Montgomery products on gfx950 in the forms the library has used, at controlled occupancy.
//   mul32 / sqr32        12 x 32-bit product scanning, inlined (bench/fp32/fp_mul_fips.hpp: a v_addc per partial product)
//   mul28 / sqr28        14 x 28-bit limbs, one 64-bit column accumulator chain (fp_mul28.hpp m28::mul / sqr)
//   call                 the library's out-of-line product (fp.hpp dh::fp_mul / fp_sqr through DH_FP_CALL)
// Each lane runs ONE dependent chain x = x * y (or x = x^2), as a pairing program or an exponentiation does, at 1, 2
// and 8 waves per SIMD (blocks of 256 threads = 1 wave per SIMD per CU). Every form's result is compared with mul32.
// Build: hipcc --offload-arch=gfx950 -O3 -o bench/microbench_fp28 bench/microbench_fp28.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include "../drand_amd/csrc/fp.hpp"
#include "fp32/fp_mul_fips.hpp"

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

using namespace dh;

constexpr int IT = 512;

struct Mul32 { static __device__ __forceinline__ void f(fp& x, const fp& y) { fips_mont_mul(x.v, x.v, y.v); } };
struct Mul28 { static __device__ __forceinline__ void f(fp& x, const fp& y) { m28::mul(x.v, x.v, y.v); } };
struct MulCall { static __device__ __forceinline__ void f(fp& x, const fp& y) { x = fp_mul(x, y); } };
struct Sqr32 { static __device__ __forceinline__ void f(fp& x, const fp&) { fips_mont_sqr(x.v, x.v); } };
struct Sqr28 { static __device__ __forceinline__ void f(fp& x, const fp&) { m28::sqr(x.v, x.v); } };
struct SqrCall { static __device__ __forceinline__ void f(fp& x, const fp&) { x = fp_sqr(x); } };

template <class Op>
__global__ __launch_bounds__(256) void k_chain(fp* out, const fp* in) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  fp x = in[gid & 1023];
  const fp y = in[(gid + 1) & 1023];
#pragma unroll 1
  for (int it = 0; it < IT; it++) Op::f(x, y);
  out[gid] = x;
}

template <typename K>
float time_kernel(K k, int blocks, fp* out, const fp* in) {
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, in);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(s);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, in);
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms;
  (void)hipEventElapsedTime(&ms, s, e);
  return ms / 3;
}

int main() {
  const int max_blocks = 256 * 8;
  const size_t n = (size_t)max_blocks * 256;
  fp *ref, *out, *in;
  CHECK(hipMalloc(&ref, n * sizeof(fp)));
  CHECK(hipMalloc(&out, n * sizeof(fp)));
  CHECK(hipMalloc(&in, 1024 * sizeof(fp)));
  static fp hin[1024];
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (int i = 0; i < 1024; i++) {
    for (int j = 0; j < 12; j++) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      hin[i].v[j] = (uint32_t)s;
    }
    hin[i].v[11] &= 0x0fffffffu;  // < p
  }
  CHECK(hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice));
  std::vector<fp> hr(n), ho(n);
  struct Form {
    const char* name;
    void (*k)(fp*, const fp*);
    int sq;
  } forms[] = {{"mul32", k_chain<Mul32>, 0}, {"mul28", k_chain<Mul28>, 0}, {"mulcall", k_chain<MulCall>, 0}, {"sqr32", k_chain<Sqr32>, 1}, {"sqr28", k_chain<Sqr28>, 1},
               {"sqrcall", k_chain<SqrCall>, 1}};
  for (int wps : {1, 2, 8}) {
    const int blocks = 256 * wps;
    const double ops = (double)blocks * 256 * IT;
    for (auto& f : forms) {
      const float ms = time_kernel(f.k, blocks, out, in);
      size_t bad = 0;
      if (wps == 8) {  // compare with the 32-bit form of the same operation
        hipLaunchKernelGGL(f.sq ? k_chain<Sqr32> : k_chain<Mul32>, dim3(blocks), dim3(256), 0, 0, ref, in);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(hr.data(), ref, n * sizeof(fp), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(ho.data(), out, n * sizeof(fp), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++) bad += memcmp(&hr[i], &ho[i], sizeof(fp)) != 0;
      }
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"G_per_s\": %.2f, \"ms\": %.3f%s%zu}\n", f.name, wps,
             ops / ms / 1e6, ms, wps == 8 ? ", \"mismatch\": " : ", \"_\": ", bad);
    }
  }
  return 0;
}
