// Pairing checks: one lane per RLC group, per-round leaves of the bisection (gfx950).
#include "kcommon.hpp"

namespace dh {


// the verification equation for signature sum S and (cofactor-cleared) hash sum H:
//   G1 signatures: e(H, pk) * e(-S, g2) == 1       G2 signatures: e(pk, H) * e(-g1, S) == 1
// (kyber-bls12381 ValidatePairing(p1,p2,p3,p4) = AddPair(p1,p2), AddPairInv(p3,p4), Check())
DH_DEV bool check_g1sig(const jac<fp>& S, const jac<fp>& H, const aff<fp2>& pk) {
  jac<fp> P[2] = {H, jac_neg(S)};
  jac<fp2> Q[2] = {jac_from_aff(pk), g2_gen()};
  return pairing_check<2>(P, Q);
}
DH_DEV bool check_g2sig(const jac<fp2>& S, const jac<fp2>& H, const aff<fp>& pk) {
  jac<fp> P[2] = {jac_from_aff(pk), jac_neg(g1_gen())};
  jac<fp2> Q[2] = {H, S};
  return pairing_check<2>(P, Q);
}

// Two lanes per group, one pair each: lane 2g evaluates the Miller loop of the hash pair (after clearing
// the cofactor of B), lane 2g+1 that of the signature pair; the odd lane hands its Miller value over LDS and
// the even lane multiplies, runs the final exponentiation and writes the verdict. Halves the Miller-loop
// latency of the (latency-bound, one-per-batch) check against the 2-pair loop in one lane.
//   G1 signatures: e([h]B, pk) * e(-A, g2) == 1       G2 signatures: e(pk, [h]B) * e(-g1, A) == 1
constexpr int GC_THREADS = 64;
template <class F>
__global__ __launch_bounds__(GC_THREADS) void k_group_check(const uint32_t* __restrict__ A, const uint32_t* __restrict__ B,
                                                            size_t ngroups, const uint32_t* __restrict__ key_aff,
                                                            uint8_t* __restrict__ pass) {
  __shared__ uint32_t fbuf[GC_THREADS / 2][144];
  const int lane = threadIdx.x;
  const size_t g = (size_t)blockIdx.x * (GC_THREADS / 2) + lane / 2;
  const bool hash_side = (lane & 1) == 0;
  fp12 f = fp12_one();
  if (g < ngroups) {
    jac<fp> P;
    jac<fp2> Q;
    if constexpr (sizeof(F) == sizeof(fp)) {
      if (hash_side) {
        P = h2c_clear_g1(ld_jac_aos<fp>(B, g));
        Q = jac_from_aff(ld_aff_aos<fp2>(key_aff, 0));
      } else {
        P = jac_neg(ld_jac_aos<fp>(A, g));
        Q = g2_gen();
      }
    } else {
      if (hash_side) {
        P = jac_from_aff(ld_aff_aos<fp>(key_aff, 0));
        Q = h2c_clear_g2(ld_jac_aos<fp2>(B, g));
      } else {
        P = jac_neg(g1_gen());
        Q = ld_jac_aos<fp2>(A, g);
      }
    }
    if (!jac_is_inf(P) && !jac_is_inf(Q)) {  // kilic's engine skips pairs with an infinity
      aff<fp> pa[1] = {jac_to_aff(P)};
      aff<fp2> qa[1] = {jac_to_aff(Q)};
      bool sk[1] = {false};
      f = miller_loop<1>(pa, qa, sk);
    }
  }
  if (!hash_side) {
    const fp2* c = &f.c0.c0;
    for (int k = 0; k < 6; k++)
      for (int w = 0; w < 12; w++) {
        fbuf[lane / 2][24 * k + w] = c[k].c0.v[w];
        fbuf[lane / 2][24 * k + 12 + w] = c[k].c1.v[w];
      }
  }
  __syncthreads();
  if (hash_side && g < ngroups) {
    fp12 h;
    fp2* c = &h.c0.c0;
    for (int k = 0; k < 6; k++)
      for (int w = 0; w < 12; w++) {
        c[k].c0.v[w] = fbuf[lane / 2][24 * k + w];
        c[k].c1.v[w] = fbuf[lane / 2][24 * k + 12 + w];
      }
    pass[g] = fp12_is_one(final_exp(fp12_mul(f, h))) ? 1 : 0;
  }
}

// bisection leaves: full per-round verification of the listed rounds
template <class F>
__global__ __launch_bounds__(64) void k_leaf_check(const uint32_t* __restrict__ entries, size_t m,
                                                   const uint32_t* __restrict__ sig_aff, const uint32_t* __restrict__ q_pts,
                                                   const uint32_t* __restrict__ key_aff, const uint8_t* __restrict__ status,
                                                   uint8_t* __restrict__ verdict) {
  size_t t = gtid();
  if (t >= m) return;
  uint32_t i = entries[t];
  if (status[i] != DEC_OK) {
    verdict[i] = 0;
    return;
  }
  jac<F> S = jac_from_aff(ld_aff_aos<F>(sig_aff, i));
  jac<F> Hq = ld_jac_aos<F>(q_pts, i);
  bool ok;
  if constexpr (sizeof(F) == sizeof(fp)) {
    ok = check_g1sig(S, h2c_clear_g1(Hq), ld_aff_aos<fp2>(key_aff, 0));
  } else {
    ok = check_g2sig(S, h2c_clear_g2(Hq), ld_aff_aos<fp>(key_aff, 0));
  }
  verdict[i] = ok ? 1 : 0;
}

// verdict for every entry of a passing group: status == OK

hipError_t launch_group_check(int sig_g2, const uint32_t* A, const uint32_t* B, size_t ngroups, const uint32_t* key_aff,
                              uint8_t* pass, hipStream_t st) {
  if (sig_g2)
    hipLaunchKernelGGL(k_group_check<fp2>, dim3(nblk(ngroups, GC_THREADS / 2)), dim3(GC_THREADS), 0, st, A, B, ngroups,
                       key_aff, pass);
  else
    hipLaunchKernelGGL(k_group_check<fp>, dim3(nblk(ngroups, GC_THREADS / 2)), dim3(GC_THREADS), 0, st, A, B, ngroups,
                       key_aff, pass);
  return hipGetLastError();
}


hipError_t launch_leaf_check(int sig_g2, const uint32_t* entries, size_t m, const uint32_t* sig_aff, const uint32_t* q_pts,
                             const uint32_t* key_aff, const uint8_t* status, uint8_t* verdict, hipStream_t st) {
  if (!m) return hipSuccess;
  if (sig_g2)
    hipLaunchKernelGGL(k_leaf_check<fp2>, dim3(nblk(m, 64)), dim3(64), 0, st, entries, m, sig_aff, q_pts, key_aff, status,
                       verdict);
  else
    hipLaunchKernelGGL(k_leaf_check<fp>, dim3(nblk(m, 64)), dim3(64), 0, st, entries, m, sig_aff, q_pts, key_aff, status,
                       verdict);
  return hipGetLastError();
}


DH_COUNTER_ACCESSOR(check)

}  // namespace dh
