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

// one lane per group: A = sum r sigma, B = sum r Q (pre-cofactor)
template <class F>
__global__ __launch_bounds__(64) void k_group_check(const uint32_t* __restrict__ A, const uint32_t* __restrict__ B,
                                                    size_t ngroups, const uint32_t* __restrict__ key_aff,
                                                    uint8_t* __restrict__ pass) {
  size_t t = gtid();
  if (t >= ngroups) return;
  jac<F> S = ld_jac_aos<F>(A, t);
  jac<F> Hq = ld_jac_aos<F>(B, t);
  bool ok;
  if constexpr (sizeof(F) == sizeof(fp)) {
    ok = check_g1sig(S, h2c_clear_g1(Hq), ld_aff_aos<fp2>(key_aff, 0));
  } else {
    ok = check_g2sig(S, h2c_clear_g2(Hq), ld_aff_aos<fp>(key_aff, 0));
  }
  pass[t] = ok ? 1 : 0;
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
    hipLaunchKernelGGL(k_group_check<fp2>, dim3(nblk(ngroups, 64)), dim3(64), 0, st, A, B, ngroups, key_aff, pass);
  else
    hipLaunchKernelGGL(k_group_check<fp>, dim3(nblk(ngroups, 64)), dim3(64), 0, st, A, B, ngroups, key_aff, pass);
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


}  // namespace dh
