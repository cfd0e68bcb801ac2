"""drand_amd/csrc/inv_bingcd.hpp (the library's variable-time Fp inverse) compiled for the host from the same source
and checked against Python's pow(y, -1, p): edge cases and random values of every size. A line-by-line Python
restatement of the algorithm (Pornin's optimized binary GCD, the factor and bound invariants asserted) is checked
against the same inputs. CPU only."""
import os
import random
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
K, ROUNDS = 31, 25

HARNESS = r"""
#include <cstdio>
#include <cstring>
#define DH_HD static inline
#include "inv_bingcd.hpp"
int main() {
  char line[256];
  while (fgets(line, sizeof line, stdin)) {
    uint32_t a[12] = {0};
    size_t n = strcspn(line, "\r\n");
    line[n] = 0;
    for (size_t k = 0; k < n; k++) {  // hex digit k from the right end
      char ch = line[n - 1 - k];
      uint32_t d = ch <= '9' ? ch - '0' : (ch | 32) - 'a' + 10;
      a[k / 8] |= d << (4 * (k % 8));
    }
    dh::bgcd::inverse(a);
    for (int i = 11; i >= 0; i--) printf("%08x", a[i]);
    printf("\n");
  }
  return 0;
}
"""


def restated_inverse(y, m=P):
    """the algorithm of inv_bingcd.hpp in Python, with its invariants asserted"""
    a, b, u, v = y, m, 1, 0
    minv = (-pow(m, -1, 1 << K)) % (1 << K)
    for _ in range(ROUNDS):
        n = max(a.bit_length(), b.bit_length(), 64)
        ab = (a & ((1 << K) - 1)) | ((a >> (n - 33)) << K)
        bb = (b & ((1 << K) - 1)) | ((b >> (n - 33)) << K)
        f0, g0, f1, g1 = 1, 0, 0, 1
        for _ in range(K):
            if ab & 1:
                if ab < bb:
                    ab, bb, f0, g0, f1, g1 = bb, ab, f1, g1, f0, g0
                ab, f0, g0 = ab - bb, f0 - f1, g0 - g1
            ab, f1, g1 = ab >> 1, 2 * f1, 2 * g1
        assert max(abs(f0), abs(g0), abs(f1), abs(g1)) <= 1 << K
        na, nb = a * f0 + b * g0, a * f1 + b * g1
        assert na % (1 << K) == 0 and nb % (1 << K) == 0
        na, nb = na >> K, nb >> K
        if na < 0:
            na, f0, g0 = -na, -f0, -g0
        if nb < 0:
            nb, f1, g1 = -nb, -f1, -g1
        assert na < 1 << 382 and nb < 1 << 382

        def lin_mod(x, fx, yv, fy):
            t = ((m - x) if fx < 0 else x) * abs(fx) + ((m - yv) if fy < 0 else yv) * abs(fy)
            t += ((t * minv) % (1 << K)) * m
            r = t >> K
            assert t % (1 << K) == 0 and r < 3 * m
            return r % m
        a, b, u, v = na, nb, lin_mod(u, f0, v, g0), lin_mod(u, f1, v, g1)
    assert b == 1 and a == 0
    return v


def _inputs():
    rng = random.Random(20261019)
    xs = [1, 2, 3, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 1 << 31, (1 << 31) - 1, (1 << 32) + 1, 1 << 63,
          (1 << 64) - 1, 1 << 380, P - (1 << 200)]
    xs += [rng.randrange(1, P) for _ in range(3000)]
    xs += [rng.randrange(1, 1 << rng.randrange(1, 381)) for _ in range(3000)]
    xs += [(rng.randrange(1, 1 << 40) << rng.randrange(0, 340)) % P or 1 for _ in range(1000)]
    return xs


def test_restatement_matches_pow():
    for y in _inputs()[:2500]:
        assert restated_inverse(y) == pow(y, -1, P), hex(y)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_inv_bingcd_host_build(tmp_path):
    src = tmp_path / "inv_check.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "inv_check"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "drand_amd", "csrc"), str(src), "-o", str(exe)])
    xs = _inputs()
    out = subprocess.run([str(exe)], input="".join("%x\n" % x for x in xs), capture_output=True, text=True,
                         check=True).stdout.split()
    assert len(out) == len(xs)
    for x, o in zip(xs, out):
        assert int(o, 16) == pow(x, -1, P), hex(x)
