"""Pure-Python BLS12-381 model — TEST INFRASTRUCTURE ONLY (small cases).

This is the slow, readable restatement used to pin curve constants against the
reference's known-answer tests and to cross-check the C oracle (`oracle/bls_oracle.c`).
It is never imported by the product path (`drand_amd/`, `libdrandhip`).

What it restates (the reference's arithmetic lives in un-vendored Go modules):
  * kyber v1.1.18 `sign/bls.Verify` / `sign/tbls` as called from
    /root/reference/crypto/schemes.go:70-72 (VerifyBeacon) and
    /root/reference/chain/beacon/chainstore.go:202,207 (Recover / VerifyRecovered);
  * kyber-bls12381 v0.2.5 point codec (ZCash compressed) and hash-to-curve DSTs;
  * kilic/bls12-381 v0.1.0 field / SSWU / isogeny / pairing.
Published algorithms followed: RFC 9380 (hash_to_curve, expand_message_xmd, SSWU,
isogeny maps of Appendix E.2/E.3), the ZCash BLS12-381 serialisation format, and the
optimal-ate pairing over |u| = 0xd201000000010000.

Pinned by: /root/reference/crypto/schemes_test.go:81-130 (TestVerifyBeacon, 4 beacons)
and /root/reference/crypto/curve_test.go:10-31 (TestBLS12381Compatv112) — see
tests/test_oracle.py (KATs in tests/kat.py).
"""
import hashlib

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
U_ABS = 0xd201000000010000  # u = -U_ABS

DST_G2 = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
DST_G1 = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"

# ----------------------------------------------------------------------------- Fp

def finv(a):
    return pow(a % P, P - 2, P)


def fsqrt(a):
    """Returns a square root of a mod P or None (p = 3 mod 4)."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def f_is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def sgn0_fp(a):
    return (a % P) & 1

# ----------------------------------------------------------------------------- Fp2 (tuples (c0, c1) = c0 + c1*i, i^2 = -1)

def f2(a, b=0):
    return (a % P, b % P)


F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2add(x, y):
    return ((x[0] + y[0]) % P, (x[1] + y[1]) % P)


def f2sub(x, y):
    return ((x[0] - y[0]) % P, (x[1] - y[1]) % P)


def f2neg(x):
    return ((-x[0]) % P, (-x[1]) % P)


def f2mul(x, y):
    a, b = x
    c, d = y
    return ((a * c - b * d) % P, (a * d + b * c) % P)


def f2sqr(x):
    return f2mul(x, x)


def f2inv(x):
    a, b = x
    n = finv(a * a + b * b)
    return (a * n % P, (-b) * n % P)


def f2conj(x):
    return (x[0], (-x[1]) % P)


def f2pow(x, e):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2mul(r, x)
        x = f2mul(x, x)
        e >>= 1
    return r


def f2_is_square(x):
    a, b = x
    return f_is_square(a * a + b * b)


def f2sqrt(x):
    """A square root of x in Fp2, or None."""
    a, b = x
    if b == 0:
        s = fsqrt(a)
        if s is not None:
            return (s, 0)
        s = fsqrt(-a)
        return (0, s)
    n = fsqrt(a * a + b * b)
    if n is None:
        return None
    inv2 = finv(2)
    t = (a + n) * inv2 % P
    s = fsqrt(t)
    if s is None:
        t = (a - n) * inv2 % P
        s = fsqrt(t)
        if s is None:
            return None
    y = (s, b * finv(2 * s) % P)
    assert f2sqr(y) == (a % P, b % P)
    return y


def sgn0_fp2(x):
    s0 = x[0] & 1
    z0 = x[0] == 0
    s1 = x[1] & 1
    return s0 | (z0 & s1)

# ----------------------------------------------------------------------------- generic short-Weierstrass ops (affine, None = infinity)
# A field "kind" bundles add/sub/mul/inv/zero/one so one implementation serves E1, E2 and E(Fp12).


class Fld:
    def __init__(self, add, sub, mul, inv, neg, zero, one, eq=None):
        self.add, self.sub, self.mul, self.inv, self.neg = add, sub, mul, inv, neg
        self.zero, self.one = zero, one
        self.eq = eq or (lambda a, b: a == b)


FP = Fld(lambda a, b: (a + b) % P, lambda a, b: (a - b) % P, lambda a, b: a * b % P,
         finv, lambda a: (-a) % P, 0, 1)
FP2 = Fld(f2add, f2sub, f2mul, f2inv, f2neg, F2_ZERO, F2_ONE)


def ec_add(F, Pt, Qt, a=None):
    if Pt is None:
        return Qt
    if Qt is None:
        return Pt
    x1, y1 = Pt
    x2, y2 = Qt
    if F.eq(x1, x2):
        if F.eq(y1, F.neg(y2)):
            return None
        return ec_dbl(F, Pt, a)
    lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def ec_dbl(F, Pt, a=None):
    if Pt is None:
        return None
    x1, y1 = Pt
    if F.eq(y1, F.zero):
        return None
    three_x2 = F.mul(F.add(F.add(F.one, F.one), F.one), F.mul(x1, x1))
    if a is not None:
        three_x2 = F.add(three_x2, a)
    lam = F.mul(three_x2, F.inv(F.add(y1, y1)))
    x3 = F.sub(F.mul(lam, lam), F.add(x1, x1))
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def ec_neg(F, Pt):
    if Pt is None:
        return None
    return (Pt[0], F.neg(Pt[1]))


def ec_mul(F, Pt, k, a=None):
    if k < 0:
        return ec_mul(F, ec_neg(F, Pt), -k, a)
    Rr = None
    Q = Pt
    while k:
        if k & 1:
            Rr = ec_add(F, Rr, Q, a)
        Q = ec_dbl(F, Q, a)
        k >>= 1
    return Rr


B1 = 4
B2 = (4, 4)


def g1_on_curve(Pt):
    if Pt is None:
        return True
    x, y = Pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(Pt):
    if Pt is None:
        return True
    x, y = Pt
    return f2sub(f2sqr(y), f2add(f2mul(f2sqr(x), x), B2)) == F2_ZERO


G1_GEN = (0x17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb,
          0x08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1)
G2_GEN = ((0x024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8,
           0x13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e),
          (0x0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801,
           0x0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be))

# ----------------------------------------------------------------------------- ZCash compressed codec


class DecodeError(Exception):
    pass


HALF_P = (P - 1) // 2


def g1_compress(Pt):
    if Pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = Pt
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    if y > HALF_P:
        b[0] |= 0x20
    return bytes(b)


def g1_decompress(b, subgroup_check=True):
    if len(b) != 48:
        raise DecodeError("bad length")
    flags = b[0]
    if not flags & 0x80:
        raise DecodeError("not compressed")
    if flags & 0x40:
        if (flags & 0x3F) != 0 or any(b[1:]):
            raise DecodeError("bad infinity encoding")
        return None
    sign = bool(flags & 0x20)
    x = int.from_bytes(bytes([flags & 0x1F]) + b[1:], "big")
    if x >= P:
        raise DecodeError("x >= p")
    y = fsqrt(x * x * x + B1)
    if y is None:
        raise DecodeError("not on curve")
    if (y > HALF_P) != sign:
        y = P - y
    Pt = (x, y)
    if subgroup_check and ec_mul(FP, Pt, R) is not None:
        raise DecodeError("not in subgroup")
    return Pt


def f2_lex_largest(y):
    if y[1] != 0:
        return y[1] > HALF_P
    return y[0] > HALF_P


def g2_compress(Pt):
    if Pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = Pt
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80
    if f2_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


def g2_decompress(b, subgroup_check=True):
    if len(b) != 96:
        raise DecodeError("bad length")
    flags = b[0]
    if not flags & 0x80:
        raise DecodeError("not compressed")
    if flags & 0x40:
        if (flags & 0x3F) != 0 or any(b[1:]):
            raise DecodeError("bad infinity encoding")
        return None
    sign = bool(flags & 0x20)
    x1 = int.from_bytes(bytes([flags & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:], "big")
    if x0 >= P or x1 >= P:
        raise DecodeError("x >= p")
    x = (x0, x1)
    y = f2sqrt(f2add(f2mul(f2sqr(x), x), B2))
    if y is None:
        raise DecodeError("not on curve")
    if f2_lex_largest(y) != sign:
        y = f2neg(y)
    Pt = (x, y)
    if subgroup_check and ec_mul(FP2, Pt, R) is not None:
        raise DecodeError("not in subgroup")
    return Pt

# ----------------------------------------------------------------------------- hash to field (RFC 9380 §5.3.1 expand_message_xmd with SHA-256)


def expand_message_xmd(msg, dst, len_in_bytes):
    b_in_bytes, s_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(s_in_bytes)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    b1 = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = b1
    prev = b1
    for i in range(2, ell + 1):
        prev = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, prev)) + bytes([i]) + dst_prime).digest()
        out += prev
    return out[:len_in_bytes]


def hash_to_field_fp(msg, dst, count):
    L = 64
    u = expand_message_xmd(msg, dst, count * L)
    return [int.from_bytes(u[i * L:(i + 1) * L], "big") % P for i in range(count)]


def hash_to_field_fp2(msg, dst, count):
    L = 64
    u = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e0 = int.from_bytes(u[(2 * i) * L:(2 * i + 1) * L], "big") % P
        e1 = int.from_bytes(u[(2 * i + 1) * L:(2 * i + 2) * L], "big") % P
        out.append((e0, e1))
    return out

# ----------------------------------------------------------------------------- SSWU + isogenies (RFC 9380 §6.6.2, §8.8, Appendix E)

# G1: E1' : y^2 = x^3 + A1' x + B1', Z = 11
A1P = 0x144698a3b8e9433d693a02c96d4982b0ea985383ee66a8d8e8981aefd881ac98936f8da0e0f97f5cf428082d584c1d
B1P = 0x12e2908d11688030018b12e8753eee3b2016c1f0f24f4070a0b9c14fcef35ef55a23215a316ceaa5d1cc48e98e172be0
Z1 = 11

# G2: E2' : y^2 = x^3 + 240 i x + 1012 (1 + i), Z = -(2 + i)
A2P = (0, 240)
B2P = (1012, 1012)
Z2 = f2(-2, -1)


def sswu_generic(F, is_square, sqrt, sgn0, A, B, Z, u):
    tv1 = F.add(F.mul(F.mul(Z, Z), F.mul(F.mul(u, u), F.mul(u, u))), F.mul(Z, F.mul(u, u)))
    if F.eq(tv1, F.zero):
        x1 = F.mul(B, F.inv(F.mul(Z, A)))
    else:
        x1 = F.mul(F.mul(F.neg(B), F.inv(A)), F.add(F.one, F.inv(tv1)))
    gx1 = F.add(F.add(F.mul(F.mul(x1, x1), x1), F.mul(A, x1)), B)
    if is_square(gx1):
        x, y = x1, sqrt(gx1)
    else:
        x2 = F.mul(F.mul(Z, F.mul(u, u)), x1)
        gx2 = F.add(F.add(F.mul(F.mul(x2, x2), x2), F.mul(A, x2)), B)
        x, y = x2, sqrt(gx2)
    if sgn0(u) != sgn0(y):
        y = F.neg(y)
    return (x, y)


def sswu_g1(u):
    return sswu_generic(FP, f_is_square, fsqrt, sgn0_fp, A1P, B1P, Z1, u)


def sswu_g2(u):
    return sswu_generic(FP2, f2_is_square, f2sqrt, sgn0_fp2, A2P, B2P, Z2, u)


ISO11_XNUM = [
    0x11a05f2b1e833340b809101dd99815856b303e88a2d7005ff2627b56cdb4e2c85610c2d5f2e62d6eaeac1662734649b7,
    0x17294ed3e943ab2f0588bab22147a81c7c17e75b2f6a8417f565e33c70d1e86b4838f2a6f318c356e834eef1b3cb83bb,
    0xd54005db97678ec1d1048c5d10a9a1bce032473295983e56878e501ec68e25c958c3e3d2a09729fe0179f9dac9edcb0,
    0x1778e7166fcc6db74e0609d307e55412d7f5e4656a8dbf25f1b33289f1b330835336e25ce3107193c5b388641d9b6861,
    0xe99726a3199f4436642b4b3e4118e5499db995a1257fb3f086eeb65982fac18985a286f301e77c451154ce9ac8895d9,
    0x1630c3250d7313ff01d1201bf7a74ab5db3cb17dd952799b9ed3ab9097e68f90a0870d2dcae73d19cd13c1c66f652983,
    0xd6ed6553fe44d296a3726c38ae652bfb11586264f0f8ce19008e218f9c86b2a8da25128c1052ecaddd7f225a139ed84,
    0x17b81e7701abdbe2e8743884d1117e53356de5ab275b4db1a682c62ef0f2753339b7c8f8c8f475af9ccb5618e3f0c88e,
    0x80d3cf1f9a78fc47b90b33563be990dc43b756ce79f5574a2c596c928c5d1de4fa295f296b74e956d71986a8497e317,
    0x169b1f8e1bcfa7c42e0c37515d138f22dd2ecb803a0c5c99676314baf4bb1b7fa3190b2edc0327797f241067be390c9e,
    0x10321da079ce07e272d8ec09d2565b0dfa7dccdde6787f96d50af36003b14866f69b771f8c285decca67df3f1605fb7b,
    0x6e08c248e260e70bd1e962381edee3d31d79d7e22c837bc23c0bf1bc24c6b68c24b1b80b64d391fa9c8ba2e8ba2d229,
]
ISO11_XDEN = [
    0x8ca8d548cff19ae18b2e62f4bd3fa6f01d5ef4ba35b48ba9c9588617fc8ac62b558d681be343df8993cf9fa40d21b1c,
    0x12561a5deb559c4348b4711298e536367041e8ca0cf0800c0126c2588c48bf5713daa8846cb026e9e5c8276ec82b3bff,
    0xb2962fe57a3225e8137e629bff2991f6f89416f5a718cd1fca64e00b11aceacd6a3d0967c94fedcfcc239ba5cb83e19,
    0x3425581a58ae2fec83aafef7c40eb545b08243f16b1655154cca8abc28d6fd04976d5243eecf5c4130de8938dc62cd8,
    0x13a8e162022914a80a6f1d5f43e7a07dffdfc759a12062bb8d6b44e833b306da9bd29ba81f35781d539d395b3532a21e,
    0xe7355f8e4e667b955390f7f0506c6e9395735e9ce9cad4d0a43bcef24b8982f7400d24bc4228f11c02df9a29f6304a5,
    0x772caacf16936190f3e0c63e0596721570f5799af53a1894e2e073062aede9cea73b3538f0de06cec2574496ee84a3a,
    0x14a7ac2a9d64a8b230b3f5b074cf01996e7f63c21bca68a81996e1cdf9822c580fa5b9489d11e2d311f7d99bbdcc5a5e,
    0xa10ecf6ada54f825e920b3dafc7a3cce07f8d1d7161366b74100da67f39883503826692abba43704776ec3a79a1d641,
    0x95fc13ab9e92ad4476d6e3eb3a56680f682b4ee96f7d03776df533978f31c1593174e4b4b7865002d6384d168ecdd0a,
    1,
]
ISO11_YNUM = [
    0x90d97c81ba24ee0259d1f094980dcfa11ad138e48a869522b52af6c956543d3cd0c7aee9b3ba3c2be9845719707bb33,
    0x134996a104ee5811d51036d776fb46831223e96c254f383d0f906343eb67ad34d6c56711962fa8bfe097e75a2e41c696,
    0xcc786baa966e66f4a384c86a3b49942552e2d658a31ce2c344be4b91400da7d26d521628b00523b8dfe240c72de1f6,
    0x1f86376e8981c217898751ad8746757d42aa7b90eeb791c09e4a3ec03251cf9de405aba9ec61deca6355c77b0e5f4cb,
    0x8cc03fdefe0ff135caf4fe2a21529c4195536fbe3ce50b879833fd221351adc2ee7f8dc099040a841b6daecf2e8fedb,
    0x16603fca40634b6a2211e11db8f0a6a074a7d0d4afadb7bd76505c3d3ad5544e203f6326c95a807299b23ab13633a5f0,
    0x4ab0b9bcfac1bbcb2c977d027796b3ce75bb8ca2be184cb5231413c4d634f3747a87ac2460f415ec961f8855fe9d6f2,
    0x987c8d5333ab86fde9926bd2ca6c674170a05bfe3bdd81ffd038da6c26c842642f64550fedfe935a15e4ca31870fb29,
    0x9fc4018bd96684be88c9e221e4da1bb8f3abd16679dc26c1e8b6e6a1f20cabe69d65201c78607a360370e577bdba587,
    0xe1bba7a1186bdb5223abde7ada14a23c42a0ca7915af6fe06985e7ed1e4d43b9b3f7055dd4eba6f2bafaaebca731c30,
    0x19713e47937cd1be0dfd0b8f1d43fb93cd2fcbcb6caf493fd1183e416389e61031bf3a5cce3fbafce813711ad011c132,
    0x18b46a908f36f6deb918c143fed2edcc523559b8aaf0c2462e6bfe7f911f643249d9cdf41b44d606ce07c8a4d0074d8e,
    0xb182cac101b9399d155096004f53f447aa7b12a3426b08ec02710e807b4633f06c851c1919211f20d4c04f00b971ef8,
    0x245a394ad1eca9b72fc00ae7be315dc757b3b080d4c158013e6632d3c40659cc6cf90ad1c232a6442d9d3f5db980133,
    0x5c129645e44cf1102a159f748c4a3fc5e673d81d7e86568d9ab0f5d396a7ce46ba1049b6579afb7866b1e715475224b,
    0x15e6be4e990f03ce4ea50b3b42df2eb5cb181d8f84965a3957add4fa95af01b2b665027efec01c7704b456be69c8b604,
]
ISO11_YDEN = [
    0x16112c4c3a9c98b252181140fad0eae9601a6de578980be6eec3232b5be72e7a07f3688ef60c206d01479253b03663c1,
    0x1962d75c2381201e1a0cbd6c43c348b885c84ff731c4d59ca4a10356f453e01f78a4260763529e3532f6102c2e49a03d,
    0x58df3306640da276faaae7d6e8eb15778c4855551ae7f310c35a5dd279cd2eca6757cd636f96f891e2538b53dbf67f2,
    0x16b7d288798e5395f20d23bf89edb4d1d115c5dbddbcd30e123da489e726af41727364f2c28297ada8d26d98445f5416,
    0xbe0e079545f43e4b00cc912f8228ddcc6d19c9f0f69bbb0542eda0fc9dec916a20b15dc0fd2ededda39142311a5001d,
    0x8d9e5297186db2d9fb266eaac783182b70152c65550d881c5ecd87b6f0f5a6449f38db9dfa9cce202c6477faaf9b7ac,
    0x166007c08a99db2fc3ba8734ace9824b5eecfdfa8d0cf8ef5dd365bc400a0051d5fa9c01a58b1fb93d1a1399126a775c,
    0x16a3ef08be3ea7ea03bcddfabba6ff6ee5a4375efa1f4fd7feb34fd206357132b920f5b00801dee460ee415a15812ed9,
    0x1866c8ed336c61231a1be54fd1d74cc4f9fb0ce4c6af5920abc5750c4bf39b4852cfe2f7bb9248836b233d9d55535d4a,
    0x167a55cda70a6e1cea820597d94a84903216f763e13d87bb5308592e7ea7d4fbc7385ea3d529b35e346ef48bb8913f55,
    0x4d2f259eea405bd48f010a01ad2911d9c6dd039bb61a6290e591b36e636a5c871a5c29f4f83060400f8b49cba8f6aa8,
    0xaccbb67481d033ff5852c1e48c50c477f94ff8aefce42d28c0f9a88cea7913516f968986f7ebbea9684b529e2561092,
    0xad6b9514c767fe3c3613144b45f1496543346d98adf02267d5ceef9a00d9b8693000763e3b90ac11e99b138573345cc,
    0x2660400eb2e4f3b628bdd0d53cd76f2bf565b94e72927c1cb748df27942480e420517bd8714cc80d1fadc1326ed06f7,
    0xe0fa1d816ddc03e6b24255e0d7819c171c40f65e273b853324efcd6356caa205ca2f570f13497804415473a1d634b8f,
    1,
]

_C = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa00
ISO3_XNUM = [
    (0x5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6,
     0x5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6),
    (0, 0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a),
    (0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e,
     0x8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d),
    (0x171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1, 0),
]
ISO3_XDEN = [
    (0, 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63),
    (0xc, 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f),
    (1, 0),
]
ISO3_YNUM = [
    (0x1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706,
     0x1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706),
    (0, 0x5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be),
    (0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c,
     0x8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f),
    (0x124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10, 0),
]
ISO3_YDEN = [
    (0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb,
     0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb),
    (0, 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3),
    (0x12, 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99),
    (1, 0),
]


def _horner(F, coeffs, x):
    acc = F.zero
    for c in reversed(coeffs):
        acc = F.add(F.mul(acc, x), c)
    return acc


def iso_map_g1(Pt):
    x, y = Pt
    xn = _horner(FP, ISO11_XNUM, x)
    xd = _horner(FP, ISO11_XDEN, x)
    yn = _horner(FP, ISO11_YNUM, x)
    yd = _horner(FP, ISO11_YDEN, x)
    if xd == 0 or yd == 0:
        return None
    return (xn * finv(xd) % P, y * yn % P * finv(yd) % P)


def iso_map_g2(Pt):
    x, y = Pt
    xn = _horner(FP2, ISO3_XNUM, x)
    xd = _horner(FP2, ISO3_XDEN, x)
    yn = _horner(FP2, ISO3_YNUM, x)
    yd = _horner(FP2, ISO3_YDEN, x)
    if xd == F2_ZERO or yd == F2_ZERO:
        return None
    return (f2mul(xn, f2inv(xd)), f2mul(f2mul(y, yn), f2inv(yd)))


H_EFF_G1 = 0xd201000000010001
H_EFF_G2 = 0xbc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551


def hash_to_g1(msg, dst):
    u0, u1 = hash_to_field_fp(msg, dst, 2)
    Q0 = iso_map_g1(sswu_g1(u0))
    Q1 = iso_map_g1(sswu_g1(u1))
    return ec_mul(FP, ec_add(FP, Q0, Q1), H_EFF_G1)


def hash_to_g2(msg, dst):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    Q0 = iso_map_g2(sswu_g2(u0))
    Q1 = iso_map_g2(sswu_g2(u1))
    return ec_mul(FP2, ec_add(FP2, Q0, Q1), H_EFF_G2)

# ----------------------------------------------------------------------------- Fp12 = Fp[w]/(w^12 - 2 w^6 + 2); i = w^6 - 1, w^6 = 1 + i


def _p12_mul(a, b):
    r = [0] * 23
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                r[i + j] += x * y
    for k in range(22, 11, -1):
        c = r[k]
        if c:
            # w^12 = 2 w^6 - 2
            r[k - 6] += 2 * c
            r[k - 12] -= 2 * c
    return tuple(v % P for v in r[:12])


def _poly_deg(a):
    d = len(a) - 1
    while d >= 0 and a[d] % P == 0:
        d -= 1
    return d


def _p12_inv(a):
    # extended Euclid over Fp[w] against the modulus
    mod = [2, 0, 0, 0, 0, 0, P - 2, 0, 0, 0, 0, 0, 1]
    lm, hm = [1] + [0] * 12, [0] * 13
    low, high = list(a) + [0], mod[:]
    while _poly_deg(low) > 0:
        dl, dh = _poly_deg(low), _poly_deg(high)
        # r = high // low
        rr = [0] * 13
        temp = high[:]
        inv_lead = finv(low[dl])
        for i in range(dh - dl, -1, -1):
            c = temp[dl + i] * inv_lead % P
            rr[i] = c
            for j in range(dl + 1):
                temp[i + j] = (temp[i + j] - c * low[j]) % P
        nm, new = hm[:], high[:]
        for i in range(13):
            for j in range(13 - i):
                nm[i + j] = (nm[i + j] - lm[i] * rr[j]) % P
                new[i + j] = (new[i + j] - low[i] * rr[j]) % P
        lm, low, hm, high = nm, new, lm, low
    inv0 = finv(low[0])
    return tuple(x * inv0 % P for x in lm[:12])


P12_ONE = (1,) + (0,) * 11
P12_ZERO = (0,) * 12
FP12 = Fld(lambda a, b: tuple((x + y) % P for x, y in zip(a, b)),
           lambda a, b: tuple((x - y) % P for x, y in zip(a, b)),
           _p12_mul, _p12_inv, lambda a: tuple((-x) % P for x in a), P12_ZERO, P12_ONE)


def _fp_to_p12(a):
    return (a % P,) + (0,) * 11


def _fp2_to_p12(a):
    # a0 + a1 i = a0 + a1 (w^6 - 1)
    r = [0] * 12
    r[0] = (a[0] - a[1]) % P
    r[6] = a[1] % P
    return tuple(r)


_W = tuple(1 if i == 1 else 0 for i in range(12))
_W2 = _p12_mul(_W, _W)
_W3 = _p12_mul(_W2, _W)
_W2_INV = _p12_inv(_W2)
_W3_INV = _p12_inv(_W3)


def untwist(Q):
    x, y = Q
    return (_p12_mul(_fp2_to_p12(x), _W2_INV), _p12_mul(_fp2_to_p12(y), _W3_INV))


def p12_pow(a, e):
    r = P12_ONE
    while e:
        if e & 1:
            r = _p12_mul(r, a)
        a = _p12_mul(a, a)
        e >>= 1
    return r


def _line(T1, T2, Pq):
    """Line through T1,T2 (points in E(Fp12)) evaluated at Pq (in E(Fp12))."""
    x1, y1 = T1
    x2, y2 = T2
    xp, yp = Pq
    if x1 != x2:
        lam = _p12_mul(FP12.sub(y2, y1), _p12_inv(FP12.sub(x2, x1)))
    elif y1 == y2:
        three = _fp_to_p12(3)
        lam = _p12_mul(_p12_mul(three, _p12_mul(x1, x1)), _p12_inv(FP12.add(y1, y1)))
    else:
        return FP12.sub(xp, x1)
    return FP12.sub(FP12.sub(yp, y1), _p12_mul(lam, FP12.sub(xp, x1)))


def miller_loop(Pt, Q):
    """f_{|u|,Q}(P), conjugation for the negative u folded in by the caller via final_exp."""
    if Pt is None or Q is None:
        return P12_ONE
    Qt = untwist(Q)
    Pp = (_fp_to_p12(Pt[0]), _fp_to_p12(Pt[1]))
    Tt = Qt
    f = P12_ONE
    for bit in bin(U_ABS)[3:]:
        f = _p12_mul(_p12_mul(f, f), _line(Tt, Tt, Pp))
        Tt = ec_dbl(FP12, Tt)
        if bit == "1":
            f = _p12_mul(f, _line(Tt, Qt, Pp))
            Tt = ec_add(FP12, Tt, Qt)
    return f


FINAL_EXP = (P ** 12 - 1) // R


def final_exp(f):
    return p12_pow(f, FINAL_EXP)


def pairing(Pt, Q):
    # u < 0: e(P,Q) = conj(f_{|u|,Q}(P))^{(p^12-1)/r} = inverse of the unconjugated value
    return _p12_inv(final_exp(miller_loop(Pt, Q)))


def pairing_check(pairs):
    """True iff prod e(P_i, Q_i) == 1."""
    f = P12_ONE
    for Pt, Q in pairs:
        f = _p12_mul(f, miller_loop(Pt, Q))
    return final_exp(f) == P12_ONE

# ----------------------------------------------------------------------------- drand schemes (crypto/schemes.go)


SCHEMES = {
    # name: (sig group, digest kind, hash DST)
    "pedersen-bls-chained": ("G2", "chained", DST_G2),
    "pedersen-bls-unchained": ("G2", "unchained", DST_G2),
    "bls-unchained-on-g1": ("G1", "unchained", DST_G2),       # legacy: G2 DST reused for hash-to-G1
    "bls-unchained-g1-rfc9380": ("G1", "unchained", DST_G1),  # quicknet (absent from the reference snapshot)
}


def digest_beacon(scheme, round_, prev):
    """crypto/schemes.go:106-114 (chained), :147-151 / :187-191 (unchained)."""
    h = hashlib.sha256()
    if SCHEMES[scheme][1] == "chained" and prev:
        h.update(prev)
    h.update(round_.to_bytes(8, "big"))
    return h.digest()


def hash_msg(scheme, msg):
    grp, _, dst = SCHEMES[scheme]
    return hash_to_g2(msg, dst) if grp == "G2" else hash_to_g1(msg, dst)


def verify(scheme, pk_bytes, msg, sig_bytes):
    """bls.Verify semantics: decode sig (with subgroup check), hash, 2-pairing check."""
    grp = SCHEMES[scheme][0]
    try:
        if grp == "G2":
            pk = g1_decompress(pk_bytes)
            sig = g2_decompress(sig_bytes)
        else:
            pk = g2_decompress(pk_bytes)
            sig = g1_decompress(sig_bytes)
    except DecodeError:
        return False
    if sig is None or pk is None:
        return False
    H = hash_msg(scheme, msg)
    if grp == "G2":
        # e(pk, H) == e(g1, sig)
        return pairing_check([(pk, H), (ec_neg(FP, G1_GEN), sig)])
    return pairing_check([(H, pk), (ec_neg(FP, sig), G2_GEN)])


def verify_beacon(scheme, pk_bytes, round_, sig_bytes, prev=b""):
    return verify(scheme, pk_bytes, digest_beacon(scheme, round_, prev), sig_bytes)


def sign(scheme, sk, msg):
    H = hash_msg(scheme, msg)
    if SCHEMES[scheme][0] == "G2":
        return g2_compress(ec_mul(FP2, H, sk))
    return g1_compress(ec_mul(FP, H, sk))


def public_key(scheme, sk):
    if SCHEMES[scheme][0] == "G2":
        return g1_compress(ec_mul(FP, G1_GEN, sk))
    return g2_compress(ec_mul(FP2, G2_GEN, sk))


def randomness(sig_bytes):
    """crypto/schemes.go:249-252."""
    return hashlib.sha256(sig_bytes).digest()
