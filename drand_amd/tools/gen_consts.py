"""Generate drand_amd/csrc/consts.hpp: BLS12-381 constants in 12x32-bit Montgomery form.

Build tool (not the oracle): it holds the curve / RFC 9380 constants itself, derives the
tower, Frobenius, psi and sqrt_ratio constants, asserts every derived identity
numerically, and writes a header of `__constant__` tables for the HIP kernels.

Sources of the constants: the BLS12-381 curve definition (u = -0xd201000000010000),
RFC 9380 §8.8.1/§8.8.2 (SSWU curves, Z), Appendix E.2/E.3 (11- and 3-isogeny maps),
Appendix F.2.1 (sqrt_ratio). Run: python drand_amd/tools/gen_consts.py
"""
import os

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
U = -0xd201000000010000
MONT = 1 << 384

G1X = 0x17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb
G1Y = 0x08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1
G2X = (0x024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8,
       0x13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e)
G2Y = (0x0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801,
       0x0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be)

A1P = 0x144698a3b8e9433d693a02c96d4982b0ea985383ee66a8d8e8981aefd881ac98936f8da0e0f97f5cf428082d584c1d
B1P = 0x12e2908d11688030018b12e8753eee3b2016c1f0f24f4070a0b9c14fcef35ef55a23215a316ceaa5d1cc48e98e172be0
Z1 = 11
A2P = (0, 240)
B2P = (1012, 1012)
Z2 = ((-2) % P, (-1) % P)

ISO11_XNUM = """11a05f2b1e833340b809101dd99815856b303e88a2d7005ff2627b56cdb4e2c85610c2d5f2e62d6eaeac1662734649b7
17294ed3e943ab2f0588bab22147a81c7c17e75b2f6a8417f565e33c70d1e86b4838f2a6f318c356e834eef1b3cb83bb
d54005db97678ec1d1048c5d10a9a1bce032473295983e56878e501ec68e25c958c3e3d2a09729fe0179f9dac9edcb0
1778e7166fcc6db74e0609d307e55412d7f5e4656a8dbf25f1b33289f1b330835336e25ce3107193c5b388641d9b6861
e99726a3199f4436642b4b3e4118e5499db995a1257fb3f086eeb65982fac18985a286f301e77c451154ce9ac8895d9
1630c3250d7313ff01d1201bf7a74ab5db3cb17dd952799b9ed3ab9097e68f90a0870d2dcae73d19cd13c1c66f652983
d6ed6553fe44d296a3726c38ae652bfb11586264f0f8ce19008e218f9c86b2a8da25128c1052ecaddd7f225a139ed84
17b81e7701abdbe2e8743884d1117e53356de5ab275b4db1a682c62ef0f2753339b7c8f8c8f475af9ccb5618e3f0c88e
80d3cf1f9a78fc47b90b33563be990dc43b756ce79f5574a2c596c928c5d1de4fa295f296b74e956d71986a8497e317
169b1f8e1bcfa7c42e0c37515d138f22dd2ecb803a0c5c99676314baf4bb1b7fa3190b2edc0327797f241067be390c9e
10321da079ce07e272d8ec09d2565b0dfa7dccdde6787f96d50af36003b14866f69b771f8c285decca67df3f1605fb7b
6e08c248e260e70bd1e962381edee3d31d79d7e22c837bc23c0bf1bc24c6b68c24b1b80b64d391fa9c8ba2e8ba2d229"""
ISO11_XDEN = """8ca8d548cff19ae18b2e62f4bd3fa6f01d5ef4ba35b48ba9c9588617fc8ac62b558d681be343df8993cf9fa40d21b1c
12561a5deb559c4348b4711298e536367041e8ca0cf0800c0126c2588c48bf5713daa8846cb026e9e5c8276ec82b3bff
b2962fe57a3225e8137e629bff2991f6f89416f5a718cd1fca64e00b11aceacd6a3d0967c94fedcfcc239ba5cb83e19
3425581a58ae2fec83aafef7c40eb545b08243f16b1655154cca8abc28d6fd04976d5243eecf5c4130de8938dc62cd8
13a8e162022914a80a6f1d5f43e7a07dffdfc759a12062bb8d6b44e833b306da9bd29ba81f35781d539d395b3532a21e
e7355f8e4e667b955390f7f0506c6e9395735e9ce9cad4d0a43bcef24b8982f7400d24bc4228f11c02df9a29f6304a5
772caacf16936190f3e0c63e0596721570f5799af53a1894e2e073062aede9cea73b3538f0de06cec2574496ee84a3a
14a7ac2a9d64a8b230b3f5b074cf01996e7f63c21bca68a81996e1cdf9822c580fa5b9489d11e2d311f7d99bbdcc5a5e
a10ecf6ada54f825e920b3dafc7a3cce07f8d1d7161366b74100da67f39883503826692abba43704776ec3a79a1d641
95fc13ab9e92ad4476d6e3eb3a56680f682b4ee96f7d03776df533978f31c1593174e4b4b7865002d6384d168ecdd0a
1"""
ISO11_YNUM = """90d97c81ba24ee0259d1f094980dcfa11ad138e48a869522b52af6c956543d3cd0c7aee9b3ba3c2be9845719707bb33
134996a104ee5811d51036d776fb46831223e96c254f383d0f906343eb67ad34d6c56711962fa8bfe097e75a2e41c696
cc786baa966e66f4a384c86a3b49942552e2d658a31ce2c344be4b91400da7d26d521628b00523b8dfe240c72de1f6
1f86376e8981c217898751ad8746757d42aa7b90eeb791c09e4a3ec03251cf9de405aba9ec61deca6355c77b0e5f4cb
8cc03fdefe0ff135caf4fe2a21529c4195536fbe3ce50b879833fd221351adc2ee7f8dc099040a841b6daecf2e8fedb
16603fca40634b6a2211e11db8f0a6a074a7d0d4afadb7bd76505c3d3ad5544e203f6326c95a807299b23ab13633a5f0
4ab0b9bcfac1bbcb2c977d027796b3ce75bb8ca2be184cb5231413c4d634f3747a87ac2460f415ec961f8855fe9d6f2
987c8d5333ab86fde9926bd2ca6c674170a05bfe3bdd81ffd038da6c26c842642f64550fedfe935a15e4ca31870fb29
9fc4018bd96684be88c9e221e4da1bb8f3abd16679dc26c1e8b6e6a1f20cabe69d65201c78607a360370e577bdba587
e1bba7a1186bdb5223abde7ada14a23c42a0ca7915af6fe06985e7ed1e4d43b9b3f7055dd4eba6f2bafaaebca731c30
19713e47937cd1be0dfd0b8f1d43fb93cd2fcbcb6caf493fd1183e416389e61031bf3a5cce3fbafce813711ad011c132
18b46a908f36f6deb918c143fed2edcc523559b8aaf0c2462e6bfe7f911f643249d9cdf41b44d606ce07c8a4d0074d8e
b182cac101b9399d155096004f53f447aa7b12a3426b08ec02710e807b4633f06c851c1919211f20d4c04f00b971ef8
245a394ad1eca9b72fc00ae7be315dc757b3b080d4c158013e6632d3c40659cc6cf90ad1c232a6442d9d3f5db980133
5c129645e44cf1102a159f748c4a3fc5e673d81d7e86568d9ab0f5d396a7ce46ba1049b6579afb7866b1e715475224b
15e6be4e990f03ce4ea50b3b42df2eb5cb181d8f84965a3957add4fa95af01b2b665027efec01c7704b456be69c8b604"""
ISO11_YDEN = """16112c4c3a9c98b252181140fad0eae9601a6de578980be6eec3232b5be72e7a07f3688ef60c206d01479253b03663c1
1962d75c2381201e1a0cbd6c43c348b885c84ff731c4d59ca4a10356f453e01f78a4260763529e3532f6102c2e49a03d
58df3306640da276faaae7d6e8eb15778c4855551ae7f310c35a5dd279cd2eca6757cd636f96f891e2538b53dbf67f2
16b7d288798e5395f20d23bf89edb4d1d115c5dbddbcd30e123da489e726af41727364f2c28297ada8d26d98445f5416
be0e079545f43e4b00cc912f8228ddcc6d19c9f0f69bbb0542eda0fc9dec916a20b15dc0fd2ededda39142311a5001d
8d9e5297186db2d9fb266eaac783182b70152c65550d881c5ecd87b6f0f5a6449f38db9dfa9cce202c6477faaf9b7ac
166007c08a99db2fc3ba8734ace9824b5eecfdfa8d0cf8ef5dd365bc400a0051d5fa9c01a58b1fb93d1a1399126a775c
16a3ef08be3ea7ea03bcddfabba6ff6ee5a4375efa1f4fd7feb34fd206357132b920f5b00801dee460ee415a15812ed9
1866c8ed336c61231a1be54fd1d74cc4f9fb0ce4c6af5920abc5750c4bf39b4852cfe2f7bb9248836b233d9d55535d4a
167a55cda70a6e1cea820597d94a84903216f763e13d87bb5308592e7ea7d4fbc7385ea3d529b35e346ef48bb8913f55
4d2f259eea405bd48f010a01ad2911d9c6dd039bb61a6290e591b36e636a5c871a5c29f4f83060400f8b49cba8f6aa8
accbb67481d033ff5852c1e48c50c477f94ff8aefce42d28c0f9a88cea7913516f968986f7ebbea9684b529e2561092
ad6b9514c767fe3c3613144b45f1496543346d98adf02267d5ceef9a00d9b8693000763e3b90ac11e99b138573345cc
2660400eb2e4f3b628bdd0d53cd76f2bf565b94e72927c1cb748df27942480e420517bd8714cc80d1fadc1326ed06f7
e0fa1d816ddc03e6b24255e0d7819c171c40f65e273b853324efcd6356caa205ca2f570f13497804415473a1d634b8f
1"""

_c = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffff
ISO3_XNUM = [
    (0x5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6,
     0x5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6),
    (0, 0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a),
    (0x11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e,
     0x8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d),
    (0x171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1, 0),
]
ISO3_XDEN = [
    (0, (_c << 16) | 0xaa63),
    (0xc, (_c << 16) | 0xaa9f),
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
    ((_c << 16) | 0xa8fb, (_c << 16) | 0xa8fb),
    (0, (_c << 16) | 0xa9d3),
    (0x12, (_c << 16) | 0xaa99),
    (1, 0),
]

# ---------------------------------------------------------------- small Fp2 helpers for derivations


def f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2mul(r, a)
        a = f2mul(a, a)
        e >>= 1
    return r


def f2inv(a):
    n = pow(a[0] * a[0] + a[1] * a[1], P - 2, P)
    return (a[0] * n % P, (-a[1]) * n % P)


def mont(x):
    return (x % P) * MONT % P


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(12)]


def c_fp(x):
    return "{" + ", ".join("0x%08xu" % v for v in limbs(mont(x))) + "}"


def c_fp28(x):
    m = (x % P) * (1 << 392) % P
    return "{" + ", ".join("0x%07xu" % ((m >> (28 * i)) & 0xFFFFFFF) for i in range(14)) + "}"


def c_fp2(a):
    return "{" + c_fp(a[0]) + ", " + c_fp(a[1]) + "}"


def c_exp_words(e):
    n = (e.bit_length() + 31) // 32
    return n, "{" + ", ".join("0x%08xu" % ((e >> (32 * i)) & 0xFFFFFFFF) for i in range(n)) + "}"


DST_G2 = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
DST_G1 = b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"
SHA_IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
SHA_K = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2]


def _ror(x, n):
    return ((x >> n) | (x << (32 - n))) & 0xFFFFFFFF


def sha_compress(h, block):
    wd = [int.from_bytes(block[4 * i:4 * i + 4], "big") for i in range(16)]
    for i in range(16, 64):
        s0 = _ror(wd[i - 15], 7) ^ _ror(wd[i - 15], 18) ^ (wd[i - 15] >> 3)
        s1 = _ror(wd[i - 2], 17) ^ _ror(wd[i - 2], 19) ^ (wd[i - 2] >> 10)
        wd.append((wd[i - 16] + s0 + wd[i - 7] + s1) & 0xFFFFFFFF)
    a, b, c, d, e, f, g, hh = h
    for i in range(64):
        t1 = (hh + (_ror(e, 6) ^ _ror(e, 11) ^ _ror(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + wd[i]) & 0xFFFFFFFF
        t2 = ((_ror(a, 2) ^ _ror(a, 13) ^ _ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & 0xFFFFFFFF
        hh, g, f, e, d, c, b, a = g, f, e, (d + t1) & 0xFFFFFFFF, c, b, a, (t1 + t2) & 0xFFFFFFFF
    return [(x + y) & 0xFFFFFFFF for x, y in zip(h, [a, b, c, d, e, f, g, hh])]


def sha_pad(m, prefix_len):
    """SHA-256 padding of m, which follows prefix_len already-compressed bytes."""
    total = prefix_len + len(m)
    m = m + b"\x80"
    while (prefix_len + len(m)) % 64 != 56:
        m += b"\x00"
    return m + (8 * total).to_bytes(8, "big")


def words(b):
    return [int.from_bytes(b[4 * i:4 * i + 4], "big") for i in range(len(b) // 4)]


def cw(ws):
    return "{" + ", ".join("0x%08xu" % v for v in ws) + "}"


def window_schedule(e, wbits):
    """Left-to-right sliding window over odd digits < 2^wbits.
    Returns [first_index, (nsq << 8) | idx, ...]; idx = (digit - 1) / 2, 0xff = squarings only."""
    b = bin(e)[2:]
    i = 0
    ops = []
    acc = None
    pending_sq = 0
    while i < len(b):
        if b[i] == "0":
            pending_sq += 1
            i += 1
            continue
        j = min(i + wbits, len(b))
        while b[j - 1] == "0":
            j -= 1
        digit = int(b[i:j], 2)
        width = j - i
        if acc is None:
            ops.append((digit - 1) // 2)
            acc = digit
        else:
            pending_sq += width
            while pending_sq > 255:
                ops.append((255 << 8) | 0xFF)
                acc <<= 255
                pending_sq -= 255
            ops.append((pending_sq << 8) | ((digit - 1) // 2))
            acc = (acc << pending_sq) + digit
        pending_sq = 0
        i = j
    if pending_sq:
        ops.append((pending_sq << 8) | 0xFF)
        acc <<= pending_sq
    assert acc == e
    return ops


def main():
    assert (P - 1) % 3 == 0 and P % 4 == 3
    xi = (1, 1)
    # --- G1 endomorphism beta: phi(P) = (beta x, y) = [-u^2] P on G1 (checked in tests/oracle)
    beta = 0x5f19672fdf76ce51ba69c6076a0f77eaddb3a93be6f89688de17d813620a00022e01fffffffefffe
    assert pow(beta, 3, P) == 1 and beta != 1
    # --- psi on the twist
    psi_x = f2inv(f2pow(xi, (P - 1) // 3))
    psi_y = f2inv(f2pow(xi, (P - 1) // 2))
    psi2_x = f2mul(f2pow(psi_x, P), psi_x)  # psi^2 coefficient (conj(conj(x)) = x)
    psi2_y = f2mul(f2pow(psi_y, P), psi_y)
    # --- Frobenius coefficients for Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)
    frob6_c1 = [f2pow(xi, (P ** k - 1) // 3) for k in (1, 2, 3)]
    frob6_c2 = [f2pow(xi, 2 * (P ** k - 1) // 3) for k in (1, 2, 3)]
    frob12_c = [f2pow(xi, (P ** k - 1) // 6) for k in (1, 2, 3)]
    # --- SSWU G1 sqrt_ratio constants (RFC 9380 F.2.1.2, q = 3 mod 4)
    sr1_c1 = (P - 3) // 4
    sr1_c2 = pow((-Z1) % P, (P + 1) // 4, P)
    assert sr1_c2 * sr1_c2 % P == (-Z1) % P
    # --- SSWU G2 sqrt_ratio constants (RFC 9380 F.2.1.1, generic)
    q = P * P
    c1 = 0
    while (q - 1) % (1 << (c1 + 1)) == 0:
        c1 += 1
    assert c1 == 3
    c2 = (q - 1) >> c1
    c3 = (c2 - 1) // 2
    c4 = (1 << c1) - 1
    c5 = 1 << (c1 - 1)
    c6 = f2pow(Z2, c2)
    c7 = f2pow(Z2, (c2 + 1) // 2)
    # --- hash_to_field: 2^256 R^2 so that mont_mul(hi, K) = hi * 2^256 * R
    k256 = (1 << 256) % P
    # --- cofactor / misc scalars
    h_eff_g1 = 0xd201000000010001
    assert h_eff_g1 == 1 - U
    out = []
    w = out.append
    w("// GENERATED by drand_amd/tools/gen_consts.py -- do not edit.")
    w("// BLS12-381 constants in Montgomery form (R = 2^384), 12 x 32-bit little-endian limbs.")
    w("#pragma once")
    w("#include <stdint.h>")
    w("namespace dh {")
    w("namespace cst {")

    def fp_const(name, x):
        w("__device__ __constant__ uint32_t %s[12] = %s;" % (name, c_fp(x)))

    def fp2_const(name, a):
        w("__device__ __constant__ uint32_t %s[2][12] = %s;" % (name, c_fp2(a)))

    fp_const("B1", 4)
    fp2_const("B2", (4, 4))
    fp_const("B2_3", 12)  # 3*b for G1 complete formulas
    fp2_const("B2_3X", (12, 12))
    fp_const("G1X", G1X)
    fp_const("G1Y", G1Y)
    fp2_const("G2X", G2X)
    fp2_const("G2Y", G2Y)
    fp_const("BETA", beta)
    fp2_const("PSI_X", psi_x)
    fp2_const("PSI_Y", psi_y)
    fp2_const("PSI2_X", psi2_x)
    fp2_const("PSI2_Y", psi2_y)
    w("__device__ __constant__ uint32_t FROB6_C1[3][2][12] = {%s};" % ", ".join(c_fp2(a) for a in frob6_c1))
    w("__device__ __constant__ uint32_t FROB6_C2[3][2][12] = {%s};" % ", ".join(c_fp2(a) for a in frob6_c2))
    w("__device__ __constant__ uint32_t FROB12_C[3][2][12] = {%s};" % ", ".join(c_fp2(a) for a in frob12_c))
    fp_const("SSWU1_A", A1P)
    fp_const("SSWU1_B", B1P)
    fp_const("SSWU1_Z", Z1)
    fp_const("SQRT_RATIO1_C2", sr1_c2)
    fp2_const("SSWU2_A", A2P)
    fp2_const("SSWU2_B", B2P)
    fp2_const("SSWU2_Z", Z2)
    fp2_const("SQRT_RATIO2_C6", c6)
    fp2_const("SQRT_RATIO2_C7", c7)
    fp_const("INV2", (P + 1) // 2)  # 1/2
    # norm-based sqrt_ratio over Fp2 (fp2_sqrt_ratio_cm): N(Z) and N(Z)^((p-3)/4)
    nz = (Z2[0] * Z2[0] + Z2[1] * Z2[1]) % P
    fp_const("SSWU2_NZ", nz)
    fp_const("SSWU2_NZ_K", pow(nz, (P - 3) // 4, P))
    w("constexpr bool SIGMA_K_NEG = %s;  // (-1)^((p-3)/4) == -1" % ("true" if pow(P - 1, (P - 3) // 4, P) != 1 else "false"))
    fp_const("K256", k256)
    fp_const("K256R", k256 * MONT % P)  # mont_mul(raw hi, K256R) = Mont(hi * 2^256)
    fp_const("R2", MONT % P)  # c_fp(R) = R^2 mod p: mont_mul(raw x, R2) = Mont(x)
    for name, txt in (("ISO11_XNUM", ISO11_XNUM), ("ISO11_XDEN", ISO11_XDEN), ("ISO11_YNUM", ISO11_YNUM),
                      ("ISO11_YDEN", ISO11_YDEN)):
        cs = [int(t, 16) for t in txt.split()]
        w("constexpr int %s_LEN = %d;" % (name, len(cs)))
        w("__device__ __constant__ uint32_t %s[%d][12] = {%s};" % (name, len(cs), ", ".join(c_fp(c) for c in cs)))
        # the same coefficients for the lazily reduced 28-bit evaluation (fp28.hpp: c 2^392 mod p, 14 x 28-bit limbs)
        w("__device__ __constant__ uint32_t %s_28[%d][14] = {%s};" % (name, len(cs), ", ".join(c_fp28(c) for c in cs)))
    for name, cs in (("ISO3_XNUM", ISO3_XNUM), ("ISO3_XDEN", ISO3_XDEN), ("ISO3_YNUM", ISO3_YNUM),
                     ("ISO3_YDEN", ISO3_YDEN)):
        w("constexpr int %s_LEN = %d;" % (name, len(cs)))
        w("__device__ __constant__ uint32_t %s[%d][2][12] = {%s};" % (name, len(cs), ", ".join(c_fp2(c) for c in cs)))
    # exponents (plain integers, little-endian 32-bit words)
    for name, e in (("EXP_P_MINUS_2", P - 2), ("EXP_P_PLUS_1_DIV_4", (P + 1) // 4),
                    ("EXP_SR1_C1", sr1_c1), ("EXP_SR2_C3", c3), ("EXP_P_MINUS_1_DIV_2", (P - 1) // 2)):
        n, txt = c_exp_words(e)
        w("constexpr int %s_WORDS = %d;" % (name, n))
        w("constexpr int %s_BITS = %d;" % (name, e.bit_length()))
        w("__device__ __constant__ uint32_t %s[%d] = %s;" % (name, n, txt))
    # sliding-window (w = 3, odd powers x^1,3,5,7) schedules for the fixed Fp exponents:
    # entry = (squarings << 8) | table index, index 0xff = squarings only (trailing zeros)
    for name, e in (("SCHED_SQRT", (P + 1) // 4), ("SCHED_SR1_C1", sr1_c1), ("SCHED_INV", P - 2),
                    ("SCHED_LEGENDRE", (P - 1) // 2), ("SCHED_SR2_C3", c3)):
        sched = window_schedule(e, 3)
        w("constexpr int %s_LEN = %d;" % (name, len(sched)))
        # 32-bit entries: a wave-uniform index into a dword table is a scalar (s_load) read; 16-bit entries can only
        # be read by per-lane vector loads, whose latency each step of the chain then waits for
        w("__device__ __constant__ uint32_t %s[%d] = {%s};" % (name, len(sched) + 1, ", ".join("0x%04x" % v for v in sched + [0])))
    w("constexpr uint32_t SR2_C4 = %du;" % c4)
    w("constexpr uint32_t SR2_C5 = %du;" % c5)
    w("constexpr int SR2_C1 = %d;" % c1)
    w("constexpr uint64_t U_ABS = 0x%016xull;" % (-U))
    w("constexpr uint64_t H_EFF_G1 = 0x%016xull;" % h_eff_g1)
    # G2 effective cofactor (RFC 9380 8.8.2), applied once per batch to the RLC sum of SSWU points
    h_eff_g2 = 0xbc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551
    n, txt = c_exp_words(h_eff_g2)
    w("constexpr int H_EFF_G2_WORDS = %d;" % n)
    w("constexpr int H_EFF_G2_BITS = %d;" % h_eff_g2.bit_length())
    w("__device__ __constant__ uint32_t H_EFF_G2[%d] = %s;" % (n, txt))
    # G1 subgroup check / Miller loop parameter |u| as words
    w("__device__ __constant__ uint32_t U_ABS_W[2] = {0x%08xu, 0x%08xu};" % ((-U) & 0xFFFFFFFF, (-U) >> 32))
    # scalar field r (8 x 32-bit limbs, plain) for tbls Lagrange
    w("__device__ __constant__ uint32_t R_LIMBS[8] = {%s};" % ", ".join("0x%08xu" % ((R >> (32 * i)) & 0xFFFFFFFF) for i in range(8)))
    # ---- expand_message_xmd(SHA-256) block templates for a 32-byte message (the beacon digest).
    # Byte layouts (RFC 9380 5.3.1): b0 = H(Z_pad || msg || I2OSP(len,2) || 0 || DST || len(DST)),
    # b_i = H((b0 ^ b_{i-1}) || I2OSP(i,1) || DST || len(DST)). Message-dependent words are zero here
    # and OR-ed in on the device.
    for dname, dst in (("G2", DST_G2), ("G1", DST_G1)):
        assert len(dst) == 43
    w("constexpr int XMD_DST_LEN = 43;")
    w("__device__ __constant__ uint32_t XMD_ZPAD_H[8] = {%s};" % ", ".join("0x%08xu" % v for v in sha_compress(SHA_IV, bytes(64))))
    b0a, b0b, bia, bib = [], [], [], []
    for dst in (DST_G2, DST_G1):
        dstp = dst + bytes([len(dst)])
        per_len = []
        for L in (128, 256):
            m = bytes(32) + L.to_bytes(2, "big") + b"\x00" + dstp
            blocks = sha_pad(m, 64)
            assert len(blocks) == 128
            per_len.append(words(blocks[:64])[8:16])
        b0a.append(per_len)
        b0b.append(words(blocks[64:128]))
        m = bytes(32) + b"\x00" + dstp
        blocks = sha_pad(m, 0)
        assert len(blocks) == 128
        bia.append(words(blocks[:64])[8:16])
        bib.append(words(blocks[64:128]))
    w("__device__ __constant__ uint32_t XMD_B0A[2][2][8] = {%s};" % ", ".join("{" + ", ".join(cw(x) for x in pl) + "}" for pl in b0a))
    w("__device__ __constant__ uint32_t XMD_B0B[2][16] = {%s};" % ", ".join(cw(x) for x in b0b))
    w("__device__ __constant__ uint32_t XMD_BIA[2][8] = {%s};" % ", ".join(cw(x) for x in bia))
    w("__device__ __constant__ uint32_t XMD_BIB[2][16] = {%s};" % ", ".join(cw(x) for x in bib))
    w("}  // namespace cst")
    w("}  // namespace dh")
    path = os.path.join(os.path.dirname(__file__), "..", "csrc", "consts.hpp")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("wrote", os.path.normpath(path))


if __name__ == "__main__":
    main()
