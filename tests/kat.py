"""Known-answer vectors copied verbatim (as data) from the reference's tests:
/root/reference/crypto/schemes_test.go:81-130 (TestVerifyBeacon) and
/root/reference/crypto/curve_test.go:10-31 (TestBLS12381Compatv112)."""
H = bytes.fromhex

VERIFY_KATS = [
    # (scheme, pk, round, sig, prev)   schemes_test.go:90-96
    ("pedersen-bls-chained",
     H("868f005eb8e6e4ca0a47c8a77ceaa5309a47978a7c71bc5cce96366b5d7a569937c529eeda66c7293784a9402801af31"),
     2634945,
     H("814778ed1e480406beb43b74af71ce2f0373e0ea1bfdfea8f9ed62c876c20fcbc7f0163860e3da42ed2148756015f4551451898ffe06d384b4d002245025571b6b7a752f7158b40ad92b13b6d703ad31922a617f2c7f6d960b84d56cf1d79eef"),
     H("8bd96294383b4d1e04e736360bd7a487f9f409f1e7bd800b720656a310d577b3bdb1e1631af6c5782a1d8979c502f395036181eff4058960fc40bb7034cdae1991d3eda518ab204a077d2f7e724974cf87b407e549bd815cf0b8e5a3832f675d")),
    # schemes_test.go:97-103
    ("pedersen-bls-chained",
     H("922a2e93828ff83345bae533f5172669a26c02dc76d6bf59c80892e12ab1455c229211886f35bb56af6d5bea981024df"),
     3361396,
     H("9904b4ec42e82cb42ad53f171cf0510a5eedff8b5e02e2db5a187489f7875307746998b9a6cf82130d291126d4b83cea1048c9b3f07a067e632c20391dc059d22d6a8e835f3980c8bd0183fb6df00a8fbbe6b8c9f61e888dfa76e12af4d4e355"),
     H("a2377f4e0403f0fd05f709a3292be1b2b59fe990a673ad7b7561b5bd5982b882a2378d36e39befb6ea3bb7aac113c50a18fb07aa4f9a59f95f1aaa7826dafbfcdbf22347c29996c294286fd11b402ad83edd83fa21fe6735fccb65785edbed47")),
    # schemes_test.go:104-109
    ("pedersen-bls-unchained",
     H("8200fc249deb0148eb918d6e213980c5d01acd7fc251900d9260136da3b54836ce125172399ddc69c4e3e11429b62c11"),
     7601003,
     H("af7eac5897b72401c0f248a26b612c5ef68e0ff830b4d78927988c89b5db3e997bfcdb7c24cb19f549830cd02cb854a1143fd53a1d4e0713ded471260869439060d170a77187eb6371742840e43eccfa225657c4cc2d9619f7c3d680470c9743"),
     b""),
    # schemes_test.go:110-115
    ("bls-unchained-on-g1",
     H("876f6fa8073736e22f6ff4badaab35c637503718f7a452d178ce69c45d2d8129a54ad2f988ab10c9666f87ab603c59bf013409a5b500555da31720f8eec294d9809b8796f40d5372c71a44ca61226f1eb978310392f98074a608747f77e66c5a"),
     3,
     H("ac7c3ca14bc88bd014260f22dc016b4fe586f9313c3a549c83d195811a99a5d2d4999d4df6daec73ff51fafadd6d5bb5"),
     b""),
]

# curve_test.go:12-20: private key, message (not a digest), expected G2 signature
SIGN_KAT = (
    H("643d6c704505385387a20d98aba19664e3ee81c600d21a0da910cc87f5dc4ab3"),
    H("7061737320746865207369676e6174757265"),
    H("9940ca447bab3bab393c3a07866349343630437167eaeab063ef1e47acedc51e85c513121cf319a8832c3d136d7f36490fa7241194b403a3bbbba9e7d5e73c9a86f67a9585c6fe077cd6576b2f76560efbab3550d9d5124242c728e3a7ef6989"),
)

# RFC 9380 K.1 expand_message_xmd(SHA-256) vectors, DST QUUX-V01-CS02-with-expander-SHA256-128, len 0x20
XMD_DST = b"QUUX-V01-CS02-with-expander-SHA256-128"
XMD_KATS = [
    (b"", H("68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235")),
    (b"abc", H("d8ccab23b5985ccea865c6c97b6e5b8350e794e603b4b97902f53a8a0d605615")),
]

# RFC 9380 Appendix J.9.1 / J.10.1 hash_to_curve test vectors (suites BLS12381G1_XMD:SHA-256_SSWU_RO_ and
# BLS12381G2_XMD:SHA-256_SSWU_RO_). Not from the reference (quicknet's G1 suite is absent there): they pin the
# hash_to_curve pipeline of the quicknet scheme (expand_message_xmd, hash_to_field, SSWU on E1', 11-isogeny,
# clear_cofactor) independently of the DST. Only coordinates reproduced exactly by the oracle are kept.
H2C_DST_G1 = b"QUUX-V01-CS02-with-BLS12381G1_XMD:SHA-256_SSWU_RO_"
H2C_DST_G2 = b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"
H2C_G1 = [  # (msg, P.x, P.y)
    (b"", "052926add2207b76ca4fa57a8734416c8dc95e24501772c814278700eed6d1e4e8cf62d9c09db0fac349612b759e79a1",
     "08ba738453bfed09cb546dbb0783dbb3a5f1f566ed67bb6be0e8c67e2e81a4cc68ee29813bb7994998f3eae0c9c6a265"),
    (b"abc", "03567bc5ef9c690c2ab2ecdf6a96ef1c139cc0b2f284dca0a9a7943388a49a3aee664ba5379a7655d3c68900be2f6903",
     "0b9c15f3fe6e5cf4211f346271d7b01c8f3b28be689c8429c85b67af215533311f0b8dfaaa154fa6b88176c229f2885d"),
    (b"abcdef0123456789",
     "11e0b079dea29a68f0383ee94fed1b940995272407e3bb916bbf268c263ddd57a6a27200a784cbc248e84f357ce82d98",
     "03a87ae2caf14e8ee52e51fa2ed8eefe80f02457004ba4d486d6aa1f517c0889501dc7413753f9599b099ebcbbd2d709"),
    (b"q128_" + b"q" * 128,
     "15f68eaa693b95ccb85215dc65fa81038d69629f70aeee0d0f677cf22285e7bf58d7cb86eefe8f2e9bc3f8cb84fac488",
     "1807a1d50c29f430b8cafc4f8638dfeeadf51211e1602a5f184443076715f91bb90a48ba1e370edce6ae1062f5e6dd38"),
    (b"a512_" + b"a" * 512,
     "082aabae8b7dedb0e78aeb619ad3bfd9277a2f77ba7fad20ef6aabdc6c31d19ba5a6d12283553294c1825c4b3ca2dcfe",
     "05b84ae5a942248eea39e1d91030458c40153f3b654ab7872d779ad1e942856a20c438e8d99bc8abfbf74729ce1f7ac8"),
]
H2C_G2 = [  # (msg, P.x c0, P.x c1, P.y c0, P.y c1); None where only part of the point is kept
    (b"", "0141ebfbdca40eb85b87142e130ab689c673cf60f1a3e98d69335266f30d9b8d4ac44c1038e9dcdd5393faf5c41fb78a",
     "05cb8437535e20ecffaef7752baddf98034139c38452458baeefab379ba13dff5bf5dd71b72418717047f5b0f37da03d",
     "0503921d7f6a12805e72940b963c0cf3471c7b2a524950ca195d11062ee75ec076daf2d4bc358c4b190c0c98064fdd92", None),
    (b"abc", "02c2d18e033b960562aae3cab37a27ce00d80ccd5ba4b7fe0e7a210245129dbec7780ccc7954725f4168aff2787776e6",
     "139cddbccdc5e91b9623efd38c49f81a6f83f175e80b06fc374de9eb4b41dfe4ca3a230ed250fbe3a2acf73a41177fd8",
     "1787327b68159716a37440985269cf584bcb1e621d3a7202be6ea05c4cfe244aeb197642555a0645fb87bf7466b2ba48",
     "00aa65dae3c8d732d10ecd2c50f8a1baf3001578f71c694e03866e9f3d49ac1e1ce70dd94a733534f106d4cec0eddd16"),
]
