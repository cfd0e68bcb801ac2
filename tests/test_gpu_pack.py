"""Two checks per wave (k_vm.hip k_vm_pairing2 / k_vm_pairing_g1j2 / k_vm_leaf_g1j2): every group check and leaf
launch of a faulty batch's bisection packed (DRANDHIP_VM_PACK=2), for a G1-signature scheme (NP2J on Jacobian sides)
and a G2-signature scheme with the one-lane cofactor clearing (DRANDHIP_NP2C=0: NP2 on affine pair records). The
rejected set must be exactly the corrupted rounds; undecodable rounds among the leaves take the packed kernels'
one-check fallback."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pack", ["2", "0"])
def test_packed_checks(pack):
    env = dict(os.environ, DRANDHIP_VM_PACK=pack, DRANDHIP_BISECT="250,15", DRANDHIP_NP2C="0", DRANDHIP_NP2C_LEAVES="0")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "vm_pack_check.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.strip().splitlines() if x.startswith("{")]
    assert [x["scheme"] for x in lines] == ["bls-unchained-g1-rfc9380", "pedersen-bls-unchained"]
    for x in lines:
        assert x["rejected"] == x["expected"], x["scheme"]
