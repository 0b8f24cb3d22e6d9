"""shortint_1bit model (src/tfhe/shortint_1bit.rs) on the CPU: the oracle's restatement pinned by the
reference's own (non-ignored) tests of the model, and the product's host side (parameters, keygen,
encryption, cleartext test vectors) equal to the oracle's.  GPU parity: tests/test_gpu_shortint1.py.

The reference's tests (shortint_1bit.rs:593-720) decrypt: test_packing_keyswitch (:593-640), the
bivariate function (:642-669), multivariate_fn_3 (:671-699) and the 3-bit parity function (:701-709).
Its 8-bit parity test (:711-716) needs 255 bootstraps (~1 min on the oracle): it runs on the GPU only.
"""
import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import shortint_1bit as S

ES = bytes([0x5A] * 32)  # oracle encryption seed (the product encrypts under its key's own seed)


@pytest.fixture(scope="module")
def okeys(oracle_mod):
    return oracle_mod.S1Keys(bytes(range(32)), threads=8)


def dec_plain(x: int) -> int:
    """decode_bit (shortint_1bit.rs:359-364): closest multiple of 2^62, then bit 62"""
    return (((int(x) + (1 << 61)) >> 62) & 1)


def test_params(oracle_mod):
    p = tfhe_aes.get_params(tfhe_aes.PARAMS_SHORTINT_1BIT)
    # shortint_1bit.rs:62-83: n 640, k 4, N 512, pbs 7 x 2^6, ks 2 x 2^6, message 2 / carry 1, MaxNoiseLevel 11
    assert (p["n"], p["k"], p["N"], p["pbs_l"], p["pbs_b"], p["ks_l"], p["ks_b"], p["max_noise_sq"]) == (
        640, 4, 512, 7, 6, 2, 6, 11)
    assert p["lwe_std"] == 4.728000245054929e-7 and p["glwe_std"] == 2.845267479601915e-15
    assert tfhe_aes.bit_len(tfhe_aes.PARAMS_SHORTINT_1BIT) == 641


def test_packing_keyswitch(okeys):
    """shortint_1bit.rs:593-640: pack [0, 1] -> coefficients 0..4 decode to 0, 1, 0, 0, 0"""
    cts = okeys.s1_encrypt([0, 1], ES, 0)
    plain = okeys.glwe_decrypt(okeys.pack(cts))
    assert [dec_plain(plain[i]) for i in range(5)] == [0, 1, 0, 0, 0]


@pytest.mark.parametrize("m0,m1", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_bivariate_fn_2(okeys, m0, m1):
    """shortint_1bit.rs:642-669"""
    table = [1, 0, 0, 1]
    cts = okeys.s1_encrypt([m0, m1], ES, 10 + 2 * m0 + m1)
    assert okeys.s1_decrypt(okeys.multivariate(cts, table))[0] == table[(m0 << 1) + m1]


@pytest.mark.parametrize("m", [(0, 0, 0), (0, 1, 1), (1, 0, 1), (1, 1, 0)])
def test_multivariate_fn_3(okeys, m):
    """shortint_1bit.rs:671-699"""
    table = [1, 0, 0, 1, 0, 1, 1, 0]
    cts = okeys.s1_encrypt(list(m), ES, 20 + 4 * m[0] + 2 * m[1] + m[2])
    assert okeys.s1_decrypt(okeys.multivariate(cts, table))[0] == table[(m[0] << 2) + (m[1] << 1) + m[2]]


@pytest.mark.parametrize("byte", [0b001, 0b000, 0b100, 0b101])
def test_multivariate_parity_fn_3(okeys, byte):
    """shortint_1bit.rs:701-709 (bits = the low 3 of the byte's MSB-first bits, :718-733)"""
    bits = [(byte >> (7 - i)) & 1 for i in range(8)][5:]
    table = [bin(v).count("1") % 2 for v in range(8)]
    cts = okeys.s1_encrypt(bits, ES, 40 + byte)
    assert okeys.s1_decrypt(okeys.multivariate(cts, table))[0] == bin(byte).count("1") % 2


def test_test_vector_from_ciphertexts_layout(okeys):
    """test_vector_from_ciphertexts (:392-492): ct0 fills [0, N/4) u [3N/4, N), ct1 [N/4, 3N/4) of the body
    phase (the add-then-rotate loops of the reference restated step by step in the oracle)"""
    cts = okeys.s1_encrypt([1, 0], ES, 60)
    plain = okeys.glwe_decrypt(okeys.tv_from_cts(cts[0], cts[1]))
    N = okeys.p["N"]
    got = [dec_plain(plain[j]) for j in range(N)]
    assert got == [1 if (j < N // 4 or j >= 3 * N // 4) else 0 for j in range(N)]


def test_bootstrap_applies_test_vector(okeys):
    """FheContext::bootstrap with test_vector_from_cleartext_fn (NOT), output back under the small key"""
    cts = okeys.s1_encrypt([0, 1], ES, 70)
    tv = okeys.tv_from_fn(1, 0)
    assert [okeys.s1_decrypt(okeys.bootstrap(c, tv))[0] for c in cts] == [1, 0]


def test_product_host_side_matches_oracle(okeys):
    """product keygen (client + the three server keys: KSK, BSK, packing keyswitch key), encryption
    and the cleartext test vectors equal the oracle's (same keygen spec)"""
    ck, (ksk, bsk, pksk) = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SHORTINT_1BIT, bytes(range(32)), threads=8)
    oksk, obsk, opk = okeys.raw_server()
    assert np.array_equal(ksk, oksk) and np.array_equal(bsk, obsk) and np.array_equal(pksk, opk)
    assert pksk.size == 640 * 2 * 5 * 512
    cts = ck.encrypt_bits_raw([1, 0, 1], start_index=77)
    assert np.array_equal(cts, okeys.s1_encrypt([1, 0, 1], bytes(range(32)), 77))
    assert list(ck.decrypt_bits_raw(cts)) == [1, 0, 1]
    ctx_stub = type("Ctx", (), {"params": tfhe_aes.get_params(tfhe_aes.PARAMS_SHORTINT_1BIT)})()
    for f0 in (0, 1):
        for f1 in (0, 1):
            tv = S.test_vector_from_cleartext_fn(ctx_stub, lambda c: tfhe_aes.Cleartext(f0 if c.value == 0 else f1))
            assert np.array_equal(tv.data, okeys.tv_from_fn(f0, f1))
