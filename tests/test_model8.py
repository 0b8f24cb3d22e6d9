"""8-bit model (shortint_woppbs_8bit, config #5) on the CPU: parameters, keygen and encryption
parity product == oracle, and the oracle pinned at the decrypted level by the reference's own tests
(src/tfhe/shortint_woppbs_8bit.rs:368-478) and the AES golden vectors."""
import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import aes_128
from tests.conftest import SEED


def test_params_8bit_match_reference(oracle_mod):
    # shortint_woppbs_8bit.rs:39-86 (k=2, N=2^10, n=785, br 6x2^7, ks 8x2^2, cb 4x2^6, pp 3x2^12)
    p = tfhe_aes.get_params(tfhe_aes.PARAMS_WOPPBS_8BIT)
    assert (p["n"], p["k"], p["N"], p["pbs_l"], p["pbs_b"], p["ks_l"], p["ks_b"], p["cbs_l"], p["cbs_b"],
            p["pfks_l"], p["pfks_b"], p["max_noise_sq"], p["model"]) == (785, 2, 1024, 6, 7, 8, 2, 4, 6, 3, 12, 11, 8)
    assert p["lwe_std"] == 1.5140301927925663e-05 and p["glwe_std"] == 0.00000000000000022148688116005568
    assert tfhe_aes.bit_len(tfhe_aes.PARAMS_WOPPBS_8BIT) == 786


def test_keygen8_bit_identical_to_oracle(product_raw8, oracle_keys8):
    ck, (ksk, bsk, pfpksk) = product_raw8
    lwe, glwe = ck.secrets()
    assert np.array_equal(lwe, oracle_keys8.lwe_sk()) and np.array_equal(glwe, oracle_keys8.glwe_sk())
    oksk, obsk, opf = oracle_keys8.raw_server()
    assert np.array_equal(ksk, oksk) and np.array_equal(bsk, obsk) and np.array_equal(pfpksk, opf)


def test_encrypt8_small_bits_and_ints(product_raw8, oracle_keys8):
    ck, _ = product_raw8
    bits = [1, 0, 1, 1, 0, 1, 0, 1]
    cts = ck.encrypt_bits_raw(bits, start_index=77)
    assert cts.shape == (8, 786)  # ClientKey::encrypt under the small key (shortint_woppbs_8bit.rs:199-214)
    assert np.array_equal(cts, oracle_keys8.encrypt_small_bits(bits, SEED, 77))
    assert list(ck.decrypt_bits_raw(cts)) == bits
    ints = ck.encrypt_ints_raw([0b10110101, 0, 255], start_index=3)
    assert np.array_equal(ints, oracle_keys8.encrypt_ints([0b10110101, 0, 255], SEED, 3))
    assert list(ck.decrypt_ints_raw(ints)) == [0b10110101, 0, 255]


def test_gf_256_mul_network_is_gf_multiplication(oracle_mod):
    """fhe_sbox_pbs::gf_256_mul (:33-53) on bits == GF(2^8) multiplication; no bit is added twice."""
    def gf(a, b):
        r = 0
        for _ in range(8):
            if b & 1:
                r ^= a
            h = a & 0x80
            a = (a << 1) & 0xFF
            if h:
                a ^= 0x1B
            b >>= 1
        return r
    for m in (1, 2, 3):
        T = oracle_mod.gf_256_mul_terms(m)
        assert T.max() <= 1
        for x in range(256):
            bits = np.array(aes_128.u8_to_bits(x))
            assert aes_128.bits_to_u8((T @ bits) & 1) == gf(x, m)
    MC = oracle_mod.mix_column_terms()
    assert MC.max() == 1 and MC.sum(axis=1).max() == 7  # noise level <= 7 + key bit 1 <= MaxNoiseLevel 11


def test_oracle8_extract_bits_from_int_byte(oracle_keys8):
    """shortint_woppbs_8bit.rs:443-458 test_extract_bits_from_int_byte."""
    K = oracle_keys8
    ict = K.encrypt_ints([0b10110101], SEED, 0)
    bits = K.extract_bits(ict[0])
    assert aes_128.bits_to_u8(K.decrypt_small_bits(bits)) == 0b10110101


def test_oracle8_bootstrap_from_bits_lut(oracle_mod, oracle_keys8):
    """shortint_woppbs_8bit.rs:427-441 test_bootstrap_from_bits_lut (f = val + 3)."""
    K = oracle_keys8
    cts = K.encrypt_small_bits(aes_128.u8_to_bits(0b10110101), SEED, 100)
    lut = oracle_mod.generate_lut_without_padding(1024, lambda v: v + 3)
    ict = K.cbs_vp_small(cts, lut, 1)
    assert int(K.decrypt_ints(ict)[0]) == 0b10110101 + 3


@pytest.mark.slow
def test_oracle8_aes_one_round(oracle_keys8, golden):
    """fhe_sbox_pbs::encrypt_block_for_rounds(.., 1): ARK0 + last round (SBOX bootstrap_with_lut)."""
    K = oracle_keys8
    g = golden["test_light"]
    ek = b"".join(aes_128.key_schedule_plain(bytes.fromhex(g["key"])))
    rk = K.encrypt_small_bits([b for byte in ek for b in aes_128.u8_to_bits(byte)], b"\x33" * 32)
    blk = bytes.fromhex(golden["chacha20_zero_seed"]["block1"])
    cts = K.encrypt_small_bits([b for byte in blk for b in aes_128.u8_to_bits(byte)], b"\x44" * 32)
    import os
    out = K.aes8_encrypt_block(rk, cts, 1, threads=min(16, os.cpu_count() or 1))
    bits = K.decrypt_small_bits(out).reshape(16, 8)
    assert bytes(aes_128.bits_to_u8(b) for b in bits).hex() == g["block1"]["1"]
