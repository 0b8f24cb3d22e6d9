"""Host-side product logic on the CPU: keygen / encryption parity with the oracle (same keygen spec),
LUT generation, BitCt noise bookkeeping (shortint_woppbs_1bit.rs:463-529), static AES noise schedule."""
import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import Cleartext, aes_128


def test_params_match_reference(oracle_mod):
    # parameters.rs:29-205
    for pid in range(6):
        prod = tfhe_aes.get_params(pid)
        model = prod.pop("model")
        assert model == {tfhe_aes.PARAMS_WOPPBS_8BIT: 8, tfhe_aes.PARAMS_SHORTINT_1BIT: 2}.get(pid, 1)
        ref = oracle_mod.params(pid)
        assert ref.pop("model") == (2 if model == 2 else 0)
        assert prod == ref
    p = tfhe_aes.get_params(tfhe_aes.PARAMS_SQRD_LVL_64)
    assert (p["n"], p["k"], p["N"], p["pbs_l"], p["pbs_b"], p["ks_l"], p["ks_b"], p["cbs_l"], p["cbs_b"],
            p["pfks_l"], p["pfks_b"], p["max_noise_sq"]) == (677, 4, 512, 3, 12, 4, 3, 1, 13, 2, 16, 64)


def test_keygen_bit_identical_to_oracle(product_raw, oracle_keys):
    ck, (ksk, bsk, pfpksk) = product_raw
    lwe, glwe = ck.secrets()
    assert np.array_equal(lwe, oracle_keys.lwe_sk())
    assert np.array_equal(glwe, oracle_keys.glwe_sk())
    oksk, obsk, opf = oracle_keys.raw_server()
    assert np.array_equal(ksk, oksk)
    assert np.array_equal(bsk, obsk)
    assert np.array_equal(pfpksk, opf)


def test_encrypt_matches_oracle_and_decrypts(product_raw, oracle_keys):
    ck, _ = product_raw
    bits = [0, 1, 1, 0, 1]
    cts = ck.encrypt_bits_raw(bits, start_index=1000)
    # the product encrypts with the key seed's ENCRYPT stream; the oracle restates it
    from tests.conftest import SEED
    ref = oracle_keys.encrypt_bits(bits, SEED, 1000)
    assert np.array_equal(cts, ref)
    assert list(ck.decrypt_bits_raw(cts)) == bits
    assert list(oracle_keys.decrypt_bits(cts)) == bits


def test_encryption_indices_never_alias(product_raw, oracle_keys):
    """Ciphertext #idx draws its mask / noise from ChaCha20(nonce 2P | (idx >> 40) << 8, counter
    (idx mod 2^40) 2^24): indices 2^40 apart no longer share a stream (the counter alone wraps), and
    the oracle restates the same rule."""
    ck, _ = product_raw
    from tests.conftest import SEED
    for i in (0, 5, 1000):
        a = ck.encrypt_bits_raw([0], start_index=i)
        b = ck.encrypt_bits_raw([0], start_index=i + (1 << 40))
        c = ck.encrypt_bits_raw([0], start_index=i + (7 << 40))
        assert not np.array_equal(a[0, :64], b[0, :64]) and not np.array_equal(a[0, :64], c[0, :64])
        assert np.array_equal(b, oracle_keys.encrypt_bits([0], SEED, i + (1 << 40)))
    masks = np.stack([ck.encrypt_bits_raw([0], start_index=s)[0, :8] for s in range(0, 1 << 44, 1 << 40)])
    assert len({m.tobytes() for m in masks}) == len(masks)


def test_encryption_index_ranges(product_raw):
    """Explicit raw indices stay below 2^63; TAE_INDEX_AUTO (start_index=None) reserves fresh ones
    from the key's counter, the region tae_encrypt uses, so auto ranges never repeat."""
    ck, _ = product_raw
    with pytest.raises(tfhe_aes.TaeError):
        ck.encrypt_bits_raw([0], start_index=1 << 63)
    with pytest.raises(tfhe_aes.TaeError):
        ck.encrypt_bits_raw([0, 1], start_index=(1 << 63) - 1)
    a, b = ck.encrypt_bits_raw([1, 0, 1]), ck.encrypt_bits_raw([1, 0, 1])
    assert not np.array_equal(a[:, :-1], b[:, :-1])
    assert list(ck.decrypt_bits_raw(a)) == [1, 0, 1] == list(ck.decrypt_bits_raw(b))


def test_context_from_raw_checks_key_arrays(product_raw):
    """Short, mistyped or wrongly sized key arrays are refused before any pointer reaches C."""
    _, (ksk, bsk, pfpksk) = product_raw
    with pytest.raises(ValueError):
        tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, (ksk[:-1], bsk, pfpksk))
    with pytest.raises(ValueError):
        tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, (ksk.astype(np.float64), bsk, pfpksk))
    with pytest.raises(ValueError):
        tfhe_aes.save_keys("/tmp/never-written.taekey", tfhe_aes.PARAMS_SQRD_LVL_64, None, (ksk, bsk[:10], pfpksk))


def test_product_lut_generator_exact_layout(golden, oracle_mod):
    """The product's context-free generate_multivariate_luts (tae_generate_multivariate_luts) against
    the reference's exact arrays (shortint_woppbs_1bit.rs:665-697): N=16 3 -> 2 (one polynomial per
    output) and N=8 5 -> 2 (multi-polynomial: 4 polynomials per output), and equal to the oracle on
    the AES LUTs."""
    lut = tfhe_aes.generate_multivariate_luts(16, 3, 2, lambda v: v)
    assert lut.size == 16 * 2
    for j, exp in enumerate(golden["lut_vertical_packing_3_2_16"]):
        assert list(lut[16 * j:16 * (j + 1)]) == [b << 63 for b in exp]
    lut = tfhe_aes.generate_multivariate_luts(8, 5, 2, lambda v: v)
    assert lut.size == 8 * 4 * 2
    for j, exp in enumerate(golden["lut_multipoly_5_2_8"]):
        assert list(lut[32 * j:32 * (j + 1)]) == [b << 63 for b in exp]
    f = lambda x: (aes_128.gf_256_mul(aes_128.SBOX[x], 1) << 16) | (aes_128.gf_256_mul(aes_128.SBOX[x], 2) << 8) | \
        aes_128.gf_256_mul(aes_128.SBOX[x], 3)
    assert np.array_equal(tfhe_aes.generate_multivariate_luts(512, 8, 24, f), oracle_mod.generate_lut(512, 8, 24, f))
    with pytest.raises(tfhe_aes.TaeError):
        tfhe_aes.generate_multivariate_luts(12, 3, 2, lambda v: v)  # not a power of two


def test_bit_encrypt_decrypt(product_raw):
    ck, _ = product_raw
    b1 = ck.encrypt(Cleartext(0))
    b2 = ck.encrypt(Cleartext(1))
    assert ck.decrypt(b1) == Cleartext(0)
    assert ck.decrypt(b2) == Cleartext(1)


def test_bit_xor(product_raw):
    """test_bit_xor (:484-503) -- on lvl_64 keys (max noise^2 64)."""
    ck, _ = product_raw
    b1, b2, b3, b4 = (ck.encrypt(Cleartext(v)) for v in (0, 1, 0, 1))
    assert ck.decrypt(b1 ^ b2) == Cleartext(1)
    assert ck.decrypt(b1 ^ b3) == Cleartext(0)
    assert ck.decrypt(b2 ^ b4) == Cleartext(0)
    assert (b1 ^ b2).noise_level_squared == 2


def test_bit_xor_above_max_noise():
    """test_bit_xor_above_max_noise (:505-518): 5-way XOR at max noise^2 4 -> NoiseTooBig."""
    ck, _ = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SQRD_LVL_4, bytes(32), threads=8)
    b = [ck.encrypt(Cleartext(v)) for v in (0, 1, 0, 1, 0)]
    acc = b[0] ^ b[1] ^ b[2] ^ b[3]
    assert acc.noise_level_squared == 4
    with pytest.raises(tfhe_aes.NoiseTooBig, match="NoiseTooBig"):
        acc ^= b[4]


def test_bit_xor_not_independent(product_raw):
    """test_bit_xor_not_independent (:520-529)."""
    ck, _ = product_raw
    b1 = ck.encrypt(Cleartext(0))
    with pytest.raises(tfhe_aes.NoiseNotIndependent, match="noise components not independent"):
        _ = b1.clone() ^ b1.clone()


def test_cleartext_out_of_bounds(product_raw):
    ck, _ = product_raw
    with pytest.raises(tfhe_aes.TaeError):
        ck.encrypt(Cleartext(2))


def test_no_gpu_means_no_context(product_raw):
    """The product has no CPU fallback: without a GPU, building a server context fails loudly."""
    if tfhe_aes.device_count() > 0:
        pytest.skip("GPU present")
    _, keys = product_raw
    with pytest.raises(tfhe_aes.NoDevice):
        tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, keys)
