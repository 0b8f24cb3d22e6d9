"""The reference's own model / AES tests, run through the C-ABI on the GPU (decrypted-level parity).

Mirrors src/tfhe/shortint_woppbs_1bit.rs tests (:463-877) and src/aes_128/fhe/fhe_impls/
shortint_woppbs_1bit.rs tests (:185-210) with test_helper.rs (:12-120).
"""
import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import Cleartext, aes_128

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def keys(product_raw, gpu_context):
    return product_raw[0], gpu_context


def u16_to_bits(v):
    return [(v >> (15 - i)) & 1 for i in range(16)]


def test_bit_encrypt_decrypt_incl_trivial(keys):
    ck, ctx = keys
    assert ck.decrypt(ck.encrypt(Cleartext(0))) == Cleartext(0)
    assert ck.decrypt(ck.encrypt(Cleartext(1))) == Cleartext(1)
    assert ck.decrypt(ctx.trivial(Cleartext(0))) == Cleartext(0)
    assert ck.decrypt(ctx.trivial(Cleartext(1))) == Cleartext(1)
    t0 = ctx.trivial(Cleartext(0))
    _ = t0.clone() ^ t0.clone() ^ t0.clone()  # trivial does not accumulate noise


@pytest.mark.parametrize("bits,words", [(3, [0b001, 0b000, 0b100, 0b101]),
                                        (8, [0b11001001, 0b01001001, 0b00101010, 0b11011001])])
def test_multivariate_parity_fn(keys, bits, words):
    """test_multivariate_parity_fn_{3,8} (:531-572)."""
    ck, ctx = keys
    parity = lambda v: sum(u16_to_bits(v)) % 2
    tv = ctx.generate_lookup_table(bits, 1, parity)
    for word in words:
        cts = [ck.encrypt(Cleartext(b)) for b in u16_to_bits(word)]
        d = ctx.circuit_bootstrap(cts[16 - bits:], tv)[0]
        assert ck.decrypt(d).value == parity(word)
        assert d.noise_level_squared == bits


@pytest.mark.parametrize("bits,words", [(3, [0b101, 0b000, 0b100]), (8, [0b11001001, 0b01001001, 0b11011001])])
def test_multivariate_multivalued_square_fn(keys, bits, words):
    """test_multivariate_multivalues_square_fn_{3,8} (:574-617)."""
    ck, ctx = keys
    sq = lambda v: (v * v) % (1 << bits)
    tv = ctx.generate_lookup_table(bits, bits, sq)
    for word in words:
        cts = [ck.encrypt(Cleartext(b)) for b in u16_to_bits(word)]
        out = ctx.circuit_bootstrap(cts[16 - bits:], tv)
        val = sum(ck.decrypt(o).value << (bits - 1 - i) for i, o in enumerate(out))
        assert val == sq(word)


def test_boot_variants(keys):
    """boot / boot_const_0 / boot_const_1 / boot_add_1 of test_noise_independence (:699-790)."""
    ck, ctx = keys
    for b in (0, 1):
        bit = ck.encrypt(Cleartext(b))
        for f, exp in ((lambda x: x, b), (lambda x: 0, 0), (lambda x: 1, 1), (lambda x: x + 1, (b + 1) & 1)):
            lut = ctx.generate_lookup_table(1, 1, f)
            assert ck.decrypt(ctx.circuit_bootstrap([bit], lut)[0]).value == exp


def test_increment_1bit_adder(keys):
    """test_increment_1bit_adder (:792-831): ripple-carry increment with 2-in/2-out bootstraps."""
    ck, ctx = keys
    lut = ctx.generate_lookup_table(2, 2, lambda v: (u16_to_bits(v)[14] + u16_to_bits(v)[15]))
    value = [ck.encrypt(Cleartext(0)) for _ in range(16)]  # low 2 bytes of the 16-byte block suffice
    for _ in range(2):
        carry = ctx.trivial(Cleartext(1))
        res = [None] * 16
        for i in reversed(range(16)):
            new_carry, new_bit = ctx.circuit_bootstrap([carry, value[i]], lut)
            carry, res[i] = new_carry, new_bit
        value = res
    out = [ck.decrypt(b).value for b in value]
    assert aes_128.bits_to_u8(out[:8]) == 0 and aes_128.bits_to_u8(out[8:]) == 2


def test_increment_8bit_adder(keys):
    """test_increment_8bit_adder (:833-877): 9-in/9-out bootstrap per byte (input bits = log2 N + 0)."""
    ck, ctx = keys
    lut = ctx.generate_lookup_table(9, 9, lambda v: (v & 0xFF) + u16_to_bits(v)[7])
    value_clear = [0, 0, 255]
    value = [[ck.encrypt(Cleartext(b)) for b in aes_128.u8_to_bits(x)] for x in value_clear]
    for _ in range(3):
        carry = ctx.trivial(Cleartext(1))
        res = [None] * len(value)
        for i in reversed(range(len(value))):
            out = ctx.circuit_bootstrap([carry] + value[i], lut)
            carry, res[i] = out[0], out[1:]
        value = res
    got = [aes_128.bits_to_u8([ck.decrypt(b).value for b in byte]) for byte in value]
    assert got == [0, 1, 2]


def test_cmux_tree_lut_bit_exact(keys, oracle_keys):
    """A LUT with 10 > log2(512) inputs (generate_lookup_table :274-289 with a WopbsLUTBase of 2
    polynomials per output): the device CMux tree over the first GGSW, then the blind rotation over
    the other 9 (tfhe-rs vertical_packing), equal to the oracle and decrypting to f(word)."""
    ck, ctx = keys
    f = lambda v: ((v * 37) ^ (v >> 3)) & 7
    lut = ctx.generate_lookup_table(10, 3, f)
    for word, start in ((0b1011001110, 70_000), (0b0100110001, 70_100)):
        cts = ck.encrypt_bits_raw([(word >> (9 - i)) & 1 for i in range(10)], start_index=start)
        out = ctx.circuit_bootstrap_raw(cts.reshape(1, 10, -1), lut)
        got = ck.decrypt_bits_raw(out[0])
        assert [int(b) for b in got] == [(f(word) >> (2 - j)) & 1 for j in range(3)], bin(word)
    assert np.array_equal(out[0], oracle_keys.circuit_bootstrap(cts, lut.as_array(), 3))


def test_multivariate_multivalues_xor_8bit():
    """test_multivariate_multivalues_xor_8bit (:626-659): params_sqrd_lvl_1 (N = 1024), a 16 -> 8 LUT
    b1 ^ b2 over a 64-polynomial WopbsLUTBase (6-level CMux tree + 10-step blind rotation)."""
    from tests.conftest import SEED
    ck, keys_raw = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SQRD_LVL_1, SEED, threads=16)
    ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_1, keys_raw, device=0)
    b1, b2 = 0b11000110, 0b10101010
    word = (b1 << 8) | b2
    xor_fn = lambda v: (v >> 8) ^ (v & 0xFF)
    tv = ctx.generate_lookup_table(16, 8, xor_fn)
    bits = [ck.encrypt(Cleartext(b)) for b in u16_to_bits(word)]
    out = ctx.circuit_bootstrap(bits, tv)
    assert aes_128.bits_to_u8([ck.decrypt(b).value for b in out]) == xor_fn(word)


def test_light_gal_mul(keys, golden):
    """test_light_gal_mul -> test_helper::test_block_encryption_vs_plain(.., 2) (:86-120)."""
    ck, ctx = keys
    g = golden["test_light"]
    key = bytes.fromhex(g["key"])
    blk = bytes.fromhex(golden["chacha20_zero_seed"]["block1"])
    ek = aes_128.encrypt_word_array(ck, aes_128.key_schedule_plain(key))
    block = aes_128.encrypt_byte_array(ck, blk)
    enc = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt.encrypt_block_for_rounds(ctx, ek, block, 2)
    assert aes_128.decrypt_byte_array(ck, enc) == aes_128.expand_key_and_encrypt_blocks(key, [blk], 2)[0]
    # noise bookkeeping of the round function: mix columns (4 x 8) + round key (1)
    assert max(b.noise_level_squared for byte in enc for b in byte) == 9


def test_full_gal_mul_with_fhe_key_schedule(keys, golden):
    """test_full_gal_mul -> test_key_expansion_and_block_encryption_vs_aes + FIPS-197 C.1
    (test_helper.rs:22-84): FHE key schedule, 10 rounds, two ChaCha blocks and the FIPS vector."""
    ck, ctx = keys
    E = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt
    g = golden["chacha20_zero_seed"]
    key = bytes.fromhex(g["key"])
    ek = E.key_schedule(ctx, aes_128.encrypt_byte_array(ck, key))
    plain_ek = aes_128.key_schedule_plain(key)
    assert [aes_128.decrypt_byte_array(ck, w) for w in ek] == plain_ek
    blocks = [bytes.fromhex(g["block1"]), bytes.fromhex(g["block2"])]
    enc = E.encrypt_blocks(ctx, ek, [aes_128.encrypt_byte_array(ck, b) for b in blocks], 10)
    assert [aes_128.decrypt_byte_array(ck, e).hex() for e in enc] == [
        golden["test_light"]["block1"]["10"], golden["test_light"]["block2"]["10"]]
    fk = bytes.fromhex(golden["fips197_c1"]["key"])
    fek = E.key_schedule(ctx, aes_128.encrypt_byte_array(ck, fk))
    out = E.encrypt_block(ctx, fek, aes_128.encrypt_byte_array(ck, bytes.fromhex(golden["fips197_c1"]["plaintext"])))
    assert aes_128.decrypt_byte_array(ck, out).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_readme_counter_mode_batched(keys, golden):
    """run_client_server_aes_scenario (main.rs:97-128) with the README key/iv, 10 counter blocks
    in one batched call, compared with the golden AES outputs."""
    ck, ctx = keys
    g = golden["readme_ctr"]
    key, iv = bytes.fromhex(g["key"]), bytes.fromhex(g["iv"])
    ek = b"".join(aes_128.key_schedule_plain(key))
    rk = ck.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=100_000)
    blocks = aes_128.counter_blocks(iv, 10)
    cts = ck.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=200_000).reshape(10, 128, -1)
    out = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt.encrypt_blocks_raw(ctx, rk, cts, rounds=10)
    got = [b.hex() for b in aes_128.bits_to_blocks(ck.decrypt_bits_raw(out))]
    assert got == [g["ciphertexts"][str(c)] for c in range(1, 11)]


def test_sbox_pbs_driver_on_1bit_model(keys, golden):
    """ShortintWoppbs1BitSboxPbsAesEncrypt (fhe_impls/shortint_woppbs_1bit.rs:47-81) on the batched device
    path.  Its reference tests test_light / test_full are #[ignore]d because the leveled MixColumns of
    fhe_sbox_pbs breaks the BitCt noise rules (:160-176; tests/test_noise_schedule.py restates why):
    - key_schedule (fhe_sbox_pbs.rs:123-171): sub_word as batched 8 -> 8 circuit bootstraps, boot_word as
      128 one-bit identity circuit bootstraps per call, decrypting to the plain AES key schedule;
    - a 1-round run (ARK, SubBytes of every byte of every block in one call, ShiftRows, ARK) decrypts to
      the reference's 1-round vectors and equals the GalMul driver's 1-round ciphertexts word for word;
    - 2 rounds raise NoiseNotIndependent where the reference panics, on both entry points."""
    ck, ctx = keys
    E = aes_128.ShortintWoppbs1BitSboxPbsAesEncrypt
    G = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt
    g = golden["test_light"]
    key = bytes.fromhex(g["key"])
    ek = E.key_schedule(ctx, aes_128.encrypt_byte_array(ck, key))
    assert [aes_128.decrypt_byte_array(ck, w) for w in ek] == aes_128.key_schedule_plain(key)
    assert max(b.noise_level_squared for w in ek[4:] for byte in w for b in byte) == 1  # identity boots
    blocks = [bytes.fromhex(golden["chacha20_zero_seed"][k]) for k in ("block1", "block2")]
    enc = [aes_128.encrypt_byte_array(ck, b) for b in blocks]
    out = E.encrypt_blocks(ctx, ek, enc, 1)
    assert [aes_128.decrypt_byte_array(ck, o).hex() for o in out] == [g["block1"]["1"], g["block2"]["1"]]
    assert max(b.noise_level_squared for o in out for byte in o for b in byte) == 9  # SBOX (8) + key bit (1)
    with pytest.raises(tfhe_aes.NoiseNotIndependent):
        E.encrypt_block_for_rounds(ctx, ek, enc[0], 2)
    # raw arrays (fresh inputs): the device key schedule and the 1-round batch
    kbits = ck.encrypt_bits_raw([b for byte in key for b in aes_128.u8_to_bits(byte)], start_index=600_000)
    rk = E.key_schedule_raw(ctx, kbits)
    kb = np.asarray(ck.decrypt_bits_raw(rk)).reshape(176, 8)
    assert bytes(aes_128.bits_to_u8(x) for x in kb) == b"".join(aes_128.key_schedule_plain(key))
    cts = ck.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=700_000).reshape(2, 128, -1)
    one = E.encrypt_blocks_raw(ctx, rk, cts, rounds=1)
    assert np.array_equal(one, G.encrypt_blocks_raw(ctx, rk, cts, rounds=1))
    assert [b.hex() for b in aes_128.bits_to_blocks(ck.decrypt_bits_raw(one))] == [g["block1"]["1"], g["block2"]["1"]]
    with pytest.raises(tfhe_aes.NoiseNotIndependent):
        E.encrypt_blocks_raw(ctx, rk, cts, rounds=2)
