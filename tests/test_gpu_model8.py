"""GPU parity for the 8-bit model (shortint_woppbs_8bit, BASELINE config #5): every stage of the HIP
path against the CPU oracle on identical inputs and keys (bit-exact, f64 FFT stages included), plus
decrypted results pinned by the reference's tests (shortint_woppbs_8bit.rs:368-478) and the AES golden
vectors (test_light, FIPS-197 C.1).  Product keygen == oracle keygen is proved in test_model8.py."""
import ctypes as C
import os

import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import _native as N
from tfhe_aes import aes_128
from tests.conftest import SEED

pytestmark = pytest.mark.gpu

K = 2 * 1024
BIG = K + 1
SMALL = 786
THREADS = min(16, os.cpu_count() or 1)
A8 = aes_128.ShortintWoppbs8BitSboxPbsAesEncrypt


def _vp(a):
    return a.ctypes.data_as(C.c_void_p)


def _stage(fn, *args):
    N.check(fn(*args))


@pytest.fixture(scope="module")
def client8(product_raw8):
    return product_raw8[0]


def test_keyswitch8_bit_exact(gpu_context8, oracle_keys8, client8):
    ints = client8.encrypt_ints_raw([0x35, 0xC2, 0x00, 0xFF], start_index=10)
    out = np.zeros((4, SMALL), dtype=np.uint64)
    _stage(N.lib().tae_stage_keyswitch, gpu_context8._h, _vp(ints), 4, _vp(out), N.TAE_MEM_HOST)
    for i in range(4):
        assert np.array_equal(out[i], oracle_keys8.keyswitch(ints[i])), i


@pytest.mark.parametrize("level", [1, 4])
def test_pbs_shift_boolean8_bit_exact(gpu_context8, oracle_keys8, client8, level):
    """homomorphic_shift_boolean with the N=1024, pbs 6 x 2^7 bootstrapping key at CBS level `level`."""
    bits = [1, 0, 1]
    small = client8.encrypt_bits_raw(bits, start_index=200 + level)
    out = np.zeros((3, BIG), dtype=np.uint64)
    _stage(N.lib().tae_stage_pbs_shift_boolean, gpu_context8._h, _vp(small), 3, level, _vp(out), N.TAE_MEM_HOST)
    for i in range(3):
        assert np.array_equal(out[i], oracle_keys8.homomorphic_shift_boolean(small[i], level)), i
        ph = oracle_keys8.phase(out[i])
        want = bits[i] << (64 - 6 * level)
        err = (ph - want) % (1 << 64)
        assert min(err, (1 << 64) - err) < 1 << (63 - 6 * level), (i, level)  # within alpha


@pytest.mark.parametrize("lat,pair,B,occ2,wide", [("1", "1", 5, "0", "1"), ("0", "1", 5, "0", "1"),
                                                  ("0", "0", 5, "0", "1"), ("1", "1", 300, "0", "1"),
                                                  ("1", "1", 513, "0", "1"), ("1", "1", 513, "1", "1"),
                                                  ("1", "1", 1027, "0", "1"), ("1", "1", 1027, "0", "0")])
def test_pbs8_kernel_variants_bit_exact(product_raw8, oracle_keys8, client8, lat, pair, B, occ2, wide):
    """The N=1024 blind-rotation variants the engine picks, all on the fused-twiddle transform (lf1k.hpp,
    the oracle's or_lf1k_*): for batches up to one ciphertext per CU the 1024-thread latency kernel
    (br1024lat, default), or with TAE_B1K_LAT=0 br1024 with one ciphertext per workgroup and two levels
    per pass (or one: TAE_B1K_PAIR=0); and two ciphertexts per workgroup (B > the CU count, odd tail
    workgroup of one); TAE_B1K_OCC2=1: large batches as one ciphertext per workgroup, two per CU; from four
    ciphertexts per CU on br1024w, four per workgroup with the ACC stash (B = 1027: a ragged last workgroup of
    three; TAE_B1K_WIDE=0: br1024 with two per workgroup instead)."""
    env = {"TAE_B1K_LAT": lat, "TAE_B1K_PAIR": pair, "TAE_B1K_OCC2": occ2, "TAE_B1K_WIDE": wide}
    os.environ.update(env)
    try:
        ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_WOPPBS_8BIT, product_raw8[1], device=0)
    finally:
        for k in env:
            del os.environ[k]
    bits = np.random.default_rng(B).integers(0, 2, size=B).astype(np.uint8)
    small = client8.encrypt_bits_raw(bits, start_index=900)
    out = np.zeros((B, BIG), dtype=np.uint64)
    _stage(N.lib().tae_stage_pbs_shift_boolean, ctx._h, _vp(small), B, 2, _vp(out), N.TAE_MEM_HOST)
    for i in sorted({0, min(3, B - 1), B // 2, B - 1}):
        assert np.array_equal(out[i], oracle_keys8.homomorphic_shift_boolean(small[i], 2)), i
    del ctx


def test_pfks8_bit_exact(gpu_context8, oracle_keys8, client8):
    small = client8.encrypt_bits_raw([1, 0], start_index=300)
    big = np.stack([oracle_keys8.homomorphic_shift_boolean(small[i], 2) for i in range(2)])
    out = np.full((2, 4, 3, 3 * 1024), 0x5A5A, dtype=np.uint64)  # [B][cbs_l][k+1][(k+1)N], poisoned
    _stage(N.lib().tae_stage_pfks_ggsw, gpu_context8._h, _vp(big), 2, 2, _vp(out), N.TAE_MEM_HOST)
    for i in range(2):
        for q in range(3):
            assert np.array_equal(out[i, 1, q], oracle_keys8.pfks(q, big[i])), (i, q)
    # the stage writes only level 2's rows; the host path hands back zeros for the other levels
    assert not out[:, [0, 2, 3]].any()


@pytest.mark.parametrize("layout", ["k", "rows"])
def test_pfks8_gemm_layouts_bit_exact(product_raw8, oracle_keys8, layout):
    """Both PFKS GEMM operand layouts on the 8-bit set (pfks 3 x 2^12: the K layout carries 2 byte limbs
    per level, 6 slots per coefficient, no offset) over 130 random big LWEs (a ragged second 128-row tile
    of the row-limb layout) plus digit-range extremes (level digits +-2048, carries, zero, all-ones)."""
    import os
    import tfhe_aes
    os.environ["TAE_PFKS_LAYOUT"] = layout
    try:
        ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_WOPPBS_8BIT, product_raw8[1], device=0)
    finally:
        del os.environ["TAE_PFKS_LAYOUT"]
    rng = np.random.default_rng(11)
    big = rng.integers(0, 2**63, size=(130, 2049), dtype=np.uint64) * np.uint64(2) + rng.integers(
        0, 2, size=(130, 2049), dtype=np.uint64)
    ext = np.array([0x8008_0080_0000_0000, 0x7FF8_0080_0000_0000, 0x8007_FF80_0000_0000, 0xFFFF_FFFF_FFFF_FFFF,
                    0, 0x8000_0000_0000_0000, 0x0008_0000_0000_0000, 0x7FF7_FF7F_F800_0000], dtype=np.uint64)
    big[3] = np.resize(ext, 2049)
    out = np.zeros((130, 4, 3, 3 * 1024), dtype=np.uint64)
    _stage(N.lib().tae_stage_pfks_ggsw, ctx._h, _vp(big), 130, 1, _vp(out), N.TAE_MEM_HOST)
    for i in (0, 3, 127, 129):
        for q in (0, 2):
            assert np.array_equal(out[i, 0, q], oracle_keys8.pfks(q, big[i])), (i, q)
    del ctx


def test_ggsw_fourier8_bit_exact(gpu_context8, oracle_keys8, client8):
    small = client8.encrypt_bits_raw([1], start_index=400)
    ggsw = oracle_keys8.circuit_bootstrap_boolean(small[0])
    out = np.zeros(4 * 3 * 3 * 512 * 2, dtype=np.float64)
    _stage(N.lib().tae_stage_ggsw_fourier, gpu_context8._h, _vp(ggsw), 1, _vp(out), N.TAE_MEM_HOST)
    ref = oracle_keys8.ggsw_to_fourier(ggsw)
    assert np.array_equal(out.view(np.uint64), ref.view(np.float64).view(np.uint64))


def test_lut_without_padding_matches_oracle(gpu_context8, oracle_mod):
    lut = gpu_context8.generate_lookup_table(8, 8, lambda v: aes_128.SBOX[v])
    ref = oracle_mod.generate_lut_without_padding(1024, lambda v: aes_128.SBOX[v])
    assert np.array_equal(lut.as_array(), ref)


def test_bootstrap_from_bits8_bit_exact(gpu_context8, oracle_keys8, oracle_mod, client8):
    """FheContext::bootstrap_from_bits: test_bootstrap_from_bits_lut (shortint_woppbs_8bit.rs:427-441,
    f = val + 3) and the identity LUT (:391-404), ciphertexts equal to the oracle's."""
    vals = [0b10110101, 0x00, 0xFC]
    bits = np.stack([client8.encrypt_bits_raw(aes_128.u8_to_bits(v), start_index=500 + 8 * i)
                     for i, v in enumerate(vals)])
    for f in (lambda v: v + 3, lambda v: v):
        lut = gpu_context8.generate_lookup_table(8, 8, f)
        ints = gpu_context8.bootstrap_from_bits_raw(bits, lut)
        assert list(client8.decrypt_ints_raw(ints)) == [f(v) & 255 for v in vals]
        ref = oracle_keys8.cbs_vp_small(bits[0], lut.as_array(), 1)
        assert np.array_equal(ints[0], ref[0])


def test_extract_bits8_bit_exact(gpu_context8, oracle_keys8, client8):
    """extract_bits_from_ciphertext: test_extract_bits_from_int_byte (shortint_woppbs_8bit.rs:443-458)."""
    vals = [0b10110101, 0x01, 0x80, 0xFF, 0x00]
    ints = client8.encrypt_ints_raw(vals, start_index=600)
    out = gpu_context8.extract_bits_from_ciphertext_raw(ints)
    for i, v in enumerate(vals):
        assert aes_128.bits_to_u8(client8.decrypt_bits_raw(out[i])) == v
    assert np.array_equal(out[0], oracle_keys8.extract_bits(ints[0]))


def test_sbox_substitute8_bit_exact(gpu_context8, oracle_keys8, client8):
    """ByteT::sbox_substitute = bootstrap_with_lut (fhe_impls/shortint_woppbs_8bit.rs:26-42) over a batch."""
    vals = [0x00, 0x01, 0x53, 0xFF, 0x9A, 0x10]
    lut = gpu_context8.generate_lookup_table(8, 8, lambda v: aes_128.SBOX[v])
    bits = np.stack([client8.encrypt_bits_raw(aes_128.u8_to_bits(v), start_index=700 + 8 * i)
                     for i, v in enumerate(vals)])
    out = gpu_context8.circuit_bootstrap_raw(bits, lut)
    for i, v in enumerate(vals):
        assert aes_128.bits_to_u8(client8.decrypt_bits_raw(out[i])) == aes_128.SBOX[v], hex(v)
    assert np.array_equal(out[2], oracle_keys8.bootstrap_with_lut8(bits[2], lut.as_array()))


def _rk_and_block(client8, golden, start):
    g = golden["test_light"]
    ek = b"".join(aes_128.key_schedule_plain(bytes.fromhex(g["key"])))
    rk = client8.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=start)
    blk = bytes.fromhex(golden["chacha20_zero_seed"]["block1"])
    cts = client8.encrypt_bits_raw(aes_128.blocks_to_bits([blk]), start_index=start + 5000).reshape(1, 128, SMALL)
    return g, rk, cts


def test_aes8_one_round_bit_exact(gpu_context8, oracle_keys8, client8, golden):
    g, rk, cts = _rk_and_block(client8, golden, 10_000)
    out = A8.encrypt_blocks_raw(gpu_context8, rk, cts, rounds=1)
    assert aes_128.bits_to_blocks(client8.decrypt_bits_raw(out))[0].hex() == g["block1"]["1"]
    ref = oracle_keys8.aes8_encrypt_block(rk, cts[0], 1, threads=THREADS)
    assert np.array_equal(out[0], ref)


def test_aes8_two_rounds_bit_exact(gpu_context8, oracle_keys8, client8, golden):
    """test_light of the 8-bit model (fhe_impls/shortint_woppbs_8bit.rs:72-82): 2 rounds incl. MixColumns."""
    g, rk, cts = _rk_and_block(client8, golden, 20_000)
    out = A8.encrypt_blocks_raw(gpu_context8, rk, cts, rounds=2)
    assert aes_128.bits_to_blocks(client8.decrypt_bits_raw(out))[0].hex() == g["block1"]["2"]
    ref = oracle_keys8.aes8_encrypt_block(rk, cts[0], 2, threads=THREADS)
    assert np.array_equal(out[0], ref)


def test_aes8_eight_blocks_one_round_bit_exact(gpu_context8, oracle_keys8, client8, golden):
    """Eight blocks in one call: every CBS and extract_bits PBS launch then has 1024 bootstraps, four per CU on 256
    CUs, the br1024w shape of the bench (64 blocks: 8192 per CBS launch); blocks 0, 3 (a workgroup's fourth
    ciphertexts) and 7 word for word against the oracle, all eight decrypted against plain AES."""
    g = golden["test_light"]
    key = bytes.fromhex(g["key"])
    ek = b"".join(aes_128.key_schedule_plain(key))
    rk = client8.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=70_000)
    blocks = [bytes([(17 * i + j) & 255 for j in range(16)]) for i in range(8)]
    cts = client8.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=75_000).reshape(8, 128, SMALL)
    out = A8.encrypt_blocks_raw(gpu_context8, rk, cts, rounds=1)
    assert aes_128.bits_to_blocks(client8.decrypt_bits_raw(out)) == aes_128.expand_key_and_encrypt_blocks(key, blocks, 1)
    for i in (0, 3, 7):
        assert np.array_equal(out[i], oracle_keys8.aes8_encrypt_block(rk, cts[i], 1, threads=THREADS)), i


def test_aes8_full_fips197_with_fhe_key_schedule(gpu_context8, client8, golden):
    """test_full (test_helper.rs:53-84) for the 8-bit model: FHE key_schedule (fhe_sbox_pbs.rs:123-171)
    then 10 rounds, FIPS-197 C.1, plus a second counter block in the same batch."""
    key = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
    kb = client8.encrypt_bits_raw([b for byte in key for b in aes_128.u8_to_bits(byte)], start_index=50_000)
    ek = A8.key_schedule_raw(gpu_context8, kb)
    plain_ek = b"".join(aes_128.key_schedule_plain(key))
    assert bytes(aes_128.bits_to_u8(client8.decrypt_bits_raw(ek)[8 * i:8 * i + 8]) for i in range(176)) == plain_ek
    blocks = [bytes.fromhex("00112233445566778899aabbccddeeff"), bytes(range(16))]
    cts = client8.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=60_000).reshape(2, 128, SMALL)
    out = A8.encrypt_blocks_raw(gpu_context8, ek, cts, rounds=10)
    got = aes_128.bits_to_blocks(client8.decrypt_bits_raw(out))
    assert got[0].hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert got == aes_128.expand_key_and_encrypt_blocks(key, blocks, 10)


@pytest.mark.parametrize("pid", [tfhe_aes.PARAMS_SQRD_LVL_1, tfhe_aes.PARAMS_SQRD_LVL_4,
                                 tfhe_aes.PARAMS_SQRD_LVL_256])
def test_other_n1024_sets_bit_exact(pid, oracle_mod):
    """The batched N=1024 blind rotation (br1024.hpp) under params_sqrd_lvl_1 (pbs 2 x 2^15, pfks
    1 x 2^24: scalar PFKS), _4 (pbs 2 x 2^15, pfks 2 x 2^16: int8 MFMA PFKS) and _256 (pbs 4 x 2^9):
    homomorphic_shift_boolean and a 4 -> 4 circuit bootstrap, equal to the oracle."""
    ck, keys = tfhe_aes.generate_keys_raw(pid, SEED, threads=THREADS)
    ctx = tfhe_aes.context_from_raw(pid, keys, device=0)
    ok = oracle_mod.Keys(pid, None, raw=keys)
    p = tfhe_aes.get_params(pid)
    big, small = p["k"] * p["N"] + 1, p["n"] + 1
    cts = ck.encrypt_bits_raw([1, 0, 1, 1], start_index=90)
    sm = np.stack([ok.keyswitch(c) for c in cts[:2]])
    out = np.zeros((2, big), dtype=np.uint64)
    _stage(N.lib().tae_stage_pbs_shift_boolean, ctx._h, _vp(sm), 2, 1, _vp(out), N.TAE_MEM_HOST)
    for i in range(2):
        assert np.array_equal(out[i], ok.homomorphic_shift_boolean(sm[i], 1)), i
    f = lambda x: (x * 7 + 3) & 15
    lut = ctx.generate_lookup_table(4, 4, f)
    res = ctx.circuit_bootstrap_raw(cts.reshape(1, 4, big), lut)
    assert np.array_equal(res[0], ok.circuit_bootstrap(cts, lut.as_array(), 4))
    assert aes_128.bits_to_u8([0] * 4 + list(ck.decrypt_bits_raw(res[0]))) == f(0b1011)
