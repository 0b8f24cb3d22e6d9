"""GPU parity: every stage of the HIP hot path against the CPU oracle on identical inputs and keys.

The bar is bit-exact for all stages, the f64 FFT ones included: the kernels execute the same fixed
sequence of IEEE f64 operations as the oracle's FFT schedule (explicit fma, -ffp-contract=off), so
ciphertexts and Fourier-domain GGSWs must match word for word.  Keys: both sides use the SEED key
set (tests/test_client.py proves product keygen == oracle keygen).
"""
import ctypes as C

import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import _native as N
from tfhe_aes import aes_128

pytestmark = pytest.mark.gpu

K = 4 * 512
BIG = K + 1
SMALL = 678


def _stage(fn, *args):
    N.check(fn(*args))


def _vp(a):
    return a.ctypes.data_as(C.c_void_p)


@pytest.fixture(scope="module")
def client(product_raw):
    return product_raw[0]


@pytest.fixture(scope="module")
def bits_cts(client):
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 2, size=24).astype(np.uint8)
    return bits, client.encrypt_bits_raw(bits, start_index=5000)


def test_keys_shared_with_oracle(product_raw, oracle_keys):
    _, (ksk, bsk, pfpksk) = product_raw
    oksk, obsk, opf = oracle_keys.raw_server()
    assert np.array_equal(ksk, oksk) and np.array_equal(bsk, obsk) and np.array_equal(pfpksk, opf)


def test_keyswitch_bit_exact(gpu_context, oracle_keys, bits_cts):
    bits, cts = bits_cts
    out = np.zeros((len(bits), SMALL), dtype=np.uint64)
    _stage(N.lib().tae_stage_keyswitch, gpu_context._h, _vp(cts), len(bits), _vp(out), N.TAE_MEM_HOST)
    for i in range(len(bits)):
        assert np.array_equal(out[i], oracle_keys.keyswitch(cts[i])), i


def test_pbs_shift_boolean_bit_exact(gpu_context, oracle_keys, bits_cts):
    bits, cts = bits_cts
    n = 4
    small = np.stack([oracle_keys.keyswitch(cts[i]) for i in range(n)])
    out = np.zeros((n, BIG), dtype=np.uint64)
    _stage(N.lib().tae_stage_pbs_shift_boolean, gpu_context._h, _vp(small), n, 1, _vp(out), N.TAE_MEM_HOST)
    for i in range(n):
        ref = oracle_keys.homomorphic_shift_boolean(small[i], 1)
        assert np.array_equal(out[i], ref), i
        # and it is an encryption of bit * 2^51
        ph = oracle_keys.phase(out[i])
        err = (ph - int(bits[i]) * (1 << 51)) % (1 << 64)
        assert min(err, (1 << 64) - err) < 1 << 45


@pytest.mark.parametrize("kernel", ["br512lat", "br512x4", "br512p16"])
def test_pbs_kernels_bit_exact(product_raw, oracle_keys, bits_cts, kernel, monkeypatch):
    """Every N=512 blind rotation on the same 7 ciphertexts: the small-batch latency kernel (one
    ciphertext per workgroup, levels in parallel) and the two throughput kernels (forced with
    TAE_BR_LAT_MAX=0; TAE_PBS_KERNEL picks br512x4, three ciphertexts per workgroup, or br512p16, two per
    workgroup with sixteen points per lane, the last workgroup holding one), each equal to the oracle word
    for word."""
    monkeypatch.setenv("TAE_BR_LAT_MAX", "256" if kernel == "br512lat" else "0")
    monkeypatch.setenv("TAE_PBS_KERNEL", "p16" if kernel == "br512p16" else "x4")
    ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, product_raw[1], device=0)
    bits, cts = bits_cts
    n = 7
    small = np.stack([oracle_keys.keyswitch(cts[i]) for i in range(n)])
    out = np.zeros((n, BIG), dtype=np.uint64)
    _stage(N.lib().tae_stage_pbs_shift_boolean, ctx._h, _vp(small), n, 1, _vp(out), N.TAE_MEM_HOST)
    for i in range(n):
        assert np.array_equal(out[i], oracle_keys.homomorphic_shift_boolean(small[i], 1)), i


@pytest.mark.parametrize("kernel", ["x4", "p16"])
def test_pbs_split_batch_bit_exact(product_raw, oracle_keys, client, kernel, monkeypatch):
    """A batch of C x 256 + 5 ciphertexts (C = 3 for br512x4, 2 for br512p16): whole rounds on the throughput
    kernel, the 5-ciphertext remainder on br512lat (Engine::bootstrap); ciphertexts from both parts equal
    the oracle's."""
    monkeypatch.setenv("TAE_PBS_KERNEL", kernel)
    gpu_context = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, product_raw[1], device=0)
    cpw = 3 if kernel == "x4" else 2
    B = cpw * 256 + 5
    bits = np.random.default_rng(7).integers(0, 2, size=B).astype(np.uint8)
    cts = client.encrypt_bits_raw(bits, start_index=40_000)
    small = np.zeros((B, SMALL), dtype=np.uint64)
    _stage(N.lib().tae_stage_keyswitch, gpu_context._h, _vp(cts), B, _vp(small), N.TAE_MEM_HOST)
    out = np.zeros((B, BIG), dtype=np.uint64)
    _stage(N.lib().tae_stage_pbs_shift_boolean, gpu_context._h, _vp(small), B, 1, _vp(out), N.TAE_MEM_HOST)
    for i in (0, 1, cpw * 256 - 1, cpw * 256, B - 1):
        assert np.array_equal(out[i], oracle_keys.homomorphic_shift_boolean(small[i], 1)), i


def test_pfks_bit_exact(gpu_context, oracle_keys, bits_cts):
    bits, cts = bits_cts
    n = 2
    big = np.stack([oracle_keys.homomorphic_shift_boolean(oracle_keys.keyswitch(cts[i]), 1) for i in range(n)])
    out = np.zeros((n, 5, 5 * 512), dtype=np.uint64)
    _stage(N.lib().tae_stage_pfks_ggsw, gpu_context._h, _vp(big), n, 1, _vp(out), N.TAE_MEM_HOST)
    for i in range(n):
        for q in range(5):
            assert np.array_equal(out[i, q], oracle_keys.pfks(q, big[i])), (i, q)


# coefficients whose base-2^16 digits hit the ends of their ranges: top digit +32768 / -32767, lower
# digit +-32768 (with and without the rounding carry), zero and all-ones
EXTREME = np.array([0x8000_8000_0000_0000, 0x7FFF_8000_0000_0000, 0x8001_7FFF_8000_0000, 0x8000_8000_8000_0000,
                    0x0000_8000_0000_0000, 0x0000_7FFF_8000_0000, 0xFFFF_8000_0000_0000, 0x7FFF_7FFF_7FFF_FFFF,
                    0, 0xFFFF_FFFF_FFFF_FFFF, 0x8000_0000_0000_0000, 0x8001_0000_8000_0000], dtype=np.uint64)


@pytest.fixture(scope="module")
def pfks_batch():
    """400 big LWEs: one full 384-ciphertext M tile of the K-layout GEMM and a ragged one (400 = 384 +
    16), three full and one ragged 128-ciphertext tiles of the row-limb layout; random coefficients,
    and rows 5 and 390 made of the digit-range extremes."""
    rng = np.random.default_rng(7)
    big = rng.integers(0, 2**63, size=(400, BIG), dtype=np.uint64) * np.uint64(2) + rng.integers(
        0, 2, size=(400, BIG), dtype=np.uint64)
    for row in (5, 390):
        big[row] = np.resize(EXTREME, BIG)
    return big


def _layout_context(product_raw, layout):
    """A context whose PFKS GEMM is forced to one operand layout (TAE_PFKS_LAYOUT, read at creation;
    the product picks the K layout from 2048 ciphertexts on)."""
    import os
    import tfhe_aes
    os.environ["TAE_PFKS_LAYOUT"] = layout
    try:
        return tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, product_raw[1], device=0)
    finally:
        del os.environ["TAE_PFKS_LAYOUT"]


@pytest.fixture(scope="module")
def layout_contexts(product_raw):
    return {lay: _layout_context(product_raw, lay) for lay in ("k", "k5", "rows")}


@pytest.mark.parametrize("layout", ["k", "k5", "rows"])
def test_pfks_gemm_ragged_bit_exact(layout_contexts, oracle_keys, pfks_batch, layout):
    """The PFKS GEMM (ksgemm::gemm_g6) in every operand layout -- K layout (4 limb slots per
    coefficient: the lower level's rare +32768 digits stored as -32768 and corrected by
    ksgemm::pfks_clamp_fixup; 384-ciphertext tiles, digit-offset correction), the same with 5 slots and no
    clamping ("k5"), and 6-bit row-tile limbs (384-row tiles = 128 ciphertexts x 3 limbs) -- on a ragged
    batch: rows from full and partial M tiles, including the digit-range extremes (rows 5 and 390 hold
    ~170 lower digits of +32768 each), equal the oracle's private functional keyswitch (the scalar u64
    kernel, used by params_sqrd_lvl_1, is pinned through
    test_gpu_model8.py::test_other_n1024_sets_bit_exact)."""
    ctx = layout_contexts[layout]
    big = pfks_batch
    out = np.zeros((len(big), 5, 5 * 512), dtype=np.uint64)
    _stage(N.lib().tae_stage_pfks_ggsw, ctx._h, _vp(big), len(big), 1, _vp(out), N.TAE_MEM_HOST)
    for i in (0, 5, 127, 128, 383, 384, 390, 399):
        for q in (0, 4):
            assert np.array_equal(out[i, q], oracle_keys.pfks(q, big[i])), (i, q)


def test_ggsw_fourier_bit_exact(gpu_context, oracle_keys, bits_cts):
    bits, cts = bits_cts
    small = oracle_keys.keyswitch(cts[0])
    ggsw = oracle_keys.circuit_bootstrap_boolean(small)
    out = np.zeros(5 * 5 * 256 * 2, dtype=np.float64)
    _stage(N.lib().tae_stage_ggsw_fourier, gpu_context._h, _vp(ggsw), 1, _vp(out), N.TAE_MEM_HOST)
    ref = oracle_keys.ggsw_to_fourier(ggsw)
    assert np.array_equal(out.view(np.uint64), ref.view(np.float64).view(np.uint64))


def test_vertical_packing_bit_exact(gpu_context, oracle_keys, oracle_mod, client):
    byte = 0xA7
    cts = client.encrypt_bits_raw(aes_128.u8_to_bits(byte), start_index=6000)
    gf = np.concatenate([oracle_keys.ggsw_to_fourier(oracle_keys.circuit_bootstrap_boolean(oracle_keys.keyswitch(c)))
                         for c in cts])
    f = lambda x: aes_128.SBOX[x]
    lut = oracle_mod.generate_lut(512, 8, 8, f)
    out = np.zeros((8, BIG), dtype=np.uint64)
    gfd = np.ascontiguousarray(gf).view(np.float64)
    _stage(N.lib().tae_stage_vertical_packing, gpu_context._h, _vp(gfd), 1, 8, _vp(lut), 8, _vp(out), N.TAE_MEM_HOST)
    for j in range(8):
        assert np.array_equal(out[j], oracle_keys.vertical_packing(lut[j * 512:(j + 1) * 512], gf, 8)), j
    assert aes_128.bits_to_u8(oracle_keys.decrypt_bits(out)) == aes_128.SBOX[byte]


def test_circuit_bootstrap_bit_exact(gpu_context, oracle_keys, client, golden):
    """FheContext::circuit_bootstrap 8 -> 24 (SBOX, 2S', 3S' with the gf quirk) for two bytes."""
    q = golden["sbox_galmul_quirk"]
    lut = gpu_context.generate_lookup_table(
        8, 24, lambda x: (q[f"{x:02x}"][0] << 16) | (q[f"{x:02x}"][1] << 8) | q[f"{x:02x}"][2])
    lut_arr = lut.as_array()
    bytes_in = [0x53, 0x00]
    cts = np.stack([client.encrypt_bits_raw(aes_128.u8_to_bits(b), start_index=7000 + 8 * i)
                    for i, b in enumerate(bytes_in)])
    out = gpu_context.circuit_bootstrap_raw(cts, lut)
    for i, b in enumerate(bytes_in):
        ref = oracle_keys.circuit_bootstrap(cts[i], lut_arr, 24)
        assert np.array_equal(out[i], ref), i
        v = client.decrypt_bits_raw(out[i])
        got = [aes_128.bits_to_u8(v[8 * m:8 * m + 8]) for m in range(3)]
        assert got == q[f"{b:02x}"]


def test_aes_one_round_bit_exact(gpu_context, oracle_keys, client, golden):
    g = golden["test_light"]
    ek = b"".join(aes_128.key_schedule_plain(bytes.fromhex(g["key"])))
    rk = client.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=10_000)
    blk = bytes.fromhex(golden["chacha20_zero_seed"]["block1"])
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits([blk]), start_index=20_000).reshape(1, 128, BIG)
    out = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt.encrypt_blocks_raw(gpu_context, rk, cts, rounds=1)
    ref = oracle_keys.aes_encrypt_block(rk, cts[0], 1, threads=16)
    assert np.array_equal(out[0], ref)
    assert aes_128.bits_to_blocks(client.decrypt_bits_raw(out))[0].hex() == g["block1"]["1"]


def test_aes_two_rounds_bit_exact_vs_oracle(gpu_context, oracle_keys, client, golden):
    """test_light_gal_mul (fhe_impls/shortint_woppbs_1bit.rs:185-193): 2 rounds vs plain, and the
    ciphertexts equal the oracle's word for word."""
    g = golden["test_light"]
    ek = b"".join(aes_128.key_schedule_plain(bytes.fromhex(g["key"])))
    rk = client.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=30_000)
    blk = bytes.fromhex(golden["chacha20_zero_seed"]["block1"])
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits([blk]), start_index=40_000).reshape(1, 128, BIG)
    out = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt.encrypt_blocks_raw(gpu_context, rk, cts, rounds=2)
    assert aes_128.bits_to_blocks(client.decrypt_bits_raw(out))[0].hex() == g["block1"]["2"]
    ref = oracle_keys.aes_encrypt_block(rk, cts[0], 2, threads=16)
    assert np.array_equal(out[0], ref)


def test_aes_ten_rounds_bit_exact_vs_oracle(gpu_context, oracle_keys, client, golden):
    """test_full (aes_128/test_helper.rs:22-84) at configs[1]: one counter block (README key / iv,
    counter 1) through all 10 rounds with a plain-expanded, encrypted round key.  Every ciphertext word
    of the output equals the oracle's, and it decrypts to the README's counter-mode block."""
    g = golden["readme_ctr"]
    ek = b"".join(aes_128.key_schedule_plain(bytes.fromhex(g["key"])))
    rk = client.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=50_000)
    blk = bytes.fromhex(g["blocks"]["1"])
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits([blk]), start_index=60_000).reshape(1, 128, BIG)
    out = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt.encrypt_blocks_raw(gpu_context, rk, cts, rounds=10)
    assert aes_128.bits_to_blocks(client.decrypt_bits_raw(out))[0].hex() == g["ciphertexts"]["1"]
    ref = oracle_keys.aes_encrypt_block(rk, cts[0], 10, threads=16)
    assert np.array_equal(out[0], ref)
