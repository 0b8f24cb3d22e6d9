"""The oracle's fused-twiddle transforms tied back to the tfhe-fft-shaped radix schedule at the PBS level.

The product matches the oracle bit for bit, and for the product's two parameter sets the oracle runs the same
fused-twiddle transforms as the GPU (or_lf_* for params_sqrd_lvl_64, or_lf1k_* for the 8-bit set; DESIGN.md
§5.2).  Part of the GPU-vs-oracle parity is therefore self-consistency.  This file is the independent check.
One key set (SEED) is built twice from the same raw arrays: once with the product's transform, and once with
the radix schedule shaped like tfhe-fft (tfhe_oracle.h or_server_key_from_raw_t, OR_TRANSFORM_RADIX, the
blind rotation of every round before round 4).  Both then run the reference's calls on the same inputs:
  - homomorphic_shift_boolean, the PBS of circuit_bootstrap_boolean (tfhe-rs wop_pbs.rs, called through
    shortint_woppbs_1bit.rs:326-331), on 64 random bits per set;
  - a whole circuit bootstrap, 8 -> 24 SBOX + GF LUT on params_sqrd_lvl_64 (shortint_woppbs_1bit.rs:292-336)
    and 8 -> 8 SBOX without padding on the 8-bit set (shortint_woppbs_8bit.rs:299-335).
The two paths give different ciphertexts: the blind rotation's digits depend on the FFT rounding of every
earlier step.  Their decryptions must agree.  What is asserted:
  - identical decrypted values, equal to the expected ones;
  - |phase(fused) - phase(radix)| below a bound taken from measurement: 2^39.2 / 2^35.0 measured, asserted
    < 2^41 / < 2^37, against decryption margins of 2^50 / 2^57;
  - the fused path's PBS noise variance at most 1.0 x the radix path's.  The noise of these outputs is
    dominated by FFT rounding (glwe_std is 2^-52).  The fused transform has fewer rounded products and
    measured 0.64 x (params_sqrd_lvl_64) and 0.60 x (8-bit set) of the radix variance.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from tfhe_aes import aes_128

MASK = (1 << 64) - 1
THREADS = min(8, os.cpu_count() or 1)


def _signed(x):
    x &= MASK
    return x - (1 << 64) if x >= 1 << 63 else x


def _radix_twin(oracle_mod, keys):
    return oracle_mod.Keys(keys.pid, None, raw=keys.raw_server(), transform="radix")


def _pbs_both_ways(oracle_mod, keys, smalls, bits):
    radix = _radix_twin(oracle_mod, keys)
    with ThreadPoolExecutor(THREADS) as ex:  # ctypes drops the GIL for the oracle calls
        fused = list(ex.map(lambda s: keys.homomorphic_shift_boolean(s, 1), smalls))
        rad = list(ex.map(lambda s: radix.homomorphic_shift_boolean(s, 1), smalls))
    delta = 1 << (64 - keys.p["cbs_b"])  # homomorphic_shift_boolean -> bit * 2^(64 - cbs_b * level)
    ef = np.array([_signed(keys.phase(o) - int(b) * delta) for o, b in zip(fused, bits)], dtype=float)
    er = np.array([_signed(keys.phase(o) - int(b) * delta) for o, b in zip(rad, bits)], dtype=float)
    diff = np.array([_signed(keys.phase(a) - keys.phase(b)) for a, b in zip(fused, rad)], dtype=float)
    return ef, er, diff, delta


@pytest.mark.parametrize("which", ["lvl64", "8bit"])
def test_pbs_fused_vs_radix(oracle_mod, oracle_keys, oracle_keys8, which):
    keys = oracle_keys if which == "lvl64" else oracle_keys8
    rng = np.random.default_rng(17 if which == "lvl64" else 18)
    bits = rng.integers(0, 2, 64)
    if which == "lvl64":  # extract_dual_bit_from_bit: big-key bit -> keyswitch -> small key
        smalls = [keys.keyswitch(c) for c in keys.encrypt_bits(bits, b"\x55" * 32, 1000)]
    else:  # the 8-bit model's bits are small-key LWEs already
        smalls = list(keys.encrypt_small_bits(bits, b"\x55" * 32, 1000))
    ef, er, diff, delta = _pbs_both_ways(oracle_mod, keys, smalls, bits)
    # identical decryptions, both equal to the input bit (|error| well inside delta / 2)
    assert np.abs(ef).max() < delta / 4 and np.abs(er).max() < delta / 4
    bound = 2.0 ** (41 if which == "lvl64" else 37)
    assert np.abs(diff).max() < bound, np.log2(np.abs(diff).max())
    assert ef.var() <= 1.0 * er.var(), (ef.var() / er.var())


def test_pbs_fused_vs_radix_shortint1(oracle_mod):
    """The shortint_1bit set (N 512, k 4, 7 levels of 2^6) runs the same fused transform as lvl_64 on the
    product (br512x4<7, true, 6>) and in the oracle (lf_set).  Tie that deep decomposition back to the radix
    schedule: apply_programmable_bootstrap (shortint_1bit.rs:264-294, before its keyswitch) with a test
    vector per ciphertext (test_vector_from_cleartext_fn, :365-390), 128 random bits and functions.
    Outputs are 2-bit shortints (message + carry, delta 2^62), so errors are taken mod 2^63; margin 2^61.
    Measured: max errors 2^33.3 / 2^34.0 (fused / radix), phase difference < 2^34.3, variance ratio 0.88."""
    keys = oracle_mod.S1Keys(bytes(range(32)), threads=THREADS)
    radix = oracle_mod.S1Keys(None, raw=keys.raw_server(), transform="radix")
    rng = np.random.default_rng(19)
    n = 128
    bits, f0, f1 = (rng.integers(0, 2, n) for _ in range(3))
    cts = keys.s1_encrypt(bits, b"\x77" * 32, 2000)
    tvs = [keys.tv_from_fn(int(a), int(b)) for a, b in zip(f0, f1)]
    with ThreadPoolExecutor(THREADS) as ex:
        fused = list(ex.map(lambda i: keys.bootstrap_big(cts[i], tvs[i]), range(n)))
        rad = list(ex.map(lambda i: radix.bootstrap_big(cts[i], tvs[i]), range(n)))

    def err63(x):  # centred residue mod 2^63 (+-2^62 both decode to the same message bit)
        x &= (1 << 63) - 1
        return x - (1 << 63) if x >= 1 << 62 else x
    want = [(int(f1[i]) if bits[i] else int(f0[i])) << 62 for i in range(n)]
    ef = np.array([err63(keys.phase(fused[i]) - want[i]) for i in range(n)], dtype=float)
    er = np.array([err63(keys.phase(rad[i]) - want[i]) for i in range(n)], dtype=float)
    diff = np.array([_signed(keys.phase(a) - keys.phase(b)) for a, b in zip(fused, rad)], dtype=float)
    assert np.abs(ef).max() < 2.0 ** 40 and np.abs(er).max() < 2.0 ** 40  # margin 2^61
    assert np.abs(diff).max() < 2.0 ** 37, np.log2(np.abs(diff).max())
    assert ef.var() <= 1.0 * er.var(), (ef.var() / er.var())


def test_circuit_bootstrap_fused_vs_radix_lvl64(oracle_mod, oracle_keys, golden):
    """One 8 -> 24 WoP-PBS (SBOX + GF multiples with the gf quirk) per input, through both transforms."""
    keys = oracle_keys
    radix = _radix_twin(oracle_mod, keys)
    q = golden["sbox_galmul_quirk"]
    f = lambda x: (q[f"{x:02x}"][0] << 16) | (q[f"{x:02x}"][1] << 8) | q[f"{x:02x}"][2]
    lut = oracle_mod.generate_lut(512, 8, 24, f)
    for x in (0x53, 0xC4):
        cts = keys.encrypt_bits([(x >> (7 - i)) & 1 for i in range(8)], b"\x66" * 32, 8 * x)
        with ThreadPoolExecutor(2) as ex:
            a, b = ex.map(lambda k: k.circuit_bootstrap(cts, lut, 24), (keys, radix))
        da, db = keys.decrypt_bits(a), keys.decrypt_bits(b)
        assert list(da) == list(db)
        assert int("".join(map(str, da)), 2) == f(x)


def test_circuit_bootstrap_fused_vs_radix_8bit(oracle_mod, oracle_keys8):
    """bootstrap_with_lut's circuit bootstrap + vertical packing (8 -> 8 SBOX LUT without padding)."""
    keys = oracle_keys8
    radix = _radix_twin(oracle_mod, keys)
    lut = oracle_mod.generate_lut_without_padding(1024, lambda v: aes_128.SBOX[v])
    for x in (0x53,):  # one input: ~30 s per transform on one thread
        cts = keys.encrypt_small_bits(aes_128.u8_to_bits(x), b"\x66" * 32, 8 * x)
        with ThreadPoolExecutor(2) as ex:
            a, b = ex.map(lambda k: k.cbs_vp_small(cts, lut, 1), (keys, radix))
        assert int(keys.decrypt_ints(a)[0]) == int(keys.decrypt_ints(b)[0]) == aes_128.SBOX[x]
