"""CPU oracle checks: the restatement is pinned by the reference's own exact tests and golden vectors
before it is trusted as the GPU checker (tfhe_oracle.h header)."""
import ctypes

import numpy as np
import pytest

MASK = (1 << 64) - 1


def test_encode_decode(oracle_mod):
    L = oracle_mod.lib()
    # shortint_woppbs_1bit.rs:447-461
    assert L.or_encode_bit(0) == 0 and L.or_encode_bit(1) == 1 << 63
    for x, b in [(0, 0), (1, 0), (MASK, 0), (1 << 63, 1), ((1 << 63) - 1, 1), ((1 << 63) + 1, 1)]:
        assert L.or_decode_bit(x) == b


@pytest.mark.parametrize("base_log,levels", [(3, 4), (12, 3), (13, 1), (16, 2), (15, 2), (9, 4), (2, 6), (24, 1)])
def test_decompose_reconstructs_closest_representable(oracle_mod, base_log, levels):
    rng = np.random.default_rng(base_log * 100 + levels)
    xs = [int(v) for v in rng.integers(0, 2**63, size=200, dtype=np.uint64) * 2 + 1] + [0, MASK, 1 << 63]
    for x in xs:
        d = oracle_mod.decompose(x, base_log, levels)
        assert all(-(1 << (base_log - 1)) <= v <= (1 << (base_log - 1)) for v in d)
        rec = sum(v << (64 - base_log * (l + 1)) for l, v in enumerate(d)) & MASK
        assert rec == oracle_mod.lib().or_closest_representable(x, base_log, levels)
        err = (x - rec) & MASK
        err = err - (1 << 64) if err >= 1 << 63 else err
        assert abs(err) <= 1 << (64 - base_log * levels - 1)


@pytest.mark.parametrize("N", [512, 1024])
def test_fft_is_a_dft(oracle_mod, N):
    F = oracle_mod.FFT(N)
    M = N // 2
    rng = np.random.default_rng(N)
    z = rng.standard_normal(M) + 1j * rng.standard_normal(M)
    Z = F.raw_fwd(z)
    ref = np.fft.fft(z)
    assert np.max(np.abs(np.sort_complex(Z) - np.sort_complex(ref))) < 1e-12
    assert np.max(np.abs(F.raw_inv(Z) / M - z)) < 1e-14


@pytest.mark.parametrize("N", [512, 1024])
def test_fft_negacyclic_product_within_bound(oracle_mod, N):
    """FFT external-product arithmetic vs the exact integer negacyclic product mod 2^64.
    Tolerance: |error| < 2^32 torus units (observed ~2^28; decryption margin is 2^62)."""
    F = oracle_mod.FFT(N)
    rng = np.random.default_rng(7 + N)
    for _ in range(3):
        a = rng.integers(0, 2**64 - 1, size=N, dtype=np.uint64)
        b = rng.integers(-2048, 2049, size=N).astype(np.int64)
        exact = oracle_mod.negacyclic_mul_exact(a, b)
        out = np.zeros(N, dtype=np.uint64)
        F.add_bwd_torus(F.fwd_torus(a) * F.fwd_int(b), out)
        err = (out - exact).astype(np.int64)
        assert np.max(np.abs(err)) < 2**32


def test_lf_transform_is_the_negacyclic_dft(oracle_mod):
    """The blind rotation's fused-twiddle transform (N = 512) computes the same negacyclic
    DFT as the radix-16 schedule: forward of digit polynomials within 1e-15 relative of it, both within
    1e-12 of the definition sum; and it has no output factor."""
    F, T = oracle_mod.FFT(512), oracle_mod.LfTransform()
    rng = np.random.default_rng(11)
    j = np.arange(256)
    pos = np.arange(256)
    W = np.exp(1j * np.pi * j / 512)[None, :] * np.exp(
        -2j * np.pi * np.outer((pos >> 4) + 16 * (pos & 15), j) / 256)
    for _ in range(5):
        d = rng.integers(-2048, 2049, size=512).astype(np.int64)
        x_lf, x_std = T.fwd_int(d), F.fwd_int(d)
        exact = W @ (d[:256] + 1j * d[256:])
        scale = np.max(np.abs(exact))
        assert np.max(np.abs(x_lf - x_std)) / scale < 1e-15
        assert np.max(np.abs(x_lf - exact)) / scale < 1e-12


def test_lf_negacyclic_product_within_bound(oracle_mod):
    """The fused transform's external-product arithmetic against the exact negacyclic product mod 2^64 with
    the BSK-side spectrum times conj(E2) (what the rescaled Fourier BSK holds): the same 2^32 bound as the
    radix-16 schedule (test_fft_negacyclic_product_within_bound), and a round trip as tight as its."""
    F, T = oracle_mod.FFT(512), oracle_mod.LfTransform()
    e2 = T.conj_e2()
    assert np.allclose(np.abs(e2), 1.0)
    rng = np.random.default_rng(12)
    for _ in range(3):
        a = rng.integers(0, 2**64 - 1, size=512, dtype=np.uint64)
        b = rng.integers(-2048, 2049, size=512).astype(np.int64)
        exact = oracle_mod.negacyclic_mul_exact(a, b)
        out = np.zeros(512, dtype=np.uint64)
        T.add_bwd_torus(F.fwd_torus(a) * e2 * T.fwd_int(b), out)
        err = (out - exact).astype(np.int64)
        assert np.max(np.abs(err)) < 2**32
        rt_lf, rt_std = np.zeros(512, dtype=np.uint64), np.zeros(512, dtype=np.uint64)
        T.add_bwd_torus(F.fwd_torus(a) * e2, rt_lf)
        F.add_bwd_torus(F.fwd_torus(a), rt_std)
        e_lf = np.max(np.abs((rt_lf - a).astype(np.int64)))
        e_std = np.max(np.abs((rt_std - a).astype(np.int64)))
        assert e_lf < 4 * max(e_std, 1) and e_lf < 2**16


def test_lf1k_transform_is_the_negacyclic_dft(oracle_mod):
    """The N = 1024 fused-twiddle transform (the 8-bit model's PBS) against the radix-8
    schedule and the definition sum (positions 64 a + 8 b + c hold frequency a + 8 b + 64 c); no output
    factor."""
    F, T = oracle_mod.FFT(1024), oracle_mod.LfTransform(1024)
    rng = np.random.default_rng(13)
    j = np.arange(512)
    pos = np.arange(512)
    freq = (pos >> 6) + 8 * ((pos >> 3) & 7) + 64 * (pos & 7)
    W = np.exp(1j * np.pi * j / 1024)[None, :] * np.exp(-2j * np.pi * np.outer(freq, j) / 512)
    for _ in range(5):
        d = rng.integers(-64, 65, size=1024).astype(np.int64)
        x_lf, x_std = T.fwd_int(d), F.fwd_int(d)
        exact = W @ (d[:512] + 1j * d[512:])
        scale = np.max(np.abs(exact))
        assert np.max(np.abs(x_lf - x_std)) / scale < 1e-15
        assert np.max(np.abs(x_lf - exact)) / scale < 1e-12


def test_lf1k_negacyclic_product_within_bound(oracle_mod):
    """The N = 1024 fused transform's external-product arithmetic against the exact negacyclic product, the
    BSK side times conj(E2): within the radix-8 schedule's bound, and a round trip as tight as its."""
    F, T = oracle_mod.FFT(1024), oracle_mod.LfTransform(1024)
    e2 = T.conj_e2()
    assert np.allclose(np.abs(e2), 1.0)
    rng = np.random.default_rng(14)
    for _ in range(3):
        a = rng.integers(0, 2**64 - 1, size=1024, dtype=np.uint64)
        b = rng.integers(-64, 65, size=1024).astype(np.int64)
        exact = oracle_mod.negacyclic_mul_exact(a, b)
        out, ref = np.zeros(1024, dtype=np.uint64), np.zeros(1024, dtype=np.uint64)
        T.add_bwd_torus(F.fwd_torus(a) * e2 * T.fwd_int(b), out)
        F.add_bwd_torus(F.fwd_torus(a) * F.fwd_int(b), ref)
        err = np.max(np.abs((out - exact).astype(np.int64)))
        err_std = np.max(np.abs((ref - exact).astype(np.int64)))
        assert err < 2**32 and err < 4 * max(err_std, 1)
        rt_lf, rt_std = np.zeros(1024, dtype=np.uint64), np.zeros(1024, dtype=np.uint64)
        T.add_bwd_torus(F.fwd_torus(a) * e2, rt_lf)
        F.add_bwd_torus(F.fwd_torus(a), rt_std)
        e_lf = np.max(np.abs((rt_lf - a).astype(np.int64)))
        e_std = np.max(np.abs((rt_std - a).astype(np.int64)))
        assert e_lf < 4 * max(e_std, 1) and e_lf < 2**16


@pytest.mark.parametrize("N,dmax", [(512, 2048), (1024, 64)])
def test_lf_transforms_extreme_digits(oracle_mod, N, dmax):
    """Both fused transforms on the decompositions' extreme digits (every coefficient +-base/2, alternating
    and constant patterns, single spikes): forward within 1e-12 relative of the radix schedule, and the
    external-product arithmetic against the exact negacyclic product inside the radix schedule's bound."""
    F, T = oracle_mod.FFT(N), oracle_mod.LfTransform(N)
    e2 = T.conj_e2()
    rng = np.random.default_rng(N + dmax)
    pats = [np.full(N, dmax), np.full(N, -dmax), np.where(np.arange(N) % 2 == 0, dmax, -dmax),
            np.where(np.arange(N) < N // 2, dmax, -dmax), np.eye(1, N, 0)[0] * dmax, np.eye(1, N, N - 1)[0] * -dmax,
            rng.choice([-dmax, dmax], size=N)]
    for d in pats:
        d = d.astype(np.int64)
        x_lf, x_std = T.fwd_int(d), F.fwd_int(d)
        assert np.max(np.abs(x_lf - x_std)) <= 1e-12 * max(np.max(np.abs(x_std)), 1.0)
        a = rng.integers(0, 2**64 - 1, size=N, dtype=np.uint64)
        exact = oracle_mod.negacyclic_mul_exact(a, d)
        out, ref = np.zeros(N, dtype=np.uint64), np.zeros(N, dtype=np.uint64)
        T.add_bwd_torus(F.fwd_torus(a) * e2 * x_lf, out)
        F.add_bwd_torus(F.fwd_torus(a) * x_std, ref)
        err = np.max(np.abs((out - exact).astype(np.int64)))
        err_std = np.max(np.abs((ref - exact).astype(np.int64)))
        assert err < 2**40 and err <= 4 * max(err_std, 1)


def test_generate_luts_exact_layout(oracle_mod, golden):
    """shortint_woppbs_1bit.rs:665-697 (vertical packing and multi-polynomial LUT layout)."""
    lut = oracle_mod.generate_lut(16, 3, 2, lambda v: v)
    assert lut.size == 16 * 2
    for j, exp in enumerate(golden["lut_vertical_packing_3_2_16"]):
        assert list(lut[16 * j:16 * (j + 1)]) == [b << 63 for b in exp]
    lut = oracle_mod.generate_lut(8, 5, 2, lambda v: v)
    assert lut.size == 8 * 4 * 2
    for j, exp in enumerate(golden["lut_multipoly_5_2_8"]):
        assert list(lut[32 * j:32 * (j + 1)]) == [b << 63 for b in exp]


def test_keyswitch_and_pbs_phases(oracle_keys):
    K = oracle_keys
    cts = K.encrypt_bits([0, 1], b"\x11" * 32)
    assert list(K.decrypt_bits(cts)) == [0, 1]
    for bit, ct in zip([0, 1], cts):
        small = K.keyswitch(ct)
        ph = K.small_phase(small)
        assert ((ph + (1 << 62)) & MASK) >> 63 == bit  # dual bit under the small key
        big = K.homomorphic_shift_boolean(small, 1)
        ph = K.phase(big)
        delta = 1 << (64 - 13)  # homomorphic_shift_boolean -> bit * 2^(64 - cbs_b * level)
        err = (ph - bit * delta) & MASK
        err = err - (1 << 64) if err >= 1 << 63 else err
        assert abs(err) < 1 << 45


def test_circuit_bootstrap_sbox_galmul(oracle_keys, oracle_mod, golden):
    """One 8 -> 24 WoP-PBS (fhe_impls/shortint_woppbs_1bit.rs:94-128) incl. the gf quirk."""
    K = oracle_keys
    q = golden["sbox_galmul_quirk"]
    f = lambda x: (q[f"{x:02x}"][0] << 16) | (q[f"{x:02x}"][1] << 8) | q[f"{x:02x}"][2]
    lut = oracle_mod.generate_lut(512, 8, 24, f)
    for x in (0x00, 0xFF):
        cts = K.encrypt_bits([(x >> (7 - i)) & 1 for i in range(8)], b"\x22" * 32, x * 8)
        out = K.circuit_bootstrap(cts, lut, 24)
        bits = K.decrypt_bits(out)
        assert int("".join(map(str, bits)), 2) == f(x)


def test_oracle_aes_one_round(oracle_keys, golden):
    """encrypt_block_for_rounds(.., 1) on the oracle: ARK0 + last round (8->8 SBOX), keys encrypted."""
    K = oracle_keys
    g = golden["test_light"]
    key = bytes.fromhex(g["key"])
    from tfhe_aes import aes_128
    ek = b"".join(aes_128.key_schedule_plain(key))
    rk = K.encrypt_bits([b for byte in ek for b in aes_128.u8_to_bits(byte)], b"\x33" * 32)
    blk = bytes.fromhex(golden["chacha20_zero_seed"]["block1"])
    cts = K.encrypt_bits([b for byte in blk for b in aes_128.u8_to_bits(byte)], b"\x44" * 32)
    out = K.aes_encrypt_block(rk, cts, 1, threads=8)
    bits = K.decrypt_bits(out).reshape(16, 8)
    assert bytes(aes_128.bits_to_u8(b) for b in bits).hex() == g["block1"]["1"]


@pytest.mark.slow
def test_oracle_aes_light_two_rounds(oracle_keys, golden):
    """test_light (test_helper.rs:86-120): 2 rounds, key schedule done in plain then encrypted."""
    K = oracle_keys
    g = golden["test_light"]
    from tfhe_aes import aes_128
    ek = b"".join(aes_128.key_schedule_plain(bytes.fromhex(g["key"])))
    rk = K.encrypt_bits([b for byte in ek for b in aes_128.u8_to_bits(byte)], b"\x33" * 32)
    blk = bytes.fromhex(golden["chacha20_zero_seed"]["block1"])
    cts = K.encrypt_bits([b for byte in blk for b in aes_128.u8_to_bits(byte)], b"\x44" * 32)
    out = K.aes_encrypt_block(rk, cts, 2, threads=8)
    bits = K.decrypt_bits(out).reshape(16, 8)
    assert bytes(aes_128.bits_to_u8(b) for b in bits).hex() == g["block1"]["2"]
