"""Host mirror of the reference's shortint_1bit model (src/tfhe/shortint_1bit.rs) over the C-ABI.

Model with each ciphertext representing one bit: a tfhe-rs shortint ciphertext (message modulus 2, carry
modulus 1, EncryptionKeyChoice::Small: an LWE [n+1] under the small key, plaintext m * 2^62), XOR by
unchecked addition, and functions by classic programmable bootstrapping with test vectors -- of one bit
(test_vector_from_cleartext_fn) or of several through the selector tree of
calculate_multivariate_function, whose inner test vectors are built from ciphertexts by the packing
keyswitch (test_vector_from_ciphertexts).  Parameters: PARAMS_SHORTINT_1BIT (:62-83, the reference's
"testing parameters").  Every bootstrap, packing keyswitch and selector level runs batched on the GPU
(tfhe-aes-2_amd/csrc: Engine::s1_*); test vectors are host arrays [(k+1)N] u64.

Use a context and client key of param set PARAMS_SHORTINT_1BIT (tfhe.generate_keys / generate_keys_raw);
bits are raw arrays (ClientKey.encrypt_bits_raw / decrypt_bits_raw) or BitCt handles.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Sequence

import numpy as np

from . import _native as N
from ._native import check, lib
from .tfhe import BitCt, Cleartext, FheContext

PARAMS = N.PARAMS_SHORTINT_1BIT


def _vp(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64)


def _clear(c) -> int:
    return c.value if isinstance(c, Cleartext) else int(c)


def _glwe_len(ctx: FheContext) -> int:
    p = ctx.params
    return (p["k"] + 1) * p["N"]


class TestVector:
    """TestVector (:293-294): the GLWE accumulator a bootstrap rotates, [(k+1)N] u64."""
    __test__ = False  # not a pytest class

    def __init__(self, data: np.ndarray):
        self.data = _u64(data)


def _bits_array(bits) -> np.ndarray:
    if isinstance(bits, np.ndarray):
        return _u64(bits)
    return _u64(np.stack([b.data(b.context.lwe_size) if isinstance(b, BitCt) else b for b in bits]))


def test_vector_from_cleartext_fn(ctx: FheContext, f: Callable[[Cleartext], Cleartext]) -> TestVector:
    """FheContext::test_vector_from_cleartext_fn (:208-221, free fn :365-390)."""
    out = np.zeros(_glwe_len(ctx), dtype=np.uint64)
    check(lib().tae_s1_test_vector_from_fn(PARAMS, _clear(f(Cleartext(0))), _clear(f(Cleartext(1))), _vp(out)))
    return TestVector(out)


def test_vectors_from_ciphertexts(ctx: FheContext, bits0, bits1) -> np.ndarray:
    """FheContext::test_vector_from_ciphertexts (:225-237, free fn :392-492) for many pairs at once: [count][(k+1)N]."""
    a, b = _bits_array(bits0), _bits_array(bits1)
    if a.shape != b.shape:
        raise ValueError("the two ciphertext lists must have the same shape")
    out = np.zeros((a.shape[0], _glwe_len(ctx)), dtype=np.uint64)
    check(lib().tae_s1_test_vectors_from_ciphertexts(ctx._h, _vp(a), _vp(b), a.shape[0], _vp(out), N.TAE_MEM_HOST))
    return out


def test_vector_from_ciphertexts(ctx: FheContext, bit0, bit1) -> TestVector:
    return TestVector(test_vectors_from_ciphertexts(ctx, [bit0], [bit1])[0])


def packing_keyswitch(ctx: FheContext, cts) -> np.ndarray:
    """FheContext::packing_keyswitch (:240-254): GLWE [(k+1)N] with ciphertext j at coefficient j."""
    a = _bits_array(cts)
    out = np.zeros(_glwe_len(ctx), dtype=np.uint64)
    check(lib().tae_s1_packing_keyswitch(ctx._h, _vp(a), a.shape[0], _vp(out), N.TAE_MEM_HOST))
    return out


def bootstrap_raw(ctx: FheContext, cts, tvs) -> np.ndarray:
    """FheContext::bootstrap (:257-262, bootstrap_assign :264-291) over many bits: cts [B][n+1], tvs one TestVector / [n_tv][(k+1)N]
    (bit b takes tvs[b % n_tv])."""
    a = _bits_array(cts)
    t = _u64(tvs.data if isinstance(tvs, TestVector) else tvs).reshape(-1, _glwe_len(ctx))
    out = np.zeros_like(a)
    check(lib().tae_s1_bootstrap(ctx._h, _vp(a), a.shape[0], _vp(t), t.shape[0], _vp(out), N.TAE_MEM_HOST))
    return out


def bootstrap(ctx: FheContext, bit: BitCt, tv: TestVector) -> BitCt:
    """FheContext::bootstrap (:257-262): a new bit, noise reset, test vector applied."""
    return ctx.bit_from_data(bootstrap_raw(ctx, [bit], tv)[0], 0)


class MultivariateTestVector:
    """MultivariateTestVector (:512-517): the function table and its 2^(bits-1) cleartext test vectors
    (generated on the device side from the table)."""
    __test__ = False

    def __init__(self, bits: int, table: Sequence[int]):
        self.bits = bits
        self.table = _u64(table)


def generate_multivariate_test_vector(ctx: FheContext, bits: int, f: Callable[[int], Cleartext]) -> MultivariateTestVector:
    """generate_multivariate_test_vector (:519-536); f takes the u8 index of the bits (MSB first)."""
    if not 0 < bits <= 8:
        raise ValueError("0 < bits <= 8 (shortint_1bit.rs:526)")
    return MultivariateTestVector(bits, [_clear(f(v)) for v in range(1 << bits)])


def calculate_multivariate_function_raw(ctx: FheContext, bits: np.ndarray, mv: Sequence[MultivariateTestVector]) -> np.ndarray:
    """calculate_multivariate_function (:538-547, apply_selectors_rec :549-576) of several functions of the same bits, over many groups:
    bits [G][nbits][n+1] -> [G][len(mv)][n+1] (one batched bootstrap + packing step per selector level)."""
    nb = mv[0].bits
    if any(m.bits != nb for m in mv):
        raise ValueError("all functions must take the same number of bits")
    a = _u64(bits).reshape(-1, nb, ctx.lwe_size)
    tabs = _u64(np.stack([m.table for m in mv]))
    out = np.zeros((a.shape[0], len(mv), ctx.lwe_size), dtype=np.uint64)
    check(lib().tae_s1_multivariate(ctx._h, _vp(a), a.shape[0], nb, _vp(tabs), len(mv), _vp(out), N.TAE_MEM_HOST))
    return out


def calculate_multivariate_function(ctx: FheContext, bit_cts, mv_test_vector: MultivariateTestVector) -> BitCt:
    """calculate_multivariate_function (:538-547): bit_cts MSB first, len == mv_test_vector.bits."""
    a = _bits_array(bit_cts)
    if a.shape[0] != mv_test_vector.bits:
        raise ValueError("number of bits does not match the test vector (:502)")
    return ctx.bit_from_data(calculate_multivariate_function_raw(ctx, a[None], [mv_test_vector])[0, 0], 0)
