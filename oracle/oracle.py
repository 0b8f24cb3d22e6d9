"""ctypes binding of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker, never the thing measured or shipped (see tfhe_oracle.h for the contract).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")

PARAMS_SQRD_LVL_1, PARAMS_SQRD_LVL_4, PARAMS_SQRD_LVL_64, PARAMS_SQRD_LVL_256 = 0, 1, 2, 3
PARAMS_WOPPBS_8BIT = 4  # shortint_woppbs_8bit.rs:39-86
PARAMS_SHORTINT_1BIT = 5  # shortint_1bit.rs:62-83
# blind-rotation transform of a server key built from raw arrays (tfhe_oracle.h or_server_key_from_raw_t)
TRANSFORMS = {"product": 0, "radix": 1}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


class _Params(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("n", "k", "N", "pbs_l", "pbs_b", "ks_l", "ks_b", "cbs_l", "cbs_b", "pfks_l", "pfks_b")] + [
        ("lwe_std", C.c_double), ("glwe_std", C.c_double), ("pfks_std", C.c_double),
        ("max_noise_sq", C.c_uint64), ("model", C.c_int)]


class _ClientKey(C.Structure):
    _fields_ = [("p", _Params), ("lwe_sk", C.POINTER(C.c_uint64)), ("glwe_sk", C.POINTER(C.c_uint64))]


class _ServerKey(C.Structure):
    _fields_ = [("p", _Params), ("ksk", C.POINTER(C.c_uint64)), ("bsk", C.POINTER(C.c_uint64)),
                ("pfpksk", C.POINTER(C.c_uint64)), ("bsk_f", C.c_void_p), ("fft", C.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        u64p = C.POINTER(C.c_uint64)
        L.or_params_get.argtypes = [C.c_int, C.POINTER(_Params)]
        L.or_gen_keys.argtypes = [C.c_int, C.c_char_p, C.c_int, C.POINTER(C.POINTER(_ClientKey)),
                                  C.POINTER(C.POINTER(_ServerKey))]
        L.or_server_key_from_raw.argtypes = [C.c_int, u64p, u64p, u64p]
        L.or_server_key_from_raw.restype = C.POINTER(_ServerKey)
        L.or_server_key_from_raw_t.argtypes = [C.c_int, u64p, u64p, u64p, C.c_int]
        L.or_server_key_from_raw_t.restype = C.POINTER(_ServerKey)
        L.or_client_key_free.argtypes = [C.c_void_p]
        L.or_server_key_free.argtypes = [C.c_void_p]
        for f in ("or_ksk_len", "or_bsk_len", "or_pfpksk_len"):
            getattr(L, f).argtypes = [C.POINTER(_Params)]
            getattr(L, f).restype = C.c_size_t
        L.or_chacha20_stream.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, C.c_char_p, C.c_size_t]
        L.or_closest_representable.argtypes = [C.c_uint64, C.c_int, C.c_int]
        L.or_closest_representable.restype = C.c_uint64
        L.or_decompose.argtypes = [C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_int64)]
        L.or_from_torus.argtypes = [C.c_double]
        L.or_from_torus.restype = C.c_uint64
        L.or_pbs_modulus_switch.argtypes = [C.c_uint64, C.c_int]
        L.or_pbs_modulus_switch.restype = C.c_uint64
        L.or_encode_bit.argtypes = [C.c_uint64]
        L.or_encode_bit.restype = C.c_uint64
        L.or_decode_bit.argtypes = [C.c_uint64]
        L.or_decode_bit.restype = C.c_uint64
        L.or_negacyclic_mul_exact.argtypes = [u64p, C.POINTER(C.c_int64), u64p, C.c_int]
        L.or_monomial_mul.argtypes = [u64p, u64p, C.c_int, C.c_int64]
        L.or_fft_new.argtypes = [C.c_int]
        L.or_fft_new.restype = C.c_void_p
        L.or_fft_free.argtypes = [C.c_void_p]
        L.or_fft_fwd_int.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_void_p]
        L.or_fft_fwd_torus.argtypes = [C.c_void_p, u64p, C.c_void_p]
        L.or_fft_add_bwd_torus.argtypes = [C.c_void_p, C.c_void_p, u64p]
        L.or_fft_raw_fwd.argtypes = [C.c_void_p, C.c_void_p]
        L.or_fft_raw_inv.argtypes = [C.c_void_p, C.c_void_p]
        L.or_encrypt_bit.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64, u64p]
        L.or_decrypt_bit.argtypes = [C.c_void_p, u64p]
        L.or_decrypt_bit.restype = C.c_uint64
        L.or_decrypt_phase.argtypes = [C.c_void_p, u64p]
        L.or_decrypt_phase.restype = C.c_uint64
        L.or_decrypt_small_phase.argtypes = [C.c_void_p, u64p]
        L.or_decrypt_small_phase.restype = C.c_uint64
        L.or_glwe_decrypt.argtypes = [C.c_void_p, u64p, u64p]
        L.or_keyswitch.argtypes = [C.c_void_p, u64p, u64p]
        L.or_external_product_add.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, u64p, u64p]
        L.or_bootstrap.argtypes = [C.c_void_p, u64p, u64p, u64p]
        L.or_homomorphic_shift_boolean.argtypes = [C.c_void_p, u64p, C.c_int, u64p]
        L.or_pfks.argtypes = [C.c_void_p, C.c_int, u64p, u64p]
        L.or_circuit_bootstrap_boolean.argtypes = [C.c_void_p, u64p, u64p]
        L.or_ggsw_to_fourier.argtypes = [C.c_void_p, u64p, C.c_int, C.c_void_p]
        L.or_vertical_packing.argtypes = [C.c_void_p, u64p, C.c_int, C.c_void_p, C.c_int, u64p]
        L.or_circuit_bootstrap.argtypes = [C.c_void_p, u64p, C.c_int, u64p, C.c_int, u64p]
        L.or_lut_small_len.argtypes = [C.c_int, C.c_int]
        L.or_lut_small_len.restype = C.c_size_t
        L.or_generate_lut.argtypes = [C.c_int, C.c_int, C.c_int, u64p, u64p]
        L.or_aes_encrypt_block.argtypes = [C.c_void_p, u64p, u64p, C.c_int, C.c_int, u64p]
        L.or_sub_bytes_gal_mul.argtypes = [C.c_void_p, u64p, C.c_int, C.c_int, u64p]
        L.or_plain_key_schedule.argtypes = [C.c_char_p, C.c_char_p]
        L.or_plain_encrypt_block.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_char_p]
        L.or_cbs_vp_small.argtypes = [C.c_void_p, u64p, C.c_int, u64p, C.c_int, u64p]
        L.or_encrypt_small_bit.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64, u64p]
        L.or_decrypt_small_bit.argtypes = [C.c_void_p, u64p]
        L.or_decrypt_small_bit.restype = C.c_uint64
        L.or_encrypt_int.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64, u64p]
        L.or_decrypt_int.argtypes = [C.c_void_p, u64p]
        L.or_decrypt_int.restype = C.c_uint64
        L.or_generate_lut_without_padding.argtypes = [C.c_int, u64p, u64p]
        L.or_extract_bits.argtypes = [C.c_void_p, u64p, C.c_int, C.c_int, u64p]
        L.or_bootstrap_with_lut8.argtypes = [C.c_void_p, u64p, u64p, u64p]
        L.or_gf_256_mul_terms.argtypes = [C.c_uint8, C.c_void_p]
        L.or_mix_column_terms.argtypes = [C.c_void_p]
        L.or_sub_bytes8.argtypes = [C.c_void_p, u64p, C.c_int, C.c_int, u64p]
        L.or_aes8_encrypt_block.argtypes = [C.c_void_p, u64p, u64p, C.c_int, C.c_int, u64p]
        L.or_gf_256_mul_quirk.argtypes = [C.c_uint8, C.c_uint8]
        L.or_gf_256_mul_quirk.restype = C.c_uint8
        L.or_s1_encrypt.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64, u64p]
        L.or_s1_decrypt.argtypes = [C.c_void_p, u64p]
        L.or_s1_decrypt.restype = C.c_uint64
        L.or_s1_tv_from_fn.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_uint64, u64p]
        L.or_s1_pks.argtypes = [C.c_void_p, u64p, u64p]
        L.or_s1_pack.argtypes = [C.c_void_p, u64p, C.c_int, u64p]
        L.or_s1_tv_from_cts.argtypes = [C.c_void_p, u64p, u64p, u64p]
        L.or_s1_bootstrap.argtypes = [C.c_void_p, u64p, u64p, u64p]
        L.or_s1_multivariate.argtypes = [C.c_void_p, u64p, C.c_int, u64p, u64p]
        _lib = L
    return _lib


def _p64(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def _pi64(a: np.ndarray):
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def params(pid: int) -> dict:
    p = _Params()
    assert lib().or_params_get(pid, C.byref(p)) == 0
    return {f: getattr(p, f) for f, _ in _Params._fields_}


class Keys:
    """Client + server key pair generated by the oracle's keygen (same spec as the product)."""

    def __init__(self, pid: int, seed: bytes, threads: int = 8, raw=None, transform: str = "product"):
        """transform (raw keys only): "product" = the blind rotation the product runs (the fused-twiddle
        transforms for params_sqrd_lvl_64 and the 8-bit set), "radix" = the tfhe-fft-shaped radix schedule."""
        L = lib()
        self.pid = pid
        self.p = params(pid)
        self.K = self.p["k"] * self.p["N"]
        self._ck = C.POINTER(_ClientKey)()
        if raw is None:
            self._sk = C.POINTER(_ServerKey)()
            assert L.or_gen_keys(pid, seed, threads, C.byref(self._ck), C.byref(self._sk)) == 0
        else:
            ksk, bsk, pfpksk = (np.ascontiguousarray(x, dtype=np.uint64) for x in raw)
            self._sk = L.or_server_key_from_raw_t(pid, _p64(ksk), _p64(bsk), _p64(pfpksk), TRANSFORMS[transform])
            self._ck = None

    def __del__(self):
        try:
            if self._ck:
                lib().or_client_key_free(C.cast(self._ck, C.c_void_p))
            if self._sk:
                lib().or_server_key_free(C.cast(self._sk, C.c_void_p))
        except Exception:
            pass

    @property
    def ck(self):
        return C.cast(self._ck, C.c_void_p)

    @property
    def sk(self):
        return C.cast(self._sk, C.c_void_p)

    def _arr(self, ptr, n):
        return np.ctypeslib.as_array(ptr, shape=(n,)).copy()

    def lwe_sk(self):
        return self._arr(self._ck.contents.lwe_sk, self.p["n"])

    def glwe_sk(self):
        return self._arr(self._ck.contents.glwe_sk, self.K)

    def raw_server(self):
        s = self._sk.contents
        pp = s.p
        L = lib()
        return (self._arr(s.ksk, L.or_ksk_len(C.byref(pp))), self._arr(s.bsk, L.or_bsk_len(C.byref(pp))),
                self._arr(s.pfpksk, L.or_pfpksk_len(C.byref(pp))))

    # --- client ---
    def encrypt_bits(self, bits, seed: bytes, start_index: int = 0) -> np.ndarray:
        out = np.zeros((len(bits), self.K + 1), dtype=np.uint64)
        for i, b in enumerate(bits):
            row = out[i]
            lib().or_encrypt_bit(self.ck, seed, start_index + i, int(b), _p64(row))
        return out

    def decrypt_bits(self, cts: np.ndarray) -> np.ndarray:
        cts = np.ascontiguousarray(cts.reshape(-1, self.K + 1))
        return np.array([lib().or_decrypt_bit(self.ck, _p64(cts[i])) for i in range(cts.shape[0])],
                        dtype=np.uint8)

    def phase(self, ct: np.ndarray) -> int:
        return lib().or_decrypt_phase(self.ck, _p64(np.ascontiguousarray(ct)))

    def small_phase(self, ct: np.ndarray) -> int:
        return lib().or_decrypt_small_phase(self.ck, _p64(np.ascontiguousarray(ct)))

    # --- server primitives ---
    def keyswitch(self, ct: np.ndarray) -> np.ndarray:
        out = np.zeros(self.p["n"] + 1, dtype=np.uint64)
        lib().or_keyswitch(self.sk, _p64(np.ascontiguousarray(ct)), _p64(out))
        return out

    def homomorphic_shift_boolean(self, small: np.ndarray, level: int = 1) -> np.ndarray:
        out = np.zeros(self.K + 1, dtype=np.uint64)
        lib().or_homomorphic_shift_boolean(self.sk, _p64(np.ascontiguousarray(small)), level, _p64(out))
        return out

    def pfks(self, q: int, big: np.ndarray) -> np.ndarray:
        out = np.zeros((self.p["k"] + 1) * self.p["N"], dtype=np.uint64)
        lib().or_pfks(self.sk, q, _p64(np.ascontiguousarray(big)), _p64(out))
        return out

    def circuit_bootstrap_boolean(self, small: np.ndarray) -> np.ndarray:
        p = self.p
        out = np.zeros(p["cbs_l"] * (p["k"] + 1) * (p["k"] + 1) * p["N"], dtype=np.uint64)
        lib().or_circuit_bootstrap_boolean(self.sk, _p64(np.ascontiguousarray(small)), _p64(out))
        return out

    def ggsw_to_fourier(self, ggsw: np.ndarray) -> np.ndarray:
        p = self.p
        out = np.zeros(p["cbs_l"] * (p["k"] + 1) * (p["k"] + 1) * (p["N"] // 2), dtype=np.complex128)
        lib().or_ggsw_to_fourier(self.sk, _p64(np.ascontiguousarray(ggsw)), p["cbs_l"],
                                 out.ctypes.data_as(C.c_void_p))
        return out

    def vertical_packing(self, lut_small: np.ndarray, ggsw_f: np.ndarray, n_in: int) -> np.ndarray:
        out = np.zeros(self.K + 1, dtype=np.uint64)
        lut_small = np.ascontiguousarray(lut_small, dtype=np.uint64)
        ggsw_f = np.ascontiguousarray(ggsw_f, dtype=np.complex128)
        lib().or_vertical_packing(self.sk, _p64(lut_small), len(lut_small) // self.p["N"],
                                  ggsw_f.ctypes.data_as(C.c_void_p), n_in, _p64(out))
        return out

    def circuit_bootstrap(self, bits: np.ndarray, lut: np.ndarray, n_out: int) -> np.ndarray:
        bits = np.ascontiguousarray(bits, dtype=np.uint64)
        n_in = bits.shape[0]
        out = np.zeros((n_out, self.K + 1), dtype=np.uint64)
        lib().or_circuit_bootstrap(self.sk, _p64(bits), n_in, _p64(np.ascontiguousarray(lut)), n_out,
                                   _p64(out))
        return out

    def sub_bytes_gal_mul(self, state_bytes: np.ndarray, threads: int) -> np.ndarray:
        state_bytes = np.ascontiguousarray(state_bytes, dtype=np.uint64)
        nb = state_bytes.size // (8 * (self.K + 1))
        out = np.zeros((nb, 24, self.K + 1), dtype=np.uint64)
        lib().or_sub_bytes_gal_mul(self.sk, _p64(state_bytes), nb, threads, _p64(out))
        return out

    def aes_encrypt_block(self, rk: np.ndarray, block: np.ndarray, rounds: int, threads: int = 8):
        out = np.zeros((128, self.K + 1), dtype=np.uint64)
        lib().or_aes_encrypt_block(self.sk, _p64(np.ascontiguousarray(rk)), _p64(np.ascontiguousarray(block)),
                                   rounds, threads, _p64(out))
        return out

    # --- 8-bit model (param id 4) ---
    def encrypt_small_bits(self, bits, seed: bytes, start_index: int = 0) -> np.ndarray:
        out = np.zeros((len(bits), self.p["n"] + 1), dtype=np.uint64)
        for i, b in enumerate(bits):
            lib().or_encrypt_small_bit(self.ck, seed, start_index + i, int(b), _p64(out[i]))
        return out

    def decrypt_small_bits(self, cts: np.ndarray) -> np.ndarray:
        cts = np.ascontiguousarray(cts.reshape(-1, self.p["n"] + 1))
        return np.array([lib().or_decrypt_small_bit(self.ck, _p64(cts[i])) for i in range(cts.shape[0])],
                        dtype=np.uint8)

    def encrypt_ints(self, values, seed: bytes, start_index: int = 0) -> np.ndarray:
        out = np.zeros((len(values), self.K + 1), dtype=np.uint64)
        for i, v in enumerate(values):
            lib().or_encrypt_int(self.ck, seed, start_index + i, int(v), _p64(out[i]))
        return out

    def decrypt_ints(self, cts: np.ndarray) -> np.ndarray:
        cts = np.ascontiguousarray(cts.reshape(-1, self.K + 1))
        return np.array([lib().or_decrypt_int(self.ck, _p64(cts[i])) for i in range(cts.shape[0])], dtype=np.uint64)

    def cbs_vp_small(self, bits: np.ndarray, lut: np.ndarray, n_out: int) -> np.ndarray:
        bits = np.ascontiguousarray(bits, dtype=np.uint64)
        out = np.zeros((n_out, self.K + 1), dtype=np.uint64)
        lib().or_cbs_vp_small(self.sk, _p64(bits), bits.shape[0], _p64(np.ascontiguousarray(lut, dtype=np.uint64)),
                              n_out, _p64(out))
        return out

    def extract_bits(self, ct: np.ndarray, delta_log: int = 56, nbits: int = 8) -> np.ndarray:
        out = np.zeros((nbits, self.p["n"] + 1), dtype=np.uint64)
        lib().or_extract_bits(self.sk, _p64(np.ascontiguousarray(ct, dtype=np.uint64)), delta_log, nbits, _p64(out))
        return out

    def bootstrap_with_lut8(self, bits: np.ndarray, lut: np.ndarray) -> np.ndarray:
        out = np.zeros((8, self.p["n"] + 1), dtype=np.uint64)
        lib().or_bootstrap_with_lut8(self.sk, _p64(np.ascontiguousarray(bits, dtype=np.uint64)),
                                     _p64(np.ascontiguousarray(lut, dtype=np.uint64)), _p64(out))
        return out

    def sub_bytes8(self, state: np.ndarray, threads: int = 8) -> np.ndarray:
        state = np.ascontiguousarray(state, dtype=np.uint64)
        nb = state.size // (8 * (self.p["n"] + 1))
        out = np.zeros((nb, 8, self.p["n"] + 1), dtype=np.uint64)
        lib().or_sub_bytes8(self.sk, _p64(state), nb, threads, _p64(out))
        return out

    def aes8_encrypt_block(self, rk: np.ndarray, block: np.ndarray, rounds: int, threads: int = 8):
        out = np.zeros((128, self.p["n"] + 1), dtype=np.uint64)
        lib().or_aes8_encrypt_block(self.sk, _p64(np.ascontiguousarray(rk, dtype=np.uint64)),
                                    _p64(np.ascontiguousarray(block, dtype=np.uint64)), rounds, threads, _p64(out))
        return out


class S1Keys(Keys):
    """shortint_1bit model (param id 5, src/tfhe/shortint_1bit.rs): bits are shortint ciphertexts under the
    SMALL key [n+1], test vectors are GLWEs [(k+1)N]."""

    def __init__(self, seed: bytes, threads: int = 8, raw=None, transform: str = "product"):
        super().__init__(PARAMS_SHORTINT_1BIT, seed, threads, raw, transform)
        self.L = self.p["n"] + 1
        self.G = (self.p["k"] + 1) * self.p["N"]

    def s1_encrypt(self, bits, seed: bytes, start_index: int = 0) -> np.ndarray:
        out = np.zeros((len(bits), self.L), dtype=np.uint64)
        for i, b in enumerate(bits):
            lib().or_s1_encrypt(self.ck, seed, start_index + i, int(b), _p64(out[i]))
        return out

    def s1_decrypt(self, cts: np.ndarray) -> np.ndarray:
        cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, self.L)
        return np.array([lib().or_s1_decrypt(self.ck, _p64(cts[i])) for i in range(cts.shape[0])], dtype=np.uint8)

    def glwe_decrypt(self, glwe: np.ndarray) -> np.ndarray:
        out = np.zeros(self.p["N"], dtype=np.uint64)
        lib().or_glwe_decrypt(self.ck, _p64(np.ascontiguousarray(glwe, dtype=np.uint64)), _p64(out))
        return out

    def tv_from_fn(self, f0: int, f1: int) -> np.ndarray:
        out = np.zeros(self.G, dtype=np.uint64)
        lib().or_s1_tv_from_fn(self.p["k"], self.p["N"], f0, f1, _p64(out))
        return out

    def pks(self, ct: np.ndarray) -> np.ndarray:
        out = np.zeros(self.G, dtype=np.uint64)
        lib().or_s1_pks(self.sk, _p64(np.ascontiguousarray(ct, dtype=np.uint64)), _p64(out))
        return out

    def pack(self, cts: np.ndarray) -> np.ndarray:
        cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, self.L)
        out = np.zeros(self.G, dtype=np.uint64)
        lib().or_s1_pack(self.sk, _p64(cts), cts.shape[0], _p64(out))
        return out

    def tv_from_cts(self, ct0: np.ndarray, ct1: np.ndarray) -> np.ndarray:
        out = np.zeros(self.G, dtype=np.uint64)
        lib().or_s1_tv_from_cts(self.sk, _p64(np.ascontiguousarray(ct0, dtype=np.uint64)),
                                _p64(np.ascontiguousarray(ct1, dtype=np.uint64)), _p64(out))
        return out

    def bootstrap_big(self, ct: np.ndarray, tv: np.ndarray) -> np.ndarray:
        """apply_programmable_bootstrap alone (blind rotation + sample extraction, before the keyswitch):
        the big-key LWE [k N + 1]"""
        out = np.zeros(self.K + 1, dtype=np.uint64)
        lib().or_bootstrap(self.sk, _p64(np.ascontiguousarray(ct, dtype=np.uint64)),
                           _p64(np.ascontiguousarray(tv, dtype=np.uint64)), _p64(out))
        return out

    def bootstrap(self, ct: np.ndarray, tv: np.ndarray) -> np.ndarray:
        out = np.zeros(self.L, dtype=np.uint64)
        lib().or_s1_bootstrap(self.sk, _p64(np.ascontiguousarray(ct, dtype=np.uint64)),
                              _p64(np.ascontiguousarray(tv, dtype=np.uint64)), _p64(out))
        return out

    def multivariate(self, bits: np.ndarray, f_table) -> np.ndarray:
        bits = np.ascontiguousarray(bits, dtype=np.uint64).reshape(-1, self.L)
        tab = np.ascontiguousarray(np.array(f_table, dtype=np.uint64))
        assert len(tab) == 1 << bits.shape[0]
        out = np.zeros(self.L, dtype=np.uint64)
        lib().or_s1_multivariate(self.sk, _p64(bits), bits.shape[0], _p64(tab), _p64(out))
        return out


def generate_lut_without_padding(N: int, f) -> np.ndarray:
    tab = np.array([f(v) for v in range(256)], dtype=np.uint64)
    out = np.zeros(max(N, 256), dtype=np.uint64)
    lib().or_generate_lut_without_padding(N, _p64(tab), _p64(out))
    return out


def gf_256_mul_terms(b: int) -> np.ndarray:
    out = np.zeros((8, 8), dtype=np.int32)
    lib().or_gf_256_mul_terms(b, out.ctypes.data_as(C.c_void_p))
    return out


def mix_column_terms() -> np.ndarray:
    out = np.zeros((32, 32), dtype=np.int32)
    lib().or_mix_column_terms(out.ctypes.data_as(C.c_void_p))
    return out


def generate_lut(N: int, input_bits: int, output_bits: int, f) -> np.ndarray:
    tab = np.array([f(v) for v in range(1 << input_bits)], dtype=np.uint64)
    small = lib().or_lut_small_len(N, input_bits)
    out = np.zeros(small * output_bits, dtype=np.uint64)
    lib().or_generate_lut(N, input_bits, output_bits, _p64(tab), _p64(out))
    return out


def plain_key_schedule(key: bytes) -> bytes:
    rk = C.create_string_buffer(176)
    lib().or_plain_key_schedule(bytes(key), rk)
    return rk.raw


def plain_encrypt_block(rk: bytes, block: bytes, rounds: int = 10) -> bytes:
    out = C.create_string_buffer(16)
    lib().or_plain_encrypt_block(bytes(rk), bytes(block), rounds, out)
    return out.raw


def chacha20_stream(key: bytes, nonce: int, counter: int, n: int) -> bytes:
    out = C.create_string_buffer(n)
    lib().or_chacha20_stream(bytes(key), nonce, counter, out, n)
    return out.raw


class FFT:
    def __init__(self, N: int):
        self.N = N
        self.h = lib().or_fft_new(N)
        assert self.h

    def __del__(self):
        try:
            lib().or_fft_free(self.h)
        except Exception:
            pass

    def fwd_int(self, poly: np.ndarray) -> np.ndarray:
        out = np.zeros(self.N // 2, dtype=np.complex128)
        lib().or_fft_fwd_int(self.h, _pi64(np.ascontiguousarray(poly, dtype=np.int64)), out.ctypes.data_as(C.c_void_p))
        return out

    def fwd_torus(self, poly: np.ndarray) -> np.ndarray:
        out = np.zeros(self.N // 2, dtype=np.complex128)
        lib().or_fft_fwd_torus(self.h, _p64(np.ascontiguousarray(poly, dtype=np.uint64)), out.ctypes.data_as(C.c_void_p))
        return out

    def add_bwd_torus(self, four: np.ndarray, out: np.ndarray) -> np.ndarray:
        four = np.ascontiguousarray(four, dtype=np.complex128)
        lib().or_fft_add_bwd_torus(self.h, four.ctypes.data_as(C.c_void_p), _p64(out))
        return out

    def raw_fwd(self, z: np.ndarray) -> np.ndarray:
        z = np.ascontiguousarray(z, dtype=np.complex128).copy()
        lib().or_fft_raw_fwd(self.h, z.ctypes.data_as(C.c_void_p))
        return z

    def raw_inv(self, z: np.ndarray) -> np.ndarray:
        z = np.ascontiguousarray(z, dtype=np.complex128).copy()
        lib().or_fft_raw_inv(self.h, z.ctypes.data_as(C.c_void_p))
        return z


class LfTransform:
    """The blind rotation's fused-twiddle transform for N = 512 or 1024 (tfhe_oracle.c or_lf_* /
    or_lf1k_*): forward of an integer digit polynomial, backward (torus add) of a spectrum that carries
    the factor E2, and E2's conjugate (the Fourier BSK rescale)."""

    def __init__(self, N: int = 512):
        assert N in (512, 1024)
        L = lib()
        self.N, self.M = N, N // 2
        pre = "or_lf_" if N == 512 else "or_lf1k_"
        new = getattr(L, "or_lf_plan_new" if N == 512 else "or_lf1k_plan_new")
        new.restype = C.c_void_p
        L.or_lf_any_free.argtypes = [C.c_void_p]
        self._fwd, self._bwd, self._e2 = (getattr(L, pre + n) for n in ("fwd", "bwd_add", "e2"))
        self._fwd.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_void_p]
        self._bwd.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
        self._e2.argtypes = [C.c_void_p, C.c_void_p]
        self.h = new()

    def __del__(self):
        try:
            lib().or_lf_any_free(self.h)
        except Exception:
            pass

    def fwd_int(self, poly: np.ndarray) -> np.ndarray:
        out = np.zeros(self.M, dtype=np.complex128)
        self._fwd(self.h, _pi64(np.ascontiguousarray(poly, dtype=np.int64)), out.ctypes.data_as(C.c_void_p))
        return out

    def add_bwd_torus(self, four: np.ndarray, out: np.ndarray) -> np.ndarray:
        four = np.ascontiguousarray(four, dtype=np.complex128)
        self._bwd(self.h, four.ctypes.data_as(C.c_void_p), _p64(out))
        return out

    def conj_e2(self) -> np.ndarray:
        out = np.zeros(self.M, dtype=np.complex128)
        self._e2(self.h, out.ctypes.data_as(C.c_void_p))
        return out


def decompose(x: int, base_log: int, levels: int):
    d = (C.c_int64 * levels)()
    lib().or_decompose(x, base_log, levels, d)
    return list(d)


def negacyclic_mul_exact(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    N = len(a)
    out = np.zeros(N, dtype=np.uint64)
    lib().or_negacyclic_mul_exact(_p64(np.ascontiguousarray(a, dtype=np.uint64)),
                                  _pi64(np.ascontiguousarray(b, dtype=np.int64)), _p64(out), N)
    return out
