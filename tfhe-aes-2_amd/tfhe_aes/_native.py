"""ctypes binding of libtfhe_aes_amd.so (include/tfhe_aes_gpu.h).

The library is built in-tree (``make -C tfhe-aes-2_amd``) and loaded from this directory.  There
is no CPU fallback: if the library is missing, importing this module raises, and every entry point
that needs the GPU returns TAE_E_NODEV on a machine without one.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TAE_LIB_PATH") or os.path.join(_HERE, "libtfhe_aes_amd.so")

TAE_OK, TAE_E_NOISE, TAE_E_INDEP, TAE_E_PARAM, TAE_E_HIP, TAE_E_ARG, TAE_E_NODEV = range(7)
TAE_MEM_HOST, TAE_MEM_DEVICE = 0, 1
TAE_INDEX_AUTO = 2**64 - 1  # tae_encrypt_*_raw: reserve fresh encryption indices from the key's counter
PARAMS_SQRD_LVL_1, PARAMS_SQRD_LVL_4, PARAMS_SQRD_LVL_64, PARAMS_SQRD_LVL_256 = 0, 1, 2, 3
PARAMS_WOPPBS_8BIT = 4  # shortint_woppbs_8bit.rs:39-86 (bits under the small key)
PARAMS_SHORTINT_1BIT = 5  # shortint_1bit.rs:62-83 (shortint bits under the small key, classic PBS)

# Every symbol include/tfhe_aes_gpu.h declares (checked by tests/test_capi_symbols.py).
EXPORTED = [
    "tae_last_error", "tae_version", "tae_device_count", "tae_get_params", "tae_generate_keys",
    "tae_server_key_sizes", "tae_generate_keys_raw", "tae_client_key_from_seed", "tae_context_create_raw", "tae_context_free",
    "tae_client_key_free", "tae_client_key_secrets", "tae_context_params", "tae_encrypt", "tae_decrypt",
    "tae_trivial", "tae_encrypt_bits_raw", "tae_decrypt_bits_raw", "tae_bit_clone", "tae_bit_free",
    "tae_bit_xor_assign", "tae_bit_noise_level", "tae_bit_data", "tae_bit_from_data",
    "tae_generate_lookup_table", "tae_lut_free", "tae_lut_data", "tae_circuit_bootstrap",
    "tae_circuit_bootstrap_raw", "tae_aes_encrypt_block_for_rounds", "tae_aes_encrypt_blocks",
    "tae_aes_key_schedule", "tae_aes_encrypt_blocks_raw", "tae_stage_keyswitch", "tae_stage_pbs_shift_boolean",
    "tae_stage_bootstrap", "tae_stage_pfks_ggsw", "tae_stage_ggsw_fourier", "tae_stage_vertical_packing",
    "tae_synchronize", "tae_set_caller_stream", "tae_set_timing", "tae_last_stage_times", "tae_bit_len", "tae_encrypt_ints_raw",
    "tae_decrypt_ints_raw", "tae_bootstrap_from_bits_raw", "tae_extract_bits_raw", "tae_aes_key_schedule_raw",
    "tae_last_stage_times_v2", "tae_keys_save", "tae_keys_file_info", "tae_keys_load",
    "tae_last_stage_times_v3", "tae_last_stage_times_v4", "tae_generate_multivariate_luts", "tae_xor_batch",
    "tae_aes_sbox_pbs_encrypt_blocks", "tae_aes_sbox_pbs_key_schedule", "tae_aes_sbox_pbs_encrypt_blocks_raw",
    "tae_aes_sbox_pbs_key_schedule_raw", "tae_aes_noise_schedule_check",
    "tae_s1_test_vector_from_fn", "tae_s1_bootstrap", "tae_s1_packing_keyswitch",
    "tae_s1_test_vectors_from_ciphertexts", "tae_s1_multivariate",
]
TAE_DRIVER_GAL_MUL, TAE_DRIVER_SBOX_PBS = 0, 1
TAE_KEYS_CLIENT, TAE_KEYS_SERVER = 1, 2


class TaeParams(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("n", "k", "N", "pbs_l", "pbs_b", "ks_l", "ks_b", "cbs_l", "cbs_b", "pfks_l", "pfks_b")] + [
        ("lwe_std", C.c_double), ("glwe_std", C.c_double), ("pfks_std", C.c_double),
        ("max_noise_sq", C.c_uint64), ("model", C.c_int)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


class TaeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class NoiseTooBig(TaeError):
    """MaxNoiseLevel::validate failure (shortint_woppbs_1bit.rs:74-76)."""


class NoiseNotIndependent(TaeError):
    """'noise components not independent' (shortint_woppbs_1bit.rs:64-70)."""


class NoDevice(TaeError):
    """No GPU: the product path has no CPU fallback."""


_ERRORS = {TAE_E_NOISE: NoiseTooBig, TAE_E_INDEP: NoiseNotIndependent, TAE_E_NODEV: NoDevice}

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C tfhe-aes-2_amd` "
                          "(the HIP path has no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    vp, u64, u64p, sz = C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_size_t
    vpp = C.POINTER(C.c_void_p)
    sig = {
        "tae_last_error": ([], C.c_char_p), "tae_version": ([], C.c_char_p),
        "tae_device_count": ([C.POINTER(C.c_int)], C.c_int),
        "tae_get_params": ([C.c_int, C.POINTER(TaeParams)], C.c_int),
        "tae_generate_keys": ([C.c_int, C.c_char_p, C.c_int, C.c_int, vpp, vpp], C.c_int),
        "tae_server_key_sizes": ([C.c_int, C.POINTER(sz), C.POINTER(sz), C.POINTER(sz)], C.c_int),
        "tae_generate_keys_raw": ([C.c_int, C.c_char_p, C.c_int, vpp, vp, vp, vp], C.c_int),
        "tae_client_key_from_seed": ([C.c_int, C.c_char_p, vpp], C.c_int),
        "tae_context_create_raw": ([C.c_int, C.c_int, vp, vp, vp, C.c_int, vpp], C.c_int),
        "tae_context_free": ([vp], None), "tae_client_key_free": ([vp], None),
        "tae_client_key_secrets": ([vp, vp, vp], C.c_int),
        "tae_context_params": ([vp, C.POINTER(TaeParams)], C.c_int),
        "tae_encrypt": ([vp, u64, vpp], C.c_int), "tae_decrypt": ([vp, vp, u64p], C.c_int),
        "tae_trivial": ([vp, u64, vpp], C.c_int),
        "tae_encrypt_bits_raw": ([vp, vp, sz, u64, vp], C.c_int),
        "tae_decrypt_bits_raw": ([vp, vp, sz, vp], C.c_int),
        "tae_bit_clone": ([vp, vpp], C.c_int), "tae_bit_free": ([vp], None),
        "tae_bit_xor_assign": ([vp, vp], C.c_int), "tae_bit_noise_level": ([vp, u64p], C.c_int),
        "tae_bit_data": ([vp, vp, sz], C.c_int), "tae_bit_from_data": ([vp, vp, sz, u64, vpp], C.c_int),
        "tae_generate_lookup_table": ([vp, C.c_int, C.c_int, vp, vpp], C.c_int),
        "tae_lut_free": ([vp], None), "tae_lut_data": ([vp, vp, sz, C.POINTER(sz)], C.c_int),
        "tae_circuit_bootstrap": ([vp, vp, sz, vp, vp], C.c_int),
        "tae_circuit_bootstrap_raw": ([vp, vp, sz, C.c_int, vp, vp, C.c_int], C.c_int),
        "tae_aes_encrypt_block_for_rounds": ([vp, vp, vp, C.c_int, vp], C.c_int),
        "tae_aes_encrypt_blocks": ([vp, vp, vp, sz, C.c_int, vp], C.c_int),
        "tae_aes_key_schedule": ([vp, vp, vp], C.c_int),
        "tae_aes_encrypt_blocks_raw": ([vp, vp, vp, sz, C.c_int, vp, C.c_int], C.c_int),
        "tae_aes_sbox_pbs_encrypt_blocks": ([vp, vp, vp, sz, C.c_int, vp], C.c_int),
        "tae_aes_sbox_pbs_key_schedule": ([vp, vp, vp], C.c_int),
        "tae_aes_sbox_pbs_encrypt_blocks_raw": ([vp, vp, vp, sz, C.c_int, vp, C.c_int], C.c_int),
        "tae_aes_sbox_pbs_key_schedule_raw": ([vp, vp, vp, C.c_int], C.c_int),
        "tae_aes_noise_schedule_check": ([C.c_int, C.c_int, C.c_int], C.c_int),
        "tae_stage_keyswitch": ([vp, vp, sz, vp, C.c_int], C.c_int),
        "tae_stage_pbs_shift_boolean": ([vp, vp, sz, C.c_int, vp, C.c_int], C.c_int),
        "tae_stage_bootstrap": ([vp, vp, sz, vp, vp, C.c_int], C.c_int),
        "tae_stage_pfks_ggsw": ([vp, vp, sz, C.c_int, vp, C.c_int], C.c_int),
        "tae_stage_ggsw_fourier": ([vp, vp, sz, vp, C.c_int], C.c_int),
        "tae_stage_vertical_packing": ([vp, vp, sz, C.c_int, vp, C.c_int, vp, C.c_int], C.c_int),
        "tae_synchronize": ([vp], C.c_int), "tae_set_timing": ([vp, C.c_int], C.c_int),
        "tae_set_caller_stream": ([vp, vp], C.c_int),
        "tae_last_stage_times": ([vp, C.POINTER(C.c_float)], C.c_int),
        "tae_bit_len": ([C.c_int, C.POINTER(sz)], C.c_int),
        "tae_encrypt_ints_raw": ([vp, vp, sz, u64, vp], C.c_int),
        "tae_decrypt_ints_raw": ([vp, vp, sz, vp], C.c_int),
        "tae_bootstrap_from_bits_raw": ([vp, vp, sz, vp, vp, C.c_int], C.c_int),
        "tae_extract_bits_raw": ([vp, vp, sz, vp, C.c_int], C.c_int),
        "tae_aes_key_schedule_raw": ([vp, vp, vp, C.c_int], C.c_int),
        "tae_last_stage_times_v2": ([vp, C.POINTER(C.c_float)], C.c_int),
        "tae_last_stage_times_v3": ([vp, C.POINTER(C.c_double)], C.c_int),
        "tae_last_stage_times_v4": ([vp, C.POINTER(C.c_double)], C.c_int),
        "tae_generate_multivariate_luts": ([C.c_int, C.c_int, C.c_int, vp, vp, sz], C.c_int),
        "tae_xor_batch": ([vp, vp, vp, sz, vp, vp, vp, C.c_int], C.c_int),
        "tae_keys_save": ([C.c_char_p, C.c_int, vp, vp, vp, vp], C.c_int),
        "tae_keys_file_info": ([C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)], C.c_int),
        "tae_keys_load": ([C.c_char_p, vpp, vp, vp, vp], C.c_int),
        "tae_s1_test_vector_from_fn": ([C.c_int, u64, u64, vp], C.c_int),
        "tae_s1_bootstrap": ([vp, vp, sz, vp, sz, vp, C.c_int], C.c_int),
        "tae_s1_packing_keyswitch": ([vp, vp, sz, vp, C.c_int], C.c_int),
        "tae_s1_test_vectors_from_ciphertexts": ([vp, vp, vp, sz, vp, C.c_int], C.c_int),
        "tae_s1_multivariate": ([vp, vp, sz, C.c_int, vp, C.c_int, vp, C.c_int], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(code: int) -> None:
    if code != TAE_OK:
        msg = lib().tae_last_error().decode()
        raise _ERRORS.get(code, TaeError)(code, msg)


def get_params(param_set: int) -> dict:
    p = TaeParams()
    check(lib().tae_get_params(param_set, C.byref(p)))
    return p.as_dict()


def bit_len(param_set: int) -> int:
    n = C.c_size_t(0)
    check(lib().tae_bit_len(param_set, C.byref(n)))
    return n.value


def device_count() -> int:
    n = C.c_int(0)
    check(lib().tae_device_count(C.byref(n)))
    return n.value
