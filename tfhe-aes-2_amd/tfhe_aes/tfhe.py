"""Python mirror of the reference's `tfhe_aes::tfhe` model API over the C-ABI.

Reference: src/tfhe.rs:11-24 (ClientKeyT / ContextT) and src/tfhe/shortint_woppbs_1bit.rs
(BitCt :26-151, FheContext :165-336, ClientKey :189-226, encode/decode :125-132).  Names follow the
reference so tests read like its own (`client_key.encrypt(Cleartext(1))`, `context.circuit_bootstrap`).
All ciphertext arithmetic happens in libtfhe_aes_amd.so on the GPU; this module only marshals.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Callable, Sequence

import numpy as np

from . import _native as N
from ._native import check, lib

__all__ = ["Cleartext", "BitCt", "FheContext", "ClientKey", "WopbsLUT", "encode_bit", "decode_bit",
           "generate_keys", "generate_keys_raw", "client_key_from_seed", "context_from_raw", "server_key_sizes",
           "generate_multivariate_luts"]


@dataclass(frozen=True)
class Cleartext:
    value: int

    def __getitem__(self, i):  # Cleartext(..).0 in Rust
        assert i == 0
        return self.value


def encode_bit(bit: Cleartext) -> int:
    """shortint_woppbs_1bit.rs:125-128"""
    assert bit.value < 2, f"cleartext out of bounds: {bit.value}"
    return (bit.value << 63) & 0xFFFFFFFFFFFFFFFF


def decode_bit(encoding: int) -> Cleartext:
    """shortint_woppbs_1bit.rs:130-132"""
    return Cleartext((((encoding + (1 << 62)) & 0xFFFFFFFFFFFFFFFF) & (1 << 63)) >> 63)


class BitCt:
    """Handle to a shortint_woppbs_1bit::BitCt (LWE under the big key + noise bookkeeping)."""

    __slots__ = ("_h", "context")

    def __init__(self, handle, context: "FheContext | None"):
        self._h = C.c_void_p(handle)
        self.context = context

    def __del__(self):
        try:
            if self._h:
                lib().tae_bit_free(self._h)
                self._h = C.c_void_p(None)
        except Exception:
            pass

    def clone(self) -> "BitCt":
        out = C.c_void_p()
        check(lib().tae_bit_clone(self._h, C.byref(out)))
        return BitCt(out.value, self.context)

    def __ixor__(self, rhs: "BitCt") -> "BitCt":  # BitXorAssign (:134-142)
        check(lib().tae_bit_xor_assign(self._h, rhs._h))
        return self

    def __xor__(self, rhs: "BitCt") -> "BitCt":  # BitXor (:144-151): consumes self in Rust
        out = self.clone()
        out ^= rhs
        return out

    @property
    def noise_level_squared(self) -> int:
        v = C.c_uint64()
        check(lib().tae_bit_noise_level(self._h, C.byref(v)))
        return v.value

    def data(self, lwe_size: int) -> np.ndarray:
        arr = np.zeros(lwe_size, dtype=np.uint64)
        check(lib().tae_bit_data(self._h, arr.ctypes.data_as(C.c_void_p), lwe_size))
        return arr


def _handles(bits: Sequence[BitCt]):
    arr = (C.c_void_p * len(bits))()
    for i, b in enumerate(bits):
        arr[i] = b._h.value
    return arr


class WopbsLUT:
    """tfhe::shortint::wopbs::WopbsLUTBase produced by FheContext::generate_lookup_table."""

    def __init__(self, handle, input_bits: int, output_bits: int):
        self._h = C.c_void_p(handle)
        self.input_bits = input_bits
        self.output_bits = output_bits

    def __del__(self):
        try:
            if self._h:
                lib().tae_lut_free(self._h)
        except Exception:
            pass

    def as_array(self) -> np.ndarray:
        n = C.c_size_t()
        check(lib().tae_lut_data(self._h, None, 0, C.byref(n)))
        arr = np.zeros(n.value, dtype=np.uint64)
        check(lib().tae_lut_data(self._h, arr.ctypes.data_as(C.c_void_p), n.value, None))
        return arr

    def get_small_lut(self, j: int) -> np.ndarray:
        a = self.as_array()
        small = a.size // self.output_bits
        return a[j * small:(j + 1) * small]


class FheContext:
    """shortint_woppbs_1bit::FheContext -- server side, bound to one GPU."""

    def __init__(self, handle, param_set: int):
        self._h = C.c_void_p(handle)
        self.param_set = param_set
        p = N.TaeParams()
        check(lib().tae_context_params(self._h, C.byref(p)))
        self.params = p.as_dict()
        self.lwe_size = N.bit_len(param_set)  # one bit: K+1 (1-bit model) or n+1 (8-bit model)
        self.int_size = self.params["k"] * self.params["N"] + 1

    def __del__(self):
        try:
            if self._h:
                lib().tae_context_free(self._h)
        except Exception:
            pass

    # ContextT::trivial (src/tfhe.rs:20-24)
    def trivial(self, bit: Cleartext) -> BitCt:
        out = C.c_void_p()
        check(lib().tae_trivial(self._h, bit.value, C.byref(out)))
        return BitCt(out.value, self)

    def bit_from_data(self, data: np.ndarray, noise_level_squared: int = 1) -> BitCt:
        data = np.ascontiguousarray(data, dtype=np.uint64)
        out = C.c_void_p()
        check(lib().tae_bit_from_data(self._h, data.ctypes.data_as(C.c_void_p), data.size,
                                      noise_level_squared, C.byref(out)))
        return BitCt(out.value, self)

    # generate_lookup_table (:274-289)
    def generate_lookup_table(self, input_bits: int, output_bits: int, f: Callable[[int], int]) -> WopbsLUT:
        tab = np.array([f(v) & 0xFFFFFFFFFFFFFFFF for v in range(1 << input_bits)], dtype=np.uint64)
        out = C.c_void_p()
        check(lib().tae_generate_lookup_table(self._h, input_bits, output_bits, tab.ctypes.data_as(C.c_void_p),
                                              C.byref(out)))
        return WopbsLUT(out.value, input_bits, output_bits)

    # circuit_bootstrap (:292-336)
    def circuit_bootstrap(self, bits: Sequence[BitCt], lut: WopbsLUT) -> list:
        outs = (C.c_void_p * lut.output_bits)()
        check(lib().tae_circuit_bootstrap(self._h, _handles(bits), len(bits), lut._h, outs))
        return [BitCt(h, self) for h in outs]

    def circuit_bootstrap_raw(self, bits: np.ndarray, lut: WopbsLUT) -> np.ndarray:
        """Batched: bits [groups][n_in][K+1] -> [groups][n_out][K+1] (host arrays)."""
        bits = np.ascontiguousarray(bits, dtype=np.uint64)
        groups, n_in = bits.shape[0], bits.shape[1]
        out = np.zeros((groups, lut.output_bits, self.lwe_size), dtype=np.uint64)
        check(lib().tae_circuit_bootstrap_raw(self._h, bits.ctypes.data_as(C.c_void_p), groups, n_in, lut._h,
                                              out.ctypes.data_as(C.c_void_p), N.TAE_MEM_HOST))
        return out

    # ---- 8-bit model (shortint_woppbs_8bit.rs:268-336) ----
    def bootstrap_from_bits_raw(self, bits: np.ndarray, lut: WopbsLUT) -> np.ndarray:
        """FheContext::bootstrap_from_bits over bytes: [groups][8][n+1] -> int ciphertexts [groups][K+1]."""
        bits = np.ascontiguousarray(bits, dtype=np.uint64)
        out = np.zeros((bits.shape[0], self.int_size), dtype=np.uint64)
        check(lib().tae_bootstrap_from_bits_raw(self._h, bits.ctypes.data_as(C.c_void_p), bits.shape[0], lut._h,
                                                out.ctypes.data_as(C.c_void_p), N.TAE_MEM_HOST))
        return out

    def extract_bits_from_ciphertext_raw(self, ints: np.ndarray) -> np.ndarray:
        """FheContext::extract_bits_from_ciphertext: [groups][K+1] -> [groups][8][n+1], MSB first."""
        ints = np.ascontiguousarray(ints, dtype=np.uint64).reshape(-1, self.int_size)
        out = np.zeros((ints.shape[0], 8, self.lwe_size), dtype=np.uint64)
        check(lib().tae_extract_bits_raw(self._h, ints.ctypes.data_as(C.c_void_p), ints.shape[0],
                                         out.ctypes.data_as(C.c_void_p), N.TAE_MEM_HOST))
        return out

    def synchronize(self):
        check(lib().tae_synchronize(self._h))

    def set_caller_stream(self, stream):
        """Order TAE_MEM_DEVICE calls after the work queued on `stream` only (a torch.cuda.Stream, a raw
        hipStream_t int, or None for the default device-wide synchronize; include/tfhe_aes_gpu.h)."""
        handle = getattr(stream, "cuda_stream", stream)
        check(lib().tae_set_caller_stream(self._h, C.c_void_p(handle) if handle else None))

    def set_timing(self, on, clock: bool = False):
        """Per-stage HIP-event times of each batched call; clock=True also stamps the throughput blind-
        rotation launches in-kernel (effective shader clock, read back synchronously: diagnostic only)."""
        check(lib().tae_set_timing(self._h, (2 if clock else 1) if on else 0))

    def last_stage_times(self) -> dict:
        arr = (C.c_double * 12)()
        check(lib().tae_last_stage_times_v4(self._h, arr))
        d = dict(zip(("keyswitch", "pbs", "pfks", "ggsw_fft", "vertical_packing", "extract_bits", "linear"), list(arr)))
        d["pbs_launches"] = int(arr[7])
        d["pbs_main"], d["pbs_main_cts"] = arr[8], arr[9]
        if arr[11] > 0:
            d["pbs_clock_ghz"], d["pbs_clock_launches"] = arr[10], int(arr[11])
        return d

    def xor_batch(self, lhs: np.ndarray, rhs: np.ndarray, lhs_noise_sq=None, rhs_noise_sq=None):
        """BitXorAssign over whole bit arrays (xor_state, data_model.rs:270-274): lhs += rhs in place
        (host arrays [count][lwe]); with squared noise levels given, NoiseTooBig is enforced and the
        summed levels are returned."""
        if not (isinstance(lhs, np.ndarray) and lhs.dtype == np.uint64 and lhs.flags.c_contiguous):
            raise ValueError("lhs must be a C-contiguous uint64 array (updated in place)")
        rhs = np.ascontiguousarray(rhs, dtype=np.uint64)
        if lhs.size != rhs.size or lhs.size % self.lwe_size:
            raise ValueError("lhs and rhs must hold the same whole number of bit ciphertexts")
        count = lhs.size // self.lwe_size
        ln = rn = out = None
        if lhs_noise_sq is not None:
            ln = np.ascontiguousarray(lhs_noise_sq, dtype=np.uint64).ravel()
            rn = np.ascontiguousarray(rhs_noise_sq, dtype=np.uint64).ravel()
            if ln.size != count or rn.size != count:
                raise ValueError("one squared noise level per bit ciphertext")
            out = np.zeros(count, dtype=np.uint64)
        p = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None
        check(lib().tae_xor_batch(self._h, p(lhs), p(rhs), count, p(ln), p(rn), p(out), N.TAE_MEM_HOST))
        return out


class ClientKey:
    """shortint_woppbs_1bit::ClientKey (ClientKeyT, src/tfhe.rs:11-18)."""

    def __init__(self, handle, param_set: int, context: FheContext | None = None):
        self._h = C.c_void_p(handle)
        self.param_set = param_set
        self.context = context
        self.params = N.get_params(param_set)
        self.lwe_size = N.bit_len(param_set)
        self.int_size = self.params["k"] * self.params["N"] + 1

    def __del__(self):
        try:
            if self._h:
                lib().tae_client_key_free(self._h)
        except Exception:
            pass

    def encrypt(self, bit: Cleartext) -> BitCt:
        out = C.c_void_p()
        check(lib().tae_encrypt(self._h, bit.value, C.byref(out)))
        return BitCt(out.value, self.context)

    def decrypt(self, bit: BitCt) -> Cleartext:
        v = C.c_uint64()
        check(lib().tae_decrypt(self._h, bit._h, C.byref(v)))
        return Cleartext(v.value)

    def encrypt_bits_raw(self, bits, start_index: int | None = None) -> np.ndarray:
        """[count][lwe] ciphertexts of `bits` at encryption indices start_index.. (explicit, below 2^63,
        never reused for another plaintext) or, with start_index=None, fresh indices from the key."""
        start_index = N.TAE_INDEX_AUTO if start_index is None else start_index
        bits = np.ascontiguousarray(np.asarray(bits, dtype=np.uint8).ravel())
        out = np.zeros((bits.size, self.lwe_size), dtype=np.uint64)
        check(lib().tae_encrypt_bits_raw(self._h, bits.ctypes.data_as(C.c_void_p), bits.size, start_index,
                                         out.ctypes.data_as(C.c_void_p)))
        return out

    def decrypt_bits_raw(self, cts: np.ndarray) -> np.ndarray:
        cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, self.lwe_size)
        out = np.zeros(cts.shape[0], dtype=np.uint8)
        check(lib().tae_decrypt_bits_raw(self._h, cts.ctypes.data_as(C.c_void_p), cts.shape[0],
                                         out.ctypes.data_as(C.c_void_p)))
        return out

    # 8-bit model integers: shortint encrypt_without_padding / decrypt_without_padding
    def encrypt_ints_raw(self, values, start_index: int | None = None) -> np.ndarray:
        start_index = N.TAE_INDEX_AUTO if start_index is None else start_index
        values = np.ascontiguousarray(np.asarray(values, dtype=np.uint8).ravel())
        out = np.zeros((values.size, self.int_size), dtype=np.uint64)
        check(lib().tae_encrypt_ints_raw(self._h, values.ctypes.data_as(C.c_void_p), values.size, start_index,
                                         out.ctypes.data_as(C.c_void_p)))
        return out

    def decrypt_ints_raw(self, cts: np.ndarray) -> np.ndarray:
        cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, self.int_size)
        out = np.zeros(cts.shape[0], dtype=np.uint8)
        check(lib().tae_decrypt_ints_raw(self._h, cts.ctypes.data_as(C.c_void_p), cts.shape[0],
                                         out.ctypes.data_as(C.c_void_p)))
        return out

    def secrets(self):
        p = self.params
        lwe = np.zeros(p["n"], dtype=np.uint64)
        glwe = np.zeros(p["k"] * p["N"], dtype=np.uint64)
        check(lib().tae_client_key_secrets(self._h, lwe.ctypes.data_as(C.c_void_p), glwe.ctypes.data_as(C.c_void_p)))
        return lwe, glwe


def generate_multivariate_luts(poly_size: int, input_bits: int, output_bits: int, f: Callable[[int], int]) -> np.ndarray:
    """generate_multivariate_luts (shortint_woppbs_1bit.rs:366-403) for any polynomial size, no context:
    [output_bits * (poly_size << max(0, input_bits - log2 poly_size))] u64 (the reference's exact layout)."""
    tab = np.array([f(v) & 0xFFFFFFFFFFFFFFFF for v in range(1 << input_bits)], dtype=np.uint64)
    log_n = poly_size.bit_length() - 1
    n = output_bits * (poly_size << max(0, input_bits - log_n))
    out = np.zeros(n, dtype=np.uint64)
    check(lib().tae_generate_multivariate_luts(poly_size, input_bits, output_bits, tab.ctypes.data_as(C.c_void_p),
                                               out.ctypes.data_as(C.c_void_p), n))
    return out


def generate_keys(param_set: int = N.PARAMS_SQRD_LVL_64, seed: bytes | None = None, device: int = 0,
                  threads: int | None = None):
    """FheContext::generate_keys_with_params (shortint_woppbs_1bit.rs:245-268) -> (ClientKey, FheContext)."""
    seed = os.urandom(32) if seed is None else bytes(seed)
    assert len(seed) == 32
    threads = threads or min(16, os.cpu_count() or 1)
    ck, ctx = C.c_void_p(), C.c_void_p()
    check(lib().tae_generate_keys(param_set, seed, device, threads, C.byref(ck), C.byref(ctx)))
    context = FheContext(ctx.value, param_set)
    return ClientKey(ck.value, param_set, context), context


def generate_keys_raw(param_set: int = N.PARAMS_SQRD_LVL_64, seed: bytes | None = None, threads: int | None = None):
    """Client key + standard-domain server key arrays (ksk, bsk, pfpksk) on the host."""
    seed = os.urandom(32) if seed is None else bytes(seed)
    threads = threads or min(16, os.cpu_count() or 1)
    sizes = [C.c_size_t() for _ in range(3)]
    check(lib().tae_server_key_sizes(param_set, *[C.byref(s) for s in sizes]))
    ksk, bsk, pfpksk = (np.zeros(s.value, dtype=np.uint64) for s in sizes)
    ck = C.c_void_p()
    check(lib().tae_generate_keys_raw(param_set, seed, threads, C.byref(ck), ksk.ctypes.data_as(C.c_void_p),
                                      bsk.ctypes.data_as(C.c_void_p), pfpksk.ctypes.data_as(C.c_void_p)))
    return ClientKey(ck.value, param_set), (ksk, bsk, pfpksk)


def client_key_from_seed(param_set: int, seed: bytes) -> ClientKey:
    """Secret keys only, from the same seed streams as generate_keys_raw."""
    ck = C.c_void_p()
    check(lib().tae_client_key_from_seed(param_set, bytes(seed), C.byref(ck)))
    return ClientKey(ck.value, param_set)


def server_key_sizes(param_set: int) -> tuple:
    """u64 lengths of (ksk, bsk, pfpksk) for the parameter set (tae_server_key_sizes)."""
    sizes = [C.c_size_t() for _ in range(3)]
    check(lib().tae_server_key_sizes(param_set, *[C.byref(s) for s in sizes]))
    return tuple(s.value for s in sizes)


def _checked_key_arrays(param_set: int, keys) -> list:
    """The three raw server-key arrays as contiguous uint64 of exactly the sizes the parameter set
    needs (the C side reads that many words from each pointer)."""
    keys = list(keys)
    if len(keys) != 3:
        raise ValueError("server keys are (ksk, bsk, pfpksk)")
    out = []
    for name, k, n in zip(("ksk", "bsk", "pfpksk"), keys, server_key_sizes(param_set)):
        a = np.asarray(k)
        if a.dtype not in (np.uint64, np.int64):
            raise ValueError(f"{name}: expected 64-bit integer words, got {a.dtype}")
        a = np.ascontiguousarray(a).view(np.uint64).ravel()
        if a.size != n:
            raise ValueError(f"{name}: expected {n} u64 words for parameter set {param_set}, got {a.size}")
        out.append(a)
    return out


def context_from_raw(param_set: int, keys, device: int = 0, mem: int = N.TAE_MEM_HOST) -> FheContext:
    """Server context from raw keys: numpy arrays (mem=HOST) or device pointers as ints (mem=DEVICE;
    the caller guarantees each buffer holds server_key_sizes(param_set) words and has been written)."""
    if mem == N.TAE_MEM_HOST:
        arrs = _checked_key_arrays(param_set, keys)
        ptrs = [a.ctypes.data_as(C.c_void_p) for a in arrs]
    else:
        ptrs = [C.c_void_p(int(k)) for k in keys]
        if len(ptrs) != 3 or not all(p.value for p in ptrs):
            raise ValueError("device keys are three non-null pointers (ksk, bsk, pfpksk)")
    ctx = C.c_void_p()
    check(lib().tae_context_create_raw(param_set, device, ptrs[0], ptrs[1], ptrs[2], mem, C.byref(ctx)))
    return FheContext(ctx.value, param_set)


# ---- on-disk keys (include/tfhe_aes_gpu.h tae_keys_*; format in csrc/keyio.cpp) ----
def save_keys(path, param_set: int, client_key: "ClientKey | None" = None, server_keys=None) -> None:
    """Write a TAEKEY02 file with the client key (seed + encryption counter) and/or the raw server
    keys (ksk, bsk, pfpksk) as returned by generate_keys_raw."""
    ptrs = [None, None, None]
    if server_keys is not None:
        arrs = _checked_key_arrays(param_set, server_keys)
        ptrs = [a.ctypes.data_as(C.c_void_p) for a in arrs]
    check(lib().tae_keys_save(os.fsencode(path), param_set, client_key._h if client_key else None, *ptrs))


def key_file_info(path) -> tuple:
    """(param_set, has_client_key, has_server_keys) from the file header."""
    ps, fl = C.c_int(), C.c_int()
    check(lib().tae_keys_file_info(os.fsencode(path), C.byref(ps), C.byref(fl)))
    return ps.value, bool(fl.value & N.TAE_KEYS_CLIENT), bool(fl.value & N.TAE_KEYS_SERVER)


def load_keys(path, client: bool = True, server: bool = True):
    """(client_key or None, (ksk, bsk, pfpksk) or None) from a TAEKEY02 file; the checksum is
    verified before anything is returned."""
    param_set, has_ck, has_sk = key_file_info(path)
    client, server = client and has_ck, server and has_sk
    ptrs, arrs = [None, None, None], None
    if server:
        arrs = tuple(np.empty(n, dtype=np.uint64) for n in server_key_sizes(param_set))
        ptrs = [a.ctypes.data_as(C.c_void_p) for a in arrs]
    ck = C.c_void_p()
    check(lib().tae_keys_load(os.fsencode(path), C.byref(ck) if client else None, *ptrs))
    return (ClientKey(ck.value, param_set) if client else None), arrs
