"""tfhe_aes -- MI355X-native homomorphic AES-128 (1-bit WoP-PBS), host mirror of the reference crate.

The crate name follows the reference (`tfhe_aes`, src/lib.rs); the compute path is the in-tree
HIP library libtfhe_aes_amd.so (no CPU fallback).
"""
from ._native import (PARAMS_SQRD_LVL_1, PARAMS_SQRD_LVL_4, PARAMS_SQRD_LVL_64, PARAMS_SQRD_LVL_256,
                      PARAMS_WOPPBS_8BIT, PARAMS_SHORTINT_1BIT, NoDevice, NoiseNotIndependent, NoiseTooBig, TaeError, bit_len, device_count,
                      get_params, lib)
from .tfhe import (BitCt, ClientKey, Cleartext, FheContext, WopbsLUT, client_key_from_seed, context_from_raw, decode_bit, encode_bit,
                   generate_keys, generate_keys_raw, key_file_info, load_keys, save_keys, server_key_sizes, generate_multivariate_luts)
from . import aes_128, shortint_1bit

__all__ = [
    "PARAMS_SQRD_LVL_1", "PARAMS_SQRD_LVL_4", "PARAMS_SQRD_LVL_64", "PARAMS_SQRD_LVL_256", "PARAMS_WOPPBS_8BIT",
    "PARAMS_SHORTINT_1BIT", "shortint_1bit",
    "bit_len", "NoDevice",
    "NoiseNotIndependent", "NoiseTooBig", "TaeError", "device_count", "get_params", "lib", "BitCt", "ClientKey",
    "Cleartext", "FheContext", "WopbsLUT", "client_key_from_seed", "context_from_raw", "decode_bit", "encode_bit", "generate_keys",
    "generate_keys_raw", "aes_128", "key_file_info", "load_keys", "save_keys", "server_key_sizes", "generate_multivariate_luts",
]
