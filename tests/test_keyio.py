"""On-disk key files (tae_keys_save / tae_keys_file_info / tae_keys_load, csrc/keyio.cpp).

The reference keeps keys in memory only, so there is no reference format to pin
against: the tests check round trips (server arrays bit-identical, the reloaded client key
encrypting identically at the same encryption index and continuing the encryption counter) and
that damaged files are rejected.  CPU only: no compute calls.
"""
import os

import numpy as np
import pytest

import tfhe_aes


@pytest.fixture(scope="module")
def key_file(product_raw, tmp_path_factory):
    ck, keys = product_raw
    path = tmp_path_factory.mktemp("keys") / "lvl64.taekey"
    tfhe_aes.save_keys(path, tfhe_aes.PARAMS_SQRD_LVL_64, ck, keys)
    return path


def test_info_and_round_trip(product_raw, key_file):
    ck, keys = product_raw
    assert tfhe_aes.key_file_info(key_file) == (tfhe_aes.PARAMS_SQRD_LVL_64, True, True)
    ck2, keys2 = tfhe_aes.load_keys(key_file)
    for a, b in zip(keys, keys2):
        assert a.dtype == b.dtype and np.array_equal(a, b)
    bits = [1, 0, 0, 1, 1]
    assert np.array_equal(ck.encrypt_bits_raw(bits, start_index=123_456),
                          ck2.encrypt_bits_raw(bits, start_index=123_456))
    assert list(ck2.decrypt_bits_raw(ck.encrypt_bits_raw(bits, start_index=9))) == bits


def test_encryption_counter_is_kept(product_raw, tmp_path):
    ck, _ = product_raw
    ck.encrypt(tfhe_aes.Cleartext(1))  # advance the counter
    path = tmp_path / "client.taekey"
    tfhe_aes.save_keys(path, tfhe_aes.PARAMS_SQRD_LVL_64, ck)
    assert tfhe_aes.key_file_info(path) == (tfhe_aes.PARAMS_SQRD_LVL_64, True, False)
    ck2, server = tfhe_aes.load_keys(path)
    assert server is None
    n = tfhe_aes.bit_len(tfhe_aes.PARAMS_SQRD_LVL_64)
    a, b = ck.encrypt(tfhe_aes.Cleartext(0)), ck2.encrypt(tfhe_aes.Cleartext(0))
    assert np.array_equal(a.data(n), b.data(n))  # same next encryption index, same randomness


def test_server_only_and_partial_load(product_raw, key_file, tmp_path):
    _, keys = product_raw
    path = tmp_path / "server.taekey"
    tfhe_aes.save_keys(path, tfhe_aes.PARAMS_SQRD_LVL_64, None, keys)
    assert tfhe_aes.key_file_info(path) == (tfhe_aes.PARAMS_SQRD_LVL_64, False, True)
    ck, keys2 = tfhe_aes.load_keys(path)
    assert ck is None and np.array_equal(keys2[1], keys[1])
    ck, none = tfhe_aes.load_keys(key_file, server=False)  # server payload skipped but checksummed
    assert ck is not None and none is None


def _damaged(src, dst, fn):
    data = bytearray(open(src, "rb").read())
    open(dst, "wb").write(fn(data))
    return dst


@pytest.mark.parametrize("how", ["flip", "truncate", "magic", "trailing"])
def test_damaged_files_are_rejected(key_file, tmp_path, how):
    def flip(d):
        d[len(d) // 2] ^= 0x10
        return d
    fn = {"flip": flip, "truncate": lambda d: d[:-100], "magic": lambda d: b"XAEKEY01" + d[8:],
          "trailing": lambda d: d + b"\0"}[how]
    bad = _damaged(key_file, tmp_path / f"{how}.taekey", fn)
    with pytest.raises(tfhe_aes.TaeError) as e:
        tfhe_aes.load_keys(bad)
    assert e.value.code == 5  # TAE_E_ARG
    assert "key file" in str(e.value)


def test_save_rejects_mismatched_params(product_raw, tmp_path):
    ck, _ = product_raw
    with pytest.raises(tfhe_aes.TaeError):
        tfhe_aes.save_keys(tmp_path / "x.taekey", tfhe_aes.PARAMS_WOPPBS_8BIT, ck)
    assert not os.path.exists(tmp_path / "y.taekey")


def _rehash(body):
    """The file checksum (keyio.cpp Hash): word-wise FNV-1a over a multiple of 8 bytes."""
    h = 0xcbf29ce484222325
    for i in range(0, len(body), 8):
        h = ((h ^ int.from_bytes(body[i:i + 8], "little")) * 0x100000001b3) & (2**64 - 1)
    return body + h.to_bytes(8, "little")


def test_legacy_v01_client_key_is_rejected(product_raw, tmp_path):
    """A TAEKEY01 client counter reserved the LOW indices its tae_encrypt ciphertexts used, which explicit
    raw ranges may now reach (tae_encrypt draws from 2^63 + counter): such a file must not load."""
    ck, _ = product_raw
    path = tmp_path / "client.taekey"
    tfhe_aes.save_keys(path, tfhe_aes.PARAMS_SQRD_LVL_64, ck)
    data = open(path, "rb").read()
    assert data[:8] == b"TAEKEY02" and len(data) == 64
    legacy = tmp_path / "legacy.taekey"
    open(legacy, "wb").write(_rehash(b"TAEKEY01" + data[8:-8]))
    with pytest.raises(tfhe_aes.TaeError) as e:
        tfhe_aes.load_keys(legacy)
    assert e.value.code == 5 and "legacy" in str(e.value)
    open(tmp_path / "v02.taekey", "wb").write(_rehash(data[:-8]))  # the re-hash itself is right
    assert tfhe_aes.load_keys(tmp_path / "v02.taekey")[0] is not None
