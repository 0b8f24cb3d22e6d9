"""The metric's own shapes on the GPU (BASELINE configs[2]) and the multi-rank device path.

- 128 counter-mode blocks in one batched call: every CBS launch is 128 x 16 x 8 = 16384 PBS, so
  Engine::bootstrap runs 21 whole rounds of br512x4 (16128 ciphertexts) plus a 256-ciphertext
  br512lat remainder, and vertical packing covers 128 x 16 x 24 outputs.  2 rounds keep it cheap
  (reduced-round semantics of plain.rs:75-103: ARK(rk0), one full round, final round with rk10).
  All 128 blocks decrypt to plain AES; the first block, the first block past the br512x4 /
  br512lat split (block 126: PBS index 16128) and the last equal the oracle word for word.
- A context built from device-resident server keys (tae_context_create_raw with TAE_MEM_DEVICE,
  what every rank > 0 of bench.py runs after the RCCL broadcast) computes the same ciphertexts as
  the host-built one, with device-resident inputs and outputs as well.
"""
import ctypes as C

import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import _native as N
from tfhe_aes import aes_128

pytestmark = pytest.mark.gpu

BIG = 4 * 512 + 1
E = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt


@pytest.fixture(scope="module")
def client(product_raw):
    return product_raw[0]


@pytest.fixture(scope="module")
def readme_setup(client, golden):
    g = golden["readme_ctr"]
    key, iv = bytes.fromhex(g["key"]), bytes.fromhex(g["iv"])
    ek = b"".join(aes_128.key_schedule_plain(key))
    rk = client.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=300_000)
    return key, iv, rk


def test_full_batch_128_blocks_two_rounds(gpu_context, oracle_keys, client, readme_setup):
    key, iv, rk = readme_setup
    nb = 128
    blocks = aes_128.counter_blocks(iv, nb)
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=400_000).reshape(nb, 128, BIG)
    out = E.encrypt_blocks_raw(gpu_context, rk, cts, rounds=2)
    got = aes_128.bits_to_blocks(client.decrypt_bits_raw(out))
    assert got == aes_128.expand_key_and_encrypt_blocks(key, blocks, 2)
    # 16384 PBS per launch = 21 x 768 (br512x4) + 256 (br512lat): block 126 starts the remainder
    for b in (0, 126, nb - 1):
        ref = oracle_keys.aes_encrypt_block(rk, cts[b], 2, threads=16)
        assert np.array_equal(out[b], ref), b


def test_full_batch_128_blocks_ten_rounds(gpu_context, oracle_keys, client, readme_setup):
    """The headline shape word for word through all 10 rounds (test_full_gal_mul,
    fhe_impls/shortint_woppbs_1bit.rs:195-210, at bench.py's 128 blocks): one batched call, every CBS
    launch 21 rounds of br512x4 + the br512lat remainder; all blocks decrypt to AES-128, and blocks 0,
    126 (the first past the br512x4 / remainder split) and 127 equal the oracle's 10-round output."""
    key, iv, rk = readme_setup
    nb = 128
    blocks = aes_128.counter_blocks(iv, nb)
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=800_000).reshape(nb, 128, BIG)
    out = E.encrypt_blocks_raw(gpu_context, rk, cts, rounds=10)
    got = aes_128.bits_to_blocks(client.decrypt_bits_raw(out))
    assert got == aes_128.expand_key_and_encrypt_blocks(key, blocks, 10)
    for b in (0, 126, nb - 1):
        ref = oracle_keys.aes_encrypt_block(rk, cts[b], 10, threads=16)
        assert np.array_equal(out[b], ref), b


def test_1024_blocks_one_call_one_round(gpu_context, oracle_keys, client, readme_setup):
    """BASELINE's largest N (1024 counter-mode blocks) in ONE call on one GPU: each CBS launch is
    1024 x 16 x 8 = 131072 PBS (43691 br512x4 workgroups, the last one holding two ciphertexts: the
    512-ciphertext remainder is too big for br512lat), 393216 vertical-packing outputs, and every
    scratch buffer grows to its size at that batch (GGSW scratch ~13 GB).  One round (ARK(rk0) + final
    round) keeps it cheap; all blocks decrypt to plain AES, the first and last equal the oracle."""
    key, iv, rk = readme_setup
    nb = 1024
    blocks = aes_128.counter_blocks(iv, nb)
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=700_000).reshape(nb, 128, BIG)
    out = E.encrypt_blocks_raw(gpu_context, rk, cts, rounds=1)
    got = aes_128.bits_to_blocks(client.decrypt_bits_raw(out))
    assert got == aes_128.expand_key_and_encrypt_blocks(key, blocks, 1)
    for b in (0, nb - 1):
        ref = oracle_keys.aes_encrypt_block(rk, cts[b], 1, threads=16)
        assert np.array_equal(out[b], ref), b


def test_configs3_rank7_of_8_shard(oracle_keys, product_raw, client):
    """BASELINE configs[3] (1024 blocks over 8 GPUs) as its LAST rank runs it, on this one GPU: exactly
    what bench.py does on rank 7 of world 8 with 128 blocks per GPU (main.rs:108-115 counters, sharded
    as main.rs:148-152 runs them): counters 897..1024 from D.counter_blocks_for_rank, encryption indices
    from D.encrypt_start_index(7, 128), a context built from torch-resident server keys with
    TAE_MEM_DEVICE (the RCCL broadcast's destination buffers), the round key resident on the device and
    encrypt_blocks_device.  2 rounds (reduced-round semantics); all 128 blocks decrypt to plain AES, and
    blocks 0, 126 (first past the br512x4 / br512lat split) and 127 equal the oracle word for word."""
    torch = pytest.importorskip("torch")
    from tfhe_aes import distributed as D
    rank, world, nb, rounds = 7, 8, 128, 2
    g_key = bytes.fromhex("76b8e0ada0f13d90405d6ae55386bd28")  # README key / iv (main.rs:108-115)
    g_iv = bytes.fromhex("bdd219b8a08ded1a")
    blocks = D.counter_blocks_for_rank(g_iv, rank, world, nb)
    assert int.from_bytes(blocks[0][8:], "big") == 897 and int.from_bytes(blocks[-1][8:], "big") == 1024
    _, keys = product_raw
    dev = [torch.from_numpy(k.view(np.int64)).to("cuda:0") for k in keys]
    ctx_d = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, [t.data_ptr() for t in dev], device=0,
                                      mem=N.TAE_MEM_DEVICE)
    ek = b"".join(aes_128.key_schedule_plain(g_key))
    rk = client.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=600_000)
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits(blocks),
                                  start_index=D.encrypt_start_index(rank, nb)).reshape(nb, 128, BIG)
    d_rk = torch.from_numpy(rk.view(np.int64)).to("cuda:0")
    d_in = torch.from_numpy(cts.view(np.int64)).to("cuda:0")
    d_out = torch.full_like(d_in, -1)
    torch.cuda.synchronize()
    E.encrypt_blocks_device(ctx_d, d_rk.data_ptr(), d_in.data_ptr(), nb, rounds, d_out.data_ptr())
    ctx_d.synchronize()
    out = d_out.cpu().numpy().view(np.uint64)
    got = aes_128.bits_to_blocks(client.decrypt_bits_raw(out))
    assert got == aes_128.expand_key_and_encrypt_blocks(g_key, blocks, rounds)
    for b in (0, 126, nb - 1):
        ref = oracle_keys.aes_encrypt_block(rk, cts[b], rounds, threads=16)
        assert np.array_equal(out[b], ref), b
    del ctx_d  # the context borrows the key buffers: free it first


def test_device_key_context_matches_host_context(gpu_context, product_raw, client, readme_setup):
    torch = pytest.importorskip("torch")
    _, keys = product_raw
    dev = [torch.from_numpy(k.view(np.int64)).to("cuda:0") for k in keys]
    ctx_d = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, [t.data_ptr() for t in dev], device=0,
                                      mem=N.TAE_MEM_DEVICE)
    key, iv, rk = readme_setup
    blocks = aes_128.counter_blocks(iv, 3)
    cts = client.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=500_000).reshape(3, 128, BIG)
    ref = E.encrypt_blocks_raw(gpu_context, rk, cts, rounds=1)
    assert np.array_equal(E.encrypt_blocks_raw(ctx_d, rk, cts, rounds=1), ref)
    # device-resident rk / blocks / output, written on torch's stream right before the call
    d_rk = torch.from_numpy(rk.view(np.int64)).to("cuda:0", non_blocking=True)
    d_in = torch.from_numpy(cts.view(np.int64)).to("cuda:0", non_blocking=True)
    d_out = torch.full_like(d_in, -1)
    E.encrypt_blocks_device(ctx_d, d_rk.data_ptr(), d_in.data_ptr(), 3, 1, d_out.data_ptr())
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), ref)
    assert aes_128.bits_to_blocks(client.decrypt_bits_raw(ref)) == aes_128.expand_key_and_encrypt_blocks(key, blocks, 1)
    del ctx_d  # the context borrows the key buffers: free it first
