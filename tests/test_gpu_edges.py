"""Edge cases of the batched device path: empty and ragged batches, argument errors.

Ragged: the blind rotations pack 3 ciphertexts (PBS / vertical packing, br512x4) or 1 (br512lat)
per workgroup, so output counts that are not multiples of 3 and single-group batches exercise the
partial workgroups; every output is compared with the oracle or decrypted.
"""
import ctypes as C
import os

import numpy as np
import pytest

import tfhe_aes
from tfhe_aes import _native as N
from tfhe_aes import aes_128

pytestmark = pytest.mark.gpu

BIG = 4 * 512 + 1


def _vp(a):
    return a.ctypes.data_as(C.c_void_p)


@pytest.fixture(scope="module")
def client(product_raw):
    return product_raw[0]


def test_empty_batches(gpu_context, client):
    lut = gpu_context.generate_lookup_table(8, 8, lambda v: aes_128.SBOX[v])
    out = gpu_context.circuit_bootstrap_raw(np.zeros((0, 8, BIG), dtype=np.uint64), lut)
    assert out.shape == (0, 8, BIG)
    rk = client.encrypt_bits_raw([0] * 1408, start_index=1 << 30)
    blocks = np.zeros((0, 128, BIG), dtype=np.uint64)
    out = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt.encrypt_blocks_raw(gpu_context, rk, blocks, 2)
    assert out.shape == (0, 128, BIG)
    z = np.zeros((1, BIG), dtype=np.uint64)
    N.check(N.lib().tae_stage_keyswitch(gpu_context._h, _vp(z), 0, _vp(z), N.TAE_MEM_HOST))
    N.check(N.lib().tae_stage_pbs_shift_boolean(gpu_context._h, _vp(z), 0, 1, _vp(z), N.TAE_MEM_HOST))


@pytest.mark.parametrize("n_out", [1, 5, 24])
def test_ragged_outputs_bit_exact(gpu_context, oracle_keys, client, n_out):
    """8 -> n_out LUTs (vertical packing with n_out % 3 != 0 and the 24-output galois LUT), two groups."""
    f = lambda v: (aes_128.SBOX[v] * 0x10101 ^ v) & ((1 << n_out) - 1)
    lut = gpu_context.generate_lookup_table(8, n_out, f)
    vals = [0x3C, 0xA7]
    bits = np.stack([client.encrypt_bits_raw(aes_128.u8_to_bits(v), start_index=80_000 + 8 * i + 100 * n_out)
                     for i, v in enumerate(vals)])
    out = gpu_context.circuit_bootstrap_raw(bits, lut)
    for g, v in enumerate(vals):
        got = [int(b) for b in client.decrypt_bits_raw(out[g])]
        assert got == [(f(v) >> (n_out - 1 - j)) & 1 for j in range(n_out)], (g, hex(v))
    assert np.array_equal(out[1], oracle_keys.circuit_bootstrap(bits[1], lut.as_array(), n_out))


def test_argument_errors(gpu_context, client):
    lut = gpu_context.generate_lookup_table(8, 8, lambda v: v)
    bits = np.zeros((1, 7, BIG), dtype=np.uint64)
    with pytest.raises(tfhe_aes.TaeError) as e:
        gpu_context.circuit_bootstrap_raw(bits, lut)  # 7 bits for an 8-input LUT
    assert e.value.code == N.TAE_E_ARG
    z = np.zeros((2, BIG), dtype=np.uint64)
    for level in (0, 2):  # params_sqrd_lvl_64 has cbs_l = 1
        with pytest.raises(tfhe_aes.TaeError):
            N.check(N.lib().tae_stage_pbs_shift_boolean(gpu_context._h, _vp(z), 1, level, _vp(z), N.TAE_MEM_HOST))
    rk = client.encrypt_bits_raw([0] * 1408, start_index=1 << 31)
    blocks = client.encrypt_bits_raw([0] * 128, start_index=(1 << 31) + 4096).reshape(1, 128, BIG)
    for rounds in (0, 11):
        with pytest.raises(tfhe_aes.TaeError) as e:
            aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt.encrypt_blocks_raw(gpu_context, rk, blocks, rounds)
        assert e.value.code == N.TAE_E_PARAM
    with pytest.raises(tfhe_aes.TaeError) as e:
        tfhe_aes.get_params(99)
    assert e.value.code == N.TAE_E_PARAM


def test_xor_batch_state(gpu_context, client):
    """tae_xor_batch = xor_state (data_model.rs:270-274) over a whole 128-bit state: decrypts to the
    XOR, noise levels add, and NoiseTooBig (max noise^2 64 at lvl_64) is raised before any write."""
    rng = np.random.default_rng(3)
    a_bits, b_bits = rng.integers(0, 2, 128), rng.integers(0, 2, 128)
    a = client.encrypt_bits_raw(a_bits, start_index=900_000)
    b = client.encrypt_bits_raw(b_bits, start_index=901_000)
    ref = (a + b).copy()
    lvl = gpu_context.xor_batch(a, b, np.full(128, 9, np.uint64), np.ones(128, np.uint64))
    assert np.array_equal(a, ref)
    assert list(lvl) == [10] * 128
    assert list(client.decrypt_bits_raw(a)) == list(a_bits ^ b_bits)
    before = a.copy()
    with pytest.raises(tfhe_aes.NoiseTooBig):
        gpu_context.xor_batch(a, b, np.full(128, 60, np.uint64), np.full(128, 5, np.uint64))
    assert np.array_equal(a, before)


def test_caller_stream_ordering(gpu_context, oracle_keys, client):
    """tae_set_caller_stream: a TAE_MEM_DEVICE call orders itself after the work queued on the caller's
    stream only (an event, no device-wide synchronize).  The input is produced by a non-blocking copy
    and an in-place fix-up on a torch side stream right before the call; the keyswitch output must equal
    the oracle's.  None restores the default."""
    torch = pytest.importorskip("torch")
    n = 6
    cts = client.encrypt_bits_raw([1, 0, 1, 1, 0, 1], start_index=1 << 31)
    side = torch.cuda.Stream()
    h = torch.from_numpy(cts.view(np.int64)).pin_memory()
    d_in = torch.zeros((n, BIG), dtype=torch.int64, device="cuda")
    d_out = torch.full((n, 678), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    try:
        gpu_context.set_caller_stream(side)
        with torch.cuda.stream(side):
            d_in.copy_(h, non_blocking=True)
            d_in.add_(0)  # more work on the same stream
        N.check(N.lib().tae_stage_keyswitch(gpu_context._h, C.c_void_p(d_in.data_ptr()), n,
                                            C.c_void_p(d_out.data_ptr()), N.TAE_MEM_DEVICE))
    finally:
        gpu_context.set_caller_stream(None)
    out = d_out.cpu().numpy().view(np.uint64)
    for i in range(n):
        assert np.array_equal(out[i], oracle_keys.keyswitch(cts[i])), i


def test_caller_stream_key_schedule(gpu_context, client):
    """The TAE_MEM_DEVICE key schedule downloads its key after the caller's stream: the key is produced
    by a non-blocking copy on a torch side stream right before the call, and the device result must
    equal the host-array call's (key schedule fhe_sbox_gal_mul_pbs.rs:134-164)."""
    torch = pytest.importorskip("torch")
    E = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt
    key = client.encrypt_bits_raw(aes_128.blocks_to_bits([bytes(range(16))])[0], start_index=3_000_000)
    ref = E.key_schedule_raw(gpu_context, key)
    side = torch.cuda.Stream()
    h = torch.from_numpy(key.view(np.int64)).pin_memory()
    d_key = torch.zeros(h.shape, dtype=torch.int64, device="cuda")
    d_out = torch.zeros((44 * 32, BIG), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    try:
        gpu_context.set_caller_stream(side)
        with torch.cuda.stream(side):
            d_key.copy_(h, non_blocking=True)
            d_key.add_(0)
        N.check(E._fn("key_schedule_raw")(gpu_context._h, C.c_void_p(d_key.data_ptr()),
                                          C.c_void_p(d_out.data_ptr()), N.TAE_MEM_DEVICE))
    finally:
        gpu_context.set_caller_stream(None)
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), ref)


def test_context_shared_across_host_threads(gpu_context, client):
    """One context used from six host threads at once (the header's promise, and the reference's
    FheContext: Send + Sync): ctypes drops the GIL, the context's lock serialises the device work, and
    every thread gets exactly what a sequential call returns (1-3 blocks, one round, distinct inputs)."""
    from concurrent.futures import ThreadPoolExecutor
    E = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt
    rk = client.encrypt_bits_raw([(i * 7 + 3) & 1 for i in range(1408)], start_index=2_000_000)
    jobs = []
    for t in range(6):
        nb = 1 + t % 3
        bits = [(t * 31 + i * 13) >> 2 & 1 for i in range(128 * nb)]
        jobs.append(client.encrypt_bits_raw(bits, start_index=2_100_000 + 1000 * t).reshape(nb, 128, BIG))
    seq = [E.encrypt_blocks_raw(gpu_context, rk, cts, rounds=1) for cts in jobs]
    with ThreadPoolExecutor(max_workers=6) as pool:
        par = list(pool.map(lambda cts: E.encrypt_blocks_raw(gpu_context, rk, cts, rounds=1), jobs))
    for t in range(6):
        assert np.array_equal(par[t], seq[t]), t


def _pbs_main_cts(B):
    """The ciphertexts Engine::bootstrap gives the throughput kernel for a batch of B (kernels.hip): whole
    rounds of 3 x CUs, a remainder of at most min(TAE_BR_LAT_MAX, CUs) going to br512lat."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    lat_max = int(os.environ.get("TAE_BR_LAT_MAX", "256"))
    if B <= lat_max:
        return 0
    per_round = 3 * cus
    rest = B % per_round
    return B - rest if (B > per_round and 0 < rest <= min(lat_max, cus)) else B


def test_timing_modes_bit_identical(gpu_context, client):
    """tae_set_timing: mode 1 (HIP events per stage) and mode 2 (plus the in-kernel clock stamps of the
    throughput blind rotation, bench.py's effective_clock_ghz) leave the ciphertexts of a batched call
    bit-identical to mode 0; mode 2 fills the clock fields with a plausible shader clock; mode 3 is
    TAE_E_ARG (before mode 2 existed any nonzero value meant "on").  8 blocks x 1 round: one SubBytes
    circuit bootstrap of 1024 bits (on 256 CUs: one br512x4 launch of 768 + a br512lat remainder of 256)."""
    E = aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt
    rk = client.encrypt_bits_raw([(i * 5 + 1) >> 1 & 1 for i in range(1408)], start_index=7_000_000)
    nb = 8
    bits = [(i * 29 + 7) >> 3 & 1 for i in range(128 * nb)]
    blocks = client.encrypt_bits_raw(bits, start_index=7_100_000).reshape(nb, 128, BIG)
    outs = {}
    try:
        for mode in (0, 1, 2):
            N.check(N.lib().tae_set_timing(gpu_context._h, mode))
            outs[mode] = (E.encrypt_blocks_raw(gpu_context, rk, blocks, 1), gpu_context.last_stage_times())
    finally:
        N.check(N.lib().tae_set_timing(gpu_context._h, 0))
    assert np.array_equal(outs[1][0], outs[0][0]) and np.array_equal(outs[2][0], outs[0][0])
    t1, t2 = outs[1][1], outs[2][1]
    assert t1["pbs"] > 0 and t1["pbs_main"] > 0 and t1["pbs_main_cts"] == _pbs_main_cts(128 * nb) and "pbs_clock_ghz" not in t1, t1
    assert t2["pbs_clock_launches"] >= 1 and 1.0 < t2["pbs_clock_ghz"] < 3.0, t2
    assert N.lib().tae_set_timing(gpu_context._h, 3) == N.TAE_E_ARG
    assert N.lib().tae_set_timing(gpu_context._h, -1) == N.TAE_E_ARG
