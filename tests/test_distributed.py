"""World-size-2 and -8 tests of the multi-GPU path on CPU (gloo): the same functions bench.py runs over
RCCL on N MI355X (tfhe_aes/distributed.py); 8 is the driver's node size (configs[3]).

Each rank derives the client key from the shared seed, encrypts only its own shard of counter
blocks with a disjoint stream range, and receives the server keys by broadcast from rank 0.  The
tests check that the keys arrive bit-identical, that the shards partition 1..world*nb, that a
ciphertext encrypted on one rank decrypts on the next, and the max-over-ranks timing reduction.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from tests.conftest import PKG, ROOT, SEED  # noqa: E402

NB = 3  # blocks per rank
IV = bytes.fromhex("bdd219b8a08ded1a")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, world):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import tfhe_aes
    from tfhe_aes import aes_128
    from tfhe_aes import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # 1. server-key broadcast: bits identical on every rank (incl. values >= 2^63)
        rng = np.random.default_rng(7)
        lens = [4099, 5, 1]
        ref = [rng.integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True) for n in lens]
        ref[0][0] = np.uint64(2**64 - 1)
        got = D.broadcast_u64(dist, ref if rank == 0 else None, lens, rank, "cpu")
        for a, t in zip(ref, got):
            assert np.array_equal(t.numpy().view(np.uint64), a)

        # 2. counter shards partition 1 .. world * NB
        ctrs = list(D.shard_counters(rank, world, NB))
        everyone = [None] * world
        dist.all_gather_object(everyone, ctrs)
        flat = [c for r in everyone for c in r]
        assert sorted(flat) == list(range(1, world * NB + 1))
        blocks = D.counter_blocks_for_rank(IV, rank, world, NB)
        assert [int.from_bytes(b[8:], "big") for b in blocks] == ctrs and all(b[:8] == IV for b in blocks)

        # 3. client key derived independently per rank; rank r + 1's ciphertexts decrypt on rank r
        pid = tfhe_aes.PARAMS_SQRD_LVL_64
        ck = tfhe_aes.client_key_from_seed(pid, SEED)
        bits = aes_128.blocks_to_bits(blocks)
        cts = ck.encrypt_bits_raw(bits, start_index=D.encrypt_start_index(rank, NB))
        allcts = [None] * world
        dist.all_gather_object(allcts, (cts, blocks))
        other_cts, other_blocks = allcts[(rank + 1) % world]
        assert aes_128.bits_to_blocks(ck.decrypt_bits_raw(other_cts)) == other_blocks
        # disjoint encryption streams: no mask is shared between the ranks' ciphertexts
        masks = {allcts[r][0][i, :8].tobytes() for r in range(world) for i in range(len(allcts[r][0]))}
        assert len(masks) == sum(len(allcts[r][0]) for r in range(world))

        # 4. timing reduction and the correctness AND
        assert D.max_over_ranks(dist, 1.0 + rank, "cpu") == float(world)
        assert D.min_over_ranks(dist, int(rank != world - 1), "cpu") == 0
        assert D.min_over_ranks(dist, 1, "cpu") == 1
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_shards_and_key_broadcast(world):
    mp.spawn(_worker, args=(_free_port(), world), nprocs=world, join=True)


def test_shard_counters_edges():
    from tfhe_aes import distributed as D
    assert list(D.shard_counters(0, 1, 0)) == []
    assert list(D.shard_counters(7, 8, 128))[0] == 7 * 128 + 1
    assert list(D.shard_counters(7, 8, 128))[-1] == 1024
    with pytest.raises(ValueError):
        D.shard_counters(2, 2, 4)
    with pytest.raises(ValueError):
        D.counter_blocks_for_rank(b"short", 0, 1, 1)
    assert D.encrypt_start_index(1, 128) - D.encrypt_start_index(0, 128) == 128 * 128
