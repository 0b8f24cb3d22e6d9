"""Multi-GPU plumbing for the counter-mode AES workload.

Counter-mode blocks are independent (reference src/bin/main.rs:141-159 runs them in parallel), so
N blocks shard contiguously over the ranks with no collective on the data path.  The only
exchanges are one-time broadcasts from rank 0 of the server keys (KSK, standard BSK, PFPKSK:
672 MB for params_sqrd_lvl_64) and of the FHE-expanded round key, plus the max-over-ranks of the
timed region.  With the "nccl" backend (= RCCL on ROCm) the tensors live in HBM and travel over
xGMI; the same functions run on CPU tensors under "gloo" for the world_size-2 tests.
"""
import numpy as np

__all__ = ["shard_counters", "counter_blocks_for_rank", "encrypt_start_index", "broadcast_u64",
           "max_over_ranks", "min_over_ranks"]


def shard_counters(rank, world, blocks_per_rank, first=1):
    """Counters owned by `rank`: a contiguous run of blocks_per_rank values (weak scaling), so the
    union over ranks is first .. first + world * blocks_per_rank - 1 (main.rs:108-115 counts from 1)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of size {world}")
    start = first + rank * blocks_per_rank
    return range(start, start + blocks_per_rank)


def counter_blocks_for_rank(iv, rank, world, blocks_per_rank):
    """16-byte counter blocks iv || ctr_be64 of this rank (main.rs:108-115)."""
    if len(iv) != 8:
        raise ValueError("iv must be 8 bytes")
    return [bytes(iv) + c.to_bytes(8, "big") for c in shard_counters(rank, world, blocks_per_rank)]


def encrypt_start_index(rank, blocks_per_rank, base=1 << 32):
    """Disjoint encryption-stream indices per rank: every block bit is encrypted with its own
    ChaCha20 stream position, so no two ranks ever reuse mask/noise randomness."""
    return base + rank * blocks_per_rank * 128


def broadcast_u64(dist, arrays, lengths, rank, device):
    """Broadcast u64 arrays from rank 0.  `arrays` (rank 0 only) are numpy u64 arrays, `lengths`
    their element counts (known on every rank, e.g. from tae_server_key_sizes).  Returns int64
    tensors on `device` holding the same bits on every rank."""
    import torch
    out = []
    for i, n in enumerate(lengths):
        if rank == 0:
            a = np.ascontiguousarray(arrays[i], dtype=np.uint64).reshape(-1)
            if a.size != n:
                raise ValueError(f"array {i}: {a.size} elements, expected {n}")
            t = torch.from_numpy(a.view(np.int64)).to(device)
        else:
            t = torch.empty(int(n), dtype=torch.int64, device=device)
        dist.broadcast(t, src=0)
        out.append(t)
    return out


def _reduce(dist, value, op, dtype, device):
    import torch
    t = torch.tensor([value], dtype=dtype, device=device)
    dist.all_reduce(t, op=op)
    return t.item()


def max_over_ranks(dist, value, device):
    """Bench contract: the timed region is the max over ranks."""
    return float(_reduce(dist, float(value), dist.ReduceOp.MAX, __import__("torch").float64, device))


def min_over_ranks(dist, value, device):
    return int(_reduce(dist, int(value), dist.ReduceOp.MIN, __import__("torch").int32, device))
