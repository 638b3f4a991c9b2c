"""Codeword sharding across GPUs.

Codewords are independent, so a job of T codewords splits into contiguous
ranges, one per rank (one process per GPU, torch.distributed over RCCL on
the box, gloo in the CPU tests).  Each rank generates its own inputs from a
counter-based seed, decodes them with no data-path collective, and only the
three integer error counters (bit errors, frame errors, codewords) are summed
at the end -- a few bytes of all-reduce.  The device generator is counted by
the global codeword index (workload.make_symbols), so a codeword's data does
not depend on which rank or batch generates it.
"""
from __future__ import annotations

import hashlib

SEED_STRIDE = 1_000_003


def interleaver_digest(inv_perm):
    """63-bit digest of an inverse interleaver (int32 bytes).  The reference's
    default inv_perm = np.argsort(perm) breaks the ties of its non-bijective perm
    by the host numpy's sort path, so ranks on different hosts
    can hold different de-interleavers: the digest goes into a sweep's config
    key and is compared across ranks before any codeword is decoded."""
    import numpy as np
    b = np.ascontiguousarray(np.asarray(inv_perm, dtype=np.int32)).tobytes()
    return int.from_bytes(hashlib.sha256(b).digest()[:8], "little") >> 1


def check_same_interleaver(inv_perm, dist=None, device="cpu"):
    """Raise if the ranks of the process group do not all hold this inv_perm
    (one all-reduce of [d, -d] with MAX: equal iff max d == min d)."""
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return
    import torch
    d = interleaver_digest(inv_perm)
    t = torch.tensor([d, -d], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if int(t[0]) != -int(t[1]):
        raise RuntimeError("ranks hold different inverse interleavers (np.argsort tie order differs between "
                           "hosts): pin inv_perm ('stable', 'numpy-avx512' or an explicit array)")


def shard_range(total, world, rank):
    """Contiguous [start, start+count) of `total` codewords owned by `rank`;
    the first total % world ranks get one extra."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(int(total), world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def shard_seed(base_seed, rank, point=0):
    """Reproducible per-(shard, sweep point) seed: base + 1_000_003*rank + 7919*point."""
    return int(base_seed) + SEED_STRIDE * int(rank) + 7919 * int(point)


def point_seed(base_seed, point=0):
    """Generator key of a sweep point.  With the counter-based generator the
    codeword's global index is the counter, so the key needs no rank term:
    every rank of every world size sees the same stream for codeword g."""
    return int(base_seed) + 7919 * int(point)


def batches(count, batch):
    """Split a shard of `count` codewords into launches of at most `batch`."""
    out, done = [], 0
    while done < count:
        n = min(batch, count - done)
        out.append((done, n))
        done += n
    return out


def reduce_counters(counters, dist=None):
    """Sum int64 counters over all ranks (in place) when a process group is up
    (one rank included: bench.py --dist-always runs the collective through RCCL)."""
    if dist is not None and dist.is_available() and dist.is_initialized():
        dist.all_reduce(counters, op=dist.ReduceOp.SUM)
    return counters


def reduce_max(value_tensor, dist=None):
    if dist is not None and dist.is_available() and dist.is_initialized():
        dist.all_reduce(value_tensor, op=dist.ReduceOp.MAX)
    return value_tensor
