"""The multi-GPU path (codeword shards, counter all-reduce) on CPU with gloo,
world_size 2: two ranks each decode their shard (oracle as the compute, this
test exercises the partition / seeding / reduction logic) and the reduced
counters and the concatenated bits equal a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from modulations_amd import sharding as S
from modulations_amd import tables as T
from oracle import oracle as O

N, RATE, TOTAL, BASE = 48, "1/3", 37, 4242


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_work(rank, world):
    """Generate + decode this rank's shard; returns (counters, bits)."""
    start, count = S.shard_range(TOTAL, world, rank)
    t, G = O.trellis()
    punct = T.PUNCTURE_PATTERNS[RATE]
    pm = T.puncture_matrix(punct)
    perm = T.interleaver(N)
    inv = T.inverse_interleaver(perm)
    bits_all, errs = [], [0, 0, 0]
    for cw in range(start, start + count):
        rng = np.random.default_rng(S.shard_seed(BASE, 0) + cw)    # per-codeword stream: placement independent
        info = rng.integers(0, 2, 2 * N)
        coded = O.encode(info, N, 1, pm, perm, t, G)
        llr = ((1 - 2.0 * coded) * 1.5 + rng.standard_normal(coded.shape) * 1.2).astype(np.float32)
        b = O.decode(llr, N, 1, pm, 8, perm, inv, t)
        e = int((b != info).sum())
        errs[0] += e
        errs[1] += int(e > 0)
        errs[2] += 1
        bits_all.append(b)
    return torch.tensor(errs, dtype=torch.int64), np.array(bits_all).reshape(count, 2 * N)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cnt, bits = _shard_work(rank, world)
    S.reduce_counters(cnt, dist)
    tmax = S.reduce_max(torch.tensor([float(rank + 1)], dtype=torch.float64), dist)
    q.put((rank, cnt.tolist(), bits, float(tmax)))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for total in (0, 1, 7, 64, 1000):
        for world in (1, 2, 3, 8):
            spans = [S.shard_range(total, world, r) for r in range(world)]
            covered = [i for s, c in spans for i in range(s, s + c)]
            assert covered == list(range(total))
    assert S.batches(10, 4) == [(0, 4), (4, 4), (8, 2)]


def test_two_rank_gloo_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single_cnt, single_bits = _shard_work(0, 1)
    for rank, cnt, _, tmax in res:
        assert cnt == single_cnt.tolist()          # all-reduced counters agree on every rank
        assert tmax == 2.0
    bits = np.concatenate([r[2] for r in res])
    assert np.array_equal(bits, single_bits)


def _inv_worker(rank, world, port, q, differ):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inv = np.argsort(np.arange(48)[::-1], kind="stable").astype(np.int32)
    if differ and rank == 1:
        inv = inv.copy()
        inv[[0, 1]] = inv[[1, 0]]        # another tie order on this "host"
    try:
        S.check_same_interleaver(inv, dist)
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, "mismatch" if "different inverse interleavers" in str(e) else repr(e)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("differ", [False, True])
def test_ranks_must_share_the_inverse_interleaver(differ):
    """the reference's default inv_perm depends on the host's numpy,
    so a multi-host job checks that every rank holds the same one (bench.py and
    ber.py call this before decoding; ber.py also keys its resume file on it)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_inv_worker, args=(r, 2, port, q, differ)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == (["mismatch"] * 2 if differ else ["ok"] * 2)
    assert S.interleaver_digest([1, 0, 2]) != S.interleaver_digest([0, 1, 2])
