"""The host restatement of the counter-based workload generator
(oracle/workload_ref.py) against Random123's published Philox4x32-10
known-answer vectors, and its batching / sharding independence."""
import numpy as np

from oracle import workload_ref as W
from modulations_amd import sharding as S


def test_philox_known_answers():
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for c, k, want in kat:
        got = W.philox4x32_10(*c, *k)
        assert tuple(int(x) for x in got) == want


def test_info_bits_are_per_codeword_streams():
    seed = 0x1234_5678_9ABC
    full = W.info_bits(np.arange(100), 752, seed)
    assert full.shape == (100, 1504) and set(np.unique(full)) == {0, 1}
    # any split of the global index range (batches, or shards of a world) gives the same rows
    for world in (2, 3, 8):
        rows = []
        for r in range(world):
            start, count = S.shard_range(100, world, r)
            rows.append(W.info_bits(np.arange(start, start + count), 752, seed))
        assert np.array_equal(np.concatenate(rows), full)
    assert 0.45 < full.mean() < 0.55


def test_awgn_moments():
    n = W.awgn(np.arange(400), 1128, 7, 0.3)
    assert abs(n.real.mean()) < 0.01 and abs(n.imag.mean()) < 0.01
    assert abs(n.real.std() - 0.3) < 0.005 and abs(n.imag.std() - 0.3) < 0.005
