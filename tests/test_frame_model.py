"""CPU model of the frame decoder's recursion engine (csrc/tdec_frame.hip).

The kernel's correctness rests on three pieces of algebra that can be checked
without a GPU, in numpy float32 with the same operations:
  1. the time-varying lane labelling: with lane l holding state rotl^t(l)
     (beta: rotr^t(rev(l))), every state's two predecessors (successors) are
     the lane itself and lane l ^ (8 >> (t % 4)), with the pair-maxima indices
     fr_lane() computes;
  2. the segment rounds: 4 segments from zero, re-runs from the predecessor's
     end until the vector equals the stored one (checked at 4-step block
     starts), the reference's second pass as a round from the first pass's
     end vector -- the stored vectors equal the serial two-pass recursion of
     dvb_rcs2_turbo.py:162-230 bit for bit;
  3. that this holds when merging is slow or impossible (NaN, tiny inputs).
"""
import numpy as np
import pytest

NEG = np.float32(-1.0e9)


def rotl4(x, r):
    r &= 3
    return ((x << r) | (x >> (4 - r))) & 15


def rotr4(x, r):
    return rotl4(x, 4 - (r & 3))


def rev4(x):
    return ((x & 1) << 3) | ((x & 2) << 1) | ((x & 4) >> 1) | ((x & 8) >> 3)


def sb(s, i):
    return (s >> i) & 1


def t_dk(s, inp):
    return ((inp >> 1) & 1) ^ (inp & 1) ^ sb(s, 2) ^ sb(s, 3)


def t_next(s, inp):
    return (sb(s, 2) << 3) | (sb(s, 1) << 2) | (sb(s, 0) << 1) | t_dk(s, inp)


def t_ow(s, inp):
    return t_dk(s, inp) ^ sb(s, 0) ^ sb(s, 1) ^ sb(s, 3)


def t_oy(s, inp):
    return t_dk(s, inp) ^ sb(s, 1) ^ sb(s, 2) ^ sb(s, 3)


def pair_ix(p, ns):
    for inp in range(4):
        if t_next(p, inp) == ns:
            return ((((inp >> 1) ^ inp) & 1) << 2) | (t_ow(p, inp) << 1) | t_oy(p, inp)
    raise AssertionError("not a successor")


def serial_pass(pm, start, beta):
    """One pass of the reference's recursion with pair maxima, natural state
    order; returns the stored vectors (entering each step) and the end vector."""
    N = pm.shape[0]
    v = start.copy()
    out = np.zeros((N, 16), np.float32)
    for u in range(N):
        k = N - 1 - u if beta else u
        out[u] = v
        nv = np.empty(16, np.float32)
        for s in range(16):
            if not beta:   # alpha: predecessors of s
                p0 = rotr4(s, 1)
                c = [v[p0] + pm[k, pair_ix(p0, s)], v[p0 ^ 8] + pm[k, pair_ix(p0 ^ 8, s)]]
            else:          # beta: successors of s
                n0 = rotl4(s, 1)
                c = [v[n0] + pm[k, pair_ix(s, n0)], v[n0 ^ 1] + pm[k, pair_ix(s, n0 ^ 1)]]
            nv[s] = np.fmax(np.fmax(NEG, np.float32(c[0])), np.float32(c[1]))
        v = (nv - nv[0]).astype(np.float32)
    return out, v


def lane_consts(beta):
    lbl = np.zeros((4, 16), int)
    idx = np.zeros((4, 16, 2), int)
    for ph in range(4):
        for l in range(16):
            if not beta:
                i, ns = rotl4(l, ph), rotl4(l, ph + 1)
                a, b = pair_ix(i, ns), pair_ix(i ^ 8, ns)
            else:
                i, s = rotr4(rev4(l), ph), rotr4(rev4(l), ph + 1)
                a, b = pair_ix(s, i), pair_ix(s, i ^ 1)
            lbl[ph, l], idx[ph, l] = i, (a, b)
    return lbl, idx


def lane_step(v, pm_row, ph, idx):
    lanes = np.arange(16)
    o = v[lanes ^ (8 >> ph)]
    n = np.fmax(np.fmax(NEG, (v + pm_row[idx[ph, :, 0]]).astype(np.float32)),
                (o + pm_row[idx[ph, :, 1]]).astype(np.float32))
    return (n - n[0]).astype(np.float32)


def frame_recursion(pm, beta, P=4, lmin=0, blk=8):
    """The kernel's engine: stored vectors [N][16] in step order (natural state
    order), after both passes, plus round statistics.  P segments per direction
    (4: one wave, TDEC_FR_WPD 1; 8: two waves, TDEC_FR_WPD 2; 16: four waves);
    a re-run compares with the stored vector at every blk-step block start
    (8: TDEC_FR_BLK8, the default; 4: its 4-step blocks)."""
    N = pm.shape[0]
    lbl, idx = lane_consts(beta)
    n = P if lmin == 0 else min(P, max(1, N // lmin))   # tdec_frame.hip fr_seg_len (TDEC_FR_LMIN)
    Ls = (N + 4 * n - 1) // (4 * n) * 4
    nseg = (N + Ls - 1) // Ls
    seg = [(g * Ls, max(0, min(Ls, N - g * Ls))) for g in range(P)]
    st = np.full((N, 16), np.nan, np.float32)
    ev = np.zeros((P, 16), np.float32)
    stats = {"rounds": 0}

    def run(g, start_nat, cmp):
        u0, ln = seg[g]
        v = start_nat[lbl[0]].astype(np.float32)          # lane l holds state lbl[0][l]
        for u in range(ln):
            ph = u % 4
            if cmp and u % blk == 0 and np.all(v == st[u0 + u][lbl[0]]):
                return False                               # merged
            st[u0 + u][lbl[ph]] = v
            k = N - 1 - (u0 + u) if beta else u0 + u
            v = lane_step(v, pm[k], ph, idx)
        ev[g][lbl[ln % 4]] = v
        return True

    src_of = lambda g: nseg - 1 if g == 0 else g - 1     # noqa: E731

    def one_round(dirty):
        stats["rounds"] += 1
        starts = {g: ev[src_of(g)].copy() for g in dirty}   # read before any group writes its end
        return [g for g in dirty if run(g, starts[g], True)]

    reached = [g for g in range(nseg) if run(g, np.zeros(16, np.float32), False)]
    dirty = [g + 1 for g in reached if g + 1 < nseg]
    spec = broken = False
    if dirty:
        # first re-run round + the second pass started speculatively on group 0
        reached = one_round([0] + dirty)
        r1 = [g for g in reached if g != 0]
        spec = (nseg - 1) not in r1
        dirty = [g + 1 for g in r1 if g + 1 < nseg]
        if not dirty and spec:
            dirty = [1] if 0 in reached and nseg > 1 else []
        else:
            spec = False
            # group 0 ran to its end: ev[0] and segment 0 now hold the speculative
            # trajectory, segment 1 still the pass-1 one -- the chain is broken at 0
            broken = 0 in reached and nseg > 1
        while not spec and dirty:
            reached = one_round(dirty)
            dirty = [g + 1 for g in reached if g + 1 < nseg]
    if not spec:
        reached = one_round([0])
        dirty = [1] if (0 in reached or broken) and nseg > 1 else []
    while dirty:
        reached = one_round(dirty)
        dirty = [g + 1 for g in reached if g + 1 < nseg]
    stats["spec"], stats["broken"] = spec, broken
    return st, stats


def reference_two_pass(pm, beta):
    s1, e1 = serial_pass(pm, np.zeros(16, np.float32), beta)
    s2, _ = serial_pass(pm, e1, beta)
    return s2


def _pm(rng, N, scale):
    g = (rng.standard_normal((N, 8)) * scale).astype(np.float32)
    return g


def test_labelling_partner_is_the_other_predecessor():
    for beta in (False, True):
        lbl, idx = lane_consts(beta)
        for ph in range(4):
            for l in range(16):
                p = l ^ (8 >> ph)
                if not beta:
                    assert lbl[ph, p] == lbl[ph, l] ^ 8
                    assert rotr4(rotl4(l, ph + 1), 1) == lbl[ph, l]
                else:
                    assert lbl[ph, p] == lbl[ph, l] ^ 1
                    assert rotl4(rotr4(rev4(l), ph + 1), 1) == lbl[ph, l]
            assert lbl[ph, 0] == 0    # state 0 stays in lane 0: the normalisation reads lane 0


@pytest.mark.parametrize("beta", [False, True])
def test_lane_step_equals_serial_step(beta):
    rng = np.random.default_rng(1)
    pm = _pm(rng, 12, 3.0)
    ref, _ = serial_pass(pm, np.zeros(16, np.float32), beta)
    lbl, idx = lane_consts(beta)
    v = np.zeros(16, np.float32)
    for u in range(12):
        ph = u % 4
        np.testing.assert_array_equal(v, ref[u][lbl[ph]])
        v = lane_step(v, pm[12 - 1 - u if beta else u], ph, idx)


@pytest.mark.parametrize("beta", [False, True])
@pytest.mark.parametrize("N", [1, 2, 3, 5, 8, 13, 16, 17, 33, 48, 101, 212])
@pytest.mark.parametrize("scale", [3.0, 1e-3])
@pytest.mark.parametrize("P", [4, 8, 16])
@pytest.mark.parametrize("lmin", [0, 32, 48])
@pytest.mark.parametrize("blk", [4, 8])
def test_segment_rounds_equal_two_pass(beta, N, scale, P, lmin, blk):
    rng = np.random.default_rng(N * 3 + int(beta))
    pm = _pm(rng, N, scale)
    st, _ = frame_recursion(pm, beta, P, lmin, blk)
    np.testing.assert_array_equal(st, reference_two_pass(pm, beta))


@pytest.mark.parametrize("beta", [False, True])
def test_segment_rounds_never_merging(beta):
    """NaN branch metrics: vectors with NaN never compare equal, so every
    segment runs to its end and the rounds hand the vectors down the chain."""
    rng = np.random.default_rng(5)
    pm = _pm(rng, 60, 2.0)
    pm[7, 3] = np.nan
    pm[40, :] = np.inf
    st, stats = frame_recursion(pm, beta)
    ref = reference_two_pass(pm, beta)
    np.testing.assert_array_equal(st, ref)


def test_segment_rounds_random_sweep_covers_every_path():
    """Random block lengths and metric scales: every control path of the rounds
    (speculative second pass kept, dropped, dropped with the chain broken at
    segment 0) is taken, and every result equals the serial two passes."""
    rng = np.random.default_rng(2025)
    seen = set()
    for trial in range(120):
        N = int(rng.integers(9, 90)) if trial % 3 else int(rng.integers(300, 420))
        scale = float(10 ** rng.uniform(-3, 1))
        pm = _pm(rng, N, scale)
        if trial % 7 == 0:
            pm[rng.integers(0, N)] = np.nan
        beta = bool(trial % 2)
        st, stats = frame_recursion(pm, beta, (4, 8, 16, 8)[trial % 4], (0, 0, 48, 32, 64)[trial % 5],
                                    (8, 4)[trial % 2 if trial % 3 else 0])
        np.testing.assert_array_equal(st, reference_two_pass(pm, beta))
        seen.add((stats["spec"], stats["broken"]))
    assert {(True, False), (False, False), (False, True)} <= seen, seen
