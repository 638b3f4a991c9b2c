"""Ordering and thread safety of one codec handle (include/tdec.h conventions).

A tdec_t owns its workspace, plane buffer, constellation table and staging
buffers.  These tests queue work that shares them without any caller-side
synchronisation and check every result against the same work run alone:

* decode_device() on a side stream, then decode_batch() (the handle's private
  stream) while the first kernel may still be running;
* two decode_device() calls on two different streams back to back;
* demap_planes_device() with two different constellations on two streams;
* several Python threads calling turbo_decode() / bcjr_max_log_map() at once
  (the module caches hand every thread the same handle);
* the device wrappers reject wrong dtypes, shapes and strides.
"""
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _llrs(B, n, seed, scale=3.0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return (torch.randn((B, n), generator=g, device="cuda") * scale).contiguous()


def test_device_then_host_decode_without_sync():
    c = M.DVBRCS2_Turbo(752, "1/3")
    B = 131_072                                     # one full wave of tiles: a ~35 ms kernel
    x = _llrs(B, c.n_coded, 1)
    ref = c.decode_device(x).clone()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    y = np.random.default_rng(2).standard_normal((4096, c.n_coded)).astype(np.float32) * 3
    ref_y = c.decode_batch(y)
    with torch.cuda.stream(side):
        out = c.decode_device(x)                    # queued on `side`
    got_y = c.decode_batch(y)                       # same handle, private stream, no sync in between
    torch.cuda.synchronize()
    assert np.array_equal(got_y, ref_y)
    assert torch.equal(out, ref)


def test_two_streams_same_handle():
    c = M.DVBRCS2_Turbo(752, "1/3")
    B = 65_536
    x1, x2 = _llrs(B, c.n_coded, 3), _llrs(B, c.n_coded, 4)
    r1 = c.decode_device(x1).clone()
    r2 = c.decode_device(x2).clone()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        o1 = c.decode_device(x1)
    with torch.cuda.stream(s2):
        o2 = c.decode_device(x2)
    torch.cuda.synchronize()
    assert torch.equal(o1, r1) and torch.equal(o2, r2)


def test_demap_planes_two_tables_two_streams():
    c = M.DVBRCS2_Turbo(752, "1/3")
    B = 8192
    S16, S256 = -(-c.n_coded // 4), -(-c.n_coded // 8)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    s16 = torch.randn((B, S16), generator=g, device="cuda", dtype=torch.complex64)
    s256 = torch.randn((B, S256), generator=g, device="cuda", dtype=torch.complex64)
    c16, c256 = D.constellation("16QAM"), D.constellation("256QAM")
    c.reserve(B)
    nb = c.planes_bytes(B) // 4
    p16, p256 = (torch.empty(nb, device="cuda") for _ in range(2))
    c.demap_planes_device(s16, c16, 4, 0.1, p16)
    r16 = p16.clone()
    c.demap_planes_device(s256, c256, 8, 0.1, p256)
    r256 = p256.clone()
    torch.cuda.synchronize()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    q16, q256 = torch.zeros_like(p16), torch.zeros_like(p256)
    with torch.cuda.stream(a):
        c.demap_planes_device(s16, c16, 4, 0.1, q16)
    with torch.cuda.stream(b):
        c.demap_planes_device(s256, c256, 8, 0.1, q256)
    torch.cuda.synchronize()
    assert torch.equal(q16, r16) and torch.equal(q256, r256)


def test_threads_share_cached_handles():
    rng = np.random.default_rng(6)
    xs = [rng.standard_normal((64, 1272)).astype(np.float32) * 3 for _ in range(6)]
    ref = [M.turbo_decode(x, 212, "1/3") for x in xs]
    nx, ow, oy, ps, pi, _ = T.trellis_tables()
    siso_in = [(rng.standard_normal((4, 212)).astype(np.float32) * 3, rng.standard_normal((2, 212)) * 5)
               for _ in range(6)]
    siso_ref = [M.bcjr_max_log_map(*lc, *la, nx, ow, oy, ps, pi, 212, 0.7) for lc, la in siso_in]
    out, errs = [None] * 6, []

    def work(i):
        try:
            for _ in range(5):
                b = M.turbo_decode(xs[i], 212, "1/3")
                s = M.bcjr_max_log_map(*siso_in[i][0], *siso_in[i][1], nx, ow, oy, ps, pi, 212, 0.7)
                if not (np.array_equal(b, ref[i]) and np.array_equal(s[0], siso_ref[i][0])
                        and np.array_equal(s[1], siso_ref[i][1])):
                    errs.append(i)
            out[i] = True
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs and all(out)


def test_device_wrappers_check_arguments():
    c = M.DVBRCS2_Turbo(48, "1/3")
    x = _llrs(8, c.n_coded, 7)
    with pytest.raises(TypeError):
        c.decode_device(x.double())
    with pytest.raises(ValueError):
        c.decode_device(x, bits=torch.empty((8, 10), dtype=torch.int32, device="cuda"))
    with pytest.raises(ValueError):
        c.decode_device(_llrs(c.n_coded, 8, 8).t())          # column-major rows
    with pytest.raises(IndexError):
        c.decode_device(x[:, :-1].contiguous())
    with pytest.raises(TypeError):
        c.decode_device(x, lfinal=torch.empty((8, 96), dtype=torch.float32, device="cuda"))
    with pytest.raises(ValueError):
        c.decode_device(x, lfinal=torch.empty((8, 95), dtype=torch.float64, device="cuda"))
    # a strided row view (stride(0) > n) is accepted and decodes the same rows
    wide = _llrs(8, c.n_coded + 17, 9)
    assert torch.equal(c.decode_device(wide[:, :c.n_coded]), c.decode_device(wide[:, :c.n_coded].contiguous()))
