"""Drop-in replacement for the reference module ``dvb_rcs2_turbo``
(poriya219/modulations, dvb_rcs2_turbo.py), decode side on MI355X.

Same names, argument meaning, dtypes and error behaviour as the reference:

* ``DVBRCS2_Turbo(N_couples, code_rate, iterations=8)``   -- :287-537
  ``.decode(llr) -> int32[2N]``, ``.encode(bits) -> int32[n_coded]`` and the
  attributes ``N, k_info, n_coded, iterations, punct, perm, inv_perm,
  next_state, out_W, out_Y, prev_state, prev_input, G_matrix``.
* ``bcjr_max_log_map(Lc_A, Lc_B, Lc_W, Lc_Y, La_A, La_B, next_st, out_W, out_Y,
  prev_st, prev_inp, N, scaling_factor) -> (Le_A, Le_B)``   -- :116-281
* ``max_star``, ``mat_mul_gf2``, ``mat_pow_gf2``, ``solve_circular_state_gf2``,
  ``INTERLEAVER_PARAMS``, ``PUNCTURE_PATTERNS``             -- :9-114
* the north-star names ``bcjr_decode_circular`` (= bcjr_max_log_map) and
  ``turbo_decode(llr, N_couples, code_rate, iterations=8)``.

Additions: ``decode_batch`` (B codewords in one launch), ``decode_device``
(torch tensors already on the GPU, stream-ordered), ``algo='log-map'``,
``inv_perm=`` / ``interleaver=`` to pin the de-interleaver.

Every decode / SISO runs in the HIP library (modulations_amd/lib/libtdec.so);
there is no host fallback.  ``encode`` is host-side numpy (it is not on the hot
path; the batched device encoder is ``encode_device``).
"""
from __future__ import annotations

import ctypes as C
import sys
import threading

import numpy as np

from . import _native as _n
from . import tables as _t
from .tables import (INTERLEAVER_PARAMS, PUNCTURE_PATTERNS, mat_mul_gf2, mat_pow_gf2, max_star,  # noqa: F401
                     solve_circular_state_gf2)

ALGOS = {"max-log": 0, "maxlog": 0, "max-log-map": 0, "log-map": 1, "logmap": 1}

_TABLES = None


def _std_tables():
    global _TABLES
    if _TABLES is None:
        _TABLES = _t.trellis_tables()
    return _TABLES


class _Handle:
    """Owns one tdec_t (device-side codec state).

    A tdec_t's staging buffers, workspace and private streams are shared by
    every call on it, and ctypes releases the GIL during a call, so calls on
    one handle are serialised by ``lock`` (``call``): the module-level caches
    hand the same handle to every Python thread, as the reference functions
    may be called from several threads at once."""

    def __init__(self, device, n, punct, iterations, algo, perm, inv_perm, tables):
        pm = np.ascontiguousarray(_t.puncture_matrix(punct))
        self._keep = (pm, np.ascontiguousarray(perm, np.int32), np.ascontiguousarray(inv_perm, np.int32),
                      np.ascontiguousarray(tables, np.int32))
        h = C.c_void_p()
        _n.check(_n.lib().tdec_create(device, n, punct["period"], _n.ptr(pm), iterations, algo,
                                      _n.ptr(self._keep[1]), _n.ptr(self._keep[2]), _n.ptr(self._keep[3]),
                                      C.byref(h)))
        self.h = h
        self.device = device
        self.llr_len = _n.lib().tdec_llr_len(h)
        self.enc_len = _n.lib().tdec_encoded_len(h)
        self.lock = threading.Lock()
        L = _n.lib()
        self.siso_staged = getattr(L, "tdec_siso_staged", None)
        self.n = n
        self._views = None

    def siso_views(self):
        """(float32-Lc views, float64-Lc views) of the handle's single-row SISO
        staging: 8 numpy arrays of N each (LcA, LcB, LcW, LcY, LaA, LaB, LeA, LeB)
        over the page-locked buffer of tdec_siso_staging (include/tdec.h)."""
        v = self._views
        if v is None:
            buf, sl = C.c_void_p(), C.c_size_t()
            self.call("tdec_siso_staging", 1, C.byref(buf), C.byref(sl))
            sl, n = sl.value, self.n
            raw = np.frombuffer((C.c_char * (8 * sl)).from_address(buf.value), np.uint8)
            f64 = [raw[i * sl:i * sl + 8 * n].view(np.float64) for i in range(8)]
            f32 = [raw[i * sl:i * sl + 4 * n].view(np.float32) for i in range(4)] + f64[4:]
            v = self._views = (f32, f64)
        return v

    def call(self, name, *args):
        """lib().<name>(self.h, *args) under the handle lock, errors raised."""
        with self.lock:
            return _n.check(getattr(_n.lib(), name)(self.h, *args))

    def __del__(self, _finalizing=sys.is_finalizing):
        # at interpreter exit the process releases the device anyway, and the
        # module globals this would need may already be gone
        h = getattr(self, "h", None)
        if h is None or not h.value or _finalizing():
            return
        lib = getattr(_n, "_lib", None) if _n is not None else None
        if lib is not None:
            lib.tdec_destroy(h)
        self.h = None


def _default_device():
    """torch's current device when torch has initialised its GPU state, else 0.
    Cheap enough for every call (no import, no device query before that): the
    per-call functions resolve it each time."""
    t = sys.modules.get("torch")
    try:
        if t is not None and t.cuda.is_initialized():
            return t.cuda.current_device()
    except Exception:  # pragma: no cover - a torch without a usable cuda module
        pass
    return 0


class DVBRCS2_Turbo:
    """DVB-RCS2 duo-binary turbo codec (reference :287-537), decode on MI355X.

    Extra keyword arguments (all optional, defaults reproduce the reference):
      algo       'max-log' (reference) or 'log-map' (build-defined max* with correction)
      inv_perm   'numpy' (default: the reference's own np.argsort(perm) (:325),
                 evaluated by this host's numpy, so the reference run on the same
                 host gets the same de-interleaver and the same bits),
                 'stable' (np.argsort(perm, kind='stable'): host independent),
                 'numpy-avx512' (the survey host's result, pinned), or an int array
      interleaver 'reference' (default; the reference's non-bijective perm) or
                 'valid-perm' (a true permutation: never used for parity)
      device     HIP device ordinal
    """

    def __init__(self, N_couples, code_rate, iterations=8, *, algo="max-log", inv_perm="numpy",
                 interleaver="reference", device=None):
        self.N = N_couples
        self.k_info = N_couples * 2
        self.iterations = iterations
        self.punct = PUNCTURE_PATTERNS[code_rate]          # KeyError for an unknown rate, as :292
        if self.N not in INTERLEAVER_PARAMS:
            raise ValueError(f"Block size {self.N} not in standard tables.")
        self.rate = code_rate
        self.algo = ALGOS[algo] if isinstance(algo, str) else int(algo)
        if interleaver == "reference":
            self.perm = _t.interleaver(self.N)
        elif interleaver == "valid-perm":
            self.perm = _t.valid_interleaver(self.N)
        else:
            raise ValueError(f"unknown interleaver {interleaver!r}")
        if isinstance(inv_perm, str):
            self.inv_perm = (_t.inverse_interleaver(self.perm, inv_perm) if interleaver == "reference"
                             else np.argsort(self.perm).astype(np.int32))
        else:
            self.inv_perm = np.ascontiguousarray(inv_perm, np.int32)
        (self.next_state, self.out_W, self.out_Y, self.prev_state, self.prev_input,
         self.G_matrix) = _std_tables()
        self.n_coded = _t.coded_size(self.N, self.punct)
        self.device = _default_device() if device is None else device
        self._h = None
        self._circ = None

    # -- device handle (created lazily so a codec can be built without a GPU) --
    @property
    def handle(self):
        if self._h is None:
            tabs = _t.packed_tables(self.next_state, self.out_W, self.out_Y, self.prev_state, self.prev_input)
            self._h = _Handle(self.device, self.N, self.punct, self.iterations, self.algo, self.perm,
                              self.inv_perm, tabs)
        return self._h

    # -- encode (host; :404-462) -----------------------------------------------------
    def encode(self, bits):
        """Encode bits into a DVB-RCS2 turbo codeword (reference :431-462), by the
        library's compiled host encoder (tdec_encode_host: no GPU needed)."""
        bits = np.array(bits, dtype=np.int32)
        if bits.ndim != 1 or bits.shape[0] < 2 * self.N:
            raise IndexError(f"index {bits.shape[0] if bits.ndim else 0} is out of bounds for axis 0 "
                             f"with size {bits.shape[0] if bits.ndim else 0}")
        return self.encode_batch(bits[None, :2 * self.N])[0]

    def encode_batch(self, bits):
        """encode() of B rows at once: int [B, 2N] -> int32 [B, n_out]."""
        bits = np.ascontiguousarray(np.asarray(bits, dtype=np.int32))
        if bits.ndim != 2 or bits.shape[1] < 2 * self.N:
            raise ValueError("encode_batch takes a [B, 2N] array")
        B = bits.shape[0]
        out = np.zeros((B, self._enc_len()), np.int32)
        pm = np.ascontiguousarray(_t.puncture_matrix(self.punct))
        perm = np.ascontiguousarray(self.perm, np.int32)
        rc = _n.lib().tdec_encode_host(self.N, self.punct["period"], _n.ptr(pm), _n.ptr(perm), B, _n.ptr(bits),
                                       bits.shape[1], _n.ptr(out), out.shape[1])
        if rc < 0:
            _n.check(int(rc))
        return out

    def _enc_len(self):
        p = self.punct
        return sum(2 + p["W1"][i % p["period"]] + p["Y1"][i % p["period"]] + p["W2"][i % p["period"]]
                   + p["Y2"][i % p["period"]] for i in range(self.N))

    # -- decode (:464-537) -----------------------------------------------------------
    def decode(self, llr):
        """Decode one codeword's LLRs (LLR = log P(0)/P(1)) into int32[2N] info bits."""
        llr = np.array(llr, dtype=np.float32)
        if llr.ndim != 1:
            raise ValueError("decode() takes one codeword; use decode_batch for [B, n] input")
        return self.decode_batch(llr[None, :])[0]

    def decode_batch(self, llr, return_lfinal=False, out=None):
        """Decode B codewords: llr [B, >= n_llr] -> int32 [B, 2N]
        (and L_final f64 [B, 2N] = Lc + La + Le1, :529-530, when asked).
        out: optional C-contiguous int32 [B, 2N] array for the bits (e.g. a
        host_buffer(), which the copies reach without runtime staging)."""
        llr = np.ascontiguousarray(np.asarray(llr, dtype=np.float32))
        if llr.ndim != 2:
            raise ValueError("decode_batch takes a [B, n] array")
        h = self.handle
        if llr.shape[1] < h.llr_len:
            raise IndexError(f"index {llr.shape[1]} is out of bounds for axis 0 with size {llr.shape[1]}")
        B = llr.shape[0]
        if out is not None:
            if out.dtype != np.int32 or out.shape != (B, self.k_info) or not out.flags.c_contiguous:
                raise ValueError("out must be a C-contiguous int32 [B, 2N] array")
            bits = out
        else:
            bits = np.zeros((B, self.k_info), np.int32)
        lf = np.zeros((B, self.k_info)) if return_lfinal else None
        if B:
            h.call("tdec_decode_batch", B, _n.ptr(llr), llr.shape[1], _n.ptr(bits), _n.ptr(lf))
        return (bits, lf) if return_lfinal else bits

    @staticmethod
    def host_buffer(shape, dtype=np.float32):
        """An uninitialised page-locked numpy array (tdec_host_alloc): LLR rows or
        bit rows in such buffers move over PCIe without the runtime's staging
        copy.  Freed when the array is garbage-collected."""
        return pinned_empty(shape, dtype)

    # -- device-resident API (torch tensors on this codec's GPU) -------------------------
    def reserve(self, max_batch):
        self.handle.call("tdec_reserve", int(max_batch))

    def planes_bytes(self, B):
        return _n.lib().tdec_planes_bytes(self.handle.h, int(B))

    # -- argument checks of the device wrappers: a wrong dtype, stride, shape or
    #    device would otherwise mean silently wrong data or out-of-bounds writes
    def _dev_check(self, t, name, dtype, shape=None, rows_contig=False):
        import torch
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda" or t.device.index != self.device:
            raise ValueError(f"{name} must be a tensor on cuda:{self.device}")
        if t.dtype != dtype:
            raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
        if rows_contig:
            if t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1) or (t.shape[0] > 1 and t.stride(0) < t.shape[1]):
                raise ValueError(f"{name} rows must be contiguous (stride(1) == 1)")
        elif not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")

    def _stream(self, stream):
        """The caller's stream, or torch's current stream on this codec's device."""
        if stream is not None:
            return _n.stream_ptr(stream)
        import torch
        return torch.cuda.current_stream(self.device).cuda_stream

    def decode_device(self, llr, bits=None, lfinal=None, stream=None):
        """llr: float32 [B, n] device tensor (rows contiguous) -> int32 [B, 2N] device tensor.
        Stream-ordered on `stream` (default: torch's current stream)."""
        import torch
        self._dev_check(llr, "llr", torch.float32, rows_contig=True)
        B = llr.shape[0]
        if B and llr.shape[1] < self.handle.llr_len:
            raise IndexError(f"index {llr.shape[1]} is out of bounds for axis 0 with size {llr.shape[1]}")
        self.reserve(B)
        if bits is None:
            bits = torch.empty((B, self.k_info), dtype=torch.int32, device=llr.device)
        self._dev_check(bits, "bits", torch.int32, (B, self.k_info))
        if lfinal is not None:
            self._dev_check(lfinal, "lfinal", torch.float64, (B, self.k_info))
        self.handle.call("tdec_decode_batch_dev", B, _n.ptr(llr), llr.stride(0) if B > 1 else llr.shape[1],
                         _n.ptr(bits), _n.ptr(lfinal), self._stream(stream))
        return bits

    def decode_planes_device(self, planes, B, bits, lfinal=None, stream=None):
        import torch
        if planes.numel() * planes.element_size() < self.planes_bytes(B):
            raise ValueError("planes buffer smaller than planes_bytes(B)")
        self._dev_check(planes, "planes", torch.float32)
        self._dev_check(bits, "bits", torch.int32, (B, self.k_info))
        if lfinal is not None:
            self._dev_check(lfinal, "lfinal", torch.float64, (B, self.k_info))
        self.handle.call("tdec_decode_planes_dev", B, _n.ptr(planes), _n.ptr(bits), _n.ptr(lfinal),
                         self._stream(stream))
        return bits

    def depuncture_device(self, llr, planes, stream=None):
        import torch
        self._dev_check(llr, "llr", torch.float32, rows_contig=True)
        self._dev_check(planes, "planes", torch.float32)
        if planes.numel() * 4 < self.planes_bytes(llr.shape[0]):
            raise ValueError("planes buffer smaller than planes_bytes(B)")
        self.handle.call("tdec_depuncture_dev", llr.shape[0], _n.ptr(llr),
                         llr.stride(0) if llr.shape[0] > 1 else llr.shape[1], _n.ptr(planes), self._stream(stream))
        return planes

    def tail_gate(self, stream=None):
        """Hold work queued after this on `stream` until this codec's latest
        throughput decode has handed out its last tiles (tdec_tail_gate)."""
        self.handle.call("tdec_tail_gate", self._stream(stream))

    def demap_planes_device(self, syms, constellation, bps, noise_var, planes, div_f32=False, stream=None):
        """Fused soft demap (decoder sign) + de-puncture of complex64 symbols [B, S]."""
        cons = np.ascontiguousarray(np.asarray(constellation))
        f64 = cons.dtype == np.complex128
        cons = cons.astype(np.complex128 if f64 else np.complex64)
        import torch
        self._dev_check(syms, "syms", torch.complex64)
        self._dev_check(planes, "planes", torch.float32)
        B, S = syms.shape[0], syms.shape[1]
        if planes.numel() * 4 < self.planes_bytes(B):
            raise ValueError("planes buffer smaller than planes_bytes(B)")
        self.handle.call("tdec_demap_planes_dev", B, _n.ptr(syms), S, _n.ptr(cons), int(f64), len(cons), bps,
                         float(noise_var), int(div_f32), _n.ptr(planes), self._stream(stream))
        return planes

    # -- fused demap + decode (one launch; tdec_demap_decode_dev) -------------------------
    def fused_available(self, constellation, bps):
        cons = np.asarray(constellation)
        return bool(_n.lib().tdec_fused_available(self.handle.h, int(cons.dtype == np.complex128), int(bps)))

    def reserve_fused(self, max_batch):
        self.handle.call("tdec_reserve_fused", int(max_batch))

    def demap_decode_device(self, syms, constellation, bps, noise_var, bits, lfinal=None, div_f32=False,
                            stream=None):
        """compute_llr (decoder sign) -> f32 -> decode of complex64 symbols [B, S] in one
        launch: the bits of demap_planes_device + decode_planes_device."""
        import torch
        cons = np.ascontiguousarray(np.asarray(constellation))
        f64 = cons.dtype == np.complex128
        cons = cons.astype(np.complex128 if f64 else np.complex64)
        self._dev_check(syms, "syms", torch.complex64)
        B, S = syms.shape[0], syms.shape[1]
        self._dev_check(bits, "bits", torch.int32, (B, self.k_info))
        if lfinal is not None:
            self._dev_check(lfinal, "lfinal", torch.float64, (B, self.k_info))
        self.handle.call("tdec_demap_decode_dev", B, _n.ptr(syms), S, _n.ptr(cons), int(f64), len(cons), bps,
                         float(noise_var), int(div_f32), _n.ptr(bits), _n.ptr(lfinal), self._stream(stream))
        return bits

    def encode_device(self, bits_u8, coded_u8=None, stream=None):
        """Batched device encoder: uint8 [B, 2N] -> uint8 [B, n_out] (same bits as encode())."""
        import torch
        self._dev_check(bits_u8, "bits", torch.uint8, (bits_u8.shape[0], self.k_info))
        B = bits_u8.shape[0]
        if coded_u8 is None:
            coded_u8 = torch.empty((B, self.handle.enc_len), dtype=torch.uint8, device=bits_u8.device)
        self._dev_check(coded_u8, "coded", torch.uint8, (B, self.handle.enc_len))
        self.handle.call("tdec_encode_dev", B, _n.ptr(bits_u8), _n.ptr(coded_u8), self._stream(stream))
        return coded_u8


class DVB_RCS2_TurboCodec(DVBRCS2_Turbo):
    """The codec name the reference's harnesses import (turbo_test_suite.py:10,
    test_sdr_with_coding.py:11; it no longer exists in the reference module):
    ``DVB_RCS2_TurboCodec(block_length=, code_rate=, n_iterations=)`` with
    ``block_length`` in couples and ``code_rate`` exposed as the float
    k_info / n_coded that turbo_test_suite.py:133 and :221 use for the noise
    variance.  Same decoder underneath."""

    def __init__(self, block_length=212, code_rate='1/2', n_iterations=8, **kw):
        super().__init__(block_length, code_rate, n_iterations, **kw)
        self.block_length = block_length
        self.n_iterations = n_iterations
        self.code_rate = self.k_info / self.n_coded


def pinned_empty(shape, dtype=np.float32):
    """Page-locked host numpy array from tdec_host_alloc, freed with its buffer."""
    import weakref
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    if n == 0:
        return np.empty(shape, dtype)
    p = C.c_void_p()
    _n.check(_n.lib().tdec_host_alloc(n, C.byref(p)))
    buf = (C.c_char * n).from_address(p.value)
    weakref.finalize(buf, _n.lib().tdec_host_free, p.value)
    return np.frombuffer(buf, dtype=dtype).reshape(shape)


# ---- module-level functions of the reference ------------------------------------------

_SISO_CACHE = {}
_CACHE_LOCK = threading.Lock()
_F32 = np.dtype(np.float32)
_F64 = np.dtype(np.float64)


def _tables_key(tabs):
    """Bytes identifying the five trellis tables (the handle cache key).  The
    usual call passes the codec's own int32 [16, 4] arrays: their bytes directly;
    anything else goes through packed_tables' conversion."""
    if all(type(t) is np.ndarray and t.dtype == np.int32 and t.size == 64 and t.flags.c_contiguous for t in tabs):
        return b"".join([t.tobytes() for t in tabs])
    return _t.packed_tables(*tabs).tobytes()


def _siso_handle(N, tkey, algo, dev):
    key = (N, tkey, algo, dev)
    h = _SISO_CACHE.get(key)
    if h is None:
        with _CACHE_LOCK:
            h = _SISO_CACHE.get(key)
            if h is None:
                ident = np.arange(N, dtype=np.int32)
                tabs = np.frombuffer(tkey, np.int32).reshape(5, 16, 4)
                h = _SISO_CACHE[key] = _Handle(dev, N, PUNCTURE_PATTERNS['1/3'], 1, algo, ident, ident, tabs)
    return h


def _short(n, N):
    return IndexError(f"index {n} is out of bounds for axis 0 with size {n}")


def _siso_inputs(Lc, La, N, ndim):
    """The SISO's inputs with numba's typing of bcjr_max_log_map (:116-160, :267):
      * channel LLRs: four float32 arrays run the float32 specialisation (each use
        widens them to f64: f64(Lc_A) + La_A, f64(par_W) * 0.5); float64 arrays
        -- or a mix, or integer / bool arrays, which numba also widens to f64 --
        run the float64 one, where those sums are formed from the unrounded
        values.  Widening is exact, so a float32 array in a mixed call gives the
        values numba uses.
      * a-priori: float64, or integer / bool arrays, which numba widens to f64
        exactly as integer channel LLRs (int64 + f64 -> f64): they are widened
        here.  With float32 (or float16) La the reference sums in_A = Lc_A + La_A
        in float32 and builds the branch metrics from a float32 m, which the shim
        that pins every fixture cannot reproduce (numpy 2 keeps 0.0 + f32 in
        float32 where numba promotes to f64), so that call is refused, not guessed.
    Returns (f64, [A, B, W, Y], [LaA, LaB]): the caller's arrays (not copied;
    integer a-priori arrays widened to float64), each checked to be ndim-D with at
    least N entries along its last axis."""
    lc = [x if type(x) is np.ndarray else np.asarray(x) for x in Lc]
    la = [x if type(x) is np.ndarray else np.asarray(x) for x in La]
    for i, x in enumerate(la):
        if x.dtype is _F64 or x.dtype == _F64:
            continue
        if x.dtype.kind in "iub" and x.dtype.itemsize <= 8:
            la[i] = x.astype(np.float64)   # exact for |v| < 2^53, as numba's int64 -> f64
            continue
        raise TypeError(f"bcjr_max_log_map: a-priori LLRs must be float64 or integer (got {x.dtype}); the "
                        "reference's float32 a-priori arithmetic is not reproducible here (parity unpinned)")
    f64 = False
    for x in lc:
        if x.dtype is not _F32 and x.dtype != _F32:
            if x.dtype.kind not in "fiub" or x.dtype.itemsize > 8 or x.dtype == np.float16:
                raise TypeError(f"bcjr_max_log_map: channel LLRs must be float32 or float64 arrays (got {x.dtype})")
            f64 = True
    for x in lc + la:
        if x.ndim != ndim:
            raise ValueError(f"bcjr_max_log_map{'_batch' if ndim == 2 else ''} takes {ndim}-D arrays")
        if x.shape[-1] < N:
            raise _short(x.shape[-1], N)
    return f64, lc, la


def bcjr_max_log_map(Lc_A, Lc_B, Lc_W, Lc_Y, La_A, La_B, next_st, out_W, out_Y, prev_st, prev_inp, N,
                     scaling_factor):
    """Max-Log-MAP SISO (reference :116-281), one codeword, on the GPU.

    Same arguments and outputs: channel LLRs (float32, or float64 -- numba's
    float64 specialisation, reproduced), float64 a-priori, the five int32
    [16,4] trellis tables, N couples and the extrinsic scaling factor; returns
    freshly allocated (Le_A, Le_B) f64 arrays.  Inputs are not mutated.

    Per call: the inputs are copied into the handle's page-locked staging
    (tdec_siso_staging) and one argument-free C call runs the SISO there.
    """
    N = int(N)
    f64, lc, la = _siso_inputs((Lc_A, Lc_B, Lc_W, Lc_Y), (La_A, La_B), N, 1)
    if N == 0:   # the reference's recursions run over range(0): empty extrinsics
        return np.zeros(0), np.zeros(0)
    h = _siso_handle(N, _tables_key((next_st, out_W, out_Y, prev_st, prev_inp)), 0, _default_device())
    if h.siso_staged is None:   # a library without the staged entry points (older A/B builds)
        LeA, LeB = bcjr_max_log_map_batch(*(x[None, :N] for x in lc + la), next_st, out_W, out_Y, prev_st, prev_inp,
                                          N, scaling_factor)
        return LeA[0], LeB[0]
    v = h.siso_views()[f64]
    with h.lock:
        for d, x in zip(v, lc + la):
            np.copyto(d, x if x.shape[0] == N else x[:N])
        rc = h.siso_staged(h.h, 1, f64, float(scaling_factor))
        if rc:
            _n.check(rc)
        return v[6].copy(), v[7].copy()


bcjr_decode_circular = bcjr_max_log_map   # historic name of the same SISO


def siso_flag_fallbacks():
    """Staged bcjr_max_log_map calls, over every cached SISO handle, that ended by
    a stream wait instead of their rows' completion flags (tdec_siso_stats; 0 when
    the flag path works)."""
    n = 0
    L = _n.lib()
    for h in list(_SISO_CACHE.values()):
        v = C.c_long(0)
        _n.check(L.tdec_siso_stats(h.h, C.byref(v)))
        n += v.value
    return n


def bcjr_max_log_map_batch(Lc_A, Lc_B, Lc_W, Lc_Y, La_A, La_B, next_st, out_W, out_Y, prev_st, prev_inp, N,
                           scaling_factor, algo="max-log", device=None):
    """bcjr_max_log_map over B codewords at once: [B, N] arrays in, (Le_A, Le_B) [B, N] out
    (channel LLRs float32 or float64 as in bcjr_max_log_map)."""
    N = int(N)
    f64, lc, la = _siso_inputs((Lc_A, Lc_B, Lc_W, Lc_Y), (La_A, La_B), N, 2)
    dt = _F64 if f64 else _F32
    A, Bv, W, Y = (np.ascontiguousarray(x[:, :N], dt) for x in lc)
    la, lb = (np.ascontiguousarray(x[:, :N], _F64) for x in la)
    if any(x.shape[0] != A.shape[0] for x in (A, Bv, W, Y, la, lb)):
        raise ValueError("bcjr_max_log_map_batch takes [B, N] arrays of one batch size")
    if N == 0:
        return np.zeros((A.shape[0], 0)), np.zeros((A.shape[0], 0))
    algo = ALGOS[algo] if isinstance(algo, str) else int(algo)
    h = _siso_handle(N, _tables_key((next_st, out_W, out_Y, prev_st, prev_inp)), algo,
                     _default_device() if device is None else device)
    B = A.shape[0]
    LeA = np.zeros((B, N))
    LeB = np.zeros((B, N))
    h.call("tdec_siso_batch_f64" if f64 else "tdec_siso_batch", B, A.ctypes.data, Bv.ctypes.data, W.ctypes.data,
           Y.ctypes.data, la.ctypes.data, lb.ctypes.data, float(scaling_factor), LeA.ctypes.data, LeB.ctypes.data)
    return LeA, LeB


_CODEC_CACHE = {}


def turbo_decode(llr, N_couples, code_rate, iterations=8, **kw):
    """Historic module-level decode: DVBRCS2_Turbo(...).decode(llr)."""
    key = (N_couples, code_rate, iterations, tuple(sorted(kw.items())))
    with _CACHE_LOCK:
        c = _CODEC_CACHE.get(key)
        if c is None:
            c = _CODEC_CACHE[key] = DVBRCS2_Turbo(N_couples, code_rate, iterations, **kw)
        h = c.handle   # created under the lock: one handle per cached codec
    llr = np.asarray(llr)
    return c.decode_batch(llr) if llr.ndim == 2 else c.decode(llr)


# ---- log-MAP primitive tables (diagnostics / test infrastructure) ---------------------
# The build-defined log-MAP evaluates its max* with the gfx950
# instructions v_exp_f32 / v_log_f32 on bounded f32 grids.  These are the grids
# and the device's exact outputs on them, for checkers that restate the
# definition (the oracle's orc_set_trans takes exactly this tuple).
TRANS_E_LO, TRANS_E_HI = 0x40F00000, 0x42400000    # t in [7.5, 48]: v_exp_f32(-t)
TRANS_L_LO, TRANS_L_HI = 0x3F000000, 0x41000000    # w in [0.5, 8]:  v_log_f32(w)


def capture_trans_tables(device=0):
    """(etab, e_lo, ltab, l_lo): v_exp_f32(-t) for every f32 t in [7.5, 48] and
    v_log_f32(w) for every f32 w in [0.5, 8], indexed by bit pattern - lo, as
    computed by `device` (tdec_selftest_trans)."""
    L = _n.lib()
    out = []
    for which, lo, hi in ((0, TRANS_E_LO, TRANS_E_HI), (1, TRANS_L_LO, TRANS_L_HI)):
        tab = np.empty(hi - lo + 1, np.float32)
        _n.check(L.tdec_selftest_trans(int(device), which, lo, tab.size, tab.ctypes.data))
        out += [tab, lo]
    return tuple(out)
