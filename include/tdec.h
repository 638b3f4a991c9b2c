/*
 * tdec.h -- C ABI of the MI355X (gfx950) DVB-RCS2 duo-binary turbo decoder.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * (poriya219/modulations, dvb_rcs2_turbo.py) has no FFI layer: its boundary is
 * the Python API of the module.  Each entry point below states which reference
 * interface it replaces; modulations_amd/dvb_rcs2_turbo.py binds them with
 * ctypes (INTEGRATION.md shows the binding a maintainer would add to the
 * reference module itself).
 *
 * Conventions
 *   - Plain pointers and sizes only.  Row-major, batch-major [B][...].
 *   - Entry points without a _dev suffix take HOST pointers and are
 *     synchronous.  _dev entry points take DEVICE pointers and a hipStream_t
 *     (passed as void*), are stream-ordered, never allocate and never
 *     synchronise once tdec_reserve() has sized the workspace.
 *   - B = 0 (an empty batch) is a no-op that returns 0; the buffers may then be
 *     null.  B < 0 is TDEC_EINVAL.
 *   - Return 0 on success, a negative TDEC_E* code otherwise;
 *     tdec_last_error() (thread-local) says why.  No exception crosses the ABI.
 *   - A handle is bound to one device.  Calls on different handles may run
 *     concurrently from different host threads.
 *   - LLR sign: LLR = log P(0)/P(1) (positive -> bit 0), as the decoder of the
 *     reference (dvb_rcs2_turbo.py:533-535).
 */
#ifndef TDEC_H
#define TDEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tdec_ctx tdec_t;

enum {
    TDEC_OK = 0,
    TDEC_EINVAL = -1,       /* bad argument (bad N, period, tables, null pointer) -> ValueError */
    TDEC_ESHORT = -2,       /* LLR vector shorter than the de-puncture walk     -> IndexError */
    TDEC_ENOMEM = -3,       /* device allocation failed                          -> MemoryError */
    TDEC_EHIP = -4,         /* HIP runtime error                                 -> RuntimeError */
    TDEC_EUNSUPPORTED = -5, /* trellis tables other than the DVB-RCS2 16-state CRSC */
    TDEC_EITER = -6,        /* iterations < 1 (the reference raises UnboundLocalError) */
    TDEC_ECAPACITY = -7     /* _dev call larger than tdec_reserve()                */
};

enum { TDEC_ALGO_MAXLOG = 0, TDEC_ALGO_LOGMAP = 1 };

/* Codec construction: replaces DVBRCS2_Turbo.__init__ (dvb_rcs2_turbo.py:288-309)
 * for the decode side.  punct = [4][4] uint8 (rows W1, Y1, W2, Y2; columns the
 * pattern phase, PUNCTURE_PATTERNS :21-26), period in 1..4.  perm / inv_perm =
 * int32[n_couples] (the reference's self.perm / self.inv_perm, :311-325).
 * tables = int32[5][16][4]: next_state, out_W, out_Y, prev_state, prev_input
 * (:327-396); anything but the DVB-RCS2 trellis returns TDEC_EUNSUPPORTED. */
int tdec_create(int device, int n_couples, int period, const uint8_t *punct, int iterations, int algo,
                const int32_t *perm, const int32_t *inv_perm, const int32_t *tables, tdec_t **out);
void tdec_destroy(tdec_t *h);
const char *tdec_last_error(void);

/* LLRs one decode reads (the de-puncture walk, :476-487). */
long tdec_llr_len(const tdec_t *h);

/* One SISO pass over B codewords: replaces bcjr_max_log_map
 * (dvb_rcs2_turbo.py:116-281; historic name bcjr_decode_circular).
 * All arrays [B][n_couples], host memory.  Outputs f64 extrinsics. */
int tdec_siso_batch(tdec_t *h, int B, const float *LcA, const float *LcB, const float *LcW, const float *LcY,
                    const double *LaA, const double *LaB, double sf, double *LeA, double *LeB);

/* The same SISO with float64 channel LLRs: bcjr_max_log_map as numba
 * specialises it for float64 Lc arrays (dvb_rcs2_turbo.py:135-160, 267-268:
 * in_A = Lc_A + La_A and the parity terms formed from the unrounded f64
 * values, the extrinsic subtracting the f64 sum).  Float32 inputs widened to
 * f64 give exactly tdec_siso_batch's results. */
int tdec_siso_batch_f64(tdec_t *h, int B, const double *LcA, const double *LcB, const double *LcW,
                        const double *LcY, const double *LaA, const double *LaB, double sf, double *LeA,
                        double *LeB);

/* The per-call form of the same SISO (one bcjr_max_log_map call is one row):
 * tdec_siso_staging returns a page-locked buffer owned by the handle, of 8
 * slots of *slot_bytes each (LcA, LcB, LcW, LcY, LaA, LaB, LeA, LeB: [rows][N]
 * rows of 8-byte elements; float32 channel LLRs fill the first half of their
 * slot).  The caller writes the six inputs there, calls tdec_siso_staged for B
 * <= rows rows and reads LeA / LeB back from the buffer: no argument pointers,
 * no host-side copies in the library.  The buffer stays valid until a later
 * tdec_siso_staging call asks for more rows, or tdec_destroy. */
int tdec_siso_staging(tdec_t *h, int rows, void **buf, size_t *slot_bytes);
int tdec_siso_staged(tdec_t *h, int B, int lc_f64, double sf);
/* Staged calls that waited for their rows' completion flags longer than the
 * library's time limit and ended by a stream synchronisation instead (a
 * diagnostic: the flags live in coherent host memory, so this stays 0). */
int tdec_siso_stats(const tdec_t *h, long *flag_fallbacks);

/* Full turbo decode of B codewords: replaces DVBRCS2_Turbo.decode
 * (dvb_rcs2_turbo.py:464-537; historic name turbo_decode).  llr rows of
 * llr_stride floats (>= tdec_llr_len), bits int32[B][2N] (A, B interleaved as
 * :534-535), lfinal (nullable) f64[B][2N] = Lc + La + Le1 (:529-530). */
int tdec_decode_batch(tdec_t *h, int B, const float *llr, long llr_stride, int32_t *bits, double *lfinal);

/* Pinned (page-locked) host memory for the host-pointer entry points: copies
 * from / to it go straight to the DMA engines, where pageable memory is staged
 * through the runtime's own pinned buffers.  No reference counterpart (numpy
 * buffers are pageable); DVBRCS2_Turbo.host_buffer() wraps it. */
int tdec_host_alloc(size_t bytes, void **out);
void tdec_host_free(void *p);

/* ---- device-pointer, stream-ordered API (what bench.py and multi-GPU use) ---- */

/* Size the workspace for batches of up to max_batch codewords. */
int tdec_reserve(tdec_t *h, int max_batch);
/* Bytes of the de-punctured plane buffer for B codewords.  Layout (opaque to
 * callers): per 64-codeword tile, [N][64] float4 {A, B, W1, Y1} followed by
 * [N][64] float2 {W2, Y2} -- 24 B per trellis step and codeword. */
size_t tdec_planes_bytes(const tdec_t *h, int B);
int tdec_depuncture_dev(tdec_t *h, int B, const float *d_llr, long llr_stride, float *d_planes, void *stream);
int tdec_decode_planes_dev(tdec_t *h, int B, const float *d_planes, int32_t *d_bits, double *d_lfinal,
                           void *stream);
int tdec_decode_batch_dev(tdec_t *h, int B, const float *d_llr, long llr_stride, int32_t *d_bits,
                          double *d_lfinal, void *stream);
/* Pipelining (no reference counterpart): enqueue on `stream` a one-wave kernel
 * that completes once h's most recent throughput decode launch (enqueued before
 * this call, on any stream) has handed out its last tiles, so work queued after
 * it on `stream` -- the next batch's demap -- is dispatched into the slots the
 * decoder's retiring waves free instead of competing with the decoder's grid
 * placement.  No-op before the first such launch; returns after ~2 s at most. */
int tdec_tail_gate(tdec_t *h, void *stream);

/* Soft demapper: compute_llr (test_sdr_with_coding.py:200-225) over any
 * labelled constellation (label i = bits MSB first).  syms: n_sym complex
 * values (f32 pairs, or f64 pairs when sym_f64); cons: M points (host memory,
 * f32 or f64 pairs).  Arithmetic dtype = f64 if either is f64.  div_f32: the
 * (min_d0 - min_d1) / noise_var division stays float32 (numpy >= 2 with a
 * Python-float noise_var).  sign = +1 reference sign (positive -> bit 1),
 * -1 decoder sign.  Output f64[n_sym * bps]. */
int tdec_demap_dev(int device, const void *d_syms, int sym_f64, long n_sym, const void *cons, int cons_f64,
                   int M, int bps, double noise_var, int div_f32, int sign, double *d_llr, void *stream);
int tdec_demap(int device, const void *syms, int sym_f64, long n_sym, const void *cons, int cons_f64, int M,
               int bps, double noise_var, int div_f32, int sign, double *llr);

/* The fixed-signature demapper of SURVEY §8(b) over the reference's built-in
 * Gray constellations (BPSK/QPSK/8PSK/16QAM: test_sdr_with_coding.py:25-100;
 * 64QAM/256QAM: sdr_modem.py:168-207): compute_llr(syms, mod, noise_var)
 * (:200-225) of n_sym complex64 symbols (host f32 pairs) with noise_var given
 * as a Python float would be, then rounded to f32 as decode() rounds its input
 * (dvb_rcs2_turbo.py:466).  sign +1 = reference sign, -1 = decoder sign.
 * llr_out: float[n_sym * bps]. */
enum { TDEC_MOD_BPSK = 0, TDEC_MOD_QPSK = 1, TDEC_MOD_8PSK = 2, TDEC_MOD_16QAM = 3, TDEC_MOD_64QAM = 4,
       TDEC_MOD_256QAM = 5 };
int tdec_demap_batch(int device, int mod, int sign, const float *syms_iq, long n_sym, float noise_var,
                     float *llr_out);
/* The label-ordered table of a built-in constellation (what compute_llr builds,
 * :207-208): M points as (re, im) double pairs in iq[2*M]; *is_f64 = 1 when
 * numpy's table is complex128 (QPSK), else every value is a float32.
 * Returns M, or a negative TDEC_E* code.  Host only (no device call). */
int tdec_constellation(int mod, double *iq, int *is_f64);

/* Fused demap -> de-puncture for the decoder: B codewords of S complex64
 * symbols each ([B][S]); LLR j of a codeword = bit j of its symbol stream
 * (zero-padded / truncated to the decoder's LLR count as
 * test_sdr_with_coding.py:474-478), decoder sign, rounded to f32 as decode()
 * does (:466).  Writes the plane buffer consumed by tdec_decode_planes_dev. */
int tdec_demap_planes_dev(tdec_t *h, int B, const float *d_syms, int S, const void *cons, int cons_f64, int M,
                          int bps, double noise_var, int div_f32, float *d_planes, void *stream);

/* Fused soft demap + turbo decode (one launch): what tdec_demap_planes_dev +
 * tdec_decode_planes_dev compute, bit for bit, with each persistent decoder wave
 * demapping its own next tile into a per-wave plane buffer.  Instantiated for
 * the BASELINE configurations: max-log with complex64 tables of 4 or 8 bits per
 * symbol (16QAM, 256QAM) or complex128 with 2 (QPSK), log-MAP with complex64
 * and 3 (8PSK); tdec_fused_available() says whether a (table dtype, bps) pair
 * has one (TDEC_EUNSUPPORTED otherwise).  tdec_reserve_fused sizes the
 * workspace and the per-wave planes for batches of up to max_batch. */
int tdec_reserve_fused(tdec_t *h, int max_batch);
int tdec_fused_available(const tdec_t *h, int cons_f64, int bps);
int tdec_demap_decode_dev(tdec_t *h, int B, const float *d_syms, int S, const void *cons, int cons_f64, int M,
                          int bps, double noise_var, int div_f32, int32_t *d_bits, double *d_lfinal, void *stream);

/* Batched encoder (workload generation): encode (dvb_rcs2_turbo.py:404-462)
 * with the handle's perm, bits uint8[B][2N] -> coded uint8[B][n_out],
 * n_out = the reference encoder's output length. */
int tdec_encode_dev(tdec_t *h, int B, const uint8_t *d_bits, uint8_t *d_coded, void *stream);
long tdec_encoded_len(const tdec_t *h);
/* The drop-in's DVBRCS2_Turbo.encode (dvb_rcs2_turbo.py:404-462) on the HOST
 * (compiled; needs no handle and no GPU): B rows of int32 info bits [2N]
 * (A, B interleaved; row stride bits_stride) -> int32 coded rows (stride
 * out_stride >= the returned length).  punct: [4][4] pattern rows W1, Y1, W2, Y2
 * as tdec_create; perm: int32[N] (any values in [0, N)).  An input
 * (A << 1) | B outside [-4, 3] is TDEC_ESHORT (numpy's IndexError in the
 * reference's next_state lookup; -4..-1 wrap as numpy's negative indices).
 * Returns the coded length per row (> 0) or a negative error code. */
long tdec_encode_host(int n_couples, int period, const uint8_t *punct, const int32_t *perm, long B,
                      const int32_t *bits, long bits_stride, int32_t *out, long out_stride);

/* ---- counter-based workload generation (not a reference API) ----
 * Codeword c of a batch has the GLOBAL index cw0 + c; its info bits and its
 * channel noise are Philox4x32-10 streams keyed by `seed` and counted by that
 * index, so they do not depend on the batch or the number of ranks a job is
 * sharded over.  Info bit j of codeword g is bit j%32 of word (j%128)/32 of
 * philox4x32_10({g_lo, g_hi, j/128, 0x1AF0}, {seed_lo, seed_hi}).
 * Needs n_couples % 4 == 0 and n_couples <= 1024 (every DVB-RCS2 block size). */

/* info bits -> encode (as tdec_encode_dev) -> label-ordered constellation
 * (cons_iq: M = 2^bps host (re, im) float pairs, label = bps coded bits MSB
 * first, the last symbol zero-padded; any other M is TDEC_EINVAL) -> complex AWGN of std-dev sigma per dimension
 * (Box-Muller on philox4x32_10({g_lo, g_hi, s/2, 0x2B0E}, seed)).  d_syms:
 * complex64 [B][ceil(n_out / bps)]; d_info (nullable): uint8 [B][2N]. */
int tdec_workload_dev(tdec_t *h, int B, int64_t cw0, uint64_t seed, const float *cons_iq, int M, int bps,
                      double sigma, float *d_syms, uint8_t *d_info, void *stream);
/* The info bits alone: uint8 [B][2N] of 0/1. */
int tdec_info_bits_dev(tdec_t *h, int B, int64_t cw0, uint64_t seed, uint8_t *d_info, void *stream);
/* Bit errors per codeword of decoded rows (int32 [B][2N], tdec_decode_*) against
 * those info bits: d_errs int32 [B]. */
int tdec_count_errors_dev(tdec_t *h, int B, int64_t cw0, uint64_t seed, const int32_t *d_bits, int32_t *d_errs,
                          void *stream);

/* ---- self-test of the demapper's exact shortcuts (test infrastructure; no
 * reference counterpart): which 0 compares the kernels' [1, 2] square root with
 * sqrtf and the correctly rounded one for every f32 in [1, 2] (n ignored);
 * which 1 / 2 compare the finite-input |z| with numpy's |z| (npm::cabs_np,
 * f32 / f64) on n pseudo-random finite pairs.  *mismatches = differing results. */
int tdec_selftest(int device, int which, long long n, unsigned long long seed, long long *mismatches);
/* which 3 (same entry point): the log-MAP primitives outside the captured
 * tables -- every f32 t >= 48 gives 0 <= v_exp_f32(-t) <= 2^-39 (+0 at t = inf),
 * NaN -> NaN for v_exp_f32 and v_log_f32, v_log_f32(1) = 0 (n, seed ignored).
 * which 4: the demapper's unscaled f64 division / square root (TDEC_DM_FAST64)
 * against the compiler's sequences on n pseudo-random operands of the ranges
 * the demapper meets (|z|, a / b, sqrt on [1, 2]).
 *
 * The exact outputs of the log-MAP primitives (the oracle's tables,
 * oracle/tdec_oracle.c orc_set_trans): out[i] = v_exp_f32(-t) (which 0) or
 * v_log_f32(w) (which 1) for the f32 whose bit pattern is lo_bits + i, i < n;
 * out is a host buffer of n floats. */
int tdec_selftest_trans(int device, int which, uint32_t lo_bits, long long n, float *out);

#ifdef __cplusplus
}
#endif
#endif /* TDEC_H */
