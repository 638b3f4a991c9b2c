/*
 * modem.h -- C ABI of the MI355X (gfx950) modem front-end kernels
 * (SURVEY.md §8(f) row 4): symbol mappers, hard-decision demodulators, RRC
 * pulse shaping / matched filtering, and the int8/uint8 IQ sample format.
 *
 * These replace the per-symbol Python loops and numpy/scipy calls of the
 * reference's front-end (poriya219/modulations):
 *   sdr_modem.py:66-266      SDRModem Gray mappers / demods, _rrc_filter :77-91, _upsample_filter :93-97
 *   sdr_modem.py:329-342     SDRModem._save_iq / _load_iq
 *   modulators.py:19-199     rrcosfilter, Modulator (natural-label mappers, argmin demods,
 *                            apply_pulse_shaping = upfirdn, matched_filter)
 *   test_sdr_with_coding.py:25-128, 228-240   the harness copies of the same functions
 * modulations_amd/modem.py binds them with ctypes behind the reference's class
 * and function names.  Tables (constellations, label maps, filter taps) are
 * computed on the host with the reference's own expressions and passed by
 * value; the per-sample work runs on the GPU.
 *
 * Conventions are those of tdec.h: plain pointers and sizes, complex values
 * as interleaved (re, im) pairs of f32 (complex64) or f64 (complex128);
 * entry points without _dev take HOST pointers and synchronise, _dev entry
 * points take DEVICE pointers and a hipStream_t (void*) and are stream-ordered.
 * Return 0 or a negative MDM_E* code; mdm_last_error() says why.
 */
#ifndef MODEM_H
#define MODEM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    MDM_OK = 0,
    MDM_EINVAL = -1, /* bad argument                                           -> ValueError */
    MDM_ENOMEM = -3, /* device allocation failed                               -> MemoryError */
    MDM_EHIP = -4,   /* HIP runtime error                                      -> RuntimeError */
    MDM_ENAN = -8    /* NaN symbol where the reference does int(NaN)           -> ValueError */
};

/* Hard-decision rules (which reference demodulator each one restates). */
enum {
    MDM_DEMOD_GT0 = 0,      /* bit = Re(s) > 0: SDRModem._bpsk_demod :104-105, Modulator.demod_bpsk :121-122 */
    MDM_DEMOD_QPSK = 1,     /* bits = (Re < 0, Im < 0): _qpsk_demod :114-118, demod_qpsk :133-136   */
    MDM_DEMOD_PSK8 = 2,     /* round(angle / (pi/4)) % 8 -> labels[]: _psk8_demod :132-140,
                               Modulator.demod_8psk :147-155 (angle in the symbols' precision)      */
    MDM_DEMOD_QAM_AXIS = 3, /* per axis: clip(round((x*scale + L-1) / 2), 0, L-1) -> labels[] (f64):
                               _qam16/64/256_demod :156-220                                          */
    MDM_DEMOD_ARGMIN = 4    /* argmin_m |s - cons[m]| (complex128, numpy's |z|), label = m MSB first:
                               Modulator._demod_qam_generic :165-171                                 */
};

/* Labels -> constellation points.  bits: n_bits bytes of 0/1, zero-padded to
 * whole symbols (the mappers' np.append(bits, 0...)); label of symbol s =
 * bits[s*bps .. s*bps+bps) MSB first; table = M = 2^bps points (host memory;
 * f32 pairs, or f64 pairs when table_f64), M <= 256 (f32) / 128 (f64).
 * Output: ceil(n_bits / bps) points in the table's dtype. */
int mdm_map_dev(int device, const uint8_t *d_bits, long n_bits, int bps, const void *table, int table_f64,
                void *d_syms, void *stream);
int mdm_map(int device, const uint8_t *bits, long n_bits, int bps, const void *table, int table_f64, void *syms);

/* Hard demodulation of n_sym symbols (f32 or f64 pairs) into n_sym*bps bit
 * bytes (MSB first).  labels (host, nullable = identity): constellation index
 * -> label, 2^bps entries (PSK8: the inverse Gray map; QAM_AXIS: per-axis
 * inverse Gray map of 2^(bps/2) entries).  scale: QAM_AXIS multiplier
 * (np.sqrt(10/42/170)).  cons (host f64 pairs, M = 2^bps <= 64): ARGMIN table.
 * nan_raises: 1 = a NaN symbol is an error (the reference's int(NaN) in its
 * per-symbol loops: MDM_ENAN from the host entry point, counted into
 * *d_nan_count by the _dev one), 0 = index 0 (numpy astype(int) of NaN on
 * x86, then % 8: Modulator.demod_8psk).  d_nan_count: nullable device uint32. */
int mdm_demod_dev(int device, int kind, const void *d_syms, int sym_f64, long n_sym, int bps, const int32_t *labels,
                  double scale, const double *cons, int nan_raises, uint8_t *d_bits, uint32_t *d_nan_count,
                  void *stream);
int mdm_demod(int device, int kind, const void *syms, int sym_f64, long n_sym, int bps, const int32_t *labels,
              double scale, const double *cons, int nan_raises, uint8_t *bits);

/* Up-sample -> FIR -> down-sample, complex128 out:
 *   out[i] = sum_k taps[k] * xu[i*down + offset - k],  i < n_out,
 *   xu[j]  = x[j / up] if j % up == 0 and 0 <= j / up < n_x, else 0.
 * Covers np.convolve(up, taps, 'same') of _upsample_filter (up = sps, offset =
 * (min(n_x*sps, n_taps) - 1) // 2), scipy upfirdn of apply_pulse_shaping
 * (offset 0) and the full convolution + [2*delay::sps] of matched_filter
 * (up 1, down sps).  taps: host f64, n_taps <= 256.  x: f32 or f64 pairs. */
int mdm_fir_dev(int device, const void *d_x, int x_f64, long n_x, const double *taps, int n_taps, int up, int down,
                long offset, long n_out, double *d_out, void *stream);
int mdm_fir(int device, const void *x, int x_f64, long n_x, const double *taps, int n_taps, int up, int down,
            long offset, long n_out, double *out);

/* _save_iq's sample conversion (sdr_modem.py:329-335): sig / (max|sig| + 1e-10)
 * * 0.95 with numpy's complex division and multiplication in the signal's
 * precision, then Re/Im * 127 clipped to +-127 and truncated to int8,
 * interleaved.  n >= 1.  d_scratch: 8 device bytes (the max). */
int mdm_iq_quantize_dev(int device, const void *d_sig, int sig_f64, long n, int8_t *d_iq, void *d_scratch,
                        void *stream);
int mdm_iq_quantize(int device, const void *sig, int sig_f64, long n, int8_t *iq);

/* _load_iq's sample conversion (sdr_modem.py:337-342): interleaved uint8 I/Q
 * -> complex64 ((x - 127.5) / 127.5 in f32).  n_pairs complex outputs. */
int mdm_iq_dequantize_dev(int device, const uint8_t *d_raw, long n_pairs, float *d_sig, void *stream);
int mdm_iq_dequantize(int device, const uint8_t *raw, long n_pairs, float *sig);

const char *mdm_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MODEM_H */
