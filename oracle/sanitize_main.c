/* sanitize_main.c -- drives every oracle entry point under AddressSanitizer +
 * UndefinedBehaviorSanitizer (race detection / sanitizers).
 *
 * TEST INFRASTRUCTURE ONLY: built and run by tests/test_oracle_sanitizers.py
 * (make -C oracle sanitize), never shipped.  Covers the edge sizes the parity
 * tests use (N = 1, 2, 3, 5, 48, 50; short LLR vectors; 0 symbols; NaN / inf /
 * +-1e30 inputs) with both max-log and log-MAP.  Exit status 0 = clean; the
 * sanitizers abort on the first finding.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void orc_trellis(int32_t *tables, int32_t *G);
void orc_siso(int N, const float *LcA, const float *LcB, const float *LcW, const float *LcY, const double *LaA,
              const double *LaB, const int32_t *tables, double sf, int algo, double *LeA, double *LeB);
int orc_decode(int N, int period, const uint8_t *punct, int iterations, int algo, const int32_t *perm,
               const int32_t *inv_perm, const int32_t *tables, const float *llr, long n_llr, int32_t *bits,
               double *lfinal);
int orc_decode_batch(int B, int N, int period, const uint8_t *punct, int iterations, int algo,
                     const int32_t *perm, const int32_t *inv_perm, const int32_t *tables, const float *llr,
                     long llr_stride, long n_llr, int32_t *bits, double *lfinal, int nthreads);
long orc_encode(int N, int period, const uint8_t *punct, const int32_t *perm, const int32_t *tables,
                const int32_t *G, const int32_t *bits, int32_t *coded);
void orc_demap_c64(const float *syms, long n_sym, const float *cons, int M, int bps, double noise_var,
                   int div_f32, double *llr);
void orc_demap_c128(const double *syms, long n_sym, const double *cons, int M, int bps, double noise_var,
                    double *llr);
void orm_map(const uint8_t *bits, long n_bits, int bps, const double *table, double *out);
void orm_demod_argmin(const double *syms, long n, int bps, const double *cons, uint8_t *bits);
void orm_fir(const double *x, long n_x, const double *h, int L, int up, int down, long off, long n_out,
             double *out);
void orm_iq_quantize_f64(const double *sig, long n, int8_t *out);
void orm_iq_dequantize(const uint8_t *raw, long n_pairs, float *out);

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static double urand(void) /* [0, 1) */
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (double)(rng >> 11) * 0x1.0p-53;
}
static float nrand(float scale) { return (float)((urand() * 2.0 - 1.0) * scale); }

#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                                       \
        }                                                                   \
    } while (0)

int main(void)
{
    int32_t tables[320], G[16];
    orc_trellis(tables, G);
    /* rows W1, Y1, W2, Y2; columns the pattern phase (PUNCTURE_PATTERNS, dvb_rcs2_turbo.py:21-26) */
    const uint8_t punct13[16] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0}; /* rate 1/3, period 1 */
    const uint8_t punct12[16] = {1, 0, 0, 0, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0}; /* rate 1/2, period 2 */
    const int sizes[] = {1, 2, 3, 5, 48, 50};
    for (size_t si = 0; si < sizeof sizes / sizeof *sizes; ++si) {
        const int N = sizes[si];
        int32_t *perm = malloc(sizeof(int32_t) * N), *inv = malloc(sizeof(int32_t) * N);
        for (int k = 0; k < N; ++k) perm[k] = (int32_t)((7L * k + 3) % N);
        for (int k = 0; k < N; ++k) inv[perm[k]] = k;
        for (int algo = 0; algo < 2; ++algo)
            for (int r = 0; r < 2; ++r) {
                const uint8_t *punct = r ? punct12 : punct13;
                const int period = r ? 2 : 1;
                const long n_llr = 6L * N, n_need = r ? 4L * N : 6L * N, B = 3;
                float *llr = malloc(sizeof(float) * B * n_llr);
                for (long i = 0; i < B * n_llr; ++i) llr[i] = nrand(8.0f);
                llr[0] = NAN; /* non-finite inputs take the same paths */
                llr[n_llr] = INFINITY;
                llr[2 * n_llr + 1] = -1e30f;
                int32_t *bits = malloc(sizeof(int32_t) * B * 2 * N);
                double *lf = malloc(sizeof(double) * B * 2 * N);
                CHECK(orc_decode_batch((int)B, N, period, punct, 3, algo, perm, inv, tables, llr, n_llr, n_llr,
                                       bits, lf, 2) == 0);
                CHECK(orc_decode(N, period, punct, 2, algo, perm, inv, tables, llr, n_llr, bits, NULL) == 0);
                /* one LLR short: the de-puncture walk reports it instead of reading past the end */
                float *tail = malloc(sizeof(float) * n_need);
                memcpy(tail, llr, sizeof(float) * (n_need - 1));
                CHECK(orc_decode(N, period, punct, 1, algo, perm, inv, tables, tail, n_need - 1, bits, NULL) == -1);
                CHECK(orc_decode(N, period, punct, 0, algo, perm, inv, tables, llr, n_llr, bits, NULL) == -2);
                free(tail);
                /* one SISO with extreme a-priori values */
                float *lc = malloc(sizeof(float) * 4 * N);
                double *la = malloc(sizeof(double) * 4 * N);
                for (int i = 0; i < 4 * N; ++i) lc[i] = nrand(30.0f), la[i] = urand() * 600.0 - 300.0;
                la[0] = 1e300;
                orc_siso(N, lc, lc + N, lc + 2 * N, lc + 3 * N, la, la + N, tables, 0.7, algo, la + 2 * N,
                         la + 3 * N);
                /* encoder */
                int32_t *info = malloc(sizeof(int32_t) * 2 * N), *coded = malloc(sizeof(int32_t) * (6 * N + 8));
                for (int i = 0; i < 2 * N; ++i) info[i] = urand() < 0.5;
                CHECK(orc_encode(N, period, punct, perm, tables, G, info, coded) == n_need);
                free(info); free(coded); free(lc); free(la); free(llr); free(bits); free(lf);
            }
        free(perm); free(inv);
    }

    /* demappers: 16QAM table, random / non-finite / empty symbol streams */
    float cons32[32];
    double cons64[32];
    const int g[4] = {0, 1, 3, 2};
    for (int m = 0; m < 16; ++m) {
        cons64[2 * m] = (2 * g[m >> 2] - 3) / sqrt(10.0);
        cons64[2 * m + 1] = (2 * g[m & 3] - 3) / sqrt(10.0);
        cons32[2 * m] = (float)cons64[2 * m];
        cons32[2 * m + 1] = (float)cons64[2 * m + 1];
    }
    const long ns = 257;
    float *s32 = malloc(sizeof(float) * 2 * ns);
    double *s64 = malloc(sizeof(double) * 2 * ns), *llr = malloc(sizeof(double) * 8 * ns);
    for (long i = 0; i < 2 * ns; ++i) s64[i] = s32[i] = nrand(2.0f);
    s32[0] = NAN, s32[3] = INFINITY, s32[5] = -1e30f;
    s64[0] = NAN, s64[3] = -INFINITY, s64[5] = 1e300;
    orc_demap_c64(s32, ns, cons32, 16, 4, 0.1, 1, llr);
    orc_demap_c64(s32, ns, cons32, 16, 4, 1e-9, 0, llr);
    orc_demap_c128(s64, ns, cons64, 16, 4, 0.1, llr);
    orc_demap_c64(s32, 0, cons32, 16, 4, 0.1, 1, llr);

    /* modem oracle: mapper (ragged bit count), argmin demod, FIR forms, IQ files */
    uint8_t *bits = malloc(4 * ns + 3), *hb = malloc(4 * ns);
    for (long i = 0; i < 4 * ns + 3; ++i) bits[i] = urand() < 0.5;
    double *mapped = malloc(sizeof(double) * 2 * (ns + 1));
    orm_map(bits, 4 * ns + 3, 4, cons64, mapped);
    orm_demod_argmin(s64, ns, 4, cons64, hb);
    double taps[33];
    for (int k = 0; k < 33; ++k) taps[k] = nrand(1.0f);
    double *fo = malloc(sizeof(double) * 2 * 8 * ns);
    orm_fir(s64, ns, taps, 33, 8, 1, 0, 8 * ns, fo);
    orm_fir(s64, ns, taps, 33, 1, 8, 16, ns / 8, fo);
    orm_fir(s64, ns, taps, 33, 3, 2, 5, ns, fo);
    int8_t *q = malloc(2 * ns);
    orm_iq_quantize_f64(s64, ns, q);
    float *dq = malloc(sizeof(float) * 2 * ns);
    orm_iq_dequantize((const uint8_t *)q, ns, dq);
    free(s32); free(s64); free(llr); free(bits); free(hb); free(mapped); free(fo); free(q); free(dq);
    puts("sanitize: clean");
    return 0;
}
