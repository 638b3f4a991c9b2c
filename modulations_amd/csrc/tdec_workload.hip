// tdec_workload.hip -- device-side workload generation for the turbo decoder
// (SURVEY §8(d), §8(f) row 1): counter-based info bits, the batched encoder
// (encode, dvb_rcs2_turbo.py:404-462), Gray mapping and complex AWGN, and the
// error counters of a BER point.
//
// Counter-based: every random number is Philox4x32-10 (Random123) of a counter
// that names the codeword by its GLOBAL index, so a codeword's info bits and
// noise do not depend on the batch it was generated in, nor on the number of
// ranks a job is sharded over:
//   info bits   ctr = {cw_lo, cw_hi, 128-bit block, 0x1AF0}, key = seed
//   noise       ctr = {cw_lo, cw_hi, symbol pair,    0x2B0E}, key = seed
// Info bit j of a codeword is bit j % 32 of word (j % 128) / 32 of block j / 128.
// Noise: Box-Muller, u = (x >> 8 + 0.5) * 2^-24 in (0, 1): one complex sample
// per symbol from two words, r = sigma * sqrt(-2 ln u1), theta = 2 pi u2.
//
// Layout (MI355X-first): one wave owns a tile of 64 codewords.  The tile's info
// couples are packed 16 per 32-bit word into LDS, [word][lane] (the encoder
// recursion is serial per codeword, one codeword per lane, and the
// interleaver read inp[perm[i]] is the same word for every lane: conflict
// free).  Everything that touches HBM is done cooperatively by the wave in
// row order -- consecutive lanes write consecutive bytes of one codeword row
// -- through small LDS chunks, so every global access is coalesced:
//   bits in    32 B per (codeword, 16 couples) item, 4 x 8-B loads
//   coded out  4-B stores (byte stores when a row is not a multiple of 4)
//   symbols    8-B complex64 stores, noise generated in the coalesced phase
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdec {

struct Philox4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11; Random123's philox4x32_R(10, ...)).
__host__ __device__ __forceinline__ Philox4 philox4x32_10(Philox4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = Philox4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    }
    return c;
}

constexpr uint32_t INFO_DOMAIN = 0x1AF0u, NOISE_DOMAIN = 0x2B0Eu;

__device__ __forceinline__ Philox4 info_block(uint64_t cw, uint32_t blk, uint64_t seed) {
    return philox4x32_10(Philox4{(uint32_t)cw, (uint32_t)(cw >> 32), blk, INFO_DOMAIN}, (uint32_t)seed,
                         (uint32_t)(seed >> 32));
}
__device__ __forceinline__ uint32_t pick(const Philox4 &r, int q) {
    return q == 0 ? r.x : (q == 1 ? r.y : (q == 2 ? r.z : r.w));
}
// info bits (bit 2i = A_i, bit 2i+1 = B_i) -> couple word (inp_i = A<<1 | B at bits 2i+1..2i)
__device__ __forceinline__ uint32_t swap_pairs(uint32_t x) { return ((x & 0x55555555u) << 1) | ((x >> 1) & 0x55555555u); }

constexpr int ENC_MAX_N = 1024;                 // couples the LDS-staged encoder holds (else the row kernel)
constexpr int ENC_NW = ENC_MAX_N / 16;          // couple words per codeword
constexpr int SYM_CHUNK = 64;                   // symbols per lane staged before a coalesced flush
constexpr int OUT_CHUNK = 8;                    // coded words (32 bits) per lane staged before a flush

struct WorkloadArgs {
    int B, N, period, bps, M;
    long n_out;                                 // coded bits per codeword
    int S;                                      // symbols per codeword = ceil(n_out / bps)
    uint64_t cw0, seed;                         // global index of codeword 0 of this batch; generator key
    float sigma;                                // noise std-dev per dimension
    unsigned char punct[16];
    int circ[16];
    const int *perm;
    const uint8_t *bits_in;                     // [B][2N] 0/1 bytes, or null: Philox info bits
    uint8_t *info_out;                          // [B][2N] 0/1 bytes (nullable)
    uint8_t *coded_out;                         // [B][n_out] (nullable)
    float2 *syms;                               // [B][S] complex64 (nullable)
    float2 cons[256];                           // label-ordered constellation (by value: no upload)
};

// Fill the wave's couple words inpw[w][lane] for codewords base .. base+63.
__device__ __forceinline__ void load_couples(const WorkloadArgs &p, long base, uint32_t (*inpw)[64], int lane) {
    const int NW = (p.N + 15) / 16;
    const long row = 2L * p.N;
    if (p.bits_in) {
        for (int t = lane; t < 64 * NW; t += 64) {
            const int l = t / NW, w = t - l * NW;
            uint32_t word = 0;
            if (base + l < p.B) {
                const uint8_t *src = p.bits_in + (base + l) * row + 32L * w;
                const int nb = (int)min(32L, row - 32L * w);   // a multiple of 8: 2N is (N % 4 == 0 or the row kernel)
                for (int c = 0; c < nb; c += 8) {
                    const uint2 v = *reinterpret_cast<const uint2 *>(src + c);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        word |= ((v.x >> (8 * k)) & 1u) << ((c + k) ^ 1);
                        word |= ((v.y >> (8 * k)) & 1u) << ((c + 4 + k) ^ 1);
                    }
                }
            }
            inpw[w][l] = word;
        }
    } else {
        const int NB = (2 * p.N + 127) / 128;    // 128-bit Philox blocks per codeword
        for (int t = lane; t < 64 * NB; t += 64) {
            const int l = t / NB, b = t - l * NB;
            const Philox4 r = info_block(p.cw0 + (uint64_t)(base + l), (uint32_t)b, p.seed);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * b + q < NW) inpw[4 * b + q][l] = swap_pairs(pick(r, q));
        }
    }
    __syncthreads();
    if (p.info_out) {   // 0/1 bytes, 4 per store, row order
        for (int t = lane; t < 64 * NW * 8; t += 64) {
            const int l = t / (NW * 8), r = t - l * (NW * 8), w = r >> 3, q = r & 7;
            const long j = 32L * w + 4 * q;      // first info bit of this store
            if (base + l < p.B && j < row) {
                const uint32_t x = inpw[w][l] >> (4 * q);
                const uint32_t bytes = ((x >> 1) & 1u) | ((x & 1u) << 8) | (((x >> 3) & 1u) << 16) | (((x >> 2) & 1u) << 24);
                *reinterpret_cast<uint32_t *>(p.info_out + (base + l) * row + j) = bytes;
            }
        }
    }
}

__device__ __forceinline__ int inp_at(uint32_t (*inpw)[64], int i, int lane) { return (inpw[i >> 4][lane] >> (2 * (i & 15))) & 3; }

__device__ __forceinline__ int enc_next(int s, int inp) {   // next_state (:357-366)
    const int dk = ((inp >> 1) & 1) ^ (inp & 1) ^ ((s >> 2) & 1) ^ ((s >> 3) & 1);
    return (((s >> 2) & 1) << 3) | (((s >> 1) & 1) << 2) | ((s & 1) << 1) | dk;
}

// Row-order flush of a chunk of coded words outw[w][lane] (w < nw) covering coded
// bits [b0, b0 + 32 nw) of every codeword: one byte per bit.
__device__ __forceinline__ void flush_coded(const WorkloadArgs &p, long base, uint32_t (*outw)[64], int nw, long b0,
                                            int lane) {
    __syncthreads();
    if ((p.n_out & 3) == 0) {
        const int per = nw * 8;                  // 4-byte stores per codeword
        for (int t = lane; t < 64 * per; t += 64) {
            const int l = t / per, r = t - l * per;
            const long j = b0 + 4L * r;
            if (base + l < p.B && j < p.n_out) {
                const uint32_t x = outw[r >> 3][l] >> (4 * (r & 7));
                const uint32_t v = (x & 1u) | (((x >> 1) & 1u) << 8) | (((x >> 2) & 1u) << 16) | (((x >> 3) & 1u) << 24);
                *reinterpret_cast<uint32_t *>(p.coded_out + (base + l) * p.n_out + j) = v;
            }
        }
    } else {
        const int per = nw * 32;
        for (int t = lane; t < 64 * per; t += 64) {
            const int l = t / per, r = t - l * per;
            const long j = b0 + r;
            if (base + l < p.B && j < p.n_out) p.coded_out[(base + l) * p.n_out + j] = (outw[r >> 5][l] >> (r & 31)) & 1u;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ float2 awgn(uint64_t cw, long s, const WorkloadArgs &p) {
    const Philox4 r = philox4x32_10(Philox4{(uint32_t)cw, (uint32_t)(cw >> 32), (uint32_t)(s >> 1), NOISE_DOMAIN},
                                    (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
    const uint32_t a = (s & 1) ? r.z : r.x, b = (s & 1) ? r.w : r.y;
    const float u1 = ((float)(a >> 8) + 0.5f) * 0x1p-24f, u2 = ((float)(b >> 8) + 0.5f) * 0x1p-24f;
    const float rad = p.sigma * sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincospif(2.0f * u2, &sn, &cs);
    return make_float2(rad * cs, rad * sn);
}

// Row-order flush of a chunk of symbol labels lab[k][lane] (k < ns): symbols
// [s0, s0 + ns) of every codeword, table point + AWGN, complex64.
__device__ __forceinline__ void flush_syms(const WorkloadArgs &p, long base, uint8_t (*lab)[64], const float2 *cons,
                                           int ns, long s0, int lane) {
    __syncthreads();
    for (int t = lane; t < 64 * ns; t += 64) {
        const int l = t / ns, k = t - l * ns;
        if (base + l < p.B) {
            const uint64_t cw = p.cw0 + (uint64_t)(base + l);
            const float2 x = cons[lab[k][l]], n = awgn(cw, s0 + k, p);
            p.syms[(base + l) * (long)p.S + s0 + k] = make_float2(x.x + n.x, x.y + n.y);
        }
    }
    __syncthreads();
}

// One wave per 64-codeword tile (block = 1 wave: no cross-wave barriers).
__global__ __launch_bounds__(64) void k_workload(WorkloadArgs p) {
    __shared__ uint32_t inpw[ENC_NW][64];
    __shared__ uint32_t outw[OUT_CHUNK][64];
    __shared__ uint8_t lab[SYM_CHUNK][64];
    __shared__ float2 cons[256];
    const int lane = threadIdx.x;
    const long base = (long)blockIdx.x * 64;
    for (int m = lane; m < p.M; m += 64) cons[m] = p.cons[m];
    load_couples(p, base, inpw, lane);
    if (!p.coded_out && !p.syms) return;
    // pass 1: final states from 0 (:433-437 of _encode_component); circular start (:438)
    int s1 = 0, s2 = 0;
    for (int i = 0; i < p.N; ++i) {
        s1 = enc_next(s1, inp_at(inpw, i, lane));
        s2 = enc_next(s2, inp_at(inpw, p.perm[i], lane));
    }
    s1 = p.circ[s1];
    s2 = p.circ[s2];
    // pass 2: the coded stream in output order (:449-460), one bit at a time
    uint32_t acc = 0;
    int nacc = 0, nw = 0;           // coded-word accumulator; words staged in outw
    long b0 = 0;                    // first coded bit of the staged chunk
    int lbl = 0, nl = 0, ns = 0;    // symbol label accumulator (MSB first); labels staged in lab
    long s0 = 0;
    auto emit = [&](int bit) {
        if (p.coded_out) {
            acc |= (uint32_t)bit << nacc;
            if (++nacc == 32) {
                outw[nw][lane] = acc;
                acc = 0;
                nacc = 0;
                if (++nw == OUT_CHUNK) {
                    flush_coded(p, base, outw, nw, b0, lane);
                    b0 += 32L * nw;
                    nw = 0;
                }
            }
        }
        if (p.syms) {
            lbl = (lbl << 1) | bit;
            if (++nl == p.bps) {
                lab[ns][lane] = (uint8_t)lbl;
                lbl = 0;
                nl = 0;
                if (++ns == SYM_CHUNK) {
                    flush_syms(p, base, lab, cons, ns, s0, lane);
                    s0 += ns;
                    ns = 0;
                }
            }
        }
    };
    for (int i = 0; i < p.N; ++i) {
        const int ph = i % p.period;
        const int i1 = inp_at(inpw, i, lane), i2 = inp_at(inpw, p.perm[i], lane);
        const int dk1 = ((i1 >> 1) & 1) ^ (i1 & 1) ^ ((s1 >> 2) & 1) ^ ((s1 >> 3) & 1);
        const int dk2 = ((i2 >> 1) & 1) ^ (i2 & 1) ^ ((s2 >> 2) & 1) ^ ((s2 >> 3) & 1);
        emit((i1 >> 1) & 1);
        emit(i1 & 1);
        if (p.punct[0 * 4 + ph]) emit(dk1 ^ (s1 & 1) ^ ((s1 >> 1) & 1) ^ ((s1 >> 3) & 1));
        if (p.punct[1 * 4 + ph]) emit(dk1 ^ ((s1 >> 1) & 1) ^ ((s1 >> 2) & 1) ^ ((s1 >> 3) & 1));
        if (p.punct[2 * 4 + ph]) emit(dk2 ^ (s2 & 1) ^ ((s2 >> 1) & 1) ^ ((s2 >> 3) & 1));
        if (p.punct[3 * 4 + ph]) emit(dk2 ^ ((s2 >> 1) & 1) ^ ((s2 >> 2) & 1) ^ ((s2 >> 3) & 1));
        s1 = enc_next(s1, i1);
        s2 = enc_next(s2, i2);
    }
    if (p.coded_out) {
        if (nacc) outw[nw++][lane] = acc;
        if (nw) flush_coded(p, base, outw, nw, b0, lane);
    }
    if (p.syms) {
        if (nl) lab[ns++][lane] = (uint8_t)(lbl << (p.bps - nl));   // zero pad of the last symbol
        if (ns) flush_syms(p, base, lab, cons, ns, s0, lane);
    }
}

// Bit errors of decoded rows against the counter-based info bits: one wave per
// codeword, each lane 4 consecutive bits (one 16-B load) per sweep.
__global__ __launch_bounds__(64) void k_count_errors(int B, int N, uint64_t cw0, uint64_t seed, const int32_t *bits,
                                                     int32_t *errs) {
    const int lane = threadIdx.x;
    const long cw = blockIdx.x;
    if (cw >= B) return;
    const int row = 2 * N;
    const int4 *r4 = reinterpret_cast<const int4 *>(bits + cw * (long)row);
    int e = 0;
    for (int j = 4 * lane; j < row; j += 256) {
        const Philox4 r = info_block(cw0 + (uint64_t)cw, (uint32_t)(j >> 7), seed);
        const uint32_t w = pick(r, (j >> 5) & 3) >> (j & 31);
        int4 v;
        if (j + 4 <= row && (row & 3) == 0) v = r4[j >> 2];
        else {
            const int32_t *q = bits + cw * (long)row + j;
            v = make_int4(q[0], j + 1 < row ? q[1] : 0, j + 2 < row ? q[2] : 0, j + 3 < row ? q[3] : 0);
        }
        e += (v.x != (int)(w & 1u)) + (j + 1 < row && v.y != (int)((w >> 1) & 1u)) +
             (j + 2 < row && v.z != (int)((w >> 2) & 1u)) + (j + 3 < row && v.w != (int)((w >> 3) & 1u));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o);
    if (lane == 0) errs[cw] = e;
}

}  // namespace tdec
