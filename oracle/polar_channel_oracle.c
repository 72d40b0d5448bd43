/*
 * polar_channel_oracle.c -- CPU restatement of the reference's C-sim frame chain and error
 * counter. TEST INFRASTRUCTURE ONLY (tests/ and bench.py's checks use it; the product
 * library never does).
 *
 * Chain, per frame f (src/testbench/sc_top_module.h:101-160 wiring):
 *   encoder   sc_encoder.h:91-122     frame f sends codeword f % ncw of a fixed table
 *                                     (cw8x4 / cw512x256 / cw1024x512), all-zero otherwise
 *   bpsk      sc_bpsk.h:50-56         bit 1 -> -1.0f, bit 0 -> +1.0f
 *   xorshift  sc_xorshift128.h:56-125 two xorshift128 streams seeded from the 8-bit seed,
 *                                     sample = 1.0f - (float)w * 2^-32
 *   awgn      sc_awgn.h:60-89         Box-Muller on (stream 1, stream 2): x = sqrtf(-2 logf(r1)),
 *                                     y = 2*pi*r2; emits x sinf(y) then x cosf(y)
 *   adder     sc_adder.h:135-154      v = bpsk + noise * sigma
 *   quantizer sc_quantizer.h:69-81    q = (short)(v * beta), clamped to [vsatn, vsatp]
 * One frame of N symbols consumes N/2 Box-Muller pairs (N/2 draws of each stream).
 *
 * Error counter (sc_error_counter.h:50-126): per frame err = #(x^ != x) held in an
 * sc_uint<10> (mod 1024); bit errors += err, frame errors += (err != 0).
 *
 * Float semantics follow the reference's C-sim on x86-64 with glibc: separate float
 * multiply / add (no contraction: this file is compiled without FMA), glibc logf / sinf /
 * cosf / sqrtf, and (short) of a float through a 32-bit truncating conversion
 * (cvttss2si: out-of-range -> 0x80000000) then truncation to 16 bits.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { uint32_t x, y, z, w; } xs128_t;

static void xs_seed(xs128_t s[2], uint32_t seed8)
{
    const uint32_t m = (seed8 & 0xFFu) * 0x01010101u;   /* (mask, mask, mask, mask) */
    s[0].x = 0x12311178u & m; s[0].y = 0x65498732u | m; s[0].z = 0xFEDCAA01u ^ m; s[0].w = 0xF489A179u + m;
    s[1].x = 0x98765432u & m; s[1].y = 0x12345678u | m; s[1].z = 0xFCBADEFFu ^ m; s[1].w = 0x12121212u + m;
}

static uint32_t xs_next(xs128_t *s)
{
    uint32_t t = s->x;
    t ^= t << 11;
    t ^= t >> 8;
    s->x = s->y;
    s->y = s->z;
    s->z = s->w;
    s->w ^= s->w >> 19;
    s->w ^= t;
    return s->w;
}

static float xs_float(uint32_t w) { return 1.0f - (float)w * (1.0f / 4294967296.0f); }

static int16_t to_short(float v)
{
    int32_t i = (v > -2147483648.0f && v < 2147483648.0f) ? (int32_t)v : (int32_t)0x80000000u;
    return (int16_t)(uint16_t)(uint32_t)i;
}

/* Stream states at the start of frame `frame0` (frame0 * N/2 draws of each stream). */
void orc_csim_states(uint32_t N, uint32_t seed8, uint64_t frame0, uint32_t *out /* 8 words */)
{
    xs128_t s[2];
    xs_seed(s, seed8);
    const uint64_t draws = frame0 * (uint64_t)(N / 2);
    for (uint64_t k = 0; k < draws; k++) {
        xs_next(&s[0]);
        xs_next(&s[1]);
    }
    memcpy(out, s, sizeof(s));
}

/* Frames frame0 .. frame0+nframes-1 of the chain. codewords: [ncw][N] bytes (0/1) or NULL
 * (all-zero); llr: [nframes][N] int8; xout (optional): [nframes][N] sent codeword bits. */
void orc_csim_frames(uint32_t N, uint32_t seed8, uint64_t frame0, int nframes, float sigma, int beta,
                     int vsatn, int vsatp, const uint8_t *codewords, int ncw, int8_t *llr, uint8_t *xout)
{
    static const float PI1 = 3.14159265358979f;
    const float PI2 = 2.0f * PI1;
    const float fbeta = (float)beta;
    xs128_t s[2];
    orc_csim_states(N, seed8, frame0, (uint32_t *)s);
    for (int f = 0; f < nframes; f++) {
        const uint64_t fi = frame0 + (uint64_t)f;
        const uint8_t *cw = (codewords && ncw > 0) ? codewords + (size_t)(fi % (uint64_t)ncw) * N : NULL;
        for (uint32_t k = 0; k < N / 2; k++) {
            const float r1 = xs_float(xs_next(&s[0]));
            const float y = PI2 * xs_float(xs_next(&s[1]));
            const float x = sqrtf(-2.0f * logf(r1));
            const float vsin = sinf(y), vcos = cosf(y);
            const float noise[2] = {x * vsin, x * vcos};
            for (int h = 0; h < 2; h++) {
                const uint32_t i = 2 * k + (uint32_t)h;
                const uint8_t bit = cw ? (cw[i] & 1u) : 0u;
                const float o = bit ? -1.0f : 1.0f;
                const float n = noise[h] * sigma;
                const float v = o + n;
                int q = to_short(v * fbeta);
                q = q > vsatn ? q : vsatn;
                q = q < vsatp ? q : vsatp;
                llr[(size_t)f * N + i] = (int8_t)q;
                if (xout) xout[(size_t)f * N + i] = bit;
            }
        }
    }
}

/* sc_error_counter: counts[0] += sum of per-frame (errors mod 1024), counts[1] += frames with
 * a non-zero wrapped count, counts[2] += exact bit errors. xhat / xref: [nframes][N] bytes. */
void orc_count_errors(uint32_t N, int nframes, const uint8_t *xhat, const uint8_t *xref, uint64_t *counts)
{
    for (int f = 0; f < nframes; f++) {
        uint32_t e = 0;
        for (uint32_t i = 0; i < N; i++) e += (xhat[(size_t)f * N + i] & 1u) != (xref[(size_t)f * N + i] & 1u);
        counts[0] += e & 1023u;
        counts[1] += (e & 1023u) != 0u;
        counts[2] += e;
    }
}
