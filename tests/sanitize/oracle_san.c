/* ASan/UBSan driver for the CPU oracle (oracle/polar_oracle.c, polar_channel_oracle.c):
 * random masks and LLRs (incl. -32, wrap-around and zero-heavy inputs) through the literal
 * FSM and the recursive restatement at every swept configuration and LLR width; the two
 * must agree. Built and run by tests/test_sanitize.py (sanitizers on the
 * CPU oracle). Exit 0 = clean and equal. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int orc_set_llr_bits(int q);
int orc_set_format(int q, int par, int ca2, int ext);
int orc_decode_fsm_cfg(int N, const uint8_t *mask, const int8_t *llr, uint8_t *xhat, int nframes,
                       long *state_counts, const int32_t *cfg7);
int orc_decode_rec_cfg(int N, const uint8_t *mask, const int8_t *llr, uint8_t *xhat, int nframes,
                       const int32_t *cfg7);
void orc_encode(int N, const uint8_t *u, uint8_t *x, int nframes);
void orc_csim_frames(uint32_t N, uint32_t seed8, uint64_t frame0, int nframes, float sigma, int beta,
                     int vsatn, int vsatp, const uint8_t *codewords, int ncw, int8_t *llr, uint8_t *xout);
void orc_count_errors(uint32_t N, int nframes, const uint8_t *xhat, const uint8_t *xref, uint64_t *counts);

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void)
{
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}

int main(void)
{
    static const int32_t cfgs[][7] = {
        {2, 1, 1, 1, 0, 0, 1}, {0, 1, 1, 1, 0, 0, 1}, {1, 1, 1, 1, 0, 0, 1}, {1, 1, 1, 1, 1, 1, 1},
        {2, 0, 0, 0, 0, 0, 0}, {2, 1, 0, 1, 0, 0, 0}, {1, 0, 1, 0, 1, 0, 1}, {2, 1, 1, 1, 1, 1, 0},
    };
    const int ncfg = (int)(sizeof cfgs / sizeof cfgs[0]);
    int bad = 0, runs = 0;
    for (int it = 0; it < 120; it++) {
        const int par = 2 << (rnd() % 6);                /* PAR 2 .. 64 */
        const int N = (2 * par > 32 ? 2 * par : 32) << (rnd() % 6);
        const int B = 1 + (int)(rnd() % 3);
        const int q = 5 + (int)(rnd() % 5);
        uint8_t *mask = malloc((size_t)N);
        int8_t *llr = malloc((size_t)N * B);
        uint8_t *x1 = malloc((size_t)N * B), *x2 = malloc((size_t)N * B);
        const uint32_t dens = rnd() % 4;
        for (int i = 0; i < N; i++) mask[i] = (uint8_t)((rnd() & 3u) <= dens);
        for (int i = 0; i < N * B; i++) {
            const uint32_t k = rnd() % 8;
            llr[i] = k == 0 ? (int8_t)-32 : k == 1 ? 0 : (int8_t)(rnd() & 0xFFu);
        }
        if (orc_set_format(q, par, (int)(rnd() & 1u), (int)(rnd() & 1u))) bad++;
        const int32_t *c = cfgs[rnd() % ncfg];
        long counts[16] = {0};
        int r1 = orc_decode_fsm_cfg(N, mask, llr, x1, B, counts, c);
        int r2 = orc_decode_rec_cfg(N, mask, llr, x2, B, c);
        runs++;
        if (r1 || r2 || memcmp(x1, x2, (size_t)N * B)) {
            fprintf(stderr, "mismatch N=%d B=%d q=%d rc=%d/%d\n", N, B, q, r1, r2);
            bad++;
        }
        free(mask); free(llr); free(x1); free(x2);
    }
    orc_set_format(6, 16, 0, 1);
    /* frame source + error counter */
    {
        const int N = 1024, B = 5;
        int8_t *llr = malloc((size_t)N * B);
        uint8_t *xs = malloc((size_t)N * B), *xh = malloc((size_t)N * B);
        orc_csim_frames(N, 0xF0, 12345, B, 0.75f, 4, -31, 31, NULL, 0, llr, xs);
        int32_t c[7] = {2, 1, 1, 1, 0, 0, 1};
        uint8_t *mask = calloc((size_t)N, 1);
        for (int i = N / 2; i < N; i++) mask[i] = 1;
        orc_decode_fsm_cfg(N, mask, llr, xh, B, NULL, c);
        uint64_t cnt[3] = {0, 0, 0};
        orc_count_errors(N, B, xh, xs, cnt);
        free(llr); free(xs); free(xh); free(mask);
    }
    /* error paths */
    if (orc_decode_fsm_cfg(48, NULL, NULL, NULL, 0, NULL, NULL) == 0) bad++;
    printf("oracle_san: %d decodes, %d mismatches\n", runs, bad);
    return bad ? 1 : 0;
}
