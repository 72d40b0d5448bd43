/*
 * polar_decode_cli.c -- plain-C caller of libpolar_sc.so (include/polar_sc.h), the shape a
 * reference-side integration takes: load a frozen table in the reference's own format,
 * build a plan, decode a file of int8 LLR frames, write x^ words.
 *
 *   polar_decode_cli <table> <K|0> <llr.bin> <xhat.bin>    decode (needs a GPU)
 *   polar_decode_cli <table> <K|0> --stats                 plan census only (host)
 *
 * <table>: Frozen_Bit_Tab/FB_N{N}_K{K}.txt (K given) or Generated_Frozen_Bit/*.txt (K = 0).
 * llr.bin: [frames][N] int8; xhat.bin: [frames][ceil(N/64)] little-endian uint64.
 * build: gcc -O2 -Iinclude examples/polar_decode_cli.c -Lsc_polar_decoder_hls_amd/lib -lpolar_sc
 */
#include "polar_sc.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAX_N (1u << 20)

static int load_mask(const char *path, uint32_t K, uint8_t *mask, uint32_t *N)
{
    if (K > 0) return polar_load_frozen_tab(path, 0, K, mask, MAX_N, N);
    return polar_load_mask_file(path, mask, MAX_N, N);
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s <table> <K|0> <llr.bin> <xhat.bin> | --stats\n", argv[0]);
        return 2;
    }
    uint8_t *mask = (uint8_t *)malloc(MAX_N);
    uint32_t N = 0;
    int rc = load_mask(argv[1], (uint32_t)strtoul(argv[2], NULL, 10), mask, &N);
    if (rc) {
        fprintf(stderr, "table: %s\n", polar_sc_strerror(rc));
        return 1;
    }
    polar_sc_plan *plan = NULL;
    rc = polar_sc_plan_create(&plan, N, mask, NULL);
    if (rc) {
        fprintf(stderr, "plan: %s\n", polar_sc_strerror(rc));
        return 1;
    }
    polar_sc_plan_stats st;
    polar_sc_plan_get_stats(plan, &st);
    if (strcmp(argv[3], "--stats") == 0) {
        printf("N=%u K=%u groups=%u R0=%u R1=%u REP=%u SPC=%u RN=%u ops=%u storage=%u\n", st.N, st.K,
               st.groups, st.n_r0, st.n_r1, st.n_rep, st.n_spc, st.n_rn, st.n_ops, st.storage);
        polar_sc_plan_destroy(plan);
        free(mask);
        return 0;
    }
    if (argc < 5) return 2;
    FILE *f = fopen(argv[3], "rb");
    if (!f) return 1;
    fseek(f, 0, SEEK_END);
    long bytes = ftell(f);
    fseek(f, 0, SEEK_SET);
    size_t frames = (size_t)bytes / N;
    int8_t *llr = (int8_t *)malloc(frames * N + 1);
    if (fread(llr, 1, frames * N, f) != frames * N) return 1;
    fclose(f);
    size_t words = (N + 63) / 64;
    uint64_t *xhat = (uint64_t *)calloc(frames * words + 1, 8);
    rc = polar_sc_decode_host(plan, llr, xhat, frames);
    if (rc) {
        fprintf(stderr, "decode: %s\n", polar_sc_strerror(rc));
        return 1;
    }
    f = fopen(argv[4], "wb");
    if (!f) return 1;
    fwrite(xhat, 8, frames * words, f);
    fclose(f);
    printf("decoded %zu frames, N=%u K=%u\n", frames, st.N, st.K);
    polar_sc_plan_destroy(plan);
    free(llr);
    free(xhat);
    free(mask);
    return 0;
}
