/* ASan/UBSan driver for the host half of libpolar_sc.so (polar_sc_host.cpp schedule
 * compiler / plans / loaders, polar_sc_jit.cpp source generators, polar_sc_tables.cpp
 * frozen-table tooling), linked against a sanitized build of the library. Only host-side
 * entry points are called: no GPU is needed. Built and run by tests/test_sanitize.py
 * (SURVEY.md 5). argv[1] = a Frozen_Bit_Tab file, argv[2] = a Generated_Frozen_Bit file. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "polar_sc.h"

static uint64_t rs = 0xD1B54A32D192ED03ull;
static uint32_t rnd(void)
{
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

static int exercise_plan(uint32_t N, const uint8_t *mask, const polar_sc_config *cfg)
{
    polar_sc_plan *p = NULL;
    int rc = polar_sc_plan_create(&p, N, mask, cfg);
    if (rc == -95) return 0;   /* ENOTSUP config */
    CHECK(rc == 0 && p);
    polar_sc_plan_stats st;
    CHECK(polar_sc_plan_get_stats(p, &st) == 0 && st.N == N);
    uint32_t n = 0;
    CHECK(polar_sc_plan_get_schedule(p, NULL, 0, &n) == 0 && n == st.n_ops);
    polar_sc_op *ops = malloc(sizeof(polar_sc_op) * n);
    CHECK(polar_sc_plan_get_schedule(p, ops, n, &n) == 0);
    CHECK(ops[n - 1].code == POLAR_OP_END);
    free(ops);
    size_t len = 0;
    rc = polar_sc_plan_kernel_source(p, NULL, 0, &len);
    if (rc == 0) {
        char *buf = malloc(len + 1);
        CHECK(polar_sc_plan_kernel_source(p, buf, len + 1, &len) == 0 && strlen(buf) == len);
        char small[17];
        CHECK(polar_sc_plan_kernel_source(p, small, sizeof small, &len) == 0 && strlen(small) == 16);
        free(buf);
    }
    /* codeword -> info on a noiseless codeword: x = 0 -> u = 0 */
    const size_t words = (N + 63) / 64;
    uint64_t *x = calloc(words * 2, 8);
    uint8_t *info = malloc((size_t)st.K * 2 + 1);
    CHECK(polar_codeword_to_info(p, x, info, 2) == 0);
    for (uint32_t i = 0; i < st.K * 2; i++) CHECK(info[i] == 0);
    free(x); free(info);
    CHECK(polar_sc_plan_destroy(p) == 0);
    return 0;
}

int main(int argc, char **argv)
{
    polar_sc_config cfg;
    CHECK(polar_sc_default_config(&cfg) == 0);
    /* random masks at every size the plans distinguish (per-mask, hybrid, HBM scratch) */
    for (int it = 0; it < 60; it++) {
        const uint32_t N = 32u << (rnd() % 10);   /* 32 .. 16384 */
        uint8_t *mask = malloc(N);
        const uint32_t dens = rnd() % 4;
        for (uint32_t i = 0; i < N; i++) mask[i] = (uint8_t)((rnd() & 3u) <= dens);
        polar_sc_config c = cfg;
        c.pruning_level = (int32_t)(rnd() % 3);
        c.elag_rep2 = (int32_t)(rnd() & 1u);
        c.elag_spc2 = (int32_t)(rnd() & 1u);
        c.llr_bits = 5 + (int32_t)(rnd() % 4);
        if (exercise_plan(N, mask, it & 1 ? &c : NULL)) return 1;
        free(mask);
    }
    /* argument validation */
    polar_sc_plan *p = NULL;
    uint8_t m[64] = {0};
    CHECK(polar_sc_plan_create(&p, 48, m, NULL) == -22);
    CHECK(polar_sc_plan_create(&p, 16, m, NULL) == -22);
    CHECK(polar_sc_plan_create(NULL, 64, m, NULL) == -22);
    polar_sc_config bad = cfg;
    bad.elag_rare = 1;
    CHECK(polar_sc_plan_create(&p, 64, m, &bad) == -95);
    CHECK(polar_sc_strerror(-95) != NULL && polar_sc_strerror(12345) != NULL);
    /* loaders */
    uint8_t *mask = malloc(1u << 20);
    uint32_t N = 0;
    if (argc > 2) {
        CHECK(polar_load_frozen_tab(argv[1], 0, 64, mask, 1u << 20, &N) == 0 && N > 0);
        CHECK(polar_load_frozen_tab(argv[1], 0, 64, mask, 4, &N) == -22);   /* capacity */
        CHECK(polar_load_mask_file(argv[2], mask, 1u << 20, &N) == 0 && N > 0);
        CHECK(polar_load_mask_file(argv[2], mask, 8, &N) == -22);
        if (exercise_plan(N, mask, NULL)) return 1;
    }
    CHECK(polar_load_mask_file("/nonexistent/file", mask, 16, &N) == -2);
    /* frozen-table tooling: order -> mask -> FB table text / polar_parameters.h -> parse */
    {
        const uint32_t NN = 256, K = 100;
        uint32_t order[300];
        for (uint32_t i = 0; i < 300; i++) order[i] = (i * 167u + 13u) % 300u;
        CHECK(polar_mask_from_order(order, 300, NN, K, mask, NN) == 0);
        size_t len = 0;
        CHECK(polar_write_frozen_tab(order, 300, NN, NULL, 0, &len) == 0);
        char *buf = malloc(len + 1);
        CHECK(polar_write_frozen_tab(order, 300, NN, buf, len + 1, &len) == 0);
        free(buf);
        for (int concat = 0; concat < 2; concat++) {
            for (uint32_t par = 4; par <= 64; par *= 2) {
                CHECK(polar_write_parameters_h(mask, NN, par, concat, NULL, 0, &len) == 0);
                buf = malloc(len + 1);
                CHECK(polar_write_parameters_h(mask, NN, par, concat, buf, len + 1, &len) == 0);
                char path[] = "/tmp/host_san_paramsXXXXXX";
                int fd = mkstemp(path);
                CHECK(fd >= 0);
                FILE *f = fdopen(fd, "w");
                fwrite(buf, 1, len, f);
                fclose(f);
                uint8_t *back = malloc(NN);
                uint32_t n2 = 0, par2 = 0;
                CHECK(polar_parse_parameters_h(path, back, NN, &n2, &par2) == 0);
                CHECK(n2 == NN && par2 == par && memcmp(back, mask, NN) == 0);
                remove(path);
                free(back);
                free(buf);
            }
        }
    }
    /* the testbench's xorshift jump-ahead (host) */
    {
        uint32_t *states = malloc(8 * 4 * 33);
        CHECK(polar_csim_states(1024, 0xF0, 1000, 33, states) == 0);
        free(states);
    }
    free(mask);
    printf("host_san: ok\n");
    return 0;
}
