// VALU issue-cost microbenchmark for gfx950: throughput (cycles per wave-instruction per
// SIMD) of the instruction classes the decode kernels use, with 8 waves per SIMD and 8
// independent chains per wave (no dependency stalls).
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_microbench.hip -o /tmp/valu_mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void __launch_bounds__(256) bench(unsigned *out, int iters)
{
    unsigned r0 = threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11, r5 = r0 * 13, r6 = r0 * 17,
             r7 = r0 * 19, k = 0x01230123u;
    for (int i = 0; i < iters; i++) {
#define OPX(n)                                                                                            \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r##n) : "v"(k));                 \
    if constexpr (OP == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r##n) : "v"(k));                 \
    if constexpr (OP == 2) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r##n) : "v"(k));              \
    if constexpr (OP == 3) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(r##n) : "v"(k));              \
    if constexpr (OP == 4) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x36" : "+v"(r##n) : "v"(k)); \
    if constexpr (OP == 5) asm volatile("v_mov_b32_dpp %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(r##n)); \
    if constexpr (OP == 6) asm volatile("v_add_u32_dpp %0, %0, %1 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(r##n) : "v"(k)); \
    if constexpr (OP == 7) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(r##n) : "v"(k));          \
    if constexpr (OP == 8) asm volatile("v_pk_ashrrev_i16 %0, 15, %0" : "+v"(r##n));                    \
    if constexpr (OP == 9) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r##n) : "v"(k));                 \
    if constexpr (OP == 10) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(r##n));                       \
    if constexpr (OP == 11) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(r##n) : "v"(k));             \
    if constexpr (OP == 12) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r##n)); \
    if constexpr (OP == 13) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double *)&r##n) : "v"(*(double *)&k)); \
    if constexpr (OP == 14) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r##n) : "v"(k));            \
    if constexpr (OP == 15) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r##n) : "v"(k));       \
    if constexpr (OP == 16) asm volatile("v_pk_mad_u16 %0, %0, %1, %1" : "+v"(r##n) : "v"(k));          \
    if constexpr (OP == 17) asm volatile("v_min_u32 %0, %0, %1" : "+v"(r##n) : "v"(k));                 \
    if constexpr (OP == 18) asm volatile("v_xor_b32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r##n) : "v"(k)); \
    if constexpr (OP == 19) asm volatile("v_min3_u32 %0, %0, %1, %1" : "+v"(r##n) : "v"(k));
        REP8(OPX)
    }
    out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}

static const char *names[] = {"v_add_u32", "v_xor_b32", "v_pk_add_u16", "v_pk_min_u16", "v_bitop3_b32",
                              "v_mov_b32_dpp row_ror", "v_add_u32_dpp", "v_and_or_b32", "v_pk_ashrrev_i16",
                              "v_add_f32", "v_lshlrev_b32", "v_bfi_b32", "v_mov_b32_dpp quad_perm", "v_pk_add_f32",
                              "v_perm_b32", "v_cndmask_b32", "v_pk_mad_u16", "v_min_u32", "v_xor_b32_dpp",
                              "v_min3_u32"};

template <int OP>
double run(unsigned *buf, int blocks, int iters)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    bench<OP><<<blocks, 256>>>(buf, iters);
    hipEventRecord(a);
    bench<OP><<<blocks, 256>>>(buf, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

template <int OP>
void one(unsigned *buf, int cus, double ghz)
{
    const int waves_per_simd = 8, iters = 4096;
    const int blocks = cus * waves_per_simd;   // 4 waves per block -> one per SIMD
    double ms = run<OP>(buf, blocks, iters);
    double insts_per_simd = (double)waves_per_simd * iters * 8;
    double cyc = ms * 1e-3 * ghz * 1e9 / insts_per_simd;
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"cycles_per_wave_inst\": %.3f}\n", names[OP], ms, cyc);
}

int main(int argc, char **argv)
{
    double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    unsigned *buf;
    hipMalloc(&buf, (size_t)prop.multiProcessorCount * 8 * 256 * 4);
    one<0>(buf, prop.multiProcessorCount, ghz);
    one<1>(buf, prop.multiProcessorCount, ghz);
    one<2>(buf, prop.multiProcessorCount, ghz);
    one<3>(buf, prop.multiProcessorCount, ghz);
    one<4>(buf, prop.multiProcessorCount, ghz);
    one<5>(buf, prop.multiProcessorCount, ghz);
    one<6>(buf, prop.multiProcessorCount, ghz);
    one<7>(buf, prop.multiProcessorCount, ghz);
    one<8>(buf, prop.multiProcessorCount, ghz);
    one<9>(buf, prop.multiProcessorCount, ghz);
    one<10>(buf, prop.multiProcessorCount, ghz);
    one<11>(buf, prop.multiProcessorCount, ghz);
    one<12>(buf, prop.multiProcessorCount, ghz);
    one<13>(buf, prop.multiProcessorCount, ghz);
    one<14>(buf, prop.multiProcessorCount, ghz);
    one<15>(buf, prop.multiProcessorCount, ghz);
    one<16>(buf, prop.multiProcessorCount, ghz);
    one<17>(buf, prop.multiProcessorCount, ghz);
    one<18>(buf, prop.multiProcessorCount, ghz);
    one<19>(buf, prop.multiProcessorCount, ghz);
    hipFree(buf);
    return 0;
}
