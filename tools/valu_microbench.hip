// VALU issue-cost microbenchmark for gfx950, timed in-kernel with the shader clock
// (s_memtime = shader cycles, MI355X_MICROARCH.md 'Per-instruction cycle constants') so that
// no clock has to be assumed. For each instruction class the decoder issues:
//   * throughput: cycles per wave64 instruction per SIMD at 1, 2, 4 and 8 waves per SIMD,
//     8 independent chains per wave (no dependency stalls);
//   * latency: one dependent chain, one wave per SIMD.
// Every wave stamps s_memtime around its loop; cycles per SIMD-instruction =
// median(wave delta) / (instructions per wave * waves per SIMD). The clock itself is
// reported as s_memtime ticks / s_memrealtime (100 MHz) ticks.
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_microbench.hip -o build_tools/valu_mb
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__device__ __forceinline__ void op(unsigned &r, unsigned k)
{
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 2) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 3) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 4) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x36" : "+v"(r) : "v"(k));
    if constexpr (OP == 5) asm volatile("v_mov_b32_dpp %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(r));
    if constexpr (OP == 6) asm volatile("v_add_u32_dpp %0, %0, %1 row_ror:8 row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(k));
    if constexpr (OP == 7) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 8) asm volatile("v_pk_ashrrev_i16 %0, 15, %0" : "+v"(r));
    if constexpr (OP == 9) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 10) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 11) asm volatile("v_pk_mad_u16 %0, %0, %1, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 12) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 13) asm volatile("v_xor_b32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r) : "v"(k));
    if constexpr (OP == 14) asm volatile("v_min3_u32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
    // encoding-size probes: the same simple op as VOP2 (4 B), VOP2 + literal (8 B), VOP2 with an
    // SGPR operand (4 B) and the VOP3 form (8 B); a 4 B / 8 B alternation
    if constexpr (OP == 15) asm volatile("v_and_b32_e32 %0, 0x7fff7fff, %0" : "+v"(r));
    if constexpr (OP == 16) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(r) : "s"(k));
    if constexpr (OP == 17) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 18) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(r) : "s"(k));
    if constexpr (OP == 19) asm volatile("v_add_u32 %0, %0, %1\n\tv_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 20) asm volatile("v_lshlrev_b32_e32 %0, 3, %0" : "+v"(r));
    if constexpr (OP == 21) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 22) asm volatile("v_add_u32 %0, %0, %1\n\tv_xor_b32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 23) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(r) : "v"(k));
    // which operand forms dual-issue (round 4): shift amount / constant in a VGPR vs inline,
    // VOP1, 16-bit VOP2, 3-source VOP3, SGPR masks, permlane
    if constexpr (OP == 24) asm volatile("v_lshlrev_b32_e32 %0, %1, %0" : "+v"(r) : "v"(k));
    if constexpr (OP == 25) asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(r) : "v"(k));
    if constexpr (OP == 26) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 27) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 28) asm volatile("v_lshrrev_b32_e32 %0, 16, %0" : "+v"(r));
    if constexpr (OP == 29) asm volatile("v_not_b32_e32 %0, %0" : "+v"(r));
    if constexpr (OP == 30) asm volatile("v_min_u32_e32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 31) asm volatile("v_min_u16_e32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 32) asm volatile("v_add_u16_e32 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 33) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[4:5]" : "+v"(r) : "v"(k));
    if constexpr (OP == 34) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 35) asm volatile("v_and_b32_e32 %0, 15, %0" : "+v"(r));
    if constexpr (OP == 36) asm volatile("v_xor_b32_e32 %0, 0x80008000, %0" : "+v"(r));
    if constexpr (OP == 37) asm volatile("v_add_u32_e32 %0, 5, %0" : "+v"(r));
    if constexpr (OP == 38) asm volatile("v_permlane16_swap_b32 %0, %0" : "+v"(r));
    if constexpr (OP == 39) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(r) : "v"(k));
    if constexpr (OP == 40) asm volatile("v_ashrrev_i32_e32 %0, %1, %0" : "+v"(r) : "v"(k));
    if constexpr (OP == 41) asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 42) asm volatile("v_sub_u32_e64 %0, %0, %1" : "+v"(r) : "v"(k));
    if constexpr (OP == 43) asm volatile("v_max_i16_e32 %0, %0, %1" : "+v"(r) : "v"(k));
}
static const char *names[] = {"v_add_u32", "v_xor_b32", "v_pk_add_u16", "v_pk_min_u16", "v_bitop3_b32",
                              "v_mov_b32_dpp row_ror", "v_add_u32_dpp row_ror", "v_and_or_b32",
                              "v_pk_ashrrev_i16", "v_add_f32", "v_fma_f32", "v_pk_mad_u16", "v_perm_b32",
                              "v_xor_b32_dpp quad_perm", "v_min3_u32", "v_and_b32_e32 literal (8 B)",
                              "v_and_b32_e32 sgpr (4 B)", "v_add_u32_e64 (VOP3, 8 B)", "v_pk_add_u16 sgpr",
                              "v_add_u32 + v_pk_add_u16 (pair)", "v_lshlrev_b32_e32 inline const",
                              "v_bfi_b32", "v_add_u32 + v_xor_b32 (pair)", "v_cndmask_b32_e32 vcc",
                              "v_lshlrev_b32_e32 vgpr shift", "v_and_b32_e32 vgpr", "v_or3_b32",
                              "v_sub_u32_e32 vgpr", "v_lshrrev_b32_e32 inline 16", "v_not_b32 (VOP1)",
                              "v_min_u32_e32", "v_min_u16_e32", "v_add_u16_e32", "v_cndmask_b32_e64 sgpr mask",
                              "v_lshl_or_b32", "v_and_b32_e32 inline 15", "v_xor_b32_e32 literal",
                              "v_add_u32_e32 inline 5", "v_permlane16_swap_b32", "v_mov_b32_e32 vgpr",
                              "v_ashrrev_i32_e32 vgpr", "v_pk_sub_u16", "v_sub_u32_e64 (VOP3)", "v_max_i16_e32"};
constexpr int NOPS = 44;

// CHAINS independent accumulators per wave; stamps[wave] = {memtime delta, memrealtime delta}
template <int OP, int CHAINS>
__global__ void __launch_bounds__(256) bench(unsigned *out, unsigned long long *stamps, int iters)
{
    unsigned r[8];
#pragma unroll
    for (int c = 0; c < 8; c++) r[c] = threadIdx.x * (2 * c + 3);
    const unsigned k = 0x01230123u;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
    // 64 instructions per loop iteration: the loop branch (an instruction-buffer refill for a
    // lone wave) stays below 2 % of the issue time
    for (int i = 0; i < iters; i += 8) {
#pragma unroll
        for (int rep = 0; rep < 64 / CHAINS; rep++) {
#pragma unroll
            for (int c = 0; c < CHAINS; c++) op<OP>(r[c], k);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
    unsigned x = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) x ^= r[c];
    out[blockIdx.x * 256 + threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        stamps[2 * w] = t1 - t0;
        stamps[2 * w + 1] = w1 - w0;
    }
}

template <int OP, int CHAINS>
void one(unsigned *buf, unsigned long long *st, int cus, int wps)
{
    const int iters = 2048, blocks = cus * wps;   // 256-thread blocks: one wave per SIMD each
    hipLaunchKernelGGL((bench<OP, CHAINS>), dim3(blocks), dim3(256), 0, 0, buf, st, iters);   // warm
    hipLaunchKernelGGL((bench<OP, CHAINS>), dim3(blocks), dim3(256), 0, 0, buf, st, iters);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * blocks * 4);
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> cyc, ghz;
    for (int w = 0; w < blocks * 4; w++) {
        cyc.push_back((double)h[2 * w]);
        ghz.push_back(h[2 * w + 1] ? (double)h[2 * w] / (double)h[2 * w + 1] / 10.0 : 0.0);
    }
    std::sort(cyc.begin(), cyc.end());
    std::sort(ghz.begin(), ghz.end());
    const double insts = 8.0 * iters;   // iters / 8 iterations x 64 instructions
    const double med = cyc[cyc.size() / 2];
    // CHAINS == 8: throughput per SIMD (waves share the SIMD); CHAINS == 1: dependent latency
    printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"cycles_per_wave_inst_per_simd\": %.3f, "
           "\"cycles_per_inst_in_wave\": %.3f, \"clock_ghz\": %.3f}\n",
           names[OP], CHAINS, wps, med / insts / wps, med / insts, ghz[ghz.size() / 2]);
}

template <int OP>
void all(unsigned *buf, unsigned long long *st, int cus, int from)
{
    if (OP >= from)
        for (int wps : {1, 2, 4, 8}) one<OP, 8>(buf, st, cus, wps);
    if (OP >= from) one<OP, 1>(buf, st, cus, 1);
    if constexpr (OP + 1 < NOPS) all<OP + 1>(buf, st, cus, from);
}

// usage: valu_mb [first op index]   (the encoding-size probes start at 15)
int main(int argc, char **argv)
{
    const int from = argc > 1 ? std::atoi(argv[1]) : 0;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    unsigned *buf;
    unsigned long long *st;
    hipMalloc(&buf, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&st, (size_t)cus * 8 * 4 * 2 * 8);
    all<0>(buf, st, cus, from);
    hipFree(buf);
    hipFree(st);
    return 0;
}
