// polar_sc_kernels.hip -- CDNA4 (gfx950) batched SC polar decoder: the generic schedule
// interpreter kernels (polar_sc_interp.h) and their launch glue. Plans with N <= 1024 and
// hybrid plans run generated per-mask code instead (polar_sc_jit.cpp).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "polar_sc_interp.h"

namespace polar {

template <bool GMEM>
__global__ void __launch_bounds__(1024) polar_sc_decode_kernel(
    const int8_t *__restrict__ llr, uint16_t *__restrict__ out, const Op *__restrict__ ops,
    uint32_t *__restrict__ scratch, int N, int batch, int out_stride, int wpg, int gpb,
    int group_dwords, int lds_dwords, int lds0)
{
    decode_body<GMEM>(llr, out, ops, scratch, N, batch, out_stride, wpg, gpb, group_dwords, lds_dwords, lds0);
}

// the same with the per-op monitor (polar_sc_trace)
template <bool GMEM>
__global__ void __launch_bounds__(1024) polar_sc_decode_trace_kernel(
    const int8_t *__restrict__ llr, uint16_t *__restrict__ out, const Op *__restrict__ ops,
    uint32_t *__restrict__ scratch, int N, int batch, int out_stride, int wpg, int gpb,
    int group_dwords, int lds_dwords, int lds0, unsigned long long *__restrict__ trace)
{
    decode_body<GMEM, true>(llr, out, ops, scratch, N, batch, out_stride, wpg, gpb, group_dwords, lds_dwords,
                            lds0, trace);
}

// cross-lane self-test: out[h*64 + lane] = lane id seen through xorlane<1<<h> (h = 0..3), then
// the two results of v_permlane16_swap (rows 4, 5) and v_permlane32_swap (rows 6, 7) of the
// lane id with itself (the frame-pair layout's cross-row steps, polar_sc_pair.h)
__global__ void polar_sc_lane_selftest_kernel(uint32_t *out)
{
    uint32_t l = threadIdx.x;
    out[0 * 64 + l] = xorlane<1>(l);
    out[1 * 64 + l] = xorlane<2>(l);
    out[2 * 64 + l] = xorlane<4>(l);
    out[3 * 64 + l] = xorlane<8>(l);
    const auto p16 = __builtin_amdgcn_permlane16_swap(l, l, false, false);
    const auto p32 = __builtin_amdgcn_permlane32_swap(l, l, false, false);
    out[4 * 64 + l] = p16[0];
    out[5 * 64 + l] = p16[1];
    out[6 * 64 + l] = p32[0];
    out[7 * 64 + l] = p32[1];
}

}  // namespace polar

// ---------------------------------------------------------------------------------------
// launch glue (called from polar_sc_host.cpp)
// ---------------------------------------------------------------------------------------
extern "C" int polar_sc_launch_decode(int gmem, const int8_t *llr, uint16_t *out, const void *ops,
                                      uint32_t *scratch, int N, long batch, int out_stride,
                                      int waves_per_group, int groups_per_block, int group_dwords,
                                      int lds_dwords, int lds0, void *stream, unsigned long long *trace)
{
    const long groups = (batch + 7) / 8;
    const long blocks = (groups + groups_per_block - 1) / groups_per_block;
    dim3 grid((unsigned)blocks), block((unsigned)(64 * waves_per_group * groups_per_block));
    hipStream_t s = (hipStream_t)stream;
    const polar::Op *o = (const polar::Op *)ops;
    const size_t lds = (size_t)groups_per_block * (size_t)lds_dwords * 4u;
    const void *fn = trace ? (gmem ? (const void *)polar::polar_sc_decode_trace_kernel<true>
                                   : (const void *)polar::polar_sc_decode_trace_kernel<false>)
                           : (gmem ? (const void *)polar::polar_sc_decode_kernel<true>
                                   : (const void *)polar::polar_sc_decode_kernel<false>);
    if (lds > 65536) {
        hipError_t ae = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (ae != hipSuccess) return -(int)ae - 1000;
    }
    if (trace) {
        if (gmem)
            hipLaunchKernelGGL(polar::polar_sc_decode_trace_kernel<true>, grid, block, lds, s, llr, out, o, scratch,
                               N, (int)batch, out_stride, waves_per_group, groups_per_block, group_dwords,
                               lds_dwords, lds0, trace);
        else
            hipLaunchKernelGGL(polar::polar_sc_decode_trace_kernel<false>, grid, block, lds, s, llr, out, o, scratch,
                               N, (int)batch, out_stride, waves_per_group, groups_per_block, group_dwords,
                               lds_dwords, lds0, trace);
    } else if (gmem) {
        hipLaunchKernelGGL(polar::polar_sc_decode_kernel<true>, grid, block, lds, s, llr, out, o, scratch, N,
                           (int)batch, out_stride, waves_per_group, groups_per_block, group_dwords, lds_dwords,
                           lds0);
    } else {
        hipLaunchKernelGGL(polar::polar_sc_decode_kernel<false>, grid, block, lds, s, llr, out, o, scratch, N,
                           (int)batch, out_stride, waves_per_group, groups_per_block, group_dwords, lds_dwords,
                           lds0);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -(int)e - 1000;
}

namespace polar {
// int8 channel -> int16 (sign extension), for plans whose generated kernel reads the int16
// channel (pair plans of 9-bit LLRs, 16-bit stage slots) decoded through the int8 entry point
__global__ void __launch_bounds__(256) polar_widen_kernel(const int8_t *__restrict__ in, int16_t *__restrict__ out,
                                                          size_t n)
{
    // (byte loads: the int8 frames need not be 4-byte aligned)
    const size_t i = ((size_t)blockIdx.x * 256u + threadIdx.x) * 4u;
    for (size_t k = i; k < i + 4u && k < n; k++) out[k] = in[k];
}

}  // namespace polar

extern "C" int polar_sc_launch_widen(const int8_t *in_dev, int16_t *out_dev, size_t n, void *stream)
{
    if (n == 0) return 0;
    const size_t blocks = (n + 1023u) / 1024u;
    hipLaunchKernelGGL(polar::polar_widen_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in_dev,
                       out_dev, n);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : -(int)e - 1000;
}


extern "C" int polar_sc_launch_selftest(uint32_t *out_dev)
{
    hipLaunchKernelGGL(polar::polar_sc_lane_selftest_kernel, dim3(1), dim3(64), 0, 0, out_dev);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return -(int)e - 1000;
    e = hipDeviceSynchronize();
    return e == hipSuccess ? 0 : -(int)e - 1000;
}
