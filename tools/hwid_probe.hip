// Where do the waves of co-resident workgroups land? Records HW_REG_HW_ID (SIMD, CU, SE,
// TG slot) for every wave of a 512-block grid with ~78 KB of LDS per block (two blocks per
// CU, the C3 hybrid kernel's shape), to check whether the lead waves chosen by
// blockIdx & (wpg - 1) of two blocks on one CU share a SIMD.
// build: hipcc --offload-arch=gfx950 -O3 tools/hwid_probe.hip -o build_tools/hwid_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) probe(unsigned *out, int spin)
{
    extern __shared__ unsigned lds[];
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * 4 + w)] = hw;
    lds[threadIdx.x] = hw;
    // keep the blocks resident together for a while
    unsigned long long t0 = __builtin_readcyclecounter();
    while (__builtin_readcyclecounter() - t0 < (unsigned long long)spin) { }
    __syncthreads();
    if (threadIdx.x == 0) lds[1000] = lds[5];
}

int main()
{
    const int blocks = 512;
    unsigned *d;
    hipMalloc(&d, blocks * 4 * 4);
    const size_t lds = 79744;
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), lds, 0, d, 200000);
    hipDeviceSynchronize();
    std::vector<unsigned> h(blocks * 4);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    for (int b = 0; b < blocks; b++)
        for (int w = 0; w < 4; w++) printf("%d %d 0x%08x\n", b, w, h[b * 4 + w]);
    return 0;
}
