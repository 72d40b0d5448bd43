// polar_sc_channel.hip -- the reference's C-sim frame chain and error counter on the GPU
// (the decoder's input generator and its BER/FER accounting).
//
// Chain per frame f (src/testbench/sc_top_module.h:101-160): encoder (codeword f % ncw of
// a fixed table, sc_encoder.h:91-122) -> BPSK (bit 1 -> -1, sc_bpsk.h:53) -> two
// xorshift128 streams (sc_xorshift128.h:56-125) -> Box-Muller (sc_awgn.h:60-89: x sin, then
// x cos) -> adder (v = bpsk + noise * sigma, sc_adder.h:135-154) -> quantizer
// ((short)(v * beta) clamped, sc_quantizer.h:69-81). The streams are sequential in the
// reference; here every frame starts from its own stream state, obtained on the host by
// GF(2) jump-ahead (xorshift128 is linear: state_f = T^(f N/2) state_0), so frames are
// generated in parallel, one thread per frame.
//
// Float results follow the reference's operation order with contraction off; logf / sinf /
// cosf are glibc's own algorithms (polar_sc_glibcf.h, checked bit for bit against the host's
// glibc over their whole input domain here), so the LLRs equal the x86 C-sim's exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "polar_sc_glibcf.h"

#include <cerrno>
#include <cstring>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------
// xorshift128 over GF(2): the 128-bit state as 4 words; a linear map as its 128 columns
// ---------------------------------------------------------------------------------------
struct S128 {
    uint32_t v[4];
};
struct M128 {
    S128 col[128];   // col[j] = image of basis vector j (word j / 32, bit j % 32)
};

inline void xs_step(S128 &s)
{
    uint32_t t = s.v[0];
    t ^= t << 11;
    t ^= t >> 8;
    s.v[0] = s.v[1];
    s.v[1] = s.v[2];
    s.v[2] = s.v[3];
    s.v[3] ^= s.v[3] >> 19;
    s.v[3] ^= t;
}

inline S128 apply(const M128 &m, const S128 &s)
{
    S128 r{{0, 0, 0, 0}};
    for (int j = 0; j < 128; j++) {
        if ((s.v[j >> 5] >> (j & 31)) & 1u) {
            for (int w = 0; w < 4; w++) r.v[w] ^= m.col[j].v[w];
        }
    }
    return r;
}

inline M128 mul(const M128 &a, const M128 &b)   // a * b (apply b first)
{
    M128 r;
    for (int j = 0; j < 128; j++) r.col[j] = apply(a, b.col[j]);
    return r;
}

M128 step_matrix()
{
    M128 m;
    for (int j = 0; j < 128; j++) {
        S128 e{{0, 0, 0, 0}};
        e.v[j >> 5] = 1u << (j & 31);
        xs_step(e);
        m.col[j] = e;
    }
    return m;
}

M128 identity()
{
    M128 m;
    for (int j = 0; j < 128; j++) {
        S128 e{{0, 0, 0, 0}};
        e.v[j >> 5] = 1u << (j & 31);
        m.col[j] = e;
    }
    return m;
}

M128 power(M128 base, uint64_t e)
{
    M128 r = identity();
    while (e) {
        if (e & 1u) r = mul(base, r);
        e >>= 1;
        if (e) base = mul(base, base);
    }
    return r;
}

void seed_streams(uint32_t seed8, S128 s[2])
{
    const uint32_t m = (seed8 & 0xFFu) * 0x01010101u;   // (mask, mask, mask, mask)
    s[0] = S128{{0x12311178u & m, 0x65498732u | m, 0xFEDCAA01u ^ m, 0xF489A179u + m}};
    s[1] = S128{{0x98765432u & m, 0x12345678u | m, 0xFCBADEFFu ^ m, 0x12121212u + m}};
}

// per-frame stream states: out[f][0..3] stream 1, out[f][4..7] stream 2
void frame_states(uint32_t N, uint32_t seed8, uint64_t frame0, size_t batch, uint32_t *out)
{
    S128 s[2];
    seed_streams(seed8, s);
    const M128 T = step_matrix();
    const M128 J = power(T, N / 2);          // one frame: N/2 draws of each stream
    if (frame0) {
        const M128 Jf = power(J, frame0);
        s[0] = apply(Jf, s[0]);
        s[1] = apply(Jf, s[1]);
    }
    for (size_t f = 0; f < batch; f++) {
        std::memcpy(out + f * 8, s[0].v, 16);
        std::memcpy(out + f * 8 + 4, s[1].v, 16);
        s[0] = apply(J, s[0]);
        s[1] = apply(J, s[1]);
    }
}

// ---------------------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xs_next(uint32_t &x, uint32_t &y, uint32_t &z, uint32_t &w)
{
    uint32_t t = x;
    t ^= t << 11;
    t ^= t >> 8;
    x = y;
    y = z;
    z = w;
    w ^= w >> 19;
    w ^= t;
    return w;
}

// (short)(float) of the reference on x86-64: 32-bit truncating conversion (out of range ->
// 0x80000000), then the low 16 bits
__device__ __forceinline__ int to_short(float v)
{
    const int32_t i = (v > -2147483648.0f && v < 2147483648.0f) ? (int32_t)v : (int32_t)0x80000000u;
    return (int)(int16_t)(uint16_t)(uint32_t)i;
}

__global__ void __launch_bounds__(256) csim_kernel(const uint32_t *__restrict__ states, const uint8_t *__restrict__ cw,
                                                  int ncw, uint64_t frame0, uint32_t N, long batch, float sigma,
                                                  float beta, int vsatn, int vsatp, int8_t *__restrict__ llr,
                                                  uint64_t *__restrict__ xref)
{
#pragma clang fp contract(off)
    const long f = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= batch) return;
    uint32_t a0 = states[f * 8 + 0], a1 = states[f * 8 + 1], a2 = states[f * 8 + 2], a3 = states[f * 8 + 3];
    uint32_t b0 = states[f * 8 + 4], b1 = states[f * 8 + 5], b2 = states[f * 8 + 6], b3 = states[f * 8 + 7];
    const uint8_t *c = ncw > 0 ? cw + (size_t)((frame0 + (uint64_t)f) % (uint64_t)ncw) * N : nullptr;
    const float PI2 = 2.0f * 3.14159265358979f;
    int8_t *row = llr + (size_t)f * N;
    uint64_t *xr = xref ? xref + (size_t)f * ((N + 63) / 64) : nullptr;
    for (uint32_t base = 0; base < N; base += 16) {
        uint32_t pk[4] = {0, 0, 0, 0};
        uint32_t bits = 0;
        for (uint32_t k = 0; k < 8; k++) {
            const float r1 = 1.0f - (float)xs_next(a0, a1, a2, a3) * (1.0f / 4294967296.0f);
            const float y = PI2 * (1.0f - (float)xs_next(b0, b1, b2, b3) * (1.0f / 4294967296.0f));
            const float x = sqrtf(-2.0f * glibcf::logf(r1));
            const float noise[2] = {x * glibcf::sinf(y), x * glibcf::cosf(y)};
            for (int h = 0; h < 2; h++) {
                const uint32_t i = base + 2 * k + (uint32_t)h;
                const uint32_t bit = c ? (c[i] & 1u) : 0u;
                const float o = bit ? -1.0f : 1.0f;
                const float n = noise[h] * sigma;
                const float v = o + n;
                int q = to_short(v * beta);
                q = q > vsatn ? q : vsatn;
                q = q < vsatp ? q : vsatp;
                const uint32_t j = 2 * k + (uint32_t)h;
                pk[j >> 2] |= ((uint32_t)q & 0xFFu) << (8 * (j & 3));
                bits |= bit << j;
            }
        }
        *(uint4 *)(row + base) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        if (xr) ((uint16_t *)xr)[base / 16] = (uint16_t)bits;
    }
    if (xr && (N % 64) != 0) ((uint16_t *)xr)[N / 16] = 0, ((uint16_t *)xr)[N / 16 + 1] = 0;
}

// sc_error_counter (sc_error_counter.h:50-126) over packed codewords; counts[0] += per-frame
// errors mod 1024 (sc_uint<10>), counts[1] += frames with a non-zero wrapped count,
// counts[2] += exact bit errors
__global__ void __launch_bounds__(256) count_errors_kernel(const uint64_t *__restrict__ xhat,
                                                          const uint64_t *__restrict__ xref, int words, long batch,
                                                          unsigned long long *__restrict__ counts)
{
    const long f = (long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long e = 0;
    if (f < batch) {
        for (int j = 0; j < words; j++) e += (unsigned long long)__popcll(xhat[f * words + j] ^ xref[f * words + j]);
    }
    unsigned long long w = e & 1023u, fe = (e & 1023u) != 0u;
    // wave reduction, one atomic per wave and counter
    for (int off = 32; off > 0; off >>= 1) {
        w += __shfl_down(w, off);
        fe += __shfl_down(fe, off);
        e += __shfl_down(e, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&counts[0], w);
        atomicAdd(&counts[1], fe);
        atomicAdd(&counts[2], e);
    }
}

}  // namespace

extern "C" {

int polar_csim_states(uint32_t N, uint32_t seed8, uint64_t frame0, size_t batch, uint32_t *states)
{
    if (N < 32 || (N & (N - 1)) || (batch > 0 && !states)) return -EINVAL;
    frame_states(N, seed8, frame0, batch, states);
    return 0;
}

int polar_csim_frames(uint32_t N, uint32_t seed8, uint64_t frame0, size_t batch, float sigma, int beta, int vsatn,
                      int vsatp, const uint8_t *codewords, uint32_t ncw, int8_t *llr_dev, uint64_t *xref_dev,
                      void *stream)
{
    if (N < 32 || (N & (N - 1)) || (batch > 0 && !llr_dev) || (ncw > 0 && !codewords)) return -EINVAL;
    if (batch == 0) return 0;
    if (((uintptr_t)llr_dev & 15u) != 0u) return -EINVAL;   // 16-byte row stores
    hipStream_t s = (hipStream_t)stream;
    std::vector<uint32_t> st(batch * 8);
    frame_states(N, seed8, frame0, batch, st.data());
    uint32_t *d_st = nullptr;
    uint8_t *d_cw = nullptr;
    if (hipMallocAsync((void **)&d_st, st.size() * 4, s) != hipSuccess) return -ENOMEM;
    if (hipMemcpyAsync(d_st, st.data(), st.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;
    if (ncw > 0) {
        if (hipMallocAsync((void **)&d_cw, (size_t)ncw * N, s) != hipSuccess) return -ENOMEM;
        if (hipMemcpyAsync(d_cw, codewords, (size_t)ncw * N, hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;
    }
    const unsigned blocks = (unsigned)((batch + 255) / 256);
    hipLaunchKernelGGL(csim_kernel, dim3(blocks), dim3(256), 0, s, d_st, d_cw, (int)ncw, frame0, N, (long)batch,
                       sigma, (float)beta, vsatn, vsatp, llr_dev, xref_dev);
    hipError_t e = hipGetLastError();
    (void)hipFreeAsync(d_st, s);
    if (d_cw) (void)hipFreeAsync(d_cw, s);
    // the host copy of the states must outlive the async upload
    if (hipStreamSynchronize(s) != hipSuccess) return -EIO;
    return e == hipSuccess ? 0 : -EIO;
}

int polar_count_errors(const uint64_t *xhat_dev, const uint64_t *xref_dev, uint32_t N, size_t batch,
                       unsigned long long *counts_dev, void *stream)
{
    if (N < 32 || (batch > 0 && (!xhat_dev || !xref_dev || !counts_dev))) return -EINVAL;
    if (batch == 0) return 0;
    const unsigned blocks = (unsigned)((batch + 255) / 256);
    hipLaunchKernelGGL(count_errors_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, xhat_dev, xref_dev,
                       (int)((N + 63) / 64), (long)batch, counts_dev);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

}  // extern "C"
