// polar_sc_glibcf.h -- logf, sinf and cosf exactly as the reference's C-sim computes them.
//
// The reference chain draws its noise with glibc's single-precision logf / sinf / cosf
// (src/testbench/sc_channel/sc_awgn/sc_awgn.h:69-76). glibc 2.35 on x86-64 implements them
// in double precision (the algorithms of sysdeps/ieee754/flt-32/e_logf.c and s_sinf.c /
// s_cosf.c, with the tables of e_logf_data.c and s_sincosf_data.c) and, on CPUs with FMA
// (every AMD EPYC / Intel Xeon host of this pool), dispatches to the -mfma build of those
// files. This header restates that build operation for operation: every multiply-add the
// FMA build fuses is an explicit fma() here, every other operation is a plain IEEE double
// operation, and the final conversion rounds to float once. The restatement is checked bit
// for bit against the host's glibc over every float input of the domain the frame chain
// uses (tests/test_channel.py builds and runs tools/glibcf_check.cpp), and the device frame
// generator (polar_sc_channel.hip) calls it, so its LLRs equal the C-sim's.
//
// Domain handled: logf on [0, +inf] (0 -> -inf, 1 -> 0, subnormals scaled), sinf / cosf on
// |y| < 120 (the chain uses 0 <= y <= 2 pi); outside it the functions return NaN.
#pragma once

#ifdef __HIPCC__
#define GLIBCF_FN __host__ __device__ __forceinline__
#define GLIBCF_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#include <math.h>
#define GLIBCF_FN static inline
#define GLIBCF_FMA(a, b, c) fma((a), (b), (c))
#endif
#include <stdint.h>

// no multiply-add contraction beyond the explicit fma() calls (clang / hipcc; the host check
// builds with -ffp-contract=off)
#if defined(__clang__)
#define GLIBCF_EXACT _Pragma("clang fp contract(off)")
#else
#define GLIBCF_EXACT
#endif

namespace glibcf {

GLIBCF_FN uint32_t fbits(float f)
{
    union { float f; uint32_t u; } v;
    v.f = f;
    return v.u;
}
GLIBCF_FN float fromfbits(uint32_t u)
{
    union { float f; uint32_t u; } v;
    v.u = u;
    return v.f;
}
GLIBCF_FN double dbl(uint64_t u)
{
    union { double d; uint64_t u; } v;
    v.u = u;
    return v.d;
}

// e_logf.c: x = 2^k z, z in [0x1.66p-1, 0x1.66p0) split into 16 subintervals; log(x) =
// k ln2 + log(c) + log1p(z/c - 1) with a degree-3 polynomial (e_logf_data.c: invc, logc,
// ln2, A[3]). FMA build: r = fma(z, invc, -1), y0 = fma(k, ln2, logc), y = fma(r, A1, A2),
// y = fma(r2, A0, y), result = fma(r2, y, r + y0).
GLIBCF_FN float logf(float x)
{
    GLIBCF_EXACT
    // {invc, logc} of the 16 subintervals, as double bit patterns
    const uint64_t T[16][2] = {
        {0x3ff661ec79f8f3beull, 0xbfd57bf7808caadeull}, {0x3ff571ed4aaf883dull, 0xbfd2bef0a7c06ddbull},
        {0x3ff49539f0f010b0ull, 0xbfd01eae7f513a67ull}, {0x3ff3c995b0b80385ull, 0xbfcb31d8a68224e9ull},
        {0x3ff30d190c8864a5ull, 0xbfc6574f0ac07758ull}, {0x3ff25e227b0b8ea0ull, 0xbfc1aa2bc79c8100ull},
        {0x3ff1bb4a4a1a343full, 0xbfba4e76ce8c0e5eull}, {0x3ff12358f08ae5baull, 0xbfb1973c5a611cccull},
        {0x3ff0953f419900a7ull, 0xbfa252f438e10c1eull}, {0x3ff0000000000000ull, 0x0000000000000000ull},
        {0x3fee608cfd9a47acull, 0x3faaa5aa5df25984ull}, {0x3feca4b31f026aa0ull, 0x3fbc5e53aa362eb4ull},
        {0x3feb2036576afce6ull, 0x3fc526e57720db08ull}, {0x3fe9c2d163a1aa2dull, 0x3fcbc2860d224770ull},
        {0x3fe886e6037841edull, 0x3fd1058bc8a07ee1ull}, {0x3fe767dcf5534862ull, 0x3fd4043057b6ee09ull},
    };
    const double LN2 = dbl(0x3fe62e42fefa39efull);
    const double A0 = dbl(0xbfd00ea348b88334ull), A1 = dbl(0x3fd5575b0be00b6aull), A2 = dbl(0xbfdffffef20a4123ull);
    uint32_t ix = fbits(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2u == 0u) return -__builtin_inff();                    // log(0) = -inf
        if (ix == 0x7f800000u) return x;                                // log(inf) = inf
        if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u) return __builtin_nanf("");
        ix = fbits(x * 8388608.0f) - (23u << 23);                       // subnormal: x 2^23
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = dbl(T[i][0]), logc = dbl(T[i][1]);
    const double z = (double)fromfbits(iz);
    const double r = GLIBCF_FMA(z, invc, -1.0);
    const double y0 = GLIBCF_FMA((double)k, LN2, logc);
    double y = GLIBCF_FMA(r, A1, A2);
    const double r2 = r * r;
    const double t = r + y0;
    y = GLIBCF_FMA(r2, A0, y);
    y = GLIBCF_FMA(r2, y, t);
    return (float)y;
}

// s_sincosf_data.c: {sign[4], hpi_inv (2/pi 2^24), hpi, c0, c1, s1, c2, s2, c3, s3, c4}, the
// second row with the polynomial signs of quadrants 2 and 3
GLIBCF_FN double sc_tab(int row, int j)
{
    const uint64_t P[2][14] = {
        {0x3ff0000000000000ull, 0xbff0000000000000ull, 0xbff0000000000000ull, 0x3ff0000000000000ull,
         0x41645f306dc9c883ull, 0x3ff921fb54442d18ull, 0x3ff0000000000000ull,
         0xbfdffffffd0c621cull, 0xbfc555545995a603ull, 0x3fa55553e1068f19ull, 0x3f81107605230bc4ull,
         0xbf56c087e89a359dull, 0xbf2994eb3774cf24ull, 0x3ef99343027bf8c3ull},
        {0x3ff0000000000000ull, 0xbff0000000000000ull, 0xbff0000000000000ull, 0x3ff0000000000000ull,
         0x41645f306dc9c883ull, 0x3ff921fb54442d18ull, 0xbff0000000000000ull,
         0x3fdffffffd0c621cull, 0xbfc555545995a603ull, 0xbfa55553e1068f19ull, 0x3f81107605230bc4ull,
         0x3f56c087e89a359dull, 0xbf2994eb3774cf24ull, 0xbef99343027bf8c3ull},
    };
    return dbl(P[row][j]);
}

// sinf_poly of s_sinf.c (FMA build): odd n -> the cosine polynomial, even n -> the sine
// polynomial of x (already multiplied by the quadrant sign)
GLIBCF_FN float sincos_poly(double x, double x2, int row, int odd)
{
    GLIBCF_EXACT
    if (!odd) {
        const double t0 = GLIBCF_FMA(x2, sc_tab(row, 12), sc_tab(row, 10));
        const double x3 = x2 * x;
        const double x5 = x2 * x3;
        const double s = GLIBCF_FMA(x3, sc_tab(row, 8), x);
        return (float)GLIBCF_FMA(t0, x5, s);
    }
    const double x4 = x2 * x2;
    const double t3 = GLIBCF_FMA(x2, sc_tab(row, 7), sc_tab(row, 6));
    const double t0 = GLIBCF_FMA(x2, sc_tab(row, 13), sc_tab(row, 11));
    const double x6 = x2 * x4;
    const double c = GLIBCF_FMA(x4, sc_tab(row, 9), t3);
    return (float)GLIBCF_FMA(t0, x6, c);
}

// reduce_fast of s_sinf.c without round-to-int instructions: n = round(x 2/pi) via the 2^24
// scaled hpi_inv, x - n pi/2 fused
GLIBCF_FN double reduce(double x, int *np)
{
    GLIBCF_EXACT
    const double r = x * sc_tab(0, 4);
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return GLIBCF_FMA(-(double)n, sc_tab(0, 5), x);
}

GLIBCF_FN float sinf(float y)
{
    GLIBCF_EXACT
    const double x = (double)y;
    const uint32_t top = (fbits(y) >> 20) & 0x7ffu;
    if (top <= 0x3f3u) {                        // |y| < pi/4
        if (top <= 0x397u) return y;            // |y| < 2^-12
        return sincos_poly(x, x * x, 0, 0);
    }
    if (top > 0x42eu) return __builtin_nanf("");   // |y| >= 120: outside the chain's domain
    int n;
    const double xr = reduce(x, &n);
    const int row = (n & 2) ? 1 : 0;
    return sincos_poly(xr * sc_tab(0, n & 3), xr * xr, row, n & 1);
}

GLIBCF_FN float cosf(float y)
{
    GLIBCF_EXACT
    const double x = (double)y;
    const uint32_t top = (fbits(y) >> 20) & 0x7ffu;
    if (top <= 0x3f3u) {
        if (top <= 0x397u) return 1.0f;
        return sincos_poly(x, x * x, 0, 1);
    }
    if (top > 0x42eu) return __builtin_nanf("");
    int n;
    const double xr = reduce(x, &n);
    const int row = (n & 2) ? 1 : 0;
    return sincos_poly(xr * sc_tab(0, n & 3), xr * xr, row, (n ^ 1) & 1);
}

}  // namespace glibcf
