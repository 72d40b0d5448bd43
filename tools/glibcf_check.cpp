// Exhaustive bit-for-bit check of sc_polar_decoder_hls_amd/csrc/polar_sc_glibcf.h against the
// host glibc: logf on every float in [0, 1] (the chain's r1), sinf / cosf on every float in
// [0, 8] (the chain's y = 2 pi u lies in [0, 2 pi]). Build: g++ -O2 -mfma -ffp-contract=off.
// argv[1] (optional): stride over the bit patterns (1 = exhaustive). Exit 0 = identical.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../sc_polar_decoder_hls_amd/csrc/polar_sc_glibcf.h"

static unsigned bits(float f) { unsigned u; std::memcpy(&u, &f, 4); return u; }
static float flt(unsigned u) { float f; std::memcpy(&f, &u, 4); return f; }

template <class A, class B>
static long check(const char *name, unsigned lo, unsigned hi, unsigned stride, A ours, B ref)
{
    long bad = 0, n = 0;
    for (unsigned long u = lo; u <= hi; u += stride, n++) {
        const float x = flt((unsigned)u);
        const float a = ours(x), b = ref(x);
        if (bits(a) != bits(b) && !(std::isnan(a) && std::isnan(b))) {
            if (bad < 5) std::printf("%s mismatch x=%a ours=%a glibc=%a\n", name, x, a, b);
            bad++;
        }
    }
    std::printf("%s: %ld inputs, %ld mismatches\n", name, n, bad);
    return bad;
}

int main(int argc, char **argv)
{
    const unsigned stride = argc > 1 ? (unsigned)std::atoi(argv[1]) : 1u;
    long bad = 0;
    bad += check("logf", 0u, bits(1.0f), stride, [](float x) { return glibcf::logf(x); },
                 [](float x) { return ::logf(x); });
    bad += check("sinf", 0u, bits(8.0f), stride, [](float x) { return glibcf::sinf(x); },
                 [](float x) { return ::sinf(x); });
    bad += check("cosf", 0u, bits(8.0f), stride, [](float x) { return glibcf::cosf(x); },
                 [](float x) { return ::cosf(x); });
    return bad ? 1 : 0;
}
