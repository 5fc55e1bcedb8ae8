// libm_check — compares rt_libm.h (the device libm restatement, compiled for
// the host here) against this machine's glibc, bit for bit.
//
// usage: libm_check [stride] [function]
//   stride 1 = exhaustive over all 2^32 float inputs (about 10 s/function
//   on 8 threads); the pytest CPU suite uses a larger stride.
// Exit status 0 iff no mismatch. NaN outputs match any NaN (the kernel only
// ever compares NaN, never inspects its payload).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rt_libm.h"

static inline bool same(float a, float b)
{
    if (std::isnan(a) && std::isnan(b)) return true;
    return rt_asuint(a) == rt_asuint(b);
}

template <class F, class G>
static long check_unary(const char* name, long stride, F ref, G mine)
{
    long bad = 0, first = -1;
#pragma omp parallel for reduction(+ : bad) schedule(static)
    for (long i = 0; i < (1L << 32); i += stride) {
        const float x = rt_asfloat((uint32_t)i);
        volatile float xv = x;
        const float r = ref(xv), m = mine(x);
        if (!same(r, m)) {
            bad++;
#pragma omp critical
            if (first < 0) {
                first = i;
                std::printf("  %s(%a [0x%08x]) glibc=%a mine=%a\n", name, x, (uint32_t)i, r, m);
            }
        }
    }
    std::printf("%-8s stride %-6ld mismatches %ld\n", name, stride, bad);
    return bad;
}

static long check_atan2(long stride)
{
    // Structured pairs: every x from a strided sweep against y drawn from a
    // set covering each binade, signs, zeros, infinities and NaN, plus the
    // pairs that occur in the kernel (unit-vector components).
    long bad = 0;
    const float ys[] = {0.0f, -0.0f, 1.0f, -1.0f, 0.5f, -0.3f, 1e-30f, -1e-30f, 3e30f, -7e20f,
                        INFINITY, -INFINITY, NAN, 0x1p-149f, -0x1p-126f, 0.70710677f, 2.4375f, -1.1875f};
    for (float y : ys) {
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (long i = 0; i < (1L << 32); i += stride * 8) {
            const float x = rt_asfloat((uint32_t)i);
            volatile float xv = x, yv = y;
            const float r = atan2f(yv, xv), m = rt_atan2f(y, x);
            if (!same(r, m)) bad++;
        }
    }
    // random unit-ish pairs
    uint32_t s = 12345;
    long bad2 = 0;
    for (long k = 0; k < 20000000 / (stride > 64 ? 8 : 1); k++) {
        s ^= s << 13; s ^= s >> 17; s ^= s << 5;
        uint32_t t = s * 2654435761u;
        const float y = (float)((int32_t)s) * 0x1p-31f, x = (float)((int32_t)t) * 0x1p-31f;
        volatile float xv = x, yv = y;
        if (!same(atan2f(yv, xv), rt_atan2f(y, x))) bad2++;
    }
    std::printf("%-8s stride %-6ld mismatches %ld (+%ld random)\n", "atan2f", stride, bad, bad2);
    return bad + bad2;
}

int main(int argc, char** argv)
{
    const long stride = argc > 1 ? std::atol(argv[1]) : 1;
    const char* only = argc > 2 ? argv[2] : nullptr;
    auto want = [&](const char* n) { return !only || !std::strcmp(only, n); };
    long bad = 0;
    if (want("expf")) bad += check_unary("expf", stride, [](float x) { return expf(x); }, rt_expf);
    if (want("sinf")) bad += check_unary("sinf", stride, [](float x) { return sinf(x); }, rt_sinf);
    if (want("cosf")) bad += check_unary("cosf", stride, [](float x) { return cosf(x); }, rt_cosf);
    if (want("sincosf")) {  // both results of the shared-reduction form, against glibc sinf / cosf
        bad += check_unary("sincos.s", stride, [](float x) { return sinf(x); },
                           [](float x) { float s, c; rt_sincosf(x, s, c); return s; });
        bad += check_unary("sincos.c", stride, [](float x) { return cosf(x); },
                           [](float x) { float s, c; rt_sincosf(x, s, c); return c; });
    }
    if (want("acosf")) bad += check_unary("acosf", stride, [](float x) { return acosf(x); }, rt_acosf);
    if (want("asinf")) bad += check_unary("asinf", stride, [](float x) { return asinf(x); }, rt_asinf);
    if (want("powf5"))
        bad += check_unary("powf5", stride, [](float x) { return powf(x, 5.0f); },
                           [](float x) { return rt_powf(x, 5.0f); });
    if (want("powfg")) {
        const float g = 1.0f / 2.2f;
        bad += check_unary("powfg", stride, [g](float x) { return powf(x, g); },
                           [g](float x) { return rt_powf(x, g); });
    }
    if (want("powfy")) {
        // sweep y at fixed x values (covers the special-case lattice)
        const float xs[] = {0.0f, -0.0f, 1.0f, -1.0f, 0.5f, -2.0f, 3.7f, INFINITY, -INFINITY, NAN, 0x1p-140f, -0x1p-140f};
        long b = 0;
        for (float x : xs) {
            b += check_unary("powf(x,y)", stride * 4, [x](float y) { return powf(x, y); },
                             [x](float y) { return rt_powf(x, y); });
        }
        bad += b;
    }
    if (want("atan2f")) bad += check_atan2(stride);
    std::printf("TOTAL mismatches %ld\n", bad);
    return bad ? 1 : 0;
}
