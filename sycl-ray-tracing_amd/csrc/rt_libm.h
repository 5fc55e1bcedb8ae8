// rt_libm.h — bit-exact restatement of the glibc 2.35 (x86_64) float
// functions that the reference render kernel calls.
//
// Why: the reference (source/render_kernel.cpp) is compiled by g++ and
// links the system libm. Its path tracer is chaotic — one ulp of difference
// in a sampled direction changes later branches — so the device code must
// return *the same bits* as the host libm, not merely an accurate result
// (glibc float functions disagree with
// the correctly-rounded result on 0.01 %–0.5 % of inputs).
//
// Which code: x86_64 glibc selects, through IFUNC, the FMA+AVX2 builds of
// the ARM optimized-routines implementations for expf, powf, sinf, cosf and
// sincosf (sysdeps/x86_64/fpu/multiarch/e_expf-fma.c, e_powf-fma.c,
// s_sinf-fma.c, s_cosf-fma.c). Those are the generic C sources
// (sysdeps/ieee754/flt-32/e_expf.c, e_powf.c, s_sinf.c, s_cosf.c,
// sincosf.h) compiled with -mfma, where GCC contracts a*b+c into vfmadd.
// The contraction points below were read from the disassembly of this
// image's libm.so.6 and are written as explicit rt_fma() calls; all other
// double operations are separate multiply/add. acosf, asinf, atan2f and
// atanf have no IFUNC variant: they are the fdlibm-derived float sources
// (sysdeps/ieee754/flt-32/e_acosf.c, e_asinf.c, e_atan2f.c, s_atanf.c)
// built for baseline x86-64 (plain SSE float arithmetic, no contraction).
// sincosf returns exactly sinf/cosf for every input (checked exhaustively),
// so call sites that GCC merged into sincosf use rt_sinf/rt_cosf.
//
// Constants are the table values of this libm (__exp2f_data,
// __powf_log2_data, __sincosf_table, __inv_pio4, fdlibm coefficients).
//
// Validation: tests/native/libm_check.cpp compares every function with the
// host libm over all 2^32 float inputs (powf over all x at the two
// exponents the kernel uses; atan2f over dense structured pairs), and the
// GPU test tests/test_gpu_libm.py re-checks the device build.
#pragma once

#include "rt_fp.h"

namespace rtlibm {

// ---------------------------------------------------------------- exp2f data
// glibc sysdeps/ieee754/flt-32/e_exp2f_data.c: tab[i] = asuint64(2^(i/32)) - (i << 47)
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint64_t EXP2F_TAB[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};

// glibc sysdeps/ieee754/flt-32/e_powf_log2_data.c: {invc, logc} pairs, N = 16
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint64_t POWF_LOG2_TAB[32] = {
    0x3ff661ec79f8f3beull, 0xbfdefec65b963019ull, 0x3ff571ed4aaf883dull, 0xbfdb0b6832d4fca4ull,
    0x3ff49539f0f010b0ull, 0xbfd7418b0a1fb77bull, 0x3ff3c995b0b80385ull, 0xbfd39de91a6dcf7bull,
    0x3ff30d190c8864a5ull, 0xbfd01d9bf3f2b631ull, 0x3ff25e227b0b8ea0ull, 0xbfc97c1d1b3b7af0ull,
    0x3ff1bb4a4a1a343full, 0xbfc2f9e393af3c9full, 0x3ff12358f08ae5baull, 0xbfb960cbbf788d5cull,
    0x3ff0953f419900a7ull, 0xbfaa6f9db6475fceull, 0x3ff0000000000000ull, 0x0000000000000000ull,
    0x3fee608cfd9a47acull, 0x3fb338ca9f24f53dull, 0x3feca4b31f026aa0ull, 0x3fc476a9543891baull,
    0x3feb2036576afce6ull, 0x3fce840b4ac4e4d2ull, 0x3fe9c2d163a1aa2dull, 0x3fd40645f0c6651cull,
    0x3fe886e6037841edull, 0x3fd88e9c2c1b9ff8ull, 0x3fe767dcf5534862ull, 0x3fdce0a44eb17bccull,
};

// glibc sysdeps/ieee754/flt-32/s_sincosf_data.c: __sincosf_table[2] (14 doubles
// each: sign[4], hpi_inv, hpi, then c0 c1 s1 c2 s2 c3 s3 c4) and __inv_pio4.
#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint64_t SINCOSF_TAB[28] = {
    0x3ff0000000000000ull, 0xbff0000000000000ull, 0xbff0000000000000ull, 0x3ff0000000000000ull,
    0x41645f306dc9c883ull, 0x3ff921fb54442d18ull, 0x3ff0000000000000ull, 0xbfdffffffd0c621cull,
    0xbfc555545995a603ull, 0x3fa55553e1068f19ull, 0x3f81107605230bc4ull, 0xbf56c087e89a359dull,
    0xbf2994eb3774cf24ull, 0x3ef99343027bf8c3ull,
    0x3ff0000000000000ull, 0xbff0000000000000ull, 0xbff0000000000000ull, 0x3ff0000000000000ull,
    0x41645f306dc9c883ull, 0x3ff921fb54442d18ull, 0xbff0000000000000ull, 0x3fdffffffd0c621cull,
    0xbfc555545995a603ull, 0xbfa55553e1068f19ull, 0x3f81107605230bc4ull, 0x3f56c087e89a359dull,
    0xbf2994eb3774cf24ull, 0xbef99343027bf8c3ull,
};

#if defined(__HIPCC__)
__device__ __constant__
#endif
static const uint32_t INV_PIO4[24] = {
    0x000000a2u, 0x0000a2f9u, 0x00a2f983u, 0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
    0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
    0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
    0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u,
};

RT_HD double tabd(const uint64_t* t, int i) { return rt_asdouble(t[i]); }

// The expf / powf tables are indexed by a lane-varying key; in device code they are
// read from an LDS copy (one 8-B LDS read instead of a global load per lookup, each
// on the dependent chain of a powf). Every kernel that evaluates expf / exp2 / powf
// fills the copy first with lds_tables_init() (k_init, k_step, k_tail, k_libm).
#if defined(__HIPCC__)
__shared__ uint64_t rt_libm_lds[64];  // [0, 32) POWF_LOG2_TAB, [32, 64) EXP2F_TAB
__device__ __forceinline__ void lds_tables_init()
{
    for (int i = (int)threadIdx.x; i < 64; i += (int)blockDim.x)
        rt_libm_lds[i] = i < 32 ? POWF_LOG2_TAB[i] : EXP2F_TAB[i - 32];
    __syncthreads();
}
#endif
RT_HD uint64_t exp2_tab(uint64_t i)  // EXP2F_TAB[i], i < 32
{
#if defined(__HIP_DEVICE_COMPILE__)
    return rt_libm_lds[32 + i];
#else
    return EXP2F_TAB[i];
#endif
}
RT_HD double log2_tab(int i)  // POWF_LOG2_TAB[i] as a double
{
#if defined(__HIP_DEVICE_COMPILE__)
    return rt_asdouble(rt_libm_lds[i]);
#else
    return rt_asdouble(POWF_LOG2_TAB[i]);
#endif
}

// __math_oflowf / __math_uflowf / __math_may_uflowf / __math_invalidf results
// (sysdeps/ieee754/flt-32/math_errf.c) under round-to-nearest.
RT_HD float oflowf(uint32_t sign) { return sign ? -__builtin_inff() : __builtin_inff(); }
RT_HD float uflowf(uint32_t sign) { return sign ? -0.0f : 0.0f; }
RT_HD float may_uflowf(uint32_t sign) { return sign ? -0x1p-149f : 0x1p-149f; }  // 0x1.4p-75f^2 rounded
RT_HD float invalidf() { return __builtin_nanf(""); }

// ---------------------------------------------------------------------- expf
// e_expf.c (FMA build). Contractions: kd = fma(InvLn2N, x, SHIFT),
// r = fma(InvLn2N, x, -kd), z = fma(C0, r, C1), y = fma(C2, r, 1), fma(z, r2, y).
RT_HD float expf_(float x)
{
    const uint32_t ix = rt_asuint(x);
    const uint32_t abstop = (ix >> 20) & 0x7ff;
    const double xd = (double)x;
    if (abstop >= 0x42b) {  // |x| >= 88 or NaN
        if (ix == 0xff800000u) return 0.0f;
        if (abstop >= 0x7f8) return x + x;
        if (x > 0x1.62e42ep6f) return oflowf(0);
        if (x < -0x1.9fe368p6f) return uflowf(0);
        if (x < -0x1.9d1d9ep6f) return may_uflowf(0);
    }
    const double InvLn2N = 0x1.71547652b82fep+5;
    const double SHIFT = 0x1.8p+52;
    double kd = rt_fma(InvLn2N, xd, SHIFT);
    const uint64_t ki = rt_asuint64(kd);
    kd -= SHIFT;
    const double r = rt_fma(InvLn2N, xd, -kd);
    uint64_t t = exp2_tab(ki % 32);
    t += ki << 47;
    const double s = rt_asdouble(t);
    const double z = rt_fma(0x1.c6af84b912394p-20, r, 0x1.ebfce50fac4f3p-13);
    const double r2 = r * r;
    double y = rt_fma(0x1.62e42ff0c52d6p-6, r, 1.0);
    y = rt_fma(z, r2, y);
    y = y * s;
    return (float)y;
}

// ---------------------------------------------------------------------- powf
// e_powf.c (FMA build).
RT_HD int checkint(uint32_t iy)
{
    const int e = (iy >> 23) & 0xff;
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
RT_HD bool zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000u - 1; }
RT_HD bool issignalingf(float x)
{
    const uint32_t ix = rt_asuint(x);
    return 2 * (ix ^ 0x00400000u) > 2u * 0x7fc00000u;
}

RT_HD double log2_inline(uint32_t ix)
{
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16);
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = log2_tab(2 * i);
    const double logc = log2_tab(2 * i + 1);
    const double z = (double)rt_asfloat(iz);
    const double r = rt_fma(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double y = rt_fma(0x1.27616c9496e0bp-2, r, -0x1.71969a075c67ap-2);
    const double p = rt_fma(0x1.ec70a6ca7baddp-2, r, -0x1.7154748bef6c8p-1);
    const double r4 = r2 * r2;
    double q = rt_fma(0x1.71547652ab82bp+0, r, y0);
    q = rt_fma(p, r2, q);
    y = rt_fma(y, r4, q);
    return y;
}

RT_HD float exp2_inline(double xd, uint32_t sign_bias)
{
    const double SHIFT = 0x1.8p+47;  // __exp2f_data.shift_scaled
    double kd = xd + SHIFT;
    const uint64_t ki = rt_asuint64(kd);
    kd -= SHIFT;
    const double r = xd - kd;
    uint64_t t = exp2_tab(ki % 32);
    const uint64_t ski = ki + sign_bias;
    t += ski << 47;
    const double s = rt_asdouble(t);
    const double z = rt_fma(0x1.c6af84b912394p-5, r, 0x1.ebfce50fac4f3p-3);
    const double r2 = r * r;
    double y = rt_fma(0x1.62e42ff0c52d6p-1, r, 1.0);
    y = rt_fma(z, r2, y);
    y = y * s;
    return (float)y;
}

RT_HD float powf_(float x, float y)
{
    uint32_t sign_bias = 0;
    uint32_t ix = rt_asuint(x);
    const uint32_t iy = rt_asuint(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || zeroinfnan(iy)) {
        if (zeroinfnan(iy)) {
            if (2 * iy == 0) return issignalingf(x) ? x + y : 1.0f;
            if (ix == 0x3f800000u) return issignalingf(y) ? x + y : 1.0f;
            if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u) return x + y;
            if (2 * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2 * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (zeroinfnan(ix)) {
            float x2 = x * x;
            uint32_t sb = 0;
            if ((ix & 0x80000000u) && checkint(iy) == 1) {
                x2 = -x2;
                sb = 1;
            }
            if (2 * ix == 0 && (iy & 0x80000000u))  // __math_divzerof(sb)
                return (sb ? -1.0f : 1.0f) / 0.0f;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {
            const int yint = checkint(iy);
            if (yint == 0) return invalidf();
            if (yint == 1) sign_bias = 1u << 16;  // SIGN_BIAS
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {
            ix = rt_asuint(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double logx = log2_inline(ix);
    const double ylogx = (double)y * logx;
    if (((rt_asuint64(ylogx) >> 47) & 0xffff) >= (rt_asuint64(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return oflowf(sign_bias);
        if (ylogx <= -150.0) return uflowf(sign_bias);
        if (ylogx < -149.0) return may_uflowf(sign_bias);
    }
    return exp2_inline(ylogx, sign_bias);
}

// ------------------------------------------------------------- sinf / cosf
// s_sinf.c / s_cosf.c / sincosf.h (FMA build).
// The two __sincosf_table rows share hpi_inv, hpi and the sine coefficients; the
// cosine coefficients c0..c4 of row 1 are those of row 0 negated, and sign[] is
// {1, -1, -1, 1} in both. The coefficients are literals here (a lane-varying row
// index into the table would be a memory load per coefficient); negating every
// coefficient of a chain of fma negates its correctly rounded result exactly.
#define RT_SC_HPI_INV 0x41645f306dc9c883ull
#define RT_SC_HPI 0x3ff921fb54442d18ull
RT_HD double sc_sign(int n) { return ((n + 1) & 2) ? -1.0 : 1.0; }  // sign[n & 3]
RT_HD double sc_c(uint64_t c, int tab) { return tab ? -rt_asdouble(c) : rt_asdouble(c); }

RT_HD float sinf_poly_sin(double xs, double x2, int tab)
{
    (void)tab;  // (the sine coefficients are the same in both rows)
    const double s1 = rt_fma(x2, rt_asdouble(0xbf2994eb3774cf24ull), rt_asdouble(0x3f81107605230bc4ull));
    const double x3 = x2 * xs;
    const double x5 = x3 * x2;
    const double s = rt_fma(x3, rt_asdouble(0xbfc555545995a603ull), xs);
    return (float)rt_fma(s1, x5, s);
}

RT_HD float sinf_poly_cos(double x2, int tab)
{
    const double x4 = x2 * x2;
    const double c1 = rt_fma(x2, sc_c(0xbfdffffffd0c621cull, tab), sc_c(0x3ff0000000000000ull, tab));
    const double c2 = rt_fma(x2, sc_c(0x3ef99343027bf8c3ull, tab), sc_c(0xbf56c087e89a359dull, tab));
    const double x6 = x4 * x2;
    const double c = rt_fma(x4, sc_c(0x3fa55553e1068f19ull, tab), c1);
    return (float)rt_fma(c2, x6, c);
}

RT_HD double reduce_fast(double x, int* np)
{
    const double r = x * rt_asdouble(RT_SC_HPI_INV);
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return rt_fma(-(double)n, rt_asdouble(RT_SC_HPI), x);
}

RT_HD double reduce_large(uint32_t xi, int* np)
{
    const uint32_t* arr = &INV_PIO4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0x7fffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = (uint32_t)(xi * arr[0]);
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921fb54442d18p-62;  // pi63
}

RT_HD float sinf_(float y)
{
    const uint32_t iy = rt_asuint(y);
    const uint32_t abstop = (iy >> 20) & 0x7ff;
    const double x = (double)y;
    if (abstop < 0x3f4) {  // |y| < pi/4
        if (abstop < 0x398) return y;  // |y| < 2^-12
        return sinf_poly_sin(x, x * x, 0);
    }
    if (abstop < 0x42f) {  // |y| < 120
        int n;
        const double xr = reduce_fast(x, &n);
        const double s = sc_sign(n);
        const int tab = (n & 2) ? 1 : 0;
        const double x2 = xr * xr;
        if ((n & 1) == 0) return sinf_poly_sin(xr * s, x2, tab);
        return sinf_poly_cos(x2, tab);
    }
    if (abstop < 0x7f8) {
        const int sign = (int)(iy >> 31);
        int n;
        const double xr = reduce_large(iy, &n);
        const double s = sc_sign(n + sign);
        const int tab = ((n + sign) & 2) ? 1 : 0;
        const double x2 = xr * xr;
        if ((n & 1) == 0) return sinf_poly_sin(xr * s, x2, tab);
        return sinf_poly_cos(x2, tab);
    }
    return invalidf();
}

RT_HD float cosf_(float y)
{
    const uint32_t iy = rt_asuint(y);
    const uint32_t abstop = (iy >> 20) & 0x7ff;
    const double x = (double)y;
    if (abstop < 0x3f4) {
        if (abstop < 0x398) return 1.0f;
        return sinf_poly_cos(x * x, 0);
    }
    if (abstop < 0x42f) {
        int n;
        const double xr = reduce_fast(x, &n);
        const double s = sc_sign(n);
        const int tab = (n & 2) ? 1 : 0;
        const double x2 = xr * xr;
        if ((n & 1) != 0) return sinf_poly_sin(xr * s, x2, tab);
        return sinf_poly_cos(x2, tab);
    }
    if (abstop < 0x7f8) {
        const int sign = (int)(iy >> 31);
        int n;
        const double xr = reduce_large(iy, &n);
        const double s = sc_sign(n + sign);
        const int tab = ((n + sign) & 2) ? 1 : 0;
        const double x2 = xr * xr;
        if ((n & 1) != 0) return sinf_poly_sin(xr * s, x2, tab);
        return sinf_poly_cos(x2, tab);
    }
    return invalidf();
}

// sinf_ and cosf_ of one argument from one reduction: the same arithmetic as the two
// functions above (both polynomials are evaluated once, each result picks its own by n & 1).
RT_HD void sincosf_(float y, float& so, float& co)
{
    const uint32_t iy = rt_asuint(y);
    const uint32_t abstop = (iy >> 20) & 0x7ff;
    const double x = (double)y;
    if (abstop < 0x3f4) {
        if (abstop < 0x398) {
            so = y;
            co = 1.0f;
            return;
        }
        const double x2 = x * x;
        so = sinf_poly_sin(x, x2, 0);
        co = sinf_poly_cos(x2, 0);
        return;
    }
    if (abstop < 0x7f8) {
        int n, nt;
        double xr;
        if (abstop < 0x42f) {
            xr = reduce_fast(x, &n);
            nt = n;
        } else {
            xr = reduce_large(iy, &n);
            nt = n + (int)(iy >> 31);
        }
        const double s = sc_sign(nt);
        const int tab = (nt & 2) ? 1 : 0;
        const double x2 = xr * xr;
        const float ps = sinf_poly_sin(xr * s, x2, tab), pc = sinf_poly_cos(x2, tab);
        so = (n & 1) == 0 ? ps : pc;
        co = (n & 1) == 0 ? pc : ps;
        return;
    }
    so = co = invalidf();
}

// --------------------------------------------------------------------- acosf
// e_acosf.c (fdlibm, float arithmetic, no contraction).
RT_HD float acosf_poly_r(float z)
{
    float p = 0x1.23de1p-15f;        // pS5
    p = p * z + 0x1.9efe08p-11f;     // pS4
    p = p * z - 0x1.48228cp-5f;      // pS3
    p = p * z + 0x1.9c155p-3f;       // pS2
    p = p * z - 0x1.4d612p-2f;       // pS1
    p = p * z + 0x1.555556p-3f;      // pS0
    p = p * z;
    float q = 0x1.3b8c5cp-4f;        // qS4
    q = q * z - 0x1.6066c2p-1f;      // qS3
    q = q * z + 0x1.02ae5ap+1f;      // qS2
    q = q * z - 0x1.33a272p+1f;      // qS1
    q = q * z + 1.0f;
    return p / q;
}

RT_HD float acosf_(float x)
{
    const int32_t hx = (int32_t)rt_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) {
        if (hx > 0) return 0.0f;
        return 0x1.4442dp-23f + 0x1.921fb4p+1f;  // pi + 2*pio2_lo
    }
    if (ix > 0x3f800000) return invalidf();
    if (ix < 0x3f000000) {  // |x| < 0.5
        if (ix <= 0x32800000) return 0x1.4442dp-24f + 0x1.921fb4p+0f;
        const float z = x * x;
        const float r = acosf_poly_r(z);
        return 0x1.921fb4p+0f - (x - (0x1.4442dp-24f - x * r));
    }
    if (hx < 0) {  // x < -0.5
        const float z = (x + 1.0f) * 0.5f;
        const float s = rt_sqrtf(z);
        const float r = acosf_poly_r(z);
        const float w = r * s - 0x1.4442dp-24f;
        const float t = w + s;
        return 0x1.921fb4p+1f - (t + t);
    }
    // x > 0.5
    const float z = (1.0f - x) * 0.5f;
    const float s = rt_sqrtf(z);
    const float df = rt_asfloat(rt_asuint(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float r = acosf_poly_r(z);
    const float w = r * s + c;
    const float t = w + df;
    return t + t;
}

// --------------------------------------------------------------------- asinf
// e_asinf.c (glibc float, degree-4 polynomial p0..p4).
RT_HD float asinf_poly(float t)
{
    float p = 0x1.596d28p-5f;       // p4
    p = p * t + 0x1.8c283cp-6f;     // p3
    p = p * t + 0x1.747e4ap-5f;     // p2
    p = p * t + 0x1.3301e4p-4f;     // p1
    p = p * t + 0x1.5555c8p-3f;     // p0
    return p * t;
}

RT_HD float asinf_(float x)
{
    const int32_t hx = (int32_t)rt_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    const float pio2_hi = 0x1.921fb6p+0f, pio2_lo = -0x1.777a5cp-25f, pio4_hi = 0x1.921fb6p-1f;
    if (ix == 0x3f800000) return x * pio2_lo + x * pio2_hi;
    if (ix > 0x3f800000) return invalidf();
    if (ix < 0x3f000000) {  // |x| < 0.5
        if (ix < 0x32000000) return x;
        const float w = asinf_poly(x * x);
        return x + w * x;
    }
    const float ax = rt_asfloat((uint32_t)ix);
    const float t = (1.0f - ax) * 0.5f;
    const float p = asinf_poly(t);
    const float s = rt_sqrtf(t);
    float res;
    if (ix > 0x3f799999) {  // |x| > 0.975
        float u = p * s + s;
        u = u + u;
        res = pio2_hi - (-pio2_lo + u);
    } else {
        const float w = rt_asfloat(rt_asuint(s) & 0xfffff000u);
        const float s2p = (s + s) * p;
        const float c = (t - w * w) / (s + w);
        const float pp = s2p - (pio2_lo - (c + c));
        const float q = pio4_hi - (w + w);
        res = pio4_hi - (pp - q);
    }
    return (hx > 0) ? res : -res;
}

// --------------------------------------------------------------------- atanf
// s_atanf.c (fdlibm float).
RT_HD float atanf_(float x)
{
    const int32_t hx = (int32_t)rt_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        if (hx > 0) return 0x1.4442dp-24f + 0x1.921fb4p+0f;
        return -0x1.921fb4p+0f - 0x1.4442dp-24f;
    }
    int id;
    float xr, hi, lo;
    if (ix < 0x3ee00000) {  // |x| < 0.4375
        if (ix < 0x31000000) return x;  // |x| < 2^-29
        id = -1;
        xr = x;
        hi = 0.0f;
        lo = 0.0f;
    } else {
        const float ax = rt_asfloat((uint32_t)ix);
        if (ix < 0x3f980000) {  // |x| < 1.1875
            if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
                id = 0;
                xr = ((ax + ax) - 1.0f) / (ax + 2.0f);
                hi = 0x1.dac67p-2f;
                lo = 0x1.586ed2p-28f;
            } else {  // 11/16 <= |x| < 19/16
                id = 1;
                xr = (ax - 1.0f) / (ax + 1.0f);
                hi = 0x1.921fb4p-1f;
                lo = 0x1.4442dp-25f;
            }
        } else {
            if (ix < 0x401c0000) {  // |x| < 2.4375
                id = 2;
                xr = (ax - 1.5f) / (ax * 1.5f + 1.0f);
                hi = 0x1.f730bcp-1f;
                lo = 0x1.281f68p-25f;
            } else {  // 2.4375 <= |x| < 2^25
                id = 3;
                xr = -1.0f / ax;
                hi = 0x1.921fb4p+0f;
                lo = 0x1.4442dp-24f;
            }
        }
    }
    const float z = xr * xr;
    const float w = z * z;
    float s1 = 0x1.0ad3aep-6f;      // aT[10]
    s1 = s1 * w + 0x1.97b4b2p-5f;   // aT[8]
    s1 = s1 * w + 0x1.10d66ap-4f;   // aT[6]
    s1 = s1 * w + 0x1.745cdcp-4f;   // aT[4]
    s1 = s1 * w + 0x1.24924ap-3f;   // aT[2]
    s1 = s1 * w + 0x1.555556p-2f;   // aT[0]
    s1 = s1 * z;
    float s2 = -0x1.2b4442p-5f;     // aT[9]
    s2 = s2 * w - 0x1.dde2d6p-5f;   // aT[7]
    s2 = s2 * w - 0x1.3b0f2ap-4f;   // aT[5]
    s2 = s2 * w - 0x1.c71c7p-4f;    // aT[3]
    s2 = s2 * w - 0x1.99999ap-3f;   // aT[1]
    s2 = s2 * w;
    const float xs = (s1 + s2) * xr;
    if (id < 0) return xr - xs;
    const float zz = hi - ((xs - lo) - xr);
    return (hx < 0) ? -zz : zz;
}

// -------------------------------------------------------------------- atan2f
// e_atan2f.c (fdlibm float).
RT_HD float atan2f_(float y, float x)
{
    const int32_t hx = (int32_t)rt_asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)rt_asuint(y);
    const int32_t iy = hy & 0x7fffffff;
    const float tiny = 0x1.4484cp-100f, pi = 0x1.921fb6p+1f, pi_o_2 = 0x1.921fb6p+0f,
                pi_o_4 = 0x1.921fb6p-1f, pi_lo_neg = 0x1.777a5cp-24f;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return atanf_(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m == 2) return tiny + pi;
        if (m == 3) return -pi - tiny;
        return y;
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : tiny + pi_o_2;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            if (m == 2) return 3.0f * pi_o_4 + tiny;
            if (m == 3) return -3.0f * pi_o_4 - tiny;
            if (m == 1) return -pi_o_4 - tiny;
            return tiny + pi_o_4;
        }
        if (m == 2) return tiny + pi;
        if (m == 3) return -pi - tiny;
        if (m == 1) return -0.0f;
        return 0.0f;
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : tiny + pi_o_2;
    const int32_t d = iy - ix;
    float z;
    if (d > 0x1e7fffff)
        z = pi_o_2 - 0x1.777a5cp-25f;
    else if (hx < 0 && (d >> 23) < -60)
        z = 0.0f;
    else
        z = atanf_(__builtin_fabsf(y / x));
    if (m == 0) return z;
    if (m == 1) return rt_asfloat(rt_asuint(z) + 0x80000000u);
    if (m == 2) return pi - (pi_lo_neg + z);
    return (z + pi_lo_neg) - pi;
}

}  // namespace rtlibm

RT_HD float rt_expf(float x) { return rtlibm::expf_(x); }
RT_HD float rt_powf(float x, float y) { return rtlibm::powf_(x, y); }
RT_HD float rt_sinf(float x) { return rtlibm::sinf_(x); }
RT_HD float rt_cosf(float x) { return rtlibm::cosf_(x); }
RT_HD void rt_sincosf(float x, float& s, float& c) { rtlibm::sincosf_(x, s, c); }
RT_HD float rt_acosf(float x) { return rtlibm::acosf_(x); }
RT_HD float rt_asinf(float x) { return rtlibm::asinf_(x); }
RT_HD float rt_atan2f(float y, float x) { return rtlibm::atan2f_(y, x); }
