// rt_fp.h — IEEE-754 helpers shared by the HIP kernel and the host code.
//
// Every function here is __host__ __device__ so the same arithmetic runs on
// gfx950 and on the host. The whole library is compiled with
// -ffp-contract=off: the reference (g++ -O2, no -march) never fuses a*b+c,
// so neither may we. Where the reference's arithmetic *does* fuse (glibc's
// FMA ifunc variants of expf/powf/sinf/cosf, see rt_libm.h) we call
// rt_fma() explicitly.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

// Marks a loaded value as needed here (device code): the compiler then issues a
// group of loads together and waits once, instead of sinking some of them behind
// the first branch that reads the others (each sunk load is one more serial memory
// round trip). No code is emitted; on the host it does nothing.
RT_HD void rt_pin(float v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::"v"(v));
#else
    (void)v;
#endif
}
RT_HD void rt_pin(int v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::"v"(v));
#else
    (void)v;
#endif
}

RT_HD uint32_t rt_asuint(float f) { return __builtin_bit_cast(uint32_t, f); }
RT_HD float rt_asfloat(uint32_t u) { return __builtin_bit_cast(float, u); }
RT_HD uint64_t rt_asuint64(double d) { return __builtin_bit_cast(uint64_t, d); }
RT_HD double rt_asdouble(uint64_t u) { return __builtin_bit_cast(double, u); }

// Correctly-rounded fused multiply-add in double (v_fma_f64 on gfx950,
// glibc fma() on the host).
RT_HD double rt_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// std::max / std::min as libstdc++ defines them (bits/stl_algobase.h):
//   max(a,b) = (a < b) ? b : a ;  min(a,b) = (b < a) ? b : a
// These differ from fmaxf/fminf when an argument is NaN, and the reference
// relies on std::max/min everywhere (render_kernel.cpp:47,137,228,253-254,...).
RT_HD float rt_max(float a, float b) { return (a < b) ? b : a; }
RT_HD float rt_min(float a, float b) { return (b < a) ? b : a; }
RT_HD int rt_maxi(int a, int b) { return (a < b) ? b : a; }
RT_HD int rt_mini(int a, int b) { return (b < a) ? b : a; }

// x86-64 cvttss2si semantics for (int)float: NaN and out-of-range values give
// INT_MIN ("integer indefinite"). gfx950's v_cvt_i32_f32 clamps instead, so
// every float->int conversion on the path goes through here.
RT_HD int rt_f2i(float f)
{
    return (f > -2147483904.0f && f < 2147483648.0f) ? (int)f : (int)0x80000000u;
}

RT_HD float rt_sqrtf(float x) { return __builtin_sqrtf(x); }  // IEEE, correctly rounded
RT_HD float rt_copysignf(float x, float s) { return __builtin_copysignf(x, s); }
RT_HD bool rt_isinf(float x) { return (rt_asuint(x) & 0x7fffffffu) == 0x7f800000u; }
RT_HD bool rt_isnan(float x) { return (rt_asuint(x) & 0x7fffffffu) > 0x7f800000u; }
