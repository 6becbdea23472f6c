// glibc's float transcendentals, restated for the device (and the host checker).
//
// Mitsuba (and the oracle) call glibc's float functions: math::sincos ->
// ::sincosf (include/mitsuba/core/math.h:219-221), std::sin / std::cos /
// std::tan / std::atan / std::atan2 / std::acos / std::exp / std::log on
// floats (src/emitters/envmap.cpp:386-387,606-607, src/bsdfs/microfacet.h:
// 573-697, src/libcore/math.cpp:103-106).  ROCm's float library returns
// another float than glibc on 6-39% of arguments (tools/math_probe.hip), and
// each such ulp can send a long specular path elsewhere.  These
// are glibc 2.35's algorithms (the image's libm, the one Mitsuba links on the
// box), step for step, so the device returns the same float:
//   sinf / cosf / sincosf  sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
//                          s_sincosf.{c,h}, s_sincosf_data.c (double
//                          polynomials, Szabolcs Nagy / Arm optimized-routines)
//   expf                   e_expf.c, e_exp2f_data.c
//   logf                   e_logf.c, e_logf_data.c
//   powf                   e_powf.c, e_powf_log2_data.c (log2 / exp2 in double)
//   atanf, atan2f, acosf   s_atanf.c, e_atan2f.c, e_acosf.c (fdlibm's float
//                          versions)
//   tanf                   s_tanf.c (the sincosf range reductions) and k_tanf.c
//                          (fdlibm's float kernel)
// On x86-64 glibc selects an FMA build of sinf / cosf / sincosf / expf / logf / powf
// at run time when the CPU has FMA (sysdeps/x86_64/fpu/multiarch, the *-fma
// variants: the same C compiled with -mfma, so a*b+c is contracted); both
// the container's Xeon and the GPU box's EPYC do, so those six use fma()
// exactly where that build contracts.  atanf, atan2f, acosf and tanf are not
// multiarch: no contraction (the device library is built with
// -ffp-contract=off).  Data tables are the published values; the
// exp2f table is round(2^(i/32)) - (i << 47) and is recomputed by the
// checker.  tools/check_glibc_mathf.cpp compares every function with the
// host's libm over all 2^32 floats (pairs for atan2f), tests/test_glibc_mathf.py
// over a strided subset; tools/math_probe.hip does the same on the GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// GMF_CALLS: entry points compiled as out-of-line calls instead of inlined
// (bit mask: 1 sincosf, 2 tanf, 4 atanf / atan2f, 8 acosf, 16 expf / logf,
// 32 powf);
// a call keeps a long function's registers out of its caller's allocation
#ifndef GMF_CALLS
#define GMF_CALLS 13   // measured r04 (C3 / C5 Msamples/s): 0: 1500 / 1378, 13: 1515 / 1427, 31: 1506 / 1430, 14: 1484 / 1370;
                       // r05: 45 (powf out of line too) C3 1509-1512 vs 1526 (13)
#endif
#define GMF __host__ __device__ __forceinline__
#define GMF_CALL __host__ __device__ inline __attribute__((noinline))
#if GMF_CALLS & 1
#define GMF_ENTRY_SC GMF_CALL
#else
#define GMF_ENTRY_SC GMF
#endif
#if GMF_CALLS & 2
#define GMF_ENTRY_TAN GMF_CALL
#else
#define GMF_ENTRY_TAN GMF
#endif
#if GMF_CALLS & 4
#define GMF_ENTRY_ATAN GMF_CALL
#else
#define GMF_ENTRY_ATAN GMF
#endif
#if GMF_CALLS & 8
#define GMF_ENTRY_ACOS GMF_CALL
#else
#define GMF_ENTRY_ACOS GMF
#endif
#if GMF_CALLS & 16
#define GMF_ENTRY_EXPLOG GMF_CALL
#else
#define GMF_ENTRY_EXPLOG GMF
#endif
#if GMF_CALLS & 32
#define GMF_ENTRY_POW GMF_CALL
#else
#define GMF_ENTRY_POW GMF
#endif
// the large-argument reductions are rare: kept out of line, so they do not
// add to the register pressure of the shading kernels that call sinf / tanf
#define GMF_COLD __host__ __device__ inline __attribute__((noinline))

namespace gmf {

// float pairs: two independent polynomials of one function evaluated side by
// side (v_pk_mul_f32 / v_pk_add_f32 on gfx950); each lane is the same IEEE
// multiply and add as the scalar expression, so the results do not change
typedef float f2 __attribute__((ext_vector_type(2)));
GMF f2 mk2(float a, float b) { f2 v; v.x = a; v.y = b; return v; }

// Division inside the 1-D functions (atanf, acosf, tanf), whose operands stay
// in the normal range: on the device a Newton-refined reciprocal and one
// Markstein correction (6 instructions instead of the 11 of the IEEE
// expansion); its quotients are checked against glibc over every float
// argument of those functions on the GPU (tools/math_probe 1).  The host
// (the exhaustive checker) divides in IEEE.  GMF_FAST_DIV=0: IEEE everywhere.
#ifndef GMF_FAST_DIV
#define GMF_FAST_DIV 1
#endif
GMF float fdiv_n(float a, float b) {
#if GMF_FAST_DIV && defined(__HIP_DEVICE_COMPILE__)
    float y = __builtin_amdgcn_rcpf(b);
    const float e = fmaf(-b, y, 1.0f);
    y = fmaf(e, y, y);
    const float q = a * y;
    const float r = fmaf(-b, q, a);
    return fmaf(r, y, q);
#else
    return a / b;
#endif
}

GMF uint32_t asuint(float f) { return __builtin_bit_cast(uint32_t, f); }
GMF float asfloat(uint32_t u) { return __builtin_bit_cast(float, u); }
GMF uint64_t asuint64(double f) { return __builtin_bit_cast(uint64_t, f); }
GMF double asdouble(uint64_t u) { return __builtin_bit_cast(double, u); }
GMF uint32_t abstop12(float x) { return (asuint(x) >> 20) & 0x7ff; }

// ---- sinf / cosf / sincosf (s_sincosf.h) ----------------------------------
// __sincosf_table[0]; entry [1] is the same with the cosine coefficients
// negated (selected for quadrants 2 and 3), which `neg` applies exactly
constexpr double kHpiInv = 0x1.45F306DC9C883p+23;   // 2/pi * 2^24 (no TOINT_INTRINSICS on x86)
constexpr double kHpi = 0x1.921FB54442D18p0;
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
                 kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;
constexpr double kPi63 = 0x1.921FB54442D18p-62;     // 2pi * 2^-64
constexpr float kPio4f = 0x1.921FB6p-1f;

// the two polynomials of sinf_poly / sincosf_poly: the sine one on x, the
// cosine one on x2 (coefficients negated when `neg`: table entry [1])
GMF double sin_poly(double x, double x2) {
    const double x3 = x * x2;
    const double s1 = fma(x2, kS3, kS2);
    const double x7 = x3 * x2;
    const double s = fma(x3, kS1, x);
    return fma(x7, s1, s);
}
GMF double cos_poly(double x2, bool neg) {
    const double c0 = neg ? -kC0 : kC0, c1 = neg ? -kC1 : kC1, c2 = neg ? -kC2 : kC2,
                 c3 = neg ? -kC3 : kC3, c4 = neg ? -kC4 : kC4;
    const double x4 = x2 * x2;
    const double cc2 = fma(x2, c4, c3);
    const double cc1 = fma(x2, c1, c0);
    const double x6 = x4 * x2;
    const double c = fma(x4, c2, cc1);
    return fma(x6, cc2, c);
}

// sinf_poly: n even -> the sine polynomial, odd -> the cosine one
GMF float sinf_poly(double x, double x2, bool neg, int n) {
    return (float)((n & 1) ? cos_poly(x2, neg) : sin_poly(x, x2));
}

// reduce_fast: |x| < 120, quadrant by scaled float-to-int conversion
GMF double reduce_fast(double x, int &n) {
    const double r = x * kHpiInv;
    n = ((int32_t)r + 0x800000) >> 24;
    return fma(-(double)n, kHpi, x);
}

// __inv_pio4[i]: bits [8i, 8i + 32) of 24 zero bits followed by 192 bits of
// 4/pi (the table's sliding window), from four 64-bit words
GMF uint32_t inv_pio4(int i) {
    const uint64_t w0 = 0x000000a2f9836e4eull, w1 = 0x441529fc2757d1f5ull, w2 = 0x34ddc0db6295993cull,
                   w3 = 0x4390410000000000ull;
    const int bit = 8 * i, k = bit >> 6, s = bit & 63;
    const uint64_t a = k == 0 ? w0 : k == 1 ? w1 : k == 2 ? w2 : w3;
    const uint64_t b = k == 0 ? w1 : k == 1 ? w2 : w3;
    const uint64_t v = s ? (a << s) | (b >> (64 - s)) : a;
    return (uint32_t)(v >> 32);
}

// reduce_large: |x| >= 120, 32x96-bit product with 4/pi in 2.62 fixed point
GMF double reduce_large(uint32_t xi, int &np) {
    const int idx = (xi >> 26) & 15;
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = (uint32_t)(xi * inv_pio4(idx));
    const uint64_t res1 = (uint64_t)xi * inv_pio4(idx + 4);
    const uint64_t res2 = (uint64_t)xi * inv_pio4(idx + 8);
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    np = (int)n;
    return x * kPi63;
}

// the |x| >= 120 path of sinf / cosf: the sign table and the negated cosine
// polynomial follow n + sign, the polynomial choice follows n
GMF_COLD void sincosf_large(float y, float *sinp, float *cosp) {
    const uint32_t xi = asuint(y);
    int n;
    const double x = reduce_large(xi, n);
    const int q = n + (int)(xi >> 31);
    const double xs = ((q + 1) & 2) ? -x : x;
    *sinp = sinf_poly(xs, x * x, (q & 2) != 0, n);
    *cosp = sinf_poly(xs, x * x, (q & 2) != 0, n ^ 1);
}

// sincosf (s_sincosf.c): the sine and cosine polynomials of sinf / cosf on one
// reduction (sincosf_poly performs the same operations as sinf_poly, so each
// result equals the separate sinf / cosf call)
GMF_ENTRY_SC void sincosf(float y, float *sinp, float *cosp) {
    const uint32_t top = abstop12(y);
    if (top >= abstop12(120.0f) && top < 0x7f8) {   // rare: out of line
        sincosf_large(y, sinp, cosp);
        return;
    }
    // |x| < pi/4 takes reduce_fast's n = 0 exactly (x - 0 * pi/2 = x), so
    // s_sincosf.c's small-argument branch is the same computation; the
    // special cases are selected at the end instead of branched to
    int n;
    const double x = reduce_fast((double)y, n);
    const double xs = ((n + 1) & 2) ? -x : x;   // sign[n & 3] = {1, -1, -1, 1}
    const double x2 = x * x;
    // both polynomials, swapped for odd quadrants (no divergent branch)
    const float ps = (float)sin_poly(xs, x2), pc = (float)cos_poly(x2, (n & 2) != 0);
    float sv = (n & 1) ? pc : ps, cv = (n & 1) ? ps : pc;
    const bool tinyArg = top < abstop12(0x1p-12f), bad = top >= 0x7f8;
    sv = tinyArg ? y : bad ? y - y : sv;
    cv = tinyArg ? 1.0f : bad ? y - y : cv;
    *sinp = sv;
    *cosp = cv;
}

GMF float sinf(float y) { float s, c; gmf::sincosf(y, &s, &c); return s; }
GMF float cosf(float y) { float s, c; gmf::sincosf(y, &s, &c); return c; }

// ---- expf (e_expf.c, EXP2F_TABLE_BITS 5) -----------------------------------
// round(2^(i/32)) - (i << 47), i = 0..31 (__exp2f_data.tab)
constexpr uint64_t kExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

GMF_ENTRY_EXPLOG float expf(float x) {
    const double xd = (double)x;
    const uint32_t abstop = abstop12(x) & 0x7ff;
    if (abstop >= abstop12(88.0f)) {
        if (asuint(x) == 0xff800000u) return 0.0f;   // -inf
        if (abstop >= abstop12(__builtin_inff())) return x + x;
        if (x > 0x1.62e42ep6f) return __builtin_inff();   // overflow
        if (x < -0x1.9fe368p6f) return 0.0f;             // underflow
    }
    constexpr double InvLn2N = 0x1.71547652b82fep+5, Shift = 0x1.8p+52;
    constexpr double C0 = 0x1.c6af84b912394p-20, C1 = 0x1.ebfce50fac4f3p-13, C2 = 0x1.62e42ff0c52d6p-6;
    // z = InvLn2N * xd feeds two additions only, so the FMA build folds the
    // product into both (GCC's convert_mult_to_fma): k and r from the exact
    // product (measured: the unfused form differs on 2 of the 2^32 floats)
    double kd = fma(InvLn2N, xd, Shift);
    const uint64_t ki = asuint64(kd);
    kd -= Shift;
    const double r = fma(InvLn2N, xd, -kd);
    uint64_t t = kExp2fTab[ki % 32];
    t += ki << 47;
    const double s = asdouble(t);
    const double z = fma(C0, r, C1);
    const double r2 = r * r;
    double y = fma(C2, r, 1.0);
    y = fma(z, r2, y);
    y = y * s;
    return (float)y;
}

// ---- logf (e_logf.c, LOGF_TABLE_BITS 4) ------------------------------------
// __logf_data.tab: {1/c, log(c)} of the 16 subintervals
constexpr double kLogfInvc[16] = {0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0, 0x1.3c995b0b80385p+0, 0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0, 0x1.0953f419900a7p+0, 0x1p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1, 0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
constexpr double kLogfLogc[16] = {-0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3, -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3, -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4, -0x1.252f438e10c1ep-5, 0x0p+0, 0x1.aa5aa5df25984p-5, 0x1.c5e53aa362eb4p-4, 0x1.526e57720db08p-3, 0x1.bc2860d22477p-3, 0x1.1058bc8a07ee1p-2, 0x1.4043057b6ee09p-2};

GMF_ENTRY_EXPLOG float logf(float x) {
    uint32_t ix = asuint(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -__builtin_inff();
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return (x - x) / (x - x);
        ix = asuint(x * 0x1p23f);   // subnormal: normalise
        ix -= 23u << 23;
    }
    constexpr uint32_t OFF = 0x3f330000u;
    constexpr double Ln2 = 0x1.62e42fefa39efp-1;
    constexpr double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    const uint32_t tmp = ix - OFF;
    const uint32_t i = (tmp >> (23 - 4)) % 16;
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = kLogfInvc[i], logc = kLogfLogc[i];
    const double z = (double)asfloat(iz);
    const double r = fma(z, invc, -1.0);
    const double y0 = fma((double)k, Ln2, logc);
    const double r2 = r * r;
    double y = fma(A1, r, A2);
    y = fma(A0, r2, y);
    y = fma(y, r2, y0 + r);
    return (float)y;
}

// ---- atanf (s_atanf.c) -----------------------------------------------------
constexpr float kAtanHi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
constexpr float kAtanLo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};

GMF_ENTRY_ATAN float atanf(float x) {
    constexpr float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                    aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                    aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                    aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const int32_t hx = (int32_t)asuint(x);
    const int32_t ix = hx & 0x7fffffff;
    // the argument reduction of each range, as one division of selected
    // operands (the same float operations as s_atanf.c's branches):
    //   id -1 |x| < 0.4375        none
    //   id 0  [0.4375, 0.6875)    (2|x| - 1) / (2 + |x|)
    //   id 1  [0.6875, 1.1875)    (|x| - 1) / (|x| + 1)
    //   id 2  [1.1875, 2.4375)    (|x| - 1.5) / (1 + 1.5|x|)
    //   id 3  [2.4375, 2^25)      -1 / |x|
    // and the special cases (|x| < 2^-29: x; |x| >= 2^25: +-atan(inf); NaN)
    // selected at the end
    const float ax = fabsf(x);
    const int id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
    const float num = id == 0 ? 2.0f * ax - 1.0f : id == 1 ? ax - 1.0f : id == 2 ? ax - 1.5f : -1.0f;
    const float den = id == 0 ? 2.0f + ax : id == 1 ? ax + 1.0f : id == 2 ? 1.0f + 1.5f * ax : ax;
    const float q = fdiv_n(num, den);
    const float xr = id < 0 ? x : q;
    const float z = xr * xr;
    const float w = z * z;
    // s1 = z (aT0 + w (aT2 + w (aT4 + w (aT6 + w (aT8 + w aT10))))),
    // s2 = w (aT1 + w (aT3 + w (aT5 + w (aT7 + w aT9)))), as a pair
    const f2 ww = mk2(w, w);
    f2 u = mk2(aT8, aT7) + ww * mk2(aT10, aT9);
    u = mk2(aT6, aT5) + ww * u;
    u = mk2(aT4, aT3) + ww * u;
    u = mk2(aT2, aT1) + ww * u;
    const float s1 = z * (aT0 + w * u.x);
    const float s2 = w * u.y;
    const float hi = id == 0 ? kAtanHi[0] : id == 1 ? kAtanHi[1] : id == 2 ? kAtanHi[2] : kAtanHi[3];
    const float lo = id == 0 ? kAtanLo[0] : id == 1 ? kAtanLo[1] : id == 2 ? kAtanLo[2] : kAtanLo[3];
    const float zz = hi - ((xr * (s1 + s2) - lo) - xr);
    float r = id < 0 ? xr - xr * (s1 + s2) : hx < 0 ? -zz : zz;
    r = ix < 0x31000000 ? x : r;
    constexpr float atanInf = kAtanHi[3] + kAtanLo[3];
    r = ix >= 0x4c000000 ? (ix > 0x7f800000 ? x + x : hx > 0 ? atanInf : -atanInf) : r;
    return r;
}

// ---- atan2f (e_atan2f.c) ---------------------------------------------------
GMF_ENTRY_ATAN float atan2f(float y, float x) {
    constexpr float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                    pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)asuint(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)asuint(y), iy = hy & 0x7fffffff;
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);   // 2 sign(x) + sign(y)
    // the general case; e_atan2f.c's special cases are selected afterwards in
    // reverse order of its tests.  x == 1 (atanf(y) there) is the general
    // case here: y / 1 is exact and atanf is odd to the bit.
    const int k = (iy - ix) >> 23;
    const float za = gmf::atanf(fabsf(y / x));
    const float z = k > 60 ? pi_o_2 + 0.5f * pi_lo : (hx < 0 && k < -60) ? 0.0f : za;
    float r = m == 0 ? z : m == 1 ? asfloat(asuint(z) ^ 0x80000000u) : m == 2 ? pi - (z - pi_lo) : (z - pi_lo) - pi;
    r = iy == 0x7f800000 ? (hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny) : r;
    if (ix == 0x7f800000) {
        const float both = m == 0 ? pi_o_4 + tiny : m == 1 ? -pi_o_4 - tiny : m == 2 ? 3.0f * pi_o_4 + tiny
                                                                                      : -3.0f * pi_o_4 - tiny;
        const float xinf = m == 0 ? 0.0f : m == 1 ? -0.0f : m == 2 ? pi + tiny : -pi - tiny;
        r = iy == 0x7f800000 ? both : xinf;
    }
    r = ix == 0 ? (hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny) : r;
    r = iy == 0 ? (m < 2 ? y : m == 2 ? pi + tiny : -pi - tiny) : r;
    r = (ix > 0x7f800000 || iy > 0x7f800000) ? x + y : r;
    return r;
}

// ---- acosf (e_acosf.c) -----------------------------------------------------
GMF_ENTRY_ACOS float acosf(float x) {
    constexpr float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f,
                    pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f,
                    pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f,
                    qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f,
                    qS4 = 7.7038154006e-02f;
    const int32_t hx = (int32_t)asuint(x), ix = hx & 0x7fffffff;
    // e_acosf.c's three ranges on one rational approximation: z = x^2
    // (|x| < 0.5), (1 + x) / 2 (x <= -0.5), (1 - x) / 2 (x >= 0.5); each
    // range's own combination, and the special cases, selected at the end
    const bool small = ix < 0x3f000000;
    const float z = small ? x * x : hx < 0 ? (1.0f + x) * 0.5f : (1.0f - x) * 0.5f;
    // p = z (pS0 + z (pS1 + ... + z pS5)), q = 1 + z (qS1 + ... + z qS4), as a pair
    const f2 zz2 = mk2(z, z);
    f2 u = mk2(pS4, qS3) + zz2 * mk2(pS5, qS4);
    u = mk2(pS3, qS2) + zz2 * u;
    u = mk2(pS2, qS1) + zz2 * u;
    u = mk2(pS1, 1.0f) + zz2 * u;
    const float p = z * (pS0 + z * u.x);
    const float q = u.y;
    const float r = fdiv_n(p, q);
    const float s = sqrtf(z);
    const float rs = pio2_hi - (x - (pio2_lo - x * r));   // |x| < 0.5
    const float rn = pi - 2.0f * (s + (r * s - pio2_lo));  // x <= -0.5
    const float df = asfloat(asuint(s) & 0xfffff000u);     // x >= 0.5
    const float c = fdiv_n(z - df * df, s + df);
    const float rp = 2.0f * (df + (r * s + c));
    float res = small ? rs : hx < 0 ? rn : rp;
    res = ix <= 0x23000000 ? pio2_hi + pio2_lo : res;
    res = ix == 0x3f800000 ? (hx > 0 ? 0.0f : pi + 2.0f * pio2_lo) : res;
    res = ix > 0x3f800000 ? (x - x) / (x - x) : res;
    return res;
}

// ---- tanf (s_tanf.c, k_tanf.c) ---------------------------------------------
// s_tanf.c's rem_pio2f: the sincosf reductions (reduce_fast below 120, the
// 4/pi product above), in s_tanf.c's own build -- not multiarch, so the
// product n * pi/2 is rounded before the subtraction -- split into a float
// head and tail for __kernel_tanf
GMF_COLD double rem_pio2f_large(float x, int &n) {
    const uint32_t xi = asuint(x);
    const double dx = reduce_large(xi, n);
    return (xi >> 31) ? -dx : dx;
}

GMF int rem_pio2f(float x, float &y0, float &y1) {
    double dx = x;
    int n;
    if (abstop12(x) < abstop12(120.0f)) {
        const double r = dx * kHpiInv;
        n = ((int32_t)r + 0x800000) >> 24;
        const double nh = (double)n * kHpi;
        dx = dx - nh;
    } else {
        dx = rem_pio2f_large(x, n);
    }
    y0 = (float)dx;
    y1 = (float)(dx - (double)y0);
    return n;
}

GMF float kernel_tanf(float x, float y, int iy) {
    constexpr float pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
    constexpr float T0 = 3.3333334327e-01f, T1 = 1.3333334029e-01f, T2 = 5.3968254477e-02f, T3 = 2.1869488060e-02f,
                    T4 = 8.8632395491e-03f, T5 = 3.5920790397e-03f, T6 = 1.4562094584e-03f, T7 = 5.8804126456e-04f,
                    T8 = 2.4646313977e-04f, T9 = 7.8179444245e-05f, T10 = 7.1407252108e-05f, T11 = -1.8558637748e-05f,
                    T12 = 2.5907305826e-05f;
    const int32_t hx = (int32_t)asuint(x), ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {   // |x| < 2^-13
        if ((int)x == 0) {
            if ((ix | (iy + 1)) == 0) return 1.0f / fabsf(x);
            if (iy == 1) return x;
            return -1.0f / x;
        }
    }
    const bool big = ix >= 0x3f2ca140;   // |x| >= 0.6744: tan(pi/4 - |x|) form
    {
        const float xa = hx < 0 ? -x : x, ya = hx < 0 ? -y : y;
        const float xb = (pio4 - xa) + (pio4lo - ya);
        x = big ? xb : x;
        y = big ? 0.0f : y;
    }
    const float nearPio4 = (float)((1 - ((hx >> 30) & 2)) * iy) * (1.0f - 2 * iy * x);   // |pi/4 - |x|| < 2^-13
    const float z = x * x;
    float w = z * z;
    // r = T1 + w (T3 + ... + w T11), v = z (T2 + w (T4 + ... + w T12)), as a pair
    const f2 ww = mk2(w, w);
    f2 u = mk2(T9, T10) + ww * mk2(T11, T12);
    u = mk2(T7, T8) + ww * u;
    u = mk2(T5, T6) + ww * u;
    u = mk2(T3, T4) + ww * u;
    u = mk2(T1, T2) + ww * u;
    float r = u.x;
    float v = z * u.y;
    const float s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T0 * s;
    w = x + r;
    // the one division of either final form: w^2 / (w + iy) (big), -1 / w
    const float vi = (float)iy;
    const float q = big ? fdiv_n(w * w, w + vi) : fdiv_n(-1.0f, w);
    const float rb = (float)(1 - ((hx >> 30) & 2)) * (vi - 2.0f * (x - (q - r)));
    // -1/(x+r) accurately: a = q
    const float zz = asfloat(asuint(w) & 0xfffff000u);
    v = r - (zz - x);
    const float t = asfloat(asuint(q) & 0xfffff000u);
    const float ss = 1.0f + t * zz;
    const float rm = t + q * (ss + t * v);
    float res = big ? (fabsf(x) < 0x1p-13f ? nearPio4 : rb) : iy == 1 ? w : rm;
    return res;
}

GMF_ENTRY_TAN float tanf(float x) {
    const int32_t ix = (int32_t)asuint(x) & 0x7fffffff;
    if (ix <= 0x3f490fda) return kernel_tanf(x, 0.0f, 1);
    if (ix >= 0x7f800000) return x - x;
    float y0, y1;
    const int n = rem_pio2f(x, y0, y1);
    return kernel_tanf(y0, y1, 1 - ((n & 1) << 1));
}

// ---- powf (e_powf.c, e_powf_log2_data.c, POWF_LOG2_TABLE_BITS 4) ----------
// The FMA build (sysdeps/x86_64/fpu/multiarch e_powf-fma.c) contracts every
// a * b + c of log2_inline and exp2_inline; y * log2(x) is not fused (it is
// also compared against the overflow bounds).  log2 table: {1/c, log2(c)} of
// the 16 subintervals (the same 1/c as logf's; log2(c) = -log2(1/c) rounded,
// checked by the host test), poly: log2(1 + r) of degree 5.
constexpr double kPowfLogc[16] = {-0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2, -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7afp-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4, -0x1.a6f9db6475fcep-5, 0x0p+0, 0x1.338ca9f24f53dp-4, 0x1.476a9543891bap-3, 0x1.e840b4ac4e4d2p-3, 0x1.40645f0c6651cp-2, 0x1.88e9c2c1b9ff8p-2, 0x1.ce0a44eb17bccp-2};

// 0: not an integer, 1: odd, 2: even (iy: a non-zero finite float's bits)
GMF int powf_checkint(uint32_t iy) {
    const int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
GMF bool powf_zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000u - 1; }
GMF bool powf_issignaling(float x) { return 2 * (asuint(x) ^ 0x00400000u) > 2u * 0x7fc00000u; }

GMF double powf_log2(uint32_t ix) {
    constexpr uint32_t OFF = 0x3f330000u;
    constexpr double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
                     A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp0;
    const uint32_t tmp = ix - OFF;
    const uint32_t i = (tmp >> (23 - 4)) % 16;
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = kLogfInvc[i], logc = kPowfLogc[i];
    const double z = (double)asfloat(iz);
    const double r = fma(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double y = fma(A0, r, A1);
    const double p = fma(A2, r, A3);
    const double r4 = r2 * r2;
    double q = fma(A4, r, y0);
    q = fma(p, r2, q);
    y = fma(y, r4, q);
    return y;
}

GMF float powf_exp2(double xd, uint32_t signBias) {
    // xd is log2 unscaled (POWF_SCALE_BITS 0 without toint intrinsics): the
    // shift rounds it to multiples of 1/32 and r is in [-1/64, 1/64], so the
    // unscaled __exp2f_data.poly applies
    constexpr double Shift = 0x1.8p+52 / 32;
    constexpr double C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3, C2 = 0x1.62e42ff0c52d6p-1;
    double kd = xd + Shift;
    const uint64_t ki = asuint64(kd);
    kd -= Shift;
    const double r = xd - kd;
    uint64_t t = kExp2fTab[ki % 32];
    const uint64_t ski = ki + signBias;
    t += ski << (52 - 5);
    const double s = asdouble(t);
    const double z = fma(C0, r, C1);
    const double r2 = r * r;
    double y = fma(C2, r, 1.0);
    y = fma(z, r2, y);
    y = y * s;
    return (float)y;
}

GMF_ENTRY_POW float powf(float x, float y) {
    constexpr uint32_t SIGN_BIAS = 1u << (5 + 11);
    uint32_t signBias = 0;
    uint32_t ix = asuint(x);
    const uint32_t iy = asuint(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || powf_zeroinfnan(iy)) {
        // x < 0x1p-126, inf or nan, or y 0, inf or nan
        if (powf_zeroinfnan(iy)) {
            if (2 * iy == 0) return powf_issignaling(x) ? x + y : 1.0f;
            if (ix == 0x3f800000u) return powf_issignaling(y) ? x + y : 1.0f;
            if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u) return x + y;
            if (2 * ix == 2 * 0x3f800000u) return 1.0f;
            if ((2 * ix < 2 * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;   // |x|<1 && y==inf or |x|>1 && y==-inf
            return y * y;
        }
        if (powf_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && powf_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        // x and y are non-zero finite
        if (ix & 0x80000000u) {
            const int yint = powf_checkint(iy);
            if (yint == 0) return (x - x) / (x - x);   // __math_invalidf
            if (yint == 1) signBias = SIGN_BIAS;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {
            // normalise a subnormal x so that its exponent becomes negative
            ix = asuint(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double logx = powf_log2(ix);
    const double ylogx = (double)y * logx;   // y is 0 if logx is 0
    if ((asuint64(ylogx) >> 47 & 0xffff) >= asuint64(126.0) >> 47) {
        // |y * log(x)| >= 126
        if (ylogx > 0x1.fffffffd1d571p+6) return signBias ? -0x1p97f * 0x1p97f : 0x1p97f * 0x1p97f;   // __math_oflowf
        if (ylogx <= -150.0) return signBias ? -0x1p-95f * 0x1p-95f : 0x1p-95f * 0x1p-95f;         // __math_uflowf
    }
    return powf_exp2(ylogx, signBias);
}

}  // namespace gmf
