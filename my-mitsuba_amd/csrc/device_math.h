// Device math helpers for the gfx950 wavefront path tracer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

// Float transcendentals of the shading code.  Mitsuba (and the oracle) call
// glibc's float functions.  Measured on gfx950 over 4M arguments per function
// (tools/math_probe.hip), ROCm's float versions return a different float than
// glibc on 6-39% of arguments, versions evaluated in double and rounded once on
// 0.06-16% (sincos: 16-21% -> 1.3%).  MTSG_CR_MATH is a bit mask of the
// functions evaluated in double.  Measured with the library's double sincos
// (mask 1): C5 parity 3.9e-4 -> 1.1e-4 of the mean, but C5 7% slower
// (k_shade scratch at its 128-VGPR limit; exp/log/pow/acos/atan2 in double spill
// more).  The default stays the float library until the short polynomial
// mt_sincos_d (variant crsc; exact vs the correctly rounded sin/cos on 20M CPU
// arguments) is measured.
#ifndef MTSG_CR_MATH
#define MTSG_CR_MATH 0   // bit mask: 1 sincos, 2 pow, 4 tan, 8 log, 16 exp, 32 atan2, 64 atan, 128 acos
#endif
#define MTSG_CR(bit, dbl, flt) ((MTSG_CR_MATH & (bit)) ? (dbl) : (flt))
// double sincos for |x| <= 1e5 (the shading code's angles stay within a few pi):
// Cody-Waite reduction by pi/2 in two parts (fdlibm's pio2_1 / pio2_1t), Taylor
// polynomials on |r| <= pi/4 to degree 17 / 18 (truncation < 1e-18)
DEV void mt_sincos_d(double x, double *s, double *c) {
    const double k = rint(x * 6.36619772367581382433e-01);
    const double r = fma(-k, 6.07710050650619224932e-11, fma(-k, 1.57079632673412561417e+00, x));
    const double z = r * r;
    double ps = 1.0 / 355687428096000.0;                      // 1/17!
    ps = fma(ps, z, -1.0 / 1307674368000.0);                  // 1/15!
    ps = fma(ps, z, 1.0 / 6227020800.0);
    ps = fma(ps, z, -1.0 / 39916800.0);
    ps = fma(ps, z, 1.0 / 362880.0);
    ps = fma(ps, z, -1.0 / 5040.0);
    ps = fma(ps, z, 1.0 / 120.0);
    ps = fma(ps, z, -1.0 / 6.0);
    const double sn = fma(ps * z, r, r);
    double pc = 1.0 / 6402373705728000.0;                     // 1/18!
    pc = fma(pc, z, -1.0 / 20922789888000.0);                 // 1/16!
    pc = fma(pc, z, 1.0 / 87178291200.0);
    pc = fma(pc, z, -1.0 / 479001600.0);
    pc = fma(pc, z, 1.0 / 3628800.0);
    pc = fma(pc, z, -1.0 / 40320.0);
    pc = fma(pc, z, 1.0 / 720.0);
    pc = fma(pc, z, -1.0 / 24.0);
    pc = fma(pc, z, 0.5);
    const double cs = fma(-pc, z, 1.0);
    const int q = (int)k & 3;
    const double s0 = (q & 1) ? cs : sn, c0 = (q & 1) ? sn : cs;
    *s = (q & 2) ? -s0 : s0;
    *c = ((q + 1) & 2) ? -c0 : c0;
}
DEV void mt_sincosf(float x, float *s, float *c) {
#if MTSG_CR_MATH & 1
    double sd, cd;
    mt_sincos_d((double)x, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
#else
    sincosf(x, s, c);
#endif
}
DEV float mt_powf(float x, float y) { return MTSG_CR(2, (float)pow((double)x, (double)y), powf(x, y)); }
DEV float mt_tanf(float x) { return MTSG_CR(4, (float)tan((double)x), tanf(x)); }
DEV float mt_logf(float x) { return MTSG_CR(8, (float)log((double)x), logf(x)); }
DEV float mt_expf(float x) { return MTSG_CR(16, (float)exp((double)x), expf(x)); }
DEV float mt_atan2f(float y, float x) { return MTSG_CR(32, (float)atan2((double)y, (double)x), atan2f(y, x)); }
DEV float mt_atanf(float x) { return MTSG_CR(64, (float)atan((double)x), atanf(x)); }
DEV float mt_acosf(float x) { return MTSG_CR(128, (float)acos((double)x), acosf(x)); }

namespace mtsg {

DEV float3 mk3(float x, float y, float z) { return make_float3(x, y, z); }
DEV float3 xyz(const float4 &v) { return make_float3(v.x, v.y, v.z); }
DEV float3 operator+(float3 a, float3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
DEV float3 operator-(float3 a, float3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
DEV float3 operator-(float3 a) { return mk3(-a.x, -a.y, -a.z); }
DEV float3 operator*(float3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
DEV float3 operator*(float s, float3 a) { return mk3(a.x * s, a.y * s, a.z * s); }
DEV float3 operator*(float3 a, float3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
DEV float3 operator/(float3 a, float s) { float r = 1.0f / s; return mk3(a.x * r, a.y * r, a.z * r); }
DEV float3 operator/(float3 a, float3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
DEV float3 &operator+=(float3 &a, float3 b) { a = a + b; return a; }
DEV float3 &operator*=(float3 &a, float3 b) { a = a * b; return a; }
DEV float dot(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEV float3 cross(float3 a, float3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DEV float length(float3 a) { return sqrtf(dot(a, a)); }
DEV float3 normalize(float3 a) { return a / length(a); }
DEV bool isZero(float3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
DEV float maxc(float3 a) { return fmaxf(a.x, fmaxf(a.y, a.z)); }
DEV float comp(float3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
DEV float3 sqrtSafe3(float3 a) { return mk3(sqrtf(fmaxf(0.f, a.x)), sqrtf(fmaxf(0.f, a.y)), sqrtf(fmaxf(0.f, a.z))); }
DEV float3 ld3(const float *p) { return mk3(p[0], p[1], p[2]); }

constexpr float kEpsilon = 1e-4f;        // constants.h:28
constexpr float kShadowEpsilon = 1e-3f;  // constants.h:29
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kPi = 3.14159265358979323846f;

// util.cpp:590-600
DEV void coordinateSystem(float3 a, float3 &b, float3 &c) {
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        c = mk3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        c = mk3(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}

struct Frame3 {
    float3 s, t, n;
    DEV float3 toLocal(float3 v) const { return mk3(dot(v, s), dot(v, t), dot(v, n)); }
    DEV float3 toWorld(float3 v) const { return s * v.x + t * v.y + n * v.z; }
};

// counter-mode RNG (DESIGN.md "RNG"; identical to oracle/oracle.cpp)
DEV uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ULL;
    x ^= x >> 27; x *= 0x94D049BB133111EBULL;
    x ^= x >> 31;
    return x;
}
DEV uint64_t counterKey(uint32_t seed, uint64_t sampleId) {
    return mix64(sampleId * 0x9E3779B97F4A7C15ULL + (uint64_t)seed);
}
DEV float counterFloat(uint64_t key, uint32_t dim) {
    uint32_t u = (uint32_t)(mix64(key + (uint64_t)(dim + 1) * 0xD1B54A32D192ED03ULL) >> 32);
    return __uint_as_float((u >> 9) | 0x3f800000u) - 1.0f;
}

}  // namespace mtsg
