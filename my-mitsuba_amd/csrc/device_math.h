// Device math helpers for the gfx950 wavefront path tracer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

#include "glibc_mathf.h"

// Float transcendentals of the shading code.  Mitsuba (and the oracle) call
// glibc's float functions; ROCm's float library returns another float on
// 6-39% of arguments, and an ulp can send a long specular path elsewhere
// (DESIGN §5).  MTSG_GLIBC_MATH=1 (the default) evaluates glibc 2.35's own
// algorithms (glibc_mathf.h: the same float for every argument, checked over
// all 2^32 floats on the host and on the GPU, tools/check_glibc_mathf.cpp,
// tools/math_probe.hip); 0 is the measurement variant on ROCm's library.
// Mitsuba's fastexp / fastlog are the double functions rounded to float on
// Linux x86-64 (include/mitsuba/core/math.h:175-199): the device's double
// exp / log, which round to the same float as glibc's but in ~2^-29 of cases.
#ifndef MTSG_GLIBC_MATH
#define MTSG_GLIBC_MATH 1
#endif
#if MTSG_GLIBC_MATH
DEV void mt_sincosf(float x, float *s, float *c) { gmf::sincosf(x, s, c); }
DEV float mt_tanf(float x) { return gmf::tanf(x); }
DEV float mt_logf(float x) { return gmf::logf(x); }
DEV float mt_expf(float x) { return gmf::expf(x); }
DEV float mt_atan2f(float y, float x) { return gmf::atan2f(y, x); }
DEV float mt_atanf(float x) { return gmf::atanf(x); }
DEV float mt_acosf(float x) { return gmf::acosf(x); }
// powf: phong (microfacet.h:219,371-373), Beckmann's visible-normal sampling
// (microfacet.h:604, Mitsuba's default roughconductor) and roughplastic's
// rough-transmittance lookup (rtrans.h)
DEV float mt_powf(float x, float y) { return gmf::powf(x, y); }
#else
DEV void mt_sincosf(float x, float *s, float *c) { sincosf(x, s, c); }
DEV float mt_tanf(float x) { return tanf(x); }
DEV float mt_logf(float x) { return logf(x); }
DEV float mt_expf(float x) { return expf(x); }
DEV float mt_atan2f(float y, float x) { return atan2f(y, x); }
DEV float mt_atanf(float x) { return atanf(x); }
DEV float mt_acosf(float x) { return acosf(x); }
DEV float mt_powf(float x, float y) { return powf(x, y); }
#endif
// math::fastexp / math::fastlog (math.h:185-199)
DEV float mt_fastexp(float x) { return (float)exp((double)x); }
DEV float mt_fastlog(float x) { return (float)log((double)x); }

namespace mtsg {

// 1.0f / x, correctly rounded (the IEEE division the oracle and Mitsuba's
// SSE build compute: dRcp of the kd traversal, kdtree_h / instance.cpp):
// v_rcp_f32 (1 ulp) and one FMA Newton step give the correctly rounded
// reciprocal for every x whose exponent field lies in [1, 252], and the other
// exponents (x or 1/x denormal or zero, inf, NaN) take the IEEE division, a
// branch the wave skips when no lane needs it -- tools/div_probe compared this
// function's sequence with 1.0f / x on all 2^32 bit patterns on the GPU: 0
// differ (profiles/r05_div_probe.txt).  5 VALU instead of the division's ~11.
#ifndef MTSG_FAST_RCP
#define MTSG_FAST_RCP 1
#endif
DEV float rcp_exact(float x) {
#if MTSG_FAST_RCP
    const uint32_t e = (__float_as_uint(x) >> 23) & 0xFFu;
    float y;
    if (__builtin_expect(e - 1u < 252u, 1)) {
        const float r = __builtin_amdgcn_rcpf(x);
        y = __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    } else {
        y = 1.0f / x;
    }
    return y;
#else
    return 1.0f / x;
#endif
}

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
