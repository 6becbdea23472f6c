// Environment emitter on the device (src/emitters/envmap.cpp:99-660 and
// TMIPMap, include/mitsuba/render/mipmap.h:503-840).  Tables are built on the
// host (my-mitsuba_amd/host/envmap.cpp) and uploaded as-is: an RGB MIP
// pyramid with half-rounded texels, the row/column sampling CDFs and the
// scene bounding sphere.
#pragma once
#include "device_math.h"
#include "mipmap.h"
#include "../../include/mtsg.h"

namespace mtsg {

constexpr float kInvTwoPi = 0.15915494309189533577f;   // constants.h:65

// MTSG_ENV_GUIDE: the CDF searches of the importance sampling start from a
// guide table (ENV_GUIDE + 1 entries per CDF: the lower_bound of g /
// ENV_GUIDE), so a search reads 1-3 CDF entries instead of ~log2(size): the
// same index as the full std::lower_bound (the answer for a sample in
// [g, g+1) / ENV_GUIDE lies between the guides of g and g + 1), with a chain
// of dependent loads 3x shorter.  0: the full search (round 3).
#ifndef MTSG_ENV_GUIDE
#define MTSG_ENV_GUIDE 1
#endif
constexpr uint32_t ENV_GUIDE = 128;   // C5 (envmap.exr): 2.4 column search steps on average instead of 9

struct DevEnv {
    const mtsg_envmap *E;        // device copy of the table header
    const float *texels;         // RGB, all levels
    const float *cdfRows, *cdfCols, *rowWeights;
    const uint32_t *guideRows;   // ENV_GUIDE + 1 entries
    const uint32_t *guideCols;   // (ENV_GUIDE + 1) per row
};

DEV DevMip env_mip(const DevEnv &V) { return DevMip{&V.E->mip, V.texels}; }   // u repeats, v clamps

DEV float3 env_rot(const float *m, float3 v) {
    return mk3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z, m[6] * v.x + m[7] * v.y + m[8] * v.z);
}

// the lookup coordinates of a local direction (envmap.cpp:386-387 and
// 606-607 compute the same two values)
DEV void env_uv(float3 v, float &ux, float &uy) {
    ux = mt_atan2f(v.x, -v.z) * kInvTwoPi;
    uy = mt_acosf(fminf(1.0f, fmaxf(-1.0f, v.y))) * kInvPi;
}

// EnvironmentMap::evalEnvironment (envmap.cpp:380-410); hasDiff: camera
// rays carrying (scaled) differentials -> EWA, otherwise bilinear level 0.
// env_eval_uv: v = the local direction and its env_uv already computed
DEV float3 env_eval_uv(const DevEnv &V, float3 v, float ux, float uy, bool hasDiff, float3 rxD, float3 ryD) {
    float3 value;
    if (!hasDiff) {
        value = mip_bilinear(env_mip(V), 0, ux, uy);
    } else {
        const float3 dvdx = env_rot(V.E->to_local, rxD) - v, dvdy = env_rot(V.E->to_local, ryD) - v;
        const float t1 = kInvTwoPi / (v.x * v.x + v.z * v.z), t2 = -kInvPi / fmaxf(sqrtf(fmaxf(0.0f, 1.0f - v.y * v.y)), kEpsilon);
        value = mip_filtered(env_mip(V), ux, uy, t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y, t1 * (dvdy.z * v.x - dvdy.x * v.z),
                             t2 * dvdy.y);
    }
    return value * V.E->scale;
}
DEV float3 env_eval(const DevEnv &V, float3 dWorld, bool hasDiff, float3 rxD, float3 ryD) {
    const float3 v = env_rot(V.E->to_local, dWorld);
    float ux, uy;
    env_uv(v, ux, uy);
    return env_eval_uv(V, v, ux, uy, hasDiff, rxD, ryD);
}

DEV float env_lum(float3 c) { return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f; }

// std::lower_bound-based sampleReuse (envmap.cpp:628-633)
__host__ __device__ inline uint32_t env_sample_reuse(const float *cdf, uint32_t size, float &sample) {   // (host: tools/check_env_guide)
    uint32_t lo = 0, len = size + 1;
    while (len > 0) {
        const uint32_t half = len >> 1;
        if (cdf[lo + half] < sample) { lo += half + 1; len -= half + 1; }
        else len = half;
    }
    const uint32_t index = min((uint32_t)max((int)lo - 1, 0), size - 1);
    sample = (sample - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return index;
}

// the same over [guide[g], guide[g + 1]] (the sample is in [0, 1): g = floor(sample * ENV_GUIDE) is exact)
__host__ __device__ inline uint32_t env_sample_reuse_guided(const float *cdf, uint32_t size, const uint32_t *guide, float &sample) {
    const uint32_t g = min((uint32_t)(sample * (float)ENV_GUIDE), ENV_GUIDE - 1u);
    uint32_t lo = guide[g];
    const uint32_t hi = min(guide[g + 1], size);
    uint32_t len = hi + 1 - lo;
    while (len > 0) {
        const uint32_t half = len >> 1;
        if (cdf[lo + half] < sample) { lo += half + 1; len -= half + 1; }
        else len = half;
    }
    const uint32_t index = min((uint32_t)max((int)lo - 1, 0), size - 1);
    sample = (sample - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return index;
}

DEV float env_tent(float sample) {   // warp.cpp:143-155
    float sign;
    if (sample < 0.5f) { sign = 1; sample *= 2; }
    else { sign = -1; sample = 2 * (sample - 0.5f); }
    return sign * (1 - sqrtf(sample));
}

// internalSampleDirection (envmap.cpp:574-600): local direction, value, pdf
DEV void env_internal_sample(const DevEnv &V, float sx, float sy, float3 &d, float3 &value, float &pdf) {
    const int W = V.E->mip.level_w[0], H = V.E->mip.level_h[0];
    const DevMip M = env_mip(V);
#if MTSG_ENV_GUIDE
    const uint32_t row = env_sample_reuse_guided(V.cdfRows, (uint32_t)H, V.guideRows, sy);
    const uint32_t col =
        env_sample_reuse_guided(V.cdfCols + row * (uint32_t)(W + 1), (uint32_t)W, V.guideCols + row * (ENV_GUIDE + 1u), sx);
#else
    const uint32_t row = env_sample_reuse(V.cdfRows, (uint32_t)H, sy);
    const uint32_t col = env_sample_reuse(V.cdfCols + row * (uint32_t)(W + 1), (uint32_t)W, sx);
#endif
    const float px = (float)col + env_tent(sx), py = (float)row + env_tent(sy);
    const int xPos = (int)floorf(px), yPos = (int)floorf(py);
    const float dx1 = px - xPos, dx2 = 1.0f - dx1, dy1 = py - yPos, dy2 = 1.0f - dy1;
    const float3 value1 = mip_texel(M, 0, xPos, yPos) * dx2 * dy2 + mip_texel(M, 0, xPos + 1, yPos) * dx1 * dy2;
    const float3 value2 = mip_texel(M, 0, xPos, yPos + 1) * dx2 * dy1 + mip_texel(M, 0, xPos + 1, yPos + 1) * dx1 * dy1;
    value = (value1 + value2) * V.E->scale;
    pdf = (env_lum(value1) * V.rowWeights[min(max(yPos, 0), H - 1)] +
           env_lum(value2) * V.rowWeights[min(max(yPos + 1, 0), H - 1)]) * V.E->normalization;
    float sinPhi, cosPhi, sinTheta, cosTheta;
    mt_sincosf(V.E->pixel_size[0] * (px + 0.5f), &sinPhi, &cosPhi);
    mt_sincosf(V.E->pixel_size[1] * (py + 0.5f), &sinTheta, &cosTheta);
    d = mk3(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
    pdf /= fmaxf(fabsf(sinTheta), kEpsilon);
}

// internalPdfDirection (envmap.cpp:603-633), local direction d and its env_uv
DEV float env_internal_pdf_uv(const DevEnv &V, float3 d, float ux, float uy) {
    const int W = V.E->mip.level_w[0], H = V.E->mip.level_h[0];
    const DevMip M = env_mip(V);
    if (!isfinite(ux) || !isfinite(uy)) return 0.0f;
    const float u = ux * W - 0.5f, v = uy * H - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    const float3 value1 = mip_texel(M, 0, xPos, yPos) * dx2 * dy2 + mip_texel(M, 0, xPos + 1, yPos) * dx1 * dy2;
    const float3 value2 = mip_texel(M, 0, xPos, yPos + 1) * dx2 * dy1 + mip_texel(M, 0, xPos + 1, yPos + 1) * dx1 * dy1;
    const float sinTheta = sqrtf(fmaxf(0.0f, 1 - d.y * d.y));
    return (env_lum(value1) * V.rowWeights[min(max(yPos, 0), H - 1)] +
            env_lum(value2) * V.rowWeights[min(max(yPos + 1, 0), H - 1)]) *
           V.E->normalization / fmaxf(fabsf(sinTheta), kEpsilon);
}
DEV float env_internal_pdf(const DevEnv &V, float3 d) {
    float ux, uy;
    env_uv(d, ux, uy);
    return env_internal_pdf_uv(V, d, ux, uy);
}

// BSphere::rayIntersect + solveQuadratic (bsphere.h:88-95, util.cpp:447-485)
DEV bool env_sphere(const DevEnv &V, float3 o, float3 d, float &nearT, float &farT) {
    const float3 oc = o - ld3(V.E->bsphere_center);
    const float A = dot(d, d), B = 2 * dot(oc, d), C = dot(oc, oc) - V.E->bsphere_radius * V.E->bsphere_radius;
    if (A == 0) {
        if (B != 0) { nearT = farT = -C / B; return true; }
        return false;
    }
    const float discrim = B * B - 4.0f * A * C;
    if (discrim < 0) return false;
    const float sq = sqrtf(discrim), temp = B < 0 ? -0.5f * (B - sq) : -0.5f * (B + sq);
    nearT = temp / A;
    farT = C / temp;
    if (nearT > farT) { const float t = nearT; nearT = farT; farT = t; }
    return true;
}

// EnvironmentMap::sampleDirect (envmap.cpp:516-543): world direction, distance
// to the bounding sphere, value / pdf; false when the sample is rejected
DEV bool env_sample_direct(const DevEnv &V, float3 ref, float sx, float sy, float3 &dWorld, float &dist, float3 &valueOverPdf,
                           float &pdf) {
    float3 dl, value;
    env_internal_sample(V, sx, sy, dl, value, pdf);
    dWorld = env_rot(V.E->to_world, dl);   // Ray(ref, trafo(d), 0): direction used as is
    float nearT, farT;
    if (isZero(value) || pdf == 0 || !env_sphere(V, ref, dWorld, nearT, farT) || nearT >= 0 || farT <= 0) return false;
    dist = farT;
    valueOverPdf = value / pdf;
    return true;
}

}  // namespace mtsg
