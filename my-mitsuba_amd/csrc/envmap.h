// Environment emitter on the device (src/emitters/envmap.cpp:99-660 and
// TMIPMap, include/mitsuba/render/mipmap.h:503-840).  Tables are built on the
// host (my-mitsuba_amd/host/envmap.cpp) and uploaded as-is: an RGB MIP
// pyramid with half-rounded texels, the row/column sampling CDFs and the
// scene bounding sphere.
#pragma once
#include "device_math.h"
#include "../../include/mtsg.h"

namespace mtsg {

constexpr float kInvTwoPi = 0.15915494309189533577f;   // constants.h:65

struct DevEnv {
    const mtsg_envmap *E;        // device copy of the table header
    const float *texels;         // RGB, all levels
    const float *cdfRows, *cdfCols, *rowWeights;
};

DEV int env_modulo(int a, int b) { int r = a % b; return r < 0 ? r + b : r; }

// evalTexel: u repeats, v clamps (mipmap.h:503-562)
DEV float3 env_texel(const DevEnv &V, int level, int x, int y) {
    const int w = V.E->level_w[level], h = V.E->level_h[level];
    if (x < 0 || x >= w) x = env_modulo(x, w);
    if (y < 0 || y >= h) y = min(max(y, 0), h - 1);
    const float *t = V.texels + V.E->level_offset[level] + 3 * ((size_t)y * w + x);
    return mk3(t[0], t[1], t[2]);
}

DEV float3 env_box(const DevEnv &V, int level, float u, float v) {   // mipmap.h:566-569
    return env_texel(V, level, (int)floorf(u * V.E->level_w[level]), (int)floorf(v * V.E->level_h[level]));
}

// evalBilinear (mipmap.h:575-596)
DEV float3 env_bilinear(const DevEnv &V, int level, float ux, float uy) {
    if (!isfinite(ux) || !isfinite(uy)) return mk3(0, 0, 0);
    if (level >= V.E->levels) return env_box(V, V.E->levels - 1, ux, uy);
    const float u = ux * V.E->level_w[level] - 0.5f, v = uy * V.E->level_h[level] - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    return env_texel(V, level, xPos, yPos) * dx2 * dy2 + env_texel(V, level, xPos, yPos + 1) * dx2 * dy1 +
           env_texel(V, level, xPos + 1, yPos) * dx1 * dy2 + env_texel(V, level, xPos + 1, yPos + 1) * dx1 * dy1;
}

// evalEWA (mipmap.h:775-840)
DEV float3 env_ewa(const DevEnv &V, int level, float ux, float uy, float A, float B, float C) {
    if (!isfinite(A + B + C + ux + uy)) return mk3(0, 0, 0);
    if (level >= V.E->levels) return env_box(V, V.E->levels - 1, ux, uy);
    const float u = ux * V.E->level_w[level] - 0.5f, v = uy * V.E->level_h[level] - 0.5f;
    const float rx = V.E->size_ratio_x[level], ry = V.E->size_ratio_y[level];
    A /= rx * rx;
    B /= rx * ry;
    C /= ry * ry;
    const float invDet = 1.0f / (-B * B + 4.0f * A * C), deltaU = 2.0f * sqrtf(C * invDet), deltaV = 2.0f * sqrtf(A * invDet);
    const int u0 = (int)ceilf(u - deltaU), u1 = (int)floorf(u + deltaU);
    const int v0 = (int)ceilf(v - deltaV), v1 = (int)floorf(v + deltaV);
    const float As = A * MTSG_MIPMAP_LUT_SIZE, Bs = B * MTSG_MIPMAP_LUT_SIZE, Cs = C * MTSG_MIPMAP_LUT_SIZE;
    float3 result = mk3(0, 0, 0);
    float denominator = 0.0f;
    const float ddq = 2 * As, uu0 = (float)u0 - u;
    for (int vt = v0; vt <= v1; ++vt) {
        const float vv = (float)vt - v;
        float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
        float dq = As * (2 * uu0 + 1) + Bs * vv;
        for (int ut = u0; ut <= u1; ++ut) {
            if (q < (float)MTSG_MIPMAP_LUT_SIZE) {
                const uint32_t qi = (uint32_t)q;
                if (qi < MTSG_MIPMAP_LUT_SIZE) {
                    const float weight = V.E->weight_lut[(int)q];
                    result += env_texel(V, level, ut, vt) * weight;
                    denominator += weight;
                }
            }
            q += dq;
            dq += ddq;
        }
    }
    if (denominator == 0) return env_bilinear(V, level, ux, uy);
    return result / denominator;
}

DEV float hypot2_env(float a, float b) {   // math.cpp:74-86
    float r;
    if (fabsf(a) > fabsf(b)) { r = b / a; r = fabsf(a) * sqrtf(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = fabsf(b) * sqrtf(1.0f + r * r); }
    else r = 0.0f;
    return r;
}

DEV float log2_m(float v) { return logf(v) * (1.0f / 0.69314718055994530942f); }   // math.cpp:103-106

// TMIPMap::eval with EEWA (mipmap.h:633-722)
DEV float3 env_filtered(const DevEnv &V, float ux, float uy, float d0x, float d0y, float d1x, float d1y) {
    const float w0 = (float)V.E->level_w[0], h0 = (float)V.E->level_h[0];
    const float du0 = d0x * w0, dv0 = d0y * h0, du1 = d1x * w0, dv1 = d1y * h0;
    float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1, F = A * C - B * B * 0.25f;
    const float root = hypot2_env(A - C, B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root);
    float majorRadius = Aprime != 0 ? sqrtf(F / Aprime) : 0, minorRadius = Cprime != 0 ? sqrtf(F / Cprime) : 0;
    if (!(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
        const float level = log2_m(fmaxf(majorRadius, kEpsilon));
        const int ilevel = (int)floorf(level);
        if (ilevel < 0) return env_bilinear(V, 0, ux, uy);
        const float a = level - ilevel;
        return env_bilinear(V, ilevel, ux, uy) * (1.0f - a) + env_bilinear(V, ilevel + 1, ux, uy) * a;
    }
    if (minorRadius * V.E->max_anisotropy < majorRadius) {
        minorRadius = majorRadius / V.E->max_anisotropy;
        const float theta = 0.5f * atanf(B / (A - C));
        float sinTheta, cosTheta;
        sincosf(theta, &sinTheta, &cosTheta);
        const float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
                    cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
        A = a2 * cosTheta2 + b2 * sinTheta2;
        B = (a2 - b2) * sin2Theta;
        C = a2 * sinTheta2 + b2 * cosTheta2;
        F = a2 * b2;
    }
    const float scale = 1.0f / F;
    A *= scale; B *= scale; C *= scale;
    const float level = fmaxf(0.0f, log2_m(minorRadius));
    const int ilevel = (int)level;
    const float a = level - ilevel;
    if (majorRadius < 1 || !(A > 0 && C > 0)) return env_bilinear(V, ilevel, ux, uy);
    return env_ewa(V, ilevel, ux, uy, A, B, C) * (1.0f - a) + env_ewa(V, ilevel + 1, ux, uy, A, B, C) * a;
}

DEV float3 env_rot(const float *m, float3 v) {
    return mk3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z, m[6] * v.x + m[7] * v.y + m[8] * v.z);
}

// EnvironmentMap::evalEnvironment (envmap.cpp:380-410); hasDiff: camera
// rays carrying (scaled) differentials -> EWA, otherwise bilinear level 0
DEV float3 env_eval(const DevEnv &V, float3 dWorld, bool hasDiff, float3 rxD, float3 ryD) {
    const float3 v = env_rot(V.E->to_local, dWorld);
    const float ux = atan2f(v.x, -v.z) * kInvTwoPi, uy = acosf(fminf(1.0f, fmaxf(-1.0f, v.y))) * kInvPi;
    float3 value;
    if (!hasDiff) {
        value = env_bilinear(V, 0, ux, uy);
    } else {
        const float3 dvdx = env_rot(V.E->to_local, rxD) - v, dvdy = env_rot(V.E->to_local, ryD) - v;
        const float t1 = kInvTwoPi / (v.x * v.x + v.z * v.z), t2 = -kInvPi / fmaxf(sqrtf(fmaxf(0.0f, 1.0f - v.y * v.y)), kEpsilon);
        value = env_filtered(V, ux, uy, t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y, t1 * (dvdy.z * v.x - dvdy.x * v.z),
                             t2 * dvdy.y);
    }
    return value * V.E->scale;
}

DEV float env_lum(float3 c) { return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f; }

// std::lower_bound-based sampleReuse (envmap.cpp:628-633)
DEV uint32_t env_sample_reuse(const float *cdf, uint32_t size, float &sample) {
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

DEV float env_tent(float sample) {   // warp.cpp:143-155
    float sign;
    if (sample < 0.5f) { sign = 1; sample *= 2; }
    else { sign = -1; sample = 2 * (sample - 0.5f); }
    return sign * (1 - sqrtf(sample));
}

// internalSampleDirection (envmap.cpp:574-600): local direction, value, pdf
DEV void env_internal_sample(const DevEnv &V, float sx, float sy, float3 &d, float3 &value, float &pdf) {
    const int W = V.E->level_w[0], H = V.E->level_h[0];
    const uint32_t row = env_sample_reuse(V.cdfRows, (uint32_t)H, sy);
    const uint32_t col = env_sample_reuse(V.cdfCols + row * (uint32_t)(W + 1), (uint32_t)W, sx);
    const float px = (float)col + env_tent(sx), py = (float)row + env_tent(sy);
    const int xPos = (int)floorf(px), yPos = (int)floorf(py);
    const float dx1 = px - xPos, dx2 = 1.0f - dx1, dy1 = py - yPos, dy2 = 1.0f - dy1;
    const float3 value1 = env_texel(V, 0, xPos, yPos) * dx2 * dy2 + env_texel(V, 0, xPos + 1, yPos) * dx1 * dy2;
    const float3 value2 = env_texel(V, 0, xPos, yPos + 1) * dx2 * dy1 + env_texel(V, 0, xPos + 1, yPos + 1) * dx1 * dy1;
    value = (value1 + value2) * V.E->scale;
    pdf = (env_lum(value1) * V.rowWeights[min(max(yPos, 0), H - 1)] +
           env_lum(value2) * V.rowWeights[min(max(yPos + 1, 0), H - 1)]) * V.E->normalization;
    float sinPhi, cosPhi, sinTheta, cosTheta;
    sincosf(V.E->pixel_size[0] * (px + 0.5f), &sinPhi, &cosPhi);
    sincosf(V.E->pixel_size[1] * (py + 0.5f), &sinTheta, &cosTheta);
    d = mk3(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
    pdf /= fmaxf(fabsf(sinTheta), kEpsilon);
}

// internalPdfDirection (envmap.cpp:603-633), local direction
DEV float env_internal_pdf(const DevEnv &V, float3 d) {
    const int W = V.E->level_w[0], H = V.E->level_h[0];
    const float ux = atan2f(d.x, -d.z) * kInvTwoPi, uy = acosf(fminf(1.0f, fmaxf(-1.0f, d.y))) * kInvPi;
    if (!isfinite(ux) || !isfinite(uy)) return 0.0f;
    const float u = ux * W - 0.5f, v = uy * H - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    const float3 value1 = env_texel(V, 0, xPos, yPos) * dx2 * dy2 + env_texel(V, 0, xPos + 1, yPos) * dx1 * dy2;
    const float3 value2 = env_texel(V, 0, xPos, yPos + 1) * dx2 * dy1 + env_texel(V, 0, xPos + 1, yPos + 1) * dx1 * dy1;
    const float sinTheta = sqrtf(fmaxf(0.0f, 1 - d.y * d.y));
    return (env_lum(value1) * V.rowWeights[min(max(yPos, 0), H - 1)] +
            env_lum(value2) * V.rowWeights[min(max(yPos + 1, 0), H - 1)]) *
           V.E->normalization / fmaxf(fabsf(sinTheta), kEpsilon);
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
