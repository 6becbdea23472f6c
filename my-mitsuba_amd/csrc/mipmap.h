// TMIPMap lookups on the device (include/mitsuba/render/mipmap.h:498-840),
// shared by the environment emitter (envmap.h) and the `bitmap` texture.
// The pyramid is built on the host (my-mitsuba_amd/host/mipmap.cpp) and
// uploaded as-is: an mtsg_mipmap header and its half-rounded RGB texels.
#pragma once
#include "device_math.h"
#include "../../include/mtsg.h"

namespace mtsg {

struct DevMip {
    const mtsg_mipmap *M;        // device copy of the header
    const float *texels;         // RGB, all levels (header offsets are relative to this)
};

DEV int mip_modulo(int a, int b) { int r = a % b; return r < 0 ? r + b : r; }   // math::modulo

// evalTexel with the boundary conditions (mipmap.h:503-562); returns false
// for EZero / EOne outside the texture (value in `c`)
DEV bool mip_wrap(int mode, int &x, int n, float &c) {
    if (x >= 0 && x < n) return true;
    switch (mode) {
        case MTSG_WRAP_REPEAT: x = mip_modulo(x, n); return true;
        case MTSG_WRAP_CLAMP: x = min(max(x, 0), n - 1); return true;
        case MTSG_WRAP_MIRROR:
            x = mip_modulo(x, 2 * n);
            if (x >= n) x = 2 * n - x - 1;
            return true;
        case MTSG_WRAP_ZERO: c = 0.0f; return false;
        default: c = 1.0f; return false;
    }
}

DEV float3 mip_texel(const DevMip &V, int level, int x, int y) {
    const int w = V.M->level_w[level], h = V.M->level_h[level];
    float c;
    if (!mip_wrap(V.M->wrap_u, x, w, c)) return mk3(c, c, c);
    if (!mip_wrap(V.M->wrap_v, y, h, c)) return mk3(c, c, c);
    const float *t = V.texels + V.M->level_offset[level] + 3 * ((size_t)y * w + x);
    return mk3(t[0], t[1], t[2]);
}

DEV float3 mip_box(const DevMip &V, int level, float u, float v) {   // mipmap.h:566-569
    return mip_texel(V, level, (int)floorf(u * V.M->level_w[level]), (int)floorf(v * V.M->level_h[level]));
}

// evalBilinear (mipmap.h:575-596)
DEV float3 mip_bilinear(const DevMip &V, int level, float ux, float uy) {
    if (!isfinite(ux) || !isfinite(uy)) return mk3(0, 0, 0);
    if (level >= V.M->levels) return mip_box(V, V.M->levels - 1, ux, uy);
    const float u = ux * V.M->level_w[level] - 0.5f, v = uy * V.M->level_h[level] - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(v);
    const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    return mip_texel(V, level, xPos, yPos) * dx2 * dy2 + mip_texel(V, level, xPos, yPos + 1) * dx2 * dy1 +
           mip_texel(V, level, xPos + 1, yPos) * dx1 * dy2 + mip_texel(V, level, xPos + 1, yPos + 1) * dx1 * dy1;
}

// evalEWA (mipmap.h:775-840)
DEV float3 mip_ewa(const DevMip &V, int level, float ux, float uy, float A, float B, float C) {
    if (!isfinite(A + B + C + ux + uy)) return mk3(0, 0, 0);
    if (level >= V.M->levels) return mip_box(V, V.M->levels - 1, ux, uy);
    const float u = ux * V.M->level_w[level] - 0.5f, v = uy * V.M->level_h[level] - 0.5f;
    const float rx = V.M->size_ratio_x[level], ry = V.M->size_ratio_y[level];
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
                    const float weight = V.M->weight_lut[(int)q];
                    result += mip_texel(V, level, ut, vt) * weight;
                    denominator += weight;
                }
            }
            q += dq;
            dq += ddq;
        }
    }
    if (denominator == 0) return mip_bilinear(V, level, ux, uy);
    return result / denominator;
}

DEV float hypot2_m(float a, float b) {   // math.cpp:74-86
    float r;
    if (fabsf(a) > fabsf(b)) { r = b / a; r = fabsf(a) * sqrtf(1.0f + r * r); }
    else if (b != 0.0f) { r = a / b; r = fabsf(b) * sqrtf(1.0f + r * r); }
    else r = 0.0f;
    return r;
}

DEV float log2_m(float v) { return mt_fastlog(v) * (1.0f / 0.69314718055994530942f); }   // math.cpp:103-106 (fastlog)

// TMIPMap::eval(uv, d0, d1): the filtered lookup (mipmap.h:633-722)
DEV float3 mip_filtered(const DevMip &V, float ux, float uy, float d0x, float d0y, float d1x, float d1y) {
    const int filter = V.M->filter;
    if (filter == MTSG_MIP_NEAREST) return mip_box(V, 0, ux, uy);
    if (filter == MTSG_MIP_BILINEAR) return mip_bilinear(V, 0, ux, uy);
    const float w0 = (float)V.M->level_w[0], h0 = (float)V.M->level_h[0];
    const float du0 = d0x * w0, dv0 = d0y * h0, du1 = d1x * w0, dv1 = d1y * h0;
    float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1, F = A * C - B * B * 0.25f;
    const float root = hypot2_m(A - C, B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root);
    float majorRadius = Aprime != 0 ? sqrtf(F / Aprime) : 0, minorRadius = Cprime != 0 ? sqrtf(F / Cprime) : 0;
    if (filter == MTSG_MIP_TRILINEAR || !(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
        const float level = log2_m(fmaxf(majorRadius, kEpsilon));
        const int ilevel = (int)floorf(level);
        if (ilevel < 0) return mip_bilinear(V, 0, ux, uy);
        const float a = level - ilevel;
        return mip_bilinear(V, ilevel, ux, uy) * (1.0f - a) + mip_bilinear(V, ilevel + 1, ux, uy) * a;
    }
    if (minorRadius * V.M->max_anisotropy < majorRadius) {
        minorRadius = majorRadius / V.M->max_anisotropy;
        const float theta = 0.5f * mt_atanf(B / (A - C));
        float sinTheta, cosTheta;
        mt_sincosf(theta, &sinTheta, &cosTheta);
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
    if (majorRadius < 1 || !(A > 0 && C > 0)) return mip_bilinear(V, ilevel, ux, uy);
    return mip_ewa(V, ilevel, ux, uy, A, B, C) * (1.0f - a) + mip_ewa(V, ilevel + 1, ux, uy, A, B, C) * a;
}

}  // namespace mtsg
