// Environment emitter preprocessing (host side, shared by the GPU upload and
// the CPU oracle through mtsg_scene_desc):
//
//   MIP pyramid      TMIPMap constructor (include/mitsuba/render/mipmap.h:155-302):
//                    level k+1 = Bitmap::resample of level k with a 2-lobe
//                    Lanczos filter, u repeating / v clamped, results clamped
//                    to [0, inf) (src/libcore/bitmap.cpp:2230-2330 driving
//                    Resampler, include/mitsuba/core/rfilter.h:107-330); every
//                    level is stored in half precision (SpectrumHalf), while
//                    the next level is computed from the float bitmap.
//   sampling CDFs    EnvironmentMap::configure (src/emitters/envmap.cpp:256-306)
//   bounding sphere  EnvironmentMap::createShape (envmap.cpp:318-325) over the
//                    scene AABB = kd-tree AABB + sensor position
//                    (src/librender/scene.cpp:410-441)
//   EWA weights      mipmap.h:296-301
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "scene.h"

namespace mtsh {
namespace {

// IEEE binary16 round trip, round-to-nearest-even (OpenEXR's half(float)).
float toHalfAndBack(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = x & 0x80000000u;
    const uint32_t ax = x & 0x7FFFFFFFu;
    uint16_t h;
    if (ax >= 0x7F800000u) {                       // inf / nan
        h = (uint16_t)(ax > 0x7F800000u ? 0x7E00 : 0x7C00);
    } else if (ax >= 0x477FF000u) {                // rounds to >= 65520 -> inf
        h = 0x7C00;
    } else if (ax < 0x38800000u) {                 // half subnormal / zero
        if (ax < 0x33000000u) {
            h = 0;
        } else {
            const uint32_t e = ax >> 23, m = (ax & 0x7FFFFFu) | 0x800000u;
            const uint32_t shift = 126 - e;        // 14 - (e - 112)
            uint32_t hm = m >> shift;
            const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
            if (rem > half || (rem == half && (hm & 1u))) ++hm;
            h = (uint16_t)hm;
        }
    } else {
        uint32_t v = ax - 0x38000000u;             // rebias exponent 127 -> 15
        const uint32_t rem = v & 0x1FFFu;
        v >>= 13;
        if (rem > 0x1000u || (rem == 0x1000u && (v & 1u))) ++v;
        h = (uint16_t)v;
    }
    // back to float
    const uint32_t he = (h >> 10) & 0x1Fu, hm = h & 0x3FFu;
    uint32_t out;
    if (he == 0) {
        if (hm == 0) {
            out = 0;
        } else {                                   // subnormal
            int e = -1;
            uint32_t m = hm;
            do { ++e; m <<= 1; } while (!(m & 0x400u));
            out = ((uint32_t)(127 - 15 - e) << 23) | ((m & 0x3FFu) << 13);
        }
    } else if (he == 31) {
        out = 0x7F800000u | (hm << 13);
    } else {
        out = ((he + 112) << 23) | (hm << 13);
    }
    out |= sign;
    float r;
    memcpy(&r, &out, 4);
    return r;
}

// LanczosSincFilter::eval (src/rfilters/lanczos.cpp:44-56), lobes = 2
float lanczos2(float x) {
    const float radius = 2.0f;
    x = std::fabs(x);
    if (x < 1e-4f) return 1.0f;        // Epsilon
    if (x > radius) return 0.0f;
    const float x1 = (float)(M_PI * x);
    const float x2 = x1 / radius;
    return (std::sin(x1) * std::sin(x2)) / (x1 * x2);
}

enum { BC_CLAMP = 0, BC_REPEAT = 1 };

// Resampler<float> in resampling mode + resampleAndClamp(min 0, max inf)
struct Resampler1D {
    int src, dst, taps, bc;
    std::vector<int> start;
    std::vector<float> w;
    Resampler1D(int sourceRes, int targetRes, int bc_) : src(sourceRes), dst(targetRes), bc(bc_) {
        float filterRadius = 2.0f, scale = 1.0f, invScale = 1.0f;
        if (targetRes < sourceRes) {
            scale = (float)sourceRes / (float)targetRes;
            invScale = 1 / scale;
            filterRadius *= scale;
        }
        taps = (int)std::ceil(filterRadius * 2);
        start.resize(targetRes);
        w.resize((size_t)taps * targetRes);
        for (int i = 0; i < targetRes; ++i) {
            const float center = (i + 0.5f) / targetRes * sourceRes;
            start[i] = (int)std::floor(center - filterRadius + 0.5f);
            float sum = 0;
            for (int j = 0; j < taps; ++j) {
                const float pos = start[i] + j + 0.5f - center;
                const float weight = lanczos2(pos * invScale);
                w[(size_t)i * taps + j] = weight;
                sum += weight;
            }
            const float normalization = 1.0f / sum;
            for (int j = 0; j < taps; ++j) w[(size_t)i * taps + j] = w[(size_t)i * taps + j] * normalization;
        }
    }
    int lookupIndex(int pos) const {
        if (pos < 0 || pos >= src) {
            if (bc == BC_CLAMP) pos = std::min(std::max(pos, 0), src - 1);
            else { pos %= src; if (pos < 0) pos += src; }   // math::modulo
        }
        return pos;
    }
    // source/target: element i at base + stride * i, 3 channels each
    void run(const float *source, size_t srcStride, float *target, size_t dstStride) const {
        for (int i = 0; i < dst; ++i)
            for (int ch = 0; ch < 3; ++ch) {
                float result = 0;
                for (int j = 0; j < taps; ++j)
                    result += source[srcStride * lookupIndex(start[i] + j) + ch] * w[(size_t)i * taps + j];
                target[dstStride * i + ch] = std::max(0.0f, result);   // min(inf, max(0, .))
            }
    }
};

// Bitmap::resample(lanczos2, Repeat (x), Clamp (y), size, 0, inf)
std::vector<float> resample(const std::vector<float> &src, int sw, int sh, int tw, int th) {
    std::vector<float> tmp;
    const std::vector<float> *cur = &src;
    int cw = sw;
    if (sw != tw) {
        Resampler1D r(sw, tw, BC_REPEAT);
        tmp.assign((size_t)tw * sh * 3, 0.0f);
        for (int y = 0; y < sh; ++y) r.run(src.data() + (size_t)y * sw * 3, 3, tmp.data() + (size_t)y * tw * 3, 3);
        cur = &tmp;
        cw = tw;
    }
    if (sh == th) return *cur;
    Resampler1D r(sh, th, BC_CLAMP);
    std::vector<float> out((size_t)cw * th * 3, 0.0f);
    for (int x = 0; x < cw; ++x) r.run(cur->data() + (size_t)x * 3, (size_t)cw * 3, out.data() + (size_t)x * 3, (size_t)cw * 3);
    return out;
}

inline float luminance(float r, float g, float b) { return r * 0.212671f + g * 0.715160f + b * 0.072169f; }

}  // namespace

void buildEnvmap(const Emitter &e, const float aabbMin[3], const float aabbMax[3], const float camPos[3],
                 std::vector<float> &texels, std::vector<float> &cdfRows, std::vector<float> &cdfCols,
                 std::vector<float> &rowWeights, mtsg_envmap &env) {
    memset(&env, 0, sizeof(env));
    const int W = e.width, H = e.height;
    // level 0: negative values are clamped (mipmap.h:232-240)
    std::vector<float> level(e.rgb);
    for (auto &v : level) if (v < 0) v = 0;
    // level count (mipmap.h:183-192)
    int levels = 1;
    {
        int w = W, h = H;
        while (w > 1 || h > 1) { w = std::max(1, (w + 1) / 2); h = std::max(1, (h + 1) / 2); ++levels; }
    }
    if (levels > MTSG_ENVMAP_MAX_LEVELS) throw std::runtime_error("envmap: too many MIP levels");
    env.levels = levels;
    texels.clear();
    int w = W, h = H;
    for (int l = 0; l < levels; ++l) {
        if (l > 0) {
            const int nw = std::max(1, (w + 1) / 2), nh = std::max(1, (h + 1) / 2);
            level = resample(level, w, h, nw, nh);
            w = nw; h = nh;
        }
        env.level_w[l] = w;
        env.level_h[l] = h;
        env.level_offset[l] = (uint32_t)texels.size();
        env.size_ratio_x[l] = (float)w / (float)W;
        env.size_ratio_y[l] = (float)h / (float)H;
        for (float v : level) texels.push_back(toHalfAndBack(v));   // SpectrumHalf storage
    }
    // sampling CDFs over the stored (half) level 0 (envmap.cpp:262-306)
    cdfCols.assign((size_t)(W + 1) * H, 0.0f);
    cdfRows.assign((size_t)H + 1, 0.0f);
    rowWeights.assign(H, 0.0f);
    size_t colPos = 0, rowPos = 0;
    float rowSum = 0.0f;
    cdfRows[rowPos++] = 0;
    for (int y = 0; y < H; ++y) {
        float colSum = 0;
        cdfCols[colPos++] = 0;
        for (int x = 0; x < W; ++x) {
            const float *t = &texels[((size_t)y * W + x) * 3];
            colSum += luminance(t[0], t[1], t[2]);
            cdfCols[colPos++] = colSum;
        }
        const float normalization = 1.0f / colSum;
        for (int x = 1; x < W; ++x) cdfCols[colPos - x - 1] *= normalization;
        cdfCols[colPos - 1] = 1.0f;
        const float weight = (float)std::sin((y + 0.5f) * M_PI / H);
        rowWeights[y] = weight;
        rowSum += colSum * weight;
        cdfRows[rowPos++] = rowSum;
    }
    {
        const float normalization = 1.0f / rowSum;
        for (int y = 1; y < H; ++y) cdfRows[rowPos - y - 1] *= normalization;
        cdfRows[rowPos - 1] = 1.0f;
    }
    if (rowSum == 0) throw std::runtime_error("The environment map is completely black -- this is not allowed.");
    if (!std::isfinite(rowSum)) throw std::runtime_error("The environment map contains an invalid floating point value (nan/inf) -- giving up.");
    env.normalization = (float)(1.0 / (rowSum * (2 * M_PI / W) * (M_PI / H)));
    env.pixel_size[0] = (float)(2 * M_PI / W);
    env.pixel_size[1] = (float)(M_PI / H);
    env.scale = e.scale;
    env.max_anisotropy = 10.0f;
    for (int i = 0; i < MTSG_MIPMAP_LUT_SIZE; ++i) {
        const float r2 = (float)i / (float)(MTSG_MIPMAP_LUT_SIZE - 1);
        env.weight_lut[i] = (float)std::exp((double)(-2.0f * r2)) - (float)std::exp(-2.0);
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            env.to_world[3 * r + c] = e.toWorld.m[r][c];
            env.to_local[3 * r + c] = e.toWorld.inv[r][c];
        }
    // scene bounding sphere x 1.5
    float mn[3], mx[3], center[3];
    for (int k = 0; k < 3; ++k) {
        mn[k] = std::min(aabbMin[k], camPos[k]);
        mx[k] = std::max(aabbMax[k], camPos[k]);
        center[k] = (mn[k] + mx[k]) * 0.5f;
    }
    const float dx = center[0] - mx[0], dy = center[1] - mx[1], dz = center[2] - mx[2];
    const float radius = std::sqrt(dx * dx + dy * dy + dz * dz);
    for (int k = 0; k < 3; ++k) env.bsphere_center[k] = center[k];
    env.bsphere_radius = std::max(1e-4f, radius * 1.5f);
}

}  // namespace mtsh
