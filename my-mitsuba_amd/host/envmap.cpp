// Environment emitter preprocessing (host side, shared by the GPU upload and
// the CPU oracle through mtsg_scene_desc):
//
//   MIP pyramid      buildMipmap (mipmap.cpp): TMIPMap with u repeating, v
//                    clamped, levels clamped to [0, inf)
//   sampling CDFs    EnvironmentMap::configure (src/emitters/envmap.cpp:256-306)
//   bounding sphere  EnvironmentMap::createShape (envmap.cpp:318-325) over the
//                    scene AABB = kd-tree AABB + sensor position
//                    (src/librender/scene.cpp:410-441)
#include <cmath>
#include <cstring>
#include <limits>
#include <stdexcept>

#include "scene.h"

namespace mtsh {
namespace {

inline float luminance(float r, float g, float b) { return r * 0.212671f + g * 0.715160f + b * 0.072169f; }

}  // namespace

void buildEnvmap(const Emitter &e, const float aabbMin[3], const float aabbMax[3], const float camPos[3],
                 std::vector<float> &texels, std::vector<float> &cdfRows, std::vector<float> &cdfCols,
                 std::vector<float> &rowWeights, mtsg_envmap &env) {
    memset(&env, 0, sizeof(env));
    const int W = e.width, H = e.height;
    // RGB pyramid: EWA, u repeats, v clamps, maximum anisotropy 10,
    // resampled levels clamped to [0, inf) (envmap.cpp:154-180; mipmap.cpp)
    texels.clear();
    buildMipmap(e.rgb, W, H, MTSG_MIP_EWA, MTSG_WRAP_REPEAT, MTSG_WRAP_CLAMP, std::numeric_limits<float>::infinity(), 10.0f,
                texels, env.mip, nullptr, nullptr);
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
