// The guided CDF searches of the device's envmap importance sampling
// (my-mitsuba_amd/csrc/envmap.h env_sample_reuse_guided, compiled here for the
// host) against the full std::lower_bound search (env_sample_reuse) on a
// scene's environment CDFs: the same row / column index and the same remapped
// sample for every draw.  Guide tables are built as mtsg.hip builds them.
//   tools/check_env_guide <scene.xml> [draws per CDF]
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "../my-mitsuba_amd/csrc/envmap.h"
#include "../include/mtsh.h"

using namespace mtsg;

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s scene.xml [draws]\n", argv[0]); return 2; }
    const int draws = argc > 2 ? atoi(argv[2]) : 2000;
    const char *defs[] = {"width=16", "height=16", "spp=1"};
    mtsh_scene *sc = mtsh_scene_load(argv[1], defs, 3);
    if (!sc) { char e[512]; mtsh_last_error(e, sizeof(e)); fprintf(stderr, "%s\n", e); return 2; }
    const mtsg_scene_desc *d = mtsh_scene_desc(sc);
    if (!d->has_envmap) { fprintf(stderr, "no environment map\n"); return 2; }
    const uint32_t W = (uint32_t)d->envmap.mip.level_w[0], H = (uint32_t)d->envmap.mip.level_h[0];
    auto guides = [](const float *cdf, uint32_t size, uint32_t *out) {
        for (uint32_t g = 0; g <= ENV_GUIDE; ++g)
            out[g] = (uint32_t)(std::lower_bound(cdf, cdf + size + 1, (float)g / (float)ENV_GUIDE) - cdf);
    };
    std::mt19937 rng(7);
    auto draw = [&]() { return (float)(rng() >> 9) * (1.0f / 8388608.0f); };
    uint64_t n = 0, bad = 0;
    auto check = [&](const float *cdf, uint32_t size, const uint32_t *gd, float s) {
        float a = s, b = s;
        const uint32_t i = env_sample_reuse(cdf, size, a), j = env_sample_reuse_guided(cdf, size, gd, b);
        ++n;
        if (i != j || a != b) ++bad;
    };
    std::vector<uint32_t> g(ENV_GUIDE + 1);
    guides(d->env_cdf_rows, H, g.data());
    for (int k = 0; k < draws * 64; ++k) check(d->env_cdf_rows, H, g.data(), draw());
    for (uint32_t y = 0; y < H; ++y) {
        const float *c = d->env_cdf_cols + (size_t)y * (W + 1);
        guides(c, W, g.data());
        for (int k = 0; k < draws; ++k) check(c, W, g.data(), draw());
        for (uint32_t q = 0; q < ENV_GUIDE; ++q) {   // the bucket edges
            check(c, W, g.data(), (float)q / (float)ENV_GUIDE);
            check(c, W, g.data(), std::nextafter((float)(q + 1) / (float)ENV_GUIDE, 0.0f));
        }
    }
    printf("%s: %ux%u, %d guide entries per CDF: %llu searches, %llu differ\n", argv[1], W, H, ENV_GUIDE,
           (unsigned long long)n, (unsigned long long)bad);
    mtsh_scene_free(sc);
    return bad != 0;
}
