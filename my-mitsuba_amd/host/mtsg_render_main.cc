// mtsg-render: command-line front end mirroring `mitsuba scene.xml`
// (src/mitsuba/mitsuba.cpp:154-418) for the `path` integrator on MI355X:
//   mtsg-render [-D name=value]... [-o out.pfm] [-g gpus] scene.xml
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mtsg.h"
#include "../../include/mtsh.h"

#include "../../include/mtsg_path.h"

int main(int argc, char **argv) {
    std::vector<std::string> defs;
    std::string out = "out.pfm", scenePath;
    int gpus = 0;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "-D" && i + 1 < argc) defs.push_back(argv[++i]);
        else if (a == "-o" && i + 1 < argc) out = argv[++i];
        else if (a == "-g" && i + 1 < argc) gpus = atoi(argv[++i]);
        else if (a == "-h" || a == "--help") {
            printf("usage: %s [-D name=value]... [-o out.pfm] [-g gpus] scene.xml\n", argv[0]);
            return 0;
        } else scenePath = a;
    }
    if (scenePath.empty()) { fprintf(stderr, "no scene given\n"); return 1; }
    std::vector<const char *> dp;
    for (auto &d : defs) dp.push_back(d.c_str());
    mtsh_scene *s = mtsh_scene_load(scenePath.c_str(), dp.data(), (int)dp.size());
    if (!s) {
        char buf[1024];
        mtsh_last_error(buf, sizeof(buf));
        fprintf(stderr, "Error while loading \"%s\": %s\n", scenePath.c_str(), buf);
        return 2;
    }
    mtsh_scene_info info;
    mtsh_scene_get_info(s, &info);
    printf("Loaded %u triangles, %u rectangles; kd-tree %u nodes (depth %u) in %.2f s\n", info.n_triangles,
           info.n_rects, info.kd_nodes, info.kd_max_depth, info.kd_build_seconds);
    mtsg_render_params p;
    mtsh_scene_render_params(s, &p);
    const int b = info.border;
    const size_t W = (size_t)p.tile_w + 2 * b, H = (size_t)p.tile_h + 2 * b;
    std::vector<float> block(W * H * 5);
    double secs = 0;
    int rc = mtsh_path_render(s, &p, gpus, block.data(), &secs);
    if (rc != MTSG_OK) {
        char buf[1024];
        mtsg_last_error(buf, sizeof(buf));
        fprintf(stderr, "render failed (%d): %s\n", rc, buf);
        return 3;
    }
    double samples = (double)p.tile_w * p.tile_h * p.spp;
    printf("Rendering finished: %.3f s, %.1f Msamples/s\n", secs, samples / secs * 1e-6);
    // crop the border (film = crop window) and develop
    std::vector<float> crop((size_t)p.tile_w * p.tile_h * 5), rgb((size_t)p.tile_w * p.tile_h * 3);
    for (int y = 0; y < p.tile_h; ++y)
        memcpy(&crop[(size_t)y * p.tile_w * 5], &block[((size_t)(y + b) * W + b) * 5], (size_t)p.tile_w * 5 * sizeof(float));
    mtsh_develop(crop.data(), p.tile_w, p.tile_h, rgb.data());
    if (mtsh_write_pfm(out.c_str(), p.tile_w, p.tile_h, rgb.data()) != 0) { fprintf(stderr, "cannot write %s\n", out.c_str()); return 4; }
    printf("Wrote %s\n", out.c_str());
    mtsh_scene_free(s);
    return 0;
}
