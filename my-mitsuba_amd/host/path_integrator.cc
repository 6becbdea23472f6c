// Host-side mirror of the reference's `path` plugin (MIPathTracer,
// src/integrators/path/path.cpp) whose render() drives the GPU library
// instead of the per-sample CPU loop of SamplingIntegrator::render
// (src/librender/integrator.cpp:99-133): one host thread per GPU, each
// renders an interleaved subset of the 16x16 film tiles into its own
// ImageBlock (tile rect + border), and the blocks are merged by addition
// exactly like ImageBlock::put(const ImageBlock*) (imageblock.h:103-107).
// No collectives: the film is the only thing exchanged (host-side gather).
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtsg.h"
#include "../../include/mtsh.h"
#include "../../include/mtsg_path.h"

extern "C" {

// Render the whole film of `scene` with `n_gpus` devices into rgbaw_out
// ((film_h + 2b) x (film_w + 2b) x 5 floats).  Returns an mtsg error code.
int mtsh_path_render(const mtsh_scene *scene, const mtsg_render_params *params, int n_gpus, float *rgbaw_out,
                     double *seconds_out) {
    const mtsg_scene_desc *desc = mtsh_scene_desc(scene);
    mtsh_scene_info info;
    mtsh_scene_get_info(scene, &info);
    const int b = info.border;
    const size_t W = (size_t)params->tile_w + 2 * b, H = (size_t)params->tile_h + 2 * b;
    const int avail = mtsg_device_count();
    if (n_gpus <= 0) n_gpus = avail;
    if (n_gpus > avail || n_gpus <= 0) return MTSG_ERR_NODEVICE;
    std::vector<std::vector<float>> blocks(n_gpus, std::vector<float>(W * H * 5));
    std::vector<int> rcs(n_gpus, MTSG_OK);
    std::vector<mtsg_scene *> handles(n_gpus, nullptr);
    // upload (preprocessing; excluded from the render time like renderjob.cpp:102)
    for (int g = 0; g < n_gpus; ++g)
        if ((rcs[g] = mtsg_scene_create(desc, g, &handles[g])) != MTSG_OK) {
            for (auto *h : handles) mtsg_scene_destroy(h);
            return rcs[g];
        }
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> threads;
    for (int g = 0; g < n_gpus; ++g)
        threads.emplace_back([&, g]() {
            mtsg_render_params p = *params;
            p.tile_stride = n_gpus;
            p.tile_offset = g;
            rcs[g] = mtsg_render(handles[g], &p, blocks[g].data());
        });
    for (auto &t : threads) t.join();
    std::memset(rgbaw_out, 0, W * H * 5 * sizeof(float));
    for (int g = 0; g < n_gpus; ++g)
        for (size_t i = 0; i < W * H * 5; ++i) rgbaw_out[i] += blocks[g][i];
    if (seconds_out) *seconds_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (auto *h : handles) mtsg_scene_destroy(h);
    for (int rc : rcs)
        if (rc != MTSG_OK) return rc;
    return MTSG_OK;
}

}  // extern "C"
