// extern "C" surface of the host-side scene library (include/mtsh.h).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mtsh.h"
#include "scene.h"

struct mtsh_scene {
    std::unique_ptr<mtsh::Scene> scene;
};

namespace {
thread_local std::string g_err;
}

extern "C" {

void mtsh_set_kd_threads(int threads) { mtsh::g_defaultKDThreads = threads; }

int mtsh_clip_triangle(const float *v, const float *box, float *out) {
    mtsh::AABB b;
    b.mn = mtsh::V3(box[0], box[1], box[2]);
    b.mx = mtsh::V3(box[3], box[4], box[5]);
    const mtsh::AABB r = mtsh::clipTriangle(mtsh::V3(v[0], v[1], v[2]), mtsh::V3(v[3], v[4], v[5]), mtsh::V3(v[6], v[7], v[8]), b);
    for (int k = 0; k < 3; ++k) { out[k] = r.mn[k]; out[3 + k] = r.mx[k]; }
    return r.valid() ? 1 : 0;
}
void mtsh_set_instancing(int mode) { mtsh::g_instancing = mode == MTSH_INSTANCING_TWO_LEVEL ? 1 : 0; }

mtsh_scene *mtsh_scene_load(const char *path, const char *const *defines, int n_defines) {
    return mtsh_scene_load_overrides(path, defines, n_defines, nullptr);
}

mtsh_scene *mtsh_scene_load_overrides(const char *path, const char *const *defines, int n_defines,
                                      const mtsh_scene_overrides *overrides) {
    try {
        std::map<std::string, std::string> defs;
        for (int i = 0; i < n_defines; ++i) {
            std::string d = defines[i];
            size_t eq = d.find('=');
            if (eq == std::string::npos) throw std::runtime_error("define must be name=value: " + d);
            defs[d.substr(0, eq)] = d.substr(eq + 1);
        }
        auto s = std::make_unique<mtsh_scene>();
        s->scene = mtsh::loadScene(path, defs, overrides);
        return s.release();
    } catch (const std::exception &e) {
        g_err = e.what();
        return nullptr;
    }
}

const mtsg_scene_desc *mtsh_scene_desc(const mtsh_scene *s) { return &s->scene->desc; }

void mtsh_scene_render_params(const mtsh_scene *s, mtsg_render_params *p) {
    memset(p, 0, sizeof(*p));
    const mtsh::Scene &sc = *s->scene;
    p->max_depth = sc.integrator.maxDepth;
    p->rr_depth = sc.integrator.rrDepth;
    p->strict_normals = sc.integrator.strictNormals;
    p->hide_emitters = sc.integrator.hideEmitters;
    p->spp = (uint32_t)sc.sampleCount;
    p->seed = 0;
    p->tile_x = sc.film.cropX;
    p->tile_y = sc.film.cropY;
    p->tile_w = sc.film.cropW;
    p->tile_h = sc.film.cropH;
    p->tile_stride = 1;
    p->tile_offset = 0;
    p->integrator = sc.integrator.type == "myPath2_OM" ? MTSG_INTEGRATOR_PATH2_OM : MTSG_INTEGRATOR_PATH;
    p->om_strategy = sc.integrator.omStrategy;
    p->om_mis = sc.integrator.omMis;
    p->om_jitter = sc.integrator.omJitter ? 1 : 0;
}

int mtsh_scene_textures(const mtsh_scene *s, mtsg_texture *out, int capacity) {
    const mtsh::Scene &sc = *s->scene;
    const int n = (int)sc.textureDesc.size();
    for (int i = 0; out && i < n && i < capacity; ++i) out[i] = sc.textureDesc[i];
    return n;
}

int64_t mtsh_scene_prim_bounds(const mtsh_scene *s, float *out, size_t capacity) {
    std::vector<float> b;
    s->scene->primBounds(b);
    if (out) {
        if (capacity < b.size()) { g_err = "mtsh_scene_prim_bounds: buffer too small"; return -2; }
        std::copy(b.begin(), b.end(), out);
    }
    return (int64_t)(b.size() / 6);
}

int mtsh_scene_set_kdtree(mtsh_scene *s, const mtsg_kdnode *nodes, uint32_t n_nodes, const uint32_t *indices, uint32_t n_indices,
                          const float *aabb_min, const float *aabb_max, uint32_t max_depth) {
    if (!s || !nodes || !n_nodes || (n_indices && !indices) || !aabb_min || !aabb_max) {
        g_err = "mtsh_scene_set_kdtree: invalid arguments";
        return -1;
    }
    const uint32_t nPrims = s->scene->desc.n_prims;
    for (uint32_t i = 0; i < n_indices; ++i)
        if (indices[i] >= nPrims) { g_err = "mtsh_scene_set_kdtree: index out of range"; return -1; }
    // the node structure (KDNode, gkdtree.h:452-600): every node reached once
    // from the root, inner children inside the array and after their parent,
    // no indirection nodes, leaf ranges inside the index list, depth within
    // max_depth -- the device traversal trusts all of it
    std::vector<uint8_t> seen(n_nodes, 0);
    std::vector<std::pair<uint32_t, uint32_t>> stack{{0u, 0u}};
    while (!stack.empty()) {
        const auto [i, depth] = stack.back();
        stack.pop_back();
        if (seen[i]) { g_err = "mtsh_scene_set_kdtree: node " + std::to_string(i) + " reached twice"; return -1; }
        seen[i] = 1;
        const uint32_t c = nodes[i].combined;
        if (c & 0x80000000u) {
            const uint32_t st = c & 0x7FFFFFFFu, en = nodes[i].data;
            if (st > en || en > n_indices) { g_err = "mtsh_scene_set_kdtree: leaf " + std::to_string(i) + " range outside the index list"; return -1; }
            continue;
        }
        if ((c & 3u) == 3u || (c & 0x40000000u)) { g_err = "mtsh_scene_set_kdtree: node " + std::to_string(i) + " is not an inner node of this encoding"; return -1; }
        const uint64_t left = (uint64_t)i + (c >> 2);
        if (left <= i || left + 1 >= n_nodes) { g_err = "mtsh_scene_set_kdtree: node " + std::to_string(i) + " has children outside the array"; return -1; }
        if (depth + 1 > max_depth) { g_err = "mtsh_scene_set_kdtree: deeper than max_depth"; return -1; }
        stack.push_back({(uint32_t)left, depth + 1});
        stack.push_back({(uint32_t)left + 1, depth + 1});
    }
    s->scene->setTree(nodes, n_nodes, indices, n_indices, aabb_min, aabb_max, max_depth);
    return 0;
}

int mtsh_scene_om(const mtsh_scene *s, mtsg_om *om, uint32_t *bits, size_t capacity) {
    const mtsh::Scene &sc = *s->scene;
    if (sc.omBits.empty()) { g_err = "the scene has no occupancy maps"; return -1; }
    if (om) *om = sc.omDesc;
    if (bits) {
        if (capacity < sc.omBits.size()) { g_err = "mtsh_scene_om: buffer too small"; return -2; }
        std::copy(sc.omBits.begin(), sc.omBits.end(), bits);
    }
    return 0;
}

void mtsh_scene_get_info(const mtsh_scene *s, mtsh_scene_info *out) {
    const mtsh::Scene &sc = *s->scene;
    memset(out, 0, sizeof(*out));
    out->n_triangles = sc.desc.n_triangles;
    out->n_rects = sc.desc.n_rects;
    out->n_shapes = sc.desc.n_shapes;
    out->n_emitters = sc.desc.n_emitters;
    out->n_bsdfs = sc.desc.n_bsdfs;
    out->kd_nodes = sc.desc.n_nodes;
    out->kd_indices = sc.desc.n_indices;
    out->kd_max_depth = sc.tree.maxDepth;
    out->kd_leaves = (uint32_t)sc.tree.leafCount;
    out->kd_nonempty_leaves = (uint32_t)sc.tree.nonEmptyLeaves;
    out->kd_build_seconds = sc.tree.buildSeconds;
    out->film_w = sc.film.width;
    out->film_h = sc.film.height;
    out->spp = sc.sampleCount;
    out->border = sc.camera.border;
    out->max_depth = sc.integrator.maxDepth;
}

void mtsh_scene_free(mtsh_scene *s) { delete s; }

void mtsh_develop(const float *rgbaw, int w, int h, float *rgb) {
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        float wt = rgbaw[5 * i + 4];
        float inv = wt != 0 ? 1.0f / wt : 0.0f;
        for (int k = 0; k < 3; ++k) rgb[3 * i + k] = rgbaw[5 * i + k] * inv;
    }
}

int mtsh_write_pfm(const char *path, int w, int h, const float *rgb) {
    try {
        std::vector<float> v(rgb, rgb + (size_t)w * h * 3);
        mtsh::writePFM(path, w, h, v);
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

int mtsh_rough_transmittance(int distribution, float alpha, float eta, int n, float *trans, float *diffuse) {
    if (n < 2 || !trans || distribution < MTSG_MF_BECKMANN || distribution > MTSG_MF_PHONG || !(alpha > 0) || !(eta > 0)) {
        g_err = "mtsh_rough_transmittance: invalid arguments";
        return -1;
    }
    mtsh::roughTransmittanceSlice(distribution, alpha, eta, n, trans);
    if (diffuse) *diffuse = mtsh::roughDiffuseTransmittance(distribution, alpha, eta);
    return 0;
}

int mtsh_read_image(const char *path, int *w, int *h, float *rgb, size_t rgb_capacity) {
    if (!path || !w || !h) { g_err = "mtsh_read_image: invalid arguments"; return -1; }
    std::string p(path), e;
    std::vector<float> img;
    const bool exr = p.size() > 4 && (p.substr(p.size() - 4) == ".exr" || p.substr(p.size() - 4) == ".EXR");
    if (!(exr ? mtsh::readEXR(p, *w, *h, img, e) : mtsh::readPFM(p, *w, *h, img, e))) { g_err = e; return -1; }
    if (rgb) {
        if (rgb_capacity < img.size()) { g_err = "mtsh_read_image: buffer too small"; return -2; }
        std::copy(img.begin(), img.end(), rgb);
    }
    return 0;
}

int mtsh_texture_image(const char *path, float gamma, int *w, int *h, float *rgb, size_t rgb_capacity) {
    if (!path || !w || !h) { g_err = "mtsh_texture_image: invalid arguments"; return -1; }
    try {
        std::vector<float> img;
        mtsh::loadTextureImage(path, gamma, *w, *h, img);
        if (rgb) {
            if (rgb_capacity < img.size()) { g_err = "mtsh_texture_image: buffer too small"; return -2; }
            std::copy(img.begin(), img.end(), rgb);
        }
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

int mtsh_build_mipmap(const float *rgb, int w, int h, int filter, int wrap_u, int wrap_v, float max_value,
                      float max_anisotropy, mtsg_mipmap *mip, float *texels, size_t texel_capacity, size_t *n_texels,
                      float *average, float *maximum) {
    if (!rgb || w <= 0 || h <= 0 || !mip || !n_texels) { g_err = "mtsh_build_mipmap: invalid arguments"; return -1; }
    try {
        std::vector<float> out;
        mtsh::buildMipmap(std::vector<float>(rgb, rgb + (size_t)w * h * 3), w, h, filter, wrap_u, wrap_v, max_value,
                          max_anisotropy, out, *mip, average, maximum);
        *n_texels = out.size();
        if (texels) {
            if (texel_capacity < out.size()) { g_err = "mtsh_build_mipmap: buffer too small"; return -2; }
            std::copy(out.begin(), out.end(), texels);
        }
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

void mtsh_last_error(char *buf, size_t size) {
    if (!size) return;
    strncpy(buf, g_err.c_str(), size - 1);
    buf[size - 1] = 0;
}

}  // extern "C"
