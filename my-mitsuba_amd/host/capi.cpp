// extern "C" surface of the host-side scene library (include/mtsh.h).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mtsh.h"
#include "digest.h"
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
    return mtsh_scene_load_props(path, defines, n_defines, overrides, nullptr, 0);
}
}  // extern "C"
namespace {
mtsh::Properties toProps(const mtsh_prop *p, int32_t n, std::map<std::string, int> *textures = nullptr);
}
extern "C" {
mtsh_scene *mtsh_scene_load_props(const char *path, const char *const *defines, int n_defines,
                                  const mtsh_scene_overrides *overrides, const mtsh_prop *scene_props, int32_t n_scene_props) {
    try {
        std::map<std::string, std::string> defs;
        for (int i = 0; i < n_defines; ++i) {
            std::string d = defines[i];
            size_t eq = d.find('=');
            if (eq == std::string::npos) throw std::runtime_error("define must be name=value: " + d);
            defs[d.substr(0, eq)] = d.substr(eq + 1);
        }
        auto s = std::make_unique<mtsh_scene>();
        const mtsh::Properties sp = toProps(scene_props, n_scene_props);
        s->scene = mtsh::loadScene(path, defs, overrides, n_scene_props > 0 ? &sp : nullptr);
        return s.release();
    } catch (const std::exception &e) {
        g_err = e.what();
        return nullptr;
    }
}

const mtsg_scene_desc *mtsh_scene_desc(const mtsh_scene *s) { return &s->scene->desc; }

}  // extern "C"

// ---- builder (the scene Mitsuba holds in memory) ----
struct mtsh_builder {
    std::unique_ptr<mtsh::Scene> scene;
    std::unique_ptr<mtsh::SceneBuilder> b;
};

namespace {
// mtsh_prop list -> Properties (and a BSDF's textured parameters)
mtsh::Properties toProps(const mtsh_prop *p, int32_t n, std::map<std::string, int> *textures) {
    if (n < 0 || (n > 0 && !p)) throw std::runtime_error("invalid property list");
    mtsh::Properties props;
    for (int32_t k = 0; k < n; ++k) {
        if (!p[k].name) throw std::runtime_error("a property without a name");
        const std::string name = p[k].name;
        if (props.has(name) || (textures && textures->count(name)))
            throw std::runtime_error("Property \"" + name + "\" was specified multiple times!");
        switch (p[k].type) {
            case MTSH_PROP_BOOLEAN: props.bools[name] = p[k].i != 0; break;
            case MTSH_PROP_INTEGER: props.ints[name] = (long long)p[k].i; break;
            case MTSH_PROP_FLOAT: props.floats[name] = p[k].f; break;
            case MTSH_PROP_POINT:
            case MTSH_PROP_VECTOR: props.points[name] = mtsh::V3(p[k].v[0], p[k].v[1], p[k].v[2]); break;
            case MTSH_PROP_SPECTRUM: props.spectra[name] = mtsh::V3(p[k].v[0], p[k].v[1], p[k].v[2]); break;
            case MTSH_PROP_STRING:
                if (!p[k].s) throw std::runtime_error("string property \"" + name + "\" without a value");
                props.strings[name] = p[k].s;
                break;
            case MTSH_PROP_TRANSFORM: {
                bool haveInv = false;
                for (int j = 0; j < 16; ++j) haveInv |= p[k].inv[j] != 0.0f;
                mtsh::Transform t;
                if (haveInv) {
                    // as Mitsuba holds it: the matrix and its inverse
                    for (int j = 0; j < 16; ++j) { t.m[j / 4][j % 4] = p[k].m[j]; t.inv[j / 4][j % 4] = p[k].inv[j]; }
                } else {
                    float a[4][4];
                    for (int j = 0; j < 16; ++j) a[j / 4][j % 4] = p[k].m[j];
                    t = mtsh::Transform::fromMatrixF(a);
                }
                props.transforms[name] = t;
                break;
            }
            case MTSH_PROP_TEXTURE:
                if (!textures) throw std::runtime_error("texture property \"" + name + "\" outside a BSDF");
                (*textures)[name] = (int)p[k].i;
                break;
            default: throw std::runtime_error("property \"" + name + "\" has an unknown type");
        }
    }
    return props;
}
template <class F> int32_t guarded(mtsh_builder *b, F &&f) {
    if (!b) { g_err = "invalid builder"; return -1; }
    try {
        return f();
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}
}  // namespace

extern "C" {

mtsh_builder *mtsh_scene_begin(const char *base_dir) {
    try {
        auto b = std::make_unique<mtsh_builder>();
        b->scene = mtsh::SceneBuilder::newScene();
        b->b = std::make_unique<mtsh::SceneBuilder>(*b->scene);
        b->b->dirStack.push_back(base_dir && *base_dir ? base_dir : ".");
        return b.release();
    } catch (const std::exception &e) {
        g_err = e.what();
        return nullptr;
    }
}

int32_t mtsh_scene_add_texture(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n) {
    return guarded(b, [&] { return (int32_t)b->b->texture(plugin ? plugin : "", toProps(props, n), ""); });
}

int32_t mtsh_scene_add_bsdf(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n, const int32_t *nested,
                            int32_t n_nested) {
    return guarded(b, [&] {
        std::map<std::string, int> tex;
        mtsh::Properties pr = toProps(props, n, &tex);
        if (n_nested < 0 || (n_nested > 0 && !nested)) throw std::runtime_error("invalid nested BSDF list");
        std::vector<int> kids(nested, nested + n_nested);
        return (int32_t)b->b->bsdf(plugin ? plugin : "", pr, tex, kids, "");
    });
}

int32_t mtsh_scene_add_emitter(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n) {
    return guarded(b, [&] { return (int32_t)b->b->emitter(plugin ? plugin : "", toProps(props, n)); });
}

int32_t mtsh_scene_add_group(mtsh_builder *b, const char *id) {
    return guarded(b, [&] { return (int32_t)b->b->group(id ? id : ""); });
}

int32_t mtsh_scene_add_shape(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n, int32_t bsdf,
                             int32_t emitter, int32_t group) {
    return guarded(b, [&] {
        b->b->shape(plugin ? plugin : "", toProps(props, n), bsdf, emitter, group);
        return 0;
    });
}

int32_t mtsh_scene_add_mesh(mtsh_builder *b, const mtsh_mesh *mesh, int32_t bsdf, int32_t emitter, int32_t group) {
    return guarded(b, [&] {
        if (!mesh || !mesh->positions || !mesh->indices || !mesh->n_vertices || !mesh->n_triangles)
            throw std::runtime_error("mtsh_scene_add_mesh: a mesh needs positions and triangles");
        mtsh::Mesh m;
        m.name = mesh->name ? mesh->name : "";
        const size_t nv = mesh->n_vertices, nt = mesh->n_triangles;
        m.p.resize(nv);
        for (size_t i = 0; i < nv; ++i) m.p[i] = mtsh::V3(mesh->positions[3 * i], mesh->positions[3 * i + 1], mesh->positions[3 * i + 2]);
        if (mesh->normals && !mesh->face_normals) {
            m.n.resize(nv);
            for (size_t i = 0; i < nv; ++i) m.n[i] = mtsh::V3(mesh->normals[3 * i], mesh->normals[3 * i + 1], mesh->normals[3 * i + 2]);
        }
        if (mesh->texcoords) m.uv.assign(mesh->texcoords, mesh->texcoords + 2 * nv);
        m.idx.assign(mesh->indices, mesh->indices + 3 * nt);
        m.faceNormals = mesh->face_normals != 0;
        mtsh::Transform tw;
        if (mesh->to_world && mesh->to_world_inv) {
            for (int j = 0; j < 16; ++j) { tw.m[j / 4][j % 4] = mesh->to_world[j]; tw.inv[j / 4][j % 4] = mesh->to_world_inv[j]; }
        } else if (mesh->to_world) {
            float a[4][4];
            for (int j = 0; j < 16; ++j) a[j / 4][j % 4] = mesh->to_world[j];
            tw = mtsh::Transform::fromMatrixF(a);
        }
        b->b->mesh(std::move(m), mesh->to_world ? &tw : nullptr, mesh->flip_normals != 0, bsdf, emitter, group);
        return 0;
    });
}

int32_t mtsh_scene_add_instance(mtsh_builder *b, int32_t group, const mtsh_prop *props, int32_t n) {
    return guarded(b, [&] {
        b->b->instance(group, toProps(props, n).getTransform("toWorld", mtsh::Transform()));
        return 0;
    });
}

int32_t mtsh_scene_set_sensor(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n) {
    return guarded(b, [&] {
        b->b->sensor(plugin ? plugin : "", toProps(props, n));
        return 0;
    });
}

int32_t mtsh_scene_set_film(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n, const char *rfilter,
                            const mtsh_prop *rprops, int32_t nr) {
    return guarded(b, [&] {
        b->b->film(plugin ? plugin : "", toProps(props, n));
        if (rfilter) b->b->rfilter(rfilter, toProps(rprops, nr));
        return 0;
    });
}

int32_t mtsh_scene_set_sampler(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n) {
    return guarded(b, [&] {
        b->b->sampler(plugin ? plugin : "", toProps(props, n));
        return 0;
    });
}

int32_t mtsh_scene_set_scene_props(mtsh_builder *b, const mtsh_prop *props, int32_t n) {
    return guarded(b, [&] {
        b->b->sceneProps(toProps(props, n));
        return 0;
    });
}

int32_t mtsh_scene_set_integrator(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n) {
    return guarded(b, [&] {
        b->b->integrator(plugin ? plugin : "", toProps(props, n));
        return 0;
    });
}

mtsh_scene *mtsh_scene_finish(mtsh_builder *b, const mtsh_scene_overrides *overrides) {
    if (!b) { g_err = "invalid builder"; return nullptr; }
    std::unique_ptr<mtsh_builder> own(b);
    try {
        own->b->finish(overrides);
        auto s = std::make_unique<mtsh_scene>();
        s->scene = std::move(own->scene);
        return s.release();
    } catch (const std::exception &e) {
        g_err = e.what();
        return nullptr;
    }
}

void mtsh_scene_abort(mtsh_builder *b) { delete b; }

int32_t mtsh_scene_digest(const mtsh_scene *s, mtsh_digest_entry *out, int32_t capacity) {
    if (!s) { g_err = "invalid scene"; return -1; }
    const auto d = mtsh::sceneDigest(s->scene->desc);
    for (int32_t i = 0; out && i < (int32_t)d.size() && i < capacity; ++i) out[i] = d[i];
    return (int32_t)d.size();
}

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
