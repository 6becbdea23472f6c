// Fingerprint of an mtsg_scene_desc (mtsh_scene_digest, include/mtsh.h):
// FNV-1a 64 of every array the descriptor points at, and of its scalar
// fields with the pointers cleared, so two routes to one scene (the XML
// loader, the in-memory builder) can be compared byte for byte.
#pragma once
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mtsg.h"
#include "../../include/mtsh.h"

namespace mtsh {

inline uint64_t fnv1a64(const void *p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    return h;
}

inline std::vector<mtsh_digest_entry> sceneDigest(const mtsg_scene_desc &d) {
    std::vector<mtsh_digest_entry> out;
    auto add = [&](const char *name, const void *p, size_t bytes) {
        mtsh_digest_entry e;
        memset(&e, 0, sizeof(e));
        strncpy(e.name, name, sizeof(e.name) - 1);
        e.bytes = p ? bytes : 0;
        e.hash = fnv1a64(p, p ? bytes : 0);
        out.push_back(e);
    };
    mtsg_scene_desc s;
    memcpy(&s, &d, sizeof(s));
    s.vtx_pos = s.vtx_nrm = s.tri_dpdu = s.emitter_cdf = s.emitter_tri_cdf = nullptr;
    s.tri_idx = s.indices = s.group_indices = nullptr;
    s.rects = nullptr; s.shapes = nullptr; s.bsdfs = nullptr; s.emitters = nullptr;
    s.nodes = s.group_nodes = nullptr; s.triaccel = nullptr;
    s.env_texels = s.env_cdf_rows = s.env_cdf_cols = s.env_row_weights = nullptr;
    s.qmc_primes = s.qmc_perm_offset = nullptr; s.qmc_perm = nullptr;
    s.sobol_matrices = nullptr; s.sobol_vdc = s.sobol_vdc_inv = nullptr;
    s.instances = nullptr; s.groups = nullptr; s.textures = nullptr;
    s.tex_texels = s.tri_uv = s.tri_dpdv = nullptr;
    s.om = nullptr; s.om_bits = nullptr;
    add("scalars", &s, sizeof(s));
    add("vtx_pos", d.vtx_pos, sizeof(float) * 3 * (size_t)d.n_vertices);
    add("vtx_nrm", d.vtx_nrm, sizeof(float) * 3 * (size_t)d.n_vertices);
    add("tri_idx", d.tri_idx, sizeof(uint32_t) * 3 * (size_t)d.n_triangles);
    add("tri_dpdu", d.tri_dpdu, sizeof(float) * 3 * (size_t)d.n_triangles);
    add("rects", d.rects, sizeof(mtsg_rect) * (size_t)d.n_rects);
    add("shapes", d.shapes, sizeof(mtsg_shape) * (size_t)d.n_shapes);
    add("bsdfs", d.bsdfs, sizeof(mtsg_bsdf) * (size_t)d.n_bsdfs);
    add("emitters", d.emitters, sizeof(mtsg_emitter) * (size_t)d.n_emitters);
    add("emitter_cdf", d.emitter_cdf, sizeof(float) * ((size_t)d.n_emitters + 1));
    add("emitter_tri_cdf", d.emitter_tri_cdf, sizeof(float) * (size_t)d.n_emitter_tri_cdf);
    add("nodes", d.nodes, sizeof(mtsg_kdnode) * (size_t)d.n_nodes);
    add("indices", d.indices, sizeof(uint32_t) * (size_t)d.n_indices);
    add("triaccel", d.triaccel, sizeof(mtsg_triaccel) * (size_t)d.n_prims);
    if (d.has_envmap) {
        const size_t w = (size_t)d.envmap.mip.level_w[0], h = (size_t)d.envmap.mip.level_h[0];
        add("env_texels", d.env_texels, sizeof(float) * (size_t)d.n_env_texels);
        add("env_cdf_rows", d.env_cdf_rows, sizeof(float) * (h + 1));
        add("env_cdf_cols", d.env_cdf_cols, sizeof(float) * (w + 1) * h);
        add("env_row_weights", d.env_row_weights, sizeof(float) * h);
    }
    if (d.qmc_primes) {
        add("qmc_primes", d.qmc_primes, sizeof(uint32_t) * MTSG_QMC_PRIMES);
        add("qmc_perm_offset", d.qmc_perm_offset, sizeof(uint32_t) * MTSG_QMC_PRIMES);
        if (d.qmc_perm)
            add("qmc_perm", d.qmc_perm,
                sizeof(uint16_t) * ((size_t)d.qmc_perm_offset[MTSG_QMC_PRIMES - 1] + d.qmc_primes[MTSG_QMC_PRIMES - 1]));
    }
    if (d.sobol_matrices) add("sobol_matrices", d.sobol_matrices, sizeof(uint32_t) * MTSG_SOBOL_DIMS * MTSG_SOBOL_COLUMNS);
    add("instances", d.instances, sizeof(mtsg_instance) * (size_t)d.n_instances);
    add("groups", d.groups, sizeof(mtsg_group) * (size_t)d.n_groups);
    add("group_nodes", d.group_nodes, sizeof(mtsg_kdnode) * (size_t)d.n_group_nodes);
    add("group_indices", d.group_indices, sizeof(uint32_t) * (size_t)d.n_group_indices);
    add("textures", d.textures, sizeof(mtsg_texture) * (size_t)d.n_textures);
    add("tex_texels", d.tex_texels, sizeof(float) * (size_t)d.n_tex_texels);
    if (d.n_textures) {
        add("tri_uv", d.tri_uv, sizeof(float) * 6 * (size_t)d.n_triangles);
        add("tri_dpdv", d.tri_dpdv, sizeof(float) * 3 * (size_t)d.n_triangles);
    }
    if (d.om) {
        add("om", d.om, sizeof(mtsg_om));
        add("om_bits", d.om_bits, sizeof(uint32_t) * MTSG_OM_COUNT * MTSG_OM_SIZE * MTSG_OM_SIZE * (MTSG_OM_SIZE / 32));
    }
    return out;
}

}  // namespace mtsh
