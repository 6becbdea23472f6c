/*
 * mtsh.h -- host-side (Mitsuba-mirror) C API: scene loading and film I/O.
 *
 * This library stands in for the CPU parts of Mitsuba that stay on the
 * reference side of the boundary: the XML SceneHandler
 * (src/librender/scenehandler.cpp), shape/BSDF/emitter plugin parameter
 * parsing, Scene::initialize and the SAH kd-tree build
 * (src/librender/scene.cpp:340-408, skdtree.cpp:68-110).  It produces the
 * flat mtsg_scene_desc consumed by libmtsg (include/mtsg.h).  No GPU code.
 */
#ifndef MTSH_H
#define MTSH_H

#include "mtsg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mtsh_scene mtsh_scene;

typedef struct mtsh_scene_info {
    uint32_t n_triangles, n_rects, n_shapes, n_emitters, n_bsdfs;
    uint32_t kd_nodes, kd_indices, kd_max_depth, kd_leaves, kd_nonempty_leaves;
    double kd_build_seconds;
    int32_t film_w, film_h, spp;
    int32_t border;           /* reconstruction filter border (rfilter.cpp:50) */
    int32_t max_depth;        /* integrator maxDepth                           */
} mtsh_scene_info;

/* Load a Mitsuba XML scene; defines are "name=value" strings (-D).
 * Returns NULL on error (see mtsh_last_error). */
mtsh_scene *mtsh_scene_load(const char *path, const char *const *defines, int n_defines);

/* The values a Mitsuba plugin holds in memory after the reference loaded the
 * scene with its own -D parameter map (mitsuba.cpp:168-174,
 * scenehandler.cpp:211): they replace the XML's values before the scene is
 * finalised, so the device renders the film, sample count and integrator
 * parameters the user asked for.  `mask` selects the groups that apply. */
enum {
    MTSH_OVERRIDE_FILM_SIZE    = 1,   /* Film::getSize (crop = the full film unless */
                                      /* FILM_CROP is given too)                    */
    MTSH_OVERRIDE_SAMPLE_COUNT = 2,   /* Sampler::getSampleCount                    */
    MTSH_OVERRIDE_INTEGRATOR   = 4,   /* MonteCarloIntegrator m_maxDepth, m_rrDepth, */
                                      /* m_strictNormals, m_hideEmitters            */
    MTSH_OVERRIDE_FILM_CROP    = 8    /* Film::getCropOffset / getCropSize          */
                                      /* (film.cpp:36-48)                           */
};
typedef struct mtsh_scene_overrides {
    uint32_t mask;
    int32_t film_width, film_height;
    int32_t sample_count;
    int32_t max_depth, rr_depth, strict_normals, hide_emitters;
    int32_t crop_x, crop_y, crop_width, crop_height;   /* MTSH_OVERRIDE_FILM_CROP */
} mtsh_scene_overrides;

/* mtsh_scene_load, then the overrides (may be NULL) before finalisation. */
mtsh_scene *mtsh_scene_load_overrides(const char *path, const char *const *defines, int n_defines,
                                      const mtsh_scene_overrides *overrides);

/* Override kd-tree build parameters before loading (0 = default). */
void mtsh_set_kd_threads(int threads);

/* How `instance` shapes of a `shapegroup` are handed to the device, for the
 * loads that follow:
 *   MTSH_INSTANCING_FLATTEN    each instance's triangles are transformed to
 *                              world space and join the one scene kd-tree
 *                              (the default);
 *   MTSH_INSTANCING_TWO_LEVEL  Mitsuba's own structure (instance.cpp:115-160,
 *                              shapegroup.cpp:94-101): one group-space kd-tree
 *                              per shape group, instances in the top-level
 *                              tree, rays transformed per instance visit. */
enum { MTSH_INSTANCING_FLATTEN = 0, MTSH_INSTANCING_TWO_LEVEL = 1 };
void mtsh_set_instancing(int mode);

const mtsg_scene_desc *mtsh_scene_desc(const mtsh_scene *scene);

/* Integrator properties + sampleCount of the scene; tile = full film. */
void mtsh_scene_render_params(const mtsh_scene *scene, mtsg_render_params *out);

void mtsh_scene_get_info(const mtsh_scene *scene, mtsh_scene_info *out);

void mtsh_scene_free(mtsh_scene *scene);

/* The scene's bitmap textures (headers as in its mtsg_scene_desc): copies
 * up to `capacity` of them to out (may be NULL) and returns their count. */
int mtsh_scene_textures(const mtsh_scene *scene, mtsg_texture *out, int capacity);

/* The myPath2_OM occupancy maps of the scene (om.cpp): the header and the
 * MTSG_OM_COUNT * 256 * 256 * 8 words of bits (either may be NULL).
 * Returns 0, -1 without maps, -2 when capacity is too small. */
int mtsh_scene_om(const mtsh_scene *scene, mtsg_om *om, uint32_t *bits, size_t capacity);

/* The top-level kd-tree's primitive boxes, 6 floats each (min xyz, max xyz;
 * an empty box for primitives it leaves out: degenerate triangles, shape
 * group triangles): the input of mtsg_kd_build.  Returns the primitive
 * count (out may be NULL), -2 when capacity is too small. */
int64_t mtsh_scene_prim_bounds(const mtsh_scene *scene, float *out, size_t capacity);

/* Replace the scene's top-level kd-tree (e.g. by mtsg_kd_build's) in its
 * descriptor; the arrays are copied.  Returns 0 or -1. */
int mtsh_scene_set_kdtree(mtsh_scene *scene, const mtsg_kdnode *nodes, uint32_t n_nodes, const uint32_t *indices,
                          uint32_t n_indices, const float *aabb_min, const float *aabb_max, uint32_t max_depth);

/* hdrfilm develop (fmtconv.cpp:962-974): rgb = (sum w*L) / (sum w). */
void mtsh_develop(const float *rgbaw, int w, int h, float *rgb_out);

/* Write an RGB float image as PFM (bitmap.cpp:347-398). Returns 0 on success. */
int mtsh_write_pfm(const char *path, int w, int h, const float *rgb);

/* roughplastic's rough dielectric transmittance (src/bsdfs/rtrans.h,
 * RoughTransmittance::eval / evalDiffuse at fixed eta and alpha): T at the
 * n warped nodes cos(theta_k) = (k/(n-1))^4, and optionally the diffuse
 * transmittance \int 2 mu T(mu) dmu.  distribution is MTSG_MF_*.
 * Returns 0, or -1 on invalid arguments. */
int mtsh_rough_transmittance(int distribution, float alpha, float eta, int n, float *trans, float *diffuse);

/* Read an OpenEXR (NO/RLE/ZIPS/ZIP/PIZ, HALF or FLOAT) or PFM image as RGB
 * float, rows top-down, as the environment emitter loads it
 * (Bitmap::readOpenEXR, bitmap.cpp:2780).  rgb == NULL: only the size.
 * Returns 0, or -1 (see mtsh_last_error; -2: rgb_capacity too small). */
int mtsh_read_image(const char *path, int *w, int *h, float *rgb, size_t rgb_capacity);

/* Triangle::getClippedAABB (src/libcore/triangle.cpp) as the kd build's
 * perfect splits use it: the bounds of triangle v[0..8] clipped to the box
 * box[0..5] = (min xyz, max xyz) go to out[0..5].  Returns 1 if the clipped
 * box is valid, 0 if the triangle lies outside (the reference's KAT:
 * src/tests/test_kd.cpp:34-84). */
int mtsh_clip_triangle(const float *v, const float *box, float *out);

/* The `bitmap` texture's input (src/textures/bitmap.cpp:246-278): PNG
 * (8/16-bit, palette, sRGB / gAMA), OpenEXR or PFM converted to linear
 * float RGB (fmtconv.cpp:1093-1160), rows top-down; gamma != 0 overrides
 * the file's gamma.  Same return convention as mtsh_read_image. */
int mtsh_texture_image(const char *path, float gamma, int *w, int *h, float *rgb, size_t rgb_capacity);

/* TMIPMap construction (include/mitsuba/render/mipmap.h:155-302) over a
 * linear RGB level 0: fills *mip, the half-rounded texels of every level
 * (*n_texels floats; texels may be NULL to query the size) and the level-0
 * average / maximum (may be NULL). */
int mtsh_build_mipmap(const float *rgb, int w, int h, int filter, int wrap_u, int wrap_v, float max_value,
                      float max_anisotropy, mtsg_mipmap *mip, float *texels, size_t texel_capacity, size_t *n_texels,
                      float *average, float *maximum);

void mtsh_last_error(char *buf, size_t size);

#ifdef __cplusplus
}
#endif
#endif /* MTSH_H */
