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
/* ... and Scene properties (mtsh_scene_set_scene_props) applied after the
 * file's own <scene>-level ones (n_scene_props may be 0). */
mtsh_scene *mtsh_scene_load_props(const char *path, const char *const *defines, int n_defines,
                                  const mtsh_scene_overrides *overrides, const struct mtsh_prop *scene_props,
                                  int32_t n_scene_props);

/* ---- building the scene Mitsuba holds in memory --------------------------
 *
 * The XML route above re-reads a scene file.  A Mitsuba-side plugin already
 * holds the parsed scene, with every `-D` substituted (mitsuba.cpp:168-174,
 * scenehandler.cpp:211): each object's plugin name and the Properties it was
 * created from (ConfigurableObject::getProperties, cobject.h:77;
 * Properties::getPluginName / getPropertyNames / getType, properties.h:49-229)
 * and each TriMesh's arrays (trimesh.h:127-153).  The builder turns exactly
 * that into the device scene: objects are added in Mitsuba's order (the order
 * fixes the descriptor's arrays), then mtsh_scene_finish builds the kd-tree,
 * the emitter CDFs and the environment tables as mtsh_scene_load does --
 * mtsh_scene_load is itself a client of the same constructors.
 *
 * Ids returned by the add calls are >= 0; -1 signals an error (message in
 * mtsh_last_error; the builder stays usable).  String properties naming
 * files resolve against base_dir unless absolute. */
typedef struct mtsh_builder mtsh_builder;

/* One entry of a Properties object (properties.h:49-70 EPropertyType, RGB
 * mode), plus references to objects created earlier in this builder. */
enum {
    MTSH_PROP_BOOLEAN = 0,   /* i                                        */
    MTSH_PROP_INTEGER,       /* i                                        */
    MTSH_PROP_FLOAT,         /* f                                        */
    MTSH_PROP_POINT,         /* v[0..2]                                  */
    MTSH_PROP_VECTOR,        /* v[0..2]                                  */
    MTSH_PROP_TRANSFORM,     /* m (row-major 4x4), inv (its inverse; all */
                             /* zero: computed in double, as Transform(m)) */
    MTSH_PROP_SPECTRUM,      /* v[0..2]: the RGB Spectrum                */
    MTSH_PROP_STRING,        /* s                                        */
    MTSH_PROP_TEXTURE        /* i: a texture id (a BSDF's textured       */
                             /* parameter: a nested <texture> child)     */
};
typedef struct mtsh_prop {
    const char *name;
    int32_t type;            /* MTSH_PROP_*                              */
    int32_t pad;
    int64_t i;
    float f;
    float v[3];
    float m[16], inv[16];
    const char *s;
} mtsh_prop;

/* A triangle mesh.  The builder runs the normal pass of TriMesh::configure
 * (TriMesh::computeNormals, trimesh.cpp:608-681) on the arrays it is given,
 * with flip_normals as that pass's m_flipNormals: NULL normals (and
 * !face_normals) are computed, then given or computed normals are negated
 * when flip_normals is set, and a face_normals mesh with flip_normals gets
 * its winding swapped.  So:
 *   - arrays read from a configured TriMesh (getVertexPositions / Normals /
 *     Triangles after configure(), world space; the Mitsuba plugin's case,
 *     INTEGRATION.md) already carry the flip: pass flip_normals = 0;
 *   - a shape's own loader arrays (object space, before configure) pass the
 *     shape's flipNormals and, optionally, to_world (16 floats row-major; NULL =
 *     identity), applied to positions and to normals by its inverse
 *     transpose, as the shape loaders do before configure. */
typedef struct mtsh_mesh {
    const char *name;
    uint32_t n_vertices, n_triangles;
    const float *positions;      /* 3 * n_vertices                       */
    const float *normals;        /* 3 * n_vertices or NULL               */
    const float *texcoords;      /* 2 * n_vertices or NULL               */
    const uint32_t *indices;     /* 3 * n_triangles                      */
    int32_t face_normals, flip_normals;
    const float *to_world;       /* NULL or 16 floats                    */
    const float *to_world_inv;   /* its inverse as Mitsuba's Transform   */
                                 /* holds it, or NULL: computed          */
} mtsh_mesh;

/* Start a scene (the instancing mode of mtsh_set_instancing applies). */
mtsh_builder *mtsh_scene_begin(const char *base_dir);
/* `bitmap` texture (bitmap.cpp:179-302) -> texture id. */
int32_t mtsh_scene_add_texture(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props);
/* BSDF plugin (diffuse, roughconductor, conductor, dielectric,
 * roughdielectric, plastic, roughplastic, twosided) -> BSDF id.  nested:
 * twosided's one or two BSDF ids (twosided.cpp:52-80), else none. */
int32_t mtsh_scene_add_bsdf(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props,
                            const int32_t *nested, int32_t n_nested);
/* Emitter: `area` (area.cpp:67-78; attach it to one shape) or `envmap`
 * (envmap.cpp:105-185; the scene's environment) -> emitter id. */
int32_t mtsh_scene_add_emitter(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props);
/* Shape group (shapegroup.cpp) -> group id for the shape calls' `group`. */
int32_t mtsh_scene_add_group(mtsh_builder *b, const char *id);
/* Shape from its plugin and Properties (ply, obj, serialized, cube,
 * rectangle): bsdf -1 = the default BSDF (shape.cpp:47-70), emitter -1 =
 * none, group -1 = the scene.  Returns 0 or -1. */
int32_t mtsh_scene_add_shape(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props,
                             int32_t bsdf, int32_t emitter, int32_t group);
/* Triangle mesh from its arrays (see mtsh_mesh).  Returns 0 or -1. */
int32_t mtsh_scene_add_mesh(mtsh_builder *b, const mtsh_mesh *mesh, int32_t bsdf, int32_t emitter, int32_t group);
/* Instance of a shape group (instance.cpp:57-130); props: its `toWorld`. */
int32_t mtsh_scene_add_instance(mtsh_builder *b, int32_t group, const mtsh_prop *props, int32_t n_props);
/* The sensor and what it holds (sensor.cpp:150-262, hdrfilm.cpp:209-220,
 * rfilter.cpp, independent.cpp / halton.cpp / ...), the integrator
 * (integrator.cpp:199-234; myPath2_OM.cpp:61-85).  Return 0 or -1. */
int32_t mtsh_scene_set_sensor(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props);
int32_t mtsh_scene_set_film(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props,
                            const char *rfilter, const mtsh_prop *rfilter_props, int32_t n_rfilter_props);
int32_t mtsh_scene_set_sampler(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props);
int32_t mtsh_scene_set_integrator(mtsh_builder *b, const char *plugin, const mtsh_prop *props, int32_t n_props);
/* The Scene's own Properties (Scene::Scene(props), scene.cpp:47-83; a
 * plugin passes scene->getProperties()): the build parameters of the scene's
 * kd-tree, kdIntersectionCost, kdTraversalCost, kdEmptySpaceBonus
 * (float), kdStopPrims, kdMaxDepth, kdExactPrimitiveThreshold,
 * kdMaxBadRefines (integer), kdClip, kdRetract, kdParallelBuild (boolean).
 * Shape groups keep the defaults (ShapeGroup builds its own ShapeKDTree,
 * shapegroup.cpp:74).  Hits do not depend on these, the tree's shape and
 * speed do.  Returns 0, or -1 for another name or a value of another type. */
int32_t mtsh_scene_set_scene_props(mtsh_builder *b, const mtsh_prop *props, int32_t n_props);
/* Finalise (kd-tree, CDFs, environment tables; overrides may be NULL) and
 * free the builder.  Returns the scene, or NULL (see mtsh_last_error). */
mtsh_scene *mtsh_scene_finish(mtsh_builder *b, const mtsh_scene_overrides *overrides);
/* Drop an unfinished builder. */
void mtsh_scene_abort(mtsh_builder *b);

/* Fingerprint of a scene's device descriptor: one entry per array of
 * mtsg_scene_desc and one ("scalars") for its other fields, FNV-1a 64 of
 * the bytes, so two routes to a scene can be compared byte for byte.
 * Returns the entry count; out (may be NULL) receives up to capacity. */
typedef struct mtsh_digest_entry {
    char name[32];
    uint64_t bytes;
    uint64_t hash;
} mtsh_digest_entry;
int32_t mtsh_scene_digest(const mtsh_scene *scene, mtsh_digest_entry *out, int32_t capacity);

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
