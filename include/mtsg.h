/*
 * mtsg.h -- C-ABI of the MI355X (gfx950) wavefront `path` integrator.
 *
 * This is the drop-in boundary.  The reference exposes the
 * `path` plugin as a C++ `SamplingIntegrator` created through
 * `extern "C" CreateInstance` (reference: include/mitsuba/core/cobject.h:99-107,
 * src/libcore/plugin.cpp:62-121); its work happens in
 *   SamplingIntegrator::render      src/librender/integrator.cpp:99-133
 *   SamplingIntegrator::renderBlock src/librender/integrator.cpp:144-197
 *   MIPathTracer::Li                src/integrators/path/path.cpp:119-294
 * A Mitsuba-side `path` plugin whose render() calls this library replaces all
 * three.  Everything here is plain C: fixed-width scalars,
 * plain pointers and sizes, integer error codes, no exceptions across the ABI.
 *
 * Ownership: the caller owns every host buffer.  mtsg_scene_create copies the
 * scene description to device memory (HBM); the description may be freed
 * after the call returns.
 *
 * Threading: one host thread per GPU.  A scene handle is bound to the device
 * it was created on.  mtsg_cancel() may be called from any thread.
 */
#ifndef MTSG_H
#define MTSG_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTSG_ABI_VERSION 8

/* ---- error codes (mtsg_last_error() gives the message) ------------------ */
enum {
    MTSG_OK             = 0,
    MTSG_ERR_INVALID    = -1,  /* malformed descriptor / parameters        */
    MTSG_ERR_DEVICE     = -2,  /* HIP runtime error                        */
    MTSG_ERR_OOM        = -3,  /* device allocation failed                 */
    MTSG_ERR_CANCELLED  = -4,  /* mtsg_cancel() was called (render() == false) */
    MTSG_ERR_NODEVICE   = -5,  /* no gfx950 device / bad device index      */
    MTSG_ERR_TRAVERSAL  = -6   /* a ray hit the kd-restart limit (a guard  */
                               /* against non-terminating traversal)       */
};

/* ---- scene description: flat arrays, all world space -------------------- */

/* 8-byte kd-tree node, bit-identical to Mitsuba's KDNode
 * (include/mitsuba/render/gkdtree.h:452-600):
 *   inner: combined = axis | (relOffsetToLeftChild << 2), data = float split bits
 *   leaf : combined = 0x80000000 | primStart,              data = primEnd
 * Children are adjacent (right = left + 1).  Indirection nodes are not used. */
typedef struct mtsg_kdnode {
    uint32_t combined;
    uint32_t data;
} mtsg_kdnode;

/* 48-byte Wald projection triangle, field order of Mitsuba's TriAccel
 * (include/mitsuba/render/triaccel.h:37-51).  k == 0xFFFFFFFF marks an
 * analytic shape (rectangle) whose index is in prim_index; k == 3 marks a
 * degenerate triangle that never intersects. */
typedef struct mtsg_triaccel {
    uint32_t k;
    float n_u, n_v, n_d;
    float a_u, a_v, b_nu, b_nv;
    float c_nu, c_nv;
    uint32_t shape_index;
    uint32_t prim_index;   /* global triangle index, or rectangle index */
} mtsg_triaccel;

#define MTSG_TRIACCEL_SHAPE 0xFFFFFFFFu

/* Analytic `rectangle` (src/shapes/rectangle.cpp:78-170). */
typedef struct mtsg_rect {
    float to_object[12];   /* world->object affine, row-major 3x4          */
    float to_world[12];    /* object->world affine, row-major 3x4          */
    float frame_s[3], frame_t[3], frame_n[3];  /* m_frame                  */
    float dpdu[3], dpdv[3];
    float inv_area;
    uint32_t shape_index;
} mtsg_rect;

/* MTSG_SHAPE_INSTANCE: a two-level `instance` of a `shapegroup`
 * (src/shapes/instance.cpp:107-160); its TriAccel record in the top-level
 * tree has k == MTSG_TRIACCEL_SHAPE and prim_index == the instance index. */
enum { MTSG_SHAPE_MESH = 0, MTSG_SHAPE_RECT = 1, MTSG_SHAPE_INSTANCE = 2 };

typedef struct mtsg_shape {
    int32_t type;          /* MTSG_SHAPE_*                                 */
    int32_t bsdf;          /* index into bsdfs                             */
    int32_t emitter;       /* index into emitters, -1 if none              */
    int32_t face_normals;  /* 1: no vertex normals (TriMesh faceNormals)   */
    uint32_t tri_begin;    /* mesh: first global triangle                  */
    uint32_t tri_count;
    uint32_t rect;         /* rectangle index                              */
    uint32_t instance;     /* instance index (MTSG_SHAPE_INSTANCE)         */
} mtsg_shape;

/* Two-level instancing (src/shapes/instance.cpp:115-160,
 * src/shapes/shapegroup.cpp:94-101).  A shape group owns a kd-tree over its
 * own triangles, in group space: its nodes are group_nodes[node_offset ..],
 * KDNode offsets relative to that root, and its leaves reference
 * group_indices[index_offset ..], which index the scene's `triaccel` array
 * (the group triangles' TriAccel records, built from group-space vertices;
 * the top-level tree never references them).  Instance::rayIntersect
 * transforms the ray by to_local (Transform::inverse(); the direction is not
 * renormalized, so t is preserved) and traverses the group tree;
 * fillIntersectionRecord maps p, dpdu and the normals back with to_world
 * (normals by the inverse transpose, i.e. to_local transposed). */
typedef struct mtsg_instance {
    float to_world[12];    /* row-major 3x4 of the instance's toWorld       */
    float to_local[12];    /* row-major 3x4 of its inverse                  */
    uint32_t group;        /* index into groups                             */
    uint32_t shape_index;  /* the instance's entry in shapes                */
    uint32_t pad[2];
} mtsg_instance;

typedef struct mtsg_group {
    uint32_t node_offset, n_nodes;      /* its KDNode[] in group_nodes     */
    uint32_t index_offset, n_indices;   /* its leaf references             */
    float aabb_min[3], aabb_max[3];     /* enlarged tree AABB, group space */
    uint32_t max_depth, pad;
} mtsg_group;

enum {
    MTSG_BSDF_DIFFUSE        = 1,   /* src/bsdfs/diffuse.cpp        */
    MTSG_BSDF_ROUGHCONDUCTOR = 2,   /* src/bsdfs/roughconductor.cpp */
    MTSG_BSDF_DIELECTRIC     = 3,   /* src/bsdfs/dielectric.cpp     */
    MTSG_BSDF_CONDUCTOR      = 4,   /* src/bsdfs/conductor.cpp      */
    MTSG_BSDF_PLASTIC        = 5,   /* src/bsdfs/plastic.cpp        */
    MTSG_BSDF_ROUGHDIELECTRIC = 6,  /* src/bsdfs/roughdielectric.cpp */
    MTSG_BSDF_ROUGHPLASTIC   = 7    /* src/bsdfs/roughplastic.cpp   */
};
enum { MTSG_MF_BECKMANN = 0, MTSG_MF_GGX = 1, MTSG_MF_PHONG = 2 };   /* microfacet.h:49-57 */

/* One BSDF record.  `twosided` (src/bsdfs/twosided.cpp) marks the record
 * of a twosided wrapper's front material: when the incident direction is on
 * the back (cosTheta(wi) <= 0 for eval/pdf, < 0 for sampling) the record
 * bsdfs[back] is used with wi.z and wo.z negated. */
#define MTSG_RTRANS_SAMPLES 100     /* m_thetaSamples of the data/microfacet tables */

typedef struct mtsg_bsdf {
    int32_t type;
    int32_t distribution;    /* MTSG_MF_*                                   */
    int32_t sample_visible;
    int32_t smooth;          /* BSDF::ESmooth set -> NEE (path.cpp:174)     */
    int32_t ref_n_zero;      /* ETransmission|EBackSide -> refN = 0 (records.inl:160-164) */
    int32_t twosided;        /* twosided wrapper front record (see above)   */
    int32_t back;            /* twosided: index of the back-side record     */
    int32_t nonlinear;       /* plastic 'nonlinear'                         */
    float reflectance[3];    /* diffuse; plastic diffuseReflectance         */
    float eta[3], k[3];      /* (rough)conductor, already divided by extEta */
    float spec_refl[3];      /* (rough)conductor / dielectric / plastic     */
    float spec_trans[3];     /* (rough)dielectric                           */
    float alpha_u, alpha_v;  /* already clamped to >= 1e-4                  */
    float ior_eta, ior_inv_eta; /* (rough)dielectric / plastic intIOR/extIOR and inverse */
    float fdr_int;           /* plastic: fresnelDiffuseReflectance(1 / eta) */
    float spec_sampling_weight; /* plastic: sAvg / (dAvg + sAvg) luminances */
    /* roughplastic: the external RoughTransmittance reduced to the material's
     * (eta, alpha) (rtrans.h:169-207, m_alphaFixed && m_etaFixed): samples at
     * warped cos(theta) nodes k/(n-1) = cos^(1/4), evaluated by
     * evalCubicInterp1D (spline.cpp:23-60); fdr_int holds
     * 1 - internal.evalDiffuse(alpha) (roughplastic.cpp:349-351) */
    float rtrans[MTSG_RTRANS_SAMPLES];
    /* 1 + index into textures when `reflectance` is a bitmap texture
     * (evaluated per hit instead of the constant above), 0 otherwise */
    int32_t texture;
    int32_t pad_tex[3];
} mtsg_bsdf;

enum { MTSG_EMITTER_AREA = 1, MTSG_EMITTER_ENVMAP = 2 };

#define MTSG_ENVMAP_MAX_LEVELS 24
#define MTSG_MIPMAP_MAX_LEVELS 24
#define MTSG_MIPMAP_LUT_SIZE 64      /* MTS_MIPMAP_LUT_SIZE (mipmap.h:37) */

/* Boundary conditions (ReconstructionFilter::EBoundaryCondition,
 * include/mitsuba/core/rfilter.h:52-64) and MIP filter types
 * (EMIPFilterType, include/mitsuba/render/mipmap.h:43-55). */
enum { MTSG_WRAP_CLAMP = 0, MTSG_WRAP_REPEAT = 1, MTSG_WRAP_MIRROR = 2, MTSG_WRAP_ZERO = 3, MTSG_WRAP_ONE = 4 };
enum { MTSG_MIP_NEAREST = 0, MTSG_MIP_BILINEAR = 1, MTSG_MIP_TRILINEAR = 2, MTSG_MIP_EWA = 3 };

/* One RGB MIP pyramid, TMIPMap<Color3, Color3h> (mipmap.h:61-860): the
 * texels of level l are 3 floats per texel, row-major, at level_offset[l]
 * of the owner's texel buffer, already rounded to half precision as the
 * reference stores them.  Nearest / bilinear pyramids have one level. */
typedef struct mtsg_mipmap {
    int32_t levels;
    int32_t filter;               /* MTSG_MIP_*                               */
    int32_t wrap_u, wrap_v;       /* MTSG_WRAP_*                              */
    int32_t level_w[MTSG_MIPMAP_MAX_LEVELS], level_h[MTSG_MIPMAP_MAX_LEVELS];
    uint32_t level_offset[MTSG_MIPMAP_MAX_LEVELS];   /* float offset of each level */
    float size_ratio_x[MTSG_MIPMAP_MAX_LEVELS], size_ratio_y[MTSG_MIPMAP_MAX_LEVELS];
    float max_anisotropy;         /* EWA only (1 otherwise, bitmap.cpp:234-235) */
    int32_t pad[3];
    float weight_lut[MTSG_MIPMAP_LUT_SIZE];   /* EWA Gaussian (mipmap.h:296-301) */
} mtsg_mipmap;

/* Environment emitter (src/emitters/envmap.cpp:99-660): lat-long RGB MIP
 * pyramid (EWA; u repeats, v clamps, envmap.cpp:160-161), row/column CDFs
 * for importance sampling, and the scene bounding sphere the shadow rays
 * end on. */
typedef struct mtsg_envmap {
    mtsg_mipmap mip;
    float scale;                  /* 'scale' property                        */
    float to_world[9], to_local[9];  /* rotation part of toWorld and its inverse (row-major) */
    float bsphere_center[3], bsphere_radius;   /* scene bsphere x 1.5 (envmap.cpp:321-325) */
    float normalization;          /* envmap.cpp:300-301                      */
    float pixel_size[2];          /* (2 pi / w, pi / h)                      */
    int32_t emitter;              /* index into emitters                     */
    int32_t pad[3];
} mtsg_envmap;

/* `bitmap` texture (src/textures/bitmap.cpp:167-591) bound to a BSDF's
 * reflectance parameter (diffuse `reflectance`, (rough)plastic
 * `diffuseReflectance`).  Texture2D::eval (src/librender/texture.cpp:112-121)
 * maps uv -> uv * uv_scale + uv_offset; with UV partials (the first hit of a
 * camera ray, records.inl:69-75) the lookup is TMIPMap::eval (filtered),
 * otherwise evalBilinear(0) (evalBox(0) for `nearest`).  `scale` is the
 * ScaleTexture that BSDF::ensureEnergyConservation wraps around a texture
 * whose maximum exceeds 1 (src/librender/bsdf.cpp:88-113), else 1. */
typedef struct mtsg_texture {
    mtsg_mipmap mip;
    float uv_offset[2], uv_scale[2];
    float scale;
    float average[3];             /* getAverage() (level 0, before the scale) */
    float maximum[3];             /* getMaximum()                            */
    int32_t pad[3];
} mtsg_texture;

typedef struct mtsg_emitter {
    int32_t type;
    int32_t shape;           /* emitting shape index                         */
    uint32_t cdf_offset;     /* mesh: area CDF (tri_count+1 floats) in emitter_tri_cdf */
    float pdf_discrete;      /* samplingWeight * normalization (scene.h:849-851) */
    float radiance[3];
    float inv_area;          /* m_invSurfaceArea of the shape                */
} mtsg_emitter;

enum { MTSG_FILTER_BOX = 0, MTSG_FILTER_GAUSSIAN = 1 };

/* Perspective sensor + film, precomputed host side
 * (src/sensors/perspective.cpp:126-176, src/librender/sensor.cpp:241-262). */
typedef struct mtsg_camera {
    float sample_to_camera[16];   /* row-major 4x4                          */
    float camera_to_world[12];    /* row-major 3x4 affine                   */
    float dx[3], dy[3];           /* near-plane differentials (m_dx, m_dy)  */
    float near_clip, far_clip;
    float inv_res_x, inv_res_y;   /* 1 / film size                          */
    int32_t film_w, film_h;       /* full film size                         */
    int32_t crop_x, crop_y, crop_w, crop_h;
    /* reconstruction filter (src/libcore/rfilter.cpp:37-57)               */
    int32_t filter_type;
    float filter_radius;
    float filter_scale;           /* MTS_FILTER_RESOLUTION / radius         */
    int32_t border;               /* ceil(radius - 0.5)                     */
    float filter_values[32];      /* MTS_FILTER_RESOLUTION + 1 entries      */
    int32_t has_alpha;            /* film stores a real alpha channel       */
    int32_t pad[3];
} mtsg_camera;

/* Sampler.  The path's sample dimensions are drawn in the
 * order of Li's next1D / next2D calls (DESIGN.md "Random numbers"):
 *   independent  src/samplers/independent.cpp:51-116, counter-mode draws
 *   halton       src/samplers/halton.cpp:101-404: radical inverse in the
 *                dim-th prime base of index offset(pixel) + stride * s, with
 *                the blocked space partition of setFilmResolution (:240-275)
 *   hammersley   src/samplers/hammersley.cpp:90-300: first dimension s / N,
 *                then radical inverses in the prime bases
 *   ldsampler    src/samplers/ldsampler.cpp:80-245: Kollig-Keller scrambled
 *                (0,2)-sequence, per-pixel random scramble and shuffle per
 *                dimension (1D and 2D requests counted separately), drawn
 *                from the counter RNG instead of a per-thread SFMT stream
 * Halton / Hammersley digit permutations (faure.cpp:23-140): scramble -1 =
 * Faure permutations (the default), 0 = none, otherwise random permutations
 * from sampleTEA seeded with the scramble value. */
enum {
    MTSG_SAMPLER_INDEPENDENT = 0, MTSG_SAMPLER_HALTON = 1, MTSG_SAMPLER_HAMMERSLEY = 2,
    MTSG_SAMPLER_LDSAMPLER = 3, MTSG_SAMPLER_SOBOL = 4
};
/* sobol (src/samplers/sobol.cpp:86-250): Gruenschloss's Sobol' enumeration
 * with Joe & Kuo's direction numbers (sobolseq.cpp / sobolseq.h), single
 * precision: value = min(XOR of the generator columns of the set bits of the
 * index, scrambled) * 2^-32; the film is bucketed (setFilmResolution with
 * bucketed = true), so the index of sample s of pixel (x, y) is
 * look_up(log2 res, s, x, y, scramble) and the first 2D request returns the
 * position inside the pixel. */
#define MTSG_SOBOL_DIMS 1024
#define MTSG_SOBOL_COLUMNS 52
#define MTSG_QMC_PRIMES 1024          /* primeTableSize (qmc.h:38)            */

typedef struct mtsg_sampler {
    int32_t type;                 /* MTSG_SAMPLER_*                          */
    int32_t scramble;             /* halton / hammersley (default -1)        */
    int32_t dimension;            /* ldsampler low-discrepancy dimensions (4) */
    int32_t pad;
} mtsg_sampler;

/* Occupancy maps of the fork's `myPath2_OM` integrator
 * (src/integrators/testOM/myOM.h, myPath2_OM.cpp:137-172): MTSG_OM_COUNT
 * bit-voxel grids of MTSG_OM_SIZE^3 over the cube around the scene's
 * triangle meshes, each the base occupancy resampled along one rotated
 * direction (generateROMA).  A shadow connection o1 -> o2 is answered by
 * the map nearest to its direction: one column's z bits (Visible). */
#define MTSG_OM_SIZE 256               /* OMSIZE                              */
#define MTSG_OM_SQRT 4                 /* OMNUMSQRT                           */
#define MTSG_OM_COUNT 16               /* OMNUM                               */
typedef struct mtsg_om {
    float aabb_min[3];            /* m_AABB.min                             */
    float grid_size_recp;         /* m_gridSizeRecp                         */
    float center[3];              /* m_center                               */
    float pad;
    float dir[MTSG_OM_COUNT][3];  /* m_dir of each rotated map              */
    float rotate[MTSG_OM_COUNT][9];  /* m_rotate (row-major 3x3)            */
} mtsg_om;

typedef struct mtsg_scene_desc {
    uint32_t abi_version;         /* = MTSG_ABI_VERSION                     */
    uint32_t n_vertices;
    const float *vtx_pos;         /* 3 * n_vertices                         */
    const float *vtx_nrm;         /* 3 * n_vertices                         */
    uint32_t n_triangles;
    const uint32_t *tri_idx;      /* 3 * n_triangles (into vtx_*)           */
    const float *tri_dpdu;        /* 3 * n_triangles: UV tangent or p1-p0   */
    uint32_t n_rects;
    const mtsg_rect *rects;
    uint32_t n_shapes;
    const mtsg_shape *shapes;
    uint32_t n_bsdfs;
    const mtsg_bsdf *bsdfs;
    uint32_t n_emitters;
    const mtsg_emitter *emitters;
    const float *emitter_cdf;     /* n_emitters + 1 (pmf.h DiscreteDistribution) */
    uint32_t n_emitter_tri_cdf;
    const float *emitter_tri_cdf; /* concatenated per-emitter triangle CDFs */
    /* kd-tree */
    uint32_t n_nodes;
    const mtsg_kdnode *nodes;
    uint32_t n_indices;
    const uint32_t *indices;
    uint32_t n_prims;             /* == n_triangles + n_rects + n_instances */
    const mtsg_triaccel *triaccel;
    float aabb_min[3], aabb_max[3];  /* enlarged tree AABB (gkdtree.h:1213-1220) */
    uint32_t max_depth;           /* deepest leaf (traversal stack bound)  */
    mtsg_camera camera;
    /* environment emitter (has_envmap = 0: none) */
    int32_t has_envmap;
    uint32_t n_env_texels;        /* floats: 3 per texel over all levels    */
    const float *env_texels;
    const float *env_cdf_rows;    /* level-0 height + 1                      */
    const float *env_cdf_cols;    /* (level-0 width + 1) * height            */
    const float *env_row_weights; /* height                                  */
    mtsg_envmap envmap;
    /* sampler and the quasi-Monte Carlo tables (halton / hammersley) */
    mtsg_sampler sampler;
    const uint32_t *qmc_primes;   /* MTSG_QMC_PRIMES primes                  */
    const uint32_t *qmc_perm_offset; /* MTSG_QMC_PRIMES offsets into qmc_perm */
    const uint16_t *qmc_perm;     /* digit permutation of base primes[i] at
                                     qmc_perm + qmc_perm_offset[i]; NULL when
                                     unscrambled (scramble 0) or unused     */
    /* sobol sampler tables (NULL unless MTSG_SAMPLER_SOBOL) */
    uint64_t sobol_scramble;      /* sampleTEA of 'scramble' (sobol.cpp:92-102), 0: none */
    const uint32_t *sobol_matrices;  /* matrices32: MTSG_SOBOL_DIMS x MTSG_SOBOL_COLUMNS */
    uint32_t sobol_vdc_rows, sobol_vdc_inv_rows;
    const uint64_t *sobol_vdc;    /* vdc_sobol_matrices[rows][MTSG_SOBOL_COLUMNS]     */
    const uint64_t *sobol_vdc_inv;   /* vdc_sobol_matrices_inv[inv rows][COLUMNS]  */
    /* two-level instancing (n_instances = 0: none) */
    uint32_t n_instances;
    const mtsg_instance *instances;
    uint32_t n_groups;
    const mtsg_group *groups;
    uint32_t n_group_nodes;
    const mtsg_kdnode *group_nodes;
    uint32_t n_group_indices;
    const uint32_t *group_indices;
    /* bitmap textures (n_textures = 0: none) and the per-triangle data their
     * lookups need (NULL without textures): tri_uv = the three vertices'
     * texture coordinates, (0,0) (1,0) (0,1) for meshes without UVs so that
     * the interpolation gives Point2(b.y, b.z) bit for bit (skdtree.h:398-405);
     * tri_dpdv = the UV tangent dpdv (trimesh.cpp:701-735) or p2 - p0 */
    uint32_t n_textures;
    const mtsg_texture *textures;
    uint32_t n_tex_texels;        /* floats: 3 per texel over all textures' levels */
    const float *tex_texels;
    const float *tri_uv;          /* 6 * n_triangles                          */
    const float *tri_dpdv;        /* 3 * n_triangles                          */
    /* myPath2_OM occupancy maps (NULL unless the scene's integrator is it):
     * om_bits[((id * SIZE + x) * SIZE + y) * (SIZE / 32) + z / 32] bit z % 32 */
    const mtsg_om *om;
    const uint32_t *om_bits;
} mtsg_scene_desc;

/* ---- render ------------------------------------------------------------- */

/* MonteCarloIntegrator properties (src/librender/integrator.cpp:199-234),
 * sample count, and the film region this call renders.  With the
 * independent sampler the counter-based RNG draws dimension j of sample s of
 * pixel (x, y) as u = hash(seed, (y * film_w + x) * spp + s, j); the other
 * samplers are described at mtsg_sampler.  See DESIGN.md. */
typedef struct mtsg_render_params {
    int32_t max_depth;            /* -1 = infinite                          */
    int32_t rr_depth;             /* default 5                              */
    int32_t strict_normals;
    int32_t hide_emitters;
    uint32_t spp;
    uint32_t seed;
    /* pixel rectangle (film coordinates, inside the crop window) whose
     * samples are generated by this call */
    int32_t tile_x, tile_y, tile_w, tile_h;
    /* multi-GPU film tiling: the rectangle is cut into a grid of 16x16 splat
     * tiles, tiles_x per row; tile (tx, ty) has the deal key
     * ty * tiles_x + (tx - ty) mod tiles_x (each row rotated by its index, so
     * N ranks get diagonal, not column, stripes) and this call renders the
     * tiles with key % tile_stride == tile_offset (tile_stride 0 or 1 = all
     * tiles).  The
     * output block always covers the whole rectangle + border; blocks of
     * different offsets are merged by addition (imageblock.h:103-107). */
    int32_t tile_stride, tile_offset;
    /* integrator: MTSG_INTEGRATOR_PATH = MIPathTracer (path.cpp);
     * MTSG_INTEGRATOR_PATH2_OM = the fork's myPath2_OM (myPath2_OM.cpp:
     * 317-485): max_depth is its maxDepthEye, next-event estimation sees
     * occupancy-map visibility instead of a shadow ray, om_strategy /
     * om_mis its `strategy` (bsdf / nee / mis) and `MISmode` (uniform /
     * balance / power), om_jitter its `jitterSample`; the film is its
     * per-pixel running mean (a 1-pixel box) */
    int32_t integrator;
    int32_t om_strategy;
    int32_t om_mis;
    int32_t om_jitter;
} mtsg_render_params;

enum { MTSG_INTEGRATOR_PATH = 0, MTSG_INTEGRATOR_PATH2_OM = 1 };
enum { MTSG_OM_STRATEGY_BSDF = 0, MTSG_OM_STRATEGY_NEE = 1, MTSG_OM_STRATEGY_MIS = 2 };
enum { MTSG_OM_MIS_UNIFORM = 0, MTSG_OM_MIS_BALANCE = 1, MTSG_OM_MIS_POWER = 2 };

/* Statistics of the last render call on a handle. */
typedef struct mtsg_stats {
    double ms_total;              /* wall time of the render call           */
    /* summed kernel times (HIP events).  A trace launch traces one bounce's
     * closest-hit rays together with the previous bounce's shadow rays:
     * ms_trace_closest sums those launches (launches_trace_closest of them),
     * ms_trace_shadow the final shadow-only launch of each batch.           */
    double ms_trace_closest;
    double ms_trace_shadow;
    double ms_shade;
    double ms_camera;
    double ms_splat;
    uint64_t launches_trace_closest;
    uint64_t rays_closest;        /* closest-hit rays traced                */
    uint64_t rays_shadow;         /* shadow rays traced                     */
    uint64_t samples;
    /* algorithmic traversal work (only when MTSG_FLAG_COUNT is set):
     * closest-hit rays, then shadow rays                                    */
    uint64_t nodes_visited;
    uint64_t leaf_refs;
    uint64_t tri_tests;
    uint64_t shadow_nodes_visited;
    uint64_t shadow_leaf_refs;
    uint64_t shadow_tri_tests;
    /* SIMD efficiency of the persistent traversal kernel (MTSG_FLAG_COUNT):
     * per wave, max-over-lanes inner-node and primitive iterations,
     * traversal steps, and active lanes summed over steps, over waves of
     * both ray kinds (booked in the wave_* fields; shadow_wave_* stay 0).
     * efficiency = (nodes_visited + shadow_nodes_visited) / (64 * wave_node_iters), etc. */
    uint64_t wave_node_iters, wave_test_iters, wave_steps, wave_active_lanes;
    uint64_t shadow_wave_node_iters, shadow_wave_test_iters, shadow_wave_steps, shadow_wave_active_lanes;
    uint64_t launches_trace_shadow;   /* shadow-only trace launches (one per batch) */
    /* traversal iterations per ray (MTSG_FLAG_COUNT): maximum, and a
     * histogram of floor(log2(iterations)), bins 0-15                      */
    uint64_t iter_max_closest, iter_max_shadow;
    uint64_t iter_hist_closest[16], iter_hist_shadow[16];
    /* instance transform visits (MTSG_FLAG_COUNT; two-level scenes)      */
    uint64_t instance_visits, shadow_instance_visits;
    /* tail mode: once a bounce starts with few paths, one k_finish launch
     * carries them through their remaining bounces (ms_finish; the paths it
     * took over; its launches).  Their traversal is not in rays_* above.   */
    double ms_finish;
    uint64_t paths_finish, launches_finish;
    /* exactness paths of the flattened traversal (MTSG_FLAG_COUNT): closest
     * rays traced again with the mailbox after an exact tie (k_tie); rays that
     * took the restart guard's one-ulp step, and those steps; kd-restarts   */
    uint64_t tie_retraces;
    uint64_t guard_rays_closest, guard_rays_shadow, guard_steps_closest, guard_steps_shadow;
    uint64_t restarts_closest, restarts_shadow;
    /* two-level (MTSG_FLAG_COUNT): instance entries whose group-box clip
     * left an empty interval (closest and shadow rays; of instance_visits +
     * shadow_instance_visits)                                              */
    uint64_t instance_rejects;
    /* ... and instance primitives the world-box prefilter skipped before any
     * entry (not counted in instance_visits)                                */
    uint64_t instance_prefiltered;
    /* ms of the ray-order sorts (k_sortwin, MTSG_OPT_RAY_ORDER; MTSG_FLAG_TIMING) */
    double ms_sort;
} mtsg_stats;

enum {
    MTSG_FLAG_TIMING = 1,         /* bracket every kernel with HIP events   */
    MTSG_FLAG_COUNT  = 2,         /* instrumented traversal (slower)        */
    MTSG_FLAG_WAVETIME = 4        /* record each traversal wave's start/exit */
};

typedef struct mtsg_scene mtsg_scene;

/* Number of visible gfx950 devices. */
int  mtsg_device_count(void);

/* PCI address ("dddd:bb:dd.f") of visible device `device`, NUL-terminated in
 * buf[len]: the identity bench.py's ranks compare to prove they drive distinct
 * GPUs (one process per GPU; no reference counterpart -- Mitsuba's workers
 * are host threads). */
int  mtsg_device_pci_id(int device, char *buf, int len);

/* Upload a scene to `device`; *out receives the handle. */
int  mtsg_scene_create(const mtsg_scene_desc *desc, int device, mtsg_scene **out);

/* Render the tile described by params.  `rgbaw_out` is a host buffer of
 * (tile_w + 2*border) * (tile_h + 2*border) * 5 floats holding the
 * ImageBlock (R, G, B, alpha, weight) of the tile including its filter
 * border (src/librender/renderproc.cpp:41-50, imageblock.h:124-204).  The
 * buffer is overwritten.  Blocking. */
int  mtsg_render(mtsg_scene *scene, const mtsg_render_params *params,
                 float *rgbaw_out);

/* Same, but accumulates into a device-resident buffer of the same layout
 * (must be zeroed by the caller before the first call) and does not copy
 * to the host.  Used by the benchmark (inputs and outputs stay in HBM). */
int  mtsg_render_device(mtsg_scene *scene, const mtsg_render_params *params,
                        float *rgbaw_device);

/* Per-tile ImageBlocks (the multi-GPU gather): instead of one block of the
 * whole rectangle, the call's tiles each get their own window of
 * window x window x 5 floats (window = 16 + 2*border: the tile plus its
 * filter border), window v holding the tile of deal key
 * tile_offset + v * tile_stride (see tile_stride above).  These are the
 * per-block ImageBlocks of BlockedRenderProcess (renderproc.cpp:41-50) that
 * ImageBlock::put(const ImageBlock *) adds into the film
 * (imageblock.h:103-107); texels outside the rectangle's block stay zero.
 * A rank copies ntiles * window^2 * 5 floats to the host instead of the
 * whole block (1/N of the tiles: 3.6 MB instead of 18.7 MB per 1/8 C3
 * share).  mtsg_tile_windows gives ntiles and window for params;
 * mtsg_render_device_tiles accumulates into a zeroed device buffer of that
 * size. */
int  mtsg_tile_windows(mtsg_scene *scene, const mtsg_render_params *params,
                       uint32_t *ntiles, int32_t *window);
int  mtsg_render_device_tiles(mtsg_scene *scene, const mtsg_render_params *params,
                              float *windows_device);

/* Explicit tile share (dynamic balancing): after this call the render calls
 * of the handle take exactly the tiles with deal keys keys[0..n) (the keys of
 * tile_stride above, distinct, each inside the params' rectangle, else the
 * render fails with MTSG_ERR_INVALID), in that order -- mtsg_render_device_tiles
 * window v holds the tile keys[v] -- instead of tile_stride / tile_offset.
 * n = 0 returns to the stride deal.  The per-sample random numbers are keyed
 * by pixel and sample, so any split of the keys over ranks sums to the
 * whole-frame image bit for bit.  The share a rank takes can then follow
 * its measured speed, as the reference's scheduler hands the next block to
 * whichever worker is free (src/libcore/sched.cpp:427-496); bench.py
 * re-cuts the shares from the warm-up steps' times. */
int  mtsg_set_tile_list(mtsg_scene *scene, const int32_t *keys, uint32_t n);

/* Device buffer helpers for mtsg_render_device (plain hipMalloc/hipMemcpy). */
int  mtsg_device_alloc(mtsg_scene *scene, size_t bytes, void **out);
int  mtsg_device_free(mtsg_scene *scene, void *ptr);
int  mtsg_device_memset(mtsg_scene *scene, void *ptr, size_t bytes);
int  mtsg_device_to_host(mtsg_scene *scene, void *dst, const void *src, size_t bytes);

/* Cancel the render running on this handle (async-safe flag, checked
 * between bounces; SamplingIntegrator::cancel, integrator.cpp:94-97): it
 * returns MTSG_ERR_CANCELLED once the lanes have drained.  The flag is
 * consumed when a render returns; set while no render runs, it cancels the
 * next one. */
void mtsg_cancel(mtsg_scene *scene);

/* Withdraw a pending cancel flag (one that was set after the render it was
 * meant for had returned).  For callers that serialise their cancel() with
 * the end of their renders, as libmtsg_path's job does. */
void mtsg_cancel_clear(mtsg_scene *scene);

/* Tile completion: after `fn` is set, mtsg_render / mtsg_render_device /
 * mtsg_render_device_tiles call fn(user, key, x, y, w, h) on the rendering
 * thread once per 16x16 tile of the call, when the last of its samples has
 * been splatted into the ImageBlock (its deal key and its rectangle in film
 * pixels, inside the params' rectangle).  The plugin's hook for
 * RenderQueue::signalWorkEnd and the progress reporter
 * (BlockedRenderProcess::processResult, renderproc.cpp:144-154,179): a
 * batch's tiles complete together (the whole frame is one batch unless
 * mtsg_set_batch_paths makes them smaller).  When fn runs the tile's samples
 * are in the device-side ImageBlock; mtsg_render copies the block into its
 * host buffer (and the path job sums the GPUs' blocks) only after the last
 * batch, so a listener uses the call for progress, not to read pixels.
 * fn = NULL removes it. */
typedef void (*mtsg_tile_fn)(void *user, int32_t key, int32_t x, int32_t y, int32_t w, int32_t h);
int  mtsg_set_tile_callback(mtsg_scene *scene, mtsg_tile_fn fn, void *user);

int  mtsg_set_flags(mtsg_scene *scene, uint32_t flags);
int  mtsg_get_stats(mtsg_scene *scene, mtsg_stats *out);
/* Debug: rays of the last MTSG_FLAG_COUNT render that needed >= 300
 * traversal iterations (up to 64 captured): 12 floats each, o.xyz, d.xyz,
 * iterations, shadow (0/1), inner nodes, primitive tests, kd-restarts, 0.
 * Returns the number captured.  No reference
 * counterpart (instrumentation in the spirit of
 * rayIntersectHavranCollectStatistics, sahkdtree3.h:310-432).             */
/* Debug: with MTSG_FLAG_WAVETIME, per wave of the last render's traversal
 * launches: start and exit time, the time it found the work list empty
 * (100-MHz wall-clock ticks; 0: never) and its loop iterations after that:
 * out[launch][wave][4], up to max_launches launches of *waves waves each.
 * Returns the number of launches recorded.                                 */
int  mtsg_debug_wavetimes(mtsg_scene *scene, uint64_t *out, uint32_t max_launches, uint32_t *waves);
int  mtsg_debug_stragglers(mtsg_scene *scene, float *out, uint32_t max_rays);

/* Wavefront batch size in paths.  Default: the whole rectangle, up to
 * 3 * 2^28 paths (280 B of path state each) and at most 3/4 of the free
 * device memory; larger renders run in equal batches. */
int  mtsg_set_batch_paths(mtsg_scene *scene, uint32_t paths);

/* Tail mode: once a bounce starts with fewer than `paths` paths, one
 * persistent launch carries them through all their remaining bounces
 * instead of a trace + shade launch per bounce (same arithmetic in the same
 * order: the image is unchanged).  0 turns it off; the default is
 * MTSG_DEFAULT_FINISH_PATHS.                                              */
#define MTSG_DEFAULT_FINISH_PATHS 524288u
int  mtsg_set_finish_paths(mtsg_scene *scene, uint32_t paths);

/* Execution options of a handle, set explicitly by the caller (no library
 * reads the environment).  They change how a render is scheduled, never its
 * pixels (every option's renders are bit-identical):
 *   MTSG_OPT_TRACE_REFILL     idle lanes that make a traversal wave refill
 *                             from the work list: 16 (default) or 32
 *   MTSG_OPT_FINISH_SHADE_MIN tail kernel: a wave shades once that many of its
 *                             busy lanes wait for shading (1..64, default 16)
 *   MTSG_OPT_LANES            concurrent batches on their own streams (1..4,
 *                             default 1; measured slower)
 *   MTSG_OPT_STAGGER          bounces between the lanes' starts (0..16)
 *   MTSG_OPT_SHADE_GENERIC    1: shade with the kernel that holds every material
 *                             class instead of the scene's own set (A/B tests)
 *   MTSG_OPT_RAY_ORDER        the order the traversal takes a bounce's rays in:
 *                             0 (default) = the order they were appended in,
 *                             1 = windows of 4096 rays sorted by direction
 *                             (measured slower)
 *   MTSG_OPT_CAMERA_DIFFS     environment scenes: 0 (default) = a camera ray
 *                             that misses recomputes its ray differentials at
 *                             bounce 0, 1 = the camera stores them in the path
 *                             state (the layout through round 5; A/B tests).
 *                             Scenes with filtered textures always store them.
 * Unknown keys and values out of range return MTSG_ERR_INVALID. */
enum {
    MTSG_OPT_TRACE_REFILL = 1,
    MTSG_OPT_FINISH_SHADE_MIN = 2,
    MTSG_OPT_LANES = 3,
    MTSG_OPT_STAGGER = 4,
    MTSG_OPT_SHADE_GENERIC = 5,
    MTSG_OPT_RAY_ORDER = 6,
    MTSG_OPT_CAMERA_DIFFS = 7
};
int  mtsg_set_option(mtsg_scene *scene, int32_t key, int64_t value);

/* TEST ONLY: the traversal's limits, to exercise the kd-restart guard
 * (tests/test_gpu_edge_rays.py; kernels.h kd_restart).  stack_cap > 0
 * shrinks every short stack to that many entries; restart_guard >= 0 is the
 * restart number from which a restart starts one ulp beyond its distance
 * (default 8; a large value turns the guard off, which can change results);
 * restart_limit >= 0 is the restart number that ends a ray with
 * MTSG_ERR_TRAVERSAL (default 511), applied to shadow rays only when
 * limit_shadow_only; no_instance_prefilter turns the two-level world-box
 * prefilter off.  Any change selects separate kernel instantiations;
 * NULL restores the defaults.  Production renders never call this: no
 * environment variable or other setting changes these limits. */
typedef struct mtsg_test_knobs {
    int32_t stack_cap, restart_guard, restart_limit, limit_shadow_only;
    int32_t no_instance_prefilter;   /* 1: the two-level traversal enters every instance primitive it meets */
                                     /* (no world-box prefilter; kernels.h inst_box), to check that the     */
                                     /* prefilter drops only entries the exact clip rejects                 */
} mtsg_test_knobs;
int  mtsg_set_test_knobs(mtsg_scene *scene, const mtsg_test_knobs *knobs);

/* Debug/parity entry points over SoA rays (host buffers).  Semantics of
 * ShapeKDTree::rayIntersect (src/librender/skdtree.cpp:112-142) including
 * the adaptive epsilon when mint == 1e-4 (Epsilon).  Misses give
 * prim = 0xFFFFFFFF.  rays: 8 floats per ray {ox,oy,oz,dx,dy,dz,mint,maxt}. */
/* Debug: environment radiance (x scale) along n world directions (3n
 * floats); rx/ry = NULL -> bilinear level-0 lookup (BSDF-sampled rays), else
 * EWA lookup with those differential directions (camera rays).
 * EnvironmentMap::evalEnvironment, src/emitters/envmap.cpp:380-410. */
int  mtsg_env_eval(mtsg_scene *scene, uint32_t n, const float *dirs, const float *rx, const float *ry, float *out);

/* Debug / parity entry: BitmapTexture::eval (src/textures/bitmap.cpp:431-499)
 * of texture `tex` at n uv points (2 floats each): the filtered TMIPMap::eval
 * with the uv partials duv = (d0.x, d0.y, d1.x, d1.y) per point, or the
 * unfiltered evalBilinear(0) / evalBox(0) when duv is NULL.  RGB out. */
int  mtsg_tex_eval(mtsg_scene *scene, int tex, uint32_t n, const float *uv, const float *duv, float *out);

/* Debug / parity entry: myPath2_OM's visibility query for n connections:
 * ids[i] = OccupancyMap::nearestOMindex(dirs[i]) (myOM.h:603-615) and
 * vis[i] = roma[ids[i]].Visible(o1[i], o2[i]) (myOM.h:383-503), 0 or 1. */
int  mtsg_om_query(mtsg_scene *scene, uint32_t n, const float *dirs, const float *o1, const float *o2, int32_t *ids,
                   int32_t *vis);

/* ---- device-side SAH kd-tree build ----------------------
 * GenericKDTree::build (include/mitsuba/render/gkdtree.h:958-1240) on the
 * GPU: breadth-first min-max binned SAH (32 bins per axis) with Mitsuba's
 * costs, straddling triangles clipped to the children (perfect splits).
 * Input: the scene's n_prims primitives as 6 floats each (min xyz, max xyz;
 * an empty box leaves the primitive out), in the order of scene->triaccel,
 * and its triangles (vtx_pos / tri_idx) for the clipping.
 * Output: host arrays in the mtsg_kdnode / index encoding of the scene
 * descriptor, the enlarged tree AABB, the deepest leaf and the build time
 * (ms, uploads and downloads included).  Free with mtsg_kd_free. */
typedef struct mtsg_kd_build_params {
    float traversal_cost;         /* 15 (gkdtree.h:734-744)                  */
    float query_cost;             /* 20                                      */
    float empty_space_bonus;      /* 0.9                                     */
    int32_t stop_prims;           /* 6 in Mitsuba; 4 measured best here and  */
                                  /* the default when params is NULL         */
    int32_t max_depth;            /* 0: 8 + 1.3 log2i(N)                     */
    int32_t pad;
} mtsg_kd_build_params;

typedef struct mtsg_kd_tree {
    mtsg_kdnode *nodes;
    uint32_t n_nodes;
    uint32_t *indices;
    uint32_t n_indices;
    float aabb_min[3], aabb_max[3];
    uint32_t max_depth, leaves;
    double ms_build;
} mtsg_kd_tree;

int  mtsg_kd_build(int device, const mtsg_scene_desc *scene, const float *prim_bounds, const mtsg_kd_build_params *params,
                   mtsg_kd_tree *out);
/* Refit (the reference rebuilds, gkdtree.h:958-1240): `tree`'s
 * node structure and split planes kept, its leaves refilled on the GPU from
 * the scene's current primitives (prim_bounds / vtx_pos / tri_idx of the same
 * primitive numbering), straddling triangles clipped to the child boxes as the
 * build clips them.  For geometry that moved or deformed between frames: every
 * primitive is referenced by every leaf its clipped box overlaps, so
 * traversal stays exact; the old planes' SAH quality is what degrades.  Leaf
 * ranges are re-laid out breadth first; the AABB is recomputed.  Free with
 * mtsg_kd_free. */
int  mtsg_kd_refit(int device, const mtsg_scene_desc *scene, const float *prim_bounds, const mtsg_kd_tree *tree,
                   mtsg_kd_tree *out);
void mtsg_kd_free(mtsg_kd_tree *tree);

/* Debug: the scene sampler's draws for sample s of film pixel (x, y): kinds[i]
 * = 1 (next1D, one float out) or 2 (next2D, two floats), in call order, as
 * Sampler::next1D / next2D after Sampler::generate(pos) + setSampleIndex(s)
 * (src/librender/sampler.cpp; samplers per mtsg_sampler).  params gives spp
 * and seed.  The first next2D is the camera's pixel jitter. */
int  mtsg_sampler_draws(mtsg_scene *scene, const mtsg_render_params *params, int x, int y, uint32_t s,
                        uint32_t n, const int32_t *kinds, float *out);

int  mtsg_trace_closest(mtsg_scene *scene, uint32_t n, const float *rays,
                        float *t, float *u, float *v, uint32_t *prim);
/* Shadow variant (skdtree.cpp:207-226): occluded[i] = 1 if any hit. */
int  mtsg_trace_shadow(mtsg_scene *scene, uint32_t n, const float *rays,
                       uint8_t *occluded);

/* Debug/parity entry point: render params' tile (must fit one wavefront
 * batch) and return the per-sample path radiance instead of the film:
 * L_out[((y - tile_y) * tile_w + (x - tile_x)) * spp + s] = {R, G, B, alpha}. */
int  mtsg_render_samples(mtsg_scene *scene, const mtsg_render_params *params,
                         float *L_out);

void mtsg_scene_destroy(mtsg_scene *scene);

/* Copies the last error message of the calling thread. */
void mtsg_last_error(char *buf, size_t size);

#ifdef __cplusplus
}
#endif
#endif /* MTSG_H */
