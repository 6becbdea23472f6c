/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * `path` hot path, used as the parity checker and as the
 * timed CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (libmtsg) never does.
 *
 * Parity pinning: the SFMT-19937 generator is pinned by the reference's
 * known-answer test (src/tests/test_random.cpp:433-507, fixture
 * tests/golden/sfmt_seed4321.json); the kd-tree traversal is pinned against
 * brute-force intersection; BSDF/emitter sampling against their pdfs by
 * chi-square tests modelled on src/tests/test_chisquare.cpp.  The reference
 * itself cannot be compiled here (Boost/Xerces/OpenEXR absent),
 * so whole-image parity against the reference binary is unpinned.
 */
#ifndef MTSG_ORACLE_H
#define MTSG_ORACLE_H

#include "../include/mtsg.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_RNG_COUNTER = 0, ORACLE_RNG_SFMT = 1 };

/* SFMT-19937 (src/libcore/random.cpp) */
typedef struct oracle_sfmt oracle_sfmt;
oracle_sfmt *oracle_sfmt_new(uint64_t seed);
oracle_sfmt *oracle_sfmt_clone(oracle_sfmt *parent);   /* Random(Random*) */
uint64_t oracle_sfmt_next_ulong(oracle_sfmt *r);
float oracle_sfmt_next_float(oracle_sfmt *r);
void oracle_sfmt_free(oracle_sfmt *r);

/* Counter-mode RNG shared with the GPU (DESIGN.md "RNG") */
float oracle_counter_float(uint32_t seed, uint64_t sample_id, uint32_t dim);

/* Ray queries, same semantics as mtsg_trace_closest / mtsg_trace_shadow,
 * traversed with the Havran TA^B_rec restatement (sahkdtree3.h:178-308). */
int oracle_trace_closest(const mtsg_scene_desc *d, uint32_t n, const float *rays,
                         float *t, float *u, float *v, uint32_t *prim, int threads);
int oracle_trace_shadow(const mtsg_scene_desc *d, uint32_t n, const float *rays,
                        uint8_t *occluded, int threads);
/* Brute force over all primitives (validates the kd-tree). */
int oracle_trace_closest_brute(const mtsg_scene_desc *d, uint32_t n, const float *rays,
                               float *t, uint32_t *prim);

typedef struct oracle_stats {
    double seconds;            /* render phase wall time                 */
    uint64_t samples;
    uint64_t rays_closest, rays_shadow;
    uint64_t nodes_visited, leaf_refs, tri_tests;   /* counting builds */
    uint64_t path_vertices;    /* sum of rRec.depth at termination       */
    int threads;
} oracle_stats;

/* Render params->tile_* with MIPathTracer::Li into an ImageBlock
 * (tile + border, 5 floats per pixel, zeroed by the call).
 * rng_mode COUNTER: identical random numbers to the GPU.
 * rng_mode SFMT: Mitsuba's independent sampler (seed 5489, one Random clone
 * per worker, 32x32 blocks in spiral order) -- the CPU baseline.
 * max_samples > 0 stops after that many samples (timing samples). */
int oracle_render(const mtsg_scene_desc *d, const mtsg_render_params *p, int rng_mode,
                  int threads, float *rgbaw_out, oracle_stats *stats);

/* Per-sample radiance of one pixel (counter mode): out = 3*spp floats. */
int oracle_pixel_samples(const mtsg_scene_desc *d, const mtsg_render_params *p,
                         int x, int y, float *out);

/* Print the path of one counter-mode sample to stderr (debugging). */
int oracle_debug_pixel_sample(const mtsg_scene_desc *d, const mtsg_render_params *p, int x, int y, int s);

/* Closest-hit rays traced along one counter-mode sample (8 floats each);
 * returns the count. */
int oracle_debug_path_rays(const mtsg_scene_desc *d, const mtsg_render_params *p, int x, int y, int s,
                           float *rays_out, int max_rays);

/* BSDF / emitter building blocks for statistical tests (local frame). */
/* sample: returns weight (3), pdf, wo(3), sampled type flags */
int oracle_bsdf_sample(const mtsg_bsdf *b, const float wi[3], float s0, float s1,
                       float wo[3], float *pdf, float weight[3]);
int oracle_bsdf_eval(const mtsg_bsdf *b, const float wi[3], const float wo[3],
                     float value[3], float *pdf);

/* batched forms for the chi-square tests: u2 = 2n sample pairs, wo/weight/value 3n */
/* As oracle_bsdf_sample(_n) with a third uniform per sample for the BSDF's
 * own sampler->next1D() draw (roughdielectric's reflect/refract choice). */
int oracle_bsdf_sample3(const mtsg_bsdf *b, const float wi[3], float s0, float s1, float s2, float wo[3], float *pdf,
                        float weight[3]);
int oracle_bsdf_sample3_n(const mtsg_bsdf *b, const float wi[3], uint32_t n, const float *u3, float *wo, float *pdf,
                          float *weight, int32_t *type);
int oracle_bsdf_sample_n(const mtsg_bsdf *b, const float wi[3], uint32_t n, const float *u2, float *wo, float *pdf,
                         float *weight, int32_t *type);
int oracle_bsdf_eval_n(const mtsg_bsdf *b, const float wi[3], uint32_t n, const float *wo, float *value, float *pdf);
/* MicrofacetDistribution (MTSG_MF_*) sampleAll / sampleVisible and pdfAll /
 * pdfVisible (wi == NULL: the "all normals" variant) */
int oracle_mf_sample_n(int type, float au, float av, const float *wi, uint32_t n, const float *u2, float *m, float *pdf);
int oracle_mf_pdf_n(int type, float au, float av, const float *wi, uint32_t n, const float *m, float *pdf);

/* environment emitter (EmitterAdapter of test_chisquare.cpp:342-388) */
int oracle_env_sample_direct_n(const mtsg_scene_desc *d, uint32_t n, const float *u2, const float ref[3], float *dir,
                               float *pdf, float *value);
int oracle_env_pdf_direct_n(const mtsg_scene_desc *d, uint32_t n, const float *dir, float *pdf);
int oracle_env_eval_n(const mtsg_scene_desc *d, uint32_t n, const float *dir, const float *rx, const float *ry, float *out);

/* sampler draws of one sample (kinds: 1 = next1D, 2 = next2D), as mtsg_sampler_draws */
int oracle_sampler_draws(const mtsg_scene_desc *d, const mtsg_render_params *p, int x, int y, uint32_t s,
                         uint32_t n, const int32_t *kinds, float *out);

const char *oracle_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
