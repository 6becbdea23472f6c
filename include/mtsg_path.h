/*
 * mtsg_path.h -- the `path` integrator's preprocess() / render() / cancel()
 * on N GPUs (libmtsg_path.so).
 *
 * Replaces SamplingIntegrator::render (reference src/librender/integrator.cpp:99-133)
 * together with BlockedRenderProcess (src/librender/renderproc.cpp:26-186):
 * instead of 32x32 blocks handed to CPU workers, the film's 16x16 tiles are
 * shared over one host thread per GPU -- each GPU takes a run of the tiles'
 * deal keys in golden-ratio order (mtsg_set_tile_list), re-cut from the GPUs'
 * measured rates between renders (mtsh_path_job_render) -- each
 * GPU renders its tiles into an ImageBlock of the full rectangle plus filter
 * border, and the blocks are merged by addition as ImageBlock::put(const
 * ImageBlock *) does (include/mitsuba/render/imageblock.h:103-107).  No
 * collectives; the RNG is keyed by (pixel, sample), so the image does not
 * depend on N.
 *
 * A job mirrors the integrator object's life cycle:
 *   mtsh_path_job_create   Integrator::preprocess (integrator.h:61-63):
 *                          the scene is uploaded to every GPU once
 *   mtsh_path_job_render   SamplingIntegrator::render (integrator.cpp:99-133)
 *   mtsh_path_job_cancel   SamplingIntegrator::cancel (integrator.cpp:94-97):
 *                          async-safe, from any thread; the running render
 *                          returns MTSG_ERR_CANCELLED (render() == false)
 */
#ifndef MTSG_PATH_H
#define MTSG_PATH_H

#include "mtsh.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mtsh_path_job mtsh_path_job;

/* Upload `scene` to n_gpus devices (<= 0: all visible gfx950 devices).
 * The host scene may be freed once this call returns. */
int mtsh_path_job_create(const mtsh_scene *scene, int n_gpus, mtsh_path_job **out);

/* Number of GPUs of the job. */
int mtsh_path_job_gpus(const mtsh_path_job *job);

/* Render params->tile_* into rgbaw_out ((tile_h + 2b) x (tile_w + 2b) x 5
 * floats, b = border).  The rectangle's 16x16 tiles selected by
 * params->tile_stride / tile_offset (all tiles when stride <= 1) are shared
 * over the job's N GPUs (mtsg_set_tile_list): GPU g renders a run of those
 * deal keys in golden-ratio order (key k at frac(k * 0.618...)), so every
 * share is spread over the whole rectangle.  The first render of a tile set
 * gives the GPUs equal runs; a render of the same set again (same rectangle,
 * deal, spp, depth and integrator) re-cuts them from the GPUs' measured
 * rates (tiles / second of the last render, damped by half), so a slower
 * share shrinks -- the job's stand-in for the reference scheduler handing
 * the next block to a free worker (src/libcore/sched.cpp:427-496).  The
 * image does not depend on the cut.
 * seconds_out (optional) receives the render time.  Blocking; returns an mtsg
 * error code (MTSG_ERR_CANCELLED after mtsh_path_job_cancel). */
int mtsh_path_job_render(mtsh_path_job *job, const mtsg_render_params *params, float *rgbaw_out,
                         double *seconds_out);

/* Share balancing on (default) or off (equal runs every render); either
 * call forgets the last render's rates. */
int mtsh_path_job_set_balance(mtsh_path_job *job, int on);

/* The last render's tiles and seconds per GPU (arrays of mtsh_path_job_gpus
 * entries; either may be NULL). */
int mtsh_path_job_shares(const mtsh_path_job *job, int32_t *tiles, double *seconds);

/* Tile completion of the job's renders: fn(user, gpu, x, y, w, h) once per
 * 16x16 tile when its ImageBlock contribution is complete on GPU `gpu` (see
 * mtsg_set_tile_callback); calls from the job's GPU threads are serialised,
 * so fn need not be thread-safe.  The plugin's RenderQueue::signalWorkEnd /
 * progress hook (renderproc.cpp:144-154,179).  fn = NULL removes it. */
typedef void (*mtsh_path_tile_fn)(void *user, int32_t gpu, int32_t x, int32_t y, int32_t w, int32_t h);
int mtsh_path_job_set_tile_callback(mtsh_path_job *job, mtsh_path_tile_fn fn, void *user);

/* Cancel the job's running render (async-safe; no effect when idle). */
void mtsh_path_job_cancel(mtsh_path_job *job);

void mtsh_path_job_destroy(mtsh_path_job *job);

/* One-shot: create a job, render, destroy.  seconds_out excludes the upload
 * (renderjob.cpp:102). */
int mtsh_path_render(const mtsh_scene *scene, const mtsg_render_params *params, int n_gpus,
                     float *rgbaw_out, double *seconds_out);

/* Last error of this library on the calling thread: names the GPU whose
 * render failed and carries the device error of that worker thread. */
void mtsh_path_last_error(char *buf, size_t size);

#ifdef __cplusplus
}
#endif
#endif
