/*
 * mtsg_path.h -- the `path` integrator's render() on N GPUs (libmtsg_path.so).
 *
 * Replaces SamplingIntegrator::render (reference src/librender/integrator.cpp:99-133)
 * together with BlockedRenderProcess (src/librender/renderproc.cpp:26-186):
 * instead of 32x32 blocks handed to CPU workers, the film's 16x16 tiles are
 * dealt round-robin to one host thread per GPU (tile t -> GPU t % N), each
 * GPU renders its tiles into an ImageBlock of the full film plus filter
 * border, and the blocks are merged by addition as ImageBlock::put(const
 * ImageBlock *) does (include/mitsuba/render/imageblock.h:103-107).  No
 * collectives; the RNG is keyed by (pixel, sample), so the image does not
 * depend on N.
 */
#ifndef MTSG_PATH_H
#define MTSG_PATH_H

#include "mtsh.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Render params->tile_* of `scene` with n_gpus devices (<= 0: all visible)
 * into rgbaw_out ((tile_h + 2b) x (tile_w + 2b) x 5 floats, b = border).
 * seconds_out (optional) receives the render time, upload excluded
 * (renderjob.cpp:102).  Returns an mtsg error code. */
int mtsh_path_render(const mtsh_scene *scene, const mtsg_render_params *params, int n_gpus,
                     float *rgbaw_out, double *seconds_out);

#ifdef __cplusplus
}
#endif
#endif
