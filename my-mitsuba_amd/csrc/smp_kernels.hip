// smp_kernels.hip -- the shading kernels (k_shade, k_finish) of one sampler.
// Compiled once per sampler with -DMTSG_TU_SAMPLER=<MTSG_SAMPLER_* value>, so the
// ENV x EXT (x MATS for k_shade) variants of both kernels of each sampler
// build in their own translation unit, in parallel (see kernels.h and the
// Makefile).
#include "kernels.h"

#ifndef MTSG_TU_SAMPLER
#error "MTSG_TU_SAMPLER must name the sampler this unit instantiates"
#endif

namespace mtsg {

// the material-specialised kernels (MATS), one for bounce 0 and one for the
// later bounces (FIRST); the generic kernel decides at run time
template <int SMP, int MATS>
void launch_shade_mats(const ShadeLaunch &a) {
    if constexpr (MATS == MATS_ALL) {
        if (a.env) hipLaunchKernelGGL((k_shade<true, SMP, false>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
        else hipLaunchKernelGGL((k_shade<false, SMP, false>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
    } else if (a.bounce == 0) {
        if (a.env) hipLaunchKernelGGL((k_shade<true, SMP, false, MATS, 1>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
        else hipLaunchKernelGGL((k_shade<false, SMP, false, MATS, 1>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
    } else {
        if (a.env) hipLaunchKernelGGL((k_shade<true, SMP, false, MATS, 0>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
        else hipLaunchKernelGGL((k_shade<false, SMP, false, MATS, 0>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
    }
}

template <>
void launch_shade_smp<MTSG_TU_SAMPLER>(const ShadeLaunch &a) {
    constexpr int SMP = MTSG_TU_SAMPLER;
#if MTSG_TU_SAMPLER == MTSG_SAMPLER_INDEPENDENT
    if (a.I->om) {   // myPath2_OM (independent sampler only)
        if (a.ext) hipLaunchKernelGGL((k_shade_om<true>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity);
        else hipLaunchKernelGGL((k_shade_om<false>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity);
        return;
    }
#endif
    if (a.ext) {
        if (a.env) hipLaunchKernelGGL((k_shade<true, SMP, true>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
        else hipLaunchKernelGGL((k_shade<false, SMP, true>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.bounce, a.qin, a.nIdentity, a.hasAlpha);
        return;
    }
    // the smallest compiled material set that holds the scene's (mats_kernel_set);
    // compiled for the independent sampler (the other samplers' units keep
    // their build time and shade with the generic kernel)
    if constexpr (SMP == MTSG_SAMPLER_INDEPENDENT) {
        switch (mats_kernel_set(a.mats)) {
            case MAT_DIFFUSE: launch_shade_mats<SMP, MAT_DIFFUSE>(a); return;
            case MAT_DIFFUSE | MAT_RC_GGX: launch_shade_mats<SMP, MAT_DIFFUSE | MAT_RC_GGX>(a); return;
            case MAT_DIFFUSE | MAT_RC_GGX | MAT_DIELECTRIC: launch_shade_mats<SMP, MAT_DIFFUSE | MAT_RC_GGX | MAT_DIELECTRIC>(a); return;
            default: break;
        }
    }
    launch_shade_mats<SMP, MATS_ALL>(a);
}

// SMP is a template parameter (not this unit's constant): every unit defines
// this template, and instantiations that differed only in their body would be
// merged by the linker
template <int SMP, bool INST, int MATS>
void launch_finish_mats(const ShadeLaunch &a) {
    if (a.env) hipLaunchKernelGGL((k_finish<true, SMP, false, INST, MATS>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.qin, a.hasAlpha, a.shadeMin);
    else hipLaunchKernelGGL((k_finish<false, SMP, false, INST, MATS>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.qin, a.hasAlpha, a.shadeMin);
}
template <int SMP, bool INST>
void launch_finish_inst(const ShadeLaunch &a) {
    if (a.ext) {
        if (a.env) hipLaunchKernelGGL((k_finish<true, SMP, true, INST>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.qin, a.hasAlpha, a.shadeMin);
        else hipLaunchKernelGGL((k_finish<false, SMP, true, INST>), a.grid, a.block, 0, a.stream, *a.S, *a.I, *a.B, *a.P, a.qin, a.hasAlpha, a.shadeMin);
        return;
    }
    // the scene's material set, as k_shade (independent sampler only)
    // (finish_uses_mats: the grid mtsg.hip sizes for it)
    if constexpr (SMP == MTSG_SAMPLER_INDEPENDENT && !INST && MTSG_FINISH_MATS) {
        switch (mats_kernel_set(a.mats)) {
            case MAT_DIFFUSE: launch_finish_mats<SMP, INST, MAT_DIFFUSE>(a); return;
            case MAT_DIFFUSE | MAT_RC_GGX: launch_finish_mats<SMP, INST, MAT_DIFFUSE | MAT_RC_GGX>(a); return;
            case MAT_DIFFUSE | MAT_RC_GGX | MAT_DIELECTRIC: launch_finish_mats<SMP, INST, MAT_DIFFUSE | MAT_RC_GGX | MAT_DIELECTRIC>(a); return;
            default: break;
        }
    }
    launch_finish_mats<SMP, INST, MATS_ALL>(a);
}

template <>
void launch_finish_smp<MTSG_TU_SAMPLER>(const ShadeLaunch &a) {
    if (a.inst) launch_finish_inst<MTSG_TU_SAMPLER, true>(a);
    else launch_finish_inst<MTSG_TU_SAMPLER, false>(a);
}

#ifdef MTSG_TU_OCCUPANCY
// persistent grid of k_finish (the register-heaviest variant bounds them all)
// mats: of the material-specialised flat kernels (4 waves/SIMD, not 3)
int finish_blocks_per_cu(bool mats) {
    int perCU = 0;
    int perCU2 = 0;
    if (mats)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(
                   &perCU, (const void *)k_finish<true, MTSG_SAMPLER_INDEPENDENT, false, false, MAT_DIFFUSE | MAT_RC_GGX | MAT_DIELECTRIC>,
                   TRACE_BLOCK, 0) == hipSuccess ? perCU : 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, (const void *)k_finish<true, MTSG_SAMPLER_INDEPENDENT, true, false>, TRACE_BLOCK,
                                                     0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU2, (const void *)k_finish<true, MTSG_SAMPLER_INDEPENDENT, true, true>, TRACE_BLOCK,
                                                     0) != hipSuccess)
        return 0;
    return std::min(perCU, perCU2);
}
#endif

}  // namespace mtsg
