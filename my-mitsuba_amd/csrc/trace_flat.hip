// trace_flat.hip -- the flat (single-level) traversal launches: k_trace_s of
// flattened scenes and its exact-tie retrace k_tie.  They live in their own
// translation unit so that they alone are compiled with the memory-clause
// scheduler (Makefile DEV_FLAT_FLAGS: -amdgpu-sched-strategy=max-memory-clause,
// which groups each iteration's node-pair and TriAccel loads into one clause:
// C3 trace -1.0%, C5 -0.6%; the two-level kernel, left in mtsg.hip, loses 3%
// under it -- DESIGN.md §3, profiles/r06_sched_strategy.txt).  Scheduling
// only: the same IEEE operations, the same hits.
// (kernels.h defines every kernel; this unit launches only the flat traversal)
#pragma clang diagnostic ignored "-Wunused-function"
#include "kernels.h"

namespace mtsg {

template <bool COUNT>
static void launch_flat(const FlatTraceLaunch &a) {
    const dim3 blk(TRACE_BLOCK);
    if (a.knobs && !COUNT) hipLaunchKernelGGL((k_trace_s<false, 16, false, true>), a.grid, blk, 0, a.stream, *a.S, *a.P, a.cIn, a.sIn, a.n, a.wt);
    else if (a.refill32) hipLaunchKernelGGL((k_trace_s<COUNT, 32>), a.grid, blk, 0, a.stream, *a.S, *a.P, a.cIn, a.sIn, a.n, a.wt);
    else hipLaunchKernelGGL((k_trace_s<COUNT, 16>), a.grid, blk, 0, a.stream, *a.S, *a.P, a.cIn, a.sIn, a.n, a.wt);
    if (a.tie) {
        if (a.knobs) hipLaunchKernelGGL((k_tie<true>), a.tieGrid, blk, 0, a.stream, *a.S, *a.P);
        else hipLaunchKernelGGL((k_tie<false>), a.tieGrid, blk, 0, a.stream, *a.S, *a.P);
    }
}

void launch_trace_flat(const FlatTraceLaunch &a) {
    if (a.count) launch_flat<true>(a);
    else launch_flat<false>(a);
}

int trace_flat_blocks_per_cu() {
    int perCU = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, (const void *)k_trace_s<false, 16>, TRACE_BLOCK, 0) != hipSuccess) return 0;
    return perCU;
}

}  // namespace mtsg
