#!/bin/bash
# Round-3 profile set in one call (copied to profiles/ by tools/collect_r03.sh):
# GPU tests, bench lines (C3 with the CPU and parity legs, two-level C3, the
# device kd tree, the 8 emulated rank shares, C2, C5), keyed PMC sets of C3,
# two-level C3 and C5, and SQ counters of both traversal kernels.
set -o pipefail
bash tools/gpu_round3.sh tests bench inst e8 kd c2 c5 || exit $?
bash tools/gpu_round3.sh pmc-c3 pmc-inst pmc-c5 || exit $?
bash tools/gpu_sq.sh r03 || exit $?
