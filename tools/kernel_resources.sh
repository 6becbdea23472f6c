#!/bin/bash
# Register / scratch / occupancy of the shading kernels of one sampler unit
# (the compiler's kernel-resource-usage remarks).  tools/kernel_resources.sh [extra hipcc flags]
# SRC=my-mitsuba_amd/csrc/mtsg.hip for the traversal / camera / splat kernels
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -munsafe-fp-atomics \
  -Wno-unused-value -Wno-unused-result -DMTSG_TU_SAMPLER=0 "$@" --cuda-device-only -c -o /tmp/kres.o \
  ${SRC:-my-mitsuba_amd/csrc/smp_kernels.hip} -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1); print(); print(cur[:70], end=""); continue
    m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
    if m and cur: print(f"  {m.group(1).split()[0]}={m.group(2)}", end="")
print()'
