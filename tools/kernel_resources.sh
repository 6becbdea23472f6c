#!/bin/bash
# VGPR / SGPR / LDS / occupancy of the device kernels (compiler remarks,
# device-only compile of one translation unit; no GPU needed).
#   tools/kernel_resources.sh [source.hip] [kernel-name-regex]
SRC=${1:-my-mitsuba_amd/csrc/mtsg.hip}
PAT=${2:-k_trace_s|k_shade|k_finish|k_camera|k_splat}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -munsafe-fp-atomics \
    -Wno-unused-value -Wno-unused-result $EXTRA --cuda-device-only -c -o /tmp/kres.o "$SRC" \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v pat="$PAT" '/Function Name:/ { name=$0; sub(/.*Function Name: /, "", name); sub(/ \[-R.*/, "", name);
                        keep = (name ~ pat) }
                     keep && /VGPRs:|SGPRs Spill|Occupancy|LDS Size|ScratchSize/ { v=$0; sub(/.*remark: +/, "", v); sub(/ \[-R.*/, "", v); printf "%s | %s\n", name, v }'
