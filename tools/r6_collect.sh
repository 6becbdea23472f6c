#!/bin/bash
# Copy round 6's final evidence from gpurun_out/ into profiles/ (after
# tools/gpu_r06.sh pmc-* and the bench / test steps ran at the final build).
set -u
P=profiles
copy() { if [ -f "$1" ]; then cp "$1" "$2"; echo "$2"; else echo "missing: $1" >&2; fi; }
last_json() { if [ -f "$1" ]; then grep '^{' "$1" | tail -1 > "$2"; echo "$2"; else echo "missing: $1" >&2; fi; }
for t in c3 c3_two_level c5 c4_share8 c2; do
  copy gpurun_out/pmc_r06_$t/pmc.json $P/r06_pmc_$t.json
  copy gpurun_out/pmc_r06_$t/stats_kernel_stats.csv $P/r06_${t}_kernel_stats.csv
done
O=gpurun_out/r6
last_json $O/bench.log $P/r06_bench_bunny15.json
last_json $O/c5.log $P/r06_bench_c5.json
last_json $O/inst.log $P/r06_bench_bunny15_two_level.json
last_json $O/c2.log $P/r06_bench_c2.json
last_json $O/e8.log $P/r06_bench_c4_e8.json
last_json $O/ranks-torchrun.log $P/r06_bench_ranks2_torchrun_shared.json
last_json $O/ranks-self.log $P/r06_bench_ranks2_self_shared.json
copy $O/ranks-refuse.log $P/r06_bench_ranks2_refusal.txt
copy $O/tests.log $P/r06_gpu_tests.log.txt
copy $O/smoke.log $P/r06_smoke.txt
