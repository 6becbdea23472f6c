#!/bin/bash
# Copy the round-3 GPU outputs (tools/gpu_final3.sh) into profiles/.
set -e
O=gpurun_out
line() { grep '^{' "$1" | tail -1; }
line $O/r3/bench.log > profiles/r03_bench_bunny15.json
line $O/r3/inst.log > profiles/r03_bench_bunny15_two_level.json
line $O/r3/e8.log > profiles/r03_bench_c4_e8.json
line $O/r3/kd.log > profiles/r03_bench_bunny15_kd_device.json
line $O/r3/c2.log > profiles/r03_bench_c2.json
line $O/r3/c5.log > profiles/r03_bench_c5.json
for t in c3 c3_two_level c5; do
  key=$(python -c "import json;print(json.dumps(json.load(open('$O/pmc_r03_$t/pmc.json'))['key']))")
  python tools/pmc_kernels.py $O/pmc_r03_$t "$key" > profiles/r03_pmc_$t.json
  cp $O/pmc_r03_$t/stats_kernel_stats.csv profiles/r03_${t}_kernel_stats.csv
done
cp $O/pmc_r03_c3/fetch_counter_collection.csv profiles/r03_bunny15_pmc_fetch_size.csv
cp $O/pmc_r03_c3/write_counter_collection.csv profiles/r03_bunny15_pmc_write_size.csv
cp $O/sq_r03/flatten_summary.txt profiles/r03_sq_flatten_summary.txt
cp $O/sq_r03/two-level_summary.txt profiles/r03_sq_two_level_summary.txt
cp $O/r3/tests.log profiles/r03_gpu_tests.log.txt
echo collected
