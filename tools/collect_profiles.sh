#!/bin/bash
# Copy a round's profile set (tools/gpu_profile_round.sh output) into profiles/
R=${1:-r01}
S=gpurun_out/prof_$R
set -e
cp $S/traffic.json profiles/${R}_traffic.json
cp $S/stats_kernel_stats.csv profiles/${R}_bunny15_kernel_stats.csv
cp $S/stats_kernel_trace.csv profiles/${R}_bunny15_kernel_trace.csv
cp $S/fetch_counter_collection.csv profiles/${R}_bunny15_pmc_fetch_size.csv
cp $S/write_counter_collection.csv profiles/${R}_bunny15_pmc_write_size.csv
grep '^{' $S/bench.log | tail -1 > profiles/${R}_bench_bunny15.json
