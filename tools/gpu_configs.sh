#!/bin/bash
# Bench lines for the other BASELINE configs: C2 (Cornell box 1280x720x256,
# maxDepth 8) and C5 (glass + envmap, 1920x1080x1024, maxDepth 64), each with
# its CPU-baseline leg; plus the emulated 8-rank share of C3 (config C4)
O=gpurun_out/configs; mkdir -p $O
timeout -k 10 300 python bench.py --workload cbox --steps 3 --warmup 1 > $O/c2.log 2>&1 || { tail $O/c2.log; exit 1; }
echo "c2 $(python tools/summarize_bench.py $O/c2.log)"
timeout -k 10 400 python bench.py --workload c5 --width 1920 --height 1080 --spp 1024 --steps 2 --warmup 1 > $O/c5.log 2>&1 || { tail $O/c5.log; exit 1; }
echo "c5 $(python tools/summarize_bench.py $O/c5.log)"
timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu --emulate-ranks 8 > $O/c4_e8.log 2>&1 || { tail $O/c4_e8.log; exit 1; }
echo "c4_e8 $(python tools/summarize_bench.py $O/c4_e8.log)"
