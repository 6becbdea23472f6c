#!/bin/bash
# L1/TLB/L2 behaviour of the traversal kernels (one bunny15 32-spp frame per pass)
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/pmc2/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 2 "gpurun_out/pmc2/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for bp in 268435456; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --batch-paths $bp > gpurun_out/pmc2/bench_bp$bp.log 2>&1 || exit $?
  python tools/summarize_bench.py gpurun_out/pmc2/bench_bp$bp.log
done
P="python tools/prof_frame.py bunny15 32"
run q1 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum --kernel-trace --output-format csv -d gpurun_out/pmc2 -o q1 -- $P
run q2 300 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TA_BUSY_avr TCP_TCP_TA_DATA_STALL_CYCLES_sum --kernel-trace --output-format csv -d gpurun_out/pmc2 -o q2 -- $P
run q3 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum TCC_BUSY_avr --kernel-trace --output-format csv -d gpurun_out/pmc2 -o q3 -- $P
run q4 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc2 -o q4 -- $P
