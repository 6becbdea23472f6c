#!/bin/bash
# memory-pipeline counters for the unified traversal (one bunny15 32-spp frame per pass)
O=gpurun_out/pmc3; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O -o $name -- python tools/prof_frame.py bunny15 32 > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; exit $rc; fi; }
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD
run p2 TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
run p3 TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum
run p4 TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_TA_BUSY GRBM_COUNT
run p5 TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr TCC_TAG_STALL_sum
run p6 SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_BUSY_CYCLES
python tools/pmc_summary.py $O/p*_counter_collection.csv > $O/summary.txt; cat $O/summary.txt | head -80
