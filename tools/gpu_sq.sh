#!/bin/bash
# SQ / TCP counters of the traversal, one C3 32-spp frame per pass, for the
# flattened and the two-level kernel:  tools/gpu_sq.sh r03 [flatten two-level]
R=${1:-r03}; shift
O=gpurun_out/sq_$R; mkdir -p $O
export TMPDIR=/tmp
for inst in ${*:-flatten two-level}; do
  run() { local name=$1; shift; timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O -o ${inst}_$name -- python tools/prof_frame.py bunny15 32 1 1 $inst > $O/${inst}_$name.log 2>&1; local rc=$?; echo "$inst $name rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/${inst}_$name.log; exit $rc; fi; }
  run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
  run p2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
  run p3 TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum
  python tools/pmc_summary.py $O/${inst}_p*_counter_collection.csv > $O/${inst}_summary.txt
done
