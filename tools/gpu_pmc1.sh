#!/bin/bash
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 "$lim" "$@" > "gpurun_out/pmc/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 "gpurun_out/pmc/$name.log"; if [ $rc -ge 124 ]; then exit $rc; fi; return 0; }
run p1 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc -o p1 -- python tools/prof_frame.py bunny15 32
run p2 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc -o p2 -- python tools/prof_frame.py bunny15 32
run p3 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/pmc -o p3 -- python tools/prof_frame.py bunny15 32
run p4 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o p4 -- python tools/prof_frame.py bunny15 32
ls gpurun_out/pmc | head -40
