#!/bin/bash
# kernel traces: 1/8 of the frame by tile stride vs the whole frame at 32 spp vs the whole frame
O=gpurun_out/tcmp; mkdir -p $O; export TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o $name -- "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 3 $O/$name.log; return $rc; }
step e8 python tools/prof_frame.py bunny15 256 3 8 && step s32 python tools/prof_frame.py bunny15 32 3 1 && step e1 python tools/prof_frame.py bunny15 256 2 1
