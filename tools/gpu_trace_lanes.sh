#!/bin/bash
O=gpurun_out/tl; mkdir -p $O; export TMPDIR=/tmp
MTSG_LANES=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o l2 -- python tools/prof_frame.py bunny15 256 2 8 > $O/l2.log 2>&1; echo rc=$?; grep frame $O/l2.log
