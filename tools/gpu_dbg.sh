#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 python tools/parity_report.py scenes/cbox_glass.xml width=24 height=24 spp=8 --replay > gpurun_out/replay.log 2>&1; rc=$?; cat gpurun_out/replay.log; exit $rc
