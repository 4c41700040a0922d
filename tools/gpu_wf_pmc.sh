#!/bin/bash
# Wavefront (north_star's streaming layout) on cornell: kernel trace + FETCH/WRITE PMC passes
export TMPDIR=/tmp
mkdir -p gpurun_out
P="python tools/prof_render.py cornell_box 1920 1080 16 wf"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/wf_trace -o run --output-format csv -- $P > gpurun_out/wf_trace.log 2>&1 || { echo trace FAIL; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/wf_fetch -o run --output-format csv -- $P > gpurun_out/wf_fetch.log 2>&1 || { echo fetch FAIL; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/wf_write -o run --output-format csv -- $P > gpurun_out/wf_write.log 2>&1 || { echo write FAIL; exit 1; }
echo ok
