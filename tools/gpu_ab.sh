#!/bin/bash
# quick perf matrix across scenes (separate processes; env read once per process)
export TMPDIR=/tmp
for W in ${WAVES:-4}; do
  for S in "cornell_box 1920 1080 256" "flying_unicorn 960 540 64" "cubes 1920 1080 128"; do
    for M in ${MODES:-mk}; do
    RT_MK_WAVES=$W timeout -k 10 120 python tools/prof_render.py $S $M > gpurun_out/ab_tmp.log 2>&1 || { echo "FAIL W=$W $S"; cat gpurun_out/ab_tmp.log; exit 1; }
    echo "W=$W $(tail -1 gpurun_out/ab_tmp.log)"
    done
  done
done
