#!/bin/bash
# BVH build A/B: binned SAH (default) vs median split (RT_BVH_SAH=0); nearest-triangle + f32 tests first
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "nearest or fp32 or extra" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sah.log 2>&1 || { tail -30 gpurun_out/pytest_sah.log; exit 1; }
tail -1 gpurun_out/pytest_sah.log
for s in 0 1; do
  for m in f32 "mk nearest"; do
    RT_BVH_SAH=$s timeout -k 10 120 python tools/prof_render.py flying_unicorn 1920 1080 64 $m > gpurun_out/sah.log 2>&1 || { cat gpurun_out/sah.log; exit 1; }
    echo "RT_BVH_SAH=$s $(cat gpurun_out/sah.log)"
  done
  RT_BVH_SAH=$s timeout -k 10 120 python tools/prof_render.py cubes 1920 1080 64 mk nearest > gpurun_out/sah.log 2>&1 || { cat gpurun_out/sah.log; exit 1; }
  echo "RT_BVH_SAH=$s $(cat gpurun_out/sah.log)"
done
