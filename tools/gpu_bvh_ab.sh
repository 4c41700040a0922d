#!/bin/bash
# GPU tests + nearest-triangle (BVH) mode vs the octree on the unicorn: interleaved BVH walks,
# fused BVH traversal (RT_MK_BVH_FUSED=1), and the walk steps per iteration.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
for S in "flying_unicorn 960 540 64" "flying_unicorn 1920 1080 64" "cubes 1920 1080 128"; do
  timeout -k 10 120 python tools/prof_render.py $S mk || exit 1
  timeout -k 10 120 python tools/prof_render.py $S mk - nearest || exit 1
  RT_MK_BVH_FUSED=1 timeout -k 10 120 python tools/prof_render.py $S mk - nearest | sed "s/^/fused /" || exit 1
done
for k in 2 4 8; do
  RT_MK_KSTEPS=$k timeout -k 10 120 python tools/prof_render.py flying_unicorn 960 540 64 mk - nearest | sed "s/^/ksteps=$k /" || exit 1
done
