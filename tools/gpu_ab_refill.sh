#!/bin/bash
# A/B of camera-buffer depth / refill threshold on cornell 1920x1080x256 (variants in lib/variants)
export TMPDIR=/tmp
run() { RT_AMD_LIB=$PWD/raytracer-server_amd/lib/variants/$1.so RT_MK_CAM_REFILL=$2 timeout -k 10 60 python tools/prof_render.py cornell_box 1920 1080 256 mk | tail -1 | sed "s/^/$1 refill=$2 /"; }
for rep in 1 2; do
  run base 24; run d1 24; run d2 24; run d2 32; run d2 40; run d2 48
done
