#!/bin/bash
# A/B over prebuilt library variants (raytracer-server_amd/lib/variants/*.so), same box, same process type
export TMPDIR=/tmp
for S in "cornell_box 1920 1080 256" "cubes 1920 1080 128" "flying_unicorn 960 540 64"; do
  for V in ${VARIANTS:-$(ls raytracer-server_amd/lib/variants/ | sed 's/.so$//')}; do
    RT_AMD_LIB=$PWD/raytracer-server_amd/lib/variants/$V.so timeout -k 10 120 python tools/prof_render.py $S mk > gpurun_out/ab_tmp.log 2>&1 || { echo "FAIL $V $S"; cat gpurun_out/ab_tmp.log; exit 1; }
    echo "$V $(tail -1 gpurun_out/ab_tmp.log)"
  done
done
