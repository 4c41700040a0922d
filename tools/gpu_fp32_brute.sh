#!/bin/bash
# f32 mode A/B: small meshes brute-forced from scalar loads (RT_F32_BRUTE=16) vs BVH walk (0)
export TMPDIR=/tmp
one() {
  env $1 timeout -k 10 300 python bench.py --fp32 --steps 2 --warmup 1 --no-cpu-baseline $2 > gpurun_out/fp32_ab.log 2>&1 || { cat gpurun_out/fp32_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/fp32_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1],d['config']['workload'],d['value'],d['ms_per_step'])" "$1"
}
for b in 0 16; do one RT_F32_BRUTE=$b "--scene cubes --spp 256"; done
one RT_F32_BRUTE=16 "--scene cornell_box --spp 256"
one RT_F32_BRUTE=16 "--scene flying_unicorn --spp 64"
timeout -k 10 300 python -u tools/fp32_probe.py > gpurun_out/fp32_probe.log 2>&1; rc=$?; cat gpurun_out/fp32_probe.log; exit $rc
