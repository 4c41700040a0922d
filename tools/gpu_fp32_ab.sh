#!/bin/bash
# f32 perf mode A/B: waves/SIMD (RT_F32_WAVES) on cornell and the unicorn; probe statistics
export TMPDIR=/tmp
one() {  # env, bench args
  env $1 timeout -k 10 300 python bench.py --fp32 --steps 2 --warmup 1 --no-cpu-baseline $2 > gpurun_out/fp32_ab.log 2>&1 || { cat gpurun_out/fp32_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/fp32_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1],d['config']['workload'],d['value'],d['ms_per_step'])" "$1"
}
for w in 4 6 8; do
  one RT_F32_WAVES=$w "--scene cornell_box --spp 256"
  one RT_F32_WAVES=$w "--scene cubes --spp 256"
  one RT_F32_WAVES=$w "--scene flying_unicorn --spp 64"
done
timeout -k 10 300 python -u tools/fp32_probe.py > gpurun_out/fp32_probe.log 2>&1; rc=$?; cat gpurun_out/fp32_probe.log; exit $rc
