#!/bin/bash
# f32 mode with the two-box BVH walk: f32 GPU tests, unicorn speed at 4/8 waves, probe statistics
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k fp32 -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1 || { tail -30 gpurun_out/pytest_fp32.log; exit 1; }
tail -1 gpurun_out/pytest_fp32.log
one() {
  env $1 timeout -k 10 300 python bench.py --fp32 --steps 2 --warmup 1 --no-cpu-baseline $2 > gpurun_out/fp32_ab.log 2>&1 || { cat gpurun_out/fp32_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/fp32_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1],d['config']['workload'],d['value'],d['ms_per_step'])" "$1"
}
for w in 4 8; do one RT_F32_WAVES=$w "--scene flying_unicorn --spp 64"; done
one RT_F32_BRUTE=0 "--scene cubes --spp 256"
timeout -k 10 300 python -u tools/fp32_probe.py > gpurun_out/fp32_probe.log 2>&1; rc=$?; cat gpurun_out/fp32_probe.log; exit $rc
