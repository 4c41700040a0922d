#!/bin/bash
# f32 perf mode: probe statistics, speed at the BASELINE sizes, kernel trace + SQ PMC on cornell
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fp32_probe.py > gpurun_out/fp32_probe.log 2>&1; rc=$?; cat gpurun_out/fp32_probe.log; [ $rc = 0 ] || exit 1
for a in "--scene cornell_box --spp 1024" "--scene cubes --spp 1024" "--scene flying_unicorn --spp 512"; do
  timeout -k 10 300 python bench.py --fp32 --steps 2 --warmup 1 --no-cpu-baseline $a > gpurun_out/fp32_bench.log 2>&1 || { cat gpurun_out/fp32_bench.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/fp32_bench.log').read().strip().splitlines()[-1]);print(d['config']['workload'],d['value'],d['ms_per_step'],d['config']['vertices_per_sample'])"
done
[ -n "$NOPMC" ] && exit 0
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/f32trace -o run --output-format csv -- python tools/prof_render.py cornell_box 1920 1080 256 f32 > gpurun_out/f32trace.log 2>&1 || { tail -5 gpurun_out/f32trace.log; exit 1; }
PMODE=f32 bash tools/gpu_pmc_mk.sh || exit 1
python tools/pmc_summary.py k_megakernel_f32
