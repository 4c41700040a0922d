#!/bin/bash
# Round profile r01h: GPU tests + smoke, headline bench (f64), f32 perf mode at the BASELINE sizes,
# f32 kernel trace (rocprofv3 --kernel-trace --stats) and SQ PMC passes
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r01h.log 2>&1 || { tail -5 gpurun_out/bench_r01h.log; exit 1; }
tail -1 gpurun_out/bench_r01h.log
: > gpurun_out/fp32_r01h.log
for a in "--scene cornell_box --spp 1024" "--scene cornell_box --spp 256" "--scene cubes --spp 1024" "--scene cubes --spp 1024 --mis" "--scene flying_unicorn --spp 512"; do
  timeout -k 10 300 python bench.py --fp32 --steps 2 --warmup 1 --no-cpu-baseline $a > gpurun_out/fp32_bench.log 2>&1 || { cat gpurun_out/fp32_bench.log; exit 1; }
  tail -1 gpurun_out/fp32_bench.log >> gpurun_out/fp32_r01h.log
  python -c "import json;d=json.loads(open('gpurun_out/fp32_bench.log').read().strip().splitlines()[-1]);print(d['config']['workload'],d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/f32trace -o run --output-format csv -- python tools/prof_render.py cornell_box 1920 1080 1024 f32 > gpurun_out/f32trace.log 2>&1 || { tail -5 gpurun_out/f32trace.log; exit 1; }
cat gpurun_out/f32trace.log
PMODE=f32 bash tools/gpu_pmc_mk.sh || exit 1
python tools/pmc_summary.py k_megakernel_f32 > gpurun_out/pmc_f32_summary.txt; cat gpurun_out/pmc_f32_summary.txt
