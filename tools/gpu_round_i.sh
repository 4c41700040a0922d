#!/bin/bash
# Round check r01i: every GPU test, smoke(), the default bench line (f64 headline + CPU baselines),
# f32 perf mode at the BASELINE sizes, kernel trace of the headline bench
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r01i.log 2>&1 || { tail -5 gpurun_out/bench_r01i.log; exit 1; }
tail -1 gpurun_out/bench_r01i.log
: > gpurun_out/fp32_r01i.log
for a in "--scene cornell_box --spp 1024" "--scene flying_unicorn --spp 512"; do
  timeout -k 10 300 python bench.py --fp32 --steps 2 --warmup 1 --no-cpu-baseline $a > gpurun_out/fp32_bench.log 2>&1 || { cat gpurun_out/fp32_bench.log; exit 1; }
  tail -1 gpurun_out/fp32_bench.log >> gpurun_out/fp32_r01i.log
  python -c "import json;d=json.loads(open('gpurun_out/fp32_bench.log').read().strip().splitlines()[-1]);print(d['config']['workload'],d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mktrace -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/mktrace.log 2>&1 || { tail -5 gpurun_out/mktrace.log; exit 1; }
tail -1 gpurun_out/mktrace.log | cut -c1-200
