#!/bin/bash
# GPU status run: parity tests, headline bench, per-scene mk/wf renders. Stops at the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo pytest ok; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_mk.log 2>&1 || { echo bench FAIL; tail -20 gpurun_out/bench_mk.log; exit 1; }
tail -1 gpurun_out/bench_mk.log
for S in "cornell_box 1920 1080 256" "cubes 1920 1080 128" "flying_unicorn 960 540 64"; do
  for M in ${MODES:-mk wf}; do
    timeout -k 10 180 python tools/prof_render.py $S $M > gpurun_out/r.log 2>&1 || { echo "FAIL $S $M"; tail -20 gpurun_out/r.log; exit 1; }
    tail -1 gpurun_out/r.log
  done
done
