#!/bin/bash
# quick GPU check: parity tests + headline bench (megakernel) + wavefront bench at 64 spp
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo pytest=$?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_mk.log 2>&1; echo mk=$?
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --spp 64 --mode wavefront --no-cpu-baseline > gpurun_out/bench_wf.log 2>&1; echo wf=$?
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --scene flying_unicorn --spp 64 --no-cpu-baseline > gpurun_out/bench_uni.log 2>&1; echo uni=$?
