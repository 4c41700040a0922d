#!/bin/bash
# Round profile (tools/gpu_profile.sh) + every BASELINE config (tools/configs_bench.py), TAG=<round tag>
export TMPDIR=/tmp
TAG=${TAG:-r01}
bash tools/gpu_profile.sh || exit 1
timeout -k 10 300 python tools/configs_bench.py > gpurun_out/configs_${TAG}.log 2>&1 || { echo configs FAIL; tail -20 gpurun_out/configs_${TAG}.log; exit 1; }
cat gpurun_out/configs_${TAG}.log
bash tools/gpu_pmc_mk.sh > gpurun_out/sq_${TAG}.log 2>&1 || { echo sq FAIL; tail -5 gpurun_out/sq_${TAG}.log; exit 1; }
python tools/pmc_summary.py k_megakernel
