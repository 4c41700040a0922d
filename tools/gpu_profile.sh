#!/bin/bash
# Round profile of the headline bench: GPU tests, bench line (with cpu_baseline), rocprofv3 kernel
# trace + stats of the same command, FETCH_SIZE / WRITE_SIZE PMC passes (separate runs).
# Output: gpurun_out/prof_<TAG>/...
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest FAIL; tail -20 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest: $(tail -1 gpurun_out/pytest_gpu.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo smoke FAIL; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 || { echo bench FAIL; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || { echo prof FAIL; tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
tail -1 gpurun_out/prof_${TAG}.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_${TAG} -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcf_${TAG}.log 2>&1 || { echo fetch FAIL; tail -5 gpurun_out/pmcf_${TAG}.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_${TAG} -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcw_${TAG}.log 2>&1 || { echo write FAIL; tail -5 gpurun_out/pmcw_${TAG}.log; exit 1; }
echo profile ok
