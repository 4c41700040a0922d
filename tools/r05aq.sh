# round-5 final: every BASELINE config's bench-style line (compute blocks from the r05ap PMC files)
export TMPDIR=/tmp; O=gpurun_out/r05aq; mkdir -p $O
TAG=r05aq bash tools/gpu_task.sh py:tools/configs_bench.py:--json
