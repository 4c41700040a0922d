# round-5 final: every BASELINE config's bench-style line (compute blocks from the r05aj / r05ak PMC files)
export TMPDIR=/tmp; O=gpurun_out/r05al; mkdir -p $O
TAG=r05al bash tools/gpu_task.sh py:tools/configs_bench.py:--json
