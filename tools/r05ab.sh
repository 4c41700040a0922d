export TMPDIR=/tmp
bash tools/r05aa.sh &&
TAG=r05ab bash tools/gpu_task.sh tests py:tools/determinism_stress.py env:RT_AMD_LIB=raytracer-server_amd/lib/variants/qcheck.so py:tools/determinism_stress.py
