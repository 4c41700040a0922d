# round-5 end: the determinism stress on the final kernels, product and RT_QCHECK libraries
export TMPDIR=/tmp
TAG=r05as bash tools/gpu_task.sh py:tools/determinism_stress.py env:RT_AMD_LIB=raytracer-server_amd/lib/variants/qcheck.so py:tools/determinism_stress.py
