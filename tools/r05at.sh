# the cubes' query-pool breakdown on the final kernels (diagnostic build: region timers and query counters)
export TMPDIR=/tmp
TAG=r05at bash tools/gpu_task.sh py:tools/dbg_mesh.py:raytracer-server_amd/lib/variants/dbg.so:cubes:1920:1080:64 py:tools/dbg_mesh.py:raytracer-server_amd/lib/variants/dbg.so:flying_unicorn:1920:1080:64
