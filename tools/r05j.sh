export TMPDIR=/tmp; O=gpurun_out/r05j; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 700 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/m1off.so 2 > $O/ab_m1.log 2>&1 &&
TAG=r05j bash tools/gpu_task.sh tests; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -c 5d85713c0b4a $O/ab_m1.log
