export TMPDIR=/tmp; O=gpurun_out/r05p; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/p752.so 3 > $O/ab_p784.log 2>&1 &&
TAG=r05p bash tools/gpu_task.sh tests; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
