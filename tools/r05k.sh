export TMPDIR=/tmp; O=gpurun_out/r05k; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 700 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/tfast0.so 3 > $O/ab_tfast.log 2>&1 &&
timeout -k 10 700 python tools/ab_libs.py cornell_box 1920 1080 256 main,$V/eb0.so 3 > $O/ab_eb.log 2>&1 &&
TAG=r05k bash tools/gpu_task.sh tests; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
