export TMPDIR=/tmp; O=gpurun_out/r05m; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/p640.so,$V/w5.so,$V/w7.so 2 > $O/ab_paths.log 2>&1 &&
timeout -k 10 300 python tools/ab_libs.py flying_unicorn 1920 1080 512 main 1 > $O/c4.log 2>&1 &&
TAG=r05m bash tools/gpu_task.sh tests; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
