export TMPDIR=/tmp; O=gpurun_out/r05ad; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 600 python tools/ab_libs.py flying_unicorn 1920 1080 128 main,$V/noxcd.so,$V/base5.so 3 > $O/ab_unicorn.log 2>&1 &&
timeout -k 10 600 python tools/ab_libs.py cubes 1920 1080 256 main,$V/noxcd.so,$V/base5.so 2 > $O/ab_cubes.log 2>&1 &&
timeout -k 10 600 python tools/ab_libs.py cornell_box 1920 1080 256 main,$V/noxcd.so 2 > $O/ab_cornell.log 2>&1 &&
TAG=r05ad bash tools/gpu_task.sh pmc:flying_unicorn:1920:1080:128; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/ab_*.log | sed 's/.*x\([0-9]*\) mk.*sha1/\1/' | sort | uniq -c
