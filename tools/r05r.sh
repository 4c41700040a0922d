export TMPDIR=/tmp; O=gpurun_out/r05r; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/rf8.so,$V/rf24.so,$V/prio0.so 2 > $O/ab_rf.log 2>&1 &&
TAG=r05r bash tools/gpu_task.sh pmc:flying_unicorn:4096:4096:64 pmc:cubes:1920:1080:1024 pmc:cornell_box:1920:1080:256 pmc:cornell_box:1920:1080:256:mis; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/ab_rf.log | sed 's/.*sha1//' | sort | uniq -c
