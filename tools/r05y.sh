export TMPDIR=/tmp; O=gpurun_out/r05y; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py cubes 1920 1080 256 main,main@RT_MK_FPOOL_REFILL=0,main@RT_MK_FPOOL_REFILL=12,$V/fprio0.so,$V/fready24.so,$V/fready8.so 2 > $O/ab_refill.log 2>&1 &&
TAG=r05y bash tools/gpu_task.sh pmc:cubes:1920:1080:1024 pmcw:cubes:1920:1080:1024; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/ab_refill.log | sed 's/.*sha1//' | sort | uniq -c
