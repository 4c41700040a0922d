export TMPDIR=/tmp; O=gpurun_out/r05x; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py cubes 1920 1080 256 main,$V/fp768.so,$V/fpold.so,main@RT_MK_FPOOL_MIN=56,main@RT_MK_FPOOL_MIN=40,main@RT_MK_FPOOL_REFILL=28 2 > $O/ab_fp2.log 2>&1 &&
TAG=r05x bash tools/gpu_task.sh tests; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
