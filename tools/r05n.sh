export TMPDIR=/tmp; O=gpurun_out/r05n; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/a32.so,$V/objg.so 2 > $O/ab_anc.log 2>&1 &&
timeout -k 10 600 python tools/ab_libs.py cubes 1920 1080 256 main,main@RT_MK_FLAT=0 1 > $O/ab_cubes_roles.log 2>&1 &&
TAG=r05n bash tools/gpu_task.sh tests; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
