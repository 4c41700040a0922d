export TMPDIR=/tmp; O=gpurun_out/r05ac; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 600 python tools/ab_libs.py cornell_box 1920 1080 256 main,$V/nofma.so,$V/noax.so,$V/base5.so 3 > $O/ab_cornell.log 2>&1 &&
timeout -k 10 600 python tools/ab_libs.py cubes 1920 1080 256 main,$V/base5.so 2 > $O/ab_cubes.log 2>&1 &&
timeout -k 10 600 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/base5.so 2 > $O/ab_unicorn.log 2>&1; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*x\([0-9]*\) mk.*sha1/\1/' | sort | uniq -c
