export TMPDIR=/tmp; O=gpurun_out/r05aa; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py cubes 1920 1080 256 main,$V/fpc0.so 3 > $O/ab_cols.log 2>&1 &&
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/pair0.so,$V/tid0.so 2 > $O/ab_walk.log 2>&1; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
