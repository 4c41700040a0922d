export TMPDIR=/tmp; O=gpurun_out/r05t; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/hoist2.so,$V/tps3.so,$V/tps1.so 2 > $O/ab_step.log 2>&1; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/ab_step.log | sed 's/.*sha1//' | sort | uniq -c
