export TMPDIR=/tmp; O=gpurun_out/r05ar; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 128 main,$V/rf8.so,$V/rf32.so 3 > $O/ab_refill.log 2>&1; grep -h median $O/ab_*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/ab_*.log | sed 's/.*x\([0-9]*\) mk.*sha1/\1/' | sort | uniq -c
