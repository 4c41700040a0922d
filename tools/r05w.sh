export TMPDIR=/tmp; O=gpurun_out/r05w; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py cubes 1920 1080 256 main,$V/fp1024.so 3 > $O/ab_fp.log 2>&1 &&
timeout -k 10 300 python tools/ab_libs.py cubes 1920 1080 1024 main,$V/fp1024.so 1 > $O/c3.log 2>&1; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
