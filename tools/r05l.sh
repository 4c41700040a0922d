export TMPDIR=/tmp; O=gpurun_out/r05l; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/b768p632.so,$V/b768w7p616.so,$V/b768p576.so 2 > $O/ab_b768.log 2>&1; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/*.log | sed 's/.*sha1//' | sort | uniq -c
