export TMPDIR=/tmp; O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py flying_unicorn 1920 1080 64 main@RT_MK_POOL=2,raytracer-server_amd/lib/variants/w3.so@RT_MK_POOL=2,raytracer-server_amd/lib/variants/w5.so@RT_MK_POOL=2,raytracer-server_amd/lib/variants/rf8.so@RT_MK_POOL=2,raytracer-server_amd/lib/variants/rf32.so@RT_MK_POOL=2,raytracer-server_amd/lib/variants/prio0.so@RT_MK_POOL=2 2 > $O/ab_roles_tune.log 2>&1 &&
timeout -k 10 300 python tools/ab_libs.py flying_unicorn 1920 1080 512 main,main@RT_MK_POOL=2 1 > $O/ab_c4.log 2>&1; cat $O/*.log | grep median
