export TMPDIR=/tmp; O=gpurun_out/r05i; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 700 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/np576.so,$V/np512.so 2 > $O/ab_np.log 2>&1 &&
timeout -k 10 300 python tools/ab_libs.py flying_unicorn 1920 1080 512 main 1 > $O/c4.log 2>&1 &&
TAG=r05i bash tools/gpu_task.sh tests; grep -h median $O/*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -c 5d85713c0b4a $O/ab_np.log; grep -h sha1 $O/c4.log | cut -c1-200
