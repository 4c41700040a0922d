export TMPDIR=/tmp; O=gpurun_out/r05au; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 900 python tools/ab_libs.py cubes 1920 1080 256 main,$V/fg.so 3 > $O/ab_cubes.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "cubes or flat or c3 or walk_culls" > $O/pytest_flat.log 2>&1; tail -n 3 $O/pytest_flat.log; grep -h median $O/ab_*.log | sed 's/raytracer-server_amd.lib.variants.//'; grep -h sha1 $O/ab_*.log | sed 's/.*x\([0-9]*\) mk.*sha1/\1/' | sort | uniq -c
