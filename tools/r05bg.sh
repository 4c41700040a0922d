export TMPDIR=/tmp; O=gpurun_out/r05bg; mkdir -p $O
V=raytracer-server_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 2 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/ab_libs.py cornell_box 1920 1080 256 main,$V/nee0.so 3 > $O/ab_cornell.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py cornell_box 1920 1080 256 main,$V/nee0.so 2 mis > $O/ab_cornell_mis.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py cubes 1920 1080 256 main,$V/nee0.so 2 mis > $O/ab_cubes_mis.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py flying_unicorn 1920 1080 64 main,$V/nee0.so 2 > $O/ab_unicorn.log 2>&1; rc=$?
for f in $O/ab_*.log; do echo "== $f"; grep -o "sha1 [0-9a-f]*" $f | sort | uniq -c; grep median $f; done; exit $rc
