export TMPDIR=/tmp; O=gpurun_out/r05bd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 2 $O/pytest_gpu.log
run() { echo "# $*" >> $O/tail.log; env "$@" >> $O/tail.log 2>&1; }
run RT_X=0 timeout -k 10 120 python tools/tail_probe.py 1024 cornell_box 1920 1080 &&
run RT_X=0 timeout -k 10 120 python tools/tail_probe.py share 512 flying_unicorn 1920 1080 8 0,7 512 &&
run RT_X=0 timeout -k 10 120 python tools/tail_probe.py share 1024 cubes 1920 1080 8 0,7 1024 &&
run RT_X=0 timeout -k 10 200 python tools/tail_probe.py share 4096 flying_unicorn 4096 4096 8 0 &&
run RT_MK_TAIL_CPS=4 RT_MK_TAIL_DIV=2 RT_MK_TAIL_CAP_DIV=2 timeout -k 10 200 python tools/tail_probe.py share 4096 flying_unicorn 4096 4096 8 0; rc=$?
grep -v "amdgpu.ids" $O/tail.log | sed 's/ samples.*Msamples\/s, vs.*efficiency/ eff/' | cut -c1-160; exit $rc
