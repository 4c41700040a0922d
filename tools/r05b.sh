export TMPDIR=/tmp; O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 60 python tools/prof_render.py flying_unicorn 64 48 8 mk > $O/small_p1.log 2>&1 &&
RT_MK_POOL=2 timeout -k 10 60 python tools/prof_render.py flying_unicorn 64 48 8 mk > $O/small_p2.log 2>&1 &&
cat $O/small_p1.log $O/small_p2.log &&
timeout -k 10 400 python tools/ab_libs.py flying_unicorn 1920 1080 64 main,main@RT_MK_POOL=2 2 > $O/ab.log 2>&1 &&
cat $O/ab.log &&
RT_MK_POOL=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_pool2.log 2>&1; tail -3 $O/pytest_pool2.log
