export TMPDIR=/tmp; O=gpurun_out/r05ax; mkdir -p $O
timeout -k 10 200 python tools/end_probe.py 1024 > $O/end.log 2>&1 &&
RT_MK_TAIL=0 timeout -k 10 200 python tools/end_probe.py 1024 >> $O/end.log 2>&1 &&
RT_MK_TAIL_CPS=16 timeout -k 10 200 python tools/end_probe.py 1024 >> $O/end.log 2>&1; rc=$?; cat $O/end.log; exit $rc
