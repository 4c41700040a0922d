export TMPDIR=/tmp; O=gpurun_out/r05ay; mkdir -p $O
timeout -k 10 200 python tools/ramp_probe.py 8 > $O/ramp.log 2>&1 && timeout -k 10 200 python tools/ramp_probe.py 2 >> $O/ramp.log 2>&1; rc=$?; cat $O/ramp.log; exit $rc
