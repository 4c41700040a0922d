export TMPDIR=/tmp; O=gpurun_out/r05ae; mkdir -p $O
TAG=r05ae bash tools/gpu_task.sh tests smoke bench trace &&
timeout -k 10 300 python tools/tail_probe.py 1024 > $O/tail_probe.log 2>&1 &&
RT_MK_TAIL_DIV=1 timeout -k 10 300 python tools/tail_probe.py 1024 > $O/tail_probe_div1.log 2>&1 &&
RT_MK_TAIL_CPS=8 timeout -k 10 300 python tools/tail_probe.py 1024 > $O/tail_probe_cps8.log 2>&1; tail -n 4 $O/tail_probe*.log
