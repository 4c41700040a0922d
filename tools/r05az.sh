export TMPDIR=/tmp; O=gpurun_out/r05az; mkdir -p $O
run() { echo "# $*" >> $O/tail.log; env "$@" timeout -k 10 120 python tools/tail_probe.py share 1024 cornell_box 1920 1080 8 0 1024 >> $O/tail.log 2>&1; }
run RT_X=0 && run RT_MK_TAIL_CPS=8 && run RT_MK_TAIL_DIV=1 && run RT_MK_TAIL_DIV=1 RT_MK_TAIL_CPS=8 &&
run RT_MK_TAIL_MUL=2 RT_MK_TAIL_DIV=1 RT_MK_TAIL_CPS=8 && run RT_MK_TAIL_MIN_LG=4 RT_MK_TAIL_CPS=16 &&
run RT_MK_TAIL_MIN_LG=4 RT_MK_TAIL_CPS=16 RT_MK_TAIL_DIV=1 && run RT_MK_TAIL_MIN_LG=3 RT_MK_TAIL_CPS=32 RT_MK_TAIL_DIV=1 &&
run RT_X=0; rc=$?; grep -v "full frame\|amdgpu.ids" $O/tail.log | sed 's/ samples.*efficiency/ eff/'; exit $rc
