export TMPDIR=/tmp; O=gpurun_out/r05bb; mkdir -p $O
run() { echo "# $*" >> $O/tail.log; env "$@" timeout -k 10 120 python tools/tail_probe.py share 512 flying_unicorn 1920 1080 8 0,7 512 >> $O/tail.log 2>&1; }
run RT_MK_TAIL_CPS=8 && run RT_MK_TAIL_CPS=8 RT_MK_TAIL_DIV=1 && run RT_MK_TAIL_CPS=8 RT_MK_TAIL_DIV=1 RT_MK_TAIL_MUL=2 &&
run RT_MK_TAIL_CPS=8 RT_MK_TAIL_DIV=1 RT_MK_TAIL_MUL=4 && run RT_MK_TAIL_CPS=16 RT_MK_TAIL_DIV=1 RT_MK_TAIL_MUL=2; rc=$?
grep -v "amdgpu.ids" $O/tail.log | sed 's/ samples.*Msamples\/s, vs.*efficiency/ eff/' | cut -c1-150; exit $rc
