export TMPDIR=/tmp; O=gpurun_out/r05ba; mkdir -p $O
run() { echo "# $*" >> $O/tail.log; env "$@" >> $O/tail.log 2>&1; }
for r in 1 2; do
run RT_X=0 timeout -k 10 120 python tools/tail_probe.py share 1024 cubes 1920 1080 8 0 1024 &&
run RT_MK_TAIL_CPS=8 timeout -k 10 120 python tools/tail_probe.py share 1024 cubes 1920 1080 8 0 1024 &&
run RT_X=0 timeout -k 10 120 python tools/tail_probe.py share 512 flying_unicorn 1920 1080 8 0 512 &&
run RT_MK_TAIL_CPS=8 timeout -k 10 120 python tools/tail_probe.py share 512 flying_unicorn 1920 1080 8 0 512 || exit 1
done
grep -v "amdgpu.ids" $O/tail.log | sed 's/ samples.*Msamples\/s, vs.*efficiency/ eff/' | cut -c1-150
