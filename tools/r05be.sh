export TMPDIR=/tmp; O=gpurun_out/r05be; mkdir -p $O
V=raytracer-server_amd/lib/variants
run() { echo "# $*" >> $O/tail.log; env "$@" timeout -k 10 120 python tools/tail_probe.py share 1024 cornell_box 1920 1080 8 0 1024 >> $O/tail.log 2>&1; }
for rep in 1 2; do
run RT_X=0 && run RT_AMD_LIB=$V/st8.so && run RT_AMD_LIB=$V/st8.so RT_MK_TAIL_CPS=16 && run RT_AMD_LIB=$V/st32.so RT_MK_TAIL_CPS=16 &&
run RT_AMD_LIB=$V/st32.so RT_MK_TAIL_CPS=32 RT_MK_TAIL_MIN_LG=3 || exit 1
done
grep -v "amdgpu.ids" $O/tail.log | sed 's/ samples.*Msamples\/s, vs.*efficiency/ eff/;s/raytracer-server_amd.lib.variants.//' | cut -c1-160
