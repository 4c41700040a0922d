export TMPDIR=/tmp; O=gpurun_out/r05aw; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/tail_probe.py 1024 cornell_box 1920 1080 > $O/tail_probe.log 2>&1; rc=$?
cat $O/tail_probe.log | grep -v "^\[\|^W2\|rocprof" | tail -n 6; find $O/kt -name "*.csv" | head; exit $rc
