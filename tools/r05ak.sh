# round-5 final measurement, part 2: C5 counters and waits, C3 with MIS, the C5 one-rank share at 4096 spp
export TMPDIR=/tmp; O=gpurun_out/r05ak; mkdir -p $O
TAG=r05ak bash tools/gpu_task.sh pmc:flying_unicorn:4096:4096:64 pmcw:flying_unicorn:4096:4096:64 pmc:cubes:1920:1080:1024:mis &&
timeout -k 10 600 python -u tools/tail_probe.py share 4096 flying_unicorn 4096 4096 8 0,7 > $O/c5_share_probe.log 2>&1 && cat $O/c5_share_probe.log
