# round-5 end, after the tri_t minors and the flat query's grid order: tests, smoke, bench, PMC + waits of C3 / C4 / C5,
# the C5 share
export TMPDIR=/tmp; O=gpurun_out/r05ap; mkdir -p $O
TAG=r05ap bash tools/gpu_task.sh tests smoke bench pmc:flying_unicorn:1920:1080:512 pmcw:flying_unicorn:1920:1080:512 pmc:cubes:1920:1080:1024 pmcw:cubes:1920:1080:1024 pmc:flying_unicorn:4096:4096:64 &&
timeout -k 10 600 python -u tools/tail_probe.py share 4096 flying_unicorn 4096 4096 8 0,7 > $O/c5_share_probe.log 2>&1 && cat $O/c5_share_probe.log
