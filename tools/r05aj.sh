# round-5 final measurement, part 1: GPU tests, smoke, bench + trace, the headline's counters, and the
# PMC + wait passes of the C3 / C4 / C5 workloads on the final kernels
export TMPDIR=/tmp
TAG=r05aj bash tools/gpu_task.sh tests smoke bench trace benchpmc pmc:flying_unicorn:1920:1080:512 pmcw:flying_unicorn:1920:1080:512 pmc:cubes:1920:1080:1024 pmcw:cubes:1920:1080:1024
