# round-5 end: fresh PMC of the cornell (MIS on / off), cubes MIS and C5 workloads on the final kernels, then every
# BASELINE config's bench-style line (compute blocks from the newest PMC files: r05bj / r05bk)
export TMPDIR=/tmp; O=gpurun_out/r05bk; mkdir -p $O
TAG=r05bk bash tools/gpu_task.sh pmc:cornell_box:1920:1080:256 pmc:cornell_box:1920:1080:256:mis pmc:cubes:1920:1080:1024:mis pmc:flying_unicorn:4096:4096:64 || exit 1
for k in cornell_box_1920x1080x256 cornell_box_1920x1080x256_mis cubes_1920x1080x1024_mis flying_unicorn_4096x4096x64; do
  python tools/pmc_report.py $O $k --out profiles/r05bk_pmc_$k.json > $O/report_$k.log 2>&1 || exit 1
  cp profiles/r05bk_pmc_$k.json $O/
done
TAG=r05bk bash tools/gpu_task.sh py:tools/configs_bench.py:--json
