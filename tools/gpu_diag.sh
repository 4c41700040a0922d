#!/bin/bash
# Diagnostics: traversal counters (debug build) on cubes/unicorn + SQ PMC passes on the cornell megakernel.
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
for S in "cubes 960 540 16" "flying_unicorn 960 540 16"; do
  timeout -k 10 120 python tools/dbg_counters.py $PWD/raytracer-server_amd/lib/variants/dbg.so $S > gpurun_out/dbg.log 2>&1 || { echo "dbg FAIL $S"; tail -20 gpurun_out/dbg.log; exit 1; }
  tail -1 gpurun_out/dbg.log
done
P="python tools/prof_render.py ${PSCENE:-cornell_box 1920 1080 64} mk"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d gpurun_out/pmc1 -o run --output-format csv -- $P > gpurun_out/pmc1.log 2>&1 || { echo p1 FAIL; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -d gpurun_out/pmc2 -o run --output-format csv -- $P > gpurun_out/pmc2.log 2>&1 || { echo p2 FAIL; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_SMEM -d gpurun_out/pmc3 -o run --output-format csv -- $P > gpurun_out/pmc3.log 2>&1 || { echo p3 FAIL; exit 1; }
echo pmc ok
