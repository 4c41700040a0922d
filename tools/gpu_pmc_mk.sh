#!/bin/bash
# SQ PMC passes on one megakernel render: PSCENE="scene w h spp" (default cornell 1920x1080x64), PMODE=mk|f32
export TMPDIR=/tmp
mkdir -p gpurun_out
P="python tools/prof_render.py ${PSCENE:-cornell_box 1920 1080 64} ${PMODE:-mk}"
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
         "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc$i -o run --output-format csv -- $P > gpurun_out/pmc$i.log 2>&1 || { echo "pmc$i FAIL"; tail -5 gpurun_out/pmc$i.log; exit 1; }
done
echo pmc ok
