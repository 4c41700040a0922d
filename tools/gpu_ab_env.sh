#!/bin/bash
# A/B over environment settings: CONFIGS="NAME:VAR=val,VAR=val ..." SCENES="scene w h spp;..."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_ab.log 2>&1 || { echo pytest FAIL; tail -30 gpurun_out/pytest_ab.log; exit 1; }
  echo "pytest ok: $(tail -1 gpurun_out/pytest_ab.log)"
fi
IFS=';' read -ra SC <<< "${SCENES:-cubes 1920 1080 128;flying_unicorn 960 540 64}"
for S in "${SC[@]}"; do
  for C in $CONFIGS; do
    NAME=${C%%:*}; VARS=${C#*:}
    env $(echo $VARS | tr ',' ' ') timeout -k 10 200 python tools/prof_render.py $S ${MODE:-mk} > gpurun_out/ab_tmp.log 2>&1 || { echo "FAIL $NAME $S"; tail -20 gpurun_out/ab_tmp.log; exit 1; }
    echo "$NAME $(tail -1 gpurun_out/ab_tmp.log)"
  done
done
