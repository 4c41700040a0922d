#!/bin/bash
# A/B of library variants on cornell + WRITE_SIZE PMC of each (scratch spill write-back check)
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in $VARIANTS; do
  RT_AMD_LIB=$PWD/raytracer-server_amd/lib/variants/$V.so timeout -k 10 120 python tools/prof_render.py cornell_box 1920 1080 256 mk | tail -1 | sed "s/^/$V /"
  RT_AMD_LIB=$PWD/raytracer-server_amd/lib/variants/$V.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/w_$V -o run --output-format csv -- python tools/prof_render.py cornell_box 1920 1080 64 mk > gpurun_out/w_$V.log 2>&1 || { echo "pmc FAIL $V"; exit 1; }
  python3 -c "import csv;print('$V WRITE_SIZE KiB', [r['Counter_Value'] for r in csv.DictReader(open('gpurun_out/w_$V/run_counter_collection.csv')) if 'megakernel' in r['Kernel_Name']])"
done
