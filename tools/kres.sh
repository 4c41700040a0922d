#!/bin/bash
# print VGPRs / occupancy per kernel of a .hip file: tools/kres.sh <file.hip>
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -c "$1" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -E 'Function Name|VGPRs:|Occupancy' | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste - - - | awk -F'\t' '{print $1" | "$2" | "$3}' | sed 's/Function Name: //'
